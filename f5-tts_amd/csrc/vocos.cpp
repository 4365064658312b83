// C ABI of the Vocos decoder (include/f5h.h, f5h_vocos_*): SURVEY §8(f1), the step after the
// CFM path (utils_infer.py:506-511: generated mel [1, 100, T] fp32 -> vocoder.decode).
//
// Layout in HBM per call (R = B*T frames, time-major rows):
//   col    [R][Kemb]      operand dtype   im2col of the k7 embed conv (Kemb = 7*C padded to 64)
//   x0, x  [R][dim]       fp32            embed output, residual stream
//   dwln   [R][dim]       operand dtype   dwconv + LayerNorm (GEMM A operand)
//   hid    [R][inter]     operand dtype   GELU(pwconv1) (GEMM A operand)
//   fln    [R][dim]       fp32            final LayerNorm (head A operand, fp32 head)
//   spec   [R][Kd]        fp32            head output -> (re, im) interleaved, Kd = 2*(n_fft/2+1) padded to 64
//   frames [R][n_fft]     fp32            windowed irfft frames (iDFT GEMM output)
// The iDFT is a GEMM against a fixed basis [n_fft][Kd] (window and irfft weights folded in,
// fp32 MFMA), followed by a deterministic overlap-add that divides by the window envelope.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/f5h.h"
#include "capi_util.h"
#include "kernels.h"
#include "reaper.h"

using namespace f5h;

#define VHIP(x)                                                                                   \
  do {                                                                                            \
    hipError_t _e = (x);                                                                          \
    if (_e != hipSuccess) return f5h_internal_fail(F5H_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)
#define VRC(x)          \
  do {                  \
    int _r = (x);       \
    if (_r) return _r;  \
  } while (0)

namespace {

struct VLin {
  void* w = nullptr;   // [Npad][K] operand dtype (bf16 or fp32)
  float* b = nullptr;  // [Npad] fp32
  int N = 0, K = 0, Npad = 0, compute = 0;
};

struct VBlock {
  float *dw_w = nullptr, *dw_b = nullptr, *ln_w = nullptr, *ln_b = nullptr, *gamma = nullptr;
  VLin pw1, pw2;
};

uint16_t f2bf_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace

struct f5h_vocos {
  f5h::UseLog uses;  // per stream, an event after the last call: what *_destroy waits for
  f5h_vocos_arch a{};
  int dev = 0;
  int bf = 0;
  int kemb = 0, kd = 0, bins = 0;
  std::vector<void*> allocs;
  VLin embed, head, idft;
  float *norm_b = nullptr, *norm_sm1 = nullptr, *fnorm_b = nullptr, *fnorm_sm1 = nullptr, *win = nullptr;
  std::vector<VBlock> blocks;

  hipStream_t mstream = nullptr;  // uploads at creation, stream-ordered frees at release (reaper.h)
  template <typename T>
  int upload(const std::vector<T>& h, T** out) {
    void* p = f5h::dev_alloc(dev, h.size() * sizeof(T) + 16, mstream);
    if (!p) return f5h_internal_fail(F5H_EHIP, "vocos device allocation");
    allocs.push_back(p);
    VHIP(hipMemcpyAsync(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, mstream));
    VHIP(hipStreamSynchronize(mstream));
    *out = reinterpret_cast<T*>(p);
    return 0;
  }
  // panel [N][K] (host, fp32, K already padded) -> device [Npad][K] in the given compute dtype
  int lin(const std::vector<float>& w, int N, int K, const std::vector<float>& bias, int compute, VLin* L) {
    L->N = N;
    L->K = K;
    L->Npad = (N + 127) / 128 * 128;
    L->compute = compute;
    std::vector<float> wp((size_t)L->Npad * K, 0.f);
    std::copy(w.begin(), w.end(), wp.begin());
    if (compute) {
      std::vector<uint16_t> b16(wp.size());
      for (size_t i = 0; i < wp.size(); ++i) b16[i] = f2bf_bits(wp[i]);
      uint16_t* p;
      VRC(upload(b16, &p));
      L->w = p;
    } else {
      float* p;
      VRC(upload(wp, &p));
      L->w = p;
    }
    if (!bias.empty()) {
      std::vector<float> bv(L->Npad, 0.f);
      std::copy(bias.begin(), bias.end(), bv.begin());
      VRC(upload(bv, &L->b));
    }
    return 0;
  }
};

namespace {

struct VW {
  std::unordered_map<std::string, std::pair<const float*, int64_t>> m;
  const float* get(const std::string& n, int64_t numel, std::string* err) const {
    auto it = m.find(n);
    if (it == m.end()) {
      *err = "missing vocos weight " + n;
      return nullptr;
    }
    if (it->second.second != numel) {
      *err = "vocos weight " + n + " has " + std::to_string(it->second.second) + " elements, expected " +
             std::to_string(numel);
      return nullptr;
    }
    return it->second.first;
  }
};

#define VGET(var, name, numel)                                      \
  const float* var = W.get(name, numel, &err);                      \
  if (!var) return f5h_internal_fail(F5H_ENOWEIGHT, err)

int vec(f5h_vocos* v, const float* p, int64_t n, float** out) { return v->upload(std::vector<float>(p, p + n), out); }

// LayerNorm(affine) runs on ln_modulate: LN(x) * (1 + scale) + shift with scale = g - 1, shift = b.
int ln_params(f5h_vocos* v, const float* g, const float* b, int d, float** shift, float** sm1) {
  std::vector<float> s(d);
  for (int i = 0; i < d; ++i) s[i] = g[i] - 1.f;
  VRC(v->upload(s, sm1));
  return vec(v, b, d, shift);
}

int pack(f5h_vocos* v, const VW& W) {
  const f5h_vocos_arch& a = v->a;
  const int C = a.input_channels, d = a.dim, I = a.intermediate_dim, nf = a.n_fft;
  std::string err;
  // embed Conv1d(C, d, k7, pad 3): panel row o, column c*7 + j (the im2col order)
  {
    VGET(w, "backbone.embed.weight", (int64_t)d * C * 7);
    VGET(b, "backbone.embed.bias", d);
    std::vector<float> p((size_t)d * v->kemb, 0.f);
    for (int o = 0; o < d; ++o)
      for (int k = 0; k < C * 7; ++k) p[(size_t)o * v->kemb + k] = w[(size_t)o * C * 7 + k];
    VRC(v->lin(p, d, v->kemb, std::vector<float>(b, b + d), v->bf, &v->embed));
  }
  {
    VGET(g, "backbone.norm.weight", d);
    VGET(b, "backbone.norm.bias", d);
    VRC(ln_params(v, g, b, d, &v->norm_b, &v->norm_sm1));
  }
  v->blocks.resize(a.num_layers);
  for (int l = 0; l < a.num_layers; ++l) {
    const std::string pf = "backbone.convnext." + std::to_string(l) + ".";
    VBlock& B = v->blocks[l];
    VGET(dw, pf + "dwconv.weight", (int64_t)d * 7);
    VGET(dwb, pf + "dwconv.bias", d);
    VGET(lw, pf + "norm.weight", d);
    VGET(lb, pf + "norm.bias", d);
    VGET(w1, pf + "pwconv1.weight", (int64_t)I * d);
    VGET(b1, pf + "pwconv1.bias", I);
    VGET(w2, pf + "pwconv2.weight", (int64_t)d * I);
    VGET(b2, pf + "pwconv2.bias", d);
    VGET(gm, pf + "gamma", d);
    VRC(vec(v, dw, (int64_t)d * 7, &B.dw_w));
    VRC(vec(v, dwb, d, &B.dw_b));
    VRC(vec(v, lw, d, &B.ln_w));
    VRC(vec(v, lb, d, &B.ln_b));
    VRC(vec(v, gm, d, &B.gamma));
    VRC(v->lin(std::vector<float>(w1, w1 + (size_t)I * d), I, d, std::vector<float>(b1, b1 + I), v->bf, &B.pw1));
    VRC(v->lin(std::vector<float>(w2, w2 + (size_t)d * I), d, I, std::vector<float>(b2, b2 + d), v->bf, &B.pw2));
  }
  {
    VGET(g, "backbone.final_layer_norm.weight", d);
    VGET(b, "backbone.final_layer_norm.bias", d);
    VRC(ln_params(v, g, b, d, &v->fnorm_b, &v->fnorm_sm1));
  }
  // head Linear(d, n_fft + 2), rows interleaved: packed row 2k = magnitude row k, 2k+1 = phase row k
  {
    const int bins = v->bins, No = 2 * bins;
    VGET(w, "head.out.weight", (int64_t)No * d);
    VGET(b, "head.out.bias", No);
    std::vector<float> p((size_t)No * d), pb(No);
    for (int k = 0; k < bins; ++k) {
      std::memcpy(&p[(size_t)(2 * k) * d], w + (size_t)k * d, d * sizeof(float));
      std::memcpy(&p[(size_t)(2 * k + 1) * d], w + (size_t)(bins + k) * d, d * sizeof(float));
      pb[2 * k] = b[k];
      pb[2 * k + 1] = b[bins + k];
    }
    VRC(v->lin(p, No, d, pb, 0, &v->head));
  }
  // iDFT basis with the periodic Hann window folded in (torch.hann_window(n_fft), vocos ISTFT):
  // frame[n] = win[n]/N * (Re X_0 + Re X_{N/2} (-1)^n + 2 sum_{0<k<N/2} (Re X_k cos - Im X_k sin)(2 pi k n / N))
  {
    std::vector<float> basis((size_t)nf * v->kd, 0.f), win(nf);
    for (int n = 0; n < nf; ++n) {
      const double wn = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / nf);
      win[n] = (float)wn;
      for (int k = 0; k < v->bins; ++k) {
        const double wk = (k == 0 || 2 * k == nf) ? 1.0 : 2.0;
        const double ang = 2.0 * M_PI * (double)(((int64_t)k * n) % nf) / nf;
        basis[(size_t)n * v->kd + 2 * k] = (float)(wk * std::cos(ang) * wn / nf);
        basis[(size_t)n * v->kd + 2 * k + 1] = (float)(-wk * std::sin(ang) * wn / nf);
      }
    }
    VRC(v->lin(basis, nf, v->kd, std::vector<float>(), 0, &v->idft));
    VRC(v->upload(win, &v->win));
  }
  return 0;
}

struct VWS {
  size_t off = 0;
  char* base = nullptr;
  template <typename T>
  T* take(size_t n) {
    const size_t o = off;
    off = (off + n * sizeof(T) + 255) / 256 * 256;
    return base ? reinterpret_cast<T*>(base + o) : nullptr;
  }
};
struct VBufs {
  void *col, *dwln, *hid;
  float *x0, *x, *fln, *spec, *frames;
};
void vlayout(const f5h_vocos* v, VWS& ws, VBufs& b, int B, int T) {
  const size_t R = (size_t)B * T, es = v->bf ? 2 : 4;
  const f5h_vocos_arch& a = v->a;
  b.col = ws.take<char>(R * v->kemb * es);
  b.x0 = ws.take<float>(R * a.dim);
  b.x = ws.take<float>(R * a.dim);
  b.dwln = ws.take<char>(R * a.dim * es);
  b.hid = ws.take<char>(R * a.intermediate_dim * es);
  b.fln = ws.take<float>(R * a.dim);
  b.spec = ws.take<float>(R * v->kd);
  b.frames = ws.take<float>(R * a.n_fft);
}

GemmArgs vg(const void* A, int64_t lda, const VLin& W, int M, void* C, int64_t ldc) {
  GemmArgs g{};
  g.A = A;
  g.lda = lda;
  g.W = W.w;
  g.ldw = W.K;
  g.M = M;
  g.N = W.N;
  g.K = W.K;
  g.bias = W.b;
  g.C = C;
  g.ldc = ldc;
  return g;
}

}  // namespace

#define VK(x)                                                                                     \
  do {                                                                                            \
    hipError_t _e = (x);                                                                          \
    if (_e != hipSuccess) return f5h_internal_fail(F5H_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

int f5h_vocos_create(const f5h_vocos_arch* arch, const f5h_weight* weights, int32_t n_weights, int32_t device,
                     f5h_vocos** out) {
  if (!out || !arch || (n_weights > 0 && !weights)) return f5h_internal_fail(F5H_EINVAL, "null argument");
  *out = nullptr;
  const f5h_vocos_arch& a = *arch;
  if (a.input_channels <= 0 || a.input_channels * 7 > 4096 || a.dim <= 0 || a.dim % 64 || a.dim > 1024 ||
      a.intermediate_dim <= 0 || a.intermediate_dim % 64 || a.num_layers < 0 || a.n_fft <= 0 || a.n_fft % 2 ||
      a.hop_length <= 0 || a.n_fft % a.hop_length || (a.compute != F5H_FP32 && a.compute != F5H_BF16))
    return f5h_internal_fail(F5H_EINVAL, "bad vocos arch (dim, intermediate_dim multiples of 64, dim <= 1024, "
                                         "n_fft even and a multiple of hop_length)");
  VHIP(hipSetDevice(device));
  f5h_vocos* v = new f5h_vocos();
  v->a = a;
  v->dev = device;
  if (hipStreamCreateWithFlags(&v->mstream, hipStreamNonBlocking) != hipSuccess) {
    delete v;
    return f5h_internal_fail(F5H_EHIP, "vocos stream");
  }
  v->bf = a.compute == F5H_BF16;
  v->kemb = (a.input_channels * 7 + 63) / 64 * 64;
  v->bins = a.n_fft / 2 + 1;
  v->kd = (2 * v->bins + 63) / 64 * 64;
  VW W;
  for (int i = 0; i < n_weights; ++i) W.m[weights[i].name] = {weights[i].data, weights[i].numel};
  const int rc = pack(v, W);
  if (rc) {
    f5h_vocos_destroy(v);
    return rc;
  }
  *out = v;
  return 0;
}

// Returns at once; the reaper thread waits for this object's own last-use events, then frees it
// (no device-wide synchronisation, reaper.h).
void f5h_vocos_destroy(f5h_vocos* v) {
  if (!v) return;
  f5h::retire(v->dev, [v] {
    for (hipEvent_t ev : v->uses.take()) {
      (void)hipEventSynchronize(ev);
      (void)hipEventDestroy(ev);
    }
    for (void* p : v->allocs) f5h::dev_free(p, v->mstream);
    if (v->mstream) (void)hipStreamDestroy(v->mstream);
    delete v;
  });
}

size_t f5h_vocos_workspace_size(const f5h_vocos* v, int32_t B, int32_t T) {
  if (!v || B <= 0 || T <= 0) return 0;
  VWS ws;
  VBufs b;
  vlayout(v, ws, b, B, T);
  return ws.off;
}

int f5h_vocos_decode(f5h_vocos* v, void* stream, int32_t B, int32_t T, const float* mel, float* audio,
                     void* workspace, size_t workspace_bytes) {
  if (!v) return f5h_internal_fail(F5H_EINVAL, "null vocos");
  if (B <= 0 || T <= 0 || (int64_t)B * T > (1 << 24)) return f5h_internal_fail(F5H_EINVAL, "bad B/T");
  if (!mel || (T > 1 && !audio) || !workspace) return f5h_internal_fail(F5H_EINVAL, "null tensor argument");
  VWS ws;
  VBufs b;
  vlayout(v, ws, b, B, T);
  if (workspace_bytes < ws.off)
    return f5h_internal_fail(F5H_ENOMEM, "vocos workspace too small: need " + std::to_string(ws.off) + " have " +
                                             std::to_string(workspace_bytes));
  ws.off = 0;
  ws.base = reinterpret_cast<char*>(workspace);
  vlayout(v, ws, b, B, T);
  VHIP(hipSetDevice(v->dev));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  f5h::UseNote used{v->uses, st};
  const f5h_vocos_arch& a = v->a;
  const int R = B * T, d = a.dim, I = a.intermediate_dim, bf = v->bf;
  // backbone (vocos VocosBackbone.forward): embed -> LayerNorm -> ConvNeXt blocks -> final LayerNorm
  VK(vocos_im2col(bf, mel, B, T, a.input_channels, v->kemb, b.col, st));
  VK(gemm(bf, EPI_STORE, vg(b.col, v->kemb, v->embed, R, b.x0, d), st));
  VK(ln_modulate(0, b.x0, 0, R, d, v->norm_b, v->norm_sm1, b.x, st));
  for (const VBlock& blk : v->blocks) {
    VK(dwconv_ln(bf, b.x, B, T, d, blk.dw_w, blk.dw_b, blk.ln_w, blk.ln_b, b.dwln, st));
    VK(gemm(bf, EPI_GELU_ERF_OP, vg(b.dwln, d, blk.pw1, R, b.hid, I), st));
    GemmArgs g = vg(b.hid, I, blk.pw2, R, b.x, d);
    g.gate = blk.gamma;  // x += gamma * pwconv2(.)
    VK(gemm(bf, EPI_RESID, g, st));
  }
  VK(ln_modulate(0, b.x, 0, R, d, v->fnorm_b, v->fnorm_sm1, b.fln, st));
  // head (ISTFTHead.forward), fp32: Linear -> (mag, phase) -> (re, im) -> iDFT frames -> overlap-add
  VK(gemm(0, EPI_STORE, vg(b.fln, d, v->head, R, b.spec, v->kd), st));
  VK(vocos_spec(b.spec, R, v->bins, v->kd, st));
  VK(gemm(0, EPI_STORE, vg(b.spec, v->kd, v->idft, R, b.frames, a.n_fft), st));
  VK(vocos_ola(b.frames, v->win, B, T, a.n_fft, a.hop_length, audio, st));
  return 0;
}
