// C ABI of the log-mel front end (include/f5h.h, f5h_mel_*): SURVEY §8(f2), the step before the
// CFM path (cfm.py:106-108 turns raw-audio conditioning into vocos log-mels).
//
// Per call (R = B*T frames): frames [R][n_fft] fp32 (reflect-padded, unwindowed) -> DFT GEMM
// against a fixed basis [2*bins][n_fft] with the periodic Hann window folded in -> spec [R][Ks]
// (re, im interleaved) -> |X| [R][Km] -> filterbank GEMM [n_mels][Km] -> log(clamp(., 1e-5))
// transposed to [B][n_mels][T]. All fp32 (v_mfma_f32_16x16x4_f32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/f5h.h"
#include "capi_util.h"
#include "kernels.h"
#include "reaper.h"

using namespace f5h;

#define MHIP(x)                                                                                   \
  do {                                                                                            \
    hipError_t _e = (x);                                                                          \
    if (_e != hipSuccess) return f5h_internal_fail(F5H_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct f5h_mel {
  f5h::UseLog uses;  // per stream, an event after the last call: what *_destroy waits for
  f5h_mel_arch a{};
  int dev = 0, bins = 0, ks = 0, km = 0;
  float *dft = nullptr, *fb = nullptr;  // [Npad][K] fp32 GEMM panels
  int dft_npad = 0, fb_npad = 0;
  std::vector<void*> allocs;
  hipStream_t mstream = nullptr;  // uploads at creation, stream-ordered frees at release (reaper.h)
  int upload(const std::vector<float>& h, float** out) {
    void* p = f5h::dev_alloc(dev, h.size() * sizeof(float) + 16, mstream);
    if (!p) return f5h_internal_fail(F5H_EHIP, "mel device allocation");
    allocs.push_back(p);
    MHIP(hipMemcpyAsync(p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, mstream));
    MHIP(hipStreamSynchronize(mstream));
    *out = reinterpret_cast<float*>(p);
    return 0;
  }
};

namespace {

// torchaudio.functional.melscale_fbanks(n_freqs, f_min=0, f_max=sr//2, n_mels, sr, norm=None,
// mel_scale="htk"): triangular filters on the HTK mel scale, fb[k][m] for frequency bin k.
std::vector<double> htk_fbanks(int n_freqs, double f_max, int n_mels, int sr) {
  auto hz2mel = [](double f) { return 2595.0 * std::log10(1.0 + f / 700.0); };
  auto mel2hz = [](double m) { return 700.0 * (std::pow(10.0, m / 2595.0) - 1.0); };
  std::vector<double> freqs(n_freqs), fpts(n_mels + 2), fb((size_t)n_freqs * n_mels, 0.0);
  for (int k = 0; k < n_freqs; ++k) freqs[k] = n_freqs > 1 ? (double)(sr / 2) * k / (n_freqs - 1) : 0.0;
  const double m0 = hz2mel(0.0), m1 = hz2mel(f_max);
  for (int i = 0; i < n_mels + 2; ++i) fpts[i] = mel2hz(m0 + (m1 - m0) * i / (n_mels + 1));
  for (int k = 0; k < n_freqs; ++k)
    for (int m = 0; m < n_mels; ++m) {
      const double down = (freqs[k] - fpts[m]) / (fpts[m + 1] - fpts[m]);
      const double up = (fpts[m + 2] - freqs[k]) / (fpts[m + 2] - fpts[m + 1]);
      fb[(size_t)k * n_mels + m] = std::max(0.0, std::min(down, up));
    }
  return fb;
}

struct MBufs {
  float *frames, *spec, *mag, *melb;
};
size_t mlayout(const f5h_mel* m, int B, int T, char* base, MBufs* b) {
  size_t off = 0;
  auto take = [&](size_t n) {
    const size_t o = off;
    off = (off + n * sizeof(float) + 255) / 256 * 256;
    return base ? reinterpret_cast<float*>(base + o) : nullptr;
  };
  const size_t R = (size_t)B * T;
  b->frames = take(R * m->a.n_fft);
  b->spec = take(R * m->ks);
  b->mag = take(R * m->km);
  b->melb = take(R * m->a.n_mels);
  return off;
}

}  // namespace

int f5h_mel_create(const f5h_mel_arch* arch, int32_t device, f5h_mel** out) {
  if (!arch || !out) return f5h_internal_fail(F5H_EINVAL, "null argument");
  *out = nullptr;
  const f5h_mel_arch& a = *arch;
  if (a.n_fft <= 0 || a.n_fft % 32 || a.hop_length <= 0 || a.n_mels <= 0 || a.n_mels > 512 || a.sample_rate <= 0)
    return f5h_internal_fail(F5H_EINVAL, "bad mel arch (n_fft a positive multiple of 32, n_mels <= 512)");
  MHIP(hipSetDevice(device));
  f5h_mel* m = new f5h_mel();
  m->a = a;
  m->dev = device;
  if (hipStreamCreateWithFlags(&m->mstream, hipStreamNonBlocking) != hipSuccess) {
    delete m;
    return f5h_internal_fail(F5H_EHIP, "mel stream");
  }
  m->bins = a.n_fft / 2 + 1;
  m->ks = (2 * m->bins + 63) / 64 * 64;
  m->km = (m->bins + 31) / 32 * 32;
  const int nf = a.n_fft, bins = m->bins;
  // DFT basis, window folded in: row 2k = w[n] cos(2 pi k n / N), row 2k+1 = -w[n] sin(2 pi k n / N)
  m->dft_npad = (2 * bins + 127) / 128 * 128;
  std::vector<float> dft((size_t)m->dft_npad * nf, 0.f);
  for (int k = 0; k < bins; ++k)
    for (int n = 0; n < nf; ++n) {
      const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / nf);
      const double ang = 2.0 * M_PI * (double)(((int64_t)k * n) % nf) / nf;
      dft[(size_t)(2 * k) * nf + n] = (float)(w * std::cos(ang));
      dft[(size_t)(2 * k + 1) * nf + n] = (float)(-w * std::sin(ang));
    }
  // filterbank panel [n_mels][km]: row m = fb[:, m]
  const std::vector<double> fbk = htk_fbanks(bins, (double)(a.sample_rate / 2), a.n_mels, a.sample_rate);
  m->fb_npad = (a.n_mels + 127) / 128 * 128;
  std::vector<float> fb((size_t)m->fb_npad * m->km, 0.f);
  for (int mm = 0; mm < a.n_mels; ++mm)
    for (int k = 0; k < bins; ++k) fb[(size_t)mm * m->km + k] = (float)fbk[(size_t)k * a.n_mels + mm];
  int rc = m->upload(dft, &m->dft);
  if (!rc) rc = m->upload(fb, &m->fb);
  if (rc) {
    f5h_mel_destroy(m);
    return rc;
  }
  *out = m;
  return 0;
}

// Returns at once; the reaper thread waits for this object's own last-use events, then frees it
// (no device-wide synchronisation, reaper.h).
void f5h_mel_destroy(f5h_mel* m) {
  if (!m) return;
  f5h::retire(m->dev, [m] {
    for (hipEvent_t ev : m->uses.take()) {
      (void)hipEventSynchronize(ev);
      (void)hipEventDestroy(ev);
    }
    for (void* p : m->allocs) f5h::dev_free(p, m->mstream);
    if (m->mstream) (void)hipStreamDestroy(m->mstream);
    delete m;
  });
}

size_t f5h_mel_workspace_size(const f5h_mel* m, int32_t B, int32_t L) {
  if (!m || B <= 0 || L <= 0) return 0;
  MBufs b;
  return mlayout(m, B, 1 + L / m->a.hop_length, nullptr, &b);
}

int f5h_mel_forward(f5h_mel* m, void* stream, int32_t B, int32_t L, const float* wav, float* mel, void* workspace,
                    size_t workspace_bytes) {
  if (!m) return f5h_internal_fail(F5H_EINVAL, "null mel");
  if (B <= 0 || L <= m->a.n_fft / 2) return f5h_internal_fail(F5H_EINVAL, "bad B/L (L must exceed n_fft/2)");
  if (!wav || !mel || !workspace) return f5h_internal_fail(F5H_EINVAL, "null tensor argument");
  const int T = 1 + L / m->a.hop_length;
  if ((int64_t)B * T > (1 << 24)) return f5h_internal_fail(F5H_EINVAL, "too many frames");
  MBufs b;
  const size_t need = mlayout(m, B, T, nullptr, &b);
  if (workspace_bytes < need)
    return f5h_internal_fail(F5H_ENOMEM, "mel workspace too small: need " + std::to_string(need));
  mlayout(m, B, T, reinterpret_cast<char*>(workspace), &b);
  MHIP(hipSetDevice(m->dev));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  f5h::UseNote used{m->uses, st};
  const int R = B * T, nf = m->a.n_fft;
  MHIP(mel_frames(wav, B, L, T, nf, m->a.hop_length, b.frames, st));
  GemmArgs g{};
  g.A = b.frames;
  g.lda = nf;
  g.W = m->dft;
  g.ldw = nf;
  g.M = R;
  g.N = 2 * m->bins;
  g.K = nf;
  g.C = b.spec;
  g.ldc = m->ks;
  MHIP(gemm(0, EPI_STORE, g, st));
  MHIP(mel_mag(b.spec, R, m->bins, m->ks, m->km, b.mag, st));
  GemmArgs f{};
  f.A = b.mag;
  f.lda = m->km;
  f.W = m->fb;
  f.ldw = m->km;
  f.M = R;
  f.N = m->a.n_mels;
  f.K = m->km;
  f.C = b.melb;
  f.ldc = m->a.n_mels;
  MHIP(gemm(0, EPI_STORE, f, st));
  MHIP(mel_log(b.melb, B, T, m->a.n_mels, mel, st));
  return 0;
}
