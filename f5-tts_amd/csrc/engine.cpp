// f5h engine: weight packing, workspace layout and the CFM.sample orchestration behind the
// C ABI declared in include/f5h.h. Host code; every kernel is enqueued on the caller's stream.
//
// Hot-path map (reference file:line -> what runs here):
//   cfm.py:211-216  t grid            -> host (caller), passed as t_grid
//   modules.py:852-862, 321-323, 342-344  time MLP + every AdaLN row for every step
//                                     -> three GEMMs before the loop (one table [nfe, depth*6d+2d])
//   dit.py:86-139 text embed (cached) -> text_embed + ConvNeXt kernels once per call (both branches)
//   dit.py:159-162 InputEmbedding.proj -> split: cond/text part hoisted (P), x part per step
//   modules.py:175-201 ConvPositionEmbedding -> conv_pos x2 (implicit-GEMM MFMA)
//   modules.py:743-757 DiTBlock x depth -> ln_modulate, QKV+RoPE GEMM, attention, out GEMM+gate,
//                                     ln_modulate, FFN1+GELU GEMM, FFN2 GEMM+gate
//   dit.py:367-368, cfm.py:190-191, torchdiffeq euler -> ln_modulate, proj_out GEMM, cfg_euler
//   cfm.py:223 final where            -> final_where
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/f5h.h"
#include "kernels.h"
#include "reaper.h"

using namespace f5h;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int f5h_internal_fail(int code, const std::string& msg) { return fail(code, msg); }
#define HIPCK(x)                                                                               \
  do {                                                                                         \
    hipError_t _e = (x);                                                                       \
    if (_e != hipSuccess) return fail(F5H_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define RC(x)              \
  do {                     \
    int _r = (x);          \
    if (_r) return _r;     \
  } while (0)

struct Lin {
  void* w = nullptr;      // [Npad][K] operand dtype
  float* b = nullptr;     // [Npad] fp32 (may be null)
  int N = 0, K = 0, Npad = 0;
};

struct CNX {
  float *dw_w = nullptr, *dw_b = nullptr, *ln_w = nullptr, *ln_b = nullptr, *gamma = nullptr, *beta = nullptr;
  Lin pw1, pw2;
};

struct Layer {
  Lin qkv, out, ff1, ff2, skip;  // skip: UNetT skip_proj [d][2d] over cat(x, skip) (later half)
  float *g_attn = nullptr, *g_ff = nullptr;  // UNetT RMSNorm gains
  Lin qkv_g, ff1_g;  // UNetT RMSNorm fold: qkv / ff1 with the norm's gain folded in, W diag(g) (same bias)
};

struct GraphKey {
  const void* ws;
  int kind;  // 0: one NFE step, 1: the call prologue (inputs staged into the workspace)
  int B, N, nt, nfe, use_cfg, batch_mask, probe, split, pad_skip, chain, lnfold;
  uint64_t kernel_epoch;  // bumped whenever a forced GEMM config changes
  uint32_t cfg_bits;
  bool operator==(const GraphKey& o) const {
    return ws == o.ws && kind == o.kind && B == o.B && N == o.N && nt == o.nt && nfe == o.nfe && kernel_epoch == o.kernel_epoch &&
           use_cfg == o.use_cfg && batch_mask == o.batch_mask && probe == o.probe && cfg_bits == o.cfg_bits &&
           split == o.split && pad_skip == o.pad_skip && chain == o.chain && lnfold == o.lnfold;
  }
};

struct f5h_engine {
  f5h_arch a{};
  int dev = 0;
  int bf = 0;          // compute mode (f5h_compute == ComputeMode): 0 fp32, 1 bf16, 2 fp16 operands
  size_t esz = 4;      // operand element size
  int tdp = 0;         // text_dim padded to 64
  std::vector<void*> allocs;  // device memory from the stream-ordered pool (dev_alloc), freed by the reaper
  hipStream_t mstream = nullptr;  // the engine's own stream: creation-time uploads/packing, frees at release
  Lin t1, t2, ada, in_x, in_ct, proj_out;
  float* text_table = nullptr;
  float* freqs = nullptr;
  std::vector<CNX> cnx;
  void* conv_w[2] = {nullptr, nullptr};
  float* conv_b[2] = {nullptr, nullptr};
  std::vector<Layer> layers;
  float* norm_out_g = nullptr;
  // hipGraph cache of one NFE step (keyed by the call's buffers and shape)
  std::mutex gm;
  std::vector<std::shared_ptr<struct GraphEntry>> graphs;
  // evicted entries whose replays may still be in flight: destroyed by a later graph_get once every
  // event recorded after their replays has completed and no caller holds them (no host wait)
  std::vector<std::shared_ptr<struct GraphEntry>> graveyard;
  std::vector<hipEvent_t> ev_pool;  // completed "replays done" events, reused
  // prologue keys seen once: the prologue is captured only when its shape repeats (a call with a
  // new shape runs it eagerly instead of paying capture + instantiate for one replay)
  std::vector<struct GraphKey> pro_seen;
  int64_t n_evicted = 0, n_reaped = 0;
  std::mutex hm;
  double last_host[8] = {};  // f5h_last_call_host_ms: the newest f5h_sample call's host phases
  hipStream_t cap = nullptr;  // private capture stream (the caller's may be the null stream)
  hipStream_t cap2 = nullptr; // second capture stream: the unconditional CFG branch
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int graph_mode = 1;
  // CFG branches as parallel captured chains: 1 = always, 0 = never, 2 = auto, which is one packed chain:
  // with the round-3 kernels the split measured C2 +2.3 %, C3 +1.0 %, C5 +1.0 % per call and C4 -0.7 %
  // (profiles/r03_ab_cfg_chains.txt; in round 1 it won C5 by 4 %). Env F5H_SPLIT_CFG, f5h_set_cfg_streams.
  int split_cfg = 2;
  // skip the dead pad-row work of the batch path (attention query blocks and out-proj row tiles of padding
  // only): f5h_set_pad_skip, env F5H_NO_PAD_SKIP=1 at creation turns it off. Bitwise identical results.
  int pad_skip = 1;
  // In-launch phase chain of the DiT block-step's row-local seams (chain.hip): f5h_set_chain, env F5H_CHAIN=1 at
  // creation turns it on. Bitwise identical results. OFF by default since round 6: with its counters correctly
  // re-zeroed on every graph replay it measured C2 58.4 vs 51.1 ms unchained (profiles/r06_ab_chain_c2.txt); the
  // round-5 gain came from a captured memset node that later replays did not apply (waits skipped, wrong results).
  int chain = 0;
  // LayerNorm fold (DESIGN.md §3 'LayerNorm fold'): on the 16-bit DiT path without row masks the AdaLN LayerNorms
  // between the residual GEMMs and their consumers run as algebra in those GEMMs (gemm_impl.h LNF) instead of as
  // launches of their own. f5h_set_ln_fold, env F5H_LNFOLD=0 at creation turns it off. lnf_ok: the engine supports
  // it (DiT, 16-bit, dim and ff a multiple of 64, dim <= 1024); lnf_w: device array [W1 of every layer, Wqkv of every
  // layer] for lnfold_uv; ada_row: floats per AdaLN table row (the modulation rows, then per layer the fold's u/v).
  // The same switch covers the UNetT RMSNorm fold (rmsf_ok: 16-bit UNetT, dim a multiple of 64, dim <= 1024; the
  // consumers read the residual stream with W diag(g), Layer::qkv_g / ff1_g).
  int lnfold = 1;
  bool lnf_ok = false, rmsf_ok = false;
  const void** lnf_w = nullptr;
  int64_t ada_row = 0;
  std::atomic<int64_t> n_lnfold{0};  // backbone passes enqueued with the fold
  // The chain's give-up word (chain.h): device memory of the engine, set by a chain wait that expired. The call's final
  // kernel then writes NaN results; a copy of it lands in a pinned host word (fault_host) at the end of every chained
  // call, and the engine's next call reads that word, fails with F5H_EHIP and switches the chain off.
  unsigned* chain_fault = nullptr;
  volatile unsigned* fault_host = nullptr;
  int fault_slot = -1;
  std::atomic<int64_t> n_chain{0};  // chain launches enqueued (eager launches and captures)
  uint64_t use_ctr = 0;
  int64_t n_captures = 0, n_replays = 0;
  // probe
  // Probed launches are timed on the device wall clock (s_memrealtime): GEMM and attention
  // kernels stamp themselves (DevProbe), the others get a stamp kernel on each side. Slots are
  // indexed by (launch site within a step, device step tick), so eager launches and graph
  // replays are timed alike. pstamp[0] (as int) = tick, bumped by every step; pslots =
  // pstamp + 64: kProbeSites x kProbeTicks start stamps, then as many end stamps.
  std::mutex pm;
  int probe_class = -1;
  unsigned long long* pstamp = nullptr;
  unsigned long long* pslots = nullptr;
  unsigned long long* ptl = nullptr;  // per-workgroup timeline of the first probed launch (kTimelineWG x 4)
  int* ptick = nullptr;
  double wall_khz = 0.0;
  // per stream, an event recorded after the last call's launches: what f5h_engine_destroy waits for
  UseLog uses;
};
static constexpr size_t kGraphCache = 16;  // cached graphs (prologue and step graphs together)
static constexpr size_t kProbeBytes = (64 + 2 * (size_t)kProbeEnd) * sizeof(unsigned long long);

// The step graph touches only workspace buffers (the ODE state, the trajectory base and the step
// index live in the workspace), so it is keyed by the workspace and the launch shape alone.
// Captured step graphs bake in the kernel choice: forcing a GEMM config or an attention variant
// (tuning/tests) moves the epoch so that later calls capture afresh.
static std::atomic<uint64_t> g_kernel_epoch{0};

// Shared by the cache and by every call replaying it: an entry evicted while another thread is
// still in its launch loop is destroyed by the last holder, after the device has drained (an
// already-submitted replay may still be executing).
struct GraphEntry {
  GraphKey key{};
  hipGraphExec_t exec = nullptr;
  uint64_t stamp = 0;
  std::vector<hipEvent_t> inflight;  // recorded after this entry's replays (guarded by f5h_engine::gm)
  // Destroyed only when nothing replays it any more: from the graveyard once `inflight` has
  // completed and no caller holds it, or by f5h_engine_destroy after a device synchronisation.
  ~GraphEntry() {
    if (exec) (void)hipGraphExecDestroy(exec);
    for (hipEvent_t ev : inflight) (void)hipEventDestroy(ev);
  }
};

// ---------------------------------------------------------------- weight packing
// Weights arrive as typed views (f5h_tensor_view: fp32/bf16/fp16, host or device memory, the
// reference's parameter dtype and placement, utils_infer.py:190-232). Host views are staged to the
// device once in their own dtype; every panel is then packed on the device by pack_strided
// (reorder, zero padding, rounding to the operand dtype), so no host fp32 copy of the model exists.
struct WView {
  const void* p;      // device pointer (staged when the caller's view was in host memory)
  int dt;             // f5h_dtype
  int64_t numel;
};
struct WMap {
  std::unordered_map<std::string, WView> m;
  const WView* get(const std::string& n, int64_t numel, std::string* err) const {
    auto it = m.find(n);
    if (it == m.end()) {
      *err = "missing weight " + n;
      return nullptr;
    }
    if (it->second.numel != numel) {
      *err = "weight " + n + " has " + std::to_string(it->second.numel) + " elements, expected " +
             std::to_string(numel);
      return nullptr;
    }
    return &it->second;
  }
};

// device buffer owned by the engine (stream-ordered pool, reaper.h: its release never syncs the device)
static int ealloc(f5h_engine* e, size_t bytes, void** out) {
  void* p = dev_alloc(e->dev, bytes, e->mstream);
  if (!p) return fail(F5H_EHIP, "device allocation of " + std::to_string(bytes) + " bytes");
  e->allocs.push_back(p);
  *out = p;
  return 0;
}

template <typename T>
static int upload(f5h_engine* e, const std::vector<T>& h, T** out) {
  void* p = nullptr;
  RC(ealloc(e, h.size() * sizeof(T) + 16, &p));
  HIPCK(hipMemcpyAsync(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, e->mstream));
  HIPCK(hipStreamSynchronize(e->mstream));  // the host vector may go away after the return
  *out = reinterpret_cast<T*>(p);
  return 0;
}

// zeroed device buffer owned by the engine
static int dalloc(f5h_engine* e, size_t bytes, void** out) {
  void* p = nullptr;
  RC(ealloc(e, bytes + 16, &p));
  HIPCK(hipMemsetAsync(p, 0, bytes + 16, e->mstream));
  *out = p;
  return 0;
}

// op element type of the engine (f5h_dtype numbering: 0 fp32, 1 bf16, 2 fp16 == f5h_compute)
static int op_dt(const f5h_engine* e) { return e->bf; }

// dst[r][dst_col + c] (row stride ld_dst, element type ddt) = src[r][col0 + c] (row stride ld_src)
static int pack_rows(const WView& v, int rows, int64_t ld_src, int col0, int ncols, void* dst, int ddt,
                     int64_t ld_dst, int dst_row0, int dst_col, hipStream_t st) {
  PackArgs pa{};
  pa.src = v.p;
  pa.src_dt = v.dt;
  pa.src_st[0] = 0;
  pa.src_st[1] = 0;
  pa.src_st[2] = ld_src;
  pa.src_st[3] = 1;
  const size_t esz = ddt ? 2 : 4;
  pa.dst = (char*)dst + ((size_t)dst_row0 * ld_dst + dst_col) * esz;
  // the source column offset goes into the base pointer
  pa.src = (const char*)v.p + (size_t)col0 * (v.dt ? 2 : 4);
  pa.dst_dt = ddt;
  pa.dst_st[0] = 0;
  pa.dst_st[1] = 0;
  pa.dst_st[2] = ld_dst;
  pa.n[0] = 1;
  pa.n[1] = 1;
  pa.n[2] = rows;
  pa.n[3] = ncols;
  HIPCK(pack_strided(pa, st));
  return 0;
}

// Build a GEMM panel [Npad][K] (operand dtype, zero padded) from column blocks of several source
// matrices stacked along N, plus an fp32 bias [Npad] from per-block bias vectors (null: zeros).
struct Block {
  const WView* src;   // [rows][ld]
  int rows, ld, col0, ncols, dst_col;
};
static int make_lin(f5h_engine* e, const std::vector<Block>& blocks, int K, const std::vector<const WView*>& biases,
                    Lin* L) {
  int N = 0;
  for (const Block& b : blocks) N += b.rows;
  L->N = N;
  L->K = K;
  L->Npad = (N + 127) / 128 * 128;
  RC(dalloc(e, (size_t)L->Npad * K * e->esz, &L->w));
  int r0 = 0;
  for (const Block& b : blocks) {
    RC(pack_rows(*b.src, b.rows, b.ld, b.col0, b.ncols, L->w, op_dt(e), K, r0, b.dst_col, e->mstream));
    r0 += b.rows;
  }
  if (!biases.empty()) {
    void* bp;
    RC(dalloc(e, (size_t)L->Npad * sizeof(float), &bp));
    L->b = reinterpret_cast<float*>(bp);
    r0 = 0;
    for (size_t i = 0; i < blocks.size(); ++i) {
      if (i < biases.size() && biases[i])
        RC(pack_rows(*biases[i], 1, 0, 0, blocks[i].rows, L->b, 0, 0, 0, r0, e->mstream));
      r0 += blocks[i].rows;
    }
  }
  return 0;
}
// Simple linear: weight [N][K] (K padded to 64), bias [N] or none.
static int lin_simple(f5h_engine* e, const WMap& W, const std::string& wn, const std::string& bn, int N, int K,
                      Lin* L, std::string* err) {
  const WView* w = W.get(wn, (int64_t)N * K, err);
  if (!w) return fail(F5H_ENOWEIGHT, *err);
  const WView* b = nullptr;
  if (!bn.empty()) {
    b = W.get(bn, N, err);
    if (!b) return fail(F5H_ENOWEIGHT, *err);
  }
  const int Kp = (K + 63) / 64 * 64;
  return make_lin(e, {Block{w, N, K, 0, K, 0}}, Kp, b ? std::vector<const WView*>{b} : std::vector<const WView*>{},
                  L);
}
// fp32 device copy of a vector parameter
static int vec_upload(f5h_engine* e, const WMap& W, const std::string& n, int64_t numel, float** out, std::string* err) {
  const WView* v = W.get(n, numel, err);
  if (!v) return fail(F5H_ENOWEIGHT, *err);
  void* p;
  RC(dalloc(e, (size_t)numel * sizeof(float), &p));
  RC(pack_rows(*v, 1, 0, 0, (int)numel, p, 0, 0, 0, 0, e->mstream));
  *out = reinterpret_cast<float*>(p);
  return 0;
}

static int pack_all(f5h_engine* e, const WMap& W) {
  const f5h_arch& a = e->a;
  const int d = a.dim, inner = a.heads * a.dim_head, F = a.ff_dim, td = a.text_dim, mel = a.mel_dim;
  const int V = a.text_num_embeds + 1;
  std::string err;
  // time MLP (modules.py:852-862)
  RC(lin_simple(e, W, "time_embed.time_mlp.0.weight", "time_embed.time_mlp.0.bias", d, 256, &e->t1, &err));
  RC(lin_simple(e, W, "time_embed.time_mlp.2.weight", "time_embed.time_mlp.2.bias", d, d, &e->t2, &err));
  // text table
  RC(vec_upload(e, W, "text_embed.text_embed.weight", (int64_t)V * td, &e->text_table, &err));
  if (a.conv_layers > 0) {
    // precompute_freqs_cis(text_dim, 8192) (modules.py:207-218)
    std::vector<float> fc((size_t)8192 * td);
    const int half = td / 2;
    for (int p = 0; p < 8192; ++p)
      for (int i = 0; i < half; ++i) {
        float f = 1.0f / std::pow(10000.0f, (float)(2 * i) / (float)td);
        float ang = (float)p * f;
        fc[(size_t)p * td + i] = std::cos(ang);
        fc[(size_t)p * td + half + i] = std::sin(ang);
      }
    RC(upload(e, fc, &e->freqs));
  }
  e->cnx.resize(a.conv_layers);
  for (int i = 0; i < a.conv_layers; ++i) {
    const std::string p = "text_embed.text_blocks." + std::to_string(i) + ".";
    CNX& c = e->cnx[i];
    RC(vec_upload(e, W, p + "dwconv.weight", (int64_t)td * 7, &c.dw_w, &err));
    RC(vec_upload(e, W, p + "dwconv.bias", td, &c.dw_b, &err));
    RC(vec_upload(e, W, p + "norm.weight", td, &c.ln_w, &err));
    RC(vec_upload(e, W, p + "norm.bias", td, &c.ln_b, &err));
    RC(vec_upload(e, W, p + "grn.gamma", 2 * td, &c.gamma, &err));
    RC(vec_upload(e, W, p + "grn.beta", 2 * td, &c.beta, &err));
    RC(lin_simple(e, W, p + "pwconv1.weight", p + "pwconv1.bias", 2 * td, td, &c.pw1, &err));
    RC(lin_simple(e, W, p + "pwconv2.weight", p + "pwconv2.bias", td, 2 * td, &c.pw2, &err));
  }
  // input projection split (dit.py:162): [x | cond | text] -> x part per step, cond|text hoisted
  {
    const int Kin = 2 * mel + td;
    const WView* w = W.get("input_embed.proj.weight", (int64_t)d * Kin, &err);
    const WView* b = w ? W.get("input_embed.proj.bias", d, &err) : nullptr;
    if (!w || !b) return fail(F5H_ENOWEIGHT, err);
    RC(make_lin(e, {Block{w, d, Kin, 0, mel, 0}}, 128, {}, &e->in_x));
    // cond columns -> [0,128), text columns -> [128, 128+tdp): two column blocks of the same rows
    const int Kct = 128 + e->tdp;
    Lin& L = e->in_ct;
    L.N = d;
    L.K = Kct;
    L.Npad = (d + 127) / 128 * 128;
    RC(dalloc(e, (size_t)L.Npad * Kct * e->esz, &L.w));
    RC(pack_rows(*w, d, Kin, mel, mel, L.w, op_dt(e), Kct, 0, 0, e->mstream));
    RC(pack_rows(*w, d, Kin, 2 * mel, td, L.w, op_dt(e), Kct, 0, 128, e->mstream));
    void* bp;
    RC(dalloc(e, (size_t)L.Npad * sizeof(float), &bp));
    L.b = reinterpret_cast<float*>(bp);
    RC(pack_rows(*b, 1, 0, 0, d, L.b, 0, 0, 0, 0, e->mstream));
  }
  // ConvPositionEmbedding: [d, d/16, 31] -> [16][31][64 out][64 in] (zero-padded to 64 channels):
  // dst (g, t, o, i) <- src ((g*cg + o)*cg + i)*31 + t
  for (int j = 0; j < 2; ++j) {
    const std::string p = "input_embed.conv_pos_embed.conv1d." + std::to_string(j * 2) + ".";
    const int cg = d / 16;
    const WView* w = W.get(p + "weight", (int64_t)d * cg * 31, &err);
    if (!w) return fail(F5H_ENOWEIGHT, err);
    RC(dalloc(e, (size_t)16 * 31 * 64 * 64 * e->esz, &e->conv_w[j]));
    PackArgs pa{};
    pa.src = w->p;
    pa.src_dt = w->dt;
    pa.src_st[0] = (int64_t)cg * cg * 31;  // g
    pa.src_st[1] = 1;                      // t
    pa.src_st[2] = (int64_t)cg * 31;       // o
    pa.src_st[3] = 31;                     // i
    pa.dst = e->conv_w[j];
    pa.dst_dt = op_dt(e);
    pa.dst_st[0] = 31 * 64 * 64;
    pa.dst_st[1] = 64 * 64;
    pa.dst_st[2] = 64;
    pa.n[0] = 16;
    pa.n[1] = 31;
    pa.n[2] = cg;
    pa.n[3] = cg;
    HIPCK(pack_strided(pa, e->mstream));
    RC(vec_upload(e, W, p + "bias", d, &e->conv_b[j], &err));
  }
  // blocks
  e->layers.resize(a.depth);
  std::vector<Block> ada_blocks;
  std::vector<const WView*> ada_bias;
  for (int l = 0; l < a.depth; ++l) {
    Layer& L = e->layers[l];
    const bool dit = a.backbone == F5H_DIT;
    const std::string p = dit ? "transformer_blocks." + std::to_string(l) + "." : "layers." + std::to_string(l) + ".";
    const std::string pa = dit ? p + "attn." : p + "2.";
    const std::string pf = dit ? p + "ff.ff." : p + "4.ff.";
    const WView* wq = W.get(pa + "to_q.weight", (int64_t)inner * d, &err);
    const WView* wk = wq ? W.get(pa + "to_k.weight", (int64_t)inner * d, &err) : nullptr;
    const WView* wv = wk ? W.get(pa + "to_v.weight", (int64_t)inner * d, &err) : nullptr;
    const WView* bq = wv ? W.get(pa + "to_q.bias", inner, &err) : nullptr;
    const WView* bk = bq ? W.get(pa + "to_k.bias", inner, &err) : nullptr;
    const WView* bv = bk ? W.get(pa + "to_v.bias", inner, &err) : nullptr;
    if (!wq || !wk || !wv || !bq || !bk || !bv) return fail(F5H_ENOWEIGHT, err);
    RC(make_lin(e, {Block{wq, inner, d, 0, d, 0}, Block{wk, inner, d, 0, d, 0}, Block{wv, inner, d, 0, d, 0}}, d,
                {bq, bk, bv}, &L.qkv));
    RC(lin_simple(e, W, pa + "to_out.0.weight", pa + "to_out.0.bias", d, inner, &L.out, &err));
    RC(lin_simple(e, W, pf + "0.0.weight", pf + "0.0.bias", F, d, &L.ff1, &err));
    RC(lin_simple(e, W, pf + "2.weight", pf + "2.bias", d, F, &L.ff2, &err));
    if (dit) {
      const WView* aw = W.get(p + "attn_norm.linear.weight", (int64_t)6 * d * d, &err);
      const WView* ab = aw ? W.get(p + "attn_norm.linear.bias", 6 * d, &err) : nullptr;
      if (!aw || !ab) return fail(F5H_ENOWEIGHT, err);
      ada_blocks.push_back(Block{aw, 6 * d, d, 0, d, 0});
      ada_bias.push_back(ab);
    } else {
      RC(vec_upload(e, W, p + "1.g", d, &L.g_attn, &err));
      RC(vec_upload(e, W, p + "3.g", d, &L.g_ff, &err));
      if (l >= a.depth / 2) {
        const WView* sw = W.get(p + "0.weight", (int64_t)d * 2 * d, &err);
        if (!sw) return fail(F5H_ENOWEIGHT, err);
        RC(make_lin(e, {Block{sw, d, 2 * d, 0, 2 * d, 0}}, 2 * d, {}, &L.skip));
      }
    }
  }
  if (a.backbone == F5H_DIT) {
    const WView* nw = W.get("norm_out.linear.weight", (int64_t)2 * d * d, &err);
    const WView* nb = nw ? W.get("norm_out.linear.bias", 2 * d, &err) : nullptr;
    if (!nw || !nb) return fail(F5H_ENOWEIGHT, err);
    ada_blocks.push_back(Block{nw, 2 * d, d, 0, d, 0});
    ada_bias.push_back(nb);
    RC(make_lin(e, ada_blocks, d, ada_bias, &e->ada));
  } else {
    RC(vec_upload(e, W, "norm_out.g", d, &e->norm_out_g, &err));
  }
  RC(lin_simple(e, W, "proj_out.weight", "proj_out.bias", mel, d, &e->proj_out, &err));
  return 0;
}

// ---------------------------------------------------------------- workspace layout
struct WS {
  size_t off = 0;
  char* base = nullptr;
  template <typename T>
  T* take(size_t n) {
    size_t o = off;
    off = (off + n * sizeof(T) + 255) / 256 * 256;
    return base ? reinterpret_cast<T*>(base + o) : nullptr;
  }
};

struct Bufs {
  float *tsin, *th, *temb, *ada;
  void* tin_op;
  float *te, *pw1o, *grn_scr;
  void *dwln, *grno;
  uint8_t* keepfill;
  void* act;
  float* P;
  void* ypad;
  float *h0, *h, *p;
  void *c1, *aop, *q, *k, *v, *o, *f;
  float2* rope;
  uint8_t* rowkeep;
  int32_t* kvlen;
  float* lnp;          // LayerNorm fold partial statistics [rows][d / 64][2]
  unsigned* chain;     // phase-chain arrival counters: [depth][5][chain_g4] (the chain runs on the packed batch only)
  int chain_g4;        // row groups per counter row, rounded up to 4 (16-B rows)
  float *ada_cur, *temb_cur, *tgrid;  // the current step's table rows; device copy of the grid
  int* kstep;                         // device-side NFE step index
  float* y;                           // ODE state [B][N][mel] fp32
  float** trajp;                      // device slot: trajectory base pointer (or null)
  // UNetT residual stream (operand dtype): xs[0..depth/2] -- layer l < depth/2 reads xs[l] (its
  // skip connection, kept) and writes xs[l+1]; later layers ping-pong between pp[0] and pp[1]
  std::vector<void*> xs;
  void* pp[2];
  // the call's inputs staged into the workspace (prologue graph): cond [B][N][mel] fp32,
  // cond_mask [B][N], text [B][<= N] (int64), duration [B]
  float* in_cond;
  uint8_t* in_mask;
  int64_t* in_text;
  int32_t* in_dur;
};

static void layout(const f5h_engine* e, WS& ws, Bufs& b, int B, int N, int nfe, int use_cfg) {
  const f5h_arch& a = e->a;
  const int d = a.dim, td = a.text_dim, S = use_cfg ? 2 * B : B;
  const int L = a.backbone == F5H_DIT ? N : N + 1;
  const size_t rows = (size_t)S * L, es = e->esz;
  const int inner = a.heads * 64;
  b.tsin = ws.take<float>((size_t)nfe * 256);
  b.th = ws.take<float>((size_t)nfe * d);
  b.temb = ws.take<float>((size_t)nfe * d);
  b.tin_op = ws.take<char>((size_t)nfe * std::max(256, d) * es);
  b.ada = a.backbone == F5H_DIT ? ws.take<float>((size_t)nfe * e->ada_row) : nullptr;
  b.te = ws.take<float>((size_t)2 * B * N * td);
  b.keepfill = ws.take<uint8_t>((size_t)2 * B * N);
  if (a.conv_layers > 0) {
    b.dwln = ws.take<char>((size_t)2 * B * N * td * es);
    b.pw1o = ws.take<float>((size_t)2 * B * N * 2 * td);
    b.grno = ws.take<char>((size_t)2 * B * N * 2 * td * es);
    b.grn_scr = ws.take<float>((size_t)((N + 63) / 64 + 1) * 2 * B * 2 * td);
  } else {
    b.dwln = b.grno = nullptr;
    b.pw1o = b.grn_scr = nullptr;
  }
  b.act = ws.take<char>((size_t)S * N * (128 + e->tdp) * es);
  b.P = ws.take<float>((size_t)S * N * d);
  b.ypad = ws.take<char>((size_t)B * N * 128 * es);
  b.h0 = ws.take<float>((size_t)S * N * d);
  b.c1 = ws.take<char>((size_t)S * N * d * es);
  b.h = a.backbone == F5H_DIT ? ws.take<float>(rows * d) : nullptr;  // DiT residual stream
  b.aop = ws.take<char>(rows * d * es);
  b.q = ws.take<char>(rows * inner * es);
  b.k = ws.take<char>(rows * inner * es);
  b.v = ws.take<char>(rows * inner * es);
  b.o = ws.take<char>(rows * inner * es);
  b.f = ws.take<char>(rows * a.ff_dim * es);
  b.p = ws.take<float>(rows * e->proj_out.Npad);  // proj_out rows padded to the GEMM tile width
  b.rope = ws.take<float2>((size_t)L * 32);
  b.rowkeep = ws.take<uint8_t>(rows);
  b.kvlen = ws.take<int32_t>(S);
  b.chain_g4 = ((int)((rows + kChainRows - 1) / kChainRows) + 3) / 4 * 4;
  b.chain = a.backbone == F5H_DIT ? ws.take<unsigned>((size_t)a.depth * 5 * b.chain_g4) : nullptr;
  b.ada_cur = a.backbone == F5H_DIT ? ws.take<float>((size_t)e->ada_row) : nullptr;
  // LayerNorm fold: per row and 64-column strip of the residual stream, (mean, M2) (float2)
  b.lnp = (e->lnf_ok || e->rmsf_ok) ? ws.take<float>(rows * (size_t)(d / 64) * 2) : nullptr;
  b.temb_cur = ws.take<float>((size_t)d);
  b.tgrid = ws.take<float>((size_t)nfe);
  b.kstep = ws.take<int>(64);
  b.y = ws.take<float>((size_t)B * N * e->a.mel_dim);
  b.trajp = ws.take<float*>(8);
  b.in_cond = ws.take<float>((size_t)B * N * a.mel_dim);
  b.in_mask = ws.take<uint8_t>((size_t)B * N);
  b.in_text = ws.take<int64_t>((size_t)B * N);
  b.in_dur = ws.take<int32_t>((size_t)B);
  b.xs.clear();
  b.pp[0] = b.pp[1] = nullptr;
  if (a.backbone == F5H_UNETT) {
    for (int i = 0; i <= a.depth / 2; ++i) b.xs.push_back(ws.take<char>(rows * d * es));
    b.pp[0] = ws.take<char>(rows * d * es);
    b.pp[1] = ws.take<char>(rows * d * es);
  }
}

// ---------------------------------------------------------------- probe
enum { KC_FFN1 = 0, KC_ATTN = 1, KC_QKV = 2, KC_FFN2 = 3, KC_CONV = 4, KC_OUT = 5, KC_NORM = 6, KC_CHAIN = 7 };
// Times one launch site when its kernel class is probed. With `kp` the kernel stamps itself
// (GemmArgs/AttnArgs::probe); without, stamp kernels bracket the launch.
struct ProbeScope {
  f5h_engine* e;
  hipStream_t st;
  bool on;
  bool self = false;
  unsigned long long* slots = nullptr;
  ProbeScope(f5h_engine* e_, int kc, hipStream_t s, int* site, DevProbe* kp = nullptr)
      : e(e_), st(s), on(e_->probe_class == kc && e_->pslots && *site < kProbeSites) {
    if (!on) return;
    const int s0 = (*site)++;
    slots = e->pslots + (size_t)s0 * kProbeRow;
    if (kp) {
      self = true;
      kp->slots = slots;
      kp->tick = e->ptick;
      kp->tl = s0 == 0 ? e->ptl : nullptr;  // the class's first launch site of a step, tick 0
    } else {
      (void)stamp_begin(slots, e->ptick, st);
    }
  }
  ~ProbeScope() {
    if (on && !self) (void)stamp_end(slots, e->ptick, st);
  }
};

// ---------------------------------------------------------------- forward pieces
struct Ctx {
  f5h_engine* e;
  hipStream_t st;
  Bufs b;
  int B, N, nt, S, L, nfe, use_cfg, batch_mask;
  int drop_audio, drop_text;  // single-branch forward only (f5h_forward with cfg_infer = 0)
  hipStream_t st2;            // second stream for the unconditional branch (step-graph capture), or null
  int site;  // probe launch-site counter, reset at the start of every step's enqueue
  int chain;  // this call may run the phase chain (engine switch, shape, and chain_admit's per-device check)
  int lnfold;  // this call runs the LayerNorm fold (engine switch, shape; never beside the chain)
  double* hp;  // host milliseconds of the call by phase (kHostPhases, f5h_last_call_host_ms), or null
};
// Host time of an f5h_sample call by phase (f5h_last_call_host_ms): a call that blocks the host shows where.
enum { HP_TOTAL = 0, HP_PROLOGUE, HP_LOCK, HP_REAP, HP_CAPTURE, HP_INSTANTIATE, HP_LAUNCH, HP_FINAL, kHostPhases };
static double host_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static GemmArgs gargs(const void* A, int64_t lda, const Lin& W, int M, void* C, int64_t ldc) {
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

#define KCK(x)                                                                                  \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess) return fail(F5H_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// Everything that depends only on the call's inputs (not on y): time/AdaLN tables, text
// embedding, hoisted input projection, masks, rope table.
static int prologue(Ctx& c, const float* t_host, int nt_vals, const float* cond, const uint8_t* cond_mask,
                    const int64_t* text, const int32_t* duration, bool text_cached = false) {
  f5h_engine* e = c.e;
  const f5h_arch& a = e->a;
  const int d = a.dim, td = a.text_dim, bf = e->bf;
  Bufs& b = c.b;
  hipStream_t st = c.st;
  KCK(rope_table(c.L, b.rope, st));
  const int off = a.backbone == F5H_DIT ? 0 : 1;
  if (c.batch_mask) {
    KCK(build_rowkeep(duration, c.B, c.S, c.L, off, b.rowkeep, st));
    KCK(build_kvlen(duration, c.B, c.S, off, b.kvlen, st));
  }
  // ---- time embedding for every grid point used, then the AdaLN table
  {
    if (t_host)
      KCK(time_sinus(t_host, nt_vals, b.tsin, st));
    else
      KCK(time_sinus_dev(b.tgrid, nt_vals, b.tsin, st));  // prologue graph: grid uploaded beforehand
    KCK(f32_to_op(bf, b.tsin, (int64_t)nt_vals * 256, b.tin_op, st));
    GemmArgs g = gargs(b.tin_op, 256, e->t1, nt_vals, b.th, d);
    KCK(gemm(bf, EPI_SILU, g, st));
    KCK(f32_to_op(bf, b.th, (int64_t)nt_vals * d, b.tin_op, st));
    g = gargs(b.tin_op, d, e->t2, nt_vals, b.temb, d);
    KCK(gemm(bf, EPI_STORE, g, st));
    if (a.backbone == F5H_DIT) {
      KCK(silu_to_op(bf, b.temb, b.tin_op, (int64_t)nt_vals * d, st));
      g = gargs(b.tin_op, d, e->ada, nt_vals, b.ada, e->ada_row);
      KCK(gemm(bf, EPI_STORE, g, st));
      if (c.lnfold) {  // every step's u / v of the folded LayerNorms (kernels.h LnFoldArgs)
        LnFoldArgs la{};
        la.table = b.ada;
        la.stride = e->ada_row;
        la.out_off = e->ada.Npad;
        la.nfe = nt_vals;
        la.depth = a.depth;
        la.d = d;
        la.F = a.ff_dim;
        la.w1 = e->lnf_w;
        la.wqkv = e->lnf_w + a.depth;
        KCK(lnfold_uv(bf, la, st));
      }
    }
  }
  // ---- text embedding, both branches (cached once per call in the reference, dit.py:294-310);
  // text_cached: the plugin's kept embedding is already in the workspace (f5h_forward text_cache 2)
  if (!text_cached) {
    TextEmbArgs t{};
    t.text = text;
    t.B = c.B;
    t.nt = c.nt;
    t.N = c.N;
    t.td = td;
    t.seq_len = (a.backbone == F5H_DIT && c.batch_mask) ? duration : nullptr;
    t.table = e->text_table;
    t.freqs = a.conv_layers > 0 ? e->freqs : nullptr;
    t.mask_padding = a.text_mask_padding;
    t.out_c = b.te;
    t.out_u = b.te + (size_t)c.B * c.N * td;
    t.keep = b.keepfill;
    KCK(text_embed(t, st));
    const int S2 = 2 * c.B, R2 = S2 * c.N;
    for (int i = 0; i < a.conv_layers; ++i) {
      CNX& x = e->cnx[i];
      KCK(dwconv_ln(bf, b.te, S2, c.N, td, x.dw_w, x.dw_b, x.ln_w, x.ln_b, b.dwln, st));
      GemmArgs g = gargs(b.dwln, td, x.pw1, R2, b.pw1o, 2 * td);
      KCK(gemm(bf, EPI_GELU_ERF, g, st));
      KCK(grn(bf, b.pw1o, S2, c.N, 2 * td, x.gamma, x.beta, b.grn_scr, b.grno, st));
      g = gargs(b.grno, 2 * td, x.pw2, R2, b.te, td);
      g.rowkeep = a.text_mask_padding ? b.keepfill : nullptr;
      KCK(gemm(bf, EPI_RESID_FILL, g, st));
    }
  }
  // ---- hoisted input projection: P = [step_cond | text] . W_ct^T + b
  KCK(build_ct(bf, cond, cond_mask, b.te, b.te + (size_t)c.B * c.N * td, c.B, c.N, td, c.S, c.drop_audio,
               c.drop_text, b.act, st));
  GemmArgs g = gargs(b.act, 128 + e->tdp, e->in_ct, c.S * c.N, b.P, d);
  KCK(gemm(bf, EPI_STORE, g, st));
  return 0;
}

// kstep buffer (64 ints): [0] the step index, [kArrive] the Euler launch's arrival counter
constexpr int kArrive = 16;

// Copy the step's table row (k = *kstep) to the fixed per-step buffer the layers read.
static int step_prep(Ctx& c) {
  f5h_engine* e = c.e;
  if (e->a.backbone == F5H_DIT)
    KCK(step_begin(c.b.kstep, c.b.ada, e->ada_row, e->ada_row, c.b.ada_cur, c.st));
  else
    KCK(step_begin(c.b.kstep, c.b.temb, e->a.dim, e->a.dim, c.b.temb_cur, c.st));
  return 0;
}

// Sequences [s0, s0+ns) of the packed cond/uncond backbone forward for the current step, enqueued
// on `st`; result in b.p rows of those sequences. Every buffer is sequence-major, so a part works on
// pointer offsets of the packed buffers; sequences never interact, so a part computes exactly what
// the packed forward computes for its rows (bitwise: GEMM tile configurations agree bit for bit).
static int backbone_part(Ctx& c, int s0, int ns, hipStream_t st) {
  f5h_engine* e = c.e;
  const f5h_arch& a = e->a;
  const int d = a.dim, bf = e->bf, H = a.heads, inner = H * 64;
  const bool dit = a.backbone == F5H_DIT;
  const size_t es = e->esz;
  Bufs& b = c.b;
  const int BN = c.B * c.N;
  const int rows = ns * c.L;
  const size_t ro = (size_t)s0 * c.L;  // first row of the part (L rows per sequence)
  const size_t no = (size_t)s0 * c.N;  // first row in the N-row input-embedding buffers
  auto op = [&](void* base, size_t row, size_t width) -> void* { return (char*)base + row * width * es; };
  const uint8_t* keep = c.batch_mask ? b.rowkeep + ro : nullptr;
  // residual stream: the operand dtype (as the reference keeps it in the parameter dtype), i.e. 16 bit
  // in the bf16/fp16 modes for DiT and UNetT alike, fp32 in the fp32 parity mode
  static const bool res32 = [] {  // F5H_RES32=1: fp32 residual on the 16-bit DiT path (A/B)
    const char* v = getenv("F5H_RES32");
    return v && *v == '1';
  }();
  const bool r16 = bf != 0 && (!dit || !res32);
  // F5H_DIAG_SKIP_LN=1: timing-only diagnostic, the 16-bit DiT path skips its LayerNorm launches
  // (wrong results; bounds what removing those launches can save). Never set in tests or benches.
  static const bool skip_ln = [] {
    const char* v = getenv("F5H_DIAG_SKIP_LN");
    const bool on = v && *v == '1';
    if (on) std::fprintf(stderr, "[f5h] F5H_DIAG_SKIP_LN=1: LayerNorm launches skipped, results are WRONG (timing only)\n");
    return on;
  }();
  const bool do_ln = !(skip_ln && r16);
  const size_t hsz = r16 ? es : sizeof(float);
  auto res = [&](void* base) -> void* { return (char*)base + ro * d * hsz; };
  void* bh = dit ? res(b.h) : res(b.xs[0]);
  void* aop = op(b.aop, ro, d);
  void* q = op(b.q, ro, inner);
  void* k = op(b.k, ro, inner);
  void* v = op(b.v, ro, inner);
  void* o = op(b.o, ro, inner);
  void* f = op(b.f, ro, a.ff_dim);
  // ---- input embedding: h0 = y.Wx^T + P, conv position embedding. Sequence s reads y[s % B]; a
  // part holding both branches computes y.Wx^T once and adds both branches' hoisted P rows.
  {
    GemmArgs g = gargs(b.ypad, 128, e->in_x, BN, b.h0 + no * d, d);
    g.bias = nullptr;
    g.add = b.P + no * d;
    g.ld_add = d;
    g.dual_rows = ns == 2 * c.B ? BN : 0;
    KCK(gemm(bf, EPI_INPROJ, g, st));
    ConvArgs cv{};
    cv.S = ns;
    cv.L = c.N;
    cv.d = d;
    cv.rowkeep = dit ? keep : nullptr;  // UNetT's InputEmbedding passes no mask (unett.py:100)
    cv.x = b.h0 + no * d;
    cv.x_f32 = 1;
    cv.w = e->conv_w[0];
    cv.bias = e->conv_b[0];
    cv.mode = 0;
    cv.y = op(b.c1, no, d);
    {
      ProbeScope ps(e, KC_CONV, st, &c.site);
      KCK(conv_pos(bf, cv, st));
    }
    cv.x = op(b.c1, no, d);
    cv.x_f32 = bf ? 0 : 1;
    cv.w = e->conv_w[1];
    cv.bias = e->conv_b[1];
    cv.mode = r16 ? 2 : 1;
    cv.y = bh;
    cv.y_seq_stride = c.L;
    cv.y_row_off = dit ? 0 : 1;
    cv.resid = b.h0 + no * d;
    KCK(conv_pos(bf, cv, st));
  }
  if (!dit) KCK(write_time_token(bf, r16, b.temb_cur, ns, c.L, d, bh, st));

  const float* ada_k = dit ? b.ada_cur : nullptr;
  const int epi_resid = r16 ? EPI_RESID16 : EPI_RESID;
  void* h = bh;             // the layer's output (residual updates land here)
  const void* h_in = nullptr;  // UNetT first half: the layer input, kept as its skip connection
  auto qkv_args = [&](const Layer& Lq) {
    GemmArgs g = gargs(aop, d, Lq.qkv, rows, nullptr, 0);
    g.rope = b.rope;
    g.seq_len = c.L;
    g.heads = H;
    g.rope_heads = a.pe_attn_head > 0 ? a.pe_attn_head : H;
    g.q = q;
    g.k = k;
    g.v = v;
    g.q_scale = 0.125f * 1.4426950408889634f;  // softmax scale 1/sqrt(64) in log2 units, folded into q
    return g;
  };
  // In-launch phase chain (chain.hip): a layer's out-proj .. FFN2 plus the next layer's LayerNorm + QKV (or
  // the final LayerNorm) as one launch. The 16-bit DiT path without row masks (single-utterance calls); not
  // while a chained class is probed (its launches are timed one by one).
  // (the packed batch only, s0 == 0: two chain launches on the two CFG streams run 72 instead of 49 ms at C2, their
  // waiting workgroups holding the slots the other stream's producers need, profiles/r05_ab_c2_prio_split.txt; for
  // the same reason c.chain is off while another stream's chained call is in flight, chain_admit)
  const bool chain_on = c.chain && dit && r16 && do_ln && !keep && d == 1024 && b.chain && s0 == 0 && ns == c.S &&
                        (e->probe_class < 0 || e->probe_class == KC_ATTN || e->probe_class == KC_CONV ||
                         e->probe_class == KC_CHAIN);
  static const bool zero_memset = [] {  // F5H_CHAIN_ZERO=memset: the counters zeroed by a memset node (A/B)
    const char* v = getenv("F5H_CHAIN_ZERO");
    return v && !strcmp(v, "memset");
  }();
  if (chain_on) {
    if (zero_memset)
      KCK(hipMemsetAsync(b.chain, 0, (size_t)a.depth * 5 * b.chain_g4 * sizeof(unsigned), st));
    else
      KCK(zero_words(b.chain, (int64_t)a.depth * 5 * b.chain_g4, st));
  }
  bool qkv_done = false;    // this layer's LayerNorm + QKV came with the previous layer's chain
  bool final_done = false;  // the final LayerNorm came with the last layer's chain
  // LayerNorm fold (engine.lnfold): the attention-norm of layers 1.. and every FFN-norm run inside the GEMMs around
  // them; the first layer's attention-norm and the final norm stay launches. lnf(l): layer l's u/v block of the
  // current step's table row (kernels.h LnFoldArgs layout)
  const bool fold_on = c.lnfold && dit && r16 && do_ln && !keep && !chain_on && b.lnp && e->lnf_ok;
  // UNetT RMSNorm fold (engine.rmsf_ok): the FFN-norm of every layer and the attention-norm of layers 1 .. depth/2 - 1
  // (whose input FFN2 of the previous layer writes) run inside the GEMMs around them; the consumers read the residual
  // stream as A with W diag(g). Masked batches too (the producers keep masked rows as they are), but never with the
  // pad-row skip on a producer (a skipped tile would leave its rows' statistics unwritten)
  const bool rms_on = c.lnfold && !dit && r16 && b.lnp && e->rmsf_ok;
  const int64_t lnf_lw = 2 * (int64_t)a.ff_dim + 6 * (int64_t)d;
  auto lnf = [&](int l) { return ada_k + e->ada.Npad + (int64_t)l * lnf_lw; };
  auto fold_consumer = [&](GemmArgs& g, const float* u, const float* v) {
    g.ln_part_in = b.lnp + ro * (size_t)(d / 64) * 2;
    g.ln_nparts = d / 64;
    g.ln_u = u;
    g.ln_v = v;
    g.ln_eps = 1e-6f;  // LayerNorm eps (modules.py:316,336)
  };
  // RMSNorm form: x / max(|x|, 1e-12) sqrt(d) = x / sqrt(ss / d) (the epsilon only keeps an all-zero row finite)
  auto rms_consumer = [&](GemmArgs& g) {
    g.ln_part_in = b.lnp + ro * (size_t)(d / 64) * 2;
    g.ln_nparts = d / 64;
    g.ln_rms = 1;
    g.ln_eps = 1e-30f;
  };
  auto rms_producer = [&](GemmArgs& g) {
    g.ln_part = b.lnp + ro * (size_t)(d / 64) * 2;
    g.ln_nparts = d / 64;
    g.ln_rms = 1;
  };
  auto fold_producer = [&](GemmArgs& g, const float* scale) {
    g.hs = aop;
    g.hs_scale = scale;
    g.ln_part = b.lnp + ro * (size_t)(d / 64) * 2;
    g.ln_nparts = d / 64;
  };
  if (fold_on || rms_on) e->n_lnfold.fetch_add(1, std::memory_order_relaxed);
  for (int l = 0; l < a.depth; ++l) {
    Layer& Ly = e->layers[l];
    const float* ad = ada_k ? ada_k + (size_t)l * 6 * d : nullptr;
    if (!dit) {
      const int half = a.depth / 2;
      if (l < half) {
        // skips.append(x) (unett.py:283-284): layer l reads xs[l] and writes xs[l+1], so xs[l] stays
        // the skip connection without a copy
        h_in = res(b.xs[l]);
        h = res(b.xs[l + 1]);
        if (!(rms_on && l > 0)) KCK(rms_norm_g(bf, h_in, r16, rows, d, Ly.g_attn, aop, st));
      } else {
        // x = skip_proj(cat(x, skips.pop())) (unett.py:288-297): ONE GEMM over K = 2d whose A columns
        // [d, 2d) come from the skip buffer; then attention/FFN update the result in place
        void* x_prev = h;
        h = res(b.pp[(l - half) & 1]);
        h_in = nullptr;
        GemmArgs g = gargs(x_prev, d, Ly.skip, rows, h, d);
        g.A2 = res(b.xs[a.depth - 1 - l]);
        g.k_split = d;
        KCK(gemm(bf, r16 ? EPI_STORE16 : EPI_STORE, g, st));
        KCK(rms_norm_g(bf, h, r16, rows, d, Ly.g_attn, aop, st));
      }
    } else {
      if (do_ln && !qkv_done && !(fold_on && l > 0))
        KCK(ln_modulate(bf, h, r16, rows, d, ad /*shift_msa*/, ad + d /*scale_msa*/, aop, st));
    }
    if (!qkv_done) {
      GemmArgs g = qkv_args(Ly);
      if (fold_on && l > 0) fold_consumer(g, lnf(l) + 2 * a.ff_dim, lnf(l) + 2 * a.ff_dim + 3 * d);
      if (rms_on && l > 0 && l < a.depth / 2) {  // A = the layer input xs[l] itself, W diag(g_attn)
        g.A = h_in;
        g.W = Ly.qkv_g.w;
        rms_consumer(g);
      }
      ProbeScope ps(e, KC_QKV, st, &c.site, &g.probe);
      KCK(gemm(bf, EPI_QKV, g, st));
    }
    qkv_done = false;
    {
      AttnArgs at{};
      at.q = q;
      at.k = k;
      at.v = v;
      at.o = o;
      at.S = ns;
      at.H = H;
      at.L = c.L;
      at.kv_len = (a.attn_mask_enabled && c.batch_mask) ? b.kvlen + s0 : nullptr;
      // pad query rows' outputs are zeroed after to_out (modules.py:551-553): their blocks are skipped
      at.q_len = (c.batch_mask && e->pad_skip) ? b.kvlen + s0 : nullptr;
      at.scale = 0.125f;
      at.prescaled = 1;
      ProbeScope ps(e, KC_ATTN, st, &c.site, &at.probe);
      KCK(attention(bf, at, st));
    }
    if (chain_on) {
      ChainArgs ca{};
      ca.out = gargs(o, inner, Ly.out, rows, h, d);
      ca.out.gate = ad + 2 * d;  // gate_msa
      ca.ln1 = LnArgs{h, aop, ad + 3 * d /*shift_mlp*/, ad + 4 * d /*scale_mlp*/};
      ca.ff1 = gargs(aop, d, Ly.ff1, rows, f, a.ff_dim);
      ca.ff2 = gargs(f, a.ff_dim, Ly.ff2, rows, h, d);
      ca.ff2.gate = ad + 5 * d;  // gate_mlp
      if (l + 1 < a.depth) {
        const float* an = ada_k + (size_t)(l + 1) * 6 * d;
        ca.ln2 = LnArgs{h, aop, an /*shift_msa*/, an + d /*scale_msa*/};
        ca.qkv = qkv_args(e->layers[l + 1]);
      } else {
        const float* fin = ada_k + (size_t)a.depth * 6 * d;  // AdaLayerNorm_Final: (scale, shift)
        ca.ln2 = LnArgs{h, aop, fin + d, fin};
      }
      ca.cnt = b.chain + (size_t)l * 5 * b.chain_g4;
      ca.groups = (rows + kChainRows - 1) / kChainRows;
      ca.fault = e->chain_fault;
      ProbeScope ps(e, KC_CHAIN, st, &c.site, &ca.probe);
      const hipError_t ce = chain_launch(bf, ca, st);
      if (ce == hipSuccess) {
        e->n_chain.fetch_add(1, std::memory_order_relaxed);
        qkv_done = l + 1 < a.depth;
        final_done = l + 1 == a.depth;
        continue;
      }
      if (ce != hipErrorInvalidValue) KCK(ce);  // shapes outside the chain: the separate launches below
    }
    {
      GemmArgs g = gargs(o, inner, Ly.out, rows, h, d);
      g.resid = h_in;                      // UNetT first half: x_in + attn(.) -> the next buffer
      g.gate = ad ? ad + 2 * d : nullptr;  // gate_msa
      g.rowkeep = keep;                    // masked_fill of pad rows (modules.py:552-554)
      // row tiles of padding only: no work at all. Only in place (h_in null): a UNetT first-half layer
      // writes x_in + attn into the next buffer, so its pad rows must still be copied there
      if (keep && !h_in && e->pad_skip && !rms_on) {
        g.live_len = b.kvlen + s0;
        g.live_seq = c.L;
      }
      if (fold_on) fold_producer(g, ad + 4 * d /*scale_mlp: hs = h (1 + scale_mlp) for FFN1*/);
      if (rms_on) rms_producer(g);  // the FFN-norm's statistics of h
      ProbeScope ps(e, KC_OUT, st, &c.site, &g.probe);
      KCK(gemm(bf, epi_resid, g, st));
    }
    if (!fold_on && !rms_on) {
      ProbeScope ps(e, KC_NORM, st, &c.site);
      if (dit) {
        if (do_ln) KCK(ln_modulate(bf, h, r16, rows, d, ad + 3 * d /*shift_mlp*/, ad + 4 * d /*scale_mlp*/, aop, st));
      }
      else
        KCK(rms_norm_g(bf, h, r16, rows, d, Ly.g_ff, aop, st));
    }
    {
      GemmArgs g = gargs(aop, d, Ly.ff1, rows, f, a.ff_dim);
      if (fold_on) fold_consumer(g, lnf(l), lnf(l) + a.ff_dim);
      if (rms_on) {  // A = h itself, W diag(g_ff)
        g.A = h;
        g.W = Ly.ff1_g.w;
        rms_consumer(g);
      }
      ProbeScope ps(e, KC_FFN1, st, &c.site, &g.probe);
      KCK(gemm(bf, EPI_GELU_TANH, g, st));
    }
    {
      GemmArgs g = gargs(f, a.ff_dim, Ly.ff2, rows, h, d);
      g.gate = ad ? ad + 5 * d : nullptr;  // gate_mlp
      // the next layer's attention-norm: hs = h (1 + scale_msa of layer l + 1) for its QKV
      if (fold_on && l + 1 < a.depth) fold_producer(g, ada_k + (size_t)(l + 1) * 6 * d + d);
      if (rms_on && l + 1 < a.depth / 2) rms_producer(g);  // the next layer's attention-norm (its input is this h)
      ProbeScope ps(e, KC_FFN2, st, &c.site, &g.probe);
      KCK(gemm(bf, epi_resid, g, st));
    }
  }
  if (dit) {
    const float* fin = ada_k + (size_t)a.depth * 6 * d;  // AdaLayerNorm_Final: (scale, shift)
    if (!final_done) KCK(ln_modulate(bf, h, r16, rows, d, fin + d, fin, aop, st));
  } else {
    KCK(rms_norm_g(bf, h, r16, rows, d, e->norm_out_g, aop, st));
  }
  // all Npad (128) columns: the padded weight rows and bias are zero, and whole-column tiles take the
  // fast epilogue; readers use the first mel_dim columns of each 128-float row
  const int pld = e->proj_out.Npad;
  GemmArgs g = gargs(aop, d, e->proj_out, rows, b.p + ro * pld, pld);
  g.N = pld;
  KCK(gemm(bf, EPI_STORE, g, st));
  return 0;
}

// One packed cond/uncond backbone forward for the current step; result in b.p [S, L, mel]. With a
// second stream (c.st2, graph capture only) the conditional and unconditional branches run as two
// independent launch chains (fork/join by events), so one chain's kernel heads and tails overlap
// the other's bodies instead of leaving CUs idle at every kernel boundary.
static int backbone_step(Ctx& c) {
  if (!c.st2 || !c.use_cfg) return backbone_part(c, 0, c.S, c.st);
  f5h_engine* e = c.e;
  KCK(hipEventRecord(e->ev_fork, c.st));
  KCK(hipStreamWaitEvent(c.st2, e->ev_fork, 0));
  RC(backbone_part(c, 0, c.B, c.st));
  RC(backbone_part(c, c.B, c.B, c.st2));
  KCK(hipEventRecord(e->ev_join, c.st2));
  KCK(hipStreamWaitEvent(c.st, e->ev_join, 0));
  return 0;
}

// ---------------------------------------------------------------- phase-chain admission and fault word
// Pinned host words the engines' fault copies land in: one slab per process (allocated once; a hipHostFree per engine
// could wait for the device), slots handed out and returned by index.
static std::mutex g_slot_m;
static unsigned* g_slots = nullptr;
static std::vector<int> g_free_slots;
static constexpr int kFaultSlots = 4096;
static int fault_slot_take(volatile unsigned** host) {
  std::lock_guard<std::mutex> lk(g_slot_m);
  if (!g_slots) {
    void* p = nullptr;
    if (hipHostMalloc(&p, kFaultSlots * 64, hipHostMallocDefault) != hipSuccess) return -1;
    g_slots = static_cast<unsigned*>(p);
    for (int i = kFaultSlots - 1; i >= 0; --i) g_free_slots.push_back(i);
  }
  if (g_free_slots.empty()) return -1;
  const int i = g_free_slots.back();
  g_free_slots.pop_back();
  *host = g_slots + (size_t)i * 16;  // one 64-B line per slot
  **host = 0u;
  return i;
}
static void fault_slot_give(int i) {
  if (i < 0) return;
  std::lock_guard<std::mutex> lk(g_slot_m);
  g_free_slots.push_back(i);
}

// Per-device admission of chained calls. Two phase-chain launches in flight at once starve each
// other: each one's waiting workgroups hold CU slots the other's producers need (C2 72 instead of 49 ms with the two
// CFG branches on their own streams, profiles/r05_ab_c2_prio_split.txt). A call that would chain while a chained
// call from ANOTHER stream is still being enqueued or still runs on the device (its "done" event not complete) takes
// the separate launches instead (bitwise identical results). Calls on one stream are ordered by the stream itself.
// Non-blocking: one hipEventQuery, no wait.
struct ChainGate {
  std::mutex m;
  hipStream_t owner = nullptr;
  bool owned = false;
  int enqueuing = 0;          // chained calls of the owner stream being enqueued
  hipEvent_t done = nullptr;  // recorded on the owner stream after its last chained call
  bool pending = false;
};
static ChainGate g_gate[64];
static std::atomic<int64_t> g_gate_refused{0};

static bool chain_admit(int dev, hipStream_t st) {
  ChainGate& g = g_gate[dev & 63];
  std::lock_guard<std::mutex> lk(g.m);
  if (g.owned && g.owner != st) {
    bool busy = g.enqueuing > 0;
    if (!busy && g.pending) {
      busy = hipEventQuery(g.done) == hipErrorNotReady;
      (void)hipGetLastError();  // hipErrorNotReady is the expected answer for a pending event
      if (!busy) g.pending = false;
    }
    if (busy) {
      g_gate_refused.fetch_add(1, std::memory_order_relaxed);
      return false;
    }
  }
  g.owner = st;
  g.owned = true;
  ++g.enqueuing;
  return true;
}
static void chain_leave(int dev, hipStream_t st) {
  ChainGate& g = g_gate[dev & 63];
  std::lock_guard<std::mutex> lk(g.m);
  --g.enqueuing;
  if (!g.done && hipEventCreateWithFlags(&g.done, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    g.done = nullptr;
    return;
  }
  if (hipEventRecord(g.done, st) == hipSuccess)
    g.pending = true;
  else
    (void)hipGetLastError();
}
// Held for one call: admits the call's chain (or not) and, on every return path, records the gate's "done" event
// after the call's launches.
struct ChainTicket {
  int dev = 0;
  hipStream_t st = nullptr;
  bool held = false;
  ~ChainTicket() {
    if (held) chain_leave(dev, st);
  }
};
// Could this call's step run the chain? (the engine switch and the shapes backbone_part checks per part); if so,
// ask the gate.
static int chain_for_call(f5h_engine* e, const Ctx& c, ChainTicket& t) {
  static const bool res32 = [] {
    const char* v = getenv("F5H_RES32");
    return v && *v == '1';
  }();
  const bool split = e->graph_mode && e->split_cfg == 1 && c.use_cfg;  // the two CFG parts: no chain
  if (!e->chain || e->a.backbone != F5H_DIT || e->bf == 0 || res32 || e->a.dim != 1024 || c.batch_mask || split ||
      !e->chain_fault)
    return 0;
  if (!chain_admit(e->dev, c.st)) return 0;
  t.dev = e->dev;
  t.st = c.st;
  t.held = true;
  return 1;
}
// Start of every sample/forward call: a give-up recorded by an earlier chained call of this engine (its copy in the
// pinned word, landed once that call completed) fails this call and switches the chain off for the engine.
static int chain_fault_check(f5h_engine* e, hipStream_t st) {
  if (!e->fault_host || *e->fault_host == 0u) return 0;
  *e->fault_host = 0u;
  {
    std::lock_guard<std::mutex> g(e->gm);
    e->chain = 0;
  }
  (void)hipMemsetAsync(e->chain_fault, 0, sizeof(unsigned), st);
  return fail(F5H_EHIP,
              "phase chain: a wait for a producer row group gave up in an earlier call of this engine (its output was "
              "set to NaN); the chain is now off for this engine (f5h_set_chain re-enables it)");
}
// End of a chained call: the fault word's copy to the pinned host word, stream-ordered behind the call
static int chain_fault_note(f5h_engine* e, hipStream_t st) {
  if (!e->fault_host) return 0;
  HIPCK(hipMemcpyAsync(const_cast<unsigned*>(e->fault_host), e->chain_fault, sizeof(unsigned), hipMemcpyDeviceToHost,
                       st));
  return 0;
}

static int check_arch(const f5h_arch* a) {
  if (!a) return fail(F5H_EINVAL, "null arch");
  if (a->backbone != F5H_DIT && a->backbone != F5H_UNETT) return fail(F5H_EINVAL, "backbone must be DiT or UNetT");
  if (a->dim_head != 64) return fail(F5H_EINVAL, "dim_head must be 64");
  if (a->dim % 128 || a->dim <= 0 || a->dim > 1024) return fail(F5H_EINVAL, "dim must be a multiple of 128, <= 1024");
  if (a->heads * 64 != a->dim) return fail(F5H_EINVAL, "heads*dim_head must equal dim");
  if (a->ff_dim % 64 || a->ff_dim <= 0) return fail(F5H_EINVAL, "ff_dim must be a positive multiple of 64");
  if (a->mel_dim != 100) return fail(F5H_EINVAL, "mel_dim must be 100");
  if (a->text_dim <= 0 || a->text_dim % 4 || a->text_dim > 512) return fail(F5H_EINVAL, "text_dim must be <= 512, % 4");
  if (a->depth <= 0 || (a->backbone == F5H_UNETT && a->depth % 2)) return fail(F5H_EINVAL, "bad depth");
  if (a->backbone == F5H_UNETT && a->conv_layers != 0) return fail(F5H_EINVAL, "UNetT with conv_layers unsupported");
  if (a->compute != F5H_FP32 && a->compute != F5H_BF16 && a->compute != F5H_FP16)
    return fail(F5H_EINVAL, "compute must be FP32, BF16 or FP16");
  return 0;
}

// ============================================================================ C ABI
extern "C" {

const char* f5h_last_error(void) { return g_err.c_str(); }
const char* f5h_version(void) { return "f5h 0.1 gfx950"; }

int f5h_engine_create_views(const f5h_arch* arch, const f5h_tensor_view* weights, int32_t n_weights, int32_t device,
                            f5h_engine** out) {
  if (!out) return fail(F5H_EINVAL, "null out");
  *out = nullptr;
  RC(check_arch(arch));
  if (n_weights < 0 || (n_weights > 0 && !weights)) return fail(F5H_EINVAL, "null weights");
  for (int i = 0; i < n_weights; ++i) {
    const f5h_tensor_view& v = weights[i];
    if (!v.name || (!v.data && v.numel > 0) || v.numel < 0) return fail(F5H_EINVAL, "bad weight view");
    if (v.dtype != F5H_DT_F32 && v.dtype != F5H_DT_BF16 && v.dtype != F5H_DT_F16)
      return fail(F5H_EINVAL, std::string("weight ") + v.name + ": dtype must be F5H_DT_F32, _BF16 or _F16");
    if (v.on_device != 0 && v.on_device != 1)
      return fail(F5H_EINVAL, std::string("weight ") + v.name + ": on_device must be 0 or 1");
  }
  HIPCK(hipSetDevice(device));
  f5h_engine* e = new f5h_engine();
  if (hipStreamCreateWithFlags(&e->mstream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return fail(F5H_EHIP, "engine stream");
  }
  e->a = *arch;
  e->dev = device;
  e->bf = arch->compute;
  e->esz = e->bf ? 2 : 4;
  e->tdp = (arch->text_dim + 63) / 64 * 64;
  if (const char* gv = getenv("F5H_GRAPH")) e->graph_mode = atoi(gv) ? 1 : 0;
  if (const char* sv = getenv("F5H_SPLIT_CFG")) e->split_cfg = std::min(2, std::max(0, atoi(sv)));
  if (const char* pv = getenv("F5H_NO_PAD_SKIP")) e->pad_skip = (*pv == '1') ? 0 : 1;
  if (const char* cv = getenv("F5H_CHAIN")) e->chain = (*cv == '1') ? 1 : 0;
  // device views are read on the engine's non-blocking stream: order it behind the null stream (so behind
  // every blocking stream's queued work, the ordering the packing had when it ran on the null stream); work
  // on other non-blocking streams must be complete (f5h.h)
  {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
      if (hipEventRecord(ev, nullptr) != hipSuccess || hipStreamWaitEvent(e->mstream, ev, 0) != hipSuccess)
        (void)hipGetLastError();
      (void)hipEventDestroy(ev);
    } else {
      (void)hipGetLastError();
    }
  }
  // host views: staged once, in their own dtype, into temporaries freed after packing
  WMap W;
  std::vector<void*> staged;
  int rc = 0;
  for (int i = 0; i < n_weights && !rc; ++i) {
    const f5h_tensor_view& v = weights[i];
    const size_t bytes = (size_t)v.numel * (v.dtype == F5H_DT_F32 ? 4 : 2);
    const void* dp = v.data;
    if (!v.on_device && bytes) {
      void* t = dev_alloc(device, bytes, e->mstream);
      if (!t) {
        rc = fail(F5H_EHIP, "weight staging allocation");
        break;
      }
      staged.push_back(t);
      if (hipMemcpyAsync(t, v.data, bytes, hipMemcpyHostToDevice, e->mstream) != hipSuccess) {
        rc = fail(F5H_EHIP, std::string("weight staging copy: ") + v.name);
        break;
      }
      dp = t;
    } else if (v.on_device && bytes) {
      hipPointerAttribute_t at{};
      if (hipPointerGetAttributes(&at, v.data) != hipSuccess || at.device != device) {
        (void)hipGetLastError();
        rc = fail(F5H_EINVAL, std::string("weight ") + v.name + ": on_device view is not memory of device " +
                                  std::to_string(device));
        break;
      }
    }
    W.m[v.name] = WView{dp, v.dtype, v.numel};
  }
  if (!rc) rc = pack_all(e, W);
  // LayerNorm fold support and the AdaLN table row length (DiT: the modulation rows, then the fold's u/v per layer)
  if (!rc && arch->backbone == F5H_DIT) {
    e->lnf_ok = e->bf != 0 && arch->dim % 64 == 0 && arch->dim <= 1024 && arch->ff_dim % 64 == 0;
    e->ada_row = e->ada.Npad + (e->lnf_ok ? (int64_t)arch->depth * (2 * (int64_t)arch->ff_dim + 6 * (int64_t)arch->dim) : 0);
    if (e->lnf_ok) {
      std::vector<const void*> wp;
      for (const Layer& L : e->layers) wp.push_back(L.ff1.w);
      for (const Layer& L : e->layers) wp.push_back(L.qkv.w);
      if (upload(e, wp, &e->lnf_w)) e->lnf_ok = false;
    }
  }
  // RMSNorm fold support (UNetT, 16-bit): every layer's QKV and FFN1 weights with their norm's gain folded in
  if (!rc && arch->backbone == F5H_UNETT && e->bf != 0 && arch->dim % 64 == 0 && arch->dim <= 1024) {
    e->rmsf_ok = true;
    for (Layer& L : e->layers) {
      L.qkv_g = L.qkv;
      L.ff1_g = L.ff1;
      if (dalloc(e, (size_t)L.qkv.Npad * L.qkv.K * e->esz, &L.qkv_g.w) ||
          dalloc(e, (size_t)L.ff1.Npad * L.ff1.K * e->esz, &L.ff1_g.w) ||
          scale_cols(e->bf, L.qkv.w, L.qkv.Npad, L.qkv.K, L.g_attn, L.qkv_g.w, e->mstream) != hipSuccess ||
          scale_cols(e->bf, L.ff1.w, L.ff1.Npad, L.ff1.K, L.g_ff, L.ff1_g.w, e->mstream) != hipSuccess) {
        e->rmsf_ok = false;
        break;
      }
    }
  }
  // default: on for DiT (C2 -2 %, profiles/r06_ab_fold_c2.txt), off for UNetT (its RMSNorm fold measured within noise
  // at C5, profiles/r06_ab_rmsfold_c5.txt); F5H_LNFOLD=0/1 or f5h_set_ln_fold overrides
  e->lnfold = arch->backbone == F5H_DIT ? 1 : 0;
  if (const char* lv = getenv("F5H_LNFOLD")) e->lnfold = (*lv == '0') ? 0 : 1;
  // packing ran on the engine's stream (no device-wide synchronisation)
  if (!rc && hipStreamSynchronize(e->mstream) != hipSuccess) rc = fail(F5H_EHIP, "weight packing");
  for (void* t : staged) dev_free(t, e->mstream);
  if (rc) {
    f5h_engine_destroy(e);
    return rc;
  }
  {
    void* p = nullptr;
    int khz = 0;
    void* tl = nullptr;
    if (dalloc(e, kProbeBytes, &p) || dalloc(e, (size_t)kTimelineWG * 4 * sizeof(unsigned long long), &tl) ||
        hipStreamSynchronize(e->mstream) != hipSuccess) {
      f5h_engine_destroy(e);
      return fail(F5H_EHIP, "probe buffers");
    }
    void* fw = nullptr;
    if (dalloc(e, 64, &fw) || hipStreamSynchronize(e->mstream) != hipSuccess) {
      f5h_engine_destroy(e);
      return fail(F5H_EHIP, "chain fault word");
    }
    e->chain_fault = reinterpret_cast<unsigned*>(fw);
    e->fault_slot = fault_slot_take(&e->fault_host);
    if (e->fault_slot < 0) {  // no pinned word: the chain stays off (its give-ups could not be reported)
      (void)hipGetLastError();
      e->chain_fault = nullptr;
    }
    e->pstamp = reinterpret_cast<unsigned long long*>(p);
    e->pslots = e->pstamp + 64;
    e->ptick = reinterpret_cast<int*>(e->pstamp);
    e->ptl = reinterpret_cast<unsigned long long*>(tl);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess) e->wall_khz = khz;
  }
  *out = e;
  return 0;
}

int f5h_engine_create(const f5h_arch* arch, const f5h_weight* weights, int32_t n_weights, int32_t device,
                      f5h_engine** out) {
  if (n_weights < 0 || (n_weights > 0 && !weights)) return fail(F5H_EINVAL, "null weights");
  std::vector<f5h_tensor_view> v((size_t)n_weights);
  for (int i = 0; i < n_weights; ++i)
    v[i] = f5h_tensor_view{weights[i].name, weights[i].data, F5H_DT_F32, 0, weights[i].numel};
  return f5h_engine_create_views(arch, v.data(), n_weights, device, out);
}

// Returns at once: the release runs on the reaper thread (reaper.h), which waits only for this engine's
// own work -- the last-use event of every stream its calls ran on and the events recorded after its graph
// replays -- and then destroys the graphs and frees the device memory. No device-wide synchronisation, so
// dropping an engine never waits for unrelated streams (the reference's ThreadPoolExecutor may be
// sampling with other models meanwhile).
void f5h_engine_destroy(f5h_engine* e) {
  if (!e) return;
  retire(e->dev, [e] {
    for (hipEvent_t ev : e->uses.take()) {
      (void)hipEventSynchronize(ev);
      (void)hipEventDestroy(ev);
    }
    {
      std::lock_guard<std::mutex> g(e->gm);
      for (auto* v : {&e->graphs, &e->graveyard})
        for (auto& x : *v)
          for (hipEvent_t ev : x->inflight) (void)hipEventSynchronize(ev);
    }
    e->graphs.clear();
    e->graveyard.clear();
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    e->ev_pool.clear();
    if (e->cap) (void)hipStreamDestroy(e->cap);
    if (e->cap2) (void)hipStreamDestroy(e->cap2);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    // stream-ordered releases into the pool: no device-wide wait (hipFree would wait for every stream)
    for (void* p : e->allocs) dev_free(p, e->mstream);
    if (e->mstream) (void)hipStreamDestroy(e->mstream);
    fault_slot_give(e->fault_slot);  // after the use events: the last fault copy has landed
    delete e;
  });
}

size_t f5h_workspace_size(const f5h_engine* e, int32_t B, int32_t N, int32_t nt, int32_t nfe, int32_t use_cfg) {
  (void)nt;
  if (!e || B <= 0 || N <= 0 || nfe <= 0) return 0;
  WS ws;
  Bufs b;
  layout(e, ws, b, B, N, nfe + 1, use_cfg);
  return ws.off;
}

static int check_ws(f5h_engine* e, int B, int N, int nfe, int use_cfg, void* w, size_t bytes, Ctx& c) {
  WS ws;
  layout(e, ws, c.b, B, N, nfe + 1, use_cfg);
  if (bytes < ws.off)
    return fail(F5H_ENOMEM, "workspace too small: need " + std::to_string(ws.off) + " have " + std::to_string(bytes));
  ws.off = 0;
  ws.base = reinterpret_cast<char*>(w);
  layout(e, ws, c.b, B, N, nfe + 1, use_cfg);
  return 0;
}

static int run_steps(Ctx& c, const f5h_sample_args* a, const void* ws);
static int graph_get(Ctx& c, const GraphKey& key, bool split, const std::function<int(Ctx&)>& body,
                     std::shared_ptr<GraphEntry>& hold, int64_t replays);
static int note_replays(f5h_engine* e, GraphEntry* g, hipStream_t st);
static bool prologue_repeats(f5h_engine* e, const GraphKey& key);

// The prologue as one captured graph per (workspace, shape): its ~56 launches otherwise cost more
// host time than device time (profiles/r02_call_gaps_c2.txt). The inputs it reads are staged into
// fixed workspace slots first, the grid is read from the device copy. F5H_PROLOGUE_GRAPH=0: eager.
static GraphKey prologue_key(const Ctx& c, const void* ws) {
  GraphKey key{};
  key.ws = ws;
  key.kind = 1;
  key.B = c.B;
  key.N = c.N;
  key.nt = c.nt;
  key.nfe = c.nfe;
  key.use_cfg = c.use_cfg;
  key.batch_mask = c.batch_mask;
  key.lnfold = c.lnfold;
  key.kernel_epoch = g_kernel_epoch.load();
  return key;
}
static int prologue_graph(Ctx& c, const f5h_sample_args* a, const GraphKey& key) {
  f5h_engine* e = c.e;
  const size_t bn = (size_t)c.B * c.N;
  HIPCK(hipMemcpyAsync(c.b.in_cond, a->cond, bn * e->a.mel_dim * sizeof(float), hipMemcpyDeviceToDevice, c.st));
  HIPCK(hipMemcpyAsync(c.b.in_mask, a->cond_mask, bn, hipMemcpyDeviceToDevice, c.st));
  if (c.nt > 0)
    HIPCK(hipMemcpyAsync(c.b.in_text, a->text, (size_t)c.B * c.nt * sizeof(int64_t), hipMemcpyDeviceToDevice, c.st));
  HIPCK(hipMemcpyAsync(c.b.in_dur, a->duration, (size_t)c.B * sizeof(int32_t), hipMemcpyDeviceToDevice, c.st));
  const Bufs& b = c.b;
  std::shared_ptr<GraphEntry> hold;
  RC(graph_get(c, key, false,
               [&](Ctx& cc) { return prologue(cc, nullptr, cc.nfe, b.in_cond, b.in_mask, b.in_text, b.in_dur); },
               hold, 1));
  HIPCK(hipGraphLaunch(hold->exec, c.st));
  return note_replays(e, hold.get(), c.st);
}

int f5h_sample(f5h_engine* e, void* stream, const f5h_sample_args* a, void* workspace, size_t workspace_bytes) {
  if (!e || !a) return fail(F5H_EINVAL, "null engine/args");
  if (a->B <= 0 || a->N <= 0 || a->nt < 0 || a->nfe <= 0 || a->nfe > 512)
    return fail(F5H_EINVAL, "bad B/N/nt/nfe");
  if (!a->cond || !a->cond_mask || !a->duration || !a->y0 || !a->t_grid || !a->out || (a->nt > 0 && !a->text))
    return fail(F5H_EINVAL, "null tensor argument");
  if (e->a.backbone == F5H_DIT && a->N > 8192) return fail(F5H_EINVAL, "N exceeds the text position table (8192)");
  HIPCK(hipSetDevice(e->dev));
  UseNote used{e->uses, reinterpret_cast<hipStream_t>(stream)};  // on every return: the engine's release waits for it
  Ctx c{};
  c.e = e;
  c.st = reinterpret_cast<hipStream_t>(stream);
  c.B = a->B;
  c.N = a->N;
  c.nt = a->nt;
  c.nfe = a->nfe;
  c.use_cfg = a->cfg_strength >= 1e-5f;
  c.S = c.use_cfg ? 2 * c.B : c.B;
  c.L = e->a.backbone == F5H_DIT ? c.N : c.N + 1;
  c.batch_mask = a->use_batch_mask ? 1 : 0;
  RC(check_ws(e, c.B, c.N, c.nfe, c.use_cfg, workspace, workspace_bytes, c));
  RC(chain_fault_check(e, c.st));
  ChainTicket ticket;  // (declared after `used`: its event is recorded first, both after every launch of the call)
  c.chain = chain_for_call(e, c, ticket);
  c.lnfold = e->lnfold && !c.chain && ((e->lnf_ok && !c.batch_mask) || e->rmsf_ok);
  double hp[kHostPhases] = {};
  c.hp = hp;
  const double h0 = host_ms();
  static const bool pro_graph = [] {
    const char* v = getenv("F5H_PROLOGUE_GRAPH");
    return !(v && *v == '0');
  }();
  HIPCK(grid_upload(a->t_grid, c.nfe + 1, c.b.tgrid, c.st));
  // the ODE evaluates fn at t_0 .. t_{nfe-1}
  const GraphKey pkey = prologue_key(c, workspace);
  if (pro_graph && e->graph_mode && c.nt <= c.N && prologue_repeats(e, pkey))
    RC(prologue_graph(c, a, pkey));
  else
    RC(prologue(c, a->t_grid, c.nfe, a->cond, a->cond_mask, a->text, a->duration));
  const double h1 = host_ms();
  const size_t ysz = (size_t)c.B * c.N * e->a.mel_dim;
  HIPCK(hipMemcpyAsync(c.b.y, a->y0, ysz * sizeof(float), hipMemcpyDeviceToDevice, c.st));
  if (a->trajectory)
    HIPCK(hipMemcpyAsync(a->trajectory, a->y0, ysz * sizeof(float), hipMemcpyDeviceToDevice, c.st));
  HIPCK(pack_y(e->bf, c.b.y, c.B * c.N, e->a.mel_dim, c.b.ypad, c.st));
  HIPCK(ptr_upload(a->trajectory, c.b.trajp, c.st));
  // step index and the Euler launch's arrival counter (kstep[kArrive]) start at 0; step 0's table row
  // is copied here, every later one by the previous step's Euler launch
  HIPCK(hipMemsetAsync(c.b.kstep, 0, 64 * sizeof(int), c.st));
  RC(step_prep(c));
  const double h2 = host_ms();
  const double g2 = hp[HP_LOCK] + hp[HP_REAP] + hp[HP_CAPTURE] + hp[HP_INSTANTIATE];
  RC(run_steps(c, a, workspace));
  const double h3 = host_ms();
  HIPCK(final_where_out(a->cond, a->cond_mask, c.b.y, a->out, c.B, c.N, e->a.mel_dim,
                        c.chain ? e->chain_fault : nullptr, c.st));
  if (c.chain) RC(chain_fault_note(e, c.st));
  const double h4 = host_ms();
  hp[HP_TOTAL] = h4 - h0;
  hp[HP_PROLOGUE] = h1 - h0;
  hp[HP_LAUNCH] = (h3 - h2) - (hp[HP_LOCK] + hp[HP_REAP] + hp[HP_CAPTURE] + hp[HP_INSTANTIATE] - g2);
  hp[HP_FINAL] = h4 - h3;
  {
    std::lock_guard<std::mutex> g(e->hm);
    std::memcpy(e->last_host, hp, sizeof(hp));
  }
  return 0;
}

// One NFE step, eager or as the graph's capture source: backbone -> CFG + Euler (dt and trajectory
// slot from the device step index), which also copies the next step's table row into the fixed
// per-step buffer and bumps the step index (folded: no step_begin / step_advance launches).
static int enqueue_step(Ctx& c, const f5h_sample_args* a) {
  f5h_engine* e = c.e;
  {
    c.site = 0;
    RC(backbone_step(c));
    EulerArgs u{};
    u.y = c.b.y;
    u.B = c.B;
    u.N = c.N;
    u.mel = e->a.mel_dim;
    u.p = c.b.p;
    u.p_seq_stride = (int64_t)c.L * e->proj_out.Npad;
    u.p_row_off = e->a.backbone == F5H_DIT ? 0 : 1;
    u.p_ld = e->proj_out.Npad;
    u.use_cfg = c.use_cfg;
    u.cfg = a->cfg_strength;
    u.dt = 0.f;
    u.kstep = c.b.kstep;
    u.tgrid = c.b.tgrid;
    u.ypad = c.b.ypad;
    u.compute = e->bf;
    u.traj = nullptr;
    u.trajp = c.b.trajp;
    const bool dit = e->a.backbone == F5H_DIT;
    u.next_src = dit ? c.b.ada : c.b.temb;
    u.next_stride = dit ? e->ada_row : e->a.dim;
    u.next_n = dit ? (int)e->ada_row : e->a.dim;
    u.next_dst = dit ? c.b.ada_cur : c.b.temb_cur;
    u.nfe = c.nfe;
    u.arrive = reinterpret_cast<unsigned*>(c.b.kstep + kArrive);
    u.tick = e->ptick;
    KCK(cfg_euler(u, c.st));
  }
  return 0;
}

// The NFE loop: eager launches, or one captured step graph replayed nfe times.
static int run_steps(Ctx& c, const f5h_sample_args* a, const void* ws) {
  f5h_engine* e = c.e;
  if (!e->graph_mode) {
    for (int k = 0; k < c.nfe; ++k) RC(enqueue_step(c, a));
    return 0;
  }
  GraphKey key{};
  key.ws = ws;
  key.B = c.B;
  key.N = c.N;
  key.nfe = c.nfe;
  key.use_cfg = c.use_cfg;
  key.batch_mask = c.batch_mask;
  key.probe = e->probe_class;
  const bool split = e->split_cfg == 1;  // auto (2): one packed chain
  key.split = split;
  key.pad_skip = e->pad_skip;
  key.chain = c.chain;
  key.lnfold = c.lnfold;
  key.kernel_epoch = g_kernel_epoch.load();
  std::memcpy(&key.cfg_bits, &a->cfg_strength, 4);
  std::shared_ptr<GraphEntry> hold;  // keeps the replayed graph alive through the launch loop
  RC(graph_get(c, key, split, [&](Ctx& cc) { return enqueue_step(cc, a); }, hold, c.nfe));
  // the replays-done event is recorded whenever any replay was enqueued, also when a later launch fails:
  // an evicted entry is destroyed only after it (reap_graphs)
  int rc = 0, k = 0;
  for (; k < c.nfe; ++k) {
    const hipError_t le = hipGraphLaunch(hold->exec, c.st);
    if (le != hipSuccess) {
      rc = fail(F5H_EHIP, std::string("hipGraphLaunch: ") + hipGetErrorString(le));
      break;
    }
  }
  if (k > 0) {
    const int r2 = note_replays(e, hold.get(), c.st);
    if (!rc) rc = r2;
  }
  return rc;
}

// F5H_HOST_TRACE=1: host time of the graph-cache phases on stderr (diagnostic)
static bool host_trace() {
  static const bool on = [] {
    const char* v = getenv("F5H_HOST_TRACE");
    return v && *v == '1';
  }();
  return on;
}
// Destroy graveyard entries that nothing replays any more: every event recorded after their
// replays has completed and no caller holds them. Non-blocking (hipEventQuery); caller holds e->gm.
static void reap_graphs(f5h_engine* e) {
  auto done = [e](GraphEntry& g) {
    size_t k = 0;
    for (hipEvent_t ev : g.inflight) {
      if (hipEventQuery(ev) == hipSuccess)
        e->ev_pool.push_back(ev);
      else
        g.inflight[k++] = ev;
    }
    (void)hipGetLastError();  // hipErrorNotReady is the expected answer for a pending event
    g.inflight.resize(k);
    return k == 0;
  };
  for (auto& g : e->graphs)
    if (g->inflight.size() > 4) done(*g);  // keep live entries' lists short
  size_t k = 0;
  for (size_t i = 0; i < e->graveyard.size(); ++i) {
    auto& g = e->graveyard[i];
    if (done(*g) && g.use_count() == 1) {
      ++e->n_reaped;
      continue;  // last reference: destroyed when the slot is overwritten or the vector shrinks
    }
    if (k != i) std::swap(e->graveyard[k], e->graveyard[i]);
    ++k;
  }
  e->graveyard.resize(k);
}

// Record, on `st`, an event after the launches just enqueued from `g` (the entry stays in the
// graveyard until it completes).
static int note_replays(f5h_engine* e, GraphEntry* g, hipStream_t st) {
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(e->gm);
    if (!e->ev_pool.empty()) {
      ev = e->ev_pool.back();
      e->ev_pool.pop_back();
    }
  }
  if (!ev) HIPCK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCK(hipEventRecord(ev, st));
  std::lock_guard<std::mutex> lk(e->gm);
  g->inflight.push_back(ev);
  return 0;
}

// The cached graph for `key`, captured from `body` on the private capture stream(s) when absent.
// An evicted entry moves to the graveyard (no device synchronisation, no wait under the mutex).
static int graph_get(Ctx& c, const GraphKey& key, bool split, const std::function<int(Ctx&)>& body,
                     std::shared_ptr<GraphEntry>& hold, int64_t replays) {
  f5h_engine* e = c.e;
  const double t0 = host_ms();
  std::lock_guard<std::mutex> g(e->gm);
  const double t1 = host_ms();
  const int64_t reaped0 = e->n_reaped;
  reap_graphs(e);
  const double t2 = host_ms();
  if (c.hp) {
    c.hp[HP_LOCK] += t1 - t0;
    c.hp[HP_REAP] += t2 - t1;
  }
  if (host_trace())
    std::fprintf(stderr, "[f5h host] graph_get kind %d: lock %.3f ms, reap %.3f ms (%lld destroyed)\n", key.kind,
                 t1 - t0, t2 - t1, (long long)(e->n_reaped - reaped0));
  for (const auto& x : e->graphs)
    if (x->key == key) hold = x;
  if (!hold) {
    if (!e->cap) HIPCK(hipStreamCreateWithFlags(&e->cap, hipStreamNonBlocking));
    if (split && !e->cap2) {
      HIPCK(hipStreamCreateWithFlags(&e->cap2, hipStreamNonBlocking));
      HIPCK(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
      HIPCK(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
    }
    auto ne = std::make_shared<GraphEntry>();
    ne->key = key;
    Ctx cc = c;
    cc.st = e->cap;
    cc.st2 = split ? e->cap2 : nullptr;
    const double c0 = host_ms();
    hipError_t be = hipStreamBeginCapture(e->cap, hipStreamCaptureModeThreadLocal);
    if (be != hipSuccess) return fail(F5H_EHIP, std::string("hipStreamBeginCapture: ") + hipGetErrorString(be));
    const int rc = body(cc);
    hipGraph_t graph = nullptr;
    const hipError_t ce = hipStreamEndCapture(e->cap, &graph);
    if (rc || ce != hipSuccess) {
      if (graph) (void)hipGraphDestroy(graph);
      if (rc) return rc;
      return fail(F5H_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
    }
    const double c1 = host_ms();
    const hipError_t ie = hipGraphInstantiate(&ne->exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (c.hp) {
      c.hp[HP_CAPTURE] += c1 - c0;
      c.hp[HP_INSTANTIATE] += host_ms() - c1;
    }
    if (host_trace())
      std::fprintf(stderr, "[f5h host] capture %.3f ms, instantiate %.3f ms\n", c1 - c0, host_ms() - c1);
    if (ie != hipSuccess) {
      ne->exec = nullptr;
      return fail(F5H_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
    }
    if (e->graphs.size() >= kGraphCache) {  // evict the least recently used graph to the graveyard
      size_t lru = 0;
      for (size_t i = 1; i < e->graphs.size(); ++i)
        if (e->graphs[i]->stamp < e->graphs[lru]->stamp) lru = i;
      e->graveyard.push_back(std::move(e->graphs[lru]));
      e->graphs.erase(e->graphs.begin() + lru);
      ++e->n_evicted;
    }
    e->graphs.push_back(ne);
    e->n_captures++;
    hold = ne;
  }
  hold->stamp = ++e->use_ctr;
  e->n_replays += replays;
  return 0;
}

// Prologue graphs pay off only when a shape repeats: true when the prologue graph for `key` is
// cached or the key was seen before (remembered in a short FIFO); a first sighting is recorded.
static bool prologue_repeats(f5h_engine* e, const GraphKey& key) {
  std::lock_guard<std::mutex> g(e->gm);
  for (const auto& x : e->graphs)
    if (x->key == key) return true;
  for (const auto& k : e->pro_seen)
    if (k == key) return true;
  if (e->pro_seen.size() >= 64) e->pro_seen.erase(e->pro_seen.begin());
  e->pro_seen.push_back(key);
  return false;
}

int f5h_forward(f5h_engine* e, void* stream, const f5h_forward_args* a, void* workspace, size_t workspace_bytes) {
  if (!e || !a) return fail(F5H_EINVAL, "null engine/args");
  if (a->B <= 0 || a->N <= 0 || a->nt < 0) return fail(F5H_EINVAL, "bad B/N/nt");
  if (!a->x || !a->cond || !a->cond_mask || !a->duration || !a->pred || (a->nt > 0 && !a->text))
    return fail(F5H_EINVAL, "null tensor argument");
  HIPCK(hipSetDevice(e->dev));
  UseNote used{e->uses, reinterpret_cast<hipStream_t>(stream)};
  Ctx c{};
  c.e = e;
  c.st = reinterpret_cast<hipStream_t>(stream);
  c.B = a->B;
  c.N = a->N;
  c.nt = a->nt;
  c.nfe = 1;
  c.use_cfg = a->cfg_infer ? 1 : 0;
  c.S = c.use_cfg ? 2 * c.B : c.B;
  c.drop_audio = (!c.use_cfg && a->drop_audio_cond) ? 1 : 0;
  c.drop_text = (!c.use_cfg && a->drop_text) ? 1 : 0;
  c.L = e->a.backbone == F5H_DIT ? c.N : c.N + 1;
  c.batch_mask = a->use_batch_mask ? 1 : 0;
  if (e->a.backbone == F5H_DIT && a->N > 8192) return fail(F5H_EINVAL, "N exceeds the text position table (8192)");
  if (a->text_cache < 0 || a->text_cache > 2) return fail(F5H_EINVAL, "text_cache must be 0, 1 or 2");
  RC(check_ws(e, c.B, c.N, 1, c.use_cfg, workspace, workspace_bytes, c));
  RC(chain_fault_check(e, c.st));
  ChainTicket ticket;
  c.chain = chain_for_call(e, c, ticket);
  c.lnfold = e->lnfold && !c.chain && ((e->lnf_ok && !c.batch_mask) || e->rmsf_ok);
  const bool cached = a->text_cache == 2;
  if (a->t_dev) {  // time read on the stream: no host round trip (dit.py:332-333 takes a tensor)
    HIPCK(hipMemcpyAsync(c.b.tgrid, a->t_dev, sizeof(float), hipMemcpyDeviceToDevice, c.st));
    RC(prologue(c, nullptr, 1, a->cond, a->cond_mask, a->text, a->duration, cached));
  } else {
    float tg[2] = {a->t, a->t};
    RC(prologue(c, tg, 1, a->cond, a->cond_mask, a->text, a->duration, cached));
  }
  HIPCK(pack_y(e->bf, a->x, c.B * c.N, e->a.mel_dim, c.b.ypad, c.st));
  HIPCK(hipMemsetAsync(c.b.kstep, 0, sizeof(int), c.st));
  auto body = [](Ctx& cc) -> int {
    cc.site = 0;
    RC(step_prep(cc));
    RC(backbone_step(cc));
    KCK(step_advance(cc.b.kstep, cc.e->ptick, cc.st));
    return 0;
  };
  if (e->graph_mode && a->text_cache != 0) {
    // a kept workspace is reused call after call (the reference's ODE loop over the plugin): the
    // backbone step (workspace buffers only) replays as one graph per (workspace, shape)
    GraphKey key{};
    key.ws = workspace;
    key.kind = 2;
    key.B = c.B;
    key.N = c.N;
    key.nt = c.nt;
    key.nfe = 1;
    key.use_cfg = c.use_cfg;
    key.batch_mask = c.batch_mask;
    key.probe = e->probe_class;
    key.pad_skip = e->pad_skip;
    key.chain = c.chain;
    key.lnfold = c.lnfold;
    key.kernel_epoch = g_kernel_epoch.load();
    std::shared_ptr<GraphEntry> hold;
    RC(graph_get(c, key, false, body, hold, 1));
    HIPCK(hipGraphLaunch(hold->exec, c.st));
    RC(note_replays(e, hold.get(), c.st));
  } else {
    RC(body(c));
  }
  HIPCK(copy_pred(c.b.p, c.S, c.L, e->a.backbone == F5H_DIT ? 0 : 1, e->a.mel_dim, e->proj_out.Npad, a->pred,
                  c.chain ? e->chain_fault : nullptr, c.st));
  if (c.chain) RC(chain_fault_note(e, c.st));
  return 0;
}

int f5h_probe_enable(f5h_engine* e, int32_t kclass, int32_t enable) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  std::lock_guard<std::mutex> g(e->pm);
  e->probe_class = enable ? kclass : -1;
  if (e->pstamp) {  // tick = 0, start stamps = max, end stamps = 0
    HIPCK(hipSetDevice(e->dev));
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipMemset(e->pstamp, 0, 64 * sizeof(unsigned long long)));
    HIPCK(hipMemset(e->pslots, 0xff, (size_t)kProbeEnd * sizeof(unsigned long long)));
    HIPCK(hipMemset(e->pslots + kProbeEnd, 0, (size_t)kProbeEnd * sizeof(unsigned long long)));
    HIPCK(hipMemset(e->ptl, 0, (size_t)kTimelineWG * 4 * sizeof(unsigned long long)));
    HIPCK(hipDeviceSynchronize());
  }
  return 0;
}

int f5h_probe_timeline(f5h_engine* e, uint64_t* stamps, int32_t max_wg, int32_t* n_wg, double* tick_khz) {
  if (!e || !stamps || max_wg <= 0) return fail(F5H_EINVAL, "null engine / buffer");
  std::lock_guard<std::mutex> g(e->pm);
  HIPCK(hipSetDevice(e->dev));
  HIPCK(hipDeviceSynchronize());
  const int n = std::min<int>(max_wg, kTimelineWG);
  HIPCK(hipMemcpy(stamps, e->ptl, (size_t)n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  int last = 0;
  for (int i = 0; i < n; ++i)
    if (stamps[4 * i]) last = i + 1;
  if (n_wg) *n_wg = last;
  if (tick_khz) *tick_khz = e->wall_khz;
  return 0;
}

int f5h_probe_read(f5h_engine* e, int64_t* launches, double* total_ms) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  std::lock_guard<std::mutex> g(e->pm);
  double ms = 0.0;
  int64_t n = 0;
  if (e->pstamp && e->wall_khz > 0.0) {
    HIPCK(hipSetDevice(e->dev));
    HIPCK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(2 * (size_t)kProbeEnd);
    HIPCK(hipMemcpy(h.data(), e->pslots, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long ticks = 0;
    for (int64_t i = 0; i < kProbeEnd; i += (int64_t)kProbeLanes * kProbeStride) {  // one (site, tick)
      unsigned long long t0 = ~0ull, t1 = 0;
      for (int l = 0; l < kProbeLanes; ++l) {
        t0 = std::min(t0, h[i + l * kProbeStride]);
        t1 = std::max(t1, h[kProbeEnd + i + l * kProbeStride]);
      }
      if (t1 == 0 || t0 == ~0ull || t1 < t0) continue;  // no finished launch at this site and tick
      ticks += t1 - t0;
      ++n;
    }
    ms = (double)ticks / e->wall_khz;
  }
  if (launches) *launches = n;
  if (total_ms) *total_ms = ms;
  return 0;
}

int f5h_set_graph_mode(f5h_engine* e, int32_t mode) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (mode != 0 && mode != 1) return fail(F5H_EINVAL, "graph mode must be 0 (eager) or 1 (step graph)");
  std::lock_guard<std::mutex> g(e->gm);
  e->graph_mode = mode;
  return 0;
}

int f5h_set_cfg_streams(f5h_engine* e, int32_t n) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (n < 0 || n > 2) return fail(F5H_EINVAL, "cfg streams must be 0 (auto), 1 or 2");
  std::lock_guard<std::mutex> g(e->gm);
  e->split_cfg = n == 0 ? 2 : (n == 2 ? 1 : 0);
  return 0;
}

int f5h_set_pad_skip(f5h_engine* e, int32_t enable) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (enable != 0 && enable != 1) return fail(F5H_EINVAL, "pad skip must be 0 or 1");
  std::lock_guard<std::mutex> g(e->gm);
  e->pad_skip = enable;
  return 0;
}

int f5h_set_chain(f5h_engine* e, int32_t enable) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (enable != 0 && enable != 1) return fail(F5H_EINVAL, "chain must be 0 or 1");
  std::lock_guard<std::mutex> g(e->gm);
  e->chain = enable;
  return 0;
}

int f5h_chain_stats(f5h_engine* e, int64_t* launches, int32_t* fault, int64_t* refused) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (launches) *launches = e->n_chain.load(std::memory_order_relaxed);
  if (refused) *refused = g_gate_refused.load(std::memory_order_relaxed);
  if (fault) {
    *fault = 0;
    if (e->chain_fault) {  // the caller has synchronised with the engine's calls (the device word is final)
      unsigned v = 0;
      HIPCK(hipSetDevice(e->dev));
      HIPCK(hipMemcpyAsync(&v, e->chain_fault, sizeof(v), hipMemcpyDeviceToHost, e->mstream));
      HIPCK(hipStreamSynchronize(e->mstream));
      *fault = v ? 1 : 0;
    }
  }
  return 0;
}

int f5h_set_ln_fold(f5h_engine* e, int32_t enable) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (enable != 0 && enable != 1) return fail(F5H_EINVAL, "ln fold must be 0 or 1");
  std::lock_guard<std::mutex> g(e->gm);
  e->lnfold = enable;
  return 0;
}

int f5h_ln_fold_stats(f5h_engine* e, int32_t* supported, int64_t* passes) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  if (supported) *supported = (e->lnf_ok || e->rmsf_ok) ? 1 : 0;
  if (passes) *passes = e->n_lnfold.load(std::memory_order_relaxed);
  return 0;
}

int f5h_last_call_host_ms(f5h_engine* e, double* ms, int32_t n) {
  if (!e || !ms || n <= 0) return fail(F5H_EINVAL, "null engine / buffer");
  std::lock_guard<std::mutex> g(e->hm);
  for (int i = 0; i < n; ++i) ms[i] = i < kHostPhases ? e->last_host[i] : 0.0;
  return 0;
}

int f5h_chain_debug_spin_limit(int64_t limit) {
  chain_set_spin_limit(limit);
  g_kernel_epoch.fetch_add(1);  // captured graphs hold the old kernel arguments
  return 0;
}

int f5h_graph_stats(f5h_engine* e, int64_t* captures, int64_t* replays, int32_t* cached) {
  if (!e) return fail(F5H_EINVAL, "null engine");
  std::lock_guard<std::mutex> g(e->gm);
  if (captures) *captures = e->n_captures;
  if (replays) *replays = e->n_replays;
  if (cached) *cached = (int32_t)e->graphs.size();
  return 0;
}

// ---------------------------------------------------------------- op-level entry points
int f5h_op_linear(void* stream, int32_t compute, int32_t M, int32_t N, int32_t K, const float* A, const float* W,
                  const float* bias, float* C, void* workspace, size_t workspace_bytes) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64) return fail(F5H_EINVAL, "op_linear needs K % 64 == 0");
  if (compute < F5H_FP32 || compute > F5H_FP16) return fail(F5H_EINVAL, "bad compute mode");
  const int Npad = (N + 127) / 128 * 128;
  const size_t es = compute ? 2 : 4;
  const size_t need = (size_t)Npad * K * es;
  if (workspace_bytes < (need + 255) / 256 * 256 + (size_t)M * K * es)
    return fail(F5H_ENOMEM, "workspace too small for op_linear");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIPCK(hipMemsetAsync(workspace, 0, need, st));
  HIPCK(f32_to_op(compute, W, (int64_t)N * K, workspace, st));
  const void* Aop = A;
  if (compute) {
    char* ab = reinterpret_cast<char*>(workspace) + (need + 255) / 256 * 256;
    HIPCK(f32_to_op(compute, A, (int64_t)M * K, ab, st));
    Aop = ab;
  }
  GemmArgs g{};
  g.A = Aop;
  g.lda = K;
  g.W = workspace;
  g.ldw = K;
  g.M = M;
  g.N = N;
  g.K = K;
  g.bias = bias;
  g.C = C;
  g.ldc = N;
  HIPCK(gemm(compute, EPI_STORE, g, st));
  return 0;
}

int f5h_gemm_force_config(int32_t cfg) {
  if (cfg != -1 && cfg != 0 && cfg != 1 && cfg != 5 && cfg != 11 && cfg != 12 && cfg != 13)
    return fail(F5H_EINVAL, "gemm config must be -1, 0, 1, 5, 11, 12 or 13");
  gemm_force_config(cfg);
  g_kernel_epoch.fetch_add(1);
  return 0;
}

int f5h_attn_force_safe(int32_t on) {
  attention_force_safe(on);
  g_kernel_epoch.fetch_add(1);  // captured graphs hold the old kernel arguments
  return 0;
}

int f5h_debug_tile_live(const int32_t* live_len, int32_t live_seq, int32_t M, int32_t m0, int32_t BM) {
  if (live_seq <= 0 || M <= 0 || BM <= 0 || m0 < 0 || m0 >= M) return fail(F5H_EINVAL, "bad tile");
  return tile_live_rows(live_len, live_seq, M, m0, BM) ? 1 : 0;
}

int f5h_op_attention(void* stream, int32_t compute, int32_t S, int32_t H, int32_t N, const float* Q, const float* K,
                     const float* V, const int32_t* kv_len, int32_t q_prescaled, float* O, void* workspace,
                     size_t workspace_bytes) {
  if (S <= 0 || H <= 0 || N <= 0) return fail(F5H_EINVAL, "bad attention shape");
  if (compute < F5H_FP32 || compute > F5H_FP16) return fail(F5H_EINVAL, "bad compute mode");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)S * H * N * 64;
  AttnArgs at{};
  at.S = S;
  at.H = H;
  at.L = N;
  at.kv_len = kv_len;
  at.scale = 0.125f;
  at.prescaled = q_prescaled ? 1 : 0;
  if (compute) {
    const size_t need = (size_t)n * 2 * 4 + 4 * 256;
    if (workspace_bytes < need) return fail(F5H_ENOMEM, "workspace too small for op_attention");
    char* w = reinterpret_cast<char*>(workspace);
    void *q = w, *k = w + n * 2, *v = w + n * 4, *o = w + n * 6;
    HIPCK(f32_to_op(compute, Q, n, q, st));
    HIPCK(f32_to_op(compute, K, n, k, st));
    HIPCK(f32_to_op(compute, V, n, v, st));
    at.q = q;
    at.k = k;
    at.v = v;
    at.o = o;
    HIPCK(attention(compute, at, st));
    HIPCK(op_to_f32(compute, o, n, O, st));
  } else {
    at.q = Q;
    at.k = K;
    at.v = V;
    at.o = O;
    HIPCK(attention(0, at, st));
  }
  return 0;
}

}  // extern "C"
