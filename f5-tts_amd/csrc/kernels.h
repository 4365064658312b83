// Launcher declarations for the engine's HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace f5h {

// Operand dtype of a compute mode (f5h_compute in include/f5h.h): GEMM/attention/conv operands are
// fp32 (parity mode), bf16 or fp16; accumulation, residual stream, norms and the ODE state stay fp32.
enum ComputeMode { F5H_C_FP32 = 0, F5H_C_BF16 = 1, F5H_C_FP16 = 2 };

enum Epi {
  EPI_STORE = 0,      // C = acc + bias                                  (fp32 out)
  EPI_SILU = 1,       // C = silu(acc + bias)                            (fp32 out)
  EPI_GELU_TANH = 2,  // C = gelu_tanh(acc + bias)                       (operand out)
  EPI_GELU_ERF = 3,   // C = gelu_erf(acc + bias)                        (fp32 out)
  EPI_RESID = 4,      // C += gate[n] * (acc + bias) * rowkeep[m]        (fp32 in/out)
  EPI_RESID_FILL = 5, // C = rowkeep[m] ? C + acc + bias : 0             (fp32 in/out)
  EPI_INPROJ = 6,     // C[m] = acc + add[m]; C[m+dual] = acc + add[m+dual]  (fp32)
  EPI_QKV = 7,        // RoPE + scatter to q/k/v [S,H,L,64]              (operand out)
  EPI_GELU_ERF_OP = 8,  // C = gelu_erf(acc + bias)                      (operand out; Vocos pwconv1)
  EPI_RESID16 = 9,   // C += gate[n] * (acc + bias) * rowkeep[m]        (operand dtype in/out: 16-bit residual)
  EPI_STORE16 = 10,  // C = acc + bias                                   (operand out: UNetT skip_proj)
};
// EPI_RESID / EPI_RESID16 read the residual from `resid` when set (else from C) and write C, so a
// layer can keep its input (UNetT skip connections) without a copy.

// In-kernel launch probe (see probe_enter/probe_exit in common.h). Per launch site a row of
// kProbeTicks x kProbeLanes entries, each on its own 128-B line (kProbeStride words): workgroup b
// stamps lane b % kProbeLanes, so same-line atomics stay few; the start rows (atomicMin) come
// first, the end rows (atomicMax) kProbeEnd words further on. Host: min/max over lanes.
// Only every kProbeEvery-th step tick is stamped (the rest run unperturbed apart from one load).
constexpr int kProbeTicks = 512, kProbeSites = 64, kProbeLanes = 16, kProbeStride = 16, kProbeEvery = 4;
constexpr int64_t kProbeRow = (int64_t)kProbeTicks * kProbeLanes * kProbeStride;
constexpr int64_t kProbeEnd = kProbeRow * kProbeSites;
struct DevProbe {
  unsigned long long* slots;  // null: not probed
  const int* tick;            // device step tick
  // per-workgroup timeline of the tick-0 launch of the first probed site (diagnostic, or null):
  // tl[wg*4 + {0: entry, 1: main loop entered (first stage landed), 2: main loop done, 3: exit}]
  unsigned long long* tl;
};
constexpr int kTimelineWG = 8192;  // workgroups recorded per timeline

struct GemmArgs {
  const void* A; int64_t lda;      // [M,K] row-major, TA elements
  const void* W; int64_t ldw;      // [Npad,K] row-major, operand elements (rows padded to 128)
  int M, N, K;                     // K: multiple of 64 (bf16) / 32 (fp32)
  const float* bias;               // [N] or null
  void* C; int64_t ldc;            // output
  const float* gate;               // EPI_RESID: [N] or null (=1)
  const uint8_t* rowkeep;          // [M] or null (=1)
  const float* add; int64_t ld_add;  // EPI_INPROJ addend
  int64_t dual_rows;               // EPI_INPROJ: second output at row m + dual_rows (0 = none)
  // EPI_QKV
  const float2* rope;              // [L][32] (cos, sin)
  int seq_len;                     // L: rows per sequence
  int heads, rope_heads;
  void* q; void* k; void* v;
  float q_scale;                   // EPI_QKV: q is stored pre-multiplied by this (0 -> 1)
  DevProbe probe;                  // in-kernel launch timing (null slots: off)
  const void* resid;               // EPI_RESID / EPI_RESID16 residual input (null: C)
  const void* A2; int k_split;     // A columns [k_split, K) come from A2 (same lda), e.g. cat(x, skip)
  // EPI_RESID / EPI_RESID16 with rowkeep: the live rows of sequence s are [s*live_seq, s*live_seq +
  // live_len[s]); a tile with no live row skips its K loop and epilogue (its rows keep the residual, as
  // the masked rows of a computed tile do). Null: every tile is computed.
  const int32_t* live_len; int live_seq;
  int group_m;                     // persistent kernel (cfg 13): tile order in groups of this many row tiles (<= 1: n-fastest)
  // LayerNorm fold (DiT 16-bit path without row masks; DESIGN.md §3 'LayerNorm fold'). The AdaLN LayerNorm between a
  // residual GEMM and its consumer, aop = LN(h) (1 + sc) + sh (modules.py:325,753), runs as algebra in the two GEMMs:
  // producer (EPI_RESID16, hs != null): besides h, writes hs = round(h' (1 + hs_scale[n])) (h' = the stored, rounded
  //   h; operand dtype, row stride ldc) and, per row and 64-column strip p, the strip's (mean, M2) of h' into
  //   ln_part[row * ln_nparts + p] (float2; ln_nparts = N / 64);
  // consumer (EPI_GELU_TANH / EPI_QKV, ln_part_in != null; A = hs): combines the row's ln_nparts partials into
  //   (mean_m, rstd_m) and applies x = rstd_m (acc - mean_m ln_u[n]) + ln_v[n] before the bias, where
  //   ln_u[n] = sum_k (1 + sc_k) W[n,k] and ln_v[n] = sum_k sh_k W[n,k] (lnfold_uv, per ODE step).
  void* hs; const float* hs_scale; float* ln_part;
  const float* ln_part_in; int ln_nparts; const float* ln_u; const float* ln_v;
  // RMSNorm form (UNetT, x_transformers RMSNorm: x / max(|x|, 1e-12) sqrt(d) g): ln_rms = 1. The producer writes
  // (0, sum of squares) per strip and no hs (hs, hs_scale null); the consumer reads the residual stream itself as A,
  // its W already carries the gain (W' = W diag(g), built once), ln_u / ln_v are null (0) and rstd = 1 / sqrt(ss / d +
  // ln_eps). ln_eps: the consumer's variance epsilon (LayerNorm: 1e-6, modules.py:316,336).
  int ln_rms; float ln_eps;
};

// Does the row tile [m0, m0 + BM) of an M-row GEMM hold a live row? Sequence s (rows [s*live_seq, (s+1)*live_seq))
// contributes the tile's rows [max(m0, r0), min(last + 1, r0 + live_seq)); its live rows are [r0, r0 +
// live_len[s]): the tile is live iff one of those overlaps is non-empty. Null live_len: always live. Host and
// device (the GEMM kernels' pad-row skip; f5h_debug_tile_live checks it from the CPU tests).
__host__ __device__ inline bool tile_live_rows(const int32_t* live_len, int live_seq, int M, int m0, int BM) {
  if (!live_len) return true;
  const int last = (m0 + BM < M ? m0 + BM : M) - 1;
  for (int s = m0 / live_seq; s <= last / live_seq; ++s) {
    const int r0 = s * live_seq;
    const int lo = m0 > r0 ? m0 : r0;
    const int hi_tile = last + 1, hi_live = r0 + live_len[s];
    if (lo < (hi_tile < hi_live ? hi_tile : hi_live)) return true;
  }
  return false;
}

// compute: ComputeMode (fp32 / bf16 / fp16 operands). A and W both in the operand dtype.
hipError_t gemm(int compute, int epi, const GemmArgs& a, hipStream_t st);
// pin the 16-bit GEMM tile configuration (0, 1, 5, 11, 12, 13; -1 = automatic choice); tuning and test hook
void gemm_force_config(int cfg);

// attention: Q,K,V [S,H,L,64] operand dtype; O [S,L,H*64] operand dtype.
struct AttnArgs {
  const void* q; const void* k; const void* v; void* o;
  int S, H, L;
  const int32_t* kv_len;  // [S] or null: keys [kv_len[s], L) masked
  // [S] or null: query rows [q_len[s], L) are dead (their output is masked to 0 after to_out,
  // modules.py:551-553): query blocks wholly past q_len[s] exit at entry and leave O unwritten
  const int32_t* q_len;
  float scale;            // 1/sqrt(64)
  int prescaled;          // q already carries scale*log2(e): scores are in log2 units
  DevProbe probe;         // in-kernel launch timing (null slots: off)
  int force_safe;         // test hook: every workgroup reruns its key loop in the lazy-max form (attention.hip)
};
hipError_t attention(int compute, const AttnArgs& a, hipStream_t st);
// test hook (f5h_attn_force_safe): 1 = every later 16-bit attention launch takes the SAFE rerun
void attention_force_safe(int on);

// grouped conv1d k=31, 16 groups, pad 15 (ConvPositionEmbedding, modules.py:175-201)
struct ConvArgs {
  const void* x; int x_f32;        // [S, L, d] input (fp32 or operand dtype)
  const void* w;                   // packed [16][31][64 out][64 in] operand dtype
  const float* bias;               // [d]
  const uint8_t* rowkeep;          // [S*L] or null: input rows masked, output rows masked
  int S, L, d;
  // output: mode 0 -> y (operand dtype) = mish(mask(conv)); mode 1 -> y fp32 = mish(mask(conv)) + resid;
  // mode 2 (16-bit operands) -> y operand dtype = mish(mask(conv)) + resid (the 16-bit residual stream)
  int mode;
  void* y; int64_t y_seq_stride; int64_t y_row_off;  // in rows
  const float* resid;              // [S, L, d] fp32 (mode 1)
};
hipError_t conv_pos(int compute, const ConvArgs& a, hipStream_t st);

// ---- elementwise / small kernels (elementwise.hip)
hipError_t time_sinus(const float* t_host, int n, float* out, hipStream_t st);  // host t[n<=512] -> [n,256]
hipError_t time_sinus_dev(const float* tg, int n, float* out, hipStream_t st);  // device t[n]
hipError_t silu_to_op(int compute, const float* x, void* y, int64_t n, hipStream_t st);
// LayerNorm(no affine, eps) * (1 + scale) + shift -> operand dtype; h: [M, d] fp32, or the operand
// dtype when h16 (the 16-bit residual stream of the bf16/fp16 DiT path)
hipError_t ln_modulate(int compute, const void* h, int h16, int M, int d, const float* shift, const float* scale,
                       void* out, hipStream_t st);
// x_transformers RMSNorm: x / max(||x||, 1e-12) * sqrt(d) * g -> operand dtype
// h: fp32, or the operand dtype when h16 (16-bit residual stream)
hipError_t rms_norm_g(int compute, const void* h, int h16, int M, int d, const float* g, void* out, hipStream_t st);
// out[n][k] = round(W[n][k] g[k]) for rows x K 16-bit W (the RMSNorm fold's W' = W diag(g), built once per engine)
hipError_t scale_cols(int compute, const void* W, int64_t rows, int K, const float* g, void* out, hipStream_t st);
hipError_t rope_table(int L, float2* out, hipStream_t st);
// text tokens -> embeddings (dit.py:86-120 / unett.py:53-64), both branches
struct TextEmbArgs {
  const int64_t* text; int B, nt, N, td;
  const int32_t* seq_len;       // [B] per-sample valid length or null (= N for all)
  const float* table;           // [V, td]
  const float* freqs;           // [8192, td] or null (no sinus pos)
  int mask_padding;
  float* out_c; float* out_u;   // [B, N, td] each
  uint8_t* keep;                // [2B*N] !fill (for masked_fill after each block) or null
};
hipError_t text_embed(const TextEmbArgs& a, hipStream_t st);
// depthwise conv k7 pad3 + bias then LayerNorm(affine, eps 1e-6) -> operand dtype. x: [S, L, C] fp32
hipError_t dwconv_ln(int compute, const float* x, int S, int L, int C, const float* dw_w, const float* dw_b,
                     const float* ln_w, const float* ln_b, void* out, hipStream_t st);
// GRN: sumsq[s,c] = sum_n x^2 ; then out = gamma*(x*Nx)+beta+x -> operand dtype
hipError_t grn(int compute, const float* x, int S, int L, int C, const float* gamma, const float* beta,
               float* scratch /*[(ceil(L/64)+1)*S*C]*/, void* out, hipStream_t st);
// A_ct [S*N, 128 + td] operand dtype: [where(cond_mask,cond,0) (zeros for uncond) pad 128 | text];
// drop_audio / drop_text apply to the first (conditional) B sequences (single-branch forward)
hipError_t build_ct(int compute, const float* cond, const uint8_t* cond_mask, const float* text_c,
                    const float* text_u, int B, int N, int td, int S, int drop_audio, int drop_text, void* out,
                    hipStream_t st);
// y (fp32 [B,N,mel]) -> ypad operand [B*N, 128]
hipError_t pack_y(int compute, const float* y, int rows, int mel, void* ypad, hipStream_t st);
// CFG + Euler: y += dt * (pc + (pc - pu) * cfg); pred rows from p with row offset/stride.
struct EulerArgs {
  float* y; int B, N, mel;
  const float* p; int64_t p_seq_stride; int p_row_off; int64_t p_ld;  // p[s, row_off + n, c]
  int use_cfg; float cfg; float dt;
  void* ypad; int compute;      // refreshed operand copy (or null)
  float* traj;                  // [B,N,mel] slot to copy y into (or null)
  // device-indexed form (graph replay): when kstep is set, dt = tgrid[k+1] - tgrid[k] and the
  // trajectory slot is traj + (k+1)*B*N*mel, k = *kstep (dt above is ignored)
  // trajectory base (or null) read from *trajp in the device-indexed form
  const int* kstep; const float* tgrid; float* const* trajp;
  // the step bookkeeping folded into this launch (device-indexed form): next_dst[0..next_n) =
  // next_src[(k+1) * next_stride ..] for k + 1 < nfe (the next step's AdaLN / time-token row), and
  // the workgroup that arrives last on *arrive (zeroed per call) bumps *kstep and *tick once every
  // workgroup has read k. next_dst null: no copy; arrive null: no bump.
  const float* next_src; int64_t next_stride; int next_n; float* next_dst; int nfe;
  unsigned* arrive; int* tick;
};
hipError_t cfg_euler(const EulerArgs& a, hipStream_t st);
// host grid t[n <= 512] -> device (by kernel argument)
hipError_t grid_upload(const float* t_host, int n, float* out, hipStream_t st);
// dst[0..n) = src[k*stride ..], k = *kstep (n, stride multiples of 4)
hipError_t step_begin(const int* kstep, const float* src, int64_t stride, int n, float* dst, hipStream_t st);
// probe stamps around a launch (DevProbe slot layout), indexed by *tick
hipError_t stamp_begin(unsigned long long* slots, const int* tick, hipStream_t st);
hipError_t stamp_end(unsigned long long* slots, const int* tick, hipStream_t st);
// *kstep += 1 and *tick += 1 (probe step tick)
hipError_t step_advance(int* kstep, int* tick, hipStream_t st);
// p[0..n) = 0 (n a multiple of 4, p 16-B aligned): a kernel, not a memset node
hipError_t zero_words(unsigned* p, int64_t n, hipStream_t st);
hipError_t final_where(const float* cond, const uint8_t* cond_mask, float* y, int B, int N, int mel,
                       hipStream_t st);
// fault: the phase-chain give-up word (or null); when set, out is filled with NaN (the results are wrong)
hipError_t final_where_out(const float* cond, const uint8_t* cond_mask, const float* y, float* out, int B, int N,
                           int mel, const unsigned* fault, hipStream_t st);
// *slot = p (stream-ordered)
hipError_t ptr_upload(float* p, float** slot, hipStream_t st);
// rowkeep[s*L + pos] = (pos - off < dur[s % B]) || pos < off ; for S sequences
hipError_t build_rowkeep(const int32_t* dur, int B, int S, int L, int off, uint8_t* keep, hipStream_t st);
// kv_len[s] = dur[s % B] + off
hipError_t build_kvlen(const int32_t* dur, int B, int S, int off, int32_t* kv, hipStream_t st);
// h[s, 0, :] = temb (UNetT time token)
hipError_t write_time_token(int compute, int h16, const float* temb, int S, int L, int d, void* h, hipStream_t st);
// extract rows [s, 1..L-1] of pred -> dst [S, L-1, mel]; NaN when *fault (as final_where_out)
hipError_t copy_pred(const float* p, int S, int L, int row_off, int mel, int64_t p_ld, float* dst,
                     const unsigned* fault, hipStream_t st);
// Vocos decoder glue (vocos.hip)
hipError_t vocos_im2col(int compute, const float* mel, int B, int T, int C, int Kp, void* out, hipStream_t st);
hipError_t vocos_spec(float* x, int64_t rows, int bins, int ld, hipStream_t st);
hipError_t vocos_ola(const float* frames, const float* win, int B, int T, int n_fft, int hop, float* y,
                     hipStream_t st);
// log-mel front end glue (melspec.hip)
hipError_t mel_frames(const float* wav, int B, int L, int T, int n_fft, int hop, float* frames, hipStream_t st);
hipError_t mel_mag(const float* spec, int64_t rows, int bins, int ld_spec, int ld_mag, float* mag, hipStream_t st);
hipError_t mel_log(const float* mel, int B, int T, int n_mels, float* out, hipStream_t st);
hipError_t f32_to_op(int compute, const float* x, int64_t n, void* out, hipStream_t st);
hipError_t op_to_f32(int compute, const void* x, int64_t n, float* out, hipStream_t st);
// Weight packing (engine creation): dst[i0*dst_st[0] + i1*dst_st[1] + i2*dst_st[2] + i3] =
// cvt(src[i0*src_st[0] + i1*src_st[1] + i2*src_st[2] + i3*src_st[3]]) for i < n; element types
// 0 = fp32, 1 = bf16, 2 = fp16 (f5h_dtype); conversions round to nearest even.
struct PackArgs {
  const void* src; int src_dt; int64_t src_st[4];
  void* dst; int dst_dt; int64_t dst_st[3];
  int n[4];
};
hipError_t pack_strided(const PackArgs& a, hipStream_t st);

// ---- In-launch phase chain (chain.hip): the row-local seams of a DiT block-step (out-proj -> LayerNorm ->
// FFN1 -> FFN2 -> LayerNorm -> next QKV) as ONE launch whose phases hand row groups (kChainRows rows) to the
// next phase through per-group arrival counters (cdna_hip_programming.md §6 Guideline 16, R1: write-through
// payload, drained, one counter add per workgroup; the consumer polls relaxed and acquires once).
constexpr int kChainRows = 64;
struct ChainDep {
  const unsigned* wait;  // the producer phase's row-group counters (null: no in-launch producer)
  int wait_mult, wait_unit;  // a complete group holds wait_mult * ceil(rows of the group / wait_unit) arrivals
  unsigned* pub;         // this phase's row-group counters (null: last phase)
  unsigned* err;         // the engine's fault word: set to 1 when a wait gives up (bounded spin); results then wrong
  unsigned spin_limit;   // polls before a wait gives up
  unsigned long long* tl;  // (set per workgroup in the kernel) its timeline row when the launch is probed, or null
};
struct LnArgs {
  const void* h;  // [M, 1024] residual stream (operand dtype)
  void* out;      // [M, 1024] LN(h) * (1 + scale) + shift
  const float* shift;
  const float* scale;
};
struct ChainArgs {
  GemmArgs out, ff1, ff2, qkv;  // qkv.M == 0: no QKV phase (the model's last layer)
  LnArgs ln1, ln2;
  unsigned* cnt;   // [5][groups] arrival counters, zero before the launch
  int groups;      // ceil(M / kChainRows) (stride of cnt)
  unsigned* fault; // the engine's give-up word (device): a wait that gives up sets it to 1 (f5h_sample then
                   // returns NaN in `out`, and the engine's next call fails with F5H_EHIP)
  DevProbe probe;  // launch timing (f5h_probe_enable "chain"); timeline row per workgroup: entry, rows acquired,
                   // results stored, exit
};
// bytes of cnt a chain launch over M rows uses (the caller zeroes them before the first layer's launch of a step:
// every layer's launch has its own [5][groups] block)
inline size_t chain_counter_bytes(int M) {
  return (size_t)5 * ((M + kChainRows - 1) / kChainRows) * sizeof(unsigned);
}
// LayerNorm fold: out[s][l*LW + {0: u1, F: v1, 2F: u2, 2F+3d: v2} + n] (LW = 2F + 6d, rows of `stride` floats,
// first column out_off) for every ODE step s < nfe and layer l < depth, with sc/sh the step's AdaLN rows of the
// layer in table[s] (modulation layout of modules.py:321-323): FFN1 (W1 [F][d], mlp scale/shift) and QKV
// (Wqkv [3d][d], msa scale/shift). u = sum_k (1 + sc_k) W[n,k], v = sum_k sh_k W[n,k], fp32.
struct LnFoldArgs {
  float* table; int64_t stride; int64_t out_off;
  int nfe, depth, d, F;
  const void* const* w1;    // [depth] device pointers (operand dtype [F][d])
  const void* const* wqkv;  // [depth] device pointers (operand dtype [3d][d])
};
hipError_t lnfold_uv(int compute, const LnFoldArgs& a, hipStream_t st);

// Launch the chain (16-bit operands, dim 1024, whole-column tiles); hipErrorInvalidValue when the shapes do not
// fit it (the caller then issues the separate launches).
hipError_t chain_launch(int compute, const ChainArgs& a, hipStream_t st);
// polls before a chain wait gives up: kChainSpinLimit by default; test hook (f5h_chain_debug_spin_limit) to force
// give-ups, -1 restores the default. Read at launch (graphs captured earlier keep their value)
void chain_set_spin_limit(long long limit);

}  // namespace f5h
