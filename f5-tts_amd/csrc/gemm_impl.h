// MFMA GEMM with fused epilogues: C[M,N] = A[M,K] . W[N,K]^T (+ epilogue).
//
// Every nn.Linear on the CFM hot path lands here: QKV + RoPE
// (modules.py:481-509), out-proj + gated residual (modules.py:548-554,751), FFN1 + GELU-tanh
// and FFN2 + gated residual (modules.py:359-361,754-755), the hoisted input projection
// (dit.py:162), proj_out (dit.py:368), the all-steps AdaLN table (modules.py:321-323) and
// the ConvNeXt pointwise convs (modules.py:265-269).
//
// Main loop: 256 threads = 4 waves as 2x2, block tile BM x 128 (BM = 128, or 64 when the
// 128-row grid would leave CUs without a second block), K staged 128 bytes per row per
// stage (64 bf16 / 32 fp32) by LDS-DMA (global_load_lds) into a double-buffered,
// XOR-swizzled LDS image; A and W are both K-contiguous operand-dtype panels, so every
// fragment is one ds_read_b128. bf16 mode: v_mfma_f32_16x16x32_bf16; fp32 parity mode:
// v_mfma_f32_16x16x4_f32 (exact f32).
// Epilogue: the fp32 accumulator tile is staged through LDS (padded rows) and re-read
// row-contiguously, so every global access of the epilogue (bias, gate, residual, RoPE
// table, q/k/v scatter) is a 16-32 byte vector access on whole rows.
//
// This header holds the kernels and their launch templates; gemm.hip holds the host-side tile
// choice and the dtype dispatcher, gemm_{bf16,f16,f32}*.hip instantiate the launchers (split so
// that hipcc builds them in parallel).
#pragma once
#include "common.h"
#include "kernels.h"
#include "chain.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace f5h {

// tile configuration for a 16-bit GEMM of this shape (forced, F5H_GEMM_CFG, F5H_GEMM_MAP, or pick_cfg)
int gemm_select_cfg(const GemmArgs& a);


// Block tile BM x BN with WGM x WGN waves; every wave owns a (BM/WGM) x (BN/WGN) sub-tile.
// KB = bytes of K per row per LDS stage: 128 (64 bf16, two MFMA k-slabs per barrier) or 64 (32 bf16,
// one slab: half the bytes per stage, so the same LDS holds a ring twice as deep).
template <int BM, int BN, int WGM, int WGN, int NS, int KB = 128>
struct GemmCfg {
  static constexpr int NW = WGM * WGN, THREADS = 64 * NW;
  static constexpr int WM = BM / WGM, WN = BN / WGN, MT = WM / 16, NT = WN / 16;
  static constexpr int CPR = KB / 16;                        // 16-B chunks per row per stage
  static constexpr int stage_bytes = (BM + BN) * KB;
  static constexpr int main_bytes = NS * stage_bytes;
  static constexpr int EPAD = WN + 4;                        // fp32 row of a wave's epilogue strip
  static constexpr int epi_bytes = NW * 16 * EPAD * 4;       // one 16-row strip per wave
  static constexpr int bytes = main_bytes > epi_bytes ? main_bytes : epi_bytes;
  static_assert(KB == 128 || KB == 64, "stage row bytes");
  static_assert(BM * CPR % THREADS == 0 && BN * CPR % THREADS == 0, "whole DMA rounds per stage");
  static_assert(MT * 16 == WM && NT * 16 == WN && MT + NT <= 15, "fragment counts (lgkmcnt <= 15)");
};

// 64-byte rows (K32 stages): chunk c of row r sits at c ^ f[(r>>2)&3], f = {0,2,3,1}: conflict-free
// for ds_read_b128, whose four 16-lane groups ({0-3,12-15,20-27}, ...) each read rows {r, r+12}
// at chunk c and rows r+4..r+11 at chunk c+1.
F5H_DEV int swz64(int row, int chunk) {
  const int b = (row >> 2) & 3;
  return chunk ^ ((0x1320 >> (4 * b)) & 3);  // f = {0,2,3,1}
}

// 128-byte rows (K64 stages) as the GEMM reads them: lane l takes row l & 15 (of a 16-row fragment
// tile) at logical chunk 4*slab + (l >> 4). ds_read_b128 serves lanes in the groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63} (MI355X_MICROARCH.md, LDS), i.e. rows
// {0-3,12-15} at one chunk and rows 4-11 at the chunk of the next lane quarter (c ^ 1). Chunk c of row
// r sits at c ^ (((r >> 1) & 7) ^ [4 <= r & 15 < 12]): every group then covers each (row parity,
// 16-B slot) pair once, so the fragment reads are conflict-free (swz128, laid out for 16 consecutive
// lanes, is 2-way here: SQ_LDS_BANK_CONFLICT ~ 0.9 x the LDS read cycles, profiles/r02_pmc_lds_gemm.txt).
F5H_DEV int swz128g(int row, int chunk) {
  const int r = row & 15;
  return chunk ^ ((r >> 1) ^ ((unsigned)(r - 4) < 8u ? 1 : 0));
}

// ds_read_b128 the compiler does not see (no waitcnt bookkeeping): the caller waits lgkmcnt itself
template <int OFF>
F5H_DEV u32x4 lds_read_b128(uint32_t addr) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// 8 consecutive fp32 values of one row
struct V8 {
  float v[8];
};

template <typename TC>
F5H_DEV void store8(TC* p, const V8& x);
template <>
F5H_DEV void store8<float>(float* p, const V8& x) {
  *reinterpret_cast<float4*>(p) = make_float4(x.v[0], x.v[1], x.v[2], x.v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(x.v[4], x.v[5], x.v[6], x.v[7]);
}
template <>
F5H_DEV void store8<bf16>(bf16* p, const V8& x) {
  bf16x8 b = {f2bf(x.v[0]), f2bf(x.v[1]), f2bf(x.v[2]), f2bf(x.v[3]),
              f2bf(x.v[4]), f2bf(x.v[5]), f2bf(x.v[6]), f2bf(x.v[7])};
  *reinterpret_cast<bf16x8*>(p) = b;
}
template <>
F5H_DEV void store8<f16>(f16* p, const V8& x) {
  f16x8 b = {(f16)x.v[0], (f16)x.v[1], (f16)x.v[2], (f16)x.v[3], (f16)x.v[4], (f16)x.v[5], (f16)x.v[6], (f16)x.v[7]};
  *reinterpret_cast<f16x8*>(p) = b;
}
F5H_DEV V8 load8(const float* p) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  return V8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}
F5H_DEV V8 load8(const bf16* p) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
  return V8{{(float)v[0], (float)v[1], (float)v[2], (float)v[3], (float)v[4], (float)v[5], (float)v[6], (float)v[7]}};
}
F5H_DEV V8 load8(const f16* p) {
  const f16x8 v = *reinterpret_cast<const f16x8*>(p);
  return V8{{(float)v[0], (float)v[1], (float)v[2], (float)v[3], (float)v[4], (float)v[5], (float)v[6], (float)v[7]}};
}
// the residual stream's element type: fp32, or the operand dtype for EPI_RESID16
template <typename TC, int EPI>
using ResT = typename std::conditional<EPI == EPI_RESID16, TC, float>::type;

// Epilogue arithmetic with explicit rounding (no FMA contraction), shared by every kernel so that
// all tile configurations stay bitwise identical whatever the compiler contracts around them.
F5H_DEV float rope_re(float a, float b, float c, float s) { return sub_nc(mul_nc(a, c), mul_nc(b, s)); }
F5H_DEV float rope_im(float a, float b, float c, float s) { return add_nc(mul_nc(b, c), mul_nc(a, s)); }
// gated residual update of a kept row; a masked (pad) row keeps its residual: masked_fill(~mask, 0) of the
// sub-layer output, then x + gate * 0 (modules.py:551-554). A select, not a multiply by the mask, so that
// the result never depends on the pad row's sub-layer output (which the pad-row skip leaves unwritten).
F5H_DEV float resid_add(float c, float gate, float x, bool keep) { return keep ? add_nc(c, mul_nc(gate, x)) : c; }

// n / d for 0 <= n < 2^24, d > 0: float quotient + one-step correction (no integer division loop)
F5H_DEV int fdiv(int n, int d) {
  int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
  q -= q * d > n;
  q += (q + 1) * d <= n;
  return q;
}

// Does the row tile [m0, m0 + BM) hold a live row (GemmArgs::live_len)? Wave-uniform (scalar loads).
// (tile_live_rows: kernels.h, host-callable too: f5h_debug_tile_live and tests/test_host.py check it)
F5H_DEV bool tile_live(const GemmArgs& g, int m0, int BM) {
  return tile_live_rows(g.live_len, g.live_seq, g.M, m0, BM);
}

// Apply the epilogue to 8 consecutive columns [col, col+8) of output row `row`.
template <typename TC, int EPI>
F5H_DEV void epi8(const GemmArgs& g, int row, int col, V8 x, const V8* pre = nullptr) {
  const bool full = col + 8 <= g.N;
  if (g.bias) {
    if (full) {
      V8 b = load8(g.bias + col);
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = add_nc(x.v[e], b.v[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = add_nc(x.v[e], col + e < g.N ? g.bias[col + e] : 0.f);
    }
  }
  if constexpr (EPI == EPI_QKV) {
    // interleaved RoPE pairs (2i, 2i+1) (x_transformers rotate_half) never straddle an 8-column chunk;
    // a 64-column head maps to one contiguous 128 B row segment of q/k/v [S,H,L,64]
    const int inner = g.heads * 64;
    const int which = fdiv(col, inner), hc = col - which * inner;
    const int head = hc >> 6, dh = hc & 63;
    const int s = fdiv(row, g.seq_len), pos = row - s * g.seq_len;
    if (which < 2 && head < g.rope_heads) {
      const float4* cs = reinterpret_cast<const float4*>(g.rope + (int64_t)pos * 32 + (dh >> 1));
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        float4 c2 = cs[pr];  // (cos, sin) of two consecutive pairs
        float a0 = x.v[4 * pr + 0], a1 = x.v[4 * pr + 1], b0 = x.v[4 * pr + 2], b1 = x.v[4 * pr + 3];
        x.v[4 * pr + 0] = rope_re(a0, a1, c2.x, c2.y);
        x.v[4 * pr + 1] = rope_im(a0, a1, c2.x, c2.y);
        x.v[4 * pr + 2] = rope_re(b0, b1, c2.z, c2.w);
        x.v[4 * pr + 3] = rope_im(b0, b1, c2.z, c2.w);
      }
    }
    if (which == 0 && g.q_scale != 0.f && g.q_scale != 1.f) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = mul_nc(x.v[e], g.q_scale);
    }
    TC* dst = reinterpret_cast<TC*>(which == 0 ? g.q : (which == 1 ? g.k : g.v));
    store8<TC>(dst + (((int64_t)s * g.heads + head) * g.seq_len + pos) * 64 + dh, x);
    return;
  }
  const int64_t off = (int64_t)row * g.ldc + col;
  const bool vec = full && (g.ldc % 4 == 0);
  if constexpr (EPI == EPI_RESID16) {
    // 16-bit residual stream: read, add in fp32 (same rounding as EPI_RESID), store rounded
    TC* C = reinterpret_cast<TC*>(g.C);
    const TC* R = reinterpret_cast<const TC*>(g.resid ? g.resid : g.C);
    const bool keep = !(g.rowkeep && !g.rowkeep[row]);
    const bool v16 = full && (g.ldc % 8 == 0);
    V8 c = v16 ? load8(R + off) : V8{};
    if (!v16)
      for (int e = 0; e < 8; ++e) c.v[e] = col + e < g.N ? to_f32(R[off + e]) : 0.f;
    V8 gt = g.gate ? (full ? load8(g.gate + col) : V8{}) : V8{{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}};
    if (g.gate && !full)
      for (int e = 0; e < 8; ++e) gt.v[e] = col + e < g.N ? g.gate[col + e] : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) x.v[e] = resid_add(c.v[e], gt.v[e], x.v[e], keep);
    if (v16) {
      store8<TC>(C + off, x);
    } else {
      for (int e = 0; e < 8; ++e)
        if (col + e < g.N) C[off + e] = from_f32<TC>(x.v[e]);
    }
    return;
  } else if constexpr (EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF_OP || EPI == EPI_STORE16) {
    if constexpr (EPI != EPI_STORE16) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        x.v[e] = EPI == EPI_GELU_ERF_OP ? gelu_erf(x.v[e])
                                        : (is16<TC>() ? gelu_tanh_fast(x.v[e]) : gelu_tanh(x.v[e]));
    }
    TC* C = reinterpret_cast<TC*>(g.C);
    if (full && g.ldc % 8 == 0) {
      store8<TC>(C + off, x);
    } else {
      for (int e = 0; e < 8; ++e)
        if (col + e < g.N) C[off + e] = from_f32<TC>(x.v[e]);
    }
    return;
  } else {
    float* C = reinterpret_cast<float*>(g.C);
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = silu(x.v[e]);
    } else if constexpr (EPI == EPI_GELU_ERF) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = gelu_erf(x.v[e]);
    } else if constexpr (EPI == EPI_RESID) {
      const bool keep = !(g.rowkeep && !g.rowkeep[row]);
      const float* R = reinterpret_cast<const float*>(g.resid ? g.resid : g.C);
      V8 c = vec ? (pre ? *pre : load8(R + off)) : V8{};
      if (!vec)
        for (int e = 0; e < 8; ++e) c.v[e] = col + e < g.N ? R[off + e] : 0.f;
      V8 gt = g.gate ? (full ? load8(g.gate + col) : V8{}) : V8{{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}};
      if (g.gate && !full)
        for (int e = 0; e < 8; ++e) gt.v[e] = col + e < g.N ? g.gate[col + e] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = resid_add(c.v[e], gt.v[e], x.v[e], keep);
    } else if constexpr (EPI == EPI_RESID_FILL) {
      const bool keep = !g.rowkeep || g.rowkeep[row];
      V8 c = vec ? load8(C + off) : V8{};
      if (!vec)
        for (int e = 0; e < 8; ++e) c.v[e] = col + e < g.N ? C[off + e] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) x.v[e] = keep ? c.v[e] + x.v[e] : 0.f;
    } else if constexpr (EPI == EPI_INPROJ) {
      const int64_t ao = (int64_t)row * g.ld_add + col;
      V8 a0 = load8(g.add + ao);
      V8 o0, o1;
#pragma unroll
      for (int e = 0; e < 8; ++e) o0.v[e] = x.v[e] + a0.v[e];
      store8<float>(C + off, o0);
      if (g.dual_rows) {
        V8 a1 = load8(g.add + ao + g.dual_rows * g.ld_add);
#pragma unroll
        for (int e = 0; e < 8; ++e) o1.v[e] = x.v[e] + a1.v[e];
        store8<float>(C + off + g.dual_rows * g.ldc, o1);
      }
      return;
    }
    if (vec) {
      store8<float>(C + off, x);
    } else {
      for (int e = 0; e < 8; ++e)
        if (col + e < g.N) C[off + e] = x.v[e];
    }
  }
}

// wait until at most n_stages * DPS + X of this wave's VMEM ops are outstanding (the n_stages
// youngest stages, plus X younger non-stage loads)
template <int DPS, int X = 0>
F5H_DEV void wait_stages(int n_stages) {
  switch (n_stages) {
    case 0: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(X) : "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DPS + X) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * DPS + X) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * DPS + X) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * DPS + X) : "memory"); break;
  }
}

// 16 bytes stored through a buffer descriptor: offsets past its extent are dropped by the hardware
// range check, so out-of-range rows need no branch around the store
// AUX: the cache-policy bits (kAuxWT: write-through, the in-launch hand-off's payload form)
template <int AUX = 0>
F5H_DEV void store16_rs(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}
template <typename TC, int AUX = 0>
F5H_DEV void store8_rs(__amdgpu_buffer_rsrc_t r, uint32_t elem, const V8& x) {
  if constexpr (is16<TC>()) {
    typedef typename Op16<TC>::v8 v8;
    const v8 b = {from_f32<TC>(x.v[0]), from_f32<TC>(x.v[1]), from_f32<TC>(x.v[2]), from_f32<TC>(x.v[3]),
                  from_f32<TC>(x.v[4]), from_f32<TC>(x.v[5]), from_f32<TC>(x.v[6]), from_f32<TC>(x.v[7])};
    store16_rs<AUX>(r, elem * 2u, __builtin_bit_cast(u32x4, b));
  } else {
    store16_rs<AUX>(r, elem * 4u, u32x4{__float_as_uint(x.v[0]), __float_as_uint(x.v[1]), __float_as_uint(x.v[2]),
                                   __float_as_uint(x.v[3])});
    store16_rs<AUX>(r, elem * 4u + 16u, u32x4{__float_as_uint(x.v[4]), __float_as_uint(x.v[5]), __float_as_uint(x.v[6]),
                                         __float_as_uint(x.v[7])});
  }
}

// ---- LayerNorm fold helpers (GemmArgs hs / ln_part_in; DESIGN.md §3 'LayerNorm fold')
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// DPP move inside each group of 8 consecutive lanes (the 8 lanes holding one 64-column row segment in the strip
// epilogue): quad_perm xor 1, quad_perm xor 2, row_half_mirror
template <int CTRL>
F5H_DEV float dpp8(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
F5H_DEV float sum8(float v) {
  v = add_nc(v, dpp8<0xB1>(v));
  v = add_nc(v, dpp8<0x4E>(v));
  return add_nc(v, dpp8<0x141>(v));
}
// The LayerNorm fold's row statistics from 64-column strip partials (mean m_p, M2 q_p): mean = the mean of the strip
// means, M2 = sum_p (q_p + 64 (m_p - mean)^2); a strip's term and the final rstd (LayerNorm eps 1e-6,
// modules.py:316,336), each rounding explicit so the per-chunk-row form (LNF 2) and the once-per-row form
// (ln_row_stats, LNF 3) agree bit for bit
F5H_DEV float ln_m2_term(float q, float mp, float mean) {
  const float d = sub_nc(mp, mean);
  return __builtin_fmaf(mul_nc(64.f, d), d, q);
}
F5H_DEV float ln_rstd(float m2, float inv_np, float eps) {
  return rsqrtf(__builtin_fmaf(m2, mul_nc(inv_np, 1.f / 64.f), eps));
}
// the 8-lane DPP sum of sum8 over lanes c = 0..7 holding a_c: ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7)) in
// every lane (xor 1, xor 2, then the half mirror: lane c adds lane 7 - c, whose pairs are the same sums)
F5H_DEV float sum8_order(const float (&a)[8]) {
  return add_nc(add_nc(add_nc(a[0], a[1]), add_nc(a[2], a[3])), add_nc(add_nc(a[4], a[5]), add_nc(a[6], a[7])));
}
// The once-per-row form of the fold consumer's statistics (LNF 3): thread t < BM of the block fetches row m0 + t's 16
// strip partials (8 x 16 B; issued whether or not the fold is on — a null descriptor reads zeros with no memory
// access — so the kernels' counted waits see a constant number of loads), and after the K loop combines them
// exactly as the per-chunk-row form does (lane c of the row's 8 held partials c and c + 8) into (mean, rstd):
// every strip holds 64 columns, so mean = the mean of the strip means, M2 = sum of the strips' M2 + 64 sum of
// (strip mean - mean)^2 (partials past ln_nparts weigh 0).
F5H_DEV void ln_row_fetch(const GemmArgs& g, int m0, int tid, int BM, u32x4 (&raw)[8]) {
  const bool on = g.ln_part_in != nullptr;
  const __amdgpu_buffer_rsrc_t st = rsrc_of(g.ln_part_in, on ? (uint64_t)g.M * g.ln_nparts * 8 : 0);
  const uint32_t base = tid < BM ? (uint32_t)(min(m0 + tid, g.M - 1) * g.ln_nparts * 8) : 0xFFFFFF00u;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    raw[e] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(st, base + 16 * e, 0, 0));
}
F5H_DEV void ln_row_stats(const GemmArgs& g, const u32x4 (&raw)[8], float* out) {
  const int np = g.ln_nparts;
  const float inv_np = 1.f / (float)np;
  auto mp = [&](int p) { return __uint_as_float(raw[p >> 1][(p & 1) * 2]); };
  auto qp = [&](int p) { return __uint_as_float(raw[p >> 1][(p & 1) * 2 + 1]); };
  float a[8], e[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float w0 = c < np ? 1.f : 0.f, w1 = c + 8 < np ? 1.f : 0.f;
    a[c] = add_nc(w0 * mp(c), w1 * mp(c + 8));
  }
  const float mean = mul_nc(sum8_order(a), inv_np);
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float w0 = c < np ? 1.f : 0.f, w1 = c + 8 < np ? 1.f : 0.f;
    e[c] = add_nc(w0 * ln_m2_term(qp(c), mp(c), mean), w1 * ln_m2_term(qp(c + 8), mp(c + 8), mean));
  }
  out[0] = mean;
  out[1] = ln_rstd(sum8_order(e), inv_np, g.ln_eps);
}

// Fast epilogue of one wave's sub-tile (whole-column tiles of the hot epilogues), per 16-row strip:
// accumulators -> the wave's LDS strip (fp32, EPAD-float rows; one ds_write_b128 per block, the swapped-operand
// layout holding four consecutive columns per lane) -> 8-column chunks of whole rows, so that every store
// instruction writes whole 128-B row segments (the register-only epilogue below stores 64-B row pieces, two
// instructions per segment: QKV +10-13 % and the residual GEMMs +5-8 % per launch at C4/C5, QKV +9 % at C2,
// profiles/r05_ab_c4_c5_epilogue.txt). A lane's
// column chunk is the same in every strip, so bias/gate/QKV head indices are loaded once, and the row
// data of strip i+1 (RoPE pairs, residual rows, row-mask bytes) is fetched before strip i stores.
// The strip loop has no control flow: bias presence is a template choice, per-lane choices (RoPE on
// this column, rows past M) are selects or the store descriptor's range check. Any branch or any
// arithmetic on a just-loaded value makes hipcc wait for that load, and on gfx9 every store issued
// before it counts in the same vmcnt: at C3 such waits made the 256x256 ping-pong epilogue 13-15 us per
// tile (profiles/r03_timeline_c3.txt). rbase/cbase: the sub-tile's first row/column.
// Shared by gemm_kernel and gemm_pp_kernel.
// PD: strips of row data fetched ahead (1: the next strip's; fetching every strip's residual up front in the 256x256
// ping-pong kernel measured equal at C4/C5, profiles/r05_ab_c4_c5_resid_prefetch.txt)
// LNF (LayerNorm fold): 0 none, 1 producer (EPI_RESID16: also hs and the row-strip statistics), 2 / 3 consumer
// (EPI_GELU_TANH / EPI_QKV: the normalisation applied to the accumulators; 2 combines each row's strip partials
// here, 3 reads the row's (mean, rstd) from ln_rows, which gemm_body filled from partials fetched before its K
// loop); see GemmArgs.
template <typename TC, int EPI, int MT, int NT, int WN, int EPAD, bool PREF, bool BIAS, int PM, int PT, int AUX = 0,
          int PD = 1, int LNF = 0>
F5H_DEV void epilogue_fast_t(const GemmArgs& g, const f32x4 (&acc)[MT][NT], float* Cs, int rbase, int cbase,
                             int lane, const V8 (&pre)[PM][PT], const float* ln_rows = nullptr) {
  constexpr bool LNCONS = LNF == 2 || LNF == 3;
  constexpr int CH = WN / 8;          // 8-column chunks per strip row
  constexpr int TPC = 16 * CH / 64;   // chunks per lane per strip
  static_assert(64 % CH == 0 && (16 * CH) % 64 == 0, "whole chunks per lane");
  static_assert(LNF == 0 || (WN == 64 && is16<TC>()), "the LayerNorm fold: 64-column wave strips, 16-bit operands");
  static_assert((LNF != 1 && LNF != 4) || EPI == EPI_RESID16, "fold producer: the 16-bit residual epilogue");
  static_assert(!LNCONS || EPI == EPI_GELU_TANH || EPI == EPI_QKV, "fold consumer: FFN1 or QKV");
  const int fr = lane & 15, q = lane >> 4;
  const int cc = lane % CH;
  const int col = cbase + cc * 8;
  V8 bias8 = V8{};
  if constexpr (BIAS) bias8 = load8(g.bias + col);
  // LayerNorm fold: producer's (1 + scale) of its columns, hs / statistics destinations, its 64-column strip; the
  // consumer's ln_u / ln_v of its columns and the partial-statistics source
  V8 lnA = V8{}, lnB = V8{};
  __amdgpu_buffer_rsrc_t ln_dst = rsrc_of(nullptr, 0), ln_st = rsrc_of(nullptr, 0);
  int ln_p = 0;
  const int ln_np = g.ln_nparts;
  if constexpr (LNF == 1 || LNF == 4) {
    if constexpr (LNF == 1) {
      lnA = load8(g.hs_scale + col);
#pragma unroll
      for (int e = 0; e < 8; ++e) lnA.v[e] = 1.f + lnA.v[e];
      ln_dst = rsrc_of(g.hs, (uint64_t)g.M * g.ldc * sizeof(TC));
    }
    ln_st = rsrc_of(g.ln_part, (uint64_t)g.M * ln_np * 8);
    ln_p = __builtin_amdgcn_readfirstlane(cbase >> 6);
  } else if constexpr (LNCONS) {
    if (g.ln_u) lnA = load8(g.ln_u + col);  // (RMSNorm form: u = v = 0, the gain is in W)
    if (g.ln_v) lnB = load8(g.ln_v + col);
    if constexpr (BIAS) {  // the bias joins v: one fused multiply-add pair per element below
#pragma unroll
      for (int e = 0; e < 8; ++e) lnB.v[e] += bias8.v[e];
    }
    if constexpr (LNF == 2) ln_st = rsrc_of(g.ln_part_in, (uint64_t)g.M * ln_np * 8);
  }
  const int lp0 = min(cc, ln_np - 1), lp1 = min(cc + 8, ln_np - 1);  // this lane's two partials (consumer)
  const float ln_w0 = cc < ln_np ? 1.f : 0.f, ln_w1 = cc + 8 < ln_np ? 1.f : 0.f;
  const float ln_inv_np = 1.f / (float)ln_np;
  V8 gate8 = V8{{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}};
  if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16)
    if (g.gate) gate8 = load8(g.gate + col);
  int which = 0, head = 0, dh = 0;
  bool rope_on = false;
  float qsc = 1.f;
  __amdgpu_buffer_rsrc_t dst;
  if constexpr (EPI == EPI_QKV) {
    // a wave's 64 columns are one head of one of q/k/v (cbase % 64 == 0): wave-uniform, so the
    // destination descriptor lives in scalar registers (a per-lane one costs a waterfall loop per store)
    static_assert(WN <= 64 && 64 % WN == 0, "a wave's columns lie in one head");
    const int inner = g.heads * 64;
    which = __builtin_amdgcn_readfirstlane(fdiv(cbase, inner));
    const int hc = col - which * inner;
    head = hc >> 6;
    dh = hc & 63;
    rope_on = which < 2 && head < g.rope_heads;
    qsc = (which == 0 && g.q_scale != 0.f) ? g.q_scale : 1.f;
    dst = rsrc_of(which == 0 ? g.q : (which == 1 ? g.k : g.v), (uint64_t)g.M * inner * sizeof(TC));
  } else {
    constexpr int OES = (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_INPROJ) ? 4 : (int)sizeof(TC);
    dst = rsrc_of(g.C, (uint64_t)(g.M + (EPI == EPI_INPROJ ? g.dual_rows : 0)) * g.ldc * OES);
  }
  // Loads only, raw bits, no arithmetic on their results here (see above): conversions happen at the
  // use, one strip later. Row indices are clamped instead of branched on (rows >= M are never stored).
  struct RowIn {
    u32x4 d0, d1;  // RoPE (cos, sin) of four pairs (QKV, fp32), the residual row chunk (RESID), the addend (INPROJ)
    u32x4 e0, e1;  // INPROJ: the second output row's addend
    uint32_t kb;   // RESID row-mask byte
    u32x2_t s0, s1;  // LayerNorm fold consumer: two (mean, M2) partials of the row
  };
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(g.rowkeep, g.rowkeep ? (uint64_t)g.M : 0);  // null: reads 0
  const bool masked = g.rowkeep != nullptr;
  // QKV: (sequence, position) of each of the lane's chunk rows, for the strip being fetched (pf) and the one being
  // stored (ps), advanced by 16 rows per strip (one division per chunk row for the whole epilogue, not two per
  // strip). Rows past M get positions too: the RoPE table index stays in range and their stores are dropped.
  int pf_sq[TPC], pf_pos[TPC], ps_sq[TPC], ps_pos[TPC];
  if constexpr (EPI == EPI_QKV) {
#pragma unroll
    for (int t = 0; t < TPC; ++t) {
      const int row0 = rbase + t * (64 / CH) + lane / CH;
      pf_sq[t] = ps_sq[t] = fdiv(row0, g.seq_len);
      pf_pos[t] = ps_pos[t] = row0 - pf_sq[t] * g.seq_len;
    }
  }
  auto advance = [&](int& sq, int& pos) {
    pos += 16;
    while (pos >= g.seq_len) {
      pos -= g.seq_len;
      ++sq;
    }
  };
  auto fetch = [&](int i, RowIn (&ri)[TPC]) {
#pragma unroll
    for (int t = 0; t < TPC; ++t) {
      const int rr = t * (64 / CH) + lane / CH;
      const int rowc = min(rbase + i * 16 + rr, g.M - 1);
      if constexpr (LNF == 2) {
        ri[t].s0 = __builtin_amdgcn_raw_buffer_load_b64(ln_st, (uint32_t)((rowc * ln_np + lp0) * 8), 0, 0);
        ri[t].s1 = __builtin_amdgcn_raw_buffer_load_b64(ln_st, (uint32_t)((rowc * ln_np + lp1) * 8), 0, 0);
      }
      if constexpr (EPI == EPI_QKV) {
        (void)rowc;
        const u32x4* p = reinterpret_cast<const u32x4*>(g.rope + pf_pos[t] * 32 + (dh >> 1));
        ri[t].d0 = p[0];
        ri[t].d1 = p[1];
        advance(pf_sq[t], pf_pos[t]);
      } else if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
        if constexpr (!PREF) {
          const u32x4* p = reinterpret_cast<const u32x4*>(reinterpret_cast<const ResT<TC, EPI>*>(
                                                              g.resid ? g.resid : g.C) + (int64_t)rowc * g.ldc + col);
          ri[t].d0 = p[0];
          if constexpr (sizeof(ResT<TC, EPI>) == 4) ri[t].d1 = p[1];  // fp32 rows: 32 B
        }
        ri[t].kb = __builtin_amdgcn_raw_buffer_load_b8(rk, (uint32_t)rowc, 0, 0);
      } else if constexpr (EPI == EPI_INPROJ) {
        const u32x4* p = reinterpret_cast<const u32x4*>(g.add + (int64_t)rowc * g.ld_add + col);
        ri[t].d0 = p[0];
        ri[t].d1 = p[1];
        const u32x4* p2 = reinterpret_cast<const u32x4*>(g.add + (int64_t)(rowc + g.dual_rows) * g.ld_add + col);
        ri[t].e0 = p2[0];  // (rows [M, M + dual_rows) of the addend; the first rows again when dual_rows = 0)
        ri[t].e1 = p2[1];
      }
    }
  };
  // the raw row data as 8 fp32 values
  auto as_v8 = [&](const RowIn& ri) -> V8 {
    if constexpr (EPI == EPI_RESID16 && is16<TC>()) {
      typedef typename Op16<TC>::v8 v8;
      const v8 h = __builtin_bit_cast(v8, ri.d0);
      return V8{{to_f32(h[0]), to_f32(h[1]), to_f32(h[2]), to_f32(h[3]), to_f32(h[4]), to_f32(h[5]), to_f32(h[6]),
                 to_f32(h[7])}};
    } else {
      return V8{{__uint_as_float(ri.d0[0]), __uint_as_float(ri.d0[1]), __uint_as_float(ri.d0[2]),
                 __uint_as_float(ri.d0[3]), __uint_as_float(ri.d1[0]), __uint_as_float(ri.d1[1]),
                 __uint_as_float(ri.d1[2]), __uint_as_float(ri.d1[3])}};
    }
  };
  constexpr int RB = PD + 1;  // row-data ring
  RowIn rbuf[RB][TPC];
  static_for<0, (PD < MT ? PD : MT)>([&](auto F) { fetch(decltype(F)::value, rbuf[decltype(F)::value % RB]); });
  static_for<0, MT>([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i + PD < MT) fetch(i + PD, rbuf[(i + PD) % RB]);
#pragma unroll
    for (int j = 0; j < NT; ++j)
      *reinterpret_cast<f32x4*>(Cs + fr * EPAD + j * 16 + 4 * q) = acc[i][j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int t = 0; t < TPC; ++t) {
      const int rr = t * (64 / CH) + lane / CH;
      const int row = rbase + i * 16 + rr;  // rows >= M: dropped by the store descriptor
      const float* src = Cs + rr * EPAD + cc * 8;
      const float4 a0 = *reinterpret_cast<const float4*>(src), a1 = *reinterpret_cast<const float4*>(src + 4);
      V8 x{{a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w}};
      const RowIn& ri = rbuf[i % RB][t];
      if constexpr (LNCONS) {
        float m, rstd;
        if constexpr (LNF == 3) {
          const float2 ms = *reinterpret_cast<const float2*>(ln_rows + 2 * (i * 16 + rr));
          m = ms.x;
          rstd = ms.y;
        } else {
        // the row's statistics from its strips' partials (two per lane, w0 / w1 = 1 where the partial exists):
        // every strip holds 64 columns, so mean = the mean of the strip means and M2 = sum of the strips' M2 +
        // 64 sum of (strip mean - mean)^2 (two sums over the row's 8 lanes, no division)
        // (every rounding written out: ln_row_stats below gives the same bits from one thread)
        const float m0 = __uint_as_float(ri.s0.x), m1 = __uint_as_float(ri.s1.x);
        m = mul_nc(sum8(add_nc(ln_w0 * m0, ln_w1 * m1)), ln_inv_np);
        const float e0 = ln_m2_term(__uint_as_float(ri.s0.y), m0, m), e1 = ln_m2_term(__uint_as_float(ri.s1.y), m1, m);
        rstd = ln_rstd(sum8(add_nc(ln_w0 * e0, ln_w1 * e1)), ln_inv_np, g.ln_eps);
        }
        // x = rstd (x - m u) + (v + bias), as packed fp32 FMAs on column pairs
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 t = f32x2{x.v[e], x.v[e + 1]} - f32x2{m, m} * f32x2{lnA.v[e], lnA.v[e + 1]};
          const f32x2 y = f32x2{rstd, rstd} * t + f32x2{lnB.v[e], lnB.v[e + 1]};
          x.v[e] = y.x;
          x.v[e + 1] = y.y;
        }
      }
      if constexpr (BIAS && !LNCONS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x.v[e] = add_nc(x.v[e], bias8.v[e]);
      }
      if constexpr (EPI == EPI_QKV) {
        const V8 cs = as_v8(ri);
        // interleaved pairs (a, b) -> (a c - b s, b c + a s) as packed products and one packed add (each
        // element rounded as rope_re / rope_im round it), then the q scale on pairs
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float c = cs.v[2 * p], sn = cs.v[2 * p + 1];
          const f32x2 ab = {x.v[2 * p], x.v[2 * p + 1]};
          f32x2 r;
          {
#pragma clang fp contract(off)
            const f32x2 pc = ab * c, ps = f32x2{ab.y, ab.x} * sn;
            r = pc + f32x2{-ps.x, ps.y};
            r = (rope_on ? r : ab) * qsc;  // exact for qsc = 1 (k, v columns)
          }
          x.v[2 * p] = r.x;
          x.v[2 * p + 1] = r.y;
        }
        (void)row;
        store8_rs<TC, AUX>(dst, (uint32_t)(((ps_sq[t] * g.heads + head) * g.seq_len + ps_pos[t]) * 64 + dh), x);
        advance(ps_sq[t], ps_pos[t]);
      } else if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
        V8 c;
        if constexpr (PREF)
          c = pre[PREF ? i : 0][PREF ? t : 0];
        else
          c = as_v8(ri);
        const bool keep = !masked || ri.kb;
        V8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = resid_add(c.v[e], gate8.v[e], x.v[e], keep);
        store8_rs<ResT<TC, EPI>, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), o);
        if constexpr (LNF == 1 || LNF == 4) {
          // the stored (rounded) h values: hs = h (1 + scale) for the consumer, and this 64-column strip's
          // (mean, M2) of h (two passes over the row's 8 lanes). RMSNorm form (LNF 4): no hs, and the strip's
          // "mean" is 0, so its M2 is the sum of squares the consumer needs
          V8 hr, hv;
          f32x2 s2 = {0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 h2 = {to_f32(from_f32<TC>(o.v[e])), to_f32(from_f32<TC>(o.v[e + 1]))};
            hr.v[e] = h2.x;
            hr.v[e + 1] = h2.y;
            if constexpr (LNF == 1) {
              const f32x2 v2 = h2 * f32x2{lnA.v[e], lnA.v[e + 1]};
              hv.v[e] = v2.x;
              hv.v[e + 1] = v2.y;
              s2 += h2;
            }
          }
          if constexpr (LNF == 1) store8_rs<TC, AUX>(ln_dst, (uint32_t)((int64_t)row * g.ldc + col), hv);
          const float mean = LNF == 4 ? 0.f : sum8(s2.x + s2.y) * (1.f / 64.f);
          f32x2 q2 = {0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 dv = f32x2{hr.v[e], hr.v[e + 1]} - f32x2{mean, mean};
            q2 += dv * dv;
          }
          const float m2 = sum8(q2.x + q2.y);
          // the row's 8 lanes store the same 8 bytes (no branch); rows >= M fall outside the descriptor
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{__float_as_uint(mean), __float_as_uint(m2)}, ln_st,
                                                (uint32_t)((row * ln_np + ln_p) * 8), 0, AUX);
        }
      } else if constexpr (EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF_OP) {
        if constexpr (EPI == EPI_GELU_TANH && is16<TC>()) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 gv = gelu_tanh_fast2(f32x2{x.v[e], x.v[e + 1]});
            x.v[e] = gv.x;
            x.v[e + 1] = gv.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) x.v[e] = EPI == EPI_GELU_ERF_OP ? gelu_erf(x.v[e]) : gelu_tanh(x.v[e]);
        }
        store8_rs<TC, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      } else if constexpr (EPI == EPI_STORE16) {
        store8_rs<TC, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      } else if constexpr (EPI == EPI_INPROJ) {
        // x.W_x^T + P for this branch's row, and for the other branch's row (same x, dit.py:162)
        V8 o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o0.v[e] = x.v[e] + __uint_as_float(ri.d0[e]);
          o0.v[e + 4] = x.v[e + 4] + __uint_as_float(ri.d1[e]);
          o1.v[e] = x.v[e] + __uint_as_float(ri.e0[e]);
          o1.v[e + 4] = x.v[e + 4] + __uint_as_float(ri.e1[e]);
        }
        // rows >= M would land in the second block: drop them explicitly (an offset past the descriptor's
        // extent, which fast_epi_ok keeps below 0xF0000000 bytes; no 32-bit wrap for either 16-B half)
        constexpr uint32_t kPast = 0xF0000000u / 4;
        store8_rs<float, AUX>(dst, row < g.M ? (uint32_t)((int64_t)row * g.ldc + col) : kPast, o0);
        if (g.dual_rows)
          store8_rs<float, AUX>(dst, row < g.M ? (uint32_t)((int64_t)(row + g.dual_rows) * g.ldc + col) : kPast, o1);
      } else {  // EPI_STORE
        store8_rs<float, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  });
}
template <typename TC, int EPI, int MT, int NT, int WN, int EPAD, bool PREF, int AUX = 0, int PD = 1, int PM, int PT>
F5H_DEV void epilogue_fast(const GemmArgs& g, const f32x4 (&acc)[MT][NT], float* Cs, int rbase, int cbase,
                           int lane, const V8 (&pre)[PM][PT], const float* ln_rows = nullptr) {
  // LayerNorm fold forms (GemmArgs hs / ln_part_in: 16-bit, 64-column wave strips; bias always present there)
  if constexpr (WN == 64 && is16<TC>() && AUX == 0) {
    if constexpr (EPI == EPI_RESID16) {
      if (g.ln_part && g.ln_rms) {
        if (g.bias)
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, true, PM, PT, AUX, PD, 4>(g, acc, Cs, rbase, cbase, lane, pre);
        else
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, false, PM, PT, AUX, PD, 4>(g, acc, Cs, rbase, cbase, lane, pre);
        return;
      }
      if (g.ln_part) {
        if (g.bias)
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, true, PM, PT, AUX, PD, 1>(g, acc, Cs, rbase, cbase, lane, pre);
        else
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, false, PM, PT, AUX, PD, 1>(g, acc, Cs, rbase, cbase, lane, pre);
        return;
      }
    } else if constexpr (EPI == EPI_GELU_TANH || EPI == EPI_QKV) {
      if (g.ln_part_in && ln_rows) {
        if (g.bias)
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, true, PM, PT, AUX, PD, 3>(g, acc, Cs, rbase, cbase, lane, pre,
                                                                                   ln_rows);
        else
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, false, PM, PT, AUX, PD, 3>(g, acc, Cs, rbase, cbase, lane, pre,
                                                                                    ln_rows);
        return;
      }
      if (g.ln_part_in) {
        if (g.bias)
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, true, PM, PT, AUX, PD, 2>(g, acc, Cs, rbase, cbase, lane, pre);
        else
          epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, false, PM, PT, AUX, PD, 2>(g, acc, Cs, rbase, cbase, lane, pre);
        return;
      }
    }
  }
  if (g.bias)
    epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, true, PM, PT, AUX, PD>(g, acc, Cs, rbase, cbase, lane, pre);
  else
    epilogue_fast_t<TC, EPI, MT, NT, WN, EPAD, PREF, false, PM, PT, AUX, PD>(g, acc, Cs, rbase, cbase, lane, pre);
}

// Direct epilogue (round 5; the persistent kernel, whose LDS holds the operand ring only): the MFMAs run with swapped operands (W fragment as A, activation fragment as B),
// so accumulator acc[i][j] holds C^T: lane l has row 16i + (l & 15) and the FOUR CONSECUTIVE columns
// 16j + 4(l >> 4) + r (r = 0..3). One v_permlane16_swap per dword between blocks j and j+1 (the odd 16-lane
// rows of block j trade with the even rows of block j+1) leaves every lane with EIGHT consecutive columns of
// its row: lanes of row q = l >> 4 hold block j + (q & 1), columns 8 (q >> 1) .. +7 (cdna_hip_programming.md
// T21, with the 16-lane swap). The epilogue then works on registers only: no accumulator round trip through
// LDS (the fast epilogue before it wrote every fp32 accumulator to an LDS strip with 4-byte stores and read it
// back by rows: 256 KB per 256x256 tile, ~1.6 us of LDS write bandwidth alone), no per-strip wave barriers.
// Per element the arithmetic is the same functions as before (bitwise identical results). The row data of
// strip i+1 (RoPE pairs, residual chunks, row-mask bytes, addends) is fetched before strip i stores.
// pre: PREF residual chunks prefetched before the K loop, [MT][NT/2].
template <typename TC, int EPI, int MT, int NT, bool PREF, bool BIAS, int PM, int PT, int AUX = 0>
F5H_DEV void epilogue_direct_t(const GemmArgs& g, const f32x4 (&acc)[MT][NT], int rbase, int cbase, int lane,
                               const V8 (&pre)[PM][PT]) {
  static_assert(NT % 2 == 0, "column blocks in pairs");
  constexpr int NP = NT / 2;
  const int fr = lane & 15, q = lane >> 4;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);  // the lane's 8-column chunk within a pair of 16-column blocks
  V8 bias8[NP], gate8[NP];
  int colp[NP];
#pragma unroll
  for (int jp = 0; jp < NP; ++jp) {
    colp[jp] = cbase + 32 * jp + coff;
    bias8[jp] = V8{};
    if constexpr (BIAS) bias8[jp] = load8(g.bias + colp[jp]);
    gate8[jp] = V8{{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}};
    if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16)
      if (g.gate) gate8[jp] = load8(g.gate + colp[jp]);
  }
  int which = 0, head = 0, dh[NP];
  bool rope_on = false;
  float qsc = 1.f;
  __amdgpu_buffer_rsrc_t dst;
  if constexpr (EPI == EPI_QKV) {
    // a wave's columns lie in one head of one of q/k/v (cbase % 32 == 0, <= 64 columns from a head start):
    // wave-uniform, so the destination descriptor lives in scalar registers
    const int inner = g.heads * 64;
    which = __builtin_amdgcn_readfirstlane(fdiv(cbase, inner));
    head = __builtin_amdgcn_readfirstlane((cbase - which * inner) >> 6);
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) dh[jp] = (colp[jp] - which * inner) & 63;
    rope_on = which < 2 && head < g.rope_heads;
    qsc = (which == 0 && g.q_scale != 0.f) ? g.q_scale : 1.f;
    dst = rsrc_of(which == 0 ? g.q : (which == 1 ? g.k : g.v), (uint64_t)g.M * inner * sizeof(TC));
  } else {
    constexpr int OES = (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_INPROJ) ? 4 : (int)sizeof(TC);
    dst = rsrc_of(g.C, (uint64_t)(g.M + (EPI == EPI_INPROJ ? g.dual_rows : 0)) * g.ldc * OES);
  }
  // Loads only, raw bits, no arithmetic on their results here: conversions happen at the use, one strip
  // later (a branch or arithmetic on a just-loaded value makes hipcc wait for it, behind every older store).
  // Row indices are clamped instead of branched on (rows >= M are never stored).
  struct RowIn {
    u32x4 d0, d1;  // RoPE (cos, sin) of four pairs (QKV), the residual chunk (RESID), the addend (INPROJ)
    u32x4 e0, e1;  // INPROJ: the second output row's addend
  };
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(g.rowkeep, g.rowkeep ? (uint64_t)g.M : 0);  // null: reads 0
  const bool masked = g.rowkeep != nullptr;
  // QKV: (sequence, position) of the lane's row for the strip being fetched (pf) and the one being stored (ps),
  // advanced by 16 rows per strip. Rows past M get positions too: the RoPE index stays in range, stores drop.
  int pf_sq = 0, pf_pos = 0, ps_sq = 0, ps_pos = 0;
  if constexpr (EPI == EPI_QKV) {
    const int row0 = rbase + fr;
    pf_sq = ps_sq = fdiv(row0, g.seq_len);
    pf_pos = ps_pos = row0 - pf_sq * g.seq_len;
  }
  auto advance = [&](int& sq, int& pos) {
    pos += 16;
    while (pos >= g.seq_len) {
      pos -= g.seq_len;
      ++sq;
    }
  };
  uint32_t kb[2] = {0u, 0u};
  auto fetch = [&](int i, RowIn (&ri)[NP], uint32_t& kbi) {
    const int rowc = min(rbase + i * 16 + fr, g.M - 1);
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) {
      if constexpr (EPI == EPI_QKV) {
        const u32x4* p = reinterpret_cast<const u32x4*>(g.rope + pf_pos * 32 + (dh[jp] >> 1));
        ri[jp].d0 = p[0];
        ri[jp].d1 = p[1];
      } else if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
        if constexpr (!PREF) {
          const u32x4* p = reinterpret_cast<const u32x4*>(reinterpret_cast<const ResT<TC, EPI>*>(
                                                              g.resid ? g.resid : g.C) + (int64_t)rowc * g.ldc + colp[jp]);
          ri[jp].d0 = p[0];
          if constexpr (sizeof(ResT<TC, EPI>) == 4) ri[jp].d1 = p[1];  // fp32 rows: 32 B
        }
      } else if constexpr (EPI == EPI_INPROJ) {
        const u32x4* p = reinterpret_cast<const u32x4*>(g.add + (int64_t)rowc * g.ld_add + colp[jp]);
        ri[jp].d0 = p[0];
        ri[jp].d1 = p[1];
        const u32x4* p2 = reinterpret_cast<const u32x4*>(g.add + (int64_t)(rowc + g.dual_rows) * g.ld_add + colp[jp]);
        ri[jp].e0 = p2[0];  // (rows [M, M + dual_rows) of the addend; the first rows again when dual_rows = 0)
        ri[jp].e1 = p2[1];
      }
    }
    if constexpr (EPI == EPI_QKV) advance(pf_sq, pf_pos);
    if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) kbi = __builtin_amdgcn_raw_buffer_load_b8(rk, (uint32_t)rowc, 0, 0);
  };
  // the raw row data as 8 fp32 values
  auto as_v8 = [&](const RowIn& ri) -> V8 {
    if constexpr (EPI == EPI_RESID16 && is16<TC>()) {
      typedef typename Op16<TC>::v8 v8;
      const v8 h = __builtin_bit_cast(v8, ri.d0);
      return V8{{to_f32(h[0]), to_f32(h[1]), to_f32(h[2]), to_f32(h[3]), to_f32(h[4]), to_f32(h[5]), to_f32(h[6]),
                 to_f32(h[7])}};
    } else {
      return V8{{__uint_as_float(ri.d0[0]), __uint_as_float(ri.d0[1]), __uint_as_float(ri.d0[2]),
                 __uint_as_float(ri.d0[3]), __uint_as_float(ri.d1[0]), __uint_as_float(ri.d1[1]),
                 __uint_as_float(ri.d1[2]), __uint_as_float(ri.d1[3])}};
    }
  };
  RowIn rbuf[2][NP];
  fetch(0, rbuf[0], kb[0]);
  static_for<0, MT>([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i + 1 < MT) fetch(i + 1, rbuf[(i + 1) & 1], kb[(i + 1) & 1]);
    const int row = rbase + i * 16 + fr;  // rows >= M: dropped by the store descriptor
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) {
      // blocks 2jp and 2jp+1 -> this lane's 8 consecutive columns colp[jp] .. +7
      V8 x;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                         __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
        x.v[r] = __uint_as_float(sw[0]);
        x.v[r + 4] = __uint_as_float(sw[1]);
      }
      const int col = colp[jp];
      if constexpr (BIAS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x.v[e] = add_nc(x.v[e], bias8[jp].v[e]);
      }
      const RowIn& ri = rbuf[i & 1][jp];
      if constexpr (EPI == EPI_QKV) {
        const V8 cs = as_v8(ri);
        // interleaved pairs (a, b) -> (a c - b s, b c + a s) as packed products and one packed add (each
        // element rounded as rope_re / rope_im round it), then the q scale on pairs
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float c = cs.v[2 * p], sn = cs.v[2 * p + 1];
          const f32x2 ab = {x.v[2 * p], x.v[2 * p + 1]};
          f32x2 rr;
          {
#pragma clang fp contract(off)
            const f32x2 pc = ab * c, ps = f32x2{ab.y, ab.x} * sn;
            rr = pc + f32x2{-ps.x, ps.y};
            rr = (rope_on ? rr : ab) * qsc;  // exact for qsc = 1 (k, v columns)
          }
          x.v[2 * p] = rr.x;
          x.v[2 * p + 1] = rr.y;
        }
        (void)row;
        store8_rs<TC, AUX>(dst, (uint32_t)(((ps_sq * g.heads + head) * g.seq_len + ps_pos) * 64 + dh[jp]), x);
      } else if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
        V8 c;
        if constexpr (PREF)
          c = pre[PREF ? i : 0][PREF ? jp : 0];
        else
          c = as_v8(ri);
        const bool keep = !masked || kb[i & 1];
        V8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = resid_add(c.v[e], gate8[jp].v[e], x.v[e], keep);
        store8_rs<ResT<TC, EPI>, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), o);
      } else if constexpr (EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF_OP) {
        if constexpr (EPI == EPI_GELU_TANH && is16<TC>()) {
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const f32x2 gv = gelu_tanh_fast2(f32x2{x.v[e], x.v[e + 1]});
            x.v[e] = gv.x;
            x.v[e + 1] = gv.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) x.v[e] = EPI == EPI_GELU_ERF_OP ? gelu_erf(x.v[e]) : gelu_tanh(x.v[e]);
        }
        store8_rs<TC, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      } else if constexpr (EPI == EPI_STORE16) {
        store8_rs<TC, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      } else if constexpr (EPI == EPI_INPROJ) {
        // x.W_x^T + P for this branch's row, and for the other branch's row (same x, dit.py:162)
        V8 o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o0.v[e] = x.v[e] + __uint_as_float(ri.d0[e]);
          o0.v[e + 4] = x.v[e + 4] + __uint_as_float(ri.d1[e]);
          o1.v[e] = x.v[e] + __uint_as_float(ri.e0[e]);
          o1.v[e + 4] = x.v[e + 4] + __uint_as_float(ri.e1[e]);
        }
        // rows >= M would land in the second block: drop them explicitly (an offset past the descriptor's
        // extent, which fast_epi_ok keeps below 0xF0000000 bytes; no 32-bit wrap for either 16-B half)
        constexpr uint32_t kPast = 0xF0000000u / 4;
        store8_rs<float, AUX>(dst, row < g.M ? (uint32_t)((int64_t)row * g.ldc + col) : kPast, o0);
        if (g.dual_rows)
          store8_rs<float, AUX>(dst, row < g.M ? (uint32_t)((int64_t)(row + g.dual_rows) * g.ldc + col) : kPast, o1);
      } else {  // EPI_STORE
        store8_rs<float, AUX>(dst, (uint32_t)((int64_t)row * g.ldc + col), x);
      }
    }
    if constexpr (EPI == EPI_QKV) advance(ps_sq, ps_pos);
  });
}
template <typename TC, int EPI, int MT, int NT, bool PREF, int AUX = 0, int PM, int PT>
F5H_DEV void epilogue_direct(const GemmArgs& g, const f32x4 (&acc)[MT][NT], int rbase, int cbase, int lane,
                             const V8 (&pre)[PM][PT]) {
  if (g.bias)
    epilogue_direct_t<TC, EPI, MT, NT, PREF, true, PM, PT, AUX>(g, acc, rbase, cbase, lane, pre);
  else
    epilogue_direct_t<TC, EPI, MT, NT, PREF, false, PM, PT, AUX>(g, acc, rbase, cbase, lane, pre);
}


// FAST: the launcher guarantees whole-column tiles (N % BN == 0, ldc % 8 == 0) for the hot
// epilogues, so the epilogue is compiled without per-element column guards (see below).
// Launch bounds: two 4-wave blocks per CU (2 waves per SIMD) must fit the register file, i.e. <= 256
// VGPR+AGPR per lane. With a minimum of 1 wave per SIMD the compiler gave the 192x128 tile 116 VGPR
// + 144 AGPR = 260: one block per CU, so the C2 QKV GEMM (480 tiles) ran as two rounds on 256 CUs
// (tools/timeline_c2.py: second half of the grid entering 24 us after the first). Declaring 2 waves
// per SIMD it fits in 212 VGPR, no spill.
// The block body of gemm_kernel: block b of nwg (XCD-remapped below) computes one BM x BN tile in the LDS
// image `lds`. PUB (the in-launch phase chain, chain.hip): stores are write-through and the tile's row groups are
// published to dep.pub; a non-null dep.wait makes the block wait for its row groups' producers before its
// first operand load; blocks past the last tile (the chain pads each phase to whole XCD rounds) do nothing.
template <typename TC, int EPI, int BM, int BN, int WGM, int WGN, int NS, bool FAST, int KB, bool PUB = false,
          bool CHAIN = false>
F5H_DEV void gemm_body(const GemmArgs& g, const int b, const int nwg, uint4* lds, const ChainDep& dep) {
  const ProbeT probe_t = probe_enter(g.probe);
  typedef GemmCfg<BM, BN, WGM, WGN, NS, KB> C;
  constexpr int E = elems16<TC>();
  constexpr int CPR = C::CPR, SLABS = KB / 64;
  constexpr int BKE = CPR * E;
  constexpr int NW = C::NW, WM = C::WM, WN = C::WN, MT = C::MT, NT = C::NT;
  constexpr int AR = BM * CPR / C::THREADS, BR = BN * CPR / C::THREADS;  // DMA rounds per stage
  constexpr int DPS = AR + BR;                                            // DMA instructions per stage per wave
  static_assert(NS >= 2 && NS <= 6 && (NS - 1) * DPS <= 63, "LDS stages");  // NS-1 stages in flight
  typedef typename Slab<TC>::frag frag;
  auto swz = [](int row, int chunk) { return KB == 128 ? swz128g(row, chunk) : swz64(row, chunk); };

  constexpr int stage_u4 = C::stage_bytes / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int ntn = (g.N + BN - 1) / BN;
  // XCD-aware remap (cdna_hip_programming.md T1, bijective form): blocks b and b+8 share an
  // XCD, so give each XCD a contiguous run of n-fastest tiles -> its L2 holds whole A panels
  const int xq = nwg >> 3, xr = nwg & 7, xcd = b & 7;
  const int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (b >> 3);
  if constexpr (CHAIN) {
    if (bid >= ((g.M + BM - 1) / BM) * ntn) return;
  }
  // with the pad skip, row tiles of padding cluster by sequence: spread the m-rows over the XCDs
  const int mrow = g.live_len ? spread8(bid / ntn, (g.M + BM - 1) / BM) : bid / ntn;
  const int m0 = mrow * BM, n0 = (bid % ntn) * BN;
  if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
    if (!tile_live(g, m0, BM)) {  // every row padding: nothing to add (C2's B = 1 never passes live_len)
      probe_exit(g.probe, probe_t);
      return;
    }
  }
  const TC* A = reinterpret_cast<const TC*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);

  // LDS-DMA by buffer_load ... lds against per-block buffers (the block's A rows and W rows): a lane's byte
  // offset in its panel is fixed across K-steps (voffset; the swizzle goes on the SOURCE chunk so that the
  // wave-uniform LDS base + lane*16 lands on the swz128 image), the K-step's a scalar (soffset) and the LDS
  // destination a scalar (M0), so a stage costs no vector instructions. Rows past M (N) are outside the
  // buffer and read as zero; they feed only unstored outputs.
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  constexpr int ESZ = (int)sizeof(TC);
  const uint32_t abytes = (uint32_t)(min(BM, g.M - m0) * g.lda * ESZ);
  const uint32_t wbytes = (uint32_t)(min(BN, g.N - n0) * g.ldw * ESZ);
  uint32_t aoff[AR], boff[BR];
  static_for<0, AR>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const int p = (i * NW + wid) * 64 + lane, row = p / CPR, slot = p % CPR;
    aoff[i] = (uint32_t)((row * g.lda + swz(row, slot) * E) * ESZ);
  });
  static_for<0, BR>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const int p = (i * NW + wid) * 64 + lane, row = p / CPR, slot = p % CPR;
    boff[i] = (uint32_t)((row * g.ldw + swz(row, slot) * E) * ESZ);
  });
  // A columns [k_split, K) come from the second panel A2 (cat(x, skip) of UNetT, unett.py:288-297):
  // a stage never straddles k_split (a multiple of the stage width)
  const TC* A2 = reinterpret_cast<const TC*>(g.A2);
  const __amdgpu_buffer_rsrc_t wrs =
      rsrc_of(W + (int64_t)n0 * g.ldw, wbytes);
  auto stage_a = [&](int buf, int k0) {
    uint4* As = lds + buf * stage_u4;
    const bool second = A2 && k0 >= g.k_split;
    const TC* Ab = second ? A2 : A;
    const int ka = second ? k0 - g.k_split : k0;
    const __amdgpu_buffer_rsrc_t ars =
        rsrc_of(Ab + (int64_t)m0 * g.lda, abytes);
    static_for<0, AR>([&](auto I) {
      constexpr int i = decltype(I)::value;
      dma16(ars, (LDS_PTR(void))(As + (i * NW + wid_s) * 64), aoff[i], ka * ESZ);
    });
  };
  auto stage_w = [&](int buf, int k0) {
    uint4* Bs = lds + buf * stage_u4 + BM * CPR;
    static_for<0, BR>([&](auto I) {
      constexpr int i = decltype(I)::value;
      dma16(wrs, (LDS_PTR(void))(Bs + (i * NW + wid_s) * 64), boff[i], k0 * ESZ);
    });
  };
  auto stage = [&](int buf, int k0) {
    stage_a(buf, k0);
    stage_w(buf, k0);
  };

  // Fragment reads are inline-asm ds_read_b128 so that hipcc does not put a vmcnt(0) (for the
  // LDS-DMA still in flight into the OTHER stages) in front of them; their completion is waited
  // for by hand (lgkmcnt(0) + sched_barrier, cdna_hip_programming.md §5.7 form iii).
  // Row r of a fragment has r & 15 == lane & 15 (swz128 reads row bits 1..3), so the swizzled
  // chunk depends only on the lane:
  // per slab one base address per lane, the 16-row tiles at immediate offsets i*2048.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  const int fr = lane & 15, q = lane >> 4;
  uint32_t abase[SLABS], bbase[SLABS];
#pragma unroll
  for (int s = 0; s < SLABS; ++s) {
    abase[s] = lds0 + (wm * WM + fr) * KB + swz(fr, s * 4 + q) * 16;
    bbase[s] = lds0 + BM * KB + (wn * WN + fr) * KB + swz(fr, s * 4 + q) * 16;
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BKE;
  if constexpr (CHAIN) {
    // phase chain: the weight panels of the first stages (no producer in the launch) are in flight while the
    // block waits for its rows; the activation panels follow the acquire. Issue order W0 .. W(NS-2), A0 ..
    // A(NS-2): the first wait below counts activation pieces only.
    for (int p = 0; p < NS - 1 && p < nk; ++p) stage_w(p, p * BKE);
    chain_wait(dep, g.M, m0, BM);
    for (int p = 0; p < NS - 1 && p < nk; ++p) stage_a(p, p * BKE);
  } else {
    for (int p = 0; p < NS - 1 && p < nk; ++p) stage(p, p * BKE);
  }
  asm volatile("" ::: "memory");  // the residual loads below stay behind the stage DMA
  // EPI_RESID: the residual rows this lane's epilogue reads are fetched right behind the first
  // operand stages (so they do not delay stage 0: the first wait leaves them in flight, the second
  // retires them), and the epilogue's read-modify-write does not expose a dependent HBM/MALL round
  // trip. Register budget: small tiles only.
  // (the strip epilogue's layout: chunk t of strip i is row 16i + (64t + lane) / CH_, 8-column chunk (64t + lane) % CH_)
  constexpr int CH_ = WN / 8, TPS = 16 * CH_ / 64;
  constexpr bool PREF = (EPI == EPI_RESID || EPI == EPI_RESID16) && is16<TC>() && (16 * CH_) % 64 == 0 &&
                        MT * TPS * 8 <= 32;
  V8 pre[PREF ? MT : 1][PREF ? TPS : 1];
  if constexpr (PREF) {
    const ResT<TC, EPI>* Cp = reinterpret_cast<const ResT<TC, EPI>*>(g.resid ? g.resid : g.C);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int t = 0; t < TPS; ++t) {
        const int idx = t * 64 + lane, rr = idx / CH_, cc = idx % CH_;
        const int row = m0 + wm * WM + i * 16 + rr, col = n0 + wn * WN + cc * 8;
        const bool ok = row < g.M && col + 8 <= g.N && g.ldc % 4 == 0;
        // unconditional (a select on the address, no branch): the loads issue back to back
        // (a branch per load made hipcc wait for each one in turn); unused when !ok
        pre[i][t] = load8(Cp + (ok ? (int64_t)row * g.ldc + col : 0));
      }
  }

  // LayerNorm fold consumer (QKV / FFN1 with GemmArgs ln_part_in): thread t < BM fetches the strip partials of the
  // block's row t (16 x 8 B) behind the first stages, and combines them after the K loop into the row's (mean,
  // rstd) in LDS, once per row (the strip epilogue's LNF 2 form combines them per chunk row, 8 lanes per row and
  // again in every column tile's waves). Issued whether or not the fold is on (a null descriptor reads zeros with
  // no memory access), so the first stage wait's count is a constant.
  constexpr bool LNC = (EPI == EPI_QKV || EPI == EPI_GELU_TANH) && is16<TC>() && WN == 64 && FAST && NT % 2 == 0 &&
                       !CHAIN && !PUB && BM <= C::THREADS;
  u32x4 lnraw[LNC ? 8 : 1];
  if constexpr (LNC) ln_row_fetch(g, m0, tid, BM, lnraw);
  constexpr int NPRE = PREF ? MT * TPS : (LNC ? 8 : 0);  // loads issued behind the first stages
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed for THIS wave once at most the younger in-flight stages remain;
    // the barrier then publishes every wave's part of it
    if (kt == 0) {
      if constexpr (CHAIN)
        wait_stages<AR, NPRE>(min(NS - 2, nk - 1));  // younger than A0: A1 .. A(NS-2) and the residual loads
      else
        wait_stages<DPS, NPRE>(min(NS - 2, nk - 1));
    } else {
      wait_stages<DPS>(min(NS - 2, nk - 1 - kt));
    }
    __builtin_amdgcn_s_barrier();
    if (kt == 0) probe_mark(g.probe, probe_t, 1);
    const uint32_t soff = (uint32_t)((kt % NS) * C::stage_bytes);
    u32x4 ar[SLABS][MT], br[SLABS][NT];
#pragma unroll
    for (int s = 0; s < SLABS; ++s) {
      static_for<0, MT>([&](auto I) {
        constexpr int i = decltype(I)::value;
        ar[s][i] = lds_read_b128<i * 16 * KB>(abase[s] + soff);
      });
      static_for<0, NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        br[s][j] = lds_read_b128<j * 16 * KB>(bbase[s] + soff);
      });
    }
    // WAR: slot (kt+NS-1)%NS == (kt-1)%NS was last read in iteration kt-1, whose reads all
    // completed before that iteration's MFMAs, i.e. before every wave reached this barrier
    if (kt + NS - 1 < nk) stage((kt + NS - 1) % NS, (kt + NS - 1) * BKE);
    if constexpr (SLABS == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(ar[0][i]));
#pragma unroll
      for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(br[0][j]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = Slab<TC>::mma(__builtin_bit_cast(frag, br[0][j]), __builtin_bit_cast(frag, ar[0][i]), acc[i][j]);
      continue;
    } else {
    // slab 0's reads are the oldest MT+NT LDS ops: consume them while slab 1's land
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(MT + NT) : "memory");
#pragma unroll
    for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(ar[0][i]));
#pragma unroll
    for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(br[0][j]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = Slab<TC>::mma(__builtin_bit_cast(frag, br[0][j]), __builtin_bit_cast(frag, ar[0][i]), acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(ar[1][i]));
#pragma unroll
    for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(br[1][j]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = Slab<TC>::mma(__builtin_bit_cast(frag, br[SLABS - 1][j]), __builtin_bit_cast(frag, ar[SLABS - 1][i]),
                                  acc[i][j]);
    }
  }
  // the K loop's last wait was vmcnt(0) (hand-written, invisible to hipcc): say so with the builtin,
  // so hipcc does not wait again (behind the epilogue's own stores) before the first use of a value
  // loaded before the loop (the residual prefetch)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched
  __syncthreads();
  probe_mark(g.probe, probe_t, 2);
  // the fold consumer's row statistics, past the wave strips: (mean, rstd) of block row r at [2r, 2r + 2)
  float* const ln_rows = reinterpret_cast<float*>(lds) + NW * 16 * C::EPAD;
  if constexpr (LNC) {
    static_assert(C::bytes >= (NW * 16 * C::EPAD + 2 * BM) * 4, "LDS for the fold's row statistics");
    if (g.ln_part_in) {  // uniform
      if (tid < BM) ln_row_stats(g, lnraw, ln_rows + 2 * tid);
      __syncthreads();
    }
  }

  // ---- epilogue, per wave and 16-row strip: accumulators -> the wave's LDS strip (fp32,
  // padded rows) -> 8-column chunks of whole rows, so the epilogue's global accesses are
  // 16-32 B vectors along rows. Strips are wave-private: LDS order within a wave suffices.
  float* Cs = reinterpret_cast<float*>(lds) + wid * 16 * C::EPAD;
  constexpr int CH = WN / 8;  // 8-column chunks per strip row
  constexpr int TPC = 16 * CH / 64;  // chunks per lane per strip
  // Fast path (whole-column tiles of the hot epilogues): a lane's column chunk is the same in
  // every strip, so bias/gate/QKV head indices are loaded once, and the row data of strip i+1
  // (RoPE pairs, residual rows, row masks) is fetched before strip i stores: no vmcnt wait in
  // the strip loop covers an older store (one strip of global round trips instead of one per
  // chunk; measured 9.5 us of a 30.6 us QKV launch before).
  constexpr bool FAST_EPI = FAST && NT % 2 == 0;
  static_assert(FAST_EPI || !PUB, "the chain publishes after the fast (LDS-strip) epilogue");
  if constexpr (FAST_EPI) {
    epilogue_fast<TC, EPI, MT, NT, WN, C::EPAD, PREF, PUB ? kAuxWT : 0>(g, acc, Cs, m0 + wm * WM, n0 + wn * WN, lane,
                                                                         pre, LNC ? ln_rows + 2 * wm * WM : nullptr);
    if constexpr (PUB) chain_publish(dep, g.M, m0, BM);
  }
  if constexpr (!FAST_EPI) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      // swapped-operand layout: the lane's row fr, four consecutive columns 16j + 4q
#pragma unroll
      for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(Cs + fr * C::EPAD + j * 16 + 4 * q) = acc[i][j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int t = 0; t < TPC; ++t) {
        const int idx = t * 64 + lane, rr = idx / CH, cc = idx % CH;
        const int row = m0 + wm * WM + i * 16 + rr, col = n0 + wn * WN + cc * 8;
        const float* src = Cs + rr * C::EPAD + cc * 8;
        float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
        if (row < g.M && col < g.N)
          epi8<TC, EPI>(g, row, col, V8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}}, PREF ? &pre[PREF ? i : 0][PREF ? t : 0] : nullptr);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  probe_exit(g.probe, probe_t);
}

template <typename TC, int EPI, int BM, int BN, int WGM, int WGN, int NS, bool FAST = false, int KB = 128>
__global__ __launch_bounds__(64 * WGM * WGN, 2) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) uint4 lds[GemmCfg<BM, BN, WGM, WGN, NS, KB>::bytes / 16];
  gemm_body<TC, EPI, BM, BN, WGM, WGN, NS, FAST, KB>(g, blockIdx.x, gridDim.x, lds, ChainDep{});
}

// ======================================================================================
// Ping-pong GEMM (bf16 operands): 512 threads = two groups of 4 waves, one block per CU.
// Group g owns output rows [g*BM/2, (g+1)*BM/2) of the BM x BN tile; its 4 waves split that
// half as WGM2 x WGN2. The groups run half a period apart, so on every SIMD one wave issues
// its MFMA cluster while its partner wave (other group) reads its next fragments from LDS and
// issues LDS-DMA (MI355X_MICROARCH.md "Two waves per SIMD"):
//
//   half-period h:  2p       2p+1     2p+2  ...
//   group 0:        mem(p)   mma(p)   mem(p+1)
//   group 1:        mma(p-1) mem(p)   mma(p)
//
// with one s_barrier between half-periods. A phase p covers KS K32-stages. The LDS ring holds
// R = D + 1 = 3 phases; phase p+2 is fetched during mem(p): group 0 brings its A rows, group 1
// its B rows (so the vmcnt counts are group constants). Visibility of phase p+1 for the
// readers of the next half-period: each issuing wave waits for its own DMA with a counted
// vmcnt before the barrier that ends its mem phase (one phase younger stays in flight).
// Slot reuse: phase p+2's slot held phase p-1, last read at half-period 2p-1 (group 1) and
// retired (lgkmcnt(0)) before the barrier that ended it.
//
// LDS image of a stage: A rows [0,BM) then W rows [0,BN), 64 bytes (K32) per row = 4 chunks of
// 16 B; chunk c of row r sits at c ^ f[(r>>2)&3], f = {0,2,3,1}: conflict-free for
// ds_read_b128, whose four 16-lane groups ({0-3,12-15,20-27}, ...) each read rows
// {r, r+12} at chunk c and rows r+4..r+11 at chunk c+1.
// ======================================================================================
template <int BM, int BN, int WGM2, int WGN2, int KS, int D>
struct PPCfg {
  static constexpr int WM = BM / 2 / WGM2, WN = BN / WGN2, MT = WM / 16, NT = WN / 16;
  static constexpr int stage_bytes = (BM + BN) * 64;
  static constexpr int R = D + 1;                              // ring phases
  static constexpr int ring_bytes = R * KS * stage_bytes;
  static constexpr int EPAD = WN + 4;
  static constexpr int epi_bytes = 8 * 16 * EPAD * 4;
  static constexpr int bytes = ring_bytes > epi_bytes ? ring_bytes : epi_bytes;
  static constexpr int NA = BM / 64, NB = BN / 64;             // glds per stage per thread of a group
  static_assert(WGM2 * WGN2 == 4, "4 waves per group");
  static_assert(MT * 16 == WM && NT * 16 == WN, "16x16 fragments");
  static_assert(NA * 64 == BM && NB * 64 == BN, "whole DMA rounds");
  static_assert(bytes <= 160 * 1024, "LDS");
};

template <typename TC, int EPI, int BM, int BN, int WGM2, int WGN2, int KS, int D, bool FAST = false>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs g) {
  const ProbeT probe_t = probe_enter(g.probe);
  typedef PPCfg<BM, BN, WGM2, WGN2, KS, D> C;
  constexpr int WM = C::WM, WN = C::WN, MT = C::MT, NT = C::NT, NA = C::NA, NB = C::NB;
  constexpr int SB = C::stage_bytes, PB = KS * SB;  // stage / phase bytes
  __shared__ __attribute__((aligned(16))) uint4 lds[C::bytes / 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, w4 = wid & 3;
  const int wm = w4 / WGN2, wn = w4 % WGN2;
  const int ntn = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x, b = blockIdx.x, xq = nwg >> 3, xr = nwg & 7, xcd = b & 7;
  const int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (b >> 3);
  // with the pad skip, row tiles of padding cluster by sequence: spread the m-rows over the XCDs
  const int mrow = g.live_len ? spread8(bid / ntn, (g.M + BM - 1) / BM) : bid / ntn;
  const int m0 = mrow * BM, n0 = (bid % ntn) * BN;
  if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
    if (!tile_live(g, m0, BM)) {
      probe_exit(g.probe, probe_t);
      return;
    }
  }
  const TC* A = reinterpret_cast<const TC*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);

  // ---- DMA: group 0 stages the A rows, group 1 the W rows. Instruction i of wave w4 covers
  // rows (i*4 + w4)*16 .. +15 of its operand; lane -> (row = lane>>2, physical chunk lane&3).
  constexpr int NI = NA > NB ? NA : NB;
  const int nI = grp == 0 ? NA : NB;
  // by buffer_load ... lds against the group's panel (its A rows or W rows): the lane's byte offset is fixed,
  // the stage's K offset a scalar (soffset), so a stage costs no vector instructions; rows past M (N) read as
  // zero and feed only unstored outputs
  const int ld = grp == 0 ? g.lda : g.ldw;
  const TC* pan = grp == 0 ? A + (int64_t)m0 * g.lda : W + (int64_t)n0 * g.ldw;
  const TC* pan2 = (grp == 0 && g.A2) ? reinterpret_cast<const TC*>(g.A2) + (int64_t)m0 * g.lda : pan;
  const uint32_t pbytes = (uint32_t)((grp == 0 ? min(BM, g.M - m0) : min(BN, g.N - n0)) * ld * 2);
  uint32_t voff[NI], dst_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int row = (i * 4 + w4) * 16 + (lane >> 2);
    const int lc = swz64(row, lane & 3);  // logical chunk held at this physical slot
    voff[i] = (uint32_t)((row * ld + lc * 8) * 2);
    dst_off[i] = (uint32_t)((grp == 0 ? 0 : BM * 64) + (i * 4 + w4) * 16 * 64);
  }
  char* lds_c = reinterpret_cast<char*>(lds);
  auto dma_phase = [&](int p) {  // this wave's part of phase p (KS stages)
    const int slot = p % C::R;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = (p * KS + s) * 32;
      const bool second = grp == 0 && g.A2 && k0 >= g.k_split;  // A columns [k_split, K) from the A2 panel
      const __amdgpu_buffer_rsrc_t rs =
          rsrc_of(second ? pan2 : pan, pbytes);
      const int ks = second ? k0 - g.k_split : k0;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        if (i < nI)
          dma16(rs, (LDS_PTR(void))(lds_c + slot * PB + s * SB + dst_off[i]), voff[i], ks * 2);
    }
  };
  // own DMA of phase `need` landed, given phases up to `issued` were issued (counted vmcnt:
  // the younger phases stay in flight)
  auto wait_dma = [&](int need, int issued) {
    const int younger = min(max(issued - need, 0), D - 1);
    static_for<0, D>([&](auto Y) {
      constexpr int y = decltype(Y)::value;
      if (younger == y) {
        if (grp == 0)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(y * KS * NA) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(y * KS * NB) : "memory");
      }
    });
  };

  // ---- fragment read addresses: row bits (r>>2)&3 are lane constants (tile bases are
  // multiples of 16), so one base per operand per ring slot, tiles at immediate offsets
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  const int fr = lane & 15, q = lane >> 4;
  const int arow = grp * (BM / 2) + wm * WM + fr, brow = wn * WN + fr;
  const uint32_t a_lane = lds0 + arow * 64 + swz64(arow, q) * 16;
  const uint32_t b_lane = lds0 + BM * 64 + brow * 64 + swz64(brow, q) * 16;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 af[KS][MT], bfr[KS][NT];
  auto read_phase = [&](int p) {
    const uint32_t so = (uint32_t)((p % C::R) * PB);
    static_for<0, KS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      static_for<0, MT>([&](auto I) {
        constexpr int i = decltype(I)::value;
        af[s][i] = lds_read_b128<s * SB + i * 1024>(a_lane + so);
      });
      static_for<0, NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        bfr[s][j] = lds_read_b128<s * SB + j * 1024>(b_lane + so);
      });
    });
  };

  const int nph = g.K / (32 * KS);
  // LayerNorm / RMSNorm fold consumer: the block's rows' strip partials (ln_row_fetch), issued AHEAD of the prologue
  // DMA, so every counted wait below stays exact (they are the oldest loads: the first wait retires them with phase
  // 0). Behind the DMA they made the first in-loop wait retire phase 2 early: +1 us of ramp per C5 FFN1 tile.
  constexpr bool LNC = (EPI == EPI_QKV || EPI == EPI_GELU_TANH) && is16<TC>() && WN == 64 && FAST && NT % 2 == 0 &&
                       BM <= 512;
  u32x4 lnraw[LNC ? 8 : 1];
  if constexpr (LNC) ln_row_fetch(g, m0, tid, BM, lnraw);
  for (int p = 0; p < D && p < nph; ++p) dma_phase(p);
  wait_dma(0, min(D, nph) - 1);
  __builtin_amdgcn_s_barrier();
  probe_mark(g.probe, probe_t, 1);
  if (grp == 1) __builtin_amdgcn_s_barrier();  // group 1 sits out half-period 0
  for (int p = 0; p < nph; ++p) {
    // ---- mem(p): fragments of phase p, DMA of phase p+2, wait for own part of phase p+1
    read_phase(p);
    if (p + D < nph) dma_phase(p + D);
    wait_dma(p + 1, min(p + D, nph - 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(af[s][i]));
#pragma unroll
      for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(bfr[s][j]));
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- mma(p)
    typedef typename Op16<TC>::v8 v8;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = Op16<TC>::mma16(__builtin_bit_cast(v8, bfr[s][j]), __builtin_bit_cast(v8, af[s][i]), acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (hand-written waits above are invisible to hipcc)
  __syncthreads();
  probe_mark(g.probe, probe_t, 2);
  float* const ln_rows = reinterpret_cast<float*>(lds) + 8 * 16 * C::EPAD;  // past the 8 wave strips
  if constexpr (LNC) {
    static_assert(C::bytes >= (8 * 16 * C::EPAD + 2 * BM) * 4, "LDS for the fold's row statistics");
    if (g.ln_part_in) {  // uniform
      if (tid < BM) ln_row_stats(g, lnraw, ln_rows + 2 * tid);
      __syncthreads();
    }
  }

  // ---- epilogue: as gemm_kernel, per wave and 16-row strip through LDS
  float* Cs = reinterpret_cast<float*>(lds) + wid * 16 * C::EPAD;
  constexpr int CH = WN / 8;
  const int rbase = m0 + grp * (BM / 2) + wm * WM, cbase = n0 + wn * WN;
  if constexpr (FAST) {
    // whole-column tiles: the strip-pipelined epilogue (the generic one below waits out every strip's
    // residual / RoPE loads before its stores: 13-15 us per 256x256 tile at C3, profiles/r03_timeline_c3.txt)
    const V8 none[1][1] = {};
    epilogue_fast<TC, EPI, MT, NT, WN, C::EPAD, false>(g, acc, Cs, rbase, cbase, lane, none,
                                                       LNC ? ln_rows + 2 * (grp * (BM / 2) + wm * WM) : nullptr);
  } else {
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
      *reinterpret_cast<f32x4*>(Cs + fr * C::EPAD + j * 16 + 4 * q) = acc[i][j];  // swapped layout
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int idx = lane; idx < 16 * CH; idx += 64) {
      const int rr = idx / CH, cc = idx % CH;
      const int row = rbase + i * 16 + rr, col = cbase + cc * 8;
      const float* sp = Cs + rr * C::EPAD + cc * 8;
      float4 x0 = *reinterpret_cast<const float4*>(sp), x1 = *reinterpret_cast<const float4*>(sp + 4);
      if (row < g.M && col < g.N) epi8<TC, EPI>(g, row, col, V8{{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w}});
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  }
  probe_exit(g.probe, probe_t);
}

// ======================================================================================
// Persistent ping-pong GEMM (cfg 13; whole-column tiles with the direct epilogue only): the gemm_pp_kernel
// schedule, but one block per CU walks a sequence of tiles and the LDS-DMA pipeline runs across tile
// boundaries -- the next tile's first phases are issued while the current tile's last phases compute, and its
// operands land while the register-only epilogue runs -- so no tile pays a ramp, and no block-dispatch gap
// separates a CU's tiles (profiles/archive/r03_timeline_c3_epilogue.txt: ~3 us between a CU's consecutive
// 256x256 tiles beside a 2 us ramp). Tile order: XCD x (blocks b with b % 8 == x) takes the contiguous run of
// n-fastest tiles the non-persistent remap gives it, its blocks dealt round-robin over the run, so an XCD's
// resident tiles share A panels in its L2. Each accumulator takes its k-slabs in the same order as every other
// configuration (bitwise identical results).
// ======================================================================================
template <typename TC, int EPI, int BM, int BN, int WGM2, int WGN2, int KS, int D>
__global__ __launch_bounds__(512, 1) void gemm_ppp_kernel(GemmArgs g) {
  const ProbeT probe_t = probe_enter(g.probe);
  typedef PPCfg<BM, BN, WGM2, WGN2, KS, D> C;
  constexpr int WM = C::WM, WN = C::WN, MT = C::MT, NT = C::NT, NA = C::NA, NB = C::NB;
  constexpr int SB = C::stage_bytes, PB = KS * SB;  // stage / phase bytes
  __shared__ __attribute__((aligned(16))) uint4 lds[C::ring_bytes / 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, w4 = wid & 3;
  const int wm = w4 / WGN2, wn = w4 % WGN2;
  const int ntn = (g.N + BN - 1) / BN, nmt = (g.M + BM - 1) / BM, T = nmt * ntn;
  // this block's run: XCD x's contiguous tile range, every nbx-th tile from the block's position in it
  const int nwg = gridDim.x, b = blockIdx.x, x = b & 7, j0 = b >> 3;
  const int nbx = (nwg - x + 7) >> 3;  // blocks of this XCD
  const int xq = T >> 3, xr = T & 7;
  const int run0 = x < xr ? x * (xq + 1) : xr * (xq + 1) + (x - xr) * xq;
  const int runn = xq + (x < xr ? 1 : 0);
  // the k-th tile of the block (sequence index k >= 0): its (m0, n0), or false past the run's end; dead tiles
  // (every row padding, RESID with live_len) are skipped by next_live
  // GM > 1 (F5H_GEMM_GROUP_M): tile ids run m-fastest inside groups of GM row tiles, so the nbx tiles an XCD
  // holds at once form a GM x (nbx / GM) block (e.g. 4 x 8) that shares both A and W panels in its L2, instead
  // of ~3 rows x every column (the W panels of all columns re-streamed per wave of tiles)
  const int GM = g.group_m > 1 ? g.group_m : 1;
  auto tile_of = [&](int k, int& m0, int& n0) -> bool {
    const int r = j0 + k * nbx;
    if (r >= runn) return false;
    const int id = run0 + r;
    int mt, nt;
    if (GM > 1) {
      const int gsz = GM * ntn, grp0 = id / gsz, in = id - grp0 * gsz;
      const int gm = min(GM, nmt - grp0 * GM);  // rows in this (possibly partial, last) group
      mt = grp0 * GM + in % gm;
      nt = in / gm;
    } else {
      mt = id / ntn;
      nt = id % ntn;
    }
    const int mrow = g.live_len ? spread8(mt, nmt) : mt;
    m0 = mrow * BM;
    n0 = nt * BN;
    return true;
  };
  auto next_live = [&](int k, int& m0, int& n0) -> int {  // the first live tile at or after k, or -1
    for (;; ++k) {
      if (!tile_of(k, m0, n0)) return -1;
      if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
        if (!tile_live(g, m0, BM)) continue;
      }
      return k;
    }
  };
  const TC* A = reinterpret_cast<const TC*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);

  // ---- DMA (as gemm_pp_kernel): group 0 stages A rows, group 1 W rows; per tile the panel base and extent
  constexpr int NI = NA > NB ? NA : NB;
  const int nI = grp == 0 ? NA : NB;
  const int ld = grp == 0 ? g.lda : g.ldw;
  uint32_t voff[NI], dst_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int row = (i * 4 + w4) * 16 + (lane >> 2);
    const int lc = swz64(row, lane & 3);
    voff[i] = (uint32_t)((row * ld + lc * 8) * 2);
    dst_off[i] = (uint32_t)((grp == 0 ? 0 : BM * 64) + (i * 4 + w4) * 16 * 64);
  }
  char* lds_c = reinterpret_cast<char*>(lds);
  const int nph = g.K / (32 * KS);
  // DMA cursor: tile dk (its m0/n0 in dm0/dn0), phase dp within it; gi = phases issued so far
  int dm0 = 0, dn0 = 0;
  int dk = next_live(0, dm0, dn0), dp = 0, gi = 0;
  auto issue = [&]() {  // this wave's part of the next phase in the block's sequence, into ring slot gi % R
    const int slot = gi % C::R;
    const TC* pan = grp == 0 ? A + (int64_t)dm0 * g.lda : W + (int64_t)dn0 * g.ldw;
    const TC* pan2 = (grp == 0 && g.A2) ? reinterpret_cast<const TC*>(g.A2) + (int64_t)dm0 * g.lda : pan;
    const uint32_t pbytes = (uint32_t)((grp == 0 ? min(BM, g.M - dm0) : min(BN, g.N - dn0)) * ld * 2);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = (dp * KS + s) * 32;
      const bool second = grp == 0 && g.A2 && k0 >= g.k_split;
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(second ? pan2 : pan, pbytes);
      const int ks = second ? k0 - g.k_split : k0;
#pragma unroll
      for (int i = 0; i < NI; ++i)
        if (i < nI) dma16(rs, (LDS_PTR(void))(lds_c + slot * PB + s * SB + dst_off[i]), voff[i], ks * 2);
    }
    ++gi;
    if (++dp == nph) {
      dp = 0;
      dk = next_live(dk + 1, dm0, dn0);
    }
  };
  auto wait_dma = [&](int need, int issued) {  // own DMA of global phase `need` landed (younger ones in flight)
    const int younger = min(max(issued - need, 0), D - 1);
    static_for<0, D>([&](auto Y) {
      constexpr int y = decltype(Y)::value;
      if (younger == y) {
        if (grp == 0)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(y * KS * NA) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(y * KS * NB) : "memory");
      }
    });
  };

  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  const int fr = lane & 15, q = lane >> 4;
  const int arow = grp * (BM / 2) + wm * WM + fr, brow = wn * WN + fr;
  const uint32_t a_lane = lds0 + arow * 64 + swz64(arow, q) * 16;
  const uint32_t b_lane = lds0 + BM * 64 + brow * 64 + swz64(brow, q) * 16;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 af[KS][MT], bfr[KS][NT];
  auto read_phase = [&](int gp) {
    const uint32_t so = (uint32_t)((gp % C::R) * PB);
    static_for<0, KS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      static_for<0, MT>([&](auto I) {
        constexpr int i = decltype(I)::value;
        af[s][i] = lds_read_b128<s * SB + i * 1024>(a_lane + so);
      });
      static_for<0, NT>([&](auto J) {
        constexpr int j = decltype(J)::value;
        bfr[s][j] = lds_read_b128<s * SB + j * 1024>(b_lane + so);
      });
    });
  };

  // compute cursor: tile ck (its m0/n0), phase cp within it; gc = global phase index
  int cm0 = 0, cn0 = 0;
  int ck = next_live(0, cm0, cn0), cp = 0, gc = 0;
  if (ck < 0) {  // no live tile for this block
    probe_exit(g.probe, probe_t);
    return;
  }
  for (int p = 0; p < D && dk >= 0; ++p) issue();
  wait_dma(0, gi - 1);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // group 1 sits out half-period 0
  const V8 none[1][1] = {};
  for (;;) {
    // ---- mem(gc): fragments of phase gc, DMA of phase gc + D (possibly the next tile's), own part of gc + 1
    read_phase(gc);
    if (dk >= 0) issue();
    wait_dma(gc + 1, gi - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(af[s][i]));
#pragma unroll
      for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(bfr[s][j]));
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- mma(gc)
    typedef typename Op16<TC>::v8 v8;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = Op16<TC>::mma16(__builtin_bit_cast(v8, bfr[s][j]), __builtin_bit_cast(v8, af[s][i]), acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    ++gc;
    if (++cp == nph) {
      // the tile's epilogue (registers and global memory only: the ring keeps filling with the next tile)
      epilogue_direct<TC, EPI, MT, NT, false>(g, acc, cm0 + grp * (BM / 2) + wm * WM, cn0 + wn * WN, lane, none);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      cp = 0;
      ck = next_live(ck + 1, cm0, cn0);
      if (ck < 0) break;
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  probe_exit(g.probe, probe_t);
}

// ======================================================================================
// 256x256 8-phase GEMM (16-bit operands; cdna_hip_programming.md §5, "The 256² 8-phase template"):
// 512 threads = 8 waves, one block per CU. K-tiles of 64 alternate between two 64 KB LDS buffers; a
// buffer holds the tile's A rows [0,256) and W rows [0,256) as four 128-row halves (A-top, A-bottom,
// B-left, B-right, 16 KB each, 128-byte rows XOR-swizzled by swz128g so every fragment read is one
// conflict-free ds_read_b128). Each K-tile runs as 4 phases, one 128x128 quadrant (A half x B half) of
// the block tile each; in a quadrant the 8 waves are 2 (M) x 4 (N), wave (wr, wc) computing rows
// wr*64..+64 and columns wc*32..+32 of it (4 x 2 fragments x 2 k-slabs = 16 MFMAs 16x16x32). A phase:
// fragment reads -> one half-tile of LDS-DMA (2 global_load_lds per thread) -> [phase 3: counted vmcnt]
// -> s_barrier -> lgkmcnt(0) -> 16 MFMAs -> s_barrier:
//   phase 0  (A-top, B-left):     reads A-top (8) + B-left (4)   DMA: A-bottom of tile t+1
//   phase 1  (A-top, B-right):    reads B-right (4)              DMA: A-top    of tile t+2 (last read in phase 0)
//   phase 2  (A-bottom, B-right): reads A-bottom (8)             DMA: B-left   of tile t+2 (last read in phase 0)
//   phase 3  (A-bottom, B-left):  no reads (registers kept)      DMA: B-right  of tile t+2 (last read in phase 1),
//            then vmcnt(6): tile t+1's last half (issued in phase 0) has landed, the three halves of tile
//            t+2 stay in flight across the barrier (never vmcnt(0) in the steady state).
// RAW: a half is read in a phase after the barrier that follows its wait. WAR: a half is restaged one phase
// after the phase that read it (every wave retired those reads by lgkmcnt(0) before the barrier ending that
// phase); A-bottom two phases after. Each accumulator takes its k-slabs and K-tiles in order, so the results
// are bitwise those of the other tile configurations.
// ======================================================================================
template <typename TC, int EPI, bool FAST = false>
__global__ __launch_bounds__(512, 1) void gemm_8p_kernel(GemmArgs g) {
  const ProbeT probe_t = probe_enter(g.probe);
  constexpr int BM = 256, BN = 256, KT = 64;
  constexpr int HALF = 128 * 128;      // bytes of one 128-row half (128-byte rows)
  constexpr int BUF = 4 * HALF;        // one K-tile: A-top, A-bottom, B-left, B-right
  constexpr int QW = 32, EPAD = QW + 4;  // a wave's columns per quadrant; epilogue strip row (fp32)
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * BUF / 16];
  typedef typename Op16<TC>::v8 v8;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int ntn = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x, b = blockIdx.x, xq = nwg >> 3, xr = nwg & 7, xcd = b & 7;
  const int bid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (b >> 3);
  // with the pad skip, row tiles of padding cluster by sequence: spread the m-rows over the XCDs
  const int mrow = g.live_len ? spread8(bid / ntn, (g.M + BM - 1) / BM) : bid / ntn;
  const int m0 = mrow * BM, n0 = (bid % ntn) * BN;
  if constexpr (EPI == EPI_RESID || EPI == EPI_RESID16) {
    if (!tile_live(g, m0, BM)) {
      probe_exit(g.probe, probe_t);
      return;
    }
  }
  const TC* A = reinterpret_cast<const TC*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);
  const TC* A2 = reinterpret_cast<const TC*>(g.A2);

  // ---- DMA sources: thread tid fills chunks p = j*512 + tid (j = 0, 1) of each half: row p >> 3, slot p & 7,
  // holding the global chunk swz128g(row, slot) (an involution: the reader XORs the same way)
  // by buffer_load ... lds against the block's A and W panels (byte offsets per lane fixed, the K-tile's a
  // scalar soffset: no vector instructions per half-tile); rows past M (N) read as zero (unstored outputs)
  uint32_t voff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = j * 512 + tid, row = p >> 3, slot = p & 7;
      const int chunk = swz128g(row, slot);
      voff[h][j] = (uint32_t)((((h & 1) * 128 + row) * (h < 2 ? g.lda : g.ldw) + chunk * 8) * 2);
    }
  const uint32_t abytes = (uint32_t)(min(256, g.M - m0) * g.lda * 2), wbytes = (uint32_t)(min(256, g.N - n0) * g.ldw * 2);
  const __amdgpu_buffer_rsrc_t wrs =
      rsrc_of(W + (int64_t)n0 * g.ldw, wbytes);
  char* lds_c = reinterpret_cast<char*>(lds);
  auto dma_half = [&](int t, int h) {  // half h (0 A-top, 1 A-bottom, 2 B-left, 3 B-right) of K-tile t
    const int k0 = t * KT;
    char* dst = lds_c + (t & 1) * BUF + h * HALF + wid * 64 * 16;
    if (h < 2) {
      const bool second = A2 && k0 >= g.k_split;
      const __amdgpu_buffer_rsrc_t ars = rsrc_of((second ? A2 : A) + (int64_t)m0 * g.lda, abytes);
      const int ka = second ? k0 - g.k_split : k0;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dma16(ars, (LDS_PTR(void))(dst + j * 512 * 16), voff[h][j], ka * 2);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dma16(wrs, (LDS_PTR(void))(dst + j * 512 * 16), voff[h][j], k0 * 2);
    }
  };

  // ---- fragment read addresses: fragment rows r satisfy r & 15 == lane & 15, so the swizzled chunk of
  // k-slab s is a lane constant; the halves and fragments sit at immediate offsets
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  const int fr = lane & 15, q = lane >> 4;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    abase[s] = lds0 + (wr * 64 + fr) * 128 + swz128g(fr, s * 4 + q) * 16;
    bbase[s] = lds0 + 2 * HALF + (wc * 32 + fr) * 128 + swz128g(fr, s * 4 + q) * 16;
  }

  f32x4 acc[2][2][4][2];  // [A half][B half][fragment row][fragment column]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 af[4][2], bl[2][2], br[2][2];  // A rows of one half (4 frags x 2 slabs); B-left, B-right (2 x 2)
  auto read_a = [&](uint32_t so, auto H) {
    constexpr int hh = decltype(H)::value;
    static_for<0, 4>([&](auto I) {
      constexpr int i = decltype(I)::value;
      af[i][0] = lds_read_b128<hh * HALF + i * 16 * 128>(abase[0] + so);
      af[i][1] = lds_read_b128<hh * HALF + i * 16 * 128>(abase[1] + so);
    });
  };
  auto read_b = [&](uint32_t so, auto H, u32x4 (&bf)[2][2]) {
    constexpr int hh = decltype(H)::value;
    static_for<0, 2>([&](auto J) {
      constexpr int j = decltype(J)::value;
      bf[j][0] = lds_read_b128<hh * HALF + j * 16 * 128>(bbase[0] + so);
      bf[j][1] = lds_read_b128<hh * HALF + j * 16 * 128>(bbase[1] + so);
    });
  };
  auto fence_regs = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      asm volatile("" : "+v"(af[i][0]));
      asm volatile("" : "+v"(af[i][1]));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      asm volatile("" : "+v"(bl[j][0]));
      asm volatile("" : "+v"(bl[j][1]));
      asm volatile("" : "+v"(br[j][0]));
      asm volatile("" : "+v"(br[j][1]));
    }
  };
  // barrier, the phase's reads retired, the quadrant's 16 MFMAs, barrier
  auto compute = [&](auto HA, auto HB, const u32x4 (&bf)[2][2]) {
    constexpr int ha = decltype(HA)::value, hb = decltype(HB)::value;
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence_regs();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[ha][hb][i][j] = Op16<TC>::mma16(__builtin_bit_cast(v8, bf[j][s]), __builtin_bit_cast(v8, af[i][s]),
                                              acc[ha][hb][i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  const int T = g.K / KT;
  // prologue: tile 0 (all four halves), tile 1 (A-top, B-left, B-right); wait for tile 0
  dma_half(0, 0);
  dma_half(0, 2);
  dma_half(0, 3);
  dma_half(0, 1);
  if (T > 1) {
    dma_half(1, 0);
    dma_half(1, 2);
    dma_half(1, 3);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  probe_mark(g.probe, probe_t, 1);
  for (int t = 0; t < T; ++t) {
    const uint32_t so = (uint32_t)((t & 1) * BUF);
    const bool more1 = t + 1 < T, more2 = t + 2 < T;
    // phase 0: (A-top, B-left)
    read_b(so, I0{}, bl);
    read_a(so, I0{});
    if (more1) dma_half(t + 1, 1);
    compute(I0{}, I0{}, bl);
    // phase 1: (A-top, B-right)
    read_b(so, I1{}, br);
    if (more2) dma_half(t + 2, 0);
    compute(I0{}, I1{}, br);
    // phase 2: (A-bottom, B-right)
    read_a(so, I1{});
    if (more2) dma_half(t + 2, 2);
    compute(I1{}, I1{}, br);
    // phase 3: (A-bottom, B-left); tile t+1 must have landed before this phase's first barrier
    if (more2) {
      dma_half(t + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    compute(I1{}, I0{}, bl);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (already so), told to hipcc
  __syncthreads();
  probe_mark(g.probe, probe_t, 2);

  // ---- epilogue per quadrant block (64 rows x 32 columns of one head for QKV), through the wave's strip
  float* Cs = reinterpret_cast<float*>(lds) + wid * 16 * EPAD;
  static_for<0, 4>([&](auto QB) {
    constexpr int ha = decltype(QB)::value >> 1, hb = decltype(QB)::value & 1;
    const int rbase = m0 + ha * 128 + wr * 64, cbase = n0 + hb * 128 + wc * QW;
    if constexpr (FAST) {
      const V8 none[1][1] = {};
      epilogue_fast<TC, EPI, 4, 2, QW, EPAD, false>(g, acc[ha][hb], Cs, rbase, cbase, lane, none);
    } else {
      constexpr int CH = QW / 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<f32x4*>(Cs + fr * EPAD + j * 16 + 4 * q) = acc[ha][hb][i][j];  // swapped layout
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int idx = lane; idx < 16 * CH; idx += 64) {
          const int rr = idx / CH, cc = idx % CH;
          const int row = rbase + i * 16 + rr, col = cbase + cc * 8;
          const float* sp = Cs + rr * EPAD + cc * 8;
          float4 x0 = *reinterpret_cast<const float4*>(sp), x1 = *reinterpret_cast<const float4*>(sp + 4);
          if (row < g.M && col < g.N)
            epi8<TC, EPI>(g, row, col, V8{{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w}});
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  });
  probe_exit(g.probe, probe_t);
}

template <typename TC, int EPI>
static void launch_8p(const GemmArgs& a, hipStream_t st);

// the fast epilogue: whole-column tiles, 16-B aligned rows, destinations a buffer descriptor covers
template <int EPI>
static bool fast_epi_ok(const GemmArgs& a, int BN) {
  const uint64_t span = (uint64_t)(a.M + a.dual_rows) * (uint64_t)std::max<int64_t>(a.ldc, a.N) * 4;
  return a.N % BN == 0 && (EPI == EPI_QKV || a.ldc % 8 == 0) && (EPI != EPI_INPROJ || a.ld_add % 8 == 0) &&
         span < 0xF0000000ull;
}

template <typename TC, int EPI, int BM, int BN, int WGM2, int WGN2, int KS, int D>
static void launch_pp(const GemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  constexpr bool HOT = EPI == EPI_QKV || EPI == EPI_RESID || EPI == EPI_RESID16 || EPI == EPI_GELU_TANH ||
                       EPI == EPI_GELU_ERF_OP || EPI == EPI_STORE || EPI == EPI_STORE16 || EPI == EPI_INPROJ;
  if constexpr (HOT) {
    if (fast_epi_ok<EPI>(a, BN)) {
      hipLaunchKernelGGL((gemm_pp_kernel<TC, EPI, BM, BN, WGM2, WGN2, KS, D, true>), dim3(tiles), dim3(512), 0, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_pp_kernel<TC, EPI, BM, BN, WGM2, WGN2, KS, D>), dim3(tiles), dim3(512), 0, st, a);
}

// cfg 13: one persistent block per CU (whole-column tiles with the direct epilogue; others take cfg 11)
int gemm_num_cus();
int gemm_group_m();
template <typename TC, int EPI, int BM, int BN, int WGM2, int WGN2, int KS, int D>
static void launch_ppp(const GemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  constexpr bool HOT = EPI == EPI_QKV || EPI == EPI_RESID || EPI == EPI_RESID16 || EPI == EPI_GELU_TANH ||
                       EPI == EPI_GELU_ERF_OP || EPI == EPI_STORE || EPI == EPI_STORE16 || EPI == EPI_INPROJ;
  if constexpr (HOT) {
    if (fast_epi_ok<EPI>(a, BN) && a.K >= 32 * KS * D) {
      const int grid = std::min(tiles, gemm_num_cus());
      GemmArgs b = a;
      b.group_m = gemm_group_m();
      hipLaunchKernelGGL((gemm_ppp_kernel<TC, EPI, BM, BN, WGM2, WGN2, KS, D>), dim3(grid), dim3(512), 0, st, b);
      return;
    }
  }
  launch_pp<TC, EPI, BM, BN, WGM2, WGN2, KS, D>(a, st);
}

// Tile configurations (16-bit operands; the fp32 parity mode always uses cfg 0):
//   0: 64x128,  4 waves (2x2, 32x64 each),  3 stages, 2 blocks/CU
//   1: 128x128, 4 waves (2x2, 64x64 each),  2 stages, 2 blocks/CU
//   5: 192x128, 4 waves (2x2, 96x64 each),  2 stages, 2 blocks/CU
//  11: 256x256 ping-pong, 8 waves as two groups of 4, 3-phase ring, 1 block/CU
// (round 1 also measured 128x256, 192x256, 256x128, 256x256 4-wave forms and seven other
// ping-pong geometries; none won a shape, so they are no longer built — DESIGN.md §3.)
// Per-CU LDS-DMA intake (~37 B/clk) bounds the small tiles: bytes per MFLOP staged =
// 64*(BM+BN)/(BM*BN) KB, so 64x128 -> 24, 128x128 -> 16, 256x256 -> 8.
template <typename TC, int EPI>
static void launch_8p(const GemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  constexpr bool HOT = EPI == EPI_QKV || EPI == EPI_RESID || EPI == EPI_RESID16 || EPI == EPI_GELU_TANH ||
                       EPI == EPI_GELU_ERF_OP || EPI == EPI_STORE || EPI == EPI_STORE16 || EPI == EPI_INPROJ;
  if constexpr (HOT) {
    if (fast_epi_ok<EPI>(a, 256)) {
      hipLaunchKernelGGL((gemm_8p_kernel<TC, EPI, true>), dim3(tiles), dim3(512), 0, st, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_8p_kernel<TC, EPI>), dim3(tiles), dim3(512), 0, st, a);
}

template <typename TC, int EPI, int BM, int BN, int WGM, int WGN, int NS, int KB = 128>
static void launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  constexpr bool HOT = EPI == EPI_QKV || EPI == EPI_RESID || EPI == EPI_RESID16 || EPI == EPI_GELU_TANH ||
                       EPI == EPI_GELU_ERF_OP || EPI == EPI_STORE || EPI == EPI_STORE16 || EPI == EPI_INPROJ;
  if constexpr (HOT) {
    if (fast_epi_ok<EPI>(a, BN)) {
      hipLaunchKernelGGL((gemm_kernel<TC, EPI, BM, BN, WGM, WGN, NS, true, KB>), dim3(tiles), dim3(64 * WGM * WGN), 0,
                         st, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_kernel<TC, EPI, BM, BN, WGM, WGN, NS, false, KB>), dim3(tiles), dim3(64 * WGM * WGN), 0, st,
                     a);
}

template <typename TC, int EPI>
static hipError_t launch_t(const GemmArgs& a, hipStream_t st) {
  if (a.M == 0) return hipSuccess;
  int cfg = 0;
  if constexpr (is16<TC>()) cfg = gemm_select_cfg(a);
  // the LayerNorm fold runs only in the strip epilogue of the 64-column-strip configurations (0, 1, 5, 11): a forced
  // 256x256 configuration without it (12: 32-column quadrant strips, 13: register-only epilogue) runs as cfg 11, the
  // same tile (every configuration gives the same bits); anything else is refused rather than ignored (the results
  // would be those of an unnormalised operand)
  if ((a.ln_part || a.ln_part_in) && (cfg == 12 || cfg == 13)) cfg = 11;
  // a 256x256 tile needs whole 256-column tiles for the strip epilogue: narrower outputs take the 128x128 tile
  if ((a.ln_part || a.ln_part_in) && cfg == 11 && !fast_epi_ok<EPI>(a, 256)) cfg = 1;
  if (a.hs || a.ln_part || a.ln_part_in) {
    // LayerNorm form: producer hs + hs_scale, consumer u + v; RMSNorm form (ln_rms): neither. Row masks only with the
    // RMSNorm form (the DiT fold runs on unmasked rows; UNetT batches keep their masks), never the pad-row skip (a
    // skipped tile would leave its rows' statistics unwritten)
    const bool prod = a.ln_part && EPI == EPI_RESID16 && (a.ln_rms ? !a.hs && !a.hs_scale : a.hs && a.hs_scale);
    const bool cons = a.ln_part_in && (EPI == EPI_GELU_TANH || EPI == EPI_QKV) &&
                      (a.ln_rms ? !a.ln_u && !a.ln_v : a.ln_u && a.ln_v);
    const int bn = cfg == 11 ? 256 : 128;
    if (!is16<TC>() || (a.ln_part && a.ln_part_in) || !(prod || cons) || a.ln_nparts <= 0 || a.ln_nparts > 16 ||
        (cfg != 0 && cfg != 1 && cfg != 5 && cfg != 11) || !fast_epi_ok<EPI>(a, bn) || (a.rowkeep && !a.ln_rms) ||
        a.live_len)
      return hipErrorInvalidValue;
  }
  switch (cfg) {
    case 0: launch_cfg<TC, EPI, 64, 128, 2, 2, 3>(a, st); break;
    case 1: launch_cfg<TC, EPI, 128, 128, 2, 2, 2>(a, st); break;
    case 5: launch_cfg<TC, EPI, 192, 128, 2, 2, 2>(a, st); break;
    default:
      if constexpr (is16<TC>()) {
        if (a.K % 64) return hipErrorInvalidValue;  // whole K64 tiles
        if (cfg != 11 && cfg != 12 && cfg != 13) return hipErrorInvalidValue;
        if (cfg == 11)
          launch_pp<TC, EPI, 256, 256, 1, 4, 1, 3>(a, st);
        else if (cfg == 13)
          launch_ppp<TC, EPI, 256, 256, 1, 4, 1, 3>(a, st);
        else
          launch_8p<TC, EPI>(a, st);
        break;
      }
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename TC>
static hipError_t launch_epi(int epi, const GemmArgs& a, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_t<TC, EPI_STORE>(a, st);
    case EPI_SILU: return launch_t<TC, EPI_SILU>(a, st);
    case EPI_GELU_TANH: return launch_t<TC, EPI_GELU_TANH>(a, st);
    case EPI_GELU_ERF: return launch_t<TC, EPI_GELU_ERF>(a, st);
    case EPI_RESID: return launch_t<TC, EPI_RESID>(a, st);
    case EPI_RESID16: return launch_t<TC, EPI_RESID16>(a, st);
    case EPI_RESID_FILL: return launch_t<TC, EPI_RESID_FILL>(a, st);
    case EPI_INPROJ: return launch_t<TC, EPI_INPROJ>(a, st);
    case EPI_QKV: return launch_t<TC, EPI_QKV>(a, st);
    case EPI_GELU_ERF_OP: return launch_t<TC, EPI_GELU_ERF_OP>(a, st);
    case EPI_STORE16: return launch_t<TC, EPI_STORE16>(a, st);
  }
  return hipErrorInvalidValue;
}


}  // namespace f5h
