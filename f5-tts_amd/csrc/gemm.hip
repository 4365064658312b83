// MFMA GEMM with fused epilogues: C[M,N] = A[M,K] . W[N,K]^T (+ epilogue).
//
// Every nn.Linear on the CFM hot path lands here: QKV + RoPE
// (modules.py:481-509), out-proj + gated residual (modules.py:548-554,751), FFN1 + GELU-tanh
// and FFN2 + gated residual (modules.py:359-361,754-755), the hoisted input projection
// (dit.py:162), proj_out (dit.py:368), the all-steps AdaLN table (modules.py:321-323) and
// the ConvNeXt pointwise convs (modules.py:265-269).
//
// Tiling: 256 threads = 4 waves as 2x2, block tile BM x BN, K staged 128 bytes per row
// per stage (64 bf16 / 32 fp32) by LDS-DMA (global_load_lds) into a double-buffered,
// XOR-swizzled LDS image; A and W are both K-contiguous operand-dtype panels, so every
// fragment is one ds_read_b128. fp32 activations are converted to the operand dtype by
// the producer (or f32_to_op) before they reach a GEMM.
// bf16 mode: v_mfma_f32_16x16x32_bf16; fp32 parity mode: v_mfma_f32_16x16x4_f32 (exact f32).
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace f5h {

// ------------------------------------------------------------ epilogue (shared by both kernels)
// C layout (16x16 MFMA): col = lane&15, row = (lane>>4)*4 + r
template <typename TC, int EPI, int BM, int BN>
F5H_DEV void epilogue(const GemmArgs& g, f32x4 (&acc)[BM / 32][BN / 32], int m0, int n0, int wm, int wn, int lane) {
  constexpr int WM = BM / 2, WN = BN / 2, MT = WM / 16, NT = WN / 16;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + wn * WN + j * 16 + (lane & 15);
      const bool cok = col < g.N;
      const float b = (g.bias && cok) ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        const bool ok = cok && row < g.M;
        float v = acc[i][j][r] + b;
        if constexpr (EPI == EPI_QKV) {
          // interleaved RoPE pairs (2i, 2i+1) sit in adjacent lanes (x_transformers rotate_half)
          float pv = __shfl_xor(v, 1, 64);
          const int inner = g.heads * 64;
          const int which = col / inner, hc = col - which * inner;
          const int head = hc >> 6, dh = hc & 63;
          const int s = row / g.seq_len, pos = row - s * g.seq_len;
          if (ok) {
            if (which < 2 && head < g.rope_heads) {
              float2 cs = g.rope[(int64_t)pos * 32 + (dh >> 1)];
              v = (dh & 1) ? (v * cs.x + pv * cs.y) : (v * cs.x - pv * cs.y);
            }
            TC* dst = reinterpret_cast<TC*>(which == 0 ? g.q : (which == 1 ? g.k : g.v));
            dst[(((int64_t)s * g.heads + head) * g.seq_len + pos) * 64 + dh] = from_f32<TC>(v);
          }
        } else {
          if (!ok) continue;
          const int64_t off = (int64_t)row * g.ldc + col;
          if constexpr (EPI == EPI_STORE) {
            reinterpret_cast<float*>(g.C)[off] = v;
          } else if constexpr (EPI == EPI_SILU) {
            reinterpret_cast<float*>(g.C)[off] = silu(v);
          } else if constexpr (EPI == EPI_GELU_TANH) {
            reinterpret_cast<TC*>(g.C)[off] = from_f32<TC>(gelu_tanh(v));
          } else if constexpr (EPI == EPI_GELU_ERF) {
            reinterpret_cast<float*>(g.C)[off] = gelu_erf(v);
          } else if constexpr (EPI == EPI_RESID) {
            float gt = g.gate ? g.gate[col] : 1.f;
            float keep = (g.rowkeep && !g.rowkeep[row]) ? 0.f : 1.f;
            float* C = reinterpret_cast<float*>(g.C);
            C[off] = C[off] + gt * (v * keep);
          } else if constexpr (EPI == EPI_RESID_FILL) {
            float* C = reinterpret_cast<float*>(g.C);
            bool keep = !g.rowkeep || g.rowkeep[row];
            C[off] = keep ? C[off] + v : 0.f;
          } else if constexpr (EPI == EPI_INPROJ) {
            float* C = reinterpret_cast<float*>(g.C);
            const int64_t ao = (int64_t)row * g.ld_add + col;
            C[off] = v + g.add[ao];
            if (g.dual_rows) C[off + g.dual_rows * g.ldc] = v + g.add[ao + g.dual_rows * g.ld_add];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- LDS-DMA (global_load_lds) variant
// A and W both in operand dtype: each wave-instruction DMAs 64 x 16 B straight into LDS at
// (wave-uniform base + lane*16); the XOR swizzle is applied to the per-lane SOURCE chunk so the
// LDS image is the same swz128 image the fragment reads expect (swizzle is an involution).
// Two stages: the DMA of stage k+1 is in flight while stage k's MFMAs run; one drain + barrier per K-step.
template <typename TC, int EPI, int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_glds_kernel(GemmArgs g) {
  constexpr int E = elems16<TC>();
  constexpr int BKE = 8 * E;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int AR = BM * 8 / 256, BR = BN * 8 / 256;  // DMA rounds per stage
  typedef typename Slab<TC>::frag frag;

  __shared__ __attribute__((aligned(16))) uint4 lds[2 * (BM + BN) * 8];
  const int stage_u4 = (BM + BN) * 8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = (g.N + BN - 1) / BN;
  const int bid = blockIdx.x;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const TC* A = reinterpret_cast<const TC*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);

  // per-lane source offsets (elements), fixed across K-steps
  int64_t aoff[AR], boff[BR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    int p = (i * 4 + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    int m = min(m0 + row, g.M - 1);
    aoff[i] = (int64_t)m * g.lda + swz128(row, slot) * E;
  }
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    int p = (i * 4 + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    boff[i] = (int64_t)(n0 + row) * g.ldw + swz128(row, slot) * E;
  }
  auto stage = [&](int buf, int k0) {
    uint4* As = lds + buf * stage_u4;
    uint4* Bs = As + BM * 8;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(A + aoff[i] + k0), (LDS_PTR(void))(As + (i * 4 + wid) * 64),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(W + boff[i] + k0), (LDS_PTR(void))(Bs + (i * 4 + wid) * 64),
                                       16, 0, 0);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BKE;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const uint4* As = lds + cur * stage_u4;
    const uint4* Bs = As + BM * 8;
    // all fragment reads of this stage BEFORE the next stage's DMA is issued: hipcc would
    // otherwise wait vmcnt(0) (the pending LDS-DMA) in front of the first ds_read
    frag af[2][MT], bfr[2][NT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        int row = wm * WM + i * 16 + (lane & 15);
        uint4 v = As[row * 8 + swz128(row, ch)];
        af[s][i] = __builtin_bit_cast(frag, v);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        int row = wn * WN + j * 16 + (lane & 15);
        uint4 v = Bs[row * 8 + swz128(row, ch)];
        bfr[s][j] = __builtin_bit_cast(frag, v);
      }
    }
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BKE);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = Slab<TC>::mma(af[s][i], bfr[s][j], acc[i][j]);
    // keep the MFMAs above the DMA drain (asm "memory" does not order register-only MFMAs)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  epilogue<TC, EPI, BM, BN>(g, acc, m0, n0, wm, wn, lane);
}

template <typename TC, int EPI>
static hipError_t launch_t(const GemmArgs& a, hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  const int grid = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_glds_kernel<TC, EPI, BM, BN>), dim3(grid), dim3(256), 0, st, a);
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
    case EPI_RESID_FILL: return launch_t<TC, EPI_RESID_FILL>(a, st);
    case EPI_INPROJ: return launch_t<TC, EPI_INPROJ>(a, st);
    case EPI_QKV: return launch_t<TC, EPI_QKV>(a, st);
  }
  return hipErrorInvalidValue;
}

hipError_t gemm(int compute, int epi, const GemmArgs& a, hipStream_t st) {
  const int bke = compute ? 64 : 32;
  if (a.K % bke != 0 || a.M < 0 || a.N <= 0 || a.lda % 8 || a.ldw % 8) return hipErrorInvalidValue;
  return compute ? launch_epi<bf16>(epi, a, st) : launch_epi<float>(epi, a, st);
}

}  // namespace f5h
