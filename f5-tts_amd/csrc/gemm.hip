// MFMA GEMM with fused epilogues: C[M,N] = A[M,K] . W[N,K]^T (+ epilogue).
//
// Every nn.Linear on the CFM hot path lands here: QKV + RoPE
// (modules.py:481-509), out-proj + gated residual (modules.py:548-554,751), FFN1 + GELU-tanh
// and FFN2 + gated residual (modules.py:359-361,754-755), the hoisted input projection
// (dit.py:162), proj_out (dit.py:368), the all-steps AdaLN table (modules.py:321-323) and
// the ConvNeXt pointwise convs (modules.py:265-269).
//
// Tiling: 256 threads = 4 waves as 2x2, block tile BM x BN, K staged 128 bytes per row
// per stage (64 bf16 / 32 fp32) through registers into a double-buffered, XOR-swizzled
// LDS image; A and W are both K-contiguous so every fragment is one ds_read_b128.
// bf16 mode: v_mfma_f32_16x16x32_bf16; fp32 parity mode: v_mfma_f32_16x16x4_f32 (exact f32).
#include "common.h"
#include "kernels.h"

namespace f5h {

template <typename TA, typename TC, int EPI, int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs g) {
  constexpr int E = elems16<TC>();       // operand elements per 16-byte chunk
  constexpr int BKE = 8 * E;              // K elements per stage (128 bytes)
  constexpr int WM = BM / 2, WN = BN / 2; // wave tile
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int ACH = BM * 8 / 256;       // A chunks per thread per stage
  constexpr int BCH = BN * 8 / 256;
  typedef typename Slab<TC>::frag frag;

  __shared__ __attribute__((aligned(16))) uint4 lds[2 * (BM + BN) * 8];
  uint4* As0 = lds;
  uint4* Bs0 = lds + BM * 8;
  const int stage_u4 = (BM + BN) * 8;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // tile mapping: n-tiles fastest so neighbouring blocks share the A panel
  const int ntn = (g.N + BN - 1) / BN;
  const int bid = blockIdx.x;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;

  const TA* A = reinterpret_cast<const TA*>(g.A);
  const TC* W = reinterpret_cast<const TC*>(g.W);

  uint4 ra[ACH], rb[BCH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      int m = m0 + row;
      ra[i] = Load16<TC, TA>::ld(A + (int64_t)(m < g.M ? m : 0) * g.lda + k0 + ch * E, m < g.M);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      rb[i] = *reinterpret_cast<const uint4*>(W + (int64_t)(n0 + row) * g.ldw + k0 + ch * E);
    }
  };
  auto sstore = [&](int buf) {
    uint4* As = As0 + buf * stage_u4;
    uint4* Bs = Bs0 + buf * stage_u4;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      As[row * 8 + swz128(row, ch)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      Bs[row * 8 + swz128(row, ch)] = rb[i];
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BKE;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BKE);
    const uint4* As = As0 + cur * stage_u4;
    const uint4* Bs = Bs0 + cur * stage_u4;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + (lane >> 4);
      frag af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        int row = wm * WM + i * 16 + (lane & 15);
        uint4 v = As[row * 8 + swz128(row, ch)];
        af[i] = *reinterpret_cast<frag*>(&v);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        int row = wn * WN + j * 16 + (lane & 15);
        uint4 v = Bs[row * 8 + swz128(row, ch)];
        bfr[j] = *reinterpret_cast<frag*>(&v);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = Slab<TC>::mma(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      __syncthreads();
      sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // ------------------------------------------------------------ epilogue
  // C layout (16x16): col = lane&15, row = (lane>>4)*4 + r
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

template <typename TA, typename TC, int EPI>
static hipError_t launch_t(const GemmArgs& a, hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  const int grid = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_kernel<TA, TC, EPI, BM, BN>), dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <typename TA, typename TC>
static hipError_t launch_epi(int epi, const GemmArgs& a, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_t<TA, TC, EPI_STORE>(a, st);
    case EPI_SILU: return launch_t<TA, TC, EPI_SILU>(a, st);
    case EPI_GELU_TANH: return launch_t<TA, TC, EPI_GELU_TANH>(a, st);
    case EPI_GELU_ERF: return launch_t<TA, TC, EPI_GELU_ERF>(a, st);
    case EPI_RESID: return launch_t<TA, TC, EPI_RESID>(a, st);
    case EPI_RESID_FILL: return launch_t<TA, TC, EPI_RESID_FILL>(a, st);
    case EPI_INPROJ: return launch_t<TA, TC, EPI_INPROJ>(a, st);
    case EPI_QKV: return launch_t<TA, TC, EPI_QKV>(a, st);
  }
  return hipErrorInvalidValue;
}

hipError_t gemm(int compute, bool a_f32, int epi, const GemmArgs& a, hipStream_t st) {
  const int bke = compute ? 64 : 32;
  if (a.K % bke != 0 || a.M < 0 || a.N <= 0) return hipErrorInvalidValue;
  if (compute) {
    return a_f32 ? launch_epi<float, bf16>(epi, a, st) : launch_epi<bf16, bf16>(epi, a, st);
  }
  return launch_epi<float, float>(epi, a, st);
}

}  // namespace f5h
