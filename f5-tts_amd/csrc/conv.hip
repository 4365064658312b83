// ConvPositionEmbedding (modules.py:175-201): Conv1d(d, d, k=31, groups=16, pad=15) [+mask] -> Mish,
// as an implicit GEMM on MFMA. One workgroup = 64 positions x the 64 output channels of one
// group of one sequence; K = 31 taps x 64 input channels. The input window (94 rows x 64 ch)
// is staged once in LDS (masked rows -> 0); the 31 weight taps stream through a
// double-buffered LDS panel. Same k-slab MFMA scheme as the GEMM (bf16 16x16x32 / fp32 16x16x4).
#include "common.h"
#include "kernels.h"

namespace f5h {

template <typename TC, typename TX>
__global__ __launch_bounds__(256, 2) void conv_kernel(ConvArgs a) {
  constexpr int E = elems16<TC>();
  constexpr int CPR = 64 / E;  // 16-byte chunks per 64-channel row (8 bf16 / 16 fp32)
  constexpr int WROWS = 64 + 30;
  typedef typename Slab<TC>::frag frag;
  __shared__ __attribute__((aligned(16))) uint4 lds[WROWS * CPR + 2 * 64 * CPR];
  uint4* Xs = lds;
  uint4* Ws0 = lds + WROWS * CPR;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * 64, grp = blockIdx.y, s = blockIdx.z;
  const int L = a.L, d = a.d;
  const TX* X = reinterpret_cast<const TX*>(a.x);
  const int cg = d / 16;  // channels per group (<= 64; padded to 64 in LDS and in the packed weights)
  const TC* Wg = reinterpret_cast<const TC*>(a.w) + (int64_t)grp * 31 * 64 * 64;

  auto swz = [](int row, int ch) { return CPR == 8 ? swz128(row, ch) : swz256(row, ch); };

  // window: rows q = n0-15 .. n0+78
  for (int idx = tid; idx < WROWS * CPR; idx += 256) {
    int row = idx / CPR, ch = idx % CPR;
    int q = n0 - 15 + row;
    bool ok = q >= 0 && q < L && ch * E < cg && (!a.rowkeep || a.rowkeep[(int64_t)s * L + q]);
    const TX* src = X + ((int64_t)s * L + (ok ? q : 0)) * d + grp * cg + (ok ? ch * E : 0);
    Xs[row * CPR + swz(row, ch)] = Load16<TC, TX>::ld(src, ok);
  }
  // weight taps stream by LDS-DMA: round r, wave w, lane l -> linear chunk p of the panel;
  // the swizzle goes on the source chunk so the LDS image is the swz() image (involution)
  constexpr int WR = CPR / 4;  // DMA rounds per tap (64 rows x CPR chunks / 256 lanes)
  int woff[WR];
  static_for<0, WR>([&](auto I) {
    constexpr int r = decltype(I)::value;
    const int p = (r * 4 + wid) * 64 + lane, row = p / CPR, slot = p % CPR;
    woff[r] = row * 64 + swz(row, slot) * E;
  });
  auto wdma = [&](int buf, int t) {
    uint4* Ws = Ws0 + buf * 64 * CPR;
    static_for<0, WR>([&](auto I) {
      constexpr int r = decltype(I)::value;
      __builtin_amdgcn_global_load_lds((const void*)(Wg + (int64_t)t * 64 * 64 + woff[r]),
                                       (LDS_PTR(void))(Ws + (r * 4 + wid) * 64), 16, 0, 0);
    });
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  wdma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < 31; ++t) {
    const int cur = t & 1;
    const uint4* Ws = Ws0 + cur * 64 * CPR;
    frag af[CPR / 4][2], bfr[CPR / 4][2];
#pragma unroll
    for (int sl = 0; sl < CPR / 4; ++sl) {
      const int ch = sl * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int row = wm * 32 + i * 16 + (lane & 15) + t;  // window row of input pos + t - 15
        af[sl][i] = __builtin_bit_cast(frag, Xs[row * CPR + swz(row, ch)]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int row = wn * 32 + j * 16 + (lane & 15);
        bfr[sl][j] = __builtin_bit_cast(frag, Ws[row * CPR + swz(row, ch)]);
      }
    }
    if (t + 1 < 31) wdma(cur ^ 1, t + 1);
#pragma unroll
    for (int sl = 0; sl < CPR / 4; ++sl)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Slab<TC>::mma(af[sl][i], bfr[sl][j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ol = wn * 32 + j * 16 + (lane & 15);
      if (ol >= cg) continue;
      const int oc = grp * cg + ol;
      const float b = a.bias[oc];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pos = n0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (pos >= L) continue;
        float v = acc[i][j][r] + b;
        if (a.rowkeep && !a.rowkeep[(int64_t)s * L + pos]) v = 0.f;
        v = mish(v);
        if (a.mode == 0) {
          reinterpret_cast<TC*>(a.y)[((int64_t)s * L + pos) * d + oc] = from_f32<TC>(v);
        } else {
          const int64_t yo = ((int64_t)s * a.y_seq_stride + a.y_row_off + pos) * d + oc;
          reinterpret_cast<float*>(a.y)[yo] = v + a.resid[((int64_t)s * L + pos) * d + oc];
        }
      }
    }
}

hipError_t conv_pos(int compute, const ConvArgs& a, hipStream_t st) {
  // groups = 16; d/16 channels per group, padded to the 64-channel tile (d % 128 == 0)
  if (a.d % 128 != 0 || a.d > 1024) return hipErrorInvalidValue;
  dim3 grid((a.L + 63) / 64, 16, a.S);
  if (compute) {
    if (a.x_f32)
      hipLaunchKernelGGL((conv_kernel<bf16, float>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv_kernel<bf16, bf16>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_kernel<float, float>), grid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace f5h
