// ConvPositionEmbedding (modules.py:175-201): Conv1d(d, d, k=31, groups=16, pad=15) [+mask] -> Mish,
// as an implicit GEMM on MFMA. One workgroup = 64 positions x the 64 output channels of one
// group of one sequence; K = 31 taps x 64 input channels. The input window (94 rows x 64 ch)
// is staged once in LDS (masked rows -> 0); the 31 weight taps stream through a
// double-buffered LDS panel, TS taps per stage (bf16: 4, so 8 barriers per block instead of 31;
// fp32: 1). Same k-slab MFMA scheme as the GEMM (bf16 16x16x32 / fp32 16x16x4).
#include "common.h"
#include "kernels.h"

namespace f5h {

// NWM x 2 waves; block = 32*NWM positions x 64 output channels (NWM = 4: 128 positions, so each
// 254 KB group weight stream from L2 serves twice the outputs of the 64-position block)
template <typename TC, typename TX, int NWM = 2>
__global__ __launch_bounds__(128 * NWM, 1) void conv_kernel(ConvArgs a) {
  constexpr int E = elems16<TC>();
  constexpr int CPR = 64 / E;  // 16-byte chunks per 64-channel row (8 bf16 / 16 fp32)
  constexpr int NT = 128 * NWM, BP = 32 * NWM;
  constexpr int WROWS = BP + 30;
  constexpr int TS = CPR == 8 ? 4 : 1;   // weight taps per LDS stage
  constexpr int NST = (31 + TS - 1) / TS;
  typedef typename Slab<TC>::frag frag;
  __shared__ __attribute__((aligned(16))) uint4 lds[WROWS * CPR + 2 * TS * 64 * CPR];
  uint4* Xs = lds;
  uint4* Ws0 = lds + WROWS * CPR;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * BP, grp = blockIdx.y, s = blockIdx.z;
  const int L = a.L, d = a.d;
  const TX* X = reinterpret_cast<const TX*>(a.x);
  const int cg = d / 16;  // channels per group (<= 64; padded to 64 in LDS and in the packed weights)
  const TC* Wg = reinterpret_cast<const TC*>(a.w) + (int64_t)grp * 31 * 64 * 64;

  auto swz = [](int row, int ch) { return CPR == 8 ? swz128(row, ch) : swz256(row, ch); };

  // window: rows q = n0-15 .. n0+78
  for (int idx = tid; idx < WROWS * CPR; idx += NT) {
    int row = idx / CPR, ch = idx % CPR;
    int q = n0 - 15 + row;
    bool ok = q >= 0 && q < L && ch * E < cg && (!a.rowkeep || a.rowkeep[(int64_t)s * L + q]);
    const TX* src = X + ((int64_t)s * L + (ok ? q : 0)) * d + grp * cg + (ok ? ch * E : 0);
    Xs[row * CPR + swz(row, ch)] = Load16<TC, TX>::ld(src, ok);
  }
  // weight taps stream by LDS-DMA: round r, wave w, lane l -> linear chunk p of the panel;
  // the swizzle goes on the source chunk so the LDS image is the swz() image (involution)
  constexpr int NWV = NT / 64;              // waves
  constexpr int WR = 64 * CPR / NT;         // DMA rounds per tap (64 rows x CPR chunks / NT lanes)
  static_assert(WR >= 1 && WR * NT == 64 * CPR, "whole DMA rounds per tap");
  int woff[WR];
  static_for<0, WR>([&](auto I) {
    constexpr int r = decltype(I)::value;
    const int p = (r * NWV + wid) * 64 + lane, row = p / CPR, slot = p % CPR;
    woff[r] = row * 64 + swz(row, slot) * E;
  });
  // stage st = taps [st*TS, st*TS + TS) (the last one shorter) into buffer buf
  auto wdma = [&](int buf, int st) {
    static_for<0, TS>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int t = st * TS + u;
      if (t < 31) {
        uint4* Ws = Ws0 + (buf * TS + u) * 64 * CPR;
        static_for<0, WR>([&](auto I) {
          constexpr int r = decltype(I)::value;
          __builtin_amdgcn_global_load_lds((const void*)(Wg + (int64_t)t * 64 * 64 + woff[r]),
                                           (LDS_PTR(void))(Ws + (r * NWV + wid) * 64), 16, 0, 0);
        });
      }
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
  for (int st = 0; st < NST; ++st) {
    const int cur = st & 1;
    if (st + 1 < NST) wdma(cur ^ 1, st + 1);  // next stage lands while this one is multiplied
#pragma unroll
    for (int u = 0; u < TS; ++u) {
      const int t = st * TS + u;
      if (t >= 31) break;
      const uint4* Ws = Ws0 + (cur * TS + u) * 64 * CPR;
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
#pragma unroll
      for (int sl = 0; sl < CPR / 4; ++sl)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = Slab<TC>::mma(af[sl][i], bfr[sl][j], acc[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue through LDS (the loop ended on a barrier, so the weight/window image is free): the
  // accumulator tile goes to a padded [BP][68] fp32 image and comes back as 8-channel row chunks,
  // so bias, mask, Mish, the residual read and the store are 16-32 B vector accesses
  constexpr int CP = 68;
  static_assert(BP * CP * 4 <= (int)sizeof(lds), "epilogue tile fits the LDS image");
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 32 + i * 16 + (lane >> 4) * 4 + r) * CP + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  for (int c = tid; c < BP * 8; c += NT) {
    const int row = c >> 3, c8 = (c & 7) * 8, pos = n0 + row;
    if (pos >= L || c8 >= cg) continue;
    const int oc = grp * cg + c8;
    const bool keep = !a.rowkeep || a.rowkeep[(int64_t)s * L + pos];
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = keep ? Cs[row * CP + c8 + e] + a.bias[oc + e] : 0.f;
      v[e] = is16<TC>() ? mish_fast(x) : mish(x);
    }
    if (a.mode == 0) {
      TC* y = reinterpret_cast<TC*>(a.y) + ((int64_t)s * L + pos) * d + oc;
      if constexpr (is16<TC>()) {
        typename Op16<TC>::v8 o = {from_f32<TC>(v[0]), from_f32<TC>(v[1]), from_f32<TC>(v[2]), from_f32<TC>(v[3]),
                                   from_f32<TC>(v[4]), from_f32<TC>(v[5]), from_f32<TC>(v[6]), from_f32<TC>(v[7])};
        *reinterpret_cast<typename Op16<TC>::v8*>(y) = o;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = from_f32<TC>(v[e]);
      }
    } else {
      float* y = reinterpret_cast<float*>(a.y) + ((int64_t)s * a.y_seq_stride + a.y_row_off + pos) * d + oc;
      const float* rs = a.resid + ((int64_t)s * L + pos) * d + oc;
      const float4 r0 = *reinterpret_cast<const float4*>(rs), r1 = *reinterpret_cast<const float4*>(rs + 4);
      *reinterpret_cast<float4*>(y) = make_float4(v[0] + r0.x, v[1] + r0.y, v[2] + r0.z, v[3] + r0.w);
      *reinterpret_cast<float4*>(y + 4) = make_float4(v[4] + r1.x, v[5] + r1.y, v[6] + r1.z, v[7] + r1.w);
    }
  }
}

hipError_t conv_pos(int compute, const ConvArgs& a, hipStream_t st) {
  // groups = 16; d/16 channels per group, padded to the 64-channel tile (d % 128 == 0)
  if (a.d % 128 != 0 || a.d > 1024) return hipErrorInvalidValue;
  if (compute == F5H_C_BF16 || compute == F5H_C_FP16) {
    dim3 grid((a.L + 127) / 128, 16, a.S);
    if (compute == F5H_C_BF16) {
      if (a.x_f32)
        hipLaunchKernelGGL((conv_kernel<bf16, float, 4>), grid, dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((conv_kernel<bf16, bf16, 4>), grid, dim3(512), 0, st, a);
    } else {
      if (a.x_f32)
        hipLaunchKernelGGL((conv_kernel<f16, float, 4>), grid, dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((conv_kernel<f16, f16, 4>), grid, dim3(512), 0, st, a);
    }
  } else {
    dim3 grid((a.L + 63) / 64, 16, a.S);
    hipLaunchKernelGGL((conv_kernel<float, float, 2>), grid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace f5h
