// ConvPositionEmbedding (modules.py:175-201): Conv1d(d, d, k=31, groups=16, pad=15) [+mask] -> Mish,
// as an implicit GEMM on MFMA: K = 31 taps x 64 input channels of one group.
//
// 16-bit operands (conv16_kernel): one workgroup = 256 positions x the 64 output channels of one
// group of one sequence (C2: 8 x 16 x 2 = 256 workgroups, one round on 256 CUs), 8 waves as
// 4 (positions) x 2 (channels), 64 x 32 outputs per wave. The input window (286 rows x 64 ch) is
// staged once in LDS (masked rows -> 0); the group's 31 weight taps (254 KB) stream through a
// 3-slot LDS-DMA ring, 4 taps per slot, one stage kept in flight across each barrier (counted
// vmcnt, raw s_barrier), so each weight byte read from L2 serves 256 positions.
// fp32 parity operands (conv_kernel): 64 positions per workgroup, one tap per stage.
// Same k-slab MFMA scheme as the GEMM (bf16/fp16 16x16x32, fp32 16x16x4).
#include "common.h"
#include "kernels.h"

namespace f5h {

// Epilogue of a conv block from its [BP][CP] fp32 LDS image: IT 8-channel row chunks per thread at a
// fixed column (c8 = (tid & 7) * 8). Everything the chunks read (bias, row-mask bytes, residual rows)
// is loaded before any chunk is stored: a load issued after a store waits for it (gfx9 counts stores
// in vmcnt), and the former per-element bias loads under the row-mask branch waited one by one.
template <typename TC, int BP, int NT, int CP, int MODE>
F5H_DEV void conv_epilogue(const ConvArgs& a, const float* Cs, int tid, int s, int n0, int grp, int cg) {
  constexpr int IT = BP * 8 / NT;
  static_assert(IT * NT == BP * 8 && NT % 8 == 0, "whole chunk passes");
  const int L = a.L, d = a.d;
  const int c8 = (tid & 7) * 8, oc = grp * cg + c8;
  if (c8 >= cg) return;  // (groups narrower than 64 channels)
  const float4 b0 = *reinterpret_cast<const float4*>(a.bias + oc), b1 = *reinterpret_cast<const float4*>(a.bias + oc + 4);
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(a.rowkeep, a.rowkeep ? (uint64_t)a.S * L : 0);
  uint32_t kb[IT];
  float4 r0[IT], r1[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int pos = min(n0 + (tid >> 3) + it * (NT / 8), L - 1);
    kb[it] = __builtin_amdgcn_raw_buffer_load_b8(rk, (uint32_t)(s * L + pos), 0, 0);
    if constexpr (MODE != 0) {
      const float* rs = a.resid + ((int64_t)s * L + pos) * d + oc;
      r0[it] = *reinterpret_cast<const float4*>(rs);
      r1[it] = *reinterpret_cast<const float4*>(rs + 4);
    }
  }
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int row = (tid >> 3) + it * (NT / 8), pos = n0 + row;
    if (pos >= L) continue;
    const bool keep = !a.rowkeep || kb[it] != 0;
    const float* c = Cs + row * CP + c8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = keep ? c[e] + bb[e] : 0.f;
      v[e] = is16<TC>() ? mish_fast(x) : mish(x);
    }
    if constexpr (MODE == 0) {
      TC* y = reinterpret_cast<TC*>(a.y) + ((int64_t)s * L + pos) * d + oc;
      if constexpr (is16<TC>()) {
        typename Op16<TC>::v8 o = {from_f32<TC>(v[0]), from_f32<TC>(v[1]), from_f32<TC>(v[2]), from_f32<TC>(v[3]),
                                   from_f32<TC>(v[4]), from_f32<TC>(v[5]), from_f32<TC>(v[6]), from_f32<TC>(v[7])};
        *reinterpret_cast<typename Op16<TC>::v8*>(y) = o;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = from_f32<TC>(v[e]);
      }
    } else if constexpr (MODE == 2) {
      if constexpr (is16<TC>()) {
        TC* y = reinterpret_cast<TC*>(a.y) + ((int64_t)s * a.y_seq_stride + a.y_row_off + pos) * d + oc;
        typename Op16<TC>::v8 o = {
            from_f32<TC>(v[0] + r0[it].x), from_f32<TC>(v[1] + r0[it].y), from_f32<TC>(v[2] + r0[it].z),
            from_f32<TC>(v[3] + r0[it].w), from_f32<TC>(v[4] + r1[it].x), from_f32<TC>(v[5] + r1[it].y),
            from_f32<TC>(v[6] + r1[it].z), from_f32<TC>(v[7] + r1[it].w)};
        *reinterpret_cast<typename Op16<TC>::v8*>(y) = o;
      }
    } else {
      float* y = reinterpret_cast<float*>(a.y) + ((int64_t)s * a.y_seq_stride + a.y_row_off + pos) * d + oc;
      *reinterpret_cast<float4*>(y) = make_float4(v[0] + r0[it].x, v[1] + r0[it].y, v[2] + r0[it].z, v[3] + r0[it].w);
      *reinterpret_cast<float4*>(y + 4) =
          make_float4(v[4] + r1[it].x, v[5] + r1[it].y, v[6] + r1[it].z, v[7] + r1[it].w);
    }
  }
}
template <typename TC, int BP, int NT, int CP>
F5H_DEV void conv_epilogue_any(const ConvArgs& a, const float* Cs, int tid, int s, int n0, int grp, int cg) {
  if (a.mode == 0)
    conv_epilogue<TC, BP, NT, CP, 0>(a, Cs, tid, s, n0, grp, cg);
  else if (a.mode == 2)
    conv_epilogue<TC, BP, NT, CP, 2>(a, Cs, tid, s, n0, grp, cg);
  else
    conv_epilogue<TC, BP, NT, CP, 1>(a, Cs, tid, s, n0, grp, cg);
}

// XCD-aware block -> (position block, group, sequence): the hardware deals workgroups round-robin over the 8
// XCDs, so with the natural grid order every XCD touched every group's 254 KB tap panel (8 L2 misses per
// panel: conv traffic 3.2x the algorithmic bytes, profiles/r03_pmc_classes.json). The bijective XCD-contiguous
// remap (cdna_hip_programming.md T1) with the group slowest gives each XCD a contiguous run of whole groups,
// so a panel leaves MALL/HBM about once.
F5H_DEV void conv_block(int& pb, int& grp, int& s) {
  const int npb = gridDim.x, ng = gridDim.y, ns = gridDim.z;
  const int nwg = npb * ng * ns;
  const int w = blockIdx.x + npb * (blockIdx.y + ng * blockIdx.z);
  const int xq = nwg >> 3, xr = nwg & 7, xcd = w & 7;
  const int id = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (w >> 3);
  grp = id / (ns * npb);
  const int rem = id - grp * (ns * npb);
  s = rem / npb;
  pb = rem - s * npb;
}

template <int N>
F5H_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// fp32 parity path: NWM x 2 waves; block = 32*NWM positions x 64 output channels, one tap per stage.
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
  int pb, grp, s;
  conv_block(pb, grp, s);
  const int n0 = pb * BP;
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
  // by buffer_load ... lds over the group's tap panel: lane offset fixed, the tap's a scalar, M0 wave-uniform
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  const __amdgpu_buffer_rsrc_t wrs = rsrc_of(Wg, (uint64_t)31 * 64 * 64 * sizeof(TC));
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
          dma16(wrs, (LDS_PTR(void))(Ws + (r * NWV + wid_s) * 64), (uint32_t)(woff[r] * (int)sizeof(TC)),
                (uint32_t)(t * 64 * 64 * (int)sizeof(TC)));
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
  conv_epilogue_any<TC, BP, NT, CP>(a, Cs, tid, s, n0, grp, cg);
}

// Input-window image: fragment reads take rows t + 16i + (lane & 15) for every tap t, so the
// conflict-free swizzle must hold for every row offset: chunk c of row r at c ^ (2 * ((r >> 1) & 3))
// covers each (row parity, 16-B slot) pair once per ds_read_b128 lane group at any offset (the
// weight panels use the GEMM's swz128g). Checked against the lane groups of MI355X_MICROARCH.md.
template <int OFF>
F5H_DEV u32x4 lds_rd128(uint32_t addr) {  // ds_read_b128 hidden from hipcc's waitcnt bookkeeping
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
F5H_DEV int swz_win(int row, int chunk) { return chunk ^ (((row >> 1) & 3) << 1); }
F5H_DEV int swz_tap(int row, int chunk) {
  const int r = row & 15;
  return chunk ^ ((r >> 1) ^ ((unsigned)(r - 4) < 8u ? 1 : 0));
}

template <typename TC, typename TX>
__global__ __launch_bounds__(512, 1) void conv16_kernel(ConvArgs a) {
  constexpr int CPR = 8;                  // 16-B chunks per 64-channel row
  constexpr int BP = 256, NT = 512;       // positions per block, threads
  constexpr int WROWS = BP + 30;          // input window rows
  constexpr int TS = 4, NST = 8, RING = 3;  // taps per stage, stages (31 taps), ring slots
  constexpr int TAPB = 64 * CPR;          // uint4 per tap panel (64 out ch x 64 in ch)
  typedef typename Slab<TC>::frag frag;
  __shared__ __attribute__((aligned(16))) uint4 lds[WROWS * CPR + RING * TS * TAPB];
  uint4* Xs = lds;
  uint4* Ws0 = lds + WROWS * CPR;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;  // 4 x 64 positions, 2 x 32 channels
  int pb, grp, s;
  conv_block(pb, grp, s);
  const int n0 = pb * BP;
  const int L = a.L, d = a.d;
  const TX* X = reinterpret_cast<const TX*>(a.x);
  const int cg = d / 16;  // channels per group (<= 64; padded to 64 in LDS and in the packed weights)
  const TC* Wg = reinterpret_cast<const TC*>(a.w) + (int64_t)grp * 31 * 64 * 64;

  // window rows q = n0-15 .. n0+270, plain loads (drained before the weight DMA is issued). Every
  // thread issues all of its loads before converting any (addresses clamped in range, so no load
  // waits on the row mask): one memory round trip instead of one per 512-chunk pass.
  {
    constexpr int NIT = (WROWS * CPR + NT - 1) / NT;
    constexpr int EPC = 16 / sizeof(TX);  // TX elements per 16-B load; 8 channels = 1 (16-bit) or 2 (fp32) loads
    // (no branch around any load: hipcc would wait for each conditional one in turn)
    uint4 raw[NIT][8 / EPC];
    uint32_t kb[NIT];
    bool okv[NIT];
    const __amdgpu_buffer_rsrc_t rk = rsrc_of(a.rowkeep, a.rowkeep ? (uint64_t)a.S * L : 0);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NT, row = idx / CPR, ch = idx % CPR;
      const int q = n0 - 15 + row;
      const int qc = min(max(q, 0), L - 1), cc = ch * 8 < cg ? ch * 8 : 0;
      okv[it] = idx < WROWS * CPR && q >= 0 && q < L && ch * 8 < cg;
      const uint4* src = reinterpret_cast<const uint4*>(X + ((int64_t)s * L + qc) * d + grp * cg + cc);
#pragma unroll
      for (int h = 0; h < 8 / EPC; ++h) raw[it][h] = src[h];  // in range for every idx (clamped row)
      kb[it] = __builtin_amdgcn_raw_buffer_load_b8(rk, (uint32_t)(s * L + qc), 0, 0);
    }
    if (a.rowkeep) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) okv[it] = okv[it] && kb[it] != 0;
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NT, row = idx / CPR, ch = idx % CPR;
      if (idx >= WROWS * CPR) continue;
      uint4 v;
      if constexpr (EPC == 8) {
        v = raw[it][0];
      } else {
        const float4 x0 = __builtin_bit_cast(float4, raw[it][0]), x1 = __builtin_bit_cast(float4, raw[it][1]);
        typename Op16<TC>::v8 o = {from_f32<TC>(x0.x), from_f32<TC>(x0.y), from_f32<TC>(x0.z), from_f32<TC>(x0.w),
                                   from_f32<TC>(x1.x), from_f32<TC>(x1.y), from_f32<TC>(x1.z), from_f32<TC>(x1.w)};
        v = __builtin_bit_cast(uint4, o);
      }
      Xs[row * CPR + swz_win(row, ch)] = okv[it] ? v : make_uint4(0, 0, 0, 0);
    }
  }
  // tap panel: lane chunk p = wid*64 + lane -> row p/8, source chunk swz_tap(row, p%8) (involution)
  const int prow = (wid * 64 + lane) / CPR, pslot = (wid * 64 + lane) % CPR;
  const int woff = prow * 64 + swz_tap(prow, pslot) * 8;
  // by buffer_load ... lds over the group's tap panel: lane offset fixed, the tap's a scalar, M0 wave-uniform
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  const __amdgpu_buffer_rsrc_t wrs = rsrc_of(Wg, (uint64_t)31 * 64 * 64 * sizeof(TC));
  auto wdma = [&](int st) {  // stage st -> ring slot st % RING; one 1 KB piece per tap per wave
    uint4* Wslot = Ws0 + (st % RING) * TS * TAPB;
#pragma unroll
    for (int u = 0; u < TS; ++u) {
      const int t = st * TS + u;
      if (t < 31)
        dma16(wrs, (LDS_PTR(void))(Wslot + u * TAPB + wid_s * 64), (uint32_t)(woff * (int)sizeof(TC)),
              (uint32_t)(t * 64 * 64 * (int)sizeof(TC)));
    }
  };
  auto taps_of = [](int st) { return st < 0 || st >= NST ? 0 : (31 - st * TS < TS ? 31 - st * TS : TS); };
  // wait until stage `st` has landed given stages up to `issued` were issued (younger stay in flight)
  auto wait_stage = [&](int st, int issued) {
    int younger = 0;
    for (int k = st + 1; k <= issued; ++k) younger += taps_of(k);
    switch (younger) {
      case 0: wait_vm<0>(); break;
      case 3: wait_vm<3>(); break;
      case 4: wait_vm<4>(); break;
      case 7: wait_vm<7>(); break;
      default: wait_vm<8>(); break;
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // window in LDS (own part)
  for (int st = 0; st < RING; ++st) wdma(st);
  wait_stage(0, RING - 1);
  __builtin_amdgcn_s_barrier();  // window + stage 0 visible to every wave

  // Fragment reads are inline asm (invisible to hipcc's waitcnt bookkeeping), two register sets: the
  // 12 reads of tap t+1 are in flight while tap t's 16 MFMAs run (the first tap of a stage waits for
  // the stage barrier). Window rows for tap t: r0 + 16 i + t; the swizzle depends on (r0 + t) only.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  const int q = lane >> 4, r0 = wm * 64 + (lane & 15);
  uint32_t bbase[2];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int row = wn * 32 + (lane & 15);
    bbase[sl] = lds0 + (uint32_t)(WROWS * CPR * 16) + row * 128 + swz_tap(row, sl * 4 + q) * 16;
  }
  typedef u32x4 FR[12];  // [0..7]: A (slab, i); [8..11]: B (slab, j)
  auto rd = [&](int t, FR& f) {
    const int rt = r0 + t, st = t / TS, u = t - st * TS;
    const uint32_t wo = (uint32_t)(((st % RING) * TS + u) * TAPB * 16);
    static_for<0, 2>([&](auto SL) {
      constexpr int sl = decltype(SL)::value;
      const uint32_t ab = lds0 + rt * 128 + swz_win(rt, sl * 4 + q) * 16;
      static_for<0, 4>([&](auto I) {
        constexpr int i = decltype(I)::value;
        f[sl * 4 + i] = lds_rd128<i * 16 * 128>(ab);
      });
      static_for<0, 2>([&](auto J) {
        constexpr int j = decltype(J)::value;
        f[8 + sl * 2 + j] = lds_rd128<j * 16 * 128>(bbase[sl] + wo);
      });
    });
  };
  auto mm = [&](FR& f) {
#pragma unroll
    for (int k = 0; k < 12; ++k) asm volatile("" : "+v"(f[k]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = Slab<TC>::mma(__builtin_bit_cast(frag, f[sl * 4 + i]), __builtin_bit_cast(frag, f[8 + sl * 2 + j]),
                                    acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  };
  FR fa, fb;
  rd(0, fa);
  for (int st = 0; st < NST; ++st) {
    // taps st*TS .. : even taps in fa, odd in fb (TS is even); tap t+1 is prefetched inside the stage
    static_for<0, TS>([&](auto U) {
      constexpr int u = decltype(U)::value;
      const int t = st * TS + u;
      if (t < 31) {
        FR& cur = (u & 1) ? fb : fa;
        FR& nxt = (u & 1) ? fa : fb;
        if (u + 1 < TS && t + 1 < 31) {
          rd(t + 1, nxt);
          asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        mm(cur);
      }
    });
    if (st + 1 < NST) {
      // stage st+1 landed (own pieces) -> barrier publishes it and retires every wave's reads of
      // slot st % RING, which stage st + RING then refills
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_stage(st + 1, st + RING - 1 < NST ? st + RING - 1 : NST - 1);
      __builtin_amdgcn_s_barrier();
      if (st + RING < NST) wdma(st + RING);
      rd((st + 1) * TS, fa);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue through LDS: [BP][68] fp32 image, 8-channel row chunks
  constexpr int CP = 68;
  static_assert(BP * CP * 4 <= (int)sizeof(lds), "epilogue tile fits the LDS image");
  float* Cs = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 64 + i * 16 + (lane >> 4) * 4 + r) * CP + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  conv_epilogue_any<TC, BP, NT, CP>(a, Cs, tid, s, n0, grp, cg);
}

hipError_t conv_pos(int compute, const ConvArgs& a, hipStream_t st) {
  // groups = 16; d/16 channels per group, padded to the 64-channel tile (d % 128 == 0)
  if (a.d % 128 != 0 || a.d > 1024) return hipErrorInvalidValue;
  if (compute == F5H_C_BF16 || compute == F5H_C_FP16) {
    dim3 grid((a.L + 255) / 256, 16, a.S);
    if (compute == F5H_C_BF16) {
      if (a.x_f32)
        hipLaunchKernelGGL((conv16_kernel<bf16, float>), grid, dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((conv16_kernel<bf16, bf16>), grid, dim3(512), 0, st, a);
    } else {
      if (a.x_f32)
        hipLaunchKernelGGL((conv16_kernel<f16, float>), grid, dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((conv16_kernel<f16, f16>), grid, dim3(512), 0, st, a);
    }
  } else {
    dim3 grid((a.L + 63) / 64, 16, a.S);
    hipLaunchKernelGGL((conv_kernel<float, float, 2>), grid, dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace f5h
