// Non-causal multi-head attention, head_dim 64 (AttnProcessor, modules.py:511-520):
// O = softmax(Q K^T * scale [+ key-padding mask]) V, flash-style (scores never materialised).
//
// 16-bit path (bf16 or fp16 operands, fp32 accumulation), one kernel templated on the operand type:
//   * workgroup = 8 waves = 256 query rows of one (sequence, head); wave = 32 rows; one
//     workgroup per CU at C2 (grid 8 x 32).
//   * S^T = K . Q^T on v_mfma_f32_32x32x16_{bf16,f16}: the query sits on the lane (column), so a
//     lane owns one query row's running max (row max = in-register max + one permlane32 swap).
//   * lazy running max folded into the MFMA: after the first tile the S^T accumulator starts at
//     -m_run, so the MFMA returns s - m_run; while no row's tile max exceeds m_run by more than
//     THR (log2 units) p = exp2(s - m_run) needs no subtraction and O is never rescaled
//     (P <= 2^THR). A wave that sees a larger jump re-bases: m_run += d, O, l *= 2^-d, s -= d
//     (cdna_hip_programming.md T13; the branch is forced by the spike tests).
//   * row sums on the matrix pipe: l^T += ones . P^T (4 extra MFMAs per tile instead of 32 VALU
//     adds), summed from the same 16-bit P that enters O.
//   * the QK^T chains start from a loop-carried -m_run block (rewritten only on a re-base), and P
//     is produced in four 16-key chunks whose MFMAs are issued between the next chunk's exp2s
//     (sched_group_barrier): on gfx950 only a wave's OWN vector work hides under its MFMAs.
//   * O^T = V^T . P^T: the S^T accumulators, packed to 16 bit, ARE the B operand; V^T comes from
//     the LDS tile with ds_read_b64_tr_b16 (hardware transpose).
//   * K/V tiles of 64 keys by LDS-DMA (global_load_lds) into a 3-deep ring shared by all waves,
//     XOR-swizzled (swz128) so every fragment read is conflict-free.
//   * q carries scale*log2(e) (QKV GEMM epilogue), so scores are in log2 units.
//   * XCD-aware block mapping: all query blocks of a (sequence, head) share one L2.
// fp32 parity path: one thread per query row on the VALU (exact fp32).
//
// Measured alternatives (rounds 1-2: wave priorities, fixed-offset softmax, software-pipelined,
// 4-wave, phase-rotated, SIMD ping-pong, deferred-P.V, mid-tile K prefetch, f32 VALU row sums;
// DESIGN.md §3) were parity-tested and none beat this schedule; they are not in the library.
#include "common.h"
#include "kernels.h"

namespace f5h {

template <int OFF>
F5H_DEV u32x4 lds_b128(uint32_t addr) {  // LDS read hidden from hipcc's waitcnt bookkeeping
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int OFF>
F5H_DEV uint2 lds_tr_b64(uint32_t addr) {  // ds_read_b64_tr_b16: 4 rows x 16 cols -> column per lane
  uint2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// value of lane ^ 32 via v_permlane32_swap (VALU; a __shfl_xor would be an LDS op, and its
// lgkmcnt wait would also drain the hand-counted V^T reads in flight)
F5H_DEV float xor32(float x) {
  const unsigned u = __float_as_uint(x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  // r[0]: lanes 0-31 keep x, lanes 32-63 get x[l-32]; r[1]: lanes 0-31 get x[l+32], 32-63 keep x
  const int hi = (__lane_id() >= 32);
  return __uint_as_float(hi ? r[0] : r[1]);
}

// XCD-aware (query block, sequence*head) of this workgroup. The hardware deals workgroups
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch); giving each XCD a contiguous run
// of logical ids keeps all query blocks of one (sequence, head) on one L2, so its K/V leave
// MALL/HBM once instead of once per XCD (bijective form, cdna_hip_programming.md T1).
F5H_DEV void attn_block(int& qb, int& bh) {
  const int nqb = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int w = blockIdx.x + nqb * blockIdx.y;
  const int xq = nwg >> 3, xr = nwg & 7, xcd = w & 7;
  const int id = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (w >> 3);
  qb = id % nqb;
  bh = id / nqb;
}

template <typename T, bool PRESCALED, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn16_kernel(AttnArgs a) {
  typedef Op16<T> OP;
  typedef typename OP::v8 v8;
  typedef typename OP::v4 v4;
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh x 2 B each)
  constexpr int NS = 3;                 // LDS ring: one tile read while two are in flight
  constexpr int CPW = 512 / (64 * NW);  // 16-B chunks of one K (or V) tile per lane
  constexpr float THR = 8.f;
  static_assert(CPW * 64 * NW == 512, "whole DMA rounds");
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const T* Q = reinterpret_cast<const T*>(a.q) + base;
  const T* K = reinterpret_cast<const T*>(a.k) + base;
  const T* V = reinterpret_cast<const T*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  v8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    // rows past L are clamped (their outputs are never stored)
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(v8, v);
    if constexpr (!PRESCALED) {  // scores in log2 units: fold scale*log2(e) into q
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = from_f32<T>(to_f32(qf[ks][j]) * c);
    }
  }
  // consume Q here: otherwise hipcc waits vmcnt(0) at its first use inside the tile loop, which
  // would also drain the LDS-DMA in flight
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  // ---- LDS-DMA of a K/V tile: chunk p = (r*NW + w)*64 + lane of the 64-row x 8-chunk image
  int dsrc[CPW];
#pragma unroll
  for (int r = 0; r < CPW; ++r) {
    const int p = (r * NW + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dsrc[r] = swz128(row, slot) * 8;  // element offset of the source chunk inside its row
  }
  auto dma = [&](int buf, int kt) {
    uint4* Ks = lds + buf * (TILE_B / 16);
    uint4* Vs = Ks + 512;
#pragma unroll
    for (int r = 0; r < CPW; ++r) {
      const int row = ((r * NW + wid) * 64 + lane) >> 3;
      const int64_t off = (int64_t)min(kt * 64 + row, L - 1) * 64 + dsrc[r];
      __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + (r * NW + wid) * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + (r * NW + wid) * 64), 16, 0, 0);
    }
  };

  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  uint32_t kaddr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int row = lane & 31;
    kaddr[ks] = lds0 + row * 128 + swz128(row, ks * 2 + h) * 16;
  }
  const int G = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  uint32_t vaddr[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g8 = 0; g8 < 2; ++g8) {
      const int r1 = 4 * (G >> 1) + q4 + 8 * g8;
      const int dh = 32 * u + 16 * (G & 1) + 4 * p4;
      vaddr[u][g8] = lds0 + 64 * 128 + r1 * 128 + swz128(r1, dh >> 3) * 16 + ((dh >> 2) & 1) * 8;
    }

  const T one = from_f32<T>(1.f);
  const v8 ones = {one, one, one, one, one, one, one, one};
  float m_run = 0.f;  // running max (log2 units), valid after tile 0
  f32x16 oacc[2], lacc, minit;  // minit: -m_run in every slot, the QK^T chains' first C operand
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
    minit[r] = 0.f;
  }

  dma(0, 0);
  if (ntile > 1) dma(1, 1);
  for (int kt = 0; kt < ntile; ++kt) {
    // tile kt landed for this wave's own DMA (tile kt+1 may stay in flight); the barrier
    // publishes every wave's part of it and retires all reads of slot (kt+2)%3 (= tile kt-1)
    if (kt + 1 < ntile)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);

    u32x4 kf[2][4];
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
    if (kt + 2 < ntile) dma((kt + 2) % NS, kt + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
    __builtin_amdgcn_sched_barrier(0);
    uint2 vf[2][2][2][2];
    auto vread = [&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto TT) {
        constexpr int t = decltype(TT)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    };

    // ---- S^T - m_run = K Q^T + (-m_run): both chains start from minit, which is rewritten only
    // when m_run changes (no per-tile accumulator initialisation)
    f32x16 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sacc[t] = OP::mma32(__builtin_bit_cast(v8, kf[t][0]), qf[0], minit);
#pragma unroll
      for (int ks = 1; ks < 4; ++ks) sacc[t] = OP::mma32(__builtin_bit_cast(v8, kf[t][ks]), qf[ks], sacc[t]);
    }
    vread(std::integral_constant<int, 0>{});
    if (kt * 64 + 64 > klen) {  // ragged last tile: keys past klen get p = 0
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sacc[t][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[t][r]);
    mx = fmaxf(mx, xor32(mx));
    if (kt == 0) {
      // first tile (>= 1 valid key): the running max starts at the tile max
      m_run = mx;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= mx;
#pragma unroll
      for (int r = 0; r < 16; ++r) minit[r] = -m_run;
    } else if (!__all(mx <= THR)) {
      // re-base the rows whose scores ran more than THR above m_run (rare: early tiles)
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] *= alpha;
        oacc[1][r] *= alpha;
        lacc[r] *= alpha;
        minit[r] = -m_run;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= d;
    }
    // exp2 / pack of 16-key chunk c = (t, sx) of P, then its three MFMAs (row sums, both O^T
    // halves), issued between chunk c+1's exp2s and packs: a wave's own VALU work issues in the
    // shadow of its MFMAs (per accumulator the MFMA order is unchanged)
    v8 pf[2][2];
    auto exp_chunk = [&](auto C) {
      constexpr int t = decltype(C)::value >> 1, sx = decltype(C)::value & 1;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[t][sx][j] = from_f32<T>(__builtin_amdgcn_exp2f(sacc[t][8 * sx + j]));
    };
    auto mma_chunk = [&](auto C) {
      constexpr int t = decltype(C)::value >> 1, sx = decltype(C)::value & 1;
      lacc = OP::mma32(ones, pf[t][sx], lacc);  // row sums: l^T += ones . P^T
#pragma unroll
      for (int u = 0; u < 2; ++u) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
        oacc[u] = OP::mma32(__builtin_bit_cast(v8, w), pf[t][sx], oacc[u]);
      }
    };
    vread(std::integral_constant<int, 1>{});
    exp_chunk(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 3>([&](auto C) {
      mma_chunk(C);
      exp_chunk(std::integral_constant<int, decltype(C)::value + 1>{});
      // per MFMA gap: 3, 3, 2 exp2 (TRANS) and 1, 1, 2 packs
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x400, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x400, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x400, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    mma_chunk(std::integral_constant<int, 3>{});
  }
  const float l_tot = lacc[0];
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    T* O = reinterpret_cast<T*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        v4 w = {from_f32<T>(oacc[u][4 * r4 + 0] * inv), from_f32<T>(oacc[u][4 * r4 + 1] * inv),
                from_f32<T>(oacc[u][4 * r4 + 2] * inv), from_f32<T>(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<v4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- one wave per SIMD, two row groups
// attn_pw_kernel: 4 waves x 64 query rows = 256 rows per workgroup, one wave per SIMD. Each wave
// owns two 32-row groups A and B and runs them half a tile apart, so while one group's softmax
// (row max, exp2, pack) is on the VALU the other group's MFMAs keep the matrix pipe busy -- on
// gfx950 only a wave's OWN vector work issues in the shadow of its MFMAs (a SIMD partner's does
// not), so the overlap has to live inside one wave:
//   alpha(kt): MFMA  QK^T(B, kt) | P.V(B, kt-1)     VALU  softmax(A, kt)
//   beta(kt):  MFMA  P.V(A, kt)  | QK^T(A, kt+1)    VALU  softmax(B, kt)
// Per group the arithmetic is attn16_kernel's (operand layouts, -m_run accumulator init, lazy
// re-base, row sums on the matrix pipe, MFMA order per accumulator), so the two are bitwise equal.
//
// Registers: two groups need more than the 256 arch VGPRs, so the MFMA operands and accumulators
// that the VALU never touches live in the accumulator file, owned by this kernel's inline asm:
//   a[0:95]    O^T halves and row sums: a[48g + 16u ...] = O^T half u of group g, a[48g + 32 ...]
//   a[96:127]  Q fragments: a[96 + 16g + 4ks ...]
//   a[128:159] K fragments of the current tile: a[128 + 16t + 4ks ...] (ds_read_b128 into AGPRs)
// The arch VGPRs hold the score blocks, -m_run blocks, packed P and V^T fragments, all
// compiler-managed. hipcc neither counts nor pads inside asm: the LDS reads are counted by hand
// (PW_LGK), every MFMA opens with the 2 wait states of a just-written operand, and score blocks
// are handed to compiler code only after the 16 states an MFMA result needs (pw_sync).
// tools/audit_attn_asm.py checks that no compiler code touches an accumulator register.
#define F5H_A10(b) "a" #b "0", "a" #b "1", "a" #b "2", "a" #b "3", "a" #b "4", "a" #b "5", "a" #b "6", "a" #b "7", \
                   "a" #b "8", "a" #b "9"
#define F5H_A0_159                                                                                          \
  "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", F5H_A10(1), F5H_A10(2), F5H_A10(3), F5H_A10(4), \
      F5H_A10(5), F5H_A10(6), F5H_A10(7), F5H_A10(8), F5H_A10(9), F5H_A10(10), F5H_A10(11), F5H_A10(12),      \
      F5H_A10(13), F5H_A10(14), F5H_A10(15)

// a[ACC:ACC+15] += A . B, A = arch VGPRs, B = arch VGPRs (P.V and row sums). PAD: open with the
// 2 wait states of a just-written A/B operand -- needed wherever hipcc may materialise an operand
// right before the statement (V^T fragments are assembled by moves, the all-ones row-sum operand
// is rematerialised from SGPRs under register pressure)
template <typename T, int ACC, bool PAD>
F5H_DEV void pw_pv(const typename Op16<T>::v8& A, const typename Op16<T>::v8& B) {
  if constexpr (PAD) {
    if constexpr (std::is_same<T, bf16>::value)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(A), "v"(B),
                   "i"(ACC), "i"(ACC + 15));
    else
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(A), "v"(B),
                   "i"(ACC), "i"(ACC + 15));
  } else {
    if constexpr (std::is_same<T, bf16>::value)
      asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(A), "v"(B), "i"(ACC),
                   "i"(ACC + 15));
    else
      asm volatile("v_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(A), "v"(B), "i"(ACC),
                   "i"(ACC + 15));
  }
}
// d = K . Q^T + c (first k-step of a score chain), K = a[KA:KA+3], Q = a[QA:QA+3]
template <typename T, int KA, int QA>
F5H_DEV void pw_qk_first(f32x16& d, const f32x16& c) {
  if constexpr (std::is_same<T, bf16>::value)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, a[%c2:%c3], a[%c4:%c5], %1"
                 : "=&v"(d)
                 : "v"(c), "i"(KA), "i"(KA + 3), "i"(QA), "i"(QA + 3));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, a[%c2:%c3], a[%c4:%c5], %1"
                 : "=&v"(d)
                 : "v"(c), "i"(KA), "i"(KA + 3), "i"(QA), "i"(QA + 3));
}
template <typename T, int KA, int QA>
F5H_DEV void pw_qk_next(f32x16& d) {
  if constexpr (std::is_same<T, bf16>::value)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                 : "+v"(d)
                 : "i"(KA), "i"(KA + 3), "i"(QA), "i"(QA + 3));
  else
    asm volatile("v_mfma_f32_32x32x16_f16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                 : "+v"(d)
                 : "i"(KA), "i"(KA + 3), "i"(QA), "i"(QA + 3));
}
// K fragment (16 B per lane) from LDS straight into a[R:R+3]
template <int R, int OFF>
F5H_DEV void pw_kread(uint32_t addr) {
  asm volatile("ds_read_b128 a[%c1:%c2], %0 offset:%c3" ::"v"(addr), "i"(R), "i"(R + 3), "i"(OFF));
}
// four 32-bit values into a[R:R+3] (Q fragments, once per workgroup)
template <int R>
F5H_DEV void pw_awrite4(uint4 v) {
  asm volatile(
      "v_accvgpr_write_b32 a%c4, %0\n\tv_accvgpr_write_b32 a%c5, %1\n\t"
      "v_accvgpr_write_b32 a%c6, %2\n\tv_accvgpr_write_b32 a%c7, %3" ::"v"(v.x),
      "v"(v.y), "v"(v.z), "v"(v.w), "i"(R), "i"(R + 1), "i"(R + 2), "i"(R + 3));
}
// a0..a95 = 0; the clobber list makes the kernel descriptor allocate a0..a159
F5H_DEV void pw_acc_zero() {
  asm volatile(
      ".irp r, 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31,32,33,34,35,"
      "36,37,38,39,40,41,42,43,44,45,46,47,48,49,50,51,52,53,54,55,56,57,58,59,60,61,62,63,64,65,66,67,68,69,70,"
      "71,72,73,74,75,76,77,78,79,80,81,82,83,84,85,86,87,88,89,90,91,92,93,94,95\n\t"
      "v_accvgpr_write_b32 a\\r, 0\n\t.endr" ::: F5H_A0_159);
}
// a[BASE .. BASE+47] *= s (one group's O^T halves and row sums: the lazy re-base)
template <int BASE>
F5H_DEV void pw_acc_scale(float s) {
  float tmp;
  asm volatile(
      "s_nop 7\n\ts_nop 7\n\t"
      ".irp r, 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31,32,33,34,35,"
      "36,37,38,39,40,41,42,43,44,45,46,47\n\t"
      "v_accvgpr_read_b32 %0, a[%c2+\\r]\n\tv_mul_f32 %0, %1, %0\n\tv_accvgpr_write_b32 a[%c2+\\r], %0\n\t"
      ".endr"
      : "=&v"(tmp)
      : "v"(s), "i"(BASE));
}
F5H_DEV float pw_max3(float x, float y, float z) {
  float r;
  asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
template <int R>
F5H_DEV float pw_aread() {  // caller has waited the 16 states after the last MFMA into a[R]
  float x;
  asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(R));
  return x;
}

template <typename T, bool PRESCALED>
__global__ __launch_bounds__(256, 1) void attn_pw_kernel(AttnArgs a) {
  typedef Op16<T> OP;
  typedef typename OP::v8 v8;
  typedef typename OP::v4 v4;
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int NW = 4;
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes
  constexpr int NS = 4;                 // ring: tiles kt-1 (V), kt, kt+1 read; kt+2 in flight
  constexpr int CPW = 512 / (64 * NW);  // 16-B chunks of one K (or V) tile per lane
  constexpr float THR = 8.f;
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const T* Q = reinterpret_cast<const T*>(a.q) + base;
  const T* K = reinterpret_cast<const T*>(a.k) + base;
  const T* V = reinterpret_cast<const T*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  pw_acc_zero();
  int qrow[2];
  static_for<0, 2>([&](auto GG) {
    constexpr int g = decltype(GG)::value;
    qrow[g] = qb * 256 + wid * 64 + g * 32 + (lane & 31);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow[g], L - 1) * 64 + ks * 16 + h * 8);
      if constexpr (!PRESCALED) {
        const float c = a.scale * 1.4426950408889634f;
        v8 q = __builtin_bit_cast(v8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = from_f32<T>(to_f32(q[j]) * c);
        v = __builtin_bit_cast(uint4, q);
      }
      pw_awrite4<96 + 16 * g + 4 * ks>(v);
    });
  });

  int dsrc[CPW];
#pragma unroll
  for (int r = 0; r < CPW; ++r) {
    const int p = (r * NW + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dsrc[r] = swz128(row, slot) * 8;
  }
  // K/V tiles are staged through registers: piece j (0..3: K or V of chunk round j/2) of a tile is
  // one 16-B global load per lane into stg[j] and, a tile later, one ds_write_b128 into the ring
  // slot. (An LDS-DMA piece costs a wave 100+ issue cycles; these two instructions a few tens.)
  // Tiles past the end are clamped re-loads into a dead slot, so every tile moves the same pieces.
  u32x4 stg[2 * CPW];  // (a native vector: HIP's uint4 struct defeats SROA here and lands in scratch)
  auto gload = [&](int kt, auto J) {
    constexpr int j = decltype(J)::value, r = j >> 1;
    const int row = ((r * NW + wid) * 64 + lane) >> 3;
    const int64_t off = (int64_t)min(kt * 64 + row, L - 1) * 64 + dsrc[r];
    stg[j] = *reinterpret_cast<const u32x4*>(((j & 1) ? V : K) + off);
  };
  auto swrite = [&](int kt, auto J) {
    constexpr int j = decltype(J)::value, r = j >> 1;
    reinterpret_cast<u32x4*>(lds)[(kt % NS) * (TILE_B / 16) + (j & 1) * 512 + (r * NW + wid) * 64 + lane] = stg[j];
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  uint32_t kaddr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int row = lane & 31;
    kaddr[ks] = lds0 + row * 128 + swz128(row, ks * 2 + h) * 16;
  }
  const int G = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  uint32_t vaddr[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g8 = 0; g8 < 2; ++g8) {
      const int r1 = 4 * (G >> 1) + q4 + 8 * g8;
      const int dh = 32 * u + 16 * (G & 1) + 4 * p4;
      vaddr[u][g8] = lds0 + 64 * 128 + r1 * 128 + swz128(r1, dh >> 3) * 16 + ((dh >> 2) & 1) * 8;
    }

  const T one = from_f32<T>(1.f);
  const v8 ones = {one, one, one, one, one, one, one, one};
  float m_run[2] = {0.f, 0.f};
  f32x16 minit[2], sacc[2][2];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int r = 0; r < 16; ++r) minit[g][r] = 0.f;
  uint2 vf[4][2][2];  // V^T fragments of 16-key chunk c: [c][O^T half u][row group]
  v8 pf[2][2][2];

  // LDS reads (inline asm: hidden from hipcc's waitcnt bookkeeping, which would otherwise also
  // drain the LDS-DMA in flight), counted by hand: PW_LGK(n) waits until n are outstanding;
  // PW_VDONE(c) then tells hipcc chunk c's V^T registers are defined.
  auto kread_half = [&](uint32_t so, auto TT) {  // K rows 32t .. 32t+31 into a[128 + 16t ...]: 4 reads
    constexpr int t = decltype(TT)::value;
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      pw_kread<128 + 16 * t + 4 * ks, 4096 * t>(kaddr[ks] + so);
    });
  };
  auto vread = [&](uint32_t so, auto C) {  // 4 reads
    constexpr int c = decltype(C)::value, t = c >> 1, sx = c & 1;
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      vf[c][u][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
      vf[c][u][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
    });
  };
#define PW_LGK(n) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(n) : "memory")
#define PW_VDONE(c) \
  asm volatile("" : "+v"(vf[c][0][0]), "+v"(vf[c][0][1]), "+v"(vf[c][1][0]), "+v"(vf[c][1][1]))
  // score blocks of group g handed to compiler code after the 12 wait states an (8-pass) MFMA
  // result needs (PW_SYNC), or as a plain hand-over where more than 12 instructions have issued
  // since the last MFMA into them (PW_TAKE)
#define PW_SYNC(g) asm volatile("s_nop 7\n\ts_nop 3" : "+v"(sacc[g][0]), "+v"(sacc[g][1]))
#define PW_TAKE(g) asm volatile("" : "+v"(sacc[g][0]), "+v"(sacc[g][1]))
#define PW_FENCE __builtin_amdgcn_sched_barrier(0)
#ifdef F5H_PW_STAMPS  // diagnostic build: per-phase shader-clock stamps of tile 12 (written over O)
  unsigned long long stamp[8] = {};
#define PW_STAMP(i)                                                                                  \
  if (kt == 12) {                                                                                    \
    PW_FENCE;                                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp[i])::"memory");                \
    PW_FENCE;                                                                                        \
  }
#else
#define PW_STAMP(i)
#endif

  // QK^T MFMA (t, ks) of group g: S^T - m_run = K Q^T + (-m_run), chains t = 0, 1
  auto qk_one = [&](auto GG, auto KS, auto TT) {
    constexpr int g = decltype(GG)::value, ks = decltype(KS)::value, t = decltype(TT)::value;
    if constexpr (ks == 0)
      pw_qk_first<T, 128 + 16 * t, 96 + 16 * g>(sacc[g][t], minit[g]);
    else
      pw_qk_next<T, 128 + 16 * t + 4 * ks, 96 + 16 * g + 4 * ks>(sacc[g][t]);
  };
  auto qk_all = [&](auto GG) {
    static_for<0, 8>([&](auto I) {
      qk_one(GG, std::integral_constant<int, decltype(I)::value / 2>{}, std::integral_constant<int, decltype(I)::value % 2>{});
    });
  };
  // one P.V MFMA of 16-key chunk c = (t, sx): i = 0 row sums, i = 1, 2 the two O^T halves
  auto pv_one = [&](auto GG, auto C, auto I) {
    constexpr int g = decltype(GG)::value;
    constexpr int c = decltype(C)::value, t = c >> 1, sx = c & 1, i = decltype(I)::value;
    if constexpr (i == 0) {
      pw_pv<T, 48 * g + 32, true>(ones, pf[g][t][sx]);
    } else {
      constexpr int u = i - 1;
      const uint4 w = make_uint4(vf[c][u][0].x, vf[c][u][0].y, vf[c][u][1].x, vf[c][u][1].y);
      pw_pv<T, 48 * g + 16 * u, true>(__builtin_bit_cast(v8, w), pf[g][t][sx]);
    }
  };
  auto smask = [&](auto GG, int kt) {  // ragged last tile: keys past klen get p = 0
    constexpr int g = decltype(GG)::value;
    if (kt * 64 + 64 > klen) {
      int lim = klen - kt * 64 - 4 * h;  // keys at offset >= lim inside the tile are padding
      // opaque here: otherwise hipcc hoists the 32 compares out of this rare branch into every tile
      asm volatile("; ragged tile" : "+v"(lim));
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (t * 32 + (r & 3) + 8 * (r >> 2) >= lim) sacc[g][t][r] = -INFINITY;
    }
  };
  // row max of group g in 8 pieces (rows 2k, 2k+1 of both score blocks); piece 7 finishes it.
  // v_max3 in asm: on asm outputs hipcc would canonicalise every operand of an fmaxf first
  auto smax_part = [&](auto GG, auto KK, float& m0, float& m1) {
    constexpr int g = decltype(GG)::value, k = decltype(KK)::value;
    if constexpr (k == 0) {
      m0 = pw_max3(sacc[g][0][0], sacc[g][0][1], sacc[g][0][1]);
      m1 = pw_max3(sacc[g][1][0], sacc[g][1][1], sacc[g][1][1]);
    } else {
      m0 = pw_max3(m0, sacc[g][0][2 * k], sacc[g][0][2 * k + 1]);
      m1 = pw_max3(m1, sacc[g][1][2 * k], sacc[g][1][2 * k + 1]);
    }
    if constexpr (k == 7) {
      m0 = pw_max3(m0, m1, m1);
      m0 = pw_max3(m0, xor32(m0), m0);
    }
  };
  auto srebase = [&](auto GG, auto FIRST, float mx) {
    constexpr int g = decltype(GG)::value;
    if constexpr (decltype(FIRST)::value) {
      m_run[g] = mx;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[g][t][r] -= mx;
#pragma unroll
      for (int r = 0; r < 16; ++r) minit[g][r] = -m_run[g];
    } else if (!__all(mx <= THR)) {
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run[g] += d;
      pw_acc_scale<48 * g>(alpha);
#pragma unroll
      for (int r = 0; r < 16; ++r) minit[g][r] -= d;  // == -m_run, in place
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[g][t][r] -= d;
    }
  };
  // p = exp2(s - m_run) of chunk c, elements [J0, J1), and the 16-bit packs of pairs [P0, P1)
  float ex[2][4][8];
  auto sexp = [&](auto GG, auto C, auto J0, auto J1) {
    constexpr int g = decltype(GG)::value;
    constexpr int c = decltype(C)::value, t = c >> 1, sx = c & 1;
    static_for<decltype(J0)::value, decltype(J1)::value>([&](auto J) {
      constexpr int j = decltype(J)::value;
      ex[g][c][j] = __builtin_amdgcn_exp2f(sacc[g][t][8 * sx + j]);
    });
  };
  auto spack = [&](auto GG, auto C, auto P0, auto P1) {
    constexpr int g = decltype(GG)::value;
    constexpr int c = decltype(C)::value, t = c >> 1, sx = c & 1;
    static_for<decltype(P0)::value, decltype(P1)::value>([&](auto P) {
      constexpr int p = decltype(P)::value;
      pf[g][t][sx][2 * p] = from_f32<T>(ex[g][c][2 * p]);
      pf[g][t][sx][2 * p + 1] = from_f32<T>(ex[g][c][2 * p + 1]);
    });
    // pin the exp2s and packs to this point (hipcc would otherwise sink them to the consumer)
    asm volatile("" : "+v"(pf[g][t][sx]));
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I6 = std::integral_constant<int, 6>;
  using I8 = std::integral_constant<int, 8>;
  // the three MFMAs of P.V chunk C of group GP with the exp2s / packs of chunk CE of group GE in
  // their shadows (3 + 3 + 2 exp2, 0 + 1 + 3 packs)
  auto pv_chunk_exp = [&](auto GP, auto C, auto GE, auto CE) {
    pv_one(GP, C, I0{});
    sexp(GE, CE, I0{}, I3{});
    PW_FENCE;
    pv_one(GP, C, I1{});
    sexp(GE, CE, I3{}, I6{});
    spack(GE, CE, I0{}, I1{});
    PW_FENCE;
    pv_one(GP, C, I2{});
    sexp(GE, CE, I6{}, I8{});
    spack(GE, CE, I1{}, I4{});
    PW_FENCE;
  };

  // ---- prologue: tiles 0..2 in flight, K(0) resident, QK^T(A, 0)
  for (int t = 0; t < 3; ++t) {
    static_for<0, 2 * CPW>([&](auto J) { gload(t, J); });
    static_for<0, 2 * CPW>([&](auto J) { swrite(t, J); });
  }
  static_for<0, 2 * CPW>([&](auto J) { gload(3, J); });  // written at the end of beta(0)
  __syncthreads();
  kread_half(0u, I0{});
  kread_half(0u, I1{});
  PW_LGK(0);
  PW_FENCE;
  qk_all(I0{});

  // One tile: alpha(kt) then beta(kt). K(kt) is resident in a[128:159] from beta(kt-1) (both
  // groups' QK^T use it) and V(kt)'s fragments stay in vf from alpha(kt) through alpha(kt+1) (both
  // groups' P.V use them): per tile a wave reads each K and V fragment once. The first tile is
  // peeled (it sets the running max and has no P.V(B, kt-1)).
  auto tile = [&](int kt, auto FIRST) {
    constexpr bool first = decltype(FIRST)::value;
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    const uint32_t sn = kt + 1 < ntile ? (uint32_t)(((kt + 1) % NS) * TILE_B) : so;
    // ---- alpha(kt): MFMA QK^T(B, kt), P.V(B, kt-1) | VALU softmax(A, kt); no LDS wait
    PW_STAMP(0);
    PW_SYNC(0);
    smask(I0{}, kt);
    PW_FENCE;
    float m0, m1;
    static_for<0, 8>([&](auto I) {
      qk_one(I1{}, std::integral_constant<int, decltype(I)::value / 2>{}, std::integral_constant<int, decltype(I)::value % 2>{});
      smax_part(I0{}, I, m0, m1);
      PW_FENCE;
    });
    PW_STAMP(1);
    srebase(I0{}, FIRST, m0);
    PW_FENCE;
    // chunk c of P.V(B, kt-1) (V(kt-1) in vf[c]) with exp2s of A; then V(kt)'s chunk c into vf[c]
    // (chunks 0-2 here, 3 in beta: at most 15 LDS reads in flight)
    static_for<0, 4>([&](auto C) {
      if constexpr (!first) {
        pv_chunk_exp(I1{}, C, I0{}, C);
      } else {
        sexp(I0{}, C, I0{}, I8{});
        spack(I0{}, C, I0{}, I4{});
      }
      if constexpr (decltype(C)::value < 3) vread(so, C);
      PW_FENCE;
    });

    // ---- beta(kt): MFMA P.V(A, kt), QK^T(A, kt+1) | VALU softmax(B, kt)
    // the barrier publishes tile kt+1 (written at the end of beta(kt-2), lgkmcnt(0) since) and
    // retires every wave's reads of tile kt-1, whose slot tile kt+3 is written at this beta's end
    PW_STAMP(2);
    __builtin_amdgcn_s_barrier();
    PW_STAMP(3);
    PW_TAKE(1);  // QK^T(B) issued before alpha's 12 P.V MFMAs
    smask(I1{}, kt);
    // LDS reads outstanding: V c0 c1 c2
    PW_LGK(8);
    PW_VDONE(0);
    vread(so, I3{});  // c1 c2 c3
    PW_FENCE;
    // P.V(A) chunks 0-1 with the row max of B in their shadows (2, 2, 1, 1, 1, 1 pieces)
    pv_one(I0{}, I0{}, I0{});
    smax_part(I1{}, I0{}, m0, m1);
    smax_part(I1{}, I1{}, m0, m1);
    PW_FENCE;
    pv_one(I0{}, I0{}, I1{});
    smax_part(I1{}, I2{}, m0, m1);
    smax_part(I1{}, I3{}, m0, m1);
    PW_FENCE;
    pv_one(I0{}, I0{}, I2{});
    smax_part(I1{}, I4{}, m0, m1);
    PW_LGK(8);
    PW_VDONE(1);
    kread_half(sn, I0{});  // c2 c3 K0 (a[128:143]: QK^T(B, kt) has issued)
    PW_FENCE;
    pv_one(I0{}, I1{}, I0{});
    smax_part(I1{}, std::integral_constant<int, 5>{}, m0, m1);
    PW_FENCE;
    pv_one(I0{}, I1{}, I1{});
    smax_part(I1{}, I6{}, m0, m1);
    PW_FENCE;
    pv_one(I0{}, I1{}, I2{});
    smax_part(I1{}, std::integral_constant<int, 7>{}, m0, m1);
    PW_FENCE;
    PW_STAMP(4);
    srebase(I1{}, FIRST, m0);
    PW_FENCE;
    PW_LGK(8);
    PW_VDONE(2);
    kread_half(sn, I1{});  // c3 K0 K1
    pv_chunk_exp(I0{}, I2{}, I1{}, I0{});
    PW_STAMP(5);
    PW_LGK(8);
    PW_VDONE(3);
    pv_chunk_exp(I0{}, I3{}, I1{}, I1{});
    PW_STAMP(6);
    // tile kt+3 (loaded during beta(kt-1)) into the slot of tile kt-1
    static_for<0, 2 * CPW>([&](auto J) { swrite(kt + 3, J); });
    // QK^T(A, kt+1) with B's last exp2s and the loads of tile kt+4. On the last tile this runs on
    // K(kt) into scores nobody reads: no branch, so hipcc keeps B's exp2s in the MFMA shadows.
    PW_LGK(0);
    PW_FENCE;
    static_for<0, 8>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 2 * CPW) gload(kt + 4, I);
      qk_one(I0{}, std::integral_constant<int, i / 2>{}, std::integral_constant<int, i % 2>{});
      sexp(I1{}, std::integral_constant<int, 2 + i / 4>{}, std::integral_constant<int, 2 * (i % 4)>{},
           std::integral_constant<int, 2 * (i % 4) + 2>{});
      spack(I1{}, std::integral_constant<int, 2 + i / 4>{}, std::integral_constant<int, i % 4>{},
            std::integral_constant<int, i % 4 + 1>{});
      PW_FENCE;
    });
    PW_STAMP(7);
  };
  tile(0, std::true_type{});
  for (int kt = 1; kt < ntile; ++kt) tile(kt, std::false_type{});

  // ---- epilogue: P.V(B, last tile) on the resident V fragments
  PW_FENCE;
  static_for<0, 4>([&](auto C) {
    pv_one(I1{}, C, I0{});
    pv_one(I1{}, C, I1{});
    pv_one(I1{}, C, I2{});
  });
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // MFMA results -> v_accvgpr_read
#undef PW_FENCE
#undef PW_LGK
#undef PW_VDONE
#undef PW_SYNC
#undef PW_TAKE
#undef PW_STAMP

  static_for<0, 2>([&](auto GG) {
    constexpr int g = decltype(GG)::value;
    float o[2][16];
    static_for<0, 16>([&](auto R) {
      constexpr int r = decltype(R)::value;
      o[0][r] = pw_aread<48 * g + r>();
      o[1][r] = pw_aread<48 * g + 16 + r>();
    });
    const float l_tot = pw_aread<48 * g + 32>();
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (qrow[g] < L) {
      T* O = reinterpret_cast<T*>(a.o) + (((int64_t)s_idx * L + qrow[g]) * a.H + head) * 64;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          v4 w = {from_f32<T>(o[u][4 * r4 + 0] * inv), from_f32<T>(o[u][4 * r4 + 1] * inv),
                  from_f32<T>(o[u][4 * r4 + 2] * inv), from_f32<T>(o[u][4 * r4 + 3] * inv)};
          *reinterpret_cast<v4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
        }
    }
  });
#ifdef F5H_PW_STAMPS
  if (lane == 0) {
    // u16 deltas from stamp 0: finite 16-bit floats while < 0x7F80, so they survive the
    // op-level conversion back to fp32
    uint16_t* d = reinterpret_cast<uint16_t*>(a.o) + ((blockIdx.y * gridDim.x + blockIdx.x) * 4 + wid) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = (uint16_t)min(stamp[i] - stamp[0], 0x7F00ull);
  }
#endif
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- fp32 parity kernel
__global__ __launch_bounds__(64) void attn_f32_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  __shared__ float Ks[32][65];
  __shared__ float Vs[32][64];
  const int lane = threadIdx.x;
  const int bh = blockIdx.y;
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const float* Q = reinterpret_cast<const float*>(a.q) + base;
  const float* K = reinterpret_cast<const float*>(a.k) + base;
  const float* V = reinterpret_cast<const float*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int qrow = blockIdx.x * 64 + lane;
  float q[64], o[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) {
    q[d] = qrow < L ? Q[(int64_t)qrow * 64 + d] : 0.f;
    o[d] = 0.f;
  }
  float m_run = -INFINITY, l_run = 0.f;
  for (int k0 = 0; k0 < klen; k0 += 32) {
    __syncthreads();
    for (int i = lane; i < 32 * 64; i += 64) {
      int r = i >> 6, d = i & 63, key = k0 + r;
      Ks[r][d] = key < klen ? K[(int64_t)key * 64 + d] : 0.f;
      Vs[r][d] = key < klen ? V[(int64_t)key * 64 + d] : 0.f;
    }
    __syncthreads();
    float sc[32];
    float mx = m_run;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) acc = fmaf(q[d], Ks[r][d], acc);
      sc[r] = (k0 + r < klen) ? (a.prescaled ? acc : acc * a.scale) : -INFINITY;
      mx = fmaxf(mx, sc[r]);
    }
    const float alpha = a.prescaled ? exp2f(m_run - mx) : expf(m_run - mx);
    m_run = mx;
    l_run *= alpha;
#pragma unroll
    for (int d = 0; d < 64; ++d) o[d] *= alpha;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      float p = a.prescaled ? exp2f(sc[r] - mx) : expf(sc[r] - mx);
      l_run += p;
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] = fmaf(p, Vs[r][d], o[d]);
    }
  }
  if (qrow < L) {
    float* O = reinterpret_cast<float*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
    const float inv = 1.f / l_run;
#pragma unroll
    for (int d = 0; d < 64; ++d) O[d] = o[d] * inv;
  }
  probe_exit(a.probe, probe_t);
}

template <typename T>
static void launch16(const AttnArgs& a, hipStream_t st) {
  static const int variant = [] {
    const char* e = getenv("F5H_ATTN");
    return e ? atoi(e) : 0;
  }();
  if (variant == 1) {
    dim3 grid((a.L + 255) / 256, a.S * a.H);
    if (a.prescaled)
      hipLaunchKernelGGL((attn_pw_kernel<T, true>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((attn_pw_kernel<T, false>), grid, dim3(256), 0, st, a);
    return;
  }
  constexpr int NW = 8;
  dim3 grid((a.L + 32 * NW - 1) / (32 * NW), a.S * a.H);
  if (a.prescaled)
    hipLaunchKernelGGL((attn16_kernel<T, true, NW>), grid, dim3(64 * NW), 0, st, a);
  else
    hipLaunchKernelGGL((attn16_kernel<T, false, NW>), grid, dim3(64 * NW), 0, st, a);
}

hipError_t attention(int compute, const AttnArgs& a, hipStream_t st) {
  if (a.S <= 0 || a.H <= 0 || a.L <= 0) return hipErrorInvalidValue;
  switch (compute) {
    case F5H_C_BF16: launch16<bf16>(a, st); break;
    case F5H_C_FP16: launch16<f16>(a, st); break;
    default: {
      dim3 grid((a.L + 63) / 64, a.S * a.H);
      hipLaunchKernelGGL(attn_f32_kernel, grid, dim3(64), 0, st, a);
    }
  }
  return hipGetLastError();
}

}  // namespace f5h
