// Non-causal multi-head attention, head_dim 64 (AttnProcessor, modules.py:511-520):
// O = softmax(Q K^T * scale [+ key-padding mask]) V, flash-style (scores never materialised).
//
// 16-bit path (bf16 or fp16 operands, fp32 accumulation), one kernel templated on the operand type:
//   * workgroup = 8 waves = 256 query rows of one (sequence, head); wave = 32 rows; one
//     workgroup per CU at C2 (grid 8 x 32).
//   * S^T = K . Q^T on v_mfma_f32_32x32x16_{bf16,f16}: the query sits on the lane (column), so a
//     lane owns one query row's running max (row max = in-register max + one permlane32 swap).
//   * running max folded into the MFMA, set once: after the first tile the S^T accumulator starts at
//     -m_run (m_run = the row's first-tile max), so the MFMA returns s - m_run and p = exp2(s - m_run)
//     needs no subtraction. Later tiles take no row max at all (round 5): P may exceed 1, which the fp32
//     O / l accumulators and the 16-bit P hold at full relative precision as long as P stays finite in the
//     operand type; after the loop every row checks l <= 2^64 (bf16) / 2^15 (fp16), which bounds every P,
//     and a workgroup with a failing row (a score more than that far above its first-tile max) reruns its
//     key loop in the lazy-max form of cdna_hip_programming.md T13 (per-tile max, re-base past 2^8; forced
//     by the spike tests and by f5h_attn_force_safe).
//   * row sums on the VALU from the fp32 exp2s: 16 packed adds per tile and wave, issued in the
//     MFMA shadow with the packs (the matrix-pipe form l^T += ones . P^T cost 4 of 20 MFMAs per tile).
//   * the QK^T chains start from a loop-carried -m_run block (rewritten only on a re-base), and P
//     is produced in four 16-key chunks whose MFMAs are issued between the next chunk's exp2s
//     (sched_group_barrier): on gfx950 only a wave's OWN vector work hides under its MFMAs.
//   * O^T = V^T . P^T: the S^T accumulators, packed to 16 bit, ARE the B operand; V^T comes from
//     the LDS tile with ds_read_b64_tr_b16 (hardware transpose).
//   * K/V tiles of 64 keys by LDS-DMA (global_load_lds) into a 4-deep ring shared by all waves,
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

#include <cstdlib>
#include <cstring>

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

// RSM: row sums on the matrix pipe (l^T += ones . P^T, one 32x32x16 MFMA per 16-key chunk) instead of 16 packed
// VALU adds per tile (F5H_ATTN_ROWSUM=mfma; an A/B switch, results agree to rounding)
template <typename T, bool PRESCALED, int NW, bool RSM>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn16_kernel(AttnArgs a) {
  typedef Op16<T> OP;
  typedef typename OP::v8 v8;
  typedef typename OP::v4 v4;
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh x 2 B each)
  constexpr int NS = 4;                 // LDS ring: one tile read while three are in flight
  constexpr int CPW = 512 / (64 * NW);  // 16-B chunks of one K (or V) tile per lane
  constexpr float THR = 8.f;
  static_assert(CPW * 64 * NW == 512, "whole DMA rounds");
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  // with the pad skip, dead query blocks cluster by sequence length: deal the (sequence, head) pairs over
  // the XCDs round-robin so every XCD holds a share of every length (all blocks of a pair stay on one XCD)
  if (a.q_len) bh = spread8(bh, gridDim.y);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  if (a.q_len && qb * (32 * NW) >= a.q_len[s_idx]) {  // dead query block (pad rows only): nothing to write
    probe_exit(a.probe, probe_t);
    return;
  }
  const int64_t base = (int64_t)bh * L * 64;
  const T* Q = reinterpret_cast<const T*>(a.q) + base;
  const T* K = reinterpret_cast<const T*>(a.k) + base;
  const T* V = reinterpret_cast<const T*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);

  // ---- LDS-DMA of a K/V tile: chunk p = (r*NW + w)*64 + lane of the 64-row x 8-chunk image, by
  // buffer_load ... lds: the lane's byte offset in the tile is fixed (voffset), the LDS destination a scalar
  // (M0), so a tile's DMA costs no vector instructions. Each tile gets its own descriptor (scalar base at the
  // tile's first key, extent = the tile's keys below L): the range check then covers every row past L from
  // voffset alone, whatever the hardware does with soffset (an extent over the whole [L,64] panel with the tile
  // offset in soffset would let the ragged last tile read the next (sequence, head)'s rows, or past V). Rows
  // past L read as zero; their keys are masked and their P is 0, so no stale NaN can reach the P.V MFMA.
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  uint32_t dvoff[CPW];
#pragma unroll
  for (int r = 0; r < CPW; ++r) {
    const int p = (r * NW + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dvoff[r] = (uint32_t)(row * 128 + swz128(row, slot) * 16);  // bytes: row, swizzled source chunk
  }
  // live: kt < ntile (so kt*64 < L); otherwise the tile may lie wholly past L (the prologue's tiles 1 and 2)
  auto dma = [&](int buf, int kt, bool live = false) {
    uint4* Ks = lds + buf * (TILE_B / 16);
    uint4* Vs = Ks + 512;
    // wave-uniform by construction; readfirstlane makes it provably so (else the descriptor sits in VGPRs and
    // hipcc wraps every DMA piece in a waterfall loop, cdna_hip_programming.md T20)
    const int rows = live ? min(64, L - kt * 64) : max(0, min(64, L - kt * 64));
    const uint32_t ext = (uint32_t)__builtin_amdgcn_readfirstlane(rows * 128);
    const __amdgpu_buffer_rsrc_t krs = rsrc_of(K + (int64_t)kt * 4096, ext);
    const __amdgpu_buffer_rsrc_t vrs = rsrc_of(V + (int64_t)kt * 4096, ext);
#pragma unroll
    for (int r = 0; r < CPW; ++r) {
      dma16(krs, (LDS_PTR(void))(Ks + (r * NW + wid_s) * 64), dvoff[r], 0);
      dma16(vrs, (LDS_PTR(void))(Vs + (r * NW + wid_s) * 64), dvoff[r], 0);
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

  typedef float f2 __attribute__((ext_vector_type(2)));
  float m_run = 0.f;  // running max (log2 units), valid after tile 0
  f32x16 oacc[2], minit;  // minit: -m_run in every slot, the QK^T chains' first C operand
  f2 lrow = {0.f, 0.f};   // this lane's part of its query's row sum (packed fp32 adds)
  f32x16 lacc;            // RSM: the row sums on the matrix pipe (every slot of a lane holds its query's sum)
#pragma unroll
  for (int r = 0; r < 16; ++r) lacc[r] = 0.f;
  v8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = from_f32<T>(1.f);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    minit[r] = 0.f;
  }

  // Tile 0's K/V, then Q, then tiles 1 and 2: one counted wait covers tile 0 and Q together (in
  // order), so Q's latency overlaps tile 0's instead of preceding it. Q is loaded by inline asm (hipcc
  // would wait vmcnt(0), draining tiles 1 and 2, before its first use) and released by the wait below.
  // Tiles 1 and 2 are issued even past the end of short rows (clamped rows into unused ring slots; the
  // last tile's vmcnt(0) drains them) so that the count of loads behind Q is fixed.
  dma(0, 0);
  u32x4 q0, q1, q2, q3;
  {
    // rows past L are clamped (their outputs are never stored)
    const T* qp = Q + (int64_t)min(qrow, L - 1) * 64 + h * 8;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(q0) : "v"(qp) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(q1) : "v"(qp) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(q2) : "v"(qp) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(q3) : "v"(qp) : "memory");
  }
  dma(1, 1);
  dma(2, 2);
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "i"(4 * CPW) : "memory");
  const u32x4 qv[4] = {q0, q1, q2, q3};
  v8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = __builtin_bit_cast(v8, qv[ks]);
    if constexpr (!PRESCALED) {  // scores in log2 units: fold scale*log2(e) into q
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = from_f32<T>(to_f32(qf[ks][j]) * c);
    }
  }
  // per-wave dead rows (batch path pad skip, q_len): a wave whose 32 query rows all lie past q_len keeps its
  // share of the K/V DMA and the barriers (the ring is shared by the workgroup) but computes and stores
  // nothing, so its SIMD partner issues alone (waves w and w + 4 share a SIMD; the dead rows are the last ones)
  const bool wave_dead = a.q_len && (qb * (32 * NW) + wid_s * 32) >= a.q_len[s_idx];
  constexpr float LMAX = std::is_same<T, f16>::value ? 32768.f : 0x1p64f;  // fp16 P must stay below 65504

  // One K/V tile. FIRST (tile 0): the running max m_run starts at the tile's row max. Later tiles are
  // exponentiated against m_run as it stands (no per-tile row max, no re-base test: 16 v_max3, a permlane
  // and the vote per tile and wave are gone): P = 2^(s - m_run) may exceed 1, which the fp32 O and l
  // accumulators and the 16-bit P carry exactly as well (relative precision does not depend on magnitude),
  // as long as P stays finite in the operand type -- checked once per row after the loop (l <= LMAX bounds
  // every P). SAFE (the rerun of a workgroup where a row failed that check, i.e. some score ran more than
  // log2(LMAX) above its row's first-tile max): the lazy running max of cdna_hip_programming.md T13 -- per
  // tile row max, re-base when it exceeds m_run by more than THR.
  f32x16 sacc[2];  // S^T - m_run of the tile between its two halves
  // tile kt landed for this wave's own DMA (tile kt+1 may stay in flight); the barrier publishes every wave's
  // part of it and retires all reads of slot (kt+3)%NS (= tile kt-1).
  auto tile_wait = [&](const int kt) __attribute__((always_inline)) {
    if (kt + 2 < ntile)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * CPW) : "memory");
    else if (kt + 1 < ntile)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // first half: K fragments, the DMA of tile kt+3, S^T = K.Q^T - m_run, ragged-tile mask, FIRST / SAFE max
  auto tile_qk = [&](auto SLOT, auto FIRST_, auto SAFE_, const int kt) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(FIRST_)::value, SAFE = decltype(SAFE_)::value;
    if (FIRST && !SAFE) probe_mark(a.probe, probe_t, 1);
    constexpr int slot = decltype(SLOT)::value;
    constexpr uint32_t so = (uint32_t)(slot * TILE_B);  // ring slot offset: an immediate of every LDS read

    u32x4 kf[2][4];
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<so>(kaddr[ks]);
      kf[1][ks] = lds_b128<so + 4096>(kaddr[ks]);
    });
    if (kt + 3 < ntile) dma((slot + 3) % NS, kt + 3, true);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
    __builtin_amdgcn_sched_barrier(0);

    // ---- S^T - m_run = K Q^T + (-m_run): both chains start from minit (= -m_run in every slot; zero in tile 0)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sacc[t] = OP::mma32(__builtin_bit_cast(v8, kf[t][0]), qf[0], minit);
#pragma unroll
      for (int ks = 1; ks < 4; ++ks) sacc[t] = OP::mma32(__builtin_bit_cast(v8, kf[t][ks]), qf[ks], sacc[t]);
    }
    if (kt * 64 + 64 > klen) {  // ragged last tile: keys past klen get p = 0
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sacc[t][r] = -INFINITY;
    }
    if constexpr (FIRST || SAFE) {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[t][r]);
      mx = fmaxf(mx, xor32(mx));
      if constexpr (FIRST) {
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
          minit[r] = -m_run;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[t][r] -= d;
        lrow *= alpha;
        if constexpr (RSM) {
#pragma unroll
          for (int r = 0; r < 16; ++r) lacc[r] *= alpha;
        }
      }
    }
  };
  // second half: V^T fragments of the tile in SLOT, P = 2^(S^T - m_run), O^T += V^T P, row sums
  auto tile_pv = [&](auto SLOT) __attribute__((always_inline)) {
    constexpr int slot = decltype(SLOT)::value;
    constexpr uint32_t so = (uint32_t)(slot * TILE_B);
    uint2 vf[2][2][2][2];
    auto vread = [&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto TT) {
        constexpr int t = decltype(TT)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<so + (32 * t + 16 * sx) * 128>(vaddr[u][0]);
          vf[u][t][sx][1] = lds_tr_b64<so + (32 * t + 16 * sx) * 128>(vaddr[u][1]);
        });
      });
    };
    // both halves of V^T first: their LDS latency hides under the exp2 of the first chunk
    vread(std::integral_constant<int, 0>{});
    vread(std::integral_constant<int, 1>{});
    // exp2 / pack of 16-key chunk c = (t, sx) of P (row sums from the fp32 exp2s, four packed
    // adds), then its two MFMAs (both O^T halves), issued between chunk c+1's exp2s and packs: a
    // wave's own VALU work issues in the shadow of its MFMAs (per accumulator the MFMA order is
    // unchanged)
    v8 pf[2][2];
    auto exp_chunk = [&](auto C) {
      constexpr int t = decltype(C)::value >> 1, sx = decltype(C)::value & 1;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f2 e = {__builtin_amdgcn_exp2f(sacc[t][8 * sx + j]), __builtin_amdgcn_exp2f(sacc[t][8 * sx + j + 1])};
        pf[t][sx][j] = from_f32<T>(e.x);
        pf[t][sx][j + 1] = from_f32<T>(e.y);
        if constexpr (!RSM) lrow += e;
      }
    };
    auto mma_chunk = [&](auto C) {
      constexpr int t = decltype(C)::value >> 1, sx = decltype(C)::value & 1;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
        oacc[u] = OP::mma32(__builtin_bit_cast(v8, w), pf[t][sx], oacc[u]);
      }
      if constexpr (RSM) lacc = OP::mma32(ones, pf[t][sx], lacc);
    };
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
      // per MFMA gap: 4 exp2 (TRANS), 2 packs and 2 row-sum adds
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x400, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x400, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    mma_chunk(std::integral_constant<int, 3>{});
  };
  using IF = std::false_type;
  using IT = std::true_type;
  // all tiles: tile 0 peeled (FIRST), the rest unrolled by the ring depth so every slot is a constant
  // A dead wave runs the same waits, barriers and DMA share in a loop of its own (a branch inside the tile
  // would make hipcc copy the O accumulators back at every tile's join)
  auto tile = [&](auto SLOT, auto FIRST_, auto SAFE_, const int kt) __attribute__((always_inline)) {
    tile_wait(kt);
    tile_qk(SLOT, FIRST_, SAFE_, kt);
    tile_pv(SLOT);
  };
  auto pass = [&](auto SAFE_) __attribute__((always_inline)) {
    if (wave_dead) {
      for (int kt = 0; kt < ntile; ++kt) {
        if (kt + 2 < ntile)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * CPW) : "memory");
        else if (kt + 1 < ntile)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 3 < ntile) dma((kt + 3) % NS, kt + 3, true);
      }
    } else {
      if (ntile > 0) tile(std::integral_constant<int, 0>{}, IT{}, SAFE_, 0);
      for (int kt0 = 0; kt0 < ntile; kt0 += NS) {
        static_for<0, NS>([&](auto S) {
          const int kt = kt0 + decltype(S)::value;
          if (kt >= 1 && kt < ntile) tile(S, IF{}, SAFE_, kt);
        });
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the loop (ntile == 0 included)
  };
  // the second-dispatched half (waves 4-7) at priority 1 for the whole loop: it otherwise loses VALU arbitration to
  // the older half at the start of every segment (cdna_hip_programming.md T5, static form; the guard must be
  // wave-uniform, or the scalar instruction runs for every wave). C2 49.08 vs 49.21 ms, attention 34.5 vs 34.7 us
  // (profiles/r05_ab_c2_prio_split.txt)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  pass(IF{});
  auto row_sum = [&]() -> float {
    if constexpr (RSM) return lacc[0];  // D[m][n] = sum_k P[n][k] for every m: lanes l and l + 32 alike
    float l = lrow.x + lrow.y;
    return l + xor32(l);  // lanes l and l + 32 hold the two key halves of one query
  };
  float l_tot = row_sum();
  {
    // Did any row of the workgroup exceed LMAX (or overflow)? One word per wave in the ring's first bytes
    // (all reads of the last tile retired: every wave waited for its LDS reads before its last MFMAs).
    const bool bad = !(l_tot <= LMAX);
    const unsigned vote = __builtin_amdgcn_ballot_w64(bad) != 0ull ? 1u : 0u;
    __builtin_amdgcn_s_barrier();
    uint32_t* flags = reinterpret_cast<uint32_t*>(lds);
    if (lane == 0) flags[wid] = vote;
    __syncthreads();
    unsigned any = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) any |= flags[w];
    if (__builtin_amdgcn_readfirstlane(any) || a.force_safe) {
      // rare: rerun the whole key loop with the lazy running max (SAFE)
      __syncthreads();  // every wave has read the flags before the DMA overwrites them
      m_run = 0.f;
      lrow = f2{0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; ++r) lacc[r] = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] = 0.f;
        oacc[1][r] = 0.f;
        minit[r] = 0.f;
      }
      dma(0, 0);
      dma(1, 1);
      dma(2, 2);
      pass(IT{});
      l_tot = row_sum();
    }
  }
  probe_mark(a.probe, probe_t, 2);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  // Epilogue (T21): lane l < 32 holds columns 8k..8k+3 of its row, lane l + 32 columns 8k+4..8k+7; one
  // permlane32 swap per dword pairs groups k and k+1, so every lane stores 16 contiguous bytes
  // (lower lanes group k, upper lanes group k+1): 4 dwordx4 stores instead of 8 dwordx2
  if (!wave_dead) {
    T* O = reinterpret_cast<T*>(a.o) + (((int64_t)s_idx * L + min(qrow, L - 1)) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; r4 += 2) {
        v4 w0 = {from_f32<T>(oacc[u][4 * r4 + 0] * inv), from_f32<T>(oacc[u][4 * r4 + 1] * inv),
                 from_f32<T>(oacc[u][4 * r4 + 2] * inv), from_f32<T>(oacc[u][4 * r4 + 3] * inv)};
        v4 w1 = {from_f32<T>(oacc[u][4 * r4 + 4] * inv), from_f32<T>(oacc[u][4 * r4 + 5] * inv),
                 from_f32<T>(oacc[u][4 * r4 + 6] * inv), from_f32<T>(oacc[u][4 * r4 + 7] * inv)};
        uint2 a2 = __builtin_bit_cast(uint2, w0), b2 = __builtin_bit_cast(uint2, w1);
        auto sx = __builtin_amdgcn_permlane32_swap(a2.x, b2.x, false, false);
        auto sy = __builtin_amdgcn_permlane32_swap(a2.y, b2.y, false, false);
        const uint4 out = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        if (qrow < L) *reinterpret_cast<uint4*>(O + 32 * u + 8 * r4 + 8 * h) = out;
      }
  }
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
  if (a.q_len && (int)blockIdx.x * 64 >= a.q_len[s_idx]) {  // dead query block
    probe_exit(a.probe, probe_t);
    return;
  }
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
  constexpr int NW = 8;  // (two 4-wave workgroups per CU measured 40.3 vs 39.6 us at C2: kept one of 8)
  dim3 grid((a.L + 32 * NW - 1) / (32 * NW), a.S * a.H);
  static const bool rsm = [] {
    const char* v = getenv("F5H_ATTN_ROWSUM");
    return v && !strcmp(v, "mfma");
  }();
  if (a.prescaled) {
    if (rsm)
      hipLaunchKernelGGL((attn16_kernel<T, true, NW, true>), grid, dim3(64 * NW), 0, st, a);
    else
      hipLaunchKernelGGL((attn16_kernel<T, true, NW, false>), grid, dim3(64 * NW), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn16_kernel<T, false, NW, false>), grid, dim3(64 * NW), 0, st, a);
  }
}

static int g_force_safe = 0;
void attention_force_safe(int on) { g_force_safe = on ? 1 : 0; }

hipError_t attention(int compute, const AttnArgs& a0, hipStream_t st) {
  if (a0.S <= 0 || a0.H <= 0 || a0.L <= 0) return hipErrorInvalidValue;
  AttnArgs a = a0;
  a.force_safe = g_force_safe;
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
