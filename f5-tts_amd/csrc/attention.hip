// Non-causal multi-head attention, head_dim 64 (AttnProcessor, modules.py:511-520):
// O = softmax(Q K^T * scale [+ key-padding mask]) V, flash-style (scores never materialised).
//
// bf16 path (one MFMA chain per wave, everything lane-local):
//   * workgroup = 4 waves = 128 query rows of one (sequence, head); wave = 32 rows.
//   * S^T = K . Q^T with v_mfma_f32_32x32x16_bf16: the query sits on the lane (col),
//     so each lane owns one query row's running max / sum (softmax needs one
//     shfl_xor(32) per tile, no LDS).
//   * O^T = V^T . P^T: the S^T accumulator registers ARE the B operand (bf16-packed),
//     V^T comes from the LDS tile with ds_read_b64_tr_b16 (hardware transpose).
//   * K/V tiles of 64 keys, register-staged, double-buffered, XOR-swizzled (swz128).
// fp32 parity path: one thread per query row on the VALU (exact fp32, small shapes only).
#include "common.h"
#include "kernels.h"

#include <cstdlib>

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

template <bool PRESCALED, int DBG>
__global__ __launch_bounds__(256, 2) void attn_bf16_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh bf16 each)
  constexpr int NS = 3;                 // LDS ring: one tile read while two are in flight
  constexpr int DPS = 4;                // DMA instructions per tile per wave (K 2 + V 2)
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5;  // lane half
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * 128 + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    // rows past L are clamped (their outputs are never stored)
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
  }
  // consume Q here: otherwise hipcc waits vmcnt(0) at its first use INSIDE the tile loop,
  // draining the LDS-DMA ring every iteration
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  // ---- LDS-DMA of a K/V tile: round r of wave w covers chunks p = (r*4+w)*64 + lane of the
  // 64-row x 8-chunk image; the swizzle is applied to the SOURCE chunk (involution).
  int dsrc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = (r * 4 + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dsrc[r] = row * 64 + swz128(row, slot) * 8;  // element offset inside the tile (before clamping)
  }
  auto dma = [&](int buf, int kt) {
    uint4* Ks = lds + buf * (TILE_B / 16);
    uint4* Vs = Ks + 512;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int row = ((r * 4 + wid) * 64 + lane) >> 3;
      // keys past L are clamped to a real row: their scores are masked (p = 0) below
      const int64_t off = (int64_t)min(kt * 64 + row, L - 1) * 64 + (dsrc[r] - row * 64);
      __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + (r * 4 + wid) * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + (r * 4 + wid) * 64), 16, 0, 0);
    }
  };

  // ---- per-lane LDS read addresses. swz128 depends on row bits 1..3, i.e. on row & 15, which
  // is a lane constant under +32t / +16s shifts (immediates); the +8-row V read needs its own base.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_PTR(void))lds;
  uint32_t kaddr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int row = lane & 31;
    kaddr[ks] = lds0 + row * 128 + swz128(row, ks * 2 + h) * 16;  // + t*4096 immediate
  }
  const int G = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  uint32_t vaddr[2][2];  // [u][first / second 4-key group]
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int g8 = 0; g8 < 2; ++g8) {
      const int r1 = 4 * (G >> 1) + q4 + 8 * g8;  // + 32t + 16s as immediates
      const int dh = 32 * u + 16 * (G & 1) + 4 * p4;
      vaddr[u][g8] = lds0 + 64 * 128 + r1 * 128 + swz128(r1, dh >> 3) * 16 + ((dh >> 2) & 1) * 8;
    }

  const float c = a.scale * 1.4426950408889634f;  // scores in log2 units (unless q carries it)
  float m_run = -INFINITY, l_run = 0.f;
  f32x16 oacc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[u][r] = 0.f;

  dma(0, 0);
  if (ntile > 1) dma(1, 1);
  for (int kt = 0; kt < ntile; ++kt) {
    if (kt + 1 < ntile)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DPS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);

    // ---- K fragments (8 reads); lgkmcnt counts at most 15 outstanding LDS ops, so the V^T
    // reads are issued in two groups of 8 around the softmax
    u32x4 kf[2][4];
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      if constexpr (DBG & 2) {
        kf[0][ks] = *(LDS_PTR(u32x4))(uintptr_t)(kaddr[ks] + so);
        kf[1][ks] = *(LDS_PTR(u32x4))(uintptr_t)(kaddr[ks] + so + 4096);
      } else {
        kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
        kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
      }
    });
    // WAR: ring slot (kt+2)%3 == (kt-1)%3 was last read in iteration kt-1, whose reads all
    // completed (lgkmcnt(0)) before that wave reached this iteration's barrier
    if (kt + 2 < ntile) dma((kt + 2) % NS, kt + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
    __builtin_amdgcn_sched_barrier(0);
    uint2 vf[2][2][2][2];  // [u][t][s][half of the 8-key fragment]
    auto vread = [&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          if constexpr (DBG & 2) {
            s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (LDS_PTR(s16x4))(uintptr_t)(vaddr[u][0] + so + (32 * t + 16 * sx) * 128));
            s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (LDS_PTR(s16x4))(uintptr_t)(vaddr[u][1] + so + (32 * t + 16 * sx) * 128));
            vf[u][t][sx][0] = __builtin_bit_cast(uint2, v1);
            vf[u][t][sx][1] = __builtin_bit_cast(uint2, v2);
          } else {
            vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
            vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
          }
        });
      });
    };

    // ---- S^T = K Q^T (two 32-key sub-tiles)
    f32x16 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sacc[t],
                                                           0, 0, 0);
    }
    vread(std::integral_constant<int, 0>{});  // V^T for dh 0..31: lands under the softmax
    // ---- online softmax; row (query) on the lane, keys in registers (+ partner lane^32)
    const int kbase = kt * 64 + 4 * h;
    const bool full = kt * 64 + 64 <= klen;  // wave-uniform: no key masking needed
    float mx = -1e30f;
    if (full) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if constexpr (!PRESCALED) sacc[t][r] *= c;
          mx = fmaxf(mx, sacc[t][r]);
        }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int key = kbase + t * 32 + (r & 3) + 8 * (r >> 2);
          float sv = key < klen ? (PRESCALED ? sacc[t][r] : sacc[t][r] * c) : -INFINITY;
          sacc[t][r] = sv;
          mx = fmaxf(mx, sv);
        }
    }
    mx = fmaxf(mx, (DBG & 1) ? __shfl_xor(mx, 32, 64) : xor32(mx));
    // the first tile always holds >= 1 valid key, so m_new is finite; exp2(-inf) = 0 for masked keys
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __builtin_amdgcn_exp2f(sacc[t][r] - m_new);
        sacc[t][r] = p;
        lsum += p;
      }
    l_run = l_run * alpha + lsum;
    if (!__all(alpha == 1.f)) {  // running max moved for some row: rescale (exact skip otherwise)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[u][r] *= alpha;
    }

    // ---- O^T += V^T P^T
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][s][j] = f2bf(sacc[t][8 * s + j]);

    asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");  // keep <= 15 LDS ops outstanding
    vread(std::integral_constant<int, 1>{});              // V^T for dh 32..63
    auto pv = [&](auto U) {
      constexpr int u = decltype(U)::value;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
      __builtin_amdgcn_sched_barrier(0);
      // O^T += V^T P^T (element j of lane half h <-> key 16s + 8(j>>2) + 4h + (j&3))
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
      __builtin_amdgcn_sched_barrier(0);
    };
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    pv(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pv(std::integral_constant<int, 1>{});
  }
  // ---- epilogue: O row = query on lane; dh = 32u + 8*r4 + 4h + c
  const float l_tot = l_run + ((DBG & 1) ? __shfl_xor(l_run, 32, 64) : xor32(l_run));
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v2
// Same lane layout as attn_bf16_kernel (S^T = K Q^T, O^T = V^T P^T on 32x32x16 MFMA), with the
// softmax VALU work cut to max + exp + pack per score:
//   * lazy running max folded into the MFMA: after the first tile the S^T accumulator starts at
//     -m_run, so the MFMA returns s - m_run; while no row's tile max exceeds m_run by more than
//     THR (log2 units) p = exp2(s - m_run) needs no subtraction and O is never rescaled (P <= 2^THR,
//     exact in fp32 accumulation, bf16 P has fp32's exponent range). A wave that sees a larger
//     jump re-bases: m_run += d, O, l *= 2^-d, s -= d (cdna_hip_programming.md T13).
//   * row sums on the matrix pipe: l^T += ones . P^T (4 extra MFMAs per tile instead of 32 VALU
//     adds), summed from the same bf16 P that enters O.
//   * NW waves x 32 query rows per workgroup (NW = 8: 256 rows, one workgroup per CU at C2),
//     K/V tiles of 64 keys by LDS-DMA into a 3-deep ring shared by all waves.
// PRIO (wave priority experiments, cdna_hip_programming.md T5): 0 none; 1 = s_setprio 1 once for
// the second half of the waves (they win VALU/MFMA arbitration, which breaks the two waves of a
// SIMD out of lockstep); 2 = s_setprio 1 around every MFMA cluster.
template <bool PRESCALED, int NW, int PRIO = 0>
__global__ __launch_bounds__(64 * NW, 1) void attn_bf16_v2_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh bf16 each)
  // PRIO 4: one barrier per TWO tiles (6-slot ring, four tiles ahead): halves the per-tile
  // barrier coupling of the 8 waves (the SQ counters' 32 % wait share)
  constexpr int TPB = PRIO == 4 ? 2 : 1;
  constexpr int NS = PRIO == 4 ? 6 : 3;
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
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {  // scores in log2 units: fold scale*log2(e) into q
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * c);
    }
  }
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

  const bf16 one = f2bf(1.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  float m_run = 0.f;  // running max (log2 units), valid after tile 0
  f32x16 oacc[2], lacc, negm;  // negm (PRIO 3): -m_run broadcast as the QK chains' first C operand
  if constexpr (PRIO == 3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }

  if constexpr (TPB == 2) {
    for (int t = 0; t < 4 && t < ntile; ++t) dma(t % NS, t);
  } else {
    dma(0, 0);
    if (ntile > 1) dma(1, 1);
  }
  if constexpr (PRIO == 1) {
    if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  for (int kt = 0; kt < ntile; ++kt) {
    if constexpr (TPB == 2) {
      if ((kt & 1) == 0) {  // tiles kt, kt+1 landed (kt+2, kt+3 may stay in flight), then refill
        const int ahead = min(ntile - (kt + 2), 2);  // tiles issued after kt+1
        if (ahead >= 2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * CPW) : "memory");
        else if (ahead == 1)
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // the slots of tiles kt-2, kt-1 were last read before this barrier
        if (kt + 4 < ntile) dma((kt + 4) % NS, kt + 4);
        if (kt + 5 < ntile) dma((kt + 5) % NS, kt + 5);
      }
    } else {
      if (kt + 1 < ntile)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);

    u32x4 kf[2][4];
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
    if constexpr (TPB == 1) {
      if (kt + 2 < ntile) dma((kt + 2) % NS, kt + 2);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
    __builtin_amdgcn_sched_barrier(0);
    uint2 vf[2][2][2][2];
    auto vread = [&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    };

    // ---- S^T - m_run = K Q^T + (-m_run)
    const float init = kt == 0 ? 0.f : -m_run;
    f32x16 sacc[2];
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (PRIO == 3) {  // chains start from negm (kept equal to -m_run; 0 before tile 0)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][0]), qf[0], negm, 0, 0, 0);
#pragma unroll
        for (int ks = 1; ks < 4; ++ks)
          sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sacc[t],
                                                             0, 0, 0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] = init;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sacc[t],
                                                             0, 0, 0);
      }
    }
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
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
    if constexpr (PRIO == 3) {  // 16 v_max3 in two chains (fmaxf would add canonicalising v_max x,x)
      float mb = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; r += 4) {
          asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mx) : "v"(mx), "v"(sacc[t][r]), "v"(sacc[t][r + 1]));
          asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mb) : "v"(mb), "v"(sacc[t][r + 2]), "v"(sacc[t][r + 3]));
        }
      mx = fmaxf(mx, mb);
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[t][r]);
    }
    mx = fmaxf(mx, xor32(mx));
    if (kt == 0) {
      // first tile (>= 1 valid key): the running max starts at the tile max
      m_run = mx;
      if constexpr (PRIO == 3) {
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[r] = -m_run;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= mx;
    } else if (!__all(mx <= THR)) {
      // re-base the rows whose scores ran more than THR above m_run (rare: early tiles)
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run += d;
      if constexpr (PRIO == 3) {
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[r] = -m_run;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] *= alpha;
        oacc[1][r] *= alpha;
        lacc[r] *= alpha;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= d;
    }
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sacc[t][8 * sx + j]));

    asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
    vread(std::integral_constant<int, 1>{});
    // row sums: l^T += ones . P^T (any key order)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
    auto pv = [&](auto U) {
      constexpr int u = decltype(U)::value;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
      if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };
    asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
    pv(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pv(std::integral_constant<int, 1>{});
  }
  const float l_tot = lacc[0];
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v8 (software-pipelined)
// v2's arithmetic with the softmax of tile j-1 moved under the MFMAs of tile j inside each wave
// (cdna_hip_programming.md T15; an MFMA holds the SIMD's vector issue for 8 of its 32 cycles,
// MI355X_MICROARCH.md cycle constants), so the two waves of a SIMD need not take turns:
//   phase A(j): S_j^T - m = K_j Q^T - m (8 MFMA)   ||  P_{j-1} = bf16(exp2(S_{j-1} - m)) (32 exp + 16 pack)
//   phase B(j): l += 1 P_{j-1}, O += V_{j-1} P_{j-1} (12 MFMA)  ||  row max of S_j
//   then the lazy re-base of tile j (rare) and the swap of the two S buffers.
// K/V tiles of 64 keys ride a 4-slot LDS-DMA ring, two tiles ahead: the V of tile j-1 is read
// in iteration j, so its slot is refilled only at iteration j+1 (with tile j+3).
template <bool PRESCALED, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bf16_v8_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh bf16 each)
  constexpr int NS = 4;
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
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * c);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  int dsrc[CPW];
#pragma unroll
  for (int r = 0; r < CPW; ++r) {
    const int p = (r * NW + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dsrc[r] = swz128(row, slot) * 8;
  }
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
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

  const bf16 one = f2bf(1.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  float m_run = 0.f;
  f32x16 oacc[2], lacc, sA[2], sB[2], negm;  // negm: -m_run broadcast, the QK chains' first C operand
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }

  // K fragments of tile kt (issued and retired here; only LDS op in flight at this point)
  auto kread = [&](int kt, u32x4 (&kf)[2][4]) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
  };
  // V^T fragments of tile kt (retired by the caller's lgkmcnt(0) before the PV MFMAs)
  auto vread = [&](int kt, uint2 (&vf)[2][2][2][2]) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto mask_tail = [&](int kt, f32x16 (&sc)[2]) {
    if (kt * 64 + 64 > klen) {  // ragged last tile: keys past klen get p = 0
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sc[t][r] = -INFINITY;
    }
  };
  auto rowmax = [&](const f32x16 (&sc)[2]) {
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[t][r]);
    return fmaxf(mx, xor32(mx));
  };
  // PV of the previous tile: l += 1 P^T, O += V^T P^T
  auto pv = [&](const bf16x8 (&pf)[2][2], uint2 (&vf)[2][2][2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0, 0);
        }
  };

  // ---- tile 0: S_0, m_run = its row max (exact first-tile base)
  dma(0);
  if (ntile > 1) dma(1);
  {
    if (ntile > 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ntile > 2) dma(2);
    u32x4 kf[2][4];
    kread(0, kf);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sA[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sA[t], 0, 0, 0);
    }
    mask_tail(0, sA);
    m_run = rowmax(sA);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] -= m_run;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = -m_run;
  }

  // ---- iteration kt >= 1: S_kt into `cur`, softmax + PV of tile kt-1 from `prev`
  auto step = [&](int kt, f32x16 (&cur)[2], f32x16 (&prev)[2]) {
    if (kt + 1 < ntile)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < ntile) dma(kt + 2);
    u32x4 kf[2][4];
    kread(kt, kf);
    uint2 vf[2][2][2][2];
    vread(kt - 1, vf);
    __builtin_amdgcn_sched_barrier(0);
    // phase A: QK^T of tile kt || exp/pack of tile kt-1, hand-interleaved (sched_barrier fences):
    // MFMA (t, ks) alternates the two accumulator chains; each gap carries 4 exp2 + 2 packs.
    bf16x8 pf[2][2];
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 8>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int t = i & 1, ks = i >> 1;           // MFMA chain t, k-step ks
      constexpr int et = i >> 2, esx = (i >> 1) & 1, ej = (i & 1) * 4;  // exp chunk of tile kt-1
      cur[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks],
                                                        ks == 0 ? negm : cur[t], 0, 0, 0);
      // pin the exp chunk to this gap: its input is (opaquely) redefined here and its packed
      // output consumed here, so no IR pass can hoist or sink it out of the fenced region
      asm volatile("" : "+v"(prev[et]));
#pragma unroll
      for (int j = 0; j < 4; ++j) pf[et][esx][ej + j] = f2bf(__builtin_amdgcn_exp2f(prev[et][8 * esx + ej + j]));
      asm volatile("" ::"v"(pf[et][esx]));
      __builtin_amdgcn_sched_barrier(0);
    });
    // phase B: PV of tile kt-1 || row max of tile kt
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
    mask_tail(kt, cur);
    float mxa = -INFINITY, mxb = -INFINITY;
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 12>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 4) {  // row sums: l^T += ones . P^T
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[i >> 1][i & 1], lacc, 0, 0, 0);
      } else {                 // O^T += V^T P^T, (u, t, sx) = bits of i - 4
        constexpr int k = i - 4, u = k >> 2, t = (k >> 1) & 1, sx = k & 1;
        const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
        oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0, 0);
      }
      if constexpr (i < 8) {  // 4 of the 32 scores of tile kt per gap (two v_max3 chains; no
        // canonicalising v_max x,x pairs as fmaxf would emit)
        constexpr int t = i >> 2, r = (i & 3) * 4;
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mxa) : "v"(mxa), "v"(cur[t][r]), "v"(cur[t][r + 1]));
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mxb) : "v"(mxb), "v"(cur[t][r + 2]), "v"(cur[t][r + 3]));
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    float mx = fmaxf(mxa, mxb);
    mx = fmaxf(mx, xor32(mx));
    __builtin_amdgcn_sched_barrier(0);
    if (!__all(mx <= THR)) {  // re-base (rare): after PV(kt-1), before exp of tile kt
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) negm[r] = -m_run;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] *= alpha;
        oacc[1][r] *= alpha;
        lacc[r] *= alpha;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[t][r] -= d;
    }
  };

  int kt = 1;
  for (; kt + 1 < ntile; kt += 2) {
    step(kt, sB, sA);
    step(kt + 1, sA, sB);
  }
  const bool last_in_b = kt < ntile;
  if (last_in_b) step(kt, sB, sA);
  // ---- drain: softmax + PV of the last tile (two static branches: a runtime-selected array
  // reference would put the S buffers in scratch)
  auto drain = [&](const f32x16 (&sl)[2]) {
    uint2 vf[2][2][2][2];
    vread(ntile - 1, vf);
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sl[t][8 * sx + j]));
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
    pv(pf, vf);
  };
  if (last_in_b)
    drain(sB);
  else
    drain(sA);
  const float l_tot = lacc[0];
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v9 (v8 + early K reads)
// v8 with the LDS reads moved off the tile start: a 5-slot ring three tiles ahead lets the barrier
// of iteration j publish tile j+1, so the K fragments of tile j+1 are read during the PV MFMAs of
// iteration j and the V fragments of tile j-1 during the QK MFMAs; no LDS round trip is exposed
// after a barrier (the v5 stamps measured ~800 cycles per tile there).
// v2's arithmetic with the softmax of tile j-1 moved under the MFMAs of tile j inside each wave
// (cdna_hip_programming.md T15; an MFMA holds the SIMD's vector issue for 8 of its 32 cycles,
// MI355X_MICROARCH.md cycle constants), so the two waves of a SIMD need not take turns:
//   phase A(j): S_j^T - m = K_j Q^T - m (8 MFMA)   ||  P_{j-1} = bf16(exp2(S_{j-1} - m)) (32 exp + 16 pack)
//   phase B(j): l += 1 P_{j-1}, O += V_{j-1} P_{j-1} (12 MFMA)  ||  row max of S_j
//   then the lazy re-base of tile j (rare) and the swap of the two S buffers.
// K/V tiles of 64 keys ride a 4-slot LDS-DMA ring, two tiles ahead: the V of tile j-1 is read
// in iteration j, so its slot is refilled only at iteration j+1 (with tile j+3).
template <bool PRESCALED, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bf16_v9_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh bf16 each)
  constexpr int NS = 5;
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
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * c);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  int dsrc[CPW];
#pragma unroll
  for (int r = 0; r < CPW; ++r) {
    const int p = (r * NW + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    dsrc[r] = swz128(row, slot) * 8;
  }
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
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

  const bf16 one = f2bf(1.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  float m_run = 0.f;
  f32x16 oacc[2], lacc, sA[2], sB[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }

  // K fragments of tile kt (issued and retired here; only LDS op in flight at this point)
  auto kread = [&](int kt, u32x4 (&kf)[2][4]) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
  };
  // V^T fragments of tile kt (retired by the caller's lgkmcnt(0) before the PV MFMAs)
  auto vread = [&](int kt, uint2 (&vf)[2][2][2][2]) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto mask_tail = [&](int kt, f32x16 (&sc)[2]) {
    if (kt * 64 + 64 > klen) {  // ragged last tile: keys past klen get p = 0
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sc[t][r] = -INFINITY;
    }
  };
  auto rowmax = [&](const f32x16 (&sc)[2]) {
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[t][r]);
    return fmaxf(mx, xor32(mx));
  };
  // PV of the previous tile: l += 1 P^T, O += V^T P^T
  auto pv = [&](const bf16x8 (&pf)[2][2], uint2 (&vf)[2][2][2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0, 0);
        }
  };

  // ---- tile 0: S_0, m_run = its row max (exact first-tile base)
  dma(0);
  if (ntile > 1) dma(1);
  if (ntile > 2) dma(2);
  if (ntile > 3) dma(3);
  u32x4 kf[2][4];  // K fragments of the next tile to multiply (loop-carried)
  {
    // tiles 0 and 1 visible; 2 and 3 may stay in flight
    if (ntile > 3)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * CPW) : "memory");
    else if (ntile > 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    kread(0, kf);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sA[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sA[t], 0, 0, 0);
    }
    mask_tail(0, sA);
    m_run = rowmax(sA);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] -= m_run;
    if (ntile > 1) kread(1, kf);
  }

  // ---- iteration kt >= 1: S_kt into `cur`, softmax + PV of tile kt-1 from `prev`
  auto step = [&](int kt, f32x16 (&cur)[2], f32x16 (&prev)[2]) {
    // publish tile kt+1 (its K is read below, during the PV MFMAs); tile kt+2 may stay in flight.
    // The barrier also retires every wave's reads of tile kt-2's slot, refilled with tile kt+3.
    if (kt + 1 < ntile) {
      if (kt + 2 < ntile)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 3 < ntile) dma(kt + 3);
    }
    uint2 vf[2][2][2][2];
    vread(kt - 1, vf);
    __builtin_amdgcn_sched_barrier(0);
    // phase A: QK^T of tile kt || exp/pack of tile kt-1, hand-interleaved (sched_barrier fences):
    // MFMA (t, ks) alternates the two accumulator chains; each gap carries 4 exp2 + 2 packs.
    bf16x8 pf[2][2];
    // K fragments of tile kt were read during the previous iteration: retire them (the V reads
    // just issued are younger; LDS returns in order, so 16 may stay in flight -> lgkmcnt counts 4 bits)
    asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 8>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int t = i & 1, ks = i >> 1;           // MFMA chain t, k-step ks
      constexpr int et = i >> 2, esx = (i >> 1) & 1, ej = (i & 1) * 4;  // exp chunk of tile kt-1
      if constexpr (ks == 0) {  // chain start: C = -m_run broadcast (v_mov, 16 per chain)
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[t][r] = -m_run;
      }
      cur[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], cur[t], 0, 0, 0);
      // pin the exp chunk to this gap: its input is (opaquely) redefined here and its packed
      // output consumed here, so no IR pass can hoist or sink it out of the fenced region
      asm volatile("" : "+v"(prev[et]));
#pragma unroll
      for (int j = 0; j < 4; ++j) pf[et][esx][ej + j] = f2bf(__builtin_amdgcn_exp2f(prev[et][8 * esx + ej + j]));
      asm volatile("" ::"v"(pf[et][esx]));
      __builtin_amdgcn_sched_barrier(0);
    });
    // phase B: PV of tile kt-1 || row max of tile kt
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
    mask_tail(kt, cur);
    float mxa = -INFINITY, mxb = -INFINITY;
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, 12>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 4) {  // row sums: l^T += ones . P^T
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[i >> 1][i & 1], lacc, 0, 0, 0);
      } else {                 // O^T += V^T P^T, (u, t, sx) = bits of i - 4
        constexpr int k = i - 4, u = k >> 2, t = (k >> 1) & 1, sx = k & 1;
        const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
        oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0, 0);
      }
      if constexpr (i == 5) {  // K fragments of tile kt+1 (published by this iteration's barrier;
        // past the last tile the read is of a stale slot and unused: no branch, no phi on kf)
        const uint32_t so = (uint32_t)(((kt + 1) % NS) * TILE_B);
        static_for<0, 4>([&](auto KS) {
          constexpr int ks = decltype(KS)::value;
          kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
          kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
        });
      }
      if constexpr (i < 8) {  // 4 of the 32 scores of tile kt per gap (two v_max3 chains; no
        // canonicalising v_max x,x pairs as fmaxf would emit)
        constexpr int t = i >> 2, r = (i & 3) * 4;
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mxa) : "v"(mxa), "v"(cur[t][r]), "v"(cur[t][r + 1]));
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(mxb) : "v"(mxb), "v"(cur[t][r + 2]), "v"(cur[t][r + 3]));
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    float mx = fmaxf(mxa, mxb);
    mx = fmaxf(mx, xor32(mx));
    __builtin_amdgcn_sched_barrier(0);
    if (!__all(mx <= THR)) {  // re-base (rare): after PV(kt-1), before exp of tile kt
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run += d;

#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] *= alpha;
        oacc[1][r] *= alpha;
        lacc[r] *= alpha;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[t][r] -= d;
    }
  };

  int kt = 1;
  for (; kt + 1 < ntile; kt += 2) {
    step(kt, sB, sA);
    step(kt + 1, sA, sB);
  }
  const bool last_in_b = kt < ntile;
  if (last_in_b) step(kt, sB, sA);
  // ---- drain: softmax + PV of the last tile (two static branches: a runtime-selected array
  // reference would put the S buffers in scratch)
  auto drain = [&](const f32x16 (&sl)[2]) {
    uint2 vf[2][2][2][2];
    vread(ntile - 1, vf);
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sl[t][8 * sx + j]));
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
    pv(pf, vf);
  };
  if (last_in_b)
    drain(sB);
  else
    drain(sA);
  const float l_tot = lacc[0];
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v3 (ping-pong)
// v2's arithmetic in a two-group schedule: 8 waves x 32 query rows; group 0 = waves 0-3,
// group 1 = waves 4-7, half a tile apart, so each SIMD pairs one wave in its MFMA half with one
// in its VALU half (MI355X_MICROARCH.md "Two waves per SIMD"):
//   M-half j: S_j = K_j Q^T - m (8 MFMA), O += V_{j-1} P_{j-1} (8), l += 1 P_{j-1} (4)
//   V-half j: softmax(S_j) -> P_j (max, exp2, pack), LDS reads of V_j and K_{j+1},
//             LDS-DMA of tile j+3, wait for own DMA of tile j+2
// One s_barrier between half-periods. Tile t must be visible before the V-half t-1 of group 0
// (half-period 2t-1): both groups waited for their own part in V-half t-2, which ends before
// that. Ring of 4 tiles: tile t+4 is fetched in V-half t+1 into the slot of tile t, whose last
// read (group 1, V-half t, half-period 2t+2) is retired (lgkmcnt(0)) before the barrier ending it.
template <bool PRESCALED>
__global__ __launch_bounds__(512, 1) void attn_bf16_v3_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int NW = 8;
  constexpr int TILE_B = 2 * 64 * 128;
  constexpr int NS = 4;
  constexpr int CPW = 512 / (64 * NW);
  constexpr float THR = 8.f;
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
      const float c = a.scale * 1.4426950408889634f;
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * c);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  const int drow = (wid * 64 + lane) >> 3;  // CPW == 1: one chunk of K and one of V per lane
  const int dsrc = swz128(drow, (wid * 64 + lane) & 7) * 8;
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
    uint4* Vs = Ks + 512;
    const int64_t off = (int64_t)min(kt * 64 + drow, L - 1) * 64 + dsrc;
    __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + wid * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + wid * 64), 16, 0, 0);
  };
  static_assert(CPW == 1, "one DMA round per tile");

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

  u32x4 kf[2][4];
  uint2 vf[2][2][2][2];
  auto kread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
  };
  auto vread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto fence_regs = [&]() {  // the asm reads above are complete (caller waited lgkmcnt)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
  };

  const bf16 one = f2bf(1.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  float m_run = 0.f;
  f32x16 oacc[2], lacc, sacc[2];
  bf16x8 pf[2][2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }

  auto pv = [&]() {  // O^T += V^T P^T, l^T += 1 P^T for the previous tile
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
  };

  dma(0);
  if (ntile > 1) dma(1);
  if (ntile > 2) dma(2);
  if (ntile > 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  kread(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  fence_regs();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < ntile; ++kt) {
    // ---------------- M-half kt (its K/V fragments were retired at the end of the last V-half)
    const float init = kt == 0 ? 0.f : -m_run;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[t][r] = init;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sacc[t],
                                                           0, 0, 0);
    }
    if (kt > 0) pv();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---------------- V-half kt
    if (kt * 64 + 64 > klen) {
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
    // S_j is complete, so the MFMAs that read kf are done: refill it (and vf) for the next M-half
    if (kt + 1 < ntile) kread(kt + 1);
    vread(kt);
    if (kt == 0) {
      m_run = mx;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= mx;
    } else if (!__all(mx <= THR)) {
      const float d = fmaxf(mx, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-d);
      m_run += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        oacc[0][r] *= alpha;
        oacc[1][r] *= alpha;
        lacc[r] *= alpha;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= d;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sacc[t][8 * sx + j]));
    if (kt + 3 < ntile) dma(kt + 3);
    // retire this half's LDS reads before the barrier: the slot they read is refilled by the
    // other group's DMA in the next half-period
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence_regs();
    if (kt + 3 < ntile)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // tile kt+2 landed, kt+3 in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  pv();
  if (grp == 0) __builtin_amdgcn_s_barrier();

  const float l_tot = lacc[0];
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v4 (fixed offset)
// Softmax with a FIXED per-row offset instead of a running max. Any offset c gives the exact
// result, softmax(s) = exp2(s - c) / sum exp2(s - c); the running max only guards the fp32
// range. v4 takes c = bf16(max of the row's first key tile) and folds "- c" into the QK^T
// MFMA chain as one extra k-step per 32-key subtile ([K | 1] . [Q | -c]^T), so a steady-state
// tile costs exp2 + pack per score and no VALU reduction at all. Row sums ride the matrix pipe
// (l^T += 1 . P^T, from the same bf16 P that enters O). If a row's scores climb more than ~90
// (log2 units) above c the sums leave the safe range; the wave detects it from l and O at the
// end and recomputes its rows with the exact online-softmax loop reading K/V from global memory
// (attn_row_exact) -- the result is then bit-for-bit that of the exact path.
//   * 8 waves x 32 query rows per workgroup; K/V tiles of 64 keys by LDS-DMA into a 4-deep ring,
//     fetched 3 tiles ahead; K fragments of tile j+1 are prefetched during tile j.
F5H_DEV void attn_row_exact(const AttnArgs& a, const bf16* Q, const bf16* K, const bf16* V, int qrow, int klen,
                            float qscale, float* o /*[64]*/) {
  // one lane = one query row, fp32, keys in sequence (rare fallback; correctness over speed)
  float q[64];
  for (int d = 0; d < 64; ++d) q[d] = bf2f(Q[(int64_t)qrow * 64 + d]) * qscale;
  float m = -INFINITY, l = 0.f;
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
  for (int k = 0; k < klen; ++k) {
    float sc = 0.f;
    for (int d = 0; d < 64; ++d) sc = fmaf(q[d], bf2f(K[(int64_t)k * 64 + d]), sc);
    const float mn = fmaxf(m, sc);
    const float al = __builtin_amdgcn_exp2f(m - mn), p = __builtin_amdgcn_exp2f(sc - mn);
    l = l * al + p;
    for (int d = 0; d < 64; ++d) o[d] = o[d] * al + p * bf2f(V[(int64_t)k * 64 + d]);
    m = mn;
  }
  const float inv = 1.f / l;
  for (int d = 0; d < 64; ++d) o[d] *= inv;
}

template <bool PRESCALED>
__global__ __launch_bounds__(512, 1) void attn_bf16_v4_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int NW = 8;
  constexpr int TILE_B = 2 * 64 * 128;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;
  const float qscale = PRESCALED ? 1.f : a.scale * 1.4426950408889634f;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * qscale);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  const int drow = (wid * 64 + lane) >> 3;
  const int dsrc = swz128(drow, (wid * 64 + lane) & 7) * 8;
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
    uint4* Vs = Ks + 512;
    const int64_t off = (int64_t)min(kt * 64 + drow, L - 1) * 64 + dsrc;
    __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + wid * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + wid * 64), 16, 0, 0);
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

  u32x4 kfA[2][4], kfB[2][4];
  uint2 vf[2][2][2][2];
  auto kread = [&](u32x4(&kf)[2][4], int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
  };
  auto kfence = [&](u32x4(&kf)[2][4]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
  };
  auto vread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto vfence = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
  };

  const bf16 one = f2bf(1.f), zero = f2bf(0.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  // the "+1" column of [K | 1]: k = 0 of the extra k-step, held by the lower half-wave
  bf16x8 kone = {zero, zero, zero, zero, zero, zero, zero, zero};
  if (h == 0) kone[0] = one;
  bf16x8 qoff = {zero, zero, zero, zero, zero, zero, zero, zero};  // [.. | -c] of [Q | -c]
  float c_off = 0.f;
  f32x16 oacc[2], lacc, sacc[2];
  bf16x8 pf[2][2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }

  // one tile: S^T (- c), P = exp2, O^T += V^T P^T, l^T += 1 P^T
  auto tile = [&](int kt, u32x4(&kc)[2][4], u32x4(&kn)[2][4]) {
    if (kt + 2 < ntile)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // tile kt+1 landed, kt+2 in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 3 < ntile) dma(kt + 3);
    vread(kt);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kc[t][ks]), qf[ks], sacc[t],
                                                           0, 0, 0);
      if (kt > 0) sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kone, qoff, sacc[t], 0, 0, 0);
    }
    if (kt + 1 < ntile) kread(kn, kt + 1);
    if (kt * 64 + 64 > klen) {  // ragged last tile
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sacc[t][r] = -INFINITY;
    }
    if (kt == 0) {  // the offset: bf16 of the first tile's row max (tile 0 holds >= 1 valid key)
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[t][r]);
      mx = fmaxf(mx, xor32(mx));
      const bf16 cb = f2bf(mx);
      c_off = bf2f(cb);
      if (h == 0) qoff[0] = f2bf(-c_off);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[t][r] -= c_off;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sacc[t][8 * sx + j]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    vfence();
    kfence(kn);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  dma(0);
  if (ntile > 1) dma(1);
  if (ntile > 2) dma(2);
  if (ntile > 2)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 landed
  else if (ntile > 1)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  kread(kfA, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  kfence(kfA);
  for (int kt = 0; kt < ntile; kt += 2) {
    tile(kt, kfA, kfB);
    if (kt + 1 < ntile) tile(kt + 1, kfB, kfA);
  }

  float l_tot = lacc[0];
  bool bad = !(l_tot < 1e30f) || !(l_tot > 0.f);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) bad |= !(fabsf(oacc[u][r]) < 3e38f);
  bad &= qrow < L;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
    if (__any(bad)) {
      if (bad) {  // rare: scores ran out of the fixed offset's range -> exact per-row recompute
        float o[64];
        attn_row_exact(a, Q, K, V, qrow, klen, qscale, o);
        if (h == 0)
          for (int d = 0; d < 64; ++d) O[d] = f2bf(o[d]);
      }
      if (bad) return;
    }
    const float inv = 1.f / l_tot;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

__device__ uint64_t g_attn_stamps[4 * 8 * 8];

template <bool PRESCALED, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void attn_bf16_v5_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  // diagnostic build only: cycles per segment of the K loop, summed (s_memtime drains lgkmcnt)
  auto stamp = [&](int seg) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      if (seg >= 0) st_acc[seg] += t - st_prev;
      st_prev = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  constexpr int NW = 8;
  constexpr int TILE_B = 2 * 64 * 128;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;
  const float qscale = PRESCALED ? 1.f : a.scale * 1.4426950408889634f;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * qscale);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  const int drow = (wid * 64 + lane) >> 3;
  const int dsrc = swz128(drow, (wid * 64 + lane) & 7) * 8;
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
    uint4* Vs = Ks + 512;
    const int64_t off = (int64_t)min(kt * 64 + drow, L - 1) * 64 + dsrc;
    __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + wid * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + wid * 64), 16, 0, 0);
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

  u32x4 kf[2][4];
  uint2 vf[2][2][2][2];
  auto kread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
  };
  auto kfence = [&]() {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
  };
  auto vread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto vfence = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
  };

  const bf16 one = f2bf(1.f), zero = f2bf(0.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  // the "+1" column of [K | 1]: k = 0 of the extra k-step, held by the lower half-wave
  bf16x8 kone = {zero, zero, zero, zero, zero, zero, zero, zero};
  if (h == 0) kone[0] = one;
  bf16x8 qoff = {zero, zero, zero, zero, zero, zero, zero, zero};  // [.. | -c] of [Q | -c]
  float c_off = 0.f;
  f32x16 oacc[2], lacc, sA[2], sB[2];
  bf16x8 pf[2][2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }


  auto qk = [&](f32x16(&sc)[2], bool off) {  // S^T (- c) from the K fragments in kf
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sc[t], 0, 0, 0);
      if (off) sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kone, qoff, sc[t], 0, 0, 0);
    }
  };
  auto softmax_pv = [&](f32x16(&sc)[2], int kt) {  // P = exp2(S - c); O^T += V^T P^T; l^T += 1 P^T
    if (kt * 64 + 64 > klen) {
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sc[t][r] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sc[t][8 * sx + j]));
    stamp(2);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
  };
  // iteration kt: S_{kt+1} on the matrix pipe while P_kt is exponentiated, then P_kt V_kt, then
  // the fragments of the next iteration (K_{kt+2}, V_{kt+1}) behind one barrier.
  auto iter = [&](int kt, f32x16(&scur)[2], f32x16(&snxt)[2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // K_{kt+1}, V_kt
    kfence();
    vfence();
    stamp(kt > 0 ? 5 : -1);
    if (kt + 1 < ntile) {
      // tile kt+2 visible to every wave (its K is read below); all V_kt reads retired, so the
      // DMA below may refill tile kt's slot
      if (kt + 3 < ntile)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // tile kt+2 landed, kt+3 in flight
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(3);
      __builtin_amdgcn_s_barrier();
      stamp(4);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < ntile) qk(snxt, true);
    stamp(0);
    softmax_pv(scur, kt);
    stamp(1);
    __builtin_amdgcn_sched_barrier(0);
    // next iteration's fragments load under P_kt V_kt on the matrix pipe
    if (kt + 1 < ntile) {
      if (kt + 4 < ntile) dma(kt + 4);
      if (kt + 2 < ntile) kread(kt + 2);
      vread(kt + 1);
    }
  };

  for (int t = 0; t < 4 && t < ntile; ++t) dma(t);
  {
    const int beyond = min(ntile, 4) - 2;  // tiles issued after tile 1
    if (beyond >= 2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (beyond == 1)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  kread(0);
  vread(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  kfence();
  __builtin_amdgcn_sched_barrier(0);
  qk(sA, false);
  {  // the offset: bf16 of the first tile's row max (tile 0 holds >= 1 valid key)
    if (64 > klen) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (4 * h + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sA[t][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sA[t][r]);
    mx = fmaxf(mx, xor32(mx));
    c_off = bf2f(f2bf(mx));
    if (h == 0) qoff[0] = f2bf(-c_off);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] -= c_off;
  }
  if (ntile > 1) kread(1);
  for (int kt = 0; kt < ntile; kt += 2) {
    iter(kt, sA, sB);
    if (kt + 1 < ntile) iter(kt + 1, sB, sA);
  }

  if constexpr (STAMP) {
    if (lane == 0 && qb == 0 && bh < 4)
      for (int k = 0; k < 6; ++k) g_attn_stamps[(bh * 8 + wid) * 8 + k] = st_acc[k];
    if (lane == 0 && qb == 0 && bh < 4) g_attn_stamps[(bh * 8 + wid) * 8 + 6] = ntile;
  }
  float l_tot = lacc[0];
  bool bad = !(l_tot < 1e30f) || !(l_tot > 0.f);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) bad |= !(fabsf(oacc[u][r]) < 3e38f);
  bad &= qrow < L;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
    if (__any(bad)) {
      if (bad) {  // rare: scores ran out of the fixed offset's range -> exact per-row recompute
        float o[64];
        attn_row_exact(a, Q, K, V, qrow, klen, qscale, o);
        if (h == 0)
          for (int d = 0; d < 64; ++d) O[d] = f2bf(o[d]);
      }
      if (bad) return;
    }
    const float inv = 1.f / l_tot;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

template <bool PRESCALED, bool STAMP = false>
__global__ __launch_bounds__(512, 1) void attn_bf16_v6_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  // diagnostic build only: cycles per segment of the K loop, summed (s_memtime drains lgkmcnt)
  auto stamp = [&](int seg) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      if (seg >= 0) st_acc[seg] += t - st_prev;
      st_prev = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  constexpr int NW = 8;
  constexpr int TILE_B = 2 * 64 * 128;
  constexpr int NS = 5;  // ring tiles (= DMA distance D)
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;
  const float qscale = PRESCALED ? 1.f : a.scale * 1.4426950408889634f;

  const int qrow = qb * (32 * NW) + wid * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow, L - 1) * 64 + ks * 16 + h * 8);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
    if constexpr (!PRESCALED) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * qscale);
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[ks]));

  const int drow = (wid * 64 + lane) >> 3;
  const int dsrc = swz128(drow, (wid * 64 + lane) & 7) * 8;
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
    uint4* Vs = Ks + 512;
    const int64_t off = (int64_t)min(kt * 64 + drow, L - 1) * 64 + dsrc;
    __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(Ks + wid * 64), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(V + off), (LDS_PTR(void))(Vs + wid * 64), 16, 0, 0);
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

  u32x4 kf[2][4];
  uint2 vf[2][2][2][2];
  auto kread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kf[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kf[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
  };
  auto kfence = [&]() {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kf[t][ks]));
  };
  auto vread = [&](int kt) {
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vf[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vf[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto vfence = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vf[u][t][sx][0]));
          asm volatile("" : "+v"(vf[u][t][sx][1]));
        }
  };

  const bf16 one = f2bf(1.f), zero = f2bf(0.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  // the "+1" column of [K | 1]: k = 0 of the extra k-step, held by the lower half-wave
  bf16x8 kone = {zero, zero, zero, zero, zero, zero, zero, zero};
  if (h == 0) kone[0] = one;
  bf16x8 qoff = {zero, zero, zero, zero, zero, zero, zero, zero};  // [.. | -c] of [Q | -c]
  float c_off = 0.f;
  f32x16 oacc[2], lacc, sA[2], sB[2];
  bf16x8 pf[2][2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    oacc[0][r] = 0.f;
    oacc[1][r] = 0.f;
    lacc[r] = 0.f;
  }


  auto qk = [&](f32x16(&sc)[2], bool off) {  // S^T (- c) from the K fragments in kf
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[t][ks]), qf[ks], sc[t], 0, 0, 0);
      if (off) sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kone, qoff, sc[t], 0, 0, 0);
    }
  };
  auto softmax = [&](f32x16(&sc)[2], int kt) {  // P = exp2(S - c)
    if (kt * 64 + 64 > klen) {
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sc[t][r] = -INFINITY;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sc[t][8 * sx + j]));
  };
  auto pvl = [&]() {  // O^T += V^T P^T; l^T += 1 P^T
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[u][t][sx][0].x, vf[u][t][sx][0].y, vf[u][t][sx][1].x, vf[u][t][sx][1].y);
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[u], 0, 0,
                                                            0);
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc, 0, 0, 0);
  };

  // Ping-pong: group g = waves 4g..4g+3; group 1 runs half an iteration behind group 0, so on
  // every SIMD one wave is in its X half while its partner is in its Y half:
  //   X_j: S_{j+1} = K_{j+1} Q^T - c (10 MFMA) beside P_j = exp2(S_j) (VALU)
  //   Y_j: O += V_j P_j, l += 1 P_j (12 MFMA) beside LDS-DMA of tile j+5 and the LDS reads of
  //        K_{j+2}, V_{j+1}; retire those reads (lgkmcnt(0)) and the own DMA of tile j+3
  // Half-period h: group 0 runs X_j at 2j, Y_j at 2j+1; group 1 one later. Tile t is read from
  // half-period 2t-3 (group 0, K) to 2t (group 1, V); its DMA is waited by both groups by the
  // end of half-period 2t-4 (Y_{t-3}), issued in Y_{t-5}; the 5-tile ring slot it fills held
  // tile t-5, whose last read retired before the barrier ending half-period 2t-10.
  auto iter = [&](int kt, f32x16(&scur)[2], f32x16(&snxt)[2]) {
    // ---- X half
    stamp(kt > 0 ? 5 : -1);
    if (kt + 1 < ntile) qk(snxt, true);
    stamp(0);
    softmax(scur, kt);
    stamp(1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stamp(2);
    // ---- Y half
    pvl();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 5 < ntile) dma(kt + 5);
    if (kt + 2 < ntile) kread(kt + 2);
    if (kt + 1 < ntile) vread(kt + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    kfence();
    vfence();
    stamp(3);
    {
      const int young = min(ntile - 1, kt + 5) - (kt + 3);  // tiles issued after tile kt+3
      if (young >= 2)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (young == 1)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stamp(4);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int t = 0; t < NS && t < ntile; ++t) dma(t);
  {
    const int beyond = min(ntile, NS) - 3;  // tiles issued after tile 2
    if (beyond >= 2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (beyond == 1)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  kread(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  kfence();
  __builtin_amdgcn_sched_barrier(0);
  qk(sA, false);
  {  // the offset: bf16 of the first tile's row max (tile 0 holds >= 1 valid key)
    if (64 > klen) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (4 * h + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sA[t][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sA[t][r]);
    mx = fmaxf(mx, xor32(mx));
    c_off = bf2f(f2bf(mx));
    if (h == 0) qoff[0] = f2bf(-c_off);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[t][r] -= c_off;
  }
  if (ntile > 1) kread(1);
  vread(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  kfence();
  vfence();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < ntile; kt += 2) {
    iter(kt, sA, sB);
    if (kt + 1 < ntile) iter(kt + 1, sB, sA);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();

  if constexpr (STAMP) {
    if (lane == 0 && qb == 0 && bh < 4)
      for (int k = 0; k < 6; ++k) g_attn_stamps[(bh * 8 + wid) * 8 + k] = st_acc[k];
    if (lane == 0 && qb == 0 && bh < 4) g_attn_stamps[(bh * 8 + wid) * 8 + 6] = ntile;
  }
  float l_tot = lacc[0];
  bool bad = !(l_tot < 1e30f) || !(l_tot > 0.f);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) bad |= !(fabsf(oacc[u][r]) < 3e38f);
  bad &= qrow < L;
  if (qrow < L) {
    bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow) * a.H + head) * 64;
    if (__any(bad)) {
      if (bad) {  // rare: scores ran out of the fixed offset's range -> exact per-row recompute
        float o[64];
        attn_row_exact(a, Q, K, V, qrow, klen, qscale, o);
        if (h == 0)
          for (int d = 0; d < 64; ++d) O[d] = f2bf(o[d]);
      }
      if (bad) return;
    }
    const float inv = 1.f / l_tot;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        bf16x4 w = {f2bf(oacc[u][4 * r4 + 0] * inv), f2bf(oacc[u][4 * r4 + 1] * inv),
                    f2bf(oacc[u][4 * r4 + 2] * inv), f2bf(oacc[u][4 * r4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
      }
  }
  probe_exit(a.probe, probe_t);
}

// ---------------------------------------------------------------- bf16 kernel, v7
// One wave per SIMD, 64 query rows per wave (two 32-row blocks b0, b1 sharing every K/V
// fragment read from LDS: half the LDS traffic per FLOP of the 32-row kernels), 4 waves =
// 256 rows per workgroup. v5's arithmetic (fixed per-row offset folded into the QK^T MFMA
// chain, exp2 + pack per score, row sums on the matrix pipe, exact fallback). With no partner
// wave on the SIMD, MFMA and VALU overlap inside the wave: each iteration is four clusters,
// every MFMA followed by a few independent VALU ops (sched_group_barrier):
//   C1: S_{j+1}[b0] (10 MFMA)            | P_j[b1], keys 0-31  = exp2 + pack (24 VALU)
//   C2: S_{j+1}[b1] (10 MFMA)            | P_j[b1], keys 32-63 (24 VALU)
//   C3: O[b0] += V_j P_j[b0], l (12 MFMA) | P_{j+1}[b0] (48 VALU; S_{j+1}[b0] done after C1)
//   C4: O[b1] += V_j P_j[b1], l (12 MFMA) | LDS reads of K_{j+2}, V_{j+1}, DMA of tile j+4
// K/V: 64-key tiles by LDS-DMA into a 4-tile ring; the K and V fragments are double-buffered
// in registers (read one iteration ahead). Tile j+2 is waited for (vmcnt) and published (one
// s_barrier) at the top of iteration j; the DMA of tile j+4 then refills tile j's slot, whose
// last reads (V_j, iteration j-1) retired at the end of iteration j-1.
template <bool PRESCALED>
__global__ __launch_bounds__(256, 1) void attn_bf16_v7_kernel(AttnArgs a) {
  const ProbeT probe_t = probe_enter(a.probe);
  constexpr int NW = 4;
  constexpr int TILE_B = 2 * 64 * 128;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  int qb, bh;
  attn_block(qb, bh);
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;
  const float qscale = PRESCALED ? 1.f : a.scale * 1.4426950408889634f;

  int qrow[2];
  bf16x8 qf[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    qrow[b] = qb * 256 + wid * 64 + b * 32 + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 v = *reinterpret_cast<const uint4*>(Q + (int64_t)min(qrow[b], L - 1) * 64 + ks * 16 + h * 8);
      qf[b][ks] = __builtin_bit_cast(bf16x8, v);
      if constexpr (!PRESCALED) {
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[b][ks][j] = f2bf(bf2f(qf[b][ks][j]) * qscale);
      }
    }
  }
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) asm volatile("" ::"v"(qf[b][ks]));

  // DMA: per tile 512 chunks of K and 512 of V; chunk p = (r*4 + w)*64 + lane, r = 0, 1
  int drow[2], dsrc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = (r * NW + wid) * 64 + lane;
    drow[r] = p >> 3;
    dsrc[r] = swz128(drow[r], p & 7) * 8;
  }
  auto dma = [&](int kt) {
    uint4* Ks = lds + (kt % NS) * (TILE_B / 16);
    uint4* Vs = Ks + 512;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t off = (int64_t)min(kt * 64 + drow[r], L - 1) * 64 + dsrc[r];
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

  u32x4 kf[2][2][4];         // [buffer][32-key subtile][k-step]
  uint2 vf[2][2][2][2][2];   // [buffer][u][t][sx][half]
  auto kread = [&](auto BUF, int kt) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    u32x4(&kb)[2][4] = kf[bb];
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      kb[0][ks] = lds_b128<0>(kaddr[ks] + so);
      kb[1][ks] = lds_b128<4096>(kaddr[ks] + so);
    });
  };
  auto vread = [&](auto BUF, int kt) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    const uint32_t so = (uint32_t)((kt % NS) * TILE_B);
    uint2(&vb)[2][2][2][2] = vf[bb];
    static_for<0, 2>([&](auto U) {
      constexpr int u = decltype(U)::value;
      static_for<0, 2>([&](auto T) {
        constexpr int t = decltype(T)::value;
        static_for<0, 2>([&](auto S) {
          constexpr int sx = decltype(S)::value;
          vb[u][t][sx][0] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][0] + so);
          vb[u][t][sx][1] = lds_tr_b64<(32 * t + 16 * sx) * 128>(vaddr[u][1] + so);
        });
      });
    });
  };
  auto fence_buf = [&](auto BUF) __attribute__((always_inline)) {  // the asm LDS reads into this buffer have retired
    constexpr int bb = decltype(BUF)::value;
    u32x4(&kb)[2][4] = kf[bb];
    uint2(&vb)[2][2][2][2] = vf[bb];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(kb[t][ks]));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          asm volatile("" : "+v"(vb[u][t][sx][0]));
          asm volatile("" : "+v"(vb[u][t][sx][1]));
        }
  };

  constexpr std::integral_constant<int, 0> I0{};
  constexpr std::integral_constant<int, 1> I1{};
  const bf16 one = f2bf(1.f), zero = f2bf(0.f);
  const bf16x8 ones = {one, one, one, one, one, one, one, one};
  bf16x8 kone = {zero, zero, zero, zero, zero, zero, zero, zero};
  if (h == 0) kone[0] = one;
  bf16x8 qoff[2];
  float c_off[2];
  f32x16 oacc[2][2], lacc[2];
  f32x16 s0[2], s1a[2], s1b[2];  // S^T of b0 (one buffer), of b1 (two buffers)
  bf16x8 p0a[2][2], p0b[2][2], p1[2][2];  // P of b0 (two buffers), of b1
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    qoff[b] = bf16x8{zero, zero, zero, zero, zero, zero, zero, zero};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      oacc[b][0][r] = 0.f;
      oacc[b][1][r] = 0.f;
      lacc[b][r] = 0.f;
    }
  }

  auto qk = [&](auto BUF, auto BI, f32x16(&sc)[2], bool off) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value, b = decltype(BI)::value;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[bb][t][ks]), qf[b][ks], sc[t],
                                                           0, 0, 0);
      if (off) sc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kone, qoff[b], sc[t], 0, 0, 0);
    }
  };
  auto mask_tile = [&](f32x16(&sc)[2], int kt) __attribute__((always_inline)) {
    if (kt * 64 + 64 > klen) {
      const int kbase = kt * 64 + 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kbase + t * 32 + (r & 3) + 8 * (r >> 2) >= klen) sc[t][r] = -INFINITY;
    }
  };
  auto expt = [&](f32x16(&sc)[2], bf16x8(&pf)[2][2], auto TI) __attribute__((always_inline)) {  // one 32-key subtile
    constexpr int t = decltype(TI)::value;
#pragma unroll
    for (int sx = 0; sx < 2; ++sx)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[t][sx][j] = f2bf(__builtin_amdgcn_exp2f(sc[t][8 * sx + j]));
  };
  auto pv = [&](auto BUF, auto BI, bf16x8(&pf)[2][2]) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value, b = decltype(BI)::value;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
          const uint4 w = make_uint4(vf[bb][u][t][sx][0].x, vf[bb][u][t][sx][0].y, vf[bb][u][t][sx][1].x,
                                     vf[bb][u][t][sx][1].y);
          oacc[b][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w), pf[t][sx], oacc[b][u],
                                                               0, 0, 0);
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx)
        lacc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[t][sx], lacc[b], 0, 0, 0);
  };
  auto interleave = [&](auto NM, auto VP) __attribute__((always_inline)) {  // NM x {1 MFMA, VP VALU} in this scheduling region
    static_for<0, decltype(NM)::value>([&](auto) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x402, decltype(VP)::value, 0);
    });
  };

  // one iteration; KB = buffer holding K_{kt+1}, V_kt; the other buffer receives K_{kt+2}, V_{kt+1}
  // S0/P0 naming: scur1/snxt1 are b1's S buffers, pcur0/pnxt0 b0's P buffers
  auto iter = [&](int kt, auto KB, auto KO, f32x16(&scur1)[2], f32x16(&snxt1)[2], bf16x8(&pcur0)[2][2],
                  bf16x8(&pnxt0)[2][2]) __attribute__((always_inline)) {
    if (kt + 2 < ntile) {
      if (kt + 3 < ntile)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile kt+2 landed, kt+3 in flight
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (kt + 4 < ntile) dma(kt + 4);
    const bool more = kt + 1 < ntile;
    __builtin_amdgcn_sched_barrier(0);
    // C1
    mask_tile(scur1, kt);
    if (more) qk(KB, I0, s0, true);
    expt(scur1, p1, I0);
    if (more) interleave(std::integral_constant<int, 10>{}, std::integral_constant<int, 3>{});
    __builtin_amdgcn_sched_barrier(0);
    // C2
    if (more) qk(KB, I1, snxt1, true);
    expt(scur1, p1, I1);
    if (more) interleave(std::integral_constant<int, 10>{}, std::integral_constant<int, 3>{});
    __builtin_amdgcn_sched_barrier(0);
    // C3
    pv(KB, I0, pcur0);
    if (more) {
      mask_tile(s0, kt + 1);
      expt(s0, pnxt0, I0);
      expt(s0, pnxt0, I1);
      interleave(std::integral_constant<int, 12>{}, std::integral_constant<int, 4>{});
    }
    __builtin_amdgcn_sched_barrier(0);
    // C4
    pv(KB, I1, p1);
    if (kt + 2 < ntile) kread(KO, kt + 2);
    if (more) vread(KO, kt + 1);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fence_buf(KO);
  };

  // ---- prologue: tiles 0..3 in flight, K_0, K_1, V_0 read; S_0 fixes the offsets
  for (int t = 0; t < NS && t < ntile; ++t) dma(t);
  {
    const int beyond = min(ntile, NS) - 2;  // tiles issued after tile 1
    if (beyond >= 2)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (beyond == 1)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  constexpr std::integral_constant<int, 0> B0{};
  constexpr std::integral_constant<int, 1> B1{};
  kread(B0, 0);
  vread(B0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  fence_buf(B0);
  qk(B0, I0, s0, false);
  qk(B0, I1, s1a, false);
  if (ntile > 1) kread(B1, 1);
  mask_tile(s0, 0);
  mask_tile(s1a, 0);
  auto fix_offset = [&](f32x16(&sc)[2], auto BI) __attribute__((always_inline)) {
    constexpr int b = decltype(BI)::value;
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[t][r]);
    mx = fmaxf(mx, xor32(mx));
    c_off[b] = bf2f(f2bf(mx));
    if (h == 0) qoff[b][0] = f2bf(-c_off[b]);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[t][r] -= c_off[b];
  };
  fix_offset(s0, I0);
  fix_offset(s1a, I1);
  expt(s0, p0a, I0);
  expt(s0, p0a, I1);
  // K_1 lives in buffer 1: iteration 0 uses KB = 1 for K_{1} but V_0 sits in buffer 0 -> move V
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  fence_buf(B1);
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) {
        vf[1][u][t][sx][0] = vf[0][u][t][sx][0];
        vf[1][u][t][sx][1] = vf[0][u][t][sx][1];
      }
  int kt = 0;
  for (; kt + 1 < ntile; kt += 2) {
    iter(kt, B1, B0, s1a, s1b, p0a, p0b);
    iter(kt + 1, B0, B1, s1b, s1a, p0b, p0a);
  }
  if (kt < ntile) iter(kt, B1, B0, s1a, s1b, p0a, p0b);

#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float l_tot = lacc[b][0];
    bool bad = !(l_tot < 1e30f) || !(l_tot > 0.f);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) bad |= !(fabsf(oacc[b][u][r]) < 3e38f);
    if (qrow[b] < L) {
      bf16* O = reinterpret_cast<bf16*>(a.o) + (((int64_t)s_idx * L + qrow[b]) * a.H + head) * 64;
      if (bad) {  // rare: scores ran out of the fixed offset's range -> exact per-row recompute
        float o[64];
        attn_row_exact(a, Q, K, V, qrow[b], klen, qscale, o);
        if (h == 0)
          for (int d = 0; d < 64; ++d) O[d] = f2bf(o[d]);
      } else {
        const float inv = 1.f / l_tot;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            bf16x4 w = {f2bf(oacc[b][u][4 * r4 + 0] * inv), f2bf(oacc[b][u][4 * r4 + 1] * inv),
                        f2bf(oacc[b][u][4 * r4 + 2] * inv), f2bf(oacc[b][u][4 * r4 + 3] * inv)};
            *reinterpret_cast<bf16x4*>(O + 32 * u + 8 * r4 + 4 * h) = w;
          }
      }
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

static int g_attn_variant = -1;
hipError_t attn_read_stamps(uint64_t* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), sizeof(uint64_t) * (n < 256 ? n : 256));
}
void attn_force_variant(int v) { g_attn_variant = v; }

hipError_t attention(int compute, const AttnArgs& a, hipStream_t st) {
  if (a.S <= 0 || a.H <= 0 || a.L <= 0) return hipErrorInvalidValue;
  if (compute) {
    static int env_ver = [] { const char* e = getenv("F5H_ATTN_V"); return e ? atoi(e) : -1; }();
    // default v2: exact running max (lazy rescale), row sums on MFMA; the others are kept as
    // measured alternatives (tools/attn_ab.py) and are covered by the parity tests
    const int ver = g_attn_variant > 0 ? g_attn_variant : (env_ver > 0 ? env_ver : 2);
    if (ver == 9) {
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v7_kernel<true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v7_kernel<false>), grid, dim3(256), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 8) {  // v6 diagnostic build with stamps
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v6_kernel<true, true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v6_kernel<false, true>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 7) {
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v6_kernel<true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v6_kernel<false>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 6) {  // v5 diagnostic build with per-segment cycle stamps
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v5_kernel<true, true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v5_kernel<false, true>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 5) {
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v5_kernel<true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v5_kernel<false>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 4) {
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v4_kernel<true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v4_kernel<false>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 3) {
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v3_kernel<true>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v3_kernel<false>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 26) {  // v9: v8 + early K reads (5-slot ring)
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v9_kernel<true, 8>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v9_kernel<false, 8>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 25) {  // v8: software-pipelined v2
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v8_kernel<true, 8>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v8_kernel<false, 8>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 27) {  // v2 with one barrier per two K/V tiles
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 8, 4>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 8, 4>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 23) {  // v2 lean: QK chains start from a -m_run operand, v_max3 row max
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 8, 3>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 8, 3>), grid, dim3(512), 0, st, a);
      return hipGetLastError();
    }
    if (ver == 21 || ver == 22) {  // v2 with wave-priority schedules (measured alternatives)
      dim3 grid((a.L + 255) / 256, a.S * a.H);
      if (ver == 21) {
        if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 8, 1>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 8, 1>), grid, dim3(512), 0, st, a);
      } else {
        if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 8, 2>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 8, 2>), grid, dim3(512), 0, st, a);
      }
      return hipGetLastError();
    }
    if (ver == 2 || ver == 24) {
      const int nw = ver == 24 ? 4 : 8;
      dim3 grid((a.L + 32 * nw - 1) / (32 * nw), a.S * a.H);
      if (nw == 8) {
        if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 8>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 8>), grid, dim3(512), 0, st, a);
      } else {
        if (a.prescaled) hipLaunchKernelGGL((attn_bf16_v2_kernel<true, 4>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((attn_bf16_v2_kernel<false, 4>), grid, dim3(256), 0, st, a);
      }
      return hipGetLastError();
    }
    dim3 grid((a.L + 127) / 128, a.S * a.H);
    static int dbg = [] { const char* e = getenv("F5H_ATTN_DBG"); return e ? atoi(e) : 0; }();
#define F5H_ATTN_LAUNCH(P, D) hipLaunchKernelGGL((attn_bf16_kernel<P, D>), grid, dim3(256), 0, st, a)
    if (a.prescaled) {
      switch (dbg) {
        case 1: F5H_ATTN_LAUNCH(true, 1); break;
        case 2: F5H_ATTN_LAUNCH(true, 2); break;
        case 3: F5H_ATTN_LAUNCH(true, 3); break;
        default: F5H_ATTN_LAUNCH(true, 0);
      }
    } else {
      switch (dbg) {
        case 1: F5H_ATTN_LAUNCH(false, 1); break;
        case 2: F5H_ATTN_LAUNCH(false, 2); break;
        case 3: F5H_ATTN_LAUNCH(false, 3); break;
        default: F5H_ATTN_LAUNCH(false, 0);
      }
    }
#undef F5H_ATTN_LAUNCH
  } else {
    dim3 grid((a.L + 63) / 64, a.S * a.H);
    hipLaunchKernelGGL(attn_f32_kernel, grid, dim3(64), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace f5h
