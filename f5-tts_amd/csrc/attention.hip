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

template <bool PRESCALED, int DBG>
__global__ __launch_bounds__(256, 2) void attn_bf16_kernel(AttnArgs a) {
  constexpr int TILE_B = 2 * 64 * 128;  // K + V tile bytes (64 keys x 64 dh bf16 each)
  constexpr int NS = 3;                 // LDS ring: one tile read while two are in flight
  constexpr int DPS = 4;                // DMA instructions per tile per wave (K 2 + V 2)
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * TILE_B / 16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5;  // lane half
  const int bh = blockIdx.y;
  const int s_idx = bh / a.H, head = bh - s_idx * a.H;
  const int L = a.L;
  const int64_t base = (int64_t)bh * L * 64;
  const bf16* Q = reinterpret_cast<const bf16*>(a.q) + base;
  const bf16* K = reinterpret_cast<const bf16*>(a.k) + base;
  const bf16* V = reinterpret_cast<const bf16*>(a.v) + base;
  int klen = L;
  if (a.kv_len) klen = min(klen, a.kv_len[s_idx]);
  const int ntile = (klen + 63) / 64;

  const int qrow = blockIdx.x * 128 + wid * 32 + (lane & 31);
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
}

// ---------------------------------------------------------------- fp32 parity kernel
__global__ __launch_bounds__(64) void attn_f32_kernel(AttnArgs a) {
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
}

hipError_t attention(int compute, const AttnArgs& a, hipStream_t st) {
  if (a.S <= 0 || a.H <= 0 || a.L <= 0) return hipErrorInvalidValue;
  if (compute) {
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
