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

namespace f5h {

template <bool PRESCALED>
__global__ __launch_bounds__(256, 2) void attn_bf16_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * 2 * 64 * 8];  // [buf][K|V][64 rows][8 chunks]
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

  // staging registers as named scalars (an array here is lowered to scratch memory)
  uint4 rk0, rk1, rv0, rv1;
  const int srow = tid >> 3, sch = tid & 7;  // this thread's chunk: rows srow and srow+32
  auto gload = [&](int kt) {
    // keys past L are clamped to a real row: their scores are masked (p = 0) below
    const int64_t o0 = (int64_t)min(kt * 64 + srow, L - 1) * 64 + sch * 8;
    const int64_t o1 = (int64_t)min(kt * 64 + srow + 32, L - 1) * 64 + sch * 8;
    rk0 = *reinterpret_cast<const uint4*>(K + o0);
    rk1 = *reinterpret_cast<const uint4*>(K + o1);
    rv0 = *reinterpret_cast<const uint4*>(V + o0);
    rv1 = *reinterpret_cast<const uint4*>(V + o1);
  };
  const int sw0 = srow * 8 + swz128(srow, sch), sw1 = (srow + 32) * 8 + swz128(srow + 32, sch);
  auto sstore = [&](int buf) {
    uint4* Ks = lds + buf * 1024;
    uint4* Vs = Ks + 512;
    Ks[sw0] = rk0;
    Ks[sw1] = rk1;
    Vs[sw0] = rv0;
    Vs[sw1] = rv1;
  };

  const float c = a.scale * 1.4426950408889634f;  // scores in log2 units (unless q carries it)
  float m_run = -INFINITY, l_run = 0.f;
  f32x16 oacc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[u][r] = 0.f;

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < ntile; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ntile) gload(kt + 1);
    const uint4* Ks = lds + cur * 1024;
    const uint4* Vs = Ks + 512;

    // ---- S^T = K Q^T (two 32-key sub-tiles)
    f32x16 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[t][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        int row = t * 32 + (lane & 31);
        uint4 kv = Ks[row * 8 + swz128(row, ks * 2 + h)];
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kv), qf[ks], sacc[t], 0, 0,
                                                           0);
      }
    }
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
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
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

    const int G = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const char* vbytes = reinterpret_cast<const char*>(Vs);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int dh = 32 * u + 16 * (G & 1) + 4 * p4;
      const int chunk = dh >> 3, half = (dh >> 2) & 1;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r1 = 32 * t + 16 * s + 4 * (G >> 1) + q4, r2 = r1 + 8;
          const char* a1 = vbytes + r1 * 128 + swz128(r1, chunk) * 16 + half * 8;
          const char* a2 = vbytes + r2 * 128 + swz128(r2, chunk) * 16 + half * 8;
          s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(a1));
          s16x4 v2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(a2));
          bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v1, v2, 0, 1, 2, 3, 4, 5, 6, 7));
          oacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[t][s], oacc[u], 0, 0, 0);
        }
    }
    if (kt + 1 < ntile) {
      __syncthreads();
      sstore(cur ^ 1);
      __syncthreads();
    }
  }
  // ---- epilogue: O row = query on lane; dh = 32u + 8*r4 + 4h + c
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
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
    if (a.prescaled)
      hipLaunchKernelGGL(attn_bf16_kernel<true>, grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(attn_bf16_kernel<false>, grid, dim3(256), 0, st, a);
  } else {
    dim3 grid((a.L + 63) / 64, a.S * a.H);
    hipLaunchKernelGGL(attn_f32_kernel, grid, dim3(64), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace f5h
