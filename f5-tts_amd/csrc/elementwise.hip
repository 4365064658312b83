// Row-wise and elementwise kernels of the CFM hot path (HBM-bound; one wave per row,
// 16-byte vector accesses). Each cites the reference op it restates.
#include "common.h"
#include "kernels.h"
#include "lnrow.h"

#include <algorithm>

namespace f5h {

static inline unsigned nblk(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// ---------------------------------------------------------------- time embedding
// SinusPositionEmbedding(256), scale 1000 (modules.py:157-169): [sin | cos](1000 t e^{-i ln1e4/127})
struct TVals {  // up to 512 NFE steps: 513 grid points (kernel-argument payload, 2 KB)
  float t[513];
};
__global__ void time_sinus_kernel(TVals tv, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 128) return;
  int r = i / 128, j = i % 128;
  const float k = logf(10000.f) / 127.f;
  float f = expf((float)j * -k);
  float e = (1000.f * tv.t[r]) * f;
  out[r * 256 + j] = sinf(e);
  out[r * 256 + 128 + j] = cosf(e);
}
// t_host: host array of n <= 512 time values, passed by value in the kernel arguments
// (no host->device copy, so the launch is graph-capturable).
hipError_t time_sinus(const float* t_host, int n, float* out, hipStream_t st) {
  if (n <= 0 || n > 512) return hipErrorInvalidValue;
  TVals tv{};
  for (int i = 0; i < n; ++i) tv.t[i] = t_host[i];
  hipLaunchKernelGGL(time_sinus_kernel, dim3(nblk(n * 128, 256)), dim3(256), 0, st, tv, n, out);
  return hipGetLastError();
}

// The same from the device copy of the grid (the prologue graph: no host values baked in)
__global__ void time_sinus_dev_kernel(const float* tg, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 128) return;
  int r = i / 128, j = i % 128;
  const float k = logf(10000.f) / 127.f;
  float f = expf((float)j * -k);
  float e = (1000.f * tg[r]) * f;
  out[r * 256 + j] = sinf(e);
  out[r * 256 + 128 + j] = cosf(e);
}
hipError_t time_sinus_dev(const float* tg, int n, float* out, hipStream_t st) {
  if (n <= 0 || n > 512) return hipErrorInvalidValue;
  hipLaunchKernelGGL(time_sinus_dev_kernel, dim3(nblk(n * 128, 256)), dim3(256), 0, st, tg, n, out);
  return hipGetLastError();
}

// The ODE grid t[0..n-1] into device memory (kernel-argument upload, capturable).
__global__ void grid_upload_kernel(TVals tv, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = tv.t[i];
}
// A host pointer value into a device slot (kernel-argument upload, stream-ordered).
__global__ void ptr_upload_kernel(float* p, float** slot) {
  if (threadIdx.x == 0) slot[0] = p;
}
hipError_t ptr_upload(float* p, float** slot, hipStream_t st) {
  hipLaunchKernelGGL(ptr_upload_kernel, dim3(1), dim3(64), 0, st, p, slot);
  return hipGetLastError();
}
hipError_t grid_upload(const float* t_host, int n, float* out, hipStream_t st) {
  if (n <= 0 || n > 513) return hipErrorInvalidValue;
  TVals tv{};
  for (int i = 0; i < n; ++i) tv.t[i] = t_host[i];
  hipLaunchKernelGGL(grid_upload_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, tv, n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- NFE-step bookkeeping
// One NFE step is a fixed launch sequence (hipGraph-replayable): step_begin copies the step's
// row of a per-call table (AdaLN shift/scale/gate rows, or the UNetT time token) to a fixed
// buffer; step_advance bumps the device-side step index after the Euler update.
__global__ void step_begin_kernel(const int* kstep, const float* src, int64_t stride, int n, float* dst) {
  const int k = *kstep;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i * 4 < n) {
    const float4* s = reinterpret_cast<const float4*>(src + (int64_t)k * stride);
    reinterpret_cast<float4*>(dst)[i] = s[i];
  }
}
hipError_t step_begin(const int* kstep, const float* src, int64_t stride, int n, float* dst, hipStream_t st) {
  if (n % 4 || stride % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(step_begin_kernel, dim3(nblk(n / 4, 256)), dim3(256), 0, st, kstep, src, stride, n, dst);
  return hipGetLastError();
}
// Probe stamps (device wall clock, s_memrealtime) around a launch that does not stamp itself:
// same slot layout as the in-kernel probe (kernels.h).
__global__ void stamp_begin_kernel(unsigned long long* slots, const int* tick) {
  const int k = *tick;
  if (threadIdx.x == 0 && k >= 0 && k < kProbeTicks && k % kProbeEvery == 0) atomicMin(slots + probe_slot(k), (unsigned long long)wall_clock64());
}
__global__ void stamp_end_kernel(unsigned long long* slots, const int* tick) {
  const int k = *tick;
  if (threadIdx.x == 0 && k >= 0 && k < kProbeTicks && k % kProbeEvery == 0)
    atomicMax(slots + kProbeEnd + probe_slot(k), (unsigned long long)wall_clock64());
}
hipError_t stamp_begin(unsigned long long* slots, const int* tick, hipStream_t st) {
  hipLaunchKernelGGL(stamp_begin_kernel, dim3(1), dim3(64), 0, st, slots, tick);
  return hipGetLastError();
}
hipError_t stamp_end(unsigned long long* slots, const int* tick, hipStream_t st) {
  hipLaunchKernelGGL(stamp_end_kernel, dim3(1), dim3(64), 0, st, slots, tick);
  return hipGetLastError();
}
__global__ void step_advance_kernel(int* kstep, int* tick) {
  if (threadIdx.x == 0) {
    kstep[0] += 1;
    tick[0] += 1;
  }
}
hipError_t step_advance(int* kstep, int* tick, hipStream_t st) {
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, st, kstep, tick);
  return hipGetLastError();
}

// ---------------------------------------------------------------- LayerNorm fold: per-step u / v vectors
// (kernels.h LnFoldArgs). u_s[n] = sum_k (1 + scale_s[k]) W[n][k] and v_s[n] = sum_k shift_s[k] W[n][k], for the
// 16 steps of a step group: a [16 steps x d] . [d x 64 columns] product per wave, on the matrix pipes. The fp32
// (1 + scale) and shift rows enter as two 16-bit parts each (hi = the rounded value, lo = the rounded remainder:
// ~2^-16 relative to the value with bf16, ~2^-22 with fp16) accumulated into the same fp32 sums; W in its own 16-bit
// type. Wave = (step group, 64 output columns of W1 or Wqkv, layer): four 16x16 column tiles, u and v, so every W
// element is read once per step group (230 MB at C2: the kernel's floor is that read). Operands straight from
// global memory (a lane's 16 B of a W row and 32 B of each table row per 32 k), two K steps' loads in flight.
// Earlier r06 forms: VALU FMAs on LDS-staged operands (~280 us per C2 call), then one operand part per wave (four
// waves re-reading every W element: 160-180 us).
template <typename T>
__global__ __launch_bounds__(256) void lnfold_uv_kernel(LnFoldArgs a) {
  typedef typename Op16<T>::v8 v8;
  const int lane = threadIdx.x & 63;
  const int d = a.d, F = a.F, nbF = F / 64, nb = nbF + 3 * d / 64, ng = (a.nfe + 15) / 16;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wv >= a.depth * nb * ng) return;  // whole wave
  const int g = wv % ng, j = (wv / ng) % nb, l = wv / (ng * nb);
  const bool ff = j < nbF;
  const int n0 = (ff ? j : j - nbF) * 64;
  const T* wr = reinterpret_cast<const T*>(ff ? a.w1[l] : a.wqkv[l]) + (int64_t)(n0 + (lane & 15)) * d + 8 * (lane >> 4);
  // AdaLN row layout per layer (modules.py:321-323): shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp
  const int64_t sh_off = (int64_t)l * 6 * d + (ff ? 3 : 0) * d, sc_off = sh_off + d;
  const float* ar = a.table + (int64_t)min(g * 16 + (lane & 15), a.nfe - 1) * a.stride + 8 * (lane >> 4);
  f32x4 acc[2][4] = {};
  auto parts = [](const float4& p0, const float4& p1, float one, v8& hi, v8& lo) {
    const float xv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = one + xv[e];
      hi[e] = from_f32<T>(x);
      lo[e] = from_f32<T>(x - to_f32(hi[e]));
    }
  };
  for (int k0 = 0; k0 < d; k0 += 64) {  // d % 64 == 0
    float4 xs[2][2], xh[2][2];
    v8 b[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = k0 + 32 * u;
      xs[u][0] = *reinterpret_cast<const float4*>(ar + sc_off + k);
      xs[u][1] = *reinterpret_cast<const float4*>(ar + sc_off + k + 4);
      xh[u][0] = *reinterpret_cast<const float4*>(ar + sh_off + k);
      xh[u][1] = *reinterpret_cast<const float4*>(ar + sh_off + k + 4);
#pragma unroll
      for (int t = 0; t < 4; ++t) b[u][t] = *reinterpret_cast<const v8*>(wr + (int64_t)t * 16 * d + k);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v8 shi, slo, hhi, hlo;
      parts(xs[u][0], xs[u][1], 1.f, shi, slo);
      parts(xh[u][0], xh[u][1], 0.f, hhi, hlo);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[0][t] = Op16<T>::mma16(shi, b[u][t], acc[0][t]);
        acc[1][t] = Op16<T>::mma16(hhi, b[u][t], acc[1][t]);
        acc[0][t] = Op16<T>::mma16(slo, b[u][t], acc[0][t]);
        acc[1][t] = Op16<T>::mma16(hlo, b[u][t], acc[1][t]);
      }
    }
  }
  // acc[uv][t][r]: step g*16 + 4 (lane >> 4) + r, column n0 + 16 t + (lane & 15)
  const int64_t LW = 2 * (int64_t)F + 6 * (int64_t)d;
  const int64_t u_off = a.out_off + l * LW + (ff ? 0 : 2 * (int64_t)F), v_off = u_off + (ff ? F : 3 * d);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = g * 16 + 4 * (lane >> 4) + r;
      if (s < a.nfe) {
        float* o = a.table + (int64_t)s * a.stride + n0 + 16 * t + (lane & 15);
        o[u_off] = acc[0][t][r];
        o[v_off] = acc[1][t][r];
      }
    }
}
hipError_t lnfold_uv(int compute, const LnFoldArgs& a, hipStream_t st) {
  if (a.d % 64 || a.F % 64 || a.nfe <= 0 || a.depth <= 0) return hipErrorInvalidValue;
  const dim3 grid((a.depth * (a.F / 64 + 3 * a.d / 64) * ((a.nfe + 15) / 16) + 3) / 4), block(256);
  if (compute == F5H_C_BF16)
    hipLaunchKernelGGL(lnfold_uv_kernel<bf16>, grid, block, 0, st, a);
  else if (compute == F5H_C_FP16)
    hipLaunchKernelGGL(lnfold_uv_kernel<f16>, grid, block, 0, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// p[0..n) = 0 by vector stores (the phase chain's arrival counters, zeroed ahead of every step)
__global__ void zero_words_kernel(uint4* p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = uint4{0u, 0u, 0u, 0u};
}
hipError_t zero_words(unsigned* p, int64_t n, hipStream_t st) {
  if (n % 4 || ((uintptr_t)p & 15)) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)std::min<int64_t>(64, nblk(n4, 256))), dim3(256), 0, st,
                     reinterpret_cast<uint4*>(p), n4);
  return hipGetLastError();
}

template <typename TO>
__global__ void silu_kernel(const float* x, TO* y, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = from_f32<TO>(silu(x[i]));
}
hipError_t silu_to_op(int compute, const float* x, void* y, int64_t n, hipStream_t st) {
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(silu_kernel<T>, dim3(nblk(n, 256)), dim3(256), 0, st, x, (T*)y, n););
  return hipGetLastError();
}

// ---------------------------------------------------------------- norms
// One wave per row, row cached in registers. NV = float4 per lane: compile-time for the widths the
// path uses (d = 256*NV), so every load is unconditional; d <= 2048, d % 4 == 0 otherwise.
constexpr int MAXV = 8;  // float4 per lane

// LayerNorm(no affine, eps 1e-6) * (1 + scale) + shift (AdaLayerNorm modules.py:325, ff_norm :753,
// AdaLayerNorm_Final :346), a wave per row (ln_mod_row, lnrow.h). The modulation rows are loaded with
// the row, before the reductions. TI: the residual stream's type (fp32, or the operand dtype on the
// 16-bit DiT path).
template <typename TO, int NV, typename TI = float>
__global__ __launch_bounds__(256) void ln_mod_kernel(const TI* h, int M, int d, const float* shift,
                                                     const float* scale, TO* out) {
  constexpr bool FIXED = NV > 0;
  constexpr int V = FIXED ? NV : MAXV;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const TI* x = h + (int64_t)row * d;
  const float4* sh = reinterpret_cast<const float4*>(shift);
  const float4* sc = reinterpret_cast<const float4*>(scale);
  const int n4 = FIXED ? 64 * NV : d >> 2;
  float4 v[V], a[V], b[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = lane + 64 * k;
    const bool ok = FIXED || i < n4;
    v[k] = ok ? load4f<TI>(x + 4 * i) : make_float4(0, 0, 0, 0);
    a[k] = ok ? sc[i] : make_float4(0, 0, 0, 0);
    b[k] = ok ? sh[i] : make_float4(0, 0, 0, 0);
  }
  ln_mod_row<TO, V, FIXED>(v, a, b, lane, n4, d, out + (int64_t)row * d);
}
// 16-bit residual stream at d = 1024: lane l holds elements 8(l + 64k) .. +7 (k < 2), so the row and the
// output move as 16-byte accesses (two per lane instead of four 8-byte ones)
template <typename T>
__global__ __launch_bounds__(256) void ln_mod16_kernel(const T* h, int M, const float* shift, const float* scale,
                                                       T* out) {
  constexpr int d = 1024;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const uint4* x = reinterpret_cast<const uint4*>(h + (int64_t)row * d);
  const float4* sh = reinterpret_cast<const float4*>(shift);
  const float4* sc = reinterpret_cast<const float4*>(scale);
  uint4 xv[2], o[2];
  float4 a[2][2], b[2][2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = lane + 64 * k;
    xv[k] = x[c];
    a[k][0] = sc[2 * c];
    a[k][1] = sc[2 * c + 1];
    b[k][0] = sh[2 * c];
    b[k][1] = sh[2 * c + 1];
  }
  ln16_row<T>(xv, a, b, o);
  uint4* op = reinterpret_cast<uint4*>(out + (int64_t)row * d);
#pragma unroll
  for (int k = 0; k < 2; ++k) op[lane + 64 * k] = o[k];
}

hipError_t ln_modulate(int compute, const void* hv, int h16, int M, int d, const float* shift, const float* scale,
                       void* out, hipStream_t st) {
  if (d % 4 || d > 4 * 64 * MAXV) return hipErrorInvalidValue;
  const dim3 g(nblk(M, 4)), b(256);
  if (h16) {  // 16-bit residual stream: input and output in the operand dtype
    if (compute != F5H_C_BF16 && compute != F5H_C_FP16) return hipErrorInvalidValue;
    auto run = [&](auto tag) {
      typedef decltype(tag) T;
      const T* x = (const T*)hv;
      switch (d) {
        case 1024: hipLaunchKernelGGL((ln_mod16_kernel<T>), g, b, 0, st, x, M, shift, scale, (T*)out); break;
        case 768: hipLaunchKernelGGL((ln_mod_kernel<T, 3, T>), g, b, 0, st, x, M, d, shift, scale, (T*)out); break;
        case 512: hipLaunchKernelGGL((ln_mod_kernel<T, 2, T>), g, b, 0, st, x, M, d, shift, scale, (T*)out); break;
        default: hipLaunchKernelGGL((ln_mod_kernel<T, 0, T>), g, b, 0, st, x, M, d, shift, scale, (T*)out);
      }
    };
    if (compute == F5H_C_BF16)
      run(bf16{});
    else
      run(f16{});
    return hipGetLastError();
  }
  const float* h = (const float*)hv;
  switch (d) {
    case 1024: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((ln_mod_kernel<T, 4>), g, b, 0, st, h, M, d, shift, scale, (T*)out);); break;
    case 768: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((ln_mod_kernel<T, 3>), g, b, 0, st, h, M, d, shift, scale, (T*)out);); break;
    case 512: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((ln_mod_kernel<T, 2>), g, b, 0, st, h, M, d, shift, scale, (T*)out);); break;
    default: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((ln_mod_kernel<T, 0>), g, b, 0, st, h, M, d, shift, scale, (T*)out););
  }
  return hipGetLastError();
}

// x_transformers RMSNorm: F.normalize(x, dim=-1) * sqrt(d) * g (unett.py:156,160,185)
template <typename TO, int NV, typename TI = float>
__global__ __launch_bounds__(256) void rms_kernel(const TI* h, int M, int d, const float* g, TO* out) {
  constexpr bool FIXED = NV > 0;
  constexpr int V = FIXED ? NV : MAXV;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const TI* x = h + (int64_t)row * d;
  const float4* gg = reinterpret_cast<const float4*>(g);
  const int n4 = FIXED ? 64 * NV : d >> 2;
  float4 v[V], a[V];
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = lane + 64 * k;
    const bool ok = FIXED || i < n4;
    v[k] = ok ? load4f<TI>(x + 4 * i) : make_float4(0, 0, 0, 0);
    a[k] = ok ? gg[i] : make_float4(0, 0, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < V; ++k) q += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  const float nrm = fmaxf(sqrtf(wave_sum_dpp(q)), 1e-12f);
  const float f = sqrtf((float)d);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = lane + 64 * k;
    if (FIXED || i < n4)
      store4<TO>(out + (int64_t)row * d + 4 * i, v[k].x / nrm * f * a[k].x, v[k].y / nrm * f * a[k].y,
                 v[k].z / nrm * f * a[k].z, v[k].w / nrm * f * a[k].w);
  }
}
// 16-bit residual stream at d = 1024: 16-byte row accesses, lane l holding elements 8(l + 64k) .. +7 (k < 2)
template <typename T>
__global__ __launch_bounds__(256) void rms16_kernel(const T* h, int M, const float* g, T* out) {
  typedef typename Op16<T>::v8 v8;
  constexpr int d = 1024;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const uint4* x = reinterpret_cast<const uint4*>(h + (int64_t)row * d);
  const float4* gg = reinterpret_cast<const float4*>(g);
  float v[2][8];
  float4 a[2][2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = lane + 64 * k;
    const v8 w = __builtin_bit_cast(v8, x[c]);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[k][e] = to_f32(w[e]);
    a[k][0] = gg[2 * c];
    a[k][1] = gg[2 * c + 1];
  }
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) q += v[k][e] * v[k][e];
  const float nrm = fmaxf(sqrtf(wave_sum_dpp(q)), 1e-12f);
  const float f = sqrtf((float)d);
  uint4* o = reinterpret_cast<uint4*>(out + (int64_t)row * d);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float av[8] = {a[k][0].x, a[k][0].y, a[k][0].z, a[k][0].w, a[k][1].x, a[k][1].y, a[k][1].z, a[k][1].w};
    v8 w;
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = from_f32<T>(v[k][e] / nrm * f * av[e]);
    o[lane + 64 * k] = __builtin_bit_cast(uint4, w);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void scale_cols_kernel(const T* W, int64_t n8, int K, const float* g, T* out) {
  typedef typename Op16<T>::v8 v8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int k0 = (int)((i * 8) % K);
    const v8 w = reinterpret_cast<const v8*>(W)[i];
    v8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = from_f32<T>(to_f32(w[e]) * g[k0 + e]);
    reinterpret_cast<v8*>(out)[i] = o;
  }
}
hipError_t scale_cols(int compute, const void* W, int64_t rows, int K, const float* g, void* out, hipStream_t st) {
  if (K % 8 || rows <= 0) return hipErrorInvalidValue;
  const int64_t n8 = rows * K / 8;
  const dim3 gr((unsigned)std::min<int64_t>((n8 + 255) / 256, 4096)), b(256);
  if (compute == F5H_C_BF16)
    hipLaunchKernelGGL(scale_cols_kernel<bf16>, gr, b, 0, st, (const bf16*)W, n8, K, g, (bf16*)out);
  else if (compute == F5H_C_FP16)
    hipLaunchKernelGGL(scale_cols_kernel<f16>, gr, b, 0, st, (const f16*)W, n8, K, g, (f16*)out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t rms_norm_g(int compute, const void* hv, int h16, int M, int d, const float* g, void* out, hipStream_t st) {
  if (d % 4 || d > 4 * 64 * MAXV) return hipErrorInvalidValue;
  const dim3 gr(nblk(M, 4)), b(256);
  if (h16) {  // 16-bit residual stream (UNetT in the 16-bit modes): input and output in the operand dtype
    if (compute != F5H_C_BF16 && compute != F5H_C_FP16) return hipErrorInvalidValue;
    auto run = [&](auto tag) {
      typedef decltype(tag) T;
      const T* x = (const T*)hv;
      switch (d) {
        case 1024: hipLaunchKernelGGL((rms16_kernel<T>), gr, b, 0, st, x, M, g, (T*)out); break;
        case 512: hipLaunchKernelGGL((rms_kernel<T, 2, T>), gr, b, 0, st, x, M, d, g, (T*)out); break;
        default: hipLaunchKernelGGL((rms_kernel<T, 0, T>), gr, b, 0, st, x, M, d, g, (T*)out);
      }
    };
    if (compute == F5H_C_BF16)
      run(bf16{});
    else
      run(f16{});
    return hipGetLastError();
  }
  const float* h = (const float*)hv;
  switch (d) {
    case 1024: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((rms_kernel<T, 4>), gr, b, 0, st, h, M, d, g, (T*)out);); break;
    case 512: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((rms_kernel<T, 2>), gr, b, 0, st, h, M, d, g, (T*)out);); break;
    default: F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL((rms_kernel<T, 0>), gr, b, 0, st, h, M, d, g, (T*)out););
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- rotary table
// x_transformers RotaryEmbedding(64): inv_freq_j = 1/10000^(2j/64), freqs[n,2j]=freqs[n,2j+1]=n*inv_freq_j
__global__ void rope_kernel(int L, float2* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L * 32) return;
  int pos = i >> 5, j = i & 31;
  float inv = 1.f / powf(10000.f, (float)(2 * j) / 64.f);
  float f = (float)pos * inv;
  out[i] = make_float2(cosf(f), sinf(f));
}
hipError_t rope_table(int L, float2* out, hipStream_t st) {
  hipLaunchKernelGGL(rope_kernel, dim3(nblk(L * 32, 256)), dim3(256), 0, st, L, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- text embedding
// TextEmbedding.forward (dit.py:86-120): tok+1 (filler 0), truncate/pad to N, per-sample
// valid mask (batched path), fill mask taken BEFORE drop_text, Embedding, + freqs_cis, masked_fill.
__global__ void text_embed_kernel(TextEmbArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= a.B * a.N) return;
  const int b = row / a.N, n = row - b * a.N;
  const bool valid = !a.seq_len || n < a.seq_len[b];
  int tok = n < a.nt ? (int)a.text[(int64_t)b * a.nt + n] + 1 : 0;
  if (!valid) tok = 0;
  const bool fill = tok == 0;
  const bool zero_row = a.mask_padding && a.freqs && fill;  // masked_fill only with extra modeling
  if (a.keep && lane == 0) {
    a.keep[row] = zero_row ? 0 : 1;
    a.keep[a.B * a.N + row] = zero_row ? 0 : 1;
  }
  for (int c = lane; c < a.td; c += 64) {
    float ec = valid ? a.table[(int64_t)tok * a.td + c] : 0.f;
    float eu = valid ? a.table[c] : 0.f;  // drop_text -> id 0
    if (a.freqs) {
      float f = valid ? a.freqs[(int64_t)n * a.td + c] : 0.f;
      ec += f;
      eu += f;
    }
    if (zero_row) ec = eu = 0.f;
    a.out_c[(int64_t)row * a.td + c] = ec;
    a.out_u[(int64_t)row * a.td + c] = eu;
  }
}
hipError_t text_embed(const TextEmbArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(text_embed_kernel, dim3(nblk((int64_t)a.B * a.N, 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ConvNeXtV2Block front half (modules.py:260-264): depthwise Conv1d(k7, pad3) + bias -> LayerNorm(affine)
template <typename TO>
__global__ void dwconv_ln_kernel(const float* x, int S, int L, int C, const float* w, const float* bias,
                                 const float* lw, const float* lb, TO* out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= S * L) return;
  const int s = row / L, n = row - s * L;
  float v[16];  // C <= 1024
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int c = lane + 64 * k;
    float acc = 0.f;
    if (c < C) {
      acc = bias[c];
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        int q = n + t - 3;
        if (q >= 0 && q < L) acc += w[c * 7 + t] * x[((int64_t)s * L + q) * C + c];
      }
    }
    v[k] = acc;
    sum += acc;
  }
  const float mean = wave_sum(sum) / C;
  float q2 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int c = lane + 64 * k;
    if (c < C) q2 += (v[k] - mean) * (v[k] - mean);
  }
  const float rstd = rsqrtf(wave_sum(q2) / C + 1e-6f);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    int c = lane + 64 * k;
    if (c < C) out[(int64_t)row * C + c] = from_f32<TO>((v[k] - mean) * rstd * lw[c] + lb[c]);
  }
}
hipError_t dwconv_ln(int compute, const float* x, int S, int L, int C, const float* dw_w, const float* dw_b,
                     const float* ln_w, const float* ln_b, void* out, hipStream_t st) {
  if (C > 1024) return hipErrorInvalidValue;
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(dwconv_ln_kernel<T>, dim3(nblk(S * L, 4)), dim3(256), 0, st, x, S, L, C, dw_w, dw_b, ln_w, ln_b, (T*)out););
  return hipGetLastError();
}

// GRN (modules.py:236-245): Gx = ||x||_2 over the TIME axis, Nx = Gx / (mean_c Gx + 1e-6),
// out = gamma * (x * Nx) + beta + x
// Deterministic two-stage column reduction: partial[z][s][c] over 64-row chunks, then a
// fixed-order sum (no float atomics: results must not depend on arrival order).
__global__ void grn_sumsq_kernel(const float* x, int S, int L, int C, float* partial) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y, z = blockIdx.z;
  if (c >= C) return;
  const int n0 = z * 64, n1 = min(L, n0 + 64);
  float acc = 0.f;
  for (int n = n0; n < n1; ++n) {
    float v = x[((int64_t)s * L + n) * C + c];
    acc += v * v;
  }
  partial[((int64_t)z * S + s) * C + c] = acc;
}
// nx[s][c] = Gx / (mean_c Gx + 1e-6), Gx = sqrt(sum_z partial)
__global__ __launch_bounds__(1024) void grn_norm_kernel(const float* partial, int nz, int S, int C, float* nx) {
  // one 1024-thread block per sequence, one channel per thread: the nz partials of a channel are
  // independent loads (kept in flight together), the channel mean is a block reduction
  const int s = blockIdx.x;
  float acc = 0.f;
  for (int c = threadIdx.x; c < C; c += 1024) {
    float ss = 0.f;
#pragma unroll 8
    for (int z = 0; z < nz; ++z) ss += partial[((int64_t)z * S + s) * C + c];
    const float g = sqrtf(ss);  // ||x||_2 over time
    nx[(int64_t)s * C + c] = g;
    acc += g;
  }
  __shared__ float red[16];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) tot += red[w];  // fixed order: deterministic
  const float mean = tot / C;
  for (int c = threadIdx.x; c < C; c += 1024) nx[(int64_t)s * C + c] = nx[(int64_t)s * C + c] / (mean + 1e-6f);
}
template <typename TO>
__global__ void grn_apply_kernel(const float* x, int L, int C, const float* nx, const float* gamma,
                                 const float* beta, TO* out, int64_t total) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int c = (int)(i % C);
  int s = (int)(i / ((int64_t)L * C));
  float v = x[i];
  out[i] = from_f32<TO>(gamma[c] * (v * nx[(int64_t)s * C + c]) + beta[c] + v);
}
hipError_t grn(int compute, const float* x, int S, int L, int C, const float* gamma, const float* beta,
               float* scratch, void* out, hipStream_t st) {
  // scratch: [nz*S*C] partials then [S*C] normalisers
  const int nz = (int)nblk(L, 64);
  float* nx = scratch + (size_t)nz * S * C;
  hipLaunchKernelGGL(grn_sumsq_kernel, dim3(nblk(C, 256), S, nz), dim3(256), 0, st, x, S, L, C, scratch);
  hipLaunchKernelGGL(grn_norm_kernel, dim3(S), dim3(1024), 0, st, scratch, nz, S, C, nx);
  scratch = nx;
  const int64_t total = (int64_t)S * L * C;
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(grn_apply_kernel<T>, dim3(nblk(total, 256)), dim3(256), 0, st, x, L, C, scratch, gamma, beta, (T*)out, total););
  return hipGetLastError();
}

// ---------------------------------------------------------------- input-projection operands
// A_ct row (s, n) = [step_cond (or 0 for the uncond branch, dit.py:155-156) pad->128 | text_e pad->tdp].
// Rows s < B are the conditional branch; a single-branch forward (cfg_infer=False, dit.py:347-350)
// may drop the audio cond (InputEmbedding drop_audio_cond) and/or use the dropped-text embedding.
template <typename TO>
__global__ void build_ct_kernel(const float* cond, const uint8_t* cmask, const float* tc, const float* tu, int B,
                                int N, int td, int tdp, int S, int drop_audio, int drop_text, TO* out) {
  const int64_t K = 128 + tdp;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * N * K) return;
  const int64_t row = i / K;
  const int col = (int)(i - row * K);
  const int s = (int)(row / N), n = (int)(row - (int64_t)s * N);
  const int b = s % B;
  float v = 0.f;
  if (col < 128) {
    if (col < 100 && s < B && !drop_audio && cmask[(int64_t)b * N + n]) v = cond[((int64_t)b * N + n) * 100 + col];
  } else if (col - 128 < td) {
    const float* t = (s < B && !drop_text) ? tc : tu;
    v = t[((int64_t)b * N + n) * td + (col - 128)];
  }
  out[i] = from_f32<TO>(v);
}
hipError_t build_ct(int compute, const float* cond, const uint8_t* cond_mask, const float* text_c,
                    const float* text_u, int B, int N, int td, int S, int drop_audio, int drop_text, void* out,
                    hipStream_t st) {
  const int tdp = (td + 63) / 64 * 64;
  const int64_t total = (int64_t)S * N * (128 + tdp);
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(build_ct_kernel<T>, dim3(nblk(total, 256)), dim3(256), 0, st, cond, cond_mask, text_c, text_u, B, N, td, tdp, S, drop_audio, drop_text, (T*)out););
  return hipGetLastError();
}

template <typename TO>
__global__ void pack_y_kernel(const float* y, int rows, int mel, TO* yp) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * 128) return;
  int64_t r = i >> 7;
  int c = (int)(i & 127);
  yp[i] = from_f32<TO>(c < mel ? y[r * mel + c] : 0.f);
}
hipError_t pack_y(int compute, const float* y, int rows, int mel, void* ypad, hipStream_t st) {
  const int64_t total = (int64_t)rows * 128;
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(pack_y_kernel<T>, dim3(nblk(total, 256)), dim3(256), 0, st, y, rows, mel, (T*)ypad););
  return hipGetLastError();
}

// ---------------------------------------------------------------- CFG + Euler update
// fn(t,x) = pred + (pred - null_pred) * cfg (cfm.py:190-191); torchdiffeq euler: y1 = y0 + dt * f
template <typename TO>
__global__ __launch_bounds__(256) void cfg_euler_kernel(EulerArgs a, TO* ypad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.N * a.mel;
  // read once: the last workgroup to arrive below bumps it. Every access to the step index and to the
  // arrival counter is atomic (agent scope), so the bump and these reads never race as plain accesses.
  const int k = a.kstep ? __hip_atomic_load(a.kstep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  if (a.kstep && a.next_dst) {
    // folded step bookkeeping (was a step_begin and a step_advance launch per NFE step): the next
    // step's table row, then (below, after the update) the step-index bump
    if (k + 1 < a.nfe) {
      const float4* src = reinterpret_cast<const float4*>(a.next_src + (int64_t)(k + 1) * a.next_stride);
      float4* dst = reinterpret_cast<float4*>(a.next_dst);
      for (int64_t j = i; j < a.next_n / 4; j += (int64_t)gridDim.x * blockDim.x) dst[j] = src[j];
    }
  }
  float dt = a.dt;
  float* traj = a.traj;
  if (a.kstep) {  // graph-replayable form: step index, grid and trajectory base live on the device
    dt = sub_nc(a.tgrid[k + 1], a.tgrid[k]);
    traj = a.trajp ? *a.trajp : nullptr;
    if (traj) traj += (int64_t)(k + 1) * total;
  }
  for (; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % a.mel);
    const int64_t bn = i / a.mel;
    const int b = (int)(bn / a.N), n = (int)(bn - (int64_t)b * a.N);
    const float pc = a.p[(int64_t)b * a.p_seq_stride + (int64_t)(a.p_row_off + n) * a.p_ld + c];
    float v = pc;
    if (a.use_cfg) {
      const float pu = a.p[(int64_t)(a.B + b) * a.p_seq_stride + (int64_t)(a.p_row_off + n) * a.p_ld + c];
      v = add_nc(pc, mul_nc(sub_nc(pc, pu), a.cfg));
    }
    const float y = add_nc(a.y[i], mul_nc(dt, v));
    a.y[i] = y;
    if (ypad) ypad[bn * 128 + c] = from_f32<TO>(y);
    if (traj) traj[i] = y;
  }
  if (a.kstep && a.arrive) {
    // every thread of this workgroup has read k above: the last workgroup to arrive bumps the step
    // index (and the probe tick) for the next step's launches
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x - 1) {
        __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(const_cast<int*>(a.kstep), k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.tick) __hip_atomic_fetch_add(a.tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}
hipError_t cfg_euler(const EulerArgs& a, hipStream_t st) {
  const int64_t total = (int64_t)a.B * a.N * a.mel;
  // at most 128 workgroups (a grid-stride loop covers the rest): the folded step-index bump costs one
  // same-word atomic per workgroup, which serialise (~90 per us, MI355X_MICROARCH.md dequeue)
  const unsigned blocks = std::min<unsigned>(128, std::max<unsigned>(1, nblk(total, 256)));
  F5H_OP_DISPATCH(a.compute, T, hipLaunchKernelGGL(cfg_euler_kernel<T>, dim3(blocks), dim3(256), 0, st, a, (T*)a.ypad););
  return hipGetLastError();
}

// out = where(cond_mask, cond, out) (cfm.py:223)
__global__ void final_where_kernel(const float* cond, const uint8_t* m, float* y, int64_t total, int mel) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  if (m[i / mel]) y[i] = cond[i];
}
hipError_t final_where(const float* cond, const uint8_t* cond_mask, float* y, int B, int N, int mel,
                       hipStream_t st) {
  const int64_t total = (int64_t)B * N * mel;
  hipLaunchKernelGGL(final_where_kernel, dim3(nblk(total, 256)), dim3(256), 0, st, cond, cond_mask, y, total, mel);
  return hipGetLastError();
}
// out = where(cond_mask, cond, y) from the workspace ODE state y. fault (or null): the engine's phase-chain give-up
// word; when a bounded wait of this call's chain launches expired, the results are wrong and out is NaN instead
__global__ void final_where_out_kernel(const float* cond, const uint8_t* m, const float* y, float* out,
                                       int64_t total, int mel, const unsigned* fault) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const bool bad = fault && __builtin_nontemporal_load(fault) != 0u;
  out[i] = bad ? __builtin_nanf("") : (m[i / mel] ? cond[i] : y[i]);
}
hipError_t final_where_out(const float* cond, const uint8_t* cond_mask, const float* y, float* out, int B, int N,
                           int mel, const unsigned* fault, hipStream_t st) {
  const int64_t total = (int64_t)B * N * mel;
  hipLaunchKernelGGL(final_where_out_kernel, dim3(nblk(total, 256)), dim3(256), 0, st, cond, cond_mask, y, out,
                     total, mel, fault);
  return hipGetLastError();
}

// ---------------------------------------------------------------- masks
__global__ void rowkeep_kernel(const int32_t* dur, int B, int S, int L, int off, uint8_t* keep) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * L) return;
  int s = (int)(i / L), pos = (int)(i - (int64_t)s * L);
  keep[i] = (pos < off || pos - off < dur[s % B]) ? 1 : 0;
}
hipError_t build_rowkeep(const int32_t* dur, int B, int S, int L, int off, uint8_t* keep, hipStream_t st) {
  hipLaunchKernelGGL(rowkeep_kernel, dim3(nblk((int64_t)S * L, 256)), dim3(256), 0, st, dur, B, S, L, off, keep);
  return hipGetLastError();
}
__global__ void kvlen_kernel(const int32_t* dur, int B, int S, int off, int32_t* kv) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < S) kv[s] = dur[s % B] + off;
}
hipError_t build_kvlen(const int32_t* dur, int B, int S, int off, int32_t* kv, hipStream_t st) {
  hipLaunchKernelGGL(kvlen_kernel, dim3(nblk(S, 64)), dim3(64), 0, st, dur, B, S, off, kv);
  return hipGetLastError();
}

template <typename TH>
__global__ void time_token_kernel(const float* temb, int S, int L, int d, TH* h) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * d) return;
  int s = (int)(i / d), c = (int)(i % d);
  h[(int64_t)s * L * d + c] = from_f32<TH>(temb[c]);
}
hipError_t write_time_token(int compute, int h16, const float* temb, int S, int L, int d, void* h, hipStream_t st) {
  const dim3 g(nblk((int64_t)S * d, 256)), b(256);
  if (!h16)
    hipLaunchKernelGGL(time_token_kernel<float>, g, b, 0, st, temb, S, L, d, (float*)h);
  else if (compute == F5H_C_BF16)
    hipLaunchKernelGGL(time_token_kernel<bf16>, g, b, 0, st, temb, S, L, d, (bf16*)h);
  else if (compute == F5H_C_FP16)
    hipLaunchKernelGGL(time_token_kernel<f16>, g, b, 0, st, temb, S, L, d, (f16*)h);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

__global__ void copy_pred_kernel(const float* p, int S, int L, int off, int mel, int64_t ld, float* dst,
                                 const unsigned* fault) {
  const int Lo = L - off;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * Lo * mel) return;
  int c = (int)(i % mel);
  int64_t r = i / mel;
  int s = (int)(r / Lo), n = (int)(r - (int64_t)s * Lo);
  const bool bad = fault && __builtin_nontemporal_load(fault) != 0u;  // as final_where_out
  dst[i] = bad ? __builtin_nanf("") : p[((int64_t)s * L + off + n) * ld + c];
}
hipError_t copy_pred(const float* p, int S, int L, int row_off, int mel, int64_t p_ld, float* dst,
                     const unsigned* fault, hipStream_t st) {
  const int64_t total = (int64_t)S * (L - row_off) * mel;
  hipLaunchKernelGGL(copy_pred_kernel, dim3(nblk(total, 256)), dim3(256), 0, st, p, S, L, row_off, mel, p_ld, dst,
                     fault);
  return hipGetLastError();
}

template <typename TO>
__global__ void cvt_kernel(const float* x, int64_t n, TO* y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = from_f32<TO>(x[i]);
}
template <typename TI>
__global__ void cvt_back_kernel(const TI* x, int64_t n, float* y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = to_f32(x[i]);
}
hipError_t f32_to_op(int compute, const float* x, int64_t n, void* out, hipStream_t st) {
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(cvt_kernel<T>, dim3(nblk(n, 256)), dim3(256), 0, st, x, n, (T*)out););
  return hipGetLastError();
}
hipError_t op_to_f32(int compute, const void* x, int64_t n, float* out, hipStream_t st) {
  F5H_OP_DISPATCH(compute, T, hipLaunchKernelGGL(cvt_back_kernel<T>, dim3(nblk(n, 256)), dim3(256), 0, st, (const T*)x, n, out););
  return hipGetLastError();
}

// ---------------------------------------------------------------- weight packing
template <typename T> F5H_DEV float ld_elem(const void* p, int64_t i) { return to_f32(reinterpret_cast<const T*>(p)[i]); }
__global__ __launch_bounds__(256) void pack_strided_kernel(PackArgs a, int64_t total) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    int64_t r = t;
    const int i3 = (int)(r % a.n[3]);
    r /= a.n[3];
    const int i2 = (int)(r % a.n[2]);
    r /= a.n[2];
    const int i1 = (int)(r % a.n[1]);
    const int i0 = (int)(r / a.n[1]);
    const int64_t si = i0 * a.src_st[0] + i1 * a.src_st[1] + i2 * a.src_st[2] + i3 * a.src_st[3];
    const int64_t di = i0 * a.dst_st[0] + i1 * a.dst_st[1] + i2 * a.dst_st[2] + i3;
    if (a.src_dt == 1 && a.dst_dt == 1) {  // same 16-bit type: bit copy
      reinterpret_cast<uint16_t*>(a.dst)[di] = reinterpret_cast<const uint16_t*>(a.src)[si];
      continue;
    }
    if (a.src_dt == 2 && a.dst_dt == 2) {
      reinterpret_cast<uint16_t*>(a.dst)[di] = reinterpret_cast<const uint16_t*>(a.src)[si];
      continue;
    }
    const float v = a.src_dt == 0 ? ld_elem<float>(a.src, si) : (a.src_dt == 1 ? ld_elem<bf16>(a.src, si)
                                                                                 : ld_elem<f16>(a.src, si));
    if (a.dst_dt == 0)
      reinterpret_cast<float*>(a.dst)[di] = v;
    else if (a.dst_dt == 1)
      reinterpret_cast<bf16*>(a.dst)[di] = f2bf(v);
    else
      reinterpret_cast<f16*>(a.dst)[di] = (f16)v;
  }
}
hipError_t pack_strided(const PackArgs& a, hipStream_t st) {
  const int64_t total = (int64_t)a.n[0] * a.n[1] * a.n[2] * a.n[3];
  if (total <= 0) return hipSuccess;
  if (a.src_dt < 0 || a.src_dt > 2 || a.dst_dt < 0 || a.dst_dt > 2) return hipErrorInvalidValue;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(pack_strided_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, total);
  return hipGetLastError();
}

}  // namespace f5h
