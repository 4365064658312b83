// One row of the AdaLN LayerNorm + modulate (AdaLayerNorm modules.py:325, ff_norm :753,
// AdaLayerNorm_Final :346): LN(x) (no affine, eps 1e-6) * (1 + scale) + shift, a wave per row, lane
// l holding elements 4(l + 64k) .. +3, used by ln_mod_kernel (elementwise.hip). (Round 3 also ran it as
// a fused tail of the residual GEMMs, which needed the same bits; measured slower and removed)
#pragma once
#include "common.h"

namespace f5h {

template <typename T> F5H_DEV void store4(T* p, float a, float b, float c, float d);
template <> F5H_DEV void store4<float>(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
template <> F5H_DEV void store4<bf16>(bf16* p, float a, float b, float c, float d) {
  bf16x4 v = {f2bf(a), f2bf(b), f2bf(c), f2bf(d)};
  *reinterpret_cast<bf16x4*>(p) = v;
}
template <> F5H_DEV void store4<f16>(f16* p, float a, float b, float c, float d) {
  f16x4 v = {(f16)a, (f16)b, (f16)c, (f16)d};
  *reinterpret_cast<f16x4*>(p) = v;
}

template <typename TI> F5H_DEV float4 load4f(const TI* p);
template <> F5H_DEV float4 load4f<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <> F5H_DEV float4 load4f<bf16>(const bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
template <> F5H_DEV float4 load4f<f16>(const f16* p) {
  const f16x4 v = *reinterpret_cast<const f16x4*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}

// Row sum over the wave, the same value in every lane: DPP butterflies inside each 16-lane row
// (xor 1, xor 2, half-mirror, mirror: VALU, no LDS round trip), then the four row sums by readlane.
F5H_DEV float wave_sum_dpp(float v) {
  auto dpp = [](float x, int ctrl) -> float {
    switch (ctrl) {  // the control word must be an immediate
      case 0xB1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
      case 0x4E: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
      case 0x141: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
      default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));
    }
  };
  v += dpp(v, 0xB1);   // quad_perm [1,0,3,2]
  v += dpp(v, 0x4E);   // quad_perm [2,3,0,1]
  v += dpp(v, 0x141);  // row_half_mirror
  v += dpp(v, 0x140);  // row_mirror: every lane of a row holds the row sum
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// Normalise + modulate one row held in v (V float4 per lane; FIXED: all 64*V float4 are the row,
// else only i = lane + 64k < n4) and store it to orow.
template <typename TO, int V, bool FIXED>
F5H_DEV void ln_mod_row(const float4 (&v)[V], const float4 (&a)[V], const float4 (&b)[V], int lane, int n4, int d,
                        TO* orow) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) s += v[k].x + v[k].y + v[k].z + v[k].w;
  const float mean = wave_sum_dpp(s) / d;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = lane + 64 * k;
    if (FIXED || i < n4) {
      float p0 = v[k].x - mean, p1 = v[k].y - mean, p2 = v[k].z - mean, p3 = v[k].w - mean;
      q += p0 * p0 + p1 * p1 + p2 * p2 + p3 * p3;
    }
  }
  const float rstd = rsqrtf(wave_sum_dpp(q) / d + 1e-6f);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int i = lane + 64 * k;
    if (FIXED || i < n4)
      store4<TO>(orow + 4 * i, (v[k].x - mean) * rstd * (1.f + a[k].x) + b[k].x,
                 (v[k].y - mean) * rstd * (1.f + a[k].y) + b[k].y, (v[k].z - mean) * rstd * (1.f + a[k].z) + b[k].z,
                 (v[k].w - mean) * rstd * (1.f + a[k].w) + b[k].w);
  }
}

// The 16-bit residual stream at d = 1024 (ln_mod16_kernel, and the chain's LayerNorm phase, chain.hip): lane l
// holds elements 8(l + 64k) .. +7 (k < 2) of the row in x[k] (raw 16-byte chunks), a/b the scale/shift of
// those elements; o[k] the normalised, modulated chunks. One function, so both launches give the same bits.
template <typename T>
F5H_DEV void ln16_row(const uint4 (&x)[2], const float4 (&a)[2][2], const float4 (&b)[2][2], uint4 (&o)[2]) {
  typedef typename Op16<T>::v8 v8;
  constexpr int d = 1024;
  float v[2][8];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const v8 w = __builtin_bit_cast(v8, x[k]);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[k][e] = to_f32(w[e]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[k][e];
  const float mean = wave_sum_dpp(s) / d;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float p = v[k][e] - mean;
      q += p * p;
    }
  const float rstd = rsqrtf(wave_sum_dpp(q) / d + 1e-6f);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float av[8] = {a[k][0].x, a[k][0].y, a[k][0].z, a[k][0].w, a[k][1].x, a[k][1].y, a[k][1].z, a[k][1].w};
    const float bv[8] = {b[k][0].x, b[k][0].y, b[k][0].z, b[k][0].w, b[k][1].x, b[k][1].y, b[k][1].z, b[k][1].w};
    v8 w;
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = from_f32<T>((v[k][e] - mean) * rstd * (1.f + av[e]) + bv[e]);
    o[k] = __builtin_bit_cast(uint4, w);
  }
}

}  // namespace f5h
