// Shared device helpers for the gfx950 CFM engine (wave64, MFMA, LDS swizzles).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kernels.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define F5H_DEV __device__ __forceinline__
#define LDS_PTR(T) __attribute__((address_space(3))) T*

// ---------------------------------------------------------------- conversions
F5H_DEV bf16 f2bf(float x) { return (bf16)x; }  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
F5H_DEV float bf2f(bf16 x) { return (float)x; }

template <typename T> F5H_DEV T from_f32(float x);
template <> F5H_DEV float from_f32<float>(float x) { return x; }
template <> F5H_DEV bf16 from_f32<bf16>(float x) { return f2bf(x); }
template <> F5H_DEV f16 from_f32<f16>(float x) { return (f16)x; }  // RNE (v_cvt_f16_f32)
F5H_DEV float to_f32(float x) { return x; }
F5H_DEV float to_f32(bf16 x) { return bf2f(x); }
F5H_DEV float to_f32(f16 x) { return (float)x; }

// 16-bit operand types (bf16 perf mode, fp16 mode = the reference's default GPU dtype,
// utils_infer.py:190-199): vector types and the two MFMA shapes (same cycles for both dtypes,
// MI355X_MICROARCH.md "Matrix cores").
template <typename T> struct Op16;
template <> struct Op16<bf16> {
  typedef bf16x8 v8;
  typedef bf16x4 v4;
  static F5H_DEV f32x4 mma16(const v8& a, const v8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static F5H_DEV f32x16 mma32(const v8& a, const v8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Op16<f16> {
  typedef f16x8 v8;
  typedef f16x4 v4;
  static F5H_DEV f32x4 mma16(const v8& a, const v8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static F5H_DEV f32x16 mma32(const v8& a, const v8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <typename T> __host__ __device__ constexpr bool is16() { return sizeof(T) == 2; }

// ---------------------------------------------------------------- activations
F5H_DEV float gelu_tanh(float x) {  // nn.GELU(approximate="tanh"), modules.py:358
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}
// Uncontracted fp32 ops (the build uses -ffp-contract=fast-honor-pragmas): epilogue arithmetic
// that must round identically in every kernel that inlines it (bitwise-identical tile configs).
F5H_DEV float mul_nc(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
F5H_DEV float add_nc(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
F5H_DEV float sub_nc(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}

// x as the fp32 op that produced it rounded it: an opaque move, so hipcc cannot fold that op (a multiply)
// into a later 16-bit conversion (v_fma_mix rounds the product once, straight to fp16, where the fast
// epilogues' packed forms round it to fp32 first; tile configs must agree bit for bit)
F5H_DEV float rounded(float x) {
  asm volatile("" : "+v"(x));
  return x;
}

// bf16-mode form: 0.5x(1+tanh(u)) == x * sigmoid(2u) = x / (1 + 2^(-2u*log2 e)); v_exp_f32 + v_rcp_f32
// (rel. error ~1e-6, far below the bf16 rounding of the result; the fp32 parity mode keeps tanhf)
F5H_DEV float gelu_tanh_fast(float x) {  // explicit rounding: identical in every kernel that inlines it
  const float k0 = 0.7978845608028654f * 2.f * 1.4426950408889634f, k1 = 0.044715f;
  const float x3 = mul_nc(mul_nc(x, x), x);
  const float u = mul_nc(k0, add_nc(x, mul_nc(k1, x3)));
  return rounded(mul_nc(x, __builtin_amdgcn_rcpf(add_nc(1.f, __builtin_amdgcn_exp2f(-u)))));
}
// The same on a pair of values with packed fp32 VALU (v_pk_mul_f32 / v_pk_add_f32: two elements per
// instruction, each rounded exactly like the scalar form, so the result is bit for bit gelu_tanh_fast's);
// the two transcendentals per element stay scalar. Epilogues are VALU-bound on this (FFN1: one exp + one rcp
// and six arithmetic ops per element with the matrix pipes idle).
typedef float f32x2 __attribute__((ext_vector_type(2)));
F5H_DEV f32x2 gelu_tanh_fast2(f32x2 x) {
#pragma clang fp contract(off)
  const float k0 = 0.7978845608028654f * 2.f * 1.4426950408889634f, k1 = 0.044715f;
  const f32x2 x3 = (x * x) * x;
  const f32x2 u = (x + x3 * k1) * k0;
  const f32x2 e = {__builtin_amdgcn_exp2f(-u.x), __builtin_amdgcn_exp2f(-u.y)};
  const f32x2 d = e + 1.f;
  const f32x2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return x * r;
}
// ---------------------------------------------------------------- in-kernel launch probe
// Kernel-side timing of probed launches (f5h_probe_*): the first thread of every workgroup
// atomicMin's the device wall clock (s_memrealtime, 100 MHz) into start[tick] at entry and
// every wave's lane 0 atomicMax's it into end[tick] at exit, so a launch's span is
// max(end) - min(start) without extra launches or events in the stream (graph-replay safe).
// slots = start row of this launch site; the end row is kProbeEnd entries further on.
// (DevProbe, kProbeTicks/kProbeSites/kProbeEnd: kernels.h)
F5H_DEV int64_t probe_slot(int k) {
  return ((int64_t)k * f5h::kProbeLanes + (blockIdx.x & (f5h::kProbeLanes - 1))) * f5h::kProbeStride;
}
// Entry: wave 0 reads the clock into registers (wait retired at once, so no SMEM op stays in
// flight under the kernels' hand-counted lgkmcnt waits) and loads the tick, consumed at exit.
struct ProbeT {
  unsigned long long t0;
  int k;
};
F5H_DEV ProbeT probe_enter(const f5h::DevProbe& p) {
  ProbeT r{0ull, -1};
  if (p.slots) {
    r.k = *p.tick;
    r.t0 = wall_clock64();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  return r;
}
// timeline stamp `idx` of this workgroup (wave 0's view; only in the timeline launch)
F5H_DEV void probe_mark(const f5h::DevProbe& p, const ProbeT& r, int idx) {
  if (p.tl && r.k == 0 && threadIdx.x == 0) {
    const int wg = blockIdx.x + gridDim.x * blockIdx.y;
    if (wg < f5h::kTimelineWG) p.tl[wg * 4 + idx] = idx == 0 ? r.t0 : (unsigned long long)wall_clock64();
  }
}
F5H_DEV void probe_exit(const f5h::DevProbe& p, const ProbeT& r) {
  if (p.slots && (threadIdx.x & 63) == 0 && r.k >= 0 && r.k < f5h::kProbeTicks && r.k % f5h::kProbeEvery == 0) {
    const int64_t i = probe_slot(r.k);
    atomicMax(p.slots + f5h::kProbeEnd + i, (unsigned long long)wall_clock64());
    if (threadIdx.x == 0) atomicMin(p.slots + i, r.t0);
  }
  probe_mark(p, r, 0);
  probe_mark(p, r, 3);
}

F5H_DEV float gelu_erf(float x) {  // nn.GELU(), modules.py:266 (explicit rounding, see gelu_tanh_fast)
  return rounded(mul_nc(mul_nc(0.5f, x), add_nc(1.f, erff(mul_nc(x, 0.7071067811865476f)))));
}
F5H_DEV float softplus(float x) {  // torch softplus (threshold 20)
  return x > 20.f ? x : log1pf(expf(x));
}
F5H_DEV float mish(float x) { return x * tanhf(softplus(x)); }  // nn.Mish, modules.py:181
// bf16-mode Mish: tanh(log1p(e^x)) = u(u+2) / (u(u+2) + 2), u = e^x (one v_exp + one v_rcp; the
// x > 20 branch is torch's softplus threshold, where tanh(softplus) == 1 in fp32)
F5H_DEV float mish_fast(float x) {
  const float u = __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
  const float n = u * (u + 2.f);
  return x > 20.f ? x : x * n * __builtin_amdgcn_rcpf(n + 2.f);
}
F5H_DEV float silu(float x) { return x / (1.f + expf(-x)); }

// ---------------------------------------------------------------- wave reductions (64 lanes)
F5H_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
F5H_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- LDS swizzle
// Tiles are stored as rows of 128 bytes = 8 chunks of 16 B. Chunk c of row r lives at
// c ^ g(r), g(r) = ((r>>1)&1)<<2 | ((r>>2)&3): conflict-free for ds_read_b128 where the
// 16 lanes of a group read 16 distinct rows at one chunk (GEMM / QK^T operands), and for
// ds_read_b64_tr_b16 reading 4 consecutive rows x 64 B (the PV operand).
F5H_DEV int swz128(int row, int chunk) {
  return chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}
// 256-byte rows (fp32 conv windows): chunk c (0..15) of row r at c ^ (r & 15).
F5H_DEV int swz256(int row, int chunk) { return chunk ^ (row & 15); }

// ---------------------------------------------------------------- MFMA per 64-byte k-slab
// One "k-slab" is 64 bytes of K per row: 32 bf16 or 16 fp32. Each lane holds 16 bytes
// of A (row lane&15, chunk lane>>4) and of B (col lane&15, chunk lane>>4).
// bf16: one v_mfma_f32_16x16x32_bf16 (lane group g supplies k = 8g..8g+7).
// fp32: four v_mfma_f32_16x16x4_f32, the j-th taking element j, so lane group g supplies
//       k = 4g + j: every k in 0..15 is summed exactly once (permuted order).
template <typename T> struct Slab;
template <> struct Slab<bf16> {
  typedef bf16x8 frag;
  static F5H_DEV f32x4 mma(const frag& a, const frag& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Slab<f16> {
  typedef f16x8 frag;
  static F5H_DEV f32x4 mma(const frag& a, const frag& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct Slab<float> {
  typedef f32x4 frag;
  static F5H_DEV f32x4 mma(const frag& a, const frag& b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
    return c;
  }
};

// 16-byte global load of 16/sizeof(T) elements of type T starting at p, converting
// from source type S (float or bf16) into compute type T; `ok` false -> zeros.
template <typename T, typename S> struct Load16;
template <> struct Load16<bf16, bf16> {
  static F5H_DEV uint4 ld(const bf16* p, bool ok) {
    return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  }
};
template <> struct Load16<float, float> {
  static F5H_DEV uint4 ld(const float* p, bool ok) {
    return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  }
};
template <> struct Load16<f16, f16> {
  static F5H_DEV uint4 ld(const f16* p, bool ok) {
    return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  }
};
template <> struct Load16<f16, float> {
  static F5H_DEV uint4 ld(const float* p, bool ok) {
    if (!ok) return make_uint4(0, 0, 0, 0);
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    f16x8 v = {(f16)a.x, (f16)a.y, (f16)a.z, (f16)a.w, (f16)b.x, (f16)b.y, (f16)b.z, (f16)b.w};
    return __builtin_bit_cast(uint4, v);
  }
};
template <> struct Load16<bf16, float> {
  static F5H_DEV uint4 ld(const float* p, bool ok) {
    if (!ok) return make_uint4(0, 0, 0, 0);
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    bf16x8 v = {f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
    return __builtin_bit_cast(uint4, v);
  }
};

template <typename T> F5H_DEV constexpr int elems16() { return 16 / (int)sizeof(T); }

// Compile-time loop: f(integral_constant<int, I>) for I in [B, E). Register arrays indexed
// through it are split into scalars by SROA (a runtime-indexed or loop-indexed array can
// be lowered to scratch before the unroller runs).
// raw buffer descriptor over [p, p + bytes): loads past the extent read 0, stores past it are dropped
// (the hardware range check), so out-of-range lanes need no branch; bytes < 2^32
// Bijection on [0, n) that deals the 8 near-equal contiguous chunks of [0, n) (the ranges the XCD-aware
// block maps give the 8 XCDs) out round-robin: element i of chunk c goes to 8 i + c. Used where the work of
// an index varies along it (the batch path's pad skip: sequences of different lengths), so that every XCD
// gets a share of every part instead of one contiguous part.
F5H_DEV int spread8(int r, int n) {
  const int q = n >> 3, rem = n & 7;
  if (q == 0) return r;
  const int big = rem * (q + 1);
  const int c = r < big ? r / (q + 1) : rem + (r - big) / q;
  const int i = r < big ? r - c * (q + 1) : (r - big) - (c - rem) * q;
  return i * 8 + c;
}

F5H_DEV __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(uint32_t)bytes, 0x00020000);
}
// one 16-byte-per-lane LDS-DMA piece (buffer_load_dwordx4 ... lds): voffset per lane, soffset scalar, the
// LDS destination wave-uniform (M0). A device-only wrapper: the builtin in a kernel body would keep hipcc's
// host pass from emitting the kernel's launch stub.
F5H_DEV void dma16(__amdgpu_buffer_rsrc_t r, LDS_PTR(void) dst, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
}

template <int B, int E, typename F>
F5H_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Launch a templated kernel body for the compute mode's operand type: T = float (F5H_C_FP32),
// bf16 (F5H_C_BF16) or f16 (F5H_C_FP16). Usage: F5H_OP_DISPATCH(compute, T, { launch<T>(...); });
#define F5H_OP_DISPATCH(compute, T, ...)  \
  do {                                     \
    switch (compute) {                     \
      case f5h::F5H_C_BF16: {              \
        typedef bf16 T;                    \
        __VA_ARGS__;                       \
      } break;                             \
      case f5h::F5H_C_FP16: {              \
        typedef f16 T;                     \
        __VA_ARGS__;                       \
      } break;                             \
      default: {                           \
        typedef float T;                   \
        __VA_ARGS__;                       \
      }                                    \
    }                                      \
  } while (0)
