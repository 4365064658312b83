// Probe: do one wave's MFMAs and its SIMD partner's VALU work overlap?
// 512-thread workgroups (waves w and w+4 share a SIMD, tools/probes/simd_map.hip), one per CU.
// mode bit 0: waves 0-3 run ITER x 16 v_mfma_f32_32x32x16_bf16 (two accumulators);
// mode bit 1: waves 4-7 run ITER x (NEXP v_exp_f32 + NADD v_fma_f32) on 32 independent values.
// mode bit 2: waves 4-7 raise their priority (s_setprio 3) first.
// mode 8: waves 0-3 interleave both streams in ONE wave (MFMA, then its share of the VALU work);
// mode 9: all 8 waves do that (two interleaving waves per SIMD).
// Prints the kernel time per mode; overlap means time(3) ~ max(time(1), time(2)).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int NEXP, int NADD>
__global__ __launch_bounds__(512, 1) void k(float* out, int mode, int iter) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  float acc = 0.f;
  if (mode >= 8) {
    if (mode == 8 && wid >= 4) return;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = (__bf16)(0.001f * (lane + j));
      b[j] = (__bf16)(0.002f * (lane - j));
    }
    f32x16 c0 = {}, c1 = {};
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = -0.001f * (lane + j);
    for (int i = 0; i < iter; ++i) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
#pragma unroll
        for (int j = 2 * r * NEXP / 16; j < (2 * r + 1) * NEXP / 16; ++j) v[j & 31] = __builtin_amdgcn_exp2f(v[j & 31]) - 1.0f;
#pragma unroll
        for (int j = 2 * r * NADD / 16; j < (2 * r + 1) * NADD / 16; ++j) v[j & 31] = __builtin_fmaf(v[j & 31], 0.999f, -0.0001f);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
#pragma unroll
        for (int j = (2 * r + 1) * NEXP / 16; j < (2 * r + 2) * NEXP / 16; ++j) v[j & 31] = __builtin_amdgcn_exp2f(v[j & 31]) - 1.0f;
#pragma unroll
        for (int j = (2 * r + 1) * NADD / 16; j < (2 * r + 2) * NADD / 16; ++j) v[j & 31] = __builtin_fmaf(v[j & 31], 0.999f, -0.0001f);
      }
    }
    for (int r = 0; r < 16; ++r) acc += c0[r] + c1[r];
#pragma unroll
    for (int j = 0; j < 32; ++j) acc += v[j];
  } else if (wid < 4) {
    if (mode & 1) {
      bf16x8 a, b;
      for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (lane + j));
        b[j] = (__bf16)(0.002f * (lane - j));
      }
      f32x16 c0 = {}, c1 = {};
      for (int i = 0; i < iter; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        }
      }
      for (int r = 0; r < 16; ++r) acc += c0[r] + c1[r];
    }
  } else if (mode & 2) {
    if (mode & 4) __builtin_amdgcn_s_setprio(3);
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = -0.001f * (lane + j);
    for (int i = 0; i < iter; ++i) {
#pragma unroll
      for (int j = 0; j < NEXP; ++j) v[j & 31] = __builtin_amdgcn_exp2f(v[j & 31]) - 1.0f;
#pragma unroll
      for (int j = 0; j < NADD; ++j) v[j & 31] = __builtin_fmaf(v[j & 31], 0.999f, -0.0001f);
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) acc += v[j];
  }
  if (acc == 12345.f) out[threadIdx.x] = acc;
}

template <int NEXP, int NADD>
static void run(const char* name, float* d, int iter) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode : {1, 2, 3, 7, 8, 9}) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL((k<NEXP, NADD>), dim3(256), dim3(512), 0, 0, d, mode, iter);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-24s mode %d (%s): %8.1f us\n", name, mode, mode == 1 ? "mfma only" : mode == 2 ? "valu only" : mode == 3 ? "both" : mode == 7 ? "both, valu prio" : mode == 8 ? "in-wave, 4 waves" : "in-wave, 8 waves", best * 1e3);
  }
}

int main() {
  float* d;
  hipMalloc(&d, 4096);
  const int iter = 2000;
  run<16, 0>("16 exp / 16 mfma", d, iter);
  run<0, 64>("64 fma / 16 mfma", d, iter);
  run<8, 32>("8 exp+32 fma / 16 mfma", d, iter);
  run<32, 0>("32 exp / 16 mfma", d, iter);
  return 0;
}
