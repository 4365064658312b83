// Probe: per-CU operand intake by staging method, no compute (what bounds the C2 GEMMs).
//   mode 0: LDS-DMA (global_load_lds 16 B/lane) into an LDS ring, counted vmcnt (the GEMM's form)
//   mode 1: global_load_dwordx4 to registers, D batches in flight, then ds_write_b128 (register staging)
//   mode 2: global_load_dwordx4 to registers only (the vector-memory path's own ceiling)
// Each wave moves P x 1 KB per batch; grid = cus x blocks-per-CU workgroups of W waves; footprint MB
// (8 MB ~ a C2 weight panel: L2/MALL-resident; a power of two). Prints GB/s per CU.
//   intake [footprint_mb]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int N>
struct IC {
  static constexpr int value = N;
};
template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    sfor<B + 1, E>(f);
  }
}

template <int MODE, int W, int D, int P>
__global__ __launch_bounds__(64 * W) void k(const uint4* src, size_t nvec, int iters, int* sink) {
  __shared__ __attribute__((aligned(16))) uint4 lds[D * W * P * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t base = ((size_t)blockIdx.x * 977 * W * P * 64) & (nvec - 1);
  auto addr = [&](int it, int i) -> const uint4* {
    return src + ((base + (size_t)it * W * P * 64 + (size_t)(i * W + wid) * 64 + lane) & (nvec - 1));
  };
  uint4 acc = make_uint4(0, 0, 0, 0);
  if constexpr (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
      const int slot = it % D;
#pragma unroll
      for (int i = 0; i < P; ++i)
        __builtin_amdgcn_global_load_lds((const void*)addr(it, i),
                                         (__attribute__((address_space(3))) void*)(lds + (slot * W * P + i * W + wid) * 64),
                                         16, 0, 0);
      if (it >= D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"((D - 1) * P) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    uint4 r[D][P];
    sfor<0, D - 1>([&](auto DD) {
#pragma unroll
      for (int i = 0; i < P; ++i) r[DD.value][i] = *addr(DD.value, i);
    });
    for (int it0 = 0; it0 < iters; it0 += D) {
      sfor<0, D>([&](auto DD) {
        constexpr int d = DD.value, dn = (d + D - 1) % D;
        const int it = it0 + d;
#pragma unroll
        for (int i = 0; i < P; ++i) r[dn][i] = *addr(it + D - 1, i);
#pragma unroll
        for (int i = 0; i < P; ++i) {
          if constexpr (MODE == 1) {
            lds[(d * W * P + i * W + wid) * 64 + lane] = r[d][i];
          } else {
            acc.x ^= r[d][i].x;
            acc.y += r[d][i].y;
          }
        }
      });
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = ((int*)lds)[lane] + acc.x + acc.y;
}

template <int MODE, int W, int D, int P>
void run(const uint4* src, size_t nvec, int iters, int* sink, int cus, int bpc) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = cus * bpc;
  hipLaunchKernelGGL((k<MODE, W, D, P>), dim3(grid), dim3(64 * W), 0, 0, src, nvec, iters, sink);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MODE, W, D, P>), dim3(grid), dim3(64 * W), 0, 0, src, nvec, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = 5.0 * grid * (double)iters * W * P * 1024;
  const double gbs_cu = bytes / (ms * 1e-3) / cus / 1e9;
  printf("mode %d (%s) waves %2d x %d blocks/CU, %d batches x %d KB/wave in flight: %7.1f GB/s per CU, chip %6.2f TB/s\n",
         MODE, MODE == 0 ? "lds-dma " : (MODE == 1 ? "reg->lds" : "reg only"), W, bpc, D, P, gbs_cu, gbs_cu * cus / 1e3);
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 8;
  const size_t nvec = mb * 1024 * 1024 / 16;
  uint4* src;
  int* sink;
  hipMalloc(&src, nvec * 16);
  hipMemset(src, 1, nvec * 16);
  hipMalloc(&sink, 8192 * 4);
  const int cus = 256, iters = 1200;
  printf("footprint %zu MB\n", mb);
  run<0, 4, 3, 2>(src, nvec, iters, sink, cus, 2);
  run<0, 4, 4, 4>(src, nvec, iters, sink, cus, 2);
  run<0, 8, 4, 2>(src, nvec, iters, sink, cus, 1);
  run<1, 4, 2, 2>(src, nvec, iters, sink, cus, 2);
  run<1, 4, 3, 2>(src, nvec, iters, sink, cus, 2);
  run<1, 4, 2, 4>(src, nvec, iters, sink, cus, 2);
  run<1, 8, 2, 2>(src, nvec, iters, sink, cus, 1);
  run<1, 8, 3, 2>(src, nvec, iters, sink, cus, 1);
  run<2, 4, 3, 2>(src, nvec, iters, sink, cus, 2);
  run<2, 4, 2, 4>(src, nvec, iters, sink, cus, 2);
  run<2, 8, 3, 2>(src, nvec, iters, sink, cus, 1);
  return 0;
}
