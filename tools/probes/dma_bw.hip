// Probe: LDS-DMA (global_load_lds_dwordx4) intake per CU from an L2/MALL-resident buffer.
// One workgroup per CU streams `iters` slabs of `slab` KB into an LDS ring with `depth` slabs
// in flight (counted vmcnt), no compute. Prints GB/s per CU and bytes/cycle at 2.1 GHz.
// Usage: dma_bw <waves> <depth> <slab_kb> <footprint_mb>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int WAVES, int DEPTH, int SLABKB>
__global__ __launch_bounds__(64 * WAVES, 1) void k(const uint4* src, size_t nvec, int iters, int* sink) {
  constexpr int PER = SLABKB * 1024 / 16 / (64 * WAVES);  // glds per wave per slab
  __shared__ __attribute__((aligned(16))) uint4 lds[DEPTH * SLABKB * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  size_t base = ((size_t)blockIdx.x * 977 * SLABKB * 64) % nvec;
  for (int it = 0; it < iters; ++it) {
    const int slot = it % DEPTH;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const size_t e = (base + ((size_t)it * SLABKB * 64) + (size_t)(i * WAVES + wid) * 64 + lane) % nvec;
      __builtin_amdgcn_global_load_lds((const void*)(src + e),
                                       (__attribute__((address_space(3))) void*)(lds + slot * SLABKB * 64 + (i * WAVES + wid) * 64),
                                       16, 0, 0);
    }
    if (it >= DEPTH - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"((DEPTH - 1) * PER) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = ((int*)lds)[lane];
}

template <int W, int D, int S>
float run(const uint4* src, size_t nvec, int iters, int* sink, int cus) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k<W, D, S>), dim3(cus), dim3(64 * W), 0, 0, src, nvec, iters, sink);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<W, D, S>), dim3(cus), dim3(64 * W), 0, 0, src, nvec, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = 5.0 * cus * (double)iters * S * 1024;
  const double gbs_cu = bytes / (ms * 1e-3) / cus / 1e9;
  printf("waves %d depth %d slab %3d KB: %7.1f GB/s per CU  %5.1f B/clk@2.1GHz  chip %6.2f TB/s\n", W, D, S, gbs_cu,
         gbs_cu / 2.1, gbs_cu * cus / 1e3);
  return ms;
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? atoi(argv[1]) : 8;
  const size_t nvec = mb * 1024 * 1024 / 16;
  uint4* src;
  int* sink;
  hipMalloc(&src, nvec * 16);
  hipMemset(src, 1, nvec * 16);
  hipMalloc(&sink, 4096 * 4);
  const int cus = 256, iters = 2000;
  printf("footprint %zu MB\n", mb);
  run<4, 2, 16>(src, nvec, iters, sink, cus);
  run<4, 4, 16>(src, nvec, iters, sink, cus);
  run<8, 2, 16>(src, nvec, iters, sink, cus);
  run<8, 4, 16>(src, nvec, iters, sink, cus);
  run<8, 8, 16>(src, nvec, iters, sink, cus);
  run<8, 2, 32>(src, nvec, iters / 2, sink, cus);
  run<8, 4, 32>(src, nvec, iters / 2, sink, cus);
  run<16, 4, 16>(src, nvec, iters, sink, cus);
  run<16, 8, 16>(src, nvec, iters, sink, cus);
  run<4, 8, 16>(src, nvec, iters, sink, cus);
  return 0;
}
