// Probe: semantics of __builtin_amdgcn_permlane32_swap on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned l = threadIdx.x;
  unsigned a = 100 + l, b = 200 + l;
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane32_swap(a, a, false, false);
  out[128 + l] = s[0];
  out[192 + l] = s[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  unsigned h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int i : {0, 1, 31, 32, 33, 63}) printf("lane %2d: swap(a,b) r0=%u r1=%u | swap(a,a) r0=%u r1=%u\n", i, h[i], h[64+i], h[128+i], h[192+i]);
  return 0;
}
