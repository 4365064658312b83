// Probe: does global_load_lds_dwordx4 + source-side swizzle give the swz128 LDS image the
// attention kernel assumes? Fills a 64x64 bf16-sized (as u16 indices) tile and reads it back.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../f5-tts_amd/csrc/common.h"
__global__ void k(const unsigned short* K, unsigned short* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint4 lds[1024];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int r = 0; r < 2; ++r) {
    const int p = (r * 4 + wid) * 64 + lane, row = p >> 3, slot = p & 7;
    const int off = row * 64 + swz128(row, slot) * 8;
    if (mode == 0)
      __builtin_amdgcn_global_load_lds((const void*)(K + off), (LDS_PTR(void))(lds + (r * 4 + wid) * 64), 16, 0, 0);
    else
      lds[row * 8 + swz128(row, swz128(row, slot))] = *(const uint4*)(K + off);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // read back logical (row, chunk) through the swizzle: out[row][chunk*8..] should equal K[row][chunk*8..]
  for (int i = tid; i < 512; i += 256) {
    int row = i >> 3, ch = i & 7;
    uint4 v = lds[row * 8 + swz128(row, ch)];
    *(uint4*)(out + row * 64 + ch * 8) = v;
  }
}
int main() {
  unsigned short h[4096], o[4096];
  for (int i = 0; i < 4096; ++i) h[i] = i;
  unsigned short *dk, *dout;
  (void)hipMalloc(&dk, 8192); (void)hipMalloc(&dout, 8192);
  (void)hipMemcpy(dk, h, 8192, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    (void)hipMemset(dout, 0, 8192);
    hipLaunchKernelGGL(k, 1, 256, 0, 0, dk, dout, mode);
    (void)hipMemcpy(o, dout, 8192, hipMemcpyDeviceToHost);
    int bad = 0, first = -1;
    for (int i = 0; i < 4096; ++i) if (o[i] != h[i]) { if (first < 0) first = i; ++bad; }
    printf("mode %d (%s): mismatches %d", mode, mode ? "register store" : "LDS-DMA", bad);
    if (first >= 0) printf("  first at %d: got %d", first, o[first]);
    printf("\n");
    if (mode == 0) { printf("row0: "); for (int c = 0; c < 64; c += 8) printf("%d ", o[c]); printf("\nrow1: "); for (int c = 0; c < 64; c += 8) printf("%d ", o[64 + c]); printf("\n"); }
  }
  return 0;
}
