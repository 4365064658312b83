// Device side of the in-launch phase chain (chain.hip): row-group hand-offs between the phases of one launch.
//
// Protocol (cdna_hip_programming.md §6 Guideline 16, R1; MI355X_MICROARCH.md 'Valid forms'):
//   producer workgroup: its payload stores are write-through (buffer stores with kAuxWT) -> every wave
//     s_waitcnt vmcnt(0) -> __syncthreads() -> ONE lane adds 1 (relaxed, agent scope) to the counter of every
//     row group its tile covers;
//   consumer workgroup: ONE wave polls each needed counter (relaxed agent loads + s_sleep, bounded) -> ONE
//     agent-scope acquire (drops this CU's L1) -> s_waitcnt vmcnt(0) -> __syncthreads() -> plain loads.
// Counters are zeroed by a kernel (zero_words) at the start of every backbone pass (Guideline 16, 'Re-initialise
// every call'; a captured memset node was not re-applied on later replays of the step graph, round 6): each layer's
// launch has its own [5][groups] block of them.
// Progress: a phase's workgroups have higher ids than every producer they wait for, and the dispatcher hands
// out ids in order on each XCD, so every producer is resident or finished before any consumer can wait on it
// (a waiting block never keeps a producer from being dispatched). The bounded spin only guards against a bug:
// it gives up after ~0.3 s, sets the ENGINE's fault word (ChainDep::err, engine-owned device memory) and lets the
// launch drain; the call's final kernel then writes NaN results, and the engine's next call fails (engine.cpp).
#pragma once
#include "common.h"
#include "kernels.h"

namespace f5h {

constexpr int kAuxWT = 16;                 // buffer-store cache policy: sc1 (write-through)
constexpr unsigned kChainSpinLimit = 1u << 18;
// between polls: 2 x 64 clocks (16 x 64, to take the pollers' loads out of the computing CUs' memory queues,
// MI355X_MICROARCH.md 'polling-cost', left the computing tiles as slow and added latency to every hand-off:
// profiles/r05_ab_c2_chain_tuning.txt)
constexpr int kChainSleep = 2;

F5H_DEV void chain_wait(const ChainDep& d, int M, int r0, int nrows) {
  if (!d.wait) return;
  // wave 0 polls with a wave-uniform loop (the polled value through readfirstlane): a loop whose exit is
  // per-lane makes everything after it divergent to the compiler (the LDS-DMA descriptors then go through
  // waterfall loops, cdna_hip_programming.md T20)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
    const int g0 = r0 / kChainRows, g1 = (min(r0 + nrows, M) - 1) / kChainRows;
    for (int gi = g0; gi <= g1; ++gi) {
      const int rows = min(kChainRows, M - gi * kChainRows);
      const unsigned need = (unsigned)(d.wait_mult * ((rows + d.wait_unit - 1) / d.wait_unit));
      for (unsigned spins = 0;; ++spins) {
        const unsigned v =
            __builtin_amdgcn_readfirstlane(__hip_atomic_load(d.wait + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (v >= need) break;
        if (spins >= d.spin_limit) {
          __hip_atomic_store(d.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(kChainSleep);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (d.tl && threadIdx.x == 0) d.tl[1] = wall_clock64();
  }
  __syncthreads();
}

// after the workgroup's write-through stores of rows [r0, r0 + nrows)
F5H_DEV void chain_publish(const ChainDep& d, int M, int r0, int nrows) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its stores have left
  __syncthreads();
  if (d.tl && threadIdx.x == 0) d.tl[2] = wall_clock64();
  if (threadIdx.x == 0) {
    const int g0 = r0 / kChainRows, g1 = (min(r0 + nrows, M) - 1) / kChainRows;
    for (int gi = g0; gi <= g1; ++gi) __hip_atomic_fetch_add(d.pub + gi, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace f5h
