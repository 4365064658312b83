// In-launch phase chain: the row-local seams of a DiT block-step as ONE launch (DESIGN.md §3 'Phase chain').
//
// After attention, a DiT block-step (modules.py:743-757) is row-local until the next attention:
//   out-proj + gated residual (h += gate_msa * o.Wo^T)      phase 0, GEMM 64x128  (cfg 0)
//   LayerNorm + modulate (aop = LN(h) (1 + scale) + shift)   phase 1, 32-row units
//   FFN1 + GELU-tanh (f = gelu(aop.W1^T + b1))               phase 2, GEMM 128x128 (cfg 1)
//   FFN2 + gated residual (h += gate_mlp * f.W2^T)           phase 3, GEMM 64x128  (cfg 0)
//   LayerNorm + modulate of the next layer (or the final)    phase 4, 32-row units
//   QKV + RoPE of the next layer                             phase 5, GEMM 192x128 (cfg 5; absent after the last)
// Separate launches drain the whole grid at every seam and fill it again (MI355X_MICROARCH.md 'boundary':
// 1.1-1.9 us each, plus the tail of the slowest tile). Here each phase's workgroups follow the previous phase's in
// block-id order and wait only for the row groups (64 rows) they read, through arrival counters (chain.h), so a
// phase starts on the rows whose producers are done while the rest of the previous phase drains.
// Per element every phase computes exactly what its separate launch computes (same bodies: gemm_body,
// ln16_row); tile configurations do not change GEMM bits (tests/test_gpu_parity.py every-tile-config test), so
// the chain is bitwise equal to the separate launches (tests/test_gpu_contract.py chain test).
#include "chain.h"
#include "gemm_impl.h"
#include "lnrow.h"

#include <algorithm>
#include <atomic>

namespace f5h {

namespace {

// phase geometry: tile configs of the GEMM phases
constexpr int kOutBM = 64, kFf1BM = 128, kFf2BM = 64, kQkvBM = 192, kBN = 128, kLnRows = 32;
typedef GemmCfg<kOutBM, kBN, 2, 2, 3> CfgOut;
typedef GemmCfg<kFf1BM, kBN, 2, 2, 2> CfgFf1;
typedef GemmCfg<kQkvBM, kBN, 2, 2, 2> CfgQkv;
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int kLdsBytes = cmax(cmax(CfgOut::bytes, CfgFf1::bytes), CfgQkv::bytes);

std::atomic<long long> g_spin_limit{(long long)kChainSpinLimit};  // test hook: chain_set_spin_limit

struct Launch {
  ChainArgs a;
  ChainDep dep[6];
  int start[7];  // first block of each phase (multiples of 8: a phase's block b and b + 8 share an XCD)
};

// LayerNorm phase: 32 rows per workgroup, 8 per wave, all eight rows' loads in flight before the first reduction
// (16-row units: 3.0 instead of 3.6 us per unit, but the phases ended later and C2 took 50.9 instead of 49.9 ms,
// profiles/r05_ab_c2_chain_tuning.txt)
template <typename T>
F5H_DEV void ln_phase(const LnArgs& l, int M, int unit, const ChainDep& dep) {
  const int r0 = unit * kLnRows;
  if (r0 >= M) return;
  chain_wait(dep, M, r0, kLnRows);
  constexpr int d = 1024, RW = kLnRows / 4;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint4* x = reinterpret_cast<const uint4*>(l.h);
  const float4* sh = reinterpret_cast<const float4*>(l.shift);
  const float4* sc = reinterpret_cast<const float4*>(l.scale);
  float4 a[2][2], b[2][2];
  uint4 xv[RW][2];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int row = min(r0 + wid * RW + i, M - 1);
#pragma unroll
    for (int k = 0; k < 2; ++k) xv[i][k] = x[(int64_t)row * (d / 8) + lane + 64 * k];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = lane + 64 * k;
    a[k][0] = sc[2 * c];
    a[k][1] = sc[2 * c + 1];
    b[k][0] = sh[2 * c];
    b[k][1] = sh[2 * c + 1];
  }
  const __amdgpu_buffer_rsrc_t dst = rsrc_of(l.out, (uint64_t)M * d * sizeof(T));
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    uint4 o[2];
    ln16_row<T>(xv[i], a, b, o);
    const int row = r0 + wid * RW + i;  // rows >= M: past the descriptor's extent, dropped
#pragma unroll
    for (int k = 0; k < 2; ++k)
      store16_rs<kAuxWT>(dst, (uint32_t)(((int64_t)row * d + 8 * (lane + 64 * k)) * sizeof(T)),
                         __builtin_bit_cast(u32x4, o[k]));
  }
  chain_publish(dep, M, r0, kLnRows);
}

template <typename TC>
__global__ __launch_bounds__(256, 2) void chain_kernel(Launch L) {
  __shared__ __attribute__((aligned(16))) uint4 lds[kLdsBytes / 16];
  const ProbeT pt = probe_enter(L.a.probe);
  const int b = blockIdx.x;
  const int M = L.a.out.M;
  int p = 0;
  while (p < 5 && b >= L.start[p + 1]) ++p;
  ChainDep d = L.dep[p];
  d.tl = (L.a.probe.tl && pt.k == 0 && b < kTimelineWG) ? L.a.probe.tl + (size_t)b * 4 : nullptr;
  if (d.tl && threadIdx.x == 0) d.tl[1] = d.tl[2] = 0ull;
  if (p == 0) {
    gemm_body<TC, EPI_RESID16, kOutBM, kBN, 2, 2, 3, true, 128, true, true>(L.a.out, b, L.start[1], lds, d);
  } else if (p == 1) {
    ln_phase<TC>(L.a.ln1, M, b - L.start[1], d);
  } else if (p == 2) {
    gemm_body<TC, EPI_GELU_TANH, kFf1BM, kBN, 2, 2, 2, true, 128, true, true>(L.a.ff1, b - L.start[2],
                                                                               L.start[3] - L.start[2], lds, d);
  } else if (p == 3) {
    gemm_body<TC, EPI_RESID16, kFf2BM, kBN, 2, 2, 3, true, 128, true, true>(L.a.ff2, b - L.start[3],
                                                                             L.start[4] - L.start[3], lds, d);
  } else if (p == 4) {
    ln_phase<TC>(L.a.ln2, M, b - L.start[4], d);
  } else {
    gemm_body<TC, EPI_QKV, kQkvBM, kBN, 2, 2, 2, true, 128, false, true>(L.a.qkv, b - L.start[5],
                                                                          L.start[6] - L.start[5], lds, d);
  }
  probe_exit(L.a.probe, pt);
}

int round8(int n) { return (n + 7) / 8 * 8; }
int ceil_div(int a, int b) { return (a + b - 1) / b; }

// whole-column tiles, 16-B rows, K in whole stages, no pad-row skip, no second A panel
bool gemm_fits(const GemmArgs& g, int N) {
  return g.N == N && g.K % 64 == 0 && g.ldc % 8 == 0 && g.lda % 8 == 0 && g.ldw % 8 == 0 && !g.live_len && !g.A2 &&
         !g.probe.slots;  // (the chain launch is timed as one: ChainArgs::probe)
}

}  // namespace

hipError_t chain_launch(int compute, const ChainArgs& a, hipStream_t st) {
  const int M = a.out.M, d = 1024;
  const bool qkv = a.qkv.M > 0;
  const int ff = a.ff1.N;
  if ((compute != F5H_C_BF16 && compute != F5H_C_FP16) || M <= 0 || a.groups != ceil_div(M, kChainRows) ||
      !a.cnt || a.ff1.M != M || a.ff2.M != M || (qkv && a.qkv.M != M) || ff % kBN || a.ff2.K != ff ||
      a.out.K % 64 || !gemm_fits(a.out, d) || !gemm_fits(a.ff1, ff) || !gemm_fits(a.ff2, d) ||
      (qkv && (!gemm_fits(a.qkv, a.qkv.N) || a.qkv.N % kBN || a.qkv.N != 3 * a.qkv.heads * 64)) ||
      a.ff1.K != d || a.ff2.ldc != d || a.out.ldc != d || M > 65536)
    return hipErrorInvalidValue;
  Launch L{};
  L.a = a;
  const int n_out = ceil_div(M, kOutBM) * (d / kBN), n_ln = ceil_div(M, kLnRows);
  const int n_ff1 = ceil_div(M, kFf1BM) * (ff / kBN), n_ff2 = ceil_div(M, kFf2BM) * (d / kBN);
  const int n_qkv = qkv ? ceil_div(M, kQkvBM) * (a.qkv.N / kBN) : 0;
  const int cnt[6] = {n_out, n_ln, n_ff1, n_ff2, n_ln, n_qkv};
  L.start[0] = 0;
  for (int p = 0; p < 6; ++p) L.start[p + 1] = L.start[p] + round8(cnt[p]);
  if (!a.fault) return hipErrorInvalidValue;
  const unsigned spin_limit = (unsigned)g_spin_limit.load(std::memory_order_relaxed);
  // producers' arrivals per complete row group: a GEMM tile adds 1 to each group it covers (its row block
  // spans whole groups), so a group is complete at (column tiles) arrivals; a LayerNorm unit covers half a group
  const int mult[6] = {d / kBN, 1, ff / kBN, d / kBN, 1, 0};
  const int unit[6] = {kChainRows, kLnRows, kChainRows, kChainRows, kLnRows, 0};
  for (int p = 0; p < 6; ++p) {
    ChainDep& x = L.dep[p];
    x.err = a.fault;
    x.spin_limit = spin_limit;
    x.pub = p < 5 ? a.cnt + (size_t)p * a.groups : nullptr;
    x.wait = p > 0 ? a.cnt + (size_t)(p - 1) * a.groups : nullptr;
    x.wait_mult = p > 0 ? mult[p - 1] : 0;
    x.wait_unit = p > 0 ? unit[p - 1] : 1;
  }
  const dim3 grid(L.start[6]), block(256);
  if (compute == F5H_C_BF16)
    hipLaunchKernelGGL(chain_kernel<bf16>, grid, block, 0, st, L);
  else
    hipLaunchKernelGGL(chain_kernel<f16>, grid, block, 0, st, L);
  return hipGetLastError();
}

void chain_set_spin_limit(long long limit) {
  g_spin_limit.store(limit < 0 ? (long long)kChainSpinLimit : std::min<long long>(limit, 0xffffffffll),
                     std::memory_order_relaxed);
}

}  // namespace f5h
