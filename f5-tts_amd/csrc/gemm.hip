// GEMM host side: the per-shape tile choice and the compute-mode dispatcher. Kernels and launch
// templates: gemm_impl.h; instantiations: gemm_bf16_*.hip, gemm_f16_*.hip, gemm_f32.hip.
#include "gemm_impl.h"

namespace f5h {

static int g_force_cfg = -1;  // f5h_gemm_force_config
static int gemm_env_cfg() {
  static int v = [] {
    const char* e = getenv("F5H_GEMM_CFG");
    return e ? atoi(e) : -1;
  }();
  return v;
}


// The 256x256 configuration of the large batches: 11 (ping-pong), 12 (8-phase) or 13 (persistent ping-pong);
// env F5H_LARGE_CFG.
static int large_cfg() {
  static const int v = [] {
    const char* e = getenv("F5H_LARGE_CFG");
    const int c = e ? atoi(e) : 11;
    return (c == 12 || c == 13) ? c : 11;
  }();
  return v;
}

// the persistent kernel's tile grouping (F5H_GEMM_GROUP_M, default 1: n-fastest, the non-persistent order)
int gemm_group_m() {
  static const int v = [] {
    const char* e = getenv("F5H_GEMM_GROUP_M");
    const int g = e ? atoi(e) : 1;
    return g > 1 && g <= 64 ? g : 1;
  }();
  return v;
}

// compute units of the current device (the persistent kernel's grid), cached per device
int gemm_num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// Tile choice for a bf16 GEMM among the 2-blocks-per-CU configurations 0, 1, 5: time ~
// rounds x tile work / relative efficiency, with rounds = ceil(tiles / 512 block slots) and
// efficiencies from tools/gemm_tune.py on MI355X (C3-sized GEMMs: 64x128 0.57, 128x128 0.74,
// 192x128 0.86 of the best). C2 picks 192x128 for QKV, 128x128 for FFN1, 64x128 for N = 1024.
static int pick_cfg(const GemmArgs& a) {
  // Large batches (C3/C4/C5: thousands of 256x256 tiles, many rounds per CU): the 8-wave
  // ping-pong 256x256 kernel (cfg 11), 5-6 % faster than the best 4-wave tile there
  // (tools/gemm_tune.py: C3 QKV 856 vs 907 us, C3 FFN2 512 vs 544 us).
  if (a.K % 64 == 0 && (int64_t)((a.M + 255) / 256) * ((a.N + 255) / 256) >= 1024) return large_cfg();
  struct Opt { int cfg, bm, bn; float eff; };
  constexpr Opt opts[3] = {{5, 192, 128, 0.86f}, {1, 128, 128, 0.74f}, {0, 64, 128, 0.57f}};
  int best = 0;
  double tbest = 1e300;
  for (const Opt& o : opts) {
    const int64_t tiles = (int64_t)((a.M + o.bm - 1) / o.bm) * ((a.N + o.bn - 1) / o.bn);
    const double t = (double)((tiles + 511) / 512) * o.bm * o.bn / o.eff;
    if (t < tbest * 0.999) tbest = t, best = o.cfg;
  }
  return best;
}

// Tuning hook: F5H_GEMM_MAP="N:K:cfg,N:K:cfg,..." pins a configuration per (N, K) shape.
static int gemm_map_cfg(int N, int K) {
  struct E { int n, k, c; };
  static std::vector<E> m = [] {
    std::vector<E> v;
    const char* e = getenv("F5H_GEMM_MAP");
    while (e && *e) {
      int n, k, c, used = 0;
      if (sscanf(e, "%d:%d:%d%n", &n, &k, &c, &used) != 3) break;
      v.push_back({n, k, c});
      e += used;
      if (*e == ',') ++e;
    }
    return v;
  }();
  for (const E& x : m)
    if (x.n == N && x.k == K) return x.c;
  return -1;
}


int gemm_select_cfg(const GemmArgs& a) {
  int cfg = g_force_cfg >= 0 ? g_force_cfg : gemm_env_cfg();
  if (cfg < 0) cfg = gemm_map_cfg(a.N, a.K);
  if (cfg < 0) cfg = pick_cfg(a);
  return cfg;
}

hipError_t gemm_launch_bf16_a(int epi, const GemmArgs& a, hipStream_t st);
hipError_t gemm_launch_bf16_b(int epi, const GemmArgs& a, hipStream_t st);
hipError_t gemm_launch_f16_a(int epi, const GemmArgs& a, hipStream_t st);
hipError_t gemm_launch_f16_b(int epi, const GemmArgs& a, hipStream_t st);
hipError_t gemm_launch_f32(int epi, const GemmArgs& a, hipStream_t st);

// the hot epilogues (QKV, RESID, RESID16, GELU-tanh, GELU-erf operand) in the *_a units, the rest in *_b
static bool hot_epi(int epi) {
  return epi == EPI_QKV || epi == EPI_RESID || epi == EPI_RESID16 || epi == EPI_GELU_TANH || epi == EPI_GELU_ERF_OP;
}

void gemm_force_config(int cfg) { g_force_cfg = cfg; }

hipError_t gemm(int compute, int epi, const GemmArgs& a, hipStream_t st) {
  const int bke = compute ? 64 : 32;
  if (a.K % bke != 0 || a.M < 0 || a.N <= 0 || a.lda % 8 || a.ldw % 8) return hipErrorInvalidValue;
  // 8-column epilogue chunks: vector paths need 16 B alignment of every operand row
  if (epi == EPI_INPROJ && (a.ldc % 8 || a.ld_add % 8 || a.N % 8)) return hipErrorInvalidValue;
  if (epi == EPI_QKV && (a.N % 64)) return hipErrorInvalidValue;
  // a second A panel starts on a stage boundary (64 bf16 / 32 fp32 columns)
  if (a.A2 && (a.k_split <= 0 || a.k_split % 64 || a.k_split >= a.K)) return hipErrorInvalidValue;
  if (a.resid && epi != EPI_RESID && epi != EPI_RESID16) return hipErrorInvalidValue;
  switch (compute) {
    case F5H_C_BF16: return hot_epi(epi) ? gemm_launch_bf16_a(epi, a, st) : gemm_launch_bf16_b(epi, a, st);
    case F5H_C_FP16: return hot_epi(epi) ? gemm_launch_f16_a(epi, a, st) : gemm_launch_f16_b(epi, a, st);
    default: return gemm_launch_f32(epi, a, st);
  }
}

}  // namespace f5h
