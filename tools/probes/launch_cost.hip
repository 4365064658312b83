// Launch-cost and implicit-sync probe (gfx950, ROCm 7.2):
//   ./launch_cost          what one dependent kernel boundary costs inside a replayed hipGraph: a graph of
//                          K kernels (empty, or each streaming `bytes` in + out) replayed R times
//   ./launch_cost sync     which host API calls wait for unrelated device work: a ~0.5 s spin kernel runs
//                          on stream B while each call is timed on the host (graph capture, instantiate,
//                          graph-exec destroy, hipMalloc / hipFree, stream and event calls)
//   ./launch_cost trace    the graph part with a progress line to stderr before every HIP call (finds the
//                          call a profiler crash happens in)
//   hipcc -O3 --offload-arch=gfx950 launch_cost.hip -o launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static bool g_trace = false;
#define CK(x)                                                                              \
  do {                                                                                     \
    if (g_trace) std::fprintf(stderr, "[call] %s\n", #x);                                  \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) b[i] = a[i];
}

// spins for `ticks` of the 100 MHz wall clock (s_memrealtime), one wave
__global__ void spin_kernel(unsigned long long ticks, int* flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  if (flag && threadIdx.x == 0) flag[0] = 1;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hipGraphExec_t make_graph(int kind, int K, int grid, uint4* a, uint4* b, int n, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < K; ++k) {
    if (kind == 0)
      hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, nullptr);
    else if (k & 1)
      hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, st, b, a, n);
    else
      hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, st, a, b, n);
  }
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  return ge;
}

static double run(int kind, int K, int R, int grid, size_t bytes, hipStream_t st) {
  uint4 *a = nullptr, *b = nullptr;
  const int n = (int)(bytes / 16);
  if (kind) {
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
  }
  hipGraphExec_t ge = make_graph(kind, K, grid, a, b, n, st);
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  CK(hipGraphExecDestroy(ge));
  if (a) CK(hipFree(a));
  if (b) CK(hipFree(b));
  return 1000.0 * ms / ((double)K * R);
}

static void sync_probe() {
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  int* flag;
  CK(hipMalloc(&flag, 64));
  hipGraphExec_t old = make_graph(0, 20, 256, nullptr, nullptr, 0, sa);
  CK(hipGraphLaunch(old, sa));
  CK(hipStreamSynchronize(sa));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const unsigned long long spin = 50000000ull;  // 0.5 s of 100 MHz ticks
  auto timed = [&](const char* what, auto&& fn) {
    CK(hipMemsetAsync(flag, 0, 4, sb));
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, sb, spin, flag);
    CK(hipGetLastError());
    // let the spin start
    const double t0 = now_ms();
    while (now_ms() - t0 < 20.0) {}
    const double t1 = now_ms();
    fn();
    const double t2 = now_ms();
    const bool busy = hipStreamQuery(sb) == hipErrorNotReady;
    (void)hipGetLastError();
    std::printf("%-44s host %8.3f ms   spin still running after: %s\n", what, t2 - t1, busy ? "yes" : "NO (waited)");
    CK(hipStreamSynchronize(sb));
  };
  timed("capture + instantiate (20 empty kernels)", [&] {
    hipGraphExec_t g = make_graph(0, 20, 256, nullptr, nullptr, 0, sa);
    CK(hipGraphExecDestroy(g));  // timed with it below, separately too
  });
  hipGraphExec_t keep = nullptr;
  timed("capture + instantiate only", [&] { keep = make_graph(0, 20, 256, nullptr, nullptr, 0, sa); });
  timed("hipGraphLaunch (replayed exec) on stream A", [&] { CK(hipGraphLaunch(keep, sa)); });
  CK(hipStreamSynchronize(sa));
  timed("hipGraphExecDestroy (idle exec)", [&] { CK(hipGraphExecDestroy(keep)); });
  timed("hipGraphExecDestroy (exec replayed earlier)", [&] { CK(hipGraphExecDestroy(old)); });
  void* p = nullptr;
  timed("hipMalloc 64 MB", [&] { CK(hipMalloc(&p, 64 << 20)); });
  timed("hipFree 64 MB", [&] { CK(hipFree(p)); });
  timed("hipEventRecord + hipEventQuery on A", [&] {
    CK(hipEventRecord(ev, sa));
    (void)hipEventQuery(ev);
    (void)hipGetLastError();
  });
  hipStream_t sc;
  timed("hipStreamCreate", [&] { CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking)); });
  timed("hipStreamDestroy", [&] { CK(hipStreamDestroy(sc)); });
  timed("hipMemsetAsync on A", [&] { CK(hipMemsetAsync(flag + 8, 0, 4, sa)); });
  CK(hipStreamSynchronize(sa));
}

// ./launch_cost count K R: replay a graph of K empty kernels R times, printing the running number of
// graph-launched dispatches to stderr after every replay (the profiler-crash threshold)
static void count_probe(int K, int R) {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipGraphExec_t ge = make_graph(0, K, 256, nullptr, nullptr, 0, st);
  for (int r = 0; r < R; ++r) {
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    std::fprintf(stderr, "[count] replays %d dispatches %d\n", r + 1, (r + 1) * K);
  }
  CK(hipGraphExecDestroy(ge));
  std::printf("count probe done: %d replays of %d kernels\n", R, K);
}

int main(int argc, char** argv) {
  if (argc > 1 && !std::strcmp(argv[1], "sync")) {
    sync_probe();
    return 0;
  }
  if (argc > 3 && !std::strcmp(argv[1], "count")) {
    count_probe(std::atoi(argv[2]), std::atoi(argv[3]));
    return 0;
  }
  g_trace = argc > 1 && !std::strcmp(argv[1], "trace");
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int K = 150, R = 20;
  for (int grid : {256, 512, 1024})
    std::printf("empty kernel, grid %4d x 256: %.2f us per kernel (graph of %d, %d replays)\n", grid,
                run(0, K, R, grid, 0, st), K, R);
  for (size_t mb : {1, 4, 8, 16})
    for (int grid : {512, 1024})
      std::printf("copy %2zu MB, grid %4d x 256: %.2f us per kernel\n", mb, grid, run(1, K, R, grid, mb << 20, st));
  return 0;
}
