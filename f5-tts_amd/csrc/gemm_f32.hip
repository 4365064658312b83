// fp32 (parity mode) GEMM launchers (see gemm_impl.h)
#include "gemm_impl.h"

namespace f5h {
hipError_t gemm_launch_f32(int epi, const GemmArgs& a, hipStream_t st) { return launch_epi<float>(epi, a, st); }
}  // namespace f5h
