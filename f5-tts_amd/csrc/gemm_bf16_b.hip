// bf16 GEMM launchers, epilogues EPI_STORE, EPI_SILU, EPI_GELU_ERF, EPI_RESID_FILL, EPI_INPROJ, EPI_STORE16 (see gemm_impl.h)
#include "gemm_impl.h"

namespace f5h {
hipError_t gemm_launch_bf16_b(int epi, const GemmArgs& a, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_t<bf16, EPI_STORE>(a, st);
    case EPI_SILU: return launch_t<bf16, EPI_SILU>(a, st);
    case EPI_GELU_ERF: return launch_t<bf16, EPI_GELU_ERF>(a, st);
    case EPI_RESID_FILL: return launch_t<bf16, EPI_RESID_FILL>(a, st);
    case EPI_INPROJ: return launch_t<bf16, EPI_INPROJ>(a, st);
    case EPI_STORE16: return launch_t<bf16, EPI_STORE16>(a, st);
  }
  return hipErrorInvalidValue;
}
}  // namespace f5h
