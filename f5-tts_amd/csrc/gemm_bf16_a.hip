// bf16 GEMM launchers, epilogues EPI_QKV, EPI_RESID, EPI_RESID16, EPI_GELU_TANH, EPI_GELU_ERF_OP (see gemm_impl.h)
#include "gemm_impl.h"

namespace f5h {
hipError_t gemm_launch_bf16_a(int epi, const GemmArgs& a, hipStream_t st) {
  switch (epi) {
    case EPI_QKV: return launch_t<bf16, EPI_QKV>(a, st);
    case EPI_RESID: return launch_t<bf16, EPI_RESID>(a, st);
    case EPI_RESID16: return launch_t<bf16, EPI_RESID16>(a, st);
    case EPI_GELU_TANH: return launch_t<bf16, EPI_GELU_TANH>(a, st);
    case EPI_GELU_ERF_OP: return launch_t<bf16, EPI_GELU_ERF_OP>(a, st);
  }
  return hipErrorInvalidValue;
}
}  // namespace f5h
