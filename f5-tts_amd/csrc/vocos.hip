// Vocos decoder kernels (mel -> waveform), gfx950. SURVEY §8(f1).
//
// The network is vocos' mel-24khz decoder (vocos package, unpinned in the reference's
// pyproject.toml:42; called at utils_infer.py:510-511 and runtime/triton_trtllm/benchmark.py:435):
//   backbone: Conv1d(100, 512, k7, pad 3) -> LayerNorm(eps 1e-6) -> 8 x ConvNeXtBlock
//             (dwconv k7 -> LayerNorm -> Linear 512->1536 -> GELU(erf) -> Linear 1536->512 ->
//              gamma * . -> + residual) -> final LayerNorm
//   head:     Linear(512, n_fft + 2) -> mag = clip(exp(.), max 100), phase -> S = mag e^{i phase}
//             -> iSTFT(n_fft 1024, hop 256, hann 1024, center) (restated in-tree by
//             runtime/triton_trtllm/scripts/export_vocoder_to_onnx.py:45-60 + conv_stft.py:201-234)
// The GEMMs run on gemm(); this file holds the glue kernels around them: the embed im2col,
// the magnitude/phase -> (re, im) map and the overlap-add with window-envelope division.
#include "common.h"
#include "kernels.h"

namespace f5h {

static inline unsigned vblk(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// out[(b*T + t)][c*7 + j] = mel[b][c][t + j - 3] (0 outside [0, T)); columns [C*7, Kp) zeroed.
// mel is vocos' channel-first [B][C][T] layout (the permute at utils_infer.py:508).
template <typename TO>
__global__ void vocos_im2col_kernel(const float* mel, int B, int T, int C, int Kp, TO* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * T * Kp) return;
  const int col = (int)(i % Kp);
  const int64_t row = i / Kp;
  const int b = (int)(row / T), t = (int)(row - (int64_t)b * T);
  float v = 0.f;
  if (col < C * 7) {
    const int c = col / 7, j = col - c * 7, q = t + j - 3;
    if (q >= 0 && q < T) v = mel[((int64_t)b * C + c) * T + q];
  }
  out[i] = from_f32<TO>(v);
}
hipError_t vocos_im2col(int compute, const float* mel, int B, int T, int C, int Kp, void* out, hipStream_t st) {
  if (Kp < C * 7 || Kp % 64) return hipErrorInvalidValue;
  const int64_t n = (int64_t)B * T * Kp;
  if (compute)
    hipLaunchKernelGGL(vocos_im2col_kernel<bf16>, dim3(vblk(n, 256)), dim3(256), 0, st, mel, B, T, C, Kp, (bf16*)out);
  else
    hipLaunchKernelGGL(vocos_im2col_kernel<float>, dim3(vblk(n, 256)), dim3(256), 0, st, mel, B, T, C, Kp,
                       (float*)out);
  return hipGetLastError();
}

// ISTFTHead.forward's pointwise part, in place on rows of ld floats: the head weight is packed
// so that columns (2k, 2k+1) = (log-magnitude, phase) of bin k; they become (re, im) =
// clip(exp(m), 100) * (cos p, sin p). Columns [2*bins, ld) are zeroed (K padding of the iDFT GEMM).
__global__ void vocos_spec_kernel(float* x, int64_t rows, int bins, int ld) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int half = ld / 2;
  if (i >= rows * half) return;
  const int64_t r = i / half;
  const int k = (int)(i - r * half);
  float2* p = reinterpret_cast<float2*>(x + r * ld) + k;
  if (k >= bins) {
    *p = make_float2(0.f, 0.f);
    return;
  }
  const float2 mp = *p;
  const float mag = fminf(expf(mp.x), 100.f);  // torch.clip(exp, max=1e2); NaN propagates as in torch
  float s, c;
  sincosf(mp.y, &s, &c);
  *p = make_float2(mag * c, mag * s);
}
hipError_t vocos_spec(float* x, int64_t rows, int bins, int ld, hipStream_t st) {
  if (ld % 2 || ld < 2 * bins) return hipErrorInvalidValue;
  const int64_t n = rows * (ld / 2);
  hipLaunchKernelGGL(vocos_spec_kernel, dim3(vblk(n, 256)), dim3(256), 0, st, x, rows, bins, ld);
  return hipGetLastError();
}

// torch.istft(center=True) tail: the iDFT GEMM already produced windowed frames
// fr[b*T + t][j] = win[j] * irfft(S[b, :, t])[j]; here y[b][n] = sum_t fr[t][p - t*hop] /
// sum_t win^2[p - t*hop], p = n + n_fft/2, over the frames covering p (output length (T-1)*hop).
// Every sample sums its <= n_fft/hop frames in a fixed order (deterministic, no atomics).
__global__ void vocos_ola_kernel(const float* fr, const float* win, int B, int T, int n_fft, int hop, float* y) {
  const int Lout = (T - 1) * hop;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * Lout) return;
  const int b = (int)(i / Lout), n = (int)(i - (int64_t)b * Lout);
  const int p = n + n_fft / 2;
  int t0 = p - n_fft + 1 > 0 ? (p - n_fft + 1 + hop - 1) / hop : 0;
  int t1 = min(p / hop, T - 1);
  float acc = 0.f, env = 0.f;
  for (int t = t0; t <= t1; ++t) {
    const int j = p - t * hop;
    const float w = win[j];
    acc += fr[((int64_t)b * T + t) * n_fft + j];
    env += w * w;
  }
  y[i] = acc / env;
}
hipError_t vocos_ola(const float* frames, const float* win, int B, int T, int n_fft, int hop, float* y,
                     hipStream_t st) {
  if (T < 1 || n_fft % hop) return hipErrorInvalidValue;
  const int64_t n = (int64_t)B * (T - 1) * hop;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(vocos_ola_kernel, dim3(vblk(n, 256)), dim3(256), 0, st, frames, win, B, T, n_fft, hop, y);
  return hipGetLastError();
}

}  // namespace f5h
