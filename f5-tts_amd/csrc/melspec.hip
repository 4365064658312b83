// Log-mel front end kernels (wav -> vocos log-mel), gfx950. SURVEY §8(f2).
//
// Reference: get_vocos_mel_spectrogram (src/f5_tts/model/modules.py:80-109), i.e.
// torchaudio.transforms.MelSpectrogram(sr 24000, n_fft 1024, win 1024, hop 256, n_mels 100,
// power 1, center, reflect pad, norm None, htk scale) followed by clamp(1e-5).log(); called by
// CFM.sample on raw-audio conditioning (cfm.py:106-108). The DFT and the filterbank run as fp32
// MFMA GEMMs (gemm()); these kernels frame the signal, take magnitudes and apply the log.
#include "common.h"
#include "kernels.h"

namespace f5h {

static inline unsigned mblk(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// frames[b*T + t][j] = wav[b][reflect(t*hop + j - n_fft/2)] (torch.stft center=True, pad_mode
// "reflect": the edge sample is not repeated). The window lives in the DFT basis.
__global__ void mel_frames_kernel(const float* wav, int B, int L, int T, int n_fft, int hop, float* frames) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * T * n_fft) return;
  const int j = (int)(i % n_fft);
  const int64_t r = i / n_fft;
  const int b = (int)(r / T), t = (int)(r - (int64_t)b * T);
  int p = t * hop + j - n_fft / 2;
  if (p < 0) p = -p;
  if (p >= L) p = 2 * (L - 1) - p;
  frames[i] = wav[(int64_t)b * L + p];
}
hipError_t mel_frames(const float* wav, int B, int L, int T, int n_fft, int hop, float* frames, hipStream_t st) {
  if (L <= n_fft / 2) return hipErrorInvalidValue;  // reflect padding needs L > n_fft/2 (as torch)
  const int64_t n = (int64_t)B * T * n_fft;
  hipLaunchKernelGGL(mel_frames_kernel, dim3(mblk(n, 256)), dim3(256), 0, st, wav, B, L, T, n_fft, hop, frames);
  return hipGetLastError();
}

// mag[r][k] = |X_k| = sqrt(re^2 + im^2) from (re, im) interleaved rows of ld_spec; k in [bins, ld_mag) -> 0
__global__ void mel_mag_kernel(const float* spec, int64_t rows, int bins, int ld_spec, int ld_mag, float* mag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * ld_mag) return;
  const int64_t r = i / ld_mag;
  const int k = (int)(i - r * ld_mag);
  float m = 0.f;
  if (k < bins) {
    const float2 z = reinterpret_cast<const float2*>(spec + r * ld_spec)[k];
    m = sqrtf(z.x * z.x + z.y * z.y);
  }
  mag[i] = m;
}
hipError_t mel_mag(const float* spec, int64_t rows, int bins, int ld_spec, int ld_mag, float* mag, hipStream_t st) {
  if (ld_spec % 2 || ld_spec < 2 * bins || ld_mag < bins) return hipErrorInvalidValue;
  const int64_t n = rows * ld_mag;
  hipLaunchKernelGGL(mel_mag_kernel, dim3(mblk(n, 256)), dim3(256), 0, st, spec, rows, bins, ld_spec, ld_mag, mag);
  return hipGetLastError();
}

// out[b][m][t] = log(max(mel[b*T + t][m], 1e-5)): the [B, n_mels, T] layout the reference returns
__global__ void mel_log_kernel(const float* mel, int B, int T, int n_mels, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * n_mels * T) return;
  const int t = (int)(i % T);
  const int64_t bm = i / T;
  const int m = (int)(bm % n_mels), b = (int)(bm / n_mels);
  out[i] = logf(fmaxf(mel[((int64_t)b * T + t) * n_mels + m], 1e-5f));
}
hipError_t mel_log(const float* mel, int B, int T, int n_mels, float* out, hipStream_t st) {
  const int64_t n = (int64_t)B * n_mels * T;
  hipLaunchKernelGGL(mel_log_kernel, dim3(mblk(n, 256)), dim3(256), 0, st, mel, B, T, n_mels, out);
  return hipGetLastError();
}

}  // namespace f5h
