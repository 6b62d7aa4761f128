// Reverb and long-kernel convolution for gfx950.
//
//   ddsp/models/modules.py:21-26   Reverb.build_impulse
//   ddsp/models/modules.py:28-35   Reverb.forward  (IR padded/cropped to len(x), fft_convolve)
//   ddsp/core.py:169-176           fft_convolve    (large-N branch)
//
// The reference computes one 2T-point fp32 FFT convolution per batch item.  Only the first
// T outputs of the linear convolution are kept and the IR is zero beyond L' = min(L, T), so
// the uniformly partitioned overlap-save convolution of upols.hip (4096-point transforms in
// LDS, two rows per complex transform) is an exact restatement.  The IR spectrum is computed
// once (ddsp_hip_reverb_spectrum) and cached by the caller.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "upols.h"

namespace ddsp {

int direct_convolve(const float* sig, const float* ker, float* out, int64_t rows,
                    int64_t kernel_rows, int64_t n, void* stream);

namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int64_t kDirectMaxN = 4096;  // fft_convolve: direct LDS convolution up to this N

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Reverb.build_impulse (modules.py:21-26), t = fl32(i / sr) as torch.arange(L) / sr.
__global__ void build_impulse_kernel(const float* __restrict__ noise, const float* __restrict__ decay,
                                     const float* __restrict__ wet, float* __restrict__ imp,
                                     int64_t L, float sr) {
  const float d = -decay[0];
  // softplus(-decay) with torch's threshold 20
  const float sp = d > 20.0f ? d : log1pf(expf(d));
  const float neg = -sp;
  const float w = 1.0f / (1.0f + expf(-wet[0]));
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < L;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float t = (float)i / sr;
    const float env = expf((neg * t) * 500.0f);
    imp[i] = i == 0 ? 1.0f : (noise[i] * env) * w;
  }
}

// Reverb.build_impulse backward (modules.py:21-26): imp[i] = noise[i] env[i] w (i >= 1),
// env = exp(-softplus(-decay) t 500), w = sigmoid(wet); imp[0] = 1 carries no gradient.
// Taps i >= grad_len (cropped away by a shorter input) have zero gradient.
// Pass 1 (grid-stride over the taps): d_noise and per-workgroup fp64 partial sums of
// sum dimp*noise*env and sum dimp*noise*env*t; pass 2 (one workgroup) reduces them in a fixed
// order (deterministic) into d_wet and d_decay.
constexpr int kImpBlocks = 128;

__global__ void __launch_bounds__(256) impulse_backward_kernel(
    const float* __restrict__ noise, const float* __restrict__ decay, const float* __restrict__ wet,
    const float* __restrict__ dimp, int64_t grad_len, int64_t L, float sr, float* __restrict__ d_noise,
    double* __restrict__ partials) {
  __shared__ double red[32];
  const float d = -decay[0];
  const float sp = d > 20.0f ? d : log1pf(expf(d));
  const float neg = -sp;
  const float w = 1.0f / (1.0f + expf(-wet[0]));
  double aw = 0.0, ad = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < L; i += (int64_t)gridDim.x * blockDim.x) {
    const float t = (float)i / sr;
    const float env = expf((neg * t) * 500.0f);
    const float gi = (i >= 1 && i < grad_len) ? dimp[i] : 0.0f;
    d_noise[i] = gi * env * w;
    const float gne = gi * noise[i] * env;
    aw += (double)gne;
    ad += (double)gne * (double)t;
  }
  block_sum_double2(aw, ad, red);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = aw;
    partials[2 * blockIdx.x + 1] = ad;
  }
}

__global__ void __launch_bounds__(64) impulse_backward_finish_kernel(const double* __restrict__ partials, int nblk,
                                                                     const float* __restrict__ decay,
                                                                     const float* __restrict__ wet,
                                                                     float* __restrict__ d_decay,
                                                                     float* __restrict__ d_wet) {
  // one wave: strided loads in flight together, then a fixed shuffle tree (deterministic)
  double aw = 0.0, ad = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 64) {
    aw += partials[2 * i];
    ad += partials[2 * i + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    aw += __shfl_down(aw, o, 64);
    ad += __shfl_down(ad, o, 64);
  }
  if (threadIdx.x != 0) return;
  const float d = -decay[0];
  const float spg = d > 20.0f ? 1.0f : 1.0f / (1.0f + expf(-d));  // softplus'(d)
  const float w = 1.0f / (1.0f + expf(-wet[0]));
  d_wet[0] = (float)(aw * (double)w * (1.0 - (double)w));
  d_decay[0] = (float)(ad * (double)w * 500.0 * (double)spg);
}

unsigned grid_for(int64_t n) {
  return (unsigned)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384);
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

size_t ddsp_hip_reverb_spectrum_floats(int64_t n_samples, int64_t ir_length) {
  if (n_samples < 1 || ir_length < 1) return 0;
  return upols_spectrum_floats(1, std::min(ir_length, n_samples));
}

size_t ddsp_hip_reverb_workspace_size(int64_t batch, int64_t n_samples, int64_t ir_length) {
  if (batch < 1 || n_samples < 1 || ir_length < 1) return 0;
  return upols_workspace_bytes(batch, n_samples, true);
}

int ddsp_hip_reverb_build_impulse(const float* noise, const float* decay, const float* wet,
                                  float* impulse, int64_t length, float sample_rate, void* stream) {
  if (length < 1 || !noise || !decay || !wet || !impulse || !(sample_rate > 0)) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(build_impulse_kernel, dim3(grid_for(length)), dim3(256), 0, S(stream), noise, decay,
                     wet, impulse, length, sample_rate);
  return launch_status();
}

int ddsp_hip_reverb_impulse_spectrum(const float* noise, const float* decay, const float* wet, int64_t ir_length,
                                     float sample_rate, int64_t n_samples, float* spectrum, void* stream) {
  if (ir_length < 1 || n_samples < 1 || !noise || !decay || !wet || !spectrum || !(sample_rate > 0))
    return DDSP_HIP_EINVAL;
  return upols_impulse_spectrum(noise, decay, wet, std::min(ir_length, n_samples), sample_rate, spectrum, stream);
}

int ddsp_hip_reverb_spectrum(const float* impulse, int64_t ir_length, int64_t n_samples,
                             float* spectrum, void* stream) {
  if (ir_length < 1 || n_samples < 1 || !impulse || !spectrum) return DDSP_HIP_EINVAL;
  return upols_spectrum(impulse, 0, std::min(ir_length, n_samples), 1, spectrum, stream);
}

int ddsp_hip_reverb_apply(const float* x, const float* spectrum, float* out, int64_t batch,
                          int64_t n_samples, int64_t ir_length, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1) return DDSP_HIP_EINVAL;
  if (batch == 0) return DDSP_HIP_OK;
  if (!x || !spectrum || !out) return DDSP_HIP_EINVAL;
  return upols_apply(x, batch, n_samples, spectrum, std::min(ir_length, n_samples), false, out,
                     workspace, workspace_bytes, stream);
}

size_t ddsp_hip_reverb_cache_bytes(int64_t n_samples, int64_t ir_length) {
  if (n_samples < 1 || ir_length < 1) return 0;
  return upols_ir_cache_bytes(std::min(ir_length, n_samples));
}

int ddsp_hip_reverb_forward(const float* x, const float* noise, const float* decay, const float* wet,
                            int64_t ir_length, float sample_rate, int force, void* cache, size_t cache_bytes,
                            float* out, int64_t batch, int64_t n_samples, void* workspace, size_t workspace_bytes,
                            void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1 || !noise || !decay || !wet || !(sample_rate > 0))
    return DDSP_HIP_EINVAL;
  if (batch > 0 && (!x || !out)) return DDSP_HIP_EINVAL;
  if (!cache || cache_bytes < ddsp_hip_reverb_cache_bytes(n_samples, ir_length)) return DDSP_HIP_EWORKSPACE;
  return upols_reverb_cached(x, batch, n_samples, noise, decay, wet, std::min(ir_length, n_samples), sample_rate,
                             force, cache, out, workspace, workspace_bytes, stream);
}

int ddsp_hip_reverb_apply_transposed(const float* grad, const float* spectrum, float* grad_x, int64_t batch,
                                     int64_t n_samples, int64_t ir_length, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1) return DDSP_HIP_EINVAL;
  if (batch == 0) return DDSP_HIP_OK;
  if (!grad || !spectrum || !grad_x) return DDSP_HIP_EINVAL;
  return upols_apply(grad, batch, n_samples, spectrum, std::min(ir_length, n_samples), false, grad_x,
                     workspace, workspace_bytes, stream, true);
}

size_t ddsp_hip_reverb_input_spectra_bytes(int64_t batch, int64_t n_samples) {
  if (batch < 1 || n_samples < 1) return 0;
  return upols_spectra_bytes(batch, n_samples);
}

size_t ddsp_hip_reverb_backward_workspace_size(int64_t batch, int64_t n_samples, int64_t ir_length,
                                               int have_input_spectra) {
  if (batch < 1 || n_samples < 1 || ir_length < 1) return 0;
  return upols_backward_workspace_bytes(batch, n_samples, ir_length, have_input_spectra != 0);
}

int ddsp_hip_reverb_backward(const float* x, const float* input_spectra, const float* spectrum, const float* grad,
                             float* grad_x, float* grad_impulse, int64_t batch, int64_t n_samples,
                             int64_t ir_length, void* workspace, size_t workspace_bytes, void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1 || (!grad_x && !grad_impulse)) return DDSP_HIP_EINVAL;
  const int64_t kc = std::min(ir_length, n_samples);
  if (grad_impulse && kc < ir_length) {  // taps past the input length were cropped: zero gradient
    hipError_t e = hipMemsetAsync(grad_impulse + kc, 0, sizeof(float) * (ir_length - kc), S(stream));
    if (e != hipSuccess) return DDSP_HIP_ELAUNCH;
  }
  if (batch == 0) {
    if (!grad_impulse) return DDSP_HIP_OK;
    hipError_t e = hipMemsetAsync(grad_impulse, 0, sizeof(float) * kc, S(stream));
    return e == hipSuccess ? DDSP_HIP_OK : DDSP_HIP_ELAUNCH;
  }
  if (!grad || !spectrum || (grad_impulse && !x && !input_spectra)) return DDSP_HIP_EINVAL;
  return upols_backward(x, input_spectra, spectrum, grad, batch, n_samples, ir_length, grad_x, grad_impulse,
                        workspace, workspace_bytes, stream);
}

int ddsp_hip_reverb_backward_params(const float* x, const float* input_spectra, const float* spectrum, const float* grad,
                                    const float* noise, const float* decay, const float* wet, float sample_rate,
                                    float* grad_x, float* grad_noise, float* grad_decay, float* grad_wet, int64_t batch,
                                    int64_t n_samples, int64_t ir_length, void* workspace, size_t workspace_bytes,
                                    void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1 || !noise || !decay || !wet || !grad_noise || !grad_decay ||
      !grad_wet || !(sample_rate > 0))
    return DDSP_HIP_EINVAL;
  if (batch == 0) {  // no signal: no gradient reaches the impulse
    hipError_t e = hipMemsetAsync(grad_noise, 0, sizeof(float) * ir_length, S(stream));
    if (e == hipSuccess) e = hipMemsetAsync(grad_decay, 0, sizeof(float), S(stream));
    if (e == hipSuccess) e = hipMemsetAsync(grad_wet, 0, sizeof(float), S(stream));
    return e == hipSuccess ? DDSP_HIP_OK : DDSP_HIP_ELAUNCH;
  }
  if (!grad || !spectrum || (!x && !input_spectra)) return DDSP_HIP_EINVAL;
  const ImpulseGrad ig{noise, decay, wet, ir_length, sample_rate, grad_noise, grad_decay, grad_wet};
  return upols_backward(x, input_spectra, spectrum, grad, batch, n_samples, ir_length, grad_x, nullptr, workspace,
                        workspace_bytes, stream, &ig);
}

size_t ddsp_hip_reverb_impulse_backward_workspace_size(int64_t length) {
  (void)length;
  return 2 * sizeof(double) * kImpBlocks;
}

int ddsp_hip_reverb_impulse_backward(const float* noise, const float* decay, const float* wet,
                                     const float* grad_impulse, int64_t length, int64_t grad_length,
                                     float sample_rate, float* grad_noise, float* grad_decay, float* grad_wet,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  if (length < 1 || grad_length < 0 || !noise || !decay || !wet || !grad_impulse || !grad_noise ||
      !grad_decay || !grad_wet || !(sample_rate > 0))
    return DDSP_HIP_EINVAL;
  if (!workspace || workspace_bytes < ddsp_hip_reverb_impulse_backward_workspace_size(length))
    return DDSP_HIP_EWORKSPACE;
  const int nblk = (int)std::min<int64_t>(kImpBlocks, (length + 255) / 256);
  double* partials = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(impulse_backward_kernel, dim3(nblk), dim3(256), 0, S(stream), noise, decay, wet,
                     grad_impulse, std::min(grad_length, length), length, sample_rate, grad_noise, partials);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(impulse_backward_finish_kernel, dim3(1), dim3(64), 0, S(stream), partials, nblk, decay, wet,
                     grad_decay, grad_wet);
  return launch_status();
}

size_t ddsp_hip_fft_convolve_workspace_size(int64_t rows, int64_t kernel_rows, int64_t n) {
  if (rows < 1 || n < 1 || n <= kDirectMaxN) return 0;
  const bool per_row = kernel_rows != 1;
  return align256(sizeof(float) * upols_spectrum_floats(kernel_rows, n)) +
         upols_workspace_bytes(rows, n, !per_row);
}

int ddsp_hip_fft_convolve(const float* signal, const float* kernel, float* out, int64_t rows,
                          int64_t kernel_rows, int64_t n, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (rows < 0 || n < 1 || (kernel_rows != 1 && kernel_rows != rows)) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!signal || !kernel || !out || rows > INT32_MAX) return DDSP_HIP_EINVAL;
  if (n <= kDirectMaxN) return direct_convolve(signal, kernel, out, rows, kernel_rows, n, stream);
  const bool per_row = kernel_rows != 1;
  const size_t spec_bytes = align256(sizeof(float) * upols_spectrum_floats(kernel_rows, n));
  if (!workspace || workspace_bytes < ddsp_hip_fft_convolve_workspace_size(rows, kernel_rows, n))
    return DDSP_HIP_EWORKSPACE;
  float* spec = reinterpret_cast<float*>(workspace);
  int st = upols_spectrum(kernel, n, n, kernel_rows, spec, stream);
  if (st) return st;
  return upols_apply(signal, rows, n, spec, n, per_row, out,
                     reinterpret_cast<char*>(workspace) + spec_bytes, workspace_bytes - spec_bytes,
                     stream);
}

const char* ddsp_hip_status_string(int status) {
  switch (status) {
    case DDSP_HIP_OK: return "ok";
    case DDSP_HIP_EINVAL: return "invalid argument or shape";
    case DDSP_HIP_ELAUNCH: return "HIP launch/runtime error";
    case DDSP_HIP_EFFT: return "FFT convolution error";
    case DDSP_HIP_EWORKSPACE: return "workspace missing or too small";
    case DDSP_HIP_ERANGE: return "input outside the supported range";
    default: return "unknown status";
  }
}

int ddsp_hip_version(void) { return 102; }

}  // extern "C"
