// Reverb and long-kernel convolution for gfx950, rocFFT-backed.
//
//   ddsp/models/modules.py:21-26   Reverb.build_impulse
//   ddsp/models/modules.py:28-35   Reverb.forward  (IR padded/cropped to len(x), fft_convolve)
//   ddsp/core.py:169-176           fft_convolve    (large-N branch)
//
// The reference computes one 2T-point fp32 FFT convolution per batch item.  Only the first
// T outputs of the linear convolution are kept and the IR is zero beyond L' = min(L, T), so
// any FFT length >= T + L' - 1 gives the same result; we pick the smallest 2^a 3^b 5^c
// length (rocFFT's native radices).  The IR spectrum is computed once
// (ddsp_hip_reverb_spectrum) and cached by the caller; a forward then costs one batched
// real-to-complex FFT, a complex scale by the shared spectrum, and one batched inverse.
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace ddsp {

int direct_convolve(const float* sig, const float* ker, float* out, int64_t rows,
                    int64_t kernel_rows, int64_t n, void* stream);

namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int64_t kDirectMaxN = 4096;  // fft_convolve: direct LDS convolution up to this N

int64_t good_fft_size(int64_t n) {
  static const bool pow2 = [] {
    const char* e = std::getenv("DDSP_HIP_FFT_POW2");
    return e && e[0] == '1';
  }();
  n = std::max<int64_t>(n, 2);
  if (pow2) {
    int64_t p = 2;
    while (p < n) p <<= 1;
    return p;
  }
  int64_t best = INT64_MAX;
  for (int64_t a = 2; a < 4 * n; a *= 2)        // even length (real transform)
    for (int64_t b = a; b < 4 * n; b *= 3)
      for (int64_t c = b; c < 4 * n; c *= 5)
        if (c >= n && c < best) best = c;
  return best;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ------------------------- rocFFT plan cache -------------------------
struct Plan {
  rocfft_plan plan = nullptr;
  size_t work = 0;
};

std::mutex g_mu;
std::map<std::tuple<int, int64_t, int64_t, int>, Plan> g_plans;  // (device, n, batch, dir)

int get_plan(int64_t n, int64_t batch, bool forward, Plan* out) {
  static std::once_flag once;
  std::call_once(once, [] { rocfft_setup(); });
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return DDSP_HIP_ELAUNCH;
  std::lock_guard<std::mutex> lock(g_mu);
  auto key = std::make_tuple(dev, n, batch, forward ? 1 : 0);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    *out = it->second;
    return DDSP_HIP_OK;
  }
  rocfft_plan_description desc = nullptr;
  if (rocfft_plan_description_create(&desc) != rocfft_status_success) return DDSP_HIP_EFFT;
  const size_t real_dist = (size_t)n + 2, cplx_dist = (size_t)n / 2 + 1, stride = 1;
  rocfft_status st;
  if (forward)
    st = rocfft_plan_description_set_data_layout(desc, rocfft_array_type_real,
                                                 rocfft_array_type_hermitian_interleaved, nullptr,
                                                 nullptr, 1, &stride, real_dist, 1, &stride, cplx_dist);
  else
    st = rocfft_plan_description_set_data_layout(desc, rocfft_array_type_hermitian_interleaved,
                                                 rocfft_array_type_real, nullptr, nullptr, 1, &stride,
                                                 cplx_dist, 1, &stride, real_dist);
  if (st != rocfft_status_success) {
    rocfft_plan_description_destroy(desc);
    return DDSP_HIP_EFFT;
  }
  Plan p;
  const size_t len = (size_t)n;
  st = rocfft_plan_create(&p.plan, rocfft_placement_inplace,
                          forward ? rocfft_transform_type_real_forward : rocfft_transform_type_real_inverse,
                          rocfft_precision_single, 1, &len, (size_t)batch, desc);
  rocfft_plan_description_destroy(desc);
  if (st != rocfft_status_success) return DDSP_HIP_EFFT;
  if (rocfft_plan_get_work_buffer_size(p.plan, &p.work) != rocfft_status_success) return DDSP_HIP_EFFT;
  g_plans[key] = p;
  *out = p;
  return DDSP_HIP_OK;
}

size_t plan_work(int64_t n, int64_t batch) {
  Plan f, i;
  if (get_plan(n, batch, true, &f) || get_plan(n, batch, false, &i)) return 0;
  return std::max(f.work, i.work);
}

int exec_plan(const Plan& p, void* buf, void* work, void* stream) {
  rocfft_execution_info info = nullptr;
  if (rocfft_execution_info_create(&info) != rocfft_status_success) return DDSP_HIP_EFFT;
  rocfft_execution_info_set_stream(info, stream);
  if (p.work) rocfft_execution_info_set_work_buffer(info, work, p.work);
  void* in[1] = {buf};
  const rocfft_status st = rocfft_execute(p.plan, in, nullptr, info);
  rocfft_execution_info_destroy(info);
  return st == rocfft_status_success ? DDSP_HIP_OK : DDSP_HIP_EFFT;
}

// ------------------------- element kernels -------------------------
// rows of `len` valid samples (source row stride src_ld) -> rows of n+2 floats, zero padded
__global__ void pad_rows_kernel(const float* __restrict__ src, int64_t src_ld, int64_t len,
                                float* __restrict__ dst, int64_t n2, int64_t rows) {
  const int64_t total = rows * n2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / n2, c = i - r * n2;
    dst[i] = c < len ? src[r * src_ld + c] : 0.0f;
  }
}

// X[r][k] *= H[r or 0][k] / n   (complex, interleaved, n/2+1 bins per row, row stride n+2 floats)
__global__ void spectrum_mul_kernel(float2* __restrict__ X, const float2* __restrict__ Hs,
                                    int64_t hs_ld /*in float2; 0 = broadcast*/, int64_t bins,
                                    int64_t ld /*float2 per row*/, int64_t rows, float scale) {
  const int64_t total = rows * bins;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / bins, k = i - r * bins;
    const float2 x = X[r * ld + k];
    const float2 h = Hs[r * hs_ld + k];
    X[r * ld + k] = make_float2((x.x * h.x - x.y * h.y) * scale, (x.x * h.y + x.y * h.x) * scale);
  }
}

__global__ void crop_rows_kernel(const float* __restrict__ src, int64_t src_ld,
                                 float* __restrict__ dst, int64_t len, int64_t rows) {
  const int64_t total = rows * len;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / len, c = i - r * len;
    dst[i] = src[r * src_ld + c];
  }
}

__global__ void copy_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

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

unsigned grid_for(int64_t n) {
  return (unsigned)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 16384);
}

// Generic FFT convolution of rows: out[r] = (sig[r] * ker[kr])[0:len] with the kernel's
// non-zero support in [0, klen).  nfft >= len + klen - 1.
int fft_conv_rows(const float* sig, int64_t sig_ld, const float* ker_spec_or_null,
                  const float* ker, int64_t ker_ld, int64_t klen, int64_t kernel_rows, float* out,
                  int64_t rows, int64_t len, int64_t nfft, void* ws, size_t ws_bytes, void* stream) {
  const int64_t n2 = nfft + 2;
  Plan fwd, inv;
  int st;
  if ((st = get_plan(nfft, rows, true, &fwd)) || (st = get_plan(nfft, rows, false, &inv))) return st;
  Plan kfwd = fwd;
  if (!ker_spec_or_null && kernel_rows != rows)
    if ((st = get_plan(nfft, kernel_rows, true, &kfwd))) return st;
  const size_t sig_bytes = align256(sizeof(float) * (size_t)(rows * n2));
  const size_t ker_bytes = ker_spec_or_null ? 0 : align256(sizeof(float) * (size_t)(kernel_rows * n2));
  const size_t work = std::max({fwd.work, inv.work, kfwd.work});
  if (!ws || ws_bytes < sig_bytes + ker_bytes + work) return DDSP_HIP_EWORKSPACE;
  float* xb = reinterpret_cast<float*>(ws);
  float* kb = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + sig_bytes);
  void* wk = reinterpret_cast<char*>(ws) + sig_bytes + ker_bytes;

  hipLaunchKernelGGL(pad_rows_kernel, dim3(grid_for(rows * n2)), dim3(256), 0, S(stream), sig, sig_ld,
                     len, xb, n2, rows);
  if ((st = launch_status())) return st;
  if ((st = exec_plan(fwd, xb, wk, stream))) return st;
  const float2* hs;
  int64_t hs_ld;
  if (ker_spec_or_null) {
    hs = reinterpret_cast<const float2*>(ker_spec_or_null);
    hs_ld = 0;
  } else {
    hipLaunchKernelGGL(pad_rows_kernel, dim3(grid_for(kernel_rows * n2)), dim3(256), 0, S(stream), ker,
                       ker_ld, klen, kb, n2, kernel_rows);
    if ((st = launch_status())) return st;
    if ((st = exec_plan(kfwd, kb, wk, stream))) return st;
    hs = reinterpret_cast<const float2*>(kb);
    hs_ld = kernel_rows == 1 ? 0 : n2 / 2;
  }
  hipLaunchKernelGGL(spectrum_mul_kernel, dim3(grid_for(rows * (nfft / 2 + 1))), dim3(256), 0, S(stream),
                     reinterpret_cast<float2*>(xb), hs, hs_ld, nfft / 2 + 1, n2 / 2, rows,
                     1.0f / (float)nfft);
  if ((st = launch_status())) return st;
  if ((st = exec_plan(inv, xb, wk, stream))) return st;
  hipLaunchKernelGGL(crop_rows_kernel, dim3(grid_for(rows * len)), dim3(256), 0, S(stream), xb, n2, out,
                     len, rows);
  return launch_status();
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int64_t ddsp_hip_reverb_fft_size(int64_t n_samples, int64_t ir_length) {
  const int64_t le = std::min(ir_length, n_samples);
  return good_fft_size(n_samples + std::max<int64_t>(le, 1) - 1);
}

size_t ddsp_hip_reverb_workspace_size(int64_t batch, int64_t n_samples, int64_t ir_length) {
  if (batch < 1 || n_samples < 1 || ir_length < 1) return 0;
  const int64_t nfft = ddsp_hip_reverb_fft_size(n_samples, ir_length);
  const size_t rows = (size_t)std::max<int64_t>(batch, 1);
  return align256(sizeof(float) * rows * (size_t)(nfft + 2)) + plan_work(nfft, batch) +
         plan_work(nfft, 1) + 256;
}

int ddsp_hip_reverb_build_impulse(const float* noise, const float* decay, const float* wet,
                                  float* impulse, int64_t length, float sample_rate, void* stream) {
  if (length < 1 || !noise || !decay || !wet || !impulse || !(sample_rate > 0)) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(build_impulse_kernel, dim3(grid_for(length)), dim3(256), 0, S(stream), noise, decay,
                     wet, impulse, length, sample_rate);
  return launch_status();
}

int ddsp_hip_reverb_spectrum(const float* impulse, int64_t ir_length, int64_t n_samples,
                             float* spectrum, void* workspace, size_t workspace_bytes,
                             void* stream) {
  if (ir_length < 1 || n_samples < 1 || !impulse || !spectrum) return DDSP_HIP_EINVAL;
  const int64_t nfft = ddsp_hip_reverb_fft_size(n_samples, ir_length);
  const int64_t le = std::min(ir_length, n_samples);
  Plan fwd;
  int st;
  if ((st = get_plan(nfft, 1, true, &fwd))) return st;
  const size_t buf = align256(sizeof(float) * (size_t)(nfft + 2));
  if (!workspace || workspace_bytes < buf + fwd.work) return DDSP_HIP_EWORKSPACE;
  float* b = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(pad_rows_kernel, dim3(grid_for(nfft + 2)), dim3(256), 0, S(stream), impulse,
                     (int64_t)0, le, b, nfft + 2, (int64_t)1);
  if ((st = launch_status())) return st;
  if ((st = exec_plan(fwd, b, reinterpret_cast<char*>(workspace) + buf, stream))) return st;
  hipLaunchKernelGGL(copy_kernel, dim3(grid_for(nfft + 2)), dim3(256), 0, S(stream), b, spectrum,
                     nfft + 2);
  return launch_status();
}

int ddsp_hip_reverb_apply(const float* x, const float* spectrum, float* out, int64_t batch,
                          int64_t n_samples, int64_t ir_length, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (batch < 0 || n_samples < 1 || ir_length < 1) return DDSP_HIP_EINVAL;
  if (batch == 0) return DDSP_HIP_OK;
  if (!x || !spectrum || !out) return DDSP_HIP_EINVAL;
  const int64_t nfft = ddsp_hip_reverb_fft_size(n_samples, ir_length);
  return fft_conv_rows(x, n_samples, spectrum, nullptr, 0, 0, 1, out, batch, n_samples, nfft, workspace,
                       workspace_bytes, stream);
}

size_t ddsp_hip_fft_convolve_workspace_size(int64_t rows, int64_t kernel_rows, int64_t n) {
  if (rows < 1 || n < 1 || n <= kDirectMaxN) return 0;
  const int64_t nfft = good_fft_size(2 * n - 1);
  return align256(sizeof(float) * (size_t)(rows * (nfft + 2))) +
         align256(sizeof(float) * (size_t)(kernel_rows * (nfft + 2))) +
         std::max(plan_work(nfft, rows), plan_work(nfft, kernel_rows)) + 256;
}

int ddsp_hip_fft_convolve(const float* signal, const float* kernel, float* out, int64_t rows,
                          int64_t kernel_rows, int64_t n, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (rows < 0 || n < 1 || (kernel_rows != 1 && kernel_rows != rows)) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!signal || !kernel || !out || rows > INT32_MAX) return DDSP_HIP_EINVAL;
  if (n <= kDirectMaxN) return direct_convolve(signal, kernel, out, rows, kernel_rows, n, stream);
  const int64_t nfft = good_fft_size(2 * n - 1);
  return fft_conv_rows(signal, n, nullptr, kernel, n, n, kernel_rows, out, rows, n, nfft, workspace,
                       workspace_bytes, stream);
}

const char* ddsp_hip_status_string(int status) {
  switch (status) {
    case DDSP_HIP_OK: return "ok";
    case DDSP_HIP_EINVAL: return "invalid argument or shape";
    case DDSP_HIP_ELAUNCH: return "HIP launch/runtime error";
    case DDSP_HIP_EFFT: return "rocFFT error";
    case DDSP_HIP_EWORKSPACE: return "workspace missing or too small";
    case DDSP_HIP_ERANGE: return "input outside the supported range";
    default: return "unknown status";
  }
}

int ddsp_hip_version(void) { return 100; }

}  // extern "C"
