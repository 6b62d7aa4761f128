// Filtered-noise path for gfx950.
//
//   ddsp/core.py:144-166   amp_to_impulse_response   (zero-phase FIR design)
//   ddsp/core.py:169-176   fft_convolve              (causal linear convolution truncated to N)
//   ddsp/models/modules.py:116-128  FilteredNoise.forward (fused)
//
// The reference convolves each block_size-sample frame of U[-1,1) noise with that frame's
// own FIR by a 2*block_size FFT and keeps the first block_size outputs (no overlap-add:
// the tail is dropped).  The FIR is a 2(NB-1)-tap zero-phase filter rolled to the ends of
// the block, so it has 2(NB-1)-1 non-zero taps: [0, n/2) and (bs-n/2, bs).  On gfx950 the
// frame is one workgroup: design the taps from the magnitudes in LDS, stage the noise in
// LDS (or draw it with Philox in registers), and run the truncated convolution directly —
// 4 outputs x 4 taps per step from two float4 LDS reads.  This is exactly the reference's
// linear convolution without the FFT's rounding, so results agree to fp32 rounding.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "twiddle4096.inc"

namespace ddsp {
namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// cos(2*pi*q/n) table, q in [0, n): fp64-evaluated, rounded once — read from the FFT
// twiddle table (same values) when n divides 4096, else computed in fp64.
__device__ __forceinline__ void fill_cos_table(float* ct, int n) {
  if (4096 % n == 0) {
    const int stride = 4096 / n;
    for (int q = threadIdx.x; q < n; q += blockDim.x) ct[q] = kTwiddle4096[2 * q * stride];
  } else {
    for (int q = threadIdx.x; q < n; q += blockDim.x) ct[q] = (float)cospi(2.0 * (double)q / (double)n);
  }
}

// irfft of NB real magnitudes (imaginary parts zero) at tap m: n = 2(NB-1),
// (1/n)(A0 + (-1)^m A_{n/2} + 2 sum_{k=1}^{n/2-1} A_k cos(2 pi k m / n)).
// The result is even in m (ir[n-m] == ir[m]), so callers evaluate m <= n/2 only.
__device__ __forceinline__ float irfft_tap(const float* A, const float* ct, int n, int m) {
  const int half = n >> 1;
  const float a0 = A[0] + ((m & 1) ? -A[half] : A[half]);
  float s0 = 0.0f, s1 = 0.0f;
  if ((n & (n - 1)) == 0) {  // power-of-two n: (k*m) mod n by mask, loads independent
    const int mask = n - 1;
    int k = 1;
    for (; k + 1 < half; k += 2) {
      s0 = fmaf(A[k], ct[(k * m) & mask], s0);
      s1 = fmaf(A[k + 1], ct[((k + 1) * m) & mask], s1);
    }
    for (; k < half; ++k) s0 = fmaf(A[k], ct[(k * m) & mask], s0);
  } else {
    int km = m % n;
    const int step = km;
    for (int k = 1; k < half; ++k) {
      s0 = fmaf(A[k], ct[km], s0);
      km += step;
      if (km >= n) km -= n;
    }
  }
  return (a0 + 2.0f * (s0 + s1)) / (float)n;
}

// ir[0..n) from its even half.
__device__ __forceinline__ void irfft_taps(const float* A, const float* ct, int n, float* ir) {
  const int half = n >> 1;
  for (int m = threadIdx.x; m <= half; m += blockDim.x) {
    const float v = irfft_tap(A, ct, n, m);
    ir[m] = v;
    if (m > 0 && m < half) ir[n - m] = v;
  }
}

// Final filter value at position j of a target-length block (core.py:158-164):
// imp1w[q] = ir[(q - n/2) mod n] * hann_n[q], padded/cropped to target, rolled by -n/2.
__device__ __forceinline__ float ir_at(const float* ir, const float* ct, int n, int target, int j) {
  const int half = n >> 1;
  int q = j + half;  // (j + half) mod target, j < target
  if (q >= target) q = half < target ? q - target : q % target;
  if (q >= n) return 0.0f;
  const float hann = 0.5f - 0.5f * ct[q];  // torch.hann_window(n), periodic
  int src = q - half;
  if (src < 0) src += n;
  return ir[src] * hann;
}

// Truncated causal convolution y[j] = sum_{m<=j} h[m] x[j-m] for j in [j0, j0+4).
// x points at a buffer with >= len4 zeros to the left of x[0]; h is zero outside its support.
// Taps are visited in [0, lo_end) and [hi_start, len4), both multiples of 4.
__device__ __forceinline__ float4 fir4(const float* __restrict__ h, const float* __restrict__ x,
                                      int j0, int lo_end, int hi_start, int len4) {
  float y0 = 0.f, y1 = 0.f, y2 = 0.f, y3 = 0.f;
  auto run = [&](int m_begin, int m_end) {
    float4 cur = *reinterpret_cast<const float4*>(x + j0 - m_begin);  // x[j0-m .. j0-m+3]
    for (int m = m_begin; m < m_end; m += 4) {
      const float4 prv = *reinterpret_cast<const float4*>(x + j0 - m - 4);  // x[j0-m-4 .. j0-m-1]
      const float4 hh = *reinterpret_cast<const float4*>(h + m);
      // tap m+d contributes h[m+d] * x[j0+r-m-d]
      y0 = fmaf(hh.x, cur.x, y0); y1 = fmaf(hh.x, cur.y, y1); y2 = fmaf(hh.x, cur.z, y2); y3 = fmaf(hh.x, cur.w, y3);
      y0 = fmaf(hh.y, prv.w, y0); y1 = fmaf(hh.y, cur.x, y1); y2 = fmaf(hh.y, cur.y, y2); y3 = fmaf(hh.y, cur.z, y3);
      y0 = fmaf(hh.z, prv.z, y0); y1 = fmaf(hh.z, prv.w, y1); y2 = fmaf(hh.z, cur.x, y2); y3 = fmaf(hh.z, cur.y, y3);
      y0 = fmaf(hh.w, prv.y, y0); y1 = fmaf(hh.w, prv.z, y1); y2 = fmaf(hh.w, prv.w, y2); y3 = fmaf(hh.w, cur.x, y3);
      cur = prv;
    }
  };
  run(0, lo_end);
  if (j0 + 3 >= hi_start && hi_start < len4) run(hi_start, len4);
  return make_float4(y0, y1, y2, y3);
}

// ---------------------------------------------------------------------------------
// amp_to_impulse_response(amp[rows, NB], target) -> [rows, target]   (core.py:144-166)
// ---------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) impulse_response_kernel(const float* __restrict__ amp,
                                                               float* __restrict__ out, int NB,
                                                               int target) {
  extern __shared__ float sm[];
  const int n = 2 * (NB - 1);
  float* ct = sm;
  float* ir = ct + n;
  float* A = ir + n;
  const int64_t row = blockIdx.x;
  fill_cos_table(ct, n);
  for (int k = threadIdx.x; k < NB; k += blockDim.x) A[k] = amp[row * NB + k];
  __syncthreads();
  irfft_taps(A, ct, n, ir);
  __syncthreads();
  for (int j = threadIdx.x; j < target; j += blockDim.x)
    out[row * target + j] = ir_at(ir, ct, n, target, j);
}

// ---------------------------------------------------------------------------------
// Fused FilteredNoise.forward: grid (frames, batch), block NT, 4 outputs per thread.
// ---------------------------------------------------------------------------------
template <bool RNG>
__global__ void __launch_bounds__(256) filtered_noise_kernel(
    const float* __restrict__ mags, const float* __restrict__ noise, uint32_t k0, uint32_t k1,
    uint32_t off0, uint32_t off1, const float* __restrict__ add, float* __restrict__ out,
    float* __restrict__ noise_out, int F, int NB, int bs) {
  extern __shared__ float4 smem4[];
  const int n = 2 * (NB - 1);
  const int bs4 = (bs + 3) & ~3;
  const int n4 = (n + 3) & ~3;
  float* h = reinterpret_cast<float*>(smem4);  // [bs4]
  float* xbuf = h + bs4;                        // [bs4 zeros | bs4 samples]
  float* x = xbuf + bs4;
  float* ct = x + bs4;                          // [n4]
  float* ir = ct + n4;                          // [n4]
  float* A = ir + n4;                           // [NB]

  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, NT = blockDim.x;
  const int64_t frame = (int64_t)b * F + f;

  fill_cos_table(ct, n);
  for (int k = tid; k < NB; k += NT) A[k] = mags[frame * NB + k];
  for (int i = tid; i < bs4; i += NT) xbuf[i] = 0.0f;
  const int quads = bs4 >> 2;
  for (int t = tid; t < quads; t += NT) {
    float4 v;
    if (RNG) {
      const uint64_t q = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(r.v[0]), uniform_pm1(r.v[1]), uniform_pm1(r.v[2]), uniform_pm1(r.v[3]));
    } else {
      const float* src = noise + frame * bs + 4 * t;
      if ((bs & 3) == 0) {
        v = *reinterpret_cast<const float4*>(src);
      } else {
        const int j = 4 * t;
        v.x = j < bs ? src[0] : 0.f;
        v.y = j + 1 < bs ? src[1] : 0.f;
        v.z = j + 2 < bs ? src[2] : 0.f;
        v.w = j + 3 < bs ? src[3] : 0.f;
      }
    }
    if (RNG && (bs & 3)) {  // zero the lanes past the frame end
      const int j = 4 * t;
      if (j + 1 >= bs) v.y = 0.f;
      if (j + 2 >= bs) v.z = 0.f;
      if (j + 3 >= bs) v.w = 0.f;
    }
    *reinterpret_cast<float4*>(x + 4 * t) = v;
  }
  __syncthreads();
  irfft_taps(A, ct, n, ir);
  __syncthreads();
  for (int j = tid; j < bs4; j += NT) h[j] = j < bs ? ir_at(ir, ct, n, bs, j) : 0.0f;
  __syncthreads();

  int lo_end = bs4, hi_start = bs4;
  if (bs >= n) {
    lo_end = std::min(((n >> 1) + 3) & ~3, bs4);
    hi_start = std::max(((bs - (n >> 1)) & ~3), lo_end);
  }
  float* ob = out + frame * bs;
  for (int t = tid; t < quads; t += NT) {
    const int j0 = 4 * t;
    float4 y = fir4(h, x, j0, lo_end, hi_start, bs4);
    if (noise_out) {
      float* nb = noise_out + frame * bs;
      if ((bs & 3) == 0) {
        *reinterpret_cast<float4*>(nb + j0) = y;
      } else {
        const float yy[4] = {y.x, y.y, y.z, y.w};
        for (int r = 0; r < 4; ++r) if (j0 + r < bs) nb[j0 + r] = yy[r];
      }
    }
    if (add) {
      const float* ab = add + frame * bs;
      if ((bs & 3) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(ab + j0);
        y.x += a.x; y.y += a.y; y.z += a.z; y.w += a.w;
      } else {
        y.x += ab[j0];
        if (j0 + 1 < bs) y.y += ab[j0 + 1];
        if (j0 + 2 < bs) y.z += ab[j0 + 2];
        if (j0 + 3 < bs) y.w += ab[j0 + 3];
      }
    }
    if ((bs & 3) == 0) {
      *reinterpret_cast<float4*>(ob + j0) = y;
    } else {
      const float yy[4] = {y.x, y.y, y.z, y.w};
      for (int r = 0; r < 4; ++r) if (j0 + r < bs) ob[j0 + r] = yy[r];
    }
  }
}

// Direct truncated convolution of whole rows (function-level fft_convolve, small N).
__global__ void __launch_bounds__(256) direct_convolve_kernel(const float* __restrict__ sig,
                                                              const float* __restrict__ ker,
                                                              float* __restrict__ out, int N,
                                                              int kernel_rows) {
  extern __shared__ float4 smem4[];
  const int N4 = (N + 3) & ~3;
  float* h = reinterpret_cast<float*>(smem4);
  float* xbuf = h + N4;
  float* x = xbuf + N4;
  const int64_t row = blockIdx.x;
  const int64_t krow = kernel_rows == 1 ? 0 : row;
  for (int i = threadIdx.x; i < N4; i += blockDim.x) {
    xbuf[i] = 0.0f;
    x[i] = i < N ? sig[row * N + i] : 0.0f;
    h[i] = i < N ? ker[krow * N + i] : 0.0f;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < (N4 >> 2); t += blockDim.x) {
    const int j0 = 4 * t;
    const float4 y = fir4(h, x, j0, N4, N4, N4);
    const float yy[4] = {y.x, y.y, y.z, y.w};
    for (int r = 0; r < 4; ++r)
      if (j0 + r < N) out[row * N + j0 + r] = yy[r];
  }
}

}  // namespace

// used by reverb.hip for the small-N branch of fft_convolve
int direct_convolve(const float* sig, const float* ker, float* out, int64_t rows,
                    int64_t kernel_rows, int64_t n, void* stream) {
  const int N4 = (int)((n + 3) & ~3);
  const int nt = (int)std::min<int64_t>(256, std::max<int64_t>(64, ((N4 / 4 + 63) / 64) * 64));
  const size_t shm = sizeof(float) * 3 * (size_t)N4;
  hipLaunchKernelGGL(direct_convolve_kernel, dim3((unsigned)rows), dim3(nt), shm, S(stream), sig, ker,
                     out, (int)n, (int)kernel_rows);
  return launch_status();
}

}  // namespace ddsp

using namespace ddsp;

extern "C" {

int ddsp_hip_amp_to_impulse_response(const float* amp, float* impulse, int64_t rows,
                                     int64_t n_bands, int64_t target_size, void* stream) {
  if (rows < 0 || n_bands < 2 || n_bands > 8193 || target_size < 1 || target_size > (1 << 24))
    return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!amp || !impulse || rows > INT32_MAX) return DDSP_HIP_EINVAL;
  const int n = 2 * (int)(n_bands - 1);
  const size_t shm = sizeof(float) * (2 * (size_t)n + (size_t)n_bands);
  hipLaunchKernelGGL(impulse_response_kernel, dim3((unsigned)rows), dim3(256), shm, S(stream), amp,
                     impulse, (int)n_bands, (int)target_size);
  return launch_status();
}

int ddsp_hip_filtered_noise(const float* magnitudes, const float* noise, uint64_t seed,
                            uint64_t offset, const float* add, float* out, float* noise_out,
                            int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                            void* stream) {
  if (batch < 0 || frames < 0 || n_bands < 2 || block_size < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!magnitudes || !out || batch > 65535 || frames > INT32_MAX) return DDSP_HIP_EINVAL;
  const int64_t n = 2 * (n_bands - 1);
  const int64_t bs4 = (block_size + 3) & ~3, n4 = (n + 3) & ~3, nb4 = (n_bands + 3) & ~3;
  const size_t shm = sizeof(float) * (size_t)(3 * bs4 + 2 * n4 + nb4);
  if (shm > 160 * 1024) return DDSP_HIP_EINVAL;
  const int nt = (int)std::min<int64_t>(256, std::max<int64_t>(64, ((bs4 / 4 + 63) / 64) * 64));
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
  if (noise)
    hipLaunchKernelGGL(filtered_noise_kernel<false>, dim3((unsigned)frames, (unsigned)batch), dim3(nt),
                       shm, S(stream), magnitudes, noise, k0, k1, o0, o1, add, out, noise_out,
                       (int)frames, (int)n_bands, (int)block_size);
  else
    hipLaunchKernelGGL(filtered_noise_kernel<true>, dim3((unsigned)frames, (unsigned)batch), dim3(nt),
                       shm, S(stream), magnitudes, nullptr, k0, k1, o0, o1, add, out, noise_out,
                       (int)frames, (int)n_bands, (int)block_size);
  return launch_status();
}

}  // extern "C"
