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
#include "noise_dsp.h"


namespace ddsp {
namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

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
// Fused FilteredNoise.forward: one wave (64 lanes) per frame, 4 frames per workgroup.
// Per frame: magnitudes -> even half of the irfft taps (lane m: tap m; tap n/2 by a wave
// reduction, since cos(pi k) = (-1)^k) -> rolled/windowed filter h[bs] in LDS -> noise
// (Philox or injected) in LDS -> truncated causal convolution:
//   * taps [0, n/2): 8 consecutive outputs per lane, a 12-float sliding window in registers,
//     one float4 LDS read of noise and one of taps per 4 taps (32 FMAs);
//   * taps (bs-n/2, bs) reach only the last n/2 outputs: lane l sums output bs-n/2+l
//     directly into an LDS tail buffer, added when the outputs are written.
// ---------------------------------------------------------------------------------
constexpr int kNoiseFramesPerWG = 4;

// RAW: `mags` are the raw noise projection (decoder.py:115), scaled here as
// FilteredNoise.get_controls does (modules.py:111-114: scale_function(mags + bias)).
template <bool RNG, bool RAW>
__global__ void __launch_bounds__(256) filtered_noise_kernel(
    const float* __restrict__ mags, const float* __restrict__ noise, uint32_t k0, uint32_t k1,
    uint32_t off0, uint32_t off1, const float* __restrict__ add, float* __restrict__ out,
    float* __restrict__ noise_out, int64_t frames, int NB, int bs, int lo_end, int tail_start,
    int pad, int per_frame, float bias) {
  extern __shared__ float4 smem4[];
  const int n = 2 * (NB - 1);
  const int half = n >> 1;
  const int n4 = (n + 3) & ~3;
  const int bs8 = (bs + 7) & ~7;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* ct = reinterpret_cast<float*>(smem4);       // [n4] shared cos table
  float* base = ct + n4 + wv * per_frame;            // this wave's frame region
  float* A = base;                                   // [NB -> 4]
  float* ir = A + ((NB + 3) & ~3);                   // [n4]
  float* h = ir + n4;                                // [bs8]
  float* tail = h + bs8;                             // [half -> 4]
  float* xbuf = tail + ((half + 3) & ~3);            // [pad zeros | bs8 samples]
  float* x = xbuf + pad;

  const int64_t frame = (int64_t)blockIdx.x * kNoiseFramesPerWG + wv;
  const bool active = frame < frames;

  fill_cos_table(ct, n);
  if (active) {
    for (int k = lane; k < NB; k += 64) {
      const float m = mags[frame * NB + k];
      A[k] = RAW ? scale_fn(m + bias) : m;
    }
    for (int i = lane; i < pad; i += 64) xbuf[i] = 0.0f;
    const int quads = bs8 >> 2;
    const int fquads = ((bs + 3) & ~3) >> 2;  // counter stride per frame (as bs4/4)
    for (int t = lane; t < quads; t += 64) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int j = 4 * t;
      if (RNG) {
        if (t < fquads) {
          const uint64_t q = (uint64_t)frame * (uint64_t)fquads + (uint64_t)t;
          const Philox4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
          v = make_float4(uniform_pm1(r.v[0]), uniform_pm1(r.v[1]), uniform_pm1(r.v[2]),
                          uniform_pm1(r.v[3]));
        }
        if (j >= bs) v.x = 0.f;
        if (j + 1 >= bs) v.y = 0.f;
        if (j + 2 >= bs) v.z = 0.f;
        if (j + 3 >= bs) v.w = 0.f;
      } else {
        const float* src = noise + frame * bs;
        if ((bs & 3) == 0) {
          if (j < bs) v = *reinterpret_cast<const float4*>(src + j);
        } else {
          v.x = j < bs ? src[j] : 0.f;
          v.y = j + 1 < bs ? src[j + 1] : 0.f;
          v.z = j + 2 < bs ? src[j + 2] : 0.f;
          v.w = j + 3 < bs ? src[j + 3] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(x + j) = v;
    }
  }
  __syncthreads();
  if (active) {
    // even half of the taps; tap n/2 = (A0 + (-1)^{n/2} A_{n/2} + 2 sum_k (-1)^k A_k) / n
    if (n == 128) {
      // 65 bands -> 128 taps (the reference's default window_size): read the irfft matrix
      // from a code-object table, coalesced across lanes (no LDS gather, no bank conflicts)
      const int m = lane;
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 8
      for (int k = 1; k < 63; k += 2) {
        s0 = fmaf(A[k], kIrCos128[k * 64 + m], s0);
        s1 = fmaf(A[k + 1], kIrCos128[(k + 1) * 64 + m], s1);
      }
      s0 = fmaf(A[63], kIrCos128[63 * 64 + m], s0);
      ir[m] = (A[0] + ((m & 1) ? -A[64] : A[64]) + 2.0f * (s0 + s1)) * (1.0f / 128.0f);
    } else {
      for (int m = lane; m < half; m += 64) ir[m] = irfft_tap(A, ct, n, m);
    }
    float alt = 0.0f;
    for (int k = 1 + lane; k < half; k += 64) alt += (k & 1) ? -A[k] : A[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) alt += __shfl_xor(alt, o, 64);
    if (lane == 0) ir[half] = (A[0] + ((half & 1) ? -A[half] : A[half]) + 2.0f * alt) / (float)n;
  }
  __syncthreads();
  if (active) {
    for (int m = lane + 1; m < half; m += 64) ir[n - m] = ir[m];
    for (int j = lane; j < bs8; j += 64) h[j] = j < bs ? ir_at(ir, ct, n, bs, j) : 0.0f;
  }
  __syncthreads();
  if (active && tail_start < bs) {
    // outputs j >= tail_start: sum_{m=tail_start}^{j} h[m] x[j-m]
    for (int l = lane; l < bs - tail_start; l += 64) {
      const int j = tail_start + l;
      float c = 0.0f;
      for (int d = 0; d <= l; ++d) c = fmaf(h[j - d], x[d], c);
      tail[l] = c;
    }
  }
  __syncthreads();
  if (!active) return;
  float* ob = out + frame * bs;
  const float* ab = add ? add + frame * bs : nullptr;
  float* nb = noise_out ? noise_out + frame * bs : nullptr;
  for (int j0 = 8 * lane; j0 < bs8; j0 += 512) {
    float y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) y[r] = 0.0f;
    // window X[o + 4] = x[j0 - m + o], o in [-4, 8)
    float X[12];
    {
      const float4 b0 = *reinterpret_cast<const float4*>(x + j0);
      const float4 b1 = *reinterpret_cast<const float4*>(x + j0 + 4);
      X[4] = b0.x; X[5] = b0.y; X[6] = b0.z; X[7] = b0.w;
      X[8] = b1.x; X[9] = b1.y; X[10] = b1.z; X[11] = b1.w;
    }
    for (int m = 0; m < lo_end; m += 4) {
      const float4 bm = *reinterpret_cast<const float4*>(x + j0 - m - 4);
      X[0] = bm.x; X[1] = bm.y; X[2] = bm.z; X[3] = bm.w;
      const float4 hh = *reinterpret_cast<const float4*>(h + m);
      const float hd[4] = {hh.x, hh.y, hh.z, hh.w};
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int r = 0; r < 8; ++r) y[r] = fmaf(hd[d], X[r - d + 4], y[r]);
#pragma unroll
      for (int i = 11; i >= 4; --i) X[i] = X[i - 4];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int j = j0 + r;
      if (j >= tail_start && j < bs) y[r] += tail[j - tail_start];
    }
    if (nb) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (j0 + r < bs) nb[j0 + r] = y[r];
    }
    if (ab) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (j0 + r < bs) y[r] += ab[j0 + r];
    }
    if ((bs & 7) == 0) {
      *reinterpret_cast<float4*>(ob + j0) = make_float4(y[0], y[1], y[2], y[3]);
      *reinterpret_cast<float4*>(ob + j0 + 4) = make_float4(y[4], y[5], y[6], y[7]);
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (j0 + r < bs) ob[j0 + r] = y[r];
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

static int filtered_noise_launch(const float* magnitudes, bool raw, float bias, const float* noise,
                                 uint64_t seed, uint64_t offset, const float* add, float* out,
                                 float* noise_out, int64_t batch, int64_t frames, int64_t n_bands,
                                 int64_t block_size, void* stream) {
  if (batch < 0 || frames < 0 || n_bands < 2 || block_size < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!magnitudes || !out || n_bands > 4097 || block_size > (1 << 16)) return DDSP_HIP_EINVAL;
  const int n = 2 * (int)(n_bands - 1), half = n / 2, bs = (int)block_size;
  const int n4 = (n + 3) & ~3, bs8 = (bs + 7) & ~7;
  // taps [0, lo_end) by the windowed loop; (bs - n/2, bs) by the tail loop when the filter
  // is shorter than the block (the usual case), else every tap by the windowed loop
  int lo_end, tail_start;
  if (bs >= n) {
    lo_end = (half + 3) & ~3;
    tail_start = bs - half;
    if (tail_start < lo_end) {  // supports overlap: run every tap in the windowed loop
      lo_end = bs8;
      tail_start = bs;
    }
  } else {
    lo_end = bs8;
    tail_start = bs;
  }
  const int pad = ((lo_end + 4 + 7) & ~7);
  const int per_frame = ((int)(n_bands + 3) & ~3) + n4 + bs8 + ((half + 3) & ~3) + pad + bs8;
  const size_t shm = sizeof(float) * ((size_t)n4 + (size_t)kNoiseFramesPerWG * per_frame);
  if (shm > 160 * 1024) return DDSP_HIP_EINVAL;
  const int64_t total = batch * frames;
  const int64_t blocks = (total + kNoiseFramesPerWG - 1) / kNoiseFramesPerWG;
  if (blocks > INT32_MAX) return DDSP_HIP_EINVAL;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
#define DDSP_NOISE_LAUNCH(RNG_, RAW_)                                                          \
  hipLaunchKernelGGL((filtered_noise_kernel<RNG_, RAW_>), dim3((unsigned)blocks), dim3(256), shm, \
                     S(stream), magnitudes, noise, k0, k1, o0, o1, add, out, noise_out, total,  \
                     (int)n_bands, bs, lo_end, tail_start, pad, per_frame, bias)
  if (noise) {
    if (raw) DDSP_NOISE_LAUNCH(false, true); else DDSP_NOISE_LAUNCH(false, false);
  } else {
    if (raw) DDSP_NOISE_LAUNCH(true, true); else DDSP_NOISE_LAUNCH(true, false);
  }
#undef DDSP_NOISE_LAUNCH
  return launch_status();
}

int ddsp_hip_filtered_noise(const float* magnitudes, const float* noise, uint64_t seed,
                            uint64_t offset, const float* add, float* out, float* noise_out,
                            int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                            void* stream) {
  return filtered_noise_launch(magnitudes, false, 0.0f, noise, seed, offset, add, out, noise_out,
                               batch, frames, n_bands, block_size, stream);
}

int ddsp_hip_filtered_noise_params(const float* raw_magnitudes, float bias, const float* noise,
                                   uint64_t seed, uint64_t offset, const float* add, float* out,
                                   float* noise_out, int64_t batch, int64_t frames, int64_t n_bands,
                                   int64_t block_size, void* stream) {
  return filtered_noise_launch(raw_magnitudes, true, bias, noise, seed, offset, add, out, noise_out,
                               batch, frames, n_bands, block_size, stream);
}

}  // extern "C"
