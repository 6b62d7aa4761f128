// Harmonic (additive oscillator bank) path for gfx950.
//
//   ddsp/core.py:64-78, 136-141        scale_function, remove_above_nyquist, upsample,
//                                      harmonic_synth (op boundary, per-sample inputs)
//   ddsp/models/modules.py:44-80       HarmonicSynth.get_controls / forward (fused)
//
// The fused frame-rate kernel is the hot one: one workgroup per (batch item, frame),
// the frame's H amplitudes staged once in LDS, the phase of every sample obtained in
// closed form from an exact fp64 prefix over earlier frames, and H sines per sample
// evaluated in registers.  Only the waveform is written to HBM.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace ddsp {
namespace {


__global__ void scale_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                             float bias) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) y[i] = scale_fn(x[i] + bias);
}

__global__ void nyquist_kernel(const float* __restrict__ amps, const float* __restrict__ f0,
                               float* __restrict__ out, int64_t rows, int H, float half_sr) {
  const int64_t n = rows * H;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const int64_t r = i / H;
    const int k = (int)(i - r * H) + 1;
    const float pitch = f0[r] * (float)k;  // fl32(f0 * k), ddsp/core.py:72
    out[i] = amps[i] * (pitch < half_sr ? kOnePlusEps : kEps);
  }
}

__global__ void upsample_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t batch,
                                int64_t frames, int64_t channels, int64_t factor) {
  // nearest interpolation to F*factor samples == repeat each frame `factor` times
  const int64_t n = batch * frames * factor * channels;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    const int64_t c = i % channels;
    const int64_t t = (i / channels) % (frames * factor);
    const int64_t b = i / (channels * frames * factor);
    y[i] = x[(b * frames + t / factor) * channels + c];
  }
}

// HarmonicSynth.get_controls (modules.py:44-67): one wave per frame row, the row's values
// held in registers (H <= 64*kCtlPer) between the sum and the normalisation.
constexpr int kCtlPer = 4;
__global__ void __launch_bounds__(256) harmonic_controls_kernel(
    const float* __restrict__ amp_raw, int64_t amp_stride, const float* __restrict__ dist_raw,
    int64_t dist_stride, const float* __restrict__ f0, float* __restrict__ amplitudes,
    float* __restrict__ dist, int64_t rows, int H, float half_sr) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float pitch0 = f0[r];
  const float* drow = dist_raw + r * dist_stride;
  float* orow = dist + r * (int64_t)H;
  float d[kCtlPer];
  double sum = 0.0;
#pragma unroll
  for (int i = 0; i < kCtlPer; ++i) {
    const int k = lane + 64 * i;
    d[i] = k < H ? controls_value(drow[k], pitch0, k, half_sr) : 0.0f;
    sum += (double)d[i];
  }
  for (int k = lane + 64 * kCtlPer; k < H; k += 64) {  // H > 256: spill to the output row
    const float v = controls_value(drow[k], pitch0, k, half_sr);
    orow[k] = v;
    sum += (double)v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  const float s = (float)sum;
#pragma unroll
  for (int i = 0; i < kCtlPer; ++i) {
    const int k = lane + 64 * i;
    if (k < H) orow[k] = d[i] / s;  // dist /= dist.sum(-1)
  }
  for (int k = lane + 64 * kCtlPer; k < H; k += 64) orow[k] = orow[k] / s;
  if (lane == 0) amplitudes[r] = scale_fn(amp_raw[r * amp_stride]);
}

// ---------------------------------------------------------------------------------
// Fused HarmonicSynth.forward (modules.py:69-80) at frame rate.
// grid (frames, batch); block NT threads; each thread SPT samples of the frame per pass.
// ---------------------------------------------------------------------------------
// RAW = true: `dist` is the raw parameter row [B,F,H+1] (decoder.py:106-108 split), and the
// controls of modules.py:44-67 (scale, Nyquist mask, normalise, times the scaled amplitude) are
// computed in the prologue — HarmonicSynth.get_controls + forward in one launch.
template <int SPT, bool RAW>
__global__ void __launch_bounds__(256) harmonic_frames_kernel(
    const float* __restrict__ f0, const float* __restrict__ amp, float* dist, int write_back,
    float* __restrict__ out, int F, int H, int bs, float sr) {
  // per harmonic k: coef[k] = (k+1, A), A = dist*amp; H rounded up to 4 with zero amplitudes.
  // Read back as wave-uniform (broadcast) LDS loads.
  extern __shared__ float2 coef[];
  __shared__ double red[16];

  const int f = blockIdx.x;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int NT = blockDim.x;
  const float* f0b = f0 + (int64_t)b * F;

  // exact fp64 prefix of the phase over earlier frames: S_f = sum_{g<f} bs * inc_g
  double part = 0.0;
  for (int g = tid; g < f; g += NT) part += (double)bs * (double)phase_inc(f0b[g], sr);
  const double S = block_sum_double(part, red);

  // stage this frame's harmonic amplitudes dist[k] * amp (modules.py:73, in place if asked)
  const int64_t row = (int64_t)b * F + f;
  const int H4 = (H + 3) & ~3;
  float a, norm = 1.0f;
  if (RAW) {
    const float* prow = dist + row * (H + 1);
    const float half_sr = sr * 0.5f;
    const float pitch0 = f0b[f];
    double part2 = 0.0;
    for (int k = tid; k < H; k += NT) {
      const float v = controls_value(prow[1 + k], pitch0, k, half_sr);
      coef[k].y = v;
      part2 += (double)v;
    }
    norm = (float)block_sum_double(part2, red);  // dist.sum(-1)
    a = scale_fn(prow[0]);
  } else {
    a = amp[row];
  }
  for (int k = tid; k < H4; k += NT) {
    float v = 0.0f;
    if (k < H) {
      if (RAW) {
        v = (coef[k].y / norm) * a;  // (dist / sum) * amp, the reference's rounding order
      } else {
        v = dist[row * H + k] * a;
        if (write_back) dist[row * H + k] = v;
      }
    }
    coef[k] = make_float2((float)(k + 1), v);
  }
  __syncthreads();

  const float inc = phase_inc(f0b[f], sr);
  const double dinc = (double)inc;
  float* ob = out + (int64_t)b * F * bs + (int64_t)f * bs;

  for (int base = 0; base < bs; base += NT * SPT) {
    float w[SPT], acc[SPT];
    bool fast = true;
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int i = base + tid + s * NT;
      w[s] = (float)(S + (double)(i + 1) * dinc);  // omega[t] = fl32(exact prefix)
      acc[s] = 0.0f;
      fast = fast && (fabsf(w[s]) * (float)H4 < kFastArgLimit);
    }
    if (fast) {
#pragma unroll 4
      for (int k = 0; k < H4; ++k) {
        const float2 c = coef[k];
#pragma unroll
        for (int s = 0; s < SPT; ++s) acc[s] = fmaf(sin_reduced(w[s] * c.x), c.y, acc[s]);
      }
    } else {
      for (int k = 0; k < H; ++k) {
        const float2 c = coef[k];
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
          const float x = w[s] * c.x;
          acc[s] = fmaf(fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x), c.y, acc[s]);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int i = base + tid + s * NT;
      if (i < bs) ob[i] = acc[s];
    }
  }
}

// ---------------------------------------------------------------------------------
// Op-boundary harmonic_synth(f0[B,T,1], amplitudes[B,T,H]) (core.py:136-141).
// Two launches: (1) exact fp64 sums of the phase increment per chunk of CHUNK samples,
// (2) per chunk: prefix of earlier chunk sums + in-chunk scan -> fp32 phase, then the
// oscillator bank with each thread owning SPT consecutive samples.
// ---------------------------------------------------------------------------------
constexpr int kScanNT = 256;
constexpr int kScanSPT = 4;
constexpr int kChunk = kScanNT * kScanSPT;  // 1024 samples per workgroup

__global__ void __launch_bounds__(kScanNT) phase_chunk_sums_kernel(const float* __restrict__ f0,
                                                                   double* __restrict__ sums,
                                                                   int64_t T, int nchunks,
                                                                   float sr) {
  __shared__ double red[16];
  const int c = blockIdx.x, b = blockIdx.y;
  const int64_t t0 = (int64_t)c * kChunk;
  const float* f0b = f0 + (int64_t)b * T;
  double part = 0.0;
  for (int i = threadIdx.x; i < kChunk; i += kScanNT) {
    const int64_t t = t0 + i;
    if (t < T) part += (double)phase_inc(f0b[t], sr);
  }
  const double s = block_sum_double(part, red);
  if (threadIdx.x == 0) sums[(int64_t)b * nchunks + c] = s;
}

// Returns the fp32 phase of this thread's kScanSPT consecutive samples.
__device__ __forceinline__ void chunk_phase(const float* __restrict__ f0b,
                                            const double* __restrict__ sums, int64_t T, int c,
                                            float sr, float (&w)[kScanSPT]) {
  __shared__ double red[16];
  __shared__ double wave_tot[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // prefix of the earlier chunks (exact; order free)
  double part = 0.0;
  for (int j = tid; j < c; j += kScanNT) part += sums[j];
  const double prefix = block_sum_double(part, red);

  const int64_t t0 = (int64_t)c * kChunk + (int64_t)tid * kScanSPT;
  double loc[kScanSPT];
  double run = 0.0;
#pragma unroll
  for (int s = 0; s < kScanSPT; ++s) {
    const int64_t t = t0 + s;
    run += (t < T) ? (double)phase_inc(f0b[t], sr) : 0.0;
    loc[s] = run;
  }
  // inclusive wave scan of the thread totals
  double incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wave_tot[wid] = incl;
  __syncthreads();
  double before = prefix;
  for (int i = 0; i < wid; ++i) before += wave_tot[i];
  before += incl - run;  // exclusive within the wave
#pragma unroll
  for (int s = 0; s < kScanSPT; ++s) w[s] = (float)(before + loc[s]);
}

__global__ void __launch_bounds__(kScanNT) phase_kernel(const float* __restrict__ f0,
                                                        const double* __restrict__ sums,
                                                        float* __restrict__ omega, int64_t T,
                                                        int nchunks, float sr) {
  const int c = blockIdx.x, b = blockIdx.y;
  float w[kScanSPT];
  chunk_phase(f0 + (int64_t)b * T, sums + (int64_t)b * nchunks, T, c, sr, w);
  const int64_t t0 = (int64_t)c * kChunk + (int64_t)threadIdx.x * kScanSPT;
#pragma unroll
  for (int s = 0; s < kScanSPT; ++s)
    if (t0 + s < T) omega[(int64_t)b * T + t0 + s] = w[s];
}

template <bool VEC4>
__global__ void __launch_bounds__(kScanNT) harmonic_samples_kernel(
    const float* __restrict__ f0, const float* __restrict__ amps, const double* __restrict__ sums,
    float* __restrict__ out, int64_t T, int nchunks, int H, float sr) {
  __shared__ float wsm[kChunk];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  {
    float w[kScanSPT];
    chunk_phase(f0 + (int64_t)b * T, sums + (int64_t)b * nchunks, T, c, sr, w);
#pragma unroll
    for (int s = 0; s < kScanSPT; ++s) wsm[tid * kScanSPT + s] = w[s];
  }
  __syncthreads();
  // synthesis: consecutive lanes own consecutive samples (coalesced output, and each
  // wave keeps only 64 amplitude rows in flight); 4 independent sines per step give ILP.
  for (int s = 0; s < kScanSPT; ++s) {
    const int i = tid + s * kScanNT;
    const int64_t t = (int64_t)c * kChunk + i;
    if (t >= T) break;
    const float w = wsm[i];
    const float* row = amps + ((int64_t)b * T + t) * H;
    float acc0 = 0.0f, acc1 = 0.0f;
    if (VEC4 && fabsf(w) * (float)H < kFastArgLimit) {
#pragma unroll 2
      for (int k = 0; k < H; k += 4) {
        const float4 A = *reinterpret_cast<const float4*>(row + k);
        acc0 = fmaf(sin_reduced(w * (float)(k + 1)), A.x, acc0);
        acc1 = fmaf(sin_reduced(w * (float)(k + 2)), A.y, acc1);
        acc0 = fmaf(sin_reduced(w * (float)(k + 3)), A.z, acc0);
        acc1 = fmaf(sin_reduced(w * (float)(k + 4)), A.w, acc1);
      }
    } else {
      for (int k = 0; k < H; ++k) {
        const float x = w * (float)(k + 1);
        const float sn = fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x);
        acc0 = fmaf(sn, row[k], acc0);
      }
    }
    out[(int64_t)b * T + t] = acc0 + acc1;
  }
}

// Tiled op-boundary kernel (H % 4 == 0, H <= 128): the [64 samples x H] amplitude tile of
// each stage is contiguous in HBM, so it is streamed with fully coalesced 16-byte loads into
// LDS (register-staged one stage ahead, overlapping the sines of the current stage), then
// 4 lanes share a sample, each summing every 4th harmonic.  LDS rows are padded to a stride
// == 4 (mod 8) floats so the 32 lanes of a half-wave (8 samples x 4 lanes) hit 32 banks.
constexpr int kStage = 64;      // samples per stage
constexpr int kTileMaxPF = 8;   // float4 per thread per stage: 64*H/4/256 = H/16 <= 8
__global__ void __launch_bounds__(kScanNT) harmonic_samples_tiled_kernel(
    const float* __restrict__ f0, const float* __restrict__ amps, const double* __restrict__ sums,
    float* __restrict__ out, int64_t T, int nchunks, int H, int Hs, float sr) {
  extern __shared__ float4 tile4[];
  float* tile = reinterpret_cast<float*>(tile4);  // [kStage][Hs]
  __shared__ float wsm[kChunk];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  {
    float w[kScanSPT];
    chunk_phase(f0 + (int64_t)b * T, sums + (int64_t)b * nchunks, T, c, sr, w);
#pragma unroll
    for (int s = 0; s < kScanSPT; ++s) wsm[tid * kScanSPT + s] = w[s];
  }
  const int64_t chunk_t0 = (int64_t)c * kChunk;
  const int valid = (int)min<int64_t>(kChunk, T - chunk_t0);
  const int nstage = (valid + kStage - 1) / kStage;
  const int H4 = H >> 2;
  const float invH4 = 1.0f / (float)H4;
  const float4* src = reinterpret_cast<const float4*>(amps + ((int64_t)b * T + chunk_t0) * H);

  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f pre[kTileMaxPF];
  auto prefetch = [&](int st) {
    const int rows = min(kStage, valid - st * kStage);
    const int n4 = rows * H4;
    const v4f* s4 = reinterpret_cast<const v4f*>(src) + (int64_t)st * kStage * H4;
#pragma unroll
    for (int i = 0; i < kTileMaxPF; ++i) {
      const int e = tid + i * kScanNT;
      if (e < n4) pre[i] = __builtin_nontemporal_load(s4 + e);
    }
  };
  auto commit = [&](int st) {
    const int rows = min(kStage, valid - st * kStage);
    const int n4 = rows * H4;
#pragma unroll
    for (int i = 0; i < kTileMaxPF; ++i) {
      const int e = tid + i * kScanNT;
      if (e < n4) {
        int row = (int)(((float)e + 0.5f) * invH4);
        const int col4 = e - row * H4;
        *reinterpret_cast<v4f*>(tile + row * Hs + 4 * col4) = pre[i];
      }
    }
  };

  const int sl = tid >> 2, q = tid & 3;
  if (nstage > 0) prefetch(0);
  for (int st = 0; st < nstage; ++st) {
    __syncthreads();  // previous stage's reads done (and wsm visible on the first pass)
    commit(st);
    __syncthreads();
    if (st + 1 < nstage) prefetch(st + 1);
    const int i = st * kStage + sl;
    const float w = wsm[i < kChunk ? i : 0];
    const float* arow = tile + sl * Hs;
    float acc0 = 0.0f, acc1 = 0.0f;
    if (fabsf(w) * (float)H < kFastArgLimit) {
      for (int k = q; k < H; k += 16) {
        // k, k+4, k+8, k+12 (H % 4 == 0 keeps k+4j < H whenever k < H - 12; guard the tail)
        acc0 = fmaf(sin_reduced(w * (float)(k + 1)), arow[k], acc0);
        if (k + 4 < H) acc1 = fmaf(sin_reduced(w * (float)(k + 5)), arow[k + 4], acc1);
        if (k + 8 < H) acc0 = fmaf(sin_reduced(w * (float)(k + 9)), arow[k + 8], acc0);
        if (k + 12 < H) acc1 = fmaf(sin_reduced(w * (float)(k + 13)), arow[k + 12], acc1);
      }
    } else {
      for (int k = q; k < H; k += 4) {
        const float x = w * (float)(k + 1);
        const float sn = fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x);
        acc0 = fmaf(sn, arow[k], acc0);
      }
    }
    float acc = acc0 + acc1;
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (q == 0 && i < valid) out[(int64_t)b * T + chunk_t0 + i] = acc;
  }
}

inline unsigned grid1d(int64_t n, int nt) {
  int64_t g = (n + nt - 1) / nt;
  return (unsigned)std::min<int64_t>(std::max<int64_t>(g, 1), 65536);
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// One workgroup per (frame, item).  4 samples per thread when the block is long enough
// (more independent sine chains per lane: measured 4% faster than 2 at block 512), else 2.
template <bool RAW>
void launch_frames(const float* f0, const float* amp, float* dist, int write_back, float* out,
                   int64_t batch, int64_t frames, int64_t H, int64_t bs, float sr, size_t shm,
                   void* stream) {
  const dim3 grid((unsigned)frames, (unsigned)batch);
  if (bs >= 256) {
    const int nt = (int)std::min<int64_t>(256, ((bs / 4 + 63) / 64) * 64);
    hipLaunchKernelGGL((harmonic_frames_kernel<4, RAW>), grid, dim3(nt), shm, S(stream), f0, amp, dist,
                       write_back, out, (int)frames, (int)H, (int)bs, sr);
  } else {
    const int nt = (int)std::max<int64_t>(64, ((bs / 2 + 63) / 64) * 64);
    hipLaunchKernelGGL((harmonic_frames_kernel<2, RAW>), grid, dim3(nt), shm, S(stream), f0, amp, dist,
                       write_back, out, (int)frames, (int)H, (int)bs, sr);
  }
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int ddsp_hip_scale_function(const float* x, float* y, int64_t n, float bias, void* stream) {
  if (n < 0 || (n > 0 && (!x || !y))) return DDSP_HIP_EINVAL;
  if (n == 0) return DDSP_HIP_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(grid1d(n, 256)), dim3(256), 0, S(stream), x, y, n, bias);
  return launch_status();
}

int ddsp_hip_remove_above_nyquist(const float* amplitudes, const float* f0, float* out,
                                  int64_t rows, int64_t n_harmonic, float sample_rate,
                                  void* stream) {
  if (rows < 0 || n_harmonic < 0 || n_harmonic > (1 << 24)) return DDSP_HIP_EINVAL;
  if (rows * n_harmonic == 0) return DDSP_HIP_OK;
  if (!amplitudes || !f0 || !out) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(nyquist_kernel, dim3(grid1d(rows * n_harmonic, 256)), dim3(256), 0, S(stream),
                     amplitudes, f0, out, rows, (int)n_harmonic, sample_rate * 0.5f);
  return launch_status();
}

int ddsp_hip_upsample(const float* x, float* y, int64_t batch, int64_t frames, int64_t channels,
                      int64_t factor, void* stream) {
  if (batch < 0 || frames < 0 || channels < 0 || factor < 1) return DDSP_HIP_EINVAL;
  const int64_t n = batch * frames * channels * factor;
  if (n == 0) return DDSP_HIP_OK;
  if (!x || !y) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(upsample_kernel, dim3(grid1d(n, 256)), dim3(256), 0, S(stream), x, y, batch,
                     frames, channels, factor);
  return launch_status();
}

int ddsp_hip_harmonic_controls(const float* amp_raw, int64_t amp_stride, const float* dist_raw,
                               int64_t dist_stride, const float* f0, float* amplitudes,
                               float* distribution, int64_t rows, int64_t n_harmonic,
                               float sample_rate, void* stream) {
  if (rows < 0 || n_harmonic < 1 || n_harmonic > (1 << 20)) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!amp_raw || !dist_raw || !f0 || !amplitudes || !distribution) return DDSP_HIP_EINVAL;
  const int64_t blocks = (rows + 3) / 4;
  if (blocks > INT32_MAX) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(harmonic_controls_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream),
                     amp_raw, amp_stride, dist_raw, dist_stride, f0, amplitudes, distribution, rows,
                     (int)n_harmonic, sample_rate * 0.5f);
  return launch_status();
}

int ddsp_hip_harmonic_synth_frames(const float* f0, const float* amplitudes, float* distribution,
                                   int write_back, float* out, int64_t batch, int64_t frames,
                                   int64_t n_harmonic, int64_t block_size, float sample_rate,
                                   void* stream) {
  if (batch < 0 || frames < 0 || n_harmonic < 1 || block_size < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!f0 || !amplitudes || !distribution || !out) return DDSP_HIP_EINVAL;
  if (frames > INT32_MAX || batch > 65535 || n_harmonic > 8192 || block_size > (1 << 20))
    return DDSP_HIP_EINVAL;
  const size_t shm = sizeof(float2) * (size_t)((n_harmonic + 3) & ~3);
  launch_frames<false>(f0, amplitudes, distribution, write_back, out, batch, frames, n_harmonic,
                       block_size, sample_rate, shm, stream);
  return launch_status();
}

int ddsp_hip_harmonic_synth_params(const float* f0, const float* param, float* out, int64_t batch,
                                   int64_t frames, int64_t n_harmonic, int64_t block_size,
                                   float sample_rate, void* stream) {
  if (batch < 0 || frames < 0 || n_harmonic < 1 || block_size < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!f0 || !param || !out) return DDSP_HIP_EINVAL;
  if (frames > INT32_MAX || batch > 65535 || n_harmonic > 8192 || block_size > (1 << 20))
    return DDSP_HIP_EINVAL;
  const size_t shm = sizeof(float2) * (size_t)((n_harmonic + 3) & ~3);
  launch_frames<true>(f0, nullptr, const_cast<float*>(param), 0, out, batch, frames, n_harmonic,
                      block_size, sample_rate, shm, stream);
  return launch_status();
}

size_t ddsp_hip_harmonic_synth_workspace_size(int64_t batch, int64_t n_samples) {
  const int64_t nchunks = (n_samples + kChunk - 1) / kChunk;
  return (size_t)std::max<int64_t>(batch * nchunks, 1) * sizeof(double);
}

static int phase_common(const float* f0, int64_t batch, int64_t T, float sr, void* ws,
                        size_t ws_bytes, void* stream, int* nchunks_out) {
  if (batch < 0 || T < 0 || batch > 65535) return DDSP_HIP_EINVAL;
  const int64_t nchunks = (T + kChunk - 1) / kChunk;
  if (nchunks > INT32_MAX) return DDSP_HIP_EINVAL;
  if (ws_bytes < ddsp_hip_harmonic_synth_workspace_size(batch, T) || !ws) return DDSP_HIP_EWORKSPACE;
  *nchunks_out = (int)nchunks;
  hipLaunchKernelGGL(phase_chunk_sums_kernel, dim3((unsigned)nchunks, (unsigned)batch),
                     dim3(kScanNT), 0, S(stream), f0, reinterpret_cast<double*>(ws), T,
                     (int)nchunks, sr);
  return launch_status();
}

int ddsp_hip_phase(const float* f0, float* omega, int64_t batch, int64_t n_samples,
                   float sample_rate, void* workspace, size_t workspace_bytes, void* stream) {
  if (batch * n_samples == 0) return batch < 0 || n_samples < 0 ? DDSP_HIP_EINVAL : DDSP_HIP_OK;
  if (!f0 || !omega) return DDSP_HIP_EINVAL;
  int nchunks = 0;
  int st = phase_common(f0, batch, n_samples, sample_rate, workspace, workspace_bytes, stream, &nchunks);
  if (st) return st;
  hipLaunchKernelGGL(phase_kernel, dim3((unsigned)nchunks, (unsigned)batch), dim3(kScanNT), 0,
                     S(stream), f0, reinterpret_cast<const double*>(workspace), omega, n_samples,
                     nchunks, sample_rate);
  return launch_status();
}

int ddsp_hip_harmonic_synth(const float* f0, const float* amplitudes, float* out, int64_t batch,
                            int64_t n_samples, int64_t n_harmonic, float sample_rate,
                            void* workspace, size_t workspace_bytes, void* stream) {
  if (batch < 0 || n_samples < 0 || n_harmonic < 0 || n_harmonic > (1 << 20)) return DDSP_HIP_EINVAL;
  if (batch * n_samples == 0) return DDSP_HIP_OK;
  if (!f0 || !out || (n_harmonic > 0 && !amplitudes)) return DDSP_HIP_EINVAL;
  if (n_harmonic == 0) {
    if (hipMemsetAsync(out, 0, sizeof(float) * batch * n_samples, S(stream)) != hipSuccess)
      return DDSP_HIP_ELAUNCH;
    return DDSP_HIP_OK;
  }
  int nchunks = 0;
  int st = phase_common(f0, batch, n_samples, sample_rate, workspace, workspace_bytes, stream, &nchunks);
  if (st) return st;
  const bool vec4 = (n_harmonic % 4 == 0) && ((reinterpret_cast<uintptr_t>(amplitudes) & 15) == 0);
  if (vec4 && n_harmonic <= 4 * kTileMaxPF * kScanNT / kStage) {
    const int H = (int)n_harmonic;
    const int Hs = H + ((12 - (H & 7)) & 7);  // smallest stride >= H with stride == 4 (mod 8)
    const size_t shm = sizeof(float) * (size_t)kStage * Hs;
    hipLaunchKernelGGL(harmonic_samples_tiled_kernel, dim3((unsigned)nchunks, (unsigned)batch),
                       dim3(kScanNT), shm, S(stream), f0, amplitudes,
                       reinterpret_cast<const double*>(workspace), out, n_samples, nchunks, H, Hs,
                       sample_rate);
  } else if (vec4)
    hipLaunchKernelGGL(harmonic_samples_kernel<true>, dim3((unsigned)nchunks, (unsigned)batch),
                       dim3(kScanNT), 0, S(stream), f0, amplitudes,
                       reinterpret_cast<const double*>(workspace), out, n_samples, nchunks,
                       (int)n_harmonic, sample_rate);
  else
    hipLaunchKernelGGL(harmonic_samples_kernel<false>, dim3((unsigned)nchunks, (unsigned)batch),
                       dim3(kScanNT), 0, S(stream), f0, amplitudes,
                       reinterpret_cast<const double*>(workspace), out, n_samples, nchunks,
                       (int)n_harmonic, sample_rate);
  return launch_status();
}

}  // extern "C"
