// Backward (vector-Jacobian) kernels of the synthesis path for training (SURVEY.md §8(f) rank 2;
// train.py:84-130 back-propagates the multiscale spectral loss through DDSPDecoder.forward).
//
// What the reference's autograd computes, restated per frame (F frames of bs samples, H
// harmonics, NB noise bands, upstream gradient g of the frame's audio):
//
//   harmonic (modules.py:69-80, core.py:136-141): out[t] = sum_k A_k sin(fl32(w_t (k+1))) with
//     A_k frame-constant (upsample is nearest), so dA_k = sum_{t in frame} g_t sin(w_t (k+1))
//     — the upsample backward (sum over the block) fused with the sine product;
//   controls (modules.py:44-67): a = scale_fn(p0), v_k = scale_fn(p_k) * mask_k, u_k = v_k / D,
//     D = sum v, A_k = a u_k:  da = sum dA_k u_k,  dv_k = a (dA_k - da) / D,
//     dp_k = dv_k mask_k scale_fn'(p_k),  dp0 = da scale_fn'(p0);
//   noise (modules.py:116-128, core.py:144-176): y = trunc_conv(x, h), h[j(q)] = ir[src(q)] hann[q]
//     for q < min(n, bs) with j(q) = (q - n/2) mod bs, src(q) = (q - n/2) mod n, ir = irfft(A):
//     dh[j] = sum_{i>=j} g_i x_{i-j},  dA_k = (c_k/n) (-1)^k sum_q dh[j(q)] hann[q] cos(2 pi q k/n),
//     c_0 = c_{n/2} = 1, else 2;  raw magnitudes: dm_k = dA_k scale_fn'(m_k + bias).
//
// f0 is an input feature in the reference's training loop (train.py:84-99: batch['pitch']),
// so no gradient flows to it; the host layer refuses f0 that requires grad.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "noise_dsp.h"

namespace ddsp {
namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// d/dx scale_function(x) = 2 ln10 sigmoid(x)^ln10 (1 - sigmoid(x)), with 1 - sigmoid formed as
// e * sigmoid (no cancellation for large x).
__device__ __forceinline__ float scale_fn_grad(float x) {
  const float e = expf(-x);
  const float sig = 1.0f / (1.0f + e);
  const float one_minus = e > 1e30f ? 1.0f : e * sig;
  const float p = exp2f(kLn10F * log2f(sig));
  return 2.0f * kLn10F * p * one_minus;
}

// acc + g * sin(x) for |x| < kFastArgLimit: the reduction and polynomial of sin_reduced with
// g applied to the reduced argument (13 VALU ops).
__device__ __forceinline__ float gsin_acc(float x, float g, float acc) {
  const float rs = reduce_signed(x);
  const float r2 = rs * rs;
  float q = fmaf(kS9, r2, kS7);
  q = fmaf(q, r2, kS5);
  q = fmaf(q, r2, kS3);
  q = fmaf(q, r2, 1.0f);
  return fmaf(rs * g, q, acc);
}

// ---------------------------------------------------------------------------------------
// scale_function backward: dx = g * scale_fn'(x + bias)
__global__ void scale_backward_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                      float* __restrict__ dx, int64_t n, float bias) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = g[i] * scale_fn_grad(x[i] + bias);
}

// upsample backward (core.py:64-67, nearest): d[b,f,c] = sum_r g[b, f*R + r, c]
__global__ void upsample_backward_kernel(const float* __restrict__ g, float* __restrict__ d,
                                         int64_t rows_out, int64_t C, int64_t R) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows_out * C;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / C, c = i - row * C;
    const float* src = g + row * R * C + c;
    float s = 0.0f;
    for (int64_t r = 0; r < R; ++r) s += src[r * C];
    d[i] = s;
  }
}

// HarmonicSynth.get_controls backward (modules.py:44-67); one wave per frame row.
__global__ void __launch_bounds__(256) controls_backward_kernel(
    const float* __restrict__ amp_raw, int64_t amp_ld, const float* __restrict__ dist_raw, int64_t dist_ld,
    const float* __restrict__ f0, const float* __restrict__ d_amp, const float* __restrict__ d_dist,
    float* __restrict__ d_amp_raw, float* __restrict__ d_dist_raw, int64_t rows, int H, float sr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* dr = dist_raw + row * dist_ld;
  const float* dd = d_dist + row * H;
  const float pitch0 = f0[row];
  const float half_sr = sr * 0.5f;
  double sv = 0.0;
  for (int k = lane; k < H; k += 64) sv += (double)controls_value(dr[k], pitch0, k, half_sr);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o, 64);
  const float D = (float)sv;
  double su = 0.0;  // sum_j du_j u_j
  for (int k = lane; k < H; k += 64) su += (double)dd[k] * (double)(controls_value(dr[k], pitch0, k, half_sr) / D);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) su += __shfl_xor(su, o, 64);
  const float s = (float)su;
  float* out = d_dist_raw + row * H;
  for (int k = lane; k < H; k += 64) {
    const float raw = dr[k];
    const float mask = (pitch0 * (float)(k + 1)) < half_sr ? kOnePlusEps : kEps;
    out[k] = ((dd[k] - s) / D) * mask * scale_fn_grad(raw);
  }
  if (lane == 0) d_amp_raw[row] = d_amp[row] * scale_fn_grad(amp_raw[row * amp_ld]);
}

// ---------------------------------------------------------------------------------------
// Harmonic backward, one workgroup per (item, frame).  Item (k, s) of the H x NS grid sums
// g_t sin(w_t (k+1)) over segment s of the frame's samples; (w_t, g_t) pairs are staged in LDS
// and read as broadcasts (all lanes of a wave share the segment).
//   PARAMS: controls recomputed from the raw projection param[B,F,H+1] -> d_param[B,F,H+1]
//   else:   amp[B,F] and the normalised distribution dist[B,F,H] -> d_amp[B,F], d_dist[B,F,H]
template <bool PARAMS>
__global__ void __launch_bounds__(1024) harmonic_backward_kernel(
    const float* __restrict__ f0, const float* __restrict__ grad, const float* __restrict__ param,
    const float* __restrict__ amp, const float* __restrict__ dist, float* __restrict__ d_param,
    float* __restrict__ d_amp, float* __restrict__ d_dist, int F, int H, int bs, float sr, int NS) {
  extern __shared__ float smem[];
  __shared__ double red[32];
  __shared__ double red2[32];
  __shared__ int fast_s;
  float2* wg = reinterpret_cast<float2*>(smem);  // [bs] (omega_t, g_t)
  float* part = smem + 2 * bs;                   // [NS * H]
  float* uk = part + NS * H;                     // [H] u_k (PARAMS: v_k first)
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, NT = blockDim.x;
  const int64_t frame = (int64_t)b * F + f;
  const float* f0b = f0 + (int64_t)b * F;
  const float pitch0 = f0b[f];
  const float half_sr = sr * 0.5f;
  const float* prow = PARAMS ? param + frame * (H + 1) : nullptr;

  double part_s = 0.0, part_d = 0.0;
  for (int q = tid; q < f; q += NT) part_s += (double)bs * (double)phase_inc(f0b[q], sr);
  for (int k = tid; k < H; k += NT) {
    if (PARAMS) {
      const float v = controls_value(prow[1 + k], pitch0, k, half_sr);
      uk[k] = v;
      part_d += (double)v;
    } else {
      uk[k] = dist[frame * H + k];
    }
  }
  const float* gf = grad + frame * bs;
  for (int j = tid; j < bs; j += NT) wg[j].y = gf[j];
  block_sum_double2(part_s, part_d, red);
  const double S0 = part_s;
  const float norm = (float)part_d;
  const double dinc = (double)phase_inc(pitch0, sr);
  for (int j = tid; j < bs; j += NT) wg[j].x = (float)(S0 + (double)(j + 1) * dinc);
  const float a = PARAMS ? scale_fn(prow[0]) : amp[frame];
  if (PARAMS)
    for (int k = tid; k < H; k += NT) uk[k] = uk[k] / norm;
  if (tid == 0) {
    const float w0 = (float)(S0 + dinc), w1 = (float)(S0 + (double)bs * dinc);
    fast_s = fmaxf(fabsf(w0), fabsf(w1)) * (float)H < kFastArgLimit;
  }
  __syncthreads();

  for (int item = tid; item < H * NS; item += NT) {
    const int s = item / H, k = item - s * H;
    const int j0 = (int)((int64_t)s * bs / NS), j1 = (int)((int64_t)(s + 1) * bs / NS);
    const float kf = (float)(k + 1);
    float acc0 = 0.0f, acc1 = 0.0f;
    if (fast_s) {
      int j = j0;
      for (; j + 1 < j1; j += 2) {
        const float2 p0 = wg[j], p1 = wg[j + 1];
        acc0 = gsin_acc(p0.x * kf, p0.y, acc0);
        acc1 = gsin_acc(p1.x * kf, p1.y, acc1);
      }
      if (j < j1) acc0 = gsin_acc(wg[j].x * kf, wg[j].y, acc0);
    } else {
      for (int j = j0; j < j1; ++j) {
        const float x = wg[j].x * kf;
        acc0 = fmaf(wg[j].y, fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x), acc0);
      }
    }
    part[s * H + k] = acc0 + acc1;
  }
  __syncthreads();

  double da_part = 0.0;
  for (int k = tid; k < H; k += NT) {
    float dA = part[k];
    for (int s = 1; s < NS; ++s) dA += part[s * H + k];
    part[k] = dA;
    da_part += (double)dA * (double)uk[k];
  }
  const float da = (float)block_sum_double(da_part, red2);  // barrier: part[0..H) complete
  if (PARAMS) {
    float* dp = d_param + frame * (H + 1);
    for (int k = tid; k < H; k += NT) {
      const float mask = (pitch0 * (float)(k + 1)) < half_sr ? kOnePlusEps : kEps;
      const float dv = a * (part[k] - da) / norm;
      dp[1 + k] = dv * mask * scale_fn_grad(prow[1 + k]);
    }
    if (tid == 0) dp[0] = da * scale_fn_grad(prow[0]);
  } else {
    for (int k = tid; k < H; k += NT) d_dist[frame * H + k] = part[k] * a;
    if (tid == 0) d_amp[frame] = da;
  }
}

// ---------------------------------------------------------------------------------------
// Filtered-noise backward, one workgroup per frame: dh at the n filter taps by direct
// correlation of g with the frame's noise (NSEG segments of the lag sum per tap), then the
// transposed filter design (a cosine transform of the windowed tap gradients) -> dA [NB].
//   RNG: the noise is regenerated from the forward's Philox (seed, offset) — same counter
//   mapping as filtered_noise_kernel / synth_frame_kernel;  RAW: chain scale_fn(m + bias).
template <bool RNG, bool RAW>
__global__ void __launch_bounds__(256) noise_backward_kernel(
    const float* __restrict__ grad, const float* __restrict__ noise, uint32_t k0, uint32_t k1,
    uint32_t off0, uint32_t off1, const float* __restrict__ mags, float bias, float* __restrict__ d_mags,
    int NB, int bs, int NSEG) {
  extern __shared__ float smem[];
  const int n = 2 * (NB - 1), half = n >> 1;
  const int qmax = min(n, bs);
  float* gl = smem;            // [bs]
  float* xl = gl + bs;         // [bs]
  float* ct = xl + bs;         // [n]
  float* e = ct + n;           // [n]   windowed tap gradients by q
  float* part = e + n;         // [NSEG * qmax]
  const int64_t frame = blockIdx.x;
  const int tid = threadIdx.x, NT = blockDim.x;
  const float* gf = grad + frame * bs;
  for (int j = tid; j < bs; j += NT) gl[j] = gf[j];
  if (RNG) {
    const int fquads = (bs + 3) >> 2;
    for (int t = tid; t < fquads; t += NT) {
      const uint64_t qc = (uint64_t)frame * (uint64_t)fquads + (uint64_t)t;
      const Philox4 r = philox4x32_10((uint32_t)qc, (uint32_t)(qc >> 32), off0, off1, k0, k1);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (4 * t + c < bs) xl[4 * t + c] = uniform_pm1(r.v[c]);
    }
  } else {
    const float* xf = noise + frame * bs;
    for (int j = tid; j < bs; j += NT) xl[j] = xf[j];
  }
  fill_cos_table(ct, n);
  __syncthreads();

  // dh[j(q)] = sum_{d=0}^{bs-1-j} g[j+d] x[d], lag range split into NSEG fixed d-segments
  for (int item = tid; item < qmax * NSEG; item += NT) {
    const int seg = item / qmax, q = item - seg * qmax;
    int j = (q - half) % bs;
    if (j < 0) j += bs;
    const int d0 = (int)((int64_t)seg * bs / NSEG);
    const int d1 = min((int)((int64_t)(seg + 1) * bs / NSEG), bs - j);
    float c0 = 0.0f, c1 = 0.0f;
    int d = d0;
    for (; d + 1 < d1; d += 2) {
      c0 = fmaf(gl[j + d], xl[d], c0);
      c1 = fmaf(gl[j + d + 1], xl[d + 1], c1);
    }
    if (d < d1) c0 = fmaf(gl[j + d], xl[d], c0);
    part[seg * qmax + q] = c0 + c1;
  }
  __syncthreads();
  for (int q = tid; q < n; q += NT) {
    float v = 0.0f;
    if (q < qmax) {
      for (int s = 0; s < NSEG; ++s) v += part[s * qmax + q];
      v *= 0.5f - 0.5f * ct[q];  // periodic Hann(n) at q
    }
    e[q] = v;
  }
  __syncthreads();

  const float inv_n = 1.0f / (float)n;
  const bool pow2 = (n & (n - 1)) == 0;
  for (int k = tid; k < NB; k += NT) {
    float s0 = 0.0f, s1 = 0.0f;
    if (pow2) {
      const int mask = n - 1;
      int q = 0;
      for (; q + 1 < n; q += 2) {
        s0 = fmaf(e[q], ct[(q * k) & mask], s0);
        s1 = fmaf(e[q + 1], ct[((q + 1) * k) & mask], s1);
      }
      for (; q < n; ++q) s0 = fmaf(e[q], ct[(q * k) & mask], s0);
    } else {
      int qk = 0;
      for (int q = 0; q < n; ++q) {
        s0 = fmaf(e[q], ct[qk], s0);
        qk += k;
        if (qk >= n) qk -= n;
      }
    }
    const float ck = (k == 0 || k == half) ? 1.0f : 2.0f;
    float dA = (s0 + s1) * ck * inv_n;
    if (k & 1) dA = -dA;
    if (RAW) dA *= scale_fn_grad(mags[frame * NB + k] + bias);
    d_mags[frame * NB + k] = dA;
  }
}

// amp_to_impulse_response backward (core.py:144-166): dimpulse[rows, target] -> damp[rows, NB]
__global__ void __launch_bounds__(256) impulse_response_backward_kernel(
    const float* __restrict__ dimp, float* __restrict__ damp, int NB, int target) {
  extern __shared__ float smem[];
  const int n = 2 * (NB - 1), half = n >> 1;
  const int qmax = min(n, target);
  float* ct = smem;   // [n]
  float* e = ct + n;  // [n]
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x, NT = blockDim.x;
  fill_cos_table(ct, n);
  __syncthreads();
  const float* dh = dimp + row * target;
  for (int q = tid; q < n; q += NT) {
    float v = 0.0f;
    if (q < qmax) {
      int j = (q - half) % target;
      if (j < 0) j += target;
      v = dh[j] * (0.5f - 0.5f * ct[q]);
    }
    e[q] = v;
  }
  __syncthreads();
  const float inv_n = 1.0f / (float)n;
  for (int k = tid; k < NB; k += NT) {
    float s = 0.0f;
    int qk = 0;
    for (int q = 0; q < n; ++q) {
      s = fmaf(e[q], ct[qk], s);
      qk += k;
      if (qk >= n) qk -= n;
    }
    const float ck = (k == 0 || k == half) ? 1.0f : 2.0f;
    float dA = s * ck * inv_n;
    damp[row * NB + k] = (k & 1) ? -dA : dA;
  }
}

// harmonic_synth backward at the op boundary (core.py:136-141): per-sample amplitudes
// dA[b,t,k] = g[b,t] * sin(fl32(w[b,t] (k+1))), 4 consecutive outputs per thread.
__global__ void harmonic_synth_backward_kernel(const float* __restrict__ omega, const float* __restrict__ g,
                                               float* __restrict__ dA, int64_t total, int H) {
  const int64_t i0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i0 >= total) return;
  int64_t t = i0 / H;
  int k = (int)(i0 - t * H);
  float w = omega[t], gv = g[t];
  float v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float x = w * (float)(k + 1);
    v[c] = gv * (fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x));
    if (++k == H && i0 + c + 1 < total) {
      k = 0;
      ++t;
      w = omega[t];
      gv = g[t];
    }
  }
  if (i0 + 3 < total && (((uintptr_t)(dA + i0)) & 15) == 0) {
    *reinterpret_cast<float4*>(dA + i0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int c = 0; c < 4 && i0 + c < total; ++c) dA[i0 + c] = v[c];
  }
}

unsigned grid1d(int64_t n, int per_block) {
  return (unsigned)std::min<int64_t>(std::max<int64_t>((n + per_block - 1) / per_block, 1), 1 << 20);
}

// NS sample segments per harmonic for the harmonic backward: fill the workgroup's waves.
void harmonic_backward_shape(int H, int bs, int& nt, int& ns) {
  double best = -1.0;
  nt = 64;
  ns = 1;
  for (int s = 1; s <= 8 && s <= bs; ++s) {
    const int items = H * s;
    if (items > 1024) break;
    const int t = ((items + 63) / 64) * 64;
    const double eff = (double)items / (double)t;
    if (eff > best + 1e-9) {
      best = eff;
      nt = t;
      ns = s;
    }
  }
  if (H > 1024) {
    nt = 1024;
    ns = 1;
  }
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int ddsp_hip_scale_function_backward(const float* x, const float* grad, float* dx, int64_t n, float bias,
                                     void* stream) {
  if (n < 0 || (n > 0 && (!x || !grad || !dx))) return DDSP_HIP_EINVAL;
  if (n == 0) return DDSP_HIP_OK;
  hipLaunchKernelGGL(scale_backward_kernel, dim3(grid1d(n, 256)), dim3(256), 0, S(stream), x, grad, dx, n,
                     bias);
  return launch_status();
}

int ddsp_hip_upsample_backward(const float* grad, float* dx, int64_t batch, int64_t frames, int64_t channels,
                               int64_t factor, void* stream) {
  if (batch < 0 || frames < 0 || channels < 0 || factor < 1) return DDSP_HIP_EINVAL;
  const int64_t n = batch * frames * channels;
  if (n == 0) return DDSP_HIP_OK;
  if (!grad || !dx) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(upsample_backward_kernel, dim3(grid1d(n, 256)), dim3(256), 0, S(stream), grad, dx,
                     batch * frames, channels, factor);
  return launch_status();
}

int ddsp_hip_harmonic_controls_backward(const float* amplitudes_raw, int64_t amp_ld,
                                        const float* distribution_raw, int64_t dist_ld, const float* f0,
                                        const float* grad_amplitudes, const float* grad_distribution,
                                        float* grad_amplitudes_raw, float* grad_distribution_raw,
                                        int64_t rows, int64_t n_harmonic, float sample_rate, void* stream) {
  if (rows < 0 || n_harmonic < 1 || amp_ld < 1 || dist_ld < n_harmonic) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!amplitudes_raw || !distribution_raw || !f0 || !grad_amplitudes || !grad_distribution ||
      !grad_amplitudes_raw || !grad_distribution_raw)
    return DDSP_HIP_EINVAL;
  const int64_t blocks = (rows + 3) / 4;
  if (blocks > INT32_MAX) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(controls_backward_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), amplitudes_raw,
                     amp_ld, distribution_raw, dist_ld, f0, grad_amplitudes, grad_distribution,
                     grad_amplitudes_raw, grad_distribution_raw, rows, (int)n_harmonic, sample_rate);
  return launch_status();
}

static int harmonic_backward_launch(bool params, const float* f0, const float* grad, const float* param,
                                    const float* amp, const float* dist, float* d_param, float* d_amp,
                                    float* d_dist, int64_t batch, int64_t frames, int64_t H, int64_t bs,
                                    float sr, void* stream) {
  if (batch < 0 || frames < 0 || H < 1 || bs < 1 || !(sr > 0)) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (batch > 65535 || frames > INT32_MAX || H > 4096 || bs > 8192) return DDSP_HIP_ERANGE;
  int nt, ns;
  harmonic_backward_shape((int)H, (int)bs, nt, ns);
  const size_t shm = sizeof(float) * ((size_t)2 * bs + (size_t)ns * H + H);
  if (shm > 150 * 1024) return DDSP_HIP_ERANGE;
  const dim3 grid((unsigned)frames, (unsigned)batch);
  if (params)
    hipLaunchKernelGGL(harmonic_backward_kernel<true>, grid, dim3(nt), shm, S(stream), f0, grad, param, nullptr,
                       nullptr, d_param, nullptr, nullptr, (int)frames, (int)H, (int)bs, sr, ns);
  else
    hipLaunchKernelGGL(harmonic_backward_kernel<false>, grid, dim3(nt), shm, S(stream), f0, grad, nullptr, amp,
                       dist, nullptr, d_amp, d_dist, (int)frames, (int)H, (int)bs, sr, ns);
  return launch_status();
}

int ddsp_hip_harmonic_synth_frames_backward(const float* f0, const float* amplitudes, const float* distribution,
                                            const float* grad, float* grad_amplitudes,
                                            float* grad_distribution, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream) {
  if (!f0 || !amplitudes || !distribution || !grad || !grad_amplitudes || !grad_distribution)
    return batch == 0 || frames == 0 ? DDSP_HIP_OK : DDSP_HIP_EINVAL;
  return harmonic_backward_launch(false, f0, grad, nullptr, amplitudes, distribution, nullptr, grad_amplitudes,
                                  grad_distribution, batch, frames, n_harmonic, block_size, sample_rate, stream);
}

int ddsp_hip_harmonic_synth_params_backward(const float* f0, const float* param, const float* grad,
                                            float* grad_param, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream) {
  if (!f0 || !param || !grad || !grad_param) return batch == 0 || frames == 0 ? DDSP_HIP_OK : DDSP_HIP_EINVAL;
  return harmonic_backward_launch(true, f0, grad, param, nullptr, nullptr, grad_param, nullptr, nullptr, batch,
                                  frames, n_harmonic, block_size, sample_rate, stream);
}

int ddsp_hip_filtered_noise_backward(const float* magnitudes, const float* noise, uint64_t seed, uint64_t offset,
                                     int raw, float bias, const float* grad, float* grad_magnitudes,
                                     int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                                     void* stream) {
  if (batch < 0 || frames < 0 || n_bands < 2 || block_size < 1) return DDSP_HIP_EINVAL;
  const int64_t nf = batch * frames;
  if (nf == 0) return DDSP_HIP_OK;
  if (!grad || !grad_magnitudes || (raw && !magnitudes)) return DDSP_HIP_EINVAL;
  if (nf > INT32_MAX || block_size > 8192 || n_bands > 4097) return DDSP_HIP_ERANGE;
  const int n = 2 * (int)(n_bands - 1), bs = (int)block_size;
  const int qmax = std::min(n, bs);
  const int nt = 256;
  const int nseg = std::max(1, std::min(8, nt / qmax));
  const size_t shm = sizeof(float) * ((size_t)2 * bs + 2 * (size_t)n + (size_t)nseg * qmax);
  if (shm > 150 * 1024) return DDSP_HIP_ERANGE;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
  const dim3 grid((unsigned)nf);
#define DDSP_NB_LAUNCH(RNG_, RAW_)                                                                            \
  hipLaunchKernelGGL((noise_backward_kernel<RNG_, RAW_>), grid, dim3(nt), shm, S(stream), grad, noise, k0, k1, o0, \
                     o1, magnitudes, bias, grad_magnitudes, (int)n_bands, bs, nseg)
  if (noise) {
    if (raw) DDSP_NB_LAUNCH(false, true); else DDSP_NB_LAUNCH(false, false);
  } else {
    if (raw) DDSP_NB_LAUNCH(true, true); else DDSP_NB_LAUNCH(true, false);
  }
#undef DDSP_NB_LAUNCH
  return launch_status();
}

int ddsp_hip_amp_to_impulse_response_backward(const float* grad_impulse, float* grad_amp, int64_t rows,
                                              int64_t n_bands, int64_t target_size, void* stream) {
  if (rows < 0 || n_bands < 2 || target_size < 1) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!grad_impulse || !grad_amp) return DDSP_HIP_EINVAL;
  if (rows > INT32_MAX || n_bands > 4097) return DDSP_HIP_ERANGE;
  const int n = 2 * (int)(n_bands - 1);
  const size_t shm = sizeof(float) * 2 * (size_t)n;
  hipLaunchKernelGGL(impulse_response_backward_kernel, dim3((unsigned)rows), dim3(256), shm, S(stream),
                     grad_impulse, grad_amp, (int)n_bands, (int)target_size);
  return launch_status();
}

int ddsp_hip_harmonic_synth_backward(const float* omega, const float* grad, float* grad_amplitudes,
                                     int64_t batch, int64_t n_samples, int64_t n_harmonic, void* stream) {
  if (batch < 0 || n_samples < 0 || n_harmonic < 1) return DDSP_HIP_EINVAL;
  const int64_t total = batch * n_samples * n_harmonic;
  if (total == 0) return DDSP_HIP_OK;
  if (!omega || !grad || !grad_amplitudes || n_harmonic > INT32_MAX) return DDSP_HIP_EINVAL;
  const int64_t threads = (total + 3) / 4;
  const int64_t blocks = (threads + 255) / 256;
  if (blocks > INT32_MAX) return DDSP_HIP_ERANGE;
  hipLaunchKernelGGL(harmonic_synth_backward_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), omega, grad,
                     grad_amplitudes, total, (int)n_harmonic);
  return launch_status();
}

}  // extern "C"
