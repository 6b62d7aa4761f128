// Multiscale STFT magnitudes and their backward: ddsp/core.py:27-41
// multiscale_fft — for each scale s, torch.stft(x, n_fft=s, hop=int(s*(1-overlap)), win_length=s,
// window=hann(s) (periodic), center=True (reflect padding by s/2), normalized=True (x s^-1/2),
// return_complex=True).abs() — the spectrograms train.py:70-76 compares.
//
// Layout: signal x[B, T]; magnitudes written frame-major M[B, frames, s/2+1] (coalesced: one
// frame's bins are contiguous); the host hands out the transposed view [B, s/2+1, frames], the
// reference's shape.
//
// Forward: two real frames ride in one complex FFT (z = frame_a + i frame_b, LDS-resident
// radix-16 Stockham, fft_radix.h), split by Z[k] +- conj(Z[N-k]).  4096/s transforms per
// 256-thread workgroup.
// Backward: per frame, dx_frame[m] = c w[m] Re(sum_{k<=s/2} G[k] e^{+2 pi i k m/s}) with
// G = dM X/|X| — an inverse FFT of the Hermitian extension of G (two frames packed again, their
// real and imaginary parts) — written frame-major to dF[B, frames, s], then
// ddsp_hip_stft_overlap_add gathers the (<= s/hop) overlapping frames and the reflect padding
// back onto each sample (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "fft_radix.h"

namespace ddsp {
namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// reflect-padded sample of row xr at padded position p (center=True pads N/2 on both sides)
__device__ __forceinline__ float reflect_load(const float* xr, int64_t T, int64_t i) {
  if (i < 0) i = -i;
  if (i >= T) i = 2 * (T - 1) - i;
  return xr[i];
}

template <int N>
__device__ __forceinline__ void load_frames(const float* __restrict__ xr, int64_t T, int hop, int frames, int fa,
                                            int t, float2 (&v)[16]) {
  constexpr int Q = N / 16, STEP = 4096 / N;
  const int fb = fa + 1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = t + Q * r;
    const float w = 0.5f - 0.5f * kTwiddle4096[2 * ((m * STEP) & 4095)];  // periodic Hann(N)
    const float a = fa < frames ? reflect_load(xr, T, (int64_t)fa * hop + m - N / 2) * w : 0.0f;
    const float b = fb < frames ? reflect_load(xr, T, (int64_t)fb * hop + m - N / 2) * w : 0.0f;
    v[r] = make_float2(a, b);
  }
}

// grid (ceil(frames / (2 * 4096/N)), B), 256 threads
template <int N>
__global__ void __launch_bounds__(256) stft_mag_kernel(const float* __restrict__ x, int64_t T, int hop,
                                                       int frames, float scale, float* __restrict__ M) {
  constexpr int Q = N / 16, TPW = 4096 / N, BINS = N / 2 + 1;
  __shared__ float2 lds_all[TPW * (N + N / 16)];
  const int tr = threadIdx.x / Q, t = threadIdx.x - tr * Q;
  float2* lds = lds_all + tr * (N + N / 16);
  const int b = blockIdx.y;
  const int fa = 2 * (blockIdx.x * TPW + tr);
  const float* xr = x + (int64_t)b * T;
  float2 v[16];
  load_frames<N>(xr, T, hop, frames, fa, t, v);
  fft_n<N, false, false>(v, lds, t);  // lds untouched so far
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[lds_idx(t + Q * r)] = v[r];
  __syncthreads();
  if (fa >= frames) return;
  float* Ma = M + ((int64_t)b * frames + fa) * BINS;
  const bool has_b = fa + 1 < frames;
  for (int k = t; k < BINS; k += Q) {
    const float2 zk = lds[lds_idx(k)], zn = lds[lds_idx((N - k) & (N - 1))];
    // X_a = (Z[k] + conj(Z[N-k])) / 2,  X_b = (Z[k] - conj(Z[N-k])) / (2i)
    const float ar = 0.5f * (zk.x + zn.x), ai = 0.5f * (zk.y - zn.y);
    const float br = 0.5f * (zk.y + zn.y), bi = -0.5f * (zk.x - zn.x);
    Ma[k] = sqrtf(fmaf(ar, ar, ai * ai)) * scale;
    if (has_b) Ma[BINS + k] = sqrtf(fmaf(br, br, bi * bi)) * scale;
  }
}

// grid as stft_mag_kernel; dF[B, frames, N] = per-frame gradient of the windowed frame
template <int N>
__global__ void __launch_bounds__(256) stft_mag_backward_kernel(const float* __restrict__ x, int64_t T, int hop,
                                                                int frames, float scale,
                                                                const float* __restrict__ gM,
                                                                float* __restrict__ dF) {
  constexpr int Q = N / 16, TPW = 4096 / N, BINS = N / 2 + 1, STEP = 4096 / N;
  __shared__ float2 lds_all[TPW * (N + N / 16)];
  const int tr = threadIdx.x / Q, t = threadIdx.x - tr * Q;
  float2* lds = lds_all + tr * (N + N / 16);
  const int b = blockIdx.y;
  const int fa = 2 * (blockIdx.x * TPW + tr);
  const float* xr = x + (int64_t)b * T;
  float2 v[16];
  load_frames<N>(xr, T, hop, frames, fa, t, v);
  fft_n<N, false, false>(v, lds, t);  // lds untouched so far
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[lds_idx(t + Q * r)] = v[r];
  __syncthreads();
  // G = dM X/|X| per frame; packed Hermitian extension H = H_a + i H_b written over Z (each
  // thread owns the index pair {k, N-k})
  const bool va = fa < frames, vb = fa + 1 < frames;
  const float* ga = gM + ((int64_t)b * frames + (va ? fa : 0)) * BINS;
  for (int k = t; k < BINS; k += Q) {
    const int kn = (N - k) & (N - 1);
    const float2 zk = lds[lds_idx(k)], zn = lds[lds_idx(kn)];
    const float ar = 0.5f * (zk.x + zn.x), ai = 0.5f * (zk.y - zn.y);
    const float br = 0.5f * (zk.y + zn.y), bi = -0.5f * (zk.x - zn.x);
    const float na = sqrtf(fmaf(ar, ar, ai * ai)), nb = sqrtf(fmaf(br, br, bi * bi));
    const float sa = (va && na > 0.0f) ? ga[k] / na : 0.0f;
    const float sb = (vb && nb > 0.0f) ? ga[BINS + k] / nb : 0.0f;
    const float2 Ga = make_float2(sa * ar, sa * ai), Gb = make_float2(sb * br, sb * bi);
    if (k == 0 || k == N / 2) {
      lds[lds_idx(k)] = make_float2(Ga.x, Gb.x);  // real parts only
    } else {
      // H_a[k] = G_a/2, H_a[N-k] = conj(G_a)/2 (same for b); H = H_a + i H_b
      lds[lds_idx(k)] = make_float2(0.5f * (Ga.x - Gb.y), 0.5f * (Ga.y + Gb.x));
      lds[lds_idx(kn)] = make_float2(0.5f * (Ga.x + Gb.y), 0.5f * (Gb.x - Ga.y));
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = lds[lds_idx(t + Q * r)];
  fft_n<N, true>(v, lds, t);
  if (!va) return;
  float* da = dF + ((int64_t)b * frames + fa) * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = t + Q * r;
    const float w = (0.5f - 0.5f * kTwiddle4096[2 * ((m * STEP) & 4095)]) * scale;
    da[m] = v[r].x * w;
    if (vb) da[N + m] = v[r].y * w;
  }
}

// dx[b, i] = sum over the padded positions p that read sample i (direct p = i + N/2 and the
// reflections) of sum_f dF[b, f, p - f hop]
__global__ void stft_overlap_add_kernel(const float* __restrict__ dF, int64_t T, int N, int hop, int frames,
                                        int64_t B, int accumulate, float* __restrict__ dx) {
  const int64_t total = B * T;
  for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = id / T, i = id - b * T;
    const int half = N / 2;
    const float* Fb = dF + b * (int64_t)frames * N;
    int64_t ps[3];
    int np = 0;
    ps[np++] = i + half;
    if (i >= 1 && i <= half) ps[np++] = half - i;                                     // left reflection
    if (i >= T - 1 - half && i <= T - 2) ps[np++] = half + 2 * (T - 1) - i;           // right reflection
    float acc = 0.0f;
    for (int c = 0; c < np; ++c) {
      const int64_t p = ps[c];
      int64_t f0 = p - N + 1 <= 0 ? 0 : (p - N + 1 + hop - 1) / hop;
      int64_t f1 = std::min<int64_t>(p / hop, frames - 1);
      for (int64_t f = f0; f <= f1; ++f) acc += Fb[f * N + (p - f * hop)];
    }
    dx[id] = accumulate ? dx[id] + acc : acc;
  }
}

template <int N>
int stft_mag_launch(const float* x, int64_t B, int64_t T, int hop, int frames, float scale, float* M,
                    void* stream) {
  constexpr int TPW = 4096 / N;
  const unsigned gx = (unsigned)((frames + 2 * TPW - 1) / (2 * TPW));
  hipLaunchKernelGGL(stft_mag_kernel<N>, dim3(gx, (unsigned)B), dim3(256), 0, S(stream), x, T, hop, frames, scale,
                     M);
  return launch_status();
}

template <int N>
int stft_bwd_launch(const float* x, int64_t B, int64_t T, int hop, int frames, float scale, const float* gM,
                    float* dF, void* stream) {
  constexpr int TPW = 4096 / N;
  const unsigned gx = (unsigned)((frames + 2 * TPW - 1) / (2 * TPW));
  hipLaunchKernelGGL(stft_mag_backward_kernel<N>, dim3(gx, (unsigned)B), dim3(256), 0, S(stream), x, T, hop,
                     frames, scale, gM, dF);
  return launch_status();
}

int check_stft(int64_t B, int64_t T, int64_t n_fft, int64_t hop) {
  if (B < 0 || T < 1 || hop < 1) return DDSP_HIP_EINVAL;
  if (n_fft < 16 || n_fft > 4096 || (n_fft & (n_fft - 1))) return DDSP_HIP_ERANGE;
  if (n_fft / 2 >= T) return DDSP_HIP_EINVAL;  // reflect padding needs T > n_fft/2 (as torch.stft)
  if (B > 65535 || T / hop + 1 > INT32_MAX) return DDSP_HIP_ERANGE;
  return DDSP_HIP_OK;
}


// ---------------------------------------------------------------------------------------
// The whole training loss of train.py:70-76 for one scale, fused: for each pair of frames
// (fa, fb) the target and reconstruction frames share one complex FFT (z = target + i recon),
// the loss terms |Mx - My| and |log(Mx + 1e-7) - log(My + 1e-7)| are summed in fp64 per
// workgroup, and dL/dMy = [sgn(My - Mx) + sgn(log My' - log Mx') / (My + 1e-7)] / count is
// turned into the reconstruction's frame gradients by one inverse FFT of the packed Hermitian
// extensions of the two frames (as stft_mag_backward_kernel).  No spectrogram reaches HBM.
// grid (ceil(frames / (2 * 4096/N)), B); partials[block] = (sum lin, sum log)
template <int N>
__global__ void __launch_bounds__(256) spectral_loss_kernel(const float* __restrict__ xt, const float* __restrict__ xr,
                                                            int64_t T, int hop, int frames, float scale,
                                                            float inv_count, int want_grad,
                                                            double* __restrict__ partials, float* __restrict__ dF) {
  constexpr int Q = N / 16, TPW = 4096 / N, BINS = N / 2 + 1, STEP = 4096 / N;
  constexpr int KPT = (BINS + Q - 1) / Q;  // bins per thread
  __shared__ float2 lds_all[TPW * (N + N / 16)];
  __shared__ double red[32];
  const int tr = threadIdx.x / Q, t = threadIdx.x - tr * Q;
  float2* lds = lds_all + tr * (N + N / 16);
  const int b = blockIdx.y;
  const int fa = 2 * (blockIdx.x * TPW + tr);
  const float* rt = xt + (int64_t)b * T;
  const float* rr = xr + (int64_t)b * T;
  const float eps = 1e-7f;
  double lin = 0.0, lg = 0.0;
  float2 G[2][KPT];  // dL/dY_recon per bin, frames fa and fb
  // both frames' samples are loaded up front: the second frame's global loads overlap the first FFT
  float2 raw[2][16];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = fa + h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t i = (int64_t)f * hop + t + Q * r - N / 2;
      raw[h][r] = f < frames ? make_float2(reflect_load(rt, T, i), reflect_load(rr, T, i)) : make_float2(0.f, 0.f);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = fa + h;
    const bool valid = f < frames;
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float w = 0.5f - 0.5f * kTwiddle4096[2 * (((t + Q * r) * STEP) & 4095)];
      v[r] = make_float2(raw[h][r].x * w, raw[h][r].y * w);
    }
    fft_n<N, false>(v, lds, t);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[lds_idx(t + Q * r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int k = t + Q * i;
      G[h][i] = make_float2(0.f, 0.f);
      if (k < BINS && valid) {
        const float2 zk = lds[lds_idx(k)], zn = lds[lds_idx((N - k) & (N - 1))];
        const float ar = 0.5f * (zk.x + zn.x), ai = 0.5f * (zk.y - zn.y);    // target
        const float br = 0.5f * (zk.y + zn.y), bi = -0.5f * (zk.x - zn.x);   // reconstruction
        const float na = sqrtf(fmaf(ar, ar, ai * ai)), nb = sqrtf(fmaf(br, br, bi * bi));
        const float mx = na * scale, my = nb * scale;
        const float dlin = mx - my;
        const float dlog = logf(mx + eps) - logf(my + eps);
        lin += (double)fabsf(dlin);
        lg += (double)fabsf(dlog);
        if (want_grad) {
          // d/dMy of |Mx - My| + |log Mx' - log My'|  (sgn(0) = 0, as torch's abs backward)
          const float s1 = dlin > 0.f ? -1.f : (dlin < 0.f ? 1.f : 0.f);
          const float s2 = dlog > 0.f ? -1.f : (dlog < 0.f ? 1.f : 0.f);
          const float gm = (s1 + s2 / (my + eps)) * inv_count;
          const float sc = nb > 0.f ? gm * scale / nb : 0.f;  // dMy/dY = c Y/|Y|
          G[h][i] = make_float2(sc * br, sc * bi);
        }
      }
    }
  }
  block_sum_double2(lin, lg, red);
  if (threadIdx.x == 0) {
    partials[2 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x)] = lin;
    partials[2 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) + 1] = lg;
  }
  if (!want_grad) return;
  __syncthreads();
  // packed Hermitian extension H = H_a + i H_b of the two frames' gradients
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    const int k = t + Q * i;
    if (k < BINS) {
      const float2 Ga = G[0][i], Gb = G[1][i];
      if (k == 0 || k == N / 2) {
        lds[lds_idx(k)] = make_float2(Ga.x, Gb.x);
      } else {
        lds[lds_idx(k)] = make_float2(0.5f * (Ga.x - Gb.y), 0.5f * (Ga.y + Gb.x));
        lds[lds_idx(N - k)] = make_float2(0.5f * (Ga.x + Gb.y), 0.5f * (Gb.x - Ga.y));
      }
    }
  }
  __syncthreads();
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = lds[lds_idx(t + Q * r)];
  fft_n<N, true>(v, lds, t);
  if (fa >= frames) return;
  const bool vb = fa + 1 < frames;
  float* da = dF + ((int64_t)b * frames + fa) * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = t + Q * r;
    const float w = 0.5f - 0.5f * kTwiddle4096[2 * ((m * STEP) & 4095)];
    da[m] = v[r].x * w;
    if (vb) da[N + m] = v[r].y * w;
  }
}

// loss = sum over scales of (sum lin + sum log) / count_s, partial sums in a fixed order
__global__ void spectral_loss_finish_kernel(const double* __restrict__ partials, const int64_t* __restrict__ offs,
                                            const double* __restrict__ inv_counts, int n_scales,
                                            float* __restrict__ loss) {
  __shared__ double red[32];
  double acc = 0.0;
  for (int sidx = 0; sidx < n_scales; ++sidx) {
    double part = 0.0;
    for (int64_t i = offs[sidx] + threadIdx.x; i < offs[sidx + 1]; i += blockDim.x)
      part += partials[2 * i] + partials[2 * i + 1];
    acc += part * inv_counts[sidx];
  }
  acc = block_sum_double(acc, red);
  if (threadIdx.x == 0) loss[0] = (float)acc;
}

template <int N>
int spectral_loss_launch(const float* xt, const float* xr, int64_t B, int64_t T, int hop, int frames,
                         float scale, float inv_count, bool grad, double* partials, float* dF, void* stream) {
  constexpr int TPW = 4096 / N;
  const unsigned gx = (unsigned)((frames + 2 * TPW - 1) / (2 * TPW));
  hipLaunchKernelGGL(spectral_loss_kernel<N>, dim3(gx, (unsigned)B), dim3(256), 0, S(stream), xt, xr, T, hop, frames,
                     scale, inv_count, (int)grad, partials, dF);
  return launch_status();
}

int64_t loss_blocks(int64_t n_fft, int64_t frames, int64_t B) {
  const int64_t tpw = 4096 / n_fft;
  return ((frames + 2 * tpw - 1) / (2 * tpw)) * B;
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int64_t ddsp_hip_stft_frames(int64_t n_samples, int64_t hop) { return hop > 0 ? n_samples / hop + 1 : 0; }

int ddsp_hip_stft_magnitude(const float* x, float* magnitudes, int64_t batch, int64_t n_samples, int64_t n_fft,
                            int64_t hop, void* stream) {
  int st = check_stft(batch, n_samples, n_fft, hop);
  if (st) return st;
  if (batch == 0) return DDSP_HIP_OK;
  if (!x || !magnitudes) return DDSP_HIP_EINVAL;
  const int frames = (int)(n_samples / hop + 1);
  const float scale = (float)(1.0 / std::sqrt((double)n_fft));
  switch (n_fft) {
    case 16: return stft_mag_launch<16>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 32: return stft_mag_launch<32>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 64: return stft_mag_launch<64>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 128: return stft_mag_launch<128>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 256: return stft_mag_launch<256>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 512: return stft_mag_launch<512>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 1024: return stft_mag_launch<1024>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    case 2048: return stft_mag_launch<2048>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
    default: return stft_mag_launch<4096>(x, batch, n_samples, (int)hop, frames, scale, magnitudes, stream);
  }
}

size_t ddsp_hip_stft_backward_workspace_size(int64_t batch, int64_t n_samples, int64_t n_fft, int64_t hop) {
  if (batch < 1 || n_samples < 1 || n_fft < 1 || hop < 1) return 0;
  return sizeof(float) * (size_t)batch * (size_t)(n_samples / hop + 1) * (size_t)n_fft;
}

int ddsp_hip_stft_magnitude_backward(const float* x, const float* grad_magnitudes, float* grad_x, int64_t batch,
                                     int64_t n_samples, int64_t n_fft, int64_t hop, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  int st = check_stft(batch, n_samples, n_fft, hop);
  if (st) return st;
  if (batch == 0) return DDSP_HIP_OK;
  if (!x || !grad_magnitudes || !grad_x) return DDSP_HIP_EINVAL;
  if (!workspace || workspace_bytes < ddsp_hip_stft_backward_workspace_size(batch, n_samples, n_fft, hop))
    return DDSP_HIP_EWORKSPACE;
  const int frames = (int)(n_samples / hop + 1);
  const float scale = (float)(1.0 / std::sqrt((double)n_fft));
  float* dF = reinterpret_cast<float*>(workspace);
  const int h = (int)hop;
  switch (n_fft) {
    case 16: st = stft_bwd_launch<16>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 32: st = stft_bwd_launch<32>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 64: st = stft_bwd_launch<64>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 128: st = stft_bwd_launch<128>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 256: st = stft_bwd_launch<256>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 512: st = stft_bwd_launch<512>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 1024: st = stft_bwd_launch<1024>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    case 2048: st = stft_bwd_launch<2048>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
    default: st = stft_bwd_launch<4096>(x, batch, n_samples, h, frames, scale, grad_magnitudes, dF, stream); break;
  }
  if (st) return st;
  const int64_t total = batch * n_samples;
  const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 1 << 20);
  hipLaunchKernelGGL(stft_overlap_add_kernel, dim3(grid), dim3(256), 0, S(stream), dF, n_samples, (int)n_fft, h,
                     frames, batch, 0, grad_x);
  return launch_status();
}

size_t ddsp_hip_spectral_loss_workspace_size(int64_t batch, int64_t n_samples, const int64_t* n_ffts,
                                             const int64_t* hops, int n_scales) {
  if (batch < 1 || n_samples < 1 || n_scales < 1 || !n_ffts || !hops) return 0;
  size_t blocks = 0, dF = 0;
  for (int i = 0; i < n_scales; ++i) {
    if (hops[i] < 1 || n_ffts[i] < 16 || n_ffts[i] > 4096) return 0;
    const int64_t frames = n_samples / hops[i] + 1;
    blocks += (size_t)loss_blocks(n_ffts[i], frames, batch);
    dF = std::max(dF, sizeof(float) * (size_t)batch * frames * n_ffts[i]);
  }
  const size_t head = ((2 * sizeof(double) * blocks + sizeof(int64_t) * (n_scales + 1) +
                        sizeof(double) * n_scales) + 255) & ~(size_t)255;
  return head + dF;
}

int ddsp_hip_spectral_loss(const float* target, const float* recon, int64_t batch, int64_t n_samples,
                           const int64_t* n_ffts, const int64_t* hops, int n_scales, float* loss, float* grad_recon,
                           void* workspace, size_t workspace_bytes, void* stream) {
  if (n_scales < 1 || !n_ffts || !hops || !loss || batch < 1) return DDSP_HIP_EINVAL;
  for (int i = 0; i < n_scales; ++i) {
    int st = check_stft(batch, n_samples, n_ffts[i], hops[i]);
    if (st) return st;
  }
  if (!target || !recon) return DDSP_HIP_EINVAL;
  const size_t need = ddsp_hip_spectral_loss_workspace_size(batch, n_samples, n_ffts, hops, n_scales);
  if (!workspace || workspace_bytes < need) return DDSP_HIP_EWORKSPACE;
  // workspace: partials (2 doubles per block, all scales) | block offsets | 1/count | dF
  size_t blocks = 0;
  int64_t offs[65];
  double inv_counts[64];
  if (n_scales > 64) return DDSP_HIP_ERANGE;
  offs[0] = 0;
  for (int i = 0; i < n_scales; ++i) {
    const int64_t frames = n_samples / hops[i] + 1;
    blocks += (size_t)loss_blocks(n_ffts[i], frames, batch);
    offs[i + 1] = (int64_t)blocks;
    inv_counts[i] = 1.0 / ((double)batch * (double)(n_ffts[i] / 2 + 1) * (double)frames);
  }
  char* w = reinterpret_cast<char*>(workspace);
  double* partials = reinterpret_cast<double*>(w);
  int64_t* d_offs = reinterpret_cast<int64_t*>(w + 2 * sizeof(double) * blocks);
  double* d_inv = reinterpret_cast<double*>(d_offs + n_scales + 1);
  const size_t head = ((2 * sizeof(double) * blocks + sizeof(int64_t) * (n_scales + 1) +
                        sizeof(double) * n_scales) + 255) & ~(size_t)255;
  float* dF = reinterpret_cast<float*>(w + head);
  if (hipMemcpyAsync(d_offs, offs, sizeof(int64_t) * (n_scales + 1), hipMemcpyHostToDevice, S(stream)) != hipSuccess ||
      hipMemcpyAsync(d_inv, inv_counts, sizeof(double) * n_scales, hipMemcpyHostToDevice, S(stream)) != hipSuccess)
    return DDSP_HIP_ELAUNCH;
  const int64_t total = batch * n_samples;
  const unsigned ola_grid = (unsigned)std::min<int64_t>((total + 255) / 256, 1 << 20);
  for (int i = 0; i < n_scales; ++i) {
    const int64_t n = n_ffts[i];
    const int h = (int)hops[i];
    const int frames = (int)(n_samples / h + 1);
    const float scale = (float)(1.0 / std::sqrt((double)n));
    const float inv_count = (float)inv_counts[i];
    double* part = partials + 2 * offs[i];
    const bool g = grad_recon != nullptr;
    int st;
    switch (n) {
      case 16: st = spectral_loss_launch<16>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 32: st = spectral_loss_launch<32>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 64: st = spectral_loss_launch<64>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 128: st = spectral_loss_launch<128>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 256: st = spectral_loss_launch<256>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 512: st = spectral_loss_launch<512>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 1024: st = spectral_loss_launch<1024>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      case 2048: st = spectral_loss_launch<2048>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
      default: st = spectral_loss_launch<4096>(target, recon, batch, n_samples, h, frames, scale, inv_count, g, part, dF, stream); break;
    }
    if (st) return st;
    if (g) {
      hipLaunchKernelGGL(stft_overlap_add_kernel, dim3(ola_grid), dim3(256), 0, S(stream), dF, n_samples, (int)n, h,
                         frames, batch, i > 0 ? 1 : 0, grad_recon);
      if ((st = launch_status())) return st;
    }
  }
  hipLaunchKernelGGL(spectral_loss_finish_kernel, dim3(1), dim3(256), 0, S(stream), partials, d_offs, d_inv, n_scales,
                     loss);
  return launch_status();
}

}  // extern "C"
