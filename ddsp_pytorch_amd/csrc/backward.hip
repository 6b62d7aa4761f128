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
#include <cstdlib>

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
// Per-frame backward of the synthesis section, one workgroup per (item, frame).
//
// Harmonic part (HMODE 1: frame controls amp[B,F], normalised dist[B,F,H] -> d_amp, d_dist;
// HMODE 2: raw projection param[B,F,H+1] -> d_param): item (kq, s) of the ceil(H/4) x NS grid
// sums g_t sin(w_t (k+1)) for the 4 harmonics k = 4kq..4kq+3 over segment s of the frame's
// samples — one LDS read of the (w_t, g_t) pair feeds 4 sine chains, and all lanes of a wave read
// the same pair (broadcast).
//
// Noise part (NOISE 1: injected noise, 2: Philox regenerated with the forward's counters;
// RAW: magnitudes are the raw projection, scale_function(m + bias) differentiated too):
//   dh at the n filter taps by direct correlation of g with the frame's noise — register-blocked
//   4 taps x 4 lags per step when n/2 % 4 == 0 and n <= bs (the long taps j < n/2 split into
//   NSEG lag segments, the short wrapped taps one segment each, so the work is even), else one
//   tap per item; then the transposed filter design, a cosine transform of the windowed tap
//   gradients folded by the even symmetry of the IR (two threads per band) with the Nyquist band
//   from an alternating block sum.
// With both parts (the backward of ddsp_hip_synth_frames) the noise's short LDS phases run beside
// other workgroups' sine loops, as in the fused forward.
constexpr int kKPT = 4;  // harmonics per thread

// sine-loop placement padding per instantiation (tools/loop_align.py)
template <int HMODE, int NOISE>
constexpr bool kBwdLoopPad = false;

template <int HMODE, int NOISE, bool RAW>
__global__ void __launch_bounds__(512) frame_backward_kernel(
    const float* __restrict__ f0, const float* __restrict__ grad, const float* __restrict__ param,
    const float* __restrict__ amp, const float* __restrict__ dist, float* __restrict__ d_param,
    float* __restrict__ d_amp, float* __restrict__ d_dist, int F, int H, int bs, float sr, int NS,
    const float* __restrict__ mags, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0,
    uint32_t off1, float bias, float* __restrict__ d_mags, int NB, int NSEG) {
  extern __shared__ float smem[];
  __shared__ double red[32];
  __shared__ double red2[32];
  __shared__ int fast_s;
  constexpr bool HARM = HMODE != 0;
  constexpr bool PARAMS = HMODE == 2;
  // LDS layout (mirrored by frame_backward_lds_floats): xl and gl start 16-B aligned
  // the NS sample segments are SL samples each (even, NS * SL >= bs; (omega, g) = 0 past bs adds exact
  // zeros), so every thread's sine loop has the same scalar trip count: no per-lane exit masks (4 VALU per
  // 8 sines before; 152 -> 146.5-147.7 us at config 2, same box, tools/ab_prof.sh bwd)
  const int SL = ((bs + NS - 1) / NS + 1) & ~1, WGN = NS * SL;
  const int hfl = HARM ? 2 * WGN + NS * H + H : 0;
  // (omega_t, g_t) per sample
  float2* wg = reinterpret_cast<float2*>(smem);  // [WGN]
  float* part = smem + 2 * WGN;                  // [NS * H]
  float* uk = part + NS * H;                     // [H] u_k (PARAMS: v_k first)
  const int n = NOISE ? 2 * (NB - 1) : 0, half = n >> 1;
  const int qmax = min(n, bs);
  const bool quads = NOISE && (half % 4 == 0) && n <= bs && (bs % 4 == 0);
  // quads: segment rows n + 4 floats apart, so the rows of one wave's segments start on different banks
  // (48.1-48.2 -> 47.2-47.5 us for the noise VJP at config 2, same box)
  const int npart_len = NSEG * (quads ? n + 4 : qmax);
  float* xl = smem + ((hfl + 3) & ~3);                              // [bs] noise
  float* ct = xl + bs;                                               // [n] cos(2 pi q / n)
  float* e = ct + n;                                                 // [n] windowed tap gradients
  float* npart = e + n;                                              // [npart_len]
  float* gl = smem + (((xl - smem) + bs + 2 * n + npart_len + 3) & ~3);  // [bs + 8] g, zero-padded
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, NT = blockDim.x;
  const int64_t frame = (int64_t)b * F + f;
  const float* gf = grad + frame * bs;

  // ---- phase 1: loads ----
  double part_s = 0.0, part_d = 0.0;
  float pitch0 = 0.0f;
  const float half_sr = sr * 0.5f;
  const float* prow = PARAMS ? param + frame * (H + 1) : nullptr;
  if (HARM) {
    const float* f0b = f0 + (int64_t)b * F;
    pitch0 = f0b[f];
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
    for (int j = tid; j < WGN; j += NT) wg[j].y = j < bs ? gf[j] : 0.0f;
  }
  if (NOISE) {
    for (int j = tid; j < bs + 8; j += NT) gl[j] = j < bs ? gf[j] : 0.0f;
    if (NOISE == 2) {
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
  }
  if (HARM) block_sum_double2(part_s, part_d, red);  // (the noise part needs only the barrier below)

  // ---- phase 2: phases, normalised distribution ----
  const double S0 = part_s;
  const float norm = (float)part_d;
  float a = 0.0f;
  if (HARM) {
    const double dinc = (double)phase_inc(pitch0, sr);
    for (int j = tid; j < WGN; j += NT) wg[j].x = j < bs ? (float)(S0 + (double)(j + 1) * dinc) : 0.0f;
    a = PARAMS ? scale_fn(prow[0]) : amp[frame];
    if (PARAMS)
      for (int k = tid; k < H; k += NT) uk[k] = uk[k] / norm;
    if (tid == 0) {
      const float w0 = (float)(S0 + dinc), w1 = (float)(S0 + (double)bs * dinc);
      fast_s = fmaxf(fabsf(w0), fabsf(w1)) * (float)H < kFastArgLimit;
    }
  }
  __syncthreads();

  // Roles: with both parts the last wave does the noise VJP while the others run the sine
  // loops (wave specialisation: the noise wave's LDS latency hides under the sine waves' VALU
  // work); otherwise every thread works on the one part.
  constexpr bool SPEC = HARM && NOISE != 0;
  const int NTH = SPEC ? NT - 64 : NT;  // harmonic threads
  const bool hthread = !SPEC || tid < NTH;
  const int ntid = SPEC ? tid - NTH : tid, NTN = SPEC ? 64 : NT;  // noise thread id / count
  const bool nthread = NOISE && (!SPEC || tid >= NTH);

  // ---- phase 3a: harmonic dA_k = sum_t g_t sin(w_t (k+1)) ----
  if (HARM && hthread) {
    const int KQ = (H + kKPT - 1) / kKPT;
    for (int item = tid; item < KQ * NS; item += NTH) {
      const int s = item / KQ, kq = item - s * KQ;
      const int j0 = s * SL, j1 = min(j0 + SL, bs);
      float kf[kKPT], acc[kKPT];
#pragma unroll
      for (int c = 0; c < kKPT; ++c) {
        kf[c] = (float)(kKPT * kq + c + 1);
        acc[c] = 0.0f;
      }
      if (fast_s) {
        float acc2[kKPT];
#pragma unroll
        for (int c = 0; c < kKPT; ++c) acc2[c] = 0.0f;
        // loop placement (tools/loop_align.py, pinned by tests/test_loop_align.py): the
        // 8-byte instructions at odd dword addresses; the alignment point makes the placement
        // independent of the code laid out before the loop, the s_nop flips it per instantiation
        if constexpr (kBwdLoopPad<HMODE, NOISE>) asm volatile(".p2align 3\n s_nop 0");
        else asm volatile(".p2align 3");
        const float2* wq = wg + j0;
        for (int i = 0; i < SL; i += 2) {  // two samples per iteration: 8 independent sine chains
          const float2 p = wq[i], p1 = wq[i + 1];
          // the 8 chains written stage by stage so the scheduler keeps them interleaved (ILP 8)
          float y[2 * kKPT];
#pragma unroll
          for (int c = 0; c < kKPT; ++c) {
            y[c] = reduce_rev(p.x * kf[c]);
            y[kKPT + c] = reduce_rev(p1.x * kf[c]);
          }
#pragma unroll
          for (int c = 0; c < kKPT; ++c) {
            acc[c] = fmaf(p.y, sin_rev(y[c]), acc[c]);
            acc2[c] = fmaf(p1.y, sin_rev(y[kKPT + c]), acc2[c]);
          }
        }
#pragma unroll
        for (int c = 0; c < kKPT; ++c) acc[c] += acc2[c];
      } else {
        for (int j = j0; j < j1; ++j) {
          const float2 p = wg[j];
#pragma unroll
          for (int c = 0; c < kKPT; ++c) {
            const float x = p.x * kf[c];
            acc[c] = fmaf(p.y, fabsf(x) < kFastArgLimit ? sin_reduced(x) : sin_slow(x), acc[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < kKPT; ++c)
        if (kKPT * kq + c < H) part[s * H + kKPT * kq + c] = acc[c];
    }
  }

  // ---- phase 3b: the noise VJP (all of it on the noise threads) ----
  float alt = 0.0f;  // sum_q (-1)^q e[q]  (the Nyquist band)
  if (nthread) {
    // local barrier of the noise threads: one wave (LDS is in order per wave) or the workgroup
    auto nsync = [&]() {
      if (SPEC) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
      } else {
        __syncthreads();
      }
    };
    // dh[j(q)] = sum_d g[j+d] x[d]
    if (quads) {
      const int nqh = n >> 3;  // quads per half: long (q >= n/2, taps j < n/2) and short
      const int seglen = ((bs + NSEG - 1) / NSEG + 3) & ~3;
      for (int item = ntid; item < nqh * NSEG + nqh; item += NTN) {
        int q0, j0, d0, d1, seg;
        if (item < nqh * NSEG) {  // long taps: lag range [0, bs - j0) in NSEG segments
          seg = item / nqh;
          q0 = half + 4 * (item - seg * nqh);
          j0 = q0 - half;
          d0 = seg * seglen;
          d1 = min(d0 + seglen, bs - j0);
        } else {  // short (wrapped) taps j0 >= bs - n/2: one segment
          seg = 0;
          q0 = 4 * (item - nqh * NSEG);
          j0 = q0 - half + bs;
          d0 = 0;
          d1 = bs - j0;
        }
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (d0 < d1) {
          float4 gc = *reinterpret_cast<const float4*>(gl + j0 + d0);
          int d = d0;
          // 8 lags per iteration with the g window ping-ponged between two registers sets (no window
          // moves) and a second accumulator set (8 independent FMA chains), summed at the end
          float4 acc2 = make_float4(0.f, 0.f, 0.f, 0.f);
          for (; d + 8 <= d1; d += 8) {
            const float4 xv = *reinterpret_cast<const float4*>(xl + d);
            const float4 xw = *reinterpret_cast<const float4*>(xl + d + 4);
            const float4 gn = *reinterpret_cast<const float4*>(gl + j0 + d + 4);
            const float4 gm = *reinterpret_cast<const float4*>(gl + j0 + d + 8);
            acc.x = fmaf(gc.x, xv.x, fmaf(gc.y, xv.y, fmaf(gc.z, xv.z, fmaf(gc.w, xv.w, acc.x))));
            acc.y = fmaf(gc.y, xv.x, fmaf(gc.z, xv.y, fmaf(gc.w, xv.z, fmaf(gn.x, xv.w, acc.y))));
            acc.z = fmaf(gc.z, xv.x, fmaf(gc.w, xv.y, fmaf(gn.x, xv.z, fmaf(gn.y, xv.w, acc.z))));
            acc.w = fmaf(gc.w, xv.x, fmaf(gn.x, xv.y, fmaf(gn.y, xv.z, fmaf(gn.z, xv.w, acc.w))));
            acc2.x = fmaf(gn.x, xw.x, fmaf(gn.y, xw.y, fmaf(gn.z, xw.z, fmaf(gn.w, xw.w, acc2.x))));
            acc2.y = fmaf(gn.y, xw.x, fmaf(gn.z, xw.y, fmaf(gn.w, xw.z, fmaf(gm.x, xw.w, acc2.y))));
            acc2.z = fmaf(gn.z, xw.x, fmaf(gn.w, xw.y, fmaf(gm.x, xw.z, fmaf(gm.y, xw.w, acc2.z))));
            acc2.w = fmaf(gn.w, xw.x, fmaf(gm.x, xw.y, fmaf(gm.y, xw.z, fmaf(gm.z, xw.w, acc2.w))));
            gc = gm;
          }
          for (; d + 4 <= d1; d += 4) {
            const float4 xv = *reinterpret_cast<const float4*>(xl + d);
            const float4 gn = *reinterpret_cast<const float4*>(gl + j0 + d + 4);
            acc.x = fmaf(gc.x, xv.x, fmaf(gc.y, xv.y, fmaf(gc.z, xv.z, fmaf(gc.w, xv.w, acc.x))));
            acc.y = fmaf(gc.y, xv.x, fmaf(gc.z, xv.y, fmaf(gc.w, xv.z, fmaf(gn.x, xv.w, acc.y))));
            acc.z = fmaf(gc.z, xv.x, fmaf(gc.w, xv.y, fmaf(gn.x, xv.z, fmaf(gn.y, xv.w, acc.z))));
            acc.w = fmaf(gc.w, xv.x, fmaf(gn.x, xv.y, fmaf(gn.y, xv.z, fmaf(gn.z, xv.w, acc.w))));
            gc = gn;
          }
          acc.x += acc2.x;
          acc.y += acc2.y;
          acc.z += acc2.z;
          acc.w += acc2.w;
          for (; d < d1; ++d) {  // g is zero past bs, so taps c > 0 need no separate bound
            const float xv = xl[d];
            acc.x = fmaf(gl[j0 + d], xv, acc.x);
            acc.y = fmaf(gl[j0 + d + 1], xv, acc.y);
            acc.z = fmaf(gl[j0 + d + 2], xv, acc.z);
            acc.w = fmaf(gl[j0 + d + 3], xv, acc.w);
          }
        }
        float* dst = npart + seg * (n + 4) + q0;
        dst[0] = acc.x;
        dst[1] = acc.y;
        dst[2] = acc.z;
        dst[3] = acc.w;
      }
    } else {
      for (int item = ntid; item < qmax * NSEG; item += NTN) {
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
        npart[seg * qmax + q] = c0 + c1;
      }
    }
    nsync();
    // e[q] = dh[j(q)] hann[q]; the alternating sum for the Nyquist band
    double alt_part = 0.0;
    for (int q = ntid; q < n; q += NTN) {
      float v = 0.0f;
      if (q < qmax) {
        if (quads) {
          const int ns_q = q >= half ? NSEG : 1;
          for (int s = 0; s < ns_q; ++s) v += npart[s * (n + 4) + q];
        } else {
          for (int s = 0; s < NSEG; ++s) v += npart[s * qmax + q];
        }
        v *= 0.5f - 0.5f * ct[q];  // periodic Hann(n) at q
      }
      e[q] = v;
      alt_part += (q & 1) ? -(double)v : (double)v;
    }
    if (SPEC) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) alt_part += __shfl_xor(alt_part, o, 64);
    } else {
      alt_part = block_sum_double(alt_part, red2);  // includes the barrier publishing e[]
    }
    alt = (float)alt_part;
    nsync();
    // dA_k = (c_k/n)(-1)^k [e0 + (-1)^k e_half + sum_{q=1}^{half-1} (e_q + e_{n-q}) cos(2 pi q k/n)],
    // k < half on two threads (q halves) each; k = half from the alternating sum.
    float* dAp = npart;  // [2][half] (npart is consumed)
    const int mid = (half + 1) >> 1;
    const bool pow2 = (n & (n - 1)) == 0;
    for (int item = ntid; item < 2 * half; item += NTN) {
      const int pr = item / half, k = item - pr * half;
      const int q0 = pr ? mid : 1, q1 = pr ? half : mid;
      float s0 = 0.0f, s1 = 0.0f;
      if (pow2) {
        const int mask = n - 1;
        int q = q0;
        for (; q + 1 < q1; q += 2) {
          s0 = fmaf(e[q] + e[n - q], ct[(q * k) & mask], s0);
          s1 = fmaf(e[q + 1] + e[n - q - 1], ct[((q + 1) * k) & mask], s1);
        }
        if (q < q1) s0 = fmaf(e[q] + e[n - q], ct[(q * k) & mask], s0);
      } else {
        int qk = (int)(((int64_t)q0 * k) % n);
        for (int q = q0; q < q1; ++q) {
          s0 = fmaf(e[q] + e[n - q], ct[qk], s0);
          qk += k;
          if (qk >= n) qk -= n;
        }
      }
      float v = s0 + s1;
      if (pr == 0) v += e[0] + ((k & 1) ? -e[half] : e[half]);
      dAp[pr * half + k] = v;
    }
    nsync();
    const float inv_n = 1.0f / (float)n;
    for (int k = ntid; k < NB; k += NTN) {
      float dA = k < half ? (dAp[k] + dAp[half + k]) * (k == 0 ? 1.0f : 2.0f) * inv_n : alt * inv_n;
      if (k & 1) dA = -dA;
      d_mags[frame * NB + k] = RAW ? dA * scale_fn_grad(mags[frame * NB + k] + bias) : dA;
    }
  }

  if (HARM) {
    // ---- phase 4: harmonic reductions and outputs ----
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
}

// ---------------------------------------------------------------------------------------
// The noise VJP alone (FilteredNoise's backward, modules.py:116-128) at the reference's 65 bands
// (n = 128 filter taps) and bs % 128 == 0, bs >= 512: one WAVE per frame, no workgroup barrier after the
// cosine table.
//   dh[j] = sum_d g[j + d] x[d] for the taps the filter has: j in [0, 64) (lags < bs - j) and
//   j in [bs - 64, bs) (lags < bs - j <= 64).  g is zero-padded past bs, so every lane runs a fixed
//   rectangle: the long taps as 8 tap groups x 8 lag segments of L = bs/8 lags (8 taps x 4 lags per
//   ds_read_b128 of g and one of x: 32 FMAs per two reads), the short taps as 8 tap groups x 8 segments
//   of 8 lags.
//   Bank-conflict-free LDS reads: ds_read_b128 serves a wave in four 16-lane groups (MI355X_MICROARCH.md
//   §LDS); each group holds the 8 tap groups of two lag segments (kNvjpLane), and every segment reads its
//   own copy of its g window [sL, sL + L + 72) and its own x run, at strides of L + 76 and L + 4 floats
//   (= 4 mod 8): the two segments of a group fall on disjoint bank halves.  (A first form with one shared
//   g array and x at 64-float segment strides ran 51 us at config 2: 4- and 8-way conflicts.)
//   e[q] = dh[j(q)] hann[q] (q >= 64: j = q - 64; q < 64: j = q - 64 + bs), then
//   dA_k = (c_k / n)(-1)^k [e_0 + (-1)^k e_64 + sum_{q=1}^{63} s_q cos(2 pi q k / n)] for k < 64 with the
//   folded sums s_q = e_q + e_{n-q}, and the Nyquist band k = 64 from the alternating sum (as
//   frame_backward_kernel).
constexpr int kNvjpWaves = 4;  // frames per workgroup
__host__ __device__ constexpr int nvjp_gstride(int L) { return L + 76; }
__host__ __device__ constexpr int nvjp_xstride(int L) { return L + 4; }
__host__ __device__ constexpr int nvjp_wave_floats(int bs) {
  return 8 * nvjp_gstride(bs / 8) + 8 * nvjp_xstride(bs / 8) + 192;
}
// lane -> 16 * (lag segment pair) + 8 * (segment in the pair) + tap group, so that the lanes of each
// ds_read_b128 group {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32) are the 16 (segment, tap group) of one
// segment pair
__device__ constexpr unsigned char kNvjpLane[64] = {
    0,  1,  2,  3,  16, 17, 18, 19, 20, 21, 22, 23, 4,  5,  6,  7,  24, 25, 26, 27, 8,  9,  10, 11,
    12, 13, 14, 15, 28, 29, 30, 31, 32, 33, 34, 35, 48, 49, 50, 51, 52, 53, 54, 55, 36, 37, 38, 39,
    56, 57, 58, 59, 40, 41, 42, 43, 44, 45, 46, 47, 60, 61, 62, 63};

// acc[i] += sum_{d < 16 NQ4} g[i + d] x[d], i < 8, with g4 / x4 at the lane's window: per 4 lags one
// ds_read_b128 of x and one of g (a 4-quad register ring, indexed statically in the unrolled body)
template <int NQ4>
__device__ __forceinline__ void corr8(const float4* __restrict__ g4, const float4* __restrict__ x4, float (&acc)[8]) {
  float4 w[4];
  w[0] = g4[0];
  w[1] = g4[1];
  w[2] = g4[2];
#pragma unroll  // fully: a loop-carried ring was scalarised into ds_read2_b32 pairs
  for (int c = 0; c < NQ4; ++c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 xv = x4[4 * c + k];
      w[(k + 3) & 3] = g4[4 * c + k + 3];
      const float4 a = w[k & 3], b = w[(k + 1) & 3], e = w[(k + 2) & 3];
      const float win[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, e.x, e.y, e.z, e.w};
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int l = 0; l < 4; ++l) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(win[i + l], xs[l], acc[i]);
      }
    }
  }
}

template <int NOISE, bool RAW>
__global__ void __launch_bounds__(64 * kNvjpWaves) noise_vjp_wave_kernel(
    const float* __restrict__ grad, const float* __restrict__ mags, const float* __restrict__ noise, uint32_t k0,
    uint32_t k1, uint32_t off0, uint32_t off1, float bias, float* __restrict__ d_mags, int64_t frames, int bs) {
  constexpr int n = 128, half = 64, NB = 65;
  extern __shared__ float4 smem_nv[];
  float* ct = reinterpret_cast<float*>(smem_nv);  // [n]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t frame = (int64_t)blockIdx.x * kNvjpWaves + wave;
  const int L = bs >> 3, Sg = nvjp_gstride(L), Sx = nvjp_xstride(L);
  // the g windows' quads (<= 7 per lane at bs <= 1024) are loaded first: their HBM latency hides under the
  // cosine table, the barrier and the Philox noise
  const float* gf = grad + (frame < frames ? frame : 0) * bs;
  const int wq = (L + 72) >> 2;  // quads per window
  float4 gq[7];
  int gdst[7];  // the quad's float offset in the window copies (-1: none)
  const float rwq = 1.0f / (float)wq;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int i = lane + 64 * r;
    int s = (int)((float)i * rwq);  // i / wq (i < 512: the float quotient is within one of it)
    s += (s + 1) * wq <= i;
    s -= s * wq > i;
    const int u = s * L + 4 * (i - s * wq);
    gdst[r] = i < 8 * wq ? s * Sg + (u - s * L) : -1;
    gq[r] = (i < 8 * wq && u < bs) ? *reinterpret_cast<const float4*>(gf + u) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  fill_cos_table(ct, n);
  __syncthreads();
  if (frame >= frames) return;
  float* gc = ct + n + wave * nvjp_wave_floats(bs);  // [8][Sg] window copies of g (zero past bs)
  float* xc = gc + 8 * Sg;                           // [8][Sx] the noise, one run per lag segment
  float* es = xc + 8 * Sx;                           // [128] e, then [64] s
  auto wsync = [] {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };

  // ---- the frame's noise, then the 8 windows of g (the upstream gradient of the frame) ----
  const int quads = bs >> 2;
  for (int t = lane; t < quads; t += 64) {
    float4 v;
    if (NOISE == 2) {  // the forward's Philox stream (synth_frame.hip / noise.hip counter layout)
      const uint64_t qc = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 r = philox4x32_10((uint32_t)qc, (uint32_t)(qc >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(r.v[0]), uniform_pm1(r.v[1]), uniform_pm1(r.v[2]), uniform_pm1(r.v[3]));
    } else {
      v = *reinterpret_cast<const float4*>(noise + frame * bs + 4 * t);
    }
    const int s = (4 * t) / L;
    *reinterpret_cast<float4*>(xc + s * Sx + (4 * t - s * L)) = v;
  }
#pragma unroll
  for (int r = 0; r < 7; ++r)
    if (gdst[r] >= 0) *reinterpret_cast<float4*>(gc + gdst[r]) = gq[r];
  wsync();

  // ---- correlation ----
  const int m = kNvjpLane[lane];
  const int tg = m & 7, seg = m >> 3;
  float accL[8], accS[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) accL[i] = accS[i] = 0.0f;
  {
    // long taps j = 8 tg + i, lags [seg L, seg L + L): window copy seg at offset 8 tg
    const float4* g4 = reinterpret_cast<const float4*>(gc + seg * Sg + 8 * tg);
    const float4* x4 = reinterpret_cast<const float4*>(xc + seg * Sx);
    int c = 0;
    for (; c + 64 <= L; c += 64) corr8<4>(g4 + c / 4, x4 + c / 4, accL);  // (L = 64 at bs = 512: one call)
    if (L & 32) {
      corr8<2>(g4 + c / 4, x4 + c / 4, accL);
      c += 32;
    }
    if (L & 16) corr8<1>(g4 + c / 4, x4 + c / 4, accL);
  }
  {
    // short taps j = bs - 64 + 8 tg + i, lags [8 seg, 8 seg + 8): in window copy 7 (which starts at bs - L)
    const float4* g4 = reinterpret_cast<const float4*>(gc + 7 * Sg + (L - 64) + 8 * tg + 8 * seg);
    const float4* x4 = reinterpret_cast<const float4*>(xc + 8 * seg);
    const float4 w0 = g4[0], w1 = g4[1], w2 = g4[2], w3 = g4[3];
    const float4 x0 = x4[0], x1 = x4[1];
    const float win[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
    const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int l = 0; l < 8; ++l) {
#pragma unroll
      for (int i = 0; i < 8; ++i) accS[i] = fmaf(win[i + l], xs[l], accS[i]);
    }
  }
  wsync();  // every lane's g / x reads are done: the partials overwrite the g windows
  float* partL = gc;        // [8 seg][64 taps]
  float* partS = gc + 512;  // [8 seg][64 taps]
  *reinterpret_cast<float4*>(partL + seg * 64 + 8 * tg) = make_float4(accL[0], accL[1], accL[2], accL[3]);
  *reinterpret_cast<float4*>(partL + seg * 64 + 8 * tg + 4) = make_float4(accL[4], accL[5], accL[6], accL[7]);
  *reinterpret_cast<float4*>(partS + seg * 64 + 8 * tg) = make_float4(accS[0], accS[1], accS[2], accS[3]);
  *reinterpret_cast<float4*>(partS + seg * 64 + 8 * tg + 4) = make_float4(accS[4], accS[5], accS[6], accS[7]);
  wsync();

  // ---- e[q] (lane l: q = l, the short tap l; q = 64 + l, the long tap l) and the alternating sum ----
  float eS = 0.0f, eL = 0.0f;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    eS += partS[s * 64 + lane];
    eL += partL[s * 64 + lane];
  }
  eS *= 0.5f - 0.5f * ct[lane];
  eL *= 0.5f - 0.5f * ct[half + lane];
  es[lane] = eS;
  es[half + lane] = eL;
  double alt = (lane & 1) ? -(double)eS - (double)eL : (double)eS + (double)eL;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) alt += __shfl_xor(alt, o, 64);
  wsync();
  float* sq = es + n;  // [64] s_q = e_q + e_{n-q} (q >= 1)
  // stored by parity: sq[(q & 1) * 32 + (q >> 1)]
  sq[(lane & 1) * 32 + (lane >> 1)] = lane ? eS + es[n - lane] : 0.0f;
  wsync();

  // ---- cosine transform, folded: c(q (64 - k)) = (-1)^q c(q k), so with E_k / O_k the even- / odd-q halves of
  // sum_q s_q c(q k), dA'_k = E_k + O_k and dA'_{64-k} = E_k - O_k: lane l < 32 forms E_l, lane 32 + l forms O_l
  // (32 terms each instead of 63), and E_32 = sum_j s_{2j} (-1)^j (O_32 = 0) comes from a wave sum ----
  const int par = lane >> 5, kk = lane & 31;
  const float* sp = sq + 32 * par;
  const int step = (2 * kk) & (n - 1);
  int idx = (par * kk) & (n - 1);  // (q k) mod n for q = 2 j + par, j = 0
  float v0 = 0.0f, v1 = 0.0f;
#pragma unroll
  for (int j4 = 0; j4 < 8; ++j4) {
    const float4 s4 = *reinterpret_cast<const float4*>(sp + 4 * j4);
    const float c0 = ct[idx];
    idx = (idx + step) & (n - 1);
    const float c1 = ct[idx];
    idx = (idx + step) & (n - 1);
    const float c2 = ct[idx];
    idx = (idx + step) & (n - 1);
    const float c3 = ct[idx];
    idx = (idx + step) & (n - 1);
    v0 = fmaf(s4.x, c0, v0);  // (s_0 = 0)
    v1 = fmaf(s4.y, c1, v1);
    v0 = fmaf(s4.z, c2, v0);
    v1 = fmaf(s4.w, c3, v1);
  }
  const float half_sum = v0 + v1;                          // E_kk (par 0) or O_kk (par 1)
  const float other = __shfl_xor(half_sum, 32, 64);        // the partner half
  float e32 = par ? 0.0f : ((kk & 1) ? -sq[kk] : sq[kk]);  // s_{2 kk} (-1)^kk
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) e32 += __shfl_xor(e32, o, 64);  // within each 32-lane half
  const float E32 = __shfl(e32, 0, 64);  // (a wave op: every lane takes part)
  int k;
  float sum;
  if (!par) {  // k = kk: E + O
    k = kk;
    sum = half_sum + other;
  } else if (kk) {  // k = 64 - kk: E - O
    k = half - kk;
    sum = other - half_sum;
  } else {  // k = 32: E_32 (O_32 = 0)
    k = 32;
    sum = E32;
  }
  const float inv_n = 1.0f / (float)n;
  float dA = (sum + es[0] + ((k & 1) ? -es[half] : es[half])) * (k == 0 ? 1.0f : 2.0f) * inv_n;
  if (k & 1) dA = -dA;
  float* dm = d_mags + frame * NB;
  const float* mg = RAW ? mags + frame * NB : nullptr;
  dm[k] = RAW ? dA * scale_fn_grad(mg[k] + bias) : dA;
  if (lane == 0) {
    const float dN = (float)alt * inv_n;  // k = half (even)
    dm[half] = RAW ? dN * scale_fn_grad(mg[half] + bias) : dN;
  }
}

// LDS floats of frame_backward_kernel (its layout, written out on the host)
size_t frame_backward_lds_floats(bool harm, bool noise, int H, int bs, int NS, int NB, int NSEG) {
  const size_t SL = (size_t)(((bs + NS - 1) / NS + 1) & ~1);
  const size_t hfl = harm ? (size_t)2 * NS * SL + (size_t)NS * H + H : 0;
  if (!noise) return hfl;
  const int n = 2 * (NB - 1);
  const int qmax = std::min(n, bs);
  const bool quads = ((n / 2) % 4 == 0) && n <= bs && bs % 4 == 0;
  const size_t npart_len = (size_t)NSEG * (quads ? n + 4 : qmax);
  const size_t off_xl = (hfl + 3) & ~(size_t)3;
  const size_t off_gl = (off_xl + (size_t)bs + 2 * (size_t)n + npart_len + 3) & ~(size_t)3;
  return off_gl + (size_t)bs + 8;
}

// noise lag segments: per long tap quad on the register-blocked path, else per tap
int noise_nseg(int nt, int NB, int bs) {
  const int n = 2 * (NB - 1);
  const bool quads = ((n / 2) % 4 == 0) && n <= bs && bs % 4 == 0;
  if (quads) {
    const int nqh = n / 8;
    return std::max(1, std::min(16, (nt - nqh) / std::max(nqh, 1)));
  }
  return std::max(1, std::min(8, nt / std::max(std::min(n, bs), 1)));
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

// Harmonic backward geometry: NS sample segments so that ceil(H/4) x NS fills about
// kBwdThreads threads (small workgroups: several per CU hide each one's latency-bound phases).
constexpr int kBwdThreads = 128;  // measured best at config 2 (64..512 swept)
int bwd_threads() { return kBwdThreads; }

void harmonic_backward_shape(int H, int bs, int& nt, int& ns) {
  const int kq = (H + kKPT - 1) / kKPT;
  const int target = bwd_threads();
  ns = std::max(1, std::min(std::min(target / kq, bs), 64));
  nt = std::min(512, ((kq * ns + 63) / 64) * 64);
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

// hmode: 0 no harmonic part, 1 frame controls, 2 raw params; noise_mode: 0 none, 1 injected, 2 Philox
static int frame_backward_launch(int hmode, int noise_mode, bool raw, const float* f0, const float* grad,
                                 const float* param, const float* amp, const float* dist, float* d_param,
                                 float* d_amp, float* d_dist, int64_t batch, int64_t frames, int64_t H,
                                 int64_t bs, float sr, const float* mags, const float* noise, uint64_t seed,
                                 uint64_t offset, float bias, float* d_mags, int64_t NB, void* stream) {
  if (batch < 0 || frames < 0 || bs < 1 || (hmode && (H < 1 || !(sr > 0)))) return DDSP_HIP_EINVAL;
  if (noise_mode && NB < 2) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (batch > 65535 || frames > INT32_MAX || H > 4096 || bs > 8192 || NB > 4097) return DDSP_HIP_ERANGE;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
  // noise alone at the reference's 65 bands: one wave per frame (noise_vjp_wave_kernel)
  if (hmode == 0 && NB == 65 && bs % 128 == 0 && bs >= 512 && bs <= 1024 && ((uintptr_t)grad & 15) == 0 &&
      (noise_mode == 2 || ((uintptr_t)noise & 15) == 0)) {
    const int64_t rows = batch * frames;
    const dim3 grid((unsigned)((rows + kNvjpWaves - 1) / kNvjpWaves));
    const size_t shm = sizeof(float) * (128 + (size_t)kNvjpWaves * nvjp_wave_floats((int)bs));  // 29.7 KB at bs 512
#define DDSP_NVJP_LAUNCH(N_, R_)                                                                                \
  hipLaunchKernelGGL((noise_vjp_wave_kernel<N_, R_>), grid, dim3(64 * kNvjpWaves), shm, S(stream), grad, mags, \
                     noise, k0, k1, o0, o1, bias, d_mags, rows, (int)bs)
    if (noise_mode == 1) {
      if (raw) DDSP_NVJP_LAUNCH(1, true); else DDSP_NVJP_LAUNCH(1, false);
    } else {
      if (raw) DDSP_NVJP_LAUNCH(2, true); else DDSP_NVJP_LAUNCH(2, false);
    }
#undef DDSP_NVJP_LAUNCH
    return launch_status();
  }
  // noise alone: 128 threads per frame (config 2: 53.8 us; 64 threads 60.5, 256 threads 70.0)
  int nt = 128, ns = 1;
  if (hmode) harmonic_backward_shape((int)H, (int)bs, nt, ns);
  // both parts: one extra wave runs the noise VJP beside the sine waves
  const bool spec = hmode && noise_mode;
  const int nseg = noise_mode ? noise_nseg(spec ? 64 : nt, (int)NB, (int)bs) : 0;
  if (spec) nt += 64;
  const size_t shm = sizeof(float) * frame_backward_lds_floats(hmode != 0, noise_mode != 0, (int)H, (int)bs, ns,
                                                               (int)NB, nseg);
  if (shm > 150 * 1024) return DDSP_HIP_ERANGE;
  const dim3 grid((unsigned)frames, (unsigned)batch);
#define DDSP_FB_LAUNCH(HM_, N_, R_)                                                                         \
  hipLaunchKernelGGL((frame_backward_kernel<HM_, N_, R_>), grid, dim3(nt), shm, S(stream), f0, grad, param, amp, \
                     dist, d_param, d_amp, d_dist, (int)frames, (int)H, (int)bs, sr, ns, mags, noise, k0, k1,  \
                     o0, o1, bias, d_mags, (int)NB, nseg)
  if (hmode == 1 && noise_mode == 0) {
    DDSP_FB_LAUNCH(1, 0, false);
  } else if (hmode == 2 && noise_mode == 0) {
    DDSP_FB_LAUNCH(2, 0, false);
  } else if (hmode == 2 && noise_mode == 1 && raw) {
    DDSP_FB_LAUNCH(2, 1, true);
  } else if (hmode == 2 && noise_mode == 2 && raw) {
    DDSP_FB_LAUNCH(2, 2, true);
  } else if (hmode == 0 && noise_mode == 1) {
    if (raw) DDSP_FB_LAUNCH(0, 1, true); else DDSP_FB_LAUNCH(0, 1, false);
  } else if (hmode == 0 && noise_mode == 2) {
    if (raw) DDSP_FB_LAUNCH(0, 2, true); else DDSP_FB_LAUNCH(0, 2, false);
  } else {
    return DDSP_HIP_EINVAL;
  }
#undef DDSP_FB_LAUNCH
  return launch_status();
}

int ddsp_hip_harmonic_synth_frames_backward(const float* f0, const float* amplitudes, const float* distribution,
                                            const float* grad, float* grad_amplitudes,
                                            float* grad_distribution, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream) {
  if (!f0 || !amplitudes || !distribution || !grad || !grad_amplitudes || !grad_distribution)
    return batch == 0 || frames == 0 ? DDSP_HIP_OK : DDSP_HIP_EINVAL;
  return frame_backward_launch(1, 0, false, f0, grad, nullptr, amplitudes, distribution, nullptr, grad_amplitudes,
                               grad_distribution, batch, frames, n_harmonic, block_size, sample_rate, nullptr,
                               nullptr, 0, 0, 0.0f, nullptr, 0, stream);
}

int ddsp_hip_harmonic_synth_params_backward(const float* f0, const float* param, const float* grad,
                                            float* grad_param, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream) {
  if (!f0 || !param || !grad || !grad_param) return batch == 0 || frames == 0 ? DDSP_HIP_OK : DDSP_HIP_EINVAL;
  return frame_backward_launch(2, 0, false, f0, grad, param, nullptr, nullptr, grad_param, nullptr, nullptr, batch,
                               frames, n_harmonic, block_size, sample_rate, nullptr, nullptr, 0, 0, 0.0f, nullptr, 0,
                               stream);
}

int ddsp_hip_synth_frames_backward(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                                   const float* noise, uint64_t seed, uint64_t offset, const float* grad_harmonic,
                                   const float* grad_noise, float* grad_param, float* grad_magnitudes,
                                   int64_t batch, int64_t frames, int64_t n_harmonic, int64_t n_bands,
                                   int64_t block_size, float sample_rate, void* stream) {
  if (batch == 0 || frames == 0) return batch < 0 || frames < 0 ? DDSP_HIP_EINVAL : DDSP_HIP_OK;
  if (!f0 || !param || !raw_magnitudes || !grad_harmonic || !grad_param || !grad_magnitudes)
    return DDSP_HIP_EINVAL;
  // The two halves as two launches on the stream: measured faster than the one-launch form whose
  // extra wave ran the noise VJP beside the sine waves (config 2, tools/exp_bwd_split.py: 176.7 vs
  // 187.6-190.3 us; the halves alone 130.4 and 47.9 us, on two streams 223 us).
  int st = frame_backward_launch(2, 0, false, f0, grad_harmonic, param, nullptr, nullptr, grad_param, nullptr,
                                 nullptr, batch, frames, n_harmonic, block_size, sample_rate, nullptr, nullptr, 0,
                                 0, 0.0f, nullptr, 0, stream);
  if (st) return st;
  return ddsp_hip_filtered_noise_backward(raw_magnitudes, noise, seed, offset, 1, bias,
                                          grad_noise ? grad_noise : grad_harmonic, grad_magnitudes, batch, frames,
                                          n_bands, block_size, stream);
}

int ddsp_hip_filtered_noise_backward(const float* magnitudes, const float* noise, uint64_t seed, uint64_t offset,
                                     int raw, float bias, const float* grad, float* grad_magnitudes,
                                     int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                                     void* stream) {
  if (batch < 0 || frames < 0 || n_bands < 2 || block_size < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!grad || !grad_magnitudes || (raw && !magnitudes)) return DDSP_HIP_EINVAL;
  return frame_backward_launch(0, noise ? 1 : 2, raw != 0, nullptr, grad, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr, batch, frames, 0, block_size, 0.0f, magnitudes, noise, seed, offset, bias,
                               grad_magnitudes, n_bands, stream);
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
