// The synthesis section of DDSPDecoder.forward (decoder.py:106-121) for one frame in one
// workgroup: harmonic controls + oscillator bank (modules.py:44-80), noise controls + filter
// design + filtered noise (modules.py:111-128), and `signal = harmonic + noise`.
//
// Why fuse: the oscillator bank is VALU-bound (6 VALU ops + one hardware sine per sample x
// harmonic) while the filtered-noise work is short, LDS- and latency-heavy phases.  In one
// kernel the noise phases of some workgroups run beside the sine loops of others on the same
// CU, the harmonic signal never makes an HBM round trip, and one launch replaces two.
//
// Mapping: thread t owns samples [4t, 4t+4) of the frame for both parts (bs <= 1024,
// bs % 4 == 0), so the harmonic and noise values of a sample meet in registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <cstdlib>

#include "common.h"
#include "noise_dsp.h"
#include "fft_radix.h"
#include "upols.h"

namespace ddsp {
namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// The oscillator bank over the (k+1, amplitude) table for 4 samples: acc[s] += A_k sin(fl32(w_s (k+1)))
// in ascending k.  H4 % 4 == 0.  (A register double buffer of the next 4 coefficients was re-rolled by
// the compiler into load-then-use; forced through inline assembly it gained the compiler's own waits
// and 11-15 extra instructions per iteration: not kept.)
__device__ __forceinline__ void osc_bank4(const float2* __restrict__ coef, int H4, const float (&w)[4],
                                          float (&acc)[4]) {
#pragma unroll 4
  for (int k = 0; k < H4; ++k) {
    const float2 c = coef[k];
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[s] = fmaf(sin_reduced(w[s] * c.x), c.y, acc[s]);
  }
}

// SPLIT (few-frame launches, e.g. the realtime stream's 4 frames per call): the workgroup has
// G times the threads of one 4-samples-per-thread frame and the oscillator bank runs one sample
// per thread, so one frame's latency is spread over G times the waves.
//
// frame_synth: one frame (f, b) by a thread group of NT threads (tid in [0, NT), whole waves starting
// at wave w0 of the workgroup) in the LDS region smem4; every wave of the workgroup calls it (its
// barriers are workgroup barriers).  On return (true: the thread's samples j0..j0+3 are in the
// frame) acc = harmonic, nz = filtered noise.
// PAD: one s_nop ahead of the (non-SPLIT) sine loop where an instantiation needs it for the loop's fast
// placement (phase 5; the controls-writing instantiations).  CTRL: also write the frame's controls
// (the dicts DDSPDecoder.forward returns) to ctrl_out.
template <bool RNG, bool SPLIT, bool PAD, bool CTRL>
__device__ __forceinline__ bool frame_synth(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float* __restrict__ ctrl_out, int B, int F, int H, int NB, int bs,
    float sr, int lo_end, int tail_start, int pad, int f, int b, int tid, int NT, float4* smem4, double* red,
    int w0, float (&acc)[4], float (&nz)[4], int& j0_out, int ldp, int ldm) {
  const int n = 2 * (NB - 1), half = n >> 1, n4 = (n + 3) & ~3;
  const int H4 = (H + 3) & ~3;
  float2* coef = reinterpret_cast<float2*>(smem4);       // [H4] (k+1, amplitude)
  float* ct = reinterpret_cast<float*>(coef + H4);       // [n4]
  float* A = ct + n4;                                     // [NB -> 4]
  float* ir = A + ((NB + 3) & ~3);                        // [half+1 -> 4]
  float* h = ir + ((half + 4) & ~3);                      // [bs]
  float* tail = h + bs;                                   // [half -> 4]
  float* xbuf = tail + ((half + 3) & ~3);                 // [pad zeros | bs samples]
  float* x = xbuf + pad;

  const int64_t frame = (int64_t)b * F + f;
  const float* f0b = f0 + (int64_t)b * F;
  const float* prow = param + frame * ldp;
  const float half_sr = sr * 0.5f;
  const float pitch0 = f0b[f];

  // ---- phase 1: independent loads and per-element work ----
  double part_s = 0.0, part_d = 0.0;
#ifdef DDSP_PROBE_NO_PREFIX
  if (false)
#endif
  for (int g = tid; g < f; g += NT) part_s += (double)bs * (double)phase_inc(f0b[g], sr);
  // the frame's H + NB + 1 scale_function values as one work list (item i at thread i mod NT, in
  // ascending i, so the distribution's partial sums keep their order): harmonic distribution
  // (modules.py:53-60 before normalisation), noise magnitudes (modules.py:113), then the amplitude
  // (modules.py:52), published through tail[0], which phase 4 overwrites only after it is read
  for (int i = tid; i < H + NB + 1; i += NT) {
    const float* src = i < H ? prow + 1 + i : (i < H + NB ? mags + frame * ldm + (i - H) : prow);
    const float raw = *src;
    const float sv = scale_fn(i >= H && i < H + NB ? raw + bias : raw);
    if (i < H) {
      const float v = sv * ((pitch0 * (float)(i + 1)) < half_sr ? kOnePlusEps : kEps);  // controls_value
      coef[i].y = v;
      part_d += (double)v;
    } else if (i < H + NB) {
      A[i - H] = sv;
    } else {
      tail[0] = sv;
    }
  }
  fill_cos_table(ct, n, tid, NT);
  for (int i = tid; i < pad; i += NT) xbuf[i] = 0.0f;
  const int quads = bs >> 2;
  if (RNG && counter) {  // graph-replayed streams: the Philox offset advances in device memory
    const uint64_t o = (((uint64_t)off1 << 32) | off0) + *counter;
    off0 = (uint32_t)o;
    off1 = (uint32_t)(o >> 32);
  }
  for (int t = tid; t < quads; t += NT) {
    float4 v;
    if (RNG) {
      const uint64_t q = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(r.v[0]), uniform_pm1(r.v[1]), uniform_pm1(r.v[2]), uniform_pm1(r.v[3]));
    } else {
      v = *reinterpret_cast<const float4*>(noise + frame * bs + 4 * t);
    }
    *reinterpret_cast<float4*>(x + 4 * t) = v;
  }
  group_sum_double2(part_s, part_d, red, w0, NT >> 6);  // includes the barrier that publishes phase 1
  const double S = part_s;                 // exact fp64 prefix over earlier frames
  const float norm = (float)part_d;        // dist.sum(-1)
  const float a = tail[0];                 // scale_function(amplitude)

  // ---- phase 2: harmonic coefficient table; even half of the noise filter taps ----
  for (int k = tid; k < H4; k += NT) {
    const float v = k < H ? (coef[k].y / norm) * a : 0.0f;  // (dist / sum) * amp
    coef[k] = make_float2((float)(k + 1), v);
  }
  if (n == 128 && NT >= 128) {
    if (tid < 64) {
      const int m = tid;
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 8
      for (int k = 1; k < 63; k += 2) {
        s0 = fmaf(A[k], kIrCos128[k * 64 + m], s0);
        s1 = fmaf(A[k + 1], kIrCos128[(k + 1) * 64 + m], s1);
      }
      s0 = fmaf(A[63], kIrCos128[63 * 64 + m], s0);
      ir[m] = (A[0] + ((m & 1) ? -A[64] : A[64]) + 2.0f * (s0 + s1)) * (1.0f / 128.0f);
    } else if (tid < 128) {  // tap n/2: cos(pi k) = (-1)^k
      float alt = (tid - 64 >= 1 && tid - 64 < 64) ? (((tid - 64) & 1) ? -A[tid - 64] : A[tid - 64]) : 0.0f;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) alt += __shfl_xor(alt, o, 64);
      if (tid == 64) ir[64] = (A[0] + A[64] + 2.0f * alt) * (1.0f / 128.0f);
    }
  } else {
    for (int m = tid; m <= half; m += NT) ir[m] = irfft_tap(A, ct, n, m);
  }
  __syncthreads();

  // ---- phase 3: rolled/windowed filter h (core.py:158-164) ----
  // only the taps the FIR reads: [0, lo_end) and [tail_start, bs) (the rest are zero)
  const int nlo = lo_end, ntaps = lo_end + (bs - tail_start);
  for (int i = tid; i < ntaps; i += NT) {
    const int j = i < nlo ? i : tail_start + (i - nlo);
    h[j] = ir_at_half(ir, ct, n, bs, j);
  }
  if (bs - tail_start == 64 && bs - 127 >= lo_end && tid < 63) h[tail_start - 63 + tid] = 0.0f;  // phase 4's padding
  __syncthreads();

  // ---- phase 4: noise tail (taps past bs - n/2 reach only the last n/2 outputs) ----
#ifdef DDSP_PROBE_NO_TAIL
  if (false)
#endif
  // with n/2 = 64 (65 bands) and h zero for the 63 positions below tail_start (written in phase 3) every
  // lane runs the same 64 taps, unrolled with no per-tap predication: the taps past l add fma(0, x, c) = c,
  // the others come in tap order, so the sums are the loop's below (measured 1.2 % faster)
  if (bs - tail_start == 64 && bs - 127 >= lo_end) {
    for (int l = tid; l < 64; l += NT) {
      const float* hj = h + tail_start + l;
      float c = 0.0f;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) c = fmaf(hj[-d], x[d], c);
      tail[l] = c;
    }
  } else
  for (int l = tid; l < bs - tail_start; l += NT) {
    const int j = tail_start + l;
    float c = 0.0f;
    for (int d = 0; d <= l; ++d) c = fmaf(h[j - d], x[d], c);
    tail[l] = c;
  }

  // ---- phase 5: oscillator bank for samples [j0, j0+4) ----
  const int j0 = 4 * tid;
  const bool active = j0 < bs;
  const double dinc = (double)phase_inc(pitch0, sr);
  j0_out = j0;
  if (!SPLIT) {
    float w[4];
    bool fast = true;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      w[s] = (float)(S + (double)(j0 + s + 1) * dinc);  // omega = fl32(exact prefix)
      acc[s] = 0.0f;
      fast = fast && (fabsf(w[s]) * (float)H4 < kFastArgLimit);
    }
    // loop placement: the sine loop runs ~10% faster when its 8-byte instructions sit at odd dword
    // addresses (tools/loop_align.py, pinned by tests/test_loop_align.py); PAD puts
    // one dword of padding after an 8-byte alignment point ahead of it where an instantiation needs
    // it (the alignment makes the placement independent of the code laid out before the kernel)
#ifdef DDSP_PROBE_CLOCK
    if (tid == 0) red[20] = (double)wall_clock64();
#endif
    if constexpr (PAD) asm volatile(".p2align 3\n s_nop 0");
    else asm volatile(".p2align 3");
#ifdef DDSP_PROBE_NO_OSC
    if (false) {
#else
    if (active) {
#endif
      if (fast) {
        osc_bank4(coef, H4, w, acc);
      } else {
        for (int k = 0; k < H; ++k) {
          const float2 c = coef[k];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xx = w[s] * c.x;
            acc[s] = fmaf(fabsf(xx) < kFastArgLimit ? sin_reduced(xx) : sin_slow(xx), c.y, acc[s]);
          }
        }
      }
    }
    __syncthreads();  // tail[] complete
#ifdef DDSP_PROBE_CLOCK
    if (tid == 0) red[21] = (double)wall_clock64();
#endif
  } else {
    // SPLIT: every thread takes samples j = tid, tid + NT, ... (the same per-sample sum over k in
    // the same order as above, so the result does not depend on the launch shape); the samples
    // meet their quad's thread through LDS after x[]
    float* hsum = x + bs;
    for (int j = tid; j < bs; j += NT) {
      const float wj = (float)(S + (double)(j + 1) * dinc);
      float a = 0.0f;
      if (fabsf(wj) * (float)H4 < kFastArgLimit) {
        for (int k = 0; k < H4; ++k) {
          const float2 c = coef[k];
          a = fmaf(sin_reduced(wj * c.x), c.y, a);
        }
      } else {
        for (int k = 0; k < H; ++k) {
          const float2 c = coef[k];
          const float xx = wj * c.x;
          a = fmaf(fabsf(xx) < kFastArgLimit ? sin_reduced(xx) : sin_slow(xx), c.y, a);
        }
      }
      hsum[j] = a;
    }
    __syncthreads();  // tail[] and hsum[] complete
    if (active) {
      const float4 h4 = *reinterpret_cast<const float4*>(hsum + j0);
      acc[0] = h4.x;
      acc[1] = h4.y;
      acc[2] = h4.z;
      acc[3] = h4.w;
    }
  }
  // the controls the reference returns (decoder.py:127-135), when asked for, from LDS after the sine loop
  // (registers are free here): ctrl_out = [amplitudes B*F | harmonic_distribution after modules.py:73's
  // in-place `*= amplitudes`, B*F*H | magnitudes B*F*NB]
  if constexpr (CTRL) {
    // (the empty asm re-defines the base here, so no address of these stores is hoisted above the sine
    // loop, where it would hold registers through it)
    float* co = ctrl_out;
    asm volatile("" : "+s"(co));
    const int64_t BF = (int64_t)B * F;
    if (tid == 0) co[frame] = a;
    for (int k = tid; k < H; k += NT) co[BF + frame * H + k] = coef[k].y;
    for (int k = tid; k < NB; k += NT) co[BF * (1 + H) + frame * NB + k] = A[k];
  }
  if (!active) return false;

  // ---- phase 6: filtered noise for the same samples ----
#ifdef DDSP_PROBE_NO_FIR
  float4 y = make_float4(x[j0], x[j0 + 1], x[j0 + 2], x[j0 + 3]);
#else
  float4 y = fir4(h, x, j0, lo_end, bs, bs);  // taps [0, lo_end); the wrapped taps are in tail[]
#endif
  nz[0] = y.x;
  nz[1] = y.y;
  nz[2] = y.z;
  nz[3] = y.w;
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (j0 + s >= tail_start) nz[s] += tail[j0 + s - tail_start];
  return true;
}

template <bool RNG, bool SPLIT, bool CTRL>
__global__ void __launch_bounds__(256) synth_frame_kernel(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float* __restrict__ out, float* __restrict__ harm_out,
    float* __restrict__ noise_out, float* __restrict__ ctrl_out, int F, int H,
    int NB, int bs, float sr, int lo_end, int tail_start, int pad, int ldp, int ldm) {
  extern __shared__ float4 smem4[];
  __shared__ double red[32];
  float acc[4], nz[4];
  int j0;
#ifdef DDSP_PROBE_CLOCK  // shader clocks and 100 MHz ticks over the workgroup's life (tools/exp_clock.py)
  const uint64_t pc0 = clock64(), pt0 = wall_clock64();
#endif
#ifndef DDSP_PAD_XOR  // A/B builds: -DDDSP_PAD_XOR=1 flips every instantiation's sine-loop padding
#define DDSP_PAD_XOR 0
#endif
  if (!frame_synth<RNG, SPLIT, /*PAD=*/(CTRL != (bool)DDSP_PAD_XOR), CTRL>(f0, param, mags, bias, noise, k0, k1, off0, off1, counter, ctrl_out,
                                      (int)gridDim.y, F, H, NB, bs, sr, lo_end, tail_start, pad, blockIdx.x,
                                      blockIdx.y, threadIdx.x, blockDim.x, smem4, red, 0, acc, nz, j0, ldp, ldm))
    return;
  const int64_t o = ((int64_t)blockIdx.y * F + blockIdx.x) * bs + j0;
#ifdef DDSP_PROBE_CLOCK  // harm_out receives the probe: [compute ticks, store ticks, cycles, total ticks]
  const uint64_t pt1 = wall_clock64();
#else
  if (harm_out) *reinterpret_cast<float4*>(harm_out + o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (noise_out) *reinterpret_cast<float4*>(noise_out + o) = make_float4(nz[0], nz[1], nz[2], nz[3]);
#endif
  *reinterpret_cast<float4*>(out + o) =
      make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121
#ifdef DDSP_PROBE_CLOCK
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t pt2 = wall_clock64();
  if (threadIdx.x == 0 && harm_out) {
    *reinterpret_cast<float4*>(harm_out + o) =
        make_float4((float)(pt0 & 0xFFFFFF), (float)((uint64_t)red[20] - pt0), (float)((uint64_t)red[21] - pt0),
                    (float)(pt2 - pt0));
    *reinterpret_cast<float2*>(harm_out + o + 4) = make_float2((float)(pt1 - pt0), (float)(clock64() - pc0));
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// Persistent, wave-specialised form of synth_frame_kernel for launches of many frames.
//
// Why: one workgroup per frame spends ~2/3 of its life in the frame's prologue (controls, filter
// design, noise; latency-bound: dependent global loads and workgroup barriers) and ~1/3 in the
// VALU-bound sine loop.  Across 12800 short-lived workgroups that leaves the VALU idle while the
// first generation of workgroups all run their prologues at once (~15-20 us at config 2) and while
// the last generation drains (~35 us of falling occupancy) — measured with DDSP_PROBE_CLOCK
// (tools/exp_clock.py --in-kernel).  Here a workgroup is NS synthesis threads (the frame's samples,
// 4 per thread, as above) plus one preparation wave, and it walks a contiguous range of frames:
// while the synthesis waves run frame i's sine loop and FIR from one LDS frame buffer, the
// preparation wave builds frame i+1's controls, coefficient table, filter and noise in the other
// (wave-local synchronisation only), and one workgroup barrier per frame swaps them.  Workgroups
// get frame ranges that differ by at most one frame, so they finish together, and the phase
// prefix S_f is carried from frame to frame (exact: every partial sum is representable).
// Arithmetic per sample is the same as synth_frame_kernel's (the noise-filter normalisation sums in
// another order: the control values' double sum may round differently in the last bit).

// LDS-visibility point for one wave: its LDS writes done before any lane's later reads
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum_double(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Frame buffer layout (floats): coef float2[H4] | ct[n4] | A[NB->4] | ir[half+1->4] | h[bs] | tail[half->4] |
// xbuf[pad | bs] | scalars (double S, double dinc, int frame) in the last 8 floats (buf_floats, a multiple
// of 4, includes them)
struct FrameBuf {
  float* base;
  int o_ct, o_A, o_ir, o_h, o_tail, o_x, o_sc;  // float offsets (workgroup-uniform)
  __device__ FrameBuf(float* b, int H4, int n4, int NB, int half, int bs, int pad, int buf_floats) : base(b) {
    o_ct = 2 * H4;
    o_A = o_ct + n4;
    o_ir = o_A + ((NB + 3) & ~3);
    o_h = o_ir + ((half + 4) & ~3);
    o_tail = o_h + bs;
    o_x = o_tail + ((half + 3) & ~3) + pad;
    o_sc = buf_floats - 8;
  }
  __device__ float2* coef() const { return reinterpret_cast<float2*>(base); }
  __device__ float* ct() const { return base + o_ct; }
  __device__ float* A() const { return base + o_A; }
  __device__ float* ir() const { return base + o_ir; }
  __device__ float* h() const { return base + o_h; }
  __device__ float* tail() const { return base + o_tail; }
  __device__ float* x() const { return base + o_x; }
  __device__ double* sc() const { return reinterpret_cast<double*>(base + o_sc); }
  __device__ int* frame() const { return reinterpret_cast<int*>(base + o_sc + 4); }  // -1: no more frames
};

// The preparation wave (lane in [0, 64)): everything frame_synth does before its sine loop, for one
// frame, into buffer fb.  carry: this frame follows the one prepared before it in the same row, whose
// prefix was carry_S.  Returns this frame's prefix S.
template <bool RNG, bool CTRL>
__device__ __forceinline__ double prep_frame(const float* __restrict__ f0, const float* __restrict__ param,
                                           const float* __restrict__ mags, float bias,
                                           const float* __restrict__ noise, uint32_t k0, uint32_t k1,
                                           uint32_t off0, uint32_t off1, float* __restrict__ ctrl_out, int B,
                                           int F, int H, int NB, int bs, float sr, int lo_end, int tail_start,
                                           int pad, int frame, FrameBuf fb, int lane, bool carry,
                                           double carry_S, int ldp, int ldm) {
  const int n = 2 * (NB - 1), half = n >> 1;
  const int H4 = (H + 3) & ~3;
  const int b = frame / F, f = frame - b * F;
  const float* f0b = f0 + (int64_t)b * F;
  const float* prow = param + (int64_t)frame * ldp;
  const float half_sr = sr * 0.5f;
#ifdef DDSP_PROBE_CLOCK
  uint64_t pts[6];
  pts[0] = wall_clock64();
#endif
  // every global load of the frame's first phase is issued before any of its uses (the compiler keeps
  // program order here: one memory latency for the phase instead of one per dependent load)
  const float pitch0 = f0b[f];
  const float praw0 = prow[0];
  const bool loop_prefix = f > 0 && !carry;
  const float fprev = (f > 0 && carry) ? f0b[f - 1] : 0.0f;
  float fv[4], pv[2], mv[2];
#pragma unroll
  for (int r = 0; r < 4; ++r) fv[r] = (loop_prefix && lane + 64 * r < f) ? f0b[lane + 64 * r] : 0.0f;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int k = lane + 64 * r;
    pv[r] = k < H ? prow[1 + k] : 0.0f;
    mv[r] = k < NB ? mags[(int64_t)frame * ldm + k] : 0.0f;
  }
  const int quads = bs >> 2;
  // noise (modules.py:119-123): Philox while the loads are in flight, or the injected samples
  for (int t = lane; t < quads; t += 64) {
    float4 v;
    if (RNG) {
      const uint64_t q = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(r.v[0]), uniform_pm1(r.v[1]), uniform_pm1(r.v[2]), uniform_pm1(r.v[3]));
    } else {
      v = *reinterpret_cast<const float4*>(noise + (int64_t)frame * bs + 4 * t);
    }
    *reinterpret_cast<float4*>(fb.x() + 4 * t) = v;
  }
  for (int i = lane; i < pad; i += 64) fb.x()[i - pad] = 0.0f;
  fill_cos_table(fb.ct(), n, lane, 64);
  // exact fp64 prefix over the row's earlier frames, carried from the previous frame when it is the
  // one before this in the same row
  double S;
  if (f == 0) {
    S = 0.0;
  } else if (carry) {
    S = carry_S + (double)bs * (double)phase_inc(fprev, sr);
  } else {
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (lane + 64 * r < f) part += (double)bs * (double)phase_inc(fv[r], sr);
    for (int g = lane + 256; g < f; g += 64) part += (double)bs * (double)phase_inc(f0b[g], sr);  // f > 256
    S = wave_sum_double(part);
  }
  // controls (modules.py:44-61, 111-114)
  double part_d = 0.0;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int k = lane + 64 * r;
    if (k < H) {
      const float v = controls_value(pv[r], pitch0, k, half_sr);
      fb.coef()[k].y = v;
      part_d += (double)v;
    }
    if (k < NB) fb.A()[k] = scale_fn(mv[r] + bias);
  }
  for (int k = lane + 128; k < H; k += 64) {  // H > 128
    const float v = controls_value(prow[1 + k], pitch0, k, half_sr);
    fb.coef()[k].y = v;
    part_d += (double)v;
  }
  for (int k = lane + 128; k < NB; k += 64) fb.A()[k] = scale_fn(mags[(int64_t)frame * ldm + k] + bias);
  const float norm = (float)wave_sum_double(part_d);  // dist.sum(-1)
  const float a = scale_fn(praw0);
  for (int k = lane; k < H4; k += 64) {  // each lane rereads only the values it wrote
    const float v = k < H ? (fb.coef()[k].y / norm) * a : 0.0f;  // (dist / sum) * amp
    fb.coef()[k] = make_float2((float)(k + 1), v);
  }
  wave_lds_sync();  // A, ct, x
#ifdef DDSP_PROBE_CLOCK
  pts[1] = wall_clock64();
#endif
  // filter design (core.py:144-166): the irfft's even half, then the rolled/windowed taps
  if (n == 128) {
    // 65 bands: lane m builds tap m from the global irfft matrix (coalesced rows of 64); the rows are read
    // through an opaque zero offset, so the compiler cannot hoist the 63 loop-invariant loads out of the
    // frame loop into registers the whole kernel would then hold
    int zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    const float* cosm = kIrCos128 + lane + zero;
    const float* A = fb.A();
    float s0 = 0.0f, s1 = 0.0f;
    // rows k = 1..64 in 4 batches of 16: each batch's loads issued together, then its FMAs in the order
    // of the per-frame kernel (s0 odd k, s1 even k, then k = 63 into s0)
#pragma unroll
    for (int kb = 1; kb < 65; kb += 16) {
      float cv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) cv[r] = kb + r < 64 ? cosm[(kb + r) * 64] : 0.0f;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int k = kb + r;
        if (k < 63) {
          s0 = fmaf(A[k], cv[r], s0);
          s1 = fmaf(A[k + 1], cv[r + 1], s1);
        } else if (k == 63) {
          s0 = fmaf(A[63], cv[r], s0);
        }
      }
    }
    fb.ir()[lane] = (A[0] + ((lane & 1) ? -A[64] : A[64]) + 2.0f * (s0 + s1)) * (1.0f / 128.0f);
    float alt = (lane >= 1) ? ((lane & 1) ? -A[lane] : A[lane]) : 0.0f;  // tap n/2: cos(pi k) = (-1)^k
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) alt += __shfl_xor(alt, o, 64);
    if (lane == 0) fb.ir()[64] = (A[0] + A[64] + 2.0f * alt) * (1.0f / 128.0f);
  } else {
    for (int m = lane; m <= half; m += 64) fb.ir()[m] = irfft_tap(fb.A(), fb.ct(), n, m);
  }
  wave_lds_sync();  // ir
#ifdef DDSP_PROBE_CLOCK
  pts[2] = wall_clock64();
#endif
  const int nlo = lo_end, ntaps = lo_end + (bs - tail_start);
  for (int i = lane; i < ntaps; i += 64) {
    const int j = i < nlo ? i : tail_start + (i - nlo);
    fb.h()[j] = ir_at_half(fb.ir(), fb.ct(), n, bs, j);
  }
  wave_lds_sync();  // h
#ifdef DDSP_PROBE_CLOCK
  pts[3] = wall_clock64();
#endif
  // noise tail: taps past bs - n/2 reach only the last n/2 outputs
  for (int l = lane; l < bs - tail_start; l += 64) {
    const int j = tail_start + l;
    const float* hh = fb.h();
    const float* xx = fb.x();
    float c = 0.0f;
    // 8 taps' operands loaded per step, then the FMAs in the per-frame kernel's order (d = 0, 1, ...)
    for (int d0 = 0; d0 <= l; d0 += 8) {
      float hv[8], xv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        hv[r] = hh[j - d0 - r];  // (in-buffer for d past l: never used)
        xv[r] = xx[d0 + r];
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (d0 + r <= l) c = fmaf(hv[r], xv[r], c);
    }
    fb.tail()[l] = c;
  }
  if (lane == 0) {
    fb.sc()[0] = S;
    fb.sc()[1] = (double)phase_inc(pitch0, sr);
  }
#ifdef DDSP_PROBE_CLOCK  // prep phase durations of this frame -> ctrl_out[8 * frame ..] (probe builds only)
  pts[4] = wall_clock64();
  if (lane == 0 && ctrl_out) {
    for (int i = 0; i < 4; ++i) ctrl_out[8 * (int64_t)frame + i] = (float)(pts[i + 1] - pts[i]);
  }
  return S;
#endif
  if constexpr (CTRL) {  // the controls the reference returns (decoder.py:127-135)
    const int64_t BF = (int64_t)B * F;
    if (lane == 0) ctrl_out[frame] = a;
    for (int k = lane; k < H; k += 64) ctrl_out[BF + (int64_t)frame * H + k] = fb.coef()[k].y;
    for (int k = lane; k < NB; k += 64) ctrl_out[BF * (1 + H) + (int64_t)frame * NB + k] = fb.A()[k];
  }
  return S;
}

// The preparation wave's work for one frame when frame_table_kernel has run (TAB): the frame's record
// (amplitudes, filter taps, S, dinc) into fb, the noise, the filter tail.
template <bool RNG>
__device__ __forceinline__ void prep_frame_tab(const float* __restrict__ table, int rec,
                                               const float* __restrict__ noise, uint32_t k0, uint32_t k1,
                                               uint32_t off0, uint32_t off1, int H, int bs, int lo_end,
                                               int tail_start, int pad, int frame, FrameBuf fb, int lane) {
  const int H4 = (H + 3) & ~3;
  const float* r = table + (int64_t)frame * rec;
  const double2 sd = *reinterpret_cast<const double2*>(r);
  const int ntaps = lo_end + (bs - tail_start);
  for (int k = lane; k < H4; k += 64) fb.coef()[k] = make_float2((float)(k + 1), r[4 + k]);
  for (int i = lane; i < ntaps; i += 64) fb.h()[i < lo_end ? i : tail_start + (i - lo_end)] = r[4 + H4 + i];
  const int quads = bs >> 2;
  for (int t = lane; t < quads; t += 64) {  // modules.py:119-123
    float4 v;
    if (RNG) {
      const uint64_t q = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 p = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(p.v[0]), uniform_pm1(p.v[1]), uniform_pm1(p.v[2]), uniform_pm1(p.v[3]));
    } else {
      v = *reinterpret_cast<const float4*>(noise + (int64_t)frame * bs + 4 * t);
    }
    *reinterpret_cast<float4*>(fb.x() + 4 * t) = v;
  }
  for (int i = lane; i < pad; i += 64) fb.x()[i - pad] = 0.0f;
  wave_lds_sync();  // h, x
  for (int l = lane; l < bs - tail_start; l += 64) {  // noise tail, in frame_synth's tap order
    const int j = tail_start + l;
    const float* hh = fb.h();
    const float* xx = fb.x();
    float c = 0.0f;
    for (int d0 = 0; d0 <= l; d0 += 8) {
      float hv[8], xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        hv[q] = hh[j - d0 - q];
        xv[q] = xx[d0 + q];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (d0 + q <= l) c = fmaf(hv[q], xv[q], c);
    }
    fb.tail()[l] = c;
  }
  if (lane == 0) {
    fb.sc()[0] = sd.x;
    fb.sc()[1] = sd.y;
  }
}

// TAB: frame_table_kernel ran first; `param` is then its table and `ldp` the record's floats (f0, mags,
// ctrl_out unused: the table kernel wrote the control dicts).
template <bool RNG, bool CTRL, bool PAD, bool TAB = false>
__global__ void __launch_bounds__(320, 5) synth_persist_kernel(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float* __restrict__ out, float* __restrict__ harm_out,
    float* __restrict__ noise_out, float* __restrict__ ctrl_out, int B, int F, int H, int NB, int bs, float sr,
    int lo_end, int tail_start, int pad, int buf_floats, uint32_t* __restrict__ tickets, int ldp, int ldm) {
  extern __shared__ float4 smem4[];
  const int NS = (int)blockDim.x - 64;  // synthesis threads; the last wave prepares
  const int tid = threadIdx.x;
  const bool prep = tid >= NS;
  const int lane = tid & 63;
  const int NF = B * F;
  const int n = 2 * (NB - 1), half = n >> 1, n4 = (n + 3) & ~3;
  const int H4 = (H + 3) & ~3;
  float* base = reinterpret_cast<float*>(smem4);
  FrameBuf fb0(base, H4, n4, NB, half, bs, pad, buf_floats), fb1 = fb0;
  fb1.base = base + buf_floats;
  if (RNG && counter) {  // graph-replayed streams: the Philox offset advances in device memory
    const uint64_t o = (((uint64_t)off1 << 32) | off0) + *counter;
    off0 = (uint32_t)o;
    off1 = (uint32_t)(o >> 32);
  }
#ifdef DDSP_PROBE_HWID  // each wave's HW_ID (SIMD, CU, SE) -> harm_out[4 * workgroup + wave]
  if (lane == 0 && harm_out)
    harm_out[4 * (int64_t)blockIdx.x + (tid >> 6)] = __int_as_float((int)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  if (harm_out) return;
#endif
  // Frames are taken one at a time from the launch's ticket counter (tickets[0]) by the preparation
  // wave, so workgroups whose SIMDs carry more synthesis waves take fewer frames (dynamic balance, as a
  // one-workgroup-per-frame launch has).  The workgroup that takes the last failing ticket (tickets[1]
  // counts them) zeroes both counters for the stream's next launch.  Iteration i: the preparation wave
  // builds the next frame in buffer (i+1)&1 while the synthesis waves run buffer i&1's; one barrier per
  // iteration.  The two roles run separate loops (the same number of barriers) so that each loop's
  // hoisted invariants stay in its own branch and hold no registers through the sine loop.
#ifdef DDSP_PROBE_CLOCK
  const uint64_t wg_t0 = wall_clock64();
  int probe_first = -1;
#endif
  if (prep) {
    // the preparation wave's instructions issue ahead of the synthesis waves' (VALU arbitration is by
    // priority, then age): its chain of short dependent steps then waits on memory and LDS only, not on
    // the sine loops that saturate the SIMD
    __builtin_amdgcn_s_setprio(3);
    auto take = [&]() -> int {
      int t = 0;
      if (lane == 0) t = (int)atomicAdd(tickets, 1u);
      t = __shfl(t, 0, 64);
      if (t >= NF) {
        if (lane == 0 && atomicAdd(tickets + 1, 1u) == gridDim.x - 1) {  // every workgroup is done taking
          tickets[0] = 0;
          tickets[1] = 0;
        }
        return -1;
      }
      return t;
    };
    int prev = -2;
    double carry_S = 0.0;
    int fr = take();
    for (int i = 0;; ++i) {
      FrameBuf nb = fb0;
      nb.base = (i & 1) ? fb1.base : fb0.base;
      if (fr >= 0) {
#ifdef DDSP_PROBE_CLOCK
        if (probe_first < 0) probe_first = fr;
#endif
        if constexpr (TAB)
          prep_frame_tab<RNG>(param, ldp, noise, k0, k1, off0, off1, H, bs, lo_end, tail_start, pad, fr, nb, lane);
        else
          carry_S = prep_frame<RNG, CTRL>(f0, param, mags, bias, noise, k0, k1, off0, off1, ctrl_out, B, F, H, NB,
                                          bs, sr, lo_end, tail_start, pad, fr, nb, lane, fr == prev + 1, carry_S, ldp,
                                          ldm);
      }
      if (lane == 0) *nb.frame() = fr;
      __syncthreads();  // buffer i&1 prepared (or marked empty); the synthesis waves released the other one
      if (fr < 0) break;
      prev = fr;
      fr = take();
    }
#ifdef DDSP_PROBE_CLOCK  // workgroup start (low 24 bits of the 100 MHz clock) and life -> ctrl_out[8 * first + 6, 7]
    if (lane == 0 && ctrl_out && probe_first >= 0) {
      ctrl_out[8 * (int64_t)probe_first + 6] = (float)(wg_t0 & 0xFFFFFF);
      ctrl_out[8 * (int64_t)probe_first + 7] = (float)(wall_clock64() - wg_t0);
    }
#endif
    return;
  }
  __syncthreads();  // the first frame prepared
  const int j0 = 4 * tid;
  for (int i = 0;; ++i) {
    FrameBuf cur = fb0;
    cur.base = (i & 1) ? fb1.base : fb0.base;
    const int fr = *cur.frame();
    if (fr < 0) break;
#ifdef DDSP_PROBE_CLOCK
    const uint64_t st0 = wall_clock64();
#endif
    if (j0 < bs) {
      const double S = cur.sc()[0], dinc = cur.sc()[1];
      float w[4], acc[4];
      bool fast = true;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        w[s] = (float)(S + (double)(j0 + s + 1) * dinc);  // omega = fl32(exact prefix)
        acc[s] = 0.0f;
        fast = fast && (fabsf(w[s]) * (float)H4 < kFastArgLimit);
      }
      const float2* coef = cur.coef();
      // loop placement as in frame_synth (tests/test_loop_align.py pins it)
      if constexpr (PAD) asm volatile(".p2align 3\n s_nop 0");
      else asm volatile(".p2align 3");
#ifdef DDSP_PROBE_NO_OSC  // timing probe: no sine loop
      if (false)
#endif
      if (fast) {
        osc_bank4(coef, H4, w, acc);
      } else {
        for (int k = 0; k < H; ++k) {
          const float2 c = coef[k];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float xx = w[s] * c.x;
            acc[s] = fmaf(fabsf(xx) < kFastArgLimit ? sin_reduced(xx) : sin_slow(xx), c.y, acc[s]);
          }
        }
      }
      const float4 y = fir4(cur.h(), cur.x(), j0, lo_end, bs, bs);  // taps [0, lo_end); wrapped ones in tail[]
      float nz[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (j0 + s >= tail_start) nz[s] += cur.tail()[j0 + s - tail_start];
      const int64_t o = (int64_t)fr * bs + j0;
      if (harm_out) *reinterpret_cast<float4*>(harm_out + o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      if (noise_out) *reinterpret_cast<float4*>(noise_out + o) = make_float4(nz[0], nz[1], nz[2], nz[3]);
      *reinterpret_cast<float4*>(out + o) =
          make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121
    }
#ifdef DDSP_PROBE_CLOCK  // synthesis time and barrier wait of this frame -> ctrl_out[8 * frame + 4, 5]
    const uint64_t st1 = wall_clock64();
    __syncthreads();
    if (tid == 0 && ctrl_out) {
      ctrl_out[8 * (int64_t)fr + 4] = (float)(st1 - st0);
      ctrl_out[8 * (int64_t)fr + 5] = (float)(wall_clock64() - st1);
    }
#else
    __syncthreads();  // frame fr's buffer free, frame fr + 1's prepared
#endif
  }
}

// ---------------------------------------------------------------------------------------------
// Two-launch form for launches of many frames: the frame table, then the synthesis.
//
// Why: a one-workgroup-per-frame launch spends ~22 of a workgroup's ~36 us in the frame's prologue
// (controls, filter design: dependent global loads, five barriers) — at the start of the launch every
// resident workgroup is in it with the VALU idle, and the last generation drains at that pace
// (DESIGN §3c).  frame_table_kernel runs those controls for every frame first (one wave per frame,
// no workgroup barriers) into a per-frame record in HBM; synth_tab_kernel's prologue is then one load
// of that record (~0.9 KB), the noise and the tail, and its workgroups are mostly sine loop.
//
// Record (floats, 16-B aligned, rec floats per frame): [S (double) | dinc (double) | amplitudes
// (dist/sum)*amp, H4 | filter taps h[j] for j in [0, lo_end) then [tail_start, bs), ntaps -> 4].
// Every value is computed by the arithmetic frame_synth uses, and the two fp64 sums in the order of
// frame_synth's nw-wave thread group (thread 64w + lane: strided partials, a shuffle tree per wave, the
// waves' totals in order), so the synthesis is bit-identical to synth_frame_kernel's.

// per-wave LDS floats of frame_table_kernel: ct[n4] | A[NB -> 4] | ir[half+1 -> 4] | vals[H4]; with 65 bands
// the workgroup also holds the 64 x 64 irfft matrix (kTableCosFloats, ahead of the waves' regions)
constexpr int kTableCosFloats = 64 * 64;
static __host__ __device__ inline int table_wave_floats(int H, int NB) {
  const int n = 2 * (NB - 1), half = n >> 1;
  return ((n + 3) & ~3) + ((NB + 3) & ~3) + ((half + 4) & ~3) + ((H + 3) & ~3);
}

// One wave per frame.  Latency is the whole cost here (12,800 short chains at config 2), so every global
// load of a frame is issued up front: the row's f0 values for the prefix, the projections, the
// magnitudes (registers, first 2 x NT of each; loops past that) and, for 65 bands, the irfft matrix
// into LDS by the whole workgroup.
// NW: the waves of frame_synth's thread group (nt / 64 of the launch, 1..4)
template <bool CTRL, int NW>
__global__ void __launch_bounds__(512) frame_table_kernel(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags, float bias,
    float* __restrict__ ctrl_out, float* __restrict__ table, int B, int F, int H, int NB, int bs, float sr,
    int lo_end, int tail_start, int rec, int ldp, int ldm) {
  constexpr int nw = NW;
  extern __shared__ float4 smem4[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t NF = (int64_t)B * F;
  const int64_t frame = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;  // one wave per frame
  const int n = 2 * (NB - 1), half = n >> 1, n4 = (n + 3) & ~3;
  const int H4 = (H + 3) & ~3;
#ifdef DDSP_PROBE_TAB_NOMAT
  const bool cos_lds = false;
#else
  const bool cos_lds = n == 128;
#endif
  float* cosL = reinterpret_cast<float*>(smem4);
  if (cos_lds) {  // rows k = 0..63 of kIrCos128 (row 0 unused), 8 floats per thread of 512
    for (int i = threadIdx.x; i < kTableCosFloats / 4; i += blockDim.x)
      reinterpret_cast<float4*>(cosL)[i] = reinterpret_cast<const float4*>(kIrCos128)[i];
  }
  const bool live = frame < NF;
  const int64_t fr = live ? frame : 0;  // a wave past the last frame only helps with the matrix
#ifdef DDSP_PROBE_TAB_EMPTY  // launch-shape floor: one store per frame
  if (live && lane == 0) table[fr * rec] = 0.0f;
  return;
#endif
  float* ct = cosL + (cos_lds ? kTableCosFloats : 0) + wv * table_wave_floats(H, NB);
  float* A = ct + n4;
  float* ir = A + ((NB + 3) & ~3);
  float* vals = ir + ((half + 4) & ~3);
  const int b = (int)(fr / F), f = (int)(fr - (int64_t)b * F);
  const float* f0b = f0 + (int64_t)b * F;
  const float* prow = param + fr * ldp;
  const float* mrow = mags + fr * ldm;
  const float half_sr = sr * 0.5f;
  const float pitch0 = f0b[f];
  const float praw0 = prow[0];
  const int NT = 64 * nw;
  // frame_synth's thread t = 64w + lane visits g (and k) = t, t + NT, ...: the first two of each here
  float fv[NW][2], pv[NW][2], mv[2];
#pragma unroll
  for (int w = 0; w < NW; ++w)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int g = 64 * w + lane + NT * j;
      fv[w][j] = g < f ? f0b[g] : 0.0f;
      pv[w][j] = g < H ? prow[1 + g] : 0.0f;
    }
#pragma unroll
  for (int j = 0; j < 2; ++j) mv[j] = lane + 64 * j < NB ? mrow[lane + 64 * j] : 0.0f;
#ifdef DDSP_PROBE_TAB_LOADS  // loads of the frame and its record's stores, no arithmetic
  if (live) {
    float* rr = table + fr * rec;
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int g = 64 * w + lane + NT * j;
        if (g < H4) rr[4 + g] = pv[w][j] + fv[w][j];
      }
    if (lane < rec - 4 - H4) rr[4 + H4 + lane] = mv[0] + mv[1] + pitch0 + praw0;
  }
  return;
#endif
  fill_cos_table(ct, n, lane, 64);
  // the fp64 prefix and dist.sum(-1), summed as frame_synth's group sums them
  double S = 0.0, D = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    {
      double ps = 0.0, pd = 0.0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int g = 64 * w + lane + NT * j;
        if (g < f) ps += (double)bs * (double)phase_inc(fv[w][j], sr);
        if (g < H) {  // modules.py:53-60 before normalisation
#ifdef DDSP_PROBE_TAB_NOCTRL
          const float v = pv[w][j];
#else
          const float v = controls_value(pv[w][j], pitch0, g, half_sr);
#endif
          vals[g] = v;
          pd += (double)v;
        }
      }
      for (int g = 64 * w + lane + 2 * NT; g < f; g += NT) ps += (double)bs * (double)phase_inc(f0b[g], sr);
      for (int k = 64 * w + lane + 2 * NT; k < H; k += NT) {
        const float v = controls_value(prow[1 + k], pitch0, k, half_sr);
        vals[k] = v;
        pd += (double)v;
      }
#ifndef DDSP_PROBE_TAB_NORED
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        ps += __shfl_down(ps, o, 64);
        pd += __shfl_down(pd, o, 64);
      }
      S += __shfl(ps, 0, 64);
      D += __shfl(pd, 0, 64);
#else
      S += ps;
      D += pd;
#endif
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (lane + 64 * j < NB) A[lane + 64 * j] = scale_fn(mv[j] + bias);  // modules.py:113
  for (int k = lane + 128; k < NB; k += 64) A[k] = scale_fn(mrow[k] + bias);
  const float norm = (float)D;
  const float a = scale_fn(praw0);
  float* r = table + fr * rec;
#ifdef DDSP_PROBE_TAB_NOMAT
  wave_lds_sync();
#else
  __syncthreads();  // the matrix; this wave's vals, A, ct
#endif
  if (!live) return;
  const int64_t BF = NF;
  for (int k = lane; k < H4; k += 64) {
    const float v = k < H ? (vals[k] / norm) * a : 0.0f;  // (dist / sum) * amp
    r[4 + k] = v;
    if (CTRL && k < H) ctrl_out[BF + frame * H + k] = v;  // modules.py:73's in-place product
  }
  if constexpr (CTRL) {
    if (lane == 0) ctrl_out[frame] = a;
    for (int k = lane; k < NB; k += 64) ctrl_out[BF * (1 + H) + frame * NB + k] = A[k];
  }
  // filter design (core.py:144-166): the irfft's even half, then the rolled/windowed taps
#ifdef DDSP_PROBE_TAB_NOFILTER
  if (lane == 0) *reinterpret_cast<double2*>(r) = make_double2(S, (double)phase_inc(pitch0, sr));
  return;
#endif
  if (cos_lds) {
    const float* cosm = cosL + lane;
    float s0 = 0.0f, s1 = 0.0f;  // frame_synth's order: s0 odd k, s1 even k, then k = 63 into s0
#pragma unroll 8
    for (int k = 1; k < 63; k += 2) {
      s0 = fmaf(A[k], cosm[k * 64], s0);
      s1 = fmaf(A[k + 1], cosm[(k + 1) * 64], s1);
    }
    s0 = fmaf(A[63], cosm[63 * 64], s0);
    ir[lane] = (A[0] + ((lane & 1) ? -A[64] : A[64]) + 2.0f * (s0 + s1)) * (1.0f / 128.0f);
    float alt = (lane >= 1) ? ((lane & 1) ? -A[lane] : A[lane]) : 0.0f;  // tap n/2: cos(pi k) = (-1)^k
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) alt += __shfl_xor(alt, o, 64);
    if (lane == 0) ir[64] = (A[0] + A[64] + 2.0f * alt) * (1.0f / 128.0f);
  } else {
    for (int m = lane; m <= half; m += 64) ir[m] = irfft_tap(A, ct, n, m);
  }
  wave_lds_sync();  // ir
  const int ntaps = lo_end + (bs - tail_start);
  for (int i = lane; i < ntaps; i += 64) {
    const int j = i < lo_end ? i : tail_start + (i - lo_end);
    r[4 + H4 + i] = ir_at_half(ir, ct, n, bs, j);
  }
  if (lane == 0) *reinterpret_cast<double2*>(r) = make_double2(S, (double)phase_inc(pitch0, sr));
}

// The synthesis of one frame (f, b) per workgroup from its frame_table_kernel record: noise, filter
// tail, oscillator bank, FIR, `harmonic + noise` — frame_synth's phases 4-6 with phases 1-3 read back.
// LDS: coef float2[H4] | h[bs] | tail[half -> 4] | xbuf[pad | bs]
template <bool RNG, bool PAD>
__global__ void __launch_bounds__(256) synth_tab_kernel(
    const float* __restrict__ table, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0,
    uint32_t off1, const uint64_t* __restrict__ counter, float* __restrict__ out, float* __restrict__ harm_out,
    float* __restrict__ noise_out, int F, int H, int NB, int bs, int lo_end, int tail_start, int pad, int rec) {
  extern __shared__ float4 smem4[];
  const int tid = threadIdx.x, NT = blockDim.x;
  const int half = NB - 1;
  const int H4 = (H + 3) & ~3;
  float2* coef = reinterpret_cast<float2*>(smem4);
  float* h = reinterpret_cast<float*>(coef + H4);
  float* tail = h + bs;
  float* xbuf = tail + ((half + 3) & ~3);
  float* x = xbuf + pad;
  const int64_t frame = (int64_t)blockIdx.y * F + blockIdx.x;
  const float* r = table + frame * rec;
  const double2 sd = *reinterpret_cast<const double2*>(r);  // workgroup-uniform: S, dinc
  for (int k = tid; k < H4; k += NT) coef[k] = make_float2((float)(k + 1), r[4 + k]);
  const int ntaps = lo_end + (bs - tail_start);
  for (int i = tid; i < ntaps; i += NT) h[i < lo_end ? i : tail_start + (i - lo_end)] = r[4 + H4 + i];
  for (int i = tid; i < pad; i += NT) xbuf[i] = 0.0f;
  if (RNG && counter) {  // graph-replayed streams: the Philox offset advances in device memory
    const uint64_t o = (((uint64_t)off1 << 32) | off0) + *counter;
    off0 = (uint32_t)o;
    off1 = (uint32_t)(o >> 32);
  }
  const int quads = bs >> 2;
  for (int t = tid; t < quads; t += NT) {  // modules.py:119-123
    float4 v;
    if (RNG) {
      const uint64_t q = (uint64_t)frame * (uint64_t)quads + (uint64_t)t;
      const Philox4 p = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);
      v = make_float4(uniform_pm1(p.v[0]), uniform_pm1(p.v[1]), uniform_pm1(p.v[2]), uniform_pm1(p.v[3]));
    } else {
      v = *reinterpret_cast<const float4*>(noise + frame * bs + 4 * t);
    }
    *reinterpret_cast<float4*>(x + 4 * t) = v;
  }
  __syncthreads();
  // noise tail (taps past bs - n/2 reach only the last n/2 outputs)
  for (int l = tid; l < bs - tail_start; l += NT) {
    const int j = tail_start + l;
    float c = 0.0f;
    for (int d = 0; d <= l; ++d) c = fmaf(h[j - d], x[d], c);
    tail[l] = c;
  }
  // oscillator bank for samples [j0, j0+4)
  const int j0 = 4 * tid;
  const bool active = j0 < bs;
  float w[4], acc[4];
  bool fast = true;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    w[s] = (float)(sd.x + (double)(j0 + s + 1) * sd.y);  // omega = fl32(exact prefix)
    acc[s] = 0.0f;
    fast = fast && (fabsf(w[s]) * (float)H4 < kFastArgLimit);
  }
  // loop placement as in frame_synth (tools/loop_align.py; tests/test_loop_align.py pins it)
  if constexpr (PAD) asm volatile(".p2align 3\n s_nop 0");
  else asm volatile(".p2align 3");
  if (active) {
    if (fast) {
      osc_bank4(coef, H4, w, acc);
    } else {
      for (int k = 0; k < H; ++k) {
        const float2 c = coef[k];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float xx = w[s] * c.x;
          acc[s] = fmaf(fabsf(xx) < kFastArgLimit ? sin_reduced(xx) : sin_slow(xx), c.y, acc[s]);
        }
      }
    }
  }
  __syncthreads();  // tail[] complete
  if (!active) return;
  const float4 y = fir4(h, x, j0, lo_end, bs, bs);  // taps [0, lo_end); the wrapped taps are in tail[]
  float nz[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (j0 + s >= tail_start) nz[s] += tail[j0 + s - tail_start];
  const int64_t o = frame * bs + j0;
  if (harm_out) *reinterpret_cast<float4*>(harm_out + o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (noise_out) *reinterpret_cast<float4*>(noise_out + o) = make_float4(nz[0], nz[1], nz[2], nz[3]);
  *reinterpret_cast<float4*>(out + o) =
      make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121
}

__global__ void counter_advance_kernel(uint64_t* counter) { *counter += 1; }

}  // namespace
}  // namespace ddsp

using namespace ddsp;

// sine-loop placement padding of the fused synthesis + forward-transform instantiations (tools/loop_align.py)
template <bool RNG>
constexpr bool kSynthForwardPad = false;

// sine-loop placement padding of the persistent instantiations (tools/loop_align.py)
template <bool RNG, bool CTRL>
constexpr bool kPersistPad = false;

// sine-loop placement padding of the frame-table synthesis instantiations (tools/loop_align.py)
template <bool RNG>
constexpr bool kTabPad = true;

// sine-loop placement padding of the persistent instantiations fed by the frame table
template <bool RNG>
constexpr bool kPersistTabPad = false;


namespace ddsp {
namespace {

// ---------------------------------------------------------------------------------------------
// Synthesis fused with the reverb's forward transform (decoder.py:106-125: the synthesis section
// and Reverb.forward's first step, modules.py:28-35 via upols.hip).  The reverb's partitioned
// convolution starts from Z_b = FFT_4096([x_b, 0]) of every 2048-sample block of two packed rows
// (x_a + i x_b); here one workgroup per (pair of rows, block) synthesises the block's 2 x (2048/bs)
// frames — a thread group of NT threads per frame, exactly frame_synth as in synth_frame_kernel —
// and transforms them in LDS, so the dry signal never goes to HBM (26 MB written and re-read at
// config 2) and the forward transform's launch disappears.  The transform: four radix-8 Stockham
// passes by 512 threads (8 points each: the frame buffers' 64-VGPR budget, which the separate
// forward kernel's 16-point radix-16 passes exceed), its buffer overlaying the frame buffers.
// Z is the layout upols_apply_spectra reads ([pair][block][4096]); the MAC and inverse follow.
struct Tw3 {
  float2 w1, w2, w4;
};
template <bool INV>
__device__ __forceinline__ Tw3 radix8_tw(int step) {
  return Tw3{twiddle(step, INV), twiddle(2 * step, INV), twiddle(4 * step, INV)};
}
__device__ __forceinline__ void radix8_twiddle(float2 (&v)[8], const Tw3& t) {
  const float2 w1 = t.w1, w2 = t.w2, w4 = t.w4;
  const float2 w3 = cmul(w1, w2);
  v[1] = cmul(v[1], w1);
  v[2] = cmul(v[2], w2);
  v[3] = cmul(v[3], w3);
  v[4] = cmul(v[4], w4);
  v[5] = cmul(v[5], cmul(w4, w1));
  v[6] = cmul(v[6], cmul(w4, w2));
  v[7] = cmul(v[7], cmul(w4, w3));
}

template <bool RNG, bool PAD>
__global__ void __launch_bounds__(1024, 8) synth_forward_kernel(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float2* __restrict__ Z, int B, int F, int H, int NB, int bs,
    float sr, int lo_end, int tail_start, int pad, int gfloats, int NT, int nb, int ldp, int ldm) {
  extern __shared__ float4 smem4[];
  __shared__ double red[32];
  const int fpb = kP / bs;  // frames per block
  const int g = threadIdx.x / NT, tid = threadIdx.x - g * NT;
  const int rr = g / fpb, fl = g - rr * fpb;  // row of the pair, frame of the block
  const int blk = blockIdx.x, pair = blockIdx.y;
  const int row = 2 * pair + rr, f = blk * fpb + fl;
  const bool valid = row < B && f < F;  // else zeros (an odd batch's missing row, frames past T)
  float acc[4], nz[4];
  int j0;
  // groups outside the signal synthesise a clamped frame (every group runs frame_synth's barriers)
  const bool act = frame_synth<RNG, false, PAD, false>(
      f0, param, mags, bias, noise, k0, k1, off0, off1, counter, nullptr, B, F, H, NB, bs, sr, lo_end, tail_start,
      pad, min(f, F - 1), min(row, B - 1), tid, NT, smem4 + (size_t)g * (gfloats >> 2), red, g * (NT >> 6), acc, nz,
      j0, ldp, ldm);
#ifdef DDSP_PROBE_SR_NOFFT  // timing probe: the synthesis alone at this launch shape (tools/exp_synth_reverb.py)
  if (act && acc[0] + nz[0] == 1234.5f) Z[threadIdx.x] = make_float2(acc[1], nz[1]);
  return;
#endif
  __syncthreads();  // every frame buffer is free: the transform buffer overlays them
  float2* buf = reinterpret_cast<float2*>(smem4);
  float* bf = reinterpret_cast<float*>(smem4);
  if (act) {
    const int p0 = fl * bs + j0;
#pragma unroll
    for (int s = 0; s < 4; ++s) bf[2 * lds_idx(p0 + s) + rr] = valid ? acc[s] + nz[s] : 0.0f;  // decoder.py:121
  }
  __syncthreads();
  constexpr int NTF = kN / 8;  // transform threads
  if (threadIdx.x < NTF) {
    const int j = threadIdx.x;
    // the passes' twiddles first: their loads' latency hides behind the first pass
    Tw3 tw[3];
#pragma unroll
    for (int pass = 1; pass < 4; ++pass) {
      const int ns = 1 << (3 * pass);
      tw[pass - 1] = radix8_tw<false>((j & (ns - 1)) * (kN / 8 / ns));
    }
    float2 v[8];
    // pass 1 (Ns = 1): inputs j + 512 r; r >= 4 is the block's zero half
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = buf[lds_idx(j + NTF * r)];
#pragma unroll
    for (int r = 4; r < 8; ++r) v[r] = make_float2(0.0f, 0.0f);
    dft8<false>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    int Ns = 1;
#pragma unroll
    for (int pass = 1; pass < 4; ++pass) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) buf[lds_idx((j / Ns) * Ns * 8 + (j & (Ns - 1)) + r * Ns)] = v[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = buf[lds_idx(j + NTF * r)];
      Ns *= 8;
      radix8_twiddle(v, tw[pass - 1]);
      dft8<false>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    }
    float2* out = Z + ((int64_t)pair * nb + blk) * kN;  // Ns = 512: natural order j + 512 r
#pragma unroll
    for (int r = 0; r < 8; ++r) out[j + NTF * r] = v[r];
  } else {
#pragma unroll
    for (int pass = 1; pass < 4; ++pass) {
      __syncthreads();
      __syncthreads();
    }
  }
}

}  // namespace
}  // namespace ddsp

// compute units of the current device (cached per device)
static int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = n;
  }
  return cached[dev];
}

// persistent workgroups per CU: ddsp_hip_set_persistent_workgroups, else DDSP_HIP_PERSIST_WPC, else 8
// (0 turns the persistent kernel off)
static std::atomic<int> g_persist_wpc{-1};
static int persist_default() {
  const char* e = getenv("DDSP_HIP_PERSIST_WPC");
  return e ? std::max(0, atoi(e)) : 0;  // off by default until it beats the per-frame kernel
}
static int persist_wgs_per_cu() {
  const int v = g_persist_wpc.load(std::memory_order_relaxed);
  return v >= 0 ? v : persist_default();
}

// The persistent kernel's ticket counters (frames taken, workgroups done), one pair per (device, stream):
// zeroed once here, then by the last workgroup of every launch, so launches on one stream (ordered) reuse
// them; a device allocation kept for the life of the process.
static uint32_t* persist_tickets(void* stream) {
  static std::mutex mu;
  static std::map<std::pair<int, void*>, uint32_t*> slots;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto it = slots.find({dev, stream});
  if (it != slots.end()) return it->second;
  uint32_t* p = nullptr;
  if (hipMalloc(&p, 2 * sizeof(uint32_t)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, 2 * sizeof(uint32_t), reinterpret_cast<hipStream_t>(stream)) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  slots[{dev, stream}] = p;
  return p;
}

// DDSP_HIP_PERSIST_LDSPAD=1: LDS per workgroup padded so that a CU holds at most wpc of them
static size_t persist_lds_floor(int wpc) {
  static int pad = -1;
  if (pad < 0) {
    const char* e = getenv("DDSP_HIP_PERSIST_LDSPAD");
    pad = e ? atoi(e) : 0;
  }
  return pad && wpc > 0 ? (size_t)(160 * 1024 / (wpc + 1) + 1024) : 0;
}

// the two-launch form (frame_table_kernel + synth_tab_kernel) for launches of many frames:
// ddsp_hip_set_frame_table, else DDSP_HIP_FRAME_TABLE, else off (measured slower in the bench step: the
// synthesis launch gains ~20 us, the table launch costs ~26 us)
static std::atomic<int> g_frame_table{-1};
static int frame_table_on() {
  const int v = g_frame_table.load(std::memory_order_relaxed);
  if (v >= 0) return v;
  const char* e = getenv("DDSP_HIP_FRAME_TABLE");
  return e ? atoi(e) != 0 : 0;
}

// frame_table_kernel's records: one grow-only device buffer per (device, stream), so launches on one
// stream (ordered) reuse it.  Never taken while the stream is capturing a graph (nullptr: the caller
// runs the one-launch kernel), so no graph holds one; a smaller buffer left by growth stays allocated.
static float* frame_table_buffer(void* stream, size_t floats) {
  static std::mutex mu;
  static std::map<std::pair<int, void*>, std::pair<float*, size_t>> slots;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(S(stream), &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  auto& slot = slots[{dev, stream}];
  if (slot.second >= floats) return slot.first;
  float* p = nullptr;
  if (hipMalloc(&p, floats * sizeof(float)) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  slot = {p, floats};
  return p;
}

// a frame's LDS layout (frame_synth): the FIR's first run [0, lo_end) and the wrapped taps from
// tail_start, the zero padding ahead of the samples, and the floats of one frame buffer
struct FrameShape {
  int lo_end, tail_start, pad;
  size_t floats;
};
static FrameShape frame_shape(int64_t n_harmonic, int64_t n_bands, int bs) {
  const int n = 2 * (int)(n_bands - 1), half = n / 2;
  FrameShape fs;
  if (bs >= n) {
    fs.lo_end = (half + 3) & ~3;
    fs.tail_start = bs - half;
    if (fs.tail_start < fs.lo_end) {
      fs.lo_end = bs;
      fs.tail_start = bs;
    }
  } else {
    fs.lo_end = bs;
    fs.tail_start = bs;
  }
  fs.pad = (fs.lo_end + 4 + 3) & ~3;
  const int H4 = ((int)n_harmonic + 3) & ~3, n4 = (n + 3) & ~3;
  fs.floats = (size_t)2 * H4 + n4 + (((int)n_bands + 3) & ~3) + ((half + 4) & ~3) + bs + ((half + 3) & ~3) +
              fs.pad + bs;
  return fs;
}

extern "C" {

static int synth_frames_launch(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                               const float* noise, uint64_t seed, uint64_t offset, uint64_t* counter, float* out,
                               float* harmonic_out, float* noise_out, float* controls_out, int64_t batch, int64_t frames,
                               int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                               void* stream, int64_t param_ld = -1, int64_t mags_ld = -1) {
  if (param_ld < 0) param_ld = n_harmonic + 1;
  if (mags_ld < 0) mags_ld = n_bands;
  if (batch < 0 || frames < 0 || n_harmonic < 1 || n_bands < 2 || block_size < 4) return DDSP_HIP_EINVAL;
  if (param_ld < n_harmonic + 1 || mags_ld < n_bands || param_ld > INT32_MAX || mags_ld > INT32_MAX) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!f0 || !param || !raw_magnitudes || !out) return DDSP_HIP_EINVAL;
  // the fused kernel's shape envelope; callers fall back to the separate kernels outside it
  if (block_size % 4 || block_size > 1024 || n_harmonic > 1024 || n_bands > 1025 || batch > 65535 ||
      frames > INT32_MAX)
    return DDSP_HIP_ERANGE;
  const int bs = (int)block_size;
  const FrameShape fs = frame_shape(n_harmonic, n_bands, bs);
  const int lo_end = fs.lo_end, tail_start = fs.tail_start, pad = fs.pad;
  const size_t floats = fs.floats;
  if (sizeof(float) * floats > 120 * 1024) return DDSP_HIP_ERANGE;
  const int nt = std::max(64, ((bs / 4 + 63) / 64) * 64);
  // few frames (far fewer workgroups than CUs): split each frame's harmonics over G thread groups
  int G = batch * frames < 512 ? std::max(1, std::min(4, 256 / nt)) : 1;
  if (sizeof(float) * (floats + (size_t)bs) > 120 * 1024) G = 1;
  const size_t shm = sizeof(float) * (floats + (G > 1 ? (size_t)bs : 0));
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
  const int64_t NF = batch * frames;
  // many frames: the frames' controls, filter taps and phase prefixes into a table first (one wave per
  // frame), then a synthesis kernel reading it
  float* table = nullptr;
  const int H4 = ((int)n_harmonic + 3) & ~3;
  const int ntaps = lo_end + (bs - tail_start);
  const int rec = 4 + H4 + ((ntaps + 3) & ~3);
  const int twf = table_wave_floats((int)n_harmonic, (int)n_bands);
  const int tcos = n_bands == 65 ? kTableCosFloats : 0;
  // frames (waves) per workgroup: 8, fewer when their LDS would not fit (the matrix is read once per workgroup)
  const int tpg = (int)std::max<int64_t>(1, std::min<int64_t>(8, (48 * 1024) / (sizeof(float) * (size_t)twf)));
  if (G == 1 && NF <= INT32_MAX && frame_table_on() && ((size_t)tpg * twf + tcos) * sizeof(float) <= 64 * 1024 &&
      (table = frame_table_buffer(stream, (size_t)NF * rec)) != nullptr) {
    const unsigned tgrid = (unsigned)((NF + tpg - 1) / tpg);
    const size_t tshm = sizeof(float) * ((size_t)tpg * twf + tcos);
#define DDSP_TABLE_LAUNCH(CTRL_, NW_)                                                                      \
    hipLaunchKernelGGL((frame_table_kernel<CTRL_, NW_>), dim3(tgrid), dim3(64 * tpg), tshm, S(stream), f0, param, \
                       raw_magnitudes, bias, controls_out, table, (int)batch, (int)frames, (int)n_harmonic,       \
                       (int)n_bands, bs, sample_rate, lo_end, tail_start, rec, (int)param_ld, (int)mags_ld)
#define DDSP_TABLE_LAUNCH_NW(CTRL_)                \
    switch (nt / 64) {                             \
      case 1: DDSP_TABLE_LAUNCH(CTRL_, 1); break;  \
      case 2: DDSP_TABLE_LAUNCH(CTRL_, 2); break;  \
      case 3: DDSP_TABLE_LAUNCH(CTRL_, 3); break;  \
      default: DDSP_TABLE_LAUNCH(CTRL_, 4); break; \
    }
    if (controls_out) DDSP_TABLE_LAUNCH_NW(true)
    else DDSP_TABLE_LAUNCH_NW(false)
#undef DDSP_TABLE_LAUNCH_NW
#undef DDSP_TABLE_LAUNCH
  }
  // many frames: the persistent, wave-specialised kernel (frame ranges per workgroup)
  const int cus = device_cus();
  const int wpc = persist_wgs_per_cu();
  const int buf_floats = (int)((floats + 8 + 3) & ~(size_t)3);
  const size_t pshm = sizeof(float) * 2 * (size_t)buf_floats;
  uint32_t* tickets = nullptr;
  if (G == 1 && wpc > 0 && cus > 0 && NF <= INT32_MAX && NF >= 2LL * cus * wpc && pshm <= 64 * 1024 &&
      (tickets = persist_tickets(stream)) != nullptr) {
    const int pgrid = cus * wpc;
    const size_t lds = std::max(pshm, persist_lds_floor(wpc));
    const dim3 pblock((unsigned)(nt + 64));
#define DDSP_SYNTH_PERSIST_LAUNCH(RNG_, CTRL_)                                                              \
    hipLaunchKernelGGL((synth_persist_kernel<RNG_, CTRL_, kPersistPad<RNG_, CTRL_>>), dim3(pgrid), pblock, lds, \
                       S(stream), f0, param, raw_magnitudes, bias, RNG_ ? nullptr : noise, k0, k1, o0, o1,      \
                       RNG_ ? counter : nullptr, out, harmonic_out, noise_out, controls_out, (int)batch,          \
                       (int)frames, (int)n_harmonic, (int)n_bands, bs, sample_rate, lo_end, tail_start, pad, buf_floats, \
                       tickets, (int)param_ld, (int)mags_ld)
#define DDSP_SYNTH_PERSIST_TAB_LAUNCH(RNG_)                                                                \
    hipLaunchKernelGGL((synth_persist_kernel<RNG_, false, kPersistTabPad<RNG_>, true>), dim3(pgrid), pblock, lds, \
                       S(stream), f0, table, raw_magnitudes, bias, RNG_ ? nullptr : noise, k0, k1, o0, o1,        \
                       RNG_ ? counter : nullptr, out, harmonic_out, noise_out, nullptr, (int)batch,               \
                       (int)frames, (int)n_harmonic, (int)n_bands, bs, sample_rate, lo_end, tail_start, pad, buf_floats, \
                       tickets, rec, (int)mags_ld)
    if (table) {
      if (noise) DDSP_SYNTH_PERSIST_TAB_LAUNCH(false);
      else DDSP_SYNTH_PERSIST_TAB_LAUNCH(true);
    } else if (noise) {
      if (controls_out) DDSP_SYNTH_PERSIST_LAUNCH(false, true);
      else DDSP_SYNTH_PERSIST_LAUNCH(false, false);
    } else {
      if (controls_out) DDSP_SYNTH_PERSIST_LAUNCH(true, true);
      else DDSP_SYNTH_PERSIST_LAUNCH(true, false);
    }
#undef DDSP_SYNTH_PERSIST_LAUNCH
#undef DDSP_SYNTH_PERSIST_TAB_LAUNCH
    if (!noise && counter) hipLaunchKernelGGL(counter_advance_kernel, dim3(1), dim3(1), 0, S(stream), counter);
    return launch_status();
  }
  const dim3 grid((unsigned)frames, (unsigned)batch), block((unsigned)(nt * G));
  if (table) {
    const int half = (int)n_bands - 1;
    const size_t sshm = sizeof(float) * ((size_t)2 * H4 + bs + ((half + 3) & ~3) + pad + bs);
    if (noise)
      hipLaunchKernelGGL((synth_tab_kernel<false, kTabPad<false>>), grid, dim3(nt), sshm, S(stream), table, noise, k0,
                         k1, o0, o1, nullptr, out, harmonic_out, noise_out, (int)frames, (int)n_harmonic,
                         (int)n_bands, bs, lo_end, tail_start, pad, rec);
    else
      hipLaunchKernelGGL((synth_tab_kernel<true, kTabPad<true>>), grid, dim3(nt), sshm, S(stream), table, nullptr, k0,
                         k1, o0, o1, counter, out, harmonic_out, noise_out, (int)frames, (int)n_harmonic,
                         (int)n_bands, bs, lo_end, tail_start, pad, rec);
    if (!noise && counter) hipLaunchKernelGGL(counter_advance_kernel, dim3(1), dim3(1), 0, S(stream), counter);
    return launch_status();
  }
#define DDSP_SYNTH_FRAME_LAUNCH(RNG_, SPLIT_)                                                             \
  do {                                                                                                  \
    if (controls_out) DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, true);                                       \
    else DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, false);                                                  \
  } while (0)
#define DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, CTRL_)                                                      \
  hipLaunchKernelGGL((synth_frame_kernel<RNG_, SPLIT_, CTRL_>), grid, block, shm, S(stream), f0, param, raw_magnitudes, \
                     bias, RNG_ ? nullptr : noise, k0, k1, o0, o1, RNG_ ? counter : nullptr, out, harmonic_out,  \
                     noise_out, controls_out, (int)frames, (int)n_harmonic, (int)n_bands, bs, sample_rate, lo_end, \
                     tail_start, pad, (int)param_ld, (int)mags_ld)
  if (noise) {
    if (G > 1) DDSP_SYNTH_FRAME_LAUNCH(false, true);
    else DDSP_SYNTH_FRAME_LAUNCH(false, false);
  } else {
    if (G > 1) DDSP_SYNTH_FRAME_LAUNCH(true, true);
    else DDSP_SYNTH_FRAME_LAUNCH(true, false);
  }
#undef DDSP_SYNTH_FRAME_LAUNCH
#undef DDSP_SYNTH_FRAME_LAUNCH_
  if (!noise && counter) hipLaunchKernelGGL(counter_advance_kernel, dim3(1), dim3(1), 0, S(stream), counter);
  return launch_status();
}

int ddsp_hip_set_persistent_workgroups(int per_cu) {
  return g_persist_wpc.exchange(per_cu < 0 ? -1 : per_cu);
}

int ddsp_hip_set_frame_table(int on) {
  return g_frame_table.exchange(on < 0 ? -1 : (on != 0));
}

int ddsp_hip_synth_frames(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                          const float* noise, uint64_t seed, uint64_t offset, float* out,
                          float* harmonic_out, float* noise_out, int64_t batch, int64_t frames,
                          int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                          void* stream) {
  return synth_frames_launch(f0, param, raw_magnitudes, bias, noise, seed, offset, nullptr, out, harmonic_out,
                             noise_out, nullptr, batch, frames, n_harmonic, n_bands, block_size, sample_rate, stream);
}

int ddsp_hip_synth_frames_controls(const float* f0, const float* param, int64_t param_ld, const float* raw_magnitudes,
                                   int64_t magnitudes_ld, float bias, const float* noise, uint64_t seed,
                                   uint64_t offset, float* out, float* harmonic_out, float* noise_out,
                                   float* controls_out, int64_t batch, int64_t frames, int64_t n_harmonic,
                                   int64_t n_bands, int64_t block_size, float sample_rate, void* stream) {
  return synth_frames_launch(f0, param, raw_magnitudes, bias, noise, seed, offset, nullptr, out, harmonic_out,
                             noise_out, controls_out, batch, frames, n_harmonic, n_bands, block_size, sample_rate,
                             stream, param_ld, magnitudes_ld);
}

int ddsp_hip_synth_frames_counter(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                                  uint64_t seed, uint64_t* counter, float* out, int64_t batch, int64_t frames,
                                  int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                  void* stream) {
  if (!counter) return DDSP_HIP_EINVAL;
  return synth_frames_launch(f0, param, raw_magnitudes, bias, nullptr, seed, 0, counter, out, nullptr, nullptr,
                             nullptr, batch, frames, n_harmonic, n_bands, block_size, sample_rate, stream);
}

size_t ddsp_hip_synth_reverb_workspace_size(int64_t batch, int64_t frames, int64_t block_size) {
  if (batch < 1 || frames < 1 || block_size < 1) return 0;
  return upols_workspace_bytes(batch, frames * block_size, true);
}

int ddsp_hip_synth_reverb_spectra(const float* f0, const float* param, int64_t param_ld, const float* raw_magnitudes,
                                  int64_t magnitudes_ld, float bias, const float* noise, uint64_t seed, uint64_t offset,
                                  float* spectra, size_t spectra_bytes, int64_t batch, int64_t frames,
                                  int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                  void* stream) {
  if (param_ld < 0) param_ld = n_harmonic + 1;
  if (magnitudes_ld < 0) magnitudes_ld = n_bands;
  if (batch < 0 || frames < 0 || n_harmonic < 1 || n_bands < 2 || block_size < 4) return DDSP_HIP_EINVAL;
  if (param_ld < n_harmonic + 1 || magnitudes_ld < n_bands || param_ld > INT32_MAX || magnitudes_ld > INT32_MAX)
    return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!f0 || !param || !raw_magnitudes || !spectra) return DDSP_HIP_EINVAL;
  // envelope: whole frames per 2048-sample block, one 64..256-thread group per frame, 2 rows x
  // (2048 / bs) groups of at least the transform's 512 threads and at most 1024
  const int bs = (int)block_size;
  if (bs % 4 || kP % bs || n_harmonic > 1024 || n_bands > 1025 || batch > 2 * 65535 || frames > INT32_MAX)
    return DDSP_HIP_ERANGE;
  const int NT = std::max(64, ((bs / 4 + 63) / 64) * 64);
  const int threads = 2 * (kP / bs) * NT;
  if (threads < kN / 8 || threads > 1024) return DDSP_HIP_ERANGE;
  const FrameShape fs = frame_shape(n_harmonic, n_bands, bs);
  const int gfloats = (int)((fs.floats + 3) & ~(size_t)3);
  const size_t shm = std::max(sizeof(float) * (size_t)gfloats * (threads / NT), sizeof(float2) * (kN + kN / 16));
  if (shm > 160 * 1024) return DDSP_HIP_ERANGE;
  const int64_t n = frames * block_size;
  const int64_t nb = upols_blocks(n), npairs = (batch + 1) / 2;
  if (nb > INT32_MAX) return DDSP_HIP_ERANGE;
  if (spectra_bytes < upols_spectra_bytes(batch, n)) return DDSP_HIP_EWORKSPACE;
  float2* Z = reinterpret_cast<float2*>(spectra);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
#define DDSP_SYNTH_FORWARD_LAUNCH(RNG_)                                                                        \
  hipLaunchKernelGGL((synth_forward_kernel<RNG_, kSynthForwardPad<RNG_>>), dim3((unsigned)nb, (unsigned)npairs),     \
                     dim3(threads), shm, S(stream), f0, param, raw_magnitudes, bias, RNG_ ? nullptr : noise, k0, k1, \
                     o0, o1, nullptr, Z, (int)batch, (int)frames, (int)n_harmonic, (int)n_bands, bs, sample_rate,    \
                     fs.lo_end, fs.tail_start, fs.pad, gfloats, NT, (int)nb, (int)param_ld, (int)magnitudes_ld)
  if (noise) DDSP_SYNTH_FORWARD_LAUNCH(false);
  else DDSP_SYNTH_FORWARD_LAUNCH(true);
#undef DDSP_SYNTH_FORWARD_LAUNCH
  return launch_status();
}

int ddsp_hip_synth_reverb(const float* f0, const float* param, int64_t param_ld, const float* raw_magnitudes,
                          int64_t magnitudes_ld, float bias, const float* noise, uint64_t seed, uint64_t offset,
                          const float* spectrum, int64_t ir_length, float* out, void* workspace,
                          size_t workspace_bytes, int64_t batch, int64_t frames, int64_t n_harmonic, int64_t n_bands,
                          int64_t block_size, float sample_rate, void* stream) {
  if (batch < 0 || frames < 0 || block_size < 4 || ir_length < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!spectrum || !out) return DDSP_HIP_EINVAL;
  const int64_t n = frames * block_size;
  if (!workspace || workspace_bytes < upols_workspace_bytes(batch, n, true)) return DDSP_HIP_EWORKSPACE;
  const size_t zb = upols_spectra_bytes(batch, n);
  int st = ddsp_hip_synth_reverb_spectra(f0, param, param_ld, raw_magnitudes, magnitudes_ld, bias, noise, seed, offset,
                                         reinterpret_cast<float*>(workspace), zb, batch, frames, n_harmonic, n_bands,
                                         block_size, sample_rate, stream);
  if (st) return st;
  return upols_apply_spectra(reinterpret_cast<const float2*>(workspace), batch, n, spectrum, std::min(ir_length, n),
                             false, out, reinterpret_cast<float2*>(reinterpret_cast<char*>(workspace) + zb), stream);
}

}  // extern "C"
