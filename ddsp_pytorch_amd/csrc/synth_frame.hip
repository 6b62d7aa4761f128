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

#include "common.h"
#include "noise_dsp.h"

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
// (the dicts DDSPDecoder.forward returns) to ctrl_out.  PREFIX: read the frame's phase prefix from
// prefix[] (long renders) instead of summing the earlier frames; its own instantiations, so the
// training / serving shapes run the code without the branch (1.9% of the kernel, same-box A/B).
template <bool RNG, bool SPLIT, bool PAD, bool CTRL, bool PREFIX>
__device__ __forceinline__ bool frame_synth(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float* __restrict__ ctrl_out, int B, int F, int H, int NB, int bs,
    float sr, int lo_end, int tail_start, int pad, int f, int b, int tid, int NT, float4* smem4, double* red,
    int w0, float (&acc)[4], float (&nz)[4], int& j0_out, int ldp, int ldm, const double* __restrict__ prefix) {
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
  if (PREFIX) {  // long renders: the item's exact frame prefix, precomputed (ddsp_hip_frame_phase_prefix)
    if (tid == 0) part_s = prefix[frame];
  } else {       // O(f) per frame: fine for the few hundred frames of a training / serving batch
    for (int g = tid; g < f; g += NT) part_s += (double)bs * (double)phase_inc(f0b[g], sr);
  }
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
    // irfft taps (core.py:150): ir[m] = (A0 + (-1)^m A64 + 2 (O(m) + E(m))) / 128 with O the odd-k and E
    // the even-k (2..62) cosine sums.  Since cos(2 pi k (64 - m) / 128) = (-1)^k cos(2 pi k m / 128),
    // ir[64 - m] = (A0 + (-1)^m A64 + 2 (E(m) - O(m))) / 128: lane 2m + p of the first wave sums one
    // parity (32 terms, k ascending as before) for m in [0, 32) and the lane pair exchanges its sums by
    // DPP, so the wave issues 32 multiply-adds instead of 63 for all 64 taps; the second wave sums
    // ir[32] across its lanes
    if (tid < 64) {
      const int m = tid >> 1, p = tid & 1;
      // k = 2j + p: even lanes k = 0 (a zero term), 2, ..., 62; odd lanes 1, ..., 63.  One base per
      // lane and fully unrolled constant offsets (128 floats per j in the table, 2 in A): a load and
      // an FMA per term, no per-term address arithmetic (the PMC probe counted ~5 VALU per term)
      const float* cm = kIrCos128 + p * 64 + m;
      const float* ap = A + p;
      float sum = fmaf(p ? ap[0] : 0.0f, cm[0], 0.0f);
#pragma unroll
      for (int j = 1; j < 32; ++j) sum = fmaf(ap[2 * j], cm[128 * j], sum);
      const float other = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sum), 0xB1, 0xF, 0xF, true));
      const float a0 = A[0] + ((m & 1) ? -A[64] : A[64]);
      if (p == 0) ir[m] = (a0 + 2.0f * (other + sum)) * (1.0f / 128.0f);       // odd + even
      else ir[64 - m] = (a0 + 2.0f * (other - sum)) * (1.0f / 128.0f);        // even - odd
    } else if (tid < 128) {  // tap n/2 = 32: A0 + A64 + 2 sum_k A_k cos(pi k / 2)
      const int k = tid - 64;
      float t = k >= 1 ? A[k] * kIrCos128[k * 64 + 32] : 0.0f;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (tid == 64) ir[32] = (A[0] + A[64] + 2.0f * t) * (1.0f / 128.0f);
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
  // With n/2 = 64 (65 bands) and h zero for the 63 positions below tail_start (written in phase 3), the
  // 64 x 64 tap triangle runs unpredicated (the taps past l add fma(0, x, c) = c) and register-blocked on
  // the first wave: lane 4g + q computes outputs 4g..4g+3 over the taps d in [16q, 16q + 16) from 4 + 5
  // ds_read_b128 (x[16q..], h[tail_start + 4g - 16q - 16 ..]), then the four tap quarters are summed across
  // the lane quad by DPP (quad_perm): ~90 wave-instructions instead of 64 x 3 for one output per lane.
  if (bs - tail_start == 64 && bs - 127 >= lo_end) {
    if (tid < 64) {
      const int g = tid >> 2, q = tid & 3;
      const float4* x4 = reinterpret_cast<const float4*>(x) + 4 * q;
      const float4* h4 = reinterpret_cast<const float4*>(h + tail_start + 4 * g - 16 * q - 16);
      float xv[16], hv[20];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = x4[i];
        xv[4 * i] = v.x; xv[4 * i + 1] = v.y; xv[4 * i + 2] = v.z; xv[4 * i + 3] = v.w;
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const float4 v = h4[i];
        hv[4 * i] = v.x; hv[4 * i + 1] = v.y; hv[4 * i + 2] = v.z; hv[4 * i + 3] = v.w;
      }
      float c[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      // output l = 4g + r, tap d = 16q + dd: h[tail_start + l - d] = hv[16 + r - dd] (hv[0] unused)
#pragma unroll
      for (int dd = 0; dd < 16; ++dd) {
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = fmaf(hv[16 + r - dd], xv[dd], c[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        c[r] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(c[r]), 0xB1, 0xF, 0xF, true));  // q ^ 1
        c[r] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(c[r]), 0x4E, 0xF, 0xF, true));  // q ^ 2
      }
      if (q == 0) *reinterpret_cast<float4*>(tail + 4 * g) = make_float4(c[0], c[1], c[2], c[3]);
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
  float4 y = fir4(h, x, j0, lo_end, bs, bs);  // taps [0, lo_end); the wrapped taps are in tail[]
  nz[0] = y.x;
  nz[1] = y.y;
  nz[2] = y.z;
  nz[3] = y.w;
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (j0 + s >= tail_start) nz[s] += tail[j0 + s - tail_start];
  return true;
}

template <bool RNG, bool SPLIT, bool CTRL, bool PREFIX>
__global__ void __launch_bounds__(256) synth_frame_kernel(
    const float* __restrict__ f0, const float* __restrict__ param, const float* __restrict__ mags,
    float bias, const float* __restrict__ noise, uint32_t k0, uint32_t k1, uint32_t off0, uint32_t off1,
    const uint64_t* __restrict__ counter, float* __restrict__ out, float* __restrict__ harm_out,
    float* __restrict__ noise_out, float* __restrict__ ctrl_out, int F, int H,
    int NB, int bs, float sr, int lo_end, int tail_start, int pad, int ldp, int ldm, const double* __restrict__ prefix) {
  extern __shared__ float4 smem4[];
  __shared__ double red[32];
  float acc[4], nz[4];
  int j0;
  if (!frame_synth<RNG, SPLIT, /*PAD=*/CTRL, CTRL, PREFIX>(f0, param, mags, bias, noise, k0, k1, off0, off1, counter, ctrl_out,
                                      (int)gridDim.y, F, H, NB, bs, sr, lo_end, tail_start, pad, blockIdx.x,
                                      blockIdx.y, threadIdx.x, blockDim.x, smem4, red, 0, acc, nz, j0, ldp, ldm,
                                      prefix))
    return;
  const int64_t o = ((int64_t)blockIdx.y * F + blockIdx.x) * bs + j0;
  if (harm_out) *reinterpret_cast<float4*>(harm_out + o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (noise_out) *reinterpret_cast<float4*>(noise_out + o) = make_float4(nz[0], nz[1], nz[2], nz[3]);
  *reinterpret_cast<float4*>(out + o) =
      make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121
}

__global__ void counter_advance_kernel(uint64_t* counter) { *counter += 1; }

// frame_prefix[b * F + f] = sum_{g < f} bs * inc_g (exclusive), one workgroup per item: every thread sums a
// contiguous run of frames, the runs' totals are scanned in LDS; every partial sum is an exact fp64 value
// (the summands are fp32 increments scaled by bs, the span stays within 53 bits), so the order is free
__global__ void __launch_bounds__(256) frame_prefix_kernel(const float* __restrict__ f0, int F, int bs, float sr,
                                                           double* __restrict__ prefix) {
  __shared__ double tot[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* f0b = f0 + (int64_t)b * F;
  double* pb = prefix + (int64_t)b * F;
  const int per = (F + 255) / 256, g0 = tid * per, g1 = min(g0 + per, F);
  double run = 0.0;
  for (int g = g0; g < g1; ++g) run += (double)bs * (double)phase_inc(f0b[g], sr);
  tot[tid] = run;
  __syncthreads();
  if (tid == 0) {
    double acc = 0.0;
    for (int i = 0; i < 256; ++i) {
      const double v = tot[i];
      tot[i] = acc;
      acc += v;
    }
  }
  __syncthreads();
  double acc = tot[tid];
  for (int g = g0; g < g1; ++g) {
    pb[g] = acc;
    acc += (double)bs * (double)phase_inc(f0b[g], sr);
  }
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

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
                               void* stream, int64_t param_ld = -1, int64_t mags_ld = -1,
                               const double* prefix = nullptr) {
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
  int G = batch * frames < 512 && !prefix ? std::max(1, std::min(4, 256 / nt)) : 1;
  if (sizeof(float) * (floats + (size_t)bs) > 120 * 1024) G = 1;
  const size_t shm = sizeof(float) * (floats + (G > 1 ? (size_t)bs : 0));
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t o0 = (uint32_t)offset, o1 = (uint32_t)(offset >> 32);
  const dim3 grid((unsigned)frames, (unsigned)batch), block((unsigned)(nt * G));
#define DDSP_SYNTH_FRAME_LAUNCH(RNG_, SPLIT_)                                                             \
  do {                                                                                                  \
    if (controls_out) DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, true);                                       \
    else DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, false);                                                  \
  } while (0)
#define DDSP_SYNTH_FRAME_LAUNCH_(RNG_, SPLIT_, CTRL_)                                                      \
  do {                                                                                                  \
    if (!SPLIT_ && prefix) DDSP_SYNTH_FRAME_LAUNCH_P(RNG_, false, CTRL_, true);                            \
    else DDSP_SYNTH_FRAME_LAUNCH_P(RNG_, SPLIT_, CTRL_, false);                                            \
  } while (0)
#define DDSP_SYNTH_FRAME_LAUNCH_P(RNG_, SPLIT_, CTRL_, PREFIX_)                                            \
  hipLaunchKernelGGL((synth_frame_kernel<RNG_, SPLIT_, CTRL_, PREFIX_>), grid, block, shm, S(stream), f0, param, raw_magnitudes, \
                     bias, RNG_ ? nullptr : noise, k0, k1, o0, o1, RNG_ ? counter : nullptr, out, harmonic_out,  \
                     noise_out, controls_out, (int)frames, (int)n_harmonic, (int)n_bands, bs, sample_rate, lo_end, \
                     tail_start, pad, (int)param_ld, (int)mags_ld, prefix)
  if (noise) {
    if (G > 1) DDSP_SYNTH_FRAME_LAUNCH(false, true);
    else DDSP_SYNTH_FRAME_LAUNCH(false, false);
  } else {
    if (G > 1) DDSP_SYNTH_FRAME_LAUNCH(true, true);
    else DDSP_SYNTH_FRAME_LAUNCH(true, false);
  }
#undef DDSP_SYNTH_FRAME_LAUNCH
#undef DDSP_SYNTH_FRAME_LAUNCH_
#undef DDSP_SYNTH_FRAME_LAUNCH_P
  if (!noise && counter) hipLaunchKernelGGL(counter_advance_kernel, dim3(1), dim3(1), 0, S(stream), counter);
  return launch_status();
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

int ddsp_hip_synth_frames_controls_prefix(const float* f0, const float* param, int64_t param_ld,
                                          const float* raw_magnitudes, int64_t magnitudes_ld, float bias,
                                          const float* noise, uint64_t seed, uint64_t offset, float* out,
                                          float* harmonic_out, float* noise_out, float* controls_out,
                                          const double* frame_prefix, int64_t batch, int64_t frames,
                                          int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                          void* stream) {
  return synth_frames_launch(f0, param, raw_magnitudes, bias, noise, seed, offset, nullptr, out, harmonic_out,
                             noise_out, controls_out, batch, frames, n_harmonic, n_bands, block_size, sample_rate,
                             stream, param_ld, magnitudes_ld, frame_prefix);
}

int ddsp_hip_frame_phase_prefix(const float* f0, int64_t batch, int64_t frames, int64_t block_size, float sample_rate,
                                double* frame_prefix, void* stream) {
  if (batch < 0 || frames < 0 || block_size < 1 || !(sample_rate > 0)) return DDSP_HIP_EINVAL;
  if (batch == 0 || frames == 0) return DDSP_HIP_OK;
  if (!f0 || !frame_prefix) return DDSP_HIP_EINVAL;
  if (batch > INT32_MAX || frames > INT32_MAX || block_size > INT32_MAX) return DDSP_HIP_ERANGE;
  hipLaunchKernelGGL(frame_prefix_kernel, dim3((unsigned)batch), dim3(256), 0, S(stream), f0, (int)frames,
                     (int)block_size, sample_rate, frame_prefix);
  return launch_status();
}

int ddsp_hip_synth_frames_counter(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                                  uint64_t seed, uint64_t* counter, float* out, int64_t batch, int64_t frames,
                                  int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                  void* stream) {
  if (!counter) return DDSP_HIP_EINVAL;
  return synth_frames_launch(f0, param, raw_magnitudes, bias, nullptr, seed, 0, counter, out, nullptr, nullptr,
                             nullptr, batch, frames, n_harmonic, n_bands, block_size, sample_rate, stream);
}

}  // extern "C"

