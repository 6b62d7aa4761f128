// Uniformly partitioned FFT convolution (UPOLS) for gfx950.
//
// Replaces the reference's one-shot 2T-point FFT convolution (ddsp/core.py:169-176, used by
// Reverb.forward, ddsp/models/modules.py:28-35) for long signals and kernels.  Only the first
// T outputs of the causal linear convolution are kept, so any exact method is a faithful
// restatement; this one is laid out for the MI355X memory system:
//
//   partition size P = 2048, FFT size N = 4096 (= 16^3: three radix-16 Stockham passes, one
//   workgroup of 256 threads per transform, 16 points per thread, 34 KB of LDS);
//   two real rows sharing one kernel are packed as z = x_a + i*x_b: the kernel is real, so
//   z (*) h = (x_a (*) h) + i (x_b (*) h) — one complex FFT serves two rows with no
//   Hermitian post-processing;
//   the overlap sits on the KERNEL side: the input blocks are zero-padded, the kernel windows
//   overlap by half (q = 0..Q, Q = ceil(L/P), h_{-1} = h_Q = 0):
//   kernel:   G_q = FFT_N([h_{q-1}, h_q]) / N                   (computed once per IR)
//   forward:  Z_b = FFT_N([x_b, 0])                             (upols_forward_kernel)
//   MAC:      Y_b = sum_{q=0..Q} Z_{b-q} G_q   per frequency bin (upols_mac_ring_kernel)
//   inverse:  y[bP, (b+1)P) = last P points of IFFT_N(Y_b)      (upols_inverse_kernel)
//   (circular convolution of [x_{b-q}, 0] with [h_{q-1}, h_q]: its second half holds exactly the
//   terms h[tau] x[bP + n - tau] with tau in ((q-1)P + n, qP + n], so the Q+1 terms cover every
//   tau once.)  Against the input-overlap form (X_b = FFT([x_{b-1}, x_b]) = Z_{b-1} + (-1)^f Z_b,
//   Q kernel spectra) each input sample is read once instead of twice, for one more MAC term.
//
// HBM traffic per real output sample: x read (4 B), Z write/read (16 B), Y write/read (16 B),
// y write (4 B).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "upols.h"
#include "fft_radix.h"

namespace ddsp {
namespace {

constexpr int kNT = 256;            // threads per transform
constexpr int kPad = kN + kN / 16;  // LDS float2 slots: one pad slot per 16 (bank spreading)

// Full 4096-point transform (three radix-16 Stockham passes, Ns = 1, 16, 256):
// v holds in[j + 256 r] on entry and out[j + 256 r] on exit.
template <bool INV>
__device__ __forceinline__ void fft4096(float2 (&v)[16], float2* lds, int j = threadIdx.x) {
  // pass twiddle steps: k * N/(Ns*16) with k = j mod Ns
  const Tw4 tw2 = load_tw<INV>((j & 15) * 16);
  const Tw4 tw3 = load_tw<INV>(j);
  dft16<INV>(v);
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[lds_idx(out_index(j, 1, r))] = v[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = lds[lds_idx(j + 256 * r)];
  __syncthreads();
  apply_tw(v, tw2);
  dft16<INV>(v);
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[lds_idx(out_index(j, 16, r))] = v[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = lds[lds_idx(j + 256 * r)];
  apply_tw(v, tw3);
  dft16<INV>(v);  // Ns = 256: output index == j + 256 r (coalesced)
}

// Complex multiply-accumulate as two packed FMAs (v_pk_fma_f32: two fp32 FMAs per lane per
// instruction): acc += a * b = a.x * (b.x, b.y) + a.y * (-b.y, b.x), with b and its rotation
// formed once per partition and shared by every accumulator.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void cmac(v2f& acc, float2 a, v2f b, v2f b_rot) {
  acc = __builtin_elementwise_fma((v2f){a.x, a.x}, b, acc);
  acc = __builtin_elementwise_fma((v2f){a.y, a.y}, b_rot, acc);
}

// MAC shape: the register-ring kernel, 25 output blocks per thread, operands prefetched 3 steps
// ahead, a G ring of 3 (25.7-26.7 us at config 2 against 29.3 us for the shifting
// window it replaced)
constexpr int kRingBlk = 25;
constexpr int kRingPF = 3;
constexpr int kRingGR = 3;

// rows of the packed signal: pair -> (row_a, row_b or -1)
__device__ __forceinline__ void pair_rows(int pair, int rows, int pairing, int& ra, int& rb) {
  if (pairing) {
    ra = 2 * pair;
    rb = 2 * pair + 1 < rows ? 2 * pair + 1 : -1;
  } else {
    ra = pair;
    rb = -1;
  }
}

// X[pair][b][:] = FFT(z[(b+off)P, (b+off+2)P)) with one half zeroed; grid (nb, npairs).
//   off = 0, zero_half = 2: Z_b = FFT([z_b, 0]), the zero-padded input blocks (forward);
//   off = -1, zero_half = 1: FFT([0, z_b]), the adjoint of the inverse transform's "keep the
//   second half" (backward).  reverse: z read time-reversed (z'[s] = z[T-1-s], the transposed
//   convolution of the input gradient).
__device__ __forceinline__ void forward_block(const float* __restrict__ x, int64_t ld, int64_t T, int rows,
                                              int pairing, int nb, int off, int zero_half, int reverse,
                                              float2* __restrict__ X, int b, int pair, float2* lds) {
  const int j = threadIdx.x;
  int ra, rb;
  pair_rows(pair, rows, pairing, ra, rb);
  const float* xa = x + (int64_t)ra * ld;
  const float* xb = rb >= 0 ? x + (int64_t)rb * ld : nullptr;
  const int64_t s0 = (int64_t)(b + off) * kP;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = s0 + j + 256 * r;
    const bool ok = s >= 0 && s < T && !(zero_half == 1 && r < 8) && !(zero_half == 2 && r >= 8);
    const int64_t si = reverse ? T - 1 - s : s;
    v[r] = make_float2(ok ? xa[si] : 0.0f, (ok && xb) ? xb[si] : 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = X + ((int64_t)pair * nb + b) * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
}

__global__ void __launch_bounds__(kNT) upols_forward_kernel(const float* __restrict__ x, int64_t ld,
                                                            int64_t T, int rows, int pairing, int nb,
                                                            int off, int zero_half, int reverse,
                                                            float2* __restrict__ X) {
  __shared__ float2 lds[kPad];
  forward_block(x, ld, T, rows, pairing, nb, off, zero_half, reverse, X, blockIdx.x, blockIdx.y, lds);
}

// The reverb's IR spectrum cached on the device and validated there on every call (Reverb.forward,
// modules.py:21-35, rebuilds it every call; a host-side cache keyed on parameter versions misses
// writes through .data).  Per kernel window q the cache keeps the spectrum G_q and a snapshot of the
// exact inputs it was built from — the noise taps of the window [(q-1)P, (q+1)P) ∩ [0, klen) bit for
// bit, decay, wet, the sample rate and klen + 1 (0 in a zero-filled cache: nothing valid yet).  The
// window's workgroup compares them with the current parameters and rebuilds G_q (the arithmetic of
// upols_impulse_spectrum_kernel, bit for bit) only when one differs or `force` is set.  Each
// window's snapshot is its own (windows overlap by P taps), so no two workgroups write one word.
constexpr int kSnapWords = 2 * kP + 4;

__device__ __forceinline__ void ir_window(const float* __restrict__ noise, const float* __restrict__ decay,
                                          const float* __restrict__ wet, int64_t klen, float sr, int force, int q,
                                          float2* __restrict__ Hs, uint32_t* __restrict__ snap, float2* lds) {
  const int j = threadIdx.x;
  uint32_t* sq = snap + (int64_t)q * kSnapWords;
  float nv[16];
  bool diff = false;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = (int64_t)(q - 1) * kP + j + 256 * r;
    const bool in = s >= 0 && s < klen;
    nv[r] = in ? noise[s] : 0.0f;
    diff |= in && __float_as_uint(nv[r]) != sq[j + 256 * r];
  }
  const float dec = decay[0], wt = wet[0];
  if (j == 0)
    diff |= sq[2 * kP] != __float_as_uint(dec) || sq[2 * kP + 1] != __float_as_uint(wt) ||
            sq[2 * kP + 2] != __float_as_uint(sr) || sq[2 * kP + 3] != (uint32_t)(klen + 1);
  if (!__syncthreads_or(diff || force)) return;  // the cached G_q is this window's spectrum
  const float d = -dec;
  const float sp = d > 20.0f ? d : log1pf(expf(d));  // softplus(-decay), torch's threshold 20
  const float neg = -sp;
  const float w = 1.0f / (1.0f + expf(-wt));
  const float inv_n = 1.0f / (float)kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = (int64_t)(q - 1) * kP + j + 256 * r;
    float h = 0.0f;
    if (s >= 0 && s < klen) {
      const float t = (float)s / sr;
      const float env = expf((neg * t) * 500.0f);
      h = s == 0 ? 1.0f : (nv[r] * env) * w;
    }
    v[r] = make_float2(h * inv_n, 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = Hs + (int64_t)q * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = (int64_t)(q - 1) * kP + j + 256 * r;
    if (s >= 0 && s < klen) sq[j + 256 * r] = __float_as_uint(nv[r]);
  }
  if (j == 0) {
    sq[2 * kP] = __float_as_uint(dec);
    sq[2 * kP + 1] = __float_as_uint(wt);
    sq[2 * kP + 2] = __float_as_uint(sr);
    sq[2 * kP + 3] = (uint32_t)(klen + 1);
  }
}

// The reverb's forward transform (Z_b = FFT([x_b, 0]), grid rows y >= 1: pair y - 1) with the IR cache's
// validation in the same launch (row y = 0, x = window — dispatched first, so the usually trivial
// validation workgroups do not trail the transforms): the MAC that follows reads a spectrum that is
// current, and no launch is added to the step.  npairs == 0: the validation alone.
__global__ void __launch_bounds__(kNT) upols_forward_ir_kernel(
    const float* __restrict__ x, int64_t T, int rows, int nb, float2* __restrict__ X, const float* __restrict__ noise,
    const float* __restrict__ decay, const float* __restrict__ wet, int64_t klen, float sr, int force, int QG,
    float2* __restrict__ Hs, uint32_t* __restrict__ snap) {
  __shared__ float2 lds[kPad];
  if (blockIdx.y == 0) {
    if ((int)blockIdx.x < QG) ir_window(noise, decay, wet, klen, sr, force, blockIdx.x, Hs, snap, lds);
  } else if ((int)blockIdx.x < nb) {
    forward_block(x, T, T, rows, 1, nb, 0, 2, 0, X, blockIdx.x, blockIdx.y - 1, lds);
  }
}

// 8-byte load at byte offset voff of one spectrum row through a raw buffer descriptor (stride 0,
// `bytes` records; offsets at or past `bytes` read as zero).  The row pointer and size are
// wave-uniform, so the descriptor lives in SGPRs.
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr int kBufferWord3 = 0x00020000;  // gfx9 raw-buffer DATA_FORMAT word
template <int AUX = 0>  // cache-policy bits of the load (gfx950: 1 sc0, 2 nt, 16 sc1)
__device__ __forceinline__ float2 row_load(const float2* row, int bytes, int voff) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(row), (short)0, bytes, kBufferWord3);
  const i32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, AUX);
  return make_float2(__int_as_float(v.x), __int_as_float(v.y));
}

// G[row][q][:] = FFT(h[row][(q-1)P, (q+1)P) (zero outside [0, klen))) / N, q = 0..Q;
// grid (Q + 1, krows)
__global__ void __launch_bounds__(kNT) upols_kernel_spectrum_kernel(const float* __restrict__ h,
                                                                    int64_t ld, int64_t klen, int QG,
                                                                    float2* __restrict__ Hs) {
  __shared__ float2 lds[kPad];
  const int q = blockIdx.x, row = blockIdx.y, j = threadIdx.x;
  const float* hr = h + (int64_t)row * ld;
  const float inv_n = 1.0f / (float)kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = (int64_t)(q - 1) * kP + j + 256 * r;
    v[r] = make_float2((s >= 0 && s < klen) ? hr[s] * inv_n : 0.0f, 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = Hs + ((int64_t)row * QG + q) * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
}

// Reverb.build_impulse (modules.py:21-26) fused into the IR's partition spectra (modules.py:30-35):
// G[q][:] = FFT(imp[(q-1)P, (q+1)P)) / N with imp[i] = noise[i] exp(-softplus(-decay) t 500) sigmoid(wet),
// t = fl32(i / sr), imp[0] = 1, zero at or past klen — the arithmetic of reverb.hip's
// build_impulse_kernel per tap, so the spectra are those of upols_spectrum(build_impulse(...)) bit for bit.
// One launch instead of two (the impulse never goes to HBM); grid (Q + 1)
__global__ void __launch_bounds__(kNT) upols_impulse_spectrum_kernel(const float* __restrict__ noise,
                                                                     const float* __restrict__ decay,
                                                                     const float* __restrict__ wet, int64_t klen,
                                                                     float sr, int QG, float2* __restrict__ Hs) {
  __shared__ float2 lds[kPad];
  const int q = blockIdx.x, j = threadIdx.x;
  const float d = -decay[0];
  const float sp = d > 20.0f ? d : log1pf(expf(d));  // softplus(-decay), torch's threshold 20
  const float neg = -sp;
  const float w = 1.0f / (1.0f + expf(-wet[0]));
  const float inv_n = 1.0f / (float)kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = (int64_t)(q - 1) * kP + j + 256 * r;
    float h = 0.0f;
    if (s >= 0 && s < klen) {
      const float t = (float)s / sr;
      const float env = expf((neg * t) * 500.0f);
      h = s == 0 ? 1.0f : (noise[s] * env) * w;
    }
    v[r] = make_float2(h * inv_n, 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = Hs + (int64_t)q * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
}

// The same sums with the Z window as a register ring indexed statically.  The p loop is unrolled by
// the ring size R = BLK + PF - 1, so the slot (m - b0) mod R of block m is a compile-time register
// at every unrolled step and the window never shifts (no v_mov).  After step p's products, block
// b0 - p - PF is loaded into the slot step p freed (block b0 + BLK - 1 - p), and G_{p+PF} into a
// G ring of GR >= PF slots (GR | R): every operand is loaded PF steps before its first use.  The
// unrolled rounds carry no per-step guards (guards made the compiler enter the round through a
// jump table, whose joins forced a wait on every load at every step): steps past the last useful
// one read the zero spectra of out-of-range descriptors (G_q, q >= Q; Z_m, m < 0) and add exact
// zeros.  grid (N/256, ceil(nb/BLK), npairs)
template <int BLK, int PF, int GR>
__global__ void __launch_bounds__(kNT) upols_mac_ring_kernel(const float2* __restrict__ X,
                                                             const float2* __restrict__ Hs,
                                                             int64_t h_pair_stride, int nb, int Q,
                                                             float2* __restrict__ Y) {
  constexpr int R = BLK + PF - 1;
  static_assert(PF >= 1 && R % GR == 0 && GR >= PF, "ring shapes");
  constexpr int kRow = kN * (int)sizeof(float2);
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int b0 = nb - (int)(gridDim.y - blockIdx.y) * BLK;
  const int pair = blockIdx.z;
  // Every spectrum row is read through a buffer descriptor built in SGPRs for that row (base =
  // the row, lane offset = 8 f): no per-lane address arithmetic, and rows outside the signal or
  // the kernel are descriptors with no records, whose loads return 0 without a select.
  const float2* Xrow = X + (int64_t)pair * nb * kN;
  const float2* Hrow = Hs + (int64_t)pair * h_pair_stride;
  const int voff = f * (int)sizeof(float2);
  float2 ring[R], g[GR];
  v2f acc[BLK];
// Cache policy of the input-spectra (Z) and kernel-spectra (G) loads: non-temporal (nt; G also
// sc0).  With the default policy the fused synthesis kernel that follows the reverb in the next
// step runs at ~2.2 instead of ~2.38 GHz: the G loads' nt bit removes that, the Z
// loads' adds a little (config-2 step 223.8-226.3 -> 208.3 us, tools/exp_timing.py, same box).
// A/B builds override them (-DDDSP_MAC_ZAUX=0 -DDDSP_MAC_GAUX=0: the round-2 policy).
#ifndef DDSP_MAC_ZAUX
#define DDSP_MAC_ZAUX 2
#endif
#ifndef DDSP_MAC_GAUX
#define DDSP_MAC_GAUX 3
#endif
  auto zload = [&](int m, float2& dst) {
    dst = row_load<DDSP_MAC_ZAUX>(Xrow + (int64_t)max(m, 0) * kN, m >= 0 ? kRow : 0, voff);
  };
  auto gload = [&](int q, float2& dst) {
    dst = row_load<DDSP_MAC_GAUX>(Hrow + (int64_t)min(q, Q - 1) * kN, q < Q ? kRow : 0, voff);
  };
#pragma unroll
  for (int d = 0; d < BLK; ++d) {
    acc[d] = (v2f){0.f, 0.f};
    zload(b0 + d, ring[d]);
  }
#pragma unroll
  for (int j = 1; j < PF; ++j) zload(b0 - j, ring[R - j]);
#pragma unroll
  for (int j = 0; j < PF; ++j) gload(j, g[j]);
  const int pmax = min(Q, b0 + BLK);
  for (int pb = 0; pb < pmax; pb += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int p = pb + u;
      const float2 h = g[u % GR];
      const v2f hb = {h.x, h.y}, hr = {-h.y, h.x};
#pragma unroll
      for (int d = 0; d < BLK; ++d) cmac(acc[d], ring[(d - u + R) % R], hb, hr);
      gload(p + PF, g[(u + PF) % GR]);
      zload(b0 - p - PF, ring[(BLK - 1 - u + R) % R]);
      // keep the scheduler from sinking the loads toward their uses (it did, to cut register
      // live ranges, which turned the prefetch into a wait on every load)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float2* Yp = Y + (int64_t)pair * nb * kN + f;
#pragma unroll
  for (int d = 0; d < BLK; ++d)
    if (b0 + d >= 0) Yp[(int64_t)(b0 + d) * kN] = make_float2(acc[d].x, acc[d].y);
}


// The same sums for a whole pair row in one thread (nb == NBK, Q <= NQ): every Z_m and G_q of the bin is
// loaded once and stays in registers (the ring kernel's two 25-block chunks re-read ~1.5x of Z: 122 vs
// 104 MB at config 2), and the outputs stream — step b issues the loads of step b + PF (Z_{b+PF},
// G_{b+PF}), then forms Y_b = sum_{q <= min(b, NQ-1)} Z_{b-q} G_q from operands already in registers and
// stores it, so loads, products and stores overlap inside every wave (166 VGPRs; grid N/256 x npairs:
// one round at 2 waves per SIMD).  Same-box A/Bs at config 2 (profiles/r05_ab_mac_vjp.log): 24.5-24.8 us
// against 32.1-32.4 us for the ring kernel on boxes where the ring runs 32 us (step -3.8 / -6.4 us), equal
// (25.0 vs 24.9-25.0 us) where the ring runs 25 us.  The ring kernel serves the other shapes.
template <int NBK, int NQ, int PF>
__global__ void __launch_bounds__(kNT) upols_mac_stream_kernel(const float2* __restrict__ X,
                                                               const float2* __restrict__ Hs,
                                                               int64_t h_pair_stride, int nb, int Q,
                                                               float2* __restrict__ Y) {
  constexpr int kRow = kN * (int)sizeof(float2);
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int pair = blockIdx.y;
  const float2* Xrow = X + (int64_t)pair * nb * kN;
  const float2* Hrow = Hs + (int64_t)pair * h_pair_stride;
  const int voff = f * (int)sizeof(float2);
  float2 z[NBK], g[NQ];
  auto zload = [&](int m) { z[m] = row_load<DDSP_MAC_ZAUX>(Xrow + (int64_t)m * kN, kRow, voff); };
  auto gload = [&](int q) { g[q] = row_load<DDSP_MAC_GAUX>(Hrow + (int64_t)min(q, Q - 1) * kN, q < Q ? kRow : 0, voff); };
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    if (s < NQ) gload(s);
    zload(s);
  }
  float2* Yp = Y + (int64_t)pair * nb * kN + f;
#pragma unroll
  for (int b = 0; b < NBK; ++b) {
    if (b + PF < NQ) gload(b + PF);
    if (b + PF < NBK) zload(b + PF);
    __builtin_amdgcn_sched_barrier(0);
    v2f acc = {0.f, 0.f}, acc2 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q <= b) {
        const float2 h = g[q];
        if (q & 1) cmac(acc2, z[b - q], (v2f){h.x, h.y}, (v2f){-h.y, h.x});
        else cmac(acc, z[b - q], (v2f){h.x, h.y}, (v2f){-h.y, h.x});
      }
    }
    Yp[(int64_t)b * kN] = make_float2(acc.x + acc2.x, acc.y + acc2.y);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The whole-row MAC forms (upols_mac_stream_kernel, upols_mac_adj_stream_kernel) for the row length they
// are built for: 50 blocks (config 2's 102400 samples), up to 25 kernel windows (a 1 s IR at 48 kHz)
constexpr int kStreamNB = 50, kStreamNQ = 25, kStreamPF = 4;

// y[row][bP + n] = IFFT(Y_b)[P + n]; grid (nb, npairs)
__global__ void __launch_bounds__(kNT) upols_inverse_kernel(const float2* __restrict__ Y, int nb,
                                                            int64_t T, int rows, int pairing, int reverse,
                                                            float* __restrict__ y, int64_t ld) {
  __shared__ float2 lds[kPad];
  const int b = blockIdx.x, pair = blockIdx.y, j = threadIdx.x;
  const float2* in = Y + ((int64_t)pair * nb + b) * kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = in[j + 256 * r];
  fft4096<true>(v, lds);
  int ra, rb;
  pair_rows(pair, rows, pairing, ra, rb);
  float* ya = y + (int64_t)ra * ld;
  float* yb = rb >= 0 ? y + (int64_t)rb * ld : nullptr;
#pragma unroll
  for (int r = 8; r < 16; ++r) {
    const int64_t s = (int64_t)b * kP + j + 256 * r - kP;
    if (s < T) {
      const int64_t so = reverse ? T - 1 - s : s;
      // non-temporal: the reverb's output is not read again by the step (16.6 vs 17.6 us at config 2,
      // the next synthesis launch unchanged, same-box A/B)
      __builtin_nontemporal_store(v[r].x, ya + so);
      if (yb) __builtin_nontemporal_store(v[r].y, yb + so);
    }
  }
}

// Backward of the partitioned convolution (Reverb.forward, modules.py:28-35), the adjoint of
// each forward step (F = unnormalised FFT, its adjoint the unnormalised inverse):
//   y_b = second half of F^-1(Y_b)           ->  dY_b = GZ_b = F([0, g_b])
//   Y_b = sum_q Z_{b-q} G_q                   ->  dZ_k = sum_q conj(G_q) GZ_{k+q}   (upols_mac_adj_kernel)
//                                                 dG_q = sum_b conj(Z_{b-q}) GZ_b  (upols_corr_kernel)
//   Z_b = F([x_b, 0])                         ->  dx_b = first half of F^-1(dZ_b) = second half of
//                                                 F^-1((-1)^f dZ_b), so the forward's inverse kernel applies
//   G_q = F([h_{q-1}, h_q]) / N               ->  dh_p = Re(first half of F^-1(dG_{p+1}) + second half of
//                                                 F^-1(dG_p)) / N = Re(second half of F^-1(dG_p + (-1)^f dG_{p+1})) / N
// For a packed pair (z = x_a + i x_b, g likewise) the real part of F^-1(conj(Z) GZ) is corr_a + corr_b:
// the packed spectra are used as they are.  GZ is shared by both gradients, and Z is the forward's.

// dG_q[f] = sum_{pair in group} sum_j conj(Z[pair][j][f]) * G[pair][j+q][f]: PC consecutive
// lags per thread with a sliding register window of conj(Z).  A workgroup is 64 bins x
// kCorrSlices waves; the waves take interleaved pairs of the group (pair = grp * S + s, stepping
// by groups * S) and are summed through LDS, so the grid has (N/64) * ceil(Q/PC) * groups
// workgroups and only `groups` partial spectra per lag reach HBM.
constexpr int kCorrSlices = 4;
template <int PC>
__global__ void __launch_bounds__(64 * kCorrSlices) upols_corr_kernel(const float2* __restrict__ Xz,
                                                                     const float2* __restrict__ Gw, int nb,
                                                                     int Q, int npairs, int groups,
                                                                     float2* __restrict__ part) {
  __shared__ float2 red[kCorrSlices][PC][64];
  const int lane = threadIdx.x & 63, s = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + lane;
  const int p0 = blockIdx.y * PC;
  const int grp = blockIdx.z;
  const float2 zero = make_float2(0.f, 0.f);
  v2f acc[PC];
#pragma unroll
  for (int d = 0; d < PC; ++d) acc[d] = (v2f){0.f, 0.f};
  for (int pair = grp * kCorrSlices + s; pair < npairs; pair += groups * kCorrSlices) {
    const float2* Xp = Xz + (int64_t)pair * nb * kN + f;
    const float2* Gp = Gw + (int64_t)pair * nb * kN + f;
    float2 win[PC];
#pragma unroll
    for (int d = 0; d < PC; ++d) win[d] = zero;
#pragma unroll 4
    for (int k = p0; k < nb; ++k) {
#pragma unroll
      for (int d = PC - 1; d > 0; --d) win[d] = win[d - 1];
      const float2 xv = Xp[(int64_t)(k - p0) * kN];
      win[0] = make_float2(xv.x, -xv.y);
      const float2 g = Gp[(int64_t)k * kN];
      const v2f gb = {g.x, g.y}, gr = {-g.y, g.x};
#pragma unroll
      for (int d = 0; d < PC; ++d) cmac(acc[d], win[d], gb, gr);
    }
  }
#pragma unroll
  for (int d = 0; d < PC; ++d) red[s][d][lane] = make_float2(acc[d].x, acc[d].y);
  __syncthreads();
  // wave s reduces partitions d = s, s + S, ... over the slices (fixed order: deterministic)
  for (int d = s; d < PC; d += kCorrSlices) {
    float2 t = red[0][d][lane];
#pragma unroll
    for (int q = 1; q < kCorrSlices; ++q) {
      t.x += red[q][d][lane].x;
      t.y += red[q][d][lane].y;
    }
    if (p0 + d < Q) part[((int64_t)grp * Q + p0 + d) * kN + f] = t;
  }
}

// The adjoint MAC on the forward MAC's register ring: the window over GZ_{j0+d+q} (d < BLK) slides
// forward, so block m sits in slot (m - j0) mod R (R = BLK + PF - 1), step u of a round reads slot
// (d + u) mod R, and after its products block j0 + q + BLK + PF - 1 is loaded into the slot step q
// freed (block j0 + q).  Blocks past the signal and windows past the kernel are descriptors with
// no records (zeros), so the unrolled rounds carry no guards.  grid (N/256, ceil(nb/BLK), npairs)
template <int BLK, int PF, int GR>
__global__ void __launch_bounds__(kNT) upols_mac_adj_ring_kernel(const float2* __restrict__ G,
                                                                 const float2* __restrict__ Hs, int nb, int Q,
                                                                 float2* __restrict__ V) {
  constexpr int R = BLK + PF - 1;
  static_assert(PF >= 1 && R % GR == 0 && GR >= PF, "ring shapes");
  constexpr int kRow = kN * (int)sizeof(float2);
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int j0 = blockIdx.y * BLK;
  const int pair = blockIdx.z;
  const float2* Grow = G + (int64_t)pair * nb * kN;
  const int voff = f * (int)sizeof(float2);
  float2 ring[R], g[GR];
  v2f acc[BLK];
  // default cache policy: the forward MAC's non-temporal bits slowed the train step here
  // (0.556 -> 0.565-0.571 ms)
  auto zload = [&](int m, float2& dst) {
    dst = row_load<0>(Grow + (int64_t)min(m, nb - 1) * kN, m < nb ? kRow : 0, voff);
  };
  auto hload = [&](int q, float2& dst) {
    dst = row_load<0>(Hs + (int64_t)min(q, Q - 1) * kN, q < Q ? kRow : 0, voff);
  };
#pragma unroll
  for (int d = 0; d < BLK; ++d) {
    acc[d] = (v2f){0.f, 0.f};
    zload(j0 + d, ring[d]);
  }
#pragma unroll
  for (int i = BLK; i < R; ++i) zload(j0 + i, ring[i]);
#pragma unroll
  for (int i = 0; i < PF; ++i) hload(i, g[i]);
  const int qmax = min(Q, nb - j0);
  for (int qb = 0; qb < qmax; qb += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int q = qb + u;
      const float2 h = g[u % GR];
      const v2f hc = {h.x, -h.y}, hcr = {h.y, h.x};  // conj(h) and its rotation
#pragma unroll
      for (int d = 0; d < BLK; ++d) cmac(acc[d], ring[(d + u) % R], hc, hcr);
      hload(q + PF, g[(u + PF) % GR]);
      zload(j0 + q + R, ring[u]);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of its use (see the forward MAC)
    }
  }
  const float sgn = (f & 1) ? -1.0f : 1.0f;
  float2* Vp = V + (int64_t)pair * nb * kN + f;
#pragma unroll
  for (int d = 0; d < BLK; ++d)
    if (j0 + d < nb) Vp[(int64_t)(j0 + d) * kN] = make_float2(sgn * acc[d].x, sgn * acc[d].y);
}

// The adjoint sums for a whole pair row in one thread (nb == NBK, Q <= NQ): every GZ_m and H_q of the
// bin is loaded once and stays in registers (the ring kernel's two chunks re-read ~1.5x of GZ), and the
// outputs stream — step s issues the loads of step s + PF (GZ_{k-PF}, H_{s+PF}), then forms V_k,
// k = NBK-1-s, from GZ_k..GZ_{k+s} and H_0..H_s already in registers and stores it, so loads, products
// and stores overlap inside every wave (166 VGPRs; grid N/256 x npairs, one round at 2 waves/SIMD).
// Config 2: 23.1-23.2 us against 29.8-29.9 for the ring kernel (same box, tools/ab_prof.sh reverb_bwd).
template <int NBK, int NQ, int PF>
__global__ void __launch_bounds__(kNT) upols_mac_adj_stream_kernel(const float2* __restrict__ G,
                                                                   const float2* __restrict__ Hs, int nb, int Q,
                                                                   float2* __restrict__ V) {
  constexpr int kRow = kN * (int)sizeof(float2);
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int pair = blockIdx.y;
  const float2* Grow = G + (int64_t)pair * nb * kN;
  const int voff = f * (int)sizeof(float2);
  float2 z[NBK], h[NQ];
  auto zload = [&](int m) { z[m] = row_load<0>(Grow + (int64_t)m * kN, kRow, voff); };
  auto hload = [&](int q) { h[q] = row_load<0>(Hs + (int64_t)min(q, Q - 1) * kN, q < Q ? kRow : 0, voff); };
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    if (s < NQ) hload(s);
    zload(NBK - 1 - s);
  }
  const float sgn = (f & 1) ? -1.0f : 1.0f;
  float2* Vp = V + (int64_t)pair * nb * kN + f;
#pragma unroll
  for (int s = 0; s < NBK; ++s) {
    const int k = NBK - 1 - s;
    if (s + PF < NQ) hload(s + PF);
    if (s + PF < NBK) zload(k - PF);
    __builtin_amdgcn_sched_barrier(0);
    v2f acc = {0.f, 0.f}, acc2 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q <= s) {
        const float2 c = h[q];
        if (q & 1) cmac(acc2, z[k + q], (v2f){c.x, -c.y}, (v2f){c.y, c.x});
        else cmac(acc, z[k + q], (v2f){c.x, -c.y}, (v2f){c.y, c.x});
      }
    }
    Vp[(int64_t)k * kN] = make_float2(sgn * (acc.x + acc2.x), sgn * (acc.y + acc2.y));
    __builtin_amdgcn_sched_barrier(0);
  }
}

// dimp[pP + n] = Re(IFFT(sum_groups part[grp][p] + (-1)^f part[grp][p+1])) [P + n] / N for n < P,
// pP + n < klen (part holds Q + 1 lags; lag Q + 1 is zero), in two kernels:
// sum[p][f] = sum_groups part[grp][p][f] + (-1)^f part[grp][p+1][f] (lag Q + 1 is zero): the group
// reduction spread over the chip (grid (N/256, Qp)) so that the per-lag transform below reads one
// spectrum (with the sum inside the 24 one-lag workgroups, each read 8 groups' spectra alone:
// 14.5 us, per-CU bandwidth)
__global__ void __launch_bounds__(kNT) upols_corr_sum_kernel(const float2* __restrict__ part, int groups, int QG,
                                                             float2* __restrict__ sum, unsigned* __restrict__ arrivals) {
  const int f = blockIdx.x * kNT + threadIdx.x, p = blockIdx.y;
  if (arrivals && f == 0 && p == 0) *arrivals = 0u;  // upols_corr_finish_impulse_kernel's counter
  const bool next = p + 1 < QG;
  const float sg = (f & 1) ? -1.0f : 1.0f;
  float2 v = make_float2(0.f, 0.f);
  for (int g = 0; g < groups; ++g) {
    const float2* in = part + ((int64_t)g * QG + p) * kN + f;
    const float2 w = in[0];
    const float2 w1 = next ? in[kN] : make_float2(0.f, 0.f);
    v.x += w.x + sg * w1.x;
    v.y += w.y + sg * w1.y;
  }
  sum[(int64_t)p * kN + f] = v;
}

// dimp[pP + n] = Re(IFFT(sum[p]))[P + n] / N for n < P, pP + n < klen; grid (Qp)
__global__ void __launch_bounds__(kNT) upols_corr_finish_kernel(const float2* __restrict__ sum, int64_t klen,
                                                                float* __restrict__ dimp) {
  __shared__ float2 lds[kPad];
  const int p = blockIdx.x, j = threadIdx.x;
  const float2* in = sum + (int64_t)p * kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = in[j + 256 * r];
  fft4096<true>(v, lds);
  const float inv_n = 1.0f / (float)kN;
#pragma unroll
  for (int r = 8; r < 16; ++r) {
    const int64_t s = (int64_t)p * kP + j + 256 * r - kP;
    if (s < klen) dimp[s] = v[r].x * inv_n;
  }
}

// upols_corr_finish_kernel fused with Reverb.build_impulse's backward (modules.py:21-26; reverb.hip
// impulse_backward_kernel, the same per-tap arithmetic, so d_noise is bit-identical): workgroup p turns its
// 2048 taps of dimp straight into d_noise and fp64 partial sums of sum dimp*noise*env and sum
// dimp*noise*env*t; the last workgroup to arrive (counter zeroed by upols_corr_sum_kernel) reduces the
// partials in index order (deterministic) into d_wet and d_decay and leaves the counter at 0.  Two launches
// fewer in the train step than dimp -> impulse_backward_kernel -> impulse_backward_finish_kernel.
__global__ void __launch_bounds__(kNT) upols_corr_finish_impulse_kernel(
    const float2* __restrict__ sum, int64_t kc, ImpulseGrad ig, double* __restrict__ partials,
    unsigned* __restrict__ arrivals, float* __restrict__ dimp) {
  __shared__ float2 lds[kPad];
  __shared__ double red[32];
  __shared__ bool last;
  const int p = blockIdx.x, j = threadIdx.x, Qp = gridDim.x;
  const float2* in = sum + (int64_t)p * kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = in[j + 256 * r];
  // the taps' envelope and noise ahead of the transform (independent of dimp; their latency hides under it)
  const float d = -ig.decay[0];
  const float sp = d > 20.0f ? d : log1pf(expf(d));
  const float neg = -sp;
  const float w = 1.0f / (1.0f + expf(-ig.wet[0]));
  float tt[8], env[8], nz[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int64_t i = (int64_t)p * kP + j + 256 * r;
    tt[r] = (float)i / ig.sr;
    env[r] = expf((neg * tt[r]) * 500.0f);
    nz[r] = i < ig.L ? ig.noise[i] : 0.0f;
  }
  fft4096<true>(v, lds);
  const float inv_n = 1.0f / (float)kN;
  double aw = 0.0, ad = 0.0;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int64_t i = (int64_t)p * kP + j + 256 * r;
    const float di = v[r + 8].x * inv_n;
    if (dimp && i < kc) dimp[i] = di;
    if (i < ig.L) {
      const float gi = (i >= 1 && i < kc) ? di : 0.0f;
      ig.d_noise[i] = gi * env[r] * w;
      const float gne = gi * nz[r] * env[r];
      aw += (double)gne;
      ad += (double)gne * (double)tt[r];
    }
  }
  // taps past the partitions (an IR longer than the signal): no gradient
  for (int64_t i = (int64_t)Qp * kP + (int64_t)p * kNT + j; i < ig.L; i += (int64_t)Qp * kNT) ig.d_noise[i] = 0.0f;
  block_sum_double2(aw, ad, red);
  if (j == 0) {
    partials[2 * p] = aw;
    partials[2 * p + 1] = ad;
    __threadfence();
    last = atomicAdd(arrivals, 1u) == (unsigned)(Qp - 1);
  }
  __syncthreads();
  if (!last || j >= 64) return;
  __threadfence();
  double sw = 0.0, sd = 0.0;
  for (int i = j; i < Qp; i += 64) {
    sw += __hip_atomic_load(partials + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sd += __hip_atomic_load(partials + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sw += __shfl_down(sw, o, 64);
    sd += __shfl_down(sd, o, 64);
  }
  if (j != 0) return;
  const float spg = d > 20.0f ? 1.0f : 1.0f / (1.0f + expf(-d));  // softplus'(d)
  ig.d_wet[0] = (float)(sw * (double)w * (1.0 - (double)w));
  ig.d_decay[0] = (float)(sd * (double)w * 500.0 * (double)spg);
  *arrivals = 0u;
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

// IR-gradient partial sums: one per group of kCorrSlices pairs, at most 8
static int64_t corr_groups(int64_t npairs) {
  return std::min<int64_t>((npairs + kCorrSlices - 1) / kCorrSlices, 8);
}

int64_t upols_partitions(int64_t klen) { return (std::max<int64_t>(klen, 1) + kP - 1) / kP; }
int64_t upols_blocks(int64_t n) { return (n + kP - 1) / kP; }

// kernel spectra per row: G_0 .. G_Q
static int64_t upols_kernel_windows(int64_t klen) { return upols_partitions(klen) + 1; }

size_t upols_spectrum_floats(int64_t krows, int64_t klen) {
  return (size_t)krows * (size_t)upols_kernel_windows(klen) * kN * 2;
}

size_t upols_workspace_bytes(int64_t rows, int64_t n, bool pairing) {
  const int64_t npairs = pairing ? (rows + 1) / 2 : rows;
  return 2 * (size_t)npairs * (size_t)upols_blocks(n) * kN * sizeof(float2);
}

int upols_spectrum(const float* h, int64_t ld, int64_t klen, int64_t krows, float* spectrum,
                   void* stream) {
  const int64_t QG = upols_kernel_windows(klen);
  if (QG > 65535 || krows > 65535) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(upols_kernel_spectrum_kernel, dim3((unsigned)QG, (unsigned)krows), dim3(kNT), 0,
                     S(stream), h, ld, klen, (int)QG, reinterpret_cast<float2*>(spectrum));
  return launch_status();
}

int upols_impulse_spectrum(const float* noise, const float* decay, const float* wet, int64_t klen, float sr,
                           float* spectrum, void* stream) {
  const int64_t QG = upols_kernel_windows(klen);
  if (QG > 65535) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(upols_impulse_spectrum_kernel, dim3((unsigned)QG), dim3(kNT), 0, S(stream), noise, decay, wet,
                     klen, sr, (int)QG, reinterpret_cast<float2*>(spectrum));
  return launch_status();
}

// Z[pair][b] = FFT of block b of the packed rows with one half zeroed (zh: 2 = [x_b, 0], 1 = [0, x_b]).
// (Measured slower: a persistent, software-pipelined variant that loads the next block under the
// current transform, 20.5 us vs 18.7 at config 2 with 2 blocks per workgroup, 26 us with 6: each
// transform is a ~4 us latency-bound chain of LDS passes, and fewer resident workgroups expose it.)
static int launch_forward(const float* x, int64_t n, int64_t rows, int pairing, int64_t nb, int64_t npairs, int off,
                          int zh, int reverse, float2* Z, void* stream) {
  hipLaunchKernelGGL(upols_forward_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream), x, n, n,
                     (int)rows, pairing, (int)nb, off, zh, reverse, Z);
  return launch_status();
}

int upols_apply_spectra(const float2* Z, int64_t rows, int64_t n, const float* spectrum, int64_t klen,
                        bool per_row_kernel, float* y, float2* Y, void* stream, bool reverse) {
  const bool pairing = !per_row_kernel;
  const int64_t npairs = pairing ? (rows + 1) / 2 : rows;
  const int64_t nb = upols_blocks(n);
  const int64_t Q = upols_kernel_windows(std::min(klen, n));
  const int64_t h_stride = per_row_kernel ? upols_kernel_windows(klen) * kN : 0;
  constexpr int RB = kRingBlk;
  if (nb > INT32_MAX || npairs > 65535 || (nb + RB - 1) / RB > 65535) return DDSP_HIP_EINVAL;
  // kRingBlk (25) output blocks per thread: each Z row is re-read (Q+BLK-1)/BLK times through L2
  // (A/B at config 2: 25 blocks 26.6 us vs 16 blocks 28.3 us, 8 and 32 no better; measured slower:
  // an LDS-tiled variant that reads Z once, 25%: lower occupancy, exposed loads; every operand
  // loaded up front from registers, 40%: 202 VGPRs, 2 waves/SIMD; one thread per (pair, bin)
  // streaming all blocks with a register ring, 8%)
  if (nb == kStreamNB && Q <= kStreamNQ)
    hipLaunchKernelGGL((upols_mac_stream_kernel<kStreamNB, kStreamNQ, kStreamPF>), dim3(kN / kNT, (unsigned)npairs),
                       dim3(kNT), 0, S(stream), Z, reinterpret_cast<const float2*>(spectrum), h_stride, (int)nb,
                       (int)Q, Y);
  else
  hipLaunchKernelGGL((upols_mac_ring_kernel<RB, kRingPF, kRingGR>),
                     dim3(kN / kNT, (unsigned)((nb + RB - 1) / RB), (unsigned)npairs), dim3(kNT), 0, S(stream), Z,
                     reinterpret_cast<const float2*>(spectrum), h_stride, (int)nb, (int)Q, Y);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(upols_inverse_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream),
                     Y, (int)nb, n, (int)rows, (int)pairing, (int)reverse, y, n);
  return launch_status();
}

int upols_apply(const float* x, int64_t rows, int64_t n, const float* spectrum, int64_t klen,
                bool per_row_kernel, float* y, void* ws, size_t ws_bytes, void* stream, bool reverse) {
  const bool pairing = !per_row_kernel;
  const int64_t npairs = pairing ? (rows + 1) / 2 : rows;
  const int64_t nb = upols_blocks(n);
  if (!ws || ws_bytes < upols_workspace_bytes(rows, n, pairing)) return DDSP_HIP_EWORKSPACE;
  if (nb > INT32_MAX || npairs > 65535) return DDSP_HIP_EINVAL;
  float2* X = reinterpret_cast<float2*>(ws);
  float2* Y = X + (size_t)npairs * nb * kN;
  // Z_b = FFT([x_b, 0])
  int st = launch_forward(x, n, rows, (int)pairing, nb, npairs, 0, 2, (int)reverse, X, stream);
  if (st) return st;
  return upols_apply_spectra(X, rows, n, spectrum, klen, per_row_kernel, y, Y, stream, reverse);
}

size_t upols_ir_cache_bytes(int64_t klen) {
  const int64_t QG = upols_kernel_windows(klen);
  return (size_t)QG * kN * sizeof(float2) + (size_t)QG * kSnapWords * sizeof(uint32_t);
}

int upols_reverb_cached(const float* x, int64_t rows, int64_t n, const float* noise, const float* decay,
                        const float* wet, int64_t klen, float sr, int force, void* cache, float* y, void* ws,
                        size_t ws_bytes, void* stream) {
  const int64_t QG = upols_kernel_windows(klen);
  const int64_t npairs = (rows + 1) / 2;
  const int64_t nb = rows > 0 ? upols_blocks(n) : 0;
  if (QG > 65535 || nb > 65535 || npairs > 65534) return DDSP_HIP_EINVAL;
  if (rows > 0 && (!ws || ws_bytes < upols_workspace_bytes(rows, n, true))) return DDSP_HIP_EWORKSPACE;
  float2* Hs = reinterpret_cast<float2*>(cache);
  uint32_t* snap = reinterpret_cast<uint32_t*>(Hs + (size_t)QG * kN);
  float2* X = reinterpret_cast<float2*>(ws);
  hipLaunchKernelGGL(upols_forward_ir_kernel, dim3((unsigned)std::max(nb, QG), (unsigned)(npairs + 1)), dim3(kNT), 0,
                     S(stream), x, n, (int)rows, (int)nb, X, noise, decay, wet, klen, sr, force, (int)QG, Hs, snap);
  int st = launch_status();
  if (st || rows == 0) return st;
  return upols_apply_spectra(X, rows, n, reinterpret_cast<const float*>(Hs), klen, false, y,
                             X + (size_t)npairs * nb * kN, stream, false);
}

size_t upols_spectra_bytes(int64_t rows, int64_t n) {
  const int64_t npairs = (rows + 1) / 2;
  return (size_t)npairs * upols_blocks(n) * kN * sizeof(float2);
}

static size_t impulse_scratch_bytes(int64_t Q) { return 256 + (((size_t)Q * 2 * sizeof(double) + 255) & ~(size_t)255); }

size_t upols_backward_workspace_bytes(int64_t rows, int64_t n, int64_t klen, bool have_x) {
  const int64_t Q = upols_kernel_windows(std::min(klen, n));
  const int64_t groups = corr_groups((rows + 1) / 2);
  // + the fused impulse gradient's partial sums and arrival counter (upols_corr_finish_impulse_kernel)
  return (have_x ? 2 : 3) * upols_spectra_bytes(rows, n) + (size_t)(groups + 1) * Q * kN * sizeof(float2) +
         impulse_scratch_bytes(Q);
}

int upols_backward(const float* x, const float* x_spectra, const float* spectrum, const float* g, int64_t rows,
                   int64_t n, int64_t klen, float* dx, float* dimp, void* ws, size_t ws_bytes, void* stream,
                   const ImpulseGrad* ig) {
  const int64_t npairs = (rows + 1) / 2;
  const int64_t nb = upols_blocks(n);
  const int64_t kc = std::min(klen, n);
  const int64_t Qp = upols_partitions(kc), Q = Qp + 1;  // output partitions of dimp; kernel windows
  const int64_t groups = corr_groups(npairs);
  const bool need_x = (dimp || ig) && !x_spectra;
  if (!ws || ws_bytes < upols_backward_workspace_bytes(rows, n, klen, !need_x)) return DDSP_HIP_EWORKSPACE;
  if (nb > INT32_MAX || npairs > 65535 || Q > 65535 || (nb + kRingBlk - 1) / kRingBlk > 65535) return DDSP_HIP_EINVAL;
  const size_t sb = upols_spectra_bytes(rows, n);
  char* w = reinterpret_cast<char*>(ws);
  float2* GZ = reinterpret_cast<float2*>(w);
  float2* V = reinterpret_cast<float2*>(w + sb);
  float2* part = reinterpret_cast<float2*>(w + 2 * sb);
  const bool want_imp = dimp || ig;
  char* scratch = w + 2 * sb + (size_t)(groups + 1) * Q * kN * sizeof(float2);
  unsigned* arrivals = reinterpret_cast<unsigned*>(scratch);
  double* partials = reinterpret_cast<double*>(scratch + 256);
  float2* Xs = need_x ? reinterpret_cast<float2*>(scratch + impulse_scratch_bytes(Q))
                      : const_cast<float2*>(reinterpret_cast<const float2*>(x_spectra));
  // GZ_b = F([0, g_b])
  int st = launch_forward(g, n, rows, 1, nb, npairs, -1, 1, 0, GZ, stream);
  if (st) return st;
  if (dx) {
    constexpr int AB = kRingBlk;
    if (nb == kStreamNB && Q <= kStreamNQ)
      hipLaunchKernelGGL((upols_mac_adj_stream_kernel<kStreamNB, kStreamNQ, kStreamPF>),
                         dim3(kN / kNT, (unsigned)npairs), dim3(kNT), 0, S(stream), GZ,
                         reinterpret_cast<const float2*>(spectrum), (int)nb, (int)Q, V);
    else
      hipLaunchKernelGGL((upols_mac_adj_ring_kernel<AB, kRingPF, kRingGR>),
                         dim3(kN / kNT, (unsigned)((nb + AB - 1) / AB), (unsigned)npairs), dim3(kNT), 0, S(stream), GZ,
                         reinterpret_cast<const float2*>(spectrum), (int)nb, (int)Q, V);
    if ((st = launch_status())) return st;
    hipLaunchKernelGGL(upols_inverse_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream), V,
                       (int)nb, n, (int)rows, 1, 0, dx, n);
    if ((st = launch_status())) return st;
  }
  if (want_imp) {
    if (need_x) {
      if (!x) return DDSP_HIP_EINVAL;
      if ((st = launch_forward(x, n, rows, 1, nb, npairs, 0, 2, 0, Xs, stream))) return st;
    }
    // Every pass over the spectra covers PC lags, so the fewest passes win: PC = 13 up to 13 kernel
    // windows, else 25 (Q = 25 at config 2: 8 lags per pass, 37.1 us -> 13, 26.8 -> 25, 24.7-25.0 us;
    // 25 lags with 2 waves per workgroup and 16 groups 26.3, 1 wave and 32 groups 28.2)
    if (Q <= 13)
      hipLaunchKernelGGL(upols_corr_kernel<13>, dim3(kN / 64, 1, (unsigned)groups), dim3(64 * kCorrSlices), 0,
                         S(stream), Xs, GZ, (int)nb, (int)Q, (int)npairs, (int)groups, part);
    else
      hipLaunchKernelGGL(upols_corr_kernel<25>, dim3(kN / 64, (unsigned)((Q + 24) / 25), (unsigned)groups),
                         dim3(64 * kCorrSlices), 0, S(stream), Xs, GZ, (int)nb, (int)Q, (int)npairs, (int)groups,
                         part);
    if ((st = launch_status())) return st;
    float2* psum = part + (size_t)groups * Q * kN;
    hipLaunchKernelGGL(upols_corr_sum_kernel, dim3(kN / kNT, (unsigned)Qp), dim3(kNT), 0, S(stream), part,
                       (int)groups, (int)Q, psum, ig ? arrivals : nullptr);
    if ((st = launch_status())) return st;
    if (ig)
      hipLaunchKernelGGL(upols_corr_finish_impulse_kernel, dim3((unsigned)Qp), dim3(kNT), 0, S(stream), psum, kc, *ig,
                         partials, arrivals, dimp);
    else
      hipLaunchKernelGGL(upols_corr_finish_kernel, dim3((unsigned)Qp), dim3(kNT), 0, S(stream), psum, kc, dimp);
    if ((st = launch_status())) return st;
  }
  return DDSP_HIP_OK;
}

}  // namespace ddsp
