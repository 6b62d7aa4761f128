// Device helpers of the filtered-noise path (FIR design and truncated convolution), shared by
// noise.hip (FilteredNoise kernels) and synth_frame.hip (the fused synthesis-frame kernel).
//   ddsp/core.py:144-166 amp_to_impulse_response, ddsp/core.py:169-176 fft_convolve
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"
#include "twiddle4096.inc"

namespace ddsp {

// cos(2*pi*q/n) table, q in [0, n): fp64-evaluated, rounded once — read from the FFT
// twiddle table (same values) when n divides 4096, else computed in fp64.
// (tid, nt): this thread's index in, and the size of, the thread group filling the table.
static __device__ __forceinline__ void fill_cos_table(float* ct, int n, int tid, int nt) {
  if (4096 % n == 0) {
    const int stride = 4096 / n;
    for (int q = tid; q < n; q += nt) ct[q] = kTwiddle4096[2 * q * stride];
  } else {
    for (int q = tid; q < n; q += nt) ct[q] = (float)cospi(2.0 * (double)q / (double)n);
  }
}
static __device__ __forceinline__ void fill_cos_table(float* ct, int n) {
  fill_cos_table(ct, n, threadIdx.x, blockDim.x);
}

// irfft of NB real magnitudes (imaginary parts zero) at tap m: n = 2(NB-1),
// (1/n)(A0 + (-1)^m A_{n/2} + 2 sum_{k=1}^{n/2-1} A_k cos(2 pi k m / n)).
// The result is even in m (ir[n-m] == ir[m]), so callers evaluate m <= n/2 only.
static __device__ __forceinline__ float irfft_tap(const float* A, const float* ct, int n, int m) {
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
static __device__ __forceinline__ void irfft_taps(const float* A, const float* ct, int n, float* ir) {
  const int half = n >> 1;
  for (int m = threadIdx.x; m <= half; m += blockDim.x) {
    const float v = irfft_tap(A, ct, n, m);
    ir[m] = v;
    if (m > 0 && m < half) ir[n - m] = v;
  }
}

// Final filter value at position j of a target-length block (core.py:158-164):
// imp1w[q] = ir[(q - n/2) mod n] * hann_n[q], padded/cropped to target, rolled by -n/2.
static __device__ __forceinline__ float ir_at(const float* ir, const float* ct, int n, int target, int j) {
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
// Taps are visited in [0, lo_end) and [hi_start, len4), both multiples of 4.  h and x are
// 16-B aligned and j0 % 4 == 0: every load is one ds_read_b128 (indexing in float4 units keeps
// that visible to the compiler; with float offsets it split them into ds_read2_b32 pairs,
// whose 16-B lane stride conflicts in the LDS banks).
static __device__ __forceinline__ float4 fir4(const float* __restrict__ h, const float* __restrict__ x,
                                      int j0, int lo_end, int hi_start, int len4) {
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
  const float4* __restrict__ h4 = reinterpret_cast<const float4*>(h);
  const int q0 = j0 >> 2;
  float y0 = 0.f, y1 = 0.f, y2 = 0.f, y3 = 0.f;
  auto run = [&](int m_begin, int m_end) {
    float4 cur = x4[q0 - (m_begin >> 2)];  // x[j0-m .. j0-m+3]
    for (int m4 = m_begin >> 2; m4 < (m_end >> 2); ++m4) {
      const float4 prv = x4[q0 - m4 - 1];  // x[j0-m-4 .. j0-m-1]
      const float4 hh = h4[m4];
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


// Final filter value at j read through the even symmetry of ir (only ir[0..n/2] needed).
static __device__ __forceinline__ float ir_at_half(const float* ir, const float* ct, int n, int target,
                                                   int j) {
  const int half = n >> 1;
  int q = j + half;
  if (q >= target) q = half < target ? q - target : q % target;
  if (q >= n) return 0.0f;
  const float hann = 0.5f - 0.5f * ct[q];
  int src = q - half;
  if (src < 0) src += n;
  if (src > half) src = n - src;
  return ir[src] * hann;
}

}  // namespace ddsp
