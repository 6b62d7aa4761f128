// Shared device helpers for the gfx950 DDSP kernels.
//
// Numerical contract (checked against the reference's golden
// vectors by tests/): the reference computes, on CPU in fp32,
//   inc   = fl32(fl32(fl32(2*pi) * f0) / sr)             ddsp/core.py:138
//   omega = fl32(sum_{s<=t} (double)inc[s])               torch.cumsum, double accumulator
//   arg_k = fl32(omega * k)                               ddsp/core.py:139
//   out   = sum_k sin(arg_k) * A_k                         ddsp/core.py:140
// Everything here is compiled with -ffp-contract=off: every fused multiply-add is an
// explicit fmaf(), so no mul->add pair the reference rounds twice is silently fused.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ddsp_hip.h"

namespace ddsp {

constexpr float kTwoPiF = 6.28318548202514648438f;        // fl32(2*pi): ATen casts the scalar
constexpr float kInvPi = 0.318309886183790671538f;
constexpr float kPiA = 3.14159274101257324219f;           // fl32(pi)
constexpr float kPiB = -8.74227765734758577075e-08f;      // fl32(pi - kPiA)
constexpr float kMagic = 12582912.0f;                     // 1.5 * 2^23: round-to-int shifter
// |x| below this keeps |x/pi| < 2^22 (the shifter yields n exactly) and, given the 1.28e-8
// representation error of kInvPi, |x - n*pi| <= 1.9, the polynomial's fitted range.
// Larger arguments take the fp64 path.
constexpr float kFastArgLimit = 8.0e6f;

// Minimax odd polynomial sin(r) = r * (1 + r^2 * P(r^2)), P of degree 3, on |r| <= 1.9
// (max approximation error 3.7e-8; fitted by the repository, not taken from a library).
constexpr float kS3 = -0.16666624f;
constexpr float kS5 = 0.008332362f;
constexpr float kS7 = -0.00019768332f;
constexpr float kS9 = 2.5307909e-06f;

// ddsp/core.py:138 — `2 * math.pi * f0 / sample_rate` on fp32 tensors: the python scalar
// 2*pi is cast to fp32, the product is rounded, then a true (IEEE) fp32 division.
__device__ __forceinline__ float phase_inc(float f0, float sr) {
  float p = kTwoPiF * f0;
  return p / sr;  // correctly rounded (hipcc default: -fhip-fp32-correctly-rounded-divide-sqrt)
}

// Reduced argument with the sign of (-1)^n folded in: sin(x) = sin(rs) for |x| < kFastArgLimit.
// n = rint(x/pi) via the shifter (the fma forms x*kInvPi exactly before its single rounding),
// r = x - n*pi by two fmas (the first exact: Cody-Waite with an fp32 pi and fma); the parity
// of n — the shifter's lsb — is moved into r's sign bit by one integer shift-and-add
// (adding 2^31 toggles bit 31).  5 VALU ops.
__device__ __forceinline__ float reduce_signed(float x) {
  const float t = fmaf(x, kInvPi, kMagic);
  const float n = t - kMagic;
  float r = fmaf(-n, kPiA, x);
  r = fmaf(-n, kPiB, r);
  return __uint_as_float(__float_as_uint(r) + (__float_as_uint(t) << 31));
}

// acc + A*sin(rs) with the amplitude folded into the polynomial coefficients
// (a = A, ac_i = A * kS_i): rs * (a + r2*(ac3 + r2*(ac5 + r2*(ac7 + r2*ac9)))) — 6 VALU ops
// including the accumulate, so 11 per (sample, harmonic) with x = w*k and the reduction.
__device__ __forceinline__ float amp_sin_acc(float rs, float a, float ac3, float ac5, float ac7,
                                             float ac9, float acc) {
  const float r2 = rs * rs;
  float q = fmaf(ac9, r2, ac7);
  q = fmaf(q, r2, ac5);
  q = fmaf(q, r2, ac3);
  q = fmaf(q, r2, a);
  return fmaf(rs, q, acc);
}

// sin(x) for |x| < kFastArgLimit by the polynomial: abs error < 2e-7 (rms 4e-8 on uniform
// arguments).  Kept as the second, independent evaluation for kernel probes and tests.
__device__ __forceinline__ float sin_poly(float x) {
  const float rs = reduce_signed(x);
  const float r2 = rs * rs;
  float q = fmaf(kS9, r2, kS7);
  q = fmaf(q, r2, kS5);
  q = fmaf(q, r2, kS3);
  q = fmaf(q, r2, 1.0f);
  return rs * q;
}

constexpr float kInv2Pi = 0.159154936671257019043f;     // fl32(1/(2*pi))
constexpr float kInv2PiLo = 6.42063824329852652e-09f;   // fl32(1/(2*pi) - kInv2Pi)

// x/(2pi) reduced to revolutions: n = rint(x/(2pi)) by the shifter (|x/(2pi)| < 2^22 for
// |x| < kFastArgLimit), then x*kInv2Pi - n formed exactly inside one fma (a single rounding
// of a value <= 0.5) and the representation error of kInv2Pi added back by a second fma:
// |y| <= 0.55, |error| <= ~3e-8 rev.  4 VALU ops.
__device__ __forceinline__ float reduce_rev(float x) {
  const float t = fmaf(x, kInv2Pi, kMagic);
  const float n = t - kMagic;
  const float y = fmaf(x, kInv2Pi, -n);
  return fmaf(x, kInv2PiLo, y);
}

// sin(2*pi*y) on the hardware sine (v_sin_f32 takes revolutions; it costs ~3 VALU issue
// slots, measured).  With reduce_rev: |error| < 3.2e-7, rms 5.3e-8 vs the fp64 sine of the same
// fp32 argument over |x| < 7.9e6 (tools/sin_probe.hip on MI355X), against the polynomial's
// 1.8e-7 / 3.5e-8 — at 1.35-1.44x its measured throughput (~9 slots per sine instead of 12).
__device__ __forceinline__ float sin_rev(float y) { return __builtin_amdgcn_sinf(y); }

// sin(x) for |x| < kFastArgLimit.
__device__ __forceinline__ float sin_reduced(float x) { return sin_rev(reduce_rev(x)); }

constexpr float kLn10F = 2.30258512496948242188f;  // fl32(math.log(10)): ATen casts the exponent
constexpr float kOnePlusEps = 1.0f + 1e-4f;          // (True).float() + 1e-4  in fp32
constexpr float kEps = 0.0f + 1e-4f;                 // (False).float() + 1e-4 in fp32

// ddsp/core.py:77-78  scale_function: 2 * sigmoid(x) ** ln(10) + 1e-7, as
//   sigmoid(x)**ln10 = 2^(-ln10 * l),  l = log2(1 + 2^a),  a = -x log2(e)
// on the raw hardware v_exp_f32 / v_log_f32 (2^x, log2 x; 3 transcendentals, ~20 VALU ops against
// ~60 for the libm expf, IEEE division, log2f and exp2f of the first form).  l is carried as a
// double-float: l = max(a, 0) + log2(1 + 2^-|a|) with a's rounding error (an fma) kept beside it, so
// the large exponents of small sigmoids (l ~ 17 at x = -12) lose no bits, and the final 2^b takes the
// low part as 2^b_hi (1 + b_lo ln2).  Relative error ~3e-7 over x in [-25, 12] with 0.5-ulp
// transcendentals (numpy emulation against fp64), ~5x below the first form's.  x < -100 is clamped
// (the result is 1e-7 there either way; keeps -inf from making a NaN; NaN stays NaN).
__device__ __forceinline__ float scale_fn(float x) {
  constexpr float kLog2E = 1.44269502162933349609f;          // fl32(log2 e)
  constexpr float kLog2ELo = 1.92596298909109e-08f;          // log2 e - kLog2E
  constexpr float kLn2 = 0.693147180559945309f;
  const float xc = x < -100.0f ? -100.0f : x;
  const float a = xc * -kLog2E;
  const float a_lo = fmaf(-xc, kLog2E, -a) + (-xc) * kLog2ELo;   // a + a_lo = -x log2(e)
  const float m = fmaxf(a, 0.0f);
  const float t = __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(-fabsf(a)));
  const float lh = m + t;
  const float ll = (a > 0.0f ? a_lo : 0.0f) + ((m - lh) + t);
  const float bh = lh * -kLn10F;
  const float bl = fmaf(lh, -kLn10F, -bh) + ll * -kLn10F;
  const float pe = __builtin_amdgcn_exp2f(bh);
  return fmaf(2.0f, fmaf(pe, bl * kLn2, pe), 1e-7f);
}

// One harmonic-distribution entry of get_controls before normalisation (modules.py:53-60):
// scale_function, then remove_above_nyquist's mask on fl32(f0 * (k+1)) (core.py:70-74).
__device__ __forceinline__ float controls_value(float raw, float pitch0, int k, float half_sr) {
  const float d = scale_fn(raw);
  return d * ((pitch0 * (float)(k + 1)) < half_sr ? kOnePlusEps : kEps);
}

// Arguments beyond kFastArgLimit (long signals at high pitch): fp64 reduction of the
// exact fp32 value and the fp64 sine, rounded.
__device__ __noinline__ float sin_slow(float x) { return (float)sin((double)x); }

// Philox4x32-10 (Salmon et al., SC'11): counter-based RNG for the on-device noise.
struct Philox4 {
  uint32_t v[4];
};

__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  Philox4 r;
  r.v[0] = c0; r.v[1] = c1; r.v[2] = c2; r.v[3] = c3;
  return r;
}

// U[-1, 1) from 24 random bits, the form of `torch.rand(...) * 2 - 1` (modules.py:119-123).
__device__ __forceinline__ float uniform_pm1(uint32_t bits) {
  float u = (float)(bits >> 8) * 5.9604644775390625e-08f;  // [0,1) step 2^-24
  return u * 2.0f - 1.0f;
}

// Block-wide sum of a double (blockDim.x multiple of 64, <= 1024). Result valid in all threads.
__device__ __forceinline__ double block_sum_double(double v, double* scratch /*>=16*/) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// Block-wide sums of two doubles (blockDim.x multiple of 64).
__device__ __forceinline__ void block_sum_double2(double& a, double& b, double* scratch /*>=32*/) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_down(a, o, 64);
    b += __shfl_down(b, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    scratch[2 * wid] = a;
    scratch[2 * wid + 1] = b;
  }
  __syncthreads();
  a = 0.0;
  b = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
    a += scratch[2 * i];
    b += scratch[2 * i + 1];
  }
}

// Sums of two doubles over the waves [w0, w0 + nw) of the workgroup (a thread group of whole
// waves); every wave of the workgroup must call it (one barrier).  Result valid in the group.
__device__ __forceinline__ void group_sum_double2(double& a, double& b, double* scratch /*>=2*waves*/, int w0,
                                                  int nw) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_down(a, o, 64);
    b += __shfl_down(b, o, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    scratch[2 * wid] = a;
    scratch[2 * wid + 1] = b;
  }
  __syncthreads();
  a = 0.0;
  b = 0.0;
  for (int i = w0; i < w0 + nw; ++i) {
    a += scratch[2 * i];
    b += scratch[2 * i + 1];
  }
}

// The exact three-term bf16 split of fp32 operands for the bf16 matrix cores (csrc/dense.hip's MLP blocks,
// csrc/gru.hip's persistent recurrence): v = hi + mid + lo with hi = v with its low 16 bits cleared, mid the
// same of v - hi, lo = v - hi - mid — each subtraction exact, each term 8 significant bits, together all 24
// of the fp32 significand; summed as the six products hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid (each
// exact in fp32; the dropped ones are below 2^-24 of the product) a product of two splits is fp32-accurate.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 8 floats -> their exact three-term bf16 split, packed as MFMA fragments (element e = value e)
__device__ __forceinline__ void split_bf16x3(const float4& a, const float4& b, u32x4_t& hi, u32x4_t& mid,
                                             u32x4_t& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t h[8], m[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t u = __float_as_uint(v[e]);
    h[e] = u & 0xffff0000u;
    const float r1 = v[e] - __uint_as_float(h[e]);  // exact
    m[e] = __float_as_uint(r1) & 0xffff0000u;
    l[e] = __float_as_uint(r1 - __uint_as_float(m[e]));  // exact, <= 8 significant bits
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // element pairs: high halves, low element first
    hi[e] = __builtin_amdgcn_perm(h[2 * e + 1], h[2 * e], 0x07060302u);
    mid[e] = __builtin_amdgcn_perm(m[2 * e + 1], m[2 * e], 0x07060302u);
    lo[e] = __builtin_amdgcn_perm(l[2 * e + 1], l[2 * e], 0x07060302u);
  }
}

__device__ __forceinline__ bf16x8_t as_bf16x8(const u32x4_t& v) { return __builtin_bit_cast(bf16x8_t, v); }

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? DDSP_HIP_OK : DDSP_HIP_ELAUNCH;
}

}  // namespace ddsp
