// Radix-16 Stockham building blocks for LDS-resident power-of-two FFTs on gfx950, shared by
// the partitioned reverb convolution (upols.hip) and the multiscale STFT (stft.hip).
// Twiddles come from one 4096-entry table (W_4096^m, fp64-evaluated, rounded once): every
// transform size used here divides 4096.
#pragma once

#include <hip/hip_runtime.h>

#include "twiddle4096.inc"

namespace ddsp {
namespace {

__device__ __forceinline__ int lds_idx(int i) { return i + (i >> 4); }

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}

__device__ __forceinline__ float2 twiddle(int m, bool inv) {
  const float2 w = reinterpret_cast<const float2*>(kTwiddle4096)[m];
  return inv ? make_float2(w.x, -w.y) : w;
}

template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 s02 = make_float2(a0.x + a2.x, a0.y + a2.y);
  const float2 d02 = make_float2(a0.x - a2.x, a0.y - a2.y);
  const float2 s13 = make_float2(a1.x + a3.x, a1.y + a3.y);
  const float2 d13 = make_float2(a1.x - a3.x, a1.y - a3.y);
  // forward: W4 = -i ; inverse: +i.  (-i)*(x+iy) = y - ix
  const float2 rot = INV ? make_float2(-d13.y, d13.x) : make_float2(d13.y, -d13.x);
  a0 = make_float2(s02.x + s13.x, s02.y + s13.y);
  a2 = make_float2(s02.x - s13.x, s02.y - s13.y);
  a1 = make_float2(d02.x + rot.x, d02.y + rot.y);
  a3 = make_float2(d02.x - rot.x, d02.y - rot.y);
}

// 16-point DFT in registers: r = 4 r1 + r0, k = k0 + 4 k1.
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
#pragma unroll
  for (int r0 = 0; r0 < 4; ++r0) dft4<INV>(v[r0], v[4 + r0], v[8 + r0], v[12 + r0]);
  // v[4*k0 + r0] now holds u[r0][k0]; internal twiddles W16^{r0*k0} = W4096^{256*r0*k0}
#pragma unroll
  for (int r0 = 1; r0 < 4; ++r0)
#pragma unroll
    for (int k0 = 1; k0 < 4; ++k0) v[4 * k0 + r0] = cmul(v[4 * k0 + r0], twiddle(256 * r0 * k0, INV));
  float2 t[16];
#pragma unroll
  for (int k0 = 0; k0 < 4; ++k0) {
    float2 a0 = v[4 * k0 + 0], a1 = v[4 * k0 + 1], a2 = v[4 * k0 + 2], a3 = v[4 * k0 + 3];
    dft4<INV>(a0, a1, a2, a3);
    t[k0 + 0] = a0; t[k0 + 4] = a1; t[k0 + 8] = a2; t[k0 + 12] = a3;  // X[k0 + 4 k1]
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// Twiddles w^r, r = 1..15, of one Stockham pass from four table loads (w, w^2, w^4, w^8):
// every other power is a product of at most three table values (error <= ~3 ulp), so a pass
// costs 4 global loads instead of 15 and they can be issued before the LDS phases.
struct Tw4 {
  float2 t1, t2, t4, t8;
};

template <bool INV>
__device__ __forceinline__ Tw4 load_tw(int step) {
  Tw4 t;
  t.t1 = twiddle(step, INV);
  t.t2 = twiddle(2 * step, INV);
  t.t4 = twiddle(4 * step, INV);
  t.t8 = twiddle(8 * step, INV);
  return t;
}

__device__ __forceinline__ void apply_tw(float2 (&v)[16], const Tw4& t) {
  const float2 w3 = cmul(t.t1, t.t2), w5 = cmul(t.t4, t.t1), w6 = cmul(t.t4, t.t2);
  const float2 w7 = cmul(t.t4, w3);
  v[1] = cmul(v[1], t.t1);
  v[2] = cmul(v[2], t.t2);
  v[3] = cmul(v[3], w3);
  v[4] = cmul(v[4], t.t4);
  v[5] = cmul(v[5], w5);
  v[6] = cmul(v[6], w6);
  v[7] = cmul(v[7], w7);
  v[8] = cmul(v[8], t.t8);
  v[9] = cmul(v[9], cmul(t.t8, t.t1));
  v[10] = cmul(v[10], cmul(t.t8, t.t2));
  v[11] = cmul(v[11], cmul(t.t8, w3));
  v[12] = cmul(v[12], cmul(t.t8, t.t4));
  v[13] = cmul(v[13], cmul(t.t8, w5));
  v[14] = cmul(v[14], cmul(t.t8, w6));
  v[15] = cmul(v[15], cmul(t.t8, w7));
}

__device__ __forceinline__ int out_index(int j, int Ns, int r) {
  return (j / Ns) * Ns * 16 + (j & (Ns - 1)) + r * Ns;
}

// Generic Stockham FFT of N = 16^a * r points (r in {1, 2, 4, 8}, N | 4096, N >= 16), one
// transform per N/16 threads: thread t (< N/16) holds v[i] = in[t + (N/16) i] on entry and
// out[t + (N/16) i] on exit.  lds: this transform's N + N/16 float2 slots.  Every thread of the
// workgroup must call it (it synchronises the workgroup between passes).
template <bool INV>
__device__ __forceinline__ void dft2(float2& a, float2& b) {
  const float2 s = make_float2(a.x + b.x, a.y + b.y), d = make_float2(a.x - b.x, a.y - b.y);
  a = s;
  b = d;
}

template <bool INV>
__device__ __forceinline__ void dft8(float2& a0, float2& a1, float2& a2, float2& a3, float2& a4, float2& a5,
                                     float2& a6, float2& a7) {
  // radix-2 over two 4-point DFTs of the even / odd inputs
  dft4<INV>(a0, a2, a4, a6);
  dft4<INV>(a1, a3, a5, a7);
  const float h = 0.70710678118654752440f;
  // odd outputs times W8^k: k=1: (1 -+ i)/sqrt2, k=2: -+i, k=3: (-1 -+ i)/sqrt2
  const float2 o1 = INV ? make_float2((a3.x - a3.y) * h, (a3.x + a3.y) * h) : make_float2((a3.x + a3.y) * h, (a3.y - a3.x) * h);
  const float2 o2 = INV ? make_float2(-a5.y, a5.x) : make_float2(a5.y, -a5.x);
  const float2 o3 = INV ? make_float2(-(a7.x + a7.y) * h, (a7.x - a7.y) * h) : make_float2((a7.y - a7.x) * h, -(a7.x + a7.y) * h);
  const float2 e0 = a0, e1 = a2, e2 = a4, e3 = a6, o0 = a1;
  a0 = make_float2(e0.x + o0.x, e0.y + o0.y);
  a4 = make_float2(e0.x - o0.x, e0.y - o0.y);
  a1 = make_float2(e1.x + o1.x, e1.y + o1.y);
  a5 = make_float2(e1.x - o1.x, e1.y - o1.y);
  a2 = make_float2(e2.x + o2.x, e2.y + o2.y);
  a6 = make_float2(e2.x - o2.x, e2.y - o2.y);
  a3 = make_float2(e3.x + o3.x, e3.y + o3.y);
  a7 = make_float2(e3.x - o3.x, e3.y - o3.y);
}

template <int N, bool INV, bool SYNC_ENTRY = true>
__device__ __forceinline__ void fft_n(float2 (&v)[16], float2* lds, int t) {
  static_assert(N >= 16 && N <= 4096 && (N & (N - 1)) == 0, "power-of-two N in [16, 4096]");
  constexpr int Q = N / 16;  // threads per transform
  constexpr int R = (N == 16 || N == 256 || N == 4096) ? 1 : (N == 32 || N == 512) ? 2 : (N == 64 || N == 1024) ? 4 : 8;
  constexpr int A = (N == 16 || N == 32 || N == 64 || N == 128) ? 1 : (N <= 2048 ? 2 : 3);  // radix-16 passes
  // the twiddles of passes 1.. are loaded up front, so their latency hides behind pass 0
  Tw4 tw[A > 1 ? A - 1 : 1];
#pragma unroll
  for (int pass = 1; pass < A; ++pass) {
    const int ns = 1 << (4 * pass);
    tw[pass - 1] = load_tw<INV>((t % ns) * (256 / ns));
  }
  int Ns = 1;
#pragma unroll
  for (int pass = 0; pass < A; ++pass) {
    if (pass > 0) apply_tw(v, tw[pass - 1]);
    dft16<INV>(v);
    if (pass == A - 1 && R == 1) return;  // last pass with Ns = N/16: natural order in registers
    // (SYNC_ENTRY = false: the caller guarantees no thread still reads lds on entry)
    if (pass > 0 || SYNC_ENTRY) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[lds_idx(out_index(t, Ns, r))] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lds[lds_idx(t + Q * r)];
    Ns *= 16;
  }
  // final radix-R pass (Ns = N/R): butterfly b = t + Q m reads v[m + (16/R) i], twiddle W_N^{b i}
  constexpr int M = 16 / R, STEP = 4096 / N;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int b = t + Q * m;
#pragma unroll
    for (int i = 1; i < R; ++i) v[m + M * i] = cmul(v[m + M * i], twiddle((b * i * STEP) & 4095, INV));
    if (R == 2) dft2<INV>(v[m], v[m + M]);
    if (R == 4) dft4<INV>(v[m], v[m + M], v[m + 2 * M], v[m + 3 * M]);
    if (R == 8)
      dft8<INV>(v[m], v[m + M], v[m + 2 * M], v[m + 3 * M], v[m + 4 * M], v[m + 5 * M], v[m + 6 * M],
                v[m + 7 * M]);
  }
}

}  // namespace
}  // namespace ddsp
