// Uniformly partitioned overlap-save (UPOLS) FFT convolution for gfx950.
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
//   kernel partitions h_p = h[pP, (p+1)P) -> H_p = FFT_N([h_p, 0]) / N   (computed once);
//   forward:  X_b = FFT_N(z[(b-1)P, (b+1)P))                 (upols_forward_kernel)
//   MAC:      Y_b = sum_p X_{b-p} H_p   per frequency bin     (upols_mac_kernel)
//   inverse:  y[bP, (b+1)P) = last P points of IFFT_N(Y_b)    (upols_inverse_kernel)
//
// HBM traffic per real output sample: x read twice (overlap, 8 B), X write/read (16 B),
// Y write/read (16 B), y write (4 B).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "upols.h"
#include "twiddle4096.inc"

namespace ddsp {
namespace {

constexpr int kNT = 256;            // threads per transform
constexpr int kPad = kN + kN / 16;  // LDS float2 slots: one pad slot per 16 (bank spreading)

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

// Full 4096-point transform (three radix-16 Stockham passes, Ns = 1, 16, 256):
// v holds in[j + 256 r] on entry and out[j + 256 r] on exit.
template <bool INV>
__device__ __forceinline__ void fft4096(float2 (&v)[16], float2* lds) {
  const int j = threadIdx.x;
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

// X[pair][b][:] = FFT(z[(b+off)P, (b+off+2)P)); grid (nb, npairs).
//   off = -1: the overlap-save input windows;  off = 0 with zero_hi: FFT([z_b, 0]) (the
//   zero-padded blocks of the IR-gradient correlation);  reverse: z read time-reversed
//   (z'[s] = z[T-1-s], the transposed convolution of the input gradient).
__global__ void __launch_bounds__(kNT) upols_forward_kernel(const float* __restrict__ x, int64_t ld,
                                                            int64_t T, int rows, int pairing, int nb,
                                                            int off, int zero_hi, int reverse,
                                                            float2* __restrict__ X) {
  __shared__ float2 lds[kPad];
  const int b = blockIdx.x, pair = blockIdx.y, j = threadIdx.x;
  int ra, rb;
  pair_rows(pair, rows, pairing, ra, rb);
  const float* xa = x + (int64_t)ra * ld;
  const float* xb = rb >= 0 ? x + (int64_t)rb * ld : nullptr;
  const int64_t s0 = (int64_t)(b + off) * kP;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t s = s0 + j + 256 * r;
    const bool ok = s >= 0 && s < T && !(zero_hi && r >= 8);
    const int64_t si = reverse ? T - 1 - s : s;
    v[r] = make_float2(ok ? xa[si] : 0.0f, (ok && xb) ? xb[si] : 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = X + ((int64_t)pair * nb + b) * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
}

// H[row][p][:] = FFT([h[row][pP, pP+P) (within klen), 0]) / N; grid (Q, krows)
__global__ void __launch_bounds__(kNT) upols_kernel_spectrum_kernel(const float* __restrict__ h,
                                                                    int64_t ld, int64_t klen, int Q,
                                                                    float2* __restrict__ Hs) {
  __shared__ float2 lds[kPad];
  const int p = blockIdx.x, row = blockIdx.y, j = threadIdx.x;
  const float* hr = h + (int64_t)row * ld;
  const float inv_n = 1.0f / (float)kN;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = j + 256 * r;
    const int64_t s = (int64_t)p * kP + n;
    v[r] = make_float2((n < kP && s < klen) ? hr[s] * inv_n : 0.0f, 0.0f);
  }
  fft4096<false>(v, lds);
  float2* out = Hs + ((int64_t)row * Q + p) * kN;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[j + 256 * r] = v[r];
}

// Y[pair][b][f] = sum_p X[pair][b-p][f] * H[p][f]; each thread one bin, BLK consecutive blocks
// with a sliding window of X in registers.  grid (N/256, ceil(nb/BLK), npairs)
// (Measured: a register double-buffered prefetch of the next partitions ran 5-10% slower — the
// extra registers cost more occupancy than the hidden latency bought.)
template <int BLK>
__global__ void __launch_bounds__(kNT) upols_mac_kernel(const float2* __restrict__ X,
                                                        const float2* __restrict__ Hs,
                                                        int64_t h_pair_stride, int nb, int Q,
                                                        float2* __restrict__ Y) {
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int b0 = blockIdx.y * BLK;
  const int pair = blockIdx.z;
  const float2* Xp = X + (int64_t)pair * nb * kN + f;
  const float2* Hp = Hs + (int64_t)pair * h_pair_stride + f;
  const float2 zero = make_float2(0.f, 0.f);
  float2 acc[BLK], win[BLK];
#pragma unroll
  for (int d = 0; d < BLK; ++d) {
    acc[d] = zero;
    // clamped load + value select (a select of pointers made hipcc go through scratch)
    const float2 xv = Xp[(int64_t)min(b0 + d, nb - 1) * kN];
    win[d] = b0 + d < nb ? xv : zero;
  }
  const int pmax = min(Q, b0 + BLK);
#pragma unroll 4
  for (int p = 0; p < pmax; ++p) {
    const float2 h = Hp[(int64_t)p * kN];
#pragma unroll
    for (int d = 0; d < BLK; ++d) {
      acc[d].x = fmaf(win[d].x, h.x, fmaf(-win[d].y, h.y, acc[d].x));
      acc[d].y = fmaf(win[d].x, h.y, fmaf(win[d].y, h.x, acc[d].y));
    }
#pragma unroll
    for (int d = BLK - 1; d > 0; --d) win[d] = win[d - 1];
    const int bn = b0 - p - 1;
    const float2 xv = Xp[(int64_t)max(bn, 0) * kN];
    win[0] = bn >= 0 ? xv : zero;
  }
  float2* Yp = Y + (int64_t)pair * nb * kN + f;
#pragma unroll
  for (int d = 0; d < BLK; ++d)
    if (b0 + d < nb) Yp[(int64_t)(b0 + d) * kN] = acc[d];
}

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
      ya[so] = v[r].x;
      if (yb) yb[so] = v[r].y;
    }
  }
}

// IR-gradient correlation (backward of Reverb.forward w.r.t. the impulse, modules.py:28-35):
//   dH_p[f] = sum_{pair in group} sum_j conj(Xz[pair][j][f]) * Gw[pair][j+p][f]
// with Xz_j = FFT([x_j, 0]) and Gw_k = FFT([g_k, g_{k+1}]): the circular correlation of the two
// 2P windows is the exact linear correlation for lags pP + [0, P).  For a packed pair
// (z = x_a + i x_b, same for g) the real part of the inverse transform is corr_a + corr_b, so
// the packed spectra are used as they are.  One bin per thread, PC consecutive partitions with
// a sliding register window of conj(Xz); grid (N/256, ceil(Q/PC), groups).
template <int PC>
__global__ void __launch_bounds__(kNT) upols_corr_kernel(const float2* __restrict__ Xz,
                                                         const float2* __restrict__ Gw, int nb, int Q,
                                                         int npairs, int pairs_per_group,
                                                         float2* __restrict__ part) {
  const int f = blockIdx.x * kNT + threadIdx.x;
  const int p0 = blockIdx.y * PC;
  const int grp = blockIdx.z;
  const float2 zero = make_float2(0.f, 0.f);
  float2 acc[PC];
#pragma unroll
  for (int d = 0; d < PC; ++d) acc[d] = zero;
  const int pr0 = grp * pairs_per_group, pr1 = min(npairs, pr0 + pairs_per_group);
  for (int pair = pr0; pair < pr1; ++pair) {
    const float2* Xp = Xz + (int64_t)pair * nb * kN + f;
    const float2* Gp = Gw + (int64_t)pair * nb * kN + f;
    float2 win[PC];
#pragma unroll
    for (int d = 0; d < PC; ++d) win[d] = zero;
    for (int k = p0; k < nb; ++k) {
#pragma unroll
      for (int d = PC - 1; d > 0; --d) win[d] = win[d - 1];
      const float2 xv = Xp[(int64_t)(k - p0) * kN];
      win[0] = make_float2(xv.x, -xv.y);
      const float2 g = Gp[(int64_t)k * kN];
#pragma unroll
      for (int d = 0; d < PC; ++d) {
        acc[d].x = fmaf(win[d].x, g.x, fmaf(-win[d].y, g.y, acc[d].x));
        acc[d].y = fmaf(win[d].x, g.y, fmaf(win[d].y, g.x, acc[d].y));
      }
    }
  }
#pragma unroll
  for (int d = 0; d < PC; ++d)
    if (p0 + d < Q) part[((int64_t)grp * Q + p0 + d) * kN + f] = acc[d];
}

// dimp[pP + n] = Re(IFFT(sum_groups part[grp][p])) [n] / N for n < P, pP + n < klen; grid (Q)
__global__ void __launch_bounds__(kNT) upols_corr_finish_kernel(const float2* __restrict__ part, int groups,
                                                                int Q, int64_t klen, float* __restrict__ dimp) {
  __shared__ float2 lds[kPad];
  const int p = blockIdx.x, j = threadIdx.x;
  float2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = make_float2(0.f, 0.f);
  for (int g = 0; g < groups; ++g) {
    const float2* in = part + ((int64_t)g * Q + p) * kN;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float2 w = in[j + 256 * r];
      v[r].x += w.x;
      v[r].y += w.y;
    }
  }
  fft4096<true>(v, lds);
  const float inv_n = 1.0f / (float)kN;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int64_t s = (int64_t)p * kP + j + 256 * r;
    if (s < klen) dimp[s] = v[r].x * inv_n;
  }
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

int64_t upols_partitions(int64_t klen) { return (std::max<int64_t>(klen, 1) + kP - 1) / kP; }
int64_t upols_blocks(int64_t n) { return (n + kP - 1) / kP; }

size_t upols_spectrum_floats(int64_t krows, int64_t klen) {
  return (size_t)krows * (size_t)upols_partitions(klen) * kN * 2;
}

size_t upols_workspace_bytes(int64_t rows, int64_t n, bool pairing) {
  const int64_t npairs = pairing ? (rows + 1) / 2 : rows;
  return 2 * (size_t)npairs * (size_t)upols_blocks(n) * kN * sizeof(float2);
}

int upols_spectrum(const float* h, int64_t ld, int64_t klen, int64_t krows, float* spectrum,
                   void* stream) {
  const int64_t Q = upols_partitions(klen);
  if (Q > 65535 || krows > 65535) return DDSP_HIP_EINVAL;
  hipLaunchKernelGGL(upols_kernel_spectrum_kernel, dim3((unsigned)Q, (unsigned)krows), dim3(kNT), 0,
                     S(stream), h, ld, klen, (int)Q, reinterpret_cast<float2*>(spectrum));
  return launch_status();
}

int upols_apply(const float* x, int64_t rows, int64_t n, const float* spectrum, int64_t klen,
                bool per_row_kernel, float* y, void* ws, size_t ws_bytes, void* stream, bool reverse) {
  const bool pairing = !per_row_kernel;
  const int64_t npairs = pairing ? (rows + 1) / 2 : rows;
  const int64_t nb = upols_blocks(n);
  const int64_t Q = upols_partitions(std::min(klen, n));
  if (!ws || ws_bytes < upols_workspace_bytes(rows, n, pairing)) return DDSP_HIP_EWORKSPACE;
  if (nb > INT32_MAX || npairs > 65535 || (nb + 15) / 16 > 65535) return DDSP_HIP_EINVAL;
  float2* X = reinterpret_cast<float2*>(ws);
  float2* Y = X + (size_t)npairs * nb * kN;
  hipLaunchKernelGGL(upols_forward_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream),
                     x, n, n, (int)rows, (int)pairing, (int)nb, -1, 0, (int)reverse, X);
  int st = launch_status();
  if (st) return st;
  const int64_t h_stride = per_row_kernel ? upols_partitions(klen) * kN : 0;
  // 16 output blocks per thread: each X row is re-read (Q+15)/16 times through L2
  // (an LDS-tiled variant that reads X once measured 25% slower: lower occupancy, exposed loads)
  hipLaunchKernelGGL(upols_mac_kernel<16>, dim3(kN / kNT, (unsigned)((nb + 15) / 16), (unsigned)npairs),
                     dim3(kNT), 0, S(stream), X, reinterpret_cast<const float2*>(spectrum), h_stride,
                     (int)nb, (int)Q, Y);
  if ((st = launch_status())) return st;
  hipLaunchKernelGGL(upols_inverse_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream),
                     Y, (int)nb, n, (int)rows, (int)pairing, (int)reverse, y, n);
  return launch_status();
}

size_t upols_corr_workspace_bytes(int64_t rows, int64_t n, int64_t klen) {
  const int64_t npairs = (rows + 1) / 2;
  const int64_t nb = upols_blocks(n);
  const int64_t Q = upols_partitions(std::min(klen, n));
  const int64_t groups = std::min<int64_t>(npairs, 16);
  return (2 * (size_t)npairs * nb + (size_t)groups * Q) * kN * sizeof(float2);
}

int upols_corr(const float* x, const float* g, int64_t rows, int64_t n, int64_t klen, float* dimp, void* ws,
               size_t ws_bytes, void* stream) {
  const int64_t npairs = (rows + 1) / 2;
  const int64_t nb = upols_blocks(n);
  const int64_t kc = std::min(klen, n);
  const int64_t Q = upols_partitions(kc);
  const int64_t groups = std::min<int64_t>(npairs, 16);
  const int64_t ppg = (npairs + groups - 1) / groups;
  if (!ws || ws_bytes < upols_corr_workspace_bytes(rows, n, klen)) return DDSP_HIP_EWORKSPACE;
  if (nb > INT32_MAX || npairs > 65535 || Q > 65535) return DDSP_HIP_EINVAL;
  float2* Xz = reinterpret_cast<float2*>(ws);
  float2* Gw = Xz + (size_t)npairs * nb * kN;
  float2* part = Gw + (size_t)npairs * nb * kN;
  hipLaunchKernelGGL(upols_forward_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream),
                     x, n, n, (int)rows, 1, (int)nb, 0, 1, 0, Xz);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(upols_forward_kernel, dim3((unsigned)nb, (unsigned)npairs), dim3(kNT), 0, S(stream),
                     g, n, n, (int)rows, 1, (int)nb, 0, 0, 0, Gw);
  if ((st = launch_status())) return st;
  hipLaunchKernelGGL(upols_corr_kernel<16>, dim3(kN / kNT, (unsigned)((Q + 15) / 16), (unsigned)groups),
                     dim3(kNT), 0, S(stream), Xz, Gw, (int)nb, (int)Q, (int)npairs, (int)ppg, part);
  if ((st = launch_status())) return st;
  hipLaunchKernelGGL(upols_corr_finish_kernel, dim3((unsigned)Q), dim3(kNT), 0, S(stream), part, (int)groups,
                     (int)Q, kc, dimp);
  return launch_status();
}

}  // namespace ddsp
