// Uniformly partitioned overlap-save convolution (upols.hip): internal API of the library.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ddsp {
constexpr int kP = 2048;  // partition (block) length
constexpr int kN = 4096;  // FFT length

int64_t upols_partitions(int64_t klen);
int64_t upols_blocks(int64_t n);
size_t upols_spectrum_floats(int64_t krows, int64_t klen);
size_t upols_workspace_bytes(int64_t rows, int64_t n, bool pairing);
// spectra of krows kernels (row stride ld, first klen taps used), scaled by 1/N
// spectra of Reverb.build_impulse(noise, decay, wet) cropped to klen taps, built in the same launch
int upols_impulse_spectrum(const float* noise, const float* decay, const float* wet, int64_t klen, float sr,
                           float* spectrum, void* stream);
int upols_spectrum(const float* h, int64_t ld, int64_t klen, int64_t krows, float* spectrum,
                   void* stream);
// y[rows, n] = (x[rows, n] (*) h)[0:n]; spectrum from upols_spectrum (one kernel shared by all
// rows, or one per row when per_row_kernel).  klen = kernel length the spectrum was made with.
// reverse: the transposed convolution y'[t] = sum_tau x[t+tau] h[tau] (input gradient), by
// reading x and writing y time-reversed.
int upols_apply(const float* x, int64_t rows, int64_t n, const float* spectrum, int64_t klen,
                bool per_row_kernel, float* y, void* ws, size_t ws_bytes, void* stream,
                bool reverse = false);
// upols_apply after its forward transform: Z = the input block spectra FFT([x_b, 0]) of the packed
// rows ([npairs][nb][kN], e.g. written by the fused synthesis kernel), Y = workspace of the same size.
int upols_apply_spectra(const float2* Z, int64_t rows, int64_t n, const float* spectrum, int64_t klen,
                        bool per_row_kernel, float* y, float2* Y, void* stream, bool reverse = false);
// The reverb with its IR spectrum cached on the device and validated against (noise, decay, wet, sr)
// on every call, per kernel window, in the forward transform's launch (force: rebuild every window).
// cache: upols_ir_cache_bytes(klen), zero-filled when new; its first upols_spectrum_floats(1, klen)
// floats are the spectrum.  rows == 0: validate / rebuild the cache only.
size_t upols_ir_cache_bytes(int64_t klen);
int upols_reverb_cached(const float* x, int64_t rows, int64_t n, const float* noise, const float* decay,
                        const float* wet, int64_t klen, float sr, int force, void* cache, float* y, void* ws,
                        size_t ws_bytes, void* stream);
// bytes of the input spectra X that upols_apply leaves at the start of its workspace (pairing)
size_t upols_spectra_bytes(int64_t rows, int64_t n);
// Backward of upols_apply with a kernel shared by all rows (pairing): dx[rows, n] (nullable) and
// dimp[tau] = sum_rows sum_t g[row][t+tau] x[row][t] for tau < min(klen, n) (nullable).  x_spectra:
// the forward's X (nullable: recomputed from x when dimp is requested).
// ig (nullable): also Reverb.build_impulse's backward (modules.py:21-26) from dimp in the same launches —
// d_noise[L] (zero at taps >= min(klen, n)) and the device scalars d_decay, d_wet; dimp may then be null.
struct ImpulseGrad {
  const float* noise;
  const float* decay;
  const float* wet;
  int64_t L;
  float sr;
  float* d_noise;
  float* d_decay;
  float* d_wet;
};
size_t upols_backward_workspace_bytes(int64_t rows, int64_t n, int64_t klen, bool have_x);
int upols_backward(const float* x, const float* x_spectra, const float* spectrum, const float* g, int64_t rows,
                   int64_t n, int64_t klen, float* dx, float* dimp, void* ws, size_t ws_bytes, void* stream,
                   const ImpulseGrad* ig = nullptr);
}  // namespace ddsp
