/*
 * ddsp_hip.h — C-ABI of the MI355X (gfx950) DDSP harmonic-plus-noise synthesis path.
 *
 * The reference (hugofloresgarcia/ddsp_pytorch) has no native ABI: its hot path is
 * six module-global Python functions in ddsp/core.py, looked up late-bound through
 * the `ddsp` package by the synth modules in ddsp/models/modules.py.  Each entry
 * point below replaces one of those functions (or one module forward) and names
 * the reference interface it stands in for (file:line under /root/reference).
 *
 * Conventions (all entry points):
 *   - plain device pointers and sizes; fp32 data, contiguous unless a stride is given;
 *     tensors are channels-last [batch, time, channel] as in the reference;
 *   - every launch is enqueued on `stream` (a hipStream_t, NULL = default stream);
 *     nothing synchronises the host;
 *   - outputs and workspaces are caller-allocated; the library never allocates
 *     device memory;
 *   - return DDSP_HIP_OK (0) or a DDSP_HIP_E* code; ddsp_hip_status_string() maps it
 *     to text.  Invalid shapes are rejected before any launch;
 *   - thread-safe and stateless: callable from any host thread, e.g. the realtime
 *     host's worker thread (ddsp_tilde.cpp:88-92).
 */
#ifndef DDSP_HIP_H
#define DDSP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  DDSP_HIP_OK = 0,
  DDSP_HIP_EINVAL = 1,      /* invalid argument / shape */
  DDSP_HIP_ELAUNCH = 2,     /* HIP launch or runtime error */
  DDSP_HIP_EFFT = 3,        /* FFT convolution error */
  DDSP_HIP_EWORKSPACE = 4,  /* workspace too small */
  DDSP_HIP_ERANGE = 5       /* input outside the exactness domain */
};

const char* ddsp_hip_status_string(int status);
int ddsp_hip_version(void);

/* ---------------- function level: ddsp/core.py ---------------- */

/* ddsp/core.py:77-78  scale_function(x) = 2*sigmoid(x)**ln(10) + 1e-7, elementwise over n values.
 * `bias` is added to x first (FilteredNoise.get_controls, modules.py:111-114 passes -5). */
int ddsp_hip_scale_function(const float* x, float* y, int64_t n, float bias, void* stream);

/* ddsp/core.py:70-74  remove_above_nyquist(amplitudes[rows,H], f0[rows,1], sr):
 * out = amps * (fl32(f0*k) < sr/2 ? 1.0001f : 1e-4f), k = 1..H. */
int ddsp_hip_remove_above_nyquist(const float* amplitudes, const float* f0, float* out,
                                  int64_t rows, int64_t n_harmonic, float sample_rate,
                                  void* stream);

/* ddsp/core.py:64-67  upsample(signal[B,F,C], factor) -> [B,F*factor,C] (nearest). */
int ddsp_hip_upsample(const float* x, float* y, int64_t batch, int64_t frames, int64_t channels,
                      int64_t factor, void* stream);

/* ddsp/core.py:136-141  harmonic_synth(f0[B,T,1], amplitudes[B,T,H], sr) -> [B,T,1].
 * Per-sample pitch and amplitudes (the op boundary).  Workspace: see *_workspace_size. */
size_t ddsp_hip_harmonic_synth_workspace_size(int64_t batch, int64_t n_samples);
int ddsp_hip_harmonic_synth(const float* f0, const float* amplitudes, float* out, int64_t batch,
                            int64_t n_samples, int64_t n_harmonic, float sample_rate,
                            void* workspace, size_t workspace_bytes, void* stream);

/* The fp32 phase omega[B,T] = cumsum(2*pi*f0/sr, time) of ddsp/core.py:138, exposed for
 * bit-exact testing of the phase accumulator (same code path as harmonic_synth). */
int ddsp_hip_phase(const float* f0, float* omega, int64_t batch, int64_t n_samples,
                   float sample_rate, void* workspace, size_t workspace_bytes, void* stream);

/* ddsp/core.py:144-166  amp_to_impulse_response(amp[rows,NB], target) -> [rows,target]. */
int ddsp_hip_amp_to_impulse_response(const float* amp, float* impulse, int64_t rows,
                                     int64_t n_bands, int64_t target_size, void* stream);

/* ddsp/core.py:169-176  fft_convolve(signal[rows,N], kernel[kernel_rows,N]) -> [rows,N]:
 * causal linear convolution truncated to N.  kernel_rows is rows or 1 (broadcast).
 * Small N runs a direct LDS convolution; large N a partitioned overlap-save FFT convolution. */
size_t ddsp_hip_fft_convolve_workspace_size(int64_t rows, int64_t kernel_rows, int64_t n);
int ddsp_hip_fft_convolve(const float* signal, const float* kernel, float* out, int64_t rows,
                          int64_t kernel_rows, int64_t n, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ---------------- module level: ddsp/models/modules.py ---------------- */

/* modules.py:44-67  HarmonicSynth.get_controls: amplitudes = scale(amp_raw),
 * dist = remove_above_nyquist(scale(dist_raw), f0, sr) / sum.  Inputs may be strided views
 * (param[..., :1] and param[..., 1:]): row r of amp_raw is amp_raw[r*amp_stride],
 * of dist_raw is dist_raw[r*dist_stride + k]. */
int ddsp_hip_harmonic_controls(const float* amp_raw, int64_t amp_stride, const float* dist_raw,
                               int64_t dist_stride, const float* f0, float* amplitudes,
                               float* distribution, int64_t rows, int64_t n_harmonic,
                               float sample_rate, void* stream);

/* modules.py:69-80  HarmonicSynth.forward fused: dist*amps (written back to `distribution`
 * in place when write_back != 0, reproducing modules.py:73), frame->sample upsampling of
 * pitch and amplitudes in registers, and harmonic_synth; [B,F,H] never leaves LDS. */
int ddsp_hip_harmonic_synth_frames(const float* f0, const float* amplitudes, float* distribution,
                                   int write_back, float* out, int64_t batch, int64_t frames,
                                   int64_t n_harmonic, int64_t block_size, float sample_rate,
                                   void* stream);

/* decoder.py:106-113 + modules.py:44-80: HarmonicSynth.get_controls and forward in one launch,
 * straight from the harmonic projection param[B,F,H+1] (amplitude column 0, distribution
 * columns 1..H, decoder.py:107-108).  The controls never reach HBM. */
int ddsp_hip_harmonic_synth_params(const float* f0, const float* param, float* out, int64_t batch,
                                   int64_t frames, int64_t n_harmonic, int64_t block_size,
                                   float sample_rate, void* stream);

/* modules.py:116-128  FilteredNoise.forward fused: per-frame zero-phase FIR from the
 * magnitudes (amp_to_impulse_response) applied to block_size noise samples by truncated
 * linear convolution (fft_convolve).  noise == NULL draws U[-1,1) on device
 * (Philox4x32-10 keyed by seed, counter offset), else noise[B,F,block_size] is used
 * (parity mode: the reference's torch.rand stream).  `add` (nullable, [B,F*bs]) is added
 * to the result (fuses decoder.py:121 `harmonic + noise`); `noise_out` (nullable)
 * receives the filtered noise alone. */
int ddsp_hip_filtered_noise(const float* magnitudes, const float* noise, uint64_t seed,
                            uint64_t offset, const float* add, float* out, float* noise_out,
                            int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                            void* stream);

/* modules.py:111-128  FilteredNoise.get_controls + forward in one launch: raw_magnitudes is the
 * noise projection [B,F,NB] (decoder.py:115); the kernel applies scale_function(x + bias)
 * (bias = initial_bias, -5 by default) before designing the filters.  Other arguments as
 * ddsp_hip_filtered_noise. */
int ddsp_hip_filtered_noise_params(const float* raw_magnitudes, float bias, const float* noise,
                                   uint64_t seed, uint64_t offset, const float* add, float* out,
                                   float* noise_out, int64_t batch, int64_t frames, int64_t n_bands,
                                   int64_t block_size, void* stream);

/* decoder.py:106-121 in one launch: HarmonicSynth.get_controls + forward from the harmonic
 * projection param[B,F,H+1], FilteredNoise.get_controls + forward from the raw noise projection
 * raw_magnitudes[B,F,NB] (scale_function(x + bias)), and signal = harmonic + noise -> out[B,F*bs].
 * noise / seed / offset as ddsp_hip_filtered_noise; harmonic_out and noise_out (nullable)
 * receive the two parts.  Shape envelope: block_size % 4 == 0 and <= 1024, H <= 1024,
 * NB <= 1025; outside it DDSP_HIP_ERANGE is returned and callers use the separate kernels. */
int ddsp_hip_synth_frames(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                          const float* noise, uint64_t seed, uint64_t offset, float* out,
                          float* harmonic_out, float* noise_out, int64_t batch, int64_t frames,
                          int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                          void* stream);

/* ddsp_hip_synth_frames that also writes the controls DDSPDecoder.forward returns
 * (decoder.py:127-135: output['harmonic_ctrls'], output['noise_ctrls']) into controls_out (nullable),
 * laid out as [amplitudes B*F | harmonic_distribution B*F*H | magnitudes B*F*NB]: amplitudes =
 * scale_function(param[...,0]), harmonic_distribution = the normalised distribution after
 * HarmonicSynth.forward's in-place `*= amplitudes` (modules.py:61,73), magnitudes =
 * scale_function(raw_magnitudes + bias) (modules.py:111-114).  param_ld / magnitudes_ld: elements between
 * consecutive frames' rows (>= H + 1 / >= NB), so both may be column slices of one projection output
 * (decoder.py:106-117 computed as a single GEMM). */
int ddsp_hip_synth_frames_controls(const float* f0, const float* param, int64_t param_ld, const float* raw_magnitudes,
                                   int64_t magnitudes_ld, float bias, const float* noise, uint64_t seed,
                                   uint64_t offset, float* out, float* harmonic_out, float* noise_out,
                                   float* controls_out, int64_t batch, int64_t frames, int64_t n_harmonic,
                                   int64_t n_bands, int64_t block_size, float sample_rate, void* stream);
/* The same with frame_prefix (nullable): the exact fp64 phase prefix of every frame,
 * frame_prefix[b * frames + f] = sum_{g < f} block_size * fl32(fl32(fl32(2 pi) f0[b, g]) / sr) (the
 * reference's cumsum, core.py:138, at each frame's start), as ddsp_hip_frame_phase_prefix writes it.
 * Without it every frame's workgroup sums its earlier frames itself: O(frames) per frame, O(frames^2)
 * per item — the right choice for a few hundred frames, not for a minute of audio (5,625 frames at
 * block 512).  Both routes give the same bits wherever every partial sum is exact in fp64, i.e. while the
 * increments' significant bits together with log2(frames * block_size) span <= 53 bits (f0 of audio pitch,
 * tests/test_gpu_long_render.py); near-zero f0 (unvoiced frames, increments with ulps far below the running
 * sum's) rounds the sums and the two summation orders may differ in the phase's last bits — inside the
 * sine's 1e-6 tolerance, and checked at that tolerance. */
int ddsp_hip_synth_frames_controls_prefix(const float* f0, const float* param, int64_t param_ld,
                                          const float* raw_magnitudes, int64_t magnitudes_ld, float bias,
                                          const float* noise, uint64_t seed, uint64_t offset, float* out,
                                          float* harmonic_out, float* noise_out, float* controls_out,
                                          const double* frame_prefix, int64_t batch, int64_t frames,
                                          int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                          void* stream);
int ddsp_hip_frame_phase_prefix(const float* f0, int64_t batch, int64_t frames, int64_t block_size, float sample_rate,
                                double* frame_prefix, void* stream);

/* ddsp_hip_synth_frames for a stream of calls replayed from a captured HIP graph (the ddsp~
 * realtime host, realtime/ddsp_tilde/ddsp_model.cpp:32-52, calling the exported model once per
 * 1024-sample buffer): the Philox offset of the on-device noise is read from the device word
 * *counter, which a second launch on the same stream then increments, so every replay draws
 * fresh noise (a graph freezes by-value arguments).  Call k draws the noise of
 * ddsp_hip_synth_frames(..., seed, offset = k, ...). */
int ddsp_hip_synth_frames_counter(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                                  uint64_t seed, uint64_t* counter, float* out, int64_t batch, int64_t frames,
                                  int64_t n_harmonic, int64_t n_bands, int64_t block_size, float sample_rate,
                                  void* stream);

/* modules.py:21-26  Reverb.build_impulse: noise[L]*exp(-softplus(-decay)*t*500)*sigmoid(wet),
 * impulse[0] = 1.  decay and wet are device scalars. */
int ddsp_hip_reverb_build_impulse(const float* noise, const float* decay, const float* wet,
                                  float* impulse, int64_t length, float sample_rate,
                                  void* stream);

/* modules.py:28-35  Reverb.forward: IR padded/cropped to n_samples, then fft_convolve.
 * Split in two so the IR spectrum is computed once and cached by the caller:
 *   ddsp_hip_reverb_spectrum: impulse[L] -> spectrum (ddsp_hip_reverb_spectrum_floats floats:
 *     partitioned-convolution spectra of the IR cropped to min(L, n_samples));
 *   ddsp_hip_reverb_apply:   x[B,T] (*) IR -> out[B,T] using that spectrum. */
size_t ddsp_hip_reverb_spectrum_floats(int64_t n_samples, int64_t ir_length);
size_t ddsp_hip_reverb_workspace_size(int64_t batch, int64_t n_samples, int64_t ir_length);
/* modules.py:21-35: Reverb.build_impulse and the IR's partition spectra (as ddsp_hip_reverb_spectrum of
 * the built impulse, bit for bit) in ONE launch — the impulse is never written.  For a reverb whose
 * parameters change every call (training: the reference rebuilds the IR in every Reverb.forward). */
int ddsp_hip_reverb_impulse_spectrum(const float* noise, const float* decay, const float* wet, int64_t ir_length,
                                     float sample_rate, int64_t n_samples, float* spectrum, void* stream);
int ddsp_hip_reverb_spectrum(const float* impulse, int64_t ir_length, int64_t n_samples,
                             float* spectrum, void* stream);
int ddsp_hip_reverb_apply(const float* x, const float* spectrum, float* out, int64_t batch,
                          int64_t n_samples, int64_t ir_length, void* workspace,
                          size_t workspace_bytes, void* stream);
/* modules.py:21-35 Reverb.forward (build_impulse, crop/pad to n_samples, fft_convolve) with the IR's partition
 * spectra cached on the device and VALIDATED there on every call: `cache` (caller-owned device memory of
 * ddsp_hip_reverb_cache_bytes bytes, zero-filled once: a zeroed cache holds nothing) keeps, per IR window,
 * the spectrum and a bit-exact copy of the inputs it was built from (the window's noise taps, decay, wet,
 * sample_rate).  The input transform's launch compares them with the current parameters and rebuilds the
 * windows that differ, so any write to the parameters (optimizer steps, writes through aliases such as
 * `.data`) is seen by the next call, and unchanged parameters cost no rebuild.  force != 0 rebuilds every
 * window (the reference's every-call rebuild).  batch == 0 validates the cache only.  The cache's first
 * ddsp_hip_reverb_spectrum_floats(n_samples, ir_length) floats are then the current spectrum (as
 * ddsp_hip_reverb_impulse_spectrum writes it, bit for bit; used by ddsp_hip_reverb_backward).  Workspace:
 * ddsp_hip_reverb_workspace_size; it then holds x's input spectra as after ddsp_hip_reverb_apply. */
size_t ddsp_hip_reverb_cache_bytes(int64_t n_samples, int64_t ir_length);
int ddsp_hip_reverb_forward(const float* x, const float* noise, const float* decay, const float* wet,
                            int64_t ir_length, float sample_rate, int force, void* cache, size_t cache_bytes,
                            float* out, int64_t batch, int64_t n_samples, void* workspace, size_t workspace_bytes,
                            void* stream);

/* ---------------- the decoder network for a few frames: core.py:122-129, decoder.py:43-68 ----------------
 * One Linear for rows <= 8 frames (the realtime stream's 1024-sample calls, ddsp_model.cpp:32-52)
 * with the previous MLP block's LayerNorm + LeakyReLU folded into its input:
 *   a[r, :] = concat over inputs s of act_s(x_s[r, :])
 *   y[r, n] = sum_k weight[n, k] a[r, k] + bias[n]          weight [out_features, K] (nn.Linear)
 * act_s: x' = x * scale + shift (the exported model's loudness normalisation, export.py:35;
 * 1 and 0 otherwise); with w1/b1 (a K=1 nn.Linear of width `width`, the first layer of
 * core.py:122's mlp(1, ...)) x is one value per row and x'' = w1[c] * x' + b1[c]; with
 * gamma/beta: leaky_relu(layer_norm(x'') * gamma + beta, 0.01), eps 1e-5 (core.py:126).
 * x_copy (nullable, w1 inputs only) receives x' per row.  Up to DDSP_HIP_DENSE_MAX_PROBLEMS
 * independent Linears share one launch.  rows <= 8, K <= 1088 (else DDSP_HIP_ERANGE). */
#define DDSP_HIP_DENSE_MAX_INPUTS 3
#define DDSP_HIP_DENSE_MAX_PROBLEMS 2
typedef struct ddsp_hip_dense_input {
  const float* x;      /* [rows, ld] (w1 inputs: x[r * ld] is the row's value) */
  int64_t ld;
  int64_t width;       /* columns contributed to K */
  float scale, shift;
  const float* w1;     /* nullable [width] */
  const float* b1;     /* [width] when w1 */
  const float* gamma;  /* nullable [width]: LayerNorm + LeakyReLU */
  const float* beta;
  float* x_copy;       /* nullable [rows] */
} ddsp_hip_dense_input;
typedef struct ddsp_hip_dense_problem {
  ddsp_hip_dense_input inputs[DDSP_HIP_DENSE_MAX_INPUTS];
  int n_inputs;
  const float* weight; /* [out_features, K] */
  const float* bias;   /* nullable [out_features] */
  float* y;            /* [rows, ldy] */
  int64_t ldy;
  int64_t out_features;
} ddsp_hip_dense_problem;
int ddsp_hip_dense_rows(const ddsp_hip_dense_problem* problems, int n_problems, int64_t rows, void* stream);

/* ddsp/core.py:122-129: one whole MLP block, y = LeakyReLU(LayerNorm(x W^T + b)), W [out, w_ld] the
 * nn.Linear weight, for out_features = 512 (else DDSP_HIP_ERANGE): the Linear on the matrix cores,
 * LayerNorm + LeakyReLU in its epilogue.  e0/e1 (nullable, per-row scalars at stride e_ld) add
 * e0[r] W[:, in] + e1[r] W[:, in + 1] — the decoder's out_mlp input [gru_out, f0, loudness]
 * (decoder.py:68) without the concatenation.  y [rows, y_ld] may be a column slice.
 * The Linear's arithmetic: at in_features 512 with 16-byte aligned rows (the decoder's blocks) both operands
 * split exactly into three bf16 terms and summed as six bf16 products per term pair on the bf16 matrix
 * cores — fp32-accurate (the dropped terms are ~2^-24 of each product), not the same bits as an fp32 fma
 * chain; flags = DDSP_HIP_MLP_EXACT_F32 (or any other shape) takes the f32-input MFMA, whose sums are
 * exactly k-ordered fp32 fma chains. */
enum { DDSP_HIP_MLP_EXACT_F32 = 1 };
int ddsp_hip_mlp_block(const float* x, int64_t x_ld, int64_t in_features, const float* w, int64_t w_ld,
                       const float* bias, const float* e0, const float* e1, int64_t e_ld, const float* gamma,
                       const float* beta, float eps, float slope, float* y, int64_t y_ld, int64_t rows,
                       int64_t out_features, int flags, void* stream);
/* ddsp/core.py:122-129 (one MLP block after its Linear, decoder.py:25-42): y = LeakyReLU(LayerNorm(h))
 * per row of cols features, h = x [rows, x_ld] or, with w1/b1 (a Linear with ONE input feature),
 * h = x[r] * w1 + b1 formed on the fly.  gamma/beta: the LayerNorm's affine; eps and the negative
 * slope as in torch (1e-5, 0.01).  y [rows, y_ld] may be a column slice of a wider buffer.  One pass
 * instead of torch's two; cols 512 or 1024 with 16-byte aligned rows, else DDSP_HIP_ERANGE. */
int ddsp_hip_layer_norm_leaky_relu(const float* x, int64_t x_ld, const float* w1, const float* b1, const float* gamma,
                                   const float* beta, float eps, float slope, float* y, int64_t y_ld, int64_t rows,
                                   int64_t cols, void* stream);

/* Weight gradient of a Linear under autograd, grad_w[m][n] = sum_r grad_y[r][m] x[r][n] (grad_w [out_features,
 * dw_ld], nn.Linear's weight layout; torch: grad_y^T @ x), on the bf16 matrix cores with the fp32-accurate
 * three-term split: the decoder MLPs' Linears and projections (core.py:122-129, decoder.py:106-117) and the GRU's
 * W_ih / W_hh (decoder.py:33-68).  Any widths (tiles past an edge are padding of the partials); split over row
 * ranges whose partials are summed in a fixed order (deterministic).  ws:
 * ddsp_hip_linear_weight_grad_workspace_size(rows, out_features, in_features) bytes.  DDSP_HIP_ERANGE when a row
 * range's byte offsets pass 2^31 (dy_ld / x_ld beyond ~2^24 floats) or a width passes 2^24: callers keep their
 * library GEMM. */
size_t ddsp_hip_linear_weight_grad_workspace_size(int64_t rows, int64_t out_features, int64_t in_features);
int ddsp_hip_linear_weight_grad(const float* grad_y, int64_t dy_ld, const float* x, int64_t x_ld, float* grad_w,
                                int64_t dw_ld, int64_t rows, int64_t out_features, int64_t in_features, void* ws,
                                size_t ws_bytes, void* stream);

/* Backward of ddsp_hip_layer_norm_leaky_relu without w1 (training: the MLP blocks' LayerNorm + LeakyReLU,
 * core.py:122-129, replacing torch's leaky_relu_backward + native_layer_norm_backward): from the pre-activation x
 * [rows, x_ld] and grad_y, grad_x [rows, dx_ld] and (each nullable) grad_gamma / grad_beta [cols], the column sums
 * over all rows (deterministic order).  The LeakyReLU's branch is taken on z = LayerNorm(x) formed as the forward
 * forms it.  ws: ddsp_hip_layer_norm_leaky_relu_backward_workspace_size(cols) bytes when a parameter gradient is
 * requested.  cols 512 or 1024 with 16-byte aligned rows, else DDSP_HIP_ERANGE. */
size_t ddsp_hip_layer_norm_leaky_relu_backward_workspace_size(int64_t cols);
int ddsp_hip_layer_norm_leaky_relu_backward(const float* x, int64_t x_ld, const float* gamma, const float* beta, float eps,
                                            float slope, const float* grad_y, int64_t dy_ld, float* grad_x, int64_t dx_ld,
                                            float* grad_gamma, float* grad_beta, int64_t rows, int64_t cols, void* ws,
                                            size_t ws_bytes, void* stream);

/* A Linear y = x W^T + b (W [out_features, w_ld], the nn.Linear / nn.GRU weight layout) on the bf16 matrix cores
 * with the fp32-accurate three-term split of ddsp_hip_mlp_block: the decoder's GRU input projection for every
 * step at once (decoder.py:41, torch.nn.GRU's x W_ih^T + b_ih; 12,800 x 1024 -> 1536 at config 2).
 * Under autograd also the input gradient of the MLP blocks' Linears (dx = dy W, W^T as the weight) and of the
 * GRU's input projection (in_features 1536 = 3 gates x 512).  in_features 512, 1024 or 1536, out_features a
 * multiple of 512, x and W 16-byte aligned with ld % 4 == 0; else DDSP_HIP_ERANGE (callers keep their library
 * GEMM). */
int ddsp_hip_linear(const float* x, int64_t x_ld, int64_t in_features, const float* w, int64_t w_ld,
                    const float* bias, float* y, int64_t y_ld, int64_t rows, int64_t out_features, void* stream);

/* decoder.py:106-117 (param = harmonic_proj(hidden), magnitudes = noise_proj(hidden)) in ONE launch on the bf16
 * matrix cores with the fp32-accurate three-term split of ddsp_hip_linear, reading both layers' parameters where
 * they lie (nn.Linear layout, W1 [n1, w1_ld], W2 [n2, w2_ld]): y[r][c] = x[r] W1[c]^T + b1[c] for c < n1 and
 * x[r] W2[c - n1]^T + b2[c - n1] for n1 <= c < n1 + n2; columns of y past n1 + n2 are not written.  Replaces
 * the two nn.Linear calls of decoder.py:106-117 (stack_rows + one library GEMM before).  in_features 512, x, W1,
 * W2 16-byte aligned with ld % 4 == 0; else DDSP_HIP_ERANGE (callers keep their library GEMM). */
int ddsp_hip_projections(const float* x, int64_t x_ld, int64_t in_features, const float* w1, int64_t w1_ld,
                         const float* b1, int64_t n1, const float* w2, int64_t w2_ld, const float* b2, int64_t n2,
                         float* y, int64_t y_ld, int64_t rows, void* stream);

/* decoder.py:106-117 (param = harmonic_proj(hidden), magnitudes = noise_proj(hidden)): the two projections'
 * parameters stacked into one zero-padded matrix w [n_pad, in_features] and
 * bias b [n_pad] (caller buffers; rows n1 + n2 .. n_pad - 1 zero), for one library GEMM over both at a
 * width it is fast at.  One launch; the parameters are read as they are at the call. */
int ddsp_hip_stack_rows(const float* w1, int64_t w1_ld, const float* b1, int64_t n1, const float* w2, int64_t w2_ld,
                        const float* b2, int64_t n2, int64_t in_features, float* w, float* b, int64_t n_pad,
                        void* stream);

/* ---------------- the decoder network's recurrence: decoder.py:33-68 (torch.nn.GRU) ----------------
 * out[B,T,H] = GRU(h0) over xp[B,T,3H] = x W_ih^T + b_ih (the input projection for every step,
 * computed by the caller's GEMM), W_hh[3H,H], b_hh[3H] in torch's (r, z, n) order; h0 [B,H]
 * (NULL = zeros); h_last [B,H] (nullable) receives h_T; gates (nullable, training) [4][B,T,H]
 * receives r, z, n and W_hn h + b_hn of every step for the backward.  One launch per time
 * step; hidden % 64 == 0 (else DDSP_HIP_ERANGE).
 * Backward (BPTT): from grad_out[B,T,H] (nullable) and grad_h_last[B,H] (nullable) ->
 * grad_xp[B,T,3H] (gradient of the input projection: dW_ih, db_ih, dx are GEMMs of it),
 * grad_gn[B,T,H] (with grad_xp's r and z planes, the gradient of W_hh h + b_hh: dW_hh and db_hh
 * are GEMMs of it against h_{t-1}), grad_h0[B,H] (nullable).  Workspace: *_workspace_size. */
int ddsp_hip_gru_forward(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                         float* h_last, float* gates, int64_t batch, int64_t steps, int64_t hidden, void* stream);
/* The same forward as ONE persistent launch (hidden 512, batch <= 64, out < 2 GiB, >= 256 CUs, a stream
 * whose kernels may use every CU, h_last != h0; else DDSP_HIP_ERANGE and the caller uses
 * ddsp_hip_gru_forward, which allows h_T over h0 in place): 8 groups
 * of 32 workgroups, group g owning items g, g + 8, ...; each workgroup keeps its 48 rows of W_hh in
 * registers for the whole sequence and the group's slots hand h_t to each other through the output
 * sequence (a per-group counter).  It needs all 256 workgroups resident together; when they are not (another
 * long-running kernel beside it, GPU sharing) every wait ends within 200 ms, the launch aborts, and a rescue
 * kernel that the call always enqueues behind it recomputes out, h_last and gates exactly as
 * ddsp_hip_gru_forward does (bit for bit) — the outputs are right either way, and the abort is reported in
 * the workspace's status word (below).  Workspace: ddsp_hip_gru_persistent_workspace_size() bytes (zeroed by
 * the call, on the stream, by a kernel of its own: the call stays capturable into a HIP graph); after the
 * stream has passed the call, the uint32 at byte offset ddsp_hip_gru_persistent_status_offset() holds
 * DDSP_HIP_GRU_STATUS_LOCAL (the hand-off stayed inside each XCD's L2), 0 (the placement-independent
 * write-through hand-off) or DDSP_HIP_GRU_STATUS_RESCUED (aborted, the outputs come from the rescue kernel).
 * flags: 0, or test hooks — DDSP_HIP_GRU_SPREAD (use the placement-independent hand-off whatever the
 * census finds), DDSP_HIP_GRU_NO_MASK_CHECK (launch on a CU-masked stream anyway: the abort path under a
 * real residency failure), DDSP_HIP_GRU_FORCE_ABORT (abort at the census). */
enum {
  DDSP_HIP_GRU_SPREAD = 1,
  DDSP_HIP_GRU_NO_MASK_CHECK = 2,
  DDSP_HIP_GRU_FORCE_ABORT = 4,
  DDSP_HIP_GRU_STATUS_LOCAL = 1,
  DDSP_HIP_GRU_STATUS_RESCUED = 2
};
size_t ddsp_hip_gru_persistent_workspace_size(void);
size_t ddsp_hip_gru_persistent_status_offset(void);
int ddsp_hip_gru_forward_persistent(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                                    float* h_last, float* gates, int64_t batch, int64_t steps, int64_t hidden,
                                    int flags, void* workspace, size_t workspace_bytes, void* stream);
/* The BPTT as ONE persistent launch (the training mirror of ddsp_hip_gru_forward_persistent: same envelope —
 * hidden 512, batch <= 64, grad_xp < 2 GiB, >= 256 CUs, a stream that may use every CU; else DDSP_HIP_ERANGE and
 * the caller uses ddsp_hip_gru_backward —, same groups, census, hand-off, flags, abort, rescue and status word):
 * each workgroup keeps its 16 units' W_hh columns in registers and the slots hand each step's gate gradients
 * (the grad_xp / grad_gn rows themselves) to each other; W_hh^T dG on the bf16 matrix cores with the
 * fp32-accurate three-term split.  Outputs as ddsp_hip_gru_backward (fp32-accurate, not the same bits).
 * Workspace: ddsp_hip_gru_persistent_workspace_size() bytes. */
int ddsp_hip_gru_backward_persistent(const float* w_hh, const float* gates, const float* out, const float* h0,
                                     const float* grad_out, const float* grad_h_last, float* grad_xp, float* grad_gn,
                                     float* grad_h0, int64_t batch, int64_t steps, int64_t hidden, int flags,
                                     void* workspace, size_t workspace_bytes, void* stream);
size_t ddsp_hip_gru_backward_workspace_size(int64_t batch, int64_t hidden);
int ddsp_hip_gru_backward(const float* w_hh, const float* gates, const float* out, const float* h0,
                          const float* grad_out, const float* grad_h_last, float* grad_xp, float* grad_gn,
                          float* grad_h0, int64_t batch, int64_t steps, int64_t hidden, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ---------------- training loss: ddsp/core.py:27-41 multiscale_fft ----------------
 * One scale of multiscale_fft: |torch.stft(x, n_fft, hop, n_fft, hann(n_fft), center=True
 * (reflect), normalized=True)| for x[batch, n_samples] (n_fft a power of two in [16, 4096],
 * n_samples > n_fft/2).  magnitudes are written frame-major [batch, frames, n_fft/2+1]
 * (frames = ddsp_hip_stft_frames(n_samples, hop) = n_samples/hop + 1); the reference's
 * [batch, n_fft/2+1, frames] is its transpose.  The backward maps grad_magnitudes (same layout)
 * to grad_x[batch, n_samples] (|Z| has zero gradient where Z = 0, as torch's abs). */
int64_t ddsp_hip_stft_frames(int64_t n_samples, int64_t hop);
int ddsp_hip_stft_magnitude(const float* x, float* magnitudes, int64_t batch, int64_t n_samples, int64_t n_fft,
                            int64_t hop, void* stream);
size_t ddsp_hip_stft_backward_workspace_size(int64_t batch, int64_t n_samples, int64_t n_fft, int64_t hop);
int ddsp_hip_stft_magnitude_backward(const float* x, const float* grad_magnitudes, float* grad_x, int64_t batch,
                                     int64_t n_samples, int64_t n_fft, int64_t hop, void* workspace,
                                     size_t workspace_bytes, void* stream);

/* train.py:70-76 + 91-104: the multiscale spectral loss of a reconstruction against a target
 * (both [batch, n_samples]), sum over scales of mean|Mx - My| + mean|log(Mx+1e-7) - log(My+1e-7)|,
 * fused per scale (no spectrogram reaches memory) -> loss (device scalar) and, when grad_recon is
 * not NULL, dloss/drecon [batch, n_samples].  n_ffts/hops: host arrays of n_scales entries
 * (hop = int(n_fft * (1 - overlap))).  Deterministic (fixed-order fp64 reductions). */
size_t ddsp_hip_spectral_loss_workspace_size(int64_t batch, int64_t n_samples, const int64_t* n_ffts,
                                             const int64_t* hops, int n_scales);
int ddsp_hip_spectral_loss(const float* target, const float* recon, int64_t batch, int64_t n_samples,
                           const int64_t* n_ffts, const int64_t* hops, int n_scales, float* loss, float* grad_recon,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ---------------- backward (training): train.py:84-130 back-propagates through the path ----------------
 * Vector-Jacobian products of the entry points above.  `grad*` inputs are the upstream
 * gradients (same shapes as the forward outputs), `grad_*` outputs are caller-allocated and
 * overwritten.  Pitch (f0) is an input feature in the reference's training loop and gets no
 * gradient. */

/* core.py:77-78 scale_function backward: dx = grad * scale'(x + bias). */
int ddsp_hip_scale_function_backward(const float* x, const float* grad, float* dx, int64_t n, float bias,
                                     void* stream);

/* core.py:64-67 upsample backward: dx[B,F,C] = sum over each block of grad[B,F*factor,C]. */
int ddsp_hip_upsample_backward(const float* grad, float* dx, int64_t batch, int64_t frames, int64_t channels,
                               int64_t factor, void* stream);

/* core.py:136-141 harmonic_synth backward w.r.t. amplitudes at the op boundary:
 * grad_amplitudes[B,T,H] = grad[B,T] * sin(fl32(omega[B,T] * k)); omega from ddsp_hip_phase. */
int ddsp_hip_harmonic_synth_backward(const float* omega, const float* grad, float* grad_amplitudes,
                                     int64_t batch, int64_t n_samples, int64_t n_harmonic, void* stream);

/* core.py:144-166 amp_to_impulse_response backward: grad_impulse[rows,target] -> grad_amp[rows,NB]. */
int ddsp_hip_amp_to_impulse_response_backward(const float* grad_impulse, float* grad_amp, int64_t rows,
                                              int64_t n_bands, int64_t target_size, void* stream);

/* modules.py:44-67 HarmonicSynth.get_controls backward: (grad_amplitudes[rows], grad_distribution
 * [rows,H]) -> gradients of the raw inputs (strided as in ddsp_hip_harmonic_controls). */
int ddsp_hip_harmonic_controls_backward(const float* amplitudes_raw, int64_t amp_stride,
                                        const float* distribution_raw, int64_t dist_stride, const float* f0,
                                        const float* grad_amplitudes, const float* grad_distribution,
                                        float* grad_amplitudes_raw, float* grad_distribution_raw,
                                        int64_t rows, int64_t n_harmonic, float sample_rate, void* stream);

/* modules.py:69-80 HarmonicSynth.forward backward (ddsp_hip_harmonic_synth_frames): the sine products
 * summed over each block, dA[b,f,k] = sum_t grad[t] sin(w_t k), then grad_distribution = dA * amp and
 * grad_amplitudes = sum_k dA * distribution.  `distribution` is the normalised distribution
 * BEFORE the in-place multiplication by the amplitudes. */
int ddsp_hip_harmonic_synth_frames_backward(const float* f0, const float* amplitudes, const float* distribution,
                                            const float* grad, float* grad_amplitudes,
                                            float* grad_distribution, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream);

/* decoder.py:106-113 + modules.py:44-80 backward (ddsp_hip_harmonic_synth_params, and the harmonic
 * half of ddsp_hip_synth_frames): grad[B,F*bs] -> grad_param[B,F,H+1]. */
int ddsp_hip_harmonic_synth_params_backward(const float* f0, const float* param, const float* grad,
                                            float* grad_param, int64_t batch, int64_t frames,
                                            int64_t n_harmonic, int64_t block_size, float sample_rate,
                                            void* stream);

/* decoder.py:106-121 backward (ddsp_hip_synth_frames): grad_param[B,F,H+1] and grad_magnitudes[B,F,NB]
 * (raw projections) from the upstream gradient of the signal, as two launches (harmonic, noise); the noise
 * is `noise` or the forward's Philox (seed, offset).  grad_noise (nullable) is a separate upstream
 * gradient for the noise half (when the parts are used separately); NULL = grad_harmonic. */
int ddsp_hip_synth_frames_backward(const float* f0, const float* param, const float* raw_magnitudes, float bias,
                                   const float* noise, uint64_t seed, uint64_t offset, const float* grad_harmonic,
                                   const float* grad_noise, float* grad_param, float* grad_magnitudes,
                                   int64_t batch, int64_t frames, int64_t n_harmonic, int64_t n_bands,
                                   int64_t block_size, float sample_rate, void* stream);

/* modules.py:111-128 FilteredNoise backward (ddsp_hip_filtered_noise[_params], the noise half of
 * ddsp_hip_synth_frames): grad[B,F*bs] -> grad_magnitudes[B,F,NB].  The noise is `noise` as given
 * to the forward, or (noise == NULL) regenerated from the forward's (seed, offset).  raw != 0:
 * `magnitudes` are the raw projections and scale_function(x + bias) is differentiated too. */
int ddsp_hip_filtered_noise_backward(const float* magnitudes, const float* noise, uint64_t seed, uint64_t offset,
                                     int raw, float bias, const float* grad, float* grad_magnitudes,
                                     int64_t batch, int64_t frames, int64_t n_bands, int64_t block_size,
                                     void* stream);

/* modules.py:28-35 Reverb.forward backward.
 *   ddsp_hip_reverb_apply_transposed: grad_x[b,t] = sum_tau grad[b,t+tau] IR[tau] (same spectrum and
 *     workspace as ddsp_hip_reverb_apply);
 *   ddsp_hip_reverb_backward: grad_x (nullable) as above and grad_impulse[tau] (nullable) =
 *     sum_b sum_t grad[b,t+tau] x[b,t] for tau < L (zero for taps cropped away when L > n_samples),
 *     sharing one transform of grad.  input_spectra (nullable): the first
 *     ddsp_hip_reverb_input_spectra_bytes bytes of the workspace ddsp_hip_reverb_apply used for this
 *     x, which hold x's partition spectra on return — kept by the caller, they spare a transform of x;
 *   ddsp_hip_reverb_impulse_backward (modules.py:21-26): grad_impulse -> grad_noise[L], and the
 *     device scalars grad_decay, grad_wet (taps >= grad_length carry no gradient). */
int ddsp_hip_reverb_apply_transposed(const float* grad, const float* spectrum, float* grad_x, int64_t batch,
                                     int64_t n_samples, int64_t ir_length, void* workspace,
                                     size_t workspace_bytes, void* stream);
size_t ddsp_hip_reverb_input_spectra_bytes(int64_t batch, int64_t n_samples);
size_t ddsp_hip_reverb_backward_workspace_size(int64_t batch, int64_t n_samples, int64_t ir_length,
                                               int have_input_spectra);
int ddsp_hip_reverb_backward(const float* x, const float* input_spectra, const float* spectrum, const float* grad,
                             float* grad_x, float* grad_impulse, int64_t batch, int64_t n_samples,
                             int64_t ir_length, void* workspace, size_t workspace_bytes, void* stream);
/* modules.py:21-35 Reverb.forward backward with respect to the signal AND the reverb's parameters in one call:
 * ddsp_hip_reverb_backward's grad_x (nullable) and ddsp_hip_reverb_impulse_backward's grad_noise[ir_length],
 * grad_decay, grad_wet (device scalars) from grad_impulse without materialising it — the partition
 * transforms of the impulse gradient also apply build_impulse's backward and reduce the decay / wet sums
 * (in a fixed order: deterministic).  Workspace: ddsp_hip_reverb_backward_workspace_size. */
int ddsp_hip_reverb_backward_params(const float* x, const float* input_spectra, const float* spectrum, const float* grad,
                                    const float* noise, const float* decay, const float* wet, float sample_rate,
                                    float* grad_x, float* grad_noise, float* grad_decay, float* grad_wet, int64_t batch,
                                    int64_t n_samples, int64_t ir_length, void* workspace, size_t workspace_bytes,
                                    void* stream);
size_t ddsp_hip_reverb_impulse_backward_workspace_size(int64_t length);
int ddsp_hip_reverb_impulse_backward(const float* noise, const float* decay, const float* wet,
                                     const float* grad_impulse, int64_t length, int64_t grad_length,
                                     float sample_rate, float* grad_noise, float* grad_decay, float* grad_wet,
                                     void* workspace, size_t workspace_bytes, void* stream);

/* Two-stage serving pipeline (ddsp_pytorch_amd.synth.PipelinedSynthPath; no reference counterpart:
 * the reference synthesises one batch at a time, decoder.py:101-136).  A HIP stream restricted to
 * the CUs whose bits are set in cu_mask (mask_words 32-bit words, bit c = CU index c; HIP deals
 * consecutive indices over the XCDs).  DDSP_HIP_ELAUNCH if the runtime refuses the mask.  The
 * caller owns the stream and releases it with ddsp_hip_stream_destroy. */
int ddsp_hip_stream_create_cu_masked(const uint32_t* cu_mask, int mask_words, void** stream);
int ddsp_hip_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DDSP_HIP_H */
