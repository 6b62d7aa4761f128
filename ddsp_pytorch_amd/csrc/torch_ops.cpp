// TorchScript-visible operators `torch.ops.ddsp_hip.*` over the C-ABI (include/ddsp_hip.h).
//
// The reference's export path (export.py:23-65) scripts the model and the realtime host
// (realtime/ddsp_tilde/ddsp_model.cpp:13-52) runs it through libtorch.  Python-level drop-ins
// are invisible to TorchScript, so the synthesis functions are registered here as operators
// with the reference's argument meaning; a scripted graph calls them like any aten op.
// Host code only: every op validates shapes, allocates outputs/workspaces with ATen on the
// tensors' device, and enqueues the C-ABI entry point on the current HIP stream.  Errors
// surface as c10::Error (RuntimeError in Python), as the reference's torch ops would.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <optional>
#include <tuple>

#include "ddsp_hip.h"

namespace {

void* stream_of(const at::Tensor& t) {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "ddsp_hip: ", name, " must be on a HIP device (no CPU fallback)");
  TORCH_CHECK(t.scalar_type() == at::kFloat, "ddsp_hip: ", name, " must be float32");
}

at::Tensor c16(const at::Tensor& t) {  // contiguous + 16-byte aligned (float4 accesses)
  at::Tensor c = t.contiguous();
  if (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16) c = c.clone();
  return c;
}

void ok(int st, const char* fn) {
  TORCH_CHECK(st == DDSP_HIP_OK, "ddsp_hip_", fn, " failed: ", ddsp_hip_status_string(st));
}

at::Tensor workspace(size_t bytes, const at::Tensor& like) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 1)}, like.options().dtype(at::kByte));
}

// ---------------- ddsp/core.py ----------------
at::Tensor scale_function(const at::Tensor& x) {  // core.py:77-78
  check_dev(x, "x");
  at::Tensor xc = c16(x), y = at::empty_like(xc);
  ok(ddsp_hip_scale_function(xc.data_ptr<float>(), y.data_ptr<float>(), xc.numel(), 0.0f, stream_of(xc)),
     "scale_function");
  return y;
}

at::Tensor remove_above_nyquist(const at::Tensor& amplitudes, const at::Tensor& f0, double sample_rate) {
  check_dev(amplitudes, "amplitudes");  // core.py:70-74
  check_dev(f0, "f0");
  TORCH_CHECK(f0.size(-1) == 1, "remove_above_nyquist: f0 must end in a size-1 dim");
  const int64_t H = amplitudes.size(-1);
  auto lead = at::infer_size(amplitudes.sizes().slice(0, amplitudes.dim() - 1), f0.sizes().slice(0, f0.dim() - 1));
  std::vector<int64_t> sa(lead), sf(lead);
  sa.push_back(H);
  sf.push_back(1);
  at::Tensor a = c16(amplitudes.expand(sa)), f = c16(f0.expand(sf));
  at::Tensor out = at::empty_like(a);
  ok(ddsp_hip_remove_above_nyquist(a.data_ptr<float>(), f.data_ptr<float>(), out.data_ptr<float>(),
                                   a.numel() / std::max<int64_t>(H, 1), H, (float)sample_rate, stream_of(a)),
     "remove_above_nyquist");
  return out;
}

at::Tensor upsample(const at::Tensor& signal, int64_t factor) {  // core.py:64-67
  check_dev(signal, "signal");
  TORCH_CHECK(signal.dim() == 3, "upsample: expected [batch, frames, channels]");
  at::Tensor x = c16(signal);
  const int64_t B = x.size(0), F = x.size(1), C = x.size(2);
  at::Tensor y = at::empty({B, F * factor, C}, x.options());
  ok(ddsp_hip_upsample(x.data_ptr<float>(), y.data_ptr<float>(), B, F, C, factor, stream_of(x)), "upsample");
  return y;
}

at::Tensor harmonic_synth(const at::Tensor& f0, const at::Tensor& amplitudes, double sample_rate) {
  check_dev(f0, "f0");  // core.py:136-141
  check_dev(amplitudes, "amplitudes");
  TORCH_CHECK(amplitudes.dim() == 3 && f0.dim() == 3 && f0.size(2) == 1 && f0.size(0) == amplitudes.size(0) &&
                  f0.size(1) == amplitudes.size(1),
              "harmonic_synth: expected f0 [B,T,1] and amplitudes [B,T,H]");
  at::Tensor f = c16(f0), a = c16(amplitudes);
  const int64_t B = a.size(0), T = a.size(1), H = a.size(2);
  at::Tensor out = at::empty({B, T, 1}, f.options());
  at::Tensor ws = workspace(ddsp_hip_harmonic_synth_workspace_size(B, T), f);
  ok(ddsp_hip_harmonic_synth(f.data_ptr<float>(), a.data_ptr<float>(), out.data_ptr<float>(), B, T, H,
                             (float)sample_rate, ws.data_ptr(), ws.numel(), stream_of(f)),
     "harmonic_synth");
  return out;
}

at::Tensor amp_to_impulse_response(const at::Tensor& amp, int64_t target_size) {  // core.py:144-166
  check_dev(amp, "amp");
  const int64_t NB = amp.size(-1);
  TORCH_CHECK(NB >= 2, "amp_to_impulse_response: need at least 2 bands");
  at::Tensor x = c16(amp);
  std::vector<int64_t> shape(amp.sizes().begin(), amp.sizes().end());
  shape.back() = target_size;
  at::Tensor out = at::empty(shape, x.options());
  ok(ddsp_hip_amp_to_impulse_response(x.data_ptr<float>(), out.data_ptr<float>(), x.numel() / NB, NB,
                                      target_size, stream_of(x)),
     "amp_to_impulse_response");
  return out;
}

at::Tensor fft_convolve(const at::Tensor& signal, const at::Tensor& kernel) {  // core.py:169-176
  check_dev(signal, "signal");
  check_dev(kernel, "kernel");
  const int64_t N = signal.size(-1);
  TORCH_CHECK(kernel.size(-1) == N, "fft_convolve: signal and kernel lengths differ");
  auto lead = at::infer_size(signal.sizes().slice(0, signal.dim() - 1), kernel.sizes().slice(0, kernel.dim() - 1));
  std::vector<int64_t> full(lead);
  full.push_back(N);
  int64_t rows = 1;
  for (auto d : lead) rows *= d;
  at::Tensor s = c16(signal.expand(full));
  at::Tensor k;
  int64_t krows;
  if (kernel.numel() == N) {
    k = c16(kernel.reshape({N}));
    krows = 1;
  } else {
    k = c16(kernel.expand(full));
    krows = rows;
  }
  at::Tensor out = at::empty(full, s.options());
  at::Tensor ws = workspace(ddsp_hip_fft_convolve_workspace_size(rows, krows, N), s);
  ok(ddsp_hip_fft_convolve(s.data_ptr<float>(), k.data_ptr<float>(), out.data_ptr<float>(), rows, krows, N,
                           ws.data_ptr(), ws.numel(), stream_of(s)),
     "fft_convolve");
  return out;
}

// ---------------- ddsp/models/modules.py (fused) ----------------
std::tuple<at::Tensor, at::Tensor> harmonic_controls(const at::Tensor& amplitudes, const at::Tensor& distribution,
                                                     const at::Tensor& f0, double sample_rate) {
  check_dev(amplitudes, "amplitudes");  // modules.py:44-67
  check_dev(distribution, "harmonic_distribution");
  check_dev(f0, "f0");
  TORCH_CHECK(distribution.dim() == 3, "harmonic_controls: distribution must be [B,F,H]");
  const int64_t B = distribution.size(0), F = distribution.size(1), H = distribution.size(2);
  TORCH_CHECK(amplitudes.sizes() == at::IntArrayRef({B, F, 1}) && f0.sizes() == at::IntArrayRef({B, F, 1}),
              "harmonic_controls: amplitudes and f0 must be [B,F,1]");
  auto rows_view = [](const at::Tensor& t) {
    at::Tensor v = t;
    if (v.stride(-1) != 1 || v.stride(0) != v.size(1) * v.stride(1)) v = v.contiguous();
    return v;
  };
  at::Tensor a = rows_view(amplitudes), d = rows_view(distribution), f = c16(f0);
  at::Tensor amp_out = at::empty({B, F, 1}, f.options()), dist_out = at::empty({B, F, H}, f.options());
  ok(ddsp_hip_harmonic_controls(a.data_ptr<float>(), a.stride(1), d.data_ptr<float>(), d.stride(1),
                                f.data_ptr<float>(), amp_out.data_ptr<float>(), dist_out.data_ptr<float>(), B * F,
                                H, (float)sample_rate, stream_of(f)),
     "harmonic_controls");
  return {amp_out, dist_out};
}

at::Tensor harmonic_synth_frames(const at::Tensor& f0, const at::Tensor& amplitudes, at::Tensor& distribution,
                                 int64_t block_size, double sample_rate, bool write_back) {
  check_dev(f0, "f0");  // modules.py:69-80
  check_dev(amplitudes, "amplitudes");
  check_dev(distribution, "harmonic_distribution");
  const int64_t B = distribution.size(0), F = distribution.size(1), H = distribution.size(2);
  at::Tensor f = c16(f0), a = c16(amplitudes);
  at::Tensor d = distribution;
  if (write_back) {
    TORCH_CHECK(d.is_contiguous() && reinterpret_cast<uintptr_t>(d.data_ptr()) % 16 == 0,
                "harmonic_synth_frames: in-place write-back needs a contiguous distribution");
  } else {
    d = c16(d);
  }
  at::Tensor out = at::empty({B, F * block_size, 1}, f.options());
  ok(ddsp_hip_harmonic_synth_frames(f.data_ptr<float>(), a.data_ptr<float>(), d.data_ptr<float>(),
                                    write_back ? 1 : 0, out.data_ptr<float>(), B, F, H, block_size,
                                    (float)sample_rate, stream_of(f)),
     "harmonic_synth_frames");
  return out;
}

at::Tensor harmonic_synth_params(const at::Tensor& f0, const at::Tensor& param, int64_t block_size,
                                 double sample_rate) {
  check_dev(f0, "f0");  // decoder.py:106-113 + modules.py:44-80
  check_dev(param, "param");
  const int64_t B = param.size(0), F = param.size(1), H1 = param.size(2);
  TORCH_CHECK(f0.sizes() == at::IntArrayRef({B, F, 1}) && H1 >= 2, "harmonic_synth_params: bad shapes");
  at::Tensor f = c16(f0), p = c16(param);
  at::Tensor out = at::empty({B, F * block_size, 1}, f.options());
  ok(ddsp_hip_harmonic_synth_params(f.data_ptr<float>(), p.data_ptr<float>(), out.data_ptr<float>(), B, F, H1 - 1,
                                    block_size, (float)sample_rate, stream_of(f)),
     "harmonic_synth_params");
  return out;
}

at::Tensor filtered_noise(const at::Tensor& magnitudes, int64_t block_size, const std::optional<at::Tensor>& noise,
                          int64_t seed, int64_t offset, const std::optional<at::Tensor>& add,
                          std::optional<double> raw_bias) {
  check_dev(magnitudes, "magnitudes");  // modules.py:111-128
  const int64_t B = magnitudes.size(0), F = magnitudes.size(1), NB = magnitudes.size(2);
  at::Tensor m = c16(magnitudes);
  at::Tensor n, a;
  if (noise.has_value()) {
    check_dev(*noise, "noise");
    TORCH_CHECK(noise->sizes() == at::IntArrayRef({B, F, block_size}), "filtered_noise: noise must be [B,F,bs]");
    n = c16(*noise);
  }
  if (add.has_value()) {
    check_dev(*add, "add");
    TORCH_CHECK(add->numel() == B * F * block_size, "filtered_noise: add must have B*F*bs elements");
    a = c16(*add);
  }
  at::Tensor out = at::empty({B, F * block_size, 1}, m.options());
  const float* np = n.defined() ? n.data_ptr<float>() : nullptr;
  const float* ap = a.defined() ? a.data_ptr<float>() : nullptr;
  int st;
  if (raw_bias.has_value())
    st = ddsp_hip_filtered_noise_params(m.data_ptr<float>(), (float)*raw_bias, np, (uint64_t)seed, (uint64_t)offset,
                                        ap, out.data_ptr<float>(), nullptr, B, F, NB, block_size, stream_of(m));
  else
    st = ddsp_hip_filtered_noise(m.data_ptr<float>(), np, (uint64_t)seed, (uint64_t)offset, ap,
                                 out.data_ptr<float>(), nullptr, B, F, NB, block_size, stream_of(m));
  ok(st, "filtered_noise");
  return out;
}

// decoder.py:106-121 in one launch (ddsp_hip_synth_frames): harmonic + filtered noise, their controls and
// the sum; outside the fused kernel's shape envelope the two module kernels (harmonic_synth_params, then
// filtered_noise adding the harmonic).  parts: the harmonic and noise signals as well.
std::tuple<at::Tensor, at::Tensor, at::Tensor> synth_frames_impl(const at::Tensor& f0, const at::Tensor& param,
                                                                 const at::Tensor& mags, int64_t block_size,
                                                                 double sample_rate, double bias,
                                                                 const std::optional<at::Tensor>& noise,
                                                                 int64_t seed, int64_t offset, bool parts) {
  check_dev(f0, "f0");
  check_dev(param, "param");
  check_dev(mags, "mags");
  TORCH_CHECK(param.dim() == 3 && mags.dim() == 3, "synth_frames: param [B,F,H+1] and mags [B,F,NB] expected");
  const int64_t B = param.size(0), F = param.size(1), H1 = param.size(2), NB = mags.size(2);
  TORCH_CHECK(f0.sizes() == at::IntArrayRef({B, F, 1}) && mags.size(0) == B && mags.size(1) == F && H1 >= 2,
              "synth_frames: f0 [B,F,1], param [B,F,H+1], mags [B,F,NB] expected");
  at::Tensor f = c16(f0), p = c16(param), m = c16(mags), n;
  if (noise.has_value()) {
    check_dev(*noise, "noise");
    TORCH_CHECK(noise->sizes() == at::IntArrayRef({B, F, block_size}), "synth_frames: noise must be [B,F,bs]");
    n = c16(*noise);
  }
  const float* np = n.defined() ? n.data_ptr<float>() : nullptr;
  at::Tensor out = at::empty({B, F * block_size, 1}, f.options());
  at::Tensor harm = parts ? at::empty_like(out) : at::Tensor();
  at::Tensor nz = parts ? at::empty_like(out) : at::Tensor();
  int st = ddsp_hip_synth_frames(f.data_ptr<float>(), p.data_ptr<float>(), m.data_ptr<float>(), (float)bias, np,
                                 (uint64_t)seed, (uint64_t)offset, out.data_ptr<float>(),
                                 parts ? harm.data_ptr<float>() : nullptr, parts ? nz.data_ptr<float>() : nullptr, B,
                                 F, H1 - 1, NB, block_size, (float)sample_rate, stream_of(f));
  if (st == DDSP_HIP_ERANGE) {  // outside the fused kernel's envelope: the two module kernels
    at::Tensor h = parts ? harm : at::empty_like(out);
    ok(ddsp_hip_harmonic_synth_params(f.data_ptr<float>(), p.data_ptr<float>(), h.data_ptr<float>(), B, F, H1 - 1,
                                      block_size, (float)sample_rate, stream_of(f)),
       "harmonic_synth_params");
    st = ddsp_hip_filtered_noise_params(m.data_ptr<float>(), (float)bias, np, (uint64_t)seed, (uint64_t)offset,
                                        h.data_ptr<float>(), out.data_ptr<float>(),
                                        parts ? nz.data_ptr<float>() : nullptr, B, F, NB, block_size, stream_of(f));
  }
  ok(st, "synth_frames");
  return {out, harm, nz};
}

at::Tensor synth_frames(const at::Tensor& f0, const at::Tensor& param, const at::Tensor& mags, int64_t block_size,
                        double sample_rate, double bias, const std::optional<at::Tensor>& noise, int64_t seed,
                        int64_t offset) {
  return std::get<0>(synth_frames_impl(f0, param, mags, block_size, sample_rate, bias, noise, seed, offset, false));
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> synth_frames_parts(const at::Tensor& f0, const at::Tensor& param,
                                                                  const at::Tensor& mags, int64_t block_size,
                                                                  double sample_rate, double bias,
                                                                  const std::optional<at::Tensor>& noise,
                                                                  int64_t seed, int64_t offset) {
  return synth_frames_impl(f0, param, mags, block_size, sample_rate, bias, noise, seed, offset, true);
}

at::Tensor reverb_build_impulse(const at::Tensor& noise, const at::Tensor& decay, const at::Tensor& wet,
                                double sample_rate) {
  check_dev(noise, "noise");  // modules.py:21-26
  check_dev(decay, "decay");
  check_dev(wet, "wet");
  at::Tensor n = c16(noise), d = decay.contiguous(), w = wet.contiguous();
  const int64_t L = n.size(0);
  at::Tensor imp = at::empty({1, L, 1}, n.options());
  ok(ddsp_hip_reverb_build_impulse(n.data_ptr<float>(), d.data_ptr<float>(), w.data_ptr<float>(),
                                   imp.data_ptr<float>(), L, (float)sample_rate, stream_of(n)),
     "reverb_build_impulse");
  return imp;
}

at::Tensor reverb_spectrum(const at::Tensor& impulse, int64_t n_samples) {
  check_dev(impulse, "impulse");
  at::Tensor h = c16(impulse.reshape({-1}));
  const int64_t L = h.numel();
  at::Tensor spec = at::empty({(int64_t)ddsp_hip_reverb_spectrum_floats(n_samples, L)}, h.options());
  ok(ddsp_hip_reverb_spectrum(h.data_ptr<float>(), L, n_samples, spec.data_ptr<float>(), stream_of(h)),
     "reverb_spectrum");
  return spec;
}

at::Tensor reverb_apply(const at::Tensor& x, const at::Tensor& spectrum, int64_t ir_length) {
  check_dev(x, "x");  // modules.py:28-35
  check_dev(spectrum, "spectrum");
  const int64_t B = x.size(0), T = x.size(1);
  TORCH_CHECK(spectrum.numel() == (int64_t)ddsp_hip_reverb_spectrum_floats(T, ir_length),
              "reverb_apply: spectrum was computed for a different length");
  at::Tensor xc = c16(x);
  at::Tensor out = at::empty({B, T, 1}, xc.options());
  at::Tensor ws = workspace(ddsp_hip_reverb_workspace_size(B, T, ir_length), xc);
  ok(ddsp_hip_reverb_apply(xc.data_ptr<float>(), spectrum.data_ptr<float>(), out.data_ptr<float>(), B, T,
                           ir_length, ws.data_ptr(), ws.numel(), stream_of(xc)),
     "reverb_apply");
  return out;
}

}  // namespace

// ---------------- decoder.py:33-68: the GRU recurrence ----------------
std::tuple<at::Tensor, at::Tensor> gru(const at::Tensor& x, const at::Tensor& w_ih, const at::Tensor& w_hh,
                                       const at::Tensor& b_ih, const at::Tensor& b_hh,
                                       const std::optional<at::Tensor>& h0) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 3, "gru: x must be [batch, time, features]");
  const int64_t B = x.size(0), T = x.size(1), H = w_hh.size(1);
  TORCH_CHECK(w_hh.size(0) == 3 * H && w_ih.size(0) == 3 * H && w_ih.size(1) == x.size(2), "gru: weight shapes");
  at::Tensor xp = at::addmm(b_ih, x.reshape({B * T, x.size(2)}), w_ih.t()).view({B, T, 3 * H});
  at::Tensor out = at::empty({B, T, H}, x.options());
  at::Tensor h_last = at::empty({1, B, H}, x.options());
  at::Tensor h0c;
  if (h0.has_value() && h0->defined()) {
    check_dev(*h0, "h0");
    TORCH_CHECK(h0->numel() == B * H, "gru: h0 must hold batch x hidden values");
    h0c = c16(h0->reshape({B, H}));
  }
  at::Tensor whh = c16(w_hh), bhh = c16(b_hh);
  ok(ddsp_hip_gru_forward(xp.data_ptr<float>(), whh.data_ptr<float>(), bhh.data_ptr<float>(),
                          h0c.defined() ? h0c.data_ptr<float>() : nullptr, out.data_ptr<float>(),
                          h_last.data_ptr<float>(), nullptr, B, T, H, stream_of(x)),
     "gru_forward");
  return {out, h_last};
}

TORCH_LIBRARY(ddsp_hip, m) {
  m.def("scale_function(Tensor x) -> Tensor");
  m.def("remove_above_nyquist(Tensor amplitudes, Tensor f0, float sample_rate) -> Tensor");
  m.def("upsample(Tensor signal, int factor) -> Tensor");
  m.def("harmonic_synth(Tensor f0, Tensor amplitudes, float sample_rate) -> Tensor");
  m.def("amp_to_impulse_response(Tensor amp, int target_size) -> Tensor");
  m.def("fft_convolve(Tensor signal, Tensor kernel) -> Tensor");
  m.def("harmonic_controls(Tensor amplitudes, Tensor harmonic_distribution, Tensor f0, float sample_rate)"
        " -> (Tensor, Tensor)");
  m.def("harmonic_synth_frames(Tensor f0, Tensor amplitudes, Tensor(a!) harmonic_distribution, int block_size,"
        " float sample_rate, bool write_back=True) -> Tensor");
  m.def("harmonic_synth_params(Tensor f0, Tensor param, int block_size, float sample_rate) -> Tensor");
  m.def("filtered_noise(Tensor magnitudes, int block_size, Tensor? noise=None, int seed=0, int offset=0,"
        " Tensor? add=None, float? raw_bias=None) -> Tensor");
  m.def("synth_frames(Tensor f0, Tensor param, Tensor mags, int block_size, float sample_rate, float bias=-5.0,"
        " Tensor? noise=None, int seed=0, int offset=0) -> Tensor");
  m.def("synth_frames_parts(Tensor f0, Tensor param, Tensor mags, int block_size, float sample_rate,"
        " float bias=-5.0, Tensor? noise=None, int seed=0, int offset=0) -> (Tensor, Tensor, Tensor)");
  m.def("reverb_build_impulse(Tensor noise, Tensor decay, Tensor wet, float sample_rate) -> Tensor");
  m.def("reverb_spectrum(Tensor impulse, int n_samples) -> Tensor");
  m.def("reverb_apply(Tensor x, Tensor spectrum, int ir_length) -> Tensor");
  m.def("gru(Tensor x, Tensor w_ih, Tensor w_hh, Tensor b_ih, Tensor b_hh, Tensor? h0=None) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(ddsp_hip, CUDA, m) {  // HIP tensors dispatch under the CUDA key on ROCm
  m.impl("scale_function", &scale_function);
  m.impl("remove_above_nyquist", &remove_above_nyquist);
  m.impl("upsample", &upsample);
  m.impl("harmonic_synth", &harmonic_synth);
  m.impl("amp_to_impulse_response", &amp_to_impulse_response);
  m.impl("fft_convolve", &fft_convolve);
  m.impl("harmonic_controls", &harmonic_controls);
  m.impl("harmonic_synth_frames", &harmonic_synth_frames);
  m.impl("harmonic_synth_params", &harmonic_synth_params);
  m.impl("filtered_noise", &filtered_noise);
  m.impl("synth_frames", &synth_frames);
  m.impl("synth_frames_parts", &synth_frames_parts);
  m.impl("reverb_build_impulse", &reverb_build_impulse);
  m.impl("reverb_spectrum", &reverb_spectrum);
  m.impl("reverb_apply", &reverb_apply);
  m.impl("gru", &gru);
}
