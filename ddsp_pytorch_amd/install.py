"""Install the gfx950 path under an imported reference ``ddsp`` package.

Function level: ``ddsp/__init__.py:1`` re-exports ``ddsp.core`` and the synth modules call
``ddsp.<fn>`` at call time (modules.py:33,53-56,74-78,113,117,125), so rebinding the six
package attributes redirects every caller.  Module level: the reference classes'
forwards are replaced by the fused ones (same instance attributes and parameters).
``uninstall()`` restores everything.
"""
from . import core, decoder, encoder, modules

FUNCTIONS = ("scale_function", "remove_above_nyquist", "upsample", "harmonic_synth",
             "amp_to_impulse_response", "fft_convolve")
# the training loss's spectrograms (core.py:27-41); train.py:9 binds them at import time, so
# install() must run before train.py is imported.  Rebound on ddsp and ddsp.core.
LOSS_FUNCTIONS = ("multiscale_fft", "safe_log")
METHODS = {
    "HarmonicSynth": ("get_controls", "forward"),
    "FilteredNoise": ("get_controls", "forward", "draw_noise"),
    "Reverb": ("build_impulse", "forward", "invalidate", "_spectrum", "_ir_cache", "_forward_cached"),
}


class Installation:
    def __init__(self, pkg, saved_fns, saved_methods):
        self.pkg, self._fns, self._methods = pkg, saved_fns, saved_methods

    def uninstall(self):
        for (obj, name), fn in self._fns.items():
            setattr(obj, name, fn)
        for (cls, name), fn in self._methods.items():
            if fn is None:
                delattr(cls, name)
            else:
                setattr(cls, name, fn)
        self._fns, self._methods = {}, {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.uninstall()


def install(pkg=None, functions=True, module_forwards=True):
    """Redirect the reference package ``pkg`` (default: ``import ddsp``) to the gfx950 kernels."""
    if pkg is None:
        import ddsp as pkg  # noqa: the reference package, when importable
    saved_fns, saved_methods = {}, {}
    if functions:
        for name in FUNCTIONS:
            saved_fns[(pkg, name)] = getattr(pkg, name)
            setattr(pkg, name, getattr(core, name))
        for obj in (pkg, getattr(pkg, "core", None)):
            for name in LOSS_FUNCTIONS:
                if obj is not None and hasattr(obj, name):
                    saved_fns[(obj, name)] = getattr(obj, name)
                    setattr(obj, name, getattr(core, name))
    if module_forwards:
        ref_modules = pkg.models.modules
        for cls_name, names in METHODS.items():
            ref_cls = getattr(ref_modules, cls_name)
            ours = getattr(modules, cls_name)
            for name in names:
                saved_methods[(ref_cls, name)] = ref_cls.__dict__.get(name)
                setattr(ref_cls, name, ours.__dict__[name])
        # the decoder network's GRU recurrence (decoder.py:43-68) on the step kernel, and
        # DDSPDecoder.forward (decoder.py:101-136) with its synthesis section on the fused kernel
        # (both synths, their controls, the sum and the returned control dicts in one launch)
        ref_decoder_mod = getattr(pkg.models, "decoder", None)
        for cls_name, fn in (("GRUDecoder", decoder.gru_decoder_forward), ("DDSPDecoder", decoder.decoder_forward)):
            ref_cls = getattr(ref_decoder_mod, cls_name, None)
            if ref_cls is not None:
                saved_methods[(ref_cls, "forward")] = ref_cls.__dict__.get("forward")
                setattr(ref_cls, "forward", fn)
        # the second caller, DDSPAutoencoder.forward (encoder.py:63-103): the same fused synthesis
        # section after its MFCC encoder (whose GRU, encoder.py:19-25, runs on the step kernel too)
        ref_encoder_mod = getattr(pkg.models, "encoder", None)
        for cls_name, fn in (("MFCCEncoder", encoder.mfcc_encoder_forward),
                             ("DDSPAutoencoder", encoder.autoencoder_forward)):
            ref_cls = getattr(ref_encoder_mod, cls_name, None)
            if ref_cls is not None:
                saved_methods[(ref_cls, "forward")] = ref_cls.__dict__.get("forward")
                setattr(ref_cls, "forward", fn)
    return Installation(pkg, saved_fns, saved_methods)
