"""install() into the REAL reference package (development container only: skipped where
/root/reference is absent, e.g. on the GPU box).

The reference is imported with SURVEY.md §8(c)'s placeholder modules for librosa, crepe and
pytorch_lightning (imported by ddsp/core.py:5-6 and ddsp/data.py:5, unused by the synthesis
path).  After install(ddsp), every method swapped onto the reference's classes must resolve on
real reference instances: each `self.<attr>` the swapped method reads must exist on the
instance (the reference's __init__ never sets noise_mode, _ir_caches or cache_spectrum, so
those may only be read through getattr with a default).  The functions must refuse CPU tensors
loudly (no CPU fallback).  uninstall() restores the reference exactly.
"""
import ast
import importlib
import inspect
import os
import sys
import textwrap
import types

import pytest
import torch

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "ddsp")),
                                reason="reference checkout not present (GPU box)")


def _import_reference():
    sys.dont_write_bytecode = True  # the reference tree is read-only
    for name in ("librosa", "crepe"):
        sys.modules.setdefault(name, types.ModuleType(name))
    pl = types.ModuleType("pytorch_lightning")
    pl.LightningDataModule = type("LightningDataModule", (), {})
    sys.modules.setdefault("pytorch_lightning", pl)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    ddsp = importlib.import_module("ddsp")
    importlib.import_module("ddsp.models.encoder")
    decoder = importlib.import_module("ddsp.models.decoder")
    modules = importlib.import_module("ddsp.models.modules")
    return ddsp, modules, decoder


def _self_reads(fn, guarded=None):
    """Attributes a method reads as plain `self.X` (not assigned earlier in it, not via getattr).
    Reads inside `if getattr(self, ...)` / `if self.flag` blocks go to ``guarded`` instead."""
    tree = ast.parse(textwrap.dedent(inspect.getsource(fn)))
    stored, reads = set(), []
    sink = [reads]

    def is_self_guard(t):
        if isinstance(t, ast.Call) and isinstance(t.func, ast.Name) and t.func.id == "getattr":
            return isinstance(t.args[0], ast.Name) and t.args[0].id == "self"
        return isinstance(t, ast.Attribute) and isinstance(t.value, ast.Name) and t.value.id == "self"

    class V(ast.NodeVisitor):
        def visit_If(self, node):
            self.visit(node.test)
            if is_self_guard(node.test) and guarded is not None:
                sink.append(guarded)
                for b in node.body:
                    self.visit(b)
                sink.pop()
            else:
                for b in node.body:
                    self.visit(b)
            for b in node.orelse:
                self.visit(b)

        def visit_Call(self, node):
            # getattr(self, "x", default) is the tolerant form: skip its target
            if isinstance(node.func, ast.Name) and node.func.id == "getattr" and len(node.args) == 3:
                for a in node.args[2:]:
                    self.visit(a)
                return
            self.generic_visit(node)

        def visit_Attribute(self, node):
            if isinstance(node.value, ast.Name) and node.value.id == "self":
                if isinstance(node.ctx, ast.Store):
                    stored.add(node.attr)
                elif node.attr not in stored:
                    sink[-1].append(node.attr)
            self.generic_visit(node)

        def visit_Assign(self, node):  # right-hand side first, then the targets
            self.visit(node.value)
            for t in node.targets:
                self.visit(t)

    V().visit(tree)
    return set(reads)


def test_install_resolves_on_reference_instances():
    ddsp, ref_modules, ref_decoder = _import_reference()
    import ddsp_pytorch_amd as dd
    install = importlib.import_module("ddsp_pytorch_amd.install")

    torch.manual_seed(0)
    model = ref_decoder.DDSPDecoder(32, 8, 9, 48000, 64, True)  # decoder.py:76-99
    instances = {"HarmonicSynth": model.harmonic_synth, "FilteredNoise": model.noise_synth,
                 "Reverb": model.reverb}
    originals = {(c, n): getattr(ref_modules, c).__dict__.get(n)
                 for c, names in install.METHODS.items() for n in names}
    orig_fns = {n: getattr(ddsp, n) for n in install.FUNCTIONS}
    orig_gru = ref_decoder.GRUDecoder.__dict__["forward"]
    orig_dec = ref_decoder.DDSPDecoder.__dict__["forward"]

    inst = dd.install(ddsp)
    try:
        for cls_name, names in install.METHODS.items():
            ref_cls = getattr(ref_modules, cls_name)
            obj = instances[cls_name]
            assert type(obj) is ref_cls
            for name in names:
                fn = ref_cls.__dict__[name]
                assert fn is getattr(dd.modules, cls_name).__dict__[name]
                missing = {a for a in _self_reads(fn) if not hasattr(obj, a)}
                assert not missing, f"{cls_name}.{name} reads {missing}, absent on reference instances"
                assert callable(getattr(obj, name))  # bound on the reference instance
        # the GRU recurrence on the step kernel, against the reference's GRUDecoder instance
        fn = ref_decoder.GRUDecoder.__dict__["forward"]
        guarded = []
        missing = {a for a in _self_reads(fn, guarded) if not hasattr(model.decoder, a)}
        assert not missing, missing
        # reads behind `if getattr(self, "add_z", False)`: present on a reference instance with z
        with_z = ref_decoder.GRUDecoder(32, z_dim=4)
        assert guarded and all(hasattr(with_z, a) for a in guarded), guarded
        # DDSPDecoder.forward with the fused synthesis section, against the reference's instance:
        # every self.X it (and decoder_synthesize) reads exists on a reference DDSPDecoder, and the
        # attributes it reads off the synth modules too
        assert ref_decoder.DDSPDecoder.__dict__["forward"] is dd.decoder.decoder_forward
        for fn in (dd.decoder.decoder_forward, dd.decoder.decoder_synthesize, dd.decoder.decoder_projections):
            missing = {a for a in _self_reads(fn) if not hasattr(model, a)}
            assert not missing, f"{fn.__name__} reads {missing}, absent on a reference DDSPDecoder"
        for attr in ("block_size", "sample_rate"):
            assert hasattr(model.harmonic_synth, attr)
        for attr in ("block_size", "initial_bias"):
            assert hasattr(model.noise_synth, attr)
        batch = {"pitch": torch.full((1, 4, 1), 220.0), "loudness": torch.zeros(1, 4, 1)}
        with pytest.raises(Exception):
            model(batch)  # CPU tensors: the synthesis refuses (no CPU fallback)
        # the rebound functions: the same names, and no CPU fallback
        for n in install.FUNCTIONS:
            assert getattr(ddsp, n) is getattr(dd.core, n)
        with pytest.raises(Exception):
            ddsp.scale_function(torch.zeros(2, 3))
        with pytest.raises(Exception):
            model.reverb(torch.zeros(1, 64, 1))  # swapped forward on a real instance: refuses CPU
    finally:
        inst.uninstall()
    for (c, n), f in originals.items():
        assert getattr(ref_modules, c).__dict__.get(n) is f
    for n, f in orig_fns.items():
        assert getattr(ddsp, n) is f
    assert ref_decoder.GRUDecoder.__dict__["forward"] is orig_gru
    assert ref_decoder.DDSPDecoder.__dict__["forward"] is orig_dec


def test_projection_hooks_keep_module_calls():
    """decoder_projections runs the two projections as one GEMM only while nothing observes the
    module calls: a forward hook (or a Linear subclass) keeps harmonic_proj/noise_proj as calls."""
    import torch
    from ddsp_pytorch_amd.decoder import _hooked
    lin = torch.nn.Linear(4, 3)
    assert not _hooked(lin)
    h = lin.register_forward_hook(lambda m, i, o: None)
    assert _hooked(lin)
    h.remove()
    assert not _hooked(lin)

    class Wrapped(torch.nn.Linear):
        def forward(self, x):
            return super().forward(x) * 2

    assert _hooked(Wrapped(4, 3))


def test_install_routes_the_autoencoder():
    """The reference's second caller of the path, DDSPAutoencoder.forward (encoder.py:63-103), and its
    MFCCEncoder.forward are swapped by install() for this package's (the fused synthesis section after
    the encoder and the z-conditioned decoder); every self.X they read resolves on real reference
    instances; the swapped forward refuses CPU tensors; uninstall() restores both."""
    ddsp, ref_modules, ref_decoder = _import_reference()
    ref_encoder = importlib.import_module("ddsp.models.encoder")
    import ddsp_pytorch_amd as dd
    torch.manual_seed(0)
    model = ref_encoder.DDSPAutoencoder(32, 8, 9, 48000, 64, True)
    orig = {c: getattr(ref_encoder, c).__dict__["forward"] for c in ("DDSPAutoencoder", "MFCCEncoder")}
    inst = dd.install(ddsp)
    try:
        assert ref_encoder.DDSPAutoencoder.__dict__["forward"] is dd.encoder.autoencoder_forward
        assert ref_encoder.MFCCEncoder.__dict__["forward"] is dd.encoder.mfcc_encoder_forward
        for fn in (dd.encoder.autoencoder_forward, dd.decoder.decoder_synthesize, dd.decoder.decoder_projections):
            missing = {a for a in _self_reads(fn) if not hasattr(model, a)}
            assert not missing, f"{fn.__name__} reads {missing}, absent on a reference DDSPAutoencoder"
        missing = {a for a in _self_reads(dd.encoder.mfcc_encoder_forward) if not hasattr(model.encoder, a)}
        assert not missing, missing
        # the z-conditioned GRUDecoder of the reference takes the swapped forward's z path
        guarded = []
        missing = {a for a in _self_reads(dd.decoder.gru_decoder_forward, guarded) if not hasattr(model.decoder, a)}
        assert not missing and all(hasattr(model.decoder, a) for a in guarded)
        # on the host the encoder (plain torch) still computes the reference's z
        mfcc = torch.randn(1, 4, 30)
        with torch.no_grad():
            z_ours = model.encoder(mfcc)
        inst.uninstall()
        with torch.no_grad():
            z_ref = model.encoder(mfcc)
        torch.testing.assert_close(z_ours, z_ref, rtol=1e-6, atol=1e-7)
        inst = dd.install(ddsp)
        batch = {"pitch": torch.full((1, 4, 1), 220.0), "loudness": torch.zeros(1, 4, 1), "mfcc": mfcc}
        with pytest.raises(Exception):
            model(batch)  # CPU tensors: the synthesis refuses (no CPU fallback)
    finally:
        inst.uninstall()
    for c, f in orig.items():
        assert getattr(ref_encoder, c).__dict__["forward"] is f
