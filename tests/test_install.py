"""install()/uninstall() host logic on a package shaped like the reference (no GPU needed):
the six late-bound functions, the training-loss functions on ddsp and ddsp.core, the three synth
modules' methods and GRUDecoder.forward are rebound, then restored exactly."""
import importlib
import types

import ddsp_pytorch_amd as dd
from ddsp_pytorch_amd import core, decoder, modules

install = importlib.import_module("ddsp_pytorch_amd.install")  # the module (the package exports the function)


def fake_reference():
    pkg = types.ModuleType("ddsp_like")
    pkg.core = types.ModuleType("ddsp_like.core")
    for name in install.FUNCTIONS + install.LOSS_FUNCTIONS:
        f = (lambda n: (lambda *a, **k: n))(name)
        setattr(pkg, name, f)
        if name in install.LOSS_FUNCTIONS:
            setattr(pkg.core, name, f)
    pkg.models = types.SimpleNamespace()
    classes = {}
    for cls_name, names in install.METHODS.items():
        classes[cls_name] = type(cls_name, (), {n: (lambda self: cls_name) for n in names if n != "_spectrum"})
    pkg.models.modules = types.SimpleNamespace(**classes)
    pkg.models.decoder = types.SimpleNamespace(GRUDecoder=type("GRUDecoder", (), {"forward": lambda self: "ref"}))
    return pkg


def test_install_roundtrip():
    pkg = fake_reference()
    before_fns = {n: getattr(pkg, n) for n in install.FUNCTIONS + install.LOSS_FUNCTIONS}
    before_core = {n: getattr(pkg.core, n) for n in install.LOSS_FUNCTIONS}
    gru_fwd = pkg.models.decoder.GRUDecoder.__dict__["forward"]
    inst = dd.install(pkg)
    for n in install.FUNCTIONS + install.LOSS_FUNCTIONS:
        assert getattr(pkg, n) is getattr(core, n)
    for n in install.LOSS_FUNCTIONS:
        assert getattr(pkg.core, n) is getattr(core, n)
    for cls_name, names in install.METHODS.items():
        ref_cls = getattr(pkg.models.modules, cls_name)
        for n in names:
            assert ref_cls.__dict__[n] is getattr(modules, cls_name).__dict__[n]
    assert pkg.models.decoder.GRUDecoder.__dict__["forward"] is decoder.gru_decoder_forward
    inst.uninstall()
    for n, f in before_fns.items():
        assert getattr(pkg, n) is f
    for n, f in before_core.items():
        assert getattr(pkg.core, n) is f
    assert pkg.models.decoder.GRUDecoder.__dict__["forward"] is gru_fwd
    assert "_spectrum" not in pkg.models.modules.Reverb.__dict__
