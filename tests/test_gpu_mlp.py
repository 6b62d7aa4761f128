"""The decoder's MLP blocks (ddsp/core.py:122-129) with LayerNorm + LeakyReLU fused into one kernel
(core.layer_norm_leaky_relu, decoder.mlp_forward) against torch's modules on the same device, incl.
the one-feature first Linear folded into the kernel and outputs written into a column slice."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dd():
    import ddsp_pytorch_amd
    return ddsp_pytorch_amd


@pytest.mark.parametrize("in_size,hidden", [(1, 512), (514, 512), (512, 1024), (1, 1024)])
def test_mlp_forward_matches_torch(dd, in_size, hidden):
    from ddsp_pytorch_amd.decoder import mlp, mlp_forward
    torch.manual_seed(0)
    m = mlp(in_size, hidden, 3).cuda().eval()
    with torch.no_grad():  # non-trivial affine parameters
        for mod in m:
            if isinstance(mod, torch.nn.LayerNorm):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    x = torch.randn(7, 33, in_size, device="cuda") * 3.0
    with torch.no_grad():
        ref = m(x)
        got = mlp_forward(m, x)
        wide = torch.full((7, 33, 3 * hidden), 7.0, device="cuda")
        into = mlp_forward(m, x, out=wide[..., hidden:2 * hidden])
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)
    assert into.data_ptr() == wide[..., hidden:].data_ptr()
    torch.testing.assert_close(wide[..., hidden:2 * hidden], ref, rtol=2e-5, atol=2e-5)
    assert torch.all(wide[..., :hidden] == 7.0) and torch.all(wide[..., 2 * hidden:] == 7.0)


def test_layer_norm_leaky_relu_kernel(dd):
    torch.manual_seed(1)
    ln = torch.nn.LayerNorm(512).cuda()
    act = torch.nn.LeakyReLU()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
        h = torch.randn(1001, 512, device="cuda") * 10 + 3
        y = dd.core.layer_norm_leaky_relu(h, ln, act)
        torch.testing.assert_close(y, act(ln(h)), rtol=1e-5, atol=1e-5)
        # outside the kernel's shapes: None (the caller keeps torch's modules)
        assert dd.core.layer_norm_leaky_relu(torch.randn(4, 100, device="cuda"), torch.nn.LayerNorm(100).cuda(),
                                             act) is None


def test_mlp_under_autograd_keeps_torch(dd):
    """Training keeps torch's modules (their autograd): the fused path is inference-only."""
    from ddsp_pytorch_amd.decoder import _mlp_fusable, mlp
    m = mlp(1, 512, 3).cuda()
    x = torch.randn(2, 5, 1, device="cuda")
    assert not _mlp_fusable(m, x)
    with torch.no_grad():
        assert _mlp_fusable(m, x)


@pytest.mark.parametrize("rows", [1, 63, 64, 65, 1000])
@pytest.mark.parametrize("in_size", [512, 33])
def test_mlp_block_kernel(dd, rows, in_size):
    """core.mlp_block (Linear on the matrix cores + LayerNorm + LeakyReLU epilogue) against torch's
    modules: row counts around the 64-row workgroup tile, K not a multiple of the 16-wide K-step."""
    torch.manual_seed(rows + in_size)
    lin = torch.nn.Linear(in_size, 512).cuda()
    ln = torch.nn.LayerNorm(512).cuda()
    act = torch.nn.LeakyReLU()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
        x = torch.randn(rows, in_size, device="cuda") * 2.0
        y = dd.core.mlp_block(x, lin, ln, act)
        torch.testing.assert_close(y, act(ln(lin(x))), rtol=2e-5, atol=2e-5)


def test_mlp_forward_extras_match_cat(dd):
    """The decoder's out_mlp input [gru_out, f0, loudness] (decoder.py:68) given as x + two per-row
    extras: the same result as torch's modules on the concatenation, with no concatenation built."""
    from ddsp_pytorch_amd.decoder import mlp, mlp_forward
    torch.manual_seed(3)
    m = mlp(514, 512, 3).cuda().eval()
    gru_out = torch.randn(5, 101, 512, device="cuda")
    f0 = torch.rand(5, 101, 1, device="cuda") * 800 + 50
    loud = torch.randn(5, 101, 1, device="cuda") * 4
    with torch.no_grad():
        ref = m(torch.cat([gru_out, f0, loud], -1))
        got = mlp_forward(m, gru_out, extras=(f0, loud))
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)
    # outside the kernel's shapes (1024 outputs): None, the caller keeps the GEMM + LayerNorm route
    big = mlp(512, 1024, 1).cuda()
    with torch.no_grad():
        assert dd.core.mlp_block(gru_out, big[0], big[1], big[2]) is None



@pytest.mark.parametrize("K,n1,n2,rows", [(512, 101, 65, 12800), (512, 65, 65, 48), (512, 129, 65, 37),
                                          (64, 21, 17, 100), (32, 208, 16, 70)])
def test_projections(dd, K, n1, n2, rows):
    """decoder.py:106-117 as one launch (core.projections: ddsp_hip_projections at 512 inputs, else one GEMM over
    both layers' parameters stacked per call) against an fp64 host matmul.  The two results are column slices
    of one buffer with 16-byte aligned rows (the kernel route: n1 + n2 rounded up to 4; the GEMM route: to 64)."""
    torch.manual_seed(2)
    l1, l2 = torch.nn.Linear(K, n1).cuda(), torch.nn.Linear(K, n2).cuda()
    x = torch.randn(rows, K, device="cuda")
    with torch.no_grad():
        a, b = dd.core.projections(x, l1, l2)
    assert a.shape == (rows, n1) and b.shape == (rows, n2)
    assert a.stride(0) == b.stride(0) and b.data_ptr() == a.data_ptr() + 4 * n1
    assert a.stride(0) == (-(-(n1 + n2) // 4) * 4 if K == 512 else -(-(n1 + n2) // 64) * 64)
    x64 = x.double().cpu()
    for got, lin in ((a, l1), (b, l2)):
        ref = x64 @ lin.weight.double().cpu().t() + lin.bias.double().cpu()
        err = (got.double().cpu() - ref).abs().max().item()
        assert err < 2e-6 * (1 + ref.abs().max().item()), err


def test_projections_read_live_parameters(dd):
    """Nothing is cached: a write through .data between calls is seen by the next call."""
    torch.manual_seed(3)
    l1, l2 = torch.nn.Linear(512, 65).cuda(), torch.nn.Linear(512, 65).cuda()
    x = torch.randn(64, 512, device="cuda")
    with torch.no_grad():
        a0 = dd.core.projections(x, l1, l2)[0].clone()
        l1.weight.data.mul_(2.0)
        l1.bias.data.mul_(2.0)
        a1 = dd.core.projections(x, l1, l2)[0]
    torch.testing.assert_close(a1, 2 * a0, rtol=1e-6, atol=1e-6)


def _mlp_block_raw(dd, x, x_ld, lin, ln, rows, e0=None, e1=None, flags=0):
    """ddsp_hip_mlp_block on a raw [rows, x_ld] buffer (x_ld > K selects the staged, unaligned-load form)."""
    L = dd._lib
    y = torch.empty(rows, 512, device="cuda")
    L.call("mlp_block", L.ptr(x), x_ld, 512, L.ptr(lin.weight), lin.weight.shape[1], L.ptr(lin.bias), L.ptr(e0),
           L.ptr(e1), 1, L.ptr(ln.weight), L.ptr(ln.bias), float(ln.eps), 0.01, L.ptr(y), 512, rows, 512, flags,
           L.stream_of(y))
    return y


@pytest.mark.parametrize("rows,extras", [(12800, False), (1000, True), (65, False), (1, True)])
def test_mlp_block_resident_form_equals_staged_form(dd, rows, extras):
    """K = 512 with MLP_EXACT_F32 runs the x-resident f32 kernel (x tile in LDS, W streamed to registers, no
    barrier in the K loop); an x buffer with row stride 514 floats runs the staged kernel.  Same MFMA operands
    in the same k order: identical outputs, bit for bit, incl. the out_mlp's two extra columns.  The default
    (bf16x3) form matches torch at the same tolerance."""
    torch.manual_seed(rows)
    lin = torch.nn.Linear(514 if extras else 512, 512).cuda()
    ln = torch.nn.LayerNorm(512).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
        wide = torch.randn(rows, 514, device="cuda") * 2.0
        x = wide[:, :512].contiguous()
        e0 = torch.randn(rows, 1, device="cuda") if extras else None
        e1 = torch.randn(rows, 1, device="cuda") if extras else None
        a = _mlp_block_raw(dd, x, 512, lin, ln, rows, e0, e1, flags=dd.core.MLP_EXACT_F32)
        b = _mlp_block_raw(dd, wide, 514, lin, ln, rows, e0, e1)
        c = _mlp_block_raw(dd, x, 512, lin, ln, rows, e0, e1)
        ref_in = torch.cat([x, e0, e1], -1) if extras else x
        ref = torch.nn.functional.leaky_relu(ln(lin(ref_in)), 0.01)
    assert torch.equal(a, b)
    torch.testing.assert_close(a, ref, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(c, ref, rtol=2e-5, atol=2e-5)


def test_mlp_block_bf16x3_is_fp32_accurate(dd):
    """The bf16x3 Linear (six exact bf16 products per operand pair) against an fp64 evaluation of the same
    block: its error is of the f32-input MFMA's order (within 2x of it, RMS and max) — fp32-accurate."""
    torch.manual_seed(7)
    rows = 4096
    lin = torch.nn.Linear(512, 512).cuda()
    ln = torch.nn.LayerNorm(512).cuda()
    with torch.no_grad():
        x = torch.randn(rows, 512, device="cuda") * 3.0
        f32 = _mlp_block_raw(dd, x, 512, lin, ln, rows, flags=dd.core.MLP_EXACT_F32)
        bf3 = _mlp_block_raw(dd, x, 512, lin, ln, rows)
        h = x.double() @ lin.weight.double().t() + lin.bias.double()
        ref = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(
            h, (512,), ln.weight.double(), ln.bias.double(), ln.eps), 0.01)
    e32, e3 = (f32.double() - ref), (bf3.double() - ref)
    rms = lambda e: float(e.pow(2).mean().sqrt())
    assert rms(e3) < 2 * rms(e32) and float(e3.abs().max()) < 2 * float(e32.abs().max()), (rms(e3), rms(e32))


@pytest.mark.parametrize("rows,K,N", [(12800, 1024, 1536), (100, 512, 512), (65, 1024, 512), (7, 96, 512),
                                        (12800, 1536, 1024), (33, 1536, 512)])
def test_linear_bf16x3(dd, rows, K, N):
    """core.linear (ddsp_hip_linear: the GRU's input projection for every step, decoder.py:41, and K = 1536, its input gradient) against an fp64
    evaluation: within 2x of the f32 GEMM's (torch.addmm) error; K = 96 is outside the kernel and runs addmm."""
    torch.manual_seed(rows + K)
    x = torch.randn(rows, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    with torch.no_grad():
        y = dd.core.linear(x, w, b)
        y32 = torch.addmm(b, x, w.t())
        ref = torch.addmm(b.double(), x.double(), w.double().t())
    rms = lambda e: float(e.pow(2).mean().sqrt())
    assert y.shape == (rows, N)
    assert rms(y.double() - ref) <= 2 * rms(y32.double() - ref) + 1e-12, (rms(y.double() - ref), rms(y32.double() - ref))
    # (the max over a few rows fluctuates more than the RMS: 3x; at 33 x 512 outputs and K = 1536 the f32 GEMM's
    # max was 1.9e-6 and this kernel's 5.0e-6 on one draw, both ~1e-6 relative)
    assert float((y.double() - ref).abs().max()) <= 3 * float((y32.double() - ref).abs().max()) + 1e-12


@pytest.mark.parametrize("rows,n1,n2,x_ld", [(12800, 101, 65, 512), (37, 101, 65, 512), (200, 129, 65, 516),
                                              (64, 101, 0, 512), (130, 65, 300, 512)])
def test_projections_bf16x3(dd, rows, n1, n2, x_ld):
    """core.projections (ddsp_hip_projections: decoder.py:106-117's harmonic_proj and noise_proj in ONE launch,
    each layer's parameters read where they lie) against an fp64 evaluation: within 2x of the f32 GEMMs'
    (torch.addmm) error, RMS and max.  Ragged rows, a second 192-column block (129 + 65, 65 + 300), one layer
    (n2 = 0, the second pointer set unused) and a row stride past the 512 features."""
    torch.manual_seed(rows + n1 + n2)
    xb = torch.randn(rows, x_ld, device="cuda") * 2.0
    x = xb[:, :512]
    lin1 = torch.nn.Linear(512, n1).cuda()
    lin2 = torch.nn.Linear(512, n2).cuda()
    with torch.no_grad():
        p, m = dd.core.projections(x, lin1, lin2)
        refs = [torch.addmm(l.bias.double(), x.double(), l.weight.double().t()) for l in (lin1, lin2)]
        f32s = [torch.addmm(l.bias, x, l.weight.t()) for l in (lin1, lin2)]
    assert p.shape == (rows, n1) and m.shape == (rows, n2)
    rms = lambda e: float(e.pow(2).mean().sqrt()) if e.numel() else 0.0
    for y, ref, y32 in zip((p, m), refs, f32s):
        if not y.numel():
            continue
        e, e32 = y.double() - ref, y32.double() - ref
        assert rms(e) <= 2 * rms(e32) + 1e-12, (rms(e), rms(e32))
        assert float(e.abs().max()) <= 2 * float(e32.abs().max()) + 1e-12


def test_projections_route_and_envelope(dd, monkeypatch):
    """the projections take the one-launch kernel at 512 inputs (no stacking launch, no library GEMM) and fall
    back to stack_rows + one GEMM outside it (256 inputs), with the same values"""
    from ddsp_pytorch_amd import _lib
    calls = []
    real = _lib.call
    monkeypatch.setattr(_lib, "call", lambda name, *a, **k: calls.append(name) or real(name, *a, **k))
    torch.manual_seed(3)
    for K in (512, 256):
        calls.clear()
        x = torch.randn(300, K, device="cuda")
        l1, l2 = torch.nn.Linear(K, 101).cuda(), torch.nn.Linear(K, 65).cuda()
        with torch.no_grad():
            p, m = dd.core.projections(x, l1, l2)
            torch.testing.assert_close(p, l1(x), rtol=2e-5, atol=2e-5)
            torch.testing.assert_close(m, l2(x), rtol=2e-5, atol=2e-5)
        assert calls[0] == "projections"
        assert ("stack_rows" in calls) == (K != 512), calls


@pytest.mark.parametrize("rows,K,N", [(12800, 512, 512), (300, 1024, 512), (77, 514, 512)])
def test_linear_fn_autograd(dd, rows, K, N):
    """grad.LinearFn (the decoder's MLP Linears under autograd: forward and input gradient on ddsp_hip_linear,
    the weight gradient on ddsp_hip_linear_weight_grad, the bias gradient on torch) against an fp64 evaluation: output and all three gradients within 2x
    of torch's fp32 Linear's error.  K = 514 (the out_mlp's first block) runs torch's GEMMs inside it."""
    from ddsp_pytorch_amd.grad import LinearFn
    torch.manual_seed(rows + K)
    lin = torch.nn.Linear(K, N).cuda()
    x = torch.randn(rows, K, device="cuda", requires_grad=True)
    gy = torch.randn(rows, N, device="cuda")
    res = {}
    for name, fn in (("ours", lambda a, w, b: LinearFn.apply(a, w, b)),
                     ("f32", torch.nn.functional.linear)):
        xi = x.detach().clone().requires_grad_(True)
        w = lin.weight.detach().clone().requires_grad_(True)
        b = lin.bias.detach().clone().requires_grad_(True)
        y = fn(xi, w, b)
        y.backward(gy)
        res[name] = (y.detach(), xi.grad, w.grad, b.grad)
    xd, wd, bd = x.detach().double(), lin.weight.detach().double(), lin.bias.detach().double()
    ref = (xd @ wd.t() + bd, gy.double() @ wd, gy.double().t() @ xd, gy.double().sum(0))
    rms = lambda e: float(e.pow(2).mean().sqrt())
    for ours, f32, r in zip(res["ours"], res["f32"], ref):
        assert rms(ours.double() - r) <= 2 * rms(f32.double() - r) + 1e-12, (rms(ours.double() - r), rms(f32.double() - r))


@pytest.mark.parametrize("rows,M,N", [(12800, 512, 512), (12800, 1536, 1024), (12800, 1536, 512), (33, 512, 512),
                                      (1, 64, 128), (5001, 192, 256), (100, 166, 512), (12800, 101, 512),
                                      (12800, 65, 512), (12800, 512, 514), (37, 3, 5)])
def test_linear_weight_grad_bf16x3(dd, rows, M, N):
    """core.linear_weight_grad (ddsp_hip_linear_weight_grad: dW = dy^T x of the decoder's MLP Linears and the
    GRU's W_ih / W_hh under autograd) against an fp64 evaluation: within 2x of the f32 GEMM's (torch.mm) error,
    RMS and (3x) max; ragged row counts (33, 1, 5001: a partial last chunk and uneven row ranges) and widths that
    are no multiple of the tile (the decoder's 101 / 65-output projections, the out_mlp's 514 inputs, 3 x 5).
    Two calls are bit-identical (the row-range partials are summed in a fixed order)."""
    torch.manual_seed(rows + M + N)
    gy = torch.randn(rows, M, device="cuda")
    x = torch.randn(rows, N, device="cuda") * 1.5
    with torch.no_grad():
        dw = dd.core.linear_weight_grad(gy, x)
        dw2 = dd.core.linear_weight_grad(gy, x)
        d32 = gy.t().mm(x)
        ref = gy.double().t() @ x.double()
    assert dw.shape == (M, N)
    assert torch.equal(dw, dw2)
    rms = lambda e: float(e.pow(2).mean().sqrt())
    # + one fp32 rounding of the result: at one row the f32 GEMM is a single rounded product, the split's
    # dropped low-order terms (~2^-24 relative) then dominate the comparison
    ulp = 2.0 ** -24
    assert rms(dw.double() - ref) <= 2 * rms(d32.double() - ref) + ulp * rms(ref), (rms(dw.double() - ref), rms(d32.double() - ref))
    assert float((dw.double() - ref).abs().max()) <= 3 * float((d32.double() - ref).abs().max()) + ulp * float(ref.abs().max())


def test_linear_weight_grad_strides(dd):
    """ddsp_hip_linear_weight_grad through the C-ABI with row strides past the columns (dy_ld, x_ld, dw_ld) and
    zero rows (dW = 0): the strided result equals the packed one bit for bit; the padding of dW is untouched."""
    from ddsp_pytorch_amd import _lib
    torch.manual_seed(5)
    rows, M, N = 3000, 128, 256
    gyb = torch.randn(rows, M + 7, device="cuda")
    xb = torch.randn(rows, N + 5, device="cuda")
    dwb = torch.full((M, N + 4), 7.0, device="cuda")
    ws = dd.core._workspace(_lib.query("linear_weight_grad_workspace_size", rows, M, N), xb.device)
    _lib.call("linear_weight_grad", _lib.ptr(gyb), M + 7, _lib.ptr(xb), N + 5, _lib.ptr(dwb), N + 4, rows, M, N,
              _lib.ptr(ws), ws.numel(), _lib.stream_of(dwb))
    packed = dd.core.linear_weight_grad(gyb[:, :M].contiguous(), xb[:, :N].contiguous())
    assert torch.equal(dwb[:, :N], packed)
    assert bool((dwb[:, N:] == 7.0).all())
    _lib.call("linear_weight_grad", _lib.ptr(gyb), M + 7, _lib.ptr(xb), N + 5, _lib.ptr(dwb), N + 4, 0, M, N,
              _lib.ptr(ws), ws.numel(), _lib.stream_of(dwb))
    assert bool((dwb[:, :N] == 0).all()) and bool((dwb[:, N:] == 7.0).all())


@pytest.mark.parametrize("rows", [12800, 37])
def test_projections_fn_autograd(dd, rows):
    """grad.ProjectionsFn (decoder.py:106-117's two projections under autograd: the forward on
    ddsp_hip_projections, dx on torch, [dW1; dW2] on ddsp_hip_linear_weight_grad) against an fp64 evaluation:
    both outputs and all five gradients within 2x of torch's fp32 Linears' error (RMS)."""
    from ddsp_pytorch_amd.grad import ProjectionsFn
    torch.manual_seed(rows)
    l1, l2 = torch.nn.Linear(512, 101).cuda(), torch.nn.Linear(512, 65).cuda()
    x = torch.randn(rows, 512, device="cuda")
    g1, g2 = torch.randn(rows, 101, device="cuda"), torch.randn(rows, 65, device="cuda")
    res = {}
    for name in ("ours", "f32"):
        xi = x.clone().requires_grad_(True)
        ps = [t.detach().clone().requires_grad_(True) for t in (l1.weight, l1.bias, l2.weight, l2.bias)]
        if name == "ours":
            y = ProjectionsFn.apply(xi, *ps)
            p, m = y[..., :101], y[..., 101:166]
        else:
            p, m = torch.nn.functional.linear(xi, ps[0], ps[1]), torch.nn.functional.linear(xi, ps[2], ps[3])
        (p * g1).sum().add((m * g2).sum()).backward()
        res[name] = [p.detach(), m.detach(), xi.grad] + [t.grad for t in ps]
    xd = x.double()
    W1, B1, W2, B2 = (t.detach().double() for t in (l1.weight, l1.bias, l2.weight, l2.bias))
    G1, G2 = g1.double(), g2.double()
    ref = [xd @ W1.t() + B1, xd @ W2.t() + B2, G1 @ W1 + G2 @ W2, G1.t() @ xd, G1.sum(0), G2.t() @ xd, G2.sum(0)]
    rms = lambda e: float(e.pow(2).mean().sqrt())
    for i, (ours, f32, r) in enumerate(zip(res["ours"], res["f32"], ref)):
        assert rms(ours.double() - r) <= 2 * rms(f32.double() - r) + 1e-12, (i, rms(ours.double() - r), rms(f32.double() - r))


def test_mlp_autograd_route(dd, monkeypatch):
    """Under autograd the decoder's MLPs (mlp_forward) run each block's Linear on LinearFn — the 512-input blocks'
    forward and input gradient on the matrix-core kernel — and match torch's modules (values and every
    parameter's gradient) to fp32 accuracy; the one-feature first block stays torch's Linear."""
    from ddsp_pytorch_amd import _lib
    from ddsp_pytorch_amd.decoder import mlp, mlp_forward
    calls = []
    real = _lib.call
    monkeypatch.setattr(_lib, "call", lambda name, *a, **k: calls.append(name) or real(name, *a, **k))
    torch.manual_seed(11)
    seq = mlp(1, 512, 3).cuda()
    x = torch.randn(8, 200, 1, device="cuda")
    y = mlp_forward(seq, x)
    y.pow(2).mean().backward()
    ours = [p.grad.clone() for p in seq.parameters()]
    assert calls.count("linear") == 4, calls  # blocks 2 and 3: forward + input gradient each
    assert calls.count("linear_weight_grad") == 2, calls  # and their weight gradients
    assert calls.count("layer_norm_leaky_relu") == 3 and calls.count("layer_norm_leaky_relu_backward") == 3, calls
    seq.zero_grad()
    y_ref = seq(x)
    y_ref.pow(2).mean().backward()
    torch.testing.assert_close(y, y_ref, rtol=1e-5, atol=1e-5)
    for g, p in zip(ours, seq.parameters()):
        torch.testing.assert_close(g, p.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("rows,cols", [(12800, 512), (37, 512), (300, 1024)])
def test_ln_leaky_fn_autograd(dd, rows, cols):
    """grad.LNLeakyFn (LeakyReLU(LayerNorm(g)) under autograd: one forward kernel, one backward pass plus the
    parameter-gradient sums) against torch's modules evaluated in fp64: the output and the gradients w.r.t. g,
    gamma and beta within 2x (+ a small floor) of torch's fp32 modules' error."""
    from ddsp_pytorch_amd.grad import LNLeakyFn
    torch.manual_seed(rows + cols)
    ln = torch.nn.LayerNorm(cols).cuda()
    with torch.no_grad():
        ln.weight.copy_(1 + 0.3 * torch.randn(cols))
        ln.bias.copy_(0.2 * torch.randn(cols))
    g = torch.randn(rows, cols, device="cuda") * 1.7 + 0.4
    gy = torch.randn(rows, cols, device="cuda")
    res = {}
    for name in ("ours", "f32", "f64"):
        dt = torch.float64 if name == "f64" else torch.float32
        gi = g.detach().to(dt).requires_grad_(True)
        w = ln.weight.detach().to(dt).requires_grad_(True)
        b = ln.bias.detach().to(dt).requires_grad_(True)
        if name == "ours":
            y = LNLeakyFn.apply(gi, w, b, ln.eps, 0.01)
        else:
            y = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(gi, (cols,), w, b, ln.eps), 0.01)
        y.backward(gy.to(dt))
        res[name] = [t.double() for t in (y.detach(), gi.grad, w.grad, b.grad)]
    rms = lambda e: float(e.pow(2).mean().sqrt())
    for ours, f32, ref in zip(res["ours"], res["f32"], res["f64"]):
        assert rms(ours - ref) <= 2 * rms(f32 - ref) + 1e-7 * (1 + rms(ref)), (rms(ours - ref), rms(f32 - ref))
