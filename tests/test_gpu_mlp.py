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
    """decoder.py:106-117 as one GEMM over both layers' parameters stacked per call (core.projections)
    against an fp64 host matmul."""
    torch.manual_seed(2)
    l1, l2 = torch.nn.Linear(K, n1).cuda(), torch.nn.Linear(K, n2).cuda()
    x = torch.randn(rows, K, device="cuda")
    with torch.no_grad():
        a, b = dd.core.projections(x, l1, l2)
    assert a.shape == (rows, n1) and b.shape == (rows, n2)
    assert a.stride(0) == b.stride(0) and b.data_ptr() == a.data_ptr() + 4 * n1 and a.stride(0) % 64 == 0
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
