"""Spectral-loss gradient vs the reference on golden g7, with the L1 terms' sign decisions frozen:
how many bins are ties (the reference's and the kernels' magnitudes order target/reconstruction
differently), and the gradient error once the oracle takes the kernels' branch at those bins.

    python tools/exp_loss_grad.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden  # noqa: E402
from oracle import torch_ref as tr  # noqa: E402
import ddsp_pytorch_amd as dd  # noqa: E402
from ddsp_pytorch_amd import loss as L  # noqa: E402


def relerr(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    return float((a - b).norm() / b.norm())


def main():
    g = load_golden("g7_stft_loss")
    scales, ov = [int(s) for s in g["scales"]], float(g["overlap"])
    sig, rec = torch.as_tensor(g["sig"]), torch.as_tensor(g["rec"])
    ori = tr.multiscale_fft(sig, scales, ov)
    ours = [m.cpu() for m in dd.core.multiscale_fft(rec.cuda(), scales, ov)]
    ours_x = [m.cpu() for m in dd.core.multiscale_fft(sig.cuda(), scales, ov)]
    rg = rec.cuda().requires_grad_(True)
    L.spectral_loss(sig.cuda(), rg, scales, ov).backward()
    fused = rg.grad.cpu()
    rs = rec.cuda().requires_grad_(True)
    L.multiscale_spec_loss(dd.core.multiscale_fft(sig.cuda(), scales, ov), dd.core.multiscale_fft(rs, scales, ov)).backward()
    route = rs.grad.cpu()
    print("fused vs golden", relerr(fused, g["grad_rec"]), " route vs golden", relerr(route, g["grad_rec"]))
    signs = []
    for s, mx, my_ref, my_ours, mx_ours in zip(scales, ori, [torch.as_tensor(g[f"stft_{s}"]) for s in scales], ours, ours_x):
        d_ref, d_ours = my_ref - mx, my_ours - mx_ours
        l_ref = torch.log(my_ref + 1e-7) - torch.log(mx + 1e-7)
        l_ours = torch.log(my_ours + 1e-7) - torch.log(mx_ours + 1e-7)
        s_lin, s_log = torch.sign(d_ref), torch.sign(l_ref)
        tie_lin, tie_log = torch.sign(d_ours) != s_lin, torch.sign(l_ours) != s_log
        s_lin[tie_lin] = torch.sign(d_ours)[tie_lin]
        s_log[tie_log] = torch.sign(l_ours)[tie_log]
        print(f"scale {s}: bins {mx.numel()}, lin ties {int(tie_lin.sum())}, log ties {int(tie_log.sum())}, "
              f"min |d| at ties {float(d_ref.abs()[tie_lin | tie_log].min()) if (tie_lin | tie_log).any() else 0:.3g}, "
              f"min My {float(my_ref.min()):.3g}")
        signs.append((s_lin, s_log))
    rc = rec.clone().requires_grad_(True)
    lo = 0
    for (s_lin, s_log), mx, my in zip(signs, ori, tr.multiscale_fft(rc, scales, ov)):
        lo = lo + (s_lin * (my - mx)).mean() + (s_log * (torch.log(my + 1e-7) - torch.log(mx + 1e-7))).mean()
    lo.backward()
    print("fused vs frozen-sign oracle", relerr(fused, rc.grad), " route vs frozen-sign oracle", relerr(route, rc.grad))


if __name__ == "__main__":
    main()
