"""Weight-gradient GEMMs of the training step (dW = dy^T x): ddsp_hip_linear_weight_grad against torch.mm
(hipBLASLt) at the decoder's shapes, then bench.py's train.py step with the kernel and with torch.mm in its
place (same process, alternating).  python tools/exp_wgrad.py [kernel]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_ms(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    from ddsp_pytorch_amd import core
    dev = "cuda"
    if sys.argv[1:] == ["kernel"]:  # for PMC passes: the W_ih shape only, 10 launches
        gy = torch.randn(12800, 1536, device=dev)
        x = torch.randn(12800, 1024, device=dev)
        for _ in range(10):
            core.linear_weight_grad(gy, x)
        torch.cuda.synchronize()
        return
    for rows, M, N, what in ((12800, 512, 512, "MLP block"), (12800, 1536, 1024, "GRU W_ih"),
                             (12800, 1536, 512, "GRU W_hh")):
        gy = torch.randn(rows, M, device=dev)
        x = torch.randn(rows, N, device=dev)
        a = t_ms(lambda: core.linear_weight_grad(gy, x))
        b = t_ms(lambda: gy.t().mm(x))
        print(f"{what:10s} {rows}x{M}x{N}: kernel {a * 1e3:7.1f} us   torch.mm {b * 1e3:7.1f} us", flush=True)
    import argparse
    import bench
    args = argparse.Namespace(batch=64, frames=200, block_size=512, harmonics=100, bands=65, sample_rate=48000)
    from ddsp_pytorch_amd.synth import make_inputs
    inp = make_inputs(64, 200, 100, 65, 512, device=dev)
    real = core.linear_weight_grad
    for rnd in range(2):
        for name, fn in (("kernel", real), ("torch.mm", lambda g, x: g.t().mm(x))):
            core.linear_weight_grad = fn
            r = bench.model_train_leg(args, inp, torch.device(dev), reps=10)
            print(f"train step [{name}] {r['ms_per_step']} ms", flush=True)
    core.linear_weight_grad = real


if __name__ == "__main__":
    main()
