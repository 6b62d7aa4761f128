"""Smoke-run of the multi-GPU collectives on ONE GPU (world size 1, RCCL): exercises the
scatter / gather / broadcast calls with device tensors exactly as bench.py's N>1 legs issue
them, and checks the pipelined result against the unsharded synthesis.

    python tools/exp_pipeline.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from ddsp_pytorch_amd import core
        from ddsp_pytorch_amd.shard import broadcast_module, gather_audio, synthesize_pipelined
        from ddsp_pytorch_amd.synth import SynthPath, make_inputs
        B, F, H, NB, bs = 16, 200, 100, 65, 512
        syn = SynthPath(bs, 48000, reverb_length=48000, noise_mode="inject").to(dev)
        broadcast_module(syn.reverb)
        inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=True)
        keys = ["f0", "param", "mags", "noise"]
        ref = syn(*[inp[k] for k in keys])
        g = gather_audio(ref, B)
        tails = [tuple(inp[k].shape[1:]) for k in keys]
        out = synthesize_pipelined(syn, [inp[k] for k in keys], B, tails, chunks=4, device=dev)
        torch.cuda.synchronize()
        e1 = float((g - ref).abs().max())
        e2 = float((out - ref).abs().max())
        print({"gather_maxdiff": e1, "pipelined_maxdiff": e2, "shape": tuple(out.shape)})
        assert e1 == 0.0 and e2 < 1e-6, (e1, e2)
        print("pipeline ok")
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
