"""bench.py's train.py step (model_train_leg, config 2) alone, for a kernel profile:
rocprofv3 --kernel-trace --stats -- python3 tools/exp_train.py"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import bench
    from ddsp_pytorch_amd.synth import make_inputs
    args = argparse.Namespace(batch=64, frames=200, block_size=512, harmonics=100, bands=65, sample_rate=48000)
    inp = make_inputs(64, 200, 100, 65, 512, device="cuda")
    print(bench.model_train_leg(args, inp, torch.device("cuda"), reps=10))
