"""Train-step timing of the synthesis path (bench.py's train_step leg alone), for library A/B through
DDSP_HIP_LIB.  (development experiment)

    python tools/exp_train_time.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402


def main():
    saved, sys.argv = sys.argv, [sys.argv[0]]
    args = bench.parse()
    sys.argv = saved
    dev = torch.device("cuda", 0)
    inp = make_inputs(args.batch, args.frames, args.harmonics, args.bands, args.block_size, seed=0, device=dev,
                      with_noise=False)
    for _ in range(2):
        r = bench.train_leg(args, inp, dev)
        print(f"train step {r['ms_per_step']:.4f} ms  events {r.get('event_ms')}", flush=True)


if __name__ == "__main__":
    main()
