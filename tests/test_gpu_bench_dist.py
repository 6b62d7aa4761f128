"""bench.py's distributed entry point on the GPU: launched by
torch.distributed.run, even at one rank, bench.py takes its N>1 branch — RCCL process group, barrier
and max-over-ranks timing, the `gathered` leg (torch.distributed.gather) and the `scatter_gather` leg
(chunked scatter of the controls, synthesis, gather of the audio, IR broadcast) — so every line of
that branch runs on RCCL before the driver's 8-GPU node.  Injected noise makes the legs
deterministic: their outputs are checked against the one-process step inside bench.py."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_under_torch_distributed_run_world1():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "3", "--warmup", "2", "--settle", "0", "--noise", "inject", "--no-cpu-baseline",
           "--no-train-leg", "--no-loss-leg", "--no-model-train-leg", "--no-decoder-leg", "--no-op-leg",
           "--no-pipelined-leg", "--no-uncached-leg"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    g, sg = line["gathered"], line["scatter_gather"]
    assert "RCCL" in g["collective"] and "RCCL" in sg["collective"]
    assert g["check_vs_local_step"]["equal"], g
    assert sg["check_vs_one_process_step"]["max_abs_diff"] == 0.0, sg
    assert line["cpu_baseline"] is None  # --no-cpu-baseline
