"""Config 3 (BASELINE.json): realtime stream, batch 1, block_size 256, 64 harmonics, no reverb,
1024-sample calls — export the model to TorchScript and time it (python loop and the C++
realtime host tools/realtime_host, which mirrors the ddsp~ external's worker-thread calls).

    python tools/realtime_bench.py [--out gpurun_out/rt]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "rt"))
    ap.add_argument("--calls", type=int, default=500)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    import ddsp_pytorch_amd as dd
    from ddsp_pytorch_amd import script
    torch.manual_seed(0)
    m = dd.DDSPDecoder(512, 64, 65, 48000, 256, False).eval()  # config.yaml model, bs 256
    path = os.path.join(args.out, "ddsp_rt.ts")
    s = script.export(m.cuda(), path, realtime=True)
    pitch = torch.full((1, 1024, 1), 220.0, device="cuda")
    loud = torch.zeros(1, 1024, 1, device="cuda")
    lat = []
    with torch.no_grad():
        for i in range(args.calls):
            p = torch.full((1, 1024, 1), 220.0).cuda()
            t0 = time.perf_counter()
            y = s(p, loud).cpu()
            lat.append((time.perf_counter() - t0) * 1e3)
    lat = sorted(lat[20:])
    res = {"python_loop": {"mean_ms": statistics.mean(lat), "p50_ms": lat[len(lat) // 2],
                           "p99_ms": lat[int(0.99 * len(lat))], "budget_ms": 1024 / 48.0}}
    # the same model on a captured HIP graph (ddsp_pytorch_amd.realtime), device noise; the
    # control network either on csrc/dense.hip (fused) or as torch's kernels inside the graph
    from ddsp_pytorch_amd.realtime import RealtimeGraph
    for key, fused in (("hip_graph", True), ("hip_graph_torch_net", False)):
        rt = RealtimeGraph(m, 1024, fused=fused)
        lat = []
        with torch.no_grad():
            for i in range(args.calls):
                p = torch.full((1, 1024, 1), 220.0 * 2 ** ((i // 20) % 12 / 12))
                t0 = time.perf_counter()
                y = rt(p, loud.cpu())
                lat.append((time.perf_counter() - t0) * 1e3)
            assert torch.isfinite(y).all()
            pd, ld = p.cuda(), loud
            for _ in range(20):
                rt(pd, ld)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                rt(pd, ld)
            e1.record()
            torch.cuda.synchronize()
        gpu_ms = e0.elapsed_time(e1) / 200
        lat = sorted(lat[20:])
        res[key] = {"mean_ms": statistics.mean(lat), "p50_ms": lat[len(lat) // 2],
                    "p99_ms": lat[int(0.99 * len(lat))], "budget_ms": 1024 / 48.0,
                    "device_ms_per_replay": gpu_ms,
                    "what": "host pitch/loudness -> one hipGraph replay (control network "
                            + ("on csrc/dense.hip" if fused else "as torch kernels") + " + GRU step kernel + fused "
                            "synthesis) -> host audio"}
    host = os.path.join(ROOT, "tools", "realtime_host")
    if os.path.exists(host):
        r = subprocess.run([host, path, os.path.join(ROOT, "ddsp_pytorch_amd", "lib", "libddsp_hip_torch.so"),
                            str(args.calls)], capture_output=True, text=True, timeout=300)
        res["cpp_host"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-500:]
    res["config"] = "config 3: batch 1, block_size 256, n_harmonic 64, n_bands 65, no reverb, 1024-sample calls"
    print(json.dumps(res))


if __name__ == "__main__":
    main()
