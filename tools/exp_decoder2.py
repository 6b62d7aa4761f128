"""Development experiment: where DDSPDecoder.forward's time goes at config 2 (B=64, F=200, hidden 512) —
host-timed pieces (after warmup) and, under rocprofv3 --kernel-trace, the kernels of each piece.

    python tools/exp_decoder2.py [piece ...]   pieces: net gru mlps outmlp outmlp_gemm net_gemm dsyn proj synth fwd
(outmlp: the out_mlp through decoder.mlp_forward, each block one core.mlp_block launch; *_gemm: the same
with core.mlp_block disabled, i.e. the GEMM + fused LayerNorm/LeakyReLU route)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.decoder import DDSPDecoder, decoder_projections, decoder_synthesize, mlp_forward  # noqa: E402

dev = "cuda"
B, F, bs, sr = 64, 200, 512, 48000
torch.manual_seed(0)
m = DDSPDecoder(512, 100, 65, sr, bs, True).to(dev).eval()
m.noise_synth.noise_mode = "device"
f0 = 50.0 * 20.0 ** torch.rand(B, F, 1, device=dev)
lo = torch.randn(B, F, 1, device=dev)


def t(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    host0 = time.perf_counter()
    fn()
    host = time.perf_counter() - host0
    torch.cuda.synchronize()
    return {"ms": round((time.perf_counter() - t0 - host) / reps * 1e3, 4), "host_ms_one_call": round(host * 1e3, 4)}


pieces = sys.argv[1:] or ["net", "gru", "mlps", "outmlp", "outmlp_gemm", "net_gemm", "dsyn", "proj", "synth", "fwd"]
_block = core.mlp_block


def gemm_route(fn):
    def run():
        core.mlp_block = lambda *a, **k: None
        try:
            return fn()
        finally:
            core.mlp_block = _block
    return run

res = {}
with torch.no_grad():
    d = m.decoder
    hidden_in = torch.cat([d.f0_mlp(f0), d.loudness_mlp(lo)], -1)
    hidden = m.decoder(f0, lo)
    param, mags = decoder_projections(m, hidden)
    for p in pieces:
        if p == "net":
            res[p] = t(lambda: m.decoder(f0, lo))
        elif p == "gru":
            res[p] = t(lambda: core.gru(hidden_in, d.gru, None))
        elif p == "mlps":
            res[p] = t(lambda: d.out_mlp(torch.cat([d.f0_mlp(f0), d.loudness_mlp(lo), f0, lo], -1)[..., :514]))
        elif p == "outmlp":
            g = core.gru(hidden_in, d.gru, None)[0]
            res[p] = t(lambda: mlp_forward(d.out_mlp, g, extras=(f0, lo)))
        elif p == "outmlp_gemm":
            g = core.gru(hidden_in, d.gru, None)[0]
            res[p] = t(gemm_route(lambda: mlp_forward(d.out_mlp, g, extras=(f0, lo))))
        elif p == "net_gemm":
            res[p] = t(gemm_route(lambda: m.decoder(f0, lo)))
        elif p == "dsyn":
            res[p] = t(lambda: decoder_synthesize(m, hidden, f0))
        elif p == "proj":
            res[p] = t(lambda: decoder_projections(m, hidden))
        elif p == "synth":
            res[p] = t(lambda: m.reverb(core.synth_frames(f0, param, mags, bs, sr, parts=True, controls=True)[0]))
        elif p == "fwd":
            res[p] = t(lambda: m({"pitch": f0, "loudness": lo}))
print(json.dumps(res), flush=True)
