"""Development experiment: time DDSPDecoder.forward pieces at config 2 (B=64, F=200, hidden 512)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd.decoder import DDSPDecoder

dev = "cuda"
B, F = 64, 200
torch.manual_seed(0)
m = DDSPDecoder(512, 100, 65, 48000, 512, True).to(dev).eval()
m.noise_synth.noise_mode = "device"
f0 = 50.0 * 20.0 ** torch.rand(B, F, 1, device=dev)
lo = torch.randn(B, F, 1, device=dev)


def t(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)


res = {}
with torch.no_grad():
    d = m.decoder
    hidden = torch.cat([d.f0_mlp(f0), d.loudness_mlp(lo)], -1)
    res["mlps_in_ms"] = t(lambda: torch.cat([d.f0_mlp(f0), d.loudness_mlp(lo)], -1))
    res["gru_ms"] = t(lambda: d.gru(hidden))
    g = d.gru(hidden)[0]
    res["out_mlp_ms"] = t(lambda: d.out_mlp(torch.cat([g, f0, lo], -1)))
    res["decoder_net_ms"] = t(lambda: m.decoder(f0, lo))
    res["forward_ms"] = t(lambda: m({"pitch": f0, "loudness": lo}))
m.train()
def fb():
    o = m({"pitch": f0, "loudness": lo})
    o["signal"].sum().backward()
res["forward_backward_ms"] = t(fb, reps=5)
print(json.dumps(res))
