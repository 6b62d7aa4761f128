import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import ddsp_pytorch_amd as dd
from ddsp_pytorch_amd import _lib
from ddsp_pytorch_amd.realtime import RealtimeGraph
import test_gpu_realtime as T
dev = torch.device("cuda", 0)
mean, std, seed = -3.0, 1.5, 77
real = _lib.call
mode = sys.argv[1]
def call(name, *a, **k):
    if name == "gru_forward_persistent" and mode == "steps":
        return _lib.ERANGE
    return real(name, *a, **k)
_lib.call = call
mg = T._model().to(dev); me = T._model().to(dev)
rt = RealtimeGraph(mg, T.N, mean, std, seed=seed, fused=False)
with torch.no_grad():
    for k, (pitch, loud) in enumerate(T._calls(4)):
        y = rt(pitch, loud).clone()
        ye, he, param, p = T._eager(me, pitch.to(dev), loud.to(dev), k, seed, mean, std)
        print(mode, k, float((y - ye.cpu()).abs().max()), float((mg.decoder.cache_gru - me.decoder.cache_gru).abs().max()), flush=True)
