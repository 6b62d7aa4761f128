import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ddsp_pytorch_amd as dd
from ddsp_pytorch_amd.realtime import RealtimeGraph
torch.manual_seed(0)
m = dd.DDSPDecoder(512, 64, 65, 48000, 256, False).eval().cuda()
rt = RealtimeGraph(m, 1024)
p = torch.full((1, 1024, 1), 220.0, device="cuda"); l = torch.zeros(1, 1024, 1, device="cuda")
for _ in range(100):
    rt(p, l)
torch.cuda.synchronize()
