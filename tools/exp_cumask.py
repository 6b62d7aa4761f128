"""Can the reverb of one batch run beside the synthesis of the next on disjoint CU sets?

Two HIP streams with complementary CU masks (hipExtStreamCreateWithCUMask): the VALU-bound
fused synthesis kernel on one set, the memory-bound UPOLS reverb on the other, independent inputs.
Prints, per reverb CU share, each group alone on its mask and both together (device time per
pair of launches), against the plain one-stream step (development experiment).

    python tools/exp_cumask.py [reverb_cus ...]
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")


def masked_stream(cus):
    """stream restricted to the CU indices in `cus` (256-bit mask, 8 words)"""
    words = [0] * 8
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * 8)(*words)
    s = ctypes.c_void_p()
    err = HIP.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), arr)
    assert err == 0, err
    return torch.cuda.ExternalStream(s.value)


def main():
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    B, F, H, NB, bs, N = 64, 200, 100, 65, 512, 60
    inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
    syn = SynthPath(bs, 48000, reverb_length=48000).to(dev)
    L = syn.reverb.length
    spec = syn.reverb._spectrum(F * bs)
    sig = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)

    def synth():
        core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)

    def reverb():
        core.reverb_apply(sig, spec, L)

    def timed(pairs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for fn, st in pairs:
            with torch.cuda.stream(st):
                for _ in range(N):
                    fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e6

    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        synth()
        reverb()
    main_s = torch.cuda.current_stream()
    base = timed([(lambda: (synth(), reverb()), main_s)])
    def pipelined(sa, sb):
        """step i: synth(i) on sa, reverb(i) on sb after it (record_stream keeps the signal's memory
        from being reused on sa before the reverb has read it)"""
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(N):
            with torch.cuda.stream(sa):
                x = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
                e = torch.cuda.Event()
                e.record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(e)
                x.record_stream(sb)
                core.reverb_apply(x, spec, L)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e6

    mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
    if mode == "plain":  # one extra unmasked stream
        print(f"one stream, all {n_cu} CUs: step {base:6.1f} us", flush=True)
        sb = torch.cuda.Stream(dev)
        for _ in range(2):
            tp = pipelined(main_s, sb)
        print(f"pipelined, two unmasked streams: {tp:6.1f} us per step", flush=True)
        return
    # "<k>:<layout>": the reverb stream on k CUs, the synthesis stream on the rest (only these two
    # streams are created in the process: hardware queues are few, and streams sharing one share
    # its CU mask)
    k, layout = mode.split(":")
    k = int(k)
    if layout == "spread":  # every (n_cu // k)-th CU index
        rcus = [i for i in range(n_cu) if i % (n_cu // k) == 0][:k]
    elif layout == "xcd":  # k/8 CUs of each 32-CU group
        per = k // 8
        rcus = [x * (n_cu // 8) + i for x in range(8) for i in range(per)]
    else:
        rcus = list(range(k))
    scus = [i for i in range(n_cu) if i not in set(rcus)]
    sr, ss = masked_stream(rcus), masked_stream(scus)
    for _ in range(2):
        ts = timed([(synth, ss)])
        tr = timed([(reverb, sr)])
        tb = timed([(synth, ss), (reverb, sr)])
        tp = pipelined(ss, sr)
    print(f"reverb on {k:3d} CUs ({layout}): synth alone {ts:6.1f}, reverb alone {tr:6.1f}, "
          f"both {tb:6.1f} us per pair, pipelined step {tp:6.1f} (one-stream step {base:6.1f})", flush=True)


if __name__ == "__main__":
    main()
