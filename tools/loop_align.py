"""Where does the fused synthesis kernel's oscillator loop sit?  Its start address mod 8 moves
the kernel by ~10 %: ≡ 4 (mod 8) measured fast, ≡ 0 slow for the shipped
instruction mix.  Prints the loop's address, size and how many of its 8-byte instructions sit
at odd dword addresses.

    python tools/loop_align.py [lib.so ...]     (default: ddsp_pytorch_amd/lib/libddsp_hip.so)
"""
import os
import tempfile
import re
import shutil
import subprocess
import sys
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernel_instructions(so, kern):
    """[(address, bytes, text)] of one kernel's instructions in the library's gfx950 code object"""
    tmp = tempfile.mkdtemp()
    local = os.path.join(tmp, os.path.basename(so))
    shutil.copy(so, local)
    subprocess.run([OBJDUMP, "--offloading", local], capture_output=True, cwd=tmp)
    dis = ""
    for f in sorted(os.listdir(tmp)):  # the code object holding the fused kernel
        if "amdgcn" in f:
            d = subprocess.run([OBJDUMP, "-d", os.path.join(tmp, f)], capture_output=True, text=True).stdout
            if re.search(kern + r".*>:", d):
                dis = d
                break
    shutil.rmtree(tmp)
    lines=dis.split("\n"); out=[]; p=False
    for l in lines:
        if re.search(kern+r".*>:",l): p=True; continue
        if p and l.strip()=="" : break
        if p: out.append(l)
    ins=[]
    for l in out:
        m=re.search(r"//\s*([0-9A-F]+):\s*((?:[0-9A-F]{8}\s*)+)",l)
        if m: ins.append((int(m.group(1),16), len(m.group(2).split())*4, l.split("//")[0].strip()))
    return ins


def kernel_sha(so, kern="synth_frame_kernelILb1ELb0ELb0ELb0EE"):
    """sha256 (16 hex) of one kernel's instruction stream (text and sizes, addresses relative to its
    entry): the key under which PMC counts of that kernel stay valid (bench.py, pmc_valu.py).  The
    literal of an s_add_u32 / s_addc_u32 (the PC-relative offset of a constant table after s_getpc_b64)
    is masked: it moves whenever other code of the library does, the kernel's work does not."""
    import hashlib
    ins = kernel_instructions(so, kern)
    if not ins:
        return None
    base = ins[0][0]
    h = hashlib.sha256()
    for addr, size, txt in ins:
        if txt.startswith(("s_add_u32", "s_addc_u32")):
            txt = re.sub(r"0x[0-9a-fA-F]+", "REL", txt)
        h.update(f"{addr - base} {size} {txt}\n".encode())
    return h.hexdigest()[:16]


def analyze(so, kern="synth_frame_kernelILb1ELb0ELb0ELb0EE"):
    """the kernel's sine loop: start address, size, 8-byte instructions at odd dword addresses"""
    ins = kernel_instructions(so, kern)
    # the hot loop: the innermost backward-branch loop holding >= 8 v_sin_f32
    best = None
    for i, (addr, size, txt) in enumerate(ins):
        m = re.match(r"s_cbranch_\w+\s+(-?\d+)", txt)
        if not m:
            continue
        target = addr + 4 + 4 * int(m.group(1)) if int(m.group(1)) < 32768 else addr + 4 + 4 * (int(m.group(1)) - 65536)
        if target >= addr:
            continue
        body = [x for x in ins if target <= x[0] <= addr]
        nsin = sum(1 for x in body if x[2].startswith("v_sin_f32"))
        # innermost: the smallest body with at least 8 sines
        if nsin >= 8 and (best is None or len(body) < len(best[2])):
            best = (nsin, target, body)
    if best is None:
        return None
    _, start, body = best
    eight = [x for x in body if x[1] == 8]
    mis = [x for x in eight if x[0] % 8 != 0]
    return {"kernel": kern, "start": start, "instrs": len(body), "bytes": sum(x[1] for x in body),
            "eight_byte": len(eight), "odd_dword": len(mis),
            "sines": sum(1 for x in body if x[2].startswith("v_sin_f32"))}


def analyze_all(so, kern="synth_frame_kernelILb1ELb0ELb0ELb0EE"):
    """every innermost sine loop of the kernel (a kernel may carry more than one copy of its loop, e.g. the
    fused forward's before- and after-the-noise-phases copies), in address order; analyze()'s fields"""
    ins = kernel_instructions(so, kern)
    loops = []
    for i, (addr, size, txt) in enumerate(ins):
        m = re.match(r"s_cbranch_\w+\s+(-?\d+)", txt)
        if not m:
            continue
        off = int(m.group(1))
        target = addr + 4 + 4 * off if off < 32768 else addr + 4 + 4 * (off - 65536)
        if target >= addr:
            continue
        body = [x for x in ins if target <= x[0] <= addr]
        if sum(1 for x in body if x[2].startswith("v_sin_f32")) >= 8:
            loops.append((target, addr, body))
    inner = [l for l in loops if not any(o is not l and l[0] <= o[0] and o[1] <= l[1] for o in loops)]
    out = []
    for start, _, body in sorted(inner, key=lambda l: l[0]):
        eight = [x for x in body if x[1] == 8]
        out.append({"kernel": kern, "start": start, "instrs": len(body), "bytes": sum(x[1] for x in body),
                    "eight_byte": len(eight), "odd_dword": len([x for x in eight if x[0] % 8 != 0]),
                    "sines": sum(1 for x in body if x[2].startswith("v_sin_f32"))})
    return out


# every shipped instantiation with a hardware-sine loop: fused forward (device noise / injected
# noise, one sample per thread for few-frame launches), the harmonic-only fused backward
SHIPPED = ("synth_frame_kernelILb1ELb0ELb0ELb0EE", "synth_frame_kernelILb0ELb0ELb0ELb0EE",
           "synth_frame_kernelILb1ELb1ELb0ELb0EE", "synth_frame_kernelILb0ELb1ELb0ELb0EE",
           "synth_frame_kernelILb1ELb0ELb1ELb0EE", "synth_frame_kernelILb0ELb0ELb1ELb0EE",
           "frame_backward_kernelILi2ELi2ELb1EE")


def report(so, kern):
    rs = analyze_all(so, kern)
    if not rs:
        print(f"{so}: no sine loop in {kern}")
    for r in rs:
        print(f"{so.split('/')[-1]} {kern}: loop @{r['start']:#x} (mod 8 = {r['start'] % 8}), {r['instrs']} "
              f"instrs, {r['bytes']} B, {r['sines']} sines, 8-byte {r['eight_byte']}, at odd dwords {r['odd_dword']}")
    return rs
if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libs = [a for a in sys.argv[1:] if a.endswith(".so")] or [
        os.path.join(root, "ddsp_pytorch_amd", "lib", "libddsp_hip.so")]
    kerns = [a for a in sys.argv[1:] if not a.endswith(".so")] or list(SHIPPED)
    for so in libs:
        for k in kerns:
            report(so, k)
