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


def analyze(so, kern="synth_frame_kernelILb1ELb0EE"):
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
    # loop: find first ds_read_b128 v[0:3], v4 ; start = previous instr
    idx=[i for i,x in enumerate(ins) if x[2].startswith("ds_read_b128 v[0:3], v4") and "offset" not in x[2]][0]-1
    start=ins[idx][0]
    end=[i for i,x in enumerate(ins[idx:]) if x[2].startswith("s_cbranch_scc0")][0]+idx
    body=ins[idx:end+1]
    eight=[x for x in body if x[1]==8]
    mis=[x for x in eight if x[0]%8!=0]
    print(f"{so.split('/')[-1]}: loop @{start:#x} (mod 8 = {start%8}), {len(body)} instrs, {sum(x[1] for x in body)} B, 8-byte {len(eight)}, misaligned {len(mis)}")
if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for so in sys.argv[1:] or [os.path.join(root, "ddsp_pytorch_amd", "lib", "libddsp_hip.so")]:
        analyze(so)
