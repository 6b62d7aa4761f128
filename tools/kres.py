"""Register / LDS / scratch use of the kernels in a built library (code-object metadata).

    python tools/kres.py [lib.so ...] [--match SUBSTR]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(so):
    tmp = tempfile.mkdtemp()
    try:
        local = os.path.join(tmp, os.path.basename(so))
        shutil.copy(so, local)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], capture_output=True, cwd=tmp)
        notes = ""
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" in f:
                notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(tmp, f)],
                                        capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(tmp)
    out = []
    for blk in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1)) if re.search(rf"\.{k}:\s+(\d+)", blk) else -1
        out.append((name.group(1), get("vgpr_count"), get("sgpr_count"), get("group_segment_fixed_size"),
                    get("private_segment_fixed_size")))
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    libs = [a for a in args if a.endswith(".so")] or ["ddsp_pytorch_amd/lib/libddsp_hip.so"]
    for so in libs:
        print(so)
        for name, v, s, lds, scr in kernels(so):
            if match in name:
                print(f"  vgpr {v:4d} sgpr {s:4d} lds {lds:6d} scratch {scr:4d}  {name[:100]}")


if __name__ == "__main__":
    main()
