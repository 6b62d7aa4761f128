"""Probe / variant builds (measurement only, never shipped): a copy of one csrc/<stem>.hip with
literal edits is compiled into build/ab_<name>.so (linked with the in-tree objects).  The synth_frame
probes edit one phase out, so PMC passes (tools/pmc_variants.sh through DDSP_HIP_LIB) give each
phase's dynamic VALU count by difference — their outputs are wrong by design; the gru_* variants
change the step kernel's tile shape (outputs equal up to summation order).

    python tools/probe_build.py [name ...]      (default: every probe below)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ddsp_pytorch_amd", "csrc")

# name -> [(literal, replacement)]; every literal must occur in the source
STEM = {"gru8": "gru", "gru16h2": "gru", "gru16h8": "gru", "gru32": "gru", "gruclk": "gru"}
# gruclk: per-step realtime stamps (100 MHz) of workgroup 0 of the persistent GRU, written after the
# sync words (tools/exp_gru_clock.py reads them): 0 step start, 1 poll passed, 2 partials in LDS,
# 3 gates stored, 4 counter added
_STAMP = "if (blockIdx.x == 0 && tid == 0) abort_word[64 + 8 * t + {k}] = (uint32_t)__builtin_amdgcn_s_memrealtime();"
PROBES = {
    "gruclk": [("constexpr int kPSyncWords = 19 * kPCounterStride;", "constexpr int kPSyncWords = 19 * kPCounterStride + 32 + 8 * 8192;"),
               ("    // the epilogue's input projection for this step: issued before the wait\n",
                "    " + _STAMP.format(k=0) + "\n"),
               ("      if (*s_abort) return;  // gru_rescue_kernel recomputes the outputs\n    }\n",
                "      if (*s_abort) return;\n    }\n    " + _STAMP.format(k=1) + "\n"),
               ("make_float4(acc[j][i], acc[j][i + 1], acc[j][i + 2], acc[j][i + 3]);\n    }\n    __syncthreads();\n",
                "make_float4(acc[j][i], acc[j][i + 1], acc[j][i + 2], acc[j][i + 3]);\n    }\n    __syncthreads();\n    " + _STAMP.format(k=2) + "\n"),
               ("      ehp = hnew;\n    }\n", "      ehp = hnew;\n    }\n    " + _STAMP.format(k=3) + "\n"),
               ("    __syncthreads();\n    float acc[6][kPI];\n", "    __syncthreads();\n    " + _STAMP.format(k=5) + "\n    float acc[6][kPI];\n"),
               ("      if (tid == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n",
                "      if (tid == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n      " + _STAMP.format(k=4) + "\n")],
    # wgclk: per-workgroup start / end realtime stamps (100 MHz) and hardware ids of the fused synthesis
    # kernel, in a device table read back by ddsp_probe_wg_stamps (tools/exp_wg_tail.py): the grid's
    # 3.125 rounds of resident workgroups and how busy the chip is in the last one
    "wgclk": [("  extern __shared__ float4 smem4[];\n  __shared__ double red[32];\n  float acc[4], nz[4];\n",
               "  extern __shared__ float4 smem4[];\n  __shared__ double red[32];\n  float acc[4], nz[4];\n"
               "  const uint64_t probe_t0 = __builtin_amdgcn_s_memrealtime();\n"),
              ("make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121\n}\n",
               "make_float4(acc[0] + nz[0], acc[1] + nz[1], acc[2] + nz[2], acc[3] + nz[3]);  // decoder.py:121\n"
               "  if (threadIdx.x == 0) {\n"
               "    uint32_t hw, xcc;\n"
               "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
               "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
               "    const uint64_t i = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;\n"
               "    if (i < kProbeWG) {\n"
               "      g_probe_stamps[3 * i] = probe_t0;\n"
               "      g_probe_stamps[3 * i + 1] = __builtin_amdgcn_s_memrealtime();\n"
               "      g_probe_stamps[3 * i + 2] = ((uint64_t)xcc << 32) | hw;\n"
               "    }\n"
               "  }\n}\n"),
              ("template <bool RNG, bool SPLIT, bool CTRL, bool PREFIX>\n__global__",
               "constexpr uint64_t kProbeWG = 65536;\n__device__ uint64_t g_probe_stamps[3 * kProbeWG];\n"
               "template <bool RNG, bool SPLIT, bool CTRL, bool PREFIX>\n__global__"),
              ("int ddsp_hip_frame_phase_prefix(",
               "int ddsp_probe_occupancy(int threads, int64_t shm) {\n"
               "  int n = -1;\n"
               "  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, synth_frame_kernel<true, false, false, false>, threads,\n"
               "                                               (size_t)shm);\n"
               "  return n;\n}\n\n"
               "int ddsp_probe_wg_stamps(uint64_t* host, int64_t n) {\n"
               "  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_probe_stamps), sizeof(uint64_t) * 3 * n, 0,\n"
               "                                  hipMemcpyDeviceToHost);\n}\n\n"
               "int ddsp_hip_frame_phase_prefix(")],
    # wgclk with the kernel's SGPRs capped at 80 (does the 14-workgroups-per-CU residency move?)
    "wgclksg": None,
    "gru8": [("gru_forward_launch<16, 32>", "gru_forward_launch<8, 64>"),
             ("gru_backward_steps<16, 32>", "gru_backward_steps<8, 64>")],
    "gru32": [("gru_forward_launch<16, 32>", "gru_forward_launch<32, 16>"),
              ("gru_backward_steps<16, 32>", "gru_backward_steps<32, 16>")],
    "gru16h2": [("constexpr int kHS = 4;", "constexpr int kHS = 2;")],
    "gru16h8": [("constexpr int kHS = 4;", "constexpr int kHS = 8;")],
    "noprefix": [("for (int g = tid; g < f; g += NT)", "for (int g = tid; g < 0; g += NT)")],
    "noscale": [("const float sv = scale_fn(i >= H && i < H + NB ? raw + bias : raw);",
                 "const float sv = raw;")],
    "norng": [("const Philox4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), off0, off1, k0, k1);",
               "Philox4 r; r.v[0] = (uint32_t)q; r.v[1] = off0; r.v[2] = k0; r.v[3] = (uint32_t)t;")],
    "noirfft": [("if (n == 128 && NT >= 128) {", "if (n == 128 && NT >= 128) { if (tid <= 64) ir[tid] = A[tid]; } else if (false) {")],
    "notail": [("if (bs - tail_start == 64 && bs - 127 >= lo_end) {\n    if (tid < 64) {",
                "if (bs - tail_start == 64 && bs - 127 >= lo_end) {\n    if (tid < 0) {")],
    "nohtaps": [("h[j] = ir_at_half(ir, ct, n, bs, j);", "h[j] = ir[j & 63];")],
    "noosc": [("osc_bank4(coef, H4, w, acc);", "acc[0] = w[0]; acc[1] = w[1]; acc[2] = w[2]; acc[3] = w[3];")],
    "nofir": [("float4 y = fir4(h, x, j0, lo_end, bs, bs);", "float4 y = make_float4(x[j0], x[j0 + 1], h[j0], h[j0 + 3]);")],
}


PROBES["wgclksg"] = PROBES["wgclk"] + [
    ("__global__ void __launch_bounds__(256) synth_frame_kernel(",
     "__global__ void __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80))) synth_frame_kernel(")]


def build(name):
    stem = STEM.get(name, "synth_frame")
    src = open(os.path.join(CSRC, stem + ".hip")).read()
    for a, b in PROBES[name]:
        if a not in src:
            raise SystemExit(f"probe {name}: pattern not found: {a[:60]}")
        src = src.replace(a, b)
    d = os.path.join(ROOT, "build", f"probe_{name}")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, stem + ".hip")
    open(path, "w").write(src)
    inc = os.path.join(ROOT, "ddsp_pytorch_amd", "csrc")
    obj = os.path.join(ROOT, "build", f"ab_{name}_{stem}.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-ffp-contract=off", f"-I{ROOT}/include", f"-I{ROOT}/build", f"-I{inc}",
                    "-Wno-unused-result", "-fno-slp-vectorize", "-c", path, "-o", obj], check=True)
    objs = [os.path.join(ROOT, "build", f) for f in sorted(os.listdir(os.path.join(ROOT, "build")))
            if f.endswith(".o") and not f.startswith("ab_") and f != stem + ".o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o",
                    os.path.join(ROOT, "build", f"ab_{name}.so")] + objs + [obj], check=True)
    print("built", f"build/ab_{name}.so", flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(PROBES):
        build(n)
