// Probe: VALU issue cost on gfx950 (cycles per wave64 instruction per SIMD) for the instruction
// classes of the oscillator loop, at 1-8 waves per SIMD.  Every wave runs ITER iterations of a
// body of independent instructions between two s_memtime reads; cycles per instruction per SIMD =
// median wave duration / (instructions per wave x waves per SIMD).
//   hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools/issue_probe && tools/issue_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int ITER = 4096;

#define REP8(X) X X X X X X X X

template <int MODE>
__global__ void __launch_bounds__(256) body(float* out, unsigned long long* cyc, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  const float m = 0.999f, c = 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (MODE == 0) {  // 8 independent v_fma_f32
      asm volatile(
          "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
          " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
          " v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
    } else if constexpr (MODE == 1) {  // 8 independent v_sin_f32
      asm volatile(
          "v_sin_f32 %0, %0\n v_sin_f32 %1, %1\n v_sin_f32 %2, %2\n v_sin_f32 %3, %3\n"
          " v_sin_f32 %4, %4\n v_sin_f32 %5, %5\n v_sin_f32 %6, %6\n v_sin_f32 %7, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (MODE == 2) {  // 8 v_fma + 2 v_sin interleaved (6:1.5 ~ the loop's 6:1 shape)
      asm volatile(
          "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_sin_f32 %2, %2\n"
          " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
          " v_sin_f32 %6, %6\n v_fma_f32 %7, %7, %8, %9\n v_fma_f32 %0, %0, %8, %9\n"
          " v_fma_f32 %1, %1, %8, %9\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
    } else if constexpr (MODE == 3) {  // 4 v_pk_fma_f32 (8 fp32 fmas)
      asm volatile(
          "v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n"
          " v_pk_fma_f32 %3, %3, %4, %5\n"
          : "+v"(*reinterpret_cast<double*>(&a0)), "+v"(*reinterpret_cast<double*>(&a2)),
            "+v"(*reinterpret_cast<double*>(&a4)), "+v"(*reinterpret_cast<double*>(&a6))
          : "v"(1.0), "v"(1e-3));
    } else if constexpr (MODE == 4) {  // 8 v_mul_f32
      asm volatile(
          "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n"
          " v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m));
    } else if constexpr (MODE == 6) {  // 12 fma then 2 sin grouped at the end (same mix as 5's count)
      asm volatile(
          "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
          " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
          " v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
          " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
          " v_sin_f32 %6, %6\n v_sin_f32 %7, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
    } else if constexpr (MODE == 7) {  // 24 fma + 8 sin grouped (the kernel loop's 6:... ratio x4 at 12-wide sin runs)
      asm volatile(
          REP8("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n")
          "v_sin_f32 %3, %3\n v_sin_f32 %4, %4\n v_sin_f32 %5, %5\n v_sin_f32 %6, %6\n"
          "v_sin_f32 %7, %7\n v_sin_f32 %3, %3\n v_sin_f32 %4, %4\n v_sin_f32 %5, %5\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
    } else if constexpr (MODE == 5) {  // 6 fma + 1 sin + 1 fma-accumulate, x2: the loop's exact mix
      asm volatile(
          "v_mul_f32 %0, %1, %8\n v_fma_f32 %2, %0, %9, %8\n v_add_f32 %2, %2, %9\n"
          " v_fma_f32 %3, %0, %9, %2\n v_fma_f32 %3, %0, %8, %3\n v_sin_f32 %3, %3\n"
          " v_fma_f32 %4, %3, %8, %4\n"
          " v_mul_f32 %5, %1, %9\n v_fma_f32 %6, %5, %9, %8\n v_add_f32 %6, %6, %9\n"
          " v_fma_f32 %7, %5, %9, %6\n v_fma_f32 %7, %5, %8, %7\n v_sin_f32 %7, %7\n"
          " v_fma_f32 %4, %7, %8, %4\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  out[gid] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if ((threadIdx.x & 63) == 0) cyc[gid >> 6] = t1 - t0;
}

// Do f32 MFMAs and fp32 VALU of different waves on the same SIMD overlap?  512-thread blocks, one
// per CU: waves 0-3 (one per SIMD) run KIND_LO, waves 4-7 run KIND_HI (0 = 8 v_fma, 1 = 4 independent
// v_mfma_f32_16x16x4_f32 chains, 2 = idle, 3 = 8 v_sin_f32 x ITER/4).
typedef float v4f __attribute__((ext_vector_type(4)));
template <int KIND_LO, int KIND_HI>
__global__ void __launch_bounds__(512) mix(float* out, unsigned long long* cyc, float seed) {
  const int wave = threadIdx.x >> 6;
  const int kind = wave < 4 ? KIND_LO : KIND_HI;
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  v4f c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const float m = 0.999f, c = 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (kind == 0) {
    for (int it = 0; it < ITER; ++it)
      asm volatile(
          "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
          " v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
          " v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(m), "v"(c));
  } else if (kind == 3) {
    for (int it = 0; it < ITER / 4; ++it)
      asm volatile(
          "v_sin_f32 %0, %0\n v_sin_f32 %1, %1\n v_sin_f32 %2, %2\n v_sin_f32 %3, %3\n"
          " v_sin_f32 %4, %4\n v_sin_f32 %5, %5\n v_sin_f32 %6, %6\n v_sin_f32 %7, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
  } else if (kind == 4) {  // bf16 MFMA chains (v_mfma_f32_16x16x32_bf16): the matrix core proper
    typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
    bf8 x = {(__bf16)a0, (__bf16)a1, (__bf16)a2, (__bf16)a3, (__bf16)a4, (__bf16)a5, (__bf16)a6, (__bf16)a7};
    for (int it = 0; it < ITER / 4; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, c3, 0, 0, 0);
    }
  } else if (kind == 1) {
    for (int it = 0; it < ITER / 4; ++it) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, a1, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, a3, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4, a5, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a6, a7, c3, 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  out[gid] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c0[0] + c1[1] + c2[2] + c3[3];
  if ((threadIdx.x & 63) == 0) cyc[gid >> 6] = t1 - t0;
}

template <int LO, int HI>
void run_mix(const char* name, int cus) {
  const int blocks = cus, waves = blocks * 8;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(float) * blocks * 512);
  hipMalloc(&cyc, sizeof(unsigned long long) * waves);
  hipLaunchKernelGGL((mix<LO, HI>), dim3(blocks), dim3(512), 0, 0, out, cyc, 0.5f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((mix<LO, HI>), dim3(blocks), dim3(512), 0, 0, out, cyc, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(waves);
  hipMemcpy(c.data(), cyc, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost);
  double lo = 0, hi = 0;
  for (int i = 0; i < waves; ++i) ((i % 8) < 4 ? lo : hi) += (double)c[i];
  printf("%-34s wall %.4f ms  mean cycles: waves0-3 %.0f  waves4-7 %.0f\n", name, ms, lo / (waves / 2),
         hi / (waves / 2));
  hipFree(out);
  hipFree(cyc);
}

template <int MODE>
void run(const char* name, int insts_per_iter, int cus) {
  for (int W : {1, 2, 4, 8}) {
    const int blocks = cus * W, waves = blocks * 4;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipMalloc(&cyc, sizeof(unsigned long long) * waves);
    hipLaunchKernelGGL(body<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0.5f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(body<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(waves);
    hipMemcpy(c.data(), cyc, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[waves / 2], mx = (double)c[waves - 1];
    const double insts = (double)ITER * insts_per_iter;
    // wall-clock throughput: wave-instructions per SIMD per ns
    const double per_simd_ns = insts * waves / (cus * 4.0) / (ms * 1e6);
    printf("%-28s W=%d  cyc/inst/SIMD(median wave) %.2f  (max wave %.2f)  clock %.2f GHz  "
           "wave-inst/SIMD/ns %.3f\n",
           name, W, med / (insts * W), mx / (insts * W), mx / (ms * 1e6), per_simd_ns);
    hipFree(out);
    hipFree(cyc);
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("CUs %d\n", cus);
  run<0>("v_fma_f32 x8", 8, cus);
  run<4>("v_mul_f32 x8", 8, cus);
  run<3>("v_pk_fma_f32 x4 (8 fma)", 4, cus);
  run<1>("v_sin_f32 x8", 8, cus);
  run<2>("8 fma + 2 sin (10 inst)", 10, cus);
  run<5>("osc mix 12 valu + 2 sin (14)", 14, cus);
  run<6>("12 fma + 2 sin grouped (14)", 14, cus);
  run<7>("24 fma + 8 sin grouped (32)", 32, cus);
  run_mix<3, 2>("sin x4 waves | idle", cus);
  run_mix<3, 0>("sin | fma", cus);
  run_mix<0, 2>("fma x4 waves | idle", cus);
  run_mix<1, 2>("mfma16x16x4f32 x4 waves | idle", cus);
  run_mix<0, 1>("fma | mfma (one of each per SIMD)", cus);
  run_mix<0, 0>("fma | fma", cus);
  run_mix<1, 1>("mfma | mfma", cus);
  run_mix<4, 2>("mfma bf16 x4 waves | idle", cus);
  run_mix<0, 4>("fma | mfma bf16", cus);
  run_mix<3, 4>("sin | mfma bf16", cus);
  return 0;
}
