// Probe: accuracy and throughput of sine evaluation variants on gfx950 for the oscillator bank.
//   0: reduce_signed + amp-folded odd minimax polynomial (amp_sin_acc)      [12 VALU]
//   1: Cody-Waite by 2pi in radians, scale to revolutions, hardware v_sin_f32
//   3, 4: 2 of 4 / 3 of 4 samples on variant 2, the rest on variant 0 (does the transcendental
//      unit issue beside the VALU?); 5: bare v_sin + fma (transcendental rate)
//   2: reduction directly in revolutions (two-term 1/(2pi) by fma), hardware v_sin_f32 [shipped:
//      common.h reduce_rev + sin_rev]
// Accuracy vs fp64 sin of the same fp32 argument (|x| < kFastArgLimit); throughput in a
// register-resident loop shaped like the fused kernel's (4 samples per thread, amplitude per k).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -Iinclude -Ibuild \
//     tools/sin_probe.hip -o tools/sin_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../ddsp_pytorch_amd/csrc/common.h"

using namespace ddsp;

__device__ __forceinline__ float sin_hw1(float x) {
  const float k2PiA = 6.28318548202514648438f;
  const float k2PiB = -1.74845553146951715e-07f;
  float t = fmaf(x, kInv2Pi, kMagic);
  float n = t - kMagic;
  float r = fmaf(-n, k2PiA, x);
  r = fmaf(-n, k2PiB, r);
  return __builtin_amdgcn_sinf(r * kInv2Pi);
}

// revolutions: y = x/(2pi) - n with the product formed exactly inside the fma
__device__ __forceinline__ float rev2(float x) {
  const float t = fmaf(x, kInv2Pi, kMagic);
  const float n = t - kMagic;
  float y = fmaf(x, kInv2Pi, -n);
  return fmaf(x, kInv2PiLo, y);
}
__device__ __forceinline__ float sin_hw2(float x) { return __builtin_amdgcn_sinf(rev2(x)); }

__global__ void eval(const float* x, float* a, float* b, float* c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    a[i] = sin_poly(x[i]);
    b[i] = sin_hw1(x[i]);
    c[i] = sin_hw2(x[i]);
  }
}

template <int V>
__global__ void bench(float* out, const float* amp, float w0, int H) {
  float w[4], acc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    w[s] = w0 + 1e-3f * (threadIdx.x * 4 + s) + 1e-5f * blockIdx.x;
    acc[s] = 0.0f;
  }
  for (int k = 0; k < H; ++k) {
    const float* c = amp + 8 * (k & 127);  // uniform loads, like the LDS coefficient broadcast
    const float a = c[0];
    const float kk = (float)(k + 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float x = w[s] * kk;
      if (V == 0) acc[s] = amp_sin_acc(reduce_signed(x), a, c[1], c[2], c[3], c[4], acc[s]);
      else if (V == 1) acc[s] = fmaf(sin_hw1(x), a, acc[s]);
      else if (V == 2) acc[s] = fmaf(sin_hw2(x), a, acc[s]);
      else if (V == 3) {  // mixed: two samples on the hardware sine, two on the polynomial
        if (s < 2) acc[s] = fmaf(sin_hw2(x), a, acc[s]);
        else acc[s] = amp_sin_acc(reduce_signed(x), a, c[1], c[2], c[3], c[4], acc[s]);
      } else if (V == 4) {  // mixed 3:1
        if (s < 3) acc[s] = fmaf(sin_hw2(x), a, acc[s]);
        else acc[s] = amp_sin_acc(reduce_signed(x), a, c[1], c[2], c[3], c[4], acc[s]);
      } else {  // transcendental rate: v_sin + one fma
        acc[s] = fmaf(__builtin_amdgcn_sinf(x), a, acc[s]);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
  const int n = 1 << 22;
  std::vector<float> hx(n);
  for (int i = 0; i < n; ++i) {
    double u = (double)i / n;
    hx[i] = (float)((i & 1 ? -1 : 1) * (i % 3 == 0 ? u * 7.9e6 : (i % 3 == 1 ? u * 3e4 : u * 8.0)));
  }
  float *dx, *da, *db, *dc;
  hipMalloc(&dx, n * 4); hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dc, n * 4);
  hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(eval, dim3(n / 256), dim3(256), 0, 0, dx, da, db, dc, n);
  std::vector<float> ha(n), hb(n), hc(n);
  hipMemcpy(ha.data(), da, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), db, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hc.data(), dc, n * 4, hipMemcpyDeviceToHost);
  const std::vector<float>* vs[3] = {&ha, &hb, &hc};
  for (int v = 0; v < 3; ++v) {
    double m = 0, s = 0, bias = 0;
    for (int i = 0; i < n; ++i) {
      double e = (*vs[v])[i] - std::sin((double)hx[i]);
      m = std::max(m, std::fabs(e)); s += e * e; bias += e;
    }
    printf("accuracy variant %d: max %.3e rms %.3e mean %.3e\n", v, m, std::sqrt(s / n), bias / n);
  }
  float* dout; hipMalloc(&dout, 25600 * 256 * 4);
  float* damp; hipMalloc(&damp, 128 * 8 * 4);
  std::vector<float> hamp(128 * 8, 0.0f);
  for (int k = 0; k < 128; ++k) {
    const float a = 0.01f;
    const float cs[5] = {a, a * kS3, a * kS5, a * kS7, a * kS9};
    for (int j = 0; j < 5; ++j) hamp[8 * k + j] = cs[j];
  }
  hipMemcpy(damp, hamp.data(), 128 * 8 * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int H = 400, blocks = 25600;
  for (int v = 0; v < 6; ++v) {
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      else if (v == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      else if (v == 2) hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      else if (v == 3) hipLaunchKernelGGL(bench<3>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      else if (v == 4) hipLaunchKernelGGL(bench<4>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      else hipLaunchKernelGGL(bench<5>, dim3(blocks), dim3(128), 0, 0, dout, damp, 0.05f, H);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep == 3)
        printf("throughput variant %d: %.3f ms, %.1f G sin/s\n", v, ms, (double)blocks * 128 * 4 * H / ms / 1e6);
    }
  }
  return 0;
}
