// Probe: accuracy and throughput of sine evaluation variants on gfx950 for the oscillator bank.
//   A: sin_reduced (Cody-Waite by pi + odd minimax polynomial)         [shipped]
//   B: Cody-Waite by 2pi, then hardware v_sin_f32 on revolutions
// Accuracy vs fp64 sin of the same fp32 argument; throughput in a register-resident loop.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../ddsp_pytorch_amd/csrc/common.h"

using namespace ddsp;

__device__ __forceinline__ float sin_hw(float x) {
  const float kInv2Pi = 0.159154943091895335769f;
  const float k2PiA = 6.28318548202514648438f;
  const float k2PiB = -1.74845553146951715e-07f;
  float t = fmaf(x, kInv2Pi, kMagic);
  float n = t - kMagic;
  float r = fmaf(-n, k2PiA, x);
  r = fmaf(-n, k2PiB, r);
  return __builtin_amdgcn_sinf(r * kInv2Pi);
}

__global__ void eval(const float* x, float* a, float* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { a[i] = sin_reduced(x[i]); b[i] = sin_hw(x[i]); }
}

template <int V>
__global__ void bench(float* out, float w0, int H) {
  float w = w0 + 1e-3f * threadIdx.x + 1e-5f * blockIdx.x;
  float acc = 0.f;
  for (int k = 1; k <= H; ++k) {
    float x = w * (float)k;
    acc = fmaf(V == 0 ? sin_reduced(x) : sin_hw(x), 0.01f, acc);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int n = 1 << 22;
  std::vector<float> hx(n);
  for (int i = 0; i < n; ++i) {
    double u = (double)i / n;
    hx[i] = (float)((i & 1 ? -1 : 1) * (i % 3 == 0 ? u * 1.2e7 : (i % 3 == 1 ? u * 3e4 : u * 8.0)));
  }
  float *dx, *da, *db;
  hipMalloc(&dx, n * 4); hipMalloc(&da, n * 4); hipMalloc(&db, n * 4);
  hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(eval, dim3(n / 256), dim3(256), 0, 0, dx, da, db, n);
  std::vector<float> ha(n), hb(n);
  hipMemcpy(ha.data(), da, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), db, n * 4, hipMemcpyDeviceToHost);
  double ma = 0, mb = 0, sa = 0, sb = 0;
  for (int i = 0; i < n; ++i) {
    double r = std::sin((double)hx[i]);
    double ea = std::fabs(ha[i] - r), eb = std::fabs(hb[i] - r);
    ma = std::max(ma, ea); mb = std::max(mb, eb); sa += ea * ea; sb += eb * eb;
  }
  printf("accuracy: poly max %.3e rms %.3e | hw max %.3e rms %.3e\n", ma, std::sqrt(sa / n), mb, std::sqrt(sb / n));
  float* dout; hipMalloc(&dout, 65536 * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(25600), dim3(256), 0, 0, dout, 0.05f, 1000);
      else hipLaunchKernelGGL(bench<1>, dim3(25600), dim3(256), 0, 0, dout, 0.05f, 1000);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2) printf("variant %s: %.3f ms, %.1f G sin/s\n", v ? "hw" : "poly", ms, 25600.0 * 256 * 1000 / ms / 1e6);
    }
  }
  return 0;
}
