// The decoder's recurrent layer on gfx950 (the network before the path;
// decoder.py:33-68 GRUDecoder, torch.nn.GRU(2*hidden, hidden, batch_first=True)).
//
// torch.nn.GRU, gate order (r, z, n):
//   r = sigmoid(xp_r + W_hr h + b_hr),  z = sigmoid(xp_z + W_hz h + b_hz),
//   n = tanh(xp_n + r * (W_hn h + b_hn)),  h' = (1 - z) * n + z * h
// where xp = x W_ih^T + b_ih for every time step at once is one plain GEMM (the caller's
// hipBLASLt matmul).  The recurrence is what MIOpen spends ~45 us per step on at batch 64,
// hidden 512: here one launch per step, 256 workgroups (hidden slices of 4 units x batch tiles
// of 32), each holding its 12 rows of W_hh in LDS and its batch tile's h chunk in registers;
// the kernel boundary is the step's grid-wide barrier (no persistent spin, no residency
// requirement).  h_t is written straight into the output sequence, which is the next step's h.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace ddsp {
namespace {

constexpr int kHS = 4;    // hidden units per workgroup
constexpr int kBS = 32;   // batch rows per workgroup
constexpr int kKC = 16;   // k-chunks (threads per batch row)
constexpr int kNT = kBS * kKC;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// grid (H / kHS, ceil(B / kBS)); LDS: W slice [3 kHS][H] + partials [kKC][3 kHS][kBS]
__global__ void __launch_bounds__(kNT) gru_step_kernel(const float* __restrict__ xp, const float* __restrict__ w_hh,
                                                       const float* __restrict__ b_hh, const float* __restrict__ h_prev,
                                                       int64_t hp_ld, float* __restrict__ h_out, int64_t ho_ld,
                                                       int B, int H, int64_t xp_ld) {
  extern __shared__ float smem[];
  constexpr int R = 3 * kHS;
  float* W = smem;                    // [R][H]
  float* part = smem + R * H;         // [kKC][R][kBS]
  const int j0 = blockIdx.x * kHS, b0 = blockIdx.y * kBS;
  const int tid = threadIdx.x;
  const int bl = tid % kBS, c = tid / kBS;
  const int b = b0 + bl;
  const int KLr = H / kKC;  // this thread's k range [c*KLr, (c+1)*KLr), a multiple of 4
  const bool hv_ok = h_prev && b < B;
  const float* hrow = h_prev + (int64_t)(hv_ok ? b : 0) * hp_ld + c * KLr;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  for (int k0 = 0; k0 < KLr; k0 += 32) {
    // issue up to 8 16-B h loads first (the first batch overlaps the W staging below)
    float4 hv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      hv[q] = (hv_ok && k0 + 4 * q < KLr) ? *reinterpret_cast<const float4*>(hrow + k0 + 4 * q)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
    if (k0 == 0) {
      // rows: gate g of unit u is W_hh row g*H + j0 + u
      for (int i = tid; i < R * H / 4; i += kNT) {
        const int r = (4 * i) / H, k = 4 * i - r * H;
        const int g = r / kHS, u = r - g * kHS;
        *reinterpret_cast<float4*>(W + r * H + k) =
            *reinterpret_cast<const float4*>(w_hh + (int64_t)(g * H + j0 + u) * H + k);
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (k0 + 4 * q < KLr) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float4 wv = *reinterpret_cast<const float4*>(W + r * H + c * KLr + k0 + 4 * q);
          acc[r] = fmaf(wv.x, hv[q].x, fmaf(wv.y, hv[q].y, fmaf(wv.z, hv[q].z, fmaf(wv.w, hv[q].w, acc[r]))));
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) part[(c * R + r) * kBS + bl] = acc[r];
  __syncthreads();
  // gates for kHS units x kBS batch rows (128 items on 256 threads)
  if (tid < kHS * kBS) {
    const int u = tid / kBS, bb = tid - u * kBS;
    const int bi = b0 + bb, j = j0 + u;
    if (bi < B) {
      float hr = 0.f, hz = 0.f, hn = 0.f;
      for (int cc = 0; cc < kKC; ++cc) {
        hr += part[(cc * R + 0 * kHS + u) * kBS + bb];
        hz += part[(cc * R + 1 * kHS + u) * kBS + bb];
        hn += part[(cc * R + 2 * kHS + u) * kBS + bb];
      }
      const float* xr = xp + (int64_t)bi * xp_ld;
      const float r = sigmoidf_(xr[j] + (hr + b_hh[j]));
      const float z = sigmoidf_(xr[H + j] + (hz + b_hh[H + j]));
      const float n = tanhf(xr[2 * H + j] + r * (hn + b_hh[2 * H + j]));
      const float hp = h_prev ? h_prev[(int64_t)bi * hp_ld + j] : 0.0f;
      h_out[(int64_t)bi * ho_ld + j] = (1.0f - z) * n + z * hp;
    }
  }
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int ddsp_hip_gru_forward(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                         float* h_last, int64_t batch, int64_t steps, int64_t hidden, void* stream) {
  if (batch < 0 || steps < 0 || hidden < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || steps == 0) return DDSP_HIP_OK;
  if (!xp || !w_hh || !b_hh || !out) return DDSP_HIP_EINVAL;
  if (hidden % (4 * kKC) || hidden % kHS || hidden > 4096 || batch > 65535 * kBS) return DDSP_HIP_ERANGE;
  const int H = (int)hidden, B = (int)batch;
  const size_t shm = sizeof(float) * ((size_t)3 * kHS * H + (size_t)kKC * 3 * kHS * kBS);
  const dim3 grid((unsigned)(H / kHS), (unsigned)((B + kBS - 1) / kBS));
  const int64_t row = steps * hidden;  // out[b] row stride: [B, T, H]
  for (int64_t t = 0; t < steps; ++t) {
    const float* hp = t == 0 ? h0 : out + (t - 1) * hidden;
    const int64_t hp_ld = t == 0 ? hidden : row;
    hipLaunchKernelGGL(gru_step_kernel, grid, dim3(kNT), shm, reinterpret_cast<hipStream_t>(stream),
                       xp + t * 3 * hidden, w_hh, b_hh, hp, hp_ld, out + t * hidden, row, B, H, steps * 3 * hidden);
    int st = launch_status();
    if (st) return st;
  }
  if (h_last) {
    hipError_t e = hipMemcpy2DAsync(h_last, sizeof(float) * hidden, out + (steps - 1) * hidden, sizeof(float) * row,
                                    sizeof(float) * hidden, batch, hipMemcpyDeviceToDevice,
                                    reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return DDSP_HIP_ELAUNCH;
  }
  return DDSP_HIP_OK;
}

}  // extern "C"
