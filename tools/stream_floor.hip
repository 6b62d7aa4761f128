// The streaming floor of the reverb's byte volumes on this chip (measurement only, never shipped):
// plain float4 streaming kernels moving exactly the bytes each UPOLS phase moves at config 2, so the
// reverb group's 58 us can be read against what those bytes cost at the chip's practical rate.
//   fwd-like  read 26.2 MB (the pair rows), write 52.4 MB (zero-padded spectra)
//   mac-like  read 52.4 MB, write 52.4 MB
//   inv-like  read 52.4 MB, write 26.2 MB
//   the three back to back (two dependent boundaries), and the 26.2 + 26.2 MB copy (x in, y out: the
//   floor of any single-pass reverb)
//     hipcc --offload-arch=gfx950 -O3 tools/stream_floor.hip -o build/stream_floor && build/stream_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

// every thread: R float4 reads and W float4 writes per item, items grid-strided
template <int R, int W>
__global__ void __launch_bounds__(256) stream_kernel(const float4* __restrict__ in, float4* __restrict__ out,
                                                     long items) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += (long)gridDim.x * blockDim.x) {
    float4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = in[i + (long)r * items];
    float4 s = v[0];
#pragma unroll
    for (int r = 1; r < R; ++r) s.x += v[r].x;
#pragma unroll
    for (int w = 0; w < W; ++w) out[i + (long)w * items] = w == 0 ? s : make_float4(s.y, s.z, s.w, s.x);
  }
}

template <int R, int W>
float time_it(const float4* in, float4* out, long items, int blocks, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((stream_kernel<R, W>), dim3(blocks), dim3(256), 0, 0, in, out, items);
  CHECK(hipEventRecord(a));
  for (int k = 0; k < reps; ++k) hipLaunchKernelGGL((stream_kernel<R, W>), dim3(blocks), dim3(256), 0, 0, in, out, items);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const long samples = 64L * 102400;          // config 2: 6.55 M samples = 26.2 MB
  const long q = samples / 4;                 // float4 items per 26.2 MB
  float4 *in, *out;
  CHECK(hipMalloc(&in, 2 * q * sizeof(float4)));
  CHECK(hipMalloc(&out, 2 * q * sizeof(float4)));
  CHECK(hipMemset(in, 0, 2 * q * sizeof(float4)));
  const int reps = 50;
  for (int blocks : {2048, 4096, 8192, 16384}) {
    const float f = time_it<1, 2>(in, out, q, blocks, reps);
    const float m = time_it<2, 2>(in, out, q, blocks, reps);
    const float v = time_it<2, 1>(in, out, q, blocks, reps);
    const float c = time_it<1, 1>(in, out, q, blocks, reps);
    // the three phases back to back, as the reverb issues them
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    for (int k = 0; k < reps; ++k) {
      hipLaunchKernelGGL((stream_kernel<1, 2>), dim3(blocks), dim3(256), 0, 0, in, out, q);
      hipLaunchKernelGGL((stream_kernel<2, 2>), dim3(blocks), dim3(256), 0, 0, out, in, q);
      hipLaunchKernelGGL((stream_kernel<2, 1>), dim3(blocks), dim3(256), 0, 0, in, out, q);
    }
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double mb = 26.2144;
    std::printf("{\"blocks\": %d, \"fwd_like_us\": %.2f, \"fwd_tbs\": %.2f, \"mac_like_us\": %.2f, \"mac_tbs\": %.2f, "
                "\"inv_like_us\": %.2f, \"inv_tbs\": %.2f, \"three_back_to_back_us\": %.2f, \"copy_x_to_y_us\": %.2f, "
                "\"copy_tbs\": %.2f}\n",
                blocks, f, 3 * mb / f, m, 4 * mb / m, v, 3 * mb / v,
                ms * 1000.f / reps, c, 2 * mb / c);
  }
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
