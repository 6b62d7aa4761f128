// Shader-clock probe (development experiment): one wave spins for `cycles` shader clocks (s_memtime)
// and records the 100 MHz constant-clock ticks (s_memrealtime) that took, so out[i] = cycles / ticks
// * 100 MHz is the SCLK at that point of a stream.  Built by tools/exp_clock.py into build/.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void clock_probe_kernel(uint64_t cycles, float* out, int i) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  const uint64_t c0 = clock64();
  uint64_t c = c0;
  while (c - c0 < cycles) c = clock64();
  const uint64_t t1 = wall_clock64();
  out[i] = (float)((double)(c - c0) / (double)(t1 - t0) * 100.0);  // MHz (wall clock: 100 MHz)
}

extern "C" int clock_probe(uint64_t cycles, float* out, int i, void* stream) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, cycles, out, i);
  return (int)hipGetLastError();
}
