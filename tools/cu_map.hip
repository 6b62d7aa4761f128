// Which physical CUs does a CU-masked stream (hipExtStreamCreateWithCUMask) run on?  Launches 4096
// one-wave workgroups on a stream with the given mask and counts the distinct (XCC, SE, SH, CU)
// the waves report through s_getreg (development probe for tools/exp_cumask.py).
//   hipcc --offload-arch=gfx950 -O2 tools/cu_map.hip -o tools/cu_map && tools/cu_map
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void where(unsigned* out) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  // spin a little so the grid spreads over the CUs the mask allows
  float a = threadIdx.x;
  for (int i = 0; i < 20000; ++i) a = a * 0.999f + 1e-3f;
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw + (a == 12345.f);
  }
}

static void run(const char* name, const std::vector<int>& cus) {
  unsigned words[8] = {0};
  for (int c : cus) words[c / 32] |= 1u << (c % 32);
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, 8, words) != hipSuccess) {
    printf("%s: mask rejected\n", name);
    return;
  }
  const int n = 4096;
  unsigned* d;
  hipMalloc(&d, sizeof(unsigned) * 2 * n);
  hipLaunchKernelGGL(where, dim3(n), dim3(64), 0, s, d);
  std::vector<unsigned> h(2 * n);
  hipMemcpyAsync(h.data(), d, sizeof(unsigned) * 2 * n, hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> used;
  std::set<unsigned> xccs;
  for (int i = 0; i < n; ++i) {
    const unsigned xcc = h[2 * i] & 0xf, hw = h[2 * i + 1];
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    used.insert({xcc, se, sh, cu});
    xccs.insert(xcc);
  }
  printf("%-28s mask CUs %3zu -> physical CUs used %3zu over %zu XCDs:", name, cus.size(), used.size(), xccs.size());
  std::vector<int> per(8, 0);
  for (auto& t : used) per[std::get<0>(t)]++;
  for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
  printf("\n");
  hipFree(d);
  hipStreamDestroy(s);
}

int main() {
  std::vector<int> all, first64, every4, first32, xcd8, odd;
  for (int i = 0; i < 256; ++i) {
    all.push_back(i);
    if (i < 64) first64.push_back(i);
    if (i < 32) first32.push_back(i);
    if (i % 4 == 0) every4.push_back(i);
    if (i % 32 < 8) xcd8.push_back(i);
    if (i % 8 == 0) odd.push_back(i);
  }
  run("all 256", all);
  run("indices 0..63", first64);
  run("indices 0..31", first32);
  run("every 4th index (64)", every4);
  run("every 8th index (32)", odd);
  run("i % 32 < 8 (64)", xcd8);
  std::vector<int> rest64;
  for (int i = 64; i < 256; ++i) rest64.push_back(i);
  run("indices 64..255", rest64);
  return 0;
}
