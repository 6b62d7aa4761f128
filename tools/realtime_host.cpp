// Realtime host for config 3: the ddsp~ Pd external's call pattern
// (realtime/ddsp_tilde/ddsp_tilde.cpp:67-98, ddsp_model.cpp:32-52) against a model exported by
// ddsp_pytorch_amd.script (TorchScript graph calling torch.ops.ddsp_hip.*).
//
// Each 1024-sample block: non-owning from_blob views of the host buffers -> device -> forward
// -> host -> memcpy, run on a worker std::thread that the next block joins first.  Reports
// per-call latency percentiles against the 1024/48000 s = 21.3 ms budget.
//
//   realtime_host <model.ts> <libddsp_hip_torch.so> [blocks]
#include <dlfcn.h>
#include <torch/script.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s model.ts libddsp_hip_torch.so [blocks]\n", argv[0]);
    return 2;
  }
  if (!dlopen(argv[2], RTLD_NOW | RTLD_GLOBAL)) {  // registers torch.ops.ddsp_hip.*
    std::fprintf(stderr, "dlopen failed: %s\n", dlerror());
    return 1;
  }
  const int blocks = argc > 3 ? std::atoi(argv[3]) : 500;
  const int N = 1024;
  torch::jit::script::Module model;
  try {  // DDSPModel::load (ddsp_model.cpp:13-30): catch and report
    model = torch::jit::load(argv[1]);
    model.to(torch::kCUDA);
    model.eval();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "load failed: %s\n", e.what());
    return 1;
  }
  torch::NoGradGuard ng;
  std::vector<float> pitch(N), loud(N), out(N);
  std::vector<double> lat;
  auto perform = [&](int blk) {  // DDSPModel::perform
    for (int i = 0; i < N; ++i) {
      pitch[i] = 220.0f * std::pow(2.0f, (float)((blk / 20) % 12) / 12.0f);
      loud[i] = -2.0f + 0.5f * std::sin(0.01f * (float)(blk * N + i));
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto p = torch::from_blob(pitch.data(), {1, N, 1}).to(torch::kCUDA);
    auto l = torch::from_blob(loud.data(), {1, N, 1}).to(torch::kCUDA);
    auto y = model.forward({p, l}).toTensor().to(torch::kCPU).contiguous();
    std::memcpy(out.data(), y.data_ptr<float>(), N * sizeof(float));
    const auto t1 = std::chrono::steady_clock::now();
    lat.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
  };
  std::thread* worker = nullptr;
  for (int b = 0; b < blocks; ++b) {  // ddsp_tilde_perform: join the previous block, spawn the next
    if (worker) {
      worker->join();
      delete worker;
    }
    worker = new std::thread(perform, b);
  }
  worker->join();
  delete worker;
  std::vector<double> s(lat.begin() + std::min<int>(20, (int)lat.size() / 2), lat.end());  // drop warm-up
  std::sort(s.begin(), s.end());
  auto pct = [&](double q) { return s[std::min<size_t>(s.size() - 1, (size_t)(q * s.size()))]; };
  double mean = 0;
  for (double v : s) mean += v;
  mean /= s.size();
  const double budget = 1000.0 * N / 48000.0;
  std::printf("{\"calls\": %zu, \"block\": %d, \"mean_ms\": %.4f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, "
              "\"max_ms\": %.4f, \"budget_ms\": %.3f, \"realtime_factor\": %.1f, \"finite\": %s}\n",
              s.size(), N, mean, pct(0.5), pct(0.99), s.back(), budget, budget / mean,
              std::isfinite(out[0]) ? "true" : "false");
  return 0;
}
