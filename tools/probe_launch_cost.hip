// Probe: host cost of a launch vs the size of its by-value kernel argument struct, and the
// launch-to-completion latency of one launch on an idle stream (the synchronous tree_mean's
// critical path starts with such a launch).
//   hipcc --offload-arch=gfx950 -O3 tools/probe_launch_cost.hip -o /tmp/plc && /tmp/plc
// One JSON line per argument size (int64 words): host_us per launch (1000 launches issued
// back to back, then one sync), idle_us = host time of launch + hipStreamSynchronize on an
// idle stream (median of 200).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

template <int N>
struct Img {
  int64_t w[N];
};

template <int N>
__global__ void k_img(Img<N> img, int64_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = img.w[N - 1];
}

using clk = std::chrono::steady_clock;

template <int N>
void run(hipStream_t s, int64_t* out) {
  Img<N> img;
  for (int i = 0; i < N; ++i) img.w[i] = i;
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_img<N>, dim3(256), dim3(256), 0, s, img, out);
  hipStreamSynchronize(s);
  auto t0 = clk::now();
  for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(k_img<N>, dim3(256), dim3(256), 0, s, img, out);
  auto t1 = clk::now();
  hipStreamSynchronize(s);
  const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000;
  std::vector<double> idle;
  for (int i = 0; i < 200; ++i) {
    auto a = clk::now();
    hipLaunchKernelGGL(k_img<N>, dim3(256), dim3(256), 0, s, img, out);
    hipStreamSynchronize(s);
    idle.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
  }
  std::sort(idle.begin(), idle.end());
  printf("{\"words\": %d, \"bytes\": %d, \"host_us\": %.3f, \"idle_launch_sync_us\": %.3f}\n", N, N * 8, host_us,
         idle[idle.size() / 2]);
}

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  int64_t* out;
  hipMalloc(&out, 64);
  run<8>(s, out);
  run<256>(s, out);
  run<512>(s, out);
  run<1024>(s, out);
  run<2048>(s, out);
  run<3584>(s, out);
  run<8>(s, out);
  hipFree(out);
  return 0;
}
