// Probe: can a launch carry its plan image in the kernel arguments, and what does
// that cost next to the pinned H2D copy the pytree path uses today?
//   hipcc --offload-arch=gfx950 -O3 tools/probe_kernarg.hip -o /tmp/probe_kernarg && /tmp/probe_kernarg
// Prints one JSON line per image size: whether the launch succeeded and read back the
// right words, and us per launch (GPU-side, events over 2000 iterations) for
//   inline : kernel with the image as a by-value argument
//   copy   : hipMemcpyAsync pinned -> device + the same kernel reading the device copy
//   bare   : the kernel with an 8-byte argument (launch floor)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("{\"error\": \"%s\", \"at\": %d}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

template <int N>
struct Img {
  int64_t w[N];
};

// every lane reads words of the image through a pointer into the argument (no copy)
template <int N>
__global__ void k_inline(Img<N> img, int64_t* out) {
  const int64_t* p = img.w;
  int64_t s = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) s += p[i] * (i + 1);
  atomicAdd((unsigned long long*)out, (unsigned long long)s);
}

__global__ void k_ptr(const int64_t* __restrict__ p, int n, int64_t* out) {
  int64_t s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i] * (i + 1);
  atomicAdd((unsigned long long*)out, (unsigned long long)s);
}

__global__ void k_bare(int64_t* out) {
  if (threadIdx.x == 0) out[1] += 1;
}

template <int N>
int run(int iters) {
  Img<N>* h;
  CK(hipHostMalloc((void**)&h, sizeof(Img<N>), hipHostMallocDefault));
  int64_t expect = 0;
  for (int i = 0; i < N; ++i) {
    h->w[i] = 3 * i + 7;
    expect += h->w[i] * (i + 1);
  }
  int64_t *d_img, *d_out;
  CK(hipMalloc(&d_img, sizeof(Img<N>)));
  CK(hipMalloc(&d_out, 16));
  CK(hipMemset(d_out, 0, 16));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipLaunchKernelGGL(k_inline<N>, dim3(1), dim3(256), 0, s, *h, d_out);
  hipError_t le = hipGetLastError();
  int64_t got[2] = {0, 0};
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(got, d_out, 16, hipMemcpyDeviceToHost));
  const bool ok = le == hipSuccess && got[0] == expect;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float t_inline = -1, t_copy = -1, t_bare = -1;
  if (ok) {
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_inline<N>, dim3(1), dim3(256), 0, s, *h, d_out);
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_inline<N>, dim3(1), dim3(256), 0, s, *h, d_out);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t_inline, e0, e1));
  }
  for (int i = 0; i < 50; ++i) {
    CK(hipMemcpyAsync(d_img, h, sizeof(Img<N>), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ptr, dim3(1), dim3(256), 0, s, d_img, N, d_out);
  }
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) {
    CK(hipMemcpyAsync(d_img, h, sizeof(Img<N>), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ptr, dim3(1), dim3(256), 0, s, d_img, N, d_out);
  }
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&t_copy, e0, e1));
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_bare, dim3(1), dim3(64), 0, s, d_out);
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_bare, dim3(1), dim3(64), 0, s, d_out);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&t_bare, e0, e1));
  printf("{\"bytes\": %zu, \"launch_ok\": %s, \"launch_error\": \"%s\", \"read_ok\": %s, "
         "\"inline_us\": %.3f, \"copy_plus_kernel_us\": %.3f, \"bare_us\": %.3f}\n",
         sizeof(Img<N>), le == hipSuccess ? "true" : "false", hipGetErrorString(le), ok ? "true" : "false",
         t_inline * 1e3 / iters, t_copy * 1e3 / iters, t_bare * 1e3 / iters);
  fflush(stdout);
  CK(hipStreamDestroy(s));
  CK(hipFree(d_img));
  CK(hipFree(d_out));
  CK(hipHostFree(h));
  return 0;
}

int main() {
  const int iters = 2000;
  if (run<64>(iters)) return 1;     // 512 B
  if (run<512>(iters)) return 1;    // 4 KiB
  if (run<1024>(iters)) return 1;   // 8 KiB
  if (run<2048>(iters)) return 1;   // 16 KiB
  if (run<3500>(iters)) return 1;   // 28 KiB
  return 0;
}
