// Dependent v_add_f32 chain latency on one wave (the stripe fold's per-client floor):
// cycles per add for a serial chain, for two interleaved chains, and for the fold's
// pattern (one ds_read_b128 feeding 4 serial adds). s_memtime cycles, one wave, idle GPU.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/valu_latency.hip -o /tmp/valu_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int N = 4096;

__global__ void chain1(const float* b, float* out, long long* cyc) {
  float x = b[threadIdx.x], y = b[threadIdx.x + 64];
  __syncthreads();
  long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) x = __fadd_rn(x, y);
  long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void chain2(const float* b, float* out, long long* cyc) {
  float x = b[threadIdx.x], x2 = b[threadIdx.x + 1], y = b[threadIdx.x + 64];
  __syncthreads();
  long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) {
    x = __fadd_rn(x, y);
    x2 = __fadd_rn(x2, y);
  }
  long long t1 = clock64();
  out[threadIdx.x] = x + x2;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__global__ void fold_lds(const float* b, float* out, long long* cyc) {
  __shared__ u32x4 tile[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) {
    u32x4 v;
    for (int e = 0; e < 4; ++e) v[e] = __float_as_uint(b[(i * 4 + e) & 127]);
    tile[i] = v;
  }
  __syncthreads();
  float acc = 0.f;
  long long t0 = clock64();
  for (int rep = 0; rep < N / 256; ++rep) {
#pragma unroll
    for (int g = 0; g < 64; g += 8) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = tile[threadIdx.x * 64 + ((g + u) ^ (threadIdx.x & 15))];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        for (int e = 0; e < 4; ++e) acc = __fadd_rn(acc, __uint_as_float(v[u][e]));
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float *b, *out;
  long long* cyc;
  hipMalloc(&b, 4096);
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 64);
  hipMemset(b, 0, 4096);
  long long h;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(chain1, dim3(1), dim3(64), 0, 0, b, out, cyc);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"chain1_cycles_per_add\": %.2f, ", (double)h / N);
    hipLaunchKernelGGL(chain2, dim3(1), dim3(64), 0, 0, b, out, cyc);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("\"chain2_cycles_per_pair\": %.2f, ", (double)h / N);
    hipLaunchKernelGGL(fold_lds, dim3(1), dim3(64), 0, 0, b, out, cyc);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("\"fold_lds_cycles_per_add\": %.2f}\n", (double)h / N);
  }
  return 0;
}
