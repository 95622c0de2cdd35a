// Read-bandwidth ceilings on MI355X (measurement tool, not product code).
//   mode 0: contiguous stream: lane i reads 16 B at (i + j*nthreads)*16, grid-stride
//   mode 1: row walk like the fold: lane owns 8 units of 16 B in a column window and
//           walks K rows (stride ld bytes), 4 rows in flight, balanced grid
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ x, int64_t n16, unsigned* sink) {
  unsigned acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  for (; i < n16; i += stride) { u32x4 v = x[i]; acc ^= v[0] ^ v[3]; }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int AUX>
__global__ __launch_bounds__(256) void k_rows(const uint8_t* __restrict__ x, int64_t ld, int64_t K,
                                               int64_t nunits, int64_t S, unsigned* sink) {
  unsigned acc = 0;
  const int64_t u0 = (int64_t)blockIdx.x * S, u1 = (u0 + S < nunits) ? u0 + S : nunits;
  for (int64_t g = u0; g < u1; g += 256 * 8) {
    uint32_t off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t u = g + j * 256 + threadIdx.x;
      if (u >= u1) u = u1 - 1;
      off[j] = (uint32_t)(u * 16);
    }
    for (int64_t k = 0; k < K; k += 4) {
      u32x4 v[4][8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (k + r) * ld), (short)0, (int)(nunits * 16), 0x00020000);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[r][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[j], 0, AUX);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= v[r][j][0] ^ v[r][j][1] ^ v[r][j][2] ^ v[r][j][3];
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int readbw(int mode, const void* x, int64_t ld_bytes, int64_t K, int64_t row_bytes,
                      int64_t grid, unsigned* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0) {
    hipLaunchKernelGGL(k_stream, dim3((unsigned)grid), dim3(256), 0, s, (const u32x4*)x,
                       (K * ld_bytes) / 16, sink);
  } else {
    const int64_t nunits = row_bytes / 16;
    const int64_t S = ((nunits + grid - 1) / grid + 63) / 64 * 64;
    const int64_t nblk = (nunits + S - 1) / S;
    hipLaunchKernelGGL(k_rows<2>, dim3((unsigned)nblk), dim3(256), 0, s, (const uint8_t*)x, ld_bytes,
                       K, nunits, S, sink);
  }
  return (int)hipGetLastError();
}

// The row walk with another cache policy on the loads (aux of buffer_load on gfx950:
// bit 0 sc0, bit 1 nt, bit 4 sc1); 2 (nt) is what the fold uses.
extern "C" int readbw_policy(int aux, const void* x, int64_t ld_bytes, int64_t K, int64_t row_bytes,
                             int64_t grid, unsigned* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t nunits = row_bytes / 16;
  const int64_t S = ((nunits + grid - 1) / grid + 63) / 64 * 64;
  const dim3 g((unsigned)((nunits + S - 1) / S));
  const uint8_t* p = (const uint8_t*)x;
#define FJ_AUX(A) case A: hipLaunchKernelGGL(k_rows<A>, g, dim3(256), 0, s, p, ld_bytes, K, nunits, S, sink); break;
  switch (aux) {
    FJ_AUX(0) FJ_AUX(1) FJ_AUX(2) FJ_AUX(3) FJ_AUX(16) FJ_AUX(17) FJ_AUX(18) FJ_AUX(19)
    default: return -1;
  }
#undef FJ_AUX
  return (int)hipGetLastError();
}
