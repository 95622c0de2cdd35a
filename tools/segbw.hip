// Read bandwidth of narrow column segments (measurement tool, not product code): a [K, P]
// slab read as P*4/seg column segments of `seg` bytes per row, every segment walked over
// rows [r0, r1) by one workgroup (grid = segments x row ranges, ~4 workgroups per CU), so
// the CU count is the same for every segment width and only the bytes read per client row
// per visit change. 16-byte nt loads, 8 in flight per lane, no arithmetic but an xor.
//   xcd = 0: segment = block % nseg (neighbouring segments on different XCDs)
//   xcd = 1: blocks of one XCD (block % 8) take neighbouring segments
// What it answers: is the stripe fold at small P bound by how many bytes of a client row
// one visit reads (DRAM bursts / row activations), independent of the fold?
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_seg(const uint8_t* __restrict__ x, int64_t ld, int64_t K, int seg,
                                             int nseg, int nrange, int xcd, unsigned* sink) {
  const int b = blockIdx.x;
  int s, rr;
  if (xcd) {  // XCD x = b % 8 owns segments [x*nseg/8, (x+1)*nseg/8) (nseg % 8 == 0)
    const int x8 = b % 8, i = b / 8, per = nseg / 8;
    s = x8 * per + i % per;
    rr = i / per;
  } else {
    s = b % nseg;
    rr = b / nseg;
  }
  const int64_t r0 = K * rr / nrange, r1 = K * (rr + 1) / nrange;
  const int lanes_per_row = seg / 16, rows_per_it = 256 / lanes_per_row;
  const int lr = threadIdx.x / lanes_per_row, lq = threadIdx.x % lanes_per_row;
  const uint8_t* base = x + (int64_t)s * seg + lq * 16;
  unsigned acc = 0;
  int64_t r = r0 + lr;
  for (; r + 7 * rows_per_it < r1; r += 8 * rows_per_it) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (r + u * rows_per_it) * ld));
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  for (; r < r1; r += rows_per_it) acc ^= reinterpret_cast<const u32x4*>(base + r * ld)[0][1];
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int segbw(const void* x, int64_t ld, int64_t K, int64_t P_bytes, int seg, int grid, int xcd,
                     void* sink, void* stream) {
  const int nseg = (int)(P_bytes / seg);
  int nrange = grid / nseg;
  if (nrange < 1) nrange = 1;
  hipLaunchKernelGGL(k_seg, dim3(nseg * nrange), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)x, ld, K, seg,
                     nseg, nrange, xcd, (unsigned*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
