// fjcomp.hip — MI355X (gfx950) kernels for FedJAX's compression aggregators
// (fedjax/aggregators/compression.py, walsh_hadamard.py). C ABI: include/fjcomp.h.
//
// A compression round in the reference is, per client and per leaf, a chain of jitted
// XLA calls: amin/amax (or std), a jax.random.uniform draw, the elementwise quantizer,
// and for the rotated variants a Walsh-Hadamard transform on each side; tree_mean then
// folds the quantized deltas. Here the round is a few launches over (client, leaf) tables:
//
//   k_row_stats / k_stats_combine  one HBM pass per row: min/max/|max| and f64 sums,
//                                  combined per row in a fixed order (deterministic),
//                                  then turned into the quantizer's per-row constants;
//   k_quant_fold                   threefry draw + quantizer + tree_mean fold in one
//                                  pass: a lane owns the element PAIR (i, i + h) that one
//                                  threefry2x32 call produces (JAX's counter layout), walks
//                                  the clients in order and keeps the running sum in a
//                                  register. Threefry costs ~31 VALU ops per element (of
//                                  ~58), so this kernel is VALU-bound, not HBM-bound
//                                  (DESIGN.md §3c);
//   k_rademacher                   the rotation signs, one bit per element, packed with
//                                  wave ballots; computed once per key and read by both the
//                                  forward and the inverse rotation;
//   k_wht                          Walsh-Hadamard in passes over LDS tiles of 8192 f32: pass 0
//                                  does the 13 low butterfly bits on contiguous tiles, later
//                                  passes 8 bits each on 256 strided rows x 32 contiguous
//                                  floats (128-byte segments: coalesced); butterflies run
//                                  radix-16 in registers (4 stages per LDS round trip); the
//                                  rotation prologue (zero pad, sign) and epilogue (sign,
//                                  / sqrt(d), truncate) are fused into the first/last pass.
//
// Arithmetic follows the reference's float32 op sequence. Division: a quotient by a
// per-row constant b is RN_f32(a * RN_f64(1/b)); the f64 error (< 2^-52 relative) is
// below the distance from a/b to any f32 rounding midpoint (>= 2^-49 relative for
// f32 a, b), so the result equals the correctly rounded f32 quotient. Per-element
// quotients use f64 division rounded once (double rounding is innocuous for p = 53 >=
// 2*24 + 2). Compiled with -ffp-contract=off: no multiply-add contraction anywhere.
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "fjcomp.h"

extern thread_local char fjagg_g_err[512];

static_assert(sizeof(fjcomp_stats) == 48, "fjcomp_stats layout");
static_assert(sizeof(fjcomp_qparams) == 24, "fjcomp_qparams layout");
static_assert(sizeof(fjcomp_row) == 16, "fjcomp_row layout");
static_assert(sizeof(fjcomp_sign_job) == 24, "fjcomp_sign_job layout");
static_assert(sizeof(fjcomp_wht_job) == 72, "fjcomp_wht_job layout");

namespace {

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(fjagg_g_err, sizeof(fjagg_g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FJAGG_EHIP, "%s: %s", what, hipGetErrorString(e));
  return FJAGG_OK;
}

// ------------------------------------------------------------------ threefry2x32-20
__host__ __device__ inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define FJ_TF_ROUND(r) \
  x0 += x1;            \
  x1 = rotl32(x1, r);  \
  x1 ^= x0;
#define FJ_TF_ROT0 FJ_TF_ROUND(13) FJ_TF_ROUND(15) FJ_TF_ROUND(26) FJ_TF_ROUND(6)
#define FJ_TF_ROT1 FJ_TF_ROUND(17) FJ_TF_ROUND(29) FJ_TF_ROUND(16) FJ_TF_ROUND(24)

// Threefry-2x32 with 20 rounds and JAX's key schedule (jax/_src/prng.py); k2 = k0 ^ k1 ^ C.
__host__ __device__ inline void threefry_k(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t& x0, uint32_t& x1) {
  x0 += k0;
  x1 += k1;
  FJ_TF_ROT0 x0 += k1; x1 += k2 + 1u;
  FJ_TF_ROT1 x0 += k2; x1 += k0 + 2u;
  FJ_TF_ROT0 x0 += k0; x1 += k1 + 3u;
  FJ_TF_ROT1 x0 += k1; x1 += k2 + 4u;
  FJ_TF_ROT0 x0 += k2; x1 += k0 + 5u;
}
// Two independent blocks through the same key, round by round (instruction-level parallelism).
#define FJ_TF_ROUND2(r) \
  a0 += a1; b0 += b1;   \
  a1 = rotl32(a1, r);   \
  b1 = rotl32(b1, r);   \
  a1 ^= a0; b1 ^= b0;
#define FJ_TF_ROT0_2 FJ_TF_ROUND2(13) FJ_TF_ROUND2(15) FJ_TF_ROUND2(26) FJ_TF_ROUND2(6)
#define FJ_TF_ROT1_2 FJ_TF_ROUND2(17) FJ_TF_ROUND2(29) FJ_TF_ROUND2(16) FJ_TF_ROUND2(24)
__device__ inline void threefry2_k(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t& a0, uint32_t& a1, uint32_t& b0,
                                   uint32_t& b1) {
  a0 += k0; a1 += k1; b0 += k0; b1 += k1;
  FJ_TF_ROT0_2 a0 += k1; a1 += k2 + 1u; b0 += k1; b1 += k2 + 1u;
  FJ_TF_ROT1_2 a0 += k2; a1 += k0 + 2u; b0 += k2; b1 += k0 + 2u;
  FJ_TF_ROT0_2 a0 += k0; a1 += k1 + 3u; b0 += k0; b1 += k1 + 3u;
  FJ_TF_ROT1_2 a0 += k1; a1 += k2 + 4u; b0 += k1; b1 += k2 + 4u;
  FJ_TF_ROT0_2 a0 += k2; a1 += k0 + 5u; b0 += k2; b1 += k0 + 5u;
}
__host__ __device__ inline void threefry(uint32_t k0, uint32_t k1, uint32_t& x0, uint32_t& x1) {
  threefry_k(k0, k1, k0 ^ k1 ^ 0x1BD11BDAu, x0, x1);
}

// jax.random.uniform's bits -> [0, 1): bitcast((b >> 9) | 1.0f) - 1
// ((b >> 9) | 0x3f800000) is one v_alignbit: the low word of (0x7f : b) >> 9.
__device__ inline float bits_to_unit(uint32_t b) {
  return __uint_as_float(__builtin_amdgcn_alignbit(0x7fu, b, 9u)) - 1.0f;
}

// ------------------------------------------------------------------ f32 helpers
// Branch-free (the branchy forms compiled to exec-mask regions inside the per-element loop).
// jnp.nan_to_num: NaN -> 0, +-inf -> +-FLT_MAX; med3 of a non-NaN x is exact (keeps -0).
__device__ inline float nan_to_num(float x) { return x != x ? 0.0f : __builtin_amdgcn_fmed3f(x, -FLT_MAX, FLT_MAX); }
// numpy's maximum(0, minimum(nan_to_num(a), 1)) (first argument wins ties, so -0 -> +0):
// NaN and everything <= 0 give +0, +inf gives 1.
// maxnum(NaN, 0) = 0, so NaN -> +0 as well; -0 may stay -0, which no caller can tell from
// +0 (every use compares u > a or scales a by a positive constant and takes floor/ceil of
// a value that then indexes level 0).
__device__ inline float clamp01_nan(float a) { return fminf(fmaxf(a, 0.0f), 1.0f); }
__device__ inline float xla_sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : x); }
// correctly rounded a / b given r = RN_f64(1 / b) (see the header comment)
__device__ inline float div_by(float a, double r) { return (float)((double)a * r); }
__device__ inline float div_rn(float a, float b) { return (float)((double)a / (double)b); }
__device__ inline double nan_min(double a, double b) { return (a != a) ? a : ((b != b) ? b : (b < a ? b : a)); }
__device__ inline double nan_max(double a, double b) { return (a != a) ? a : ((b != b) ? b : (b > a ? b : a)); }

// Segment of block b in a running-sum table prefix[nseg + 1] (skips empty segments).
// Wave-parallel 64-ary search: each round lane i tests pivot lo + i*step with ONE vector
// load and a ballot, so up to 4096 segments cost two dependent loads instead of log2(nseg)
// scalar ones (that latency was a large share of the short-lived blocks of k_row_stats,
// k_wht and k_rademacher). Every lane of the wave must call it with the same b (kernel
// entry, before any divergence); the result is wave-uniform.
__device__ inline int64_t find_segment(const int64_t* __restrict__ prefix, int64_t nseg, int64_t b) {
  const int64_t lane = threadIdx.x & 63;
  int64_t lo = 0, hi = nseg;  // prefix[lo] <= b < prefix[hi]
  while (hi - lo > 1) {
    const int64_t step = (hi - lo + 63) >> 6;
    const int64_t idx = lo + lane * step;
    // lane 0 always passes; prefix[] is nondecreasing, so the passing lanes are a prefix
    const uint64_t m = __ballot(idx < hi && prefix[idx] <= b);
    lo += (int64_t)(63 - __builtin_clzll(m)) * step;
    hi = lo + step < hi ? lo + step : hi;
  }
  return lo;
}

// ------------------------------------------------------------------ random bits
__global__ __launch_bounds__(256) void k_random_bits(uint32_t k0, uint32_t k1, int64_t n, uint32_t* __restrict__ out,
                                                      float* __restrict__ outf) {
  const int64_t h = (n + 1) >> 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= h) return;
  uint32_t x0 = (uint32_t)i, x1 = (uint32_t)(i + h < n ? i + h : 0);
  threefry(k0, k1, x0, x1);
  if (out) {
    out[i] = x0;
    if (i + h < n) out[i + h] = x1;
  } else {
    outf[i] = fmaxf(0.0f, bits_to_unit(x0));
    if (i + h < n) outf[i + h] = fmaxf(0.0f, bits_to_unit(x1));
  }
}

// ------------------------------------------------------------------ rademacher signs
// Sign of element g is bit 31 of its uniform draw's bits (uniform < 0.5 <=> +1).
// A workgroup owns `block_pairs` (256 x rounds, at most FJCOMP_SIGN_BLOCK_PAIRS) consecutive
// pairs of one job and each wave a run of rounds x 64 of them: the segment search, the job record and the key schedule
// are paid once per 8 threefry calls of a lane, and the wave's 2 x 16 sign words are
// stored once, coalesced, instead of 4 single-lane stores per 64 pairs.
constexpr int kSignRounds = FJCOMP_SIGN_BLOCK_PAIRS / 256;
static_assert(kSignRounds % 2 == 0 && 2 * kSignRounds <= 64, "a wave's sign words fit its lanes");
__global__ __launch_bounds__(256) void k_rademacher(const fjcomp_sign_job* __restrict__ jobs,
                                                     const int64_t* __restrict__ prefix, int64_t J, int rounds) {
  const int64_t b = blockIdx.x;
  const int64_t j = find_segment(prefix, J, b);
  const fjcomp_sign_job jb = jobs[j];
  const int64_t d = jb.d, h = (d + 1) >> 1;
  const uint32_t k0 = jb.key[0], k1 = jb.key[1], k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  const int lane = threadIdx.x & 63;
  if (d < 64) {  // one or two words, written by the first lane of the job's first wave
    if (b != prefix[j] || threadIdx.x >= 64) return;
    uint32_t x0 = (uint32_t)lane, x1 = (uint32_t)(lane + h < d ? lane + h : 0);
    threefry_k(k0, k1, k2, x0, x1);
    const uint64_t m0 = __ballot(lane < h && (x0 >> 31));
    const uint64_t m1 = __ballot(lane < h && lane + h < d && (x1 >> 31));
    if (lane == 0) {
      const uint64_t lo = m0 & ((1ull << h) - 1), hi = m1 & ((1ull << (d - h)) - 1);
      const uint64_t all = lo | (hi << h);  // d <= 63 bits
      jb.words[0] = (uint32_t)all;
      if (d > 32) jb.words[1] = (uint32_t)(all >> 32);
    }
    return;
  }
  const int w = threadIdx.x >> 6;
  if (h & 31) {
    // halves that are not whole words (lengths other than a multiple of 64, none of them from
    // the aggregators, which pad to powers of two): element-major, a lane per element, so a
    // ballot is two whole words. Twice the threefry calls; the block covers 2 x its pairs.
    const int64_t e0 = (b - prefix[j]) * (512 * (int64_t)rounds) + (int64_t)w * 128 * rounds;
    for (int r = 0; r < 2 * rounds; ++r) {
      const int64_t g0 = e0 + 64 * r;
      if (g0 >= d) return;  // wave-uniform
      const int64_t g = g0 + lane, i = g < h ? g : g - h;
      uint32_t x0 = (uint32_t)i, x1 = (uint32_t)(i + h < d ? i + h : 0);
      threefry_k(k0, k1, k2, x0, x1);
      const uint64_t m = __ballot(g < d && ((g < h ? x0 : x1) >> 31));
      if (lane == 0) {
        jb.words[g0 >> 5] = (uint32_t)m;
        if (g0 + 32 < d) jb.words[(g0 >> 5) + 1] = (uint32_t)(m >> 32);
      }
    }
    return;
  }
  // h is a multiple of 32, so words never straddle the two halves. Lane 0 parks
  // each round's two 64-bit ballots in LDS; at the end lane t of the wave stores word t of
  // both runs (one coalesced store each instead of single-lane stores per round).
  __shared__ uint64_t masks[4][2][kSignRounds];
  const int64_t p0 = (b - prefix[j]) * (256 * rounds) + (int64_t)w * 64 * rounds;
  const bool lead = lane == 0;
  if (p0 < h) {  // wave-uniform
    if (!(d & 1) && p0 + 64 * rounds <= h && h + (int64_t)h <= 0xffffffffll) {
      // common case (every DRIVE / rotation job: d even, so i + h < d <=> i < h; the whole
      // run is inside the job; 32-bit counters): no masks, 32-bit index arithmetic
      const uint32_t hh = (uint32_t)h;
      uint32_t ctr = (uint32_t)p0 + (uint32_t)lane;
#pragma unroll 1
      for (int r = 0; r < rounds; ++r, ctr += 64u) {
        uint32_t a0 = ctr, a1 = ctr + hh;
        // opaque to the optimizer: otherwise loop strength reduction rewrites the first
        // rounds as sums of induction variables (7 extra adds per pair, measured in the ISA)
        asm("" : "+v"(a0), "+v"(a1));
        threefry_k(k0, k1, k2, a0, a1);
        const uint64_t m0 = __ballot((int)a0 < 0), m1 = __ballot((int)a1 < 0);
        if (lead) {
          masks[w][0][r] = m0;
          masks[w][1][r] = m1;
        }
      }
    } else {  // pairs past h are masked out of the ballots; their words are not stored
#pragma unroll 1
      for (int r = 0; r < rounds; ++r) {
        if (p0 + r * 64 >= h) break;  // wave-uniform
        const int64_t i = p0 + r * 64 + lane;
        uint32_t a0 = (uint32_t)i, a1 = (uint32_t)(i + h < d ? i + h : 0);
        threefry_k(k0, k1, k2, a0, a1);
        const uint64_t m0 = __ballot(i < h && (a0 >> 31)), m1 = __ballot(i < h && i + h < d && (a1 >> 31));
        if (lead) {
          masks[w][0][r] = m0;
          masks[w][1][r] = m1;
        }
      }
    }
  }
  __syncthreads();
  if (p0 < h && lane < 2 * rounds && p0 + 32 * lane < h) {
    const uint32_t* m = reinterpret_cast<const uint32_t*>(masks[w][0]);
    const uint32_t* n = reinterpret_cast<const uint32_t*>(masks[w][1]);
    jb.words[(p0 >> 5) + lane] = m[lane];
    jb.words[((p0 + h) >> 5) + lane] = n[lane];
  }
}

// ------------------------------------------------------------------ row statistics
constexpr int kStatsThreads = 256;
constexpr int kStatsChunk = FJCOMP_STATS_CHUNK;

struct Partial {
  double mn, mx, amx, s1, s2, sa;
};
static_assert(sizeof(Partial) == 48, "Partial");

__device__ inline void merge(Partial& a, const Partial& b) {
  a.mn = nan_min(a.mn, b.mn);
  a.mx = nan_max(a.mx, b.mx);
  a.amx = nan_max(a.amx, b.amx);
  a.s1 += b.s1;
  a.s2 += b.s2;
  a.sa += b.sa;
}

__device__ inline Partial shfl_xor(const Partial& p, int m) {
  Partial q;
  q.mn = __shfl_xor(p.mn, m);
  q.mx = __shfl_xor(p.mx, m);
  q.amx = __shfl_xor(p.amx, m);
  q.s1 = __shfl_xor(p.s1, m);
  q.s2 = __shfl_xor(p.s2, m);
  q.sa = __shfl_xor(p.sa, m);
  return q;
}

// Per-lane accumulator: min / max / |max| in f32 (exact; NaN tracked by a flag, as the
// f64 nan_min / nan_max fold it into), sums in f64. v*v of an f32 v is exact in f64, so
// fma(v, v, s) is the rounding of s + v*v.
struct LaneStats {
  float mn = INFINITY, mx = -INFINITY, amx = -INFINITY;
  double s1 = 0.0, s2 = 0.0, sa = 0.0;
  bool nan = false;
  __device__ inline void add(float x) {
    nan |= x != x;
    mn = fminf(mn, x);
    mx = fmaxf(mx, x);
    amx = fmaxf(amx, fabsf(x));
    const double v = (double)x;
    s1 += v;
    s2 = __fma_rn(v, v, s2);
    sa += fabs(v);  // |double(x)| == double(|x|): the abs is a free source modifier
  }
  __device__ inline Partial partial() const {
    const double qn = __longlong_as_double(0x7ff8000000000000ll);
    return Partial{nan ? qn : (double)mn, nan ? qn : (double)mx, nan ? qn : (double)amx, s1, s2, sa};
  }
};

// Min / max / |max| of a workgroup's values (the order-independent part of LaneStats) and,
// with `sums`, the f64 sums of squares and of magnitudes (DRIVE's sumsq / sumabs), stored
// as a Partial (sum 0) by thread 0 after wave butterflies and an LDS combine. Every
// thread of the workgroup must call store().
struct MinMax {
  float mn = INFINITY, mx = -INFINITY, amx = -INFINITY;
  double s2 = 0.0, sa = 0.0;
  bool nan = false;
  __device__ inline void add(float x, bool sums) {
    nan |= x != x;
    mn = fminf(mn, x);
    mx = fmaxf(mx, x);
    amx = fmaxf(amx, fabsf(x));
    if (sums) {
      const double v = (double)x;
      s2 = __fma_rn(v, v, s2);
      sa += fabs(v);
    }
  }
  __device__ inline void store(Partial* out, bool sums) const {
    // f32 wave reduction (min / max are exact in any order; NaN as one wave vote), then
    // the waves through LDS: a few dozen cross-lane ops per tile
    float a = mn, b = mx, c = amx;
    double q = s2, r = sa;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      a = fminf(a, __shfl_xor(a, m));
      b = fmaxf(b, __shfl_xor(b, m));
      c = fmaxf(c, __shfl_xor(c, m));
    }
    if (sums) {
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        q += __shfl_xor(q, m);
        r += __shfl_xor(r, m);
      }
    }
    const bool any_nan = __any(nan);
    __shared__ float sp[16][4];  // waves of the widest caller (k_wht: 512 threads)
    __shared__ double sq[16][2];
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      const int w = threadIdx.x >> 6;
      sp[w][0] = a;
      sp[w][1] = b;
      sp[w][2] = c;
      sp[w][3] = any_nan ? 1.0f : 0.0f;
      sq[w][0] = q;
      sq[w][1] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float n = sp[0][3];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
        a = fminf(a, sp[w][0]);
        b = fmaxf(b, sp[w][1]);
        c = fmaxf(c, sp[w][2]);
        n = fmaxf(n, sp[w][3]);
        q += sq[w][0];
        r += sq[w][1];
      }
      const double qn = __longlong_as_double(0x7ff8000000000000ll);
      *out = Partial{n != 0.0f ? qn : (double)a, n != 0.0f ? qn : (double)b, n != 0.0f ? qn : (double)c, 0.0,
                     sums ? q : 0.0, sums ? r : 0.0};
    }
  }
};

// One workgroup per 16 Ki-element chunk of a row: a scalar head up to the first 16-byte
// boundary, float4 loads eight deep per lane, a scalar tail; then the fixed-order wave
// butterfly and a per-workgroup combine in wave order (deterministic).
__global__ __launch_bounds__(kStatsThreads) void k_row_stats(const fjcomp_row* __restrict__ rows,
                                                              const int64_t* __restrict__ prefix, int64_t R,
                                                              Partial* __restrict__ part) {
  const int64_t b = blockIdx.x;
  const int64_t r = find_segment(prefix, R, b);
  const fjcomp_row row = rows[r];
  const int64_t c0 = (b - prefix[r]) * kStatsChunk;
  const int64_t c1 = min(row.n, c0 + kStatsChunk);
  const float* __restrict__ x = row.ptr + c0;
  const int n = (int)(c1 - c0);
  const bool vec = ((uintptr_t)x & 3) == 0;  // else everything goes through the scalar tail
  const int head = vec ? min(n, (int)(((16 - ((uintptr_t)x & 15)) & 15) >> 2)) : 0;
  const int nv = vec ? (n - head) >> 2 : 0;
  LaneStats st;
  if ((int)threadIdx.x < head) st.add(x[threadIdx.x]);
  const float4* __restrict__ xv = reinterpret_cast<const float4*>(x + head);
  int i = threadIdx.x;
  for (; i + 7 * kStatsThreads < nv; i += 8 * kStatsThreads) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xv[i + u * kStatsThreads];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      st.add(v[u].x);
      st.add(v[u].y);
      st.add(v[u].z);
      st.add(v[u].w);
    }
  }
  for (; i < nv; i += kStatsThreads) {
    const float4 v = xv[i];
    st.add(v.x);
    st.add(v.y);
    st.add(v.z);
    st.add(v.w);
  }
  for (int e = head + 4 * nv + threadIdx.x; e < n; e += kStatsThreads) st.add(x[e]);
  Partial p = st.partial();
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) merge(p, shfl_xor(p, m));
  __shared__ Partial sp[kStatsThreads / 64];
  if ((threadIdx.x & 63) == 0) sp[threadIdx.x >> 6] = p;
  __syncthreads();
  if (threadIdx.x == 0) {
    Partial t = sp[0];
    for (int w = 1; w < kStatsThreads / 64; ++w) merge(t, sp[w]);
    part[b] = t;
  }
}

// One wave per row: lane j merges chunks j, j + 64, ... in order, then a fixed butterfly.
__global__ __launch_bounds__(256) void k_stats_combine(const fjcomp_row* __restrict__ rows,
                                                        const int64_t* __restrict__ prefix, int64_t R,
                                                        const Partial* __restrict__ part, int method,
                                                        fjcomp_stats* __restrict__ stats,
                                                        fjcomp_qparams* __restrict__ qp) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  Partial t = {INFINITY, -INFINITY, -INFINITY, 0.0, 0.0, 0.0};
  for (int64_t c = prefix[r] + lane; c < prefix[r + 1]; c += 64) merge(t, part[c]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) merge(t, shfl_xor(t, m));
  if (lane != 0) return;
  stats[r] = fjcomp_stats{t.mn, t.mx, t.amx, t.s1, t.s2, t.sa};
  if (!qp) return;
  fjcomp_qparams q;
  if (method == FJCOMP_TERNGRAD) {
    // jnp.std (ddof 0) in f64, rounded once; thr = f32(2.5) * sigma (compression.py:331-332)
    const double n = (double)rows[r].n;
    const double mean = t.s1 / n;
    double var = t.s2 / n - mean * mean;
    var = var > 0.0 ? var : (var == var ? 0.0 : var);
    const float sigma = (float)sqrt(var);
    const float thr = 2.5f * sigma;
    const float amx = (float)t.amx;
    // amax(|clip(v)|): clipped entries become exactly thr (compression.py:333-335)
    const float vmax = (amx > thr) ? thr : amx;
    q.vmin = 0.0f;
    q.vmax = vmax;
    q.range = vmax - 0.0f;
    q.thr = thr;
  } else {
    q.vmin = (float)t.mn;
    q.vmax = (float)t.mx;
    q.range = q.vmax - q.vmin;
    q.thr = 0.0f;
  }
  q.rcp_range = 1.0 / (double)q.range;
  qp[r] = q;
}

// ------------------------------------------------------------------ quantize + fold
constexpr int kQThreads = 256;
constexpr int kQGroup = 4;  // clients whose deltas k_quant_fold loads one group ahead
constexpr int kHistLdsBins = 4096;

struct UniformQ {
  float lm1;
  double rcp_lm1;
  static constexpr bool kTable = false;
  static constexpr bool kPair = false;
  // uniform_stochastic_quantize (compression.py:84-97); *level = chosen level index
  __device__ inline float operator()(float v, float u, const fjcomp_qparams& p, float* level) const {
    const float a = clamp01_nan(div_by(v - p.vmin, p.rcp_range));
    const float fl = floorf(a * lm1), ce = ceilf(a * lm1);
    const float v_ceil = div_by(ce, rcp_lm1);
    const float v_floor = div_by(fl, rcp_lm1);
    const float thr = nan_to_num(div_rn(a - v_floor, v_ceil - v_floor));
    const bool down = u > thr;
    *level = down ? fl : ce;
    const float q = down ? v_floor : v_ceil;
    return p.vmin + q * p.range;
  }
};

// UniformQ with the per-level constants in LDS (num_levels <= kLevelTable): level j's value
// lev[j] = RN_f32(j / lm1) (the v_floor / v_ceil above) and rd[j] = RN_f64(1 / (lev[j+1] -
// lev[j])), so the threshold is RN_f32(num * rd[fl]) instead of an f32 division. That is
// the correctly rounded num / den whenever it is a normal float (the argument of the file
// header), and every other case gives the same decision u > thr: num is 0 or at least
// 2^-55 in magnitude unless fl = 0, where num = a >= 0 and any threshold below 2^-23
// compares like 0 against u (u is 0 or >= 2^-23). When ce == fl both branches pick the
// same level, so thr (and the unused rd[lm1] = 0) does not matter; no nan_to_num needed.
// One 16-byte entry per level, {lev[j], lev[j+1], rd[j]} (lev[lm1+1] := lev[lm1]), so a
// lane reads everything its element needs with one ds_read_b128 at j << 4.
constexpr int kLevelTable = 4096;
typedef float f2 __attribute__((ext_vector_type(2)));
struct UniformTQ {
  float lm1;
  int num_levels;
  double rcp_lm1;
  const uint4* tab;  // LDS, num_levels entries
  static constexpr bool kTable = true;
  static size_t lds_bytes(int num_levels) { return (size_t)num_levels * sizeof(uint4) + 16; }
  __device__ inline void build(void* smem) {
    uint4* e = reinterpret_cast<uint4*>(smem);
    const int top = num_levels - 1;  // == lm1
    for (int j = threadIdx.x; j <= top; j += blockDim.x) e[j].x = __float_as_uint(div_by((float)j, rcp_lm1));
    __syncthreads();
    for (int j = threadIdx.x; j <= top; j += blockDim.x) {
      const float lv = __uint_as_float(e[j].x), nx = j < top ? __uint_as_float(e[j + 1].x) : lv;
      const double r = j < top ? 1.0 / (double)(nx - lv) : 0.0;
      const uint64_t rb = (uint64_t)__double_as_longlong(r);
      e[j].y = __float_as_uint(nx);
      e[j].z = (uint32_t)rb;
      e[j].w = (uint32_t)(rb >> 32);
    }
    __syncthreads();
    tab = e;
  }
  __device__ inline float operator()(float v, float u, const fjcomp_qparams& p, float* level) const {
    const float a = clamp01_nan(div_by(v - p.vmin, p.rcp_range));
    const float s = a * lm1;
    const float fl = floorf(s), ce = ceilf(s);
    const uint4 t = tab[(int)fl];
    const float v_floor = __uint_as_float(t.x), v_next = __uint_as_float(t.y);
    const double rd = __longlong_as_double((long long)(((uint64_t)t.w << 32) | t.z));
    const float v_ceil = ce != fl ? v_next : v_floor;
    const float thr = (float)((double)(a - v_floor) * rd);
    const bool down = u > thr;
    *level = down ? fl : ce;
    const float q = down ? v_floor : v_ceil;
    return p.vmin + q * p.range;
  }
  // The same for a lane's element pair: the ops that take both elements through the same
  // constant (v - vmin, a * lm1, a - v_floor, vmin + q * range) are packed f32 ops.
  static constexpr bool kPair = true;
  __device__ inline f2 pair(f2 v, f2 u, const fjcomp_qparams& p, float* l0, float* l1) const {
    const f2 d = v - p.vmin;
    const f2 a = {clamp01_nan(div_by(d.x, p.rcp_range)), clamp01_nan(div_by(d.y, p.rcp_range))};
    const f2 s = a * lm1;
    const f2 fl = {floorf(s.x), floorf(s.y)}, ce = {ceilf(s.x), ceilf(s.y)};
    const uint4 t0 = tab[(int)fl.x], t1 = tab[(int)fl.y];
    const f2 v_floor = {__uint_as_float(t0.x), __uint_as_float(t1.x)};
    const f2 v_ceil = {ce.x != fl.x ? __uint_as_float(t0.y) : v_floor.x, ce.y != fl.y ? __uint_as_float(t1.y) : v_floor.y};
    const double rd0 = __longlong_as_double((long long)(((uint64_t)t0.w << 32) | t0.z));
    const double rd1 = __longlong_as_double((long long)(((uint64_t)t1.w << 32) | t1.z));
    const f2 num = a - v_floor;
    const bool down0 = u.x > (float)((double)num.x * rd0), down1 = u.y > (float)((double)num.y * rd1);
    *l0 = down0 ? fl.x : ce.x;
    *l1 = down1 ? fl.y : ce.y;
    const f2 q = {down0 ? v_floor.x : v_ceil.x, down1 ? v_floor.y : v_ceil.y};
    return p.vmin + q * p.range;
  }
};

struct BinaryQ {
  static constexpr bool kTable = false;
  static constexpr bool kPair = true;
  template <class Self>
  __device__ static inline f2 pair_of(const Self& q, f2 v, f2 u, const fjcomp_qparams& p) {
    return f2{q(v.x, u.x, p, nullptr), q(v.y, u.y, p, nullptr)};
  }
  __device__ inline f2 pair(f2 v, f2 u, const fjcomp_qparams& p, float*, float*) const { return pair_of(*this, v, u, p); }
  // binary_stochastic_quantize (compression.py:58-63)
  __device__ inline float operator()(float v, float u, const fjcomp_qparams& p, float*) const {
    const float a = clamp01_nan(div_by(v - p.vmin, p.rcp_range));
    return (u > a) ? p.vmin : p.vmax;
  }
};

struct TernQ {
  static constexpr bool kTable = false;
  static constexpr bool kPair = true;
  template <class Self>
  __device__ static inline f2 pair_of(const Self& q, f2 v, f2 u, const fjcomp_qparams& p) {
    return f2{q(v.x, u.x, p, nullptr), q(v.y, u.y, p, nullptr)};
  }
  __device__ inline f2 pair(f2 v, f2 u, const fjcomp_qparams& p, float*, float*) const { return pair_of(*this, v, u, p); }
  // terngrad_quantize (compression.py:323-336) with binary_stochastic_quantize(|v|, 0, vmax)
  __device__ inline float operator()(float v, float u, const fjcomp_qparams& p, float*) const {
    const float vc = (fabsf(v) > p.thr) ? p.thr * xla_sign(v) : v;
    const float av = fabsf(vc);
    const float a = clamp01_nan(div_by(av - 0.0f, p.rcp_range));
    const float r = (u > a) ? 0.0f : p.vmax;
    return r * xla_sign(vc);
  }
};

template <class Q, bool HIST>
__global__ __launch_bounds__(kQThreads) void k_quant_fold(Q quant, const float* const* __restrict__ in_ptrs,
                                                           const uint32_t* __restrict__ keys,
                                                           const fjcomp_qparams* __restrict__ qps,
                                                           const float* __restrict__ w, int64_t K, int64_t L,
                                                           const int64_t* __restrict__ leaf_n,
                                                           const int64_t* __restrict__ prefix, float scale,
                                                           int flags, float* const* __restrict__ out_ptrs,
                                                           int32_t* __restrict__ hist, int nbins) {
  const int64_t b = blockIdx.x;
  const int64_t l = find_segment(prefix, L, b);
  if constexpr (Q::kTable) {
    extern __shared__ __attribute__((aligned(16))) unsigned char qtab[];
    quant.build(qtab);
  }
  const int64_t n = leaf_n[l], h = (n + 1) >> 1;
  const int64_t i0 = (b - prefix[l]) * kQThreads, i = i0 + threadIdx.x;
  const bool valid = i < h, second = i + h < n;
  // Deltas are read with buffer loads: per client, two descriptors (this block's first
  // element, and the element h further) built on the scalar unit from the row pointer,
  // and one loop-invariant lane offset, so a load costs no address VALU. Every lane loads
  // unconditionally (no branch around the loads, so waiting for one group's deltas never
  // waits for the next group's as well); lanes past the leaf read zeros (range check).
  const uint32_t lane_off = threadIdx.x * 4u;
  const int lim_a = (int)((n - i0) * 4 < 0x7fffffffll ? (n - i0) * 4 : 0x7fffffffll);
  const int lim_b = (int)((n - i0 - h) * 4 < 0x7fffffffll ? (n - i0 - h) * 4 : 0x7fffffffll);
  typedef __attribute__((address_space(1))) float GFloatOut;
  GFloatOut* out = (GFloatOut*)out_ptrs[l];
  const bool accumulate = flags & FJAGG_ACCUMULATE;
  float s0 = 0.0f, s1 = 0.0f;
  if (valid && accumulate) {
    s0 = out[i];
    if (second) s1 = out[i + h];
  }
  __shared__ int32_t sh[HIST ? kHistLdsBins : 1];
  const bool lds_hist = HIST && nbins <= kHistLdsBins;
  const int hist_group = lds_hist ? kHistLdsBins / nbins : 1;  // clients per LDS histogram cycle
  int hslot = 0;
  // Per-client constants of this leaf (row pointer, key, weight, quantizer constants) are
  // staged in LDS, kQThreads clients at a time, by one coalesced pass of the block: read
  // straight from the (client, leaf) tables with scalar loads, every client cost a
  // scalar-cache miss and a wait in every wave (the rows of one leaf are L entries apart).
  struct QClient {
    uint64_t ptr;
    uint32_t k0, k1, k2, wbits;
    fjcomp_qparams p;
  };
  __shared__ QClient qc[kQThreads];
  constexpr int G = kQGroup;
  // A lane walks all K clients, so one dependent HBM round trip per client would bound
  // the kernel. The deltas of the next G clients are loaded before this group's threefry
  // draws and quantizers run, which hide their latency. Fold order unchanged.
  auto fetch = [&](int64_t j, int64_t jn, float (&a)[G], float (&c)[G]) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint64_t pv = qc[j + u < jn ? j + u : jn - 1].ptr;
      const uint64_t pb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv);
      float* x = reinterpret_cast<float*>(pb) + i0;
      a[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          __builtin_amdgcn_make_buffer_rsrc(x, (short)0, lim_a, 0x00020000), lane_off, 0, 0));
      c[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          __builtin_amdgcn_make_buffer_rsrc(x + h, (short)0, lim_b, 0x00020000), lane_off, 0, 0));
    }
  };
  // fold chunk clients j .. j+G-1 (those < jn; global index kc + j) from their deltas a / c
  auto fold_group = [&](int64_t kc, int64_t j, int64_t jn, const float (&a)[G], const float (&c)[G]) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (j + u >= jn) break;  // wave-uniform
      const int64_t k = kc + j + u;
      const QClient& e = qc[j + u];
      const uint32_t k0 = e.k0, k1 = e.k1, k2 = e.k2;
      const fjcomp_qparams p = e.p;
      const float wk = __uint_as_float(e.wbits);
      float lv0 = -1.0f, lv1 = -1.0f;
      if constexpr (Q::kPair) {
        // Both elements, on every lane: lanes past the leaf (they read zeros) and lanes
        // without a second element fold junk that is never stored. No branch, so the
        // compiler can interleave the independent threefry chains of the group's clients.
        uint32_t c0 = (uint32_t)i, c1 = (uint32_t)(second ? i + h : 0);
        threefry_k(k0, k1, k2, c0, c1);
        const f2 uu = {__uint_as_float(__builtin_amdgcn_alignbit(0x7fu, c0, 9u)),
                       __uint_as_float(__builtin_amdgcn_alignbit(0x7fu, c1, 9u))};
        const f2 t = quant.pair(f2{a[u], c[u]}, uu - 1.0f, p, &lv0, &lv1) * wk;
        f2 sv = {s0, s1};
        sv = (k == 0 && !accumulate) ? t : sv + t;
        s0 = sv.x;
        s1 = sv.y;
      } else if (valid) {
        const float v0 = a[u];
        const float v1 = c[u];  // used only when `second`
        uint32_t c0 = (uint32_t)i, c1 = (uint32_t)(second ? i + h : 0);
        threefry_k(k0, k1, k2, c0, c1);
        const float q0 = quant(v0, bits_to_unit(c0), p, &lv0);
        const float t0 = q0 * wk;
        s0 = (k == 0 && !accumulate) ? t0 : s0 + t0;
        if (second) {
          const float q1 = quant(v1, bits_to_unit(c1), p, &lv1);
          const float t1 = q1 * wk;
          s1 = (k == 0 && !accumulate) ? t1 : s1 + t1;
        }
      }
      if constexpr (HIST) {
        int32_t* __restrict__ hrow = hist + (k * L + l) * nbins;
        const int top = nbins - 1;
        auto bin = [&](float lv) { return (lv >= 0.0f && lv < (float)top) ? (int)lv : top; };
        if (lds_hist) {
          // hist_group consecutive clients share one zero / count / flush cycle: client
          // j counts into LDS slot j % hist_group, the slots go out together (2 barriers
          // per group instead of 3 per client)
          // (hslot: this client's slot, counted per chunk; wave-uniform)
          if (hslot == 0) {  // first client of a group
            for (int e2 = threadIdx.x; e2 < hist_group * nbins; e2 += kQThreads) sh[e2] = 0;
            __syncthreads();
          }
          int32_t* hs = sh + hslot * nbins;
          if (valid) {
            atomicAdd(&hs[bin(lv0)], 1);
            if (second) atomicAdd(&hs[bin(lv1)], 1);
          }
          if (hslot == hist_group - 1 || j + u == jn - 1) {  // last client of a group
            __syncthreads();
            const int64_t g0 = k - hslot;  // the group's first client
            for (int e2 = threadIdx.x; e2 < (hslot + 1) * nbins; e2 += kQThreads) {
              const int c = e2 / nbins;  // 32-bit: at most kHistLdsBins entries
              if (sh[e2]) atomicAdd(&hist[((g0 + c) * L + l) * nbins + (e2 - c * nbins)], sh[e2]);
            }
            __syncthreads();
            hslot = 0;
          } else {
            ++hslot;
          }
        } else if (valid) {
          atomicAdd(&hrow[bin(lv0)], 1);
          if (second) atomicAdd(&hrow[bin(lv1)], 1);
        }
      }
    }
  };
  for (int64_t kc = 0; kc < K; kc += kQThreads) {
    const int64_t jn = K - kc < kQThreads ? K - kc : kQThreads;
    if (kc) __syncthreads();  // every wave is done with the previous chunk's entries
    if (threadIdx.x < jn) {
      const int64_t k = kc + threadIdx.x, row = k * L + l;
      QClient e;
      e.ptr = (uint64_t)in_ptrs[row];
      e.k0 = keys[2 * row];
      e.k1 = keys[2 * row + 1];
      e.k2 = e.k0 ^ e.k1 ^ 0x1BD11BDAu;
      e.wbits = __float_as_uint(w[k]);
      e.p = qps[row];
      qc[threadIdx.x] = e;
    }
    __syncthreads();
    // Two register sets in turn (no copies between them, which would wait for the loads):
    // while one group is folded, the next group's loads are in flight.
    float xa[G], xb[G], ya[G], yb[G];
    fetch(0, jn, xa, xb);
    for (int64_t j = 0; j < jn; j += 2 * G) {
      fetch(j + G, jn, ya, yb);
      fold_group(kc, j, jn, xa, xb);
      if (j + G >= jn) break;  // wave-uniform
      fetch(j + 2 * G, jn, xa, xb);
      fold_group(kc, j + G, jn, ya, yb);
    }
  }
  if (!valid) return;
  if (flags & FJAGG_SCALE) {
    s0 = s0 * scale;
    s1 = s1 * scale;
  }
  out[i] = s0;
  if (second) out[i + h] = s1;
}

// ------------------------------------------------------------------ Walsh-Hadamard
constexpr int kWhtBits = 13;    // butterfly bits of pass 0 (contiguous tiles of 8192)
constexpr int kWhtHighBits = 8; // later passes: 2^8 strided rows x >= 32 contiguous floats (128 B)
constexpr int kWhtTile = 1 << kWhtBits;
constexpr int kWhtThreads = 512;

__host__ __device__ inline int wht_passes(int m) {
  return m <= kWhtBits ? 1 : 1 + (m - kWhtBits + kWhtHighBits - 1) / kWhtHighBits;
}

// Tiling of pass p of a 2^m job: the pass does butterfly bits [lo, lo + nb); a tile holds
// all 2^nb values of those bits for c consecutive values of the lower bits.
struct WhtTiling {
  int lo, nb, lc;
  int64_t c, tile, tiles;
};
__host__ __device__ inline WhtTiling wht_tiling(int m, int pass) {
  WhtTiling t;
  t.lo = pass == 0 ? 0 : kWhtBits + kWhtHighBits * (pass - 1);
  const int cap = pass == 0 ? kWhtBits : kWhtHighBits;
  t.nb = m - t.lo < cap ? m - t.lo : cap;
  if (t.nb < 0) t.nb = 0;
  const int64_t span = (int64_t)1 << t.lo;
  const int64_t cmax = (int64_t)kWhtTile >> t.nb;
  t.c = span < cmax ? span : cmax;
  t.lc = 0;
  while (((int64_t)1 << t.lc) < t.c) ++t.lc;
  t.tile = t.c << t.nb;
  t.tiles = ((int64_t)1 << m) / t.tile;
  return t;
}

__device__ inline int lds_pad(int e) { return e + (e >> 5); }

template <int G>
__device__ inline void wht_group(float* sm, int64_t tile, int p) {
  const int nq = (int)(tile >> G);
  for (int q = threadIdx.x; q < nq; q += kWhtThreads) {
    const int base = ((q >> p) << (p + G)) | (q & ((1 << p) - 1));
    float v[1 << G];
#pragma unroll
    for (int r = 0; r < (1 << G); ++r) v[r] = sm[lds_pad(base + (r << p))];
#pragma unroll
    for (int s = 0; s < G; ++s)
#pragma unroll
      for (int r = 0; r < (1 << G); ++r)
        if (!(r & (1 << s))) {
          const float a = v[r], c = v[r | (1 << s)];
          v[r] = a + c;
          v[r | (1 << s)] = a - c;
        }
#pragma unroll
    for (int r = 0; r < (1 << G); ++r) sm[lds_pad(base + (r << p))] = v[r];
  }
}

__device__ inline float sign_of(const uint32_t* __restrict__ s, int64_t g) {
  return ((s[g >> 5] >> (g & 31)) & 1u) ? -1.0f : 1.0f;
}

__global__ __launch_bounds__(kWhtThreads) void k_wht(const fjcomp_wht_job* __restrict__ jobs,
                                                      const int64_t* __restrict__ prefix, int64_t J, int pass) {
  __shared__ float sm[kWhtTile + kWhtTile / 32];
  const int64_t b = blockIdx.x;
  const int64_t j = find_segment(prefix, J, b);
  const fjcomp_wht_job jb = jobs[j];
  const int m = jb.log2d;
  const WhtTiling t = wht_tiling(m, pass);
  const int64_t tix = b - prefix[j];
  const int64_t cph = ((int64_t)1 << t.lo) / t.c;
  const int64_t base = ((tix / cph) << (t.lo + t.nb)) + (tix % cph) * t.c;
  const bool first = pass == 0, last = pass == wht_passes(m) - 1;
  const int kind = jb.kind;
  const double rcp_sqrt_d = 1.0 / (double)jb.sqrt_d;
  double rcp_b = 0.0;
  float A = 0.0f;
  if (first && kind == FJCOMP_WHT_UNROTATE_DRIVE) {
    A = (float)jb.stats->sumsq;
    rcp_b = 1.0 / (double)(float)jb.stats->sumabs;
  }
  const float* __restrict__ src = first ? jb.src : jb.mid;
  // Tile element e sits at g(e); runs of consecutive g are the whole tile in pass 0 (c = 1)
  // and c >= 32 floats later. When runs are multiples of 4, lanes move 16-byte quads (e and
  // g both multiples of 4, same sign word, lds_pad(e + u) = lds_pad(e) + u); the element
  // arithmetic is the scalar path's, so results are bitwise the same.
  const bool quads = ((t.lo == 0 ? t.tile : t.c) & 3) == 0;
  if (quads && ((uintptr_t)src & 15) == 0) {
    for (int e = 4 * threadIdx.x; e < t.tile; e += 4 * kWhtThreads) {
      const int64_t g = base + ((int64_t)(e >> t.lc) << t.lo) + (e & (t.c - 1));
      float v[4];
      if (first && kind == FJCOMP_WHT_ROTATE) {
        if (g + 3 < jb.n_in) {
          const float4 q = *reinterpret_cast<const float4*>(src + g);
          v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = g + u < jb.n_in ? src[g + u] : 0.0f;
        }
        const uint32_t sw = jb.signs[g >> 5] >> (g & 31);
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = v[u] * (((sw >> u) & 1u) ? -1.0f : 1.0f);
      } else {
        const float4 q = *reinterpret_cast<const float4*>(src + g);
        v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        if (first && kind == FJCOMP_WHT_UNROTATE_DRIVE) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = div_by(A * xla_sign(v[u]), rcp_b);
        }
      }
      const int o = lds_pad(e);
#pragma unroll
      for (int u = 0; u < 4; ++u) sm[o + u] = v[u];
    }
  } else {
    for (int e = threadIdx.x; e < t.tile; e += kWhtThreads) {
      const int64_t g = base + ((int64_t)(e >> t.lc) << t.lo) + (e & (t.c - 1));
      float v;
      if (first && kind == FJCOMP_WHT_ROTATE) {
        v = g < jb.n_in ? src[g] : 0.0f;
        v = v * sign_of(jb.signs, g);
      } else if (first && kind == FJCOMP_WHT_UNROTATE_DRIVE) {
        v = div_by(A * xla_sign(src[g]), rcp_b);  // drive_pytree: (sum(y^2) * sign(y)) / sum(|y|)
      } else {
        v = src[g];
      }
      sm[lds_pad(e)] = v;
    }
  }
  __syncthreads();
  for (int s0 = 0; s0 < t.nb; s0 += 4) {
    const int p = t.lc + s0;
    switch (t.nb - s0 < 4 ? t.nb - s0 : 4) {
      case 1: wht_group<1>(sm, t.tile, p); break;
      case 2: wht_group<2>(sm, t.tile, p); break;
      case 3: wht_group<3>(sm, t.tile, p); break;
      default: wht_group<4>(sm, t.tile, p); break;
    }
    __syncthreads();
  }
  float* __restrict__ dptr = last ? jb.dst : jb.mid;
  // ROTATE with a partials pointer: this tile's min / max / |max| of the rotated values
  // (order-independent, so the row's combine equals k_row_stats' exactly; sums stay 0)
  const bool tile_stats = last && kind == FJCOMP_WHT_ROTATE && jb.stats;
  const bool tile_sums = tile_stats && (jb.flags & FJCOMP_WHT_F_SUMS);
  MinMax mm;
  if (quads && ((uintptr_t)dptr & 15) == 0) {
    for (int e = 4 * threadIdx.x; e < t.tile; e += 4 * kWhtThreads) {
      const int64_t g = base + ((int64_t)(e >> t.lc) << t.lo) + (e & (t.c - 1));
      const int o = lds_pad(e);
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = sm[o + u];
      if (last) {
        if (g >= jb.n_out) continue;
        if (kind == FJCOMP_WHT_ROTATE) {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = div_by(v[u], rcp_sqrt_d);
          if (tile_stats) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (g + u < jb.n_out) mm.add(v[u], tile_sums);
          }
        } else if (kind != FJCOMP_WHT_PLAIN) {
          const uint32_t sw = jb.signs[g >> 5] >> (g & 31);
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = div_by(v[u] * (((sw >> u) & 1u) ? -1.0f : 1.0f), rcp_sqrt_d);
        }
        if (g + 3 >= jb.n_out) {  // truncated to the leaf's n_out elements
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (g + u < jb.n_out) dptr[g + u] = v[u];
          continue;
        }
      }
      *reinterpret_cast<float4*>(dptr + g) = make_float4(v[0], v[1], v[2], v[3]);
    }
    if (tile_stats) mm.store(reinterpret_cast<Partial*>(const_cast<fjcomp_stats*>(jb.stats)) + tix, tile_sums);
    return;
  }
  for (int e = threadIdx.x; e < t.tile; e += kWhtThreads) {
    const int64_t g = base + ((int64_t)(e >> t.lc) << t.lo) + (e & (t.c - 1));
    float v = sm[lds_pad(e)];
    if (!last) {
      jb.mid[g] = v;
      continue;
    }
    if (g >= jb.n_out) continue;
    if (kind == FJCOMP_WHT_ROTATE) {
      v = div_by(v, rcp_sqrt_d);
      if (tile_stats) mm.add(v, tile_sums);
    } else if (kind != FJCOMP_WHT_PLAIN) {
      v = div_by(v * sign_of(jb.signs, g), rcp_sqrt_d);
    }
    jb.dst[g] = v;
  }
  if (tile_stats) mm.store(reinterpret_cast<Partial*>(const_cast<fjcomp_stats*>(jb.stats)) + tix, tile_sums);
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

void host_split(const uint32_t key[2], int64_t num, uint32_t* out) {
  // threefry_2x32(key, iota(2*num)).reshape(num, 2): flat = [y0 | y1]
  std::vector<uint32_t> flat(2 * num);
  for (int64_t i = 0; i < num; ++i) {
    uint32_t x0 = (uint32_t)i, x1 = (uint32_t)(num + i);
    threefry(key[0], key[1], x0, x1);
    flat[i] = x0;
    flat[num + i] = x1;
  }
  memcpy(out, flat.data(), sizeof(uint32_t) * 2 * num);
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

int fjcomp_abi_version(void) { return FJCOMP_ABI_VERSION; }

int fjcomp_threefry2x32(const uint32_t key[2], const uint32_t* x0, const uint32_t* x1, int64_t n, uint32_t* y0,
                        uint32_t* y1) {
  fjagg_g_err[0] = 0;
  if (!key || n < 0 || (n && (!x0 || !x1 || !y0 || !y1))) return fail(FJAGG_EINVAL, "threefry2x32: bad arguments");
  for (int64_t i = 0; i < n; ++i) {
    uint32_t a = x0[i], b = x1[i];
    threefry(key[0], key[1], a, b);
    y0[i] = a;
    y1[i] = b;
  }
  return FJAGG_OK;
}

int fjcomp_random_split(const uint32_t* keys, int64_t nkeys, int64_t num, uint32_t* out) {
  fjagg_g_err[0] = 0;
  if (nkeys < 0 || num < 0 || ((nkeys && num) && (!keys || !out)) || num > (int64_t)1 << 31)
    return fail(FJAGG_EINVAL, "random_split: bad arguments (nkeys=%lld num=%lld)", (long long)nkeys, (long long)num);
  for (int64_t k = 0; k < nkeys; ++k) host_split(keys + 2 * k, num, out + 2 * num * k);
  return FJAGG_OK;
}

int fjcomp_prng_sequence(uint32_t key[2], int64_t n, uint32_t* subkeys) {
  fjagg_g_err[0] = 0;
  if (!key || n < 0 || (n && !subkeys)) return fail(FJAGG_EINVAL, "prng_sequence: bad arguments");
  uint32_t two[4];
  for (int64_t i = 0; i < n; ++i) {  // haiku: reserve(1) = split(key, 2); key <- [0]; yield [1]
    host_split(key, 2, two);
    key[0] = two[0];
    key[1] = two[1];
    subkeys[2 * i] = two[2];
    subkeys[2 * i + 1] = two[3];
  }
  return FJAGG_OK;
}

static int random_common(uint32_t k0, uint32_t k1, int64_t n, uint32_t* out, float* outf, void* stream) {
  fjagg_g_err[0] = 0;
  if (n < 0 || n > (int64_t)UINT32_MAX) return fail(FJAGG_EINVAL, "random: n=%lld outside [0, 2^32)", (long long)n);
  if (n == 0) return FJAGG_OK;
  if (!out && !outf) return fail(FJAGG_EINVAL, "random: null output");
  const int64_t h = (n + 1) >> 1;
  hipLaunchKernelGGL(k_random_bits, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, as_stream(stream), k0, k1, n,
                     out, outf);
  return check_launch("k_random_bits");
}

int fjcomp_random_bits(uint32_t k0, uint32_t k1, int64_t n, uint32_t* out, void* stream) {
  return random_common(k0, k1, n, out, nullptr, stream);
}

int fjcomp_uniform(uint32_t k0, uint32_t k1, int64_t n, float* out, void* stream) {
  return random_common(k0, k1, n, nullptr, out, stream);
}

int fjcomp_rademacher(const fjcomp_sign_job* jobs, const int64_t* block_prefix, int64_t J, int64_t nblocks,
                      int block_pairs, void* stream) {
  fjagg_g_err[0] = 0;
  if (J < 0 || nblocks < 0 || (J && (!jobs || !block_prefix)) || nblocks > INT32_MAX)
    return fail(FJAGG_EINVAL, "rademacher: bad arguments");
  if (block_pairs < 256 || block_pairs > FJCOMP_SIGN_BLOCK_PAIRS || block_pairs % 256)
    return fail(FJAGG_EINVAL, "rademacher: block_pairs=%d (a multiple of 256, at most %d)", block_pairs,
                FJCOMP_SIGN_BLOCK_PAIRS);
  if (!J || !nblocks) return FJAGG_OK;
  hipLaunchKernelGGL(k_rademacher, dim3((unsigned)nblocks), dim3(256), 0, as_stream(stream), jobs, block_prefix, J,
                     block_pairs / 256);
  return check_launch("k_rademacher");
}

int64_t fjcomp_row_stats_workspace_bytes(int64_t nchunks) { return nchunks < 1 ? 0 : nchunks * (int64_t)sizeof(Partial); }

int fjcomp_row_stats(const fjcomp_row* rows, const int64_t* chunk_prefix, int64_t R, int64_t nchunks, int method,
                     fjcomp_stats* stats, fjcomp_qparams* qparams, void* ws, int64_t ws_bytes, void* stream) {
  fjagg_g_err[0] = 0;
  if (R < 0 || nchunks < R || (R && (!rows || !chunk_prefix || !stats)) || nchunks > INT32_MAX)
    return fail(FJAGG_EINVAL, "row_stats: bad arguments (R=%lld nchunks=%lld)", (long long)R, (long long)nchunks);
  if (qparams && method != FJCOMP_UNIFORM && method != FJCOMP_TERNGRAD && method != FJCOMP_BINARY)
    return fail(FJAGG_EINVAL, "row_stats: qparams need method UNIFORM, BINARY or TERNGRAD, got %d", method);
  if (!R) return FJAGG_OK;
  if (!ws || ws_bytes < fjcomp_row_stats_workspace_bytes(nchunks))
    return fail(FJAGG_EINVAL, "row_stats: workspace %lld B < %lld B", (long long)ws_bytes,
                (long long)fjcomp_row_stats_workspace_bytes(nchunks));
  hipStream_t s = as_stream(stream);
  Partial* part = static_cast<Partial*>(ws);
  hipLaunchKernelGGL(k_row_stats, dim3((unsigned)nchunks), dim3(kStatsThreads), 0, s, rows, chunk_prefix, R, part);
  if (int rc = check_launch("k_row_stats")) return rc;
  hipLaunchKernelGGL(k_stats_combine, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, s, rows, chunk_prefix, R, part,
                     method, stats, qparams);
  return check_launch("k_stats_combine");
}

int fjcomp_stats_combine(const fjcomp_row* rows, const int64_t* part_prefix, int64_t R, int method,
                         const void* part, fjcomp_stats* stats, fjcomp_qparams* qparams, void* stream) {
  fjagg_g_err[0] = 0;
  if (R < 0 || (R && (!rows || !part_prefix || !part || !stats)))
    return fail(FJAGG_EINVAL, "stats_combine: bad arguments (R=%lld)", (long long)R);
  if (qparams && method != FJCOMP_UNIFORM && method != FJCOMP_BINARY)
    return fail(FJAGG_EINVAL, "stats_combine: min/max partials give qparams for UNIFORM or BINARY only, got %d",
                method);
  if (!R) return FJAGG_OK;
  hipLaunchKernelGGL(k_stats_combine, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, as_stream(stream), rows,
                     part_prefix, R, static_cast<const Partial*>(part), method, stats, qparams);
  return check_launch("k_stats_combine");
}

int fjcomp_quant_fold(int method, const float* const* in_ptrs, const uint32_t* keys, const fjcomp_qparams* qparams,
                      const float* w, int64_t K, int64_t L, const int64_t* leaf_n, const int64_t* block_prefix,
                      int64_t nblocks, int num_levels, float scale, int flags, float* const* out_ptrs, int32_t* hist,
                      void* stream) {
  fjagg_g_err[0] = 0;
  if (K < 1 || L < 0 || nblocks < 0 || nblocks > INT32_MAX)
    return fail(FJAGG_EINVAL, "quant_fold: bad sizes (K=%lld L=%lld nblocks=%lld)", (long long)K, (long long)L,
                (long long)nblocks);
  if (L && (!in_ptrs || !keys || !qparams || !w || !leaf_n || !block_prefix || !out_ptrs))
    return fail(FJAGG_EINVAL, "quant_fold: null table");
  if (flags & ~(FJAGG_SCALE | FJAGG_ACCUMULATE)) return fail(FJAGG_EINVAL, "quant_fold: unsupported flags %#x", flags);
  if (!L || !nblocks) return FJAGG_OK;
  hipStream_t s = as_stream(stream);
  if (method == FJCOMP_UNIFORM) {
    if (num_levels < 1) return fail(FJAGG_EINVAL, "quant_fold: num_levels=%d", num_levels);
    if (num_levels <= kLevelTable) {  // level constants in LDS, no per-element division
      UniformTQ q{};
      q.lm1 = (float)(num_levels - 1);
      q.num_levels = num_levels;
      q.rcp_lm1 = 1.0 / (double)q.lm1;
      const size_t smem = UniformTQ::lds_bytes(num_levels);
      if (hist)
        hipLaunchKernelGGL((k_quant_fold<UniformTQ, true>), dim3((unsigned)nblocks), dim3(kQThreads), smem, s, q,
                           in_ptrs, keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist,
                           num_levels + 1);
      else
        hipLaunchKernelGGL((k_quant_fold<UniformTQ, false>), dim3((unsigned)nblocks), dim3(kQThreads), smem, s, q,
                           in_ptrs, keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist, 0);
      return check_launch("k_quant_fold");
    }
    UniformQ q;
    q.lm1 = (float)(num_levels - 1);
    q.rcp_lm1 = 1.0 / (double)q.lm1;
    if (hist) {
      hipLaunchKernelGGL((k_quant_fold<UniformQ, true>), dim3((unsigned)nblocks), dim3(kQThreads), 0, s, q, in_ptrs,
                         keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist, num_levels + 1);
    } else {
      hipLaunchKernelGGL((k_quant_fold<UniformQ, false>), dim3((unsigned)nblocks), dim3(kQThreads), 0, s, q, in_ptrs,
                         keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist, 0);
    }
  } else if (method == FJCOMP_BINARY) {
    if (hist) return fail(FJAGG_EINVAL, "quant_fold: histogram only for UNIFORM");
    hipLaunchKernelGGL((k_quant_fold<BinaryQ, false>), dim3((unsigned)nblocks), dim3(kQThreads), 0, s, BinaryQ{},
                       in_ptrs, keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist, 0);
  } else if (method == FJCOMP_TERNGRAD) {
    if (hist) return fail(FJAGG_EINVAL, "quant_fold: histogram only for UNIFORM");
    hipLaunchKernelGGL((k_quant_fold<TernQ, false>), dim3((unsigned)nblocks), dim3(kQThreads), 0, s, TernQ{}, in_ptrs,
                       keys, qparams, w, K, L, leaf_n, block_prefix, scale, flags, out_ptrs, hist, 0);
  } else {
    return fail(FJAGG_EINVAL, "quant_fold: unknown method %d", method);
  }
  return check_launch("k_quant_fold");
}

int64_t fjcomp_wht_tiles(int log2d, int pass) {
  if (log2d < 0 || log2d > FJCOMP_WHT_MAX_LOG2 || pass < 0 || pass >= wht_passes(log2d)) return 0;
  return wht_tiling(log2d, pass).tiles;
}

int fjcomp_wht(const fjcomp_wht_job* jobs, const int64_t* pass_prefix, int64_t J, int npass, const int64_t* pass_tiles,
               void* stream) {
  fjagg_g_err[0] = 0;
  if (J < 0 || npass < 0 || npass > wht_passes(FJCOMP_WHT_MAX_LOG2) || (J && (!jobs || !pass_prefix || !pass_tiles)))
    return fail(FJAGG_EINVAL, "wht: bad arguments (J=%lld npass=%d)", (long long)J, npass);
  hipStream_t s = as_stream(stream);
  for (int p = 0; p < npass && J; ++p) {
    if (pass_tiles[p] < 0 || pass_tiles[p] > INT32_MAX) return fail(FJAGG_EINVAL, "wht: pass %d tiles", p);
    if (!pass_tiles[p]) continue;
    hipLaunchKernelGGL(k_wht, dim3((unsigned)pass_tiles[p]), dim3(kWhtThreads), 0, s, jobs, pass_prefix + p * (J + 1),
                       J, p);
    if (int rc = check_launch("k_wht")) return rc;
  }
  return FJAGG_OK;
}

}  // extern "C"
