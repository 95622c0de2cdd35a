// fjtree.hip — per-call tree ops (tree_weight / tree_add / tree_inverse_weight /
// tree_l2_norm of fedjax/core/tree_util.py:29-114) over at most FJTREE_MAX_LEAVES
// leaves, with the leaf table in the kernel arguments. C ABI: include/fjtree.h.
//
// These calls sit in the per-client loop of FedJAX's library algorithms
// (fedjax/algorithms/fed_avg.py:132-146): one or two pytrees in, one out, a few MB per
// call. What costs at that size is the host side of a launch, so the design removes
// every per-call transfer: the (operand, leaf) pointers, leaf sizes, weights and the
// workgroup -> leaf map are all kernel arguments (~2.4 KB), read from the kernarg
// segment by the scalar unit. The GPU side is a plain streaming pass:
//
//   * a workgroup (4 waves) owns kChunk = 4096 consecutive elements of one leaf; lane j
//     owns elements e0 + 4 (j + 256 i) + c, i, c = 0..3, so every lane has 4 x 16 bytes
//     of each operand in flight before it computes (vector path), or the same elements
//     with scalar loads when a leaf's pointers are not 16-byte aligned;
//   * the fold is the reference's op sequence (fl(x*w), fl(s+t), fl(s*scale)) with
//     __fmul_rn / __fadd_rn and -ffp-contract=off;
//   * the optional l2 norm reads the operand the fold already loaded: per-lane partials
//     in element order, xor butterfly, waves in order, then the last workgroup to finish
//     (completion counter, agent-scope stores and loads) adds the workgroup partials in order and
//     resets the counter. The lane -> element map is the same on both paths, so the norm
//     does not depend on alignment.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fjagg.h"
#include "fjtree.h"

extern thread_local char fjagg_g_err[512];

static_assert(sizeof(fjtree_leaves) == 2104, "fjtree_leaves layout (mirrored by _lib.TreeLeaves)");

namespace {

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(fjagg_g_err, sizeof(fjagg_g_err), fmt, ap);
  va_end(ap);
  return code;
}

constexpr int kThreads = 256;
constexpr int kPer = 4;                        // float4 units per lane
constexpr int64_t kChunk = kThreads * kPer * 4;  // elements per workgroup
constexpr int kWsHeader = 256;                 // bytes before the partials (counter at 0)

struct Args {
  const float* x[FJTREE_MAX_OPERANDS][FJTREE_MAX_LEAVES];
  float* out[FJTREE_MAX_LEAVES];
  int64_t n[FJTREE_MAX_LEAVES];
  int32_t blk0[FJTREE_MAX_LEAVES + 1];
  uint64_t vec_mask;  // leaf l: every pointer 16-byte aligned
  float w[FJTREE_MAX_OPERANDS];
  float scale;
  int L, nblk, scale_on;
  int norm_operand;
  int ordered;  // FJTREE_ORDERED
  float* norm_out;
  unsigned* counter;
  float* partials;
};
static_assert(sizeof(Args) <= 4096 - 64, "kernel arguments");

template <int K, bool OUT, bool NORM>
__global__ __launch_bounds__(kThreads) void k_leaves(const Args a) {
  __shared__ float wsum[kThreads / 64];
  __shared__ int last;
  const int b = blockIdx.x;
  // leaf of this workgroup: blk0 is non-decreasing and padded with INT32_MAX, so counting
  // the entries <= b needs no data-dependent loop (the scalar unit loads blk0 in a few
  // wide independent loads instead of one dependent load per leaf)
  int l = 0;
#pragma unroll
  for (int i = 1; i < FJTREE_MAX_LEAVES; ++i) l += a.blk0[i] <= b;
  const int64_t n = a.n[l];
  const int64_t e0 = (int64_t)(b - a.blk0[l]) * kChunk;
  const int64_t e1 = e0 + kChunk < n ? e0 + kChunk : n;
  const int j = threadIdx.x;
  const float* x0 = a.x[0][l];
  const float* x1 = K == 2 ? a.x[1][l] : nullptr;
  float* o = OUT ? a.out[l] : nullptr;
  const float w0 = a.w[0], w1 = K == 2 ? a.w[1] : 0.f, sc = a.scale;
  const bool scale_on = a.scale_on;
  float acc = 0.f;
  const bool vec = (a.vec_mask >> l) & 1;
  float v0[kPer][4], v1[kPer][4];
  if (e0 < e1) {
    if (vec) {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int64_t e = e0 + 4 * (j + kThreads * i);
        if (e + 4 <= e1) {
          const float4 p = *reinterpret_cast<const float4*>(x0 + e);
          v0[i][0] = p.x, v0[i][1] = p.y, v0[i][2] = p.z, v0[i][3] = p.w;
          if (K == 2) {
            const float4 q = *reinterpret_cast<const float4*>(x1 + e);
            v1[i][0] = q.x, v1[i][1] = q.y, v1[i][2] = q.z, v1[i][3] = q.w;
          }
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            v0[i][c] = e + c < e1 ? x0[e + c] : 0.f;
            if (K == 2) v1[i][c] = e + c < e1 ? x1[e + c] : 0.f;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int64_t e = e0 + 4 * (j + kThreads * i);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          v0[i][c] = e + c < e1 ? x0[e + c] : 0.f;
          if (K == 2) v1[i][c] = e + c < e1 ? x1[e + c] : 0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int64_t e = e0 + 4 * (j + kThreads * i);
      float r[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (NORM && e + c < e1) {
          const float v = (K == 2 && a.norm_operand == 1) ? v1[i][c] : v0[i][c];
          acc = __fadd_rn(acc, __fmul_rn(v, v));
        }
        if (OUT) {
          float s = __fmul_rn(v0[i][c], w0);
          if (K == 2) s = __fadd_rn(s, __fmul_rn(v1[i][c], w1));
          if (scale_on) s = __fmul_rn(s, sc);
          r[c] = s;
        }
      }
      if (OUT) {
        if (vec && e + 4 <= e1) {
          *reinterpret_cast<float4*>(o + e) = make_float4(r[0], r[1], r[2], r[3]);
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (e + c < e1) o[e + c] = r[c];
        }
      }
    }
  }
  if constexpr (NORM) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc = __fadd_rn(acc, __shfl_xor(acc, off));
    if ((j & 63) == 0) wsum[j >> 6] = acc;
    __syncthreads();
    if (j == 0) {
      float p = wsum[0];
#pragma unroll
      for (int w = 1; w < kThreads / 64; ++w) p = __fadd_rn(p, wsum[w]);
      // Publish the partial, then count it (include/fjtree.h).
      __hip_atomic_store(a.partials + b, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned old;
      if (a.ordered) {
        // memory-model ordering: the release half orders the partial before the count, the
        // acquire half orders the last workgroup's reads after every other count
        old = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        // gfx950 hand-off (MI355X guide, Guideline 16 R1): the agent-scope store above is
        // write-through (sc1); draining it before the counter add means it has reached the
        // device-coherent level when the add is seen, with no release fence (on gfx950 a
        // whole-L2 write-back, outputs included: 10.9 -> 15.1 us per fused add + norm)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      last = old == (unsigned)(a.nblk - 1);
    }
    __syncthreads();
    // (the partials are read with agent-scope sc1 loads, which bypass this CU's L1: no
    // acquire instruction is needed for them; the compiler fence keeps them below the count)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (last && j < 64) {  // agent-scope loads read the partials past the (per-XCD) L2
      float t = 0.f;
      for (int q = j; q < a.nblk; q += 64)
        t = __fadd_rn(t, __hip_atomic_load(a.partials + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) t = __fadd_rn(t, __shfl_xor(t, off));
      if (j == 0) {
        a.norm_out[0] = t;
        a.norm_out[1] = (float)sqrt((double)t);  // correctly rounded (p = 53 >= 2*24 + 2)
        __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

int64_t blocks_of(const fjtree_leaves* t, int32_t* blk0) {
  int64_t nb = 0;
  for (int l = 0; l < t->L; ++l) {
    if (blk0) blk0[l] = (int32_t)nb;
    nb += (t->n[l] + kChunk - 1) / kChunk;
  }
  // entries past the last leaf never count (see k_leaves); blk0[L] == nb is not read
  if (blk0)
    for (int l = t->L; l <= FJTREE_MAX_LEAVES; ++l) blk0[l] = INT32_MAX;
  return nb;
}

int validate(const fjtree_leaves* t) {
  if (!t) return fail(FJAGG_EINVAL, "null table");
  if (t->K < 1 || t->K > FJTREE_MAX_OPERANDS) return fail(FJAGG_EINVAL, "K must be 1 or 2, got %d", t->K);
  if (t->L < 1 || t->L > FJTREE_MAX_LEAVES)
    return fail(FJAGG_EINVAL, "L must be in [1, %d], got %d", FJTREE_MAX_LEAVES, t->L);
  if (t->flags & ~(FJAGG_SCALE | FJTREE_NORM | FJTREE_NO_OUT | FJTREE_ORDERED))
    return fail(FJAGG_EINVAL, "unknown flags");
  const bool norm = t->flags & FJTREE_NORM, out = !(t->flags & FJTREE_NO_OUT);
  if (!norm && !out) return fail(FJAGG_EINVAL, "FJTREE_NO_OUT needs FJTREE_NORM");
  if (!out && (t->K != 1 || t->norm_operand != 0)) return fail(FJAGG_EINVAL, "FJTREE_NO_OUT takes K = 1");
  if (norm && (t->norm_operand < 0 || t->norm_operand >= t->K || !t->norm_out || !t->ws))
    return fail(FJAGG_EINVAL, "FJTREE_NORM needs norm_operand < K, norm_out and ws");
  for (int l = 0; l < t->L; ++l) {
    if (t->n[l] < 0) return fail(FJAGG_EINVAL, "leaf %d: negative size", l);
    if (!t->n[l]) continue;
    for (int k = 0; k < t->K; ++k)
      if (!t->x[k][l]) return fail(FJAGG_EINVAL, "leaf %d: null operand %d", l, k);
    if (out && !t->out[l]) return fail(FJAGG_EINVAL, "leaf %d: null output", l);
  }
  if (blocks_of(t, nullptr) > INT32_MAX) return fail(FJAGG_EINVAL, "too many elements");
  return FJAGG_OK;
}

template <int K, bool OUT, bool NORM>
int launch(const Args& a, hipStream_t s) {
  hipLaunchKernelGGL((k_leaves<K, OUT, NORM>), dim3(a.nblk), dim3(kThreads), 0, s, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? FJAGG_OK : fail(FJAGG_EHIP, "k_leaves: %s", hipGetErrorString(e));
}

// The lazy norms' fill (fjtree_norms_fill): sq[i] = l2sq[i], nrm[i] = sqrt(l2sq[i]), the square
// root correctly rounded (IEEE binary32, as jnp.sqrt on XLA:CPU; tree_util.py:112-114).
__global__ void k_norms_fill(const float* __restrict__ l2sq, float* __restrict__ sq, float* __restrict__ nrm,
                             int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) {
    const float v = l2sq[i];
    sq[i] = v;
    nrm[i] = (float)sqrt((double)v);  // correctly rounded (p = 53 >= 2*24 + 2); __fsqrt_rn is 1 ulp off at times
  }
}

}  // namespace

extern "C" {

int fjtree_abi_version(void) { return FJTREE_ABI_VERSION; }

int fjtree_norms_fill(const float* l2sq, float* sq_out, float* norm_out, int64_t n, void* stream) {
  fjagg_g_err[0] = 0;
  if (n < 0 || n > (int64_t(1) << 30)) return fail(FJAGG_EINVAL, "norms_fill: n = %lld", (long long)n);
  if (n == 0) return FJAGG_OK;
  if (!l2sq || !sq_out || !norm_out) return fail(FJAGG_EINVAL, "norms_fill: null pointer");
  const unsigned blocks = static_cast<unsigned>((n + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(k_norms_fill, dim3(blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), l2sq,
                     sq_out, norm_out, n);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? FJAGG_OK : fail(FJAGG_EHIP, "k_norms_fill: %s", hipGetErrorString(e));
}

int64_t fjtree_workspace_bytes(const fjtree_leaves* t) {
  if (!t || !(t->flags & FJTREE_NORM) || t->L < 1 || t->L > FJTREE_MAX_LEAVES) return 0;
  int64_t nb = blocks_of(t, nullptr);
  return kWsHeader + 4 * (nb > 0 ? nb : 1);
}

int fjtree_fold_leaves(const fjtree_leaves* t, void* stream) {
  fjagg_g_err[0] = 0;
  if (int rc = validate(t)) return rc;
  const bool norm = t->flags & FJTREE_NORM, out = !(t->flags & FJTREE_NO_OUT);
  Args a;
  memset(&a, 0, sizeof(a));
  const int64_t nb = blocks_of(t, a.blk0);
  if (nb == 0 && !norm) return FJAGG_OK;  // only empty leaves
  a.nblk = (int)(nb > 0 ? nb : 1);         // a norm of empty leaves still writes {0, 0}
  if (norm && t->ws_bytes < kWsHeader + 4 * (int64_t)a.nblk)
    return fail(FJAGG_EINVAL, "workspace of %lld bytes < %lld", (long long)t->ws_bytes,
                (long long)(kWsHeader + 4 * (int64_t)a.nblk));
  a.L = t->L;
  for (int l = 0; l < t->L; ++l) {
    uintptr_t bits = 0;
    for (int k = 0; k < t->K; ++k) {
      a.x[k][l] = t->x[k][l];
      bits |= reinterpret_cast<uintptr_t>(t->x[k][l]);
    }
    if (out) {
      a.out[l] = t->out[l];
      bits |= reinterpret_cast<uintptr_t>(t->out[l]);
    }
    a.n[l] = t->n[l];
    if ((bits & 15) == 0) a.vec_mask |= 1ull << l;
  }
  for (int k = 0; k < t->K; ++k) a.w[k] = t->w[k];
  a.scale = t->scale;
  a.scale_on = (t->flags & FJAGG_SCALE) != 0;
  a.norm_operand = t->norm_operand;
  a.ordered = (t->flags & FJTREE_ORDERED) != 0;
  a.norm_out = t->norm_out;
  if (norm) {
    a.counter = reinterpret_cast<unsigned*>(t->ws);
    a.partials = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(t->ws) + kWsHeader);
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!out) return launch<1, false, true>(a, s);
  if (t->K == 1) return norm ? launch<1, true, true>(a, s) : launch<1, true, false>(a, s);
  return norm ? launch<2, true, true>(a, s) : launch<2, true, false>(a, s);
}

}  // extern "C"
