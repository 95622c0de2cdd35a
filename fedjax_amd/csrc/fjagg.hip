// fjagg.hip — MI355X (gfx950) kernels and C ABI for FedJAX's client-delta aggregation.
//
// The hot path is the weighted fold of tree_mean (fedjax/core/tree_util.py:76-96):
// for every parameter element p, s = sum_k fl(x_k[p] * w_k) in client order, then
// y[p] = fl(s * f32(1/W)). It is a streaming reduction over K*P input bytes with
// 2 flops per element read: HBM-bound, no MFMA. Design:
//
//   * one lane owns E "units" of 16 bytes (4 f32 / 8 bf16) of the parameter axis and
//     walks all K clients in order, so the fold is the reference's exact sequence
//     (no cross-lane reduction, no FMA: compiled with -ffp-contract=off);
//   * each client row is read through a buffer descriptor built on the scalar unit
//     (SGPRs) with a loop-invariant 32-bit lane offset: no address VGPRs per load,
//     range-checked rows;
//   * U clients are loaded before they are folded, giving E*U 16-byte loads in
//     flight per lane (latency hiding through MLP, not through LDS: no reuse);
//   * the grid is "balanced": the same number of workgroups on every CU, each with
//     an equal contiguous share of the parameter axis (no tail of late workgroups);
//   * element tails and unaligned leaves use the same body with 1-element units;
//   * the pytree path walks a device-resident (client, leaf) pointer table with a
//     workgroup table of unit ranges, so ONE launch covers every leaf of every client;
//   * epilogue variants: per-client l2 norms accumulated during the same pass
//     (k_dense_l2), and the server optimizer step consuming the mean in registers
//     (k_dense_opt);
//   * FJAGG_MODE_SPLIT splits the client axis over blockIdx.y for shapes whose
//     parameter axis cannot fill 256 CUs, and combines the range sums in order;
//   * FJAGG_HOST_TABLES: the weights (dense) or the whole plan image + weights
//     (pytree) travel in the kernel arguments instead of a pinned upload in front of
//     the fold on the stream (a blit kernel and its dependency, ~5-10 us per call).
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <cstring>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "fjagg.h"
#include "fjagg_dev.h"

// Shared with fjcomp.hip (same library): the thread-local message behind fjagg_last_error().
__attribute__((visibility("hidden"))) thread_local char fjagg_g_err[512] = "";

namespace {

// ------------------------------------------------------------- fused l2 hooks
// Per-client sum of squares accumulated during the fold (fjagg_wsum_l2_*). The
// reference's norm is an XLA reduction (tree_util.py:105-114) whose order is not
// pinned, so this one is free to pick the cheapest fixed order (deterministic; the
// tests bound it against an f64 norm):
//   * each lane accumulates its units' squares of client k with packed FMAs into a
//     float2 (lanes of invalid units load zeros, fold() points them past the row);
//   * a group of N clients is reduced across the wave together, in registers, with
//     no LDS round trip: v_permlane32_swap halves the lanes and pairs clients
//     (q0 | q2), v_permlane16_swap pairs the rows (one client per 16-lane row), and
//     four DPP row rotations finish each row's sum (row c holds client c);
//   * lane 16c adds client k+c's total to its wave's LDS slot [wave][k+c].
// The plain fold instantiates NoNorm: nothing of this is emitted.
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float swap32_sum(float a, float b) {  // [a.lo+a.hi | b.lo+b.hi]
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __fadd_rn(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// rows r0..r3 of 16 lanes: [a.r0+a.r1, b.r0+b.r1, a.r2+a.r3, b.r2+b.r3]
__device__ __forceinline__ float swap16_sum(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __fadd_rn(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {  // v + v[DPP CTRL]
  return __fadd_rn(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false)));
}
__device__ __forceinline__ float row16_sum(float v) {  // every lane: the sum of its 16-lane row
  v = dpp_add<0x128>(v);  // row_ror:8
  v = dpp_add<0x124>(v);  // row_ror:4
  v = dpp_add<0x122>(v);  // row_ror:2
  return dpp_add<0x121>(v);  // row_ror:1
}

struct NoNorm {
  static constexpr bool kOn = false;
  template <int N>
  __device__ __forceinline__ void commit(const f32x2 (&)[N], int64_t) {}
};
struct LdsNorm {
  static constexpr bool kOn = true;
  float* slot;  // this wave's K floats in LDS
  // clients k .. k+N-1 (N = 1, 2, 4 or 8): lane partials -> the wave's LDS slots
  template <int N>
  __device__ __forceinline__ void commit(const f32x2 (&q2)[N], int64_t k) {
    static_assert(N == 1 || N == 2 || N == 4 || N == 8, "LdsNorm::commit reduces groups of 1, 2, 4 or 8 clients");
    const int lane = threadIdx.x & 63;
    if constexpr (N == 8) {
      const f32x2 a[4] = {q2[0], q2[1], q2[2], q2[3]}, b[4] = {q2[4], q2[5], q2[6], q2[7]};
      commit<4>(a, k);
      commit<4>(b, k + 4);
    } else {
      float q[N];
#pragma unroll
      for (int i = 0; i < N; ++i) q[i] = __fadd_rn(q2[i].x, q2[i].y);
      float v;
      if constexpr (N == 4) {
        v = row16_sum(swap16_sum(swap32_sum(q[0], q[2]), swap32_sum(q[1], q[3])));  // row c: client c
      } else if constexpr (N == 2) {
        const float h = swap32_sum(q[0], q[1]);  // lanes 0-31: client 0, 32-63: client 1
        v = row16_sum(swap16_sum(h, h));          // rows 0, 1: client 0; rows 2, 3: client 1
      } else {
        const float h = swap32_sum(q[0], q[0]);
        v = row16_sum(swap16_sum(h, h));  // every row: the client
      }
      constexpr int kStep = 64 / N;  // lane holding client c: c * kStep
      if ((lane & (kStep - 1)) == 0) {
        float* s = slot + k + lane / kStep;
        *s = __fadd_rn(*s, v);
      }
    }
  }
};

// a lane's squares of one unit into its client's packed accumulator
template <class T, int V>
__device__ __forceinline__ void sq_acc(const T (&t)[V], f32x2& q) {
  if constexpr (V == 1) {
    q.x = __builtin_fmaf((float)t[0], (float)t[0], q.x);
  } else {
#pragma unroll
    for (int i = 0; i < V; i += 2) {
      const f32x2 p = {(float)t[i], (float)t[i + 1]};
      q = __builtin_elementwise_fma(p, p, q);
    }
  }
}

// ----------------------------------------------------------------- epilogues
// PlainEpi: the fold's result goes to the output (tree_mean). OptEpi: the mean
// y = fl(s * scale) feeds the server optimizer step of the round in registers
// (optax sgd / trace / adam op sequence, fedjax/core/optimizers.py:57-66,148-178,
// 227-250) and only the updated params and optimizer state are written.
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float sqrt_rn(float a) { return (float)__dsqrt_rn((double)a); }
// jax.lax.rsqrt restated as 1 / sqrt evaluated in f64 (each op correctly rounded) and
// rounded once to f32 (XLA's own rsqrt is not pinned by any reference test)
__device__ __forceinline__ float rsqrt_rn(float a) { return (float)__ddiv_rn(1.0, __dsqrt_rn((double)a)); }
// jnp.sign: -1 / 0 / +1, NaN stays NaN
__device__ __forceinline__ float xla_sign(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : x); }

struct PlainEpi {};
struct OptEpi {
  fjagg_server_opt o;
  float* __restrict__ params;
  float* __restrict__ m;
  float* __restrict__ v;
  float* __restrict__ mean;  // optional: also store the mean (diagnostics)
  __device__ __forceinline__ void apply(int64_t e, float g) const {
    if (mean) mean[e] = g;
    float p = params[e], u;
    if (o.kind == FJAGG_OPT_SGD) {
      u = g;
    } else if (o.kind == FJAGG_OPT_MOMENTUM) {  // optax.trace: g + decay * t
      const float t = __fadd_rn(g, __fmul_rn(o.decay, m[e]));
      m[e] = t;
      u = o.nesterov ? __fadd_rn(g, __fmul_rn(o.decay, t)) : t;
    } else if (o.kind == FJAGG_OPT_ADAM) {  // optax.scale_by_adam
      const float mu = __fadd_rn(__fmul_rn(o.one_minus_b1, g), __fmul_rn(o.b1, m[e]));
      const float nu = __fadd_rn(__fmul_rn(o.one_minus_b2, __fmul_rn(g, g)), __fmul_rn(o.b2, v[e]));
      m[e] = mu;
      v[e] = nu;
      // f32 div / sqrt evaluated in f64 and rounded once: correctly rounded (53 >=
      // 2*24 + 2, double rounding is innocuous), as IEEE binary32 div/sqrt must be.
      const float mh = div_rn(mu, o.bc1), nh = div_rn(nu, o.bc2);
      u = div_rn(mh, __fadd_rn(sqrt_rn(__fadd_rn(nh, o.eps_root)), o.eps));
    } else if (o.kind == FJAGG_OPT_ADAGRAD) {  // optax.scale_by_rss
      const float ss = __fadd_rn(__fmul_rn(g, g), v[e]);
      v[e] = ss;
      u = __fmul_rn(ss > 0.0f ? rsqrt_rn(__fadd_rn(ss, o.eps)) : 0.0f, g);
    } else if (o.kind == FJAGG_OPT_RMSPROP) {  // optax.rmsprop: scale_by_rms | scale_by_stddev, lr, [trace]
      const float nu = __fadd_rn(__fmul_rn(o.one_minus_b2, __fmul_rn(g, g)), __fmul_rn(o.b2, v[e]));
      v[e] = nu;
      float den = nu;
      if (o.flags & FJAGG_OPT_F_CENTERED) {  // scale_by_stddev: mu = (1 - decay) g + decay mu
        const float mu = __fadd_rn(__fmul_rn(o.one_minus_b2, g), __fmul_rn(o.b2, m[e]));
        m[e] = mu;
        den = __fsub_rn(nu, __fmul_rn(mu, mu));
      }
      u = __fmul_rn(g, rsqrt_rn(__fadd_rn(den, o.eps)));
      if (o.flags & FJAGG_OPT_F_MOMENTUM) {  // the trace follows scale_by_learning_rate in this chain
        const float s = __fmul_rn(o.neg_lr, u);
        const float t = __fadd_rn(s, __fmul_rn(o.decay, m[e]));
        m[e] = t;
        params[e] = __fadd_rn(p, o.nesterov ? __fadd_rn(s, __fmul_rn(o.decay, t)) : t);
        return;
      }
    } else {  // optax.scale_by_yogi: nu - (1 - b2) * sign(nu - g^2) * g^2, no bias correction
      const float mu = __fadd_rn(__fmul_rn(o.one_minus_b1, g), __fmul_rn(o.b1, m[e]));
      const float g2 = __fmul_rn(g, g), nv = v[e];
      const float nu = __fsub_rn(nv, __fmul_rn(__fmul_rn(o.one_minus_b2, xla_sign(__fsub_rn(nv, g2))), g2));
      m[e] = mu;
      v[e] = nu;
      u = div_rn(mu, __fadd_rn(sqrt_rn(__fadd_rn(nu, o.eps_root)), o.eps));
    }
    params[e] = __fadd_rn(p, __fmul_rn(o.neg_lr, u));  // scale_by_learning_rate, apply_updates
  }
};

// ------------------------------------------------------------------ fold body
// Each lane folds E units; unit j of this lane sits at byte offset off[j] of every
// client row (a 32-bit lane constant) and is written to outp[j]. row(k) returns the
// wave-uniform base address of client k. Clients are folded in order 0..K-1.
// The output of the unit at input byte offset off is at obase + off / sizeof(IN) *
// sizeof(OUT) (same element index); valid[j] == false skips unit j's store.
template <int IN, class ACC, int OUT, int V, int E, int U, bool NT, bool BURST = true, class RowFn,
          class NORM = NoNorm, class EPI = PlainEpi>
__device__ __forceinline__ void fold(RowFn row, uint32_t row_bytes, int64_t K,
                                     const uint32_t (&off)[E],
                                     uint8_t* __restrict__ obase, const bool (&valid)[E],
                                     const typename ACC::T* __restrict__ w, bool do_scale,
                                     float scale, bool accumulate, NORM nrm = NORM(),
                                     const EPI& epi = EPI()) {
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B;
  auto outp = [&](int j) { return obase + (size_t)(off[j] / IB) * OB; };
  using T = typename ACC::T;
  using Raw = typename Unit<IN, V>::Raw;
  // With norms, loads of an invalid unit (a lane past its range) point past every row
  // descriptor's range, so they read zeros without touching memory: the unit's store is
  // skipped, and the squares need no masking. outp() keeps the caller's in-bounds offset.
  // (The plain fold keeps the caller's clamped offsets: its code is unchanged.)
  uint32_t loff[E];
#pragma unroll
  for (int j = 0; j < E; ++j) loff[j] = (!NORM::kOn || valid[j]) ? off[j] : 0x80000000u;
  T acc[E][V];
  {  // client 0: s_0 = t_0 (tree_util.py:89-91) or out + t_0 (running sum)
    const auto r = row_rsrc(row(0), row_bytes);
    Raw v[E];
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = load_unit<IN, V, NT>(r, loff[j]);
    const T w0 = ACC::weight(w[0]);
    f32x2 q[1] = {{0.f, 0.f}};
#pragma unroll
    for (int j = 0; j < E; ++j) {
      T t[V];
      decode<IN, ACC, V>(v[j], t);
      if constexpr (NORM::kOn) sq_acc<T, V>(t, q[0]);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[j][i] = ACC::mul(t[i], w0);
    }
    nrm.template commit<1>(q, 0);
    if (accumulate) {
#pragma unroll
      for (int j = 0; j < E; ++j) {
        unsigned b[V];
        load_out_unit<OUT, V>(outp(j), b);
#pragma unroll
        for (int i = 0; i < V; ++i) acc[j][i] = ACC::add(init_from<OUT, ACC>(b[i]), acc[j][i]);
      }
    }
  }
  int64_t k = 1;
  // Row bases of the next group are fetched while this group's loads are in flight:
  // on the pytree path row(k) is a scalar load from the pointer table, and fetching
  // it at the top of each group would leave the vector memory pipe idle for that
  // latency once per group. Clamped to K-1 so the table is never read past its end.
  const uint8_t* nxt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) nxt[u] = row(k + u < K ? k + u : K - 1);
  for (; k + U <= K; k += U) {
    Raw v[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const auto r = row_rsrc(nxt[u], row_bytes);
#pragma unroll
      for (int j = 0; j < E; ++j) v[u][j] = load_unit<IN, V, NT>(r, loff[j]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t kn = k + U + u;
      nxt[u] = row(kn < K ? kn : K - 1);
    }
    // BURST (default): every load of the group is issued before the first is consumed
    // (E*U in flight per lane); otherwise the scheduler interleaves loads and folds. Burst
    // is faster with one workgroup per CU, interleaved with two or more full tiles per CU
    // (k_dense picks per launch, launch_dense_v).
    if constexpr (BURST) __builtin_amdgcn_sched_barrier(0);
    f32x2 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = f32x2{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const T wk = ACC::weight(w[k + u]);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        T t[V];
        decode<IN, ACC, V>(v[u][j], t);
        if constexpr (NORM::kOn) sq_acc<T, V>(t, q[u]);
#pragma unroll
        for (int i = 0; i < V; ++i) acc[j][i] = ACC::add(acc[j][i], ACC::mul(t[i], wk));
      }
    }
    nrm.template commit<U>(q, k);
  }
  for (; k < K; ++k) {
    const auto r = row_rsrc(row(k), row_bytes);
    const T wk = ACC::weight(w[k]);
    f32x2 q[1] = {{0.f, 0.f}};
#pragma unroll
    for (int j = 0; j < E; ++j) {
      T t[V];
      decode<IN, ACC, V>(load_unit<IN, V, NT>(r, loff[j]), t);
      if constexpr (NORM::kOn) sq_acc<T, V>(t, q[0]);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[j][i] = ACC::add(acc[j][i], ACC::mul(t[i], wk));
    }
    nrm.template commit<1>(q, k);
  }
#pragma unroll
  for (int j = 0; j < E; ++j) {
    if (!valid[j]) continue;
    if constexpr (std::is_same<EPI, OptEpi>::value) {
      const int64_t e0 = off[j] / IB;
#pragma unroll
      for (int i = 0; i < V; ++i) epi.apply(e0 + i, __uint_as_float(finish<FJAGG_F32, ACC>(acc[j][i], do_scale, scale)));
    } else {
      unsigned b[V];
#pragma unroll
      for (int i = 0; i < V; ++i) b[i] = finish<OUT, ACC>(acc[j][i], do_scale, scale);
      store_unit<OUT, V>(outp(j), b);
    }
  }
}

// Dense slab: client k at x + k*ld_bytes; P = nunits*V + tail_n elements.
// Block 0 folds the tail (if any) with 1-element units. Every other block owns the
// contiguous unit range [b*S, min((b+1)*S, nunits)) and walks it in groups of
// kThreads*E units (lane tid takes units g + j*kThreads + tid), folding all clients
// of a group before moving on. The host sizes S so that the grid is one resident
// wave of workgroups with equal byte shares ("balanced"), or S = kThreads*E for the
// classic one-tile-per-block launch.
// blockIdx.y selects a client range [y*kchunk, min(K, (y+1)*kchunk)) and writes to
// out + y*out_ystride_bytes (FJAGG_MODE_SPLIT); exact mode has gridDim.y == 1.
// MINW > 0 asks for MINW waves per SIMD (caps VGPRs: 8 -> 64 registers).
// WK > 0: the weights are kw.w (FJAGG_HOST_TABLES), not w.
template <int IN, class ACC, int OUT, int V, int E, int U, bool NT, int MINW, bool BURST = false, int WK = 0>
__global__ __launch_bounds__(kThreads, MINW) void k_dense(
    const uint8_t* __restrict__ x, int64_t ld_bytes, int64_t K, int64_t nunits, int tail_n,
    const typename ACC::T* __restrict__ w, float scale, int do_scale, int accumulate,
    uint8_t* __restrict__ out, int64_t kchunk, int64_t out_ystride_bytes, int64_t S,
    const KargF32<(WK > 0 ? WK : 1)> kw) {
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B;
  const int tid = threadIdx.x;
  const int64_t k0 = (int64_t)blockIdx.y * kchunk;
  const int64_t kn = (K - k0 < kchunk) ? (K - k0) : kchunk;
  const uint8_t* xb = x + k0 * ld_bytes;
  const typename ACC::T* wb = (WK > 0 ? reinterpret_cast<const typename ACC::T*>(kw.w) : w) + k0;
  uint8_t* ob = out + (int64_t)blockIdx.y * out_ystride_bytes;
  auto row = [=](int64_t k) { return xb + k * ld_bytes; };
  const uint32_t row_bytes = (uint32_t)((nunits * V + tail_n) * IB);
  int64_t b = blockIdx.x;
  if (tail_n > 0) {
    if (b == 0) {
      if (tid < tail_n) {
        const int64_t e = nunits * V + tid;
        const uint32_t off[1] = {(uint32_t)(e * IB)};
        const bool valid[1] = {true};
        fold<IN, ACC, OUT, 1, 1, U, NT>(row, row_bytes, kn, off, ob, valid, wb, do_scale != 0,
                                        scale, accumulate != 0);
      }
      return;
    }
    b -= 1;
  }
  const int64_t u_begin = b * S;
  const int64_t u_end = (u_begin + S < nunits) ? u_begin + S : nunits;
  for (int64_t g = u_begin; g < u_end; g += (int64_t)kThreads * E) {
    uint32_t off[E];
    bool valid[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
      int64_t u = g + j * kThreads + tid;
      valid[j] = u < u_end;
      if (!valid[j]) u = u_end - 1;  // keep the load in bounds; the store is skipped
      off[j] = (uint32_t)(u * (V * IB));
    }
    fold<IN, ACC, OUT, V, E, U, NT, BURST>(row, row_bytes, kn, off, ob, valid, wb, do_scale != 0,
                                           scale, accumulate != 0);
  }
}

// Where the combined norms go: operand k >= first gets its squared norm in sq[k - first] and,
// when nrm is set, its correctly rounded square root in nrm[k - first] (IEEE binary32 sqrt, as
// jnp.sqrt: tree_util.py:111-114). fjagg_wsum_l2_*: {l2sq, nullptr, 0}; fjagg_wsum_l2_ptrs_rows:
// a deferred running sum's two norm rows, skipping operand 0 (its base). done: the completion
// counter of a FJAGG_ZEROED_WS workspace when the fold's last workgroup combines (combine_last),
// nullptr when k_l2_combine does.
struct L2Out {
  float* sq;
  float* nrm;
  int64_t first;
  unsigned* done;
};
constexpr int kCombineWaves = 16, kCombineBatch = 16;
// The last-workgroup combine serves K <= kFusedCombineMax: partial rows padded to K4 =
// round_up(K, 4) floats (float4 columns: 16 x K4/4 column sums over 256 lanes, at most two
// per lane; the pad columns are summed and never written). Above that one workgroup would
// issue too many dependent loads and k_l2_combine's wider grid wins.
constexpr int64_t kFusedCombineMax = 128;
__host__ __device__ __forceinline__ int64_t round4(int64_t K) { return (K + 3) & ~(int64_t)3; }

__device__ __forceinline__ void write_norm(const L2Out& out, int64_t k, float t) {
  if (k < out.first) return;
  if (out.sq) out.sq[k - out.first] = t;
  if (out.nrm) out.nrm[k - out.first] = sqrt_rn(t);  // (__fsqrt_rn measured 1 ulp off on gfx950)
}

// The completion hand-off of a fused-norm fold whose last workgroup combines (the counter form
// of the HIP guide's inter-workgroup recipe, no fences): every workgroup stores its partial row
// write-through (sc1, 4 B per lane), every storing wave drains its stores, the workgroup
// barrier, then ONE lane adds 1 to the agent-scope counter; the workgroup whose add returns
// nb - 1 is last, and reads every row with sc1 loads only (they bypass this CU's L1, so no
// acquire is needed), adds them and re-arms the counter at 0. That is the guide's measured form for
// one workgroup of the launch per CU (not an architectural guarantee): the launchers keep the grid
// to one wave of workgroups and reserve more than half a CU's LDS per workgroup (l2_smem), so two
// cannot share a CU. lds: 16 x K4 floats + the flag.
// The sum order is k_l2_combine's exactly (column wv of 16 adds partials b = wv, wv+16, ... in
// order from +0, then the 16 column sums in wv order): bitwise the two-launch norms.
__device__ __forceinline__ void combine_last(const float* __restrict__ ws, int64_t K, const L2Out& out,
                                             float* lds) {
  const int tid = threadIdx.x;
  const int64_t nb = gridDim.x, K4 = round4(K), q = K4 / 4;
  unsigned* last = reinterpret_cast<unsigned*>(lds + kCombineWaves * K4);  // in the one dynamic LDS array
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 partials are out
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(out.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a counter that was not zero at the call (a caller that did not zero it, fjagg.h): the word
    // after it records that this call's norms are not valid (sticky; the caller clears it)
    if (old >= (unsigned)nb) __hip_atomic_fetch_or(out.done + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = old == (unsigned)(nb - 1);
  }
  __syncthreads();
  if (!*last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below)
  const auto r = row_rsrc(reinterpret_cast<const uint8_t*>(ws), row_range(nb * K4 * 4));
  auto add4 = [](float4& s, const u32x4& v) {
    s.x = __fadd_rn(s.x, __uint_as_float(v[0]));
    s.y = __fadd_rn(s.y, __uint_as_float(v[1]));
    s.z = __fadd_rn(s.z, __uint_as_float(v[2]));
    s.w = __fadd_rn(s.w, __uint_as_float(v[3]));
  };
  const int qi = (int)q;
  if (nb <= kCombineWaves * kCombineBatch) {
    // the launchers keep nb <= the CU count, so one batch of 16 rows per column: a lane's (at most
    // two) columns have all their loads in flight together — one memory round trip for any K <= 128
    constexpr int kCols = (kCombineWaves * kFusedCombineMax / 4 + kThreads - 1) / kThreads;
    int wv[kCols], c[kCols];
#pragma unroll
    for (int j = 0; j < kCols; ++j) {
      const int p = tid + j * kThreads;
      wv[j] = p < kCombineWaves * qi ? p / qi : -1;
      c[j] = wv[j] >= 0 ? p - wv[j] * qi : 0;
    }
    u32x4 a[kCols][kCombineBatch];
#pragma unroll
    for (int j = 0; j < kCols; ++j)
#pragma unroll
      for (int i = 0; i < kCombineBatch; ++i) {  // rows past nb, and idle lanes, lie past the range: zeros
        const int b = wv[j] + i * kCombineWaves;
        const uint32_t off = wv[j] >= 0 ? (uint32_t)((b * qi + c[j]) * 16) : 0x80000000u;
        a[j][i] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);  // aux 16 = sc1
      }
#pragma unroll
    for (int j = 0; j < kCols; ++j) {
      if (wv[j] < 0) continue;
      float4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < kCombineBatch; ++i) add4(s, a[j][i]);
      reinterpret_cast<float4*>(lds + wv[j] * K4)[c[j]] = s;
    }
  } else {
    for (int p = tid; p < kCombineWaves * qi; p += kThreads) {
      const int wv = p / qi, c = p - wv * qi;
      float4 s = {0.f, 0.f, 0.f, 0.f};
      for (int64_t b0 = wv; b0 < nb; b0 += (int64_t)kCombineWaves * kCombineBatch) {
        u32x4 a[kCombineBatch];
#pragma unroll
        for (int i = 0; i < kCombineBatch; ++i) {
          const int64_t b = b0 + (int64_t)i * kCombineWaves;
          a[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)((b * qi + c) * 16), 0, 16);
        }
#pragma unroll
        for (int i = 0; i < kCombineBatch; ++i) add4(s, a[i]);
      }
      reinterpret_cast<float4*>(lds + wv * K4)[c] = s;
    }
  }
  __syncthreads();
  for (int64_t k = tid; k < K; k += kThreads) {
    float t = lds[k];
#pragma unroll
    for (int i = 1; i < kCombineWaves; ++i) t = __fadd_rn(t, lds[i * K4 + k]);
    write_norm(out, k, t);
  }
  if (tid == 0) __hip_atomic_store(out.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A fused-norm workgroup's epilogue: its (kThreads/64) wave rows of LDS norms -> the partial
// row ws[b*ld + k] (ld = K; with a completion counter ld = round4(K), sc1 stores, then the
// last-workgroup combine).
__device__ __forceinline__ void l2_epilogue(float* l2lds, float* __restrict__ ws, int64_t K, const L2Out& out,
                                            int64_t row) {
  __syncthreads();
  if (out.done) {
    const int64_t ld = round4(K);
    for (int64_t k = threadIdx.x; k < K; k += kThreads) {
      float t = l2lds[k];
#pragma unroll
      for (int i = 1; i < kThreads / 64; ++i) t = __fadd_rn(t, l2lds[i * K + k]);
      __hip_atomic_store(reinterpret_cast<unsigned*>(ws) + row * ld + k, __float_as_uint(t),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through (sc1)
    }
    combine_last(ws, K, out, l2lds);  // (its first barrier also ends the reads of l2lds above)
    return;
  }
  for (int64_t k = threadIdx.x; k < K; k += kThreads) {
    float t = l2lds[k];
#pragma unroll
    for (int i = 1; i < kThreads / 64; ++i) t = __fadd_rn(t, l2lds[i * K + k]);
    ws[row * K + k] = t;
  }
}

// k_dense + per-client squared norms (exact mode, float fold). Dynamic LDS holds
// (kThreads/64) x K floats (16 x K with a completion counter); block b writes its
// per-client partials to ws[b*K + k], added in block order by the last workgroup
// (combine_last) or by k_l2_combine.
template <int IN, int OUT, int V, int E, int U, bool NT>
__global__ __launch_bounds__(kThreads) void k_dense_l2(
    const uint8_t* __restrict__ x, int64_t ld_bytes, int64_t K, int64_t nunits, int tail_n,
    const float* __restrict__ w, float scale, int do_scale, int accumulate,
    uint8_t* __restrict__ out, int64_t S, float* __restrict__ ws, const L2Out l2out) {
  extern __shared__ __attribute__((aligned(16))) float l2lds[];
  constexpr int IB = Elem<IN>::B;
  const int tid = threadIdx.x;
  for (int64_t i = tid; i < (kThreads / 64) * K; i += kThreads) l2lds[i] = 0.f;
  __syncthreads();
  LdsNorm nrm{l2lds + (tid >> 6) * K};
  auto row = [=](int64_t k) { return x + k * ld_bytes; };
  const uint32_t row_bytes = (uint32_t)((nunits * V + tail_n) * IB);
  int64_t b = blockIdx.x;
  bool is_tail = false;
  if (tail_n > 0) {
    if (b == 0) {
      is_tail = true;
      const bool active = tid < tail_n;  // every lane joins the wave reductions
      const int64_t e = nunits * V + (active ? tid : 0);
      const uint32_t off[1] = {(uint32_t)(e * IB)};
      const bool valid[1] = {active};
      fold<IN, AccF, OUT, 1, 1, U, NT>(row, row_bytes, K, off, out, valid, w, do_scale != 0,
                                       scale, accumulate != 0, nrm);
    }
    b -= 1;
  }
  if (!is_tail) {
    const int64_t u_begin = b * S;
    const int64_t u_end = (u_begin + S < nunits) ? u_begin + S : nunits;
    for (int64_t g = u_begin; g < u_end; g += (int64_t)kThreads * E) {
      uint32_t off[E];
      bool valid[E];
#pragma unroll
      for (int j = 0; j < E; ++j) {
        int64_t u = g + j * kThreads + tid;
        valid[j] = u < u_end;
        if (!valid[j]) u = u_end - 1;
        off[j] = (uint32_t)(u * (V * IB));
      }
      fold<IN, AccF, OUT, V, E, U, NT>(row, row_bytes, K, off, out, valid, w, do_scale != 0,
                                       scale, accumulate != 0, nrm);
    }
  }
  l2_epilogue(l2lds, ws, K, l2out, blockIdx.x);
}

// out[k] = sum over b of ws[b*K + k]. Workgroup = 64 clients x 16 waves: wave w sums
// partials b = w, w+16, ... in that order (coalesced 256-B rows), then the 16 wave sums
// are added in wave order: deterministic. The kernel runs after the fold, on a few
// workgroups, so it is latency-bound: each lane issues a batch of 16 loads before it adds
// any (one memory round trip per 256 partials per client; the fold's ~256 workgroups are
// one batch). Output as L2Out says (its done is unused here).
__global__ __launch_bounds__(64 * kCombineWaves) void k_l2_combine(const float* __restrict__ ws,
                                                                   int64_t nb, int64_t K, L2Out out) {
  __shared__ float part[kCombineWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t k = (int64_t)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (k < K) {
    for (int64_t b0 = wv; b0 < nb; b0 += (int64_t)kCombineWaves * kCombineBatch) {
      float a[kCombineBatch];
#pragma unroll
      for (int i = 0; i < kCombineBatch; ++i) {
        const int64_t b = b0 + (int64_t)i * kCombineWaves;
        a[i] = b < nb ? ws[b * K + k] : 0.f;
      }
      // partials are sums of squares (>= +0), so adding the +0 of an absent one keeps s
#pragma unroll
      for (int i = 0; i < kCombineBatch; ++i) s = __fadd_rn(s, a[i]);
    }
  }
  part[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && k < K) {
    float t = part[0][lane];
#pragma unroll
    for (int i = 1; i < kCombineWaves; ++i) t = __fadd_rn(t, part[i][lane]);
    write_norm(out, k, t);
  }
}

// after a fused-norm fold: nothing when its last workgroup combined (out.done), else k_l2_combine
int launch_l2_combine(const float* ws, int64_t nb, int64_t K, L2Out out, hipStream_t s) {
  if (out.done) return FJAGG_OK;
  hipLaunchKernelGGL(k_l2_combine, dim3((unsigned)((K + 63) / 64)), dim3(64 * kCombineWaves), 0, s, ws, nb, K, out);
  return check_launch("k_l2_combine");
}

// combine_last's hand-off is the guide's measured form for ONE workgroup of the launch per CU
// (MI355X_MICROARCH.md, "Valid forms", first row). A grid of at most as many workgroups as CUs
// does not make the dispatcher place them so: two may share a CU. A fold that combines in its
// last workgroup therefore reserves more than half of the CU's 160 KiB of LDS per workgroup, so
// two of its workgroups cannot share a CU whatever the placement (the plan has one wave of
// workgroups anyway). FJAGG_L2_ONE_PER_CU=0 drops the reservation (A/B runs only).
constexpr size_t kOnePerCuLds = 80 * 1024 + 16;
inline bool one_per_cu_lds() {
  static const bool on = [] {
    const char* e = getenv("FJAGG_L2_ONE_PER_CU");
    return !(e && e[0] == '0');
  }();
  return on;
}

// dynamic LDS of a fused-norm fold: the wave rows, or combine_last's 16 columns (and the
// one-workgroup-per-CU reservation). reserve = false: the bytes the code uses, which size the
// dense path's balanced grid — the reservation must not change the partition (the norms' order).
inline size_t l2_smem(int64_t K, const L2Out& out, bool reserve = true) {
  if (!out.done) return (size_t)(kThreads / 64) * K * sizeof(float);
  const size_t need = (size_t)(kCombineWaves * round4(K) + 4) * sizeof(float);
  return reserve && one_per_cu_lds() && need < kOnePerCuLds ? kOnePerCuLds : need;
}

// Lets `kern` launch with `bytes` of dynamic LDS (above the default 64 KiB: once per kernel).
int allow_lds(const void* kern, size_t bytes) {
  if (bytes <= 64 * 1024) return FJAGG_OK;
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> done;
  std::lock_guard<std::mutex> g(mu);
  auto it = done.find(kern);
  if (it != done.end() && it->second >= bytes) return FJAGG_OK;
  if (hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes)) {
    (void)hipGetLastError();
    return fail(FJAGG_EHIP, "hipFuncSetAttribute(max dynamic LDS %zu): %s", bytes, hipGetErrorString(e));
  }
  done[kern] = bytes;
  return FJAGG_OK;
}

// Exact fold of the slab + the server optimizer step in the epilogue (no mean
// round trip through HBM). Same grid/unit layout as k_dense.
template <int IN, int V, int E, int U, bool NT>
__global__ __launch_bounds__(kThreads) void k_dense_opt(
    const uint8_t* __restrict__ x, int64_t ld_bytes, int64_t K, int64_t nunits, int tail_n,
    const float* __restrict__ w, float scale, int64_t S, OptEpi epi) {
  constexpr int IB = Elem<IN>::B;
  const int tid = threadIdx.x;
  auto row = [=](int64_t k) { return x + k * ld_bytes; };
  const uint32_t row_bytes = (uint32_t)((nunits * V + tail_n) * IB);
  int64_t b = blockIdx.x;
  if (tail_n > 0) {
    if (b == 0) {
      if (tid < tail_n) {
        const uint32_t off[1] = {(uint32_t)((nunits * V + tid) * IB)};
        const bool valid[1] = {true};
        fold<IN, AccF, FJAGG_F32, 1, 1, U, NT>(row, row_bytes, K, off, nullptr, valid, w, true,
                                               scale, false, NoNorm(), epi);
      }
      return;
    }
    b -= 1;
  }
  const int64_t u_begin = b * S;
  const int64_t u_end = (u_begin + S < nunits) ? u_begin + S : nunits;
  for (int64_t g = u_begin; g < u_end; g += (int64_t)kThreads * E) {
    uint32_t off[E];
    bool valid[E];
#pragma unroll
    for (int j = 0; j < E; ++j) {
      int64_t u = g + j * kThreads + tid;
      valid[j] = u < u_end;
      if (!valid[j]) u = u_end - 1;
      off[j] = (uint32_t)(u * (V * IB));
    }
    fold<IN, AccF, FJAGG_F32, V, E, U, NT>(row, row_bytes, K, off, nullptr, valid, w, true, scale,
                                           false, NoNorm(), epi);
  }
}

// Walks the unit range [u0, u1) of one leaf (units of VV elements): in groups of
// kThreads*8 units (E=8, U=4: the dense default; lanes past the range are masked)
// when the range gives a lane more than one unit, else in groups of kThreads units
// (E=1, U=8).
template <int IN, class ACC, int OUT, int VV, bool NT, bool BURST, class RowFn, class NORM, class EPI>
__device__ __forceinline__ void walk_units(RowFn row, uint32_t row_bytes, int64_t K, int64_t u0, int64_t u1,
                                           uint8_t* ob, const typename ACC::T* __restrict__ w, bool dsc,
                                           float scale, bool acm, NORM nrm, const EPI& epi) {
  constexpr int IB = Elem<IN>::B;
  const int tid = threadIdx.x;
  if (u1 - u0 > (int64_t)kThreads) {
    for (int64_t g = u0; g < u1; g += (int64_t)kThreads * 8) {
      uint32_t off[8];
      bool valid[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int64_t u = g + j * kThreads + tid;
        valid[j] = u < u1;
        if (!valid[j]) u = u1 - 1;
        off[j] = (uint32_t)(u * (VV * IB));
      }
      fold<IN, ACC, OUT, VV, 8, 4, NT, BURST>(row, row_bytes, K, off, ob, valid, w, dsc, scale, acm, nrm, epi);
    }
    return;
  }
  for (int64_t g = u0; g < u1; g += kThreads) {
    int64_t u = g + tid;
    const bool valid[1] = {u < u1};
    if (!valid[0]) u = u1 - 1;
    const uint32_t off[1] = {(uint32_t)(u * (VV * IB))};
    fold<IN, ACC, OUT, VV, 1, 8, NT>(row, row_bytes, K, off, ob, valid, w, dsc, scale, acm, nrm, epi);
  }
}

// The plan entry of hardware workgroup h of nb when XCD x (= h % 8) takes the consecutive
// entries [x*q + min(x, r), +q + (x < r)), q = nb / 8, r = nb % 8: a permutation of [0, nb).
__device__ __forceinline__ int64_t xcd_plan_index(int64_t h, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, x = h & 7, i = h >> 3;
  return x * q + (x < r ? x : r) + i;
}

// Pytree path. image = in_ptrs[K*L] | out_ptrs[L] | leaf_n[L] | blocks[2*nblk].
// Block b: word 0 = first unit (bits 0..39) | leaf (40..61) | tail flag (62) |
// element flag (63); word 1 = end unit (exclusive). A workgroup walks its unit range
// of one leaf with walk_units. Units are V elements, or single elements when the
// element flag is set: a leaf whose client or output pointers are not 16-byte
// aligned (fjagg_ptrs_plan_leaves) takes element units without pulling the other
// leaves of the launch off the 16-byte path.
// IW > 0 (FJAGG_HOST_TABLES): the image is ki.w and the K f32 weights follow its
// blocks (word K*L + 2L + 2*nblk, nblk = gridDim.x); img_p and w_p are unused.
template <int IN, class ACC, int OUT, int V, bool NT, bool L2 = false, bool BURST = true, int IW = 0>
__global__ __launch_bounds__(kThreads) void k_ptrs(const int64_t* __restrict__ img_p, int L,
                                                   int64_t K,
                                                   const typename ACC::T* __restrict__ w_p,
                                                   float scale, int do_scale, int accumulate,
                                                   float* __restrict__ ws, const L2Out l2out,
                                                   const KargWords<(IW > 0 ? IW : 1)> ki) {
  constexpr int IB = Elem<IN>::B;
  const int tid = threadIdx.x;
  const int64_t* img = IW > 0 ? ki.w : img_p;
  const typename ACC::T* w =
      IW > 0 ? reinterpret_cast<const typename ACC::T*>(ki.w + K * L + 2 * L + 2 * (int64_t)gridDim.x) : w_p;
  const int64_t* in_ptrs = img;
  const int64_t* out_ptrs = img + K * L;
  const int64_t* leaf_n = out_ptrs + L;
  // accumulate bit 1 (FJAGG_XCD_REMAP, the launchers): workgroups are dealt round-robin over the
  // 8 XCDs, so hardware workgroup h runs on XCD h % 8; plan entry bid = xcd_plan_index(h) gives
  // each XCD a run of consecutive plan entries (neighbouring unit ranges of one leaf: the same
  // pages of every client's row in that XCD's L2 and translation caches). Each entry is folded
  // exactly as without it, and its norm partial keeps its row: the same bits.
  const int64_t bid = (accumulate & 2) ? xcd_plan_index(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  const int64_t* blk = leaf_n + L + 2 * bid;
  const int64_t be = blk[0];
  const int leaf = (int)((be >> 40) & 0x3fffff);
  const bool tail = (be >> 62) & 1;
  const bool elem = ((uint64_t)be >> 63) != 0;
  const int64_t u0 = be & ((1ll << 40) - 1);
  const int64_t u1 = blk[1];
  const int64_t n = leaf_n[leaf];
  const int64_t nunits = n / V;
  // Rebase every row at this workgroup's first element: lane offsets stay 32-bit for a
  // leaf of any size (a workgroup's range is a few MB at most).
  const int64_t e_base = tail ? nunits * V : ((V > 1 && elem) ? u0 : u0 * V);
  uint8_t* ob = reinterpret_cast<uint8_t*>(out_ptrs[leaf]) + e_base * Elem<OUT>::B;
  auto row = [=](int64_t k) { return reinterpret_cast<const uint8_t*>(in_ptrs[k * L + leaf]) + e_base * IB; };
  const uint32_t row_bytes = row_range((n - e_base) * IB);
  const bool dsc = do_scale != 0, acm = (accumulate & 1) != 0;
  // L2: per-client squared norms of this block's units, (kThreads/64) x K floats in LDS
  extern __shared__ __attribute__((aligned(16))) float l2lds[];
  using Norm = typename std::conditional<L2, LdsNorm, NoNorm>::type;
  Norm nrm{};
  if constexpr (L2) {
    for (int64_t i = tid; i < (kThreads / 64) * K; i += kThreads) l2lds[i] = 0.f;
    __syncthreads();
    nrm = LdsNorm{l2lds + (tid >> 6) * K};
  }
  if (tail) {
    const bool active = tid < n - nunits * V;
    if (L2 || active) {  // with L2 every lane joins the per-client wave reductions
      const int64_t e = active ? tid : 0;
      const uint32_t off[1] = {(uint32_t)(e * IB)};
      const bool valid[1] = {active};
      fold<IN, ACC, OUT, 1, 1, 8, NT>(row, row_bytes, K, off, ob, valid, w, dsc, scale, acm, nrm);
    }
  } else if (V > 1 && elem) {
    walk_units<IN, ACC, OUT, 1, NT, BURST>(row, row_bytes, K, 0, u1 - u0, ob, w, dsc, scale, acm, nrm, PlainEpi());
  } else {
    walk_units<IN, ACC, OUT, V, NT, BURST>(row, row_bytes, K, 0, u1 - u0, ob, w, dsc, scale, acm, nrm, PlainEpi());
  }
  if constexpr (L2) l2_epilogue(l2lds, ws, K, l2out, bid);
}

// Pytree path + server optimizer step in the epilogue (fjagg_server_update_ptrs): the
// plan image of k_ptrs with out_ptrs[L] = the params leaves; state[3L] = m | v | mean leaf
// pointers (0 where absent). Each workgroup owns one leaf's unit range, so its OptEpi
// points at that leaf's params / moments and indexes them by the element within the leaf.
template <int IN, int V, bool NT>
__global__ __launch_bounds__(kThreads) void k_ptrs_opt(const int64_t* __restrict__ img, int L, int64_t K,
                                                       const float* __restrict__ w, float scale,
                                                       fjagg_server_opt opt, const int64_t* __restrict__ state) {
  constexpr int IB = Elem<IN>::B;
  const int tid = threadIdx.x;
  const int64_t* in_ptrs = img;
  const int64_t* out_ptrs = img + K * L;
  const int64_t* leaf_n = out_ptrs + L;
  const int64_t* blk = leaf_n + L + 2 * (int64_t)blockIdx.x;
  const int64_t be = blk[0];
  const int leaf = (int)((be >> 40) & 0x3fffff);
  const bool tail = (be >> 62) & 1;
  const bool elem = ((uint64_t)be >> 63) != 0;
  const int64_t u0 = be & ((1ll << 40) - 1);
  const int64_t u1 = blk[1];
  const int64_t n = leaf_n[leaf];
  const int64_t nunits = n / V;
  // rebased at the workgroup's first element, as in k_ptrs (the epilogue's element index too)
  const int64_t e_base = tail ? nunits * V : ((V > 1 && elem) ? u0 : u0 * V);
  auto at = [=](int64_t p) { return p ? reinterpret_cast<float*>(p) + e_base : nullptr; };
  const OptEpi epi{opt, at(out_ptrs[leaf]), at(state[leaf]), at(state[L + leaf]), at(state[2 * L + leaf])};
  auto row = [=](int64_t k) { return reinterpret_cast<const uint8_t*>(in_ptrs[k * L + leaf]) + e_base * IB; };
  const uint32_t row_bytes = row_range((n - e_base) * IB);
  if (tail) {
    if (tid < n - nunits * V) {
      const uint32_t off[1] = {(uint32_t)(tid * IB)};
      const bool valid[1] = {true};
      fold<IN, AccF, FJAGG_F32, 1, 1, 8, NT>(row, row_bytes, K, off, nullptr, valid, w, true, scale, false,
                                             NoNorm(), epi);
    }
    return;
  }
  if (V > 1 && elem)
    walk_units<IN, AccF, FJAGG_F32, 1, NT, true>(row, row_bytes, K, 0, u1 - u0, nullptr, w, true, scale, false,
                                                 NoNorm(), epi);
  else
    walk_units<IN, AccF, FJAGG_F32, V, NT, true>(row, row_bytes, K, 0, u1 - u0, nullptr, w, true, scale, false,
                                                 NoNorm(), epi);
}

// Narrow parameter axis, many clients (exact mode). The exact fold walks the clients in
// order per element, so the only parallelism is the parameter axis: at 16 Ki-128 Ki f32
// params the 16-byte-unit kernels above have 4 K-32 K lanes for the whole chip and keep
// too few loads in flight (0.7-4.3 TB/s, profiles/r02i_*). Here a workgroup owns 64
// consecutive elements; all four waves load client rows into an LDS tile (each wave a
// quarter of the tile's clients, kNarrowTile/4 loads in flight per lane), and wave 0
// folds the previous tile from LDS in client order while the next tile is in flight
// (double buffer). One element per lane, so 64-element rows of 256 B per wave-load and
// 4x the lanes of the 16-byte path; any alignment. Same op sequence as fold(): bitwise.
constexpr int kNarrowCols = 64;

// TILE clients per LDS tile: 128 (2 x 32 KiB buffers: two workgroups per CU) when the grid
// has at least two stripes per CU, 256 (2 x 64 KiB: one per CU, twice the bytes in flight
// per workgroup) below that.
// Client rows of a dense slab: computed, nothing to stage.
struct SlabRows {
  const uint8_t* base;  // client 0's row at the stripe's first element
  int64_t ld_bytes;
  __device__ __forceinline__ void fetch(int64_t, int64_t) {}
  __device__ __forceinline__ void commit(int) {}
  __device__ __forceinline__ const uint8_t* row(int, int64_t k, int64_t) const { return base + k * ld_bytes; }
};

// Client rows of the pytree plan: pointers from the K x L table, staged through LDS
// (kRowSlots tiles of pointers; a per-row scalar load from the table would put one more
// memory round trip in front of every tile's loads). fetch() reads one tile's pointers
// into a register three tiles ahead of their use, commit() writes them to their slot.
constexpr int kRowSlots = 4;
template <int TILE>
struct TableRows {
  const int64_t* in_ptrs;
  int L, leaf;
  int64_t eoff;           // the stripe's first element, in bytes
  unsigned long long* lds;  // [kRowSlots][TILE] row pointers
  unsigned long long pr;    // this thread's fetched pointer (threads < TILE)
  __device__ __forceinline__ void fetch(int64_t k0, int64_t K) {
    if (threadIdx.x < TILE) {
      int64_t k = k0 + threadIdx.x;
      k = k < K ? k : K - 1;
      pr = (unsigned long long)in_ptrs[k * L + leaf];
    }
  }
  __device__ __forceinline__ void commit(int slot) {
    if (threadIdx.x < TILE) lds[slot * TILE + threadIdx.x] = pr;
  }
  __device__ __forceinline__ const uint8_t* row(int slot, int64_t k, int64_t k0) const {
    return reinterpret_cast<const uint8_t*>(lds[slot * TILE + (k - k0)]) + eoff;
  }
};

// Pipeline per workgroup (t = tile of kNarrowTile clients): while wave 0 folds tile t from
// LDS buffer t&1, the loads of tile t+1 (register set A) and tile t+2 (set B) are in
// flight; then tile t+1 goes to LDS buffer (t+1)&1. Two tiles in flight per workgroup:
// with one, each step waited out a full memory round trip for ~32 KiB (profiles/r02i_*).
template <int IN, class ACC, int OUT, bool NT, int kNarrowTile, class Rows>
__device__ __forceinline__ void narrow_fold(Rows rows, int64_t K, int64_t ncols,
                                            const typename ACC::T* __restrict__ w, float scale, int do_scale,
                                            int accumulate, uint8_t* __restrict__ out) {
  // rows: client k's row at this stripe's first element (SlabRows / TableRows); ncols <=
  // kNarrowCols valid elements; out: the stripe's first output element
  using T = typename ACC::T;
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B;
  constexpr int PER = kNarrowTile / (kThreads / 64);  // client rows per wave per tile
  __shared__ unsigned tile[2][kNarrowTile][kNarrowCols];
  __shared__ T wt[2][kNarrowTile];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool active = lane < ncols;
  const uint32_t coff = (uint32_t)((active ? lane : ncols - 1) * IB);
  const int64_t ntiles = (K + kNarrowTile - 1) / kNarrowTile;
  unsigned ra[PER], rb[PER];
  T wa = T(0), wb = T(0);
  auto load = [&](int64_t t, unsigned(&r)[PER], T& wr) {  // this wave's rows of tile t -> registers
    const int64_t k0 = t * kNarrowTile;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int64_t k = k0 + wave + (int64_t)(kThreads / 64) * i;
      k = k < K ? k : K - 1;
      const uint8_t* p = rows.row((int)(t % kRowSlots), k, k0) + coff;
      if constexpr (IB == 4) {
        r[i] = NT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p))
                  : *reinterpret_cast<const unsigned*>(p);
      } else {
        r[i] = NT ? (unsigned)__builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(p))
                  : (unsigned)*reinterpret_cast<const unsigned short*>(p);
      }
    }
    if (threadIdx.x < kNarrowTile) {
      const int64_t k = k0 + threadIdx.x;
      wr = ACC::weight(w[k < K ? k : K - 1]);
    }
  };
  auto store = [&](int64_t t, const unsigned(&r)[PER], T wr) {  // registers -> LDS buffer t & 1
    unsigned(*b)[kNarrowCols] = tile[t & 1];
#pragma unroll
    for (int i = 0; i < PER; ++i) b[wave + (kThreads / 64) * i][lane] = r[i];
    if (threadIdx.x < kNarrowTile) wt[t & 1][threadIdx.x] = wr;
  };
  T acc = T(0);
  auto fold_tile = [&](int64_t t) {  // wave 0: clients of tile t, in order, from LDS
    const unsigned(*b)[kNarrowCols] = tile[t & 1];
    const T* wk = wt[t & 1];
    const int64_t k0 = t * kNarrowTile;
    const int n = (int)(K - k0 < kNarrowTile ? K - k0 : kNarrowTile);
    int j = 0;
    if (t == 0) {  // client 0: s_0 = t_0, or out + t_0 (running sum)
      T v[1];
      decode<IN, ACC, 1>(b[0][lane], v);
      acc = ACC::mul(v[0], wk[0]);
      if (accumulate && active) {
        unsigned ob[1];
        load_out_unit<OUT, 1>(out + lane * OB, ob);
        acc = ACC::add(init_from<OUT, ACC>(ob[0]), acc);
      }
      j = 1;
    }
    // 8 clients' LDS reads in flight before their folds: the chain of adds is serial,
    // the reads are not (a read-fold-read loop waits out the LDS latency per client)
    for (; j + 8 <= n; j += 8) {
      unsigned raw[8];
      T wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        raw[u] = b[j + u][lane];
        wv[u] = wk[j + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        T v[1];
        decode<IN, ACC, 1>(raw[u], v);
        acc = ACC::add(acc, ACC::mul(v[0], wv[u]));
      }
    }
    for (; j < n; ++j) {
      T v[1];
      decode<IN, ACC, 1>(b[j][lane], v);
      acc = ACC::add(acc, ACC::mul(v[0], wk[j]));
    }
  };
  // one step of the pipeline: `cur` holds tile t+1's loads, `nxt` receives tile t+2's
  auto step = [&](int64_t t, unsigned(&cur)[PER], T& curw, unsigned(&nxt)[PER], T& nxtw) {
    if (t + 2 < ntiles) load(t + 2, nxt, nxtw);
    if (wave == 0) fold_tile(t);
    if (t + 1 < ntiles) store(t + 1, cur, curw);  // buffer (t+1)&1 was last read at step t-1
    if (t + 3 < ntiles) rows.commit((int)((t + 3) % kRowSlots));  // slot of tile t-1: done
    if (t + 4 < ntiles) rows.fetch((t + 4) * kNarrowTile, K);
    __syncthreads();
  };
  for (int64_t t = 0; t < 3 && t < ntiles; ++t) {  // row pointers of tiles 0..2
    rows.fetch(t * kNarrowTile, K);
    rows.commit((int)t);
  }
  __syncthreads();
  load(0, ra, wa);
  store(0, ra, wa);
  if (ntiles > 3) rows.fetch(3 * (int64_t)kNarrowTile, K);
  __syncthreads();
  if (ntiles > 1) load(1, ra, wa);
  for (int64_t t = 0; t < ntiles; t += 2) {
    step(t, ra, wa, rb, wb);
    if (t + 1 >= ntiles) break;
    step(t + 1, rb, wb, ra, wa);
  }
  if (wave == 0 && active) {
    const unsigned b[1] = {finish<OUT, ACC>(acc, do_scale != 0, scale)};
    store_unit<OUT, 1>(out + lane * OB, b);
  }
}

template <int IN, class ACC, int OUT, bool NT, int kNarrowTile>
__global__ __launch_bounds__(kThreads) void k_dense_narrow(const uint8_t* __restrict__ x, int64_t ld_bytes,
                                                           int64_t K, int64_t P,
                                                           const typename ACC::T* __restrict__ w, float scale,
                                                           int do_scale, int accumulate, uint8_t* __restrict__ out) {
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B;
  const int64_t c0 = (int64_t)blockIdx.x * kNarrowCols;
  const int64_t ncols = P - c0 < kNarrowCols ? P - c0 : kNarrowCols;
  narrow_fold<IN, ACC, OUT, NT, kNarrowTile>(SlabRows{x + c0 * IB, ld_bytes}, K, ncols, w, scale, do_scale,
                                             accumulate, out + c0 * OB);
}

// The same over the pytree plan image (FJAGG_NARROW): block b's words give its leaf and a
// range of at most kNarrowCols elements (fjagg_ptrs_plan_leaves with FJAGG_NARROW); the
// client rows come from the K x L pointer table.
template <int IN, class ACC, int OUT, bool NT, int kNarrowTile>
__global__ __launch_bounds__(kThreads) void k_ptrs_narrow(const int64_t* __restrict__ img, int L, int64_t K,
                                                          const typename ACC::T* __restrict__ w, float scale,
                                                          int do_scale, int accumulate) {
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B;
  __shared__ unsigned long long rowp[kRowSlots * kNarrowTile];
  const int64_t* in_ptrs = img;
  const int64_t* out_ptrs = img + K * L;
  const int64_t* leaf_n = out_ptrs + L;
  const int64_t* blk = leaf_n + L + 2 * (int64_t)blockIdx.x;
  const int64_t be = blk[0];
  const int leaf = (int)((be >> 40) & 0x3fffff);
  const int64_t e0 = be & ((1ll << 40) - 1), e1 = blk[1];
  uint8_t* ob = reinterpret_cast<uint8_t*>(out_ptrs[leaf]) + e0 * OB;
  narrow_fold<IN, ACC, OUT, NT, kNarrowTile>(TableRows<kNarrowTile>{in_ptrs, L, leaf, e0 * IB, rowp, 0ull}, K,
                                             e1 - e0, w, scale, do_scale, accumulate, ob);
}

// Per-client sum of squares: grid (nb, K); ws[k*nb + b] = block partial (f32),
// then k_l2sq_combine sums the nb partials of each client in block order.
template <int IN>
__global__ __launch_bounds__(kThreads) void k_l2sq_partial(const uint8_t* __restrict__ x,
                                                          int64_t ld_bytes, int64_t P,
                                                          int64_t per_block,
                                                          float* __restrict__ ws) {
  constexpr int IB = Elem<IN>::B;
  constexpr int VW = vec_width<IN>();
  const int64_t k = blockIdx.y;
  const uint8_t* r = x + k * ld_bytes;
  const int64_t e0 = (int64_t)blockIdx.x * per_block;
  const int64_t e1 = (e0 + per_block < P) ? e0 + per_block : P;
  float s = 0.f;
  const bool vec = ((reinterpret_cast<uintptr_t>(r) & 15) == 0) && (per_block % VW == 0);
  if (vec) {
    const int64_t nfull = (e1 - e0) / VW;
    for (int64_t u = threadIdx.x; u < nfull; u += kThreads) {
      float t[VW];
      decode<IN, AccF, VW>(load_unit_ptr<IN, VW, true>(r + (e0 + u * VW) * IB), t);
#pragma unroll
      for (int i = 0; i < VW; ++i) s = __fadd_rn(s, __fmul_rn(t[i], t[i]));
    }
    for (int64_t e = e0 + nfull * VW + threadIdx.x; e < e1; e += kThreads) {
      float t[1];
      decode<IN, AccF, 1>(load_unit_ptr<IN, 1, false>(r + e * IB), t);
      s = __fadd_rn(s, __fmul_rn(t[0], t[0]));
    }
  } else {
    for (int64_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
      float t[1];
      decode<IN, AccF, 1>(load_unit_ptr<IN, 1, false>(r + e * IB), t);
      s = __fadd_rn(s, __fmul_rn(t[0], t[0]));
    }
  }
  // wave reduction (fixed shuffle tree) then the 4 wave sums in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s = __fadd_rn(s, __shfl_xor(s, o, 64));
  __shared__ float red[kThreads / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int i = 1; i < kThreads / 64; ++i) t = __fadd_rn(t, red[i]);
    ws[k * gridDim.x + blockIdx.x] = t;
  }
}

__global__ void k_l2sq_combine(const float* __restrict__ ws, int64_t nb, int64_t K,
                               float* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float s = 0.f;
  for (int64_t b = 0; b < nb; ++b) s = __fadd_rn(s, ws[k * nb + b]);
  out[k] = s;
}

// Pytree form: rows r = 0..R-1 at arbitrary addresses (image = ptrs[R] | n[R]);
// grid (nbx, R); block b of row r sums elements [b*per, (b+1)*per) of that row.
template <int IN>
__global__ __launch_bounds__(kThreads) void k_l2sq_rows(const int64_t* __restrict__ img, int64_t R,
                                                       int64_t per, float* __restrict__ ws) {
  constexpr int IB = Elem<IN>::B;
  const int64_t r = blockIdx.y;
  const uint8_t* x = reinterpret_cast<const uint8_t*>(img[r]);
  const int64_t n = img[R + r];
  const int64_t e0 = (int64_t)blockIdx.x * per;
  const int64_t e1 = (e0 + per < n) ? e0 + per : n;
  float s = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
    float t[1];
    decode<IN, AccF, 1>(load_unit_ptr<IN, 1, false>(x + e * IB), t);
    s = __fadd_rn(s, __fmul_rn(t[0], t[0]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s = __fadd_rn(s, __shfl_xor(s, o, 64));
  __shared__ float red[kThreads / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int i = 1; i < kThreads / 64; ++i) t = __fadd_rn(t, red[i]);
    ws[r * gridDim.x + blockIdx.x] = t;
  }
}

// out[g] = sum over rows [g*rows_per_group, (g+1)*rows_per_group) and their nb partials,
// in order; sqrt of it when take_sqrt.
__global__ void k_l2sq_groups(const float* __restrict__ ws, int64_t nb, int64_t G,
                              int64_t rows_per_group, int take_sqrt, float* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  float s = 0.f;
  for (int64_t i = 0; i < rows_per_group * nb; ++i) s = __fadd_rn(s, ws[g * rows_per_group * nb + i]);
  out[g] = take_sqrt ? sqrt_rn(s) : s;  // correctly rounded, via f64
}

// Synthetic deltas (tests/bench only): bit-identical to oracle/fold_ref.c.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <int DT>
__global__ __launch_bounds__(kThreads) void k_fill(uint8_t* __restrict__ x, int64_t ld, int64_t K,
                                                  int64_t P, int64_t k0, uint64_t seed,
                                                  float amp) {
  const int64_t total = K * P;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kThreads) {
    const int64_t k = i / P, p = i - k * P;
    const uint64_t h = mix64(seed ^ mix64(((uint64_t)(k0 + k) << 32) | ((uint64_t)p & 0xffffffffull)));
    const float u = __fsub_rn(__fmul_rn((float)(uint32_t)(h >> 40), 1.0f / 8388608.0f), 1.0f);
    const float v = __fmul_rn(amp, u);
    if constexpr (DT == FJAGG_BF16)
      reinterpret_cast<unsigned short*>(x)[k * ld + p] = (unsigned short)f32_to_bf16(v);
    else
      reinterpret_cast<float*>(x)[k * ld + p] = v;
  }
}

// ------------------------------------------------------------------ host side
struct Combo {
  int in, acc, out;
};
bool combo_ok(int in, int acc, int out) {
  static const Combo ok[] = {{FJAGG_F32, FJAGG_F32, FJAGG_F32},  {FJAGG_F32, FJAGG_F32, FJAGG_BF16},
                             {FJAGG_BF16, FJAGG_F32, FJAGG_BF16},
                             {FJAGG_BF16, FJAGG_F32, FJAGG_F32}, {FJAGG_I32, FJAGG_F32, FJAGG_F32},
                             {FJAGG_I32, FJAGG_I32, FJAGG_I32},  {FJAGG_I32, FJAGG_I32, FJAGG_F32},
                             {FJAGG_BF16, FJAGG_BF16, FJAGG_BF16}};
  for (const Combo& c : ok)
    if (c.in == in && c.acc == acc && c.out == out) return true;
  return false;
}
int elem_bytes(int dt) { return dt == FJAGG_BF16 ? 2 : 4; }
int vwidth(int dt) { return 16 / elem_bytes(dt); }

// Kernel variants of the dense path: (E units per lane, U clients in flight).
// Variant 0 is the default chosen from the measurements in profiles/.
struct DenseArgs {
  const uint8_t* x;
  int64_t ld_bytes, K, nunits;
  int tail_n;
  const void* w;
  float scale;
  int do_scale, accumulate;
  uint8_t* out;
  int64_t kchunk, out_ystride;
  bool balanced;
  bool host_w;  // FJAGG_HOST_TABLES: w is host memory (K <= kKargWeights)
};

// (CUs, workgroups of `kern` per CU at once), cached per kernel and device. Used
// only to size balanced grids: never needed for correctness.
struct Residency {
  int cus, per_cu;
};
Residency residency(const void* kern, size_t smem = 0) {
  static std::mutex mu;
  static std::unordered_map<const void*, Residency> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const void* key = reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(kern) ^
                                                  ((uintptr_t)dev << 56) ^ ((uintptr_t)smem << 40));
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, smem) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  (void)hipGetLastError();
  const Residency r{cus, per_cu};
  std::lock_guard<std::mutex> g(mu);
  cache[key] = r;
  return r;
}

// Balanced grid (see launch_dense_t): units per workgroup S and workgroup count.
void balanced_grid(const Residency& r, int64_t nunits, int64_t tile, int64_t gy, int64_t* S_out,
                   int64_t* nblk_out) {
  const int64_t ntiles = (nunits + tile - 1) / tile;
  const int64_t cus = (r.cus + gy - 1) / gy;
  int64_t c = (ntiles + cus - 1) / cus;
  if (c > r.per_cu) c = r.per_cu;
  if (c < 1) c = 1;
  int64_t S = ((nunits + cus * c - 1) / (cus * c) + 63) / 64 * 64;
  if (S < 64) S = 64;
  *S_out = S;
  *nblk_out = (nunits + S - 1) / S;
}

template <int IN, class ACC, int OUT, int V, int E, int U, bool NT, int MINW, bool BURST = false, int WK = 0>
void launch_dense_t(const DenseArgs& a, int64_t gy, hipStream_t s) {
  auto kern = k_dense<IN, ACC, OUT, V, E, U, NT, MINW, BURST, WK>;
  const int64_t tile = (int64_t)kThreads * E;
  const int64_t ntiles = (a.nunits + tile - 1) / tile;
  int64_t nblk = ntiles, S = tile;
  if (a.balanced && ntiles > 0) {
    // The same number of workgroups on every CU (c <= what fits at once), each
    // with an equal, wave-aligned share of the parameter axis: every CU streams
    // the same bytes and no workgroup waits for a slot (profiles/r01_sweep3.jsonl).
    balanced_grid(residency(reinterpret_cast<const void*>(kern)), a.nunits, tile, gy, &S, &nblk);
  }
  dim3 grid((unsigned)(nblk + (a.tail_n > 0 ? 1 : 0)), (unsigned)gy);
  KargF32<(WK > 0 ? WK : 1)> kw;  // host weights copied into the kernel arguments
  if constexpr (WK > 0)
    std::memcpy(kw.w, a.w, sizeof(float) * (size_t)a.K);
  else
    kw.w[0] = 0.f;
  hipLaunchKernelGGL(kern, grid, dim3(kThreads), 0, s, a.x, a.ld_bytes, a.K, a.nunits, a.tail_n,
                     WK > 0 ? nullptr : reinterpret_cast<const typename ACC::T*>(a.w), a.scale, a.do_scale,
                     a.accumulate, a.out, a.kchunk, a.out_ystride, S, kw);
}

struct VariantShape {
  int E, U, minw;
};
// Index 0 is "auto" (resolved by pick_variant); 1.. are explicit shapes for tuning.
constexpr VariantShape kVariants[] = {{0, 0, 0},  {2, 8, 0},  {1, 8, 0},  {1, 16, 0},
                                      {2, 16, 0}, {4, 4, 0},  {4, 8, 0},  {1, 32, 0},
                                      {2, 8, 8},  {2, 4, 8},  {1, 16, 8}, {4, 4, 4},
                                      {8, 4, 0},  {8, 8, 0},  {4, 16, 0}, {4, 12, 0},
                                      {8, 4, 0} /* 16: E8U4 burst */, {8, 4, 0} /* 17: E8U4 interleaved */};
constexpr int kNarrowVariant = 18;  // k_dense_narrow (LDS-staged, one element per lane)
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]) + 1 + 4;  // + k_dense_stripe 19..22

// Default shape: E=8 x U=4 (8 units = 128 B per lane per client, 4 clients = 32
// loads in flight per lane, 3 workgroups per CU) on the balanced grid: fastest or
// within 2 % of the fastest on every swept shape with K >= 32 and >= 512 Ki f32
// params; E=1 x U=8 below that (profiles/r01_sweep3.jsonl, r01_sweep4.jsonl).
int pick_variant(int64_t nunits, int64_t K) {
  // few clients (short folds) or a narrow parameter axis: many light workgroups
  if (K < 32 || nunits < 131072) return 2;  // E=1 x U=8
  // up to 1 Mi f32 per row the balanced E=8 grid leaves most lanes of its single
  // workgroup per CU masked (4.6-4.9 TB/s at 512 Ki); E=4 x U=4 streams at 6.6-7.1
  // (profiles/r01n_sweep.jsonl: the per-bucket shapes of the sharded pipeline)
  if (nunits < 262144) return 5;  // E=4 x U=4 (at 1 Mi, burst E=8: profiles/r01s_probe_bucket.jsonl)
  return 12;                       // E=8 x U=4
}

// (in, acc, out) combinations built with FJAGG_HOST_TABLES weights (fjagg.h)
template <int IN, class ACC, int OUT>
constexpr bool kHostWeights = std::is_same<ACC, AccF>::value &&
                              ((IN == FJAGG_F32 && OUT == FJAGG_F32) || IN == FJAGG_BF16);

// The shapes pick_variant and launch_dense_v's variant 12 choose, with the weights in
// the kernel arguments (FJAGG_HOST_TABLES); other variants are not built that way.
template <int IN, class ACC, int OUT, int V, bool NT>
int launch_dense_hostw(int variant, const DenseArgs& a, int64_t gy, hipStream_t s) {
  if constexpr (!kHostWeights<IN, ACC, OUT>) {
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: dtype combination not built with kernel-argument weights");
  } else if constexpr (V == 1) {
    launch_dense_t<IN, ACC, OUT, 1, 1, 8, NT, 0, false, kKargWeights>(a, gy, s);
  } else {
    switch (variant) {
      case 2: launch_dense_t<IN, ACC, OUT, V, 1, 8, NT, 0, false, kKargWeights>(a, gy, s); break;
      case 5: launch_dense_t<IN, ACC, OUT, V, 4, 4, NT, 0, false, kKargWeights>(a, gy, s); break;
      case 12: {
        const int64_t ntiles = (a.nunits + (int64_t)kThreads * 8 - 1) / ((int64_t)kThreads * 8);
        const int cus = residency(reinterpret_cast<const void*>(k_dense<IN, ACC, OUT, V, 8, 4, NT, 0>)).cus;
        if (!a.balanced || ntiles * gy >= 2 * (int64_t)cus)
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, false, kKargWeights>(a, gy, s);
        else
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, true, kKargWeights>(a, gy, s);
        break;
      }
      case 16: launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, true, kKargWeights>(a, gy, s); break;
      case 17: launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, false, kKargWeights>(a, gy, s); break;
      default:
        return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: variant %d is not built with kernel-argument weights",
                    variant);
    }
  }
  return check_launch("k_dense");
}

template <int IN, class ACC, int OUT, int V, bool NT>
int launch_dense_v(int variant, const DenseArgs& a, int64_t gy, hipStream_t s) {
  if (a.host_w) return launch_dense_hostw<IN, ACC, OUT, V, NT>(variant, a, gy, s);
  if constexpr (V == 1) {  // element-granular path (tails, unaligned rows): one shape
    launch_dense_t<IN, ACC, OUT, 1, 1, 8, NT, 0>(a, gy, s);
    return check_launch("k_dense");
  } else if constexpr (ACC::DT == FJAGG_BF16) {  // the shapes pick_variant chooses
    switch (variant) {
      case 2: launch_dense_t<IN, ACC, OUT, V, 1, 8, NT, 0>(a, gy, s); break;
      case 5: launch_dense_t<IN, ACC, OUT, V, 4, 4, NT, 0>(a, gy, s); break;
      case 12: {
        const int64_t ntiles = (a.nunits + (int64_t)kThreads * 8 - 1) / ((int64_t)kThreads * 8);
        const int cus = residency(reinterpret_cast<const void*>(k_dense<IN, ACC, OUT, V, 8, 4, NT, 0>)).cus;
        if (!a.balanced || ntiles * gy >= 2 * (int64_t)cus)
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0>(a, gy, s);
        else
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, true>(a, gy, s);
        break;
      }
      default: return fail(FJAGG_EUNSUPPORTED, "variant %d is not built for the bf16 reference fold", variant);
    }
    return check_launch("k_dense");
  } else {
    switch (variant) {
      case 1: launch_dense_t<IN, ACC, OUT, V, 2, 8, NT, 0>(a, gy, s); break;
      case 2: launch_dense_t<IN, ACC, OUT, V, 1, 8, NT, 0>(a, gy, s); break;
      case 3: launch_dense_t<IN, ACC, OUT, V, 1, 16, NT, 0>(a, gy, s); break;
      case 4: launch_dense_t<IN, ACC, OUT, V, 2, 16, NT, 0>(a, gy, s); break;
      case 5: launch_dense_t<IN, ACC, OUT, V, 4, 4, NT, 0>(a, gy, s); break;
      case 6: launch_dense_t<IN, ACC, OUT, V, 4, 8, NT, 0>(a, gy, s); break;
      case 7: launch_dense_t<IN, ACC, OUT, V, 1, 32, NT, 0>(a, gy, s); break;
      case 8: launch_dense_t<IN, ACC, OUT, V, 2, 8, NT, 8>(a, gy, s); break;
      case 9: launch_dense_t<IN, ACC, OUT, V, 2, 4, NT, 8>(a, gy, s); break;
      case 10: launch_dense_t<IN, ACC, OUT, V, 1, 16, NT, 8>(a, gy, s); break;
      case 11: launch_dense_t<IN, ACC, OUT, V, 4, 4, NT, 4>(a, gy, s); break;
      case 12: {
        // Interleaved schedule when the balanced grid has >= 2 full E=8 tiles per CU
        // (several workgroups per CU hide latency), burst below that (one workgroup
        // per CU needs every load of a group in flight): profiles/r01s_probe_bucket.jsonl.
        const int64_t ntiles = (a.nunits + (int64_t)kThreads * 8 - 1) / ((int64_t)kThreads * 8);
        const int cus = residency(reinterpret_cast<const void*>(k_dense<IN, ACC, OUT, V, 8, 4, NT, 0>)).cus;
        if (!a.balanced || ntiles * gy >= 2 * (int64_t)cus)
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0>(a, gy, s);
        else
          launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, true>(a, gy, s);
        break;
      }
      case 16: launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0, true>(a, gy, s); break;
      case 17: launch_dense_t<IN, ACC, OUT, V, 8, 4, NT, 0>(a, gy, s); break;
      case 13: launch_dense_t<IN, ACC, OUT, V, 8, 8, NT, 0>(a, gy, s); break;
      case 14: launch_dense_t<IN, ACC, OUT, V, 4, 16, NT, 0>(a, gy, s); break;
      case 15: launch_dense_t<IN, ACC, OUT, V, 4, 12, NT, 0>(a, gy, s); break;
      default: return fail(FJAGG_EINVAL, "unknown kernel variant %d", variant);
    }
    return check_launch("k_dense");
  }
}

template <int IN, class ACC, int OUT>
int launch_dense_io(bool vec, bool nt, int variant, const DenseArgs& a, int64_t gy, hipStream_t s) {
  constexpr int VW = vec_width<IN>();
  if (vec) {
    return nt ? launch_dense_v<IN, ACC, OUT, VW, true>(variant, a, gy, s)
              : launch_dense_v<IN, ACC, OUT, VW, false>(variant, a, gy, s);
  }
  return nt ? launch_dense_v<IN, ACC, OUT, 1, true>(variant, a, gy, s)
            : launch_dense_v<IN, ACC, OUT, 1, false>(variant, a, gy, s);
}

int launch_dense_dispatch(int in, int acc, int out, bool vec, bool nt, int variant,
                          const DenseArgs& a, int64_t gy, hipStream_t s) {
#define FJ_CASE(I, A, O, ACCT)                                                          \
  if (in == I && acc == A && out == O)                                                  \
    return launch_dense_io<I, ACCT, O>(vec, nt, variant, a, gy, s);
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
  FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
  return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination (%d,%d,%d)", in, acc, out);
}

int64_t split_count(int64_t K, int64_t P) {
  // enough workgroups to give every one of the 256 CUs ~8 of them, each range
  // keeping >= 8 clients
  const int64_t nb = (P / 4 + kThreads * 2 - 1) / (kThreads * 2) + 1;
  int64_t s = (2048 + nb - 1) / nb;
  if (s > K / 8) s = K / 8;
  if (s > kSplitMax) s = kSplitMax;
  return s < 1 ? 1 : s;
}

int validate_common(int in, int acc, int out, int64_t K, int flags, float scale) {
  if (!combo_ok(in, acc, out))
    return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination (in=%d, acc=%d, out=%d)", in,
                acc, out);
  if (K < 1) return fail(FJAGG_EINVAL, "K must be >= 1 (got %lld)", (long long)K);
  if (acc == FJAGG_I32 && out == FJAGG_I32 && (flags & FJAGG_SCALE))
    return fail(FJAGG_EINVAL, "FJAGG_SCALE needs a float output");
  if ((flags & FJAGG_ACCUMULATE) && !((acc == FJAGG_F32 && out != FJAGG_I32) ||
                                      (acc == FJAGG_I32 && out == FJAGG_I32) ||
                                      (acc == FJAGG_BF16 && out == FJAGG_BF16)))
    return fail(FJAGG_EINVAL, "FJAGG_ACCUMULATE needs the output in the fold's type");
  (void)scale;
  return FJAGG_OK;
}

// One dense launch over elements [0, P) of rows that start at x (row stride ld_bytes).

template <int IN, class ACC, int OUT>
int launch_narrow_t(const uint8_t* x, int64_t ld_bytes, int64_t K, int64_t P, const void* w, float scale,
                    uint8_t* y, int flags, hipStream_t s) {
  const int64_t stripes = (P + kNarrowCols - 1) / kNarrowCols;
  const dim3 grid((unsigned)stripes);
  const auto* wt = reinterpret_cast<const typename ACC::T*>(w);
  const int dsc = (flags & FJAGG_SCALE) ? 1 : 0, acm = (flags & FJAGG_ACCUMULATE) ? 1 : 0;
  const bool nt = flags & FJAGG_NONTEMPORAL;
  const bool wide = stripes < 2 * (int64_t)cu_count() && K > 128;
#define FJ_NARROW(NTV, TILE)                                                                             \
  hipLaunchKernelGGL((k_dense_narrow<IN, ACC, OUT, NTV, TILE>), grid, dim3(kThreads), 0, s, x, ld_bytes, K, P, \
                     wt, scale, dsc, acm, y)
  if (nt && wide) FJ_NARROW(true, 256);
  else if (nt) FJ_NARROW(true, 128);
  else if (wide) FJ_NARROW(false, 256);
  else FJ_NARROW(false, 128);
#undef FJ_NARROW
  return check_launch("k_dense_narrow");
}

int launch_narrow(int in, int acc, int out, const uint8_t* x, int64_t ld_bytes, int64_t K, int64_t P,
                  const void* w, float scale, uint8_t* y, int flags, hipStream_t s) {
  if (K < 1 || P < 1) return FJAGG_OK;
#define FJ_CASE(I, A, O, ACCT) \
  if (in == I && acc == A && out == O) return launch_narrow_t<I, ACCT, O>(x, ld_bytes, K, P, w, scale, y, flags, s);
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
  FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
  return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination (%d,%d,%d)", in, acc, out);
}

constexpr int kStripeVariant = 19;  // k_dense_stripe (fjstripe.hip): 19 auto width, 20 / 21 / 22 = 64 / 32 / 16
constexpr int64_t kStripeMinClients = 512;

int dense_exact(int in, int acc, int out, const uint8_t* x, int64_t ld_bytes, int64_t K,
                int64_t P, const void* w, float scale, uint8_t* y, int flags, hipStream_t s,
                int64_t kchunk, int64_t gy, int64_t y_ystride) {
  const int ib = elem_bytes(in), ob = elem_bytes(out), vw = vwidth(in);
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 == 0) &&
                   (ld_bytes % 16 == 0) && (y_ystride % 16 == 0) && P >= vw;
  const int V = vec ? vw : 1;
  int variant = (flags >> 8) & 0xff;
  if (variant >= kNumVariants) return fail(FJAGG_EINVAL, "unknown kernel variant %d", variant);
  // a narrow parameter axis with many clients: the LDS-staged kernel (k_dense_narrow);
  // from 256 Ki f32 up the 16-byte kernels keep enough loads in flight (profiles/r02i_*)
  // with >= 512 clients the stripe pipeline (fjstripe.hip) is faster still at every swept
  // narrow shape (profiles/r03b_stripe_sweep.jsonl); below that k_dense_narrow's shorter
  // pipeline wins
  if (variant == 0 && gy == 1 && K >= 16 && P * ib <= (512 << 10))
    variant = (K >= kStripeMinClients && !(flags & FJAGG_HOST_TABLES) && fjagg_stripe_ok(x, ld_bytes, P, w, ib))
                  ? kStripeVariant
                  : kNarrowVariant;
  if (variant == 0) variant = pick_variant(P / V, K);
  if (variant == kNarrowVariant && (flags & FJAGG_HOST_TABLES))  // (fjagg_wsum_dense checks this first)
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: the narrow kernel takes device weights");
  if (variant == kNarrowVariant && gy == 1) return launch_narrow(in, acc, out, x, ld_bytes, K, P, w, scale, y, flags, s);
  if (variant >= kStripeVariant && variant <= kStripeVariant + 3) {
    if (gy != 1 || (flags & FJAGG_HOST_TABLES) || !fjagg_stripe_ok(x, ld_bytes, P, w, ib))
      return fail(FJAGG_EUNSUPPORTED, "k_dense_stripe: exact mode, device weights, 16-byte aligned rows");
    return fjagg_launch_stripe(variant, in, acc, out, x, ld_bytes, K, P, w, scale, y, flags, s);
  }
  DenseArgs a;
  a.x = x;
  a.ld_bytes = ld_bytes;
  a.K = K;
  a.nunits = P / V;
  a.tail_n = (int)(P - a.nunits * V);
  a.w = w;
  a.scale = scale;
  a.do_scale = (flags & FJAGG_SCALE) ? 1 : 0;
  a.accumulate = (flags & FJAGG_ACCUMULATE) ? 1 : 0;
  a.out = y;
  a.kchunk = kchunk;
  a.out_ystride = y_ystride;
  a.balanced = !(flags & FJAGG_UNBALANCED);
  a.host_w = (flags & FJAGG_HOST_TABLES) != 0;
  (void)ob;
  (void)ib;
  return launch_dense_dispatch(in, acc, out, vec, (flags & FJAGG_NONTEMPORAL) != 0, variant, a,
                               gy, s);
}

// Row bytes are addressed with 32-bit lane offsets: launch column chunks of <= 1 GiB.
constexpr int64_t kMaxRowBytes = 1ll << 30;

int dense_exact_chunked(int in, int acc, int out, const uint8_t* x, int64_t ld_bytes, int64_t K,
                        int64_t P, const void* w, float scale, uint8_t* y, int flags,
                        hipStream_t s, int64_t kchunk, int64_t gy, int64_t y_ystride) {
  const int64_t ib = elem_bytes(in), ob = elem_bytes(out);
  const int64_t chunk = kMaxRowBytes / ib;
  for (int64_t p0 = 0; p0 < P; p0 += chunk) {
    const int64_t n = (P - p0 < chunk) ? (P - p0) : chunk;
    int rc = dense_exact(in, acc, out, x + p0 * ib, ld_bytes, K, n, w, scale, y + p0 * ob, flags,
                         s, kchunk, gy, y_ystride);
    if (rc) return rc;
  }
  return FJAGG_OK;
}

// k_ptrs' XCD-aware plan order (xcd_plan_index), carried in bit 1 of its accumulate argument.
// FJAGG_XCD_REMAP=1 turns it on (A/B runs).
inline int xcd_remap_bit() {
  static const int on = [] {
    const char* e = getenv("FJAGG_XCD_REMAP");
    return (e && e[0] == '1') ? 2 : 0;
  }();
  return on;
}

template <int IN, class ACC, int OUT, int V>
int launch_ptrs_t(bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w,
                  float scale, int do_scale, int accumulate, float* ws, L2Out l2, hipStream_t s) {
  const auto* wt = reinterpret_cast<const typename ACC::T*>(w);
  accumulate = (accumulate ? 1 : 0) | xcd_remap_bit();
  if constexpr (std::is_same<ACC, AccF>::value) {
    if (ws) {  // fused per-client squared l2 norms: block partials, then ordered combine
      if (nblk > cu_count()) l2.done = nullptr;  // combine_last: a grid of one wave of workgroups
      const size_t smem = l2_smem(K, l2);
      const void* kf = nt ? reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, true, true>)
                          : reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, false, true>);
      if (int rc = allow_lds(kf, smem)) return rc;
      if (nt)
        hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true, true>), dim3((unsigned)nblk), dim3(kThreads), smem, s,
                           img, L, K, wt, scale, do_scale, accumulate, ws, l2, KargWords<1>{});
      else
        hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false, true>), dim3((unsigned)nblk), dim3(kThreads), smem,
                           s, img, L, K, wt, scale, do_scale, accumulate, ws, l2, KargWords<1>{});
      if (int rc = check_launch("k_ptrs (l2)")) return rc;
      return launch_l2_combine(ws, nblk, K, l2, s);
    }
  }
  // fold schedule as for the dense path (launch_dense_v): interleaved once the plan has
  // two or more workgroups per CU, burst below that
  const bool burst = nblk < 2 * (int64_t)residency(reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, true>)).cus;
  if (nt && burst)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true>), dim3((unsigned)nblk), dim3(kThreads), 0, s,
                       img, L, K, wt, scale, do_scale, accumulate, nullptr, L2Out{}, KargWords<1>{});
  else if (nt)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true, false, false>), dim3((unsigned)nblk), dim3(kThreads), 0, s,
                       img, L, K, wt, scale, do_scale, accumulate, nullptr, L2Out{}, KargWords<1>{});
  else if (burst)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false>), dim3((unsigned)nblk), dim3(kThreads), 0, s,
                       img, L, K, wt, scale, do_scale, accumulate, nullptr, L2Out{}, KargWords<1>{});
  else
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false, false, false>), dim3((unsigned)nblk), dim3(kThreads), 0, s,
                       img, L, K, wt, scale, do_scale, accumulate, nullptr, L2Out{}, KargWords<1>{});
  return check_launch("k_ptrs");
}

template <int IN, class ACC, int OUT>
int launch_ptrs_narrow(bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w, float scale,
                       int do_scale, int accumulate, hipStream_t s) {
  const auto* wt = reinterpret_cast<const typename ACC::T*>(w);
  const bool wide = nblk < 2 * (int64_t)cu_count() && K > 128;  // as launch_narrow_t
  const dim3 grid((unsigned)nblk);
#define FJ_NARROW(NTV, TILE) \
  hipLaunchKernelGGL((k_ptrs_narrow<IN, ACC, OUT, NTV, TILE>), grid, dim3(kThreads), 0, s, img, L, K, wt, scale, \
                     do_scale, accumulate)
  if (nt && wide) FJ_NARROW(true, 256);
  else if (nt) FJ_NARROW(true, 128);
  else if (wide) FJ_NARROW(false, 256);
  else FJ_NARROW(false, 128);
#undef FJ_NARROW
  return check_launch("k_ptrs_narrow");
}

template <int IN, class ACC, int OUT>
int launch_ptrs_io(bool vec, bool nt, const int64_t* img, int L, int64_t K, int64_t nblk,
                   const void* w, float scale, int do_scale, int accumulate, float* ws, L2Out l2,
                   hipStream_t s) {
  if (vec)
    return launch_ptrs_t<IN, ACC, OUT, vec_width<IN>()>(nt, img, L, K, nblk, w, scale, do_scale,
                                                        accumulate, ws, l2, s);
  return launch_ptrs_t<IN, ACC, OUT, 1>(nt, img, L, K, nblk, w, scale, do_scale, accumulate, ws, l2, s);
}

template <int IN, int OUT, int V, int E, int U, bool NT>
int launch_dense_l2_t(const DenseArgs& a, float* ws, int64_t ws_floats, L2Out l2, hipStream_t s) {
  auto kern = k_dense_l2<IN, OUT, V, E, U, NT>;
  size_t smem = l2_smem(a.K, l2);
  if (int rc = allow_lds(reinterpret_cast<const void*>(kern), smem)) return rc;
  int64_t S = (int64_t)kThreads * E, nblk = 0;
  balanced_grid(residency(reinterpret_cast<const void*>(kern), l2_smem(a.K, l2, false)), a.nunits,
                (int64_t)kThreads * E, 1, &S, &nblk);
  if (a.nunits == 0) nblk = 0;
  const int64_t grid = nblk + (a.tail_n > 0 ? 1 : 0);
  if (l2.done && grid > cu_count()) {  // combine_last: a grid of one wave of workgroups
    l2.done = nullptr;
    smem = l2_smem(a.K, l2);
  }
  if (grid * (l2.done ? round4(a.K) : a.K) > ws_floats)
    return fail(FJAGG_EINVAL, "l2 workspace too small (%lld workgroups x %lld clients)",
                (long long)grid, (long long)a.K);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), smem, s, a.x, a.ld_bytes, a.K,
                     a.nunits, a.tail_n, reinterpret_cast<const float*>(a.w), a.scale, a.do_scale,
                     a.accumulate, a.out, S, ws, l2);
  int rc = check_launch("k_dense_l2");
  if (rc) return rc;
  return launch_l2_combine(ws, grid, a.K, l2, s);
}

template <int IN, int OUT>
int launch_dense_l2_io(bool vec, bool nt, int variant, const DenseArgs& a, float* ws,
                       int64_t ws_floats, L2Out l2, hipStream_t s) {
  constexpr int VW = vec_width<IN>();
  if (!vec)
    return nt ? launch_dense_l2_t<IN, OUT, 1, 1, 8, true>(a, ws, ws_floats, l2, s)
              : launch_dense_l2_t<IN, OUT, 1, 1, 8, false>(a, ws, ws_floats, l2, s);
  if (variant == 12)
    return nt ? launch_dense_l2_t<IN, OUT, VW, 8, 4, true>(a, ws, ws_floats, l2, s)
              : launch_dense_l2_t<IN, OUT, VW, 8, 4, false>(a, ws, ws_floats, l2, s);
  return nt ? launch_dense_l2_t<IN, OUT, VW, 1, 8, true>(a, ws, ws_floats, l2, s)
            : launch_dense_l2_t<IN, OUT, VW, 1, 8, false>(a, ws, ws_floats, l2, s);
}

template <int IN, int V, int E, int U, bool NT>
int launch_dense_opt_t(const DenseArgs& a, const OptEpi& epi, hipStream_t s) {
  auto kern = k_dense_opt<IN, V, E, U, NT>;
  int64_t S = (int64_t)kThreads * E, nblk = 0;
  balanced_grid(residency(reinterpret_cast<const void*>(kern)), a.nunits, (int64_t)kThreads * E, 1,
                &S, &nblk);
  if (a.nunits == 0) nblk = 0;
  const int64_t grid = nblk + (a.tail_n > 0 ? 1 : 0);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), 0, s, a.x, a.ld_bytes, a.K,
                     a.nunits, a.tail_n, reinterpret_cast<const float*>(a.w), a.scale, S, epi);
  return check_launch("k_dense_opt");
}

template <int IN>
int launch_dense_opt_io(bool vec, bool nt, int variant, const DenseArgs& a, const OptEpi& epi,
                        hipStream_t s) {
  constexpr int VW = vec_width<IN>();
  if (!vec)
    return nt ? launch_dense_opt_t<IN, 1, 1, 8, true>(a, epi, s)
              : launch_dense_opt_t<IN, 1, 1, 8, false>(a, epi, s);
  if (variant == 12)
    return nt ? launch_dense_opt_t<IN, VW, 8, 4, true>(a, epi, s)
              : launch_dense_opt_t<IN, VW, 8, 4, false>(a, epi, s);
  return nt ? launch_dense_opt_t<IN, VW, 1, 8, true>(a, epi, s)
            : launch_dense_opt_t<IN, VW, 1, 8, false>(a, epi, s);
}

constexpr int64_t kL2MaxClients = 4096;
constexpr int64_t kL2Header = 16;  // fused-norm workspaces: the FJAGG_ZEROED_WS completion counter  // (kThreads/64) x K floats of LDS <= 64 KiB

}  // namespace

// Whether an exact-mode dense fold of K x P (one launch per <= 1 GiB column chunk) can
// take FJAGG_HOST_TABLES weights: FJAGG_OK or FJAGG_EUNSUPPORTED (message set). Callers
// that launch several folds (fjcomm's buckets) check every one before the first launch.
__attribute__((visibility("hidden"))) int fjagg_host_weights_check(int in_dtype, int acc_dtype, int out_dtype,
                                                                   int64_t K, int64_t P, int flags) {
  const int variant = (flags >> 8) & 0xff;
  const int64_t ib = elem_bytes(in_dtype), chunk = kMaxRowBytes / ib;
  const int64_t last = P > 0 ? P - (P - 1) / chunk * chunk : 0;
  if (K > kKargWeights)
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: K = %lld > %d weights", (long long)K, kKargWeights);
  if (acc_dtype != FJAGG_F32 || !((in_dtype == FJAGG_F32 && out_dtype == FJAGG_F32) || in_dtype == FJAGG_BF16))
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: dtype combination not built with kernel-argument weights");
  if (!(variant == 0 || variant == 2 || variant == 5 || variant == 12 || variant == 16 || variant == 17))
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: variant %d takes device weights", variant);
  if (variant == 0 && K >= 16 && last * ib <= (512 << 10))  // dense_exact's narrow rule (last chunk)
    return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: the narrow kernel takes device weights");
  return FJAGG_OK;
}

namespace {
// n words of v at p (split mode's unit weights): a kernel, not hipMemsetD32Async, whose node in a
// captured graph takes effect on the first replay only (measured: tools/probe_memset_node.py)
__global__ __launch_bounds__(256) void k_fill_u32(unsigned* __restrict__ p, unsigned v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* fjagg_last_error(void) { return g_err; }

int fjagg_abi_version(void) { return FJAGG_ABI_VERSION; }

int64_t fjagg_split_workspace_bytes(int64_t K, int64_t P) {
  if (K < 1 || P < 1) return 0;
  const int64_t s = split_count(K, P);
  if (s <= 1) return 0;
  return kSplitHeader + s * ((P * 4 + 255) / 256 * 256);
}

int fjagg_wsum_dense(int in_dtype, int acc_dtype, int out_dtype, const void* x_dev, int64_t ld,
                     int64_t K, int64_t P, const void* w_dev, float scale, void* out_dev,
                     int flags, int mode, void* ws_dev, int64_t ws_bytes, void* stream) {
  g_err[0] = 0;
  int rc = validate_common(in_dtype, acc_dtype, out_dtype, K, flags, scale);
  if (rc) return rc;
  if (P < 0 || ld < P) return fail(FJAGG_EINVAL, "need 0 <= P <= ld (P=%lld ld=%lld)", (long long)P, (long long)ld);
  if (P == 0) return FJAGG_OK;
  if (!x_dev || !w_dev || !out_dev) return fail(FJAGG_EINVAL, "null pointer argument");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* x = reinterpret_cast<const uint8_t*>(x_dev);
  uint8_t* y = reinterpret_cast<uint8_t*>(out_dev);
  const int64_t ib = elem_bytes(in_dtype);
  if (flags & FJAGG_HOST_TABLES) {  // checked up front: nothing may launch before a refusal
    if (mode != FJAGG_MODE_EXACT) return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: exact mode only");
    if (int rc = fjagg_host_weights_check(in_dtype, acc_dtype, out_dtype, K, P, flags)) return rc;
  }
  if (mode == FJAGG_MODE_EXACT)
    return dense_exact_chunked(in_dtype, acc_dtype, out_dtype, x, ld * ib, K, P, w_dev, scale, y,
                               flags, s, K, 1, 0);
  if (mode != FJAGG_MODE_SPLIT) return fail(FJAGG_EINVAL, "unknown mode %d", mode);
  if (acc_dtype == FJAGG_BF16)
    return fail(FJAGG_EUNSUPPORTED, "split mode reorders the fold; the bf16 reference fold runs in exact mode");
  const int64_t S = split_count(K, P);
  if (S <= 1)  // nothing to split: the exact path already fills the chip
    return dense_exact_chunked(in_dtype, acc_dtype, out_dtype, x, ld * ib, K, P, w_dev, scale, y,
                               flags, s, K, 1, 0);
  const int64_t need = fjagg_split_workspace_bytes(K, P);
  if (!ws_dev || ws_bytes < need)
    return fail(FJAGG_EINVAL, "split mode needs %lld workspace bytes (got %lld)", (long long)need,
                (long long)ws_bytes);
  uint8_t* ws = reinterpret_cast<uint8_t*>(ws_dev);
  const int64_t pstride = (P * 4 + 255) / 256 * 256;  // bytes per range partial
  const int64_t kchunk = (K + S - 1) / S;
  const int64_t gy = (K + kchunk - 1) / kchunk;
  // 1) each client range folds into its own partial (fold type, no scale)
  const int flags1 = flags & ~(FJAGG_SCALE | FJAGG_ACCUMULATE);
  rc = dense_exact_chunked(in_dtype, acc_dtype, acc_dtype, x, ld * ib, K, P, w_dev, 1.0f,
                           ws + kSplitHeader, flags1, s, kchunk, gy, pstride);
  if (rc) return rc;
  // 2) ordered combine of the gy partials = unit-weight fold (x*1 is exact)
  const unsigned one_bits = acc_dtype == FJAGG_F32 ? 0x3f800000u : 1u;
  hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)((kSplitMax + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<unsigned*>(ws), one_bits, (int64_t)kSplitMax);
  if (int rc2 = check_launch("k_fill_u32")) return rc2;
  const int flags2 = flags & (FJAGG_SCALE | FJAGG_ACCUMULATE);
  return dense_exact_chunked(acc_dtype, acc_dtype, out_dtype, ws + kSplitHeader, pstride, gy, P,
                             ws, scale, y, flags2, s, gy, 1, 0);
}

int64_t fjagg_ptrs_plan(int in_dtype, int flags, const int64_t* leaf_n, int L, int64_t* blocks,
                        int64_t blocks_cap) {
  return fjagg_ptrs_plan_leaves(in_dtype, flags, leaf_n, nullptr, L, blocks, blocks_cap);
}

}  // extern "C"


extern "C" {

int64_t fjagg_ptrs_plan_leaves(int in_dtype, int flags, const int64_t* leaf_n, const uint8_t* leaf_elem, int L,
                               int64_t* blocks, int64_t blocks_cap) {
  g_err[0] = 0;
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16 && in_dtype != FJAGG_I32)
    return fail(FJAGG_EINVAL, "bad dtype %d", in_dtype);
  if (L < 0 || L >= (1 << 22)) return fail(FJAGG_EINVAL, "bad leaf count %d", L);
  if (flags & FJAGG_NARROW) {
    // stripes of kNarrowCols elements of every leaf (k_ptrs_narrow), or of C = 64 / 32 / 16
    // elements with FJAGG_VARIANT(20 / 21 / 22) (k_ptrs_stripe)
    const int variant = (flags >> 8) & 0xff;
    const int64_t width = variant == 20 ? 64 : variant == 21 ? 32 : variant == 22 ? 16 : kNarrowCols;
    int64_t nblk = 0;
    for (int l = 0; l < L; ++l) {
      if (leaf_n[l] < 0 || leaf_n[l] >= (1ll << 40))
        return fail(FJAGG_EINVAL, "leaf %d: %lld elements unsupported", l, (long long)leaf_n[l]);
      for (int64_t e = 0; e < leaf_n[l]; e += width, ++nblk) {
        if (nblk < blocks_cap) {
          blocks[2 * nblk] = ((int64_t)l << 40) | e;
          blocks[2 * nblk + 1] = e + width < leaf_n[l] ? e + width : leaf_n[l];
        }
      }
    }
    return nblk;
  }
  const int64_t V = (flags & FJAGG_UNALIGNED) ? 1 : vwidth(in_dtype);
  int64_t total = 0;
  for (int l = 0; l < L; ++l) {
    const int64_t n = leaf_n[l];
    // unit offsets are 40-bit in the block words; rows are rebased per workgroup
    if (n < 0 || n >= (1ll << 40))
      return fail(FJAGG_EINVAL, "leaf %d: %lld elements unsupported", l, (long long)n);
    total += (leaf_elem && leaf_elem[l]) ? (n + V - 1) / V : n / V;  // balance by bytes
  }
  // balanced unit share per workgroup, as for the dense path (balanced_grid): the
  // same number of E=8 workgroups on every CU, at most kPlanPerCU of them per CU
  const int cus = cu_count();
  constexpr int64_t kPlanPerCU = 3;  // E=8 x U=4 fold: 3 workgroups per CU (VGPR-limited)
  const int64_t tile = (int64_t)kThreads * 8;
  const int64_t ntiles = (total + tile - 1) / tile;
  int64_t c = (ntiles + cus - 1) / cus;
  if (c > kPlanPerCU) c = kPlanPerCU;
  if (c < 1) c = 1;
  int64_t S = ((total + cus * c - 1) / (cus * c) + 63) / 64 * 64;
  if (S < 64) S = 64;
  int64_t nblk = 0;
  auto put = [&](int64_t w0, int64_t w1) {
    if (nblk < blocks_cap) {
      blocks[2 * nblk] = w0;
      blocks[2 * nblk + 1] = w1;
    }
    ++nblk;
  };
  // element-unit leaves (V > 1 only): units are single elements, ranges of S of them.
  // A workgroup's time is set by its sequential walks over the K clients (one per
  // group of kThreads*8 units), not by its bytes, so element ranges keep the unit
  // count of the vector ranges: S*V elements would take V times as many walks.
  auto is_elem = [&](int l) { return V > 1 && leaf_elem && leaf_elem[l]; };
  for (int l = 0; l < L; ++l)  // tails first: latency-bound, start them early
    if (!is_elem(l) && leaf_n[l] % V) put(((int64_t)l << 40) | (1ll << 62), 0);
  for (int l = 0; l < L; ++l) {
    const bool el = is_elem(l);
    const int64_t nunits = el ? leaf_n[l] : leaf_n[l] / V, step = S;
    const int64_t flag = el ? (int64_t)(1ull << 63) : 0;
    for (int64_t u = 0; u < nunits; u += step)
      put(flag | ((int64_t)l << 40) | u, (u + step < nunits) ? u + step : nunits);
  }
  return nblk;
}

namespace {
// FJAGG_HOST_TABLES on the pytree path: the host image and the K f32 weights are copied
// into ONE kernel-argument struct (k_ptrs<..., NW>), float32 leaves, 16-byte units. The
// struct comes in three sizes (NW = 1024, 2048, kKargWords words) and the launch takes the
// smallest that holds the image: the host cost of a launch grows with its argument bytes
// (tools/probe_launch_cost.hip: 3.3 us at 8 KiB, 4.4 at 16 KiB, 7.5 at 28 KiB per launch on
// MI355X), and a synchronous tree_mean waits for its first launch.
extern "C++" {
template <int NW>
int launch_ptrs_karg_n(bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w, float scale,
                       int ds, int ac, float* ws, L2Out l2, hipStream_t s) {
  constexpr int IN = FJAGG_F32, OUT = FJAGG_F32, V = 4;
  using ACC = AccF;
  ac = (ac ? 1 : 0) | xcd_remap_bit();
  KargWords<NW> ki;
  const int64_t nimg = K * L + 2 * (int64_t)L + 2 * nblk;
  std::memcpy(ki.w, img, sizeof(int64_t) * (size_t)nimg);
  ki.w[nimg + (K + 1) / 2 - 1] = 0;  // the odd weight slot, if any
  std::memcpy(ki.w + nimg, w, sizeof(float) * (size_t)K);
  const dim3 grid((unsigned)nblk), block(kThreads);
  if (ws) {
    if (nblk > cu_count()) l2.done = nullptr;  // combine_last: a grid of one wave of workgroups
    const size_t smem = l2_smem(K, l2);
    const void* kf = nt ? reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, true, true, true, NW>)
                        : reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, false, true, true, NW>);
    if (int rc = allow_lds(kf, smem)) return rc;
    if (nt)
      hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true, true, true, NW>), grid, block, smem, s, nullptr, L,
                         K, nullptr, scale, ds, ac, ws, l2, ki);
    else
      hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false, true, true, NW>), grid, block, smem, s, nullptr, L,
                         K, nullptr, scale, ds, ac, ws, l2, ki);
    if (int rc = check_launch("k_ptrs (l2, kernel-argument image)")) return rc;
    return launch_l2_combine(ws, nblk, K, l2, s);
  }
  // the schedule rule of launch_ptrs_t
  const bool burst = nblk < 2 * (int64_t)residency(reinterpret_cast<const void*>(k_ptrs<IN, ACC, OUT, V, true>)).cus;
  if (nt && burst)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true, false, true, NW>), grid, block, 0, s, nullptr, L, K,
                       nullptr, scale, ds, ac, nullptr, L2Out{}, ki);
  else if (nt)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, true, false, false, NW>), grid, block, 0, s, nullptr, L, K,
                       nullptr, scale, ds, ac, nullptr, L2Out{}, ki);
  else if (burst)
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false, false, true, NW>), grid, block, 0, s, nullptr, L, K,
                       nullptr, scale, ds, ac, nullptr, L2Out{}, ki);
  else
    hipLaunchKernelGGL((k_ptrs<IN, ACC, OUT, V, false, false, false, NW>), grid, block, 0, s, nullptr, L, K,
                       nullptr, scale, ds, ac, nullptr, L2Out{}, ki);
  return check_launch("k_ptrs (kernel-argument image)");
}
}  // extern "C++"

int launch_ptrs_karg(bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w, float scale,
                     int ds, int ac, float* ws, L2Out l2, hipStream_t s) {
  const int64_t words = fjagg_karg_image_words(K, L, nblk);
  if (words <= 1024) return launch_ptrs_karg_n<1024>(nt, img, L, K, nblk, w, scale, ds, ac, ws, l2, s);
  if (words <= 2048) return launch_ptrs_karg_n<2048>(nt, img, L, K, nblk, w, scale, ds, ac, ws, l2, s);
  return launch_ptrs_karg_n<kKargWords>(nt, img, L, K, nblk, w, scale, ds, ac, ws, l2, s);
}

int wsum_ptrs_impl(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L,
                   int64_t K, int64_t nblk, const void* w_dev, float scale, int flags, float* ws,
                   L2Out l2, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool vec = !(flags & FJAGG_UNALIGNED);
  const bool nt = (flags & FJAGG_NONTEMPORAL) != 0;
  const int ds = (flags & FJAGG_SCALE) ? 1 : 0, ac = (flags & FJAGG_ACCUMULATE) ? 1 : 0;
  if (flags & FJAGG_HOST_TABLES) {
    if (in_dtype != FJAGG_F32 || acc_dtype != FJAGG_F32 || out_dtype != FJAGG_F32)
      return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: float32 leaves and fold only");
    if (flags & (FJAGG_UNALIGNED | FJAGG_NARROW))
      return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: 16-byte unit plans only (no UNALIGNED / NARROW)");
    const int64_t words = fjagg_karg_image_words(K, L, nblk);
    if (words > kKargWords)
      return fail(FJAGG_EUNSUPPORTED, "FJAGG_HOST_TABLES: %lld words > %d", (long long)words, kKargWords);
    return launch_ptrs_karg(nt, image_dev, L, K, nblk, w_dev, scale, ds, ac, ws, l2, s);
  }
  if (flags & FJAGG_NARROW) {
    if (ws) return fail(FJAGG_EINVAL, "FJAGG_NARROW plans fold only (no fused norms)");
    const int variant = (flags >> 8) & 0xff;
    if (variant >= 20 && variant <= 22) {  // k_ptrs_stripe over C-element stripes (fjstripe.hip)
      if (flags & FJAGG_UNALIGNED) return fail(FJAGG_EINVAL, "stripe plans need 16-byte aligned pointers");
      return fjagg_launch_ptrs_stripe(variant == 20 ? 64 : variant == 21 ? 32 : 16, in_dtype, acc_dtype, out_dtype,
                                      nt, image_dev, L, K, nblk, w_dev, scale, ds, ac, s);
    }
#define FJ_CASE(I, A, O, ACCT)                                                                          \
    if (in_dtype == I && acc_dtype == A && out_dtype == O)                                              \
      return launch_ptrs_narrow<I, ACCT, O>(nt, image_dev, L, K, nblk, w_dev, scale, ds, ac, s);
    FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
    FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
    FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
    FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
    FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
    FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
    FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
    return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination");
  }
#define FJ_CASE(I, A, O, ACCT)                                                                 \
  if (in_dtype == I && acc_dtype == A && out_dtype == O)                                       \
    return launch_ptrs_io<I, ACCT, O>(vec, nt, image_dev, L, K, nblk, w_dev, scale, ds, ac, ws, l2, s);
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
  FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
  return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination");
}
}  // namespace

int64_t fjagg_karg_image_words(int64_t K, int L, int64_t nblk) {
  if (K < 0 || L < 0 || nblk < 0) return -1;
  return K * L + 2 * (int64_t)L + 2 * nblk + (K + 1) / 2;
}

int fjagg_wsum_ptrs(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L,
                    int64_t K, int64_t nblk, const void* w_dev, float scale, int flags,
                    void* stream) {
  g_err[0] = 0;
  int rc = validate_common(in_dtype, acc_dtype, out_dtype, K, flags, scale);
  if (rc) return rc;
  if (nblk == 0) return FJAGG_OK;
  if (nblk < 0 || nblk > 0x7fffffff || !image_dev || !w_dev || L < 1)
    return fail(FJAGG_EINVAL, "bad plan (nblk=%lld, L=%d)", (long long)nblk, L);
  return wsum_ptrs_impl(in_dtype, acc_dtype, out_dtype, image_dev, L, K, nblk, w_dev, scale, flags,
                        nullptr, L2Out{nullptr, nullptr, 0}, stream);
}

}  // extern "C"
namespace {
bool opt_needs_m(const fjagg_server_opt& o) {
  return o.kind == FJAGG_OPT_MOMENTUM || o.kind == FJAGG_OPT_ADAM || o.kind == FJAGG_OPT_YOGI ||
         (o.kind == FJAGG_OPT_RMSPROP && (o.flags & (FJAGG_OPT_F_MOMENTUM | FJAGG_OPT_F_CENTERED)));
}
bool opt_needs_v(const fjagg_server_opt& o) { return o.kind >= FJAGG_OPT_ADAM; }
bool opt_valid(const fjagg_server_opt* o) {
  if (!o || o->kind < FJAGG_OPT_SGD || o->kind > FJAGG_OPT_YOGI) return false;
  const int known = o->kind == FJAGG_OPT_RMSPROP ? (FJAGG_OPT_F_MOMENTUM | FJAGG_OPT_F_CENTERED) : FJAGG_OPT_F_MOMENTUM;
  if (o->flags & ~known) return false;
  return (o->flags & (FJAGG_OPT_F_MOMENTUM | FJAGG_OPT_F_CENTERED)) != (FJAGG_OPT_F_MOMENTUM | FJAGG_OPT_F_CENTERED);
}
}  // namespace
extern "C" {

int fjagg_server_update_ptrs(int in_dtype, const int64_t* image_dev, int L, int64_t K, int64_t nblk,
                             const float* w_dev, float scale, const fjagg_server_opt* opt,
                             const int64_t* state_dev, int flags, void* stream) {
  g_err[0] = 0;
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16)
    return fail(FJAGG_EUNSUPPORTED, "server update: f32 or bf16 deltas");
  if (!opt_valid(opt)) return fail(FJAGG_EINVAL, "server update: bad optimizer descriptor");
  if (K < 1) return fail(FJAGG_EINVAL, "need K >= 1");
  if (nblk == 0) return FJAGG_OK;
  if (nblk < 0 || nblk > 0x7fffffff || !image_dev || !w_dev || !state_dev || L < 1)
    return fail(FJAGG_EINVAL, "bad plan (nblk=%lld, L=%d)", (long long)nblk, L);
  if (flags & ~(FJAGG_NONTEMPORAL | FJAGG_UNALIGNED))
    return fail(FJAGG_EINVAL, "flags may hold FJAGG_NONTEMPORAL and FJAGG_UNALIGNED only");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool vec = !(flags & FJAGG_UNALIGNED), nt = (flags & FJAGG_NONTEMPORAL) != 0;
  const dim3 grid((unsigned)nblk), block(kThreads);
#define FJ_OPT_LAUNCH(I, VV)                                                                         \
  do {                                                                                               \
    if (nt)                                                                                          \
      hipLaunchKernelGGL((k_ptrs_opt<I, VV, true>), grid, block, 0, s, image_dev, L, K, w_dev, scale, \
                         *opt, state_dev);                                             \
    else                                                                                             \
      hipLaunchKernelGGL((k_ptrs_opt<I, VV, false>), grid, block, 0, s, image_dev, L, K, w_dev, scale, \
                         *opt, state_dev);                                             \
  } while (0)
  if (in_dtype == FJAGG_F32) {
    if (vec) FJ_OPT_LAUNCH(FJAGG_F32, 4); else FJ_OPT_LAUNCH(FJAGG_F32, 1);
  } else {
    if (vec) FJ_OPT_LAUNCH(FJAGG_BF16, 8); else FJ_OPT_LAUNCH(FJAGG_BF16, 1);
  }
#undef FJ_OPT_LAUNCH
  return check_launch("k_ptrs_opt");
}

int64_t fjagg_wsum_l2_ptrs_workspace_bytes(int64_t K, int64_t nblk) {
  return (K < 1 || nblk < 1) ? 0 : kL2Header + round4(K) * nblk * 4;
}

namespace {
// The norm partials of a fused-norm call and where its combine runs: with FJAGG_ZEROED_WS the
// workspace's first kL2Header bytes are the completion counter (zero between calls) and the
// partials follow; the fold's last workgroup combines when K fits combine_last.
L2Out l2_layout(L2Out out, void* ws_dev, int64_t K, int flags, float** ws) {
  *ws = reinterpret_cast<float*>(ws_dev);
  if (!(flags & FJAGG_ZEROED_WS)) return out;
  *ws += kL2Header / 4;
  if (K <= kFusedCombineMax && reinterpret_cast<uintptr_t>(ws_dev) % 16 == 0)
    out.done = reinterpret_cast<unsigned*>(ws_dev);
  return out;
}

int wsum_l2_ptrs_checked(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L, int64_t K,
                         int64_t nblk, const void* w_dev, float scale, L2Out out, int flags, void* ws_dev,
                         int64_t ws_bytes, void* stream);
}  // namespace

int fjagg_wsum_l2_ptrs(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L,
                       int64_t K, int64_t nblk, const void* w_dev, float scale, float* l2sq_dev,
                       int flags, void* ws_dev, int64_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (!l2sq_dev) return fail(FJAGG_EINVAL, "null pointer argument");
  return wsum_l2_ptrs_checked(in_dtype, acc_dtype, out_dtype, image_dev, L, K, nblk, w_dev, scale,
                              L2Out{l2sq_dev, nullptr, 0}, flags, ws_dev, ws_bytes, stream);
}

int fjagg_wsum_l2_ptrs_rows(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L,
                            int64_t K, int64_t nblk, const void* w_dev, float scale, float* sq_dev,
                            float* norm_dev, int64_t first, int flags, void* ws_dev, int64_t ws_bytes,
                            void* stream) {
  g_err[0] = 0;
  if (!sq_dev && !norm_dev) return fail(FJAGG_EINVAL, "null pointer argument");
  if (first < 0 || first > K) return fail(FJAGG_EINVAL, "first = %lld outside [0, K]", (long long)first);
  return wsum_l2_ptrs_checked(in_dtype, acc_dtype, out_dtype, image_dev, L, K, nblk, w_dev, scale,
                              L2Out{sq_dev, norm_dev, first}, flags, ws_dev, ws_bytes, stream);
}

}  // extern "C"
namespace {
int wsum_l2_ptrs_checked(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev, int L, int64_t K,
                         int64_t nblk, const void* w_dev, float scale, L2Out out, int flags, void* ws_dev,
                         int64_t ws_bytes, void* stream) {
  int rc = validate_common(in_dtype, acc_dtype, out_dtype, K, flags, scale);
  if (rc) return rc;
  if (acc_dtype != FJAGG_F32 || in_dtype == FJAGG_I32)
    return fail(FJAGG_EUNSUPPORTED, "fused l2 norms need float inputs and a float fold");
  if (K > kL2MaxClients)
    return fail(FJAGG_EUNSUPPORTED, "fused l2 norms support K <= %lld", (long long)kL2MaxClients);
  if (nblk < 1 || nblk > 0x7fffffff || !image_dev || !w_dev || L < 1)
    return fail(FJAGG_EINVAL, "bad plan (nblk=%lld, L=%d)", (long long)nblk, L);
  if (!ws_dev) return fail(FJAGG_EINVAL, "null pointer argument");
  if (ws_bytes < fjagg_wsum_l2_ptrs_workspace_bytes(K, nblk))
    return fail(FJAGG_EINVAL, "l2 workspace too small (need %lld bytes)",
                (long long)fjagg_wsum_l2_ptrs_workspace_bytes(K, nblk));
  float* ws = nullptr;
  out = l2_layout(out, ws_dev, K, flags, &ws);
  return wsum_ptrs_impl(in_dtype, acc_dtype, out_dtype, image_dev, L, K, nblk, w_dev, scale, flags, ws, out,
                        stream);
}
}  // namespace
extern "C" {

int fjagg_server_update_dense(int in_dtype, const void* x_dev, int64_t ld, int64_t K, int64_t P,
                              const float* w_dev, float scale, const fjagg_server_opt* opt,
                              float* params_dev, float* m_dev, float* v_dev, float* mean_dev,
                              int flags, void* stream) {
  g_err[0] = 0;
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16)
    return fail(FJAGG_EUNSUPPORTED, "server update: f32 or bf16 deltas");
  if (!opt_valid(opt)) return fail(FJAGG_EINVAL, "server update: bad optimizer descriptor");
  if (K < 1 || P < 1 || ld < P) return fail(FJAGG_EINVAL, "bad shape (K=%lld, P=%lld)", (long long)K, (long long)P);
  if (P * elem_bytes(in_dtype) > kMaxRowBytes) return fail(FJAGG_EUNSUPPORTED, "rows > 1 GiB");
  if (!x_dev || !w_dev || !params_dev) return fail(FJAGG_EINVAL, "null pointer argument");
  if (opt_needs_m(*opt) && !m_dev) return fail(FJAGG_EINVAL, "optimizer state m is null");
  if (opt_needs_v(*opt) && !v_dev) return fail(FJAGG_EINVAL, "optimizer state v is null");
  const int ib = elem_bytes(in_dtype), vw = vwidth(in_dtype);
  const uint8_t* x = reinterpret_cast<const uint8_t*>(x_dev);
  const bool vec = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && ((ld * ib) % 16 == 0) && P >= vw;
  const int V = vec ? vw : 1;
  DenseArgs a;
  a.x = x;
  a.ld_bytes = ld * ib;
  a.K = K;
  a.nunits = P / V;
  a.tail_n = (int)(P - a.nunits * V);
  a.w = w_dev;
  a.scale = scale;
  a.do_scale = 1;
  a.accumulate = 0;
  a.out = nullptr;
  a.kchunk = K;
  a.out_ystride = 0;
  a.balanced = true;
  const OptEpi epi{*opt, params_dev, m_dev, v_dev, mean_dev};
  const int variant = pick_variant(a.nunits, K);
  const bool nt = (flags & FJAGG_NONTEMPORAL) != 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (in_dtype == FJAGG_F32) return launch_dense_opt_io<FJAGG_F32>(vec, nt, variant, a, epi, s);
  return launch_dense_opt_io<FJAGG_BF16>(vec, nt, variant, a, epi, s);
}

int64_t fjagg_wsum_l2_workspace_bytes(int64_t K, int64_t P) {
  if (K < 1 || P < 1) return 0;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  (void)hipGetLastError();
  const int64_t max_blocks = (int64_t)cus * (2048 / kThreads) + 1;  // resident cap + tail block
  return kL2Header + max_blocks * round4(K) * 4;
}

int fjagg_wsum_l2_dense(int in_dtype, int acc_dtype, int out_dtype, const void* x_dev, int64_t ld,
                        int64_t K, int64_t P, const void* w_dev, float scale, void* out_dev,
                        float* l2sq_dev, int flags, void* ws_dev, int64_t ws_bytes, void* stream) {
  g_err[0] = 0;
  int rc = validate_common(in_dtype, acc_dtype, out_dtype, K, flags, scale);
  if (rc) return rc;
  if (acc_dtype != FJAGG_F32 || in_dtype == FJAGG_I32 || out_dtype == FJAGG_I32)
    return fail(FJAGG_EUNSUPPORTED, "fused l2 norms need float inputs and a float fold");
  if (K > kL2MaxClients)
    return fail(FJAGG_EUNSUPPORTED, "fused l2 norms support K <= %lld", (long long)kL2MaxClients);
  if (P < 1 || ld < P) return fail(FJAGG_EINVAL, "need 1 <= P <= ld");
  if (P * elem_bytes(in_dtype) > kMaxRowBytes)
    return fail(FJAGG_EUNSUPPORTED, "fused l2 norms need rows <= 1 GiB");
  if (!x_dev || !w_dev || !out_dev || !l2sq_dev || !ws_dev)
    return fail(FJAGG_EINVAL, "null pointer argument");
  const int ib = elem_bytes(in_dtype), vw = vwidth(in_dtype);
  const uint8_t* x = reinterpret_cast<const uint8_t*>(x_dev);
  uint8_t* y = reinterpret_cast<uint8_t*>(out_dev);
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) % 16 == 0) &&
                   ((ld * ib) % 16 == 0) && P >= vw;
  const int V = vec ? vw : 1;
  DenseArgs a;
  a.x = x;
  a.ld_bytes = ld * ib;
  a.K = K;
  a.nunits = P / V;
  a.tail_n = (int)(P - a.nunits * V);
  a.w = w_dev;
  a.scale = scale;
  a.do_scale = (flags & FJAGG_SCALE) ? 1 : 0;
  a.accumulate = (flags & FJAGG_ACCUMULATE) ? 1 : 0;
  a.out = y;
  a.kchunk = K;
  a.out_ystride = 0;
  a.balanced = true;
  const int variant = pick_variant(a.nunits, K);
  const bool nt = (flags & FJAGG_NONTEMPORAL) != 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* ws = nullptr;
  const L2Out l2 = l2_layout(L2Out{l2sq_dev, nullptr, 0, nullptr}, ws_dev, K, flags, &ws);
  const int64_t wsf = (ws_bytes - (flags & FJAGG_ZEROED_WS ? kL2Header : 0)) / 4;
  if (in_dtype == FJAGG_F32 && out_dtype == FJAGG_F32)
    return launch_dense_l2_io<FJAGG_F32, FJAGG_F32>(vec, nt, variant, a, ws, wsf, l2, s);
  if (in_dtype == FJAGG_BF16 && out_dtype == FJAGG_BF16)
    return launch_dense_l2_io<FJAGG_BF16, FJAGG_BF16>(vec, nt, variant, a, ws, wsf, l2, s);
  if (in_dtype == FJAGG_BF16 && out_dtype == FJAGG_F32)
    return launch_dense_l2_io<FJAGG_BF16, FJAGG_F32>(vec, nt, variant, a, ws, wsf, l2, s);
  return fail(FJAGG_EUNSUPPORTED, "fused l2 norms: unsupported dtype combination");
}

int64_t fjagg_l2sq_workspace_bytes(int64_t K, int64_t P) {
  if (K < 1 || P < 1) return 0;
  const int64_t per = 64 * 1024;  // elements per workgroup
  const int64_t nb = (P + per - 1) / per;
  return K * nb * 4;
}

int fjagg_l2sq_dense(int in_dtype, const void* x_dev, int64_t ld, int64_t K, int64_t P,
                     float* out_dev, void* ws_dev, int64_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16)
    return fail(FJAGG_EUNSUPPORTED, "l2sq supports f32 and bf16 inputs");
  if (K < 1 || P < 1 || ld < P) return fail(FJAGG_EINVAL, "bad shape");
  if (K > 65535) return fail(FJAGG_EINVAL, "l2sq: K > 65535 unsupported");
  const int64_t need = fjagg_l2sq_workspace_bytes(K, P);
  if (!ws_dev || ws_bytes < need)
    return fail(FJAGG_EINVAL, "l2sq needs %lld workspace bytes", (long long)need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t per = 64 * 1024, nb = (P + per - 1) / per;
  const int64_t ldb = ld * elem_bytes(in_dtype);
  float* ws = reinterpret_cast<float*>(ws_dev);
  const uint8_t* x = reinterpret_cast<const uint8_t*>(x_dev);
  dim3 grid((unsigned)nb, (unsigned)K);
  if (in_dtype == FJAGG_F32)
    hipLaunchKernelGGL(k_l2sq_partial<FJAGG_F32>, grid, dim3(kThreads), 0, s, x, ldb, P, per, ws);
  else
    hipLaunchKernelGGL(k_l2sq_partial<FJAGG_BF16>, grid, dim3(kThreads), 0, s, x, ldb, P, per, ws);
  int rc = check_launch("k_l2sq_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(k_l2sq_combine, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, ws, nb, K,
                     out_dev);
  return check_launch("k_l2sq_combine");
}

int64_t fjagg_l2sq_rows_workspace_bytes(int64_t R, int64_t max_n) {
  if (R < 1 || max_n < 1) return 0;
  const int64_t per = 64 * 1024;
  return R * ((max_n + per - 1) / per) * 4;
}

int fjagg_l2sq_rows(int in_dtype, const int64_t* image_dev, int64_t R, int64_t max_n,
                    int64_t rows_per_group, int take_sqrt, float* out_dev, void* ws_dev,
                    int64_t ws_bytes, void* stream) {
  g_err[0] = 0;
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16)
    return fail(FJAGG_EUNSUPPORTED, "l2sq supports f32 and bf16 inputs");
  if (R < 1 || max_n < 0 || rows_per_group < 1 || R % rows_per_group || R > 65535)
    return fail(FJAGG_EINVAL, "bad row grouping (R=%lld, rows_per_group=%lld)", (long long)R,
                (long long)rows_per_group);
  const int64_t per = 64 * 1024, nb = max_n > 0 ? (max_n + per - 1) / per : 1;
  const int64_t need = R * nb * 4;
  if (!ws_dev || ws_bytes < need || !image_dev || !out_dev)
    return fail(FJAGG_EINVAL, "l2sq_rows needs %lld workspace bytes", (long long)need);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* ws = reinterpret_cast<float*>(ws_dev);
  dim3 grid((unsigned)nb, (unsigned)R);
  if (in_dtype == FJAGG_F32)
    hipLaunchKernelGGL(k_l2sq_rows<FJAGG_F32>, grid, dim3(kThreads), 0, s, image_dev, R, per, ws);
  else
    hipLaunchKernelGGL(k_l2sq_rows<FJAGG_BF16>, grid, dim3(kThreads), 0, s, image_dev, R, per, ws);
  int rc = check_launch("k_l2sq_rows");
  if (rc) return rc;
  const int64_t G = R / rows_per_group;
  hipLaunchKernelGGL(k_l2sq_groups, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, s, ws, nb, G,
                     rows_per_group, take_sqrt, out_dev);
  return check_launch("k_l2sq_groups");
}

int fjagg_fill_synth(int dtype, void* x_dev, int64_t ld, int64_t K, int64_t P, int64_t k0,
                     uint64_t seed, float amp, void* stream) {
  g_err[0] = 0;
  if (K < 0 || P < 0 || ld < P) return fail(FJAGG_EINVAL, "bad shape");
  if (K == 0 || P == 0) return FJAGG_OK;
  if (!x_dev) return fail(FJAGG_EINVAL, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = K * P;
  int64_t nb = (total + kThreads - 1) / kThreads;
  if (nb > 65536) nb = 65536;
  uint8_t* x = reinterpret_cast<uint8_t*>(x_dev);
  if (dtype == FJAGG_F32)
    hipLaunchKernelGGL(k_fill<FJAGG_F32>, dim3((unsigned)nb), dim3(kThreads), 0, s, x, ld, K, P, k0,
                       seed, amp);
  else if (dtype == FJAGG_BF16)
    hipLaunchKernelGGL(k_fill<FJAGG_BF16>, dim3((unsigned)nb), dim3(kThreads), 0, s, x, ld, K, P, k0,
                       seed, amp);
  else
    return fail(FJAGG_EUNSUPPORTED, "fill supports f32 and bf16");
  return check_launch("k_fill");
}

}  // extern "C"
