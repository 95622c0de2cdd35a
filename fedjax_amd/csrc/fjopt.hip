// fjopt.hip — the adafactor server step (fedjax.optimizers.adafactor,
// fedjax/core/optimizers.py:284-348 = optax.adafactor). C ABI and arithmetic: include/fjopt.h.
//
// Adafactor's update of a leaf needs reductions that the fused fold epilogue of fjagg.h
// cannot give (means along the two factored axes, then a mean of those, then block RMS of
// the update and of the params), so it runs after the fold as a short chain of launches
// over ALL leaves at once (each launch a grid over a job table, block -> job by binary
// search on the jobs' first blocks):
//
//   Q0 reduce    f64 partial sums of g*g+eps along d0 and d1, and of p*p, over chunks of
//                the reduced axis ([O, N, I] views; thread per (chunk, o, i), coalesced
//                over i)
//   Q1 finalize  partials -> means -> v_row / v_col state (d*v + (1-d)*mean), and the
//                param block RMS
//   Q2 rcm       mean of the new v_row along d1
//   Q3 factors   row factors (v_row / rcm) ** -0.5, column factors v_col ** -0.5
//   Q4 usq       the scaled update u (unfactored leaves: the new v, stored) and f64
//                per-block sums of u*u (clip_by_block_rms)
//   Q5 clip      per-leaf clip denominator
//   Q6 apply     u again, then clip, lr, param scale, ema, weight decay, p -= u
//
// Every sum is accumulated in float64 in a fixed order (sequential per thread, then a
// fixed LDS tree), so the step is deterministic. Roofline: HBM — g is read 4 times (two
// reductions, Q4, Q6), p twice, p/m/v written once; the statistics are O(n / dim).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "fjagg.h"
#include "fjopt.h"

static_assert(sizeof(fjopt_af_leaf) == 112 && sizeof(fjopt_af_hparams) == 56, "layouts mirrored by _lib.AfLeaf / AfHparams");

extern thread_local char fjagg_g_err[512];

namespace {

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(fjagg_g_err, sizeof(fjagg_g_err), fmt, ap);
  va_end(ap);
  return code;
}

constexpr int kThreads = 256;
constexpr int64_t kElemsPerBlock = 4 * kThreads;  // Q4 / Q6: 4 elements per thread
constexpr int kPhases = 7;
constexpr int kHdrWords = 32, kLeafWords = 24, kJobWords = 16;

// table layout (int64 words): header | leaf records | jobs
enum Hdr { kHL = 21, kHLeafOff = 22, kHJobOff = 23, kHWs = 24, kHFlags = 25 };
enum Leaf {
  kLG, kLP, kLVRow, kLVCol, kLV, kLM, kLN, kLDims, kLFactored = kLDims + 5, kLD0Lo, kLDecayW, kLRf, kLCf, kLPrms,
  kLClipd, kLUsq, kLUsqBlocks, kLRcm
};
enum Job { kJType, kJLeaf, kJSrc, kJDst, kJAux, kJO, kJN, kJI, kJCh, kJS, kJBlk0, kJNblk, kJCount };
enum JobType { kRedG, kRedP, kFinV, kFinS, kRcm, kRowF, kColF, kUsq, kClip, kApply };
enum Flags { kFClip = 1, kFScale = 2, kFMom = 4 };

struct StepArgs {
  const int64_t* leaves;
  const int64_t* jobs;
  int64_t job0, njobs;
  uint8_t* ws;
  fjopt_af_hparams hp;
};

__device__ __forceinline__ const int64_t* find_job(const StepArgs& a, int64_t b, int64_t* local) {
  int64_t lo = a.job0, hi = a.job0 + a.njobs - 1;
  while (lo < hi) {  // last job with blk0 <= b
    int64_t mid = (lo + hi + 1) >> 1;
    if (a.jobs[mid * kJobWords + kJBlk0] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* j = a.jobs + lo * kJobWords;
  *local = b - j[kJBlk0];
  return j;
}

template <class T>
__device__ __forceinline__ T* at(uint8_t* ws, int64_t off) {
  return reinterpret_cast<T*>(ws + off);
}

// fixed-order workgroup sum of one double per thread (thread 0 gets the total)
__device__ __forceinline__ double block_sum(double v, double* lds) {
  const int t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
#pragma unroll
  for (int s = kThreads / 2; s > 0; s >>= 1) {
    if (t < s) lds[t] += lds[t + s];
    __syncthreads();
  }
  double r = lds[0];
  __syncthreads();
  return r;
}

// sum over n in [n0, n1) of f(load(n)) in n order, with U loads in flight (a loop of
// dependent load-then-add would wait one memory latency per term)
template <int U, class Load, class F>
__device__ __forceinline__ double ordered_sum(int64_t n0, int64_t n1, int64_t step, Load load, F f) {
  double acc = 0.0;
  int64_t n = n0;
  for (; n + (U - 1) * step < n1; n += U * step) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load(n + u * step);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += f(v[u]);
  }
  for (; n < n1; n += step) acc += f(load(n));
  return acc;
}

__device__ __forceinline__ float rsqrt_rn(float x) {  // x ** -0.5, correctly rounded via f64
  return (float)(1.0 / sqrt((double)x));
}
__device__ __forceinline__ float div_rn(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }

// the factored update factor indices of element i: v_row drops d0, v_col drops d1
struct Factored {
  int64_t A, nlo, B, nhi, C;
  bool d0lo;
  __device__ __forceinline__ void idx(int64_t i, int64_t* r, int64_t* c) const {
    int64_t cc = i % C, t = i / C;
    int64_t xh = t % nhi;
    t /= nhi;
    int64_t b = t % B;
    t /= B;
    int64_t xl = t % nlo, a = t / nlo;
    int64_t drop_lo = ((a * B + b) * nhi + xh) * C + cc;  // index without the lo axis
    int64_t drop_hi = ((a * nlo + xl) * B + b) * C + cc;  // without the hi axis
    *r = d0lo ? drop_lo : drop_hi;
    *c = d0lo ? drop_hi : drop_lo;
  }
};

__device__ __forceinline__ Factored factored_of(const int64_t* L) {
  return Factored{L[kLDims], L[kLDims + 1], L[kLDims + 2], L[kLDims + 3], L[kLDims + 4], L[kLD0Lo] != 0};
}

// u of element i before the block transforms (scale_by_factored_rms); stores the new v of
// an unfactored leaf when `store_v`
__device__ __forceinline__ float factored_rms_update(const int64_t* L, const StepArgs& a, int64_t i, float g,
                                                     bool store_v, bool v_is_new) {
  if (L[kLFactored]) {
    int64_t r, c;
    factored_of(L).idx(i, &r, &c);
    const float rf = at<float>(a.ws, L[kLRf])[r], cf = at<float>(a.ws, L[kLCf])[c];
    return __fmul_rn(__fmul_rn(g, rf), cf);  // grad * row_factor * col_factor
  }
  float* v = reinterpret_cast<float*>(L[kLV]);
  float nv;
  if (v_is_new) {
    nv = v[i];
  } else {
    const float gs = __fadd_rn(__fmul_rn(g, g), a.hp.eps);
    nv = __fadd_rn(__fmul_rn(a.hp.decay_rate_t, v[i]), __fmul_rn(a.hp.one_minus_decay, gs));
    if (store_v) v[i] = nv;
  }
  return __fmul_rn(g, rsqrt_rn(nv));
}

__global__ __launch_bounds__(kThreads) void k_af_reduce(StepArgs a) {
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t O = j[kJO], N = j[kJN], I = j[kJI], ch = j[kJCh], S = j[kJS];
  const int64_t t = lb * kThreads + threadIdx.x;
  if (j[kJAux]) {  // row mode (I == 1): a wave per (chunk, o), lanes along the row, xor tree
    const int64_t w = t >> 6;
    const int lane = threadIdx.x & 63;
    if (w >= S * O) return;  // whole waves
    const int64_t s = w / O, o = w % O;
    const float* x = reinterpret_cast<const float*>(j[kJSrc]) + o * N;
    const bool add_eps = j[kJType] == kRedG;
    const int64_t n1 = min(N, (s + 1) * ch);
    const float eps = a.hp.eps;
    double acc = ordered_sum<8>(s * ch + lane, n1, 64, [&](int64_t n) { return x[n]; }, [&](float v) {
      const float q = __fmul_rn(v, v);
      return (double)(add_eps ? __fadd_rn(q, eps) : q);
    });
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) at<double>(a.ws, j[kJDst])[s * O + o] = acc;
    return;
  }
  if (t >= S * O * I) return;
  const int64_t oi = t % (O * I), s = t / (O * I), o = oi / I, ii = oi % I;
  const float* x = reinterpret_cast<const float*>(j[kJSrc]);
  const bool add_eps = j[kJType] == kRedG;
  const float eps = a.hp.eps;
  const int64_t n1 = min(N, (s + 1) * ch);
  const float* xo = x + o * N * I + ii;
  const double acc = ordered_sum<8>(s * ch, n1, 1, [&](int64_t n) { return xo[n * I]; }, [&](float v) {
    const float q = __fmul_rn(v, v);
    return (double)(add_eps ? __fadd_rn(q, eps) : q);
  });
  at<double>(a.ws, j[kJDst])[s * O * I + oi] = acc;
}

__global__ __launch_bounds__(kThreads) void k_af_finalize(StepArgs a) {
  __shared__ double lds[kThreads];
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const double* part = at<double>(a.ws, j[kJSrc]);
  const int64_t S = j[kJS], N = j[kJN], cnt = j[kJCount];
  if (j[kJType] == kFinS) {  // param block RMS: max(sqrt(mean(p*p)), min_scale)
    double acc = 0.0;
    for (int64_t s = threadIdx.x; s < S; s += kThreads) acc += part[s];
    const double tot = block_sum(acc, lds);
    if (threadIdx.x == 0) {
      const float mean = (float)(tot / (double)N);
      at<float>(a.ws, j[kJDst])[0] = fmaxf(sqrt_rn(mean), a.hp.min_scale);
    }
    return;
  }
  if (j[kJAux]) {  // kFinV, many chunks: a wave per statistic, lanes over the chunks, xor tree
    const int64_t k = (lb * kThreads + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (k >= cnt) return;  // whole waves
    double acc = 0.0;
    for (int64_t s = lane; s < S; s += 64) acc += part[s * cnt + k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {
      const float mean = (float)(acc / (double)N);
      float* v = reinterpret_cast<float*>(j[kJDst]);
      v[k] = __fadd_rn(__fmul_rn(a.hp.decay_rate_t, v[k]), __fmul_rn(a.hp.one_minus_decay, mean));
    }
    return;
  }
  const int64_t k = lb * kThreads + threadIdx.x;  // kFinV: one statistic
  if (k >= cnt) return;
  double acc = 0.0;  // (S partials in chunk order, 8 loads in flight)
  int64_t s = 0;
  for (; s + 8 <= S; s += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(s + u) * cnt + k];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < S; ++s) acc += part[s * cnt + k];
  const float mean = (float)(acc / (double)N);
  float* v = reinterpret_cast<float*>(j[kJDst]);
  v[k] = __fadd_rn(__fmul_rn(a.hp.decay_rate_t, v[k]), __fmul_rn(a.hp.one_minus_decay, mean));
}

__global__ __launch_bounds__(kThreads) void k_af_rcm(StepArgs a) {
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t O = j[kJO], N = j[kJN], I = j[kJI];
  const int64_t k = lb * kThreads + threadIdx.x;
  if (k >= O * I) return;
  const int64_t o = k / I, ii = k % I;
  const float* v = reinterpret_cast<const float*>(j[kJSrc]) + o * N * I + ii;
  const double acc = ordered_sum<8>(0, N, 1, [&](int64_t n) { return v[n * I]; }, [](float x) { return (double)x; });
  at<float>(a.ws, j[kJDst])[k] = (float)(acc / (double)N);
}

__global__ __launch_bounds__(kThreads) void k_af_factors(StepArgs a) {
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t k = lb * kThreads + threadIdx.x;
  if (k >= j[kJCount]) return;
  const float* v = reinterpret_cast<const float*>(j[kJSrc]);
  float* out = at<float>(a.ws, j[kJDst]);
  if (j[kJType] == kRowF) {  // (v_row / row_col_mean) ** -0.5; rcm index drops v_row's d1 axis
    const int64_t N = j[kJN], I = j[kJI];
    const float rcm = at<float>(a.ws, j[kJAux])[(k / (N * I)) * I + k % I];
    out[k] = rsqrt_rn(div_rn(v[k], rcm));
  } else {  // v_col ** -0.5
    out[k] = rsqrt_rn(v[k]);
  }
}

__global__ __launch_bounds__(kThreads) void k_af_usq(StepArgs a) {
  __shared__ double lds[kThreads];
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t* L = a.leaves + j[kJLeaf] * kLeafWords;
  const int64_t n = L[kLN];
  const float* g = reinterpret_cast<const float*>(L[kLG]);
  const bool clip = a.hp.clip != 0;
  double acc = 0.0;
  const int64_t e0 = lb * kElemsPerBlock;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i = e0 + q * kThreads + threadIdx.x;
    if (i < n) {
      const float u = factored_rms_update(L, a, i, g[i], true, false);
      acc += (double)__fmul_rn(u, u);
    }
  }
  if (!clip) return;  // (launched for the v update of unfactored leaves only)
  const double tot = block_sum(acc, lds);
  if (threadIdx.x == 0) at<double>(a.ws, L[kLUsq])[lb] = tot;
}

__global__ __launch_bounds__(kThreads) void k_af_clip(StepArgs a) {
  __shared__ double lds[kThreads];
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t* L = a.leaves + j[kJLeaf] * kLeafWords;
  const double* part = at<double>(a.ws, L[kLUsq]);
  const int64_t S = L[kLUsqBlocks];
  double acc = 0.0;
  for (int64_t s = threadIdx.x; s < S; s += kThreads) acc += part[s];
  const double tot = block_sum(acc, lds);
  if (threadIdx.x == 0) {
    const float mean = (float)(tot / (double)L[kLN]);
    // jnp.maximum(1.0, jnp.sqrt(jnp.mean(abs_sq(u))) / threshold)
    at<float>(a.ws, L[kLClipd])[0] = fmaxf(1.0f, div_rn(sqrt_rn(mean), a.hp.clip_threshold));
  }
}

__global__ __launch_bounds__(kThreads) void k_af_apply(StepArgs a) {
  int64_t lb;
  const int64_t* j = find_job(a, blockIdx.x, &lb);
  const int64_t* L = a.leaves + j[kJLeaf] * kLeafWords;
  const int64_t n = L[kLN];
  const float* g = reinterpret_cast<const float*>(L[kLG]);
  float* p = reinterpret_cast<float*>(L[kLP]);
  float* m = reinterpret_cast<float*>(L[kLM]);
  const fjopt_af_hparams& hp = a.hp;
  const float clipd = hp.clip ? at<float>(a.ws, L[kLClipd])[0] : 1.0f;
  const float prms = hp.param_scale ? at<float>(a.ws, L[kLPrms])[0] : 1.0f;
  const bool wd = hp.weight_decay && L[kLDecayW];
  const int64_t e0 = lb * kElemsPerBlock;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i = e0 + q * kThreads + threadIdx.x;
    if (i >= n) continue;
    // unfactored leaves: Q4 stored the new v; without clipping Q4 ran for that alone
    float u = factored_rms_update(L, a, i, g[i], false, true);
    if (hp.clip) u = div_rn(u, clipd);
    if (hp.has_lr) u = __fmul_rn(u, hp.lr);
    const float pi = p[i];
    if (hp.param_scale) u = __fmul_rn(u, prms);
    if (hp.momentum) {
      u = __fadd_rn(__fmul_rn(hp.one_minus_mom, u), __fmul_rn(hp.mom_decay, m[i]));
      m[i] = u;
    }
    if (wd) u = __fadd_rn(u, __fmul_rn(hp.wd, pi));
    p[i] = __fadd_rn(pi, -u);  // scale(-1), apply_updates
  }
}

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

extern "C" {

int fjopt_abi_version(void) { return FJOPT_ABI_VERSION; }

int64_t fjopt_adafactor_plan(const fjopt_af_leaf* leaves, int L, const fjopt_af_hparams* hp, int64_t* table,
                             int64_t table_words, int64_t* ws_bytes) {
  fjagg_g_err[0] = 0;
  if (L < 1 || !leaves || !hp || !ws_bytes) return fail(FJAGG_EINVAL, "fjopt_adafactor_plan: L >= 1, leaves, hp, ws_bytes");
  const bool clip = hp->clip != 0, pscale = hp->param_scale != 0, mom = hp->momentum != 0;
  for (int l = 0; l < L; ++l) {
    const fjopt_af_leaf& f = leaves[l];
    if (f.n < 1 || !f.g || !f.p) return fail(FJAGG_EINVAL, "leaf %d: n >= 1, g and p", l);
    if (mom && !f.m) return fail(FJAGG_EINVAL, "leaf %d: momentum needs m", l);
    int64_t prod = 1;
    for (int d = 0; d < 5; ++d) {
      if (f.dims[d] < 1) return fail(FJAGG_EINVAL, "leaf %d: dims must be >= 1", l);
      prod *= f.dims[d];
    }
    if (prod != f.n) return fail(FJAGG_EINVAL, "leaf %d: dims do not multiply to n", l);
    if (f.factored ? (!f.v_row || !f.v_col) : !f.v) return fail(FJAGG_EINVAL, "leaf %d: missing state", l);
  }
  // jobs per phase
  struct J {
    int64_t w[kJobWords];
  };
  std::vector<J> ph[kPhases];
  std::vector<int64_t> recs((size_t)L * kLeafWords, 0);
  int64_t ws = 0;
  auto alloc = [&](int64_t bytes) {
    int64_t o = ws;
    ws += (bytes + 255) & ~int64_t(255);
    return o;
  };
  auto job = [&](int q, int type, int l, int64_t src, int64_t dst, int64_t aux, int64_t O, int64_t N, int64_t I,
                 int64_t ch, int64_t S, int64_t count, int64_t nblk) {
    J j{};
    j.w[kJType] = type;
    j.w[kJLeaf] = l;
    j.w[kJSrc] = src;
    j.w[kJDst] = dst;
    j.w[kJAux] = aux;
    j.w[kJO] = O;
    j.w[kJN] = N;
    j.w[kJI] = I;
    j.w[kJCh] = ch;
    j.w[kJS] = S;
    j.w[kJCount] = count;
    j.w[kJNblk] = nblk;
    ph[q].push_back(j);
  };
  // an [O, N, I] axis sum: S chunks of ch rows, ~64 K threads in all (at least one row each)
  // an [O, N, I] axis sum in S chunks of ch rows. I > 1: a thread per (chunk, o, i),
  // coalesced over i, ~64 K threads in all. I == 1 (rows): a wave per (chunk, o), chunks of
  // >= 256 elements, <= ~64 K waves.
  auto reduce = [&](int type, int l, const float* src, int64_t O, int64_t N, int64_t I, int64_t* S_out) {
    const bool rows = I == 1 && N >= 64;
    int64_t ch;
    if (rows) {
      ch = ceil_div(N * O, 65536);
      ch = ch < 256 ? 256 : ch;
    } else {
      int64_t S = ceil_div(65536, O * I);
      S = S < 1 ? 1 : (S > N ? N : S);
      ch = ceil_div(N, S);
    }
    ch = ch > N ? N : ch;
    const int64_t S = ceil_div(N, ch);
    const int64_t part = alloc(8 * S * O * I);
    const int64_t threads = rows ? S * O * 64 : S * O * I;
    job(0, type, l, (int64_t)src, part, rows ? 1 : 0, O, N, I, ch, S, S * O * I, ceil_div(threads, kThreads));
    *S_out = S;
    return part;
  };
  for (int l = 0; l < L; ++l) {
    const fjopt_af_leaf& f = leaves[l];
    int64_t* r = recs.data() + (size_t)l * kLeafWords;
    r[kLG] = (int64_t)f.g;
    r[kLP] = (int64_t)f.p;
    r[kLVRow] = (int64_t)f.v_row;
    r[kLVCol] = (int64_t)f.v_col;
    r[kLV] = (int64_t)f.v;
    r[kLM] = (int64_t)f.m;
    r[kLN] = f.n;
    for (int d = 0; d < 5; ++d) r[kLDims + d] = f.dims[d];
    r[kLFactored] = f.factored != 0;
    r[kLD0Lo] = f.d0_is_lo != 0;
    r[kLDecayW] = f.decay_weights != 0;
    const int64_t A = f.dims[0], nlo = f.dims[1], B = f.dims[2], nhi = f.dims[3], C = f.dims[4];
    if (f.factored) {
      // sums over the lo axis ([A, nlo, B*nhi*C]) and over the hi axis ([A*nlo*B, nhi, C])
      int64_t Slo, Shi;
      const int64_t plo = reduce(kRedG, l, f.g, A, nlo, B * nhi * C, &Slo);
      const int64_t phi = reduce(kRedG, l, f.g, A * nlo * B, nhi, C, &Shi);
      const int64_t drop_lo = A * B * nhi * C, drop_hi = A * nlo * B * C;
      // v_row = mean over d0, v_col = mean over d1
      float* vr = f.v_row;
      float* vc = f.v_col;
      // (>= 64 chunks: a wave per statistic)
      auto fin = [&](int64_t part, float* v, int64_t N, int64_t S, int64_t cnt) {
        const bool waves = S >= 64;
        job(1, kFinV, l, part, (int64_t)v, waves ? 1 : 0, 0, N, 0, 0, S, cnt,
            ceil_div(waves ? cnt * 64 : cnt, kThreads));
      };
      if (f.d0_is_lo) {
        fin(plo, vr, nlo, Slo, drop_lo);
        fin(phi, vc, nhi, Shi, drop_hi);
      } else {
        fin(phi, vr, nhi, Shi, drop_hi);
        fin(plo, vc, nlo, Slo, drop_lo);
      }
      // row_col_mean: mean of v_row along d1 (v_row = [A, B, nhi, C] when d0 is lo, else [A, nlo, B, C])
      const int64_t rO = f.d0_is_lo ? A * B : A, rN = f.d0_is_lo ? nhi : nlo, rI = f.d0_is_lo ? C : B * C;
      r[kLRcm] = alloc(4 * rO * rI);
      job(2, kRcm, l, (int64_t)vr, r[kLRcm], 0, rO, rN, rI, 0, 0, rO * rI, ceil_div(rO * rI, kThreads));
      const int64_t nr = f.d0_is_lo ? drop_lo : drop_hi, nc = f.d0_is_lo ? drop_hi : drop_lo;
      r[kLRf] = alloc(4 * nr);
      r[kLCf] = alloc(4 * nc);
      job(3, kRowF, l, (int64_t)vr, r[kLRf], r[kLRcm], 0, rN, rI, 0, 0, nr, ceil_div(nr, kThreads));
      job(3, kColF, l, (int64_t)vc, r[kLCf], 0, 0, 0, 0, 0, 0, nc, ceil_div(nc, kThreads));
    }
    if (pscale) {
      int64_t Sp;
      const int64_t pp = reduce(kRedP, l, f.p, 1, f.n, 1, &Sp);
      r[kLPrms] = alloc(4);
      job(1, kFinS, l, pp, r[kLPrms], 0, 0, f.n, 0, 0, Sp, 1, 1);
    }
    const int64_t eb = ceil_div(f.n, kElemsPerBlock);
    if (clip || !f.factored) {
      r[kLUsqBlocks] = eb;
      if (clip) r[kLUsq] = alloc(8 * eb);
      job(4, kUsq, l, 0, 0, 0, 0, 0, 0, 0, 0, f.n, eb);
    }
    if (clip) {
      r[kLClipd] = alloc(4);
      job(5, kClip, l, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1);
    }
    job(6, kApply, l, 0, 0, 0, 0, 0, 0, 0, 0, f.n, eb);
  }
  int64_t njobs = 0;
  for (int q = 0; q < kPhases; ++q) njobs += (int64_t)ph[q].size();
  const int64_t words = kHdrWords + (int64_t)L * kLeafWords + njobs * kJobWords;
  *ws_bytes = ws > 0 ? ws : 256;
  if (!table) return words;
  if (table_words < words) return fail(FJAGG_EINVAL, "fjopt_adafactor_plan: table needs %lld words", (long long)words);
  memset(table, 0, sizeof(int64_t) * kHdrWords);
  int64_t j0 = 0;
  int64_t* jobs = table + kHdrWords + (int64_t)L * kLeafWords;
  for (int q = 0; q < kPhases; ++q) {
    int64_t blk = 0;
    table[3 * q] = j0;
    table[3 * q + 1] = (int64_t)ph[q].size();
    for (J& j : ph[q]) {
      j.w[kJBlk0] = blk;
      blk += j.w[kJNblk];
      memcpy(jobs + j0 * kJobWords, j.w, sizeof(j.w));
      ++j0;
    }
    table[3 * q + 2] = blk;
    if (blk > INT32_MAX) return fail(FJAGG_EINVAL, "fjopt_adafactor_plan: grid too large");
  }
  table[kHL] = L;
  table[kHLeafOff] = kHdrWords;
  table[kHJobOff] = kHdrWords + (int64_t)L * kLeafWords;
  table[kHWs] = *ws_bytes;
  table[kHFlags] = (clip ? kFClip : 0) | (pscale ? kFScale : 0) | (mom ? kFMom : 0);
  memcpy(table + kHdrWords, recs.data(), sizeof(int64_t) * recs.size());
  return words;
}

int fjopt_adafactor_step(const int64_t* table_host, const int64_t* table_dev, const fjopt_af_hparams* hp, void* ws,
                         int64_t ws_bytes, void* stream) {
  fjagg_g_err[0] = 0;
  if (!table_host || !table_dev || !hp || !ws) return fail(FJAGG_EINVAL, "fjopt_adafactor_step: null argument");
  const int flags = (hp->clip ? kFClip : 0) | (hp->param_scale ? kFScale : 0) | (hp->momentum ? kFMom : 0);
  if (flags != table_host[kHFlags]) return fail(FJAGG_EINVAL, "fjopt_adafactor_step: hp flags differ from the plan's");
  if (ws_bytes < table_host[kHWs]) return fail(FJAGG_EINVAL, "fjopt_adafactor_step: workspace smaller than planned");
  if (reinterpret_cast<uintptr_t>(ws) % 256 != 0) return fail(FJAGG_EINVAL, "fjopt_adafactor_step: workspace alignment");
  StepArgs a;
  a.leaves = table_dev + table_host[kHLeafOff];
  a.jobs = table_dev + table_host[kHJobOff];
  a.ws = static_cast<uint8_t*>(ws);
  a.hp = *hp;
  hipStream_t s = static_cast<hipStream_t>(stream);
  void (*kernels[kPhases])(StepArgs) = {k_af_reduce, k_af_finalize, k_af_rcm, k_af_factors,
                                        k_af_usq,    k_af_clip,     k_af_apply};
  for (int q = 0; q < kPhases; ++q) {
    a.job0 = table_host[3 * q];
    a.njobs = table_host[3 * q + 1];
    const int64_t nb = table_host[3 * q + 2];
    if (a.njobs == 0 || nb == 0) continue;
    hipLaunchKernelGGL(kernels[q], dim3((unsigned)nb), dim3(kThreads), 0, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FJAGG_EHIP, "fjopt_adafactor_step phase %d: %s", q, hipGetErrorString(e));
  }
  return FJAGG_OK;
}

}  // extern "C"
