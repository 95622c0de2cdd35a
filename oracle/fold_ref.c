/*
 * oracle/fold_ref.c — TEST INFRASTRUCTURE ONLY. CPU restatement of FedJAX's
 * weighted-mean aggregation, used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker / reported CPU baseline. Nothing
 * on the product path (fedjax_amd/) links, loads or calls this file.
 *
 * Reference restated: fedjax/core/tree_util.py @ google/fedjax 0.0.17
 *   tree_weight  :29-32   t = l * weight            (jit; weight cast to leaf dtype)
 *   _tree_add_eq :47-54   s = s + t                 (jit, donated: in place)
 *   tree_mean    :76-96   s_0 = t_0; s_k = s_{k-1} + t_k; W += w (Python f64)
 *   _tree_inverse_weight_eq :58-61   y = s * f32(1/W), or s * 0 when W <= 0
 * The arithmetic itself lives in XLA:CPU (jax/jaxlib, unpinned, setup.py:38-47):
 * elementwise IEEE-754 binary32 multiply and add, each in its own jit dispatch,
 * so no FMA contraction across them. This file is compiled with
 * -ffp-contract=off so the C compiler does not contract either.
 *
 * Parity pinning: the known-answer tests of the reference
 * (fedjax/aggregators/aggregator_test.py:24-37, fedjax/core/tree_util_test.py:27-62,
 * examples/fed_avg_test.py:52-56, fedjax/algorithms/fed_avg_test.py:57-61) are
 * checked against this restatement in tests/test_oracle.py.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- synthetic inputs: bit-identical to fjagg_fill_synth (fedjax_amd/csrc) ---- */
static inline uint64_t fj_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline float fj_synth(uint64_t seed, uint64_t k, uint64_t p, float amp) {
  uint64_t h = fj_mix64(seed ^ fj_mix64((k << 32) | (p & 0xffffffffull)));
  float u = (float)(uint32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f; /* exact */
  return amp * u;
}
static inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40); /* quiet NaN */
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

void oracle_fill_synth_f32(float* x, int64_t ld, int64_t K, int64_t P, int64_t k0,
                           uint64_t seed, float amp) {
  for (int64_t k = 0; k < K; ++k)
    for (int64_t p = 0; p < P; ++p) x[k * ld + p] = fj_synth(seed, (uint64_t)(k0 + k), (uint64_t)p, amp);
}
void oracle_fill_synth_bf16(uint16_t* x, int64_t ld, int64_t K, int64_t P, int64_t k0,
                            uint64_t seed, float amp) {
  for (int64_t k = 0; k < K; ++k)
    for (int64_t p = 0; p < P; ++p)
      x[k * ld + p] = f32_to_bf16(fj_synth(seed, (uint64_t)(k0 + k), (uint64_t)p, amp));
}
/* The same generator restricted to n sampled columns cols[] of clients k0..k0+K-1:
 * x[k * n + i] = synth(k0 + k, cols[i]); bf16 != 0 rounds each value to bf16 (RNE) and
 * returns it widened back to f32 (the value a bf16 slab holds). Lets a checker regenerate
 * exactly the columns it compares without the whole K x P slab. */
void oracle_synth_cols_f32(float* x, int64_t K, int64_t k0, const int64_t* cols, int64_t n,
                           uint64_t seed, float amp, int bf16) {
  for (int64_t k = 0; k < K; ++k)
    for (int64_t i = 0; i < n; ++i) {
      float v = fj_synth(seed, (uint64_t)(k0 + k), (uint64_t)cols[i], amp);
      x[k * n + i] = bf16 ? bf16_to_f32(f32_to_bf16(v)) : v;
    }
}

/* ---- single-pass restatement (same bits as the reference op sequence) ----
 * y[p] = fl(fold_k(fl(x_k[p]*w_k)) * scale); init: s_0 = t_0 (tree_util.py:89-91),
 * or s_0 = fl(y[p] + t_0) when accumulate != 0 (fedjax/algorithms/fed_avg.py:137-138). */
void oracle_wsum_f32(const float* x, int64_t ld, int64_t K, int64_t P, const float* w,
                     float scale, int apply_scale, int accumulate, float* y) {
  for (int64_t p = 0; p < P; ++p) {
    float s = x[p] * w[0];
    if (accumulate) s = y[p] + s;
    for (int64_t k = 1; k < K; ++k) {
      float t = x[k * ld + p] * w[k];
      s = s + t;
    }
    y[p] = apply_scale ? s * scale : s;
  }
}

/* f64 oracle for bf16 inputs (and error bounds): exact products, f64 sums. */
void oracle_wsum_bf16_f64(const uint16_t* x, int64_t ld, int64_t K, int64_t P,
                          const double* w, double scale, double* y) {
  for (int64_t p = 0; p < P; ++p) {
    double s = 0.0;
    for (int64_t k = 0; k < K; ++k) s += (double)bf16_to_f32(x[k * ld + p]) * w[k];
    y[p] = s * scale;
  }
}

/* Reference semantics for bf16 leaves: every op rounds to bf16 and the weak-typed
 * f32 weight / 1/W are rounded to bf16 first. Reported beside
 * the build's f32-accumulating result; not the parity target. */
void oracle_wsum_bf16_refsem(const uint16_t* x, int64_t ld, int64_t K, int64_t P,
                             const float* w, float scale, uint16_t* y) {
  for (int64_t p = 0; p < P; ++p) {
    float wb = bf16_to_f32(f32_to_bf16(w[0]));
    float s = bf16_to_f32(f32_to_bf16(bf16_to_f32(x[p]) * wb));
    for (int64_t k = 1; k < K; ++k) {
      wb = bf16_to_f32(f32_to_bf16(w[k]));
      float t = bf16_to_f32(f32_to_bf16(bf16_to_f32(x[k * ld + p]) * wb));
      s = bf16_to_f32(f32_to_bf16(s + t));
    }
    float sb = bf16_to_f32(f32_to_bf16(scale));
    y[p] = f32_to_bf16(s * sb);
  }
}

/* Per-element error bound of any summation order (DESIGN.md "tolerance"):
 * |y - y_ref| <= (K+2) * 2^-24 * |scale| * sum_k |fl(x_k w_k)| + 2^-24 |y_ref|. */
void oracle_wsum_bound_f32(const float* x, int64_t ld, int64_t K, int64_t P, const float* w,
                           float scale, const float* y_ref, double* bound) {
  const double u = ldexp(1.0, -24);
  for (int64_t p = 0; p < P; ++p) {
    double a = 0.0;
    for (int64_t k = 0; k < K; ++k) a += fabs((double)(x[k * ld + p] * w[k]));
    bound[p] = (double)(K + 2) * u * fabs((double)scale) * a + u * fabs((double)y_ref[p]);
  }
}

/* ---- the reference's op sequence, as the timed CPU baseline ----
 * Per client: allocate t = w*x (tree_weight returns a fresh buffer, :88), add it
 * into the running sum in place (_tree_add_eq donates the sum, :93), free t (:94);
 * finally scale in place (:96). Threads split the element range; each thread runs
 * the same per-element op sequence, so the bits do not depend on the thread count. */
struct refseq_job {
  const float* x;
  int64_t ld, K, p0, p1;
  const float* w;
  float scale;
  float* y;
};
static void* refseq_worker(void* arg) {
  struct refseq_job* j = (struct refseq_job*)arg;
  const int64_t n = j->p1 - j->p0;
  if (n <= 0) return NULL;
  float* s = j->y + j->p0;
  for (int64_t k = 0; k < j->K; ++k) {
    const float* xk = j->x + k * j->ld + j->p0;
    float* t = (float*)malloc((size_t)n * sizeof(float)); /* tree_weight's output */
    const float wk = j->w[k];
    for (int64_t p = 0; p < n; ++p) t[p] = xk[p] * wk;
    if (k == 0) {
      memcpy(s, t, (size_t)n * sizeof(float)); /* s_0 = t_0, owned, no copy in JAX */
    } else {
      for (int64_t p = 0; p < n; ++p) s[p] = s[p] + t[p];
    }
    free(t);
  }
  for (int64_t p = 0; p < n; ++p) s[p] = s[p] * j->scale;
  return NULL;
}
int oracle_tree_mean_refseq_f32(const float* x, int64_t ld, int64_t K, int64_t P,
                                const float* w, float scale, float* y, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 4096) nthreads = 4096;
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  struct refseq_job* jobs = (struct refseq_job*)calloc((size_t)nthreads, sizeof(struct refseq_job));
  int* spawned = (int*)calloc((size_t)nthreads, sizeof(int));
  if (!th || !jobs || !spawned) {
    free(th);
    free(jobs);
    free(spawned);
    return -1;
  }
  const int64_t chunk = ((P + nthreads - 1) / nthreads + 15) / 16 * 16;
  for (int i = 0; i < nthreads; ++i) {
    int64_t p0 = (int64_t)i * chunk, p1 = p0 + chunk;
    if (p0 > P) p0 = P;
    if (p1 > P) p1 = P;
    jobs[i] = (struct refseq_job){x, ld, K, p0, p1, w, scale, y};
    if (i == 0) continue;
    if (pthread_create(&th[i], NULL, refseq_worker, &jobs[i]) == 0)
      spawned[i] = 1;
    else
      refseq_worker(&jobs[i]); /* could not spawn: run this slice inline */
  }
  refseq_worker(&jobs[0]);
  for (int i = 1; i < nthreads; ++i)
    if (spawned[i]) pthread_join(th[i], NULL);
  free(th);
  free(jobs);
  free(spawned);
  return 0;
}
