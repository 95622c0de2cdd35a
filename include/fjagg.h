/*
 * fjagg.h — C ABI of the MI355X-native FedJAX aggregation library (libfjagg.so).
 *
 * This library replaces the arithmetic of FedJAX's server-side client-update
 * aggregation, i.e. the weighted fold that `fedjax.tree_util.tree_mean` performs
 * over K client-delta pytrees:
 *
 *     reference                                   replaced by
 *     ------------------------------------------  ---------------------------------
 *     tree_weight   fedjax/core/tree_util.py:29-32  fjagg_wsum_* (per-client multiply)
 *     _tree_add_eq  fedjax/core/tree_util.py:47-54  fjagg_wsum_* (fused running add)
 *     _tree_inverse_weight_eq  tree_util.py:58-61   fjagg_wsum_* with FJAGG_SCALE
 *     tree_mean loop tree_util.py:76-96             one fjagg_wsum_* launch per bucket
 *     tree_sum       tree_util.py:64-73             fjagg_wsum_* with unit weights
 *     tree_add       tree_util.py:47-50             fjagg_wsum_* K=2, unit weights
 *     tree_l2_squared tree_util.py:105-108          fjagg_l2sq_*
 *
 * The reference has no native code: each of those rows is a `jax.jit` dispatch
 * into XLA. The Python mirror of the reference's API
 * (fedjax_amd/tree_util.py, fedjax_amd/aggregators/) is the only caller inside
 * this repository; INTEGRATION.md shows the ctypes binding a FedJAX maintainer
 * would add.
 *
 * Conventions
 *   - every entry point returns 0 on success or a negative FJAGG_E* code; the
 *     message of the last failure on the calling thread is fjagg_last_error().
 *   - every launch is asynchronous on the given hipStream_t (passed as void*;
 *     NULL = the null stream). No entry point allocates, frees or synchronises,
 *     so launches may be captured into a hipGraph.
 *   - pointers named *_dev are device pointers; everything else is host memory.
 *   - inputs are never written (reference ownership rule, tree_util_test.py:50-51).
 *
 * Arithmetic contract (FJAGG_MODE_EXACT, the default): for every element p
 *     t_k = fl(x_k[p] * w_k)            (IEEE single, round to nearest, no FMA)
 *     s_0 = t_0                          (s_0 = fl(out[p] + t_0) with FJAGG_ACCUMULATE)
 *     s_k = fl(s_{k-1} + t_k)            k = 1 .. K-1, in client order
 *     out[p] = fl(s_{K-1} * scale)       with FJAGG_SCALE, else s_{K-1}
 * which is bit-for-bit the sequence XLA executes for tree_mean.
 * FJAGG_MODE_SPLIT folds contiguous client ranges independently and combines
 * the range sums in range order: not bitwise, within the bound in DESIGN.md.
 */
#ifndef FJAGG_H_
#define FJAGG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FJAGG_ABI_VERSION 3

/* element types */
enum fjagg_dtype {
  FJAGG_F32 = 0,   /* IEEE binary32 */
  FJAGG_BF16 = 1,  /* bfloat16 (stored as uint16) */
  FJAGG_I32 = 2,   /* two's complement int32, wrapping arithmetic like XLA */
};

/* flags (bitwise OR) */
enum fjagg_flags {
  FJAGG_SCALE = 1 << 0,       /* multiply the fold by `scale` (tree_mean's f32(1/W)) */
  FJAGG_ACCUMULATE = 1 << 1,  /* fold starts from the current contents of the output */
  FJAGG_NONTEMPORAL = 1 << 2, /* non-temporal (streaming) loads of the client deltas */
  FJAGG_UNALIGNED = 1 << 3,   /* ptrs path: some pointer is not 16-byte aligned */
  FJAGG_UNBALANCED = 1 << 4,  /* dense path: one tile per workgroup instead of a balanced
                                 resident grid (tuning / A-B only) */
  FJAGG_NARROW = 1 << 5,      /* pytree path, plan AND launch: 64-element stripes per workgroup,
                                 client rows staged through LDS (k_ptrs_narrow) — for small
                                 leaves and many clients; fold only (no fused norms). With
                                 FJAGG_VARIANT(20 / 21 / 22) in both calls: stripes of 64 / 32 / 16
                                 elements folded by the stripe pipeline (k_ptrs_stripe: LDS-
                                 transposed products, one fold wave per stripe); every client and
                                 output pointer must then be 16-byte aligned */
  FJAGG_HOST_TABLES = 1 << 6, /* the weights (and on the pytree path the plan image) are HOST
                                 pointers: the launch copies them into the kernel arguments, so
                                 no upload or staging copy runs on the stream before the fold and
                                 the caller's buffers are free again when the call returns.
                                 Dense: K <= FJAGG_KARG_MAX_WEIGHTS, (in, acc, out) one of
                                 (F32,F32,F32) (BF16,F32,BF16) (BF16,F32,F32), not FJAGG_NARROW
                                 shapes. Pytree: (F32,F32,F32), 16-byte units (no FJAGG_UNALIGNED,
                                 no FJAGG_NARROW), fjagg_karg_image_words(K, L, nblk) <=
                                 FJAGG_KARG_MAX_WORDS. Anything else returns FJAGG_EUNSUPPORTED
                                 (nothing launched): upload the tables and call without the flag. */
  FJAGG_ZEROED_WS = 1 << 7,   /* fused-norm calls (fjagg_wsum_l2_*): the workspace's first 16 bytes
                                 are a completion counter that is zero before the call — zero it
                                 once when the workspace is allocated; every call leaves it zero —
                                 and the norm partials follow it. With K <= 128 and a 16-byte
                                 aligned workspace the fold's last workgroup then adds the
                                 partials itself, with no second (combine) launch; the norms are
                                 bitwise the same either way. Without the flag the 16 bytes are
                                 unused. As always, one workspace serves one call at a time.
                                 Bytes 4..7 are an error word: a call that finds the counter
                                 non-zero sets it to 1 (sticky: that call's norms are not valid;
                                 zero both words to recover).
                                 Graph capture: zero it before the capture (every replayed call
                                 leaves it zero) or with a kernel inside it; a hipMemsetAsync
                                 recorded into a graph acts on the first replay only (ROCm 7,
                                 measured: tools/probe_memset_node.py).
                                 (fedjax_amd's callers pass it unless FJAGG_L2_COMBINE_LAUNCH=1.) */
};
/* kernel-argument capacity of FJAGG_HOST_TABLES launches */
#define FJAGG_KARG_MAX_WEIGHTS 1024 /* dense path: 4 KiB of weights */
#define FJAGG_KARG_MAX_WORDS 3584   /* pytree path: 28 KiB = image words + ceil(K/2) weight words */
/* bits 8..15 of flags select a kernel shape of the dense path: 0 = automatic,
 * 1..17 = fixed (units per lane, clients in flight, waves/SIMD) for tuning, 18 = the
 * LDS-staged narrow fold, 19 = the stripe pipeline (fjstripe.hip) with automatic stripe
 * width, 20 / 21 / 22 = with 64 / 32 / 16 columns; see fjagg.hip */
#define FJAGG_VARIANT(v) (((v)&0xff) << 8)

enum fjagg_mode {
  FJAGG_MODE_EXACT = 0, /* sequential per-element fold: bitwise equal to the reference */
  FJAGG_MODE_SPLIT = 1, /* client axis split over workgroups, ordered combine */
};

/* error codes */
#define FJAGG_OK 0
#define FJAGG_EINVAL (-1)
#define FJAGG_EHIP (-2)
#define FJAGG_EUNSUPPORTED (-3)

/* Message of the last failed call on this thread ("" if none). */
const char* fjagg_last_error(void);
/* FJAGG_ABI_VERSION of the loaded library. */
int fjagg_abi_version(void);

/*
 * Dense client-major slab: client k's delta is x_dev + k*ld elements, P
 * contiguous elements each. acc_dtype is FJAGG_F32 (w_dev is float[K]),
 * FJAGG_I32 (integer fold, w_dev is int32[K]) or FJAGG_BF16 (the reference's bfloat16
 * arithmetic, w_dev is float[K]: each weight and the scale are rounded to bf16, every
 * product and sum is rounded to bf16 — jnp on bf16 leaves with weakly typed weights,
 * tree_util.py:32,50,60). Supported (in, acc, out):
 *   (F32,F32,F32) (F32,F32,BF16) (BF16,F32,BF16) (BF16,F32,F32) (I32,F32,F32) (I32,I32,I32)
 *   (I32,I32,F32) (BF16,BF16,BF16); the pytree path supports the same set except
 *   (F32,F32,BF16).
 * mode FJAGG_MODE_SPLIT needs ws_dev of fjagg_split_workspace_bytes(K, P) bytes
 * (ws may be NULL in exact mode); acc FJAGG_BF16 runs in exact mode only.
 * Replaces: the per-client loop of tree_mean, fedjax/core/tree_util.py:85-96.
 */
int fjagg_wsum_dense(int in_dtype, int acc_dtype, int out_dtype, const void* x_dev,
                     int64_t ld, int64_t K, int64_t P, const void* w_dev, float scale,
                     void* out_dev, int flags, int mode, void* ws_dev, int64_t ws_bytes,
                     void* stream);

/* Workspace bytes FJAGG_MODE_SPLIT needs for a K x P fold (0 if split is not used). */
int64_t fjagg_split_workspace_bytes(int64_t K, int64_t P);

/*
 * Pytree path: K clients x L leaves, each leaf a separate allocation.
 * Launches ONE kernel over every leaf. The plan image is an int64 array in
 * device memory laid out as
 *     in_ptrs [K*L]    client k, leaf l at k*L + l (device addresses)
 *     out_ptrs[L]
 *     leaf_n  [L]      elements per leaf
 *     blocks  [2*nblk] from fjagg_ptrs_plan(): per workgroup (first unit | leaf | tail
 *                      flag | element flag, end unit), unit ranges balanced across the CUs
 * Replaces: jax.tree.map over leaves inside tree_weight/tree_add,
 * fedjax/core/tree_util.py:32,50, for the whole tree_mean loop :85-96.
 */
/* Fills blocks[] (2 int64 per workgroup, up to blocks_cap workgroups) for leaves of
 * leaf_n[l] elements and returns the number of workgroups the plan needs (negative
 * FJAGG_E* on error); call with blocks_cap = 0 to size the array. flags: FJAGG_UNALIGNED if any client or
 * output pointer is not 16-byte aligned (the same flag must go to the launch). */
int64_t fjagg_ptrs_plan(int in_dtype, int flags, const int64_t* leaf_n, int L, int64_t* blocks,
                        int64_t blocks_cap);
/* fjagg_ptrs_plan with a per-leaf choice of unit: leaf_elem[l] != 0 marks a leaf whose
 * client or output pointers are not all 16-byte aligned. Its workgroups walk single
 * elements (the element flag, bit 63 of block word 0; ranges of as many units as the
 * vector ranges, since a workgroup's time is its walks over the K clients) while every other leaf keeps
 * 16-byte units, so one misaligned leaf does not slow the whole launch. Launch the
 * plan WITHOUT FJAGG_UNALIGNED. leaf_elem == NULL is fjagg_ptrs_plan. Replaces the same
 * reference loop as fjagg_ptrs_plan (tree_util.py:85-96); a caller-held pytree may be
 * views into one buffer at any element offset (e.g. deserialized msgpack leaves,
 * fedjax/core/serialization.py:79-87). */
int64_t fjagg_ptrs_plan_leaves(int in_dtype, int flags, const int64_t* leaf_n, const uint8_t* leaf_elem,
                               int L, int64_t* blocks, int64_t blocks_cap);
int fjagg_wsum_ptrs(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev,
                    int L, int64_t K, int64_t nblk, const void* w_dev, float scale,
                    int flags, void* stream);
/* int64 words a FJAGG_HOST_TABLES pytree launch carries in its kernel arguments: the
 * image (K*L + 2*L + 2*nblk words; image_dev and w_dev are then host pointers) and the
 * K f32 weights packed two per word. Compare with FJAGG_KARG_MAX_WORDS. */
int64_t fjagg_karg_image_words(int64_t K, int L, int64_t nblk);

/*
 * fjagg_wsum_ptrs fused with every client's squared L2 norm over ALL L leaves, in the
 * same pass (same plan image and nblk as fjagg_wsum_ptrs; the outputs are bitwise
 * the fjagg_wsum_ptrs ones). l2sq_dev[k] = sum over leaves and elements of x^2 in f32,
 * fixed order: per lane a packed-FMA sum of its units' squares -> the wave's lanes by
 * v_permlane32_swap / v_permlane16_swap and DPP row rotations (groups of clients at once)
 * -> LDS per wave -> workgroup partials ws[b*K + k] added in workgroup order (XLA's own
 * reduction order is not pinned; the tests bound it against an f64 norm) by a second launch,
 * or by the fold's last workgroup under FJAGG_ZEROED_WS. Float inputs, float fold, K <= 4096;
 * ws_dev of fjagg_wsum_l2_ptrs_workspace_bytes(K, nblk) bytes.
 * Replaces the per-client tree_l2_norm(delta) of examples/fed_avg.py:79-81
 * (tree_util.py:105-114) next to the tree_mean of the same deltas (:82).
 */
int64_t fjagg_wsum_l2_ptrs_workspace_bytes(int64_t K, int64_t nblk);
int fjagg_wsum_l2_ptrs(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev,
                       int L, int64_t K, int64_t nblk, const void* w_dev, float scale,
                       float* l2sq_dev, int flags, void* ws_dev, int64_t ws_bytes, void* stream);
/*
 * fjagg_wsum_l2_ptrs writing the norms where a deferred running sum's lazy norm views read
 * them: operand k >= first gets its squared norm in sq_dev[k - first] and its correctly
 * rounded square root in norm_dev[k - first] (either may be NULL, not both); operands below
 * `first` are not written. The per-client delta_l2_norm of the library loop
 * (fedjax/algorithms/fed_avg.py:142-144, tree_util.py:111-114) straight from the fold's norm
 * combine, without a separate fill launch. 0 <= first <= K.
 */
int fjagg_wsum_l2_ptrs_rows(int in_dtype, int acc_dtype, int out_dtype, const int64_t* image_dev,
                            int L, int64_t K, int64_t nblk, const void* w_dev, float scale,
                            float* sq_dev, float* norm_dev, int64_t first, int flags, void* ws_dev,
                            int64_t ws_bytes, void* stream);

/*
 * fjagg_wsum_dense (exact mode) fused with the per-client squared L2 norms of the
 * same deltas, in ONE pass over the K x P slab: out as fjagg_wsum_dense (bitwise
 * the same), l2sq_dev[k] = sum_p x_k[p]^2 in f32 with a fixed reduction order
 * (lane partials -> wave xor-butterfly -> LDS per wave -> workgroups in order).
 * Replaces the per-client tree_l2_norm pass of examples/fed_avg.py:79-81 and
 * fedjax/algorithms/fed_avg.py:142-144 (tree_util.py:105-114) for the whole round.
 * Float inputs (f32, bf16), float fold, K <= 4096, rows <= 1 GiB.
 */
int64_t fjagg_wsum_l2_workspace_bytes(int64_t K, int64_t P);
int fjagg_wsum_l2_dense(int in_dtype, int acc_dtype, int out_dtype, const void* x_dev,
                        int64_t ld, int64_t K, int64_t P, const void* w_dev, float scale,
                        void* out_dev, float* l2sq_dev, int flags, void* ws_dev,
                        int64_t ws_bytes, void* stream);

/*
 * Server optimizer step fused into the fold's epilogue. The round's mean
 * g = fl(fold * scale) (bitwise the fjagg_wsum_dense value) is consumed in
 * registers by the server optimizer of examples/fed_avg.py:97-101 /
 * fedjax/algorithms/fed_avg.py:150-154, restating optax's op sequence
 * (fedjax/core/optimizers.py:57-66 apply = update + apply_updates):
 *   SGD       p += neg_lr * g
 *   MOMENTUM  t = g + decay*t; u = nesterov ? g + decay*t : t; p += neg_lr * u
 *   ADAM      mu = (1-b1) g + b1 mu; nu = (1-b2) g*g + b2 nu;
 *             u = (mu/bc1) / (sqrt(nu/bc2 + eps_root) + eps); p += neg_lr * u
 *   ADAGRAD   v = g*g + v; u = (v > 0 ? rsqrt(v + eps) : 0) * g; p += neg_lr * u
 *   RMSPROP   v = (1-b2) g*g + b2 v; u = g * rsqrt(v + eps);
 *             [F_MOMENTUM: t = u + decay*m; u = nesterov ? u + decay*t : t]; p += neg_lr * u
 *   YOGI      mu = (1-b1) g + b1 mu; nu = nu - ((1-b2) sign(nu - g*g)) g*g;
 *             u = mu / (sqrt(nu + eps_root) + eps); p += neg_lr * u
 * (rsqrt = 1/sqrt evaluated in f64, rounded once; div / sqrt correctly rounded)
 * with every constant pre-rounded to f32 on the host as JAX's weak typing does
 * (bc1 = f32(1 - b1^t), bc2 = f32(1 - b2^t) for the step count t after the
 * increment). params, m (mu / trace) and v (nu) are float32[P], updated in place;
 * mean_dev (optional) also receives g. Only the params/state are written: the
 * mean never round-trips through HBM.
 */
enum fjagg_opt_kind {
  FJAGG_OPT_SGD = 1,      /* optimizers.py:227-250 (momentum None)                          */
  FJAGG_OPT_MOMENTUM = 2, /* optimizers.py:227-250, optax.trace (m)                          */
  FJAGG_OPT_ADAM = 3,     /* optimizers.py:148-178, optax.scale_by_adam (m, v)               */
  FJAGG_OPT_ADAGRAD = 4,  /* optimizers.py:117-145, optax.scale_by_rss (v = sum of squares)  */
  FJAGG_OPT_RMSPROP = 5,  /* optimizers.py:181-224, optax.scale_by_rms (v) [+ trace (m)]     */
  FJAGG_OPT_YOGI = 6      /* optimizers.py:253-281, optax.scale_by_yogi (m, v)               */
};
/* RMSPROP: b2 / one_minus_b2 = decay / 1 - decay. optax.rmsprop's chain is the rescale,
 * then scale_by_learning_rate, then (flags & FJAGG_OPT_F_MOMENTUM) optax.trace(decay = this
 * struct's `decay`, nesterov) of the lr-scaled update (m holds that trace), then
 * apply_updates. flags & FJAGG_OPT_F_CENTERED: the rescale is optax.scale_by_stddev
 * (m holds mu: u = g * rsqrt(nu - mu*mu + eps)); not combinable with the momentum flag
 * (a third state). */
#define FJAGG_OPT_F_MOMENTUM 1
#define FJAGG_OPT_F_CENTERED 2
typedef struct fjagg_server_opt {
  int kind;
  int nesterov;
  float neg_lr;
  float decay;
  float one_minus_b1, b1, one_minus_b2, b2;
  float bc1, bc2;
  float eps, eps_root;
  int flags;
} fjagg_server_opt;
int fjagg_server_update_dense(int in_dtype, const void* x_dev, int64_t ld, int64_t K, int64_t P,
                              const float* w_dev, float scale, const fjagg_server_opt* opt,
                              float* params_dev, float* m_dev, float* v_dev, float* mean_dev,
                              int flags, void* stream);
/* The same step on the pytree path: the plan image of fjagg_wsum_ptrs (same blocks,
 * nblk; weights f32) with out_ptrs[L] = the float32 params leaves (updated in place)
 * and state_dev[3*L] (device) = m leaves | v leaves | mean leaves (0 where absent; m
 * for MOMENTUM/ADAM, v for ADAM; mean optional). flags: FJAGG_NONTEMPORAL,
 * FJAGG_UNALIGNED. Replaces tree_mean + server_optimizer.apply over the pytrees of
 * examples/fed_avg.py:82,97-101 in one pass. */
int fjagg_server_update_ptrs(int in_dtype, const int64_t* image_dev, int L, int64_t K, int64_t nblk,
                             const float* w_dev, float scale, const fjagg_server_opt* opt,
                             const int64_t* state_dev, int flags, void* stream);

/*
 * Squared L2 norm of each of K client deltas (the per-client diagnostic of
 * examples/fed_avg.py:79-81 -> tree_util.py:105-108), accumulated in f32 per
 * workgroup and combined in a fixed order: deterministic, not bitwise equal to
 * XLA's reduction tree. out_dev is float[K]; ws_dev needs
 * fjagg_l2sq_workspace_bytes(K, P) bytes.
 */
int64_t fjagg_l2sq_workspace_bytes(int64_t K, int64_t P);
int fjagg_l2sq_dense(int in_dtype, const void* x_dev, int64_t ld, int64_t K, int64_t P,
                     float* out_dev, void* ws_dev, int64_t ws_bytes, void* stream);

/*
 * Pytree form of the squared norm: R rows at arbitrary device addresses, the
 * image is int64 [ptrs[R] | n[R]]; rows are grouped in consecutive runs of
 * rows_per_group (one client's leaves), out_dev[g] = sum of the group's squares
 * (sqrt of it when take_sqrt != 0: tree_l2_norm, tree_util.py:111-114). Each row
 * is summed in 64 Ki-element blocks and the partials are added in row/block order.
 */
int64_t fjagg_l2sq_rows_workspace_bytes(int64_t R, int64_t max_n);
int fjagg_l2sq_rows(int in_dtype, const int64_t* image_dev, int64_t R, int64_t max_n,
                    int64_t rows_per_group, int take_sqrt, float* out_dev, void* ws_dev,
                    int64_t ws_bytes, void* stream);

/*
 * Synthetic client deltas for tests and benchmarks (never on the product path):
 *   x[k][p] = amp * u(seed, k0 + k, p),  u = uniform in [-1, 1) with 2^-23 steps,
 * from a counter-based hash shared bit-for-bit with oracle/fold_ref.c.
 */
int fjagg_fill_synth(int dtype, void* x_dev, int64_t ld, int64_t K, int64_t P, int64_t k0,
                     uint64_t seed, float amp, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FJAGG_H_ */
