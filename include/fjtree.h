/*
 * fjtree.h — per-call tree ops of fedjax.tree_util with the leaf table in the kernel
 * arguments (part of libfjagg.so; conventions as in fjagg.h).
 *
 * FedJAX's library algorithms aggregate with a running sum, one client at a time
 * (fedjax/algorithms/fed_avg.py:132-146; the same loop in fed_prox.py:127-140,
 * mime.py:186-197, mime_lite.py:129-148, agnostic_fed_avg.py:278-289,
 * apfl.py:207-220, hyp_cluster.py:284-304):
 *
 *     s = tree_zeros_like(params)
 *     for each client: s = tree_add(s, tree_weight(delta, n));  tree_l2_norm(delta)
 *     mean = tree_inverse_weight(s, sum n)
 *
 * Each call touches one or two pytrees of L leaves. The pytree path of fjagg.h
 * (fjagg_wsum_ptrs) reads its (client, leaf) table from device memory, which costs a
 * host-to-device upload per call. Here the whole table — at most FJTREE_MAX_LEAVES
 * leaves of up to FJTREE_MAX_OPERANDS operands — travels in the kernel arguments: one
 * launch per call, nothing uploaded. The caller fills an fjtree_leaves in host memory;
 * the library copies it into the launch.
 *
 * Arithmetic (float32, IEEE round to nearest, no FMA; compiled -ffp-contract=off), per
 * leaf l and element p, with t_k = fl(x[k][l][p] * w[k]):
 *     s = t_0;  s = fl(s + t_1) (K = 2);  out[l][p] = FJAGG_SCALE ? fl(s * scale) : s
 * which is bitwise, for float32 leaves:
 *     K = 1, w = {w}            tree_weight(x, w)                 tree_util.py:29-32
 *     K = 1, w = {f32(1/W)}     tree_inverse_weight(x, W)         tree_util.py:35-38
 *     K = 2, w = {1, 1}         tree_add(a, b)                    tree_util.py:47-50
 *     K = 2, w = {1, n}         tree_add(s, tree_weight(x, n))    fed_avg.py:137-138
 * (x * 1 is exact in IEEE arithmetic, so the K = 2 fold is the reference's jnp.add of
 * the weighted tree.)
 *
 * With FJTREE_NORM the same pass also sums the squares of operand norm_operand over all
 * leaves — tree_l2_squared / tree_l2_norm of that (unweighted) operand,
 * tree_util.py:105-114 — into norm_out[0] (sum of squares) and norm_out[1] (its
 * correctly rounded sqrt). The order is fixed: each lane adds the squares of the
 * elements it owns in order, a wave combines lanes by an xor butterfly, a workgroup its
 * 4 waves in order, and the last workgroup to finish adds the workgroup partials in
 * workgroup order. The lane/element assignment does not depend on pointer alignment, so
 * the result depends only on the leaf sizes and values: a fused norm and a standalone
 * one (FJTREE_NO_OUT, K = 1) of the same tree have the same bits. Not XLA's reduction
 * tree (unpinned).
 *
 * Cross-workgroup ordering of that last step. Default: each partial is an
 * agent-scope (write-through, sc1) store, the storing wave drains it (s_waitcnt vmcnt(0))
 * before its relaxed agent-scope counter add, and the last workgroup reads the partials
 * with agent-scope (sc1) loads: the gfx950 hand-off form of the MI355X guide (Guideline 16,
 * R1), ordered by the hardware, not by the HIP memory model. FJTREE_ORDERED instead makes
 * the counter add an acquire-release RMW at agent scope, ordered by the memory model (a
 * release fence: on gfx950 a whole-L2 write-back per workgroup). Both give the same bits.
 */
#ifndef FJTREE_H_
#define FJTREE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FJTREE_ABI_VERSION 1
#define FJTREE_MAX_LEAVES 64
#define FJTREE_MAX_OPERANDS 2

/* flags, besides FJAGG_SCALE (fjagg.h) */
#define FJTREE_NORM (1 << 8)   /* also write norm_out = {sum x^2, sqrt} of operand norm_operand */
#define FJTREE_NO_OUT (1 << 9) /* norm only: out[] is not written (may be NULL) */
#define FJTREE_ORDERED (1 << 10) /* FJTREE_NORM combine ordered by release/acquire atomics */

typedef struct fjtree_leaves {
  int K;                                                   /* operands, 1 or 2 */
  int L;                                                   /* leaves, 1 .. FJTREE_MAX_LEAVES */
  const float* x[FJTREE_MAX_OPERANDS][FJTREE_MAX_LEAVES];  /* device, n[l] floats each */
  float* out[FJTREE_MAX_LEAVES];                           /* device; may alias x[k][l] */
  int64_t n[FJTREE_MAX_LEAVES];                            /* elements per leaf, >= 0 */
  float w[FJTREE_MAX_OPERANDS];
  float scale;
  int flags;         /* FJAGG_SCALE | FJTREE_NORM | FJTREE_NO_OUT | FJTREE_ORDERED */
  int norm_operand;  /* 0 .. K-1 */
  float* norm_out;   /* device float[2] (FJTREE_NORM) */
  void* ws;          /* device, fjtree_workspace_bytes(table) bytes (FJTREE_NORM); its first
                        4 bytes are a completion counter that must be 0 before the first use
                        (the kernel leaves it 0: reuse the workspace on the same stream). Under
                        graph capture zero it before the capture or with a kernel: a recorded
                        hipMemsetAsync acts on the first replay only (ROCm 7, measured) */
  int64_t ws_bytes;
} fjtree_leaves;

int fjtree_abi_version(void);
/* Bytes of workspace FJTREE_NORM needs for this table (0 without FJTREE_NORM). */
int64_t fjtree_workspace_bytes(const fjtree_leaves* t);
/* One launch on `stream`; t is read during the call only. */
int fjtree_fold_leaves(const fjtree_leaves* t, void* stream);
/* The deferred running sum's lazy norms (fedjax_amd.tree_util): for i < n,
 * sq_out[i] = l2sq[i] and norm_out[i] = sqrt(l2sq[i]) (correctly rounded), one launch on
 * `stream`. Replaces, for the per-client tree_l2_squared / tree_l2_norm of the deltas a fold
 * covered (fedjax/core/tree_util.py:105-114, called at fedjax/algorithms/fed_avg.py:142-144),
 * the copy and the sqrt the fold's squared norms would otherwise take as two launches.
 * Device pointers, float32; n <= 2^30. */
int fjtree_norms_fill(const float* l2sq, float* sq_out, float* norm_out, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FJTREE_H_ */
