/* fjcomp.h — C ABI of the compression-aggregator kernels (libfjagg.so).
 *
 * FedJAX's compression aggregators (fedjax/aggregators/compression.py) quantize
 * every client delta with jax.random draws, optionally inside a randomized
 * Walsh-Hadamard rotation (fedjax/aggregators/walsh_hadamard.py), and feed the
 * results to tree_mean. In the reference each step is a jax.jit dispatch per
 * client per leaf; here the steps are a handful of launches per round over
 * device-resident (client, leaf) tables:
 *
 *   fjcomp_row_stats      jnp.amin / amax / std and the DRIVE sums per (client, leaf)
 *                         compression.py:58-61,84-87,331,275
 *   fjcomp_quant_fold     uniform_stochastic_quantize / terngrad_quantize with the
 *                         jax.random.uniform draw, fused with tree_mean's fold
 *                         compression.py:66-97,323-336 + tree_util.py:76-96
 *   fjcomp_rademacher     jax.random.rademacher signs, bit-packed
 *                         walsh_hadamard.py:148,170
 *   fjcomp_wht            walsh_hadamard_transform with the structured_rotation /
 *                         inverse_structured_rotation (and DRIVE) pre/epilogues
 *                         walsh_hadamard.py:25-176, compression.py:269-277
 *   fjcomp_random_bits / fjcomp_uniform   jax.random.bits / uniform of one key
 *
 * Randomness is jax.random's threefry2x32 (non-partitionable counter layout) and
 * haiku.PRNGSequence; the key schedule runs on the host (fjcomp_random_split,
 * fjcomp_prng_sequence), the draws on the device. All device pointers; all
 * launches are asynchronous on the given hipStream_t. Return 0 or FJAGG_E*;
 * fjagg_last_error() has the message. Table layouts are fixed (static_assert'd
 * in fjcomp.hip) so hosts can build them as plain structured arrays.
 */
#ifndef FJCOMP_H_
#define FJCOMP_H_

#include <stdint.h>

#include "fjagg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FJCOMP_ABI_VERSION 1

/* fjcomp_quant_fold methods */
#define FJCOMP_UNIFORM 1  /* uniform_stochastic_quantize, compression.py:66-97 */
#define FJCOMP_TERNGRAD 2 /* terngrad_quantize, compression.py:323-336 */
#define FJCOMP_BINARY 3   /* binary_stochastic_quantize, compression.py:43-63 */

/* fjcomp_wht job kinds */
#define FJCOMP_WHT_PLAIN 0          /* y = H x                                   walsh_hadamard.py:25-98 */
#define FJCOMP_WHT_ROTATE 1         /* y = H(pad(x) * D) / sqrt(d)               walsh_hadamard.py:127-148 */
#define FJCOMP_WHT_UNROTATE 2       /* y = (H x * D) / sqrt(d), first n_out      walsh_hadamard.py:151-176 */
#define FJCOMP_WHT_UNROTATE_DRIVE 3 /* x -> (A sign(x)) / B, then UNROTATE       compression.py:269-277 */

#define FJCOMP_WHT_MAX_LOG2 34 /* 2^34 floats; 13 + 8 + 8 + 8 bits: four passes */

/* per-row statistics (f64 accumulation, fixed combine order) */
typedef struct fjcomp_stats {
  double min, max;   /* NaN-propagating, like lax.min/max */
  double absmax;
  double sum, sumsq, sumabs;
} fjcomp_stats;

/* per-row quantizer parameters derived from fjcomp_stats by fjcomp_row_stats */
typedef struct fjcomp_qparams {
  float vmin, vmax; /* UNIFORM / BINARY: amin, amax. TERNGRAD: 0, amax(|clip(v)|) */
  float range;      /* vmax - vmin (f32) */
  float thr;        /* TERNGRAD: f32(2.5 * std) clip threshold; unused otherwise */
  double rcp_range; /* 1 / (double)range: correctly rounded f32 quotients, see fjcomp.hip */
} fjcomp_qparams;

typedef struct fjcomp_row {
  const float* ptr;
  int64_t n;
} fjcomp_row;

typedef struct fjcomp_sign_job {
  uint32_t key[2];
  int64_t d;        /* number of signs */
  uint32_t* words;  /* ceil(d / 32) words; bit (g % 32) of word g / 32 set <=> sign -1 */
} fjcomp_sign_job;

typedef struct fjcomp_wht_job {
  const float* src;           /* pass 0 input */
  float* mid;                 /* intermediate of a multi-pass job (d floats; may alias src) */
  float* dst;                 /* last-pass output, n_out floats */
  const uint32_t* signs;      /* ROTATE / UNROTATE*: d sign bits (fjcomp_rademacher) */
  const fjcomp_stats* stats;  /* UNROTATE_DRIVE: sumsq / sumabs of src. ROTATE: optional (may be NULL) per-tile
                                 partials of dst for fjcomp_stats_combine (min / max / |max|, and with
                                 FJCOMP_WHT_F_SUMS sumsq / sumabs in f64), one slot of
                                 fjcomp_row_stats_workspace_bytes(1) B per last-pass tile */
  int64_t n_in;               /* valid src elements (ROTATE zero-pads to d) */
  int64_t n_out;              /* elements written to dst (<= d) */
  int32_t log2d;
  int32_t kind;
  float sqrt_d;               /* f32(sqrt(d)), correctly rounded */
  int32_t flags;              /* ROTATE with stats: FJCOMP_WHT_F_SUMS also accumulates sumsq / sumabs */
} fjcomp_wht_job;
#define FJCOMP_WHT_F_SUMS 1

int fjcomp_abi_version(void);

/* ---- host key algebra (no device work) ---- */
/* Threefry-2x32-20 of n counter pairs. */
int fjcomp_threefry2x32(const uint32_t key[2], const uint32_t* x0, const uint32_t* x1, int64_t n,
                        uint32_t* y0, uint32_t* y1);
/* jax.random.split of each of nkeys keys into num: out[nkeys][num][2]. */
int fjcomp_random_split(const uint32_t* keys, int64_t nkeys, int64_t num, uint32_t* out);
/* n draws of haiku.PRNGSequence(key): key (in/out) advances, subkeys[n][2]. */
int fjcomp_prng_sequence(uint32_t key[2], int64_t n, uint32_t* subkeys);

/* ---- device ---- */
/* jax.random.bits(key, (n,), uint32) / jax.random.uniform(key, (n,), float32). */
int fjcomp_random_bits(uint32_t k0, uint32_t k1, int64_t n, uint32_t* out, void* stream);
int fjcomp_uniform(uint32_t k0, uint32_t k1, int64_t n, float* out, void* stream);

/* Bit-packed jax.random.rademacher(key, (d,)) for J jobs. A workgroup takes block_pairs
 * (a multiple of 256, at most FJCOMP_SIGN_BLOCK_PAIRS) consecutive element pairs of one job:
 * block_prefix[J+1] (device) is the running sum of ceil(ceil(d/2) / block_pairs) over jobs,
 * nblocks its last entry. Large blocks amortise the per-workgroup setup; small ones fill the
 * chip when there are few pairs in total. */
#define FJCOMP_SIGN_BLOCK_PAIRS 8192
int fjcomp_rademacher(const fjcomp_sign_job* jobs, const int64_t* block_prefix, int64_t J,
                      int64_t nblocks, int block_pairs, void* stream);

/* Statistics of R rows (f32). chunk_prefix[R+1] (device): running sum of
 * max(1, ceil(n / FJCOMP_STATS_CHUNK)); nchunks its last entry. Writes stats[R] and, when
 * method is FJCOMP_UNIFORM, FJCOMP_BINARY or FJCOMP_TERNGRAD, qparams[R] (may be NULL).
 * Workspace: fjcomp_row_stats_workspace_bytes(nchunks). */
#define FJCOMP_STATS_CHUNK 16384
int64_t fjcomp_row_stats_workspace_bytes(int64_t nchunks);
/* Statistics and (qparams != NULL) UNIFORM / BINARY qparams of R rows from per-tile
 * partials written by fjcomp_wht (ROTATE jobs with a stats pointer): row r owns partials
 * part_prefix[r] .. part_prefix[r+1]-1 (device). min / max / |max| equal fjcomp_row_stats';
 * sumsq / sumabs (FJCOMP_WHT_F_SUMS) are f64 sums in tile order, sum is 0. */
int fjcomp_stats_combine(const fjcomp_row* rows, const int64_t* part_prefix, int64_t R, int method,
                         const void* part, fjcomp_stats* stats, fjcomp_qparams* qparams, void* stream);
int fjcomp_row_stats(const fjcomp_row* rows, const int64_t* chunk_prefix, int64_t R, int64_t nchunks,
                     int method, fjcomp_stats* stats, fjcomp_qparams* qparams, void* ws,
                     int64_t ws_bytes, void* stream);

/* Quantize K clients x L leaves and fold them in client order (tree_mean):
 *   q = Q(x[k][l], key[k][l], qparams[k][l]);  s = (k == 0 && !ACCUMULATE) ? fl(q*w_k) : fl(s + fl(q*w_k))
 *   out[l] = SCALE ? fl(s * scale) : s
 * in_ptrs[K*L] (client-major), keys[K*L][2], qparams[K*L], w[K] f32, out_ptrs[L],
 * leaf_n[L], block_prefix[L+1] (running sum of ceil(ceil(n/2) / 256)). For
 * FJCOMP_UNIFORM, hist (optional, int32 [K*L][num_levels + 1], zeroed by the caller)
 * receives per-row counts of the quantization level index (bin num_levels: non-finite). */
int fjcomp_quant_fold(int method, const float* const* in_ptrs, const uint32_t* keys,
                      const fjcomp_qparams* qparams, const float* w, int64_t K, int64_t L,
                      const int64_t* leaf_n, const int64_t* block_prefix, int64_t nblocks,
                      int num_levels, float scale, int flags, float* const* out_ptrs, int32_t* hist,
                      void* stream);

/* Walsh-Hadamard jobs. pass_prefix[npass][J+1] (device): per pass, the running sum of
 * that job's tiles in the pass (0 if the job has fewer passes); pass_tiles[npass] (host):
 * the totals. A job of d = 2^log2d has one pass for log2d <= 13, else
 * 1 + ceil((log2d - 13) / 8) (pass 0: bits 0..12; pass p >= 1: the next 8 bits). */
int fjcomp_wht(const fjcomp_wht_job* jobs, const int64_t* pass_prefix, int64_t J, int npass,
               const int64_t* pass_tiles, void* stream);

/* tiles of pass p for a job of 2^log2d (host helper, mirrors the kernel's tiling) */
int64_t fjcomp_wht_tiles(int log2d, int pass);

#ifdef __cplusplus
}
#endif

#endif /* FJCOMP_H_ */
