/*
 * fjopt.h — the adafactor server step (part of libfjagg.so; conventions as in fjagg.h).
 *
 * Replaces fedjax.optimizers.adafactor (fedjax/core/optimizers.py:284-348), i.e.
 * optax.adafactor applied by create_optimizer_from_optax (optimizers.py:57-66) to the
 * round's mean delta, for float32 leaves:
 *
 *   scale_by_factored_rms   per leaf, step count c (before the increment):
 *       d = 1 - (c - decay_offset + 1) ** -decay_rate            (decay_rate_t, host)
 *       factored (rank >= 2 and the second-largest dimension >= min_dim_size_to_factor;
 *       d0 = the largest axis, d1 = the second largest, numpy argsort order):
 *           v_row = d * v_row + (1 - d) * mean(g*g + eps, axis=d0)
 *           v_col = d * v_col + (1 - d) * mean(g*g + eps, axis=d1)
 *           u = g * (v_row / mean(v_row, axis=d1')) ** -0.5 * v_col ** -0.5
 *       otherwise:  v = d * v + (1 - d) * (g*g + eps);  u = g * v ** -0.5
 *   clip_by_block_rms       u = u / max(1, sqrt(mean(u*u)) / clipping_threshold)
 *   scale_by_learning_rate  u = u * lr
 *   scale_by_param_block_rms  u = u * max(sqrt(mean(p*p)), 1e-3)
 *   ema (momentum)          m = (1 - momentum) * u + momentum * m;  u = m
 *   add_decayed_weights     u = u + weight_decay_rate * p   (masked leaves)
 *   scale(-1), apply_updates  p = p + (-u)
 *
 * Every elementwise op is one IEEE float32 op in that order (no FMA, -ffp-contract=off;
 * divisions and ** -0.5 correctly rounded). The means (jnp.mean) are sums of the float32
 * terms accumulated in float64 in a fixed order, divided by the count and rounded once:
 * deterministic and at least as accurate as XLA's float32 reductions, not XLA's order
 * (optax is not in this image: parity unpinned).
 *
 * A leaf's factored view is its shape as [A, n_lo, B, n_hi, C] with the two factored axes
 * as lo (the earlier) and hi; d0_is_lo says which of them is the largest. v_row has the
 * shape without d0, v_col the shape without d1 (optax's state shapes).
 *
 * Use: fjopt_adafactor_plan (host only) writes a table for the leaves and the flags of
 * the hyperparameters; the caller uploads it and calls fjopt_adafactor_step with the host
 * and device copies and a device workspace of the planned size. The step is 5-7 launches
 * on the caller's stream; no allocation or synchronisation inside.
 */
#ifndef FJOPT_H_
#define FJOPT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FJOPT_ABI_VERSION 1

typedef struct fjopt_af_leaf {
  const float* g;  /* the mean delta (pseudo-gradient), n floats */
  float* p;        /* params, updated in place */
  float* v_row;    /* factored: second-moment row statistics (state, in place) */
  float* v_col;    /* factored: column statistics */
  float* v;        /* unfactored: per-element second moments, n floats */
  float* m;        /* ema state when momentum is on, else NULL */
  int64_t n;       /* elements */
  int64_t dims[5]; /* factored: A, n_lo, B, n_hi, C (product n); else 1, n, 1, 1, 1 */
  int32_t factored;
  int32_t d0_is_lo;
  int32_t decay_weights; /* add_decayed_weights applies to this leaf */
  int32_t reserved;
} fjopt_af_leaf;

typedef struct fjopt_af_hparams {
  float decay_rate_t;      /* f32: 1 - (c - decay_offset + 1) ** -decay_rate */
  float one_minus_decay;   /* f32: 1 - decay_rate_t */
  float eps;
  int32_t clip;            /* clipping_threshold is not None */
  float clip_threshold;
  int32_t has_lr;          /* learning_rate is not None */
  float lr;                /* the schedule's value at this step, or the constant */
  int32_t param_scale;     /* multiply_by_parameter_scale */
  float min_scale;         /* 1e-3 (optax.scale_by_param_block_rms) */
  int32_t momentum;        /* momentum is not None */
  float mom_decay;         /* momentum */
  float one_minus_mom;     /* f32: 1 - momentum */
  int32_t weight_decay;    /* weight_decay_rate is not None */
  float wd;
} fjopt_af_hparams;

int fjopt_abi_version(void);

/* Plan for L leaves: writes at most table_words int64 words into table (NULL: size query)
 * and the workspace bytes into *ws_bytes. Returns the table's words, or < 0 on error
 * (fjagg_last_error). Host only. */
int64_t fjopt_adafactor_plan(const fjopt_af_leaf* leaves, int L, const fjopt_af_hparams* hp, int64_t* table,
                             int64_t table_words, int64_t* ws_bytes);

/* One adafactor step for the planned leaves: table_host / table_dev are the host and
 * device copies of the plan, ws a device workspace of the planned bytes. hp must have the
 * flags it was planned with (the values may change from step to step). */
int fjopt_adafactor_step(const int64_t* table_host, const int64_t* table_dev, const fjopt_af_hparams* hp, void* ws,
                         int64_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FJOPT_H_ */
