/*
 * fjcomm.h — C ABI of the client-sharded aggregation over the GPUs of one node
 * (part of libfjagg.so; conventions as in fjagg.h).
 *
 * The reference has no device-side reduction: ForEachClientPmapBackend spreads
 * client training over jax.local_devices() and copies every client output back
 * to devices[0] (fedjax/core/for_each_client.py:266-357, gather at :351-353),
 * where tree_mean (fedjax/core/tree_util.py:76-96) folds all K clients. Here
 * every GPU (one process per GPU) folds its own K/N clients and the N float32
 * partials are summed by RCCL over xGMI. The step is issued by ONE call:
 *
 *     stream (compute)     fold b0 | fold b1 | ... | fold bL | wait(done) | reduce bL
 *                               \ev0      \ev1
 *     comm stream (RCCL)         reduce b0  reduce b1 ... done
 *
 * so the reduce of parameter bucket b overlaps the fold of bucket b+1, and the
 * last bucket is reduced on the caller's stream (no cross-queue hop back at the
 * end of the step; with one bucket the step is fold + reduce on one stream). The
 * cross-stream events are created with a device-scope release (no system-scope
 * cache write-back: the RCCL kernels run on the same device and read the
 * partial through its L2).
 *
 * RCCL is the library torch already loaded (resolved with dlopen(RTLD_NOLOAD)
 * of librccl.so.1, then a regular dlopen), so one RCCL runtime serves both
 * torch.distributed and this communicator.
 */
#ifndef FJCOMM_H_
#define FJCOMM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FJCOMM_ABI_VERSION 1
#define FJCOMM_ID_BYTES 128 /* sizeof(ncclUniqueId) */
#define FJCOMM_MAX_BUCKETS 64

int fjcomm_abi_version(void);

/* ncclGetUniqueId: rank 0 creates the id, every rank passes it to fjcomm_init. */
int fjcomm_unique_id(uint8_t* id /* FJCOMM_ID_BYTES */);

/* ncclCommInitRank on the current HIP device (collective: every rank calls it), plus
 * the communicator's stream (high priority) and its events. Allocates; call once. */
int fjcomm_init(void** comm, const uint8_t* id, int nranks, int rank);
int fjcomm_destroy(void* comm);

/* ncclCommAbort: ends the communicator's outstanding collectives without waiting for the other
 * ranks (a rank that missed a deadline on a collective that never completes calls it; every
 * rank must then stop using this communicator). Every later step on it returns FJAGG_EINVAL;
 * fjcomm_destroy still frees it (waiting at most 10 s for its stream). Non-blocking on the
 * collective; no other rank's participation is needed. FJAGG_EUNSUPPORTED when the loaded RCCL
 * has no ncclCommAbort. Replaces nothing in the reference (jax's pmap has no such control,
 * fedjax/core/for_each_client.py:266-357): it bounds the bench's exchange auto-tune. */
int fjcomm_abort(void* comm);

/* Test support: one wave that spins on the real-time counter for `us` microseconds (<= 60 s)
 * on `stream` (reads no memory), so tests can enqueue a collective behind running work. */
int fjcomm_test_block(int64_t us, void* stream);

/*
 * One round of the sharded weighted mean on this rank:
 *   out_dev[p] = fl(sum_{k<K} fl(x_k[p] * w_k)) * scale        (this rank's partial,
 *                 bitwise fjagg_wsum_dense with FJAGG_SCALE on the bucket)
 * then out_dev += the other ranks' partials (ncclReduce to `root`, or ncclAllReduce
 * when root < 0), bucket by bucket as described above. x_dev is this rank's client-
 * major slab [K x ld] of in_dtype (F32 or BF16); w_dev float[K]; the partial and the
 * result are float32 [P]. `stream` waits for the last collective, so work queued on
 * it afterwards sees the reduced result (valid on root, or everywhere with root < 0).
 * fold_events: NULL, or 2*nbuckets events made by fjagg_event_create; the fold of
 * bucket b is bracketed by fold_events[2b], fold_events[2b+1] on `stream`.
 * K may be 0 (the rank contributes zeros). flags: FJAGG_NONTEMPORAL, the
 * FJAGG_VARIANT bits of fjagg_wsum_dense, and FJAGG_HOST_TABLES (w_dev is then a HOST
 * float[K] carried in each bucket fold's kernel arguments; every bucket is checked
 * before the first launch and FJAGG_EUNSUPPORTED means nothing was issued).
 * Replaces: the gather-to-devices[0] + tree_mean of for_each_client.py:351-353 and
 * tree_util.py:85-96 for one round.
 */
int fjcomm_sharded_wsum_dense(void* comm, int in_dtype, const void* x_dev, int64_t ld, int64_t K,
                              int64_t P, const void* w_dev, float scale, float* out_dev,
                              int nbuckets, int root, int flags, void* stream, void* const* fold_events);

/*
 * The same step over explicit bucket edges: bucket b is elements [edges[b], edges[b+1]),
 * edges[0] = 0, edges[nbuckets] = P, strictly increasing, every edge but the last a
 * multiple of FJCOMM_BUCKET_ALIGN elements (keeps the rows' 16-byte alignment). Unequal
 * buckets let a tapered schedule (e.g. 4:2:1) hide each reduce behind the next, smaller
 * fold, so only the small last bucket's reduce is exposed at the end of the step.
 * fjcomm_sharded_wsum_dense is this call with equal buckets.
 */
#define FJCOMM_BUCKET_ALIGN 1024
int fjcomm_sharded_wsum_dense_edges(void* comm, int in_dtype, const void* x_dev, int64_t ld, int64_t K,
                                    int64_t P, const void* w_dev, float scale, float* out_dev,
                                    const int64_t* edges, int nbuckets, int root, int flags, void* stream,
                                    void* const* fold_events);

/*
 * Single process, several GPUs. FedJAX's server is ONE Python process over
 * jax.local_devices() (fedjax/core/for_each_client.py:266-357, devices at :289-293);
 * these entry points give such a process the sharded aggregation without a launcher:
 *
 * fjcomm_init_all: ncclCommInitAll over devs[0..ndev) (distinct HIP device ordinals);
 * comms[d] is the handle of devs[d] (rank d), with its own stream and events on that
 * device. Destroy each handle with fjcomm_destroy. The calling thread's current device
 * is restored on return.
 *
 * fjcomm_multi_wsum_dense: one round over all devices, issued from one thread. Device d
 * folds its client slab (x_dev[d]: K[d] rows of ld[d] elements, w_dev[d] float[K[d]],
 * both on devs[d]) into out_dev[d] (float32 [P] on devs[d]) scaled by `scale`, on
 * streams[d]; the partials are then summed by ncclReduce to device `root` (ncclAllReduce
 * when root < 0), bucket by bucket over `edges` as in fjcomm_sharded_wsum_dense_edges.
 * The collectives of one bucket are one ncclGroupStart/End group (required when one
 * thread drives several ranks). streams[d] waits for the last collective of device d.
 * K[d] may be 0 (device d contributes zeros). flags as fjcomm_sharded_wsum_dense
 * (with FJAGG_HOST_TABLES, w_dev[d] are host arrays).
 */
#define FJCOMM_MAX_DEVICES 16
int fjcomm_init_all(void** comms, int ndev, const int* devs);
int fjcomm_multi_wsum_dense(void* const* comms, int ndev, int in_dtype, const void* const* x_dev,
                            const int64_t* ld, const int64_t* K, int64_t P, const void* const* w_dev, float scale,
                            float* const* out_dev, const int64_t* edges, int nbuckets, int root, int flags,
                            void* const* streams);

/* Timing events without the system-scope fence (hipEventDisableSystemFence): recording
 * one costs no cache write-back, so bracketing every launch does not perturb it. */
int fjagg_event_create(void** ev);
int fjagg_event_destroy(void* ev);
int fjagg_event_record(void* ev, void* stream);
int fjagg_event_elapsed_ms(float* ms, void* start, void* end); /* synchronises on `end` */

#ifdef __cplusplus
}
#endif

#endif /* FJCOMM_H_ */
