/*
 * fjalloc.h — opt-in segment allocator for client-delta memory (part of libfjagg.so).
 *
 * No reference counterpart: FedJAX's deltas are XLA buffers (fedjax/core/tree_util.py
 * folds whatever jax.Array objects the clients return). Here the caller's deltas are torch
 * allocations, and where they live changes the pytree fold's speed (separate
 * allocations cost compulsory address-translation misses). These entry points are a
 * torch.cuda CUDAPluggableAllocator pair: segments for torch's caching allocator carved from
 * one reserved virtual range per device (hipMemAddressReserve), each backed by its own
 * hipMemCreate allocation mapped at a granularity-aligned address. fedjax_amd.memory.delta_pool
 * wraps them in a torch.cuda.MemPool, used per scope (torch.cuda.use_mem_pool).
 */
#ifndef FJALLOC_H_
#define FJALLOC_H_

#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* torch CUDAPluggableAllocator malloc: a segment of >= size bytes on device, or NULL. */
void* fjalloc_alloc(ssize_t size, int device, void* stream);
/* torch CUDAPluggableAllocator free: waits for `stream`, unmaps and releases the segment
 * (its virtual range is kept for a later segment of the same size). */
void fjalloc_free(void* ptr, size_t size, int device, void* stream);
/* out[8] = mapped bytes, live segments, segments created, ranges reused, failures,
 * granularity, bump offset, reserved base address. 0, or -1 for a bad device / NULL out. */
int fjalloc_stats(int device, int64_t* out);
/* Virtual bytes to reserve per device at its first allocation (default 512 GiB). */
int fjalloc_set_reserve_bytes(int64_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* FJALLOC_H_ */
