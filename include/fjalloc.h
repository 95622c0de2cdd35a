/*
 * fjalloc.h — opt-in segment allocator for client-delta memory (part of libfjagg.so).
 *
 * No reference counterpart: FedJAX's deltas are XLA buffers (fedjax/core/tree_util.py
 * folds whatever jax.Array objects the clients return). Here the caller's deltas are torch
 * allocations, and where they live changes the pytree fold's speed (separate
 * allocations cost compulsory address-translation misses). These entry points are a
 * torch.cuda CUDAPluggableAllocator pair whose segments for torch's caching allocator are
 * slices of a few large allocations, so the deltas a round allocates share their translations. fedjax_amd.memory.delta_pool
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
/* torch CUDAPluggableAllocator free: waits for `stream`, then gives the segment back. Mode 2:
 * its range (with its stagger bytes) is merged with free neighbours of its chunk and reused
 * best-fit for any later segment that fits; an emptied chunk is hipFree'd. Modes 0 / 1: the
 * mapping is released and the virtual range kept for a later segment of the same size. */
void fjalloc_free(void* ptr, size_t size, int device, void* stream);
/* out[13] = mapped bytes, live segments, segments created, ranges reused, failures,
 * granularity, bump offset, base address, last failure ((step << 16) | hipError_t; steps
 * 1 reserve, 2 create, 3 map, 4 access, 5 range full), segments reserved at the address
 * hint, segments reserved elsewhere, chunks (mode 2), free bytes inside the chunks (mode 2).
 * 0, or -1 for a bad device. */
int fjalloc_stats(int device, int64_t* out);
/* Before the first allocation on any device (-1 afterwards; serialised against fjalloc_alloc):
 * the mode — 2 (default) segments are slices of hipMalloc'd chunks of reserve_bytes (default
 * 1 GiB, or one segment's size if larger; a chunk is freed when its last slice is, and freed
 * ranges are coalesced and reused best-fit), a new slice starting (n mod 31) x stagger_bytes
 * (default 68 KiB) after the previous one's end; 1 one VMM reservation + hipMemCreate per
 * segment; 0 VMM sub-ranges of one reservation of reserve_bytes — and the segment size multiple
 * (default 64 KiB; rounded up to the runtime's granularity in modes 0 and 1). 0, or -1 for an
 * invalid value. */
int fjalloc_configure(int64_t reserve_bytes, int64_t align_bytes, int mode, int64_t stagger_bytes);

#ifdef __cplusplus
}
#endif

#endif /* FJALLOC_H_ */
