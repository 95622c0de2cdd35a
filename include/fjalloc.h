/*
 * fjalloc.h — opt-in segment allocator for client-delta memory (part of libfjagg.so).
 *
 * No reference counterpart: FedJAX's deltas are XLA buffers (fedjax/core/tree_util.py
 * folds whatever jax.Array objects the clients return). Here the caller's deltas are torch
 * allocations, and where they live changes the pytree fold's speed (separate
 * allocations cost compulsory address-translation misses). These entry points are a
 * torch.cuda CUDAPluggableAllocator pair: segments for torch's caching allocator placed one
 * after another in the device's virtual address space (hipMemAddressReserve at the next
 * address), each backed by its own hipMemCreate allocation. fedjax_amd.memory.delta_pool
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
/* out[11] = mapped bytes, live segments, segments created, ranges reused, failures,
 * granularity, bump offset, base address, last failure ((step << 16) | hipError_t; steps
 * 1 reserve, 2 create, 3 map, 4 access, 5 range full), segments reserved at the address
 * hint, segments reserved elsewhere. 0, or -1 for a bad device. */
int fjalloc_stats(int device, int64_t* out);
/* Before a device's first allocation: the virtual bytes to reserve for it (mode 0, default
 * 512 GiB), the segment size / address multiple (default 2 MiB, rounded up to the runtime's
 * granularity) and the mode: 1 (default) one reservation per segment at the address after the
 * previous one, 0 sub-ranges of one reservation. 0, or -1 for an invalid value. */
int fjalloc_configure(int64_t reserve_bytes, int64_t align_bytes, int mode);

#ifdef __cplusplus
}
#endif

#endif /* FJALLOC_H_ */
