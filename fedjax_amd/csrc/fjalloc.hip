// fjalloc.hip — an opt-in segment allocator for client-delta memory (host code only; part of
// libfjagg.so, C ABI in include/fjalloc.h).
//
// Callers of tree_mean hold every (client, leaf) delta as its own torch allocation. The pytree
// fold (k_ptrs) walks all K client rows from every CU, and rows that live in separately
// hipMalloc'd segments cost compulsory address-translation misses (23 K UTCL1
// misses per configs[1] launch against 5 when the same bytes are views of one allocation,
// 94.6 vs 87.6 us). This allocator gives torch's caching allocator its segments as slices of a
// few large hipMalloc'd chunks (1 GiB by default), each slice staggered from the previous one,
// so the deltas a round allocates share a few large mappings (mode 2, the default; modes 1 and
// 0 are the VMM designs that were measured and kept for comparison, see g_mode). It is plugged
// in per scope through torch.cuda.MemPool(CUDAPluggableAllocator(libfjagg.so, "fjalloc_alloc",
// "fjalloc_free")) (fedjax_amd.memory.delta_pool); the caching allocator still splits and
// caches blocks inside the segments. A freed slice's range is coalesced with free neighbours
// and reused best-fit for any later segment that fits (or returned to the chunk's bump tail); a
// chunk goes back to the runtime when its last slice is freed (torch frees a pool's segments
// when the pool is released). Nothing else in the library uses it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <unordered_map>
#include <vector>

#include "fjalloc.h"

namespace {

struct Segment {
  size_t size;
  hipMemGenericAllocationHandle_t handle;
  bool own_reservation;
  bool chunk_slice;  // mode 2: a slice of a chunk (freed by chunk_free whatever g_mode is then)
  size_t pad = 0;    // mode 2: stagger bytes in front of the slice, owned by it (freed with it)
};

struct Chunk {  // mode 2
  char* base;
  size_t size, top;
  int64_t live;  // slices in use
};

struct Arena {
  std::mutex mu;
  char* base = nullptr;  // reserved virtual range
  size_t reserved = 0;
  size_t top = 0;   // bump offset
  size_t gran = 0;  // mapping granularity
  std::multimap<size_t, char*> free_ranges;  // modes 0, 1: unmapped ranges by size, reused for equal sizes
  std::unordered_map<uintptr_t, Segment> live;
  std::vector<Chunk> chunks;  // mode 2; an empty chunk is returned to the runtime
  // mode 2: free ranges inside the chunks by address (start -> bytes), coalesced with their
  // free neighbours in the same chunk; a range that reaches its chunk's bump offset is
  // given back to the bump tail instead
  std::map<char*, size_t> chunk_free_ranges;
  int64_t mapped_bytes = 0, segments = 0, reuses = 0, failures = 0;
  int64_t last_error = 0;  // (step << 16) | hipError_t of the last failed request
  int64_t hinted = 0, hint_missed = 0;  // mode 1: reservations placed at / away from the hint
};

// record a failed request: which step (1 reserve, 2 create, 3 map, 4 access, 5 range) and the
// runtime's error code, readable through fjalloc_stats
inline void* failed(Arena& a, int step, hipError_t e) {
  ++a.failures;
  a.last_error = (int64_t(step) << 16) | int64_t(e);
  return nullptr;
}

constexpr int kMaxDevices = 64;
Arena g_arena[kMaxDevices];
size_t g_reserve_bytes = size_t(512) << 30;  // virtual only: 512 GiB per device
size_t g_align = size_t(64) << 10;  // segment size multiple (modes 0 and 1: >= the runtime's granularity)
// 2 (default): segments are slices of large hipMalloc'd chunks (g_chunk_bytes each), so many
// segments share one allocation and its large translation fragments; 1: every segment is its
// own VMM reservation + hipMemCreate, requested at the address after the previous one; 0: VMM
// sub-ranges of ONE reservation. Measured (profiles/r04k_pool/): 1 places segments apart (the
// runtime ignores the hint) and keeps every (client, leaf)'s translation misses (23,320 per
// configs[1] fold, as torch's own segments); 0 fails in this torch's ROCm 7.0 runtime
// (hipMemSetAccess -> hipErrorInvalidValue on later sub-ranges, tools/probe_fjalloc.py).
int g_mode = 2;
size_t g_chunk_bytes = size_t(1) << 30;
// mode 2: segment n starts (n mod 31) x g_stagger bytes past the previous segment's end, so the
// clients' rows (the caching allocator places a leaf at the same offset of every segment) do
// not all share their address residue modulo 2 MiB: rows with equal residues contend for the
// same L2 tags (one allocation with 2 MiB-aligned rows, 91.7 vs 87.6 us).
size_t g_stagger = size_t(68) << 10;
// The layout globals above are written by fjalloc_configure under an exclusive lock and read
// by fjalloc_alloc under a shared one, so no allocation sees a half-applied configuration.
std::shared_mutex g_config_mu;

hipMemAllocationProp prop_for(int device) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

hipError_t ensure_reserved(Arena& a, int device) {
  if (a.base) return hipSuccess;
  hipMemAllocationProp p = prop_for(device);
  size_t g = 0;
  hipError_t e = hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityRecommended);
  if (e != hipSuccess) return e;
  if (g == 0) return hipErrorInvalidValue;
  a.gran = (g_align + g - 1) / g * g;  // a multiple of the runtime's granularity
  void* va = nullptr;
  const size_t want = (g_reserve_bytes + a.gran - 1) / a.gran * a.gran;
  e = hipMemAddressReserve(&va, want, a.gran, nullptr, 0);
  if (e != hipSuccess) return e;
  if (!va) return hipErrorOutOfMemory;
  a.base = static_cast<char*>(va);
  a.reserved = want;
  return hipSuccess;
}

// mode 2: the chunk holding address p, or nullptr
Chunk* chunk_of(Arena& a, const char* p) {
  for (Chunk& c : a.chunks)
    if (p >= c.base && p < c.base + c.size) return &c;
  return nullptr;
}

// mode 2: the range [p, p + size) of chunk c is free again: merged with free neighbours of the
// same chunk, and returned to the bump tail when it reaches the chunk's bump offset.
void chunk_release_range(Arena& a, Chunk& c, char* p, size_t size) {
  auto next = a.chunk_free_ranges.lower_bound(p);
  if (next != a.chunk_free_ranges.end() && next->first == p + size && next->first < c.base + c.size) {
    size += next->second;
    next = a.chunk_free_ranges.erase(next);
  }
  if (next != a.chunk_free_ranges.begin()) {
    auto prev = std::prev(next);
    if (prev->first >= c.base && prev->first + prev->second == p) {
      p = prev->first;
      size += prev->second;
      a.chunk_free_ranges.erase(prev);
    }
  }
  if (p + size == c.base + c.top) {
    c.top = static_cast<size_t>(p - c.base);
  } else {
    a.chunk_free_ranges.emplace(p, size);
  }
}

// mode 2: slice p of `size` bytes (and its `pad` stagger bytes in front) is free again: its
// range goes back to the chunk (chunk_release_range); when it was the chunk's last live slice,
// the chunk (and the free ranges in it) goes back to the runtime.
void chunk_free(Arena& a, int device, char* p, size_t size, size_t pad) {
  Chunk* c = chunk_of(a, p);
  if (!c) return;
  if (--c->live > 0) {
    chunk_release_range(a, *c, p - pad, size + pad);
    return;
  }
  for (auto it = a.chunk_free_ranges.begin(); it != a.chunk_free_ranges.end();)
    it = (it->first >= c->base && it->first < c->base + c->size) ? a.chunk_free_ranges.erase(it) : std::next(it);
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  (void)hipFree(c->base);
  if (prev >= 0) (void)hipSetDevice(prev);
  a.chunks.erase(a.chunks.begin() + (c - a.chunks.data()));
  a.base = a.chunks.empty() ? nullptr : a.chunks[0].base;
}

// mode 2: a slice of >= size bytes: the best-fitting free range of any chunk (split, the rest
// stays free), else the bump tail of a chunk with room (staggered), else a new chunk — so a
// request that fits in freed space never needs a new hipMalloc (torch's out-of-memory retry
// frees its cached segments and asks again).
void* chunk_alloc(Arena& a, int device, size_t size) {
  a.gran = g_align;
  const size_t sz = (size + a.gran - 1) / a.gran * a.gran;
  size_t pad = (static_cast<size_t>(a.segments) % 31) * g_stagger;
  char* va = nullptr;
  auto best = a.chunk_free_ranges.end();
  for (auto it = a.chunk_free_ranges.begin(); it != a.chunk_free_ranges.end(); ++it)
    if (it->second >= sz && (best == a.chunk_free_ranges.end() || it->second < best->second)) best = it;
  if (best != a.chunk_free_ranges.end()) {
    va = best->first;
    const size_t rest = best->second - sz;
    a.chunk_free_ranges.erase(best);
    if (rest > 0) a.chunk_free_ranges.emplace(va + sz, rest);
    pad = 0;
    ++a.reuses;
    if (Chunk* c = chunk_of(a, va)) ++c->live;
  } else {
    for (Chunk& c : a.chunks)
      if (c.size - c.top >= sz + pad) {
        va = c.base + c.top + pad;
        c.top += pad + sz;
        ++c.live;
        break;
      }
    if (!va) {
      const size_t csz = std::max(g_chunk_bytes, sz);
      int prev = -1;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(device);
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, csz);
      if (prev >= 0) (void)hipSetDevice(prev);
      if (e != hipSuccess || !p) return failed(a, 2, e != hipSuccess ? e : hipErrorOutOfMemory);
      a.chunks.push_back(Chunk{static_cast<char*>(p), csz, sz, 1});
      if (a.chunks.size() == 1) a.base = static_cast<char*>(p);
      va = static_cast<char*>(p);
      pad = 0;
    }
  }
  a.live[reinterpret_cast<uintptr_t>(va)] = Segment{sz, hipMemGenericAllocationHandle_t{}, false, true, pad};
  a.mapped_bytes += static_cast<int64_t>(sz);
  ++a.segments;
  return va;
}

}  // namespace

extern "C" {

void* fjalloc_alloc(ssize_t size, int device, void* /*stream*/) {
  if (size <= 0 || device < 0 || device >= kMaxDevices) return nullptr;
  Arena& a = g_arena[device];
  std::shared_lock<std::shared_mutex> config(g_config_mu);
  std::lock_guard<std::mutex> lock(a.mu);
  if (g_mode == 2) return chunk_alloc(a, device, static_cast<size_t>(size));
  if (g_mode == 0) {
    if (hipError_t e = ensure_reserved(a, device)) return failed(a, 1, e);
  } else if (a.gran == 0) {
    hipMemAllocationProp p = prop_for(device);
    size_t g = 0;
    if (hipError_t e = hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityRecommended))
      return failed(a, 1, e);
    a.gran = (g_align + (g ? g : 1) - 1) / (g ? g : 1) * (g ? g : 1);
  }
  const size_t sz = (static_cast<size_t>(size) + a.gran - 1) / a.gran * a.gran;
  char* va = nullptr;
  bool own = false;
  auto it = a.free_ranges.find(sz);
  if (it != a.free_ranges.end()) {
    va = it->second;
    a.free_ranges.erase(it);
    ++a.reuses;
  } else if (g_mode == 0) {
    if (a.top + sz > a.reserved) return failed(a, 5, hipErrorOutOfMemory);
    va = a.base + a.top;
    a.top += sz;
  } else {
    void* hint = a.base ? a.base + a.top : nullptr;
    void* got = nullptr;
    if (hipError_t e = hipMemAddressReserve(&got, sz, a.gran, hint, 0)) return failed(a, 1, e);
    va = static_cast<char*>(got);
    if (!a.base) a.base = va;
    if (hint && va == hint) ++a.hinted;
    else if (hint) ++a.hint_missed;
    if (va >= a.base) a.top = std::max(a.top, static_cast<size_t>(va - a.base) + sz);
    own = true;
  }
  auto give_back = [&]() { a.free_ranges.emplace(sz, va); };  // the range stays reserved for a later segment
  hipMemAllocationProp p = prop_for(device);
  hipMemGenericAllocationHandle_t h;
  if (hipError_t e = hipMemCreate(&h, sz, &p, 0)) {
    give_back();
    return failed(a, 2, e);
  }
  if (hipError_t e = hipMemMap(va, sz, 0, h, 0)) {
    (void)hipMemRelease(h);
    give_back();
    return failed(a, 3, e);
  }
  hipMemAccessDesc d{};
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = device;
  d.flags = hipMemAccessFlagsProtReadWrite;
  if (hipError_t e = hipMemSetAccess(va, sz, &d, 1)) {
    (void)hipMemUnmap(va, sz);
    (void)hipMemRelease(h);
    give_back();
    return failed(a, 4, e);
  }
  a.live[reinterpret_cast<uintptr_t>(va)] = Segment{sz, h, own, false};
  a.mapped_bytes += static_cast<int64_t>(sz);
  ++a.segments;
  return va;
}

void fjalloc_free(void* ptr, size_t /*size*/, int device, void* stream) {
  if (!ptr || device < 0 || device >= kMaxDevices) return;
  Arena& a = g_arena[device];
  // torch's caching allocator releases a segment only when none of its blocks is in use
  // (empty_cache, or an out-of-memory retry); wait for work queued on the segment's stream
  (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
  std::lock_guard<std::mutex> lock(a.mu);
  auto it = a.live.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == a.live.end()) return;
  const Segment s = it->second;
  a.live.erase(it);
  a.mapped_bytes -= static_cast<int64_t>(s.size);
  if (s.chunk_slice) {
    chunk_free(a, device, static_cast<char*>(ptr), s.size, s.pad);
    return;
  }
  (void)hipMemUnmap(ptr, s.size);
  (void)hipMemRelease(s.handle);
  a.free_ranges.emplace(s.size, static_cast<char*>(ptr));
}

int fjalloc_stats(int device, int64_t* out) {
  if (!out || device < 0 || device >= kMaxDevices) return -1;
  Arena& a = g_arena[device];
  std::lock_guard<std::mutex> lock(a.mu);
  out[0] = a.mapped_bytes;
  out[1] = static_cast<int64_t>(a.live.size());
  out[2] = a.segments;
  out[3] = a.reuses;
  out[4] = a.failures;
  out[5] = static_cast<int64_t>(a.gran);
  out[6] = static_cast<int64_t>(g_mode == 2 ? (a.chunks.empty() ? 0 : a.chunks[0].top) : a.top);  // (mode 2: of the first chunk)
  out[7] = reinterpret_cast<int64_t>(a.base);
  out[8] = a.last_error;
  out[9] = a.hinted;
  out[10] = a.hint_missed;
  out[11] = static_cast<int64_t>(a.chunks.size());
  int64_t fr = 0;
  for (const auto& r : a.chunk_free_ranges) fr += static_cast<int64_t>(r.second);
  out[12] = fr;
  return 0;
}

int fjalloc_configure(int64_t reserve_bytes, int64_t align_bytes, int mode, int64_t stagger_bytes) {
  if (reserve_bytes <= 0 || align_bytes <= 0 || mode < 0 || mode > 2 || stagger_bytes < 0 || stagger_bytes % 256)
    return -1;
  std::unique_lock<std::shared_mutex> config(g_config_mu);  // no allocation runs meanwhile
  for (Arena& a : g_arena) {  // the layout is fixed once any device has a segment
    std::lock_guard<std::mutex> lock(a.mu);
    if (a.segments > 0) return -1;
  }
  g_stagger = static_cast<size_t>(stagger_bytes);
  g_reserve_bytes = static_cast<size_t>(reserve_bytes);
  g_chunk_bytes = static_cast<size_t>(reserve_bytes);  // mode 2: the chunk size
  g_align = static_cast<size_t>(align_bytes);
  g_mode = mode;
  return 0;
}

}  // extern "C"
