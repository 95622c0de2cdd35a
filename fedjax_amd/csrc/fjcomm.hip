// fjcomm.hip — client-sharded weighted mean over the GPUs of one node: each rank folds
// its clients with the dense fold of fjagg.hip, RCCL sums the per-rank partials over
// xGMI. C ABI and the pipeline it issues: include/fjcomm.h.
//
// Every bucket but the last is reduced on the communicator's own high-priority stream,
// waiting only for that bucket's fold (an event with a device-scope release), so those
// reduces overlap the following folds; the last bucket is reduced on the caller's
// stream, because a cross-queue hop back costs ~30 us of GPU-side latency on MI355X
// (profiles/r01g_*) and nothing is left to overlap it with.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <thread>

#include "fjagg.h"
#include "fjcomm.h"

extern thread_local char fjagg_g_err[512];
// fjagg.hip (same library): whether a dense fold can take FJAGG_HOST_TABLES weights
int fjagg_host_weights_check(int in_dtype, int acc_dtype, int out_dtype, int64_t K, int64_t P, int flags);

namespace {

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(fjagg_g_err, sizeof(fjagg_g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(FJAGG_EHIP, "%s: %s", what, hipGetErrorString(e));
}

// ------------------------------------------------------------------ RCCL, resolved at run time
// Declared here with the ABI of rccl.h (ncclResult_t / ncclDataType_t / ncclRedOp_t are
// C enums, ncclComm_t a pointer, ncclUniqueId 128 opaque bytes).
struct NcclId {
  char internal[FJCOMM_ID_BYTES];
};
typedef void* NcclComm;
constexpr int kNcclSuccess = 0;
constexpr int kNcclFloat32 = 7;
constexpr int kNcclSum = 0;

struct Rccl {
  int (*get_unique_id)(NcclId*) = nullptr;
  int (*comm_init_rank)(NcclComm*, int, NcclId, int) = nullptr;
  int (*comm_init_all)(NcclComm*, int, const int*) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  int (*comm_destroy)(NcclComm) = nullptr;
  int (*comm_abort)(NcclComm) = nullptr;  // (optional: fjcomm_abort)
  int (*reduce)(const void*, void*, size_t, int, int, int, NcclComm, hipStream_t) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, NcclComm, hipStream_t) = nullptr;
  const char* (*error_string)(int) = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl t;
    // the copy torch loaded (libtorch_hip needs librccl.so.1), else the system one
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return t;
    t.get_unique_id = reinterpret_cast<decltype(t.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    t.comm_init_rank = reinterpret_cast<decltype(t.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    t.comm_destroy = reinterpret_cast<decltype(t.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    t.comm_abort = reinterpret_cast<decltype(t.comm_abort)>(dlsym(h, "ncclCommAbort"));
    t.comm_init_all = reinterpret_cast<decltype(t.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    t.group_start = reinterpret_cast<decltype(t.group_start)>(dlsym(h, "ncclGroupStart"));
    t.group_end = reinterpret_cast<decltype(t.group_end)>(dlsym(h, "ncclGroupEnd"));
    t.reduce = reinterpret_cast<decltype(t.reduce)>(dlsym(h, "ncclReduce"));
    t.all_reduce = reinterpret_cast<decltype(t.all_reduce)>(dlsym(h, "ncclAllReduce"));
    t.error_string = reinterpret_cast<decltype(t.error_string)>(dlsym(h, "ncclGetErrorString"));
    t.ok = t.get_unique_id && t.comm_init_rank && t.comm_destroy && t.reduce && t.all_reduce && t.error_string &&
           t.comm_init_all && t.group_start && t.group_end;
    return t;
  }();
  return r;
}

int nccl_fail(int rc, const char* what) {
  return fail(FJAGG_EHIP, "%s: RCCL error %d (%s)", what, rc, rccl().error_string ? rccl().error_string(rc) : "?");
}

int need_rccl() {
  if (!rccl().ok) return fail(FJAGG_EUNSUPPORTED, "librccl.so.1 (ncclGetUniqueId, ncclCommInitRank, ...) not found");
  return FJAGG_OK;
}

struct Comm {
  NcclComm nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
  bool aborted = false;  // fjcomm_abort ran: every later step is refused
  hipStream_t cs = nullptr;
  hipEvent_t ready[FJCOMM_MAX_BUCKETS] = {};
  hipEvent_t done = nullptr;
};

// Cross-stream dependency events: no timing, device-scope release.
hipError_t make_dep_event(hipEvent_t* e) {
  hipError_t rc = hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice);
  if (rc != hipSuccess) {  // runtime without the release flags: plain untimed event
    (void)hipGetLastError();
    rc = hipEventCreateWithFlags(e, hipEventDisableTiming);
  }
  return rc;
}

// The communicator's own stream (highest priority) and its events, on the current device.
hipError_t make_comm_resources(Comm* c) {
  hipError_t e = hipGetDevice(&c->device);
  int lo = 0, hi = 0;
  if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->cs, hipStreamNonBlocking, hi);
  for (int b = 0; e == hipSuccess && b < FJCOMM_MAX_BUCKETS; ++b) e = make_dep_event(&c->ready[b]);
  if (e == hipSuccess) e = make_dep_event(&c->done);
  return e;
}

// Restores the calling thread's current HIP device on scope exit.
struct DeviceGuard {
  int saved = -1;
  DeviceGuard() { (void)hipGetDevice(&saved); }
  ~DeviceGuard() {
    if (saved >= 0) (void)hipSetDevice(saved);
  }
};

int check_edges(const int64_t* edges, int nbuckets, int64_t P) {
  if (nbuckets < 1 || nbuckets > FJCOMM_MAX_BUCKETS)
    return fail(FJAGG_EINVAL, "nbuckets must be in [1, %d]", FJCOMM_MAX_BUCKETS);
  if (!edges) return fail(FJAGG_EINVAL, "null edges");
  if (edges[0] != 0 || edges[nbuckets] != P)
    return fail(FJAGG_EINVAL, "edges must run from 0 to P = %lld", (long long)P);
  for (int b = 0; b < nbuckets; ++b) {
    if (edges[b + 1] <= edges[b]) return fail(FJAGG_EINVAL, "edges must increase strictly (bucket %d)", b);
    if (edges[b] % FJCOMM_BUCKET_ALIGN)
      return fail(FJAGG_EINVAL, "edge %lld is not a multiple of %d elements", (long long)edges[b],
                  FJCOMM_BUCKET_ALIGN);
  }
  return FJAGG_OK;
}

}  // namespace

extern "C" {

int fjcomm_abi_version(void) { return FJCOMM_ABI_VERSION; }

int fjcomm_unique_id(uint8_t* id) {
  fjagg_g_err[0] = 0;
  if (int rc = need_rccl()) return rc;
  if (!id) return fail(FJAGG_EINVAL, "null id");
  NcclId u;
  if (int rc = rccl().get_unique_id(&u)) return nccl_fail(rc, "ncclGetUniqueId");
  memcpy(id, u.internal, FJCOMM_ID_BYTES);
  return FJAGG_OK;
}

int fjcomm_init(void** comm, const uint8_t* id, int nranks, int rank) {
  fjagg_g_err[0] = 0;
  if (int rc = need_rccl()) return rc;
  if (!comm || !id) return fail(FJAGG_EINVAL, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(FJAGG_EINVAL, "bad rank %d of %d", rank, nranks);
  Comm* c = new Comm();
  c->nranks = nranks;
  c->rank = rank;
  hipError_t e = make_comm_resources(c);
  if (e != hipSuccess) {
    int rc = hip_fail(e, "fjcomm_init");
    fjcomm_destroy(c);
    return rc;
  }
  NcclId u;
  memcpy(u.internal, id, FJCOMM_ID_BYTES);
  if (int rc = rccl().comm_init_rank(&c->nc, nranks, u, rank)) {
    rc = nccl_fail(rc, "ncclCommInitRank");
    c->nc = nullptr;
    fjcomm_destroy(c);
    return rc;
  }
  *comm = c;
  return FJAGG_OK;
}

int fjcomm_destroy(void* comm) {
  Comm* c = reinterpret_cast<Comm*>(comm);
  if (!c) return FJAGG_OK;
  DeviceGuard guard;  // the communicator's resources live on its device
  (void)hipSetDevice(c->device);
  if (c->aborted && c->cs) {
    // after an abort the stream may still hold work that never ends: wait a bounded time, and
    // past it leave the stream and its events alive (leaked) rather than block the caller
    const auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(c->cs) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
        delete c;
        return fail(FJAGG_EHIP, "fjcomm_destroy: the aborted communicator's stream did not drain in 10 s (leaked)");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  } else if (c->cs) {
    (void)hipStreamSynchronize(c->cs);
  }
  if (c->nc && rccl().ok) rccl().comm_destroy(c->nc);
  for (hipEvent_t& e : c->ready)
    if (e) (void)hipEventDestroy(e);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->cs) (void)hipStreamDestroy(c->cs);
  delete c;
  return FJAGG_OK;
}

int fjcomm_abort(void* comm) {
  fjagg_g_err[0] = 0;
  Comm* c = reinterpret_cast<Comm*>(comm);
  if (!c) return fail(FJAGG_EINVAL, "null communicator");
  if (c->aborted) return FJAGG_OK;
  if (!rccl().comm_abort) return fail(FJAGG_EUNSUPPORTED, "librccl.so.1 has no ncclCommAbort");
  DeviceGuard guard;
  (void)hipSetDevice(c->device);
  c->aborted = true;
  NcclComm nc = c->nc;
  c->nc = nullptr;
  if (nc) {
    if (int rc = rccl().comm_abort(nc)) return nccl_fail(rc, "ncclCommAbort");
  }
  return FJAGG_OK;
}

namespace {
// n zero floats at p (a shard without clients): a kernel, not hipMemsetAsync, whose node in a
// captured graph takes effect on the first replay only (measured: tools/probe_memset_node.py)
__global__ __launch_bounds__(256) void k_zero_f32(float* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0.0f;
}
int zero_f32(float* p, int64_t n, hipStream_t s) {
  if (n <= 0) return FJAGG_OK;
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(k_zero_f32, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s, p, n);
  if (hipError_t e = hipGetLastError()) return hip_fail(e, "k_zero_f32 launch");
  return FJAGG_OK;
}

// a bounded spin on the real-time counter (read-only; no memory is touched): one wave
__global__ void k_block(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

int fjcomm_test_block(int64_t us, void* stream) {
  fjagg_g_err[0] = 0;
  if (us < 0 || us > 60LL * 1000 * 1000) return fail(FJAGG_EINVAL, "us must be in [0, 60 s]");
  int dev = 0, khz = 0;
  if (hipError_t e = hipGetDevice(&dev)) return hip_fail(e, "hipGetDevice");
  if (hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev)) return hip_fail(e, "wall clock rate");
  if (khz <= 0) khz = 100000;  // (gfx9's s_memrealtime: 100 MHz)
  hipLaunchKernelGGL(k_block, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), (long long)(us * khz / 1000));
  if (hipError_t e = hipGetLastError()) return hip_fail(e, "k_block launch");
  return FJAGG_OK;
}

int fjcomm_sharded_wsum_dense(void* comm, int in_dtype, const void* x_dev, int64_t ld, int64_t K,
                              int64_t P, const void* w_dev, float scale, float* out_dev,
                              int nbuckets, int root, int flags, void* stream, void* const* fold_events) {
  fjagg_g_err[0] = 0;
  if (nbuckets < 1 || nbuckets > FJCOMM_MAX_BUCKETS)
    return fail(FJAGG_EINVAL, "nbuckets must be in [1, %d]", FJCOMM_MAX_BUCKETS);
  if (P <= 0)  // nothing to cut; the edges variant validates the rest
    return fjcomm_sharded_wsum_dense_edges(comm, in_dtype, x_dev, ld, K, P, w_dev, scale, out_dev, nullptr, 1,
                                           root, flags, stream, fold_events);
  // equal buckets of a multiple of FJCOMM_BUCKET_ALIGN elements (the last one shorter)
  int64_t step = (P + nbuckets - 1) / nbuckets;
  step = (step + FJCOMM_BUCKET_ALIGN - 1) / FJCOMM_BUCKET_ALIGN * FJCOMM_BUCKET_ALIGN;
  const int nb = (int)((P + step - 1) / step);
  int64_t edges[FJCOMM_MAX_BUCKETS + 1];
  for (int b = 0; b < nb; ++b) edges[b] = b * step;
  edges[nb] = P;
  return fjcomm_sharded_wsum_dense_edges(comm, in_dtype, x_dev, ld, K, P, w_dev, scale, out_dev, edges, nb, root,
                                         flags, stream, fold_events);
}

int fjcomm_sharded_wsum_dense_edges(void* comm, int in_dtype, const void* x_dev, int64_t ld, int64_t K,
                                    int64_t P, const void* w_dev, float scale, float* out_dev,
                                    const int64_t* edges, int nbuckets, int root, int flags, void* stream,
                                    void* const* fold_events) {
  fjagg_g_err[0] = 0;
  Comm* c = reinterpret_cast<Comm*>(comm);
  if (c && c->aborted) return fail(FJAGG_EINVAL, "the communicator was aborted (fjcomm_abort)");
  if (!c || !c->nc) return fail(FJAGG_EINVAL, "not an initialised communicator");
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16) return fail(FJAGG_EINVAL, "in_dtype must be F32 or BF16");
  if (K < 0 || P < 0 || ld < P) return fail(FJAGG_EINVAL, "need K >= 0 and 0 <= P <= ld");
  if (nbuckets < 1 || nbuckets > FJCOMM_MAX_BUCKETS)
    return fail(FJAGG_EINVAL, "nbuckets must be in [1, %d]", FJCOMM_MAX_BUCKETS);
  if (root >= c->nranks) return fail(FJAGG_EINVAL, "root %d >= nranks %d", root, c->nranks);
  if (P == 0) return FJAGG_OK;
  if (int rc = check_edges(edges, nbuckets, P)) return rc;
  if (!out_dev || (K > 0 && (!x_dev || !w_dev))) return fail(FJAGG_EINVAL, "null pointer argument");
  if (flags & ~(FJAGG_NONTEMPORAL | FJAGG_HOST_TABLES | FJAGG_VARIANT(0xff)))
    return fail(FJAGG_EINVAL, "flags may hold FJAGG_NONTEMPORAL, FJAGG_HOST_TABLES and FJAGG_VARIANT bits only");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t esz = in_dtype == FJAGG_BF16 ? 2 : 4;
  const int nb = nbuckets;
  if ((flags & FJAGG_HOST_TABLES) && K > 0)  // every bucket's fold must take them: refuse before any launch
    for (int b = 0; b < nb; ++b)
      if (int rc = fjagg_host_weights_check(in_dtype, FJAGG_F32, FJAGG_F32, K, edges[b + 1] - edges[b], flags))
        return rc;
  for (int b = 0; b < nb; ++b) {
    const int64_t p0 = edges[b];
    const int64_t n = edges[b + 1] - p0;
    float* seg = out_dev + p0;
    if (fold_events) {
      if (hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(fold_events[2 * b]), s))
        return hip_fail(e, "hipEventRecord");
    }
    if (K > 0) {
      const uint8_t* xb = reinterpret_cast<const uint8_t*>(x_dev) + p0 * esz;
      if (int rc = fjagg_wsum_dense(in_dtype, FJAGG_F32, FJAGG_F32, xb, ld, K, n, w_dev, scale, seg,
                                    flags | FJAGG_SCALE, FJAGG_MODE_EXACT, nullptr, 0, stream))
        return rc;
    } else if (int rc = zero_f32(seg, n, s)) {
      return rc;
    }
    if (fold_events) {
      if (hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(fold_events[2 * b + 1]), s))
        return hip_fail(e, "hipEventRecord");
    }
    // Buckets before the last reduce on the communicator's stream, overlapping the next
    // fold. The last one is reduced on the caller's stream itself: a cross-queue hop costs
    // ~30 us of GPU-side latency on MI355X (profiles/r01g_*), and nothing is left to overlap.
    hipStream_t rs = s;
    if (b + 1 < nb) {
      if (hipError_t e = hipEventRecord(c->ready[b], s)) return hip_fail(e, "hipEventRecord");
      if (hipError_t e = hipStreamWaitEvent(c->cs, c->ready[b], 0)) return hip_fail(e, "hipStreamWaitEvent");
      rs = c->cs;
    } else if (nb > 1) {  // collectives of one communicator stay in issue order
      if (hipError_t e = hipEventRecord(c->done, c->cs)) return hip_fail(e, "hipEventRecord");
      if (hipError_t e = hipStreamWaitEvent(s, c->done, 0)) return hip_fail(e, "hipStreamWaitEvent");
    }
    const int rc = root >= 0
                       ? rccl().reduce(seg, seg, (size_t)n, kNcclFloat32, kNcclSum, root, c->nc, rs)
                       : rccl().all_reduce(seg, seg, (size_t)n, kNcclFloat32, kNcclSum, c->nc, rs);
    if (rc != kNcclSuccess) return nccl_fail(rc, root >= 0 ? "ncclReduce" : "ncclAllReduce");
  }
  return FJAGG_OK;
}

int fjcomm_init_all(void** comms, int ndev, const int* devs) {
  fjagg_g_err[0] = 0;
  if (int rc = need_rccl()) return rc;
  if (!comms || !devs) return fail(FJAGG_EINVAL, "null argument");
  if (ndev < 1 || ndev > FJCOMM_MAX_DEVICES) return fail(FJAGG_EINVAL, "ndev must be in [1, %d]", FJCOMM_MAX_DEVICES);
  for (int d = 0; d < ndev; ++d) {
    comms[d] = nullptr;
    for (int e = 0; e < d; ++e)
      if (devs[e] == devs[d]) return fail(FJAGG_EINVAL, "device %d listed twice", devs[d]);
  }
  DeviceGuard guard;
  Comm* cs[FJCOMM_MAX_DEVICES] = {};
  NcclComm nc[FJCOMM_MAX_DEVICES] = {};
  int rc = FJAGG_OK;
  for (int d = 0; d < ndev && rc == FJAGG_OK; ++d) {
    cs[d] = new Comm();
    cs[d]->nranks = ndev;
    cs[d]->rank = d;
    hipError_t e = hipSetDevice(devs[d]);
    if (e == hipSuccess) e = make_comm_resources(cs[d]);
    if (e != hipSuccess) rc = hip_fail(e, "fjcomm_init_all");
  }
  if (rc == FJAGG_OK) {
    if (int nr = rccl().comm_init_all(nc, ndev, devs)) rc = nccl_fail(nr, "ncclCommInitAll");
  }
  if (rc != FJAGG_OK) {
    for (int d = 0; d < ndev; ++d)
      if (cs[d]) {
        cs[d]->nc = nc[d];
        (void)hipSetDevice(cs[d]->device);
        fjcomm_destroy(cs[d]);
      }
    return rc;
  }
  for (int d = 0; d < ndev; ++d) {
    cs[d]->nc = nc[d];
    comms[d] = cs[d];
  }
  return FJAGG_OK;
}

int fjcomm_multi_wsum_dense(void* const* comms, int ndev, int in_dtype, const void* const* x_dev,
                            const int64_t* ld, const int64_t* K, int64_t P, const void* const* w_dev, float scale,
                            float* const* out_dev, const int64_t* edges, int nbuckets, int root, int flags,
                            void* const* streams) {
  fjagg_g_err[0] = 0;
  if (!comms || !x_dev || !ld || !K || !w_dev || !out_dev || !streams) return fail(FJAGG_EINVAL, "null argument");
  if (ndev < 1 || ndev > FJCOMM_MAX_DEVICES) return fail(FJAGG_EINVAL, "ndev must be in [1, %d]", FJCOMM_MAX_DEVICES);
  if (in_dtype != FJAGG_F32 && in_dtype != FJAGG_BF16) return fail(FJAGG_EINVAL, "in_dtype must be F32 or BF16");
  if (P < 0) return fail(FJAGG_EINVAL, "P < 0");
  if (root >= ndev) return fail(FJAGG_EINVAL, "root %d >= ndev %d", root, ndev);
  if (flags & ~(FJAGG_NONTEMPORAL | FJAGG_HOST_TABLES | FJAGG_VARIANT(0xff)))
    return fail(FJAGG_EINVAL, "flags may hold FJAGG_NONTEMPORAL, FJAGG_HOST_TABLES and FJAGG_VARIANT bits only");
  Comm* cs[FJCOMM_MAX_DEVICES];
  for (int d = 0; d < ndev; ++d) {
    cs[d] = reinterpret_cast<Comm*>(comms[d]);
    if (cs[d] && cs[d]->aborted) return fail(FJAGG_EINVAL, "comms[%d] was aborted (fjcomm_abort)", d);
    if (!cs[d] || !cs[d]->nc) return fail(FJAGG_EINVAL, "comms[%d] is not an initialised communicator", d);
    if (cs[d]->rank != d || cs[d]->nranks != ndev)
      return fail(FJAGG_EINVAL, "comms[%d] is rank %d of %d, not %d of %d (pass fjcomm_init_all's handles in order)",
                  d, cs[d]->rank, cs[d]->nranks, d, ndev);
    if (K[d] < 0 || ld[d] < P || !out_dev[d] || (K[d] > 0 && (!x_dev[d] || !w_dev[d])))
      return fail(FJAGG_EINVAL, "device %d: need K >= 0, ld >= P and non-null pointers", d);
  }
  if (P == 0) return FJAGG_OK;
  if (int rc = check_edges(edges, nbuckets, P)) return rc;
  DeviceGuard guard;
  const int64_t esz = in_dtype == FJAGG_BF16 ? 2 : 4;
  const int nb = nbuckets;
  if (flags & FJAGG_HOST_TABLES)  // every device's every bucket must take them: refuse before any launch
    for (int d = 0; d < ndev; ++d)
      for (int b = 0; K[d] > 0 && b < nb; ++b)
        if (int rc = fjagg_host_weights_check(in_dtype, FJAGG_F32, FJAGG_F32, K[d], edges[b + 1] - edges[b], flags))
          return rc;
  for (int b = 0; b < nb; ++b) {
    const int64_t p0 = edges[b], n = edges[b + 1] - p0;
    // every device folds its clients' share of bucket b on its own stream, then signals
    // its communicator stream (all but the last bucket, as in the one-rank-per-process path)
    for (int d = 0; d < ndev; ++d) {
      Comm* c = cs[d];
      hipStream_t s = reinterpret_cast<hipStream_t>(streams[d]);
      if (hipError_t e = hipSetDevice(c->device)) return hip_fail(e, "hipSetDevice");
      float* seg = out_dev[d] + p0;
      if (K[d] > 0) {
        const uint8_t* xb = reinterpret_cast<const uint8_t*>(x_dev[d]) + p0 * esz;
        if (int rc = fjagg_wsum_dense(in_dtype, FJAGG_F32, FJAGG_F32, xb, ld[d], K[d], n, w_dev[d], scale, seg,
                                      flags | FJAGG_SCALE, FJAGG_MODE_EXACT, nullptr, 0, s))
          return rc;
      } else if (int rc = zero_f32(seg, n, s)) {
        return rc;
      }
      if (b + 1 < nb) {
        if (hipError_t e = hipEventRecord(c->ready[b], s)) return hip_fail(e, "hipEventRecord");
        if (hipError_t e = hipStreamWaitEvent(c->cs, c->ready[b], 0)) return hip_fail(e, "hipStreamWaitEvent");
      } else if (nb > 1) {
        if (hipError_t e = hipEventRecord(c->done, c->cs)) return hip_fail(e, "hipEventRecord");
        if (hipError_t e = hipStreamWaitEvent(s, c->done, 0)) return hip_fail(e, "hipStreamWaitEvent");
      }
    }
    // one process drives every device: the collectives of a bucket are one RCCL group
    if (int r = rccl().group_start()) return nccl_fail(r, "ncclGroupStart");
    int rc = kNcclSuccess;
    for (int d = 0; d < ndev && rc == kNcclSuccess; ++d) {
      Comm* c = cs[d];
      hipStream_t rs = b + 1 < nb ? c->cs : reinterpret_cast<hipStream_t>(streams[d]);
      float* seg = out_dev[d] + p0;
      rc = root >= 0 ? rccl().reduce(seg, seg, (size_t)n, kNcclFloat32, kNcclSum, root, c->nc, rs)
                     : rccl().all_reduce(seg, seg, (size_t)n, kNcclFloat32, kNcclSum, c->nc, rs);
    }
    const int ge = rccl().group_end();
    if (rc != kNcclSuccess) return nccl_fail(rc, root >= 0 ? "ncclReduce" : "ncclAllReduce");
    if (ge != kNcclSuccess) return nccl_fail(ge, "ncclGroupEnd");
  }
  return FJAGG_OK;
}

int fjagg_event_create(void** ev) {
  fjagg_g_err[0] = 0;
  if (!ev) return fail(FJAGG_EINVAL, "null argument");
  hipEvent_t e = nullptr;
  hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  if (rc != hipSuccess) {
    (void)hipGetLastError();
    rc = hipEventCreateWithFlags(&e, hipEventDefault);
  }
  if (rc != hipSuccess) return hip_fail(rc, "hipEventCreateWithFlags");
  *ev = e;
  return FJAGG_OK;
}

int fjagg_event_destroy(void* ev) {
  if (ev) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev));
  return FJAGG_OK;
}

int fjagg_event_record(void* ev, void* stream) {
  fjagg_g_err[0] = 0;
  if (hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(ev), reinterpret_cast<hipStream_t>(stream)))
    return hip_fail(e, "hipEventRecord");
  return FJAGG_OK;
}

int fjagg_event_elapsed_ms(float* ms, void* start, void* end) {
  fjagg_g_err[0] = 0;
  if (!ms) return fail(FJAGG_EINVAL, "null argument");
  if (hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(end))) return hip_fail(e, "hipEventSynchronize");
  if (hipError_t e = hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(end)))
    return hip_fail(e, "hipEventElapsedTime");
  return FJAGG_OK;
}

}  // extern "C"
