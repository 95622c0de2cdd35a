// fjagg_dev.h — device helpers shared by the fold kernels of libfjagg.so (fjagg.hip) and
// the stripe-pipeline kernel (fjstripe.hip): element types, fold arithmetic policies
// (AccF / AccI / AccB: the reference's f32, int32 and bf16 op sequences), 16-byte units,
// buffer-resource row loads and the output encoders. Internal to the library (anonymous
// namespace: each translation unit gets its own copy); the C ABI is include/fjagg.h.
#pragma once
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "fjagg.h"

// The thread-local message behind fjagg_last_error() (defined in fjagg.hip).
extern __attribute__((visibility("hidden"))) thread_local char fjagg_g_err[512];
#define g_err fjagg_g_err

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));


int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FJAGG_EHIP, "%s: %s", what, hipGetErrorString(e));
  return FJAGG_OK;
}

constexpr int kThreads = 256;   // 4 waves of 64
constexpr int kSplitMax = 64;   // max client ranges in FJAGG_MODE_SPLIT
constexpr int64_t kSplitHeader = 256;  // bytes of ones at the head of the split workspace

// FJAGG_HOST_TABLES: tables passed BY VALUE in the kernel arguments. An aggregate
// kernel argument lives in the kernarg segment, and the kernels read it in place
// through a pointer (scalar loads, no private copy: these kernels have no scratch).
// The launch copies the struct, so the caller's host tables are free on return.
// Kernels built without the feature take a 4-byte placeholder (N = 1).
template <int N> struct KargWords { int64_t w[N]; };
template <int N> struct KargF32 { float w[N]; };
constexpr int kKargWeights = FJAGG_KARG_MAX_WEIGHTS;  // dense: f32 / i32 weights
constexpr int kKargWords = FJAGG_KARG_MAX_WORDS;      // pytree: image + packed f32 weights

// ---------------------------------------------------------------- element types
template <int DT> struct Elem;
template <> struct Elem<FJAGG_F32> { static constexpr int B = 4; };
template <> struct Elem<FJAGG_BF16> { static constexpr int B = 2; };
template <> struct Elem<FJAGG_I32> { static constexpr int B = 4; };

template <int IN> constexpr int vec_width() { return 16 / Elem<IN>::B; }

__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ unsigned f32_to_bf16(float f) {  // RNE, NaN stays NaN
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return ((u >> 16) | 0x40u) & 0xffffu;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// Fold arithmetic policies: T is the fold state, weight() maps a weight as stored in
// w_dev (and the final scale) to the value the fold multiplies by.
struct AccF {
  using T = float;
  static constexpr int DT = FJAGG_F32;
  static __device__ __forceinline__ T weight(T w) { return w; }
  static __device__ __forceinline__ T mul(T x, T w) { return __fmul_rn(x, w); }
  static __device__ __forceinline__ T add(T a, T b) { return __fadd_rn(a, b); }
};
struct AccI {  // XLA int32 arithmetic wraps
  using T = int;
  static constexpr int DT = FJAGG_I32;
  static __device__ __forceinline__ T weight(T w) { return w; }
  static __device__ __forceinline__ T mul(T x, T w) { return (int)((unsigned)x * (unsigned)w); }
  static __device__ __forceinline__ T add(T a, T b) { return (int)((unsigned)a + (unsigned)b); }
};
// The reference's bfloat16 arithmetic (jnp on bf16 leaves, tree_util.py:32,50,60, weights
// weakly typed): the weight and the scale become bf16, every product and every sum is
// rounded to bf16. Each op runs in f32 and is rounded once to bf16 (RNE): the product of
// two bf16 values is exact in f32, and for sums f32's 24 bits >= 2*8 + 2 make the double
// rounding innocuous (Figueroa), so every op is the correctly rounded bf16 op. Values
// stay bf16-representable floats; NaNs that reach rnd() come from bf16 data or from the
// hardware's default NaN (low 16 bits zero), so the NaN-preserving branch is not needed
// there — weight() keeps it for caller-supplied weights.
struct AccB {
  using T = float;
  static constexpr int DT = FJAGG_BF16;
  static __device__ __forceinline__ T rnd(T f) {
    const unsigned u = __float_as_uint(f);
    return __uint_as_float((u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
  }
  static __device__ __forceinline__ T weight(T w) { return __uint_as_float(f32_to_bf16(w) << 16); }
  static __device__ __forceinline__ T mul(T x, T w) { return rnd(__fmul_rn(x, w)); }
  static __device__ __forceinline__ T add(T a, T b) { return rnd(__fadd_rn(a, b)); }
};

// A "unit" is what one lane loads per client: 16 bytes (V = vec_width) or one
// element (V = 1).
template <int IN, int V> struct Unit {
  static constexpr int BYTES = V * Elem<IN>::B;
  using Raw = typename std::conditional<(BYTES == 16), u32x4, unsigned>::type;
};

// Buffer resource over one client row: base in SGPRs, range-checked to `bytes`
// (out-of-range lanes read zeros). gfx950 word-3 flags as in the HIP guide (T8).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const uint8_t* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

// One unit of a client row via buffer_load with a 32-bit lane offset: no per-load
// address VGPRs (aux 2 = nt).
// Bytes a rebased row descriptor covers: what is left of the row, capped to the
// descriptor's 31-bit record count (a workgroup never reaches that far).
__device__ __forceinline__ uint32_t row_range(int64_t bytes) {
  return (uint32_t)(bytes < 0x7fffffffll ? bytes : 0x7fffffffll);
}

template <int IN, int V, bool NT>
__device__ __forceinline__ typename Unit<IN, V>::Raw load_unit(__amdgpu_buffer_rsrc_t r,
                                                               uint32_t off) {
  constexpr int aux = NT ? 2 : 0;
  if constexpr (Unit<IN, V>::BYTES == 16) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, aux);
  } else if constexpr (Elem<IN>::B == 4) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, aux);
  } else {
    return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, aux);
  }
}

template <int IN, int V, bool NT>
__device__ __forceinline__ typename Unit<IN, V>::Raw load_unit_ptr(const uint8_t* p) {
  if constexpr (Unit<IN, V>::BYTES == 16) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  } else if constexpr (Elem<IN>::B == 4) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p));
    else return *reinterpret_cast<const unsigned*>(p);
  } else {
    if constexpr (NT) return (unsigned)__builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(p));
    else return (unsigned)*reinterpret_cast<const unsigned short*>(p);
  }
}

// One 16-byte unit through a GLOBAL (address space 1) pointer: global_load, counted in
// vmcnt only. (A generic pointer becomes a flat load, which also counts in lgkmcnt, so every
// LDS wait of the kernel would wait for it too.)
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
template <bool NT>
__device__ __forceinline__ u32x4 load16_global(const uint8_t* p) {
  gu32x4* g = (gu32x4*)(reinterpret_cast<uintptr_t>(p));
  if constexpr (NT) return __builtin_nontemporal_load(g);
  else return *g;
}

template <int IN, class ACC, int V>
__device__ __forceinline__ void decode(typename Unit<IN, V>::Raw r, typename ACC::T (&o)[V]) {
  if constexpr (V == 1) {
    if constexpr (IN == FJAGG_BF16) o[0] = bf16_lo(r);
    else if constexpr (IN == FJAGG_F32) o[0] = __uint_as_float(r);
    else if constexpr (ACC::DT == FJAGG_F32) o[0] = (float)(int)r;
    else o[0] = (int)r;
  } else if constexpr (IN == FJAGG_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = bf16_lo(r[i]);
      o[2 * i + 1] = bf16_hi(r[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (IN == FJAGG_F32) o[i] = __uint_as_float(r[i]);
      else if constexpr (ACC::DT == FJAGG_F32) o[i] = (float)(int)r[i];
      else o[i] = (int)r[i];
    }
  }
}

// fold state -> output element bits
template <int OUT, class ACC>
__device__ __forceinline__ unsigned finish(typename ACC::T s, bool do_scale, float scale) {
  if constexpr (ACC::DT == FJAGG_F32) {
    float f = do_scale ? __fmul_rn(s, scale) : s;
    if constexpr (OUT == FJAGG_BF16) return f32_to_bf16(f);
    else return __float_as_uint(f);
  } else if constexpr (ACC::DT == FJAGG_BF16) {  // out is bf16: fl_bf16(s * bf16(scale))
    return f32_to_bf16(do_scale ? ACC::mul(s, ACC::weight(scale)) : s);
  } else {
    if constexpr (OUT == FJAGG_I32) return (unsigned)s;  // scale rejected on the host
    else return __float_as_uint(do_scale ? __fmul_rn((float)s, scale) : (float)s);
  }
}

// output element bits -> fold state (FJAGG_ACCUMULATE)
template <int OUT, class ACC>
__device__ __forceinline__ typename ACC::T init_from(unsigned bits) {
  if constexpr (ACC::DT != FJAGG_I32) {
    if constexpr (OUT == FJAGG_BF16) return __uint_as_float(bits << 16);
    else return __uint_as_float(bits);
  } else {
    return (int)bits;
  }
}

template <int OUT, int V>
__device__ __forceinline__ void store_unit(uint8_t* p, const unsigned (&b)[V]) {
  constexpr int OB = Elem<OUT>::B;
  if constexpr (V == 1) {
    if constexpr (OB == 4) *reinterpret_cast<unsigned*>(p) = b[0];
    else *reinterpret_cast<unsigned short*>(p) = (unsigned short)b[0];
  } else if constexpr (OB == 2 && V == 8) {  // 8 bf16 (bf16 input units) -> 16 B
    u32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = b[2 * i] | (b[2 * i + 1] << 16);
    *reinterpret_cast<u32x4*>(p) = v;
  } else if constexpr (OB == 2) {  // 4 bf16 (float32 input units) -> 8 B
    static_assert(V == 4, "bf16 output units are 4 or 8 elements");
    u32x2 v;
    v[0] = b[0] | (b[1] << 16);
    v[1] = b[2] | (b[3] << 16);
    *reinterpret_cast<u32x2*>(p) = v;
  } else {  // V*4 bytes, V in {4, 8}
#pragma unroll
    for (int c = 0; c < V / 4; ++c) {
      u32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = b[4 * c + i];
      reinterpret_cast<u32x4*>(p)[c] = v;
    }
  }
}

template <int OUT, int V>
__device__ __forceinline__ void load_out_unit(const uint8_t* p, unsigned (&b)[V]) {
  constexpr int OB = Elem<OUT>::B;
  if constexpr (V == 1) {
    if constexpr (OB == 4) b[0] = *reinterpret_cast<const unsigned*>(p);
    else b[0] = *reinterpret_cast<const unsigned short*>(p);
  } else if constexpr (OB == 2 && V == 8) {
    u32x4 v = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      b[2 * i] = v[i] & 0xffffu;
      b[2 * i + 1] = v[i] >> 16;
    }
  } else if constexpr (OB == 2) {  // 4 bf16 of a float32 input unit: 8 B
    static_assert(V == 4, "bf16 output units are 4 or 8 elements");
    u32x2 v = *reinterpret_cast<const u32x2*>(p);
    b[0] = v[0] & 0xffffu;
    b[1] = v[0] >> 16;
    b[2] = v[1] & 0xffffu;
    b[3] = v[1] >> 16;
  } else {
#pragma unroll
    for (int c = 0; c < V / 4; ++c) {
      u32x4 v = reinterpret_cast<const u32x4*>(p)[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) b[4 * c + i] = v[i];
    }
  }
}

// CUs of the current device, queried once per device.
inline int cu_count() {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;
  }
  int c = __atomic_load_n(&cached[dev], __ATOMIC_RELAXED);
  if (c <= 0) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
    (void)hipGetLastError();
    __atomic_store_n(&cached[dev], c, __ATOMIC_RELAXED);
  }
  return c;
}

}  // namespace

// fjstripe.hip: k_dense_stripe launch (variant 19 auto width, 20 / 21 / 22 = 64 / 32 / 16
// columns) and the shapes it takes.
__attribute__((visibility("hidden"))) bool fjagg_stripe_ok(const uint8_t* x, int64_t ld_bytes, int64_t P,
                                                            const void* w, int ib);
__attribute__((visibility("hidden"))) int fjagg_launch_stripe(int variant, int in, int acc, int out,
                                                              const uint8_t* x, int64_t ld_bytes, int64_t K,
                                                              int64_t P, const void* w, float scale, uint8_t* y,
                                                              int flags, hipStream_t s);
// fjstripe.hip: k_ptrs_stripe launch over a FJAGG_NARROW plan of C-element stripes
// (C = 64 / 32 / 16: FJAGG_VARIANT 20 / 21 / 22); every client and output pointer 16-byte aligned.
__attribute__((visibility("hidden"))) int fjagg_launch_ptrs_stripe(int C, int in, int acc, int out, bool nt,
                                                                   const int64_t* img, int L, int64_t K,
                                                                   int64_t nblk, const void* w, float scale,
                                                                   int dsc, int acm, hipStream_t s);
