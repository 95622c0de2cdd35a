// fjstripe.hip — k_dense_stripe, the exact fold for a narrow parameter axis and many
// clients (fjagg_wsum_dense variants 19-22; chosen by fjagg.hip's dense_exact). Its own
// translation unit: the fold contract is fjagg.h's (bitwise the reference op sequence of
// fedjax/core/tree_util.py:85-96), the shared device helpers are fjagg_dev.h's.
#include "fjagg_dev.h"

namespace {

// ------------------------------------------------- stripe pipeline (narrow P, many K)
// k_dense_narrow's fold wave pays ~44 cycles per client (an LDS read, the weight, the
// multiply, the add, plus its share of the loads and the tile barrier), so a workgroup
// streams ~14 GB/s whatever the shape, and small P has too few stripes to fill the chip
// (16384 x 4 Ki f32: 64 stripes, 0.9 TB/s). The exact fold is a serial chain of K adds per
// element, so the fold wave must do nothing but those adds. Here:
//   * wave 0 only folds: per 4 clients one ds_read_b128 + 4 v_add (the tile is stored
//     transposed, column-major, 4 consecutive clients of one column in 16 bytes);
//   * waves 1-3 stream the stripe's rows with 16-byte buffer loads (D tiles in flight in
//     registers), multiply each value by its client's weight (t = fl(x*w), the product the
//     fold adds) and write the products transposed into the next LDS tile;
//   * stripes are C = 64, 32 or 16 columns wide, so P/C stripes fill the chip at small P;
//     stripe order is XCD-contiguous (neighbouring stripes share L2 lines);
//   * rows >= K of the last tile hold -0.0 (the additive identity: s + -0 == s for every s,
//     sign of zero included), and the fold starts from -0.0 (-0 + t_0 == t_0), so every
//     tile folds the same way and the per-element sequence is fold()'s: bitwise.
// Tile = 48 KiB of products (T = 12288 / C clients); two tile buffers + a 3-slot weight
// ring: one workgroup per CU.
constexpr int kStripeLoaders = 3;
template <int IB, int C>
struct StripeShape {
  static constexpr int VPL = 16 / IB;       // values per 16-byte load
  static constexpr int LPR = C / VPL;       // lanes per row segment
  static constexpr int RPI = 64 / LPR;      // rows per wave-instruction
  static constexpr int T = 12288 / C;       // clients per tile
  static constexpr int NI = T / RPI / kStripeLoaders;  // loads per loader lane per tile
  static constexpr int R4 = RPI / 4;        // 4-client groups per wave-instruction
  static_assert(NI * RPI * kStripeLoaders == T && T % 64 == 0 && LPR >= 1, "stripe shape");
};
constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }
// LDS swizzle: column c's 4-client group g lives at 16-byte slot (g ^ swz(c)) of its column.
// swz is a bijection of the 16 columns a ds_read_b128 lane group reads (reads conflict-free,
// 2-way on bf16 C=32) and spreads one wave-instruction's transposed ds_write_b32 over the
// banks (2-way, free on ds_write_b32); checked by tools/stripe_lds_banks.py.
template <int VPL, int R4>
__host__ __device__ constexpr int swz_h(int m) {  // m's bits into the positions (c/VPL)*R4 leaves free
  int h = 0, j = 0;
  for (int b = 0; b < 4; ++b) {
    if (b >= ilog2c(R4) && b < ilog2c(R4) + ilog2c(16 / VPL)) continue;
    h |= ((m >> j) & 1) << b;
    ++j;
  }
  return h;
}
template <int VPL, int R4>
__device__ __forceinline__ int stripe_swz(int c) {
  return (((c / VPL) * R4) ^ swz_h<VPL, R4>(c % VPL)) & 15;
}

// 32-bit patterns <-> fold values. (A bit_cast builtin applied to an ext_vector element,
// v[e], compiled to element 0 for every e with this toolchain: go through a scalar.)
template <class T>
__device__ __forceinline__ T from_bits(unsigned u) {
  if constexpr (std::is_same<T, float>::value) return __uint_as_float(u);
  else return (T)u;
}
template <class T>
__device__ __forceinline__ unsigned to_bits(T v) {
  if constexpr (std::is_same<T, float>::value) return __float_as_uint(v);
  else return (unsigned)v;
}

template <int IN, class ACC, int OUT, int C, bool NT, int D>
__global__ __launch_bounds__(kThreads) void k_dense_stripe(const uint8_t* __restrict__ x, int64_t ld_bytes,
                                                           int64_t K, int64_t P,
                                                           const typename ACC::T* __restrict__ w, float scale,
                                                           int do_scale, int accumulate, uint8_t* __restrict__ out) {
  using Sh = StripeShape<Elem<IN>::B, C>;
  using T = typename ACC::T;
  using Raw = typename Unit<IN, vec_width<IN>()>::Raw;
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B, VPL = Sh::VPL, TT = Sh::T, NI = Sh::NI, RPI = Sh::RPI,
                LPR = Sh::LPR, R4 = Sh::R4;
  __shared__ __attribute__((aligned(16))) unsigned tile[2][C * TT];
  __shared__ __attribute__((aligned(16))) T wts[3][TT];
  const int64_t nstripes = gridDim.x;
  const int64_t b = blockIdx.x;
  // XCD-contiguous stripes: blocks go to XCDs round-robin (b % 8), so block b takes stripe
  // (b % 8) * (n / 8) + b / 8 and each XCD's L2 sees a contiguous run (speed only)
  const int64_t stripe = (nstripes % 8 == 0) ? (b % 8) * (nstripes / 8) + b / 8 : b;
  const int64_t c0 = stripe * C;
  const int64_t ntiles = (K + TT - 1) / TT;
  // wave-uniform in SGPRs: the loaders' row offsets are buffer soffsets (a VGPR soffset
  // would turn every load into a waterfall loop)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  T identity;
  if constexpr (ACC::DT == FJAGG_I32) identity = 0;
  else identity = -0.0f;

  if (wave == 0) {
    // ------------------------------------------------------------ fold wave
    __builtin_amdgcn_s_setprio(3);
    const int cl = lane % C;  // lanes >= C shadow column lane % C (same address: broadcast, never stored)
    const int fsw = stripe_swz<VPL, R4>(cl);
    const int64_t ncols = P - c0 < C ? P - c0 : C;
    T acc = identity;
    if (accumulate && lane < ncols) {
      unsigned ob[1];
      load_out_unit<OUT, 1>(out + (c0 + lane) * OB, ob);
      acc = init_from<OUT, ACC>(ob[0]);
    }
    auto add4 = [&](u32x4 v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned u = v[e];
        acc = ACC::add(acc, from_bits<T>(u));
      }
    };
    __syncthreads();  // weights of tiles 0, 1 staged
    __syncthreads();  // tile 0 in buffer 0
    const int64_t nsteps = (ntiles + D - 1) / D * D;  // the loaders' padded step count
    for (int64_t s = 0; s < nsteps; ++s) {
      if (s >= ntiles) {
        __syncthreads();
        continue;
      }
      const u32x4* p = reinterpret_cast<const u32x4*>(&tile[s & 1][cl * TT]);
      // two batches of 8 groups in flight: the reads of one batch land while the other's adds run
      u32x4 va[8], vb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) va[u] = p[u ^ fsw];
      // (scheduling barriers keep each batch's 8 reads issued ahead of the other batch's
      // 32 adds; left alone the scheduler pulls every read next to its use and the serial
      // add chain waits out the LDS latency once per group)
      for (int g = 0; g < TT / 4; g += 16) {
#pragma unroll
        for (int u = 0; u < 8; ++u) vb[u] = p[(g + 8 + u) ^ fsw];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 8; ++u) add4(va[u]);
        __builtin_amdgcn_sched_barrier(0);
        if (g + 16 < TT / 4) {
#pragma unroll
          for (int u = 0; u < 8; ++u) va[u] = p[(g + 16 + u) ^ fsw];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 8; ++u) add4(vb[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
    }
    if (lane < ncols) {
      const unsigned ob[1] = {finish<OUT, ACC>(acc, do_scale != 0, scale)};
      store_unit<OUT, 1>(out + (c0 + lane) * OB, ob);
    }
    return;
  }

  // -------------------------------------------------------------- loader waves
  const int l = wave - 1;
  const int r = lane / LPR, q = lane % LPR;
  const uint32_t voff = (uint32_t)(r * ld_bytes + q * 16);
  // bytes of a tile's rows from c0: (rows - 1) full rows + the last row to P, rounded up to
  // 16 B (within the last row's 16-byte granule: no page can be crossed)
  const int64_t last_row_bytes = ((P - c0) * IB + 15) / 16 * 16;
  const uint8_t* xs = x + c0 * IB;
  const int wl = l * 64 + lane;  // this lane stages weights [4 wl, 4 wl + 4) of each tile
  const bool wlane = 4 * wl < TT;
  Raw d[D][NI];
  unsigned wr[D][4];
  // Loads are issued unconditionally (tiles past the last, and weight lanes past the tile,
  // read through descriptors clamped to the valid bytes: zeros, never a fault), so every
  // path through a step has the same loads in flight and the compiler's s_waitcnt counts
  // stay exact; a conditional issue made it wait for every outstanding tile.
  auto issue = [&](int64_t t, Raw(&dd)[NI], unsigned(&ww)[4]) {
    const int64_t k0 = t * TT;
    const int64_t rows = K - k0 < TT ? K - k0 : TT;
    const int64_t wbytes = (K - k0) * 4;
    const auto wrs = row_rsrc(reinterpret_cast<const uint8_t*>(w) + (rows > 0 ? k0 * 4 : 0),
                              rows > 0 ? row_range(wbytes) : 0u);
#pragma unroll
    for (int e = 0; e < 4; ++e) ww[e] = __builtin_amdgcn_raw_buffer_load_b32(wrs, (4 * wl + e) * 4, 0, 0);
    const auto rs = row_rsrc(xs + (rows > 0 ? k0 * ld_bytes : 0),
                             rows > 0 ? row_range((rows - 1) * ld_bytes + last_row_bytes) : 0u);
    constexpr int aux = NT ? 2 : 0;
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const uint32_t soff = (uint32_t)((int64_t)((l * NI + n) * RPI) * ld_bytes);
      dd[n] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, aux);
    }
  };
  auto stage_w = [&](int64_t t, const unsigned(&ww)[4]) {  // weights of tile t -> ring slot t % 3
    if (wlane) {
      T* dst = &wts[t % 3][4 * wl];
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = ACC::weight(from_bits<T>(ww[e]));
    }
  };
  // per-lane parts of the transposed address: column c = q*VPL + v, client group G of the
  // instruction (compile-time high part + r/4): slot (G ^ swz(c)) of column c
  int mv[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) mv[v] = (r >> 2) ^ stripe_swz<VPL, R4>(q * VPL + v);
  const int lbase = q * VPL * TT + (r & 3);
  auto put_t = [&](auto last_tag, int64_t t, const Raw(&dd)[NI]) {  // products of tile t -> buffer t & 1
    constexpr bool LAST = decltype(last_tag)::value;
    const int64_t k0 = t * TT;
    unsigned* buf = tile[t & 1];
    const T* wt = wts[t % 3];
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const int i = l * NI + n;
      const int rr = i * RPI + r;  // row within the tile
      const T wk = wt[rr];
      T v[VPL];
      decode<IN, ACC, vec_width<IN>()>(dd[n], v);
      const int ghi = (i * R4) & ~15, glo = (i * R4) & 15;
      bool pad = false;
      if constexpr (LAST) pad = k0 + rr >= K;
#pragma unroll
      for (int e = 0; e < VPL; ++e) {
        T prod = ACC::mul(v[e], wk);
        if constexpr (LAST) prod = pad ? identity : prod;
        buf[lbase + e * TT + 4 * (ghi + (glo ^ mv[e]))] = to_bits(prod);
      }
    }
  };
  auto put = [&](int64_t t, const Raw(&dd)[NI]) {
    if (t * TT + TT > K) put_t(std::true_type(), t, dd);
    else put_t(std::false_type(), t, dd);
  };
  // prologue: tiles 0 .. D-1 in flight; weights of tiles 0, 1 staged; tile 0 to buffer 0
#pragma unroll
  for (int j = 0; j < D; ++j) issue(j, d[j], wr[j]);
  stage_w(0, wr[0]);
  if (ntiles > 1) stage_w(1, wr[1]);
  __syncthreads();
  put(0, d[0]);
  issue(D, d[0], wr[0]);
  __syncthreads();
  // step s: stage weights of tile s+2, products of tile s+1 (register set (s+1) % D), issue
  // tile s+1+D into the freed set; wave 0 folds tile s meanwhile
  // (steps run in whole groups of D, padded past the last tile: no early exit, so every
  // path issues the same loads; the fold wave waits at the padding steps' barriers too)
  for (int64_t s0 = 0; s0 < ntiles; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int64_t s = s0 + j;
      const int nx = (j + 1) % D, n2 = (j + 2) % D;
      if (s + 2 < ntiles) stage_w(s + 2, wr[n2]);
      if (s + 1 < ntiles) put(s + 1, d[nx]);
      issue(s + 1 + D, d[nx], wr[nx]);
      __syncthreads();
    }
  }
}

// k_dense_stripe: variant 19 = automatic stripe width, 20 / 21 / 22 = C 64 / 32 / 16.
template <int IN, class ACC, int OUT, int C>
int launch_stripe_c(const uint8_t* x, int64_t ld_bytes, int64_t K, int64_t P, const void* w, float scale,
                    uint8_t* y, int flags, hipStream_t s) {
  constexpr int D = 3;
  const dim3 grid((unsigned)((P + C - 1) / C));
  const auto* wt = reinterpret_cast<const typename ACC::T*>(w);
  const int dsc = (flags & FJAGG_SCALE) ? 1 : 0, acm = (flags & FJAGG_ACCUMULATE) ? 1 : 0;
  if (flags & FJAGG_NONTEMPORAL)
    hipLaunchKernelGGL((k_dense_stripe<IN, ACC, OUT, C, true, D>), grid, dim3(kThreads), 0, s, x, ld_bytes, K, P,
                       wt, scale, dsc, acm, y);
  else
    hipLaunchKernelGGL((k_dense_stripe<IN, ACC, OUT, C, false, D>), grid, dim3(kThreads), 0, s, x, ld_bytes, K,
                       P, wt, scale, dsc, acm, y);
  return check_launch("k_dense_stripe");
}

// Stripe width: the widest of 64 / 32 / 16 columns that still gives every CU a stripe
// (wider stripes read longer row segments), else 16.
int stripe_cols(int variant, int64_t P) {
  if (variant == 20) return 64;
  if (variant == 21) return 32;
  if (variant == 22) return 16;
  const int64_t cus = cu_count();
  if ((P + 63) / 64 >= cus) return 64;
  if ((P + 31) / 32 >= cus) return 32;
  return 16;
}

}  // namespace

// Shapes k_dense_stripe takes: 16-byte aligned rows and slab, 4-byte aligned weights, and
// a tile's rows addressable with 32-bit buffer offsets.
__attribute__((visibility("hidden"))) bool fjagg_stripe_ok(const uint8_t* x, int64_t ld_bytes, int64_t P,
                                                            const void* w, int ib) {
  return (reinterpret_cast<uintptr_t>(x) % 16 == 0) && ld_bytes % 16 == 0 &&
         (reinterpret_cast<uintptr_t>(w) % 4 == 0) && P * ib <= ld_bytes &&
         (int64_t)768 * ld_bytes < (1ll << 31);
}

namespace {
template <int IN, class ACC, int OUT>
int launch_stripe_t(int variant, const uint8_t* x, int64_t ld_bytes, int64_t K, int64_t P, const void* w,
                    float scale, uint8_t* y, int flags, hipStream_t s) {
  switch (stripe_cols(variant, P)) {
    case 64: return launch_stripe_c<IN, ACC, OUT, 64>(x, ld_bytes, K, P, w, scale, y, flags, s);
    case 32: return launch_stripe_c<IN, ACC, OUT, 32>(x, ld_bytes, K, P, w, scale, y, flags, s);
    default: return launch_stripe_c<IN, ACC, OUT, 16>(x, ld_bytes, K, P, w, scale, y, flags, s);
  }
}

}  // namespace

__attribute__((visibility("hidden"))) int fjagg_launch_stripe(int variant, int in, int acc, int out,
                                                              const uint8_t* x, int64_t ld_bytes, int64_t K,
                                                              int64_t P, const void* w, float scale, uint8_t* y,
                                                              int flags, hipStream_t s) {
  if (K < 1 || P < 1) return FJAGG_OK;
#define FJ_CASE(I, A, O, ACCT) \
  if (in == I && acc == A && out == O)   \
    return launch_stripe_t<I, ACCT, O>(variant, x, ld_bytes, K, P, w, scale, y, flags, s);
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
  FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
  return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination (%d,%d,%d)", in, acc, out);
}

