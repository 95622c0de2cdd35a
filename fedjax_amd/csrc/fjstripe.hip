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

// Work of one workgroup: a list of stripes, walked as ONE pipeline of (stripe, tile) steps
// so the loads of the next stripe are in flight while the fold wave finishes this one. The
// grid is one workgroup per CU (the LDS tile buffers allow no more); with S stripes and G
// workgroups, workgroup b on XCD x = b % 8 takes stripes of XCD x's contiguous eighth,
// round-robin over that XCD's workgroups, so the stripes an XCD streams at once are
// neighbours (they share L2 lines). Speed only: any mapping gives the same results.
struct StripeList {
  int64_t first, step, count;  // stripes first, first + step, ... (count of them)
  __device__ __forceinline__ int64_t at(int64_t j) const { return first + j * step; }
};
__device__ __forceinline__ StripeList stripes_of(int64_t b, int64_t G, int64_t S) {
  if (G % 8 == 0 && S % 8 == 0 && S >= G) {
    const int64_t x = b % 8, i = b / 8, per_x = S / 8, wg_x = G / 8;
    return {x * per_x + i, wg_x, (per_x - i + wg_x - 1) / wg_x};
  }
  return {b, G, (S - b + G - 1) / G};
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
  const int64_t S = (P + C - 1) / C;
  const StripeList sl = stripes_of(blockIdx.x, gridDim.x, S);
  const int64_t ntiles = (K + TT - 1) / TT;      // tiles per stripe
  const int64_t nsteps_all = sl.count * ntiles;  // pipeline steps of this workgroup
  // wave-uniform in SGPRs: the loaders' row offsets are buffer soffsets (a VGPR soffset
  // would turn every load into a waterfall loop)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  T identity;
  if constexpr (ACC::DT == FJAGG_I32) identity = 0;
  else identity = -0.0f;
  const int64_t nsteps = (nsteps_all + D - 1) / D * D;  // the loaders' padded step count

  if (wave == 0) {
    // ------------------------------------------------------------ fold wave
    __builtin_amdgcn_s_setprio(3);
    const int cl = lane % C;  // lanes >= C shadow column lane % C (same address: broadcast, never stored)
    const int fsw = stripe_swz<VPL, R4>(cl);
    T acc = identity;
    auto start = [&](int64_t js) {  // fold state of stripe js's column: -0 (or the output)
      acc = identity;
      const int64_t c0 = sl.at(js) * C;
      if (accumulate && lane < (P - c0 < C ? P - c0 : C)) {
        unsigned ob[1];
        load_out_unit<OUT, 1>(out + (c0 + lane) * OB, ob);
        acc = init_from<OUT, ACC>(ob[0]);
      }
    };
    auto add4 = [&](u32x4 v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned u = v[e];
        acc = ACC::add(acc, from_bits<T>(u));
      }
    };
    if (sl.count > 0) start(0);
    __syncthreads();  // weights of tiles 0, 1 staged
    __syncthreads();  // tile 0 in buffer 0
    int64_t js = 0, tt = 0;  // stripe and tile of step s
    for (int64_t s = 0; s < nsteps; ++s) {
      if (s >= nsteps_all) {
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
      if (++tt == ntiles) {  // the stripe's last tile: its column is done
        const int64_t c0 = sl.at(js) * C;
        if (lane < (P - c0 < C ? P - c0 : C)) {
          const unsigned ob[1] = {finish<OUT, ACC>(acc, do_scale != 0, scale)};
          store_unit<OUT, 1>(out + (c0 + lane) * OB, ob);
        }
        tt = 0;
        if (++js < sl.count) start(js);
      }
      __syncthreads();
    }
    return;
  }

  // -------------------------------------------------------------- loader waves
  const int l = wave - 1;
  const int r = lane / LPR, q = lane % LPR;
  const uint32_t voff = (uint32_t)(r * ld_bytes + q * 16);
  const int wl = l * 64 + lane;  // this lane stages weights [4 wl, 4 wl + 4) of each tile
  const bool wlane = 4 * wl < TT;
  Raw d[D][NI];
  unsigned wr[D][4];
  // Loads are issued unconditionally (steps past the last, and weight lanes past the tile,
  // read through descriptors clamped to the valid bytes: zeros, never a fault), so every
  // path through a step has the same loads in flight and the compiler's s_waitcnt counts
  // stay exact; a conditional issue made it wait for every outstanding tile.
  // (stripe, tile) of a pipeline step, advanced one step at a time (no 64-bit divisions)
  struct Cursor {
    int64_t js, tt;
    __device__ __forceinline__ void next(int64_t ntiles) {
      if (++tt == ntiles) {
        tt = 0;
        ++js;
      }
    }
  };
  auto issue = [&](const Cursor& c, Raw(&dd)[NI], unsigned(&ww)[4]) {  // the loads of step (c.js, c.tt)
    const bool live = c.js < sl.count;
    const int64_t js = live ? c.js : 0, tt = live ? c.tt : 0;
    const int64_t c0 = sl.at(js) * C, k0 = tt * TT;
    const int64_t rows = live ? (K - k0 < TT ? K - k0 : TT) : 0;
    const auto wrs = row_rsrc(reinterpret_cast<const uint8_t*>(w) + k0 * 4, rows > 0 ? row_range((K - k0) * 4) : 0u);
#pragma unroll
    for (int e = 0; e < 4; ++e) ww[e] = __builtin_amdgcn_raw_buffer_load_b32(wrs, (4 * wl + e) * 4, 0, 0);
    // bytes of the tile's rows from c0: (rows - 1) full rows + the last row to P, rounded
    // up to 16 B (within the last row's 16-byte granule: no page can be crossed)
    const int64_t last_row_bytes = ((P - c0) * IB + 15) / 16 * 16;
    const auto rs = row_rsrc(x + c0 * IB + k0 * ld_bytes,
                             rows > 0 ? row_range((rows - 1) * ld_bytes + last_row_bytes) : 0u);
    constexpr int aux = NT ? 2 : 0;
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const uint32_t soff = (uint32_t)((int64_t)((l * NI + n) * RPI) * ld_bytes);
      dd[n] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, aux);
    }
  };
  auto stage_w = [&](int64_t g, const unsigned(&ww)[4]) {  // weights of step g -> ring slot g % 3
    if (wlane) {
      T* dst = &wts[(unsigned)g % 3u][4 * wl];
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
  auto put_t = [&](auto last_tag, int64_t g, int64_t k0, const Raw(&dd)[NI]) {  // step g's products -> buffer g & 1
    constexpr bool LAST = decltype(last_tag)::value;
    unsigned* buf = tile[(unsigned)g & 1u];
    const T* wt = wts[(unsigned)g % 3u];
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
  auto put = [&](int64_t g, const Cursor& c, const Raw(&dd)[NI]) {
    const int64_t k0 = c.tt * TT;
    if (k0 + TT > K) put_t(std::true_type(), g, k0, dd);  // rows >= K: the identity
    else put_t(std::false_type(), g, k0, dd);
  };
  // prologue: steps 0 .. D-1 in flight; weights of steps 0, 1 staged; step 0 to buffer 0
  Cursor ic{0, 0};  // the next step to issue
#pragma unroll
  for (int j = 0; j < D; ++j) {
    issue(ic, d[j], wr[j]);
    ic.next(ntiles);
  }
  stage_w(0, wr[0]);
  if (nsteps_all > 1) stage_w(1, wr[1]);
  __syncthreads();
  Cursor pc{0, 0};  // the next step to put
  if (nsteps_all > 0) put(0, pc, d[0]);
  pc.next(ntiles);
  issue(ic, d[0], wr[0]);
  ic.next(ntiles);
  __syncthreads();
  // step s: stage weights of step s+2, products of step s+1 (register set (s+1) % D), issue
  // step s+1+D into the freed set; wave 0 folds step s meanwhile. (Steps run in whole
  // groups of D, padded past the last: no early exit, so every path issues the same loads;
  // the fold wave waits at the padding steps' barriers too.)
  for (int64_t s0 = 0; s0 < nsteps; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int64_t s = s0 + j;
      const int nx = (j + 1) % D, n2 = (j + 2) % D;
      if (s + 2 < nsteps_all) stage_w(s + 2, wr[n2]);
      if (s + 1 < nsteps_all) put(s + 1, pc, d[nx]);
      pc.next(ntiles);
      issue(ic, d[nx], wr[nx]);
      ic.next(ntiles);
      __syncthreads();
    }
  }
}

// The pytree form (fjagg_wsum_ptrs with FJAGG_NARROW | FJAGG_VARIANT(20..22)): the stripes
// are the plan's blocks (leaf, [e0, e1) of at most C elements, fjagg_ptrs_plan_leaves) and
// client k's row of a stripe is in_ptrs[k*L + leaf] + e0. Those row pointers cannot be
// formed from a stride, so the fold wave — which issues no other vector-memory loads, so
// waiting for these never stalls the loaders' pipeline — stages each step's TT row
// pointers in an LDS ring, D+2 steps ahead of the loaders that use them. Loads are 16-byte
// flat loads from every lane's own row pointer; a lane whose 16 bytes start past the
// stripe's last element reads the stripe's first granule instead (never stored), so no
// load leaves the 16-byte granules of the leaf (all pointers are 16-byte aligned: the host
// checks). Everything else is k_dense_stripe's: transposed products, the -0.0 identity for
// rows >= K, one pipeline of (stripe, tile) steps per workgroup.
template <int IN, class ACC, int OUT, int C, bool NT, int D>
__global__ __launch_bounds__(kThreads) void k_ptrs_stripe(const int64_t* __restrict__ img, int L, int64_t K,
                                                          int64_t nblk, const typename ACC::T* __restrict__ w,
                                                          float scale, int do_scale, int accumulate) {
  using Sh = StripeShape<Elem<IN>::B, C>;
  using T = typename ACC::T;
  using Raw = typename Unit<IN, vec_width<IN>()>::Raw;
  constexpr int IB = Elem<IN>::B, OB = Elem<OUT>::B, VPL = Sh::VPL, TT = Sh::T, NI = Sh::NI, RPI = Sh::RPI,
                LPR = Sh::LPR, R4 = Sh::R4, PR = D + 2;
  __shared__ __attribute__((aligned(16))) unsigned tile[2][C * TT];
  __shared__ __attribute__((aligned(16))) T wts[3][TT];
  __shared__ __attribute__((aligned(16))) unsigned long long rowp[PR][TT];
  const int64_t* in_ptrs = img;
  const int64_t* out_ptrs = img + K * L;
  const int64_t* blocks = out_ptrs + 2 * (int64_t)L;  // after out_ptrs[L] and leaf_n[L]
  const StripeList sl = stripes_of(blockIdx.x, gridDim.x, nblk);
  const int64_t ntiles = (K + TT - 1) / TT;
  const int64_t nsteps_all = sl.count * ntiles;
  const int64_t nsteps = (nsteps_all + D - 1) / D * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  T identity;
  if constexpr (ACC::DT == FJAGG_I32) identity = 0;
  else identity = -0.0f;
  struct Blk {
    int leaf;
    int64_t e0, n;  // first element, elements (<= C)
  };
  auto blk = [&](int64_t js) {  // stripe js of this workgroup
    const int64_t j = sl.at(js < sl.count ? js : 0);
    const int64_t be = blocks[2 * j];
    const int64_t e0 = be & ((1ll << 40) - 1);
    return Blk{(int)((be >> 40) & 0x3fffff), e0, blocks[2 * j + 1] - e0};
  };

  if (wave == 0) {
    // ------------------------------------------------------------ fold wave
    __builtin_amdgcn_s_setprio(3);
    constexpr int PP = TT / 64;  // row pointers per lane per step
    unsigned long long pr[PP];
    int64_t fjs = 0, ftt = 0;  // the step fetch() reads next (steps are fetched in order)
    auto fetch = [&](int64_t g) {  // row pointers of step g -> registers (rows >= K: row K-1)
      const bool live = g < nsteps_all;
      const int64_t js = live ? fjs : 0, tt = live ? ftt : 0;
      if (++ftt == ntiles) {
        ftt = 0;
        ++fjs;
      }
      const Blk bb = blk(js);
#pragma unroll
      for (int m = 0; m < PP; ++m) {
        int64_t k = tt * TT + lane + 64 * m;
        k = k < K ? k : K - 1;
        pr[m] = (unsigned long long)in_ptrs[k * L + bb.leaf] + (unsigned long long)(bb.e0 * IB);
      }
    };
    auto commit = [&](int64_t g) {
#pragma unroll
      for (int m = 0; m < PP; ++m) rowp[(unsigned)g % (unsigned)PR][lane + 64 * m] = pr[m];
    };
    for (int64_t g = 0; g < PR; ++g) {  // steps 0 .. D+1: everything the prologue and step 0 issue
      fetch(g);
      commit(g);
    }
    __syncthreads();  // row pointers of steps 0 .. D+1 staged
    fetch(PR);
    const int cl = lane % C;
    const int fsw = stripe_swz<VPL, R4>(cl);
    T acc = identity;
    auto start = [&](int64_t js) {
      acc = identity;
      const Blk bb = blk(js);
      if (accumulate && lane < bb.n) {
        unsigned ob[1];
        load_out_unit<OUT, 1>(reinterpret_cast<const uint8_t*>(out_ptrs[bb.leaf]) + (bb.e0 + lane) * OB, ob);
        acc = init_from<OUT, ACC>(ob[0]);
      }
    };
    auto add4 = [&](u32x4 v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned u = v[e];
        acc = ACC::add(acc, from_bits<T>(u));
      }
    };
    if (sl.count > 0) start(0);
    __syncthreads();  // weights of steps 0, 1 staged
    __syncthreads();  // step 0 in buffer 0
    int64_t js = 0, tt = 0;
    for (int64_t s = 0; s < nsteps; ++s) {
      commit(s + PR);  // row pointers of step s+D+2 (fetched one step ago), then the next ones
      fetch(s + PR + 1);
      if (s < nsteps_all) {
        const u32x4* p = reinterpret_cast<const u32x4*>(&tile[s & 1][cl * TT]);
        u32x4 va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) va[u] = p[u ^ fsw];
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
        if (++tt == ntiles) {
          const Blk bb = blk(js);
          if (lane < bb.n) {
            const unsigned ob[1] = {finish<OUT, ACC>(acc, do_scale != 0, scale)};
            store_unit<OUT, 1>(reinterpret_cast<uint8_t*>(out_ptrs[bb.leaf]) + (bb.e0 + lane) * OB, ob);
          }
          tt = 0;
          if (++js < sl.count) start(js);
        }
      }
      __syncthreads();
    }
    return;
  }

  // -------------------------------------------------------------- loader waves
  const int l = wave - 1;
  const int r = lane / LPR, q = lane % LPR;
  const int wl = l * 64 + lane;
  const bool wlane = 4 * wl < TT;
  Raw d[D][NI];
  unsigned wr[D][4];
  __syncthreads();  // the row pointers of steps 0 .. D+1
  struct Cursor {
    int64_t js, tt;
    __device__ __forceinline__ void next(int64_t ntiles) {
      if (++tt == ntiles) {
        tt = 0;
        ++js;
      }
    }
  };
  auto issue = [&](int64_t g, const Cursor& c, Raw(&dd)[NI], unsigned(&ww)[4]) {
    const bool live = c.js < sl.count;
    const int64_t js = live ? c.js : 0, tt = live ? c.tt : 0;
    const int64_t k0 = tt * TT;
    const int64_t rows = live ? (K - k0 < TT ? K - k0 : TT) : 0;
    const auto wrs = row_rsrc(reinterpret_cast<const uint8_t*>(w) + k0 * 4, rows > 0 ? row_range((K - k0) * 4) : 0u);
#pragma unroll
    for (int e = 0; e < 4; ++e) ww[e] = __builtin_amdgcn_raw_buffer_load_b32(wrs, (4 * wl + e) * 4, 0, 0);
    const int64_t ncols = blk(js).n;
    const uint32_t qoff = q * VPL < ncols ? (uint32_t)(q * 16) : 0u;
    const unsigned long long* rp = rowp[(unsigned)g % (unsigned)PR];
    unsigned long long base[NI];
#pragma unroll
    for (int n = 0; n < NI; ++n) base[n] = rp[(l * NI + n) * RPI + r];
#pragma unroll
    for (int n = 0; n < NI; ++n)
      dd[n] = load16_global<NT>(reinterpret_cast<const uint8_t*>(base[n] + qoff));
  };
  auto stage_w = [&](int64_t g, const unsigned(&ww)[4]) {
    if (wlane) {
      T* dst = &wts[(unsigned)g % 3u][4 * wl];
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = ACC::weight(from_bits<T>(ww[e]));
    }
  };
  int mv[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) mv[v] = (r >> 2) ^ stripe_swz<VPL, R4>(q * VPL + v);
  const int lbase = q * VPL * TT + (r & 3);
  auto put_t = [&](auto last_tag, int64_t g, int64_t k0, const Raw(&dd)[NI]) {
    constexpr bool LAST = decltype(last_tag)::value;
    unsigned* buf = tile[(unsigned)g & 1u];
    const T* wt = wts[(unsigned)g % 3u];
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const int i = l * NI + n;
      const int rr = i * RPI + r;
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
  auto put = [&](int64_t g, const Cursor& c, const Raw(&dd)[NI]) {
    const int64_t k0 = c.tt * TT;
    if (k0 + TT > K) put_t(std::true_type(), g, k0, dd);
    else put_t(std::false_type(), g, k0, dd);
  };
  Cursor ic{0, 0}, pc{0, 0};
#pragma unroll
  for (int j = 0; j < D; ++j) {
    issue(j, ic, d[j], wr[j]);
    ic.next(ntiles);
  }
  stage_w(0, wr[0]);
  if (nsteps_all > 1) stage_w(1, wr[1]);
  __syncthreads();
  if (nsteps_all > 0) put(0, pc, d[0]);
  pc.next(ntiles);
  issue(D, ic, d[0], wr[0]);
  ic.next(ntiles);
  __syncthreads();
  for (int64_t s0 = 0; s0 < nsteps; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int64_t s = s0 + j;
      const int nx = (j + 1) % D, n2 = (j + 2) % D;
      if (s + 2 < nsteps_all) stage_w(s + 2, wr[n2]);
      if (s + 1 < nsteps_all) put(s + 1, pc, d[nx]);
      pc.next(ntiles);
      issue(s + 1 + D, ic, d[nx], wr[nx]);
      ic.next(ntiles);
      __syncthreads();
    }
  }
}

// k_dense_stripe: variant 19 = automatic stripe width, 20 / 21 / 22 = C 64 / 32 / 16.
template <int IN, class ACC, int OUT, int C>
int launch_stripe_c(const uint8_t* x, int64_t ld_bytes, int64_t K, int64_t P, const void* w, float scale,
                    uint8_t* y, int flags, hipStream_t s) {
  constexpr int D = 3;
  // persistent: at most one workgroup per CU (the tile buffers take ~105 KiB of LDS), each
  // walking its list of stripes as one pipeline
  const int64_t stripes = (P + C - 1) / C, cus = cu_count();
  const dim3 grid((unsigned)(stripes < cus ? stripes : cus));
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

namespace {
template <int IN, class ACC, int OUT, int C>
int launch_ptrs_stripe_c(bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w, float scale,
                         int dsc, int acm, hipStream_t s) {
  constexpr int D = 3;
  const int64_t cus = cu_count();
  const dim3 grid((unsigned)(nblk < cus ? nblk : cus));
  const auto* wt = reinterpret_cast<const typename ACC::T*>(w);
  if (nt)
    hipLaunchKernelGGL((k_ptrs_stripe<IN, ACC, OUT, C, true, D>), grid, dim3(kThreads), 0, s, img, L, K, nblk, wt,
                       scale, dsc, acm);
  else
    hipLaunchKernelGGL((k_ptrs_stripe<IN, ACC, OUT, C, false, D>), grid, dim3(kThreads), 0, s, img, L, K, nblk, wt,
                       scale, dsc, acm);
  return check_launch("k_ptrs_stripe");
}
template <int IN, class ACC, int OUT>
int launch_ptrs_stripe_t(int C, bool nt, const int64_t* img, int L, int64_t K, int64_t nblk, const void* w,
                         float scale, int dsc, int acm, hipStream_t s) {
  switch (C) {
    case 64: return launch_ptrs_stripe_c<IN, ACC, OUT, 64>(nt, img, L, K, nblk, w, scale, dsc, acm, s);
    case 32: return launch_ptrs_stripe_c<IN, ACC, OUT, 32>(nt, img, L, K, nblk, w, scale, dsc, acm, s);
    default: return launch_ptrs_stripe_c<IN, ACC, OUT, 16>(nt, img, L, K, nblk, w, scale, dsc, acm, s);
  }
}
}  // namespace

__attribute__((visibility("hidden"))) int fjagg_launch_ptrs_stripe(int C, int in, int acc, int out, bool nt,
                                                                   const int64_t* img, int L, int64_t K,
                                                                   int64_t nblk, const void* w, float scale,
                                                                   int dsc, int acm, hipStream_t s) {
  if (K < 1 || nblk < 1) return FJAGG_OK;
#define FJ_CASE(I, A, O, ACCT) \
  if (in == I && acc == A && out == O)   \
    return launch_ptrs_stripe_t<I, ACCT, O>(C, nt, img, L, K, nblk, w, scale, dsc, acm, s);
  FJ_CASE(FJAGG_F32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_BF16, AccF)
  FJ_CASE(FJAGG_BF16, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_F32, FJAGG_F32, AccF)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_I32, AccI)
  FJ_CASE(FJAGG_I32, FJAGG_I32, FJAGG_F32, AccI)
  FJ_CASE(FJAGG_BF16, FJAGG_BF16, FJAGG_BF16, AccB)
#undef FJ_CASE
  return fail(FJAGG_EUNSUPPORTED, "unsupported dtype combination (%d,%d,%d)", in, acc, out);
}
