// rg_kernels.h — gfx950 kernels of the batched Rabia phase evaluator.
//
// Layout: bit-sliced planes (one bit per slot, 32 slots per word), so one VALU
// op evaluates a boolean over 32 slots. Each thread owns W consecutive words
// (W*32 slots) of every plane and loads them as one 16/8/4-B vector per plane:
// coalesced, read exactly once, no LDS staging needed (no reuse exists).
// Counts over the n replica lanes are bit-sliced ripple counters.
//
// REF mode needs, per VQ slot, the index of its StdRng draw = number of VQ slots
// before it in ascending slot order (engine.rs:567-611 consumes the engine's one
// RNG stream). That is an exclusive prefix sum across the launch, done in the
// same pass by a decoupled look-back over tiles in blockIdx order.
#pragma once

#include <type_traits>

#include "rg_common.h"

namespace rg {

// Plane addressing: word w of plane pl of a buffer lives at
//   (w >> tshift) * tile_stride + pl * pstride + (w & tmask)
// planar      : tshift 63, tmask ~0, tile_stride 0, pstride = stride
// slot-tiled T: tshift log2 T, tmask T-1, tile_stride = planes * T, pstride = T
// (the planes of one T-word slot tile are stored back to back).
struct Layout {
  uint32_t tshift;
  uint64_t tmask, tile_stride, pstride;
  RG_HD uint64_t base(uint64_t w) const { return (w >> tshift) * tile_stride + (w & tmask); }
};

struct StepParams {
  const uint32_t* votes;          // 4N+1 planes (layout lin)
  unsigned long long* stats;      // [n_tiles][kStatGranules] tagged granules
  uint32_t* out;                  // 8 planes (layout lout)
  unsigned long long* lookback;   // [n_tiles] {tag:32 | value:32} granules
  Record* rec;                    // ring of 2
  DevState* state;
  DevResult* result;              // ctx-internal, always written
  DevResult* result_user;         // optional copy
  Layout lin, lout;
  uint64_t n_slots;
  uint64_t n_words;
  uint64_t slot_base;
  uint64_t max_phase;
  uint64_t phase;
  uint64_t coin_stream;
  Key key;                        // REF: StdRng key; WMVC: coin key
  uint32_t q, fp1;
  int32_t self_lane;
  uint32_t seq;
  uint32_t n_tiles;
  uint32_t diag;                  // diagnostic build switches (0 in production):
                                  //  1 skip the look-back wait, 2 skip finish_tile, 4 stamps
  unsigned long long* dbg;        // [n_tiles][8] s_memrealtime stamps when diag & 4
  uint64_t in_bytes, out_bytes;   // the plane buffers' extents
  uint32_t* vq_rec;               // sharded REF: the window's record region (rg_common.h): chunk
  uint64_t vq_cap;                //   table [rec_tw words], then [vq_cap] draw records
  uint64_t rec_pitch;             //   words per window region (rg_record_window_words)
  uint32_t rec_tw;                //   chunk-table words
  // Sharded REF over n_win windows in one launch (grid.y = window; tiled kernel): window
  // w reads votes + w * win_in_pitch, writes out + w * win_out_pitch, its shard's slot
  // ids start at slot_base + w * win_id_stride, its record region at vq_rec + w * rec_pitch, its
  // row at result_user[w]; its look-back chain and statistics granules are its own
  // (lookback / stats + w * n_tiles tiles). n_win = 1: one window, as before.
  uint32_t n_win;
  uint64_t win_in_pitch, win_out_pitch, win_id_stride;
};

// finish_tile flavours
constexpr int kFinRef = 0, kFinWmvc = 1, kFinShard = 2;

__device__ __forceinline__ void stamp(const StepParams& p, uint32_t tile, int k, int tid) {
  if ((p.diag & 4u) && tid == 0) {
    p.dbg[(uint64_t)tile * 8 + k] = __builtin_amdgcn_s_memrealtime();
    // placement of the tile: XCC id (hwreg 20, gfx950) and HW_ID (hwreg 4: CU, SH, SE)
    if (k == 0) p.dbg[(uint64_t)tile * 8 + 6] = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    if (k == 0) p.dbg[(uint64_t)tile * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
}

constexpr int ctr_bits(int n) { return n < 2 ? 1 : n < 4 ? 2 : n < 8 ? 3 : n < 16 ? 4 : 5; }

// ---- bit-sliced counters --------------------------------------------------
template <int B>
struct Ctr {
  uint32_t b[B];
};

template <int B>
RG_HD void ctr_zero(Ctr<B>& c) {
#pragma unroll
  for (int i = 0; i < B; i++) c.b[i] = 0;
}

template <int B>
RG_HD void ctr_add(Ctr<B>& c, uint32_t m) {
#pragma unroll
  for (int i = 0; i < B; i++) {
    uint32_t t = c.b[i] & m;
    c.b[i] ^= m;
    m = t;
  }
}

// Per-slot mask of (count >= q) for a wave-uniform 1 <= q < 2^B: the carry out of
// count + (2^B - q), one majority per bit whose addend bit is a uniform 0 / ~0 (one
// v_bitop3 per bit on gfx950).
template <int B>
RG_HD uint32_t ctr_ge(const Ctr<B>& c, uint32_t q) {
  const uint32_t k = (1u << B) - q;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < B; i++) {
    const uint32_t kb = ((k >> i) & 1u) ? ~0u : 0u;
    cy = (c.b[i] & kb) | (cy & (c.b[i] | kb));
  }
  return cy;
}

// Bit-sliced population count of N masks (count of set bits per slot position) as a
// carry-save (Wallace) tree: full adders (xor3, majority: one v_bitop3 each on
// gfx950) over triples, then the weight-1 sums and weight-2 carries counted the same
// way and added. n = 5: 6 operations (sequential ctr_add: ~17); n = 9: 14 (~45).
template <int N>
struct Csa {
  static RG_HD void count(const uint32_t* m, uint32_t* out) {
    if constexpr (N == 1) {
      out[0] = m[0];
    } else if constexpr (N == 2) {
      out[0] = m[0] ^ m[1];
      out[1] = m[0] & m[1];
    } else if constexpr (N == 3) {
      out[0] = m[0] ^ m[1] ^ m[2];
      out[1] = (m[0] & m[1]) | (m[2] & (m[0] ^ m[1]));
    } else if constexpr (N >= 4) {
      constexpr int G = N / 3, R = N % 3, S = G + R;
      uint32_t sums[S], carries[G];
#pragma unroll
      for (int g = 0; g < G; g++) {
        const uint32_t a = m[3 * g], b = m[3 * g + 1], c = m[3 * g + 2];
        sums[g] = a ^ b ^ c;
        carries[g] = (a & b) | (c & (a ^ b));
      }
#pragma unroll
      for (int r = 0; r < R; r++) sums[G + r] = m[3 * G + r];
      constexpr int BS = ctr_bits(S), BC = ctr_bits(G), B = ctr_bits(N);
      uint32_t a[BS], b[BC];
      Csa<S>::count(sums, a);
      Csa<G>::count(carries, b);
      out[0] = a[0];  // a + 2b, ripple
      uint32_t k = 0;
#pragma unroll
      for (int i = 1; i < B; i++) {
        const uint32_t x = i < BS ? a[i] : 0u, y = i - 1 < BC ? b[i - 1] : 0u;
        out[i] = x ^ y ^ k;
        k = (x & y) | (k & (x ^ y));
      }
    }
  }
};
template <int N>
RG_HD Ctr<ctr_bits(N)> ctr_count(const uint32_t (&m)[N]) {
  Ctr<ctr_bits(N)> c;
  Csa<N>::count(m, c.b);
  return c;
}

template <int B>
RG_HD uint32_t ctr_nz(const Ctr<B>& c) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < B; i++) r |= c.b[i];
  return r;
}

template <int B>
RG_HD uint32_t ctr_at(const Ctr<B>& c, int bit) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < B; i++) v |= ((c.b[i] >> bit) & 1u) << i;
  return v;
}

// Per-slot masks of (a > b) and (a < b) for two bit-sliced counters.
template <int B>
RG_HD void ctr_cmp(const Ctr<B>& a, const Ctr<B>& b, uint32_t& gt, uint32_t& lt) {
  uint32_t eq = ~0u;
  gt = lt = 0;
#pragma unroll
  for (int i = B - 1; i >= 0; i--) {
    gt |= eq & a.b[i] & ~b.b[i];
    lt |= eq & ~a.b[i] & b.b[i];
    eq &= ~(a.b[i] ^ b.b[i]);
  }
}

// ---- vector plane access ----------------------------------------------------
// Vote planes are read exactly once: non-temporal loads (measured +5-15 % on
// this pattern, tools/probe_layout.py).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int W>
__device__ __forceinline__ void load_words(const uint32_t* p, uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (W == 2) {
    const u32x2 x = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    v[0] = x.x; v[1] = x.y;
  } else {
    v[0] = __builtin_nontemporal_load(p);
  }
}

// Output planes are written once and not read by this launch: non-temporal stores.
template <int W>
__device__ __forceinline__ void store_words_nt(uint32_t* p, const uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    u32x4 x;
    x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  } else if constexpr (W == 2) {
    u32x2 x;
    x.x = v[0]; x.y = v[1];
    __builtin_nontemporal_store(x, reinterpret_cast<u32x2*>(p));
  } else {
    __builtin_nontemporal_store(v[0], p);
  }
}

__device__ __forceinline__ uint32_t valid_mask(uint64_t w, uint64_t n_words, uint64_t n_slots) {
  if (w >= n_words) return 0u;
  if (w == n_words - 1 && (n_slots & 31u)) return (1u << (n_slots & 31u)) - 1u;
  return ~0u;
}

// Mask of local bits b with slot_base + 32w + b <= max_phase (max_phase 0 = no limit).
__device__ __forceinline__ uint32_t phase_limit_mask(uint64_t slot_base, uint64_t w,
                                                     uint64_t max_phase) {
  if (max_phase == 0) return ~0u;
  uint64_t first = slot_base + 32 * w;
  if (first > max_phase) return 0u;
  uint64_t lim = max_phase - first;
  return lim >= 31 ? ~0u : ((2u << lim) - 1u);
}

// ---- wave / block reductions -------------------------------------------------
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_max64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}
__device__ __forceinline__ unsigned long long wave_min64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
// Inclusive prefix within each 16-lane row: DPP row shifts (zero fill), no LDS
// round trip (a __shfl_up ladder is six ds_bpermute + lgkmcnt waits).
__device__ __forceinline__ uint32_t row_incl_scan32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v, int lane) {
  v = row_incl_scan32(v);
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
                 r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = lane >> 4;
  return v + (row >= 1 ? r0 : 0u) + (row >= 2 ? r1 : 0u) + (row >= 3 ? r2 : 0u);
}

__device__ __forceinline__ unsigned long long atomic_load_agent(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void atomic_store_agent(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only. __syncthreads() also drains every
// outstanding global load and store (its workgroup-scope release waits on
// vmcnt), which would serialise the tile's HBM traffic behind each barrier.
// Bounded spins: a wait that lasts longer than kSpinTicks of the constant 100 MHz
// s_memrealtime clock is a protocol fault, not a wait (the caller raises an error
// flag instead of hanging). Elapsed time, not an iteration count: other processes'
// kernels on the same GPU may legitimately delay a ticket holder for a while.
constexpr unsigned long long kSpinTicks = 400000000ull;  // 4 s
struct SpinBound {
  unsigned long long t0 = 0;
  __device__ __forceinline__ bool expired() {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (t0 == 0) {
      t0 = t | 1ull;
      return false;
    }
    return t - t0 > kSpinTicks;
  }
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- decoupled look-back (run by all 64 lanes of wave 0) ----------------------
// Granule = {tag:32 | value:32}, tag = seq<<1 | inclusive, written by ONE 8-B
// agent-scope store and read by agent-scope loads (MI355X_MICROARCH.md,
// visibility: "R2" granules need no separate flag or fence). seq changes every
// launch, so the array is never re-zeroed. Tiles are blockIdx.x: workgroups
// are dispatched in blockIdx order on each XCD, so the lowest unfinished tile is
// always resident and every wait terminates (ticket atomics on one address
// serialise at ~12 ns each: measured slower). The spin is still bounded; a
// timeout raises Record.error and the step reports RG_ESTATE.
__device__ __forceinline__ uint32_t lookback_exclusive(unsigned long long* status, uint32_t tile,
                                                       uint32_t seq, uint32_t agg, int lane,
                                                       unsigned long long* err) {
  const uint32_t tag_agg = seq << 1, tag_inc = (seq << 1) | 1u;
  if (tile == 0) {
    if (lane == 0) atomic_store_agent(status, ((unsigned long long)tag_inc << 32) | agg);
    return 0;
  }
  if (lane == 0) atomic_store_agent(status + tile, ((unsigned long long)tag_agg << 32) | agg);
  uint32_t excl = 0;
  int64_t pos = (int64_t)tile - 1;
  SpinBound spin;
  for (;;) {
    const int64_t pidx = pos - lane;
    unsigned long long g = pidx >= 0 ? atomic_load_agent(status + pidx)
                                     : ((unsigned long long)tag_inc << 32);
    const uint32_t tag = (uint32_t)(g >> 32);
    const bool ready = (tag >> 1) == seq;
    const bool incl = ready && (tag & 1u);
    const unsigned long long incl_mask = __ballot(incl);
    const unsigned long long notready = __ballot(!ready);
    const int first = incl_mask ? __builtin_ctzll(incl_mask) : 64;
    const unsigned long long need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if (notready & need) {
      if (spin.expired()) {
        if (lane == 0) {
          atomicOr(err, 1ull);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint32_t v = (lane <= first) ? (uint32_t)g : 0u;
    excl += (uint32_t)wave_sum64(v);
    if (first < 64) break;
    pos -= 64;
  }
  if (lane == 0)
    atomic_store_agent(status + tile, ((unsigned long long)tag_inc << 32) | (agg + excl));
  return excl;
}

// Look-back polling K x 64 predecessor granules per round trip (lane l loads the
// granules at distance 64k + l + 1, k < K, all in flight at once). kfirst = K of
// the first poll, knext = K of the later ones; sleep = s_sleep between spins.
// Used by the first-generation tiles of launches of <= 1024 tiles (ref_step_kernel).
template <int KMAX>
__device__ __forceinline__ uint32_t lookback_exclusive_wide(unsigned long long* status, uint32_t tile, uint32_t seq,
                                                            uint32_t agg, int lane, unsigned long long* err,
                                                            int kfirst, int knext, int sleep) {
  const uint32_t tag_agg = seq << 1, tag_inc = (seq << 1) | 1u;
  if (tile == 0) {
    if (lane == 0) atomic_store_agent(status, ((unsigned long long)tag_inc << 32) | agg);
    return 0;
  }
  if (lane == 0) atomic_store_agent(status + tile, ((unsigned long long)tag_agg << 32) | agg);
  uint32_t excl = 0;
  int64_t pos = (int64_t)tile - 1;  // distance 0 = tile - 1
  SpinBound spin;
  int K = kfirst;
  for (;;) {
    unsigned long long g[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      const int64_t pidx = pos - lane - 64 * k;
      g[k] = (k < K && pidx >= 0) ? atomic_load_agent(status + pidx) : ((unsigned long long)tag_inc << 32);
    }
    // newest inclusive granule (smallest distance) and readiness of everything before it
    int first = 64 * KMAX;  // distance of the newest inclusive
    bool blocked = false;
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      if (k >= K) break;
      const uint32_t tag = (uint32_t)(g[k] >> 32);
      const bool ready = (tag >> 1) == seq;
      const unsigned long long im = __ballot(ready && (tag & 1u));
      const unsigned long long nr = __ballot(!ready);
      if (first == 64 * KMAX) {
        const int f = im ? __builtin_ctzll(im) : 64;
        const unsigned long long need = f >= 63 ? ~0ull : ((2ull << f) - 1ull);
        if (nr & need) { blocked = true; break; }
        if (f < 64) first = 64 * k + f;
      }
    }
    if (blocked) {
      if (spin.expired()) {
        if (lane == 0) {
          atomicOr(err, 1ull);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        break;
      }
      for (int z = 0; z < sleep; z++) __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < KMAX; k++)
      if (k < K && 64 * k + lane <= first) v += (uint32_t)g[k];
    excl += (uint32_t)wave_sum64(v);
    if (first < 64 * KMAX) break;
    pos -= 64 * K;
    K = knext;
  }
  if (lane == 0) atomic_store_agent(status + tile, ((unsigned long long)tag_inc << 32) | (agg + excl));
  return excl;
}

constexpr int kLBWide = 8;  // granules per lane in a first-generation tile's poll

// ---- per-tile statistics -> granules; the last tile reduces them ------------
// Per tile, two 8-B granules written with agent-scope stores by one lane:
//   g0 = tag:13 | n_decided:17 | n_v1:17 | n_pending_r1:17
//   g1 = tag:13 | n_draws:17 | (largest V1 slot offset commit_phase accepts) + 1 (0 = none):17
//             | smallest undecided slot offset (0x1FFFF = none):17
// (a tile holds <= 65536 slots, so every field fits 17 bits). tag = 0x1000 |
// (seq & 0xFFF) is never 0, and the host zeroes the array whenever seq & 0xFFF
// wraps, so a granule from an earlier launch never carries the current tag. The
// tile with the last index polls and folds every tile's pair (all loads of a
// thread's tiles in flight at once). No per-tile atomics on shared words:
// thousands of same-address atomics per launch serialise at the memory side.
constexpr int kStatGranules = 2;
constexpr uint32_t kStatNone = 0x1FFFFu;

struct TileStats {
  uint32_t dec, v1, pend, draws, max_off1, min_off;
};

__device__ __forceinline__ unsigned long long stat_tag(uint32_t seq) {
  return (unsigned long long)(0x1000u | (seq & 0xFFFu)) << 51;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {  // (wave-uniform result)
  v = row_incl_scan32(v);
  return __builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31) + __builtin_amdgcn_readlane(v, 47) +
         __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { uint32_t t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
  return v;
}
__device__ __forceinline__ uint32_t wave_min32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { uint32_t t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
  return v;
}

// The four sums travel as 16-bit fields of one u64 through ONE wave reduction
// (a wave covers 64 * W * 32 <= 65535 slots, so no field overflows). The two
// offsets need no reduction: a thread's offsets are relative to the tile and
// threads own ascending word ranges, so the block maximum of max_off1 is the
// value of the highest thread that has one, and the minimum of min_off that of
// the lowest (a ballot plus a uniform readlane per wave, then the same pick
// across waves).
template <int BLOCK>
__device__ __forceinline__ TileStats block_reduce_stats(TileStats s, int lane, int wave) {
  constexpr int WAVES = BLOCK / 64;
  __shared__ unsigned long long red[WAVES][2];
  unsigned long long packed = (unsigned long long)s.dec | ((unsigned long long)s.v1 << 16) |
                              ((unsigned long long)s.pend << 32) | ((unsigned long long)s.draws << 48);
  packed = wave_sum64(packed);
  const unsigned long long hmx = __ballot(s.max_off1 != 0u), hmn = __ballot(s.min_off != ~0u);
  const uint32_t mx = hmx ? __builtin_amdgcn_readlane(s.max_off1, 63 - __builtin_clzll(hmx)) : 0u;
  const uint32_t mn = hmn ? __builtin_amdgcn_readlane(s.min_off, __builtin_ctzll(hmn)) : ~0u;
  if (lane == 0) {
    red[wave][0] = packed;
    red[wave][1] = ((unsigned long long)mn << 32) | mx;
  }
  lds_barrier();
  TileStats r{0, 0, 0, 0, 0, ~0u};
#pragma unroll
  for (int w = 0; w < WAVES; w++) {
    const unsigned long long x = red[w][0];
    r.dec += (uint32_t)(x & 0xFFFFu);
    r.v1 += (uint32_t)((x >> 16) & 0xFFFFu);
    r.pend += (uint32_t)((x >> 32) & 0xFFFFu);
    r.draws += (uint32_t)(x >> 48);
    const uint32_t wmx = (uint32_t)red[w][1], wmn = (uint32_t)(red[w][1] >> 32);
    r.max_off1 = wmx > r.max_off1 ? wmx : r.max_off1;
    r.min_off = wmn < r.min_off ? wmn : r.min_off;
  }
  return r;
}

template <int BLOCK>
__device__ __forceinline__ void block_reduce_totals(unsigned long long (&v)[7], int lane, int wave) {
  constexpr int WAVES = BLOCK / 64;
  __shared__ unsigned long long red[WAVES][7];
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = wave_sum64(v[k]);
  v[4] = wave_max64(v[4]);
  v[5] = wave_min64(v[5]);
  v[6] = wave_max64(v[6]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 7; k++) red[wave][k] = v[k];
  lds_barrier();
  unsigned long long r[7] = {0, 0, 0, 0, 0, ~0ull, 0};
#pragma unroll 1  // one wave's row at a time: unrolled, the rows' 64-bit reads set the kernel's VGPR peak
  for (int w = 0; w < WAVES; w++) {
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] += red[w][k];
    r[4] = red[w][4] > r[4] ? red[w][4] : r[4];
    r[5] = red[w][5] < r[5] ? red[w][5] : r[5];
    r[6] = red[w][6] > r[6] ? red[w][6] : r[6];
  }
#pragma unroll
  for (int k = 0; k < 7; k++) v[k] = r[k];
}

template <int FIN>
__device__ __forceinline__ void step_commit(const StepParams& p, const unsigned long long (&v)[7], const DevState& s,
                                            unsigned long long err);

// Publish this tile's statistics; the tile with the last index folds every
// tile's granules, advances the device engine state and writes the step result.
#ifndef RG_FOLD_PREFETCH
#define RG_FOLD_PREFETCH 1
#endif
template <int FIN, int BLOCK, int W, int kBatch = 4>  // kBatch: tiles per thread with loads in flight together (4: the prefetched state fits without spills)
__device__ __forceinline__ void finish_tile(const StepParams& p, Record* rec, TileStats ts,
                                            uint32_t tile, int tid, int lane, int wave) {
  constexpr uint64_t kTileSlots = (uint64_t)BLOCK * W * 32;
  static_assert(64 * W * 32 <= 0xFFFF, "per-wave sums must fit the 16-bit packed fields");
  const TileStats b = block_reduce_stats<BLOCK>(ts, lane, wave);
  const unsigned long long tag = stat_tag(p.seq);
  if (tid == 0) {
    unsigned long long* g = p.stats + (uint64_t)tile * kStatGranules;
    const uint32_t mn = b.min_off == ~0u ? kStatNone : b.min_off;
    atomic_store_agent(g + 0, tag | ((unsigned long long)b.pend << 34) | ((unsigned long long)b.v1 << 17) | b.dec);
    atomic_store_agent(g + 1, tag | ((unsigned long long)mn << 34) | ((unsigned long long)b.max_off1 << 17) | b.draws);
  }
  if (tile != p.n_tiles - 1) return;
#if RG_FOLD_PREFETCH
  // the engine state for step_commit, loaded by every thread ahead of the granule polls (a
  // load under `if (tid == 0)` is waited for at once; unconditional, its round trip hides
  // behind the polls). The state changes only in this launch's step_commit and in earlier,
  // stream-ordered launches.
  const DevState st = *p.state;
#endif

  unsigned long long v[7] = {0, 0, 0, 0, 0, ~0ull, 0};  // dec v1 pend draws max(id+1) min(id) fault
  constexpr unsigned long long kTagMask = ~0ull << 51;
  for (uint32_t i0 = tid; i0 < p.n_tiles; i0 += kBatch * BLOCK) {
    unsigned long long g[kBatch][2];
#pragma unroll
    for (int k = 0; k < kBatch; k++) {
      const uint32_t i = i0 + (uint32_t)k * BLOCK;
      const unsigned long long* gp = p.stats + (uint64_t)i * kStatGranules;
      g[k][0] = i < p.n_tiles ? atomic_load_agent(const_cast<unsigned long long*>(gp)) : tag;
      g[k][1] = i < p.n_tiles ? atomic_load_agent(const_cast<unsigned long long*>(gp) + 1) : tag;
    }
    SpinBound spin;
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int k = 0; k < kBatch; k++) ready &= ((g[k][0] & kTagMask) == tag) & ((g[k][1] & kTagMask) == tag);
      if (ready) break;
      if (spin.expired()) { v[6] = 2; break; }
      __builtin_amdgcn_s_sleep(2);
#pragma unroll
      for (int k = 0; k < kBatch; k++) {
        const uint32_t i = i0 + (uint32_t)k * BLOCK;
        unsigned long long* gp = p.stats + (uint64_t)i * kStatGranules;
        if ((g[k][0] & kTagMask) != tag) g[k][0] = atomic_load_agent(gp);
        if ((g[k][1] & kTagMask) != tag) g[k][1] = atomic_load_agent(gp + 1);
      }
    }
#pragma unroll
    for (int k = 0; k < kBatch; k++) {
      const uint32_t i = i0 + (uint32_t)k * BLOCK;
      if (i >= p.n_tiles) continue;
      const uint32_t dec = (uint32_t)(g[k][0] & kStatNone), v1 = (uint32_t)((g[k][0] >> 17) & kStatNone);
      const uint32_t pend = (uint32_t)((g[k][0] >> 34) & kStatNone);
      const uint32_t draws = (uint32_t)(g[k][1] & kStatNone), mx = (uint32_t)((g[k][1] >> 17) & kStatNone);
      const uint32_t mn = (uint32_t)((g[k][1] >> 34) & kStatNone);
      const unsigned long long tb = p.slot_base + (unsigned long long)i * kTileSlots;
      v[0] += dec; v[1] += v1; v[2] += pend; v[3] += draws;
      if (mx && tb + mx > v[4]) v[4] = tb + mx;
      if (mn != kStatNone && tb + mn < v[5]) v[5] = tb + mn;
    }
  }
#if RG_FOLD_PREFETCH
  // every tile's granules are in, so are the error bits it raised before publishing them:
  // the error word's read goes out now, from every thread (one line per wave), beside the
  // block fold
  const unsigned long long err = atomic_load_agent(&rec->error.v);
#endif
  block_reduce_totals<BLOCK>(v, lane, wave);
  stamp(p, tile, 5, tid);
  if (tid != 0) return;
#if RG_FOLD_PREFETCH
  step_commit<FIN>(p, v, st, err);
#else
  step_commit<FIN>(p, v, *p.state, atomicAdd(&rec->error.v, 0ull));
#endif
}

// The launch's totals (dec v1 pend draws max(id+1) min(id) fault) -> step result and
// engine state. Run by ONE thread after every tile's statistics are in. Each flavour
// writes only the DevState fields it owns: the sharded step may run on one stream
// while the fix-up and commit of an earlier window (rng_next, last_committed,
// commit_watermark, steps) run on another.
// s: the engine state as the launch found it; err0: the launch record's error word.
template <int FIN>
__device__ __forceinline__ void step_commit(const StepParams& p, const unsigned long long (&v)[7], const DevState& s,
                                            unsigned long long err0) {
  const unsigned long long err = err0 | v[6];
  DevResult r;
  r.n_slots = p.n_slots;
  r.n_decided = v[0];
  r.n_v1 = v[1];
  r.n_pending_r1 = v[2];
  r.n_draws = v[3];
  const unsigned long long end = p.slot_base + p.n_slots;
  const unsigned long long fu = v[5] < end ? v[5] : end;
  if constexpr (FIN == kFinShard) {
    // Shard row before the fix-up: VQ slots are not in the counts / extremes
    // (their decisions wait for the global draw positions); draws advance only
    // the provisional counter. The global engine state is left to the fix-up and
    // rg_shard_commit (state.rs:65-103 over the whole window).
    // (a multi-window launch draws every window from the same provisional position and
    // leaves shard_draws alone: the fix-up re-draws every VQ slot at its global position)
    r.last_committed_max = v[4] ? v[4] - 1 : 0;
    r.first_undecided = fu;
    r.rng_next = s.shard_draws + r.n_draws;
    r.commit_watermark = 0;
    r.flags = err;
    if (p.n_win <= 1) p.state->shard_draws = r.rng_next;
    if (p.result) *p.result = r;
    if (p.result_user) *p.result_user = r;
    return;
  }
  unsigned long long lc = s.last_committed;          // commit_phase: monotonic max,
  if (v[4] && v[4] - 1 > lc) lc = v[4] - 1;          // state.rs:77-99
  unsigned long long wm = s.commit_watermark;
  if (p.slot_base <= wm && wm < fu) wm = fu;
  r.last_committed_max = lc;
  r.first_undecided = fu;
  r.rng_next = FIN == kFinRef ? s.rng_next + r.n_draws : s.rng_next;
  r.commit_watermark = wm;
  r.flags = err;
  p.state->rng_next = r.rng_next;
  p.state->last_committed = lc;
  p.state->commit_watermark = wm;
  p.state->steps = s.steps + 1;
  *p.result = r;
  if (p.result_user) *p.result_user = r;
}

// Called once per tile right after it learns its index. The holder of the last
// tile resets the OTHER record of the ring for the next launch (the previous
// launch, which used it, completed before this one started: stream order).
// A tile index outside the launch (a ring that was not reset) exits before any
// memory access and raises a fault bit instead of indexing out of bounds.
__device__ __forceinline__ bool tile_prologue(const StepParams& p, Record* rec, uint32_t tile, int tid) {
  if (tile >= p.n_tiles) {
    if (tid == 0) atomicOr(&rec->error.v, 4ull);
    return false;
  }
  if (tid == 0 && tile == p.n_tiles - 1) {
    Record* nxt = p.rec + ((p.seq + 1) & 1u);
    atomic_store_agent(&nxt->error.v, 0ull);
    atomic_store_agent(&nxt->ticket.v, 0ull);
    atomic_store_agent(&nxt->done.v, 0ull);
  }
  return true;
}

// Per-thread statistics; offsets are relative to the tile's first slot.
template <int W>
__device__ __forceinline__ TileStats thread_stats(const uint32_t (&committed)[W], const uint32_t (&v1)[W],
                                                  const uint32_t (&pend)[W], const uint32_t (&vm)[W],
                                                  uint32_t draws, uint64_t w0, uint32_t tw0,
                                                  const StepParams& p) {
  TileStats t{0, 0, 0, draws, 0, ~0u};
#pragma unroll
  for (int i = 0; i < W; i++) {
    t.dec += __builtin_popcount(committed[i]);
    t.v1 += __builtin_popcount(v1[i]);
    t.pend += __builtin_popcount(pend[i]);
  }
#pragma unroll
  for (int i = W - 1; i >= 0; i--) {
    const uint32_t m = v1[i] & phase_limit_mask(p.slot_base, w0 + i, p.max_phase);
    if (m && !t.max_off1) t.max_off1 = 32u * (tw0 + i) + (31u - __builtin_clz(m)) + 1u;
  }
#pragma unroll
  for (int i = 0; i < W; i++) {
    const uint32_t m = ~committed[i] & vm[i];
    if (m && t.min_off == ~0u) t.min_off = 32u * (tw0 + i) + __builtin_ctz(m);
  }
  return t;
}

// ============================================================================
// REF phase step: engine.rs:483-682 on the final vote sets of every slot.
// ============================================================================
// Occupancy: 4 waves per SIMD (<= 128 VGPRs) so that at least two 512-thread or
// four 256-thread tiles are resident per CU and one tile's look-back / stores
// overlap another's loads.
// Plane loads without a branch: a thread past the window loads word 0 instead
// (its valid masks are 0, so the values are never used). A conditional load makes
// hipcc wait for it right away, which would drain the ring's prefetch.
template <int N, int W>
__device__ __forceinline__ void load_planes_any(const StepParams& p, uint64_t w0, int first_plane,
                                                uint32_t (&lo)[N][W], uint32_t (&hi)[N][W]) {
  const uint32_t* base = p.votes + p.lin.base(w0 < p.n_words ? w0 : 0);
  const uint64_t ps = p.lin.pstride;
#pragma unroll
  for (int j = 0; j < N; j++) {
    load_words<W>(base + (first_plane + 2 * j) * ps, lo[j]);
    load_words<W>(base + (first_plane + 2 * j + 1) * ps, hi[j]);
  }
}

// Decisions of count_votes(R2') for both possible own votes at once:
// A = own V0 on the VQ slots, B = own V1 (engine.rs:540-542, 613-628). The other
// lanes are tallied once; the self lane is added per variant. On non-VQ slots the
// own vote is already known (V0, V1, or none when round 1 is pending), so A == B.
template <int N, int W>
__device__ __forceinline__ void r2_decision_ab(const uint32_t (&lo)[N][W], const uint32_t (&hi)[N][W], int i,
                                               uint32_t q, int self, uint32_t v1, uint32_t vq, uint32_t pend,
                                               uint32_t& alo, uint32_t& ahi, uint32_t& blo, uint32_t& bhi) {
  constexpr int B = ctr_bits(N);
  uint32_t m0[N], m1[N], mq[N];
  uint32_t sl = 0, sh = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint32_t keep = j == self ? 0u : ~0u;  // wave-uniform: the self lane counts as absent here
    const uint32_t l = lo[j][i], h = hi[j][i];
    sl |= l & ~keep;
    sh |= h & ~keep;
    m0[j] = ~l & ~h & keep;
    m1[j] = l & ~h & keep;
    mq[j] = ~l & h & keep;
  }
  const Ctr<B> c0 = ctr_count<N>(m0), c1 = ctr_count<N>(m1), cq = ctr_count<N>(mq);
  const bool has_self = (unsigned)self < (unsigned)N;  // self_lane -1: no own vote joins R2
#pragma unroll
  for (int v = 0; v < 2; v++) {
    const uint32_t own = v ? (v1 | vq) : v1;
    const uint32_t l = has_self ? (sl & pend) | (own & ~pend) : ~0u, h = has_self ? sh & pend : ~0u;
    Ctr<B> d0c = c0, d1c = c1, dqc = cq;
    ctr_add(d0c, ~l & ~h);
    ctr_add(d1c, l & ~h);
    ctr_add(dqc, ~l & h);
    const uint32_t d0 = ctr_ge(d0c, q);
    const uint32_t d1 = ~d0 & ctr_ge(d1c, q);
    const uint32_t dq = ~d0 & ~d1 & ctr_ge(dqc, q);
    const uint32_t dn = ~(d0 | d1 | dq);
    (v ? blo : alo) = d1 | dn;
    (v ? bhi : ahi) = dq | dn;
  }
}

// SHARD = the sharded-REF flavour (rg_phase_step_shard_async): the draws come from
// the shard's provisional stream position, every VQ slot also leaves a draw
// record (its decision under both own votes) for rg_shard_fixup_async, and the
// tile statistics leave the VQ slots out.
// The R2 loads go out after the round-1 tally (the R1 registers are dead by then),
// so the kernel fits 4 waves per SIMD: two 512-thread tiles resident per CU, one
// tile's look-back overlapping the other's loads.
// ChaCha block computed by the 4 lanes of a quad (rand_chacha 0.3.1 layout, as
// chacha_block): lane q holds column q (words q, 4+q, 8+q, 12+q), so a column round
// is one quarter round per lane; for a diagonal round lane q takes rows b, c, d from
// lanes q+1, q+2, q+3 of its quad (DPP quad permutes) and hands them back after it.
// A quarter of the dependent-instruction chain of one lane per block. Every lane of
// a quad must be active.
__device__ __forceinline__ uint32_t quad_rot(uint32_t v, int by) {  // lane q <- lane (q + by) & 3
  if (by == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x39, 0xF, 0xF, false);
  if (by == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x93, 0xF, 0xF, false);
}
template <int ROUNDS>
__device__ __forceinline__ void chacha_block_quad(const Key& key, uint64_t counter, uint64_t stream, int q,
                                                  uint32_t (&o)[4]) {
  // the key words as wave-uniform values first: selecting among struct fields by a
  // lane index otherwise becomes a per-lane load from the kernel arguments (a vector
  // memory load whose wait covers every plane load in flight)
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = __builtin_amdgcn_readfirstlane(key.k[i]);
  const uint32_t a0 = q == 0 ? 0x61707865u : (q == 1 ? 0x3320646eu : (q == 2 ? 0x79622d32u : 0x6b206574u));
  const uint32_t b0 = q == 0 ? k[0] : (q == 1 ? k[1] : (q == 2 ? k[2] : k[3]));
  const uint32_t c0 = q == 0 ? k[4] : (q == 1 ? k[5] : (q == 2 ? k[6] : k[7]));
  const uint32_t d0 = q == 0 ? (uint32_t)counter
                             : (q == 1 ? (uint32_t)(counter >> 32) : (q == 2 ? (uint32_t)stream : (uint32_t)(stream >> 32)));
  uint32_t a = a0, b = b0, c = c0, d = d0;
#define RG_QR1()                                  \
  a += b; d = rotl32(d ^ a, 16);                  \
  c += d; b = rotl32(b ^ c, 12);                  \
  a += b; d = rotl32(d ^ a, 8);                   \
  c += d; b = rotl32(b ^ c, 7);
#pragma unroll
  for (int r = 0; r < ROUNDS; r += 2) {
    RG_QR1()
    b = quad_rot(b, 1); c = quad_rot(c, 2); d = quad_rot(d, 3);
    RG_QR1()
    b = quad_rot(b, 3); c = quad_rot(c, 2); d = quad_rot(d, 1);
  }
#undef RG_QR1
  o[0] = a + a0; o[1] = b + b0; o[2] = c + c0; o[3] = d + d0;
}

#ifndef RG_STEP_QUAD
#define RG_STEP_QUAD 1
#endif
template <int N, int W, int BLOCK, bool SHARD>
__global__ __launch_bounds__(BLOCK, 4) void ref_step_kernel(StepParams p_arg) {
  StepParams p = p_arg;
  if constexpr (SHARD) {
    if (p.n_win > 1) {  // window blockIdx.y of a multi-window shard launch (uniform values)
      const uint32_t w = blockIdx.y;
      p.votes += w * p.win_in_pitch;
      p.out += w * p.win_out_pitch;
      p.slot_base += w * p.win_id_stride;
      p.lookback += (uint64_t)w * p.n_tiles;
      p.stats += (uint64_t)w * p.n_tiles * kStatGranules;
      p.vq_rec += w * p.rec_pitch;
      p.result_user += w;
      if (w + 1 != p.n_win) p.result = nullptr;  // the context's result: the last window's row
    }
  }
  constexpr int B = ctr_bits(N);
  constexpr int WAVES = BLOCK / 64;
  __shared__ uint32_t s_wave[WAVES];
  __shared__ uint32_t s_excl;
  __shared__ uint32_t s_cls[2 * W][BLOCK];  // (c1 > c0), (c1 < c0) of the VQ slots, parked in LDS
  Record* rec = p.rec + (p.seq & 1u);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tile = blockIdx.x;
  if (!tile_prologue(p, rec, tile, tid)) return;
  stamp(p, tile, 0, tid);
  const uint32_t tw0 = (uint32_t)tid * W;  // word offset inside the tile
  const uint64_t w0 = (uint64_t)tile * BLOCK * W + tw0;
  const bool active = w0 < p.n_words;

  uint32_t r1lo[N][W], r1hi[N][W], r2lo[N][W], r2hi[N][W];
  load_planes_any<N, W>(p, w0, 0, r1lo, r1hi);  // branchless: past the window they read word 0

  // ---- round 1: count_votes + |votes| >= quorum fallback (engine.rs:495-505).
  // Only what the draws need survives the tally: per-slot (c1 > c0), (c1 < c0).
  uint32_t r1v1[W], r1vq[W], pend[W];
  uint32_t vq_count = 0;
  uint32_t seq0 = 0;  // a zero the compiler cannot see through, chaining word i+1 after word i
#pragma unroll
  for (int i = 0; i < W; i++) {
    const uint32_t vm = valid_mask(w0 + i, p.n_words, p.n_slots);
    uint32_t m0[N], m1[N], mp[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint32_t lo = r1lo[j][i], hi = r1hi[j][i];
      m0[j] = ~lo & ~hi;
      m1[j] = lo & ~hi;
      mp[j] = ~(lo & hi);
    }
    m0[0] |= seq0; m1[0] |= seq0; mp[0] |= seq0;  // (the words tally one after another: no 4-word ILP)
    const Ctr<B> c0 = ctr_count<N>(m0), c1 = ctr_count<N>(m1), cp = ctr_count<N>(mp);
    const uint32_t g0 = ctr_ge(c0, p.q), g1 = ctr_ge(c1, p.q), gp = ctr_ge(cp, p.q);
    const uint32_t v0 = g0 & vm;
    r1v1[i] = ~g0 & g1 & vm;
    r1vq[i] = ~g0 & ~g1 & gp & vm;  // cq >= q implies present >= q
    pend[i] = ~(v0 | r1v1[i] | r1vq[i]) & vm;
    uint32_t gt, lt;
    ctr_cmp(c1, c0, gt, lt);
    s_cls[2 * i][tid] = gt & r1vq[i];
    s_cls[2 * i + 1][tid] = lt & r1vq[i];
    vq_count += __builtin_popcount(r1vq[i]);
    asm volatile("" : "+v"(seq0), "+v"(r1v1[i]), "+v"(r1vq[i]), "+v"(pend[i]));
  }
  load_planes_any<N, W>(p, w0, 2 * N, r2lo, r2hi);

  // ---- exclusive prefix of VQ slots: block scan + cross-tile look-back
  const uint32_t incl = wave_incl_scan32(vq_count, lane);
  if (lane == 63) s_wave[wave] = incl;
  lds_barrier();
  uint32_t wave_off = 0, tile_total = 0;
  {  // one LDS read per lane, the sums as wave-uniform scalars
    const uint32_t sw = lane < WAVES ? s_wave[lane] : 0u;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (int w = 0; w < WAVES; w++) {
      const uint32_t x = __builtin_amdgcn_readlane(sw, w);
      wave_off += (w < wv) ? x : 0u;
      tile_total += x;
    }
  }
  stamp(p, tile, 1, tid);
  if (wave == 0) {
    // The launch's first tiles all start together, and tile t needs the aggregates of
    // all t predecessors: with 64 granules per poll the inclusive frontier crosses the
    // first generation in t/64 round trips while the later tiles hold their CUs.
    // In launches of at most 1024 tiles (a single 2^20 window: 14.1 -> 13.2 us) those
    // tiles poll kLBWide x 64 predecessors at once; larger launches keep the
    // one-granule-per-lane poll (wider polls measured slower there).
    uint32_t e = 0;
    if (!(p.diag & 1u)) {
      if (tile < 64u * kLBWide && p.n_tiles <= 1024u && !(p.diag & 16u)) {
        const int kf = (int)((tile + 63u) / 64u);
        e = lookback_exclusive_wide<kLBWide>(p.lookback, tile, p.seq, tile_total, lane, &rec->error.v, kf, kLBWide, 1);
      } else {
        e = lookback_exclusive(p.lookback, tile, p.seq, tile_total, lane, &rec->error.v);
      }
    }
    if (lane == 0) s_excl = e;
  }
  // both-outcome decisions while wave 0 looks back; the R2 registers die here,
  // before the ChaCha12 blocks need theirs
  uint32_t dalo[W], dahi[W], dblo[W], dbhi[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    r2_decision_ab<N, W>(r2lo, r2hi, i, p.q, p.self_lane, r1v1[i], r1vq[i], pend[i], dalo[i], dahi[i], dblo[i],
                         dbhi[i]);
    // pin the results here (volatile asm keeps its order with the barrier below):
    // otherwise the decisions sink to their use and R2 stays live across ChaCha
    asm volatile("" : "+v"(dalo[i]), "+v"(dahi[i]), "+v"(dblo[i]), "+v"(dbhi[i]));
  }
  lds_barrier();
  stamp(p, tile, 2, tid);

  // ---- own round-2 vote (engine.rs:523-537; VQ -> one StdRng draw, 567-611).
  // The tile's draws are ONE contiguous index range [k_tile, k_tile + tile_total):
  // its ChaCha12 blocks are computed once, one per thread, and staged in LDS.
  const unsigned long long k_base = SHARD ? p.state->shard_draws : p.state->rng_next;
  const unsigned long long k_tile = k_base + s_excl;
  const unsigned long long k_first = k_tile + wave_off + incl - vq_count;  // this thread's first draw
  unsigned long long k = k_first;
  uint32_t own_lo[W], mq[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    own_lo[i] = r1v1[i];
    mq[i] = r1vq[i];
  }
  if (tile_total) {
    // RG_STEP_QUAD: block r by the lanes 4r .. 4r + 3 (chacha_block_quad: a quarter of one
    // lane's dependent chain), else one block per thread. The draws sit on the launch's
    // critical path after the look-back; a small tile has few of them (a 4,096-slot tile of
    // the 2^20 sweep: ~5 blocks), so the chain's latency, not the issue, is what counts.
    constexpr int kRows = RG_STEP_QUAD ? BLOCK / 4 : (BLOCK < 128 ? BLOCK : 128);
    __shared__ uint32_t s_blk[kRows][17];  // +1 word: conflict-free rows
    const unsigned long long b_first = k_tile >> 3, b_last = (k_tile + tile_total - 1) >> 3;
    for (unsigned long long cb = b_first; cb <= b_last; cb += kRows) {
      if constexpr (RG_STEP_QUAD != 0) {
        const uint32_t r = (uint32_t)tid >> 2;  // (quad-uniform condition)
        if (cb + r <= b_last) {
          uint32_t o[4];
          chacha_block_quad<12>(p.key, cb + r, 0, tid & 3, o);
          const int q = tid & 3;
          s_blk[r][q] = o[0];
          s_blk[r][4 + q] = o[1];
          s_blk[r][8 + q] = o[2];
          s_blk[r][12 + q] = o[3];
        }
      } else if (tid < kRows && cb + tid <= b_last) {
        uint32_t x[16];
        chacha_block<12>(p.key, cb + tid, 0, x);
#pragma unroll
        for (int j = 0; j < 16; j++) s_blk[tid][j] = x[j];
      }
      lds_barrier();
      const unsigned long long k_lim = (cb + kRows) << 3;
#pragma unroll
      for (int i = 0; i < W; i++) {
        if (!mq[i] || k >= k_lim) continue;
        const uint32_t gtm = s_cls[2 * i][tid], ltm = s_cls[2 * i + 1][tid];
        while (mq[i] && k < k_lim) {
          const int b = __builtin_ctz(mq[i]);
          mq[i] &= mq[i] - 1;
          const uint32_t row = (uint32_t)((k >> 3) - cb), ws = (uint32_t)(k & 7u) * 2u;
          const unsigned long long u =
              (unsigned long long)s_blk[row][ws] | ((unsigned long long)s_blk[row][ws + 1] << 32);
          const bool gt = (gtm >> b) & 1u, lt = (ltm >> b) & 1u;
          const bool v1 = gt ? (u < kP90) : (lt ? (u >= kP90) : (u < kP80));
          own_lo[i] |= (uint32_t)v1 << b;
          k++;
        }
      }
      lds_barrier();
    }
  }

  // ---- own vote joins round2_votes (engine.rs:540-542); decision (613-628),
  // one word at a time; only the decision masks stay live for the stores
  uint32_t dlo[W], dhi[W];
  unsigned long long kr = k_first - k_base;  // SHARD: local draw number of this thread's first VQ slot
  if constexpr (SHARD) {  // the record segment this thread's words start: its first record
    if ((w0 & (kRecChunkWords - 1)) == 0 && active) p.vq_rec[w0 / kRecChunkWords] = (uint32_t)kr;
  }
#pragma unroll
  for (int i = 0; i < W; i++) {
    const uint32_t sel = own_lo[i] & r1vq[i];  // VQ slots whose draw gave V1
    dlo[i] = (dalo[i] & ~sel) | (dblo[i] & sel);
    dhi[i] = (dahi[i] & ~sel) | (dbhi[i] & sel);
    if constexpr (SHARD) {  // draw records: both decisions are at hand already
      uint32_t m = r1vq[i];
      const uint32_t gtm = m ? s_cls[2 * i][tid] : 0u, ltm = m ? s_cls[2 * i + 1][tid] : 0u;
      while (m) {  // indexed by local draw number (ascending slot order)
        const int b = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t own = (own_lo[i] >> b) & 1u;
        const uint32_t d_v0 = ((dalo[i] >> b) & 1u) | (((dahi[i] >> b) & 1u) << 1);
        const uint32_t d_v1 = ((dblo[i] >> b) & 1u) | (((dbhi[i] >> b) & 1u) << 1);
        const uint32_t cls = ((gtm >> b) & 1u) ? kRecGt : (((ltm >> b) & 1u) ? kRecLt : 0u);
        const uint32_t info = cls | (d_v0 << 2) | (d_v1 << 4) | (own << 6);
        const uint32_t off = (uint32_t)(32u * (w0 + i) + b);
        if (kr < p.vq_cap) p.vq_rec[p.rec_tw + kr] = rec_make(off, info);
        kr++;
      }
    }
    const uint32_t vm = valid_mask(w0 + i, p.n_words, p.n_slots);
    dlo[i] &= vm;
    dhi[i] &= vm;
  }
  uint32_t st_dec[W], st_v1[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    st_dec[i] = ~dhi[i] & valid_mask(w0 + i, p.n_words, p.n_slots);  // committed iff not VQuestion
    st_v1[i] = dlo[i] & ~dhi[i];  // V1: apply_batch + commit_phase
  }
  if (active) {  // plane by plane from the masks (include/rabia_gpu.h output planes)
    uint32_t* ob = p.out + p.lout.base(w0);
    const uint64_t ps = p.lout.pstride;
    uint32_t v[W];
#pragma unroll
    for (int i = 0; i < W; i++) v[i] = r1v1[i] | pend[i];
    store_words_nt<W>(ob, v);
#pragma unroll
    for (int i = 0; i < W; i++) v[i] = r1vq[i] | pend[i];
    store_words_nt<W>(ob + ps, v);
#pragma unroll
    for (int i = 0; i < W; i++) v[i] = own_lo[i] | pend[i];
    store_words_nt<W>(ob + 2 * ps, v);
    store_words_nt<W>(ob + 3 * ps, pend);
    store_words_nt<W>(ob + 4 * ps, dlo);
    store_words_nt<W>(ob + 5 * ps, dhi);
    store_words_nt<W>(ob + 6 * ps, st_dec);
    store_words_nt<W>(ob + 7 * ps, st_v1);
  }
  stamp(p, tile, 3, tid);
  if (p.diag & 2u) return;
  uint32_t st_vm[W];
#pragma unroll
  for (int i = 0; i < W; i++) {  // SHARD: VQ slots are counted by the fix-up
    const uint32_t keep = SHARD ? ~r1vq[i] : ~0u;
    st_dec[i] &= keep;
    st_v1[i] &= keep;
    st_vm[i] = valid_mask(w0 + i, p.n_words, p.n_slots) & keep;
  }
  const TileStats ts = thread_stats<W>(st_dec, st_v1, pend, st_vm, vq_count, w0, tw0, p);
  finish_tile<SHARD ? kFinShard : kFinRef, BLOCK, W>(p, rec, ts, tile, tid, lane, wave);
  stamp(p, tile, 4, tid);
}

// ============================================================================
// Persistent REF step with dynamic tile tickets and a one-tile lag (large launches).
//
// The tiled kernel above makes every tile wait for its VQ prefix between its plane
// loads and its stores; under full streaming load a look-back poll is a 3-4 us
// round trip through the CU's own memory queue (MI355X_MICROARCH.md handoff-1to1),
// during which the tile's 8 waves hold half the CU and move nothing. Here a
// workgroup never waits for its own tile: it publishes the tile's aggregate, parks
// what the draws still need in LDS, and takes its next tile; the parked tile is
// finished (draws, decisions, stores) one iteration later, while the next tile's
// round-2 planes are in flight. By then every predecessor published its aggregate
// long ago, so the look-back almost never spins.
//
// Tile order is a ticket from one counter per launch (Record.ticket), not
// blockIdx: a tile index is only ever held by a running workgroup and a workgroup
// only waits for lower tickets, whose holders never wait on it (the lowest
// unfinished ticket always progresses). Forward progress therefore needs no
// dispatch-order assumption, and two such launches sharing a GPU cannot wait on
// each other (the tiled kernel's cross-kernel cycle).
//
// Look-back of the parked tile p: the workgroup knows the inclusive prefix of its
// own previous tile pp (< p), so the scan ends at pp at the latest; any newer
// inclusive granule ends it earlier. kLagPoll x 64 granules per poll, issued at the
// top of the iteration (ahead of the round-1 loads) and resolved after the tally.
// Statistics accumulate per thread over all of a workgroup's tiles; each
// workgroup publishes one record and the last to arrive (Record.done) folds them.
// ============================================================================
constexpr int kLagPoll = 4;
// The 512-thread lag kernel (2 waves per SIMD) keeps <= 224 VGPRs, so one 64-VGPR wave of
// the exchange kernels (the fix-up, finish, commit and decision lists of the previous step,
// on a second stream) fits beside the sharded step on every SIMD (2 x 224 + 64 = 512); at
// n = 9 it would take 232 (n <= 8: <= 216 anyway), and the exchange chain then waits for
// the whole step kernel at each launch. (The request is in units gfx950 doubles, unified
// VGPR/AGPR file; it cannot depend on the template arguments, so the single evaluator's
// instantiations carry it too; ignored where the shape's own budget is lower: the
// 1024-thread forms get 128.)
#define RG_LAG_REGS __attribute__((amdgpu_num_vgpr(112)))
constexpr int kLagStatGranules = 6;  // dec v1 pend draws max_off1 min_off, {tag:13 | value:51}

// Poll granules at distances d = 64k + lane below `pos` (index pos - d); indices at
// or below pp are never read (their value is synthetic: pp is inclusive).
__device__ __forceinline__ void lag_poll(const unsigned long long* status, int32_t pos, int32_t pp, int lane,
                                         unsigned long long (&g)[kLagPoll]) {
#pragma unroll
  for (int k = 0; k < kLagPoll; k++) {
    const int32_t idx = pos - lane - 64 * k;
    // branchless: an index at or below pp reads granule 0 and the value is ignored
    g[k] = atomic_load_agent(const_cast<unsigned long long*>(status) + (idx > pp ? idx : 0));
  }
}

// One pass of the look-back of tile p over a poll g at `pos` (wave 0, all lanes):
// adds the values up to the newest inclusive granule to excl and returns true when
// that granule was in the poll (the prefix is complete); false with blocked = some
// needed granule is not published yet (poll again at the same pos), or blocked =
// false: everything was an aggregate (continue below pos - 64 * kLagPoll).
__device__ __forceinline__ bool lag_eval(const unsigned long long (&g)[kLagPoll], int32_t pos, int32_t pp,
                                         uint32_t incl_pp, uint32_t seq, int lane, uint32_t& excl,
                                         bool& blocked) {
  int first = 64 * kLagPoll;
  bool blk = false;
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < kLagPoll; k++) {
    const int32_t idx = pos - lane - 64 * k;
    const uint32_t tag = (uint32_t)(g[k] >> 32);
    const bool synth = idx <= pp;
    const bool ready = synth || (tag >> 1) == seq;
    const bool incl = synth || (ready && (tag & 1u));
    const unsigned long long im = __ballot(incl), nr = __ballot(!ready);
    const bool open = first == 64 * kLagPoll && !blk;  // wave-uniform
    const int f = im ? __builtin_ctzll(im) : 64;
    const unsigned long long need = f >= 63 ? ~0ull : ((2ull << f) - 1ull);
    if (open && (nr & need)) blk = true;
    if (open && !(nr & need)) {
      if (lane <= f) v += idx == pp ? incl_pp : (synth ? 0u : (uint32_t)g[k]);
      if (f < 64) first = 64 * k + f;
    }
  }
  blocked = blk;
  if (blk) return false;
  excl += wave_sum32(v);
  return first < 64 * kLagPoll;
}

// The rest of a look-back that lag_eval left open (pos/excl as it left them).
__device__ __forceinline__ uint32_t lag_finish(const unsigned long long* status, int32_t pos, int32_t pp,
                                               uint32_t incl_pp, uint32_t seq, int lane, uint32_t excl,
                                               bool blocked, unsigned long long* err) {
  SpinBound spin;
  for (;;) {
    if (blocked) {
      if (spin.expired()) {
        if (lane == 0) {
          atomicOr(err, 1ull);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
    } else {
      pos -= 64 * kLagPoll;
    }
    unsigned long long g[kLagPoll];
    lag_poll(status, pos, pp, lane, g);
    if (lag_eval(g, pos, pp, incl_pp, seq, lane, excl, blocked)) return excl;
  }
}

// W consecutive words of one thread in LDS (one ds_read/write_b128 at W = 4)
template <int W>
__device__ __forceinline__ void lds_ld(const uint32_t* s, uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    const u32x4 x = *reinterpret_cast<const u32x4*>(s);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (W == 2) {
    const u32x2 x = *reinterpret_cast<const u32x2*>(s);
    v[0] = x.x; v[1] = x.y;
  } else {
    v[0] = s[0];
  }
}
template <int W>
__device__ __forceinline__ void lds_st(uint32_t* s, const uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    u32x4 x;
    x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
    *reinterpret_cast<u32x4*>(s) = x;
  } else if constexpr (W == 2) {
    u32x2 x;
    x.x = v[0]; x.y = v[1];
    *reinterpret_cast<u32x2*>(s) = x;
  } else {
    s[0] = v[0];
  }
}

// Plane access of the lag kernel through buffer resources: the tile's uniform base in
// SGPRs, the thread's offset in ONE VGPR for every plane, the plane offset in an SGPR
// (a global load needs a 64-bit VGPR address per plane: 20 of them in flight at n = 5).
// A tile of kTW words starts on a layout-tile boundary (both powers of two), so
// Layout::base(tile_start + x) = base(tile_start) + base(x).
// num_records = 2^31: an offset of kOffNone (a lane past the window) is out of range,
// so its store is dropped by the buffer unit instead of being branched around (a
// conditional store between a load and its use makes the compiler's waitcnt merge
// wait for everything). The host keeps every real offset below 2^31.
constexpr uint32_t kOffNone = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const uint32_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(base), (short)0, (int)kOffNone, 0x00020000);
}
constexpr int kAuxNT = 2;  // non-temporal (read or written once; default policy measured slower)

template <int W>
__device__ __forceinline__ void buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kAuxNT);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (W == 2) {
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kAuxNT);
    v[0] = x.x; v[1] = x.y;
  } else {
    v[0] = __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, kAuxNT);
  }
}
template <int W>
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, const uint32_t (&v)[W]) {
  if constexpr (W == 4) {
    u32x4 x;
    x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
    __builtin_amdgcn_raw_buffer_store_b128(x, r, voff, soff, kAuxNT);
  } else if constexpr (W == 2) {
    u32x2 x;
    x.x = v[0]; x.y = v[1];
    __builtin_amdgcn_raw_buffer_store_b64(x, r, voff, soff, kAuxNT);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(v[0], r, voff, soff, kAuxNT);
  }
}
// 2N vote planes starting at plane `first` (lo, hi per replica lane)
template <int N, int W>
__device__ __forceinline__ void buf_ld_planes(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t pbytes, int first,
                                              uint32_t (&lo)[N][W], uint32_t (&hi)[N][W]) {
#pragma unroll
  for (int j = 0; j < N; j++) {
    buf_ld<W>(r, voff, (uint32_t)(first + 2 * j) * pbytes, lo[j]);
    buf_ld<W>(r, voff, (uint32_t)(first + 2 * j + 1) * pbytes, hi[j]);
  }
}

// Parked per-thread state of a tile, s_park[buffer][field][tid][word]; two buffers
// (by iteration parity): the tile being tallied writes one while the parked tile's
// finish reads the other, so no tile state waits in registers across the finish.
//   0 plane-0 value (V1 | pending; plane 2 = this | the VQ slots whose draw gave V1)
//   1 pending (round 1 without quorum)
//   2 e0 = VQ & !(c1 < c0), 3 e1 = VQ & !(c1 > c0)   (VQ = e0 | e1; gt = e0 & !e1, lt = e1 & !e0)
//   4-5 decision (lo, hi) if the own round-2 vote is V0, 6-7 if it is V1
constexpr int kParkFields = 8;

// Next tile ticket. The address is made divergent-looking so that LLVM's atomic
// optimizer leaves the returning atomic alone: its wave-aggregated form reads the
// result back at once (s_waitcnt vmcnt(0)), i.e. waits for every store in flight.
// 32-bit (the low word of Record.ticket): a 64-bit result register pair whose high
// half is dead gets reused while the atomic is in flight, which forces a wait.
__device__ __forceinline__ uint32_t take_ticket(Record* rec) {
  const uint32_t zero = __builtin_amdgcn_mbcnt_lo(0u, 0u);  // 0, divergent to the compiler
  return atomicAdd(reinterpret_cast<unsigned int*>(&rec->ticket.v) + zero, 1u);
}

// Where a ticket's tile lives: window w of a multi-window launch, tile c inside it.
struct TileLoc {
  uint32_t w, c;
};

// Multi-window lag launch: the last workgroup folds the per-tile granules (finish_tile's
// format, tile-relative offsets) window by window, one wave per window, and writes each
// window's shard row (the kFinShard row of step_commit: VQ slots left to the fix-up, every
// window drawn from the same provisional position, shard_draws left alone).
template <int WAVES, uint32_t kTileSlots>
__device__ __forceinline__ void lag_fold_windows(const StepParams& p, Record* rec, int lane, int wave) {
  constexpr int kB = 4;  // tiles per lane with their loads in flight together
  constexpr unsigned long long kTagMask = ~0ull << 51;
  const unsigned long long tag = stat_tag(p.seq);
  const unsigned long long err0 = atomicAdd(&rec->error.v, 0ull);
  for (uint32_t w = (uint32_t)wave; w < p.n_win; w += WAVES) {
    const unsigned long long* st = p.stats + (uint64_t)w * p.n_tiles * kStatGranules;
    const unsigned long long sbase = p.slot_base + (unsigned long long)w * p.win_id_stride;
    unsigned long long v[7] = {0, 0, 0, 0, 0, ~0ull, 0};  // dec v1 pend draws max(id+1) min(id) fault
    for (uint32_t i0 = (uint32_t)lane; i0 < p.n_tiles; i0 += 64 * kB) {
      unsigned long long g[kB][2];
#pragma unroll
      for (int k = 0; k < kB; k++) {
        const uint32_t i = i0 + 64u * k;
        unsigned long long* gp = const_cast<unsigned long long*>(st) + (uint64_t)i * kStatGranules;
        g[k][0] = i < p.n_tiles ? atomic_load_agent(gp) : tag;
        g[k][1] = i < p.n_tiles ? atomic_load_agent(gp + 1) : tag;
      }
      SpinBound spin;
      for (;;) {  // visible already (arrival counter): a guard, not a wait
        bool ready = true;
#pragma unroll
        for (int k = 0; k < kB; k++) ready &= ((g[k][0] & kTagMask) == tag) & ((g[k][1] & kTagMask) == tag);
        if (ready) break;
        if (spin.expired()) { v[6] = 2; break; }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < kB; k++) {
          unsigned long long* gp = const_cast<unsigned long long*>(st) + (uint64_t)(i0 + 64u * k) * kStatGranules;
          if ((g[k][0] & kTagMask) != tag) g[k][0] = atomic_load_agent(gp);
          if ((g[k][1] & kTagMask) != tag) g[k][1] = atomic_load_agent(gp + 1);
        }
      }
#pragma unroll
      for (int k = 0; k < kB; k++) {
        const uint32_t i = i0 + 64u * k;
        if (i >= p.n_tiles) continue;
        const uint32_t dec = (uint32_t)(g[k][0] & kStatNone), v1 = (uint32_t)((g[k][0] >> 17) & kStatNone);
        const uint32_t pend = (uint32_t)((g[k][0] >> 34) & kStatNone);
        const uint32_t draws = (uint32_t)(g[k][1] & kStatNone), mx = (uint32_t)((g[k][1] >> 17) & kStatNone);
        const uint32_t mn = (uint32_t)((g[k][1] >> 34) & kStatNone);
        const unsigned long long tb = sbase + (unsigned long long)i * kTileSlots;
        v[0] += dec; v[1] += v1; v[2] += pend; v[3] += draws;
        if (mx && tb + mx > v[4]) v[4] = tb + mx;
        if (mn != kStatNone && tb + mn < v[5]) v[5] = tb + mn;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = wave_sum64(v[k]);
    v[4] = wave_max64(v[4]);
    v[5] = wave_min64(v[5]);
    v[6] = wave_max64(v[6]);
    if (lane == 0) {
      DevResult r;
      r.n_slots = p.n_slots;
      r.n_decided = v[0];
      r.n_v1 = v[1];
      r.n_pending_r1 = v[2];
      r.n_draws = v[3];
      const unsigned long long end = sbase + p.n_slots;
      r.last_committed_max = v[4] ? v[4] - 1 : 0;
      r.first_undecided = v[5] < end ? v[5] : end;
      r.rng_next = p.state->shard_draws + r.n_draws;
      r.commit_watermark = 0;
      r.flags = err0 | v[6];
      p.result_user[w] = r;
      if (w + 1 == p.n_win && p.result) *p.result = r;
    }
  }
}

// MW = the multi-window sharded launch (rg_phase_step_shard_windows_async, SHARD only):
// tickets run window-major over n_win windows of n_tiles tiles each (ticket t = window
// t / n_tiles, tile t % n_tiles), so the grid streams through the K windows as through
// one long launch and pays the ramp and drain once. Each window keeps its own look-back
// chain (its tile 0 publishes an inclusive prefix; a look-back never reads below its
// window's first ticket), its own draw records and its own row. The statistics are per
// tile (two tagged granules, as the tiled kernel's), published one iteration after the
// tile's stores by wave 0, and the last workgroup to arrive folds them window by window
// (one wave per window).
template <int N, int W, int BLOCK, bool SHARD, int OCC = 4, bool MW = false>
__global__ __launch_bounds__(BLOCK, OCC) RG_LAG_REGS void ref_lag_kernel(StepParams p) {  // OCC waves/SIMD: 2 x 512 or 1 x 1024 per CU
  static_assert(!MW || SHARD, "multi-window lag launches are sharded launches");
  constexpr int B = ctr_bits(N);
  constexpr int WAVES = BLOCK / 64;
  constexpr int kRows = BLOCK / 4;  // ChaCha12 blocks per pass, one per quad of lanes
  constexpr uint32_t kTW = (uint32_t)BLOCK * W;  // words per tile
  const uint32_t n_tix = MW ? p.n_tiles * p.n_win : p.n_tiles;  // tickets of the launch
  auto loc_of = [&](uint32_t t) -> TileLoc {
    if constexpr (MW) {
      const uint32_t w = t / p.n_tiles;
      return {w, t - w * p.n_tiles};
    } else {
      return {0u, t};
    }
  };
  __shared__ __attribute__((aligned(16))) uint32_t s_park[2][kParkFields][BLOCK][W];
  __shared__ uint32_t s_blk[kRows][17];  // ChaCha12 blocks of the parked tile's draws (+1 word: no conflicts)
  // Broadcast slots written before a barrier and read after it are double-buffered by
  // iteration parity: the next iteration's writes come before ITS barrier, so with one
  // buffer a wave still reading this iteration's value could see them.
  __shared__ uint32_t s_wave[2][WAVES];
  __shared__ unsigned long long s_lb[2][8];  // per-wave look-back result: sum | inclusive << 32 | blocked << 33
  __shared__ uint32_t s_bcast[2][4];        // [0] next ticket, [1] parked tile's prefix (continued look-back)
  Record* rec = p.rec + (p.seq & 1u);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tag_agg = p.seq << 1, tag_inc = tag_agg | 1u;
  const unsigned long long k_base = SHARD ? p.state->shard_draws : p.state->rng_next;  // StdRng position
  // diag & 4: per-workgroup phase times (s_memrealtime, 100 MHz) -> p.dbg[blockIdx.x][12]:
  //   0 start->loop, 1 tally (incl. the round-1 wait), 2 scan barrier, 3 decisions (incl.
  //   the round-2 wait), 4 draws of the parked tile, 5 its stores, 6 loop end->record, 7 iterations,
  //   [8] look-back completion inside the draws, [9] continued look-backs, [10] start, [11] end (absolute),
  //   inside the draws (thread 0): [12] ChaCha blocks, [13] the barrier after them, [14] the selection loop
  // (thread 0 keeps them in LDS: 13 live 64-bit accumulators would cost the loop SGPRs)
  const bool stamps = (p.diag & 4u) != 0 && tid == 0;
  __shared__ unsigned long long s_st[16];  // [0-12] accumulators, [13] last stamp, [14] start
  if (stamps) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 13; k++) s_st[k] = 0;
    s_st[13] = s_st[14] = t0;
  }
  auto lap = [&](int k) {
    if (stamps) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      s_st[k] += t - s_st[13];
      s_st[13] = t;
    }
  };

  // this thread's byte offsets inside a tile's planes; plane strides in bytes
  const uint32_t in_lane = (uint32_t)p.lin.base((uint64_t)tid * W) * 4u;
  const uint32_t out_lane = (uint32_t)p.lout.base((uint64_t)tid * W) * 4u;
  uint32_t in_pb = (uint32_t)p.lin.pstride * 4u, out_pb = (uint32_t)p.lout.pstride * 4u;
  // (MW: window l.w's planes start l.w pitches after window 0's)
  auto in_rsrc = [&](TileLoc l) {
    return plane_rsrc(p.votes + (MW ? (uint64_t)l.w * p.win_in_pitch : 0ull) + p.lin.base((uint64_t)l.c * kTW));
  };
  auto out_rsrc = [&](TileLoc l) {
    return plane_rsrc(p.out + (MW ? (uint64_t)l.w * p.win_out_pitch : 0ull) + p.lout.base((uint64_t)l.c * kTW));
  };
  auto active = [&](TileLoc l) { return (uint64_t)l.c * kTW + (uint64_t)tid * W < p.n_words; };
  // a thread past the window loads its tile's first word (valid; its masks are 0)
  // and its stores go out of range (dropped)
  auto in_off = [&](TileLoc l) { return active(l) ? in_lane : 0u; };
  auto out_off = [&](TileLoc l) { return active(l) ? out_lane : kOffNone; };
  // tickets: c = the tile being tallied (its round-1 planes were loaded during the
  // previous iteration); the ticket after it is requested one iteration ahead
  uint32_t nt = 0;
  if (tid == 0) s_bcast[1][0] = take_ticket(rec);
  lds_barrier();
  uint32_t c = s_bcast[1][0];
  TileLoc cl = loc_of(c < n_tix ? c : 0u);
  if (tid == 0) nt = take_ticket(rec);
  uint32_t r1lo[N][W], r1hi[N][W];
  unsigned long long lbg;  // the look-back poll of the tile parked next (issued before its successor's loads)

  int32_t prev_tile = -1;   // this workgroup's last finished tile (ticket) and its inclusive prefix
  uint32_t prev_incl = 0;
  int32_t park_tile = -1;   // the parked tile (ticket), its VQ total and this thread's offset in it
  TileLoc park_l{0u, 0u};
  uint32_t park_total = 0, park_thr = 0;
  uint32_t pk = 0;          // park buffer of the tile being tallied (the parked tile: pk ^ 1)
  uint32_t a_dec = 0, a_v1 = 0, a_pend = 0, a_draws = 0, a_max1 = 0, a_min = ~0u;  // launch-relative offsets
  // MW: per-tile statistics, one row per wave {dec | v1 << 16, pend, max_off1, min_off} of the
  // tile stored last (by parity), published by wave 0 after the next barrier
  __shared__ uint32_t s_tst[MW ? 2 : 1][MW ? WAVES : 1][4];
  int32_t st_tile = -1;     // the tile whose statistics wait for publication, its draws
  uint32_t st_draws = 0;

  // ---- look-back of the parked tile p: every wave polls 64 predecessor granules
  // (wave w: distances 64w .. 64w + 63 below p; one load per lane, so every wave
  // issues the same memory operations) with the round-1 planes' wait, evaluates them
  // after the tally, and the waves' results combine after the scan barrier.
  // The look-back floor: granules at or below it are known (synthetic). Single window:
  // this workgroup's last finished tile (inclusive). MW: the same if it lies in the
  // parked tile's window, else the ticket before the window's first (a prefix of 0).
  constexpr int kPollWaves = WAVES < 8 ? WAVES : 8;  // 512 granules per poll (waves 8-15 repeat 0-7)
  auto lb_floor = [&]() -> int32_t {
    if constexpr (MW) {
      const int32_t ws = park_tile - (int32_t)park_l.c;
      return prev_tile >= ws ? prev_tile : ws - 1;
    } else {
      return prev_tile;
    }
  };
  auto lb_floor_incl = [&]() -> uint32_t {
    if constexpr (MW) return prev_tile >= park_tile - (int32_t)park_l.c ? prev_incl : 0u;
    else return prev_incl;
  };
  auto lb_poll = [&](int32_t tile) -> unsigned long long {
    const int32_t idx = tile - 1 - (64 * (wave % kPollWaves) + lane);
    return atomic_load_agent(p.lookback + (idx > lb_floor() ? idx : 0));
  };
  auto lb_eval = [&](unsigned long long g) {
    if (wave >= kPollWaves) return;
    const int32_t floor = lb_floor();
    const int32_t idx = park_tile - 1 - (64 * wave + lane);
    const uint32_t tag = (uint32_t)(g >> 32);
    const bool synth = idx <= floor;  // the floor is inclusive (known to this WG)
    const bool ready = synth || (tag >> 1) == p.seq;
    const bool incl = synth || (ready && (tag & 1u));
    const unsigned long long im = __ballot(incl), nr = __ballot(!ready);
    const int f = im ? __builtin_ctzll(im) : 64;
    const unsigned long long need = f >= 63 ? ~0ull : ((2ull << f) - 1ull);
    const uint32_t val = idx == floor ? lb_floor_incl() : (synth ? 0u : (uint32_t)g);
    const uint32_t sum = wave_sum32(lane <= f ? val : 0u);
    if (lane == 0)
      s_lb[pk][wave] = (unsigned long long)sum | ((unsigned long long)(f < 64) << 32) |
                   ((unsigned long long)((nr & need) != 0) << 33);
  };
  // after the barrier (uniform): true and the prefix when the polls reached an inclusive
  auto lb_combine = [&](uint32_t& excl) -> bool {
    excl = 0;
#pragma unroll
    for (int w = 0; w < kPollWaves; w++) {
      const unsigned long long x = s_lb[pk][w];
      if (x >> 33) return false;  // a granule it needs is not published yet
      excl += (uint32_t)x;
      if ((x >> 32) & 1u) return true;
    }
    return false;  // every polled granule was an aggregate: continue further back
  };

  // ChaCha12 blocks cb .. min(cb + kRows, b_last + 1) - 1 into s_blk, block r by the
  // lanes 4r .. 4r + 3 (quad-uniform condition)
  auto chacha_rows = [&](unsigned long long cb, unsigned long long b_last) {
    const uint32_t r = (uint32_t)tid >> 2;
    if (cb + r <= b_last) {
      uint32_t o[4];
      chacha_block_quad<12>(p.key, cb + r, 0, tid & 3, o);
      const int q = tid & 3;
      s_blk[r][q] = o[0];
      s_blk[r][4 + q] = o[1];
      s_blk[r][8 + q] = o[2];
      s_blk[r][12 + q] = o[3];
    }
  };

  // Draws of the parked tile: own round-2 votes of its VQ slots (bits set = V1).
  // (Its ChaCha blocks computed right after the scan barrier instead, while the
  // round-2 planes are in flight: 727 vs 713 us per 2^30 slots, not kept.)
  auto draw_parked = [&](uint32_t (&own)[W]) {
    uint32_t(&pp)[kParkFields][BLOCK][W] = s_park[pk ^ 1u];
    uint32_t excl;
    const bool lb_done = lb_combine(excl);
    if (!lb_done) {  // uniform: the rare continued look-back (wave 0, 256 granules per poll)
      if (wave == 0) {
        const uint32_t e = lag_finish(p.lookback, park_tile - 1 + 64 * kLagPoll, lb_floor(), lb_floor_incl(), p.seq,
                                      lane, 0u, false, &rec->error.v);
        if (lane == 0) s_bcast[pk][1] = e;
      }
      lds_barrier();
      excl = s_bcast[pk][1];
    }
    if (stamps) s_st[9] += lb_done ? 0 : 1;
    lap(8);
    if (tid == 0)
      atomic_store_agent(p.lookback + park_tile, ((unsigned long long)tag_inc << 32) | (excl + park_total));
    prev_tile = park_tile;
    prev_incl = excl + park_total;
    const unsigned long long k_tile = k_base + excl;
#pragma unroll
    for (int i = 0; i < W; i++) own[i] = 0;
    if constexpr (SHARD) {
      // Sharded step: no draws here. Every VQ slot is re-drawn at its global stream
      // position by the fix-up (a provisional draw at this shard's position would be
      // redrawn anyway), so the step takes the LIKELY outcome of the draw as its
      // provisional own vote, deterministically: c1 > c0 -> V1 (the draw gives V1 with
      // p = 0.9), c1 < c0 -> V0 (0.9), tie -> V1 (0.8) (engine.rs:567-611), i.e. own = e0.
      // The fix-up then patches the 10-20 % of VQ slots whose draw disagrees. One record
      // per VQ slot (index = local draw number, ascending slot order): offset, class,
      // the decision under each own vote, the provisional own vote. No ChaCha12 pass and
      // no barrier in the sharded step.
      uint32_t* const vq_reg = p.vq_rec + (MW ? (uint64_t)park_l.w * p.rec_pitch : 0ull);
      {  // the record segment this thread's words start: its first record
        const uint32_t pw = park_l.c * kTW + (uint32_t)tid * W;
        if ((pw & (kRecChunkWords - 1)) == 0 && pw < p.n_words)
          vq_reg[pw / kRecChunkWords] = (uint32_t)(k_tile + park_thr - k_base);
      }
      if (park_total) {
        uint32_t* const vq_rec = vq_reg + p.rec_tw;
        unsigned long long k = k_tile + park_thr;
#pragma unroll
        for (int i = 0; i < W; i++) {
          const uint32_t e0 = pp[2][tid][i], e1 = pp[3][tid][i];
          uint32_t m = e0 | e1;
          own[i] = e0;
          if (!m) continue;
          uint32_t dv[4];
#pragma unroll
          for (int j = 0; j < 4; j++) dv[j] = pp[4 + j][tid][i];
          while (m) {
            const int b = __builtin_ctz(m);
            m &= m - 1;
            const bool x0 = (e0 >> b) & 1u, x1 = (e1 >> b) & 1u;  // gt: 1/0, lt: 0/1, tie: 1/1
            const uint32_t cls = (x0 && !x1) ? kRecGt : ((x1 && !x0) ? kRecLt : 0u);
            const uint32_t d4 = ((dv[0] >> b) & 1u) | (((dv[1] >> b) & 1u) << 1) | (((dv[2] >> b) & 1u) << 2) |
                                (((dv[3] >> b) & 1u) << 3);
            const uint32_t info = cls | (d4 << 2) | ((uint32_t)x0 << 6);
            const unsigned long long kr = k - k_base;
            const uint32_t off = 32u * (park_l.c * kTW + (uint32_t)tid * W + i) + b;  // window-relative
            if (kr < p.vq_cap) vq_rec[kr] = rec_make(off, info);
            k++;
          }
        }
      }
    } else if (park_total) {  // VQ slots whose draw gave V1 (engine.rs:523-537, 567-611)
      uint32_t mq[W];
      {
        uint32_t e0[W], e1[W];
        lds_ld<W>(pp[2][tid], e0);
        lds_ld<W>(pp[3][tid], e1);
#pragma unroll
        for (int i = 0; i < W; i++) mq[i] = e0[i] | e1[i];
      }
      unsigned long long k = k_tile + park_thr;
      const unsigned long long b_first = k_tile >> 3, b_last = (k_tile + park_total - 1) >> 3;
      for (unsigned long long cb = b_first; cb <= b_last; cb += kRows) {
        chacha_rows(cb, b_last);
        lap(10);
        lds_barrier();
        lap(11);
        const unsigned long long k_lim = (cb + kRows) << 3;
#pragma unroll
        for (int i = 0; i < W; i++) {
          if (!mq[i] || k >= k_lim) continue;
          const uint32_t e0 = pp[2][tid][i], e1 = pp[3][tid][i];
          while (mq[i] && k < k_lim) {
            const int b = __builtin_ctz(mq[i]);
            mq[i] &= mq[i] - 1;
            const uint32_t row = (uint32_t)((k >> 3) - cb), ws = (uint32_t)(k & 7u) * 2u;
            const unsigned long long u =
                (unsigned long long)s_blk[row][ws] | ((unsigned long long)s_blk[row][ws + 1] << 32);
            const bool x0 = (e0 >> b) & 1u, x1 = (e1 >> b) & 1u;  // gt: 1/0, lt: 0/1, tie: 1/1
            const bool v1 = (x0 && !x1) ? (u < kP90) : ((x1 && !x0) ? (u >= kP90) : (u < kP80));
            own[i] |= (uint32_t)v1 << b;
            k++;
          }
        }
        lap(12);
        // only between passes: after the last one the next iteration's scan barrier
        // orders these reads before the next writes of s_blk (686.5 -> 670.9 us per
        // 2^30 slots, interleaved A/B)
        if (cb + kRows <= b_last) lds_barrier();
      }
    }
  };

  // Decisions, stores and statistics of the parked tile (after draw_parked). Every
  // lane stores (a lane past the window out of range): no branch between the plane
  // loads in flight and their use.
  // Without a parked tile (a workgroup's first iteration) it issues the same stores
  // out of range and counts nothing: every path into the next tally then has the
  // same memory operations in flight behind the round-1 loads.
  auto store_parked = [&](const uint32_t (&own)[W], bool have_park) {
    uint32_t(&pp)[kParkFields][BLOCK][W] = s_park[pk ^ 1u];
    const TileLoc pl = have_park ? park_l : TileLoc{0u, 0u};
    const uint32_t pw0 = pl.c * kTW + (uint32_t)tid * W;  // window-relative word of this thread
    const __amdgpu_buffer_rsrc_t orr = out_rsrc(pl);
    const uint32_t oo = have_park ? out_off(pl) : kOffNone;
    {  // plane 2: own round-2 vote lo
      uint32_t v[W];
      lds_ld<W>(pp[0][tid], v);
#pragma unroll
      for (int i = 0; i < W; i++) v[i] |= own[i];
      buf_st<W>(orr, oo, 2 * out_pb, v);
    }
    uint32_t dlo[W], dhi[W];  // own vote joins round2_votes (engine.rs:540-542); decision (613-628)
    {
      uint32_t alo[W], ahi[W], blo[W], bhi[W];
      lds_ld<W>(pp[4][tid], alo);
      lds_ld<W>(pp[5][tid], ahi);
      lds_ld<W>(pp[6][tid], blo);
      lds_ld<W>(pp[7][tid], bhi);
#pragma unroll
      for (int i = 0; i < W; i++) {
        dlo[i] = (alo[i] & ~own[i]) | (blo[i] & own[i]);
        dhi[i] = (ahi[i] & ~own[i]) | (bhi[i] & own[i]);
      }
    }
    buf_st<W>(orr, oo, 4 * out_pb, dlo);
    buf_st<W>(orr, oo, 5 * out_pb, dhi);
    uint32_t keep[W];  // SHARD: VQ slots are counted by the fix-up
#pragma unroll
    for (int i = 0; i < W; i++) keep[i] = have_park ? ~0u : 0u;
    if constexpr (SHARD) {
      uint32_t e0[W], e1[W];
      lds_ld<W>(pp[2][tid], e0);
      lds_ld<W>(pp[3][tid], e1);
#pragma unroll
      for (int i = 0; i < W; i++) keep[i] &= ~(e0[i] | e1[i]);
    }
    // slot offset of this thread's first word: launch-relative (one window), tile-relative (MW)
    const uint32_t toff = 32u * (MW ? (uint32_t)tid * W : pw0);
    const uint64_t sbase = MW ? p.slot_base + (uint64_t)pl.w * p.win_id_stride : p.slot_base;
    uint32_t t_dec = 0, t_v1 = 0, t_max1 = 0, t_min = ~0u;
#pragma unroll
    for (int i = 0; i < W; i++) {
      const uint32_t vm = valid_mask(pw0 + i, p.n_words, p.n_slots);
      const uint32_t pdec = ~dhi[i] & vm;    // committed iff not VQuestion
      const uint32_t pv1 = dlo[i] & ~dhi[i];  // V1: apply_batch + commit_phase
      dlo[i] = pdec;
      dhi[i] = pv1;
      const uint32_t cd = pdec & keep[i], c1 = pv1 & keep[i];
      t_dec += __builtin_popcount(cd);
      t_v1 += __builtin_popcount(c1);
      const uint32_t m1 = c1 & phase_limit_mask(sbase, pw0 + i, p.max_phase);
      const uint32_t o1 = m1 ? toff + 32u * i + (31u - __builtin_clz(m1)) + 1u : 0u;
      t_max1 = o1 > t_max1 ? o1 : t_max1;
      const uint32_t und = ~pdec & vm & keep[i];
      const uint32_t o0 = und ? toff + 32u * i + __builtin_ctz(und) : ~0u;
      t_min = o0 < t_min ? o0 : t_min;
    }
    buf_st<W>(orr, oo, 6 * out_pb, dlo);
    buf_st<W>(orr, oo, 7 * out_pb, dhi);
    if constexpr (MW) {
      // the tile's row per wave: sums by DPP, the extremes from the highest / lowest lane
      // holding one (threads own ascending words of the tile); pend recounted from the
      // parked pending plane (the tally counted it into no accumulator)
      if (have_park) {
        uint32_t pd[W], t_pend = 0;
        lds_ld<W>(pp[1][tid], pd);
#pragma unroll
        for (int i = 0; i < W; i++) t_pend += __builtin_popcount(pd[i]);
        const uint32_t s0 = wave_sum32(t_dec | (t_v1 << 16)), s1 = wave_sum32(t_pend);
        const unsigned long long hmx = __ballot(t_max1 != 0u), hmn = __ballot(t_min != ~0u);
        const uint32_t mx = hmx ? __builtin_amdgcn_readlane(t_max1, 63 - __builtin_clzll(hmx)) : 0u;
        const uint32_t mn = hmn ? __builtin_amdgcn_readlane(t_min, __builtin_ctzll(hmn)) : ~0u;
        if (lane == 0) {
          s_tst[pk][wave][0] = s0;
          s_tst[pk][wave][1] = s1;
          s_tst[pk][wave][2] = mx;
          s_tst[pk][wave][3] = mn;
        }
        st_tile = park_tile;
        st_draws = park_total;
      }
    } else {
      a_dec += t_dec;
      a_v1 += t_v1;
      a_max1 = t_max1 > a_max1 ? t_max1 : a_max1;
      a_min = t_min < a_min ? t_min : a_min;
    }
  };

  // MW: wave 0 publishes the statistics of tile st_tile from row buffer `buf` (after a
  // barrier that follows their writes) as the two tagged granules of finish_tile.
  auto publish_tile_stats = [&](uint32_t buf) {
    if constexpr (MW) {
      if (wave != 0 || st_tile < 0) return;
      const bool have = lane < WAVES;
      uint32_t x0 = 0, x1 = 0, mx = 0, mn = ~0u;
      if (have) {
        x0 = s_tst[buf][lane][0];
        x1 = s_tst[buf][lane][1];
        mx = s_tst[buf][lane][2];
        mn = s_tst[buf][lane][3];
      }
      const uint32_t dec_v1_lo = wave_sum32(x0 & 0xFFFFu), v1 = wave_sum32(x0 >> 16), pend = wave_sum32(x1);
      const unsigned long long hmx = __ballot(mx != 0u), hmn = __ballot(mn != ~0u);
      const uint32_t bmx = hmx ? __builtin_amdgcn_readlane(mx, 63 - __builtin_clzll(hmx)) : 0u;
      const uint32_t bmn = hmn ? __builtin_amdgcn_readlane(mn, __builtin_ctzll(hmn)) : kStatNone;
      if (lane == 0) {
        const unsigned long long tag = stat_tag(p.seq);
        unsigned long long* g = p.stats + (uint64_t)st_tile * kStatGranules;
        atomic_store_agent(g + 0, tag | ((unsigned long long)pend << 34) | ((unsigned long long)v1 << 17) | dec_v1_lo);
        atomic_store_agent(g + 1, tag | ((unsigned long long)bmn << 34) | ((unsigned long long)bmx << 17) | st_draws);
      }
      st_tile = -1;
    } else {
      (void)buf;
    }
  };

  // Software pipeline. Tile c's round-1 planes (r1) were issued right after the
  // previous tile's tally and its round-2 planes (r2) right after the previous
  // tile's decisions, so one tile of planes is in flight through the whole
  // iteration. The vector memory counter retires in issue order and every operation
  // below is issued on every path (dummy loads past the last tile, out-of-range
  // stores without a parked tile), so the compiler's waits count exactly:
  //   tally(c) <- r1  | early stores | look-back eval (poll of the last iteration)
  //   | scan barrier | r1 <- next | decisions(c) <- r2 | r2 <- next | park c
  //   | draws + stores of the parked tile | poll for c
  uint32_t r2lo[N][W], r2hi[N][W];
  {  // in the order the loop leaves them: r1, r2, five stores (here out of range), poll
    const bool any = c < n_tix;  // (cl: the tile of c, or tile 0 without one)
    const uint32_t voff0 = any ? in_off(cl) : 0u;
    buf_ld_planes<N, W>(in_rsrc(cl), voff0, in_pb, 0, r1lo, r1hi);
    // every round-1 load before the first round-2 load, as the loop issues them: the
    // compiler's vmcnt wait at the loop head is the minimum over the paths into it, and
    // with the two groups interleaved here the tally waited for the round-2 planes too
    // (vmcnt(7) instead of vmcnt(16) at n = 5)
    __builtin_amdgcn_sched_barrier(0);
    buf_ld_planes<N, W>(in_rsrc(cl), voff0, in_pb, 2 * N, r2lo, r2hi);
    const uint32_t z[W] = {};
    const __amdgpu_buffer_rsrc_t orr = out_rsrc(TileLoc{0u, 0u});
#pragma unroll
    for (int k = 0; k < 5; k++) buf_st<W>(orr, kOffNone, (uint32_t)k * 4u, z);
    lbg = lb_poll(park_tile);  // no parked tile yet: a harmless poll
  }
  lap(0);
  while (c < n_tix) {
    // opaque per iteration: the 28 plane offsets (k * stride) are recomputed by SALU
    // next to their loads and stores instead of living in SGPRs across the loop
    asm volatile("" : "+s"(in_pb), "+s"(out_pb));
    const bool have_park = park_tile >= 0;
    uint32_t(&pc)[kParkFields][BLOCK][W] = s_park[pk];
    // (1) round 1 of tile c: count_votes + |votes| >= quorum fallback (engine.rs:495-505);
    //     the round-1-only output planes (final already) and the tile's state to LDS
    const uint32_t w0 = cl.c * kTW + (uint32_t)tid * W;  // window-relative
    uint32_t vq_count = 0;
    {
      uint32_t v1[W], vq[W], pd[W], e0[W], e1[W];
      uint32_t seq0 = 0;  // a zero the compiler cannot see through: the words tally one after another
#pragma unroll
      for (int i = 0; i < W; i++) {
        const uint32_t vm = valid_mask(w0 + i, p.n_words, p.n_slots);
        uint32_t m0[N], m1[N], mp[N];
#pragma unroll
        for (int j = 0; j < N; j++) {
          const uint32_t lo = r1lo[j][i], hi = r1hi[j][i];
          m0[j] = ~lo & ~hi;
          m1[j] = lo & ~hi;
          mp[j] = ~(lo & hi);
        }
        m0[0] |= seq0; m1[0] |= seq0; mp[0] |= seq0;  // (a zero: the words tally one after another)
        const Ctr<B> c0 = ctr_count<N>(m0), c1 = ctr_count<N>(m1), cp = ctr_count<N>(mp);
        const uint32_t g0 = ctr_ge(c0, p.q), g1 = ctr_ge(c1, p.q), gp = ctr_ge(cp, p.q);
        const uint32_t x0 = g0 & vm;
        v1[i] = ~g0 & g1 & vm;
        vq[i] = ~g0 & ~g1 & gp & vm;  // cq >= q implies present >= q
        pd[i] = ~(x0 | v1[i] | vq[i]) & vm;
        uint32_t gt, lt;
        ctr_cmp(c1, c0, gt, lt);
        e0[i] = vq[i] & ~lt;
        e1[i] = vq[i] & ~gt;
        vq_count += __builtin_popcount(vq[i]);
        a_pend += __builtin_popcount(pd[i]);
        asm volatile("" : "+v"(seq0), "+v"(v1[i]), "+v"(vq[i]), "+v"(pd[i]));
      }
      uint32_t x[W];
#pragma unroll
      for (int i = 0; i < W; i++) x[i] = v1[i] | pd[i];
      lds_st<W>(pc[0][tid], x);
      lds_st<W>(pc[1][tid], pd);
      lds_st<W>(pc[2][tid], e0);
      lds_st<W>(pc[3][tid], e1);
      const __amdgpu_buffer_rsrc_t orr = out_rsrc(cl);
      const uint32_t oo = out_off(cl);
      buf_st<W>(orr, oo, 0, x);
#pragma unroll
      for (int i = 0; i < W; i++) x[i] = vq[i] | pd[i];
      buf_st<W>(orr, oo, out_pb, x);
      buf_st<W>(orr, oo, 3 * out_pb, pd);
    }
    lb_eval(lbg);
    lap(1);
    // (2) VQ prefix inside the tile; publish the tile's aggregate; the next tickets
    const uint32_t incl = wave_incl_scan32(vq_count, lane);
    if (lane == 63) s_wave[pk][wave] = incl;
    if (tid == 0) s_bcast[pk][0] = nt;
    lds_barrier();
    uint32_t wave_off = 0, total = 0;
    {
      const uint32_t sw = lane < WAVES ? s_wave[pk][lane] : 0u;
      const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
      for (int w = 0; w < WAVES; w++) {
        const uint32_t x = __builtin_amdgcn_readlane(sw, w);
        wave_off += (w < wv) ? x : 0u;
        total += x;
      }
    }
    const uint32_t nx = s_bcast[pk][0];
    lap(2);
    if (tid == 0) {  // (a window's first tile starts its chain: inclusive)
      atomic_store_agent(p.lookback + c, ((unsigned long long)(cl.c == 0 ? tag_inc : tag_agg) << 32) | total);
      if (nx < n_tix) nt = take_ticket(rec);
    }
    publish_tile_stats(pk ^ 1u);  // MW: the tile stored in the last iteration

    // (3) the next tile's round-1 planes in flight (past the last tile: tile c's first word)
    const bool more = nx < n_tix;
    const TileLoc nl = more ? loc_of(nx) : cl;
    const __amdgpu_buffer_rsrc_t nrr = in_rsrc(nl);
    const uint32_t noff = more ? in_off(nl) : 0u;
    buf_ld_planes<N, W>(nrr, noff, in_pb, 0, r1lo, r1hi);
    // (4) round-2 decisions of tile c for both own votes (engine.rs:540-542, 613-628);
    //     then the next tile's round-2 planes in flight
    {
      uint32_t x[W], pd[W], e0[W], e1[W];
      lds_ld<W>(pc[0][tid], x);
      lds_ld<W>(pc[1][tid], pd);
      lds_ld<W>(pc[2][tid], e0);
      lds_ld<W>(pc[3][tid], e1);
      uint32_t alo[W], ahi[W], blo[W], bhi[W];
#pragma unroll
      for (int i = 0; i < W; i++) {
        r2_decision_ab<N, W>(r2lo, r2hi, i, p.q, p.self_lane, x[i] & ~pd[i], e0[i] | e1[i], pd[i], alo[i], ahi[i],
                             blo[i], bhi[i]);
        const uint32_t vm = valid_mask(w0 + i, p.n_words, p.n_slots);
        alo[i] &= vm; ahi[i] &= vm; blo[i] &= vm; bhi[i] &= vm;
      }
      buf_ld_planes<N, W>(nrr, noff, in_pb, 2 * N, r2lo, r2hi);
      lds_st<W>(pc[4][tid], alo);
      lds_st<W>(pc[5][tid], ahi);
      lds_st<W>(pc[6][tid], blo);
      lds_st<W>(pc[7][tid], bhi);
    }
    lap(3);
    // (5) the parked tile: draws, decisions, stores
    uint32_t own[W] = {};
    if (have_park) draw_parked(own);
    lap(4);
    store_parked(own, have_park);
    lap(5);
    if (stamps) s_st[7]++;
    a_draws += vq_count;
    park_tile = (int32_t)c;  // tile c is parked; its look-back poll (prev_tile: the tile just finished)
    park_l = cl;
    park_total = total;
    park_thr = wave_off + incl - vq_count;
    lbg = lb_poll(park_tile);  // (issued ahead of the next round-2 loads instead: 877 vs 705 us per 2^30
                               // slots, its predecessors not yet published: continued look-backs)
    pk ^= 1u;
    c = nx;
    cl = nl;
  }
  if (park_tile >= 0) {  // the last parked tile (its poll went out in the last iteration)
    lb_eval(lbg);
    lds_barrier();
    publish_tile_stats(pk ^ 1u);  // MW: the tile stored in the last iteration
    uint32_t own[W];
    draw_parked(own);
    store_parked(own, true);
    if constexpr (MW) {
      lds_barrier();
      publish_tile_stats(pk);
    }
  }

  if constexpr (MW) {  // arrival; the last workgroup folds every window's tile granules
    __shared__ uint32_t s_last_mw;
    if (stamps) {
      lap(6);
      for (int k = 0; k < 10; k++) p.dbg[(uint64_t)blockIdx.x * 16 + k] = s_st[k];
    }
    if (tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's granules are out
      const unsigned long long arrived = atomicAdd(&rec->done.v, 1ull);
      s_last_mw = arrived == gridDim.x - 1 ? 1u : 0u;
    }
    lds_barrier();
    if (!s_last_mw) return;
    lag_fold_windows<WAVES, kTW * 32u>(p, rec, lane, wave);
    if (tid == 0) {
      Record* nxt = p.rec + ((p.seq + 1) & 1u);  // the next launch's record (the previous launch completed)
      atomic_store_agent(&nxt->error.v, 0ull);
      atomic_store_agent(&nxt->ticket.v, 0ull);
      atomic_store_agent(&nxt->done.v, 0ull);
    }
    return;
  }

  // ---- per-workgroup record; the last workgroup to arrive folds them all
  {
    __shared__ unsigned long long red[WAVES][4];
    __shared__ uint32_t s_last;
    const unsigned long long s0 = wave_sum64((unsigned long long)a_dec | ((unsigned long long)a_v1 << 32));
    const unsigned long long s1 = wave_sum64((unsigned long long)a_pend | ((unsigned long long)a_draws << 32));
    const uint32_t mx = wave_max32(a_max1), mn = wave_min32(a_min);
    if (lane == 0) { red[wave][0] = s0; red[wave][1] = s1; red[wave][2] = mx; red[wave][3] = mn; }
    lds_barrier();
    if (stamps) {
      lap(6);
      for (int k = 0; k < 10; k++) p.dbg[(uint64_t)blockIdx.x * 16 + k] = s_st[k];
      p.dbg[(uint64_t)blockIdx.x * 16 + 10] = s_st[14];
      p.dbg[(uint64_t)blockIdx.x * 16 + 11] = s_st[13];
      for (int k = 10; k < 13; k++) p.dbg[(uint64_t)blockIdx.x * 16 + k + 2] = s_st[k];
    }
    if (tid == 0) {
      unsigned long long t[kLagStatGranules] = {0, 0, 0, 0, 0, 0xFFFFFFFFull};
#pragma unroll 1
      for (int w = 0; w < WAVES; w++) {
        t[0] += red[w][0] & 0xFFFFFFFFull; t[1] += red[w][0] >> 32;
        t[2] += red[w][1] & 0xFFFFFFFFull; t[3] += red[w][1] >> 32;
        t[4] = red[w][2] > t[4] ? red[w][2] : t[4];
        t[5] = red[w][3] < t[5] ? red[w][3] : t[5];
      }
      const unsigned long long tag = stat_tag(p.seq);
      unsigned long long* gr = p.stats + (uint64_t)blockIdx.x * kLagStatGranules;
#pragma unroll
      for (int k = 0; k < kLagStatGranules; k++) atomic_store_agent(gr + k, tag | t[k]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long arrived = atomicAdd(&rec->done.v, 1ull);
      s_last = arrived == gridDim.x - 1 ? 1u : 0u;
    }
    lds_barrier();
    if (!s_last) return;
  }
  unsigned long long v[7] = {0, 0, 0, 0, 0, ~0ull, 0};  // dec v1 pend draws max(id+1) min(id) fault
  constexpr unsigned long long kTagMask = ~0ull << 51;
  const unsigned long long tag = stat_tag(p.seq);
  for (uint32_t g = tid; g < gridDim.x; g += BLOCK) {
    const unsigned long long* gr = p.stats + (uint64_t)g * kLagStatGranules;
    unsigned long long x[kLagStatGranules];
#pragma unroll
    for (int k = 0; k < kLagStatGranules; k++) x[k] = atomic_load_agent(const_cast<unsigned long long*>(gr) + k);
    SpinBound spin;
    for (;;) {  // visible already (arrival counter): a guard, not a wait
      bool ok = true;
#pragma unroll
      for (int k = 0; k < kLagStatGranules; k++) ok &= (x[k] & kTagMask) == tag;
      if (ok) break;
      if (spin.expired()) { v[6] = 2; break; }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int k = 0; k < kLagStatGranules; k++) x[k] = atomic_load_agent(const_cast<unsigned long long*>(gr) + k);
    }
#pragma unroll
    for (int k = 0; k < kLagStatGranules; k++) x[k] &= ~kTagMask;
    v[0] += x[0]; v[1] += x[1]; v[2] += x[2]; v[3] += x[3];
    if (x[4] && p.slot_base + x[4] > v[4]) v[4] = p.slot_base + x[4];
    if (x[5] != 0xFFFFFFFFull && p.slot_base + x[5] < v[5]) v[5] = p.slot_base + x[5];
  }
  block_reduce_totals<BLOCK>(v, lane, wave);
  if (tid != 0) return;
  Record* nxt = p.rec + ((p.seq + 1) & 1u);  // the next launch's record (the previous launch completed)
  atomic_store_agent(&nxt->error.v, 0ull);
  atomic_store_agent(&nxt->ticket.v, 0ull);
  atomic_store_agent(&nxt->done.v, 0ull);
  step_commit<SHARD ? kFinShard : kFinRef>(p, v, *p.state, atomicAdd(&rec->error.v, 0ull));
}

// ============================================================================
// Sharded REF: one engine (one StdRng stream) over a window split into
// contiguous shards, one per GPU. Draw k of shard r sits at global
// stream position  rng_next(window start) + VQ slots of shards 0..r-1 + k
// (ascending slot order over the whole window, engine.rs:567-611). The step ran
// with a provisional position; the fix-up re-draws every VQ slot of the shard at
// its global position from its draw record, XOR-patches the output bits that
// change (own round-2 vote; decision, committed, V1 planes) and counts the VQ
// slots into the shard's statistics. One thread per ChaCha12 block (8 draws),
// grid-stride; one atomic per changed (plane, word) run of a thread.
// ============================================================================
// Statistics partials: (sum, sum, max, min) quadruples, one per workgroup.
// fold4: element j of the 4 waves' values in red[wave][j];
// fold_partials: n quadruples at acc folded by one 256-thread block (result in thread 0's a).
__device__ __forceinline__ unsigned long long fold4(const unsigned long long (&red)[4][4], int j) {
  unsigned long long x = red[0][j];
  for (int w = 1; w < 4; w++) {
    const unsigned long long y = red[w][j];
    x = j < 2 ? x + y : (j == 2 ? (y > x ? y : x) : (y < x ? y : x));
  }
  return x;
}
template <int U = 8>  // U quadruples per thread in flight at once
__device__ __forceinline__ void fold_partials(const unsigned long long* acc, uint32_t n, unsigned long long (&red)[4][4],
                                              unsigned long long (&a)[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a[0] = 0; a[1] = 0; a[2] = 0; a[3] = ~0ull;
  for (uint32_t b0 = threadIdx.x; b0 < n; b0 += 256 * U) {
    unsigned long long x[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t b = b0 + 256u * u;
#pragma unroll
      for (int j = 0; j < 4; j++) x[u][j] = b < n ? acc[(uint64_t)b * 4 + j] : (j == 3 ? ~0ull : 0ull);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      a[0] += x[u][0];
      a[1] += x[u][1];
      a[2] = x[u][2] > a[2] ? x[u][2] : a[2];
      a[3] = x[u][3] < a[3] ? x[u][3] : a[3];
    }
  }
  a[0] = wave_sum64(a[0]);
  a[1] = wave_sum64(a[1]);
  a[2] = wave_max64(a[2]);
  a[3] = wave_min64(a[3]);
  if (lane == 0) for (int j = 0; j < 4; j++) red[wave][j] = a[j];
  __syncthreads();
  for (int j = 0; j < 4; j++) a[j] = fold4(red, j);
  __syncthreads();  // red may be rewritten by the caller's next fold
}

struct FixParams {
  const uint32_t* rec;            // the step's record region (chunk table, then [vq_cap] records)
  const DevResult* rows;          // [n_shards] step rows of every shard, rank order
  uint32_t shard, n_shards;
  DevState* state;
  uint32_t* out;
  Layout lout;
  uint64_t slot_base, max_phase, vq_cap;
  Key key;
  // per-workgroup partials [n_win][n_part][4]: decided, V1, max V1 id + 1, min undecided
  // id (folded by the finish kernel: one same-address atomic per workgroup serialises
  // at one memory channel, 4 x 4096 of them cost ~200 us per 2^30-slot fix-up)
  unsigned long long* acc;
  uint32_t n_part;
  // n_win windows (grid.y): window w's outputs at out + w * out_pitch, slot ids + w *
  // id_stride, record region + w * rec_pitch; rows [n_shards][n_win] (rank-major, as an
  // all-gather of every shard's n_win rows lays them out)
  uint32_t n_win;
  uint64_t out_pitch, id_stride;
  uint64_t n_slots, n_words;      // per window
  uint64_t rec_pitch;             // words per window record region
  uint32_t rec_tw;                // chunk-table words
};

// Sum of one 64-bit value per thread over a 256-thread workgroup, returned to every
// thread (red: 4 LDS words; the trailing barrier lets the caller reuse them).
__device__ __forceinline__ unsigned long long block_sum256(unsigned long long v, unsigned long long* red) {
  v = wave_sum64(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return v;
}

// Global stream position of local draw 0 of window w of shard f.shard: the engine
// position at the first window + every shard's draws of the earlier windows + the
// lower shards' draws of window w (ascending slot order, engine.rs:567-611). Summed by
// the whole workgroup, one row per thread: round 5 ran it as a chain of n_shards x w
// dependent scalar loads in every thread (256 at the 8-GPU C5 shape, 32 windows), which
// was most of the fix-up's time there.
__device__ __forceinline__ unsigned long long fix_first_draw(const FixParams& f, uint32_t w, unsigned long long* red) {
  unsigned long long pre = 0;
  const uint64_t n_rows = (uint64_t)f.n_shards * f.n_win;
  for (uint64_t i = threadIdx.x; i < n_rows; i += 256) {
    const uint32_t r = (uint32_t)(i / f.n_win), v = (uint32_t)(i % f.n_win);
    if (v < w || (v == w && r < f.shard)) pre += f.rows[i].n_draws;
  }
  return f.state->rng_next + block_sum256(pre, red);
}

// The fix-up, one thread per ChaCha12 block of the window's global draw positions
// (grid-stride): the thread loads the (up to) 8 records whose draws the block holds
// (records are indexed by local draw number, so block b holds records 8b - g0 ..
// 8b + 7 - g0), re-draws their VQ slots, counts them into the statistics and
// XOR-patches the own-vote bits that change, one atomic per changed word of its run
// (records are in slot order: a block's changes fall in a few neighbouring words), and
// the rare decision changes (the own vote decides the round-2 count). Every lane works
// on a block of its own, so no lane idles on a partial pass; the statistics are one
// partial per workgroup. Records are 4 B with segment-relative offsets (rg_common.h):
// the workgroup stages the window's segment table in LDS and each thread finds its first
// record's segment by binary search there, then walks forward.
// (Round 6 also tried a fix-up that writes plane 2 whole, one workgroup per 2^15-slot
// chunk, so the step could skip its plane-2 store: fewer bytes on paper, but its per-chunk
// barriers kept it resident beside the whole next step kernel: 0.780 vs 0.732 ms per
// C2 step, profiles/r06/c2_sharded_chunk_fixup_kernel_stats.csv. Not kept.)
#ifndef RG_FIX_GRID
#define RG_FIX_GRID 2048
#endif
constexpr uint32_t kFixGrid = RG_FIX_GRID;  // fix-up workgroups at most, all windows (grid-stride beyond)
// The exchange-stage kernels (fix-up, finish, commit, decision lists) run on a second
// stream while the NEXT step's persistent lag kernel holds every CU: one 512-thread
// workgroup per CU at 2 waves per SIMD, 232 VGPRs each at n = 9 (168 at n = 5) and 129 KB
// of LDS. A wave of these kernels fits beside it only within the 48 VGPRs per SIMD that
// leaves; above that it cannot be placed before the lag kernel ends, so every kernel of
// the exchange chain waited a whole step kernel (round 5: the finish kernel's 266 us).
// So: the exchange kernels at <= 64 VGPRs (8 waves per SIMD, the hardware's maximum, is
// the lowest budget the compiler takes), and the lag kernel at <= 224 (RG_LAG_REGS).
constexpr uint32_t kRecSegMax = 264;  // segment-table words staged in LDS (windows < 2^32 slots)
#ifndef RG_FIX_RECS
#define RG_FIX_RECS 2
#endif
static __global__ __launch_bounds__(256, 8) void shard_fixup_kernel(FixParams f) {
  __shared__ unsigned long long sred[4];
  __shared__ uint32_t s_seg[kRecSegMax];
  const uint32_t win = blockIdx.y;
  const unsigned long long n = f.rows[(uint64_t)f.shard * f.n_win + win].n_draws;
  const unsigned long long g0 = fix_first_draw(f, win, sred);  // global position of local draw 0
  if (win) {  // this window's outputs, slot ids, records
    f.out += win * f.out_pitch;
    f.slot_base += win * f.id_stride;
    f.rec += win * f.rec_pitch;
  }
  const unsigned long long nn = n < f.vq_cap ? n : f.vq_cap;
  const uint32_t n_seg = (uint32_t)rec_chunks(f.n_slots);
  for (uint32_t i = threadIdx.x; i < n_seg; i += 256) s_seg[i] = f.rec[i];
  __syncthreads();
  const uint32_t* recs = f.rec + f.rec_tw;
  // per-thread statistics in 32 bits (window-relative offsets: max V1 offset + 1, min
  // undecided offset), widened for the workgroup fold
  uint32_t dec = 0, v1 = 0, mx = 0, mn = ~0u;
  const uint64_t lim = f.max_phase == 0 ? ~0ull : (f.max_phase >= f.slot_base ? f.max_phase - f.slot_base : 0);
  const bool any_in = f.max_phase == 0 || f.max_phase >= f.slot_base;  // some slot id <= max_phase
  uint32_t* p2 = f.out + 2 * f.lout.pstride;
  const unsigned long long b_end = (g0 + nn + 7) >> 3;
  for (unsigned long long b = (g0 >> 3) + (unsigned long long)blockIdx.x * 256 + threadIdx.x; nn && b < b_end;
       b += (unsigned long long)gridDim.x * 256) {
    const long long k0 = (long long)(b << 3) - (long long)g0;  // local index of the block's first draw
    // the block first, then the records: the ChaCha state and the 8 records are never live
    // together, so the kernel fits the 64 VGPRs it may take beside the next step's lag kernel
    // the segment of the block's first record: the last segment whose first record <= it
    uint32_t seg = 0;
    {
      const uint32_t kf = k0 > 0 ? (uint32_t)k0 : 0u;
      uint32_t lo = 0, hi = n_seg;  // s_seg[lo] <= kf (s_seg[0] = 0)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_seg[mid] <= kf) lo = mid; else hi = mid;
      }
      seg = lo;
    }
    uint32_t seg_end = seg + 1 < n_seg ? s_seg[seg + 1] : ~0u;  // first record of the next segment
    uint32_t x[16];
    chacha_block<12>(f.key, b, 0, x);
    uint32_t cur_w = ~0u, cur_m = 0;  // the run's word being patched and its XOR mask
    const bool whole = k0 >= 0 && (unsigned long long)k0 + 8 <= nn;  // all but the ends
    constexpr int kFR = RG_FIX_RECS;  // records per batch (register budget)
#pragma unroll
    for (int h = 0; h < 8 / kFR; h++) {
      uint32_t rr[kFR];
#pragma unroll
      for (int jj = 0; jj < kFR; jj++) {
        const long long k = k0 + kFR * h + jj;
        rr[jj] = (whole || (k >= 0 && (unsigned long long)k < nn)) ? recs[k] : kRecNone;
      }
#pragma unroll
      for (int jj = 0; jj < kFR; jj++) {
        const int j = kFR * h + jj;
        const uint32_t r = rr[jj];
        if (r == kRecNone) continue;
        const uint32_t kk = (uint32_t)(k0 + j);
        while (kk >= seg_end) {  // (records ascend: the walk only moves up; rare)
          seg++;
          seg_end = seg + 1 < n_seg ? s_seg[seg + 1] : ~0u;
        }
        const uint32_t off = (seg << kRecChunkShift) | (r & ((1u << kRecChunkShift) - 1u)), info = r >> kRecChunkShift;
        const unsigned long long u = (unsigned long long)x[2 * j] | ((unsigned long long)x[2 * j + 1] << 32);
        const uint32_t cls = info & 3u;
        const uint32_t own = cls == kRecGt ? (u < kP90) : (cls == kRecLt ? (u >= kP90) : (u < kP80));
        const uint32_t prov = (info >> 6) & 1u;
        const uint32_t d = own ? (info >> 4) & 3u : (info >> 2) & 3u;
        if (d <= kCodeV1) {
          dec++;
          if (d == kCodeV1) {
            v1++;
            if (any_in && off <= lim && off + 1 > mx) mx = off + 1;
          }
        } else if (off < mn) {
          mn = off;
        }
        if (own != prov) {
          const uint32_t w = off >> 5, bit = 1u << (off & 31u);
          if (w != cur_w) {
            if (cur_m) atomicXor(p2 + f.lout.base(cur_w), cur_m);
            cur_w = w;
            cur_m = 0;
          }
          cur_m ^= bit;
          const uint32_t dp = prov ? (info >> 4) & 3u : (info >> 2) & 3u;
          const uint32_t dd = d ^ dp;
          if (dd || (d <= kCodeV1) != (dp <= kCodeV1)) {  // the decision changed: rare
            const uint64_t base = f.lout.base(w);
            if (dd & 1u) atomicXor(f.out + base + 4 * f.lout.pstride, bit);
            if (dd & 2u) atomicXor(f.out + base + 5 * f.lout.pstride, bit);
            if ((d <= kCodeV1) != (dp <= kCodeV1)) atomicXor(f.out + base + 6 * f.lout.pstride, bit);
            if ((d == kCodeV1) != (dp == kCodeV1)) atomicXor(f.out + base + 7 * f.lout.pstride, bit);
          }
        }
      }
    }
    if (cur_m) atomicXor(p2 + f.lout.base(cur_w), cur_m);
  }
  __shared__ unsigned long long red[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long dsum = wave_sum64(dec), vsum = wave_sum64(v1);
  const unsigned long long mxx = wave_max64(mx ? f.slot_base + mx : 0ull);  // max V1 id + 1
  const unsigned long long mnn = wave_min64(mn != ~0u ? f.slot_base + mn : ~0ull);
  if (lane == 0) { red[wave][0] = dsum; red[wave][1] = vsum; red[wave][2] = mxx; red[wave][3] = mnn; }
  __syncthreads();
  // every workgroup writes its partial (zeros / all ones when it had no records)
  if (threadIdx.x < 4) f.acc[((uint64_t)win * f.n_part + blockIdx.x) * 4 + threadIdx.x] = fold4(red, threadIdx.x);
}


// The shard's final rows: VQ-slot counts and extremes folded in, the engine's stream
// position advanced past the whole window's draws (every shard's). One workgroup per
// window (round 5 folded the windows one after another in one workgroup: 266 us at the
// 8-GPU C5 shape, 32 windows, longer than the step kernel): window w's partials, and
// its position = the engine position + every shard's draws of windows 0..w. The
// context's rng_next is read by every workgroup and written by the last to arrive.
static __global__ __launch_bounds__(256, 8) void shard_fixup_finish_kernel(FixParams f, DevResult* row_ctx,
                                                                        DevResult* row_user, unsigned int* arrivals) {
  __shared__ unsigned long long red[4][4];
  __shared__ unsigned long long sred[4];
  const uint32_t w = blockIdx.x;
  unsigned long long a[4];  // the window's workgroup partials (shard_fixup_kernel)
  fold_partials<2>(f.acc + (uint64_t)w * f.n_part * 4, f.n_part, red, a);  // <= 2 x 256 partials per window
  unsigned long long upto = 0, all = 0;  // draws of windows <= w, of every window (every shard)
  const uint64_t n_rows = (uint64_t)f.n_shards * f.n_win;
  for (uint64_t i = threadIdx.x; i < n_rows; i += 256) {
    const unsigned long long d = f.rows[i].n_draws;
    all += d;
    if (i % f.n_win <= w) upto += d;
  }
  upto = block_sum256(upto, sred);
  all = block_sum256(all, sred);
  if (threadIdx.x != 0) return;
  const unsigned long long base = f.state->rng_next;  // before any workgroup's arrival (below)
  DevResult r = f.rows[(uint64_t)f.shard * f.n_win + w];
  r.n_decided += a[0];
  r.n_v1 += a[1];
  if (a[2] && a[2] - 1 > r.last_committed_max) r.last_committed_max = a[2] - 1;
  if (a[3] < r.first_undecided) r.first_undecided = a[3];
  if (r.n_draws > f.vq_cap) r.flags |= 8ull;  // records did not fit: the patch is incomplete
  r.rng_next = base + upto;
  r.commit_watermark = 0;
  if (w + 1 == f.n_win) *row_ctx = r;
  if (row_user) row_user[w] = r;
  __threadfence();
  // only rng_next: a later window's shard step (shard_draws) may run on another stream
  if (atomicAdd(arrivals, 1u) + 1u == f.n_win) {
    f.state->rng_next = base + all;
    __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Fold the shards' final rows of consecutive windows into the engine state exactly as
// one evaluator over the windows in order: commit_phase max (state.rs:77-99), first
// undecided = min over shards, contiguous watermark advance. One thread per window
// loads and folds its window's rows (round 5: one thread for every window and shard,
// 17 us at 32 windows x 8 shards); thread 0 then chains last_committed and the
// watermark over the window values in LDS. und_chk = list capacity + 1 (0: no check): a
// shard with more undecided slots than the capacity flags the window (32: its undecided
// list is truncated).
constexpr uint32_t kCommitBlock = 256;
static __global__ __launch_bounds__(kCommitBlock, 8) void shard_commit_kernel(
    const DevResult* rows_all, uint32_t n_shards, uint32_t n_win, uint64_t window_base0, uint64_t window_slots,
    DevState* state, DevResult* res_ctx, DevResult* res_user, uint64_t und_chk) {
  __shared__ unsigned long long s_fu[kCommitBlock], s_lc[kCommitBlock], s_wm[kCommitBlock];
  const uint32_t tid = threadIdx.x;
  unsigned long long lc = 0, wm = 0, steps = 0;  // thread 0: the chain
  if (tid == 0) {
    lc = state->last_committed;
    wm = state->commit_watermark;
    steps = state->steps;
  }
  for (uint32_t c0 = 0; c0 < n_win; c0 += kCommitBlock) {
    const uint32_t w = c0 + tid;
    DevResult g;
    g.n_slots = g.n_decided = g.n_v1 = g.n_pending_r1 = g.n_draws = g.flags = 0;
    const uint64_t window_base = window_base0 + (uint64_t)w * window_slots;
    unsigned long long lcx = 0, fu = window_base + window_slots;
    if (w < n_win) {
      for (uint32_t r = 0; r < n_shards; r++) {
        const DevResult& x = rows_all[(uint64_t)r * n_win + w];
        g.n_slots += x.n_slots;
        g.n_decided += x.n_decided;
        g.n_v1 += x.n_v1;
        g.n_pending_r1 += x.n_pending_r1;
        g.n_draws += x.n_draws;
        g.flags |= x.flags;
        if (und_chk && x.n_slots - x.n_decided >= und_chk) g.flags |= 32ull;
        if (x.last_committed_max > lcx) lcx = x.last_committed_max;
        if (x.n_slots && x.first_undecided < fu) fu = x.first_undecided;
      }
      if (g.n_slots != window_slots) g.flags |= 16ull;  // the rows do not tile the window
      s_fu[tid] = fu;
      s_lc[tid] = lcx;
    }
    __syncthreads();
    if (tid == 0) {  // the chain: in window order
      const uint32_t m = n_win - c0 < kCommitBlock ? n_win - c0 : kCommitBlock;
      for (uint32_t i = 0; i < m; i++) {
        const uint64_t b = window_base0 + (uint64_t)(c0 + i) * window_slots;
        if (s_lc[i] > lc) lc = s_lc[i];
        if (b <= wm && wm < s_fu[i]) wm = s_fu[i];
        s_lc[i] = lc;
        s_wm[i] = wm;
      }
    }
    __syncthreads();
    if (w < n_win) {
      g.last_committed_max = s_lc[tid];
      g.first_undecided = fu;
      g.rng_next = rows_all[w].rng_next;  // the fixed rows carry the position after window w
      g.commit_watermark = s_wm[tid];
      if (w + 1 == n_win) *res_ctx = g;
      if (res_user) res_user[w] = g;
    }
    __syncthreads();  // s_* are rewritten by the next chunk
  }
  if (tid == 0) {  // the fields it owns (the shard step and fix-up own the others)
    state->last_committed = lc;
    state->commit_watermark = wm;
    state->steps = steps + n_win;
  }
}

// ============================================================================
// Follower side of a decided window (handle_decision, engine.rs:708-746): the
// window's decisions arrive as an output buffer (plane 6 committed, plane 7 V1);
// in ascending PhaseId order the one gate is "PhaseId > last_committed at the
// window's start" (a batch decided inside the window only raises last_committed
// to its own id, below every later slot), so applied = V1 & (id > L_in), and
// last_committed = max(L_in, applied ids <= max_phase) (commit_phase, state.rs:65-103).
// ============================================================================
struct FollowParams {
  const uint32_t* out;
  Layout lout;
  uint64_t n_slots, n_words, slot_base, max_phase;
  DevState* state;
  uint32_t* applied;          // optional: one plane of n_words words
  // per-workgroup partials [n_part][4]: applied, committed, max applied id + 1 (<= max_phase),
  // min uncommitted id (folded by the finish kernel: no same-address atomics)
  unsigned long long* acc;
  uint32_t n_part;
};
constexpr uint32_t kFollowGrid = 2048;  // follower_kernel workgroups at most (grid-stride)

static __global__ __launch_bounds__(256) void follower_kernel(FollowParams f) {
  const unsigned long long lc = f.state->last_committed;
  unsigned long long app = 0, com = 0, mx = 0, mn = ~0ull;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < f.n_words; w += (uint64_t)gridDim.x * 256) {
    const uint64_t b = f.lout.base(w);
    const uint32_t vm = valid_mask(w, f.n_words, f.n_slots);
    const uint32_t committed = f.out[b + 6 * f.lout.pstride] & vm, v1 = f.out[b + 7 * f.lout.pstride] & vm;
    const uint64_t first = f.slot_base + 32 * w;  // PhaseId of bit 0
    uint32_t gate = ~0u;                          // bits with PhaseId > lc
    if (first <= lc) gate = lc - first >= 31 ? 0u : ~((2u << (lc - first)) - 1u);
    const uint32_t ap = v1 & gate;
    if (f.applied) f.applied[w] = ap;
    app += __builtin_popcount(ap);
    com += __builtin_popcount(committed);
    const uint32_t apl = ap & phase_limit_mask(f.slot_base, w, f.max_phase);
    if (apl) {
      const unsigned long long id1 = first + (31u - __builtin_clz(apl)) + 1u;
      mx = id1 > mx ? id1 : mx;
    }
    const uint32_t und = ~committed & vm;
    if (und) {
      const unsigned long long id = first + __builtin_ctz(und);
      mn = id < mn ? id : mn;
    }
  }
  __shared__ unsigned long long red[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  app = wave_sum64(app);
  com = wave_sum64(com);
  mx = wave_max64(mx);
  mn = wave_min64(mn);
  if (lane == 0) { red[wave][0] = app; red[wave][1] = com; red[wave][2] = mx; red[wave][3] = mn; }
  __syncthreads();
  if (threadIdx.x < 4) f.acc[(uint64_t)blockIdx.x * 4 + threadIdx.x] = fold4(red, threadIdx.x);
}

static __global__ __launch_bounds__(256) void follower_finish_kernel(FollowParams f, unsigned long long* gate_out,
                                                                     DevResult* res_ctx, DevResult* res_user) {
  __shared__ unsigned long long red[4][4];
  unsigned long long a[4];
  fold_partials(f.acc, f.n_part, red, a);
  if (threadIdx.x != 0) return;
  DevState s = *f.state;
  DevResult r;
  r.n_slots = f.n_slots;
  r.n_v1 = a[0];
  r.n_decided = a[1];
  r.n_pending_r1 = 0;
  r.n_draws = 0;
  if (gate_out) *gate_out = s.last_committed;
  unsigned long long lc = s.last_committed;
  if (a[2] && a[2] - 1 > lc) lc = a[2] - 1;
  const unsigned long long end = f.slot_base + f.n_slots;
  const unsigned long long fu = a[3] < end ? a[3] : end;
  unsigned long long wm = s.commit_watermark;
  if (f.slot_base <= wm && wm < fu) wm = fu;
  r.last_committed_max = lc;
  r.first_undecided = fu;
  r.rng_next = s.rng_next;
  r.commit_watermark = wm;
  r.flags = 0;
  f.state->last_committed = lc;
  f.state->commit_watermark = wm;
  *res_ctx = r;
  if (res_user) *res_user = r;
}

// ============================================================================
// WMVC phase step, one replica's view (weak_mvc.ivy:129-191).
// ============================================================================
__device__ __forceinline__ uint32_t coin_word(const Key& key, uint64_t stream, uint64_t phase,
                                              uint64_t g0, unsigned long long& cur,
                                              uint32_t (&blk)[16]) {
  uint32_t words[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint64_t id = g0 + 32u * h;
    const unsigned long long bi = ((phase - 1) << 40) | (id >> 9);
    if (bi != cur) {
      chacha_block<12>(key, bi, stream, blk);
      cur = bi;
    }
    words[h] = select16(blk, (uint32_t)(id >> 5) & 15u);
    if (h == 0 && (g0 & 31u) == 0) return words[0];
  }
  const uint32_t sh = (uint32_t)(g0 & 31u);
  return (words[0] >> sh) | (words[1] << (32u - sh));
}

template <int N, int W, int BLOCK>
__global__ __launch_bounds__(BLOCK, 4) void wmvc_step_kernel(StepParams p) {
  constexpr int B = ctr_bits(N);
  Record* rec = p.rec + (p.seq & 1u);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tile = blockIdx.x;  // no cross-tile dependency
  if (!tile_prologue(p, rec, tile, tid)) return;
  const uint32_t tw0 = (uint32_t)tid * W;
  const uint64_t w0 = (uint64_t)tile * BLOCK * W + tw0;
  const bool active = w0 < p.n_words;
  uint32_t r1lo[N][W], r1hi[N][W], r2lo[N][W], r2hi[N][W], st_in[W];
  if (active) {
    const uint32_t* base = p.votes + p.lin.base(w0);
    const uint64_t ps = p.lin.pstride;
#pragma unroll
    for (int j = 0; j < N; j++) {
      load_words<W>(base + (2 * j) * ps, r1lo[j]);
      load_words<W>(base + (2 * j + 1) * ps, r1hi[j]);
      load_words<W>(base + (2 * N + 2 * j) * ps, r2lo[j]);
      load_words<W>(base + (2 * N + 2 * j + 1) * ps, r2hi[j]);
    }
    load_words<W>(base + (4 * N) * ps, st_in);
  } else {
#pragma unroll
    for (int i = 0; i < W; i++) {
      st_in[i] = 0;
#pragma unroll
      for (int j = 0; j < N; j++) r1lo[j][i] = r1hi[j][i] = r2lo[j][i] = r2hi[j][i] = ~0u;
    }
  }
  uint32_t o[kOutPlanes][W];
  uint32_t pend_w[W], cm[W], n_coin = 0, any_coin = 0;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const uint32_t vm = valid_mask(w0 + i, p.n_words, p.n_slots);
    // round 1 (phase_rnd1): >= q messages, vote v if #v >= q else ?
    Ctr<B> c0, c1, cp;
    ctr_zero(c0); ctr_zero(c1); ctr_zero(cp);
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint32_t lo = r1lo[j][i], hi = r1hi[j][i];
      ctr_add(c0, ~lo & ~hi);
      ctr_add(c1, lo & ~hi);
      ctr_add(cp, ~(lo & hi));
    }
    const uint32_t gp = ctr_ge(cp, p.q), g0 = ctr_ge(c0, p.q), g1 = ctr_ge(c1, p.q);
    const uint32_t pend1 = ~gp;
    const uint32_t v1 = gp & ~g0 & g1, vq = gp & ~g0 & ~g1;
    // round 2 (phase_rnd2): own vote at self lane
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j == p.self_lane) {
        r2lo[j][i] = (r2lo[j][i] & pend1) | (v1 & ~pend1);
        r2hi[j][i] = (r2hi[j][i] & pend1) | (vq & ~pend1);
      }
    }
    Ctr<B> e0, e1, ep;
    ctr_zero(e0); ctr_zero(e1); ctr_zero(ep);
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint32_t lo = r2lo[j][i], hi = r2hi[j][i];
      ctr_add(e0, ~lo & ~hi);
      ctr_add(e1, lo & ~hi);
      ctr_add(ep, ~(lo & hi));
    }
    const uint32_t live = ~pend1 & ctr_ge(ep, p.q);
    const uint32_t f0 = ctr_ge(e0, p.fp1), f1 = ctr_ge(e1, p.fp1);
    const uint32_t nz0 = ctr_nz(e0), nz1 = ctr_nz(e1);
    const uint32_t d0 = live & f0, d1 = live & ~f0 & f1;
    const uint32_t open = live & ~f0 & ~f1;
    const uint32_t a1 = open & ~nz0 & nz1;
    cm[i] = open & ~nz0 & ~nz1 & vm;  // all round-2 votes '?': common coin
    any_coin |= cm[i];
    o[0][i] = (v1 | pend1) & vm;
    o[1][i] = (vq | pend1) & vm;
    o[2][i] = o[0][i];
    o[3][i] = o[1][i];
    o[4][i] = ~d0 & vm;
    o[5][i] = ~(d0 | d1) & vm;
    o[6][i] = (d0 | d1) & vm;
    o[7][i] = (d1 | a1 | (~live & st_in[i])) & vm;  // coin bits join below
    pend_w[i] = pend1 & vm;
    n_coin += __builtin_popcount(cm[i]);
  }
  // Common coins (coin(p, v), weak_mvc.ivy:173-186): the tile's slots span at most
  // kRows coin blocks, computed once (one per thread) and staged in LDS.
  {
    constexpr int kRows = BLOCK * W * 32 / 512 + 2;
    static_assert(kRows <= BLOCK, "one coin block per thread");
    __shared__ uint32_t s_any[BLOCK / 64];
    __shared__ uint32_t s_coin[kRows][17];
    const unsigned long long wave_any = __ballot(any_coin != 0);
    if (lane == 0) s_any[wave] = wave_any != 0;
    lds_barrier();
    uint32_t tile_any = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; w++) tile_any |= s_any[w];
    if (tile_any) {
      const uint64_t tile_w0 = (uint64_t)tile * BLOCK * W;
      const uint64_t r0 = (p.slot_base + 32 * tile_w0) >> 9;
      if (tid < kRows) {
        uint32_t x[16];
        chacha_block<12>(p.key, ((p.phase - 1) << 40) | (r0 + tid), p.coin_stream, x);
#pragma unroll
        for (int j = 0; j < 16; j++) s_coin[tid][j] = x[j];
      }
      lds_barrier();
#pragma unroll
      for (int i = 0; i < W; i++) {
        if (cm[i]) {
          const uint64_t g0 = p.slot_base + 32 * (w0 + i);
          const uint32_t sh = (uint32_t)(g0 & 31u);
          uint32_t coin = s_coin[(uint32_t)((g0 >> 9) - r0)][(g0 >> 5) & 15u];
          if (sh) {
            const uint64_t g1 = g0 + 32;
            coin = (coin >> sh) | (s_coin[(uint32_t)((g1 >> 9) - r0)][(g1 >> 5) & 15u] << (32u - sh));
          }
          o[7][i] |= cm[i] & coin;
        }
      }
    }
  }
  if (active) {
    uint32_t* ob = p.out + p.lout.base(w0);
#pragma unroll
    for (int pl = 0; pl < kOutPlanes; pl++) store_words_nt<W>(ob + pl * p.lout.pstride, o[pl]);
  }
  uint32_t vm_all[W], dv1[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    vm_all[i] = valid_mask(w0 + i, p.n_words, p.n_slots);
    dv1[i] = o[6][i] & o[4][i];  // committed with decision code lo bit set = V1
  }
  if (p.diag & 2u) return;
  const TileStats ts = thread_stats<W>(o[6], dv1, pend_w, vm_all, n_coin, w0, tw0, p);
  finish_tile<kFinWmvc, BLOCK, W>(p, rec, ts, tile, tid, lane, wave);
}

// ============================================================================
// Exchange stage: digest majority (weak_mvc.ivy:109-128). One wave = 128 slots:
// lane l owns slots 2l and 2l+1 and reads them with one 16-B non-temporal load
// per replica (1 KiB per wave instruction, all N in flight); the two per-lane
// majority bits are bit-interleaved into the wave's 128-slot mask. When the
// digest rows are not 16-B aligned, lane l owns slots l and 64+l (8-B loads).
// ============================================================================
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long spread32(uint32_t x) {
  unsigned long long v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

template <int N>
__device__ __forceinline__ bool digest_major(const uint64_t (&d)[N], uint32_t q) {
  bool st = false;
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < N; j++) c += (d[j] == d[i]) ? 1u : 0u;
    st |= (d[i] != 0) && (c >= q);
  }
  return st;
}

template <int N, bool VEC>
__global__ __launch_bounds__(kBlock) void digest_kernel(const uint64_t* __restrict__ dg,
                                                        uint64_t dstride, uint32_t* out,
                                                        uint64_t n_slots, uint32_t q) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t s0 = ((uint64_t)blockIdx.x * kWaves + wave) * 128;
  if (s0 >= n_slots) return;
  unsigned long long lo, hi;
  if constexpr (VEC) {
    const uint64_t s = s0 + 2 * lane;
    uint64_t d0[N], d1[N];
    if (s + 1 < n_slots) {
#pragma unroll
      for (int j = 0; j < N; j++) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(dg + (uint64_t)j * dstride + s));
        d0[j] = x.x;
        d1[j] = x.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; j++) {
        d0[j] = s < n_slots ? dg[(uint64_t)j * dstride + s] : 0ull;
        d1[j] = 0ull;
      }
    }
    const unsigned long long ev = __ballot(digest_major<N>(d0, q) && s < n_slots);
    const unsigned long long od = __ballot(digest_major<N>(d1, q) && s + 1 < n_slots);
    lo = spread32((uint32_t)ev) | (spread32((uint32_t)od) << 1);
    hi = spread32((uint32_t)(ev >> 32)) | (spread32((uint32_t)(od >> 32)) << 1);
  } else {
    unsigned long long masks[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint64_t s = s0 + 64 * h + lane;
      const bool valid = s < n_slots;
      uint64_t d[N];
#pragma unroll
      for (int j = 0; j < N; j++) d[j] = valid ? dg[(uint64_t)j * dstride + s] : 0ull;
      masks[h] = __ballot(digest_major<N>(d, q) && valid);
    }
    lo = masks[0];
    hi = masks[1];
  }
  if (lane == 0) {
    *reinterpret_cast<uint4*>(out + s0 / 32) =
        make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

static __global__ void coin_kernel(Key key, uint64_t stream, uint64_t phase, uint64_t slot_base,
                            uint64_t n_slots, uint32_t* out) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n_words = (n_slots + 31) / 32;
  if (w >= n_words) return;
  unsigned long long cur = ~0ull;
  uint32_t blk[16];
  out[w] = coin_word(key, stream, phase, slot_base + 32 * w, cur, blk) & valid_mask(w, n_words, n_slots);
}

// Decision bitmaps of a step's output (planes 6 committed, 7 V1/apply) as two
// contiguous bit arrays: what the multi-GPU exchange all-gathers.
static __global__ void bitmap_kernel(const uint32_t* out, Layout lout, uint64_t n_words, uint32_t* committed,
                              uint32_t* v1, uint64_t out_pitch, uint64_t bm_pitch) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_words) return;
  out += blockIdx.y * out_pitch;  // window blockIdx.y of a multi-window call
  committed += blockIdx.y * bm_pitch;
  v1 += blockIdx.y * bm_pitch;
  const uint64_t b = lout.base(w);
  committed[w] = out[b + 6 * lout.pstride];
  v1[w] = out[b + 7 * lout.pstride];
}

// ---- the decided-slot exchange payload (rg_decision_lists_windows_async) ------------
// Per window of a shard: the list of its UNDECIDED slots (committed bit 0), ascending,
// as slot offsets from the shard's first slot, and optionally the V1 bitmap (plane 7 as
// one contiguous bit array, bits past n_slots cleared). At agree90 ~0.04 % of the slots
// are undecided, so the list replaces a committed bitmap that is ~99.96 % ones (1 bit
// per slot) with ~0.013 bits per slot. Two passes over 4096-word chunks (131,072 slots,
// one 256-thread workgroup each; a thread reads 16-B groups, so a wave keeps 8 KiB in
// flight: these kernels run beside the next step's lag kernel, one wave per SIMD, and
// must pull their bytes with few waves):
//  (1) list_scan: the chunk's V1 words, its undecided count, and its words holding an
//      undecided slot as (word, mask) pairs in word order (at most kListPairs; more: the
//      second pass re-reads the chunk's committed plane);
//  (2) list_emit: the chunk's offset in the list = the counts of the chunks before it;
//      every pair expands into slot offsets.
// The list holds at most `cap` entries; its first word is the true count (count > cap:
// truncated).
constexpr uint32_t kListChunkWords = 4096, kListPairs = 128;
struct ListParams {
  const uint32_t* out;  // window w at out + w * out_pitch
  Layout lout;
  uint64_t n_words, n_slots, out_pitch;
  uint32_t* v1;         // optional: window w at v1 + w * v1_pitch
  uint64_t v1_pitch;
  uint32_t* lists;      // [n_win][1 + cap]
  uint32_t cap;
  uint32_t* counts;     // [n_win][n_chunks] undecided slots of the chunk
  uint32_t* nz;         // [n_win][n_chunks] words of the chunk holding one
  uint2* pairs;         // [n_win][n_chunks][kListPairs] (word, undecided mask)
  uint32_t n_chunks;
};

// Exclusive prefix over a 256-thread workgroup of one u32 per thread (returned) and the
// total (tot); buf: two parity halves of 4 words, par alternating between calls.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t c, uint32_t (&buf)[2][4], int par, uint32_t& tot) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t incl = wave_incl_scan32(c, (int)lane);
  if (lane == 63) buf[par][wave] = incl;
  // an LDS-only barrier: __syncthreads() would also drain the caller's outstanding stores
  // (a half is rewritten two calls later, after every thread read it)
  lds_barrier();
  uint32_t pre = 0;
  tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t t = buf[par][k];
    pre += k < wave ? t : 0u;
    tot += t;
  }
  return pre + incl - c;
}

// The 4 words [w, w + 4) of a plane, w a multiple of 4 (one 16-B load: a group never
// crosses a slot tile, T >= 64, or a 4-word-multiple planar stride).
__device__ __forceinline__ u32x4 load_group(const uint32_t* out, const Layout& lo, uint64_t w, int plane) {
  return *reinterpret_cast<const u32x4*>(out + lo.base(w) + plane * lo.pstride);
}

static __global__ __launch_bounds__(256, 8) void list_scan_kernel(ListParams L) {
  __shared__ uint32_t sbuf[2][4];
  __shared__ unsigned long long sred[4];
  const uint32_t win = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const uint32_t* out = L.out + win * L.out_pitch;
  const uint64_t cidx = (uint64_t)win * L.n_chunks + chunk;
  uint2* pairs = L.pairs + cidx * kListPairs;
  // every 16-B group of the chunk in flight at once (8 loads per thread): these waves run
  // one per SIMD beside the lag kernel, so a load round trip per slice would bound them
  u32x4 cg[4], vg[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t w = (uint64_t)chunk * kListChunkWords + j * 1024 + 4 * tid;
    cg[j] = w < L.n_words ? load_group(out, L.lout, w, 6) : u32x4{~0u, ~0u, ~0u, ~0u};
    vg[j] = (L.v1 && w < L.n_words) ? load_group(out, L.lout, w, 7) : u32x4{0u, 0u, 0u, 0u};
  }
  uint32_t run = 0, pop = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t w = (uint64_t)chunk * kListChunkWords + j * 1024 + 4 * tid;
    uint32_t und[4] = {0, 0, 0, 0};
    if (w < L.n_words) {
      const uint32_t cw[4] = {cg[j].x, cg[j].y, cg[j].z, cg[j].w};
      const uint32_t vw[4] = {vg[j].x, vg[j].y, vg[j].z, vg[j].w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t vm = valid_mask(w + q, L.n_words, L.n_slots);
        und[q] = ~cw[q] & vm;
        if (L.v1 && w + q < L.n_words) L.v1[win * L.v1_pitch + w + q] = vw[q] & vm;
      }
    }
    uint32_t nzc = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      nzc += und[q] ? 1u : 0u;
      pop += (uint32_t)__builtin_popcount(und[q]);
    }
    uint32_t tot;
    uint32_t pos = run + block_excl_scan256(nzc, sbuf, j & 1, tot);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (und[q]) {
        if (pos < kListPairs) pairs[pos] = make_uint2((uint32_t)(w + q), und[q]);
        pos++;
      }
    }
    run += tot;
  }
  const unsigned long long c = block_sum256(pop, sred);
  if (tid == 0) {
    L.counts[cidx] = (uint32_t)c;
    L.nz[cidx] = run;
  }
}

static __global__ __launch_bounds__(256, 8) void list_emit_kernel(ListParams L) {
  __shared__ unsigned long long sred[4];
  __shared__ uint32_t sbuf[2][4];
  const uint32_t win = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const uint32_t* cnts = L.counts + (uint64_t)win * L.n_chunks;
  unsigned long long before = 0, total = 0;
  for (uint32_t c = tid; c < L.n_chunks; c += 256) {
    const uint32_t x = cnts[c];
    total += x;
    if (c < chunk) before += x;
  }
  before = block_sum256(before, sred);
  total = block_sum256(total, sred);
  uint32_t* lst = L.lists + (uint64_t)win * (1ull + L.cap);
  if (chunk == 0 && tid == 0) lst[0] = (uint32_t)total;
  if (cnts[chunk] == 0 || before >= L.cap) return;  // uniform: nothing of this chunk is listed
  const uint64_t cidx = (uint64_t)win * L.n_chunks + chunk;
  const uint32_t nz = L.nz[cidx];
  if (nz <= kListPairs) {  // the pairs, one per thread (kListPairs <= the workgroup size)
    uint2 pr = make_uint2(0u, 0u);
    if (tid < nz) pr = L.pairs[cidx * kListPairs + tid];
    uint32_t tot;
    unsigned long long pos = before + block_excl_scan256((uint32_t)__builtin_popcount(pr.y), sbuf, 0, tot);
    uint32_t m = pr.y;
    while (m) {
      if (pos < L.cap) lst[1 + pos] = 32u * pr.x + (uint32_t)__builtin_ctz(m);
      pos++;
      m &= m - 1u;
    }
    return;
  }
  // more words with undecided slots than pairs: re-read the chunk's committed plane
  const uint32_t* out = L.out + win * L.out_pitch;
  unsigned long long run = before;
#pragma unroll 1
  for (int j = 0; j < 4; j++) {
    const uint64_t w = (uint64_t)chunk * kListChunkWords + j * 1024 + 4 * tid;
    uint32_t und[4] = {0, 0, 0, 0};
    if (w < L.n_words) {
      const u32x4 c = load_group(out, L.lout, w, 6);
      const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int q = 0; q < 4; q++) und[q] = ~cw[q] & valid_mask(w + q, L.n_words, L.n_slots);
    }
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) c += (uint32_t)__builtin_popcount(und[q]);
    uint32_t tot;
    unsigned long long pos = run + block_excl_scan256(c, sbuf, j & 1, tot);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint32_t m = und[q];
      while (m) {
        if (pos < L.cap) lst[1 + pos] = (uint32_t)(32 * (w + q) + (uint32_t)__builtin_ctz(m));
        pos++;
        m &= m - 1u;
      }
    }
    run += tot;
  }
}

// ---- own round-1 votes for received proposals (engine.rs:380-481) -------------
// determine_round1_vote: a slot whose PhaseData already holds a proposed value
// votes that value if the proposal matches it, VQuestion otherwise; the first
// proposal of a slot (no proposed value yet) takes randomized_vote: V0 -> one
// StdRng draw, V0 iff u < P70, else VQuestion; V1 -> V1 iff u < P80, else
// VQuestion; VQuestion -> VQuestion without a draw. Draws are consumed in message
// order from the engine's stream (the context's rng_next). `track` = 0 restates
// the reference as it runs today (phases are never created, update_phase is a
// no-op, state.rs:166-185), so every proposal takes randomized_vote.
constexpr uint64_t kP70 = 0xB333333333333000ull;  // (0.7 * 2^64) as u64
constexpr int kR1vBlock = 256;

struct R1vArgs {
  const uint64_t* phase_ids;
  const uint8_t* values;
  uint64_t n, n_slots, slot_base, stride;
  uint32_t* proposed;       // 2 planar planes (lo, hi), code 3 = none
  uint32_t* cells;          // [n_slots] first message index per slot (0xFFFFFFFF = none)
  uint32_t* block_draws;    // [blocks] draws per block, then exclusive offsets
  unsigned long long* base; // [1] rng_next at the start of the batch
  DevState* state;
  uint8_t* votes;
  Key key;
  uint32_t track;
};

__device__ __forceinline__ uint32_t proposed_code(const R1vArgs& a, uint64_t off) {
  const uint32_t w = off >> 5, b = off & 31u;
  return ((a.proposed[w] >> b) & 1u) | (((a.proposed[a.stride + w] >> b) & 1u) << 1);
}

// 1: the first message of each slot without a proposed value claims the slot
static __global__ void r1v_claim_kernel(R1vArgs a) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= a.n || !a.track) return;
  const uint64_t ph = a.phase_ids[m];
  if (ph < a.slot_base || ph - a.slot_base >= a.n_slots) return;
  const uint64_t off = ph - a.slot_base;
  if (proposed_code(a, off) == 3u) atomicMin(a.cells + off, (uint32_t)m);
}

__device__ __forceinline__ bool r1v_draws(const R1vArgs& a, uint64_t m, bool* first, uint64_t* off) {
  const uint64_t ph = a.phase_ids[m];
  *first = false;
  if (ph < a.slot_base || ph - a.slot_base >= a.n_slots) return false;
  *off = ph - a.slot_base;
  *first = !a.track || a.cells[*off] == (uint32_t)m;  // claimed only if no proposal before
  return *first && a.values[m] <= 1;
}

// 2: draws per block
static __global__ __launch_bounds__(kR1vBlock) void r1v_count_kernel(R1vArgs a) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool first = false, d = false;
  uint64_t off = 0;
  if (m < a.n) d = r1v_draws(a, m, &first, &off);
  const int c = __syncthreads_count(d);
  if (threadIdx.x == 0) a.block_draws[blockIdx.x] = (uint32_t)c;
}

// 3: one workgroup: exclusive offsets of the block counts; the batch's draws are
// taken from the engine stream here (rng_next advances by the total)
static __global__ __launch_bounds__(1024) void r1v_scan_kernel(R1vArgs a, uint32_t blocks) {
  __shared__ unsigned long long s_sum[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (blocks + 1023) / 1024, lo = t * per, hi = lo + per < blocks ? lo + per : blocks;
  unsigned long long sum = 0;
  for (uint32_t b = lo; b < hi; b++) sum += a.block_draws[b];
  s_sum[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const unsigned long long v = t >= o ? s_sum[t - o] : 0;
    __syncthreads();
    s_sum[t] += v;
    __syncthreads();
  }
  unsigned long long run = s_sum[t] - sum;
  for (uint32_t b = lo; b < hi; b++) {
    const uint32_t c = a.block_draws[b];
    a.block_draws[b] = (uint32_t)run;
    run += c;
  }
  if (t == 1023) {
    const unsigned long long r0 = a.state->rng_next;
    *a.base = r0;
    a.state->rng_next = r0 + s_sum[1023];
  }
}

// 4: votes, proposed values, cell reset
static __global__ __launch_bounds__(kR1vBlock) void r1v_vote_kernel(R1vArgs a) {
  __shared__ uint32_t s_w[kR1vBlock / 64];
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bool first = false, d = false;
  uint64_t off = 0;
  if (m < a.n) d = r1v_draws(a, m, &first, &off);
  const uint32_t incl = wave_incl_scan32(d ? 1u : 0u, lane);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (int w = 0; w < wave; w++) before += s_w[w];
  if (m >= a.n) return;
  const uint64_t ph = a.phase_ids[m];
  const uint32_t val = a.values[m];
  uint8_t vote;
  if (ph < a.slot_base || ph - a.slot_base >= a.n_slots) {
    vote = 3;                                          // not in this window
  } else if (first) {
    if (d) {
      const unsigned long long k = *a.base + a.block_draws[blockIdx.x] + before + incl - 1;
      uint32_t blk[16];
      chacha_block<12>(a.key, k >> 3, 0, blk);
      const uint32_t ws = (uint32_t)(k & 7u) * 2u;
      const unsigned long long u =
          (unsigned long long)select16(blk, ws) | ((unsigned long long)select16(blk, ws + 1) << 32);
      vote = (uint8_t)((u < (val == 0 ? kP70 : kP80)) ? val : 2u);  // engine.rs:454-481
    } else {
      vote = 2;                                        // VQuestion proposal
    }
    if (a.track) {                                     // phase.proposed_value = Some(value)
      const uint32_t bit = 1u << (off & 31);
      uint32_t* lo = a.proposed + (off >> 5);
      uint32_t* hi = lo + a.stride;
      if (val & 1u) atomicOr(lo, bit); else atomicAnd(lo, ~bit);
      if (val & 2u) atomicOr(hi, bit); else atomicAnd(hi, ~bit);
    }
  } else {
    // a proposal already recorded for the slot: before this batch, or by this
    // batch's first message for the slot (engine.rs:430-441)
    // (cells[] is set only for slots without a proposal before the batch, and only
    // first messages write the proposed planes, so neither read races a write)
    const uint32_t c = a.cells[off];
    const uint32_t cur = c != 0xFFFFFFFFu ? (uint32_t)a.values[c] : proposed_code(a, off);
    vote = (uint8_t)(cur == val ? val : 2u);
  }
  a.votes[m] = vote;
}

// 5: re-arm the claim cells touched by this batch
static __global__ void r1v_reset_kernel(R1vArgs a) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= a.n || !a.track) return;
  const uint64_t ph = a.phase_ids[m];
  if (ph < a.slot_base || ph - a.slot_base >= a.n_slots) return;
  a.cells[ph - a.slot_base] = 0xFFFFFFFFu;
}

static __global__ void draws_kernel(Key key, uint64_t first, uint64_t count, unsigned long long* out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  const uint64_t k = first + t;
  uint32_t blk[16];
  chacha_block<12>(key, k >> 3, 0, blk);
  const uint32_t ws = (uint32_t)(k & 7u) * 2u;
  out[t] = (unsigned long long)select16(blk, ws) | ((unsigned long long)select16(blk, ws + 1) << 32);
}

// Synthetic traces, one thread per 32-slot word (restated in oracle/rabia_oracle.c:or_trace).
static __global__ void trace_kernel(int kind, int n, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                             Layout lay, uint32_t* planes) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n_words = (n_slots + 31) / 32;
  if (w >= n_words) return;
  const uint64_t kmaj = trace_key(seed, 0), kst = trace_key(seed, 1), krot = trace_key(seed, 2);
  uint32_t lo[2][kMaxReplicas], hi[2][kMaxReplicas];
#pragma unroll
  for (int r = 0; r < 2; r++)
#pragma unroll
    for (int j = 0; j < kMaxReplicas; j++) lo[r][j] = hi[r][j] = 0;
  uint32_t stw = 0;
  const int nv0 = (n - 1) / 2;
  const uint32_t vm = valid_mask(w, n_words, n_slots);
  for (int b = 0; b < 32; b++) {
    if (!((vm >> b) & 1u)) break;
    const uint64_t id = slot_base + 32 * w + b;
    const uint32_t m = (uint32_t)(mix64(kmaj + id) & 1u);
    stw |= (uint32_t)(mix64(kst + id) & 1u) << b;
    const uint32_t rot = (uint32_t)(mix64(krot + id) % (uint64_t)n);
#pragma unroll
    for (int r = 0; r < 2; r++) {
#pragma unroll
      for (int j = 0; j < kMaxReplicas; j++) {
        if (j >= n) continue;
        const uint64_t u = mix64(trace_key(seed, 16u + (uint32_t)r * 16u + (uint32_t)j) + id);
        uint32_t c;
        if (kind == 0) {
          c = (uint32_t)(u & 3u);
        } else if (kind == 1) {
          if (u < kTraceP90) {
            c = m;
          } else {
            const uint32_t pick = (uint32_t)u % 3u;
            c = pick == 0 ? 1u - m : (pick == 1 ? kCodeVQ : kCodeNone);
          }
        } else {
          if (r) {
            c = kCodeVQ;
          } else {
            const int l = (int)((j + rot) % (uint32_t)n);
            c = l < nv0 ? kCodeV0 : (l < n - 1 ? kCodeV1 : kCodeVQ);
          }
        }
        lo[r][j] |= (c & 1u) << b;
        hi[r][j] |= ((c >> 1) & 1u) << b;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 2; r++)
#pragma unroll
    for (int j = 0; j < kMaxReplicas; j++) {
      if (j >= n) continue;
      planes[lay.base(w) + (uint64_t)(2 * n * r + 2 * j) * lay.pstride] = lo[r][j];
      planes[lay.base(w) + (uint64_t)(2 * n * r + 2 * j + 1) * lay.pstride] = hi[r][j];
    }
  planes[lay.base(w) + (uint64_t)(4 * n) * lay.pstride] = stw;
}

static __global__ void digest_trace_kernel(int n, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                                    uint64_t dstride, unsigned long long* dg) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const uint64_t id = slot_base + s;
  const uint64_t maj = mix64(trace_key(seed, 3) + id) | 1u;
  for (int j = 0; j < n; j++) {
    const uint64_t u = mix64(trace_key(seed, 64u + (uint32_t)j) + id);
    uint64_t d;
    if (u < kTraceP90) d = maj;
    else if ((u & 15u) == 0) d = 0;
    else d = mix64(u) | 1u;
    dg[(uint64_t)j * dstride + s] = d;
  }
}

// ============================================================================
// WMVC cluster view (config 3): all n replicas of a slot run weak_mvc.ivy
// phase_rnd1 / phase_rnd2 (ivy:129-191) phase after phase, under a deterministic
// adversarial scheduler (each receiver hears itself + q-1 others picked by a keyed
// hash), until every replica decided or max_phases. One lane per slot; replica
// sets are n-bit masks, so each round is popcounts. Restated in
// oracle/rabia_oracle.c:or_wmvc_cluster.
// ============================================================================
__device__ __forceinline__ uint64_t cluster_key(uint64_t seed, uint32_t phase, uint32_t round, int r) {
  return mix64(seed ^ (((uint64_t)phase << 32) | ((uint64_t)round << 16) | (uint64_t)r) *
                          0x9E6C63D0676A9A99ull);
}

// Scheduler hash (the build's own definition; version 2, round 4):
// 32-bit arithmetic. The receiver's key is the low word of cluster_key (a table per
// workgroup: it does not depend on the slot); the slot id enters folded to 32 bits
// (once per slot); h = fmix32(key ^ slot) (murmur3's finaliser: two 32-bit multiplies
// instead of mix64's two 64-bit ones, i.e. 2 instead of 8 quarter-rate multiplies);
// pick i uses 6-bit chunk i % 5 of word i / 5 (word j + 1 = fmix32(word j + golden))
// and maps it to [0, span) by a multiply-shift (a full-rate 24-bit multiply) instead
// of a modulo. Restated in oracle/rabia_oracle.c:or_heard and oracle/rabia_ref.py:heard.
RG_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
RG_HD uint32_t slot_fold32(uint64_t slot) { return (uint32_t)slot ^ ((uint32_t)(slot >> 32) * 0x9E3779B9u); }

// The receiver's heard set: itself + q - 1 others, pick i the k-th lowest still
// available sender, picked branch-free (every lane steps through span - 1 clears and
// keeps the k-th; a loop of k clears diverged across the wave).
template <int N>
__device__ __forceinline__ uint32_t heard_mask_k(uint32_t ck, uint32_t s32, int r, uint32_t q) {
  uint32_t h = fmix32(ck ^ s32);
  uint32_t avail = ((1u << N) - 1u) & ~(1u << r);
  uint32_t mask = 1u << r;
#pragma unroll
  for (uint32_t i = 0; i + 1 < (uint32_t)N; i++) {
    if (i + 1 >= q) break;
    if (i && i % 5 == 0) h = fmix32(h + 0x9E3779B9u);
    const uint32_t span = N - 1 - i;
    const uint32_t k = (((h >> (6 * (i % 5))) & 63u) * span) >> 6;  // (a 24-bit product)
    uint32_t a = avail, sel = avail;
#pragma unroll
    for (uint32_t t = 1; t < span; t++) {
      a &= a - 1;
      sel = t == k ? a : sel;
    }
    const uint32_t pick = sel & (~sel + 1u);
    mask |= pick;
    avail &= ~pick;
  }
  return mask;
}

// The same heard set from a per-workgroup LDS table: the set depends only on the
// receiver r and the pick ranks k_i = ((chunk i of h) * span_i) >> 6 (span_i = N - 1 - i),
// so it is tabulated once per launch over (r, k_0, .., k_{q-2}) (N * (N-1)!/(N-q)!
// entries: 60 at n = 5, 840 at 7, 15,120 at 9) and a lookup replaces the q - 1 branch-free
// k-th-bit selections (heard_mask_k, which fills the table: bit-identical by construction).
// Picks past the fifth re-mix h (heard_mask_k); tables are used only for q - 1 <= 5 picks.
constexpr uint32_t kHeardTabMax = 16384;  // entries (u16): 32 KB of LDS
template <int N>
__host__ __device__ constexpr uint32_t heard_tab_size(uint32_t q) {
  if (q < 1 || q > 6) return 0;
  uint32_t n = N;
  for (uint32_t i = 0; i + 1 < q; i++) {
    n *= (uint32_t)N - 1 - i;
    if (n > kHeardTabMax) return 0;
  }
  return n;
}
// Entry e of the table: (r, k_0, .., k_{q-2}) in mixed radix (r most significant).
template <int N>
__device__ __forceinline__ uint32_t heard_tab_entry(uint32_t e, uint32_t q) {
  uint32_t k[6] = {0, 0, 0, 0, 0, 0};
  for (int i = (int)q - 2; i >= 0; i--) {
    const uint32_t span = (uint32_t)N - 1 - (uint32_t)i;
    k[i] = e % span;
    e /= span;
  }
  const uint32_t r = e;
  uint32_t avail = ((1u << N) - 1u) & ~(1u << r), mask = 1u << r;
  for (uint32_t i = 0; i + 1 < q; i++) {
    uint32_t a = avail;
    for (uint32_t t = 0; t < k[i]; t++) a &= a - 1;
    const uint32_t pick = a & (~a + 1u);
    mask |= pick;
    avail &= ~pick;
  }
  return mask;
}
template <int N>
__device__ __forceinline__ uint32_t heard_mask_tab(const uint16_t* tab, uint32_t ck, uint32_t s32, int r, uint32_t q) {
  const uint32_t h = fmix32(ck ^ s32);
  uint32_t idx = (uint32_t)r;
#pragma unroll
  for (uint32_t i = 0; i + 1 < (uint32_t)N && i < 5; i++) {
    if (i + 1 >= q) break;
    const uint32_t span = N - 1 - i;
    idx = idx * span + ((((h >> (6 * i)) & 63u) * span) >> 6);
  }
  return tab[idx];
}

constexpr int kClusterStats = 8;  // all_decided, v1, sum_phases, max_phases, sum_coin_phases, sum_first, slots, -

// Common-coin table of the cluster kernel: each workgroup computes the ChaCha12 blocks
// of phases 1..P that its chunk's slots read (one block per 512 slots and phase: at most
// kClusterChunk / 512 + 1 blocks per phase) into LDS in its prologue, so the coins of
// those phases are LDS reads (later phases, rare, compute theirs inline). Round 6: this
// replaced coin_table_kernel, a launch ahead of the cluster kernel that wrote the table
// ([P][n_words]) to global memory (14 µs at 8 phases x 2^24 slots, four times its ChaCha
// issue time; the in-kernel blocks add ~4 µs of issue to a VALU-bound kernel).
constexpr uint32_t kClusterCoinPhases = 8;  // 16: 0.498 ms per C3 step, 8: 0.465-0.468, 4: 0.475-0.478 (profiles/r05/c3_ab.json)

// Lane-compacted cluster kernel: each workgroup owns a contiguous chunk of slots;
// a lane whose slot terminated takes the next slot of the chunk (wave-aggregated
// LDS counter), so a wave never idles on its slowest slot (phases per slot vary
// 1..max). Coins of phases <= coin_phases come from the chunk's LDS table. The chunk's
// initial-state words are staged in LDS first (<= kClusterChunk slots: the host sizes
// the grid for it), so a refill reads LDS instead of waiting on global loads.
// bm_dec / bm_v1 (both or neither): the decided / V1 bitmaps of the run, built in LDS
// as slots finish and written once per chunk word (what cluster_bitmap_kernel makes
// from info in a second pass, 26 µs at C3's 2^24 slots).
// Q: the quorum as a compile-time constant (the host picks Q = N / 2 + 1, the majority,
// when the context's quorum is that, else Q = 0 and q at run time). With Q fixed the
// phase body is straight-line: the 2N heard sets of a phase are independent of each other
// and of the votes, so the keys' LDS reads, the hashes and the table reads of both rounds
// are all issued before the first popcount (round 4's body was one dependent LDS round
// trip after another, per receiver, behind uniform branches on q).
// PK (packed tallies, n <= 5 with q = fp1 = n / 2 + 1, i.e. n = 1, 3, 5 at their
// defaults): every count test of the phase is a subset test when the decide threshold
// equals the quorum and every heard set has exactly q members (round 1: c1 >= q iff the
// heard set lies inside the 1-voters, c0 < q iff it meets them; round 2 likewise over V1,
// VQ and their union), so the N receivers' heard sets are packed into one word, N bits
// per receiver, and all N tests of a kind are one AND plus a field-wise nonzero test
// (packed_nz) instead of 2N popcounts (half-rate on gfx950, as v_mul_lo_u32 is:
// tools/valu_peak.hip) and 2N compares. The heard sets come from a table indexed by the
// raw hash bits the picks read (ClusterRaw), pre-shifted into the receiver's field: the
// hash's bit extraction is one v_bfe instead of the picks' multiply-shift index arithmetic.
// Bit-identical to the unpacked body (the same heard sets and rules).
template <int N, int Q>
struct ClusterRaw {  // raw-bits heard table of the packed body: bits [lo, lo + nb) of h
  static constexpr int kPicks = Q - 1;
  static constexpr int kSpan0 = N - 1;
  static constexpr int kLog0 = kSpan0 == 4 ? 2 : kSpan0 == 2 ? 1 : kSpan0 == 1 ? 0 : -1;
  static constexpr int lo = kPicks >= 1 && kLog0 >= 0 ? 6 - kLog0 : 0;
  static constexpr int nb = kPicks >= 1 ? 6 * kPicks - lo : 0;
  static constexpr uint32_t size = nb <= 12 ? (uint32_t)N << nb : 1u;  // (only n <= 5 instantiates the table)
};
template <int N>
__host__ __device__ constexpr uint32_t packed_rep() {  // x * rep: the N-bit x in every receiver's field
  uint32_t r = 0;
  for (int i = 0; i < N; i++) r |= 1u << (N * i);
  return r;
}
// flags at the top bit of each N-bit field: field != 0 (fields hold values < 2^N)
template <int N>
__device__ __forceinline__ uint32_t packed_nz(uint32_t x) {
  constexpr uint32_t L = packed_rep<N>() * ((1u << (N - 1)) - 1u), H = packed_rep<N>() << (N - 1);
  return (((x & L) + L) | x) & H;
}
// field flags (top bits) -> an N-bit mask, bit r = field r: one multiply gathers the
// flags into bits [T, T + N) with T = (N - 1)^2 (no two partial products share a bit)
template <int N>
__host__ __device__ constexpr uint32_t packed_gather_mul() {
  uint32_t m = 0;
  for (int r = 0; r < N; r++) m |= 1u << ((N - 1) * (N - 1) - (N - 1) * r);
  return m;
}
template <int N>
__device__ __forceinline__ uint32_t packed_compress(uint32_t f) {
  constexpr int T = (N - 1) * (N - 1);
  return (__umul24(f >> (N - 1), packed_gather_mul<N>()) >> T) & ((1u << N) - 1u);
}
template <int N>
__host__ __device__ constexpr bool packed_compress_exact() {  // every flag pattern gathers exactly
  for (uint32_t m = 0; m < (1u << N); m++) {
    uint64_t f = 0;
    for (int r = 0; r < N; r++)
      if (m >> r & 1u) f |= 1ull << (N * r);  // (already shifted down by N - 1)
    if (((f * packed_gather_mul<N>()) >> ((N - 1) * (N - 1)) & ((1u << N) - 1u)) != m) return false;
  }
  return true;
}
static_assert(packed_compress_exact<1>() && packed_compress_exact<3>() && packed_compress_exact<5>(),
              "packed_compress gathers every flag pattern");

constexpr uint32_t kClusterChunk = 8192;
constexpr uint32_t kClusterCoinBlocks = kClusterChunk / 512 + 1;  // blocks a chunk's slots span, per phase
template <int N, int Q, bool PK = false>
#ifndef RG_CLUSTER_WAVES
#define RG_CLUSTER_WAVES 6  // waves per SIMD asked of n <= 6 (larger n: spills); n = 5 packed: 83 -> 80 VGPRs, 5 -> 6 waves per SIMD: 0.2724 / 0.2732 / 0.2723 -> 0.2683 / 0.2695 / 0.2686 ms per C3 step (profiles/r06/c3_occ_ab.json)
#endif
__global__ __launch_bounds__(256, (N <= 6 ? RG_CLUSTER_WAVES : 1)) void wmvc_cluster_lc_kernel(const uint32_t* states, uint64_t stride,
                                                              uint64_t n_slots, uint64_t slot_base, uint32_t q_rt,
                                                              uint32_t fp1, Key ckey, uint64_t coin_stream,
                                                              uint64_t dseed, uint32_t max_phases, uint32_t* info,
                                                              unsigned long long* partials, uint32_t coin_phases, uint64_t chunk, uint32_t* bm_dec,
                                                              uint32_t* bm_v1) {
  constexpr uint32_t kAll = (1u << N) - 1u;
  constexpr uint32_t kKeyPhases = 32;  // cluster_key table: phases 1..32 (later phases compute theirs)
  constexpr uint32_t kStageWords = kClusterChunk / 32 + 1;
  __shared__ uint32_t s_next;  // the chunk's next slot (n_slots < 2^32)
  __shared__ uint32_t s_ck[kKeyPhases][2][N];
  using StT = typename std::conditional<(N <= 8), uint8_t, uint16_t>::type;
  __shared__ StT s_stb[kClusterChunk];  // the chunk's initial states, N bits per slot
  __shared__ uint32_t s_bd[kStageWords], s_b1[kStageWords];  // the chunk's decided / V1 bitmap words
  constexpr uint32_t kTabCap = heard_tab_size<N>((uint32_t)N / 2 + 1) ? heard_tab_size<N>((uint32_t)N / 2 + 1) : 1;
  __shared__ uint16_t s_heard[kTabCap];     // heard sets at the majority quorum (heard_mask_tab)
  __shared__ uint32_t s_raw[PK ? ClusterRaw<N, (Q ? Q : 1)>::size : 1];  // PK: raw-bits heard table, pre-shifted
  __shared__ uint32_t s_coin[kClusterCoinPhases * kClusterCoinBlocks * 16];  // coin blocks [phase][block][word]
  const uint32_t q = Q ? (uint32_t)Q : q_rt;
  const uint32_t tab_n = heard_tab_size<N>(q);
  const bool use_tab = tab_n != 0 && tab_n <= kTabCap;  // (uniform; a constant when Q is)
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
  const uint64_t c1 = c0 + chunk < n_slots ? c0 + chunk : n_slots;
  const uint64_t w0 = c0 / 32;
  if (threadIdx.x == 0) s_next = (uint32_t)c0;
  for (uint32_t e = threadIdx.x; e < kKeyPhases * 2 * N; e += blockDim.x) {
    const uint32_t ph = e / (2 * N), rd = (e / N) % 2, rr = e % N;
    s_ck[ph][rd][rr] = (uint32_t)cluster_key(dseed, ph + 1, rd + 1, (int)rr);
  }
  if constexpr (PK) {
    static_assert(N <= 5 && Q == N / 2 + 1, "packed tallies: N fields of N bits, majority quorum");
    using Raw = ClusterRaw<N, Q>;
    for (uint32_t e = threadIdx.x; e < Raw::size; e += blockDim.x) {
      const uint32_t r = e >> Raw::nb;
      const uint32_t h = (e & ((1u << Raw::nb) - 1u)) << Raw::lo;  // the bits the picks read
      uint32_t avail = kAll & ~(1u << r), mask = 1u << r;
      for (int i = 0; i < Raw::kPicks; i++) {  // heard_mask_k's picks, from the raw bits
        const uint32_t span = (uint32_t)N - 1 - (uint32_t)i;
        const uint32_t k = (((h >> (6 * i)) & 63u) * span) >> 6;
        uint32_t a = avail;
        for (uint32_t t = 0; t < k; t++) a &= a - 1;
        const uint32_t pick = a & (~a + 1u);
        mask |= pick;
        avail &= ~pick;
      }
      s_raw[e] = mask << (N * r);
    }
  } else if (use_tab) {
    for (uint32_t e = threadIdx.x; e < tab_n; e += blockDim.x) s_heard[e] = (uint16_t)heard_tab_entry<N>(e, q);
  }
  const uint32_t nw = c1 > c0 ? (uint32_t)((c1 - 1) / 32 - w0 + 1) : 0u;  // <= kStageWords (chunk <= kClusterChunk)
  // the coin blocks of phases 1..coin_phases over the chunk's ids (coin_kernel's bits:
  // phase p, id -> block ((p - 1) << 40) | (id >> 9), word (id >> 5) & 15, bit id & 31)
  const uint64_t cb0 = (slot_base + c0) >> 9;
  const uint32_t n_cb = c1 > c0 ? (uint32_t)(((slot_base + c1 - 1) >> 9) - cb0 + 1) : 0u;  // <= kClusterCoinBlocks
  for (uint32_t e = threadIdx.x; e < coin_phases * n_cb; e += blockDim.x) {
    const uint32_t ph = e / n_cb, j = e - ph * n_cb;
    uint32_t x[16];
    chacha_block<12>(ckey, ((uint64_t)ph << 40) | (cb0 + j), coin_stream, x);
    u32x4* dst = reinterpret_cast<u32x4*>(s_coin + (ph * kClusterCoinBlocks + j) * 16);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      u32x4 v;
      v.x = x[4 * k]; v.y = x[4 * k + 1]; v.z = x[4 * k + 2]; v.w = x[4 * k + 3];
      dst[k] = v;
    }
  }
  // the state words transposed to one element per slot (a refill reads one byte / short
  // instead of N words and N bit extractions); the host makes c0 a multiple of 32, so
  // slot c0 + i is element i
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
    uint32_t x[N];
#pragma unroll
    for (int r = 0; r < N; r++) x[r] = states[(uint64_t)r * stride + w0 + w];
    constexpr int kPer = 4 / (int)sizeof(StT);  // slots per 32-bit store
#pragma unroll
    for (int q4 = 0; q4 < 32 / kPer; q4++) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < kPer; j++) {
        uint32_t e = 0;
#pragma unroll
        for (int r = 0; r < N; r++) e |= ((x[r] >> (kPer * q4 + j)) & 1u) << r;
        v |= e << (8 * (int)sizeof(StT) * j);
      }
      if (32 * w + kPer * q4 < kClusterChunk) reinterpret_cast<uint32_t*>(s_stb)[(32 / kPer) * w + q4] = v;
    }
  }
  if (bm_dec)
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) s_bd[w] = s_b1[w] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t acc[kClusterStats] = {0, 0, 0, 0, 0, 0, 0, 0};  // per lane: <= chunk slots, sums < 2^32
  bool active = false;
  uint32_t s = 0;  // the lane's slot (window-relative)
  uint64_t id = 0;
  uint32_t s32 = 0, st = 0, decided = 0, decv = 0, p = 0, first = 0, coins = 0;
  // running offsets: the LDS coin word of the current phase, the slot's phase-1 coin word,
  // the phase's key row in s_ck (one add per phase instead of address arithmetic)
  constexpr uint32_t kCoinRow = kClusterCoinBlocks * 16;
  uint32_t c_off = 0, c_w1 = 0, k_off = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!active);
    if (idle) {
      const uint32_t cnt = (uint32_t)__builtin_popcountll(idle);
      const int leader = __builtin_ctzll(idle);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&s_next, cnt);
      base = __shfl(base, leader, 64);
      if (!active) {
        const uint32_t rank = (uint32_t)__builtin_popcountll(idle & ((1ull << lane) - 1ull));
        const uint32_t ns = base + rank;
        if (ns < (uint32_t)c1) {
          s = ns;
          id = slot_base + s;
          s32 = slot_fold32(id);
          st = s_stb[s - (uint32_t)c0];
          decided = decv = first = coins = 0;
          c_w1 = c_off = (uint32_t)((id >> 5) - (cb0 << 4));
          k_off = 0;
          p = 1;
          active = true;
        }
      }
    }
    if (!__ballot(active)) break;
    if (!active) continue;
    // ---- one phase of every replica of slot s (same rules as wmvc_cluster_kernel)
    // the coin word of this phase, read ahead (its latency hides behind the heard sets;
    // unconditional, phase 1's row standing in for later phases)
    const bool coin_tabbed = p <= coin_phases;
    const uint32_t coin_w = s_coin[coin_tabbed ? c_off : c_w1];
    uint32_t ck[2][N];
    if (p <= kKeyPhases) {
#pragma unroll
      for (int rd = 0; rd < 2; rd++)
#pragma unroll
        for (int r = 0; r < N; r++) ck[rd][r] = (&s_ck[0][0][0])[k_off + rd * N + r];
    } else {
#pragma unroll
      for (int rd = 0; rd < 2; rd++)
#pragma unroll
        for (int r = 0; r < N; r++) ck[rd][r] = (uint32_t)cluster_key(dseed, p, (uint32_t)rd + 1, r);
    }
    uint32_t nv1 = 0, need_coin = 0, newly = 0, newv = 0;  // per replica: round-2 vote 1, coin, decides now
    uint32_t coin_tab_bit;
    if constexpr (PK) {
      using Raw = ClusterRaw<N, Q>;
      constexpr uint32_t rep = packed_rep<N>(), H = rep << (N - 1);
      uint32_t ph[2] = {0u, 0u};  // both rounds' heard sets, receiver r in bits [N r, N r + N)
#pragma unroll
      for (int rd = 0; rd < 2; rd++)
#pragma unroll
        for (int r = 0; r < N; r++) {
          // fmix32 without its last step: h = x ^ (x >> 16), and only h's bits [lo, lo + nb)
          // are read, so the byte offset of the table entry is taken from x directly
          uint32_t x = ck[rd][r] ^ s32;
          x ^= x >> 16;
          x *= 0x85EBCA6Bu;
          x ^= x >> 13;
          x *= 0xC2B2AE35u;
          uint32_t a = 0;
          if constexpr (Raw::nb > 0)
            a = ((x >> (Raw::lo - 2)) ^ (x >> (Raw::lo + 14))) & (((1u << Raw::nb) - 1u) << 2);
          ph[rd] |= *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(s_raw) +
                                                       ((uint32_t)r << (Raw::nb + 2)) + a);
        }
      // round 1: v1 = all heard voted 1, vq = heard both values
      const uint32_t rs = __umul24(st, rep);
      const uint32_t some1 = packed_nz<N>(ph[0] & rs), some0 = packed_nz<N>(ph[0] & ~rs);
      const uint32_t v1 = packed_compress<N>(H & ~some0), vq = packed_compress<N>(some1 & some0);
      uint32_t coin_word = coin_w;  // consumed here, as in the unpacked body below
      asm volatile("" : "+v"(coin_word));
      coin_tab_bit = (coin_word >> ((uint32_t)id & 31u)) & 1u;
      // round 2 (fp1 = q): d0 = none of V1 / VQ heard, d1 = only V1 heard; undecided:
      // 1 if only V1 / VQ heard and some V1, the coin if only VQ heard
      const uint32_t rv1 = __umul24(v1, rep), rvq = __umul24(vq, rep);
      const uint32_t rnz = rv1 | rvq;
      const uint32_t s1 = packed_nz<N>(ph[1] & rv1), snz = packed_nz<N>(ph[1] & rnz);
      const uint32_t sn1 = packed_nz<N>(ph[1] & ~rv1), s0 = packed_nz<N>(ph[1] & ~rnz);
      const uint32_t snq = packed_nz<N>(ph[1] & ~rvq);
      const uint32_t d1f = H & ~sn1, d0f = H & ~snz;
      newly = packed_compress<N>(d0f | d1f);
      newv = packed_compress<N>(d1f);
      nv1 = packed_compress<N>(d1f | (s1 & ~s0));
      need_coin = packed_compress<N>(H & ~snq);
    } else {
      uint32_t hm[2][N];  // heard sets of both rounds: independent of the votes
#pragma unroll
      for (int rd = 0; rd < 2; rd++)
#pragma unroll
        for (int r = 0; r < N; r++)
          hm[rd][r] = use_tab ? heard_mask_tab<N>(s_heard, ck[rd][r], s32, r, q) : heard_mask_k<N>(ck[rd][r], s32, r, q);
      uint32_t v1 = 0, vq = 0;
#pragma unroll
      for (int r = 0; r < N; r++) {
        const uint32_t c1r = __builtin_popcount(hm[0][r] & st), c0r = __builtin_popcount(hm[0][r] & ~st);
        v1 |= (uint32_t)(c1r >= q) << r;
        vq |= (uint32_t)(c1r < q && c0r < q) << r;
      }
      // the coin word consumed on every phase, after the round-1 tally (a load left unconsumed
      // let its register be reused, which put a wait for it at the top of the next phase)
      uint32_t coin_word = coin_w;
      asm volatile("" : "+v"(coin_word));  // (materialised here: the compiler would sink it into the coin branch)
      coin_tab_bit = (coin_word >> ((uint32_t)id & 31u)) & 1u;
#pragma unroll
      for (int r = 0; r < N; r++) {
        const uint32_t c1r = __builtin_popcount(hm[1][r] & v1), cq = __builtin_popcount(hm[1][r] & vq);
        const uint32_t c0r = q - c1r - cq;
        const bool d0 = c0r >= fp1, d1 = !d0 && c1r >= fp1;
        newly |= (uint32_t)(d0 || d1) << r;
        newv |= (uint32_t)d1 << r;
        // undecided this phase: 0 if any 0 was heard, else 1 if any 1, else the coin
        nv1 |= (uint32_t)(d1 || (!d0 && c0r == 0 && c1r > 0)) << r;
        need_coin |= (uint32_t)(!d0 && !d1 && c0r == 0 && c1r == 0) << r;
      }
    }
    newly &= ~decided;
    if (newly && !first) first = p;
    decided |= newly;
    decv |= newv & newly;
    uint32_t nst = nv1;
    if (need_coin) {  // one coin per slot and phase, counted whenever a replica needs it
      uint32_t coin;
      if (coin_tabbed) {
        coin = coin_tab_bit;
      } else {
        uint32_t blk[16];
        chacha_block<12>(ckey, ((uint64_t)(p - 1) << 40) | (id >> 9), coin_stream, blk);
        coin = (select16(blk, (uint32_t)(id >> 5) & 15u) >> (id & 31)) & 1u;
      }
      coins++;
      nst |= coin ? need_coin : 0u;
    }
    st = (nst & ~decided) | (decv & decided);
    const bool all = decided == kAll;
    if (all || p >= max_phases) {
      const uint32_t phases = all ? p : 0u;
      const uint32_t dec = all ? ((decv == 0 || decv == kAll) ? (decv & 1u) : kCodeVQ) : kCodeNone;
      info[s] = dec | (phases << 8) | (first << 16) | (coins << 24);
      if (bm_dec && dec <= kCodeV1) {
        const uint32_t wl = s / 32 - (uint32_t)w0, bit = 1u << (s & 31);
        atomicOr(&s_bd[wl], bit);
        if (dec == kCodeV1) atomicOr(&s_b1[wl], bit);
      }
      acc[0] += all;
      acc[1] += dec == kCodeV1;
      acc[2] += phases;
      acc[3] = phases > acc[3] ? phases : acc[3];
      acc[4] += coins;
      acc[5] += first;
      acc[6] += 1;
      active = false;
    } else {
      p++;
      c_off += kCoinRow;
      k_off += 2 * N;
    }
  }
  __shared__ unsigned long long red[4][kClusterStats];
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kClusterStats; k++) {
    const unsigned long long x = k == 3 ? wave_max64(acc[k]) : wave_sum64(acc[k]);
    if (lane == 0) red[wave][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < kClusterStats) {
    const int k = threadIdx.x;
    unsigned long long v = 0;
    for (int w = 0; w < 4; w++) v = k == 3 ? (red[w][k] > v ? red[w][k] : v) : v + red[w][k];
    partials[(uint64_t)blockIdx.x * kClusterStats + k] = v;
  }
  // the chunk's bitmap words (the host makes chunk a multiple of 32: no word is shared
  // with another workgroup; bits past n_slots stay 0)
  if (bm_dec)
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
      bm_dec[w0 + w] = s_bd[w];
      bm_v1[w0 + w] = s_b1[w];
    }
}

// Decided / V1 bitmaps of a cluster run's info words (one wave ballot per 64 slots):
// the per-shard payload the C3 multi-GPU exchange all-gathers.
static __global__ __launch_bounds__(256) void cluster_bitmap_kernel(const uint32_t* info, uint64_t n_slots,
                                                                    uint32_t* decided, uint32_t* v1) {
  const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t d = s < n_slots ? (info[s] & 255u) : kCodeNone;
  const unsigned long long bd = __ballot(d <= kCodeV1), b1 = __ballot(d == kCodeV1);
  const int lane = threadIdx.x & 63;
  const uint64_t w = (s - lane) / 32;  // this wave's first word
  const uint64_t n_words = (n_slots + 31) / 32;
  if (lane == 0 && w < n_words) { decided[w] = (uint32_t)bd; v1[w] = (uint32_t)b1; }
  if (lane == 32 && w + 1 < n_words) { decided[w + 1] = (uint32_t)(bd >> 32); v1[w + 1] = (uint32_t)(b1 >> 32); }
}

// One 256-thread block: thread t folds field t % 8 of blocks t / 8, t / 8 + 32, ...
// (every load of a thread in flight together), then the 32 partial folds per field.
// The cluster run's statistics: the workgroups' partials folded by one 1024-thread
// workgroup, 16 loads per thread in flight at once (a 256-thread loop of dependent
// accumulations took 19 µs for 2,048 partials), then wave shuffles over the lanes that
// hold the same statistic (lane % 8) and one LDS step.
constexpr int kStatsBlock = 1024;
static __global__ __launch_bounds__(kStatsBlock) void cluster_stats_kernel(const unsigned long long* partials,
                                                                           uint32_t nblocks, unsigned long long* out) {
  static_assert(kClusterStats == 8, "lane % 8 holds statistic k");
  constexpr uint32_t kRows = kStatsBlock / kClusterStats;  // partial rows per pass
  const int t = threadIdx.x, k = t % kClusterStats, lane = t & 63, wave = t >> 6;
  unsigned long long v = 0;
  for (uint32_t b0 = (uint32_t)t / kClusterStats; b0 < nblocks; b0 += kRows * 16) {
    unsigned long long x[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t b = b0 + (uint32_t)j * kRows;
      x[j] = b < nblocks ? partials[(uint64_t)b * kClusterStats + k] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) v = k == 3 ? (x[j] > v ? x[j] : v) : v + x[j];
  }
  for (int o = 8; o < 64; o <<= 1) {  // the wave's lanes with the same k
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = k == 3 ? (y > v ? y : v) : v + y;
  }
  __shared__ unsigned long long red[kStatsBlock / 64][kClusterStats];
  if (lane < kClusterStats) red[wave][lane] = v;
  __syncthreads();
  if (t >= kClusterStats) return;
  v = 0;
  for (int w = 0; w < kStatsBlock / 64; w++) v = k == 3 ? (red[w][k] > v ? red[w][k] : v) : v + red[w][k];
  out[k] = v;
}

// Initial states of the adversarial cluster trace (restated in or_cluster_trace).
static __global__ void cluster_trace_kernel(int n, uint64_t seed, uint64_t slot_base, uint64_t n_slots, uint64_t stride,
                                     uint32_t* states) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n_words = (n_slots + 31) / 32;
  if (w >= n_words) return;
  const uint64_t krot = trace_key(seed, 4);
  const uint32_t vm = valid_mask(w, n_words, n_slots);
  uint32_t planes[kMaxReplicas];
#pragma unroll
  for (int r = 0; r < kMaxReplicas; r++) planes[r] = 0;
  for (int b = 0; b < 32; b++) {
    if (!((vm >> b) & 1u)) break;
    const uint32_t rot = (uint32_t)(mix64(krot + slot_base + 32 * w + b) % (uint64_t)n);
#pragma unroll
    for (int r = 0; r < kMaxReplicas; r++)
      if (r < n && ((uint32_t)r + rot) % (uint32_t)n < (uint32_t)(n - 1) / 2) planes[r] |= 1u << b;
  }
#pragma unroll
  for (int r = 0; r < kMaxReplicas; r++)
    if (r < n) states[(uint64_t)r * stride + w] = planes[r];
}

// Diagnostic: the REF kernel's memory pattern with no protocol (reads NIN planes,
// writes NOUT planes of XOR mixes). The achievable-bandwidth reference for it.
// T = 0: planar planes `stride` words apart; T > 0: slot-tiled, the planes of a
// T-word slot tile stored back to back. NT: non-temporal loads/stores.
template <bool NT>
__device__ __forceinline__ uint4 ld4(const uint32_t* p) {
  u32x4 x;
  if constexpr (NT) x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else x = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(x.x, x.y, x.z, x.w);
}
template <bool NT>
__device__ __forceinline__ void st4(uint32_t* p, uint4 v) {
  u32x4 x = {v.x, v.y, v.z, v.w};
  if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = x;
}

template <int NIN, int NOUT, bool NT>
__global__ __launch_bounds__(256) void stream_probe_kernel(const uint32_t* in, uint32_t* out, uint64_t stride,
                                                           uint64_t n_words, uint32_t T) {
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (w0 >= n_words) return;
  uint64_t ib, ob, ps_in, ps_out;
  if (T) {
    ib = (w0 / T) * (uint64_t)(NIN + 1) * T + (w0 % T);
    ob = (w0 / T) * (uint64_t)NOUT * T + (w0 % T);
    ps_in = ps_out = T;
  } else {
    ib = ob = w0;
    ps_in = ps_out = stride;
  }
  uint4 v[NIN];
#pragma unroll
  for (int j = 0; j < NIN; j++) v[j] = ld4<NT>(in + ib + j * ps_in);
#pragma unroll
  for (int k = 0; k < NOUT; k++) {
    uint4 a = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NIN; j++) {
      const int r = (j + k) & 31;
      a.x ^= rotl32(v[j].x, r); a.y ^= rotl32(v[j].y, r); a.z ^= rotl32(v[j].z, r); a.w ^= rotl32(v[j].w, r);
    }
    st4<NT>(out + ob + k * ps_out, a);
  }
}

}  // namespace rg
