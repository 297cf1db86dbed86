// rabia_gpu.hip — C ABI (include/rabia_gpu.h) over the gfx950 kernels.
//
// The context is the GPU-side twin of the reference's per-engine state: the
// StdRng position, last_committed_phase and the commit watermark live in device
// memory and are advanced by the last workgroup of every step, so consecutive
// steps on one stream never round-trip through the host.
#include "rabia_gpu.h"
#include "rabia_gpu_debug.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "rg_ctx.h"
#include "rg_kernels.h"

using namespace rg;

namespace rg {
void launch_ref_shard(int n, int block, int words, uint32_t grid, hipStream_t s, const StepParams& p);
}

namespace {

thread_local std::string g_err;  // errors before a context exists

// Look-back launches of the tiled kernels (ref_step_kernel, wmvc_step_kernel) rely on
// dispatch order for forward progress, so two of them running at once on one GPU can
// wait on each other across kernels. While more than one context lives
// on a device, every such launch is chained behind the device's previous one through
// one event (a stream wait when the previous launch came from another context or
// stream). Large REF launches run the ticketed lag kernel and need no chain.
struct DevChain {
  std::mutex mu;
  int live = 0;                  // contexts on the device
  hipEvent_t ev = nullptr;       // after the device's last chained launch
  const rg_ctx* owner = nullptr;
  hipStream_t stream = nullptr;
};
constexpr int kMaxDevices = 64;
DevChain g_chain[kMaxDevices];

int fail(rg_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  else g_err = msg;
  return code;
}

int hip_fail(rg_ctx* ctx, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(ctx, RG_EHIP, m);
}

#define RG_HIP(ctx, call)                                   \
  do {                                                      \
    hipError_t e_ = (call);                                 \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call);  \
  } while (0)

constexpr int wmax_for(int n) { return n <= 5 ? 4 : (n <= 10 ? 2 : 1); }
// persistent lag kernel: one workgroup per CU with 2048-word tiles (launches of >= 2
// 1024 x lag_words(n)-word tiles per CU), else two 512-thread workgroups per CU with
// tiles of 512 x lag_words(n) words. The one-per-CU tile runs as 512 threads x 4 words
// (16-byte plane loads per lane) at every n <= 10: n = 5, 662.6 vs 668.2 us per 2^30
// slots against 1024 x 2 (profiles/r04_ab_lag_w4_2e30.json); n = 9, 259.5 vs 298.8 us
// per 2^28 slots against 1024 x 1 (profiles/r05/c5_probe_n9_k32_shapes.json). No
// scratch up to n = 10 (256 VGPRs at 8 waves per CU).
constexpr int kLagBlock = 1024, kLagBlockSmall = 512;
constexpr int lag_words(int n) { return n <= 5 ? 2 : 1; }
constexpr int lag_one_block(int) { return 512; }
constexpr int lag_one_words(int) { return 4; }
constexpr uint64_t kLagOneTileWords = 2048;

// Tile shapes of the tiled kernel: {threads, words per thread}. Big tiles keep the
// per-launch count of tiles and look-back hand-offs low on large windows; small
// tiles fill the 256 CUs on single 2^20-slot windows. (Large REF launches run the
// persistent lag kernel instead.)
enum TileCfg { kCfgBig = 0, kCfgMid = 1, kCfgSmall = 2 };
constexpr int cfg_block(int c) { return c == kCfgBig ? 512 : (c == kCfgSmall ? 128 : 256); }
inline int cfg_words(int c, int n) { return c == kCfgSmall ? 1 : wmax_for(n); }

int pick_cfg(int n, uint64_t n_words) {
  const uint64_t wm = (uint64_t)wmax_for(n);
  if (n_words / (512 * wm) >= 256) return kCfgBig;
  if (n_words / (256 * wm) >= 128) return kCfgMid;
  return kCfgSmall;
}

using StepLaunch = void (*)(int, uint32_t, hipStream_t, const StepParams&);

template <int N>
struct Disp {
  static constexpr int WM = wmax_for(N);
  static void ref(int c, uint32_t grid, hipStream_t s, const StepParams& p) {
    if (c == kCfgBig) hipLaunchKernelGGL((ref_step_kernel<N, WM, 512, false>), dim3(grid), dim3(512), 0, s, p);
    else if (c == kCfgMid) hipLaunchKernelGGL((ref_step_kernel<N, WM, 256, false>), dim3(grid), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((ref_step_kernel<N, 1, 128, false>), dim3(grid), dim3(128), 0, s, p);
  }
  // persistent lag kernel (large launches): grid = resident workgroups, tiles by ticket
  static void ref_lag(uint32_t grid, hipStream_t s, const StepParams& p) {  // n <= 10 (step_impl)
    if constexpr (N <= 10)  // 8 waves per CU, up to 256 VGPRs each
      hipLaunchKernelGGL((ref_lag_kernel<N, lag_one_words(N), lag_one_block(N), false, 2>), dim3(grid),
                         dim3(lag_one_block(N)), 0, s, p);
  }
  static void ref_lag512(uint32_t grid, hipStream_t s, const StepParams& p) {
    if constexpr (N <= 10)
      hipLaunchKernelGGL((ref_lag_kernel<N, lag_words(N), kLagBlockSmall, false>), dim3(grid), dim3(kLagBlockSmall),
                         0, s, p);
  }
  static void wmvc(int c, uint32_t grid, hipStream_t s, const StepParams& p) {
    if (c == kCfgBig) hipLaunchKernelGGL((wmvc_step_kernel<N, WM, 512>), dim3(grid), dim3(512), 0, s, p);
    else if (c == kCfgMid) hipLaunchKernelGGL((wmvc_step_kernel<N, WM, 256>), dim3(grid), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((wmvc_step_kernel<N, 1, 128>), dim3(grid), dim3(128), 0, s, p);
  }
  static void digest(uint32_t grid, hipStream_t s, const uint64_t* dg, uint64_t ds, uint32_t* out,
                     uint64_t n, uint32_t q) {
    if ((reinterpret_cast<uintptr_t>(dg) & 15u) == 0 && (ds & 1u) == 0)  // rows 16-B aligned
      hipLaunchKernelGGL((digest_kernel<N, true>), dim3(grid), dim3(kBlock), 0, s, dg, ds, out, n, q);
    else
      hipLaunchKernelGGL((digest_kernel<N, false>), dim3(grid), dim3(kBlock), 0, s, dg, ds, out, n, q);
  }
  static void cluster_lc(uint32_t grid, hipStream_t s, const uint32_t* st, uint64_t stride, uint64_t n_slots,
                         uint64_t base, uint32_t q, uint32_t fp1, Key key, uint64_t cs, uint64_t dseed,
                         uint32_t maxp, uint32_t* info, unsigned long long* part, uint32_t coin_phases,
                         uint64_t chunk, uint32_t* bm_dec, uint32_t* bm_v1) {
    constexpr bool kPackable = N <= 5 && N % 2 == 1;  // N fields of N bits; q = fp1 = N / 2 + 1 by default
    if (kPackable && q == (uint32_t)(N / 2 + 1) && fp1 == q) {  // subset tests instead of popcounts
      if constexpr (kPackable)
        hipLaunchKernelGGL((wmvc_cluster_lc_kernel<N, N / 2 + 1, true>), dim3(grid), dim3(256), 0, s, st, stride,
                           n_slots, base, q, fp1, key, cs, dseed, maxp, info, part, coin_phases, chunk, bm_dec,
                           bm_v1);
    } else if (q == (uint32_t)(N / 2 + 1))  // the majority quorum: the straight-line instantiation
      hipLaunchKernelGGL((wmvc_cluster_lc_kernel<N, N / 2 + 1>), dim3(grid), dim3(256), 0, s, st, stride, n_slots,
                         base, q, fp1, key, cs, dseed, maxp, info, part, coin_phases, chunk, bm_dec, bm_v1);
    else
      hipLaunchKernelGGL((wmvc_cluster_lc_kernel<N, 0>), dim3(grid), dim3(256), 0, s, st, stride, n_slots, base, q,
                         fp1, key, cs, dseed, maxp, info, part, coin_phases, chunk, bm_dec, bm_v1);
  }
};

using DigestLaunch = void (*)(uint32_t, hipStream_t, const uint64_t*, uint64_t, uint32_t*, uint64_t,
                              uint32_t);

#define RG_TABLE(fn)                                                                          \
  {nullptr, &Disp<1>::fn, &Disp<2>::fn, &Disp<3>::fn, &Disp<4>::fn, &Disp<5>::fn,             \
   &Disp<6>::fn, &Disp<7>::fn, &Disp<8>::fn, &Disp<9>::fn, &Disp<10>::fn, &Disp<11>::fn,     \
   &Disp<12>::fn, &Disp<13>::fn, &Disp<14>::fn, &Disp<15>::fn, &Disp<16>::fn}

const StepLaunch kRefLaunch[17] = RG_TABLE(ref);
using LagLaunch = void (*)(uint32_t, hipStream_t, const StepParams&);
const LagLaunch kRefLagLaunch[17] = RG_TABLE(ref_lag);
const LagLaunch kRefLag512Launch[17] = RG_TABLE(ref_lag512);
const StepLaunch kWmvcLaunch[17] = RG_TABLE(wmvc);
const DigestLaunch kDigestLaunch[17] = RG_TABLE(digest);
using ClusterLcLaunch = void (*)(uint32_t, hipStream_t, const uint32_t*, uint64_t, uint64_t, uint64_t, uint32_t,
                                 uint32_t, Key, uint64_t, uint64_t, uint32_t, uint32_t*, unsigned long long*,
                                 uint32_t, uint64_t, uint32_t*, uint32_t*);
const ClusterLcLaunch kClusterLcLaunch[17] = RG_TABLE(cluster_lc);

hipStream_t pick_stream(rg_ctx* ctx, void* stream) {
  return stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
}

Record fresh_record() {
  Record r;
  std::memset(&r, 0, sizeof r);
  return r;
}

// Scratch a launch of `slots` slots over `windows` windows may need (rg_reserve):
// look-back / statistics granules (the smallest tile is 128 words = 4,096 slots, every
// window a ragged tail; the lag kernel keeps >= 3 x its grid of <= 2 workgroups per CU),
// fix-up partials (<= kFixGrid per window), decision-list chunk counts.
uint64_t tiles_for(const rg_ctx* ctx, uint64_t slots, uint32_t windows) {
  return slots / 4096 + 1 + windows + 6ull * ctx->n_cu;
}
uint64_t list_chunks_for(uint64_t slots, uint32_t windows) { return slots / (32ull * kListChunkWords) + 1 + windows; }

// Size the context's scratch for launches of up to max_slots slots over up to max_windows
// windows (grow only). Synchronous: it frees buffers launches in flight may use, so it
// is the one place that synchronises the device; the _async entry points never grow
// scratch and return RG_EINVAL past the reservation instead (include/rabia_gpu.h).
int reserve_impl(rg_ctx* ctx, uint64_t max_slots, uint32_t max_windows) {
  if (max_windows < 1) max_windows = 1;
  if (max_slots < ctx->res_slots) max_slots = ctx->res_slots;
  if (max_windows < ctx->res_windows) max_windows = ctx->res_windows;
  const uint64_t tiles = tiles_for(ctx, max_slots, max_windows);
  const uint64_t acc = 4ull * kFixGrid * max_windows;
  const uint64_t chunks = list_chunks_for(max_slots, max_windows);
  if (tiles <= ctx->tile_cap && acc <= ctx->fix_acc_cap && chunks <= ctx->list_counts_cap) {
    ctx->res_slots = max_slots;
    ctx->res_windows = max_windows;
    return RG_OK;
  }
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipDeviceSynchronize());
  ctx->res_slots = 0;  // until every array below is in place
  ctx->res_windows = 0;
  if (tiles > ctx->tile_cap) {
    (void)hipFree(ctx->lookback);
    (void)hipFree(ctx->stats);
    ctx->lookback = nullptr;
    ctx->stats = nullptr;
    ctx->tile_cap = 0;
    RG_HIP(ctx, hipMalloc(&ctx->lookback, tiles * 8));
    RG_HIP(ctx, hipMalloc(&ctx->stats, tiles * kStatGranules * 8));
    // zeroed, so no stale tag can match a live launch sequence number
    RG_HIP(ctx, hipMemset(ctx->lookback, 0, tiles * 8));
    RG_HIP(ctx, hipMemset(ctx->stats, 0, tiles * kStatGranules * 8));
    ctx->tile_cap = tiles;
  }
  if (acc > ctx->fix_acc_cap) {
    (void)hipFree(ctx->fix_acc);
    ctx->fix_acc = nullptr;
    ctx->fix_acc_cap = 0;
    RG_HIP(ctx, hipMalloc(&ctx->fix_acc, acc * sizeof(unsigned long long)));
    ctx->fix_acc_cap = acc;
  }
  if (chunks > ctx->list_counts_cap) {
    (void)hipFree(ctx->list_counts);
    (void)hipFree(ctx->list_nz);
    (void)hipFree(ctx->list_pairs);
    ctx->list_counts = ctx->list_nz = nullptr;
    ctx->list_pairs = nullptr;
    ctx->list_counts_cap = 0;
    RG_HIP(ctx, hipMalloc(&ctx->list_counts, chunks * 4));
    RG_HIP(ctx, hipMalloc(&ctx->list_nz, chunks * 4));
    RG_HIP(ctx, hipMalloc(&ctx->list_pairs, chunks * kListPairs * sizeof(uint2)));
    ctx->list_counts_cap = chunks;
  }
  RG_HIP(ctx, hipDeviceSynchronize());
  ctx->res_slots = max_slots;
  ctx->res_windows = max_windows;
  return RG_OK;
}

int beyond_reservation(rg_ctx* ctx, const char* who) {
  return fail(ctx, RG_EINVAL, std::string(who) + ": the launch exceeds the context's reservation (" +
                                  std::to_string(ctx->res_slots) + " slots, " + std::to_string(ctx->res_windows) +
                                  " windows per call): call rg_reserve first (an _async call never allocates)");
}

// Plane addressing for a buffer of `planes` planes in the context's layout and
// the number of words the buffer must hold for n_words words per plane.
int make_layout(rg_ctx* ctx, uint32_t planes, uint64_t n_words, uint64_t stride, Layout* lay,
                uint64_t* words_needed, const char* who) {
  const uint32_t T = ctx->cfg.tile_words;
  if (T == 0) {
    if (stride % 4 || stride < n_words)
      return fail(ctx, RG_EINVAL, std::string(who) + ": stride_words must be a multiple of 4 and >= ceil(n_slots/32)");
    lay->tshift = 63;
    lay->tmask = ~0ull;
    lay->tile_stride = 0;
    lay->pstride = stride;
    *words_needed = (uint64_t)planes * stride;
  } else {
    if (stride != 0 && stride != T)
      return fail(ctx, RG_EINVAL, std::string(who) + ": slot-tiled layout: stride_words must be 0 or tile_words");
    lay->tshift = (uint32_t)__builtin_ctz(T);
    lay->tmask = T - 1;
    lay->tile_stride = (uint64_t)planes * T;
    lay->pstride = T;
    *words_needed = ((n_words + T - 1) / T) * (uint64_t)planes * T;
  }
  return RG_OK;
}

// Multi-window buffers: window w's copy of a P-plane buffer starts w * pitch words after
// window 0's. Slot-tiled: a window's planes are one block of `need` words, so pitch >=
// need. Planar (plane p of window w at w * pitch + p * stride): either plane-major (the
// windows side by side inside each plane: pitch >= n_words and the last window's words
// end within the plane, (n_win - 1) * pitch + n_words <= stride) or window-major (each
// window's P planes one after another: pitch >= (P - 1) * stride + n_words). Anything
// else aliases some word of two windows, which the fix-up would XOR-patch twice.
bool windows_disjoint(const rg_ctx* ctx, uint32_t planes, uint64_t n_words, uint64_t stride, uint64_t pitch,
                      uint64_t need, uint32_t n_win) {
  if (n_win <= 1) return true;
  if (ctx->cfg.tile_words) return pitch >= need;
  const bool plane_major = pitch >= n_words && (uint64_t)(n_win - 1) * pitch + n_words <= stride;
  const bool window_major = pitch >= (uint64_t)(planes - 1) * stride + n_words;
  return plane_major || window_major;
}

}  // namespace

int rg_set_error(rg_ctx* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }

extern "C" {

int rg_abi_version(void) { return RG_ABI_VERSION; }

uint64_t rg_record_window_words(uint64_t n_slots, uint64_t records_cap) {
  return rec_table_words(n_slots) + records_cap;
}

int rg_device_count(int* out) {
  if (!out) return fail(nullptr, RG_EINVAL, "rg_device_count: null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *out = 0;
    return hip_fail(nullptr, e, "hipGetDeviceCount");
  }
  *out = n;
  return RG_OK;
}

uint64_t rg_plane_stride(uint64_t n_slots) { return ((n_slots + 127) / 128) * 4; }

const char* rg_last_error(const rg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int rg_create(rg_ctx** out, const rg_config* cfg) {
  if (!out || !cfg) return fail(nullptr, RG_EINVAL, "rg_create: null argument");
  *out = nullptr;
  const uint32_t n = cfg->n_replicas;
  if (n < 1 || n > RG_MAX_REPLICAS) return fail(nullptr, RG_EINVAL, "rg_create: n_replicas must be 1..16");
  const uint32_t q = cfg->quorum ? cfg->quorum : n / 2 + 1;
  const uint32_t fp1 = cfg->decide_threshold ? cfg->decide_threshold : (n - 1) / 2 + 1;
  if (q < 1 || q > n) return fail(nullptr, RG_EINVAL, "rg_create: quorum must be 1..n");
  if (fp1 < 1 || fp1 > n) return fail(nullptr, RG_EINVAL, "rg_create: decide_threshold must be 1..n");
  if (cfg->mode != RG_MODE_REF && cfg->mode != RG_MODE_WMVC)
    return fail(nullptr, RG_EINVAL, "rg_create: unknown mode");
  if (cfg->tile_words && (cfg->tile_words < 64 || (cfg->tile_words & (cfg->tile_words - 1))))
    return fail(nullptr, RG_EINVAL, "rg_create: tile_words must be 0 (planar) or a power of two >= 64");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, RG_ENODEV, "rg_create: no HIP device (the evaluator has no CPU fallback)");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, RG_EINVAL, "rg_create: bad device ordinal");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess)
    return fail(nullptr, RG_ENODEV, "rg_create: hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(nullptr, RG_ENODEV, std::string("rg_create: device is ") + prop.gcnArchName +
                                        ", this build targets gfx950 only");
  rg_ctx* ctx = new (std::nothrow) rg_ctx();
  if (!ctx) return fail(nullptr, RG_ENOMEM, "rg_create: host allocation failed");
  ctx->cfg = *cfg;
  ctx->n_cu = prop.multiProcessorCount > 0 ? (uint32_t)prop.multiProcessorCount : 256u;
  ctx->cfg.quorum = q;
  ctx->cfg.decide_threshold = fp1;
  ctx->q = q;
  ctx->fp1 = fp1;
  seed_from_u64(cfg->seed, ctx->ref_key.k);
  seed_from_u64(cfg->coin_seed, ctx->coin_key.k);
  ctx->coin_stream = cfg->epoch | kCoinStreamBit;
  auto bail = [&](hipError_t e, const char* what) {
    int rc = hip_fail(nullptr, e, what);
    rg_destroy(ctx);
    return rc;
  };
  hipError_t e;
  if ((e = hipSetDevice(cfg->device)) != hipSuccess) return bail(e, "hipSetDevice");
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault)) != hipSuccess)
    return bail(e, "hipStreamCreate");
  if (cfg->device < kMaxDevices) {
    DevChain& dc = g_chain[cfg->device];
    std::lock_guard<std::mutex> lk(dc.mu);
    if (!dc.ev && (e = hipEventCreateWithFlags(&dc.ev, hipEventDisableTiming)) != hipSuccess)
      return bail(e, "hipEventCreate(chain)");
    dc.live++;
    ctx->chained = true;
  }
  if ((e = hipMalloc(&ctx->rec, 2 * sizeof(Record))) != hipSuccess) return bail(e, "hipMalloc(rec)");
  if ((e = hipMalloc(&ctx->state, sizeof(DevState))) != hipSuccess) return bail(e, "hipMalloc(state)");
  if ((e = hipMalloc(&ctx->result, sizeof(DevResult))) != hipSuccess) return bail(e, "hipMalloc(result)");
  if ((e = hipMalloc(&ctx->stage_result, 3 * sizeof(DevResult))) != hipSuccess) return bail(e, "hipMalloc(stage_result)");
  if ((e = hipMalloc(&ctx->fix_arrivals, sizeof(unsigned int))) != hipSuccess) return bail(e, "hipMalloc(fix_arrivals)");
  if ((e = hipMemset(ctx->fix_arrivals, 0, sizeof(unsigned int))) != hipSuccess) return bail(e, "init fix_arrivals");
  if ((e = hipMalloc(&ctx->follow_acc, 4ull * kFollowGrid * sizeof(unsigned long long))) != hipSuccess)
    return bail(e, "hipMalloc(follow_acc)");
  Record recs[2] = {fresh_record(), fresh_record()};
  DevState st{0, 0, 1, 0, 0};  // PhaseIds start at 1 (state.rs:59-63)
  DevResult res;
  std::memset(&res, 0, sizeof res);
  if ((e = hipMemcpy(ctx->rec, recs, sizeof recs, hipMemcpyHostToDevice)) != hipSuccess) return bail(e, "init rec");
  if ((e = hipMemcpy(ctx->state, &st, sizeof st, hipMemcpyHostToDevice)) != hipSuccess) return bail(e, "init state");
  if ((e = hipMemcpy(ctx->result, &res, sizeof res, hipMemcpyHostToDevice)) != hipSuccess) return bail(e, "init result");
  if ((e = hipMemset(ctx->stage_result, 0, 3 * sizeof(DevResult))) != hipSuccess) return bail(e, "init stage results");
  if ((e = hipDeviceSynchronize()) != hipSuccess) return bail(e, "init sync");
  if (reserve_impl(ctx, RG_RESERVE_DEFAULT_SLOTS, RG_RESERVE_DEFAULT_WINDOWS) != RG_OK) {
    g_err = ctx->err;
    rg_destroy(ctx);
    return RG_EHIP;
  }
  *out = ctx;
  return RG_OK;
}

int rg_destroy(rg_ctx* ctx) {
  if (!ctx) return RG_OK;
  (void)hipSetDevice(ctx->cfg.device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  rg_comm_release(ctx);
  if (ctx->chained) {
    DevChain& dc = g_chain[ctx->cfg.device];
    std::lock_guard<std::mutex> lk(dc.mu);
    dc.live--;
    if (dc.owner == ctx) dc.owner = nullptr;  // (its launches are complete: the caller synchronised)
  }
  (void)hipFree(ctx->rec);
  (void)hipFree(ctx->state);
  (void)hipFree(ctx->result);
  (void)hipFree(ctx->lookback);
  (void)hipFree(ctx->stats);
  (void)hipFree(ctx->dbg);
  (void)hipFree(ctx->r1v_cells);
  (void)hipFree(ctx->r1v_blocks);
  (void)hipFree(ctx->r1v_base);
  (void)hipFree(ctx->cluster_part);
  (void)hipFree(ctx->cluster_stats);
  (void)hipFree(ctx->fix_acc);
  (void)hipFree(ctx->fix_arrivals);
  (void)hipFree(ctx->list_counts);
  (void)hipFree(ctx->list_nz);
  (void)hipFree(ctx->list_pairs);
  (void)hipFree(ctx->follow_acc);
  (void)hipFree(ctx->stage_result);
  (void)hipFree(ctx->d_votes);
  (void)hipFree(ctx->d_out);
  (void)hipFree(ctx->d_user_result);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RG_OK;
}

int rg_get_config(const rg_ctx* ctx, rg_config* out) {
  if (!ctx || !out) return fail(nullptr, RG_EINVAL, "rg_get_config: null argument");
  *out = ctx->cfg;
  return RG_OK;
}

int rg_set_state(rg_ctx* ctx, const rg_engine_state* st) {
  if (!ctx || !st) return fail(ctx, RG_EINVAL, "rg_set_state: null argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipDeviceSynchronize());
  DevState s{st->rng_next, st->last_committed, st->commit_watermark, st->steps, 0};
  RG_HIP(ctx, hipMemcpy(ctx->state, &s, sizeof s, hipMemcpyHostToDevice));
  return RG_OK;
}

int rg_get_state(rg_ctx* ctx, rg_engine_state* st) {
  if (!ctx || !st) return fail(ctx, RG_EINVAL, "rg_get_state: null argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipDeviceSynchronize());
  DevState s;
  RG_HIP(ctx, hipMemcpy(&s, ctx->state, sizeof s, hipMemcpyDeviceToHost));
  st->rng_next = s.rng_next;
  st->last_committed = s.last_committed;
  st->commit_watermark = s.commit_watermark;
  st->steps = s.steps;
  return RG_OK;
}

// Multi-window sharded launches (rg_phase_step_shard_windows_async): window w at
// votes + w * in_pitch, out + w * out_pitch, slot ids + w * id_stride.
struct WinArgs {
  uint32_t n = 1;
  uint64_t in_pitch = 0, out_pitch = 0, id_stride = 0;
};

static int step_impl(rg_ctx* ctx, const uint32_t* votes_dev, uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
              uint64_t slot_base, uint64_t phase, uint64_t max_phase, rg_step_result* result_dev, void* stream,
              bool shard, uint32_t* records_dev, uint64_t records_cap, WinArgs win = WinArgs()) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_phase_step: null context");
  if (shard && ctx->cfg.mode != RG_MODE_REF)
    return fail(ctx, RG_EINVAL, "rg_phase_step_shard: REF mode only (WMVC coins are shard-invariant already)");
  if (shard && !records_dev) return fail(ctx, RG_EINVAL, "rg_phase_step_shard: null records buffer");
  if (n_slots == 0) return fail(ctx, RG_EINVAL, "rg_phase_step: n_slots must be > 0");
  if (n_slots >= (1ull << 32)) return fail(ctx, RG_EINVAL, "rg_phase_step: n_slots must be < 2^32 per call");
  if (!votes_dev || !out_dev) return fail(ctx, RG_EINVAL, "rg_phase_step: null plane pointer");
  if ((reinterpret_cast<uintptr_t>(votes_dev) | reinterpret_cast<uintptr_t>(out_dev)) & 15u)
    return fail(ctx, RG_EINVAL, "rg_phase_step: plane pointers must be 16-byte aligned");
  const bool wmvc = ctx->cfg.mode == RG_MODE_WMVC;
  if (wmvc && (phase < 1 || phase > (1ull << 24)))
    return fail(ctx, RG_EINVAL, "rg_phase_step: WMVC phase must be 1..2^24");
  if (wmvc && slot_base + n_slots > (1ull << 49))
    return fail(ctx, RG_EINVAL, "rg_phase_step: WMVC slot ids must be < 2^49 (coin counter layout)");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const int n = (int)ctx->cfg.n_replicas;
  const uint64_t n_words = (n_slots + 31) / 32;
  Layout lin, lout;
  uint64_t need_in, need_out;
  if (int rc = make_layout(ctx, 4 * n + 1, n_words, stride_words, &lin, &need_in, "rg_phase_step")) return rc;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need_out, "rg_phase_step")) return rc;
  // window w's planes must not overlap another window's (the fix-up patches them by XOR)
  if (!windows_disjoint(ctx, 4 * n + 1, n_words, stride_words, win.in_pitch, need_in, win.n) ||
      !windows_disjoint(ctx, kOutPlanes, n_words, stride_words, win.out_pitch, need_out, win.n))
    return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: the windows' planes overlap (slot-tiled: pitch >= "
                                "the window's tiles; planar: plane-major, pitch >= ceil(n_slots/32) and "
                                "(n_windows - 1) * pitch + ceil(n_slots/32) <= stride, or window-major, pitch >= "
                                "(planes - 1) * stride + ceil(n_slots/32))");
  uint32_t force = (ctx->diag >> 8) & 7u;  // diagnostics: force a tile shape of the tiled kernel
  if (force > 3) force = 0;
  int cfg = force ? (int)force - 1 : pick_cfg(n, n_words);
  // Large REF launches run the persistent lag kernel (tiles taken by ticket): one
  // 1024-thread workgroup per CU when the launch gives every CU >= 2 such tiles, else
  // two 512-thread workgroups per CU. diag bit 20 keeps the tiled kernel (A/B), bit 21
  // forces the lag kernel at any size, bit 22 forces the 512-thread shape.
  const bool lag_ok = !wmvc && !force && !(ctx->diag & 0x3u);  // (diag 4: stamps, both kernels)
  // (its buffer offsets are 31-bit: every plane of a tile within 2 GiB of the tile base)
  const bool lag_fits = (uint64_t)(4 * n + 1) * lin.pstride * 4 + 4096 < (1ull << 31) &&
                        (uint64_t)kOutPlanes * lout.pstride * 4 + 4096 < (1ull << 31);
  // n <= 10: the lag kernel's planes fit its registers without spills; above that the
  // tiled kernel runs (no configuration of SURVEY.md §8 has n > 9)
  // Measured (tools/ab_variants.py, tools/gpu_c5diag.sh): the lag kernel wins once every
  // CU runs many of its tiles (n = 5: 2^30 slots 700 vs 732 us), the tiled kernel below
  // that (2^28: 195 vs 203; n = 9, 2^26: 90 vs 96; 2^23: 21 vs 41) -> lag from 32
  // 1024-thread tiles per CU. A multi-window shard launch counts all its windows' words
  // (its tickets run through every window): n = 9, 32 windows of 2^23 slots: 0.59 of the
  // HBM peak for one 2^28-slot lag launch against 0.54 for the tiled K-window launch
  // (profiles/r05/c5_probe_n9_k32_before.json).
  const bool mw = shard && win.n > 1;
  const uint64_t launch_words = n_words * (mw ? win.n : 1u);
  const bool lag_big = launch_words >= 32ull * ctx->n_cu * kLagBlock * (uint64_t)lag_words(n);
  const uint64_t tiles_one = (n_words + kLagOneTileWords - 1) / kLagOneTileWords;
  const bool mw_fits = !mw || tiles_one * win.n < (1ull << 30);  // tickets and look-back indices are 31-bit
  const bool lag = lag_fits && mw_fits && n <= 10 &&
                   ((ctx->diag & 0x200000u) ? !wmvc
                                            : (lag_ok && lag_big && !(ctx->diag & 0x100000u) &&
                                               (mw || cfg == kCfgBig)));
  // multi-window launches run only the one-workgroup-per-CU shape
  const bool lag1024 = lag && (mw || (!(ctx->diag & 0x400000u) &&
                                      n_words >= 2ull * ctx->n_cu * kLagBlock * (uint64_t)lag_words(n)));
  uint64_t tile_words = lag ? (lag1024 ? kLagOneTileWords : (uint64_t)kLagBlockSmall * lag_words(n))
                            : (uint64_t)cfg_block(cfg) * cfg_words(cfg, n);
  uint64_t n_tiles = (n_words + tile_words - 1) / tile_words;  // per window
  const uint64_t launch_tiles = n_tiles * (mw ? win.n : 1u);
  const uint32_t grid_force = (ctx->diag >> 24) & 0xFFu;  // diagnostics: lag-kernel grid (tests: many tiles per WG)
  const uint64_t lag_grid_max = grid_force ? grid_force : (lag1024 ? 1ull : 2ull) * ctx->n_cu;
  const uint32_t lag_grid = (uint32_t)(launch_tiles < lag_grid_max ? launch_tiles : lag_grid_max);
  const uint64_t gran_tiles = lag ? (launch_tiles > 3ull * lag_grid ? launch_tiles : 3ull * lag_grid)
                                  : n_tiles * win.n;
  if (gran_tiles > ctx->tile_cap || n_slots * win.n > ctx->res_slots || win.n > ctx->res_windows)
    return beyond_reservation(ctx, "rg_phase_step");
  hipStream_t s = pick_stream(ctx, stream);
  // Statistics granules carry 12 bits of seq and look-back granules 31: start a
  // fresh epoch on zeroed granules whenever either wraps (zeroed on the launch's
  // stream: the context's phase steps are stream-ordered, and nothing else reads them).
  if (++ctx->seq >= (1u << 31) || (ctx->seq & 0xFFFu) == 0) {
    RG_HIP(ctx, hipMemsetAsync(ctx->lookback, 0, ctx->tile_cap * 8, s));
    RG_HIP(ctx, hipMemsetAsync(ctx->stats, 0, ctx->tile_cap * kStatGranules * 8, s));
    ctx->seq = 2 - (ctx->seq & 1u);  // keep the record-ring parity
  }
  StepParams p;
  p.votes = votes_dev;
  p.out = out_dev;
  p.lookback = ctx->lookback;
  p.stats = ctx->stats;
  p.rec = ctx->rec;
  p.state = ctx->state;
  p.result = ctx->result;
  p.result_user = reinterpret_cast<DevResult*>(result_dev);
  p.lin = lin;
  p.lout = lout;
  p.n_slots = n_slots;
  p.n_words = n_words;
  p.slot_base = slot_base;
  p.max_phase = max_phase;
  p.phase = phase;
  p.coin_stream = ctx->coin_stream;
  p.key = wmvc ? ctx->coin_key : ctx->ref_key;
  p.q = ctx->q;
  p.fp1 = ctx->fp1;
  p.self_lane = ctx->cfg.self_lane;
  p.seq = ctx->seq;
  p.n_tiles = (uint32_t)n_tiles;
  p.diag = ctx->diag & 0xffu;
  p.dbg = nullptr;
  p.in_bytes = need_in * 4;
  p.out_bytes = need_out * 4;
  p.vq_rec = records_dev;
  p.vq_cap = records_cap;
  p.rec_tw = (uint32_t)rec_table_words(n_slots);
  p.rec_pitch = p.rec_tw + records_cap;
  p.n_win = win.n;
  p.win_in_pitch = win.in_pitch;
  p.win_out_pitch = win.out_pitch;
  p.win_id_stride = win.id_stride;
  if (ctx->diag & 4u) {  // stamps: [n_tiles][8] (tiled kernel) or [grid][16] (lag kernel)
    const uint64_t words = lag && 16ull * lag_grid > 8 * n_tiles ? 16ull * lag_grid : 8 * n_tiles;
    if (ctx->dbg_cap < words) {
      RG_HIP(ctx, hipDeviceSynchronize());
      (void)hipFree(ctx->dbg);
      ctx->dbg = nullptr;
      RG_HIP(ctx, hipMalloc(&ctx->dbg, words * 8));
      ctx->dbg_cap = words;
    }
    RG_HIP(ctx, hipMemsetAsync(ctx->dbg, 0, words * 8, pick_stream(ctx, stream)));
    p.dbg = ctx->dbg;
  }
  ctx->last_launch[0] = lag ? 1u : (wmvc ? 2u : 0u);
  ctx->last_launch[1] = shard ? 1u : 0u;
  ctx->last_launch[2] = lag ? (uint32_t)(lag1024 ? lag_one_block(n) : kLagBlockSmall) : (uint32_t)cfg_block(cfg);
  ctx->last_launch[3] = lag ? (uint32_t)(lag1024 ? lag_one_words(n) : lag_words(n)) : (uint32_t)cfg_words(cfg, n);
  ctx->last_launch[4] = lag ? lag_grid : (uint32_t)n_tiles;
  ctx->last_launch[5] = win.n;
  std::unique_lock<std::mutex> chain_lk;
  DevChain* dc = (!lag && ctx->chained) ? &g_chain[ctx->cfg.device] : nullptr;
  if (dc) {
    chain_lk = std::unique_lock<std::mutex>(dc->mu);
    if (dc->live < 2) dc = nullptr;
    else if (dc->owner && (dc->owner != ctx || dc->stream != s)) RG_HIP(ctx, hipStreamWaitEvent(s, dc->ev, 0));
  }
  if (shard)
    launch_ref_shard(n, lag ? (mw ? -2 : (lag1024 ? -1 : 0)) : cfg_block(cfg), cfg_words(cfg, n),
                     lag ? lag_grid : (uint32_t)n_tiles, s, p);
  else if (lag1024) kRefLagLaunch[n](lag_grid, s, p);
  else if (lag) kRefLag512Launch[n](lag_grid, s, p);
  else (wmvc ? kWmvcLaunch : kRefLaunch)[n](cfg, (uint32_t)n_tiles, s, p);
  RG_HIP(ctx, hipGetLastError());
  if (dc) {
    RG_HIP(ctx, hipEventRecord(dc->ev, s));
    dc->owner = ctx;
    dc->stream = s;
  }
  return RG_OK;
}

int rg_phase_step_async(rg_ctx* ctx, const uint32_t* votes_dev, uint32_t* out_dev, uint64_t n_slots,
                        uint64_t stride_words, uint64_t slot_base, uint64_t phase, uint64_t max_phase,
                        rg_step_result* result_dev, void* stream) {
  return step_impl(ctx, votes_dev, out_dev, n_slots, stride_words, slot_base, phase, max_phase, result_dev, stream,
                   false, nullptr, 0);
}

int rg_phase_step_shard_async(rg_ctx* ctx, const uint32_t* votes_dev, uint32_t* out_dev, uint64_t n_slots,
                              uint64_t stride_words, uint64_t slot_base, uint64_t max_phase, uint32_t* records_dev,
                              uint64_t records_cap, rg_step_result* row_dev, void* stream) {
  return step_impl(ctx, votes_dev, out_dev, n_slots, stride_words, slot_base, 1, max_phase, row_dev, stream, true,
                   records_dev, records_cap);
}

int rg_phase_step_shard_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* votes_dev,
                                      uint64_t votes_pitch_words, uint32_t* out_dev, uint64_t out_pitch_words,
                                      uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                                      uint64_t window_stride, uint64_t max_phase, uint32_t* records_dev,
                                      uint64_t records_cap, rg_step_result* rows_dev, void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_phase_step_shard_windows: null context");
  if (n_windows < 1 || n_windows > 65535) return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: 1..65535 windows");
  if (n_windows > 1 && !rows_dev) return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: null rows buffer");
  if (n_windows > 1) {
    if ((votes_pitch_words | out_pitch_words) & 3u)
      return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: pitches must be multiples of 4 words (16 B)");
    if (window_stride < n_slots)
      return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: window_stride must be >= n_slots (disjoint windows)");
    if (records_cap && !records_dev) return fail(ctx, RG_EINVAL, "rg_phase_step_shard_windows: null records buffer");
  }
  WinArgs win;
  win.n = n_windows;
  win.in_pitch = votes_pitch_words;
  win.out_pitch = out_pitch_words;
  win.id_stride = window_stride;
  return step_impl(ctx, votes_dev, out_dev, n_slots, stride_words, slot_base, 1, max_phase, rows_dev, stream, true,
                   records_dev, records_cap, win);
}

static int fixup_impl(rg_ctx* ctx, uint32_t n_win, uint32_t* out_dev, uint64_t out_pitch, uint64_t n_slots,
                      uint64_t stride_words, uint64_t slot_base, uint64_t id_stride, uint64_t max_phase,
                      const uint32_t* records_dev, uint64_t records_cap, const rg_step_result* rows_dev,
                      uint32_t shard, uint32_t n_shards, rg_step_result* rows_out_dev, void* stream,
                      hipEvent_t patched = nullptr) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_shard_fixup: null context");
  if (ctx->cfg.mode != RG_MODE_REF) return fail(ctx, RG_EINVAL, "rg_shard_fixup: REF mode only");
  if (!out_dev || !records_dev || !rows_dev || n_shards == 0 || shard >= n_shards || n_slots == 0 || n_win == 0 ||
      n_win > 65535)
    return fail(ctx, RG_EINVAL, "rg_shard_fixup: bad argument");
  if (n_win > 1 && (((out_pitch & 3u) != 0) || id_stride < n_slots))
    return fail(ctx, RG_EINVAL, "rg_shard_fixup_windows: out pitch must be a multiple of 4 words, window_stride >= n_slots");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t n_words = (n_slots + 31) / 32;
  Layout lout;
  uint64_t need;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need, "rg_shard_fixup")) return rc;
  if (!windows_disjoint(ctx, kOutPlanes, n_words, stride_words, out_pitch, need, n_win))
    return fail(ctx, RG_EINVAL, "rg_shard_fixup_windows: the windows' output planes overlap (same rule as the step)");
  // one thread per ChaCha12 block of the records' global positions, grid-stride over
  // at most kFixGrid workgroups (the record count lives on the device)
  const uint64_t rec_most = records_cap < n_slots ? records_cap : n_slots;
  const uint64_t blk_most = rec_most / 8 + 2;
  // at most kFixGrid workgroups over ALL windows (>= 16 per window): the fix-up is launched
  // the moment a step kernel ends, and a grid of n_win x 513 mostly empty workgroups (the
  // record capacity, not the record count, sized it) took the CUs the next step kernel's
  // workgroups were waiting for (20-30 us between step kernels at 32 windows)
  const uint64_t per_win = std::max<uint64_t>(kFixGrid / n_win, 16);
  const uint32_t n_part = (uint32_t)std::min<uint64_t>((blk_most + 255) / 256, per_win);
  if (4ull * n_part * n_win > ctx->fix_acc_cap || n_win > ctx->res_windows)
    return beyond_reservation(ctx, "rg_shard_fixup");
  hipStream_t s = pick_stream(ctx, stream);
  FixParams f;
  f.rec = records_dev;
  f.rows = reinterpret_cast<const DevResult*>(rows_dev);
  f.shard = shard;
  f.n_shards = n_shards;
  f.state = ctx->state;
  f.out = out_dev;
  f.lout = lout;
  f.slot_base = slot_base;
  f.max_phase = max_phase;
  f.vq_cap = records_cap;
  f.key = ctx->ref_key;
  f.acc = ctx->fix_acc;
  f.n_part = n_part;
  f.n_win = n_win;
  f.out_pitch = out_pitch;
  f.id_stride = id_stride;
  f.n_slots = n_slots;
  f.n_words = n_words;
  f.rec_tw = (uint32_t)rec_table_words(n_slots);
  f.rec_pitch = f.rec_tw + records_cap;
  hipLaunchKernelGGL(shard_fixup_kernel, dim3(n_part, n_win), dim3(256), 0, s, f);
  // (the exchange forks the decision lists off here: the outputs are final, the rows not yet)
  if (patched) RG_HIP(ctx, hipEventRecord(patched, s));
  hipLaunchKernelGGL(shard_fixup_finish_kernel, dim3(n_win), dim3(256), 0, s, f, ctx->stage_result + 0,
                     reinterpret_cast<DevResult*>(rows_out_dev), ctx->fix_arrivals);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_shard_fixup_async(rg_ctx* ctx, uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
                         uint64_t slot_base, uint64_t max_phase, const uint32_t* records_dev,
                         uint64_t records_cap, const rg_step_result* rows_dev, uint32_t shard,
                         uint32_t n_shards, rg_step_result* row_dev, void* stream) {
  return fixup_impl(ctx, 1, out_dev, 0, n_slots, stride_words, slot_base, n_slots, max_phase, records_dev, records_cap,
                    rows_dev, shard, n_shards, row_dev, stream);
}

int rg_shard_fixup_fork(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words, uint64_t n_slots,
                        uint64_t stride_words, uint64_t slot_base, uint64_t window_stride, uint64_t max_phase,
                        const uint32_t* records_dev, uint64_t records_cap, const rg_step_result* rows_dev,
                        uint32_t shard, uint32_t n_shards, rg_step_result* rows_out_dev, void* stream,
                        hipEvent_t patched) {
  return fixup_impl(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, slot_base, window_stride,
                    max_phase, records_dev, records_cap, rows_dev, shard, n_shards, rows_out_dev, stream, patched);
}

int rg_shard_fixup_windows_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                 uint64_t n_slots, uint64_t stride_words, uint64_t slot_base, uint64_t window_stride,
                                 uint64_t max_phase, const uint32_t* records_dev, uint64_t records_cap,
                                 const rg_step_result* rows_dev, uint32_t shard, uint32_t n_shards,
                                 rg_step_result* rows_out_dev, void* stream) {
  return fixup_impl(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, slot_base, window_stride,
                    max_phase, records_dev, records_cap, rows_dev, shard, n_shards, rows_out_dev, stream);
}

int rg_follower_commit_async(rg_ctx* ctx, const uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
                             uint64_t slot_base, uint64_t max_phase, uint32_t* applied_dev, uint64_t* gate_dev,
                             rg_step_result* result_dev, void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_follower_commit: null context");
  if (!out_dev || n_slots == 0) return fail(ctx, RG_EINVAL, "rg_follower_commit: bad argument");
  if (n_slots >= (1ull << 32)) return fail(ctx, RG_EINVAL, "rg_follower_commit: n_slots must be < 2^32 per call");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t n_words = (n_slots + 31) / 32;
  Layout lout;
  uint64_t need;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need, "rg_follower_commit")) return rc;
  hipStream_t s = pick_stream(ctx, stream);
  FollowParams f;
  f.out = out_dev;
  f.lout = lout;
  f.n_slots = n_slots;
  f.n_words = n_words;
  f.slot_base = slot_base;
  f.max_phase = max_phase;
  f.state = ctx->state;
  f.applied = applied_dev;
  f.acc = ctx->follow_acc;
  const uint64_t g = (n_words + 255) / 256;
  f.n_part = (uint32_t)(g < kFollowGrid ? g : kFollowGrid);
  hipLaunchKernelGGL(follower_kernel, dim3(f.n_part), dim3(256), 0, s, f);
  hipLaunchKernelGGL(follower_finish_kernel, dim3(1), dim3(256), 0, s, f,
                     reinterpret_cast<unsigned long long*>(gate_dev), ctx->stage_result + 2,
                     reinterpret_cast<DevResult*>(result_dev));
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_shard_commit_impl(rg_ctx* ctx, uint32_t n_windows, const rg_step_result* rows_dev, uint32_t n_shards,
                         uint64_t window_base, uint64_t window_slots, rg_step_result* results_dev, uint64_t und_chk,
                         void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_shard_commit: null context");
  if (!rows_dev || n_shards == 0 || window_slots == 0 || n_windows == 0)
    return fail(ctx, RG_EINVAL, "rg_shard_commit: bad argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(shard_commit_kernel, dim3(1), dim3(kCommitBlock), 0, pick_stream(ctx, stream),
                     reinterpret_cast<const DevResult*>(rows_dev), n_shards, n_windows, window_base, window_slots,
                     ctx->state, ctx->stage_result + 1, reinterpret_cast<DevResult*>(results_dev), und_chk);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_shard_commit_async(rg_ctx* ctx, const rg_step_result* rows_dev, uint32_t n_shards, uint64_t window_base,
                          uint64_t window_slots, rg_step_result* result_dev, void* stream) {
  return rg_shard_commit_impl(ctx, 1, rows_dev, n_shards, window_base, window_slots, result_dev, 0, stream);
}

int rg_shard_commit_windows_async(rg_ctx* ctx, uint32_t n_windows, const rg_step_result* rows_dev, uint32_t n_shards,
                                  uint64_t window_base, uint64_t window_slots, rg_step_result* results_dev,
                                  void* stream) {
  return rg_shard_commit_impl(ctx, n_windows, rows_dev, n_shards, window_base, window_slots, results_dev, 0, stream);
}

int rg_reserve(rg_ctx* ctx, uint64_t max_slots, uint32_t max_windows) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_reserve: null context");
  if (max_slots == 0 || max_slots > (1ull << 40) || max_windows == 0 || max_windows > 65535)
    return fail(ctx, RG_EINVAL, "rg_reserve: 1..2^40 slots, 1..65535 windows");
  return reserve_impl(ctx, max_slots, max_windows);
}

int rg_decision_lists_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* out_dev, uint64_t out_pitch_words,
                                    uint64_t n_slots, uint64_t stride_words, uint32_t* lists_dev, uint32_t cap,
                                    uint32_t* v1_dev, uint64_t v1_pitch_words, void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_decision_lists_windows: null context");
  if (!out_dev || !lists_dev || n_slots == 0 || n_slots >= (1ull << 32) || n_windows == 0 || n_windows > 65535)
    return fail(ctx, RG_EINVAL, "rg_decision_lists_windows: bad argument");
  const uint64_t n_words = (n_slots + 31) / 32;
  if (v1_dev && n_windows > 1 && v1_pitch_words < n_words)
    return fail(ctx, RG_EINVAL, "rg_decision_lists_windows: V1 bitmap pitch < ceil(n_slots/32)");
  Layout lout;
  uint64_t need;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need, "rg_decision_lists_windows"))
    return rc;
  const uint64_t n_chunks = (n_words + kListChunkWords - 1) / kListChunkWords;
  if (n_chunks * n_windows > ctx->list_counts_cap || n_windows > ctx->res_windows)
    return beyond_reservation(ctx, "rg_decision_lists_windows");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  ListParams L;
  L.out = out_dev;
  L.lout = lout;
  L.n_words = n_words;
  L.n_slots = n_slots;
  L.out_pitch = out_pitch_words;
  L.v1 = v1_dev;
  L.v1_pitch = v1_pitch_words;
  L.lists = lists_dev;
  L.cap = cap;
  L.counts = ctx->list_counts;
  L.nz = ctx->list_nz;
  L.pairs = ctx->list_pairs;
  L.n_chunks = (uint32_t)n_chunks;
  hipStream_t s = pick_stream(ctx, stream);
  hipLaunchKernelGGL(list_scan_kernel, dim3((uint32_t)n_chunks, n_windows), dim3(256), 0, s, L);
  hipLaunchKernelGGL(list_emit_kernel, dim3((uint32_t)n_chunks, n_windows), dim3(256), 0, s, L);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_last_result(rg_ctx* ctx, rg_step_result* out_host) {
  if (!ctx || !out_host) return fail(ctx, RG_EINVAL, "rg_last_result: null argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipDeviceSynchronize());
  RG_HIP(ctx, hipMemcpy(out_host, ctx->result, sizeof(DevResult), hipMemcpyDeviceToHost));
  if (out_host->flags) return fail(ctx, RG_ESTATE, "device-side protocol fault (look-back timeout)");
  return RG_OK;
}

int rg_last_stage_result(rg_ctx* ctx, int stage, rg_step_result* out_host) {
  if (!ctx || !out_host) return fail(ctx, RG_EINVAL, "rg_last_stage_result: null argument");
  if (stage < 0 || stage > 2) return fail(ctx, RG_EINVAL, "rg_last_stage_result: stage must be 0..2");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipDeviceSynchronize());
  RG_HIP(ctx, hipMemcpy(out_host, ctx->stage_result + stage, sizeof(DevResult), hipMemcpyDeviceToHost));
  return RG_OK;
}

int rg_phase_step(rg_ctx* ctx, const uint32_t* votes_host, uint32_t* out_host, uint64_t n_slots,
                  uint64_t stride_words, uint64_t slot_base, uint64_t phase, uint64_t max_phase,
                  rg_step_result* result_host) {
  if (!ctx || !votes_host || !out_host) return fail(ctx, RG_EINVAL, "rg_phase_step: null argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t n = ctx->cfg.n_replicas, n_words = (n_slots + 31) / 32;
  Layout lay;
  uint64_t vw, ow;
  if (int rc = make_layout(ctx, (uint32_t)(4 * n + 1), n_words, stride_words, &lay, &vw, "rg_phase_step")) return rc;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lay, &ow, "rg_phase_step")) return rc;
  if (vw > ctx->stage_votes_words) {
    RG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->d_votes);
    ctx->d_votes = nullptr;
    RG_HIP(ctx, hipMalloc(&ctx->d_votes, vw * 4));
    ctx->stage_votes_words = vw;
  }
  if (ow > ctx->stage_out_words) {
    RG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->d_out);
    ctx->d_out = nullptr;
    RG_HIP(ctx, hipMalloc(&ctx->d_out, ow * 4));
    ctx->stage_out_words = ow;
  }
  RG_HIP(ctx, hipMemcpyAsync(ctx->d_votes, votes_host, vw * 4, hipMemcpyHostToDevice, ctx->stream));
  int rc = rg_phase_step_async(ctx, ctx->d_votes, ctx->d_out, n_slots, stride_words, slot_base, phase,
                               max_phase, nullptr, ctx->stream);
  if (rc) return rc;
  RG_HIP(ctx, hipMemcpyAsync(out_host, ctx->d_out, ow * 4, hipMemcpyDeviceToHost, ctx->stream));
  rg_step_result tmp;
  RG_HIP(ctx, hipMemcpyAsync(&tmp, ctx->result, sizeof tmp, hipMemcpyDeviceToHost, ctx->stream));
  RG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (result_host) *result_host = tmp;
  if (tmp.flags) return fail(ctx, RG_ESTATE, "device-side protocol fault (look-back timeout)");
  return RG_OK;
}

int rg_digest_majority_async(rg_ctx* ctx, const uint64_t* digests_dev, uint64_t digest_stride,
                             uint32_t* state_dev, uint64_t n_slots, void* stream) {
  if (!ctx || !digests_dev || !state_dev) return fail(ctx, RG_EINVAL, "rg_digest_majority: null argument");
  if (n_slots == 0 || digest_stride < n_slots) return fail(ctx, RG_EINVAL, "rg_digest_majority: bad sizes");
  if (reinterpret_cast<uintptr_t>(state_dev) & 15u)
    return fail(ctx, RG_EINVAL, "rg_digest_majority: state plane must be 16-byte aligned");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t waves = (n_slots + 127) / 128;
  const uint64_t grid = (waves + kWaves - 1) / kWaves;
  kDigestLaunch[ctx->cfg.n_replicas]((uint32_t)grid, pick_stream(ctx, stream), digests_dev, digest_stride,
                                     state_dev, n_slots, ctx->q);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_coin_async(rg_ctx* ctx, uint64_t slot_base, uint64_t n_slots, uint64_t phase, uint32_t* out_dev,
                  void* stream) {
  if (!ctx || !out_dev || n_slots == 0) return fail(ctx, RG_EINVAL, "rg_coin: bad argument");
  if (phase < 1 || phase > (1ull << 24)) return fail(ctx, RG_EINVAL, "rg_coin: phase must be 1..2^24");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t n_words = (n_slots + 31) / 32;
  hipLaunchKernelGGL(coin_kernel, dim3((uint32_t)((n_words + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), ctx->coin_key, ctx->coin_stream, phase, slot_base, n_slots,
                     out_dev);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_decision_bitmap_async(rg_ctx* ctx, const uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
                             uint32_t* committed_dev, uint32_t* v1_dev, void* stream) {
  if (!ctx || !out_dev || !committed_dev || !v1_dev || n_slots == 0)
    return fail(ctx, RG_EINVAL, "rg_decision_bitmap: bad argument");
  const uint64_t n_words = (n_slots + 31) / 32;
  Layout lout;
  uint64_t need;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need, "rg_decision_bitmap")) return rc;
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(bitmap_kernel, dim3((uint32_t)((n_words + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), out_dev, lout, n_words, committed_dev, v1_dev, 0ull, 0ull);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_decision_bitmap_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* out_dev,
                                     uint64_t out_pitch_words, uint64_t n_slots, uint64_t stride_words,
                                     uint32_t* committed_dev, uint32_t* v1_dev, uint64_t bitmap_pitch_words,
                                     void* stream) {
  if (!ctx || !out_dev || !committed_dev || !v1_dev || n_slots == 0 || n_windows == 0 || n_windows > 65535)
    return fail(ctx, RG_EINVAL, "rg_decision_bitmap_windows: bad argument");
  const uint64_t n_words = (n_slots + 31) / 32;
  if (n_windows > 1 && bitmap_pitch_words < n_words)
    return fail(ctx, RG_EINVAL, "rg_decision_bitmap_windows: bitmap pitch < ceil(n_slots/32)");
  Layout lout;
  uint64_t need;
  if (int rc = make_layout(ctx, kOutPlanes, n_words, stride_words, &lout, &need, "rg_decision_bitmap_windows"))
    return rc;
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(bitmap_kernel, dim3((uint32_t)((n_words + 255) / 256), n_windows), dim3(256), 0,
                     pick_stream(ctx, stream), out_dev, lout, n_words, committed_dev, v1_dev, out_pitch_words,
                     bitmap_pitch_words);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_round1_votes_async(rg_ctx* ctx, const uint64_t* phase_ids_dev, const uint8_t* values_dev, uint64_t n_props,
                          uint32_t* proposed_dev, uint64_t stride_words, uint64_t n_slots, uint64_t slot_base,
                          uint32_t track_proposals, uint8_t* votes_dev, void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_round1_votes: null context");
  if (ctx->cfg.mode != RG_MODE_REF) return fail(ctx, RG_EINVAL, "rg_round1_votes: REF mode only (engine.rs:424-481)");
  if (n_props == 0) return RG_OK;
  if (!phase_ids_dev || !values_dev || !votes_dev || (track_proposals && (!proposed_dev || !n_slots)))
    return fail(ctx, RG_EINVAL, "rg_round1_votes: null buffer");
  if (n_props > (1ull << 31)) return fail(ctx, RG_EINVAL, "rg_round1_votes: more than 2^31 proposals");
  if (track_proposals && (stride_words < (n_slots + 31) / 32))
    return fail(ctx, RG_EINVAL, "rg_round1_votes: stride_words < ceil(n_slots/32)");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint32_t blocks = (uint32_t)((n_props + kR1vBlock - 1) / kR1vBlock);
  if ((track_proposals && n_slots > ctx->r1v_cells_cap) || blocks > ctx->r1v_blocks_cap || !ctx->r1v_base) {
    RG_HIP(ctx, hipDeviceSynchronize());
    if (track_proposals && n_slots > ctx->r1v_cells_cap) {
      (void)hipFree(ctx->r1v_cells);
      ctx->r1v_cells = nullptr;
      ctx->r1v_cells_cap = 0;
      RG_HIP(ctx, hipMalloc(&ctx->r1v_cells, n_slots * 4));
      RG_HIP(ctx, hipMemset(ctx->r1v_cells, 0xFF, n_slots * 4));
      ctx->r1v_cells_cap = n_slots;
    }
    if (blocks > ctx->r1v_blocks_cap) {
      (void)hipFree(ctx->r1v_blocks);
      ctx->r1v_blocks = nullptr;
      ctx->r1v_blocks_cap = 0;
      RG_HIP(ctx, hipMalloc(&ctx->r1v_blocks, (uint64_t)blocks * 4));
      ctx->r1v_blocks_cap = blocks;
    }
    if (!ctx->r1v_base) RG_HIP(ctx, hipMalloc(&ctx->r1v_base, 8));
    RG_HIP(ctx, hipDeviceSynchronize());
  }
  R1vArgs a;
  a.phase_ids = phase_ids_dev;
  a.values = values_dev;
  a.n = n_props;
  a.n_slots = track_proposals ? n_slots : 0;
  a.slot_base = slot_base;
  a.stride = stride_words;
  a.proposed = proposed_dev;
  a.cells = ctx->r1v_cells;
  a.block_draws = ctx->r1v_blocks;
  a.base = ctx->r1v_base;
  a.state = ctx->state;
  a.votes = votes_dev;
  a.key = ctx->ref_key;
  a.track = track_proposals ? 1u : 0u;
  if (!track_proposals) {  // every proposal is "first": no window, all phase ids accepted
    a.slot_base = 0;
    a.n_slots = ~0ull;
  }
  hipStream_t s = pick_stream(ctx, stream);
  hipLaunchKernelGGL(r1v_claim_kernel, dim3(blocks), dim3(kR1vBlock), 0, s, a);
  hipLaunchKernelGGL(r1v_count_kernel, dim3(blocks), dim3(kR1vBlock), 0, s, a);
  hipLaunchKernelGGL(r1v_scan_kernel, dim3(1), dim3(1024), 0, s, a, blocks);
  hipLaunchKernelGGL(r1v_vote_kernel, dim3(blocks), dim3(kR1vBlock), 0, s, a);
  hipLaunchKernelGGL(r1v_reset_kernel, dim3(blocks), dim3(kR1vBlock), 0, s, a);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_ref_draws_async(rg_ctx* ctx, uint64_t first, uint64_t count, uint64_t* out_dev, void* stream) {
  if (!ctx || !out_dev || count == 0) return fail(ctx, RG_EINVAL, "rg_ref_draws: bad argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(draws_kernel, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), ctx->ref_key, first, count,
                     reinterpret_cast<unsigned long long*>(out_dev));
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_trace_generate_async(rg_ctx* ctx, int kind, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                            uint64_t stride_words, uint32_t* votes_dev, void* stream) {
  if (!ctx || !votes_dev || n_slots == 0) return fail(ctx, RG_EINVAL, "rg_trace_generate: bad argument");
  if (kind < 0 || kind > 2) return fail(ctx, RG_EINVAL, "rg_trace_generate: unknown kind");
  const uint64_t n_words = (n_slots + 31) / 32;
  Layout lay;
  uint64_t need;
  if (int rc = make_layout(ctx, 4 * ctx->cfg.n_replicas + 1, n_words, stride_words, &lay, &need, "rg_trace_generate"))
    return rc;
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(trace_kernel, dim3((uint32_t)((n_words + 127) / 128)), dim3(128), 0,
                     pick_stream(ctx, stream), kind, (int)ctx->cfg.n_replicas, seed, slot_base, n_slots,
                     lay, votes_dev);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_digest_trace_async(rg_ctx* ctx, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                          uint64_t digest_stride, uint64_t* digests_dev, void* stream) {
  if (!ctx || !digests_dev || n_slots == 0 || digest_stride < n_slots)
    return fail(ctx, RG_EINVAL, "rg_digest_trace: bad argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(digest_trace_kernel, dim3((uint32_t)((n_slots + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), (int)ctx->cfg.n_replicas, seed, slot_base, n_slots,
                     digest_stride, reinterpret_cast<unsigned long long*>(digests_dev));
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

static int cluster_run(rg_ctx* ctx, const uint32_t* states_dev, uint64_t stride_words, uint64_t n_slots,
                       uint64_t slot_base, uint64_t delivery_seed, uint32_t max_phases, uint32_t* info_dev,
                       uint64_t* stats_dev, uint32_t* decided_dev, uint32_t* v1_dev, void* stream) {
  if (!ctx || !states_dev || !info_dev || n_slots == 0) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster: bad argument");
  if (stride_words < (n_slots + 31) / 32) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster: stride too small");
  if (max_phases < 1 || max_phases > 255) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster: max_phases must be 1..255");
  if (slot_base + n_slots > (1ull << 49)) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster: slot ids must be < 2^49");
  if (n_slots >= (1ull << 32)) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster: n_slots must be < 2^32 per call");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  // one slot per lane to start with, at most 2048 workgroups, unless that leaves a
  // workgroup more than kClusterChunk slots (its initial states are staged in LDS)
  constexpr uint32_t kGrid = 2048;
  const uint64_t need = (n_slots + 255) / 256;
  const uint64_t by_chunk = (n_slots + kClusterChunk - 1) / kClusterChunk;
  uint64_t g64 = need < kGrid ? need : kGrid;
  if (g64 < by_chunk) g64 = by_chunk;
  const uint32_t grid = (uint32_t)g64;
  if (grid > ctx->cluster_part_cap) {
    RG_HIP(ctx, hipDeviceSynchronize());
    (void)hipFree(ctx->cluster_part);
    ctx->cluster_part = nullptr;
    ctx->cluster_part_cap = 0;
    RG_HIP(ctx, hipMalloc(&ctx->cluster_part, (uint64_t)grid * kClusterStats * 8));
    ctx->cluster_part_cap = grid;
  }
  if (!ctx->cluster_stats) RG_HIP(ctx, hipMalloc(&ctx->cluster_stats, kClusterStats * 8));
  hipStream_t s = pick_stream(ctx, stream);
  // coin bits of the first phases from per-workgroup LDS tables (one ChaCha12 block per
  // 512 slots and phase instead of one per lane and phase); later phases (rare) compute inline
#ifndef RG_COIN_TABLE_PHASES
#define RG_COIN_TABLE_PHASES 8
#endif
  static_assert(RG_COIN_TABLE_PHASES <= kClusterCoinPhases, "the cluster kernel's LDS coin table holds kClusterCoinPhases");
  constexpr uint32_t kCoinTablePhases = RG_COIN_TABLE_PHASES;
  const uint32_t coin_phases = max_phases < kCoinTablePhases ? max_phases : kCoinTablePhases;
  // whole bitmap words per workgroup (<= kClusterChunk still: grid >= n_slots / kClusterChunk
  // and kClusterChunk is a multiple of 32); trailing workgroups may get an empty chunk
  const uint64_t chunk = ((n_slots + grid - 1) / grid + 31) / 32 * 32;
  kClusterLcLaunch[ctx->cfg.n_replicas](grid, s, states_dev, stride_words, n_slots, slot_base, ctx->q, ctx->fp1,
                                        ctx->coin_key, ctx->coin_stream, delivery_seed, max_phases, info_dev,
                                        ctx->cluster_part, coin_phases, chunk, decided_dev, v1_dev);
  unsigned long long* dst = stats_dev ? reinterpret_cast<unsigned long long*>(stats_dev) : ctx->cluster_stats;
  hipLaunchKernelGGL(cluster_stats_kernel, dim3(1), dim3(kStatsBlock), 0, s, ctx->cluster_part, grid, dst);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_wmvc_cluster_async(rg_ctx* ctx, const uint32_t* states_dev, uint64_t stride_words, uint64_t n_slots,
                          uint64_t slot_base, uint64_t delivery_seed, uint32_t max_phases, uint32_t* info_dev,
                          uint64_t* stats_dev, void* stream) {
  return cluster_run(ctx, states_dev, stride_words, n_slots, slot_base, delivery_seed, max_phases, info_dev,
                     stats_dev, nullptr, nullptr, stream);
}

int rg_wmvc_cluster_bitmaps_async(rg_ctx* ctx, const uint32_t* states_dev, uint64_t stride_words, uint64_t n_slots,
                                  uint64_t slot_base, uint64_t delivery_seed, uint32_t max_phases,
                                  uint32_t* info_dev, uint64_t* stats_dev, uint32_t* decided_dev, uint32_t* v1_dev,
                                  void* stream) {
  if (!decided_dev || !v1_dev) return fail(ctx, RG_EINVAL, "rg_wmvc_cluster_bitmaps: null bitmap");
  return cluster_run(ctx, states_dev, stride_words, n_slots, slot_base, delivery_seed, max_phases, info_dev,
                     stats_dev, decided_dev, v1_dev, stream);
}

int rg_cluster_bitmap_async(rg_ctx* ctx, const uint32_t* info_dev, uint64_t n_slots, uint32_t* decided_dev,
                            uint32_t* v1_dev, void* stream) {
  if (!ctx || !info_dev || !decided_dev || !v1_dev || n_slots == 0)
    return fail(ctx, RG_EINVAL, "rg_cluster_bitmap: bad argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(cluster_bitmap_kernel, dim3((uint32_t)((n_slots + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), info_dev, n_slots, decided_dev, v1_dev);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_cluster_trace_async(rg_ctx* ctx, uint64_t seed, uint64_t slot_base, uint64_t n_slots, uint64_t stride_words,
                           uint32_t* states_dev, void* stream) {
  if (!ctx || !states_dev || n_slots == 0 || stride_words < (n_slots + 31) / 32)
    return fail(ctx, RG_EINVAL, "rg_cluster_trace: bad argument");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  const uint64_t n_words = (n_slots + 31) / 32;
  hipLaunchKernelGGL(cluster_trace_kernel, dim3((uint32_t)((n_words + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), (int)ctx->cfg.n_replicas, seed, slot_base, n_slots, stride_words,
                     states_dev);
  RG_HIP(ctx, hipGetLastError());
  return RG_OK;
}

int rg_stream_sync(rg_ctx* ctx, void* stream) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_stream_sync: null context");
  RG_HIP(ctx, hipSetDevice(ctx->cfg.device));
  RG_HIP(ctx, hipStreamSynchronize(pick_stream(ctx, stream)));
  return RG_OK;
}

int rg_pack_codes(const uint8_t* codes, uint32_t n, uint64_t n_slots, uint64_t stride, uint32_t* planes) {
  if (!codes || !planes || n < 1 || n > RG_MAX_REPLICAS || stride < (n_slots + 31) / 32)
    return fail(nullptr, RG_EINVAL, "rg_pack_codes: bad argument");
  std::memset(planes, 0, sizeof(uint32_t) * stride * 2 * n);
  for (uint64_t s = 0; s < n_slots; s++) {
    const uint8_t* c = codes + s * n;
    const uint32_t bit = 1u << (s & 31);
    for (uint32_t j = 0; j < n; j++) {
      if (c[j] & 1u) planes[(uint64_t)(2 * j) * stride + s / 32] |= bit;
      if (c[j] & 2u) planes[(uint64_t)(2 * j + 1) * stride + s / 32] |= bit;
    }
  }
  return RG_OK;
}

int rg_unpack_planes(const uint32_t* planes, uint32_t n, uint64_t n_slots, uint64_t stride, uint8_t* codes) {
  if (!codes || !planes || n < 1 || n > RG_MAX_REPLICAS || stride < (n_slots + 31) / 32)
    return fail(nullptr, RG_EINVAL, "rg_unpack_planes: bad argument");
  for (uint64_t s = 0; s < n_slots; s++) {
    const uint32_t sh = (uint32_t)(s & 31);
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t lo = (planes[(uint64_t)(2 * j) * stride + s / 32] >> sh) & 1u;
      const uint32_t hi = (planes[(uint64_t)(2 * j + 1) * stride + s / 32] >> sh) & 1u;
      codes[s * n + j] = (uint8_t)(lo | (hi << 1));
    }
  }
  return RG_OK;
}

int rg_planar_to_tiled(const uint32_t* planar, uint32_t n_planes, uint64_t n_words, uint64_t stride,
                       uint32_t tile_words, uint32_t* tiled) {
  if (!planar || !tiled || !n_planes || stride < n_words || tile_words < 64 || (tile_words & (tile_words - 1)))
    return fail(nullptr, RG_EINVAL, "rg_planar_to_tiled: bad argument");
  const uint64_t T = tile_words, n_t = (n_words + T - 1) / T;
  std::memset(tiled, 0, sizeof(uint32_t) * n_t * n_planes * T);
  for (uint64_t t = 0; t < n_t; t++)
    for (uint32_t pl = 0; pl < n_planes; pl++) {
      const uint64_t w_lo = t * T, cnt = (w_lo + T <= n_words) ? T : n_words - w_lo;
      std::memcpy(tiled + (t * n_planes + pl) * T, planar + pl * stride + w_lo, cnt * 4);
    }
  return RG_OK;
}

int rg_tiled_to_planar(const uint32_t* tiled, uint32_t n_planes, uint64_t n_words, uint32_t tile_words,
                       uint64_t stride, uint32_t* planar) {
  if (!planar || !tiled || !n_planes || stride < n_words || tile_words < 64 || (tile_words & (tile_words - 1)))
    return fail(nullptr, RG_EINVAL, "rg_tiled_to_planar: bad argument");
  const uint64_t T = tile_words, n_t = (n_words + T - 1) / T;
  std::memset(planar, 0, sizeof(uint32_t) * n_planes * stride);
  for (uint64_t t = 0; t < n_t; t++)
    for (uint32_t pl = 0; pl < n_planes; pl++) {
      const uint64_t w_lo = t * T, cnt = (w_lo + T <= n_words) ? T : n_words - w_lo;
      std::memcpy(planar + pl * stride + w_lo, tiled + (t * n_planes + pl) * T, cnt * 4);
    }
  return RG_OK;
}

// ---- diagnostics (include/rabia_gpu_debug.h) ---------------------------------
int rg_debug_set(rg_ctx* ctx, uint32_t diag) {
  if (!ctx) return fail(nullptr, RG_EINVAL, "rg_debug_set: null context");
  ctx->diag = diag;
  return RG_OK;
}

int rg_debug_last_launch(const rg_ctx* ctx, uint32_t* out6) {
  if (!ctx || !out6) return fail(nullptr, RG_EINVAL, "rg_debug_last_launch: null argument");
  std::memcpy(out6, ctx->last_launch, sizeof ctx->last_launch);
  return RG_OK;
}

int rg_debug_stamps(rg_ctx* ctx, uint64_t* host_out, uint64_t n_words) {
  if (!ctx || !host_out) return fail(ctx, RG_EINVAL, "rg_debug_stamps: null argument");
  if (!ctx->dbg) return fail(ctx, RG_EINVAL, "rg_debug_stamps: no stamps recorded (diag & 4)");
  RG_HIP(ctx, hipDeviceSynchronize());
  const uint64_t n = n_words < ctx->dbg_cap ? n_words : ctx->dbg_cap;
  RG_HIP(ctx, hipMemcpy(host_out, ctx->dbg, n * 8, hipMemcpyDeviceToHost));
  return RG_OK;
}

int rg_debug_stream_probe(const uint32_t* in_dev, uint32_t* out_dev, uint64_t n_words, uint64_t stride,
                          uint32_t tile_words, uint32_t nt, void* stream) {
  if (!in_dev || !out_dev || n_words % 4 || stride % 4 || (tile_words && (tile_words % 4 || n_words % tile_words)))
    return fail(nullptr, RG_EINVAL, "rg_debug_stream_probe: bad arguments");
  const dim3 grid((uint32_t)((n_words + 1023) / 1024));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (nt) hipLaunchKernelGGL((stream_probe_kernel<20, 8, true>), grid, dim3(256), 0, s, in_dev, out_dev, stride, n_words, tile_words);
  else hipLaunchKernelGGL((stream_probe_kernel<20, 8, false>), grid, dim3(256), 0, s, in_dev, out_dev, stride, n_words, tile_words);
  RG_HIP(nullptr, hipGetLastError());
  return RG_OK;
}

}  // extern "C"
