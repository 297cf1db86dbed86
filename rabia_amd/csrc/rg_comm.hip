// rg_comm.hip — the multi-GPU exchange of the sharded REF pipeline behind the C ABI
// (include/rabia_gpu.h, "Multi-GPU exchange"): an RCCL communicator attached to a
// context, and the all-gathers of the shard rows, the final rows and the decision
// bitmaps on the caller's stream. It replaces, for the decided-slot exchange,
// NetworkTransport::broadcast (rabia-core/src/network.rs:36-51): instead of every
// engine broadcasting its decisions message by message, each GPU's rows and bitmaps
// for a batch of windows travel in one ncclAllGather over xGMI.
//
// RCCL is loaded at run time (dlopen of the ROCm install's librccl, symbols resolved
// from that handle): the library needs no RCCL to load, a process that never creates a
// communicator never initialises one, and the symbols cannot bind to another RCCL copy
// a host process may carry (torch bundles its own).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "rg_ctx.h"

using rg::DevResult;

namespace {

struct Rccl {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string load_error;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

// Loads RCCL once per process: $RG_RCCL_LIB, else the ROCm install's librccl.so.1.
const Rccl* rccl() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.h) return &g_rccl;
  if (!g_rccl.load_error.empty()) return nullptr;
  const char* env = std::getenv("RG_RCCL_LIB");
  const char* cands[] = {env, "/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"};
  std::string tried;
  for (const char* c : cands) {
    if (!c || !*c) continue;
    void* h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      tried += std::string(" ") + c + " (" + dlerror() + ")";
      continue;
    }
    Rccl r;
    r.h = h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    if (r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.all_reduce && r.error_string) {
      g_rccl = r;
      return &g_rccl;
    }
    tried += std::string(" ") + c + " (missing symbols)";
    dlclose(h);
  }
  g_rccl.load_error = "RCCL not loadable:" + tried;
  return nullptr;
}

std::string rccl_msg(const Rccl* r, ncclResult_t e, const char* what) {
  return std::string(what) + ": " + (r ? r->error_string(e) : "RCCL not loaded");
}

}  // namespace

struct RgComm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  DevResult* rows_all = nullptr;   // [world][windows] shard rows (stage 2)
  DevResult* fixed = nullptr;      // [windows] this rank's final rows (stage 3)
  DevResult* fixed_all = nullptr;  // [world][windows] final rows (stage 4)
  uint32_t res_windows = 0;        // rg_comm_reserve: windows per call the rows are sized for
  uint32_t* payload = nullptr;     // this rank's decision payload (bitmaps, or lists + V1 bitmaps)
  uint64_t payload_cap = 0;        // words
  double* scalars = nullptr;       // rg_comm_barrier / rg_comm_max_f64 (device, 64 doubles)
  // rg_shard_exchange_decisions_async forks the decision lists onto `aux` once the fix-up's
  // re-draw has patched the outputs, so they run beside the finish, the final-row gather and
  // the commit (each of those a short latency-bound kernel or collective), and joins them
  // before the payload gather
  hipStream_t aux = nullptr;
  hipEvent_t ev_patched = nullptr, ev_lists = nullptr;
};

constexpr uint32_t kCommScalars = 64;
constexpr uint32_t kCommDefaultWindows = 128;

void rg_comm_release(rg_ctx* ctx) {
  if (!ctx || !ctx->comm) return;
  RgComm* c = ctx->comm;
  const Rccl* r = rccl();
  if (c->comm && r) r->comm_destroy(c->comm);
  (void)hipFree(c->rows_all);
  (void)hipFree(c->fixed);
  (void)hipFree(c->fixed_all);
  (void)hipFree(c->payload);
  (void)hipFree(c->scalars);
  if (c->ev_patched) (void)hipEventDestroy(c->ev_patched);
  if (c->ev_lists) (void)hipEventDestroy(c->ev_lists);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  delete c;
  ctx->comm = nullptr;
}

namespace {

int need_comm(rg_ctx* ctx, const char* who) {
  if (!ctx) return rg_set_error(nullptr, RG_EINVAL, std::string(who) + ": null context");
  if (!ctx->comm) return rg_set_error(ctx, RG_EINVAL, std::string(who) + ": no communicator (rg_comm_create)");
  return RG_OK;
}

int hip_err(rg_ctx* ctx, hipError_t e, const char* what) {
  return rg_set_error(ctx, RG_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Reserve the rows for max_windows windows and a payload of payload_words words (grow
// only; the caller synchronised the device). The capacities are published only once every
// array is in place, so a failed allocation leaves no array the capacity claims.
int comm_reserve_impl(rg_ctx* ctx, uint32_t max_windows, uint64_t payload_words) {
  RgComm* c = ctx->comm;
  hipError_t e;
  if (max_windows > c->res_windows) {
    const uint64_t n = (uint64_t)max_windows * (uint64_t)c->world;
    c->res_windows = 0;
    DevResult** arrs[3] = {&c->rows_all, &c->fixed, &c->fixed_all};
    for (DevResult** a : arrs) {
      (void)hipFree(*a);
      *a = nullptr;
    }
    for (DevResult** a : arrs)
      if ((e = hipMalloc(reinterpret_cast<void**>(a), n * sizeof(DevResult))) != hipSuccess)
        return hip_err(ctx, e, "hipMalloc(exchange rows)");
    c->res_windows = max_windows;
  }
  if (payload_words > c->payload_cap) {
    (void)hipFree(c->payload);
    c->payload = nullptr;
    c->payload_cap = 0;
    if ((e = hipMalloc(&c->payload, payload_words * 4)) != hipSuccess) return hip_err(ctx, e, "hipMalloc(exchange payload)");
    c->payload_cap = payload_words;
  }
  return RG_OK;
}

int comm_beyond(rg_ctx* ctx, const char* who) {
  return rg_set_error(ctx, RG_EINVAL, std::string(who) + ": the exchange exceeds the communicator's reservation (" +
                                          std::to_string(ctx->comm->res_windows) + " windows, " +
                                          std::to_string(ctx->comm->payload_cap) +
                                          " payload words): call rg_comm_reserve first (an _async call never allocates)");
}

int gather(rg_ctx* ctx, const void* send, void* recv, uint64_t bytes, hipStream_t s, const char* what) {
  const Rccl* r = rccl();
  if (!r) return rg_set_error(ctx, RG_EHIP, g_rccl.load_error);
  // 8-byte elements when the payload allows it (rows), else bytes (bitmaps: 4-byte words)
  const bool wide = bytes % 8 == 0;
  const ncclResult_t e = r->all_gather(send, recv, wide ? bytes / 8 : bytes, wide ? ncclUint64 : ncclUint8,
                                       ctx->comm->comm, s);
  if (e != ncclSuccess) return rg_set_error(ctx, RG_EHIP, rccl_msg(r, e, what));
  return RG_OK;
}

// Stages 2-4 of a K-window step: the rows all-gathered (rank-major [world][K]), this
// shard's VQ slots re-drawn at their global positions, the final rows all-gathered and
// folded window by window into the engine state and results_dev[K].
int exchange_rows(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words, uint64_t n_slots,
                  uint64_t stride_words, uint64_t slot_base, uint64_t window_base, uint64_t window_slots,
                  uint64_t max_phase, const uint32_t* records_dev, uint64_t records_cap, const rg_step_result* rows_dev,
                  rg_step_result* results_dev, uint64_t und_chk, hipStream_t s, hipEvent_t patched = nullptr) {
  RgComm* c = ctx->comm;
  const uint64_t row_bytes = (uint64_t)n_windows * sizeof(DevResult);
  if (int rc = gather(ctx, rows_dev, c->rows_all, row_bytes, s, "ncclAllGather(rows)")) return rc;
  if (int rc = rg_shard_fixup_fork(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, slot_base,
                                   window_slots, max_phase, records_dev, records_cap,
                                   reinterpret_cast<const rg_step_result*>(c->rows_all), (uint32_t)c->rank,
                                   (uint32_t)c->world, reinterpret_cast<rg_step_result*>(c->fixed), s, patched))
    return rc;
  if (int rc = gather(ctx, c->fixed, c->fixed_all, row_bytes, s, "ncclAllGather(final rows)")) return rc;
  return rg_shard_commit_impl(ctx, n_windows, reinterpret_cast<const rg_step_result*>(c->fixed_all),
                              (uint32_t)c->world, window_base, window_slots, results_dev, und_chk, s);
}

}  // namespace

extern "C" {

int rg_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return rg_set_error(nullptr, RG_EINVAL, "rg_comm_unique_id: null argument");
  const Rccl* r = rccl();
  if (!r) return rg_set_error(nullptr, RG_EHIP, g_rccl.load_error);
  ncclUniqueId id;
  const ncclResult_t e = r->get_unique_id(&id);
  if (e != ncclSuccess) return rg_set_error(nullptr, RG_EHIP, rccl_msg(r, e, "ncclGetUniqueId"));
  static_assert(sizeof id == RG_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof id);
  return RG_OK;
}

int rg_comm_create(rg_ctx* ctx, const uint8_t* id, int rank, int world) {
  if (!ctx || !id) return rg_set_error(ctx, RG_EINVAL, "rg_comm_create: null argument");
  if (world < 1 || rank < 0 || rank >= world) return rg_set_error(ctx, RG_EINVAL, "rg_comm_create: bad rank / world");
  if (ctx->comm) return rg_set_error(ctx, RG_EINVAL, "rg_comm_create: the context already has a communicator");
  const Rccl* r = rccl();
  if (!r) return rg_set_error(ctx, RG_EHIP, g_rccl.load_error);
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  RgComm* c = new (std::nothrow) RgComm();
  if (!c) return rg_set_error(ctx, RG_ENOMEM, "rg_comm_create: host allocation failed");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  const ncclResult_t e = r->comm_init_rank(&c->comm, world, uid, rank);
  if (e != ncclSuccess) {
    delete c;
    return rg_set_error(ctx, RG_EHIP, rccl_msg(r, e, "ncclCommInitRank"));
  }
  c->rank = rank;
  c->world = world;
  if ((he = hipMalloc(&c->scalars, kCommScalars * sizeof(double))) != hipSuccess) {
    r->comm_destroy(c->comm);
    delete c;
    return hip_err(ctx, he, "hipMalloc(comm scalars)");
  }
  ctx->comm = c;
  if ((he = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking)) != hipSuccess ||
      (he = hipEventCreateWithFlags(&c->ev_patched, hipEventDisableTiming)) != hipSuccess ||
      (he = hipEventCreateWithFlags(&c->ev_lists, hipEventDisableTiming)) != hipSuccess) {
    rg_comm_release(ctx);
    return hip_err(ctx, he, "rg_comm_create: aux stream / events");
  }
  if (int rc = comm_reserve_impl(ctx, kCommDefaultWindows, 0)) {
    rg_comm_release(ctx);
    return rc;
  }
  return RG_OK;
}

int rg_comm_reserve(rg_ctx* ctx, uint32_t max_windows, uint64_t max_slots, uint32_t undecided_cap) {
  if (int rc = need_comm(ctx, "rg_comm_reserve")) return rc;
  if (max_windows == 0 || max_windows > 65535 || max_slots == 0 || max_slots >= (1ull << 32))
    return rg_set_error(ctx, RG_EINVAL, "rg_comm_reserve: 1..65535 windows, 1..2^32-1 slots per window");
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  if ((he = hipDeviceSynchronize()) != hipSuccess) return hip_err(ctx, he, "hipDeviceSynchronize");
  const uint64_t nw = (max_slots + 31) / 32, K = max_windows;
  const uint64_t bitmaps = K * 2 * nw, lists = K * (1 + (uint64_t)undecided_cap) + K * nw;
  if (int rc = comm_reserve_impl(ctx, max_windows, bitmaps > lists ? bitmaps : lists)) return rc;
  // the calls the exchange makes on the context (fix-up partials, decision lists)
  return rg_reserve(ctx, max_slots * K, max_windows);
}

int rg_comm_destroy(rg_ctx* ctx) {
  if (!ctx) return rg_set_error(nullptr, RG_EINVAL, "rg_comm_destroy: null context");
  (void)hipSetDevice(ctx->cfg.device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  rg_comm_release(ctx);
  return RG_OK;
}

int rg_comm_rank(const rg_ctx* ctx, int* rank, int* world) {
  if (!ctx || !rank || !world) return rg_set_error(nullptr, RG_EINVAL, "rg_comm_rank: null argument");
  if (!ctx->comm) return rg_set_error(const_cast<rg_ctx*>(ctx), RG_EINVAL, "rg_comm_rank: no communicator");
  *rank = ctx->comm->rank;
  *world = ctx->comm->world;
  return RG_OK;
}

int rg_comm_allgather_async(rg_ctx* ctx, const void* send_dev, void* recv_dev, uint64_t bytes, void* stream) {
  if (int rc = need_comm(ctx, "rg_comm_allgather")) return rc;
  if (!send_dev || !recv_dev || bytes == 0) return rg_set_error(ctx, RG_EINVAL, "rg_comm_allgather: bad argument");
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  return gather(ctx, send_dev, recv_dev, bytes, s, "ncclAllGather");
}

int rg_shard_exchange_windows_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                    uint64_t n_slots, uint64_t stride_words, uint64_t slot_base, uint64_t window_base,
                                    uint64_t window_slots, uint64_t max_phase, const uint32_t* records_dev,
                                    uint64_t records_cap, const rg_step_result* rows_dev, rg_step_result* results_dev,
                                    uint32_t* bitmaps_all_dev, void* stream) {
  if (int rc = need_comm(ctx, "rg_shard_exchange_windows")) return rc;
  if (!rows_dev || !results_dev || n_windows == 0 || n_windows > 65535 || n_slots == 0 || window_slots < n_slots)
    return rg_set_error(ctx, RG_EINVAL, "rg_shard_exchange_windows: bad argument");
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  RgComm* c = ctx->comm;
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  const uint64_t K = n_windows, nw = (n_slots + 31) / 32;
  if (n_windows > c->res_windows || (bitmaps_all_dev && K * 2 * nw > c->payload_cap))
    return comm_beyond(ctx, "rg_shard_exchange_windows");
  if (int rc = exchange_rows(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, slot_base, window_base,
                             window_slots, max_phase, records_dev, records_cap, rows_dev, results_dev, 0, s))
    return rc;
  if (bitmaps_all_dev) {  // committed / V1 bitmaps of every shard, [world][K][2][words]
    if (int rc = rg_decision_bitmap_windows_async(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words,
                                                  c->payload, c->payload + nw, 2 * nw, s))
      return rc;
    if (int rc = gather(ctx, c->payload, bitmaps_all_dev, K * 2 * nw * 4, s, "ncclAllGather(bitmaps)")) return rc;
  }
  return RG_OK;
}

int rg_shard_exchange_decisions_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                      uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                                      uint64_t window_base, uint64_t window_slots, uint64_t max_phase,
                                      const uint32_t* records_dev, uint64_t records_cap,
                                      const rg_step_result* rows_dev, rg_step_result* results_dev,
                                      uint32_t undecided_cap, uint32_t with_v1, uint32_t* decisions_all_dev,
                                      void* stream) {
  if (int rc = need_comm(ctx, "rg_shard_exchange_decisions")) return rc;
  if (!rows_dev || !results_dev || !decisions_all_dev || n_windows == 0 || n_windows > 65535 || n_slots == 0 ||
      n_slots >= (1ull << 32) || window_slots < n_slots)
    return rg_set_error(ctx, RG_EINVAL, "rg_shard_exchange_decisions: bad argument");
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  RgComm* c = ctx->comm;
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
  const uint64_t K = n_windows, nw = (n_slots + 31) / 32, lw = 1 + (uint64_t)undecided_cap;
  const uint64_t P = K * lw + (with_v1 ? K * nw : 0);  // payload words per rank
  if (n_windows > c->res_windows) return comm_beyond(ctx, "rg_shard_exchange_decisions");
  // stages 2-4; the commit flags (32) a window where a shard has more undecided slots than a list holds
  if (int rc = exchange_rows(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, slot_base, window_base,
                             window_slots, max_phase, records_dev, records_cap, rows_dev, results_dev,
                             (uint64_t)undecided_cap + 1, s, c->ev_patched))
    return rc;
  // this rank's payload (K lists, then with_v1 K V1 bitmaps) built in place at its own slot of
  // the receive buffer, on the aux stream from the moment the outputs are patched, and one
  // in-place all-gather once both branches are done: no scratch, no local copy of it
  uint32_t* mine = decisions_all_dev + (uint64_t)c->rank * P;
  if ((he = hipStreamWaitEvent(c->aux, c->ev_patched, 0)) != hipSuccess) return hip_err(ctx, he, "hipStreamWaitEvent");
  if (int rc = rg_decision_lists_windows_async(ctx, n_windows, out_dev, out_pitch_words, n_slots, stride_words, mine,
                                               undecided_cap, with_v1 ? mine + K * lw : nullptr, nw, c->aux))
    return rc;
  if ((he = hipEventRecord(c->ev_lists, c->aux)) != hipSuccess) return hip_err(ctx, he, "hipEventRecord");
  if ((he = hipStreamWaitEvent(s, c->ev_lists, 0)) != hipSuccess) return hip_err(ctx, he, "hipStreamWaitEvent");
  return gather(ctx, mine, decisions_all_dev, P * 4, s, "ncclAllGather(decisions)");
}

int rg_comm_barrier(rg_ctx* ctx) {
  if (int rc = need_comm(ctx, "rg_comm_barrier")) return rc;
  const Rccl* r = rccl();
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  // no exchange of this communicator may still run on another stream (include/rabia_gpu.h)
  if ((he = hipDeviceSynchronize()) != hipSuccess) return hip_err(ctx, he, "hipDeviceSynchronize");
  const ncclResult_t e = r->all_reduce(ctx->comm->scalars, ctx->comm->scalars, 1, ncclFloat64, ncclMax,
                                       ctx->comm->comm, ctx->stream);
  if (e != ncclSuccess) return rg_set_error(ctx, RG_EHIP, rccl_msg(r, e, "ncclAllReduce(barrier)"));
  if ((he = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_err(ctx, he, "hipStreamSynchronize");
  return RG_OK;
}

int rg_comm_max_f64(rg_ctx* ctx, double* values, uint32_t count) {
  if (int rc = need_comm(ctx, "rg_comm_max_f64")) return rc;
  if (!values || count == 0 || count > kCommScalars)
    return rg_set_error(ctx, RG_EINVAL, "rg_comm_max_f64: 1..64 values");
  const Rccl* r = rccl();
  hipError_t he = hipSetDevice(ctx->cfg.device);
  if (he != hipSuccess) return hip_err(ctx, he, "hipSetDevice");
  if ((he = hipDeviceSynchronize()) != hipSuccess) return hip_err(ctx, he, "hipDeviceSynchronize");
  double* d = ctx->comm->scalars;
  if ((he = hipMemcpyAsync(d, values, count * sizeof(double), hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
    return hip_err(ctx, he, "hipMemcpyAsync");
  const ncclResult_t e = r->all_reduce(d, d, count, ncclFloat64, ncclMax, ctx->comm->comm, ctx->stream);
  if (e != ncclSuccess) return rg_set_error(ctx, RG_EHIP, rccl_msg(r, e, "ncclAllReduce(max)"));
  if ((he = hipMemcpyAsync(values, d, count * sizeof(double), hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
    return hip_err(ctx, he, "hipMemcpyAsync");
  if ((he = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_err(ctx, he, "hipStreamSynchronize");
  return RG_OK;
}

}  // extern "C"
