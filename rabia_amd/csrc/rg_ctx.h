// rg_ctx.h — the context behind the C ABI's opaque rg_ctx (private to the library's
// translation units: rabia_gpu.hip owns it, rg_comm.hip attaches the RCCL exchange).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "rabia_gpu.h"
#include "rg_common.h"

struct RgComm;  // rg_comm.hip

struct rg_ctx {
  rg_config cfg{};
  uint32_t q = 0, fp1 = 0;
  rg::Key ref_key{}, coin_key{};
  uint64_t coin_stream = 0;
  hipStream_t stream = nullptr;
  rg::Record* rec = nullptr;
  rg::DevState* state = nullptr;
  rg::DevResult* result = nullptr;
  unsigned long long* lookback = nullptr;
  unsigned long long* stats = nullptr;
  uint64_t tile_cap = 0;
  uint32_t seq = 0;
  uint32_t* d_votes = nullptr;
  uint32_t* d_out = nullptr;
  rg::DevResult* d_user_result = nullptr;
  uint64_t stage_votes_words = 0, stage_out_words = 0;
  uint32_t diag = 0;
  unsigned long long* dbg = nullptr;
  uint64_t dbg_cap = 0;
  uint32_t* r1v_cells = nullptr;   // round-1 votes: per-slot claim cells (0xFFFFFFFF)
  uint64_t r1v_cells_cap = 0;
  uint32_t* r1v_blocks = nullptr;  // per-block draw counts / offsets
  uint64_t r1v_blocks_cap = 0;
  unsigned long long* r1v_base = nullptr;
  unsigned long long* cluster_part = nullptr;  // [blocks][kClusterStats]
  uint64_t cluster_part_cap = 0;                // blocks
  unsigned long long* cluster_stats = nullptr;  // [kClusterStats]
  unsigned long long* fix_acc = nullptr;        // sharded REF fix-up partials [windows][kFixGrid][4]
  uint64_t fix_acc_cap = 0;                     // u64 elements
  unsigned int* fix_arrivals = nullptr;         // fix-up finish: workgroups arrived (reset by the last)
  uint32_t* list_counts = nullptr;              // decision lists: per-chunk undecided counts,
  uint32_t* list_nz = nullptr;                  //   words holding one, and their (word, mask)
  uint2* list_pairs = nullptr;                  //   pairs [chunks][kListPairs]
  uint64_t list_counts_cap = 0;                 // chunks
  // rg_reserve: the largest launch the context's scratch is sized for (slots over all
  // windows of one call, windows of one call); *_async calls past it return RG_EINVAL
  uint64_t res_slots = 0;
  uint32_t res_windows = 0;
  unsigned long long* follow_acc = nullptr;     // follower commit partials [kFollowGrid][4]
  // results of the shard fix-up / shard commit / follower commit: each stage writes
  // its own (a fix-up may run on another stream than the next window's step, whose
  // result is ctx->result, the one rg_last_result reads)
  rg::DevResult* stage_result = nullptr;        // [3]
  uint32_t n_cu = 256;                          // compute units (persistent lag-kernel grid)
  bool chained = false;                         // counted in g_chain[device].live
  uint32_t last_launch[6] = {};                 // rg_debug_last_launch: kind, shard, block, words, grid, windows
  RgComm* comm = nullptr;                       // RCCL communicator and exchange scratch (rg_comm.hip)
  std::string err;
};

// rg_comm.hip: releases the context's communicator (rg_destroy)
void rg_comm_release(rg_ctx* ctx);
// rabia_gpu.hip: records msg as the context's (or the thread's) last error, returns code
int rg_set_error(rg_ctx* ctx, int code, const std::string& msg);
// rabia_gpu.hip: rg_shard_commit_windows_async with the undecided-list check: und_chk =
// list capacity + 1 flags (32) a window where some shard has more undecided slots than
// the capacity; 0 = no check
extern "C" int rg_shard_commit_impl(rg_ctx* ctx, uint32_t n_windows, const rg_step_result* rows_dev,
                                    uint32_t n_shards, uint64_t window_base, uint64_t window_slots,
                                    rg_step_result* results_dev, uint64_t und_chk, void* stream);
// rabia_gpu.hip: rg_shard_fixup_windows_async that also records `patched` on the stream
// between the re-draw kernel (the outputs final) and the finish kernel (the final rows)
extern "C" int rg_shard_fixup_fork(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                   uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                                   uint64_t window_stride, uint64_t max_phase, const uint32_t* records_dev,
                                   uint64_t records_cap, const rg_step_result* rows_dev, uint32_t shard,
                                   uint32_t n_shards, rg_step_result* rows_out_dev, void* stream,
                                   hipEvent_t patched);
