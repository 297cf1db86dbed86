/*
 * rabia_gpu.h — C ABI of the MI355X batched Rabia phase evaluator.
 *
 * Drop-in boundary for the phase-evaluation step of rabia-rs's RabiaEngine
 * (reference @ /root/reference). One call evaluates, for every slot (PhaseId)
 * of a window, what the reference's handlers compute for that slot one
 * message at a time:
 *
 *   handle_vote_round1 / has_round1_majority  rabia-engine/src/engine.rs:483-509,
 *                                              rabia-core/src/messages.rs:177-211
 *   proceed_to_round2 + randomized round-2     engine.rs:511-611
 *   handle_vote_round2 / make_decision         engine.rs:613-682
 *   PhaseData::set_decision                    messages.rs:217-222
 *   EngineState::commit_phase (watermark)      rabia-engine/src/state.rs:65-103
 *   Weak-MVC rounds + common coin (WMVC mode)  docs/weak_mvc.ivy:109-191
 *
 * Plain C types only (no HIP/torch types): streams are passed as `void*`
 * (a hipStream_t; NULL = the context's own stream, a blocking stream: it orders
 * with the legacy default stream, e.g. torch's default-stream fills). Every entry point returns
 * RG_OK (0) or a negative rg_status; rg_last_error() gives the text. No entry
 * point throws, retains a caller pointer past return, or falls back to the CPU:
 * without a usable gfx950 device rg_create fails with RG_ENODEV.
 *
 * Vote codes (StateValue serde variant order, rabia-core/src/types.rs:286-294):
 *   V0 = 0, V1 = 1, VQuestion = 2, 3 = absent voter / None / pending.
 *
 * Layout: bit-sliced planes of 32-bit words; slot s of a
 * window is bit (s % 32) of word (s / 32). Plane pointers must be 16-B aligned;
 * a step reads and writes whole 16-B groups (128 slots), so windows sharing a buffer
 * start on 128-slot boundaries.
 * Two plane arrangements, chosen per context by rg_config.tile_words:
 *  - planar (tile_words = 0): plane p starts at p * stride_words; stride_words is
 *    a multiple of 4 and >= ceil(n_slots/32) (rg_plane_stride() gives the minimum);
 *  - slot-tiled (tile_words = T, a power of two >= 64): the window is cut into
 *    slot tiles of 32*T slots; the planes of one tile are stored back to back, so
 *    word w of plane p is at (w / T) * (P * T) + p * T + (w % T) for a buffer of P
 *    planes, and a buffer holds ceil(ceil(n_slots/32) / T) * P * T words.
 *    stride_words arguments must be 0 or T. This is the faster arrangement
 *    (one contiguous region per tile; tools/probe_layout.py).
 *   votes  = (4n + 1) planes: [0, 2n)   round-1 received votes, lane j at 2j (bit0), 2j+1 (bit1)
 *                             [2n, 4n)  round-2 received votes, same order
 *                             4n        WMVC own state bit (unused in REF mode)
 *   output = 8 planes: 0-1 round-1 result code, 2-3 own round-2 vote code,
 *            4-5 decision code, 6 committed (decision in {V0,V1}),
 *            7 value (REF: decision == V1, i.e. batch applied; WMVC: next state).
 * Replica lane j = position of the voter's NodeId in the sorted cluster membership.
 */
#ifndef RABIA_GPU_H
#define RABIA_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_ABI_VERSION 6  /* 6: 4-B draw records in per-window regions (rg_record_window_words) */
#define RG_MAX_REPLICAS 16
#define RG_OUT_PLANES 8
/* rg_create's scratch reservation (rg_reserve): launches of up to 2^32 slots over up to
 * 128 windows per call. */
#define RG_RESERVE_DEFAULT_SLOTS (1ull << 32)
#define RG_RESERVE_DEFAULT_WINDOWS 128u

typedef struct rg_ctx rg_ctx;

typedef enum rg_status {
  RG_OK = 0,
  RG_EINVAL = -1,  /* bad argument (maps to RabiaError::Internal)               */
  RG_EHIP = -2,    /* HIP runtime error                                         */
  RG_ENOMEM = -3,  /* device allocation failed                                  */
  RG_ENODEV = -4,  /* no gfx950 device                                          */
  RG_ESTATE = -5,  /* device-side protocol fault (e.g. look-back timeout)       */
} rg_status;

typedef enum rg_mode {
  RG_MODE_REF = 0,  /* what engine.rs computes (majority quorum, biased StdRng draw) */
  RG_MODE_WMVC = 1, /* Weak-MVC of the paper / weak_mvc.ivy (f+1 decide, common coin) */
} rg_mode;

typedef enum rg_trace_kind {
  RG_TRACE_UNIFORM = 0, /* every code uniform over {V0,V1,VQ,absent}              */
  RG_TRACE_AGREE90 = 1, /* per-slot majority value, each vote agrees w.p. 0.9       */
  RG_TRACE_SPLIT = 2,   /* adversarial split round 1, all-VQ round 2                */
} rg_trace_kind;

/* Mirrors RabiaConfig (rabia-engine/src/config.rs:4-37) + ClusterConfig
 * (rabia-core/src/network.rs:7-21) fields the path reads. */
typedef struct rg_config {
  uint32_t n_replicas;       /* ClusterConfig.all_nodes.len(), 1..16               */
  uint32_t quorum;           /* 0 => n/2 + 1 (network.rs:15)                       */
  uint32_t decide_threshold; /* WMVC f+1; 0 => (n-1)/2 + 1                         */
  int32_t self_lane;         /* this node's lane, -1 = none                        */
  uint32_t mode;             /* rg_mode                                            */
  int32_t device;            /* HIP device ordinal                                 */
  uint64_t seed;             /* RabiaConfig.randomization_seed (StdRng)            */
  uint64_t coin_seed;        /* WMVC cluster-wide common-coin seed                 */
  uint64_t epoch;            /* WMVC configuration epoch (coin stream)             */
  uint32_t tile_words;       /* plane layout: 0 = planar, else slot-tiled (see top) */
  uint32_t reserved;
} rg_config;

/* Per-step result (host or device memory). flags (nonzero = RG_ESTATE; values OR'ed):
 *   1  look-back wait timed out (a predecessor tile never published)
 *   2  statistics fold timed out (a workgroup's granules never arrived)
 *   4  stale launch-record ring (a step ran while the previous launch's record was live)
 *   8  draw-record overflow (shard step: n_draws > records_cap; set by the fix-up)
 *   16 the shard rows do not tile the window (commit: their n_slots sum != window_slots)
 *   32 undecided-list overflow (exchange: some shard has more undecided slots than the
 *      list capacity; its list is truncated, the rows and state are still exact) */
typedef struct rg_step_result {
  uint64_t n_slots;
  uint64_t n_decided;          /* PhaseData.is_committed slots                      */
  uint64_t n_v1;               /* decision V1 (batch applied via apply_commands)    */
  uint64_t n_pending_r1;       /* round-1 result not yet available                  */
  uint64_t n_draws;            /* REF StdRng draws / WMVC coin flips consumed       */
  uint64_t last_committed_max; /* EngineState.last_committed_phase after the step   */
  uint64_t first_undecided;    /* min slot id not committed (or slot_base+n_slots)  */
  uint64_t rng_next;           /* REF draw index after the step                     */
  uint64_t commit_watermark;   /* contiguous total-order watermark after the step   */
  uint64_t flags;              /* nonzero = device-side fault (RG_ESTATE)           */
} rg_step_result;

/* Device-resident engine state carried across steps (EngineState mirror,
 * rabia-engine/src/state.rs:13-29): next StdRng draw index,
 * last_committed_phase, contiguous commit watermark (first slot id not yet
 * known decided; PhaseIds start at 1). */
typedef struct rg_engine_state {
  uint64_t rng_next;
  uint64_t last_committed;
  uint64_t commit_watermark;
  uint64_t steps;
} rg_engine_state;

int rg_abi_version(void);
int rg_device_count(int* out);
uint64_t rg_plane_stride(uint64_t n_slots);

int rg_create(rg_ctx** out, const rg_config* cfg);
int rg_destroy(rg_ctx* ctx);
const char* rg_last_error(const rg_ctx* ctx);
int rg_get_config(const rg_ctx* ctx, rg_config* out);

/* Scratch reservation. The phase-step, sharded-pipeline and decision-list entry points
 * (rg_phase_step*_async, rg_shard_fixup*_async, rg_shard_commit*_async,
 * rg_decision_lists_windows_async, and the exchange calls below with rg_comm_reserve)
 * NEVER allocate or synchronise the device: their scratch is sized here, and a call past
 * the reservation returns RG_EINVAL (nothing enqueued). rg_reserve sizes it for calls of
 * up to max_slots slots (over all windows of one call) and max_windows windows; it only
 * grows, and it synchronises the device (it frees buffers launches in flight may use),
 * so call it before a pipeline starts. rg_create reserves RG_RESERVE_DEFAULT_SLOTS /
 * RG_RESERVE_DEFAULT_WINDOWS. (The round-1 vote, cluster, kv and ingest entry points
 * still grow their scratch on first use of a larger size, synchronising the device.) */
int rg_reserve(rg_ctx* ctx, uint64_t max_slots, uint32_t max_windows);

/* Engine state (synchronous w.r.t. the context's stream). */
int rg_set_state(rg_ctx* ctx, const rg_engine_state* st);
int rg_get_state(rg_ctx* ctx, rg_engine_state* st);

/* Phase step over one slot window [slot_base, slot_base + n_slots).
 * `phase` is the WMVC phase number (>= 1; ignored in REF). `max_phase` is
 * EngineState.current_phase for commit_phase's ordering check (state.rs:70-75);
 * 0 disables it. Phase steps on one context must be stream-ordered (they share the
 * context's launch records). Steps of different contexts may be issued on
 * concurrent streams of one device: large REF launches take their tiles by ticket,
 * so no launch waits on a tile another launch keeps off the GPU; the tiled kernels
 * of smaller launches rely on dispatch order, so while several contexts live on a
 * device the library chains those launches behind each other (one event per device;
 * DESIGN.md §4). Processes sharing one GPU must order such launches themselves.
 *  _async: device pointers, enqueued on `stream`; result_dev may be NULL
 *          (then fetch it with rg_last_result: the last phase step's result).
 *  plain : host pointers; copies in, runs, copies out, synchronises. */
int rg_phase_step_async(rg_ctx* ctx, const uint32_t* votes_dev, uint32_t* out_dev,
                        uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                        uint64_t phase, uint64_t max_phase, rg_step_result* result_dev,
                        void* stream);
int rg_phase_step(rg_ctx* ctx, const uint32_t* votes_host, uint32_t* out_host,
                  uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                  uint64_t phase, uint64_t max_phase, rg_step_result* result_host);
int rg_last_result(rg_ctx* ctx, rg_step_result* out_host);
/* The latest result of a later stage, synchronising the device: stage 0 = the shard
 * fix-up's final row (rg_shard_fixup*_async), 1 = the shard commit's global result
 * (rg_shard_commit*_async; of the last window), 2 = the follower commit's result
 * (rg_follower_commit_async). For callers that pass NULL row/result pointers. */
int rg_last_stage_result(rg_ctx* ctx, int stage, rg_step_result* out_host);

/* ---- Sharded REF: ONE engine (one StdRng stream, engine.rs:59-62) over a window
 * split into contiguous shards, one per GPU. Draw k of shard r is
 * the engine's draw  rng_next + (VQ slots of shards 0..r-1) + k  — ascending slot
 * order over the whole window, as one evaluator (engine.rs:567-611). Per window:
 *  1. every shard: rg_phase_step_shard_async — evaluates its slots with draws taken
 *     at a provisional position (no cross-GPU wait), writes one 4-B draw record per
 *     VQ slot into its record region (records_dev: rg_record_window_words(n_slots,
 *     records_cap) u32 words, a segment table then records_cap records; records_cap =
 *     n_slots always suffices) and its row (rg_step_result): counts, extremes and
 *     n_draws of its NON-VQ slots.
 *     Draw-record overflow (n_draws > records_cap: the records past the cap are not
 *     written) is NOT flagged in this row: the step cannot know it before its
 *     statistics fold. The fix-up flags it (flags value 8) in its final row, and the
 *     commit carries the bit into the window's result, so a caller checks the
 *     fix-up's or the commit's row, not the step's;
 *  2. exchange the rows (all-gather, rank order) -> rows_dev[n_shards];
 *  3. every shard: rg_shard_fixup_async — re-draws its VQ slots at their global
 *     positions, XOR-patches the output bits that change, and writes its final row
 *     (VQ slots counted in; rng_next = the engine position after the window); the
 *     context's rng_next advances past every shard's draws;
 *  4. exchange the final rows; every shard: rg_shard_commit_async folds them into
 *     the context's engine state (last_committed, contiguous watermark, steps),
 *     leaving every rank's state equal to one evaluator's over the whole window.
 * Steps (1) never wait on (2)-(4), so they pipeline: the output buffer of a window
 * must not be reused before its fix-up ran. Stage (1) may run on one stream while
 * (3)-(4) of earlier windows run on another: each stage writes only the engine
 * fields it owns (shard_draws; rng_next; last_committed / watermark / steps) and its
 * own context-internal scratch. Each stage's calls must be stream-ordered among
 * themselves, and (3)/(4) of a window after (3)/(4) of the window before it.
 * row_dev / result_dev may be NULL: the context then keeps the latest fix-up's and
 * commit's result for rg_last_stage_result (rg_last_result returns phase steps'
 * results only — a fix-up may run on another stream than the next window's step). */
/* u32 words of one window's draw-record region: the segment table (one word per 2^24
 * slots + 1, rounded up to 4) followed by records_cap records. A record: bits 0-23 the VQ
 * slot's offset inside its 2^24-slot segment, bits 24-30 the class / both decisions / the
 * provisional own vote (rabia_amd/csrc/rg_common.h). */
uint64_t rg_record_window_words(uint64_t n_slots, uint64_t records_cap);
int rg_phase_step_shard_async(rg_ctx* ctx, const uint32_t* votes_dev, uint32_t* out_dev,
                              uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                              uint64_t max_phase, uint32_t* records_dev, uint64_t records_cap,
                              rg_step_result* row_dev, void* stream);
/* Stage (1) for n_windows consecutive windows of this shard in ONE launch (the shard
 * step's fixed ramp/drain cost is paid once, not per window): window w's shard is
 * [slot_base + w * window_stride, + n_slots), its planes at votes_dev + w *
 * votes_pitch_words / out_dev + w * out_pitch_words (each a buffer in the context
 * layout, stride_words as for one window), its record region at records_dev + w *
 * rg_record_window_words(n_slots, records_cap), its row at rows_dev[w] (required).
 * Equivalent to n_windows calls of rg_phase_step_shard_async in window order, except
 * that every window takes its provisional draws from the same position and
 * shard_draws does not advance (the
 * fix-up re-draws every VQ slot at its global position, so the fixed outputs, rows
 * and engine state are the same). Stages (2)-(4) then run per window as above, with
 * that window's out buffer, records and rows. The context's last result is the last
 * window's row. For n_windows > 1 no word may belong to two windows, else RG_EINVAL
 * (overlapping windows would be patched twice by the fix-up). Slot-tiled: pitch >= the
 * window's tiles x planes x tile_words. Planar (plane p of window w at w * pitch + p *
 * stride_words), one of: plane-major, pitch >= ceil(n_slots/32) and (n_windows - 1) *
 * pitch + ceil(n_slots/32) <= stride_words; window-major, pitch >= (planes - 1) *
 * stride_words + ceil(n_slots/32). */
int rg_phase_step_shard_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* votes_dev,
                                      uint64_t votes_pitch_words, uint32_t* out_dev, uint64_t out_pitch_words,
                                      uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                                      uint64_t window_stride, uint64_t max_phase, uint32_t* records_dev,
                                      uint64_t records_cap, rg_step_result* rows_dev, void* stream);
int rg_shard_fixup_async(rg_ctx* ctx, uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
                         uint64_t slot_base, uint64_t max_phase, const uint32_t* records_dev,
                         uint64_t records_cap, const rg_step_result* rows_dev, uint32_t shard,
                         uint32_t n_shards, rg_step_result* row_dev, void* stream);
/* Stages (3) and (4) for n_windows consecutive windows at once (after
 * rg_phase_step_shard_windows_async): rows_dev = every shard's n_windows rows,
 * rank-major [n_shards][n_windows] (one all-gather of each shard's rows); window w's
 * outputs at out_dev + w * out_pitch_words, its slot ids + w * window_stride, its
 * record region at records_dev + w * rg_record_window_words(n_slots, records_cap);
 * rows_out_dev[w] = its final row. The
 * commit folds [n_shards][n_windows] final rows window by window (window w =
 * [window_base + w * window_slots, + window_slots)) into results_dev[w]. Equivalent
 * to the per-window calls in window order. window_slots of the commit must equal the
 * window_stride the step and the fix-up were given (window w's slot ids), and
 * out_pitch_words obeys the step's pitch rule. */
int rg_shard_fixup_windows_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                 uint64_t n_slots, uint64_t stride_words, uint64_t slot_base, uint64_t window_stride,
                                 uint64_t max_phase, const uint32_t* records_dev, uint64_t records_cap,
                                 const rg_step_result* rows_dev, uint32_t shard, uint32_t n_shards,
                                 rg_step_result* rows_out_dev, void* stream);
int rg_shard_commit_windows_async(rg_ctx* ctx, uint32_t n_windows, const rg_step_result* rows_dev, uint32_t n_shards,
                                  uint64_t window_base, uint64_t window_slots, rg_step_result* results_dev,
                                  void* stream);
int rg_shard_commit_async(rg_ctx* ctx, const rg_step_result* rows_dev, uint32_t n_shards,
                          uint64_t window_base, uint64_t window_slots, rg_step_result* result_dev,
                          void* stream);

/* ---- Multi-GPU exchange (RCCL over xGMI). Replaces, for the decided-slot exchange of
 * the sharded pipeline, NetworkTransport::broadcast (rabia-core/src/network.rs:36-51):
 * each GPU's rows and decision bitmaps for a batch of windows travel in one
 * ncclAllGather instead of per-decision messages. One context per rank, each on its own
 * GPU. Rank 0 makes the 128-byte id (rg_comm_unique_id) and the host's own channel
 * (the reference's TCP transport, a rendezvous store) carries it to every rank; every
 * rank then calls rg_comm_create (collective: it returns when all ranks joined). RCCL
 * is loaded at run time ($RG_RCCL_LIB, else the ROCm install's librccl.so.1); the
 * library itself needs no RCCL until rg_comm_unique_id / rg_comm_create.
 * Exchange calls of one context must be stream-ordered among themselves (they share the
 * communicator's scratch) and follow the stage rules above. Their scratch is sized by
 * rg_comm_reserve (synchronous; rg_comm_create reserves rows for 128 windows and no
 * decision payload); an exchange past the reservation returns RG_EINVAL. */
#define RG_COMM_ID_BYTES 128
int rg_comm_unique_id(uint8_t* id_out /* RG_COMM_ID_BYTES */);
int rg_comm_create(rg_ctx* ctx, const uint8_t* id /* RG_COMM_ID_BYTES */, int rank, int world);
int rg_comm_destroy(rg_ctx* ctx); /* also done by rg_destroy */
int rg_comm_rank(const rg_ctx* ctx, int* rank, int* world);
/* Size the exchange scratch for up to max_windows windows per call, shards of up to
 * max_slots slots per window, and undecided lists of up to undecided_cap entries (also
 * covers the committed + V1 bitmap payload of rg_shard_exchange_windows_async). Grows
 * only; synchronises the device. Also reserves the context (rg_reserve) for the calls. */
int rg_comm_reserve(rg_ctx* ctx, uint32_t max_windows, uint64_t max_slots, uint32_t undecided_cap);
/* Rank-ordered all-gather: recv_dev = world x `bytes` (send_dev of rank r at r x bytes). */
int rg_comm_allgather_async(rg_ctx* ctx, const void* send_dev, void* recv_dev, uint64_t bytes, void* stream);
/* Stages (2)-(4) of the sharded pipeline for n_windows windows of this rank's shard
 * (shard = comm rank, n_shards = comm world), after rg_phase_step_shard_async (n_windows
 * = 1) or rg_phase_step_shard_windows_async: rows_dev = the step's n_windows rows; the
 * rows are all-gathered, the shard's VQ slots re-drawn (rg_shard_fixup_windows_async:
 * out_dev / out_pitch_words / n_slots / stride_words / slot_base / max_phase / records
 * as the step had them, window_stride = window_slots), the final rows all-gathered and
 * folded (rg_shard_commit_windows_async over windows [window_base + w * window_slots,
 * + window_slots)) into results_dev[w], identical on every rank. bitmaps_all_dev
 * (optional) receives every rank's committed and V1 bitmaps, [world][n_windows][2]
 * [ceil(n_slots/32)] words (rg_decision_bitmap_windows_async's payload). */
int rg_shard_exchange_windows_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                    uint64_t n_slots, uint64_t stride_words, uint64_t slot_base, uint64_t window_base,
                                    uint64_t window_slots, uint64_t max_phase, const uint32_t* records_dev,
                                    uint64_t records_cap, const rg_step_result* rows_dev, rg_step_result* results_dev,
                                    uint32_t* bitmaps_all_dev, void* stream);
/* The same stages (2)-(4), with the decided-slot payload as undecided lists instead of
 * committed bitmaps (rg_decision_lists_windows_async per rank, one all-gather): every
 * rank receives decisions_all_dev = [world][P] u32 words, P = n_windows * (1 +
 * undecided_cap) + (with_v1 ? n_windows * ceil(n_slots/32) : 0): rank r's undecided list
 * of window w at r * P + w * (1 + undecided_cap) (count, then up to undecided_cap slot
 * offsets from rank r's shard start, ascending), then, with_v1, its V1 bitmap of window w
 * at r * P + n_windows * (1 + undecided_cap) + w * ceil(n_slots/32). A slot of rank r's
 * shard is committed iff it is not listed; the lists are complete iff no result has flags
 * value 32 (then fetch the bitmaps: rg_decision_bitmap_windows_async + an all-gather).
 * with_v1 = 0 for callers that apply only their own shard's batches (the lists and rows
 * still give every rank the global commit order and watermark). */
int rg_shard_exchange_decisions_async(rg_ctx* ctx, uint32_t n_windows, uint32_t* out_dev, uint64_t out_pitch_words,
                                      uint64_t n_slots, uint64_t stride_words, uint64_t slot_base,
                                      uint64_t window_base, uint64_t window_slots, uint64_t max_phase,
                                      const uint32_t* records_dev, uint64_t records_cap,
                                      const rg_step_result* rows_dev, rg_step_result* results_dev,
                                      uint32_t undecided_cap, uint32_t with_v1, uint32_t* decisions_all_dev,
                                      void* stream);
/* Host-synchronous helpers for the caller's control loop (bench timing, shutdown):
 * a barrier over all ranks, and the element-wise max over ranks of 1..64 host doubles.
 * Both synchronise the device first (so no exchange of the communicator is still running
 * on another stream when their collective starts), then run on the context's stream. */
int rg_comm_barrier(rg_ctx* ctx);
int rg_comm_max_f64(rg_ctx* ctx, double* values, uint32_t count);

/* Follower side of a decided window (RabiaEngine::handle_decision,
 * engine.rs:708-746): the window's decisions, as an output buffer in the context's
 * layout (plane 6 committed, plane 7 V1), applied in ascending PhaseId order. A V1
 * batch is applied iff its PhaseId > last_committed (engine.rs:723-728); within one
 * window that gate is last_committed at the window's start (the context's state at
 * call time), since every batch applied in the window is below the later slots.
 * last_committed then advances as commit_phase does (max, refused above max_phase;
 * state.rs:65-103), the contiguous watermark as in a phase step.
 *  applied_dev (optional): one plane of ceil(n_slots/32) words, the applied bits;
 *  gate_dev (optional): receives last_committed before the window — the gate
 *    rg_kv_mark_applied_async (rabia_kv.h) takes;
 *  result_dev (optional): n_decided = committed slots, n_v1 = batches applied. */
int rg_follower_commit_async(rg_ctx* ctx, const uint32_t* out_dev, uint64_t n_slots,
                             uint64_t stride_words, uint64_t slot_base, uint64_t max_phase,
                             uint32_t* applied_dev, uint64_t* gate_dev,
                             rg_step_result* result_dev, void* stream);

/* Exchange stage: state bit = 1 iff some proposal digest is held by >= quorum
 * replicas (weak_mvc.ivy:109-128). digests_dev = [n][digest_stride] u64 (0 = no
 * proposal received), state_dev = one plane of stride_words. */
int rg_digest_majority_async(rg_ctx* ctx, const uint64_t* digests_dev,
                             uint64_t digest_stride, uint32_t* state_dev,
                             uint64_t n_slots, void* stream);

/* Common coin bits for slots [slot_base, slot_base+n_slots) at `phase` (>=1). */
int rg_coin_async(rg_ctx* ctx, uint64_t slot_base, uint64_t n_slots, uint64_t phase,
                  uint32_t* out_dev, void* stream);

/* Own round-1 votes for received proposals, in message order (REF mode):
 * RabiaEngine::handle_propose -> determine_round1_vote / randomized_vote
 * (engine.rs:380-481). phase_ids_dev[m], values_dev[m] (StateValue code) of
 * proposal m; votes_dev[m] receives the vote code to send back (3 = phase id
 * outside [slot_base, slot_base + n_slots)). track_proposals = 1: the window's
 * PhaseData exist and record proposed_value in proposed_dev (2 planar planes of
 * stride_words, lo/hi bit of the code, 3 = none; updated in place): a slot's first
 * proposal takes randomized_vote (V0: StdRng draw < P70 -> V0 else VQuestion; V1:
 * draw < P80 -> V1 else VQuestion; VQuestion: no draw), later ones vote the
 * proposed value if equal, else VQuestion. track_proposals = 0 restates the
 * reference as it runs (phases are never created, state.rs:166-185): every
 * proposal takes randomized_vote; proposed_dev / n_slots / slot_base are ignored.
 * Draws come from the engine stream in message order and advance rng_next. */
int rg_round1_votes_async(rg_ctx* ctx, const uint64_t* phase_ids_dev, const uint8_t* values_dev,
                          uint64_t n_props, uint32_t* proposed_dev, uint64_t stride_words,
                          uint64_t n_slots, uint64_t slot_base, uint32_t track_proposals,
                          uint8_t* votes_dev, void* stream);

/* Decision bitmaps of a step's output buffer (layout as the context's): committed
 * (output plane 6) and V1/apply (plane 7) as contiguous bit arrays of
 * ceil(n_slots/32) words each — the per-shard payload of the multi-GPU exchange. */
int rg_decision_bitmap_async(rg_ctx* ctx, const uint32_t* out_dev, uint64_t n_slots, uint64_t stride_words,
                             uint32_t* committed_dev, uint32_t* v1_dev, void* stream);
/* The same for n_windows windows (outputs at out_dev + w * out_pitch_words, bitmaps
 * at committed_dev / v1_dev + w * bitmap_pitch_words). */
int rg_decision_bitmap_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* out_dev,
                                     uint64_t out_pitch_words, uint64_t n_slots, uint64_t stride_words,
                                     uint32_t* committed_dev, uint32_t* v1_dev, uint64_t bitmap_pitch_words,
                                     void* stream);
/* The compact exchange payload of n_windows windows of a shard: lists_dev[w * (1 + cap)]
 * = the window's count of UNDECIDED slots (output plane 6 clear), followed by the first
 * min(count, cap) of their offsets in the window (slot id - the window's first slot id),
 * ascending; v1_dev (optional) = the V1 bitmap (plane 7, bits past n_slots cleared) of
 * window w at v1_dev + w * v1_pitch_words. */
int rg_decision_lists_windows_async(rg_ctx* ctx, uint32_t n_windows, const uint32_t* out_dev, uint64_t out_pitch_words,
                                    uint64_t n_slots, uint64_t stride_words, uint32_t* lists_dev, uint32_t cap,
                                    uint32_t* v1_dev, uint64_t v1_pitch_words, void* stream);

/* StdRng::seed_from_u64(seed).next_u64() draws first..first+count-1 (random access;
 * the stream the REF mode consumes, engine.rs:461-604). */
int rg_ref_draws_async(rg_ctx* ctx, uint64_t first, uint64_t count, uint64_t* out_dev,
                       void* stream);

/* Synthetic traces (seeded, counter-based) straight into device planes. */
int rg_trace_generate_async(rg_ctx* ctx, int kind, uint64_t seed, uint64_t slot_base,
                            uint64_t n_slots, uint64_t stride_words, uint32_t* votes_dev,
                            void* stream);
int rg_digest_trace_async(rg_ctx* ctx, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                          uint64_t digest_stride, uint64_t* digests_dev, void* stream);

/* Weak-MVC to termination, cluster view (config 3): every replica of each slot
 * runs phase_rnd1/phase_rnd2 (weak_mvc.ivy:129-191) under a deterministic
 * adversarial scheduler (each receiver hears itself + quorum-1 others chosen by
 * a hash keyed by delivery_seed, slot, phase, round, receiver) with the common
 * coin, until all replicas decided or max_phases (<= 255).
 * states_dev: n planar planes (replica r's initial state bit), stride_words apart.
 * info_dev[s] = decision (0 V0, 1 V1, 3 not all decided, 2 replicas disagree — an
 *               agreement violation that must never occur) | phases << 8 |
 *               first decision phase << 16 | coin phases << 24.
 * stats_dev (8 x u64, may be NULL): slots all decided, decided V1, sum of phases,
 * max phases, sum of coin phases, sum of first-decision phases, slots, 0. */
int rg_wmvc_cluster_async(rg_ctx* ctx, const uint32_t* states_dev, uint64_t stride_words,
                          uint64_t n_slots, uint64_t slot_base, uint64_t delivery_seed,
                          uint32_t max_phases, uint32_t* info_dev, uint64_t* stats_dev, void* stream);
/* rg_wmvc_cluster_async plus the run's decided and V1 bitmaps (as rg_cluster_bitmap_async
 * makes them from info_dev, ceil(n_slots/32) words each), built inside the cluster
 * kernel: one pass instead of two. */
int rg_wmvc_cluster_bitmaps_async(rg_ctx* ctx, const uint32_t* states_dev, uint64_t stride_words,
                                  uint64_t n_slots, uint64_t slot_base, uint64_t delivery_seed,
                                  uint32_t max_phases, uint32_t* info_dev, uint64_t* stats_dev,
                                  uint32_t* decided_dev, uint32_t* v1_dev, void* stream);
/* Decided (all replicas decided) and V1 bitmaps of a cluster run's info words,
 * ceil(n_slots/32) words each: the per-shard payload of the C3 multi-GPU exchange. */
int rg_cluster_bitmap_async(rg_ctx* ctx, const uint32_t* info_dev, uint64_t n_slots,
                            uint32_t* decided_dev, uint32_t* v1_dev, void* stream);
int rg_cluster_trace_async(rg_ctx* ctx, uint64_t seed, uint64_t slot_base, uint64_t n_slots,
                           uint64_t stride_words, uint32_t* states_dev, void* stream);

int rg_stream_sync(rg_ctx* ctx, void* stream);

/* Host-side layout helpers (no device work). */
int rg_planar_to_tiled(const uint32_t* planar, uint32_t n_planes, uint64_t n_words, uint64_t stride,
                       uint32_t tile_words, uint32_t* tiled);
int rg_tiled_to_planar(const uint32_t* tiled, uint32_t n_planes, uint64_t n_words, uint32_t tile_words,
                       uint64_t stride, uint32_t* planar);
/* Host-side packing helpers (no device work): slot-major codes [S][n] <-> planar planes. */
int rg_pack_codes(const uint8_t* codes, uint32_t n, uint64_t n_slots, uint64_t stride_words,
                  uint32_t* planes);
int rg_unpack_planes(const uint32_t* planes, uint32_t n, uint64_t n_slots,
                     uint64_t stride_words, uint8_t* codes);

#ifdef __cplusplus
}
#endif
#endif /* RABIA_GPU_H */
