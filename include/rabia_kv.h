/*
 * rabia_kv.h — C ABI of the device-resident kvstore apply.
 *
 * After a phase step (rabia_gpu.h) the V1-decided slots' batches are applied to
 * the replicated state machine in total order (ascending slot, then command order
 * inside the batch): engine.rs:646-655 (proposer) and 727-735 (follower) call
 * StateMachine::apply_commands, which for the kvstore example is
 * KVStoreSMR::apply_commands (examples/kvstore_smr/src/smr_impl.rs:72-127) over
 * KVStore::set/get/delete/exists (examples/kvstore_smr/src/store.rs:144-262).
 * The store lives in HBM: an open-addressing table of keys plus a byte heap of key
 * and value bytes; commands arrive as their Command.data bytes (bincode 1.3.3 of
 * KVOperation, operations.rs:10-19) and are decoded on the device.
 *
 * Same conventions as rabia_gpu.h: plain C types, streams as void* (NULL = the
 * store's own stream), RG_OK (0) or a negative rg_status, rg_kv_last_error() for
 * the text, no CPU fallback (rg_kv_create fails with RG_ENODEV without gfx950).
 *
 * Result codes, one byte per command (KVResult, operations.rs:55-63, and
 * StoreError, operations.rs:97-108):
 *   0 Success   1 NotFound   2 Error(InvalidKey "Key cannot be empty")
 *   3 Error(InvalidKey "Key too long")   4 Error(ValueTooLarge)   5 Error(StoreFull)
 *   6 Command.data is not a bincode KVOperation   7 not applied (slot not decided V1)
 *   8 refused: the store's capacity (table slots / heap bytes) cannot hold the batch;
 *     the whole batch was refused before any write (rg_kv_stats.flags says which)
 *
 * Value bytes are allocated in size classes (powers of two >= 16): a SET whose value
 * fits its key's current allocation overwrites it in place, so updates of existing
 * keys never grow the heap; only new keys and outgrown values take heap bytes.
 *
 * Paths of a batch (rg_kv_stats.last_path), all exact: 0 keyed (StoreFull cannot
 * fire: live + keys created <= max_keys); 3 keyed with the creates ranked (StoreFull
 * can fire, no DELETE meets a live key: the live count only grows, so a create
 * succeeds iff fewer than max_keys - live creates precede it in command order); 1
 * ordered replay, one thread (StoreFull can fire and a DELETE frees a key mid-batch,
 * or a hash run holds more than 8 keys); 2 refused (capacity).
 */
#ifndef RABIA_KV_H
#define RABIA_KV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rg_kv rg_kv;

enum {
  RG_KV_SUCCESS = 0,
  RG_KV_NOT_FOUND = 1,
  RG_KV_E_KEY_EMPTY = 2,
  RG_KV_E_KEY_LONG = 3,
  RG_KV_E_VALUE_LARGE = 4,
  RG_KV_E_FULL = 5,
  RG_KV_E_DECODE = 6,
  RG_KV_NOT_APPLIED = 7,
  RG_KV_E_CAPACITY = 8,
};

/* KVStoreConfig (store.rs:17-42) fields the apply reads, plus device capacities. */
typedef struct rg_kv_config {
  uint64_t max_keys;             /* KVStoreConfig.max_keys; 0 => 1,000,000               */
  uint64_t max_value_size;       /* KVStoreConfig.max_value_size; 0 => 1 MiB             */
  uint32_t enable_notifications; /* KVStoreConfig.enable_notifications (drives version)  */
  int32_t device;                /* HIP device ordinal                                   */
  uint64_t table_slots;          /* power of two; 0 => next pow2 >= 2 * max_keys          */
  uint64_t heap_bytes;           /* key + value byte heap; 0 => 64 * table_slots          */
  uint32_t hash_bits;            /* test hook: keep only the low hash_bits bits of the key
                                    hash (0 = all 64) to force hash-collision runs        */
  uint32_t bucket_bits;          /* test hook: sort bucket width (0 = 31 bits); a narrow
                                    bucket puts keys with distinct full hashes in one run */
} rg_kv_config;

/* Store counters (host copy). */
typedef struct rg_kv_stats {
  uint64_t live_keys;        /* KVStore.data.len()                                     */
  uint64_t version;          /* KVStore.version (store.rs:486-489)                     */
  uint64_t total_operations; /* StoreStats.total_operations (store.rs:480-484)         */
  uint64_t occupied_slots;   /* table slots holding a key (live or deleted)            */
  uint64_t heap_used;        /* bytes of the key/value heap in use                     */
  uint64_t batches;          /* rg_kv_apply calls                                      */
  uint64_t ordered_batches;  /* batches applied on the exact in-order path (StoreFull
                                reachable or a hash collision group too large)          */
  uint64_t flags;            /* nonzero: a capacity fault (1 table slots, 2 heap bytes)
                                refused a batch; that batch changed nothing. Bit 4: a
                                capacity fault inside the commit pass (the pre-check
                                should make it impossible): that batch is PARTIALLY
                                written and its results do not describe the store —
                                treat the store as lost; the bit stays set and every
                                later batch is refused (results RG_KV_E_CAPACITY)      */
  uint64_t last_path;        /* the last batch: 0 keyed replay, 1 ordered replay,
                                2 refused (capacity fault, results RG_KV_E_CAPACITY),
                                3 keyed replay with the creates ranked (StoreFull)     */
} rg_kv_stats;

int rg_kv_create(rg_kv** out, const rg_kv_config* cfg);
int rg_kv_destroy(rg_kv* kv);
const char* rg_kv_last_error(const rg_kv* kv);

/* Which commands to apply: apply_mask[c] = 1 iff command c belongs to a slot whose
 * decision is V1 (output plane 7 of an rg_phase_step over the same window) and,
 * when gate_dev is given, whose PhaseId slot_base + s is above *gate_dev.
 *  gate_dev = NULL: the proposer (make_decision applies every V1 decision,
 *                   engine.rs:641-650);
 *  gate_dev = the follower's last_committed before the window (handle_decision
 *             applies only if phase_id > last_committed, engine.rs:723-728; e.g. the
 *             gate written by rg_follower_commit_async, rabia_gpu.h).
 * slot_cmd_off[n_slots + 1] = CSR offsets of each slot's batch in the command list.
 * out_dev / stride_words / tile_words = the step's output buffer and its layout
 * (rabia_gpu.h "Layout"). */
int rg_kv_mark_applied_async(rg_kv* kv, const uint32_t* out_dev, uint64_t stride_words,
                             uint32_t tile_words, uint64_t n_slots, uint64_t slot_base,
                             const uint64_t* gate_dev, const uint64_t* slot_cmd_off_dev,
                             uint8_t* apply_mask_dev, void* stream);

/* Apply n_cmds commands in total order. Command c's bytes are
 * data_dev[cmd_off_dev[c] .. cmd_off_dev[c+1]). apply_mask_dev may be NULL (apply
 * all). results_dev[c] receives the result code. Equivalent to calling
 * KVStoreSMR::apply_command on each applied command in order. */
int rg_kv_apply_async(rg_kv* kv, const uint8_t* data_dev, const uint64_t* cmd_off_dev,
                      uint64_t n_cmds, const uint8_t* apply_mask_dev, uint8_t* results_dev,
                      void* stream);

/* Counters (synchronises the device). */
int rg_kv_get_stats(rg_kv* kv, rg_kv_stats* out);

/* get_all_data (store.rs / smr_impl.rs:97-104) as raw arrays: copies the table
 * (hashes[table_slots], entries[table_slots][4] = {key_off, val_off, version,
 * key_len | val_len << 32}; version 0 = not live) and heap[heap_used] to host
 * buffers of at least those sizes. Synchronous. */
int rg_kv_dump(rg_kv* kv, uint64_t* hashes, uint64_t* entries, uint8_t* heap, uint64_t heap_cap);
int rg_kv_table_slots(const rg_kv* kv, uint64_t* out);

/* Synthetic C4 commands: n_cmds bincode KVOperations (Set 85 %, Get 10 %, Delete 3 %,
 * Exists 2 %) over `key_space` keys "k<decimal>" (16-byte keys) with 32-byte values,
 * written to data_dev (capacity data_cap bytes) with offsets cmd_off_dev[n_cmds + 1]. */
int rg_kv_trace_async(rg_kv* kv, uint64_t seed, uint64_t n_cmds, uint64_t key_space,
                      uint8_t* data_dev, uint64_t data_cap, uint64_t* cmd_off_dev, void* stream);

int rg_kv_sync(rg_kv* kv, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RABIA_KV_H */
