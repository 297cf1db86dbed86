// rg_kv.hip — device-resident kvstore apply (include/rabia_kv.h).
//
// Semantics: KVStoreSMR::apply_commands (examples/kvstore_smr/src/smr_impl.rs:72-127)
// over KVStore (store.rs:144-262) applied to the commands in total order. Parallel
// form (one launch chain per batch, no host round trip):
//   1 decode    one thread per command: bincode KVOperation (operations.rs:10-19),
//               key/value validation (store.rs:463-478), 64-bit key hash
//   2 sort      stable radix sort of (hash, command index): each key's commands
//               become one contiguous run, still in total order
//   3 plan      one thread per hash run ("walker"): looks every distinct key of its
//               run up in the table, replays the key's commands in order and sizes
//               what the commit writes (new key bytes + final value bytes)
//   4 decide    one thread folds the per-block plan partials: can StoreFull (the
//               only cross-key dependency: store.rs:153-158 reads data.len()) occur?
//               live + keys created <= max_keys => no, the keyed replay is exact.
//   5 commit    the same walkers write results, table entries and heap bytes at
//               offsets from an exclusive scan of the plan sizes
//   6 ordered   otherwise ONE thread replays the batch in total order (exact,
//               slow; counted in rg_kv_stats.ordered_batches)
//   7 finish    folds the per-block counter deltas into the store counters
// Key equality is byte equality (hash runs are split by comparing key bytes).
// Deleted keys keep their table slot (version 0 = not live) so probe chains stay
// intact; a later SET of the same key reuses it with a fresh ValueEntry (version 1).
#include "rabia_kv.h"

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <new>
#include <string>

namespace {

constexpr uint64_t kEmpty = 0;
constexpr uint64_t kInvalidKey = ~0ull;    // full hash of commands that are not applied
// Sort key: a 31-bit bucket of the full hash (equal hashes -> equal buckets), so the
// radix sort runs 4 digit passes instead of 8; commands that are not applied get
// kInvalidBucket and sort last. A bucket run may hold several hashes: the walkers
// already split runs into keys by comparing key bytes, and look each key up with
// its own full hash.
constexpr uint64_t kInvalidBucket = 0xFFFFFFFFull;
// Command bytes sit at arbitrary byte offsets: multi-byte fields, key compares and
// copies go through 1-byte-aligned types (gfx950 global memory takes unaligned
// dword accesses; little-endian like bincode's fixint encoding).
typedef uint64_t u64_unaligned __attribute__((aligned(1)));
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
constexpr int kSortBits = 32;
__device__ __forceinline__ uint64_t hash_bucket(uint64_t h) { return (h ^ (h >> 32)) & 0x7FFFFFFFull; }
constexpr uint32_t kMaxKeyLen = 256;       // store.rs:467
constexpr int kBlock = 256;
constexpr int kMaxRunKeys = 8;             // distinct keys per hash run on the keyed path
constexpr uint8_t kPending = 0xFF;

enum : uint64_t { kFaultTable = 1, kFaultHeap = 2 };

struct KvEntry {        // one table slot (the hash lives in its own array for probing)
  uint64_t key_off;     // heap offset of the key bytes
  uint64_t val_off;     // heap offset of the value bytes
  uint64_t version;     // ValueEntry.version; 0 = not live (deleted / never set)
  uint32_t key_len;
  uint32_t val_len;
};
static_assert(sizeof(KvEntry) == 32, "entry layout is part of rg_kv_dump");

struct KvOp {           // decoded command
  uint64_t key_off;     // offset into the batch's data bytes
  uint64_t val_off;
  uint32_t key_len;
  uint32_t val_len;
  uint32_t kind;        // 0 Set 1 Get 2 Delete 3 Exists
  uint32_t status;      // kPending or a final result code
};

struct KvCounters {
  unsigned long long live, version, total_ops, occupied, heap_top;
  unsigned long long batches, ordered, flags;
  unsigned long long mode;        // per batch: 0 keyed commit, 1 ordered replay, 2 fault
  unsigned long long batch_base;  // heap top before the batch (keyed commit offsets)
};

// Per-block partials of the plan / commit walks.
enum { kPCreated = 0, kPNewSlots, kPOverflow, kPLiveDelta, kPVersion, kPOps, kPCount };

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__device__ __forceinline__ uint64_t key_hash(const uint8_t* p, uint32_t n, uint64_t hmask) {
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a 64, then a finaliser for the probe bits
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {  // one 8-byte load, bytes folded in order from the register
    uint64_t w = *(const u64_unaligned*)(p + i);
#pragma unroll
    for (int k = 0; k < 8; k++, w >>= 8) h = (h ^ (w & 0xFFu)) * 0x100000001b3ull;
  }
  for (; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  h = fmix64(h ^ n) & hmask;
  if (h == kEmpty) h = 1;
  if (h == kInvalidKey) h = kInvalidKey - 1;
  return h;
}

__device__ __forceinline__ uint64_t ld_u64(const uint8_t* p) { return *(const u64_unaligned*)p; }
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) { return *(const u32_unaligned*)p; }

// std::str::from_utf8 acceptance (no overlongs, no surrogates, <= U+10FFFF):
// serde's String visitor rejects anything else, so bincode::deserialize fails.
__device__ bool utf8_valid(const uint8_t* p, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    if (i + 8 <= n && (ld_u64(p + i) & 0x8080808080808080ull) == 0) { i += 8; continue; }  // 8 ASCII bytes
    const uint32_t c = p[i];
    if (c < 0x80) { i++; continue; }
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return false;
    if (i + need >= n) return false;
    const uint32_t c1 = p[i + 1];
    if (c1 < lo || c1 > hi) return false;
    for (uint32_t k = 2; k <= need; k++) {
      const uint32_t ck = p[i + k];
      if (ck < 0x80 || ck > 0xBF) return false;
    }
    i += need + 1;
  }
  return true;
}

// Key/value bytes sit at arbitrary byte offsets: compare and copy them 8 bytes at a
// time through 1-byte-aligned u64 accesses, then the tail byte by byte; nothing past
// the n bytes is touched.

__device__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8)
    if (*(const u64_unaligned*)(a + i) != *(const u64_unaligned*)(b + i)) return false;
  for (; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

__device__ __forceinline__ void bytes_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) *(u64_unaligned*)(dst + i) = *(const u64_unaligned*)(src + i);
  for (; i < n; i++) dst[i] = src[i];
}

// ---- 1 decode ----------------------------------------------------------------
__global__ void kv_decode_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                 uint64_t n, const uint8_t* __restrict__ mask, uint64_t max_value, uint64_t hmask,
                                 KvOp* __restrict__ ops, uint64_t* __restrict__ sort_key, uint64_t* __restrict__ full_hash,
                                 uint32_t* __restrict__ sort_idx, uint8_t* __restrict__ results) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  KvOp op{0, 0, 0, 0, 0, kPending};
  uint64_t key = kInvalidKey;
  if (mask && !mask[c]) {
    op.status = RG_KV_NOT_APPLIED;
  } else {
    const uint64_t b = off[c], e = off[c + 1];
    const uint64_t len = e > b ? e - b : 0;
    const uint8_t* p = data + b;
    op.status = RG_KV_E_DECODE;
    if (len >= 12) {
      const uint32_t kind = ld_u32(p);
      const uint64_t klen = ld_u64(p + 4);
      if (kind <= 3 && klen <= len - 12) {
        uint64_t pos = 12 + klen;
        uint64_t vlen = 0;
        bool ok = true;
        if (kind == 0) {
          if (len - pos < 8) ok = false;
          else {
            vlen = ld_u64(p + pos);
            if (vlen > len - pos - 8) ok = false;
          }
        }
        if (ok && utf8_valid(p + 12, klen) && (kind != 0 || utf8_valid(p + pos + 8, vlen))) {
          op.kind = kind;
          op.key_off = b + 12;
          op.key_len = (uint32_t)(klen > 0xFFFFFFFFull ? 0xFFFFFFFFull : klen);
          op.val_off = b + pos + 8;
          op.val_len = (uint32_t)(vlen > 0xFFFFFFFFull ? 0xFFFFFFFFull : vlen);
          if (klen == 0) op.status = RG_KV_E_KEY_EMPTY;                 // store.rs:464-466
          else if (klen > kMaxKeyLen) op.status = RG_KV_E_KEY_LONG;     // store.rs:467-469
          else if (kind == 0 && vlen > max_value) op.status = RG_KV_E_VALUE_LARGE;  // 473-477
          else {
            op.status = kPending;
            key = key_hash(p + 12, (uint32_t)klen, hmask);
          }
        }
      }
    }
  }
  ops[c] = op;
  sort_key[c] = key == kInvalidKey ? kInvalidBucket : hash_bucket(key);
  full_hash[c] = key;
  sort_idx[c] = (uint32_t)c;
  if (op.status != kPending) results[c] = (uint8_t)op.status;
}

// ---- table lookup ------------------------------------------------------------
// Returns the slot holding `key` (live or not) or -1. Linear probing; an empty
// slot ends the chain. Concurrent inserts by other walkers carry other hashes.
__device__ int64_t table_find(const uint64_t* hashes, const KvEntry* ent, const uint8_t* heap,
                              uint64_t mask, uint64_t h, const uint8_t* key, uint32_t klen) {
  uint64_t s = h & mask;
  for (uint64_t probes = 0; probes <= mask; probes++) {
    const uint64_t th = __hip_atomic_load(hashes + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (th == kEmpty) return -1;
    if (th == h) {
      const KvEntry e = ent[s];
      if (e.key_len == klen && bytes_eq(heap + e.key_off, key, klen)) return (int64_t)s;
    }
    s = (s + 1) & mask;
  }
  return -1;
}

__device__ int64_t table_claim(uint64_t* hashes, uint64_t mask, uint64_t h) {
  uint64_t s = h & mask;
  for (uint64_t probes = 0; probes <= mask; probes++) {
    unsigned long long expected = kEmpty;
    if (__hip_atomic_compare_exchange_strong((unsigned long long*)(hashes + s), &expected,
                                             (unsigned long long)h, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return (int64_t)s;
    s = (s + 1) & mask;
  }
  return -1;
}

struct StoreView {
  uint64_t* hashes;
  KvEntry* ent;
  uint8_t* heap;
  uint64_t mask;
  uint64_t heap_cap;
  KvCounters* ctr;
  uint64_t max_keys;
  uint32_t notify;
};

struct BatchView {
  const uint8_t* data;
  const KvOp* ops;
  const uint64_t* skey;   // sorted hash buckets
  const uint64_t* hfull;  // full key hash per command index
  const uint32_t* sidx;   // command index per sorted position
  uint64_t n;
  uint8_t* results;
  uint8_t* done;          // per sorted position: handled by an earlier key of its run
  uint64_t* need;         // per sorted position: plan bytes (run heads only)
  uint64_t* heap_off;     // exclusive scan of need
  unsigned long long* part;  // [blocks][kPCount]
};

__device__ __forceinline__ bool same_key(const BatchView& b, const KvOp& x, const KvOp& y) {
  return x.key_len == y.key_len && bytes_eq(b.data + x.key_off, b.data + y.key_off, x.key_len);
}

// Replay one key's commands [first .. run_end) (those equal to the leader's key)
// in total order. Returns the final state; writes results when COMMIT.
struct KeyOutcome {
  bool live0, live1, wrote_value, any_set;
  uint64_t ver1;
  uint32_t last_set;     // command index of the final value's SET
  uint64_t n_ops, n_version;
};

template <bool COMMIT>
__device__ KeyOutcome replay_key(const BatchView& b, const StoreView& st, uint64_t first,
                                 uint64_t run_end, const KvOp& lead, int64_t slot,
                                 bool mark_done) {
  KeyOutcome o{};
  o.live0 = slot >= 0 && st.ent[slot].version > 0;
  bool live = o.live0;
  uint64_t ver = o.live0 ? st.ent[slot].version : 0;
  for (uint64_t i = first; i < run_end; i++) {
    if (b.done[i]) continue;
    const uint32_t c = b.sidx[i];
    const KvOp op = b.ops[c];
    if (i != first && !same_key(b, op, lead)) continue;
    if (mark_done) b.done[i] = 1;
    uint8_t r;
    if (op.kind == 0) {                 // SET: update or insert (store.rs:151-163)
      ver = live ? ver + 1 : 1;
      live = true;
      o.wrote_value = true;
      o.any_set = true;
      o.last_set = c;
      o.n_version += st.notify;
      r = RG_KV_SUCCESS;
    } else if (op.kind == 2) {          // DELETE (store.rs:220-251)
      r = live ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
      if (live) o.n_version += st.notify;
      if (live) o.wrote_value = false;
      live = false;
    } else {                            // GET / EXISTS (smr_impl.rs:79-94)
      r = live ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
    }
    o.n_ops++;
    if (COMMIT) b.results[c] = r;
  }
  o.live1 = live;
  o.ver1 = ver;
  return o;
}

__device__ __forceinline__ void block_add_partials(unsigned long long (&v)[kPCount],
                                                   unsigned long long* part) {
  __shared__ unsigned long long red[kBlock / 64][kPCount];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kPCount; k++) {
    unsigned long long x = v[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) red[wave][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < kPCount) {
    unsigned long long s = 0;
    for (int w = 0; w < kBlock / 64; w++) s += red[w][threadIdx.x];
    part[(uint64_t)blockIdx.x * kPCount + threadIdx.x] = s;
  }
}

// ---- 3 plan / 5 commit -------------------------------------------------------
template <bool COMMIT>
__global__ __launch_bounds__(kBlock) void kv_walk_kernel(BatchView b, StoreView st) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long acc[kPCount] = {0, 0, 0, 0, 0, 0};
  const bool go = !COMMIT || st.ctr->mode == 0;
  if (go && i < b.n) {
    const uint64_t h = b.skey[i];
    if (h != kInvalidBucket && (i == 0 || b.skey[i - 1] != h)) {
      uint64_t end = i + 1;
      while (end < b.n && b.skey[end] == h) end++;
      uint64_t need = 0, heap_pos = COMMIT ? st.ctr->batch_base + b.heap_off[i] : 0;
      int keys = 0;
      for (uint64_t first = i; first < end; first++) {
        if (b.done[first]) continue;
        if (++keys > kMaxRunKeys) { acc[kPOverflow] = 1; break; }
        const KvOp lead = b.ops[b.sidx[first]];
        const uint64_t hl = b.hfull[b.sidx[first]];
        const uint8_t* kp = b.data + lead.key_off;
        const int64_t slot = table_find(st.hashes, st.ent, st.heap, st.mask, hl, kp, lead.key_len);
        const KeyOutcome o = replay_key<COMMIT>(b, st, first, end, lead, slot, true);
        acc[kPOps] += o.n_ops;
        acc[kPVersion] += o.n_version;
        acc[kPLiveDelta] += (unsigned long long)((int64_t)o.live1 - (int64_t)o.live0);
        // keys that become live at some point of the batch (bound on data.len())
        acc[kPCreated] += !o.live0 && o.any_set;
        const bool new_slot = slot < 0 && o.live1;
        acc[kPNewSlots] += new_slot;
        const uint64_t kbytes = new_slot ? lead.key_len : 0;
        const uint64_t vbytes = (o.live1 && o.wrote_value) ? b.ops[o.last_set].val_len : 0;
        need += kbytes + vbytes;
        if (COMMIT) {
          int64_t s = slot;
          if (new_slot) {
            s = table_claim(st.hashes, st.mask, hl);
            if (s < 0) { atomicOr(&st.ctr->flags, kFaultTable); continue; }
            uint8_t* dst = st.heap + heap_pos;
            bytes_copy(dst, kp, lead.key_len);
            st.ent[s].key_off = heap_pos;
            st.ent[s].key_len = lead.key_len;
            heap_pos += kbytes;
          }
          if (s >= 0 && (o.live0 || o.live1)) {
            if (o.live1 && o.wrote_value) {
              const KvOp& sop = b.ops[o.last_set];
              const uint8_t* src = b.data + sop.val_off;
              uint8_t* dst = st.heap + heap_pos;
              bytes_copy(dst, src, sop.val_len);
              st.ent[s].val_off = heap_pos;
              st.ent[s].val_len = sop.val_len;
              heap_pos += vbytes;
            }
            st.ent[s].version = o.live1 ? o.ver1 : 0;
          }
        }
      }
      if (!COMMIT) b.need[i] = need;
    } else if (!COMMIT) {
      b.need[i] = 0;
    }
  } else if (!COMMIT && i < b.n) {
    b.need[i] = 0;
  }
  block_add_partials(acc, b.part);
}

// ---- 4 decide ----------------------------------------------------------------
__global__ void kv_decide_kernel(StoreView st, const unsigned long long* part, uint32_t blocks,
                                 const uint64_t* need, const uint64_t* heap_off, uint64_t n) {
  __shared__ unsigned long long red[kBlock][3];
  unsigned long long c = 0, ns = 0, ov = 0;
  for (uint32_t k = threadIdx.x; k < blocks; k += blockDim.x) {
    c += part[(uint64_t)k * kPCount + kPCreated];
    ns += part[(uint64_t)k * kPCount + kPNewSlots];
    ov |= part[(uint64_t)k * kPCount + kPOverflow];
  }
  red[threadIdx.x][0] = c; red[threadIdx.x][1] = ns; red[threadIdx.x][2] = ov;
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int t = 1; t < (int)blockDim.x; t++) {
    c += red[t][0]; ns += red[t][1]; ov |= red[t][2];
  }
  KvCounters* k = st.ctr;
  const uint64_t bytes = n ? heap_off[n - 1] + need[n - 1] : 0;
  unsigned long long mode = 0;
  // StoreFull unreachable iff live + created <= max_keys (size never exceeds it).
  if (ov || k->live + c > st.max_keys) mode = 1;
  // capacities: at most 7/8 of the table occupied; heap bytes available
  const uint64_t cap = st.mask + 1;
  if (mode == 0 && (k->occupied + ns > cap - cap / 8 || k->heap_top + bytes > st.heap_cap)) mode = 2;
  k->mode = mode;
  k->batches += 1;
  if (mode == 0) {
    k->occupied += ns;
    k->batch_base = k->heap_top;  // commit writes [batch_base + heap_off[i], ...)
    k->heap_top += bytes;
  } else if (mode == 2) {
    k->flags |= (k->occupied + ns > cap - cap / 8) ? kFaultTable : kFaultHeap;
  }
}

// ---- 6 ordered replay (StoreFull reachable) -------------------------------------
__global__ void kv_ordered_kernel(const uint8_t* data, const KvOp* ops, const uint64_t* okey, uint64_t n,
                                  uint8_t* results, StoreView st) {
  if (threadIdx.x != 0 || st.ctr->mode != 1) return;
  KvCounters* k = st.ctr;
  unsigned long long live = k->live, ver = k->version, tops = k->total_ops, occ = k->occupied, top = k->heap_top;
  const uint64_t cap = st.mask + 1;
  for (uint64_t c = 0; c < n; c++) {
    const KvOp op = ops[c];
    if (op.status != kPending) continue;
    const uint8_t* kp = data + op.key_off;
    const uint64_t h = okey[c];
    int64_t s = table_find(st.hashes, st.ent, st.heap, st.mask, h, kp, op.key_len);
    const bool is_live = s >= 0 && st.ent[s].version > 0;
    uint8_t r;
    if (op.kind == 0) {
      if (!is_live && live >= st.max_keys) {     // store.rs:153-158
        results[c] = RG_KV_E_FULL;
        continue;
      }
      if (s < 0) {
        if (occ + 1 > cap - cap / 8 || top + op.key_len > st.heap_cap) { k->flags |= kFaultTable; break; }
        s = table_claim(st.hashes, st.mask, h);
        if (s < 0) { k->flags |= kFaultTable; break; }
        occ++;
        bytes_copy(st.heap + top, kp, op.key_len);
        st.ent[s].key_off = top;
        st.ent[s].key_len = op.key_len;
        st.ent[s].version = 0;
        top += op.key_len;
      }
      if (top + op.val_len > st.heap_cap) { k->flags |= kFaultHeap; break; }
      bytes_copy(st.heap + top, data + op.val_off, op.val_len);
      st.ent[s].val_off = top;
      st.ent[s].val_len = op.val_len;
      top += op.val_len;
      st.ent[s].version = is_live ? st.ent[s].version + 1 : 1;
      if (!is_live) live++;
      ver += st.notify;
      r = RG_KV_SUCCESS;
    } else if (op.kind == 2) {
      r = is_live ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
      if (is_live) {
        st.ent[s].version = 0;
        live--;
        ver += st.notify;
      }
    } else {
      r = is_live ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
    }
    tops++;
    results[c] = r;
  }
  k->live = live; k->version = ver; k->total_ops = tops; k->occupied = occ; k->heap_top = top;
  k->ordered += 1;
}

// ---- 7 finish (keyed path counters) ----------------------------------------------
__global__ void kv_finish_kernel(KvCounters* k, const unsigned long long* part, uint32_t blocks) {
  __shared__ unsigned long long red[kBlock][3];
  unsigned long long ld = 0, vv = 0, ops = 0;
  for (uint32_t b = threadIdx.x; b < blocks; b += blockDim.x) {
    ld += part[(uint64_t)b * kPCount + kPLiveDelta];
    vv += part[(uint64_t)b * kPCount + kPVersion];
    ops += part[(uint64_t)b * kPCount + kPOps];
  }
  red[threadIdx.x][0] = ld; red[threadIdx.x][1] = vv; red[threadIdx.x][2] = ops;
  __syncthreads();
  if (threadIdx.x != 0 || k->mode != 0) return;
  for (int t = 1; t < (int)blockDim.x; t++) {
    ld += red[t][0]; vv += red[t][1]; ops += red[t][2];
  }
  k->live += ld;  // two's-complement sum of +-1 deltas
  k->version += vv;
  k->total_ops += ops;
}

// ---- mark applied commands from the phase step's decision plane -----------------
// gate (follower, handle_decision engine.rs:723-728): a V1 slot's batch is applied
// only if its PhaseId is above last_committed (*gate); NULL = the proposer's
// make_decision, which applies every V1 decision (engine.rs:641-650).
__global__ void kv_mark_kernel(const uint32_t* out, uint64_t stride, uint32_t tile_words, uint64_t n_slots,
                               uint64_t slot_base, const unsigned long long* gate, const uint64_t* slot_off,
                               uint8_t* mask) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_slots) return;
  const unsigned long long lc = gate ? *gate : 0ull;
  const uint64_t w = s >> 5;
  uint64_t idx;
  if (tile_words) {
    const uint64_t T = tile_words;
    idx = (w / T) * (8 * T) + 7 * T + (w % T);
  } else {
    idx = 7 * stride + w;
  }
  const uint8_t v = (uint8_t)(((out[idx] >> (s & 31)) & 1u) && (!gate || slot_base + s > lc));
  for (uint64_t c = slot_off[s]; c < slot_off[s + 1]; c++) mask[c] = v;
}

// ---- synthetic C4 commands ---------------------------------------------------
__device__ __forceinline__ uint64_t mix(uint64_t seed, uint64_t i) { return fmix64(seed * 0x9E3779B97F4A7C15ull + i + 1); }

__global__ void kv_trace_size_kernel(uint64_t seed, uint64_t n, uint64_t* size) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > n) return;
  if (c == n) { size[c] = 0; return; }
  const uint32_t r = (uint32_t)(mix(seed, c) % 100);
  size[c] = r < 85 ? 68 : 28;   // SET: 4 + 8 + 16 + 8 + 32; others: 4 + 8 + 16
}

__global__ void kv_trace_fill_kernel(uint64_t seed, uint64_t n, uint64_t key_space, uint8_t* data,
                                     const uint64_t* off) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint64_t h = mix(seed, c);
  const uint32_t r = (uint32_t)(h % 100);
  const uint32_t kind = r < 85 ? 0 : (r < 95 ? 1 : (r < 98 ? 2 : 3));
  const uint64_t key = fmix64(h ^ 0x5bd1e995ull) % (key_space ? key_space : 1);
  uint8_t* p = data + off[c];
  for (int i = 0; i < 4; i++) p[i] = (uint8_t)(kind >> (8 * i));
  for (int i = 0; i < 8; i++) p[4 + i] = (uint8_t)(16ull >> (8 * i));
  p[12] = 'k';
  uint64_t kk = key;
  for (int i = 15; i >= 1; i--) { p[12 + i] = (uint8_t)('0' + kk % 10); kk /= 10; }
  if (kind == 0) {
    for (int i = 0; i < 8; i++) p[28 + i] = (uint8_t)(32ull >> (8 * i));
    uint64_t v = fmix64(h + 0x632be59bd9b4e019ull);
    for (int i = 0; i < 32; i++) {
      if ((i & 15) == 0 && i) v = fmix64(v);
      p[36 + i] = (uint8_t)("0123456789abcdef"[(v >> (4 * (i & 15))) & 15]);
    }
  }
}

}  // namespace

// ============================================================================
struct rg_kv {
  rg_kv_config cfg{};
  hipStream_t stream = nullptr;
  uint64_t* hashes = nullptr;
  KvEntry* ent = nullptr;
  uint8_t* heap = nullptr;
  KvCounters* ctr = nullptr;
  uint64_t mask = 0;
  // per-batch scratch
  uint64_t cap_cmds = 0;
  KvOp* ops = nullptr;
  uint64_t *key_a = nullptr, *key_b = nullptr, *hfull = nullptr, *need = nullptr, *heap_off = nullptr;
  uint32_t *idx_a = nullptr, *idx_b = nullptr;
  uint8_t* done = nullptr;
  unsigned long long* part = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  std::string err;
};

namespace {
thread_local std::string g_kv_err;

int kfail(rg_kv* kv, int code, const std::string& m) {
  if (kv) kv->err = m;
  else g_kv_err = m;
  return code;
}

#define KV_HIP(kv, call)                                                           \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) return kfail(kv, -2, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

StoreView view(rg_kv* kv) {
  return StoreView{kv->hashes, kv->ent, kv->heap, kv->mask, kv->cfg.heap_bytes, kv->ctr,
                   kv->cfg.max_keys, kv->cfg.enable_notifications ? 1u : 0u};
}

void free_scratch(rg_kv* kv) {
  (void)hipFree(kv->ops); (void)hipFree(kv->key_a); (void)hipFree(kv->key_b); (void)hipFree(kv->hfull);
  (void)hipFree(kv->need); (void)hipFree(kv->heap_off); (void)hipFree(kv->idx_a);
  (void)hipFree(kv->idx_b); (void)hipFree(kv->done); (void)hipFree(kv->part); (void)hipFree(kv->tmp);
  kv->ops = nullptr; kv->key_a = kv->key_b = kv->hfull = kv->need = kv->heap_off = nullptr;
  kv->idx_a = kv->idx_b = nullptr; kv->done = nullptr; kv->part = nullptr; kv->tmp = nullptr;
  kv->cap_cmds = 0; kv->tmp_bytes = 0;
}

int ensure_scratch(rg_kv* kv, uint64_t n) {
  if (n <= kv->cap_cmds) return 0;
  KV_HIP(kv, hipDeviceSynchronize());  // scratch may be in use on a caller stream
  free_scratch(kv);
  uint64_t cap = 1024;
  while (cap < n) cap *= 2;
  const uint64_t blocks = (cap + kBlock - 1) / kBlock;
  KV_HIP(kv, hipMalloc(&kv->ops, cap * sizeof(KvOp)));
  KV_HIP(kv, hipMalloc(&kv->key_a, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->key_b, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->hfull, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->need, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->heap_off, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->idx_a, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->idx_b, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->done, cap));
  KV_HIP(kv, hipMalloc(&kv->part, blocks * kPCount * 8));
  size_t t1 = 0, t2 = 0;
  KV_HIP(kv, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, kv->key_a, kv->key_b, kv->idx_a, kv->idx_b,
                                                  (int)cap, 0, kSortBits, kv->stream));
  KV_HIP(kv, hipcub::DeviceScan::ExclusiveSum(nullptr, t2, kv->need, kv->heap_off, (int)cap, kv->stream));
  kv->tmp_bytes = t1 > t2 ? t1 : t2;
  KV_HIP(kv, hipMalloc(&kv->tmp, kv->tmp_bytes));
  kv->cap_cmds = cap;
  return 0;
}

bool device_ok(int dev, std::string* why) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) { *why = "no HIP device"; return false; }
  if (dev < 0 || dev >= count) { *why = "device ordinal out of range"; return false; }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) { *why = "hipGetDeviceProperties failed"; return false; }
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) { *why = std::string("not gfx950: ") + prop.gcnArchName; return false; }
  return true;
}

}  // namespace

extern "C" {

int rg_kv_create(rg_kv** out, const rg_kv_config* cfg) {
  if (!out || !cfg) return kfail(nullptr, -1, "rg_kv_create: null argument");
  *out = nullptr;
  std::string why;
  if (!device_ok(cfg->device, &why)) return kfail(nullptr, -4, "rg_kv_create: " + why);
  rg_kv_config c = *cfg;
  if (!c.max_keys) c.max_keys = 1000000;
  if (!c.max_value_size) c.max_value_size = 1024 * 1024;
  if (c.max_value_size > 0xFFFFFFFFull) return kfail(nullptr, -1, "rg_kv_create: max_value_size must be < 4 GiB");
  if (!c.table_slots) {
    c.table_slots = 1024;
    while (c.table_slots < 2 * c.max_keys) c.table_slots *= 2;
  }
  if (c.table_slots & (c.table_slots - 1)) return kfail(nullptr, -1, "rg_kv_create: table_slots must be a power of two");
  if (!c.heap_bytes) c.heap_bytes = 64 * c.table_slots;
  rg_kv* kv = new (std::nothrow) rg_kv();
  if (!kv) return kfail(nullptr, -3, "rg_kv_create: host allocation failed");
  kv->cfg = c;
  kv->mask = c.table_slots - 1;
  int rc = 0;
  auto chk = [&](hipError_t e, const char* w) {
    if (e != hipSuccess && !rc) rc = kfail(nullptr, e == hipErrorOutOfMemory ? -3 : -2, std::string(w) + ": " + hipGetErrorString(e));
  };
  chk(hipSetDevice(c.device), "hipSetDevice");
  chk(hipStreamCreateWithFlags(&kv->stream, hipStreamDefault), "hipStreamCreate");
  chk(hipMalloc(&kv->hashes, c.table_slots * 8), "hipMalloc(table)");
  chk(hipMalloc(&kv->ent, c.table_slots * sizeof(KvEntry)), "hipMalloc(entries)");
  chk(hipMalloc(&kv->heap, c.heap_bytes ? c.heap_bytes : 1), "hipMalloc(heap)");
  chk(hipMalloc(&kv->ctr, sizeof(KvCounters)), "hipMalloc(counters)");
  if (!rc) {
    chk(hipMemsetAsync(kv->hashes, 0, c.table_slots * 8, kv->stream), "hipMemset");
    chk(hipMemsetAsync(kv->ent, 0, c.table_slots * sizeof(KvEntry), kv->stream), "hipMemset");
    chk(hipMemsetAsync(kv->ctr, 0, sizeof(KvCounters), kv->stream), "hipMemset");
    chk(hipStreamSynchronize(kv->stream), "hipStreamSynchronize");
  }
  if (rc) {
    rg_kv_destroy(kv);
    return rc;
  }
  *out = kv;
  return 0;
}

int rg_kv_destroy(rg_kv* kv) {
  if (!kv) return 0;
  if (kv->stream) (void)hipStreamSynchronize(kv->stream);
  free_scratch(kv);
  (void)hipFree(kv->hashes); (void)hipFree(kv->ent); (void)hipFree(kv->heap); (void)hipFree(kv->ctr);
  if (kv->stream) (void)hipStreamDestroy(kv->stream);
  delete kv;
  return 0;
}

const char* rg_kv_last_error(const rg_kv* kv) { return kv ? kv->err.c_str() : g_kv_err.c_str(); }

int rg_kv_mark_applied_async(rg_kv* kv, const uint32_t* out_dev, uint64_t stride_words, uint32_t tile_words,
                             uint64_t n_slots, uint64_t slot_base, const uint64_t* gate_dev,
                             const uint64_t* slot_cmd_off_dev, uint8_t* apply_mask_dev, void* stream) {
  if (!kv) return kfail(nullptr, -1, "rg_kv_mark_applied_async: null store");
  if (!n_slots) return 0;
  if (!out_dev || !slot_cmd_off_dev || !apply_mask_dev) return kfail(kv, -1, "rg_kv_mark_applied_async: null buffer");
  if (tile_words && (tile_words & (tile_words - 1))) return kfail(kv, -1, "rg_kv_mark_applied_async: tile_words must be a power of two");
  if (!tile_words && stride_words < (n_slots + 31) / 32) return kfail(kv, -1, "rg_kv_mark_applied_async: stride_words too small");
  hipStream_t s = stream ? (hipStream_t)stream : kv->stream;
  hipLaunchKernelGGL(kv_mark_kernel, dim3((uint32_t)((n_slots + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     out_dev, stride_words, tile_words, n_slots, slot_base,
                     reinterpret_cast<const unsigned long long*>(gate_dev), slot_cmd_off_dev, apply_mask_dev);
  KV_HIP(kv, hipGetLastError());
  return 0;
}

int rg_kv_apply_async(rg_kv* kv, const uint8_t* data_dev, const uint64_t* cmd_off_dev, uint64_t n_cmds,
                      const uint8_t* apply_mask_dev, uint8_t* results_dev, void* stream) {
  if (!kv) return kfail(nullptr, -1, "rg_kv_apply_async: null store");
  if (!n_cmds) return 0;
  if (!data_dev || !cmd_off_dev || !results_dev) return kfail(kv, -1, "rg_kv_apply_async: null buffer");
  if (n_cmds >= (1ull << 31)) return kfail(kv, -1, "rg_kv_apply_async: more than 2^31 - 1 commands");
  if (int rc = ensure_scratch(kv, n_cmds)) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : kv->stream;
  const uint32_t blocks = (uint32_t)((n_cmds + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(kv_decode_kernel, dim3(blocks), dim3(kBlock), 0, s, data_dev, cmd_off_dev, n_cmds,
                     apply_mask_dev, kv->cfg.max_value_size,
                     kv->cfg.hash_bits && kv->cfg.hash_bits < 64 ? (1ull << kv->cfg.hash_bits) - 1 : ~0ull,
                     kv->ops, kv->key_a, kv->hfull, kv->idx_a, results_dev);
  KV_HIP(kv, hipGetLastError());
  size_t tb = kv->tmp_bytes;
  KV_HIP(kv, hipcub::DeviceRadixSort::SortPairs(kv->tmp, tb, kv->key_a, kv->key_b, kv->idx_a, kv->idx_b,
                                                  (int)n_cmds, 0, kSortBits, s));
  KV_HIP(kv, hipMemsetAsync(kv->done, 0, n_cmds, s));
  BatchView b{data_dev, kv->ops, kv->key_b, kv->hfull, kv->idx_b, n_cmds, results_dev, kv->done, kv->need,
              kv->heap_off, kv->part};
  const StoreView st = view(kv);
  hipLaunchKernelGGL(kv_walk_kernel<false>, dim3(blocks), dim3(kBlock), 0, s, b, st);
  KV_HIP(kv, hipGetLastError());
  tb = kv->tmp_bytes;
  KV_HIP(kv, hipcub::DeviceScan::ExclusiveSum(kv->tmp, tb, kv->need, kv->heap_off, (int)n_cmds, s));
  hipLaunchKernelGGL(kv_decide_kernel, dim3(1), dim3(kBlock), 0, s, st, kv->part, blocks, kv->need,
                     kv->heap_off, n_cmds);
  KV_HIP(kv, hipMemsetAsync(kv->done, 0, n_cmds, s));
  hipLaunchKernelGGL(kv_walk_kernel<true>, dim3(blocks), dim3(kBlock), 0, s, b, st);
  hipLaunchKernelGGL(kv_ordered_kernel, dim3(1), dim3(64), 0, s, data_dev, kv->ops, kv->hfull, n_cmds,
                     results_dev, st);
  hipLaunchKernelGGL(kv_finish_kernel, dim3(1), dim3(kBlock), 0, s, kv->ctr, kv->part, blocks);
  KV_HIP(kv, hipGetLastError());
  return 0;
}

int rg_kv_get_stats(rg_kv* kv, rg_kv_stats* out) {
  if (!kv || !out) return kfail(kv, -1, "rg_kv_get_stats: null argument");
  KvCounters c;
  KV_HIP(kv, hipDeviceSynchronize());  // applies may sit on caller streams
  KV_HIP(kv, hipMemcpy(&c, kv->ctr, sizeof(c), hipMemcpyDeviceToHost));
  out->live_keys = c.live;
  out->version = c.version;
  out->total_operations = c.total_ops;
  out->occupied_slots = c.occupied;
  out->heap_used = c.heap_top;
  out->batches = c.batches;
  out->ordered_batches = c.ordered;
  out->flags = c.flags;
  out->last_path = c.mode;
  return 0;
}

int rg_kv_table_slots(const rg_kv* kv, uint64_t* out) {
  if (!kv || !out) return -1;
  *out = kv->mask + 1;
  return 0;
}

int rg_kv_dump(rg_kv* kv, uint64_t* hashes, uint64_t* entries, uint8_t* heap, uint64_t heap_cap) {
  if (!kv || !hashes || !entries) return kfail(kv, -1, "rg_kv_dump: null argument");
  KvCounters c;
  KV_HIP(kv, hipDeviceSynchronize());
  KV_HIP(kv, hipMemcpy(&c, kv->ctr, sizeof(c), hipMemcpyDeviceToHost));
  if (c.heap_top > heap_cap || (c.heap_top && !heap)) return kfail(kv, -1, "rg_kv_dump: heap buffer too small");
  const uint64_t slots = kv->mask + 1;
  KV_HIP(kv, hipMemcpy(hashes, kv->hashes, slots * 8, hipMemcpyDeviceToHost));
  KV_HIP(kv, hipMemcpy(entries, kv->ent, slots * sizeof(KvEntry), hipMemcpyDeviceToHost));
  if (c.heap_top) KV_HIP(kv, hipMemcpy(heap, kv->heap, c.heap_top, hipMemcpyDeviceToHost));
  return 0;
}

int rg_kv_trace_async(rg_kv* kv, uint64_t seed, uint64_t n_cmds, uint64_t key_space, uint8_t* data_dev,
                      uint64_t data_cap, uint64_t* cmd_off_dev, void* stream) {
  if (!kv) return kfail(nullptr, -1, "rg_kv_trace_async: null store");
  if (!data_dev || !cmd_off_dev) return kfail(kv, -1, "rg_kv_trace_async: null buffer");
  if (data_cap < 68 * n_cmds) return kfail(kv, -1, "rg_kv_trace_async: data_cap < 68 * n_cmds");
  if (!key_space) return kfail(kv, -1, "rg_kv_trace_async: key_space must be > 0");
  if (n_cmds >= (1ull << 31)) return kfail(kv, -1, "rg_kv_trace_async: too many commands");
  if (int rc = ensure_scratch(kv, n_cmds + 1)) return rc;
  hipStream_t s = stream ? (hipStream_t)stream : kv->stream;
  const uint32_t blocks = (uint32_t)((n_cmds + 1 + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(kv_trace_size_kernel, dim3(blocks), dim3(kBlock), 0, s, seed, n_cmds, kv->need);
  size_t tb = kv->tmp_bytes;
  KV_HIP(kv, hipcub::DeviceScan::ExclusiveSum(kv->tmp, tb, kv->need, cmd_off_dev, (int)(n_cmds + 1), s));
  hipLaunchKernelGGL(kv_trace_fill_kernel, dim3(blocks), dim3(kBlock), 0, s, seed, n_cmds, key_space, data_dev,
                     cmd_off_dev);
  KV_HIP(kv, hipGetLastError());
  return 0;
}

int rg_kv_sync(rg_kv* kv, void* stream) {
  if (!kv) return -1;
  KV_HIP(kv, hipStreamSynchronize(stream ? (hipStream_t)stream : kv->stream));
  return 0;
}

}  // extern "C"
