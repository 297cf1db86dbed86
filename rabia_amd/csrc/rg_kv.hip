// rg_kv.hip — device-resident kvstore apply (include/rabia_kv.h).
//
// Semantics: KVStoreSMR::apply_commands (examples/kvstore_smr/src/smr_impl.rs:72-127)
// over KVStore (store.rs:144-262) applied to the commands in total order. Parallel
// form (one stream-ordered launch chain per batch, no host round trip):
//   1 decode    thread per command: bincode KVOperation (operations.rs:10-19), UTF-8
//               and key/value validation (store.rs:463-478), 64-bit key hash, a u32
//               sort key (hash bucket; "not applied" sorts last), per-block worst-case
//               growth for the capacity refusal; short commands in one load round trip
//   2 sort      stable sort of the applied commands by bucket (two levels of 8-bit
//               counting passes, hand-written): each key's commands become one
//               contiguous run, still in total order; the rest sort last
//   3 plan      workgroup per 512 sorted positions, decoded fields staged in LDS; run
//               heads compacted per wave, each lane replays one key's commands in
//               order (one table lookup per key), writes the result bytes and a
//               per-key commit record (slot, version, key/value sources, in-place or
//               new allocation); multi-key runs (bucket or hash collisions) take a
//               general path over global memory
//   4 decide    workgroups of 64 walk blocks fold the plan partials, the last to
//               arrive folds theirs: can StoreFull (the only cross-key dependency:
//               store.rs:153-158 reads data.len()) occur? live + keys created <=
//               max_keys => no, the keyed replay is exact; capacity refusal; scan of
//               the heap bytes (group and block bases); the keyed path's counters
//   5 commit    lookup-free write pass over the commit records: table claims for new
//               keys, key/value bytes at the scanned heap offsets, entry fields; the
//               same launch runs the ordered replay instead (one thread, only when
//               StoreFull can fire: exact, slow, counted in
//               rg_kv_stats.ordered_batches) or writes the refusal results
// Key equality is byte equality (hash runs are split by comparing key bytes).
// Deleted keys keep their table slot (version 0 = not live) so probe chains stay
// intact; a later SET of the same key reuses it with a fresh ValueEntry (version 1).
#include "rabia_kv.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <string>

namespace {

constexpr uint64_t kEmpty = 0;
constexpr uint64_t kInvalidKey = ~0ull;    // full hash of commands that are not applied
// Sort key: a bucket of the full hash (equal hashes -> equal buckets) narrow enough
// for 3-4 radix digit passes instead of 8; commands that are not applied get the
// invalid bucket and sort last. A bucket run may hold several hashes: the walkers
// already split runs into keys by comparing key bytes, and look each key up with
// its own full hash.
// (The bucket width vbits is chosen per batch; the invalid bucket is 1 << vbits, and
// the sort drops those commands: they need no plan.)
// Command bytes sit at arbitrary byte offsets: multi-byte fields, key compares and
// copies go through 1-byte-aligned types (gfx950 global memory takes unaligned
// dword accesses; little-endian like bincode's fixint encoding).
typedef uint64_t u64_unaligned __attribute__((aligned(1)));
typedef uint32_t u32_unaligned __attribute__((aligned(1)));
__device__ __forceinline__ uint64_t hash_bucket(uint64_t h, uint64_t bmask) { return (h ^ (h >> 32)) & bmask; }
constexpr uint32_t kMaxKeyLen = 256;       // store.rs:467
constexpr int kBlock = 256;
constexpr int kMaxRunKeys = 8;             // distinct keys per hash run on the keyed path
constexpr uint8_t kPending = 0xFF;

// kFaultPartial: a capacity fault raised inside the commit pass (the whole-batch
// pre-check should make it impossible): that batch is partially written.
enum : uint64_t { kFaultTable = 1, kFaultHeap = 2, kFaultPartial = 4 };

// Value allocations come in size classes (0, then powers of two >= 16): a SET whose
// value's class is not above the class of the slot's current value length
// overwrites the bytes in place, so updating a key never grows the heap; only new
// keys and values outgrowing their allocation take heap bytes.
__device__ __forceinline__ uint64_t val_class(uint64_t len) {
  if (len == 0) return 0;
  uint64_t c = 16;
  while (c < len) c <<= 1;
  return c;
}

struct KvEntry {        // one table slot (the hash lives in its own array for probing)
  uint64_t key_off;     // heap offset of the key bytes
  uint64_t val_off;     // heap offset of the value bytes
  uint64_t version;     // ValueEntry.version; 0 = not live (deleted / never set)
  uint32_t key_len;
  uint32_t val_len;
};
static_assert(sizeof(KvEntry) == 32, "entry layout is part of rg_kv_dump");

struct KvOp {           // decoded command
  uint64_t key_off;     // offset into the batch's data bytes (a SET's value follows at
                        // key_off + key_len + 8, after its u64 length: kv_val_off)
  uint64_t hash;        // full key hash (kInvalidKey: not applied); one gather gives both
  uint32_t key_len;
  uint32_t val_len;
  uint32_t kind;        // 0 Set 1 Get 2 Delete 3 Exists
  uint32_t status;      // kPending or a final result code
};

__device__ __forceinline__ uint64_t kv_val_off(const KvOp& op) { return op.key_off + op.key_len + 8; }

struct KvCounters {
  unsigned long long live, version, total_ops, occupied, heap_top;
  unsigned long long batches, ordered, flags;
  unsigned long long mode;        // per batch: 0 keyed commit, 1 ordered replay, 2 fault, 3 capacity-ranked
  unsigned long long batch_base;  // heap top before the batch (keyed commit offsets)
  unsigned long long cut;         // mode 3: command index of the first create StoreFull refuses
                                  // (kCutBits: the refused creates are the kEvRefused bitmap)
};

// Per-block partials of the plan walk. kPLiveDel: DELETEs that hit a live key (the
// all-succeed replay); none in a batch => the live count only grows (mode 3).
enum { kPCreated = 0, kPNewSlots, kPOverflow, kPLiveDelta, kPVersion, kPOps, kPNeed, kPLiveDel, kPCount };
constexpr uint32_t kNoCreate = 0xFFFFFFFFu;
constexpr unsigned long long kCutBits = ~0ull - 1;

// What the commit writes for one key, decided by the plan (one record per distinct
// key of a hash run, at the run head's sorted position + the key's rank in the run).
struct KeyRec {
  int64_t slot;         // table slot (-1: the key gets a new slot)
  uint64_t ver1;        // version after the batch (0 = not live)
  uint64_t hash;        // full key hash (claiming the new slot)
  uint64_t key_src;     // batch data offset of the key bytes (new slot)
  uint64_t val_src;     // batch data offset of the final value
  uint64_t val_dst;     // heap offset of the slot's current value (in-place write)
  uint32_t key_len, val_len;
  uint32_t flags;
  uint32_t create;      // command index of the SET that creates the key (kNoCreate: none)
};
enum : uint32_t { kRecNew = 1, kRecValue = 2, kRecInPlace = 4, kRecVersion = 8, kRecLast = 16 };
constexpr int kWalkPerLane = 2;                              // sorted positions per walker lane
constexpr int kWalkSpan = 64 * kWalkPerLane;                 // positions per wave
constexpr int kWalkBlockSpan = kBlock * kWalkPerLane;        // positions per block
constexpr uint32_t kDecGroup = 256;                          // walk blocks per decide workgroup (one per thread)

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

// ---- decode fast path ----------------------------------------------------------
// A byte range [0, u) at q (u <= 8 * W, u > 0, q - 8 readable when u < 8) held as W
// words: word j starts at s_j = min(8j, u - 8), so every load stays inside the
// command and all of them issue at once (one round trip instead of one per loop
// iteration of utf8_valid / key_hash). Bytes of word j at offsets o hold range
// bytes s_j + o.
template <int W>
struct Span {
  uint64_t w[W];
  int32_t s[W];
  int nw;
};
template <int W>
__device__ __forceinline__ void span_load(Span<W>& sp, const uint8_t* q, uint32_t u) {
  sp.nw = (int)((u + 7) >> 3);
#pragma unroll
  for (int j = 0; j < W; j++) {
    const int32_t sj = min((int32_t)(8 * j), (int32_t)u - 8);
    sp.s[j] = sj;
    sp.w[j] = j < sp.nw ? ld_u64(q + sj) : 0;
  }
}
// mask of the bytes of word j that hold range bytes [lo, hi)
__device__ __forceinline__ uint64_t byte_mask(int32_t sj, int32_t lo, int32_t hi) {
  const int32_t a = max(lo - sj, 0), b = min(hi - sj, 8);
  if (b <= a) return 0;
  const uint64_t top = b == 8 ? ~0ull : ((1ull << (8 * b)) - 1ull);
  return top & ~((1ull << (8 * a)) - 1ull);
}
// all range bytes [0, n) are ASCII (n <= u)
template <int W>
__device__ __forceinline__ bool span_ascii(const Span<W>& sp, uint32_t n) {
  uint64_t acc = 0;
#pragma unroll
  for (int j = 0; j < W; j++)
    if (j < sp.nw) acc |= sp.w[j] & byte_mask(sp.s[j], 0, (int32_t)n);
  return (acc & 0x8080808080808080ull) == 0;
}
// key_hash over range bytes [0, n) (n == u), byte order as key_hash's
template <int W>
__device__ __forceinline__ uint64_t span_key_hash(const Span<W>& sp, uint32_t n, uint64_t hmask) {
  uint64_t h = 0xcbf29ce484222325ull;
#pragma unroll
  for (int b = 0; b < 8 * W; b++) {
    if (b < (int)n) {
      const int j = b >> 3;
      h = (h ^ ((sp.w[j] >> (8 * (b - sp.s[j]))) & 0xFFu)) * 0x100000001b3ull;
    }
  }
  h = fmix64(h ^ n) & hmask;
  if (h == kEmpty) h = 1;
  if (h == kInvalidKey) h = kInvalidKey - 1;
  return h;
}
template <int W>
__device__ __forceinline__ void span_store(uint8_t* dst, const Span<W>& sp) {
#pragma unroll
  for (int j = 0; j < W; j++)
    if (j < sp.nw) *(u64_unaligned*)(dst + sp.s[j]) = sp.w[j];  // overlapping words carry equal bytes
}
// Copy of n bytes with every load issued before the first store (the byte pointers
// may alias as far as the compiler knows, so a load-store loop is one round trip per
// word); n in [8, 64], else the word loop.
__device__ __forceinline__ void copy_fast(uint8_t* dst, const uint8_t* src, uint32_t n) {
  if (n >= 8 && n <= 64) {
    Span<8> sp;
    span_load(sp, src, n);
    span_store(dst, sp);
  } else {
    bytes_copy(dst, src, n);
  }
}
// Byte equality of two n-byte strings, n in [8, 16] with all four words in flight at
// once (bytes_eq's early-exit loop is one round trip per word), else bytes_eq.
__device__ __forceinline__ bool eq_fast(const uint8_t* a, const uint8_t* b, uint32_t n) {
  if (n >= 8 && n <= 16) {
    Span<2> x, y;
    span_load(x, a, n);
    span_load(y, b, n);
    return x.w[0] == y.w[0] && x.w[1] == y.w[1];  // equal offsets on both sides; word 1 is 0 when absent
  }
  return bytes_eq(a, b, n);
}
constexpr uint32_t kFastKey = 16, kFastVal = 64;  // decode fast path: key <= 16 B, value region <= 64 B

// Event bitmaps of a batch that may meet StoreFull (BatchView.cbits), one bit per
// command index, plane p at cbits + p * kv_plane(n): kEvCreate = SETs on a key that is not
// live in the all-succeed replay, kEvDelete = DELETEs of a live key there, kEvTail = the
// creates that are their key's last SET / DELETE of the batch, kEvRefused = the creates
// StoreFull refuses (decide, batches with live-key DELETEs). Decode zeroes the first three.
enum { kEvCreate = 0, kEvDelete = 1, kEvTail = 2, kEvRefused = 3, kEvPlanes = 4 };
__host__ __device__ __forceinline__ uint64_t kv_plane(uint64_t n) { return (n + 31) / 32; }

// ---- 1 decode ----------------------------------------------------------------
constexpr int kSetPart = 3;  // decode partials per block: pending SETs, their worst-case bytes, pending DELETEs
__global__ __launch_bounds__(kBlock) void kv_decode_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ off, uint64_t n, const uint8_t* __restrict__ mask,
    uint64_t max_value, uint64_t hmask, uint64_t bmask, uint32_t invalid_bucket, KvOp* __restrict__ ops,
    uint32_t* __restrict__ sort_key, uint8_t* __restrict__ results,
    unsigned long long* __restrict__ set_part, uint8_t* __restrict__ done, uint32_t* __restrict__ cbits,
    unsigned long long* __restrict__ cbytes) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sets = 0, set_bytes = 0, dels = 0;  // worst-case growth of the batch (the refusal check)
  if (c < n) {
  KvOp op{0, kInvalidKey, 0, 0, 0, kPending};
  uint64_t key = kInvalidKey;
  if (mask && !mask[c]) {
    op.status = RG_KV_NOT_APPLIED;
  } else {
    const uint64_t b = off[c], e = off[c + 1];
    const uint64_t len = e > b ? e - b : 0;
    const uint8_t* p = data + b;
    op.status = RG_KV_E_DECODE;
    const uint32_t kind0 = len >= 12 ? ld_u32(p) : 0xFFFFFFFFu;
    const uint64_t klen0 = len >= 12 ? ld_u64(p + 4) : ~0ull;
    // fast path (short ASCII key, SET value region <= 64 B): the key words, the value
    // length and the value region's words are loaded together
    const uint64_t urest = kind0 == 0 && klen0 <= len - 12 && len - 12 - klen0 >= 8 ? len - 20 - klen0 : ~0ull;
    const bool fast = kind0 <= 3 && klen0 >= 1 && klen0 <= kFastKey && klen0 <= len - 12 &&
                      (kind0 != 0 || urest <= kFastVal);
    bool done = false;
    if (fast) {
      const uint32_t kl = (uint32_t)klen0;
      Span<2> ks;
      span_load(ks, p + 12, kl);
      uint64_t vlen = 0;
      bool vok = true;
      if (kind0 == 0) {
        const uint32_t u = (uint32_t)urest;
        vlen = ld_u64(p + 12 + kl);
        Span<8> vs;
        if (u) span_load(vs, p + 20 + kl, u);
        if (vlen > u) vok = false;               // decode error (slow path reports it)
        else if (vlen && !span_ascii(vs, (uint32_t)vlen)) vok = false;
      }
      if (vok && span_ascii(ks, kl)) {
        op.kind = kind0;
        op.key_off = b + 12;
        op.key_len = kl;
        op.val_len = (uint32_t)vlen;
        if (kind0 == 0 && vlen > max_value) op.status = RG_KV_E_VALUE_LARGE;  // store.rs:473-477
        else {
          op.status = kPending;
          key = span_key_hash(ks, kl, hmask);
        }
        done = true;
      }
    }
    if (!done && len >= 12) {
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
  op.hash = key;
  ops[c] = op;
  sort_key[c] = key == kInvalidKey ? invalid_bucket : (uint32_t)hash_bucket(key, bmask);
  done[c] = 0;  // the plan's per-sorted-position marks (multi-key runs), cleared here: no memset launch
  if (cbits) {  // the event bitmaps and reservations (when StoreFull can fire), likewise
    if ((c & 31u) == 0) {
      const uint64_t pl = kv_plane(n);
      cbits[c >> 5] = 0;
      cbits[pl + (c >> 5)] = 0;
      cbits[2 * pl + (c >> 5)] = 0;
    }
    cbytes[c] = 0;
  }
  if (op.status != kPending) results[c] = (uint8_t)op.status;
  if (op.status == kPending && op.kind == 0) {
    sets = 1;
    set_bytes = op.key_len + val_class(op.val_len);
  }
  dels = op.status == kPending && op.kind == 2;
  }
  __shared__ unsigned long long red[kBlock / 64][3];
  for (int o = 32; o > 0; o >>= 1) {
    sets += __shfl_xor(sets, o, 64);
    set_bytes += __shfl_xor(set_bytes, o, 64);
    dels += __shfl_xor(dels, o, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red[wave][0] = sets; red[wave][1] = set_bytes; red[wave][2] = dels; }
  __syncthreads();
  if (threadIdx.x < kSetPart) {
    unsigned long long t = 0;
    for (int w = 0; w < kBlock / 64; w++) t += red[w][threadIdx.x];
    set_part[(uint64_t)blockIdx.x * kSetPart + threadIdx.x] = t;
  }
}

// ---- table lookup ------------------------------------------------------------
// Returns the slot holding `key` (live or not) or -1, and its entry in *out.
// Linear probing; an empty slot ends the chain. Concurrent inserts by other walkers
// carry other hashes. Entries are read with agent-scope loads: plain loads of
// entries the previous batch's commit wrote field by field were measured to return
// stale fields on the next batch (a version or value length of 0 on a live key).
__device__ int64_t table_find(const uint64_t* hashes, const KvEntry* ent, const uint8_t* heap,
                              uint64_t mask, uint64_t h, const uint8_t* key, uint32_t klen, KvEntry* out) {
  uint64_t s = h & mask;
  for (uint64_t probes = 0; probes <= mask; probes++) {
    const uint64_t th = __hip_atomic_load(hashes + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (th == kEmpty) return -1;
    if (th == h) {
      KvEntry e;
      const unsigned long long* ep = reinterpret_cast<const unsigned long long*>(ent + s);
      e.key_off = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e.val_off = __hip_atomic_load(ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e.version = __hip_atomic_load(ep + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long lens = __hip_atomic_load(ep + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e.key_len = (uint32_t)lens;
      e.val_len = (uint32_t)(lens >> 32);
      if (e.key_len == klen && eq_fast(heap + e.key_off, key, klen)) {
        *out = e;
        return (int64_t)s;
      }
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
  const uint32_t* skey;   // sorted hash buckets
  const uint32_t* sidx;   // command index per sorted position (0xFFFFFFFF in the not-applied tail)
  uint64_t n;
  uint8_t* results;
  uint8_t* done;          // per sorted position: handled by an earlier key of its run (multi-key runs)
  uint64_t* need;         // per sorted position: plan bytes (run heads only)
  uint64_t* block_base;   // per walk block: heap offset of its first byte inside its decide group
  uint64_t* group_base;   // per decide group (kDecGroup walk blocks): heap offset of its first byte
  KeyRec* recs;           // per sorted position: plan -> commit records (run head + key rank)
  uint32_t invalid_bucket;  // sort key of the commands that are not applied (sorted last)
  unsigned long long* part;  // [blocks][kPCount]
  uint32_t* cbits;           // event bitmaps by command index, 4 planes of kv_plane(n) words (kEv*),
                             // NULL when StoreFull cannot fire
  unsigned long long* cbytes;  // per command: heap bytes its key reserves when it is the key's last create
};

__device__ __forceinline__ bool same_key(const BatchView& b, const KvOp& x, const KvOp& y) {
  return x.key_len == y.key_len && bytes_eq(b.data + x.key_off, b.data + y.key_off, x.key_len);
}

// One key's replay state over its commands in total order.
struct KeyOutcome {
  bool live0, live1, wrote_value, any_set;
  uint64_t ver0, ver1;
  uint32_t last_set;     // command index of the final value's SET
  uint32_t last_create;  // position of the last SET on a non-live key (kNoCreate: none)
  uint32_t last_mut;     // position of the last SET or DELETE
  uint64_t n_ops, n_version, n_live_del;
};

__device__ __forceinline__ KeyOutcome key_start(int64_t slot, const KvEntry& e) {
  KeyOutcome o{};
  o.live0 = o.live1 = slot >= 0 && e.version > 0;
  o.ver0 = o.ver1 = o.live0 ? e.version : 0;
  o.last_create = o.last_mut = kNoCreate;
  return o;
}

// Applies one command of the key; returns its result code.
__device__ __forceinline__ uint8_t key_step(KeyOutcome& o, uint32_t kind, uint32_t c, uint32_t notify) {
  uint8_t r;
  if (kind == 0) {                    // SET: update or insert (store.rs:151-163)
    if (!o.live1) o.last_create = c;
    o.last_mut = c;
    o.ver1 = o.live1 ? o.ver1 + 1 : 1;
    o.live1 = true;
    o.wrote_value = true;
    o.any_set = true;
    o.last_set = c;
    o.n_version += notify;
    r = RG_KV_SUCCESS;
  } else if (kind == 2) {             // DELETE (store.rs:220-251)
    r = o.live1 ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
    o.last_mut = c;
    if (o.live1) {
      o.n_version += notify;
      o.wrote_value = false;
      o.n_live_del++;
    }
    o.live1 = false;
    o.ver1 = 0;
  } else {                            // GET / EXISTS (smr_impl.rs:79-94)
    r = o.live1 ? RG_KV_SUCCESS : RG_KV_NOT_FOUND;
  }
  o.n_ops++;
  return r;
}

// key_step plus the command's event bits (cmd: its command index; ev: the event planes
// of a batch that may meet StoreFull, else NULL).
__device__ __forceinline__ uint8_t key_step_ev(KeyOutcome& o, uint32_t kind, uint32_t pos, uint32_t cmd,
                                               uint32_t notify, uint32_t* ev, uint64_t plane) {
  if (ev) {
    const uint32_t bit = 1u << (cmd & 31u);
    if (kind == 0 && !o.live1) atomicOr(ev + kEvCreate * plane + (cmd >> 5), bit);
    else if (kind == 2 && o.live1) atomicOr(ev + kEvDelete * plane + (cmd >> 5), bit);
  }
  return key_step(o, kind, pos, notify);
}

// Folds a replayed key into the block partials and its commit record; returns the
// heap bytes the commit will take for it (new key bytes + a new value allocation).
// (vsrc, vlen: the final value's bytes, from the SET the replay recorded in last_set.)
// (create: the command index of the key's last create, o.last_create translated by the
// caller; tail: it is also the key's last SET / DELETE. When StoreFull can fire, the
// key's plan bytes are reserved at the create and a tail create gets its kEvTail bit:
// refusing it changes nothing else in the batch.)
__device__ uint64_t plan_key(const KeyOutcome& o, int64_t slot, const KvEntry& e, uint64_t key_off,
                             uint32_t key_len, uint64_t vsrc, uint32_t vlen, uint64_t hl, uint32_t create, bool tail,
                             uint32_t* cbits, uint64_t plane, unsigned long long* cbytes,
                             unsigned long long (&acc)[kPCount], KeyRec& r) {
  acc[kPLiveDel] += o.n_live_del;
  acc[kPOps] += o.n_ops;
  acc[kPVersion] += o.n_version;
  acc[kPLiveDelta] += (unsigned long long)((int64_t)o.live1 - (int64_t)o.live0);
  acc[kPCreated] += !o.live0 && o.any_set;  // keys live at some point of the batch (bound on data.len())
  const bool new_slot = slot < 0 && o.live1;
  acc[kPNewSlots] += new_slot;
  const bool value = o.live1 && o.wrote_value;
  if (!value) {
    vsrc = 0;
    vlen = 0;
  }
  // in place when the final value's class fits the slot's current allocation
  const bool in_place = value && slot >= 0 && val_class(vlen) <= val_class(e.val_len);
  r.slot = slot;
  r.ver1 = o.live1 ? o.ver1 : 0;
  r.hash = hl;
  r.key_src = key_off;
  r.val_src = vsrc;
  r.val_dst = e.val_off;
  r.key_len = key_len;
  r.val_len = vlen;
  r.flags = (new_slot ? kRecNew : 0u) | (value ? kRecValue : 0u) | (in_place ? kRecInPlace : 0u) |
            ((slot >= 0 || new_slot) && (o.any_set || o.live0 != o.live1) ? kRecVersion : 0u);
  r.create = create;
  const uint64_t need = (new_slot ? key_len : 0) + (value && !in_place ? val_class(vlen) : 0);
  if (cbits && create != kNoCreate) {  // StoreFull reachable: the key's reservation, the tail bit
    cbytes[create] = need;
    if (tail) atomicOr(cbits + kEvTail * plane + (create >> 5), 1u << (create & 31u));
  }
  return need;
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
// Each wave owns kWalkSpan consecutive sorted positions (a block kWalkBlockSpan).
// Plan: every lane first loads its positions' command index and kind and whether
// the command's key equals the previous position's (phase A, all loads in
// parallel, kept in LDS); the run heads are compacted per wave and each lane then
// replays one head's run at a time out of LDS (phase B): one table lookup per key,
// results written, and a KeyRec telling the commit what to write. A run that holds
// several keys (a bucket collision) or continues past the block takes the general
// path over global memory. The block totals go to the partials; decide scans the
// plan bytes into per-block bases and commit, a separate launch over the same
// heads, writes table entries and heap bytes from the records at offsets from a
// block scan of the plan sizes: no lookups, no replay.
__device__ __forceinline__ uint32_t collect_heads(const BatchView& b, uint64_t wbase, int lane, bool go,
                                                  uint16_t* heads) {
  uint32_t nh = 0;
#pragma unroll
  for (int k = 0; k < kWalkPerLane; k++) {
    const uint64_t i = wbase + 64 * k + lane;
    bool head = false;
    if (go && i < b.n) {
      const uint32_t h = b.skey[i];
      head = h != b.invalid_bucket && (i == 0 || b.skey[i - 1] != h);
    }
    const unsigned long long m = __ballot(head);
    if (head) heads[nh + __builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint16_t)(64 * k + lane);
    nh += (uint32_t)__builtin_popcountll(m);
  }
  __builtin_amdgcn_wave_barrier();
  return nh;
}

enum : uint8_t { kInfCont = 4, kInfSame = 8 };  // bits 0-1: kind

// LDS written by this wave's lanes, then read by other lanes of the same wave.
__device__ __forceinline__ void lds_wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Waves per SIMD the plan is compiled for (its VGPR budget; LDS allows 10).
#ifndef RG_KV_PLAN_WAVES
#define RG_KV_PLAN_WAVES 5  // 4 (103 VGPRs): apply 545.2 / 546.0 us, 5 (83, no spill): 538.7 / 538.6, 6 (80 + spills): 545.1 / 544.4 (profiles/r06/c4_plan_occ_ab.json)
#endif
__global__ __launch_bounds__(kBlock, RG_KV_PLAN_WAVES) void kv_plan_kernel(BatchView b, StoreView st) {
  __shared__ uint32_t s_c[kWalkBlockSpan];
  __shared__ uint8_t s_inf[kWalkBlockSpan];
  __shared__ uint16_t s_heads[kBlock / 64][kWalkSpan];
  // each position's decoded command fields, gathered once (phase A) and read by the
  // same-key compare of the next position, the run head's lookup and the final
  // value's source: no second gather of a KvOp on the single-key path
  __shared__ uint64_t s_hash[kWalkBlockSpan];
  __shared__ uint64_t s_koff[kWalkBlockSpan];
  __shared__ uint32_t s_klen[kWalkBlockSpan];
  __shared__ uint32_t s_vlen[kWalkBlockSpan];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long acc[kPCount] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t bbase = (uint64_t)blockIdx.x * kWalkBlockSpan;
  const uint32_t wl = (uint32_t)wave * kWalkSpan;
  const uint64_t plane = kv_plane(b.n);
  if (b.skey[bbase] == b.invalid_bucket) {  // the sorted tail of commands not applied: nothing to plan
    if (threadIdx.x < kPCount) b.part[(uint64_t)blockIdx.x * kPCount + threadIdx.x] = 0;
    return;
  }
  // phase A1: per position, command index, kind, continues the previous bucket, and
  // the command's fields into LDS (all gathers of the wave in flight at once)
#pragma unroll
  for (int k = 0; k < kWalkPerLane; k++) {
    const uint32_t l = wl + 64 * k + lane;
    const uint64_t i = bbase + l;
    uint32_t c = 0, inf = 0;
    if (i < b.n) {
      const uint32_t h = b.skey[i];
      if (h != b.invalid_bucket) {
        c = b.sidx[i];
        const KvOp op = b.ops[c];
        inf = (op.kind & 3u) | (i > 0 && b.skey[i - 1] == h ? kInfCont : 0u);
        s_hash[l] = op.hash;
        s_koff[l] = op.key_off;
        s_klen[l] = op.key_len;
        s_vlen[l] = op.val_len;
      }
    }
    s_c[l] = c;
    s_inf[l] = (uint8_t)inf;
  }
  lds_wave_sync();
  // phase A2: same key as the previous position (key bytes decide); run heads
  // compacted per wave. The previous position is in this wave's LDS except for the
  // wave's first one.
  uint32_t nh = 0;
#pragma unroll
  for (int k = 0; k < kWalkPerLane; k++) {
    const uint32_t l = wl + 64 * k + lane;
    const uint64_t i = bbase + l;
    uint32_t inf = s_inf[l];
    const bool head = i < b.n && b.skey[i] != b.invalid_bucket && !(inf & kInfCont);
    if (inf & kInfCont) {
      uint64_t ph, pko;
      uint32_t pkl;
      if (l > wl) {
        ph = s_hash[l - 1];
        pko = s_koff[l - 1];
        pkl = s_klen[l - 1];
      } else {
        const KvOp pp = b.ops[b.sidx[i - 1]];
        ph = pp.hash;
        pko = pp.key_off;
        pkl = pp.key_len;
      }
      const uint32_t kl = s_klen[l];
      const bool eq = s_hash[l] == ph && kl == pkl && eq_fast(b.data + s_koff[l], b.data + pko, kl);
      if (eq) s_inf[l] = (uint8_t)(inf | kInfSame);
    }
    const unsigned long long m = __ballot(head);
    if (head) s_heads[wave][nh + __builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint16_t)(64 * k + lane);
    nh += (uint32_t)__builtin_popcountll(m);
  }
  __syncthreads();
  // phase B: one run per lane at a time
  for (uint32_t h = lane; h < nh; h += 64) {
    const uint32_t l0 = wl + s_heads[wave][h];
    const uint64_t i = bbase + l0;
    uint32_t l = l0 + 1;
    bool single = true;
    while (l < (uint32_t)kWalkBlockSpan && (s_inf[l] & kInfCont)) {
      single = single && (s_inf[l] & kInfSame);
      l++;
    }
    if (l == (uint32_t)kWalkBlockSpan && bbase + l < b.n && b.skey[bbase + l] == b.skey[i]) single = false;
    uint64_t need = 0;
    if (single) {  // one key, every command in LDS
      const uint64_t hl = s_hash[l0], koff = s_koff[l0];
      const uint32_t klen = s_klen[l0];
      KvEntry e{};
      const int64_t slot = table_find(st.hashes, st.ent, st.heap, st.mask, hl, b.data + koff, klen, &e);
      KeyOutcome o = key_start(slot, e);
      for (uint32_t q = l0; q < l; q++)  // last_set / last_create record the LDS position here
        b.results[s_c[q]] = key_step_ev(o, s_inf[q] & 3u, q, s_c[q], st.notify, b.cbits, plane);
      const uint32_t ls = o.last_set;
      KeyRec r;
      need = plan_key(o, slot, e, koff, klen, s_koff[ls] + s_klen[ls] + 8, s_vlen[ls], hl,
                      o.last_create == kNoCreate ? kNoCreate : s_c[o.last_create], o.last_create == o.last_mut,
                      b.cbits, plane, b.cbytes, acc, r);
      r.flags |= kRecLast;
      b.recs[i] = r;
    } else {       // general: split the bucket run into keys by their bytes
      const uint32_t hb = b.skey[i];
      uint64_t end = i + 1;
      while (end < b.n && b.skey[end] == hb) end++;
      uint32_t keys = 0;
      KeyRec r;
      for (uint64_t first = i; first < end; first++) {
        if (b.done[first]) continue;
        if (keys == (uint32_t)kMaxRunKeys) { acc[kPOverflow] = 1; break; }
        if (keys) b.recs[i + keys - 1] = r;
        keys++;
        const uint32_t c0 = b.sidx[first];
        const KvOp lead = b.ops[c0];
        const uint64_t hl = lead.hash;
        KvEntry e{};
        const int64_t slot = table_find(st.hashes, st.ent, st.heap, st.mask, hl, b.data + lead.key_off,
                                        lead.key_len, &e);
        KeyOutcome o = key_start(slot, e);
        for (uint64_t q = first; q < end; q++) {
          if (b.done[q]) continue;
          const uint32_t c = b.sidx[q];
          const KvOp op = b.ops[c];
          if (q != first && !(op.hash == hl && same_key(b, op, lead))) continue;
          b.done[q] = 1;
          b.results[c] = key_step_ev(o, op.kind, c, c, st.notify, b.cbits, plane);
        }
        uint64_t vsrc = 0;
        uint32_t vlen = 0;
        if (o.wrote_value) {
          const KvOp v = b.ops[o.last_set];
          vsrc = kv_val_off(v);
          vlen = v.val_len;
        }
        need += plan_key(o, slot, e, lead.key_off, lead.key_len, vsrc, vlen, hl, o.last_create,
                         o.last_create == o.last_mut, b.cbits, plane, b.cbytes, acc, r);
      }
      if (keys) {
        r.flags |= kRecLast;
        b.recs[i + keys - 1] = r;
      }
    }
    b.need[i] = need;
    acc[kPNeed] += need;
  }
  block_add_partials(acc, b.part);
}

__device__ void kv_ordered(const uint8_t* data, const KvOp* ops, uint64_t n, uint8_t* results, StoreView st);

// Mode 3, a key whose (last) create StoreFull refuses (its command index >= the cut, or
// its kEvRefused bit): from the create on, the key stays absent (store.rs:153-158: the
// SET fails; no later SET or DELETE of the key: without live-key DELETEs the store stays
// full, with them decide checked that the create is the key's last mutation), so its
// SETs answer StoreFull and its GETs / EXISTS NotFound. Its commands are the bucket run's (one key) or, in a run of several
// keys, those with its hash and key bytes. The counters lose what the all-succeed
// replay counted for it: the live key, the slot of a new key, and per refused SET one
// operation and (notifications on) one version.
struct RefuseCorr {
  unsigned long long live, occupied, ops, version;
};
__device__ void refuse_key(const BatchView& b, uint64_t i, const KeyRec& r, bool one_key, uint32_t notify,
                           RefuseCorr& corr) {
  const uint32_t bucket = b.skey[i];
  for (uint64_t q = i; q < b.n && b.skey[q] == bucket; q++) {
    const uint32_t c = b.sidx[q];
    if (c < r.create) continue;  // before the create the key is absent either way
    const KvOp op = b.ops[c];
    if (!one_key && !(op.hash == r.hash && op.key_len == r.key_len &&
                      bytes_eq(b.data + op.key_off, b.data + r.key_src, r.key_len)))
      continue;
    if (op.kind == 0) {
      b.results[c] = RG_KV_E_FULL;
      corr.ops++;
      corr.version += notify;
    } else {
      b.results[c] = RG_KV_NOT_FOUND;
    }
  }
  corr.live++;
  corr.occupied += (r.flags & kRecNew) ? 1u : 0u;
}

// The commit launch also closes the batch on the other two paths decide may pick (one
// launch fewer per batch than a separate close kernel): mode 1, the exact in-order
// replay (one thread); mode 2, the refusal (every pending command gets
// RG_KV_E_CAPACITY, grid-stride). Mode 3 is mode 0 with the keys whose create is
// refused left out (refuse_key).
#ifndef RG_KV_COMMIT_WAVES
#define RG_KV_COMMIT_WAVES 5  // 86 VGPRs; 6 (80 + spills): no gain (539.9 / 541.0 us with the plan at 5)
#endif
__global__ __launch_bounds__(kBlock, RG_KV_COMMIT_WAVES) void kv_commit_kernel(BatchView b, StoreView st) {
  __shared__ uint16_t s_heads[kBlock / 64][kWalkSpan];
  __shared__ unsigned long long s_wsum[kBlock / 64];
  const unsigned long long mode = st.ctr->mode;  // uniform over the grid
  if (mode == 1) {
    if (blockIdx.x == 0 && threadIdx.x == 0) kv_ordered(b.data, b.ops, b.n, b.results, st);
    return;
  }
  if (mode == 2) {
    for (uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x; c < b.n; c += (uint64_t)gridDim.x * kBlock)
      if (b.ops[c].status == kPending) b.results[c] = RG_KV_E_CAPACITY;
    return;
  }
  if (b.skey[(uint64_t)blockIdx.x * kWalkBlockSpan] == b.invalid_bucket) return;  // no heads in the tail
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t wbase = (uint64_t)blockIdx.x * kWalkBlockSpan + (uint64_t)wave * kWalkSpan;
  const uint32_t nh = collect_heads(b, wbase, lane, true, s_heads[wave]);
  const unsigned long long cut = mode == 3 ? st.ctr->cut : ~0ull;
  const uint32_t* evr = b.cbits ? b.cbits + kEvRefused * kv_plane(b.n) : nullptr;
  auto refused = [&](uint32_t cr) {  // mode 3: StoreFull refuses the key's (last) create
    if (cr == kNoCreate) return false;
    if (cut == kCutBits) return ((evr[cr >> 5] >> (cr & 31u)) & 1u) != 0;
    return cr >= cut;
  };
  // this lane's heap offset: block base + exclusive prefix of plan sizes over (wave, lane)
  // (mode 3: the sizes of the keys that are not refused, and the workgroup's base from
  // one atomic on the heap top: the decide scan counted the refused keys too)
  unsigned long long mine = 0;
  if (mode == 3) {
    for (uint32_t h = lane; h < nh; h += 64)
      for (uint64_t k = wbase + s_heads[wave][h]; k < b.n; k++) {
        const KeyRec r = b.recs[k];
        if (!refused(r.create))
          mine += (r.flags & kRecNew) ? r.key_len + val_class(r.val_len)
                                      : ((r.flags & kRecValue) && !(r.flags & kRecInPlace) ? val_class(r.val_len) : 0);
        if (r.flags & kRecLast) break;
      }
  } else {
    for (uint32_t h = lane; h < nh; h += 64) mine += b.need[wbase + s_heads[wave][h]];
  }
  unsigned long long incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  unsigned long long before = 0;
  for (int w = 0; w < wave; w++) before += s_wsum[w];
  __shared__ unsigned long long s_base;
  if (mode == 3) {
    if (threadIdx.x == 0) {
      unsigned long long tot = 0;
      for (int w = 0; w < kBlock / 64; w++) tot += s_wsum[w];
      s_base = tot ? atomicAdd(&st.ctr->heap_top, tot) : 0ull;
    }
    __syncthreads();
  }
  uint64_t heap_pos = (mode == 3 ? s_base
                                 : st.ctr->batch_base + b.group_base[blockIdx.x / kDecGroup] + b.block_base[blockIdx.x]) +
                      before + incl - mine;
  RefuseCorr corr{0, 0, 0, 0};
  for (uint32_t h = lane; h < nh; h += 64) {
    const uint64_t i = wbase + s_heads[wave][h];
    // a run holds at most kMaxRunKeys records (more sends the batch to the ordered
    // path); the bounds below only guard against a plan/commit mismatch
    for (uint64_t k = i; k < b.n && k < i + kMaxRunKeys; k++) {
      const KeyRec r = b.recs[k];
      int64_t s = r.slot;
      if (refused(r.create)) {  // mode 3: StoreFull refuses this key's create
        refuse_key(b, i, r, k == i && (r.flags & kRecLast), st.notify, corr);
        // a key live before the batch and deleted in it before the refused create ends
        // absent (the create is its last mutation): its entry's version goes to 0
        if (s >= 0) st.ent[s].version = 0;
        if (r.flags & kRecLast) break;
        continue;
      }
      if (r.flags & kRecNew) {  // a new key always ends live with a value: the whole entry at once
        s = table_claim(st.hashes, st.mask, r.hash);
        const uint64_t koff = heap_pos, voff = heap_pos + r.key_len;
        heap_pos += r.key_len + val_class(r.val_len);
        if (s < 0 || heap_pos > st.heap_cap) {
          atomicOr(&st.ctr->flags, (s < 0 ? kFaultTable : kFaultHeap) | kFaultPartial);
        } else {
          if (r.key_len >= 8 && r.key_len <= 16 && r.val_len >= 8 && r.val_len <= 64) {
            Span<2> ks;  // key and value words all in flight before the stores
            Span<8> vs;
            span_load(ks, b.data + r.key_src, r.key_len);
            span_load(vs, b.data + r.val_src, r.val_len);
            span_store(st.heap + koff, ks);
            span_store(st.heap + voff, vs);
          } else {
            bytes_copy(st.heap + koff, b.data + r.key_src, r.key_len);
            bytes_copy(st.heap + voff, b.data + r.val_src, r.val_len);
          }
          const KvEntry e{koff, voff, r.ver1, r.key_len, r.val_len};
          st.ent[s] = e;
        }
        if (r.flags & kRecLast) break;
        continue;
      }
      if (s >= 0 && (r.flags & kRecValue)) {
        uint64_t dst = r.val_dst;
        if (!(r.flags & kRecInPlace)) {
          dst = heap_pos;
          heap_pos += val_class(r.val_len);
        }
        if (dst + r.val_len > st.heap_cap) {
          atomicOr(&st.ctr->flags, kFaultHeap | kFaultPartial);
        } else {
          copy_fast(st.heap + dst, b.data + r.val_src, r.val_len);
          st.ent[s].val_off = dst;
          st.ent[s].val_len = r.val_len;
        }
      }
      if (s >= 0 && (r.flags & kRecVersion)) st.ent[s].version = r.ver1;
      if (r.flags & kRecLast) break;
    }
  }
  if (mode != 3) return;  // (uniform)
  unsigned long long v[4] = {corr.live, corr.occupied, corr.ops, corr.version};
#pragma unroll
  for (int q = 0; q < 4; q++)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
  __shared__ unsigned long long s_corr[kBlock / 64][4];
  if (lane == 0)
    for (int q = 0; q < 4; q++) s_corr[wave][q] = v[q];
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
    for (int w = 0; w < kBlock / 64; w++) t += s_corr[w][threadIdx.x];
    unsigned long long* dst[4] = {&st.ctr->live, &st.ctr->occupied, &st.ctr->total_ops, &st.ctr->version};
    if (t) atomicAdd(dst[threadIdx.x], ~t + 1ull);  // subtract (two's complement)
  }
}

// ---- 4 decide ----------------------------------------------------------------
// Folds the plan partials and picks the batch's path:
//   0 keyed commit: StoreFull unreachable (live + keys created <= max_keys);
//   1 ordered replay: exact in-order path;
//   2 refused: a capacity (table slots or heap bytes) cannot hold the batch's
//     worst case — nothing is written, every pending command gets RG_KV_E_CAPACITY.
// Multi-workgroup: workgroup g owns walk blocks [256g, 256g + 256) and a share of the
// decode partials. It folds them (every load in flight at once), scans its walk blocks'
// plan bytes (block_base = the offset inside the group) and publishes one row of
// dpart; the last workgroup to arrive folds the rows, scans the group totals into
// group_base (the commit adds both), picks the path and, on the keyed path, applies
// the counter deltas (live, version, total_operations: nothing reads them between here
// and the next batch's decide). Round 4 ran this as one 1024-thread workgroup (20 us
// per 2^22 commands: a chain of dependent loads on one CU) plus a second fold in a
// close kernel.
constexpr int kDecBlock = 256;
static_assert(kDecGroup == (uint32_t)kDecBlock, "decide: one walk block per thread");
enum {
  kDCreated = 0, kDNewSlots, kDOverflow, kDSets, kDSetBytes, kDNeed, kDLive, kDVersion, kDOps, kDLiveDel, kDDels,
  kDCount
};

__device__ __forceinline__ void dec_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long dec_load(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kDecBlock) void kv_decide_kernel(StoreView st, const unsigned long long* part,
                                                              uint32_t walk_blocks, const unsigned long long* set_part,
                                                              uint32_t blocks, uint64_t* block_base,
                                                              uint64_t* group_base, unsigned long long* dpart,
                                                              unsigned long long* arrivals, uint32_t* cbits,
                                                              const unsigned long long* cbytes, uint64_t n_cmds) {
  __shared__ unsigned long long red[kDecBlock / 64][kDCount];
  __shared__ uint32_t s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t g = blockIdx.x, D = gridDim.x;
  // the store counters the last workgroup decides with, loaded now (the previous batch
  // wrote them: stream order) so the load is not on the fold's dependent chain
  KvCounters* k = st.ctr;
  const unsigned long long live0 = k->live, occ0 = k->occupied, top0 = k->heap_top, flags0 = k->flags;
  const unsigned long long batches0 = k->batches, ver0 = k->version, ops0 = k->total_ops;
  unsigned long long v[kDCount] = {};
  {  // this group's walk blocks, one per thread: folds + the in-group scan of plan bytes
    const uint32_t wb = g * kDecGroup + (uint32_t)tid;
    unsigned long long x[kPCount] = {};
    if (wb < walk_blocks)
#pragma unroll
      for (int k = 0; k < kPCount; k++) x[k] = part[(uint64_t)wb * kPCount + k];
    v[kDCreated] = x[kPCreated];
    v[kDNewSlots] = x[kPNewSlots];
    v[kDOverflow] = x[kPOverflow];
    v[kDLive] = x[kPLiveDelta];
    v[kDVersion] = x[kPVersion];
    v[kDOps] = x[kPOps];
    v[kDLiveDel] = x[kPLiveDel];
    unsigned long long incl = x[kPNeed];  // inclusive scan: over the wave, then the waves before
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    __shared__ unsigned long long s_wtot[kDecBlock / 64];
    if (lane == 63) s_wtot[wave] = incl;
    __syncthreads();
    for (int w = 0; w < wave; w++) incl += s_wtot[w];
    if (wb < walk_blocks) block_base[wb] = incl - x[kPNeed];
    v[kDNeed] = x[kPNeed];
  }
  {  // this group's share of the decode partials (pending SETs, their worst-case bytes)
    const uint32_t per = (blocks + D - 1) / D, r0 = g * per, r1 = r0 + per < blocks ? r0 + per : blocks;
    for (uint32_t r = r0 + (uint32_t)tid; r < r1; r += kDecBlock) {
      v[kDSets] += set_part[(uint64_t)r * kSetPart];
      v[kDSetBytes] += set_part[(uint64_t)r * kSetPart + 1];
      v[kDDels] += set_part[(uint64_t)r * kSetPart + 2];
    }
  }
#pragma unroll
  for (int k = 0; k < kDCount; k++) {  // (overflow: any nonzero sum)
    unsigned long long t = v[k];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) red[wave][k] = t;
  }
  __syncthreads();
  if (tid < kDCount) {
    unsigned long long t = 0;
    for (int w = 0; w < kDecBlock / 64; w++) t += red[w][tid];
    dec_store(dpart + (uint64_t)g * kDCount + tid, t);
  }
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    s_last = atomicAdd(arrivals, 1ull) == D - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  // the last workgroup: fold every group's row; exclusive scan of the groups' plan bytes
  const uint32_t per = (D + kDecBlock - 1) / kDecBlock;
  const uint32_t lo = (uint32_t)tid * per, hi = lo + per < D ? lo + per : D;
  unsigned long long f[kDCount] = {};
  for (uint32_t q = lo; q < hi; q++)
#pragma unroll
    for (int k = 0; k < kDCount; k++) f[k] += dec_load(dpart + (uint64_t)q * kDCount + k);
  __shared__ unsigned long long s_scan[kDecBlock];
  s_scan[tid] = f[kDNeed];
  __syncthreads();
  for (int o = 1; o < kDecBlock; o <<= 1) {  // inclusive Hillis-Steele over the thread sums
    const unsigned long long t = tid >= o ? s_scan[tid - o] : 0ull;
    __syncthreads();
    s_scan[tid] += t;
    __syncthreads();
  }
  unsigned long long off = s_scan[tid] - f[kDNeed];
  for (uint32_t q = lo; q < hi; q++) {
    group_base[q] = off;
    off += dec_load(dpart + (uint64_t)q * kDCount + kDNeed);
  }
#pragma unroll
  for (int k = 0; k < kDCount; k++) {
    unsigned long long t = f[k];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) red[wave][k] = t;
  }
  __syncthreads();
  __shared__ unsigned long long s_tot[kDCount], s_path, s_cut, s_failed;
  __shared__ uint32_t s_violate;
  if (tid < kDCount) {
    unsigned long long t = 0;
    for (int w = 0; w < kDecBlock / 64; w++) t += red[w][tid];
    s_tot[tid] = t;
  }
  __syncthreads();
  const unsigned long long c = s_tot[kDCreated], ov = s_tot[kDOverflow];
  const unsigned long long free_keys = live0 < st.max_keys ? st.max_keys - live0 : 0;
  // StoreFull unreachable iff live + created <= max_keys (size never exceeds it): the
  // keyed commit (0). Reachable: if no DELETE meets a live key, the live count only
  // grows through the batch, so a create succeeds iff fewer than max_keys - live
  // creates precede it in command order: the keyed commit with the creates ranked
  // (3, the cut below). With live-key DELETEs the live count is a clamped walk over the
  // batch's events (the scan below): still the keyed commit (3, refused creates by
  // bitmap) when every refused create is its key's last SET / DELETE, else the ordered
  // replay (1).
  unsigned long long path = 0;
  const bool dels = s_tot[kDLiveDel] != 0;
  if (ov || live0 + c > st.max_keys) path = (!ov && cbits && live0 <= st.max_keys) ? 3 : 1;
  if (path == 3 && dels) {
    // live count L over the batch: a create sets L = min(max_keys, L + 1) (refused when
    // L = max_keys), a live-key DELETE L - 1. Maps x -> min(C, x + D) compose, so each
    // thread folds its range of words into (C, D), a workgroup scan gives each range its
    // starting L, and each thread replays its range: the refused creates' bits, their
    // reserved heap bytes, and whether one of them is not its key's last mutation
    const long long M = (long long)st.max_keys, kInf = 1ll << 62;
    const uint64_t pl = kv_plane(n_cmds), W = pl, per_w = (W + kDecBlock - 1) / kDecBlock;
    const uint64_t w0 = (uint64_t)tid * per_w, w1 = w0 + per_w < W ? w0 + per_w : W;
    const uint32_t* evc = cbits + kEvCreate * pl;
    const uint32_t* evd = cbits + kEvDelete * pl;
    const uint32_t* evt = cbits + kEvTail * pl;
    uint32_t* evr = cbits + kEvRefused * pl;
    long long C = kInf, D = 0;
    for (uint64_t w = w0; w < w1; w++) {
      const uint32_t cw = evc[w], dw = evd[w];
      if (!dw) {
        const long long k = __builtin_popcount(cw);
        C = C + k < M ? C + k : M;
        D += k;
      } else if (!cw) {
        const long long k = __builtin_popcount(dw);
        C -= k;
        D -= k;
      } else {
        for (uint32_t x = cw | dw; x; x &= x - 1) {
          if (cw & x & (~x + 1u)) { C = C + 1 < M ? C + 1 : M; D++; }
          else { C--; D--; }
        }
      }
    }
    __shared__ long long s_sc[kDecBlock], s_sd[kDecBlock];
    s_sc[tid] = C;
    s_sd[tid] = D;
    if (tid == 0) s_violate = 0;
    __syncthreads();
    for (int o = 1; o < kDecBlock; o <<= 1) {  // inclusive scan: ranges 0..tid composed in order
      long long pc = 0, pd = 0;
      const bool has = tid >= o;
      if (has) { pc = s_sc[tid - o]; pd = s_sd[tid - o]; }
      __syncthreads();
      if (has) {
        const long long cc = s_sc[tid], dd = s_sd[tid];
        s_sc[tid] = cc < pc + dd ? cc : pc + dd;
        s_sd[tid] = pd + dd;
      }
      __syncthreads();
    }
    long long L = (long long)live0;
    if (tid > 0) {
      const long long ec = s_sc[tid - 1], ed = s_sd[tid - 1];
      L = ec < L + ed ? ec : L + ed;
    }
    unsigned long long fb = 0;
    uint32_t bad = 0;
    for (uint64_t w = w0; w < w1; w++) {
      const uint32_t cw = evc[w], dw = evd[w];
      uint32_t rw = 0;
      if (!dw && L + __builtin_popcount(cw) <= M) {
        L += __builtin_popcount(cw);
      } else if (!dw && L >= M) {
        rw = cw;
      } else if (!cw) {
        L -= __builtin_popcount(dw);
      } else {
        for (uint32_t x = cw | dw; x; x &= x - 1) {
          const uint32_t bit = x & (~x + 1u);
          if (cw & bit) {
            if (L >= M) rw |= bit;
            else L++;
          } else {
            L--;
          }
        }
      }
      evr[w] = rw;
      bad |= rw & ~evt[w];
      for (uint32_t x = rw; x; x &= x - 1) fb += cbytes[w * 32 + (uint64_t)__builtin_ctz(x)];
    }
    if (bad) s_violate = 1;  // (benign race: every writer stores 1)
    for (int o = 32; o > 0; o >>= 1) fb += __shfl_xor(fb, o, 64);
    if (lane == 0) red[wave][0] = fb;
    __syncthreads();
    if (tid == 0) s_failed = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    if (s_violate) path = 1;  // a refused key is mutated again: its later SETs depend on the order
    if (tid == 0) s_cut = kCutBits;
    __syncthreads();
  } else if (path == 3) {
    // the cut = command index of the create of rank max_keys - live (0-based) in
    // command order, from the plan's create bitmap: each thread popcounts a contiguous
    // range of words, a workgroup scan finds the range that holds it
    const uint64_t W = (n_cmds + 31) / 32, per_w = (W + kDecBlock - 1) / kDecBlock;
    const uint64_t w0 = (uint64_t)tid * per_w, w1 = w0 + per_w < W ? w0 + per_w : W;
    unsigned long long cnt = 0;
    for (uint64_t w = w0; w < w1; w++) cnt += __builtin_popcount(cbits[w]);
    s_scan[tid] = cnt;
    if (tid == 0) s_cut = n_cmds;  // (every create fits: not reached, c > free)
    __syncthreads();
    for (int o = 1; o < kDecBlock; o <<= 1) {
      const unsigned long long t = tid >= o ? s_scan[tid - o] : 0ull;
      __syncthreads();
      s_scan[tid] += t;
      __syncthreads();
    }
    const unsigned long long incl = s_scan[tid], excl = incl - cnt;
    if (excl <= free_keys && free_keys < incl) {
      unsigned long long r = free_keys - excl;
      for (uint64_t w = w0; w < w1; w++) {
        uint32_t x = cbits[w];
        const unsigned long long pc = __builtin_popcount(x);
        if (r < pc) {
          for (; r; r--) x &= x - 1;  // drop the r lowest creates of the word
          s_cut = w * 32 + (uint64_t)__builtin_ctz(x);
          break;
        }
        r -= pc;
      }
    }
    __syncthreads();
    // heap bytes the refused keys reserved in the plan (cbytes at their creates)
    unsigned long long fb = 0;
    for (uint64_t q = s_cut + (uint64_t)tid; q < n_cmds; q += kDecBlock) fb += cbytes[q];
    for (int o = 32; o > 0; o >>= 1) fb += __shfl_xor(fb, o, 64);
    if (lane == 0) red[wave][0] = fb;
    __syncthreads();
    if (tid == 0) s_failed = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    __syncthreads();
  }
  if (tid != 0) return;
  const unsigned long long ns = s_tot[kDNewSlots], sets = s_tot[kDSets], set_bytes = s_tot[kDSetBytes];
  // mode 3: the accepted creates take at most max_keys - live new slots, and the heap
  // bytes without the refused keys' reservations
  // (with live-key DELETEs each frees at most one key for a later create)
  const unsigned long long room3 = dels ? free_keys + s_tot[kDLiveDel] : free_keys;
  const unsigned long long slots = path == 3 && ns > room3 ? room3 : ns;
  // the ordered replay creates at most max_keys - live keys plus one per DELETE (each
  // frees at most one), so it needs at most that many new slots
  const unsigned long long room = free_keys + s_tot[kDDels];
  const unsigned long long slots1 = room < sets ? room : sets;
  const unsigned long long bytes = s_tot[kDNeed] - (path == 3 ? s_failed : 0ull);
  *arrivals = 0;  // for the next batch (stream order)
  // an earlier commit pass faulted and left a batch partially written: the store is
  // lost, and every later batch is refused (the fault bit stays set)
  // capacities: at most 7/8 of the table occupied; heap bytes available. The ordered
  // replay is checked against its worst case (every pending SET a new key and a new
  // value allocation), so a batch either fits whole or is refused before any write.
  const uint64_t cap = st.mask + 1, slot_cap = cap - cap / 8;
  unsigned long long mode = path;
  if (path != 1 && (occ0 + slots > slot_cap || top0 + bytes > st.heap_cap)) mode = 2;
  if (path == 1 && (occ0 + slots1 > slot_cap || top0 + set_bytes > st.heap_cap)) mode = 2;
  const bool lost = (flags0 & kFaultPartial) != 0;
  if (lost) mode = 2;
  k->mode = mode;
  k->batches = batches0 + 1;
  if (mode == 0 || mode == 3) {  // (mode 3: the commit subtracts what refused keys added)
    k->occupied = occ0 + ns;
    k->batch_base = top0;  // mode 0: commit writes [batch_base + group_base + block_base + ..., ...)
    if (mode == 0) k->heap_top = top0 + bytes;  // (mode 3: the commit's workgroups bump heap_top)
    k->live = live0 + s_tot[kDLive];  // two's-complement sum of +-1 deltas
    k->version = ver0 + s_tot[kDVersion];
    k->total_ops = ops0 + s_tot[kDOps];
    k->cut = mode == 3 ? s_cut : ~0ull;
  } else if (mode == 2 && !lost) {
    const bool table = occ0 + (path == 1 ? slots1 : slots) > slot_cap;
    k->flags = flags0 | (table ? kFaultTable : kFaultHeap);
  }
}

// Refused batch (mode 2): every command still pending gets RG_KV_E_CAPACITY.

// ---- 6 ordered replay (StoreFull reachable) -------------------------------------
__device__ void kv_ordered(const uint8_t* data, const KvOp* ops, uint64_t n, uint8_t* results, StoreView st) {
  KvCounters* k = st.ctr;
  unsigned long long live = k->live, ver = k->version, tops = k->total_ops, occ = k->occupied, top = k->heap_top;
  for (uint64_t c = 0; c < n; c++) {
    const KvOp op = ops[c];
    if (op.status != kPending) continue;
    const uint8_t* kp = data + op.key_off;
    const uint64_t h = op.hash;
    KvEntry e{};
    int64_t s = table_find(st.hashes, st.ent, st.heap, st.mask, h, kp, op.key_len, &e);
    const bool is_live = s >= 0 && e.version > 0;
    uint8_t r;
    if (op.kind == 0) {
      if (!is_live && live >= st.max_keys) {     // store.rs:153-158
        results[c] = RG_KV_E_FULL;
        continue;
      }
      // capacity for the worst case was checked before the batch (kv_decide_kernel)
      bool fits = false;
      if (s < 0) {
        s = table_claim(st.hashes, st.mask, h);
        occ++;
        bytes_copy(st.heap + top, kp, op.key_len);
        st.ent[s].key_off = top;
        st.ent[s].key_len = op.key_len;
        st.ent[s].val_len = 0;
        st.ent[s].version = 0;
        top += op.key_len;
      } else {
        fits = val_class(op.val_len) <= val_class(e.val_len);
      }
      uint64_t voff = e.val_off;
      if (!fits) {
        voff = top;
        st.ent[s].val_off = top;
        top += val_class(op.val_len);
      }
      bytes_copy(st.heap + voff, data + kv_val_off(op), op.val_len);
      st.ent[s].val_len = op.val_len;
      st.ent[s].version = is_live ? e.version + 1 : 1;
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

// ---- 2 sort: stable (bucket, command index) over the applied commands only --------
// Two levels, every pass a stable counting sort by an 8-bit digit (so equal buckets
// keep the total order of their commands):
//   L1  over the whole batch, grid-wide: the top 8 bits of the bucket. Each block
//       ranks a 4096-command chunk (kv_l1_hist_kernel counts, kv_l1_scan_kernel turns
//       the [chunk][digit] counts into global offsets, digit-major, kv_l1_scatter_kernel
//       writes); commands that are not applied are dropped, so only the applied ones
//       (about half of a C4 batch) are sorted, and their count lands on the device.
//   L2  one workgroup per top-digit bin (kv_l2_sort_kernel): LSD over the remaining
//       bucket bits (<= 23: up to 3 digit passes), in LDS when the bin fits one chunk,
//       else streamed through global memory chunk by chunk (a hot key's bin). It also
//       fills the sorted tail [n_applied, n) with the invalid bucket.
// Chunk ranking (rank_chunk): a wave owns 64 x PER consecutive commands; per round
// the lanes with equal digits find each other with 8 ballots, the lowest one adds the
// round's count to the wave's digit counter in LDS, and per-wave counters become
// per-wave offsets (waves in order): the chunk's commands sorted by digit, stably.
constexpr int kRadix = 256;

template <int BLOCK>
struct RankLds {
  static constexpr int kWaves = BLOCK / 64;
  uint32_t wcnt[kWaves][kRadix];  // per-wave digit counts -> exclusive offsets over the waves
  uint32_t dstart[kRadix + 1];    // chunk-local exclusive scan of the digit totals
  uint32_t scan[kWaves];
};

// Exclusive scan of one value per thread of the first kRadix threads (BLOCK >= kRadix);
// every thread of the block must call it.
template <int BLOCK>
__device__ __forceinline__ uint32_t radix_excl_scan(RankLds<BLOCK>& s, uint32_t v, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63 && wave < kRadix / 64) s.scan[wave] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kRadix / 64; w++) {
    const uint32_t x = s.scan[w];
    before += w < wave ? x : 0u;
    all += x;
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

// Stable rank of the chunk's commands by digit (key >> shift) & 255; valid[r] marks the
// commands of round r that take part. Returns each one's chunk-local sorted position;
// s.dstart holds the digit starts, s.dstart[256] the number of valid commands.
template <int BLOCK, int PER>
__device__ __forceinline__ void rank_chunk(RankLds<BLOCK>& s, const uint32_t (&key)[PER], uint32_t valid,
                                           uint32_t shift, uint32_t (&pos)[PER]) {
  constexpr int kWaves = BLOCK / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += BLOCK) (&s.wcnt[0][0])[i] = 0u;
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const bool v = (valid >> r) & 1u;
    const uint32_t d = (key[r] >> shift) & 255u;
    unsigned long long peers = __ballot(v);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t below = (uint32_t)__builtin_popcountll(peers & lt);
    // one wave's LDS accesses complete in issue order: this round's reads return the
    // counters before the leaders' writes below, the next round's reads after them
    const uint32_t base = v ? s.wcnt[wave][d] : 0u;
    pos[r] = base + below;
    if (v && below == 0) s.wcnt[wave][d] = base + (uint32_t)__builtin_popcountll(peers);
  }
  __syncthreads();
  uint32_t tot = 0;
  if (threadIdx.x < kRadix) {
    const int d = threadIdx.x;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
      const uint32_t c = s.wcnt[w][d];
      s.wcnt[w][d] = tot;
      tot += c;
    }
  }
  uint32_t all;
  const uint32_t ex = radix_excl_scan(s, threadIdx.x < kRadix ? tot : 0u, &all);
  if (threadIdx.x < kRadix) s.dstart[threadIdx.x] = ex;
  if (threadIdx.x == 0) s.dstart[kRadix] = all;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < PER; r++) {
    if (!((valid >> r) & 1u)) continue;
    const uint32_t d = (key[r] >> shift) & 255u;
    pos[r] += s.dstart[d] + s.wcnt[wave][d];
  }
}

// chunk position of thread's round-r command: a wave owns 64 x PER consecutive ones
template <int BLOCK, int PER>
__device__ __forceinline__ uint32_t chunk_pos(int r) {
  return (uint32_t)(threadIdx.x >> 6) * (64u * PER) + (uint32_t)r * 64u + (threadIdx.x & 63);
}

constexpr int kL1Block = 256, kL1Per = 16, kL1Chunk = kL1Block * kL1Per;   // 4096 commands per L1 chunk
constexpr int kL2Block = 1024, kL2Per = 16, kL2Chunk = kL2Block * kL2Per;  // 16384 per L2 chunk (in LDS)

struct SortArgs {
  const uint32_t* key_in;   // decode's buckets, all n commands (invalid_bucket: not applied)
  uint64_t n;
  uint32_t invalid_bucket;
  uint32_t shift1;          // L1 digit = key >> shift1 (the top <= 8 bucket bits)
  uint32_t passes2;         // L2 digit passes over bits [0, shift1)
  uint32_t chunks;          // L1 chunks
  uint32_t* hist;           // [chunks][256] L1 counts, then each digit's count in the chunks before
  uint32_t* bin_tot;        // [256] L1 bin sizes (applied commands per top digit)
  uint32_t *a_key, *a_idx;  // L2 ping-pong buffers
  uint32_t *b_key, *b_idx;  // (L1 writes b; pass p reads b/a and writes a/b; the last writes the final pair)
};

__global__ __launch_bounds__(kL1Block) void kv_l1_hist_kernel(SortArgs a) {
  __shared__ uint32_t h[kRadix];
  for (int d = threadIdx.x; d < kRadix; d += kL1Block) h[d] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kL1Chunk;
#pragma unroll
  for (int r = 0; r < kL1Per; r++) {
    const uint64_t i = base + chunk_pos<kL1Block, kL1Per>(r);
    if (i < a.n) {
      const uint32_t k = a.key_in[i];
      if (k != a.invalid_bucket) atomicAdd(&h[(k >> a.shift1) & 255u], 1u);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRadix; d += kL1Block) a.hist[(uint64_t)blockIdx.x * kRadix + d] = h[d];
}

// One workgroup per digit: column d of [chunks][256] -> its exclusive prefix over the
// chunks (in place) and the digit's total.
constexpr int kColBlock = 256;
__global__ __launch_bounds__(kColBlock) void kv_l1_colscan_kernel(SortArgs a) {
  __shared__ uint32_t w_sum[kColBlock / 64];
  const uint32_t d = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < a.chunks; c0 += kColBlock) {
    const uint32_t c = c0 + threadIdx.x;
    const uint32_t v = c < a.chunks ? a.hist[(uint64_t)c * kRadix + d] : 0u;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) w_sum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kColBlock / 64; w++) {
      before += w < wave ? w_sum[w] : 0u;
      all += w_sum[w];
    }
    __syncthreads();
    if (c < a.chunks) a.hist[(uint64_t)c * kRadix + d] = carry + before + incl - v;
    carry += all;
  }
  if (threadIdx.x == 0) a.bin_tot[d] = carry;
}

// The L1 bin starts: exclusive scan of the 256 bin totals into s_lo[0..256]
// (every thread of the block calls it; BLOCK >= 256).
template <int BLOCK>
__device__ __forceinline__ void bin_starts(RankLds<BLOCK>& s, const SortArgs& a, uint32_t* s_lo) {
  uint32_t all;
  const uint32_t t = threadIdx.x < kRadix ? a.bin_tot[threadIdx.x] : 0u;
  const uint32_t ex = radix_excl_scan(s, t, &all);
  if (threadIdx.x < kRadix) s_lo[threadIdx.x] = ex;
  if (threadIdx.x == 0) s_lo[kRadix] = all;
  __syncthreads();
}

struct L1Lds {
  RankLds<kL1Block> r;
  uint32_t key[kL1Chunk];  // the chunk, sorted by digit
  uint32_t idx[kL1Chunk];
};

__global__ __launch_bounds__(kL1Block) void kv_l1_scatter_kernel(SortArgs a) {
  __shared__ L1Lds s;
  __shared__ uint32_t goff[kRadix + 1];
  const uint64_t base = (uint64_t)blockIdx.x * kL1Chunk;
  bin_starts(s.r, a, goff);
  for (int d = threadIdx.x; d < kRadix; d += kL1Block) goff[d] += a.hist[(uint64_t)blockIdx.x * kRadix + d];
  uint32_t key[kL1Per], pos[kL1Per], valid = 0;
#pragma unroll
  for (int r = 0; r < kL1Per; r++) {
    const uint64_t i = base + chunk_pos<kL1Block, kL1Per>(r);
    key[r] = i < a.n ? a.key_in[i] : a.invalid_bucket;
    valid |= (key[r] != a.invalid_bucket ? 1u : 0u) << r;
  }
  rank_chunk(s.r, key, valid, a.shift1, pos);
#pragma unroll
  for (int r = 0; r < kL1Per; r++) {
    if (!((valid >> r) & 1u)) continue;
    s.key[pos[r]] = key[r];
    s.idx[pos[r]] = (uint32_t)(base + chunk_pos<kL1Block, kL1Per>(r));
  }
  __syncthreads();
  const uint32_t nv = s.r.dstart[kRadix];
  for (uint32_t p = threadIdx.x; p < nv; p += kL1Block) {  // runs of one digit go to consecutive addresses
    const uint32_t k = s.key[p], d = (k >> a.shift1) & 255u;
    const uint32_t dst = goff[d] + (p - s.r.dstart[d]);
    a.b_key[dst] = k;
    a.b_idx[dst] = s.idx[p];
  }
}

// L2: one workgroup per L1 bin [lo, hi); pass p sorts by bits [8p, 8p + 8) of the
// bucket (below shift1). A bin that fits one chunk (the common case) is sorted in LDS:
// its keys are loaded once and the passes permute a 16-bit index array (two buffers),
// so neither the keys nor the command indices move until the final gather (a command
// index is read from global memory, L2-resident, once). A larger bin (a hot key's) is
// streamed: pass p reads (p even ? b : a) and writes (p even ? a : b), chunk by chunk.
// Final pair: a when the pass count is odd, else b.
struct L2Lds {
  RankLds<kL2Block> r;
  uint32_t key[kL2Chunk];
  uint16_t perm[2][kL2Chunk];  // sorted position -> bin-local command
};

__global__ __launch_bounds__(kL2Block) void kv_l2_sort_kernel(SortArgs a) {
  __shared__ L2Lds s;
  __shared__ uint32_t s_hist[kRadix], s_run[kRadix], s_lo[kRadix + 1];
  bin_starts(s.r, a, s_lo);
  const uint32_t lo = s_lo[blockIdx.x], hi = s_lo[blockIdx.x + 1];
  const uint32_t n_app = s_lo[kRadix];
  // the sorted tail: commands that are not applied (the plan's walks stop there)
  uint32_t* const fin_key = (a.passes2 & 1u) ? a.a_key : a.b_key;
  uint32_t* const fin_idx = (a.passes2 & 1u) ? a.a_idx : a.b_idx;
  // (the tail's command index is a sentinel, never a stale index of an earlier batch: readers
  // stop at the invalid bucket, and one that did not would index out of range loudly)
  for (uint64_t i = n_app + (uint64_t)blockIdx.x * kL2Block + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * kL2Block) {
    fin_key[i] = a.invalid_bucket;
    fin_idx[i] = 0xFFFFFFFFu;
  }
  const uint32_t cnt = hi - lo;
  if (a.passes2 == 0 || cnt <= 1) {
    if (cnt == 1 && (a.passes2 & 1u) && threadIdx.x == 0) {  // a single command: just move it
      a.a_key[lo] = a.b_key[lo];
      a.a_idx[lo] = a.b_idx[lo];
    }
    return;
  }
  uint32_t key[kL2Per], pos[kL2Per];
  if (cnt <= (uint32_t)kL2Chunk) {
    for (uint32_t q = threadIdx.x; q < cnt; q += kL2Block) {
      s.key[q] = a.b_key[lo + q];
      s.perm[0][q] = (uint16_t)q;
    }
    __syncthreads();
    uint32_t valid = 0;
#pragma unroll
    for (int r = 0; r < kL2Per; r++) valid |= (chunk_pos<kL2Block, kL2Per>(r) < cnt ? 1u : 0u) << r;
    uint32_t cur = 0;
    for (uint32_t p = 0; p < a.passes2; p++, cur ^= 1u) {
      uint32_t j[kL2Per];
#pragma unroll
      for (int r = 0; r < kL2Per; r++) {
        const uint32_t q = chunk_pos<kL2Block, kL2Per>(r);
        j[r] = q < cnt ? s.perm[cur][q] : 0u;
        key[r] = s.key[j[r]];
      }
      rank_chunk(s.r, key, valid, 8 * p, pos);
#pragma unroll
      for (int r = 0; r < kL2Per; r++)
        if ((valid >> r) & 1u) s.perm[cur ^ 1u][pos[r]] = (uint16_t)j[r];
      __syncthreads();
    }
    // gather every command index first: the final pair may be b itself (an even pass
    // count), so no write may land before every read
    uint32_t jj[kL2Per], ci[kL2Per];
#pragma unroll
    for (int r = 0; r < kL2Per; r++) {
      const uint32_t q = (uint32_t)r * kL2Block + threadIdx.x;
      jj[r] = q < cnt ? s.perm[cur][q] : 0u;
      ci[r] = q < cnt ? a.b_idx[lo + jj[r]] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kL2Per; r++) {
      const uint32_t q = (uint32_t)r * kL2Block + threadIdx.x;
      if (q < cnt) {
        fin_key[lo + q] = s.key[jj[r]];
        fin_idx[lo + q] = ci[r];
      }
    }
    return;
  }
  // streamed (a bin larger than one chunk: a hot key's): per pass a digit histogram
  // over the bin, then the chunks in order
  for (uint32_t p = 0; p < a.passes2; p++) {
    const uint32_t* sk = (p & 1u) ? a.a_key : a.b_key;
    const uint32_t* si = (p & 1u) ? a.a_idx : a.b_idx;
    uint32_t* dk = (p & 1u) ? a.b_key : a.a_key;
    uint32_t* di = (p & 1u) ? a.b_idx : a.a_idx;
    const uint32_t shift = 8 * p;
    for (int d = threadIdx.x; d < kRadix; d += kL2Block) s_hist[d] = 0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kL2Block) atomicAdd(&s_hist[(sk[i] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t all;
    const uint32_t ex = radix_excl_scan(s.r, threadIdx.x < kRadix ? s_hist[threadIdx.x] : 0u, &all);
    if (threadIdx.x < kRadix) s_run[threadIdx.x] = lo + ex;
    __syncthreads();
    for (uint32_t c = lo; c < hi; c += kL2Chunk) {
      uint32_t valid = 0;
#pragma unroll
      for (int r = 0; r < kL2Per; r++) {
        const uint32_t i = c + chunk_pos<kL2Block, kL2Per>(r);
        valid |= (i < hi ? 1u : 0u) << r;
        key[r] = i < hi ? sk[i] : 0u;
      }
      rank_chunk(s.r, key, valid, shift, pos);
#pragma unroll
      for (int r = 0; r < kL2Per; r++) {  // chunk-local sorted position -> chunk offset
        if (!((valid >> r) & 1u)) continue;
        s.key[pos[r]] = key[r];
        s.perm[0][pos[r]] = (uint16_t)chunk_pos<kL2Block, kL2Per>(r);
      }
      __syncthreads();
      const uint32_t nv = s.r.dstart[kRadix];
      for (uint32_t q = threadIdx.x; q < nv; q += kL2Block) {
        const uint32_t k = s.key[q], d = (k >> shift) & 255u;
        const uint32_t dst = s_run[d] + (q - s.r.dstart[d]);
        dk[dst] = k;
        di[dst] = si[c + s.perm[0][q]];
      }
      __syncthreads();
      if (threadIdx.x < kRadix) s_run[threadIdx.x] += s.r.dstart[threadIdx.x + 1] - s.r.dstart[threadIdx.x];
      __syncthreads();
    }
  }
}

// ---- exclusive scan of u64 (the synthetic trace's command offsets) ----------------
constexpr int kScanBlock = 1024, kScanPer = 4, kScanChunk = kScanBlock * kScanPer;
__device__ __forceinline__ unsigned long long block_excl_scan64(unsigned long long v, unsigned long long* total) {
  __shared__ unsigned long long w_sum[kScanBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) w_sum[wave] = incl;
  __syncthreads();
  unsigned long long before = 0, all = 0;
  for (int w = 0; w < kScanBlock / 64; w++) {
    before += w < wave ? w_sum[w] : 0ull;
    all += w_sum[w];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}
__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(const uint64_t* in, uint64_t n, uint64_t* sums) {
  const uint64_t b = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanPer;
  unsigned long long v = 0;
  for (int k = 0; k < kScanPer; k++) v += b + k < n ? in[b + k] : 0ull;
  unsigned long long all;
  (void)block_excl_scan64(v, &all);
  if (threadIdx.x == 0) sums[blockIdx.x] = all;
}
// one block: the chunk sums scanned in place (sequential over pieces of kScanBlock)
__global__ __launch_bounds__(kScanBlock) void scan_top_kernel(uint64_t* sums, uint64_t chunks) {
  unsigned long long carry = 0;
  for (uint64_t c0 = 0; c0 < chunks; c0 += kScanBlock) {
    const uint64_t c = c0 + threadIdx.x;
    const unsigned long long v = c < chunks ? sums[c] : 0ull;
    unsigned long long all;
    const unsigned long long ex = block_excl_scan64(v, &all);
    if (c < chunks) sums[c] = carry + ex;
    carry += all;
  }
}
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint64_t* in, uint64_t n, const uint64_t* sums,
                                                               uint64_t* out) {
  const uint64_t b = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanPer;
  unsigned long long x[kScanPer], v = 0;
  for (int k = 0; k < kScanPer; k++) {
    x[k] = b + k < n ? in[b + k] : 0ull;
    v += x[k];
  }
  unsigned long long all;
  unsigned long long run = sums[blockIdx.x] + block_excl_scan64(v, &all);
  for (int k = 0; k < kScanPer; k++) {
    if (b + k < n) out[b + k] = run;
    run += x[k];
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
  uint64_t *need = nullptr, *block_base = nullptr, *group_base = nullptr;
  unsigned long long* dpart = nullptr;     // [decide groups][kDCount] decide rows
  unsigned long long* arrivals = nullptr;  // decide workgroups arrived (0 between batches)
  uint32_t *key_a = nullptr, *key_b = nullptr, *idx_a = nullptr, *idx_b = nullptr;
  uint32_t* sort_hist = nullptr;           // [L1 chunks][256] digit counts -> offsets
  uint32_t* bin_lo = nullptr;              // [256] L1 bin sizes
  uint64_t* scan_sums = nullptr;           // trace generator's offset scan: per-chunk sums
  KeyRec* recs = nullptr;
  uint8_t* done = nullptr;
  unsigned long long* part = nullptr;
  unsigned long long* set_part = nullptr;  // [blocks][2] decode partials: pending SETs, worst-case bytes
  uint32_t* cbits = nullptr;               // [kEvPlanes][cap / 32 + 1] event bitmaps (mode 3)
  unsigned long long* cbytes = nullptr;    // [cap] heap bytes reserved at each create (mode 3)
  // host-side upper bound of the live keys after every enqueued batch (exact after a
  // synchronising call): a batch marks its creates only when it could meet StoreFull
  uint64_t live_ub = 0;
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
  (void)hipFree(kv->ops); (void)hipFree(kv->key_a); (void)hipFree(kv->key_b);
  (void)hipFree(kv->need); (void)hipFree(kv->block_base); (void)hipFree(kv->idx_a);
  (void)hipFree(kv->idx_b); (void)hipFree(kv->done); (void)hipFree(kv->part);
  (void)hipFree(kv->set_part); (void)hipFree(kv->recs); (void)hipFree(kv->cbits); (void)hipFree(kv->cbytes);
  kv->cbits = nullptr; kv->cbytes = nullptr;
  (void)hipFree(kv->group_base); (void)hipFree(kv->dpart); (void)hipFree(kv->arrivals);
  kv->group_base = nullptr; kv->dpart = nullptr; kv->arrivals = nullptr;
  (void)hipFree(kv->sort_hist); (void)hipFree(kv->bin_lo); (void)hipFree(kv->scan_sums);
  kv->set_part = nullptr; kv->recs = nullptr;
  kv->sort_hist = kv->bin_lo = nullptr; kv->scan_sums = nullptr;
  kv->ops = nullptr; kv->need = kv->block_base = nullptr;
  kv->key_a = kv->key_b = kv->idx_a = kv->idx_b = nullptr; kv->done = nullptr; kv->part = nullptr;
  kv->cap_cmds = 0;
}

int ensure_scratch(rg_kv* kv, uint64_t n) {
  if (n <= kv->cap_cmds) return 0;
  KV_HIP(kv, hipDeviceSynchronize());  // scratch may be in use on a caller stream
  free_scratch(kv);
  uint64_t cap = 1024;
  while (cap < n) cap *= 2;
  const uint64_t blocks = (cap + kBlock - 1) / kBlock;
  KV_HIP(kv, hipMalloc(&kv->ops, cap * sizeof(KvOp)));
  KV_HIP(kv, hipMalloc(&kv->key_a, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->key_b, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->recs, cap * sizeof(KeyRec)));
  KV_HIP(kv, hipMalloc(&kv->need, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->block_base, (cap / kWalkBlockSpan + 1) * 8));
  const uint64_t groups = cap / kWalkBlockSpan / kDecGroup + 2;
  KV_HIP(kv, hipMalloc(&kv->group_base, groups * 8));
  KV_HIP(kv, hipMalloc(&kv->dpart, groups * kDCount * 8));
  KV_HIP(kv, hipMalloc(&kv->arrivals, 8));
  KV_HIP(kv, hipMemset(kv->arrivals, 0, 8));
  KV_HIP(kv, hipMalloc(&kv->idx_a, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->idx_b, cap * 4));
  KV_HIP(kv, hipMalloc(&kv->done, cap));
  KV_HIP(kv, hipMalloc(&kv->part, blocks * kPCount * 8));
  KV_HIP(kv, hipMalloc(&kv->set_part, blocks * kSetPart * 8));
  KV_HIP(kv, hipMalloc(&kv->cbits, kEvPlanes * (cap / 32 + 1) * 4));
  KV_HIP(kv, hipMalloc(&kv->cbytes, cap * 8));
  KV_HIP(kv, hipMalloc(&kv->sort_hist, (cap / kL1Chunk + 1) * kRadix * 4));
  KV_HIP(kv, hipMalloc(&kv->bin_lo, (kRadix + 1) * 4));
  KV_HIP(kv, hipMalloc(&kv->scan_sums, (cap / kScanChunk + 2) * 8));
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
  // sort width: bucket bits enough that distinct keys rarely share a bucket (about
  // 2^8 buckets per command, so a run rarely needs the multi-key path), at most 31
  // (+1 bit for the invalid bucket, so the sort key is a u32)
  int vbits = 14;
  while (vbits < 31 && (1ull << (vbits - 8)) < n_cmds) vbits++;
  if (kv->cfg.bucket_bits && (int)kv->cfg.bucket_bits < vbits) vbits = (int)kv->cfg.bucket_bits;
  const uint32_t invalid_bucket = 1u << vbits;
  // StoreFull can fire only if live + keys created > max_keys; a batch creates at most
  // n_cmds keys, so below the bound the plan keeps no create bitmap (mode 3 unneeded)
  const bool may_fill = kv->live_ub + n_cmds > kv->cfg.max_keys;
  kv->live_ub = kv->live_ub + n_cmds < kv->live_ub ? ~0ull : kv->live_ub + n_cmds;
  uint32_t* cbits = may_fill ? kv->cbits : nullptr;
  unsigned long long* cbytes = may_fill ? kv->cbytes : nullptr;
  hipLaunchKernelGGL(kv_decode_kernel, dim3(blocks), dim3(kBlock), 0, s, data_dev, cmd_off_dev, n_cmds,
                     apply_mask_dev, kv->cfg.max_value_size,
                     kv->cfg.hash_bits && kv->cfg.hash_bits < 64 ? (1ull << kv->cfg.hash_bits) - 1 : ~0ull,
                     (uint64_t)invalid_bucket - 1, invalid_bucket, kv->ops, kv->key_a, results_dev, kv->set_part,
                     kv->done, cbits, cbytes);
  KV_HIP(kv, hipGetLastError());
  // stable (bucket, index) sort of the applied commands (two levels of 8-bit digits)
  SortArgs sa;
  sa.key_in = kv->key_a;
  sa.n = n_cmds;
  sa.invalid_bucket = invalid_bucket;
  sa.shift1 = (uint32_t)(vbits > 8 ? vbits - 8 : 0);
  sa.passes2 = (sa.shift1 + 7) / 8;
  sa.hist = kv->sort_hist;
  sa.bin_tot = kv->bin_lo;
  sa.a_key = kv->key_a;
  sa.a_idx = kv->idx_a;
  sa.b_key = kv->key_b;
  sa.b_idx = kv->idx_b;
  const uint32_t chunks = (uint32_t)((n_cmds + kL1Chunk - 1) / kL1Chunk);
  sa.chunks = chunks;
  hipLaunchKernelGGL(kv_l1_hist_kernel, dim3(chunks), dim3(kL1Block), 0, s, sa);
  hipLaunchKernelGGL(kv_l1_colscan_kernel, dim3(kRadix), dim3(kColBlock), 0, s, sa);
  hipLaunchKernelGGL(kv_l1_scatter_kernel, dim3(chunks), dim3(kL1Block), 0, s, sa);
  hipLaunchKernelGGL(kv_l2_sort_kernel, dim3(kRadix), dim3(kL2Block), 0, s, sa);
  KV_HIP(kv, hipGetLastError());
  const bool fin_a = (sa.passes2 & 1u) != 0;
  BatchView b{data_dev, kv->ops, fin_a ? kv->key_a : kv->key_b, fin_a ? kv->idx_a : kv->idx_b, n_cmds, results_dev,
              kv->done, kv->need, kv->block_base, kv->group_base, kv->recs, invalid_bucket, kv->part, cbits, cbytes};
  const StoreView st = view(kv);
  const uint32_t walk_blocks = (uint32_t)((n_cmds + kWalkBlockSpan - 1) / kWalkBlockSpan);
  hipLaunchKernelGGL(kv_plan_kernel, dim3(walk_blocks), dim3(kBlock), 0, s, b, st);
  KV_HIP(kv, hipGetLastError());
  const uint32_t groups = (walk_blocks + kDecGroup - 1) / kDecGroup;
  hipLaunchKernelGGL(kv_decide_kernel, dim3(groups), dim3(kDecBlock), 0, s, st, kv->part, walk_blocks, kv->set_part,
                     blocks, kv->block_base, kv->group_base, kv->dpart, kv->arrivals, cbits, cbytes, n_cmds);
  hipLaunchKernelGGL(kv_commit_kernel, dim3(walk_blocks), dim3(kBlock), 0, s, b, st);
  KV_HIP(kv, hipGetLastError());
  return 0;
}

int rg_kv_get_stats(rg_kv* kv, rg_kv_stats* out) {
  if (!kv || !out) return kfail(kv, -1, "rg_kv_get_stats: null argument");
  KvCounters c;
  KV_HIP(kv, hipDeviceSynchronize());  // applies may sit on caller streams
  KV_HIP(kv, hipMemcpy(&c, kv->ctr, sizeof(c), hipMemcpyDeviceToHost));
  kv->live_ub = c.live;  // exact: every apply has completed
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
  const uint64_t m = n_cmds + 1, sc = (m + kScanChunk - 1) / kScanChunk;  // exclusive scan of the sizes
  hipLaunchKernelGGL(scan_sums_kernel, dim3((uint32_t)sc), dim3(kScanBlock), 0, s, kv->need, m, kv->scan_sums);
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanBlock), 0, s, kv->scan_sums, sc);
  hipLaunchKernelGGL(scan_apply_kernel, dim3((uint32_t)sc), dim3(kScanBlock), 0, s, kv->need, m, kv->scan_sums,
                     cmd_off_dev);
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
