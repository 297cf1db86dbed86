// rg_ingest.hip — device-side vote ingestion (include/rabia_ingest.h).
//
// Three launches per batch of messages, no host round trip:
//   parse   one thread per message: bincode ProtocolMessage -> (round, sender lane,
//           slot, code) or a rejection category; valid in-window votes claim their
//           (round, lane, slot) cell with atomicMax(message index + 1), so the LAST
//           message of the batch wins (HashMap::insert, messages.rs:169-175)
//   count   one thread per message: winner or superseded
//   pack    one thread per (round, lane, plane word): folds the 32 cells of the
//           word into the lo/hi vote planes (coalesced), keeps the planes' previous
//           bits where the batch had no vote, and re-zeroes the cells it consumed
// The cell array (2 * n * n_slots u32) is all-zero between calls.
#include "rabia_ingest.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <string>

namespace {

constexpr int kBlock = 256;
constexpr uint64_t kNoKey = ~0ull;
constexpr uint64_t kSkewMs = 60000;  // ValidationConfig::default().max_clock_skew_ms

struct Members {
  uint8_t id[16][16];
  uint32_t n;
};

// Frames sit at arbitrary byte offsets: fields are read through 1-byte-aligned types
// (gfx950 global memory takes unaligned dword accesses).
typedef uint64_t u64_unaligned __attribute__((aligned(1)));
typedef uint32_t u32_unaligned __attribute__((aligned(1)));

struct Reader {
  const uint8_t* p;
  uint64_t len, pos;
  bool ok;
  __device__ bool need(uint64_t k) {
    if (!ok || pos > len || len - pos < k) ok = false;
    return ok;
  }
  __device__ uint64_t u64() {
    if (!need(8)) return 0;
    const uint64_t v = *(const u64_unaligned*)(p + pos);  // bincode fixint: little-endian
    pos += 8;
    return v;
  }
  __device__ uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = *(const u32_unaligned*)(p + pos);
    pos += 4;
    return v;
  }
  __device__ uint32_t u8() {
    if (!need(1)) return 0;
    return p[pos++];
  }
  // Uuid via serialize_bytes: u64 length (must be 16) + 16 bytes. Returns its offset.
  __device__ uint64_t uuid() {
    const uint64_t l = u64();
    if (ok && l != 16) ok = false;
    if (!need(16)) return 0;
    const uint64_t at = pos;
    pos += 16;
    return at;
  }
};

enum Cat { kR1 = 0, kR2, kSuperseded, kOther, kOutside, kInvalid, kSender, kMalformed, kCats };

__device__ int lane_of(const Members& m, const uint8_t* id) {
  for (uint32_t l = 0; l < m.n; l++) {
    bool eq = true;
    for (int b = 0; b < 16; b++) eq &= m.id[l][b] == id[b];
    if (eq) return (int)l;
  }
  return -1;
}

__device__ __forceinline__ void block_count(const uint32_t cat, unsigned long long* part) {
  __shared__ unsigned int cnt[kCats];
  if (threadIdx.x < kCats) cnt[threadIdx.x] = 0;
  __syncthreads();
  if (cat < kCats) atomicAdd(&cnt[cat], 1u);  // LDS atomics
  __syncthreads();
  if (threadIdx.x < kCats) part[(uint64_t)blockIdx.x * kCats + threadIdx.x] = cnt[threadIdx.x];
}

struct ParseArgs {
  const uint8_t* msgs;
  const uint64_t* off;
  const uint8_t* sender;
  uint64_t n_msgs, now_ms, n_slots, slot_base;
  uint32_t* cells;        // [2][n][n_slots]
  uint64_t* mkey;         // per message: cell index or kNoKey
  uint8_t* mcode;         // per message: vote code
  unsigned long long* part;
  Members mem;
};

__global__ __launch_bounds__(kBlock) void ingest_parse_kernel(ParseArgs a) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t cat = kCats;  // none (padding threads)
  if (m < a.n_msgs) {
    uint64_t key = kNoKey;
    const uint64_t b = a.off[m], e = a.off[m + 1];
    Reader r{a.msgs + b, e > b ? e - b : 0, 0, true};
    r.uuid();                              // id
    const uint64_t from_at = r.uuid();     // from
    const uint32_t tag = r.u8();           // to: Option<NodeId>
    if (r.ok && tag > 1) r.ok = false;
    if (tag == 1) r.uuid();
    const uint64_t ts = r.u64();
    const uint32_t variant = r.u32();
    if (r.ok && variant > 8) r.ok = false;  // MessageType has 9 variants
    if (!r.ok) {
      cat = kMalformed;
    } else if (variant != 1 && variant != 2) {
      cat = kOther;
    } else {
      const uint64_t phase = r.u64();
      r.uuid();                            // batch_id
      const uint32_t vote = r.u32();
      r.uuid();                            // voter_id (not used: votes are keyed by sender)
      if (r.ok && vote > 2) r.ok = false;
      uint64_t count = 0;
      if (variant == 2) {
        count = r.u64();
        if (r.ok && count > (r.len - r.pos) / 28) r.ok = false;  // 24 B NodeId + 4 B StateValue each
        for (uint64_t k = 0; r.ok && k < count; k++) {
          r.uuid();
          if (r.u32() > 2 && r.ok) r.ok = false;
        }
      }
      if (!r.ok) {
        cat = kMalformed;
      } else if (ts > a.now_ms + kSkewMs || (a.now_ms > ts && a.now_ms - ts > 10 * kSkewMs) ||
                 (variant == 2 && count == 0)) {
        cat = kInvalid;                    // validation.rs:40-52, 68-79
      } else {
        const int lane = lane_of(a.mem, r.p + from_at);
        if (lane < 0 || (a.sender && a.sender[m] != (uint8_t)lane)) {
          cat = kSender;                   // engine.rs:357-364
        } else if (phase < a.slot_base || phase - a.slot_base >= a.n_slots) {
          cat = kOutside;
        } else {
          const uint32_t round = variant - 1;
          key = ((uint64_t)round * a.mem.n + (uint64_t)lane) * a.n_slots + (phase - a.slot_base);
          atomicMax(a.cells + key, (uint32_t)(m + 1));
          a.mcode[m] = (uint8_t)vote;
          cat = round ? kR2 : kR1;         // winners / superseded sorted out by the count pass
        }
      }
    }
    a.mkey[m] = key;
  }
  block_count(cat, a.part);
}

__global__ __launch_bounds__(kBlock) void ingest_count_kernel(const uint64_t* mkey, const uint32_t* cells,
                                                             uint64_t n_msgs, uint64_t n_slots, uint32_t n,
                                                             unsigned long long* part) {
  const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t cat = kCats;
  if (m < n_msgs && mkey[m] != kNoKey) {
    const uint64_t key = mkey[m];
    const bool r2 = key >= (uint64_t)n * n_slots;
    cat = cells[key] == (uint32_t)(m + 1) ? (r2 ? kR2 : kR1) : kSuperseded;
  }
  block_count(cat, part);
}

// One thread per (round, lane, word). Plane address as in rg_kernels.h Layout.
__global__ __launch_bounds__(kBlock) void ingest_pack_kernel(uint32_t* cells, const uint8_t* mcode,
                                                            uint32_t* votes, uint64_t n_slots, uint32_t n,
                                                            uint64_t stride, uint32_t tile_words) {
  const uint64_t n_words = (n_slots + 31) / 32;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2ull * n * n_words) return;
  const uint64_t w = t % n_words, rl = t / n_words;  // rl = round * n + lane
  uint32_t* c = cells + rl * n_slots + 32 * w;
  const uint32_t cnt = (uint32_t)((n_slots - 32 * w) < 32 ? (n_slots - 32 * w) : 32);
  uint32_t set = 0, lo = 0, hi = 0;
  for (uint32_t b = 0; b < cnt; b++) {
    const uint32_t v = c[b];
    if (v) {
      const uint32_t code = mcode[v - 1];
      set |= 1u << b;
      lo |= (code & 1u) << b;
      hi |= (code >> 1) << b;
      c[b] = 0;
    }
  }
  if (!set) return;
  const uint32_t round = (uint32_t)(rl / n), lane = (uint32_t)(rl % n);
  const uint64_t p_lo = (uint64_t)round * 2 * n + 2 * lane;  // R1 planes [0, 2n), R2 [2n, 4n)
  const uint64_t P = 4ull * n + 1;
  uint64_t base;
  uint64_t ps;
  if (tile_words) {
    base = (w / tile_words) * (P * tile_words) + (w % tile_words);
    ps = tile_words;
  } else {
    base = w;
    ps = stride;
  }
  uint32_t* wl = votes + base + p_lo * ps;
  uint32_t* wh = wl + ps;
  *wl = (*wl & ~set) | lo;
  *wh = (*wh & ~set) | hi;
}

__global__ void ingest_fold_kernel(const unsigned long long* part, uint32_t blocks, uint64_t* stats,
                                   bool count_pass) {
  __shared__ unsigned long long red[kBlock][kCats];
  unsigned long long v[kCats] = {0};
  for (uint32_t k = threadIdx.x; k < blocks; k += blockDim.x)
    for (int c = 0; c < kCats; c++) v[c] += part[(uint64_t)k * kCats + c];
  for (int c = 0; c < kCats; c++) red[threadIdx.x][c] = v[c];
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int t = 1; t < (int)blockDim.x; t++)
    for (int c = 0; c < kCats; c++) v[c] += red[t][c];
  // parse pass: every category but the vote ones; count pass: winners / superseded
  for (int c = 0; c < kCats; c++) {
    const bool vote_cat = c == kR1 || c == kR2 || c == kSuperseded;
    if (vote_cat == count_pass) stats[c] += v[c];
  }
}

}  // namespace

struct rg_ingest {
  rg_ingest_config cfg{};
  Members mem{};
  hipStream_t stream = nullptr;
  uint32_t* cells = nullptr;
  uint64_t cells_cap = 0;  // entries
  uint64_t* mkey = nullptr;
  uint8_t* mcode = nullptr;
  unsigned long long* part = nullptr;
  uint64_t msg_cap = 0;
  std::string err;
};

namespace {
thread_local std::string g_ing_err;
int ifail(rg_ingest* g, int code, const std::string& m) {
  if (g) g->err = m;
  else g_ing_err = m;
  return code;
}
#define ING_HIP(g, call)                                                                  \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) return ifail(g, -2, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
}  // namespace

extern "C" {

int rg_ingest_create(rg_ingest** out, const rg_ingest_config* cfg) {
  if (!out || !cfg) return ifail(nullptr, -1, "rg_ingest_create: null argument");
  *out = nullptr;
  if (cfg->n_replicas < 1 || cfg->n_replicas > 16) return ifail(nullptr, -1, "rg_ingest_create: n_replicas must be 1..16");
  if (cfg->tile_words && (cfg->tile_words < 64 || (cfg->tile_words & (cfg->tile_words - 1))))
    return ifail(nullptr, -1, "rg_ingest_create: tile_words must be 0 or a power of two >= 64");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return ifail(nullptr, -4, "rg_ingest_create: no HIP device");
  if (cfg->device < 0 || cfg->device >= count) return ifail(nullptr, -4, "rg_ingest_create: bad device ordinal");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return ifail(nullptr, -4, "rg_ingest_create: device is not gfx950");
  rg_ingest* g = new (std::nothrow) rg_ingest();
  if (!g) return ifail(nullptr, -3, "rg_ingest_create: host allocation failed");
  g->cfg = *cfg;
  std::memcpy(g->mem.id, cfg->members, sizeof(g->mem.id));
  g->mem.n = cfg->n_replicas;
  if (hipSetDevice(cfg->device) != hipSuccess ||
      hipStreamCreateWithFlags(&g->stream, hipStreamDefault) != hipSuccess) {
    delete g;
    return ifail(nullptr, -2, "rg_ingest_create: stream creation failed");
  }
  *out = g;
  return 0;
}

int rg_ingest_destroy(rg_ingest* g) {
  if (!g) return 0;
  (void)hipDeviceSynchronize();
  (void)hipFree(g->cells); (void)hipFree(g->mkey); (void)hipFree(g->mcode); (void)hipFree(g->part);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  delete g;
  return 0;
}

const char* rg_ingest_last_error(const rg_ingest* g) { return g ? g->err.c_str() : g_ing_err.c_str(); }

int rg_ingest_votes_async(rg_ingest* g, const uint8_t* msgs_dev, const uint64_t* msg_off_dev,
                          const uint8_t* sender_lane_dev, uint64_t n_msgs, uint64_t now_ms, uint32_t* votes_dev,
                          uint64_t n_slots, uint64_t stride_words, uint64_t slot_base, uint64_t* stats_dev,
                          void* stream) {
  if (!g) return ifail(nullptr, -1, "rg_ingest_votes_async: null handle");
  if (!n_msgs || !n_slots) return 0;
  if (!msgs_dev || !msg_off_dev || !votes_dev || !stats_dev) return ifail(g, -1, "rg_ingest_votes_async: null buffer");
  if (n_msgs >= 0xFFFFFFFFull) return ifail(g, -1, "rg_ingest_votes_async: too many messages");
  if (!g->cfg.tile_words && (stride_words < (n_slots + 31) / 32 || stride_words % 4))
    return ifail(g, -1, "rg_ingest_votes_async: stride_words must be a multiple of 4 and >= ceil(n_slots/32)");
  if (g->cfg.tile_words && stride_words && stride_words != g->cfg.tile_words)
    return ifail(g, -1, "rg_ingest_votes_async: stride_words must be 0 or tile_words for the slot-tiled layout");
  const uint32_t n = g->cfg.n_replicas;
  const uint64_t cells = 2ull * n * n_slots;
  if (cells > g->cells_cap || n_msgs > g->msg_cap) ING_HIP(g, hipDeviceSynchronize());
  if (cells > g->cells_cap) {
    (void)hipFree(g->cells);
    g->cells = nullptr;
    g->cells_cap = 0;
    ING_HIP(g, hipMalloc(&g->cells, cells * 4));
    ING_HIP(g, hipMemset(g->cells, 0, cells * 4));
    // hipMemset runs on the null stream, which does not order against the
    // non-blocking launch stream: finish it before the parse kernel claims cells.
    ING_HIP(g, hipDeviceSynchronize());
    g->cells_cap = cells;
  }
  if (n_msgs > g->msg_cap) {
    uint64_t cap = 1024;
    while (cap < n_msgs) cap *= 2;
    (void)hipFree(g->mkey); (void)hipFree(g->mcode); (void)hipFree(g->part);
    g->mkey = nullptr; g->mcode = nullptr; g->part = nullptr; g->msg_cap = 0;
    ING_HIP(g, hipMalloc(&g->mkey, cap * 8));
    ING_HIP(g, hipMalloc(&g->mcode, cap));
    ING_HIP(g, hipMalloc(&g->part, ((cap + kBlock - 1) / kBlock) * kCats * 8));
    g->msg_cap = cap;
  }
  hipStream_t s = stream ? (hipStream_t)stream : g->stream;
  const uint32_t blocks = (uint32_t)((n_msgs + kBlock - 1) / kBlock);
  ParseArgs a{msgs_dev, msg_off_dev, sender_lane_dev, n_msgs, now_ms, n_slots, slot_base,
              g->cells, g->mkey, g->mcode, g->part, g->mem};
  hipLaunchKernelGGL(ingest_parse_kernel, dim3(blocks), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(ingest_fold_kernel, dim3(1), dim3(kBlock), 0, s, g->part, blocks, stats_dev, false);
  hipLaunchKernelGGL(ingest_count_kernel, dim3(blocks), dim3(kBlock), 0, s, g->mkey, g->cells, n_msgs, n_slots, n,
                     g->part);
  hipLaunchKernelGGL(ingest_fold_kernel, dim3(1), dim3(kBlock), 0, s, g->part, blocks, stats_dev, true);
  const uint64_t work = 2ull * n * ((n_slots + 31) / 32);
  hipLaunchKernelGGL(ingest_pack_kernel, dim3((uint32_t)((work + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     g->cells, g->mcode, votes_dev, n_slots, n, stride_words, g->cfg.tile_words);
  ING_HIP(g, hipGetLastError());
  return 0;
}

}  // extern "C"
