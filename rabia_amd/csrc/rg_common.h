// rg_common.h — shared host/device definitions of the MI355X Rabia phase evaluator.
//
// Everything here is integer arithmetic; the only "randomness" is counter-mode
// ChaCha (random access by block counter), so any slot's draw or coin can be
// computed by the thread that owns the slot.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RG_HD __host__ __device__ __forceinline__

namespace rg {

constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
constexpr int kWaves = kBlock / 64;
constexpr int kOutPlanes = 8;        // output planes per step (include/rabia_gpu.h)
constexpr int kMaxReplicas = 16;
constexpr uint32_t kCodeV0 = 0, kCodeV1 = 1, kCodeVQ = 2, kCodeNone = 3;

// rand 0.8.5 Bernoulli p_int = (p * 2^64) as u64 for the engine's probabilities
// (engine.rs:587/595 -> 0.9, engine.rs:604 -> 0.8).
constexpr uint64_t kP90 = 0xE666666666666800ull;
constexpr uint64_t kP80 = 0xCCCCCCCCCCCCD000ull;
constexpr uint64_t kCoinStreamBit = 0x8000000000000000ull;

RG_HD uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

// rand_core 0.6.4 SeedableRng::seed_from_u64 (PCG32 key fill); engine.rs:59-62.
inline void seed_from_u64(uint64_t state, uint32_t key[8]) {
  const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
  for (int i = 0; i < 8; i++) {
    state = state * MUL + INC;
    uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    key[i] = (xs >> rot) | (xs << ((32u - rot) & 31u));
  }
}

struct Key {
  uint32_t k[8];
};

#define RG_QR(a, b, c, d)                                          \
  x##a += x##b; x##d = rotl32(x##d ^ x##a, 16);                    \
  x##c += x##d; x##b = rotl32(x##b ^ x##c, 12);                    \
  x##a += x##b; x##d = rotl32(x##d ^ x##a, 8);                     \
  x##c += x##d; x##b = rotl32(x##b ^ x##c, 7);

// ChaCha block, 64-bit counter (words 12-13) + 64-bit stream (words 14-15):
// the rand_chacha 0.3.1 layout (ChaCha12Rng = StdRng, rounds = 12).
template <int ROUNDS>
RG_HD void chacha_block(const Key& key, uint64_t counter, uint64_t stream, uint32_t out[16]) {
  const uint32_t s0 = 0x61707865u, s1 = 0x3320646eu, s2 = 0x79622d32u, s3 = 0x6b206574u;
  uint32_t x0 = s0, x1 = s1, x2 = s2, x3 = s3;
  uint32_t x4 = key.k[0], x5 = key.k[1], x6 = key.k[2], x7 = key.k[3];
  uint32_t x8 = key.k[4], x9 = key.k[5], x10 = key.k[6], x11 = key.k[7];
  uint32_t x12 = (uint32_t)counter, x13 = (uint32_t)(counter >> 32);
  uint32_t x14 = (uint32_t)stream, x15 = (uint32_t)(stream >> 32);
#pragma unroll
  for (int r = 0; r < ROUNDS; r += 2) {
    RG_QR(0, 4, 8, 12) RG_QR(1, 5, 9, 13) RG_QR(2, 6, 10, 14) RG_QR(3, 7, 11, 15)
    RG_QR(0, 5, 10, 15) RG_QR(1, 6, 11, 12) RG_QR(2, 7, 8, 13) RG_QR(3, 4, 9, 14)
  }
  out[0] = x0 + s0; out[1] = x1 + s1; out[2] = x2 + s2; out[3] = x3 + s3;
  out[4] = x4 + key.k[0]; out[5] = x5 + key.k[1]; out[6] = x6 + key.k[2]; out[7] = x7 + key.k[3];
  out[8] = x8 + key.k[4]; out[9] = x9 + key.k[5]; out[10] = x10 + key.k[6]; out[11] = x11 + key.k[7];
  out[12] = x12 + (uint32_t)counter; out[13] = x13 + (uint32_t)(counter >> 32);
  out[14] = x14 + (uint32_t)stream; out[15] = x15 + (uint32_t)(stream >> 32);
}
#undef RG_QR

// Select out[i] for a runtime i without dynamic register indexing (no scratch).
RG_HD uint32_t select16(const uint32_t v[16], uint32_t i) {
  uint32_t r = v[0];
#pragma unroll
  for (uint32_t j = 1; j < 16; j++) r = (i == j) ? v[j] : r;
  return r;
}

// SplitMix64 finaliser: the trace generator's counter-based hash.
RG_HD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
RG_HD uint64_t trace_key(uint64_t seed, uint32_t key) {
  return mix64(seed ^ ((uint64_t)(key + 1) * 0xD1B54A32D192ED03ull));
}
constexpr uint64_t kTraceP90 = 0xE666666666666800ull;

// ---------------------------------------------------------------------------
// Device-resident bookkeeping. Each hot field sits on its own 128-B line so the
// per-workgroup atomics of one launch spread over memory channels.
// ---------------------------------------------------------------------------
struct alignas(128) Line {
  unsigned long long v;
  unsigned long long pad[15];
};

// One per launch parity (seq & 1). The last tile of launch e resets record
// (e+1)&1 for the next launch, so no host memset sits between steps.
struct Record {
  Line error;      // device protocol fault bits
  Line ticket;     // lag kernel: next tile ticket (dynamic tile order)
  Line done;       // lag kernel: workgroups that published their statistics
};

struct DevState {
  unsigned long long rng_next;
  unsigned long long last_committed;
  unsigned long long commit_watermark;
  unsigned long long steps;
  // Sharded REF (rg_phase_step_shard_async): provisional stream position of this
  // shard's draws, advanced by the shard's own VQ count only. Never read by the
  // single-evaluator path; the fix-up re-draws at the global position.
  unsigned long long shard_draws;
};

// Sharded REF draw record (4 B), one per VQ slot of a shard step, indexed by the slot's
// local draw number: bits 0-23 the slot's offset inside its record segment (2^24 slots =
// 2^19 words of the window), bits 24-30 info:
//   info bits 0-1 (c1 vs c0 over R1: 0 tie, 1 c1 > c0, 2 c1 < c0),
//   bits 2-3 decision code if the own round-2 vote is V0, bits 4-5 if it is V1,
//   bit 6 the provisional own vote (the likelier outcome of the draw).
// A window's record region (include/rabia_gpu.h rg_record_window_words) is the segment
// table, then the records: table[s] = local draw number of segment s's first VQ slot
// (written by the thread whose words start segment s), so segment s's records are
// [table[s], table[s + 1]). Round 5's records were 8 B (a 32-bit window offset).
constexpr uint32_t kRecGt = 1u, kRecLt = 2u;
constexpr uint32_t kRecChunkShift = 24, kRecChunkWords = 1u << (kRecChunkShift - 5);  // a segment: 2^24 slots
constexpr uint32_t kRecNone = 0xFFFFFFFFu;  // (bit 31 is 0 in every record)
RG_HD uint64_t rec_chunks(uint64_t n_slots) { return (n_slots + (1ull << kRecChunkShift) - 1) >> kRecChunkShift; }
RG_HD uint64_t rec_table_words(uint64_t n_slots) { return (rec_chunks(n_slots) + 1 + 3) & ~3ull; }
RG_HD uint32_t rec_make(uint32_t off, uint32_t info) {
  return (off & ((1u << kRecChunkShift) - 1u)) | (info << kRecChunkShift);
}

struct DevResult {  // layout-identical to rg_step_result
  unsigned long long n_slots, n_decided, n_v1, n_pending_r1, n_draws;
  unsigned long long last_committed_max, first_undecided, rng_next, commit_watermark, flags;
};

}  // namespace rg
