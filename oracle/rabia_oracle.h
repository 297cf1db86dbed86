/*
 * rabia_oracle.h — CPU restatement of the rabia-rs phase-evaluation path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in rabia_amd/ links, loads or calls this.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline, never as the product path.
 *
 * Parity status: the tally/decision restatement is "parity unpinned" against the
 * reference itself: the reference is Rust (no cargo/rustc in this image) and its
 * tests hold no golden vectors for count_votes / the phase handlers
 * (SURVEY.md §4, §8c). Pinned pieces: the ChaCha core at 20 rounds against
 * RFC 7539 A.1 and openssl-generated keystreams (tests/golden/chacha20_kat.json).
 * The tally is cross-checked against an independent pure-Python restatement
 * (oracle/rabia_ref.py) through committed exhaustive truth tables.
 *
 * Vote codes follow the serde/bincode variant order of StateValue
 * (rabia-core/src/types.rs:286-294): V0=0, V1=1, VQuestion=2; 3 = absent / none.
 */
#ifndef RABIA_ORACLE_H
#define RABIA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_V0 = 0, OR_V1 = 1, OR_VQ = 2, OR_NONE = 3 };

typedef struct or_result {
  uint64_t n_slots;
  uint64_t n_decided;          /* decision in {V0,V1} (PhaseData.is_committed) */
  uint64_t n_v1;               /* decision == V1 (batch applied)               */
  uint64_t n_pending_r1;       /* round-1 result not yet available             */
  uint64_t n_draws;            /* REF RNG draws consumed / WMVC coin flips     */
  uint64_t last_committed_max; /* EngineState.last_committed_phase after step  */
  uint64_t first_undecided;    /* min slot id not committed, or end of window  */
  uint64_t rng_next;           /* REF draw index after this step               */
  uint64_t commit_watermark;   /* contiguous watermark after this step         */
} or_result;

/* --- scalar building blocks ------------------------------------------------ */
int or_count_votes(const uint8_t* codes, int n, int q);
int or_ref_round1(const uint8_t* codes, int n, int q);
void or_seed_from_u64(uint64_t seed, uint32_t key[8]);
void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream,
                     int rounds, uint32_t out[16]);
uint64_t or_ref_draw(const uint32_t key[8], uint64_t k);
uint64_t or_bernoulli_p_int(double p);
int or_ref_round2_vote_for_question(int c0, int c1, uint64_t u);
int or_coin(const uint32_t coin_key[8], uint64_t epoch, uint64_t slot, uint64_t phase);

/* --- batch steps over slot-major code arrays [S][n] ------------------------- */
int or_ref_step(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base,
                uint64_t slot_base, uint64_t max_phase, uint64_t last_committed_in,
                uint64_t watermark_in, const uint8_t* r1, const uint8_t* r2,
                uint64_t S, uint8_t* o_r1, uint8_t* o_r2own, uint8_t* o_dec,
                uint8_t* o_committed, uint8_t* o_value, or_result* res);

int or_wmvc_step(int n, int q, int fp1, int self_lane, uint64_t coin_seed,
                 uint64_t epoch, uint64_t phase, uint64_t slot_base,
                 uint64_t last_committed_in, uint64_t watermark_in,
                 const uint8_t* r1, const uint8_t* r2, const uint8_t* state_in,
                 uint64_t S, uint8_t* o_r1, uint8_t* o_r2own, uint8_t* o_dec,
                 uint8_t* o_committed, uint8_t* o_value, or_result* res);

/* --- sharded REF: one engine over a window split into shards ---------------- */
/* The product's protocol (include/rabia_gpu.h "Sharded REF"): stage 1
 * evaluates a shard with a provisional own vote for every VQ slot and leaves one 4-B draw
 * record per VQ slot in a record region (a segment table of the first record of every
 * 2^24-slot segment, then the records: offset inside the segment | info << 24, info bits 0-1
 * c1-vs-c0 class (0 tie, 1 c1 > c0, 2 c1 < c0), 2-3 the decision under own V0, 4-5 under
 * own V1, 6 the provisional own vote) and a row of its non-VQ slots; stage 3 re-draws
 * every VQ slot at its global stream position g0 + k and patches the outputs and the row. */
uint64_t or_record_table_words(uint64_t S);
int or_shard_step(int n, int q, int self_lane, uint64_t slot_base, uint64_t max_phase,
                  const uint8_t* r1, const uint8_t* r2, uint64_t S, uint8_t* o_r1, uint8_t* o_r2own,
                  uint8_t* o_dec, uint8_t* o_committed, uint8_t* o_value, uint32_t* region,
                  uint64_t records_cap, or_result* row);
int or_shard_fixup(uint64_t seed, uint64_t g0, uint64_t slot_base, uint64_t max_phase, uint64_t S,
                   const uint32_t* region, uint64_t records_cap, uint8_t* o_r2own, uint8_t* o_dec,
                   uint8_t* o_committed, uint8_t* o_value, const or_result* row, uint64_t rng_after,
                   or_result* out_row, uint64_t* flags);

void or_digest_majority(int n, int q, const uint64_t* digests /*[n][S]*/,
                        uint64_t S, uint8_t* state_out);

void or_coin_range(uint64_t coin_seed, uint64_t epoch, uint64_t phase,
                   uint64_t slot_base, uint64_t S, uint8_t* out);

/* --- WMVC cluster view: all n replicas of a slot, phases to termination ----- */
typedef struct or_cluster_out {
  uint8_t dec;        /* OR_V0 / OR_V1 / OR_NONE (not every replica decided)   */
  uint8_t phases;     /* phase at which the last replica decided, 0 = none     */
  uint8_t first;      /* phase of the first decision, 0 = none                 */
  uint8_t coins;      /* phases in which some replica took the common coin     */
} or_cluster_out;
uint32_t or_heard(uint64_t delivery_seed, uint64_t slot, uint32_t phase, uint32_t round,
                  int r, int n, int q);
int or_wmvc_cluster(int n, int q, int fp1, uint64_t coin_seed, uint64_t epoch,
                    uint64_t delivery_seed, uint32_t max_phases, uint64_t slot_base,
                    const uint8_t* states /*[S][n]*/, uint64_t S, or_cluster_out* out);
void or_cluster_trace(int n, uint64_t seed, uint64_t slot_base, uint64_t S, uint8_t* states);

/* --- structure-faithful REF path (CPU baseline) ----------------------------- */
int or_ref_structured(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base,
                      uint64_t slot_base, const uint8_t* r1, const uint8_t* r2,
                      uint64_t S, uint8_t* o_dec, or_result* res);

/* --- fast CPU path (bench all-core baseline; rabia_cpu_soa.c) --------------- */
/* or_ref_step on the device's planar plane layout (votes: (4n+1) planes of
 * `stride` u32 words, stride even), 64 slots per u64 op, OpenMP over chunks
 * (n_threads <= 0: OpenMP default). out: 8 planes x stride (may be NULL). */
int or_ref_step_soa(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base, uint64_t slot_base,
                    uint64_t max_phase, uint64_t last_committed_in, uint64_t watermark_in,
                    const uint32_t* votes, uint64_t stride, uint64_t S, uint32_t* out, or_result* res,
                    int n_threads);
int or_omp_max_threads(void);

/* --- synthetic traces (restatement of the device generator) ----------------- */
void or_trace(int kind, int n, uint64_t seed, uint64_t slot_base, uint64_t S,
              uint8_t* r1, uint8_t* r2, uint8_t* state);
void or_digest_trace(int n, uint64_t seed, uint64_t slot_base, uint64_t S,
                     uint64_t* digests /*[n][S]*/);

/* --- bit-plane packing (restatement of the device layout) ------------------- */
void or_pack_planes(const uint8_t* codes, int n, uint64_t S, uint64_t stride_words,
                    uint32_t* planes /*[2n][stride]*/);
void or_unpack_planes(const uint32_t* planes, int n, uint64_t S, uint64_t stride_words,
                      uint8_t* codes);

#ifdef __cplusplus
}
#endif
#endif
