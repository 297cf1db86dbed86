/*
 * rabia_oracle.c — CPU restatement of the rabia-rs phase-evaluation hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rabia_oracle.h). Parity unpinned for the tally
 * and for the REF RNG stream (no Rust toolchain, no reference golden vectors);
 * ChaCha core pinned at 20 rounds by RFC 7539 A.1 / openssl keystreams.
 *
 * Each function names the reference file:line it restates. Third-party
 * arithmetic absent from /root/reference is restated from the published
 * algorithms of the crate versions pinned in /root/reference/Cargo.lock:
 *   rand 0.8.5 (Rng::gen_bool -> Bernoulli), rand_chacha 0.3.1 (StdRng =
 *   ChaCha12Rng), rand_core 0.6.4 (SeedableRng::seed_from_u64, BlockRng::next_u64).
 */
#include "rabia_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* count_votes: rabia-core/src/messages.rs:185-211                            */
/* V0 if c0>=q, else V1 if c1>=q, else VQuestion if cq>=q, else None.         */
/* Absent voters (code 3) are simply not in the HashMap.                      */
/* ------------------------------------------------------------------------- */
int or_count_votes(const uint8_t* codes, int n, int q) {
  int c0 = 0, c1 = 0, cq = 0;
  for (int j = 0; j < n; j++) {
    if (codes[j] == OR_V0) c0++;
    else if (codes[j] == OR_V1) c1++;
    else if (codes[j] == OR_VQ) cq++;
  }
  if (c0 >= q) return OR_V0;
  if (c1 >= q) return OR_V1;
  if (cq >= q) return OR_VQ;
  return OR_NONE;
}

/* handle_vote_round1 rule: rabia-engine/src/engine.rs:495-505.
 * Majority -> that value; else if |round1_votes| >= quorum -> VQuestion;
 * else still pending (NONE). */
int or_ref_round1(const uint8_t* codes, int n, int q) {
  int r = or_count_votes(codes, n, q);
  if (r != OR_NONE) return r;
  int present = 0;
  for (int j = 0; j < n; j++) present += codes[j] != OR_NONE;
  return present >= q ? OR_VQ : OR_NONE;
}

/* rand_core 0.6.4 SeedableRng::seed_from_u64: PCG32 (MUL/INC below) fills the
 * 32-byte ChaCha key 4 bytes at a time, little endian. Called from
 * rabia-engine/src/engine.rs:59-62 (RabiaConfig.randomization_seed). */
void or_seed_from_u64(uint64_t state, uint32_t key[8]) {
  const uint64_t MUL = 6364136223846793005ULL;
  const uint64_t INC = 11634580027462260723ULL;
  for (int i = 0; i < 8; i++) {
    state = state * MUL + INC;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    key[i] = (xorshifted >> rot) | (xorshifted << ((32u - rot) & 31u));
  }
}

#define OR_ROTL(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define OR_QR(a, b, c, d)                                             \
  x[a] += x[b]; x[d] ^= x[a]; x[d] = OR_ROTL(x[d], 16);               \
  x[c] += x[d]; x[b] ^= x[c]; x[b] = OR_ROTL(x[b], 12);               \
  x[a] += x[b]; x[d] ^= x[a]; x[d] = OR_ROTL(x[d], 8);                \
  x[c] += x[d]; x[b] ^= x[c]; x[b] = OR_ROTL(x[b], 7);

/* ChaCha block function (RFC 7539 §2.3 layout with rand_chacha's 64-bit block
 * counter in words 12-13 and 64-bit stream id in words 14-15). rand_chacha
 * 0.3.1 ChaCha12Rng = rounds 12, stream 0. */
void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream,
                     int rounds, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    (uint32_t)counter, (uint32_t)(counter >> 32),
                    (uint32_t)stream, (uint32_t)(stream >> 32)};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
  for (int r = 0; r < rounds; r += 2) {
    OR_QR(0, 4, 8, 12) OR_QR(1, 5, 9, 13) OR_QR(2, 6, 10, 14) OR_QR(3, 7, 11, 15)
    OR_QR(0, 5, 10, 15) OR_QR(1, 6, 11, 12) OR_QR(2, 7, 8, 13) OR_QR(3, 4, 9, 14)
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

/* Draw k of StdRng: rand_core BlockRng::next_u64 reads results[i] | results[i+1]<<32
 * with i even (the engine only ever draws u64s: gen_bool -> gen::<u64>()), so draw k
 * is keystream words 2k, 2k+1: block k/8, words 2(k%8), 2(k%8)+1. */
uint64_t or_ref_draw(const uint32_t key[8], uint64_t k) {
  uint32_t b[16];
  or_chacha_block(key, k >> 3, 0, 12, b);
  unsigned w = (unsigned)(k & 7) * 2;
  return (uint64_t)b[w] | ((uint64_t)b[w + 1] << 32);
}

/* rand 0.8.5 Bernoulli::new: p_int = (p * 2^64) as u64; sample: u < p_int. */
uint64_t or_bernoulli_p_int(double p) {
  if (p >= 1.0) return UINT64_MAX;
  return (uint64_t)(p * 18446744073709551616.0);
}

/* determine_round2_vote_for_question: rabia-engine/src/engine.rs:567-611.
 * c1 > c0: V1 w.p. 0.9 (engine.rs:587); c1 < c0: V0 w.p. 0.9 (:595);
 * tie: V1 w.p. 0.8 (:604). Counts are over the received round-1 votes. */
int or_ref_round2_vote_for_question(int c0, int c1, uint64_t u) {
  const uint64_t P90 = 0xE666666666666800ULL, P80 = 0xCCCCCCCCCCCCD000ULL;
  if (c1 > c0) return u < P90 ? OR_V1 : OR_V0;
  if (c1 < c0) return u < P90 ? OR_V0 : OR_V1;
  return u < P80 ? OR_V1 : OR_V0;
}

/* Common coin (WMVC; weak_mvc.ivy:173-186 `coin(p, v)`; paper §4 "Common Coin":
 * seeded per slot + configuration epoch, identical at every replica without
 * communication). The reference implements no coin; this definition is the
 * build's own: ChaCha12, key = seed_from_u64(coin_seed),
 * stream = epoch | 2^63, block counter = (phase-1)<<40 | slot>>9, coin = bit
 * (slot & 511) of the 512-bit block (LE words). 1 -> V1, 0 -> V0. */
int or_coin(const uint32_t coin_key[8], uint64_t epoch, uint64_t slot, uint64_t phase) {
  uint32_t b[16];
  or_chacha_block(coin_key, ((phase - 1) << 40) | (slot >> 9),
                  epoch | 0x8000000000000000ULL, 12, b);
  return (int)((b[(slot >> 5) & 15] >> (slot & 31)) & 1u);
}

static void count3(const uint8_t* codes, int n, int* c0, int* c1, int* cq, int* present) {
  *c0 = *c1 = *cq = 0;
  for (int j = 0; j < n; j++) {
    if (codes[j] == OR_V0) (*c0)++;
    else if (codes[j] == OR_V1) (*c1)++;
    else if (codes[j] == OR_VQ) (*cq)++;
  }
  *present = *c0 + *c1 + *cq;
}

static void finish_result(or_result* res, uint64_t slot_base, uint64_t S,
                          uint64_t last_committed_in, uint64_t watermark_in,
                          uint64_t max_v1_plus1, uint64_t first_undecided) {
  res->n_slots = S;
  res->last_committed_max = last_committed_in;
  if (max_v1_plus1 && max_v1_plus1 - 1 > last_committed_in)
    res->last_committed_max = max_v1_plus1 - 1;
  res->first_undecided = first_undecided;
  res->commit_watermark = watermark_in;
  if (slot_base <= watermark_in && watermark_in < first_undecided)
    res->commit_watermark = first_undecided;
}

/* ------------------------------------------------------------------------- */
/* REF phase step (final-vote-set semantics):               */
/*   r1      = handle_vote_round1 rule            engine.rs:483-509          */
/*   own r2  = proceed_to_round2                  engine.rs:511-565, 567-611 */
/*             (one StdRng draw per VQ slot, ascending slot order)           */
/*   R2'     = R2 with own vote at self_lane      engine.rs:540-542          */
/*   d       = has_round2_majority(R2')           engine.rs:624-628          */
/*   commit  = set_decision                        messages.rs:217-222        */
/*   lc      = commit_phase on V1 decisions        engine.rs:643-650,        */
/*             (max, refused if id > max_phase)   state.rs:65-103            */
/* ------------------------------------------------------------------------- */
int or_ref_step(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base,
                uint64_t slot_base, uint64_t max_phase, uint64_t last_committed_in,
                uint64_t watermark_in, const uint8_t* r1, const uint8_t* r2,
                uint64_t S, uint8_t* o_r1, uint8_t* o_r2own, uint8_t* o_dec,
                uint8_t* o_committed, uint8_t* o_value, or_result* res) {
  if (n < 1 || n > 16 || q < 1) return -1;
  uint32_t key[8];
  or_seed_from_u64(seed, key);
  memset(res, 0, sizeof *res);
  uint64_t k = rng_base, max_v1p1 = 0, first_und = slot_base + S;
  uint8_t votes2[16];
  for (uint64_t s = 0; s < S; s++) {
    const uint8_t* x1 = r1 + s * n;
    int c0, c1, cq, present;
    count3(x1, n, &c0, &c1, &cq, &present);
    int res1 = or_ref_round1(x1, n, q);
    int own = OR_NONE;
    if (res1 == OR_V0 || res1 == OR_V1) {
      own = res1;
    } else if (res1 == OR_VQ) {
      own = or_ref_round2_vote_for_question(c0, c1, or_ref_draw(key, k));
      k++;
    } else {
      res->n_pending_r1++;
    }
    memcpy(votes2, r2 + s * n, (size_t)n);
    if (own != OR_NONE && self_lane >= 0 && self_lane < n) votes2[self_lane] = (uint8_t)own;
    int d = or_count_votes(votes2, n, q);
    int committed = (d == OR_V0 || d == OR_V1);
    uint64_t id = slot_base + s;
    o_r1[s] = (uint8_t)res1;
    o_r2own[s] = (uint8_t)own;
    o_dec[s] = (uint8_t)d;
    o_committed[s] = (uint8_t)committed;
    o_value[s] = (uint8_t)(d == OR_V1);
    res->n_decided += (uint64_t)committed;
    if (d == OR_V1) {
      res->n_v1++;
      if (max_phase == 0 || id <= max_phase) max_v1p1 = id + 1;
    }
    if (!committed && id < first_und) first_und = id;
  }
  res->n_draws = k - rng_base;
  res->rng_next = k;
  finish_result(res, slot_base, S, last_committed_in, watermark_in, max_v1p1, first_und);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Sharded REF, stage 1 (the SHARD step; rabia_amd/csrc/rg_kernels.h           */
/* ref_lag_kernel<..., SHARD>): or_ref_step over one shard of a window, except  */
/* that a VQ slot takes no draw (its global stream position, engine.rs:567-611, */
/* depends on the VQ slots of the lower shards, which this shard does not see): */
/* its provisional own vote is the likelier outcome of the draw (c1 > c0: V1,   */
/* c1 < c0: V0, tie: V1, the branches of engine.rs:583-607), and it leaves a    */
/* draw record with the decision under either own vote (engine.rs:540-542,      */
/* 624-628). The row counts the NON-VQ slots only; n_draws = the VQ slots;     */
/* rng_next = n_draws (the provisional position from 0); watermark 0.           */
/* The record region (the device's format, include/rabia_gpu.h                 */
/* rg_record_window_words): a segment table, table[s] = local draw number of   */
/* the first VQ slot at or after slot s * 2^24, then the 4-B records (offset    */
/* inside the segment | info << 24).                                           */
/* ------------------------------------------------------------------------- */
uint64_t or_record_table_words(uint64_t S) { return (((S + 0xFFFFFFull) >> 24) + 1 + 3) & ~3ull; }

int or_shard_step(int n, int q, int self_lane, uint64_t slot_base, uint64_t max_phase,
                  const uint8_t* r1, const uint8_t* r2, uint64_t S, uint8_t* o_r1, uint8_t* o_r2own,
                  uint8_t* o_dec, uint8_t* o_committed, uint8_t* o_value, uint32_t* region,
                  uint64_t records_cap, or_result* row) {
  if (n < 1 || n > 16 || q < 1) return -1;
  memset(row, 0, sizeof *row);
  uint64_t k = 0, max_v1p1 = 0, first_und = slot_base + S;
  uint8_t votes2[16];
  const int lane_ok = self_lane >= 0 && self_lane < n;
  uint32_t* records = region + or_record_table_words(S);
  for (uint64_t s = 0; s < S; s++) {
    if ((s & 0xFFFFFFull) == 0) region[s >> 24] = (uint32_t)k;
    const uint8_t* x1 = r1 + s * n;
    int c0, c1, cq, present;
    count3(x1, n, &c0, &c1, &cq, &present);
    const int res1 = or_ref_round1(x1, n, q);
    const uint64_t id = slot_base + s;
    memcpy(votes2, r2 + s * n, (size_t)n);
    o_r1[s] = (uint8_t)res1;
    if (res1 == OR_VQ) {
      const uint32_t cls = c1 > c0 ? 1u : (c1 < c0 ? 2u : 0u);
      const int prov = cls == 2u ? OR_V0 : OR_V1;
      if (lane_ok) votes2[self_lane] = OR_V0;
      const uint32_t d0 = (uint32_t)or_count_votes(votes2, n, q);
      if (lane_ok) votes2[self_lane] = OR_V1;
      const uint32_t d1 = (uint32_t)or_count_votes(votes2, n, q);
      const uint32_t d = prov == OR_V1 ? d1 : d0;
      o_r2own[s] = (uint8_t)prov;
      o_dec[s] = (uint8_t)d;
      o_committed[s] = (uint8_t)(d <= OR_V1);
      o_value[s] = (uint8_t)(d == OR_V1);
      const uint32_t info = cls | (d0 << 2) | (d1 << 4) | ((uint32_t)(prov == OR_V1) << 6);
      if (k < records_cap) records[k] = ((uint32_t)s & 0xFFFFFFu) | (info << 24);
      k++;
      continue;  /* counted by the fix-up */
    }
    int own = OR_NONE;
    if (res1 == OR_V0 || res1 == OR_V1) own = res1;
    else row->n_pending_r1++;
    if (own != OR_NONE && lane_ok) votes2[self_lane] = (uint8_t)own;
    const int d = or_count_votes(votes2, n, q);
    const int committed = (d == OR_V0 || d == OR_V1);
    o_r2own[s] = (uint8_t)own;
    o_dec[s] = (uint8_t)d;
    o_committed[s] = (uint8_t)committed;
    o_value[s] = (uint8_t)(d == OR_V1);
    row->n_decided += (uint64_t)committed;
    if (d == OR_V1) {
      row->n_v1++;
      if (max_phase == 0 || id <= max_phase) max_v1p1 = id + 1;
    }
    if (!committed && id < first_und) first_und = id;
  }
  row->n_slots = S;
  row->n_draws = k;
  row->rng_next = k;
  row->last_committed_max = max_v1p1 ? max_v1p1 - 1 : 0;
  row->first_undecided = first_und;
  row->commit_watermark = 0;
  return 0;
}

/* Sharded REF, stage 3 (the fix-up; rg_kernels.h shard_fixup_kernel and
 * shard_fixup_finish_kernel): record k of the shard is the engine's draw g0 + k, where
 * g0 = the engine position at the step's first window + every shard's draws of the
 * earlier windows + the lower shards' draws of this window (ascending slot order over
 * the whole window, engine.rs:567-611). The draw picks the own vote
 * (or_ref_round2_vote_for_question) and with it the recorded decision; the outputs of
 * the VQ slots are rewritten and the VQ slots counted into the row (n_decided, n_v1,
 * last_committed_max within max_phase, first_undecided). out_row.rng_next = rng_after
 * (the engine position after this window, every shard's draws); *flags |= 8 when the
 * records did not fit (n_draws > records_cap: the outputs past the cap stay provisional). */
int or_shard_fixup(uint64_t seed, uint64_t g0, uint64_t slot_base, uint64_t max_phase, uint64_t S,
                   const uint32_t* region, uint64_t records_cap, uint8_t* o_r2own, uint8_t* o_dec,
                   uint8_t* o_committed, uint8_t* o_value, const or_result* row, uint64_t rng_after,
                   or_result* out_row, uint64_t* flags) {
  uint32_t key[8];
  or_seed_from_u64(seed, key);
  *out_row = *row;
  const uint64_t nn = row->n_draws < records_cap ? row->n_draws : records_cap;
  const uint64_t n_chunks = (S + 0xFFFFFFull) >> 24;
  const uint32_t* records = region + or_record_table_words(S);
  uint64_t max_v1p1 = row->last_committed_max ? row->last_committed_max + 1 : 0;
  uint64_t c = 0;
  for (uint64_t k = 0; k < nn; k++) {
    while (c + 1 < n_chunks && region[c + 1] <= k) c++;  /* record k's segment */
    const uint32_t off = (uint32_t)((c << 24) | (records[k] & 0xFFFFFFu)), info = (records[k] >> 24) & 0x7Fu;
    const uint32_t cls = info & 3u;
    const int c1 = cls == 1u, c0 = cls == 2u;  /* only the comparison matters */
    const int own = or_ref_round2_vote_for_question(c0, c1, or_ref_draw(key, g0 + k));
    const uint32_t d = own == OR_V1 ? (info >> 4) & 3u : (info >> 2) & 3u;
    const uint64_t id = slot_base + off;
    o_r2own[off] = (uint8_t)own;
    o_dec[off] = (uint8_t)d;
    o_committed[off] = (uint8_t)(d <= OR_V1);
    o_value[off] = (uint8_t)(d == OR_V1);
    if (d <= OR_V1) {
      out_row->n_decided++;
      if (d == OR_V1) {
        out_row->n_v1++;
        if ((max_phase == 0 || id <= max_phase) && id + 1 > max_v1p1) max_v1p1 = id + 1;
      }
    } else if (id < out_row->first_undecided) {
      out_row->first_undecided = id;
    }
  }
  out_row->last_committed_max = max_v1p1 ? max_v1p1 - 1 : 0;
  out_row->rng_next = rng_after;
  out_row->commit_watermark = 0;
  if (row->n_draws > records_cap) *flags |= 8u;
  return 0;
}

/* ------------------------------------------------------------------------- */
/* WMVC phase step, one replica's view (docs/weak_mvc.ivy:129-191; paper     */
/* Alg. 2). q = majority (n/2+1), fp1 = f+1.                                  */
/*   round 1 (phase_rnd1, ivy:129-143): needs >= q round-1 messages; vote2 = */
/*     v if #{R1 == v} >= q (v in {V0,V1}), else VQ.                          */
/*   round 2 (phase_rnd2, ivy:145-191): own vote inserted at self_lane;      */
/*     needs own vote and >= q round-2 messages; decide v if #{R2' == v} >=  */
/*     fp1 (V0 checked first, as in count_votes); else adopt a received non-? */
/*     value (V0 first); else state = coin(phase).                            */
/*   Pending (either round short of q): no decision, state unchanged.        */
/* ------------------------------------------------------------------------- */
int or_wmvc_step(int n, int q, int fp1, int self_lane, uint64_t coin_seed,
                 uint64_t epoch, uint64_t phase, uint64_t slot_base,
                 uint64_t last_committed_in, uint64_t watermark_in,
                 const uint8_t* r1, const uint8_t* r2, const uint8_t* state_in,
                 uint64_t S, uint8_t* o_r1, uint8_t* o_r2own, uint8_t* o_dec,
                 uint8_t* o_committed, uint8_t* o_value, or_result* res) {
  if (n < 1 || n > 16 || q < 1 || fp1 < 1 || phase < 1) return -1;
  uint32_t ckey[8];
  or_seed_from_u64(coin_seed, ckey);
  memset(res, 0, sizeof *res);
  uint64_t max_v1p1 = 0, first_und = slot_base + S;
  uint8_t votes2[16];
  for (uint64_t s = 0; s < S; s++) {
    int c0, c1, cq, present;
    count3(r1 + s * n, n, &c0, &c1, &cq, &present);
    int res1;
    if (present < q) res1 = OR_NONE;
    else if (c0 >= q) res1 = OR_V0;
    else if (c1 >= q) res1 = OR_V1;
    else res1 = OR_VQ;
    int st = state_in[s] & 1, d = OR_NONE;
    uint64_t id = slot_base + s;
    if (res1 == OR_NONE) {
      res->n_pending_r1++;
    } else {
      memcpy(votes2, r2 + s * n, (size_t)n);
      if (self_lane >= 0 && self_lane < n) votes2[self_lane] = (uint8_t)res1;
      count3(votes2, n, &c0, &c1, &cq, &present);
      if (present >= q) {
        if (c0 >= fp1) { d = OR_V0; st = 0; }
        else if (c1 >= fp1) { d = OR_V1; st = 1; }
        else if (c0 > 0) st = 0;
        else if (c1 > 0) st = 1;
        else { st = or_coin(ckey, epoch, id, phase); res->n_draws++; }
      }
    }
    int committed = d != OR_NONE;
    o_r1[s] = (uint8_t)res1;
    o_r2own[s] = (uint8_t)res1;
    o_dec[s] = (uint8_t)d;
    o_committed[s] = (uint8_t)committed;
    o_value[s] = (uint8_t)st;
    res->n_decided += (uint64_t)committed;
    if (d == OR_V1) { res->n_v1++; max_v1p1 = id + 1; }
    if (!committed && id < first_und) first_und = id;
  }
  finish_result(res, slot_base, S, last_committed_in, watermark_in, max_v1p1, first_und);
  return 0;
}

/* Exchange stage (docs/weak_mvc.ivy:109-128 initial_vote1; paper Alg. 2 l.1-7):
 * state = 1 iff some proposal digest is held by >= q replicas. Digest 0 = no
 * proposal received from that replica. */
void or_digest_majority(int n, int q, const uint64_t* digests, uint64_t S,
                        uint8_t* state_out) {
  for (uint64_t s = 0; s < S; s++) {
    int st = 0;
    for (int i = 0; i < n && !st; i++) {
      uint64_t d = digests[(uint64_t)i * S + s];
      if (!d) continue;
      int c = 0;
      for (int j = 0; j < n; j++) c += digests[(uint64_t)j * S + s] == d;
      st = c >= q;
    }
    state_out[s] = (uint8_t)st;
  }
}

void or_coin_range(uint64_t coin_seed, uint64_t epoch, uint64_t phase,
                   uint64_t slot_base, uint64_t S, uint8_t* out) {
  uint32_t ckey[8];
  or_seed_from_u64(coin_seed, ckey);
  for (uint64_t s = 0; s < S; s++) out[s] = (uint8_t)or_coin(ckey, epoch, slot_base + s, phase);
}

/* ------------------------------------------------------------------------- */
/* Structure-faithful REF path, the CPU baseline: per slot a  */
/* PhaseData with two NodeId->StateValue hash maps (messages.rs:138-175), one */
/* handler call per arriving vote (engine.rs:483-509, 613-632), get_phase     */
/* cloning the PhaseData on every read (state.rs:187-189), count_votes re-run */
/* on every arrival. round-2 own vote / decision act at the slot's final      */
/* arrival (final-vote-set semantics), so outputs equal or_ref_step.          */
/* ------------------------------------------------------------------------- */
typedef struct { uint8_t id[16]; uint8_t vote; uint8_t used; } or_entry;
typedef struct { or_entry e[32]; int len; } or_map; /* open addressing, cap 32 */
typedef struct {
  uint64_t phase_id;
  or_map round1, round2;
  int proposed, decision, committed;
} or_phase;

static void node_id_from_u32(uint32_t v, uint8_t id[16]) { /* types.rs:49-75 */
  for (int i = 0; i < 16; i += 4) {
    id[i] = (uint8_t)(v >> 24); id[i + 1] = (uint8_t)(v >> 16);
    id[i + 2] = (uint8_t)(v >> 8); id[i + 3] = (uint8_t)v;
  }
}
static uint32_t id_hash(const uint8_t id[16]) {
  uint32_t h = 2166136261u;
  for (int i = 0; i < 16; i++) h = (h ^ id[i]) * 16777619u;
  return h;
}
static void map_insert(or_map* m, const uint8_t id[16], uint8_t vote) {
  uint32_t h = id_hash(id) & 31u;
  for (;;) {
    or_entry* e = &m->e[h];
    if (!e->used) { memcpy(e->id, id, 16); e->vote = vote; e->used = 1; m->len++; return; }
    if (!memcmp(e->id, id, 16)) { e->vote = vote; return; } /* last write wins */
    h = (h + 1) & 31u;
  }
}
static int map_count_votes(const or_map* m, int q) {
  int c0 = 0, c1 = 0, cq = 0;
  for (int i = 0; i < 32; i++) {
    if (!m->e[i].used) continue;
    if (m->e[i].vote == OR_V0) c0++;
    else if (m->e[i].vote == OR_V1) c1++;
    else cq++;
  }
  if (c0 >= q) return OR_V0;
  if (c1 >= q) return OR_V1;
  if (cq >= q) return OR_VQ;
  return OR_NONE;
}

int or_ref_structured(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base,
                      uint64_t slot_base, const uint8_t* r1, const uint8_t* r2,
                      uint64_t S, uint8_t* o_dec, or_result* res) {
  if (n < 1 || n > 16) return -1;
  uint32_t key[8];
  or_seed_from_u64(seed, key);
  memset(res, 0, sizeof *res);
  uint8_t ids[16][16];
  for (int j = 0; j < n; j++) node_id_from_u32((uint32_t)j + 1, ids[j]);
  uint64_t k = rng_base;
  or_phase* ph = (or_phase*)calloc(1, sizeof(or_phase));
  or_phase* snap = (or_phase*)malloc(sizeof(or_phase));
  if (!ph || !snap) { free(ph); free(snap); return -2; }
  for (uint64_t s = 0; s < S; s++) {
    memset(ph, 0, sizeof *ph);          /* get_or_create_phase */
    ph->phase_id = slot_base + s;
    ph->proposed = OR_V1;
    ph->decision = OR_NONE;
    const uint8_t* x1 = r1 + s * n;
    const uint8_t* x2 = r2 + s * n;
    int last1 = -1, last2 = -1;
    for (int j = 0; j < n; j++) { if (x1[j] != OR_NONE) last1 = j; if (x2[j] != OR_NONE) last2 = j; }
    int own = OR_NONE;
    for (int j = 0; j < n; j++) {        /* handle_vote_round1 per arrival */
      if (x1[j] == OR_NONE) continue;
      map_insert(&ph->round1, ids[j], x1[j]);          /* update_phase */
      memcpy(snap, ph, sizeof *snap);                 /* get_phase clone */
      int maj = map_count_votes(&snap->round1, q);
      int res1 = maj != OR_NONE ? maj : (snap->round1.len >= q ? OR_VQ : OR_NONE);
      if (j == last1 && res1 != OR_NONE) {             /* proceed_to_round2 */
        if (res1 == OR_VQ) {
          int c0 = 0, c1 = 0;
          for (int i = 0; i < 32; i++) if (snap->round1.e[i].used) {
            c0 += snap->round1.e[i].vote == OR_V0; c1 += snap->round1.e[i].vote == OR_V1;
          }
          own = or_ref_round2_vote_for_question(c0, c1, or_ref_draw(key, k));
          k++;
        } else {
          own = res1;
        }
        if (self_lane >= 0 && self_lane < n) map_insert(&ph->round2, ids[self_lane], (uint8_t)own);
      }
    }
    if (own == OR_NONE) res->n_pending_r1++;
    volatile int dd = OR_NONE;
    for (int j = 0; j < n; j++) {        /* handle_vote_round2 per arrival */
      if (x2[j] == OR_NONE || (own != OR_NONE && j == self_lane)) continue;
      map_insert(&ph->round2, ids[j], x2[j]);
      memcpy(snap, ph, sizeof *snap);
      dd = map_count_votes(&snap->round2, q);  /* re-evaluated on every arrival */
    }
    (void)last2;
    (void)dd;
    memcpy(snap, ph, sizeof *snap);       /* the slot's final handler invocation */
    int d = map_count_votes(&snap->round2, q);
    ph->decision = d;                     /* make_decision -> set_decision */
    ph->committed = d == OR_V0 || d == OR_V1;
    o_dec[s] = (uint8_t)d;
    res->n_decided += (uint64_t)ph->committed;
    if (d == OR_V1) {
      res->n_v1++;
      if (ph->phase_id > res->last_committed_max) res->last_committed_max = ph->phase_id;
    }
  }
  free(ph);
  free(snap);
  res->n_slots = S;
  res->n_draws = k - rng_base;
  res->rng_next = k;
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Synthetic traces: counter-based, keyed by (seed, slot, lane, round), so    */
/* any shard regenerates its slots independently.             */
/*   kind 0 uniform : every code uniform over {V0,V1,VQ,absent}               */
/*   kind 1 agree90 : per-slot majority m (V1 w.p. 1/2); each vote = m w.p.   */
/*                    0.9, else uniform over {other, VQ, absent}              */
/*   kind 2 split   : R1 lanes rotate {V0 x (n-1)/2, V1 x rest, VQ}; R2 all VQ */
/* state plane: bit from its own key.                                         */
/* ------------------------------------------------------------------------- */
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static uint64_t trace_key(uint64_t seed, uint32_t key) {
  return mix64(seed ^ ((uint64_t)(key + 1) * 0xD1B54A32D192ED03ULL));
}
#define OR_TRACE_P90 0xE666666666666800ULL

static uint8_t split_code(int n, int lane) {
  int nv0 = (n - 1) / 2;
  if (lane < nv0) return OR_V0;
  if (lane < n - 1) return OR_V1;
  return OR_VQ;
}

void or_trace(int kind, int n, uint64_t seed, uint64_t slot_base, uint64_t S,
              uint8_t* r1, uint8_t* r2, uint8_t* state) {
  uint64_t kmaj = trace_key(seed, 0), kst = trace_key(seed, 1), krot = trace_key(seed, 2);
  for (uint64_t s = 0; s < S; s++) {
    uint64_t id = slot_base + s;
    uint8_t m = (uint8_t)(mix64(kmaj + id) & 1u);
    state[s] = (uint8_t)(mix64(kst + id) & 1u);
    uint32_t rot = (uint32_t)(mix64(krot + id) % (uint64_t)n);
    for (int r = 0; r < 2; r++) {
      uint8_t* out = (r ? r2 : r1) + s * n;
      for (int j = 0; j < n; j++) {
        uint64_t u = mix64(trace_key(seed, 16u + (uint32_t)r * 16u + (uint32_t)j) + id);
        uint8_t c;
        if (kind == 0) {
          c = (uint8_t)(u & 3u);
        } else if (kind == 1) {
          if (u < OR_TRACE_P90) c = m;
          else {
            uint32_t pick = (uint32_t)u % 3u;
            c = pick == 0 ? (uint8_t)(1 - m) : (pick == 1 ? OR_VQ : OR_NONE);
          }
        } else {
          c = r ? OR_VQ : split_code(n, (int)((j + rot) % (uint32_t)n));
        }
        out[j] = c;
      }
    }
  }
}

/* Digest trace (config 4): per slot a majority digest; each replica holds it
 * w.p. 0.9, else a replica-private digest, or nothing (0) w.p. 1/16 of those. */
void or_digest_trace(int n, uint64_t seed, uint64_t slot_base, uint64_t S, uint64_t* digests) {
  uint64_t kmaj = trace_key(seed, 3);
  for (int j = 0; j < n; j++) {
    uint64_t kj = trace_key(seed, 64u + (uint32_t)j);
    for (uint64_t s = 0; s < S; s++) {
      uint64_t id = slot_base + s;
      uint64_t u = mix64(kj + id), d;
      if (u < OR_TRACE_P90) d = mix64(kmaj + id) | 1u;
      else if ((u & 15u) == 0) d = 0;
      else d = mix64(u) | 1u;
      digests[(uint64_t)j * S + s] = d;
    }
  }
}

/* ------------------------------------------------------------------------- */
/* WMVC cluster view (DESIGN.md §Spec "cluster"): every replica of one slot   */
/* runs docs/weak_mvc.ivy phase_rnd1 / phase_rnd2 (ivy:129-191) each phase;  */
/* in each round replica r hears exactly q messages: its own and q-1 of the  */
/* other n-1, chosen by a keyed hash of (slot, phase, round, r) -- a          */
/* deterministic adversarial scheduler. A decided replica keeps voting its   */
/* decision (ivy:158-160). Runs until every replica decided or max_phases.   */
/* ------------------------------------------------------------------------- */
static uint64_t cluster_key(uint64_t seed, uint32_t phase, uint32_t round, int r) {
  return mix64(seed ^ (((uint64_t)phase << 32) | ((uint64_t)round << 16) | (uint64_t)r) *
                          0x9E6C63D0676A9A99ULL);
}

/* Bit mask (bit j = sender j heard) of receiver r's round `round` in `phase`:
 * itself plus q-1 of the other senders (scheduler hash version 2):
 * h = fmix32(low word of cluster_key ^ slot folded to 32 bits); pick i takes the
 * k-th (ascending) still available sender, k = (6-bit chunk i % 5 of word i / 5)
 * * span >> 6, word j + 1 = fmix32(word j + 0x9E3779B9). */
static uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
uint32_t or_heard(uint64_t delivery_seed, uint64_t slot, uint32_t phase, uint32_t round,
                  int r, int n, int q) {
  uint32_t s32 = (uint32_t)slot ^ ((uint32_t)(slot >> 32) * 0x9E3779B9u);
  uint32_t h = fmix32((uint32_t)cluster_key(delivery_seed, phase, round, r) ^ s32);
  uint32_t avail = ((1u << n) - 1u) & ~(1u << r);
  uint32_t mask = 1u << r;
  for (int i = 0; i < q - 1; i++) {
    if (i && i % 5 == 0) h = fmix32(h + 0x9E3779B9u);
    int span = n - 1 - i;
    int k = (int)((((h >> (6 * (i % 5))) & 63u) * (uint32_t)span) >> 6);
    uint32_t a = avail;
    for (int t = 0; t < k; t++) a &= a - 1;
    uint32_t pick = a & (~a + 1u);  /* lowest remaining set bit */
    mask |= pick;
    avail &= ~pick;
  }
  return mask;
}

int or_wmvc_cluster(int n, int q, int fp1, uint64_t coin_seed, uint64_t epoch,
                    uint64_t delivery_seed, uint32_t max_phases, uint64_t slot_base,
                    const uint8_t* states, uint64_t S, or_cluster_out* out) {
  if (n < 1 || n > 16 || q < 1 || q > n || fp1 < 1 || max_phases < 1 || max_phases > 255) return -1;
  uint32_t ckey[8];
  or_seed_from_u64(coin_seed, ckey);
  const uint32_t all = (n == 32) ? ~0u : ((1u << n) - 1u);
  for (uint64_t s = 0; s < S; s++) {
    const uint64_t id = slot_base + s;
    uint32_t st = 0, decided = 0, decv = 0;  /* bit r: replica r's state / decided / decision */
    for (int r = 0; r < n; r++) st |= (uint32_t)(states[s * n + r] & 1u) << r;
    or_cluster_out o = {OR_NONE, 0, 0, 0};
    for (uint32_t p = 1; p <= max_phases && decided != all; p++) {
      /* round 1 (phase_rnd1): vote2 = v if all q heard states are v, else '?' */
      uint32_t v1 = 0, vq = 0;  /* bit r: replica r votes V1 / '?' in round 2 */
      for (int r = 0; r < n; r++) {
        uint32_t h = or_heard(delivery_seed, id, p, 1, r, n, q);
        int c1 = __builtin_popcount(h & st), c0 = __builtin_popcount(h & ~st);
        if (c1 >= q) v1 |= 1u << r;
        else if (c0 < q) vq |= 1u << r;
      }
      /* round 2 (phase_rnd2) */
      uint32_t nst = 0;
      int coin = -1;
      for (int r = 0; r < n; r++) {
        uint32_t h = or_heard(delivery_seed, id, p, 2, r, n, q);
        int c1 = __builtin_popcount(h & v1), cq = __builtin_popcount(h & vq);
        int c0 = q - c1 - cq;
        int nv;
        if (c0 >= fp1) nv = 0;
        else if (c1 >= fp1) nv = 1;
        else nv = -1;
        if (nv >= 0 && !((decided >> r) & 1u)) {
          decided |= 1u << r;
          decv |= (uint32_t)nv << r;
          if (!o.first) o.first = (uint8_t)p;
        }
        if (nv < 0) {
          if (c0 > 0) nv = 0;
          else if (c1 > 0) nv = 1;
          else {
            if (coin < 0) { coin = or_coin(ckey, epoch, id, p); o.coins++; }
            nv = coin;
          }
        }
        if ((decided >> r) & 1u) nv = (int)((decv >> r) & 1u);
        nst |= (uint32_t)nv << r;
      }
      st = nst;
      if (decided == all) o.phases = (uint8_t)p;
    }
    /* agreement (weak_mvc.ivy invariants): every replica decided the same value;
     * a disagreement would be reported as OR_VQ (a safety violation, never seen) */
    if (decided == all) o.dec = (uint8_t)((decv == 0 || decv == all) ? (decv & 1u) : OR_VQ);
    out[s] = o;
  }
  return 0;
}

/* Initial states for the adversarial cluster trace (config 3): (n-1)/2 replicas
 * hold 1, the rest 0, rotated per slot. */
void or_cluster_trace(int n, uint64_t seed, uint64_t slot_base, uint64_t S, uint8_t* states) {
  uint64_t krot = trace_key(seed, 4);
  for (uint64_t s = 0; s < S; s++) {
    uint32_t rot = (uint32_t)(mix64(krot + slot_base + s) % (uint64_t)n);
    for (int r = 0; r < n; r++) states[s * n + r] = (uint8_t)(((uint32_t)r + rot) % (uint32_t)n < (uint32_t)(n - 1) / 2);
  }
}

/* Bit-plane layout: plane 2j+b holds bit b of lane j's code;
 * slot s lives in word s/32, bit s%32. */
void or_pack_planes(const uint8_t* codes, int n, uint64_t S, uint64_t stride,
                    uint32_t* planes) {
  memset(planes, 0, sizeof(uint32_t) * stride * (uint64_t)(2 * n));
  for (uint64_t s = 0; s < S; s++)
    for (int j = 0; j < n; j++) {
      uint8_t c = codes[s * n + j];
      if (c & 1u) planes[(uint64_t)(2 * j) * stride + s / 32] |= 1u << (s % 32);
      if (c & 2u) planes[(uint64_t)(2 * j + 1) * stride + s / 32] |= 1u << (s % 32);
    }
}

void or_unpack_planes(const uint32_t* planes, int n, uint64_t S, uint64_t stride,
                      uint8_t* codes) {
  for (uint64_t s = 0; s < S; s++)
    for (int j = 0; j < n; j++) {
      uint32_t lo = (planes[(uint64_t)(2 * j) * stride + s / 32] >> (s % 32)) & 1u;
      uint32_t hi = (planes[(uint64_t)(2 * j + 1) * stride + s / 32] >> (s % 32)) & 1u;
      codes[s * n + j] = (uint8_t)(lo | (hi << 1));
    }
}
