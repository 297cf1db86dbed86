/*
 * rabia_cpu_soa.c — the FAST CPU path of the REF phase step, for the bench's
 * all-core CPU baseline ("the SoA OpenMP tally on all cores").
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see rabia_oracle.h): nothing in rabia_amd/
 * links or calls it. It computes exactly or_ref_step (rabia_oracle.c, which cites
 * engine.rs:483-682 / messages.rs:185-222 / state.rs:65-103 line by line), but the
 * way a CPU does it best: the device's plane layout (votes = (4n+1) planar bit
 * planes of `stride` u32 words), 64 slots per u64 operation with bit-sliced
 * counters, OpenMP over chunks of words. The StdRng draw index of a VQ slot (the
 * VQ slots before it, engine.rs:567-611) comes from a two-pass scan: count VQ slots
 * per chunk, exclusive prefix over chunks, evaluate.
 *
 * Function multiversioning picks AVX-512 / AVX2 / baseline code at load time, so
 * the library built in this container runs on whatever x86-64 host the GPU box has.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "rabia_oracle.h"

#define OR_P80 0xCCCCCCCCCCCCD000ULL
#define OR_P90 0xE666666666666800ULL
#define CHUNK_WORDS 2048 /* u64 words (131072 slots) per scheduling unit */

#if defined(__x86_64__) && defined(__GNUC__) && !defined(__clang__) && !defined(__SANITIZE_ADDRESS__)
#define OR_MULTIVERSION __attribute__((target_clones("avx512f", "avx2", "default")))
#else
#define OR_MULTIVERSION
#endif

typedef struct {
  uint64_t dec, v1, pend, draws, max_v1p1, min_und;
} chunk_stats;

static inline __attribute__((always_inline)) void ctr_add(uint64_t* c, const int B, uint64_t m) {
  for (int i = 0; i < B; i++) {
    const uint64_t t = c[i] & m;
    c[i] ^= m;
    m = t;
  }
}

static inline __attribute__((always_inline)) uint64_t ctr_ge(const uint64_t* c, const int B, uint32_t q) {
  uint64_t gt = 0, eq = ~0ULL;
  for (int i = B - 1; i >= 0; i--) {
    const uint64_t qb = ((q >> i) & 1u) ? ~0ULL : 0ULL;
    gt |= eq & c[i] & ~qb;
    eq &= ~(c[i] ^ qb);
  }
  return gt | eq;
}

static inline __attribute__((always_inline)) void ctr_cmp(const uint64_t* a, const uint64_t* b, const int B,
                                                          uint64_t* gt, uint64_t* lt) {
  uint64_t eq = ~0ULL, g = 0, l = 0;
  for (int i = B - 1; i >= 0; i--) {
    g |= eq & a[i] & ~b[i];
    l |= eq & ~a[i] & b[i];
    eq &= ~(a[i] ^ b[i]);
  }
  *gt = g;
  *lt = l;
}

static inline uint64_t valid64(uint64_t w, uint64_t S) {
  const uint64_t first = 64 * w;
  if (first >= S) return 0;
  const uint64_t left = S - first;
  return left >= 64 ? ~0ULL : ((1ULL << left) - 1);
}

static inline uint64_t ld64(const uint32_t* plane, uint64_t w) {
  return (uint64_t)plane[2 * w] | ((uint64_t)plane[2 * w + 1] << 32);
}

/* round 1 of one u64 word (engine.rs:495-505) */
static inline __attribute__((always_inline)) void round1(const uint32_t* votes, uint64_t stride, int n, const int B,
                                                         uint32_t q, uint64_t w, uint64_t vm, uint64_t* v1,
                                                         uint64_t* vq, uint64_t* pend, uint64_t* gt, uint64_t* lt) {
  uint64_t c0[5] = {0}, c1[5] = {0}, cp[5] = {0};
  for (int j = 0; j < n; j++) {
    const uint64_t lo = ld64(votes + (uint64_t)(2 * j) * stride, w);
    const uint64_t hi = ld64(votes + (uint64_t)(2 * j + 1) * stride, w);
    ctr_add(c0, B, ~lo & ~hi);
    ctr_add(c1, B, lo & ~hi);
    ctr_add(cp, B, ~(lo & hi));
  }
  const uint64_t g0 = ctr_ge(c0, B, q), g1 = ctr_ge(c1, B, q), gp = ctr_ge(cp, B, q);
  *v1 = ~g0 & g1 & vm;
  *vq = ~g0 & ~g1 & gp & vm;
  *pend = ~((g0 & vm) | *v1 | *vq) & vm;
  ctr_cmp(c1, c0, B, gt, lt);
}

static inline __attribute__((always_inline)) uint64_t count_chunk(const uint32_t* votes, uint64_t stride, int n,
                                                                  const int B, uint32_t q, uint64_t w0, uint64_t w1,
                                                                  uint64_t S) {
  uint64_t c = 0;
  for (uint64_t w = w0; w < w1; w++) {
    uint64_t v1, vq, pend, gt, lt;
    round1(votes, stride, n, B, q, w, valid64(w, S), &v1, &vq, &pend, &gt, &lt);
    c += (uint64_t)__builtin_popcountll(vq);
  }
  return c;
}

static inline __attribute__((always_inline)) void eval_chunk(const uint32_t* votes, uint64_t stride, int n,
                                                             const int B, uint32_t q, int self_lane,
                                                             const uint32_t key[8], uint64_t k, uint64_t slot_base,
                                                             uint64_t max_phase, uint64_t w0, uint64_t w1, uint64_t S,
                                                             uint32_t* out, chunk_stats* st) {
  uint32_t blk[16];
  uint64_t blk_id = ~0ULL;
  const uint32_t* r2 = votes + (uint64_t)(2 * n) * stride;
  for (uint64_t w = w0; w < w1; w++) {
    const uint64_t vm = valid64(w, S);
    uint64_t v1, vq, pend, gt, lt;
    round1(votes, stride, n, B, q, w, vm, &v1, &vq, &pend, &gt, &lt);
    uint64_t own = v1, m = vq;
    while (m) { /* one StdRng draw per VQ slot, ascending slot order */
      const int b = __builtin_ctzll(m);
      m &= m - 1;
      if ((k >> 3) != blk_id) {
        blk_id = k >> 3;
        or_chacha_block(key, blk_id, 0, 12, blk);
      }
      const uint32_t ws = (uint32_t)(k & 7u) * 2u;
      const uint64_t u = (uint64_t)blk[ws] | ((uint64_t)blk[ws + 1] << 32);
      const int g = (int)((gt >> b) & 1u), l = (int)((lt >> b) & 1u);
      const int vote1 = g ? (u < OR_P90) : (l ? (u >= OR_P90) : (u < OR_P80));
      own |= (uint64_t)vote1 << b;
      k++;
    }
    uint64_t c0[5] = {0}, c1[5] = {0}, cq[5] = {0};
    for (int j = 0; j < n; j++) {
      uint64_t lo = ld64(r2 + (uint64_t)(2 * j) * stride, w);
      uint64_t hi = ld64(r2 + (uint64_t)(2 * j + 1) * stride, w);
      if (j == self_lane) { /* own vote joins round2_votes (engine.rs:540-542) */
        lo = (lo & pend) | (own & ~pend);
        hi &= pend;
      }
      ctr_add(c0, B, ~lo & ~hi);
      ctr_add(c1, B, lo & ~hi);
      ctr_add(cq, B, ~lo & hi);
    }
    const uint64_t d0 = ctr_ge(c0, B, q);
    const uint64_t d1 = ~d0 & ctr_ge(c1, B, q);
    const uint64_t dq = ~d0 & ~d1 & ctr_ge(cq, B, q);
    const uint64_t dn = ~(d0 | d1 | dq);
    const uint64_t committed = (d0 | d1) & vm, dv1 = d1 & vm;
    if (out) {
      const uint64_t o[8] = {(v1 | pend) & vm, (vq | pend) & vm, (own | pend) & vm, pend,
                             (d1 | dn) & vm, (dq | dn) & vm, committed, dv1};
      for (int pl = 0; pl < 8; pl++) {
        out[(uint64_t)pl * stride + 2 * w] = (uint32_t)o[pl];
        if (2 * w + 1 < stride) out[(uint64_t)pl * stride + 2 * w + 1] = (uint32_t)(o[pl] >> 32);
      }
    }
    st->dec += (uint64_t)__builtin_popcountll(committed);
    st->v1 += (uint64_t)__builtin_popcountll(dv1);
    st->pend += (uint64_t)__builtin_popcountll(pend);
    st->draws += (uint64_t)__builtin_popcountll(vq);
    uint64_t mv = dv1;
    while (mv) {
      const int b = 63 - __builtin_clzll(mv);
      const uint64_t id = slot_base + 64 * w + (uint64_t)b;
      if (max_phase == 0 || id <= max_phase) {
        if (id + 1 > st->max_v1p1) st->max_v1p1 = id + 1;
        break;
      }
      mv &= ~(1ULL << b);
    }
    const uint64_t und = ~committed & vm;
    if (und && st->min_und == ~0ULL) st->min_und = slot_base + 64 * w + (uint64_t)__builtin_ctzll(und);
  }
}

#define DISPATCH_B(B_, CALL)   \
  switch (B_) {                \
    case 1: { const int B = 1; CALL; } break; \
    case 2: { const int B = 2; CALL; } break; \
    case 3: { const int B = 3; CALL; } break; \
    case 4: { const int B = 4; CALL; } break; \
    default: { const int B = 5; CALL; } break; \
  }

/* the per-chunk bodies, compiled once per ISA level (called from the OpenMP
 * regions, which GCC outlines before cloning) */
OR_MULTIVERSION __attribute__((noinline))
uint64_t or_soa_count_chunk(const uint32_t* votes, uint64_t stride, int n, int Bn, uint32_t q, uint64_t w0,
                            uint64_t w1, uint64_t S) {
  uint64_t cnt = 0;
  DISPATCH_B(Bn, cnt = count_chunk(votes, stride, n, B, q, w0, w1, S));
  return cnt;
}

OR_MULTIVERSION __attribute__((noinline))
void or_soa_eval_chunk(const uint32_t* votes, uint64_t stride, int n, int Bn, uint32_t q, int self_lane,
                       const uint32_t key[8], uint64_t k, uint64_t slot_base, uint64_t max_phase, uint64_t w0,
                       uint64_t w1, uint64_t S, uint32_t* out, chunk_stats* st) {
  DISPATCH_B(Bn, eval_chunk(votes, stride, n, B, q, self_lane, key, k, slot_base, max_phase, w0, w1, S, out, st));
}

int or_ref_step_soa(int n, int q, int self_lane, uint64_t seed, uint64_t rng_base, uint64_t slot_base,
                    uint64_t max_phase, uint64_t last_committed_in, uint64_t watermark_in,
                    const uint32_t* votes, uint64_t stride, uint64_t S, uint32_t* out, or_result* res,
                    int n_threads) {
  if (n < 1 || n > 16 || q < 1 || (stride & 1u) || stride * 32 < S || !votes || !res) return -1;
  uint32_t key[8];
  or_seed_from_u64(seed, key);
  const int Bn = n < 2 ? 1 : n < 4 ? 2 : n < 8 ? 3 : n < 16 ? 4 : 5;
  const uint64_t words = (S + 63) / 64;
  const uint64_t chunks = (words + CHUNK_WORDS - 1) / CHUNK_WORDS;
  uint64_t* base = (uint64_t*)malloc((chunks + 1) * sizeof(uint64_t));
  chunk_stats* cs = (chunk_stats*)malloc((chunks ? chunks : 1) * sizeof(chunk_stats));
  if (!base || !cs) { free(base); free(cs); return -2; }
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  const uint64_t stride64 = stride; /* ld64 indexes u32 planes by 2w */
  /* pass 1: VQ slots per chunk */
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < (int64_t)chunks; c++) {
    const uint64_t w0 = (uint64_t)c * CHUNK_WORDS, w1 = w0 + CHUNK_WORDS < words ? w0 + CHUNK_WORDS : words;
    base[c] = or_soa_count_chunk(votes, stride64, n, Bn, (uint32_t)q, w0, w1, S);
  }
  uint64_t acc = rng_base;
  for (uint64_t c = 0; c < chunks; c++) {
    const uint64_t x = base[c];
    base[c] = acc;
    acc += x;
  }
  /* pass 2: evaluate with each chunk's first draw index */
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < (int64_t)chunks; c++) {
    const uint64_t w0 = (uint64_t)c * CHUNK_WORDS, w1 = w0 + CHUNK_WORDS < words ? w0 + CHUNK_WORDS : words;
    chunk_stats st = {0, 0, 0, 0, 0, ~0ULL};
    or_soa_eval_chunk(votes, stride64, n, Bn, (uint32_t)q, self_lane, key, base[c], slot_base, max_phase, w0, w1,
                      S, out, &st);
    cs[c] = st;
  }
  memset(res, 0, sizeof *res);
  uint64_t max_v1p1 = 0, first_und = slot_base + S;
  for (uint64_t c = 0; c < chunks; c++) {
    res->n_decided += cs[c].dec;
    res->n_v1 += cs[c].v1;
    res->n_pending_r1 += cs[c].pend;
    res->n_draws += cs[c].draws;
    if (cs[c].max_v1p1 > max_v1p1) max_v1p1 = cs[c].max_v1p1;
    if (cs[c].min_und < first_und) first_und = cs[c].min_und;
  }
  res->rng_next = rng_base + res->n_draws;
  res->n_slots = S;
  res->last_committed_max = last_committed_in;
  if (max_v1p1 && max_v1p1 - 1 > last_committed_in) res->last_committed_max = max_v1p1 - 1;
  res->first_undecided = first_und;
  res->commit_watermark = watermark_in;
  if (slot_base <= watermark_in && watermark_in < first_und) res->commit_watermark = first_und;
  free(base);
  free(cs);
  return 0;
}

int or_omp_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
