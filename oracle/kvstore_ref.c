/*
 * kvstore_ref.c — sequential C restatement of the kvstore_smr apply path.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: tests/ use it as the checker for full-size
 * (2^22-command) device applies, and tools/bench_c4.py times it as the CPU
 * baseline of the C4 apply. Nothing in rabia_amd/ links or calls it.
 *
 * Semantics are exactly oracle/kvstore_ref.py (which is pinned by the outcomes of
 * the reference's own kvstore tests, tests/golden/kv_reference_cases.json) and
 * restate, reference @ /root/reference read as text:
 *   KVOperation bincode 1.3.3 wire form      examples/kvstore_smr/src/operations.rs:10-19
 *   KVStoreSMR::apply_command(s)             examples/kvstore_smr/src/smr_impl.rs:72-127
 *   KVStore::set / get / delete / exists     examples/kvstore_smr/src/store.rs:144-262
 *   validate_key / validate_value            store.rs:463-478
 *   ValueEntry versions                      store.rs:55-80
 *   KVStore.version (get_version per notify) store.rs:486-489
 * One thread, one open-addressing table (FNV-1a 64, linear probing, grown at 50 %
 * load), key and value bytes in one arena; a deleted key keeps its slot
 * (tombstone) so probe chains stay intact, like the device table.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { K_SET = 0, K_GET = 1, K_DELETE = 2, K_EXISTS = 3 };
enum { R_OK = 0, R_NOT_FOUND, R_KEY_EMPTY, R_KEY_LONG, R_VALUE_LARGE, R_FULL, R_DECODE, R_NOT_APPLIED };

typedef struct {
  uint64_t hash;     /* 0 = empty slot */
  uint64_t key_off;  /* arena offsets */
  uint64_t val_off;
  uint32_t key_len, val_len, val_cap;
  uint32_t version;  /* 0 = deleted (tombstone) */
} kv_slot;

typedef struct or_kv {
  uint64_t max_keys, max_value;
  int notify;
  kv_slot* t;
  uint64_t cap, used; /* slots holding a key (live or tombstone) */
  uint64_t live, version, total_ops;
  uint8_t* arena;
  uint64_t arena_len, arena_cap;
} or_kv;

static uint64_t fnv1a(const uint8_t* p, uint64_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ULL;
  return h ? h : 1; /* 0 marks an empty slot */
}

/* std::string::String::from_utf8 (core::str::from_utf8): well-formed UTF-8 only
 * (no overlongs, no surrogates, <= U+10FFFF). */
static int utf8_ok(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t need, cp;
    if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
    else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
    else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
    else return 0;
    for (uint32_t k = 1; k <= need; k++) {
      if (i + k >= n) return 0;
      const uint8_t d = s[i + k];
      if ((d & 0xC0) != 0x80) return 0;
      cp = (cp << 6) | (d & 0x3F);
    }
    if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return 0;
    if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return 0;
    i += need + 1;
  }
  return 1;
}

static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

static int arena_put(or_kv* kv, const uint8_t* p, uint64_t n, uint64_t* off) {
  if (kv->arena_len + n > kv->arena_cap) {
    uint64_t c = kv->arena_cap ? kv->arena_cap : (1u << 20);
    while (c < kv->arena_len + n) c *= 2;
    uint8_t* a = (uint8_t*)realloc(kv->arena, c);
    if (!a) return -1;
    kv->arena = a;
    kv->arena_cap = c;
  }
  memcpy(kv->arena + kv->arena_len, p, n);
  *off = kv->arena_len;
  kv->arena_len += n;
  return 0;
}

static int grow(or_kv* kv) {
  const uint64_t nc = kv->cap ? kv->cap * 2 : 1024;
  kv_slot* nt = (kv_slot*)calloc(nc, sizeof(kv_slot));
  if (!nt) return -1;
  for (uint64_t i = 0; i < kv->cap; i++) {
    const kv_slot* e = &kv->t[i];
    if (!e->hash) continue;
    uint64_t h = e->hash & (nc - 1);
    while (nt[h].hash) h = (h + 1) & (nc - 1);
    nt[h] = *e;
  }
  free(kv->t);
  kv->t = nt;
  kv->cap = nc;
  return 0;
}

/* slot of key (existing, live or tombstone) or the empty slot it would take */
static kv_slot* find(or_kv* kv, const uint8_t* key, uint32_t klen, uint64_t h) {
  uint64_t i = h & (kv->cap - 1);
  for (;;) {
    kv_slot* e = &kv->t[i];
    if (!e->hash) return e;
    if (e->hash == h && e->key_len == klen && !memcmp(kv->arena + e->key_off, key, klen)) return e;
    i = (i + 1) & (kv->cap - 1);
  }
}

or_kv* or_kv_create(uint64_t max_keys, uint64_t max_value_size, int enable_notifications) {
  or_kv* kv = (or_kv*)calloc(1, sizeof(or_kv));
  if (!kv) return NULL;
  kv->max_keys = max_keys ? max_keys : 1000000;      /* store.rs:35 */
  kv->max_value = max_value_size ? max_value_size : 1024 * 1024; /* store.rs:39 */
  kv->notify = enable_notifications;
  if (grow(kv)) { free(kv); return NULL; }
  return kv;
}

void or_kv_destroy(or_kv* kv) {
  if (!kv) return;
  free(kv->t);
  free(kv->arena);
  free(kv);
}

/* KVStoreSMR::apply_command on Command.data (smr_impl.rs:72-127) */
static int apply_one(or_kv* kv, const uint8_t* d, uint64_t len) {
  if (len < 12) return R_DECODE;
  const uint32_t kind = rd32(d);
  const uint64_t klen = rd64(d + 4);
  if (kind > 3 || klen > len - 12) return R_DECODE;
  const uint8_t* key = d + 12;
  const uint8_t* val = NULL;
  uint64_t vlen = 0;
  if (kind == K_SET) {
    const uint64_t pos = 12 + klen;
    if (len - pos < 8) return R_DECODE;
    vlen = rd64(d + pos);
    if (vlen > len - pos - 8) return R_DECODE;
    val = d + pos + 8;
  }
  if (!utf8_ok(key, klen) || (vlen && !utf8_ok(val, vlen))) return R_DECODE;
  if (klen == 0) return R_KEY_EMPTY;   /* store.rs:463-471 */
  if (klen > 256) return R_KEY_LONG;
  const uint64_t h = fnv1a(key, klen);
  kv_slot* e = find(kv, key, (uint32_t)klen, h);
  const int live = e->hash && e->version;
  if (kind == K_SET) {                 /* store.rs:144-189 */
    if (vlen > kv->max_value) return R_VALUE_LARGE;
    if (live) {
      e->version += 1;                 /* ValueEntry::update */
    } else {
      if (kv->live >= kv->max_keys) return R_FULL; /* store.rs:153-158 */
      if (!e->hash) {
        if ((kv->used + 1) * 2 > kv->cap) {
          if (grow(kv)) return R_FULL;
          e = find(kv, key, (uint32_t)klen, h);
        }
        if (arena_put(kv, key, klen, &e->key_off)) return R_FULL;
        e->hash = h;
        e->key_len = (uint32_t)klen;
        e->val_cap = 0;
        kv->used++;
      }
      e->version = 1;                  /* ValueEntry::new (fresh after a delete) */
      kv->live++;
    }
    if (vlen > e->val_cap) {           /* values live in the arena; reuse when they fit */
      if (arena_put(kv, val, vlen, &e->val_off)) return R_FULL;
      e->val_cap = (uint32_t)vlen;
    } else if (vlen) {
      memcpy(kv->arena + e->val_off, val, vlen);
    }
    e->val_len = (uint32_t)vlen;
    kv->total_ops++;
    if (kv->notify) kv->version++;
    return R_OK;
  }
  kv->total_ops++;
  if (kind == K_DELETE) {              /* store.rs:217-251 */
    if (!live) return R_NOT_FOUND;
    e->version = 0;
    kv->live--;
    if (kv->notify) kv->version++;
    return R_OK;
  }
  return live ? R_OK : R_NOT_FOUND;    /* Get / Exists, store.rs:191-201, 254-262 */
}

/* Commands 0..n-1 in order: data[off[c] .. off[c+1]); mask NULL = apply all, else
 * commands with mask[c] == 0 get R_NOT_APPLIED (their slot was not decided V1). */
int or_kv_apply(or_kv* kv, const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* mask,
                uint8_t* results) {
  if (!kv || (n && (!data || !off || !results))) return -1;
  for (uint64_t c = 0; c < n; c++) {
    if (mask && !mask[c]) { results[c] = R_NOT_APPLIED; continue; }
    results[c] = (uint8_t)apply_one(kv, data + off[c], off[c + 1] - off[c]);
  }
  return 0;
}

/* live keys, KVStore.version, total_operations, and the bytes a dump needs */
void or_kv_stats(const or_kv* kv, uint64_t out[5]) {
  uint64_t kb = 0, vb = 0;
  for (uint64_t i = 0; i < kv->cap; i++)
    if (kv->t[i].hash && kv->t[i].version) { kb += kv->t[i].key_len; vb += kv->t[i].val_len; }
  out[0] = kv->live; out[1] = kv->version; out[2] = kv->total_ops; out[3] = kb; out[4] = vb;
}

/* live entries: key_off[live + 1], keys, val_off[live + 1], vals, versions[live] */
int or_kv_dump(const or_kv* kv, uint64_t* key_off, uint8_t* keys, uint64_t* val_off, uint8_t* vals,
               uint32_t* versions) {
  uint64_t j = 0, kp = 0, vp = 0;
  key_off[0] = val_off[0] = 0;
  for (uint64_t i = 0; i < kv->cap; i++) {
    const kv_slot* e = &kv->t[i];
    if (!e->hash || !e->version) continue;
    memcpy(keys + kp, kv->arena + e->key_off, e->key_len);
    memcpy(vals + vp, kv->arena + e->val_off, e->val_len);
    kp += e->key_len;
    vp += e->val_len;
    versions[j] = e->version;
    key_off[++j] = kp;
    val_off[j] = vp;
  }
  return 0;
}

/* All-core CPU baseline of the same apply (BASELINE INFRASTRUCTURE ONLY,
 * tools/bench_c4.py): the commands are partitioned by key hash over `parts`
 * independent stores, each replayed in total order by one thread. Exact when the
 * store's only cross-key dependency (StoreFull, store.rs:153-158) cannot fire, i.e.
 * when live keys + keys created stay below max_keys (every partition gets the whole
 * max_keys); a command that does not decode goes to partition 0 (it touches no
 * store). threads <= 0: the OpenMP default. Results are per command, in command order; out[0..2] = live keys,
 * KVStore.version and total_operations summed over the partitions. */
static uint64_t part_of(const uint8_t* d, uint64_t len, uint32_t parts) {
  if (len < 12) return 0;
  const uint64_t klen = rd64(d + 4);
  if (klen > len - 12 || klen == 0 || klen > 256) return 0;
  return fnv1a(d + 12, klen) % parts;
}

int or_kv_apply_partitioned(uint32_t parts, int threads, uint64_t max_keys, uint64_t max_value_size,
                            int enable_notifications, const uint8_t* data, const uint64_t* off, uint64_t n,
                            const uint8_t* mask, uint8_t* results, uint64_t out[3]) {
  if (!parts || (n && (!data || !off || !results))) return -1;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#else
  threads = 1;
#endif
  uint32_t* pc = (uint32_t*)malloc(n * sizeof(uint32_t) + 1);
  uint64_t* cnt = (uint64_t*)calloc((size_t)parts + 1, sizeof(uint64_t));
  uint64_t* idx = (uint64_t*)malloc(n * sizeof(uint64_t) + 8);
  uint64_t* tot = (uint64_t*)calloc((size_t)parts * 3, sizeof(uint64_t));
  if (!pc || !cnt || !idx || !tot) { free(pc); free(cnt); free(idx); free(tot); return -1; }
  int64_t nn = (int64_t)n;
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t c = 0; c < nn; c++) {
    if (mask && !mask[c]) { results[c] = R_NOT_APPLIED; pc[c] = parts; continue; }
    pc[c] = (uint32_t)part_of(data + off[c], off[c + 1] - off[c], parts);
  }
  for (uint64_t c = 0; c < n; c++) if (pc[c] < parts) cnt[pc[c] + 1]++;
  for (uint32_t p = 0; p < parts; p++) cnt[p + 1] += cnt[p];
  {
    uint64_t* cur = (uint64_t*)malloc((size_t)parts * sizeof(uint64_t));
    if (!cur) { free(pc); free(cnt); free(idx); free(tot); return -1; }
    memcpy(cur, cnt, (size_t)parts * sizeof(uint64_t));
    for (uint64_t c = 0; c < n; c++) if (pc[c] < parts) idx[cur[pc[c]]++] = c;  /* ascending within a part */
    free(cur);
  }
  int err = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err) num_threads(threads)
  for (int64_t p = 0; p < (int64_t)parts; p++) {
    or_kv* kv = or_kv_create(max_keys, max_value_size, enable_notifications);
    if (!kv) { err |= 1; continue; }
    for (uint64_t k = cnt[p]; k < cnt[p + 1]; k++) {
      const uint64_t c = idx[k];
      results[c] = (uint8_t)apply_one(kv, data + off[c], off[c + 1] - off[c]);
    }
    tot[3 * p] = kv->live; tot[3 * p + 1] = kv->version; tot[3 * p + 2] = kv->total_ops;
    or_kv_destroy(kv);
  }
  out[0] = out[1] = out[2] = 0;
  for (uint32_t p = 0; p < parts; p++) { out[0] += tot[3 * p]; out[1] += tot[3 * p + 1]; out[2] += tot[3 * p + 2]; }
  free(pc); free(cnt); free(idx); free(tot);
  return err ? -1 : 0;
}
