/* Sanitizer self-test of the oracle (test infrastructure only): exercises every
 * entry point under ASan/UBSan and checks the batch REF step against the
 * structure-faithful REF path. Exit code 0 = pass. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rabia_oracle.h"

int main(void) {
  const uint64_t S = 3000;
  for (int n = 1; n <= 16; n++) {
    int q = n / 2 + 1;
    uint8_t* r1 = malloc(S * n);
    uint8_t* r2 = malloc(S * n);
    uint8_t* st = malloc(S);
    uint8_t* o[5];
    for (int i = 0; i < 5; i++) o[i] = malloc(S);
    uint8_t* d2 = malloc(S);
    for (int kind = 0; kind < 3; kind++) {
      or_trace(kind, n, 42 + kind, 1, S, r1, r2, st);
      or_result a, b, c;
      if (or_ref_step(n, q, n - 1, 42, 0, 1, 0, 0, 1, r1, r2, S, o[0], o[1], o[2], o[3], o[4], &a)) return 1;
      if (or_ref_structured(n, q, n - 1, 42, 0, 1, r1, r2, S, d2, &b)) return 2;
      if (memcmp(o[2], d2, S) || a.n_draws != b.n_draws || a.n_decided != b.n_decided ||
          a.last_committed_max != b.last_committed_max) {
        fprintf(stderr, "mismatch n=%d kind=%d\n", n, kind);
        return 3;
      }
      if (or_wmvc_step(n, q, (n - 1) / 2 + 1, 0, 7, 1, 1, 1, 0, 1, r1, r2, st, S, o[0], o[1], o[2], o[3], o[4], &c)) return 4;
    }
    uint32_t* planes = malloc(sizeof(uint32_t) * 2 * n * ((S + 127) / 128 * 4));
    uint8_t* back = malloc(S * n);
    or_pack_planes(r1, n, S, (S + 127) / 128 * 4, planes);
    or_unpack_planes(planes, n, S, (S + 127) / 128 * 4, back);
    if (memcmp(back, r1, S * n)) return 5;
    uint64_t* dg = malloc(sizeof(uint64_t) * n * S);
    or_digest_trace(n, 9, 1, S, dg);
    or_digest_majority(n, q, dg, S, st);
    or_coin_range(7, 1, 3, 100, S, st);
    free(dg); free(planes); free(back);
    free(r1); free(r2); free(st); free(d2);
    for (int i = 0; i < 5; i++) free(o[i]);
  }
  puts("oracle selftest ok");
  return 0;
}
