/* tsan_oracle.c -- ThreadSanitizer run of the CPU restatement's multi-threaded combine ("test under
 * -fsanitize=thread on the CPU restatement"): or_execute's worker pool (one task per segment, shared table under a
 * mutex, GroupByCombineOperator.processSegments :125-197) over 24 synthetic segments on 8 threads, checked equal to
 * the 1-thread run.  Test infrastructure only (tests/test_sanitize_cpu.py). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/pinot_oracle.h"

#define NSEG 24
#define NCOL 3

int main(void) {
  static or_column cols[NSEG][NCOL];
  static or_segment segs[NSEG];
  const int32_t card[NCOL] = {97, 13, 1000};  /* g1, g2, m */
  double* vals[NCOL];
  int64_t* hl[NCOL];
  int32_t* gid[NCOL];
  for (int c = 0; c < NCOL; c++) {
    vals[c] = malloc(sizeof(double) * card[c]);
    hl[c] = malloc(sizeof(int64_t) * card[c]);
    gid[c] = malloc(sizeof(int32_t) * card[c]);
    for (int i = 0; i < card[c]; i++) vals[c][i] = i * 3 - 7, hl[c][i] = i * 3 - 7, gid[c][i] = i;
  }
  unsigned long long x = 88172645463325252ull;
  for (int s = 0; s < NSEG; s++) {
    const int32_t n = 20000 + 37 * s;
    for (int c = 0; c < NCOL; c++) {
      int32_t* ids = malloc(sizeof(int32_t) * n);
      for (int i = 0; i < n; i++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        ids[i] = (int32_t)(x % (unsigned long long)card[c]);
      }
      const int bits = or_num_bits_per_value(card[c] - 1);
      uint8_t* fwd = calloc((size_t)or_fixed_bit_num_bytes(n, bits) + 8, 1);
      or_fixed_bit_write(ids, n, bits, fwd);
      free(ids);
      cols[s][c] = (or_column){card[c], bits, fwd, NULL, vals[c], hl[c], NULL, gid[c]};
    }
    segs[s] = (or_segment){n, NCOL, cols[s]};
  }
  const int32_t gcols[2] = {0, 1};
  const int64_t gcard[2] = {97, 13};
  const int32_t fn[5] = {OR_AGG_COUNT, OR_AGG_SUM, OR_AGG_MIN, OR_AGG_MAX, OR_AGG_HLL};
  const int32_t acol[5] = {-1, 2, 2, 2, 2};
  or_query q;
  memset(&q, 0, sizeof q);
  q.num_group_by = 2, q.group_cols = gcols, q.group_global_card = gcard;
  q.num_aggs = 5, q.agg_fn = fn, q.agg_col = acol, q.log2m = 8, q.num_groups_limit = 100000;
  or_result r1, r8;
  or_execute(&q, segs, NSEG, 1, &r1);
  or_execute(&q, segs, NSEG, 8, &r8);
  int ok = r1.num_groups == r8.num_groups && r1.num_docs_scanned == r8.num_docs_scanned;
  /* keys arrive in merge order: compare per key */
  for (int64_t i = 0; ok && i < r1.num_groups; i++) {
    int64_t j = 0;
    while (j < r8.num_groups && r8.keys[j] != r1.keys[i]) j++;
    ok = j < r8.num_groups && memcmp(r1.aggs + i * 5, r8.aggs + j * 5, sizeof(double) * 5) == 0 &&
         memcmp(r1.hll + i * 256, r8.hll + j * 256, 256) == 0;
  }
  printf("groups %lld docs %lld: 8-thread combine %s the 1-thread run\n", (long long)r1.num_groups,
         (long long)r1.num_docs_scanned, ok ? "equals" : "DIFFERS FROM");
  or_result_free(&r1);
  or_result_free(&r8);
  return ok ? 0 : 1;
}
