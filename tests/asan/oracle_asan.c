/* Host sanitizer run of the oracle (test infrastructure):
 * every oracle entry point on seeded random clusters, built with
 * -fsanitize=address,undefined by oracle/Makefile's asan target.  Exit 0
 * when clean (ASan / UBSan abort otherwise). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned long long u64;
int oracle_build(int64_t n, int64_t K, const int64_t* lab_off, const int32_t* lab_key,
                 const int32_t* lab_val, int64_t P, const int64_t* ws_off, const int32_t* ws_key,
                 const int32_t* ws_val, const int64_t* wa_off, const int32_t* wa_key,
                 const int32_t* wa_val, u64* M, u64* sel_out, u64* alw_out);
int oracle_lists(int64_t n, int64_t P, const u64* sets, int64_t* off, int32_t* list);
int oracle_column_checks(int64_t n, const u64* M, int64_t cols_begin, int64_t cols_end,
                         uint8_t* reach, uint8_t* isol);
int oracle_crosscheck(int64_t n, const u64* M, const int32_t* gid, int64_t cols_begin,
                      int64_t cols_end, uint8_t* cross);
int oracle_shadow(int64_t n_lists, int64_t nbits, const int64_t* off, const int32_t* lst,
                  const u64* allow, int64_t c_begin, int64_t c_end, int64_t cap, int32_t* out,
                  int64_t* count);
int64_t oracle_path(int64_t n, int64_t W, const u64* M, int64_t hops, u64* P);

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd(uint32_t m) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return (uint32_t)(rs % m);
}

static int run(int64_t n, int64_t P, int64_t K) {
  const int64_t W = (n + 63) / 64;
  int64_t* lab_off = calloc((size_t)n + 1, sizeof(int64_t));
  int32_t* lab_key = malloc(sizeof(int32_t) * (size_t)(n * K + 1));
  int32_t* lab_val = malloc(sizeof(int32_t) * (size_t)(n * K + 1));
  int64_t e = 0;
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t k = 0; k < K; ++k)
      if (rnd(4) != 0) { lab_key[e] = (int32_t)k; lab_val[e] = (int32_t)rnd(5); ++e; }
    lab_off[i + 1] = e;
  }
  int64_t *so = calloc((size_t)P + 1, sizeof(int64_t)), *ao = calloc((size_t)P + 1, sizeof(int64_t));
  int32_t *sk = malloc(sizeof(int32_t) * (size_t)(3 * P + 1)), *sv = malloc(sizeof(int32_t) * (size_t)(3 * P + 1));
  int32_t *ak = malloc(sizeof(int32_t) * (size_t)(3 * P + 1)), *av = malloc(sizeof(int32_t) * (size_t)(3 * P + 1));
  int64_t es = 0, ea = 0;
  for (int64_t p = 0; p < P; ++p) {
    for (int t = (int)rnd(3); t > 0; --t) { sk[es] = (int32_t)rnd((uint32_t)K + 1) - 1; sv[es] = (int32_t)rnd(6) - 1; ++es; }
    for (int t = (int)rnd(3); t > 0; --t) { ak[ea] = (int32_t)rnd((uint32_t)K + 1) - 1; av[ea] = (int32_t)rnd(6) - 1; ++ea; }
    so[p + 1] = es; ao[p + 1] = ea;
  }
  u64* M = malloc(sizeof(u64) * (size_t)(n * W + 1));
  u64* sel = malloc(sizeof(u64) * (size_t)(P * W + 1));
  u64* alw = malloc(sizeof(u64) * (size_t)(P * W + 1));
  if (oracle_build(n, K, lab_off, lab_key, lab_val, P, so, sk, sv, ao, ak, av, M, sel, alw)) return 1;
  /* per-container lists (transpose of the select sets) */
  int64_t* loff = calloc((size_t)n + 1, sizeof(int64_t));
  int32_t* lst = malloc(sizeof(int32_t) * (size_t)(n * P + 1));
  if (oracle_lists(n, P, sel, loff, NULL)) return 2;   /* offsets, then the lists */
  if (oracle_lists(n, P, sel, loff, lst)) return 2;
  uint8_t *reach = malloc((size_t)n + 1), *isol = malloc((size_t)n + 1), *cross = malloc((size_t)n + 1);
  if (oracle_column_checks(n, M, 0, n, reach, isol)) return 3;
  int32_t* gid = malloc(sizeof(int32_t) * (size_t)(n + 1));
  for (int64_t i = 0; i < n; ++i) gid[i] = (int32_t)rnd(3);
  if (oracle_crosscheck(n, M, gid, 0, n, cross)) return 4;
  int64_t cnt = 0;
  int32_t* out = malloc(sizeof(int32_t) * 2 * 1000);
  if (oracle_shadow(n, n, loff, lst, alw, 0, n, 1000, out, &cnt)) return 5;
  u64* Pm = malloc(sizeof(u64) * (size_t)(n * W + 1));
  (void)oracle_path(n, W, M, 2, Pm);
  printf("n=%lld P=%lld shadow=%lld\n", (long long)n, (long long)P, (long long)cnt);
  free(lab_off); free(lab_key); free(lab_val); free(so); free(ao); free(sk); free(sv); free(ak);
  free(av); free(M); free(sel); free(alw); free(loff); free(lst); free(reach); free(isol);
  free(cross); free(gid); free(out); free(Pm);
  return 0;
}

int main(void) {
  const int64_t cases[][3] = {{1, 1, 1}, {5, 4, 2}, {63, 10, 3}, {64, 7, 4}, {65, 20, 3}, {300, 40, 5}};
  for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
    const int rc = run(cases[c][0], cases[c][1], cases[c][2]);
    if (rc) { printf("case %zu failed rc=%d\n", c, rc); return rc; }
  }
  printf("oracle sanitizer run clean\n");
  return 0;
}
