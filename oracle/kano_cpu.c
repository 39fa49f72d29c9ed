/*
 * kano_cpu.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py's
 * cpu_baseline leg.  The reference's reachability build and checks
 * (kano_py, the same per-element work as oracle/kano_oracle.c, which follows
 * kano_py's loops one for one) spread over the host's cores with OpenMP, so
 * that the whole benchmark cluster is timed instead of extrapolated from a
 * sample.  Results are the reference's (tests/test_cpu_baseline.py checks
 * them against the single-threaded oracle and bench.py against kano_py's
 * golden record of the cluster).  The product never links or calls it.
 *
 *   cpu_build          kano_py/kano/model.py:125-165   (policies in parallel:
 *                      presence AND + predicate refine per policy, model.py
 *                      :136-156; then matrix[idx] |= allow_set, :158-160, with
 *                      the words split across threads -- OR is order-free)
 *   cpu_col_reduce     kano_py/kano/algorithm.py:4-17  (getcol + count per
 *                      column; the 64 getcols of one word column share a
 *                      pass over the rows; all_reachable and all_isolated
 *                      each make their own pass, as the reference does)
 *   cpu_crosscheck     kano_py/kano/algorithm.py:20-42 (user_hashmap group
 *                      bitsets once, then getcol + ~group & col per column)
 *   cpu_shadow         kano_py/kano/algorithm.py:58-80 (containers in
 *                      parallel, pairs concatenated in container order)
 *
 * Bit sets are LSB-first uint64 words (bit j in word j>>6), W = ceil(n/64).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef uint64_t u64;

static inline int getbit(const u64* w, int64_t j) { return (int)((w[j >> 6] >> (j & 63)) & 1u); }
static inline void setbit(u64* w, int64_t j) { w[j >> 6] |= (u64)1 << (j & 63); }
static inline void clrbit(u64* w, int64_t j) { w[j >> 6] &= ~((u64)1 << (j & 63)); }

int cpu_threads(int want) {
  if (want > 0) omp_set_num_threads(want);
  int t = 1;
#pragma omp parallel
  {
#pragma omp single
    t = omp_get_num_threads();
  }
  return t;
}

/* model.py:95-111 on interned ids (as oracle/kano_oracle.c predicate) */
static int predicate(const int32_t* lk, const int32_t* lv, int64_t nl, const int32_t* tk,
                     const int32_t* tv, int64_t nt) {
  for (int64_t a = 0; a < nl; ++a)
    for (int64_t b = 0; b < nt; ++b)
      if (tk[b] == lk[a]) {
        if (tv[b] != lv[a] || lv[a] < 0) return 0;
        break;
      }
  return 1;
}

/* build_matrix: M[n*W], sel[P*W], alw[P*W] caller-allocated (written whole). */
int cpu_build(int64_t n, int64_t K, const int64_t* lab_off, const int32_t* lab_key,
              const int32_t* lab_val, int64_t P, const int64_t* ws_off, const int32_t* ws_key,
              const int32_t* ws_val, const int64_t* wa_off, const int32_t* wa_key,
              const int32_t* wa_val, u64* M, u64* sel, u64* alw) {
  const int64_t W = (n + 63) / 64;
  const u64 last = (n & 63) ? (((u64)1 << (n & 63)) - 1) : ~(u64)0;
  u64* labelMap = (u64*)calloc((size_t)(K > 0 ? K : 1) * (size_t)(W > 0 ? W : 1), sizeof(u64));
  if (!labelMap) return -1;
  /* model.py:131-133 */
  for (int64_t i = 0; i < n; ++i)
    for (int64_t a = lab_off[i]; a < lab_off[i + 1]; ++a) setbit(labelMap + lab_key[a] * W, i);
  /* model.py:135-156, one policy per iteration */
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t p = 0; p < P; ++p) {
    u64* ss = sel + p * W;
    u64* as = alw + p * W;
    for (int64_t w = 0; w < W; ++w) ss[w] = as[w] = ~(u64)0;
    if (W) { ss[W - 1] &= last; as[W - 1] &= last; }
    for (int64_t t = ws_off[p]; t < ws_off[p + 1]; ++t)
      if (ws_key[t] >= 0)
        for (int64_t w = 0; w < W; ++w) ss[w] &= labelMap[ws_key[t] * W + w];
    for (int64_t t = wa_off[p]; t < wa_off[p + 1]; ++t)
      if (wa_key[t] >= 0)
        for (int64_t w = 0; w < W; ++w) as[w] &= labelMap[wa_key[t] * W + w];
    for (int64_t idx = 0; idx < n; ++idx) {
      const int32_t* lk = lab_key + lab_off[idx];
      const int32_t* lv = lab_val + lab_off[idx];
      const int64_t nl = lab_off[idx + 1] - lab_off[idx];
      if (getbit(ss, idx) &&
          !predicate(lk, lv, nl, ws_key + ws_off[p], ws_val + ws_off[p], ws_off[p + 1] - ws_off[p]))
        clrbit(ss, idx);
      if (getbit(as, idx) &&
          !predicate(lk, lv, nl, wa_key + wa_off[p], wa_val + wa_off[p], wa_off[p + 1] - wa_off[p]))
        clrbit(as, idx);
    }
  }
  free(labelMap);
  /* model.py:158-160: matrix[idx] |= allow_set for idx in select_set, the
   * row words split across threads */
  const int64_t WB = 64;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t w0 = 0; w0 < W; w0 += WB) {
    const int64_t w1 = w0 + WB < W ? w0 + WB : W;
    for (int64_t i = 0; i < n; ++i) memset(M + i * W + w0, 0, sizeof(u64) * (size_t)(w1 - w0));
    for (int64_t p = 0; p < P; ++p) {
      const u64* ss = sel + p * W;
      const u64* as = alw + p * W;
      for (int64_t sw = 0; sw < W; ++sw) {
        u64 bits = ss[sw];
        while (bits) {
          const int64_t idx = sw * 64 + __builtin_ctzll(bits);
          bits &= bits - 1;
          u64* row = M + idx * W;
          for (int64_t w = w0; w < w1; ++w) row[w] |= as[w];
        }
      }
    }
  }
  return 0;
}

/* 64 x 64 bit transpose in place: afterwards a[k] bit r == (before) a[r]
 * bit k (block-swap recursion, as the engine's transpose32) */
static void transpose64(u64* a) {
  static const u64 mask[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                              0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
  for (int s = 0, j = 32; j; ++s, j >>= 1)
    for (int r = 0; r < 64; ++r) {
      if (r & j) continue;
      const u64 t = ((a[r] >> j) ^ a[r + j]) & mask[s];
      a[r + j] ^= t;
      a[r] ^= t << j;
    }
}

/* getcol (model.py:180-184) and its count, for the 512 columns of 8
 * consecutive word columns at once: 64 rows x 8 words (one cache line per
 * row) are read, transposed to 64-row pieces of each column, and each piece
 * goes to the caller's per-column fold -- every bit the reference's getcol
 * calls gather, in a cache- and TLB-friendly order. */
#define COLBLK 8
typedef void (*piece_fn)(int64_t col, int64_t q, u64 piece, void* st);

static void getcol_pieces(int64_t n, int64_t W, const u64* M, int64_t w0, piece_fn fn, void* st) {
  u64 blk[COLBLK][64];
  const int nw = (int)(W - w0 < COLBLK ? W - w0 : COLBLK);
  for (int64_t q = 0; q < W; ++q) {
    const int64_t i0 = q * 64;
    for (int r = 0; r < 64; ++r) {
      const u64* row = M + (i0 + r) * W + w0;
      for (int k = 0; k < COLBLK; ++k) blk[k][r] = (i0 + r < n && k < nw) ? row[k] : 0;
    }
    for (int k = 0; k < nw; ++k) {
      transpose64(blk[k]);
      for (int b = 0; b < 64; ++b) {
        const int64_t col = (w0 + k) * 64 + b;
        if (col < n) fn(col, q, blk[k][b], st);
      }
    }
  }
}

struct count_st { int64_t* cnt; int64_t base; };
static void count_piece(int64_t col, int64_t q, u64 piece, void* st) {
  (void)q;
  struct count_st* s = (struct count_st*)st;
  s->cnt[col - s->base] += __builtin_popcountll(piece);
}

/* all_reachable (mode 0: count == n) or all_isolated (mode 1: count == 0)
 * over every column: getcol then count, as the reference does per column
 * (each function makes its own pass).  flags[n]. */
int cpu_col_reduce(int64_t n, const u64* M, int mode, uint8_t* flags) {
  const int64_t W = (n + 63) / 64;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t w0 = 0; w0 < W; w0 += COLBLK) {
    int64_t cnt[64 * COLBLK];
    memset(cnt, 0, sizeof(cnt));
    struct count_st st = {cnt, w0 * 64};
    getcol_pieces(n, W, M, w0, count_piece, &st);
    for (int64_t c = 0; c < 64 * COLBLK && w0 * 64 + c < n; ++c)
      flags[w0 * 64 + c] = mode == 0 ? (cnt[c] == n) : (cnt[c] == 0);
  }
  return 0;
}

struct cross_st { const u64* grp; const int32_t* gid; int64_t W; u64* acc; int64_t base; };
static void cross_piece(int64_t col, int64_t q, u64 piece, void* st) {
  struct cross_st* s = (struct cross_st*)st;
  s->acc[col - s->base] |= ~s->grp[(int64_t)s->gid[col] * s->W + q] & piece;
}

/* user_crosscheck (algorithm.py:27-42): user_hashmap (:20-24) builds one
 * bitset per group; per column i, getcol(i) and any bit of ~group(g(i)) &
 * col.  gid in [0, G). */
int cpu_crosscheck(int64_t n, const u64* M, const int32_t* gid, uint8_t* flags) {
  const int64_t W = (n + 63) / 64;
  int32_t G = 0;
  for (int64_t i = 0; i < n; ++i) G = gid[i] + 1 > G ? gid[i] + 1 : G;
  u64* grp = (u64*)calloc((size_t)(G > 0 ? G : 1) * (size_t)(W > 0 ? W : 1), sizeof(u64));
  if (!grp) return -1;
  for (int64_t k = 0; k < n; ++k) setbit(grp + (int64_t)gid[k] * W, k);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t w0 = 0; w0 < W; w0 += COLBLK) {
    u64 acc[64 * COLBLK];
    memset(acc, 0, sizeof(acc));
    struct cross_st st = {grp, gid, W, acc, w0 * 64};
    getcol_pieces(n, W, M, w0, cross_piece, &st);
    for (int64_t c = 0; c < 64 * COLBLK && w0 * 64 + c < n; ++c) flags[w0 * 64 + c] = acc[c] != 0;
  }
  free(grp);
  return 0;
}

/* policy_shadow (algorithm.py:58-80): the per-container lists (CSR), the
 * allow sets; pairs in container order into out (capacity cap pairs),
 * *count = the full count. */
int cpu_shadow(int64_t n_lists, int64_t nbits, const int64_t* off, const int32_t* lst,
               const u64* allow, int64_t cap, int32_t* out, int64_t* count) {
  const int64_t W = (nbits + 63) / 64;
  const int nt = cpu_threads(0);
  int64_t* tcount = (int64_t*)calloc((size_t)nt + 1, sizeof(int64_t));
  int32_t** tbuf = (int32_t**)calloc((size_t)nt, sizeof(int32_t*));
  int64_t* tcap = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
  if (!tcount || !tbuf || !tcap) return -1;
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num();
    int64_t cnt = 0;
    /* contiguous container ranges per thread: concatenation keeps the order */
    const int64_t c0 = n_lists * t / nt, c1 = n_lists * (t + 1) / nt;
    for (int64_t i = c0; i < c1; ++i)
      for (int64_t a = off[i]; a < off[i + 1]; ++a)
        for (int64_t b = off[i]; b < off[i + 1]; ++b) {
          const int32_t j = lst[a], k = lst[b];
          if (j == k) continue;
          const u64* aj = allow + (int64_t)j * W;
          const u64* ak = allow + (int64_t)k * W;
          int64_t c = 0; /* ((j_allow & k_allow) ^ k_allow).count() */
          for (int64_t w = 0; w < W; ++w) c += __builtin_popcountll((aj[w] & ak[w]) ^ ak[w]);
          if (c == 0) {
            if (cnt == tcap[t]) {
              tcap[t] = tcap[t] ? 2 * tcap[t] : 4096;
              tbuf[t] = (int32_t*)realloc(tbuf[t], sizeof(int32_t) * 2 * (size_t)tcap[t]);
            }
            tbuf[t][2 * cnt] = j;
            tbuf[t][2 * cnt + 1] = k;
            ++cnt;
          }
        }
    tcount[t + 1] = cnt;
  }
  for (int t = 0; t < nt; ++t) tcount[t + 1] += tcount[t];
  for (int t = 0; t < nt; ++t) {
    const int64_t c = tcount[t + 1] - tcount[t];
    for (int64_t q = 0; q < c; ++q)
      if (tcount[t] + q < cap && out) {
        out[2 * (tcount[t] + q)] = tbuf[t][2 * q];
        out[2 * (tcount[t] + q) + 1] = tbuf[t][2 * q + 1];
      }
    free(tbuf[t]);
  }
  *count = tcount[nt];
  free(tcount);
  free(tbuf);
  free(tcap);
  return 0;
}

/* Container.select_policies (model.py:161): the build appends p to the list
 * of every container it selects, policies in order -- ascending ids per
 * container.  off[n+1] then list (two calls; set bits only). */
int cpu_lists(int64_t n, int64_t P, const u64* sets, int64_t* off, int32_t* list) {
  const int64_t W = (n + 63) / 64;
  if (!list) {
    memset(off, 0, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t p = 0; p < P; ++p)
      for (int64_t w = 0; w < W; ++w)
        for (u64 b = sets[p * W + w]; b; b &= b - 1) off[w * 64 + __builtin_ctzll(b) + 1] += 1;
    for (int64_t i = 0; i < n; ++i) off[i + 1] += off[i];
    return 0;
  }
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!cur) return -1;
  memcpy(cur, off, sizeof(int64_t) * (size_t)n);
  for (int64_t p = 0; p < P; ++p)
    for (int64_t w = 0; w < W; ++w)
      for (u64 b = sets[p * W + w]; b; b &= b - 1) list[cur[w * 64 + __builtin_ctzll(b)]++] = (int32_t)p;
  free(cur);
  return 0;
}
