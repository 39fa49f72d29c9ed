/*
 * kano_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's reachability build and checks, used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker.
 * The product (kubernetes-verification_amd/) never links or calls it.
 *
 * It follows the reference's loops one for one, on interned integers instead
 * of Python objects (values are equality classes of Python ==, see
 * oracle/kano_oracle.py):
 *   build_matrix      kano_py/kano/model.py:125-165
 *   select_policy /   kano_py/kano/model.py:95-111
 *   allow_policy
 *   getcol            kano_py/kano/model.py:180-184
 *   all_reachable     kano_py/kano/algorithm.py:4-9
 *   all_isolated      kano_py/kano/algorithm.py:12-17
 *   user_crosscheck   kano_py/kano/algorithm.py:20-42
 *   system_isolation  kano_py/kano/algorithm.py:45-55
 *   policy_shadow     kano_py/kano/algorithm.py:58-80
 * Parity of this restatement is pinned by tests/golden/ (vectors produced by
 * running kano_py itself, tests/golden/make_golden.py).
 *
 * Bit sets are LSB-first uint64 words (bit j in word j>>6), W = ceil(n/64).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;

static inline int getbit(const u64* w, int64_t j) { return (int)((w[j >> 6] >> (j & 63)) & 1u); }
static inline void setbit(u64* w, int64_t j, int v) {
  if (v) w[j >> 6] |= (u64)1 << (j & 63);
  else   w[j >> 6] &= ~((u64)1 << (j & 63));
}

/* The per-container predicate (model.py:95-111): iterate the CONTAINER's
 * labels; a label whose key is in the working dict must match its rule. */
static int predicate(const int32_t* lk, const int32_t* lv, int64_t nl,
                     const int32_t* tk, const int32_t* tv, int64_t nt) {
  for (int64_t a = 0; a < nl; ++a) {
    for (int64_t b = 0; b < nt; ++b) {
      if (tk[b] == lk[a]) {               /* k in sl.keys() */
        if (tv[b] != lv[a] || lv[a] < 0)  /* not matcher.match(sl[k], v) */
          return 0;
        break;
      }
    }
  }
  return 1;
}

/*
 * build_matrix.  Inputs:
 *   lab_off[n+1], lab_key[], lab_val[]   container labels (key ids 0..K-1)
 *   ws_*, wa_*                            working selector / allow terms per
 *                                         policy; key -1 = key carried by no
 *                                         container (dropped by the presence
 *                                         loop, model.py:143,146)
 * Outputs (caller-allocated, zeroed here): M[n*W], sel[P*W], alw[P*W]
 * (sel/alw may be NULL).
 */
int oracle_build(int64_t n, int64_t K, const int64_t* lab_off, const int32_t* lab_key,
                 const int32_t* lab_val, int64_t P, const int64_t* ws_off, const int32_t* ws_key,
                 const int32_t* ws_val, const int64_t* wa_off, const int32_t* wa_key,
                 const int32_t* wa_val, u64* M, u64* sel_out, u64* alw_out) {
  const int64_t W = (n + 63) / 64;
  u64* labelMap = (u64*)calloc((size_t)(K > 0 ? K : 1) * (size_t)(W > 0 ? W : 1), sizeof(u64));
  u64* select_set = (u64*)malloc(sizeof(u64) * (size_t)(W > 0 ? W : 1));
  u64* allow_set = (u64*)malloc(sizeof(u64) * (size_t)(W > 0 ? W : 1));
  if (!labelMap || !select_set || !allow_set) {
    free(labelMap); free(select_set); free(allow_set);
    return -1;
  }
  memset(M, 0, sizeof(u64) * (size_t)(n * W));
  /* model.py:131-133 */
  for (int64_t i = 0; i < n; ++i)
    for (int64_t a = lab_off[i]; a < lab_off[i + 1]; ++a) setbit(labelMap + lab_key[a] * W, i, 1);

  for (int64_t p = 0; p < P; ++p) {
    /* model.py:136-139: setall(True) */
    for (int64_t w = 0; w < W; ++w) { select_set[w] = ~(u64)0; allow_set[w] = ~(u64)0; }
    if (n & 63) {
      select_set[W - 1] &= ((u64)1 << (n & 63)) - 1;
      allow_set[W - 1] &= ((u64)1 << (n & 63)) - 1;
    }
    /* model.py:142-147: AND the presence bitsets of known keys */
    for (int64_t t = ws_off[p]; t < ws_off[p + 1]; ++t)
      if (ws_key[t] >= 0)
        for (int64_t w = 0; w < W; ++w) select_set[w] &= labelMap[ws_key[t] * W + w];
    for (int64_t t = wa_off[p]; t < wa_off[p + 1]; ++t)
      if (wa_key[t] >= 0)
        for (int64_t w = 0; w < W; ++w) allow_set[w] &= labelMap[wa_key[t] * W + w];
    /* model.py:150-154: refine with the predicates */
    for (int64_t idx = 0; idx < n; ++idx) {
      const int32_t* lk = lab_key + lab_off[idx];
      const int32_t* lv = lab_val + lab_off[idx];
      const int64_t nl = lab_off[idx + 1] - lab_off[idx];
      if (getbit(select_set, idx) &&
          !predicate(lk, lv, nl, ws_key + ws_off[p], ws_val + ws_off[p], ws_off[p + 1] - ws_off[p]))
        setbit(select_set, idx, 0);
      if (getbit(allow_set, idx) &&
          !predicate(lk, lv, nl, wa_key + wa_off[p], wa_val + wa_off[p], wa_off[p + 1] - wa_off[p]))
        setbit(allow_set, idx, 0);
    }
    /* model.py:156 store_bcp */
    if (sel_out) memcpy(sel_out + p * W, select_set, sizeof(u64) * (size_t)W);
    if (alw_out) memcpy(alw_out + p * W, allow_set, sizeof(u64) * (size_t)W);
    /* model.py:158-160: matrix[idx] |= allow_set */
    for (int64_t idx = 0; idx < n; ++idx)
      if (getbit(select_set, idx))
        for (int64_t w = 0; w < W; ++w) M[idx * W + w] |= allow_set[w];
  }
  free(labelMap); free(select_set); free(allow_set);
  return 0;
}

/* Per-container lists appended by build (model.py:161,163): ascending p with
 * bit i of sets[p].  Two calls: off only (list == NULL), then fill. */
int oracle_lists(int64_t n, int64_t P, const u64* sets, int64_t* off, int32_t* list) {
  const int64_t W = (n + 63) / 64;
  if (!list) {
    memset(off, 0, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t p = 0; p < P; ++p)
      for (int64_t i = 0; i < n; ++i) off[i + 1] += getbit(sets + p * W, i);
    for (int64_t i = 0; i < n; ++i) off[i + 1] += off[i];
    return 0;
  }
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!cur) return -1;
  for (int64_t i = 0; i < n; ++i) cur[i] = off[i];
  for (int64_t p = 0; p < P; ++p)
    for (int64_t i = 0; i < n; ++i)
      if (getbit(sets + p * W, i)) list[cur[i]++] = (int32_t)p;
  free(cur);
  return 0;
}

/* getcol (model.py:180-184) */
static void getcol(int64_t n, const u64* M, int64_t j, u64* col) {
  const int64_t W = (n + 63) / 64;
  for (int64_t i = 0; i < n; ++i) setbit(col, i, getbit(M + i * W, j));
}

static int64_t count_bits(const u64* v, int64_t W) {
  int64_t c = 0;
  for (int64_t w = 0; w < W; ++w) c += __builtin_popcountll(v[w]);
  return c;
}

/* all_reachable / all_isolated (algorithm.py:4-17): flags[j] = 1 when column j
 * is all ones / all zeros.  cols_begin/cols_end bound the columns scanned (the
 * bench times a column sample). */
int oracle_column_checks(int64_t n, const u64* M, int64_t cols_begin, int64_t cols_end,
                         uint8_t* reach, uint8_t* isol) {
  const int64_t W = (n + 63) / 64;
  u64* col = (u64*)calloc((size_t)(W > 0 ? W : 1), sizeof(u64));
  if (!col) return -1;
  for (int64_t j = cols_begin; j < cols_end; ++j) {
    getcol(n, M, j, col);
    const int64_t c = count_bits(col, W);
    if (reach) reach[j] = (c == n);
    if (isol) isol[j] = (c == 0);
  }
  free(col);
  return 0;
}

/* user_crosscheck (algorithm.py:27-42): gid[i] = user group of container i.
 * flags[i] = (~user_map[g(i)] & getcol(i)).count() != 0 */
int oracle_crosscheck(int64_t n, const u64* M, const int32_t* gid, int64_t cols_begin,
                      int64_t cols_end, uint8_t* flags) {
  const int64_t W = (n + 63) / 64;
  u64* col = (u64*)calloc((size_t)(W > 0 ? W : 1), sizeof(u64));
  u64* grp = (u64*)calloc((size_t)(W > 0 ? W : 1), sizeof(u64));
  if (!col || !grp) { free(col); free(grp); return -1; }
  for (int64_t i = cols_begin; i < cols_end; ++i) {
    /* user_hashmap bitset of g(i) (algorithm.py:20-24) */
    memset(grp, 0, sizeof(u64) * (size_t)W);
    for (int64_t k = 0; k < n; ++k)
      if (gid[k] == gid[i]) setbit(grp, k, 1);
    getcol(n, M, i, col);
    int64_t c = 0;
    for (int64_t w = 0; w < W; ++w) c += __builtin_popcountll(~grp[w] & col[w]);
    flags[i] = c != 0;
  }
  free(col); free(grp);
  return 0;
}

/* policy_shadow (algorithm.py:58-80) over per-container lists (CSR) and the
 * policies' allow sets.  Writes up to cap pairs, returns the full count in
 * *count.  Containers [c_begin, c_end) only (the bench times a sample). */
int oracle_shadow(int64_t n_lists, int64_t nbits, const int64_t* off, const int32_t* lst,
                  const u64* allow, int64_t c_begin, int64_t c_end, int64_t cap, int32_t* out,
                  int64_t* count) {
  const int64_t W = (nbits + 63) / 64;
  int64_t cnt = 0;
  (void)n_lists;
  for (int64_t i = c_begin; i < c_end; ++i) {
    for (int64_t a = off[i]; a < off[i + 1]; ++a) {
      for (int64_t b = off[i]; b < off[i + 1]; ++b) {
        const int32_t j = lst[a], k = lst[b];
        if (j == k) continue;
        const u64* aj = allow + (int64_t)j * W;
        const u64* ak = allow + (int64_t)k * W;
        int64_t c = 0; /* ((j_allow & k_allow) ^ k_allow).count() */
        for (int64_t w = 0; w < W; ++w) c += __builtin_popcountll((aj[w] & ak[w]) ^ ak[w]);
        if (c == 0) {
          if (cnt < cap && out) { out[2 * cnt] = j; out[2 * cnt + 1] = k; }
          ++cnt;
        }
      }
    }
  }
  *count = cnt;
  return 0;
}

/*
 * Multi-hop reachability: kubesv's `path` relation,
 *   path(src, dst) :- edge(src, dst).
 *   path(src, dst) :- edge(src, sel), edge(sel, dst).
 * (kubesv/kubesv/constraint.py:233-237), over kano's matrix as `edge`.
 * hops = 2 is that rule: P = M | M.M.  hops = k >= 1 extends it to paths of
 * at most k edges, hops = 0 to the transitive closure M+ (any length >= 1).
 * Row i after step k: P_k[i] = M[i] | OR_{j in P_{k-1}[i]} M[j], P_1 = M,
 * iterated until k = hops or nothing changes.  M and P are n rows of W words.
 * Returns the number of composition steps that changed some row.
 */
int64_t oracle_path(int64_t n, int64_t W, const u64* M, int64_t hops, u64* P) {
  u64* cur = (u64*)malloc(sizeof(u64) * (size_t)(n * W + 1));
  if (!cur) return -1;
  memcpy(P, M, sizeof(u64) * (size_t)(n * W));
  int64_t steps = 0;
  for (int64_t k = 2; hops == 0 || k <= hops; ++k) {
    memcpy(cur, P, sizeof(u64) * (size_t)(n * W));
    int changed = 0;
    for (int64_t i = 0; i < n; ++i) {
      u64* out = P + i * W;
      const u64* ri = cur + i * W;
      for (int64_t j = 0; j < n; ++j) {
        if (!getbit(ri, j)) continue;          /* edge / path (i, j) */
        const u64* mj = M + j * W;             /* edge (j, dst) */
        for (int64_t w = 0; w < W; ++w) out[w] |= mj[w];
      }
      for (int64_t w = 0; w < W; ++w) changed |= out[w] != ri[w];
    }
    if (!changed) break;
    ++steps;
  }
  free(cur);
  return steps;
}
