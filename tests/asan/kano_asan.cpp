// Host sanitizer run of the engine ("build host code with
// ASan/UBSan in CPU tests"): the C ABI of libkano_hip driven end to end with
// the host side built -fsanitize=address,undefined (device code unchanged:
// -Xarch_host), on a seeded cluster, against a naive restatement of
// build_matrix and the checks (kano_py/kano/model.py:125-165,
// algorithm.py:4-55) over the interned tables, plus the ABI's error paths,
// row shards with the combine, incremental updates and row digests.
// Exit 0 clean, 77 without a device, 1 on a wrong result; the sanitizers
// abort on a memory or UB error.  Built by __graft_entry__.build().
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "kano_hip.h"

typedef uint64_t u64;
static int fails = 0;
static kano_ctx* g_ctx = nullptr;   // the main context: its last error goes with a failure
#define CHECK(c)                                                                    \
  do {                                                                              \
    if (!(c)) {                                                                     \
      std::printf("FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, #c,       \
                  g_ctx ? kano_last_error(g_ctx) : "");                             \
      ++fails;                                                                      \
    }                                                                               \
  } while (0)

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(uint32_t m) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (uint32_t)(rs % m);
}

struct Cluster {
  int64_t n = 0, P = 0;
  int32_t ncols = 0;
  std::vector<int32_t> pv;                    // ncols x n, -1 absent
  std::vector<int64_t> so, ao;
  std::vector<int32_t> sc, sv, ac, av;
};

static Cluster make(int64_t n, int64_t P, int32_t ncols) {
  Cluster c;
  c.n = n;
  c.P = P;
  c.ncols = ncols;
  c.pv.resize((size_t)(ncols * n));
  for (int32_t k = 0; k < ncols; ++k)
    for (int64_t i = 0; i < n; ++i) c.pv[(size_t)(k * n + i)] = rnd(5) == 0 ? -1 : (int32_t)rnd(6);
  c.so.push_back(0);
  c.ao.push_back(0);
  for (int64_t p = 0; p < P; ++p) {
    for (int t = (int)rnd(3); t > 0; --t) {
      c.sc.push_back((int32_t)rnd(ncols));
      c.sv.push_back((int32_t)rnd(6));
    }
    for (int t = (int)rnd(3); t > 0; --t) {
      c.ac.push_back((int32_t)rnd(ncols));
      c.av.push_back((int32_t)rnd(6));
    }
    c.so.push_back((int64_t)c.sc.size());
    c.ao.push_back((int64_t)c.ac.size());
  }
  return c;
}

// model.py:95-111, 142-154 on interned ids: every term (col, val) equal
static bool match(const Cluster& c, const std::vector<int64_t>& off, const std::vector<int32_t>& col,
                  const std::vector<int32_t>& val, int64_t p, int64_t i) {
  for (int64_t t = off[(size_t)p]; t < off[(size_t)p + 1]; ++t)
    if (c.pv[(size_t)(col[(size_t)t] * c.n + i)] != val[(size_t)t]) return false;
  return true;
}

// M[i] = OR over p with sel_p(i) of allow_p (model.py:158-160), P policies
static std::vector<u64> naive_matrix(const Cluster& c, int64_t P) {
  const int64_t W = (c.n + 63) / 64;
  std::vector<u64> M((size_t)(c.n * W), 0), allow((size_t)(P * W), 0);
  for (int64_t p = 0; p < P; ++p)
    for (int64_t j = 0; j < c.n; ++j)
      if (match(c, c.ao, c.ac, c.av, p, j)) allow[(size_t)(p * W + j / 64)] |= 1ull << (j % 64);
  for (int64_t i = 0; i < c.n; ++i)
    for (int64_t p = 0; p < P; ++p)
      if (match(c, c.so, c.sc, c.sv, p, i))
        for (int64_t w = 0; w < W; ++w) M[(size_t)(i * W + w)] |= allow[(size_t)(p * W + w)];
  return M;
}

static bool bit(const std::vector<u64>& M, int64_t W, int64_t i, int64_t j) {
  return (M[(size_t)(i * W + j / 64)] >> (j % 64)) & 1u;
}

static int upload(kano_ctx* ctx, const Cluster& c) {
  int rc = kano_set_pods(ctx, c.n, c.ncols, c.pv.data());
  if (rc) return rc;
  return kano_set_policies(ctx, c.P, c.so.data(), c.sc.data(), c.sv.data(), c.ao.data(),
                           c.ac.data(), c.av.data());
}

int main() {
  kano_ctx* ctx = nullptr;
  int rc = kano_create(0, &ctx);
  if (rc == -ENODEV) {
    std::printf("no HIP device: skipped\n");
    return 77;
  }
  if (rc) {
    std::printf("kano_create rc=%d\n", rc);
    return 1;
  }
  g_ctx = ctx;
  const Cluster c = make(3000, 300, 3);
  const int64_t n = c.n, W = (n + 63) / 64;
  std::vector<int32_t> gid((size_t)n);
  for (int64_t i = 0; i < n; ++i) gid[(size_t)i] = (int32_t)rnd(4);
  CHECK(upload(ctx, c) == 0);
  CHECK(kano_set_groups(ctx, gid.data(), 0) == 0);
  const std::vector<u64> M = naive_matrix(c, c.P);

  // kano_verify: build + every check
  std::vector<int32_t> idx((size_t)(4 * n));
  std::vector<int32_t> pairs(2 * 4000000);
  int64_t counts[4] = {0, 0, 0, 0}, shadow = 0;
  rc = kano_verify(ctx, KANO_PATH_AUTO, gid.data(), 0, 0, idx.data(), counts, pairs.data(),
                   4000000, &shadow);
  CHECK(rc == 0);
  std::vector<u64> rows((size_t)(n * W));
  CHECK(kano_get_rows(ctx, 0, n, rows.data()) == 0);
  CHECK(rows == M);
  // all_reachable / all_isolated / user_crosscheck / system_isolation(0)
  std::vector<int32_t> reach, isol, cross, sys;
  for (int64_t j = 0; j < n; ++j) {
    bool all = true, none = true, cr = false;
    for (int64_t i = 0; i < n; ++i) {
      const bool b = bit(M, W, i, j);
      all &= b;
      none &= !b;
      cr |= b && gid[(size_t)i] != gid[(size_t)j];
    }
    if (all) reach.push_back((int32_t)j);
    if (none) isol.push_back((int32_t)j);
    if (cr) cross.push_back((int32_t)j);
    if (!bit(M, W, 0, j)) sys.push_back((int32_t)j);
  }
  size_t o = 0;
  for (const auto* want : {&reach, &isol, &cross, &sys}) {
    const int r = (int)(want == &reach ? 0 : want == &isol ? 1 : want == &cross ? 2 : 3);
    CHECK(counts[r] == (int64_t)want->size());
    if (counts[r] == (int64_t)want->size() && !want->empty())
      CHECK(std::memcmp(idx.data() + o, want->data(), sizeof(int32_t) * want->size()) == 0);
    o += (size_t)std::max<int64_t>(counts[r], 0);
  }
  // count-only policy_shadow gives the same count
  int64_t shadow2 = -1;
  CHECK(kano_verify(ctx, KANO_PATH_MFMA, gid.data(), 0, 0, idx.data(), counts, nullptr, -1,
                    &shadow2) == 0);
  CHECK(shadow2 == shadow);
  CHECK(kano_shadow_fetch(ctx, pairs.data()) != 0);   // no pairs after a count-only pass
  std::vector<u64> dig((size_t)n);
  CHECK(kano_rows_digest(ctx, 0, n, dig.data()) == 0);

  // pipelined calls (page-locked results: the direct tail, where the next
  // call's prologue is queued behind its gate), then a matrix read (unprime)
  {
    void* pidx = nullptr;
    void* ppairs = nullptr;
    CHECK(kano_host_alloc(sizeof(int32_t) * (size_t)(4 * n), &pidx) == 0);
    CHECK(kano_host_alloc(sizeof(int32_t) * 2 * (size_t)4000000, &ppairs) == 0);
    CHECK(kano_set_pipeline(ctx, 1) == 0);
    for (int rep = 0; rep < 3; ++rep) {
      int64_t cnt2[4] = {0, 0, 0, 0}, sh2 = -1;
      CHECK(kano_verify(ctx, KANO_PATH_AUTO, gid.data(), 0, 0, static_cast<int32_t*>(pidx), cnt2,
                        static_cast<int32_t*>(ppairs), 4000000, &sh2) == 0);
      CHECK(sh2 == shadow);
      CHECK((int64_t)isol.size() == cnt2[1]);
    }
    CHECK(kano_get_rows(ctx, 0, n, rows.data()) == 0);
    CHECK(rows == M);
    CHECK(kano_verify(ctx, KANO_PATH_AUTO, gid.data(), 0, 0, static_cast<int32_t*>(pidx), counts,
                      static_cast<int32_t*>(ppairs), 4000000, &shadow2) == 0);
    CHECK(kano_settle(ctx) == 0);
    CHECK(kano_set_pipeline(ctx, 0) == 0);
    kano_host_free(pidx);
    kano_host_free(ppairs);
  }

  // error paths: every one returns an error code, none faults
  CHECK(kano_get_rows(ctx, n - 1, 2, rows.data()) == -EINVAL);
  CHECK(kano_get_rows(ctx, -1, 1, rows.data()) == -EINVAL);
  CHECK(kano_verify(ctx, KANO_PATH_AUTO, nullptr, 0, 0, idx.data(), nullptr, nullptr, 0,
                    nullptr) == -EINVAL);
  CHECK(kano_verify(ctx, 7, nullptr, 0, 0, idx.data(), counts, nullptr, 0, nullptr) != 0);
  int64_t bad = c.P + 5;
  CHECK(kano_remove_policies(ctx, 1, &bad) == -EINVAL);
  CHECK(kano_set_shard(ctx, 5, 2) != 0);
  CHECK(kano_rows_digest(ctx, 0, n + 1, dig.data()) == -EINVAL);
  CHECK(std::strlen(kano_last_error(ctx)) > 0);
  std::vector<int32_t> badg(gid);
  badg[7] = -2;
  CHECK(kano_set_groups(ctx, badg.data(), 0) == -EINVAL);

  // incremental: remove the first 10 policies, then the naive matrix over
  // the rest; add one back
  std::vector<int64_t> gone;
  for (int64_t p = 0; p < 10; ++p) gone.push_back(p);
  CHECK(kano_remove_policies(ctx, (int64_t)gone.size(), gone.data()) == 0);
  {
    Cluster k = c;   // the kept policies
    k.so.assign(1, 0);
    k.ao.assign(1, 0);
    k.sc.clear(); k.sv.clear(); k.ac.clear(); k.av.clear();
    for (int64_t p = 10; p < c.P; ++p) {
      for (int64_t t = c.so[(size_t)p]; t < c.so[(size_t)p + 1]; ++t) {
        k.sc.push_back(c.sc[(size_t)t]);
        k.sv.push_back(c.sv[(size_t)t]);
      }
      for (int64_t t = c.ao[(size_t)p]; t < c.ao[(size_t)p + 1]; ++t) {
        k.ac.push_back(c.ac[(size_t)t]);
        k.av.push_back(c.av[(size_t)t]);
      }
      k.so.push_back((int64_t)k.sc.size());
      k.ao.push_back((int64_t)k.ac.size());
    }
    k.P = c.P - 10;
    CHECK(kano_get_rows(ctx, 0, n, rows.data()) == 0);
    CHECK(rows == naive_matrix(k, k.P));
  }

  // row shards on this device: verify_shard into one gathered buffer, then
  // each shard's combine gives the whole-matrix lists
  {
    const int N = 3;
    u64* g = nullptr;
    CHECK(hipMalloc(&g, sizeof(u64) * 3 * W * N) == hipSuccess);
    std::vector<kano_ctx*> sh(N, nullptr);
    for (int r = 0; r < N; ++r) {
      CHECK(kano_create(0, &sh[(size_t)r]) == 0);
      CHECK(upload(sh[(size_t)r], c) == 0);
      CHECK(kano_set_shard(sh[(size_t)r], r * n / N, (r + 1) * n / N) == 0);
      CHECK(kano_verify_shard(sh[(size_t)r], KANO_PATH_AUTO, gid.data(), 0, 0, 1,
                              g + (size_t)(3 * W * r)) == 0);
    }
    CHECK(hipDeviceSynchronize() == hipSuccess);
    int64_t total = 0;
    for (int r = 0; r < N; ++r) {
      int64_t cnt[4], s = 0;
      CHECK(kano_verify_combine(sh[(size_t)r], g, N, idx.data(), cnt, pairs.data(), 4000000,
                                &s) == 0);
      CHECK(cnt[0] == (int64_t)reach.size() && cnt[1] == (int64_t)isol.size() &&
            cnt[2] == (int64_t)cross.size());
      CHECK(r == 0 ? cnt[3] == (int64_t)sys.size() : cnt[3] == -1);
      std::vector<u64> d((size_t)(n / N + 2));
      const int64_t r0 = r * n / N, r1 = (r + 1) * n / N;
      CHECK(kano_rows_digest(sh[(size_t)r], r0, r1 - r0, d.data()) == 0);
      CHECK(std::memcmp(d.data(), dig.data() + r0, sizeof(u64) * (size_t)(r1 - r0)) == 0);
      total += s;
      kano_destroy(sh[(size_t)r]);
    }
    CHECK(total == shadow);
    (void)hipFree(g);
  }
  // one process over two members on this device (kano_group: persistent
  // member threads, device-copy exchange): upload, stored groups, verify
  {
    kano_group* g = nullptr;
    const int devs[2] = {0, 0};
    CHECK(kano_group_create(2, devs, &g) == 0);
    const int64_t half = ((W / 2) * 64 < n) ? (W / 2) * 64 : n;
    const int64_t bounds[4] = {0, half, half, n};
    CHECK(kano_group_upload(g, c.n, c.ncols, c.pv.data(), 0, nullptr, nullptr, nullptr, nullptr,
                            c.P, c.so.data(), c.sc.data(), c.sv.data(), c.ao.data(), c.ac.data(),
                            c.av.data(), bounds) == 0);
    CHECK(kano_group_set_groups(g, gid.data(), 0) == 0);
    for (int rep = 0; rep < 2; ++rep) {
      int64_t cnt[4], s = 0;
      CHECK(kano_group_verify(g, KANO_PATH_AUTO, nullptr, KANO_STORED_GROUPS, 0, 1, idx.data(),
                              cnt, pairs.data(), 4000000, &s) == 0);
      CHECK(cnt[0] == (int64_t)reach.size() && cnt[1] == (int64_t)isol.size() &&
            cnt[2] == (int64_t)cross.size() && cnt[3] == (int64_t)sys.size());
      CHECK(s == shadow);
    }
    CHECK(kano_group_build(g, KANO_PATH_BITWISE) == 0);
    // a failing upload (a term column past the table) reports, destroys once
    std::vector<int32_t> badc(c.sc);
    if (!badc.empty()) badc[0] = c.ncols + 3;
    CHECK(kano_group_upload(g, c.n, c.ncols, c.pv.data(), 0, nullptr, nullptr, nullptr, nullptr,
                            c.P, c.so.data(), badc.data(), c.sv.data(), c.ao.data(), c.ac.data(),
                            c.av.data(), bounds) != 0);
    CHECK(std::strlen(kano_group_last_error(g)) > 0);
    kano_group_destroy(g);
  }
  g_ctx = nullptr;
  kano_destroy(ctx);
  std::printf("%s: %d failed checks, shadow pairs %lld\n", fails ? "FAIL" : "ok", fails,
              (long long)shadow);
  std::fflush(stdout);
  // End without the runtime's static teardown: ASan's quarantine (kept on,
  // so freed host memory is poisoned and use-after-free is caught during
  // the run) would otherwise recycle HIP allocations from a runtime thread
  // after the HIP runtime has unloaded -- an allocator CHECK at exit, after
  // every check above has run.
  std::_Exit(fails ? 1 : 0);
}
