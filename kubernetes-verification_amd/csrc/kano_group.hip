// kano_group.hip -- one process over G devices (SURVEY.md §8(b) kano_init(ngpu),
// §8(e) row sharding; the C ABI of include/kano_hip.h, kano_group_*).
//
// A group owns G member contexts; member r holds rows [r0_r, r1_r) of M on
// device dev[r] with its own streams.  The build needs no communication
// (kano_py/kano/model.py:125-165 per row shard); the column checks
// (algorithm.py:4-42) exchange each member's [OR | cross | NAND] words
// (3 W u64): ncclAllGather over xGMI (communicators from ncclCommInitAll)
// when the G devices are distinct and RCCL loads, else device-to-device
// copies (G members on one device: the tests) -- and every member ORs the
// gathered words on its device (kano_verify_combine).
//
// Every member runs on its own persistent host thread (a worker per member,
// started with the group): a call hands the members one job and waits for
// them, so the members' uploads, builds, host syncs and result copies
// overlap and no thread is created per call.  A job with an exchange runs it
// between two worker barriers inside the same hand-off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "kano_hip.h"
#include "kano_internal.hpp"

using i64 = int64_t;
using u64 = uint64_t;

namespace {

using clk = std::chrono::steady_clock;

inline void cpu_relax() { __builtin_ia32_pause(); }

// G workers meet here; sense by generation
struct SpinBarrier {
  std::atomic<int> count{0};
  std::atomic<uint64_t> gen{0};
  int n = 1;
  void wait() {
    const uint64_t g = gen.load(std::memory_order_acquire);
    if (count.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
      count.store(0, std::memory_order_relaxed);
      gen.fetch_add(1, std::memory_order_acq_rel);
      return;
    }
    for (uint32_t s = 1; gen.load(std::memory_order_acquire) == g; ++s) {
      cpu_relax();
      if ((s & 0xffff) == 0) std::this_thread::yield();
    }
  }
};

// one persistent host thread per member
struct Pool {
  int G = 0;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint64_t> seq{0};
  std::atomic<int> pending{0};
  std::atomic<bool> quit{false};
  const std::function<int(int)>* job = nullptr;
  std::vector<int> rc;
  SpinBarrier bar;

  void worker(int r, int dev) {
    (void)hipSetDevice(dev);
    uint64_t seen = 0;
    for (;;) {
      // spin a little (back-to-back calls hand over within microseconds),
      // then sleep on the condition variable
      auto t0 = clk::now();
      uint64_t s;
      for (uint32_t k = 1; (s = seq.load(std::memory_order_acquire)) == seen &&
                           !quit.load(std::memory_order_acquire);
           ++k) {
        cpu_relax();
        if ((k & 0x3ff) == 0 && clk::now() - t0 > std::chrono::milliseconds(2)) {
          std::unique_lock<std::mutex> lk(mu);
          // (no timeout: run() and stop() change seq / quit under the mutex)
          cv.wait(lk, [&] { return seq.load(std::memory_order_acquire) != seen || quit.load(); });
          t0 = clk::now();
        }
      }
      if (quit.load(std::memory_order_acquire)) return;
      seen = s;
      rc[(size_t)r] = (*job)(r);
      pending.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  void start(const std::vector<int>& dev) {
    G = (int)dev.size();
    rc.assign((size_t)G, 0);
    bar.n = G;
    for (int r = 0; r < G; ++r) th.emplace_back(&Pool::worker, this, r, dev[(size_t)r]);
  }

  // run f(r) on every member's worker; returns when all are done
  void run(const std::function<int(int)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      job = &f;
      pending.store(G, std::memory_order_relaxed);
      seq.fetch_add(1, std::memory_order_acq_rel);
    }
    cv.notify_all();
    const auto t0 = clk::now();
    for (uint32_t k = 1; pending.load(std::memory_order_acquire) > 0; ++k) {
      cpu_relax();
      if ((k & 0xfff) == 0 && clk::now() - t0 > std::chrono::milliseconds(5))
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    job = nullptr;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit.store(true, std::memory_order_release);
    }
    cv.notify_all();
    for (auto& t : th)
      if (t.joinable()) t.join();
    th.clear();
  }
};

// RCCL's entry points, resolved at run time from the librccl already mapped
// into the process (torch's) or the system one; the types are rccl.h's own
struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok() const { return init_all && group_start && group_end && destroy && all_gather; }
  const char* what(ncclResult_t e) const {
    return error_string ? error_string(e) : "(no ncclGetErrorString)";
  }
};

template <typename F>
void resolve(F& f, const char* name) {
  f = reinterpret_cast<F>(kano_int::rccl_symbol(name));
}

const Rccl& rccl_syms() {
  static Rccl r = [] {
    Rccl x;
    resolve(x.init_all, "ncclCommInitAll");
    resolve(x.group_start, "ncclGroupStart");
    resolve(x.group_end, "ncclGroupEnd");
    resolve(x.destroy, "ncclCommDestroy");
    resolve(x.all_gather, "ncclAllGather");
    resolve(x.error_string, "ncclGetErrorString");
    return x;
  }();
  return r;
}

// why the last kano_group_create failed (no group to hold it):
// kano_group_last_error(NULL)
thread_local std::string g_create_err;

}  // namespace

struct kano_group {
  int G = 0;
  std::vector<int> dev;
  std::vector<kano_ctx*> m;
  int mode = 2;                       // 1 RCCL all-gather, 2 device copies
  std::vector<ncclComm_t> comms;
  std::vector<hipEvent_t> ev;         // a member's words are written
  std::vector<void*> xw, xg;          // members' exchange buffers (device)
  std::string err;
  std::vector<int32_t*> idx;          // per-member pinned scratch: 4n list entries
  std::vector<int32_t*> pairs;        // per-member pinned pairs
  std::vector<i64> pair_cap;
  i64 idx_n = -1;
  Pool pool;
  std::atomic<int> failed{0};         // a member's step failed (inside one job)
  // an update that reached some members and not others: the shards hold
  // different policy lists, so every later call refuses until a new upload
  std::string poisoned;
  // the verify exchange's time on member 0's stream (kano_group_exchange_timing)
  bool xtime_on = false;
  bool xtime_pending = false;
  hipEvent_t xt0 = nullptr, xt1 = nullptr;
  double xt_calls = 0, xt_sum = 0, xt_max = 0;
};

#define KANO_GROUP_TRY(expr) \
  do {                       \
    const int rc_ = (expr);  \
    if (rc_) return rc_;     \
  } while (0)

namespace {

int gfail(kano_group* g, int code, const std::string& msg) {
  g->err = msg;
  return code;
}

// calls on a group whose members diverged (a partial update) fail loudly
int group_usable(kano_group* g) {
  if (g->poisoned.empty()) return 0;
  return gfail(g, -EPROTO, g->poisoned + "; upload the tables again (kano_group_upload)");
}

// f(r) on every member's worker; the first error wins
int group_each(kano_group* g, const std::function<int(int)>& f) {
  g->failed.store(0);
  g->pool.run(f);
  // (the member whose step failed first, not the ones it cancelled)
  for (int pass = 0; pass < 2; ++pass)
    for (int r = 0; r < g->G; ++r) {
      const int rc = g->pool.rc[(size_t)r];
      if (rc && (pass == 1 || rc != -ECANCELED)) {
        const char* e = kano_last_error(g->m[(size_t)r]);
        return gfail(g, rc, "member " + std::to_string(r) + ": " + (e ? e : ""));
      }
    }
  return 0;
}

// inside a job: member s's nw words at send[s] (written on its stream) ->
// every member's recv[r] holds all of them, rank-major (send[s] may alias
// recv[s] + s nw: RCCL's in-place all-gather).  Called by every worker; the
// workers meet at the barriers even when one failed.  timed: the exchange is
// bracketed by g->xt0 / xt1 on member 0's stream.
int member_exchange(kano_group* g, int r, int rc, const std::vector<void*>& send,
                    const std::vector<void*>& recv, i64 nw, bool timed) {
  kano_ctx* c = g->m[(size_t)r];
  hipStream_t st = kano_int::ctx_stream(c);
  if (rc) g->failed.store(1);
  if (g->mode == 2 && !rc && nw > 0 && hipEventRecord(g->ev[(size_t)r], st) != hipSuccess) {
    g->failed.store(1);
    rc = kano_int::ctx_fail(c, -EIO, "recording the member's words event failed");
  }
  g->pool.bar.wait();
  if (g->failed.load()) return rc ? rc : -ECANCELED;
  // (the timing events live on member 0's device: kano_group_create makes
  // them there; a failed record leaves this call untimed, never half-timed)
  const bool timing = timed && r == 0 && nw > 0 && hipEventRecord(g->xt0, st) == hipSuccess;
  if (nw > 0 && g->mode == 1) {
    // one thread issues the grouped all-gather over every communicator
    if (r == 0) {
      const Rccl& R = rccl_syms();
      ncclResult_t e = R.group_start();
      for (int s = 0; e == ncclSuccess && s < g->G; ++s)
        e = R.all_gather(send[(size_t)s], recv[(size_t)s], (size_t)nw, ncclUint64,
                         g->comms[(size_t)s], kano_int::ctx_stream(g->m[(size_t)s]));
      const ncclResult_t e2 = R.group_end();
      if (e != ncclSuccess || e2 != ncclSuccess) {
        g->failed.store(1);
        rc = kano_int::ctx_fail(c, -EIO, std::string("ncclAllGather over the group failed: ") +
                                             R.what(e != ncclSuccess ? e : e2));
      }
    }
  } else if (nw > 0) {
    // device copies: this member pulls every other member's words onto its stream
    for (int s = 0; s < g->G && !rc; ++s) {
      void* dst = static_cast<u64*>(recv[(size_t)r]) + (i64)s * nw;
      if (dst == send[(size_t)s]) continue;
      if (hipStreamWaitEvent(st, g->ev[(size_t)s], 0) != hipSuccess ||
          hipMemcpyAsync(dst, send[(size_t)s], sizeof(u64) * nw, hipMemcpyDefault, st) !=
              hipSuccess) {
        g->failed.store(1);
        rc = kano_int::ctx_fail(c, -EIO, "the words' device copy failed");
      }
    }
  }
  if (timing && hipEventRecord(g->xt1, st) == hipSuccess) g->xtime_pending = true;
  g->pool.bar.wait();
  if (g->failed.load()) return rc ? rc : -ECANCELED;
  return 0;
}

// the last verify's exchange time, once its events are done
void exchange_time_collect(kano_group* g) {
  if (!g->xtime_pending) return;
  g->xtime_pending = false;
  float ms = 0.f;
  if (hipEventSynchronize(g->xt1) == hipSuccess &&
      hipEventElapsedTime(&ms, g->xt0, g->xt1) == hipSuccess) {
    g->xt_calls += 1;
    g->xt_sum += ms;
    g->xt_max = std::max<double>(g->xt_max, ms);
  }
}

int group_buffers(kano_group* g) {
  const i64 n = kano_int::ctx_n(g->m[0]);
  g->xw.assign((size_t)g->G, nullptr);
  g->xg.assign((size_t)g->G, nullptr);
  for (int r = 0; r < g->G; ++r) {
    kano_ctx* ctx = g->m[(size_t)r];
    if (kano_int::ctx_n(ctx) != n) return gfail(g, -EINVAL, "members hold different pod counts");
    if (kano_int::ctx_exchange_buffers(ctx, g->G, &g->xw[(size_t)r], &g->xg[(size_t)r]))
      return gfail(g, -ENOMEM, "member " + std::to_string(r) + ": " + kano_last_error(ctx));
  }
  if (g->idx_n != n) {
    for (auto p : g->idx) (void)hipHostFree(p);
    g->idx.assign((size_t)g->G, nullptr);
    for (int r = 0; r < g->G; ++r)
      if (hipHostMalloc(reinterpret_cast<void**>(&g->idx[(size_t)r]),
                        sizeof(int32_t) * (size_t)std::max<i64>(16, 4 * n)) != hipSuccess)
        return gfail(g, -ENOMEM, "pinned list buffers");
    g->idx_n = n;
  }
  if ((int)g->pairs.size() != g->G) {
    g->pairs.assign((size_t)g->G, nullptr);
    g->pair_cap.assign((size_t)g->G, 0);
  }
  return 0;
}

// the global lists from member 0, system_isolation from its owner
void group_lists(kano_group* g, const std::vector<std::array<int64_t, 4>>& cnt, int32_t* idx,
                 int64_t* counts) {
  i64 o = 0;
  for (int k = 0; k < 3; ++k) {
    const i64 c = cnt[0][(size_t)k];
    i64 src = 0;
    for (int q = 0; q < k; ++q) src += cnt[0][(size_t)q];
    if (c > 0) std::memcpy(idx + o, g->idx[0] + src, sizeof(int32_t) * (size_t)c);
    counts[k] = c;
    o += c;
  }
  counts[3] = -1;
  for (int r = 0; r < g->G; ++r) {
    const i64 c = cnt[(size_t)r][3];
    if (c < 0) continue;
    const i64 src = cnt[(size_t)r][0] + cnt[(size_t)r][1] + cnt[(size_t)r][2];
    if (c > 0) std::memcpy(idx + o, g->idx[(size_t)r] + src, sizeof(int32_t) * (size_t)c);
    counts[3] = c;
    break;
  }
}

// member r's page-locked pair buffer, at least cap pairs
int member_pairs(kano_group* g, int r, i64 cap) {
  if (g->pairs[(size_t)r] && g->pair_cap[(size_t)r] >= cap) return 0;
  if (g->pairs[(size_t)r]) (void)hipHostFree(g->pairs[(size_t)r]);
  g->pairs[(size_t)r] = nullptr;
  g->pair_cap[(size_t)r] = std::max<i64>(cap, 1 << 16);
  if (hipHostMalloc(reinterpret_cast<void**>(&g->pairs[(size_t)r]),
                    sizeof(int32_t) * 2 * (size_t)g->pair_cap[(size_t)r]) != hipSuccess) {
    g->pair_cap[(size_t)r] = 0;
    return kano_int::ctx_fail(g->m[(size_t)r], -ENOMEM, "pinned pair buffer");
  }
  return 0;
}

}  // namespace

static int group_create(int ngpu, const int* devices, int flags, kano_group** out);

extern "C" {

int kano_group_create(int ngpu, const int* devices, kano_group** out) {
  return group_create(ngpu, devices, 0, out);
}

int kano_group_create_lean(int ngpu, const int* devices, kano_group** out) {
  return group_create(ngpu, devices, KANO_GROUP_LEAN, out);
}

int kano_group_create_ex(int ngpu, const int* devices, int flags, kano_group** out) {
  return group_create(ngpu, devices, flags, out);
}

}  // extern "C"

static int create_fail(kano_group* g, int cur, int code, const std::string& msg) {
  g_create_err = msg;
  if (g) kano_group_destroy(g);
  (void)hipSetDevice(cur);
  return code;
}

static int group_create(int ngpu, const int* devices, int flags, kano_group** out) {
  g_create_err.clear();
  if (!out || ngpu < 1) {
    g_create_err = "kano_group_create: ngpu < 1 or out NULL";
    return -EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_create_err = "kano_group_create: no HIP device";
    return -ENODEV;
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  kano_group* g = new kano_group();
  g->G = ngpu;
  for (int r = 0; r < ngpu; ++r) {
    const int d = devices ? devices[r] : r;
    if (d < 0 || d >= ndev)
      return create_fail(g, cur, -EINVAL,
                         "kano_group_create: device " + std::to_string(d) + " of member " +
                             std::to_string(r) + " does not exist (" + std::to_string(ndev) +
                             " devices)");
    g->dev.push_back(d);
  }
  const bool lean = flags & KANO_GROUP_LEAN;
  // the member contexts, created at once by their own threads (a context's
  // streams, events and pinned buffers: ~7 ms each, serial for G members)
  g->pool.start(g->dev);
  g->m.assign((size_t)ngpu, nullptr);
  g->ev.assign((size_t)ngpu, nullptr);
  const std::function<int(int)> make = [g, lean](int r) -> int {
    kano_ctx* c = nullptr;
    const int rc = lean ? kano_create_lean(g->dev[(size_t)r], &c) : kano_create(g->dev[(size_t)r], &c);
    if (rc) return rc;
    g->m[(size_t)r] = c;
    return hipEventCreateWithFlags(&g->ev[(size_t)r], hipEventDisableTiming) == hipSuccess ? 0
                                                                                          : -EIO;
  };
  g->pool.run(make);
  for (int r = 0; r < ngpu; ++r)
    if (g->pool.rc[(size_t)r])
      return create_fail(g, cur, g->pool.rc[(size_t)r],
                         "kano_group_create: member " + std::to_string(r) + "'s context failed");
  // the exchange-timing events on member 0's device (they are recorded on its
  // stream), whatever the calling thread's current device
  if (hipSetDevice(g->dev[0]) != hipSuccess || hipEventCreate(&g->xt0) != hipSuccess ||
      hipEventCreate(&g->xt1) != hipSuccess)
    return create_fail(g, cur, -EIO, "kano_group_create: timing events");
  // the exchange: RCCL over xGMI (one communicator per device,
  // ncclCommInitAll) when the devices are distinct, or when asked for
  // (KANO_GROUP_RCCL: also one member, so that the transport runs on a
  // one-GPU box); device copies when members share a device or when asked
  // for (KANO_GROUP_COPY / env KANO_GROUP_COPY).  An RCCL that should run and
  // does not is an error, never a silent fall back to copies.
  std::vector<int> sorted(g->dev);
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  // (the environment is the Python layer's business: kano/multi.py passes
  // KANO_GROUP_COPY / KANO_GROUP_RCCL through the flags)
  const bool copy = flags & KANO_GROUP_COPY;
  const bool want = (flags & KANO_GROUP_RCCL) || (ngpu > 1 && distinct && !copy);
  if (want) {
    if (!distinct)
      return create_fail(g, cur, -EINVAL,
                         "kano_group_create: the RCCL exchange needs distinct devices");
    const Rccl& R = rccl_syms();
    if (!R.ok())
      return create_fail(g, cur, -ENOSYS,
                         "kano_group_create: RCCL is not loadable (librccl: ncclCommInitAll / "
                         "ncclAllGather missing); KANO_GROUP_COPY selects device copies");
    g->comms.assign((size_t)ngpu, nullptr);
    const ncclResult_t e = R.init_all(g->comms.data(), ngpu, g->dev.data());
    if (e != ncclSuccess) {
      g->comms.clear();
      return create_fail(g, cur, -EIO,
                         std::string("kano_group_create: ncclCommInitAll failed: ") + R.what(e) +
                             "; KANO_GROUP_COPY selects device copies");
    }
    g->mode = 1;
  }
  (void)hipSetDevice(cur);
  *out = g;
  return 0;
}

extern "C" {

void kano_group_destroy(kano_group* g) {
  if (!g) return;
  g->pool.stop();
  for (kano_ctx* c : g->m)
    if (c) kano_destroy(c);
  if (!g->comms.empty()) {
    const Rccl& R = rccl_syms();
    for (ncclComm_t c : g->comms)
      if (c && R.destroy) (void)R.destroy(c);
  }
  for (hipEvent_t e : g->ev)
    if (e) (void)hipEventDestroy(e);
  if (g->xt0) (void)hipEventDestroy(g->xt0);
  if (g->xt1) (void)hipEventDestroy(g->xt1);
  for (auto p : g->idx) (void)hipHostFree(p);
  for (auto p : g->pairs)
    if (p) (void)hipHostFree(p);
  delete g;
}

const char* kano_group_last_error(const kano_group* g) {
  return g ? g->err.c_str() : g_create_err.c_str();
}

int kano_group_info(kano_group* g, int32_t* out /* 2 */) {
  if (!g || !out) return -EINVAL;
  out[0] = g->G;
  out[1] = g->mode;
  return 0;
}

int kano_group_member(kano_group* g, int r, kano_ctx** ctx) {
  if (!g || !ctx || r < 0 || r >= g->G) return -EINVAL;
  *ctx = g->m[(size_t)r];
  return 0;
}

int kano_group_upload(kano_group* g, int64_t n, int32_t ncols, const int32_t* pod_val, int32_t E,
                      const int32_t* ecol, const int32_t* eop, const int64_t* eoff,
                      const int32_t* evals, int64_t P, const int64_t* sel_off,
                      const int32_t* sel_col, const int32_t* sel_val, const int64_t* alw_off,
                      const int32_t* alw_col, const int32_t* alw_val, const int64_t* bounds) {
  if (!g) return -EINVAL;
  if (!bounds) return gfail(g, -EINVAL, "kano_group_upload: bounds NULL");
  g->poisoned.clear();   // (every member's tables and policy list replaced)
  for (int r = 0; r < g->G; ++r)
    if (bounds[2 * r] < 0 || bounds[2 * r + 1] < bounds[2 * r] || bounds[2 * r + 1] > n)
      return gfail(g, -EINVAL, "kano_group_upload: bad row range of member " + std::to_string(r));
  return group_each(g, [&](int r) {
    kano_ctx* c = g->m[(size_t)r];
    int rc = kano_set_pods(c, n, ncols, pod_val);
    if (!rc && E > 0) rc = kano_set_expressions(c, E, ecol, eop, eoff, evals);
    if (!rc)
      rc = kano_set_policies(c, P, sel_off, sel_col, sel_val, alw_off, alw_col, alw_val);
    if (!rc) rc = kano_set_shard(c, bounds[2 * r], bounds[2 * r + 1]);
    return rc;
  });
}

int kano_group_build(kano_group* g, int path) {
  if (!g) return -EINVAL;
  KANO_GROUP_TRY(group_usable(g));
  return group_each(g, [&](int r) { return kano_build(g->m[(size_t)r], path); });
}

int kano_group_set_groups(kano_group* g, const int32_t* gid, int32_t ngroups) {
  if (!g) return -EINVAL;
  KANO_GROUP_TRY(group_usable(g));
  return group_each(g, [&](int r) { return kano_set_groups(g->m[(size_t)r], gid, ngroups); });
}

int kano_group_verify(kano_group* g, int path, const int32_t* gid, int32_t ngroups,
                      int64_t sys_row, int with_shadow, int32_t* idx, int64_t* counts,
                      int32_t* shadow_pairs, int64_t shadow_cap, int64_t* shadow_count) {
  if (!g) return -EINVAL;
  if (!counts || !idx) return gfail(g, -EINVAL, "kano_group_verify: idx / counts NULL");
  KANO_GROUP_TRY(group_usable(g));
  if (with_shadow && !shadow_count)
    return gfail(g, -EINVAL, "kano_group_verify: shadow_count NULL with with_shadow");
  KANO_GROUP_TRY(group_buffers(g));
  const bool count_only = with_shadow == 2;
  std::vector<std::array<int64_t, 4>> cnt((size_t)g->G);
  std::vector<int64_t> sc((size_t)g->G, 0);
  // one hand-off: every member's build and checks up to its column words,
  // the exchange between two worker barriers, then every member's combine
  // (the three global lists, its system row, its policy_shadow pairs)
  KANO_GROUP_TRY(group_each(g, [&](int r) {
    kano_ctx* c = g->m[(size_t)r];
    int rc = kano_verify_shard(c, path, gid, ngroups, sys_row, with_shadow,
                               static_cast<uint64_t*>(g->xw[(size_t)r]));
    rc = member_exchange(g, r, rc, g->xw, g->xg, 3 * kano_int::ctx_W(g->m[0]), g->xtime_on);
    if (rc) return rc;
    int32_t* pp = nullptr;
    i64 cap = -1;
    if (with_shadow && !count_only) {
      if (member_pairs(g, r, 0)) return -ENOMEM;
      pp = g->pairs[(size_t)r];
      cap = g->pair_cap[(size_t)r];
    }
    rc = kano_verify_combine(c, static_cast<const uint64_t*>(g->xg[(size_t)r]), g->G,
                             g->idx[(size_t)r], cnt[(size_t)r].data(), pp, cap,
                             with_shadow ? &sc[(size_t)r] : nullptr);
    if (rc) return rc;
    if (pp && sc[(size_t)r] > cap) {   // grow and fetch the member's pairs
      if (member_pairs(g, r, 2 * sc[(size_t)r])) return -ENOMEM;
      rc = kano_shadow_fetch(c, g->pairs[(size_t)r]);
    }
    return rc;
  }));
  exchange_time_collect(g);
  group_lists(g, cnt, idx, counts);
  if (with_shadow) {
    i64 total = 0;
    for (int r = 0; r < g->G; ++r) total += sc[(size_t)r];
    *shadow_count = total;
    if (!count_only && shadow_pairs && total <= shadow_cap) {
      i64 o = 0;
      for (int r = 0; r < g->G; ++r) {
        if (sc[(size_t)r] > 0)
          std::memcpy(shadow_pairs + 2 * o, g->pairs[(size_t)r],
                      sizeof(int32_t) * 2 * (size_t)sc[(size_t)r]);
        o += sc[(size_t)r];
      }
    }
  }
  return 0;
}

int kano_group_checks(kano_group* g, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                      int32_t* idx, int64_t* counts) {
  if (!g) return -EINVAL;
  if (!counts || !idx) return gfail(g, -EINVAL, "kano_group_checks: idx / counts NULL");
  KANO_GROUP_TRY(group_usable(g));
  KANO_GROUP_TRY(group_buffers(g));
  std::vector<std::array<int64_t, 4>> cnt((size_t)g->G);
  KANO_GROUP_TRY(group_each(g, [&](int r) {
    kano_ctx* c = g->m[(size_t)r];
    int rc = kano_checks_shard(c, gid, ngroups, sys_row, static_cast<uint64_t*>(g->xw[(size_t)r]));
    rc = member_exchange(g, r, rc, g->xw, g->xg, 3 * kano_int::ctx_W(g->m[0]), false);
    if (rc) return rc;
    return kano_verify_combine(c, static_cast<const uint64_t*>(g->xg[(size_t)r]), g->G,
                               g->idx[(size_t)r], cnt[(size_t)r].data(), nullptr, -1, nullptr);
  }));
  group_lists(g, cnt, idx, counts);
  return 0;
}

int kano_group_exchange_timing(kano_group* g, int enable, double* out, int reset) {
  if (!g) return -EINVAL;
  exchange_time_collect(g);
  if (enable >= 0) g->xtime_on = enable != 0;
  if (out) {
    out[0] = g->xt_calls;
    out[1] = g->xt_sum;
    out[2] = g->xt_max;
  }
  if (reset) g->xt_calls = g->xt_sum = g->xt_max = 0;
  return 0;
}

// incremental updates on every member's row shard (kano_add_policies /
// kano_remove_policies write only the member's rows; model.py:125-165 over
// the updated policy list)
int kano_group_add_policies(kano_group* g, int64_t Pn, int32_t ncols_x, const int32_t* xval,
                            const int64_t* sel_off, const int32_t* sel_col,
                            const int32_t* sel_val, const int64_t* alw_off,
                            const int32_t* alw_col, const int32_t* alw_val, int64_t* first_id) {
  if (!g) return -EINVAL;
  KANO_GROUP_TRY(group_usable(g));
  std::vector<int64_t> first((size_t)g->G, -1);
  const int rc = group_each(g, [&](int r) {
    return kano_add_policies(g->m[(size_t)r], Pn, ncols_x, xval, sel_off, sel_col, sel_val,
                             alw_off, alw_col, alw_val, &first[(size_t)r]);
  });
  // members apply the update independently: one that failed while others
  // succeeded leaves the shards on different policy lists
  const auto partial = [&](const std::string& why) {
    bool any = false;
    for (int r = 0; r < g->G; ++r) any |= first[(size_t)r] >= 0;
    if (any) g->poisoned = "kano_group: a partial kano_group_add_policies (" + why + ")";
  };
  if (rc) {
    const std::string why = g->err;
    partial(why);
    g->err = why;
    return rc;
  }
  for (int r = 1; r < g->G; ++r)
    if (first[(size_t)r] != first[0]) {
      partial("the members' policy ids diverged");
      return gfail(g, -EPROTO, "kano_group_add_policies: the members' policy ids diverged");
    }
  if (first_id) *first_id = first[0];
  return 0;
}

int kano_group_remove_policies(kano_group* g, int64_t count, const int64_t* ids) {
  if (!g) return -EINVAL;
  KANO_GROUP_TRY(group_usable(g));
  std::vector<int> done((size_t)g->G, 0);
  const int rc = group_each(g, [&](int r) {
    const int rc1 = kano_remove_policies(g->m[(size_t)r], count, ids);
    done[(size_t)r] = rc1 == 0;
    return rc1;
  });
  if (rc && std::find(done.begin(), done.end(), 1) != done.end())
    g->poisoned = "kano_group: a partial kano_group_remove_policies (" + g->err + ")";
  return rc;
}

// kubesv's path relation (kubesv/kubesv/constraint.py:233-237) over the
// group's row-sharded matrix: every member writes its rows' part of the
// one-hop table (kano_path_shard), one exchange gathers the parts (the same
// transport as the column words: in-place ncclAllGather or device copies),
// then every member's rows of the path matrix are written into dst's member
// on the same device (kano_path_combine).  dst: a group over the same
// devices and row bounds whose members hold a matrix of the same size.
int kano_group_path(kano_group* src, kano_group* dst, int hops, int mode, int64_t* info) {
  if (!src || !dst || src == dst) return -EINVAL;
  if (dst->G != src->G || dst->dev != src->dev)
    return gfail(src, -EINVAL, "kano_group_path: the groups' devices differ");
  KANO_GROUP_TRY(group_usable(src));
  KANO_GROUP_TRY(group_usable(dst));
  const int G = src->G;
  std::vector<int64_t> nws((size_t)G, 0);
  KANO_GROUP_TRY(group_each(src, [&](int r) {
    return kano_path_shard_words(src->m[(size_t)r], &nws[(size_t)r]);
  }));
  for (int r = 1; r < G; ++r)
    if (nws[(size_t)r] != nws[0])
      return gfail(src, -EPROTO, "kano_group_path: the members' column classes differ");
  const i64 nw = nws[0];
  std::vector<void*> recv((size_t)G, nullptr), send((size_t)G, nullptr);
  std::vector<std::array<int64_t, 6>> inf((size_t)G);
  const int rc = group_each(src, [&](int r) {
    kano_ctx* c = src->m[(size_t)r];
    int rc1 = 0;
    if (nw > 0 && hipMalloc(&recv[(size_t)r], sizeof(u64) * (size_t)(nw * G)) != hipSuccess)
      rc1 = kano_int::ctx_fail(c, -ENOMEM, "kano_group_path: the gathered table");
    if (!rc1 && nw > 0) {
      send[(size_t)r] = static_cast<u64*>(recv[(size_t)r]) + (i64)r * nw;
      rc1 = kano_path_shard(c, static_cast<uint64_t*>(send[(size_t)r]));
    }
    // (every member's buffers exist before anyone reads them: the exchange's
    // first barrier)
    rc1 = member_exchange(src, r, rc1, send, recv, nw, false);
    if (!rc1 && hipStreamSynchronize(kano_int::ctx_stream(c)) != hipSuccess)
      rc1 = kano_int::ctx_fail(c, -EIO, "kano_group_path: the exchange failed");
    if (!rc1) {
      rc1 = kano_path_combine(c, dst->m[(size_t)r], static_cast<const uint64_t*>(recv[(size_t)r]),
                              G, hops, mode, inf[(size_t)r].data());
      if (rc1)
        (void)kano_int::ctx_fail(c, rc1, std::string("kano_path_combine: ") +
                                             kano_last_error(dst->m[(size_t)r]));
    }
    return rc1;
  });
  // cleanup: a member that failed after queuing its copies (mode 2) may still
  // read the other members' recv buffers on its stream -- every member drains
  // its own stream and meets the others before any buffer is freed
  group_each(src, [&](int r) {
    (void)hipStreamSynchronize(kano_int::ctx_stream(src->m[(size_t)r]));
    src->pool.bar.wait();
    if (recv[(size_t)r]) (void)hipFree(recv[(size_t)r]);
    return 0;
  });
  if (rc) return rc;
  if (info) std::memcpy(info, inf[0].data(), sizeof(int64_t) * 6);
  return 0;
}

}  // extern "C"
