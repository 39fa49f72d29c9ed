// kano_hip.hip -- MI355X (gfx950) engine for the Kano reachability matrix and
// checks: host orchestration and the C ABI (include/kano_hip.h).  Kernels:
// kano_kernels.hpp.  Design: DESIGN.md.
//
// Reference being replaced (qiyueyao/Kubernetes-verification, kano_py/):
//   ReachabilityMatrix.build_matrix   kano/model.py:125-165
//   matrix accessors                  kano/model.py:167-184
//   all_reachable / all_isolated      kano/algorithm.py:4-17
//   user_crosscheck                   kano/algorithm.py:20-42
//   system_isolation                  kano/algorithm.py:45-55
//   policy_shadow / policy_conflict   kano/algorithm.py:58-100
//
// One build, all on the context stream, two host syncs (list sizes):
//   classes  row classes  = pods hashed on the working-SELECTOR keys,
//            column classes = pods hashed on the working-ALLOW keys.  A
//            predicate on those keys cannot tell members of a class apart,
//            so S(i) is a function of the row class and allow_p(j) of the
//            column class (model.py:95-111, 142-154 depend on nothing else).
//   allow    AC[p][ca]: policy p allows column class ca (and the same bits
//            class-major, ACT); per policy the allowed classes and pods
//   select   selT[pb][c]: bit q = policy 64*pb+q selects row class c
//   plan     per row class |S(c)|, rebuild cost, work items, heavy flag
//   heavy    rows whose rebuild is expensive: Mc = OR over S(c) of AC rows
//            (bitwise) or the fp4 MFMA contraction Sel x Allow over column
//            classes (dense path), then expanded to pods at the first member
//   rows     (class, <=ch members, column chunk) work items: LDS row from the
//            allowed-pod lists (light) or a copy (heavy), streamed to the
//            member rows; column OR / NAND folded in
#include "kano_engine.hpp"
#include "kano_kernels.hpp"

namespace kano_eng {

int fail(kano_ctx* ctx, int code, const std::string& msg) {
  ctx->err = msg;
  return code;
}

int settle(kano_ctx* ctx);

int dalloc(kano_ctx* ctx, DBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.p && b.bytes >= bytes) return 0;
  if (b.p) {
    KTRY(settle(ctx));    // an asynchronously completing matrix write may still use it
    KCHK(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  const hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    b.p = nullptr;
    return fail(ctx, -ENOMEM, "hipMalloc(" + std::to_string(bytes) + " bytes) -> " +
                                  hipGetErrorString(e));
  }
  b.bytes = bytes;
  return 0;
}

void dfree(DBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}


// A launch whose own dispatch marks ev (when given) -- a separate
// hipEventRecord costs the stream ~4.5 us (scripts/micro/event_cost.hip).
// Always through hipExtLaunchKernel with the kernel's handle: a triple-chevron
// launch through the function-pointer parameter (hipLaunchKernelGGL's macro
// form) launched nothing in the host-sanitizer build (tests/asan: the first
// scan's host signal never came)
template <typename... KArgs, typename... Args>
void launch_marked(void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t st,
                   hipEvent_t ev, Args... args) {
  hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, st, nullptr, ev, 0, args...);
}

// ---- device-wide scans: batches of k_scan_lb jobs ------------------------
inline i64 scan_tiles(i64 n, int items = SCAN_ITEMS) {
  return (n + (i64)TPB * items - 1) / ((i64)TPB * items);
}

// status slots per region >= slots (grows, zeroing both regions in order)
int scan_reserve(kano_ctx* ctx, i64 slots, bool side = false) {
  i64& cap = side ? ctx->scan_cap2 : ctx->scan_cap;
  if (slots <= cap) return 0;
  slots = std::max<i64>(slots, 2 * cap);
  const size_t bytes = sizeof(u64) * 2 * (size_t)slots;
  DBuf& tmp = side ? ctx->scan_tmp2 : ctx->scan_tmp;
  KTRY(dalloc(ctx, tmp, bytes));
  KCHK(hipMemsetAsync(tmp.p, 0, bytes, side ? ctx->stream2 : ctx->stream));
  cap = slots;
  (side ? ctx->scan_parity2 : ctx->scan_parity) = 0;
  return 0;
}

// several exclusive scans in one launch: out[0..n] with out[n] = total
struct ScanBatch {
  ScanJobs jobs{};
  kano_ctx* ctx;
  bool side = false;   // on stream2 with its own status regions (no host totals)
  explicit ScanBatch(kano_ctx* c, bool on_side = false) : ctx(c), side(on_side) {
    jobs.count = 0;
    jobs.npub = 0;
  }
  // copy size slot `slot` (written by an earlier kernel) to its host mirror
  // in this launch
  void publish(int slot) {
    if (!ctx->gmirror_dev || jobs.npub == MAX_PUBLISH) return;
    jobs.pub_src[jobs.npub] = P_<u64>(ctx->sizes) + slot;
    jobs.pub_dst[jobs.npub] = ctx->gmirror_dev + slot;
    ++jobs.npub;
  }
  template <typename Tin, typename Tout>
  int add(const Tin* in, i64 n, Tout* out, int total_slot = -1) {
    static_assert(sizeof(Tin) == 4 || sizeof(Tin) == 8, "int32 / int64 scans");
    static_assert(sizeof(Tout) == 4 || sizeof(Tout) == 8, "int32 / int64 scans");
    if (jobs.count == MAX_SCAN_JOBS) KTRY(run());
    ScanJob& j = jobs.j[jobs.count++];
    j.in = in;
    j.out = out;
    j.total = total_slot >= 0 ? P_<u64>(ctx->sizes) + total_slot : nullptr;
    j.total_host = total_slot >= 0 && ctx->gmirror_dev ? ctx->gmirror_dev + total_slot : nullptr;
    j.n = n;
    j.st = 0;                  // (status offsets: run(), once the tile length is chosen)
    j.in64 = sizeof(Tin) == 8;
    j.out64 = sizeof(Tout) == 8;
    j.gen = 0;
    j.gcnt = nullptr;
    return 0;
  }
  // class-id scan over the representative flags of pods [m0, m0 + n), the
  // flags generated inside the scan (no flag pass)
  int add_rep_flags(ClassSet& cs, int pbits, i64 n, int total_slot) {
    KTRY(add(static_cast<const int32_t*>(nullptr), n, P_<int32_t>(cs.cid), total_slot));
    ScanJob& j = jobs.j[jobs.count - 1];
    j.gen = 1;
    j.gsmin = P_<int32_t>(cs.smin);
    j.gtab = P_<u64>(cs.table);
    j.gpb = pbits;
    j.gslot = P_<int32_t>(cs.slot_of);
    j.gm0 = cs.m0;
    return 0;
  }
  // policy_shadow's pair offsets over pods [m0, m0 + n): each pod's count is
  // its class's segment length in loff, generated inside the scan
  int add_class_lengths(const int32_t* cls, const i64* loff, i64 m0, i64 n, i64* out,
                        int total_slot) {
    KTRY(add(static_cast<const int32_t*>(nullptr), n, out, total_slot));
    ScanJob& j = jobs.j[jobs.count - 1];
    j.gen = 2;
    j.gslot = cls;
    j.gloff = loff;
    j.gm0 = m0;
    return 0;
  }
  // the same offsets from the per-class counts themselves (cnt[c] = loff[c +
  // 1] - loff[c]): queued beside loff's own scan, not after it
  int add_class_counts(const int32_t* cls, const i64* cnt, i64 m0, i64 n, i64* out,
                       int total_slot) {
    KTRY(add(static_cast<const int32_t*>(nullptr), n, out, total_slot));
    ScanJob& j = jobs.j[jobs.count - 1];
    j.gen = 3;
    j.gslot = cls;
    j.gcnt = cnt;
    j.gm0 = m0;
    return 0;
  }
  // the launch with only the used job slots in its kernel argument
  template <int NJ, int IT>
  void launch_n(dim3 g, u64* cur, u64* nxt, hipEvent_t mark) {
    ScanJobsN<NJ> a;
    for (int q = 0; q < NJ; ++q) a.j[q] = jobs.j[q];
    a.count = jobs.count;
    a.npub = jobs.npub;
    for (int q = 0; q < MAX_PUBLISH; ++q) {
      a.pub_src[q] = jobs.pub_src[q];
      a.pub_dst[q] = jobs.pub_dst[q];
    }
    a.sig_host = jobs.sig_host;
    a.sig_val = jobs.sig_val;
    a.sig_ctr = jobs.sig_ctr;
    a.sig_n = jobs.sig_n;
    launch_marked(k_scan_lb<NJ, IT>, g, dim3(TPB), 0, side ? ctx->stream2 : ctx->stream, mark, a,
                  cur, nxt, side ? ctx->scan_cap2 : ctx->scan_cap);
  }
  template <int IT>
  void launch_it(dim3 g, u64* cur, u64* nxt, hipEvent_t mark) {
    switch (jobs.count) {
      case 1: launch_n<1, IT>(g, cur, nxt, mark); break;
      case 2: launch_n<2, IT>(g, cur, nxt, mark); break;
      case 3: launch_n<3, IT>(g, cur, nxt, mark); break;
      case 4: launch_n<4, IT>(g, cur, nxt, mark); break;
      case 5: launch_n<5, IT>(g, cur, nxt, mark); break;
      case 6: launch_n<6, IT>(g, cur, nxt, mark); break;
      case 7: launch_n<7, IT>(g, cur, nxt, mark); break;
      default: launch_n<MAX_SCAN_JOBS, IT>(g, cur, nxt, mark); break;
    }
  }
  // mark: an event this launch's dispatch marks (none when no job is queued)
  int run(hipEvent_t mark = nullptr) {
    if (jobs.count == 0) return 0;
    // the tile length, 256 x 8 elements (round 4: longer tiles -- fewer
    // look-back hops -- measured slower on C3's <= 100k-entry scans: 32 per
    // thread 0.432 ms a step against 0.377 at 8, 16 0.380)
    const int items = SCAN_ITEMS;
    i64 slots = 0, maxt = 1;
    for (int q = 0; q < jobs.count; ++q) {
      jobs.j[q].st = slots;
      slots += 1 + scan_tiles(jobs.j[q].n, items);
      maxt = std::max<i64>(maxt, scan_tiles(jobs.j[q].n, items));
    }
    KTRY(scan_reserve(ctx, slots, side));
    // the host signal: raised once every host mirror of this launch is written
    int writers = jobs.npub > 0 ? 1 : 0;
    for (int q = 0; q < jobs.count; ++q) writers += jobs.j[q].total_host ? 1 : 0;
    jobs.sig_host = nullptr;
    // (the signal and its arrival counter belong to the engine stream: a side
    // scan's host totals are plain mirror stores, read once the engine
    // stream has joined the side stream)
    if (side) writers = 0;
    if (writers > 0 && ctx->sig_ctr.p) {
      jobs.sig_host = ctx->gmirror_dev + SZ_SIGNAL;
      jobs.sig_val = ++ctx->sig_seq;
      jobs.sig_ctr = reinterpret_cast<uint32_t*>(ctx->sig_ctr.p);
      jobs.sig_n = writers;
      ctx->sig_armed = jobs.sig_val;
    } else if (writers > 0) {
      ctx->sig_armed = 0;
    }
    u64* st = P_<u64>(side ? ctx->scan_tmp2 : ctx->scan_tmp);
    const i64 cap = side ? ctx->scan_cap2 : ctx->scan_cap;
    int& parity = side ? ctx->scan_parity2 : ctx->scan_parity;
    u64* cur = st + (parity ? cap : 0);
    u64* nxt = st + (parity ? 0 : cap);
    const dim3 g((unsigned)maxt, (unsigned)jobs.count);
    if (items == 32) launch_it<32>(g, cur, nxt, mark);
    else if (items == 16) launch_it<16>(g, cur, nxt, mark);
    else if (items == 4) launch_it<4>(g, cur, nxt, mark);
    else launch_it<SCAN_ITEMS>(g, cur, nxt, mark);
    KLAUNCH();
    parity ^= 1;
    jobs.count = 0;
    jobs.npub = 0;
    return 0;
  }
};

template <typename Tin, typename Tout>
int scan_excl(kano_ctx* ctx, const Tin* in, i64 n, Tout* out) {
  ScanBatch sb(ctx);
  KTRY(sb.add(in, n, out));
  return sb.run();
}

// several device fills in one launch (k_fill_many)
struct FillBatch {
  FillJobs jobs{};
  kano_ctx* ctx;
  hipStream_t st = nullptr;   // (nullptr: the engine stream)
  explicit FillBatch(kano_ctx* c, hipStream_t s = nullptr) : ctx(c), st(s) { jobs.count = 0; }
  int add(DBuf& b, size_t bytes, uint32_t value);
  int add_raw(void* p, size_t bytes, uint32_t value) {
    if (bytes == 0) return 0;
    if (jobs.count == MAX_FILLS) KTRY(run());
    jobs.j[jobs.count++] = FillJob{static_cast<uint32_t*>(p), (i64)(bytes / 4), value};
    return 0;
  }
  int run();
  // the pending jobs, for a launch that carries them (fill_item); none left
  FillJobs take() {
    FillJobs j = jobs;
    jobs.count = 0;
    return j;
  }
};

// blocks a launch adds for carried fills (0 when there are none)
unsigned fill_ride_blocks(const FillJobs& fj) {
  if (fj.count == 0) return 0;
  i64 most = 0;
  for (int q = 0; q < fj.count; ++q) most = std::max(most, fj.j[q].words);
  return (unsigned)std::max<i64>(1, std::min<i64>(FILL_RIDE_BLOCKS, (most + TPB - 1) / TPB));
}

int FillBatch::add(DBuf& b, size_t bytes, uint32_t value) {
  if (bytes == 0) return 0;
  if (bytes % 4 != 0 || bytes > b.bytes) return fail(ctx, -EINVAL, "internal: bad fill job");
  if (jobs.count == MAX_FILLS) KTRY(run());
  jobs.j[jobs.count++] = FillJob{reinterpret_cast<uint32_t*>(b.p), (i64)(bytes / 4), value};
  return 0;
}

int FillBatch::run() {
  if (jobs.count == 0) return 0;
  i64 most = 0;
  for (int q = 0; q < jobs.count; ++q) most = std::max(most, jobs.j[q].words);
  const unsigned grid = (unsigned)std::max<i64>(1, std::min<i64>(2048, (most + TPB - 1) / TPB));
  hipLaunchKernelGGL(k_fill_many, dim3(grid), dim3(TPB), 0, st ? st : ctx->stream, jobs);
  KLAUNCH();
  jobs.count = 0;
  return 0;
}

// the two physical sets of k_rows' inputs exchanged (pointers only)
void swap_rows_ptrs(kano_ctx* ctx) {
  RowsInputs& a = ctx->rin_alt;
  std::swap(ctx->wioff, a.wioff);
  std::swap(ctx->wicls, a.wicls);
  std::swap(ctx->soffc, a.soffc);
  std::swap(ctx->slist, a.slist);
  std::swap(ctx->aloff, a.aloff);
  std::swap(ctx->alist, a.alist);
  std::swap(ctx->alcoff, a.alcoff);
  std::swap(ctx->alc, a.alc);
  std::swap(ctx->rc.moff, a.rmoff);
  std::swap(ctx->rc.mem, a.rmem);
  std::swap(ctx->cc.moff, a.cmoff);
  std::swap(ctx->cc.mem, a.cmem);
  std::swap(ctx->cc.cls, a.ccls);
  std::swap(ctx->hflag, a.hflag);
  std::swap(ctx->hlist, a.hlist);
  std::swap(ctx->Mc, a.Mc);
  ctx->rows_set ^= 1;
}

// ---- pipelined calls: the next kano_verify's prologue behind a gate ------
// (kano_set_pipeline; the fields' comment in kano_engine.hpp)
void ring_bell(kano_ctx* ctx) {
  if (ctx->bell) __atomic_store_n(ctx->bell, ctx->bell_seq, __ATOMIC_SEQ_CST);
}

// a primed prologue not taken by a kano_verify: open the gate, let it run
// (into the private size slots and the next input set), put both back
int unprime(kano_ctx* ctx) {
  if (!ctx->primed || ctx->priming) return 0;
  ctx->primed = false;
  ring_bell(ctx);
  ctx->gate_forced = ctx->bell_seq;           // (not a step boundary: kano_gate_timing)
  KCHK(hipStreamSynchronize(ctx->stream));
  KCHK(hipStreamSynchronize(ctx->stream2));   // (its member lists run on stream2)
  std::swap(ctx->sizes, ctx->sizes_alt);
  swap_rows_ptrs(ctx);
  ctx->alist_valid = ctx->prime_alist_valid;
  return 0;
}

int sync(kano_ctx* ctx) {
  KTRY(unprime(ctx));
  KCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// an asynchronously completing kano_verify's matrix write, finished
int settle(kano_ctx* ctx) {
  KTRY(unprime(ctx));
  if (!ctx->async_pending) return 0;
  ctx->async_pending = false;
  KCHK(hipSetDevice(ctx->device));
  KCHK(hipStreamSynchronize(ctx->stream3));
  if (ctx->stream3m) KCHK(hipStreamSynchronize(ctx->stream3m));
  if (ctx->stream3x) KCHK(hipStreamSynchronize(ctx->stream3x));
  return sync(ctx);
}

// a k_rows launch's time, once its end event is complete (block: wait for
// it; else leave it pending while the launch still runs)
int resolve_rows_slot(kano_ctx* ctx, int k, bool block) {
  if (!ctx->rows_time_pending[k]) return 0;
  if (!block) {
    const hipError_t q = hipEventQuery(ctx->ev_rt[k][1]);
    if (q == hipErrorNotReady) return 0;
    KCHK(q);
  }
  ctx->rows_time_pending[k] = false;
  KCHK(hipEventSynchronize(ctx->ev_rt[k][1]));
  float ms = 0.f;
  KCHK(hipEventElapsedTime(&ms, ctx->ev_rt[k][0], ctx->ev_rt[k][1]));
  ctx->rows_ms_last = ms;
  if (ctx->rows_ms_n == 0 || ms < ctx->rows_ms_min) ctx->rows_ms_min = ms;
  if (ctx->rows_ms_n == 0 || ms > ctx->rows_ms_max) ctx->rows_ms_max = ms;
  ctx->rows_ms_sum += ms;
  ctx->rows_ms_n += 1;
  return 0;
}

int resolve_rows_time(kano_ctx* ctx, bool block = true) {
  for (int k = 0; k < 2; ++k) KTRY(resolve_rows_slot(ctx, k, block));
  return 0;
}

// Back-to-back kano_verify: the previous call's matrix write may still read
// its inputs; this build takes the other set (written once the write two
// calls back, which last read it, has ended -- an event wait on the engine
// stream, not on the host)
int swap_rows_inputs(kano_ctx* ctx) {
  swap_rows_ptrs(ctx);
  ctx->alist_valid = false;
  // (usually long over: then no wait packet on the engine stream)
  if (ctx->rows_end_rec[ctx->rows_set]) {
    const hipError_t q = hipEventQuery(ctx->rows_end_ev[ctx->rows_set]);
    if (q == hipErrorNotReady)
      KCHK(hipStreamWaitEvent(ctx->stream, ctx->rows_end_ev[ctx->rows_set], 0));
    else
      KCHK(q);
  }
  return 0;
}


// the last build's MFMA contraction time, once its end event is complete
int resolve_mfma_time(kano_ctx* ctx) {
  if (!ctx->mfma_time_pending) return 0;
  ctx->mfma_time_pending = false;
  KCHK(hipEventSynchronize(ctx->ev_m1));
  float ms = 0.f;
  KCHK(hipEventElapsedTime(&ms, ctx->ev_m0, ctx->ev_m1));
  ctx->mfma_ms_sum += ms;
  ctx->mfma_ops_sum += ctx->mfma_ops_last;
  ctx->mfma_n += 1;
  return 0;
}

// size slots [first, first + count) to the host: one copy, one sync
int read_slots(kano_ctx* ctx, int first, int count, i64* out) {
  KCHK(hipMemcpyAsync(ctx->ghost, P_<u64>(ctx->sizes) + first, sizeof(u64) * count,
                      hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  for (int k = 0; k < count; ++k) out[k] = (i64)ctx->ghost[k];
  return 0;
}

// the overlapped syncs: the slots reach their host mirror inside the scans
// (totals) or by a scan's publish list (atomic slots); the host records an
// event behind them now (unless a scan raises the host signal), queues more
// work, and later waits and reads the mirror -- no copy
// A device -> host copy of the results: a kernel storing straight into the
// caller's page-locked buffer when it is one (hipHostMalloc'd, e.g.
// kano_host_alloc), else the runtime's copy
// the device address of a page-locked host buffer (16-byte aligned), else null
void* pinned_dev(void* host) {
  if (!host || (reinterpret_cast<uintptr_t>(host) & 15)) return nullptr;
  hipPointerAttribute_t at{};
  void* dptr = nullptr;
  if (hipPointerGetAttributes(&at, host) == hipSuccess && at.type == hipMemoryTypeHost &&
      at.devicePointer)
    dptr = at.devicePointer;
  (void)hipGetLastError();
  return dptr;
}

int copy_out(kano_ctx* ctx, void* host, const void* dev, size_t bytes, hipStream_t st) {
  if (bytes == 0) return 0;
  hipPointerAttribute_t at{};
  void* dptr = nullptr;
  if (hipPointerGetAttributes(&at, host) == hipSuccess && at.type == hipMemoryTypeHost &&
      at.devicePointer)
    dptr = at.devicePointer;
  (void)hipGetLastError();
  if (!dptr || (reinterpret_cast<uintptr_t>(dptr) & 15) || (reinterpret_cast<uintptr_t>(dev) & 15)) {
    KCHK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
    return 0;
  }
  const i64 n16 = (i64)(bytes / 16);
  const int ntail = (int)((bytes % 16) / 4);
  const unsigned grid = (unsigned)std::max<i64>(1, std::min<i64>(1024, nblk(std::max<i64>(1, n16))));
  hipLaunchKernelGGL(k_copy_out, dim3(grid), dim3(TPB), 0, st, static_cast<const uint4*>(dev),
                     static_cast<uint4*>(dptr), n16,
                     reinterpret_cast<const uint32_t*>(static_cast<const char*>(dev) + n16 * 16),
                     reinterpret_cast<uint32_t*>(static_cast<char*>(dptr) + n16 * 16), ntail);
  KLAUNCH();
  return 0;
}

int mirror_begin(kano_ctx* ctx) {
  // the latest scan with host totals raises the host signal: nothing to queue
  if (ctx->sig_armed) {
    ctx->sig_wait = ctx->sig_armed;
    ctx->sig_armed = 0;
    return 0;
  }
  ctx->sig_wait = 0;
  KCHK(hipEventRecord(ctx->ev_sizes, ctx->stream));
  return 0;
}

// Poll the host signal word (the syncs' waits are 30-100 us: the host spins,
// it does not sleep -- a sleeping host's wake-up is at the scheduler's
// mercy).  The sequence numbers only grow, so any value >= val means the
// slots arrived.  Past a second (a slow device, a failed launch) the
// stream's own synchronisation decides.
int wait_signal(kano_ctx* ctx, u64 val) {
  volatile u64* sig = ctx->gmirror + SZ_SIGNAL;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint32_t spin = 1; *sig < val; ++spin) {
    __builtin_ia32_pause();
    if ((spin & 0xfff) != 0) continue;
    if (clk::now() - t0 > std::chrono::seconds(1)) {
      KCHK(hipStreamSynchronize(ctx->stream));
      if (*sig < val)
        return fail(ctx, -EIO, "internal: host signal not raised (wait " +
                                   std::to_string(ctx->ht_wait) + ": want " + std::to_string(val) +
                                   ", have " + std::to_string((u64)*sig) + ")");
      break;
    }
  }
  return 0;
}

int mirror_wait(kano_ctx* ctx, int first, int count, i64* out) {
  const auto t0 = std::chrono::steady_clock::now();
  if (ctx->sig_wait) {
    const u64 v = ctx->sig_wait;
    ctx->sig_wait = 0;
    KTRY(wait_signal(ctx, v));
  } else {
    KCHK(hipEventSynchronize(ctx->ev_sizes));
  }
  const double w =
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  ctx->ht_wait_cur += w;
  const int k = 9 + std::min(ctx->ht_wait++, 2);
  ctx->ht[k] = std::max(ctx->ht[k], w);
  for (int q = 0; q < count; ++q) out[q] = (i64)((volatile u64*)ctx->gmirror)[first + q];
  return 0;
}

// stage-boundary events (kano_stage_times) only when asked for: each record
// costs host time on the launch path.  The k_rows events (7, 8) always run:
// the bench's roofline needs them.
int stage_mark(kano_ctx* ctx, int k, hipStream_t st) {
  if (ctx->stage_timing) KCHK(hipEventRecord(ctx->ev[k], st));
  return 0;
}

i64 rows_local(const kano_ctx* ctx) { return ctx->r1 - ctx->r0; }

// ---- classes ---------------------------------------------------------------
i64 table_size(i64 n) {
  i64 T = 64;
  while (T < 2 * n) T <<= 1;
  return T;
}

// Packed sides whose key and smallest member fit one word together keep the
// member in the slot itself, key << pbits | pod: a block's first probe of a
// slot inserts or finds its class and lowers the member in one atomic
// round trip (no smin array); 0 when they do not fit (the smin form)
int cls_pod_bits(const kano_ctx* ctx, const ClassSet& cs) {
  if (!cs.packed) return 0;
  int pb = 1;
  while (pb < 31 && ((i64)1 << pb) < ctx->n) ++pb;
  return cs.tbits + pb <= 63 ? pb : 0;
}

int classify_alloc1(kano_ctx* ctx, ClassSet& cs, FillBatch& fb) {
  const i64 n = ctx->n, T = table_size(n);
  KTRY(dalloc(ctx, cs.table, sizeof(u64) * T));   // int32 pods, or u64 packed keys
  KTRY(dalloc(ctx, cs.smin, sizeof(int32_t) * T));
  KTRY(dalloc(ctx, cs.slot_of, sizeof(int32_t) * std::max<i64>(1, n)));
  KTRY(dalloc(ctx, cs.flag, sizeof(int32_t) * std::max<i64>(1, n)));
  KTRY(dalloc(ctx, cs.cid, sizeof(int32_t) * (n + 1)));
  KTRY(dalloc(ctx, cs.cls, sizeof(int32_t) * std::max<i64>(1, n)));
  KTRY(fb.add(cs.table, (cs.packed ? sizeof(u64) : sizeof(int32_t)) * T, 0xffffffffu));
  if (!cls_pod_bits(ctx, cs)) KTRY(fb.add(cs.smin, sizeof(int32_t) * T, 0x7fffffffu));
  // per-class arrays of phase 2a, sized by the side's pods (>= its classes)
  // so that they need not wait for the class count
  const i64 m = std::max<i64>(1, cs.m1 - cs.m0);
  KTRY(dalloc(ctx, cs.rep, sizeof(int32_t) * m));
  KTRY(dalloc(ctx, cs.mcnt, sizeof(int32_t) * m));
  KTRY(dalloc(ctx, cs.mcur, sizeof(int32_t) * m));
  KTRY(dalloc(ctx, cs.moff, sizeof(int32_t) * (m + 1)));
  KTRY(dalloc(ctx, cs.mem, sizeof(int32_t) * m));
  return 0;   // (mcnt is zeroed by k_cls_insert, one entry per pod)
}

ClsSide cls_side(kano_ctx* ctx, ClassSet& cs) {
  ClsSide a{};
  a.keys = P_<int32_t>(cs.keys_d);
  a.KS = cs.KS;
  a.packed = cs.packed;
  a.pbits = cls_pod_bits(ctx, cs);
  a.tmask = (uint32_t)(table_size(ctx->n) - 1);
  a.table = P_<int32_t>(cs.table);
  a.slot_of = P_<int32_t>(cs.slot_of);
  a.smin = P_<int32_t>(cs.smin);
  a.flag = P_<int32_t>(cs.flag);
  a.cid = P_<int32_t>(cs.cid);
  a.cls = P_<int32_t>(cs.cls);
  a.rep = P_<int32_t>(cs.rep);
  a.mcnt = P_<int32_t>(cs.mcnt);
  a.mcur = P_<int32_t>(cs.mcur);
  a.moff = P_<int32_t>(cs.moff);
  a.mem = P_<int32_t>(cs.mem);
  a.cval = P_<int32_t>(cs.cval);
  a.m0 = cs.m0;
  a.m1 = cs.m1;
  a.U = cs.U;
  return a;
}

// phase 1, both sides: hash insert + smallest member per slot, first-member
// flags, class-id scan (no sync)
// (row classes cover only this shard's pods [r0, r1); column classes all pods)
int classify_phase1(kano_ctx* ctx) {
  const i64 n = ctx->n;
  ClsPair pr{{cls_side(ctx, ctx->rc), cls_side(ctx, ctx->cc)}};
  const i64 nr = ctx->rc.m1 - ctx->rc.m0, na = ctx->cc.m1 - ctx->cc.m0;
  const i64 most = std::max(nr, na);
  if (most > 0) {
    hipLaunchKernelGGL(k_cls_insert, dim3(nblk(most), 2), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->pv), n, pr);
    KLAUNCH();
  }
  // class ids: a scan over the representative flags (generated in the scan).
  // (Atomic ids drawn by the inserting pod, without this scan, measured
  // slower: the two counters serialise ~21k atomics each, k_cls_insert 25 ->
  // 58 us, and ids in creation order cost k_rows ~10 % -- smallest-member
  // order keeps its member rows closer to address order.)
  ScanBatch sb(ctx);
  KTRY(sb.add_rep_flags(ctx->rc, cls_pod_bits(ctx, ctx->rc), nr, SZ_UR));
  KTRY(sb.add_rep_flags(ctx->cc, cls_pod_bits(ctx, ctx->cc), na, SZ_UA));
  return sb.run();
}

int classify_alloc2(kano_ctx* ctx, ClassSet& cs) {
  return dalloc(ctx, cs.cval, sizeof(int32_t) * std::max<i64>(1, (i64)cs.KS * cs.U));
}

// phase 2a, both sides, without the class counts (the host reads them
// meanwhile): ids, member counts, their offsets (scanned over the side's pod
// count; the entries past U are zero), member lists of pods [m0, m1)
// mark: an event the member-list fill's dispatch marks (returns false, and
// marks nothing, when there is no fill)
int classify_phase2a(kano_ctx* ctx) {
  ClsPair pr{{cls_side(ctx, ctx->rc), cls_side(ctx, ctx->cc)}};
  const i64 mr = ctx->rc.m1 - ctx->rc.m0, ma = ctx->cc.m1 - ctx->cc.m0;
  const i64 rl = std::max(mr, ma);
  // The member lists (their offsets' scan and the fill) feed only the side
  // work, the lists' consumers past the side stream's join (k_pods_own: the
  // column classes' members) and the matrix write: they run on stream2,
  // forked at the member-count pass (its dispatch marks ev_pre), so the
  // engine stream goes from the class ids straight to the join (two launches
  // fewer on it).  Without stream2 they stay on the engine stream.
  hipStream_t side = ctx->mlists_side ? ctx->stream2 : nullptr;
  if (rl > 0) {   // ids and member counts in one pass
    // (several pods a thread when the previous build had few classes; the
    // kernel is correct for any count -- a full LDS table goes global)
    const i64 prevU = std::max(ctx->rc.U, ctx->cc.U);
    const int ipt = ctx->assign_ipt > 0 ? ctx->assign_ipt
                                        : (prevU > 0 && prevU <= 1024 ? ASSIGN_IPT : 1);
    launch_marked(k_cls_assign_count, dim3(nblk(rl, (i64)TPB * ipt), 2), dim3(TPB), 0,
                  ctx->stream, side ? ctx->ev_pre : nullptr, pr, ipt);
    KLAUNCH();
  } else if (side) {
    KCHK(hipEventRecord(ctx->ev_pre, ctx->stream));
  }
  if (side) KCHK(hipStreamWaitEvent(side, ctx->ev_pre, 0));
  ScanBatch sb(ctx, side != nullptr);
  KTRY(sb.add(P_<int32_t>(ctx->rc.mcnt), mr, P_<int32_t>(ctx->rc.moff)));
  KTRY(sb.add(P_<int32_t>(ctx->cc.mcnt), ma, P_<int32_t>(ctx->cc.moff)));
  KTRY(sb.run());
  if (rl > 0) {
    hipLaunchKernelGGL(k_cls_mfill, dim3(nblk(rl), 2), dim3(TPB), 0, side ? side : ctx->stream, pr,
                       (const int32_t*)nullptr, 0, (int32_t*)nullptr, (int32_t*)nullptr,
                       reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_ERR));
    KLAUNCH();
  }
  return 0;
}

// phase 2b (U known): representative values, slot-major cval[k * U + c];
// fj: fills that need not precede it, carried by the same launch
int classify_phase2b(kano_ctx* ctx, FillJobs fj) {
  ClsPair pr{{cls_side(ctx, ctx->rc), cls_side(ctx, ctx->cc)}};
  const i64 U = std::max(ctx->rc.U, ctx->cc.U);
  if (U > 0) {
    const unsigned nbv = nblk(U), nbf = fill_ride_blocks(fj);
    hipLaunchKernelGGL(k_cls_vals, dim3(nbv + nbf, 2), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->pv), ctx->n, pr, fj, nbv);
    KLAUNCH();
  } else if (fj.count > 0) {
    hipLaunchKernelGGL(k_fill_many, dim3(fill_ride_blocks(fj)), dim3(TPB), 0, ctx->stream, fj);
    KLAUNCH();
  }
  return 0;
}

// ---- policy -> class matching (hash join, dense fallback) -------------------
// sx.pstart / sx.plen: policy p matches the classes
// sx.gmem[pstart[p] .. pstart[p] + plen[p]).
int match_alloc(kano_ctx* ctx, SideMatch& sx, ClassSet& cs, FillBatch& fb) {
  const i64 P = ctx->P, U = cs.U;
  KTRY(dalloc(ctx, sx.pstart, sizeof(i64) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, sx.plen, sizeof(int32_t) * std::max<i64>(1, P)));
  if (P == 0) return 0;
  if (U == 0) {
    KTRY(fb.add(sx.pstart, sizeof(i64) * P, 0u));
    KTRY(fb.add(sx.plen, sizeof(int32_t) * P, 0u));
    return 0;
  }
  if (sx.dense) return 0;
  const int NM = sx.NM;
  sx.T = table_size(U);
  const i64 NT = std::max<i64>(1, (i64)NM * sx.T);
  KTRY(dalloc(ctx, sx.table, sizeof(int32_t) * NT));
  KTRY(dalloc(ctx, sx.pslot, sizeof(int32_t) * std::max<i64>(1, (i64)NM * U)));
  KTRY(dalloc(ctx, sx.gcnt, sizeof(int32_t) * NT));
  KTRY(dalloc(ctx, sx.gcur, sizeof(int32_t) * std::max<i64>(1, (i64)NM * U)));
  KTRY(dalloc(ctx, sx.goff, sizeof(int32_t) * (NT + 1)));
  KTRY(dalloc(ctx, sx.gmem, sizeof(int32_t) * ((i64)NM * U + U)));
  if (NM > 0) {
    KTRY(fb.add(sx.table, sizeof(int32_t) * NT, 0xffffffffu));
    KTRY(fb.add(sx.gcnt, sizeof(int32_t) * NT, 0u));
  }
  return 0;
}

JoinSide join_side(kano_ctx* ctx, SideMatch& sx, ClassSet& cs) {
  JoinSide a{};
  a.cval = P_<int32_t>(cs.cval);
  a.U = cs.U;
  a.moff = P_<int32_t>(sx.moff);
  a.mslot = P_<int32_t>(sx.mslot);
  a.table = P_<int32_t>(sx.table);
  a.T = sx.T;
  a.pslot = P_<int32_t>(sx.pslot);
  a.gcnt = P_<int32_t>(sx.gcnt);
  a.goff = P_<int32_t>(sx.goff);
  a.gcur = P_<int32_t>(sx.gcur);
  a.gmem = P_<int32_t>(sx.gmem);
  a.toff = P_<i64>(sx.toff);
  a.tval = P_<int32_t>(sx.tval);
  a.pmask = P_<int32_t>(sx.pmask);
  a.pstart = P_<i64>(sx.pstart);
  a.plen = P_<int32_t>(sx.plen);
  a.NM = sx.NM;
  a.live = (ctx->P > 0 && cs.U > 0 && !sx.dense) ? 1 : 0;
  a.ctab = P_<u64>(cs.table);
  a.ctmask = (uint32_t)(table_size(ctx->n) - 1);
  a.csmin = P_<int32_t>(cs.smin);
  a.cpb = cls_pod_bits(ctx, cs);
  a.ccid = P_<int32_t>(cs.cid);
  a.cm0 = cs.m0;
  a.kbits = P_<int32_t>(cs.keys_d) + cs.KS;
  a.KS = cs.KS;
  return a;
}

int match_dense(kano_ctx* ctx, SideMatch& sx, ClassSet& cs);

// hash join of both sides in the same launches: side 0 = allow side on the
// column classes, side 1 = select side on the row classes; a dense side
// (too many masks) takes match_dense instead
int match_both(kano_ctx* ctx) {
  JoinPair pr{{join_side(ctx, ctx->am, ctx->cc), join_side(ctx, ctx->sm, ctx->rc)}};
  const JoinSide &a0 = pr.s[0], &a1 = pr.s[1];
  const i64 maxU = std::max(a0.live ? a0.U : 0, a1.live ? a1.U : 0);
  const unsigned rows_i = (a0.live ? a0.NM : 0) + (a1.live ? a1.NM : 0);
  const unsigned rows_f = (a0.live ? a0.NM + 1 : 0) + (a1.live ? a1.NM + 1 : 0);
  if (rows_i > 0) {
    hipLaunchKernelGGL(k_join_insert, dim3(nblk(maxU), rows_i), dim3(TPB), 0, ctx->stream, pr);
    KLAUNCH();
    ScanBatch sb(ctx);
    for (int q = 0; q < 2; ++q) {
      SideMatch& sx = q ? ctx->sm : ctx->am;
      if (pr.s[q].live && sx.NM > 0)
        KTRY(sb.add(P_<int32_t>(sx.gcnt), (i64)sx.NM * sx.T, P_<int32_t>(sx.goff)));
    }
    KTRY(sb.run());
  }
  if (rows_f > 0) {   // the group members and every policy's group, one launch
    const unsigned nbf = nblk(maxU), nbm = nblk(ctx->P);
    hipLaunchKernelGGL(k_join_fill_match, dim3(std::max(nbf, nbm), rows_f + 2), dim3(TPB), 0,
                       ctx->stream, ctx->P, pr, (int)rows_f, nbf, nbm);
    KLAUNCH();
  }
  if (ctx->P > 0 && ctx->cc.U > 0 && ctx->am.dense) KTRY(match_dense(ctx, ctx->am, ctx->cc));
  if (ctx->P > 0 && ctx->rc.U > 0 && ctx->sm.dense) KTRY(match_dense(ctx, ctx->sm, ctx->rc));
  return 0;
}

// dense fallback: evaluate every (policy, class) predicate (one extra sync)
int match_dense(kano_ctx* ctx, SideMatch& sx, ClassSet& cs) {
  const i64 P = ctx->P, U = cs.U;
  const i64 UW = (U + 63) / 64, ld = std::max<i64>(2, (UW + 1) & ~(i64)1);
  KTRY(dalloc(ctx, sx.bits, sizeof(u64) * P * ld));
  KTRY(dalloc(ctx, sx.boff, sizeof(i64) * (P + 1)));
  hipLaunchKernelGGL(k_class_eval, dim3(nblk(U), (unsigned)ctx->PB), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(cs.cval), U, P, P_<i64>(sx.toff), P_<int32_t>(sx.tslot),
                     P_<int32_t>(sx.tval), (u64*)nullptr, P_<u64>(sx.bits), ld);
  KLAUNCH();
  hipLaunchKernelGGL(k_popc_rows, dim3((unsigned)P), dim3(TPB), 0, ctx->stream, P_<u64>(sx.bits),
                     ld, UW, P_<int32_t>(sx.plen));
  KLAUNCH();
  KTRY((scan_excl<int32_t, i64>(ctx, P_<int32_t>(sx.plen), P, P_<i64>(sx.boff))));
  i64 nnz = 0;
  KCHK(hipMemcpyAsync(&nnz, P_<i64>(sx.boff) + P, 8, hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  KTRY(dalloc(ctx, sx.gmem, sizeof(int32_t) * std::max<i64>(1, nnz)));
  hipLaunchKernelGGL(k_bits_to_lists, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                     P_<u64>(sx.bits), ld, UW, P_<i64>(sx.boff), P_<int32_t>(sx.gmem));
  KLAUNCH();
  hipLaunchKernelGGL(k_offsets_to_start, dim3(nblk(P)), dim3(TPB), 0, ctx->stream,
                     P_<i64>(sx.boff), P, P_<i64>(sx.pstart));
  KLAUNCH();
  return 0;
}

// classes of both sides, both matchings, allow counts, select counts and the
// per-class plan; two host syncs (class counts, list sizes)
// policies per block of k_pol_counts / k_sel_place: combine the per-class
// atomics in LDS when many policies share few row classes (broad selectors)
// policies per block of the class-indexed LDS forms: ~256 blocks (each
// block flushes its whole table: fewer, fuller blocks)
int sel_spb(const kano_ctx* ctx) {
  return ctx->P >= 8 * std::max<i64>(1, ctx->rc.U) ? TPB : WPB;
}

// The front end's first fills: size slots, both sides' hash tables and
// smallest-member slots
int front_fills(kano_ctx* ctx, FillBatch& fb) {
  KTRY(dalloc(ctx, ctx->sizes, sizeof(u64) * SZ_SLOTS));
  KTRY(fb.add(ctx->sizes, sizeof(u64) * SZ_SLOTS, 0u));
  KTRY(classify_alloc1(ctx, ctx->rc, fb));
  KTRY(classify_alloc1(ctx, ctx->cc, fb));
  return 0;
}

int select_engine_streams(kano_ctx* ctx);

// The build's prologue, up to the member lists: it reads only the resident
// inputs (the label tables), so a pipelined kano_verify queues it for the
// next call behind the gate (prime_next)
int front_a(kano_ctx* ctx) {
  KTRY(select_engine_streams(ctx));
  ctx->rc.m0 = ctx->r0;
  ctx->rc.m1 = ctx->r1;
  ctx->cc.m0 = 0;
  ctx->cc.m1 = ctx->n;
  {
    FillBatch fb(ctx);
    KTRY(front_fills(ctx, fb));
    KTRY(fb.run());
  }
  KTRY(classify_phase1(ctx));
  // host sync 1 of the build (the class counts), overlapped: the counts
  // travel while phase 2a runs
  KTRY(mirror_begin(ctx));
  // the member lists and then the side work of do_back_pre go to stream2,
  // forked at the member counts (ev_pre)
  ctx->mlists_side = ctx->stream2 != nullptr && ctx->mlists_side_ok;
  if (!ctx->mlists_side && ctx->stream2) {
    KTRY(classify_phase2a(ctx));
    KCHK(hipEventRecord(ctx->ev_pre, ctx->stream));
    return 0;
  }
  return classify_phase2a(ctx);
}

// primed: the prologue was queued by the previous kano_verify (its gate is
// open: kano_verify rang the bell on entry)
int do_front(kano_ctx* ctx, int path, bool primed = false) {
  if (primed) {
    ctx->primed = false;
    ring_bell(ctx);
    ctx->rc.m0 = ctx->r0;
    ctx->rc.m1 = ctx->r1;
    ctx->cc.m0 = 0;
    ctx->cc.m1 = ctx->n;
    ctx->sig_wait = ctx->prime_sig;   // (its class-count scan raises this signal)
  } else {
    KTRY(front_a(ctx));
  }
  ctx->pre_forked = ctx->stream2 != nullptr;
  i64 u[2] = {0, 0};
  KTRY(mirror_wait(ctx, SZ_UR, 2, u));
  // an earlier matrix write's time, when it has ended (no wait: the
  // previous kano_verify's write may still run beside this build)
  KTRY(resolve_rows_time(ctx, false));
  ctx->rc.U = u[0];
  ctx->cc.U = u[1];
  KTRY(stage_mark(ctx, 1, ctx->stream));

  const i64 P = ctx->P, Ur = ctx->rc.U, Ua = ctx->cc.U;
  ctx->UAW = (Ua + 63) / 64;
  ctx->ldC = std::max<i64>(2, (ctx->UAW + 1) & ~(i64)1);
  FillJobs carried{};
  {
    FillBatch fb(ctx);
    KTRY(classify_alloc2(ctx, ctx->rc));
    KTRY(classify_alloc2(ctx, ctx->cc));
    KTRY(match_alloc(ctx, ctx->am, ctx->cc, fb));
    KTRY(match_alloc(ctx, ctx->sm, ctx->rc, fb));
    KTRY(dalloc(ctx, ctx->nca, sizeof(int32_t) * std::max<i64>(1, P)));
    KTRY(dalloc(ctx, ctx->acnt, sizeof(int32_t) * std::max<i64>(1, P)));
    KTRY(dalloc(ctx, ctx->alcoff, sizeof(i64) * (P + 1)));
    KTRY(dalloc(ctx, ctx->aloff, sizeof(i64) * (P + 1)));
    KTRY(dalloc(ctx, ctx->scnt, sizeof(int32_t) * std::max<i64>(1, Ur)));
    KTRY(dalloc(ctx, ctx->cost, sizeof(u64) * std::max<i64>(1, Ur)));
    KTRY(dalloc(ctx, ctx->wicnt, sizeof(int32_t) * std::max<i64>(1, Ur)));
    KTRY(dalloc(ctx, ctx->hflag, sizeof(int32_t) * std::max<i64>(1, Ur)));
    KTRY(dalloc(ctx, ctx->sq, sizeof(i64) * std::max<i64>(1, Ur)));
    KTRY(dalloc(ctx, ctx->soffc, sizeof(i64) * (Ur + 1)));
    KTRY(dalloc(ctx, ctx->wioff, sizeof(int32_t) * (Ur + 1)));
    KTRY(dalloc(ctx, ctx->hoff, sizeof(int32_t) * (Ur + 1)));
    KTRY(dalloc(ctx, ctx->pfoff, sizeof(i64) * (Ur + 1)));
    KTRY(dalloc(ctx, ctx->scur, sizeof(int32_t) * std::max<i64>(1, Ur)));
    KTRY(fb.add(ctx->scnt, sizeof(int32_t) * Ur, 0u));
    KTRY(fb.add(ctx->cost, sizeof(u64) * Ur, 0u));
    KTRY(fb.add(ctx->scur, sizeof(int32_t) * Ur, 0u));   // (k_sel_place's cursors)
    carried = fb.take();   // (carried by k_cls_vals' launch)
  }
  KTRY(classify_phase2b(ctx, carried));
  KTRY(match_both(ctx));
  KTRY(stage_mark(ctx, 2, ctx->stream));
  // allowed classes / pods per policy, then |S(c)| and the rebuild cost
  // (one wave per policy, both sides)
  // broad selectors over few row classes (the previous build's |S| sum >= 32
  // per class): the class counters meet in LDS tables (k_pol_counts_dx,
  // k_sel_place_dx); either form gives the same counts and lists
  ctx->dense_sel = ctx->dx_on && Ur > 0 && Ur <= DX_MAX &&
                   (ctx->dx_on == 2 || ctx->nnz_sel >= 32 * Ur);   // (dx=2: forced)
  if (P > 0 && ctx->dense_sel) {
    // the select side as bit matrices (k_selrows_dx -> k_ptrans -> counts):
    // SA[pw][c] is also the GEMM's A when every class is heavy
    const i64 ldU = (Ur + 63) / 64;
    ctx->dx_ldY = (Ur + 255) / 256 * 256;
    ctx->dx_PBo = (ctx->PB + GK_KC - 1) / GK_KC * GK_KC;
    KTRY(dalloc(ctx, ctx->dx_sc, sizeof(u64) * (size_t)(P * ldU)));
    KTRY(dalloc(ctx, ctx->dx_sa, sizeof(u64) * (size_t)(ctx->dx_PBo * ctx->dx_ldY)));
    hipLaunchKernelGGL(k_selrows_dx, dim3(nblk(P, WPB)), dim3(TPB), sizeof(u64) * WPB * ldU,
                       ctx->stream, P, P_<i64>(ctx->am.pstart), P_<int32_t>(ctx->am.plen),
                       P_<int32_t>(ctx->am.gmem), P_<int32_t>(ctx->cc.mcnt), P_<int32_t>(ctx->nca),
                       P_<int32_t>(ctx->acnt), P_<i64>(ctx->sm.pstart), P_<int32_t>(ctx->sm.plen),
                       P_<int32_t>(ctx->sm.gmem), ldU, P_<u64>(ctx->dx_sc));
    KLAUNCH();
    const i64 tiles = ctx->dx_PBo * (ctx->dx_ldY / 64);
    hipLaunchKernelGGL(k_ptrans, dim3(nblk(tiles, WPB)), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->dx_sc), ldU, P, P_<u64>(ctx->dx_sa), ctx->dx_ldY, ctx->dx_PBo,
                       (const int32_t*)nullptr);
    KLAUNCH();
    hipLaunchKernelGGL(k_cls_counts_dx, dim3((unsigned)Ur), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->dx_sa), ctx->dx_ldY, ctx->PB, Ur, P_<int32_t>(ctx->acnt),
                       P_<int32_t>(ctx->scnt), P_<unsigned long long>(ctx->cost));
    KLAUNCH();
  } else if (P > 0) {
    const bool sel = Ur > 0;
    hipLaunchKernelGGL(k_pol_counts, dim3(nblk(P, sel_spb(ctx))), dim3(TPB), 0, ctx->stream, P,
                       P_<i64>(ctx->am.pstart), P_<int32_t>(ctx->am.plen),
                       P_<int32_t>(ctx->am.gmem), P_<int32_t>(ctx->cc.mcnt), P_<int32_t>(ctx->nca),
                       P_<int32_t>(ctx->acnt), P_<i64>(ctx->sm.pstart), P_<int32_t>(ctx->sm.plen),
                       sel ? P_<int32_t>(ctx->sm.gmem) : (const int32_t*)nullptr,
                       P_<int32_t>(ctx->scnt), P_<unsigned long long>(ctx->cost), sel_spb(ctx));
    KLAUNCH();
  }
  if (Ur > 0) {
    ClassPlan a;
    a.U = Ur;
    a.scnt = P_<int32_t>(ctx->scnt);
    a.cost = P_<unsigned long long>(ctx->cost);
    a.mcnt = P_<int32_t>(ctx->rc.mcnt);
    a.W = ctx->W;
    a.ch = ctx->rows_ch;
    a.force = path == KANO_PATH_MFMA ? 2 : 0;
    a.wicnt = P_<int32_t>(ctx->wicnt);
    a.hflag = P_<int32_t>(ctx->hflag);
    a.sq = P_<i64>(ctx->sq);
    a.maxs = reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_MAXSEL);  // low half
    a.light = P_<unsigned long long>(ctx->sizes) + SZ_LIGHT;
    a.hsel = P_<unsigned long long>(ctx->sizes) + SZ_HSEL;
    hipLaunchKernelGGL(k_class_plan, dim3(nblk(Ur)), dim3(TPB), 0, ctx->stream, a);
    KLAUNCH();
  }
  ScanBatch sb(ctx);
  KTRY(sb.add(P_<int32_t>(ctx->nca), P, P_<i64>(ctx->alcoff), SZ_NNZ_ALC));
  KTRY(sb.add(P_<int32_t>(ctx->acnt), P, P_<i64>(ctx->aloff), SZ_NNZ_ALW));
  KTRY(sb.add(P_<int32_t>(ctx->scnt), Ur, P_<i64>(ctx->soffc), SZ_NNZ_SEL));
  KTRY(sb.add(P_<int32_t>(ctx->wicnt), Ur, P_<int32_t>(ctx->wioff), SZ_WI));
  KTRY(sb.add(P_<int32_t>(ctx->hflag), Ur, P_<int32_t>(ctx->hoff), SZ_HEAVY));
  KTRY(sb.add(P_<i64>(ctx->sq), Ur, P_<i64>(ctx->pfoff), SZ_NFLAGS));
  sb.publish(SZ_MAXSEL);   // k_class_plan's atomics, for the host's sync 2
  sb.publish(SZ_LIGHT);
  sb.publish(SZ_HSEL);
  KTRY(sb.run());
  return 0;
}

// host sync 2 of the build: every list size at once
int read_sizes(kano_ctx* ctx) {
  i64 v[SZ_HSEL - SZ_NNZ_SEL + 1];
  KTRY(mirror_wait(ctx, SZ_NNZ_SEL, SZ_HSEL - SZ_NNZ_SEL + 1, v));
  ctx->nnz_sel = v[SZ_NNZ_SEL - SZ_NNZ_SEL];
  ctx->nnz_alc = v[SZ_NNZ_ALC - SZ_NNZ_SEL];
  ctx->nnz_alw = v[SZ_NNZ_ALW - SZ_NNZ_SEL];
  ctx->nflags = v[SZ_NFLAGS - SZ_NNZ_SEL];
  ctx->wi_total = v[SZ_WI - SZ_NNZ_SEL];
  ctx->heavy_count = v[SZ_HEAVY - SZ_NNZ_SEL];
  ctx->max_sel = (int)(v[SZ_MAXSEL - SZ_NNZ_SEL] & 0xffffffff);
  ctx->light_cost = v[SZ_LIGHT - SZ_NNZ_SEL];
  ctx->heavy_sel = v[SZ_HSEL - SZ_NNZ_SEL];
  return 0;
}

// column OR / NAND at class level (all_isolated / all_reachable)
int mc_cols(kano_ctx* ctx) {
  const i64 U = ctx->rc.U;
  if (rows_local(ctx) > 0 && U > 0) {
    hipLaunchKernelGGL(k_mc_cols, dim3(nblk(ctx->UAW, 64), nblk(U, 128)), dim3(TPB), 0,
                       ctx->stream, P_<u64>(ctx->Mc), ctx->ldC, ctx->UAW, ctx->cc.U, U,
                       P_<int32_t>(ctx->rc.mcnt), P_<u64>(ctx->col_or_c), P_<u64>(ctx->col_nand_c));
    KLAUNCH();
  }
  return 0;
}

// allowed-pod lists per policy (members of its allowed column classes)
PolPodsArgs pol_pods_args(kano_ctx* ctx) {
  return PolPodsArgs{ctx->P, P_<i64>(ctx->alcoff), P_<int32_t>(ctx->alc),
                     P_<int32_t>(ctx->cc.moff), P_<int32_t>(ctx->cc.mem), P_<i64>(ctx->aloff),
                     P_<int32_t>(ctx->alist)};
}

// launch: false -- allocate only (the caller launches k_pol_pods' blocks
// inside k_pods_scatter)
int build_alist(kano_ctx* ctx, hipStream_t st = nullptr, bool launch = true) {
  const i64 P = ctx->P;
  KTRY(dalloc(ctx, ctx->alist, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_alw)));
  if (launch && P > 0 && ctx->cc.U > 0) {
    hipLaunchKernelGGL(k_pol_pods, dim3(nblk(P, WPB)), dim3(TPB), 0, st ? st : ctx->stream,
                       pol_pods_args(ctx));
    KLAUNCH();
  }
  ctx->alist_valid = true;
  return 0;
}

// the part of the back end that needs only the class counts: zeroed AC,
// Mc, cursors and class-level column words, then the caller's fills and
// launches (kano_verify: the crosscheck's group keys) -- queued while the
// list sizes travel to the host
// AC[p] built whole in a wave's LDS row (pol_allow_item's lds_row form: at
// most 32 KB a block, so that the launch fits beside a wide k_rows_w block):
// every row is stored whole, so AC needs no zero fill
bool ac_whole_rows(const kano_ctx* ctx) {
  return ctx->ac_lds && ctx->P > 0 && ctx->cc.U > 0 &&
         sizeof(u64) * (size_t)ctx->ldC * WPB <= 32 * 1024;
}

using PreLaunch = std::function<int(FillBatch&)>;
using PreRun = std::function<int(hipStream_t)>;
// With the side work forked (ev_pre, recorded after the classes), all of it
// runs on stream2 beside the join chain and do_back joins it (ev_pre_done).
int do_back_pre(kano_ctx* ctx, const PreLaunch& pre_fill, const PreRun& pre_run) {
  const i64 U = ctx->rc.U, P = ctx->P, ldMc = ctx->ldC;
  const bool side = ctx->pre_forked;
  ctx->pre_forked = false;
  hipStream_t ss = side ? ctx->stream2 : nullptr;
  if (side) KCHK(hipStreamWaitEvent(ss, ctx->ev_pre, 0));
  KTRY(dalloc(ctx, ctx->AC, sizeof(u64) * std::max<i64>(1, P * ctx->ldC)));
  KTRY(dalloc(ctx, ctx->Mc, sizeof(u64) * std::max<i64>(1, U * ldMc)));
  KTRY(dalloc(ctx, ctx->col_or_c, sizeof(u64) * ldMc));
  KTRY(dalloc(ctx, ctx->col_nand_c, sizeof(u64) * ldMc));
  // (AC written whole by its builder: no fill, no join before the lists)
  const bool ac_fill = !ac_whole_rows(ctx);
  if (side && ac_fill) {   // AC first: the lists' launch needs it before anything else here
    FillBatch fa(ctx, ss);
    KTRY(fa.add(ctx->AC, sizeof(u64) * P * ctx->ldC, 0u));
    KTRY(fa.run());
    KCHK(hipEventRecord(ctx->ev_pre_ac, ss));
    ctx->pre_ac_pending = true;
  }
  {
    FillBatch fb(ctx, ss);
    if (!side && ac_fill) KTRY(fb.add(ctx->AC, sizeof(u64) * P * ctx->ldC, 0u));
    KTRY(fb.add(ctx->Mc, sizeof(u64) * U * ldMc, 0u));
    KTRY(fb.add(ctx->col_or_c, sizeof(u64) * ldMc, 0u));
    KTRY(fb.add(ctx->col_nand_c, sizeof(u64) * ldMc, 0u));
    if (pre_fill) KTRY(pre_fill(fb));
    KTRY(fb.run());
  }
  if (pre_run) KTRY(pre_run(ss));
  if (side) {
    KCHK(hipEventRecord(ctx->ev_pre_done, ss));
    ctx->pre_side_pending = true;
  }
  return 0;
}

// lists (S(c) ascending, allowed classes + bits + pods per policy, heavy
// list) and the compressed matrix Mc (row classes x column classes): light
// classes by scatter, heavy classes by bitwise OR or the fp4 MFMA
// contraction; column checks at class level
// the engine stream waits for e -- unless e has completed already: a wait
// packet on a done event still held the stream ~5 us (the side work's joins)
int join_event(kano_ctx* ctx, hipEvent_t e) {
  const hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return 0;
  if (q != hipErrorNotReady) KCHK(q);
  KCHK(hipStreamWaitEvent(ctx->stream, e, 0));
  return 0;
}

// S(c) of the dense path, ascending, from the class-indexed bits
int sel_place_dx(kano_ctx* ctx, i64 cap) {
  const i64 U = ctx->rc.U;
  // (ecls feeds only the scatter form of Mc, taken by rows wider than the
  // owner form's LDS: see do_back)
  const bool need_ecls = (size_t)ctx->ldC * 8 * (TPB / 64) > 64 * 1024;
  hipLaunchKernelGGL(k_sel_lists_dx, dim3(nblk(U, WPB)), dim3(TPB),
                     sizeof(int32_t) * WPB * SEL_DX_BUF, ctx->stream, P_<u64>(ctx->dx_sa),
                     ctx->dx_ldY, ctx->PB, U, P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist),
                     need_ecls ? P_<int32_t>(ctx->ecls) : (int32_t*)nullptr, cap);
  KLAUNCH();
  return 0;
}

int do_back(kano_ctx* ctx, int path, const std::function<int(FillBatch&)>& extra) {
  const i64 U = ctx->rc.U, P = ctx->P, H = ctx->heavy_count, ldMc = ctx->ldC;
  // the dense contraction's kernel: the tiled GEMM when it has enough wave
  // tiles to fill the chip without a split, else the split-K kernel
  auto wave_tiles = [&](int tm, int tn) {
    return ((H + 32 * tm - 1) / (32 * tm)) * ((ctx->cc.U + 32 * tn - 1) / (32 * tn));
  };
  // (2 x 2 wave tiles: 64 KB of LDS and 140 registers a wave, so two blocks
  // share a CU -- as fast as 4 x 4 alone, and 0.47 -> 0.39 ms in D1's step,
  // where the previous step's heavy-row write holds part of every CU;
  // profiles/r06_f4/d1_tile_ab.jsonl)
  int hg = ctx->heavy_gemm;
  if (hg < 0) hg = 22;
  const int tmg = hg / 10, tng = hg % 10;
  const i64 gtiles = tmg > 0 ? wave_tiles(tmg, tng) : 0;
  const bool gemm_fits = tmg > 0 && (ctx->PB + GK_KC) * 8 * (TPB / 64) <= 64 * 1024 &&
                         gtiles >= ctx->heavy_gemm_min;
  ctx->heavy_path = 0;
  bool mfma = false;
  if (H > 0) {
    mfma = path == KANO_PATH_MFMA;
    if (path == KANO_PATH_AUTO) {
      if (gemm_fits) {
        // the MFMA does 2 H P Ua ops whatever the density, the OR reads
        // ldMc words per (heavy class, policy in S(c)): the cheaper by the
        // measured rates ("The dense path: crossover")
        // (the GEMM's rate falls below ~2,048 wave tiles: the 2 x 2 tile at
        // H = Ua = 2,000, 1,024 tiles, 2,190 TOP/s against 4,670 at 8,000)
        const double fill = std::pow(std::min(1.0, (double)gtiles / 2048.0), 0.85);
        const double t_mfma =
            2.0 * (double)H * (double)P * (double)ctx->cc.U / (ctx->xo_mfma * fill);
        const double t_or = 8.0 * (double)ctx->heavy_sel * (double)ldMc / ctx->xo_or;
        mfma = t_mfma < t_or;
      } else {
        // (the split-K kernel, few heavy rows: dense when the average |S(c)|
        // is a large share of P)
        const double avg_s = (double)ctx->nnz_sel / std::max<i64>(1, U);
        mfma = H >= 32 && ctx->cc.U >= 64 && avg_s * 16.0 >= (double)P;
      }
    }
    ctx->heavy_path = mfma ? 2 : 1;
  }
  const bool gemm = mfma && gemm_fits;
  ctx->heavy_kernel = H == 0 ? 0 : !mfma ? 1 : gemm ? 3 : 2;
  // the staged GEMM's padded operands (k_heavy_gemm_f4): A [PBp][ldA],
  // ACT [PBp][ldB]; the unstaged kernels use ldA = H, ldB = Ua, PBp = PB
  const bool glds = gemm;
  const i64 ldA0 = glds ? (H + 64 * tmg - 1) / (64 * tmg) * (64 * tmg) : H;
  // (every class heavy on the dense path: A is SA as it stands -- zero past
  // U, pitch dx_ldY -- when that pitch is a whole number of block tiles; no
  // gather)
  const bool a_is_sa = glds && ctx->dense_sel && H == U && ctx->dx_ldY >= ldA0 &&
                       ctx->dx_ldY % (64 * tmg) == 0;
  const i64 ldA = a_is_sa ? ctx->dx_ldY : ldA0;
  const i64 ldB = glds ? (ctx->cc.U + 64 * tng - 1) / (64 * tng) * (64 * tng) : ctx->cc.U;
  const i64 PBp = glds ? (ctx->PB + GK_KC - 1) / GK_KC * GK_KC : ctx->PB;
  // k_sel_place went out before the sizes (sel_place_early): kept when the
  // list fitted its capacity, else the sized placement below, on zeroed
  // cursors, once the early one has ended
  const bool early_ok = ctx->sel_early_cap >= 0 && ctx->nnz_sel <= ctx->sel_early_cap;
  if (ctx->sel_early_cap >= 0 && !early_ok) {
    KCHK(hipStreamSynchronize(ctx->stream));
    KCHK(hipMemsetAsync(ctx->scur.p, 0, sizeof(int32_t) * std::max<i64>(1, U), ctx->stream));
  }
  ctx->sel_early_cap = -1;
  FillJobs carried{};
  {
    FillBatch fb(ctx);
    KTRY(dalloc(ctx, ctx->slist, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_sel)));
    KTRY(dalloc(ctx, ctx->ecls, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_sel)));
    KTRY(dalloc(ctx, ctx->alc, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_alc)));
    KTRY(dalloc(ctx, ctx->hlist, sizeof(int32_t) * std::max<i64>(1, H)));
    KTRY(dalloc(ctx, ctx->wicls, sizeof(int32_t) * std::max<i64>(1, ctx->wi_total)));
    if (mfma) {
      KTRY(dalloc(ctx, ctx->ACT, sizeof(u64) * std::max<i64>(1, PBp * ldB)));
      if (!ctx->dense_sel) KTRY(fb.add(ctx->ACT, sizeof(u64) * PBp * ldB, 0u));
      // (the GEMM's A is written whole, padding included, by k_heavy_selT: no fill)
      const i64 aw = gemm ? PBp * ldA : ctx->PB * U;
      KTRY(dalloc(ctx, ctx->scratch_words, sizeof(u64) * std::max<i64>(1, aw)));
      if (!gemm) KTRY(fb.add(ctx->scratch_words, sizeof(u64) * ctx->PB * U, 0u));
    }
    if (extra) KTRY(extra(fb));   // the caller's fills (kano_verify: crosscheck, shadow)
    // (carried by k_sel_place's launch -- or by the lists' launch after an
    // early placement -- neither of which reads or writes them)
    if (U > 0 && P > 0) carried = fb.take();
    else KTRY(fb.run());
  }
  if (U > 0 && P > 0 && !early_ok && ctx->dense_sel) {
    KTRY(sel_place_dx(ctx, std::max<i64>(1, ctx->nnz_sel)));
  } else if (U > 0 && P > 0 && !early_ok) {
    const unsigned nbs = nblk(P, sel_spb(ctx)), nbf = fill_ride_blocks(carried);
    hipLaunchKernelGGL(k_sel_place, dim3(nbs + nbf), dim3(TPB), 0, ctx->stream, P,
                       P_<i64>(ctx->sm.pstart), P_<int32_t>(ctx->sm.plen),
                       P_<int32_t>(ctx->sm.gmem), P_<i64>(ctx->soffc), P_<int32_t>(ctx->scur),
                       P_<int32_t>(ctx->slist), P_<int32_t>(ctx->ecls), sel_spb(ctx), carried, nbs,
                       std::max<i64>(1, ctx->nnz_sel));
    KLAUNCH();
    carried = FillJobs{};
  }
  // S(c) sorted, heavy list and work-item map (k_class_lists) and the
  // allowed classes + bits per policy (k_pol_allow_fill): independent, one
  // launch when both run
  const bool lists_on = U > 0, allow_on = P > 0 && ctx->cc.U > 0;
  // (the long lists' sort: bitmap windows of at most SORT_LDS_WW words per wave)
  const i64 sort_pw = (P + 63) / 64, sort_ww = std::min<i64>(sort_pw, ctx->sort_ww);
  const bool sort_on = P > 0 && !ctx->dense_sel;   // (the dense lists come sorted)
  const bool sort_big = sort_on && ctx->max_sel > SORT_WAVE_MAX;
  if (sort_big && sort_pw > sort_ww)
    KTRY(dalloc(ctx, ctx->slist_tmp, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_sel)));
  const ClassListsArgs cla{P_<i64>(ctx->soffc), U, P, P_<int32_t>(ctx->slist), sort_on ? 1 : 0,
                           P_<int32_t>(ctx->hflag), P_<int32_t>(ctx->hoff), P_<int32_t>(ctx->hlist),
                           P_<int32_t>(ctx->wioff), P_<int32_t>(ctx->wicls), std::max<i64>(1, sort_ww),
                           P_<int32_t>(ctx->slist_tmp)};
  const PolAllowArgs paa{P, P_<i64>(ctx->am.pstart), P_<int32_t>(ctx->am.plen),
                         P_<int32_t>(ctx->am.gmem), P_<i64>(ctx->alcoff), P_<int32_t>(ctx->alc),
                         P_<u64>(ctx->AC), ctx->ldC};
  size_t lds = sort_big ? sizeof(u64) * (size_t)sort_ww * (TPB / 64) : 0;
  // AC[p] built in the wave's LDS row when the rows fit (k_pol_allow; at
  // most 32 KB, so that the launch fits beside a wide k_rows_w block)
  const size_t ac_lds = sizeof(u64) * (size_t)ctx->ldC * WPB;
  const int ac_rows = ac_whole_rows(ctx) ? 1 : 0;   // (do_back_pre skipped AC's fill)
  if (ac_rows) lds = std::max(lds, ac_lds);
  // the side work's joins: AC zeroed before the lists, the rest (Mc, the
  // crosscheck's fills and key sort) before the Mc writers below
  if (ctx->pre_ac_pending) {
    ctx->pre_ac_pending = false;
    KTRY(join_event(ctx, ctx->ev_pre_ac));
  }
  // (the fork point of kano_verify's side stream, when it has one: marked by
  // this dispatch itself, not by a separate event record)
  hipEvent_t fev = ctx->fork_hook ? ctx->ev_fork2 : nullptr;
  if (!(lists_on && allow_on) && carried.count > 0) {
    hipLaunchKernelGGL(k_fill_many, dim3(fill_ride_blocks(carried)), dim3(TPB), 0, ctx->stream,
                       carried);
    KLAUNCH();
    carried = FillJobs{};
  }
  if (lists_on && allow_on) {
    const unsigned nb1 = nblk(U, TPB / 64), nb2 = nblk(P, WPB);
    launch_marked(k_lists_allow, dim3(nb1 + nb2 + fill_ride_blocks(carried)), dim3(TPB), lds,
                  ctx->stream, fev, cla, paa, nb1, nb2, carried, ac_rows);
    KLAUNCH();
  } else if (lists_on) {
    launch_marked(k_class_lists, dim3(nblk(U, TPB / 64)), dim3(TPB), lds, ctx->stream, fev, cla);
    KLAUNCH();
  } else if (allow_on) {
    launch_marked(k_pol_allow_fill, dim3(nblk(P, WPB)), dim3(TPB), ac_rows ? ac_lds : 0,
                  ctx->stream, fev, paa, ac_rows);
    KLAUNCH();
  } else {
    fev = nullptr;
  }
  const bool fork_marked = fev != nullptr;   // (the hook runs at the end: the
                                             // engine stream's launches go first)
  if (ctx->pre_side_pending) {
    ctx->pre_side_pending = false;
    KTRY(join_event(ctx, ctx->ev_pre_done));
  }
  // Light rows read either the flat allowed-pod lists (materialised here,
  // one pass over nnz_alw entries) or the column-class member lists (n
  // entries, cache-resident).  The flat lists win wherever the light rows
  // read them at all (measured: C3 at 1/8 of the rows k_rows 99 -> 49 us; C5
  // 21.8 -> 20.9 ms); where nearly every class is heavy (C4) building them
  // is pure cost (+0.45 ms a step)
  ctx->alist_valid = false;
  ctx->rows_use_alist = ctx->light_cost > 0 && ctx->light_cost * 16 > ctx->nnz_alw &&
                        ctx->nnz_alw * 4 <= (2ll << 30);
  // (k_pol_pods' blocks ride in the Mc launch when both run)
  const McScatterArgs msa{ctx->nnz_sel, P_<int32_t>(ctx->ecls), P_<int32_t>(ctx->slist),
                          P_<i64>(ctx->alcoff), P_<int32_t>(ctx->alc), P_<int32_t>(ctx->rc.mcnt),
                          H > 0 ? P_<int32_t>(ctx->hflag) : (const int32_t*)nullptr,
                          P_<u64>(ctx->Mc), ldMc};
  const bool scatter_on = U > 0 && ctx->nnz_sel > 0;
  const bool pods_in_scatter = ctx->rows_use_alist && scatter_on && P > 0 && ctx->cc.U > 0;
  if (ctx->rows_use_alist) KTRY(build_alist(ctx, nullptr, !pods_in_scatter));
  ctx->rin_marked = false;
  if (U == 0) return ctx->fork_hook ? ctx->fork_hook(fork_marked) : 0;
  // (with no heavy rows and the column checks deferred, the owner launch
  // below is the last producer of every k_rows input: its dispatch marks
  // ev_rin_e, where kano_verify's write may start -- beside this call's tail
  // instead of behind it)
  hipEvent_t rin_mark = H == 0 && ctx->cols_deferred ? ctx->ev_rin_e : nullptr;
  if (scatter_on && (size_t)ldMc * 8 * (TPB / 64) <= 64 * 1024) {
    // light Mc rows by their owner (a wave per row class, the row in LDS,
    // plain stores)
    const size_t lds = sizeof(u64) * (size_t)ldMc * (TPB / 64);
    const McOwnArgs moa{U, P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), P_<i64>(ctx->alcoff),
                        P_<int32_t>(ctx->alc), P_<int32_t>(ctx->rc.mcnt),
                        H > 0 ? P_<int32_t>(ctx->hflag) : (const int32_t*)nullptr,
                        P_<u64>(ctx->Mc), ldMc};
    if (pods_in_scatter) {
      const unsigned nb1 = nblk(P, WPB);
      hipExtLaunchKernelGGL(k_pods_own, dim3(nb1 + nblk(U, TPB / 64)), dim3(TPB), lds,
                            ctx->stream, nullptr, rin_mark, 0, pol_pods_args(ctx), moa, nb1);
    } else {
      hipExtLaunchKernelGGL(k_mc_own, dim3(nblk(U, TPB / 64)), dim3(TPB), lds, ctx->stream,
                            nullptr, rin_mark, 0, moa);
    }
    KLAUNCH();
    ctx->rin_marked = rin_mark != nullptr;
  } else if (scatter_on) {
    // very wide class-level rows: the select entries' allowed classes OR-ed
    // into Mc with atomics (one wave per select entry)
    if (pods_in_scatter) {
      const unsigned nb1 = nblk(P, WPB);
      hipExtLaunchKernelGGL(k_pods_scatter, dim3(nb1 + nblk(ctx->nnz_sel, TPB / 64)), dim3(TPB),
                            0, ctx->stream, nullptr, rin_mark, 0, pol_pods_args(ctx), msa, nb1);
    } else {
      hipExtLaunchKernelGGL(k_mc_scatter, dim3(nblk(ctx->nnz_sel, TPB / 64)), dim3(TPB), 0,
                            ctx->stream, nullptr, rin_mark, 0, msa);
    }
    KLAUNCH();
    ctx->rin_marked = rin_mark != nullptr;
  }
  if (H > 0) {
    if (mfma) {
      const i64 Ua = ctx->cc.U;
      if (ctx->dense_sel) {
        // (ACT = AC's 64 x 64 bit blocks transposed: every word written)
        hipLaunchKernelGGL(k_ptrans, dim3(nblk(PBp * ((ldB + 63) / 64), WPB)), dim3(TPB), 0,
                           ctx->stream, P_<u64>(ctx->AC), ctx->ldC, P, P_<u64>(ctx->ACT), ldB,
                           PBp, (const int32_t*)nullptr);
      } else {
        // (the contraction without the dense front end: forced, or past
        // DX_MAX row classes)
        hipLaunchKernelGGL(k_classbits, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                           P_<i64>(ctx->am.pstart), P_<int32_t>(ctx->am.plen),
                           P_<int32_t>(ctx->am.gmem), ldB, P_<u64>(ctx->ACT));
      }
      KLAUNCH();
      // class-major selector bits: selT[pb][c] (the split-K kernel's A; the
      // GEMM builds its own, heavy rows only)
      if (!gemm) {
        hipLaunchKernelGGL(k_classbits, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                           P_<i64>(ctx->sm.pstart), P_<int32_t>(ctx->sm.plen),
                           P_<int32_t>(ctx->sm.gmem), U, P_<u64>(ctx->scratch_words));
        KLAUNCH();
      }
      const u64* selT = P_<u64>(ctx->scratch_words);
      uint32_t* out = reinterpret_cast<uint32_t*>(P_<u64>(ctx->Mc));
      if (gemm) {
        // many heavy rows: the tiled GEMM, no split-K, on the heavy rows'
        // own select bits (A, from the sorted S(c) lists)
        const i64 nb = ((H + 64 * tmg - 1) / (64 * tmg)) * ((Ua + 64 * tng - 1) / (64 * tng));
        const dim3 grid((unsigned)(8 * ((nb + 7) / 8)));
        const int32_t* hl = P_<int32_t>(ctx->hlist);
        u64* A = P_<u64>(ctx->scratch_words);
        if (a_is_sa && PBp == ctx->dx_PBo) {
          A = P_<u64>(ctx->dx_sa);   // every class heavy: SA is A as it stands
        } else if (ctx->dense_sel) {
          hipLaunchKernelGGL(k_sa_gather, dim3(nblk(PBp * ldA)), dim3(TPB), 0, ctx->stream,
                             P_<u64>(ctx->dx_sa), ctx->dx_ldY, hl, H, PBp, A, ldA);
          KLAUNCH();
        } else {
          hipLaunchKernelGGL(k_heavy_selT, dim3(nblk(ldA, TPB / 64)), dim3(TPB),
                             sizeof(u64) * (size_t)PBp * (TPB / 64), ctx->stream, hl, H, ldA,
                             P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), PBp, A);
          KLAUNCH();
        }
        KTRY(resolve_mfma_time(ctx));
        KCHK(hipEventRecord(ctx->ev_m0, ctx->stream));
        {
          const size_t lds =
              sizeof(u64) * 2 * gemm_kc(tmg, tng) * (size_t)(64 * tmg + 64 * tng);
          if (hg == 22)
            hipLaunchKernelGGL((k_heavy_gemm_f4<2, 2, gemm_kc(2, 2)>), grid, dim3(TPB), lds, ctx->stream, A,
                               ldA, hl, H, P_<u64>(ctx->ACT), ldB, Ua, PBp, out, ldMc);
          else if (hg == 44)
            hipLaunchKernelGGL((k_heavy_gemm_f4<4, 4, gemm_kc(4, 4)>), grid, dim3(TPB), lds, ctx->stream, A,
                               ldA, hl, H, P_<u64>(ctx->ACT), ldB, Ua, PBp, out, ldMc);
          else
            hipLaunchKernelGGL((k_heavy_gemm_f4<4, 2, gemm_kc(4, 2)>), grid, dim3(TPB), lds, ctx->stream, A,
                               ldA, hl, H, P_<u64>(ctx->ACT), ldB, Ua, PBp, out, ldMc);
        }
        KLAUNCH();
        KCHK(hipEventRecord(ctx->ev_m1, ctx->stream));
        ctx->mfma_time_pending = true;
        ctx->mfma_ops_last = 2.0 * (double)H * (double)P * (double)Ua;
      } else {
      // split K (policy blocks) so that the launch has ~2048 waves whatever
      // the number of 32-column tiles
      const i64 tiles = 2 * ldMc;
      // (at least MFMA_KMIN policy blocks per wave: the epilogue, 16 ballots
      // and OR-atomics per 32-row tile, must not dominate)
      const i64 ksplit = std::max<i64>(
          1, std::min<i64>((ctx->PB + MFMA_KMIN - 1) / MFMA_KMIN, 2048 / std::max<i64>(1, tiles)));
      const i64 kchunk = (ctx->PB + ksplit - 1) / ksplit;
      const unsigned gy = (unsigned)((ctx->PB + kchunk - 1) / kchunk);
      KTRY(resolve_mfma_time(ctx));
      KCHK(hipEventRecord(ctx->ev_m0, ctx->stream));
      for (i64 h0 = 0; h0 < H; h0 += HT_ROWS) {
        const int hh = (int)std::min<i64>(HT_ROWS, H - h0);
        const int32_t* hl = P_<int32_t>(ctx->hlist) + h0;
        dim3 grid(nblk(tiles, TPB / 64), gy);
        if (hh <= 32)
          hipLaunchKernelGGL(k_heavy_mc_mfma<1>, grid, dim3(TPB), 0, ctx->stream, selT, U, hl, hh,
                             P_<u64>(ctx->ACT), Ua, ctx->PB, out, ldMc, kchunk);
        else if (hh <= 64)
          hipLaunchKernelGGL(k_heavy_mc_mfma<2>, grid, dim3(TPB), 0, ctx->stream, selT, U, hl, hh,
                             P_<u64>(ctx->ACT), Ua, ctx->PB, out, ldMc, kchunk);
        else
          hipLaunchKernelGGL(k_heavy_mc_mfma<4>, grid, dim3(TPB), 0, ctx->stream, selT, U, hl, hh,
                             P_<u64>(ctx->ACT), Ua, ctx->PB, out, ldMc, kchunk);
        KLAUNCH();
      }
      KCHK(hipEventRecord(ctx->ev_m1, ctx->stream));
      ctx->mfma_time_pending = true;
      // algorithmic work: the heavy rows' boolean product over every policy,
      // 2 ops (multiply, add) per (row class, policy, column class)
      ctx->mfma_ops_last = 2.0 * (double)H * (double)P * (double)Ua;
      }
    } else {
      // (timed like the contraction when asked, hortime=1: the same
      // algorithmic work, for the dense-path crossover, scripts/mfma_sweep.py)
      if (ctx->time_or) {
        KTRY(resolve_mfma_time(ctx));
        KCHK(hipEventRecord(ctx->ev_m0, ctx->stream));
      }
      hipLaunchKernelGGL(k_heavy_mc_or, dim3((unsigned)H, nblk(ldMc, 64)), dim3(TPB), 0, ctx->stream,
                         P_<int32_t>(ctx->hlist), P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist),
                         P_<u64>(ctx->AC), ctx->ldC, ctx->UAW, P_<u64>(ctx->Mc), ldMc);
      KLAUNCH();
      if (ctx->time_or) {
        KCHK(hipEventRecord(ctx->ev_m1, ctx->stream));
        ctx->mfma_time_pending = true;
        ctx->mfma_ops_last = 2.0 * (double)H * (double)P * (double)ctx->cc.U;
      }
    }
    // (the heavy rows' Mc was the write's last input: kano_verify's write
    // may start here, beside the crosscheck pass and the tail -- C5's 5 ms
    // PCIe copy of the pairs, until now in front of a 19 ms write).  rheavy=2
    // (default): only for a wide-row write; C3's 0.35 ms write beside the
    // tail measured 1% slower (profiles/r05_c5_rheavy_ab)
    const bool early = ctx->rows_early_heavy == 1 ||
                       (ctx->rows_early_heavy == 2 &&
                        std::min<i64>(ctx->ldM, ctx->rows_cww) > 4096);
    if (early && ctx->cols_deferred && !ctx->rin_marked) {
      KCHK(hipEventRecord(ctx->ev_rin_e, ctx->stream));
      ctx->rin_marked = true;
    }
  }
  if (!ctx->cols_deferred) KTRY(mc_cols(ctx));
  // kano_verify's side stream forks from the lists (ev_fork2)
  if (ctx->fork_hook) KTRY(ctx->fork_hook(fork_marked));
  return 0;
}

// heavy rows expanded from Mc into the first member's row; then the rows
int do_rows(kano_ctx* ctx) {
  const i64 ldM = ctx->ldM, n = ctx->n;
  if (n > 0) {
    hipLaunchKernelGGL(k_cols_expand, dim3(nblk(ldM * 64)), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->col_or_c), P_<u64>(ctx->col_nand_c), P_<int32_t>(ctx->cc.cls),
                       n, ldM, P_<u64>(ctx->color), P_<u64>(ctx->colnand));
    KLAUNCH();
  } else {
    KCHK(hipMemsetAsync(ctx->color.p, 0, sizeof(u64) * ldM, ctx->stream));
    KCHK(hipMemsetAsync(ctx->colnand.p, 0, sizeof(u64) * ldM, ctx->stream));
  }
  return 0;
}

// The matrix write, timed by its own dispatch (hipExtLaunchKernelGGL's start
// / stop events ev_rt[set]: no marker packets around it; the bench's
// roofline reads them through kano_rows_timing): heavy rows expanded from
// Mc first, then every light class row rebuilt from the allowed-pod lists
// in LDS and streamed to its members (k_rows).  It runs on stream3 behind
// the engine stream's marker ev_rin; unless rows_overlap (kano_verify's
// asynchronous completion) the engine stream then waits for it.
// The CU-masked write stream (~15 ms to create; it serves only the
// pipelined kano_verify steps: kano_create_lean skips it)
thread_local bool g_create_lean = false;
void rows_cu_mask(int K, uint32_t* mask) {
  const int t = K < 4 ? 1 : K / 4, beta = K < 4 ? K : 4;
  for (int w = 0; w < 8; ++w) {
    mask[w] = 0xffffffffu;
    for (int bit = 0; bit < 32; ++bit) {
      const int i = w * 32 + bit, a = i / 32, b = (i / 8) % 4, c = i % 8;
      if (((c - a) & 7) < t && b < beta) mask[w] &= ~(1u << bit);
    }
  }
}
int ensure_masked_stream(kano_ctx* ctx) {
  if (ctx->stream3m || ctx->stream3m_tried || ctx->rows_cu_off <= 0) return 0;
  ctx->stream3m_tried = true;
  // bit i = 32a + 8b + c off when (c - a) mod 8 < t and b < beta, K = t * beta:
  // K CUs of every XCD whether the CUs are numbered XCD-major (XCD a) or
  // round-robin (XCD c)
  uint32_t mask[8];
  rows_cu_mask(ctx->rows_cu_off, mask);
  // (no masked stream: every write takes stream3)
  if (hipExtStreamCreateWithCUMask(&ctx->stream3m, 8, mask) != hipSuccess) ctx->stream3m = nullptr;
  return 0;
}

// CUs of XCDs [x0, x1) (CU i on XCD i / 32: the masks' numbering, measured --
// the round-robin reading gave the write every CU's time)
void xcd_mask(int x0, int x1, uint32_t* mask) {
  for (int w = 0; w < 8; ++w) mask[w] = (w >= x0 && w < x1) ? 0xffffffffu : 0u;
}
int ensure_xcd_streams(kano_ctx* ctx) {
  if (ctx->stream_x || ctx->xcd_tried) return 0;
  ctx->xcd_tried = true;
  uint32_t wm[8], em[8], am[8];
  xcd_mask(0, ctx->xcd_write, wm);
  xcd_mask(ctx->xcd_eng0 < 0 ? ctx->xcd_write : ctx->xcd_eng0, 8, em);
  xcd_mask(0, 8, am);
  hipStream_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  if (hipExtStreamCreateWithCUMask(&a, 8, em) != hipSuccess ||
      hipExtStreamCreateWithCUMask(&b, 8, em) != hipSuccess ||
      hipExtStreamCreateWithCUMask(&c, 8, wm) != hipSuccess ||
      hipExtStreamCreateWithCUMask(&d, 8, am) != hipSuccess) {
    for (hipStream_t x : {a, b, c, d})
      if (x) (void)hipStreamDestroy(x);
    return 0;   // (no split: the spread mask stays)
  }
  ctx->stream_x = a;
  ctx->stream2_x = b;
  ctx->stream3x = c;
  ctx->stream2_u = d;
  return 0;
}
// The engine streams for the build about to start (front_a): the engine
// stream on XCDs 3-7 when the last build qualified; the side stream with it
// when that build had heavy classes, else on a stream masked to every XCD
// (C3, no heavy classes: 5 % faster; C4's heavy side work beside the write on
// XCDs 0-2: 6 % slower, r06_xcd_side_ab.jsonl -- and the original unmasked
// side stream beside the masked ones: 0.64 ms, r06_xcd_side_auto_ab.jsonl).
// A switch orders the new streams behind everything queued on the old ones.
void side_swap(kano_ctx* ctx, int mode) {
  if (mode == 1) std::swap(ctx->stream2, ctx->stream2_x);
  if (mode == 2) std::swap(ctx->stream2, ctx->stream2_u);
}
int select_engine_streams(kano_ctx* ctx) {
  const bool want = ctx->xcd_split && ctx->own_stream && ctx->pipeline && ctx->xcd_last_ok &&
                    ctx->stream3m && ctx->num_cus == 256;
  if (want) KTRY(ensure_xcd_streams(ctx));
  const bool eng = want && ctx->stream_x;
  const bool heavy_side = ctx->xcd_side < 0 ? ctx->heavy_count > 0 : ctx->xcd_side == 1;
  const int side = !eng ? 0 : heavy_side ? 1 : 2;
  if (eng == ctx->eng_on_xcd && side == ctx->side_mode) return 0;
  KCHK(hipEventRecord(ctx->ev_sw, ctx->stream));
  KCHK(hipEventRecord(ctx->ev_sw2, ctx->stream2));
  if (eng != ctx->eng_on_xcd) std::swap(ctx->stream, ctx->stream_x);
  if (side != ctx->side_mode) {
    side_swap(ctx, ctx->side_mode);   // (back to stream2, then to the new one)
    side_swap(ctx, side);
  }
  for (hipStream_t t : {ctx->stream, ctx->stream2}) {
    KCHK(hipStreamWaitEvent(t, ctx->ev_sw, 0));
    KCHK(hipStreamWaitEvent(t, ctx->ev_sw2, 0));
  }
  ctx->eng_on_xcd = eng;
  ctx->side_mode = side;
  return 0;
}
// back to the unmasked streams, everything drained (kano_set_stream)
int leave_xcd_streams(kano_ctx* ctx) {
  if (!ctx->eng_on_xcd && !ctx->side_mode) return 0;
  for (hipStream_t t : {ctx->stream, ctx->stream2, ctx->stream_x, ctx->stream2_x, ctx->stream2_u})
    KCHK(hipStreamSynchronize(t));
  if (ctx->eng_on_xcd) std::swap(ctx->stream, ctx->stream_x);
  side_swap(ctx, ctx->side_mode);
  ctx->eng_on_xcd = false;
  ctx->side_mode = 0;
  return 0;
}

int launch_rows(kano_ctx* ctx) {
  const i64 U = ctx->rc.U, W = ctx->W, ldM = ctx->ldM, n = ctx->n;
  const i64 rl = rows_local(ctx);
  ctx->rows_kernel = 0;
  if (rl == 0 || W == 0) return 0;
  // (the CU mask only where the write overlaps the next call's build --
  // kano_verify's asynchronous completion; a write the caller waits for
  // takes every CU)
  const bool masked = ctx->rows_overlap && ctx->stream3m &&
                      (i64)sizeof(u64) * rl * ldM <= ctx->rows_cu_bytes;
  const bool on_xcd = masked && ctx->eng_on_xcd;
  hipStream_t rs = on_xcd ? ctx->stream3x : masked ? ctx->stream3m : ctx->stream3;
  ctx->rows_cus = on_xcd ? 32 * ctx->xcd_write : ctx->num_cus - (masked ? 8 * ctx->rows_cu_off : 0);
  // (the next build's streams: the split when this write is masked, large
  // enough to bound the step -- C3's and C4's 1.25 GB; a half-row shard's
  // 0.63 GB is shorter than the build beside it and measured +5 % with the
  // split -- and the build took no GEMM: the dense contraction wants every
  // XCD)
  ctx->xcd_last_ok = masked && ctx->heavy_kernel != 3 &&
                     (i64)sizeof(u64) * rl * ldM >= ctx->xcd_min_bytes;
  const int set = ctx->rows_set;
  // this set's pair was last used two writes back (ended: the engine stream
  // waited for it before this build wrote the set)
  KTRY(resolve_rows_slot(ctx, set, true));
  // (an event record costs the engine stream ~4.5 us: reuse one that stands
  // at the same place, e.g. the tail's copy-done event)
  hipEvent_t rin = ctx->rows_in;
  if (!rin) {
    KCHK(hipEventRecord(ctx->ev_rin, ctx->stream));
    rin = ctx->ev_rin;
  }
  if (ctx->wi_total == 0) return 0;
  KCHK(hipStreamWaitEvent(rs, rin, 0));
  // writes stay in order across the two write streams (M, the input sets)
  if (ctx->rows_last && ctx->rows_last != rs && ctx->rows_end_rec[set ^ 1])
    KCHK(hipStreamWaitEvent(rs, ctx->rows_end_ev[set ^ 1], 0));
  ctx->rows_last = rs;
  if (ctx->rows_after) KCHK(hipStreamWaitEvent(rs, ctx->rows_after, 0));
  hipEvent_t e0 = ctx->ev_rt[set][0], e1 = ctx->ev_rt[set][1];
  // (the write's time: from the first kernel's start to k_rows' end)
  hipEvent_t e0_rows = e0;
  bool heavy_whole = false, rows_needed = true, rows_wide_used = false;
  if (ctx->heavy_count > 0) {
    const i64 H = ctx->heavy_count, ldMc = ctx->ldC;
    {
      // the heavy classes' first member rows (hexplds=3: every member row,
      // k_rows then skips them) from McT (k_ptrans of their Mc rows) by
      // wave transposes
      const i64 HW = (H + 63) / 64, ldT = std::max<i64>(1, ctx->cc.U);
      KTRY(dalloc(ctx, ctx->mct, sizeof(u64) * (size_t)(HW * ldT)));
      hipExtLaunchKernelGGL(k_ptrans, dim3(nblk(HW * ((ldT + 63) / 64), WPB)), dim3(TPB), 0, rs,
                            e0, nullptr, 0, P_<u64>(ctx->Mc), ldMc, H, P_<u64>(ctx->mct), ldT,
                            HW, P_<int32_t>(ctx->hlist));
      KLAUNCH();
      e0_rows = nullptr;
      // (every member row: the members split over Z blocks, so that ~2,048
      // blocks run whatever the class sizes -- C4's 99 classes of ~1,000 pods)
      // whole (every member row) for small heavy classes (D1: 12.5 pods a
      // class, step 1.40 -> 1.32 ms), first rows + k_rows' copies for large
      // ones (C4: ~1,000 pods a class, 0.465 against 0.488 ms)
      const bool whole = ctx->heavy_expand_lds == 3 ||
                         (ctx->heavy_expand_lds == 2 && rows_local(ctx) <= 32 * H);
      const i64 nxy = (i64)nblk(ldM, HXB) * HW;
      const unsigned Z = whole ? (unsigned)std::min<i64>(64, std::max<i64>(1, 2048 / nxy)) : 1u;
      // (every class heavy and written whole: no k_rows, this launch ends the write)
      const bool last = whole && H == U;
      hipExtLaunchKernelGGL(k_heavy_rows_t, dim3(nblk(ldM, HXB), (unsigned)HW, Z), dim3(TPB), 0,
                            rs, nullptr, last ? e1 : nullptr, 0, P_<u64>(ctx->mct), ldT,
                            P_<int32_t>(ctx->hlist), H, P_<int32_t>(ctx->cc.cls), n,
                            P_<int32_t>(ctx->rc.moff), P_<int32_t>(ctx->rc.mem), P_<u64>(ctx->M),
                            ldM, ctx->r0, whole ? 0 : 1);
      KLAUNCH();
      heavy_whole = whole;
      rows_needed = !last;
    }
    KLAUNCH();
  }
  const int cww = (int)std::min<i64>(ldM, ctx->rows_cww);
  const unsigned ncc = (unsigned)((ldM + cww - 1) / cww);
  RowsArgs a{};
  a.wioff = P_<int32_t>(ctx->wioff);
  a.wicls = P_<int32_t>(ctx->wicls);
  a.U = U;
  a.soffc = P_<i64>(ctx->soffc);
  a.slist = P_<int32_t>(ctx->slist);
  a.aloff = ctx->rows_use_alist ? P_<i64>(ctx->aloff) : nullptr;
  a.alist = ctx->rows_use_alist ? P_<int32_t>(ctx->alist) : nullptr;
  a.alcoff = P_<i64>(ctx->alcoff);
  a.alc = P_<int32_t>(ctx->alc);
  a.cmoff = P_<int32_t>(ctx->cc.moff);
  a.cmem = P_<int32_t>(ctx->cc.mem);
  a.moff = P_<int32_t>(ctx->rc.moff);
  a.mem = P_<int32_t>(ctx->rc.mem);
  a.hflag = ctx->heavy_count > 0 ? P_<int32_t>(ctx->hflag) : nullptr;
  a.M = P_<u64>(ctx->M);
  a.ldM = ldM;
  a.wW = ldM;
  a.r0 = ctx->r0;
  a.n = n;
  a.W = W;
  a.ch = ctx->rows_ch;
  a.cww = cww;
  a.color = nullptr;  // column checks come from Mc
  a.colnand = nullptr;
  a.heavy_skip = heavy_whole ? 1 : 0;
  // wide chunks hold few blocks per CU (LDS): give those blocks more waves
  const int nt = cww > 4096 ? 1024 : (cww > 2048 ? 512 : 256);
  const size_t lds = sizeof(u64) * cww;
  const dim3 grid((unsigned)ctx->wi_total, ncc);
  if (!rows_needed) {
    // (the heavy rows' launch carries the write's stop event)
  } else if ((nt == 1024 || ctx->rows_wide == 2) && ctx->rows_wide && a.alist &&
             ctx->rows_ch <= 64) {
    rows_wide_used = true;
    // wide chunks: the items' chains resolved ahead (k_rows_prep), then
    // persistent blocks (one per CU, or rwg: a grid of that many, the parity
    // variants' multi-unit blocks) drawing (item, chunk) units by ticket
    const i64 nitems = ctx->wi_total;
    KTRY(dalloc(ctx, ctx->rw_items, sizeof(RowsItem) * (size_t)nitems));
    KTRY(dalloc(ctx, ctx->rw_segs, sizeof(RowsSeg) * (size_t)std::max<i64>(1, ctx->nnz_sel)));
    RowsItem* items = P_<RowsItem>(ctx->rw_items);
    RowsSeg* segs = P_<RowsSeg>(ctx->rw_segs);
    const i64 per_cu = lds <= 72 * 1024 ? 2 : 1;
    const i64 slots = ctx->rows_w_grid > 0 ? ctx->rows_w_grid : per_cu * ctx->rows_cus;
    const i64 nunits = nitems * (i64)ncc;
    const bool persist = nunits > slots;
    int32_t* ticket = nullptr;
    if (persist) {
      KTRY(dalloc(ctx, ctx->rw_ticket, sizeof(int32_t)));
      ticket = P_<int32_t>(ctx->rw_ticket);
    }
    hipLaunchKernelGGL(k_rows_prep, dim3(nblk(nitems, TPB / 64)), dim3(TPB), 0, rs, a, nitems,
                       items, segs, ticket);
    KLAUNCH();
    const unsigned gx = (unsigned)(persist ? slots : nunits);
    hipExtLaunchKernelGGL(k_rows_w<1024>, dim3(gx), dim3(1024), lds, rs, e0_rows, e1, 0, a,
                          (const RowsItem*)items, nitems, (const RowsSeg*)segs, ticket,
                          (int)ncc);
  } else if (nt == 1024) {
    hipExtLaunchKernelGGL(k_rows<1024>, grid, dim3(1024), lds, rs, e0_rows, e1, 0, a);
  } else if (nt == 512) {
    hipExtLaunchKernelGGL(k_rows<512>, grid, dim3(512), lds, rs, e0_rows, e1, 0, a);
  } else {
    hipExtLaunchKernelGGL(k_rows<256>, grid, dim3(256), lds, rs, e0_rows, e1, 0, a);
  }
  KLAUNCH();
  // (KANO_INFO_ROWS_KERNEL: 2 k_rows, 3 k_rows_prep + k_rows_w, 4 the heavy
  // rows whole with no k_rows, 5 the heavy rows then k_rows, 6 the heavy rows
  // then k_rows_w)
  ctx->rows_kernel = !rows_needed ? 4
                     : e0_rows == nullptr ? (rows_wide_used ? 6 : 5)
                                          : (rows_wide_used ? 3 : 2);
  ctx->rows_timed = true;
  ctx->rows_time_pending[set] = true;
  ctx->rows_end_ev[set] = e1;
  ctx->rows_end_rec[set] = true;
  if (!ctx->rows_overlap) KCHK(hipStreamWaitEvent(ctx->stream, e1, 0));
  return 0;
}

int ensure_built(kano_ctx* ctx) {
  if (!ctx) return -EINVAL;
  if (!ctx->built) return fail(ctx, -EINVAL, "matrix not built");
  KCHK(hipSetDevice(ctx->device));
  return settle(ctx);
}

int ensure_matrix(kano_ctx* ctx) {
  KTRY(ensure_built(ctx));
  if (ctx->lists_mode) return fail(ctx, -EINVAL, "context holds policy lists, not a matrix");
  if (ctx->vs_open)
    return fail(ctx, -EINVAL,
                "matrix read between kano_verify_shard and kano_verify_combine (the combine "
                "writes the shard's rows)");
  if (ctx->rows_deferred) {    // kano_build_classes: the matrix, now
    ctx->rows_deferred = false;
    KTRY(dalloc(ctx, ctx->M, sizeof(u64) * std::max<i64>(1, rows_local(ctx) * ctx->ldM)));
    KTRY(launch_rows(ctx));
  }
  return 0;
}

// identity "classes" over the local rows (after an edit of M): row r is its
// own class with itself as the only member
int ensure_identity(kano_ctx* ctx, const int32_t** moff, const int32_t** mem) {
  const i64 rl = rows_local(ctx);
  KTRY(dalloc(ctx, ctx->ident, sizeof(int32_t) * (3 * rl + 1)));
  std::vector<int32_t> h(3 * rl + 1);
  for (i64 r = 0; r <= rl; ++r) h[r] = (int32_t)r;
  for (i64 r = 0; r < rl; ++r) h[rl + 1 + r] = (int32_t)(ctx->r0 + r);
  for (i64 r = 0; r < rl; ++r) h[2 * rl + 1 + r] = 1;
  KCHK(hipMemcpyAsync(ctx->ident.p, h.data(), sizeof(int32_t) * (3 * rl + 1),
                      hipMemcpyHostToDevice, ctx->stream));
  KTRY(sync(ctx));
  *moff = P_<int32_t>(ctx->ident);
  *mem = *moff + rl + 1;
  return 0;
}

// column OR / NAND recomputed from M itself (after kano_set_bit / put_rows)
int recompute_cols(kano_ctx* ctx) {
  const i64 rl = rows_local(ctx), W = ctx->W, ldM = ctx->ldM;
  KCHK(hipMemsetAsync(ctx->color.p, 0, sizeof(u64) * ldM, ctx->stream));
  KCHK(hipMemsetAsync(ctx->colnand.p, 0, sizeof(u64) * ldM, ctx->stream));
  if (rl == 0 || W == 0) {
    ctx->cols_valid = true;
    return 0;
  }
  const int32_t *moff = nullptr, *mem = nullptr;
  KTRY(ensure_identity(ctx, &moff, &mem));
  const int cww = (int)std::min<i64>(ldM, MAX_CWW);
  RowsArgs a{};
  a.wioff = moff;  // one work item per row
  a.wicls = moff;  // identity
  a.U = rl;
  a.moff = moff;
  a.mem = mem;
  a.hflag = mem + rl;  // every row "prebuilt": copy + column fold, no writes
  a.M = P_<u64>(ctx->M);
  a.ldM = ldM;
  a.wW = ldM;
  a.r0 = ctx->r0;
  a.n = ctx->n;
  a.W = W;
  a.ch = 1;
  a.cww = cww;
  a.color = P_<u64>(ctx->color);
  a.colnand = P_<u64>(ctx->colnand);
  hipLaunchKernelGGL(k_rows<TPB>, dim3((unsigned)rl, (unsigned)((ldM + cww - 1) / cww)),
                     dim3(TPB), sizeof(u64) * cww, ctx->stream, a);
  KLAUNCH();
  KTRY(sync(ctx));
  ctx->cols_valid = true;
  return 0;
}

// ngroups > 0: the caller declares every gid in [0, ngroups) (no host scan;
// the kernels flag a violation in ctx->err_dev); ngroups <= 0: scanned here
// ---- user_crosscheck at class level, in stages ------------------------------
// (kano_verify interleaves the stages with policy_shadow's so that their
// fills and scans share launches)
struct CrossPlan {
  bool on = false;           // class-level pass needed (pods, rows, words present)
  const int32_t* gdev = nullptr;
  int32_t G = 0;
  bool key_lds = false;
  i64 knb = 0, kslots = 0;
};

// host checks, group upload (no fills): cp.on, cp.gdev, cp.G
int cross_setup(kano_ctx* ctx, const int32_t* gid, int32_t ngroups, CrossPlan& cp,
                hipStream_t st = nullptr) {
  const i64 n = ctx->n, W = ctx->W, ldM = ctx->ldM;
  KTRY(dalloc(ctx, ctx->gid, sizeof(int32_t) * std::max<i64>(1, n)));
  KTRY(dalloc(ctx, ctx->cross, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->sizes, sizeof(u64) * SZ_SLOTS));
  cp.on = false;
  if (n == 0 || rows_local(ctx) == 0 || W == 0) return 0;
  int32_t G = ngroups;
  cp.gdev = P_<int32_t>(ctx->gid);
  if (!gid) {   // the groups stored by kano_set_groups (already on the device)
    if (ctx->groups_n != n) return fail(ctx, -EINVAL, "crosscheck: no stored groups for these pods");
    G = ctx->groups_G;
    cp.gdev = P_<int32_t>(ctx->gids);
  } else {
    if (G <= 0) {
      G = 0;
      for (i64 i = 0; i < n; ++i) {
        if (gid[i] < 0) return fail(ctx, -EINVAL, "kano_crosscheck: negative group id");
        G = std::max(G, gid[i] + 1);
      }
    }
    KCHK(hipMemcpyAsync(ctx->gid.p, gid, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                        st ? st : ctx->stream));
  }
  cp.G = G;
  cp.on = true;
  return 0;
}

// cross_setup (unless done), allocations; fills go to fb
int cross_prepare(kano_ctx* ctx, const int32_t* gid, int32_t ngroups, CrossPlan& cp,
                  FillBatch& fb, bool setup_done = false) {
  const i64 ldM = ctx->ldM;
  if (!setup_done) KTRY(cross_setup(ctx, gid, ngroups, cp, fb.st));
  int32_t* err = reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_ERR);
  KTRY(fb.add_raw(err, sizeof(u64), 0u));
  KTRY(fb.add(ctx->cross, sizeof(u64) * ldM, 0u));
  if (!cp.on) return 0;
  const int32_t G = cp.G;
  if (ctx->rows_dirty) return 0;   // the M-based path allocates its own
  const i64 U = ctx->rc.U, ldC = ctx->ldC;
  KTRY(dalloc(ctx, ctx->gmin, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->gmax, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->R, sizeof(u64) * std::max<i64>(1, (i64)G * ldC)));
  KTRY(dalloc(ctx, ctx->ckey, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->corder, sizeof(int32_t) * std::max<i64>(1, U)));
  cp.key_lds = (i64)G + 1 <= KEY_LDS_MAX;
  cp.knb = std::max<i64>(1, nblk(U, (i64)TPB * KEY_ITEMS));
  cp.kslots = cp.key_lds ? ((i64)G + 1) * cp.knb : (i64)G + 1;
  KTRY(dalloc(ctx, ctx->kcnt, sizeof(int32_t) * 2 * ((i64)G + 1) + sizeof(int32_t) * cp.kslots));
  KTRY(dalloc(ctx, ctx->koff, sizeof(int32_t) * (cp.kslots + 1)));
  KTRY(dalloc(ctx, ctx->multi, sizeof(u64) * ldC));
  KTRY(dalloc(ctx, ctx->A1, sizeof(u64) * ldC));
  KTRY(dalloc(ctx, ctx->A2, sizeof(u64) * ldC));
  KTRY(fb.add(ctx->gmin, sizeof(int32_t) * U, 0x7fffffffu));
  KTRY(fb.add(ctx->gmax, sizeof(int32_t) * U, 0xffffffffu));
  KTRY(fb.add(ctx->R, sizeof(u64) * (i64)G * ldC, 0u));
  for (DBuf* b : {&ctx->multi, &ctx->A1, &ctx->A2}) KTRY(fb.add(*b, sizeof(u64) * ldC, 0u));
  KTRY(fb.add(ctx->kcnt, sizeof(int32_t) * 2 * ((i64)G + 1), 0u));   // counts + cursors
  return 0;
}

// group range per class, group keys and their histogram; the key scan job
// goes to sb
KeySort cross_sort(kano_ctx* ctx, const CrossPlan& cp) {
  KeySort k{};
  k.U = ctx->rc.U;
  k.nb = cp.knb;
  k.mcnt = P_<int32_t>(ctx->rc.mcnt);
  k.gmin = P_<int32_t>(ctx->gmin);
  k.gmax = P_<int32_t>(ctx->gmax);
  k.G = cp.G;
  k.ckey = P_<int32_t>(ctx->ckey);
  k.hist = P_<int32_t>(ctx->kcnt) + 2 * ((i64)cp.G + 1);
  k.hoff = P_<int32_t>(ctx->koff);
  k.order = P_<int32_t>(ctx->corder);
  return k;
}

// (st: stream2 for the build's side work, with sb a side batch; the side
// form of the LDS key sort has no scan: k_key_place_scan scans the histogram)
int cross_stage_a(kano_ctx* ctx, const CrossPlan& cp, ScanBatch& sb, hipStream_t st = nullptr) {
  if (!cp.on) return 0;
  const i64 U = ctx->rc.U, G = cp.G, rl = rows_local(ctx);
  const hipStream_t s = st ? st : ctx->stream;
  int32_t* err = reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_ERR);
  // group range of every row class along its member list
  hipLaunchKernelGGL(k_cls_group_range_m, dim3(nblk(rl)), dim3(TPB), 0, s, cp.gdev,
                     (int32_t)G, P_<int32_t>(ctx->rc.cls), P_<int32_t>(ctx->rc.mem), rl,
                     P_<int32_t>(ctx->gmin), P_<int32_t>(ctx->gmax), err);
  KLAUNCH();
  int32_t* kcnt = P_<int32_t>(ctx->kcnt);
  if (cp.key_lds) {   // classes in group order: per-block LDS histograms
    const KeySort ks = cross_sort(ctx, cp);
    hipLaunchKernelGGL(k_key_hist, dim3((unsigned)cp.knb), dim3(TPB),
                       sizeof(int32_t) * (size_t)(G + 1), s, ks);
    KLAUNCH();
    if (!st) KTRY(sb.add(ks.hist, cp.kslots, P_<int32_t>(ctx->koff)));
  } else {
    hipLaunchKernelGGL(k_cls_key, dim3(nblk(U)), dim3(TPB), 0, s, U,
                       P_<int32_t>(ctx->rc.mcnt), P_<int32_t>(ctx->gmin), P_<int32_t>(ctx->gmax),
                       (int32_t)G, P_<int32_t>(ctx->ckey), kcnt);
    KLAUNCH();
    KTRY(sb.add(kcnt, G + 1, P_<int32_t>(ctx->koff)));
  }
  return 0;
}

// classes placed in group order, one pass over Mc (R[g], MULTI, and the
// column checks when the build deferred them), group overlaps A1 / A2
int cross_stage_b1(kano_ctx* ctx, const CrossPlan& cp, hipStream_t st = nullptr) {
  if (!cp.on) return 0;
  const i64 U = ctx->rc.U, G = cp.G;
  const hipStream_t s = st ? st : ctx->stream;
  int32_t* kcnt = P_<int32_t>(ctx->kcnt);
  if (cp.key_lds && st) {
    hipLaunchKernelGGL(k_key_place_scan, dim3((unsigned)cp.knb), dim3(TPB),
                       sizeof(int32_t) * (size_t)(G + 1), s, cross_sort(ctx, cp));
  } else if (cp.key_lds) {
    hipLaunchKernelGGL(k_key_place_lds, dim3((unsigned)cp.knb), dim3(TPB),
                       sizeof(int32_t) * (size_t)(G + 1), s, cross_sort(ctx, cp));
  } else {
    hipLaunchKernelGGL(k_cls_key_place, dim3(nblk(U)), dim3(TPB), 0, s, U,
                       P_<int32_t>(ctx->ckey), P_<int32_t>(ctx->koff), kcnt + G + 1,
                       P_<int32_t>(ctx->corder));
  }
  KLAUNCH();
  return 0;
}

int cross_stage_b2(kano_ctx* ctx, const CrossPlan& cp) {
  if (!cp.on) return 0;
  const i64 U = ctx->rc.U, G = cp.G, ldC = ctx->ldC, UAW = ctx->UAW;
  const bool cols = ctx->cols_deferred;
  const int32_t* nlive = P_<int32_t>(ctx->koff) + cp.kslots;   // the key scan's total
  {
    const int32_t* ord = P_<int32_t>(ctx->corder);
    const int32_t* ck = P_<int32_t>(ctx->ckey);
    u64* co = cols ? P_<u64>(ctx->col_or_c) : nullptr;
    u64* cn = cols ? P_<u64>(ctx->col_nand_c) : nullptr;
    // 32 row classes per wave, their Mc words loaded together (measured C3:
    // 16.9 us vs 24-27 us for a serial walk of 16)
    const dim3 g(nblk(UAW, 64), nblk(U, (TPB / 64) * FOLD_PER_WAVE));
    hipLaunchKernelGGL(k_mc_fold, g, dim3(TPB), 0, ctx->stream, P_<u64>(ctx->Mc), ldC, UAW,
                       ctx->cc.U, ord, nlive, ck, (int32_t)G, P_<u64>(ctx->R),
                       P_<u64>(ctx->multi), co, cn);
  }
  KLAUNCH();
  ctx->cols_deferred = false;
  hipLaunchKernelGGL(k_cross_groups, dim3((unsigned)G, nblk(UAW)), dim3(TPB), 0, ctx->stream,
                     P_<u64>(ctx->R), ldC, UAW, P_<u64>(ctx->A1), P_<u64>(ctx->A2));
  KLAUNCH();
  ctx->cross_G = (int32_t)G;
  return 0;
}

int crosscheck_impl(kano_ctx* ctx, const int32_t* gid, int32_t ngroups = 0) {
  const i64 n = ctx->n, W = ctx->W, ldM = ctx->ldM;
  CrossPlan cp;
  {
    FillBatch fb(ctx);
    KTRY(cross_prepare(ctx, gid, ngroups, cp, fb));
    KTRY(fb.run());
  }
  if (!cp.on) return 0;
  const int32_t G = cp.G;
  const int32_t* gdev = cp.gdev;
  int32_t* err = reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_ERR);
  if (!ctx->rows_dirty) {
    // class level: rows of a row class are equal, columns of a column class
    // are equal; everything runs on Mc (U_r x U_a bits)
    ScanBatch sb(ctx);
    KTRY(cross_stage_a(ctx, cp, sb));
    KTRY(sb.run());
    KTRY(cross_stage_b1(ctx, cp));
    KTRY(cross_stage_b2(ctx, cp));
    hipLaunchKernelGGL(k_cross_pod, dim3(nblk(W * 64)), dim3(TPB), 0, ctx->stream,
                       gdev, G, P_<int32_t>(ctx->cc.cls), n, P_<u64>(ctx->R),
                       ctx->ldC, P_<u64>(ctx->multi), P_<u64>(ctx->A1), P_<u64>(ctx->A2), W,
                       P_<u64>(ctx->cross), err);
    KLAUNCH();
    return 0;
  }

  // M edited: every row is its own class, rows read from M
  KTRY(dalloc(ctx, ctx->multi, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->A1, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->A2, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->own, sizeof(u64) * ldM));
  for (DBuf* b : {&ctx->multi, &ctx->A1, &ctx->A2, &ctx->own})
    KCHK(hipMemsetAsync(b->p, 0, sizeof(u64) * ldM, ctx->stream));
  const int32_t *moff = nullptr, *mem = nullptr;
  KTRY(ensure_identity(ctx, &moff, &mem));
  const i64 nclass = rows_local(ctx);
  KTRY(dalloc(ctx, ctx->cgroup, sizeof(int32_t) * std::max<i64>(1, nclass)));
  hipLaunchKernelGGL(k_cross_classgroup, dim3(nblk(nclass)), dim3(TPB), 0, ctx->stream,
                     gdev, moff, mem, nclass, P_<int32_t>(ctx->cgroup));
  KLAUNCH();
  // groups in batches so that R fits ~2 GiB
  const i64 budget_rows = std::max<i64>(1, (2ll << 30) / (8 * ldM));
  const unsigned ycols = std::max<unsigned>(1, nblk(W, TPB * 4));
  for (int32_t g0 = 0; g0 < G; g0 += (int32_t)budget_rows) {
    const int32_t g1 = (int32_t)std::min<i64>(G, (i64)g0 + budget_rows);
    const i64 ng = g1 - g0;
    KTRY(dalloc(ctx, ctx->R, sizeof(u64) * ng * ldM));
    KCHK(hipMemsetAsync(ctx->R.p, 0, sizeof(u64) * ng * ldM, ctx->stream));
    hipLaunchKernelGGL(k_cross_accum, dim3((unsigned)nclass, ycols), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cgroup), moff, mem, P_<u64>(ctx->M), ldM, ctx->r0, W, g0,
                       g1, P_<u64>(ctx->R), P_<u64>(ctx->multi));
    KLAUNCH();
    hipLaunchKernelGGL(k_cross_groups, dim3((unsigned)ng, ycols), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->R), ldM, W, P_<u64>(ctx->A1), P_<u64>(ctx->A2));
    KLAUNCH();
    hipLaunchKernelGGL(k_cross_own, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                       gdev, n, P_<u64>(ctx->R), ldM, g0, g1, P_<u64>(ctx->own));
    KLAUNCH();
  }
  hipLaunchKernelGGL(k_cross_final, dim3(nblk(W)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->multi),
                     P_<u64>(ctx->A1), P_<u64>(ctx->A2), P_<u64>(ctx->own), W, n,
                     P_<u64>(ctx->cross));
  KLAUNCH();
  return 0;
}

}  // namespace kano_eng

using namespace kano_eng;

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int kano_create_lean(int device, kano_ctx** out) {
  g_create_lean = true;
  const int rc = kano_create(device, out);
  g_create_lean = false;
  return rc;
}

int kano_create(int device, kano_ctx** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -ENODEV;
  if (device < 0 || device >= ndev) return -EINVAL;
  // KANO_CREATE_TRACE=1: the time of each part of context creation (stderr)
  const bool trace = getenv("KANO_CREATE_TRACE") != nullptr;
  auto tc0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!trace) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "kano_create %s %.3f ms\n", what,
                 std::chrono::duration<double, std::milli>(t - tc0).count());
    tc0 = t;
  };
  if (hipSetDevice(device) != hipSuccess) return -EIO;
  mark("set_device");
  kano_ctx* ctx = new kano_ctx();
  ctx->device = device;
  (void)hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device);
  // test hooks (KANO_TUNE="key=value,..."): forms that compute the same
  // results, forced for the parity tests (see kano_ctx)
  if (const char* t = getenv("KANO_TUNE")) {
    std::string spec(t);
    size_t pos = 0;
    while (pos < spec.size()) {
      size_t end = spec.find(',', pos);
      if (end == std::string::npos) end = spec.size();
      const std::string kv = spec.substr(pos, end - pos);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos) {
        const std::string k = kv.substr(0, eq);
        const int v = atoi(kv.c_str() + eq + 1);
        if (k == "timing") ctx->stage_timing = v;
        if (k == "packed") ctx->cls_packed = v;
        if (k == "rw" && v >= 0 && v <= 2) ctx->rows_wide = v;   // 2: at every width
        if (k == "rwg" && v >= 0) ctx->rows_w_grid = v;
        if (k == "rheavy" && v >= 0 && v <= 2) ctx->rows_early_heavy = v;
        if (k == "aipt" && v >= 0 && v <= ASSIGN_IPT) ctx->assign_ipt = v;
        if (k == "sww" && v >= 1 && v <= SORT_LDS_WW) ctx->sort_ww = v;
        if (k == "cww" && v >= 16 && v <= MAX_CWW_KNOB && v % 16 == 0) ctx->rows_cww = v;
        if (k == "rch" && v >= 1 && v <= 1024) ctx->rows_ch = v;
        if (k == "async") ctx->async_rows = v;
        if (k == "shcount" && v >= 0 && v <= 2) ctx->shadow_count_mode = v;
        if (k == "pathdens" && v >= 0 && v <= 101) ctx->path_dens = v;
        if (k == "pathtm" && (v == 1 || v == 2 || v == 4)) ctx->path_tm = v;
        if (k == "pathlds") ctx->path_lds = v;
        if (k == "pathtn" && (v == 2 || v == 4)) ctx->path_tn = v;
        if (k == "shgsub") ctx->shg_sub_lds = v;
        if (k == "shr" && (v == 1 || v == 2 || v == 4 || v == 8)) ctx->shadow_r = v;
        if (k == "rcu" && v >= 0 && v <= 28 && (v < 4 || v % 4 == 0)) ctx->rows_cu_off = v;
        if (k == "rcubytes" && v >= 0) ctx->rows_cu_bytes = (i64)v << 30;
        if (k == "xcd") ctx->xcd_split = v;
        if (k == "xcdmin" && v >= 0) ctx->xcd_min_bytes = (i64)v << 10;
        if (k == "xcdw" && v >= 1 && v <= 7) ctx->xcd_write = v;
        if (k == "xcde" && v >= 0 && v <= 7) ctx->xcd_eng0 = v;
        if (k == "xcdside" && v >= -1 && v <= 1) ctx->xcd_side = v;
        if (k == "hgemm" && (v == -1 || v == 0 || v == 22 || v == 42 || v == 44))
          ctx->heavy_gemm = v;
        if (k == "hgemmmin" && v > 0) ctx->heavy_gemm_min = v;
        if (k == "hortime") ctx->time_or = v;
        if (k == "hexplds" && v >= 2 && v <= 4) ctx->heavy_expand_lds = v;
        if (k == "dx") ctx->dx_on = v;
        if (k == "aclds") ctx->ac_lds = v;
        if (k == "mlside") ctx->mlists_side_ok = v;
        if (k == "xomfma" && v > 0) ctx->xo_mfma = (double)v * 1e12;
        if (k == "xoor" && v > 0) ctx->xo_or = (double)v * 1e9;
      }
      pos = end + 1;
    }
  }
  // the engine stream and stream2 at the device's greatest priority: a
  // build's short kernels take the CUs first that the previous call's matrix
  // write (stream3, normal priority) frees
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  (void)prio_lo;

  // (round 4: the engine streams confined to the CUs the write leaves, and
  // stream2 at normal priority, measured neutral at C3 and slower where the
  // engine kernels are heavy: D1, C5 row shards)
  const int prio_main = prio_hi;
  if (hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_main) != hipSuccess) {
    delete ctx;
    return -EIO;
  }
  ctx->own_stream = true;
  mark("stream");
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  mark("stage_events");
  // the staged GEMM's LDS (128 KB at 4 x 4) is above the default dynamic cap
  {
    const int lds44 = (int)(sizeof(u64) * 2 * GK_KC * (256 + 256));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<4, 4, gemm_kc(4, 4)>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds44);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<4, 2, gemm_kc(4, 2)>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds44);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<2, 2, gemm_kc(2, 2)>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds44);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rows<1024>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(u64) * MAX_CWW_KNOB);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rows_w<1024>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(u64) * MAX_CWW_KNOB);
  }
  mark("func_attributes");
  if (hipStreamCreateWithFlags(&ctx->stream3, hipStreamNonBlocking) != hipSuccess) {
    ctx->stream3 = nullptr;
    kano_destroy(ctx);
    return -EIO;
  }
  // (the CU-masked write stream right after stream3: created later -- on the
  // first overlapped write -- it shared a hardware queue with the engine
  // stream and the pipelined step went 0.38 -> 0.68 ms; a lean context, for
  // builds the caller waits for, has none)
  if (!g_create_lean) KTRY(ensure_masked_stream(ctx));
  mark("write_streams");
  if (hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, prio_main) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_sizes, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_tail, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rin, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rin_e, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pre, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pre_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pre_ac, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_sw, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_sw2, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_pairs, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&ctx->ev_m0) != hipSuccess || hipEventCreate(&ctx->ev_m1) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rows_end[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_rows_end[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&ctx->ev_rt[0][0]) != hipSuccess || hipEventCreate(&ctx->ev_rt[0][1]) != hipSuccess ||
      hipEventCreate(&ctx->ev_rt[1][0]) != hipSuccess || hipEventCreate(&ctx->ev_rt[1][1]) != hipSuccess) {
    kano_destroy(ctx);
    return -EIO;
  }
  mark("stream2_events");
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->ghost), sizeof(u64) * SZ_SLOTS,
                    hipHostMallocDefault) != hipSuccess) {
    kano_destroy(ctx);
    return -ENOMEM;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->gmirror), sizeof(u64) * (SZ_SIGNAL + 1),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->gmirror_dev), ctx->gmirror, 0) !=
          hipSuccess) {
    kano_destroy(ctx);
    return -ENOMEM;
  }
  for (int k = 0; k <= SZ_SIGNAL; ++k) ctx->gmirror[k] = 0;
  // the pipelined prologue's bell (kano_set_pipeline): one coherent word the
  // gate kernel polls; its timeout in wall-clock ticks (200 ms)
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->bell), 64,
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->bell_dev), ctx->bell, 0) !=
          hipSuccess) {
    kano_destroy(ctx);
    return -ENOMEM;
  }
  ctx->bell[0] = 0;
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess ||
        khz <= 0)
      khz = 100000;   // (gfx950's wall clock: 100 MHz)
    ctx->gate_ticks = (u64)khz * 200;
    ctx->wall_khz = (u64)khz;
  }
  // page-locked staging for short row reads (system_isolation's row)
  if (hipHostMalloc(&ctx->row_stage, ROW_STAGE_BYTES, hipHostMallocDefault) != hipSuccess)
    ctx->row_stage = nullptr;
  if (dalloc(ctx, ctx->sig_ctr, sizeof(uint32_t) * 4) != 0 ||
      hipMemset(ctx->sig_ctr.p, 0, sizeof(uint32_t) * 4) != hipSuccess) {
    kano_destroy(ctx);
    return -ENOMEM;
  }
  mark("pinned_and_device_buffers");
  *out = ctx;
  return 0;
}

void kano_destroy(kano_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  ring_bell(ctx);   // (a primed prologue's gate opens: the syncs below finish)
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  if (ctx->stream3) (void)hipStreamSynchronize(ctx->stream3);
  if (ctx->stream3m) (void)hipStreamSynchronize(ctx->stream3m);
  for (hipStream_t t : {ctx->stream_x, ctx->stream2_x, ctx->stream3x, ctx->stream2_u})
    if (t) (void)hipStreamSynchronize(t);
  if (ctx->ghost) (void)hipHostFree(ctx->ghost);
  if (ctx->gmirror) (void)hipHostFree(ctx->gmirror);
  if (ctx->row_stage) (void)hipHostFree(ctx->row_stage);
  if (ctx->bell) (void)hipHostFree(ctx->bell);
  dfree(ctx->sizes_alt);
  dfree(ctx->gate_wait);
  for (ClassSet* cs : {&ctx->rc, &ctx->cc}) {
    DBuf* b[] = {&cs->keys_d, &cs->table, &cs->smin, &cs->slot_of, &cs->flag, &cs->cid, &cs->cls,
                 &cs->rep,    &cs->mcnt,  &cs->mcur, &cs->moff,    &cs->mem,  &cs->cval};
    for (DBuf* x : b) dfree(*x);
  }
  for (SideMatch* sx : {&ctx->sm, &ctx->am}) {
    DBuf* b[] = {&sx->toff,  &sx->tslot, &sx->tval, &sx->pmask,  &sx->moff, &sx->mslot,
                 &sx->table, &sx->pslot, &sx->gcnt, &sx->goff,   &sx->gcur, &sx->gmem,
                 &sx->pstart, &sx->plen, &sx->bits, &sx->bcnt,   &sx->boff};
    for (DBuf* x : b) dfree(*x);
  }
  DBuf* bufs[] = {&ctx->pv,     &ctx->scnt,    &ctx->cost,    &ctx->soffc,     &ctx->scur,
                  &ctx->slist,  &ctx->maxs,    &ctx->wicnt,   &ctx->wioff,     &ctx->hflag,
                  &ctx->hoff,   &ctx->hlist,   &ctx->sq,      &ctx->pfoff,     &ctx->ACT,
                  &ctx->AC,     &ctx->nca,     &ctx->acnt,    &ctx->alcoff,    &ctx->alc,
                  &ctx->aloff,  &ctx->alist,   &ctx->M,       &ctx->Mc,        &ctx->color,
                  &ctx->colnand, &ctx->col_and, &ctx->col_or_c, &ctx->col_nand_c, &ctx->scan_tmp, &ctx->scan_tmp2,
                  &ctx->shg_h,  &ctx->shg_tkey, &ctx->shg_trep, &ctx->shg_slot, &ctx->shg_isrep,
                  &ctx->shg_gidx, &ctx->shg_gid, &ctx->shg_reps, &ctx->shg_sub, &ctx->shg_err, &ctx->sig_ctr,
                  &ctx->gid,    &ctx->cgroup,  &ctx->R,       &ctx->multi,     &ctx->A1,
                  &ctx->A2,     &ctx->own,     &ctx->cross,   &ctx->gmin,      &ctx->gmax,
                  &ctx->flags,  &ctx->T,       &ctx->loff,    &ctx->L,         &ctx->tp,
                  &ctx->poff,   &ctx->out,     &ctx->scratch_words, &ctx->ident, &ctx->ecls,
                  &ctx->tcnt,   &ctx->toff,    &ctx->sizes,   &ctx->icnt,      &ctx->ioff,
                  &ctx->sysrow, &ctx->wicls,   &ctx->idxd,
                  &ctx->ckey,   &ctx->corder,  &ctx->kcnt,    &ctx->koff,
                  &ctx->gids,
                  &ctx->pT,     &ctx->pR[0],   &ctx->pR[1],   &ctx->pD[0],     &ctx->pD[1],
                  &ctx->pA,     &ctx->pB,      &ctx->pcnt,
                  &ctx->xv,     &ctx->asel,    &ctx->aalw,    &ctx->iterm,     &ctx->idead,
                  &ctx->irows,  &ctx->xw,      &ctx->xg,
                  &ctx->rw_items, &ctx->rw_segs, &ctx->rw_ticket, &ctx->slist_tmp,
                  &ctx->dx_sc, &ctx->dx_sa, &ctx->mct};
  for (DBuf* b : bufs) dfree(*b);
  RowsInputs& ra = ctx->rin_alt;
  for (DBuf* b : {&ra.wioff, &ra.wicls, &ra.soffc, &ra.slist, &ra.aloff, &ra.alist, &ra.alcoff,
                  &ra.alc, &ra.rmoff, &ra.rmem, &ra.cmoff, &ra.cmem, &ra.ccls, &ra.hflag,
                  &ra.hlist, &ra.Mc})
    dfree(*b);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->stream3) (void)hipStreamDestroy(ctx->stream3);
  if (ctx->stream3m) (void)hipStreamDestroy(ctx->stream3m);
  for (hipStream_t t : {ctx->stream_x, ctx->stream2_x, ctx->stream3x, ctx->stream2_u})
    if (t) (void)hipStreamDestroy(t);
  for (hipEvent_t e : {ctx->ev_sw, ctx->ev_sw2})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {ctx->ev_fork, ctx->ev_tail, ctx->ev_rin, ctx->ev_rin_e, ctx->ev_sizes,
                       ctx->ev_fork2, ctx->ev_join2, ctx->ev_pre, ctx->ev_pre_done, ctx->ev_pre_ac, ctx->ev_pairs, ctx->ev_m0, ctx->ev_m1, ctx->ev_rows_end[0],
                       ctx->ev_rows_end[1], ctx->ev_rt[0][0], ctx->ev_rt[0][1], ctx->ev_rt[1][0],
                       ctx->ev_rt[1][1]})
    if (e) (void)hipEventDestroy(e);
  delete ctx;
}

const char* kano_last_error(const kano_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int kano_set_stream(kano_ctx* ctx, void* s) {
  if (!ctx) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  KTRY(leave_xcd_streams(ctx));
  KCHK(hipStreamSynchronize(ctx->stream2));
  KCHK(hipStreamSynchronize(ctx->stream3));
  if (ctx->stream3m) KCHK(hipStreamSynchronize(ctx->stream3m));
  if (ctx->stream3x) KCHK(hipStreamSynchronize(ctx->stream3x));
  if (ctx->own_stream && ctx->stream) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    ctx->stream = nullptr;
    ctx->own_stream = false;
  }
  if (s) {
    ctx->stream = (hipStream_t)s;
  } else {
    KCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    ctx->own_stream = true;
  }
  return 0;
}

int kano_set_pods(kano_ctx* ctx, int64_t n, int32_t ncols, const int32_t* pod_val) {
  if (!ctx) return -EINVAL;
  if (n < 0 || ncols < 0 || n >= (int64_t)INT32_MAX / 2 || (n * ncols > 0 && !pod_val))
    return fail(ctx, -EINVAL, "kano_set_pods: bad arguments");
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  ctx->n = n;
  ctx->W = (n + 63) / 64;
  ctx->ldM = std::max<i64>(LD_ALIGN, (ctx->W + LD_ALIGN - 1) / LD_ALIGN * LD_ALIGN);
  ctx->ncols = ncols;
  // bit width of every column's (value id + 1): key tuples that fit 63 bits
  // are hashed and compared as one packed word (no gathers of pod values)
  // (pod value ids are >= -3: -1 absent, -3 never matches; packed as v + 3;
  // a column with anything lower is marked unpackable, 64 bits)
  ctx->colbits.assign(ncols, 1);
  for (int32_t c = 0; c < ncols; ++c) {
    int32_t mx = 0, mn = 0;
    const int32_t* col = pod_val + (i64)c * n;
    for (i64 i = 0; i < n; ++i) {
      mx = std::max(mx, col[i] + 3);
      mn = std::min(mn, col[i] + 3);
    }
    int b = 1;
    while (b < 31 && (1 << b) <= mx) ++b;
    ctx->colbits[c] = mn < 0 ? 64 : b;
  }
  KTRY(dalloc(ctx, ctx->pv, sizeof(int32_t) * std::max<i64>(1, n * ncols)));
  if (n * ncols > 0)
    KCHK(hipMemcpyAsync(ctx->pv.p, pod_val, sizeof(int32_t) * n * ncols, hipMemcpyHostToDevice,
                        ctx->stream));
  ctx->r0 = 0;
  ctx->r1 = n;
  ctx->have_pods = true;
  ctx->have_pols = false;
  ctx->built = false;
  return sync(ctx);
}

// One side of the policies: the columns its terms reference become the class
// keys of that side (slots); each policy's terms are sorted by slot and
// deduplicated (two different values for one slot match nothing); the
// distinct slot sets become the masks of the hash join.
int kano_set_expressions(kano_ctx* ctx, int32_t E, const int32_t* col, const int32_t* op,
                         const int64_t* off, const int32_t* vals) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods) return fail(ctx, -EINVAL, "kano_set_expressions before kano_set_pods");
  if (E < 0 || (E > 0 && (!col || !op || !off))) return fail(ctx, -EINVAL, "kano_set_expressions");
  if (E == 0) return 0;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  const i64 n = ctx->n, nc = ctx->ncols;
  for (int32_t e = 0; e < E; ++e) {
    if (col[e] >= nc || op[e] < 0 || op[e] > 3 || off[e + 1] < off[e])
      return fail(ctx, -EINVAL, "kano_set_expressions: bad requirement");
    for (i64 k = off[e] + 1; k < off[e + 1]; ++k)
      if (vals[k - 1] >= vals[k]) return fail(ctx, -EINVAL, "kano_set_expressions: unsorted set");
  }
  // the pod table grows by E columns, computed on the device
  DBuf grown;
  KTRY(dalloc(ctx, grown, sizeof(int32_t) * std::max<i64>(1, n * (nc + E))));
  if (n * nc > 0)
    KCHK(hipMemcpyAsync(grown.p, ctx->pv.p, sizeof(int32_t) * n * nc, hipMemcpyDeviceToDevice,
                        ctx->stream));
  const i64 nv = off[E];
  std::vector<uint8_t> h(sizeof(int32_t) * 2 * E + sizeof(i64) * (E + 1) +
                         sizeof(int32_t) * std::max<i64>(1, nv) + 16);
  std::memcpy(h.data(), off, sizeof(i64) * (E + 1));
  int32_t* hb = reinterpret_cast<int32_t*>(h.data() + sizeof(i64) * (E + 1));
  std::memcpy(hb, col, sizeof(int32_t) * E);
  std::memcpy(hb + E, op, sizeof(int32_t) * E);
  if (nv) std::memcpy(hb + 2 * E, vals, sizeof(int32_t) * nv);
  DBuf args;
  KTRY(dalloc(ctx, args, h.size()));
  KCHK(hipMemcpyAsync(args.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream));
  if (n > 0) {
    const i64* d_off = P_<i64>(args);
    const int32_t* d_b = reinterpret_cast<const int32_t*>(d_off + E + 1);
    hipLaunchKernelGGL(k_expr_cols, dim3(nblk(n), (unsigned)E), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(grown), n, d_b, d_b + E, d_off, d_b + 2 * E,
                       P_<int32_t>(grown) + n * nc);
    KLAUNCH();
  }
  KTRY(sync(ctx));
  dfree(args);
  dfree(ctx->pv);
  ctx->pv = grown;
  ctx->ncols = (int32_t)(nc + E);
  ctx->colbits.resize((size_t)ctx->ncols, 3);   // values 0 / 1 pack as 3 / 4
  ctx->have_pols = false;
  ctx->built = false;
  return 0;
}

static constexpr int MAX_MASKS = 64;

static int prepare_side(kano_ctx* ctx, i64 P, const int64_t* off, const int32_t* col,
                        const int32_t* val, ClassSet& cs, SideMatch& sx) {
  const i64 nt = off[P];
  std::vector<int32_t> slot(ctx->ncols, -1);
  for (i64 t = 0; t < nt; ++t) {
    if (col[t] < 0 || col[t] >= ctx->ncols) return fail(ctx, -EINVAL, "term column out of range");
    slot[col[t]] = 0;
  }
  cs.keys.clear();
  for (int32_t c = 0; c < ctx->ncols; ++c)
    if (slot[c] == 0) {
      slot[c] = (int32_t)cs.keys.size();
      cs.keys.push_back(c);
    }
  cs.KS = (int)cs.keys.size();
  // keys_d = [columns | bits]; packed when the bits sum to at most 63
  std::vector<int32_t> kd(cs.keys);
  int tb = 0;
  for (int32_t c : cs.keys) {
    kd.push_back(ctx->colbits[c]);
    tb += ctx->colbits[c];
  }
  // (KS = 0 -- no policy, or only empty selectors -- is one class: packed
  // too, so its pods meet in LDS instead of CAS-ing one global slot)
  cs.packed = (tb <= 63 && ctx->cls_packed) ? 1 : 0;
  cs.tbits = tb;
  KTRY(dalloc(ctx, cs.keys_d, sizeof(int32_t) * std::max<size_t>(1, kd.size())));
  if (cs.KS > 0)   // uploaded once per policy set, not per build
    KCHK(hipMemcpy(cs.keys_d.p, kd.data(), sizeof(int32_t) * kd.size(), hipMemcpyHostToDevice));
  std::vector<i64> toff(P + 1, 0);
  std::vector<int32_t> tslot, tval, pmask(std::max<i64>(1, P), -1), moff(1, 0), mslot;
  std::vector<std::vector<int32_t>> masks;
  std::vector<std::pair<int32_t, int32_t>> terms;
  tslot.reserve(nt);
  tval.reserve(nt);
  for (i64 p = 0; p < P; ++p) {
    terms.clear();
    for (i64 t = off[p]; t < off[p + 1]; ++t) terms.emplace_back(slot[col[t]], val[t]);
    std::sort(terms.begin(), terms.end());
    bool contradict = false;
    std::vector<int32_t> sl;
    for (size_t k = 0; k < terms.size(); ++k) {
      if (k > 0 && terms[k].first == terms[k - 1].first) {
        if (terms[k].second != terms[k - 1].second) contradict = true;
        continue;
      }
      sl.push_back(terms[k].first);
      tslot.push_back(terms[k].first);
      tval.push_back(terms[k].second);
    }
    toff[p + 1] = (i64)tslot.size();
    if (contradict) {
      pmask[p] = -1;
    } else if (sl.empty()) {
      pmask[p] = -2;
    } else {
      int id = -1;
      for (size_t m = 0; m < masks.size(); ++m)
        if (masks[m] == sl) { id = (int)m; break; }
      if (id < 0) {
        id = (int)masks.size();
        masks.push_back(sl);
      }
      pmask[p] = id;
    }
  }
  sx.nterms = (i64)tslot.size();
  sx.dense = masks.size() > (size_t)MAX_MASKS;
  sx.NM = sx.dense ? 0 : (int)masks.size();
  if (sx.dense) {
    // dense evaluation ignores masks; contradictory policies keep both terms
    // and fail the predicate naturally
    for (i64 p = 0; p < P; ++p)
      if (pmask[p] == -1) {
        tslot.push_back(0);
        tval.push_back(-4);  // never equals a value id
      }
    // rebuild offsets with the sentinel term appended per contradictory policy
    std::vector<i64> o2(P + 1, 0);
    std::vector<int32_t> s2, v2;
    i64 extra = (i64)toff[P];
    for (i64 p = 0; p < P; ++p) {
      for (i64 t = toff[p]; t < toff[p + 1]; ++t) {
        s2.push_back(tslot[t]);
        v2.push_back(tval[t]);
      }
      if (pmask[p] == -1) {
        s2.push_back(tslot[extra]);
        v2.push_back(tval[extra]);
        ++extra;
      }
      o2[p + 1] = (i64)s2.size();
    }
    toff.swap(o2);
    tslot.swap(s2);
    tval.swap(v2);
    sx.nterms = (i64)tslot.size();
  } else {
    // A policy naming every class key of a packed side selects at most one
    // class, found in the classification's own table (pmask -3): its mask
    // needs no join table (C3: a quarter of the policies on each side)
    if (cs.packed && cs.KS > 0) {
      int f = -1;
      for (size_t m = 0; m < masks.size(); ++m)
        if ((int)masks[m].size() == cs.KS) f = (int)m;
      if (f >= 0) {
        for (i64 p = 0; p < P; ++p) {
          if (pmask[p] == f) pmask[p] = -3;
          else if (pmask[p] > f) --pmask[p];
        }
        masks.erase(masks.begin() + f);
        sx.NM = (int)masks.size();
      }
    }
    for (auto& m : masks) {
      mslot.insert(mslot.end(), m.begin(), m.end());
      moff.push_back((int32_t)mslot.size());
    }
  }
  KTRY(dalloc(ctx, sx.toff, sizeof(i64) * (P + 1)));
  KTRY(dalloc(ctx, sx.tslot, sizeof(int32_t) * std::max<size_t>(1, tslot.size())));
  KTRY(dalloc(ctx, sx.tval, sizeof(int32_t) * std::max<size_t>(1, tval.size())));
  KTRY(dalloc(ctx, sx.pmask, sizeof(int32_t) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, sx.moff, sizeof(int32_t) * moff.size()));
  KTRY(dalloc(ctx, sx.mslot, sizeof(int32_t) * std::max<size_t>(1, mslot.size())));
  KCHK(hipMemcpyAsync(sx.toff.p, toff.data(), sizeof(i64) * (P + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  if (!tslot.empty()) {
    KCHK(hipMemcpyAsync(sx.tslot.p, tslot.data(), sizeof(int32_t) * tslot.size(),
                        hipMemcpyHostToDevice, ctx->stream));
    KCHK(hipMemcpyAsync(sx.tval.p, tval.data(), sizeof(int32_t) * tval.size(),
                        hipMemcpyHostToDevice, ctx->stream));
  }
  if (P > 0)
    KCHK(hipMemcpyAsync(sx.pmask.p, pmask.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice,
                        ctx->stream));
  KCHK(hipMemcpyAsync(sx.moff.p, moff.data(), sizeof(int32_t) * moff.size(), hipMemcpyHostToDevice,
                      ctx->stream));
  if (!mslot.empty())
    KCHK(hipMemcpyAsync(sx.mslot.p, mslot.data(), sizeof(int32_t) * mslot.size(),
                        hipMemcpyHostToDevice, ctx->stream));
  return sync(ctx);  // host vectors are temporaries
}

int kano_set_policies(kano_ctx* ctx, int64_t P, const int64_t* sel_off, const int32_t* sel_col,
                      const int32_t* sel_val, const int64_t* alw_off, const int32_t* alw_col,
                      const int32_t* alw_val) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods) return fail(ctx, -EINVAL, "kano_set_policies before kano_set_pods");
  if (P < 0 || !sel_off || !alw_off) return fail(ctx, -EINVAL, "kano_set_policies: bad arguments");
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  ctx->P = P;
  ctx->PB = (P + 63) / 64;
  KTRY(prepare_side(ctx, P, sel_off, sel_col, sel_val, ctx->rc, ctx->sm));
  KTRY(prepare_side(ctx, P, alw_off, alw_col, alw_val, ctx->cc, ctx->am));
  ctx->have_pols = true;
  ctx->built = false;
  return 0;
}

int kano_set_shard(kano_ctx* ctx, int64_t row_begin, int64_t row_end) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods || row_begin < 0 || row_end < row_begin || row_end > ctx->n)
    return fail(ctx, -EINVAL, "kano_set_shard: bad row range");
  KTRY(settle(ctx));
  ctx->r0 = row_begin;
  ctx->r1 = row_end;
  ctx->built = false;
  return 0;
}

}  // extern "C"

namespace {
// rows_now: launch the matrix write here; defer_cols: leave the column
// checks to the crosscheck pass over Mc (kano_verify), finish_cols() after
using ExtraFills = std::function<int(FillBatch&)>;
// k_sel_place before the host has the list sizes (build sync 2): into the
// lists as the previous build left them, whose capacity bounds the writes;
// do_back keeps it when the total fitted.  The placement then runs in the
// sync's round trip instead of after it (C3: ~13 us of the step)
int sel_place_early(kano_ctx* ctx) {
  ctx->sel_early_cap = -1;
  const i64 U = ctx->rc.U, P = ctx->P;
  if (U == 0 || P == 0 || !ctx->slist.p || !ctx->ecls.p) return 0;
  const i64 cap = (i64)(std::min(ctx->slist.bytes, ctx->ecls.bytes) / sizeof(int32_t));
  if (ctx->dense_sel) {
    KTRY(sel_place_dx(ctx, cap));
    ctx->sel_early_cap = cap;
    return 0;
  }
  hipLaunchKernelGGL(k_sel_place, dim3(nblk(P, sel_spb(ctx))), dim3(TPB), 0, ctx->stream, P,
                     P_<i64>(ctx->sm.pstart), P_<int32_t>(ctx->sm.plen), P_<int32_t>(ctx->sm.gmem),
                     P_<i64>(ctx->soffc), P_<int32_t>(ctx->scur), P_<int32_t>(ctx->slist),
                     P_<int32_t>(ctx->ecls), sel_spb(ctx), FillJobs{}, nblk(P, sel_spb(ctx)), cap);
  KLAUNCH();
  ctx->sel_early_cap = cap;
  return 0;
}

int build_impl(kano_ctx* ctx, int path, bool rows_now, bool defer_cols = false,
               const ExtraFills& extra = ExtraFills(), const ExtraFills& pre_fill = ExtraFills(),
               const PreRun& pre_run = PreRun()) {
  if (!ctx) return -EINVAL;
  // (a primed prologue is this build's only when kano_verify's front asked)
  const bool consume = ctx->primed && ctx->consume_prime;
  ctx->consume_prime = false;
  if (!consume) KTRY(unprime(ctx));
  if (!ctx->have_pods || !ctx->have_pols) return fail(ctx, -EINVAL, "kano_build: inputs not set");
  if (path < 0 || path > 2) return fail(ctx, -EINVAL, "kano_build: unknown path");
  KCHK(hipSetDevice(ctx->device));
  ctx->built = false;
  ctx->rows_deferred = false;
  ctx->lists_mode = false;
  ctx->rows_timed = false;
  ctx->rows_dirty = false;
  ctx->cols_valid = false;
  ctx->shadow_total = -1;
  ctx->sig_armed = 0;   // the syncs below wait on this build's scans only
  ctx->sel_early_cap = -1;
  ctx->shg_prefilled = false;   // (set by this build's shadow_prepare only)
  const i64 rl = rows_local(ctx);
  if (!ctx->defer_alloc)   // kano_build_classes: M is allocated on first use
    KTRY(dalloc(ctx, ctx->M, sizeof(u64) * std::max<i64>(1, rl * ctx->ldM)));
  KTRY(dalloc(ctx, ctx->color, sizeof(u64) * ctx->ldM));
  KTRY(dalloc(ctx, ctx->colnand, sizeof(u64) * ctx->ldM));
  KTRY(stage_mark(ctx, 0, ctx->stream));
  KTRY(do_front(ctx, path, consume));
  // host sync 2 (the list sizes), overlapped with the size-independent part
  // of the back end (zeroed AC / Mc, the crosscheck's group-key sort)
  KTRY(mirror_begin(ctx));
  KTRY(do_back_pre(ctx, pre_fill, pre_run));
  KTRY(sel_place_early(ctx));
  KTRY(read_sizes(ctx));
  KTRY(stage_mark(ctx, 3, ctx->stream));
  ctx->cols_deferred = defer_cols;
  KTRY(do_back(ctx, path, extra));
  if (!defer_cols) KTRY(do_rows(ctx));
  if (rows_now) KTRY(launch_rows(ctx));
  KTRY(stage_mark(ctx, 4, ctx->stream));
  ctx->cols_valid = true;
  ctx->built = true;
  // a build discards earlier incremental updates and edits
  ctx->inc_A = 0;
  ctx->inc_xcols = 0;
  ctx->dead.assign((size_t)ctx->P, 0);
  ctx->user_edited = false;
  return 0;
}

}  // namespace

extern "C" {

int kano_build(kano_ctx* ctx, int path) { return build_impl(ctx, path, true); }

int kano_build_classes(kano_ctx* ctx, int path) {
  if (!ctx) return -EINVAL;
  ctx->defer_alloc = true;
  const int rc = build_impl(ctx, path, false);
  ctx->defer_alloc = false;
  if (rc == 0) ctx->rows_deferred = true;
  return rc;
}

int kano_info(kano_ctx* ctx, int64_t* out) {
  if (!ctx || !out) return -EINVAL;
  for (int k = 0; k < KANO_INFO_NSLOTS; ++k) out[k] = 0;
  out[KANO_INFO_N] = ctx->n;
  out[KANO_INFO_W] = ctx->W;
  out[KANO_INFO_P] = ctx->P;
  out[KANO_INFO_U] = ctx->rc.U;
  out[KANO_INFO_NNZ_SEL] = ctx->nnz_sel;
  out[KANO_INFO_NNZ_ALW] = ctx->nnz_alw;
  out[KANO_INFO_HEAVY] = ctx->heavy_count;
  out[KANO_INFO_ROW0] = ctx->r0;
  out[KANO_INFO_ROW1] = ctx->r1;
  out[KANO_INFO_MAXSEL] = ctx->max_sel;
  out[KANO_INFO_UA] = ctx->cc.U;
  out[KANO_INFO_HEAVY_PATH] = ctx->heavy_path;
  out[KANO_INFO_ROWS_CUS] = ctx->rows_cus;
  out[KANO_INFO_HEAVY_SEL] = ctx->heavy_sel;
  out[KANO_INFO_HEAVY_KERNEL] = ctx->heavy_kernel;
  out[KANO_INFO_WORK_ITEMS] = ctx->wi_total;
  out[KANO_INFO_ROWS_KERNEL] = ctx->rows_kernel;
  return 0;
}

int kano_col_checks(kano_ctx* ctx, uint64_t* col_and, uint64_t* col_or) {
  KTRY(ensure_matrix(ctx));
  if (!ctx->cols_valid) KTRY(recompute_cols(ctx));
  const i64 W = ctx->W;
  if (W == 0) return sync(ctx);
  KTRY(dalloc(ctx, ctx->col_and, sizeof(u64) * W));
  hipLaunchKernelGGL(k_col_final, dim3(nblk(W)), dim3(TPB), 0, ctx->stream,
                     P_<u64>(ctx->colnand), W, ctx->n, P_<u64>(ctx->col_and));
  KLAUNCH();
  if (col_and)
    KCHK(hipMemcpyAsync(col_and, ctx->col_and.p, sizeof(u64) * W, hipMemcpyDeviceToHost,
                        ctx->stream));
  if (col_or)
    KCHK(hipMemcpyAsync(col_or, ctx->color.p, sizeof(u64) * W, hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

int kano_col_flags_dev(kano_ctx* ctx, uint8_t* flags_dev) {
  KTRY(ensure_matrix(ctx));
  if (!ctx->cols_valid) KTRY(recompute_cols(ctx));
  const i64 n = ctx->n;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_unpack_flags, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<u64>(ctx->color), n, flags_dev);
  KLAUNCH();
  hipLaunchKernelGGL(k_unpack_flags, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<u64>(ctx->colnand), n, flags_dev + 2 * n);
  KLAUNCH();
  return 0;
}

int kano_crosscheck(kano_ctx* ctx, const int32_t* gid, uint64_t* cross) {
  KTRY(ensure_matrix(ctx));
  if (!gid && ctx->n > 0) return fail(ctx, -EINVAL, "kano_crosscheck: gid is NULL");
  KTRY(crosscheck_impl(ctx, gid));
  if (cross && ctx->W > 0)
    KCHK(hipMemcpyAsync(cross, ctx->cross.p, sizeof(u64) * ctx->W, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

int kano_crosscheck_dev(kano_ctx* ctx, const int32_t* gid, uint8_t* flags_dev) {
  KTRY(ensure_matrix(ctx));
  if (!gid && ctx->n > 0) return fail(ctx, -EINVAL, "kano_crosscheck_dev: gid is NULL");
  KTRY(crosscheck_impl(ctx, gid));
  if (ctx->n > 0) {
    hipLaunchKernelGGL(k_unpack_flags, dim3(nblk(ctx->n)), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->cross), ctx->n, flags_dev + ctx->n);
    KLAUNCH();
  }
  return sync(ctx);  // gid is caller memory read by an async copy
}

int kano_get_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, uint64_t* dst) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!dst && nrows > 0))
    return fail(ctx, -EINVAL, "kano_get_rows: rows outside this shard");
  if (nrows == 0 || ctx->W == 0) return 0;
  const size_t bytes = sizeof(u64) * (size_t)ctx->W * (size_t)nrows;
  const bool staged = ctx->row_stage && bytes <= ROW_STAGE_BYTES;
  const u64* src = P_<u64>(ctx->M) + (r0 - ctx->r0) * ctx->ldM;
  void* to = staged ? ctx->row_stage : dst;
  // (contiguous rows: a linear copy -- the first strided copy of a process
  // set up its blit kernel, ~8 ms on the first system_isolation call)
  if (nrows == 1 || ctx->ldM == ctx->W)
    KCHK(hipMemcpyAsync(to, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  else
    KCHK(hipMemcpy2DAsync(to, sizeof(u64) * ctx->W, src, sizeof(u64) * ctx->ldM,
                          sizeof(u64) * ctx->W, (size_t)nrows, hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  if (staged) std::memcpy(dst, ctx->row_stage, bytes);
  return 0;
}

int kano_rows_digest(kano_ctx* ctx, int64_t r0, int64_t nrows, uint64_t* out) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!out && nrows > 0))
    return fail(ctx, -EINVAL, "kano_rows_digest: rows outside this shard");
  if (nrows == 0) return 0;
  DBuf d;
  KTRY(dalloc(ctx, d, sizeof(u64) * (size_t)nrows));
  int rc = 0;
  for (i64 q = 0; q < nrows && rc == 0; q += 1 << 30) {   // grid.x limit
    const i64 cnt = std::min<i64>(nrows - q, 1 << 30);
    hipLaunchKernelGGL(k_row_digest, dim3((unsigned)cnt), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->M) + (r0 - ctx->r0 + q) * ctx->ldM, ctx->ldM, ctx->W,
                       P_<u64>(d) + q);
    if (hipGetLastError() != hipSuccess) rc = fail(ctx, -EIO, "kano_rows_digest: launch");
  }
  if (rc == 0 &&
      hipMemcpyAsync(out, d.p, sizeof(u64) * nrows, hipMemcpyDeviceToHost, ctx->stream) !=
          hipSuccess)
    rc = fail(ctx, -EIO, "kano_rows_digest: copy");
  if (rc == 0) rc = sync(ctx);
  else (void)sync(ctx);
  dfree(d);
  return rc;
}

int kano_put_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, const uint64_t* src) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!src && nrows > 0))
    return fail(ctx, -EINVAL, "kano_put_rows: rows outside this shard");
  if (nrows == 0 || ctx->W == 0) return 0;
  KCHK(hipMemcpy2DAsync(P_<u64>(ctx->M) + (r0 - ctx->r0) * ctx->ldM, sizeof(u64) * ctx->ldM, src,
                        sizeof(u64) * ctx->W, sizeof(u64) * ctx->W, (size_t)nrows,
                        hipMemcpyHostToDevice, ctx->stream));
  KTRY(sync(ctx));
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  ctx->user_edited = true;
  return 0;
}

int kano_get_col(kano_ctx* ctx, int64_t j, uint64_t* dst) {
  KTRY(ensure_matrix(ctx));
  if (j < 0 || j >= ctx->n || !dst) return fail(ctx, -EINVAL, "kano_get_col: bad column");
  const i64 rl = rows_local(ctx);
  if (rl == 0) return 0;
  const i64 nw = (rl + 63) / 64;
  KTRY(dalloc(ctx, ctx->scratch_words, sizeof(u64) * nw));
  hipLaunchKernelGGL(k_get_col, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->M),
                     ctx->ldM, rl, (i64)j, P_<u64>(ctx->scratch_words));
  KLAUNCH();
  KCHK(hipMemcpyAsync(dst, ctx->scratch_words.p, sizeof(u64) * nw, hipMemcpyDeviceToHost,
                      ctx->stream));
  return sync(ctx);
}

int kano_get_bit(kano_ctx* ctx, int64_t i, int64_t j, int* value) {
  KTRY(ensure_matrix(ctx));
  if (i < ctx->r0 || i >= ctx->r1 || j < 0 || j >= ctx->n || !value)
    return fail(ctx, -EINVAL, "kano_get_bit: index out of range");
  u64 w = 0;
  KCHK(hipMemcpyAsync(&w, P_<u64>(ctx->M) + (i - ctx->r0) * ctx->ldM + (j >> 6), sizeof(u64),
                      hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  *value = (int)((w >> (j & 63)) & 1ull);
  return 0;
}

int kano_set_bit(kano_ctx* ctx, int64_t i, int64_t j, int value) {
  KTRY(ensure_matrix(ctx));
  if (i < ctx->r0 || i >= ctx->r1 || j < 0 || j >= ctx->n)
    return fail(ctx, -EINVAL, "kano_set_bit: index out of range");
  u64* addr = P_<u64>(ctx->M) + (i - ctx->r0) * ctx->ldM + (j >> 6);
  u64 w = 0;
  KCHK(hipMemcpyAsync(&w, addr, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  const u64 bit = 1ull << (j & 63);
  w = value ? (w | bit) : (w & ~bit);
  KCHK(hipMemcpyAsync(addr, &w, sizeof(u64), hipMemcpyHostToDevice, ctx->stream));
  KTRY(sync(ctx));
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  ctx->user_edited = true;
  return 0;
}

int kano_get_policy_sets(kano_ctx* ctx, int64_t p, uint64_t* sel, uint64_t* allow) {
  KTRY(ensure_matrix(ctx));
  if (p < 0 || p >= ctx->P) return fail(ctx, -EINVAL, "kano_get_policy_sets: bad policy");
  const i64 W = ctx->W, n = ctx->n;
  if (W == 0) return 0;
  KTRY(dalloc(ctx, ctx->scratch_words, sizeof(u64) * 2 * W));
  u64* s = P_<u64>(ctx->scratch_words);
  if (sel) {
    hipLaunchKernelGGL(k_sel_row, dim3(nblk(n)), dim3(TPB), 0, ctx->stream, P_<i64>(ctx->soffc),
                       P_<int32_t>(ctx->slist), P_<int32_t>(ctx->rc.cls), n, ctx->r0, ctx->r1,
                       (i64)p, s);
    KLAUNCH();
    KCHK(hipMemcpyAsync(sel, s, sizeof(u64) * W, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (allow) {
    hipLaunchKernelGGL(k_allow_row, dim3(nblk(n)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->AC),
                       ctx->ldC, (i64)p, P_<int32_t>(ctx->cc.cls), n, s + W);
    KLAUNCH();
    KCHK(hipMemcpyAsync(allow, s + W, sizeof(u64) * W, hipMemcpyDeviceToHost, ctx->stream));
  }
  return sync(ctx);
}

int kano_get_classes(kano_ctx* ctx, int32_t* cls) {
  KTRY(ensure_matrix(ctx));
  if (cls && ctx->n > 0) {   // row classes exist for this shard's pods only: -1 elsewhere
    for (i64 i = 0; i < ctx->n; ++i)
      if (i < ctx->r0 || i >= ctx->r1) cls[i] = -1;
    if (rows_local(ctx) > 0)
      KCHK(hipMemcpyAsync(cls + ctx->r0, P_<int32_t>(ctx->rc.cls) + ctx->r0,
                          sizeof(int32_t) * rows_local(ctx), hipMemcpyDeviceToHost, ctx->stream));
  }
  return sync(ctx);
}

int kano_get_select_csr(kano_ctx* ctx, int64_t* off, int32_t* pol) {
  KTRY(ensure_matrix(ctx));
  if (off)
    KCHK(hipMemcpyAsync(off, ctx->soffc.p, sizeof(i64) * (ctx->rc.U + 1), hipMemcpyDeviceToHost,
                        ctx->stream));
  if (pol && ctx->nnz_sel > 0)
    KCHK(hipMemcpyAsync(pol, ctx->slist.p, sizeof(int32_t) * ctx->nnz_sel, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

int kano_get_allow_csr(kano_ctx* ctx, int64_t* off, int32_t* pods) {
  KTRY(ensure_matrix(ctx));
  if (!ctx->alist_valid) KTRY(build_alist(ctx));
  if (off)
    KCHK(hipMemcpyAsync(off, ctx->aloff.p, sizeof(i64) * (ctx->P + 1), hipMemcpyDeviceToHost,
                        ctx->stream));
  if (pods && ctx->nnz_alw > 0)
    KCHK(hipMemcpyAsync(pods, ctx->alist.p, sizeof(int32_t) * ctx->nnz_alw, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

}  // extern "C"

namespace {
// policy_shadow up to its one sync: flags, per-class counts, per-pod offsets;
// the caller gathers toff[nt] (list length) and poff[rl] (pairs) with its own
// scalars
struct ShadowPlan {
  i64 U = 0, rl = 0, nf = 0, nt = 0;
};

i64 shg_table_size(i64 P) {
  i64 Th = 64;
  while (Th < 2 * P) Th <<= 1;
  return Th;
}

int shadow_prepare(kano_ctx* ctx, ShadowPlan& sp, FillBatch& fb) {
  sp.U = ctx->rc.U;
  sp.rl = rows_local(ctx);
  sp.nf = ctx->nflags;
  sp.nt = (sp.nf + SH_TILE - 1) / SH_TILE;
  KTRY(dalloc(ctx, ctx->sizes, sizeof(u64) * SZ_SLOTS));
  // (the candidate pairs' flags as bits, one 64-bit word per 64 pairs)
  KTRY(dalloc(ctx, ctx->flags, ctx->vs_count_only ? 16 : 8 * ((sp.nf + 63) / 64) + 16));
  KTRY(dalloc(ctx, ctx->T, sizeof(i64) * std::max<i64>(1, sp.U)));
  KTRY(dalloc(ctx, ctx->loff, sizeof(i64) * (sp.U + 1)));
  KTRY(dalloc(ctx, ctx->tp, sizeof(i64) * std::max<i64>(1, sp.rl)));
  KTRY(dalloc(ctx, ctx->poff, sizeof(i64) * (sp.rl + 1)));
  // (the tiles' pair counts and their offsets feed only the compaction: the
  // count-only form has none -- at D1, 2e7 tiles, a 160 MB fill and a
  // 0.3 ms scan)
  if (!ctx->vs_count_only) {
    KTRY(dalloc(ctx, ctx->tcnt, sizeof(i64) * std::max<i64>(1, sp.nt)));
    KTRY(dalloc(ctx, ctx->toff, sizeof(i64) * (sp.nt + 1)));
    KTRY(fb.add(ctx->tcnt, sizeof(i64) * sp.nt, 0u));   // accumulated
  }
  if (ctx->vs_count_only && ctx->P > 0 && sp.U > 0) {
    // the grouped count's hash table and error word, cleared with the build's
    // fills (three runtime fills on the side stream cost it ~30 us at C4)
    const i64 Th = shg_table_size(ctx->P);
    KTRY(dalloc(ctx, ctx->shg_tkey, sizeof(u64) * Th));
    KTRY(dalloc(ctx, ctx->shg_trep, sizeof(int32_t) * Th));
    KTRY(dalloc(ctx, ctx->shg_err, sizeof(int32_t) * 4));
    KTRY(fb.add(ctx->shg_tkey, sizeof(u64) * Th, 0xffffffffu));
    KTRY(fb.add(ctx->shg_trep, sizeof(int32_t) * Th, 0x7f7f7f7fu));
    KTRY(fb.add(ctx->shg_err, sizeof(int32_t) * 4, 0u));
    ctx->shg_prefilled = true;
  }
  return fb.add(ctx->T, sizeof(i64) * sp.U, 0u);
}

// the grouped count (count-only policy_shadow): T[c] per row class
int shadow_group_launch(kano_ctx* ctx, const ShadowPlan& sp, hipStream_t st) {
  const i64 P = ctx->P, U = sp.U;
  ctx->shg_ran = false;
  if (P == 0 || U == 0) return 0;
  const i64 Th = shg_table_size(P);
  const i64 GW = (SHG_MAX + 63) / 64;
  KTRY(dalloc(ctx, ctx->shg_h, sizeof(u64) * P));
  KTRY(dalloc(ctx, ctx->shg_tkey, sizeof(u64) * Th));
  KTRY(dalloc(ctx, ctx->shg_trep, sizeof(int32_t) * Th));
  KTRY(dalloc(ctx, ctx->shg_slot, sizeof(int32_t) * P));
  KTRY(dalloc(ctx, ctx->shg_isrep, sizeof(int32_t) * P));
  KTRY(dalloc(ctx, ctx->shg_gidx, sizeof(int32_t) * (P + 1)));
  KTRY(dalloc(ctx, ctx->shg_gid, sizeof(int32_t) * P));
  KTRY(dalloc(ctx, ctx->shg_reps, sizeof(int32_t) * SHG_MAX));
  KTRY(dalloc(ctx, ctx->shg_sub, sizeof(u64) * SHG_MAX * GW));
  KTRY(dalloc(ctx, ctx->shg_err, sizeof(int32_t) * 4));
  if (!ctx->shg_prefilled) {
    KCHK(hipMemsetAsync(ctx->shg_tkey.p, 0xff, sizeof(u64) * Th, st));
    KCHK(hipMemsetAsync(ctx->shg_trep.p, 0x7f, sizeof(int32_t) * Th, st));
    KCHK(hipMemsetAsync(ctx->shg_err.p, 0, sizeof(int32_t) * 4, st));
  }
  ctx->shg_prefilled = false;
  const u64* AC = P_<u64>(ctx->AC);
  hipLaunchKernelGGL(k_shg_hash, dim3(nblk(P, WPB)), dim3(TPB), 0, st, P, AC, ctx->ldC, ctx->UAW,
                     P_<u64>(ctx->shg_h));
  KLAUNCH();
  hipLaunchKernelGGL(k_shg_insert, dim3(nblk(P)), dim3(TPB), 0, st, P, P_<u64>(ctx->shg_h),
                     P_<unsigned long long>(ctx->shg_tkey), P_<int32_t>(ctx->shg_trep),
                     P_<int32_t>(ctx->shg_slot), (uint32_t)(Th - 1));
  KLAUNCH();
  hipLaunchKernelGGL(k_shg_verify, dim3(nblk(P, WPB)), dim3(TPB), 0, st, P,
                     P_<int32_t>(ctx->shg_slot), P_<int32_t>(ctx->shg_trep), AC, ctx->ldC,
                     ctx->UAW, P_<int32_t>(ctx->shg_isrep), P_<int32_t>(ctx->shg_err));
  KLAUNCH();
  hipLaunchKernelGGL(k_shg_scan, dim3(1), dim3(1024), 0, st, P, P_<int32_t>(ctx->shg_isrep),
                     P_<int32_t>(ctx->shg_gidx));
  KLAUNCH();
  hipLaunchKernelGGL(k_shg_assign, dim3(nblk(P)), dim3(TPB), 0, st, P, P_<int32_t>(ctx->shg_slot),
                     P_<int32_t>(ctx->shg_trep), P_<int32_t>(ctx->shg_isrep),
                     P_<int32_t>(ctx->shg_gidx), P_<int32_t>(ctx->shg_gid),
                     P_<int32_t>(ctx->shg_reps));
  KLAUNCH();
  const int32_t* Gp = P_<int32_t>(ctx->shg_gidx) + P;
  const u64* nfp = P_<u64>(ctx->sizes) + SZ_NFLAGS;
  const int force = ctx->shadow_count_mode == 2 ? 2 : 0;
  // (a's allowed classes in LDS, b's through its class list: shgsub=0 the
  // word-by-word form)
  const size_t shg_lds = sizeof(u64) * (size_t)WPB * (size_t)ctx->UAW;
  const int shg_lds_row = ctx->shg_sub_lds && shg_lds <= 64 * 1024 ? 1 : 0;
  hipLaunchKernelGGL(k_shg_sub, dim3(nblk(std::min<i64>(P, SHG_MAX), WPB)), dim3(TPB),
                     shg_lds_row ? shg_lds : 0, st, Gp, P_<int32_t>(ctx->shg_reps), AC, ctx->ldC,
                     ctx->UAW, P_<u64>(ctx->shg_sub), GW, P_<int32_t>(ctx->shg_err), nfp, force,
                     P_<int32_t>(ctx->nca), P_<i64>(ctx->alcoff), P_<int32_t>(ctx->alc),
                     shg_lds_row);
  KLAUNCH();
  ShadowArgs a{};
  a.U = U;
  a.soffc = P_<i64>(ctx->soffc);
  a.slist = P_<int32_t>(ctx->slist);
  a.mcnt = P_<int32_t>(ctx->rc.mcnt);
  a.pfoff = P_<i64>(ctx->pfoff);
  a.nca = P_<int32_t>(ctx->nca);
  a.alcoff = P_<i64>(ctx->alcoff);
  a.alc = P_<int32_t>(ctx->alc);
  a.AC = AC;
  a.ldC = ctx->ldC;
  a.flags = nullptr;
  a.T = P_<i64>(ctx->T);
  a.shg_nf = nfp;
  a.shg_force = force;
  hipLaunchKernelGGL(k_shg_count, dim3((unsigned)U), dim3(TPB), 0, st, a,
                     P_<int32_t>(ctx->shg_gid), Gp, P_<u64>(ctx->shg_sub), GW,
                     P_<int32_t>(ctx->shg_err));
  KLAUNCH();
  ctx->shg_ran = true;
  return 0;
}

constexpr i64 SH_YIELD_GRID = 8192;   // 32 blocks per CU

// subset tests; the list-offset scans go to sb.  Count only: the grouped
// count and the flag-free pairwise test are both queued, the device picks
// one (shg_grouped) once the allow-set groups are known; knob shcount 1 / 2
// forces the pairwise / grouped form.
int shadow_test_launch(kano_ctx* ctx, const ShadowPlan& sp, hipStream_t st) {
  KTRY(stage_mark(ctx, 5, st));
  const int mode = ctx->vs_count_only ? ctx->shadow_count_mode : -1;
  ctx->shg_ran = false;
  if (mode == 0 || mode == 2) KTRY(shadow_group_launch(ctx, sp, st));
  if (mode == 2) return 0;
  if (sp.nt > 0) {
    ShadowArgs a{};
    if (mode == 0 && ctx->shg_ran) {   // the pairwise test yields to the grouped count
      a.shg_G = P_<int32_t>(ctx->shg_gidx) + ctx->P;
      a.shg_err = P_<int32_t>(ctx->shg_err);
      a.shg_nf = P_<u64>(ctx->sizes) + SZ_NFLAGS;
    }
    a.U = sp.U;
    a.soffc = P_<i64>(ctx->soffc);
    a.slist = P_<int32_t>(ctx->slist);
    a.mcnt = P_<int32_t>(ctx->rc.mcnt);
    a.pfoff = P_<i64>(ctx->pfoff);
    a.nca = P_<int32_t>(ctx->nca);
    a.alcoff = P_<i64>(ctx->alcoff);
    a.alc = P_<int32_t>(ctx->alc);
    a.AC = P_<u64>(ctx->AC);
    a.ldC = ctx->ldC;
    a.flags = ctx->vs_count_only ? nullptr : P_<uint8_t>(ctx->flags);   // count only: T[c]
    a.T = P_<i64>(ctx->T);
    // (one block per virtual block of R x 256 pairs, or a capped striding
    // grid when the test may yield to the grouped count); R = 8 once the
    // candidate pairs run to ~10^7 (C5 row shards: 7e7 pairs, the test 2.39
    // -> 1.65 ms at R = 4, the step 7.76 -> 6.91 ms; R = 8 6.77), 1 below
    // (C3: ~10^6, on the side stream)
    const int R = ctx->shadow_r > 0 ? ctx->shadow_r : (sp.nf >= (i64)1 << 24 ? 8 : 1);
    const i64 nvb = (sp.nf + (i64)TPB * R - 1) / ((i64)TPB * R);
    i64 grid = a.shg_G ? std::min<i64>(nvb, SH_YIELD_GRID) : nvb;
    i64* tc = ctx->vs_count_only ? (i64*)nullptr : P_<i64>(ctx->tcnt);
    // (direct launches, no kernel-pointer variable: tests/test_launch_ir.py)
#define KANO_SHT(RR)                                                                        \
  hipLaunchKernelGGL((k_shadow_test1s<1024, RR>), dim3((unsigned)grid), dim3(TPB), 0, st, a, \
                     sp.nf, tc)
    if (R == 8) KANO_SHT(8);
    else if (R == 4) KANO_SHT(4);
    else if (R == 2) KANO_SHT(2);
    else KANO_SHT(1);
#undef KANO_SHT
    KLAUNCH();
  }
  return 0;
}

int shadow_stage_a_scans(kano_ctx* ctx, const ShadowPlan& sp, ScanBatch& sb) {
  if (!ctx->vs_count_only) KTRY(sb.add(P_<i64>(ctx->tcnt), sp.nt, P_<i64>(ctx->toff), SZ_NL));
  KTRY(sb.add(P_<i64>(ctx->T), sp.U, P_<i64>(ctx->loff)));
  return 0;
}

int shadow_stage_a(kano_ctx* ctx, const ShadowPlan& sp, ScanBatch& sb) {
  KTRY(shadow_test_launch(ctx, sp, ctx->stream));
  return shadow_stage_a_scans(ctx, sp, sb);
}

// pairs per pod; the per-pod offset scan goes to sb
int shadow_stage_b(kano_ctx* ctx, const ShadowPlan& sp, ScanBatch& sb) {
  if (sp.rl > 0) {
    hipLaunchKernelGGL(k_shadow_podcount, dim3(nblk(sp.rl)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->rc.cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                       P_<i64>(ctx->tp));
    KLAUNCH();
  }
  return sb.add(P_<i64>(ctx->tp), sp.rl, P_<i64>(ctx->poff), SZ_PAIRS);
}

// policy_shadow up to its one sync (the caller reads SZ_NL, SZ_PAIRS)
int shadow_front(kano_ctx* ctx) {
  ShadowPlan sp;
  {
    FillBatch fb(ctx);
    KTRY(shadow_prepare(ctx, sp, fb));
    KTRY(fb.run());
  }
  {
    ScanBatch sb(ctx);
    KTRY(shadow_stage_a(ctx, sp, sb));
    KTRY(sb.run());
  }
  ScanBatch sb(ctx);
  KTRY(shadow_stage_b(ctx, sp, sb));
  return sb.run();
}

int shadow_back(kano_ctx* ctx, i64 nl, i64 total, hipStream_t st = nullptr) {
  if (!st) st = ctx->stream;
  const i64 U = ctx->rc.U, rl = rows_local(ctx), nf = ctx->nflags;
  const i64 nt = (nf + SH_TILE - 1) / SH_TILE;
  KTRY(dalloc(ctx, ctx->L, sizeof(int2) * std::max<i64>(1, nl)));
  KTRY(dalloc(ctx, ctx->out, sizeof(int2) * std::max<i64>(1, total)));
  if (nt > 0 && nl > 0) {
    hipLaunchKernelGGL(k_shadow_compact, dim3((unsigned)nt), dim3(TPB), 0, st,
                       P_<i64>(ctx->soffc), U, P_<int32_t>(ctx->slist), P_<i64>(ctx->pfoff),
                       P_<uint8_t>(ctx->flags), nf, P_<i64>(ctx->toff), P_<int2>(ctx->L), nl);
    KLAUNCH();
  }
  if (rl > 0 && total > 0) {
    hipLaunchKernelGGL(k_shadow_emit, dim3(nblk(rl)), dim3(TPB), 0, st,
                       P_<int32_t>(ctx->rc.cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                       P_<int2>(ctx->L), P_<i64>(ctx->poff), P_<int2>(ctx->out), total,
                       (const i64*)nullptr, nl);
    KLAUNCH();
  }
  KTRY(stage_mark(ctx, 6, st));
  ctx->shadow_total = total;
  return 0;
}

}  // namespace

extern "C" {

int kano_shadow(kano_ctx* ctx, int64_t* count) {
  KTRY(ensure_built(ctx));
  ctx->vs_count_only = false;   // (the pairs: a count-only kano_verify may have run last)
  KTRY(shadow_front(ctx));
  i64 tot[2] = {0, 0};
  KTRY(read_slots(ctx, SZ_NL, 2, tot));
  KTRY(shadow_back(ctx, tot[0], tot[1]));
  if (count) *count = tot[1];
  return 0;
}

int kano_shadow_fetch(kano_ctx* ctx, int32_t* pairs) {
  KTRY(ensure_built(ctx));
  if (ctx->shadow_total < 0) return fail(ctx, -EINVAL, "kano_shadow_fetch before kano_shadow");
  if (ctx->shadow_total > 0) {
    if (!pairs) return fail(ctx, -EINVAL, "kano_shadow_fetch: NULL buffer");
    KCHK(hipMemcpyAsync(pairs, ctx->out.p, sizeof(int2) * ctx->shadow_total,
                        hipMemcpyDeviceToHost, ctx->stream));
  }
  return sync(ctx);
}

int kano_shadow_lists(kano_ctx* ctx, int64_t n_lists, int64_t nbits, int64_t P,
                      const int64_t* soff, const int32_t* slist, const uint64_t* allow_rows,
                      int64_t* count) {
  if (!ctx) return -EINVAL;
  if (n_lists < 0 || nbits < 0 || P < 0 || !soff || n_lists >= (int64_t)INT32_MAX / 2)
    return fail(ctx, -EINVAL, "kano_shadow_lists: bad arguments");
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  const i64 nnz = soff[n_lists];
  for (i64 e = 0; e < nnz; ++e)
    if (slist[e] < 0 || slist[e] >= P)
      return fail(ctx, -ERANGE, "kano_shadow_lists: policy index out of range");
  // every list is its own row class; every pod its own column class
  ctx->built = false;
  ctx->lists_mode = true;
  ctx->n = nbits;
  ctx->W = (nbits + 63) / 64;
  ctx->ldM = std::max<i64>(2, (ctx->W + 1) & ~(i64)1);
  ctx->P = P;
  ctx->PB = (P + 63) / 64;
  ctx->r0 = 0;
  ctx->r1 = n_lists;
  ctx->nnz_sel = nnz;
  ctx->rc.U = n_lists;
  ctx->cc.U = nbits;
  ctx->UAW = ctx->W;
  ctx->ldC = ctx->ldM;
  const i64 U = n_lists;
  KTRY(dalloc(ctx, ctx->soffc, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->slist, sizeof(int32_t) * std::max<i64>(1, nnz)));
  KTRY(dalloc(ctx, ctx->rc.cls, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->rc.mcnt, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->sq, sizeof(i64) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->pfoff, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->AC, sizeof(u64) * std::max<i64>(1, P * ctx->ldC)));
  KTRY(dalloc(ctx, ctx->nca, sizeof(int32_t) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, ctx->acnt, sizeof(int32_t) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, ctx->alcoff, sizeof(i64) * (P + 1)));
  std::vector<int32_t> iota(std::max<i64>(1, U)), ones(std::max<i64>(1, U), 1);
  for (i64 c = 0; c < U; ++c) iota[c] = (int32_t)c;
  KCHK(hipMemcpyAsync(ctx->soffc.p, soff, sizeof(i64) * (U + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  if (nnz > 0)
    KCHK(hipMemcpyAsync(ctx->slist.p, slist, sizeof(int32_t) * nnz, hipMemcpyHostToDevice,
                        ctx->stream));
  if (U > 0) {
    KCHK(hipMemcpyAsync(ctx->rc.cls.p, iota.data(), sizeof(int32_t) * U, hipMemcpyHostToDevice,
                        ctx->stream));
    KCHK(hipMemcpyAsync(ctx->rc.mcnt.p, ones.data(), sizeof(int32_t) * U, hipMemcpyHostToDevice,
                        ctx->stream));
    hipLaunchKernelGGL(k_sq_from_off, dim3(nblk(U)), dim3(TPB), 0, ctx->stream,
                       P_<i64>(ctx->soffc), U, P_<i64>(ctx->sq));
    KLAUNCH();
  }
  KTRY((scan_excl<i64, i64>(ctx, P_<i64>(ctx->sq), U, P_<i64>(ctx->pfoff))));
  if (P > 0 && ctx->W > 0) {
    KCHK(hipMemcpy2DAsync(ctx->AC.p, sizeof(u64) * ctx->ldC, allow_rows, sizeof(u64) * ctx->W,
                          sizeof(u64) * ctx->W, (size_t)P, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_pol_count, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->AC), ctx->ldC, ctx->UAW, (const int32_t*)nullptr,
                       P_<int32_t>(ctx->nca), P_<int32_t>(ctx->acnt));
    KLAUNCH();
  } else if (P > 0) {
    KCHK(hipMemsetAsync(ctx->nca.p, 0, sizeof(int32_t) * P, ctx->stream));
  }
  KTRY((scan_excl<int32_t, i64>(ctx, P_<int32_t>(ctx->nca), P, P_<i64>(ctx->alcoff))));
  i64 hv[2] = {0, 0};
  KCHK(hipMemcpyAsync(&hv[0], P_<i64>(ctx->alcoff) + P, 8, hipMemcpyDeviceToHost, ctx->stream));
  KCHK(hipMemcpyAsync(&hv[1], P_<i64>(ctx->pfoff) + U, 8, hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));  // also retires the host vectors above
  ctx->nnz_alc = hv[0];
  ctx->nflags = hv[1];
  KTRY(dalloc(ctx, ctx->alc, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_alc)));
  if (P > 0 && ctx->W > 0) {
    hipLaunchKernelGGL(k_pol_classes, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->AC), ctx->ldC, ctx->UAW, P_<i64>(ctx->alcoff),
                       P_<int32_t>(ctx->alc));
    KLAUNCH();
  }
  ctx->built = true;
  return kano_shadow(ctx, count);
}

int kano_conflict(kano_ctx* ctx, int* raises) {
  KTRY(ensure_built(ctx));
  if (!raises) return fail(ctx, -EINVAL, "kano_conflict: NULL");
  *raises = ctx->max_sel >= 2 ? 1 : 0;
  return 0;
}

}  // extern "C"

namespace {
// kano_verify in two halves.  verify_front: the build and every check up to
// the column words (k_verify_cols; with words_dev also this shard's
// [OR | cross | NAND] words for the ranks' gather).  verify_back: (combine
// the gathered words of all shards,) list the results, the matrix write,
// policy_shadow's pairs, the copies to the host.
// ncclAllGather, resolved once: from the process first (the library that
// created the caller's communicator -- torch ships its own librccl), else
// librccl.so.  The engine does not link RCCL: without it only
// kano_verify_gather is unavailable.
typedef int (*RcclAllGather)(const void*, void*, size_t, int, void*, hipStream_t);
constexpr int RCCL_UINT64 = 5;   // ncclUint64 (rccl.h)
int rccl_find_loaded(struct dl_phdr_info* info, size_t, void* out) {
  const char* name = info->dlpi_name;
  if (name && std::strstr(name, "librccl")) {
    *static_cast<std::string*>(out) = name;
    return 1;
  }
  return 0;
}
RcclAllGather rccl_all_gather() {
  static RcclAllGather fn = [] {
    // a librccl already mapped into the process (torch's, loaded RTLD_LOCAL
    // as a dependency: not visible to RTLD_DEFAULT)
    std::string path;
    dl_iterate_phdr(rccl_find_loaded, &path);
    void* f = nullptr;
    if (!path.empty()) {
      if (void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD)) f = dlsym(h, "ncclAllGather");
    }
    if (!f) f = dlsym(RTLD_DEFAULT, "ncclAllGather");
    if (!f) {
      void* h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (h) f = dlsym(h, "ncclAllGather");
    }
    return reinterpret_cast<RcclAllGather>(f);
  }();
  return fn;
}

int verify_front(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                 bool want_shadow, u64* words_dev, bool count_only = false) {
  ctx->vs_count_only = want_shadow && count_only;
  // the previous call's matrix write may still run: build into the other
  // input set instead of waiting for it (a primed prologue already writes it)
  ctx->consume_prime = ctx->primed;
  if (ctx->async_pending && !ctx->primed) KTRY(swap_rows_inputs(ctx));
  const bool stored = !gid && ngroups == KANO_STORED_GROUPS;
  const bool want_cross = gid || stored;
  // the crosscheck and policy_shadow buffers are filled in the build's last
  // fill launch
  CrossPlan cp;
  ShadowPlan sp;
  // the crosscheck's fills and group-key sort need only the class counts:
  // they run while the list sizes travel (build sync 2)
  auto pre_fill = [&](FillBatch& fb) -> int {
    return want_cross ? cross_prepare(ctx, gid, ngroups, cp, fb) : 0;
  };
  auto pre_run = [&](hipStream_t st) -> int {
    if (!want_cross || !cp.on) return 0;
    ScanBatch sb(ctx, st != nullptr);
    KTRY(cross_stage_a(ctx, cp, sb, st));
    KTRY(sb.run());
    return cross_stage_b1(ctx, cp, st);
  };
  auto extra = [&](FillBatch& fb) -> int {
    return want_shadow ? shadow_prepare(ctx, sp, fb) : 0;
  };
  ctx->vs_open = false;
  // policy_shadow's subset tests need only the lists and AC: they run on
  // stream2 beside the Mc chain (scatter, fold), forked (ev_fork2) and issued
  // where the lists and AC are complete.  In pairs mode (side_tail) the rest
  // of policy_shadow up to its emission follows them there -- the offset
  // scans, the compaction, the per-pod pair counts and their scan -- and the
  // engine stream joins it (ev_pairs) only before the emission.
  ctx->fork_pending = false;
  ctx->tail_compacted = false;
  bool fork_marked = false;
  const bool side_sh = want_shadow && !count_only;
  if (want_shadow) {
    ctx->fork_hook = [&](bool marked) -> int {
      if (!marked) KCHK(hipEventRecord(ctx->ev_fork2, ctx->stream));
      KCHK(hipStreamWaitEvent(ctx->stream2, ctx->ev_fork2, 0));
      KTRY(shadow_test_launch(ctx, sp, ctx->stream2));
      fork_marked = true;
      return 0;
    };
  }
  const int brc = build_impl(ctx, path, false, want_cross, extra, pre_fill, pre_run);
  ctx->fork_hook = nullptr;
  KTRY(brc);
  const i64 n = ctx->n, W = ctx->W;
  const bool have_sys = sys_row >= ctx->r0 && sys_row < ctx->r1;
  const bool cross_on = want_cross && cp.on;
  // the crosscheck's pass over Mc first (the engine stream's next work: its
  // launches go out before the side stream's), then policy_shadow's tests on
  // stream2 and their scans (or here)
  if (cross_on) KTRY(cross_stage_b2(ctx, cp));
  const bool side_run = fork_marked && side_sh;
  if (!side_run && fork_marked) {
    KCHK(hipEventRecord(ctx->ev_join2, ctx->stream2));
    ctx->fork_pending = true;
  }
  if (want_shadow && !side_run) {
    ScanBatch sb(ctx);
    if (ctx->fork_pending) {
      KCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_join2, 0));
      ctx->fork_pending = false;
      KTRY(shadow_stage_a_scans(ctx, sp, sb));
    } else {
      KTRY(shadow_stage_a(ctx, sp, sb));
    }
    KTRY(sb.run());
  }
  if (ctx->cols_deferred) {   // no crosscheck pass ran (empty shard / matrix)
    ctx->cols_deferred = false;
    KTRY(mc_cols(ctx));
  }
  // (policy_shadow's per-pod pair counts come out of k_verify_cols below;
  // their scan joins verify_back's batch)
  // the column tail in one pass (k_verify_cols)
  const i64 nb = std::max<i64>(1, nblk(W * 64));
  KTRY(dalloc(ctx, ctx->col_and, sizeof(u64) * std::max<i64>(1, W)));
  KTRY(dalloc(ctx, ctx->sysrow, sizeof(u64) * std::max<i64>(1, W)));
  KTRY(dalloc(ctx, ctx->icnt, sizeof(i64) * 4 * nb));
  KTRY(dalloc(ctx, ctx->ioff, sizeof(i64) * 4 * (nb + 1)));
  KTRY(dalloc(ctx, ctx->idxd, sizeof(int32_t) * std::max<i64>(1, 4 * n) + 16));
  const bool sys_on = have_sys && W > 0;
  if (n > 0 && W > 0) {
    FinishArgs fa{};
    fa.cla = P_<int32_t>(ctx->cc.cls);
    fa.n = n;
    fa.W = W;
    fa.nb = nb;
    fa.col_or_c = P_<u64>(ctx->col_or_c);
    fa.col_nand_c = P_<u64>(ctx->col_nand_c);
    fa.color = P_<u64>(ctx->color);
    fa.colnand = P_<u64>(ctx->colnand);
    fa.col_and = P_<u64>(ctx->col_and);
    fa.ldC = ctx->ldC;
    if (cross_on) {
      fa.gid = cp.gdev;
      fa.G = cp.G;
      fa.R = P_<u64>(ctx->R);
      fa.multi = P_<u64>(ctx->multi);
      fa.A1 = P_<u64>(ctx->A1);
      fa.A2 = P_<u64>(ctx->A2);
      fa.cross = P_<u64>(ctx->cross);
      fa.err = reinterpret_cast<int32_t*>(P_<u64>(ctx->sizes) + SZ_ERR);
    }
    if (sys_on) {
      fa.Mc = P_<u64>(ctx->Mc);
      fa.clr = P_<int32_t>(ctx->rc.cls);
      fa.sys_row = sys_row;
      fa.sysrow = P_<u64>(ctx->sysrow);
    }
    fa.icnt = P_<i64>(ctx->icnt);
    fa.words = words_dev;
    if (want_shadow && sp.rl > 0 && !side_run) {
      fa.rcls = P_<int32_t>(ctx->rc.cls);
      fa.loff = P_<i64>(ctx->loff);
      fa.tp = P_<i64>(ctx->tp);
      fa.r0 = ctx->r0;
      fa.r1 = ctx->r1;
    }
    // (round 6: the four lists written by the column pass itself, with a
    // decoupled look-back over the tiles -- k_verify_cols_f -- measured slower
    // than this pass plus the count scan and k_idx_write at every config: C3
    // 0.355 -> 0.348 ms, C4 0.396 -> 0.391, D1 0.887 -> 0.879,
    // profiles/r06_c3_vfused_ab.jsonl, r06_c4_vfused_ab.jsonl)
    hipLaunchKernelGGL(k_verify_cols, dim3((unsigned)nb), dim3(TPB), 0, ctx->stream, fa);
    KLAUNCH();
  } else {
    KCHK(hipMemsetAsync(ctx->icnt.p, 0, sizeof(i64) * 4 * nb, ctx->stream));
  }
  // (issued after the column checks: the engine stream does not wait for it)
  if (side_run) {
    // the offset scans (toff: SZ_NL; loff), the compaction and the per-pod
    // pair counts, then their offsets (poff: SZ_PAIRS), all behind the tests
    hipStream_t s2 = ctx->stream2;
    {   // with them, the per-pod pair offsets from the class counts T (poff:
        // SZ_PAIRS); the compaction follows, its dispatch marks ev_pairs
      ScanBatch sbs(ctx, true);
      KTRY(shadow_stage_a_scans(ctx, sp, sbs));
      KTRY(sbs.add_class_counts(P_<int32_t>(ctx->rc.cls), P_<i64>(ctx->T), ctx->r0, sp.rl,
                                P_<i64>(ctx->poff), SZ_PAIRS));
      KTRY(sbs.run(sp.nt > 0 ? nullptr : ctx->ev_pairs));
    }
    KTRY(dalloc(ctx, ctx->L, sizeof(int2) * std::max<i64>(1, sp.nf)));
    if (sp.nt > 0) {
      launch_marked(k_shadow_compact, dim3((unsigned)sp.nt), dim3(TPB), 0, s2, ctx->ev_pairs,
                    P_<i64>(ctx->soffc), ctx->rc.U, P_<int32_t>(ctx->slist),
                    P_<i64>(ctx->pfoff), P_<uint8_t>(ctx->flags), sp.nf, P_<i64>(ctx->toff),
                    P_<int2>(ctx->L), sp.nf);
      KLAUNCH();
    }
    ctx->tail_compacted = true;
  }
  ctx->vs_open = true;
  ctx->vs_shadow = want_shadow;
  ctx->vs_cross_want = want_cross;
  ctx->vs_cross_on = cross_on;
  ctx->vs_have_sys = have_sys;
  ctx->vs_sys_on = sys_on;
  ctx->vs_rows = true;
  ctx->vs_nb = nb;
  ctx->vs_rl = sp.rl;
  return 0;
}

// spin on an event (the syncs' waits are tens of microseconds: no sleep)
int spin_event(kano_ctx* ctx, hipEvent_t e) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint32_t spin = 1;; ++spin) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) KCHK(q);
    __builtin_ia32_pause();
    if ((spin & 0xff) == 0 && clk::now() - t0 > std::chrono::seconds(1)) {
      KCHK(hipEventSynchronize(e));
      return 0;
    }
  }
}

// The next kano_verify's prologue (front_a) behind a gate on the engine
// stream: into the next input set (the write just launched reads this one)
// and the private size slots; the next call rings the bell, anything else
// unprimes.  Nothing of it runs before the next call asks (or the gate's
// 200 ms timeout: then it has run on the same resident inputs).
int prime_next(kano_ctx* ctx) {
  if (ctx->primed || !ctx->bell || ctx->stage_timing) return 0;
  KTRY(dalloc(ctx, ctx->sizes_alt, sizeof(u64) * SZ_SLOTS));
  ctx->prime_alist_valid = ctx->alist_valid;
  KTRY(swap_rows_inputs(ctx));
  std::swap(ctx->sizes, ctx->sizes_alt);
  ctx->primed = true;
  ctx->priming = true;
  const u64 armed = ctx->sig_armed, waiting = ctx->sig_wait;
  if (!ctx->gate_wait.p) {
    KTRY(dalloc(ctx, ctx->gate_wait, sizeof(u64) * GATE_RING));
    KCHK(hipMemsetAsync(ctx->gate_wait.p, 0, sizeof(u64) * GATE_RING, ctx->stream));
  }
  hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, ctx->stream, (const u64*)ctx->bell_dev,
                     ++ctx->bell_seq, ctx->gate_ticks, P_<u64>(ctx->gate_wait));
  int rc = hipGetLastError() == hipSuccess ? 0 : fail(ctx, -EIO, "k_gate launch failed");
  if (!rc) {
    ctx->sig_armed = 0;
    rc = front_a(ctx);
  }
  ctx->priming = false;
  if (rc) {
    (void)unprime(ctx);
    return rc;
  }
  ctx->prime_sig = ctx->sig_wait;
  ctx->sig_armed = armed;
  ctx->sig_wait = waiting;
  return 0;
}

// compacted: policy_shadow's compaction ran on stream2 (verify_front; its
// end is ev_pairs)
int verify_back_direct(kano_ctx* ctx, int32_t* idx, void* idx_h, int64_t* counts,
                       int32_t* shadow_pairs, void* pairs_h, int64_t shadow_cap,
                       int64_t* shadow_count, bool async, bool compacted = false) {
  using clk = std::chrono::steady_clock;
  auto tmark = clk::now();
  auto part = [&](int k) {
    const auto t = clk::now();
    ctx->ht[k] = std::max(ctx->ht[k], std::chrono::duration<double, std::micro>(t - tmark).count());
    tmark = t;
  };
  const i64 n = ctx->n, rl = ctx->vs_rl;
  const bool want_shadow = ctx->vs_shadow;
  const bool pairs_mode = want_shadow && shadow_cap >= 0;
  hipStream_t st = ctx->stream;
  const i64 nf = ctx->nflags, nt = (nf + SH_TILE - 1) / SH_TILE;
  i64 out_cap = 0;
  const bool pairs_job = pairs_mode && pairs_h && rl > 0;
  const u64* tots = P_<u64>(ctx->sizes) + SZ_IDX0;
  if (pairs_mode) {
    // L never exceeds the candidate pairs; out keeps the largest total seen
    KTRY(dalloc(ctx, ctx->L, sizeof(int2) * std::max<i64>(1, nf)));
    KTRY(dalloc(ctx, ctx->out, sizeof(int2) * 1024));
    out_cap = (i64)(ctx->out.bytes / sizeof(int2));
    if (compacted) KCHK(hipStreamWaitEvent(st, ctx->ev_pairs, 0));
    if (nt > 0 && !compacted) {
      hipLaunchKernelGGL(k_shadow_compact, dim3((unsigned)nt), dim3(TPB), 0, st,
                         P_<i64>(ctx->soffc), ctx->rc.U, P_<int32_t>(ctx->slist),
                         P_<i64>(ctx->pfoff), P_<uint8_t>(ctx->flags), nf, P_<i64>(ctx->toff),
                         P_<int2>(ctx->L), nf);
      KLAUNCH();
    }
    if (rl > 0) {
      hipLaunchKernelGGL(k_shadow_emit, dim3(nblk(rl)), dim3(TPB), 0, st,
                         P_<int32_t>(ctx->rc.cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                         P_<int2>(ctx->L), P_<i64>(ctx->poff), P_<int2>(ctx->out), out_cap,
                         nt > 0 ? P_<i64>(ctx->toff) + nt : (const i64*)nullptr, nf);
      KLAUNCH();
    }
  }
  // the lists (one job, or one per row when the column pass wrote row r at
  // idxd[r * n]) and the pairs; the copy's own dispatch marks ev_tail (no
  // separate record: ~3 us less on the engine stream), which also starts the
  // matrix write
  CopySegs cj{};
  int njobs = 0;
  cj.j[njobs++] = CopySeg{static_cast<const char*>(ctx->idxd.p), static_cast<char*>(idx_h),
                          tots, 4, nullptr, 0, 4, 4 * n};
  if (pairs_job) {
    cj.j[njobs++] = CopySeg{static_cast<const char*>(ctx->out.p), static_cast<char*>(pairs_h),
                            reinterpret_cast<const u64*>(P_<i64>(ctx->poff) + rl), 1, nullptr, 0,
                            8, std::min<i64>(shadow_cap, out_cap)};
  }
  if (njobs > 0) {
    hipExtLaunchKernelGGL(k_copy_segs, dim3(256, njobs), dim3(TPB), 0, st, nullptr, ctx->ev_tail,
                          0, cj);
    KLAUNCH();
  }
  if (ctx->vs_rows) {
    ctx->rows_overlap = async;
    // (the build's last Mc launch, when it marked one: the write need not
    // wait for the checks, the pairs and the copies)
    ctx->rows_in = ctx->rin_marked ? ctx->ev_rin_e : ctx->ev_tail;
    ctx->rin_marked = false;
    const int rc = launch_rows(ctx);
    ctx->rows_overlap = false;
    ctx->rows_in = nullptr;
    KTRY(rc);
  }
  // the next call's prologue, queued behind its gate while this call's tail
  // still runs (kano_set_pipeline)
  if (async && ctx->pipeline) KTRY(prime_next(ctx));
  part(12);
  const auto tw0 = clk::now();
  KTRY(spin_event(ctx, ctx->ev_tail));
  ctx->ht[18] += std::chrono::duration<double, std::micro>(clk::now() - tw0).count();
  part(14);
  ctx->sig_wait = 0;
  constexpr int NS = SZ_ERR - SZ_NL + 1;
  i64 v[NS];
  for (int q = 0; q < NS; ++q) v[q] = (i64)((volatile u64*)ctx->gmirror)[SZ_NL + q];
  if (ctx->vs_cross_on && (v[SZ_ERR - SZ_NL] & 0xffffffff)) {
    (void)settle(ctx);
    (void)sync(ctx);
    return fail(ctx, -EINVAL, "kano_verify: a group id lies outside [0, ngroups)");
  }
  for (int r = 0; r < 4; ++r) counts[r] = v[SZ_IDX0 - SZ_NL + r];
  if (!ctx->vs_have_sys) counts[3] = -1;
  if (want_shadow) {
    const i64 total = v[SZ_PAIRS - SZ_NL];
    *shadow_count = total;
    ctx->shadow_total = pairs_mode ? total : -1;
    if (pairs_mode && total > out_cap) {
      // past the emission buffer: the sized emission, then the copy (on a
      // stream without the gate: the next call builds unprimed)
      KTRY(unprime(ctx));
      KTRY(dalloc(ctx, ctx->out, sizeof(int2) * (total + total / 4)));
      if (rl > 0) {
        hipLaunchKernelGGL(k_shadow_emit, dim3(nblk(rl)), dim3(TPB), 0, st,
                           P_<int32_t>(ctx->rc.cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                           P_<int2>(ctx->L), P_<i64>(ctx->poff), P_<int2>(ctx->out), total,
                           (const i64*)nullptr, nf);
        KLAUNCH();
      }
      if (shadow_pairs && total <= shadow_cap)
        KTRY(copy_out(ctx, shadow_pairs, ctx->out.p, sizeof(int2) * total, st));
      KCHK(hipEventRecord(ctx->ev_tail, st));
      KCHK(hipEventSynchronize(ctx->ev_tail));
    }
  }
  part(15);
  if (async) {
    ctx->async_pending = true;
    return 0;
  }
  KTRY(sync(ctx));
  return 0;
}

int verify_back(kano_ctx* ctx, const u64* gathered, int32_t nranks, int32_t* idx, int64_t* counts,
                int32_t* shadow_pairs, int64_t shadow_cap, int64_t* shadow_count,
                bool may_async = false) {
  if (!ctx->vs_open) return fail(ctx, -EINVAL, "kano_verify_combine without kano_verify_shard");
  ctx->vs_open = false;
  const i64 n = ctx->n, W = ctx->W, nb = ctx->vs_nb;
  const bool want_shadow = ctx->vs_shadow;
  // a gathered combine lists the crosscheck whenever it was asked for (other
  // shards may hold its rows)
  const bool cross_row = gathered ? ctx->vs_cross_want : ctx->vs_cross_on;
  const bool pairs_mode = want_shadow && shadow_cap >= 0;
  if (want_shadow && ctx->vs_count_only && shadow_cap >= 0) {
    (void)sync(ctx);
    return fail(ctx, -EINVAL, "kano_verify_combine: the shard ran policy_shadow count-only "
                              "(with_shadow = 2); pass shadow_cap < 0");
  }
  void* idx_h = n > 0 ? pinned_dev(idx) : nullptr;
  void* pairs_h = pairs_mode && shadow_pairs ? pinned_dev(shadow_pairs) : nullptr;
  const bool direct = n > 0 && W > 0 && idx_h && (!pairs_mode || !shadow_pairs || pairs_h);
  // policy_shadow's scans, per-pod counts and compaction ran on stream2
  // (verify_front): the direct tail joins it before the emission; the host's
  // sync below needs its sizes, so that path joins it here
  const bool side_sh = want_shadow && ctx->tail_compacted;
  const bool compacted = side_sh && direct && pairs_mode;
  if (side_sh && !compacted) KCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_pairs, 0));
  ctx->tail_compacted = false;
  ScanBatch sb(ctx);
  if (want_shadow && !side_sh)
    KTRY(sb.add(P_<i64>(ctx->tp), ctx->vs_rl, P_<i64>(ctx->poff), SZ_PAIRS));
  if (gathered && n > 0 && W > 0) {
    if (cross_row) KTRY(dalloc(ctx, ctx->cross, sizeof(u64) * ctx->ldM));
    hipLaunchKernelGGL(k_combine_cols, dim3((unsigned)nb), dim3(TPB), 0, ctx->stream, gathered,
                       nranks, n, W, nb, P_<u64>(ctx->color), P_<u64>(ctx->colnand),
                       P_<u64>(ctx->col_and), cross_row ? P_<u64>(ctx->cross) : nullptr,
                       P_<i64>(ctx->icnt));
    KLAUNCH();
  }
  // the four result rows as index lists: all_reachable, all_isolated,
  // user_crosscheck, system_isolation
  for (int r = 0; r < 4; ++r)   // one job per row; row totals land in SZ_IDX0..3
    KTRY(sb.add(P_<i64>(ctx->icnt) + r * nb, nb, P_<i64>(ctx->ioff) + r * (nb + 1),
                SZ_IDX0 + r));
  sb.publish(SZ_ERR);   // the group-id check's atomics, for the host's sync 3
  // (an earlier scan's total: one host signal for all; the side scans store
  // their totals to the host directly)
  if (want_shadow && !compacted) sb.publish(SZ_NL);
  if (sb.jobs.count == 0) ctx->sig_armed = 0;   // (no scan raises the signal: an event)
  KTRY(sb.run());
  IdxRows ir{};
  ir.W = W;
  ir.n = n;
  ir.nb = nb;
  ir.row[0] = P_<u64>(ctx->col_and);
  ir.row[1] = P_<u64>(ctx->color);
  ir.inv[1] = 1;
  ir.row[2] = cross_row ? P_<u64>(ctx->cross) : nullptr;
  ir.row[3] = ctx->vs_sys_on ? P_<u64>(ctx->sysrow) : nullptr;
  ir.inv[3] = 1;
  int32_t* idx_dev = P_<int32_t>(ctx->idxd);
  if (n > 0 && W > 0) {
    hipLaunchKernelGGL(k_idx_write, dim3((unsigned)nb, 4), dim3(TPB), 0, ctx->stream, ir,
                       P_<i64>(ctx->ioff), nb + 1, P_<u64>(ctx->sizes) + SZ_IDX0, idx_dev);
    KLAUNCH();
  }
  // Page-locked result buffers (kano_host_alloc): the whole tail is queued
  // at once on the engine stream, sized on the device -- policy_shadow's
  // compaction and emission into buffers sized from the subset-test count and
  // the last call, the copies of scan-total length -- and the host waits
  // once, for the results; no host round trip between the scans and the
  // tail.  A total past a buffer's capacity leaves that step undone and the
  // host redoes it sized (first call, or a larger output).
  if (direct)
    return verify_back_direct(ctx, idx, idx_h, counts, shadow_pairs, pairs_h, shadow_cap,
                              shadow_count, may_async && ctx->async_rows, compacted);
  // the list sizes, policy_shadow's sizes and the group check travel to the
  // host: it waits on the signal (or the event) only, then queues the tail
  // (policy_shadow's compaction and emission, the copies) on stream2 and the
  // matrix write behind the tail on stream3.  The tail runs on a quiet
  // device (beside a matrix write its short latency-bound kernels took ~3x
  // longer); the write then overlaps the host's return and, under
  // asynchronous completion, the next call's build
  constexpr int NS = SZ_ERR - SZ_NL + 1;
  using clk = std::chrono::steady_clock;
  auto tmark = clk::now();
  auto part = [&](int k) {   // max host time of back's parts (kano_host_times)
    const auto t = clk::now();
    ctx->ht[k] = std::max(ctx->ht[k], std::chrono::duration<double, std::micro>(t - tmark).count());
    tmark = t;
  };
  const bool signalled = ctx->sig_armed != 0;
  KTRY(mirror_begin(ctx));
  hipEvent_t tail_ev = signalled ? nullptr : ctx->ev_sizes;
  const bool async = may_async && ctx->async_rows;
  if (!tail_ev) {
    KCHK(hipEventRecord(ctx->ev_sizes, ctx->stream));
    tail_ev = ctx->ev_sizes;
  }
  part(12);
  i64 v[NS];
  KTRY(mirror_wait(ctx, SZ_NL, NS, v));
  tmark = clk::now();
  if (ctx->vs_cross_on && (v[SZ_ERR - SZ_NL] & 0xffffffff)) {
    (void)sync(ctx);
    return fail(ctx, -EINVAL, "kano_verify: a group id lies outside [0, ngroups)");
  }
  i64 nidx = 0;
  for (int r = 0; r < 4; ++r) {
    counts[r] = v[SZ_IDX0 - SZ_NL + r];
    nidx += counts[r];
  }
  if (!ctx->vs_have_sys) counts[3] = -1;
  // the tail on stream2 (the shadow tests there have joined the engine
  // stream already): policy_shadow's compaction and emission, the list and
  // pair copies
  hipStream_t cs = ctx->stream2;
  KCHK(hipStreamWaitEvent(cs, tail_ev, 0));
  i64 total = 0;
  if (want_shadow) {
    total = v[SZ_PAIRS - SZ_NL];
    if (shadow_cap >= 0) {
      KTRY(shadow_back(ctx, v[0], total, cs));
      part(13);
      ctx->shadow_total = total;
    } else {
      // count only: every subset test ran (the flags and the per-pod counts
      // above); the pairs are neither compacted nor emitted (C4: ~1e11)
      ctx->shadow_total = -1;
    }
    *shadow_count = total;
  }
  tmark = clk::now();
  if (nidx > 0) {
    KTRY(copy_out(ctx, idx, idx_dev, sizeof(int32_t) * nidx, cs));
  }
  part(15);
  if (want_shadow && shadow_pairs && total > 0 && total <= shadow_cap)
    KTRY(copy_out(ctx, shadow_pairs, ctx->out.p, sizeof(int2) * total, cs));
  part(16);
  // asynchronous completion: the host waits for the result copies only; the
  // matrix write ends on stream3 (settle, or the next kano_verify's build
  // beside it on the other input set)
  KCHK(hipEventRecord(ctx->ev_tail, cs));
  if (ctx->vs_rows) {
    ctx->rows_overlap = async;
    ctx->rows_after = ctx->ev_tail;
    const int rc = launch_rows(ctx);
    ctx->rows_overlap = false;
    ctx->rows_after = nullptr;
    KTRY(rc);
  }
  // later work on the main stream (a fetch of the pairs, the next build)
  // follows the tail
  KCHK(hipEventRecord(ctx->ev_fork, cs));
  KCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_fork, 0));
  part(17);
  if (async) {
    KCHK(hipEventSynchronize(ctx->ev_tail));
    part(14);
    ctx->async_pending = true;
    return 0;
  }
  KTRY(sync(ctx));
  part(14);
  return 0;
}
// host time of one kano_verify / kano_verify_gather call by phase
// (kano_host_times): a stall names its phase
void host_time_record(kano_ctx* ctx, std::chrono::steady_clock::time_point t0,
                      std::chrono::steady_clock::time_point t1,
                      std::chrono::steady_clock::time_point t2) {
  auto us = [](std::chrono::steady_clock::duration d) {
    return std::chrono::duration<double, std::micro>(d).count();
  };
  double* h = ctx->ht;
  if (h[0] > 0) h[4] += us(t0 - ctx->ht_last);
  h[0] += 1;
  h[1] += us(t1 - t0);
  h[2] += us(t2 - t1);
  h[3] += ctx->ht_wait_cur;
  h[5] = std::max(h[5], us(t1 - t0));
  h[6] = std::max(h[6], us(t2 - t1));
  h[7] = std::max(h[7], ctx->ht_wait_cur);
  h[8] = std::max(h[8], us(t2 - t0));
  ctx->ht_last = t2;
}
}  // namespace

extern "C" {

int kano_verify(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                int64_t* shadow_count) {
  if (!ctx) return -EINVAL;
  if (!counts || (!idx && ctx->n > 0))
    return fail(ctx, -EINVAL, "kano_verify: idx / counts must not be NULL");
  ring_bell(ctx);   // (a primed prologue starts now: this call takes it)
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  ctx->ht_wait = 0;
  ctx->ht_wait_cur = 0.0;
  KTRY(verify_front(ctx, path, gid, ngroups, sys_row, shadow_count != nullptr, nullptr,
                    shadow_cap < 0));
  const auto t1 = clk::now();
  const int rc =
      verify_back(ctx, nullptr, 0, idx, counts, shadow_pairs, shadow_cap, shadow_count, true);
  host_time_record(ctx, t0, t1, clk::now());
  return rc;
}

int kano_set_pipeline(kano_ctx* ctx, int on) {
  if (!ctx) return -EINVAL;
  if (!on) KTRY(unprime(ctx));
  ctx->pipeline = on ? 1 : 0;
  return 0;
}

int kano_settle(kano_ctx* ctx) {
  if (!ctx) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  return settle(ctx);
}

int kano_gate_timing(kano_ctx* ctx, int reset, int64_t* gates, double* mean_us,
                     double* max_us) {
  if (!ctx) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));   // (every queued gate open and ended)
  // (the latest gate is left out when an unprime opened it: it waited for
  // whatever came after the last call, not for the next call)
  const u64 last = ctx->bell_seq - (ctx->gate_forced == ctx->bell_seq ? 1 : 0);
  const u64 n = last > ctx->gate_seq0 ? std::min<u64>(last - ctx->gate_seq0, GATE_RING) : 0;
  double sum = 0.0, mx = 0.0;
  if (n > 0 && ctx->gate_wait.p) {
    u64 ring[GATE_RING];
    KCHK(hipMemcpy(ring, ctx->gate_wait.p, sizeof(ring), hipMemcpyDeviceToHost));
    for (u64 q = 0; q < n; ++q) {
      const double us = (double)ring[(last - q) % GATE_RING] * 1e3 / (double)ctx->wall_khz;
      sum += us;
      mx = std::max(mx, us);
    }
  }
  if (gates) *gates = (int64_t)n;
  if (mean_us) *mean_us = n ? sum / (double)n : 0.0;
  if (max_us) *max_us = mx;
  if (reset) ctx->gate_seq0 = ctx->bell_seq;
  return 0;
}

int kano_host_times(kano_ctx* ctx, double* out, int reset) {
  if (!ctx || !out) return -EINVAL;
  for (int k = 0; k < 20; ++k) out[k] = ctx->ht[k];
  if (reset)
    for (double& v : ctx->ht) v = 0.0;
  return 0;
}

int kano_verify_shard(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups,
                      int64_t sys_row, int with_shadow, uint64_t* words_dev) {
  if (!ctx) return -EINVAL;
  if (!words_dev) return fail(ctx, -EINVAL, "kano_verify_shard: words_dev is NULL");
  return verify_front(ctx, path, gid, ngroups, sys_row, with_shadow != 0,
                      reinterpret_cast<u64*>(words_dev), with_shadow == 2);
}

int kano_verify_combine(kano_ctx* ctx, const uint64_t* gathered_dev, int32_t nranks,
                        int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                        int64_t* shadow_count) {
  if (!ctx) return -EINVAL;
  if (!counts || (!idx && ctx->n > 0) || !gathered_dev || nranks < 1)
    return fail(ctx, -EINVAL, "kano_verify_combine: bad arguments");
  if (ctx->vs_open && ctx->vs_shadow && !shadow_count)
    return fail(ctx, -EINVAL, "kano_verify_combine: shadow_count is NULL but the shard ran policy_shadow");
  // (gathered_dev is written on the context's stream: the combine may
  // complete asynchronously like kano_verify)
  return verify_back(ctx, reinterpret_cast<const u64*>(gathered_dev), nranks, idx, counts,
                     shadow_pairs, shadow_cap, shadow_count, true);
}

int kano_verify_gather(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups,
                       int64_t sys_row, int with_shadow, void* comm, int32_t nranks,
                       int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                       int64_t* shadow_count) {
  if (!ctx) return -EINVAL;
  if (nranks < 1) return fail(ctx, -EINVAL, "kano_verify_gather: bad communicator");
  if (!counts || (!idx && ctx->n > 0))
    return fail(ctx, -EINVAL, "kano_verify_gather: idx / counts must not be NULL");
  if (with_shadow && !shadow_count)
    return fail(ctx, -EINVAL, "kano_verify_gather: shadow_count is NULL but with_shadow is set");
  ring_bell(ctx);   // (a primed prologue starts now: this call takes it)
  // comm NULL: rank 0 of nranks emulated on this device (a timing diagnostic:
  // the other ranks' words are zero, the all-gather a device copy)
  const RcclAllGather ag = comm ? rccl_all_gather() : nullptr;
  if (comm && !ag)
    return fail(ctx, -ENOSYS, "kano_verify_gather: no RCCL in the process (ncclAllGather)");
  const i64 nw = 3 * ctx->W;     // [OR | cross | NAND] words of a shard (same W on every rank)
  KTRY(dalloc(ctx, ctx->xw, sizeof(u64) * std::max<i64>(1, nw)));
  const void* xg_before = ctx->xg.p;
  KTRY(dalloc(ctx, ctx->xg, sizeof(u64) * std::max<i64>(1, nw * nranks)));
  if (!comm && (ctx->xg.p != xg_before || ctx->xg_emul != nw * nranks)) {
    KCHK(hipMemsetAsync(ctx->xg.p, 0, sizeof(u64) * std::max<i64>(1, nw * nranks), ctx->stream));
    ctx->xg_emul = nw * nranks;
  }
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  ctx->ht_wait = 0;
  ctx->ht_wait_cur = 0.0;
  KTRY(verify_front(ctx, path, gid, ngroups, sys_row, with_shadow != 0, P_<u64>(ctx->xw),
                    with_shadow == 2));
  if (comm) ctx->xg_emul = -1;
  if (nw > 0 && comm) {
    const int rc = ag(ctx->xw.p, ctx->xg.p, (size_t)nw, RCCL_UINT64, comm, ctx->stream);
    if (rc != 0) {
      (void)sync(ctx);
      return fail(ctx, -EIO, "kano_verify_gather: ncclAllGather returned " + std::to_string(rc));
    }
  } else if (nw > 0) {
    KCHK(hipMemcpyAsync(ctx->xg.p, ctx->xw.p, sizeof(u64) * nw, hipMemcpyDeviceToDevice,
                        ctx->stream));
  }
  const auto t1 = clk::now();
  const int rc = verify_back(ctx, P_<u64>(ctx->xg), nranks, idx, counts, shadow_pairs,
                             shadow_cap, shadow_count, true);
  host_time_record(ctx, t0, t1, clk::now());
  return rc;
}

int kano_checks_shard(kano_ctx* ctx, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                      uint64_t* words_dev) {
  KTRY(ensure_matrix(ctx));
  if (!words_dev) return fail(ctx, -EINVAL, "kano_checks_shard: words_dev is NULL");
  const i64 n = ctx->n, W = ctx->W;
  const bool stored = !gid && ngroups == KANO_STORED_GROUPS;
  const bool want_cross = gid || stored;
  // column OR / NAND of the rows as they stand (after incremental updates
  // or edits: from M; otherwise the build's own)
  if (!ctx->cols_valid) KTRY(recompute_cols(ctx));
  bool cross_on = false;
  if (want_cross) {
    KTRY(crosscheck_impl(ctx, stored ? nullptr : gid, stored ? 0 : ngroups));
    cross_on = n > 0 && rows_local(ctx) > 0 && W > 0;
  }
  const i64 nb = std::max<i64>(1, nblk(W * 64));
  KTRY(dalloc(ctx, ctx->col_and, sizeof(u64) * std::max<i64>(1, W)));
  KTRY(dalloc(ctx, ctx->sysrow, sizeof(u64) * std::max<i64>(1, W)));
  KTRY(dalloc(ctx, ctx->icnt, sizeof(i64) * 4 * nb));
  KTRY(dalloc(ctx, ctx->ioff, sizeof(i64) * 4 * (nb + 1)));
  KTRY(dalloc(ctx, ctx->idxd, sizeof(int32_t) * std::max<i64>(1, 4 * n) + 16));
  KTRY(dalloc(ctx, ctx->sizes, sizeof(u64) * SZ_SLOTS));
  if (W > 0) {
    KCHK(hipMemcpyAsync(words_dev, ctx->color.p, sizeof(u64) * W, hipMemcpyDeviceToDevice,
                        ctx->stream));
    if (cross_on)
      KCHK(hipMemcpyAsync(words_dev + W, ctx->cross.p, sizeof(u64) * W, hipMemcpyDeviceToDevice,
                          ctx->stream));
    else
      KCHK(hipMemsetAsync(words_dev + W, 0, sizeof(u64) * W, ctx->stream));
    KCHK(hipMemcpyAsync(words_dev + 2 * W, ctx->colnand.p, sizeof(u64) * W,
                        hipMemcpyDeviceToDevice, ctx->stream));
  }
  const bool have_sys = sys_row >= ctx->r0 && sys_row < ctx->r1;
  const bool sys_on = have_sys && W > 0;
  if (sys_on)
    KCHK(hipMemcpyAsync(ctx->sysrow.p, P_<u64>(ctx->M) + (sys_row - ctx->r0) * ctx->ldM,
                        sizeof(u64) * W, hipMemcpyDeviceToDevice, ctx->stream));
  // icnt rows 0-2 come from kano_verify_combine's k_combine_cols, row 3 here
  hipLaunchKernelGGL(k_row_zero_counts, dim3((unsigned)nb), dim3(TPB), 0, ctx->stream,
                     sys_on ? P_<u64>(ctx->sysrow) : (const u64*)nullptr, n, W,
                     P_<i64>(ctx->icnt) + 3 * nb);
  KLAUNCH();
  // the combine half is kano_verify_combine's: no rows to write, no shadow
  ctx->vs_open = true;
  ctx->vs_shadow = false;
  ctx->vs_cross_want = want_cross;
  ctx->vs_cross_on = cross_on;
  ctx->vs_have_sys = have_sys;
  ctx->vs_sys_on = sys_on;
  ctx->vs_rows = false;
  ctx->vs_nb = nb;
  ctx->vs_rl = rows_local(ctx);
  return 0;
}

int kano_set_groups(kano_ctx* ctx, const int32_t* gid, int32_t ngroups) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods) return fail(ctx, -EINVAL, "kano_set_groups before kano_set_pods");
  const i64 n = ctx->n;
  if (n > 0 && !gid) return fail(ctx, -EINVAL, "kano_set_groups: gid is NULL");
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  int32_t G = 0;
  for (i64 i = 0; i < n; ++i) {
    if (gid[i] < 0) return fail(ctx, -EINVAL, "kano_set_groups: negative group id");
    G = std::max(G, gid[i] + 1);
  }
  if (ngroups > 0 && ngroups < G) return fail(ctx, -EINVAL, "kano_set_groups: id >= ngroups");
  if (ngroups > 0) G = ngroups;
  KTRY(dalloc(ctx, ctx->gids, sizeof(int32_t) * std::max<i64>(1, n)));
  if (n > 0)
    KCHK(hipMemcpyAsync(ctx->gids.p, gid, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                        ctx->stream));
  KTRY(sync(ctx));
  ctx->groups_n = n;
  ctx->groups_G = G;
  return 0;
}

int kano_host_alloc(size_t bytes, void** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  if (hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) return -ENOMEM;
  return 0;
}

void kano_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int kano_stage_times(kano_ctx* ctx, float* ms) {
  if (!ctx || !ms) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  KTRY(sync(ctx));
  for (int k = 0; k < 8; ++k) ms[k] = 0.f;
  if (ctx->built && !ctx->lists_mode) {
    if (ctx->stage_timing) {
      for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&ms[k], ctx->ev[k], ctx->ev[k + 1]);
      (void)hipEventElapsedTime(&ms[5], ctx->ev[0], ctx->ev[4]);
    }
    KTRY(resolve_rows_time(ctx));
    if (ctx->rows_timed) ms[6] = ctx->rows_ms_last;
  }
  if (ctx->stage_timing && ctx->shadow_total >= 0)
    (void)hipEventElapsedTime(&ms[4], ctx->ev[5], ctx->ev[6]);
  return 0;
}

int kano_mfma_timing(kano_ctx* ctx, double* out, int reset) {
  if (!ctx || !out) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  KTRY(sync(ctx));
  KTRY(resolve_mfma_time(ctx));
  out[0] = ctx->mfma_ms_sum;
  out[1] = (double)ctx->mfma_n;
  out[2] = ctx->mfma_ops_sum;
  out[3] = ctx->mfma_ops_last;
  if (reset) {
    ctx->mfma_ms_sum = ctx->mfma_ops_sum = 0.0;
    ctx->mfma_n = 0;
  }
  return 0;
}

int kano_rows_timing(kano_ctx* ctx, double* out, int reset) {
  if (!ctx || !out) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  KTRY(settle(ctx));
  KTRY(sync(ctx));
  KTRY(resolve_rows_time(ctx));
  out[0] = ctx->rows_ms_sum;
  out[1] = (double)ctx->rows_ms_n;
  out[2] = ctx->rows_ms_min;
  out[3] = ctx->rows_ms_max;
  if (reset) {
    ctx->rows_ms_sum = ctx->rows_ms_min = ctx->rows_ms_max = 0.0;
    ctx->rows_ms_n = 0;
  }
  return 0;
}

}  // extern "C"

// ===========================================================================
// What the multi-device group (kano_group.hip, its own translation unit)
// needs of a member context (kano_internal.hpp)
// ===========================================================================
namespace kano_int {

int ctx_device(const kano_ctx* ctx) { return ctx->device; }
hipStream_t ctx_stream(const kano_ctx* ctx) { return ctx->stream; }
int64_t ctx_n(const kano_ctx* ctx) { return ctx->n; }
int64_t ctx_W(const kano_ctx* ctx) { return ctx->W; }

int ctx_fail(kano_ctx* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }

// the member's exchange buffers: its [OR | cross | NAND] words (3 W u64) and
// every rank's (3 W nranks), written by the group's exchange -- not an
// emulated gather's zeros any more (the next comm-NULL kano_verify_gather
// clears them again)
int ctx_exchange_buffers(kano_ctx* ctx, int32_t nranks, void** xw, void** xg) {
  const i64 nw = 3 * ctx->W;
  KCHK(hipSetDevice(ctx->device));
  KTRY(dalloc(ctx, ctx->xw, sizeof(u64) * std::max<i64>(1, nw)));
  KTRY(dalloc(ctx, ctx->xg, sizeof(u64) * std::max<i64>(1, nw * nranks)));
  ctx->xg_emul = -1;
  *xw = ctx->xw.p;
  *xg = ctx->xg.p;
  return 0;
}

void* rccl_symbol(const char* name) {
  static void* h = [] {
    std::string path;
    dl_iterate_phdr(rccl_find_loaded, &path);
    void* x = nullptr;
    if (!path.empty()) x = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!x) x = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!x) x = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    return x;
  }();
  return h ? dlsym(h, name) : nullptr;
}

}  // namespace kano_int

