// kano_engine.hpp -- what the engine's host translation units share: the
// context (kano_ctx) and its buffers, the error macros and the helpers
// defined in kano_hip.hip (allocation, syncs, the matrix's presence).
// kano_hip.hip holds the build, the checks and the C ABI's core;
// kano_ext.hip the extensions of SURVEY.md §8(f) (multi-hop paths, the row
// format, incremental updates, kubesv's edge relation).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <array>
#include <chrono>
#include <ctime>
#include <cstdio>
#include <dlfcn.h>
#include <link.h>
#include <thread>

#include "kano_hip.h"
#include "kano_internal.hpp"
#include "kano_prims.hpp"

using namespace kano;

namespace {
constexpr int MAX_CWW = 8192;   // column-chunk width in words (64 KB of LDS)
// (the pipelined write's chunk: whole rows up to 1M columns in 128 KB of LDS,
// one block per CU -- measured C5 rank 0 of 8: each chunk re-reads every
// allowed-pod entry of S(c), so two 64-KB chunks cost 0.3 ms of row builds a
// step, 8.4 -> 8.0 ms; C5 on one GPU neutral)
constexpr int MAX_CWW_KNOB = 16384;
constexpr int XCD_WRITE = 3;   // whole XCDs the write takes in the XCD split (96 CUs)
constexpr long long XCD_MIN_BYTES = 1ll << 30;   // the split for writes of >= 1 GiB
constexpr int HT_ROWS = 128;    // heavy rows per MFMA launch (HT = 4)
// member rows per k_rows work item (each item rebuilds its class row: C3,
// 300-step A/Bs, 16 -> 24 took the masked write 0.362 -> 0.355 ms and the
// step 0.373-0.377 -> 0.361-0.365; 8: 0.443; 64: 0.372)
constexpr int ROWS_CH = 24;
constexpr int LD_ALIGN = 16;    // M row pitch multiple, in words (128-B rows: measured +22% k_rows)
constexpr int MFMA_KMIN = 8;    // min policy blocks (64 policies each) per MFMA wave

}  // namespace

struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct ClassSet {
  std::vector<int32_t> keys;     // pod_val columns hashed
  int KS = 0;
  int packed = 0;                // the key tuple fits one u64 (bits per key: keys_d[KS..2KS))
  int tbits = 0;                 // the packed key's bits
  i64 U = 0;
  i64 m0 = 0, m1 = 0;            // pods whose membership is listed
  DBuf keys_d, table, smin, slot_of, flag, cid, cls, rep, mcnt, mcur, moff, mem, cval;
};

// One side of the policies (working selector or working allow): terms sorted
// by class-key slot, the distinct slot sets ("masks") and, after matching,
// each policy's class list pcls[pstart[p] .. + plen[p]).
// What the matrix write reads (launch_rows: k_heavy_rows_t, k_rows) -- held
// twice: back-to-back kano_verify calls build into one set while the previous
// call's k_rows still reads the other (swap_rows_inputs)
struct RowsInputs {
  DBuf wioff, wicls, soffc, slist, aloff, alist, alcoff, alc, rmoff, rmem, cmoff, cmem, ccls,
      hflag, hlist, Mc;
};

struct SideMatch {
  i64 nterms = 0;
  int NM = 0;                     // distinct masks (hash join); 0 with dense
  bool dense = false;             // too many masks: predicate evaluation
  DBuf toff, tslot, tval, pmask, moff, mslot;
  DBuf table, pslot, gcnt, goff, gcur, gmem, pstart, plen, bits, bcnt, boff;
  i64 T = 0;
};

// size slots (u64) written by the kernels that produce them (scan totals,
// counters) and read by the host with one copy per sync
enum {
  SZ_UR = 0, SZ_UA, SZ_NNZ_SEL, SZ_NNZ_ALC, SZ_NNZ_ALW, SZ_NFLAGS, SZ_WI, SZ_HEAVY, SZ_MAXSEL,
  SZ_LIGHT, SZ_HSEL, SZ_NL, SZ_PAIRS, SZ_IDX0, SZ_IDX1, SZ_IDX2, SZ_IDX3, SZ_ERR, SZ_SLOTS = 18,
  SZ_SIGNAL = SZ_SLOTS   // host mirror only: the scans' host signal word
};

constexpr size_t ROW_STAGE_BYTES = 256 * 1024;

struct kano_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;

  i64 n = 0, W = 0, ldM = 0, P = 0, PB = 0;
  int ncols = 0;
  std::vector<int32_t> colbits;  // bits of (value id + 1) per pod_val column
  i64 r0 = 0, r1 = -1;
  bool have_pods = false, have_pols = false, built = false;
  bool lists_mode = false;   // kano_shadow_lists context: no matrix
  bool cols_valid = false;   // color/colnand describe M
  bool rows_dirty = false;   // M edited: classes no longer describe it
  bool rows_deferred = false;  // kano_build_classes: M is written on first use
  bool defer_alloc = false;    // (inside kano_build_classes: no M allocation)
  bool rows_timed = false;
  bool alist_valid = false;
  bool cols_deferred = false;
  int32_t cross_G = 0;         // group count of the last class-level crosscheck
  i64 groups_n = -1;           // kano_set_groups: pods covered (-1: none stored)
  int32_t groups_G = 0;      // group count of the stored groups
  // Test hooks (KANO_TUNE, parsed in kano_create).  Each selects between
  // shipped forms that compute the same results; none changes a result.
  int stage_timing = 0;      // timing=1: the stage events of kano_stage_times (slots 0-5)
  int cls_packed = 1;        // packed=0: classification without packed keys (the wide-key form)
  int rows_wide = 1;         // rw=0: wide row chunks through k_rows, not k_rows_prep + k_rows_w
                             // (rw=2: k_rows_w at every chunk width -- the parity variants)
  DBuf rw_items, rw_segs, rw_ticket;  // k_rows_prep's work-item descriptors, S(c) segments
  DBuf slist_tmp;            // k_class_lists' windowed sort of long S(c) lists (P > 49k)
  int sort_ww = 768;         // sww: that sort's window (bitmap words per wave, <= SORT_LDS_WW)
  i64 rows_w_grid = 0;       // rwg: k_rows_w's persistent grid (0: one block per CU slot)
  int rows_early_heavy = 2;  // rheavy: with heavy classes the write starts after their Mc, not the tail (0: never, 1: always, 2: wide rows)
  int assign_ipt = 0;        // aipt: pods a thread in k_cls_assign_count (0: by class count)
  int async_rows = 1;        // async=0: kano_verify waits for its matrix write
  int shadow_count_mode = 0; // shcount=1|2: count-only policy_shadow pairwise | grouped
                             // (0: the device picks, shg_grouped)
  int path_dens = 8;         // pathdens: kano_path auto takes an MFMA step when the delta
                             // holds more than path_dens % of the class-level bits
  int path_tm = 2;           // pathtm / pathtn: k_path_mfma tiles per wave
  int path_tn = 2;
  int heavy_gemm = -1;       // hgemm: k_heavy_gemm_f4's wave tile (TM TN: 22, 42, 44; 0:
                             // the split-K kernel whatever the size; -1: 22)
  // AUTO's dense-path rates (xomfma TOP/s, xoor GB/s): the GEMM's 0/1 MACs x 2
  // and the bitwise OR's Mc-word reads per second, as measured on the
  // crossover sweep (scripts/mfma_sweep.py; round 6, the fp4 GEMM's 2 x 2 tile:
  // 4,500-4,700 TOP/s at >= 2,048 wave tiles, profiles/r06_mfma_sweep.jsonl)
  double xo_mfma = 4500e12, xo_or = 8500e9;
  i64 heavy_gemm_min = 512;     // HEAVY_GEMM_MIN_TILES (kano_kernels.hpp)   // hgemmmin: the GEMM's minimum wave tiles
  int time_or = 0;           // hortime=1: k_heavy_mc_or timed like the MFMA kernels
  int heavy_expand_lds = 2;  // hexplds: heavy rows by wave transposes (k_heavy_rows_t):
                             // every member row (3), the first member's with k_rows
                             // copying it (4), or by class size (2)
  int dx_on = 1;             // dx=0: never the dense path's bit matrices (k_*_dx); 2: always
  DBuf dx_sc, dx_sa;         // its SC (policy-major) and SA (class-indexed policy words)
  DBuf mct;                  // the heavy rows' McT (k_heavy_rows_t)
  bool shg_prefilled = false;  // the grouped count's table cleared by the build's fills
  i64 dx_ldY = 0, dx_PBo = 0;
  bool dense_sel = false;    // this build takes them (do_front)
  int ac_lds = 1;            // aclds=0: AC / ACT bits by global atomics, not LDS rows
  int mlists_side_ok = 1;    // mlside=0: the member lists on the engine stream
  bool mlists_side = false;  // this build's member lists went to stream2 (classify_phase2a)
  bool rin_marked = false;   // this build's last Mc launch marked ev_rin_e
  i64 sel_early_cap = -1;    // the early placement's list capacity (-1: none this build)
  int path_lds = 1;          // pathlds=0: k_path_expand16 without the LDS table
  int rows_ch = ROWS_CH;     // rch=: member rows per k_rows work item
  int rows_cww = MAX_CWW_KNOB;   // cww: k_rows column chunk (words); the chunking wide matrices
                             // (n > 524k) take, forced at small n
  int shadow_r = 0;          // shr=1/2/4/8: k_shadow_test1s's 256-pair rounds per block (0: auto)
  int shg_sub_lds = 1;       // shgsub=0: forces k_shg_sub's word-by-word row compare (the
                             // form rows wider than 64 KB of LDS take)
  // The matrix write shares the device with the next kano_verify's build
  // (asynchronous completion): a write that saturates HBM starves the
  // build's latency-bound kernels (fill 6 -> 62-107 us, class insert 25 ->
  // 50-63 us beside it).  A write of at most rows_cu_bytes therefore runs on
  // a CU-masked stream that leaves rows_cu_off CUs per XCD to the build
  // (C3: 96 of 256 CUs, k_rows 0.26 -> 0.35 ms, step 0.52 -> 0.43 ms); a
  // larger write, which outlasts any build (C5: 125 GB), takes every CU.
  int rows_cu_off = 20;      // rcu=K (0: no masked stream)
  // The XCD split (xcd=0: off): when the last build's write ran CU-masked
  // beside the next build (pipelined calls, a matrix under rows_cu_bytes) and
  // took no GEMM, the next builds run their engine streams on XCDs 3-7 and
  // the write on whole XCDs 0-2 (its own L2s), instead of every XCD with 96
  // CUs spread over them for the write.  The unmasked pair is kept in
  // stream_x / stream2_x while the masked pair is in use (and vice versa).
  int xcd_split = 1;
  i64 xcd_min_bytes = XCD_MIN_BYTES;   // xcdmin=KiB (the parity test forces small ones)
  int xcd_write = XCD_WRITE;           // xcdw: XCDs 0..xcdw-1 for the write
  int xcd_eng0 = -1;                   // xcde: first XCD of the build's streams (-1: xcdw)
  bool xcd_tried = false, eng_on_xcd = false, xcd_last_ok = false;
  int side_mode = 0;   // the side stream in use: 0 stream2, 1 stream2_x (XCDs 3-7), 2 stream2_u
  int xcd_side = -1;   // xcdside: the side stream on XCDs 3-7 (1), on all (0), -1: 1 when heavy
  hipStream_t stream_x = nullptr, stream2_x = nullptr, stream3x = nullptr;
  hipStream_t stream2_u = nullptr;   // the side stream with an every-XCD mask (its own queue)
  hipEvent_t ev_sw = nullptr, ev_sw2 = nullptr;
  i64 rows_cu_bytes = 8ll << 30;   // rcubytes=G (GiB)
  int num_cus = 0, rows_cus = 0;   // the device's CUs; those of the last write's stream

  ClassSet rc, cc;           // row classes (selector keys), column classes (allow keys)
  SideMatch sm, am;          // selector side, allow side
  i64 UAW = 0, ldC = 0;      // words per class-level row (column classes)
  i64 nnz_sel = 0, nnz_alc = 0, nnz_alw = 0, heavy_count = 0, wi_total = 0, nflags = 0;
  i64 heavy_sel = 0;         // sum of |S(c)| over the heavy classes (the bitwise OR's work)
  i64 light_cost = 0;        // allowed-pod entries the light classes' rows read
  bool rows_use_alist = false;
  int max_sel = 0;
  int heavy_path = 0;        // 1 bitwise, 2 mfma (last build)
  int heavy_kernel = 0;      // KANO_INFO_HEAVY_KERNEL (last build)
  int rows_kernel = 0;       // the last matrix write: 2 k_rows, 0 none

  DBuf pv;
  DBuf scnt, cost, soffc, scur, slist, ecls, wicls, maxs, wicnt, wioff, hflag, hoff, hlist, sq, pfoff;
  DBuf ACT, AC, nca, acnt, alcoff, alc, aloff, alist;
  DBuf M, Mc, color, colnand, col_and, col_or_c, col_nand_c;
  DBuf scan_tmp;
  i64 scan_cap = 0;          // tiles per status region of scan_tmp
  int scan_parity = 0;
  // stream2's scans (the build's side work): their own status regions
  DBuf scan_tmp2;
  i64 scan_cap2 = 0;
  int scan_parity2 = 0;
  // The build's size-independent side work on stream2 beside the join chain:
  // AC / Mc zero fills and the crosscheck's group-key sort, forked after the
  // classes (ev_pre) and joined before the lists (ev_pre_done).
  // (ev_pre_ac: AC zeroed, joined before the lists; ev_pre_done: the rest,
  // joined before the Mc writers -- each join well after its work ends, so
  // the engine stream's barrier finds it complete)
  hipEvent_t ev_pre = nullptr, ev_pre_done = nullptr, ev_pre_ac = nullptr;
  bool pre_forked = false, pre_side_pending = false, pre_ac_pending = false;
  // policy_shadow's offset scans and compaction on stream2 right after its
  // tests (pairs mode), beside the crosscheck pass and the column checks;
  // the emission stays on the engine stream behind the index lists
  bool tail_compacted = false;
  hipEvent_t ev_pairs = nullptr;   // the compaction done (stream2)
  DBuf gid, gids, cgroup, R, multi, A1, A2, own, cross, gmin, gmax, ckey, corder, kcnt, koff;
  DBuf flags, T, loff, L, tp, poff, out, tcnt, toff;
  DBuf scratch_words, ident;
  DBuf xw, xg;               // kano_verify_gather: this shard's words, all ranks' words
  i64 xg_emul = -1;          // words of xg zeroed for the emulated gather (comm NULL)
  // kano_path (in the destination context): T, R / delta ping-pong buffers,
  // the MFMA operands, the step counter
  DBuf pT, pR[2], pD[2], pA, pB, pcnt;
  // incremental updates: added policies' pod-level sets (A x W words each),
  // their extra label columns, alive flags over build + added ids
  DBuf xv, asel, aalw, iterm, idead, irows;
  i64 inc_A = 0, inc_acap = 0, inc_xcols = 0;
  std::vector<uint8_t> dead;       // P + inc_A entries
  bool user_edited = false;        // put_rows / set_bit / import: removal cannot rewrite rows
  i64 shadow_total = -1;
  // policy_shadow count-only (kano_verify with shadow_cap < 0): the grouped
  // count (k_shg_*) instead of the pair-by-pair flags
  bool vs_count_only = false;
  bool shg_ran = false;      // the grouped count was queued (its G / err exist)
  DBuf shg_h, shg_tkey, shg_trep, shg_slot, shg_isrep, shg_gidx, shg_gid, shg_reps, shg_sub,
      shg_err;
  DBuf sizes;                // SZ_* slots: list sizes the host reads at its syncs
  DBuf icnt, ioff, sysrow, idxd;
  u64* ghost = nullptr;      // pinned landing buffer for the size slots
  // pinned, coherent mirror of the size slots that the scans write directly
  // (slot-indexed): the overlapped syncs poll the host signal word the last
  // scan with host totals raises (or wait on an event when no scan does)
  void* row_stage = nullptr;  // page-locked, ROW_STAGE_BYTES (kano_get_rows)
  u64* gmirror = nullptr;     // SZ_SLOTS slots + the host signal word (SZ_SIGNAL)
  u64* gmirror_dev = nullptr;
  DBuf sig_ctr;              // the scans' arrival counter (one u32, zero between launches)
  u64 sig_seq = 0;           // last signal value handed to a scan
  u64 sig_armed = 0;         // the value the latest scan with host totals will raise
  u64 sig_wait = 0;          // what mirror_wait polls for (0: the event)
  // kano_verify's host time per call (always on: a few clock reads), read by
  // kano_host_times: [calls, front sum, back sum, wait sum, gap sum,
  // front max, back max, wait max, call max, size waits 1..3 max, back's
  // parts max: lists + matrix-write launch, policy_shadow's emission launches,
  // tail wait, list copy, pair copy, event records; the direct tail's wait
  // sum]
  double ht[20] = {};
  double ht_wait_cur = 0.0;
  int ht_wait = 0;
  std::chrono::steady_clock::time_point ht_last{};

  hipEvent_t ev[10] = {};
  // policy_shadow's subset tests run on stream2 beside the Mc chain (forked
  // at ev_fork2 once the lists and AC exist, joined through ev_join2)
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork2 = nullptr, ev_join2 = nullptr;
  bool fork_pending = false;
  std::function<int(bool)> fork_hook;   // (true: ev_fork2 marked by the lists' dispatch)
  // kano_verify's tail (result copies, policy_shadow's emission) runs on
  // stream2 too (after the shadow tests' join), beside the matrix write,
  // which has stream3 to itself (normal priority: a high-priority tail slowed
  // k_rows 10%): the next kano_verify's build runs on the engine stream
  // while the previous matrix write ends
  hipStream_t stream3 = nullptr;
  hipStream_t stream3m = nullptr;    // CU-masked (rows_cu_off), for writes <= rows_cu_bytes
  bool stream3m_tried = false;       // (made on first use, ensure_masked_stream)
  hipStream_t rows_last = nullptr;   // the stream of the last matrix write
  RowsInputs rin_alt;        // the other set of k_rows' inputs
  int rows_set = 0;          // which physical set the ctx fields hold
  bool rows_overlap = false; // launch_rows: leave the engine stream free of the write
  hipEvent_t rows_after = nullptr;   // launch_rows: the write also waits for this
  // launch_rows: the inputs' marker is this event, already recorded on the
  // engine stream where the write may start (instead of recording ev_rin)
  hipEvent_t rows_in = nullptr;
  hipEvent_t ev_rin = nullptr;          // k_rows' inputs complete (engine stream)
  hipEvent_t ev_rin_e = nullptr;        // the same, marked by do_back's last launch
  hipEvent_t ev_rows_end[2] = {};       // (spare)
  // set k's matrix write done: the stop event of its k_rows dispatch (a
  // separate record cost the write stream ~4.5 us between two writes)
  hipEvent_t rows_end_ev[2] = {};
  bool rows_end_rec[2] = {false, false};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_sizes = nullptr;
  // asynchronous completion: kano_verify returns once its host results
  // (index lists, pairs) are in host memory; the matrix write ends on the
  // engine stream, behind which every later engine operation queues, and
  // every other entry point settles it first
  bool async_pending = false;
  // Pipelined calls (kano_set_pipeline): an asynchronously completing
  // kano_verify queues the next call's prologue -- the build's fills and
  // classification up to the member lists, which read only the resident
  // inputs -- behind a gate kernel (k_gate) on the engine stream, into the
  // next input set and a private size-slot array.  The next kano_verify
  // rings the bell (a store to page-locked memory) instead of issuing those
  // launches; any other entry point rings it, waits, and puts both sets back
  // (unprime).  So no work moves ahead of the call that asks for it; the
  // host's issue of the prologue moves off the step's critical path.
  int pipeline = 0;
  bool primed = false;
  bool priming = false;            // (prime_next is queuing it: no unprime from inside)
  bool consume_prime = false;      // verify_front -> build_impl: this build takes it
  bool prime_pre_marked = false;   // the prologue's member-list fill marked ev_pre
  bool prime_alist_valid = false;  // (restored by unprime)
  u64 prime_sig = 0;               // the prologue's class-count scan's host signal
  u64* bell = nullptr;             // page-locked, coherent; bell_dev its device address
  u64* bell_dev = nullptr;
  u64 bell_seq = 0;
  u64 gate_ticks = 0;              // k_gate's timeout in wall-clock ticks (200 ms)
  u64 wall_khz = 100000;           // the device's wall clock (k_gate's ticks)
  DBuf gate_wait;                  // k_gate's waits, a ring of GATE_RING slots
  u64 gate_seq0 = 0;               // bell_seq at kano_gate_timing's last reset
  u64 gate_forced = 0;             // the last gate an unprime opened
  DBuf sizes_alt;                  // the size slots the primed prologue writes
  hipEvent_t ev_tail = nullptr;    // the result copies of kano_verify's tail
  // the matrix write's launch times (ev_rt[set][0] -> [1], recorded by its
  // own dispatch), resolved once the launch is known to be complete: the
  // last one, and sums since kano_rows_timing's reset
  hipEvent_t ev_rt[2][2] = {};
  bool rows_time_pending[2] = {false, false};
  // the heavy classes' MFMA contraction (k_heavy_gemm_f4 / k_heavy_mc_mfma, every launch
  // of a build between one pair of events), for kano_mfma_timing
  hipEvent_t ev_m0 = nullptr, ev_m1 = nullptr;
  bool mfma_time_pending = false;
  double mfma_ops_last = 0.0, mfma_ops_sum = 0.0, mfma_ms_sum = 0.0;
  i64 mfma_n = 0;
  float rows_ms_last = 0.f;
  double rows_ms_sum = 0.0, rows_ms_min = 0.0, rows_ms_max = 0.0;
  i64 rows_ms_n = 0;
  // kano_verify halves (kano_verify_shard -> kano_verify_combine)
  bool vs_open = false, vs_shadow = false, vs_cross_want = false, vs_cross_on = false;
  bool vs_have_sys = false, vs_sys_on = false;
  bool vs_rows = false;      // the combine writes the shard's rows (not after kano_checks_shard)
  i64 vs_nb = 0, vs_rl = 0;
};

#define KCHK(expr)                                                                 \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      ctx->err = std::string(#expr) + " -> " + hipGetErrorString(e_);             \
      return -EIO;                                                                 \
    }                                                                              \
  } while (0)

#define KLAUNCH()                                                                  \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      ctx->err = std::string("kernel launch at line ") + std::to_string(__LINE__) + \
                 " -> " + hipGetErrorString(e_);                                   \
      return -EIO;                                                                 \
    }                                                                              \
  } while (0)

#define KTRY(expr)       \
  do {                   \
    int rc_ = (expr);    \
    if (rc_) return rc_; \
  } while (0)

namespace kano_eng {

int fail(kano_ctx* ctx, int code, const std::string& msg);
int settle(kano_ctx* ctx);
int dalloc(kano_ctx* ctx, DBuf& b, size_t bytes);
void dfree(DBuf& b);
int sync(kano_ctx* ctx);
int ensure_built(kano_ctx* ctx);
int ensure_matrix(kano_ctx* ctx);
i64 rows_local(const kano_ctx* ctx);

template <typename T>
T* P_(DBuf& b) {
  return reinterpret_cast<T*>(b.p);
}

inline unsigned nblk(i64 n, i64 per = TPB) { return (unsigned)((n + per - 1) / per); }

}  // namespace kano_eng

