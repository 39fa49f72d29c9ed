/*
 * kano_hip.h -- C ABI of libkano_hip.so, the MI355X (gfx950) engine behind the
 * drop-in `kano` Python API (reference: qiyueyao/Kubernetes-verification,
 * kano_py/).  Every entry point names the reference operation it replaces.
 *
 * Conventions
 *   - return 0 on success, a negative errno-style code on failure; the message
 *     is kept in the context and returned by kano_last_error().
 *   - all pointers are HOST pointers (caller-owned) unless the name ends in
 *     _dev, in which case they are device pointers on the context's device.
 *   - device memory is owned by the context; one context = one build of the
 *     reachability matrix (or one row shard of it) on one GPU.
 *   - bit order: LSB-first inside little-endian uint64 words: bit j of a bit
 *     row lives in word j >> 6, bit j & 63.  The Python layer converts to the
 *     reference's bitarray (big-endian bytes) where the API exposes bitarrays.
 *   - not re-entrant per context; work is issued on the context's stream
 *     (kano_set_stream) and every call that returns host data synchronises it.
 *
 * Interned inputs (built by the Python host layer, kano/_intern.py):
 *   pod_val[c * n + i]  value id of label column c on pod i; -1 = pod i lacks
 *                       the key (value ids are equality classes of Python ==).
 *   sel_off/sel_col/sel_val   CSR, per policy, of the WORKING-SELECTOR terms
 *   alw_off/alw_col/alw_val   CSR, per policy, of the WORKING-ALLOW terms
 *                       (ingress/egress side swap already applied,
 *                       kano_py/kano/model.py:82-93; terms whose key no pod
 *                       carries already dropped, model.py:142-147; a rule value
 *                       no pod carries is -2 and matches nothing).
 */
#ifndef KANO_HIP_H
#define KANO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kano_ctx kano_ctx;

/* Build paths for kano_build(). */
#define KANO_PATH_AUTO    0   /* per-class choice by estimated cost          */
#define KANO_PATH_BITWISE 1   /* LDS scatter / bitwise OR of allow rows      */
#define KANO_PATH_MFMA    2   /* heavy classes by the MFMA contraction       */

/* kano_info() slots */
#define KANO_INFO_N        0
#define KANO_INFO_W        1
#define KANO_INFO_P        2
#define KANO_INFO_U        3   /* row classes (pods with equal selector keys) */
#define KANO_INFO_NNZ_SEL  4   /* sum over classes of |S(c)|                  */
#define KANO_INFO_NNZ_ALW  5   /* sum over policies of |allow_p|              */
#define KANO_INFO_HEAVY    6   /* classes built by the heavy (dense) path     */
#define KANO_INFO_ROW0     7
#define KANO_INFO_ROW1     8
#define KANO_INFO_MAXSEL   9   /* max over classes of |S(c)|                  */
#define KANO_INFO_UA      10   /* column classes (pods with equal allow keys) */
#define KANO_INFO_HEAVY_PATH 11 /* 0 none, 1 bitwise OR, 2 MFMA (fp4)         */
#define KANO_INFO_WORK_ITEMS 12 /* (class, member chunk) items of the list-based row kernel */
#define KANO_INFO_ROWS_KERNEL 13 /* the last matrix write: 2 k_rows, 3 k_rows_prep + k_rows_w
                                    (wide rows), 4 k_ptrans + k_heavy_rows_t (every class
                                    heavy, k_rows not launched), 5 the same then k_rows,
                                    6 the same then k_rows_w; 0 none yet */
#define KANO_INFO_ROWS_CUS 14   /* CUs the last matrix write's stream may use  */
#define KANO_INFO_HEAVY_SEL 15  /* sum of |S(c)| over the heavy classes       */
#define KANO_INFO_HEAVY_KERNEL 16 /* 0 none, 1 k_heavy_mc_or, 2 k_heavy_mc_mfma (split K), 3 k_heavy_gemm */
#define KANO_INFO_NSLOTS   17

/* Lifetime.  No reference counterpart: the reference keeps its state in
 * Python objects (kano_py/kano/model.py:167-169 ReachabilityMatrix.__init__). */
int  kano_create(int device, kano_ctx** out);
/* kano_create for builds the caller waits for (the drop-in build_matrix): no
 * CU-masked write stream (~15 ms of the 23 ms creation); a kano_verify step
 * on it still overlaps its matrix write with the next call, on every CU */
int  kano_create_lean(int device, kano_ctx** out);
void kano_destroy(kano_ctx* ctx);
const char* kano_last_error(const kano_ctx* ctx);
int  kano_set_stream(kano_ctx* ctx, void* hip_stream);   /* NULL = own stream */

/* Inputs.  Replace the key-presence bitsets of build_matrix
 * (kano_py/kano/model.py:128-133) and the per-policy selector dicts it reads
 * through Policy.working_selector / working_allow (model.py:82-93, 142-147). */
int kano_set_pods(kano_ctx* ctx, int64_t n, int32_t ncols, const int32_t* pod_val);
int kano_set_policies(kano_ctx* ctx, int64_t P,
                      const int64_t* sel_off, const int32_t* sel_col, const int32_t* sel_val,
                      const int64_t* alw_off, const int32_t* alw_col, const int32_t* alw_val);
/* Row shard [row_begin, row_end) of M owned by this context (multi-GPU row
 * partition); default = all rows. */
int kano_set_shard(kano_ctx* ctx, int64_t row_begin, int64_t row_end);

/* ReachabilityMatrix.build_matrix (kano_py/kano/model.py:125-165): row classes
 * (pods with equal working-selector key values) and column classes (equal
 * working-allow key values), selector evaluation on both, the per-policy
 * allowed pods and the matrix rows M[i] = OR_{p in S(i)} allow_p. */
int kano_build(kano_ctx* ctx, int path);
int kano_info(kano_ctx* ctx, int64_t* out /* KANO_INFO_NSLOTS */);

/* all_reachable / all_isolated (kano_py/kano/algorithm.py:4-17): column AND
 * and column OR of this shard's rows, W = ceil(n/64) words each. */
int kano_col_checks(kano_ctx* ctx, uint64_t* col_and, uint64_t* col_or);
/* Same, unpacked to one byte per column into device memory laid out as
 * [or(n) | cross(n) | nand(n)] so that ranks can combine with a MAX all-reduce
 * (RCCL has no bitwise reduction).  cross is filled only when a gid array was
 * passed to kano_crosscheck_dev. */
int kano_col_flags_dev(kano_ctx* ctx, uint8_t* flags_dev);

/* user_crosscheck (kano_py/kano/algorithm.py:20-42): bit j set iff some row i
 * of this shard has M[i,j] and gid[i] != gid[j]; gid = interned
 * container.getValueOrDefault(label, "") (algorithm.py:23,38), all n pods. */
int kano_crosscheck(kano_ctx* ctx, const int32_t* gid, uint64_t* cross);
int kano_crosscheck_dev(kano_ctx* ctx, const int32_t* gid, uint8_t* flags_dev);

/* Matrix access: getrow / getcol / __getitem__ / __setitem__
 * (kano_py/kano/model.py:171-184); system_isolation reads a row
 * (algorithm.py:45-55).  Rows are global indices inside this shard. */
int kano_get_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, uint64_t* dst);
/* Overwrite rows (assignment to ReachabilityMatrix.matrix rows / the
 * ReachabilityMatrix(container_size, matrix) constructor, model.py:167-169). */
int kano_put_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, const uint64_t* src);
/* Per-row 64-bit digests of rows [r0, r0 + nrows) (no reference counterpart:
 * a full-size matrix does not fit the host; the tests compare digests of
 * two builds of the same rows, e.g. bitwise vs MFMA, sharded vs unsharded).
 * digest = sum_k mix64(row[k] ^ k * 0xD6E8FEB86659FD93) mod 2^64 over the W
 * words, mix64 the splitmix64 finaliser. */
int kano_rows_digest(kano_ctx* ctx, int64_t r0, int64_t nrows, uint64_t* out);
int kano_get_col(kano_ctx* ctx, int64_t j, uint64_t* dst /* ceil(rows/64) */);
int kano_get_bit(kano_ctx* ctx, int64_t i, int64_t j, int* value);
int kano_set_bit(kano_ctx* ctx, int64_t i, int64_t j, int value);

/* Policy.working_select_set / working_allow_set (model.py:119-121, 156):
 * the n-bit sets of policy p (on a row shard, select bits exist for the
 * shard's pods only; the others read 0). */
int kano_get_policy_sets(kano_ctx* ctx, int64_t p, uint64_t* sel, uint64_t* allow);
/* Container.select_policies (model.py:158-161): row class of every pod and the
 * class-level ascending policy lists, CSR over classes (row classes cover the
 * shard's pods; cls is -1 outside the shard). */
int kano_get_classes(kano_ctx* ctx, int32_t* cls /* n */);
int kano_get_select_csr(kano_ctx* ctx, int64_t* off /* U+1 */, int32_t* pol /* nnz_sel */);
/* Container.allow_policies (model.py:162-163) and the allow sets as pod
 * lists (grouped by column class, not sorted), CSR over policies. */
int kano_get_allow_csr(kano_ctx* ctx, int64_t* off /* P+1 */, int32_t* pods /* nnz_alw */);

/* policy_shadow (kano_py/kano/algorithm.py:58-80): emits, for this shard's
 * pods in ascending order, every ordered pair (j,k) of policies selecting the
 * pod with j != k and allow_k a subset of allow_j.  kano_shadow computes and
 * returns the pair count; kano_shadow_fetch copies 2*count int32. */
int kano_shadow(kano_ctx* ctx, int64_t* count);
int kano_shadow_fetch(kano_ctx* ctx, int32_t* pairs);

/* policy_shadow over explicit inputs: n_lists per-container policy lists
 * (CSR soff/slist, the values of Container.select_policies, possibly
 * accumulated over several builds, quirk Q5) and the P allow sets as bit rows
 * of nbits bits (Policy.working_allow_set).  The context holds no matrix
 * afterwards; fetch the pairs with kano_shadow_fetch. */
int kano_shadow_lists(kano_ctx* ctx, int64_t n_lists, int64_t nbits, int64_t P,
                      const int64_t* soff, const int32_t* slist, const uint64_t* allow_rows,
                      int64_t* count);

/* policy_conflict (kano_py/kano/algorithm.py:83-100) raises AttributeError
 * as soon as any container has two selecting policies: *raises = 1 iff some
 * pod of this shard has |S(i)| >= 2. */
int kano_conflict(kano_ctx* ctx, int* raises);

/* The whole verification pass in one call (the sequence kano_py's
 * sample/example.py and tests/test_basic.py run: build_matrix, then
 * all_reachable, all_isolated, user_crosscheck, system_isolation and
 * policy_shadow) with three host syncs in total.  Results are the
 * reference's return values: ascending pod-index lists, concatenated in idx
 * (capacity 4*n) with counts[4] =
 *   [all_reachable (algorithm.py:4-9), all_isolated (:12-17),
 *    user_crosscheck for the group ids gid (:20-42; 0 when gid is NULL;
 *    ngroups > 0 declares every gid < ngroups, checked on the device, so the
 *    host does not scan gid; ngroups <= 0 scans it; gid NULL with ngroups ==
 *    KANO_STORED_GROUPS uses the groups stored by kano_set_groups),
 *    system_isolation(sys_row) (:45-55; -1 when sys_row is not in this shard)].
 * On a row shard the column lists cover only this shard's rows (combine
 * with kano_col_flags_dev / kano_crosscheck_dev across shards instead).
 * When shadow_count is non-NULL, policy_shadow runs too (kano_shadow) and
 * the pairs are copied to shadow_pairs if count <= shadow_cap (otherwise
 * fetch them with kano_shadow_fetch).  shadow_cap < 0 asks for the count
 * only: every subset test still runs, the pairs are not emitted (broad
 * selectors give ~1e11 of them; kano_shadow_fetch then fails).
 * Completion: the call returns once idx, counts and the pairs are in host
 * memory.  The matrix write (model.py:158-160) may still be running on the
 * context's stream then (KANO_TUNE=async=0 waits for it): every later call
 * on the context is ordered after it, and every entry point other than
 * kano_verify / kano_verify_shard / kano_verify_combine / kano_verify_gather /
 * kano_info waits for it first, so no
 * caller can observe an unfinished matrix. */
int kano_verify(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                int64_t* shadow_count);

/* Pipelined verification (no reference counterpart: a serving loop that
 * re-runs build_matrix + the checks on the resident inputs, as the benchmark
 * does).  With on != 0, a kano_verify / kano_verify_gather that completes
 * asynchronously also queues the NEXT call's prologue -- the build's fills
 * and classification up to the member lists, which read only the uploaded
 * tables -- on the context stream behind a gate kernel that polls a
 * page-locked word; the next kano_verify / kano_verify_gather opens the gate
 * on entry (nothing runs before the call that asks for it), so the host's
 * issue of those launches leaves the step's critical path.  Every other entry
 * point, and kano_set_pipeline(ctx, 0), opens the gate, waits and puts the
 * context back as the last call left it.  A device-wide synchronisation
 * outside the engine (hipDeviceSynchronize, torch.cuda.synchronize) while a
 * prologue is queued waits for the gate's timeout (200 ms): call
 * kano_settle first.  Default off. */
int kano_set_pipeline(kano_ctx* ctx, int on);

/* The context's queued work finished: a primed prologue's gate opened (the
 * prologue runs and is put back), an asynchronously completing matrix write
 * waited for.  Afterwards no engine work is pending on the device. */
int kano_settle(kano_ctx* ctx);

/* The pipelined calls' gates (kano_set_pipeline): how long each held the
 * engine stream -- from the end of the previous call's last engine-stream
 * kernel to the next call's bell, i.e. that stream's idle time at the step
 * boundary, timed on the device's wall clock without a profiler.  Over the
 * last min(64, gates since the last reset) gates; settles first.  reset != 0
 * starts a new window. */
int kano_gate_timing(kano_ctx* ctx, int reset, int64_t* gates, double* mean_us,
                     double* max_us);

/* kano_verify for one row shard of a multi-GPU build, in two
 * halves around the ranks' exchange step.
 *   kano_verify_shard: the build of this shard's rows and every check up to
 *     the column words, written to words_dev (DEVICE memory, 3*W uint64:
 *     [column OR | cross | column NAND] over this shard's rows; cross is 0
 *     without groups).  Asynchronous on the context stream.
 *   (the caller gathers the nranks word sets rank-major into one device
 *     buffer on the same stream, e.g. an RCCL all-gather over xGMI)
 *   kano_verify_combine: OR of the gathered sets -- all_isolated[j] = no
 *     shard reaches j (algorithm.py:12-17), all_reachable[j] = no shard
 *     misses j (:4-9), user_crosscheck[j] = some shard crosses (:27-42) --
 *     then the same outputs as kano_verify: the three global lists, this
 *     shard's system_isolation row (-1 when sys_row is elsewhere), and this
 *     shard's policy_shadow pairs (rank order = the reference's order).
 * with_shadow: 0 no policy_shadow, 1 the pairs, 2 the pair count only (then
 * kano_verify_combine takes shadow_cap < 0). */
int kano_verify_shard(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups,
                      int64_t sys_row, int with_shadow, uint64_t* words_dev);
int kano_verify_combine(kano_ctx* ctx, const uint64_t* gathered_dev, int32_t nranks,
                        int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                        int64_t* shadow_count);

/* kano_verify_shard, the exchange and kano_verify_combine in ONE call, the
 * exchange being an RCCL all-gather issued by the engine itself on the
 * context stream: comm is the caller's ncclComm_t (e.g. torch's
 * ProcessGroupNCCL._comm_ptr()) over nranks ranks, this context's rank
 * among them being the comm's own.  No host code runs between the shard's
 * checks and the combine (the caller's per-collective overhead is gone).
 * The RCCL symbols are resolved at the first call from the process (the
 * library that created comm, e.g. torch's bundled librccl), else
 * librccl.so; without them the call fails (-ENOSYS) and nothing runs.
 * comm NULL emulates rank 0 of nranks on this device (a timing diagnostic,
 * bench.py --rank-of: the all-gather becomes a device copy into rank 0's
 * slot, the other ranks' words stay zero, so the lists are partial).
 * Outputs as kano_verify_combine; with_shadow as kano_verify_shard. */
int kano_verify_gather(kano_ctx* ctx, int path, const int32_t* gid, int32_t ngroups,
                       int64_t sys_row, int with_shadow, void* comm, int32_t nranks,
                       int32_t* idx, int64_t* counts, int32_t* shadow_pairs, int64_t shadow_cap,
                       int64_t* shadow_count);

/* The checks of kano_verify_shard over the matrix rows AS THEY STAND --
 * after kano_add_policies / kano_remove_policies (or edits), which
 * kano_verify, a rebuild from the tables, would undo: this shard's
 * [OR | cross | NAND] column words to words_dev (3*W u64), the system row
 * kept if owned.  Gather the ranks' words and finish with
 * kano_verify_combine (shadow_count NULL); one rank: nranks = 1 with its own
 * words.  Column checks of algorithm.py:4-42 and system_isolation (:45-55)
 * on an incrementally updated, row-sharded matrix. */
int kano_checks_shard(kano_ctx* ctx, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                      uint64_t* words_dev);

/* user_hashmap (algorithm.py:20-24) as resident input: the group id of
 * every pod uploaded once (like the label tables), for kano_verify with
 * gid = NULL, ngroups = KANO_STORED_GROUPS.  ngroups <= 0: max(gid) + 1. */
#define KANO_STORED_GROUPS (-1)
int kano_set_groups(kano_ctx* ctx, const int32_t* gid, int32_t ngroups);

/* Timing of the last kano_build / kano_shadow stages on the context stream
 * (HIP events), milliseconds: [classes, allow, select + plan, rows stage,
 * shadow, build total, k_rows kernel alone, 0].  Slots 0-5 are recorded only
 * when the context was created with KANO_TUNE=timing=1 (each event costs
 * host time on the launch path); slot 6 always. */
int kano_stage_times(kano_ctx* ctx, float* ms /* 8 */);

/* k_rows launch times (the matrix write of model.py:158-160; HIP events on
 * its stream) accumulated over the launches since the last reset: out[4] =
 * [sum ms, launches, min ms, max ms]; reset != 0 zeroes the sums after
 * reading.  Waits for the context's work first (a benchmark reads it after
 * its timed region, kano_verify's own launches stay asynchronous). */
int kano_rows_timing(kano_ctx* ctx, double* out /* 4 */, int reset);

/* The heavy classes' MFMA contraction (k_heavy_gemm_f4 / k_heavy_mc_mfma on
 * the block-scaled fp4 MFMA, 0/1 operands; the dense path of build_matrix,
 * model.py:158-160 as Sel x Allow thresholded > 0) timed per build (HIP
 * events around its launches on the context stream): out[4] = [sum ms,
 * builds timed, sum of algorithmic ops (2 x heavy row classes x policies x
 * column classes per build), the last build's ops];
 * reset != 0 zeroes the sums after reading. */
int kano_mfma_timing(kano_ctx* ctx, double* out /* 4 */, int reset);

/* Multi-hop reachability, replacing kubesv's
 * `path` relation (kubesv/kubesv/constraint.py:233-237: path :- edge;
 * path :- edge o edge) with kano's matrix as `edge`.  Writes into dst's matrix
 *   hops = 2: P = M | M.M  (the kubesv rule),
 *   hops = k >= 1: pairs joined by a path of at most k edges,
 *   hops = 0: the transitive closure M+ (paths of any length >= 1),
 * computed from src's build at class level (row / column classes; identity
 * classes after an edit of src's matrix).  dst is a context of the same n
 * holding a matrix (e.g. a build with no policies); afterwards it is an
 * edited matrix that every query and check of this header reads.  src must
 * hold every row (no row shard).  mode: KANO_PATH_AUTO picks per step
 * between the semi-naive bit-packed OR (sparse delta) and the fp4 MFMA
 * contraction (dense); KANO_PATH_BITWISE / KANO_PATH_MFMA force one.
 * info (nullable, 6 slots): [composition steps that added pairs, steps run,
 * steps on the MFMA, row classes, column classes, identity classes]. */
int kano_path(kano_ctx* src, kano_ctx* dst, int hops, int mode, int64_t* info);

/* kano_path on one row shard of a multi-GPU build, in two
 * halves around one exchange: T, the one-hop table over column classes, is
 * an OR over all rows, everything else is per row.
 *   kano_path_shard_words: words of T (0 for an edited shard: unsupported).
 *   kano_path_shard: this shard's part of T into t_dev (DEVICE memory).
 *   (the caller gathers the ranks' parts rank-major into one device buffer,
 *   e.g. an RCCL all-gather over xGMI)
 *   kano_path_combine: OR of the parts, then this shard's rows of the path
 *   matrix into dst (a matrix context over the same rows). */
int kano_path_shard_words(kano_ctx* src, int64_t* words);
int kano_path_shard(kano_ctx* src, uint64_t* t_dev);
int kano_path_combine(kano_ctx* src, kano_ctx* dst, const uint64_t* gathered_dev, int32_t nranks,
                      int hops, int mode, int64_t* info);

/* The on-disk / tooling row format: rows of M as
 * kano_py holds them, bitarray bytes in bitarray's default big-endian bit
 * order (kano_py/kano/model.py:136-139,158-160; bitarray.tobytes(): bit j of
 * a row is bit 7 - (j & 7) of byte j >> 3, pad bits zero), ceil(n / 8) bytes
 * per row, rows [r0, r0 + nrows) of this shard.  kano_import_rows writes such
 * rows back (an edit of M, like kano_put_rows; pad bits are cleared). */
int kano_export_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, uint8_t* dst);
int kano_import_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, const uint8_t* src);

/* Incremental policy updates.  The matrix after
 * the update equals ReachabilityMatrix.build_matrix over the updated policy
 * list (kano_py/kano/model.py:125-165); only rows the changed policies select
 * are written.  Policy ids are stable: the build's 0..P-1, then added ones in
 * order (first_id returns the batch's first).  kano_add_policies takes the
 * new policies' working terms as kano_set_policies does; term columns
 * >= the build's ncols index ncols_x extra pod columns (xval[c*n + i], the
 * batch's new keys / custom matchers, appended to earlier batches' extras).
 * kano_remove_policies marks ids removed and rewrites the rows they selected
 * from the alive policies (-EINVAL after an explicit edit of M).  Afterwards
 * the matrix reads as an edited one; kano_build / kano_verify rebuild from
 * the uploaded tables and drop the updates.  kano_added_policy_sets returns
 * an added policy's working_select_set / working_allow_set (model.py:119-121). */
int kano_add_policies(kano_ctx* ctx, int64_t Pn, int32_t ncols_x, const int32_t* xval,
                      const int64_t* sel_off, const int32_t* sel_col, const int32_t* sel_val,
                      const int64_t* alw_off, const int32_t* alw_col, const int32_t* alw_val,
                      int64_t* first_id);
int kano_remove_policies(kano_ctx* ctx, int64_t count, const int64_t* ids);
int kano_added_policy_sets(kano_ctx* ctx, int64_t id, uint64_t* sel, uint64_t* allow);

/* Kubernetes matchExpressions requirements (an
 * extension of kano_py's equality selectors; semantics of the requirements
 * kubesv adapts, kubesv/kubesv/model.py:127-160).  Appends E pod columns
 * ncols .. ncols+E-1 computed on the device: 1 where pod i meets requirement
 * e, else 0 -- op 0 In (the key's value id listed in vals[off[e]..off[e+1]),
 * sorted), 1 NotIn (absent or not listed), 2 Exists, 3 DoesNotExist; col[e]
 * is the key's column (-1: no pod carries it).  Policies then use the term
 * (ncols + e, 1).  Call after kano_set_pods, before kano_set_policies. */
int kano_set_expressions(kano_ctx* ctx, int32_t E, const int32_t* col, const int32_t* op,
                         const int64_t* off, const int32_t* vals);

/* kubesv's edge relation (kubesv/kubesv/
 * constraint.py:191-231, which replaces kano's M with a K8s reading of the
 * policies: namespaces, namespaceSelector, per-direction rules).  in_t and
 * eg_t hold full n x n builds, in_t[sel][src] = ingress_traffic(src, sel) and
 * eg_t[sel][dst] = egress_traffic(dst, sel) (one kano policy per (policy,
 * peer), built by the host from the K8s objects); dst (an n x n context, e.g.
 * kano_create + kano_set_pods with no policies) receives
 *   edge[src][dst] = OR_sel in_t[sel][src] AND eg_t[sel][dst]
 *                    | eg_t[src][dst]          if flags & KANO_K8S_SELF
 * (check_self_ingress_traffic: ingress_traffic(sel, sel)), or every pair if
 * flags & KANO_K8S_ALL (check_select_by_no_policy with a pod selected by no
 * policy: that pod receives from and sends to everyone).  dst then reads as
 * an edited matrix (every check, kano_path for kubesv's path relation).
 * dst may hold a row shard [r0, r1) (kano_set_shard): only its rows are
 * written (class-level form; the sources are full builds, typically made
 * with kano_build_classes so their own matrices are never written).
 * Two forms: class level when both sources are unedited builds (edge[src]
 * [dst] = Ec[cc_i(src)][cc_e(dst)] | Mc_e[rc_e(src)][cc_e(dst)], Ec from two
 * OR-products over the builds' classes, then one expansion to pods), else --
 * or with KANO_K8S_PODS -- pod level (InT transposed, one OR-product).
 * info (nullable): [0] the bits the pod-level product added beyond the self
 * term (-1 for the class-level form). */
#define KANO_K8S_SELF 1
#define KANO_K8S_ALL  2
#define KANO_K8S_PODS 4
/* KANO_K8S_DST_EG: dst is itself a build of eg_t's tables over its row range
 * (kano_build writes EgT's rows, the self term), and the product is OR-ed
 * into it in place -- no expansion of the egress classes. */
#define KANO_K8S_DST_EG 8
int kano_k8s_edge(kano_ctx* in_t, kano_ctx* eg_t, kano_ctx* dst, int flags, int64_t* info);

/* kano_build without the matrix write (model.py:125-165 up to the class-level
 * matrix Mc, the lists and the column checks): M is written on first use
 * (kano_get_rows, kano_path, ...).  For sources of kano_k8s_edge, which reads
 * only Mc and the classes. */
int kano_build_classes(kano_ctx* ctx, int path);

/* Host time of kano_verify (no reference counterpart; diagnostics for the
 * benchmark, always recorded: a few clock reads per call), microseconds:
 * out[20] = [calls, front sum, back sum, size-wait sum, gap between calls sum,
 *            front max, back max, size-wait max, call max,
 *            size wait 1 max, size wait 2 max, size wait 3 max,
 *            back's parts max: lists + matrix-write launch, policy_shadow's
 *            emission launches, wait for the tail's copies, list copy issue,
 *            pair copy issue, event records, 0, 0];
 * "front" is the build and checks up to the column words, "back" the result
 * lists, the matrix write's launch and the wait for the host results.
 * reset != 0 zeroes them after reading. */
int kano_host_times(kano_ctx* ctx, double* out /* 20 */, int reset);

/* One process over G devices (SURVEY.md §8(b) kano_init(ngpu), §8(e) row
 * sharding; no reference counterpart: kano_py is single-process).  The group
 * owns G member contexts, member r on device devices[r] (NULL: r) with its
 * own streams, each driven by its own persistent host thread (started with
 * the group): a group call hands every member its part and returns when all
 * are done, so the members' uploads, builds and host syncs overlap.  The
 * column checks exchange the members' [OR | cross | NAND] words: ncclAllGather
 * over xGMI (communicators from ncclCommInitAll; mode 1) when the devices are
 * distinct or the flag KANO_GROUP_RCCL asks for it (also for one member),
 * device-to-device copies (mode 2) when members share a device or
 * KANO_GROUP_COPY (flag or environment variable) asks for them; every member
 * ORs the gathered words on its device.  An RCCL exchange that should run and
 * cannot (librccl missing, ncclCommInitAll failing) fails the create: there is
 * no silent fall back to copies.  kano_group_last_error(NULL) says why the
 * last create on this thread failed.
 *   kano_group_upload: kano_set_pods (+ kano_set_expressions when E > 0) +
 *     kano_set_policies on every member, member r's rows [bounds[2r],
 *     bounds[2r+1]) (kano_set_shard) -- the inputs of ReachabilityMatrix.
 *     build_matrix (kano_py/kano/model.py:125-165), all members at once.
 *   kano_group_build: kano_build on every member at once (the whole matrix).
 *   kano_group_set_groups: kano_set_groups on every member (user_hashmap's
 *     groups, algorithm.py:20-24); kano_group_verify / _checks then take
 *     gid = NULL, ngroups = KANO_STORED_GROUPS.  gid holds n entries (n of
 *     kano_group_upload), as for kano_set_groups: the members read all n.
 *   kano_group_verify: kano_verify over the whole matrix -- the three
 *     column lists (all_reachable, all_isolated, user_crosscheck) of every
 *     row, system_isolation(sys_row) from the row's owner, policy_shadow's
 *     pairs concatenated in rank order (= the reference's container order);
 *     arguments as kano_verify_shard / kano_verify_combine (with_shadow 0 /
 *     1 pairs / 2 count only).  One hand-off: every member's shard step, the
 *     exchange between two barriers of the member threads, every combine.
 *   kano_group_checks: the same checks over the members' matrices as they
 *     stand (kano_checks_shard), no policy_shadow.
 *   kano_group_add_policies / kano_group_remove_policies: kano_add_policies /
 *     kano_remove_policies on every member's rows (§8(f) rank 4); the
 *     members' new policy ids agree (first_id).
 *   kano_group_path: kubesv's path relation (kubesv/kubesv/constraint.py:
 *     233-237) of src's row-sharded matrix into dst (a group over the same
 *     devices and row bounds holding an n x n matrix): every member's part of
 *     the one-hop table (kano_path_shard), one exchange (the transport
 *     above), every member's rows (kano_path_combine); info as kano_path.
 *   kano_group_exchange_timing: enable >= 0 switches timing of the verify
 *     exchange (two events on member 0's stream) on / off; out (may be NULL)
 *     = [exchanges timed, total ms, max ms]; reset != 0 zeroes them.
 * kano_group_info: out[0] = G, out[1] = exchange mode. */
typedef struct kano_group kano_group;
#define KANO_GROUP_LEAN 1   /* lean members (kano_create_lean) */
#define KANO_GROUP_RCCL 2   /* the RCCL exchange even for one member; an error if it fails */
#define KANO_GROUP_COPY 4   /* device copies even over distinct devices */
int  kano_group_create(int ngpu, const int* devices, kano_group** out);
/* the same with lean members (kano_create_lean): for the drop-in build_matrix */
int  kano_group_create_lean(int ngpu, const int* devices, kano_group** out);
int  kano_group_create_ex(int ngpu, const int* devices, int flags /* KANO_GROUP_* */,
                          kano_group** out);
void kano_group_destroy(kano_group* g);
const char* kano_group_last_error(const kano_group* g);
int  kano_group_info(kano_group* g, int32_t* out /* 2 */);
int  kano_group_member(kano_group* g, int r, kano_ctx** ctx);
int  kano_group_upload(kano_group* g, int64_t n, int32_t ncols, const int32_t* pod_val,
                       int32_t E, const int32_t* ecol, const int32_t* eop, const int64_t* eoff,
                       const int32_t* evals, int64_t P, const int64_t* sel_off,
                       const int32_t* sel_col, const int32_t* sel_val, const int64_t* alw_off,
                       const int32_t* alw_col, const int32_t* alw_val,
                       const int64_t* bounds /* 2 G */);
int  kano_group_build(kano_group* g, int path);
int  kano_group_set_groups(kano_group* g, const int32_t* gid, int32_t ngroups);
int  kano_group_verify(kano_group* g, int path, const int32_t* gid, int32_t ngroups,
                       int64_t sys_row, int with_shadow, int32_t* idx, int64_t* counts,
                       int32_t* shadow_pairs, int64_t shadow_cap, int64_t* shadow_count);
int  kano_group_checks(kano_group* g, const int32_t* gid, int32_t ngroups, int64_t sys_row,
                       int32_t* idx, int64_t* counts);
int  kano_group_add_policies(kano_group* g, int64_t Pn, int32_t ncols_x, const int32_t* xval,
                             const int64_t* sel_off, const int32_t* sel_col,
                             const int32_t* sel_val, const int64_t* alw_off,
                             const int32_t* alw_col, const int32_t* alw_val, int64_t* first_id);
int  kano_group_remove_policies(kano_group* g, int64_t count, const int64_t* ids);
int  kano_group_path(kano_group* src, kano_group* dst, int hops, int mode, int64_t* info /* 6 */);
int  kano_group_exchange_timing(kano_group* g, int enable, double* out /* 3 */, int reset);

/* Page-locked host buffers for fast device-to-host result copies. */
int  kano_host_alloc(size_t bytes, void** out);
void kano_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* KANO_HIP_H */
