// kano_ext.hip -- the extensions of SURVEY.md §8(f) on an engine context
// (include/kano_hip.h): multi-hop reachability (kubesv/kubesv/constraint.py:
// 233-237), the matrix row format (kano_py/kano/model.py:136-139 bitarray
// bytes), incremental policy updates (model.py:125-165 over an updated policy
// list) and kubesv's edge relation (kubesv/kubesv/constraint.py:191-231).
// Shares the context and its helpers with kano_hip.hip (kano_engine.hpp).
#include "kano_engine.hpp"
#include "kano_inc.hpp"
#include "kano_k8s.hpp"
#include "kano_path.hpp"

using namespace kano_eng;

// ===========================================================================
// Multi-hop reachability (kubesv/kubesv/
// constraint.py:233-237).  See kano_path.hpp for the class-level recurrence.
// ===========================================================================
namespace {

struct PathGeom {
  bool identity = false;   // an edited M: every pod is its own row / column class
  i64 rows = 0;            // row classes (or n)
  i64 Ua = 0;              // column classes (or n)
  i64 KW = 0;              // words of a class-level row holding bits (ceil(Ua / 64))
  i64 ldR = 0;             // pitch of the class-level rows
  const u64* base = nullptr;   // R_1 = Mc (or M)
  const u64* T = nullptr;      // one hop out of a column class (pitch ldR)
};

template <int CW>
int path_or_launch(kano_ctx* ctx, const u64* D, u64* R, u64* Dn, const PathGeom& g) {
  const i64 nch = (g.ldR + 64 * CW - 1) / (64 * CW);
  hipLaunchKernelGGL(k_path_or<CW>, dim3(nblk(g.rows * nch, TPB / 64)), dim3(TPB), 0, ctx->stream,
                     D, R, Dn, g.ldR, g.T, g.ldR, g.rows, g.KW, nch, P_<u64>(ctx->pcnt));
  KLAUNCH();
  return 0;
}

template <int TM, int TN>
int path_mfma_launch(kano_ctx* ctx, const PathMfmaArgs& a, i64 tiles) {
  hipLaunchKernelGGL((k_path_mfma<TM, TN>), dim3(nblk(tiles, TPB / 64)), dim3(TPB), 0, ctx->stream,
                     a);
  KLAUNCH();
  return 0;
}

// this context's rows' part of T (all of T for a full build): T[b] = OR of
// Mc[rc(j)] over the members j of column class b in [r0, r1)
int path_t_local(kano_ctx* src, kano_ctx* ctx, u64* Tout) {
  const i64 n = src->n, Ua = src->cc.U, ldR = src->ldC, KW = (Ua + 63) / 64;
  const u64* base = P_<u64>(src->Mc);
  const i64 nch = (ldR + 255) / 256;
  if (KW <= 4 && Ua <= 65536) {
    // narrow class rows: slices of the column classes' member lists
    KTRY(dalloc(ctx, ctx->pB, sizeof(int32_t) * (Ua + 1)));
    KCHK(hipMemsetAsync(Tout, 0, sizeof(u64) * Ua * ldR, ctx->stream));
    hipLaunchKernelGGL(k_path_t_items, dim3(1), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(src->cc.moff), Ua, P_<int32_t>(ctx->pB));
    KLAUNCH();
    const i64 nitems = (n + 64 * NT_SLICE - 1) / (64 * NT_SLICE) + Ua;   // upper bound
    hipLaunchKernelGGL(k_path_t_narrow, dim3(nblk(nitems, TPB / 64)), dim3(TPB), 0, ctx->stream,
                       base, ldR, P_<int32_t>(src->rc.cls), P_<int32_t>(src->cc.moff),
                       P_<int32_t>(src->cc.mem), Ua, KW, P_<int32_t>(ctx->pB), nitems, src->r0,
                       src->r1, Tout);
  } else {
    hipLaunchKernelGGL(k_path_t<4>, dim3(nblk(Ua * nch, TPB / 64)), dim3(TPB), 0, ctx->stream,
                       base, ldR, P_<int32_t>(src->rc.cls), P_<int32_t>(src->cc.moff),
                       P_<int32_t>(src->cc.mem), Ua, KW, nch, src->r0, src->r1, Tout);
  }
  KLAUNCH();
  return 0;
}

int path_impl(kano_ctx* src, kano_ctx* ctx, int hops, int mode, int64_t* info, bool t_ready) {
  const i64 n = src->n, W = src->W, ldM = src->ldM;
  PathGeom g;
  g.identity = src->rows_dirty;
  if (g.identity) {
    g.rows = n;
    g.Ua = n;
    g.KW = W;
    g.ldR = ldM;
    g.base = P_<u64>(src->M);
    g.T = P_<u64>(src->M);   // T[b] = M[b]: column class b is pod b
  } else {
    g.rows = src->rc.U;
    g.Ua = src->cc.U;
    g.KW = (g.Ua + 63) / 64;
    g.ldR = src->ldC;
    g.base = P_<u64>(src->Mc);
  }
  const i64 Rw = g.rows * g.ldR;   // words of one class-level matrix
  i64 steps = 0, used = 0, mfma_steps = 0;
  if (n > 0 && W > 0 && hops != 1 && g.rows > 0 && g.Ua > 0) {
    if (!g.identity) {
      if (!t_ready) KTRY(path_t_local(src, ctx, P_<u64>(ctx->pT)));
      g.T = P_<u64>(ctx->pT);
    }
    // R[0] (the identity case writes the destination matrix in place), R[1]
    // for the MFMA's out-of-place steps, two delta buffers
    u64* Rb[2];
    if (g.identity) {
      Rb[0] = P_<u64>(ctx->M);
    } else {
      KTRY(dalloc(ctx, ctx->pR[0], sizeof(u64) * Rw));
      Rb[0] = P_<u64>(ctx->pR[0]);
    }
    KTRY(dalloc(ctx, ctx->pD[0], sizeof(u64) * Rw));
    KTRY(dalloc(ctx, ctx->pD[1], sizeof(u64) * Rw));
    KTRY(dalloc(ctx, ctx->pcnt, sizeof(u64) * PATH_CNT_SLOTS * PATH_CNT_STRIDE));
    // (the MFMA step writes the words its tiles cover: the rest stay zero)
    KCHK(hipMemsetAsync(ctx->pD[0].p, 0, sizeof(u64) * Rw, ctx->stream));
    KCHK(hipMemsetAsync(ctx->pD[1].p, 0, sizeof(u64) * Rw, ctx->stream));
    Rb[1] = nullptr;
    u64* Db[2] = {P_<u64>(ctx->pD[0]), P_<u64>(ctx->pD[1])};
    KCHK(hipMemcpyAsync(Rb[0], g.base, sizeof(u64) * Rw, hipMemcpyDeviceToDevice, ctx->stream));
    // the delta of step 1 is R_1 itself; its size decides the first step
    const u64* D = g.base;
    KCHK(hipMemsetAsync(ctx->pcnt.p, 0, sizeof(u64) * PATH_CNT_SLOTS * PATH_CNT_STRIDE, ctx->stream));
    hipLaunchKernelGGL(k_popcount_words, dim3(std::min<i64>(2048, nblk(Rw))), dim3(TPB), 0,
                       ctx->stream, g.base, Rw, P_<u64>(ctx->pcnt));
    KLAUNCH();
    std::vector<u64> slots(PATH_CNT_SLOTS * PATH_CNT_STRIDE);
    auto read_count = [&](u64& out) -> int {
      KCHK(hipMemcpyAsync(slots.data(), ctx->pcnt.p, sizeof(u64) * slots.size(),
                          hipMemcpyDeviceToHost, ctx->stream));
      KTRY(sync(ctx));
      out = 0;
      for (int k = 0; k < PATH_CNT_SLOTS; ++k) out += slots[(size_t)k * PATH_CNT_STRIDE];
      return 0;
    };
    u64 dbits = 0;
    KTRY(read_count(dbits));
    int ri = 0, di = 0;
    const i64 TMr = 32 * ctx->path_tm;
    const i64 Rpad = (g.rows + 255) / 256 * 256, Upad = (g.Ua + 255) / 256 * 256;
    bool have_b = false;
    const double cells = (double)g.rows * (double)g.Ua;
    for (i64 k = 2; (hops == 0 || k <= hops) && dbits > 0; ++k) {
      bool mf = mode == KANO_PATH_MFMA;
      if (mode == KANO_PATH_AUTO) mf = (double)dbits * 100.0 > ctx->path_dens * cells;
      KCHK(hipMemsetAsync(ctx->pcnt.p, 0, sizeof(u64) * PATH_CNT_SLOTS * PATH_CNT_STRIDE, ctx->stream));
      if (!mf) {
        if (g.ldR <= 128) KTRY(path_or_launch<2>(ctx, D, Rb[ri], Db[di], g));
        else KTRY(path_or_launch<4>(ctx, D, Rb[ri], Db[di], g));
      } else {
        if (!have_b) {   // T bit-transposed: B[kw][c] bit t = T[64 kw + t][c]
          KTRY(dalloc(ctx, ctx->pB, sizeof(u64) * g.KW * Upad));
          // (T rows b = column classes; out row kw = 64 of them, Upad columns)
          const i64 CG = (Upad / 64 + 15) / 16;
          hipLaunchKernelGGL(k_bit_transpose<false>, dim3(nblk(g.KW * CG, TPB / 64)), dim3(TPB),
                             0, ctx->stream, g.T, g.ldR, g.Ua, g.KW, CG, Upad,
                             (void*)P_<u64>(ctx->pB), Upad, (i64)0);
          KLAUNCH();
          have_b = true;
        }
        KTRY(dalloc(ctx, ctx->pA, sizeof(u64) * g.KW * Rpad));
        hipLaunchKernelGGL(k_word_transpose, dim3(nblk(g.KW, 64), (unsigned)(Rpad / 64)),
                           dim3(TPB), 0, ctx->stream, Rb[ri], g.ldR, g.rows, g.KW,
                           P_<u64>(ctx->pA), Rpad, g.KW);
        KLAUNCH();
        if (!Rb[1]) {
          KTRY(dalloc(ctx, ctx->pR[1], sizeof(u64) * Rw));
          Rb[1] = P_<u64>(ctx->pR[1]);
          KCHK(hipMemsetAsync(Rb[1], 0, sizeof(u64) * Rw, ctx->stream));
        }
        PathMfmaArgs a{};
        a.A = P_<u64>(ctx->pA);
        a.B = P_<u64>(ctx->pB);
        a.ldA = Rpad;
        a.ldB = Upad;
        a.KW = g.KW;
        a.base = g.base;
        a.old = Rb[ri];
        a.out = Rb[ri ^ 1];
        a.delta = Db[di];
        a.ldR = g.ldR;
        a.rows = g.rows;
        const int TNc = ctx->path_tn == 4 ? 4 : 2;
        const i64 TMc = ctx->path_tn == 4 ? 64 : TMr;
        a.tiles_n = Upad / (32 * TNc);
        a.cnt = P_<u64>(ctx->pcnt);
        // (2 x 2 waves per block, XCD-grouped block order: 8 * ceil(blocks / 8))
        const i64 blocks = (Rpad / (2 * TMc)) * (a.tiles_n / 2);
        const i64 tiles = (blocks + 7) / 8 * 8 * (TPB / 64);
        if (ctx->path_tn == 4) KTRY((path_mfma_launch<2, 4>(ctx, a, tiles)));
        else if (ctx->path_tm == 1) KTRY((path_mfma_launch<1, 2>(ctx, a, tiles)));
        else if (ctx->path_tm == 4) KTRY((path_mfma_launch<4, 2>(ctx, a, tiles)));
        else KTRY((path_mfma_launch<2, 2>(ctx, a, tiles)));
        ri ^= 1;
        ++mfma_steps;
      }
      KTRY(read_count(dbits));
      D = Db[di];
      di ^= 1;
      ++used;
      if (dbits > 0) ++steps;
    }
    if (g.identity) {
      if (ri != 0)
        KCHK(hipMemcpyAsync(Rb[0], Rb[ri], sizeof(u64) * Rw, hipMemcpyDeviceToDevice,
                            ctx->stream));
    } else {
      // P[i] bit j = R[rc(i)][cc(j)]: R bit-transposed into 16-row groups,
      // then one block per (group, word range)
      const i64 ng = (g.rows + 15) / 16, RW = (g.rows + 63) / 64, CWn = (g.Ua + 63) / 64;
      KTRY(dalloc(ctx, ctx->pA, sizeof(uint16_t) * ng * g.Ua));
      const i64 CG = (CWn + 15) / 16;
      hipLaunchKernelGGL(k_bit_transpose<true>, dim3(nblk(RW * CG, TPB / 64)), dim3(TPB), 0,
                         ctx->stream, Rb[ri], g.ldR, g.rows, RW, CG, g.Ua, ctx->pA.p, g.Ua, ng);
      KLAUNCH();
      constexpr int SUB = 2;
      // member slices when the (group, word range) blocks alone cannot fill
      // the chip and the classes are large (broad selectors)
      const i64 gxy = (i64)nblk(ldM, (i64)TPB * SUB) * ng;
      const i64 avg_members = (n + g.rows - 1) / g.rows;
      const i64 Z = std::max<i64>(1, std::min<i64>({(2048 + gxy - 1) / gxy, avg_members / 8, 64}));
      const dim3 grid(nblk(ldM, (i64)TPB * SUB), (unsigned)ng, (unsigned)Z);
      const size_t lds = sizeof(uint16_t) * (size_t)g.Ua;
      const uint16_t* rt16 = reinterpret_cast<const uint16_t*>(ctx->pA.p);
      const bool use_lds = lds <= 64 * 1024 && ctx->path_lds;
      const bool staged = avg_members >= 16;
      auto launch = [&](auto kern, size_t shm) {   // (by handle: see launch_marked)
        hipExtLaunchKernelGGL(kern, grid, dim3(TPB), (std::uint32_t)shm, ctx->stream, nullptr,
                              nullptr, 0, rt16, g.Ua, g.rows,
                           P_<int32_t>(src->cc.cls), n, P_<int32_t>(src->rc.moff),
                           P_<int32_t>(src->rc.mem), P_<u64>(ctx->M), ldM, src->r0);
      };
      if (use_lds && staged) launch(k_path_expand16<SUB, true, true>, lds);
      else if (use_lds) launch(k_path_expand16<SUB, true, false>, lds);
      else if (staged) launch(k_path_expand16<SUB, false, true>, 0);
      else launch(k_path_expand16<SUB, false, false>, 0);
      KLAUNCH();
    }
  } else if (n > 0 && W > 0) {
    // one hop (or an empty class set): the matrix itself
    KCHK(hipMemcpyAsync(ctx->M.p, src->M.p, sizeof(u64) * rows_local(src) * ldM,
                        hipMemcpyDeviceToDevice, ctx->stream));
  }
  KTRY(sync(ctx));
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  if (info) {
    info[0] = steps;
    info[1] = used;
    info[2] = mfma_steps;
    info[3] = g.rows;
    info[4] = g.Ua;
    info[5] = g.identity ? 1 : 0;
  }
  return 0;
}

}  // namespace

extern "C" {

int kano_path(kano_ctx* src, kano_ctx* dst, int hops, int mode, int64_t* info) {
  if (!src || !dst) return -EINVAL;
  if (src == dst) return fail(dst, -EINVAL, "kano_path: the destination must be another context");
  if (hops < 0) return fail(dst, -EINVAL, "kano_path: hops < 0");
  if (mode < KANO_PATH_AUTO || mode > KANO_PATH_MFMA)
    return fail(dst, -EINVAL, "kano_path: unknown mode");
  if (src->device != dst->device) return fail(dst, -EINVAL, "kano_path: contexts on two devices");
  kano_ctx* ctx = dst;
  KCHK(hipSetDevice(dst->device));
  {
    const int rc = ensure_matrix(src);
    if (rc) return fail(dst, rc, "kano_path: source: " + src->err);
  }
  if (src->r0 != 0 || src->r1 != src->n)
    return fail(dst, -ENOTSUP, "kano_path: the source holds a row shard (needs every row)");
  KTRY(ensure_matrix(dst));
  if (dst->n != src->n || dst->r0 != 0 || dst->r1 != dst->n || dst->ldM != src->ldM)
    return fail(dst, -EINVAL, "kano_path: the destination must hold a matrix of the same size");
  {
    const int rc = sync(src);   // the source's matrix and classes are complete
    if (rc) return fail(dst, rc, "kano_path: source: " + src->err);
  }
  KTRY(dalloc(ctx, ctx->pT, sizeof(u64) * std::max<i64>(1, src->cc.U * src->ldC)));
  return path_impl(src, dst, hops, mode, info, false);
}

int kano_path_shard_words(kano_ctx* src, int64_t* words) {
  if (!src || !words) return -EINVAL;
  KTRY(ensure_matrix(src));
  *words = src->rows_dirty ? 0 : src->cc.U * src->ldC;
  return 0;
}

int kano_path_shard(kano_ctx* src, uint64_t* t_dev) {
  if (!src) return -EINVAL;
  kano_ctx* ctx = src;
  KCHK(hipSetDevice(src->device));
  KTRY(ensure_matrix(src));
  if (src->rows_dirty)
    return fail(src, -ENOTSUP, "kano_path_shard: an edited row shard (needs every row)");
  if (src->cc.U * src->ldC > 0) {
    if (!t_dev) return fail(src, -EINVAL, "kano_path_shard: t_dev is NULL");
    KTRY(path_t_local(src, src, reinterpret_cast<u64*>(t_dev)));
  }
  return sync(src);
}

int kano_path_combine(kano_ctx* src, kano_ctx* dst, const uint64_t* gathered_dev, int32_t nranks,
                      int hops, int mode, int64_t* info) {
  if (!src || !dst || src == dst) return -EINVAL;
  kano_ctx* ctx = dst;
  if (hops < 0 || nranks < 1 || mode < KANO_PATH_AUTO || mode > KANO_PATH_MFMA)
    return fail(dst, -EINVAL, "kano_path_combine: bad arguments");
  if (src->device != dst->device) return fail(dst, -EINVAL, "kano_path_combine: two devices");
  KCHK(hipSetDevice(dst->device));
  {
    const int rc = ensure_matrix(src);
    if (rc) return fail(dst, rc, "kano_path_combine: source: " + src->err);
  }
  if (src->rows_dirty) return fail(dst, -ENOTSUP, "kano_path_combine: an edited row shard");
  KTRY(ensure_matrix(dst));
  if (dst->n != src->n || dst->r0 != src->r0 || dst->r1 != src->r1 || dst->ldM != src->ldM)
    return fail(dst, -EINVAL, "kano_path_combine: the destination must hold the same rows");
  {
    const int rc = sync(src);
    if (rc) return fail(dst, rc, "kano_path_combine: source: " + src->err);
  }
  const i64 nw = src->cc.U * src->ldC;
  KTRY(dalloc(ctx, ctx->pT, sizeof(u64) * std::max<i64>(1, nw)));
  if (nw > 0) {
    if (!gathered_dev) return fail(dst, -EINVAL, "kano_path_combine: gathered_dev is NULL");
    hipLaunchKernelGGL(k_or_parts, dim3(std::min<i64>(4096, nblk(nw))), dim3(TPB), 0,
                       ctx->stream, reinterpret_cast<const u64*>(gathered_dev), nranks, nw,
                       P_<u64>(ctx->pT));
    KLAUNCH();
  }
  return path_impl(src, dst, hops, mode, info, true);
}


int kano_export_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, uint8_t* dst) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!dst && nrows > 0))
    return fail(ctx, -EINVAL, "kano_export_rows: rows outside this shard");
  const i64 nb = (ctx->n + 7) / 8;
  if (nrows == 0 || nb == 0) return 0;
  // staged through scratch in chunks of <= 64 MB
  const i64 chunk = std::max<i64>(1, (64ll << 20) / nb);
  KTRY(dalloc(ctx, ctx->scratch_words, (size_t)(std::min(chunk, (i64)nrows) * nb + 16)));
  uint8_t* st = reinterpret_cast<uint8_t*>(ctx->scratch_words.p);
  for (i64 c0 = 0; c0 < nrows; c0 += chunk) {
    const i64 cr = std::min<i64>(chunk, nrows - c0);
    const i64 q = (nb + 3) / 4;
    hipLaunchKernelGGL(k_words_to_bytes, dim3(nblk(cr * q)), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->M) + (r0 - ctx->r0 + c0) * ctx->ldM, ctx->ldM, cr, nb, st);
    KLAUNCH();
    KCHK(hipMemcpyAsync(dst + c0 * nb, st, (size_t)(cr * nb), hipMemcpyDeviceToHost, ctx->stream));
    KTRY(sync(ctx));
  }
  return 0;
}

int kano_import_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, const uint8_t* src) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!src && nrows > 0))
    return fail(ctx, -EINVAL, "kano_import_rows: rows outside this shard");
  const i64 nb = (ctx->n + 7) / 8;
  if (nrows == 0 || nb == 0) return 0;
  const i64 chunk = std::max<i64>(1, (64ll << 20) / nb);
  KTRY(dalloc(ctx, ctx->scratch_words, (size_t)(std::min(chunk, (i64)nrows) * nb + 16)));
  uint8_t* st = reinterpret_cast<uint8_t*>(ctx->scratch_words.p);
  for (i64 c0 = 0; c0 < nrows; c0 += chunk) {
    const i64 cr = std::min<i64>(chunk, nrows - c0);
    KCHK(hipMemcpyAsync(st, src + c0 * nb, (size_t)(cr * nb), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_bytes_to_words, dim3(nblk(cr * ctx->ldM)), dim3(TPB), 0, ctx->stream, st,
                       cr, nb, ctx->n, P_<u64>(ctx->M) + (r0 - ctx->r0 + c0) * ctx->ldM,
                       ctx->ldM);
    KLAUNCH();
    KTRY(sync(ctx));
  }
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  ctx->user_edited = true;
  return 0;
}


// ---------------------------------------------------------------------------
// Incremental policy updates (kano_inc.hpp)

int kano_add_policies(kano_ctx* ctx, int64_t Pn, int32_t ncols_x, const int32_t* xval,
                      const int64_t* sel_off, const int32_t* sel_col, const int32_t* sel_val,
                      const int64_t* alw_off, const int32_t* alw_col, const int32_t* alw_val,
                      int64_t* first_id) {
  KTRY(ensure_matrix(ctx));
  if (Pn < 0 || ncols_x < 0 || (Pn > 0 && (!sel_off || !alw_off)) ||
      (ncols_x > 0 && !xval && ctx->n > 0))
    return fail(ctx, -EINVAL, "kano_add_policies: bad arguments");
  const i64 n = ctx->n, W = ctx->W;
  if (first_id) *first_id = ctx->P + ctx->inc_A;
  if (Pn == 0) return 0;
  const i64 ns = sel_off[Pn], na = alw_off[Pn];
  const int32_t ncol_all = ctx->ncols + (int32_t)(ctx->inc_xcols + ncols_x);
  for (i64 t = 0; t < ns; ++t)
    if (sel_col[t] < 0 || sel_col[t] >= ncol_all)
      return fail(ctx, -EINVAL, "kano_add_policies: select term column out of range");
  for (i64 t = 0; t < na; ++t)
    if (alw_col[t] < 0 || alw_col[t] >= ncol_all)
      return fail(ctx, -EINVAL, "kano_add_policies: allow term column out of range");
  // the extra columns append to the ones earlier additions brought
  if (ncols_x > 0 && n > 0) {
    const i64 have = ctx->inc_xcols * n, add = (i64)ncols_x * n;
    DBuf grown;
    KTRY(dalloc(ctx, grown, sizeof(int32_t) * (have + add)));
    if (have > 0)
      KCHK(hipMemcpyAsync(grown.p, ctx->xv.p, sizeof(int32_t) * have, hipMemcpyDeviceToDevice,
                          ctx->stream));
    KCHK(hipMemcpyAsync(P_<int32_t>(grown) + have, xval, sizeof(int32_t) * add,
                        hipMemcpyHostToDevice, ctx->stream));
    KTRY(sync(ctx));
    dfree(ctx->xv);
    ctx->xv = grown;
  }
  ctx->inc_xcols += ncols_x;
  // pod-level sets of the added policies (A x W words each side)
  const i64 A0 = ctx->inc_A, A1 = A0 + Pn;
  if (A1 > ctx->inc_acap) {
    const i64 cap = std::max<i64>(A1, 2 * ctx->inc_acap);
    DBuf s2, a2;
    KTRY(dalloc(ctx, s2, sizeof(u64) * std::max<i64>(1, cap * W)));
    KTRY(dalloc(ctx, a2, sizeof(u64) * std::max<i64>(1, cap * W)));
    if (A0 > 0 && W > 0) {
      KCHK(hipMemcpyAsync(s2.p, ctx->asel.p, sizeof(u64) * A0 * W, hipMemcpyDeviceToDevice,
                          ctx->stream));
      KCHK(hipMemcpyAsync(a2.p, ctx->aalw.p, sizeof(u64) * A0 * W, hipMemcpyDeviceToDevice,
                          ctx->stream));
    }
    KTRY(sync(ctx));
    dfree(ctx->asel);
    dfree(ctx->aalw);
    ctx->asel = s2;
    ctx->aalw = a2;
    ctx->inc_acap = cap;
  }
  // the batch's terms: [soff | aoff] (i64) then [scol | sval | acol | aval] (i32)
  const size_t hdr = sizeof(i64) * 2 * (Pn + 1);
  const size_t body = sizeof(int32_t) * 2 * (ns + na);
  std::vector<uint8_t> h(hdr + body + 16);
  std::memcpy(h.data(), sel_off, sizeof(i64) * (Pn + 1));
  std::memcpy(h.data() + sizeof(i64) * (Pn + 1), alw_off, sizeof(i64) * (Pn + 1));
  int32_t* hb = reinterpret_cast<int32_t*>(h.data() + hdr);
  if (ns) std::memcpy(hb, sel_col, sizeof(int32_t) * ns);
  if (ns) std::memcpy(hb + ns, sel_val, sizeof(int32_t) * ns);
  if (na) std::memcpy(hb + 2 * ns, alw_col, sizeof(int32_t) * na);
  if (na) std::memcpy(hb + 2 * ns + na, alw_val, sizeof(int32_t) * na);
  KTRY(dalloc(ctx, ctx->iterm, h.size()));
  KCHK(hipMemcpyAsync(ctx->iterm.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream));
  const i64* d_soff = P_<i64>(ctx->iterm);
  const i64* d_aoff = d_soff + (Pn + 1);
  const int32_t* d_b = reinterpret_cast<const int32_t*>(P_<uint8_t>(ctx->iterm) + hdr);
  u64* sel = P_<u64>(ctx->asel) + A0 * W;
  u64* alw = P_<u64>(ctx->aalw) + A0 * W;
  if (n > 0) {
    hipLaunchKernelGGL(k_inc_eval, dim3(nblk(n), (unsigned)Pn, 2), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->pv), n, ctx->ncols, P_<int32_t>(ctx->xv), d_soff, d_b,
                       d_b + ns, d_aoff, d_b + 2 * ns, d_b + 2 * ns + na, W, sel, alw);
    KLAUNCH();
    const i64 rl = rows_local(ctx);
    if (rl > 0)
      hipLaunchKernelGGL(k_inc_or, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream,
                         P_<u64>(ctx->asel), P_<u64>(ctx->aalw), W, A0, Pn, ctx->r0, rl,
                         P_<u64>(ctx->M), ctx->ldM);
    KLAUNCH();
  }
  KTRY(sync(ctx));
  ctx->inc_A = A1;
  ctx->dead.resize((size_t)(ctx->P + A1), 0);
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  return 0;
}

int kano_remove_policies(kano_ctx* ctx, int64_t count, const int64_t* ids) {
  KTRY(ensure_matrix(ctx));
  if (count < 0 || (count > 0 && !ids)) return fail(ctx, -EINVAL, "kano_remove_policies");
  if (ctx->user_edited)
    return fail(ctx, -EINVAL, "kano_remove_policies: the matrix was edited; rebuild instead");
  const i64 Ptot = ctx->P + ctx->inc_A;
  std::vector<uint8_t> newdead((size_t)std::max<i64>(1, Ptot), 0);
  i64 fresh = 0;
  for (i64 k = 0; k < count; ++k) {
    if (ids[k] < 0 || ids[k] >= Ptot) return fail(ctx, -EINVAL, "kano_remove_policies: bad id");
    if (ctx->dead[ids[k]]) return fail(ctx, -EINVAL, "kano_remove_policies: id already removed");
    if (!newdead[ids[k]]) ++fresh;
    newdead[ids[k]] = 1;
  }
  if (fresh == 0) return 0;
  for (i64 p = 0; p < Ptot; ++p) ctx->dead[p] |= newdead[p];
  const i64 n = ctx->n, W = ctx->W, rl = rows_local(ctx);
  // [newdead | dead] flags, the row list, its count
  KTRY(dalloc(ctx, ctx->idead, 2 * (size_t)std::max<i64>(1, Ptot) + 16));
  KCHK(hipMemcpyAsync(ctx->idead.p, newdead.data(), (size_t)Ptot, hipMemcpyHostToDevice,
                      ctx->stream));
  KCHK(hipMemcpyAsync(P_<uint8_t>(ctx->idead) + Ptot, ctx->dead.data(), (size_t)Ptot,
                      hipMemcpyHostToDevice, ctx->stream));
  KTRY(dalloc(ctx, ctx->irows, sizeof(int32_t) * std::max<i64>(1, rl) + 64));
  u64* cnt = reinterpret_cast<u64*>(P_<int32_t>(ctx->irows) + std::max<i64>(1, rl) + 8);
  cnt = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(cnt) + 7) & ~(uintptr_t)7);
  KCHK(hipMemsetAsync(cnt, 0, sizeof(u64), ctx->stream));
  const bool classes = ctx->rc.U > 0 && rl > 0;
  if (rl > 0) {
    hipLaunchKernelGGL(k_inc_mark, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream,
                       classes ? P_<int32_t>(ctx->rc.cls) : (const int32_t*)nullptr,
                       P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), P_<uint8_t>(ctx->idead),
                       ctx->P, P_<u64>(ctx->asel), W, ctx->inc_A, ctx->r0, rl,
                       P_<int32_t>(ctx->irows), cnt);
    KLAUNCH();
  }
  u64 nrows = 0;
  KCHK(hipMemcpyAsync(&nrows, cnt, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
  KTRY(sync(ctx));
  if (nrows > 0) {
    const size_t lds = sizeof(u64) * (size_t)std::max<i64>(1, ctx->ldC);
    if (lds > 64 * 1024) return fail(ctx, -ENOTSUP, "kano_remove_policies: too many column classes");
    hipLaunchKernelGGL(k_inc_rewrite, dim3((unsigned)nrows), dim3(TPB), lds, ctx->stream,
                       P_<int32_t>(ctx->irows),
                       classes ? P_<int32_t>(ctx->rc.cls) : (const int32_t*)nullptr,
                       P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist),
                       P_<uint8_t>(ctx->idead) + Ptot, ctx->P, P_<u64>(ctx->AC), ctx->ldC,
                       P_<int32_t>(ctx->cc.cls), n, P_<u64>(ctx->asel), P_<u64>(ctx->aalw), W,
                       ctx->inc_A, ctx->r0, P_<u64>(ctx->M), ctx->ldM);
    KLAUNCH();
  }
  KTRY(sync(ctx));
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  return 0;
}

int kano_added_policy_sets(kano_ctx* ctx, int64_t id, uint64_t* sel, uint64_t* allow) {
  KTRY(ensure_matrix(ctx));
  const i64 q = id - ctx->P;
  if (q < 0 || q >= ctx->inc_A) return fail(ctx, -EINVAL, "kano_added_policy_sets: bad id");
  const i64 W = ctx->W;
  if (W == 0) return 0;
  if (sel)
    KCHK(hipMemcpyAsync(sel, P_<u64>(ctx->asel) + q * W, sizeof(u64) * W, hipMemcpyDeviceToHost,
                        ctx->stream));
  if (allow)
    KCHK(hipMemcpyAsync(allow, P_<u64>(ctx->aalw) + q * W, sizeof(u64) * W,
                        hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

// kubesv's edge relation (kubesv/kubesv/constraint.py:191-231) from the two
// per-direction kano matrices: see kano_k8s.hpp.
int kano_k8s_edge(kano_ctx* in_t, kano_ctx* eg_t, kano_ctx* dst, int flags, int64_t* info) {
  if (!in_t || !eg_t || !dst) return -EINVAL;
  if (dst == in_t || dst == eg_t)
    return fail(dst, -EINVAL, "kano_k8s_edge: the destination must be another context");
  if (in_t->device != dst->device || eg_t->device != dst->device)
    return fail(dst, -EINVAL, "kano_k8s_edge: contexts on two devices");
  kano_ctx* ctx = dst;
  KCHK(hipSetDevice(dst->device));
  for (kano_ctx* s : {in_t, eg_t}) {
    const int rc = ensure_built(s);
    if (rc) return fail(dst, rc, "kano_k8s_edge: source: " + s->err);
    if (s->lists_mode) return fail(dst, -EINVAL, "kano_k8s_edge: a source holds policy lists");
    if (s->r0 != 0 || s->r1 != s->n)
      return fail(dst, -ENOTSUP, "kano_k8s_edge: a source holds a row shard (needs every row)");
  }
  KTRY(ensure_matrix(dst));
  const i64 n = dst->n, W = dst->W, ldM = dst->ldM, r0 = dst->r0, rl = rows_local(dst);
  if (in_t->n != n || eg_t->n != n || in_t->ldM != ldM || eg_t->ldM != ldM)
    return fail(dst, -EINVAL, "kano_k8s_edge: the three matrices must have the same size");
  const bool classes = !in_t->rows_dirty && !eg_t->rows_dirty && in_t->rc.U > 0 &&
                       eg_t->rc.U > 0 && in_t->cc.U > 0 && eg_t->cc.U > 0 &&
                       !(flags & KANO_K8S_PODS);
  const bool pod_form = !(flags & KANO_K8S_ALL) && !classes;
  if ((flags & KANO_K8S_DST_EG) && (pod_form || dst->rows_dirty || dst->P != eg_t->P))
    return fail(dst, -EINVAL, "kano_k8s_edge: KANO_K8S_DST_EG needs dst = an unedited build "
                              "of the egress policies (class-level form)");
  if (pod_form) {
    if (r0 != 0 || rl != n)
      return fail(dst, -ENOTSUP, "kano_k8s_edge: the pod-level form needs every row");
    for (kano_ctx* s : {in_t, eg_t}) {
      const int rc = ensure_matrix(s);   // (a deferred matrix write runs now)
      if (rc) return fail(dst, rc, "kano_k8s_edge: source: " + s->err);
    }
  }
  for (kano_ctx* s : {in_t, eg_t}) {
    const int rc = sync(s);   // the sources' classes / matrices are complete
    if (rc) return fail(dst, rc, "kano_k8s_edge: source: " + s->err);
  }
  u64* E = P_<u64>(dst->M);
  u64 added = 0;
  const int self = (flags & KANO_K8S_SELF) ? 1 : 0;
  if (rl > 0 && W > 0) {
    if (flags & KANO_K8S_ALL) {
      hipLaunchKernelGGL(k_k8s_ones, dim3(nblk(rl * ldM)), dim3(TPB), 0, ctx->stream, E, ldM, rl,
                         n, W);
      KLAUNCH();
    } else if (classes) {
      // class level (kano_k8s.hpp): B, EgA, Mc_i transposed, Ec, expansion;
      // only Mc and the class ids of the two builds are read
      const i64 Ui = in_t->rc.U, Xi = in_t->cc.U, Ue = eg_t->rc.U, Ye = eg_t->cc.U;
      const i64 ldCe = eg_t->ldC, ldCi = in_t->ldC;
      const i64 KWb = (Ue + 63) / 64, KWa = (Ui + 63) / 64, NWe = (Ye + 63) / 64;
      KTRY(dalloc(ctx, ctx->pA, sizeof(u64) * Ui * KWb));
      KTRY(dalloc(ctx, ctx->pB, sizeof(u64) * Ui * ldCe));
      KTRY(dalloc(ctx, ctx->pT, sizeof(u64) * Xi * KWa));
      KTRY(dalloc(ctx, ctx->pR[0], sizeof(u64) * Xi * ldCe));
      KCHK(hipMemsetAsync(ctx->pA.p, 0, sizeof(u64) * Ui * KWb, ctx->stream));
      hipLaunchKernelGGL(k_k8s_pairs, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                         P_<int32_t>(in_t->rc.cls), P_<int32_t>(eg_t->rc.cls), n,
                         P_<u64>(ctx->pA), KWb);
      KLAUNCH();
      const i64 nch = (ldCe + 255) / 256;
      hipLaunchKernelGGL(k_k8s_or_rows<4>, dim3(nblk(Ui * nch, TPB / 64)), dim3(TPB), 0,
                         ctx->stream, P_<u64>(ctx->pA), KWb, KWb, P_<u64>(eg_t->Mc), ldCe, NWe,
                         P_<u64>(ctx->pB), ldCe, Ui, nch);
      KLAUNCH();
      const i64 CGi = ((Xi + 63) / 64 + 15) / 16;
      hipLaunchKernelGGL(k_k8s_transpose, dim3(nblk(KWa * CGi, TPB / 64)), dim3(TPB), 0,
                         ctx->stream, P_<u64>(in_t->Mc), ldCi, Ui, KWa, CGi, Xi,
                         P_<u64>(ctx->pT), KWa);
      KLAUNCH();
      hipLaunchKernelGGL(k_k8s_or_rows<4>, dim3(nblk(Xi * nch, TPB / 64)), dim3(TPB), 0,
                         ctx->stream, P_<u64>(ctx->pT), KWa, KWa, P_<u64>(ctx->pB), ldCe, NWe,
                         P_<u64>(ctx->pR[0]), ldCe, Xi, nch);
      KLAUNCH();
      // class rows of <= K8S_STAGE_W words are staged in LDS by the expansion
      // (launched by handle: see launch_marked)
      auto K8S_EXPAND = ldCe <= K8S_STAGE_W ? k_k8s_expand<true> : k_k8s_expand<false>;
      const int32_t* cci = P_<int32_t>(in_t->cc.cls);
      const int32_t* rce = P_<int32_t>(eg_t->rc.cls);
      const int32_t* cce = P_<int32_t>(eg_t->cc.cls);
      // KANO_K8S_DST_EG: dst already holds the shard's EgT rows (a build of
      // the egress policies), so the self term needs no expansion
      const bool in_place = self && (flags & KANO_K8S_DST_EG);
      const i64 Us = (self && !in_place) ? Ue : 0;
      if (Xi + Us <= std::max<i64>(rl / 2, 1) && ldM % 2 == 0) {
        // expand the class rows once (Ec's Xi rows; for self traffic Mc_e's
        // Ue rows, i.e. EgT by egress row class), then stream them to the
        // shard's pod rows
        KTRY(dalloc(ctx, ctx->pR[1], sizeof(u64) * (Xi + Us) * ldM));
        u64* Xe = P_<u64>(ctx->pR[1]);
        u64* Se = Xe + Xi * ldM;
        hipExtLaunchKernelGGL(K8S_EXPAND, dim3(nblk(ldM, K8S_XW), nblk(Xi, K8S_XR)), dim3(TPB), 0,
                           ctx->stream, nullptr, nullptr, 0, P_<u64>(ctx->pR[0]), ldCe, (const int32_t*)nullptr,
                           (const u64*)nullptr, ldCe, (const int32_t*)nullptr, cce, 0, (i64)0, Xi,
                           n, W, Xe, ldM);
        KLAUNCH();
        if (Us) {
          hipExtLaunchKernelGGL(K8S_EXPAND, dim3(nblk(ldM, K8S_XW), nblk(Ue, K8S_XR)), dim3(TPB),
                              0, ctx->stream, nullptr, nullptr, 0, P_<u64>(eg_t->Mc), ldCe, (const int32_t*)nullptr,
                             (const u64*)nullptr, ldCe, (const int32_t*)nullptr, cce, 0, (i64)0,
                             Ue, n, W, Se, ldM);
          KLAUNCH();
        }
        if (in_place) {
          hipLaunchKernelGGL(k_k8s_or_into, dim3(nblk(rl * (ldM / 2))), dim3(TPB), 0, ctx->stream,
                             Xe, cci, r0, rl, ldM, E);
        } else {
          hipLaunchKernelGGL(k_k8s_rows, dim3(nblk(rl * (ldM / 2))), dim3(TPB), 0, ctx->stream,
                             Xe, cci, Se, rce, self, r0, rl, ldM, E);
        }
        KLAUNCH();
      } else {
        hipExtLaunchKernelGGL(K8S_EXPAND, dim3(nblk(ldM, K8S_XW), nblk(rl, K8S_XR)), dim3(TPB), 0,
                           ctx->stream, nullptr, nullptr, 0, P_<u64>(ctx->pR[0]), ldCe, cci, P_<u64>(eg_t->Mc), ldCe,
                           rce, cce, self, r0, rl, n, W, E, ldM);
        KLAUNCH();
      }
      added = (u64)-1;
    } else {
      // pod level: edge starts as EgT (self ingress traffic: sel = src) or
      // empty, then edge[src] |= OR_{sel in In[src]} EgT[sel], In = InT^T
      if (self)
        KCHK(hipMemcpyAsync(E, eg_t->M.p, sizeof(u64) * n * ldM, hipMemcpyDeviceToDevice,
                            ctx->stream));
      else
        KCHK(hipMemsetAsync(E, 0, sizeof(u64) * n * ldM, ctx->stream));
      KTRY(dalloc(ctx, ctx->pA, sizeof(u64) * n * ldM));
      KTRY(dalloc(ctx, ctx->pB, sizeof(u64) * n * ldM));
      KTRY(dalloc(ctx, ctx->pcnt, sizeof(u64) * PATH_CNT_SLOTS * PATH_CNT_STRIDE));
      KCHK(hipMemsetAsync(ctx->pcnt.p, 0, sizeof(u64) * PATH_CNT_SLOTS * PATH_CNT_STRIDE,
                          ctx->stream));
      const i64 CG = (W + 15) / 16;
      hipLaunchKernelGGL(k_k8s_transpose, dim3(nblk(W * CG, TPB / 64)), dim3(TPB), 0, ctx->stream,
                         P_<u64>(in_t->M), ldM, n, W, CG, n, P_<u64>(ctx->pA), ldM);
      KLAUNCH();
      PathGeom g;
      g.identity = true;
      g.rows = n;
      g.Ua = n;
      g.KW = W;
      g.ldR = ldM;
      g.T = P_<u64>(eg_t->M);
      if (ldM <= 128) KTRY(path_or_launch<2>(ctx, P_<u64>(ctx->pA), E, P_<u64>(ctx->pB), g));
      else KTRY(path_or_launch<4>(ctx, P_<u64>(ctx->pA), E, P_<u64>(ctx->pB), g));
      std::vector<u64> slots(PATH_CNT_SLOTS * PATH_CNT_STRIDE);
      KCHK(hipMemcpyAsync(slots.data(), ctx->pcnt.p, sizeof(u64) * slots.size(),
                          hipMemcpyDeviceToHost, ctx->stream));
      KTRY(sync(ctx));
      for (int k = 0; k < PATH_CNT_SLOTS; ++k) added += slots[(size_t)k * PATH_CNT_STRIDE];
    }
  }
  KTRY(sync(ctx));
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  if (info) info[0] = (int64_t)added;
  return 0;
}

}  // extern "C"
