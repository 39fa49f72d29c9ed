// kano_inc.hpp -- incremental policy updates: the
// matrix after adding or removing policies equals a build over the updated
// policy list (kano_py/kano/model.py:125-165), but only the rows the changed
// policies select are touched.
//   add:    sel_q / allow_q of the new policies evaluated per pod (the
//           predicate of model.py:95-111 on interned ids), then
//           M[i] |= allow_q for i in sel_q.
//   remove: the rows selected by a removed policy are rewritten from the
//           alive policies: the class part OR_{p in S(rc(i)), alive} AC[p]
//           (expanded through the column classes) | OR of the alive added
//           policies that select i.
#pragma once
#include "kano_prims.hpp"

namespace kano {

// One side (blockIdx.z: 0 select, 1 allow) of new policy blockIdx.y over pods
// blockIdx.x * TPB + threadIdx.x: all terms (col, val) must hold; columns
// past ncols live in the extra-column table xv.  A term whose value id is
// negative (no pod carries the rule) never matches.  One ballot per wave
// gives the word.
__global__ __launch_bounds__(TPB) void k_inc_eval(const int32_t* __restrict__ pv, i64 n,
                                                  int32_t ncols, const int32_t* __restrict__ xv,
                                                  const i64* __restrict__ soff,
                                                  const int32_t* __restrict__ scol,
                                                  const int32_t* __restrict__ sval,
                                                  const i64* __restrict__ aoff,
                                                  const int32_t* __restrict__ acol,
                                                  const int32_t* __restrict__ aval, i64 W,
                                                  u64* __restrict__ sel, u64* __restrict__ alw) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  const i64 q = blockIdx.y;
  const bool allow = blockIdx.z == 1;
  const i64* off = allow ? aoff : soff;
  const int32_t* col = allow ? acol : scol;
  const int32_t* val = allow ? aval : sval;
  bool ok = j < n;
  if (ok) {
    for (i64 t = off[q]; t < off[q + 1]; ++t) {
      const int32_t c = col[t];
      const int32_t v = c < ncols ? pv[(i64)c * n + j] : xv[(i64)(c - ncols) * n + j];
      if (val[t] < 0 || v != val[t]) {
        ok = false;
        break;
      }
    }
  }
  const u64 bal = __ballot(ok);
  const i64 w = j >> 6;
  if ((threadIdx.x & 63) == 0 && w < W) (allow ? alw : sel)[q * W + w] = bal;
}

// M[i] |= allow_q for every new policy q selecting local row i.  Block = 256
// local rows; the (row, policy) pairs it finds are OR-ed one after the other
// by the whole block (rows of one block are disjoint from other blocks').
__global__ __launch_bounds__(TPB) void k_inc_or(const u64* __restrict__ sel,
                                                const u64* __restrict__ alw, i64 W, i64 q0,
                                                i64 nq, i64 r0, i64 rl, u64* __restrict__ M,
                                                i64 ldM) {
  __shared__ int32_t pr[TPB], pq[TPB];
  __shared__ int32_t npairs;
  const i64 base = (i64)blockIdx.x * TPB;
  for (i64 qa = 0; qa < nq; qa += 1) {
    if (threadIdx.x == 0) npairs = 0;
    __syncthreads();
    const i64 r = base + threadIdx.x;
    if (r < rl) {
      const i64 i = r0 + r;
      const i64 q = q0 + qa;
      if ((sel[q * W + (i >> 6)] >> (i & 63)) & 1ull) {
        const int k = atomicAdd(&npairs, 1);
        pr[k] = (int32_t)r;
        pq[k] = (int32_t)q;
      }
    }
    __syncthreads();
    const int np = npairs;
    for (int k = 0; k < np; ++k) {
      u64* row = M + (i64)pr[k] * ldM;
      const u64* a = alw + (i64)pq[k] * W;
      for (i64 w = threadIdx.x; w < W; w += TPB) row[w] |= a[w];
    }
    __syncthreads();
  }
}

// Rows to rewrite after a removal: local row i whose class lists a newly
// removed build policy, or selected by a newly removed added policy.
__global__ __launch_bounds__(TPB) void k_inc_mark(const int32_t* __restrict__ rcls,
                                                  const i64* __restrict__ soffc,
                                                  const int32_t* __restrict__ slist,
                                                  const uint8_t* __restrict__ newdead, i64 P,
                                                  const u64* __restrict__ asel, i64 W, i64 A,
                                                  i64 r0, i64 rl, int32_t* __restrict__ rows,
                                                  u64* __restrict__ count) {
  const i64 r = (i64)blockIdx.x * TPB + threadIdx.x;
  bool hit = false;
  if (r < rl) {
    const i64 i = r0 + r;
    if (rcls) {
      const int32_t c = rcls[i];
      for (i64 k = soffc[c]; k < soffc[c + 1] && !hit; ++k) hit = newdead[slist[k]] != 0;
    }
    for (i64 q = 0; q < A && !hit; ++q)
      hit = newdead[P + q] && ((asel[q * W + (i >> 6)] >> (i & 63)) & 1ull);
  }
  if (hit) rows[atomicAdd(count, 1ull)] = (int32_t)r;
}

// Rewrite local row rows[blockIdx.x] from the alive policies: the class row
// OR_{p in S(c), alive} AC[p] built in LDS (ldC words), expanded through the
// column classes (bit j = row[cc(j)]), OR the alive added policies selecting
// the row.  Without classes (rcls == nullptr: the build had no policies) only
// the added part remains.
__global__ __launch_bounds__(TPB) void k_inc_rewrite(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ rcls,
    const i64* __restrict__ soffc, const int32_t* __restrict__ slist,
    const uint8_t* __restrict__ dead, i64 P, const u64* __restrict__ AC, i64 ldC,
    const int32_t* __restrict__ ccls, i64 n, const u64* __restrict__ asel,
    const u64* __restrict__ aalw, i64 W, i64 A, i64 r0, u64* __restrict__ M, i64 ldM) {
  extern __shared__ u64 crow[];
  const i64 r = rows[blockIdx.x], i = r0 + r;
  const int32_t c = rcls ? rcls[i] : -1;
  if (c >= 0) {
    for (i64 w = threadIdx.x; w < ldC; w += TPB) {
      u64 x = 0;
      for (i64 k = soffc[c]; k < soffc[c + 1]; ++k) {
        const int32_t p = slist[k];
        if (!dead[p]) x |= AC[(i64)p * ldC + w];
      }
      crow[w] = x;
    }
  }
  __syncthreads();
  for (i64 w = threadIdx.x; w < ldM; w += TPB) {
    u64 word = 0;
    if (w < W) {
      if (c >= 0) {
        for (int b = 0; b < 64; ++b) {
          const i64 j = w * 64 + b;
          if (j >= n) break;
          const int32_t cc = ccls[j];
          word |= ((crow[cc >> 6] >> (cc & 63)) & 1ull) << b;
        }
      }
      for (i64 q = 0; q < A; ++q)
        if (!dead[P + q] && ((asel[q * W + (i >> 6)] >> (i & 63)) & 1ull)) word |= aalw[q * W + w];
    }
    M[r * ldM + w] = word;
  }
}

}  // namespace kano
