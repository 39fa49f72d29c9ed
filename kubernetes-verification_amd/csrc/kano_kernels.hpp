// kano_kernels.hpp -- HIP kernels of the Kano engine for gfx950.
// Host orchestration and the C ABI: kano_hip.hip.  Design: DESIGN.md.
//
// Reference semantics (qiyueyao/Kubernetes-verification, kano_py/kano/):
//   selector predicate         model.py:95-111 + 142-147
//   matrix rows                model.py:158-160   M[i] |= allow_p for p in S(i)
//   column checks              algorithm.py:4-17
//   user_crosscheck            algorithm.py:27-42
//   policy_shadow              algorithm.py:58-80
#pragma once
#include "kano_prims.hpp"

namespace kano {

// ===========================================================================
// Classes: pods hashed on the values of a key set.  Pods of one class are
// indistinguishable to every predicate on those keys.
// ===========================================================================
// Both sides (row classes on the working-selector keys, column classes on
// the working-allow keys) run in the same launches: blockIdx.y = side.
struct ClsSide {
  const int32_t* keys;   // KS columns, then their bit widths (packed mode)
  int KS;
  int packed;
  int pbits;             // > 0: packed slots hold key << pbits | smallest member (no smin)
  uint32_t tmask;
  int32_t* table;
  int32_t* slot_of;
  int32_t* smin;
  int32_t* flag;
  const int32_t* cid;
  int32_t* cls;
  int32_t* rep;
  int32_t* mcnt;
  int32_t* mcur;         // rank of pod i among its class's members, [i - m0]
  const int32_t* moff;
  int32_t* mem;
  int32_t* cval;
  i64 m0, m1, U;
};
struct ClsPair {
  ClsSide s[2];
};

// ---- user_crosscheck's group keys (a counting sort of the row classes) -----
// Key of row class c: g when all its local members are in group g, G when
// they mix groups (MULTI), -1 without local members.  Small key spaces
// (G + 1 <= KEY_LDS_MAX): per-block histograms in LDS, no global atomics;
// hist is bin-major, hist[k * nb + b], so its exclusive scan (hoff) is every
// (bin, block) start.  Block b covers classes [b, b + 1) * TPB * KEY_ITEMS.
constexpr int KEY_LDS_MAX = 8192;
constexpr int KEY_ITEMS = 8;   // classes per thread
struct KeySort {
  i64 U;                 // row classes
  i64 nb;                // blocks of the sort (0: none)
  const int32_t* mcnt;
  const int32_t* gmin;
  const int32_t* gmax;
  int32_t G;
  int32_t* ckey;
  int32_t* hist;
  const int32_t* hoff;
  int32_t* order;
};

// (block-uniform: every thread of the block calls it)
// (the histogram's LDS is dynamic, (G + 1) words: a static 32 KB table kept
// the sort off the CUs a wide k_rows_w block fills -- C5's 1/8 shard: 0.32 ->
// 2.64 ms beside the write, the next build's Mc chain waiting for it)
__device__ __forceinline__ void key_hist_block(const KeySort& k, i64 b) {
  extern __shared__ int32_t h[];
  const int nk = k.G + 1;
  for (int q = threadIdx.x; q < nk; q += TPB) h[q] = 0;
  __syncthreads();
  const i64 c0 = b * TPB * KEY_ITEMS;
  for (int q = 0; q < KEY_ITEMS; ++q) {
    const i64 c = c0 + (i64)q * TPB + threadIdx.x;
    if (c >= k.U) break;
    int32_t key = -1;
    if (k.mcnt[c] > 0 && k.gmin[c] <= k.gmax[c]) key = k.gmin[c] == k.gmax[c] ? k.gmin[c] : k.G;
    k.ckey[c] = key;
    if (key >= 0) atomicAdd(&h[key], 1);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < nk; q += TPB) k.hist[(i64)q * k.nb + b] = h[q];
}

__device__ __forceinline__ void key_place_block(const KeySort& k, i64 b) {
  extern __shared__ int32_t h[];
  const int nk = k.G + 1;
  for (int q = threadIdx.x; q < nk; q += TPB) h[q] = k.hoff[(i64)q * k.nb + b];
  __syncthreads();
  const i64 c0 = b * TPB * KEY_ITEMS;
  for (int q = 0; q < KEY_ITEMS; ++q) {
    const i64 c = c0 + (i64)q * TPB + threadIdx.x;
    if (c >= k.U) break;
    const int32_t key = k.ckey[c];
    if (key >= 0) k.order[atomicAdd(&h[key], 1)] = (int32_t)c;
  }
}

// Block-level combining (the packed mode): the block's pods first meet in an
// LDS table keyed by the packed tuple, so only one thread per distinct tuple
// per block probes the global table and posts the block's smallest member to
// smin -- with few, large classes (broad selectors: C4 has ~100 row classes)
// thousands of pods otherwise send their CAS / atomicMin to the same slot.
constexpr int CLS_LDS = 512;   // LDS slots per block (2 x TPB)

// LDS table of a block's classes (int32 keys, CLS_LDS slots, -1 empty):
// the slot of c, inserting it if absent; -1 when the table is full and c is
// not in it (the caller then goes to global memory directly; once full the
// table stays full, so a later probe for c fails the same way).
__device__ __forceinline__ int lds_class_slot(int32_t* lkey, int32_t c, bool insert) {
  uint32_t h = hfin(hmix(0x2545f491u, (uint32_t)c)) & (CLS_LDS - 1);
  for (int probe = 0; probe < CLS_LDS; ++probe) {
    int32_t cur = lkey[h];
    if (cur == -1 && insert) {
      cur = atomicCAS(&lkey[h], -1, c);
      if (cur == -1) return (int)h;
    }
    if (cur == c) return (int)h;
    if (cur == -1) return -1;            // (lookup only) absent
    h = (h + 1) & (CLS_LDS - 1);
  }
  return -1;
}

// Policies per block (spb) of the select-side kernels below that combine
// their per-class atomics in LDS (k_pol_counts, k_sel_place): waves take the
// block's policies in turn.  With spb == WPB (one policy per wave) they post
// their atomics directly.  At C4 ~10,000 policies select one of ~100 classes
// each, so the per-class counters otherwise see thousands of atomics; at C3
// a class sees ~3 and the direct form is faster (more blocks).

__device__ __forceinline__ uint32_t cls_packed_slot(const u64* tab, uint32_t tmask, u64 key) {
  uint32_t s = hfin(hmix(hmix(0x9747b28cu, (uint32_t)key), (uint32_t)(key >> 32))) & tmask;
  u64* t = const_cast<u64*>(tab);
  for (;;) {
    u64 cur = t[s];   // plain read: slots only go from empty to a key
    if (cur == ~0ull) {
      const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&t[s]), ~0ull,
                                 (unsigned long long)key);
      if (prev == ~0ull) break;
      cur = prev;
    }
    if (cur == key) break;
    s = (s + 1) & tmask;
  }
  return s;
}

__global__ __launch_bounds__(TPB) void k_cls_insert(const int32_t* __restrict__ pv, i64 n,
                                                    ClsPair pr) {
  const ClsSide a = blockIdx.y ? pr.s[1] : pr.s[0];
  const i64 i = a.m0 + (i64)blockIdx.x * TPB + threadIdx.x;   // pods [m0, m1) of the side
  const bool act = i < a.m1;
  if (act) a.mcnt[i - a.m0] = 0;                   // the member counts of k_cls_assign_count
  if (a.packed) {                                  // block-uniform branch (one side per block)
    __shared__ u64 lkey[CLS_LDS];
    __shared__ int32_t lmin[CLS_LDS], lslot[CLS_LDS];
    for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
      lkey[t] = ~0ull;
      lmin[t] = INT32_MAX;
    }
    __syncthreads();
    // the key tuple as one word, (value + 3) per key (ids are >= -3)
    u64 key = 0;
    int t = -1;
    bool lead = false;
    if (act) {
      for (int k = 0; k < a.KS; ++k)
        key = (key << a.keys[a.KS + k]) | (u64)(uint32_t)(pv[(i64)a.keys[k] * n + i] + 3);
      // 256 pods in 512 slots: the probe always ends
      uint32_t h = hfin(hmix(hmix(0x2545f491u, (uint32_t)key), (uint32_t)(key >> 32))) &
                   (CLS_LDS - 1);
      for (;;) {
        const u64 prev = atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h]), ~0ull,
                                   (unsigned long long)key);
        if (prev == ~0ull) { lead = true; break; }
        if (prev == key) break;
        h = (h + 1) & (CLS_LDS - 1);
      }
      t = (int)h;
      atomicMin(&lmin[t], (int32_t)i);
    }
    __syncthreads();
    if (lead && a.pbits) {
      // one atomic per probed slot: the CAS inserts the block's class with
      // its smallest member, or returns the slot's word; a word of the same
      // key with a larger member is lowered (no return value awaited)
      unsigned long long* tb = reinterpret_cast<unsigned long long*>(a.table);
      const u64 mine = (key << a.pbits) | (u64)(uint32_t)lmin[t];
      uint32_t s = hfin(hmix(hmix(0x9747b28cu, (uint32_t)key), (uint32_t)(key >> 32))) & a.tmask;
      for (;;) {
        const u64 prev = atomicCAS(&tb[s], ~0ull, (unsigned long long)mine);
        if (prev == ~0ull) break;
        if ((prev >> a.pbits) == key) {
          if (prev > mine) atomicMin(&tb[s], (unsigned long long)mine);
          break;
        }
        s = (s + 1) & a.tmask;
      }
      lslot[t] = (int32_t)s;
    } else if (lead) {
      const uint32_t s = cls_packed_slot(reinterpret_cast<const u64*>(a.table), a.tmask, key);
      lslot[t] = (int32_t)s;
      if (lmin[t] < a.smin[s]) atomicMin(&a.smin[s], lmin[t]);
    }
    __syncthreads();
    if (act) a.slot_of[i] = lslot[t];
    return;
  }
  if (!act) return;
  uint32_t s;
  uint32_t h = 0x9747b28cu;
  for (int k = 0; k < a.KS; ++k) h = hmix(h, (uint32_t)pv[(i64)a.keys[k] * n + i]);
  s = hfin(h) & a.tmask;
  // linear probing; the table has >= 2n slots, so this ends.  Slots only
  // go from -1 to a pod id, so a plain (possibly stale) read is safe: a stale
  // -1 just sends us to the CAS, which returns the real occupant.
  for (;;) {
    int32_t cur = a.table[s];
    if (cur < 0) {
      const int32_t prev = atomicCAS(&a.table[s], -1, (int32_t)i);
      if (prev < 0) break;
      cur = prev;
    }
    bool eq = true;
    for (int k = 0; k < a.KS; ++k) {
      const int32_t* col = pv + (i64)a.keys[k] * n;
      if (col[cur] != col[i]) { eq = false; break; }
    }
    if (eq) break;
    s = (s + 1) & a.tmask;
  }
  a.slot_of[i] = (int32_t)s;
  // smallest member per slot (the class representative); smin only falls.
  // Pods rise with the lane, so among the lanes of a wave that share a slot
  // the lowest holds the smallest pod: only it needs the atomic (popular
  // classes otherwise send every member's atomic to one address).
  const int lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1ull;
  bool first = true;
  u64 pend = __ballot(true);   // lanes that returned early (i >= m1) are off
  for (int round = 0; round < 4 && pend; ++round) {
    const int leader = __ffsll((long long)pend) - 1;
    const uint32_t sl = __shfl(s, leader, 64);
    const u64 same = __ballot(s == sl);
    if (s == sl && (same & below)) first = false;
    pend &= ~same;
  }
  if (first && (int32_t)i < a.smin[s]) atomicMin(&a.smin[s], (int32_t)i);
}



// k_cls_assign and k_cls_mcount in one pass: the class id of every pod of
// [m0, m1), the representatives, the member counts
// ipt pods a thread (<= ASSIGN_IPT): with few classes (C4: ~100 row and
// ~160 column classes) the per-block reservations still put ~300 global
// atomics on each class counter; ipt blocks' worth of pods per block cut them
// ipt-fold.  A pod whose class finds the LDS table full takes its place with a
// global atomic of its own (the table then never needs to hold every class).
constexpr int ASSIGN_IPT = 8;
__global__ __launch_bounds__(TPB) void k_cls_assign_count(ClsPair pr, int ipt) {
  const ClsSide a = blockIdx.y ? pr.s[1] : pr.s[0];
  // the block's pods are counted per class in LDS; one atomic per distinct
  // class per block reserves the block's places in the class's member list
  // (the counter's old value + the pod's LDS rank is its place: k_cls_mfill
  // then scatters without atomics)
  __shared__ int32_t lkey[CLS_LDS], lcnt[CLS_LDS], lbase[CLS_LDS];
  for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
    lkey[t] = -1;
    lcnt[t] = 0;
  }
  __syncthreads();
  int32_t cs[ASSIGN_IPT], ts[ASSIGN_IPT], rs[ASSIGN_IPT];
  bool lead[ASSIGN_IPT];
  const i64 i0 = a.m0 + (i64)blockIdx.x * TPB * ipt + threadIdx.x;
#pragma unroll
  for (int k = 0; k < ASSIGN_IPT; ++k) {
    ts[k] = -2;                                     // -2: no pod
    lead[k] = false;
    const i64 i = i0 + (i64)k * TPB;
    if (k >= ipt || i >= a.m1) continue;
    const int32_t sl = a.slot_of[i];
    const int32_t rp = a.pbits ? (int32_t)(reinterpret_cast<const u64*>(a.table)[sl] &
                                           ((1ull << a.pbits) - 1ull))
                               : a.smin[sl];
    const int32_t c = a.cid[rp - a.m0];
    cs[k] = c;
    a.cls[i] = c;
    if (rp == (int32_t)i) a.rep[c] = (int32_t)i;
    uint32_t h = hfin(hmix(0x2545f491u, (uint32_t)c)) & (CLS_LDS - 1);
    int t = -1;
    for (int probe = 0; probe < CLS_LDS; ++probe) {
      const int32_t prev = atomicCAS(&lkey[h], -1, c);
      if (prev == -1) { lead[k] = true; t = (int)h; break; }
      if (prev == c) { t = (int)h; break; }
      h = (h + 1) & (CLS_LDS - 1);
    }
    ts[k] = t;
    if (t >= 0) rs[k] = atomicAdd(&lcnt[t], 1);
    else a.mcur[i - a.m0] = atomicAdd(&a.mcnt[c], 1);   // (the table is full)
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ASSIGN_IPT; ++k)
    if (lead[k]) lbase[ts[k]] = atomicAdd(&a.mcnt[cs[k]], lcnt[ts[k]]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ASSIGN_IPT; ++k)
    if (ts[k] >= 0) a.mcur[i0 + (i64)k * TPB - a.m0] = lbase[ts[k]] + rs[k];
}


// member lists: pod i at its rank (from k_cls_assign_count) in its class.
// With gid (kano_verify's crosscheck), the row side also folds the group
// range of every row class (gmin / gmax: k_cls_group_range's work, one
// launch fewer); a group id outside [0, G) sets *err.
__global__ __launch_bounds__(TPB) void k_cls_mfill(ClsPair pr, const int32_t* __restrict__ gid,
                                                   int32_t G, int32_t* gmin, int32_t* gmax,
                                                   int32_t* err) {
  const ClsSide a = blockIdx.y ? pr.s[1] : pr.s[0];
  const i64 i = a.m0 + (i64)blockIdx.x * TPB + threadIdx.x;
  const bool act = i < a.m1;
  const int32_t c = act ? a.cls[i] : 0;
  if (act) a.mem[a.moff[c] + a.mcur[i - a.m0]] = (int32_t)i;
  if (blockIdx.y == 0 && gid) {                    // block-uniform
    // the block's ranges meet in LDS first, then one check-before-atomic per
    // distinct class: few, large classes (C4: ~100 for 100k pods) otherwise
    // serialise every pod's atomics on a handful of addresses
    __shared__ int32_t lk[CLS_LDS], lmn[CLS_LDS], lmx[CLS_LDS];
    for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
      lk[t] = -1;
      lmn[t] = INT32_MAX;
      lmx[t] = INT32_MIN;
    }
    __syncthreads();
    const int32_t g = act ? gid[i] : 0;
    if (act && (g < 0 || g >= G)) {                // caller-declared group count violated
      atomicOr(err, 1);
    } else if (act) {
      const int t = lds_class_slot(lk, c, true);   // TPB pods in 2 x TPB slots: always found
      atomicMin(&lmn[t], g);
      atomicMax(&lmx[t], g);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
      const int32_t k = lk[t];
      if (k < 0) continue;
      if (lmn[t] < gmin[k]) atomicMin(&gmin[k], lmn[t]);   // (a stale read only costs an atomic)
      if (lmx[t] > gmax[k]) atomicMax(&gmax[k], lmx[t]);
    }
  }
}

// key values of each class's representative, slot-major: cval[k * U + c]
// (blocks x >= nbv carry the fills fj: row y = 0 only)
__global__ __launch_bounds__(TPB) void k_cls_vals(const int32_t* __restrict__ pv, i64 n,
                                                  ClsPair pr, FillJobs fj, unsigned nbv) {
  if (blockIdx.x >= nbv) {                         // block-uniform
    if (blockIdx.y == 0) fill_item(fj, blockIdx.x - nbv, gridDim.x - nbv);
    return;
  }
  const ClsSide a = blockIdx.y ? pr.s[1] : pr.s[0];
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c < a.U) {
    const int32_t r = a.rep[c];
    for (int k = 0; k < a.KS; ++k) a.cval[(i64)k * a.U + c] = pv[(i64)a.keys[k] * n + r];
  }
}

// matchExpressions columns (kano/model.py
// LabelExpression): out[e * n + i] = 1 when pod i meets requirement e, else 0.
// v = the pod's value id in the key's column (-1: absent, also when no pod
// carries the key: col < 0), set = sorted value ids.  In: v listed; NotIn:
// absent or not listed; Exists: present; DoesNotExist: absent.
__global__ __launch_bounds__(TPB) void k_expr_cols(const int32_t* __restrict__ pv, i64 n,
                                                   const int32_t* __restrict__ ecol,
                                                   const int32_t* __restrict__ eop,
                                                   const i64* __restrict__ eoff,
                                                   const int32_t* __restrict__ eval,
                                                   int32_t* __restrict__ out) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  const i64 e = blockIdx.y;
  if (i >= n) return;
  const int32_t c = ecol[e];
  const int32_t v = c >= 0 ? pv[(i64)c * n + i] : -1;
  bool listed = false;
  if (v >= 0) {
    i64 lo = eoff[e], hi = eoff[e + 1];
    while (lo < hi) {
      const i64 mid = (lo + hi) >> 1;
      if (eval[mid] < v) lo = mid + 1; else hi = mid;
    }
    listed = lo < eoff[e + 1] && eval[lo] == v;
  }
  const int op = eop[e];
  const bool present = v != -1;
  const bool m = op == 0 ? listed : op == 1 ? !listed : op == 2 ? present : !present;
  out[e * n + i] = m ? 1 : 0;
}

// ===========================================================================
// Predicate evaluation on classes.
//   match(p, c) = AND over terms (slot, v): cval[slot][c] == v
// One thread per class, 64 policies per grid row.  Emits the class-major
// word outT[pb][c] (bit q = policy 64*pb+q) and/or, through a ballot per
// policy, the policy-major word outP[p][c/64] (bit c%64).
// ===========================================================================
__global__ __launch_bounds__(TPB) void k_class_eval(const int32_t* __restrict__ cval, i64 U, i64 P,
                                                    const i64* __restrict__ off,
                                                    const int32_t* __restrict__ slot,
                                                    const int32_t* __restrict__ val,
                                                    u64* __restrict__ outT,
                                                    u64* __restrict__ outP, i64 ldP) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  const i64 pb = blockIdx.y;
  const i64 p0 = pb * 64;
  const int qn = (int)min((i64)64, P - p0);
  const bool live = c < U;
  const bool lane0 = (threadIdx.x & 63) == 0;
  const i64 cw = c >> 6;
  u64 word = 0;
  for (int q = 0; q < qn; ++q) {
    const i64 p = p0 + q;
    const i64 t0 = off[p], t1 = off[p + 1];
    bool ok = live;
    for (i64 t = t0; t < t1 && ok; ++t) ok = cval[(i64)slot[t] * U + c] == val[t];
    word |= (u64)ok << q;
    if (outP) {
      const u64 b = __ballot(ok);
      if (lane0 && cw * 64 < U) outP[p * ldP + cw] = b;
    }
  }
  if (live && outT) outT[pb * U + c] = word;
}

// ===========================================================================
// Allow side: policy -> allowed column classes -> allowed pods
// ===========================================================================
// block per policy: nca[p] = #allowed classes, acnt[p] = #allowed pods
__global__ __launch_bounds__(TPB) void k_pol_count(const u64* __restrict__ AC, i64 ldC, i64 UW,
                                                   const int32_t* __restrict__ cmoff,
                                                   int32_t* __restrict__ nca,
                                                   int32_t* __restrict__ acnt) {
  __shared__ i64 sm[4];
  const i64 p = blockIdx.x;
  i64 nc = 0, np = 0;
  for (i64 w = threadIdx.x; w < UW; w += TPB) {
    u64 v = AC[p * ldC + w];
    nc += __popcll(v);
    if (cmoff) {
      while (v) {
        const i64 ca = w * 64 + __builtin_ctzll(v);
        np += cmoff[ca + 1] - cmoff[ca];
        v &= v - 1;
      }
    }
  }
  nc = block_sum(nc, sm);
  np = block_sum(np, sm);
  if (threadIdx.x == 0) {
    nca[p] = (int32_t)nc;
    acnt[p] = (int32_t)(cmoff ? np : nc);
  }
}

// block per policy: ascending list of allowed classes
__global__ __launch_bounds__(TPB) void k_pol_classes(const u64* __restrict__ AC, i64 ldC, i64 UW,
                                                     const i64* __restrict__ alcoff,
                                                     int32_t* __restrict__ alc) {
  __shared__ int sm[4];
  const i64 p = blockIdx.x;
  i64 base = alcoff[p];
  for (i64 w0 = 0; w0 < UW; w0 += TPB) {
    const i64 w = w0 + threadIdx.x;
    u64 v = (w < UW) ? AC[p * ldC + w] : 0ull;
    int tot;
    i64 pos = base + block_excl_scan((int)__popcll(v), sm, tot);
    while (v) {
      alc[pos++] = (int32_t)(w * 64 + __builtin_ctzll(v));
      v &= v - 1;
    }
    base += tot;
  }
}

// block per policy: the allowed pods (members of the allowed classes)
// Per-policy kernels below run one wave per policy (WPB policies per block):
// most policies match a handful of classes, so a block per policy leaves
// most of its lanes idle and quadruples the waves to schedule.
constexpr int WPB = TPB / 64;
__device__ __forceinline__ i64 wave_policy() {
  return (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
}

// allowed pods of policy p: members of its allowed column classes, streamed
// 64 classes at a time as one flat range (no per-class round trips)
struct PolPodsArgs {
  i64 P;
  const i64* alcoff;
  const int32_t* alc;
  const int32_t* cmoff;
  const int32_t* cmem;
  const i64* aloff;
  int32_t* alist;
};
// (vb: the block index within this job, so that a launch can carry other
// jobs' blocks too -- k_pods_scatter; no block barrier)
__device__ __forceinline__ void pol_pods_item(const PolPodsArgs& a, i64 vb) {
  const i64 P = a.P;
  const i64* __restrict__ alcoff = a.alcoff;
  const int32_t* __restrict__ alc = a.alc;
  const int32_t* __restrict__ cmoff = a.cmoff;
  const int32_t* __restrict__ cmem = a.cmem;
  const i64* __restrict__ aloff = a.aloff;
  int32_t* __restrict__ alist = a.alist;
  __shared__ int32_t seg_m0[WPB][64];
  __shared__ int32_t seg_pre[WPB][65];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const i64 p = vb * WPB + wid;
  if (p >= P) return;                      // wave-uniform
  i64 out = aloff[p];
  const i64 e1 = alcoff[p + 1];
  for (i64 e0 = alcoff[p]; e0 < e1; e0 += 64) {
    const int ns = (int)min((i64)64, e1 - e0);
    int32_t m0 = 0, len = 0;
    if (lane < ns) {
      const int32_t ca = alc[e0 + lane];
      m0 = cmoff[ca];
      len = cmoff[ca + 1] - m0;
    }
    int32_t tot;
    const int32_t pre = wave_excl_scan(len, tot);
    seg_m0[wid][lane] = m0;
    seg_pre[wid][lane] = pre;
    if (lane == 0) seg_pre[wid][ns] = tot;
    __builtin_amdgcn_wave_barrier();
    for (int32_t id = lane; id < tot; id += 64) {
      int lo = 0, hi = ns - 1;               // last segment with prefix <= id
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seg_pre[wid][mid] <= id) lo = mid; else hi = mid - 1;
      }
      alist[out + id] = cmem[seg_m0[wid][lo] + (id - seg_pre[wid][lo])];
    }
    out += tot;
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(TPB) void k_pol_pods(PolPodsArgs a) { pol_pods_item(a, blockIdx.x); }

// ===========================================================================
// Policy -> class matching by hash join.  The terms of a policy fix the values
// of a set of class-key slots (its "mask"); a class matches iff its
// projection onto the mask equals the policy's values.  Classes are grouped
// by projection, one open-addressing table per distinct mask; a policy
// probes its mask's table once and gets its whole class list (a group).
// O(P + U * masks) instead of the O(P * U) predicate evaluation.
// ===========================================================================
__device__ __forceinline__ uint32_t proj_hash(const int32_t* __restrict__ cval, i64 U, i64 c,
                                              const int32_t* __restrict__ slots, int ns) {
  uint32_t h = 0x2545f491u;
  for (int k = 0; k < ns; ++k) h = hmix(h, (uint32_t)cval[(i64)slots[k] * U + c]);
  return hfin(h);
}

// Both sides in one launch: grid.y enumerates (side 0 rows, side 1 rows); a
// side contributes NM mask rows (+1 iota row in k_join_fill) when live.
struct JoinSide {
  const int32_t* cval;
  i64 U;
  const int32_t* moff;   // mask -> slot list
  const int32_t* mslot;
  int32_t* table;        // NM tables of T slots
  i64 T;
  int32_t* pslot;        // [m * U + c] = group slot of class c under mask m
  int32_t* gcnt;
  const int32_t* goff;
  int32_t* gcur;         // [m * U + c] = rank of class c in its group (k_join_insert)
  int32_t* gmem;         // NM * U grouped classes, then the iota block
  const i64* toff;       // policy terms (sorted by slot)
  const int32_t* tval;
  const int32_t* pmask;
  i64* pstart;
  int32_t* plen;
  int NM;
  int live;
  // pmask -3 (a policy naming every class key of a packed side): its one
  // class comes straight from the classification's table -- the side's
  // packed-key table, representatives and class ids
  const u64* ctab;
  uint32_t ctmask;
  const int32_t* csmin;
  int cpb;               // the classification's pod bits (ClsSide::pbits)
  const int32_t* ccid;
  i64 cm0;
  const int32_t* kbits;   // bits per key (keys_d + KS)
  int KS;
};
struct JoinPair {
  JoinSide s[2];
};

__device__ __forceinline__ int join_row(const JoinPair& pr, int y, int extra, int* m) {
  const int r0 = pr.s[0].live ? pr.s[0].NM + extra : 0;
  if (y < r0) { *m = y; return 0; }
  *m = y - r0;
  return 1;
}

// group id of class c under mask m = its table slot
// group id of class c under mask m = its table slot; the group sizes are
// counted in the same pass (k_join_count folded in)
__global__ __launch_bounds__(TPB) void k_join_insert(JoinPair pr) {
  int m;
  const JoinSide a = join_row(pr, blockIdx.y, 0, &m) ? pr.s[1] : pr.s[0];
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  const bool act = c < a.U;
  uint32_t s = 0;
  if (act) {
    const int32_t* sl = a.mslot + a.moff[m];
    const int ns = a.moff[m + 1] - a.moff[m];
    int32_t* tab = a.table + (i64)m * a.T;
    const uint32_t tm = (uint32_t)(a.T - 1);
    s = proj_hash(a.cval, a.U, c, sl, ns) & tm;
    for (;;) {
      int32_t cur = tab[s];   // plain read: see k_cls_insert
      if (cur < 0) {
        const int32_t prev = atomicCAS(&tab[s], -1, (int32_t)c);
        if (prev < 0) break;
        cur = prev;
      }
      bool eq = true;
      for (int k = 0; k < ns; ++k) {
        const int32_t* col = a.cval + (i64)sl[k] * a.U;
        if (col[cur] != col[c]) { eq = false; break; }
      }
      if (eq) break;
      s = (s + 1) & tm;
    }
    a.pslot[(i64)m * a.U + c] = (int32_t)s;
  }
  const int32_t r = wave_agg_inc(a.gcnt, act ? (i64)m * a.T + s : 0, act);
  if (act) a.gcur[(i64)m * a.U + c] = r;   // place in the group (k_join_fill scatters)
}


// grouped class lists; the extra row per side writes the iota block (the
// class list of policies without terms)
__device__ __forceinline__ void join_fill_item(const JoinPair& pr, int y, i64 bx) {
  int m;
  const JoinSide a = join_row(pr, y, 1, &m) ? pr.s[1] : pr.s[0];
  const i64 c = bx * TPB + threadIdx.x;
  if (m == a.NM) {
    if (c < a.U) a.gmem[(i64)a.NM * a.U + c] = (int32_t)c;
    return;
  }
  if (c >= a.U) return;
  const i64 g = (i64)m * a.T + a.pslot[(i64)m * a.U + c];
  a.gmem[a.goff[g] + a.gcur[(i64)m * a.U + c]] = (int32_t)c;
}

// thread per policy: its matched classes = gmem[pstart, pstart + plen)
//   pmask -1: contradictory terms (matches nothing); -3: every class key
//   (one class, from the classification's table); -2: no terms (all
//   classes: the iota block); terms sorted by slot = mask order
__device__ __forceinline__ void join_match_item(i64 P, const JoinPair& pr, int side, i64 bx) {
  const JoinSide a = side ? pr.s[1] : pr.s[0];
  const i64 p = bx * TPB + threadIdx.x;
  if (!a.live || p >= P) return;
  const int m = a.pmask[p];
  i64 st = 0;
  int32_t len = 0;
  if (m == -3) {
    // every class key named: the class whose packed key equals the terms'
    // (k_cls_insert's packing and hash), if a pod of this side has it
    const i64 t0 = a.toff[p];
    bool possible = true;
    u64 key = 0;
    for (int k = 0; k < a.KS; ++k) {
      const int32_t v = a.tval[t0 + k];
      possible = possible && v >= 0;
      key = (key << a.kbits[k]) | (u64)(uint32_t)(v + 3);
    }
    if (possible && a.U > 0) {
      uint32_t s = hfin(hmix(hmix(0x9747b28cu, (uint32_t)key), (uint32_t)(key >> 32))) & a.ctmask;
      for (;;) {
        const u64 cur = a.ctab[s];
        if (cur == ~0ull) break;
        if ((a.cpb ? cur >> a.cpb : cur) == key) {
          const int32_t r = a.cpb ? (int32_t)(cur & ((1ull << a.cpb) - 1ull)) : a.csmin[s];
          st = (i64)a.NM * a.U + a.ccid[r - a.cm0];   // (the iota block)
          len = 1;
          break;
        }
        s = (s + 1) & a.ctmask;
      }
    }
  } else if (m == -2) {
    st = (i64)a.NM * a.U;
    len = (int32_t)a.U;
  } else if (m >= 0) {
    const i64 t0 = a.toff[p];
    const int32_t* sl = a.mslot + a.moff[m];
    const int ns = a.moff[m + 1] - a.moff[m];
    bool possible = true;
    uint32_t h = 0x2545f491u;
    for (int k = 0; k < ns; ++k) {
      const int32_t v = a.tval[t0 + k];
      possible = possible && v >= 0;
      h = hmix(h, (uint32_t)v);
    }
    if (possible && a.U > 0) {
      const int32_t* tab = a.table + (i64)m * a.T;
      const uint32_t tm = (uint32_t)(a.T - 1);
      uint32_t s = hfin(h) & tm;
      for (;;) {
        const int32_t cur = tab[s];
        if (cur < 0) break;
        bool eq = true;
        for (int k = 0; k < ns; ++k)
          if (a.cval[(i64)sl[k] * a.U + cur] != a.tval[t0 + k]) { eq = false; break; }
        if (eq) {
          const i64 g = (i64)m * a.T + s;
          st = a.goff[g];
          len = a.goff[g + 1] - a.goff[g];
          break;
        }
        s = (s + 1) & tm;
      }
    }
  }
  a.pstart[p] = st;
  a.plen[p] = len;
}

// k_join_fill and k_join_match in one launch (both need only the group
// offsets): grid rows [0, rows_f) fill, the next two match (side 0, 1)
__global__ __launch_bounds__(TPB) void k_join_fill_match(i64 P, JoinPair pr, int rows_f,
                                                         unsigned nbf, unsigned nbm) {
  const int y = blockIdx.y;
  if (y < rows_f) {
    if (blockIdx.x < nbf) join_fill_item(pr, y, blockIdx.x);
  } else if (blockIdx.x < nbm) {
    join_match_item(P, pr, y - rows_f, blockIdx.x);
  }
}

// dense fallback (too many distinct masks): per-policy class lists from the
// policy-major bits of k_class_eval
__global__ __launch_bounds__(TPB) void k_bits_to_lists(const u64* __restrict__ bits, i64 ld,
                                                       i64 UW, const i64* __restrict__ off,
                                                       int32_t* __restrict__ lst) {
  __shared__ int sm[4];
  const i64 p = blockIdx.x;
  i64 base = off[p];
  for (i64 w0 = 0; w0 < UW; w0 += TPB) {
    const i64 w = w0 + threadIdx.x;
    u64 v = (w < UW) ? bits[p * ld + w] : 0ull;
    int tot;
    i64 pos = base + block_excl_scan((int)__popcll(v), sm, tot);
    while (v) {
      lst[pos++] = (int32_t)(w * 64 + __builtin_ctzll(v));
      v &= v - 1;
    }
    base += tot;
  }
}

__global__ __launch_bounds__(TPB) void k_popc_rows(const u64* __restrict__ bits, i64 ld, i64 UW,
                                                   int32_t* __restrict__ cnt) {
  __shared__ int sm[4];
  const i64 p = blockIdx.x;
  int s = 0;
  for (i64 w = threadIdx.x; w < UW; w += TPB) s += __popcll(bits[p * ld + w]);
  s = block_sum(s, sm);
  if (threadIdx.x == 0) cnt[p] = s;
}

__global__ __launch_bounds__(TPB) void k_offsets_to_start(const i64* __restrict__ off, i64 P,
                                                          i64* __restrict__ pstart) {
  const i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
  if (p < P) pstart[p] = off[p];
}


// S(c) placement (model.py:161 appends p to select_policies): the block's
// entries are counted per class in LDS, one atomic per distinct class per
// block reserves their places, then the entries are walked again and placed
// with LDS cursors (order inside S(c) is fixed by the sort that follows).
// (blocks >= nbs carry the fills fj)
__global__ __launch_bounds__(TPB) void k_sel_place(i64 P, const i64* __restrict__ pstart,
                                                   const int32_t* __restrict__ plen,
                                                   const int32_t* __restrict__ pcls,
                                                   const i64* __restrict__ soffc, int32_t* scur,
                                                   int32_t* __restrict__ slist,
                                                   int32_t* __restrict__ ecls, int spb,
                                                   FillJobs fj, unsigned nbs, i64 cap) {
  // cap: the entries slist / ecls hold -- launched before the host knows
  // their total (the previous build's capacity), an entry past it is dropped
  // and the host, seeing the total, places again into a larger list
  if (blockIdx.x >= nbs) {                         // block-uniform
    fill_item(fj, blockIdx.x - nbs, gridDim.x - nbs);
    return;
  }
  __shared__ int32_t lkey[CLS_LDS], lcnt[CLS_LDS], lbase[CLS_LDS];
  const bool comb = spb > WPB;                        // block-uniform
  if (comb) {
    for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
      lkey[t] = -1;
      lcnt[t] = 0;
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // one policy per wave (q), or per lane when spb == TPB (short lists)
  const bool lp = spb == TPB;
  const int q0 = lp ? threadIdx.x : wv, qs = lp ? TPB : TPB / 64;
  const int k0 = lp ? 0 : lane, ks = lp ? 1 : 64;
  for (int q = q0; q < spb; q += qs) {                // pass 1: count, or place directly
    const i64 p = (i64)blockIdx.x * spb + q;
    if (p >= P) break;
    const int32_t* L = pcls + pstart[p];
    const int32_t len = plen[p];
    for (int32_t k = k0; k < len; k += ks) {
      const int32_t c = L[k];
      const int t = comb ? lds_class_slot(lkey, c, true) : -1;
      if (t >= 0) {
        atomicAdd(&lcnt[t], 1);
      } else {
        const i64 e = soffc[c] + atomicAdd(&scur[c], 1);
        if (e < cap) {
          slist[e] = (int32_t)p;
          ecls[e] = c;
        }
      }
    }
  }
  if (!comb) return;
  __syncthreads();
  for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
    const int32_t c = lkey[t];
    if (c >= 0) {
      lbase[t] = atomicAdd(&scur[c], lcnt[t]);
      lcnt[t] = 0;
    }
  }
  __syncthreads();
  for (int q = q0; q < spb; q += qs) {                // pass 2: the counted entries
    const i64 p = (i64)blockIdx.x * spb + q;
    if (p >= P) break;
    const int32_t* L = pcls + pstart[p];
    const int32_t len = plen[p];
    for (int32_t k = k0; k < len; k += ks) {
      const int32_t c = L[k];
      const int t = lds_class_slot(lkey, c, false);
      if (t < 0) continue;                            // placed in pass 1
      const i64 e = soffc[c] + lbase[t] + atomicAdd(&lcnt[t], 1);
      if (e < cap) {
        slist[e] = (int32_t)p;
        ecls[e] = c;
      }
    }
  }
}

// sort S(c) ascending (the reference appends p in policy order,
// model.py:161); entries are distinct.  One wave per class with s <= 64: a
// rank sort in registers; larger lists are left to k_sort_lists_big (block
// bitmap over all policies).
constexpr int SORT_WAVE_MAX = 64;
constexpr int SORT_LDS_WW = 768;   // bitmap words per wave (WPB x 6 KB)

// One wave per class, three jobs in one launch: the class's entry in the
// heavy list, its k_rows work items' owner map (k_flag_list), and S(c)
// sorted ascending (with sort != 0): a rank sort in registers for s <= 64,
// else the wave's own LDS bitmap over windows of sort_ww words of policy ids
// (dynamic LDS: WPB x sort_ww words, passed only when some list is longer
// than 64).  One window covers all P policies up to 49k policies; past that
// (C5: 100k) the windows write the sorted list to stmp, copied back at the
// end -- the block's LDS stays within 24 KB, so the lists run beside a wide
// k_rows_w block (125 KB) on the same CU.
struct ClassListsArgs {
  const i64* soffc;
  i64 U, P;
  int32_t* slist;
  int sort;
  const int32_t* hflag;
  const int32_t* hoff;
  int32_t* hlist;
  const int32_t* wioff;
  int32_t* wicls;
  i64 sort_ww;           // bitmap words per wave (window)
  int32_t* stmp;         // nnz_sel entries (windows past the first)
};
__device__ __forceinline__ void class_lists_item(const ClassListsArgs& a, i64 vb) {
  const i64* __restrict__ soffc = a.soffc;
  const i64 U = a.U, P = a.P;
  int32_t* __restrict__ slist = a.slist;
  const int sort = a.sort;
  const int32_t* __restrict__ hflag = a.hflag;
  const int32_t* __restrict__ hoff = a.hoff;
  int32_t* __restrict__ hlist = a.hlist;
  const int32_t* __restrict__ wioff = a.wioff;
  int32_t* __restrict__ wicls = a.wicls;
  extern __shared__ __attribute__((aligned(16))) u64 lds_bm[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const i64 c = vb * (TPB / 64) + wid;
  if (c >= U) return;                       // wave-uniform; waves never meet at a barrier
  if (lane == 0 && hflag[c]) hlist[hoff[c]] = (int32_t)c;
  for (int32_t w = wioff[c] + lane; w < wioff[c + 1]; w += 64) wicls[w] = (int32_t)c;
  if (!sort) return;
  const i64 s0 = soffc[c], s = soffc[c + 1] - s0;
  if (s <= 1) return;
  int32_t* L = slist + s0;
  if (s <= SORT_WAVE_MAX) {
    const int32_t v = lane < s ? L[lane] : 0x7fffffff;
    int r = 0;
    for (int k = 0; k < s; ++k) r += __shfl(v, k, 64) < v;
    if (lane < s) L[r] = v;
    return;
  }
  const i64 PW = (P + 63) / 64, WW = a.sort_ww;
  u64* bm = lds_bm + (i64)wid * WW;
  const bool multi = PW > WW;       // (the first window's writes would clobber L)
  int32_t* out = multi ? a.stmp + s0 : L;
  i64 base = 0;
  for (i64 v0 = 0; v0 < PW; v0 += WW) {
    const i64 nwin = min(WW, PW - v0);
    for (i64 w = lane; w < nwin; w += 64) bm[w] = 0ull;
    __builtin_amdgcn_wave_barrier();
    for (i64 k = lane; k < s; k += 64) {
      const int32_t v = L[k];
      const i64 vw = (i64)(v >> 6) - v0;
      if (vw >= 0 && vw < nwin) atomicOr(&bm[vw], 1ull << (v & 63));
    }
    __builtin_amdgcn_wave_barrier();
    for (i64 w0 = 0; w0 < nwin; w0 += 64) {
      const i64 w = w0 + lane;
      u64 v = w < nwin ? bm[w] : 0ull;
      i64 tot;
      i64 pos = base + wave_excl_scan((i64)__popcll(v), tot);
      while (v) {
        out[pos++] = (int32_t)((v0 + w) * 64 + __builtin_ctzll(v));
        v &= v - 1;
      }
      base += tot;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (multi) {
    __builtin_amdgcn_s_waitcnt(0);   // the wave's scratch stores before its reads
    __builtin_amdgcn_wave_barrier();
    for (i64 k = lane; k < s; k += 64) L[k] = out[k];
  }
}

__global__ __launch_bounds__(TPB) void k_class_lists(ClassListsArgs a) {
  class_lists_item(a, blockIdx.x);
}


// ---- allow side: per policy the allowed column classes and pods -----------
// k_pol_allow_count and k_sel_count in one pass: policy p's allowed classes
// and pods (allow-side group), then its selected classes' |S(c)| and rebuild
// cost (select-side group), the pod count passed in registers
__global__ __launch_bounds__(TPB) void k_pol_counts(i64 P, const i64* __restrict__ apstart,
                                                    const int32_t* __restrict__ aplen,
                                                    const int32_t* __restrict__ apcls,
                                                    const int32_t* __restrict__ csize,
                                                    int32_t* __restrict__ nca,
                                                    int32_t* __restrict__ acnt,
                                                    const i64* __restrict__ spstart,
                                                    const int32_t* __restrict__ splen,
                                                    const int32_t* __restrict__ spcls,
                                                    int32_t* scnt, unsigned long long* cost,
                                                    int spb) {
  __shared__ int32_t lkey[CLS_LDS], lcnt[CLS_LDS];
  __shared__ unsigned long long lcost[CLS_LDS];
  const bool comb = spb > WPB;                        // block-uniform
  if (comb) {
    for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
      lkey[t] = -1;
      lcnt[t] = 0;
      lcost[t] = 0;
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (spb == TPB) {   // one policy per lane (short lists: broad selectors)
    const i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
    if (p < P) {
      const int32_t* L = apcls + apstart[p];
      const int32_t len = aplen[p];
      i64 pods = 0;
      for (int32_t k = 0; k < len; ++k) pods += csize[L[k]];
      nca[p] = len;
      acnt[p] = (int32_t)pods;
      if (spcls) {
        const int32_t* S = spcls + spstart[p];
        const int32_t slen = splen[p];
        const unsigned long long a = (unsigned long long)(int32_t)pods;
        for (int32_t k = 0; k < slen; ++k) {
          const int32_t c = S[k];
          const int t = lds_class_slot(lkey, c, true);
          if (t >= 0) {
            atomicAdd(&lcnt[t], 1);
            if (a) atomicAdd(&lcost[t], a);
          } else {
            atomicAdd(&scnt[c], 1);
            if (a) atomicAdd(&cost[c], a);
          }
        }
      }
    }
  }
  for (int q = wv; q < spb && spb != TPB; q += TPB / 64) {
    const i64 p = (i64)blockIdx.x * spb + q;
    if (p >= P) break;                               // wave-uniform
    const int32_t* L = apcls + apstart[p];
    const int32_t len = aplen[p];
    i64 pods = 0;
    for (int32_t k = lane; k < len; k += 64) pods += csize[L[k]];
    pods = wave_sum(pods);
    if (lane == 0) {
      nca[p] = len;
      acnt[p] = (int32_t)pods;
    }
    if (!spcls) continue;
    const int32_t* S = spcls + spstart[p];
    const int32_t slen = splen[p];
    const unsigned long long a = (unsigned long long)(int32_t)pods;
    for (int32_t k = lane; k < slen; k += 64) {
      const int32_t c = S[k];
      const int t = comb ? lds_class_slot(lkey, c, true) : -1;
      if (t >= 0) {
        atomicAdd(&lcnt[t], 1);
        if (a) atomicAdd(&lcost[t], a);
      } else {
        atomicAdd(&scnt[c], 1);
        if (a) atomicAdd(&cost[c], a);
      }
    }
  }
  if (!comb) return;
  __syncthreads();
  for (int t = threadIdx.x; t < CLS_LDS; t += TPB) {
    const int32_t c = lkey[t];
    if (c >= 0) {
      atomicAdd(&scnt[c], lcnt[t]);
      if (lcost[t]) atomicAdd(&cost[c], lcost[t]);
    }
  }
}


// ---- broad selectors over few row classes (D1: every class selected by
// ~2,250 of 10^4 policies, 18M select entries on 8,000 classes) as bit
// matrices instead of per-entry counters and cursors:
//   k_selrows_dx   each policy's selected classes as a bit row SC[p] (U bits,
//                  built in the wave's LDS row, stored whole), and its allowed
//                  classes' and pods' counts (nca, acnt);
//   k_ptrans       64 x 64 bit-block transposes, policy-major bit rows ->
//                  class-indexed policy words: SA[pw][c] bit q = policy
//                  64 pw + q selects c (also ACT from AC on the allow side,
//                  the GEMM's operands as they are);
//   k_cls_counts_dx |S(c)| and the rebuild cost from SA's column c;
//   k_sel_lists_dx S(c) ascending (set-bit order) at soffc[c], with ecls.
// (round 4's k_pol_counts_dx / k_sel_place_dx put the 18M entries through
// LDS class counters and cursors: 193 + 486 us at D1, plus a sort)
constexpr int DX_MAX = 8192;
constexpr int SR_UNROLL = 8;   // the same in k_selrows_dx
__global__ __launch_bounds__(TPB) void k_selrows_dx(i64 P, const i64* __restrict__ apstart,
                                                    const int32_t* __restrict__ aplen,
                                                    const int32_t* __restrict__ apcls,
                                                    const int32_t* __restrict__ csize,
                                                    int32_t* __restrict__ nca,
                                                    int32_t* __restrict__ acnt,
                                                    const i64* __restrict__ spstart,
                                                    const int32_t* __restrict__ splen,
                                                    const int32_t* __restrict__ spcls, i64 ldU,
                                                    u64* __restrict__ SC) {
  extern __shared__ __attribute__((aligned(16))) u64 dx[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 p = (i64)blockIdx.x * WPB + wv;
  if (p >= P) return;                                // wave-uniform; no block barrier
  u64* r = dx + (i64)wv * ldU;
  for (i64 w = lane; w < ldU; w += 64) r[w] = 0ull;
  const int32_t* L = apcls + apstart[p];
  const int32_t len = aplen[p];
  i64 pods = 0;
  for (int32_t k0 = lane; k0 < len; k0 += 64 * SR_UNROLL) {
    int32_t c[SR_UNROLL];
#pragma unroll
    for (int u = 0; u < SR_UNROLL; ++u) c[u] = k0 + 64 * u < len ? L[k0 + 64 * u] : -1;
#pragma unroll
    for (int u = 0; u < SR_UNROLL; ++u) pods += c[u] >= 0 ? csize[c[u]] : 0;
  }
  pods = wave_sum(pods);
  if (lane == 0) {
    nca[p] = len;
    acnt[p] = (int32_t)pods;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  const int32_t* S = spcls + spstart[p];
  const int32_t slen = splen[p];
  for (int32_t k0 = lane; k0 < slen; k0 += 64 * SR_UNROLL) {
    int32_t c[SR_UNROLL];
#pragma unroll
    for (int u = 0; u < SR_UNROLL; ++u) c[u] = k0 + 64 * u < slen ? S[k0 + 64 * u] : -1;
#pragma unroll
    for (int u = 0; u < SR_UNROLL; ++u)
      if (c[u] >= 0) atomicOr(&r[c[u] >> 6], 1ull << (c[u] & 63));
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
  for (i64 w = lane; w < ldU; w += 64) SC[p * ldU + w] = r[w];
}

// 64 x 64 bit transpose across a wave: lane r holds row r (bit c = element
// (r, c)); returns lane r's column r (bit j = element (j, r)).  Six butterfly
// stages, each swapping the off-diagonal s x s blocks between lanes r and
// r ^ s (a 64-bit shuffle and six bit operations a stage, against 64 ballots)
__device__ __forceinline__ u64 wave_transpose64(u64 x, int lane) {
  constexpr u64 MS[6] = {0x00000000ffffffffull, 0x0000ffff0000ffffull, 0x00ff00ff00ff00ffull,
                         0x0f0f0f0f0f0f0f0full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int sft = 32 >> k;
    const u64 m = MS[k];
    const u64 y = __shfl_xor(x, sft, 64);
    x = (lane & sft) ? ((x & ~m) | ((y & ~m) >> sft)) : ((x & m) | ((y & m) << sft));
  }
  return x;
}

// Y[pw][c] (c < ldY, pw < PBo) = the policy word of class c: bit q = bit c of
// X's row 64 pw + q (rows >= P and words >= ldX read as zero; rmap: row r is
// X's row rmap[r]).  One wave per 64 x 64 tile: lane r holds row 64 pw + r's
// word g, wave_transpose64 turns it.
__global__ __launch_bounds__(TPB) void k_ptrans(const u64* __restrict__ X, i64 ldX, i64 P,
                                                u64* __restrict__ Y, i64 ldY, i64 PBo,
                                                const int32_t* __restrict__ rmap) {
  const int lane = threadIdx.x & 63;
  const i64 G = (ldY + 63) / 64;
  const i64 t = (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (t >= PBo * G) return;
  const i64 pw = t / G, g = t - pw * G;
  const i64 row = pw * 64 + lane;
  const u64 x = row < P && g < ldX ? X[(rmap ? (i64)rmap[row] : row) * ldX + g] : 0ull;
  const u64 y = wave_transpose64(x, lane);
  const i64 c = g * 64 + lane;
  if (c < ldY) Y[pw * ldY + c] = y;
}

// |S(c)| and the rebuild cost sum_{p in S(c)} |allowed pods(p)|, one block
// per class over SA's column c, a policy word a thread (C4's 100 classes: a
// wave per class walked ~500 set bits a lane, 48-68 us)
__global__ __launch_bounds__(TPB) void k_cls_counts_dx(const u64* __restrict__ SA, i64 ldY,
                                                       i64 PB, i64 U,
                                                       const int32_t* __restrict__ acnt,
                                                       int32_t* __restrict__ scnt,
                                                       unsigned long long* __restrict__ cost) {
  __shared__ i64 sm[4];
  const i64 c = blockIdx.x;
  if (c >= U) return;                               // block-uniform
  i64 cnt = 0, cs = 0;
  for (i64 pw = threadIdx.x; pw < PB; pw += TPB) {
    u64 w = SA[pw * ldY + c];
    cnt += __popcll(w);
    while (w) {
      cs += acnt[pw * 64 + __builtin_ctzll(w)];
      w &= w - 1;
    }
  }
  cnt = block_sum(cnt, sm);
  cs = block_sum(cs, sm);
  if (threadIdx.x == 0) {
    scnt[c] = (int32_t)cnt;
    cost[c] = (unsigned long long)cs;
  }
}

// S(c) ascending at soffc[c] (entries past cap dropped: the early placement
// into the previous build's capacity), ecls[e] = c (nullable: only the
// scatter form of Mc reads it).  One wave per class; each 64-word chunk of
// SA's column is expanded into the wave's LDS buffer (dynamic LDS: WPB x
// SEL_DX_BUF entries) and copied out in coalesced stores.
constexpr int SEL_DX_BUF = 4096;
__global__ __launch_bounds__(TPB) void k_sel_lists_dx(const u64* __restrict__ SA, i64 ldY,
                                                      i64 PB, i64 U,
                                                      const i64* __restrict__ soffc,
                                                      int32_t* __restrict__ slist,
                                                      int32_t* __restrict__ ecls, i64 cap) {
  extern __shared__ int32_t lbuf[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const i64 c = (i64)blockIdx.x * WPB + wid;
  if (c >= U) return;                                // wave-uniform; no block barrier
  int32_t* buf = lbuf + wid * SEL_DX_BUF;
  i64 base = soffc[c];
  for (i64 pw0 = 0; pw0 < PB; pw0 += 64) {
    const i64 pw = pw0 + lane;
    u64 w = pw < PB ? SA[pw * ldY + c] : 0ull;
    int tot;
    int pos = wave_excl_scan((int)__popcll(w), tot);
    while (w) {
      buf[pos++] = (int32_t)(pw * 64 + __builtin_ctzll(w));
      w &= w - 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (int k = lane; k < tot; k += 64) {
      const i64 e = base + k;
      if (e < cap) {
        slist[e] = buf[k];
        if (ecls) ecls[e] = (int32_t)c;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    base += tot;
  }
}

// the GEMM's A over the heavy classes: A[pw][h] = SA[pw][hlist[h]] (zero
// past H), when the heavy classes are not all of them
__global__ __launch_bounds__(TPB) void k_sa_gather(const u64* __restrict__ SA, i64 ldY,
                                                   const int32_t* __restrict__ hlist, i64 H,
                                                   i64 PBo, u64* __restrict__ A, i64 ldA) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= PBo * ldA) return;
  const i64 pw = i / ldA, h = i - pw * ldA;
  A[i] = h < H ? SA[pw * ldY + hlist[h]] : 0ull;
}

// block per policy: allowed class list (alc) and its bits AC[p]
struct PolAllowArgs {
  i64 P;
  const i64* pstart;
  const int32_t* plen;
  const int32_t* pcls;
  const i64* alcoff;
  int32_t* alc;
  u64* AC;
  i64 ldC;
};

constexpr int PA_UNROLL = 8;
// (lds_row: the wave builds AC[p] in its LDS row of ldC words and stores it
// whole -- long allow lists put thousands of same-word global atomics on
// one row; the row needs ldC * 8 * WPB bytes of the launch's dynamic LDS)
__device__ __forceinline__ void pol_allow_item(const PolAllowArgs& a, i64 vb, bool lds_row) {
  const i64 p = vb * WPB + (threadIdx.x >> 6);
  if (p >= a.P) return;                          // wave-uniform; no block barrier
  const int32_t* L = a.pcls + a.pstart[p];
  const int32_t len = a.plen[p];
  int32_t* out = a.alc + a.alcoff[p];
  const int lane = threadIdx.x & 63;
  if (lds_row) {
    extern __shared__ __attribute__((aligned(16))) u64 lds_rows[];
    u64* r = lds_rows + (i64)(threadIdx.x >> 6) * a.ldC;
    for (i64 w = lane; w < a.ldC; w += 64) r[w] = 0ull;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // (PA_UNROLL list loads in flight per lane: D1's lists hold ~1,760 classes)
    for (int32_t k0 = lane; k0 < len; k0 += 64 * PA_UNROLL) {
      int32_t ca[PA_UNROLL];
#pragma unroll
      for (int u = 0; u < PA_UNROLL; ++u) ca[u] = k0 + 64 * u < len ? L[k0 + 64 * u] : -1;
#pragma unroll
      for (int u = 0; u < PA_UNROLL; ++u) {
        if (ca[u] < 0) continue;
        out[k0 + 64 * u] = ca[u];
        atomicOr(&r[ca[u] >> 6], 1ull << (ca[u] & 63));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
    for (i64 w = lane; w < a.ldC; w += 64) a.AC[p * a.ldC + w] = r[w];
    return;
  }
  for (int32_t k = lane; k < len; k += 64) {
    const int32_t ca = L[k];
    out[k] = ca;
    atomicOr(&a.AC[p * a.ldC + (ca >> 6)], 1ull << (ca & 63));
  }
}
__global__ __launch_bounds__(TPB) void k_pol_allow_fill(PolAllowArgs a, int lds_row) {
  pol_allow_item(a, blockIdx.x, lds_row != 0);
}

// k_class_lists and k_pol_allow_fill in one launch (independent; both one
// wave per item, no block barrier): blocks [0, nb1) take the class lists
// (fills riding in the launch: blocks past nb1 + nb2)
__global__ __launch_bounds__(TPB) void k_lists_allow(ClassListsArgs a, PolAllowArgs b,
                                                     unsigned nb1, unsigned nb2, FillJobs fj,
                                                     int lds_row) {
  if (blockIdx.x < nb1) class_lists_item(a, blockIdx.x);
  else if (blockIdx.x < nb1 + nb2) pol_allow_item(b, blockIdx.x - nb1, lds_row != 0);
  else fill_item(fj, blockIdx.x - nb1 - nb2, gridDim.x - nb1 - nb2);
}

// class-major policy bits for the MFMA path: out[pb][c] bit p%64 = policy p
// matches class c (ACT over column classes, selT over row classes)
__global__ __launch_bounds__(TPB) void k_classbits(const i64* __restrict__ pstart,
                                                   const int32_t* __restrict__ plen,
                                                   const int32_t* __restrict__ pcls, i64 Uc,
                                                   u64* out) {
  const i64 p = blockIdx.x;
  const int32_t* L = pcls + pstart[p];
  for (int32_t k = threadIdx.x; k < plen[p]; k += TPB)
    atomicOr(&out[(p >> 6) * Uc + L[k]], 1ull << (p & 63));
}

// ---- compressed matrix Mc[c] over column classes (row classes x col classes)
// light classes: one wave per select entry (c, p) scatters p's allowed-class
// list into row c (balanced over entries, not classes)
struct McScatterArgs {
  i64 nnz;
  const int32_t* ecls;
  const int32_t* slist;
  const i64* alcoff;
  const int32_t* alc;
  const int32_t* mcnt;
  const int32_t* hflag;
  u64* Mc;
  i64 ldMc;
};
__device__ __forceinline__ void mc_scatter_item(const McScatterArgs& a, i64 vb) {
  const i64 e = vb * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= a.nnz) return;
  const int32_t c = a.ecls[e];
  if (a.mcnt[c] == 0 || (a.hflag && a.hflag[c])) return;
  u64* row = a.Mc + (i64)c * a.ldMc;
  const int32_t p = a.slist[e];
  for (i64 k = a.alcoff[p] + lane; k < a.alcoff[p + 1]; k += 64) {
    const int32_t ca = a.alc[k];
    atomicOr(&row[ca >> 6], 1ull << (ca & 63));
  }
}
__global__ __launch_bounds__(TPB) void k_mc_scatter(McScatterArgs a) {
  mc_scatter_item(a, blockIdx.x);
}

// The light rows of Mc by their OWNER: one wave per row class ORs the
// allowed-class lists of S(c) into an LDS row (lanes over the entries of
// S(c), each walking its policy's list) and stores only the nonzero words
// (Mc is zeroed before) -- no global atomics: the select-entry scatter's
// 57,644 device-scope atomics cost 25-28 us at C3, and writing whole rows
// (k_mc_rows) stores the 58 MB of mostly-zero words.
struct McOwnArgs {
  i64 U;
  const i64* soffc;
  const int32_t* slist;
  const i64* alcoff;
  const int32_t* alc;
  const int32_t* mcnt;
  const int32_t* hflag;
  u64* Mc;
  i64 ldMc;
};
// vb: the block index within this job; NW = TPB / 64 rows of ldMc words of
// dynamic LDS (mrow) per block
__device__ __forceinline__ void mc_own_item(const McOwnArgs& a, i64 vb, u64* mrow) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 c = vb * (TPB / 64) + wv;
  if (c >= a.U) return;                               // wave-uniform; no block barrier below
  if (a.mcnt[c] == 0 || (a.hflag && a.hflag[c])) return;
  const i64 e0 = a.soffc[c], e1 = a.soffc[c + 1];
  if (e1 == e0) return;
  u64* row = mrow + (i64)wv * a.ldMc;
  for (i64 w = lane; w < a.ldMc; w += 64) row[w] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  for (i64 e = e0 + lane; e < e1; e += 64) {
    const int32_t p = a.slist[e];
    const i64 q1 = a.alcoff[p + 1];
    for (i64 q = a.alcoff[p]; q < q1; ++q) {
      const int32_t ca = a.alc[q];
      atomicOr(&row[ca >> 6], 1ull << (ca & 63));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
  u64* dst = a.Mc + c * a.ldMc;
  for (i64 w = lane; w < a.ldMc; w += 64) {
    const u64 v = row[w];
    if (v) dst[w] = v;
  }
}
__global__ __launch_bounds__(TPB) void k_mc_own(McOwnArgs a) {
  extern __shared__ __attribute__((aligned(16))) u64 mrow[];
  mc_own_item(a, blockIdx.x, mrow);
}

// k_pol_pods and k_mc_scatter in one launch (independent; one wave per
// item): blocks [0, nb1) build the flat allowed-pod lists
__global__ __launch_bounds__(TPB) void k_pods_scatter(PolPodsArgs a, McScatterArgs b,
                                                      unsigned nb1) {
  if (blockIdx.x < nb1) pol_pods_item(a, blockIdx.x);
  else mc_scatter_item(b, blockIdx.x - nb1);
}
// k_pol_pods and k_mc_own in one launch: blocks [0, nb1) build the flat
// allowed-pod lists, the rest one thread per row class
__global__ __launch_bounds__(TPB) void k_pods_own(PolPodsArgs a, McOwnArgs b, unsigned nb1) {
  extern __shared__ __attribute__((aligned(16))) u64 mrow[];
  if (blockIdx.x < nb1) pol_pods_item(a, blockIdx.x);
  else mc_own_item(b, blockIdx.x - nb1, mrow);
}


// column OR and NAND over the classes with local members, at class level
// block: 64 words x (4 waves x 32 classes)
__global__ __launch_bounds__(TPB) void k_mc_cols(const u64* __restrict__ Mc, i64 ldMc, i64 UW,
                                                 i64 Ua, i64 U, const int32_t* __restrict__ mcnt,
                                                 u64* col_or_c, u64* col_nand_c) {
  __shared__ u64 red[2][4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const i64 w = (i64)blockIdx.x * 64 + lane;
  const i64 c0 = (i64)blockIdx.y * 128 + wid * 32;
  const u64 vm = w < UW ? valid_mask(w, Ua) : 0ull;
  u64 o = 0, na = 0;
  if (w < UW) {
    for (i64 c = c0; c < min(c0 + 32, U); ++c) {
      if (mcnt[c] == 0) continue;
      const u64 v = Mc[c * ldMc + w];
      o |= v;
      na |= ~v & vm;
    }
  }
  red[0][wid][lane] = o;
  red[1][wid][lane] = na;
  __syncthreads();
  if (wid == 0 && w < UW) {
    o = red[0][0][lane] | red[0][1][lane] | red[0][2][lane] | red[0][3][lane];
    na = red[1][0][lane] | red[1][1][lane] | red[1][2][lane] | red[1][3][lane];
    if (o) atomicOr(&col_or_c[w], o);
    if (na) atomicOr(&col_nand_c[w], na);
  }
}

// pod-level column words from class-level bits: bit j = X[cla[j]]
__global__ __launch_bounds__(TPB) void k_cols_expand(const u64* __restrict__ col_or_c,
                                                     const u64* __restrict__ col_nand_c,
                                                     const int32_t* __restrict__ cla, i64 n,
                                                     i64 ldM, u64* __restrict__ color,
                                                     u64* __restrict__ colnand) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  if (((j >> 6) << 6) >= ldM * 64) return;
  bool o = false, na = false;
  if (j < n) {
    const int32_t ca = cla[j];
    o = (col_or_c[ca >> 6] >> (ca & 63)) & 1ull;
    na = (col_nand_c[ca >> 6] >> (ca & 63)) & 1ull;
  }
  const u64 bo = __ballot(o), bn = __ballot(na);
  if ((threadIdx.x & 63) == 0) {
    color[j >> 6] = bo;
    colnand[j >> 6] = bn;
  }
}



// The same ranges read along the class-grouped member list (mem, moff over
// the shard's pods): a wave's lanes hold mostly one class, so one atomic pair
// per class run instead of per-lane or per-unique-key merging.
__global__ __launch_bounds__(TPB) void k_cls_group_range_m(const int32_t* __restrict__ gid,
                                                           int32_t G,
                                                           const int32_t* __restrict__ cls,
                                                           const int32_t* __restrict__ mem,
                                                           i64 rl, int32_t* gmin, int32_t* gmax,
                                                           int32_t* err) {
  const i64 k = (i64)blockIdx.x * TPB + threadIdx.x;
  bool act = k < rl;
  const int32_t i = act ? mem[k] : 0;
  const int32_t c = act ? cls[i] : -1, g = act ? gid[i] : 0;
  if (act && (g < 0 || g >= G)) {   // caller-declared group count violated
    atomicOr(err, 1);
    act = false;
  }
  wave_seg_minmax(gmin, gmax, c, g, act);
}

// Classes keyed by their group for one pass over Mc: key = g for classes
// whose local members are all in group g, G for classes mixing groups (MULTI),
// -1 for classes without local members.  Counted per key (counting sort).
__global__ __launch_bounds__(TPB) void k_cls_key(i64 U, const int32_t* __restrict__ mcnt,
                                                 const int32_t* __restrict__ gmin,
                                                 const int32_t* __restrict__ gmax, int32_t G,
                                                 int32_t* __restrict__ ckey, int32_t* kcnt) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  int32_t key = -1;
  if (c < U && mcnt[c] > 0 && gmin[c] <= gmax[c]) key = gmin[c] == gmax[c] ? gmin[c] : G;
  if (c < U) ckey[c] = key;
  (void)wave_agg_inc(kcnt, key < 0 ? 0 : key, key >= 0);
}

__global__ __launch_bounds__(TPB) void k_cls_key_place(i64 U, const int32_t* __restrict__ ckey,
                                                       const int32_t* __restrict__ koff,
                                                       int32_t* kcur, int32_t* __restrict__ order) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  const int32_t key = c < U ? ckey[c] : -1;
  const int32_t r = wave_agg_inc(kcur, key < 0 ? 0 : key, key >= 0);
  if (key >= 0) order[koff[key] + r] = (int32_t)c;
}

// the standalone launches of the group-key sort (KeySort above): grid = nb
__global__ __launch_bounds__(TPB) void k_key_hist(KeySort k) { key_hist_block(k, blockIdx.x); }
__global__ __launch_bounds__(TPB) void k_key_place_lds(KeySort k) {
  key_place_block(k, blockIdx.x);
}

// k_key_place_lds without the scan launch before it: every block scans the
// (small, bin-major) histogram itself and keeps the exclusive offsets of its
// own (bin, block) entries; block 0 writes the total to hoff[nk * nb] (the
// live-class count k_mc_fold reads).  Used on the side stream, which has no
// scan status region of its own.
constexpr int KEY_SCAN_ITEMS = 8;
__global__ __launch_bounds__(TPB) void k_key_place_scan(KeySort k) {
  extern __shared__ int32_t h[];
  __shared__ i64 sm[TPB / 64];
  const int nk = k.G + 1;
  const i64 b = blockIdx.x, nb = k.nb, ns = (i64)nk * nb;
  i64 carry = 0;
  for (i64 t0 = 0; t0 < ns; t0 += (i64)TPB * KEY_SCAN_ITEMS) {
    const i64 e0 = t0 + (i64)threadIdx.x * KEY_SCAN_ITEMS;
    int32_t v[KEY_SCAN_ITEMS];
    i64 sum = 0;
#pragma unroll
    for (int q = 0; q < KEY_SCAN_ITEMS; ++q) {
      v[q] = e0 + q < ns ? k.hist[e0 + q] : 0;
      sum += v[q];
    }
    i64 total;
    i64 pre = carry + block_excl_scan_nw<TPB / 64>(sum, sm, total);
#pragma unroll
    for (int q = 0; q < KEY_SCAN_ITEMS; ++q) {
      const i64 e = e0 + q;
      if (e < ns && e % nb == b) h[e / nb] = (int32_t)pre;
      pre += v[q];
    }
    carry += total;
  }
  if (b == 0 && threadIdx.x == 0) const_cast<int32_t*>(k.hoff)[ns] = (int32_t)carry;
  __syncthreads();
  const i64 c0 = b * TPB * KEY_ITEMS;
  for (int q = 0; q < KEY_ITEMS; ++q) {
    const i64 c = c0 + (i64)q * TPB + threadIdx.x;
    if (c >= k.U) break;
    const int32_t key = k.ckey[c];
    if (key >= 0) k.order[atomicAdd(&h[key], 1)] = (int32_t)c;
  }
}

// One pass over Mc in group order: R[g] |= Mc[c] (g = key), MULTI for key G;
// with col_or / col_nand non-null also the column OR / NAND of
// all_reachable / all_isolated.  Block = 64 words x (4 waves x 16 sorted
// classes); runs of equal key are OR-ed in registers, one atomic per run.
constexpr int FOLD_PER_WAVE = 32;
// FOLD_PER_WAVE classes per wave, their class ids and keys in one round trip
// (lane q holds entry k0+q) and all their Mc words in flight together
__global__ __launch_bounds__(TPB) void k_mc_fold(const u64* __restrict__ Mc, i64 ldMc, i64 UW,
                                                 i64 Ua, const int32_t* __restrict__ order,
                                                 const int32_t* __restrict__ nlive_p,
                                                 const int32_t* __restrict__ ckey,
                                                 int32_t G, u64* R, u64* multi, u64* col_or,
                                                 u64* col_nand) {
  constexpr int PW = FOLD_PER_WAVE;
  __shared__ u64 red[2][TPB / 64][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const i64 w = (i64)blockIdx.x * 64 + lane;
  const i64 nlive = *nlive_p;
  const i64 k0 = ((i64)blockIdx.y * (TPB / 64) + wid) * PW;
  const i64 k1 = min(nlive, k0 + PW);
  const bool wok = w < UW;
  const u64 vm = wok ? valid_mask(w, Ua) : 0ull;
  u64 o = 0, na = 0, acc = 0;
  int32_t cur = -1;
  int32_t myc = 0, myk = 0;
  if (lane < PW && k0 + lane < k1) {
    myc = order[k0 + lane];
    myk = ckey[myc];
  }
  const int cnt = (int)max((i64)0, k1 - k0);
  u64 v[PW];
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const int32_t c = __shfl(myc, q, 64);
    v[q] = (wok && q < cnt) ? Mc[(i64)c * ldMc + w] : 0ull;
  }
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const int32_t key = __shfl(myk, q, 64);
    if (q < cnt) {
      o |= v[q];
      na |= ~v[q] & vm;
      if (key != cur) {
        if (acc) atomicOr(cur == G ? &multi[w] : &R[(i64)cur * ldMc + w], acc);
        cur = key;
        acc = 0;
      }
      acc |= v[q];
    }
  }
  if (acc) atomicOr(cur == G ? &multi[w] : &R[(i64)cur * ldMc + w], acc);
  if (col_or) {
    red[0][wid][lane] = o;
    red[1][wid][lane] = na;
    __syncthreads();
    if (wid == 0 && wok) {
      o = red[0][0][lane] | red[0][1][lane] | red[0][2][lane] | red[0][3][lane];
      na = red[1][0][lane] | red[1][1][lane] | red[1][2][lane] | red[1][3][lane];
      if (o) atomicOr(&col_or[w], o);
      if (na) atomicOr(&col_nand[w], na);
    }
  }
}


// cross[j] = MULTI(ca) | A2(ca) | (A1(ca) & ~R[g(j)](ca)),  ca = cla[j]
__global__ __launch_bounds__(TPB) void k_cross_pod(const int32_t* __restrict__ gid, int32_t G,
                                                   const int32_t* __restrict__ cla, i64 n,
                                                   const u64* __restrict__ R, i64 ldMc,
                                                   const u64* __restrict__ multi,
                                                   const u64* __restrict__ A1,
                                                   const u64* __restrict__ A2, i64 W,
                                                   u64* __restrict__ cross, int32_t* err) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  if (((j >> 6) << 6) >= W * 64) return;
  bool bit = false;
  if (j < n) {
    const int32_t ca = cla[j], g = gid[j];
    const i64 cw = ca >> 6;
    const u64 m = 1ull << (ca & 63);
    bool own = false;
    if (g < 0 || g >= G) atomicOr(err, 1);
    else own = (R[(i64)g * ldMc + cw] & m) != 0;
    bit = ((multi[cw] | A2[cw]) & m) || ((A1[cw] & m) && !own);
  }
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0) cross[j >> 6] = bal;
}

// ===========================================================================
// Select side: per row class, |S(c)|, rebuild cost, work items, heavy flag
// ===========================================================================
struct ClassPlan {
  i64 U;
  const int32_t* scnt;     // |S(c)|
  const unsigned long long* cost;  // sum over S(c) of |allow_p| (rebuild scatter work)
  const int32_t* mcnt;     // local members per class
  i64 W;                   // words per matrix row
  int ch;                  // members per work item
  int force;               // 0 cost-based, 2 heavy whenever S(c) is non-empty
  int32_t* wicnt;          // out work items of the class
  int32_t* hflag;          // out 1 = heavy (row built once from Mc, then copied)
  i64* sq;                 // out |S(c)|^2 for classes with local members
  int32_t* maxs;           // out max |S(c)| over classes with local members
  unsigned long long* light;  // out sum of cost * chunks over light classes
  unsigned long long* hsel;   // out sum of |S(c)| over heavy classes
};

// A light class rebuilds its row per member chunk by scattering its allowed
// pods (cost atomics per chunk); a heavy one expands Mc once (about 64*W lane
// operations) and every chunk copies it (W words).  Heavy iff cheaper.
__global__ __launch_bounds__(TPB) void k_class_plan(ClassPlan a) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  int32_t smax = 0;
  unsigned long long light = 0, hsel = 0;
  if (c < a.U) {
    const int32_t s = a.scnt[c];
    const int32_t m = a.mcnt[c];
    const i64 cost = (i64)a.cost[c];
    const int32_t chunks = (m + a.ch - 1) / a.ch;
    a.wicnt[c] = chunks;
    int hv = 0;
    if (m > 0 && s > 0) {
      if (a.force == 2) hv = 1;
      else hv = cost * chunks > 64 * a.W + (i64)chunks * a.W;
    }
    a.hflag[c] = hv;
    a.sq[c] = m > 0 ? (i64)s * s : 0;
    if (m > 0) smax = s;
    if (m > 0 && !hv) light = (unsigned long long)cost * (unsigned long long)chunks;
    if (hv) hsel = (unsigned long long)s;
  }
  // one atomic pair per block (per wave, the two slots took ~700 contended
  // atomics on C3)
  __shared__ unsigned long long sl[TPB / 64], sh[TPB / 64];
  __shared__ int32_t sx[TPB / 64];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) smax = max(smax, __shfl_xor(smax, d, 64));
  light = wave_sum(light);
  hsel = wave_sum(hsel);
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = light;
    sh[threadIdx.x >> 6] = hsel;
    sx[threadIdx.x >> 6] = smax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < TPB / 64; ++w) {
      light += sl[w];
      hsel += sh[w];
      smax = max(smax, sx[w]);
    }
    if (smax > 0) atomicMax(a.maxs, smax);
    if (light) atomicAdd(a.light, light);
    if (hsel) atomicAdd(a.hsel, hsel);
  }
}

__global__ __launch_bounds__(TPB) void k_sq_from_off(const i64* __restrict__ off, i64 U,
                                                     i64* __restrict__ sq) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c < U) sq[c] = (off[c + 1] - off[c]) * (off[c + 1] - off[c]);
}


// ===========================================================================
// Heavy rows: the row of the class over COLUMN classes, Mc[h] = OR_{p in S}
// AllowC[p], then expanded to pods (bit j = Mc[h][cla[j]]).
// ===========================================================================
// bitwise: block per (heavy class, chunk of <= 64 Mc words); the threads
// split the policies of S(c) as well as the words, then OR-reduce in LDS
__global__ __launch_bounds__(TPB) void k_heavy_mc_or(const int32_t* __restrict__ hlist,
                                                     const i64* __restrict__ soffc,
                                                     const int32_t* __restrict__ slist,
                                                     const u64* __restrict__ AC, i64 ldC, i64 UW,
                                                     u64* __restrict__ Mc, i64 ldMc) {
  __shared__ u64 red[TPB];
  const int32_t c = hlist[blockIdx.x];
  const i64 w0 = (i64)blockIdx.y * 64;
  const int wc = (int)min((i64)64, ldMc - w0);
  int wc2 = 1;
  while (wc2 < wc) wc2 <<= 1;
  const int npp = TPB / wc2;
  const int wl = threadIdx.x & (wc2 - 1), pp = threadIdx.x / wc2;
  const i64 w = w0 + wl;
  u64 acc = 0;
  if (wl < wc && w < UW) {
    const i64 s1 = soffc[c + 1];
    for (i64 e = soffc[c] + pp; e < s1; e += npp) acc |= AC[(i64)slist[e] * ldC + w];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = npp >> 1; st >= 1; st >>= 1) {
    if (pp < st) red[threadIdx.x] |= red[threadIdx.x + st * wc2];
    __syncthreads();
  }
  if (pp == 0 && wl < wc) Mc[(i64)c * ldMc + w] = red[threadIdx.x];
}

// MFMA contraction (the dense path):
//   C[h][ca] = sum_p Sel[h][p] * Allow[p][ca]   (0/1 operands),  bit = C > 0
// A = selT[pb][c] bits of the heavy row classes, B = ACT[pb][ca] bits of the
// column classes (class-major), both expanded in registers.  The 32x32 MFMA
// forms: lane l supplies row / column l&31 of A / B and half l>>5 of the
// K-step; accumulator reg g of lane l holds row (g&3)+8*(g>>2)+4*(l>>5),
// column l&31 (cdna_hip_programming.md §3).  Any consistent k order gives the
// same sum, so A and B share one bit -> element order.
// One wave = up to 32*HT heavy rows x 32 column classes; K = all policies.
// The block-scaled fp4 MFMA's operand from 32 bits (e2m1, unit scales): nibble
// j of register v holds bit 4 j + v of x in place -- x & 0x11.. (0.5), x &
// 0x22.. (1.0), x & 0x44.. (2.0) -- and bit 4 j + 3 (the nibble's sign bit)
// moved down one, (x >> 1) & 0x44.. (2.0): five instructions for the four
// registers.  Every element is 0 or positive, so a product sum is > 0 iff
// some k has both bits (sums of 0.25 / 1 / 4 stay exact in f32); registers
// 4..7 (the fp8 width) are unused by e2m1.
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));
constexpr int FP4_ONE_SCALE = 127;   // e8m0 2^0
__device__ __forceinline__ i32x8 bits_to_fp4(uint32_t x) {
  i32x8 r;
  r[0] = (int32_t)(x & 0x11111111u);
  r[1] = (int32_t)(x & 0x22222222u);
  r[2] = (int32_t)(x & 0x44444444u);
  r[3] = (int32_t)((x >> 1) & 0x44444444u);
  r[4] = r[5] = r[6] = r[7] = 0;
  return r;
}

// Split-K: blockIdx.y takes policy blocks [y*kchunk, (y+1)*kchunk); the
// thresholded partial contractions are OR-ed into Mc (zeroed; OR over the
// splits of "some p in the split" is exactly "some p"), so the K loop of a
// wave is short and the grid fills the chip even for a handful of column
// tiles.
template <int HT>
__global__ __launch_bounds__(TPB) void k_heavy_mc_mfma(const u64* __restrict__ selT, i64 U,
                                                       const int32_t* __restrict__ hlist, int H,
                                                       const u64* __restrict__ ACT, i64 Ua,
                                                       i64 PB, uint32_t* __restrict__ Mc32,
                                                       i64 ldMc, i64 kchunk) {
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const i64 jt = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);  // 32-column tile
  if (jt >= 2 * ldMc) return;                                        // wave-uniform
  const i64 ca = jt * 32 + l32;
  int32_t hc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    const int h = t * 32 + l32;
    hc[t] = h < H ? hlist[h] : -1;
  }
  f32x16 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[t][g] = 0.f;
  const i64 pb0 = (i64)blockIdx.y * kchunk, pb1 = min(PB, pb0 + kchunk);
  for (i64 pb = pb0; pb < pb1; ++pb) {
    // (one fp4 MFMA per 64-policy word: lane half `half` takes 32 of its bits)
    const u64 bw = ca < Ua ? ACT[pb * Ua + ca] : 0ull;
    const i32x8 bfrag = bits_to_fp4((uint32_t)(bw >> (32 * half)));
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      const u64 aw = hc[t] >= 0 ? selT[pb * U + hc[t]] : 0ull;
      const i32x8 afrag = bits_to_fp4((uint32_t)(aw >> (32 * half)));
      acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(afrag, bfrag, acc[t], 4, 4, 0,
                                                               FP4_ONE_SCALE, 0, FP4_ONE_SCALE);
    }
  }
#pragma unroll
  for (int t = 0; t < HT; ++t) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const u64 bal = __ballot(acc[t][g] > 0.f);
      // (the class of row 32 t + r from lane r's hc[t], loaded before the K loop)
      const int r = (g & 3) + 8 * (g >> 2);
      const int32_t c0 = __builtin_amdgcn_readlane(hc[t], r);
      const int32_t c1 = __builtin_amdgcn_readlane(hc[t], r + 4);
      if (lane == 0 || lane == 32) {
        const int32_t c = lane == 0 ? c0 : c1;
        const uint32_t word = lane == 0 ? (uint32_t)bal : (uint32_t)(bal >> 32);
        if (c >= 0 && word) atomicOr(&Mc32[(i64)c * ldMc * 2 + jt], word);
      }
    }
  }
}

// The GEMM's A operand, heavy rows only: A[pb][h] bit q = policy 64 pb + q
// selects heavy class hlist[h] -- one wave per heavy class sets the bits of
// its (sorted) S(c) in an LDS column of PB words, then stores the column
// (PB x H words; the k_classbits form sets U-wide columns with one global
// atomic per select entry, 2e7 of them at the dense sweep's largest point).
// LDS: PB words per wave (dynamic).
// (ldA >= H columns, PBp >= PB rows: the padding -- columns h >= H, rows
// w >= PB -- is written as zeros, the staged GEMM reads whole tiles)
__global__ __launch_bounds__(TPB) void k_heavy_selT(const int32_t* __restrict__ hlist, i64 H,
                                                    i64 ldA, const i64* __restrict__ soffc,
                                                    const int32_t* __restrict__ slist, i64 PBp,
                                                    u64* __restrict__ A) {
  extern __shared__ __attribute__((aligned(16))) u64 col[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 h = (i64)blockIdx.x * (TPB / 64) + wv;
  if (h >= ldA) return;                               // wave-uniform; no block barrier
  u64* cw = col + (i64)wv * PBp;
  for (i64 w = lane; w < PBp; w += 64) cw[w] = 0ull;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if (h < H) {
    const int32_t c = hlist[h];
    const i64 e1 = soffc[c + 1];
    for (i64 e = soffc[c] + lane; e < e1; e += 64) {
      const int32_t p = slist[e];
      atomicOr(&cw[p >> 6], 1ull << (p & 63));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
  for (i64 w = lane; w < PBp; w += 64) A[w * ldA + h] = cw[w];
}

// The dense contraction at scale (many heavy row classes, broad selectors):
// Mc[h][ca] = (sum_p Sel[h][p] Allow[p][ca] > 0) as a GEMM on 0/1 operands
// tiled like k_path_mfma -- one wave = (32 TM heavy rows) x (32 TN column
// classes), each A fragment feeding TN MFMAs and each B fragment TM; block =
// 2 x 2 waves; K = all policies, 64 per step, no split (the grid has >=
// HEAVY_GEMM_MIN_TILES wave tiles).  A is the heavy rows' select bits [pb][h]
// (k_heavy_selT), B is ACT[pb][ca].  Every (row, 32-column word) belongs to
// one wave: plain stores of the thresholded ballots into the zeroed Mc.
// Blocks of one XCD (blockIdx mod 8) walk a contiguous range of the tile
// order (GM block-rows at a time) so that they share A and B panels in their
// L2.  A block's A and B panels for KC K-steps at a time (KC x (64 TM + 64
// TN) words) are copied global -> LDS by the async 16-byte LDS-DMA loads
// (global_load_lds_dwordx4, no register staging), double-buffered: chunk c+1
// is in flight while chunk c's MFMAs run, so the loads' latency (the operands
// sit in the MALL, ~1-2 us away) hides behind the matrix work of KC K-steps
// instead of one.  The operands are padded (zero) to whole block tiles and K
// chunks (ldA = H rounded up to 64 TM, ldB = Ua rounded up to 64 TN, PB
// rounded up to GK_KC, a multiple of every KC), so no load leaves its array.
// LDS: 2 x KC x (64 TM + 64 TN) x 8 B (KC K-steps a chunk: 32 KB at 2 x 2 and
// KC = 8, the engine's form; 128 KB at 4 x 4 and KC = 16).
constexpr i64 HEAVY_GEMM_MIN_TILES = 512;
constexpr int GK_KC = 16;
// the engine's chunk depth for a wave tile: 2 x 2 stages 8 K-steps (32 KB, so
// that several blocks share a CU), the wide tiles 16
constexpr int gemm_kc(int tm, int tn) { return tm == 2 && tn == 2 ? 8 : GK_KC; }

// The MFMA is the block-scaled fp4 form (v_mfma_scale_f32_32x32x64_f8f6f4,
// e2m1 operands, unit scales): the cycles of the i8 32x32x32 form at twice
// the K, so one instruction per 64-policy word instead of two.  A 0/1 bit
// becomes a positive fp4 value or 0, so the f32 sum is > 0 iff some policy
// has both bits -- the bit an i8 contraction gives.  The expansion needs no
// spread: any K order shared by A and B gives the same sum, so a lane's 32
// bits go to its four operand registers as whole nibbles (bits_to_fp4, five
// instructions; the round-5 i8 form spread 4 bits to 4 bytes with a multiply,
// three instructions a register and twice the registers per K;
// scripts/micro/gemm_f4.hip: D1's 8,000 x 10,000 x 8,000 in 0.338 ms against
// 0.577, identical Mc).
template <int TM, int TN, int KC>
__global__ __launch_bounds__(TPB) void k_heavy_gemm_f4(const u64* __restrict__ A, i64 ldA,
                                                       const int32_t* __restrict__ hlist, i64 H,
                                                       const u64* __restrict__ B, i64 ldB,
                                                       i64 Ua, i64 PBp,
                                                       uint32_t* __restrict__ Mc32, i64 ldMc) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int STAGE = KC * (BM + BN);        // words per buffer
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wv = threadIdx.x >> 6;
  constexpr i64 GM = 8;
  const i64 nbm = (H + BM - 1) / BM, nbn = (Ua + BN - 1) / BN;
  const i64 total = nbm * nbn, per = (total + 7) / 8;
  const i64 L = (i64)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= total) return;                             // block-uniform
  const i64 grp = L / (GM * nbn), first = grp * GM;
  const i64 gm = nbm - first < GM ? nbm - first : GM;
  const i64 in = L - grp * GM * nbn;
  const i64 bm = first + in % gm, bn = in / gm;
  const i64 rb0 = bm * BM, cb0 = bn * BN;
  auto stage = [&](int buf, i64 k0) {
    u64* dst = smem + (size_t)buf * STAGE;
    constexpr int PIECES = KC * (BM + BN) / 128;
    for (int q = wv; q < PIECES; q += TPB / 64) {
      const int w0 = q * 128;
      const int kk = w0 < KC * BM ? w0 / BM : (w0 - KC * BM) / BN;
      const u64* src = w0 < KC * BM
                           ? A + (k0 + kk) * ldA + rb0 + (w0 - kk * BM)
                           : B + (k0 + kk) * ldB + cb0 + (w0 - KC * BM - kk * BN);
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(src + 2 * lane),
          (__attribute__((address_space(3))) void*)(dst + w0), 16, 0, 0);
    }
  };
  const int wr = wv >> 1, wc = wv & 1;
  // lane l32 holds the class of the wave's row 32 t + l32 (-1 past H)
  int32_t hrow[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const i64 row = rb0 + wr * 32 * TM + 32 * t + l32;
    hrow[t] = row < H ? hlist[row] : -1;
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
  const i64 nchunks = PBp / KC;
  stage(0, 0);
  for (i64 c = 0; c < nchunks; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                  // chunk c in LDS, chunk c-1 read by all
    if (c + 1 < nchunks) stage((int)((c + 1) & 1), (c + 1) * KC);
    // (a lane's 32 bits: half `half` of its row's / column's word)
    const uint32_t* As = reinterpret_cast<const uint32_t*>(smem + (size_t)(c & 1) * STAGE) +
                         2 * (wr * 32 * TM + l32) + half;
    const uint32_t* Bs = reinterpret_cast<const uint32_t*>(smem + (size_t)(c & 1) * STAGE +
                                                           KC * BM) +
                         2 * (wc * 32 * TN + l32) + half;
#pragma unroll 4
    for (int kk = 0; kk < KC; ++kk) {
      i32x8 af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = bits_to_fp4(As[2 * (kk * BM + 32 * t)]);
#pragma unroll
      for (int u = 0; u < TN; ++u) bf[u] = bits_to_fp4(Bs[2 * (kk * BN + 32 * u)]);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              af[t], bf[u], acc[t][u], 4, 4, 0, FP4_ONE_SCALE, 0, FP4_ONE_SCALE);
    }
  }
  const i64 cb = cb0 + wc * 32 * TN;
  const i64 ld32 = 2 * ldMc;
  // (the rows' classes were loaded before the K loop: a load here would put a
  // wait for every store issued so far in front of each row's ballots)
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int r = (g & 3) + 8 * (g >> 2);
      const int32_t hr0 = __builtin_amdgcn_readlane(hrow[t], r);
      const int32_t hr1 = __builtin_amdgcn_readlane(hrow[t], r + 4);
      const int32_t hr = half ? hr1 : hr0;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const u64 bal = __ballot(acc[t][u][g] > 0.f);
        const i64 c32 = (cb + 32 * u) >> 5;
        if (l32 == 0 && hr >= 0 && c32 < ld32)
          Mc32[(i64)hr * ld32 + c32] = half ? (uint32_t)(bal >> 32) : (uint32_t)bal;
      }
    }
}

// Heavy rows straight from the class-level matrix, every member row: McT
// (k_ptrans of Mc's heavy rows: McT[hw][a] bit i = heavy class 64 hw + i
// reaches column class a).  Block (64-word range, heavy word hw): lane j of
// a wave looks up pod 64 w + j's column class in McT, a wave transpose turns
// the 64 pods x 64 classes bits into the 64 classes' words of row word w, kept in
// LDS; then the first member row of each class (first_only: k_rows copies
// it to the others in whole-row stores) or every member row takes the 512-B
// segment.  (The round-4 form gathered 64 bits per output word from LDS:
// 0.63 ms at D1 before k_rows' 0.60 ms copy.)
constexpr int HXB = 64;          // row words per block
constexpr int HXS = HXB + 2;     // LDS row stride (16-B aligned rows)
__global__ __launch_bounds__(TPB) void k_heavy_rows_t(const u64* __restrict__ McT, i64 ldT,
                                                      const int32_t* __restrict__ hlist, i64 H,
                                                      const int32_t* __restrict__ cla, i64 n,
                                                      const int32_t* __restrict__ moff,
                                                      const int32_t* __restrict__ mem,
                                                      u64* __restrict__ M, i64 ldM, i64 r0,
                                                      int first_only) {
  __shared__ __attribute__((aligned(16))) u64 T[64 * HXS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const i64 hw = blockIdx.y;
  const i64 w0 = (i64)blockIdx.x * HXB;
  const int nwb = (int)min((i64)HXB, ldM - w0);     // even: ldM and HXB are
  for (int q = wid; q < nwb; q += WPB) {
    const i64 pod = (w0 + q) * 64 + lane;
    const int32_t a = pod < n ? cla[pod] : -1;
    const u64 x = a >= 0 ? McT[hw * ldT + a] : 0ull;
    T[lane * HXS + q] = wave_transpose64(x, lane);
  }
  __syncthreads();
  // a wave per class, two member rows per store instruction (32 lanes x 16 B)
  const int nh = (int)min((i64)64, H - hw * 64);
  const int half = lane >> 5, l = lane & 31;
  for (int i = wid; i < nh; i += WPB) {
    const int32_t c = hlist[hw * 64 + i];
    const int32_t mb = moff[c], me = first_only ? min(moff[c + 1], mb + 1) : moff[c + 1];
    const u64* src = T + i * HXS;
    // (members mb + z, mb + z + Z, ... : blockIdx.z of gridDim.z = Z)
    const int32_t Z = (int32_t)gridDim.z;
    for (int32_t k0 = mb + (int32_t)blockIdx.z; k0 < me; k0 += 64 * Z) {
      const int32_t idx = k0 + lane * Z;
      const int32_t mv = idx < me ? mem[idx] : -1;
      const int cnt = min(64, (me - k0 + Z - 1) / Z);
      for (int t = 0; t < cnt; t += 2) {
        const int32_t pod = __shfl(mv, t + half, 64);
        if (t + half >= cnt) continue;
        u64* dst = M + (i64)(pod - r0) * ldM + w0;
        for (int u = 2 * l; u < nwb; u += 64)
          __builtin_nontemporal_store(*(const u64x2*)&src[u], (u64x2*)&dst[u]);
      }
    }
  }
}

// ===========================================================================
// Matrix rows (model.py:158-160).  One block = one work item (class, up to
// ch member pods, column chunk of cww words).  Light classes rebuild their
// row in LDS from the allowed-pod lists of S(c) (LDS 64-bit atomic OR);
// heavy classes copy the row prebuilt at their first member.  The row is then
// streamed to every member row (16-byte stores).  The first chunk of every
// class folds the row into the column OR / NAND (all_isolated /
// all_reachable) with global atomics, skipping saturated words.
// ===========================================================================
struct RowsArgs {
  const int32_t* wioff;  // U+1
  const int32_t* wicls;  // work item -> class (nullable: binary search in wioff)
  i64 U;
  const i64* soffc;      // U+1
  const int32_t* slist;
  const i64* aloff;      // allowed-pod lists per policy (nullable: use the
  const int32_t* alist;  //   column-class member lists below instead)
  const i64* alcoff;     // allowed column classes per policy (CSR)
  const int32_t* alc;
  const int32_t* cmoff;  // members of each column class
  const int32_t* cmem;
  const int32_t* moff;   // U+1
  const int32_t* mem;
  const int32_t* hflag;  // U (nullable)
  u64* M;
  i64 ldM;
  i64 wW;                // words written per row (<= ldM)
  i64 r0;
  i64 n, W;
  int ch;
  int cww;
  int heavy_skip;        // heavy classes' rows written whole by k_heavy_rows_t
  u64* color;
  u64* colnand;
};

constexpr int ROWS_UNROLL = 4;
// segments (policies of S(c)) of the flattened walk: a fixed small table, so
// that the static LDS does not cost the wide (NT = 1024, 64 KB row) blocks
// their second slot per CU
constexpr int ROWS_SEG = 256;
// the row of light class c over columns [64*base, 64*(base + nw)) built in
// LDS from the allowed-pod lists of S(c) (zeroed first; ends in a barrier)
template <int NT>
__device__ __forceinline__ void build_light_row(const RowsArgs& a, i64 c, i64 base, int nw,
                                                u64* row) {
  constexpr int NW = NT / 64;
  for (int w = threadIdx.x; w < nw; w += NT) row[w] = 0ull;
  __syncthreads();
  const i64 s0 = a.soffc[c], s1 = a.soffc[c + 1];
  const i64 col_lo = base * 64, col_hi = (base + nw) * 64;
  if (a.alist && s1 - s0 <= ROWS_SEG) {
    // the allowed-pod lists of S(c) as one flat range: a segment table
    // (start, prefix) in LDS, then every thread streams entries with
    // ROWS_UNROLL loads in flight -- no per-policy round trips
    __shared__ i64 seg_start[ROWS_SEG];
    __shared__ i64 seg_pre[ROWS_SEG + 1];
    __shared__ i64 sm_scan[NT / 64];
    const int ns = (int)(s1 - s0);
    i64 len = 0, st = 0;
    if ((int)threadIdx.x < ns) {   // ns <= ROWS_SEG <= NT
      const int32_t p = a.slist[s0 + threadIdx.x];
      st = a.aloff[p];
      len = a.aloff[p + 1] - st;
    }
    i64 total;
    const i64 pre = block_excl_scan_nw<NT / 64>(len, sm_scan, total);
    if ((int)threadIdx.x < ns) {
      seg_start[threadIdx.x] = st;
      seg_pre[threadIdx.x] = pre;
    }
    if (threadIdx.x == 0) seg_pre[ns] = total;
    __syncthreads();
    for (i64 i0 = threadIdx.x; i0 < total; i0 += (i64)NT * ROWS_UNROLL) {
      int32_t jv[ROWS_UNROLL];
#pragma unroll
      for (int u = 0; u < ROWS_UNROLL; ++u) {
        const i64 id = i0 + (i64)u * NT;
        jv[u] = -1;
        if (id < total) {
          int lo = 0, hi = ns - 1;   // last segment with seg_pre <= id
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (seg_pre[mid] <= id) lo = mid; else hi = mid - 1;
          }
          jv[u] = a.alist[seg_start[lo] + (id - seg_pre[lo])];
        }
      }
#pragma unroll
      for (int u = 0; u < ROWS_UNROLL; ++u) {
        const int32_t j = jv[u];
        if (j >= col_lo && j < col_hi) atomicOr(&row[(j >> 6) - base], 1ull << (j & 63));
      }
    }
  } else if (a.alist) {
    // the flat allowed-pod list of each policy of S(c), across all threads
    for (i64 e = s0; e < s1; ++e) {
      const int32_t p = a.slist[e];
      const int32_t* L = a.alist + a.aloff[p];
      const i64 cnt = a.aloff[p + 1] - a.aloff[p];
      for (i64 k = threadIdx.x; k < cnt; k += NT) {
        const int32_t j = L[k];
        if (j >= col_lo && j < col_hi) atomicOr(&row[(j >> 6) - base], 1ull << (j & 63));
      }
    }
  } else {
    // (policy, allowed column class) entries dealt round-robin to the
    // waves, the class's members across the lanes
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int t = 0;
    for (i64 e = s0; e < s1; ++e) {
      const int32_t p = a.slist[e];
      const i64 q1 = a.alcoff[p + 1];
      for (i64 q = a.alcoff[p]; q < q1; ++q, ++t) {
        if (t % NW != wid) continue;
        const int32_t ca = a.alc[q];
        const int32_t k1 = a.cmoff[ca + 1];
        for (int32_t k = a.cmoff[ca] + lane; k < k1; k += 64) {
          const int32_t j = a.cmem[k];
          if (j >= col_lo && j < col_hi) atomicOr(&row[(j >> 6) - base], 1ull << (j & 63));
        }
      }
    }
  }
  __syncthreads();
}

// one work item (class c, <= ch member rows, column chunk blockIdx.y) of
// k_rows; b = work item index.  Returns uniformly for the whole block.
template <int NT>
__device__ __forceinline__ void rows_item(const RowsArgs& a, i64 b, u64* row) {
  const i64 c = a.wicls ? (i64)a.wicls[b] : upper_bound_i32(a.wioff, a.U + 1, b) - 1;
  if (c < 0 || c >= a.U) return;
  const i64 chunk = b - a.wioff[c];
  const i64 base = (i64)blockIdx.y * a.cww;
  const i64 ldw = a.ldM;
  const int nw = (int)min((i64)a.cww, a.wW - base);
  if (nw <= 0) return;
  const int32_t m_begin = a.moff[c], m_end = a.moff[c + 1];
  const int32_t m0 = m_begin + (int32_t)(chunk * a.ch);
  const int32_t m1 = min(m_end, m0 + a.ch);
  const bool heavy = a.hflag && a.hflag[c];
  if (heavy && a.heavy_skip) return;
  // a class no policy selects (C3: 9,143 of 21,535 row classes): its rows are
  // zero -- stored straight from registers, no row build, no barrier
  if (!heavy && a.soffc[c + 1] == a.soffc[c]) {
    const u64x2 z = {0ull, 0ull};
    for (int32_t m = m0; m < m1; ++m) {
      const int32_t pod = __builtin_amdgcn_readfirstlane(a.mem[m]);
      u64* dst = a.M + (i64)(pod - a.r0) * ldw + base;
      for (int w = threadIdx.x * 2; w < nw; w += NT * 2)
        __builtin_nontemporal_store(z, (u64x2*)&dst[w]);
    }
    if (chunk == 0 && a.color) {
      for (int w = threadIdx.x; w < nw; w += NT) {
        const i64 gw = base + w;
        if (gw >= a.W) break;
        const u64 vm = valid_mask(gw, a.n);
        if (vm & ~a.colnand[gw]) atomicOr(&a.colnand[gw], vm);
      }
    }
    return;
  }

  if (heavy) {
    const u64* src = a.M + (i64)(a.mem[m_begin] - a.r0) * ldw + base;
    for (int w = threadIdx.x * 2; w < nw; w += NT * 2)
      *(u64x2*)&row[w] = *(const u64x2*)&src[w];
    __syncthreads();
  } else {
    build_light_row<NT>(a, c, base, nw, row);
  }
  // non-temporal 16-byte stores (round 2: 5-7 % faster than plain stores
  // alone; round 5: plain stores beside the next build evict its working
  // set, C3 step 0.37 -> 0.50 ms)
  for (int32_t m = m0; m < m1; ++m) {
    if (heavy && m == m_begin) continue;
    u64* dst = a.M + (i64)(a.mem[m] - a.r0) * ldw + base;
    for (int w = threadIdx.x * 2; w < nw; w += NT * 2)
      __builtin_nontemporal_store(*(const u64x2*)&row[w], (u64x2*)&dst[w]);
  }
  if (chunk == 0 && a.color) {
    for (int w = threadIdx.x; w < nw; w += NT) {
      const i64 gw = base + w;
      if (gw >= a.W) break;
      const u64 v = row[w];
      const u64 vm = valid_mask(gw, a.n);
      if (v & ~a.color[gw]) atomicOr(&a.color[gw], v);
      const u64 nv = ~v & vm;
      if (nv & ~a.colnand[gw]) atomicOr(&a.colnand[gw], nv);
    }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_rows(RowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) u64 row[];
  rows_item<NT>(a, blockIdx.x, row);
}

// ---------------------------------------------------------------------------
// Wide rows (a row chunk of more than 4,096 words, e.g. C5's 125 KB rows): the
// chunk fills most of a CU's LDS, so one k_rows block runs per CU and nothing
// hides its work item's chain of dependent loads (item -> class -> S(c) ->
// list offsets -> allowed pods -> member ids; at C5's 1/8 row shard, ~3
// member rows per class, the SQ counters put 68 % of k_rows' wave cycles in
// s_waitcnt).  k_rows_prep resolves the chain ahead, one wave per work item:
// its member range, its kind, its S(c) range and the flattened length of its
// allowed-pod lists, and (first item of a class) each S(c) entry's list
// start re-based on the entry's prefix within the class.  k_rows_w then
// walks the items persistently with the next item's descriptor in flight,
// the member ids and segment table read together, each wave streaming its
// own slice of the class's flattened lists (no block scan, no table in LDS).
// ---------------------------------------------------------------------------
struct RowsItem {     // 32 B
  i64 s0;             // S(c) = slist[s0, s0 + ns)
  i64 total;          // sum of |allowed pods(p)| over p in S(c) (light items)
  int32_t m0, m1;     // member rows mem[m0, m1)
  int32_t ns;
  int32_t src;        // >= 0: heavy (copy row src, prebuilt); -1 light; -2 zero row
};
struct RowsSeg {      // entry e of S(c): alist index of flat id f = base + f
  i64 base, pre;      // pre: flat id of the entry's first pod
};

__global__ __launch_bounds__(TPB) void k_rows_prep(RowsArgs a, i64 nitems,
                                                   RowsItem* __restrict__ items,
                                                   RowsSeg* __restrict__ segs,
                                                   int32_t* __restrict__ ticket) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (ticket && blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0;
  const i64 b = (i64)blockIdx.x * (TPB / 64) + wid;
  if (b >= nitems) return;                  // wave-uniform
  const int32_t c = a.wicls[b];
  const i64 chunk = b - a.wioff[c];
  const int32_t mb = a.moff[c], me = a.moff[c + 1];
  const int32_t m0 = mb + (int32_t)(chunk * a.ch);
  int32_t m1 = min(me, m0 + a.ch);
  const i64 s0 = a.soffc[c], s1 = a.soffc[c + 1];
  int32_t src = -1;
  i64 run = 0;
  if (a.hflag && a.hflag[c]) {
    src = a.mem[mb];
    if (a.heavy_skip) m1 = m0;       // (written whole by k_heavy_rows_t)
  } else if (s1 == s0) {
    src = -2;
  } else {
    for (i64 e0 = s0; e0 < s1; e0 += 64) {
      const i64 e = e0 + lane;
      i64 st = 0, len = 0;
      if (e < s1) {
        const int32_t p = a.slist[e];
        st = a.aloff[p];
        len = a.aloff[p + 1] - st;
      }
      i64 tot;
      const i64 pre = run + wave_excl_scan(len, tot);
      if (chunk == 0 && e < s1) segs[e] = RowsSeg{st - pre, pre};
      run += tot;
    }
  }
  if (lane == 0) items[b] = RowsItem{s0, run, m0, m1, (int32_t)(s1 - s0), src};
}

__device__ __forceinline__ i64 readlane64(i64 v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)((u64)v >> 32), l);
  return (i64)(((u64)(uint32_t)hi << 32) | (uint32_t)lo);
}

constexpr int ROWSW_UNROLL = 8;
// Units are (item, column chunk) pairs, u = item * ncc + chunk (a chunk
// holds up to 16,384 words: one chunk per row up to 1M pods; half-row chunks
// measured 3.78 -> 5.22 ms at C5's 1/8 shard, each chunk walking every
// entry).  ticket (persistent grids): the next unit is gridDim.x +
// ticket[0]++, drawn at the start of the current unit's build and its
// descriptor loaded during the current unit's stores; nullptr: one unit per
// block (or a static stride)
template <int NT>
__global__ __launch_bounds__(NT) void k_rows_w(RowsArgs a, const RowsItem* __restrict__ items,
                                               i64 nitems, const RowsSeg* __restrict__ segs,
                                               int32_t* __restrict__ ticket, int ncc) {
  __shared__ i64 s_next;
  extern __shared__ __attribute__((aligned(16))) u64 row[];
  constexpr int NW = NT / 64;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const i64 nunits = nitems * ncc;
  const i64 G = gridDim.x;
  for (int w = threadIdx.x; w < a.cww; w += NT) row[w] = 0ull;
  __syncthreads();
  i64 u = blockIdx.x;
  RowsItem nx{};
  if (u < nunits) nx = items[u / ncc];
  while (u < nunits) {
    const RowsItem d = nx;
    if (ticket && threadIdx.x == 0) s_next = G + atomicAdd(ticket, 1);
    const i64 base = (u % ncc) * a.cww;
    const int nw = (int)min((i64)a.cww, a.wW - base);   // even (ldM and cww are), > 0
    const i64 col_lo = base * 64, col_hi = (base + nw) * 64;
    const int nm = d.m1 - d.m0;                       // <= 64 (host: ch <= 64)
    const int32_t mv = lane < nm ? a.mem[d.m0 + lane] : -1;
    if (d.src >= 0) {
      const u64* src = a.M + (i64)(d.src - a.r0) * a.ldM + base;
      for (int w = threadIdx.x * 2; w < nw; w += NT * 2)
        *(u64x2*)&row[w] = *(const u64x2*)&src[w];
    } else if (d.src == -1) {
      // this wave's slice [r0, r1) of the class's flattened lists
      const i64 T = d.total;
      const i64 r0 = T * wid / NW, r1 = T * (wid + 1) / NW;
      for (int i0 = 0; i0 < d.ns && r0 < r1; i0 += 64) {
        const int e = i0 + lane;
        i64 sb = 0, sp = T, sn = T;
        if (e < d.ns) {
          const RowsSeg s = segs[d.s0 + e];
          sb = s.base;
          sp = s.pre;
          if (e + 1 < d.ns) sn = segs[d.s0 + e + 1].pre;
        }
        const int cnt = min(64, d.ns - i0);
        for (int i = 0; i < cnt; ++i) {
          const i64 lo = max(readlane64(sp, i), r0), hi = min(readlane64(sn, i), r1);
          if (lo >= hi) continue;                     // wave-uniform
          const int32_t* L = a.alist + readlane64(sb, i);
          for (i64 j0 = lo; j0 < hi; j0 += 64 * ROWSW_UNROLL) {
            int32_t jv[ROWSW_UNROLL];
#pragma unroll
            for (int u = 0; u < ROWSW_UNROLL; ++u) {
              const i64 j = j0 + lane + 64 * u;
              jv[u] = j < hi ? L[j] : -1;
            }
#pragma unroll
            for (int u = 0; u < ROWSW_UNROLL; ++u) {
              const i64 j = jv[u];
              if (j >= col_lo && j < col_hi) atomicOr(&row[(j >> 6) - base], 1ull << (j & 63));
            }
          }
        }
      }
    }
    __syncthreads();
    const i64 next = ticket ? s_next : u + G;
    if (next < nunits) nx = items[next / ncc];        // in flight during the stores
    for (int k = 0; k < nm; ++k) {
      const int32_t pod = __builtin_amdgcn_readlane(mv, k);
      if (pod == d.src) continue;
      u64* dst = a.M + (i64)(pod - a.r0) * a.ldM + base;
      for (int w = threadIdx.x * 2; w < nw; w += NT * 2)
        __builtin_nontemporal_store(*(const u64x2*)&row[w], (u64x2*)&dst[w]);
    }
    // each thread clears the words it streamed (the next item's atomics
    // start after the barrier)
    const u64x2 z = {0ull, 0ull};
    for (int w = threadIdx.x * 2; w < nw; w += NT * 2) *(u64x2*)&row[w] = z;
    __syncthreads();
    u = next;
  }
}



// ===========================================================================
// Row digests (full-size property checks: a 1M-pod matrix is 125 GB, too big
// to bring to the host).  digest(row) = sum over k < W of
// mix64(row[k] ^ k * 0xD6E8FEB86659FD93) mod 2^64, mix64 = splitmix64's
// finaliser; tests/_golden.py row_digest is the same on the host.
// ===========================================================================
__device__ __forceinline__ u64 mix64(u64 z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// one block per row
__global__ __launch_bounds__(TPB) void k_row_digest(const u64* __restrict__ M, i64 ldM, i64 W,
                                                    u64* __restrict__ out) {
  const u64* r = M + (i64)blockIdx.x * ldM;
  u64 h = 0;
  for (i64 k = threadIdx.x; k < W; k += TPB) h += mix64(r[k] ^ ((u64)k * 0xD6E8FEB86659FD93ull));
  __shared__ u64 part[TPB / 64];
  h = wave_sum(h);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 t = 0;
    for (int w = 0; w < TPB / 64; ++w) t += part[w];
    out[blockIdx.x] = t;
  }
}

// ===========================================================================
// Checks
// ===========================================================================
__global__ __launch_bounds__(TPB) void k_col_final(const u64* __restrict__ colnand, i64 W, i64 n,
                                                   u64* __restrict__ col_and) {
  const i64 w = (i64)blockIdx.x * TPB + threadIdx.x;
  if (w < W) col_and[w] = ~colnand[w] & valid_mask(w, n);
}

// one byte per column
__global__ __launch_bounds__(TPB) void k_unpack_flags(const u64* __restrict__ words, i64 n,
                                                      uint8_t* __restrict__ out) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  if (j < n) out[j] = (uint8_t)((words[j >> 6] >> (j & 63)) & 1ull);
}

// user_crosscheck.  cross[j] = exists row i: M[i,j] and g(i) != g(j).
// Rows of a class are equal; a class whose local members carry >= 2 groups
// reaches every set column from another group (MULTI); single-group classes
// are ORed per group into R[g].  Then with A1 = OR_g R[g], A2 = bits set by
// >= 2 groups (atomicOr's previous value), own[j] = R[g(j)][j]:
//   cross = MULTI | A2 | (A1 & ~own)
__global__ __launch_bounds__(TPB) void k_cross_classgroup(const int32_t* __restrict__ gid,
                                                          const int32_t* __restrict__ moff,
                                                          const int32_t* __restrict__ mem, i64 U,
                                                          int32_t* __restrict__ cgroup) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  const int32_t m0 = moff[c], m1 = moff[c + 1];
  int32_t g = -2;  // -2: no local members, -1: several groups
  if (m1 > m0) {
    g = gid[mem[m0]];
    for (int32_t m = m0 + 1; m < m1; ++m)
      if (gid[mem[m]] != g) { g = -1; break; }
  }
  cgroup[c] = g;
}

__global__ __launch_bounds__(TPB) void k_cross_accum(const int32_t* __restrict__ cgroup,
                                                     const int32_t* __restrict__ moff,
                                                     const int32_t* __restrict__ mem,
                                                     const u64* __restrict__ M, i64 ldM, i64 r0,
                                                     i64 W, int32_t g0, int32_t g1,
                                                     u64* __restrict__ R, u64* __restrict__ multi) {
  const i64 c = blockIdx.x;
  const int32_t g = cgroup[c];
  if (g == -2) return;
  const bool is_multi = g == -1;
  if (is_multi && g0 != 0) return;  // multi rows are folded in by the first pass only
  if (!is_multi && (g < g0 || g >= g1)) return;
  const u64* src = M + (i64)(mem[moff[c]] - r0) * ldM;
  u64* dst = is_multi ? multi : R + (i64)(g - g0) * ldM;
  for (i64 w = (i64)blockIdx.y * TPB + threadIdx.x; w < W; w += (i64)gridDim.y * TPB) {
    const u64 v = src[w];
    if (v) atomicOr(&dst[w], v);
  }
}

__global__ __launch_bounds__(TPB) void k_cross_groups(const u64* __restrict__ R, i64 ldM, i64 W,
                                                      u64* __restrict__ A1, u64* __restrict__ A2) {
  const i64 g = blockIdx.x;
  for (i64 w = (i64)blockIdx.y * TPB + threadIdx.x; w < W; w += (i64)gridDim.y * TPB) {
    const u64 r = R[g * ldM + w];
    if (!r) continue;
    const u64 old = atomicOr(&A1[w], r);
    if (old & r) atomicOr(&A2[w], old & r);
  }
}

__global__ __launch_bounds__(TPB) void k_cross_own(const int32_t* __restrict__ gid, i64 n,
                                                   const u64* __restrict__ R, i64 ldM, int32_t g0,
                                                   int32_t g1, u64* __restrict__ own) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  bool bit = false;
  if (j < n) {
    const int32_t g = gid[j];
    if (g >= g0 && g < g1) bit = (R[(i64)(g - g0) * ldM + (j >> 6)] >> (j & 63)) & 1ull;
  }
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && bal) atomicOr(&own[j >> 6], bal);
}

__global__ __launch_bounds__(TPB) void k_cross_final(const u64* __restrict__ multi,
                                                     const u64* __restrict__ A1,
                                                     const u64* __restrict__ A2,
                                                     const u64* __restrict__ own, i64 W, i64 n,
                                                     u64* __restrict__ cross) {
  const i64 w = (i64)blockIdx.x * TPB + threadIdx.x;
  if (w < W) cross[w] = (multi[w] | A2[w] | (A1[w] & ~own[w])) & valid_mask(w, n);
}

// getcol (model.py:180-184): bit r = M[r][j] over the local rows
__global__ __launch_bounds__(TPB) void k_get_col(const u64* __restrict__ M, i64 ldM, i64 rows,
                                                 i64 j, u64* __restrict__ out) {
  const i64 r = (i64)blockIdx.x * TPB + threadIdx.x;
  const bool bit = r < rows && ((M[r * ldM + (j >> 6)] >> (j & 63)) & 1ull);
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && r < rows) out[r >> 6] = bal;
}

// working_select_set of policy p over all pods: p in S(cls(i)) (sorted lists)
__global__ __launch_bounds__(TPB) void k_sel_row(const i64* __restrict__ soffc,
                                                 const int32_t* __restrict__ slist,
                                                 const int32_t* __restrict__ cls, i64 n,
                                                 i64 r0, i64 r1, i64 p,
                                                 u64* __restrict__ out) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  bool bit = false;
  if (i < n && i >= r0 && i < r1) {   // row classes exist for this shard's pods
    const int32_t c = cls[i];
    i64 lo = soffc[c], hi = soffc[c + 1];
    while (lo < hi) {
      const i64 mid = (lo + hi) >> 1;
      if (slist[mid] < p) lo = mid + 1; else hi = mid;
    }
    bit = lo < soffc[c + 1] && slist[lo] == p;
  }
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && i < n) out[i >> 6] = bal;
}

// working_allow_set of policy p over all pods
__global__ __launch_bounds__(TPB) void k_allow_row(const u64* __restrict__ AC, i64 ldC, i64 p,
                                                   const int32_t* __restrict__ cla, i64 n,
                                                   u64* __restrict__ out) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  bool bit = false;
  if (j < n) {
    const int32_t ca = cla[j];
    bit = (AC[p * ldC + (ca >> 6)] >> (ca & 63)) & 1ull;
  }
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && j < n) out[j >> 6] = bal;
}

// ===========================================================================
// policy_shadow (algorithm.py:58-80) on row classes.  Pair (a, b) of S(c)
// positions, a != b:  flag = allow_{S[b]} is a subset of allow_{S[a]}, tested
// on column classes (they partition the pods and none is empty, so the pod
// sets nest exactly when the class sets do).
// ===========================================================================
__device__ __forceinline__ bool subset_of(int32_t k, int32_t j, const int32_t* nca,
                                          const i64* alcoff, const int32_t* alc, const u64* AC,
                                          i64 ldC) {
  const int32_t ck = nca[k];
  if (ck == 0) return true;
  if (ck > nca[j]) return false;
  const int32_t* L = alc + alcoff[k];
  const u64* aj = AC + (i64)j * ldC;
  for (int32_t e = 0; e < ck; ++e) {
    const int32_t x = L[e];
    if (!((aj[x >> 6] >> (x & 63)) & 1ull)) return false;
  }
  return true;
}

struct ShadowArgs {
  i64 U;
  const i64* soffc;
  const int32_t* slist;
  const int32_t* mcnt;
  const i64* pfoff;
  const int32_t* nca;
  const i64* alcoff;
  const int32_t* alc;
  const u64* AC;
  i64 ldC;
  uint8_t* flags;
  i64* T;
  // count only (flags null): the grouped count's verdict (shg_grouped),
  // when set the pairwise test leaves T to it
  const int32_t* shg_G;
  const int32_t* shg_err;
  const u64* shg_nf;
  int shg_force;
};

// Count-only policy_shadow, decided on the device once the allow-set groups
// are known: the grouped count (k_shg_sub's G^2 row compares + per class
// m_c^2 bit tests) when G <= SHG_MAX, no hash collision and G^2 <= nf / 4
// (nf = the pairwise candidate pairs), else the pairwise test (k_shadow_test1
// without flags).  C3: G = 4,092, nf = 5.8e7 -> pairwise (29 us; grouped
// 5.2 ms); C4: G = 111 -> grouped.  force 2: grouped whatever G (the count
// falls back pair by pair per class past SHG_MAX or on a collision).
constexpr int SHG_MAX = 4096;
__device__ __forceinline__ bool shg_grouped(const int32_t* Gp, const int32_t* err, const u64* nfp,
                                            int force) {
  if (force == 2) return true;
  const i64 G = *Gp;
  if (*err || G > SHG_MAX) return false;
  return (u64)(G * G) <= *nfp / 4;
}

// The candidate pairs of every row class c are (x, y) in [0, s_c)^2, laid out
// flat at pfoff[c] (class-major, x-major).  Both kernels take SH_TILE
// consecutive pairs per block, so the work is balanced whatever the |S(c)|
// distribution.
constexpr int SH_ITEMS = 8;
constexpr i64 SH_TILE = (i64)TPB * SH_ITEMS;

// last class c in [lo, hi] with pfoff[c] <= t
__device__ __forceinline__ i64 class_of_pair(const i64* __restrict__ pfoff, i64 lo, i64 hi,
                                             i64 t) {
  while (lo < hi) {
    const i64 mid = (lo + hi + 1) >> 1;
    if (pfoff[mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// last class c in [lo, hi] with pfoff[c] <= t (pfoff[lo] <= t), searched by
// one whole wave (uniform arguments): 64 pivots per round, so the 21.5k
// classes of C3 take 3 dependent loads instead of the 15 of a binary search
// (the block's first loads, before any test can start)
__device__ __forceinline__ i64 wave_class_of(const i64* __restrict__ pfoff, i64 lo, i64 hi,
                                             i64 t) {
  const int lane = threadIdx.x & 63;
  while (hi > lo) {
    const i64 step = (hi - lo + 64) / 64;
    const i64 idx = lo + (i64)lane * step;
    const bool ok = idx <= hi && pfoff[idx] <= t;
    const u64 m = __ballot(ok);                 // a prefix of the lanes (lane 0 set)
    lo += (i64)(63 - __builtin_clzll(m)) * step;
    hi = min(hi, lo + step - 1);
  }
  return lo;
}

// the class range of this block's tile: two searches over all classes, by
// two waves, then every thread searches only inside the range
__device__ __forceinline__ void tile_class_range(const i64* __restrict__ pfoff, i64 U,
                                                 i64 nflags, i64* s_rng) {
  const i64 b0 = (i64)blockIdx.x * SH_TILE;
  const i64 b1 = min(b0 + SH_TILE, nflags) - 1;
  const int wv = threadIdx.x >> 6;
  if (wv < 2) {
    const i64 c = wave_class_of(pfoff, 0, U - 1, wv == 0 ? b0 : b1);
    if ((threadIdx.x & 63) == 0) s_rng[wv] = c;
  }
  __syncthreads();
}



// The same test with the block's select-list data staged in LDS first: the
// classes of the block's 256 pairs (pfoff, soffc, mcnt), then their S(c)
// entries (policy, allowed-class count, list offset, first allowed class) --
// one short dependent chain per block instead of ~10 dependent loads per
// thread.  A thread then reads its pair's class and policies from LDS and
// usually decides with one global load (the first allowed class of k missing
// from AC[j]).  Blocks whose class range or S(c) segment does not fit fall
// back to the global form.
constexpr int SHS_CLS = TPB + 2;
// SEG: staged S(c) entries per block (1024: ~25 KB of LDS; 512, ten blocks
// per CU, measured slightly slower beside the main stream's kernels)
constexpr int SHS_U = 8;
// R: 256-pair rounds per block on one staging (the class range and the S(c)
// segment of all R x 256 pairs): with ~7e7 candidate pairs (C5 row shards)
// the per-block staging chain -- two wave searches, then the classes, then
// the segment, each a dependent global round trip -- was the kernel's time
// (C5 rank 0 of 8: 2.39 -> 1.65 ms at R = 4, a little less at 8).  A per-policy 64-bit allow-set
// signature tested before AC (round 5) measured slower there too (1.78 ms).
template <int SHS_SEG, int R>
__global__ __launch_bounds__(TPB) void k_shadow_test1s(ShadowArgs a, i64 nflags,
                                                      i64* __restrict__ tile_cnt) {
  __shared__ i64 sm[4];
  __shared__ i64 rng[2];
  __shared__ i64 s_pf[SHS_CLS];
  __shared__ i64 s_so[SHS_CLS];
  __shared__ int32_t s_mc[SHS_CLS];
  __shared__ i64 s_ao[SHS_SEG];
  __shared__ int32_t s_pol[SHS_SEG];
  __shared__ int32_t s_nca[SHS_SEG];
  __shared__ int32_t s_x0[SHS_SEG];
  static_assert(SH_TILE % (TPB * R) == 0, "a block's pairs stay inside one tile");
  if (a.shg_G && shg_grouped(a.shg_G, a.shg_err, a.shg_nf, a.shg_force)) return;
  constexpr i64 PB = (i64)TPB * R;               // pairs per virtual block
  const i64 nvb = (nflags + PB - 1) / PB;
  for (i64 vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    const i64 B0 = vb * PB;
    if (B0 >= nflags) break;                     // block-uniform (B0 rises with vb)
    const i64 B1 = min(B0 + PB, nflags) - 1;
    if ((threadIdx.x >> 6) < 2) {
      const int wv = threadIdx.x >> 6;
      const i64 cr = wave_class_of(a.pfoff, 0, a.U - 1, wv == 0 ? B0 : B1);
      if ((threadIdx.x & 63) == 0) rng[wv] = cr;
    }
    __syncthreads();
    const i64 c0 = rng[0], c1 = rng[1];
    const i64 ncls = c1 - c0 + 1;
    const bool staged_cls = ncls + 1 <= SHS_CLS;
    i64 seg0 = 0, nseg = SHS_SEG + 1;
    if (staged_cls) {
      for (i64 k = threadIdx.x; k <= ncls; k += TPB) {
        s_pf[k] = a.pfoff[c0 + k];
        s_so[k] = a.soffc[c0 + k];
        if (k < ncls) s_mc[k] = a.mcnt[c0 + k];
      }
      __syncthreads();
      seg0 = s_so[0];
      nseg = s_so[ncls] - seg0;
    }
    const bool staged = staged_cls && nseg <= SHS_SEG;   // block-uniform
    if (staged) {
      for (i64 e = threadIdx.x; e < nseg; e += TPB) {
        const int32_t p = a.slist[seg0 + e];
        const int32_t cnt = a.nca[p];
        const i64 ao = a.alcoff[p];
        s_pol[e] = p;
        s_nca[e] = cnt;
        s_ao[e] = ao;
        s_x0[e] = cnt > 0 ? a.alc[ao] : 0;
      }
      __syncthreads();
    }
    for (int r = 0; r < R; ++r) {
      const i64 b0 = B0 + (i64)r * TPB;
      if (b0 >= nflags) break;                   // block-uniform
      const i64 tile = b0 / SH_TILE;
      const i64 t = b0 + threadIdx.x;
      int f = 0;
      i64 c = -1;
      if (t < nflags) {
        if (staged) {
          i64 lo = 0, hi = ncls - 1;             // last class with pfoff <= t
          while (lo < hi) {
            const i64 mid = (lo + hi + 1) >> 1;
            if (s_pf[mid] <= t) lo = mid; else hi = mid - 1;
          }
          c = c0 + lo;
          const i64 e0 = s_so[lo] - seg0, s = s_so[lo + 1] - s_so[lo], q = t - s_pf[lo];
          const i64 x = q / s, y = q - x * s;
          if (s_mc[lo] > 0 && x != y) {
            const int32_t j = s_pol[e0 + x], kk = s_pol[e0 + y];
            const int32_t ck = s_nca[e0 + y];
            if (j != kk) {
              if (ck == 0) {
                f = 1;
              } else if (ck <= s_nca[e0 + x]) {
                const u64* aj = a.AC + (i64)j * a.ldC;
                int32_t xe = s_x0[e0 + y];
                bool ok = (aj[xe >> 6] >> (xe & 63)) & 1ull;
                // the rest of k's list SHS_U entries at a time: the loads of
                // a round are independent (a subset's full walk is the long
                // pole of a wave)
                const int32_t* L = a.alc + s_ao[e0 + y];
                for (int32_t e = 1; ok && e < ck; e += SHS_U) {
                  int32_t xs[SHS_U];
#pragma unroll
                  for (int u = 0; u < SHS_U; ++u) xs[u] = e + u < ck ? L[e + u] : xe;
                  u64 ws[SHS_U];
#pragma unroll
                  for (int u = 0; u < SHS_U; ++u) ws[u] = aj[xs[u] >> 6];
#pragma unroll
                  for (int u = 0; u < SHS_U; ++u) ok = ok && ((ws[u] >> (xs[u] & 63)) & 1ull);
                }
                f = ok;
              }
            }
          }
        } else {
          c = class_of_pair(a.pfoff, c0, c1, t);
          const i64 s0 = a.soffc[c], s = a.soffc[c + 1] - s0, q = t - a.pfoff[c];
          const i64 x = q / s, y = q - x * s;
          if (a.mcnt[c] > 0 && x != y) {
            const int32_t j = a.slist[s0 + x], kk = a.slist[s0 + y];
            f = (j != kk) && subset_of(kk, j, a.nca, a.alcoff, a.alc, a.AC, a.ldC);
          }
        }
      }
      // the flags as bits, one ballot word per wave (the wave's 64 pairs are
      // consecutive: b0 is a multiple of 256); null: count only (T[c])
      {
        const u64 bal = __ballot(f != 0);
        const i64 w0 = b0 + (i64)(threadIdx.x & ~63);
        if (a.flags && (threadIdx.x & 63) == 0 && w0 < nflags)
          reinterpret_cast<u64*>(a.flags)[w0 >> 6] = bal;
      }
      const i64 cw = __shfl(c, 0, 64);
      if (__all(c == cw || c < 0)) {
        const int rr = wave_sum(f);
        if ((threadIdx.x & 63) == 0 && rr && cw >= 0)
          atomicAdd(reinterpret_cast<unsigned long long*>(&a.T[cw]), (unsigned long long)rr);
      } else if (f) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.T[c]), 1ull);
      }
      const i64 tot = block_sum((i64)f, sm);
      if (threadIdx.x == 0 && tot && tile_cnt)   // (null: count only)
        atomicAdd(reinterpret_cast<unsigned long long*>(&tile_cnt[tile]), (unsigned long long)tot);
    }
    if ((i64)gridDim.x >= nvb) break;           // one virtual block per block (uniform)
    __syncthreads();                             // LDS reused by the next virtual block
  }
}

// ---------------------------------------------------------------------------
// policy_shadow's pair count without the pairs (kano_verify, shadow_cap < 0):
// algorithm.py:58-80 counts, per pod i, the ordered pairs j != k of S(i) with
// allow_k a subset of allow_j.  Policies with equal allow sets answer every
// subset test alike, so the policies are grouped by their class-level allow
// row AC[p] (hash, then a full-row check against the group's first policy);
// sub[a][b] = allow(b) <= allow(a) is tested once per pair of groups, and a
// row class with group counts n_c contributes  n_c' Sub n_c - |S(c)|  pairs
// per member.  Broad selectors (C4): ~10^8 pair tests become ~10^4 group
// tests.  On a hash collision or more than SHG_MAX groups every class falls
// back to the pair-by-pair test (same result, slower).
// ---------------------------------------------------------------------------
// one wave per policy: 64-bit hash of AC[p] (never the empty key ~0)
__global__ __launch_bounds__(TPB) void k_shg_hash(i64 P, const u64* __restrict__ AC, i64 ldC,
                                                  i64 UAW, u64* __restrict__ h) {
  const i64 p = (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  const u64* r = AC + p * ldC;
  u64 x = 0;
  for (i64 w = lane; w < UAW; w += 64) x += mix64(r[w] ^ ((u64)w * 0xD6E8FEB86659FD93ull));
  x = wave_sum(x);
  if (lane == 0) h[p] = x == ~0ull ? 0ull : x;
}

// open-addressing insert keyed by the hash; the slot keeps its smallest policy
__global__ __launch_bounds__(TPB) void k_shg_insert(i64 P, const u64* __restrict__ h,
                                                    unsigned long long* __restrict__ tkey,
                                                    int32_t* __restrict__ trep,
                                                    int32_t* __restrict__ slot_of, uint32_t tmask) {
  const i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
  if (p >= P) return;
  const unsigned long long key = h[p];
  uint32_t s = (uint32_t)(key ^ (key >> 29)) & tmask;
  // (a read before the CAS and the min: C4's 10^4 policies fall into ~10^2
  // groups, and every atomic on a taken slot serialised behind the others)
  for (;;) {
    const unsigned long long cur = __hip_atomic_load(&tkey[s], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) break;
    if (cur == ~0ull) {
      const unsigned long long prev = atomicCAS(&tkey[s], ~0ull, key);
      if (prev == ~0ull || prev == key) break;
    }
    s = (s + 1) & tmask;
  }
  if (__hip_atomic_load(&trep[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (int32_t)p)
    atomicMin(&trep[s], (int32_t)p);
  slot_of[p] = (int32_t)s;
}

// isrep[p] (the group's first policy); a policy whose row differs from its
// representative's (a hash collision) sets err
__global__ __launch_bounds__(TPB) void k_shg_verify(i64 P, const int32_t* __restrict__ slot_of,
                                                    const int32_t* __restrict__ trep,
                                                    const u64* __restrict__ AC, i64 ldC, i64 UAW,
                                                    int32_t* __restrict__ isrep,
                                                    int32_t* __restrict__ err) {
  const i64 p = (i64)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  const int32_t r = trep[slot_of[p]];
  if (lane == 0) isrep[p] = r == p ? 1 : 0;
  if (r == p) return;
  const u64* a = AC + p * ldC;
  const u64* b = AC + (i64)r * ldC;
  bool diff = false;
  for (i64 w = lane; w < UAW; w += 64) diff |= a[w] != b[w];
  if (__any(diff) && lane == 0) atomicOr(err, 1);
}

// exclusive scan of isrep in one block (gidx[P] = the group count)
__global__ __launch_bounds__(1024) void k_shg_scan(i64 P, const int32_t* __restrict__ isrep,
                                                   int32_t* __restrict__ gidx) {
  __shared__ int32_t sm[16];
  const i64 per = (P + 1023) / 1024;
  const i64 b0 = threadIdx.x * per, b1 = min(P, b0 + per);
  int32_t s = 0;
  for (i64 q = b0; q < b1; ++q) s += isrep[q];
  int32_t tot;
  int32_t pre = block_excl_scan_nw<16>(s, sm, tot);
  for (i64 q = b0; q < b1; ++q) {
    gidx[q] = pre;
    pre += isrep[q];
  }
  if (threadIdx.x == 0) gidx[P] = tot;
}

// gid[p] = dense group of p; reps[g] = the group's first policy
__global__ __launch_bounds__(TPB) void k_shg_assign(i64 P, const int32_t* __restrict__ slot_of,
                                                    const int32_t* __restrict__ trep,
                                                    const int32_t* __restrict__ isrep,
                                                    const int32_t* __restrict__ gidx,
                                                    int32_t* __restrict__ gid,
                                                    int32_t* __restrict__ reps) {
  const i64 p = (i64)blockIdx.x * TPB + threadIdx.x;
  if (p >= P) return;
  const int32_t g = gidx[trep[slot_of[p]]];
  gid[p] = g;
  if (isrep[p] && g < SHG_MAX) reps[g] = (int32_t)p;
}

// sub[a][b / 64] bit b = allow(reps[b]) <= allow(reps[a]); one wave per a.
// With lds_row, a's row sits in LDS and b is tested through its class list
// (alc: |allow(b)| bit probes, the first miss ends it; a longer list than a's
// rejects at once) -- the word-by-word compare read each b's row from HBM per
// a, 64 rows per wave-load (D1: 0.46 ms for ~2,000 groups).
__global__ __launch_bounds__(TPB) void k_shg_sub(const int32_t* __restrict__ Gp,
                                                 const int32_t* __restrict__ reps,
                                                 const u64* __restrict__ AC, i64 ldC, i64 UAW,
                                                 u64* __restrict__ sub, i64 GW,
                                                 const int32_t* __restrict__ err,
                                                 const u64* __restrict__ nfp, int force,
                                                 const int32_t* __restrict__ nca,
                                                 const i64* __restrict__ alcoff,
                                                 const int32_t* __restrict__ alc, int lds_row) {
  extern __shared__ __attribute__((aligned(16))) u64 shg_rows[];
  const int32_t G = *Gp;
  if (G > SHG_MAX || !shg_grouped(Gp, err, nfp, force)) return;   // block-uniform
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const i64 a = (i64)blockIdx.x * WPB + wid;
  const bool act = a < G;
  const int32_t pa = act ? reps[a] : 0;
  const u64* ra = AC + (i64)pa * ldC;
  u64* rl = shg_rows + (i64)wid * UAW;
  if (lds_row) {
    if (act)
      for (i64 w = lane; w < UAW; w += 64) rl[w] = ra[w];
    __syncthreads();
  }
  if (!act) return;
  const int32_t na = nca[pa];
  for (i64 hb = 0; hb * 64 < G; ++hb) {
    const i64 b = hb * 64 + lane;
    bool ok = false;
    if (b < G) {
      const int32_t pb = reps[b];
      if (lds_row) {
        const int32_t nb = nca[pb];
        if (nb <= na) {
          ok = true;
          if (nb <= UAW) {
            const int32_t* L = alc + alcoff[pb];
            for (int32_t e = 0; e < nb && ok; ++e) {
              const int32_t x = L[e];
              ok = (rl[x >> 6] >> (x & 63)) & 1ull;
            }
          } else {
            const u64* rb = AC + (i64)pb * ldC;
            for (i64 w = 0; w < UAW && ok; ++w) ok = (rb[w] & ~rl[w]) == 0;
          }
        }
      } else {
        const u64* rb = AC + (i64)pb * ldC;
        ok = true;
        for (i64 w = 0; w < UAW && ok; ++w) ok = (rb[w] & ~ra[w]) == 0;
      }
    }
    const u64 bits = __ballot(ok);
    if (lane == 0) sub[a * GW + hb] = bits;
  }
}

// T[c] = flagged pairs of row class c (one block per class)
// (not shg_grouped: T is the pairwise test's)
__global__ __launch_bounds__(TPB) void k_shg_count(ShadowArgs a, const int32_t* __restrict__ gid,
                                                   const int32_t* __restrict__ Gp,
                                                   const u64* __restrict__ sub, i64 GW,
                                                   const int32_t* __restrict__ err) {
  __shared__ int32_t hist[SHG_MAX];
  __shared__ int32_t gl[SHG_MAX];
  __shared__ int32_t ngl;
  __shared__ i64 sm[4];
  if (!shg_grouped(Gp, err, a.shg_nf, a.shg_force)) return;
  const i64 c = blockIdx.x;
  if (a.mcnt[c] == 0) return;                    // no local member: T[c] stays 0
  const i64 s0 = a.soffc[c], s = a.soffc[c + 1] - s0;
  if (s < 2) return;
  const int32_t G = *Gp;
  i64 acc = 0;
  if (*err || G > SHG_MAX) {
    // the pair-by-pair test (algorithm.py:76-79 at class level)
    for (i64 q = threadIdx.x; q < s * s; q += TPB) {
      const i64 x = q / s, y = q - x * s;
      if (x == y) continue;
      const int32_t j = a.slist[s0 + x], kk = a.slist[s0 + y];
      acc += (j != kk) && subset_of(kk, j, a.nca, a.alcoff, a.alc, a.AC, a.ldC);
    }
    const i64 tot = block_sum(acc, sm);
    if (threadIdx.x == 0) a.T[c] = tot;
    return;
  }
  for (int g = threadIdx.x; g < G; g += TPB) hist[g] = 0;
  if (threadIdx.x == 0) ngl = 0;
  __syncthreads();
  for (i64 e = threadIdx.x; e < s; e += TPB) {
    const int32_t g = gid[a.slist[s0 + e]];
    if (atomicAdd(&hist[g], 1) == 0) gl[atomicAdd(&ngl, 1)] = g;
  }
  __syncthreads();
  const i64 m = ngl;
  for (i64 q = threadIdx.x; q < m * m; q += TPB) {
    const int32_t ga = gl[q / m], gb = gl[q % m];
    if ((sub[(i64)ga * GW + (gb >> 6)] >> (gb & 63)) & 1ull) acc += (i64)hist[ga] * hist[gb];
  }
  const i64 tot = block_sum(acc, sm);
  if (threadIdx.x == 0) a.T[c] = tot - s;
}

// the flagged pairs in flat order: L[tile_off[b] + rank] = (j, k)
__global__ __launch_bounds__(TPB) void k_shadow_compact(const i64* __restrict__ soffc, i64 U,
                                                        const int32_t* __restrict__ slist,
                                                        const i64* __restrict__ pfoff,
                                                        const uint8_t* __restrict__ flags,
                                                        i64 nflags,
                                                        const i64* __restrict__ tile_off,
                                                        int2* __restrict__ L, i64 L_cap) {
  __shared__ i64 sm[4];
  __shared__ i64 rng[2];
  // (sized before the list length is known: past L_cap nothing is written,
  // the host sees the total and runs the sized launch)
  if (tile_off[gridDim.x] > L_cap) return;        // grid-uniform
  tile_class_range(pfoff, U, nflags, rng);
  const i64 base = (i64)blockIdx.x * SH_TILE + (i64)threadIdx.x * SH_ITEMS;
  static_assert(SH_ITEMS == 8, "one flag byte (8 pairs) per thread");
  // (flags are bits, pair t at bit t & 7 of byte t >> 3; bits past nflags are 0)
  const uint32_t packed = base < nflags ? flags[base >> 3] : 0u;
  const i64 cnt = __popc(packed);
  i64 tot;
  i64 pos = block_excl_scan(cnt, sm, tot) + tile_off[blockIdx.x];
  if (cnt == 0) return;
  i64 c = class_of_pair(pfoff, rng[0], rng[1], base);
  i64 s0 = soffc[c], s = soffc[c + 1] - s0, p0 = pfoff[c], p1 = pfoff[c + 1];
  for (int k = 0; k < SH_ITEMS; ++k) {
    if (!((packed >> k) & 1u)) continue;
    const i64 t = base + k;
    while (t >= p1) {
      ++c;
      s0 = soffc[c];
      s = soffc[c + 1] - s0;
      p0 = p1;
      p1 = pfoff[c + 1];
    }
    const i64 q = t - p0, x = q / s, y = q - x * s;
    L[pos++] = make_int2(slist[s0 + x], slist[s0 + y]);
  }
}

__global__ __launch_bounds__(TPB) void k_shadow_podcount(const int32_t* __restrict__ cls, i64 r0,
                                                         i64 r1, const i64* __restrict__ loff,
                                                         i64* __restrict__ tp) {
  const i64 i = r0 + (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= r1) return;
  const int32_t c = cls[i];
  tp[i - r0] = loff[c + 1] - loff[c];
}

// one thread per pod: out[poff[i] ...] = L_cls(i) (most pods emit 0-3 pairs)
__global__ __launch_bounds__(TPB) void k_shadow_emit(const int32_t* __restrict__ cls, i64 r0,
                                                     i64 r1, const i64* __restrict__ loff,
                                                     const int2* __restrict__ L,
                                                     const i64* __restrict__ poff,
                                                     int2* __restrict__ out, i64 out_cap,
                                                     const i64* __restrict__ L_total, i64 L_cap) {
  // a wave per 64 consecutive pods, whose pairs are one contiguous range of
  // out: lane q of each 64-pair step finds its pod (the last lane whose
  // offset is <= q: pods with no pairs share the next one's offset) by a
  // binary search over the lanes' offsets, so loads and stores are
  // coalesced (a thread walking its own pod's list wrote 64 streams a wave:
  // 4.2 ms for C5's 33M pairs)
  const int lane = threadIdx.x & 63;
  const i64 wb = r0 + ((i64)blockIdx.x * TPB + threadIdx.x - lane);
  if (wb >= r1) return;
  if (poff[r1 - r0] > out_cap || (L_total && *L_total > L_cap)) return;   // as k_shadow_compact
  const i64 we = min(wb + 64, r1), i = wb + lane;
  const i64 ob = poff[wb - r0], oe = poff[we - r0];
  i64 l0 = 0, o = oe;
  if (i < we) {
    l0 = loff[cls[i]];
    o = poff[i - r0];
  }
  if (oe - ob > (i64)INT32_MAX) {   // (past 2^31 pairs a wave: each lane its own list)
    if (i < we)
      for (i64 k = 0, len = poff[i + 1 - r0] - o; k < len; ++k) out[o + k] = L[l0 + k];
    return;
  }
  const int rel = (int)(o - ob), tot = (int)(oe - ob);
  for (int q0 = 0; q0 < tot; q0 += 64) {
    const int q = q0 + lane;
    int j = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
      if (__shfl(rel, j + s, 64) <= q) j += s;
    const int rj = __shfl(rel, j, 64);
    const i64 lj = __shfl(l0, j, 64);
    if (q < tot) out[ob + q] = L[lj + (q - rj)];
  }
}

// ===========================================================================
// Bit rows -> ascending index lists (the reference's check results are lists
// of pod indices, algorithm.py:4-55).  Up to 4 rows; a row may be inverted
// (all_isolated, system_isolation report the zero bits).  Output rows are
// concatenated; block b of row r writes at boff[r * nb + b].
// ===========================================================================
struct IdxRows {
  const u64* row[4];
  int32_t inv[4];
  i64 W, n, nb;
};

// kano_verify's column tail in one pass, thread per pod j (ca = its column
// class): the column checks expanded from class level (all_isolated /
// all_reachable words), user_crosscheck's cross bit from the group rows
// (cross = MULTI | A2 | (A1 & ~R[g(j)])), the system row from Mc, and per
// block of TPB pods the count of each result row's listed pods.
struct FinishArgs {
  const int32_t* cla;
  i64 n, W, nb;
  const u64* col_or_c;
  const u64* col_nand_c;
  u64* color;
  u64* colnand;
  u64* col_and;
  const int32_t* gid;    // nullable: no crosscheck
  int32_t G;
  const u64* R;
  i64 ldC;
  const u64* multi;
  const u64* A1;
  const u64* A2;
  u64* cross;
  int32_t* err;
  const u64* Mc;         // nullable: no system row
  const int32_t* clr;    // row class of each pod
  i64 sys_row;
  u64* sysrow;
  i64* icnt;             // [r * nb + b], r: reachable, isolated, cross, sys-isolated
  u64* words;            // nullable: this shard's [OR | cross | NAND] words (3 W) for the gather
  // policy_shadow's per-pod pair counts (k_shadow_podcount folded in):
  // tp[i - r0] = loff[c + 1] - loff[c] for the shard's pods (tp nullable)
  const int32_t* rcls;
  const i64* loff;
  i64* tp;
  i64 r0, r1;
};

__device__ __forceinline__ bool mc_bit(const u64* row, int32_t ca) {
  return (row[ca >> 6] >> (ca & 63)) & 1ull;
}

// per-block counts of a row's zero bits (system_isolation's list sizes,
// icnt row 3) from a row of M; all zero when the row is not this shard's
__global__ __launch_bounds__(TPB) void k_row_zero_counts(const u64* __restrict__ row, i64 n,
                                                         i64 W, i64* __restrict__ icnt3) {
  __shared__ i64 sm[4];
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;   // grid covers W * 64
  const bool z = row && j < n && !((row[j >> 6] >> (j & 63)) & 1ull);
  const i64 c = block_sum((i64)z, sm);
  if (threadIdx.x == 0) icnt3[blockIdx.x] = c;
}

__global__ __launch_bounds__(TPB) void k_verify_cols(FinishArgs a) {
  __shared__ i64 sm[4];
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;   // grid covers W * 64
  const bool live = j < a.n;
  if (a.tp && j >= a.r0 && j < a.r1) {
    const int32_t c = a.rcls[j];
    a.tp[j - a.r0] = a.loff[c + 1] - a.loff[c];
  }
  const int32_t ca = live ? a.cla[j] : 0;
  const bool orb = live && mc_bit(a.col_or_c, ca);
  const bool nab = live && mc_bit(a.col_nand_c, ca);
  bool crb = false;
  if (a.gid && live) {
    const int32_t g = a.gid[j];
    bool own = false;
    if (g < 0 || g >= a.G) atomicOr(a.err, 1);
    else own = mc_bit(a.R + (i64)g * a.ldC, ca);
    crb = mc_bit(a.multi, ca) || mc_bit(a.A2, ca) || (mc_bit(a.A1, ca) && !own);
  }
  const bool syb = a.Mc && live && mc_bit(a.Mc + (i64)a.clr[a.sys_row] * a.ldC, ca);
  const u64 wo = __ballot(orb), wn = __ballot(nab), wc = __ballot(crb), ws = __ballot(syb);
  const i64 w = j >> 6;
  if ((threadIdx.x & 63) == 0 && w < a.W) {   // the grid's tail waves hold no word
    a.color[w] = wo;
    a.colnand[w] = wn;
    a.col_and[w] = ~wn & valid_mask(w, a.n);
    if (a.gid) a.cross[w] = wc;
    if (a.Mc) a.sysrow[w] = ws;
    if (a.words) {
      a.words[w] = wo;
      a.words[a.W + w] = wc;
      a.words[2 * a.W + w] = wn;
    }
  }
  const i64 c0 = block_sum((i64)(live && !nab), sm);
  const i64 c1 = block_sum((i64)(live && !orb), sm);
  const i64 c2 = block_sum((i64)crb, sm);
  const i64 c3 = block_sum((i64)(a.Mc && live && !syb), sm);
  if (threadIdx.x == 0) {
    a.icnt[blockIdx.x] = c0;
    a.icnt[a.nb + blockIdx.x] = c1;
    a.icnt[2 * a.nb + blockIdx.x] = c2;
    a.icnt[3 * a.nb + blockIdx.x] = c3;
  }
}

// Up to five device -> host copies sized on the device (kano_verify's
// tail): job y's element count is the sum of cnt[0..ncnt), its destination
// offset (elements) the sum of off[0..noff); a job past its capacity copies
// nothing (the host sees the counts and takes the sized path).
struct CopySeg {
  const char* src;
  char* dst;
  const u64* cnt;
  int ncnt;
  const u64* off;
  int noff;
  int esize;
  i64 cap;
};
struct CopySegs {
  CopySeg j[5];
};
__global__ __launch_bounds__(TPB) void k_copy_segs(CopySegs jobs) {
  const CopySeg a = jobs.j[blockIdx.y];
  i64 cnt = 0, off = 0;
  for (int q = 0; q < a.ncnt; ++q) cnt += (i64)a.cnt[q];
  for (int q = 0; q < a.noff; ++q) off += (i64)a.off[q];
  if (cnt + off > a.cap) return;                   // block-uniform
  const i64 bytes = cnt * a.esize;
  char* dst = a.dst + off * a.esize;
  const i64 stride = (i64)gridDim.x * TPB;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const i64 n16 = bytes >> 4;
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (i64 k = (i64)blockIdx.x * TPB + threadIdx.x; k < n16; k += stride) d[k] = src[k];
    const int ntail = (int)((bytes & 15) >> 2);
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail)
      reinterpret_cast<uint32_t*>(dst + n16 * 16)[threadIdx.x] =
          reinterpret_cast<const uint32_t*>(a.src + n16 * 16)[threadIdx.x];
  } else {
    // a 4-byte aligned destination (a list after another list's odd count):
    // up to 3 words alone, then 16-byte stores to the host (PCIe writes of 4
    // bytes per lane run at a fraction of the link), the tail alone
    const i64 n4 = bytes >> 2;
    const int head = (int)min<i64>(n4, (16 - (i64)(reinterpret_cast<uintptr_t>(dst) & 15)) >> 2);
    const uint32_t* __restrict__ src = reinterpret_cast<const uint32_t*>(a.src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    if (blockIdx.x == 0 && (int)threadIdx.x < head) d[threadIdx.x] = src[threadIdx.x];
    const i64 n16 = (n4 - head) >> 2;
    uint4* d16 = reinterpret_cast<uint4*>(d + head);
    const uint32_t* s4 = src + head;
    for (i64 k = (i64)blockIdx.x * TPB + threadIdx.x; k < n16; k += stride)
      d16[k] = make_uint4(s4[4 * k], s4[4 * k + 1], s4[4 * k + 2], s4[4 * k + 3]);
    const i64 t0 = head + 4 * n16;
    if (blockIdx.x == 0 && (i64)threadIdx.x < n4 - t0) d[t0 + threadIdx.x] = src[t0 + threadIdx.x];
  }
}

// Row shards combined (kano_verify_combine): thread per pod j, the gathered
// [OR | cross | NAND] words of nr shards (rank-major, 3 W words each) OR-ed
// (all_isolated = no shard has a row reaching j, all_reachable = no shard
// has a row missing j, user_crosscheck = some shard has a cross row), and the
// per-block counts of result rows 0..2 (row 3, the system row, stays local).
__global__ __launch_bounds__(TPB) void k_combine_cols(const u64* __restrict__ g, int32_t nr, i64 n,
                                                      i64 W, i64 nb, u64* __restrict__ color,
                                                      u64* __restrict__ colnand,
                                                      u64* __restrict__ col_and,
                                                      u64* __restrict__ cross,
                                                      i64* __restrict__ icnt) {
  __shared__ i64 sm[4];
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;   // grid covers W * 64
  const i64 w = j >> 6;
  u64 o = 0, c = 0, na = 0;
  if (w < W) {
    for (int32_t r = 0; r < nr; ++r) {
      const u64* s = g + (i64)r * 3 * W;
      o |= s[w];
      c |= s[W + w];
      na |= s[2 * W + w];
    }
    const u64 vm = valid_mask(w, n);
    o &= vm;
    c &= vm;
    na &= vm;
    if ((threadIdx.x & 63) == 0) {
      color[w] = o;
      colnand[w] = na;
      col_and[w] = ~na & vm;
      if (cross) cross[w] = c;
    }
  }
  const bool live = j < n;
  const int bit = (int)(j & 63);
  const bool orb = (o >> bit) & 1ull, nab = (na >> bit) & 1ull;
  const bool crb = cross && ((c >> bit) & 1ull);
  const i64 c0 = block_sum((i64)(live && !nab), sm);
  const i64 c1 = block_sum((i64)(live && !orb), sm);
  const i64 c2 = block_sum((i64)(live && crb), sm);
  if (threadIdx.x == 0) {
    icnt[blockIdx.x] = c0;
    icnt[nb + blockIdx.x] = c1;
    icnt[2 * nb + blockIdx.x] = c2;
  }
}

// thread per pod: row r's listed pods in ascending order; row r starts after
// the totals of rows < r (rowtot: 4 size slots)
__global__ __launch_bounds__(TPB) void k_idx_write(IdxRows a, const i64* __restrict__ boff,
                                                   i64 ldo, const u64* __restrict__ rowtot,
                                                   int32_t* __restrict__ idx) {
  __shared__ i64 sm[4];
  const int r = blockIdx.y;
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  bool bit = false;
  if (a.row[r] && j < a.n) bit = ((a.row[r][j >> 6] >> (j & 63)) & 1ull) != (a.inv[r] != 0);
  i64 row0 = 0;
  for (int q = 0; q < r; ++q) row0 += (i64)rowtot[q];
  i64 tot;
  const i64 pos = block_excl_scan((i64)bit, sm, tot) + row0 + boff[r * ldo + blockIdx.x];
  if (bit) idx[pos] = (int32_t)j;
}

}  // namespace kano
