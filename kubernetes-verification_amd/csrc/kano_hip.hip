// kano_hip.hip -- MI355X (gfx950) engine for the Kano reachability matrix and
// checks.  C ABI: include/kano_hip.h.  Design: DESIGN.md.
//
// Reference being replaced (qiyueyao/Kubernetes-verification, kano_py/):
//   ReachabilityMatrix.build_matrix   kano/model.py:125-165
//   matrix accessors                  kano/model.py:167-184
//   all_reachable / all_isolated      kano/algorithm.py:4-17
//   user_crosscheck                   kano/algorithm.py:20-42
//   system_isolation                  kano/algorithm.py:45-55
//   policy_shadow / policy_conflict   kano/algorithm.py:58-100
//
// Data flow of one build (all on the context stream):
//   classes   pods hashed on the values of every key a working selector
//             references; pods of one class have identical S(i), hence
//             identical matrix rows (model.py:150-161 depends on nothing else)
//   select    SelT[pb][c]: bit q = policy 64*pb+q selects class c
//   allow     Allow[p][w]: the allow set of policy p as a bit row over pods,
//             plus the same set as a sorted pod list (CSR over policies)
//   rows      one work item = (class, <=CH member pods, column chunk): the
//             class row is rebuilt in LDS from its policies' allow sets
//             (scatter of sparse lists, OR of dense rows) and streamed to the
//             member rows of M; column OR / NAND for all_isolated /
//             all_reachable are folded in by the first member chunk
//   heavy     classes whose rebuild would cost more than their writes are
//             built once (int8 MFMA contraction or wide OR) into the row of
//             their representative and copied to the other members.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kano_hip.h"

typedef unsigned long long u64;
typedef long long i64;

namespace {

constexpr int TPB = 256;              // threads per block for every kernel here
constexpr int SCAN_ITEMS = 8;         // elements per thread in the scan tiles
constexpr int SCAN_TILE = TPB * SCAN_ITEMS;
constexpr int MAX_CWW = 8192;         // column-chunk width in words (64 KB of LDS)

// ---------------------------------------------------------------------------
// wave / block primitives
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// Exclusive scan over a 256-thread block.  smem: >= 4 elements.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* smem, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) smem[wid] = inc;
  __syncthreads();
  T pre = 0;
  for (int w = 0; w < wid; ++w) pre += smem[w];
  total = smem[0] + smem[1] + smem[2] + smem[3];
  __syncthreads();
  return pre + inc - v;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* smem) {
  T tot;
  (void)block_excl_scan(v, smem, tot);
  return tot;
}

// ---------------------------------------------------------------------------
// device-wide exclusive scan: out[0..n] with out[n] = total
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout>
__global__ __launch_bounds__(TPB) void k_scan_sums(const Tin* __restrict__ in, i64 n,
                                                   Tout* __restrict__ sums) {
  __shared__ Tout sm[4];
  const i64 base = (i64)blockIdx.x * SCAN_TILE + (i64)threadIdx.x * SCAN_ITEMS;
  Tout s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (base + k < n) s += (Tout)in[base + k];
  Tout tot = block_sum(s, sm);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(TPB) void k_scan_tiles(const Tin* __restrict__ in, i64 n,
                                                    const Tout* __restrict__ tile_off,
                                                    Tout* __restrict__ out) {
  __shared__ Tout sm[4];
  const i64 base = (i64)blockIdx.x * SCAN_TILE + (i64)threadIdx.x * SCAN_ITEMS;
  Tout v[SCAN_ITEMS];
  Tout s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = (base + k < n) ? (Tout)in[base + k] : (Tout)0;
    s += v[k];
  }
  Tout tot;
  Tout pre = block_excl_scan(s, sm, tot) + (tile_off ? tile_off[blockIdx.x] : (Tout)0);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < n) out[base + k] = pre;
    pre += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == TPB - 1) out[n] = pre;
}

// ---------------------------------------------------------------------------
// row classes: hash the selector-key values of every pod
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hmix(uint32_t h, uint32_t v) {
  v *= 0xcc9e2d51u;
  v = (v << 15) | (v >> 17);
  v *= 0x1b873593u;
  h ^= v;
  h = (h << 13) | (h >> 19);
  return h * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t hfin(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

__global__ __launch_bounds__(TPB) void k_class_insert(const int32_t* __restrict__ pv, i64 n,
                                                      const int32_t* __restrict__ ckeys, int KS,
                                                      int32_t* table, uint32_t tmask,
                                                      int32_t* __restrict__ slot_of) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  uint32_t h = 0x9747b28cu;
  for (int k = 0; k < KS; ++k) h = hmix(h, (uint32_t)pv[(i64)ckeys[k] * n + i]);
  uint32_t s = hfin(h) & tmask;
  for (;;) {
    int32_t cur = __hip_atomic_load(&table[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur < 0) {
      int32_t prev = atomicCAS(&table[s], -1, (int32_t)i);
      if (prev < 0) { slot_of[i] = (int32_t)s; return; }
      cur = prev;
    }
    bool eq = true;
    for (int k = 0; k < KS; ++k) {
      const int32_t* col = pv + (i64)ckeys[k] * n;
      if (col[cur] != col[i]) { eq = false; break; }
    }
    if (eq) { slot_of[i] = (int32_t)s; return; }
    s = (s + 1) & tmask;
  }
}

__global__ __launch_bounds__(TPB) void k_class_min(const int32_t* __restrict__ slot_of, i64 n,
                                                   int32_t* smin) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i < n) atomicMin(&smin[slot_of[i]], (int32_t)i);
}

__global__ __launch_bounds__(TPB) void k_class_flag(const int32_t* __restrict__ slot_of, i64 n,
                                                    const int32_t* __restrict__ smin,
                                                    int32_t* __restrict__ flag) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i < n) flag[i] = (smin[slot_of[i]] == (int32_t)i) ? 1 : 0;
}

__global__ __launch_bounds__(TPB) void k_class_assign(const int32_t* __restrict__ slot_of, i64 n,
                                                      const int32_t* __restrict__ smin,
                                                      const int32_t* __restrict__ cid,
                                                      int32_t* __restrict__ cls,
                                                      int32_t* __restrict__ rep) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const int32_t r = smin[slot_of[i]];
  const int32_t c = cid[r];
  cls[i] = c;
  if (r == (int32_t)i) rep[c] = (int32_t)i;
}

// member lists of the classes, restricted to this shard's rows [r0, r1)
__global__ __launch_bounds__(TPB) void k_member_count(const int32_t* __restrict__ cls, i64 r0,
                                                      i64 r1, int32_t* mcnt) {
  const i64 i = r0 + (i64)blockIdx.x * TPB + threadIdx.x;
  if (i < r1) atomicAdd(&mcnt[cls[i]], 1);
}

__global__ __launch_bounds__(TPB) void k_member_fill(const int32_t* __restrict__ cls, i64 r0,
                                                     i64 r1, const int32_t* __restrict__ moff,
                                                     int32_t* mcur, int32_t* __restrict__ mem) {
  const i64 i = r0 + (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= r1) return;
  const int32_t c = cls[i];
  mem[moff[c] + atomicAdd(&mcur[c], 1)] = (int32_t)i;
}

__global__ __launch_bounds__(TPB) void k_class_vals(const int32_t* __restrict__ pv, i64 n,
                                                    const int32_t* __restrict__ ckeys, int KS,
                                                    const int32_t* __restrict__ rep, i64 U,
                                                    int32_t* __restrict__ cval) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  const int32_t r = rep[c];
  for (int k = 0; k < KS; ++k) cval[(i64)k * U + c] = pv[(i64)ckeys[k] * n + r];
}

// ---------------------------------------------------------------------------
// selector evaluation
//   sel_p(c) = AND over working-selector terms (slot, v): cval[slot][c] == v
//   (kano_py/kano/model.py:95-102 + 142-147 restated on interned values)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void k_sel_eval(const int32_t* __restrict__ cval, i64 U, i64 P,
                                                  const i64* __restrict__ soff,
                                                  const int32_t* __restrict__ sslot,
                                                  const int32_t* __restrict__ sval,
                                                  u64* __restrict__ selT) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  const i64 pb = blockIdx.y;
  const i64 p0 = pb * 64;
  const int qn = (int)min((i64)64, P - p0);
  const bool live = c < U;
  u64 word = 0;
  for (int q = 0; q < qn; ++q) {
    const i64 p = p0 + q;
    const i64 t0 = soff[p], t1 = soff[p + 1];
    bool ok = live;
    for (i64 t = t0; t < t1 && ok; ++t) ok = cval[(i64)sslot[t] * U + c] == sval[t];
    word |= (u64)ok << q;
  }
  if (live) selT[pb * U + c] = word;
}

// |S(c)| for every class, plus max over classes with local members
__global__ __launch_bounds__(TPB) void k_sel_count(const u64* __restrict__ selT, i64 U, i64 PB,
                                                   const int32_t* __restrict__ mcnt,
                                                   int32_t* __restrict__ scnt, int32_t* maxs) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  int s = 0;
  for (i64 pb = 0; pb < PB; ++pb) s += __popcll(selT[pb * U + c]);
  scnt[c] = s;
  if (mcnt[c] > 0) atomicMax(maxs, s);
}

__global__ __launch_bounds__(TPB) void k_sel_fill(const u64* __restrict__ selT, i64 U, i64 PB,
                                                  const i64* __restrict__ soffc,
                                                  int32_t* __restrict__ slist) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  i64 pos = soffc[c];
  for (i64 pb = 0; pb < PB; ++pb) {
    u64 w = selT[pb * U + c];
    while (w) {
      const int q = __builtin_ctzll(w);
      slist[pos++] = (int32_t)(pb * 64 + q);
      w &= w - 1;
    }
  }
}

// allow side over pods: one wave = one 64-pod word, ballot per policy.
// Pod values of the referenced columns are staged in LDS (ncols <= 32).
template <bool STAGE>
__global__ __launch_bounds__(TPB) void k_allow_eval(const int32_t* __restrict__ pv, i64 n, int ncols,
                                                    i64 W, i64 P, int pch,
                                                    const i64* __restrict__ aoff,
                                                    const int32_t* __restrict__ acol,
                                                    const int32_t* __restrict__ aval,
                                                    u64* __restrict__ allow, i64 ldA) {
  __shared__ int32_t sv[STAGE ? 32 * TPB : 1];
  const int lane = threadIdx.x & 63;
  const i64 w = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const i64 i = w * 64 + lane;
  const bool valid = (w < W) && (i < n);
  if (STAGE) {
    for (int k = 0; k < ncols; ++k) sv[k * TPB + threadIdx.x] = valid ? pv[(i64)k * n + i] : -1;
    __syncthreads();
  }
  if (w >= W) return;
  const i64 p0 = (i64)blockIdx.y * pch;
  const i64 p1 = min(P, p0 + pch);
  for (i64 p = p0; p < p1; ++p) {
    const i64 t0 = aoff[p], t1 = aoff[p + 1];
    bool ok = valid;
    for (i64 t = t0; t < t1; ++t) {
      const int32_t col = acol[t];
      const int32_t v = STAGE ? sv[col * TPB + threadIdx.x] : (valid ? pv[(i64)col * n + i] : -1);
      ok = ok && (v == aval[t]);
    }
    const u64 b = __ballot(ok);
    if (lane == 0) allow[p * ldA + w] = b;
  }
}

// block per policy: |allow_p|
__global__ __launch_bounds__(TPB) void k_allow_count(const u64* __restrict__ allow, i64 W, i64 ldA,
                                                     int32_t* __restrict__ acnt) {
  __shared__ int sm[4];
  const i64 p = blockIdx.x;
  int s = 0;
  for (i64 w = threadIdx.x; w < W; w += TPB) s += __popcll(allow[p * ldA + w]);
  s = block_sum(s, sm);
  if (threadIdx.x == 0) acnt[p] = s;
}

// block per policy: ascending pod list of allow_p
__global__ __launch_bounds__(TPB) void k_allow_fill(const u64* __restrict__ allow, i64 W, i64 ldA,
                                                    const i64* __restrict__ aloff,
                                                    int32_t* __restrict__ alist) {
  __shared__ int sm[4];
  const i64 p = blockIdx.x;
  i64 base = aloff[p];
  for (i64 w0 = 0; w0 < W; w0 += TPB) {
    const i64 w = w0 + threadIdx.x;
    u64 v = (w < W) ? allow[p * ldA + w] : 0ull;
    int tot;
    i64 pos = base + block_excl_scan((int)__popcll(v), sm, tot);
    while (v) {
      alist[pos++] = (int32_t)(w * 64 + __builtin_ctzll(v));
      v &= v - 1;
    }
    base += tot;
  }
}

// work items per class = ceil(local members / CH)
__global__ __launch_bounds__(TPB) void k_wi_count(const int32_t* __restrict__ mcnt, i64 U, int ch,
                                                  int32_t* __restrict__ wicnt) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c < U) wicnt[c] = (mcnt[c] + ch - 1) / ch;
}

__device__ __forceinline__ i64 upper_bound_i32(const int32_t* a, i64 n, i64 key) {
  i64 lo = 0, hi = n;
  while (lo < hi) {
    const i64 mid = (lo + hi) >> 1;
    if ((i64)a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ i64 lower_bound_i32(const int32_t* a, i64 n, i64 key) {
  i64 lo = 0, hi = n;
  while (lo < hi) {
    const i64 mid = (lo + hi) >> 1;
    if ((i64)a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ u64 valid_mask(i64 w, i64 n) {
  const i64 lo = w * 64;
  if (lo + 64 <= n) return ~0ull;
  if (lo >= n) return 0ull;
  return (1ull << (n - lo)) - 1ull;
}

// ---------------------------------------------------------------------------
// rows: the reachability matrix (kano_py/kano/model.py:158-160)
// ---------------------------------------------------------------------------
struct RowsArgs {
  const int32_t* wioff;  // U+1
  i64 U;
  const i64* soffc;      // U+1
  const int32_t* slist;
  const int32_t* acnt;
  const i64* aloff;
  const int32_t* alist;
  const u64* allow;
  i64 ldA;
  const int32_t* moff;   // U+1
  const int32_t* mem;
  const uint8_t* heavy;  // U, 1 = row prebuilt at M[first member]
  u64* M;
  i64 ldM;
  i64 r0;
  i64 n, W;
  int ch;
  int cww;
  u64* color;
  u64* colnand;
};

__global__ __launch_bounds__(TPB) void k_rows(RowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) u64 row[];
  const i64 b = blockIdx.x;
  const i64 c = upper_bound_i32(a.wioff, a.U + 1, b) - 1;
  if (c < 0 || c >= a.U) return;
  const i64 chunk = b - a.wioff[c];
  const i64 base = (i64)blockIdx.y * a.cww;
  const i64 ldw = a.ldM;                 // words incl. padding, even
  const int nw = (int)min((i64)a.cww, ldw - base);
  if (nw <= 0) return;
  const int32_t m_begin = a.moff[c], m_end = a.moff[c + 1];
  const int32_t m0 = m_begin + (int32_t)(chunk * a.ch);
  const int32_t m1 = min(m_end, m0 + a.ch);

  if (a.heavy && a.heavy[c]) {
    // row prebuilt at the first member; copy it (skip the source itself)
    const u64* src = a.M + (i64)(a.mem[m_begin] - a.r0) * ldw + base;
    for (int w = threadIdx.x * 2; w < nw; w += TPB * 2)
      *(ulonglong2*)&row[w] = *(const ulonglong2*)&src[w];
    __syncthreads();
  } else {
    for (int w = threadIdx.x; w < nw; w += TPB) row[w] = 0ull;
    __syncthreads();
    const i64 s0 = a.soffc[c], s1 = a.soffc[c + 1];
    const i64 col_lo = base * 64, col_hi = (base + nw) * 64;
    for (i64 e = s0; e < s1; ++e) {
      const int32_t p = a.slist[e];
      const i64 cnt = a.acnt[p];
      if (cnt == 0) continue;
      if (cnt > (i64)nw) {
        const u64* ar = a.allow + (i64)p * a.ldA + base;
        const int lim = (int)min((i64)nw, a.W - base);
        for (int w = threadIdx.x; w < lim; w += TPB) {
          const u64 v = ar[w];
          if (v) atomicOr(&row[w], v);
        }
      } else {
        const int32_t* L = a.alist + a.aloff[p];
        i64 lo = 0, hi = cnt;
        if (base > 0 || col_hi < a.n) {
          lo = lower_bound_i32(L, cnt, col_lo);
          hi = lower_bound_i32(L, cnt, col_hi);
        }
        for (i64 k = lo + threadIdx.x; k < hi; k += TPB) {
          const int32_t j = L[k];
          atomicOr(&row[(j >> 6) - base], 1ull << (j & 63));
        }
      }
    }
    __syncthreads();
  }
  const bool skip_first = a.heavy && a.heavy[c];
  for (int32_t m = m0; m < m1; ++m) {
    if (skip_first && m == m_begin) continue;
    u64* dst = a.M + (i64)(a.mem[m] - a.r0) * ldw + base;
    for (int w = threadIdx.x * 2; w < nw; w += TPB * 2)
      *(ulonglong2*)&dst[w] = *(const ulonglong2*)&row[w];
  }
  if (chunk == 0 && a.color) {
    for (int w = threadIdx.x; w < nw; w += TPB) {
      const i64 gw = base + w;
      if (gw >= a.W) break;
      const u64 v = row[w];
      const u64 vm = valid_mask(gw, a.n);
      if (v) atomicOr(&a.color[gw], v);
      const u64 nv = ~v & vm;
      if (nv && __hip_atomic_load(&a.colnand[gw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != vm)
        atomicOr(&a.colnand[gw], nv);
    }
  }
}

// heavy classes, bitwise path: row = OR over S(c) of dense allow rows.
// grid (heavy classes, column blocks of 512 words); the block's 4 waves split
// the policy list and reduce through LDS.
__global__ __launch_bounds__(TPB) void k_heavy_or(const int32_t* __restrict__ hlist,
                                                  const i64* __restrict__ soffc,
                                                  const int32_t* __restrict__ slist,
                                                  const u64* __restrict__ allow, i64 ldA, i64 W,
                                                  const int32_t* __restrict__ moff,
                                                  const int32_t* __restrict__ mem,
                                                  u64* __restrict__ M, i64 ldM, i64 r0) {
  __shared__ __attribute__((aligned(16))) u64 red[4][128];
  const int32_t c = hlist[blockIdx.x];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const i64 wbase = (i64)blockIdx.y * 128;
  const i64 s0 = soffc[c], s1 = soffc[c + 1];
  const i64 w0 = wbase + lane * 2;
  u64 acc0 = 0, acc1 = 0;
  if (w0 < W) {
    for (i64 e = s0 + wid; e < s1; e += 4) {
      const u64* ar = allow + (i64)slist[e] * ldA;
      const ulonglong2 v = *(const ulonglong2*)&ar[w0];
      acc0 |= v.x;
      acc1 |= v.y;
    }
  }
  red[wid][lane * 2] = acc0;
  red[wid][lane * 2 + 1] = acc1;
  __syncthreads();
  if (threadIdx.x < 128) {
    const i64 w = wbase + threadIdx.x;
    if (w < ldM) {
      u64 v = red[0][threadIdx.x] | red[1][threadIdx.x] | red[2][threadIdx.x] | red[3][threadIdx.x];
      if (w >= W) v = 0;
      M[(i64)(mem[moff[c]] - r0) * ldM + w] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// int8 MFMA contraction for heavy classes (dense path):
//   C[h][j] = sum_p Sel[h][p] * Allow[p][j]  (i8 x i8 -> i32), M bit = C > 0.
// A = class-major selector bits (selT), B = pod-major allow bits (allowT),
// both bit-packed in HBM and expanded to 0/1 bytes in registers.
// v_mfma_i32_32x32x32_i8: lane l supplies A[l&31][16*(l>>5) .. +15] and
// B[16*(l>>5) .. +15][l&31]; C/D reg g of lane l = row (g&3)+8*(g>>2)+4*(l>>5),
// col l&31 (cdna_hip_programming.md §3; map checked by tests/test_gpu_parity).
// One wave computes all heavy rows (up to 32*HT) x 32 pod columns.
// ---------------------------------------------------------------------------
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t spread4(uint32_t b4) {
  // 4 bits -> 4 bytes of 0/1
  return ((b4 & 1u)) | ((b4 & 2u) << 7) | ((b4 & 4u) << 14) | ((b4 & 8u) << 21);
}
__device__ __forceinline__ i32x4 expand16(uint32_t b16) {
  i32x4 r;
  r[0] = (int32_t)spread4(b16 & 15u);
  r[1] = (int32_t)spread4((b16 >> 4) & 15u);
  r[2] = (int32_t)spread4((b16 >> 8) & 15u);
  r[3] = (int32_t)spread4((b16 >> 12) & 15u);
  return r;
}

template <int HT>
__global__ __launch_bounds__(TPB) void k_heavy_mfma(const u64* __restrict__ selT, i64 U,
                                                    const int32_t* __restrict__ hlist, int H,
                                                    const u64* __restrict__ allowT, i64 n, i64 PB,
                                                    const int32_t* __restrict__ moff,
                                                    const int32_t* __restrict__ mem,
                                                    uint32_t* __restrict__ M32, i64 ldM, i64 r0) {
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const i64 jt = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);  // 32-column tile
  const i64 j = jt * 32 + l32;
  if (jt * 32 >= n) return;
  int32_t hc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    const int h = t * 32 + l32;
    hc[t] = h < H ? hlist[h] : -1;
  }
  i32x16 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[t][g] = 0;
  for (i64 pb = 0; pb < PB; ++pb) {
    const u64 bw = j < n ? allowT[pb * n + j] : 0ull;
    u64 aw[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) aw[t] = hc[t] >= 0 ? selT[pb * U + hc[t]] : 0ull;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int sh = ks * 32 + half * 16;
      const i32x4 bfrag = expand16((uint32_t)(bw >> sh) & 0xffffu);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const i32x4 afrag = expand16((uint32_t)(aw[t] >> sh) & 0xffffu);
        acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag, bfrag, acc[t], 0, 0, 0);
      }
    }
  }
  // epilogue: threshold, pack 32 columns per row with ballots, store 32-bit halves
#pragma unroll
  for (int t = 0; t < HT; ++t) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const u64 bal = __ballot(acc[t][g] > 0);
      const int rlo = t * 32 + (g & 3) + 8 * (g >> 2);  // rows rlo (lanes 0-31) and rlo+4
      if (lane == 0 || lane == 32) {
        const int r = rlo + (lane == 32 ? 4 : 0);
        const uint32_t bits = lane == 0 ? (uint32_t)bal : (uint32_t)(bal >> 32);
        if (r < H) {
          const int32_t c = hlist[r];
          const i64 row = (i64)mem[moff[c]] - r0;
          M32[row * ldM * 2 + jt] = bits;
        }
      }
    }
  }
}

// pod-major allow bits: allowT[pb][j], bit q = policy 64*pb+q allows pod j
__global__ __launch_bounds__(TPB) void k_allow_transpose(const u64* __restrict__ allow, i64 ldA,
                                                         i64 W, i64 P, i64 n,
                                                         u64* __restrict__ allowT) {
  // block: 4 waves, each one 64-pod word w for one policy block pb
  const int lane = threadIdx.x & 63;
  const i64 w = (i64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const i64 pb = blockIdx.y;
  if (w >= W) return;
  const i64 p = pb * 64 + lane;
  const u64 mine = p < P ? allow[p * ldA + w] : 0ull;  // lane q holds policy q's word
  u64 out = 0;
  for (int b = 0; b < 64; ++b) {
    const u64 bal = __ballot((mine >> b) & 1ull);
    if (lane == b) out = bal;
  }
  const i64 j = w * 64 + lane;
  if (j < n) allowT[pb * n + j] = out;
}

// heavy selection: a class is heavy when rebuilding its row per member chunk
// would cost more than a copy of it, i.e. sum over S(c) of min(|allow_p|, W)
// exceeds the row width, and it has more than one member chunk.
__global__ __launch_bounds__(TPB) void k_heavy_mark(const i64* __restrict__ soffc,
                                                    const int32_t* __restrict__ slist,
                                                    const int32_t* __restrict__ acnt,
                                                    const int32_t* __restrict__ mcnt, i64 U, i64 W,
                                                    int ch, int force, uint8_t* __restrict__ heavy,
                                                    int32_t* hcount, int32_t* hlist) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  uint8_t hv = 0;
  if (mcnt[c] > 0) {
    i64 cost = 0;
    for (i64 e = soffc[c]; e < soffc[c + 1]; ++e) cost += min((i64)acnt[slist[e]], W);
    if (force == 1) hv = 0;
    else if (force == 2) hv = (soffc[c + 1] > soffc[c]) ? 1 : 0;
    else hv = (mcnt[c] > ch && cost > 4 * W) ? 1 : 0;
  }
  heavy[c] = hv;
  if (hv) hlist[atomicAdd(hcount, 1)] = (int32_t)c;
}

// ---------------------------------------------------------------------------
// checks
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void k_col_final(const u64* __restrict__ color,
                                                   const u64* __restrict__ colnand, i64 W, i64 n,
                                                   u64* __restrict__ col_and) {
  const i64 w = (i64)blockIdx.x * TPB + threadIdx.x;
  if (w < W) col_and[w] = ~colnand[w] & valid_mask(w, n);
}

// one byte per column: [or | cross | nand]
__global__ __launch_bounds__(TPB) void k_unpack_flags(const u64* __restrict__ words, i64 n,
                                                      uint8_t* __restrict__ out) {
  const i64 j = (i64)blockIdx.x * TPB + threadIdx.x;
  if (j < n) out[j] = (uint8_t)((words[j >> 6] >> (j & 63)) & 1ull);
}

// crosscheck step 1: group range of the local members of every class
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

// step 2: R[g] |= class rows of single-group classes, MULTI |= multi-group rows
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

// step 3: A1 |= R[g]; A2 |= R[g] & (bits already set by another group)
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

// step 4: own[j] = R[gid(j)][j]
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

// getcol: bit r-r0 = M[r][j]
__global__ __launch_bounds__(TPB) void k_get_col(const u64* __restrict__ M, i64 ldM, i64 rows,
                                                 i64 j, u64* __restrict__ out) {
  const i64 r = (i64)blockIdx.x * TPB + threadIdx.x;
  const bool bit = r < rows && ((M[r * ldM + (j >> 6)] >> (j & 63)) & 1ull);
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && r < rows) out[r >> 6] = bal;
}

// working_select_set of policy p over all pods
__global__ __launch_bounds__(TPB) void k_sel_row(const u64* __restrict__ selT, i64 U,
                                                 const int32_t* __restrict__ cls, i64 n, i64 p,
                                                 u64* __restrict__ out) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  const bool bit = i < n && ((selT[(p >> 6) * U + cls[i]] >> (p & 63)) & 1ull);
  const u64 bal = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && i < n) out[i >> 6] = bal;
}

// ---------------------------------------------------------------------------
// policy_shadow (kano_py/kano/algorithm.py:58-80) on row classes:
//   pair (a, b) of S(c) positions, a != b:  flag = allow_{S[b]} subset of allow_{S[a]}
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void k_shadow_sq(const i64* __restrict__ soffc,
                                                   const int32_t* __restrict__ mcnt, i64 U,
                                                   i64* __restrict__ sq) {
  const i64 c = (i64)blockIdx.x * TPB + threadIdx.x;
  if (c >= U) return;
  const i64 s = soffc[c + 1] - soffc[c];
  sq[c] = mcnt[c] > 0 ? s * s : 0;
}

__device__ __forceinline__ bool subset_of(int32_t k, int32_t j, const int32_t* acnt,
                                          const i64* aloff, const int32_t* alist,
                                          const u64* allow, i64 ldA) {
  const int32_t ck = acnt[k];
  if (ck == 0) return true;
  if (ck > acnt[j]) return false;
  const int32_t* L = alist + aloff[k];
  const u64* aj = allow + (i64)j * ldA;
  for (int32_t e = 0; e < ck; ++e) {
    const int32_t x = L[e];
    if (!((aj[x >> 6] >> (x & 63)) & 1ull)) return false;
  }
  return true;
}

__global__ __launch_bounds__(TPB) void k_shadow_test(const i64* __restrict__ soffc,
                                                     const int32_t* __restrict__ slist,
                                                     const int32_t* __restrict__ mcnt,
                                                     const i64* __restrict__ pfoff,
                                                     const int32_t* __restrict__ acnt,
                                                     const i64* __restrict__ aloff,
                                                     const int32_t* __restrict__ alist,
                                                     const u64* __restrict__ allow, i64 ldA,
                                                     uint8_t* __restrict__ flags,
                                                     i64* __restrict__ T) {
  __shared__ i64 sm[4];
  const i64 c = blockIdx.x;
  if (mcnt[c] == 0) {
    if (threadIdx.x == 0) T[c] = 0;
    return;
  }
  const i64 s0 = soffc[c];
  const i64 s = soffc[c + 1] - s0;
  const i64 ss = s * s;
  i64 cnt = 0;
  for (i64 t = threadIdx.x; t < ss; t += TPB) {
    const i64 a = t / s, b = t - a * s;
    uint8_t f = 0;
    if (a != b) {
      const int32_t j = slist[s0 + a], k = slist[s0 + b];
      f = (j != k) && subset_of(k, j, acnt, aloff, alist, allow, ldA);
    }
    flags[pfoff[c] + t] = f;
    cnt += f;
  }
  cnt = block_sum(cnt, sm);
  if (threadIdx.x == 0) T[c] = cnt;
}

__global__ __launch_bounds__(TPB) void k_shadow_compact(const i64* __restrict__ soffc,
                                                        const int32_t* __restrict__ slist,
                                                        const i64* __restrict__ pfoff,
                                                        const uint8_t* __restrict__ flags,
                                                        const i64* __restrict__ loff,
                                                        int2* __restrict__ L) {
  __shared__ i64 sm[4];
  const i64 c = blockIdx.x;
  i64 out = loff[c];
  if (loff[c + 1] == out) return;
  const i64 s0 = soffc[c];
  const i64 s = soffc[c + 1] - s0;
  const i64 ss = s * s;
  for (i64 t0 = 0; t0 < ss; t0 += TPB) {
    const i64 t = t0 + threadIdx.x;
    const i64 f = (t < ss) ? flags[pfoff[c] + t] : 0;
    i64 tot;
    const i64 pos = out + block_excl_scan(f, sm, tot);
    if (f) {
      const i64 a = t / s, b = t - a * s;
      L[pos] = make_int2(slist[s0 + a], slist[s0 + b]);
    }
    out += tot;
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

// one wave per pod: out[poff[i] ...] = L_cls(i)
__global__ __launch_bounds__(TPB) void k_shadow_emit(const int32_t* __restrict__ cls, i64 r0,
                                                     i64 r1, const i64* __restrict__ loff,
                                                     const int2* __restrict__ L,
                                                     const i64* __restrict__ poff,
                                                     int2* __restrict__ out) {
  const i64 i = r0 + (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (i >= r1) return;
  const int lane = threadIdx.x & 63;
  const int32_t c = cls[i];
  const i64 l0 = loff[c], len = loff[c + 1] - l0;
  const i64 o = poff[i - r0];
  for (i64 k = lane; k < len; k += 64) out[o + k] = L[l0 + k];
}

}  // namespace

// ===========================================================================
// context
// ===========================================================================
struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct kano_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;

  i64 n = 0, W = 0, ldM = 0, P = 0, PB = 0;
  int ncols = 0, KS = 0;
  i64 r0 = 0, r1 = -1;
  bool have_pods = false, have_pols = false, built = false;
  i64 U = 0, nnz_sel = 0, nnz_alw = 0, wi_total = 0, heavy_count = 0;
  int max_sel = 0;
  int ch = 16;
  bool cols_valid = false;   // color/colnand reflect M (false after set_bit)
  bool rows_dirty = false;   // set_bit happened: classes no longer describe M
  bool lists_mode = false;   // kano_shadow_lists context: no matrix
  bool rows_timed = false;   // ev[7]..ev[8] bracket the last k_rows launch

  // host copies of the policy CSRs (for the class-key remap)
  std::vector<int32_t> ckeys;

  DBuf pv, ckeys_d, soff, sslot, sval, aoff, acol, aval;
  DBuf table, slot_of, smin, flag, cid, cls, rep, mcnt, moff, mcur, mem, cval;
  DBuf selT, scnt, soffc, slist, maxs;
  DBuf allow, acnt, aloff, alist, allowT;
  DBuf wicnt, wioff, heavy, hcount, hlist;
  DBuf M, color, colnand, col_and;
  DBuf scan_tmp;
  DBuf gid, cgroup, R, multi, A1, A2, own, cross;
  DBuf sq, pfoff, flags, T, loff, L, tp, poff, out;
  DBuf pinned_small;  // host pinned, 256 B
  i64 shadow_total = -1;
  DBuf scratch_words;

  hipEvent_t ev[10] = {};
  float stage_ms[8] = {};
};

namespace {

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

#define KTRY(expr)            \
  do {                        \
    int rc_ = (expr);         \
    if (rc_) return rc_;      \
  } while (0)

int fail(kano_ctx* ctx, int code, const std::string& msg) {
  ctx->err = msg;
  return code;
}

int dalloc(kano_ctx* ctx, DBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.p && b.bytes >= bytes) return 0;
  if (b.p) {
    KCHK(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  hipError_t e = hipMalloc(&b.p, bytes);
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

template <typename T>
T* P_(DBuf& b) {
  return reinterpret_cast<T*>(b.p);
}

inline unsigned nblk(i64 n, i64 per = TPB) { return (unsigned)((n + per - 1) / per); }

// exclusive scan of n elements, out has n+1 slots (out[n] = total).  The
// per-level tile sums live in ctx->scan_tmp, reserved once per input size
// (scan_reserve) so that no allocation happens between queued kernels.
size_t scan_scratch_bytes(i64 n) {
  size_t b = 0;
  while (n > SCAN_TILE) {
    const i64 t = (n + SCAN_TILE - 1) / SCAN_TILE;
    b += ((sizeof(i64) * (2 * t + 1) + 255) / 256) * 256;
    n = t;
  }
  return b + 256;
}

int scan_reserve(kano_ctx* ctx, i64 n) {
  return dalloc(ctx, ctx->scan_tmp, scan_scratch_bytes(n));
}

template <typename Tin, typename Tout>
int scan_level(kano_ctx* ctx, const Tin* in, i64 n, Tout* out, char* scratch) {
  if (n == 0) {
    KCHK(hipMemsetAsync(out, 0, sizeof(Tout), ctx->stream));
    return 0;
  }
  const i64 tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 1) {
    hipLaunchKernelGGL((k_scan_tiles<Tin, Tout>), dim3(1), dim3(TPB), 0, ctx->stream, in, n,
                       (const Tout*)nullptr, out);
    KLAUNCH();
    return 0;
  }
  Tout* sums = reinterpret_cast<Tout*>(scratch);
  Tout* offs = sums + tiles;
  char* next = scratch + ((sizeof(i64) * (2 * tiles + 1) + 255) / 256) * 256;
  hipLaunchKernelGGL((k_scan_sums<Tin, Tout>), dim3((unsigned)tiles), dim3(TPB), 0, ctx->stream,
                     in, n, sums);
  KLAUNCH();
  KTRY((scan_level<Tout, Tout>(ctx, sums, tiles, offs, next)));
  hipLaunchKernelGGL((k_scan_tiles<Tin, Tout>), dim3((unsigned)tiles), dim3(TPB), 0, ctx->stream,
                     in, n, (const Tout*)offs, out);
  KLAUNCH();
  return 0;
}

template <typename Tin, typename Tout>
int scan_excl(kano_ctx* ctx, const Tin* in, i64 n, Tout* out) {
  if (ctx->scan_tmp.bytes < scan_scratch_bytes(n))
    return fail(ctx, -EINVAL, "internal: scan scratch not reserved for " + std::to_string(n));
  return scan_level<Tin, Tout>(ctx, in, n, out, reinterpret_cast<char*>(ctx->scan_tmp.p));
}

int sync(kano_ctx* ctx) {
  KCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

template <typename T>
int read_scalar(kano_ctx* ctx, const T* dptr, T* hval) {
  KCHK(hipMemcpyAsync(hval, dptr, sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
  KCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

i64 rows_local(const kano_ctx* ctx) { return ctx->r1 - ctx->r0; }

int do_classes(kano_ctx* ctx) {
  const i64 n = ctx->n;
  i64 T = 1;
  while (T < 2 * n) T <<= 1;
  if (T < 64) T = 64;
  KTRY(dalloc(ctx, ctx->table, sizeof(int32_t) * T));
  KTRY(dalloc(ctx, ctx->smin, sizeof(int32_t) * T));
  KTRY(dalloc(ctx, ctx->slot_of, sizeof(int32_t) * n));
  KTRY(dalloc(ctx, ctx->flag, sizeof(int32_t) * n));
  KTRY(dalloc(ctx, ctx->cid, sizeof(int32_t) * (n + 1)));
  KTRY(dalloc(ctx, ctx->cls, sizeof(int32_t) * n));
  KCHK(hipMemsetAsync(ctx->table.p, 0xff, sizeof(int32_t) * T, ctx->stream));
  KCHK(hipMemsetAsync(ctx->smin.p, 0x7f, sizeof(int32_t) * T, ctx->stream));
  if (n > 0) {
  hipLaunchKernelGGL(k_class_insert, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(ctx->pv), n, P_<int32_t>(ctx->ckeys_d), ctx->KS,
                     P_<int32_t>(ctx->table), (uint32_t)(T - 1), P_<int32_t>(ctx->slot_of));
  KLAUNCH();
  hipLaunchKernelGGL(k_class_min, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(ctx->slot_of), n, P_<int32_t>(ctx->smin));
  KLAUNCH();
  hipLaunchKernelGGL(k_class_flag, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(ctx->slot_of), n, P_<int32_t>(ctx->smin), P_<int32_t>(ctx->flag));
  KLAUNCH();
  }
  KTRY((scan_excl<int32_t, int32_t>(ctx, P_<int32_t>(ctx->flag), n, P_<int32_t>(ctx->cid))));
  int32_t U32 = 0;
  KTRY(read_scalar(ctx, P_<int32_t>(ctx->cid) + n, &U32));
  const i64 U = U32;
  ctx->U = U;
  KTRY(dalloc(ctx, ctx->rep, sizeof(int32_t) * U));
  if (n > 0)
  hipLaunchKernelGGL(k_class_assign, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(ctx->slot_of), n, P_<int32_t>(ctx->smin), P_<int32_t>(ctx->cid),
                     P_<int32_t>(ctx->cls), P_<int32_t>(ctx->rep));
  KLAUNCH();
  // members of the local shard
  const i64 rl = rows_local(ctx);
  KTRY(dalloc(ctx, ctx->mcnt, sizeof(int32_t) * U));
  KTRY(dalloc(ctx, ctx->mcur, sizeof(int32_t) * U));
  KTRY(dalloc(ctx, ctx->moff, sizeof(int32_t) * (U + 1)));
  KTRY(dalloc(ctx, ctx->mem, sizeof(int32_t) * std::max<i64>(rl, 1)));
  KCHK(hipMemsetAsync(ctx->mcnt.p, 0, sizeof(int32_t) * U, ctx->stream));
  KCHK(hipMemsetAsync(ctx->mcur.p, 0, sizeof(int32_t) * U, ctx->stream));
  if (rl > 0) {
    hipLaunchKernelGGL(k_member_count, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cls), ctx->r0, ctx->r1, P_<int32_t>(ctx->mcnt));
    KLAUNCH();
  }
  KTRY((scan_excl<int32_t, int32_t>(ctx, P_<int32_t>(ctx->mcnt), U, P_<int32_t>(ctx->moff))));
  if (rl > 0) {
    hipLaunchKernelGGL(k_member_fill, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cls), ctx->r0, ctx->r1, P_<int32_t>(ctx->moff),
                       P_<int32_t>(ctx->mcur), P_<int32_t>(ctx->mem));
    KLAUNCH();
  }
  KTRY(dalloc(ctx, ctx->cval, sizeof(int32_t) * std::max<i64>(1, (i64)ctx->KS * U)));
  if (ctx->KS > 0 && U > 0) {
    hipLaunchKernelGGL(k_class_vals, dim3(nblk(U)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->pv), n, P_<int32_t>(ctx->ckeys_d), ctx->KS,
                       P_<int32_t>(ctx->rep), U, P_<int32_t>(ctx->cval));
    KLAUNCH();
  }
  return 0;
}

int do_select(kano_ctx* ctx) {
  const i64 U = ctx->U, P = ctx->P, PB = ctx->PB;
  KTRY(dalloc(ctx, ctx->selT, sizeof(u64) * std::max<i64>(1, PB * U)));
  KTRY(dalloc(ctx, ctx->scnt, sizeof(int32_t) * U));
  KTRY(dalloc(ctx, ctx->soffc, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->maxs, sizeof(int32_t)));
  KCHK(hipMemsetAsync(ctx->maxs.p, 0, sizeof(int32_t), ctx->stream));
  if (PB > 0 && U > 0) {
    hipLaunchKernelGGL(k_sel_eval, dim3(nblk(U), (unsigned)PB), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cval), U, P, P_<i64>(ctx->soff), P_<int32_t>(ctx->sslot),
                       P_<int32_t>(ctx->sval), P_<u64>(ctx->selT));
    KLAUNCH();
  }
  if (U > 0) {
    hipLaunchKernelGGL(k_sel_count, dim3(nblk(U)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->selT),
                       U, PB, P_<int32_t>(ctx->mcnt), P_<int32_t>(ctx->scnt),
                       P_<int32_t>(ctx->maxs));
    KLAUNCH();
  }
  KTRY((scan_excl<int32_t, i64>(ctx, P_<int32_t>(ctx->scnt), U, P_<i64>(ctx->soffc))));
  return 0;
}

int do_allow(kano_ctx* ctx) {
  const i64 n = ctx->n, W = ctx->W, P = ctx->P;
  const i64 ldA = ctx->ldM;
  KTRY(dalloc(ctx, ctx->allow, sizeof(u64) * std::max<i64>(1, P * ldA)));
  KTRY(dalloc(ctx, ctx->acnt, sizeof(int32_t) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, ctx->aloff, sizeof(i64) * (P + 1)));
  if (P > 0 && W > 0) {
    const int pch = 32;
    dim3 grid(nblk(W, TPB / 64), (unsigned)((P + pch - 1) / pch));
    if (ctx->ncols <= 32)
      hipLaunchKernelGGL(k_allow_eval<true>, grid, dim3(TPB), 0, ctx->stream, P_<int32_t>(ctx->pv),
                         n, ctx->ncols, W, P, pch, P_<i64>(ctx->aoff), P_<int32_t>(ctx->acol),
                         P_<int32_t>(ctx->aval), P_<u64>(ctx->allow), ldA);
    else
      hipLaunchKernelGGL(k_allow_eval<false>, grid, dim3(TPB), 0, ctx->stream,
                         P_<int32_t>(ctx->pv), n, ctx->ncols, W, P, pch, P_<i64>(ctx->aoff),
                         P_<int32_t>(ctx->acol), P_<int32_t>(ctx->aval), P_<u64>(ctx->allow), ldA);
    KLAUNCH();
    hipLaunchKernelGGL(k_allow_count, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->allow), W, ldA, P_<int32_t>(ctx->acnt));
    KLAUNCH();
  } else if (P > 0) {
    KCHK(hipMemsetAsync(ctx->acnt.p, 0, sizeof(int32_t) * P, ctx->stream));
  }
  KTRY((scan_excl<int32_t, i64>(ctx, P_<int32_t>(ctx->acnt), P, P_<i64>(ctx->aloff))));
  return 0;
}

int do_rows(kano_ctx* ctx, int path) {
  const i64 U = ctx->U, W = ctx->W, ldM = ctx->ldM, n = ctx->n;
  const i64 rl = rows_local(ctx);
  // the second host sync of the build: list sizes
  i64 hv[4] = {0, 0, 0, 0};
  {
    int32_t ms = 0;
    KCHK(hipMemcpyAsync(&hv[0], P_<i64>(ctx->soffc) + U, sizeof(i64), hipMemcpyDeviceToHost,
                        ctx->stream));
    KCHK(hipMemcpyAsync(&hv[1], P_<i64>(ctx->aloff) + ctx->P, sizeof(i64), hipMemcpyDeviceToHost,
                        ctx->stream));
    KCHK(hipMemcpyAsync(&ms, P_<int32_t>(ctx->maxs), sizeof(int32_t), hipMemcpyDeviceToHost,
                        ctx->stream));
    KCHK(hipStreamSynchronize(ctx->stream));
    ctx->max_sel = ms;
  }
  ctx->nnz_sel = hv[0];
  ctx->nnz_alw = hv[1];
  KTRY(dalloc(ctx, ctx->slist, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_sel)));
  KTRY(dalloc(ctx, ctx->alist, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_alw)));
  if (U > 0) {
    hipLaunchKernelGGL(k_sel_fill, dim3(nblk(U)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->selT), U,
                       ctx->PB, P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist));
    KLAUNCH();
  }
  if (ctx->P > 0 && W > 0) {
    hipLaunchKernelGGL(k_allow_fill, dim3((unsigned)ctx->P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->allow), W, ldM, P_<i64>(ctx->aloff), P_<int32_t>(ctx->alist));
    KLAUNCH();
  }
  // M and the column-check accumulators
  KTRY(dalloc(ctx, ctx->M, sizeof(u64) * std::max<i64>(1, rl * ldM)));
  KTRY(dalloc(ctx, ctx->color, sizeof(u64) * std::max<i64>(1, ldM)));
  KTRY(dalloc(ctx, ctx->colnand, sizeof(u64) * std::max<i64>(1, ldM)));
  KCHK(hipMemsetAsync(ctx->color.p, 0, sizeof(u64) * ldM, ctx->stream));
  KCHK(hipMemsetAsync(ctx->colnand.p, 0, sizeof(u64) * ldM, ctx->stream));
  if (rl == 0 || W == 0) {
    ctx->cols_valid = true;
    return 0;
  }
  // heavy classes
  KTRY(dalloc(ctx, ctx->heavy, std::max<i64>(U, 1)));
  KTRY(dalloc(ctx, ctx->hcount, sizeof(int32_t)));
  KTRY(dalloc(ctx, ctx->hlist, sizeof(int32_t) * std::max<i64>(U, 1)));
  KCHK(hipMemsetAsync(ctx->hcount.p, 0, sizeof(int32_t), ctx->stream));
  const int force = path == KANO_PATH_MFMA ? 2 : 0;
  hipLaunchKernelGGL(k_heavy_mark, dim3(nblk(U)), dim3(TPB), 0, ctx->stream, P_<i64>(ctx->soffc),
                     P_<int32_t>(ctx->slist), P_<int32_t>(ctx->acnt), P_<int32_t>(ctx->mcnt), U, W,
                     ctx->ch, force, P_<uint8_t>(ctx->heavy), P_<int32_t>(ctx->hcount),
                     P_<int32_t>(ctx->hlist));
  KLAUNCH();
  int32_t H = 0;
  KTRY(read_scalar(ctx, P_<int32_t>(ctx->hcount), &H));
  ctx->heavy_count = H;
  if (H > 0) {
    // deterministic order of the heavy list does not matter for the result
    bool use_mfma = (path == KANO_PATH_MFMA) || (path == KANO_PATH_AUTO && H >= 16);
    if (use_mfma) {
      KTRY(dalloc(ctx, ctx->allowT, sizeof(u64) * std::max<i64>(1, ctx->PB * n)));
      hipLaunchKernelGGL(k_allow_transpose, dim3(nblk(W, 4), (unsigned)ctx->PB), dim3(TPB), 0,
                         ctx->stream, P_<u64>(ctx->allow), ldM, W, ctx->P, n,
                         P_<u64>(ctx->allowT));
      KLAUNCH();
      // zero the heavy rows' padding word (the MFMA tiles write 32-bit halves up to n)
      for (int32_t h0 = 0; h0 < H; h0 += 128) {
        const int hh = std::min<int32_t>(128, H - h0);
        const int32_t* hl = P_<int32_t>(ctx->hlist) + h0;
        dim3 grid(nblk((n + 31) / 32, TPB / 64));
        if (hh <= 32)
          hipLaunchKernelGGL(k_heavy_mfma<1>, grid, dim3(TPB), 0, ctx->stream, P_<u64>(ctx->selT),
                             U, hl, hh, P_<u64>(ctx->allowT), n, ctx->PB, P_<int32_t>(ctx->moff),
                             P_<int32_t>(ctx->mem), P_<uint32_t>(ctx->M), ldM, ctx->r0);
        else if (hh <= 64)
          hipLaunchKernelGGL(k_heavy_mfma<2>, grid, dim3(TPB), 0, ctx->stream, P_<u64>(ctx->selT),
                             U, hl, hh, P_<u64>(ctx->allowT), n, ctx->PB, P_<int32_t>(ctx->moff),
                             P_<int32_t>(ctx->mem), P_<uint32_t>(ctx->M), ldM, ctx->r0);
        else
          hipLaunchKernelGGL(k_heavy_mfma<4>, grid, dim3(TPB), 0, ctx->stream, P_<u64>(ctx->selT),
                             U, hl, hh, P_<u64>(ctx->allowT), n, ctx->PB, P_<int32_t>(ctx->moff),
                             P_<int32_t>(ctx->mem), P_<uint32_t>(ctx->M), ldM, ctx->r0);
        KLAUNCH();
      }
    } else {
      dim3 grid((unsigned)H, nblk(ldM, 128));
      hipLaunchKernelGGL(k_heavy_or, grid, dim3(TPB), 0, ctx->stream, P_<int32_t>(ctx->hlist),
                         P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), P_<u64>(ctx->allow), ldM, W,
                         P_<int32_t>(ctx->moff), P_<int32_t>(ctx->mem), P_<u64>(ctx->M), ldM,
                         ctx->r0);
      KLAUNCH();
    }
  }
  // work items
  KTRY(dalloc(ctx, ctx->wicnt, sizeof(int32_t) * U));
  KTRY(dalloc(ctx, ctx->wioff, sizeof(int32_t) * (U + 1)));
  hipLaunchKernelGGL(k_wi_count, dim3(nblk(U)), dim3(TPB), 0, ctx->stream, P_<int32_t>(ctx->mcnt),
                     U, ctx->ch, P_<int32_t>(ctx->wicnt));
  KLAUNCH();
  KTRY((scan_excl<int32_t, int32_t>(ctx, P_<int32_t>(ctx->wicnt), U, P_<int32_t>(ctx->wioff))));
  // upper bound on work items: sum ceil(m_c/ch) <= U + rl/ch
  const i64 wi_ub = std::min<i64>(U + rl / ctx->ch + 1, rl);
  const int cww = (int)std::min<i64>(ldM, MAX_CWW);
  const unsigned ncc = (unsigned)((ldM + cww - 1) / cww);
  RowsArgs a;
  a.wioff = P_<int32_t>(ctx->wioff);
  a.U = U;
  a.soffc = P_<i64>(ctx->soffc);
  a.slist = P_<int32_t>(ctx->slist);
  a.acnt = P_<int32_t>(ctx->acnt);
  a.aloff = P_<i64>(ctx->aloff);
  a.alist = P_<int32_t>(ctx->alist);
  a.allow = P_<u64>(ctx->allow);
  a.ldA = ldM;
  a.moff = P_<int32_t>(ctx->moff);
  a.mem = P_<int32_t>(ctx->mem);
  a.heavy = H > 0 ? P_<uint8_t>(ctx->heavy) : nullptr;
  a.M = P_<u64>(ctx->M);
  a.ldM = ldM;
  a.r0 = ctx->r0;
  a.n = n;
  a.W = W;
  a.ch = ctx->ch;
  a.cww = cww;
  a.color = P_<u64>(ctx->color);
  a.colnand = P_<u64>(ctx->colnand);
  KCHK(hipEventRecord(ctx->ev[7], ctx->stream));
  hipLaunchKernelGGL(k_rows, dim3((unsigned)wi_ub, ncc), dim3(TPB), sizeof(u64) * cww, ctx->stream,
                     a);
  KLAUNCH();
  KCHK(hipEventRecord(ctx->ev[8], ctx->stream));
  ctx->rows_timed = true;
  ctx->wi_total = wi_ub;
  ctx->cols_valid = true;
  return 0;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int kano_create(int device, kano_ctx** out) {
  if (!out) return -EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -ENODEV;
  if (device < 0 || device >= ndev) return -EINVAL;
  if (hipSetDevice(device) != hipSuccess) return -EIO;
  kano_ctx* ctx = new kano_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return -EIO;
  }
  ctx->own_stream = true;
  for (auto& e : ctx->ev) (void)hipEventCreate(&e);
  *out = ctx;
  return 0;
}

void kano_destroy(kano_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  DBuf* bufs[] = {&ctx->pv,     &ctx->ckeys_d, &ctx->soff,    &ctx->sslot,  &ctx->sval,
                  &ctx->aoff,   &ctx->acol,    &ctx->aval,    &ctx->table,  &ctx->slot_of,
                  &ctx->smin,   &ctx->flag,    &ctx->cid,     &ctx->cls,    &ctx->rep,
                  &ctx->mcnt,   &ctx->moff,    &ctx->mcur,    &ctx->mem,    &ctx->cval,
                  &ctx->selT,   &ctx->scnt,    &ctx->soffc,   &ctx->slist,  &ctx->maxs,
                  &ctx->allow,  &ctx->acnt,    &ctx->aloff,   &ctx->alist,  &ctx->allowT,
                  &ctx->wicnt,  &ctx->wioff,   &ctx->heavy,   &ctx->hcount, &ctx->hlist,
                  &ctx->M,      &ctx->color,   &ctx->colnand, &ctx->col_and, &ctx->scan_tmp,
                  &ctx->gid,    &ctx->cgroup,  &ctx->R,       &ctx->multi,  &ctx->A1,
                  &ctx->A2,     &ctx->own,     &ctx->cross,   &ctx->sq,     &ctx->pfoff,
                  &ctx->flags,  &ctx->T,       &ctx->loff,    &ctx->L,      &ctx->tp,
                  &ctx->poff,   &ctx->out,     &ctx->scratch_words};
  for (DBuf* b : bufs) dfree(*b);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* kano_last_error(const kano_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int kano_set_stream(kano_ctx* ctx, void* s) {
  if (!ctx) return -EINVAL;
  KCHK(hipSetDevice(ctx->device));
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
  if (!ctx || n < 0 || ncols < 0 || n >= (int64_t)INT32_MAX || (n * ncols > 0 && !pod_val))
    return ctx ? fail(ctx, -EINVAL, "kano_set_pods: bad arguments") : -EINVAL;
  KCHK(hipSetDevice(ctx->device));
  ctx->n = n;
  ctx->W = (n + 63) / 64;
  ctx->ldM = (ctx->W + 1) & ~(i64)1;
  if (ctx->ldM == 0) ctx->ldM = 2;
  ctx->ncols = ncols;
  KTRY(dalloc(ctx, ctx->pv, sizeof(int32_t) * std::max<i64>(1, n * ncols)));
  if (n * ncols > 0)
    KCHK(hipMemcpyAsync(ctx->pv.p, pod_val, sizeof(int32_t) * n * ncols, hipMemcpyHostToDevice,
                        ctx->stream));
  ctx->r0 = 0;
  ctx->r1 = n;
  ctx->have_pods = true;
  ctx->built = false;
  return sync(ctx);
}

int kano_set_policies(kano_ctx* ctx, int64_t P, const int64_t* sel_off, const int32_t* sel_col,
                      const int32_t* sel_val, const int64_t* alw_off, const int32_t* alw_col,
                      const int32_t* alw_val) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods) return fail(ctx, -EINVAL, "kano_set_policies before kano_set_pods");
  if (P < 0 || !sel_off || !alw_off) return fail(ctx, -EINVAL, "kano_set_policies: bad arguments");
  KCHK(hipSetDevice(ctx->device));
  const i64 ns = sel_off[P], na = alw_off[P];
  // class keys = columns referenced by any working-selector term
  std::vector<int32_t> slot(ctx->ncols, -1);
  ctx->ckeys.clear();
  for (i64 t = 0; t < ns; ++t) {
    const int32_t c = sel_col[t];
    if (c < 0 || c >= ctx->ncols) return fail(ctx, -EINVAL, "selector term column out of range");
    if (slot[c] < 0) { slot[c] = 0; }
  }
  for (int32_t c = 0; c < ctx->ncols; ++c)
    if (slot[c] == 0) { slot[c] = (int32_t)ctx->ckeys.size(); ctx->ckeys.push_back(c); }
  std::vector<int32_t> sslot(std::max<i64>(ns, 1));
  for (i64 t = 0; t < ns; ++t) sslot[t] = slot[sel_col[t]];
  for (i64 t = 0; t < na; ++t)
    if (alw_col[t] < 0 || alw_col[t] >= ctx->ncols)
      return fail(ctx, -EINVAL, "allow term column out of range");
  ctx->KS = (int)ctx->ckeys.size();
  ctx->P = P;
  ctx->PB = (P + 63) / 64;
  KTRY(dalloc(ctx, ctx->ckeys_d, sizeof(int32_t) * std::max<size_t>(1, ctx->ckeys.size())));
  KTRY(dalloc(ctx, ctx->soff, sizeof(i64) * (P + 1)));
  KTRY(dalloc(ctx, ctx->sslot, sizeof(int32_t) * std::max<i64>(1, ns)));
  KTRY(dalloc(ctx, ctx->sval, sizeof(int32_t) * std::max<i64>(1, ns)));
  KTRY(dalloc(ctx, ctx->aoff, sizeof(i64) * (P + 1)));
  KTRY(dalloc(ctx, ctx->acol, sizeof(int32_t) * std::max<i64>(1, na)));
  KTRY(dalloc(ctx, ctx->aval, sizeof(int32_t) * std::max<i64>(1, na)));
  if (!ctx->ckeys.empty())
    KCHK(hipMemcpyAsync(ctx->ckeys_d.p, ctx->ckeys.data(), sizeof(int32_t) * ctx->ckeys.size(),
                        hipMemcpyHostToDevice, ctx->stream));
  KCHK(hipMemcpyAsync(ctx->soff.p, sel_off, sizeof(i64) * (P + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  KCHK(hipMemcpyAsync(ctx->aoff.p, alw_off, sizeof(i64) * (P + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  if (ns > 0) {
    KCHK(hipMemcpyAsync(ctx->sslot.p, sslot.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice,
                        ctx->stream));
    KCHK(hipMemcpyAsync(ctx->sval.p, sel_val, sizeof(int32_t) * ns, hipMemcpyHostToDevice,
                        ctx->stream));
  }
  if (na > 0) {
    KCHK(hipMemcpyAsync(ctx->acol.p, alw_col, sizeof(int32_t) * na, hipMemcpyHostToDevice,
                        ctx->stream));
    KCHK(hipMemcpyAsync(ctx->aval.p, alw_val, sizeof(int32_t) * na, hipMemcpyHostToDevice,
                        ctx->stream));
  }
  ctx->have_pols = true;
  ctx->built = false;
  return sync(ctx);  // sslot is a stack temporary
}

int kano_set_shard(kano_ctx* ctx, int64_t row_begin, int64_t row_end) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods || row_begin < 0 || row_end < row_begin || row_end > ctx->n)
    return fail(ctx, -EINVAL, "kano_set_shard: bad row range");
  ctx->r0 = row_begin;
  ctx->r1 = row_end;
  ctx->built = false;
  return 0;
}

int kano_build(kano_ctx* ctx, int path) {
  if (!ctx) return -EINVAL;
  if (!ctx->have_pods || !ctx->have_pols) return fail(ctx, -EINVAL, "kano_build: inputs not set");
  if (path < 0 || path > 2) return fail(ctx, -EINVAL, "kano_build: unknown path");
  KCHK(hipSetDevice(ctx->device));
  ctx->built = false;
  ctx->lists_mode = false;
  ctx->rows_timed = false;
  ctx->shadow_total = -1;
  ctx->rows_dirty = false;
  KTRY(scan_reserve(ctx, std::max<i64>({ctx->n, ctx->P, (i64)1})));
  KCHK(hipEventRecord(ctx->ev[0], ctx->stream));
  KTRY(do_classes(ctx));
  KCHK(hipEventRecord(ctx->ev[1], ctx->stream));
  KTRY(do_select(ctx));
  KCHK(hipEventRecord(ctx->ev[2], ctx->stream));
  KTRY(do_allow(ctx));
  KCHK(hipEventRecord(ctx->ev[3], ctx->stream));
  KTRY(do_rows(ctx, path));
  KCHK(hipEventRecord(ctx->ev[4], ctx->stream));
  ctx->built = true;
  return 0;
}

int kano_info(kano_ctx* ctx, int64_t* out) {
  if (!ctx || !out) return -EINVAL;
  for (int k = 0; k < KANO_INFO_NSLOTS; ++k) out[k] = 0;
  out[KANO_INFO_N] = ctx->n;
  out[KANO_INFO_W] = ctx->W;
  out[KANO_INFO_P] = ctx->P;
  out[KANO_INFO_U] = ctx->U;
  out[KANO_INFO_NNZ_SEL] = ctx->nnz_sel;
  out[KANO_INFO_NNZ_ALW] = ctx->nnz_alw;
  out[KANO_INFO_HEAVY] = ctx->heavy_count;
  out[KANO_INFO_ROW0] = ctx->r0;
  out[KANO_INFO_ROW1] = ctx->r1;
  out[KANO_INFO_MAXSEL] = ctx->max_sel;
  return 0;
}

static int ensure_built(kano_ctx* ctx) {
  if (!ctx) return -EINVAL;
  if (!ctx->built) return fail(ctx, -EINVAL, "matrix not built");
  KCHK(hipSetDevice(ctx->device));
  return 0;
}

static int ensure_matrix(kano_ctx* ctx) {
  KTRY(ensure_built(ctx));
  if (ctx->lists_mode) return fail(ctx, -EINVAL, "context holds policy lists, not a matrix");
  return 0;
}

// Recompute column OR / NAND from M itself (after a kano_set_bit).
static int recompute_cols(kano_ctx* ctx) {
  const i64 rl = rows_local(ctx), W = ctx->W, ldM = ctx->ldM;
  KCHK(hipMemsetAsync(ctx->color.p, 0, sizeof(u64) * ldM, ctx->stream));
  KCHK(hipMemsetAsync(ctx->colnand.p, 0, sizeof(u64) * ldM, ctx->stream));
  if (rl == 0 || W == 0) {
    ctx->cols_valid = true;
    return 0;
  }
  // treat every row as its own class with no policies but a prebuilt row:
  // reuse k_rows' column epilogue through the heavy copy path
  KTRY(dalloc(ctx, ctx->scratch_words, sizeof(int32_t) * (3 * rl + 2) + rl));
  int32_t* wioff = P_<int32_t>(ctx->scratch_words);
  int32_t* moff = wioff + (rl + 1);
  int32_t* mem = moff + (rl + 1);
  uint8_t* heavy = reinterpret_cast<uint8_t*>(mem + rl);
  std::vector<int32_t> h_off(rl + 1), h_mem(rl);
  for (i64 r = 0; r <= rl; ++r) h_off[r] = (int32_t)r;
  for (i64 r = 0; r < rl; ++r) h_mem[r] = (int32_t)(ctx->r0 + r);
  KCHK(hipMemcpyAsync(wioff, h_off.data(), sizeof(int32_t) * (rl + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  KCHK(hipMemcpyAsync(moff, h_off.data(), sizeof(int32_t) * (rl + 1), hipMemcpyHostToDevice,
                      ctx->stream));
  KCHK(hipMemcpyAsync(mem, h_mem.data(), sizeof(int32_t) * rl, hipMemcpyHostToDevice, ctx->stream));
  KCHK(hipMemsetAsync(heavy, 1, rl, ctx->stream));
  const int cww = (int)std::min<i64>(ldM, MAX_CWW);
  RowsArgs a{};
  a.wioff = wioff;
  a.U = rl;
  a.moff = moff;
  a.mem = mem;
  a.heavy = heavy;
  a.M = P_<u64>(ctx->M);
  a.ldM = ldM;
  a.r0 = ctx->r0;
  a.n = ctx->n;
  a.W = W;
  a.ch = 1;
  a.cww = cww;
  a.color = P_<u64>(ctx->color);
  a.colnand = P_<u64>(ctx->colnand);
  hipLaunchKernelGGL(k_rows, dim3((unsigned)rl, (unsigned)((ldM + cww - 1) / cww)), dim3(TPB),
                     sizeof(u64) * cww, ctx->stream, a);
  KLAUNCH();
  KTRY(sync(ctx));
  ctx->cols_valid = true;
  return 0;
}

int kano_col_checks(kano_ctx* ctx, uint64_t* col_and, uint64_t* col_or) {
  KTRY(ensure_matrix(ctx));
  if (!ctx->cols_valid) KTRY(recompute_cols(ctx));
  const i64 W = ctx->W;
  if (W == 0) return sync(ctx);
  KTRY(dalloc(ctx, ctx->col_and, sizeof(u64) * W));
  hipLaunchKernelGGL(k_col_final, dim3(nblk(W)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->color),
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

static int crosscheck_impl(kano_ctx* ctx, const int32_t* gid) {
  const i64 n = ctx->n, W = ctx->W, ldM = ctx->ldM, U = ctx->U;
  KTRY(dalloc(ctx, ctx->gid, sizeof(int32_t) * std::max<i64>(1, n)));
  KTRY(dalloc(ctx, ctx->cross, sizeof(u64) * ldM));
  if (n == 0) return 0;
  KCHK(hipMemcpyAsync(ctx->gid.p, gid, sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
  int32_t G = 0;
  for (i64 i = 0; i < n; ++i) G = std::max(G, gid[i] + 1);
  KTRY(dalloc(ctx, ctx->multi, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->A1, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->A2, sizeof(u64) * ldM));
  KTRY(dalloc(ctx, ctx->own, sizeof(u64) * ldM));
  for (DBuf* b : {&ctx->multi, &ctx->A1, &ctx->A2, &ctx->own})
    KCHK(hipMemsetAsync(b->p, 0, sizeof(u64) * ldM, ctx->stream));
  if (rows_local(ctx) == 0 || W == 0) {
    KCHK(hipMemsetAsync(ctx->cross.p, 0, sizeof(u64) * ldM, ctx->stream));
    return 0;
  }
  // classes: after a set_bit the class structure no longer describes M, so
  // every row becomes its own class
  const int32_t* moff = P_<int32_t>(ctx->moff);
  const int32_t* mem = P_<int32_t>(ctx->mem);
  i64 nclass = U;
  DBuf ident;
  const bool per_row = ctx->rows_dirty;
  if (per_row) {
    const i64 rl = rows_local(ctx);
    KTRY(dalloc(ctx, ident, sizeof(int32_t) * (2 * rl + 1)));
    std::vector<int32_t> h(2 * rl + 1);
    for (i64 r = 0; r <= rl; ++r) h[r] = (int32_t)r;
    for (i64 r = 0; r < rl; ++r) h[rl + 1 + r] = (int32_t)(ctx->r0 + r);
    KCHK(hipMemcpyAsync(ident.p, h.data(), sizeof(int32_t) * (2 * rl + 1), hipMemcpyHostToDevice,
                        ctx->stream));
    KCHK(hipStreamSynchronize(ctx->stream));
    moff = P_<int32_t>(ident);
    mem = moff + rl + 1;
    nclass = rl;
  }
  KTRY(dalloc(ctx, ctx->cgroup, sizeof(int32_t) * std::max<i64>(1, nclass)));
  hipLaunchKernelGGL(k_cross_classgroup, dim3(nblk(nclass)), dim3(TPB), 0, ctx->stream,
                     P_<int32_t>(ctx->gid), moff, mem, nclass, P_<int32_t>(ctx->cgroup));
  KLAUNCH();
  // groups in batches so that R fits a budget of ~2 GiB
  const i64 budget_rows = std::max<i64>(1, (2ll << 30) / (8 * ldM));
  const unsigned ycols = nblk(W, TPB * 4) > 0 ? nblk(W, TPB * 4) : 1;
  for (int32_t g0 = 0; g0 < std::max<int32_t>(G, 1); g0 += (int32_t)budget_rows) {
    const int32_t g1 = (int32_t)std::min<i64>(G, (i64)g0 + budget_rows);
    const i64 ng = std::max<i64>(1, g1 - g0);
    KTRY(dalloc(ctx, ctx->R, sizeof(u64) * ng * ldM));
    KCHK(hipMemsetAsync(ctx->R.p, 0, sizeof(u64) * ng * ldM, ctx->stream));
    hipLaunchKernelGGL(k_cross_accum, dim3((unsigned)nclass, ycols), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cgroup), moff, mem, P_<u64>(ctx->M), ldM, ctx->r0, W, g0, g1,
                       P_<u64>(ctx->R), P_<u64>(ctx->multi));
    KLAUNCH();
    if (g1 > g0) {
      hipLaunchKernelGGL(k_cross_groups, dim3((unsigned)(g1 - g0), ycols), dim3(TPB), 0,
                         ctx->stream, P_<u64>(ctx->R), ldM, W, P_<u64>(ctx->A1), P_<u64>(ctx->A2));
      KLAUNCH();
      hipLaunchKernelGGL(k_cross_own, dim3(nblk(n)), dim3(TPB), 0, ctx->stream,
                         P_<int32_t>(ctx->gid), n, P_<u64>(ctx->R), ldM, g0, g1, P_<u64>(ctx->own));
      KLAUNCH();
    }
    if (G == 0) break;
  }
  hipLaunchKernelGGL(k_cross_final, dim3(nblk(W)), dim3(TPB), 0, ctx->stream, P_<u64>(ctx->multi),
                     P_<u64>(ctx->A1), P_<u64>(ctx->A2), P_<u64>(ctx->own), W, n,
                     P_<u64>(ctx->cross));
  KLAUNCH();
  if (ident.p) {
    KCHK(hipStreamSynchronize(ctx->stream));
    dfree(ident);
  }
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
  return 0;
}

int kano_get_rows(kano_ctx* ctx, int64_t r0, int64_t nrows, uint64_t* dst) {
  KTRY(ensure_matrix(ctx));
  if (nrows < 0 || r0 < ctx->r0 || r0 + nrows > ctx->r1 || (!dst && nrows > 0))
    return fail(ctx, -EINVAL, "kano_get_rows: rows outside this shard");
  if (nrows == 0 || ctx->W == 0) return 0;
  KCHK(hipMemcpy2DAsync(dst, sizeof(u64) * ctx->W, P_<u64>(ctx->M) + (r0 - ctx->r0) * ctx->ldM,
                        sizeof(u64) * ctx->ldM, sizeof(u64) * ctx->W, (size_t)nrows,
                        hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
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
  // the class factorisation no longer describes M: column checks are
  // recomputed from M and crosscheck runs per row from now on
  ctx->cols_valid = false;
  ctx->rows_dirty = true;
  return 0;
}

int kano_get_policy_sets(kano_ctx* ctx, int64_t p, uint64_t* sel, uint64_t* allow) {
  KTRY(ensure_matrix(ctx));
  if (p < 0 || p >= ctx->P) return fail(ctx, -EINVAL, "kano_get_policy_sets: bad policy");
  const i64 W = ctx->W;
  if (W == 0) return 0;
  if (sel) {
    KTRY(dalloc(ctx, ctx->scratch_words, sizeof(u64) * W));
    hipLaunchKernelGGL(k_sel_row, dim3(nblk(ctx->n)), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->selT), ctx->U, P_<int32_t>(ctx->cls), ctx->n, (i64)p,
                       P_<u64>(ctx->scratch_words));
    KLAUNCH();
    KCHK(hipMemcpyAsync(sel, ctx->scratch_words.p, sizeof(u64) * W, hipMemcpyDeviceToHost,
                        ctx->stream));
  }
  if (allow)
    KCHK(hipMemcpyAsync(allow, P_<u64>(ctx->allow) + p * ctx->ldM, sizeof(u64) * W,
                        hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

int kano_get_classes(kano_ctx* ctx, int32_t* cls) {
  KTRY(ensure_matrix(ctx));
  if (cls && ctx->n > 0)
    KCHK(hipMemcpyAsync(cls, ctx->cls.p, sizeof(int32_t) * ctx->n, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

int kano_get_select_csr(kano_ctx* ctx, int64_t* off, int32_t* pol) {
  KTRY(ensure_matrix(ctx));
  if (off)
    KCHK(hipMemcpyAsync(off, ctx->soffc.p, sizeof(i64) * (ctx->U + 1), hipMemcpyDeviceToHost,
                        ctx->stream));
  if (pol && ctx->nnz_sel > 0)
    KCHK(hipMemcpyAsync(pol, ctx->slist.p, sizeof(int32_t) * ctx->nnz_sel, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

int kano_get_allow_csr(kano_ctx* ctx, int64_t* off, int32_t* pods) {
  KTRY(ensure_matrix(ctx));
  if (off)
    KCHK(hipMemcpyAsync(off, ctx->aloff.p, sizeof(i64) * (ctx->P + 1), hipMemcpyDeviceToHost,
                        ctx->stream));
  if (pods && ctx->nnz_alw > 0)
    KCHK(hipMemcpyAsync(pods, ctx->alist.p, sizeof(int32_t) * ctx->nnz_alw, hipMemcpyDeviceToHost,
                        ctx->stream));
  return sync(ctx);
}

int kano_shadow(kano_ctx* ctx, int64_t* count) {
  KTRY(ensure_built(ctx));
  const i64 U = ctx->U, rl = rows_local(ctx);
  KCHK(hipEventRecord(ctx->ev[5], ctx->stream));
  KTRY(dalloc(ctx, ctx->sq, sizeof(i64) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->pfoff, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->T, sizeof(i64) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->loff, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->tp, sizeof(i64) * std::max<i64>(1, rl)));
  KTRY(dalloc(ctx, ctx->poff, sizeof(i64) * (rl + 1)));
  if (U > 0) {
    hipLaunchKernelGGL(k_shadow_sq, dim3(nblk(U)), dim3(TPB), 0, ctx->stream, P_<i64>(ctx->soffc),
                       P_<int32_t>(ctx->mcnt), U, P_<i64>(ctx->sq));
    KLAUNCH();
  }
  KTRY((scan_excl<i64, i64>(ctx, P_<i64>(ctx->sq), U, P_<i64>(ctx->pfoff))));
  i64 nflags = 0;
  KTRY(read_scalar(ctx, P_<i64>(ctx->pfoff) + U, &nflags));
  KTRY(dalloc(ctx, ctx->flags, std::max<i64>(1, nflags)));
  if (U > 0) {
    hipLaunchKernelGGL(k_shadow_test, dim3((unsigned)U), dim3(TPB), 0, ctx->stream,
                       P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), P_<int32_t>(ctx->mcnt),
                       P_<i64>(ctx->pfoff), P_<int32_t>(ctx->acnt), P_<i64>(ctx->aloff),
                       P_<int32_t>(ctx->alist), P_<u64>(ctx->allow), ctx->ldM,
                       P_<uint8_t>(ctx->flags), P_<i64>(ctx->T));
    KLAUNCH();
  }
  KTRY((scan_excl<i64, i64>(ctx, P_<i64>(ctx->T), U, P_<i64>(ctx->loff))));
  i64 nl = 0;
  KTRY(read_scalar(ctx, P_<i64>(ctx->loff) + U, &nl));
  KTRY(dalloc(ctx, ctx->L, sizeof(int2) * std::max<i64>(1, nl)));
  if (U > 0 && nl > 0) {
    hipLaunchKernelGGL(k_shadow_compact, dim3((unsigned)U), dim3(TPB), 0, ctx->stream,
                       P_<i64>(ctx->soffc), P_<int32_t>(ctx->slist), P_<i64>(ctx->pfoff),
                       P_<uint8_t>(ctx->flags), P_<i64>(ctx->loff), P_<int2>(ctx->L));
    KLAUNCH();
  }
  if (rl > 0) {
    hipLaunchKernelGGL(k_shadow_podcount, dim3(nblk(rl)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                       P_<i64>(ctx->tp));
    KLAUNCH();
  }
  KTRY((scan_excl<i64, i64>(ctx, P_<i64>(ctx->tp), rl, P_<i64>(ctx->poff))));
  i64 total = 0;
  KTRY(read_scalar(ctx, P_<i64>(ctx->poff) + rl, &total));
  KTRY(dalloc(ctx, ctx->out, sizeof(int2) * std::max<i64>(1, total)));
  if (rl > 0 && total > 0) {
    hipLaunchKernelGGL(k_shadow_emit, dim3(nblk(rl, TPB / 64)), dim3(TPB), 0, ctx->stream,
                       P_<int32_t>(ctx->cls), ctx->r0, ctx->r1, P_<i64>(ctx->loff),
                       P_<int2>(ctx->L), P_<i64>(ctx->poff), P_<int2>(ctx->out));
    KLAUNCH();
  }
  KCHK(hipEventRecord(ctx->ev[6], ctx->stream));
  ctx->shadow_total = total;
  if (count) *count = total;
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

int kano_conflict(kano_ctx* ctx, int* raises) {
  KTRY(ensure_built(ctx));
  if (!raises) return fail(ctx, -EINVAL, "kano_conflict: NULL");
  *raises = ctx->max_sel >= 2 ? 1 : 0;
  return 0;
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
  return 0;
}

int kano_shadow_lists(kano_ctx* ctx, int64_t n_lists, int64_t nbits, int64_t P,
                      const int64_t* soff, const int32_t* slist, const uint64_t* allow_rows,
                      int64_t* count) {
  if (!ctx) return -EINVAL;
  if (n_lists < 0 || nbits < 0 || P < 0 || !soff || n_lists >= (int64_t)INT32_MAX)
    return fail(ctx, -EINVAL, "kano_shadow_lists: bad arguments");
  KCHK(hipSetDevice(ctx->device));
  const i64 nnz = soff[n_lists];
  for (i64 e = 0; e < nnz; ++e)
    if (slist[e] < 0 || slist[e] >= P)
      return fail(ctx, -ERANGE, "kano_shadow_lists: policy index out of range");
  ctx->built = false;
  ctx->lists_mode = true;
  ctx->n = nbits;
  ctx->W = (nbits + 63) / 64;
  ctx->ldM = std::max<i64>(2, (ctx->W + 1) & ~(i64)1);
  ctx->P = P;
  ctx->PB = (P + 63) / 64;
  ctx->U = n_lists;
  ctx->r0 = 0;
  ctx->r1 = n_lists;
  ctx->nnz_sel = nnz;
  KTRY(scan_reserve(ctx, std::max<i64>({n_lists, P, (i64)1})));
  const i64 U = n_lists, W = ctx->W, ldM = ctx->ldM;
  KTRY(dalloc(ctx, ctx->soffc, sizeof(i64) * (U + 1)));
  KTRY(dalloc(ctx, ctx->slist, sizeof(int32_t) * std::max<i64>(1, nnz)));
  KTRY(dalloc(ctx, ctx->cls, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->mcnt, sizeof(int32_t) * std::max<i64>(1, U)));
  KTRY(dalloc(ctx, ctx->allow, sizeof(u64) * std::max<i64>(1, P * ldM)));
  KTRY(dalloc(ctx, ctx->acnt, sizeof(int32_t) * std::max<i64>(1, P)));
  KTRY(dalloc(ctx, ctx->aloff, sizeof(i64) * (P + 1)));
  std::vector<int32_t> iota(std::max<i64>(1, U)), ones(std::max<i64>(1, U), 1);
  for (i64 c = 0; c < U; ++c) iota[c] = (int32_t)c;
  KCHK(hipMemcpyAsync(ctx->soffc.p, soff, sizeof(i64) * (U + 1), hipMemcpyHostToDevice, ctx->stream));
  if (nnz > 0)
    KCHK(hipMemcpyAsync(ctx->slist.p, slist, sizeof(int32_t) * nnz, hipMemcpyHostToDevice,
                        ctx->stream));
  if (U > 0) {
    KCHK(hipMemcpyAsync(ctx->cls.p, iota.data(), sizeof(int32_t) * U, hipMemcpyHostToDevice,
                        ctx->stream));
    KCHK(hipMemcpyAsync(ctx->mcnt.p, ones.data(), sizeof(int32_t) * U, hipMemcpyHostToDevice,
                        ctx->stream));
  }
  if (P > 0 && W > 0) {
    KCHK(hipMemcpy2DAsync(ctx->allow.p, sizeof(u64) * ldM, allow_rows, sizeof(u64) * W,
                          sizeof(u64) * W, (size_t)P, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_allow_count, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->allow), W, ldM, P_<int32_t>(ctx->acnt));
    KLAUNCH();
  } else if (P > 0) {
    KCHK(hipMemsetAsync(ctx->acnt.p, 0, sizeof(int32_t) * P, ctx->stream));
  }
  KTRY((scan_excl<int32_t, i64>(ctx, P_<int32_t>(ctx->acnt), P, P_<i64>(ctx->aloff))));
  KTRY(read_scalar(ctx, P_<i64>(ctx->aloff) + P, &ctx->nnz_alw));
  KTRY(dalloc(ctx, ctx->alist, sizeof(int32_t) * std::max<i64>(1, ctx->nnz_alw)));
  if (P > 0 && W > 0) {
    hipLaunchKernelGGL(k_allow_fill, dim3((unsigned)P), dim3(TPB), 0, ctx->stream,
                       P_<u64>(ctx->allow), W, ldM, P_<i64>(ctx->aloff), P_<int32_t>(ctx->alist));
    KLAUNCH();
  }
  KTRY(sync(ctx));  // host vectors above are temporaries
  ctx->built = true;
  return kano_shadow(ctx, count);
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
  KTRY(sync(ctx));
  for (int k = 0; k < 8; ++k) ms[k] = 0.f;
  if (ctx->built) {
    for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&ms[k], ctx->ev[k], ctx->ev[k + 1]);
    (void)hipEventElapsedTime(&ms[5], ctx->ev[0], ctx->ev[4]);
  }
  if (ctx->shadow_total >= 0) (void)hipEventElapsedTime(&ms[4], ctx->ev[5], ctx->ev[6]);
  if (ctx->built && ctx->rows_timed) (void)hipEventElapsedTime(&ms[6], ctx->ev[7], ctx->ev[8]);
  return 0;
}

}  // extern "C"
