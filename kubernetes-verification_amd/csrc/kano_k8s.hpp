// kubesv's edge relation over kano's matrices.
//
// kubesv/kubesv/constraint.py:191-231 defines
//   ingress_traffic(src, sel) :- selected_by_pol(sel, pol), ingress_allow_by_pol(src, pol)
//                              | sel = src                       (check_self_ingress_traffic)
//   egress_traffic(dst, sel)  :- selected_by_pol(sel, pol), egress_allow_by_pol(dst, pol)
//   edge(src, dst)            :- ingress_traffic(src, sel), egress_traffic(dst, sel)
// The host builds InT[sel][src] and EgT[sel][dst] as two kano matrices (one
// kano policy per (policy, peer)); here edge = EgT (self traffic) | In . EgT
// with In = InT transposed, the product run by k_path_or (kano_path.hpp) as
// one semi-naive step: edge[src] |= OR_{sel in In[src]} EgT[sel].
#pragma once

namespace kano {

// dst[c][rw] = bits X[64 rw + t][c], t = 0..63: X transposed into row-major
// bit rows (pitch ldd words).  One wave per 64 rows x 16 words of X: lane t
// loads its row's 16 words, 64 ballots transpose each 64 x 64 block, lane c
// stores column c's word.
__global__ __launch_bounds__(TPB) void k_k8s_transpose(const u64* __restrict__ X, i64 ldX,
                                                       i64 rows, i64 RW, i64 CG, i64 ncols,
                                                       u64* __restrict__ dst, i64 ldd) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= RW * CG) return;                        // wave-uniform
  const i64 rw = item / CG, cw0 = (item % CG) * 16;
  const i64 r = rw * 64 + lane;
  u64 x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = (r < rows && cw0 + k < ldX) ? X[r * ldX + cw0 + k] : 0ull;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if ((cw0 + k) * 64 >= ncols) break;               // wave-uniform
    u64 mine = 0;
#pragma unroll 8
    for (int c = 0; c < 64; ++c) {
      const u64 bal = __ballot((x[k] >> c) & 1ull);
      if (lane == c) mine = bal;
    }
    const i64 col = (cw0 + k) * 64 + lane;
    if (col < ncols) dst[col * ldd + rw] = mine;
  }
}

// M := every pair (kubesv's edge when check_select_by_no_policy holds and some
// pod is selected by no policy: constraint.py:207-212,222-227); pad bits and
// pad words zero.
__global__ __launch_bounds__(TPB) void k_k8s_ones(u64* __restrict__ M, i64 ldM, i64 rows, i64 n,
                                                 i64 W) {
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= rows * ldM) return;
  const i64 w = t % ldM;
  const int tail = (int)(n & 63);
  u64 v = 0;
  if (w < W) v = (w == W - 1 && tail) ? ((1ull << tail) - 1ull) : ~0ull;
  M[t] = v;
}

// ---------------------------------------------------------------------------
// Class-level form.  InT[sel][src] = Mc_i[rc_i(sel)][cc_i(src)] and
// EgT[sel][dst] = Mc_e[rc_e(sel)][cc_e(dst)] (row classes rc, column classes
// cc of the two builds), so
//   edge[src][dst] = Ec[cc_i(src)][cc_e(dst)] | Mc_e[rc_e(src)][cc_e(dst)] (self)
//   Ec[x] = OR_{a : Mc_i[a][x]} EgA[a],  EgA[a] = OR_{b in B[a]} Mc_e[b],
//   B[a]  = { rc_e(i) : rc_i(i) = a }   (the egress classes of in-class a's pods)
// -- two OR-products over classes, then one expansion to pods.
// ---------------------------------------------------------------------------

// B[a] bit b for every pod i with (rc_i(i), rc_e(i)) = (a, b)
__global__ __launch_bounds__(TPB) void k_k8s_pairs(const int32_t* __restrict__ rci,
                                                   const int32_t* __restrict__ rce, i64 n,
                                                   u64* __restrict__ B, i64 ldB) {
  const i64 i = (i64)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const i64 a = rci[i], b = rce[i];
  atomicOr(reinterpret_cast<unsigned long long*>(B + a * ldB + (b >> 6)), 1ull << (b & 63));
}

// out[r][w] = OR_{k in D[r]} T[k][w] for w < NW, 0 for NW <= w < ldO.  One wave
// per (row, 64*CW-word chunk); D rows hold KWd words.
template <int CW>
__global__ __launch_bounds__(TPB) void k_k8s_or_rows(const u64* __restrict__ D, i64 ldD, i64 KWd,
                                                     const u64* __restrict__ T, i64 ldT, i64 NW,
                                                     u64* __restrict__ out, i64 ldO, i64 rows,
                                                     i64 nch) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= rows * nch) return;                     // wave-uniform
  const i64 r = item / nch, w0 = (item % nch) * 64 * CW;
  u64 acc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) acc[k] = 0;
  const u64* drow = D + r * ldD;
  for (i64 kw0 = 0; kw0 < KWd; kw0 += 64) {
    const u64 dw = kw0 + lane < KWd ? drow[kw0 + lane] : 0ull;
    u64 nz = __ballot(dw != 0ull);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      u64 d = __shfl(dw, l, 64);
      const i64 kbase = (kw0 + l) * 64;
      while (d) {
        const u64* trow = T + (kbase + __builtin_ctzll(d)) * ldT;
        d &= d - 1;
#pragma unroll
        for (int k = 0; k < CW; ++k) {
          const i64 w = w0 + lane + 64 * k;
          if (w < NW) acc[k] |= trow[w];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CW; ++k) {
    const i64 w = w0 + lane + 64 * k;
    if (w < ldO) out[r * ldO + w] = w < NW ? acc[k] : 0ull;
  }
}

// Pod rows from class rows: a block is 16 words (1024 dst pods) x 64 src
// rows (local row r is pod g0 + r; cci == nullptr: row r is class r).  The 1024 column-class ids sit in LDS; per src row each lane gathers
// its pod's bit from the src's class row(s), a ballot packs 64 pods into one
// word, and lanes 0-15 store the row's 16 contiguous words (128 B).
constexpr int K8S_XW = 16, K8S_XR = 64, K8S_STAGE_W = 32;
// STAGE (class rows of <= K8S_STAGE_W words): the block's 64 class rows,
// OR-ed with their self-term rows, are staged in LDS first, so the per-pod
// gathers read LDS; each lane keeps its 16 column-class ids in registers.
template <bool STAGE>
__global__ __launch_bounds__(TPB) void k_k8s_expand(const u64* __restrict__ Ec, i64 ldE,
                                                    const int32_t* __restrict__ cci,
                                                    const u64* __restrict__ Mce, i64 ldCe,
                                                    const int32_t* __restrict__ rce,
                                                    const int32_t* __restrict__ cce, int self,
                                                    i64 g0, i64 rows, i64 n, i64 W,
                                                    u64* __restrict__ M, i64 ldM) {
  __shared__ int32_t cid[K8S_XW * 64];
  __shared__ u64 rowbuf[STAGE ? K8S_XR * K8S_STAGE_W : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 w0 = (i64)blockIdx.x * K8S_XW, r0 = (i64)blockIdx.y * K8S_XR;
  for (int t = threadIdx.x; t < K8S_XW * 64; t += TPB) {
    const i64 j = w0 * 64 + t;
    cid[t] = j < n ? cce[j] : -1;
  }
  const i64 r1 = r0 + K8S_XR < rows ? r0 + K8S_XR : rows;
  if (STAGE) {
    for (int t = threadIdx.x; t < K8S_XR * ldE; t += TPB) {
      const i64 rr = t / ldE, w = t % ldE, r = r0 + rr;
      u64 v = 0;
      if (r < r1) {
        v = Ec[(cci ? (i64)cci[g0 + r] : r) * ldE + w];
        if (self) v |= Mce[(i64)rce[g0 + r] * ldCe + w];
      }
      rowbuf[t] = v;
    }
  }
  __syncthreads();
  int cr[K8S_XW];
#pragma unroll
  for (int k = 0; k < K8S_XW; ++k) cr[k] = cid[k * 64 + lane];
  // wave wv takes rows r0 + wv, r0 + wv + 4, ...: all 16 words of each
  for (i64 r = r0 + wv; r < r1; r += TPB / 64) {
    const u64* er = STAGE ? rowbuf + (r - r0) * ldE
                          : Ec + (cci ? (i64)cci[g0 + r] : r) * ldE;
    const u64* sr = (!STAGE && self) ? Mce + (i64)rce[g0 + r] * ldCe : nullptr;
    u64 mine = 0;
#pragma unroll
    for (int k = 0; k < K8S_XW; ++k) {
      const int c = cr[k];
      int bit = 0;
      if (c >= 0) {
        u64 v = er[c >> 6];
        if (!STAGE && self) v |= sr[c >> 6];
        bit = (int)((v >> (c & 63)) & 1ull);
      }
      const u64 b = __ballot(bit);
      if (lane == k) mine = b;
    }
    if (lane < K8S_XW) {
      const i64 w = w0 + lane;
      if (w < ldM) M[r * ldM + w] = w < W ? mine : 0ull;
    }
  }
}

// M[r] = X[cci[g0 + r]] | S[rce[g0 + r]] (self) -- the expanded class rows
// streamed to the pod rows of a shard, 16 bytes per lane; S holds EgT by
// egress row class (the self term, ingress_traffic(sel, sel)).
__global__ __launch_bounds__(TPB) void k_k8s_rows(const u64* __restrict__ X,
                                                  const int32_t* __restrict__ cci,
                                                  const u64* __restrict__ S,
                                                  const int32_t* __restrict__ rce, int self,
                                                  i64 g0, i64 rows, i64 ldM,
                                                  u64* __restrict__ M) {
  const i64 h = ldM / 2;                                  // ldM is a multiple of 16
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= rows * h) return;
  const i64 r = t / h, q = t % h;
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  u64x2 v = reinterpret_cast<const u64x2*>(X + (i64)cci[g0 + r] * ldM)[q];
  if (self) v |= reinterpret_cast<const u64x2*>(S + (i64)rce[g0 + r] * ldM)[q];
  reinterpret_cast<u64x2*>(M + r * ldM)[q] = v;
}

// M[r] |= X[cci[g0 + r]]: the destination already holds EgT's rows of the
// shard (a build of the egress policies: the self term written by k_rows),
// the expanded Ec rows are OR-ed in place.
__global__ __launch_bounds__(TPB) void k_k8s_or_into(const u64* __restrict__ X,
                                                     const int32_t* __restrict__ cci, i64 g0,
                                                     i64 rows, i64 ldM, u64* __restrict__ M) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const i64 h = ldM / 2;
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= rows * h) return;
  const i64 r = t / h, q = t % h;
  u64x2* m = reinterpret_cast<u64x2*>(M + r * ldM) + q;
  *m |= reinterpret_cast<const u64x2*>(X + (i64)cci[g0 + r] * ldM)[q];
}


}  // namespace kano
