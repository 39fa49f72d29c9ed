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
__global__ __launch_bounds__(TPB) void k_k8s_ones(u64* __restrict__ M, i64 ldM, i64 n, i64 W) {
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= n * ldM) return;
  const i64 w = t % ldM;
  const int tail = (int)(n & 63);
  u64 v = 0;
  if (w < W) v = (w == W - 1 && tail) ? ((1ull << tail) - 1ull) : ~0ull;
  M[t] = v;
}

}  // namespace kano
