// kano_path.hpp -- multi-hop reachability over the built matrix (SURVEY.md
// §8(f) rank 3): kubesv's `path` relation (kubesv/kubesv/constraint.py:233-237,
// path :- edge; path :- edge o edge) with kano's M as `edge`, extended to
// paths of at most k edges and to the transitive closure.
//
// Everything runs at class level.  M[i, j] = Mc[rc(i), cc(j)] (row classes
// rc, column classes cc), so the pods reachable from row class r in at most
// k hops are a set of whole column classes R_k[r]:
//   R_1 = Mc,   R_{k+1}[r] = Mc[r] | OR_{b in R_k[r]} T[b],
//   T[b] = OR_{j : cc(j) = b} Mc[rc(j)]          (one hop out of class b)
// (every pod of a reached column class is reached, and the hop out of pod j
// depends on rc(j) only).  Two kernels compute the step:
//   * k_path_or: semi-naive bit-packed OR -- only the bits that are new in
//     R_k (the delta D_k) are expanded: R_{k+1} = R_k | OR_{b in D_k} T[b].
//   * k_path_mfma: the boolean contraction R_k . T as an int8 MFMA GEMM
//     (v_mfma_i32_32x32x32_i8) on bits expanded in registers, thresholded
//     > 0 and OR-ed with Mc in the epilogue (dense R_k).
// k_path_expand writes the pod matrix: P[i] bit j = R[rc(i)][cc(j)].
// After an edit of M the classes are the pods themselves (identity).
#pragma once
#include "kano_prims.hpp"

namespace kano {

// T[b] = OR of Mc[rc(j)] over the members j of column class b.  One wave per
// (class, chunk of 64*CW words); consecutive members of one row class are
// read once.
template <int CW>
__global__ __launch_bounds__(TPB) void k_path_t(const u64* __restrict__ Mc, i64 ldC,
                                                const int32_t* __restrict__ rcls,
                                                const int32_t* __restrict__ moff,
                                                const int32_t* __restrict__ mem, i64 Ua,
                                                i64 KW, i64 nch, u64* __restrict__ T) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= Ua * nch) return;                       // wave-uniform
  const i64 b = item / nch, w0 = (item % nch) * 64 * CW;
  u64 acc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) acc[k] = 0;
  int32_t prev = -1;
  for (int32_t m = moff[b]; m < moff[b + 1]; ++m) {
    const int32_t r = rcls[mem[m]];
    if (r == prev) continue;
    prev = r;
    const u64* src = Mc + (i64)r * ldC;
#pragma unroll
    for (int k = 0; k < CW; ++k) {
      const i64 w = w0 + lane + 64 * k;
      if (w < KW) acc[k] |= src[w];
    }
  }
#pragma unroll
  for (int k = 0; k < CW; ++k) {
    const i64 w = w0 + lane + 64 * k;
    if (w < ldC) T[b * ldC + w] = acc[k];
  }
}

// One semi-naive step.  Wave = (row r, chunk of 64*CW words): new bits
// acc = OR_{b in D[r]} T[b] over the chunk, Dn[r] = acc & ~R[r], R[r] |= Dn[r];
// cnt += popcount(Dn) (one atomic per wave).  D and Dn have pitch ldR, T ldT.
template <int CW>
__global__ __launch_bounds__(TPB) void k_path_or(const u64* __restrict__ D, u64* __restrict__ R,
                                                 u64* __restrict__ Dn, i64 ldR,
                                                 const u64* __restrict__ T, i64 ldT, i64 rows,
                                                 i64 KW, i64 nch, u64* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= rows * nch) return;                     // wave-uniform
  const i64 r = item / nch, w0 = (item % nch) * 64 * CW;
  u64 acc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) acc[k] = 0;
  const u64* drow = D + r * ldR;
  for (i64 kw0 = 0; kw0 < KW; kw0 += 64) {
    const u64 dw = kw0 + lane < KW ? drow[kw0 + lane] : 0ull;
    u64 nz = __ballot(dw != 0ull);
    while (nz) {
      const int l = __builtin_ctzll(nz);
      nz &= nz - 1;
      u64 d = __shfl(dw, l, 64);
      const i64 bbase = (kw0 + l) * 64;
      while (d) {
        const i64 b = bbase + __builtin_ctzll(d);
        d &= d - 1;
        const u64* trow = T + b * ldT;
#pragma unroll
        for (int k = 0; k < CW; ++k) {
          const i64 w = w0 + lane + 64 * k;
          if (w < KW) acc[k] |= trow[w];
        }
      }
    }
  }
  int pc = 0;
#pragma unroll
  for (int k = 0; k < CW; ++k) {
    const i64 w = w0 + lane + 64 * k;
    if (w < ldR) {
      const u64 old = R[r * ldR + w];
      const u64 nd = w < KW ? acc[k] & ~old : 0ull;
      if (nd) R[r * ldR + w] = old | nd;
      Dn[r * ldR + w] = nd;
      pc += __popcll(nd);
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pc += __shfl_xor(pc, d, 64);
  if (lane == 0 && pc) atomicAdd(cnt, (u64)pc);
}

// dst[kw][r] = src[r][kw]: word transpose through a 64 x 64 LDS tile; rows
// in [rows, ldd) and words past KW are written as zero.
__global__ __launch_bounds__(TPB) void k_word_transpose(const u64* __restrict__ src, i64 lds,
                                                        i64 rows, i64 KW, u64* __restrict__ dst,
                                                        i64 ldd, i64 KWd) {
  __shared__ u64 s[64][65];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 kw0 = (i64)blockIdx.x * 64, r0 = (i64)blockIdx.y * 64;
  for (int i = wv; i < 64; i += TPB / 64) {
    const i64 r = r0 + i, kw = kw0 + lane;
    s[i][lane] = (r < rows && kw < KW) ? src[r * lds + kw] : 0ull;
  }
  __syncthreads();
  for (int i = wv; i < 64; i += TPB / 64) {
    const i64 kw = kw0 + i, r = r0 + lane;
    if (kw < KWd && r < ldd) dst[kw * ldd + r] = s[lane][i];
  }
}

// Bit transpose of T (rows b, columns c): dst[kw][c] bit t = T[64*kw + t][c].
// One wave per 64 x 64 bit block: lane t holds row 64*kw + t, 64 ballots
// give the transposed words, lane c keeps word c.
__global__ __launch_bounds__(TPB) void k_bit_transpose(const u64* __restrict__ T, i64 ldT,
                                                       i64 rowsT, i64 KW, i64 CWn,
                                                       u64* __restrict__ dst, i64 ldd) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= KW * CWn) return;                       // wave-uniform
  const i64 kw = item / CWn, cw = item % CWn;
  const i64 b = kw * 64 + lane;
  const u64 x = (b < rowsT && cw < ldT) ? T[b * ldT + cw] : 0ull;
  u64 mine = 0;
#pragma unroll 8
  for (int c = 0; c < 64; ++c) {
    const u64 bal = __ballot((x >> c) & 1ull);
    if (lane == c) mine = bal;
  }
  const i64 col = cw * 64 + lane;
  if (col < ldd) dst[kw * ldd + col] = mine;
}

typedef int32_t p_i32x16 __attribute__((ext_vector_type(16)));
typedef int32_t p_i32x4 __attribute__((ext_vector_type(4)));

// 16 bits -> 16 int8 lanes of 0 / 1 (bit t -> byte t)
__device__ __forceinline__ uint32_t pspread4(uint32_t b4) {
  return (b4 & 1u) | ((b4 & 2u) << 7) | ((b4 & 4u) << 14) | ((b4 & 8u) << 21);
}
__device__ __forceinline__ p_i32x4 pexpand16(uint32_t b16) {
  p_i32x4 r;
  r[0] = (int32_t)pspread4(b16 & 15u);
  r[1] = (int32_t)pspread4((b16 >> 4) & 15u);
  r[2] = (int32_t)pspread4((b16 >> 8) & 15u);
  r[3] = (int32_t)pspread4((b16 >> 12) & 15u);
  return r;
}

struct PathMfmaArgs {
  const u64* A;      // [KW][ldA]: R_k word-transposed (rows = row classes)
  const u64* B;      // [KW][ldB]: T bit-transposed (columns = column classes)
  i64 ldA, ldB, KW;
  const u64* base;   // Mc (pitch ldR): OR-ed into the product
  const u64* old;    // R_k (pitch ldR): for the change count
  u64* out;          // R_{k+1} (pitch ldR)
  u64* delta;        // R_{k+1} & ~R_k (pitch ldR): the next semi-naive step's input
  i64 ldR, rows, tiles_n;
  u64* cnt;          // bits of R_{k+1} not in R_k
};

// R_{k+1} = Mc | (R_k . T > 0).  One wave = (32*TM rows) x (32*TN columns);
// K = 64 column classes per step, two v_mfma_i32_32x32x32_i8 per tile pair.
// A and B fragments are the same 16-bit slices of their words expanded to
// int8 0/1 (the same k order on both sides gives the same dot product).
template <int TM, int TN>
__global__ __launch_bounds__(TPB) void k_path_mfma(PathMfmaArgs a) {
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const i64 wave = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const i64 tm = wave / a.tiles_n, tn = wave % a.tiles_n;
  const i64 rb = tm * 32 * TM, cb = tn * 32 * TN;
  if (rb >= a.ldA) return;                            // wave-uniform
  p_i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  const u64* pa = a.A + rb + l32;
  const u64* pb = a.B + cb + l32;
  for (i64 kw = 0; kw < a.KW; ++kw) {
    u64 aw[TM], bw[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) aw[t] = pa[kw * a.ldA + 32 * t];
#pragma unroll
    for (int u = 0; u < TN; ++u) bw[u] = pb[kw * a.ldB + 32 * u];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int sh = ks * 32 + half * 16;
      p_i32x4 af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) af[t] = pexpand16((uint32_t)(aw[t] >> sh) & 0xffffu);
#pragma unroll
      for (int u = 0; u < TN; ++u) bf[u] = pexpand16((uint32_t)(bw[u] >> sh) & 0xffffu);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], bf[u], acc[t][u], 0, 0, 0);
    }
  }
  // epilogue: accumulator g of lane (l32, half) is row (g&3) + 8*(g>>2) +
  // 4*half, column l32 of its tile; one ballot per g gives 32 columns of two
  // rows (lanes 0-31: half 0, lanes 32-63: half 1)
  const uint32_t* base32 = reinterpret_cast<const uint32_t*>(a.base);
  const uint32_t* old32 = reinterpret_cast<const uint32_t*>(a.old);
  uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out);
  const i64 ld32 = 2 * a.ldR;
  int pc = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const i64 c32 = (cb + 32 * u) >> 5;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const u64 bal = __ballot(acc[t][u][g] > 0);
        if (l32 == 0) {
          const i64 row = rb + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
          if (row < a.rows && c32 < ld32) {
            const uint32_t w = (half ? (uint32_t)(bal >> 32) : (uint32_t)bal) |
                               base32[row * ld32 + c32];
            const uint32_t nd = w & ~old32[row * ld32 + c32];
            out32[row * ld32 + c32] = w;
            reinterpret_cast<uint32_t*>(a.delta)[row * ld32 + c32] = nd;
            pc += __builtin_popcount(nd);
          }
        }
      }
    }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pc += __shfl_xor(pc, d, 64);
  if (lane == 0 && pc) atomicAdd(a.cnt, (u64)pc);
}

// cnt += popcount of words [0, nw)
__global__ __launch_bounds__(TPB) void k_popcount_words(const u64* __restrict__ w, i64 nw,
                                                        u64* __restrict__ cnt) {
  u64 pc = 0;
  for (i64 i = (i64)blockIdx.x * TPB + threadIdx.x; i < nw; i += (i64)gridDim.x * TPB)
    pc += __popcll(w[i]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pc += __shfl_xor(pc, d, 64);
  if ((threadIdx.x & 63) == 0 && pc) atomicAdd(cnt, pc);
}

// P[i] bit j = R[rc(i)][cc(j)] for the members i of row classes
// [blockIdx.y * RT, + RT), words [blockIdx.x * 256, + 256) (64 per wave).
// Lane l of a wave holds the column classes of pod 64 * (w + s) + l for its
// 64 words s; per row class the row is staged in LDS, 64 ballots give the
// wave's 64 words (lane s keeps word s) and each member row gets one
// 512-byte store.
template <int RT>
__global__ __launch_bounds__(TPB) void k_path_expand(const u64* __restrict__ R, i64 ldR,
                                                     i64 rows, const int32_t* __restrict__ ccls,
                                                     i64 n, const int32_t* __restrict__ moff,
                                                     const int32_t* __restrict__ mem,
                                                     u64* __restrict__ M, i64 ldM) {
  extern __shared__ u64 row[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 wb = (i64)blockIdx.x * TPB + wv * 64;     // first word of this wave
  int32_t cid[64];
#pragma unroll
  for (int s = 0; s < 64; ++s) {
    const i64 j = (wb + s) * 64 + lane;
    cid[s] = j < n ? ccls[j] : -1;
  }
  const i64 c0 = (i64)blockIdx.y * RT, c1 = c0 + RT < rows ? c0 + RT : rows;
  for (i64 c = c0; c < c1; ++c) {
    __syncthreads();
    for (i64 w = threadIdx.x; w < ldR; w += TPB) row[w] = R[c * ldR + w];
    __syncthreads();
    u64 mine = 0;
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int32_t b = cid[s];
      const bool bit = b >= 0 && ((row[b >> 6] >> (b & 63)) & 1ull);
      const u64 bal = __ballot(bit);
      if (lane == s) mine = bal;
    }
    if (wb + lane < ldM) {
      for (int32_t m = moff[c]; m < moff[c + 1]; ++m) M[(i64)mem[m] * ldM + wb + lane] = mine;
    }
  }
}

}  // namespace kano
