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
//   * k_path_mfma: the boolean contraction R_k . T as an MFMA GEMM on the
//     block-scaled fp4 form (v_mfma_scale_f32_32x32x64_f8f6f4) over bits
//     expanded in registers, thresholded > 0 and OR-ed with Mc in the
//     epilogue (dense R_k).
// k_path_expand writes the pod matrix: P[i] bit j = R[rc(i)][cc(j)].
// After an edit of M the classes are the pods themselves (identity).
#pragma once
#include "kano_prims.hpp"

namespace kano {

// step counters: one 128-byte line per slot, waves spread over the slots
// (same-address atomics from every wave serialise)
constexpr int PATH_CNT_SLOTS = 256, PATH_CNT_STRIDE = 16;
__device__ __forceinline__ void path_count(u64* cnt, u64 v) {
  const unsigned slot = (blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)) & (PATH_CNT_SLOTS - 1);
  if (v) atomicAdd(cnt + slot * PATH_CNT_STRIDE, v);
}

// T[b] = OR of Mc[rc(j)] over the members j of column class b.  One wave per
// (class, chunk of 64*CW words); consecutive members of one row class are
// read once.
template <int CW>
__global__ __launch_bounds__(TPB) void k_path_t(const u64* __restrict__ Mc, i64 ldC,
                                                const int32_t* __restrict__ rcls,
                                                const int32_t* __restrict__ moff,
                                                const int32_t* __restrict__ mem, i64 Ua,
                                                i64 KW, i64 nch, i64 r0, i64 r1,
                                                u64* __restrict__ T) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= Ua * nch) return;                       // wave-uniform
  const i64 b = item / nch, w0 = (item % nch) * 64 * CW;
  u64 acc[CW];
#pragma unroll
  for (int k = 0; k < CW; ++k) acc[k] = 0;
  int32_t prev = -1;
  for (int32_t m = moff[b]; m < moff[b + 1]; ++m) {
    const int32_t j = mem[m];
    if (j < r0 || j >= r1) continue;                  // a row shard: its own pods only
    const int32_t r = rcls[j];
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

// The same for narrow class rows (KW <= 4 words) and large classes: the 64
// lanes of a wave split the class's members, each ORs its members' Mc rows
// into registers, and the wave reduces.  One wave per column class.
// Work item = (class b, slice of 64 * NT_SLICE members): the wave ORs into T
// (zeroed) with one atomic per word, so large classes spread over many waves.
constexpr int NT_SLICE = 4;
__global__ __launch_bounds__(TPB) void k_path_t_narrow(const u64* __restrict__ Mc, i64 ldC,
                                                       const int32_t* __restrict__ rcls,
                                                       const int32_t* __restrict__ moff,
                                                       const int32_t* __restrict__ mem, i64 Ua,
                                                       i64 KW, const int32_t* __restrict__ ioff,
                                                       i64 nitems, i64 r0, i64 r1,
                                                       u64* __restrict__ T) {
  const int lane = threadIdx.x & 63;
  const i64 item = (i64)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  if (item >= nitems) return;                         // wave-uniform
  // class of this item: ioff[b] = first item of class b (binary search)
  i64 lo = 0, hi = Ua - 1;
  while (lo < hi) {
    const i64 mid = (lo + hi + 1) >> 1;
    if (ioff[mid] <= item) lo = mid; else hi = mid - 1;
  }
  const i64 b = lo;
  const int32_t mb = moff[b] + (int32_t)(item - ioff[b]) * 64 * NT_SLICE;
  const int32_t me = min(moff[b + 1], mb + 64 * NT_SLICE);
  u64 acc[4] = {0, 0, 0, 0};
  int32_t prev = -1;
  for (int32_t m = mb + lane; m < me; m += 64) {
    const int32_t j = mem[m];
    if (j < r0 || j >= r1) continue;
    const int32_t r = rcls[j];
    if (r == prev) continue;
    prev = r;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < KW) acc[k] |= Mc[(i64)r * ldC + k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc[k] |= __shfl_xor(acc[k], d, 64);
  }
  const u64 mine = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
  if (lane < KW && lane < 4 && mine) atomicOr(T + b * ldC + lane, mine);
}

// items per class for k_path_t_narrow: ioff[b] = sum_{b' < b} ceil(size / slice)
// (one block, serial scan over Ua <= a few thousand classes is not needed:
// a wave-wide scan per 64 classes)
__global__ __launch_bounds__(TPB) void k_path_t_items(const int32_t* __restrict__ moff, i64 Ua,
                                                      int32_t* __restrict__ ioff) {
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (i64 b0 = 0; b0 <= Ua; b0 += TPB) {
    const i64 b = b0 + threadIdx.x;
    int32_t v = 0;
    if (b < Ua) {
      const int32_t sz = moff[b + 1] - moff[b];
      v = sz > 0 ? (sz + 64 * NT_SLICE - 1) / (64 * NT_SLICE) : 0;
    }
    __shared__ int32_t tmp[TPB / 64];
    int32_t total;
    const int32_t ex = block_excl_scan(v, tmp, total);
    if (b <= Ua) ioff[b] = carry + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry += total;
    __syncthreads();
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
  if (lane == 0) path_count(cnt, (u64)pc);
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

// Bit transpose of a bit matrix X (rows r < rows, pitch ldX words):
// out word (rw, c) = bits X[64 rw + t][c], t = 0..63.  One wave per 64 rows x
// 16 words: lane t loads its row's 16 words (one 128-byte line), 64 ballots
// per word transpose the 64 x 64 block, lane c keeps word c.  OUT16 stores
// each transposed word as four 16-row groups dst16[4 rw + q][c], else
// dst[rw][c] (ldd = columns per output row).
template <bool OUT16>
__global__ __launch_bounds__(TPB) void k_bit_transpose(const u64* __restrict__ X, i64 ldX,
                                                       i64 rows, i64 RW, i64 CG, i64 ncols,
                                                       void* __restrict__ dstv, i64 ldd,
                                                       i64 ngroups) {
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
    if (cw0 + k >= (ncols + 63) / 64) break;          // wave-uniform
    u64 mine = 0;
#pragma unroll 8
    for (int c = 0; c < 64; ++c) {
      const u64 bal = __ballot((x[k] >> c) & 1ull);
      if (lane == c) mine = bal;
    }
    const i64 col = (cw0 + k) * 64 + lane;
    if (col < ldd) {
      if (OUT16) {
        uint16_t* dst = reinterpret_cast<uint16_t*>(dstv);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const i64 g = rw * 4 + q;
          if (g < ngroups) dst[g * ldd + col] = (uint16_t)(mine >> (16 * q));
        }
      } else {
        reinterpret_cast<u64*>(dstv)[rw * ldd + col] = mine;
      }
    }
  }
}

typedef float p_f32x16 __attribute__((ext_vector_type(16)));
typedef int32_t p_i32x8 __attribute__((ext_vector_type(8)));

// 32 bits -> the block-scaled fp4 MFMA's operand (e2m1, unit scales): nibble
// j of register v holds bit 4 j + v in place (0.5 / 1.0 / 2.0) or, for the
// nibble's sign bit, moved down one (2.0); every element is 0 or positive
// (kano_kernels.hpp bits_to_fp4, the same map)
__device__ __forceinline__ p_i32x8 pbits_to_fp4(uint32_t x) {
  p_i32x8 r;
  r[0] = (int32_t)(x & 0x11111111u);
  r[1] = (int32_t)(x & 0x22222222u);
  r[2] = (int32_t)(x & 0x44444444u);
  r[3] = (int32_t)((x >> 1) & 0x44444444u);
  r[4] = r[5] = r[6] = r[7] = 0;
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
  i64 ldR, rows, tiles_n;   // tiles_n = 32 TN-column tiles (even); ldA = a multiple of 64 TM
  u64* cnt;          // bits of R_{k+1} not in R_k
};

// R_{k+1} = Mc | (R_k . T > 0).  One wave = (32*TM rows) x (32*TN columns);
// K = 64 column classes per step, one v_mfma_scale_f32_32x32x64_f8f6f4 per
// tile pair (fp4 operands, f32 sums of positive terms: > 0 iff some k has
// both bits).  Lane half h takes bits 32 h .. 32 h + 31 of its A and B words
// (the same k order on both sides gives the same dot product).
template <int TM, int TN>
__global__ __launch_bounds__(TPB) void k_path_mfma(PathMfmaArgs a) {
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  // block = 2 x 2 waves; blocks of one XCD (blockIdx.x mod 8 under the
  // round-robin dispatch) take one contiguous range of the block order, which
  // walks GM block-rows at a time column by column, so that the blocks
  // resident on an XCD share A and B panels in its L2
  constexpr i64 GM = 8;
  const i64 nbm = a.ldA / (64 * TM), nbn = a.tiles_n / 2, total = nbm * nbn;
  const i64 per = (total + 7) / 8;
  const i64 L = (i64)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= total) return;                             // block-uniform
  const i64 grp = L / (GM * nbn), first = grp * GM;
  const i64 gm = nbm - first < GM ? nbm - first : GM;
  const i64 in = L - grp * GM * nbn;
  const i64 bm = first + in % gm, bn = in / gm;
  const int wv = threadIdx.x >> 6;
  const i64 tm = bm * 2 + (wv >> 1), tn = bn * 2 + (wv & 1);
  const i64 rb = tm * 32 * TM, cb = tn * 32 * TN;
  if (rb >= a.ldA) return;                            // wave-uniform
  p_f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
  // (the lane's 32-bit half of each word)
  const uint32_t* pa = reinterpret_cast<const uint32_t*>(a.A + rb + l32) + half;
  const uint32_t* pb = reinterpret_cast<const uint32_t*>(a.B + cb + l32) + half;
  for (i64 kw = 0; kw < a.KW; ++kw) {
    p_i32x8 af[TM], bf[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) af[t] = pbits_to_fp4(pa[2 * (kw * a.ldA + 32 * t)]);
#pragma unroll
    for (int u = 0; u < TN; ++u) bf[u] = pbits_to_fp4(pb[2 * (kw * a.ldB + 32 * u)]);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[t], bf[u], acc[t][u], 4, 4,
                                                                    0, 127, 0, 127);
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
        const u64 bal = __ballot(acc[t][u][g] > 0.f);
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
  if (lane == 0) path_count(a.cnt, (u64)pc);
}

// cnt += popcount of words [0, nw)
__global__ __launch_bounds__(TPB) void k_popcount_words(const u64* __restrict__ w, i64 nw,
                                                        u64* __restrict__ cnt) {
  u64 pc = 0;
  for (i64 i = (i64)blockIdx.x * TPB + threadIdx.x; i < nw; i += (i64)gridDim.x * TPB)
    pc += __popcll(w[i]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pc += __shfl_xor(pc, d, 64);
  if ((threadIdx.x & 63) == 0) path_count(cnt, pc);
}

// P[i] bit j = R[rc(i)][cc(j)].  Block = (16 row classes of group
// blockIdx.y, words [blockIdx.x * 256 * SUB, + 256 * SUB), member slice z of
// Z = gridDim.z: member k of a class goes to slice k mod Z, so that few large
// classes (broad selectors) still fill the chip).  The group's bits per
// column class (tab[c], 16 bits, from k_bit_transpose<true>) sit in LDS
// (USE_LDS) or are read from L2.  Per 256-word chunk, lane l of wave v owns
// word w = 64 v + l: it loads the column classes of its 64 pods (all loads in
// flight), looks up their 16-bit entries and packs bit t of entry k into bit
// k of class t's word, kept in LDS.  Then the waves stream the chunk to the
// member rows, one 2-KB row piece per wave at a time (16-byte stores) --
// STAGED, for large classes; otherwise each lane stores its own word to every
// member row right away (512 bytes per wave store; measured faster with ~5
// members per class, C3: 0.42 vs 0.50 ms; staged C4: 0.45 vs 0.72 ms).
template <int SUB, bool USE_LDS, bool STAGED>
__global__ __launch_bounds__(TPB) void k_path_expand16(const uint16_t* __restrict__ RT16, i64 Ua,
                                                       i64 rows, const int32_t* __restrict__ ccls,
                                                       i64 n, const int32_t* __restrict__ moff,
                                                       const int32_t* __restrict__ mem,
                                                       u64* __restrict__ M, i64 ldM, i64 r0) {
  const int32_t Z = (int32_t)gridDim.z, z = (int32_t)blockIdx.z;
  extern __shared__ uint16_t tab[];
  __shared__ u64 cw[STAGED ? 16 : 1][TPB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const i64 g = blockIdx.y;
  const uint16_t* grow = RT16 + g * Ua;
  if (USE_LDS) {
    for (i64 c = threadIdx.x; c < Ua; c += TPB) tab[c] = grow[c];
    __syncthreads();
  }
  const int nc = (int)(rows - 16 * g < 16 ? rows - 16 * g : 16);
  for (int sub = 0; sub < SUB; ++sub) {
    const i64 cb = ((i64)blockIdx.x * SUB + sub) * TPB;   // first word of the chunk
    if (cb >= ldM) break;                                 // block-uniform
    const i64 w = cb + wv * 64 + lane, j0 = w * 64;
    uint32_t x[64];
    if (j0 + 64 <= n) {
      const int4* src = reinterpret_cast<const int4*>(ccls + j0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int4 v = src[q];
        x[4 * q] = (uint32_t)v.x;
        x[4 * q + 1] = (uint32_t)v.y;
        x[4 * q + 2] = (uint32_t)v.z;
        x[4 * q + 3] = (uint32_t)v.w;
      }
#pragma unroll
      for (int k = 0; k < 64; ++k) x[k] = USE_LDS ? tab[x[k]] : grow[x[k]];
    } else {
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        const i64 j = j0 + k;
        x[k] = j < n ? (USE_LDS ? tab[ccls[j]] : grow[ccls[j]]) : 0u;
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        lo |= ((x[k] >> t) & 1u) << k;
        hi |= ((x[k + 32] >> t) & 1u) << k;
      }
      const u64 word = ((u64)hi << 32) | lo;
      if (STAGED) {
        cw[t][wv * 64 + lane] = word;
      } else if (t < nc && w < ldM) {
        const i64 c = 16 * g + t;
        const int32_t m1 = moff[c + 1];
        int32_t m = moff[c] + z;
        for (; m + 3 * Z < m1; m += 4 * Z) {   // four member rows' stores in flight
          const int32_t a0 = mem[m], a1 = mem[m + Z], a2 = mem[m + 2 * Z], a3 = mem[m + 3 * Z];
          M[(a0 - r0) * ldM + w] = word;
          M[(a1 - r0) * ldM + w] = word;
          M[(a2 - r0) * ldM + w] = word;
          M[(a3 - r0) * ldM + w] = word;
        }
        for (; m < m1; m += Z) M[(mem[m] - r0) * ldM + w] = word;
      }
    }
    if (!STAGED) continue;
    __syncthreads();
    // stream: the (class, member) pieces of this slice, round-robin over waves
    const i64 nw = ldM - cb < TPB ? ldM - cb : TPB;       // words in this chunk
    int q = 0;
    for (int t = 0; t < nc; ++t) {
      const i64 c = 16 * g + t;
      const int32_t m1 = moff[c + 1];
      for (int32_t m = moff[c] + z; m < m1; m += Z, ++q) {
        if ((q & 3) != wv) continue;
        u64* dst = M + (mem[m] - r0) * ldM + cb;
#pragma unroll
        for (int h = 0; h < TPB / 128; ++h) {
          const int k = 2 * (h * 64 + lane);
          if (k + 1 < nw) {
            u64x2 v;
            v.x = cw[t][k];
            v.y = cw[t][k + 1];
            *reinterpret_cast<u64x2*>(dst + k) = v;
          } else if (k < nw) {
            dst[k] = cw[t][k];
          }
        }
      }
    }
    __syncthreads();
  }
}

// bitarray byte rows (kano_py's M rows, model.py:136-139,158-160, bitarray's
// default big-endian bit order: bit j -> byte j >> 3, bit 7 - (j & 7)) from
// LSB-first words and back.  One thread per 4 bytes of a row of nb bytes.
__global__ __launch_bounds__(TPB) void k_words_to_bytes(const u64* __restrict__ M, i64 ldM,
                                                        i64 nrows, i64 nb,
                                                        uint8_t* __restrict__ out) {
  const i64 q = (nb + 3) / 4;
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= nrows * q) return;
  const i64 r = t / q, k0 = (t % q) * 4;
  const uint32_t w = reinterpret_cast<const uint32_t*>(M + r * ldM)[k0 >> 2];
  // reverse the bits inside every byte: reverse the dword, then its bytes
  const uint32_t v = __builtin_bswap32(__builtin_bitreverse32(w));
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (k0 + b < nb) out[r * nb + k0 + b] = (uint8_t)(v >> (8 * b));
}

__global__ __launch_bounds__(TPB) void k_bytes_to_words(const uint8_t* __restrict__ in, i64 nrows,
                                                        i64 nb, i64 nbits,
                                                        u64* __restrict__ M, i64 ldM) {
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= nrows * ldM) return;
  const i64 r = t / ldM, w = t % ldM;
  u64 x = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const i64 k = w * 8 + b;
    if (k < nb) x |= (u64)__builtin_bitreverse8(in[r * nb + k]) << (8 * b);
  }
  // pad bits past the row's length stay zero (bitarray zeroes them in
  // tobytes(); a file may carry anything there)
  const i64 j0 = w * 64;
  if (j0 + 64 > nbits) x = j0 >= nbits ? 0ull : x & ((1ull << (nbits - j0)) - 1ull);
  M[r * ldM + w] = x;
}

// T = OR of the ranks' parts (gathered rank-major, nw words each)
__global__ __launch_bounds__(TPB) void k_or_parts(const u64* __restrict__ parts, int32_t nranks,
                                                  i64 nw, u64* __restrict__ out) {
  for (i64 w = (i64)blockIdx.x * TPB + threadIdx.x; w < nw; w += (i64)gridDim.x * TPB) {
    u64 x = 0;
    for (int32_t r = 0; r < nranks; ++r) x |= parts[(i64)r * nw + w];
    out[w] = x;
  }
}

}  // namespace kano
