// kano_expand.hpp -- the matrix write (kano_py/kano/model.py:158-160) from the
// class-level matrix, in address order.
//
// M[i][j] = Mc[rc(i)][cc(j)]: row i's bits are its row class's Mc row read
// through the column class of every pod j.  A block owns 32 consecutive rows
// of M (one contiguous 32 * ldM-word tile) and writes them word column by
// word column, so the chip sweeps M in address order with 512-byte wave
// stores -- the store shape the write-rate micro measured fastest (DESIGN.md,
// "the matrix write").  Per tile:
//   table   T[b] (32 bits, one per tile row): bit r = Mc[rc(row r)][b], for
//           every column class b; built in LDS from the 32 Mc rows by 32 x 32
//           bit transposes of their words.
//   expand  lane w: the column classes of pods 64w .. 64w+63, their 64 table
//           entries (bit r = M[row r][pod]), two 32 x 32 bit transposes ->
//           word w of all 32 rows, 32 stores (each wave store covers 512
//           contiguous bytes of one row).
// Per output word: 2 LDS lookups, ~20 VALU ops, no global reads beyond the
// column-class ids (L2-resident) and the tile's Mc rows.
#pragma once
#include "kano_prims.hpp"

namespace kano {

// In-place 32 x 32 bit transpose: afterwards a[k] bit r == (before) a[r] bit k.
// Block-swap recursion (16, 8, 4, 2, 1): swapping the off-diagonal j x j blocks
// of each 2j x 2j block transposes the matrix once the recursion bottoms out.
__host__ __device__ __forceinline__ void transpose32(uint32_t* a) {
#define KANO_T32_STAGE(J, MASK)                                  \
  _Pragma("unroll") for (int r = 0; r < 32; ++r) {               \
    if (r & (J)) continue;                                       \
    const uint32_t t = ((a[r] >> (J)) ^ a[r + (J)]) & (MASK);    \
    a[r + (J)] ^= t;                                             \
    a[r] ^= t << (J);                                            \
  }
  KANO_T32_STAGE(16, 0x0000FFFFu)
  KANO_T32_STAGE(8, 0x00FF00FFu)
  KANO_T32_STAGE(4, 0x0F0F0F0Fu)
  KANO_T32_STAGE(2, 0x33333333u)
  KANO_T32_STAGE(1, 0x55555555u)
#undef KANO_T32_STAGE
}

constexpr int XR = 32;   // rows of M per tile (bits of a table entry)

// LDS position of table entry b: one pad word per 64 entries, so that the
// table build's lanes (64 consecutive entries each) write to distinct banks
__device__ __forceinline__ uint32_t tpos(uint32_t b) { return b + (b >> 6); }
inline size_t rows_mc_lds_bytes(int64_t Ua) {
  return sizeof(uint32_t) * (size_t)(Ua + 1 + (Ua + 1) / 64 + 1);
}

struct RowsMcArgs {
  const u64* Mc;         // row classes x ldC words (column-class bits)
  i64 ldC;
  i64 UAW;               // words of a class-level row that hold column classes
  i64 Ua;                // column classes (entry Ua of the table is the all-zero sentinel)
  const int32_t* rcls;   // row class of pod i (global index; rows r0 .. r0+rl)
  const void* cct;       // column classes word-transposed: cct[j * ldM + w] = class of pod
                         // 64w + j (Ua past the last pod); uint16_t when Ua < 65535, else int32
  i64 ldM;               // M row pitch (words); words W .. ldM-1 come out 0
  i64 r0, rl;            // the rows held: [r0, r0 + rl)
  u64* M;                // local row r at M + r * ldM
};

// the column classes of every pod, word-transposed (k_rows_mc's lanes read
// pod j of word w at cct[j * ldM + w]: 64 coalesced loads per lane)
template <typename IdT>
__global__ __launch_bounds__(TPB) void k_cc_transpose(const int32_t* __restrict__ ccls, i64 n,
                                                      i64 ldM, int32_t Ua, IdT* __restrict__ cct) {
  const i64 t = (i64)blockIdx.x * TPB + threadIdx.x;
  if (t >= 64 * ldM) return;
  const i64 j = t / ldM, w = t - j * ldM;
  const i64 pod = w * 64 + j;
  cct[t] = (IdT)(pod < n ? ccls[pod] : Ua);
}

// the 32 x 32 bit transposes of one table word column: Mc words q of the
// tile's rows -> T[64q .. 64q+63]
__device__ __forceinline__ void rows_mc_table_word(const RowsMcArgs& a, const int32_t* rc, i64 q,
                                                   uint32_t* T) {
  uint32_t lo[32], hi[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    const int32_t c = rc[r];
    const u64 v = c >= 0 ? a.Mc[(i64)c * a.ldC + q] : 0ull;
    lo[r] = (uint32_t)v;
    hi[r] = (uint32_t)(v >> 32);
  }
  transpose32(lo);
  transpose32(hi);
  const uint32_t b0 = (uint32_t)q * 64;
  uint32_t* t0 = T + tpos(b0);   // entries b0 .. b0+63 are contiguous (one pad word after)
  if (b0 + 64 <= (uint32_t)a.Ua) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      t0[k] = lo[k];
      t0[32 + k] = hi[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (b0 + k < (uint32_t)a.Ua) t0[k] = lo[k];
      if (b0 + 32 + k < (uint32_t)a.Ua) t0[32 + k] = hi[k];
    }
  }
}

template <int NT, typename IdT>
__global__ __launch_bounds__(NT) void k_rows_mc(RowsMcArgs a) {
  extern __shared__ uint32_t T[];    // tpos(0 .. Ua) entries
  __shared__ int32_t rc[XR];
  const i64 t0 = (i64)blockIdx.x * XR;          // first local row of the tile
  const int nr = (int)min((i64)XR, a.rl - t0);  // block-uniform
  if (nr <= 0) return;
  if (threadIdx.x < XR) rc[threadIdx.x] = (int)threadIdx.x < nr ? a.rcls[a.r0 + t0 + threadIdx.x] : -1;
  if (threadIdx.x == 0) T[tpos((uint32_t)a.Ua)] = 0u;   // the sentinel past the last pod
  __syncthreads();
  for (i64 q = threadIdx.x; q < a.UAW; q += NT) rows_mc_table_word(a, rc, q, T);
  __syncthreads();
  const IdT* __restrict__ cct = static_cast<const IdT*>(a.cct);
  u64* __restrict__ out = a.M + t0 * a.ldM;
  for (i64 w = threadIdx.x; w < a.ldM; w += NT) {
    uint32_t lo[32], hi[32];
    const IdT* col = cct + w;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      lo[k] = (uint32_t)col[(i64)k * a.ldM];
      hi[k] = (uint32_t)col[(i64)(k + 32) * a.ldM];
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      lo[k] = T[tpos(lo[k])];
      hi[k] = T[tpos(hi[k])];
    }
    transpose32(lo);
    transpose32(hi);
    if (nr == XR) {
#pragma unroll
      for (int r = 0; r < XR; ++r)
        __builtin_nontemporal_store(((u64)hi[r] << 32) | lo[r], out + (i64)r * a.ldM + w);
    } else {
#pragma unroll
      for (int r = 0; r < XR; ++r)
        if (r < nr) __builtin_nontemporal_store(((u64)hi[r] << 32) | lo[r], out + (i64)r * a.ldM + w);
    }
  }
}

}  // namespace kano
