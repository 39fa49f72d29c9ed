// Dense-path GEMM micro (round 5): Mc[h][ca] = (sum_p Sel[h][p] Allow[p][ca] > 0)
// on bit-packed operands, D1's shape (8,000 x 10,000 x 8,000), three kernels:
//   base   k_heavy_gemm_lds<4,4> (the engine's, kano_kernels.hpp): every wave
//          expands its own 4 A + 4 B fragments bit -> byte in VALU
//   noexp  the same loop with the expansion replaced by a reinterpretation
//          of the bits (wrong results; what the MFMAs cost without it)
//   x      k_heavy_gemm_x: the block's 256 A rows and 256 B columns of a
//          K-step expanded ONCE (one word per lane) into LDS, the 2 x 2 waves'
//          fragments read from there (ds_read_b128), double-buffered
// Checks x (and base) against a host reference on sampled rows.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I kubernetes-verification_amd/csrc \
//          -o gemm_bits scripts/micro/gemm_bits.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "kano_kernels.hpp"
#include "gemm_i8_ref.hpp"

using namespace kano;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

// the no-expansion timing variant of k_heavy_gemm_lds<4,4>
template <int TM, int TN>
__global__ __launch_bounds__(TPB) void k_gemm_noexp(const u64* __restrict__ A, i64 ldA,
                                                    const int32_t* __restrict__ hlist, i64 H,
                                                    const u64* __restrict__ B, i64 ldB, i64 Ua,
                                                    i64 PBp, uint32_t* __restrict__ Mc32,
                                                    i64 ldMc) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int STAGE = GK_KC * (BM + BN);
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wv = threadIdx.x >> 6;
  const i64 nbm = (H + BM - 1) / BM, nbn = (Ua + BN - 1) / BN;
  const i64 total = nbm * nbn, per = (total + 7) / 8;
  const i64 L = (i64)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= total) return;
  const i64 bm = L % nbm, bn = L / nbm;
  const i64 rb0 = bm * BM, cb0 = bn * BN;
  auto stage = [&](int buf, i64 k0) {
    u64* dst = smem + (size_t)buf * STAGE;
    constexpr int PIECES = GK_KC * (BM + BN) / 128;
    for (int q = wv; q < PIECES; q += TPB / 64) {
      const int w0 = q * 128;
      const int kk = w0 < GK_KC * BM ? w0 / BM : (w0 - GK_KC * BM) / BN;
      const u64* src = w0 < GK_KC * BM ? A + (k0 + kk) * ldA + rb0 + (w0 - kk * BM)
                                       : B + (k0 + kk) * ldB + cb0 + (w0 - GK_KC * BM - kk * BN);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + 2 * lane),
                                       (__attribute__((address_space(3))) void*)(dst + w0), 16,
                                       0, 0);
    }
  };
  const int wr = wv >> 1, wc = wv & 1;
  i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  const i64 nchunks = PBp / GK_KC;
  stage(0, 0);
  for (i64 c = 0; c < nchunks; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 < nchunks) stage((int)((c + 1) & 1), (c + 1) * GK_KC);
    const u64* As = smem + (size_t)(c & 1) * STAGE;
    const u64* Bs = As + GK_KC * BM;
#pragma unroll 2
    for (int kk = 0; kk < GK_KC; ++kk) {
      u64 aw[TM], bw[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) aw[t] = As[kk * BM + wr * 32 * TM + 32 * t + l32];
#pragma unroll
      for (int u = 0; u < TN; ++u) bw[u] = Bs[kk * BN + wc * 32 * TN + 32 * u + l32];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        i32x4 af[TM], bf[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          af[t][0] = (int32_t)aw[t]; af[t][1] = (int32_t)(aw[t] >> 32);
          af[t][2] = ks; af[t][3] = half;
        }
#pragma unroll
        for (int u = 0; u < TN; ++u) {
          bf[u][0] = (int32_t)bw[u]; bf[u][1] = (int32_t)(bw[u] >> 32);
          bf[u][2] = ks; bf[u][3] = half;
        }
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], bf[u], acc[t][u], 0, 0, 0);
      }
    }
  }
  const i64 rb = rb0 + wr * 32 * TM, cb = cb0 + wc * 32 * TN;
  const i64 ld32 = 2 * ldMc;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const i64 row = rb + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int32_t hr = row < H ? hlist[row] : -1;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const u64 bal = __ballot(acc[t][u][g] > 0);
        const i64 c32 = (cb + 32 * u) >> 5;
        if (l32 == 0 && hr >= 0 && c32 < ld32)
          Mc32[(i64)hr * ld32 + c32] = half ? (uint32_t)(bal >> 32) : (uint32_t)bal;
      }
    }
}

// k_heavy_gemm_lds with the LDS reads software-pipelined: the next K-step's
// operand words are read into registers before this step's MFMAs issue, and
// the 16-bit fields come from 32-bit halves (no 64-bit shifts).  EXP = false:
// timing only (no expansion).
template <bool EXP>
__global__ __launch_bounds__(TPB) void k_gemm_pipe(const u64* __restrict__ A, i64 ldA,
                                                   const int32_t* __restrict__ hlist, i64 H,
                                                   const u64* __restrict__ B, i64 ldB, i64 Ua,
                                                   i64 PBp, uint32_t* __restrict__ Mc32,
                                                   i64 ldMc) {
  constexpr int TM = 4, TN = 4;
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int STAGE = GK_KC * (BM + BN);
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wv = threadIdx.x >> 6;
  constexpr i64 GM = 8;
  const i64 nbm = (H + BM - 1) / BM, nbn = (Ua + BN - 1) / BN;
  const i64 total = nbm * nbn, per = (total + 7) / 8;
  const i64 L = (i64)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= total) return;
  const i64 grp = L / (GM * nbn), first = grp * GM;
  const i64 gm = nbm - first < GM ? nbm - first : GM;
  const i64 in = L - grp * GM * nbn;
  const i64 bm = first + in % gm, bn = in / gm;
  const i64 rb0 = bm * BM, cb0 = bn * BN;
  auto stage = [&](int buf, i64 k0) {
    u64* dst = smem + (size_t)buf * STAGE;
    constexpr int PIECES = GK_KC * (BM + BN) / 128;
    for (int q = wv; q < PIECES; q += TPB / 64) {
      const int w0 = q * 128;
      const int kk = w0 < GK_KC * BM ? w0 / BM : (w0 - GK_KC * BM) / BN;
      const u64* src = w0 < GK_KC * BM ? A + (k0 + kk) * ldA + rb0 + (w0 - kk * BM)
                                       : B + (k0 + kk) * ldB + cb0 + (w0 - GK_KC * BM - kk * BN);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + 2 * lane),
                                       (__attribute__((address_space(3))) void*)(dst + w0), 16,
                                       0, 0);
    }
  };
  const int wr = wv >> 1, wc = wv & 1;
  i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  const i64 nchunks = PBp / GK_KC;
  const int hs = half * 16;
  stage(0, 0);
  for (i64 c = 0; c < nchunks; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 < nchunks) stage((int)((c + 1) & 1), (c + 1) * GK_KC);
    const u64* As = smem + (size_t)(c & 1) * STAGE + wr * 32 * TM + l32;
    const u64* Bs = smem + (size_t)(c & 1) * STAGE + GK_KC * BM + wc * 32 * TN + l32;
    u64 aw[TM], bw[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) aw[t] = As[32 * t];
#pragma unroll
    for (int u = 0; u < TN; ++u) bw[u] = Bs[32 * u];
#pragma unroll 2
    for (int kk = 0; kk < GK_KC; ++kk) {
      u64 an[TM], bn[TN];
      const int kn = kk + 1 < GK_KC ? kk + 1 : kk;
#pragma unroll
      for (int t = 0; t < TM; ++t) an[t] = As[kn * BM + 32 * t];
#pragma unroll
      for (int u = 0; u < TN; ++u) bn[u] = Bs[kn * BN + 32 * u];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        i32x4 af[TM], bf[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          const uint32_t w32 = ks ? (uint32_t)(aw[t] >> 32) : (uint32_t)aw[t];
          if (EXP) {
            af[t] = expand16(__builtin_amdgcn_ubfe(w32, hs, 16));
          } else {
            af[t][0] = (int32_t)w32; af[t][1] = hs; af[t][2] = ks; af[t][3] = 1;
          }
        }
#pragma unroll
        for (int u = 0; u < TN; ++u) {
          const uint32_t w32 = ks ? (uint32_t)(bw[u] >> 32) : (uint32_t)bw[u];
          if (EXP) {
            bf[u] = expand16(__builtin_amdgcn_ubfe(w32, hs, 16));
          } else {
            bf[u][0] = (int32_t)w32; bf[u][1] = hs; bf[u][2] = ks; bf[u][3] = 1;
          }
        }
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u)
            acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], bf[u], acc[t][u], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < TM; ++t) aw[t] = an[t];
#pragma unroll
      for (int u = 0; u < TN; ++u) bw[u] = bn[u];
    }
  }
  const i64 rb = rb0 + wr * 32 * TM, cb = cb0 + wc * 32 * TN;
  const i64 ld32 = 2 * ldMc;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const i64 row = rb + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int32_t hr = row < H ? hlist[row] : -1;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const u64 bal = __ballot(acc[t][u][g] > 0);
        const i64 c32 = (cb + 32 * u) >> 5;
        if (l32 == 0 && hr >= 0 && c32 < ld32)
          Mc32[(i64)hr * ld32 + c32] = half ? (uint32_t)(bal >> 32) : (uint32_t)bal;
      }
    }
}

// No LDS: each wave streams its own operand words from global memory (the
// panels are L2 / MALL-resident) into a ring of registers PD K-steps deep,
// and the bit -> byte expansion of the next half-step is interleaved with
// the current half-step's 16 MFMAs (sched_group_barrier: 1 MFMA, 6 VALU).
template <int PD>
__global__ __launch_bounds__(TPB) void k_gemm_reg(const u64* __restrict__ A, i64 ldA,
                                                  const int32_t* __restrict__ hlist, i64 H,
                                                  const u64* __restrict__ B, i64 ldB, i64 Ua,
                                                  i64 PBp, uint32_t* __restrict__ Mc32,
                                                  i64 ldMc) {
  constexpr int TM = 4, TN = 4;
  constexpr int BM = 64 * TM, BN = 64 * TN;
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wv = threadIdx.x >> 6;
  constexpr i64 GM = 8;
  const i64 nbm = (H + BM - 1) / BM, nbn = (Ua + BN - 1) / BN;
  const i64 total = nbm * nbn, per = (total + 7) / 8;
  const i64 L = (i64)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= total) return;
  const i64 grp = L / (GM * nbn), first = grp * GM;
  const i64 gm = nbm - first < GM ? nbm - first : GM;
  const i64 in = L - grp * GM * nbn;
  const i64 bm = first + in % gm, bn = in / gm;
  const int wr = wv >> 1, wc = wv & 1;
  const i64 rb = bm * BM + wr * 32 * TM, cb = bn * BN + wc * 32 * TN;
  const u64* pa = A + rb + l32;
  const u64* pb = B + cb + l32;
  const int hs = half * 16;
  u64 wa[PD][TM], wb[PD][TN];
#pragma unroll
  for (int d = 0; d < PD; ++d) {
#pragma unroll
    for (int t = 0; t < TM; ++t) wa[d][t] = pa[(i64)d * ldA + 32 * t];
#pragma unroll
    for (int u = 0; u < TN; ++u) wb[d][u] = pb[(i64)d * ldB + 32 * u];
  }
  i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  i32x4 a0[TM], b0[TN], a1[TM], b1[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t) a0[t] = expand16(__builtin_amdgcn_ubfe((uint32_t)wa[0][t], hs, 16));
#pragma unroll
  for (int u = 0; u < TN; ++u) b0[u] = expand16(__builtin_amdgcn_ubfe((uint32_t)wb[0][u], hs, 16));
  for (i64 k0 = 0; k0 < PBp; k0 += PD) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const i64 k = k0 + j;
      // phase A: ks 0 of step k; the ks 1 halves of step k expanded beside it
#pragma unroll
      for (int t = 0; t < TM; ++t)
        a1[t] = expand16(__builtin_amdgcn_ubfe((uint32_t)(wa[j][t] >> 32), hs, 16));
#pragma unroll
      for (int u = 0; u < TN; ++u)
        b1[u] = expand16(__builtin_amdgcn_ubfe((uint32_t)(wb[j][u] >> 32), hs, 16));
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[t], b0[u], acc[t][u], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 6, 0);
      }
      // the slot of step k refilled with step k + PD
      const i64 kn = k + PD;
      if (kn < PBp) {
#pragma unroll
        for (int t = 0; t < TM; ++t) wa[j][t] = pa[kn * ldA + 32 * t];
#pragma unroll
        for (int u = 0; u < TN; ++u) wb[j][u] = pb[kn * ldB + 32 * u];
      }
      // phase B: ks 1 of step k; ks 0 of step k + 1 expanded beside it
      const int jn = (j + 1) % PD;
#pragma unroll
      for (int t = 0; t < TM; ++t)
        a0[t] = expand16(__builtin_amdgcn_ubfe((uint32_t)wa[jn][t], hs, 16));
#pragma unroll
      for (int u = 0; u < TN; ++u)
        b0[u] = expand16(__builtin_amdgcn_ubfe((uint32_t)wb[jn][u], hs, 16));
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[t], b1[u], acc[t][u], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x2, 6, 0);
      }
    }
  }
  const i64 ld32 = 2 * ldMc;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const i64 row = rb + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int32_t hr = row < H ? hlist[row] : -1;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const u64 bal = __ballot(acc[t][u][g] > 0);
        const i64 c32 = (cb + 32 * u) >> 5;
        if (l32 == 0 && hr >= 0 && c32 < ld32)
          Mc32[(i64)hr * ld32 + c32] = half ? (uint32_t)(bal >> 32) : (uint32_t)bal;
      }
    }
}

// the MFMA ceiling: the same MFMA count per wave (PBp x 32) on register
// operands, no loads, no LDS, the same epilogue
__global__ __launch_bounds__(TPB) void k_gemm_pure(i64 H, i64 Ua, i64 PBp,
                                                   uint32_t* __restrict__ Mc32, i64 ldMc,
                                                   int seed) {
  constexpr int TM = 4, TN = 4;
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wv = threadIdx.x >> 6;
  const i64 nbm = (H + 255) / 256, nbn = (Ua + 255) / 256;
  const i64 L = blockIdx.x;
  if (L >= nbm * nbn) return;
  i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  i32x4 af[TM], bf[TN];
#pragma unroll
  for (int t = 0; t < TM; ++t) af[t] = i32x4{seed + t, lane, half, 1};
#pragma unroll
  for (int u = 0; u < TN; ++u) bf[u] = i32x4{seed - u, lane, 1, half};
  for (i64 k = 0; k < PBp * 2; ++k) {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], bf[u], acc[t][u], 0, 0, 0);
  }
  const i64 ld32 = 2 * ldMc;
  i64 s = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) s += acc[t][u][g];
  if (s == 12345) Mc32[(L * 4 + wv) % (H * ld32)] = (uint32_t)s;
}

// ---------------------------------------------------------------------------
// k_heavy_gemm_x: the block tile is 256 rows x 256 columns (2 x 2 waves of
// 128 x 128, 4 x 4 tiles of v_mfma_i32_32x32x32_i8).  Per K-step (64
// policies, one word per row / column) every lane expands ONE A word and ONE
// B word (its row rb0 + threadIdx.x, its column cb0 + threadIdx.x) into 64
// bytes in LDS; the waves then read their fragments with ds_read_b128.  Rows
// of the expanded images are 80 B apart (64 + 16 of padding): the lane groups
// of ds_read_b128 and ds_write_b128 then meet 16 distinct 16-B bank groups.
// The operand words come from global memory into registers XD K-steps ahead.
// ---------------------------------------------------------------------------
constexpr int GX_RS = 80;                  // bytes per expanded row
constexpr int GX_IMG = 256 * GX_RS;        // one operand's image per K-step
constexpr int GX_XD = 4;                   // K-steps of operand words in flight

__device__ __forceinline__ void gx_expand_store(u64 w, char* row) {
  // 64 bits -> 64 bytes 0/1, four 16-byte stores
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t b16 = (uint32_t)(w >> (16 * q)) & 0xffffu;
    *reinterpret_cast<i32x4*>(row + 16 * q) = expand16(b16);
  }
}

__global__ __launch_bounds__(TPB) void k_heavy_gemm_x(const u64* __restrict__ A, i64 ldA,
                                                      const int32_t* __restrict__ hlist, i64 H,
                                                      const u64* __restrict__ B, i64 ldB, i64 Ua,
                                                      i64 PB, uint32_t* __restrict__ Mc32,
                                                      i64 ldMc) {
  constexpr int TM = 4, TN = 4, BM = 256, BN = 256;
  extern __shared__ __attribute__((aligned(16))) char xs[];   // 2 x (A image, B image)
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
  // this lane's operand words: row rb0 + tid of A, column cb0 + tid of B
  // (ldA >= rb0 + 256, ldB >= cb0 + 256: the operands are padded)
  const u64* pa = A + rb0 + threadIdx.x;
  const u64* pb = B + cb0 + threadIdx.x;
  u64 ra[GX_XD], rbw[GX_XD];
#pragma unroll
  for (int d = 0; d < GX_XD; ++d) {
    ra[d] = d < PB ? pa[(i64)d * ldA] : 0ull;
    rbw[d] = d < PB ? pb[(i64)d * ldB] : 0ull;
  }
  const int wr = wv >> 1, wc = wv & 1;
  i32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0;
  // K-step 0's images
  gx_expand_store(ra[0], xs + threadIdx.x * GX_RS);
  gx_expand_store(rbw[0], xs + GX_IMG + threadIdx.x * GX_RS);
  ra[0] = GX_XD < PB ? pa[(i64)GX_XD * ldA] : 0ull;   // slot 0 now carries K-step XD
  rbw[0] = GX_XD < PB ? pb[(i64)GX_XD * ldB] : 0ull;
  __syncthreads();
  const int arow = (wr * 32 * TM + l32) * GX_RS + half * 16;
  const int bcol = (wc * 32 * TN + l32) * GX_RS + half * 16;
  for (i64 k = 0; k < PB; ++k) {
    const int cur = (int)(k & 1);
    const char* xa = xs + cur * 2 * GX_IMG;
    const char* xb = xa + GX_IMG;
    // the next K-step's images into the other buffer (read by nobody now:
    // the barrier at the end of the previous step)
    if (k + 1 < PB) {
      char* na = xs + (cur ^ 1) * 2 * GX_IMG;
      const int d = (int)((k + 1) % GX_XD);
      u64 wa = 0, wb = 0;
#pragma unroll
      for (int q = 0; q < GX_XD; ++q)
        if (q == d) { wa = ra[q]; wb = rbw[q]; }
      gx_expand_store(wa, na + threadIdx.x * GX_RS);
      gx_expand_store(wb, na + GX_IMG + threadIdx.x * GX_RS);
      // refill the slot of K-step k + 1 with K-step k + 1 + XD
      const i64 kn = k + 1 + GX_XD;
#pragma unroll
      for (int q = 0; q < GX_XD; ++q)
        if (q == d) {
          ra[q] = kn < PB ? pa[kn * ldA] : 0ull;
          rbw[q] = kn < PB ? pb[kn * ldB] : 0ull;
        }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      i32x4 af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t)
        af[t] = *reinterpret_cast<const i32x4*>(xa + arow + t * 32 * GX_RS + ks * 32);
#pragma unroll
      for (int u = 0; u < TN; ++u)
        bf[u] = *reinterpret_cast<const i32x4*>(xb + bcol + u * 32 * GX_RS + ks * 32);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t], bf[u], acc[t][u], 0, 0, 0);
    }
    __syncthreads();
  }
  const i64 rb = rb0 + wr * 32 * TM, cb = cb0 + wc * 32 * TN;
  const i64 ld32 = 2 * ldMc;
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const i64 row = rb + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int32_t hr = row < H ? hlist[row] : -1;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const u64 bal = __ballot(acc[t][u][g] > 0);
        const i64 c32 = (cb + 32 * u) >> 5;
        if (l32 == 0 && hr >= 0 && c32 < ld32)
          Mc32[(i64)hr * ld32 + c32] = half ? (uint32_t)(bal >> 32) : (uint32_t)bal;
      }
    }
}

int main(int argc, char** argv) {
  const i64 H = argc > 1 ? atol(argv[1]) : 8000, Ua = argc > 2 ? atol(argv[2]) : 8000;
  const i64 P = argc > 3 ? atol(argv[3]) : 10000;
  const double dens = argc > 4 ? atof(argv[4]) : 0.05;
  const int reps = argc > 5 ? atoi(argv[5]) : 20;
  const i64 PB = (P + 63) / 64, PBp = (PB + GK_KC - 1) / GK_KC * GK_KC;
  const i64 ldA = (H + 255) / 256 * 256, ldB = (Ua + 255) / 256 * 256;
  const i64 ldMc = std::max<i64>(2, ((Ua + 63) / 64 + 1) & ~1ll);
  std::mt19937_64 rng(7);
  std::vector<u64> hA(PBp * ldA, 0), hB(PBp * ldB, 0);
  auto bits = [&](std::vector<u64>& v, i64 ld, i64 rows) {
    // density dens per bit, K-word-major [kw][row]
    std::bernoulli_distribution bd(dens);
    for (i64 kw = 0; kw < PB; ++kw)
      for (i64 r = 0; r < rows; ++r) {
        u64 w = 0;
        for (int b = 0; b < 64; ++b)
          if (kw * 64 + b < P && bd(rng)) w |= 1ull << b;
        v[kw * ld + r] = w;
      }
  };
  bits(hA, ldA, H);
  bits(hB, ldB, Ua);
  std::vector<int32_t> hl(H);
  for (i64 h = 0; h < H; ++h) hl[h] = (int32_t)h;
  u64 *dA, *dB, *dM0, *dM1;
  int32_t* dl;
  const size_t mcb = sizeof(u64) * (size_t)(H * ldMc);
  CK(hipMalloc(&dA, sizeof(u64) * hA.size()));
  CK(hipMalloc(&dB, sizeof(u64) * hB.size()));
  CK(hipMalloc(&dM0, mcb));
  CK(hipMalloc(&dM1, mcb));
  CK(hipMalloc(&dl, sizeof(int32_t) * H));
  CK(hipMemcpy(dA, hA.data(), sizeof(u64) * hA.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), sizeof(u64) * hB.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, hl.data(), sizeof(int32_t) * H, hipMemcpyHostToDevice));
  const int lds44 = (int)(sizeof(u64) * 2 * GK_KC * (256 + 256));
  const int ldsx = 2 * 2 * GX_IMG;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_lds<4, 4>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds44));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_noexp<4, 4>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds44));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_pipe<true>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds44));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_pipe<false>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds44));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_x),
                         hipFuncAttributeMaxDynamicSharedMemorySize, ldsx));
  const i64 nb = ((H + 255) / 256) * ((Ua + 255) / 256);
  const dim3 grid((unsigned)(8 * ((nb + 7) / 8)));
  uint32_t* o0 = reinterpret_cast<uint32_t*>(dM0);
  uint32_t* o1 = reinterpret_cast<uint32_t*>(dM1);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double ops = 2.0 * H * (double)P * Ua;
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    std::printf("%-8s H=%lld Ua=%lld P=%lld dens=%.3f  median %.4f ms  best %.4f ms  %.0f TOPS  "
                "frac %.3f\n", name, (long long)H, (long long)Ua, (long long)P, dens, med, t[0],
                ops / med * 1e-9, ops / med * 1e-9 / 5000.0);
  };
  CK(hipMemset(dM0, 0, mcb));
  CK(hipMemset(dM1, 0, mcb));
  timeit("base", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_lds<4, 4>), grid, dim3(TPB), lds44, 0, dA, ldA, dl, H, dB,
                       ldB, Ua, PBp, o0, ldMc);
  });
  timeit("noexp", [&] {
    hipLaunchKernelGGL((k_gemm_noexp<4, 4>), grid, dim3(TPB), lds44, 0, dA, ldA, dl, H, dB, ldB,
                       Ua, PBp, o1, ldMc);
  });
  timeit("pipe_nx", [&] {
    hipLaunchKernelGGL((k_gemm_pipe<false>), grid, dim3(TPB), lds44, 0, dA, ldA, dl, H, dB, ldB,
                       Ua, PBp, o1, ldMc);
  });
  CK(hipMemset(dM1, 0, mcb));
  timeit("pipe", [&] {
    hipLaunchKernelGGL((k_gemm_pipe<true>), grid, dim3(TPB), lds44, 0, dA, ldA, dl, H, dB, ldB,
                       Ua, PBp, o1, ldMc);
  });
  CK(hipDeviceSynchronize());
  {
    std::vector<u64> a(H * ldMc), b(H * ldMc);
    CK(hipMemcpy(a.data(), dM0, mcb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dM1, mcb, hipMemcpyDeviceToHost));
    i64 d = 0;
    for (size_t i = 0; i < a.size(); ++i) d += a[i] != b[i];
    std::printf("pipe vs base: %lld differing words\n", (long long)d);
    if (d) return 2;
  }
  for (int pdv : {4, 8}) {
    CK(hipMemset(dM1, 0, mcb));
    timeit(pdv == 4 ? "reg4" : "reg8", [&] {
      if (pdv == 4)
        hipLaunchKernelGGL((k_gemm_reg<4>), grid, dim3(TPB), 0, 0, dA, ldA, dl, H, dB, ldB, Ua,
                           PBp, o1, ldMc);
      else
        hipLaunchKernelGGL((k_gemm_reg<8>), grid, dim3(TPB), 0, 0, dA, ldA, dl, H, dB, ldB, Ua,
                           PBp, o1, ldMc);
    });
    CK(hipDeviceSynchronize());
    std::vector<u64> a(H * ldMc), b(H * ldMc);
    CK(hipMemcpy(a.data(), dM0, mcb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dM1, mcb, hipMemcpyDeviceToHost));
    i64 d = 0;
    for (size_t i = 0; i < a.size(); ++i) d += a[i] != b[i];
    std::printf("reg%d vs base: %lld differing words\n", pdv, (long long)d);
    if (d) return 3;
  }
  timeit("pure", [&] {
    hipLaunchKernelGGL(k_gemm_pure, grid, dim3(TPB), 0, 0, H, Ua, PBp, o1, ldMc, 3);
  });
  CK(hipMemset(dM1, 0, mcb));
  timeit("x", [&] {
    hipLaunchKernelGGL(k_heavy_gemm_x, grid, dim3(TPB), ldsx, 0, dA, ldA, dl, H, dB, ldB, Ua, PB,
                       o1, ldMc);
  });
  CK(hipDeviceSynchronize());
  std::vector<u64> m0(H * ldMc), m1(H * ldMc);
  CK(hipMemcpy(m0.data(), dM0, mcb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(m1.data(), dM1, mcb, hipMemcpyDeviceToHost));
  i64 diff = 0;
  for (size_t i = 0; i < m0.size(); ++i) diff += m0[i] != m1[i];
  // host reference on sampled rows
  i64 bad = 0;
  std::uniform_int_distribution<i64> rd(0, H - 1);
  for (int s = 0; s < 24; ++s) {
    const i64 h = s == 0 ? 0 : s == 1 ? H - 1 : rd(rng);
    for (i64 ca = 0; ca < Ua; ++ca) {
      bool hit = false;
      for (i64 kw = 0; kw < PB && !hit; ++kw) hit = (hA[kw * ldA + h] & hB[kw * ldB + ca]) != 0;
      const bool g0 = (m0[h * ldMc + (ca >> 6)] >> (ca & 63)) & 1;
      bad += g0 != hit;
    }
  }
  std::printf("x vs base: %lld differing words; base vs host reference: %lld wrong bits "
              "(24 sampled rows)\n", (long long)diff, (long long)bad);
  return diff || bad ? 1 : 0;
}
