// The round-4/5 engine's dense contraction on v_mfma_i32_32x32x32_i8 (bits
// spread to 0/1 bytes in VALU, two MFMAs per 64-policy word), kept for the
// micros' A/B against k_heavy_gemm_f4 (kano_kernels.hpp), which replaced it
// in the engine in round 6.  Staging, tiling and epilogue as k_heavy_gemm_f4.
#pragma once
#include "kano_kernels.hpp"

namespace kano {

// bits -> int8 0/1 bytes (the round-5 expansion)
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// bit i of b4 -> bit 8 i: b4 * (1 + 2^7 + 2^14 + 2^21) puts bit i at i, i+7,
// i+14, i+21 (no carries); the mask keeps bit 8 i (one v_mul_u32_u24 + and)
__device__ __forceinline__ uint32_t spread4(uint32_t b4) {
  return __umul24(b4, 0x204081u) & 0x01010101u;
}
__device__ __forceinline__ i32x4 expand16(uint32_t b16) {
  i32x4 r;
  r[0] = (int32_t)spread4(b16 & 15u);
  r[1] = (int32_t)spread4((b16 >> 4) & 15u);
  r[2] = (int32_t)spread4((b16 >> 8) & 15u);
  r[3] = (int32_t)spread4((b16 >> 12) & 15u);
  return r;
}

template <int TM, int TN>
__global__ __launch_bounds__(TPB) void k_heavy_gemm_lds(const u64* __restrict__ A, i64 ldA,
                                                        const int32_t* __restrict__ hlist, i64 H,
                                                        const u64* __restrict__ B, i64 ldB,
                                                        i64 Ua, i64 PBp,
                                                        uint32_t* __restrict__ Mc32, i64 ldMc) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int STAGE = GK_KC * (BM + BN);     // words per buffer
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
  // the copy of one chunk: per K-step a row of BM words of A and BN of B,
  // 128 words (1 KB) per wave instruction, the block's 4 waves round-robin
  auto stage = [&](int buf, i64 k0) {
    u64* dst = smem + (size_t)buf * STAGE;
    constexpr int PIECES = GK_KC * (BM + BN) / 128;
    for (int q = wv; q < PIECES; q += TPB / 64) {
      const int w0 = q * 128;                         // word offset in the stage
      const int kk = w0 < GK_KC * BM ? w0 / BM : (w0 - GK_KC * BM) / BN;
      const u64* src = w0 < GK_KC * BM
                           ? A + (k0 + kk) * ldA + rb0 + (w0 - kk * BM)
                           : B + (k0 + kk) * ldB + cb0 + (w0 - GK_KC * BM - kk * BN);
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(src + 2 * lane),
          (__attribute__((address_space(3))) void*)(dst + w0), 16, 0, 0);
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
    __syncthreads();                                  // chunk c in LDS, chunk c-1 read by all
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
        const int sh = ks * 32 + half * 16;
        i32x4 af[TM], bf[TN];
#pragma unroll
        for (int t = 0; t < TM; ++t) af[t] = expand16((uint32_t)(aw[t] >> sh) & 0xffffu);
#pragma unroll
        for (int u = 0; u < TN; ++u) bf[u] = expand16((uint32_t)(bw[u] >> sh) & 0xffffu);
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


}  // namespace kano
