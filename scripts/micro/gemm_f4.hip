// Dense-path GEMM micro (round 6): Mc[h][ca] = (sum_p Sel[h][p] Allow[p][ca] > 0)
// on bit-packed operands, D1's shape (8,000 x 10,000 x 8,000) by default:
//   i8   k_heavy_gemm_lds<4,4>  (v_mfma_i32_32x32x32_i8, bits spread to bytes)
//   f4   k_heavy_gemm_f4<4,4>   (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 nibbles)
//   f4_42 / f4_22               (smaller wave tiles; f4_22k8: 8 K-steps a chunk,
//                               the engine's form)
// Every form's Mc must equal the i8 form's word for word, and the i8 form a
// host reference on sampled rows.  Prints one line per kernel: median / best
// of `reps` launches, TOP/s, and the fraction of the int8 (5 POP/s) and fp4
// (10 POP/s) dense peaks.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I kubernetes-verification_amd/csrc \
//          -o gemm_f4 scripts/micro/gemm_f4.hip
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

// Timing variants of k_heavy_gemm_f4 (results wrong unless MODE == 0):
//   MODE 0  k_heavy_gemm_f4 with GK_KC = KC (K-steps per staged chunk)
//   MODE 1  no expansion: the raw 32 bits fill the operand registers
//   MODE 2  no LDS fragment reads: the operands are built from the K index
//   MODE 3  MODE 2 without the staging (no global loads, no barriers)
template <int TM, int TN, int KC, int MODE>
__global__ __launch_bounds__(TPB) void k_f4_var(const u64* __restrict__ A, i64 ldA,
                                                const int32_t* __restrict__ hlist, i64 H,
                                                const u64* __restrict__ B, i64 ldB, i64 Ua,
                                                i64 PBp, uint32_t* __restrict__ Mc32, i64 ldMc) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int STAGE = KC * (BM + BN);
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
    constexpr int PIECES = KC * (BM + BN) / 128;
    for (int q = wv; q < PIECES; q += TPB / 64) {
      const int w0 = q * 128;
      const int kk = w0 < KC * BM ? w0 / BM : (w0 - KC * BM) / BN;
      const u64* src = w0 < KC * BM ? A + (k0 + kk) * ldA + rb0 + (w0 - kk * BM)
                                    : B + (k0 + kk) * ldB + cb0 + (w0 - KC * BM - kk * BN);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + 2 * lane),
                                       (__attribute__((address_space(3))) void*)(dst + w0), 16,
                                       0, 0);
    }
  };
  const int wr = wv >> 1, wc = wv & 1;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
  const i64 nchunks = PBp / KC;
  if (MODE != 3) stage(0, 0);
  for (i64 c = 0; c < nchunks; ++c) {
    if (MODE != 3) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (c + 1 < nchunks) stage((int)((c + 1) & 1), (c + 1) * KC);
    }
    const uint32_t* As = reinterpret_cast<const uint32_t*>(smem + (size_t)(c & 1) * STAGE) +
                         2 * (wr * 32 * TM + l32) + half;
    const uint32_t* Bs = reinterpret_cast<const uint32_t*>(smem + (size_t)(c & 1) * STAGE +
                                                           KC * BM) +
                         2 * (wc * 32 * TN + l32) + half;
#pragma unroll 4
    for (int kk = 0; kk < KC; ++kk) {
      i32x8 af[TM], bf[TN];
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t x = MODE >= 2 ? (uint32_t)(kk * 7 + t + (int)c) : As[2 * (kk * BM + 32 * t)];
        if (MODE == 1) {
          af[t] = i32x8{(int32_t)x, (int32_t)x, (int32_t)x, (int32_t)x, 0, 0, 0, 0};
        } else {
          af[t] = bits_to_fp4(x);
        }
      }
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const uint32_t x = MODE >= 2 ? (uint32_t)(kk * 5 + u + (int)c) : Bs[2 * (kk * BN + 32 * u)];
        if (MODE == 1) {
          bf[u] = i32x8{(int32_t)x, (int32_t)x, (int32_t)x, (int32_t)x, 0, 0, 0, 0};
        } else {
          bf[u] = bits_to_fp4(x);
        }
      }
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              af[t], bf[u], acc[t][u], 4, 4, 0, FP4_ONE_SCALE, 0, FP4_ONE_SCALE);
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
        const u64 bal = __ballot(acc[t][u][g] > 0.f);
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
  // a few all-ones rows / columns (every sum at its largest: exactness)
  for (i64 kw = 0; kw < PB; ++kw) {
    const u64 full = (kw + 1) * 64 <= P ? ~0ull : (1ull << (P - kw * 64)) - 1;
    hA[kw * ldA + 0] = full;
    hB[kw * ldB + 0] = full;
  }
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
  auto lds_of = [](int tm, int tn) { return (int)(sizeof(u64) * 2 * GK_KC * (64 * tm + 64 * tn)); };
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_lds<4, 4>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 4)));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<4, 4, 16>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 4)));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<4, 2, 16>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 2)));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<2, 2, 16>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(2, 2)));
  auto grid_of = [&](int tm, int tn) {
    const i64 nb = ((H + 64 * tm - 1) / (64 * tm)) * ((Ua + 64 * tn - 1) / (64 * tn));
    return dim3((unsigned)(8 * ((nb + 7) / 8)));
  };
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
    std::printf("%-6s H=%lld Ua=%lld P=%lld dens=%.3f  median %.4f ms  best %.4f ms  %.0f TOPS  "
                "frac_i8 %.3f  frac_f4 %.3f\n", name, (long long)H, (long long)Ua, (long long)P,
                dens, med, t[0], ops / med * 1e-9, ops / med * 1e-9 / 5000.0,
                ops / med * 1e-9 / 10000.0);
    std::fflush(stdout);
  };
  auto compare = [&](const char* name) {
    CK(hipDeviceSynchronize());
    std::vector<u64> a(H * ldMc), b(H * ldMc);
    CK(hipMemcpy(a.data(), dM0, mcb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dM1, mcb, hipMemcpyDeviceToHost));
    i64 d = 0;
    for (size_t i = 0; i < a.size(); ++i) d += a[i] != b[i];
    std::printf("%s vs i8: %lld differing words\n", name, (long long)d);
    return d;
  };
  CK(hipMemset(dM0, 0, mcb));
  timeit("i8", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_lds<4, 4>), grid_of(4, 4), dim3(TPB), lds_of(4, 4), 0, dA,
                       ldA, dl, H, dB, ldB, Ua, PBp, o0, ldMc);
  });
  i64 bad_forms = 0;
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_f4<4, 4, 16>), grid_of(4, 4), dim3(TPB), lds_of(4, 4), 0, dA,
                       ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4") != 0;
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4_42", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_f4<4, 2, 16>), grid_of(4, 2), dim3(TPB), lds_of(4, 2), 0, dA,
                       ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4_42") != 0;
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4_22", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_f4<2, 2, 16>), grid_of(2, 2), dim3(TPB), lds_of(2, 2), 0, dA,
                       ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4_22") != 0;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<2, 2, 8>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(2, 2) / 2));
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4_22k8", [&] {   // the engine's form
    hipLaunchKernelGGL((k_heavy_gemm_f4<2, 2, 8>), grid_of(2, 2), dim3(TPB), lds_of(2, 2) / 2, 0,
                       dA, ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4_22k8") != 0;
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4_22k4", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_f4<2, 2, 4>), grid_of(2, 2), dim3(TPB), lds_of(2, 2) / 4, 0,
                       dA, ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4_22k4") != 0;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_heavy_gemm_f4<4, 2, 8>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 2) / 2));
  CK(hipMemset(dM1, 0, mcb));
  timeit("f4_42k8", [&] {
    hipLaunchKernelGGL((k_heavy_gemm_f4<4, 2, 8>), grid_of(4, 2), dim3(TPB), lds_of(4, 2) / 2, 0,
                       dA, ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
  });
  bad_forms += compare("f4_42k8") != 0;
  {
    const int l8 = (int)(sizeof(u64) * 2 * 8 * 512), l32 = (int)(sizeof(u64) * 2 * 32 * 256);
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<4, 4, 8, 0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, l8));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<4, 4, 16, 1>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 4)));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<4, 4, 16, 2>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 4)));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<2, 2, 32, 0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, l32));
    CK(hipMemset(dM1, 0, mcb));
    timeit("kc8", [&] {
      hipLaunchKernelGGL((k_f4_var<4, 4, 8, 0>), grid_of(4, 4), dim3(TPB), l8, 0, dA, ldA, dl, H,
                         dB, ldB, Ua, PBp, o1, ldMc);
    });
    bad_forms += compare("kc8") != 0;
    CK(hipMemset(dM1, 0, mcb));
    timeit("22kc32", [&] {
      hipLaunchKernelGGL((k_f4_var<2, 2, 32, 0>), grid_of(2, 2), dim3(TPB), l32, 0, dA, ldA, dl,
                         H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    if (PBp % 32 == 0) bad_forms += compare("22kc32") != 0;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<2, 2, 8, 0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(u64) * 2 * 8 * 256)));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<2, 2, 16, 0>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(2, 2)));
    CK(hipMemset(dM1, 0, mcb));
    timeit("22kc8", [&] {
      hipLaunchKernelGGL((k_f4_var<2, 2, 8, 0>), grid_of(2, 2), dim3(TPB), (int)(sizeof(u64) * 2 * 8 * 256), 0, dA, ldA, dl,
                         H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    bad_forms += compare("22kc8") != 0;
    CK(hipMemset(dM1, 0, mcb));
    timeit("22kc16v", [&] {
      hipLaunchKernelGGL((k_f4_var<2, 2, 16, 0>), grid_of(2, 2), dim3(TPB), lds_of(2, 2), 0, dA, ldA, dl,
                         H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    bad_forms += compare("22kc16v") != 0;
    timeit("noexp", [&] {
      hipLaunchKernelGGL((k_f4_var<4, 4, 16, 1>), grid_of(4, 4), dim3(TPB), lds_of(4, 4), 0, dA,
                         ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_f4_var<4, 4, 16, 3>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_of(4, 4)));
    timeit("pure", [&] {
      hipLaunchKernelGGL((k_f4_var<4, 4, 16, 3>), grid_of(4, 4), dim3(TPB), lds_of(4, 4), 0, dA,
                         ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    timeit("pure0", [&] {
      hipLaunchKernelGGL((k_f4_var<4, 4, 16, 3>), grid_of(4, 4), dim3(TPB), 0, 0, dA,
                         ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
    });
    timeit("nolds", [&] {
      hipLaunchKernelGGL((k_f4_var<4, 4, 16, 2>), grid_of(4, 4), dim3(TPB), lds_of(4, 4), 0, dA,
                         ldA, dl, H, dB, ldB, Ua, PBp, o1, ldMc);
    });
  }
  std::vector<u64> m0(H * ldMc);
  CK(hipMemcpy(m0.data(), dM0, mcb, hipMemcpyDeviceToHost));
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
  std::printf("i8 vs host reference: %lld wrong bits (24 sampled rows); forms differing: %lld\n",
              (long long)bad, (long long)bad_forms);
  return bad || bad_forms ? 1 : 0;
}
