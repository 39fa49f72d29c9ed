// MFMA issue-rate calibration (round 6): back-to-back MFMAs on 16 (32x32) or
// 64 (16x16) independent accumulators, one wave per SIMD, 4 waves a block,
// 1,024 blocks; the operands change every iteration (no constant folding).
// Prints per form: the time, the ns per MFMA per SIMD, the cycles at 2.4 GHz
// and the TOP/s over the whole chip.  The product (one bit each) is folded
// into a store so the loop is live.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mfma_rate scripts/micro/mfma_rate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 2048;

// FORM 0: fp4 32x32x64 scaled; 1: fp4 16x16x128 scaled; 2: i8 32x32x32;
// 3: bf16 32x32x16; 4: fp8 32x32x64 scaled; 5: fp4 32x32x64 on a 4 x 4 tile
// whose 8 operands are expanded from bits every iteration (the GEMM's loop
// without its LDS reads); 6: the same 4 x 4 tile, operands fixed
__device__ __forceinline__ i32x8 b2f4(uint32_t x) {
  return i32x8{(int)((x << 1) & 0x22222222u), (int)(x & 0x22222222u),
               (int)((x >> 1) & 0x22222222u), (int)((x >> 2) & 0x22222222u), 0, 0, 0, 0};
}
// 8: a 4 x 2 tile per wave, 8 waves a block (two a SIMD), operands expanded
// every iteration; 9: FORM 5 with the 5-instruction expansion (nibble values
// 0.5 / 1 / 2 / 2 by register: x & 0x11.., x & 0x22.., x & 0x44..,
// (x >> 1) & 0x44..)
__device__ __forceinline__ i32x8 b2f4c(uint32_t x) {
  return i32x8{(int)(x & 0x11111111u), (int)(x & 0x22222222u), (int)(x & 0x44444444u),
               (int)((x >> 1) & 0x44444444u), 0, 0, 0, 0};
}
template <int FORM>
__global__ __launch_bounds__(FORM == 8 ? 512 : 256) void k_rate(int seed, float* out) {
  const int lane = threadIdx.x & 63;
  if constexpr (FORM == 8 || FORM == 9) {
    constexpr int TN = FORM == 8 ? 2 : 4;
    f32x16 acc[4][TN];
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < TN; ++u)
        for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
    for (int it = 0; it < ITERS;
         ++it) {
      const uint32_t x = (uint32_t)(seed + it * 0x9E3779B9u + lane);
      i32x8 af[4], bf[TN];
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = FORM == 9 ? b2f4c(x + t) : b2f4(x + t);
#pragma unroll
      for (int u = 0; u < TN; ++u)
        bf[u] = FORM == 9 ? b2f4c(x ^ (u * 0x01234567u)) : b2f4(x ^ (u * 0x01234567u));
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[t], bf[u], acc[t][u], 4,
                                                                      4, 0, 127, 0, 127);
    }
    float s = 0.f;
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < TN; ++u)
        for (int g = 0; g < 16; ++g) s += acc[t][u][g];
    if (s == 12345.f) out[blockIdx.x] = s;
  } else if constexpr (FORM == 7) {
    // FORM 5 with the operands double-buffered: the fragments of iteration
    // it + 1 are expanded into the other register set while it's MFMAs run
    f32x16 acc[4][4];
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < 4; ++u)
        for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
    i32x8 a0[4], b0[4], a1[4], b1[4];
    auto fill = [&](i32x8* a, i32x8* b, int it) {
      const uint32_t x = (uint32_t)(seed + it * 0x9E3779B9u + lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = b2f4(x + t);
        b[t] = b2f4(x ^ (t * 0x01234567u));
      }
    };
    auto mm = [&](const i32x8* a, const i32x8* b) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[t], b[u], acc[t][u], 4, 4,
                                                                      0, 127, 0, 127);
    };
    fill(a0, b0, 0);
    for (int it = 0; it < ITERS; it += 2) {
      fill(a1, b1, it + 1);
      mm(a0, b0);
      fill(a0, b0, it + 2);
      mm(a1, b1);
    }
    float s = 0.f;
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < 4; ++u)
        for (int g = 0; g < 16; ++g) s += acc[t][u][g];
    if (s == 12345.f) out[blockIdx.x] = s;
  } else if constexpr (FORM == 5 || FORM == 6) {
    f32x16 acc[4][4];
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < 4; ++u)
        for (int g = 0; g < 16; ++g) acc[t][u][g] = 0.f;
    i32x8 af[4], bf[4];
    for (int t = 0; t < 4; ++t) {
      af[t] = b2f4((uint32_t)(seed * 7 + t + lane));
      bf[t] = b2f4((uint32_t)(seed * 5 + t + lane * 3));
    }
    for (int it = 0; it < ITERS; ++it) {
      if constexpr (FORM == 5) {
        const uint32_t x = (uint32_t)(seed + it * 0x9E3779B9u + lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          af[t] = b2f4(x + t);
          bf[t] = b2f4(x ^ (t * 0x01234567u));
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[t], bf[u], acc[t][u], 4,
                                                                      4, 0, 127, 0, 127);
    }
    float s = 0.f;
    for (int t = 0; t < 4; ++t)
      for (int u = 0; u < 4; ++u)
        for (int g = 0; g < 16; ++g) s += acc[t][u][g];
    if (s == 12345.f) out[blockIdx.x] = s;
  } else if constexpr (FORM == 0 || FORM == 2 || FORM == 3 || FORM == 4) {
    f32x16 accf[16];
    i32x16 acci[16];
    for (int t = 0; t < 16; ++t)
      for (int g = 0; g < 16; ++g) { accf[t][g] = 0.f; acci[t][g] = 0; }
    for (int it = 0; it < ITERS; ++it) {
      const uint32_t x = (uint32_t)(seed + it * 0x9E3779B9u + lane) & 0x22222222u;
      if constexpr (FORM == 0 || FORM == 4) {
        const i32x8 a = {(int)x, (int)(x >> 1), (int)x, (int)(x << 1),
                         FORM == 4 ? (int)x : 0, FORM == 4 ? (int)x : 0,
                         FORM == 4 ? (int)x : 0, FORM == 4 ? (int)x : 0};
#pragma unroll
        for (int t = 0; t < 16; ++t)
          accf[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              a, a, accf[t], FORM == 0 ? 4 : 0, FORM == 0 ? 4 : 0, 0, 127, 0, 127);
      } else if constexpr (FORM == 2) {
        const i32x4 a = {(int)(x & 0x01010101u), (int)((x >> 1) & 0x01010101u), (int)x, 0};
#pragma unroll
        for (int t = 0; t < 16; ++t)
          acci[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, acci[t], 0, 0, 0);
      } else {
        bf16x8 a;
        for (int j = 0; j < 8; ++j) a[j] = (__bf16)(float)((x >> j) & 1);
#pragma unroll
        for (int t = 0; t < 16; ++t)
          accf[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, accf[t], 0, 0, 0);
      }
    }
    float s = 0.f;
    for (int t = 0; t < 16; ++t)
      for (int g = 0; g < 16; ++g) s += accf[t][g] + (float)acci[t][g];
    if (s == 12345.f) out[blockIdx.x] = s;
  } else {
    f32x4 acc[64];
    for (int t = 0; t < 64; ++t)
      for (int g = 0; g < 4; ++g) acc[t][g] = 0.f;
    for (int it = 0; it < ITERS / 4; ++it) {
      const uint32_t x = (uint32_t)(seed + it * 0x9E3779B9u + lane) & 0x22222222u;
      const i32x8 a = {(int)x, (int)(x >> 1), (int)x, (int)(x << 1), 0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 64; ++t)
        acc[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, acc[t], 4, 4, 0, 127, 0,
                                                                  127);
    }
    float s = 0.f;
    for (int t = 0; t < 64; ++t)
      for (int g = 0; g < 4; ++g) s += acc[t][g];
    if (s == 12345.f) out[blockIdx.x] = s;
  }
}

int main() {
  float* out;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 1024;
  auto run = [&](const char* name, auto launch, double mfmas_per_wave, double ops_per_mfma) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 10; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double ms = t[t.size() / 2];
    const double waves = blocks * 4.0, simds = 1024.0;
    const double per_simd = mfmas_per_wave * waves / simds;
    const double ns = ms * 1e6 / per_simd;
    std::printf("%-14s %.4f ms  %.2f ns/MFMA/SIMD  %.1f cyc@2.4GHz  %.0f TOP/s\n", name, ms, ns,
                ns * 2.4, mfmas_per_wave * waves * ops_per_mfma / (ms * 1e-3) * 1e-12);
    std::fflush(stdout);
  };
  const double m32 = 16.0 * ITERS;
  run("fp4 32x32x64", [&] { hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  run("fp4 16x16x128", [&] { hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      64.0 * (ITERS / 4), 2.0 * 16 * 16 * 128);
  run("i8 32x32x32", [&] { hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 32);
  run("bf16 32x32x16", [&] { hipLaunchKernelGGL(k_rate<3>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 16);
  run("fp8 32x32x64", [&] { hipLaunchKernelGGL(k_rate<4>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  run("fp4 4x4 expand", [&] { hipLaunchKernelGGL(k_rate<5>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  run("fp4 4x4 fixed", [&] { hipLaunchKernelGGL(k_rate<6>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  run("fp4 4x4 pingpong", [&] { hipLaunchKernelGGL(k_rate<7>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  run("fp4 4x4 cheapx", [&] { hipLaunchKernelGGL(k_rate<9>, dim3(blocks), dim3(256), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  // (8 waves a block: per SIMD twice the waves, each half the MFMAs an iteration)
  run("fp4 4x2 x8w", [&] { hipLaunchKernelGGL(k_rate<8>, dim3(blocks), dim3(512), 0, 0, 1, out); },
      m32, 2.0 * 32 * 32 * 64);
  return 0;
}
