// Store-rate control for the k_rows roofline: 1.25 GB written with 16-byte
// stores per lane (plain and non-temporal), (a) contiguously, (b) as 12.5 KB
// rows in a random row order (k_rows' pattern), one block per row.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
template <int NT_STORE>
__global__ __launch_bounds__(256) void k_rows_rand(u64* M, const int* perm, long ldw, int W) {
  const long r = perm[blockIdx.x];
  u64* dst = M + r * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
  for (int w = threadIdx.x * 2; w < W; w += 512) {
    if (NT_STORE) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
    else *(u64x2*)&dst[w] = v;
  }
}
template <int NT_STORE>
__global__ __launch_bounds__(256) void k_flat(u64* M, long nw) {
  const u64x2 v = {1ull, 2ull};
  for (long w = ((long)blockIdx.x * 256 + threadIdx.x) * 2; w < nw; w += (long)gridDim.x * 512) {
    if (NT_STORE) __builtin_nontemporal_store(v, (u64x2*)&M[w]);
    else *(u64x2*)&M[w] = v;
  }
}
// 4 stores in flight per lane per iteration
template <int NT_STORE>
__global__ __launch_bounds__(256) void k_flat4(u64* M, long nw) {
  const u64x2 v = {1ull, 2ull};
  const long step = (long)gridDim.x * 2048;
  for (long w = (long)blockIdx.x * 2048 + threadIdx.x * 2; w < nw; w += step) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long x = w + u * 512;
      if (x < nw) {
        if (NT_STORE) __builtin_nontemporal_store(v, (u64x2*)&M[x]);
        else *(u64x2*)&M[x] = v;
      }
    }
  }
}
// rows with 1024-thread blocks (one store per lane per row-sweep for W <= 2048)
__global__ __launch_bounds__(1024) void k_rows_1k(u64* M, const int* perm, long ldw, int W, int rows_per_block, int n) {
  const u64x2 v = {7ull, 1ull};
  for (int q = 0; q < rows_per_block; ++q) {
    const long i = (long)blockIdx.x * rows_per_block + q;
    if (i >= n) return;
    u64* dst = M + (long)perm[i] * ldw;
    for (int w = threadIdx.x * 2; w < W; w += 2048) *(u64x2*)&dst[w] = v;
  }
}
// the ROCm fill blit's shape: grid-stride, one 16-B store per lane per step
__global__ __launch_bounds__(256) void k_fill_like(u64* M, long nw, u64 val) {
  const u64x2 v = {val, val};
  const long step = (long)gridDim.x * 512;
  for (long w = ((long)blockIdx.x * 256 + threadIdx.x) * 2; w < nw; w += step)
    *(u64x2*)&M[w] = v;
}
template <int MODE>
__device__ __forceinline__ void st16(u64* dst, u64x2 v) {
  if (MODE == 0) asm volatile("global_store_dwordx4 %0, %1, off" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" : : "v"(dst), "v"(v) : "memory");
  if (MODE == 6) asm volatile("global_store_dwordx4 %0, %1, off sc0" : : "v"(dst), "v"(v) : "memory");
}
template <int MODE>
__global__ __launch_bounds__(256) void k_rows_mode(u64* M, const int* perm, long ldw, int W) {
  const long r = perm[blockIdx.x];
  u64* dst = M + r * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
  for (int w = threadIdx.x * 2; w < W; w += 512) st16<MODE>(&dst[w], v);
}
// the ROCm fill blit's per-lane shape: every lane writes a contiguous chunk
// (CH x 16 B) over CH store instructions; one wave per row
template <int CH>
__global__ __launch_bounds__(256) void k_rows_chunk(u64* M, const int* perm, long ldw, int W, int n) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long i = (long)blockIdx.x * 4 + wv;
  if (i >= n) return;
  u64* dst = M + (long)perm[i] * ldw;
  const u64x2 v = {(u64)i, 3ull};
  for (int w0 = lane * 2 * CH; w0 < W; w0 += 64 * 2 * CH) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int w = w0 + 2 * c;
      if (w < W) *(u64x2*)&dst[w] = v;
    }
  }
}
// torch's vectorized fill shape: one-shot blocks, 32 contiguous bytes per lane
__global__ __launch_bounds__(256) void k_flat32(u64* M, long nw) {
  const long w = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const u64x2 v = {1ull, 2ull};
  if (w + 3 < nw) {
    *(u64x2*)&M[w] = v;
    *(u64x2*)&M[w + 2] = v;
  }
}
// k_rows' shape with 32 bytes per lane: block per row
__global__ __launch_bounds__(256) void k_rows32(u64* M, const int* perm, long ldw, int W) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 5ull};
  for (int w = threadIdx.x * 4; w < W; w += 1024) {
    *(u64x2*)&dst[w] = v;
    if (w + 2 < W) *(u64x2*)&dst[w + 2] = v;
  }
}
// one-shot blocks of CHUNK bytes each, 16 or 32 B per lane, chunks in
// order or permuted
template <int PER_LANE>
__global__ __launch_bounds__(256) void k_chunks(u64* M, const int* cperm, long nchunks) {
  const long c = cperm ? cperm[blockIdx.x] : (long)blockIdx.x;
  constexpr int WPL = PER_LANE / 8;                     // words per lane
  const long w = c * 256 * WPL + (long)threadIdx.x * WPL;
  const u64x2 v = {(u64)c, 9ull};
  *(u64x2*)&M[w] = v;
  if (WPL == 4) *(u64x2*)&M[w + 2] = v;
}
int main() {
  const int n = 100000, W = 1563;
  const long ldw = 1568;
  u64* M;
  hipMalloc(&M, sizeof(u64) * ldw * n);
  std::vector<int> perm(n);
  for (int i = 0; i < n; ++i) perm[i] = i;
  int* dperm;
  hipMalloc(&dperm, sizeof(int) * n);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 8.0 * W * n;
  for (int shuffled = 0; shuffled < 2; ++shuffled) {
    if (shuffled) std::shuffle(perm.begin(), perm.end(), std::mt19937(1));
    hipMemcpy(dperm, perm.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    for (int nt = 0; nt < 2; ++nt) {
      float best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(a);
        if (nt) hipLaunchKernelGGL(k_rows_rand<1>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W);
        else hipLaunchKernelGGL(k_rows_rand<0>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
      }
      printf("rows %s %s: %.1f us  %.0f GB/s\n", shuffled ? "random" : "in-order", nt ? "nt" : "plain",
             best * 1e3, bytes / (best * 1e-3) / 1e9);
    }
  }
  for (int nt = 0; nt < 2; ++nt) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      if (nt) hipLaunchKernelGGL(k_flat<1>, dim3(8192), dim3(256), 0, 0, M, (long)W * n);
      else hipLaunchKernelGGL(k_flat<0>, dim3(8192), dim3(256), 0, 0, M, (long)W * n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("flat %s: %.1f us  %.0f GB/s\n", nt ? "nt" : "plain", best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  for (int nt = 0; nt < 2; ++nt) for (int g : {2048, 8192, 32768}) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      if (nt) hipLaunchKernelGGL(k_flat4<1>, dim3(g), dim3(256), 0, 0, M, (long)W * n);
      else hipLaunchKernelGGL(k_flat4<0>, dim3(g), dim3(256), 0, 0, M, (long)W * n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("flat4 %s grid %d: %.1f us  %.0f GB/s\n", nt ? "nt" : "plain", g, best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      hipMemsetAsync(M, 0, (size_t)8 * W * n, 0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("hipMemsetAsync: %.1f us  %.0f GB/s\n", best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  for (u64 val : {0ull, 0x0123456789abcdefull}) for (int g : {512, 1024, 2048, 4096, 16384}) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_fill_like, dim3(g), dim3(256), 0, 0, M, (long)W * n, val);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("fill-like val %s grid %d: %.1f us  %.0f GB/s\n", val ? "rand" : "zero", g, best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  {
    const char* names[] = {"plain", "nt", "sc1", "sc0 sc1", "sc0 sc1 nt", "sc1 nt", "sc0"};
    for (int mode = 0; mode < 7; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(a);
        switch (mode) {
          case 0: hipLaunchKernelGGL(k_rows_mode<0>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 1: hipLaunchKernelGGL(k_rows_mode<1>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 2: hipLaunchKernelGGL(k_rows_mode<2>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 3: hipLaunchKernelGGL(k_rows_mode<3>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 4: hipLaunchKernelGGL(k_rows_mode<4>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 5: hipLaunchKernelGGL(k_rows_mode<5>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
          case 6: hipLaunchKernelGGL(k_rows_mode<6>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
      }
      printf("rows random store %s: %.1f us  %.0f GB/s\n", names[mode], best * 1e3, bytes / (best * 1e-3) / 1e9);
    }
  }
  for (int ch : {1, 2, 4, 8, 16}) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      switch (ch) {
        case 1: hipLaunchKernelGGL(k_rows_chunk<1>, dim3((n + 3) / 4), dim3(256), 0, 0, M, dperm, ldw, W, n); break;
        case 2: hipLaunchKernelGGL(k_rows_chunk<2>, dim3((n + 3) / 4), dim3(256), 0, 0, M, dperm, ldw, W, n); break;
        case 4: hipLaunchKernelGGL(k_rows_chunk<4>, dim3((n + 3) / 4), dim3(256), 0, 0, M, dperm, ldw, W, n); break;
        case 8: hipLaunchKernelGGL(k_rows_chunk<8>, dim3((n + 3) / 4), dim3(256), 0, 0, M, dperm, ldw, W, n); break;
        case 16: hipLaunchKernelGGL(k_rows_chunk<16>, dim3((n + 3) / 4), dim3(256), 0, 0, M, dperm, ldw, W, n); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("rows random wave-per-row lane chunk %d x 16B: %.1f us  %.0f GB/s\n", ch, best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  for (int kind = 0; kind < 2; ++kind) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      if (kind == 0) hipLaunchKernelGGL(k_flat32, dim3((unsigned)(((long)W * n / 4 + 255) / 256)), dim3(256), 0, 0, M, (long)W * n);
      else hipLaunchKernelGGL(k_rows32, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("%s: %.1f us  %.0f GB/s\n", kind ? "rows random 32B/lane" : "flat 32B/lane one-shot", best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  {
    for (int per : {16, 32}) for (int permuted = 0; permuted < 2; ++permuted) {
      const long chunk_words = 256L * per / 8;
      const long nch = (long)W * n / chunk_words;
      std::vector<int> cp(nch);
      for (long i = 0; i < nch; ++i) cp[i] = (int)i;
      if (permuted) std::shuffle(cp.begin(), cp.end(), std::mt19937(3));
      int* dcp;
      hipMalloc(&dcp, sizeof(int) * nch);
      hipMemcpy(dcp, cp.data(), sizeof(int) * nch, hipMemcpyHostToDevice);
      float best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(a);
        if (per == 16) hipLaunchKernelGGL(k_chunks<16>, dim3((unsigned)nch), dim3(256), 0, 0, M, dcp, nch);
        else hipLaunchKernelGGL(k_chunks<32>, dim3((unsigned)nch), dim3(256), 0, 0, M, dcp, nch);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
      }
      hipFree(dcp);
      const double by = 8.0 * chunk_words * nch;
      printf("chunks %ld B, %d B/lane, %s: %.1f us  %.0f GB/s\n", chunk_words * 8, per,
             permuted ? "random order" : "in order", best * 1e3, by / (best * 1e-3) / 1e9);
    }
  }
  for (int rpb : {1, 4}) {
    float best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_rows_1k, dim3((n + rpb - 1) / rpb), dim3(1024), 0, 0, M, dperm, ldw, W, rpb, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    printf("rows random 1024-thread blocks, %d rows/block: %.1f us  %.0f GB/s\n", rpb, best * 1e3, bytes / (best * 1e-3) / 1e9);
  }
  return 0;
}
