// Store-shape micro, round 2 (session 3): does the random-row write rate of
// k_rows' shape depend on the allocation (physical placement)?  Eight
// matrices of the C3 shape (100,000 x 1,568 words, 1.25 GB each) allocated
// at once, each written with random rows (one 256-thread block per row, 16 B
// per lane, non-temporal), three rounds; then freed and re-allocated once.
// Build: hipcc --offload-arch=gfx950 -O3 -o store_bw4 store_bw4.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rows16(u64* M, const int* perm, long ldw, int W) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
  for (int w = threadIdx.x * 2; w < W; w += 512) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
}

int main() {
  const int n = 100000, W = 1563, NB = 8;
  const long ldw = 1568;
  std::vector<int> rnd(n);
  for (int i = 0; i < n; ++i) rnd[i] = i;
  std::shuffle(rnd.begin(), rnd.end(), std::mt19937(1));
  int* dp;
  hipMalloc(&dp, sizeof(int) * n);
  hipMemcpy(dp, rnd.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 8.0 * W * n;
  for (int gen = 0; gen < 2; ++gen) {
    std::vector<u64*> M(NB);
    for (int k = 0; k < NB; ++k) hipMalloc(&M[k], sizeof(u64) * ldw * n);
    for (int round = 0; round < 3; ++round) {
      printf("gen %d round %d:", gen, round);
      for (int k = 0; k < NB; ++k) {
        std::vector<float> ts;
        for (int rep = 0; rep < 7; ++rep) {
          hipEventRecord(a);
          hipLaunchKernelGGL(k_rows16, dim3(n), dim3(256), 0, 0, M[k], dp, ldw, W);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf(" %4.0f", bytes / (ts[3] * 1e-3) / 1e9);
      }
      printf("  GB/s (median of 7, per matrix)\n");
      fflush(stdout);
    }
    for (int k = 0; k < NB; ++k) hipFree(M[k]);
  }
  return 0;
}
