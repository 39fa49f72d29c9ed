// Placement micro (round 2): which 1.25 GB allocations take k_rows' random-row
// store shape fast?  12 hipMalloc'd matrices held at once, then freed and 12
// again, then 12 more after a 40 GB allocation is held; per matrix: virtual
// address and the median of 5 probe writes (one block per row, random row
// order, 16-B non-temporal lanes).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rows16(u64* M, const int* perm, long ldw, int W) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {0ull, 0ull};
  for (int w = threadIdx.x * 2; w < W; w += 512) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
}

int main() {
  const int n = 100000, W = 1568, NB = 12;
  const long ldw = 1568;
  const size_t bytes = sizeof(u64) * ldw * n;
  std::vector<int> rnd(n);
  for (int i = 0; i < n; ++i) rnd[i] = i;
  std::shuffle(rnd.begin(), rnd.end(), std::mt19937(1));
  int* dp;
  hipMalloc(&dp, sizeof(int) * n);
  hipMemcpy(dp, rnd.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto probe = [&](u64* M) {
    std::vector<float> ts;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      hipLaunchKernelGGL(k_rows16, dim3(n), dim3(256), 0, 0, M, dp, ldw, W);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return 8.0 * 1563 * n / (ts[2] * 1e-3) / 1e9;
  };
  void* big = nullptr;
  for (int gen = 0; gen < 3; ++gen) {
    if (gen == 2) hipMalloc(&big, (size_t)40 << 30);
    std::vector<u64*> M(NB);
    for (int k = 0; k < NB; ++k) hipMalloc(&M[k], bytes);
    for (int k = 0; k < NB; ++k)
      printf("gen %d cand %2d va %#llx  %.0f GB/s\n", gen, k, (unsigned long long)M[k], probe(M[k]));
    fflush(stdout);
    for (int k = 0; k < NB; ++k) hipFree(M[k]);
  }
  // a 12.5 GB block, probed at 10 offsets of 1.25 GB
  u64* B;
  hipMalloc(&B, bytes * 10);
  for (int k = 0; k < 10; ++k)
    printf("block offset %d  %.0f GB/s\n", k, probe(B + (size_t)k * ldw * n));
  return 0;
}
