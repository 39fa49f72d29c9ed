// Store-shape micro, round 3 session 2: does k_rows' random-row write lose
// to the runtime's memset because every row ends in a partly written 64-B
// piece (W = 1,563 words of a 1,568-word pitch: the last 16-B store ends 32 B
// into a 64-B piece), or because of the row order?  Rows written to the full
// pitch cover whole 128-B lines.
//   rowsW   one 256-thread block per row, 16 B per lane, W words of each row
//   rowsWu  the same with the row's four 4-KB pieces issued back to back
//   cls16   k_rows' shape: a block per class of up to 16 member rows, the
//           row in LDS, streamed to each member (random members)
//   win R   rows in random order inside windows of R rows, windows in order
// Build: hipcc --offload-arch=gfx950 -O3 -o store_bw6 store_bw6.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rowsW(u64* M, const int* perm, long ldw, int W) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
  for (int w = threadIdx.x * 2; w < W; w += 512) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
}
__global__ __launch_bounds__(256) void k_rowsWu(u64* M, const int* perm, long ldw, int W) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int w = threadIdx.x * 2 + u * 512;
    if (w < W) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
  }
}
// members of "class" b: rows perm[16b .. 16b+16)
__global__ __launch_bounds__(256) void k_cls16(u64* M, const int* perm, long ldw, int W, int n, int ch) {
  extern __shared__ __attribute__((aligned(16))) u64 row[];
  for (int w = threadIdx.x; w < W; w += 256) row[w] = (u64)w * 3 + blockIdx.x;
  __syncthreads();
  const int m0 = blockIdx.x * ch, m1 = min(n, m0 + ch);
  for (int m = m0; m < m1; ++m) {
    u64* dst = M + (long)perm[m] * ldw;
    for (int w = threadIdx.x * 2; w < W; w += 512)
      __builtin_nontemporal_store(*(const u64x2*)&row[w], (u64x2*)&dst[w]);
  }
}
__global__ __launch_bounds__(256) void k_flat4(u64* M, long nw) {
  const u64x2 v = {1ull, 2ull};
  const long step = (long)gridDim.x * 2048;
  for (long w = (long)blockIdx.x * 2048 + threadIdx.x * 2; w < nw; w += step) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long x = w + u * 512;
      if (x < nw) __builtin_nontemporal_store(v, (u64x2*)&M[x]);
    }
  }
}

int main() {
  const int n = 100000;
  const long ldw = 1568;
  u64* M;
  hipMalloc(&M, sizeof(u64) * ldw * n);
  std::vector<int> ident(n), rnd(n);
  for (int i = 0; i < n; ++i) ident[i] = rnd[i] = i;
  std::shuffle(rnd.begin(), rnd.end(), std::mt19937(1));
  auto windowed = [&](int R) {
    std::vector<int> v(ident);
    std::mt19937 g(7);
    for (int s = 0; s < n; s += R) std::shuffle(v.begin() + s, v.begin() + std::min(n, s + R), g);
    return v;
  };
  auto up = [&](const std::vector<int>& h) {
    int* d;
    hipMalloc(&d, sizeof(int) * n);
    hipMemcpy(d, h.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    return d;
  };
  int *did = up(ident), *drnd = up(rnd), *dw512 = up(windowed(512)), *dw2k = up(windowed(2048)),
      *dw8k = up(windowed(8192));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto timeit = [&](const char* name, double bytes, auto launch) {
    std::vector<float> ts;
    for (int rep = 0; rep < 9; ++rep) {
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-40s best %.1f us  median %.1f us  %.0f GB/s (median)\n", name, ts[0] * 1e3, ts[4] * 1e3,
           bytes / (ts[4] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const int Ws[2] = {1563, 1568};
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    timeit("memset", 8.0 * ldw * n, [&] { hipMemsetAsync(M, 0, (size_t)8 * ldw * n, 0); });
    timeit("flat4 grid 32768", 8.0 * ldw * n,
           [&] { hipLaunchKernelGGL(k_flat4, dim3(32768), dim3(256), 0, 0, M, ldw * n); });
    for (int W : Ws) {
      char nm[96];
      const double by = 8.0 * W * n;
      snprintf(nm, sizeof nm, "rowsW W=%d in order", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsW, dim3(n), dim3(256), 0, 0, M, did, ldw, W); });
      snprintf(nm, sizeof nm, "rowsW W=%d random", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsW, dim3(n), dim3(256), 0, 0, M, drnd, ldw, W); });
      snprintf(nm, sizeof nm, "rowsWu W=%d random", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsWu, dim3(n), dim3(256), 0, 0, M, drnd, ldw, W); });
      snprintf(nm, sizeof nm, "rowsW W=%d win 512", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsW, dim3(n), dim3(256), 0, 0, M, dw512, ldw, W); });
      snprintf(nm, sizeof nm, "rowsW W=%d win 2048", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsW, dim3(n), dim3(256), 0, 0, M, dw2k, ldw, W); });
      snprintf(nm, sizeof nm, "rowsW W=%d win 8192", W);
      timeit(nm, by, [&] { hipLaunchKernelGGL(k_rowsW, dim3(n), dim3(256), 0, 0, M, dw8k, ldw, W); });
      for (int ch : {4, 16}) {
        const unsigned nb = (unsigned)((n + ch - 1) / ch);
        snprintf(nm, sizeof nm, "cls%d W=%d random", ch, W);
        timeit(nm, by, [&] {
          hipLaunchKernelGGL(k_cls16, dim3(nb), dim3(256), 8 * ldw, 0, M, drnd, ldw, W, n, ch);
        });
        snprintf(nm, sizeof nm, "cls%d W=%d win 2048", ch, W);
        timeit(nm, by, [&] {
          hipLaunchKernelGGL(k_cls16, dim3(nb), dim3(256), 8 * ldw, 0, M, dw2k, ldw, W, n, ch);
        });
        snprintf(nm, sizeof nm, "cls%d W=%d in order", ch, W);
        timeit(nm, by, [&] {
          hipLaunchKernelGGL(k_cls16, dim3(nb), dim3(256), 8 * ldw, 0, M, did, ldw, W, n, ch);
        });
      }
    }
  }
  return 0;
}
