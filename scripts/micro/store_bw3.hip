// Store-shape micro, round 2 (session 3): is k_rows' random-row penalty a
// per-XCD translation (TLB) effect?  The C3 matrix (100,000 rows x 1,563
// words, pitch 1,568) written one 256-thread block per row, 16 B per lane,
// non-temporal, rows in:
//   random      a random permutation (k_rows' class order)
//   xcd-local   random rows, but block b (dispatched to XCD b mod 8) only
//               writes rows of region b mod 8 (n/8 consecutive rows)
//   xcd-inorder block b writes row (b mod 8) * n/8 + b / 8: in order per XCD
//   in order    block b writes row b
// Build: hipcc --offload-arch=gfx950 -O3 -o store_bw3 store_bw3.hip
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
  const int n = 100000, W = 1563;
  const long ldw = 1568;
  u64* M;
  hipMalloc(&M, sizeof(u64) * ldw * n);
  std::mt19937 g(1);
  std::vector<int> rnd(n), loc(n), xin(n), ord(n);
  for (int i = 0; i < n; ++i) rnd[i] = ord[i] = i;
  std::shuffle(rnd.begin(), rnd.end(), g);
  const int R = n / 8;
  std::vector<std::vector<int>> reg(8);
  for (int r = 0; r < 8; ++r) {
    for (int i = r * R; i < (r == 7 ? n : (r + 1) * R); ++i) reg[r].push_back(i);
    std::shuffle(reg[r].begin(), reg[r].end(), g);
  }
  std::vector<size_t> pos(8, 0);
  for (int b = 0; b < n; ++b) {
    int r = b % 8;
    if (pos[r] >= reg[r].size()) r = 7;   // the tail region holds the remainder
    loc[b] = reg[r][pos[r]++];
  }
  for (int r = 0; r < 8; ++r) std::sort(reg[r].begin(), reg[r].end());
  std::fill(pos.begin(), pos.end(), 0);
  for (int b = 0; b < n; ++b) {
    int r = b % 8;
    if (pos[r] >= reg[r].size()) r = 7;
    xin[b] = reg[r][pos[r]++];
  }
  int* d[4];
  const std::vector<int>* src[4] = {&rnd, &loc, &xin, &ord};
  const char* names[4] = {"random", "xcd-local random", "xcd-local in order", "in order"};
  for (int k = 0; k < 4; ++k) {
    hipMalloc(&d[k], sizeof(int) * n);
    hipMemcpy(d[k], src[k]->data(), sizeof(int) * n, hipMemcpyHostToDevice);
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 8.0 * W * n;
  for (int pass = 0; pass < 3; ++pass) {
    for (int k = 0; k < 4; ++k) {
      std::vector<float> ts;
      for (int rep = 0; rep < 9; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_rows16, dim3(n), dim3(256), 0, 0, M, d[k], ldw, W);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      printf("pass %d %-20s median %.1f us  %.0f GB/s\n", pass, names[k], ts[4] * 1e3,
             bytes / (ts[4] * 1e-3) / 1e9);
    }
    std::vector<float> ts;
    for (int rep = 0; rep < 9; ++rep) {
      hipEventRecord(a);
      hipMemsetAsync(M, 0, sizeof(u64) * ldw * n, 0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("pass %d %-20s median %.1f us  %.0f GB/s\n", pass, "memset", ts[4] * 1e3,
           bytes / (ts[4] * 1e-3) / 1e9);
  }
  return 0;
}
