// Store-shape micro, round 3 session 2: bytes per lane.  The runtime's memset
// writes 1.25 GB at 6.4-6.6 TB/s; flat grid-stride 16-B-per-lane stores at
// 5.5-5.6.  Does a lane writing 32 or 64 contiguous bytes (2 or 4
// dwordx4 stores at consecutive addresses), plain or non-temporal, close the
// gap -- flat, and in k_rows' shape (rows of 1,568 words, random / windowed /
// in order, one 256-thread block per row)?
// Build: hipcc --offload-arch=gfx950 -O3 -o store_bw7 store_bw7.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <int K, int NT>
__device__ __forceinline__ void put(u64* p, u64x2 v) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (NT) __builtin_nontemporal_store(v, (u64x2*)(p + 2 * k));
    else *(u64x2*)(p + 2 * k) = v;
  }
}
// flat: lane covers K*16 contiguous bytes, grid-stride
template <int K, int NT>
__global__ __launch_bounds__(256) void k_flat(u64* M, long nw) {
  const u64x2 v = {1ull, 2ull};
  const long per = 2L * K;   // words per lane
  const long step = (long)gridDim.x * 256 * per;
  for (long w = ((long)blockIdx.x * 256 + threadIdx.x) * per; w < nw; w += step)
    if (w + per <= nw) put<K, NT>(M + w, v);
}
// rows: one block per row; lane covers K*16 contiguous bytes, block strides
template <int K, int NT>
__global__ __launch_bounds__(256) void k_rows(u64* M, const int* perm, long ldw) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 1ull};
  const int per = 2 * K;
  for (int w = threadIdx.x * per; w < ldw; w += 256 * per)
    if (w + per <= ldw) put<K, NT>(dst + w, v);
}

int main() {
  const int n = 100000;
  const long ldw = 1568;   // 12,544 B = 196 x 64 B
  u64* M;
  hipMalloc(&M, sizeof(u64) * ldw * n);
  std::vector<int> ident(n), rnd(n), win(n);
  for (int i = 0; i < n; ++i) ident[i] = rnd[i] = win[i] = i;
  std::shuffle(rnd.begin(), rnd.end(), std::mt19937(1));
  {
    std::mt19937 g(7);
    for (int s = 0; s < n; s += 2048) std::shuffle(win.begin() + s, win.begin() + std::min(n, s + 2048), g);
  }
  auto up = [&](const std::vector<int>& h) {
    int* d;
    hipMalloc(&d, sizeof(int) * n);
    hipMemcpy(d, h.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    return d;
  };
  int *did = up(ident), *drnd = up(rnd), *dwin = up(win);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 8.0 * ldw * n;
  auto timeit = [&](const char* name, auto launch) {
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
    printf("%-36s best %.1f us  median %.1f us  %.0f GB/s (median)\n", name, ts[0] * 1e3, ts[4] * 1e3,
           bytes / (ts[4] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const long nw = ldw * n;
#define FLAT(K, NT, G)                                                                       \
  timeit("flat " #K "x16B nt" #NT " grid " #G,                                               \
         [&] { hipLaunchKernelGGL((k_flat<K, NT>), dim3(G), dim3(256), 0, 0, M, nw); })
#define ROWS(K, NT, P, NM)                                                                   \
  timeit("rows " #K "x16B nt" #NT " " NM,                                                    \
         [&] { hipLaunchKernelGGL((k_rows<K, NT>), dim3(n), dim3(256), 0, 0, M, P, ldw); })
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    timeit("memset", [&] { hipMemsetAsync(M, 0, (size_t)8 * ldw * n, 0); });
    FLAT(1, 0, 8192); FLAT(1, 1, 8192); FLAT(2, 0, 8192); FLAT(2, 1, 8192);
    FLAT(4, 0, 8192); FLAT(4, 1, 8192); FLAT(4, 0, 2048); FLAT(4, 0, 32768);
    ROWS(1, 1, drnd, "random"); ROWS(1, 0, drnd, "random");
    ROWS(2, 0, drnd, "random"); ROWS(2, 1, drnd, "random");
    ROWS(4, 0, drnd, "random"); ROWS(4, 1, drnd, "random");
    ROWS(1, 1, dwin, "win 2048"); ROWS(4, 0, dwin, "win 2048"); ROWS(4, 1, dwin, "win 2048");
    ROWS(1, 1, did, "in order"); ROWS(4, 0, did, "in order"); ROWS(4, 1, did, "in order");
  }
  return 0;
}
