// The matrix write as a copy from a table of distinct rows (C3: 3,928
// distinct select lists, 12.5 KB rows = 49 MB, Infinity-Cache resident):
// M[i] = T[map[i]] for 100,000 rows, one-shot blocks in address order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef long i64;

// each thread one 16-B piece; block = 256 threads = 4 KB of M
template <bool NT>
__global__ __launch_bounds__(256) void k_copy1(u64* __restrict__ M, const u64* __restrict__ T,
                                               const int* __restrict__ map, i64 rows, i64 ldM) {
  const i64 piece = (i64)blockIdx.x * 256 + threadIdx.x;   // 16-B pieces of M
  const i64 w = piece * 2;
  const i64 r = w / ldM, c = w - r * ldM;
  if (r >= rows) return;
  const u64x2 v = *(const u64x2*)(T + (i64)map[r] * ldM + c);
  if (NT) __builtin_nontemporal_store(v, (u64x2*)(M + w));
  else *(u64x2*)(M + w) = v;
}
// U pieces per thread, block-contiguous
template <int U>
__global__ __launch_bounds__(256) void k_copyU(u64* __restrict__ M, const u64* __restrict__ T,
                                               const int* __restrict__ map, i64 rows, i64 ldM) {
  const i64 base = (i64)blockIdx.x * 256 * U;
  u64x2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const i64 w = (base + u * 256 + threadIdx.x) * 2;
    const i64 r = w / ldM, c = w - r * ldM;
    v[u] = r < rows ? *(const u64x2*)(T + (i64)map[r] * ldM + c) : u64x2{0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const i64 w = (base + u * 256 + threadIdx.x) * 2;
    if (w / ldM < rows) *(u64x2*)(M + w) = v[u];
  }
}

int main() {
  const i64 rows = 100000, ldM = 1568, U = 3928;
  std::vector<int> map(rows);
  std::mt19937 g(1);
  for (auto& x : map) x = (int)(g() % U);
  u64 *M, *T;
  int* dmap;
  hipMalloc(&M, rows * ldM * 8);
  hipMalloc(&T, U * ldM * 8);
  hipMalloc(&dmap, rows * 4);
  hipMemset(T, 0x5a, U * ldM * 8);
  hipMemcpy(dmap, map.data(), rows * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)rows * ldM * 8;
  auto run = [&](const char* name, auto fn) {
    for (int i = 0; i < 2; ++i) fn();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-36s %.4f ms  %.0f GB/s written\n", name, ms, bytes / ms / 1e6);
  };
  const i64 pieces = rows * ldM / 2;
  run("copy U1 plain", [&] { hipLaunchKernelGGL(k_copy1<false>, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, 0, M, T, dmap, rows, ldM); });
  run("copy U1 nt", [&] { hipLaunchKernelGGL(k_copy1<true>, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, 0, M, T, dmap, rows, ldM); });
  run("copy U2", [&] { hipLaunchKernelGGL(k_copyU<2>, dim3((unsigned)((pieces + 511) / 512)), dim3(256), 0, 0, M, T, dmap, rows, ldM); });
  run("copy U4", [&] { hipLaunchKernelGGL(k_copyU<4>, dim3((unsigned)((pieces + 1023) / 1024)), dim3(256), 0, 0, M, T, dmap, rows, ldM); });
  run("memset", [&] { hipMemsetAsync(M, 0, rows * ldM * 8, 0); });
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
