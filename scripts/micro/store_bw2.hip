// Store-shape micro, round 3: what write shape of k_rows' C3 matrix (100,000
// rows x 1,563 words in random row order) gets closest to the runtime's
// memset on the same box?
//   rows16      one 256-thread block per row, 16 B per lane (k_rows' shape)
//   rowsdw      one 256-thread block per row, one dword per lane (256 B per
//               wave-instruction: MI355X_MICROARCH.md's 6.0-6.2 TB/s shape)
//   persist K   rows16 / rowsdw over a grid of K blocks per CU
//   copy        the two-phase form's second phase: M[i] = T[cls[i]] in pod
//               order from a class-row table T (11,500 rows, 144 MB: MALL)
// Build: hipcc --offload-arch=gfx950 -O3 -o store_bw2 store_bw2.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include <cstdlib>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <int NTS>
__global__ __launch_bounds__(256) void k_rows16(u64* M, const int* perm, long ldw, int W, int n) {
  for (long r = blockIdx.x; r < n; r += gridDim.x) {
    u64* dst = M + (long)perm[r] * ldw;
    const u64x2 v = {(u64)r, 1ull};
    for (int w = threadIdx.x * 2; w < W; w += 512) {
      if (NTS) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
      else *(u64x2*)&dst[w] = v;
    }
  }
}
// 4 stores in flight per lane, grid-stride over the whole buffer in order
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
__global__ __launch_bounds__(256) void k_rowsdw(u64* M, const int* perm, long ldw, int W, int n) {
  const int Wd = 2 * W;
  for (long r = blockIdx.x; r < n; r += gridDim.x) {
    unsigned* dst = (unsigned*)(M + (long)perm[r] * ldw);
    for (int w = threadIdx.x; w < Wd; w += 256) dst[w] = (unsigned)r;
  }
}
// dword per lane, each wave writing 4 wave-instructions of 256 B at 1 KB apart
__global__ __launch_bounds__(256) void k_rowsdw4(u64* M, const int* perm, long ldw, int W, int n) {
  const int Wd = 2 * W;
  for (long r = blockIdx.x; r < n; r += gridDim.x) {
    unsigned* dst = (unsigned*)(M + (long)perm[r] * ldw);
    for (int w0 = threadIdx.x; w0 < Wd; w0 += 1024) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (w0 + u * 256 < Wd) dst[w0 + u * 256] = (unsigned)r;
    }
  }
}
// 16 B per lane, the row's four 4-KB pieces issued back to back per lane
__global__ __launch_bounds__(256) void k_rows16u(u64* M, const int* perm, long ldw, int W, int n) {
  for (long r = blockIdx.x; r < n; r += gridDim.x) {
    u64* dst = M + (long)perm[r] * ldw;
    const u64x2 v = {(u64)r, 1ull};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int w = threadIdx.x * 2 + u * 512;
      if (w < W) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
    }
  }
}
// one-shot blocks of 8 KB (32 B per lane), chunk order given by cperm (or in
// order); value 0 or the chunk index
__global__ __launch_bounds__(256) void k_chunk32(u64* M, const int* cperm, int zero) {
  const long c = cperm ? cperm[blockIdx.x] : (long)blockIdx.x;
  const long w = c * 1024 + (long)threadIdx.x * 4;
  const u64x2 v = {zero ? 0ull : (u64)c, zero ? 0ull : 9ull};
  __builtin_nontemporal_store(v, (u64x2*)&M[w]);
  __builtin_nontemporal_store(v, (u64x2*)&M[w + 2]);
}
// block per row, 32 B per lane (8 KB per block iteration)
__global__ __launch_bounds__(256) void k_rows32(u64* M, const int* perm, long ldw, int W, int n) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 5ull};
  for (int w = threadIdx.x * 4; w < W; w += 1024) {
    __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
    if (w + 2 < W) __builtin_nontemporal_store(v, (u64x2*)&dst[w + 2]);
  }
}
// 1024-thread block per row, 16 B per lane (the row in one store per lane)
__global__ __launch_bounds__(1024) void k_rows1k(u64* M, const int* perm, long ldw, int W, int n) {
  u64* dst = M + (long)perm[blockIdx.x] * ldw;
  const u64x2 v = {(u64)blockIdx.x, 5ull};
  const int w = threadIdx.x * 2;
  if (w < W) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
}
// phase 2 of the two-phase form: M in pod order from the class-row table
template <int NTS>
__global__ __launch_bounds__(256) void k_copy(u64* M, const u64* T, const int* cls, long ldw, int W, int n) {
  for (long r = blockIdx.x; r < n; r += gridDim.x) {
    const u64* src = T + (long)cls[r] * ldw;
    u64* dst = M + r * ldw;
    u64x2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int w = threadIdx.x * 2 + u * 512;
      if (w < W) v[u] = *(const u64x2*)&src[w];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int w = threadIdx.x * 2 + u * 512;
      if (w < W) {
        if (NTS) __builtin_nontemporal_store(v[u], (u64x2*)&dst[w]);
        else *(u64x2*)&dst[w] = v[u];
      }
    }
  }
}

int main() {
  const int n = 100000, W = 1563, ncls = 11500;
  const long ldw = 1568;
  u64 *M, *T;
  hipMalloc(&M, sizeof(u64) * 2048 * n);
  hipMalloc(&T, sizeof(u64) * ldw * ncls);
  hipMemset(T, 0x5a, sizeof(u64) * ldw * ncls);
  std::vector<int> perm(n), cls(n);
  for (int i = 0; i < n; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), std::mt19937(1));
  std::mt19937 g2(2);
  for (int i = 0; i < n; ++i) cls[i] = (int)(g2() % ncls);
  std::vector<int> ident(n), blk(n);
  for (int i = 0; i < n; ++i) ident[i] = i;
  {  // random order of 64-row runs, rows in order inside a run
    std::vector<int> runs((n + 63) / 64);
    for (size_t i = 0; i < runs.size(); ++i) runs[i] = (int)i;
    std::shuffle(runs.begin(), runs.end(), std::mt19937(5));
    int k = 0;
    for (int r : runs) for (int i = r * 64; i < std::min(n, r * 64 + 64); ++i) blk[k++] = i;
  }
  int *dident, *dblk;
  hipMalloc(&dident, sizeof(int) * n);
  hipMalloc(&dblk, sizeof(int) * n);
  hipMemcpy(dident, ident.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  hipMemcpy(dblk, blk.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  int *dperm, *dcls;
  hipMalloc(&dperm, sizeof(int) * n);
  hipMalloc(&dcls, sizeof(int) * n);
  hipMemcpy(dperm, perm.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  hipMemcpy(dcls, cls.data(), sizeof(int) * n, hipMemcpyHostToDevice);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 8.0 * W * n;
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
    printf("%-34s best %.1f us  median %.1f us  %.0f GB/s (median)\n", name, ts[0] * 1e3, ts[4] * 1e3,
           bytes / (ts[4] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const long nch = (long)ldw * n / 1024;
  std::vector<int> cpv(nch);
  for (long i = 0; i < nch; ++i) cpv[i] = (int)i;
  std::shuffle(cpv.begin(), cpv.end(), std::mt19937(3));
  int* dcp;
  hipMalloc(&dcp, sizeof(int) * nch);
  hipMemcpy(dcp, cpv.data(), sizeof(int) * nch, hipMemcpyHostToDevice);
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d (b)\n", pass);
    timeit("memset", [&] { hipMemsetAsync(M, 0, (size_t)8 * ldw * n, 0); });
    timeit("chunk32 in order zero", [&] { hipLaunchKernelGGL(k_chunk32, dim3(nch), dim3(256), 0, 0, M, (const int*)nullptr, 1); });
    timeit("chunk32 in order value", [&] { hipLaunchKernelGGL(k_chunk32, dim3(nch), dim3(256), 0, 0, M, (const int*)nullptr, 0); });
    timeit("chunk32 random zero", [&] { hipLaunchKernelGGL(k_chunk32, dim3(nch), dim3(256), 0, 0, M, dcp, 1); });
    timeit("chunk32 random value", [&] { hipLaunchKernelGGL(k_chunk32, dim3(nch), dim3(256), 0, 0, M, dcp, 0); });
    timeit("rows32 random", [&] { hipLaunchKernelGGL(k_rows32, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    timeit("rows32 in order", [&] { hipLaunchKernelGGL(k_rows32, dim3(n), dim3(256), 0, 0, M, dident, ldw, W, n); });
    timeit("rows1k random", [&] { hipLaunchKernelGGL(k_rows1k, dim3(n), dim3(1024), 0, 0, M, dperm, ldw, W, n); });
    timeit("rows1k in order", [&] { hipLaunchKernelGGL(k_rows1k, dim3(n), dim3(1024), 0, 0, M, dident, ldw, W, n); });
    timeit("rows16 nt random", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
  }
  if (getenv("ONLY_B")) return 0;
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    timeit("memset", [&] { hipMemsetAsync(M, 0, (size_t)8 * ldw * n, 0); });
    timeit("rows16 nt in order", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dident, ldw, W, n); });
    timeit("rows16 nt 64-row runs", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dblk, ldw, W, n); });
    timeit("rows16 plain in order", [&] { hipLaunchKernelGGL(k_rows16<0>, dim3(n), dim3(256), 0, 0, M, dident, ldw, W, n); });
    timeit("rows16u nt in order", [&] { hipLaunchKernelGGL(k_rows16u, dim3(n), dim3(256), 0, 0, M, dident, ldw, W, n); });
    timeit("flat4 nt grid 32768", [&] { hipLaunchKernelGGL(k_flat4, dim3(32768), dim3(256), 0, 0, M, (long)ldw * n); });
    timeit("rows16 nt random, pitch 2048", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dperm, 2048L, W, n); });
    timeit("rows16 nt in order, pitch 2048", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dident, 2048L, W, n); });
    timeit("rows16 plain", [&] { hipLaunchKernelGGL(k_rows16<0>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    timeit("rows16 nt", [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    timeit("rows16u nt", [&] { hipLaunchKernelGGL(k_rows16u, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    timeit("rowsdw", [&] { hipLaunchKernelGGL(k_rowsdw, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    timeit("rowsdw4", [&] { hipLaunchKernelGGL(k_rowsdw4, dim3(n), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    for (int k : {1, 2, 4, 8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "rows16 nt persist %d/CU", k);
      timeit(nm, [&] { hipLaunchKernelGGL(k_rows16<1>, dim3(k * ncu), dim3(256), 0, 0, M, dperm, ldw, W, n); });
      snprintf(nm, sizeof nm, "rowsdw persist %d/CU", k);
      timeit(nm, [&] { hipLaunchKernelGGL(k_rowsdw, dim3(k * ncu), dim3(256), 0, 0, M, dperm, ldw, W, n); });
    }
    timeit("copy T->M plain", [&] { hipLaunchKernelGGL(k_copy<0>, dim3(n), dim3(256), 0, 0, M, T, dcls, ldw, W, n); });
    timeit("copy T->M nt", [&] { hipLaunchKernelGGL(k_copy<1>, dim3(n), dim3(256), 0, 0, M, T, dcls, ldw, W, n); });
    timeit("copy T->M nt persist 4/CU", [&] { hipLaunchKernelGGL(k_copy<1>, dim3(4 * ncu), dim3(256), 0, 0, M, T, dcls, ldw, W, n); });
  }
  return 0;
}
