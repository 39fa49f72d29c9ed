// Does the ORDER in which k_rows' blocks write their rows cost store
// bandwidth?  C3 shape (100,000 rows x 1,568 words = 1.25 GB): each block
// writes R whole rows (16 B per lane, the k_rows store loop) picked from a
// row list -- in address order, or a random permutation (k_rows' member
// rows: a class's pods are scattered over the matrix).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef long i64;

template <int R, bool NT>
__global__ __launch_bounds__(256) void k_rows_list(u64* M, i64 ldM, const int* rows, int nrows) {
  const i64 r0 = (i64)blockIdx.x * R;
  for (int q = 0; q < R; ++q) {
    if (r0 + q >= nrows) return;
    u64* dst = M + (i64)rows[r0 + q] * ldM;
    const u64x2 v = {(u64)q, (u64)r0};
    for (i64 w = threadIdx.x * 2; w < ldM; w += 512) {
      if (NT) __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
      else *(u64x2*)&dst[w] = v;
    }
  }
}

// 32 B per lane: two adjacent 16-B stores
template <int R, bool NT>
__global__ __launch_bounds__(256) void k_rows_list32(u64* M, i64 ldM, const int* rows, int nrows) {
  const i64 r0 = (i64)blockIdx.x * R;
  for (int q = 0; q < R; ++q) {
    if (r0 + q >= nrows) return;
    u64* dst = M + (i64)rows[r0 + q] * ldM;
    const u64x2 v = {(u64)q, (u64)r0};
    for (i64 w = threadIdx.x * 4; w < ldM; w += 1024) {
      if (NT) {
        __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
        if (w + 2 < ldM) __builtin_nontemporal_store(v, (u64x2*)&dst[w + 2]);
      } else {
        *(u64x2*)&dst[w] = v;
        if (w + 2 < ldM) *(u64x2*)&dst[w + 2] = v;
      }
    }
  }
}
// one-shot: block = (row, 1024-word chunk), 32 B per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_chunk32(u64* M, i64 ldM, const int* rows, int nrows) {
  const i64 nch = (ldM + 1023) / 1024;
  const i64 b = blockIdx.x, r = b / nch, ch = b % nch;
  if (r >= nrows) return;
  u64* dst = M + (i64)rows[r] * ldM + ch * 1024;
  const i64 w = threadIdx.x * 4;
  if (ch * 1024 + w >= ldM) return;
  const u64x2 v = {(u64)r, (u64)ch};
  if (NT) {
    __builtin_nontemporal_store(v, (u64x2*)&dst[w]);
    __builtin_nontemporal_store(v, (u64x2*)&dst[w + 2]);
  } else {
    *(u64x2*)&dst[w] = v;
    *(u64x2*)&dst[w + 2] = v;
  }
}

template <int R, bool NT, int KIND = 0>
float run(u64* M, i64 ldM, const int* rows, int nrows) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned grid = KIND == 2 ? (unsigned)(nrows * ((ldM + 1023) / 1024))
                                   : (unsigned)((nrows + R - 1) / R);
  std::vector<float> t;
  for (int rep = 0; rep < 12; ++rep) {
    hipEventRecord(e0);
    if (KIND == 0)
      hipLaunchKernelGGL((k_rows_list<R, NT>), dim3(grid), dim3(256), 0, 0, M, ldM, rows, nrows);
    else if (KIND == 1)
      hipLaunchKernelGGL((k_rows_list32<R, NT>), dim3(grid), dim3(256), 0, 0, M, ldM, rows, nrows);
    else
      hipLaunchKernelGGL((k_chunk32<NT>), dim3(grid), dim3(256), 0, 0, M, ldM, rows, nrows);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep >= 2) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const int n = 100000;
  const i64 ldM = 1568;
  const double bytes = (double)n * ldM * 8;
  u64* M;
  if (hipMalloc(&M, (size_t)bytes) != hipSuccess) return 1;
  std::vector<int> seq(n), rnd(n), blk(n);
  std::iota(seq.begin(), seq.end(), 0);
  rnd = seq;
  std::mt19937 g(7);
  std::shuffle(rnd.begin(), rnd.end(), g);
  // random 16-row groups, each group's rows ascending (a sorted member list)
  blk = rnd;
  for (int i = 0; i < n; i += 16) std::sort(blk.begin() + i, blk.begin() + std::min(n, i + 16));
  int *dseq, *drnd, *dblk;
  hipMalloc(&dseq, n * 4);
  hipMalloc(&drnd, n * 4);
  hipMalloc(&dblk, n * 4);
  hipMemcpy(dseq, seq.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(drnd, rnd.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dblk, blk.data(), n * 4, hipMemcpyHostToDevice);
  hipMemset(M, 0, (size_t)bytes);
  hipDeviceSynchronize();
  struct L { const char* name; const int* rows; };
  for (L l : {L{"address-order", dseq}, L{"random", drnd}, L{"random, 16 sorted", dblk}}) {
    printf("%-18s R=1 nt %.0f plain %.0f | R=4 nt %.0f plain %.0f | R=16 nt %.0f plain %.0f GB/s\n",
           l.name, bytes / run<1, true>(M, ldM, l.rows, n) / 1e6,
           bytes / run<1, false>(M, ldM, l.rows, n) / 1e6,
           bytes / run<4, true>(M, ldM, l.rows, n) / 1e6,
           bytes / run<4, false>(M, ldM, l.rows, n) / 1e6,
           bytes / run<16, true>(M, ldM, l.rows, n) / 1e6,
           bytes / run<16, false>(M, ldM, l.rows, n) / 1e6);
    printf("%-18s 32B/lane R=1 nt %.0f plain %.0f | R=16 nt %.0f plain %.0f | chunk32 nt %.0f plain %.0f GB/s\n",
           l.name, bytes / run<1, true, 1>(M, ldM, l.rows, n) / 1e6,
           bytes / run<1, false, 1>(M, ldM, l.rows, n) / 1e6,
           bytes / run<16, true, 1>(M, ldM, l.rows, n) / 1e6,
           bytes / run<16, false, 1>(M, ldM, l.rows, n) / 1e6,
           bytes / run<1, true, 2>(M, ldM, l.rows, n) / 1e6,
           bytes / run<1, false, 2>(M, ldM, l.rows, n) / 1e6);
  }
  // the runtime's fill of the same bytes
  {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> t;
    for (int rep = 0; rep < 12; ++rep) {
      hipEventRecord(e0);
      hipMemsetAsync(M, rep, (size_t)bytes);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("hipMemset %.0f GB/s\n", bytes / t[t.size() / 2] / 1e6);
  }
  hipFree(M);
  return 0;
}
