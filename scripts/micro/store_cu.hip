// Store rate against the CUs a stream may use (round 4): the pipelined
// matrix write runs on a CU-masked stream (96 of 256 CUs at C3) and reaches
// ~3.5 TB/s there.  Is that the CUs' store ceiling or k_rows' own cost (the
// LDS row builds between the stores)?  1.25 GB written with 16-B
// non-temporal lane stores:
//   flat    grid-stride over the whole buffer, 8 blocks per CU of the mask
//   rows16  k_rows' shape without the build: a 256-thread block per class of
//           16 random member rows of 1,568 words, the row from LDS
// on streams masked to K CUs of every XCD, K = 4 .. 32.
// Round 4, one box: rows16 4.75 / 4.75 / 4.87 / 4.79 TB/s on 256 / 192 / 160
// / 128 CUs (37 GB/s per CU at 128); flat 4.2 / 5.45 / 5.82 / 3.90; the run
// stopped at its time limit in the 96-CU stream (not understood; the
// engine's own 96-CU stream runs every bench step), so that point is missing.
// Build: hipcc --offload-arch=gfx950 -O3 -o store_cu store_cu.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__global__ __launch_bounds__(256) void k_flat(u64* M, long nvec) {
  u64x2 v = {(u64)blockIdx.x, ~0ull};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(v, (u64x2*)M + i);
}

__global__ __launch_bounds__(256) void k_rows16(u64* M, const int* perm, long n, long ldw, int W) {
  extern __shared__ __attribute__((aligned(16))) u64 row[];
  for (int w = threadIdx.x; w < W; w += 256) row[w] = (u64)w * 0x9E3779B97F4A7C15ull ^ blockIdx.x;
  __syncthreads();
  const long m0 = (long)blockIdx.x * 16, m1 = m0 + 16 < n ? m0 + 16 : n;
  for (long m = m0; m < m1; ++m) {
    u64* dst = M + (long)perm[m] * ldw;
    for (int w = threadIdx.x * 2; w < W; w += 512)
      __builtin_nontemporal_store(*(const u64x2*)&row[w], (u64x2*)&dst[w]);
  }
}

// K CUs off in every XCD (the engine's ensure_masked_stream mask)
static void make_mask(int K, uint32_t* mask) {
  const int t = K < 4 ? 1 : K / 4, beta = K < 4 ? K : 4;
  for (int w = 0; w < 8; ++w) {
    mask[w] = 0xffffffffu;
    for (int bit = 0; bit < 32; ++bit) {
      const int i = w * 32 + bit, a = i / 32, b = (i / 8) % 4, c = i % 8;
      if (((c - a) & 7) < t && b < beta) mask[w] &= ~(1u << bit);
    }
  }
}

int main() {
  const long n = 100000, ldw = 1568;
  const int W = 1563;
  const size_t bytes = sizeof(u64) * n * ldw;
  u64* M;
  int* perm;
  CK(hipMalloc(&M, bytes));
  CK(hipMalloc(&perm, sizeof(int) * n));
  std::vector<int> hp(n);
  for (long i = 0; i < n; ++i) hp[i] = (int)i;
  std::mt19937 rng(1);
  std::shuffle(hp.begin(), hp.end(), rng);
  CK(hipMemcpy(perm, hp.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double algo = 8.0 * n * W;
  for (int off : {0, 8, 12, 16, 20, 24, 28}) {
    uint32_t mask[8];
    make_mask(off, mask);
    hipStream_t s;
    if (off == 0) CK(hipStreamCreate(&s));
    else CK(hipExtStreamCreateWithCUMask(&s, 8, mask));
    const int cus = 256 - 8 * off;
    for (int kind = 0; kind < 2; ++kind) {
      std::vector<float> ts;
      for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0, s));
        if (kind == 0)
          hipLaunchKernelGGL(k_flat, dim3(8 * cus), dim3(256), 0, s, M, (long)(bytes / 16));
        else
          hipLaunchKernelGGL(k_rows16, dim3((unsigned)((n + 15) / 16)), dim3(256),
                             sizeof(u64) * ldw, s, M, perm, n, ldw, W);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double ms = ts[ts.size() / 2];
      const double b = kind == 0 ? (double)bytes : algo;
      printf("{\"cus\": %d, \"shape\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"GBps_per_cu\": %.1f}\n",
             cus, kind == 0 ? "flat" : "rows16", ms, b / ms / 1e9, b / ms / 1e6 / cus);
      fflush(stdout);
    }
    CK(hipStreamDestroy(s));
  }
  CK(hipFree(M));
  CK(hipFree(perm));
  return 0;
}
