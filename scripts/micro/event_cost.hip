// GPU-side cost of stream markers between dependent kernels (round 3): a
// chain of 40 short kernels (782 blocks, one 8-B load + store per thread) on
// one stream, with nothing between them, with a hipEventRecord (timing
// disabled) after each, with a hipStreamWaitEvent on an already complete
// event before each, with a record after each that a second stream waits on,
// and with hipStreamWriteValue32 after each.  Median of 15 chains, device
// time between two timing events around the chain.
// Build: hipcc --offload-arch=gfx950 -O3 -o event_cost event_cost.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_step(unsigned long long* a, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] = a[i] * 3 + 1;
}

int main() {
  const int n = 782 * 256, L = 40;
  unsigned long long* a;
  unsigned* flag;
  hipMalloc(&a, 8 * n);
  hipMalloc(&flag, 64);
  hipMemset(a, 0, 8 * n);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t t0, t1, mk, done;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventCreateWithFlags(&mk, hipEventDisableTiming);
  hipEventCreateWithFlags(&done, hipEventDisableTiming);
  hipEventRecord(done, s1);
  hipStreamSynchronize(s1);
  hipEvent_t mkt;
  hipEventCreate(&mkt);
  const char* names[] = {"plain chain", "record after each", "wait (complete) before each",
                         "record after each, stream2 waits", "writeValue32 after each",
                         "ext launch stop event (no timing)", "ext launch stop event, s2 waits",
                         "ext launch stop event (timing), s2 waits"};
  for (int pass = 0; pass < 2; ++pass) {
    for (int mode = 0; mode < 8; ++mode) {
      std::vector<float> ts;
      for (int rep = 0; rep < 15; ++rep) {
        hipEventRecord(t0, s1);
        for (int k = 0; k < L; ++k) {
          if (mode == 2) hipStreamWaitEvent(s1, done, 0);
          if (mode >= 5)
            hipExtLaunchKernelGGL(k_step, dim3(782), dim3(256), 0, s1, nullptr,
                                  mode == 7 ? mkt : mk, 0, a, n);
          else
            hipLaunchKernelGGL(k_step, dim3(782), dim3(256), 0, s1, a, n);
          if (mode == 6) hipStreamWaitEvent(s2, mk, 0);
          if (mode == 7) hipStreamWaitEvent(s2, mkt, 0);
          if (mode == 1 || mode == 3) hipEventRecord(mk, s1);
          if (mode == 3) hipStreamWaitEvent(s2, mk, 0);
          if (mode == 4) hipStreamWriteValue32(s1, flag, (unsigned)k, 0);
        }
        hipEventRecord(t1, s1);
        hipEventSynchronize(t1);
        hipStreamSynchronize(s2);
        float ms;
        hipEventElapsedTime(&ms, t0, t1);
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      printf("%-36s %.2f us per kernel (median chain %.1f us)\n", names[mode], ts[7] * 1e3 / L,
             ts[7] * 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
