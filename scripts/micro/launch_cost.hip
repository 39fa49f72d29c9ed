// Host cost of a kernel launch on this runtime: empty kernels with small and
// large (ScanJobs-sized) argument structs, back to back on one stream.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
struct Small { void* p[4]; long n; };
struct Big { char b[768]; };
__global__ void k_small(Small s) { if (s.n == -7) ((int*)s.p[0])[0] = 1; }
__global__ void k_big(Big s) { if (s.b[5] == 99) ((int*)0)[0] = 1; }
int main() {
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  Small a{}; Big b{};
  for (int rep = 0; rep < 2; ++rep) {
    for (int kind = 0; kind < 2; ++kind) {
      const int N = 20000;
      hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) {
        if (kind == 0) hipLaunchKernelGGL(k_small, dim3(782), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(k_big, dim3(782), dim3(256), 0, st, b);
      }
      auto t1 = std::chrono::steady_clock::now();
      hipStreamSynchronize(st);
      auto t2 = std::chrono::steady_clock::now();
      printf("%s args: host %.2f us/launch, total %.2f us/kernel\n", kind ? "768B" : "40B",
             std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
             std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
    }
  }
  // event record / query costs
  hipEvent_t ev; hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 20000; ++i) hipEventRecord(ev, st);
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(st);
  printf("hipEventRecord: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 20000);
  return 0;
}
