// Host and GPU cost of a 20-kernel chain: direct launches vs one captured
// hipGraph (with a fork/join over a second stream and an event record in
// the middle that the host waits on).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
struct Args { int* p; long n; char pad[256]; };
__global__ void k_step(Args a, int v) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.p[i] += v;
}
int main() {
  const long n = 100000;
  int* d;
  hipMalloc(&d, sizeof(int) * n);
  hipMemset(d, 0, sizeof(int) * n);
  hipStream_t s, s2;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1, mid, fork, join;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventCreateWithFlags(&mid, hipEventDisableTiming);
  hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  hipEventCreateWithFlags(&join, hipEventDisableTiming);
  Args a{d, n, {}};
  auto chain = [&](bool with_fork) {
    for (int k = 0; k < 20; ++k) {
      hipLaunchKernelGGL(k_step, dim3((n + 255) / 256), dim3(256), 0, s, a, k);
      if (k == 9) hipEventRecord(mid, s);
      if (with_fork && k == 5) {
        hipEventRecord(fork, s);
        hipStreamWaitEvent(s2, fork, 0);
        hipLaunchKernelGGL(k_step, dim3((n + 255) / 256), dim3(256), 0, s2, a, 100);
        hipEventRecord(join, s2);
      }
      if (with_fork && k == 12) hipStreamWaitEvent(s, join, 0);
    }
  };
  for (int rep = 0; rep < 3; ++rep) {
    // direct
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    const int N = 200;
    hipEventRecord(e0, s);
    for (int i = 0; i < N; ++i) chain(true);
    auto t1 = std::chrono::steady_clock::now();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    auto t2 = std::chrono::steady_clock::now();
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("direct: host %.1f us/chain, total %.1f us/chain, gpu %.1f us/chain\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / N, ms * 1e3 / N);
    // graph
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
    chain(true);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipDeviceSynchronize();
    t0 = std::chrono::steady_clock::now();
    hipEventRecord(e0, s);
    for (int i = 0; i < N; ++i) hipGraphLaunch(ge, s);
    t1 = std::chrono::steady_clock::now();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    t2 = std::chrono::steady_clock::now();
    hipEventElapsedTime(&ms, e0, e1);
    printf("graph:  host %.1f us/chain, total %.1f us/chain, gpu %.1f us/chain\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / N, ms * 1e3 / N);
    // host waits on the mid event recorded inside the graph
    hipDeviceSynchronize();
    t0 = std::chrono::steady_clock::now();
    hipGraphLaunch(ge, s);
    hipError_t em = hipEventSynchronize(mid);
    t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    t2 = std::chrono::steady_clock::now();
    printf("graph mid-event wait: %s, %.1f us vs full %.1f us\n", hipGetErrorString(em),
           std::chrono::duration<double, std::micro>(t1 - t0).count(),
           std::chrono::duration<double, std::micro>(t2 - t0).count());
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }
  int h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("check %d\n", h);
  return 0;
}
