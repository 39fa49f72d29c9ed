// Does a triple-chevron launch through a kernel function-pointer parameter
// dispatch?  (Round 3: under the host sanitizers such launches of the engine
// "launched nothing".)  Built several ways by scripts/micro/indirect_launch.sh;
// prints, per launch form, whether the kernel wrote its word and what
// hipGetLastError said, plus the addresses involved.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstring>

struct Big {            // a ScanJobsN-sized by-value argument
  unsigned long long w[100];
  int v;
};

__global__ void k_set(int* p, int v) { p[threadIdx.x] = v; }
__global__ void k_set_big(int* p, Big b) { p[threadIdx.x] = b.v + (int)b.w[99]; }

template <int N>
__global__ void k_tset(int* p, Big b) { p[threadIdx.x] = b.v + N; }

// the engine's round-3 launch helper as it was (commit 2a907f0): the handle
// form with an event, the triple-chevron form without
template <typename... KArgs, typename... Args>
__attribute__((noinline)) void launch_marked_r3(void (*kernel)(KArgs...), dim3 grid, dim3 block,
                                                size_t lds, hipStream_t st, hipEvent_t ev,
                                                Args... args) {
  if (ev) hipExtLaunchKernelGGL(kernel, grid, block, lds, st, nullptr, ev, 0, args...);
  else hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
}

template <typename... KArgs, typename... Args>
__attribute__((noinline)) void via_ptr(void (*kernel)(KArgs...), hipStream_t st, Args... args) {
  hipLaunchKernelGGL(kernel, dim3(1), dim3(64), 0, st, args...);
}
template <typename... KArgs, typename... Args>
__attribute__((noinline)) void via_handle(void (*kernel)(KArgs...), hipStream_t st, Args... args) {
  hipExtLaunchKernelGGL(kernel, dim3(1), dim3(64), 0u, st, nullptr, nullptr, 0, args...);
}

int check(const char* what, int* d, int want, hipStream_t st) {
  int h[64];
  hipError_t le = hipGetLastError();
  hipError_t se = hipStreamSynchronize(st);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int ok = 1;
  for (int i = 0; i < 64; ++i) ok &= h[i] == want;
  std::printf("%-34s wrote=%d lastError=%s sync=%s\n", what, ok, hipGetErrorString(le),
              hipGetErrorString(se));
  (void)hipMemset(d, 0, sizeof(h));
  return ok;
}

int main() {
  int* d = nullptr;
  hipStream_t st;
  if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipMemset(d, 0, 64 * sizeof(int));
  void (*fp)(int*, int) = k_set;
  std::printf("handle k_set=%p (as seen here), fp=%p, *(void**)fp=%p\n", (void*)k_set, (void*)fp,
              *reinterpret_cast<void* const*>(reinterpret_cast<const void*>(fp)));
  int bad = 0;
  hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, st, d, 7);
  bad += !check("direct <<<>>>", d, 7, st);
  via_ptr(k_set, st, d, 8);
  bad += !check("function pointer <<<>>>", d, 8, st);
  via_handle(k_set, st, d, 9);
  bad += !check("function pointer, by handle", d, 9, st);
  Big b;
  std::memset(&b, 0, sizeof(b));
  b.v = 10;
  b.w[99] = 1;
  via_ptr(k_set_big, st, d, b);
  bad += !check("function pointer <<<>>>, 808-B arg", d, 11, st);
  via_handle(k_set_big, st, d, b);
  bad += !check("by handle, 808-B arg", d, 11, st);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  b.v = 20;
  launch_marked_r3(k_tset<2>, dim3(1), dim3(64), 0, st, (hipEvent_t) nullptr, d, b);
  bad += !check("r3 helper, template, no event", d, 22, st);
  launch_marked_r3(k_tset<3>, dim3(1), dim3(64), 0, st, ev, d, b);
  bad += !check("r3 helper, template, event", d, 23, st);
  launch_marked_r3(k_tset<4>, dim3(2), dim3(64), 0, st, (hipEvent_t) nullptr, d, b);
  bad += !check("r3 helper, template, no event, 2 blk", d, 24, st);
  std::printf("%s\n", bad ? "SOME LAUNCHES DID NOTHING" : "all launches dispatched");
  return bad ? 1 : 0;
}
