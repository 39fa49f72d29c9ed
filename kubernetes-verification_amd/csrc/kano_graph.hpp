// kano_graph.hpp -- replay of kano_verify's launch sequences as hipGraphs.
//
// A kano_verify step issues ~40 small launches and three host syncs; the
// host needs 5-7 us per launch (hipLaunchKernel alone 3.3 us, median on the
// MI355X boxes) while many of the kernels take 4-10 us, so the GPU waits for
// the host after every sync and, on row shards (1/8 of the rows), almost
// throughout.  Here every HIP operation of kano_verify is RECORDED instead of
// issued (kernel, grid, block, LDS bytes, stream and the argument bytes;
// memsets, device copies, event records and waits) and a segment -- the
// operations between two host waits -- is issued at its end:
//   * as a cached hipGraphExec when an identical sequence (same kernels,
//     same launch shapes, same argument bytes: pointers and sizes included)
//     was captured before;
//   * captured into a new graph when the previous step issued the same
//     sequence (so every buffer already has its final size);
//   * otherwise directly, operation by operation.
// The host code still runs every step (it is what decides the sequence);
// only the HIP calls are batched.  Anything that must reach the device
// early -- a host wait, a free -- flushes the pending operations first, so
// a recorded sequence is always issued before the host depends on it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace kano_rec {

enum OpKind { OP_LAUNCH, OP_MEMSET, OP_MEMCPY, OP_MEMCPY2D, OP_EVENT, OP_WAIT };

struct Op {
  OpKind kind;
  const void* fn = nullptr;
  dim3 g{}, b{};
  size_t shm = 0;
  hipStream_t st = nullptr;
  size_t arg0 = 0, narg = 0;      // into Recorder::offs
  void* dst = nullptr;
  const void* src = nullptr;
  size_t bytes = 0, dpitch = 0, spitch = 0, width = 0, height = 0;
  int val = 0;
  hipMemcpyKind mk = hipMemcpyDefault;
  hipEvent_t ev = nullptr;
  unsigned flags = 0;
};

struct Recorder {
  std::vector<Op> ops;
  std::vector<unsigned char> arena;
  std::vector<size_t> offs;
  uint64_t hash = 1469598103934665603ull;
  bool capturable = true;          // host-memory copies are issued directly
  void clear() {
    ops.clear();
    arena.clear();
    offs.clear();
    hash = 1469598103934665603ull;
    capturable = true;
  }
  void mix(const void* p, size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      std::memcpy(&w, c + i, 8);
      hash = (hash ^ w) * 0x100000001b3ull;
      hash ^= hash >> 29;
    }
    for (; i < n; ++i) hash = (hash ^ c[i]) * 1099511628211ull;
  }
  template <typename T>
  void mixv(const T& v) {
    mix(&v, sizeof(T));
  }
  size_t put(const void* p, size_t n) {
    size_t at = (arena.size() + 15) & ~size_t(15);
    arena.resize(at + n);
    std::memcpy(arena.data() + at, p, n);
    mix(p, n);
    return at;
  }
};

// the recorder of the segment being recorded on this thread (null: issue now)
inline thread_local Recorder* g_rec = nullptr;
// device-writing operations issued on this thread (launches, memsets,
// copies): lets a context tell that nothing ran since it last did
inline thread_local uint64_t g_ops = 0;

template <typename Tup, size_t... I>
inline hipError_t launch_tuple(const void* f, dim3 g, dim3 b, size_t shm, hipStream_t st, Tup& t,
                               std::index_sequence<I...>) {
  void* args[] = {static_cast<void*>(&std::get<I>(t))...};
  return hipLaunchKernel(f, g, b, args, shm, st);
}

template <typename Tup, size_t... I>
inline void record_tuple(Recorder& r, Op& op, Tup& t, std::index_sequence<I...>) {
  op.arg0 = r.offs.size();
  op.narg = sizeof...(I);
  (r.offs.push_back(r.put(&std::get<I>(t), sizeof(std::get<I>(t)))), ...);
}

// hipLaunchKernelGGL, recorded or issued (the arguments converted to the
// kernel's parameter types, as the triple-chevron launch would)
template <typename... P, typename... A>
inline void launch(void (*f)(P...), dim3 g, dim3 b, size_t shm, hipStream_t st, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  std::tuple<std::decay_t<P>...> t(static_cast<std::decay_t<P>>(std::forward<A>(a))...);
  ++g_ops;
  if (!g_rec) {
    (void)launch_tuple(reinterpret_cast<const void*>(f), g, b, shm, st, t,
                       std::index_sequence_for<P...>{});
    return;
  }
  Recorder& r = *g_rec;
  Op op;
  op.kind = OP_LAUNCH;
  op.fn = reinterpret_cast<const void*>(f);
  op.g = g;
  op.b = b;
  op.shm = shm;
  op.st = st;
  r.mixv(op.kind);
  r.mixv(op.fn);
  r.mixv(g.x); r.mixv(g.y); r.mixv(g.z);
  r.mixv(b.x); r.mixv(b.y); r.mixv(b.z);
  r.mixv(shm);
  r.mixv(st);
  record_tuple(r, op, t, std::index_sequence_for<P...>{});
  r.ops.push_back(op);
}

inline hipError_t memsetAsync(void* p, int v, size_t n, hipStream_t st) {
  ++g_ops;
  if (!g_rec) return ::hipMemsetAsync(p, v, n, st);
  Op op;
  op.kind = OP_MEMSET;
  op.dst = p;
  op.val = v;
  op.bytes = n;
  op.st = st;
  g_rec->mixv(op.kind); g_rec->mixv(p); g_rec->mixv(v); g_rec->mixv(n); g_rec->mixv(st);
  g_rec->ops.push_back(op);
  return hipSuccess;
}

inline hipError_t memcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t st) {
  ++g_ops;
  if (!g_rec) return ::hipMemcpyAsync(d, s, n, k, st);
  Op op;
  op.kind = OP_MEMCPY;
  op.dst = d;
  op.src = s;
  op.bytes = n;
  op.mk = k;
  op.st = st;
  if (k != hipMemcpyDeviceToDevice) g_rec->capturable = false;
  g_rec->mixv(op.kind); g_rec->mixv(d); g_rec->mixv(s); g_rec->mixv(n); g_rec->mixv(k);
  g_rec->mixv(st);
  g_rec->ops.push_back(op);
  return hipSuccess;
}

inline hipError_t memcpy2DAsync(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h,
                                hipMemcpyKind k, hipStream_t st) {
  ++g_ops;
  if (!g_rec) return ::hipMemcpy2DAsync(d, dp, s, sp, w, h, k, st);
  Op op;
  op.kind = OP_MEMCPY2D;
  op.dst = d;
  op.dpitch = dp;
  op.src = s;
  op.spitch = sp;
  op.width = w;
  op.height = h;
  op.mk = k;
  op.st = st;
  if (k != hipMemcpyDeviceToDevice) g_rec->capturable = false;
  g_rec->mixv(op.kind); g_rec->mixv(d); g_rec->mixv(dp); g_rec->mixv(s); g_rec->mixv(sp);
  g_rec->mixv(w); g_rec->mixv(h); g_rec->mixv(k); g_rec->mixv(st);
  g_rec->ops.push_back(op);
  return hipSuccess;
}

inline hipError_t eventRecord(hipEvent_t e, hipStream_t st) {
  if (!g_rec) return ::hipEventRecord(e, st);
  Op op;
  op.kind = OP_EVENT;
  op.ev = e;
  op.st = st;
  g_rec->mixv(op.kind); g_rec->mixv(e); g_rec->mixv(st);
  g_rec->ops.push_back(op);
  return hipSuccess;
}

inline hipError_t streamWaitEvent(hipStream_t st, hipEvent_t e, unsigned flags) {
  if (!g_rec) return ::hipStreamWaitEvent(st, e, flags);
  Op op;
  op.kind = OP_WAIT;
  op.ev = e;
  op.st = st;
  op.flags = flags;
  g_rec->mixv(op.kind); g_rec->mixv(e); g_rec->mixv(st); g_rec->mixv(flags);
  g_rec->ops.push_back(op);
  return hipSuccess;
}

// the recorded operations, in order, directly
inline hipError_t issue(const Recorder& r, size_t from = 0) {
  std::vector<void*> args;
  for (size_t i = from; i < r.ops.size(); ++i) {
    const Op& op = r.ops[i];
    hipError_t e = hipSuccess;
    switch (op.kind) {
      case OP_LAUNCH:
        args.resize(op.narg);
        for (size_t a = 0; a < op.narg; ++a)
          args[a] = const_cast<unsigned char*>(r.arena.data()) + r.offs[op.arg0 + a];
        e = hipLaunchKernel(op.fn, op.g, op.b, args.data(), op.shm, op.st);
        break;
      case OP_MEMSET: e = ::hipMemsetAsync(op.dst, op.val, op.bytes, op.st); break;
      case OP_MEMCPY: e = ::hipMemcpyAsync(op.dst, op.src, op.bytes, op.mk, op.st); break;
      case OP_MEMCPY2D:
        e = ::hipMemcpy2DAsync(op.dst, op.dpitch, op.src, op.spitch, op.width, op.height, op.mk,
                               op.st);
        break;
      case OP_EVENT: e = ::hipEventRecord(op.ev, op.st); break;
      case OP_WAIT: e = ::hipStreamWaitEvent(op.st, op.ev, op.flags); break;
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace kano_rec

// every HIP operation of the engine goes through the recorder
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(K, G, B, S, ST, ...) \
  ::kano_rec::launch((K), dim3(G), dim3(B), (size_t)(S), (ST), ##__VA_ARGS__)
#define hipMemsetAsync ::kano_rec::memsetAsync
#define hipMemcpyAsync ::kano_rec::memcpyAsync
#define hipMemcpy2DAsync ::kano_rec::memcpy2DAsync
#define hipEventRecord ::kano_rec::eventRecord
#define hipStreamWaitEvent ::kano_rec::streamWaitEvent
