// kano_prims.hpp -- wave64 / block primitives and the device-wide scan used
// by the engine (kano_hip.hip).  gfx950: 64-lane waves, 256-thread blocks.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

namespace kano {

constexpr int TPB = 256;              // threads per block for every kernel
constexpr int SCAN_ITEMS = 8;         // elements per thread in a scan tile
constexpr int SCAN_TILE = TPB * SCAN_ITEMS;

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive scan over a 256-thread block; smem holds >= 4 elements.
// the same for a block of NW waves (smem: NW entries)
template <int NW, typename T>
__device__ __forceinline__ T block_excl_scan_nw(T v, T* smem, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) smem[wid] = inc;
  __syncthreads();
  T pre = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wid) pre += smem[w];
    total += smem[w];
  }
  __syncthreads();
  return pre + inc - v;
}

template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* smem, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = wave_incl_scan(v);
  if (lane == 63) smem[wid] = inc;
  __syncthreads();
  T pre = 0;
  for (int w = 0; w < wid; ++w) pre += smem[w];
  total = smem[0] + smem[1] + smem[2] + smem[3];
  __syncthreads();
  return pre + inc - v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

// exclusive scan over the 64 lanes of a wave; total = sum of all lanes
template <typename T>
__device__ __forceinline__ T wave_excl_scan(T v, T& total) {
  const T inc = wave_incl_scan(v);
  total = __shfl(inc, 63, 64);
  return inc - v;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* smem) {
  T tot;
  (void)block_excl_scan(v, smem, tot);
  return tot;
}

// ---- device-wide exclusive scan: out[0..n] with out[n] = total -----------
template <typename Tin, typename Tout>
__global__ __launch_bounds__(TPB) void k_scan_sums(const Tin* __restrict__ in, i64 n,
                                                   Tout* __restrict__ sums) {
  __shared__ Tout sm[4];
  const i64 base = (i64)blockIdx.x * SCAN_TILE + (i64)threadIdx.x * SCAN_ITEMS;
  Tout s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (base + k < n) s += (Tout)in[base + k];
  Tout tot = block_sum(s, sm);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(TPB) void k_scan_tiles(const Tin* __restrict__ in, i64 n,
                                                    const Tout* __restrict__ tile_off,
                                                    Tout* __restrict__ out) {
  __shared__ Tout sm[4];
  const i64 base = (i64)blockIdx.x * SCAN_TILE + (i64)threadIdx.x * SCAN_ITEMS;
  Tout v[SCAN_ITEMS];
  Tout s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    v[k] = (base + k < n) ? (Tout)in[base + k] : (Tout)0;
    s += v[k];
  }
  Tout tot;
  Tout pre = block_excl_scan(s, sm, tot) + (tile_off ? tile_off[blockIdx.x] : (Tout)0);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    if (base + k < n) out[base + k] = pre;
    pre += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == TPB - 1) out[n] = pre;
}

// ---- single-pass scan (decoupled look-back) --------------------------------
// status[0] is the tile ticket, status[1 + t] the published state of tile t:
// (flag << 62) | value, flag 1 = tile aggregate, 2 = inclusive prefix.  The
// caller alternates two status regions: each scan zeroes the other one for
// the next scan (stream order makes that safe), so no separate memset.
constexpr u64 LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1;

__device__ __forceinline__ u64 lb_load(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Up to MAX_SCAN_JOBS independent scans in one launch (blockIdx.y = job),
// int32 or int64 on either side, arithmetic in int64.  Job j's ticket and
// tile states live at status[st], status[st + 1 + t].
struct ScanJob {
  const void* in;
  void* out;
  u64* total;   // nullable: the total also lands here (a host-read size slot)
  u64* total_host;   // nullable: ... and here (the slot's pinned host mirror)
  i64 n;
  i64 st;
  int in64, out64;
  // generated input instead of `in`.  gen = 1: element x is 1 iff pod
  // m0 + x is the smallest member of its hash slot (a class representative),
  // smin[slot_of[m0 + x]] == m0 + x.  gen = 2: element x is the length of
  // pod m0 + x's class segment, loff[c + 1] - loff[c] with c = gslot[m0 + x]
  // (policy_shadow's pairs per pod: gslot = the row classes)
  int gen;
  int gpb;              // gen = 1 with pod-in-slot tables: the member is gtab[slot]'s low gpb bits
  const int32_t* gsmin;
  const u64* gtab;
  const int32_t* gslot;
  const i64* gloff;
  i64 gm0;
  // gen = 3: element x is gcnt[gslot[m0 + x]] (policy_shadow's pairs per pod
  // straight from the per-class counts T, before the lists are compacted)
  const i64* gcnt;
};
constexpr int MAX_SCAN_JOBS = 8;
constexpr int MAX_PUBLISH = 4;
// NJ job slots: the launch passes only the slots it uses (the kernel
// argument of an 8-slot batch is ~800 B, and a launch costs the host ~1.4 us
// more at 768 B than at 40 B: scripts/micro/launch_cost.hip)
template <int NJ>
struct ScanJobsN {
  ScanJob j[NJ];
  int count;
  // size slots produced by earlier kernels (atomics), copied by one thread
  // to their host mirrors: they travel with the scan's own totals
  int npub;
  const u64* pub_src[MAX_PUBLISH];
  u64* pub_dst[MAX_PUBLISH];
  // host signal (nullable): after the sig_n writers of host mirrors (one per
  // job with total_host, one for the publish list) have stored their values,
  // the last of them stores sig_val to *sig_host -- the host polls that word
  // instead of waiting on an event (an event record costs the stream ~6 us)
  u64* sig_host;
  u64 sig_val;
  uint32_t* sig_ctr;   // arrivals (zero between launches: the last arrival resets it)
  int sig_n;
};
using ScanJobs = ScanJobsN<MAX_SCAN_JOBS>;

// A host mirror word: a system-scope (write-through) store, so that once the
// store is acknowledged the host sees it -- no cache write-back needed.
__device__ __forceinline__ void mirror_store(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One writer of host mirrors is done.  Its mirror stores are acknowledged
// (s_waitcnt on every counter) before it counts itself, and the last writer
// raises the host signal after seeing every other count: the host, seeing
// the signal, sees every mirror word.  (A system-scope fence here wrote back
// the XCD's L2 per writer: ~5 us on the scan that carries the signal.)
template <class J>
__device__ __forceinline__ void scan_sig_arrive(const J& jobs) {
  if (!jobs.sig_host) return;
  __builtin_amdgcn_s_waitcnt(0);
  const uint32_t old =
      __hip_atomic_fetch_add(jobs.sig_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == (uint32_t)jobs.sig_n) {
    __hip_atomic_store(jobs.sig_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mirror_store(jobs.sig_host, jobs.sig_val);
  }
}

// IT: elements per thread (tile = 256 IT); short arrays take long tiles --
// fewer tiles, a shorter look-back chain (each hop a cross-XCD round trip)
template <int NJ, int IT = SCAN_ITEMS>
__global__ __launch_bounds__(TPB) void k_scan_lb(ScanJobsN<NJ> jobs, u64* status,
                                                 u64* __restrict__ clear, i64 nclear) {
  constexpr i64 TILE = (i64)TPB * IT;
  __shared__ i64 sm[4];
  __shared__ i64 s_tile;
  __shared__ i64 s_prefix;
  const i64 lin = (i64)blockIdx.y * gridDim.x + blockIdx.x;
  const i64 nthr = (i64)gridDim.x * gridDim.y * TPB;
  for (i64 i = lin * TPB + threadIdx.x; i < nclear; i += nthr) clear[i] = 0;
  if (lin == 0 && threadIdx.x == 0 && jobs.npub > 0) {
    for (int q = 0; q < jobs.npub; ++q) mirror_store(jobs.pub_dst[q], *jobs.pub_src[q]);
    scan_sig_arrive(jobs);
  }
  ScanJob jb = jobs.j[0];   // select, not a dynamic index (kernarg stays in SGPRs)
#pragma unroll
  for (int q = 1; q < NJ; ++q)
    if ((int)blockIdx.y == q) jb = jobs.j[q];
  const i64 tiles = (jb.n + TILE - 1) / TILE;
  if (jb.n == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (jb.out64) static_cast<i64*>(jb.out)[0] = 0;
      else static_cast<int32_t*>(jb.out)[0] = 0;
      if (jb.total) *jb.total = 0;
      if (jb.total_host) {
        mirror_store(jb.total_host, 0);
        scan_sig_arrive(jobs);
      }
    }
    return;
  }
  u64* st = status + jb.st;
  if (threadIdx.x == 0)
    s_tile = (i64)__hip_atomic_fetch_add(st, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const i64 tile = s_tile;
  if (tile >= tiles) return;
  const i64 base = tile * TILE + (i64)threadIdx.x * IT;
  i64 v[IT];
  i64 s = 0;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const i64 x = base + k;
    if (x >= jb.n) v[k] = 0;
    else if (jb.gen == 1) {
      const int32_t sl = jb.gslot[jb.gm0 + x];
      const int32_t r = jb.gpb ? (int32_t)(jb.gtab[sl] & ((1ull << jb.gpb) - 1ull)) : jb.gsmin[sl];
      v[k] = r == (int32_t)(jb.gm0 + x) ? 1 : 0;
    }
    else if (jb.gen == 2) {
      const int32_t c = jb.gslot[jb.gm0 + x];
      v[k] = jb.gloff[c + 1] - jb.gloff[c];
    }
    else if (jb.gen == 3) v[k] = jb.gcnt[jb.gslot[jb.gm0 + x]];
    else v[k] = jb.in64 ? static_cast<const i64*>(jb.in)[x]
                        : (i64) static_cast<const int32_t*>(jb.in)[x];
    s += v[k];
  }
  i64 tot;
  i64 pre = block_excl_scan(s, sm, tot);
  // look-back by wave 0: its 64 lanes read 64 predecessor states at once and
  // sum back to the nearest inclusive prefix, so a tile waits only for its
  // predecessors' aggregates, never for a chain of prefixes
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    u64* ts = st + 1;
    i64 excl = 0;
    if (tile == 0) {
      if (lane == 0) lb_store(&ts[0], LB_INC | ((u64)tot & LB_VAL));
    } else {
      if (lane == 0) lb_store(&ts[tile], LB_AGG | ((u64)tot & LB_VAL));
      for (i64 q0 = tile - 1;; q0 -= 64) {
        const i64 q = q0 - lane;
        u64 w = LB_INC;                  // before tile 0: an inclusive zero
        if (q >= 0) {
          do { w = lb_load(&ts[q]); } while (w == 0);
        }
        const u64 inc = __ballot((w & ~LB_VAL) == LB_INC);
        const int f = inc ? __ffsll((long long)inc) - 1 : 63;
        const i64 part = wave_sum(lane <= f ? (i64)(w & LB_VAL) : (i64)0);
        excl += part;
        if (inc) break;
      }
      if (lane == 0) lb_store(&ts[tile], LB_INC | ((u64)(excl + tot) & LB_VAL));
    }
    if (lane == 0) s_prefix = excl;
  }
  __syncthreads();
  pre += s_prefix;
  if (jb.out64) {
    i64* o = static_cast<i64*>(jb.out);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      if (base + k < jb.n) o[base + k] = pre;
      pre += v[k];
    }
    if (tile == tiles - 1 && threadIdx.x == TPB - 1) {
      o[jb.n] = pre;
      if (jb.total) *jb.total = (u64)pre;
      if (jb.total_host) {
        mirror_store(jb.total_host, (u64)pre);
        scan_sig_arrive(jobs);
      }
    }
  } else {
    int32_t* o = static_cast<int32_t*>(jb.out);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      if (base + k < jb.n) o[base + k] = (int32_t)pre;
      pre += v[k];
    }
    if (tile == tiles - 1 && threadIdx.x == TPB - 1) {
      o[jb.n] = (int32_t)pre;
      if (jb.total) *jb.total = (u64)pre;
      if (jb.total_host) {
        mirror_store(jb.total_host, (u64)pre);
        scan_sig_arrive(jobs);
      }
    }
  }
}

// Look-back for NJ scans that share their tiles: wave w publishes the
// aggregates of jobs w, w + 4, ... of this tile and sums each job's
// predecessors back to the nearest inclusive prefix (64 predecessors per
// round, as k_scan_lb).  st: job q's tile states at st[q * tiles + t];
// tot / excl: LDS, NJ entries each.  Every thread of the block calls it.
template <int NJ>
__device__ __forceinline__ void lookback_jobs(u64* st, i64 tiles, i64 tile, const i64* tot,
                                              i64* excl) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int jq = wid; jq < NJ; jq += TPB / 64) {
    u64* ts = st + (i64)jq * tiles;
    const i64 t = tot[jq];
    i64 ex = 0;
    if (tile == 0) {
      if (lane == 0) lb_store(&ts[0], LB_INC | ((u64)t & LB_VAL));
    } else {
      if (lane == 0) lb_store(&ts[tile], LB_AGG | ((u64)t & LB_VAL));
      for (i64 q0 = tile - 1;; q0 -= 64) {
        const i64 q = q0 - lane;
        u64 w = LB_INC;
        if (q >= 0) {
          do { w = lb_load(&ts[q]); } while (w == 0);
        }
        const u64 inc = __ballot((w & ~LB_VAL) == LB_INC);
        const int f = inc ? __ffsll((long long)inc) - 1 : 63;
        ex += wave_sum(lane <= f ? (i64)(w & LB_VAL) : (i64)0);
        if (inc) break;
      }
      if (lane == 0) lb_store(&ts[tile], LB_INC | ((u64)(ex + t) & LB_VAL));
    }
    if (lane == 0) excl[jq] = ex;
  }
  __syncthreads();
}

// True in exactly one block of the launch -- the last to get here.  Every
// other block's memory operations before its call have completed by then
// (each block waits for its own -- s_waitcnt -- before it counts itself), so
// the last block reads their atomics' results with atomic loads.  No
// agent-scope fence: on gfx950 it writes back and invalidates the whole L2
// (buffer_wbl2 / buffer_inv sc1), per block.
__device__ __forceinline__ bool last_block_done(u64* done_ctr, i64 nblocks) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const u64 old =
        __hip_atomic_fetch_add(done_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old + 1 == (u64)nblocks;
  }
  __syncthreads();
  return s_last != 0;
}

// job q's total after every tile has looked back: the last tile's inclusive
// state (st as lookback_jobs)
__device__ __forceinline__ i64 lookback_total(u64* st, i64 tiles, int q) {
  u64 w;
  do { w = lb_load(&st[(i64)q * tiles + tiles - 1]); } while ((w & ~LB_VAL) != LB_INC);
  return (i64)(w & LB_VAL);
}

// several fills in one launch: (ptr, count of 32-bit words, value)
struct FillJob {
  uint32_t* ptr;
  i64 words;
  uint32_t value;
};
constexpr int MAX_FILLS = 24;
struct FillJobs {
  FillJob j[MAX_FILLS];
  int count;
};
// the fills on blocks [0, nvb) of whatever launch carries them (vb = the
// block's index among them): k_fill_many, or extra blocks of a kernel that
// runs independently of the fills (k_cls_vals, k_sel_place)
__device__ __forceinline__ void fill_item(const FillJobs& jobs, i64 vb, i64 nvb) {
  const i64 stride = nvb * TPB;
  for (int q = 0; q < jobs.count; ++q) {
    uint32_t* p = jobs.j[q].ptr;
    const uint32_t v = jobs.j[q].value;
    const i64 nw = jobs.j[q].words;
    for (i64 i = vb * TPB + threadIdx.x; i < nw; i += stride) p[i] = v;
  }
}
static __global__ __attribute__((unused)) __launch_bounds__(TPB) void k_fill_many(FillJobs jobs) {
  fill_item(jobs, blockIdx.x, gridDim.x);
}
constexpr int FILL_RIDE_BLOCKS = 512;   // blocks a carried fill gets (grid-stride)

// The gate in front of a primed prologue (kano_set_pipeline): one lane polls
// the bell -- a word in page-locked, coherent host memory that the next
// kano_verify stores -- with system-scope loads, sleeping between polls,
// until it reaches `want`; past `ticks` of the wall clock it opens by itself,
// so the engine stream never stays closed (the prologue reads only resident
// inputs, so it is valid whenever it runs).  One wave, no other work.
// (waited: the ticks the gate held the engine stream, into slot want % 64 of
// a device ring -- the engine stream's idle time at the step boundary,
// measured without a profiler: kano_gate_timing)
constexpr int GATE_RING = 64;
static __global__ __attribute__((unused)) __launch_bounds__(64) void k_gate(const u64* bell,
                                                                            u64 want, u64 ticks,
                                                                            u64* waited) {
  if (threadIdx.x != 0) return;
  const u64 t0 = wall_clock64();
  while (__hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if (wall_clock64() - t0 > ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (waited) waited[want % GATE_RING] = wall_clock64() - t0;
}

// atomicAdd(&ctr[key], 1) for every active lane, lanes with equal keys merged
// into one atomic: up to AGG_ROUNDS rounds each take the first remaining
// lane's key and every lane sharing it (Zipf keys: the hot keys repeat
// inside a wave); the rest add one by one.  Returns the lane's slot (old
// value + rank).  Every lane of the wave must call it.
constexpr int AGG_ROUNDS = 4;
__device__ __forceinline__ int32_t wave_agg_inc(int32_t* ctr, i64 key, bool active) {
  const int lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1ull;
  u64 rem = __ballot(active);
  bool done = !active;
  int32_t res = 0;
  for (int round = 0; round < AGG_ROUNDS && rem; ++round) {
    const int leader = __ffsll((long long)rem) - 1;
    const i64 k0 = __shfl(key, leader, 64);
    const bool same = !done && key == k0;
    const u64 smask = __ballot(same);
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(&ctr[k0], (int32_t)__popcll(smask));
    base = __shfl(base, leader, 64);
    if (same) {
      res = base + (int32_t)__popcll(smask & below);
      done = true;
    }
    rem &= ~smask;
  }
  if (!done) res = atomicAdd(&ctr[key], 1);
  return res;
}

// atomicMin(&lo[key], v), atomicMax(&hi[key], v) with the same merging
__device__ __forceinline__ void wave_agg_minmax(int32_t* lo, int32_t* hi, i64 key, int32_t v,
                                                bool active) {
  const int lane = threadIdx.x & 63;
  u64 rem = __ballot(active);
  bool done = !active;
  for (int round = 0; round < AGG_ROUNDS && rem; ++round) {
    const int leader = __ffsll((long long)rem) - 1;
    const i64 k0 = __shfl(key, leader, 64);
    const bool same = !done && key == k0;
    const u64 smask = __ballot(same);
    int32_t mn = same ? v : INT32_MAX, mx = same ? v : INT32_MIN;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      mn = min(mn, __shfl_xor(mn, d, 64));
      mx = max(mx, __shfl_xor(mx, d, 64));
    }
    if (lane == leader) {
      atomicMin(&lo[k0], mn);
      atomicMax(&hi[k0], mx);
    }
    if (same) done = true;
    rem &= ~smask;
  }
  if (!done) {
    atomicMin(&lo[key], v);
    atomicMax(&hi[key], v);
  }
}

// atomicMin(&lo[key], v), atomicMax(&hi[key], v) for keys that come in
// contiguous runs along the lanes (a class-grouped member list): a segmented
// min / max over the wave, one atomic pair per run.  Every lane must call it.
__device__ __forceinline__ void wave_seg_minmax(int32_t* lo, int32_t* hi, i64 key, int32_t v,
                                                bool active) {
  const int lane = threadIdx.x & 63;
  int32_t mn = active ? v : INT32_MAX, mx = active ? v : INT32_MIN;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const i64 ko = __shfl_up(key, d, 64);
    const int32_t a = __shfl_up(mn, d, 64), b = __shfl_up(mx, d, 64);
    if (lane >= d && ko == key) {
      mn = min(mn, a);
      mx = max(mx, b);
    }
  }
  const i64 kn = __shfl_down(key, 1, 64);
  const bool last = lane == 63 || kn != key;
  if (last && mn <= mx) {
    atomicMin(&lo[key], mn);
    atomicMax(&hi[key], mx);
  }
}

// ---- small helpers ---------------------------------------------------------
__device__ __forceinline__ i64 upper_bound_i32(const int32_t* a, i64 n, i64 key) {
  i64 lo = 0, hi = n;
  while (lo < hi) {
    const i64 mid = (lo + hi) >> 1;
    if ((i64)a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// *p |= v with the atomic skipped when every bit of v is already set.  Bits
// only ever get set, so a stale read can only show fewer of them (one atomic
// too many), never more: the skip is safe without coherence.  Saturating OR
// targets (column words hit by every block) then take one atomic per new bit
// group instead of one per block.  (Measured on k_mc_fold's column words:
// the read before the atomic cost more than the atomics it saved.)
__device__ __forceinline__ void or_if_new(u64* p, u64 v) {
  if (v & ~*p) atomicOr(p, v);
}

// bits of word w that lie below n
__device__ __forceinline__ u64 valid_mask(i64 w, i64 n) {
  const i64 lo = w * 64;
  if (lo + 64 <= n) return ~0ull;
  if (lo >= n) return 0ull;
  return (1ull << (n - lo)) - 1ull;
}

__device__ __forceinline__ uint32_t hmix(uint32_t h, uint32_t v) {
  v *= 0xcc9e2d51u;
  v = (v << 15) | (v >> 17);
  v *= 0x1b873593u;
  h ^= v;
  h = (h << 13) | (h >> 19);
  return h * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t hfin(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

// Device -> host result copy as a kernel writing the caller's page-locked
// host buffer directly (16 bytes per lane, a grid-stride loop): the
// runtime's copy of a D2H range into the same buffer occasionally stalled the
// host ~7 ms inside hipMemcpyAsync (kano_verify's tail, MI355X).
static __global__ __attribute__((unused)) __launch_bounds__(TPB) void k_copy_out(const uint4* __restrict__ src, uint4* dst,
                                                 i64 n16, const uint32_t* __restrict__ src_tail,
                                                 uint32_t* dst_tail, int ntail) {
  const i64 stride = (i64)gridDim.x * TPB;
  for (i64 k = (i64)blockIdx.x * TPB + threadIdx.x; k < n16; k += stride) dst[k] = src[k];
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

// The same copy sized on the device: up to two jobs (blockIdx.y), each of
// sum(cnt[0..ncnt)) elements of esize bytes (a scan total, no host round
// trip); a job past its capacity copies nothing (the host sees the count and
// takes the sized path).
struct CopyJob {
  const char* src;
  char* dst;
  const u64* cnt;
  int ncnt;
  int esize;
  i64 cap;
};
struct CopyJobs {
  CopyJob j[2];
};
static __global__ __attribute__((unused)) __launch_bounds__(TPB) void k_copy_out_dev(CopyJobs jobs) {
  const CopyJob a = jobs.j[blockIdx.y];
  i64 cnt = 0;
  for (int q = 0; q < a.ncnt; ++q) cnt += (i64)a.cnt[q];
  if (cnt > a.cap) return;                          // block-uniform
  const i64 bytes = cnt * a.esize, n16 = bytes >> 4;
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.src);
  uint4* dst = reinterpret_cast<uint4*>(a.dst);
  const i64 stride = (i64)gridDim.x * TPB;
  for (i64 k = (i64)blockIdx.x * TPB + threadIdx.x; k < n16; k += stride) dst[k] = src[k];
  const int ntail = (int)((bytes & 15) >> 2);
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail)
    reinterpret_cast<uint32_t*>(a.dst + n16 * 16)[threadIdx.x] =
        reinterpret_cast<const uint32_t*>(a.src + n16 * 16)[threadIdx.x];
}

}  // namespace kano
