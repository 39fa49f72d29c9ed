// Store patterns for the matrix write at C3 shape (100,000 rows x 1,568
// words = 1.25 GB): flat streams and 32-row tiles written word column by
// word column with 8 / 16 / 32 bytes per lane, plain and non-temporal.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef long i64;

template <bool NT>
__device__ __forceinline__ void st2(u64* p, u64x2 v) {
  if (NT) __builtin_nontemporal_store(v, (u64x2*)p);
  else *(u64x2*)p = v;
}
template <bool NT>
__device__ __forceinline__ void st1(u64* p, u64 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// flat: grid-stride 16 B per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_flat(u64* M, i64 nw) {
  const u64x2 v = {1ull, 2ull};
  for (i64 w = ((i64)blockIdx.x * 256 + threadIdx.x) * 2; w < nw; w += (i64)gridDim.x * 512) st2<NT>(M + w, v);
}
// tile of 32 rows per block; lane covers LW words (8 B * LW) of one word column group
template <int NT_, int LW, bool NT>
__global__ __launch_bounds__(NT_) void k_tile(u64* M, i64 rows, i64 ldM) {
  const i64 t0 = (i64)blockIdx.x * 32;
  u64* out = M + t0 * ldM;
  const int nr = (int)min((i64)32, rows - t0);
  for (i64 w = (i64)threadIdx.x * LW; w < ldM; w += (i64)NT_ * LW) {
#pragma unroll
    for (int r = 0; r < 32; ++r) {
      if (r >= nr) break;
      u64* p = out + (i64)r * ldM + w;
      if (LW == 1) st1<NT>(p, (u64)w ^ r);
      else {
#pragma unroll
        for (int q = 0; q < LW; q += 2) st2<NT>(p + q, u64x2{(u64)w, (u64)r});
      }
    }
  }
}
// tile of 32 rows per block, row-major inside the tile: each wave streams
// whole rows (16 B per lane)
template <int NT_, bool NT>
__global__ __launch_bounds__(NT_) void k_tile_rows(u64* M, i64 rows, i64 ldM) {
  const i64 t0 = (i64)blockIdx.x * 32;
  const int nr = (int)min((i64)32, rows - t0);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int r = wv; r < nr; r += NT_ / 64) {
    u64* p = M + (t0 + r) * ldM;
    for (i64 w = lane * 2; w < ldM; w += 128) st2<NT>(p + w, u64x2{(u64)w, (u64)r});
  }
}

// one-shot: each thread writes U consecutive-across-block 16-B pieces
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_oneshot(u64* M, i64 nw) {
  const i64 base = (i64)blockIdx.x * 256 * 2 * U;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const i64 w = base + ((i64)u * 256 + threadIdx.x) * 2;
    if (w < nw) st2<NT>(M + w, u64x2{(u64)w, 1ull});
  }
}
// chunked: block b writes words [b*CW, (b+1)*CW) sequentially, 16 B per lane
template <int NT_, bool NT>
__global__ __launch_bounds__(NT_) void k_chunk(u64* M, i64 nw, i64 cw) {
  const i64 c0 = (i64)blockIdx.x * cw, c1 = min(nw, c0 + cw);
  for (i64 w = c0 + threadIdx.x * 2; w < c1; w += NT_ * 2) st2<NT>(M + w, u64x2{(u64)w, 1ull});
}

// tile-chunk blocks: block (t, k) writes rows [32t, 32t+32) x words
// [k*cw, (k+1)*cw), 16 B per lane (word pairs), row after row; blocks in
// address order (k fastest)
template <int NT_, int RT>
__global__ __launch_bounds__(NT_) void k_tchunk(u64* M, i64 rows, i64 ldM, i64 cw, int K) {
  const i64 t = blockIdx.x / K, k = blockIdx.x % K;
  const i64 w0 = k * cw, w1 = min(ldM, w0 + cw);
  const i64 npair = (w1 - w0) / 2;
  for (i64 e = threadIdx.x; e < RT * npair; e += NT_) {
    const i64 r = e / npair, q = e - r * npair;
    const i64 row = t * RT + r;
    if (row < rows) *(u64x2*)(M + row * ldM + w0 + 2 * q) = u64x2{(u64)row, (u64)q};
  }
}

int main() {
  const i64 rows = 100000, ldM = 1568, nw = rows * ldM;
  u64* M;
  hipMalloc(&M, nw * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)nw * 8;
  auto run = [&](const char* name, auto fn) {
    for (int i = 0; i < 2; ++i) fn();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-40s %.4f ms  %.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  const unsigned tiles = (unsigned)((rows + 31) / 32);
  run("flat 16B nt", [&] { hipLaunchKernelGGL(k_flat<true>, dim3(4096), dim3(256), 0, 0, M, nw); });
  run("flat 16B plain", [&] { hipLaunchKernelGGL(k_flat<false>, dim3(4096), dim3(256), 0, 0, M, nw); });
  run("tile 8B/lane nt 512t", [&] { hipLaunchKernelGGL((k_tile<512, 1, true>), dim3(tiles), dim3(512), 0, 0, M, rows, ldM); });
  run("tile 8B/lane plain 512t", [&] { hipLaunchKernelGGL((k_tile<512, 1, false>), dim3(tiles), dim3(512), 0, 0, M, rows, ldM); });
  run("tile 16B/lane nt 256t", [&] { hipLaunchKernelGGL((k_tile<256, 2, true>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile 16B/lane plain 256t", [&] { hipLaunchKernelGGL((k_tile<256, 2, false>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile 16B/lane nt 512t", [&] { hipLaunchKernelGGL((k_tile<512, 2, true>), dim3(tiles), dim3(512), 0, 0, M, rows, ldM); });
  run("tile 32B/lane nt 256t", [&] { hipLaunchKernelGGL((k_tile<256, 4, true>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile 32B/lane plain 256t", [&] { hipLaunchKernelGGL((k_tile<256, 4, false>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile rows 16B nt 256t", [&] { hipLaunchKernelGGL((k_tile_rows<256, true>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile rows 16B plain 256t", [&] { hipLaunchKernelGGL((k_tile_rows<256, false>), dim3(tiles), dim3(256), 0, 0, M, rows, ldM); });
  run("tile rows 16B nt 512t", [&] { hipLaunchKernelGGL((k_tile_rows<512, true>), dim3(tiles), dim3(512), 0, 0, M, rows, ldM); });
  run("oneshot U1 nt", [&] { hipLaunchKernelGGL((k_oneshot<1, true>), dim3((unsigned)((nw + 511) / 512)), dim3(256), 0, 0, M, nw); });
  run("oneshot U1 plain", [&] { hipLaunchKernelGGL((k_oneshot<1, false>), dim3((unsigned)((nw + 511) / 512)), dim3(256), 0, 0, M, nw); });
  run("oneshot U4 plain", [&] { hipLaunchKernelGGL((k_oneshot<4, false>), dim3((unsigned)((nw + 2047) / 2048)), dim3(256), 0, 0, M, nw); });
  run("oneshot U4 nt", [&] { hipLaunchKernelGGL((k_oneshot<4, true>), dim3((unsigned)((nw + 2047) / 2048)), dim3(256), 0, 0, M, nw); });
  run("oneshot U16 plain", [&] { hipLaunchKernelGGL((k_oneshot<16, false>), dim3((unsigned)((nw + 8191) / 8192)), dim3(256), 0, 0, M, nw); });
  for (i64 cw : {8192l, 50176l}) {
    char nm[64];
    snprintf(nm, 64, "chunk %ld KB plain 256t", cw * 8 / 1024);
    run(nm, [&] { hipLaunchKernelGGL((k_chunk<256, false>), dim3((unsigned)((nw + cw - 1) / cw)), dim3(256), 0, 0, M, nw, cw); });
    snprintf(nm, 64, "chunk %ld KB nt 256t", cw * 8 / 1024);
    run(nm, [&] { hipLaunchKernelGGL((k_chunk<256, true>), dim3((unsigned)((nw + cw - 1) / cw)), dim3(256), 0, 0, M, nw, cw); });
    snprintf(nm, 64, "chunk %ld KB plain 512t", cw * 8 / 1024);
    run(nm, [&] { hipLaunchKernelGGL((k_chunk<512, false>), dim3((unsigned)((nw + cw - 1) / cw)), dim3(512), 0, 0, M, nw, cw); });
  }
  for (int K : {4, 8, 16, 32}) {
    const i64 cw = ((ldM + K - 1) / K + 1) & ~1l;
    char nm[64];
    snprintf(nm, 64, "tile32 chunks K=%d 256t", K);
    run(nm, [&] { hipLaunchKernelGGL((k_tchunk<256, 32>), dim3((unsigned)(tiles * K)), dim3(256), 0, 0, M, rows, ldM, cw, K); });
    snprintf(nm, 64, "tile16 chunks K=%d 256t", K);
    run(nm, [&] { hipLaunchKernelGGL((k_tchunk<256, 16>), dim3((unsigned)((rows + 15) / 16 * K)), dim3(256), 0, 0, M, rows, ldM, cw, K); });
  }
  hipMemset(M, 0, 8);
  run("hipMemsetAsync", [&] { hipMemsetAsync(M, 0, nw * 8, 0); });
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
