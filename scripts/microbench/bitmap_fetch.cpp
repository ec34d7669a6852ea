// Fetch-pattern microbenchmark for the bit-matrix Gram's stages (count.hip
// k_pair_gram_fp4): T40I10D100M geometry (1024 item rows x 1.5625 M words = 12.8 GB),
// 10 upper-triangle tile pairs of 256 rows x a k-chunk of words per workgroup, stages
// of 8 words per row staged through LDS.  Layout 0 = row-major (row stride Wp words:
// every stage touches 512 rows 12.5 MB apart, 64 B each); layout 1 = 8-word blocks,
// [W / 8][rows][8] (a stage's 256 rows are 16 KB contiguous).  Also times the build-side
// store pattern (one workgroup writes 8 words of every row).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bitmap_fetch bitmap_fetch.cpp
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kRows = 1024, kB = 8, kT = 256;

__device__ __forceinline__ int64_t at(int layout, int64_t Wp, int row, int64_t w) {
  return layout ? (w / kB) * (int64_t)kRows * kB + (int64_t)row * kB + (w % kB) : (int64_t)row * Wp + w;
}

__global__ __launch_bounds__(256) void k_fetch(const uint64_t* __restrict__ bm, int64_t Wp, int64_t kchunk, int layout,
                                               uint64_t* __restrict__ out) {
  __shared__ uint64_t S[2][kT * kB];
  const int tp = blockIdx.x % 10;
  const int64_t kc = blockIdx.x / 10;
  int ti = 0, tj = tp;
  while (tj >= 4 - ti) { tj -= 4 - ti; ++ti; }
  tj += ti;
  const int64_t k0 = kc * kchunk, k1 = min(Wp, k0 + kchunk);
  uint64_t x = 0;
  for (int64_t k = k0; k < k1; k += kB) {
#pragma unroll
    for (int it = 0; it < kT * kB / 256; ++it) {
      const int idx = threadIdx.x + it * 256, row = idx / kB, w = idx % kB;
      S[0][idx] = bm[at(layout, Wp, ti * kT + row, k + w)];
      S[1][idx] = bm[at(layout, Wp, tj * kT + row, k + w)];
    }
    __syncthreads();
    x ^= S[0][(threadIdx.x * 9) & (kT * kB - 1)] + S[1][(threadIdx.x * 7) & (kT * kB - 1)];
    __syncthreads();
  }
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void k_store(uint64_t* __restrict__ bm, int64_t Wp, int layout) {
  const int64_t w0 = (int64_t)blockIdx.x * kB;
  for (int i = threadIdx.x; i < kRows * kB; i += 256) {
    const int row = i / kB, w = i % kB;
    bm[at(layout, Wp, row, w0 + w)] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
  }
}

int main() {
  const int64_t Wp = 1562500 / kB * kB;
  const size_t bytes = (size_t)kRows * Wp * 8;
  uint64_t *bm, *out;
  if (hipMalloc(&bm, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  const int64_t nk = 409, kchunk = (Wp + nk - 1) / nk / kB * kB + kB;
  (void)hipMalloc(&out, (size_t)nk * 10 * 256 * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep)
    for (int layout = 0; layout < 2; ++layout) {
      float ms_s = 0.f, ms_f = 0.f;
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(k_store, dim3((unsigned)(Wp / kB)), dim3(256), 0, 0, bm, Wp, layout);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&ms_s, a, b);
      (void)hipEventRecord(a, 0);
      hipLaunchKernelGGL(k_fetch, dim3((unsigned)(nk * 10)), dim3(256), 0, 0, bm, Wp, kchunk, layout, out);
      (void)hipEventRecord(b, 0);
      (void)hipEventSynchronize(b);
      (void)hipEventElapsedTime(&ms_f, a, b);
      printf("layout %s: store %.2f ms (%.0f GB/s)  gram fetch %.2f ms (%.0f GB/s of L2 reads)\n",
             layout ? "blocked" : "row-major", ms_s, bytes / ms_s * 1e-6, ms_f, 2.0 * 10 / 4 * bytes / ms_f * 1e-6);
    }
  (void)hipFree(bm);
  (void)hipFree(out);
  return 0;
}
