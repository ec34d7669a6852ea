// End-of-kernel accumulator flush: n_wg workgroups each add C u32 counters into the same
// C global counters at once (the slab kernel's flush, count.hip k_count_slab_rec), as
// (0) one global atomicAdd per nonzero counter, (1) plain stores into a per-workgroup
// slice + a column-sum kernel, for C = 8K .. 64K and n_wg = 256 / 512.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o flush_atomics flush_atomics.cpp
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_atomic(uint32_t* __restrict__ out, int C) {
  for (int i = threadIdx.x; i < C; i += blockDim.x) atomicAdd(&out[i], (uint32_t)(blockIdx.x + i) | 1u);
}

__global__ __launch_bounds__(1024) void k_store(uint32_t* __restrict__ part, int C) {
  uint32_t* p = part + (size_t)blockIdx.x * C;
  for (int i = threadIdx.x; i < C; i += blockDim.x) p[i] = (uint32_t)(blockIdx.x + i) | 1u;
}

__global__ __launch_bounds__(256) void k_colsum(const uint32_t* __restrict__ part, int C, int nwg,
                                               uint32_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C) return;
  uint32_t s = 0;
  for (int w = 0; w < nwg; ++w) s += part[(size_t)w * C + i];
  out[i] += s;
}

int main() {
  uint32_t *out, *part;
  (void)hipMalloc(&out, 64 << 12);
  (void)hipMalloc(&part, (size_t)512 * 65536 * 4);
  (void)hipMemset(out, 0, 64 << 12);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int nwg : {256, 512})
    for (int C : {8192, 24576, 65536}) {
      float ms[2] = {0.f, 0.f};
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(k_atomic, dim3(nwg), dim3(1024), 0, 0, out, C);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[0], a, b);
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(k_store, dim3(nwg), dim3(1024), 0, 0, part, C);
        hipLaunchKernelGGL(k_colsum, dim3((C + 255) / 256), dim3(256), 0, 0, part, C, nwg, out);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[1], a, b);
      }
      printf("n_wg %d C %d: atomics %.1f us  stores + column sum %.1f us\n", nwg, C, ms[0] * 1e3, ms[1] * 1e3);
    }
  (void)hipFree(out);
  (void)hipFree(part);
  return 0;
}
