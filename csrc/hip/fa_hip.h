// Common definitions for the CDNA4 (gfx950) kernels of FastApriori-AMD.
//
// All kernels are written for 64-lane wavefronts and launched from thin
// extern "C" launchers (ctypes ABI: raw device pointers + hipStream_t), which
// return the hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FA_API extern "C" __attribute__((visibility("default")))

#define FA_LAUNCH_RET() return (int)hipGetLastError()

namespace fa {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// 64-bit popcount-accumulate: lowers to two accumulating v_bcnt_u32_b32.
__device__ __forceinline__ uint32_t popc64_acc(uint64_t x, uint32_t acc) {
  return acc + (uint32_t)__popc((uint32_t)x) + (uint32_t)__popc((uint32_t)(x >> 32));
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical ids land on the same XCD's L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  const uint32_t nx = 8;
  if (nwg < nx) return orig;
  uint32_t q = nwg / nx, r = nwg % nx, xcd = orig % nx;
  uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nx;
}

}  // namespace fa
