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

// Inclusive wave64 prefix sum on the VALU with DPP (no LDS traffic, unlike
// __shfl_up which lowers to ds_bpermute): row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast:15 and row_bcast:31 across rows (GFX9-family DPP).
__device__ __forceinline__ int wave_scan_incl_dpp(int v) {
  const int lane = (int)(threadIdx.x & 63);
  const int r = lane & 15;
  int t;
  t = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false); if (r >= 1) v += t;   // row_shr:1
  t = __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false); if (r >= 2) v += t;   // row_shr:2
  t = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false); if (r >= 4) v += t;   // row_shr:4
  t = __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false); if (r >= 8) v += t;   // row_shr:8
  t = __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); if ((lane & 31) >= 16) v += t;  // row_bcast:15
  t = __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); if (lane >= 32) v += t;          // row_bcast:31
  return v;
}

__device__ __forceinline__ int wave_last(int v) { return __builtin_amdgcn_readlane(v, 63); }

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

// Orders this wave's LDS accesses across lanes.  The LDS executes one wave's DS
// instructions in issue order, so a read issued after another lane's write sees
// it: only the compiler must not reorder or cache them.  (A memory-model fence
// would also emit s_waitcnt vmcnt(0), draining every prefetched global load of
// a software-pipelined loop at each call: that cost the pair kernel ~7 ms.)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  __asm__ __volatile__("" ::: "memory");
}

// Row-start masks for U consecutive 64-position windows of a wave's CSR span.
// Lane l owns row l = [srel, ...) (rows non-empty, so starts are distinct);
// bit j of S[u] is set when a row starts at position q0 + 64u + j.  words: U
// per-wave LDS scratch words.  The owner row of position q0 + 64u + lane is then
// (starts before the window) + popc(S[u] & lanes <= lane) - 1.
template <int U>
__device__ __forceinline__ void window_starts(unsigned long long* words, int srel, int q0,
                                              unsigned long long (&S)[U]) {
  const int lane = (int)(threadIdx.x & 63);
  if (lane < U) words[lane] = 0ull;
  wave_lds_sync();
  const int b = srel - q0;
  if (b >= 0 && b < 64 * U) atomicOr(&words[b >> 6], 1ull << (b & 63));
  wave_lds_sync();
#pragma unroll
  for (int u = 0; u < U; ++u) S[u] = words[u];
  wave_lds_sync();
}

__device__ __forceinline__ unsigned long long lanes_le_mask() {
  const int lane = (int)(threadIdx.x & 63);
  return lane == 63 ? ~0ull : ((2ull << lane) - 1);
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
