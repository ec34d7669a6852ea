// Issue-rate microbenchmark for the FP4 bit-matrix Gram's inner loop (count.hip
// k_pair_gram_fp4): what a wave per SIMD sustains on v_mfma_scale_f32_32x32x64_f8f6f4
// with a 4 x 4 accumulator tile (256 AGPRs) when the loop adds
//   mode 0: nothing (MFMA only, operands rotated between two register sets)
//   mode 1: the bits -> e2m1 unpacking of the next word's 8 operands (VALU)
//   mode 2: mode 1 plus the next word's 8 ds_read_b32
//   mode 3: mode 2 with the reads two words ahead (raw words double-buffered), so the
//           unpacking never waits on LDS
// at tile 4 x 4 (one wave per SIMD) and 2 x 4 (two waves per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/gram_mfma gram_mfma.cpp
// Prints one line per mode: ms, MFMA count, cycles per MFMA per SIMD at the measured clock.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v8i unpack(uint32_t x) {
  v8i r;
  r[0] = (int)(x & 0x11111111u);
  r[1] = (int)((x >> 1) & 0x11111111u);
  r[2] = (int)((x >> 2) & 0x11111111u);
  r[3] = (int)((x >> 3) & 0x11111111u);
  r[4] = 0; r[5] = 0; r[6] = 0; r[7] = 0;
  return r;
}

template <int MODE, int TI>
__global__ __launch_bounds__(256, TI == 2 ? 2 : 1) void k_bench(const uint32_t* __restrict__ in, float* __restrict__ out, int iters) {
  __shared__ uint32_t S[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) S[i] = in[i & 1023] ^ (uint32_t)i;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  v16f acc[TI][4];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16f{0};
  v8i fa0[TI], fb0[4], fa1[TI], fb1[4];
  uint32_t ra[TI], rb[4];
#pragma unroll
  for (int i = 0; i < TI; ++i) fa0[i] = fa1[i] = unpack(in[lane + 64 * i]);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb0[j] = fb1[j] = unpack(in[lane + 64 * j + 512]);
  uint32_t x = in[lane];
  const int base = (threadIdx.x >> 6) * 1024 + lane * 9;
  uint32_t qa[TI], qb[4];                   // mode 3: the word after next
#pragma unroll
  for (int i = 0; i < TI; ++i) qa[i] = ra[i] = in[lane + 64 * i + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) qb[j] = rb[j] = in[lane + 64 * j + 513];
  auto step = [&](v8i* fa, v8i* fb, v8i* na, v8i* nb, uint32_t* ca, uint32_t* cb, uint32_t* la, uint32_t* lb,
                  int w) {
    if (MODE >= 2) {
#pragma unroll
      for (int i = 0; i < TI; ++i) la[i] = S[(base + 288 * i + w) & 4095];
#pragma unroll
      for (int j = 0; j < 4; ++j) lb[j] = S[(base + 288 * j + 144 + w) & 4095];
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < TI; ++i) la[i] = x + (uint32_t)(i * 77 + w);
#pragma unroll
      for (int j = 0; j < 4; ++j) lb[j] = x ^ (uint32_t)(j * 91 + w);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[i], fb[j], acc[i][j], 4, 4, 0, 128, 0, 128);
    if (MODE >= 1) {
#pragma unroll
      for (int i = 0; i < TI; ++i) na[i] = unpack(ca[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) nb[j] = unpack(cb[j]);
    }
    if (MODE >= 2) {
      __builtin_amdgcn_sched_group_barrier(0x100, TI + 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MODE == 3 ? 1 : 3, 0);
#pragma unroll
      for (int q = MODE == 3 ? 1 : 3; q < TI * 4; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, TI == 4 ? 5 : 6, 0);
      }
    }
  };
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
    if (MODE == 3) {
      // unpack what the previous step loaded, load the word after next
      step(fa0, fb0, fa1, fb1, ra, rb, qa, qb, 2 * it + 2);
      step(fa1, fb1, fa0, fb0, qa, qb, ra, rb, 2 * it + 3);
    } else {
      step(fa0, fb0, fa1, fb1, ra, rb, ra, rb, 2 * it + 1);
      step(fa1, fb1, fa0, fb0, ra, rb, ra, rb, 2 * it + 2);
    }
    x = x * 1664525u + 1013904223u;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) s += acc[i][j][g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int TI>
static void run(const uint32_t* din, float* dout, int wgs, int iters, double clk_ghz, int simds) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((k_bench<MODE, TI>), dim3(wgs), dim3(256), 0, 0, din, dout, 4);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL((k_bench<MODE, TI>), dim3(wgs), dim3(256), 0, 0, din, dout, iters);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double mfma = (double)wgs * 4 * iters * 2 * TI * 4;
  const double cyc = ms * 1e-3 * clk_ghz * 1e9 * simds / mfma;
  printf("mode %d tile %dx4: %.3f ms  %.3g MFMA  %.1f cycles/MFMA/SIMD at %.2f GHz\n", MODE, TI, ms, mfma, cyc,
         clk_ghz);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const double clk = p.clockRate * 1e-6;   // kHz -> GHz (the peak engine clock)
  const int cus = p.multiProcessorCount, simds = 4 * cus;
  printf("%s  %d CUs  clock %.2f GHz\n", p.gcnArchName, cus, clk);
  uint32_t* din;
  float* dout;
  const int wgs = cus * 8;
  (void)hipMalloc(&din, 4096 * 4);
  (void)hipMalloc(&dout, (size_t)wgs * 256 * 4 * 2);
  uint32_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (uint32_t)i * 2654435761u;
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 2000;
  run<0, 4>(din, dout, wgs, iters, clk, simds);
  run<1, 4>(din, dout, wgs, iters, clk, simds);
  run<2, 4>(din, dout, wgs, iters, clk, simds);
  run<3, 4>(din, dout, wgs, iters, clk, simds);
  run<0, 2>(din, dout, wgs * 2, iters, clk, simds);
  run<1, 2>(din, dout, wgs * 2, iters, clk, simds);
  run<2, 2>(din, dout, wgs * 2, iters, clk, simds);
  run<3, 2>(din, dout, wgs * 2, iters, clk, simds);
  (void)hipFree(din);
  (void)hipFree(dout);
  return 0;
}
