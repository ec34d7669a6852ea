// Host cost of launching a kernel by the size of its by-value argument struct
// (levels.hip passes DlLevels, ~2.5 KB, by value to the plan and threshold kernels).
//   hipcc --offload-arch=gfx950 -O2 kernarg_launch.cpp -o kernarg_launch && ./kernarg_launch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int N>
struct Big { long long v[N]; };

template <int N>
__global__ void k_big(Big<N> b, long long* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[N - 1] == -7) out[0] = b.v[0];
}

template <int N>
static double per_launch_us(hipStream_t st, long long* out, int reps) {
  Big<N> b{};
  for (int i = 0; i < N; ++i) b.v[i] = i;
  (void)hipStreamSynchronize(st);
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_big<N>, dim3(1), dim3(64), 0, st, b, out);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(st);
  auto t2 = std::chrono::steady_clock::now();
  const double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
  const double all = std::chrono::duration<double, std::micro>(t2 - t0).count() / reps;
  printf("arg %5zu B: host %.2f us / launch, host+gpu %.2f us / launch\n", sizeof(Big<N>), host, all);
  return host;
}

int main() {
  hipStream_t st;
  (void)hipStreamCreate(&st);
  long long* out;
  (void)hipMalloc(&out, 64);
  for (int pass = 0; pass < 2; ++pass) {
    per_launch_us<1>(st, out, 200);
    per_launch_us<32>(st, out, 200);
    per_launch_us<128>(st, out, 200);
    per_launch_us<320>(st, out, 200);
    per_launch_us<500>(st, out, 200);
  }
  return 0;
}
