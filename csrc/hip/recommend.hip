// First-match recommendation (AssociationRules.scala:80-106): for each distinct
// basket U, the consequent of the first rule (in confidence order) whose
// antecedent is a subset of U and whose consequent is not in U.
//
// One wavefront per basket.  The basket is a bitset over ranks in LDS; each
// step tests 64 consecutive rules, one per lane, and __ballot + ffs picks the
// earliest match, so the scan stops at the first 64-rule chunk that hits.
#include "fa_hip.h"

namespace fa {

constexpr int kRecWaves = 4;

__global__ __launch_bounds__(256) void k_recommend(
    const int64_t* __restrict__ ante_off, const int32_t* __restrict__ ante, const int32_t* __restrict__ cons,
    int64_t R, int32_t F1, const int64_t* __restrict__ boff, const int32_t* __restrict__ bask, int64_t M,
    int32_t* __restrict__ out) {
  extern __shared__ uint32_t bits[];   // [kRecWaves][words]
  const int words = (F1 + 31) >> 5;
  const int wv = threadIdx.x >> 6, lane = lane_id();
  uint32_t* bs = bits + wv * words;
  const int64_t u = (int64_t)blockIdx.x * kRecWaves + wv;
  for (int i = lane; i < words; i += kWave) bs[i] = 0;
  __syncthreads();
  if (u < M) {
    const int64_t s = boff[u], e = boff[u + 1];
    for (int64_t i = s + lane; i < e; i += kWave) atomicOr(&bs[bask[i] >> 5], 1u << (bask[i] & 31));
  }
  __syncthreads();
  if (u >= M) return;
  const int64_t usz = boff[u + 1] - boff[u];
  int32_t rec = -1;
  if (usz > 0) {
    for (int64_t base = 0; base < R; base += kWave) {
      const int64_t r = base + lane;
      bool ok = false;
      if (r < R) {
        const int32_t c = cons[r];
        const int64_t a0 = ante_off[r], a1 = ante_off[r + 1];
        ok = !((bs[c >> 5] >> (c & 31)) & 1u) && (a1 - a0) <= usz;
        for (int64_t i = a0; ok && i < a1; ++i) {
          const int32_t a = ante[i];
          ok = (bs[a >> 5] >> (a & 31)) & 1u;
        }
      }
      const unsigned long long mask = __ballot(ok);
      if (mask) {
        const int first = __ffsll((long long)mask) - 1;
        rec = cons[base + first];
        break;
      }
    }
  }
  if (lane == 0) out[u] = rec;
}

// Indexed first match for large rule tables.  Rule r is listed under the
// last (highest-rank, i.e. least frequent) item of its antecedent; ante ⊆ U
// needs that item in U, so a basket only visits the lists of its own items.
// Lists hold rule ids in ascending (= recommendation) order: a list is scanned
// 64 rules per step until its first hit or until its ids pass the best hit so
// far, and the smallest hit over the basket's lists is the first match of the
// full ordered scan.
__global__ __launch_bounds__(256) void k_recommend_indexed(
    const int64_t* __restrict__ list_off, const int32_t* __restrict__ list_rule,
    const int64_t* __restrict__ ante_off, const int32_t* __restrict__ ante, const int32_t* __restrict__ cons,
    int64_t R, int32_t F1, const int64_t* __restrict__ boff, const int32_t* __restrict__ bask, int64_t M,
    int32_t* __restrict__ out) {
  extern __shared__ uint32_t bits[];   // [kRecWaves][words]
  const int words = (F1 + 31) >> 5;
  const int wv = threadIdx.x >> 6, lane = lane_id();
  uint32_t* bs = bits + wv * words;
  const int64_t u = (int64_t)blockIdx.x * kRecWaves + wv;
  for (int i = lane; i < words; i += kWave) bs[i] = 0;
  __syncthreads();
  if (u < M) {
    const int64_t s = boff[u], e = boff[u + 1];
    for (int64_t i = s + lane; i < e; i += kWave) atomicOr(&bs[bask[i] >> 5], 1u << (bask[i] & 31));
  }
  __syncthreads();
  if (u >= M) return;
  const int64_t s = boff[u], e = boff[u + 1];
  const int64_t usz = e - s;
  int32_t best = (int32_t)R;
  for (int64_t j = s; j < e; ++j) {
    const int32_t item = bask[j];
    const int64_t lo = list_off[item], hi = list_off[item + 1];
    for (int64_t base = lo; base < hi; base += kWave) {
      if (list_rule[base] >= best) break;            // wave-uniform: the rest of the list is later
      const int64_t q = base + lane;
      const int32_t r = q < hi ? list_rule[q] : INT32_MAX;
      bool ok = false;
      if (r < best) {
        const int32_t c = cons[r];
        const int64_t a0 = ante_off[r], a1 = ante_off[r + 1];
        ok = !((bs[c >> 5] >> (c & 31)) & 1u) && (a1 - a0) <= usz;
        for (int64_t i = a0; ok && i < a1 - 1; ++i) {   // the last item is `item`, in U
          const int32_t a = ante[i];
          ok = (bs[a >> 5] >> (a & 31)) & 1u;
        }
      }
      const unsigned long long mask = __ballot(ok);
      if (mask) {
        best = __builtin_amdgcn_readlane(r, __ffsll((long long)mask) - 1);
        break;
      }
    }
  }
  if (lane == 0) out[u] = best < R ? cons[best] : -1;
}

}  // namespace fa

using namespace fa;

FA_API int fa_hip_recommend(const int64_t* ante_off, const int32_t* ante, const int32_t* cons, int64_t R,
                            int32_t F1, const int64_t* boff, const int32_t* bask, int64_t M, int32_t* out,
                            hipStream_t st) {
  if (M <= 0) return 0;
  const size_t words = (size_t)((F1 + 31) / 32);
  const size_t lds = std::max<size_t>(4, words * 4 * kRecWaves);
  if (lds > 64 * 1024) return 2;   // caller falls back to the host path
  dim3 g((unsigned)((M + kRecWaves - 1) / kRecWaves));
  hipLaunchKernelGGL(k_recommend, g, dim3(256), lds, st, ante_off, ante, cons, R, F1, boff, bask, M, out);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_recommend_indexed(const int64_t* list_off, const int32_t* list_rule, const int64_t* ante_off,
                                    const int32_t* ante, const int32_t* cons, int64_t R, int32_t F1,
                                    const int64_t* boff, const int32_t* bask, int64_t M, int32_t* out,
                                    hipStream_t st) {
  if (M <= 0) return 0;
  if (R >= (int64_t)INT32_MAX) return 3;
  const size_t words = (size_t)((F1 + 31) / 32);
  const size_t lds = std::max<size_t>(4, words * 4 * kRecWaves);
  if (lds > 64 * 1024) return 2;   // caller falls back to the host path
  dim3 g((unsigned)((M + kRecWaves - 1) / kRecWaves));
  hipLaunchKernelGGL(k_recommend_indexed, g, dim3(256), lds, st, list_off, list_rule, ante_off, ante, cons, R, F1,
                     boff, bask, M, out);
  FA_LAUNCH_RET();
}
