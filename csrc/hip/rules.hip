// Association rules on the device: subset index + confidence, level-wise
// redundancy cut, and emission of the sorted rule table.
//
// Reference behaviour (AssociationRules.scala):
//   * genRules (:122-145): every frequent S (|S| = k >= 2) and every position p
//     gives the rule (S - {S[p]}) -> S[p], conf = count(S).toDouble / count(S - {S[p]}).
//     The reference finds S - {S[p]} with a linear scan of all (k-1)-itemsets; here
//     one thread per (S, p) binary-searches the lexicographically sorted level k-1
//     (the "subset index" sub_k[S][p]).
//   * cut (:147-182): a rule A -> r with |A| >= 2 survives iff for every a in A the
//     rule (A - {a}) -> r survived one level down with strictly smaller confidence.
//     That child rule lives in itemset S - {a} = S - {S[q]}, whose index is the
//     subset index sub_k[S][q]; inside it the consequent r sits at position
//     p - (q < p).  So the cut is a dense lookup — no hash table of rules, unlike
//     the reference's per-level broadcast of a groupBy map (:158-160).
//   * order (:116-120): torch stable sorts on the device (conf desc, consequent
//     tie position asc, antecedent size asc, antecedent index asc: a total order);
//     k_rule_emit then writes the antecedent rows of the sorted rules.
// Host counterpart (same semantics, CPU runs and tests): csrc/host/rules.cpp.
#include "fa_hip.h"

namespace fa {

constexpr int kRuleTPB = 256;

// Lexicographic compare of the (k-1)-row `a` with row S minus position p.
__device__ __forceinline__ int cmp_skip(const int32_t* __restrict__ a, const int32_t* __restrict__ s, int k,
                                        int p) {
  for (int i = 0, j = 0; i < k - 1; ++i, ++j) {
    if (j == p) ++j;
    const int32_t x = a[i], y = s[j];
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

// One thread per (itemset s, position p) of level k.  Rows of a wave share
// the same few itemsets, so the binary-search probes of neighbouring lanes
// mostly hit the same cache lines of level k-1.
__global__ __launch_bounds__(kRuleTPB) void k_rule_gen(
    const int32_t* __restrict__ S, int64_t nS, int k, const int32_t* __restrict__ A, int64_t nA,
    const int64_t* __restrict__ cS, const int64_t* __restrict__ cA, int32_t* __restrict__ sub,
    double* __restrict__ conf) {
  const int64_t idx = (int64_t)blockIdx.x * kRuleTPB + threadIdx.x;
  if (idx >= nS * k) return;
  const int64_t s = idx / k;
  const int p = (int)(idx - s * k);
  const int32_t* row = S + s * k;
  int64_t lo = 0, hi = nA, found = -1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int c = cmp_skip(A + mid * (k - 1), row, k, p);
    if (c == 0) { found = mid; break; }
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  sub[idx] = (int32_t)found;
  conf[idx] = found >= 0 ? (double)cS[s] / (double)cA[found] : 0.0;
}

// Level-wise cut for level k >= 3 (antecedent size k-1 >= 2).  kept_prev /
// conf_prev: the level k-1 rules ([n_{k-1}][k-1]).
__global__ __launch_bounds__(kRuleTPB) void k_rule_cut(
    const int32_t* __restrict__ sub, const double* __restrict__ conf, int64_t nS, int k,
    const uint8_t* __restrict__ kept_prev, const double* __restrict__ conf_prev, uint8_t* __restrict__ kept) {
  const int64_t idx = (int64_t)blockIdx.x * kRuleTPB + threadIdx.x;
  if (idx >= nS * k) return;
  const int64_t s = idx / k;
  const int p = (int)(idx - s * k);
  const double c = conf[idx];
  const int32_t* srow = sub + s * k;
  bool ok = true;
  for (int q = 0; q < k && ok; ++q) {
    if (q == p) continue;
    const int32_t child = srow[q];
    if (child < 0) { ok = false; break; }
    const int64_t ci = (int64_t)child * (k - 1) + (p - (q < p ? 1 : 0));
    // strict: a child with equal (or higher) confidence makes this rule redundant
    ok = kept_prev[ci] && !(conf_prev[ci] >= c);
  }
  kept[idx] = ok ? 1 : 0;
}

// Antecedent rows of the sorted rules.  rows_all: every level's rows
// concatenated; base[m]: element offset of level m (antecedent size m).
__global__ __launch_bounds__(kRuleTPB) void k_rule_emit(
    const int32_t* __restrict__ rows_all, const int64_t* __restrict__ base, const int32_t* __restrict__ msz,
    const int32_t* __restrict__ ante_idx, const int64_t* __restrict__ ante_off, int64_t R,
    int32_t* __restrict__ ante) {
  const int64_t i = (int64_t)blockIdx.x * kRuleTPB + threadIdx.x;
  if (i >= R) return;
  const int m = msz[i];
  const int32_t* src = rows_all + base[m] + (int64_t)ante_idx[i] * m;
  int32_t* dst = ante + ante_off[i];
  for (int j = 0; j < m; ++j) dst[j] = src[j];
}

inline dim3 rule_grid(int64_t n) { return dim3((unsigned)((n + kRuleTPB - 1) / kRuleTPB)); }

}  // namespace fa

using namespace fa;

FA_API int fa_hip_rule_gen(const int32_t* S, int64_t nS, int k, const int32_t* A, int64_t nA, const int64_t* cS,
                           const int64_t* cA, int32_t* sub, double* conf, hipStream_t st) {
  if (nS <= 0 || k < 2) return 0;
  if (nA >= (int64_t)INT32_MAX) return 3;
  hipLaunchKernelGGL(k_rule_gen, rule_grid(nS * k), dim3(kRuleTPB), 0, st, S, nS, k, A, nA, cS, cA, sub, conf);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_rule_cut(const int32_t* sub, const double* conf, int64_t nS, int k, const uint8_t* kept_prev,
                           const double* conf_prev, uint8_t* kept, hipStream_t st) {
  if (nS <= 0 || k < 3) return 0;
  hipLaunchKernelGGL(k_rule_cut, rule_grid(nS * k), dim3(kRuleTPB), 0, st, sub, conf, nS, k, kept_prev,
                     conf_prev, kept);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_rule_emit(const int32_t* rows_all, const int64_t* base, const int32_t* msz,
                            const int32_t* ante_idx, const int64_t* ante_off, int64_t R, int32_t* ante,
                            hipStream_t st) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(k_rule_emit, rule_grid(R), dim3(kRuleTPB), 0, st, rows_all, base, msz, ante_idx, ante_off,
                     R, ante);
  FA_LAUNCH_RET();
}
