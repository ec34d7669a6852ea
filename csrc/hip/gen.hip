// Candidate generation (apriori-gen: join + full subset prune) on the GPU.
//
// Reference behaviour: FastApriori.scala:167-193 — for every frequent
// (k-1)-itemset x the extensions are ranks y > max(x) such that (x - x_i) + y
// is frequent for every x_i; groups with no extension are dropped.  Bitset
// formulation (same as the host apriori_gen.cpp fast path): for every
// (m-1)-prefix Q that starts a class of the sorted F_{k-1}, Ext(Q) = bitset of
// the class's last items; then
//     ext(x) = { y > x[m-1] } AND Ext(x[0..m-2]) AND  AND_{p < m-1} Ext(x - x[p]).
// One wave per row, lane w owning bitset word w (ranks < 64 * 64 = 4096), so a
// row's m-1 subset lookups are wave-uniform hash probes and its extensions come
// out ascending from a popcount + DPP prefix scan over the lanes.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "fa_hip.h"

namespace fa {

__device__ __forceinline__ uint64_t ag_mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// hash of row r's items except position `skip` (skip = m-1: the row's (m-1)-prefix)
__device__ __forceinline__ uint64_t ag_hash_drop(const int32_t* __restrict__ r, int m, int skip) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(m - 1);
  for (int q = 0; q < m; ++q)
    if (q != skip) h = ag_mix(h ^ (uint32_t)r[q]);
  return h;
}

// true when row a's first m-1 items equal row b's items except b[skip]
__device__ __forceinline__ bool ag_eq_drop(const int32_t* __restrict__ a, const int32_t* __restrict__ b, int m,
                                           int skip) {
  for (int q = 0, t = 0; q < m; ++q) {
    if (q == skip) continue;
    if (a[t++] != b[q]) return false;
  }
  return true;
}

// insert the class starts: slot <- start row id (open addressing, linear probing)
__global__ __launch_bounds__(256) void k_ag_insert(const int32_t* __restrict__ P, int64_t n, int m,
                                                   int32_t* __restrict__ table, uint32_t mask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t* r = P + i * m;
  if (i > 0) {
    const int32_t* pr = P + (i - 1) * m;
    bool same = true;
    for (int q = 0; q < m - 1; ++q) same = same && r[q] == pr[q];
    if (same) return;                       // not a class start
  }
  uint32_t at = (uint32_t)ag_hash_drop(r, m, m - 1) & mask;
  while (atomicCAS(&table[at], -1, (int32_t)i) != -1) at = (at + 1) & mask;
}

__device__ __forceinline__ int32_t ag_find(const int32_t* __restrict__ P, int m, const int32_t* __restrict__ table,
                                           uint32_t mask, const int32_t* __restrict__ x, int skip) {
  uint32_t at = (uint32_t)ag_hash_drop(x, m, skip) & mask;
  for (;;) {
    const int32_t s = table[at];
    if (s < 0) return -1;
    if (ag_eq_drop(P + (int64_t)s * m, x, m, skip)) return s;
    at = (at + 1) & mask;
  }
}

// Ext bitsets keyed by class start row: ext[s * nw + w]
__global__ __launch_bounds__(256) void k_ag_ext(const int32_t* __restrict__ P, int64_t n, int m,
                                                const int32_t* __restrict__ table, uint32_t mask, int nw,
                                                unsigned long long* __restrict__ ext) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t* r = P + i * m;
  const int32_t s = ag_find(P, m, table, mask, r, m - 1);
  const int32_t y = r[m - 1];
  atomicOr(&ext[(int64_t)s * nw + (y >> 6)], 1ull << (y & 63));
}

// Extension bits of row i: its own class's Ext restricted to y > last, pruned by
// Ext of every other (m-1)-subset.  Lane `lane` owns bitset words [lane * NWL,
// lane * NWL + NWL), so one wave covers F1 <= 4096 * NWL ranks and the extensions
// come out ascending in lane order.  Returns the lane's extension count.
template <int NWL>
__device__ __forceinline__ int ag_row_bits(const int32_t* __restrict__ P, int64_t i, int m,
                                           const int32_t* __restrict__ table, uint32_t mask, int nw,
                                           const unsigned long long* __restrict__ ext, int lane,
                                           unsigned long long (&a)[NWL]) {
  const int32_t* x = P + i * m;
  const int32_t last = x[m - 1];
  const int lw = last >> 6;
  if (m <= 64) {
    // lane p < m probes the class of x without x[p] (p = m - 1: x's own class), so the
    // m probe chains (table load, row compare, Ext load: dependent round trips) are in
    // flight at once; walked one after another they made every speculative level's
    // row kernel 20-35 us of latency at m = 5-9 (the 12.5M-row shard's generator time)
    const int32_t s = lane < m ? ag_find(P, m, table, mask, x, lane) : 0;
    if (__ballot(s < 0) != 0ull) {
#pragma unroll
      for (int j = 0; j < NWL; ++j) a[j] = 0;
      return 0;
    }
    const int32_t s0 = __shfl(s, m - 1, 64);
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int w = lane * NWL + j;
      unsigned long long v = 0;
      if (w < nw && w >= lw) {
        v = ext[(int64_t)s0 * nw + w];
        if (w == lw) v &= (last & 63) == 63 ? 0ull : (~0ull << ((last & 63) + 1));
      }
      a[j] = v;
    }
    // the other m - 1 subsets' Ext words, four loads in flight per step (a step past
    // m - 2 re-reads x's own class: a subset of it already)
    for (int p0 = 0; p0 < m - 1; p0 += 4) {
      unsigned long long t[4][NWL];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int sp = __shfl(s, p0 + u < m - 1 ? p0 + u : m - 1, 64);
#pragma unroll
        for (int j = 0; j < NWL; ++j) {
          const int w = lane * NWL + j;
          t[u][j] = w < nw ? ext[(int64_t)sp * nw + w] : 0ull;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < NWL; ++j) a[j] &= t[u][j];
    }
    int c = 0;
#pragma unroll
    for (int j = 0; j < NWL; ++j) c += __popcll(a[j]);
    return c;
  }
  const int32_t s0 = ag_find(P, m, table, mask, x, m - 1);
  unsigned long long any = 0;
#pragma unroll
  for (int j = 0; j < NWL; ++j) {
    const int w = lane * NWL + j;
    unsigned long long v = 0;
    if (w < nw && w >= lw) {
      v = ext[(int64_t)s0 * nw + w];
      if (w == lw) v &= (last & 63) == 63 ? 0ull : (~0ull << ((last & 63) + 1));
    }
    a[j] = v;
    any |= v;
  }
  for (int p = 0; p < m - 1 && __ballot(any != 0) != 0ull; ++p) {
    const int32_t sp = ag_find(P, m, table, mask, x, p);
    any = 0;
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int w = lane * NWL + j;
      if (sp < 0) a[j] = 0;
      else if (w < nw) a[j] &= ext[(int64_t)sp * nw + w];
      any |= a[j];
    }
    if (sp < 0) break;
  }
  int c = 0;
#pragma unroll
  for (int j = 0; j < NWL; ++j) c += __popcll(a[j]);
  return c;
}

// the extension ids of a row at out[o ..] (and, with rows, the candidate rows (x, y))
template <int NWL>
__device__ __forceinline__ void ag_emit(const unsigned long long (&a)[NWL], int lane, const int32_t* __restrict__ x,
                                        int m, int64_t o, int32_t* __restrict__ out, int32_t* __restrict__ rows) {
#pragma unroll
  for (int j = 0; j < NWL; ++j)
    for (unsigned long long v = a[j]; v; v &= v - 1) {
      const int32_t y = (lane * NWL + j) * 64 + __builtin_ctzll(v);
      out[o] = y;
      if (rows) {   // the full candidate row (x, y): the next speculative level's input
        int32_t* r = rows + o * (m + 1);
        for (int q = 0; q < m; ++q) r[q] = x[q];
        r[m] = y;
      }
      ++o;
    }
}

// pass 0: cnt[i] = number of extensions of row i;  pass 1: write them at off[i].
template <bool kEmit, int NWL = 1>
__global__ __launch_bounds__(256) void k_ag_rows(const int32_t* __restrict__ P, int64_t n, int m,
                                                 const int32_t* __restrict__ table, uint32_t mask, int nw,
                                                 const unsigned long long* __restrict__ ext,
                                                 int32_t* __restrict__ cnt, const int64_t* __restrict__ off,
                                                 int32_t* __restrict__ out, int32_t* __restrict__ rows = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += nwave) {
    unsigned long long a[NWL];
    const int c = ag_row_bits<NWL>(P, i, m, table, mask, nw, ext, lane, a);
    const int incl = wave_scan_incl_dpp(c);
    if (!kEmit) {
      if (lane == 63) cnt[i] = incl;
    } else {
      ag_emit<NWL>(a, lane, P + i * m, m, off[i] + (incl - c), out, rows);
    }
  }
}

// bitset words per lane for nw words: 1, 2, 4 or 8 (F1 <= 32768)
static inline int ag_nwl(int nw) { return nw <= 64 ? 1 : nw <= 128 ? 2 : nw <= 256 ? 4 : 8; }
constexpr int kAgMaxF1 = 64 * 64 * 8;
// u32 words of a chain's used-item bitset (ops.primitives.ag_mark_words mirrors this)
static inline int ag_mark_words(int F1) { return std::max(128, (F1 + 31) / 32); }
// LAUNCH(N) for the lane width N of nw bitset words
#define FA_AG_NWL_SWITCH(nw, LAUNCH) \
  switch (ag_nwl(nw)) {              \
    case 1: LAUNCH(1) break;         \
    case 2: LAUNCH(2) break;         \
    case 4: LAUNCH(4) break;         \
    default: LAUNCH(8) break;        \
  }

}  // namespace fa

using namespace fa;

// Table: int32 [mask + 1] filled with -1 by the caller; ext: u64 [n * nw] zeroed.
FA_API int fa_hip_ag_build(const int32_t* P, int64_t n, int m, int32_t* table, uint32_t mask, int nw, void* ext,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (m < 2 || nw > kAgMaxF1 / 64) return 1;
  dim3 g((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(k_ag_insert, g, dim3(256), 0, st, P, n, m, table, mask);
  hipLaunchKernelGGL(k_ag_ext, g, dim3(256), 0, st, P, n, m, table, mask, nw, (unsigned long long*)ext);
  FA_LAUNCH_RET();
}

// emit = 0: cnt[n] = extensions per row;  emit = 1: out[off[i] ...] = row i's extensions.
FA_API int fa_hip_ag_rows(const int32_t* P, int64_t n, int m, const int32_t* table, uint32_t mask, int nw,
                          const void* ext, int32_t* cnt, const int64_t* off, int32_t* out, int emit, hipStream_t st) {
  if (n <= 0) return 0;
  if (m < 2 || nw > kAgMaxF1 / 64) return 1;
  const unsigned nwg = (unsigned)std::min<int64_t>((n + 3) / 4, 65536);
#define FA_AG_ROWS(N)                                                                                      \
  if (emit)                                                                                                \
    hipLaunchKernelGGL((k_ag_rows<true, N>), dim3(nwg), dim3(256), 0, st, P, n, m, table, mask, nw,       \
                       (const unsigned long long*)ext, cnt, off, out, nullptr);                            \
  else                                                                                                     \
    hipLaunchKernelGGL((k_ag_rows<false, N>), dim3(nwg), dim3(256), 0, st, P, n, m, table, mask, nw,      \
                       (const unsigned long long*)ext, cnt, off, out, nullptr);
  FA_AG_NWL_SWITCH(nw, FA_AG_ROWS)
#undef FA_AG_ROWS
  FA_LAUNCH_RET();
}

// One call: apriori-gen of P (device, [n][m], sorted) with every step on the
// stream and two synchronisations, into the pinned host buffer
//   host = cnt [n] | ext [C] | candidate rows [C][m+1].
// ws: device workspace.  sizes[0] = C; on rc 5 / 6 sizes[1] = bytes of workspace /
// int32 of host buffer needed (the caller grows its buffer and calls again).
FA_API int fa_hip_ag_gen(const int32_t* P, int64_t n, int m, int F1, void* ws, int64_t ws_bytes, int32_t* host,
                         int64_t host_cap, int64_t* sizes, hipStream_t st) {
  sizes[0] = 0;
  if (n <= 0) return 0;
  if (m < 2 || F1 > kAgMaxF1) return 1;
  const int nw = (F1 + 63) / 64;
  uint32_t cap = 16;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  size_t cub_bytes = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, cub_bytes, (const int32_t*)nullptr, (int64_t*)nullptr, (int)n, st);
  const int64_t fixed = al(4 * (int64_t)cap) + al(8 * n * nw) + al(4 * n) + al(8 * (n + 1)) + al((int64_t)cub_bytes);
  if (fixed > ws_bytes) { sizes[1] = fixed; return 5; }
  char* w = static_cast<char*>(ws);
  int32_t* table = reinterpret_cast<int32_t*>(w); w += al(4 * (int64_t)cap);
  unsigned long long* ext = reinterpret_cast<unsigned long long*>(w); w += al(8 * n * nw);
  int32_t* cnt = reinterpret_cast<int32_t*>(w); w += al(4 * n);
  int64_t* off = reinterpret_cast<int64_t*>(w); w += al(8 * (n + 1));
  void* cub_tmp = w; w += al((int64_t)cub_bytes);
  (void)hipMemsetAsync(table, 0xFF, 4 * (size_t)cap, st);
  (void)hipMemsetAsync(ext, 0, 8 * (size_t)n * nw, st);
  (void)hipMemsetAsync(off, 0, 8, st);
  dim3 g((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(k_ag_insert, g, dim3(256), 0, st, P, n, m, table, cap - 1);
  hipLaunchKernelGGL(k_ag_ext, g, dim3(256), 0, st, P, n, m, table, cap - 1, nw, ext);
  const unsigned nwg = (unsigned)std::min<int64_t>((n + 3) / 4, 65536);
#define FA_AG_CNT(N)                                                                                        \
  hipLaunchKernelGGL((k_ag_rows<false, N>), dim3(nwg), dim3(256), 0, st, P, n, m, table, cap - 1, nw, ext, cnt, \
                     nullptr, nullptr, nullptr);
  FA_AG_NWL_SWITCH(nw, FA_AG_CNT)
  (void)hipcub::DeviceScan::InclusiveSum(cub_tmp, cub_bytes, cnt, off + 1, (int)n, st);
  int64_t C = 0;
  (void)hipMemcpyAsync(&C, off + n, 8, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  const int64_t need_ws = fixed + al(4 * C) + al(4 * C * (m + 1));
  if (need_ws > ws_bytes) { sizes[1] = need_ws; return 5; }
  const int64_t need_host = n + C + C * (m + 1);
  if (need_host > host_cap) { sizes[1] = need_host; return 6; }
  int32_t* ext_out = reinterpret_cast<int32_t*>(w); w += al(4 * C);
  int32_t* rows_out = reinterpret_cast<int32_t*>(w);
#define FA_AG_EMIT(N)                                                                                        \
  hipLaunchKernelGGL((k_ag_rows<true, N>), dim3(nwg), dim3(256), 0, st, P, n, m, table, cap - 1, nw, ext, nullptr, \
                     off, ext_out, rows_out);
  if (C) { FA_AG_NWL_SWITCH(nw, FA_AG_EMIT) }
  (void)hipMemcpyAsync(host, cnt, 4 * (size_t)n, hipMemcpyDeviceToHost, st);
  if (C) {
    (void)hipMemcpyAsync(host + n, ext_out, 4 * (size_t)C, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(host + n + C, rows_out, 4 * (size_t)C * (m + 1), hipMemcpyDeviceToHost, st);
  }
  (void)hipStreamSynchronize(st);
  sizes[0] = C;
  FA_LAUNCH_RET();
}

// Speculative level chain for level bundling (fastapriori_amd FastApriori._plan_bundle):
// starting from level k's candidate rows P0 [n0][m0] (device), generate level
// k+1 from them, then k+2 from those, ... on the stream, with one 8-byte
// readback per level (its candidate count) instead of a host round trip per
// level.  A level is accepted while C > 0, C <= growth * C_prev, the bundle
// total stays <= tmax (the slab accumulator capacity) and fewer than
// max_levels were accepted; the first rejected level ends the chain.
//   sizes[0] = accepted levels L; sizes[2 + l] = C_l;  rc 5 / 6: sizes[1] = bytes of
//   workspace / int32 of host buffer to retry with.
//   host, per accepted level l: cnt [n_l] | ext [C_l] | rows [C_l][m_l + 1]
//   (n_{l+1} = C_l, m_{l+1} = m_l + 1).
// Bundle accumulator limit (fastapriori_amd ops.primitives.slab_capacity / slab_total_limit):
// slab capacity for n_used items and C candidates, and the largest total t with
// t <= capacity(t).
static int64_t ag_slab_cap(int64_t n_used, int64_t C, double lds) {
  for (int sw : {16, 32, 8, 4}) {      // plan.cpp slab_width order
    const int64_t cap = (int64_t)((lds - (double)n_used * (sw + 2) * 8) / 4);
    if (cap >= std::min<int64_t>(C, 8192) || (sw == 4 && cap >= 1024)) return cap;
  }
  return 0;
}
static int64_t ag_total_limit(int64_t n_used, double lds) {
  int64_t lo = 0, hi = (int64_t)1 << 31;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) / 2;
    if (mid <= ag_slab_cap(n_used, mid, lds)) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Per-level workspace init of the chain: hash table <- -1, Ext bitsets <- 0, off[0] <- 0.
__global__ __launch_bounds__(256) void k_ag_init(int32_t* __restrict__ table, int64_t cap,
                                                 unsigned long long* __restrict__ ext, int64_t n_ext,
                                                 int64_t* __restrict__ off) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cap; i += stride) table[i] = -1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_ext; i += stride) ext[i] = 0ull;
  if (blockIdx.x == 0 && threadIdx.x == 0) off[0] = 0;
}

// Bitset of the items in rows (MW u32 words): privatised in LDS per workgroup, then
// one global atomicOr per non-zero word (every thread OR-ing into the same global
// words serialised: 2.6 ms per call on T40I10's 150K-candidate levels).
__global__ __launch_bounds__(256) void k_ag_mark(const int32_t* __restrict__ rows, int64_t n,
                                                 uint32_t* __restrict__ bits, int MW) {
  __shared__ uint32_t lb[kAgMaxF1 / 32];
  for (int q = threadIdx.x; q < MW; q += 256) lb[q] = 0u;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicOr(&lb[rows[i] >> 5], 1u << (rows[i] & 31));
  __syncthreads();
  for (int q = threadIdx.x; q < MW; q += 256)
    if (lb[q]) atomicOr(&bits[q], lb[q]);
}

static int ag_chain_dev(const int32_t* P1, int64_t n1, int m1, int nw, char* w0, char* w, int64_t ws_bytes,
                        int32_t* host, int64_t hoff, int64_t host_cap, int max_levels, double growth, int64_t total,
                        int64_t last, const uint32_t* mark, int MW, double lds, int64_t* sizes, hipStream_t st);

// first_free = 1 (lds > 0): P0 is F_{k-1} itself; level 0 (= level k's candidates)
// is always emitted, its used items (a device bitset, read back with level 1's
// count) give n_used and the bundle limit tmax, and the chain continues only if
// level k alone fits one accumulator pass.  host[0 .. 128) then holds that bitset
// and the levels start at host[128].
FA_API int fa_hip_ag_chain(const int32_t* P0, int64_t n0, int m0, int F1, void* ws, int64_t ws_bytes, int32_t* host,
                           int64_t host_cap, int max_levels, double growth, int64_t total0, int64_t tmax,
                           int64_t* sizes, hipStream_t st, int first_free, double lds) {
  sizes[0] = 0;
  if (n0 <= 0 || max_levels <= 0) return 0;
  if (m0 < 2 || F1 > kAgMaxF1) return 1;
  const int nw = (F1 + 63) / 64;
  const int MW = ag_mark_words(F1);
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  char* const w0 = static_cast<char*>(ws);
  char* w = w0;
  const int32_t* P = P0;
  int64_t n = n0, last = n0, total = total0, hoff = first_free ? MW : 0;
  int m = m0, L = 0;
  uint32_t* mark = nullptr;
  if (first_free) {
    if (host_cap < MW) { sizes[1] = 1 << 20; return 6; }
    mark = reinterpret_cast<uint32_t*>(w); w += al(4 * MW);
    (void)hipMemsetAsync(mark, 0, 4 * MW, st);
  }
  int64_t* Cdev = nullptr;
  int64_t Ch = 0;
  for (int l = 0; l < max_levels; ++l) {
    uint32_t cap = 16;
    while (cap < 2 * (uint64_t)n) cap <<= 1;
    size_t cub_bytes = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, cub_bytes, (const int32_t*)nullptr, (int64_t*)nullptr, (int)n,
                                           st);
    const int64_t fixed = al(4 * (int64_t)cap) + al(8 * n * nw) + al(4 * n) + al(8 * (n + 1)) + al((int64_t)cub_bytes);
    if ((w - w0) + fixed > ws_bytes) { (void)hipStreamSynchronize(st); sizes[1] = 2 * ((w - w0) + fixed); return 5; }
    int32_t* table = reinterpret_cast<int32_t*>(w); w += al(4 * (int64_t)cap);
    unsigned long long* ext = reinterpret_cast<unsigned long long*>(w); w += al(8 * n * nw);
    int64_t* off = reinterpret_cast<int64_t*>(w); w += al(8 * (n + 1));
    void* cub_tmp = w; w += al((int64_t)cub_bytes);
    // cnt | ext_out | rows_out contiguous (the host layout): one readback per level
    int32_t* cnt = reinterpret_cast<int32_t*>(w);
    hipLaunchKernelGGL(k_ag_init, dim3((unsigned)std::min<int64_t>((cap + 255) / 256, 4096)), dim3(256), 0, st,
                       table, (int64_t)cap, ext, n * nw, off);
    dim3 g((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(k_ag_insert, g, dim3(256), 0, st, P, n, m, table, cap - 1);
    hipLaunchKernelGGL(k_ag_ext, g, dim3(256), 0, st, P, n, m, table, cap - 1, nw, ext);
    const unsigned nwg = (unsigned)std::min<int64_t>((n + 3) / 4, 65536);
    FA_AG_NWL_SWITCH(nw, FA_AG_CNT)
    (void)hipcub::DeviceScan::InclusiveSum(cub_tmp, cub_bytes, cnt, off + 1, (int)n, st);
    Cdev = off + n;
    (void)hipMemcpyAsync(&Ch, Cdev, 8, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    const int64_t C = Ch;
    if (first_free && l == 1) {
      // level k's used items arrived with this sync: the bundle limit
      int64_t n_used = 0;
      for (int q = 0; q < MW; ++q) n_used += __builtin_popcount((uint32_t)host[q]);
      tmax = ag_total_limit(n_used, lds);
      if (total > ag_slab_cap(n_used, total, lds)) break;   // level k alone needs several passes
    }
    if (C == 0) break;
    if (!(first_free && l == 0) && ((double)C > growth * (double)last || total + C > tmax)) break;
    const int64_t need_ws = (w - w0) + al(4 * (n + C + C * (m + 1)));
    if (need_ws > ws_bytes) { sizes[1] = 2 * need_ws; return 5; }
    const int64_t need_host = hoff + n + C + C * (m + 1);
    if (need_host > host_cap) { (void)hipStreamSynchronize(st); sizes[1] = 2 * need_host; return 6; }
    int32_t* ext_out = cnt + n;
    int32_t* rows_out = ext_out + C;
    w += al(4 * (n + C + C * (m + 1)));
    FA_AG_NWL_SWITCH(nw, FA_AG_EMIT)
    (void)hipMemcpyAsync(host + hoff, cnt, 4 * (size_t)(n + C + C * (m + 1)), hipMemcpyDeviceToHost, st);
    if (first_free && l == 0) {
      hipLaunchKernelGGL(k_ag_mark, dim3((unsigned)std::min<int64_t>((C * (m + 1) + 255) / 256, 1024)), dim3(256), 0,
                         st, rows_out, C * (m + 1), mark, MW);
      (void)hipMemcpyAsync(host, mark, 4 * MW, hipMemcpyDeviceToHost, st);
    }
    hoff = need_host;
    sizes[2 + l] = C;
    ++L;
    total += C;
    last = C;
    P = rows_out;
    n = C;
    ++m;
    // levels 1.. without a host round trip per level (other chains: the loop below)
    if (first_free && l == 0)
      return ag_chain_dev(P, n, m, nw, w0, w, ws_bytes, host, hoff, host_cap, max_levels, growth, total, last, mark,
                          MW, lds, sizes, st);
  }
  (void)hipStreamSynchronize(st);
  sizes[0] = L;
  FA_LAUNCH_RET();
}

// ---------------------------------------------------------------------------
// Device helpers of the speculative chains below: the slab accumulator limit
// (ops.primitives.slab_capacity) and one row's pruned extension bits.
// (A single cooperative kernel for the whole chain, every level's phases split by
// grid barriers, measured slower than the kernel boundaries: removed.)
// ---------------------------------------------------------------------------
namespace fa {

// accb: LDS bytes per accumulator (4, or 2 for count.hip's packed u16 counters)
// capmax (fa_hip_set_cap_max): a bundle may take a narrower slab when that is what holds
// all of its candidates (the first width whose capacity is >= C, else the largest
// capacity); 0: the first width holding min(C, 8192), as plan.cpp slab_width
__device__ int64_t d_slab_cap(int64_t n_used, int64_t C, double lds, double accb, int capmax = 0) {
  const int sws[4] = {16, 32, 8, 4};   // plan.cpp slab_width order
  int64_t best = 0;
  for (int q = 0; q < 4; ++q) {
    const int sw = sws[q];
    const int64_t cap = (int64_t)((lds - (double)n_used * (sw + 2) * 8) / accb);
    if (capmax) {
      if (cap >= C && (sw != 4 || cap >= 1024)) return cap;
      if (cap > best) best = cap;
      continue;
    }
    if (cap >= (C < 8192 ? C : 8192) || (sw == 4 && cap >= 1024)) return cap;
  }
  return capmax ? best : 0;
}

__device__ int64_t d_total_limit(int64_t n_used, double lds, double accb) {
  int64_t lo = 0, hi = (int64_t)1 << 31;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) / 2;
    if (mid <= d_slab_cap(n_used, mid, lds, accb)) lo = mid; else hi = mid - 1;
  }
  return lo;
}

}  // namespace fa

// ---------------------------------------------------------------------------
// Device-sized speculative levels (first_free chains, after level 0).
//
// fa_hip_ag_chain used to read every speculative level's candidate count back
// before it could size and launch the next level: one host round trip per level
// (~0.1 ms of GPU idle each; 7 of them for the T10I4 bundle 5-12).  Here every
// kernel of level l reads its row count from a device control block and exits
// once the chain has stopped, the acceptance rule (C > 0, C <= growth * C_prev,
// bundle total <= tmax) runs at the end of the one-workgroup scan kernel, and
// tmax itself comes from level 0's used-item bitset on the device.  Buffers are
// sized by bounds (C_l <= min(growth * n_l, accumulator limit)); levels are
// enqueued in batches of kAgdBatch with one control-block readback per batch,
// then the accepted levels are copied out.  (A single cooperative kernel was
// measured slower: its grid barriers cost more than these kernel boundaries.)
//   ctl (device int64): 0 stop, 1 accepted levels (incl. level 0), 2 total,
//   3 last C, 4 tmax, 8 + l: n_l (input rows of level l), 40 + l: C_l.
// ---------------------------------------------------------------------------
namespace fa {

constexpr int kAgdMaxLevels = 30;
constexpr int kAgdBatch = 4;

__global__ void k_agd_setup(long long* __restrict__ c, int64_t n1, int64_t total, int64_t last,
                            const uint32_t* __restrict__ mark, int MW, double lds) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t n_used = 0;
  for (int q = 0; q < MW; ++q) n_used += __popc(mark[q]);
  c[0] = total > d_slab_cap(n_used, total, lds, 4.0) ? 1 : 0;   // level k alone needs several passes
  c[1] = 1;
  c[2] = total;
  c[3] = last;
  c[4] = d_total_limit(n_used, lds, 4.0);
  c[9] = n1;
}

// clear the hash tables (-1) and Ext bitsets (0) of a batch of levels: region q is
// [p[q], p[q] + len[q]) words of 32 bits, value val[q]
struct AgdClear {
  uint32_t* p[2 * kAgdBatch];
  int64_t len[2 * kAgdBatch];
  uint32_t val[2 * kAgdBatch];
  int nreg;
};

__global__ __launch_bounds__(256) void k_agd_clear(AgdClear A, const long long* __restrict__ c) {
  if (c[0]) return;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int q = 0; q < A.nreg; ++q)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < A.len[q]; i += stride) A.p[q][i] = A.val[q];
}

__global__ __launch_bounds__(256) void k_agd_insert(const int32_t* __restrict__ P, int m, int32_t* __restrict__ table,
                                                    uint32_t mask, const long long* __restrict__ c, int l) {
  if (c[0]) return;
  const int64_t n = c[8 + l];
  // grid-stride (the grid is sized for the level's bound, capped: a stopped chain's
  // launches then cost a few workgroups each)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* r = P + i * m;
    if (i > 0) {
      const int32_t* pr = P + (i - 1) * m;
      bool same = true;
      for (int q = 0; q < m - 1; ++q) same = same && r[q] == pr[q];
      if (same) continue;
    }
    uint32_t at = (uint32_t)ag_hash_drop(r, m, m - 1) & mask;
    while (atomicCAS(&table[at], -1, (int32_t)i) != -1) at = (at + 1) & mask;
  }
}

__global__ __launch_bounds__(256) void k_agd_ext(const int32_t* __restrict__ P, int m,
                                                 const int32_t* __restrict__ table, uint32_t mask, int nw,
                                                 unsigned long long* __restrict__ ext, const long long* __restrict__ c,
                                                 int l) {
  if (c[0]) return;
  const int64_t n = c[8 + l];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* r = P + i * m;
    const int32_t s = ag_find(P, m, table, mask, r, m - 1);
    const int32_t y = r[m - 1];
    atomicOr(&ext[(int64_t)s * nw + (y >> 6)], 1ull << (y & 63));
  }
}

// kEmit = false: cnt[i] = extensions of row i;  true (accepted levels only): ext ids at
// cnt + n + off[i] (the host layout cnt | ext) and the candidate rows at rows + off[i] * (m + 1)
template <bool kEmit, int NWL = 1>
__global__ __launch_bounds__(256) void k_agd_rows(const int32_t* __restrict__ P, int m,
                                                  const int32_t* __restrict__ table, uint32_t mask, int nw,
                                                  const unsigned long long* __restrict__ ext, int32_t* __restrict__ cnt,
                                                  const int64_t* __restrict__ off, int32_t* __restrict__ rows,
                                                  const long long* __restrict__ c, int l) {
  if (c[0]) return;
  const int64_t n = c[8 + l];
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += nwave) {
    unsigned long long a[NWL];
    const int cc = ag_row_bits<NWL>(P, i, m, table, mask, nw, ext, lane, a);
    const int incl = wave_scan_incl_dpp(cc);
    if (!kEmit) {
      if (lane == 63) cnt[i] = incl;
    } else {
      ag_emit<NWL>(a, lane, P + i * m, m, off[i] + (incl - cc), cnt + n, rows);
    }
  }
}

// off[0 .. n] = exclusive offsets of cnt[0 .. n) (one workgroup), then the acceptance of
// level l by thread 0: C_l = off[n_l]
__global__ __launch_bounds__(1024) void k_agd_scan_decide(const int32_t* __restrict__ cnt, int64_t* __restrict__ off,
                                                          long long* __restrict__ c, int l, double growth,
                                                          int64_t c_bound) {
  __shared__ int64_t part[16];
  __shared__ int64_t carry;
  if (c[0]) return;
  const int64_t n = c[8 + l];
  if (threadIdx.x == 0) { carry = 0; off[0] = 0; }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t b = 0; b < n; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const int v = i < n ? cnt[i] : 0;
    const int incl = wave_scan_incl_dpp(v);
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int q = 0; q < wv; ++q) before += part[q];
    if (i < n) off[i + 1] = before + incl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const int64_t C = carry;
  const int64_t total = c[2], last = c[3], tmax = c[4];
  if (C == 0 || (double)C > growth * (double)last || total + C > tmax || C > c_bound) { c[0] = 1; return; }
  c[40 + l] = C;
  c[1] = l + 1;
  c[2] = total + C;
  c[3] = C;
  c[8 + l + 1] = C;
}

}  // namespace fa

// Levels 1 .. of a first_free chain (see above).  P1 = level 0's candidate rows
// (device, [n1][m1]), mark = level 0's used-item bitset (device, 128 words).  The
// host layout continues at host[hoff].  On return (rc 0) sizes[0] = accepted
// levels including level 0 and sizes[2 + l] = C_l for l >= 1.
static int ag_chain_dev(const int32_t* P1, int64_t n1, int m1, int nw, char* w0, char* w, int64_t ws_bytes,
                        int32_t* host, int64_t hoff, int64_t host_cap, int max_levels, double growth, int64_t total,
                        int64_t last, const uint32_t* mark, int MW, double lds, int64_t* sizes, hipStream_t st) {
  using namespace fa;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  const int LM = std::min(max_levels - 1, kAgdMaxLevels - 2);
  long long* c = reinterpret_cast<long long*>(w); w += al(8 * 72);
  const int64_t acc_max = (int64_t)(lds / 4);         // no bundle total passes the accumulator capacity
  struct Lv { int32_t* cnt; int32_t* rows; int m; };
  Lv lv[kAgdMaxLevels];
  int64_t nb = n1;
  int m = m1;
  const int32_t* P = P1;
  long long ch[72];
  ch[0] = LM <= 0;
  ch[1] = 1;
  hipLaunchKernelGGL(k_agd_setup, dim3(1), dim3(64), 0, st, c, n1, total, last, mark, MW, lds);
  for (int l0 = 1; l0 <= LM && !ch[0]; l0 += kAgdBatch) {
    const int l1 = std::min(LM, l0 + kAgdBatch - 1);
    struct Bufs { int32_t* table; uint32_t cap; unsigned long long* ext; int64_t* off; int64_t nb, cb; };
    Bufs bf[kAgdBatch];
    AgdClear clr{};
    int64_t clr_max = 0;
    for (int l = l0; l <= l1; ++l) {
      const int64_t cb = std::min<int64_t>(acc_max, (int64_t)(growth * (double)nb) + 1);
      uint32_t cap = 16;
      while (cap < 2 * (uint64_t)nb) cap <<= 1;
      const int64_t need = al(4 * (int64_t)cap) + al(8 * nb * nw) + al(8 * (nb + 1)) + al(4 * (nb + cb)) +
                           al(4 * cb * (m + 1));
      if ((w - w0) + need > ws_bytes) { (void)hipStreamSynchronize(st); sizes[1] = 2 * ((w - w0) + need); return 5; }
      Bufs& b = bf[l - l0];
      b.table = reinterpret_cast<int32_t*>(w); w += al(4 * (int64_t)cap);
      b.ext = reinterpret_cast<unsigned long long*>(w); w += al(8 * nb * nw);
      b.off = reinterpret_cast<int64_t*>(w); w += al(8 * (nb + 1));
      b.cap = cap; b.nb = nb; b.cb = cb;
      lv[l].cnt = reinterpret_cast<int32_t*>(w); w += al(4 * (nb + cb));
      lv[l].rows = reinterpret_cast<int32_t*>(w); w += al(4 * cb * (m + 1));
      lv[l].m = m;
      clr.p[clr.nreg] = reinterpret_cast<uint32_t*>(b.table); clr.len[clr.nreg] = cap; clr.val[clr.nreg++] = ~0u;
      clr.p[clr.nreg] = reinterpret_cast<uint32_t*>(b.ext); clr.len[clr.nreg] = 2 * nb * nw; clr.val[clr.nreg++] = 0u;
      clr_max = std::max<int64_t>(clr_max, std::max<int64_t>(cap, 2 * nb * nw));
      nb = cb;
      ++m;
    }
    hipLaunchKernelGGL(k_agd_clear, dim3((unsigned)std::min<int64_t>((clr_max + 255) / 256, 1024)), dim3(256), 0, st,
                       clr, c);
    for (int l = l0; l <= l1; ++l) {
      const Bufs& b = bf[l - l0];
      const int ml = lv[l].m;
      const dim3 g((unsigned)std::min<int64_t>((b.nb + 255) / 256, 512));
      hipLaunchKernelGGL(k_agd_insert, g, dim3(256), 0, st, P, ml, b.table, b.cap - 1, c, l);
      hipLaunchKernelGGL(k_agd_ext, g, dim3(256), 0, st, P, ml, b.table, b.cap - 1, nw, b.ext, c, l);
      const unsigned nwg = (unsigned)std::min<int64_t>((b.nb + 3) / 4, 2048);
#define FA_AGD_ROWS(E, N)                                                                                   \
  hipLaunchKernelGGL((k_agd_rows<E, N>), dim3(nwg), dim3(256), 0, st, P, ml, b.table, b.cap - 1, nw, b.ext,   \
                     lv[l].cnt, b.off, lv[l].rows, c, l);
#define FA_AGD_CNT(N) FA_AGD_ROWS(false, N)
#define FA_AGD_EMIT(N) FA_AGD_ROWS(true, N)
      FA_AG_NWL_SWITCH(nw, FA_AGD_CNT)
      hipLaunchKernelGGL(k_agd_scan_decide, dim3(1), dim3(1024), 0, st, lv[l].cnt, b.off, c, l, growth, b.cb);
      FA_AG_NWL_SWITCH(nw, FA_AGD_EMIT)
#undef FA_AGD_EMIT
#undef FA_AGD_CNT
#undef FA_AGD_ROWS
      P = lv[l].rows;
    }
    (void)hipMemcpyAsync(ch, c, sizeof(ch), hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return 7;
  }
  const int L = (int)ch[1];
  for (int l = 1; l < L; ++l) {
    const int64_t n = ch[8 + l], C = ch[40 + l];
    const int ml = lv[l].m;
    const int64_t need_host = hoff + n + C + C * (ml + 1);
    if (need_host > host_cap) { (void)hipStreamSynchronize(st); sizes[1] = 2 * need_host; return 6; }
    (void)hipMemcpyAsync(host + hoff, lv[l].cnt, 4 * (size_t)(n + C), hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(host + hoff + n + C, lv[l].rows, 4 * (size_t)(C * (ml + 1)), hipMemcpyDeviceToHost, st);
    hoff = need_host;
    sizes[2 + l] = C;
  }
  (void)hipStreamSynchronize(st);
  sizes[0] = L;
  FA_LAUNCH_RET();
}

// ---------------------------------------------------------------------------
// Device-resident level bundles (fastapriori_amd FastApriori._mine_device).
//
// The host loop above reads every bundle's candidate rows back, plans the count
// in C++ and thresholds on the host: ~2 ms of GPU idle per run, most of the
// 12.5M-row shard's host gap.  Here the candidates never leave the GPU: level 0
// of a bundle is generated from F_{k-1} rows that are themselves on the device
// (the previous bundle's thresholded output, or F_2), its row count comes from
// a device word, and the host learns only what it must decide on: C_0, the
// used-item bitset (trimming, slab width) and whether level k alone fits one
// accumulator pass.  The speculative levels 1.. follow with the batched device
// acceptance of ag_chain_dev, without copying any level out.  Planning
// (levels.hip fa_hip_dl_plan), counting and thresholding (fa_hip_dl_threshold)
// then run on the same stream.
//   ctl (device int64 [kDlCtl]): 0 stop  1 accepted levels  2 total  3 last C
//     5 multi (level 0 needs several accumulator passes: host path)  6 n_used
//     7 end (|F_{k-1}| < k or C_0 = 0: mining is over)  8 + l: n_l  40 + l: C_l
//     72 + l: G_l (parent rows with >= 1 candidate: the reference's group count)
//     104 (kDlEmpty): the chain stopped on a speculative level with no candidates
//     512 .. 1023: used-item bitset of level 0 (kDlBitsW words: F1 <= 32768 bits)
// ---------------------------------------------------------------------------
namespace fa {

constexpr int kDlCtl = 1024;
constexpr int kDlBits = 512;       // first word of the used-item bitset in ctl
constexpr int kDlBitsW = 512;      // its 64-bit words (F1 <= kAgMaxF1 = 32768)
constexpr int kDlEmpty = 104;      // 1: the chain stopped on a level without candidates

__device__ int64_t agd_block_scan(const int32_t* __restrict__ cnt, int64_t* __restrict__ off, int64_t n,
                                  int64_t* groups = nullptr) {
  // exclusive offsets off[0 .. n] of cnt[0 .. n) by one 1024-thread workgroup; returns off[n].
  // groups (thread 0's copy): rows with cnt > 0, the reference's prefix-group count
  // (genCandidates drops empty groups, FastApriori.scala:189-190)
  __shared__ int64_t part[16];
  __shared__ int64_t carry;
  __shared__ unsigned int nz;
  if (threadIdx.x == 0) { carry = 0; off[0] = 0; nz = 0u; }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t b = 0; b < n; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const int v = i < n ? cnt[i] : 0;
    const int incl = wave_scan_incl_dpp(v);
    const unsigned long long had = __ballot(v > 0);
    if (lane == 0 && had) atomicAdd(&nz, (unsigned int)__popcll(had));
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int q = 0; q < wv; ++q) before += part[q];
    if (i < n) off[i + 1] = before + incl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (groups && threadIdx.x == 0) *groups = (int64_t)nz;
  return carry;
}

// ctl[4] = 1: the device row count n_src[0] exceeds n_bound (the buffers' size):
// nothing runs and the host raises
__global__ __launch_bounds__(kDlCtl) void k_dl_setup0(long long* __restrict__ c, const long long* __restrict__ n_src,
                                                      int64_t n_const, int kmin, int64_t n_bound) {
  c[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t n = n_src ? (int64_t)n_src[0] : n_const;
    if (n > n_bound) { c[4] = 1; c[0] = 1; return; }
    c[8] = n;
    c[7] = n < kmin ? 1 : 0;       // the reference's loop test |F_{k-1}| >= k (FastApriori.scala:111)
    c[0] = c[7];
  }
}

// level 0: the exclusive scan, then C_0 > c_bound (the level's output buffer, sized for
// one accumulator pass) marks it "multi" (host path); C_0 = 0 ends the mining
__global__ __launch_bounds__(1024) void k_dl_decide0(const int32_t* __restrict__ cnt, int64_t* __restrict__ off,
                                                      long long* __restrict__ c, int64_t c_bound) {
  if (c[0]) return;
  int64_t g = 0;
  const int64_t C = agd_block_scan(cnt, off, c[8], &g);
  if (threadIdx.x != 0) return;
  c[40] = C;
  c[72] = g;
  if (C == 0) { c[7] = 1; c[0] = 1; return; }
  if (C > c_bound) { c[5] = 1; c[0] = 1; return; }
  c[1] = 1; c[2] = C; c[3] = C; c[9] = C;
}

// Level 0's scan over many workgroups when F_{k-1} is large (T40I10D100M's bundles start
// from up to ~157K parent rows, where the one-workgroup k_dl_decide0 took ~78 us):
// (1) kDsBlk-row block scans into off[] (block-local) with the block totals, (2) one
// workgroup scans the totals and takes k_dl_decide0's decisions, (3) the block bases
// are added to off[].  bs: int64 scratch [3 * nblk].
constexpr int kDsBlk = 4096;

__global__ __launch_bounds__(1024) void k_ds_blocks(const int32_t* __restrict__ cnt, int64_t* __restrict__ off,
                                                    const long long* __restrict__ c, int64_t* __restrict__ bs,
                                                    int nblk) {
  if (c[0]) return;
  const int64_t n = c[8];
  const int64_t b0 = (int64_t)blockIdx.x * kDsBlk;
  if (b0 >= n) {
    if (threadIdx.x == 0) { bs[blockIdx.x] = 0; bs[nblk + blockIdx.x] = 0; }
    return;
  }
  __shared__ int wpart[16];
  __shared__ int wnz[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // four consecutive rows per thread, in order
  int v[4], t = 0, nz = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = b0 + 4 * (int64_t)threadIdx.x + u;
    v[u] = i < n ? cnt[i] : 0;
    t += v[u];
    nz += v[u] > 0;
  }
  const int incl = wave_scan_incl_dpp(t);
  const int nzs = (int)wave_sum_u32((uint32_t)nz);
  if (lane == 63) wpart[wv] = incl;
  if (lane == 0) wnz[wv] = nzs;
  __syncthreads();
  int64_t run = incl - t;
  for (int q = 0; q < wv; ++q) run += wpart[q];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = b0 + 4 * (int64_t)threadIdx.x + u;
    run += v[u];
    if (i < n) off[i + 1] = run;
  }
  if (threadIdx.x == 0) {
    int64_t tot = 0, z = 0;
    for (int q = 0; q < 16; ++q) { tot += wpart[q]; z += wnz[q]; }
    bs[blockIdx.x] = tot;
    bs[nblk + blockIdx.x] = z;
  }
}

__global__ __launch_bounds__(1024) void k_ds_decide0(int64_t* __restrict__ off, long long* __restrict__ c,
                                                     int64_t* __restrict__ bs, int nblk, int64_t c_bound) {
  if (c[0]) return;
  __shared__ int64_t part[16];
  __shared__ int64_t carry, gz;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) { carry = 0; gz = 0; off[0] = 0; }
  __syncthreads();
  for (int q0 = 0; q0 < nblk; q0 += 1024) {
    const int q = q0 + threadIdx.x;
    const int64_t v = q < nblk ? bs[q] : 0;
    const int64_t z = q < nblk ? bs[nblk + q] : 0;
    // 64-bit inclusive scan by shuffles (block totals can pass 2^31 only in theory; cheap here)
    int64_t incl = v;
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    int64_t zs = z;
    for (int d = 32; d > 0; d >>= 1) zs += __shfl_xor(zs, d, 64);
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < wv; ++k) before += part[k];
    if (q < nblk) bs[2 * nblk + q] = before + incl - v;     // exclusive block base
    if (lane == 0) atomicAdd((unsigned long long*)&gz, (unsigned long long)zs);
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const int64_t C = carry;
  c[40] = C;
  c[72] = gz;
  if (C == 0) { c[7] = 1; c[0] = 1; return; }
  if (C > c_bound) { c[5] = 1; c[0] = 1; return; }
  c[1] = 1; c[2] = C; c[3] = C; c[9] = C;
}

__global__ __launch_bounds__(1024) void k_ds_add(int64_t* __restrict__ off, const long long* __restrict__ c,
                                                 const int64_t* __restrict__ bs, int nblk) {
  // after k_ds_decide0: a multi / empty level 0 (c[0] set) is regenerated or ends, its
  // offsets unused; c[8] and the block bases are final either way
  if (c[4]) return;                                     // n past the buffers' bound: nothing ran
  const int64_t n = c[8];
  const int64_t b0 = (int64_t)blockIdx.x * kDsBlk;
  if (b0 >= n || blockIdx.x == 0) return;               // block 0's base is 0
  const int64_t base = bs[2 * nblk + blockIdx.x];
  for (int k = threadIdx.x; k < kDsBlk; k += 1024) {
    const int64_t i = b0 + k;
    if (i < n) off[i + 1] += base;
  }
}

// used items of level 0's candidate rows (LDS-privatised, one global atomicOr per word);
// w32: the bitset's u32 words in use ((F1 + 31) / 32)
__global__ __launch_bounds__(256) void k_dl_mark(const int32_t* __restrict__ rows, int m1,
                                                 long long* __restrict__ c, int w32) {
  __shared__ uint32_t lb[2 * kDlBitsW];
  if (c[0] && !c[5]) return;         // (a multi level still reports its used items)
  for (int q = threadIdx.x; q < w32; q += 256) lb[q] = 0u;
  __syncthreads();
  const int64_t n = c[5] ? 0 : c[40] * (int64_t)m1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicOr(&lb[rows[i] >> 5], 1u << (rows[i] & 31));
  __syncthreads();
  uint32_t* mk = reinterpret_cast<uint32_t*>(c + kDlBits);
  for (int q = threadIdx.x; q < w32; q += 256)
    if (lb[q]) atomicOr(&mk[q], lb[q]);
}

// n_used, and whether level 0 alone exceeds one accumulator pass
__global__ __launch_bounds__(64) void k_dl_post0(long long* __restrict__ c, double lds, double accb, int w32,
                                                  int capmax) {
  if (blockIdx.x != 0) return;
  const uint32_t* mk = reinterpret_cast<const uint32_t*>(c + kDlBits);
  uint32_t part = 0;
  for (int q = threadIdx.x; q < w32; q += 64) part += __popc(mk[q]);
  const int64_t n_used = (int64_t)wave_sum_u32(part);
  if (threadIdx.x != 0) return;
  c[6] = n_used;
  if (c[1] == 1 && c[40] > d_slab_cap(n_used, c[40], lds, accb, capmax)) { c[5] = 1; c[0] = 1; }
}

// acceptance of speculative level l >= 1 (same rule as k_agd_scan_decide, with the
// exact one-pass test total + C <= slab capacity(n_used, total + C))
__global__ __launch_bounds__(1024) void k_dl_decide(const int32_t* __restrict__ cnt, int64_t* __restrict__ off,
                                                     long long* __restrict__ c, int l, double growth, int64_t c_bound,
                                                     double lds, double accb, int capmax) {
  if (c[0]) return;
  int64_t g = 0;
  const int64_t C = agd_block_scan(cnt, off, c[8 + l], &g);
  if (threadIdx.x != 0) return;
  const int64_t total = c[2], last = c[3];
  if (C == 0 || (double)C > growth * (double)last || C > c_bound ||
      total + C > d_slab_cap(c[6], total + C, lds, accb, capmax)) {
    c[0] = 1;
    // no candidates even from the previous level's candidates (a superset of its
    // frequent rows): the mining ends with this bundle (the host skips the next one)
    if (C == 0) c[kDlEmpty] = 1;
    return;
  }
  c[40 + l] = C;
  c[72 + l] = g;
  c[1] = l + 1;
  c[2] = total + C;
  c[3] = C;
  c[8 + l + 1] = C;
}

// Speculative level l >= 2 of a device bundle with the next level's structures fused
// in.  Level l+1's parent rows are level l's candidates (x, y): the candidates of one
// parent row x are contiguous and form exactly one class of level l+1 (its first m
// items are x), starting at off[i].  So the class's Ext bitset is the parent's own
// extension bits a[] and its hash-table entry is hash(x) -> off[i]: the emit pass of
// level l writes both (no insert / ext kernels, no Ext clear: only class starts are
// ever looked up), and the count pass clears level l+1's hash table (ntab, ncap
// entries) while it runs.  kEmit = false: cnt[i] = extensions of row i (+ the clear);
// true: ext ids at cnt + n + off[i], candidate rows at rows + off[i] * (m + 1), and
// level l+1's Ext / table (next_ext, ntab; nullptr when no level follows).
template <bool kEmit, int NWL = 1>
__global__ __launch_bounds__(256) void k_dl_rows(const int32_t* __restrict__ P, int m,
                                                 const int32_t* __restrict__ table, uint32_t mask, int nw,
                                                 const unsigned long long* __restrict__ ext, int32_t* __restrict__ cnt,
                                                 const int64_t* __restrict__ off, int32_t* __restrict__ rows,
                                                 const long long* __restrict__ c, int l, int32_t* __restrict__ ntab,
                                                 uint32_t ncap, unsigned long long* __restrict__ next_ext) {
  if (c[0]) return;
  const int64_t n = c[8 + l];
  if (!kEmit && ntab) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < (int64_t)ncap; q += stride) ntab[q] = -1;
  }
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += nwave) {
    unsigned long long a[NWL];
    const int cc = ag_row_bits<NWL>(P, i, m, table, mask, nw, ext, lane, a);
    const int incl = wave_scan_incl_dpp(cc);
    if (!kEmit) {
      if (lane == 63) cnt[i] = incl;
      continue;
    }
    const int64_t o = off[i];
    ag_emit<NWL>(a, lane, P + i * m, m, o + (incl - cc), cnt + n, rows);
    if (next_ext && wave_last(incl) > 0) {
#pragma unroll
      for (int j = 0; j < NWL; ++j)
        if (lane * NWL + j < nw) next_ext[o * nw + lane * NWL + j] = a[j];
      if (lane == 0) {
        // = ag_hash_drop(candidate row (x, y), m + 1, m): x's items, seed m
        const int32_t* x = P + i * m;
        uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)m;
        for (int q = 0; q < m; ++q) h = ag_mix(h ^ (uint32_t)x[q]);
        uint32_t at = (uint32_t)h & (ncap - 1);
        while (atomicCAS(&ntab[at], -1, (int32_t)o) != -1) at = (at + 1) & (ncap - 1);
      }
    }
  }
}

}  // namespace fa

// Slab capacity rule of the device bundles (d_slab_cap capmax), set by
// fastapriori_amd.ops.primitives before a bundle is generated (TUNING.slab_cap_max)
static int g_cap_max = 0;
FA_API void fa_hip_set_cap_max(int on) { g_cap_max = on; }

// Level 0 of a device bundle: candidates of F_{k-1} = P0 [n][m0] (device; n from
// n_src[0] when given, else n_const; n_bound >= n sizes the buffers), generated
// into the front of ws; with sync, ONE synchronisation copies ctl to ctl_host
// (without it the caller queues fa_hip_dl_more and reads everything once).
// c_bound: the largest C_0 the level may have (one accumulator pass); a larger
// level is reported as multi (ctl[5]) without its rows.  lds: LDS bytes the slab
// kernel has for slab + accumulators; accb: bytes per accumulator (4, or 2: u16).  info (int64 out): 0 ws bytes used,
// 1 cnt (ext ids at cnt + n), 2 off, 3 candidate rows [C_0][m0 + 1].
// Returns 0, 1 (bad arguments) or 5 (ws too small: info[0] = bytes needed).
FA_API int fa_hip_dl_level0(const int32_t* P0, const long long* n_src, int64_t n_const, int64_t n_bound, int m0,
                            int F1, void* ws, int64_t ws_bytes, long long* ctl, long long* ctl_host,
                            int64_t c_bound, double lds, double accb, int64_t* info, int sync, hipStream_t st) {
  if (m0 < 2 || F1 > kAgMaxF1 || F1 < 1 || n_bound < 0 || c_bound < 1) return 1;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  const int nw = (F1 + 63) / 64;
  const int64_t nb = std::max<int64_t>(n_bound, 1);
  uint32_t cap = 16;
  while (cap < 2 * (uint64_t)nb) cap <<= 1;
  const int nds = nb > 4 * kDsBlk ? (int)((nb + kDsBlk - 1) / kDsBlk) : 0;   // multi-workgroup scan blocks
  const int64_t need = al(4 * (int64_t)cap) + al(8 * nb * nw) + al(8 * (nb + 1)) + al(4 * (nb + c_bound)) +
                       al(4 * c_bound * (m0 + 1)) + al(8 * 3 * (int64_t)nds);
  info[0] = need;
  if (need > ws_bytes) return 5;
  char* w = static_cast<char*>(ws);
  int32_t* table = reinterpret_cast<int32_t*>(w); w += al(4 * (int64_t)cap);
  unsigned long long* ext = reinterpret_cast<unsigned long long*>(w); w += al(8 * nb * nw);
  int64_t* off = reinterpret_cast<int64_t*>(w); w += al(8 * (nb + 1));
  int32_t* cnt = reinterpret_cast<int32_t*>(w); w += al(4 * (nb + c_bound));
  int32_t* rows = reinterpret_cast<int32_t*>(w); w += al(4 * c_bound * (m0 + 1));
  int64_t* ds = reinterpret_cast<int64_t*>(w);
  info[1] = (int64_t)(intptr_t)cnt; info[2] = (int64_t)(intptr_t)off; info[3] = (int64_t)(intptr_t)rows;
  hipLaunchKernelGGL(k_dl_setup0, dim3(1), dim3(kDlCtl), 0, st, ctl, n_src, n_const, m0 + 1, nb);
  AgdClear clr{};
  clr.p[0] = reinterpret_cast<uint32_t*>(table); clr.len[0] = cap; clr.val[0] = ~0u;
  clr.p[1] = reinterpret_cast<uint32_t*>(ext); clr.len[1] = 2 * nb * nw; clr.val[1] = 0u;
  clr.nreg = 2;
  const int64_t clr_max = std::max<int64_t>(cap, 2 * nb * nw);
  hipLaunchKernelGGL(k_agd_clear, dim3((unsigned)std::min<int64_t>((clr_max + 255) / 256, 1024)), dim3(256), 0, st,
                     clr, ctl);
  const dim3 g((unsigned)std::min<int64_t>((nb + 255) / 256, 512));
  hipLaunchKernelGGL(k_agd_insert, g, dim3(256), 0, st, P0, m0, table, cap - 1, ctl, 0);
  hipLaunchKernelGGL(k_agd_ext, g, dim3(256), 0, st, P0, m0, table, cap - 1, nw, ext, ctl, 0);
  const unsigned nwg = (unsigned)std::min<int64_t>((nb + 3) / 4, 2048);
#define FA_DL0_ROWS(E, N)                                                                                   \
  hipLaunchKernelGGL((k_agd_rows<E, N>), dim3(nwg), dim3(256), 0, st, P0, m0, table, cap - 1, nw, ext, cnt, off, \
                     rows, ctl, 0);
#define FA_DL0_CNT(N) FA_DL0_ROWS(false, N)
#define FA_DL0_EMIT(N) FA_DL0_ROWS(true, N)
  FA_AG_NWL_SWITCH(nw, FA_DL0_CNT)
  if (nds) {
    hipLaunchKernelGGL(k_ds_blocks, dim3((unsigned)nds), dim3(1024), 0, st, cnt, off, ctl, ds, nds);
    hipLaunchKernelGGL(k_ds_decide0, dim3(1), dim3(1024), 0, st, off, ctl, ds, nds, c_bound);
    hipLaunchKernelGGL(k_ds_add, dim3((unsigned)nds), dim3(1024), 0, st, off, ctl, ds, nds);
  } else {
    hipLaunchKernelGGL(k_dl_decide0, dim3(1), dim3(1024), 0, st, cnt, off, ctl, c_bound);
  }
  FA_AG_NWL_SWITCH(nw, FA_DL0_EMIT)
#undef FA_DL0_EMIT
#undef FA_DL0_CNT
#undef FA_DL0_ROWS
  const int w32 = (F1 + 31) / 32;
  hipLaunchKernelGGL(k_dl_mark, dim3((unsigned)std::min<int64_t>((c_bound * (m0 + 1) + 255) / 256, 1024)), dim3(256),
                     0, st, rows, m0 + 1, ctl, w32);
  hipLaunchKernelGGL(k_dl_post0, dim3(1), dim3(64), 0, st, ctl, lds, accb, w32, g_cap_max);
  if (sync) {
    (void)hipMemcpyAsync(ctl_host, ctl, sizeof(long long) * kDlCtl, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return 7;
  }
  FA_LAUNCH_RET();
}

// Speculative levels 1 .. max_levels-1 of a device bundle, queued right after
// fa_hip_dl_level0 (with or without its synchronisation): batches of kAgdBatch
// levels sized by bounds (n_1 <= n1_bound), each followed by an asynchronous copy of
// the control block into one of two pinned mirrors.  The next batch is queued
// before the host waits on the previous one, so the GPU does not idle while the
// host reads a batch's acceptance; levels of a stopped chain exit at once.  One
// final synchronisation copies ctl to ctl_host.  ws + ws_used is free; desc (int64
// [32][8], host) holds level 0's pointers and m on entry (rows 0..3 and 4) and
// receives every accepted level l:
//   0 parent rows P_l  1 cnt (ext ids at cnt + n_l)  2 off  3 candidate rows
//   4 m_l (parent row length)  5 n_l  6 C_l  7 base (candidates of levels < l)
// Returns 0 (ctl_host[1] = accepted levels incl. level 0), 5 (ws too small:
// info[0] = bytes needed) or 7.
//
// post (optional, host DlPost): right after the synchronisation, with no return to
// the host interpreter in between, the bundle's device piece plan is queued
// (levels.hip fa_hip_dl_plan), the transaction-trimming decision is taken
// (FastApriori._trim_worth_it, the same binomial estimate), and when no trim is
// due the slab count itself is queued (count.hip fa_hip_count_slab_rec): the GPU
// then counts while the host does its bookkeeping.  post->done: 0 nothing queued
// (stopped chain, multi-pass level, buffers too small), 1 planned (the caller trims,
// then counts), 2 planned and counted into post->out.
struct DlPost {
  // plan buffers (grow-only, the caller's): item_map int32 [F1], rec int4 [3 * rec_cap],
  // part int32 [part_cap], out uint32 [out_cap]
  int32_t* item_map; void* rec; int32_t* part; uint32_t* out;
  int64_t rec_cap, part_cap, out_cap;
  // the count's rows and LDS budget
  const int64_t* roff; const int32_t* ranks; const int32_t* src; const int32_t* wword;
  int64_t ncols; double lds_kernel; double lds_budget;
  // trimming decision (trim_ok = 0: never): c1 int64 [F1] item supports, alive uint8 [F1],
  // len_hist int64 [256] (nullptr: decided by the caller), T rows, nnz, min rows, level k
  const int64_t* c1; const uint8_t* alive; const int64_t* len_hist;
  int64_t T, nnz, trim_min_rows, trim_ok, k;
  // out
  int64_t done, sw, cap, n_wg, C, trim;
  // prefix slab rows of levels with prefixes past 12 ids (levels.hip gpre), int32 [gpre_cap]
  int32_t* gpre; int64_t gpre_cap;
  // LDS bytes per accumulator: 4, or 2 (unit weights: count.hip's packed u16 counters)
  double accb;
  // trim when the estimate keeps fewer than this share of the rows, or of the items
  // (FastApriori._trim_worth_it, TUNING.trim_rows_frac / trim_nnz_frac)
  double trim_rows_frac, trim_nnz_frac;
};
static_assert(sizeof(DlPost) == 33 * 8, "DlPost layout (ops.primitives.DlPostC)");

FA_API int fa_hip_dl_plan(const int64_t* desc, int L, long long* ctl, int F1, int32_t* item_map, void* rec,
                          int64_t max_pieces, int32_t* part, int64_t part_cap, int32_t* gpre, int64_t gpre_cap,
                          int sw, hipStream_t st);
FA_API int fa_hip_count_slab_rec_cls(const int64_t* roff, const int32_t* ranks, const int32_t* src, int64_t ncols,
                                     const int32_t* item_map, int F1, int n_used, const int32_t* gpre,
                                     const void* rec, int G, int C, const int32_t* wword, uint32_t* out, int sw,
                                     int n_wg, const uint64_t* bm, int64_t Wp, hipStream_t st,
                                     const int32_t* bm_rows, const int32_t* g_dev, int cls);

// P[Binom(L, p) >= k] (the regularised incomplete beta of FastApriori._trim_worth_it)
static double binom_tail(int L, double p, int k) {
  if (L < k) return 0.0;
  if (p <= 0.0) return k <= 0 ? 1.0 : 0.0;
  if (p >= 1.0) return 1.0;
  double pmf = std::pow(1.0 - p, (double)L), below = 0.0;
  const double r = p / (1.0 - p);
  for (int i = 0; i < k; ++i) {
    below += pmf;
    pmf *= (double)(L - i) / (double)(i + 1) * r;
  }
  return std::min(1.0, std::max(0.0, 1.0 - below));
}

static void dl_post(DlPost* P, const int64_t* desc, int L, long long* ctl, const long long* ch, int F1,
                    hipStream_t st) {
  P->done = 0;
  if (ch[0] && ch[1] == 0) return;                 // nothing accepted
  if (ch[4] || ch[5] || ch[7] || L < 1) return;    // bound error, multi-pass level, end of mining
  int64_t C = 0, R = 0;
  for (int l = 0; l < L; ++l) { C += desc[8 * l + 6]; R += desc[8 * l + 5]; }
  const int64_t n_used = ch[6];
  P->C = C;
  if (C < 1 || C > P->rec_cap || C > P->out_cap || 8 * ((R + 255) / 256) > P->part_cap) return;
  // slab width: plan.cpp slab_width order, one accumulator pass
  int sw = 0;
  int64_t cap = 0;
  for (int w : {16, 32, 8, 4}) {
    cap = (int64_t)((P->lds_budget - (double)n_used * (w + 2) * 8) / P->accb);
    const bool fits = g_cap_max ? cap >= C && (w != 4 || cap >= 1024)
                                : cap >= std::min<int64_t>(C, 8192) || (w == 4 && cap >= 1024);
    if (fits) { sw = w; break; }
  }
  if (sw == 0 || C > cap) return;
  if (fa_hip_dl_plan(desc, L, ctl, F1, P->item_map, P->rec, C, P->part, P->part_cap, P->gpre, P->gpre_cap, sw,
                     st) != 0)
    return;                                        // (e.g. long prefixes past gpre_cap: the caller plans)
  (void)hipMemsetAsync(P->out, 0, 4 * (size_t)C, st);
  P->sw = sw;
  P->cap = cap;
  P->done = 1;
  // trimming before level k: the rows that keep >= k of the bundle's items
  P->trim = 0;
  if (!P->trim_ok || P->T <= 0) {
    // no trimming
  } else if (!P->len_hist || P->T < P->trim_min_rows) {
    if (!P->len_hist && P->T >= P->trim_min_rows) return;   // the caller decides (and counts)
  } else {
    const uint64_t* mk = reinterpret_cast<const uint64_t*>(ch + kDlBits);
    double num = 0.0, den = 0.0;
    for (int r = 0; r < F1; ++r) {
      if (P->alive[r]) den += (double)P->c1[r];
      if ((mk[r >> 6] >> (r & 63)) & 1ull) num += (double)P->c1[r];
    }
    if (den > 0.0) {
      const double p = num / den;
      double est_rows = 0.0, est_nnz = 0.0;
      for (int Lr = 0; Lr < 256; ++Lr) {
        const double h = (double)P->len_hist[Lr];
        if (h == 0.0) continue;
        est_rows += h * binom_tail(Lr, p, (int)P->k);
        est_nnz += h * Lr * p;
      }
      const double T = (double)std::max<int64_t>(P->T, 1), nnz = (double)std::max<int64_t>(P->nnz, 1);
      P->trim = (est_rows < P->trim_rows_frac * T || est_nnz < P->trim_nnz_frac * nnz) ? 1 : 0;
    }
  }
  if (P->trim) return;                                      // the caller trims, then counts
  const int64_t W = (P->ncols + 63) / 64, nslabs = (W + sw - 1) / sw;
  const int64_t map_b = F1 <= 8192 ? (((int64_t)F1 * 2 + 15) & ~(int64_t)15) : 0;
  const bool acc16 = P->accb == 2.0 && !P->wword;
  const int64_t nacc = acc16 ? (C + 1) / 2 : C;
  const int64_t lds_k = n_used * (sw + 2) * 8 + ((nacc + 3) & ~(int64_t)3) * 4 + map_b;
  const int64_t per_cu = std::min<int64_t>(std::max<int64_t>(1, (int64_t)P->lds_kernel / std::max<int64_t>(lds_k, 1)), 2);
  P->n_wg = std::max<int64_t>(1, std::min<int64_t>(nslabs, 256 * per_cu));
  if (fa_hip_count_slab_rec_cls(P->roff, P->ranks, P->src, P->ncols, P->item_map, F1, (int)n_used, P->gpre, P->rec,
                                0, (int)C, P->wword, P->out, sw, (int)P->n_wg, nullptr, 0, st, nullptr,
                                reinterpret_cast<const int32_t*>(ctl + 221), acc16 ? 4 : 0) != 0)
    return;
  P->done = 2;
}

FA_API int fa_hip_dl_more(int F1, void* ws, int64_t ws_bytes, int64_t ws_used, long long* ctl, long long* ctl_host,
                          double growth, int max_levels, double lds, double accb, int64_t n1_bound, int64_t* desc,
                          int64_t* info,
                          hipStream_t st, void* post) {
  using namespace fa;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  const int nw = (F1 + 63) / 64;
  char* const w0 = static_cast<char*>(ws);
  char* w = w0 + ws_used;
  const int LM = std::min(max_levels, 31);
  const int64_t acc_max = (int64_t)(lds / accb);
  int64_t nb = n1_bound;
  int m = (int)desc[4] + 1;
  const int32_t* P = reinterpret_cast<const int32_t*>((intptr_t)desc[3]);
  struct Lv { int32_t* cnt; int64_t* off; int32_t* rows; int m; };
  Lv lv[32];
  // two pinned mirrors of the control block and their events (allocated once)
  static long long* mirror = nullptr;
  static hipEvent_t ev[2];
  if (!mirror) {
    if (hipHostMalloc(reinterpret_cast<void**>(&mirror), 2 * sizeof(long long) * kDlCtl) != hipSuccess) return 7;
    for (int k = 0; k < 2; ++k) (void)hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
  }
  int nbatch = 0;
  // level l's hash table and Ext bitsets; for l >= 2 allocated while enqueuing level
  // l - 1, whose emit pass fills them (k_dl_rows)
  struct Tab { int32_t* table = nullptr; uint32_t cap = 0; unsigned long long* ext = nullptr; };
  Tab cur;
  auto tab_alloc = [&](int64_t rows, Tab& t) -> bool {
    uint32_t cap = 16;
    while (cap < 2 * (uint64_t)rows) cap <<= 1;
    const int64_t need = al(4 * (int64_t)cap) + al(8 * rows * nw);
    if ((w - w0) + need > ws_bytes) { info[0] = 2 * ((w - w0) + need); return false; }
    t.table = reinterpret_cast<int32_t*>(w); w += al(4 * (int64_t)cap);
    t.ext = reinterpret_cast<unsigned long long*>(w); w += al(8 * rows * nw);
    t.cap = cap;
    return true;
  };
  auto enqueue = [&](int l0) -> int {
    const int l1 = std::min(LM - 1, l0 + kAgdBatch - 1);
    for (int l = l0; l <= l1; ++l) {
      const int64_t cb = std::min<int64_t>(acc_max, (int64_t)(growth * (double)nb) + 1);
      if (l == 1) {
        // level 1's parents are level 0's candidates, emitted by fa_hip_dl_level0: its
        // table and Ext are built here (clear, insert, ext)
        if (!tab_alloc(nb, cur)) return 5;
        AgdClear clr{};
        clr.p[0] = reinterpret_cast<uint32_t*>(cur.table); clr.len[0] = cur.cap; clr.val[0] = ~0u;
        clr.p[1] = reinterpret_cast<uint32_t*>(cur.ext); clr.len[1] = 2 * nb * nw; clr.val[1] = 0u;
        clr.nreg = 2;
        const int64_t clr_max = std::max<int64_t>(cur.cap, 2 * nb * nw);
        hipLaunchKernelGGL(k_agd_clear, dim3((unsigned)std::min<int64_t>((clr_max + 255) / 256, 1024)), dim3(256), 0,
                           st, clr, ctl);
        const dim3 g((unsigned)std::min<int64_t>((nb + 255) / 256, 512));
        hipLaunchKernelGGL(k_agd_insert, g, dim3(256), 0, st, P, m, cur.table, cur.cap - 1, ctl, l);
        hipLaunchKernelGGL(k_agd_ext, g, dim3(256), 0, st, P, m, cur.table, cur.cap - 1, nw, cur.ext, ctl, l);
      }
      const int64_t need = al(8 * (nb + 1)) + al(4 * (nb + cb)) + al(4 * cb * (m + 1));
      if ((w - w0) + need > ws_bytes) {
        info[0] = 2 * ((w - w0) + need);
        return 5;
      }
      lv[l].off = reinterpret_cast<int64_t*>(w); w += al(8 * (nb + 1));
      lv[l].cnt = reinterpret_cast<int32_t*>(w); w += al(4 * (nb + cb));
      lv[l].rows = reinterpret_cast<int32_t*>(w); w += al(4 * cb * (m + 1));
      lv[l].m = m;
      Tab nxt;
      if (l + 1 < LM && !tab_alloc(cb, nxt)) return 5;
      const unsigned nwg = (unsigned)std::min<int64_t>((nb + 3) / 4, 2048);
#define FA_DLR(E, N)                                                                                          \
      hipLaunchKernelGGL((k_dl_rows<E, N>), dim3(nwg), dim3(256), 0, st, P, m, cur.table, cur.cap - 1, nw,      \
                         cur.ext, lv[l].cnt, lv[l].off, lv[l].rows, ctl, l, nxt.table, nxt.cap, nxt.ext);
#define FA_DLR_CNT(N) FA_DLR(false, N)
#define FA_DLR_EMIT(N) FA_DLR(true, N)
      FA_AG_NWL_SWITCH(nw, FA_DLR_CNT)
      hipLaunchKernelGGL(k_dl_decide, dim3(1), dim3(1024), 0, st, lv[l].cnt, lv[l].off, ctl, l, growth, cb, lds, accb,
                         g_cap_max);
      FA_AG_NWL_SWITCH(nw, FA_DLR_EMIT)
#undef FA_DLR_EMIT
#undef FA_DLR_CNT
#undef FA_DLR
      P = lv[l].rows;
      cur = nxt;
      nb = cb;
      ++m;
    }
    long long* hb = mirror + (nbatch & 1) * kDlCtl;
    (void)hipMemcpyAsync(hb, ctl, sizeof(long long) * kDlCtl, hipMemcpyDeviceToHost, st);
    (void)hipEventRecord(ev[nbatch & 1], st);
    ++nbatch;
    return 0;
  };
  int next = 1;                 // first level of the next batch to queue
  int rc = 0;
  for (int q = 0; q < 2 && next < LM && rc == 0; ++q, next += kAgdBatch) rc = enqueue(next);
  for (int waited = 0; rc == 0 && waited < nbatch; ++waited) {
    if (hipEventSynchronize(ev[waited & 1]) != hipSuccess) return 7;
    if (mirror[(waited & 1) * kDlCtl]) break;                     // the chain stopped
    if (next < LM) { rc = enqueue(next); next += kAgdBatch; }     // keep one batch ahead
  }
  (void)hipMemcpyAsync(ctl_host, ctl, sizeof(long long) * kDlCtl, hipMemcpyDeviceToHost, st);
  if (hipStreamSynchronize(st) != hipSuccess) return 7;
  if (rc) return rc;
  desc[5] = ctl_host[8];
  desc[6] = ctl_host[40];
  desc[7] = 0;
  const int L = (int)ctl_host[1];
  int64_t base = desc[6];
  for (int l = 1; l < L; ++l) {
    int64_t* d = desc + 8 * l;
    d[0] = desc[8 * (l - 1) + 3];
    d[1] = (int64_t)(intptr_t)lv[l].cnt;
    d[2] = (int64_t)(intptr_t)lv[l].off;
    d[3] = (int64_t)(intptr_t)lv[l].rows;
    d[4] = lv[l].m;
    d[5] = ctl_host[8 + l];
    d[6] = ctl_host[40 + l];
    d[7] = base;
    base += d[6];
  }
  info[0] = w - w0;
  if (post) dl_post(static_cast<DlPost*>(post), desc, L, ctl, ctl_host, F1, st);
  FA_LAUNCH_RET();
}
