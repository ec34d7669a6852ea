// Device-side parsing of a transaction file's bytes (numeric and dictionary vocabularies).
//
// Same input semantics as the host parser (csrc/host/parse.cpp, Utils.scala:19-27):
//   * lines end at '\n', at '\r\n' or at a lone '\r' (Hadoop LineRecordReader);
//   * each line -> trim() (bytes <= 0x20) -> split on [ \t\x0B\f]+; a blank line
//     is the single token "" (id 0);
//   * numeric ids: id = value + 1 for canonical decimals "0" | [1-9][0-9]* with
//     value <= 2^31 - 2; any other token raises the `bad` flag and the caller
//     re-parses the shard on the host (dictionary mode);
//   * ids inside one line are distinct, in first-occurrence order; every
//     repeated occurrence goes to `extras` (F1 counts occurrences).
//
// Pipeline (the file's bytes are already in HBM, padded to 64 + a multiple of 64):
//   k_line_count  16 KB tiles, 64 bytes per thread (4 x 16-byte loads): line ends per tile
//   k_line_ends   same tiles; block scan of per-thread counts -> position of every line end
//   k_parse_lines one thread per line: trim, tokenise, validate, de-duplicate (the first
//                 64 distinct ids in a per-thread LDS column, the rest re-read from the
//                 thread's own output), write into an upper-bound slot of (len + 1) / 2 ids
//   k_compact     one thread per line: copy ids and extras to their scanned offsets
#include "fa_hip.h"

namespace fa {

constexpr int kLT = 256;              // threads per line-scan block
constexpr int kLB = 64;               // bytes per thread
constexpr int kLTile = kLT * kLB;     // 16 KB
constexpr int kPT = 128;              // threads per parse block
constexpr int kSeen = 64;             // distinct ids kept in LDS per thread

__device__ __forceinline__ bool is_term_at(const uint8_t* __restrict__ buf, int64_t n, int64_t i, uint32_t c) {
  return c == '\n' || (c == '\r' && (i + 1 >= n || buf[i + 1] != '\n'));
}

// Line ends among this thread's 64 bytes: count (mode 0) or write (mode 1).
template <int MODE>
__device__ __forceinline__ int scan_bytes(const uint8_t* __restrict__ buf, int64_t n, int64_t base,
                                          int64_t* __restrict__ out) {
  int cnt = 0;
  if (base >= n) return 0;
  const uint4* p = reinterpret_cast<const uint4*>(buf + base);
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const uint4 w = p[v];
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t x = ws[q];
      // any '\n' (0x0a) or '\r' (0x0d) byte in this dword?  (zero-byte test on x ^ pattern)
      const uint32_t a = x ^ 0x0a0a0a0au, b = x ^ 0x0d0d0d0du;
      const uint32_t za = (a - 0x01010101u) & ~a & 0x80808080u;
      const uint32_t zb = (b - 0x01010101u) & ~b & 0x80808080u;
      if (!(za | zb)) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = base + v * 16 + q * 4 + k;
        const uint32_t c = (x >> (8 * k)) & 0xffu;
        if (i < n && is_term_at(buf, n, i, c)) {
          if (MODE == 1) out[cnt] = i;
          ++cnt;
        }
      }
    }
  }
  return cnt;
}

__global__ __launch_bounds__(kLT) void k_line_count(const uint8_t* __restrict__ buf, int64_t n,
                                                    int32_t* __restrict__ tile_cnt) {
  __shared__ int part[kLT / kWave];
  const int64_t base = (int64_t)blockIdx.x * kLTile + (int64_t)threadIdx.x * kLB;
  const uint32_t c = wave_sum_u32((uint32_t)scan_bytes<0>(buf, n, base, nullptr));
  if (lane_id() == 0) part[threadIdx.x >> 6] = (int)c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kLT / kWave; ++w) t += part[w];
    tile_cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kLT) void k_line_ends(const uint8_t* __restrict__ buf, int64_t n,
                                                   const int64_t* __restrict__ tile_base,
                                                   int64_t* __restrict__ ends) {
  __shared__ int part[kLT / kWave];
  const int64_t base = (int64_t)blockIdx.x * kLTile + (int64_t)threadIdx.x * kLB;
  const int mine = scan_bytes<0>(buf, n, base, nullptr);
  const int incl = wave_scan_incl_dpp(mine);
  if (lane_id() == 63) part[threadIdx.x >> 6] = incl;
  __syncthreads();
  int before = 0;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) before += part[w];
  if (mine) scan_bytes<1>(buf, n, base, ends + tile_base[blockIdx.x] + before + incl - mine);
}

// One thread per line.  bound_off[j]: first slot of line j in scratch/xscratch
// (room for (len + 1) / 2 ids, >= 1).  flags[0] |= 1 on a non-numeric token,
// flags[1] = max id.
__global__ __launch_bounds__(kPT) void k_parse_lines(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ ends, int64_t nl,
    const int64_t* __restrict__ bound_off, int32_t* __restrict__ scratch, int32_t* __restrict__ xscratch,
    int32_t* __restrict__ dcnt, int32_t* __restrict__ xcnt, int32_t* __restrict__ flags) {
  __shared__ int32_t seen[kSeen * kPT];      // column per thread: conflict-free
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * kPT + tid;
  int32_t mx = 0;
  bool bad = false;
  if (j < nl) {
    int64_t s = j ? ends[j - 1] + 1 : 0;
    int64_t e = ends[j];
    while (s < e && buf[s] <= 0x20) ++s;
    while (e > s && buf[e - 1] <= 0x20) --e;
    const int64_t bo = bound_off[j];
    int D = 0, X = 0;
    if (s == e) {
      scratch[bo] = 0;     // blank line: the single token ""
      D = 1;
    } else {
      uint64_t v = 0;
      int nd = 0;
      bool lead0 = false;
      for (int64_t i = s; i <= e; ++i) {
        const uint32_t c = i < e ? buf[i] : (uint32_t)' ';
        const uint32_t dg = c - '0';
        if (dg <= 9) {
          if (nd == 0) { v = 0; lead0 = dg == 0; }
          v = v * 10 + dg;
          if (++nd > 10) { bad = true; break; }
          continue;
        }
        if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
          if (nd) {
            if ((lead0 && nd > 1) || v > 2147483646ull) { bad = true; break; }
            const int32_t id = (int32_t)(v + 1);
            bool dup = false;
            const int lim = D < kSeen ? D : kSeen;
            for (int q = 0; q < lim && !dup; ++q) dup = seen[q * kPT + tid] == id;
            for (int q = kSeen; q < D && !dup; ++q) dup = scratch[bo + q] == id;
            if (dup) {
              xscratch[bo + X++] = id;
            } else {
              if (D < kSeen) seen[D * kPT + tid] = id;
              scratch[bo + D++] = id;
              mx = id > mx ? id : mx;
            }
            nd = 0;
          }
          continue;
        }
        bad = true;   // a byte that is neither digit, separator nor (trimmed) blank
        break;
      }
    }
    dcnt[j] = D;
    xcnt[j] = X;
  }
  // wave-level flag / max (every lane reaches here)
  const unsigned long long anybad = __ballot(bad);
  int32_t m = mx;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int32_t t = __shfl_xor(m, o, 64); m = t > m ? t : m; }
  if (lane_id() == 0) {
    if (anybad) atomicOr(&flags[0], 1);
    if (m > 0) atomicMax(&flags[1], m);
  }
}

__global__ __launch_bounds__(256) void k_compact_lines(
    const int32_t* __restrict__ scratch, const int32_t* __restrict__ xscratch, const int64_t* __restrict__ bound_off,
    const int32_t* __restrict__ dcnt, const int32_t* __restrict__ xcnt, const int64_t* __restrict__ off,
    const int64_t* __restrict__ xoff, int64_t nl, int32_t* __restrict__ items, int32_t* __restrict__ extras) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= nl) return;
  const int64_t bo = bound_off[j];
  const int32_t d = dcnt[j], x = xcnt[j];
  int32_t* dst = items + off[j];
  for (int q = 0; q < d; ++q) dst[q] = scratch[bo + q];
  if (x) {
    int32_t* xd = extras + xoff[j];
    for (int q = 0; q < x; ++q) xd[q] = xscratch[bo + q];
  }
}

// ---------------------------------------------------------------------------
// Dictionary (string) vocabularies on the device.  Same tokenisation; every token
// gets the host parser's 64-bit identity hash (csrc/host/fa_common.h hash_bytes:
// FNV-1a over the bytes, then the splitmix64 finaliser of h ^ length) and is
// inserted into a global open-addressing table keyed by that hash (0 = empty; a
// hash of 0 is stored as 1).  A token's id here is its table slot; k_slot_ids
// turns occupied slots into dense ids (slot order, i.e. hash order) afterwards.
// The slot's (byte offset, length) of one occurrence lets the host decode the
// strings it needs (frequent items) without a dictionary of every token.
// flags[0] |= 2 when a probe sequence exceeds kMaxProbe (table too full), |= 4 when
// k_dict_verify finds two distinct tokens sharing a hash: the caller then falls
// back to the host parser.
// ---------------------------------------------------------------------------
constexpr int kMaxProbe = 256;

__device__ __forceinline__ uint64_t dmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t dict_insert(unsigned long long* __restrict__ keys, int64_t* __restrict__ tpos,
                                               int32_t* __restrict__ tlen, uint32_t mask, uint64_t h, int64_t pos,
                                               int32_t len) {
  if (h == 0) h = 1;
  uint32_t at = (uint32_t)(h >> 20) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {
    const unsigned long long k = keys[at];
    if (k == h) return (int32_t)at;
    if (k == 0) {
      const unsigned long long old = atomicCAS(&keys[at], 0ull, (unsigned long long)h);
      if (old == 0) {
        tpos[at] = pos;
        tlen[at] = len;
        return (int32_t)at;
      }
      if (old == h) return (int32_t)at;
    }
    at = (at + 1) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(kPT) void k_parse_lines_dict(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ ends, int64_t nl,
    const int64_t* __restrict__ bound_off, int32_t* __restrict__ scratch, int32_t* __restrict__ xscratch,
    int32_t* __restrict__ dcnt, int32_t* __restrict__ xcnt, int32_t* __restrict__ flags,
    unsigned long long* __restrict__ keys, int64_t* __restrict__ tpos, int32_t* __restrict__ tlen, uint32_t mask) {
  __shared__ int32_t seen[kSeen * kPT];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * kPT + tid;
  bool full = false;
  if (j < nl) {
    int64_t s = j ? ends[j - 1] + 1 : 0;
    int64_t e = ends[j];
    while (s < e && buf[s] <= 0x20) ++s;
    while (e > s && buf[e - 1] <= 0x20) --e;
    const int64_t bo = bound_off[j];
    int D = 0, X = 0;
    auto add = [&](int64_t ts, int64_t te, uint64_t h) {
      const int32_t id = dict_insert(keys, tpos, tlen, mask, dmix64(h ^ (uint64_t)(te - ts)), ts, (int32_t)(te - ts));
      if (id < 0) { full = true; return; }
      bool dup = false;
      const int lim = D < kSeen ? D : kSeen;
      for (int q = 0; q < lim && !dup; ++q) dup = seen[q * kPT + tid] == id;
      for (int q = kSeen; q < D && !dup; ++q) dup = scratch[bo + q] == id;
      if (dup) {
        xscratch[bo + X++] = id;
      } else {
        if (D < kSeen) seen[D * kPT + tid] = id;
        scratch[bo + D++] = id;
      }
    };
    if (s == e) {
      add(s, s, 0xCBF29CE484222325ull);     // blank line: the single token ""
    } else {
      int64_t ts = -1;
      uint64_t h = 0;
      for (int64_t i = s; i <= e && !full; ++i) {
        const uint32_t c = i < e ? buf[i] : (uint32_t)' ';
        if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
          if (ts >= 0) { add(ts, i, h); ts = -1; }
          continue;
        }
        if (ts < 0) { ts = i; h = 0xCBF29CE484222325ull; }
        h = (h ^ c) * 0x100000001B3ull;
      }
    }
    dcnt[j] = D;
    xcnt[j] = X;
  }
  if (__ballot(full) != 0ull && lane_id() == 0) atomicOr(&flags[0], 2);
}

// Identity check of the table: a slot is keyed by the 64-bit hash alone, so two
// distinct tokens with one hash would share an id.  After k_parse_lines_dict every
// slot's representative (tpos, tlen) is written; this pass re-tokenises every line
// and compares each token's bytes with its slot's representative.  flags[0] |= 4 on
// any difference (the caller then parses the shard on the host, which reports the
// collision as an error, csrc/host/parse.cpp).
__device__ __forceinline__ bool dict_same(const uint8_t* __restrict__ buf, const unsigned long long* __restrict__ keys,
                                          const int64_t* __restrict__ tpos, const int32_t* __restrict__ tlen,
                                          uint32_t mask, uint64_t h, int64_t pos, int32_t len) {
  if (h == 0) h = 1;
  uint32_t at = (uint32_t)(h >> 20) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {
    const unsigned long long k = keys[at];
    if (k == h) {
      if (tlen[at] != len) return false;
      const int64_t q = tpos[at];
      for (int32_t i = 0; i < len; ++i)
        if (buf[q + i] != buf[pos + i]) return false;
      return true;
    }
    if (k == 0) return false;
    at = (at + 1) & mask;
  }
  return false;
}

__global__ __launch_bounds__(kPT) void k_dict_verify(const uint8_t* __restrict__ buf, const int64_t* __restrict__ ends,
                                                     int64_t nl, int32_t* __restrict__ flags,
                                                     const unsigned long long* __restrict__ keys,
                                                     const int64_t* __restrict__ tpos, const int32_t* __restrict__ tlen,
                                                     uint32_t mask) {
  const int64_t j = (int64_t)blockIdx.x * kPT + threadIdx.x;
  bool bad = false;
  if (j < nl) {
    int64_t s = j ? ends[j - 1] + 1 : 0;
    int64_t e = ends[j];
    while (s < e && buf[s] <= 0x20) ++s;
    while (e > s && buf[e - 1] <= 0x20) --e;
    if (s < e) {        // (a blank line's token "" has length 0: nothing to compare)
      int64_t ts = -1;
      uint64_t h = 0;
      for (int64_t i = s; i <= e && !bad; ++i) {
        const uint32_t c = i < e ? buf[i] : (uint32_t)' ';
        if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
          if (ts >= 0) {
            bad = !dict_same(buf, keys, tpos, tlen, mask, dmix64(h ^ (uint64_t)(i - ts)), ts, (int32_t)(i - ts));
            ts = -1;
          }
          continue;
        }
        if (ts < 0) { ts = i; h = 0xCBF29CE484222325ull; }
        h = (h ^ c) * 0x100000001B3ull;
      }
    }
  }
  if (__ballot(bad) != 0ull && lane_id() == 0) atomicOr(&flags[0], 4);
}

// dense id of every occupied slot (exclusive scan of occupancy done by the caller)
__global__ __launch_bounds__(256) void k_slot_remap(int32_t* __restrict__ ids, int64_t n,
                                                    const int32_t* __restrict__ slot_id) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    ids[i] = slot_id[ids[i]];
}

}  // namespace fa

using namespace fa;

FA_API int fa_hip_parse_lines_dict(const uint8_t* buf, const int64_t* ends, int64_t nl, const int64_t* bound_off,
                                   int32_t* scratch, int32_t* xscratch, int32_t* dcnt, int32_t* xcnt,
                                   int32_t* flags, void* keys, int64_t* tpos, int32_t* tlen, int64_t cap,
                                   hipStream_t st) {
  if (nl <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) || cap > ((int64_t)1 << 31)) return 1;
  hipLaunchKernelGGL(k_parse_lines_dict, dim3((unsigned)((nl + kPT - 1) / kPT)), dim3(kPT), 0, st, buf, ends, nl,
                     bound_off, scratch, xscratch, dcnt, xcnt, flags, (unsigned long long*)keys, tpos, tlen,
                     (uint32_t)(cap - 1));
  FA_LAUNCH_RET();
}

FA_API int fa_hip_dict_verify(const uint8_t* buf, const int64_t* ends, int64_t nl, int32_t* flags, const void* keys,
                              const int64_t* tpos, const int32_t* tlen, int64_t cap, hipStream_t st) {
  if (nl <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) || cap > ((int64_t)1 << 31)) return 1;
  hipLaunchKernelGGL(k_dict_verify, dim3((unsigned)((nl + kPT - 1) / kPT)), dim3(kPT), 0, st, buf, ends, nl, flags,
                     (const unsigned long long*)keys, tpos, tlen, (uint32_t)(cap - 1));
  FA_LAUNCH_RET();
}

FA_API int fa_hip_slot_remap(int32_t* ids, int64_t n, const int32_t* slot_id, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_slot_remap, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)), dim3(256), 0, st, ids,
                     n, slot_id);
  FA_LAUNCH_RET();
}

FA_API int64_t fa_hip_parse_tiles(int64_t n) { return (n + kLTile - 1) / kLTile; }

FA_API int fa_hip_line_count(const uint8_t* buf, int64_t n, int32_t* tile_cnt, hipStream_t st) {
  const int64_t tiles = (n + kLTile - 1) / kLTile;
  if (tiles <= 0) return 0;
  if (tiles >= (int64_t)INT32_MAX) return 3;
  hipLaunchKernelGGL(k_line_count, dim3((unsigned)tiles), dim3(kLT), 0, st, buf, n, tile_cnt);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_line_ends(const uint8_t* buf, int64_t n, const int64_t* tile_base, int64_t* ends,
                            hipStream_t st) {
  const int64_t tiles = (n + kLTile - 1) / kLTile;
  if (tiles <= 0) return 0;
  hipLaunchKernelGGL(k_line_ends, dim3((unsigned)tiles), dim3(kLT), 0, st, buf, n, tile_base, ends);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_parse_lines(const uint8_t* buf, const int64_t* ends, int64_t nl, const int64_t* bound_off,
                              int32_t* scratch, int32_t* xscratch, int32_t* dcnt, int32_t* xcnt, int32_t* flags,
                              hipStream_t st) {
  if (nl <= 0) return 0;
  hipLaunchKernelGGL(k_parse_lines, dim3((unsigned)((nl + kPT - 1) / kPT)), dim3(kPT), 0, st, buf, ends, nl,
                     bound_off, scratch, xscratch, dcnt, xcnt, flags);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_compact_lines(const int32_t* scratch, const int32_t* xscratch, const int64_t* bound_off,
                                const int32_t* dcnt, const int32_t* xcnt, const int64_t* off, const int64_t* xoff,
                                int64_t nl, int32_t* items, int32_t* extras, hipStream_t st) {
  if (nl <= 0) return 0;
  hipLaunchKernelGGL(k_compact_lines, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, st, scratch, xscratch,
                     bound_off, dcnt, xcnt, off, xoff, nl, items, extras);
  FA_LAUNCH_RET();
}
