// Transaction-file parser: mmap + multithreaded tokeniser -> CSR of token ids.
//
// Reproduces the reference's input semantics (Utils.scala:19-27):
//   * lines split like Hadoop's LineRecordReader (\n, \r\n or \r);
//   * each line -> trim() -> split("\\s+"); an empty line is the single token "";
//   * a byte range [begin, end) owns exactly the lines that START inside it, so
//     disjoint ranges partition the file (used for one shard per rank).
// Output invariant used by every kernel downstream: the ids inside one
// transaction are DISTINCT.  Repeated tokens of a line are reported separately
// as "extras" (one entry per repeated occurrence) because the reference's F1
// counts occurrences (FastApriori.scala:55) while k>=2 counts sets (:69).
//
// Two id spaces:
//   numeric : every token is a canonical decimal "0" | [1-9][0-9]* <= 2^31-2;
//             id = value + 1, id 0 = the empty token "".  No dictionary needed
//             and ids agree across ranks by construction.
//   dict    : any other vocabulary; per-shard dictionary (id -> bytes) plus a
//             64-bit hash per entry used to agree on identity across ranks.
#include <immintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <unordered_map>

#include "fa_common.h"
#include "txndb.h"

namespace fa {

static inline bool is_sep(uint8_t c) { return c == ' ' || c == '\t' || c == 0x0B || c == '\f'; }

int64_t next_line_start(const char* d, int64_t size, int64_t pos) {
  if (pos <= 0) return 0;
  for (int64_t i = pos - 1; i < size; ++i) {
    char c = d[i];
    if (c == '\n') return i + 1;
    if (c == '\r') return (i + 1 < size && d[i + 1] == '\n') ? i + 2 : i + 1;
  }
  return size;
}

// Calls tok(ptr, len) for every token of the line [ls, le) (terminator excluded).
template <class F>
static inline void for_each_token(const char* d, int64_t ls, int64_t le, F&& tok) {
  while (ls < le && (uint8_t)d[ls] <= 0x20) ++ls;
  while (le > ls && (uint8_t)d[le - 1] <= 0x20) --le;
  if (ls == le) { tok(d + ls, 0); return; }
  int64_t i = ls;
  while (i < le) {
    int64_t s = i;
    while (i < le && !is_sep((uint8_t)d[i])) ++i;
    tok(d + s, i - s);
    while (i < le && is_sep((uint8_t)d[i])) ++i;
  }
}

// Returns id (>=0) for a canonical numeric token, or -1.
static inline int32_t numeric_id(const char* p, int64_t n) {
  if (n == 0) return 0;
  if (n > 10) return -1;
  if (p[0] == '0' && n > 1) return -1;
  uint64_t v = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint8_t c = (uint8_t)p[i] - '0';
    if (c > 9) return -1;
    v = v * 10 + c;
  }
  if (v > 2147483646ull) return -1;
  return (int32_t)(v + 1);
}

// Appends the distinct ids of `line` to items; repeats go to extras.
static inline void emit_distinct(std::vector<int32_t>& line, std::vector<int32_t>& items,
                                 std::vector<int32_t>& extras, std::vector<int32_t>& table) {
  const size_t L = line.size();
  if (L <= 24) {
    for (size_t i = 0; i < L; ++i) {
      bool dup = false;
      for (size_t j = 0; j < i; ++j) if (line[j] == line[i]) { dup = true; break; }
      if (dup) extras.push_back(line[i]); else items.push_back(line[i]);
    }
    return;
  }
  size_t cap = 64;
  while (cap < 2 * L) cap <<= 1;
  table.assign(cap, -1);
  for (size_t i = 0; i < L; ++i) {
    int32_t v = line[i];
    size_t h = (size_t)mix64((uint64_t)(uint32_t)v) & (cap - 1);
    bool dup = false;
    while (table[h] != -1) {
      if (table[h] == v) { dup = true; break; }
      h = (h + 1) & (cap - 1);
    }
    if (dup) { extras.push_back(v); continue; }
    table[h] = v;
    items.push_back(v);
  }
}

struct MappedFile {
  const char* data = nullptr;
  int64_t size = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    size = st.st_size;
    if (size == 0) return true;
    void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (p == MAP_FAILED) return false;
    madvise(p, size, MADV_SEQUENTIAL);
    data = (const char*)p;
    return true;
  }
  ~MappedFile() {
    if (data) munmap((void*)data, size);
    if (fd >= 0) ::close(fd);
  }
};

// Per-thread dictionary: open addressing on the 64-bit token hash (hash_bytes, the
// identity the ranks agree on), verified by the bytes, so a 64-bit collision inside
// a shard is reported (parse error 7) instead of merging two tokens.
struct ThreadDict {
  struct Slot { uint64_t h; int32_t id; int32_t pad; };
  std::vector<Slot> slot;               // id -1 = empty; the hash lives in the slot (one miss per probe)
  std::vector<uint64_t> hash;           // per local id
  std::vector<std::string_view> strs;   // per local id
  bool collision = false;
  ThreadDict() : slot(1 << 12, Slot{0, -1, 0}) {}
  // Identity inside a thread is the 64-bit hash (as across ranks); equal hashes of
  // different tokens are caught by merge_dicts' byte comparison across threads
  // and by the length check here.
  int32_t get(std::string_view s) {
    const uint64_t h = hash_bytes(s.data(), s.size());
    const size_t mask = slot.size() - 1;
    size_t at = (size_t)h & mask;
    for (;;) {
      const Slot& e = slot[at];
      if (e.id < 0) break;
      if (e.h == h) {
        if (strs[(size_t)e.id].size() != s.size()) collision = true;
        return e.id;
      }
      at = (at + 1) & mask;
    }
    const int32_t id = (int32_t)strs.size();
    slot[at] = Slot{h, id, 0};
    hash.push_back(h);
    strs.push_back(s);
    if (strs.size() * 2 > slot.size()) grow();
    return id;
  }
  void grow() {
    std::vector<Slot> ns(slot.size() * 2, Slot{0, -1, 0});
    const size_t mask = ns.size() - 1;
    for (size_t id = 0; id < strs.size(); ++id) {
      size_t at = (size_t)hash[id] & mask;
      while (ns[at].id >= 0) at = (at + 1) & mask;
      ns[at] = Slot{hash[id], (int32_t)id, 0};
    }
    slot.swap(ns);
  }
};

// Merge the thread dictionaries into one shard dictionary in parallel: entries are
// partitioned by the top hash bits, each partition is sorted by hash and gets a
// contiguous id range (ids in hash order: deterministic for any thread count).
// remap[t][local id] = shard id.  Returns false on a 64-bit collision.
static bool merge_dicts(std::vector<ThreadDict>& dicts, int nthreads, TxnDB* db,
                        std::vector<std::vector<int32_t>>& remap) {
  const int nt = (int)dicts.size();
  constexpr int kBits = 8, kB = 1 << kBits;
  struct Ent { uint64_t h; int32_t t, id; };
  std::vector<std::vector<int64_t>> cnt(nt, std::vector<int64_t>(kB + 1, 0));
  parallel_for_threads(std::max(1, std::min(nthreads, nt)), [&](int w) {
    for (int t = w; t < nt; t += std::max(1, std::min(nthreads, nt)))
      for (uint64_t h : dicts[t].hash) cnt[t][(h >> (64 - kBits)) + 1] += 1;
  });
  // bucket-major offsets: bucket b's entries of thread t start at off[b][t]
  std::vector<int64_t> bstart(kB + 1, 0);
  std::vector<std::vector<int64_t>> off(kB, std::vector<int64_t>(nt, 0));
  int64_t o = 0;
  for (int b = 0; b < kB; ++b) {
    bstart[b] = o;
    for (int t = 0; t < nt; ++t) { off[b][t] = o; o += cnt[t][b + 1]; }
  }
  bstart[kB] = o;
  std::vector<Ent> ents((size_t)o);
  parallel_for_threads(std::max(1, std::min(nthreads, nt)), [&](int w) {
    for (int t = w; t < nt; t += std::max(1, std::min(nthreads, nt))) {
      std::vector<int64_t> pos(kB);
      for (int b = 0; b < kB; ++b) pos[b] = off[b][t];
      const auto& H = dicts[t].hash;
      for (size_t id = 0; id < H.size(); ++id) ents[(size_t)pos[H[id] >> (64 - kBits)]++] = {H[id], t, (int32_t)id};
    }
  });
  // per bucket: sort by hash, distinct count
  std::vector<int64_t> nd(kB + 1, 0);
  std::atomic<bool> bad{false};
  parallel_for_threads(std::max(1, nthreads), [&](int w) {
    for (int b = w; b < kB; b += std::max(1, nthreads)) {
      auto* a = ents.data() + bstart[b];
      const int64_t n = bstart[b + 1] - bstart[b];
      std::sort(a, a + n, [](const Ent& x, const Ent& y) { return x.h < y.h || (x.h == y.h && x.t < y.t); });
      int64_t d = 0;
      for (int64_t i = 0; i < n; ++i) {
        if (i == 0 || a[i].h != a[i - 1].h) { ++d; continue; }
        if (dicts[a[i].t].strs[(size_t)a[i].id] != dicts[a[i - 1].t].strs[(size_t)a[i - 1].id]) bad = true;
      }
      nd[b + 1] = d;
    }
  });
  for (auto& td : dicts) if (td.collision) bad = true;
  if (bad) return false;
  for (int b = 0; b < kB; ++b) nd[b + 1] += nd[b];
  const int64_t V = nd[kB];
  remap.assign(nt, {});
  for (int t = 0; t < nt; ++t) remap[t].assign(dicts[t].strs.size(), -1);
  db->dict_off.assign((size_t)V + 1, 0);
  db->dict_hash.assign((size_t)V, 0);
  std::vector<std::string_view> first((size_t)V);
  parallel_for_threads(std::max(1, nthreads), [&](int w) {
    for (int b = w; b < kB; b += std::max(1, nthreads)) {
      const auto* a = ents.data() + bstart[b];
      const int64_t n = bstart[b + 1] - bstart[b];
      int64_t g = nd[b] - 1;
      for (int64_t i = 0; i < n; ++i) {
        if (i == 0 || a[i].h != a[i - 1].h) {
          ++g;
          db->dict_hash[(size_t)g] = a[i].h;
          first[(size_t)g] = dicts[a[i].t].strs[(size_t)a[i].id];
        }
        remap[a[i].t][(size_t)a[i].id] = (int32_t)g;
      }
    }
  });
  int64_t bytes = 0;
  for (int64_t g = 0; g < V; ++g) { db->dict_off[(size_t)g] = bytes; bytes += (int64_t)first[(size_t)g].size(); }
  db->dict_off[(size_t)V] = bytes;
  db->dict_blob.resize((size_t)bytes);
  parallel_for_threads(std::max(1, nthreads), [&](int w) {
    const int nw = std::max(1, nthreads);
    for (int64_t g = V * w / nw, e = V * (w + 1) / nw; g < e; ++g)
      if (!first[(size_t)g].empty())
        std::memcpy(&db->dict_blob[(size_t)db->dict_off[(size_t)g]], first[(size_t)g].data(), first[(size_t)g].size());
  });
  db->vocab = V;
  return true;
}

// Numeric fast path for one line starting at p: a single pass in which digits
// accumulate into the value and separators emit it; ids go straight into
// `items` (duplicates of the line to `extras`).  Returns the position of the
// line terminator, or -1 when the line needs the exact slow path (a byte that
// is neither a digit, a separator nor a terminator: e.g. a trimmed control
// character, or a non-numeric / non-canonical token) -- then nothing was emitted.
static inline int64_t fast_numeric_line(const uint8_t* d, int64_t size, int64_t p, std::vector<int32_t>& items,
                                        std::vector<int32_t>& extras, int32_t& mx) {
  const size_t base = items.size();
  uint64_t v = 0;
  int nd = 0;                 // digits of the current token (0 = not in a token)
  bool lead0 = false;
  auto emit = [&]() -> bool {
    if (nd > 10 || (lead0 && nd > 1) || v > 2147483646ull) return false;
    const int32_t id = (int32_t)(v + 1);
    for (size_t j = base; j < items.size(); ++j)
      if (items[j] == id) { extras.push_back(id); return true; }
    items.push_back(id);
    mx = std::max(mx, id);
    return true;
  };
  int64_t q = p;
  for (; q < size; ++q) {
    const uint8_t c = d[q];
    const uint8_t dg = (uint8_t)(c - '0');
    if (dg <= 9) {
      if (nd == 0) { v = 0; lead0 = dg == 0; }
      v = v * 10 + dg;
      ++nd;
      continue;
    }
    if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
      if (nd) { if (!emit()) { items.resize(base); return -1; } nd = 0; }
      continue;
    }
    if (c == '\n' || c == '\r') break;
    items.resize(base);
    return -1;
  }
  if (nd && !emit()) { items.resize(base); return -1; }
  if (items.size() == base) {          // blank line (after trim): the single token ""
    items.push_back(0);
    mx = std::max(mx, 0);
  }
  return q;
}

// Parse lines starting in [b, e) of an in-memory buffer.
static int parse_buffer(const char* d, int64_t size, int64_t b, int64_t e, int mode, int nthreads,
                        TxnDB* db) {
  b = std::max<int64_t>(0, std::min(b, size));
  e = std::max<int64_t>(b, std::min(e, size));
  int64_t first = next_line_start(d, size, b);
  // per-thread sub-ranges with the same ownership rule
  int nt = std::max(1, nthreads);
  if (e - b < (int64_t)nt * 65536) nt = std::max<int64_t>(1, (e - b) / 65536);
  std::vector<int64_t> cuts(nt + 1);
  for (int t = 0; t <= nt; ++t) cuts[t] = b + (e - b) * t / nt;
  db->chunks.assign(nt, TxnChunk());
  std::vector<std::vector<int32_t>> extras(nt);
  std::vector<ThreadDict> dicts(mode == 1 ? nt : 0);
  std::vector<int32_t> tmax(nt, -1);
  std::atomic<bool> non_numeric{false};

  parallel_for_threads(nt, [&](int t) {
    int64_t lo = (t == 0) ? first : next_line_start(d, size, cuts[t]);
    int64_t hi = cuts[t + 1];
    // Everything a thread appends to lives on its own stack and is moved into
    // the shared arrays at the end: the vector headers of db->chunks[] and
    // extras[] sit side by side, and updating them per token false-shares
    // (measured 4x slower than serial on a 16-thread EPYC box).
    struct Local {
      TxnChunk ch;
      std::vector<int32_t> ex;
      int32_t mx = -1;
      TxnChunk& dst_ch;
      std::vector<int32_t>& dst_ex;
      int32_t& dst_mx;
      ~Local() { dst_ch = std::move(ch); dst_ex = std::move(ex); dst_mx = mx; }
    } L{TxnChunk(), {}, -1, db->chunks[t], extras[t], tmax[t]};
    TxnChunk& ch = L.ch;
    int32_t& mx = L.mx;
    std::vector<int32_t> line, table;
    ch.items.reserve((size_t)std::max<int64_t>(0, (hi - lo) / 3));
    ch.lens.reserve((size_t)std::max<int64_t>(0, (hi - lo) / 24));
    int64_t p = lo;
    while (p < hi && p < size) {
      int64_t q;
      if (mode == 0 && (q = fast_numeric_line((const uint8_t*)d, size, p, ch.items, L.ex, mx)) >= 0) {
        ch.lens.push_back((int64_t)(ch.items.size()));
        if (q >= size) { p = size; break; }
        p = (d[q] == '\r' && q + 1 < size && d[q + 1] == '\n') ? q + 2 : q + 1;
        continue;
      }
      q = p;
      while (q < size && d[q] != '\n' && d[q] != '\r') ++q;
      line.clear();
      if (mode == 0) {
        bool ok = true;
        for_each_token(d, p, q, [&](const char* s, int64_t n) {
          int32_t id = numeric_id(s, n);
          if (id < 0) ok = false; else line.push_back(id);
        });
        if (!ok) { non_numeric.store(true); return; }
      } else {
        ThreadDict& td = dicts[t];
        for_each_token(d, p, q, [&](const char* s, int64_t n) {
          line.push_back(td.get(std::string_view(s, (size_t)n)));
        });
      }
      if (mode == 0)
        for (int32_t v : line) mx = std::max(mx, v);
      emit_distinct(line, ch.items, L.ex, table);
      ch.lens.push_back((int64_t)(ch.items.size()));  // cumulative end within chunk
      if (q >= size) { p = size; break; }
      p = (d[q] == '\r' && q + 1 < size && d[q + 1] == '\n') ? q + 2 : q + 1;
      if (non_numeric.load(std::memory_order_relaxed)) return;
    }
  });
  if (mode == 0 && non_numeric.load()) return 1;

  db->numeric = (mode == 0);
  if (mode == 0) {
    int32_t mx = -1;
    for (int32_t m : tmax) mx = std::max(mx, m);
    db->vocab = (int64_t)mx + 1;
  } else {
    // merge thread dictionaries into one shard dictionary, remap ids (parallel)
    std::vector<std::vector<int32_t>> remap;
    if (!merge_dicts(dicts, nthreads, db, remap)) return 7;
    parallel_for_threads(std::max(1, std::min(nthreads, nt)), [&](int w) {
      for (int t = w; t < nt; t += std::max(1, std::min(nthreads, nt))) {
        for (auto& v : db->chunks[t].items) v = remap[t][(size_t)v];
        for (auto& v : extras[t]) v = remap[t][(size_t)v];
      }
    });
  }
  for (auto& ex : extras) db->extras.insert(db->extras.end(), ex.begin(), ex.end());
  return 0;
}

}  // namespace fa

using namespace fa;

// mode: 0 = auto (numeric if every token is canonical numeric, else dict), 1 = dict.
// On failure returns nullptr and sets *err (1 = cannot open, 2 = mmap, 7 = 64-bit
// token hash collision inside the shard).
FA_API TxnDB* fa_parse_file(const char* path, int64_t byte_begin, int64_t byte_end, int mode,
                            int nthreads, int* err) {
  *err = 0;
  MappedFile mf;
  if (!mf.open(path)) { *err = 1; return nullptr; }
  if (byte_end < 0) byte_end = mf.size;
  auto* db = new TxnDB();
  if (mode == 0) {
    if (parse_buffer(mf.data, mf.size, byte_begin, byte_end, 0, nthreads, db) == 0) return db;
    delete db;
    db = new TxnDB();
  }
  if (parse_buffer(mf.data, mf.size, byte_begin, byte_end, 1, nthreads, db) != 0) {
    delete db;
    *err = 7;          // two distinct tokens share a 64-bit hash
    return nullptr;
  }
  return db;
}

FA_API TxnDB* fa_parse_buffer(const char* data, int64_t size, int mode, int nthreads) {
  auto* db = new TxnDB();
  if (mode == 0) {
    if (parse_buffer(data, size, 0, size, 0, nthreads, db) == 0) return db;
    delete db;
    db = new TxnDB();
  }
  if (parse_buffer(data, size, 0, size, 1, nthreads, db) != 0) { delete db; return nullptr; }
  return db;
}

FA_API int64_t fa_file_size(const char* path) {
  struct stat st;
  if (stat(path, &st) != 0) return -1;
  return st.st_size;
}

// Line start helper exposed for tests of the sharding rule.
FA_API int64_t fa_next_line_start(const char* data, int64_t size, int64_t pos) {
  return next_line_start(data, size, pos);
}

// Line structure of one chunk of a file as it lands in a pinned buffer (the device
// parser's streamed regions, utils/io.py): info[0] = '\n' bytes, info[1] = offset of
// the last '\n' (-1: none), info[2] = 1 when any '\r' occurs (lone '\r' ends a line
// too: such chunks leave the rest of the file to the whole-region path).  Eight
// bytes per step with an exact zero-byte test, so one host thread keeps up with
// its share of the pread ring.
// AVX2 form of the scan: 64 bytes per step (two compares, movemasks and popcounts per
// 32 bytes); the reader threads call it on every 32 MB chunk as it lands in the pinned
// ring, so its rate is taken from the pread pipeline's (8 bytes per step: ~3 GB/s).
__attribute__((target("avx2"))) static void chunk_scan_avx2(const uint8_t* p, int64_t m, int64_t* nl_out,
                                                           uint64_t* cr_out, int64_t* done) {
  const __m256i nlv = _mm256_set1_epi8('\n'), crv = _mm256_set1_epi8('\r');
  int64_t nl = 0;
  uint32_t cr = 0;
  int64_t i = 0;
  for (; i + 64 <= m; i += 64) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i + 32));
    nl += __builtin_popcount((uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, nlv)));
    nl += __builtin_popcount((uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, nlv)));
    cr |= (uint32_t)_mm256_movemask_epi8(_mm256_or_si256(_mm256_cmpeq_epi8(a, crv), _mm256_cmpeq_epi8(b, crv)));
  }
  *nl_out = nl;
  *cr_out = cr;
  *done = i;
}

FA_API void fa_chunk_scan(const uint8_t* p, int64_t m, int64_t* info) {
  const uint64_t lo7 = 0x7F7F7F7F7F7F7F7Full;
  auto zeros = [lo7](uint64_t t) { return ~(((t & lo7) + lo7) | t | lo7); };   // 0x80 per zero byte
  int64_t nl = 0;
  uint64_t cr = 0;
  int64_t i = 0;
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) chunk_scan_avx2(p, m, &nl, &cr, &i);
  for (; i + 8 <= m; i += 8) {
    uint64_t x;
    std::memcpy(&x, p + i, 8);
    nl += __builtin_popcountll(zeros(x ^ 0x0A0A0A0A0A0A0A0Aull));
    cr |= zeros(x ^ 0x0D0D0D0D0D0D0D0Dull);
  }
  for (; i < m; ++i) {
    nl += p[i] == '\n';
    cr |= p[i] == '\r';
  }
  int64_t last = -1;
  for (int64_t j = m - 1; j >= 0; --j)
    if (p[j] == '\n') { last = j; break; }
  info[0] = nl;
  info[1] = last;
  info[2] = cr ? 1 : 0;
}
