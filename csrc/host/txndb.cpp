// C ABI accessors for TxnDB: sizes, export into caller-owned arrays, free.
#include "fa_common.h"
#include "txndb.h"

using namespace fa;

// info[0]=n_lines info[1]=nnz info[2]=n_extras info[3]=numeric info[4]=vocab info[5]=dict_bytes
FA_API void fa_txndb_info(TxnDB* db, int64_t* info) {
  int64_t n = 0, nnz = 0, bytes = 0;
  for (auto& ch : db->chunks) { n += (int64_t)ch.lens.size(); nnz += (int64_t)ch.items.size(); }
  bytes = (int64_t)db->dict_blob.size();
  info[0] = n; info[1] = nnz; info[2] = (int64_t)db->extras.size();
  info[3] = db->numeric ? 1 : 0; info[4] = db->vocab; info[5] = bytes;
}

// offsets: n_lines+1 int64, items: nnz int32, extras: n_extras int32.
// Chunks are released as they are copied so peak memory stays ~1x.
FA_API void fa_txndb_export(TxnDB* db, int64_t* offsets, int32_t* items, int32_t* extras,
                            int nthreads) {
  const int nc = (int)db->chunks.size();
  std::vector<int64_t> line_base(nc + 1, 0), item_base(nc + 1, 0);
  for (int c = 0; c < nc; ++c) {
    line_base[c + 1] = line_base[c] + (int64_t)db->chunks[c].lens.size();
    item_base[c + 1] = item_base[c] + (int64_t)db->chunks[c].items.size();
  }
  offsets[0] = 0;
  parallel_for_threads(std::max(1, std::min(nthreads, nc)), [&](int t) {
    int nt = std::max(1, std::min(nthreads, nc));
    for (int c = t; c < nc; c += nt) {
      TxnChunk& ch = db->chunks[c];
      int64_t lb = line_base[c], ib = item_base[c];
      for (size_t i = 0; i < ch.lens.size(); ++i) offsets[lb + 1 + (int64_t)i] = ib + ch.lens[i];
      if (!ch.items.empty()) std::memcpy(items + ib, ch.items.data(), ch.items.size() * 4);
      std::vector<int64_t>().swap(ch.lens);
      std::vector<int32_t>().swap(ch.items);
    }
  });
  if (!db->extras.empty()) std::memcpy(extras, db->extras.data(), db->extras.size() * 4);
}

// Dictionary export: concatenated bytes + (n+1) offsets + 64-bit hash per entry.
FA_API void fa_txndb_export_dict(TxnDB* db, char* buf, int64_t* str_off, uint64_t* hashes, int nthreads) {
  const int64_t n = db->vocab;
  (void)nthreads;
  if (!db->dict_blob.empty()) std::memcpy(buf, db->dict_blob.data(), db->dict_blob.size());
  if (n > 0) {
    std::memcpy(str_off, db->dict_off.data(), (size_t)(n + 1) * 8);
    std::memcpy(hashes, db->dict_hash.data(), (size_t)n * 8);
  } else {
    str_off[0] = 0;
  }
}

// Hashes of n tokens given as one byte blob + (n+1) offsets (the same hash the
// parser gives dictionary entries): maps token strings to shard ids without
// Python loops over a vocabulary.
FA_API void fa_hash_tokens(const char* blob, const int64_t* off, int64_t n, uint64_t* out, int nthreads) {
  const int nt = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, n / 4096)));
  parallel_for_threads(nt, [&](int t) {
    for (int64_t i = n * t / nt, e = n * (t + 1) / nt; i < e; ++i)
      out[i] = hash_bytes(blob + off[i], (size_t)(off[i + 1] - off[i]));
  });
}

FA_API void fa_txndb_free(TxnDB* db) { delete db; }

FA_API uint64_t fa_hash_bytes(const char* p, int64_t n) { return hash_bytes(p, (size_t)n); }
