// In-memory transaction shard produced by the parser or the synthetic generator.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fa {

struct TxnChunk {
  std::vector<int64_t> lens;   // cumulative item count at the end of each line (within chunk)
  std::vector<int32_t> items;  // distinct ids per line, concatenated
};

struct TxnDB {
  std::vector<TxnChunk> chunks;
  std::vector<int32_t> extras;     // one id per repeated occurrence inside a line
  bool numeric = true;
  int64_t vocab = 0;               // id space size
  // dict mode: id -> token bytes, as one blob + (vocab + 1) offsets, and the
  // 64-bit hash of every entry (hash_bytes)
  std::string dict_blob;
  std::vector<int64_t> dict_off;
  std::vector<uint64_t> dict_hash;
};

int64_t next_line_start(const char* d, int64_t size, int64_t pos);

}  // namespace fa
