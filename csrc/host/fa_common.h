// Shared helpers for the FastApriori-AMD native host library (libfa_host.so).
//
// Everything here is plain C++17 compiled with g++; the library exposes a C ABI
// consumed through ctypes by fastapriori_amd/ops/_native.py.
#pragma once

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#define FA_API extern "C" __attribute__((visibility("default")))

namespace fa {

// Persistent worker pool: thread start-up (~50 us per std::thread) would dominate
// the small per-level host steps.  Recreated after fork().
class ThreadPool {
 public:
  static ThreadPool& get() {
    static ThreadPool* pool = nullptr;
    static pid_t owner = 0;
    static std::mutex m;
    std::lock_guard<std::mutex> g(m);
    if (!pool || owner != getpid()) { pool = new ThreadPool(); owner = getpid(); }  // old one leaks after fork
    return *pool;
  }
  // Runs f(0..n-1); f(0) on the caller.  Calls are serialised.
  void run(int n, const std::function<void(int)>& f) {
    std::lock_guard<std::mutex> call(call_mu_);
    ensure(n - 1);
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f; njob_ = n; next_ = 1; remaining_ = n - 1; ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return remaining_ == 0; });
    job_ = nullptr;
  }

 private:
  void ensure(int k) {
    while ((int)th_.size() < k) th_.emplace_back([this] { loop(); });
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen && next_ < njob_; });
      seen = gen_;
      while (next_ < njob_) {
        const int id = next_++;
        const std::function<void(int)>* f = job_;
        lk.unlock();
        (*f)(id);
        lk.lock();
        if (--remaining_ == 0) done_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int njob_ = 0, next_ = 0, remaining_ = 0;
  uint64_t gen_ = 0;
};

// Run f(tid) for tid in [0, nthreads) on the pool (tid 0 runs on the caller).
inline void parallel_for_threads(int nthreads, const std::function<void(int)>& f) {
  if (nthreads <= 1) { f(0); return; }
  ThreadPool::get().run(nthreads, f);
}

// Dynamic chunked parallel loop over [0, n).
inline void parallel_for(int64_t n, int nthreads, int64_t grain,
                         const std::function<void(int64_t, int64_t, int)>& body) {
  if (n <= 0) return;
  if (nthreads <= 1 || n <= grain) { body(0, n, 0); return; }
  std::atomic<int64_t> next{0};
  parallel_for_threads(nthreads, [&](int tid) {
    for (;;) {
      int64_t b = next.fetch_add(grain);
      if (b >= n) break;
      body(b, std::min(n, b + grain), tid);
    }
  });
}

// splitmix64 finaliser: a strong 64-bit mixer (used for hashing and RNG seeding).
inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Deterministic 64-bit string hash (FNV-1a core + splitmix finaliser).  Used to
// agree on token identity across ranks in dictionary mode.
inline uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (size_t i = 0; i < n; ++i) { h ^= (uint8_t)p[i]; h *= 0x100000001B3ull; }
  return mix64(h ^ (uint64_t)n);
}

// xoshiro256** PRNG, seeded through splitmix64.
struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t z = seed;
    for (int i = 0; i < 4; ++i) { z += 0x9E3779B97F4A7C15ull; s[i] = mix64(z); }
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  inline uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  inline double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  inline uint64_t below(uint64_t n) { return (uint64_t)(((__uint128_t)next() * n) >> 64); }
};

}  // namespace fa
