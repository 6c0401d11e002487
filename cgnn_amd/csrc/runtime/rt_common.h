// Shared helpers of the host runtime (_rt): stateless hashing and a storage-free
// bijective permutation of [0, n) (used for shuffled node ids, so a rank can map
// any id without the permutation table of a 10^8-node graph).
#pragma once
#include <cstdint>

namespace cgnn_rt {

// splitmix64: cheap, well-mixed stateless hash used for deterministic sampling
inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline double unit01(uint64_t h) { return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

// 4-round Feistel network over 2*half bits, cycle-walked into [0, n): a seeded
// bijection of [0, n) evaluated in O(1) (expected < 4 walks since 2^(2 half) < 4n).
struct IdPermutation {
  uint64_t n = 1, half = 1, mask = 1, key[4] = {0, 0, 0, 0};
  IdPermutation() = default;
  IdPermutation(uint64_t n_, uint64_t seed) : n(n_ ? n_ : 1) {
    uint64_t bits = 1;
    while ((1ull << bits) < n) ++bits;
    half = (bits + 1) / 2;
    mask = (1ull << half) - 1;
    for (int r = 0; r < 4; ++r) key[r] = mix64(seed * 4 + r + 0x5EEDull);
  }
  uint64_t once(uint64_t v) const {
    uint64_t L = v >> half, R = v & mask;
    for (int r = 0; r < 4; ++r) {
      const uint64_t t = L ^ (mix64(R ^ key[r]) & mask);
      L = R;
      R = t;
    }
    return (L << half) | R;
  }
  uint64_t operator()(uint64_t v) const {
    do { v = once(v); } while (v >= n);
    return v;
  }
  uint64_t inverse_once(uint64_t v) const {
    uint64_t L = v >> half, R = v & mask;
    for (int r = 3; r >= 0; --r) {
      const uint64_t t = R ^ (mix64(L ^ key[r]) & mask);
      R = L;
      L = t;
    }
    return (L << half) | R;
  }
  uint64_t inverse(uint64_t v) const {
    do { v = inverse_once(v); } while (v >= n);
    return v;
  }
};

}  // namespace cgnn_rt
