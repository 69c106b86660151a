// Input-pipeline order of one training epoch (reference make_ds,
// src/trainer.py:115-117: ds.shuffle(50000).batch(B)).
//
// tf.data's shuffle(buffer_size) keeps a buffer of the next buffer_size elements; each output
// draws a uniformly random slot of the buffer, emits it and refills the slot with the next input
// element; once the input is exhausted the buffer drains the same way (reshuffle_each_iteration
// defaults to True, so every epoch draws a new order). The reference leaves the shuffle unseeded,
// so no particular order is its output; what a drop-in must keep is the window: output i is input
// j with j < i + buffer_size, every element exactly once. This is that process, on the host (it is
// sequential by nature: ~20 ns per element), with a counter-based splitmix64 stream seeded by
// (seed, epoch) so every data-parallel rank computes the same global order without an exchange.
// The index order is then uploaded once per epoch and batches are gathered on the device.
#include <cstdint>
#include <vector>

#include "common.hpp"

namespace rs {
namespace {

struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  // uniform in [0, n) without modulo bias (Lemire's multiply-shift with rejection)
  uint64_t below(uint64_t n) {
    unsigned __int128 m = (unsigned __int128)next() * n;
    uint64_t lo = (uint64_t)m;
    if (lo < n) {
      const uint64_t t = (0 - n) % n;
      while (lo < t) {
        m = (unsigned __int128)next() * n;
        lo = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
};

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" {

int rs_shuffle_buffer_order_i64(int64_t n, int64_t buffer_size, uint64_t seed, uint64_t epoch, int64_t* order) {
  RS_REQUIRE(n >= 0 && buffer_size >= 1 && (n == 0 || order), "rs_shuffle_buffer_order_i64: bad args");
  if (n == 0) return RS_OK;
  SplitMix64 rng{seed * 0xD1B54A32D192ED03ull ^ (epoch + 1) * 0x9E3779B97F4A7C15ull};
  const int64_t cap = buffer_size < n ? buffer_size : n;
  std::vector<int64_t> buf((size_t)cap);
  for (int64_t i = 0; i < cap; ++i) buf[(size_t)i] = i;
  int64_t next = cap, live = cap;
  for (int64_t o = 0; o < n; ++o) {
    const int64_t j = (int64_t)rng.below((uint64_t)live);
    order[o] = buf[(size_t)j];
    if (next < n) {
      buf[(size_t)j] = next++;  // refill the drawn slot with the next input element
    } else {
      buf[(size_t)j] = buf[(size_t)(live - 1)];  // input exhausted: drain
      --live;
    }
  }
  return RS_OK;
}

}  // extern "C"
