#include <chrono>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
inline uint32_t ap(const uint32_t* t, uint32_t v) {
  return t[v & 0xFFu] ^ t[256 + ((v >> 8) & 0xFFu)] ^ t[512 + ((v >> 16) & 0xFFu)] ^ t[768 + (v >> 24)];
}
int main() {
  std::mt19937 g(1);
  std::vector<uint32_t> t(1024), raw(14 * 64);
  for (auto& x : t) x = g();
  for (auto& x : raw) x = g();
  const int R = 14, W = 64, iters = 20000;
  uint32_t sink = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int it = 0; it < iters; ++it) {
    raw[it % raw.size()] ^= it;
    for (int r = 0; r < R; ++r) {
      uint32_t x = 0;
      for (int w = 0; w < W; ++w) x = ap(t.data(), x) ^ raw[r * W + w];
      sink ^= x;
    }
  }
  auto t1 = std::chrono::steady_clock::now();
  for (int it = 0; it < iters; ++it) {
    raw[it % raw.size()] ^= it;
    uint32_t x[14] = {0};
    for (int w = 0; w < W; ++w)
      for (int r = 0; r < R; ++r) x[r] = ap(t.data(), x[r]) ^ raw[r * W + w];
    for (int r = 0; r < R; ++r) sink ^= x[r];
  }
  auto t2 = std::chrono::steady_clock::now();
  printf("row-serial %.3f us, interleaved %.3f us (sink %u)\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count() / iters,
         std::chrono::duration<double, std::micro>(t2 - t1).count() / iters, sink);
}
