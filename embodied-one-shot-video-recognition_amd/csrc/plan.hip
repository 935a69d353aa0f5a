// Episode-plan service: n-way k-shot episode plans drawn in the reference's
// RNG order, on the host, without rebuilding a class -> videos dict per episode.
//
// The reference (episode_novel_dataloader.py:25-70) draws from Python's `random` module:
//   random.sample(keys, n_way)                    :35
//   random.sample(aim_class_names, 1)[0]          :37
//   random.sample(videos, k_shot + 1 | k_shot)    :48 / :58, class by class in sampled order
// This restates CPython 3.10's generator exactly: MT19937 seeded by init_by_array over the
// seed's 32-bit digits (random.seed(int)), getrandbits(k <= 32) = genrand >> (32 - k),
// _randbelow = rejection over getrandbits(n.bit_length()), and Random.sample's two
// strategies (pool swap when n <= setsize, else a rejection set), so a plan equals
// eosv/episodes.py:sample_episodes(..., seed=s) draw for draw.  Host-only code: no HIP call.
#include <cmath>
#include <cstdint>
#include <string>
#include <unordered_set>
#include <vector>

#include "common.h"

namespace eosv {
namespace {

class PyMT {
 public:
  explicit PyMT(uint64_t seed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    init_by_array(key, key[1] ? 2 : 1);
  }
  uint32_t genrand() {
    if (mti_ >= N) twist();
    uint32_t y = mt_[mti_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  // random._randbelow_with_getrandbits(n), n >= 1
  uint32_t randbelow(uint32_t n) {
    int k = 0;
    while (k < 32 && (n >> k)) ++k;  // n.bit_length()
    uint32_t r = genrand() >> (32 - k);
    while (r >= n) r = genrand() >> (32 - k);
    return r;
  }

 private:
  static constexpr int N = 624, M = 397;
  uint32_t mt_[N];
  int mti_ = N + 1;

  void init_genrand(uint32_t s) {
    mt_[0] = s;
    for (int i = 1; i < N; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
    mti_ = N;
  }
  void init_by_array(const uint32_t* key, int len) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = N > len ? N : len; k; --k) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i, ++j;
      if (i >= N) mt_[0] = mt_[N - 1], i = 1;
      if (j >= len) j = 0;
    }
    for (int k = N - 1; k; --k) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      if (++i >= N) mt_[0] = mt_[N - 1], i = 1;
    }
    mt_[0] = 0x80000000u;
  }
  void twist() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int kk = 0;
    uint32_t y;
    for (; kk < N - M; ++kk) {
      y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
      mt_[kk] = mt_[kk + M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < N - 1; ++kk) {
      y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
      mt_[kk] = mt_[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt_[N - 1] & 0x80000000u) | (mt_[0] & 0x7fffffffu);
    mt_[N - 1] = mt_[M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    mti_ = 0;
  }
};

// Random.sample(range(n), k) -> positions, CPython 3.10 Lib/random.py
void sample_positions(PyMT& rng, int n, int k, int* out, std::vector<int>& pool) {
  int setsize = 21;
  if (k > 5) setsize += (int)std::pow(4.0, std::ceil(std::log((double)(k * 3)) / std::log(4.0)));
  if (n <= setsize) {
    pool.resize(n);
    for (int i = 0; i < n; ++i) pool[i] = i;
    for (int i = 0; i < k; ++i) {
      const int j = (int)rng.randbelow((uint32_t)(n - i));
      out[i] = pool[j];
      pool[j] = pool[n - i - 1];
    }
  } else {
    std::unordered_set<int> selected;
    for (int i = 0; i < k; ++i) {
      int j = (int)rng.randbelow((uint32_t)n);
      while (selected.count(j)) j = (int)rng.randbelow((uint32_t)n);
      selected.insert(j);
      out[i] = j;
    }
  }
}

}  // namespace
}  // namespace eosv

extern "C" int eosv_plan_episodes(const int32_t* class_sizes, int n_classes, int n_way, int k_shot, uint64_t seed,
                                  int n_episodes, int32_t* classes, int32_t* query, int32_t* support) {
  using eosv::set_error;
  if (n_episodes == 0) return EOSV_OK;
  if (!class_sizes || !classes || !query || !support || n_episodes < 0 || n_way < 1 || k_shot < 0)
    return set_error("eosv_plan_episodes: null or negative argument"), EOSV_ERR_ARG;
  if (n_way > n_classes) return set_error("eosv_plan_episodes: Sample larger than population (n_way)"), EOSV_ERR_ARG;
  eosv::PyMT rng(seed);
  std::vector<int> pool, pos(n_way > k_shot + 1 ? n_way : k_shot + 1);
  for (int e = 0; e < n_episodes; ++e) {
    int32_t* cls = classes + (size_t)e * n_way;
    int32_t* sup = support + (size_t)e * n_way * k_shot;
    eosv::sample_positions(rng, n_classes, n_way, pos.data(), pool);  // :35
    for (int i = 0; i < n_way; ++i) cls[i] = pos[i];
    int qpos;
    eosv::sample_positions(rng, n_way, 1, &qpos, pool);  // :37, a position in the sampled order
    query[2 * e] = qpos;
    for (int i = 0; i < n_way; ++i) {  // :45-70, class by class
      const int nv = class_sizes[cls[i]], take = i == qpos ? k_shot + 1 : k_shot;
      if (take > nv) return set_error("eosv_plan_episodes: Sample larger than population (videos of class " +
                                      std::to_string(cls[i]) + ")"), EOSV_ERR_ARG;
      eosv::sample_positions(rng, nv, take, pos.data(), pool);
      const int* p = pos.data();
      if (i == qpos) query[2 * e + 1] = *p++;
      for (int s = 0; s < k_shot; ++s) sup[i * k_shot + s] = p[s];
    }
  }
  return EOSV_OK;
}
