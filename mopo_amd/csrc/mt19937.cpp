// Host replica of numpy's legacy RandomState stream (MT19937), bit-exact.
//
// The reference draws all rollout randomness from numpy's global legacy RandomState:
//   np.random.normal (fake_env.py:72)        -> legacy_gauss: polar Box-Muller, caches the 2nd value
//   np.random.choice(elites, B) (bnn.py:343) -> elites[randint(0, M, B)]
//   np.random.randint(0, size, B) (flexible_replay_pool.py:87) -> masked rejection on 32-bit draws
// NEP 19 froze that stream, so the published algorithm (MT19937 init_genrand seeding, 53-bit
// doubles from two 32-bit draws, polar gauss, masked bounded ints) is reproduced here and
// checked against numpy itself in tests/test_rng.py.  State can be exchanged with
// np.random.get_state()/set_state() so the device rollout can consume the caller's stream.
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/mopo_hip.h"

namespace mopo {
int fail(const std::string& msg);
}

namespace {
constexpr int N = 624, M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

struct MT {
  uint32_t key[N];
  int pos;
  int has_gauss;
  double gauss;

  void seed(uint32_t s) {
    for (int i = 0; i < N; ++i) {
      key[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    pos = N;
    has_gauss = 0;
    gauss = 0.0;
  }
  void reload() {
    int i = 0;
    uint32_t y;
    for (; i < N - M; ++i) {
      y = (key[i] & UPPER) | (key[i + 1] & LOWER);
      key[i] = key[i + M] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
    }
    for (; i < N - 1; ++i) {
      y = (key[i] & UPPER) | (key[i + 1] & LOWER);
      key[i] = key[i + (M - N)] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
    }
    y = (key[N - 1] & UPPER) | (key[0] & LOWER);
    key[N - 1] = key[M - 1] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
    pos = 0;
  }
  static uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  uint32_t next32() {
    if (pos == N) reload();
    return temper(key[pos++]);
  }
  // The rest of the current block tempered into t (reloading first when it is used up); returns its
  // length.  The caller advances pos by what it consumes, so the stream position stays exact.
  int block(uint32_t* t) {
    if (pos == N) reload();
    const int cnt = N - pos;
    for (int j = 0; j < cnt; ++j) t[j] = temper(key[pos + j]);
    return cnt;
  }
  // n values of randint(low, low + rng + 1): the same masked rejection as bounded(), a block of tempered
  // draws at a time with a branch-free accept (a rejected value is overwritten by the next draw)
  template <typename T>
  void bounded_fill(T* out, int64_t n, int64_t low, uint32_t rng) {
    if (rng == 0 || rng == 0xffffffffu) {
      for (int64_t i = 0; i < n; ++i) out[i] = (T)(low + (int64_t)bounded(rng));
      return;
    }
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t t[N];
    int64_t k = 0;
    while (k < n) {
      const int cnt = block(t);
      int j = 0;
      for (; j < cnt && k < n; ++j) {
        const uint32_t v = t[j] & mask;
        out[k] = (T)(low + (int64_t)v);
        k += (v <= rng);
      }
      pos += j;
    }
  }
  // n doubles of random_sample: two tempered draws each (a pair may straddle a reload)
  void random_fill(double* out, int64_t n) {
    uint32_t t[N];
    int64_t i = 0;
    while (i < n) {
      if ((N - pos) < 2 || pos == N) {
        out[i++] = next_double();
        continue;
      }
      const int cnt = block(t) & ~1;
      int j = 0;
      for (; j < cnt && i < n; j += 2, ++i) {
        const int32_t a = (int32_t)(t[j] >> 5), b = (int32_t)(t[j + 1] >> 6);
        out[i] = (a * 67108864.0 + b) / 9007199254740992.0;
      }
      pos += j;
    }
  }
  double next_double() {
    int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  double next_gauss() {
    if (has_gauss) {
      double t = gauss;
      has_gauss = 0;
      gauss = 0.0;
      return t;
    }
    double f, x1, x2, r2;
    do {
      x1 = 2.0 * next_double() - 1.0;
      x2 = 2.0 * next_double() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    f = std::sqrt(-2.0 * std::log(r2) / r2);
    gauss = f * x1;
    has_gauss = 1;
    return f * x2;
  }
  // bounded value in [0, rng] (inclusive), rng < 2^32, masked rejection
  uint32_t bounded(uint32_t rng) {
    if (rng == 0) return 0;
    if (rng == 0xffffffffu) return next32();
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > rng) {
    }
    return v;
  }
};
}  // namespace

extern "C" int mopo_mt_create(mopo_mt_t* out, uint32_t seed) {
  if (!out) return mopo::fail("mopo_mt_create: NULL out");
  MT* m = new MT();
  m->seed(seed);
  *out = reinterpret_cast<mopo_mt_t>(m);
  return 0;
}

extern "C" int mopo_mt_destroy(mopo_mt_t h) {
  delete reinterpret_cast<MT*>(h);
  return 0;
}

extern "C" int mopo_mt_seed(mopo_mt_t h, uint32_t seed) {
  if (!h) return mopo::fail("mopo_mt_seed: NULL handle");
  reinterpret_cast<MT*>(h)->seed(seed);
  return 0;
}

extern "C" int mopo_mt_set_state(mopo_mt_t h, const uint32_t* key, int pos, int has_gauss, double gauss) {
  if (!h || !key) return mopo::fail("mopo_mt_set_state: NULL argument");
  if (pos < 0 || pos > N) return mopo::fail("mopo_mt_set_state: pos out of range");
  MT* m = reinterpret_cast<MT*>(h);
  std::memcpy(m->key, key, sizeof(m->key));
  m->pos = pos;
  m->has_gauss = has_gauss ? 1 : 0;
  m->gauss = gauss;
  return 0;
}

extern "C" int mopo_mt_get_state(mopo_mt_t h, uint32_t* key, int* pos, int* has_gauss, double* gauss) {
  if (!h || !key || !pos || !has_gauss || !gauss) return mopo::fail("mopo_mt_get_state: NULL argument");
  MT* m = reinterpret_cast<MT*>(h);
  std::memcpy(key, m->key, sizeof(m->key));
  *pos = m->pos;
  *has_gauss = m->has_gauss;
  *gauss = m->gauss;
  return 0;
}

extern "C" int mopo_mt_normal(mopo_mt_t h, double* out, int64_t n) {
  if (!h || (!out && n)) return mopo::fail("mopo_mt_normal: NULL argument");
  MT* m = reinterpret_cast<MT*>(h);
  for (int64_t i = 0; i < n; ++i) out[i] = m->next_gauss();
  return 0;
}

extern "C" int mopo_mt_random_sample(mopo_mt_t h, double* out, int64_t n) {
  if (!h || (!out && n)) return mopo::fail("mopo_mt_random_sample: NULL argument");
  reinterpret_cast<MT*>(h)->random_fill(out, n);
  return 0;
}

extern "C" int mopo_mt_randint(mopo_mt_t h, int64_t* out, int64_t n, int64_t low, int64_t high) {
  if (!h || (!out && n)) return mopo::fail("mopo_mt_randint: NULL argument");
  if (high <= low) return mopo::fail("mopo_mt_randint: low >= high");
  const uint64_t rng = (uint64_t)(high - 1 - low);
  if (rng > 0xffffffffull) return mopo::fail("mopo_mt_randint: range >= 2^32 not supported");
  reinterpret_cast<MT*>(h)->bounded_fill(out, n, low, (uint32_t)rng);
  return 0;
}

extern "C" int mopo_mt_randint_i32(mopo_mt_t h, int32_t* out, int64_t n, int64_t low, int64_t high) {
  if (!h || (!out && n)) return mopo::fail("mopo_mt_randint_i32: NULL argument");
  if (high <= low) return mopo::fail("mopo_mt_randint_i32: low >= high");
  if (low < INT32_MIN || high - 1 > INT32_MAX) return mopo::fail("mopo_mt_randint_i32: values outside int32");
  reinterpret_cast<MT*>(h)->bounded_fill(out, n, low, (uint32_t)(high - 1 - low));
  return 0;
}
