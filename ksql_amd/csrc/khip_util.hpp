// khip_util.hpp — shared host/device helpers for libksqldb_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <string>

#include "../../include/ksqldb_hip.h"

namespace khip {

// ----------------------------------------------------------------- errors
void set_error(const std::string& msg);
void clear_error();

#define KHIP_TRY_HIP(expr)                                                            \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      ::khip::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));           \
      return KHIP_E_DEVICE;                                                           \
    }                                                                                 \
  } while (0)

#define KHIP_TRY(expr)              \
  do {                              \
    khip_status _s = (expr);        \
    if (_s != KHIP_OK) return _s;   \
  } while (0)

inline khip_status fail(khip_status s, const std::string& msg) {
  set_error(msg);
  return s;
}

// Tuning knobs (tile sizes, unroll factors, LDS budget...).  Only the tuning build
// (make TUNING=1 → libksqldb_hip_tune.so) reads them from the environment, for GPU sweeps;
// the release library always uses the measured defaults, so a stray variable cannot change
// what it computes or how fast.
inline int64_t knob(const char* name, int64_t dflt) {
#ifdef KHIP_TUNING
  const char* e = getenv(name);
  return e ? atoll(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

// Grow-only device buffer, owned: freed when it goes out of scope (a function's scratch) or with its
// handle; moved, never copied.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) {
    o.p = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      bytes = o.bytes;
      o.p = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  khip_status ensure(size_t want) {
    if (want <= bytes) return KHIP_OK;
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
    size_t b = want < 256 ? 256 : want;
    if (hipMalloc(&p, b) != hipSuccess) {
      p = nullptr;
      return fail(KHIP_E_NOMEM, "hipMalloc failed for " + std::to_string(b) + " bytes");
    }
    bytes = b;
    return KHIP_OK;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// Pinned host staging buffer (grow-only).
struct HostBuf {
  void* p = nullptr;
  size_t bytes = 0;
  khip_status ensure(size_t want) {
    if (want <= bytes) return KHIP_OK;
    if (p) hipHostFree(p);
    p = nullptr;
    bytes = 0;
    size_t b = want < 256 ? 256 : want;
    if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return fail(KHIP_E_NOMEM, "hipHostMalloc failed");
    }
    bytes = b;
    return KHIP_OK;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// RAII device guard.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

// --------------------------------------------------------------- device helpers

__host__ __device__ inline uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}

// Hash of a (key, windowStart) group.
__host__ __device__ inline uint64_t group_hash(int64_t key, int64_t ws) {
  return mix64((uint64_t)key ^ mix64((uint64_t)ws + 0x9E3779B97F4A7C15ULL));
}

__device__ inline bool bit_get(const uint8_t* bm, int64_t i) {
  return bm == nullptr ? true : ((bm[i >> 3] >> (i & 7)) & 1);
}

// Total-order key for Java Double.compareTo (NaN canonical & largest, -0.0 < 0.0):
// signed comparison of the returned key == Double.compare.  Involution on non-NaN.
__host__ __device__ inline int64_t f64_order_key(double d) {
  uint64_t u;
  __builtin_memcpy(&u, &d, 8);
  if ((u & 0x7ff0000000000000ULL) == 0x7ff0000000000000ULL && (u & 0x000fffffffffffffULL))
    u = 0x7ff8000000000000ULL;
  int64_t k = (int64_t)u;
  return k ^ ((k >> 63) & 0x7fffffffffffffffLL);
}
__host__ __device__ inline double f64_from_order_key(int64_t k) {
  int64_t b = k ^ ((k >> 63) & 0x7fffffffffffffffLL);
  double d;
  __builtin_memcpy(&d, &b, 8);
  return d;
}

__host__ __device__ inline int64_t grace_of(const khip_agg_desc& d) {
  if (d.window_kind == KHIP_WINDOW_NONE) return 0;
  if (d.grace_ms >= 0) return d.grace_ms;
  // EMIT FINAL without GRACE PERIOD: the analyzer substitutes zero grace
  // (ksqldb-engine/.../analyzer/RewrittenAnalysis.java:65,149-154)
  if (d.emit == KHIP_EMIT_FINAL) return 0;
  int64_t g = 86400000LL - d.size_ms;
  return g > 0 ? g : 0;
}

// TimeWindows.windowsFor first window start.
__host__ __device__ inline int64_t first_window_start(int64_t ts, int64_t size, int64_t adv) {
  int64_t lo = ts - size + adv;
  if (lo < 0) lo = 0;
  return (lo / adv) * adv;
}

// Unsigned 64-bit division by a launch-constant divisor without the ~50-instruction
// software divide: Granlund & Montgomery, "Division by Invariant Integers using
// Multiplication" (1994), Fig. 4.1.  l = ceil(log2 d), m = floor(2^64 (2^l - d) / d) + 1,
// q = (t + ((n - t) >> min(l,1))) >> max(l-1,0), t = mulhi(m, n).  Exact for all n, d >= 1.
struct FastDiv {
  uint64_t m;
  uint32_t sh1, sh2;
};

inline FastDiv make_fastdiv(uint64_t d) {
  uint32_t l = 0;
  while (l < 64 && (1ULL << l) < d) l++;
  const unsigned __int128 two_l = (unsigned __int128)1 << l;
  const unsigned __int128 num = ((unsigned __int128)1 << 64) * (two_l - d);
  FastDiv f;
  f.m = (uint64_t)(num / d) + 1;
  f.sh1 = l < 1 ? l : 1;
  f.sh2 = l > 1 ? l - 1 : 0;
  return f;
}

__host__ __device__ inline uint64_t fast_udiv(uint64_t n, const FastDiv& f) {
#ifdef __HIP_DEVICE_COMPILE__
  const uint64_t t = __umul64hi(f.m, n);
#else
  const uint64_t t = (uint64_t)(((unsigned __int128)f.m * n) >> 64);
#endif
  return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

// 32-bit variant for dividends below 2^32 (window indices relative to a push's time base):
// q = (hi32(m * n) + ((n - hi) >> sh1)) >> sh2, d in [1, 2^31].
struct FastDiv32 {
  uint32_t m, sh1, sh2;
};

inline FastDiv32 make_fastdiv32(uint32_t d) {
  uint32_t l = 0;
  while (l < 32 && (1ULL << l) < d) l++;
  FastDiv32 f;
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  f.sh1 = l < 1 ? l : 1;
  f.sh2 = l > 1 ? l - 1 : 0;
  return f;
}

__host__ __device__ inline uint32_t fast_udiv32(uint32_t n, const FastDiv32& f) {
#ifdef __HIP_DEVICE_COMPILE__
  const uint32_t t = __umulhi(f.m, n);
#else
  const uint32_t t = (uint32_t)(((uint64_t)f.m * n) >> 32);
#endif
  return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

// first_window_start with the division by `adv` done through `fd` (= make_fastdiv(adv)).
__host__ __device__ inline int64_t first_window_start_fd(int64_t ts, int64_t size, int64_t adv, const FastDiv& fd) {
  int64_t lo = ts - size + adv;
  if (lo < 0) lo = 0;
  return (int64_t)fast_udiv((uint64_t)lo, fd) * adv;
}

inline int64_t next_pow2(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace khip
