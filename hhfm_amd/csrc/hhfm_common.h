// Shared device helpers for the gfx950 FM-family kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/hhfm.h"

#define HHFM_DEV __device__ __forceinline__

namespace hhfm {

constexpr int kWave = 64;  // CDNA wavefront

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte load; NT = non-temporal (streamed once: does not displace the
// hot, re-read data — e.g. the FM bias table — from L2 / Infinity Cache)
template <bool NT>
HHFM_DEV u32x4_t load16(const void* p) {
  const u32x4_t* q = reinterpret_cast<const u32x4_t*>(p);
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}

template <bool NT>
HHFM_DEV int32_t load_i32(const int32_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// 16-byte chunk of an embedding row, widened to fp32.
// fp32 rows: 4 elements per chunk; bf16 rows: 8 elements per chunk.
template <bool BF16>
struct Chunk;

template <>
struct Chunk<false> {
  static constexpr int kElems = 4;
  float v[4];
  template <bool NT = false>
  HHFM_DEV void load(const void* p) {
    const u32x4_t x = load16<NT>(p);
    v[0] = __uint_as_float(x[0]); v[1] = __uint_as_float(x[1]);
    v[2] = __uint_as_float(x[2]); v[3] = __uint_as_float(x[3]);
  }
};

template <>
struct Chunk<true> {
  static constexpr int kElems = 8;
  float v[8];
  template <bool NT = false>
  HHFM_DEV void load(const void* p) {
    const u32x4_t x = load16<NT>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(x[i] << 16);             // low bf16
      v[2 * i + 1] = __uint_as_float(x[i] & 0xffff0000u);  // high bf16
    }
  }
};

HHFM_DEV float bf16_to_f32(uint16_t b) { return __uint_as_float(uint32_t(b) << 16); }

// Out-of-range ids are clamped to row 0 so a bad index can never fault the
// device; the Python layer validates ids and raises (TF embedding_lookup
// raises InvalidArgumentError on them).
HHFM_DEV int32_t clamp_id(int32_t id, int64_t M) {
  return (uint64_t)(uint32_t)id < (uint64_t)M ? id : 0;
}

// Record that this wave met an id outside [0, M) in the caller's status word
// (include/hhfm.h, HHFM_STATUS_BAD_ID): one vector atomic per wave that saw
// one, none otherwise; NULL = the caller did not ask.  Every lane of the wave
// must call it (kernel epilogue).
HHFM_DEV void report_bad_id(int32_t* status, bool bad) {
  if (status == nullptr) return;
  const uint64_t m = __ballot(bad);
  if (m != 0 && (threadIdx.x & (kWave - 1)) == (unsigned)(__ffsll((long long)m) - 1))
    atomicOr(status, HHFM_STATUS_BAD_ID);
}

// Query-column id check of hhfm_catalog_topk_ex (status.hip).
int launch_check_query_ids(const int32_t* q, int64_t B, int ncols, int ucol, int c0, int c1,
                           int t0, int t1, int64_t M, int32_t* status, hipStream_t s);

// Butterfly sum over aligned groups of G lanes (G a power of two <= 64).
template <int G>
HHFM_DEV float group_sum(float x) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, kWave);
  return x;
}

// CUs of the device that owns `st` (the stream's device, not the calling
// thread's current one), cached per device: the persistent grids ask per call
inline int stream_cu_count(hipStream_t st) {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipStreamGetDevice(st, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev < 0 || dev >= 64) return 256;
  int c = cache[dev].load(std::memory_order_relaxed);
  if (c <= 0) {
    c = 256;
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    cache[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

}  // namespace hhfm
