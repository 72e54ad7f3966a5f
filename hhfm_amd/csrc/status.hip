// Id validation (status word) and the HBM read probe.
//
//   hhfm_check_ids / hhfm_status_read   — the InvalidArgumentError that
//       tf.nn.embedding_lookup raises on ids outside [0, features_M)
//       (Newcode/FM.py:99, OurModel7.py:105, AFM.py:104, DFM.py:105), for C
//       callers: kernels read such ids as row 0 (they can never fault) and
//       OR HHFM_STATUS_BAD_ID into a caller-owned device word, which
//       hhfm_status_read turns into HHFM_EINVAL.
//   hhfm_probe_stream_read — measurement only: one sequential 16-B-per-lane
//       read of a device buffer, the box's HBM read ceiling for bench.py.
#include "hhfm_common.h"

namespace hhfm {

// every element of idx[0..n)
__global__ __launch_bounds__(256) void check_ids_kernel(const int32_t* __restrict__ idx,
                                                        int64_t n, int64_t M,
                                                        int32_t* __restrict__ status) {
  bool bad = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    bad |= clamp_id(idx[i], M) != idx[i];
  report_bad_id(status, bad);
}

// the columns a catalog query reads: user, ctx [c0,c1), time [t0,t1)
__global__ __launch_bounds__(256) void check_query_ids_kernel(
    const int32_t* __restrict__ q, int64_t B, int ncols, int ucol, int c0, int c1, int t0,
    int t1, int64_t M, int32_t* __restrict__ status) {
  bool bad = false;
  const int64_t n = B * ncols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % ncols);
    const bool used = c == ucol || (c >= c0 && c < c1) || (c >= t0 && c < t1);
    bad |= used && clamp_id(q[i], M) != q[i];
  }
  report_bad_id(status, bad);
}

static int check_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

int launch_check_query_ids(const int32_t* q, int64_t B, int ncols, int ucol, int c0, int c1,
                           int t0, int t1, int64_t M, int32_t* status, hipStream_t s) {
  if (!status || B == 0) return HHFM_OK;
  hipLaunchKernelGGL(check_query_ids_kernel, dim3(check_grid(B * ncols)), dim3(256), 0, s, q,
                     B, ncols, ucol, c0, c1, t0, t1, M, status);
  return (int)hipGetLastError();
}

// mode 0: grid-stride (each wave 1 KiB, consecutive waves adjacent)
__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4_t* __restrict__ p,
                                                          int64_t n16, float* sink) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4_t a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= p[i];
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1.f;
}

// modes 1/2: each workgroup streams one contiguous chunk, 8 loads in flight
// per lane; NT = non-temporal loads
template <bool NT>
__global__ __launch_bounds__(256) void stream_read_chunk_kernel(const u32x4_t* __restrict__ p,
                                                                int64_t n16, int64_t chunk,
                                                                float* sink) {
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < n16 ? b0 + chunk : n16;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  int64_t i = b0 + threadIdx.x;
  for (; i + 7 * 256 < b1; i += 8 * 256) {
    u32x4_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = load16<NT>(p + i + j * 256);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j];
  }
  for (; i < b1; i += 256) acc ^= load16<NT>(p + i);
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1.f;
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_check_ids(const int32_t* idx, int64_t n, int64_t features_M,
                              int32_t* status, void* stream) {
  if (n < 0 || features_M < 1 || !status) return HHFM_EINVAL;
  if (n == 0) return HHFM_OK;
  if (!idx) return HHFM_EINVAL;
  hipLaunchKernelGGL(check_ids_kernel, dim3(check_grid(n)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), idx, n, features_M, status);
  return (int)hipGetLastError();
}

extern "C" int hhfm_status_read(int32_t* status, void* stream) {
  if (!status) return HHFM_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int32_t h = 0;
  hipError_t e = hipMemcpyAsync(&h, status, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && h != 0) e = hipMemsetAsync(status, 0, sizeof(int32_t), s);
  if (e != hipSuccess) return (int)e;
  return (h & HHFM_STATUS_BAD_ID) ? HHFM_EINVAL : HHFM_OK;
}

extern "C" int hhfm_probe_stream_read(const void* buf, int64_t bytes, int32_t mode,
                                      float* sink, void* stream) {
  if (!buf || !sink || bytes < 16 || (bytes & 15) || mode < 0 || mode > 2 ||
      (reinterpret_cast<uintptr_t>(buf) & 15))
    return HHFM_EINVAL;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const u32x4_t* p = reinterpret_cast<const u32x4_t*>(buf);
  const int64_t n16 = bytes / 16;
  if (mode == 0) {
    hipLaunchKernelGGL(stream_read_kernel, dim3(cus * 8), dim3(256), 0, s, p, n16, sink);
  } else {
    const int64_t grid = (int64_t)cus * 8;
    const int64_t step = 8 * 256;
    const int64_t chunk = ((n16 + grid - 1) / grid + step - 1) / step * step;
    const int64_t nb = (n16 + chunk - 1) / chunk;
    if (mode == 1)
      hipLaunchKernelGGL(stream_read_chunk_kernel<false>, dim3((int)nb), dim3(256), 0, s, p,
                         n16, chunk, sink);
    else
      hipLaunchKernelGGL(stream_read_chunk_kernel<true>, dim3((int)nb), dim3(256), 0, s, p,
                         n16, chunk, sink);
  }
  return (int)hipGetLastError();
}
