// Diagnostic (not product): the DeepFM ITEM-projection row grouping
// (dfm_fused.hip dfm_order_rows, counting-sort branch) at the C5 bench shape
// (12.5 M rows, F = 5, 957 users, key field 0), current scatter against a
// slice-local sort whose writes are ordered (dword-parallel runs per user;
// "ord" — the product's dfm_group_scatter, which additionally limits its bins
// to the slice's key range) and per-row ordered writes ("ordrow").  Bins here
// = the 957 users; results in profiles/r02_groupbench.txt.
// Prints ms per grouping (best of 7) and checks each variant's output.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kBins = 8192;

template <int ROWS>
__global__ __launch_bounds__(1024) void hist(const int32_t* idx, int64_t B, int F, int kf, int nb,
                                             uint32_t* count) {
  __shared__ uint32_t h[kBins];
  for (int b = threadIdx.x; b < nb; b += 1024) h[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * ROWS, r1 = r0 + ROWS < B ? r0 + ROWS : B;
  for (int64_t m = r0 + threadIdx.x; m < r1; m += 1024) atomicAdd(&h[idx[m * F + kf]], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += 1024)
    if (h[b]) atomicAdd(&count[b], h[b]);
}

__global__ __launch_bounds__(1024) void scan(const uint32_t* count, int64_t M, uint32_t* start) {
  __shared__ uint32_t part[1024];
  const int per = (int)((M + 1023) / 1024);
  const int b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int b = b0; b < b0 + per && b < M; ++b) s += count[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (int b = b0; b < b0 + per && b < M; ++b) { start[b] = run; run += count[b]; }
}

// current product scatter
template <int ROWS>
__global__ __launch_bounds__(1024) void scatter_cur(const int32_t* idx, int64_t B, int F, int kf,
                                                    int nb, const uint32_t* start, uint32_t* cursor,
                                                    int32_t* rows, int32_t* order) {
  __shared__ uint32_t h[kBins];
  for (int b = threadIdx.x; b < nb; b += 1024) h[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * ROWS, r1 = r0 + ROWS < B ? r0 + ROWS : B;
  for (int64_t m = r0 + threadIdx.x; m < r1; m += 1024) atomicAdd(&h[idx[m * F + kf]], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += 1024)
    if (h[b]) h[b] = start[b] + atomicAdd(&cursor[b], h[b]);
  __syncthreads();
  for (int64_t m = r0 + threadIdx.x; m < r1; m += 1024) {
    const uint32_t pos = atomicAdd(&h[idx[m * F + kf]], 1u);
    for (int f = 0; f < F; ++f) rows[(int64_t)pos * F + f] = idx[m * F + f];
    order[pos] = (int32_t)m;
  }
}

// slice-local counting sort in LDS, then ordered dword-parallel writes
template <int ROWS>
__global__ __launch_bounds__(1024) void scatter_ord(const int32_t* idx, int64_t B, int F, int kf,
                                                    int nb, const uint32_t* start, uint32_t* cursor,
                                                    int32_t* rows, int32_t* order) {
  constexpr int PER = ROWS / 1024;
  __shared__ uint32_t h[kBins];       // count -> local start
  __shared__ int32_t delta[kBins];    // global position - local start
  __shared__ uint32_t lrow[ROWS];     // local sorted position -> (key << 16 | local row)
  __shared__ uint32_t wsum[16];
  for (int b = threadIdx.x; b < nb; b += 1024) h[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int n = (int)(r0 + ROWS < B ? ROWS : B - r0);
  int key[PER];
  uint32_t rk[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = threadIdx.x + i * 1024;
    if (j < n) { key[i] = idx[(r0 + j) * F + kf]; rk[i] = atomicAdd(&h[key[i]], 1u); }
  }
  __syncthreads();
  // exclusive scan of h[0, nb): per-thread chunk, then wave + block scan
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int b = b0; b < b0 + per && b < nb; ++b) s += h[b];
  uint32_t inc = s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(inc, off, 64);
    if (lane >= off) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wb = 0;
  for (int i = 0; i < w; ++i) wb += wsum[i];
  uint32_t run = wb + inc - s;
  for (int b = b0; b < b0 + per && b < nb; ++b) {
    const uint32_t c = h[b];
    h[b] = run;
    delta[b] = c ? (int32_t)(start[b] + atomicAdd(&cursor[b], c)) - (int32_t)run : 0;
    run += c;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = threadIdx.x + i * 1024;
    if (j < n) lrow[h[key[i]] + rk[i]] = ((uint32_t)key[i] << 16) | (uint32_t)j;
  }
  __syncthreads();
  for (int x = threadIdx.x; x < n * F; x += 1024) {
    const int j = x / F, f = x - j * F;
    const uint32_t e = lrow[j];
    const int jl = (int)(e & 0xffff), kk = (int)(e >> 16);
    const int64_t dest = (int64_t)delta[kk] + j;
    rows[dest * F + f] = idx[(r0 + jl) * F + f];
    if (f == 0) order[dest] = (int32_t)(r0 + jl);
  }
}

// same, rows written by consecutive lanes (F words each)
template <int ROWS>
__global__ __launch_bounds__(1024) void scatter_ordrow(const int32_t* idx, int64_t B, int F, int kf,
                                                    int nb, const uint32_t* start, uint32_t* cursor,
                                                    int32_t* rows, int32_t* order) {
  constexpr int PER = ROWS / 1024;
  __shared__ uint32_t h[kBins];       // count -> local start
  __shared__ int32_t delta[kBins];    // global position - local start
  __shared__ uint32_t lrow[ROWS];     // local sorted position -> (key << 16 | local row)
  __shared__ uint32_t wsum[16];
  for (int b = threadIdx.x; b < nb; b += 1024) h[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int n = (int)(r0 + ROWS < B ? ROWS : B - r0);
  int key[PER];
  uint32_t rk[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = threadIdx.x + i * 1024;
    if (j < n) { key[i] = idx[(r0 + j) * F + kf]; rk[i] = atomicAdd(&h[key[i]], 1u); }
  }
  __syncthreads();
  // exclusive scan of h[0, nb): per-thread chunk, then wave + block scan
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int b = b0; b < b0 + per && b < nb; ++b) s += h[b];
  uint32_t inc = s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(inc, off, 64);
    if (lane >= off) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wb = 0;
  for (int i = 0; i < w; ++i) wb += wsum[i];
  uint32_t run = wb + inc - s;
  for (int b = b0; b < b0 + per && b < nb; ++b) {
    const uint32_t c = h[b];
    h[b] = run;
    delta[b] = c ? (int32_t)(start[b] + atomicAdd(&cursor[b], c)) - (int32_t)run : 0;
    run += c;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = threadIdx.x + i * 1024;
    if (j < n) lrow[h[key[i]] + rk[i]] = ((uint32_t)key[i] << 16) | (uint32_t)j;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += 1024) {
    const uint32_t e = lrow[j];
    const int jl = (int)(e & 0xffff), kk = (int)(e >> 16);
    const int64_t dest = (int64_t)delta[kk] + j;
    const int32_t* src = idx + (r0 + jl) * F;
    for (int f = 0; f < F; ++f) rows[dest * F + f] = src[f];
    order[dest] = (int32_t)(r0 + jl);
  }
}

int main() {
  const int64_t B = 12500000;
  const int F = 5, nu = 957, ni = 4082;
  std::vector<int32_t> h(B * F);
  srand(7);
  for (int64_t m = 0; m < B; ++m) {
    h[m * F] = rand() % nu;
    h[m * F + 1] = nu + rand() % ni;
    h[m * F + 2] = nu + ni + rand() % 7;
    h[m * F + 3] = nu + ni + 7 + rand() % 2;
    h[m * F + 4] = nu + ni + 9 + rand() % 3;
  }
  int32_t *idx, *rows, *order;
  uint32_t *count, *cursor, *start;
  CK(hipMalloc(&idx, B * F * 4));
  CK(hipMalloc(&rows, B * F * 4));
  CK(hipMalloc(&order, B * 4));
  CK(hipMalloc(&count, 3 * kBins * 4));
  cursor = count + kBins;
  start = count + 2 * kBins;
  CK(hipMemcpy(idx, h.data(), B * F * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<int32_t> hr(B * F), ho(B);
  auto run = [&](const char* name, auto launch_hist, auto launch_scatter) {
    float best = 1e9, bh = 1e9;
    for (int rep = 0; rep < 7; ++rep) {
      CK(hipMemsetAsync(count, 0, 2 * kBins * 4, 0));
      CK(hipEventRecord(a));
      launch_hist();
      hipLaunchKernelGGL(scan, dim3(1), dim3(1024), 0, 0, count, (int64_t)nu, start);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float t0;
      CK(hipEventElapsedTime(&t0, a, b));
      CK(hipEventRecord(a));
      launch_scatter();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float t1;
      CK(hipEventElapsedTime(&t1, a, b));
      best = std::min(best, t1);
      bh = std::min(bh, t0);
    }
    CK(hipGetLastError());
    CK(hipMemcpy(hr.data(), rows, B * F * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ho.data(), order, B * 4, hipMemcpyDeviceToHost));
    // check: order is a permutation, rows[p] = idx[order[p]], keys non-decreasing
    std::vector<char> seen(B, 0);
    long bad = 0;
    for (int64_t p = 0; p < B; ++p) {
      const int64_t m = ho[p];
      if (m < 0 || m >= B || seen[m]) { ++bad; continue; }
      seen[m] = 1;
      for (int f = 0; f < F; ++f) bad += hr[p * F + f] != h[m * F + f];
      if (p && hr[p * F] < hr[(p - 1) * F]) ++bad;
    }
    printf("%-22s hist+scan %.3f ms  scatter %.3f ms  bad=%ld\n", name, bh, best, bad);
  };
#define HIST(R) [&] { hipLaunchKernelGGL(hist<R>, dim3((B + R - 1) / R), dim3(1024), 0, 0, idx, B, F, 0, nu, count); }
#define SC(K, R) [&] { hipLaunchKernelGGL(K<R>, dim3((B + R - 1) / R), dim3(1024), 0, 0, idx, B, F, 0, nu, start, cursor, rows, order); }
  run("cur 8192", HIST(8192), SC(scatter_cur, 8192));
  run("cur 4096", HIST(8192), SC(scatter_cur, 4096));
  run("cur 16384", HIST(16384), SC(scatter_cur, 16384));
  run("ord 4096", HIST(8192), SC(scatter_ord, 4096));
  run("ord 8192", HIST(8192), SC(scatter_ord, 8192));
  run("ord 16384", HIST(16384), SC(scatter_ord, 16384));
  run("ordrow 4096", HIST(8192), SC(scatter_ordrow, 4096));
  run("ordrow 8192", HIST(8192), SC(scatter_ordrow, 8192));
  run("ordrow 2048", HIST(8192), SC(scatter_ordrow, 2048));
  run("ord 2048", HIST(8192), SC(scatter_ord, 2048));
  return 0;
}
