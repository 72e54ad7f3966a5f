// H5 on the device — Train.sample_negative (Newcode/FM.py:284-294) with
// numpy's own random stream ("rejection sampling in a
// kernel").
//
//   samples = np.random.randint(n_user, n_user + n_item, size=(len(data), num))
//   for i, j in row-major order:
//       while samples[i, j] in positive_feedback[key_i]:
//           samples[i, j] = np.random.randint(n_user, n_user + n_item)
//
// numpy's legacy RandomState (numpy/random/mtrand.pyx randint -> the
// _bounded_integers _rand_int64 fill with use_masked = True ->
// random_bounded_uint64_fill -> buffered_bounded_masked_uint32) draws every
// value, block or scalar, the same way: take 32-bit MT19937 outputs in order,
// AND them with the smallest all-ones mask covering rng = hi - 1 - lo, reject
// while the result exceeds rng; the value is lo + result.  (rng = 0 draws
// nothing.)  So the whole call — block and re-draws — reads ONE sequential
// stream of accepted values, and the final generator state is fixed by the
// last word read.  This file reproduces that stream on the device:
//
//   * MT19937 as the linear recurrence x[n+624] = x[n+397] ^ twist(x[n],
//     x[n+1]) over the untempered words (numpy's mt19937_gen restated; the
//     state's key[624] is x[624b .. 624b+624) for some b, pos the offset of
//     the next word).  Words n .. n+226 depend only on earlier words, and the
//     next 227 on those and on earlier ones, so ONE workgroup produces 454
//     words per barrier (an LDS ring of the last 1,078 words);
//   * accepted values: tempering + mask + (<= rng) per word, a block count, a
//     scan and a compaction (value, word position) in stream order;
//   * the block: samples[e] = lo + value[e], e < rows·num; the membership of
//     every block sample in its row's key (binary searches in the sorted
//     (key rank << 32 | item) codes of hhfm_pf_contains, the key's code range
//     found once per row), the rejected entries compacted in row-major order;
//   * the re-draws: one workgroup walks the rejected entries in order, 256 at
//     a time, each taking the next accepted value; the first one whose value
//     is again a positive makes the entries before it final and repeats with
//     the following value — exactly the reference's sequential loop;
//   * the state after the last word read goes back to the caller (key[624],
//     pos), which np.random.set_state restores on the host.
// If the accepted values of one generation round run out, another round
// continues the stream from the last 624 words (the window slides; rounds
// end on block boundaries, so the final key is always in the window).
#include "hhfm_common.h"

namespace hhfm {

constexpr int kMtN = 624, kMtM = 397, kMtStep = kMtN - kMtM;   // 227
constexpr int kMtRing = 2048;                                   // > 624 + 2·227
constexpr int kScanBlock = 1024;                                // stream items per count block

HHFM_DEV uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

HHFM_DEV uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// x[n0 .. n1) from x[n0-624 .. n0) (n1 - n0 a multiple of 624): one
// workgroup, thread t computes word n + t and then n + 227 + t — the second
// needs x[n + t] (its own first word) and x[n + t - 397 .. - 396] (< n, ready
// before the barrier), so two steps of 227 run per barrier.
__global__ __launch_bounds__(256) void mt_generate(uint32_t* __restrict__ x, int64_t n0,
                                                   int64_t n1) {
  __shared__ uint32_t ring[kMtRing];
  const int t = threadIdx.x;
  for (int i = t; i < kMtN; i += blockDim.x) {
    const int64_t g = n0 - kMtN + i;
    ring[g & (kMtRing - 1)] = x[g];
  }
  __syncthreads();
  for (int64_t n = n0; n < n1; n += 2 * kMtStep) {
    if (t < kMtStep) {
      const int64_t g0 = n + t, g1 = g0 + kMtStep;
      const uint32_t v0 = mt_twist(ring[(g0 - kMtN) & (kMtRing - 1)],
                                   ring[(g0 - kMtN + 1) & (kMtRing - 1)],
                                   ring[(g0 - kMtStep) & (kMtRing - 1)]);
      if (g0 < n1) {
        ring[g0 & (kMtRing - 1)] = v0;
        x[g0] = v0;
      }
      if (g1 < n1) {
        const uint32_t v1 = mt_twist(ring[(g1 - kMtN) & (kMtRing - 1)],
                                     ring[(g1 - kMtN + 1) & (kMtRing - 1)], v0);
        ring[g1 & (kMtRing - 1)] = v1;
        x[g1] = v1;
      }
    }
    __syncthreads();
  }
}

struct Bounded {
  uint32_t mask, rng;
  HHFM_DEV bool accept(uint32_t word, uint32_t& val) const {
    val = mt_temper(word) & mask;
    return val <= rng;
  }
};

// per kScanBlock stream items: how many words are accepted
__global__ __launch_bounds__(256) void mt_accept_count(const uint32_t* __restrict__ x,
                                                       int64_t s0, int64_t L, Bounded bd,
                                                       int32_t* __restrict__ cnt) {
  __shared__ int red[4];
  const int64_t j0 = (int64_t)blockIdx.x * kScanBlock;
  int c = 0;
#pragma unroll
  for (int q = 0; q < kScanBlock / 256; ++q) {
    const int64_t j = j0 + q * 256 + threadIdx.x;
    uint32_t v;
    c += j < L && bd.accept(x[s0 + j], v);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, kWave);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of n block counts in place (one workgroup of 1024), the
// total (+ base) written to *total
__global__ __launch_bounds__(1024) void scan_counts(int32_t* __restrict__ cnt, int64_t n,
                                                    int64_t base, int64_t* __restrict__ total) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = base;
  __syncthreads();
  for (int64_t o = 0; o < n; o += 1024) {
    const int64_t i = o + threadIdx.x;
    const int64_t v = i < n ? cnt[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive
      const int64_t a = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += a;
      __syncthreads();
    }
    const int64_t excl = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (i < n) cnt[i] = (int32_t)excl;   // offsets fit: stream rounds < 2^31 items
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// the workgroup's exclusive prefix of flag f over its 256 threads (stream
// order: thread-major within one 256-item slice)
HHFM_DEV int block_prefix(bool f, int* wsum, int& total) {
  const uint64_t b = __ballot(f);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int in_wave = __popcll(b & ((1ull << lane) - 1));
  if (lane == 0) wsum[w] = __popcll(b);
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    before += i < w ? wsum[i] : 0;
    total += wsum[i];
  }
  __syncthreads();
  return before + in_wave;
}

// accepted words in stream order: val[k], pos[k] (stream index), k from the
// block offsets of scan_counts
__global__ __launch_bounds__(256) void mt_accept_compact(const uint32_t* __restrict__ x,
                                                         int64_t s0, int64_t L, Bounded bd,
                                                         const int32_t* __restrict__ off,
                                                         uint32_t* __restrict__ val,
                                                         int32_t* __restrict__ pos) {
  __shared__ int wsum[4];
  const int64_t j0 = (int64_t)blockIdx.x * kScanBlock;
  int64_t o = off[blockIdx.x];
#pragma unroll
  for (int q = 0; q < kScanBlock / 256; ++q) {
    const int64_t j = j0 + q * 256 + threadIdx.x;
    uint32_t v = 0;
    const bool a = j < L && bd.accept(x[s0 + j], v);
    int tot;
    const int p = block_prefix(a, wsum, tot);
    if (a) {
      val[o + p] = v;
      pos[o + p] = (int32_t)j;
    }
    o += tot;
  }
}

// per row: the code range of its key in the sorted codes, and whether the
// key's positives cover the whole range [lo, hi) (the reference would loop
// forever on such a row: reported as an error)
__global__ __launch_bounds__(256) void pf_row_ranges(
    const int32_t* __restrict__ keys, int64_t nkeys, const int64_t* __restrict__ codes,
    int64_t ncodes, const int32_t* __restrict__ rows, int64_t B, int ncols, int item_col,
    int64_t lo, int64_t hi, int64_t* __restrict__ range, int32_t* __restrict__ hang) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* row = rows + b * ncols;
    int64_t a = 0, e = nkeys;
    while (a < e) {
      const int64_t mid = (a + e) >> 1;
      int c = 0;
      const int32_t* key = keys + mid * (ncols - 1);
      for (int col = 0, c2 = 0; col < ncols && c == 0; ++col) {
        if (col == item_col) continue;
        const int32_t u = row[col], v = key[c2++];
        c = u == v ? 0 : (u < v ? -1 : 1);
      }
      if (c > 0) a = mid + 1;
      else e = mid;
    }
    bool found = a < nkeys;
    if (found) {
      const int32_t* key = keys + a * (ncols - 1);
      for (int col = 0, c2 = 0; col < ncols; ++col) {
        if (col == item_col) continue;
        found = found && row[col] == key[c2++];
      }
    }
    int64_t cs = 0, ce = 0;
    if (found) {
      auto lower = [&](int64_t code) {
        int64_t l = 0, h = ncodes;
        while (l < h) {
          const int64_t mid = (l + h) >> 1;
          if (codes[mid] < code) l = mid + 1;
          else h = mid;
        }
        return l;
      };
      cs = lower((a << 32) | (int64_t)(uint32_t)lo);
      ce = lower((a << 32) | (int64_t)(uint32_t)hi);   // items in [lo, hi) only
      if (ce - cs >= hi - lo) atomicOr(hang, 1);
    }
    range[2 * b] = cs;
    range[2 * b + 1] = ce;
  }
}

// code present in codes[cs .. ce)?
HHFM_DEV bool in_range(const int64_t* codes, int64_t cs, int64_t ce, int64_t code) {
  int64_t l = cs, h = ce;
  while (l < h) {
    const int64_t mid = (l + h) >> 1;
    if (codes[mid] < code) l = mid + 1;
    else h = mid;
  }
  return l < ce && codes[l] == code;
}

// block entries e in [e0, e1): samples[e] = lo + val[e - e0 + v0]
__global__ __launch_bounds__(256) void fill_block(const uint32_t* __restrict__ val, int64_t v0,
                                                  int64_t e0, int64_t e1, int64_t lo,
                                                  int64_t* __restrict__ samples) {
  for (int64_t e = e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e1;
       e += (int64_t)gridDim.x * blockDim.x)
    samples[e] = lo + (int64_t)val[e - e0 + v0];
}

HHFM_DEV bool sample_bad(const int64_t* samples, int64_t e, int num, const int64_t* range,
                         const int64_t* codes) {
  const int64_t b = e / num;
  const int64_t cs = range[2 * b], ce = range[2 * b + 1];
  if (cs == ce) return false;
  const int64_t rank = codes[cs] >> 32;
  return in_range(codes, cs, ce, (rank << 32) | (int64_t)(uint32_t)samples[e]);
}

__global__ __launch_bounds__(256) void bad_count(const int64_t* __restrict__ samples,
                                                 int64_t n, int num,
                                                 const int64_t* __restrict__ range,
                                                 const int64_t* __restrict__ codes,
                                                 int32_t* __restrict__ cnt) {
  __shared__ int red[4];
  const int64_t j0 = (int64_t)blockIdx.x * kScanBlock;
  int c = 0;
#pragma unroll
  for (int q = 0; q < kScanBlock / 256; ++q) {
    const int64_t j = j0 + q * 256 + threadIdx.x;
    c += j < n && sample_bad(samples, j, num, range, codes);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, kWave);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void bad_compact(const int64_t* __restrict__ samples,
                                                   int64_t n, int num,
                                                   const int64_t* __restrict__ range,
                                                   const int64_t* __restrict__ codes,
                                                   const int32_t* __restrict__ off,
                                                   int32_t* __restrict__ bad) {
  __shared__ int wsum[4];
  const int64_t j0 = (int64_t)blockIdx.x * kScanBlock;
  int64_t o = off[blockIdx.x];
#pragma unroll
  for (int q = 0; q < kScanBlock / 256; ++q) {
    const int64_t j = j0 + q * 256 + threadIdx.x;
    const bool f = j < n && sample_bad(samples, j, num, range, codes);
    int tot;
    const int p = block_prefix(f, wsum, tot);
    if (f) bad[o + p] = (int32_t)j;
    o += tot;
  }
}

// The re-draw loop (FM.py:291-293) over the rejected entries bad[prog[0] ..
// nb), the accepted values val[prog[1] .. navail) of this round.  256 entries
// at a time take the next 256 values; the first entry whose value is again a
// positive (or that finds no value left) ends the batch: the entries before
// it are final, it takes the value after its own next time.  prog = (next
// entry, next value) on exit.
__global__ __launch_bounds__(256) void redraw(const int32_t* __restrict__ bad, int64_t nb,
                                              const uint32_t* __restrict__ val, int64_t navail,
                                              int64_t lo, int num,
                                              const int64_t* __restrict__ range,
                                              const int64_t* __restrict__ codes,
                                              int64_t* __restrict__ samples,
                                              int64_t* __restrict__ prog) {
  __shared__ int first;
  __shared__ int wmin[4];
  int64_t e0 = prog[0], v = prog[1];
  while (e0 < nb && v < navail) {
    const int t = threadIdx.x;
    const int64_t e = e0 + t, vi = v + t;
    const bool live = e < nb;
    bool stop = false;
    int64_t s = 0, idx = 0;
    if (live) {
      if (vi >= navail) {
        stop = true;
      } else {
        idx = bad[e];
        s = lo + (int64_t)val[vi];
        const int64_t b = idx / num;
        const int64_t cs = range[2 * b], ce = range[2 * b + 1];
        stop = cs != ce &&
               in_range(codes, cs, ce, ((codes[cs] >> 32) << 32) | (int64_t)(uint32_t)s);
      }
    }
    // first stopping thread of the workgroup
    const uint64_t m = __ballot(stop);
    if ((t & 63) == 0) wmin[t >> 6] = m ? (t & ~63) + __ffsll((long long)m) - 1 : 256;
    __syncthreads();
    if (t == 0) first = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
    __syncthreads();
    const int f = first;
    if (live && t < f) samples[idx] = s;
    const int64_t nlive = nb - e0 < 256 ? nb - e0 : 256;
    if (f >= nlive) {        // every live entry accepted its value
      e0 += nlive;
      v += nlive;
    } else if (v + f >= navail) {   // entry e0 + f found no value: next round
      e0 += f;
      v += f;
      break;
    } else {                 // entry e0 + f drew a positive: it takes the next value
      e0 += f;
      v += f + 1;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    prog[0] = e0;
    prog[1] = v;
  }
}

// key[0..624) = x[wb .. wb + 624), pos = p (the state numpy resumes from)
__global__ void mt_state_out(const uint32_t* __restrict__ x, int64_t wb, int32_t p,
                             uint32_t* __restrict__ state) {
  for (int i = threadIdx.x; i < kMtN; i += blockDim.x) state[i] = x[wb + i];
  if (threadIdx.x == 0) state[kMtN] = (uint32_t)p;
}

__global__ void fill_const(int64_t* __restrict__ out, int64_t n, int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v;
}

static unsigned grid_of(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (unsigned)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

static int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// words generated per round: enough for the block plus 1/16 re-draws and a
// margin, at acceptance (rng + 1) / (mask + 1) >= 1/2, in whole 624-blocks
static int64_t round_words(int64_t count) {
  return align_up(2 * (count + count / 16 + 4096), kMtN);
}

struct SamplerWs {
  uint32_t* x;        // [624 + W] untempered words of the round's window
  uint32_t* val;      // [W + 1024] accepted values
  int32_t* pos;       // [W + 1024] their stream indices
  int32_t* cnt;       // [max(W, count) / 1024 + 1] block counts / offsets
  int32_t* bad;       // [count] rejected entries
  int64_t* range;     // [2B] key code range per row
  int64_t* scal;      // [8]: total, prog[2], hang
  int64_t W;
  size_t bytes;
};

static SamplerWs sampler_layout(void* base, int64_t B, int64_t count) {
  SamplerWs w{};
  w.W = round_words(count);
  char* p = reinterpret_cast<char*>(base);
  size_t o = 0;
  auto take = [&](size_t n) {
    char* r = p ? p + o : nullptr;
    o += (n + 255) & ~size_t(255);
    return r;
  };
  const int64_t nblk = (w.W > count ? w.W : count) / kScanBlock + 2;
  w.x = reinterpret_cast<uint32_t*>(take((size_t)(kMtN + w.W) * 4));
  w.val = reinterpret_cast<uint32_t*>(take((size_t)(w.W + kScanBlock) * 4));
  w.pos = reinterpret_cast<int32_t*>(take((size_t)(w.W + kScanBlock) * 4));
  w.cnt = reinterpret_cast<int32_t*>(take((size_t)nblk * 4));
  w.bad = reinterpret_cast<int32_t*>(take((size_t)(count > 0 ? count : 1) * 4));
  w.range = reinterpret_cast<int64_t*>(take((size_t)(B > 0 ? B : 1) * 16));
  w.scal = reinterpret_cast<int64_t*>(take(64));
  w.bytes = o;
  return w;
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_sample_negative_workspace(int64_t B, int32_t num, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || num < 1 || B * (int64_t)num >= ((int64_t)1 << 30)) return HHFM_EINVAL;
  *ws_bytes = sampler_layout(nullptr, B, B * num).bytes;
  return HHFM_OK;
}

extern "C" int hhfm_sample_negative(uint32_t* mt_state, int64_t lo, int64_t hi,
                                    const int32_t* rows, int64_t B, int32_t ncols,
                                    int32_t item_col, int32_t num, const int32_t* keys,
                                    int64_t nkeys, const int64_t* codes, int64_t ncodes,
                                    int64_t* samples, void* workspace, size_t ws_bytes,
                                    void* stream) {
  if (B < 0 || num < 1 || ncols < 2 || ncols > 64 || item_col < 0 || item_col >= ncols)
    return HHFM_EINVAL;
  if (lo >= hi || lo < 0 || hi > ((int64_t)1 << 31)) return HHFM_EINVAL;
  if (nkeys < 0 || ncodes < 0) return HHFM_EINVAL;
  const int64_t count = B * (int64_t)num;
  if (count >= ((int64_t)1 << 30)) return HHFM_EINVAL;
  if (count == 0) return HHFM_OK;
  if (!mt_state || !rows || !samples || !workspace || (nkeys && !keys) || (ncodes && !codes))
    return HHFM_EINVAL;
  const SamplerWs w = sampler_layout(workspace, B, count);
  if (ws_bytes < w.bytes) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t rng = (uint64_t)(hi - 1 - lo);
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  const Bounded bd{mask, (uint32_t)rng};
  int64_t hst[4] = {0, 0, 0, 0};

  // key code ranges per row; a row whose positives cover [lo, hi) would make
  // the reference loop forever
  if (hipMemsetAsync(w.scal, 0, 64, st) != hipSuccess) return (int)hipGetLastError();
  hipLaunchKernelGGL(pf_row_ranges, dim3(grid_of(B)), dim3(256), 0, st, keys, nkeys, codes,
                     ncodes, rows, B, ncols, item_col, lo, hi, w.range,
                     reinterpret_cast<int32_t*>(w.scal + 3));
  if (rng == 0) {   // randint(lo, lo + 1) draws nothing (random_bounded_uint64_fill)
    hipLaunchKernelGGL(fill_const, dim3(grid_of(count)), dim3(256), 0, st, samples, count, lo);
    if (hipMemcpyAsync(hst, w.scal, 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return (int)hipGetLastError();
    return (int32_t)hst[3] ? HHFM_EINVAL : HHFM_OK;
  }

  // round 0: the window starts with the caller's key; the stream at pos
  uint32_t pos0 = 0;
  if (hipMemcpyAsync(w.x, mt_state, kMtN * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipMemcpyAsync(&pos0, mt_state + kMtN, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return (int)hipGetLastError();
  if (pos0 > (uint32_t)kMtN) return HHFM_EINVAL;
  int64_t s0 = pos0;          // stream start within the window
  int64_t filled = 0;         // block entries placed
  int64_t nb = -1;            // rejected entries (known once the block is placed)
  int64_t last_word = -1;     // window index of the last word read
  int64_t e_next = 0;         // next rejected entry to re-draw
  for (int round = 0;; ++round) {
    if (round > 0) {          // slide: the last block becomes the window's head
      if (hipMemcpyAsync(w.x, w.x + w.W, kMtN * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return (int)hipGetLastError();
      s0 = kMtN;
    }
    hipLaunchKernelGGL(mt_generate, dim3(1), dim3(256), 0, st, w.x, (int64_t)kMtN,
                       (int64_t)kMtN + w.W);
    const int64_t L = kMtN + w.W - s0;   // stream items in this window
    const int64_t nblk = (L + kScanBlock - 1) / kScanBlock;
    hipLaunchKernelGGL(mt_accept_count, dim3((unsigned)nblk), dim3(256), 0, st, w.x, s0, L, bd,
                       w.cnt);
    hipLaunchKernelGGL(scan_counts, dim3(1), dim3(1024), 0, st, w.cnt, nblk, (int64_t)0, w.scal);
    hipLaunchKernelGGL(mt_accept_compact, dim3((unsigned)nblk), dim3(256), 0, st, w.x, s0, L, bd,
                       w.cnt, w.val, w.pos);
    if (hipMemcpyAsync(hst, w.scal, 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return (int)hipGetLastError();
    if (round == 0 && (int32_t)hst[3]) return HHFM_EINVAL;   // the reference would hang
    const int64_t navail = hst[0];
    int64_t v = 0;   // next accepted value of this round
    if (filled < count) {
      const int64_t m = navail < count - filled ? navail : count - filled;
      hipLaunchKernelGGL(fill_block, dim3(grid_of(m)), dim3(256), 0, st, w.val, (int64_t)0,
                         filled, filled + m, lo, samples);
      filled += m;
      v = m;
      if (filled == count) {   // the whole block is placed: its rejected entries
        const int64_t cb = (count + kScanBlock - 1) / kScanBlock;
        hipLaunchKernelGGL(bad_count, dim3((unsigned)cb), dim3(256), 0, st, samples, count, num,
                           w.range, codes, w.cnt);
        hipLaunchKernelGGL(scan_counts, dim3(1), dim3(1024), 0, st, w.cnt, cb, (int64_t)0,
                           w.scal + 4);
        hipLaunchKernelGGL(bad_compact, dim3((unsigned)cb), dim3(256), 0, st, samples, count,
                           num, w.range, codes, w.cnt, w.bad);
        if (hipMemcpyAsync(&nb, w.scal + 4, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
          return (int)hipGetLastError();
      }
    }
    if (nb >= 0 && e_next < nb && v < navail) {
      const int64_t pr[2] = {e_next, v};
      if (hipMemcpyAsync(w.scal + 1, pr, 16, hipMemcpyHostToDevice, st) != hipSuccess)
        return (int)hipGetLastError();
      hipLaunchKernelGGL(redraw, dim3(1), dim3(256), 0, st, w.bad, nb, w.val, navail, lo, num,
                         w.range, codes, samples, w.scal + 1);
      int64_t pg[2];
      if (hipMemcpyAsync(pg, w.scal + 1, 16, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return (int)hipGetLastError();
      e_next = pg[0];
      v = pg[1];
    }
    if (v > 0) {   // the word of the last value read this round
      int32_t p = 0;
      if (hipMemcpyAsync(&p, w.pos + (v - 1), 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return (int)hipGetLastError();
      last_word = s0 + p;
    }
    if (filled == count && nb >= 0 && e_next >= nb) break;
    if (round > 64 + count / 1024) return HHFM_EINVAL;   // runaway guard
  }
  // numpy's state after reading window word last_word: key = the 624-block
  // holding it, pos = the offset just past it (624: the next read twists)
  const int64_t e = last_word + 1;
  const int64_t b = (e - 1) / kMtN;
  hipLaunchKernelGGL(mt_state_out, dim3(1), dim3(256), 0, st, w.x, b * kMtN,
                     (int32_t)(e - b * kMtN), mt_state);
  return (int)hipGetLastError();
}
