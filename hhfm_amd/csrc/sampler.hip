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
//   * the re-draws: one workgroup walks the rejected entries in order, 1,024
//     at a time, each entry testing the next 32 values it could draw, and
//     resolves in LDS which value each entry takes (redraw_spec) — exactly
//     the reference's sequential loop; membership by per-key bitmaps of the
//     positives when the workspace holds them (hhfm_sample_negative_workspace_ex);
//   * the state after the last word read goes back to the caller (key[624],
//     pos), which np.random.set_state restores on the host.
// If the accepted values of one generation round run out, another round
// continues the stream from the last 624 words (the window slides; rounds
// end on block boundaries, so the final key is always in the window).
#include <algorithm>
#include <mutex>
#include <vector>

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

// Words [n0b, n1b) of one segment per workgroup b: n0b = n0 + b·nstride,
// n1b = min(n0b + seg, nend); the 624 words before n0b come from win + b·
// wstride (win[i] = word n0b - 624 + i), the words go to out + b·ostride at
// their positions (out[g], g in [n0b, n1b)), and with copy_win the window too
// (out[n0b - 624 + i]).  Thread t computes word n + t and then n + 227 + t —
// the second needs x[n + t] (its own first word) and x[n + t - 397 .. - 396]
// (< n, ready before the barrier), so two steps of 227 run per barrier.
__global__ __launch_bounds__(256) void mt_generate(const uint32_t* __restrict__ win,
                                                   int64_t wstride, uint32_t* __restrict__ out,
                                                   int64_t ostride, int64_t n0, int64_t nstride,
                                                   int64_t seg, int64_t nend, int copy_win) {
  __shared__ uint32_t ring[kMtRing];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t n0b = n0 + b * nstride;
  const int64_t n1b = n0b + seg < nend ? n0b + seg : nend;
  win += b * wstride;
  out += b * ostride;
  for (int i = t; i < kMtN; i += blockDim.x) {
    const int64_t g = n0b - kMtN + i;
    const uint32_t v = win[i];
    ring[g & (kMtRing - 1)] = v;
    if (copy_win) out[g] = v;
  }
  __syncthreads();
  for (int64_t n = n0b; n < n1b; n += 2 * kMtStep) {
    if (t < kMtStep) {
      const int64_t g0 = n + t, g1 = g0 + kMtStep;
      const uint32_t v0 = mt_twist(ring[(g0 - kMtN) & (kMtRing - 1)],
                                   ring[(g0 - kMtN + 1) & (kMtRing - 1)],
                                   ring[(g0 - kMtStep) & (kMtRing - 1)]);
      if (g0 < n1b) {
        ring[g0 & (kMtRing - 1)] = v0;
        out[g0] = v0;
      }
      if (g1 < n1b) {
        const uint32_t v1 = mt_twist(ring[(g1 - kMtN) & (kMtRing - 1)],
                                     ring[(g1 - kMtN + 1) & (kMtRing - 1)], v0);
        ring[g1 & (kMtRing - 1)] = v1;
        out[g1] = v1;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// MT19937 jump-ahead.  The generator is linear over GF(2): its 19,937-bit
// state (the top bit of word n and words n+1 .. n+623) advances by a matrix A
// whose characteristic polynomial P has degree 19,937, so A^J = r(A) with r =
// x^J mod P (Cayley-Hamilton), and the state J words on is Σ_i r_i·(state i
// words on): word J + k = XOR over the set bits i of r of word i + k, for k =
// 1 .. 623 (and the top bit for k = 0).  The host finds P once per process
// (Berlekamp-Massey over the top bits of 39,938 words) and r for J = 624·2^e
// by squaring; the device forms the 19,937 words after a state (mt_generate
// on one workgroup), XORs the words at r's set bits (mt_correlate, the set
// bits split over workgroups) and combines the parts (mt_combine).  A round's
// window of W words is cut into S <= 128 segments of J: their start states by
// a binary tree of jumps (log2 S levels), then every segment generated at once.
// ---------------------------------------------------------------------------
constexpr int kMtDeg = 19937;
constexpr int kPolyW = (kMtDeg + 63) / 64;          // 312 words: degree < 19,937
constexpr int kPreWords = kMtDeg + kMtN;            // a state and the 19,937 words after it
constexpr int kJumpParts = 64;                      // workgroups per jump (set-bit slices)
constexpr int kMaxSegs = 128;
constexpr int64_t kMinSegWords = (int64_t)kMtN * 32;

__global__ __launch_bounds__(256) void mt_correlate(const uint32_t* __restrict__ pre,
                                                    const uint64_t* __restrict__ r,
                                                    uint32_t* __restrict__ part) {
  const int g = blockIdx.x, j = blockIdx.y, t = threadIdx.x;
  const uint32_t* pj = pre + (int64_t)j * kPreWords;
  const int w0 = g * kPolyW / kJumpParts, w1 = (g + 1) * kPolyW / kJumpParts;
  uint32_t a0 = 0, a1 = 0, a2 = 0;   // words k = t, t + 256, t + 512 (< 624)
  const bool has2 = t + 512 < kMtN;
  // the set bits 8 at a time: their 24 loads in flight together
  int idx[8];
  int n = 0;
  auto flush = [&]() {
    uint32_t v[8][3];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < n) {
        v[q][0] = pj[idx[q] + t];
        v[q][1] = pj[idx[q] + t + 256];
        v[q][2] = has2 ? pj[idx[q] + t + 512] : 0u;
      }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < n) {
        a0 ^= v[q][0];
        a1 ^= v[q][1];
        a2 ^= v[q][2];
      }
    n = 0;
  };
  for (int w = w0; w < w1; ++w) {
    uint64_t bits = r[w];   // uniform
    while (bits) {
      idx[n++] = 64 * w + __builtin_ctzll(bits);
      bits &= bits - 1;
      if (n == 8) flush();
    }
  }
  flush();
  uint32_t* o = part + ((int64_t)j * kJumpParts + g) * kMtN;
  o[t] = a0;
  o[t + 256] = a1;
  if (has2) o[t + 512] = a2;
}

// state of segment dst(j) = dbase + j·dstride: the XOR of jump j's parts
__global__ __launch_bounds__(256) void mt_combine(const uint32_t* __restrict__ part,
                                                  uint32_t* __restrict__ st, int64_t dbase,
                                                  int64_t dstride) {
  const int j = blockIdx.x;
  for (int k = threadIdx.x; k < kMtN; k += blockDim.x) {
    uint32_t a = 0;
#pragma unroll
    for (int g = 0; g < kJumpParts; ++g) a ^= part[((int64_t)j * kJumpParts + g) * kMtN + k];
    st[(dbase + j * dstride) * kMtN + k] = a;
  }
}

// ---- host: P and x^(624·2^e) mod P, once per process ----
namespace mtjump {

using Poly = std::vector<uint64_t>;

// bit i of a polynomial = the coefficient of x^i
inline bool bit(const Poly& a, int64_t i) { return (a[i >> 6] >> (i & 63)) & 1u; }

// 64 bits of v starting at bit pos (zero past the end)
inline uint64_t bits64(const Poly& v, int64_t pos) {
  const int64_t w = pos >> 6;
  const int sh = (int)(pos & 63);
  const uint64_t lo = w < (int64_t)v.size() ? v[w] : 0;
  if (sh == 0) return lo;
  const uint64_t hi = w + 1 < (int64_t)v.size() ? v[w + 1] : 0;
  return (lo >> sh) | (hi << (64 - sh));
}

// a ^= b << m
inline void xor_shifted(Poly& a, const Poly& b, int64_t m) {
  const int64_t ws = m >> 6;
  const int sh = (int)(m & 63);
  for (int64_t i = (int64_t)b.size() - 1; i >= 0; --i) {
    if (!b[i]) continue;
    if (i + ws < (int64_t)a.size()) a[i + ws] ^= b[i] << sh;
    if (sh && i + ws + 1 < (int64_t)a.size()) a[i + ws + 1] ^= b[i] >> (64 - sh);
  }
}

// the characteristic polynomial of MT19937's state map: Berlekamp-Massey over
// the top bits of the words of any nonzero state (numpy's seed-5489 key)
inline Poly char_poly() {
  const int64_t N = 2 * (int64_t)kMtDeg + 64;
  std::vector<uint32_t> x((size_t)N);
  x[0] = 5489u;
  for (int i = 1; i < kMtN; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
  for (int64_t i = kMtN; i < N; ++i) {
    const uint32_t y = (x[i - kMtN] & 0x80000000u) | (x[i - kMtN + 1] & 0x7fffffffu);
    x[i] = x[i - kMtStep] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  // R_k = s_{N-1-k} (s_n = top bit of word n): Σ_i C_i s_{n-i} = <C, R from N-1-n>
  const int64_t NW = (N + 63) / 64 + 2;
  Poly R((size_t)NW, 0);
  for (int64_t n = 0; n < N; ++n)
    if (x[n] >> 31) R[(N - 1 - n) >> 6] |= 1ull << ((N - 1 - n) & 63);
  Poly C((size_t)NW, 0), Bp((size_t)NW, 0);
  C[0] = Bp[0] = 1;
  int64_t L = 0, m = 1;
  for (int64_t n = 0; n < N; ++n) {
    uint64_t acc = 0;
    const int64_t off = N - 1 - n;
    for (int64_t w = 0; w <= (L >> 6); ++w) acc ^= C[w] & bits64(R, off + 64 * w);
    if (!__builtin_parityll(acc)) {
      ++m;
    } else if (2 * L <= n) {
      Poly T = C;
      xor_shifted(C, Bp, m);
      L = n + 1 - L;
      Bp = T;
      m = 1;
    } else {
      xor_shifted(C, Bp, m);
      ++m;
    }
  }
  if (L != kMtDeg) return {};
  Poly P((size_t)kPolyW + 1, 0);   // P_i = C_{L-i}
  for (int64_t i = 0; i <= L; ++i)
    if (bit(C, L - i)) P[i >> 6] |= 1ull << (i & 63);
  return P;
}

struct Tables {
  Poly P;
  std::vector<Poly> Pshift;   // P << r, r < 64
  std::vector<Poly> pw;       // pw[t] = x^(624·2^t) mod P
  bool ok = false;
};

// a^2 mod P (a of degree < 19,937)
inline Poly sqr_mod(const Tables& T, const Poly& a) {
  Poly q((size_t)2 * kPolyW + 2, 0);
  auto spread = [](uint32_t v) {
    uint64_t r = v;
    r = (r | (r << 16)) & 0x0000FFFF0000FFFFull;
    r = (r | (r << 8)) & 0x00FF00FF00FF00FFull;
    r = (r | (r << 4)) & 0x0F0F0F0F0F0F0F0Full;
    r = (r | (r << 2)) & 0x3333333333333333ull;
    r = (r | (r << 1)) & 0x5555555555555555ull;
    return r;
  };
  for (int i = 0; i < kPolyW; ++i) {
    q[2 * i] = spread((uint32_t)a[i]);
    q[2 * i + 1] = spread((uint32_t)(a[i] >> 32));
  }
  for (int64_t k = 2 * (int64_t)(kMtDeg - 1); k >= kMtDeg; --k) {
    if (!bit(q, k)) continue;
    const int64_t d = k - kMtDeg;
    const Poly& ps = T.Pshift[d & 63];
    const int64_t w0 = d >> 6;
    for (size_t i = 0; i < ps.size() && w0 + (int64_t)i < (int64_t)q.size(); ++i) q[w0 + i] ^= ps[i];
  }
  q.resize(kPolyW);
  return q;
}

inline Tables& tables() {
  static Tables T;
  return T;
}
inline std::mutex& tables_mu() {
  static std::mutex mu;
  return mu;
}

// x^(624·2^t) mod P for t = 0 .. tmax (computed on first need); false when P
// could not be found (the caller then generates serially)
inline bool powers(int tmax, std::vector<Poly>& out) {
  std::lock_guard<std::mutex> lk(tables_mu());
  Tables& T = tables();
  if (T.P.empty() && !T.ok) {
    T.P = char_poly();
    T.ok = !T.P.empty();
    if (T.ok) {
      T.Pshift.assign(64, Poly((size_t)kPolyW + 2, 0));
      for (int r = 0; r < 64; ++r) xor_shifted(T.Pshift[r], T.P, r);
      Poly x624((size_t)kPolyW, 0);
      x624[kMtN >> 6] = 1ull << (kMtN & 63);
      T.pw.push_back(x624);
    }
  }
  if (!T.ok) return false;
  while ((int)T.pw.size() <= tmax) T.pw.push_back(sqr_mod(T, T.pw.back()));
  out.assign(T.pw.begin(), T.pw.begin() + tmax + 1);
  return true;
}

}  // namespace mtjump

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

// ---------------------------------------------------------------------------
// The re-draw walk (FM.py:291-293) over the rejected entries, speculative: the
// walk's only sequential state is the shift s = values consumed - entries
// finished; entry t of a batch draws value v0 + t + s, and each positive it
// draws moves s up by one.  So every entry of a batch of kRdT tests the kRdD
// values v0 + t + d, d < kRdD, at once (bit d of ok[t]: not a positive, or
// past the round's values), and the shifts are resolved in LDS: wave w takes
// entries 64w .. 64w + 63 from every start shift (lane L = start L), giving
// per start the entry's chosen shift d_t = the first ok bit >= s, and s := d_t
// for the next entry; the 16 segment maps compose in order.  The walk stops
// at the first entry whose shift would pass kRdD - 1 (it then resumes with
// the next batch) or whose value lies past the round's values.  The values
// assigned are the sequential loop's, exactly.  Membership by the key
// bitmaps (BM) or the binary searches of hhfm_pf_contains.
// ---------------------------------------------------------------------------
constexpr int kRdT = 1024, kRdD = 32, kRdW = kRdT / 64;
constexpr int kRdStop = 1 << 16;

template <bool BM>
__global__ __launch_bounds__(kRdT) void redraw_spec(
    const int32_t* __restrict__ bad, int64_t nb, const int32_t* __restrict__ er,
    const uint32_t* __restrict__ bm, int64_t bmw, const uint32_t* __restrict__ val,
    int64_t navail, int64_t lo, int num, const int64_t* __restrict__ range,
    const int64_t* __restrict__ codes, int64_t* __restrict__ samples,
    int64_t* __restrict__ prog) {
  __shared__ uint32_t okm[kRdT];
  __shared__ uint32_t vals[kRdT + kRdD];
  // [segment][start shift][entry] -> d, rows of 68 B (17 banks apart: the
  // lanes' dword writes do not collide)
  __shared__ uint32_t traj[kRdW][kRdD][17];
  __shared__ int32_t fmap[kRdW][kRdD];       // end shift, or kRdStop | entry
  __shared__ int32_t seg_start[kRdW];
  __shared__ int32_t ctl[2];                 // stop entry, final shift
  __shared__ int32_t wmin[kRdW];
  const int t = threadIdx.x, w = t >> 6, L = t & 63;
  int64_t e0 = prog[0], v0 = prog[1];
  while (e0 < nb && v0 < navail) {
    const int64_t e = e0 + t;
    const bool live = e < nb;
    const int nlive = nb - e0 < kRdT ? (int)(nb - e0) : kRdT;
    for (int x = t; x < kRdT + kRdD; x += kRdT) {
      const int64_t j = v0 + x;
      vals[x] = j < navail ? val[j] : 0u;
    }
    int64_t idx = 0;
    int32_t rank = -1;
    int64_t cs = 0, ce = 0;
    if (live) {
      idx = bad[e];
      if constexpr (BM) {
        rank = er[e];
      } else {
        const int64_t b = idx / num;
        cs = range[2 * b];
        ce = range[2 * b + 1];
      }
    }
    __syncthreads();
    uint32_t m = 0xffffffffu;   // dead entries: accept at any shift
    if (live) {
      m = 0;
#pragma unroll 4
      for (int d = 0; d < kRdD; ++d) {
        const int64_t j = v0 + t + d;
        const uint32_t u = vals[t + d];
        bool pos = false;
        if (j < navail) {
          if constexpr (BM) {
            pos = rank >= 0 && ((bm[(int64_t)rank * bmw + (u >> 5)] >> (u & 31)) & 1u);
          } else {
            pos = cs != ce && in_range(codes, cs, ce,
                                       ((codes[cs] >> 32) << 32) | (int64_t)(uint32_t)(lo + u));
          }
        }
        m |= (pos ? 0u : 1u) << d;
      }
    }
    okm[t] = m;
    __syncthreads();
    if (L < kRdD) {   // segment w from start shift L: the masks 16 at a time
      int sh = L, stop = -1;
      const uint4* om = reinterpret_cast<const uint4*>(okm + 64 * w);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint4 q4[4] = {om[4 * c], om[4 * c + 1], om[4 * c + 2], om[4 * c + 3]};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t q[4] = {q4[h].x, q4[h].y, q4[h].z, q4[h].w};
          uint32_t packed = 0;
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            if (stop < 0) {
              const uint32_t mm = q[x] >> sh;
              if (mm == 0u) stop = 16 * c + 4 * h + x;
              else sh += __builtin_ctz(mm);
            }
            packed |= (uint32_t)sh << (8 * x);
          }
          traj[w][L][4 * c + h] = packed;
        }
      }
      fmap[w][L] = stop >= 0 ? (kRdStop | stop) : sh;
    }
    __syncthreads();
    if (w == 0) {   // compose the segment maps in order (lane L holds start L)
      int f[kRdW];
#pragma unroll
      for (int g = 0; g < kRdW; ++g) f[g] = L < kRdD ? fmap[g][L] : 0;
      int sh = 0, stop = kRdT;
#pragma unroll
      for (int g = 0; g < kRdW; ++g) {
        if (stop == kRdT) {
          if (L == 0) seg_start[g] = sh;
          const int r = __builtin_amdgcn_readlane(f[g], sh);
          if (r & kRdStop) stop = 64 * g + (r & 0xff);
          else sh = r;
        }
      }
      if (L == 0) {
        ctl[0] = stop;
        ctl[1] = sh;
      }
    }
    __syncthreads();
    const int stop = ctl[0];
    int d = 0;
    bool over = false;
    if (live && t < stop) {
      d = (int)((traj[w][seg_start[w]][L >> 2] >> (8 * (L & 3))) & 0xffu);
      over = v0 + t + d >= navail;
    }
    const uint64_t ob = __ballot(over);
    if (L == 0) wmin[w] = ob ? 64 * w + __ffsll((long long)ob) - 1 : kRdT;
    __syncthreads();
    int first_over = kRdT;
    for (int g = 0; g < kRdW; ++g) first_over = min(first_over, wmin[g]);
    const int f = min(min(stop, first_over), nlive);
    if (live && t < f) samples[idx] = lo + (int64_t)vals[t + d];
    if (first_over < stop && first_over < nlive) {   // the round's values ran out
      e0 += first_over;
      v0 = navail;
      break;
    } else if (stop < nlive) {   // entry `stop` drew kRdD - s positives: resume there
      e0 += stop;
      v0 += stop + kRdD;
    } else {
      e0 += nlive;
      v0 += nlive + ctl[1];
    }
    __syncthreads();
  }
  if (t == 0) {
    prog[0] = e0;
    prog[1] = v0;
  }
}

// bitmaps of the keys' positives over [lo, hi): bit (item - lo) of key rank r
// at bm[r * bmw + ...] (bm zeroed before)
__global__ __launch_bounds__(256) void pf_bitmap(const int64_t* __restrict__ codes, int64_t ncodes,
                                                 int64_t lo, int64_t hi, int64_t bmw,
                                                 uint32_t* __restrict__ bm) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncodes;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t code = codes[c];
    const int64_t item = (int64_t)(uint32_t)code, r = code >> 32;
    if (item >= lo && item < hi) {
      const int64_t u = item - lo;
      atomicOr(bm + r * bmw + (u >> 5), 1u << (u & 31));
    }
  }
}

// per rejected entry: its row's key rank (-1: no positives)
__global__ __launch_bounds__(256) void bad_rank(const int32_t* __restrict__ bad, int64_t nb, int num,
                                                const int64_t* __restrict__ range,
                                                const int64_t* __restrict__ codes,
                                                int32_t* __restrict__ er) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nb;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = bad[e] / num;
    const int64_t cs = range[2 * b], ce = range[2 * b + 1];
    er[e] = cs != ce ? (int32_t)(codes[cs] >> 32) : -1;
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
  uint32_t* jst;      // [kMaxSegs][624] segment start states (jump-ahead)
  uint32_t* jpre;     // [kMaxSegs / 2][kPreWords] a state + the 19,937 words after it
  uint32_t* jpart;    // [kMaxSegs / 2][kJumpParts][624] partial jumped states
  uint64_t* jr;       // [7][kPolyW] jump polynomials of the tree's levels
  int32_t* er;        // [count] key rank per rejected entry (bitmap path)
  uint32_t* bm;       // [nkeys][bmw] key bitmaps over [lo, hi) (bitmap path)
  int64_t W;
  size_t bytes;
};

// key bitmaps when they take at most this much workspace
constexpr size_t kBitmapCap = size_t(256) << 20;

static size_t bitmap_bytes(int64_t lo, int64_t hi, int64_t nkeys) {
  if (hi <= lo || nkeys <= 0) return 0;
  const size_t b = (size_t)nkeys * (size_t)((hi - lo + 31) / 32) * 4;
  return b <= kBitmapCap ? b : 0;
}

static SamplerWs sampler_layout(void* base, int64_t B, int64_t count, size_t bm_bytes = 0) {
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
  w.jst = reinterpret_cast<uint32_t*>(take((size_t)kMaxSegs * kMtN * 4));
  w.jpre = reinterpret_cast<uint32_t*>(take((size_t)(kMaxSegs / 2) * kPreWords * 4));
  w.jpart = reinterpret_cast<uint32_t*>(take((size_t)(kMaxSegs / 2) * kJumpParts * kMtN * 4));
  w.jr = reinterpret_cast<uint64_t*>(take((size_t)7 * kPolyW * 8));
  if (bm_bytes) {
    w.er = reinterpret_cast<int32_t*>(take((size_t)(count > 0 ? count : 1) * 4));
    w.bm = reinterpret_cast<uint32_t*>(take(bm_bytes));
  }
  w.bytes = o;
  return w;
}

// words [624, 624 + Wr) of the round's window from its first 624 (x[0 ..
// 624)): segments of J = 624·2^e words (at least 32 blocks, at most kMaxSegs
// of them), their start states by the jump tree, then all generated at once;
// one workgroup when the window is shorter than two segments
static hipError_t mt_fill(const SamplerWs& w, int64_t Wr, hipStream_t st) {
  const int64_t nend = kMtN + Wr;
  int e = 0;
  while (((int64_t)kMtN << e) < kMinSegWords) ++e;
  while (((int64_t)kMtN << e) * kMaxSegs < Wr) ++e;
  const int64_t J = (int64_t)kMtN << e;
  const int64_t S = (Wr + J - 1) / J;
  int lv = 0;
  while (((int64_t)1 << lv) < S) ++lv;
  std::vector<mtjump::Poly> pw;
  if (S < 2 || !mtjump::powers(e + lv - 1, pw)) {
    hipLaunchKernelGGL(mt_generate, dim3(1), dim3(256), 0, st, w.x, (int64_t)0, w.x, (int64_t)0,
                       (int64_t)kMtN, (int64_t)0, Wr, nend, 0);
    return hipGetLastError();
  }
  // the levels' polynomials: x^(J·2^l) mod P = pw[e + l] (a pageable copy:
  // staged by the runtime before hipMemcpyAsync returns)
  std::vector<uint64_t> up((size_t)lv * kPolyW);
  for (int l = 0; l < lv; ++l)
    std::copy(pw[e + l].begin(), pw[e + l].begin() + kPolyW, up.begin() + (size_t)l * kPolyW);
  hipError_t err = hipMemcpyAsync(w.jr, up.data(), up.size() * 8, hipMemcpyHostToDevice, st);
  if (err == hipSuccess) err = hipMemcpyAsync(w.jst, w.x, kMtN * 4, hipMemcpyDeviceToDevice, st);
  if (err != hipSuccess) return err;
  for (int l = lv - 1; l >= 0; --l) {
    const int64_t step = (int64_t)1 << l;   // segments jumped at this level
    const int64_t nj = (S - step + 2 * step - 1) / (2 * step);
    if (nj <= 0) continue;
    // jump j: from segment 2j·step to 2j·step + step
    hipLaunchKernelGGL(mt_generate, dim3((unsigned)nj), dim3(256), 0, st, w.jst, 2 * step * kMtN,
                       w.jpre, (int64_t)kPreWords, (int64_t)kMtN, (int64_t)0, (int64_t)kMtDeg,
                       (int64_t)kPreWords, 1);
    hipLaunchKernelGGL(mt_correlate, dim3(kJumpParts, (unsigned)nj), dim3(256), 0, st, w.jpre,
                       w.jr + (size_t)l * kPolyW, w.jpart);
    hipLaunchKernelGGL(mt_combine, dim3((unsigned)nj), dim3(256), 0, st, w.jpart, w.jst, step,
                       2 * step);
  }
  hipLaunchKernelGGL(mt_generate, dim3((unsigned)S), dim3(256), 0, st, w.jst, (int64_t)kMtN, w.x,
                     (int64_t)0, (int64_t)kMtN, J, J, nend, 0);
  return hipGetLastError();
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_sample_negative_workspace(int64_t B, int32_t num, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || num < 1 || B * (int64_t)num >= ((int64_t)1 << 30)) return HHFM_EINVAL;
  *ws_bytes = sampler_layout(nullptr, B, B * num).bytes;
  return HHFM_OK;
}

extern "C" int hhfm_sample_negative_workspace_ex(int64_t B, int32_t num, int64_t lo, int64_t hi,
                                                 int64_t nkeys, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || num < 1 || B * (int64_t)num >= ((int64_t)1 << 30) || nkeys < 0)
    return HHFM_EINVAL;
  *ws_bytes = sampler_layout(nullptr, B, B * num, bitmap_bytes(lo, hi, nkeys)).bytes;
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
  if (ws_bytes < sampler_layout(nullptr, B, count).bytes) return HHFM_EWORKSPACE;
  // the bitmap path when the workspace was sized for it (_ex)
  const size_t bmb = bitmap_bytes(lo, hi, nkeys);
  const bool use_bm = bmb && ncodes && ws_bytes >= sampler_layout(nullptr, B, count, bmb).bytes;
  const SamplerWs w = sampler_layout(workspace, B, count, use_bm ? bmb : 0);
  const int64_t bmw = (hi - lo + 31) / 32;
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
  // words per round from this draw's acceptance (rng + 1) / (mask + 1): the
  // block, 1/16 re-draws and a margin (a shortfall only costs another round),
  // within the workspace's worst-case window (acceptance >= 1/2)
  const double acc = ((double)rng + 1.0) / ((double)mask + 1.0);
  int64_t Wr = align_up((int64_t)((double)(count + count / 16 + 4096) / acc * 1.02) + 4096, kMtN);
  Wr = Wr < w.W ? Wr : w.W;
  // safety bound on rounds (host loop): 16x the words of a worst case where
  // every entry is a positive until (hi - lo) draws on average — pf_row_ranges
  // already refuses the only endless case (a key covering [lo, hi))
  const double max_rounds =
      64.0 + 16.0 * (double)count * (double)(hi - lo) / acc / (double)Wr;

  // key code ranges per row; a row whose positives cover [lo, hi) would make
  // the reference loop forever
  if (hipMemsetAsync(w.scal, 0, 64, st) != hipSuccess) return (int)hipGetLastError();
  if (use_bm) {
    if (hipMemsetAsync(w.bm, 0, bmb, st) != hipSuccess) return (int)hipGetLastError();
    hipLaunchKernelGGL(pf_bitmap, dim3(grid_of(ncodes)), dim3(256), 0, st, codes, ncodes, lo, hi,
                       bmw, w.bm);
  }
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
      if (hipMemcpyAsync(w.x, w.x + Wr, kMtN * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return (int)hipGetLastError();
      s0 = kMtN;
    }
    if (mt_fill(w, Wr, st) != hipSuccess) return (int)hipGetLastError();
    const int64_t L = kMtN + Wr - s0;   // stream items in this window
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
        if (use_bm && nb > 0)
          hipLaunchKernelGGL(bad_rank, dim3(grid_of(nb)), dim3(256), 0, st, w.bad, nb, num,
                             w.range, codes, w.er);
      }
    }
    if (nb >= 0 && e_next < nb && v < navail) {
      const int64_t pr[2] = {e_next, v};
      if (hipMemcpyAsync(w.scal + 1, pr, 16, hipMemcpyHostToDevice, st) != hipSuccess)
        return (int)hipGetLastError();
      if (use_bm)
        hipLaunchKernelGGL(redraw_spec<true>, dim3(1), dim3(kRdT), 0, st, w.bad, nb, w.er, w.bm,
                           bmw, w.val, navail, lo, num, w.range, codes, samples, w.scal + 1);
      else
        hipLaunchKernelGGL(redraw_spec<false>, dim3(1), dim3(kRdT), 0, st, w.bad, nb, w.er, w.bm,
                           bmw, w.val, navail, lo, num, w.range, codes, samples, w.scal + 1);
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
    if (round > max_rounds) return HHFM_EINVAL;   // runaway guard (a defect, not a draw)
  }
  // numpy's state after reading window word last_word: key = the 624-block
  // holding it, pos = the offset just past it (624: the next read twists)
  const int64_t e = last_word + 1;
  const int64_t b = (e - 1) / kMtN;
  hipLaunchKernelGGL(mt_state_out, dim3(1), dim3(256), 0, st, w.x, b * kMtN,
                     (int32_t)(e - b * kMtN), mt_state);
  return (int)hipGetLastError();
}
