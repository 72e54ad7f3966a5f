// Shared LDS-tiled MFMA GEMM (K3 DeepFM MLP, K4 AFM attention).
//   C = epi(A · Bt^T + bias), tile 128 x 128 per 256-thread workgroup
//   (4 waves 2x2, 64x64 each), double-buffered LDS, one barrier per K-step.
//   bf16 mode: v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
//   f32  mode: v_mfma_f32_16x16x4_f32 (exact fp32 fmaf chains).
// A operand: dense rows, rows gathered as the concat of F field embeddings,
// or (f32) AFM pair products E[x_i] ⊙ E[x_j].  Epilogues: 0 = bias+ReLU
// store, 1 = bias+ReLU+dot(v) over the tile -> per-row partial,
// 2 = grouped dot over G-column groups (AFM attention logits).
#pragma once
#include "topk_common.h"

namespace hhfm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

// fp32 -> three bf16 pieces, x == p0 + p1 + p2 exactly for normal x: p0 =
// RNE(x) takes the top 8 significant bits, x - p0 is exact (Sterbenz) and
// keeps <= 16, the next piece 8 of those, the last piece the rest.
HHFM_DEV uint32_t bf16x2_rne(float lo, float hi) {   // v_cvt_pk_bf16_f32
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  const bf16x2v v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
HHFM_DEV void split3x8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  u32x4_t w0, w1, w2;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const float a = x[2 * v], b = x[2 * v + 1];
    const uint32_t u0 = bf16x2_rne(a, b);
    const float ra = a - __uint_as_float(u0 << 16), rb = b - __uint_as_float(u0 & 0xffff0000u);
    const uint32_t u1 = bf16x2_rne(ra, rb);
    const uint32_t u2 = bf16x2_rne(ra - __uint_as_float(u1 << 16),
                                   rb - __uint_as_float(u1 & 0xffff0000u));
    w0[v] = u0;
    w1[v] = u1;
    w2[v] = u2;
  }
  p0 = __builtin_bit_cast(bf16x8, w0);
  p1 = __builtin_bit_cast(bf16x8, w1);
  p2 = __builtin_bit_cast(bf16x8, w2);
}

// x with at most 16 significant bits (a product of two bf16 values, exact in
// fp32) -> two bf16 pieces, x == p0 + p1 exactly: x − RNE(x) is a multiple of
// x's last bit no larger than 2^7 of them, so 8 bits hold it (split3x8's
// third piece of such x is +0).
HHFM_DEV void split2x8(const float (&x)[8], bf16x8& p0, bf16x8& p1) {
  u32x4_t w0, w1;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const float a = x[2 * v], b = x[2 * v + 1];
    const uint32_t u0 = bf16x2_rne(a, b);
    w0[v] = u0;
    w1[v] = bf16x2_rne(a - __uint_as_float(u0 << 16), b - __uint_as_float(u0 & 0xffff0000u));
  }
  p0 = __builtin_bit_cast(bf16x8, w0);
  p1 = __builtin_bit_cast(bf16x8, w1);
}

constexpr int GBM = 128, GBN = 128;

// Column order of the projected layer 0 for the bf16 fused DeepFM kernel
// (dfm_fused.hip): unit n = 32t + 8g + 4h + e of a 32x32x16 result tile sits
// in lane half h, register 4g + e, so storing it at 32t + 16h + 4g + e makes
// each lane's 16 units of a tile contiguous.
HHFM_DEV int dfm_proj_pos(int n) {
  return (n & ~31) | (((n >> 2) & 1) << 4) | (((n >> 3) & 3) << 2) | (n & 3);
}

struct GemmArgs {
  int64_t M;
  int N, K;
  const void* A;       // dense A [M][lda] in compute dtype
  int64_t lda;
  int a_src_bf16;       // dense A stored as bf16 while computing in f32
  int pair_mode;        // A[r] = T[idx[r/P][i]] ⊙ T[idx[r/P][j]] (AFM pairs, f32 only)
  int P;                // pairs per row in pair mode
  const int32_t* gidx;  // gather mode: idx [M][F]; A[m] = concat_f T[idx[m][f]]
  const void* T;        // table [Mtab][kf]
  int64_t Mtab;
  int F, kf, t_bf16;    // table row width / dtype
  const void* Bt;       // weights, transposed: [N][ldb] (K contiguous), compute dtype
  int64_t ldb;
  int b_src_bf16;       // Bt stored as bf16 while computing in f32
  const float* rowbias; // epilogue 0: added to every element of row m (or null)
  const float* bias;    // [N] or null
  int relu;
  void* C;              // epilogue store: [M][ldc]
  int64_t ldc;
  int c_bf16;
  const float* dotv;    // epilogue dot: v[N] (grouped dot: v[G], repeated per group)
  float* partial;       // [M][gridDim.y] (grouped dot: [M][ldp])
  int G;                // grouped dot: group size (16, 32 or 64)
  int mod;              // grouped dot: bias / v are indexed by n % mod
  int64_t ldp;          // grouped dot: row stride of partial
  int c_perm32;         // epilogue 0: column n stored at dfm_proj_pos(n)
  int ksplit;           // split-K (epilogue 0): blockIdx.z covers K range
                        // [z*ksplit, (z+1)*ksplit), ksplit % 32 == 0, and
  int64_t cz_stride;    // stores to C + z*cz_stride (elements); 0 = no split
  // FM pair table C[a][b] (dfm_fm_pairs): per field f, [2f] = 0x7fffffff − min
  // id, [2f+1] = max id; a tile no (f < g) pair of ranges touches is skipped
  // (its entries are never read).  Null: every tile.
  const int32_t* tile_ranges;
  int tr_F;
};

// (i, j) of pair p among i<j<F in the reference's loop order (AFM.py:107-110)
HHFM_DEV void pair_ij(int p, int F, int& i, int& j) {
  i = 0;
  while (p >= F - 1 - i) {
    p -= F - 1 - i;
    ++i;
  }
  j = i + 1 + p;
}

HHFM_DEV uint16_t f2bf(float f) {  // round to nearest even (finite inputs)
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Load the 16-B chunk of A at (row m, k offset kk) in compute dtype.
template <bool BF>
HHFM_DEV u32x4_t load_a_chunk(const GemmArgs& g, int64_t m, int kk) {
  u32x4_t z = {0, 0, 0, 0};
  if (m >= g.M || kk >= g.K) return z;
  if (!g.gidx) {
    if (!BF && g.a_src_bf16) {  // 4 bf16 -> 4 f32
      const uint2 x = *reinterpret_cast<const uint2*>(
          reinterpret_cast<const uint16_t*>(g.A) + m * g.lda + kk);
      u32x4_t r = {x.x << 16, x.x & 0xffff0000u, x.y << 16, x.y & 0xffff0000u};
      return r;
    }
    const char* p = reinterpret_cast<const char*>(g.A) + (m * g.lda + kk) * (BF ? 2 : 4);
    return *reinterpret_cast<const u32x4_t*>(p);
  }
  if (!BF && g.pair_mode) {
    const int64_t row = m / g.P;
    int i, j;
    pair_ij((int)(m - row * g.P), g.F, i, j);
    const int32_t a = clamp_id(g.gidx[row * g.F + i], g.Mtab);
    const int32_t b = clamp_id(g.gidx[row * g.F + j], g.Mtab);
    float x[4], y[4];
    if (g.t_bf16) {
      const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(g.T) + (int64_t)a * g.kf + kk);
      const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(g.T) + (int64_t)b * g.kf + kk);
      x[0] = __uint_as_float(u.x << 16); x[1] = __uint_as_float(u.x & 0xffff0000u);
      x[2] = __uint_as_float(u.y << 16); x[3] = __uint_as_float(u.y & 0xffff0000u);
      y[0] = __uint_as_float(v.x << 16); y[1] = __uint_as_float(v.x & 0xffff0000u);
      y[2] = __uint_as_float(v.y << 16); y[3] = __uint_as_float(v.y & 0xffff0000u);
    } else {
      const float4 u = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g.T) + (int64_t)a * g.kf + kk);
      const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g.T) + (int64_t)b * g.kf + kk);
      x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
      y[0] = v.x; y[1] = v.y; y[2] = v.z; y[3] = v.w;
    }
    u32x4_t r = {__float_as_uint(x[0] * y[0]), __float_as_uint(x[1] * y[1]),
                 __float_as_uint(x[2] * y[2]), __float_as_uint(x[3] * y[3])};
    return r;
  }
  const int f = kk / g.kf, c = kk - f * g.kf;
  const int32_t id = clamp_id(g.gidx[m * g.F + f], g.Mtab);
  if (g.t_bf16) {
    const uint16_t* row = reinterpret_cast<const uint16_t*>(g.T) + (int64_t)id * g.kf + c;
    if (BF) return *reinterpret_cast<const u32x4_t*>(row);   // 8 bf16
    const uint2 x = *reinterpret_cast<const uint2*>(row);      // 4 bf16 -> 4 f32
    u32x4_t r = {x.x << 16, x.x & 0xffff0000u, x.y << 16, x.y & 0xffff0000u};
    return r;
  }
  const float* row = reinterpret_cast<const float*>(g.T) + (int64_t)id * g.kf + c;
  if (!BF) return *reinterpret_cast<const u32x4_t*>(row);      // 4 f32
  const float4 a = *reinterpret_cast<const float4*>(row);      // 8 f32 -> 8 bf16
  const float4 b = *reinterpret_cast<const float4*>(row + 4);
  u32x4_t r = {(uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16),
               (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16),
               (uint32_t)f2bf(b.x) | ((uint32_t)f2bf(b.y) << 16),
               (uint32_t)f2bf(b.z) | ((uint32_t)f2bf(b.w) << 16)};
  return r;
}

template <bool BF>
HHFM_DEV u32x4_t load_b_chunk(const GemmArgs& g, int n, int kk) {
  u32x4_t z = {0, 0, 0, 0};
  if (n >= g.N || kk >= g.K) return z;
  if (!BF && g.b_src_bf16) {  // 4 bf16 -> 4 f32
    const uint2 x = *reinterpret_cast<const uint2*>(
        reinterpret_cast<const uint16_t*>(g.Bt) + (int64_t)n * g.ldb + kk);
    u32x4_t r = {x.x << 16, x.x & 0xffff0000u, x.y << 16, x.y & 0xffff0000u};
    return r;
  }
  const char* p = reinterpret_cast<const char*>(g.Bt) + ((int64_t)n * g.ldb + kk) * (BF ? 2 : 4);
  return *reinterpret_cast<const u32x4_t*>(p);
}

template <bool BF, int EPI>
__global__ __launch_bounds__(256) void gemm_mfma(GemmArgs g) {
  constexpr int EL = BF ? 8 : 4;          // elements per 16-B chunk
  constexpr int BK = BF ? 32 : 16;        // K per stage (= 4 chunks per row)
  constexpr int CPR = BK / EL;            // chunks per tile row (4)
  constexpr int LDR = CPR + 1;            // LDS row stride in chunks (+1 pad)
  __shared__ u32x4_t As[2][GBM * LDR];
  __shared__ u32x4_t Bs[2][GBN * LDR];
  __shared__ float red[2][GBM];

  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int64_t m0 = (int64_t)blockIdx.x * GBM;
  const int n0 = blockIdx.y * GBN;
  if (g.tile_ranges) {   // uniform: the whole block leaves before any barrier
    bool need = false;
    for (int f = 0; f + 1 < g.tr_F && !need; ++f) {
      const int64_t flo = 0x7fffffff - g.tile_ranges[2 * f], fhi = g.tile_ranges[2 * f + 1];
      if (fhi < m0 || flo >= m0 + GBM) continue;
      for (int h = f + 1; h < g.tr_F && !need; ++h) {
        const int hlo = 0x7fffffff - g.tile_ranges[2 * h], hhi = g.tile_ranges[2 * h + 1];
        need = !(hhi < n0 || hlo >= n0 + GBN);
      }
    }
    if (!need) return;
  }
  const int kb = g.ksplit ? (int)blockIdx.z * g.ksplit : 0;
  const int ke = g.ksplit ? min(g.K, kb + g.ksplit) : g.K;
  const int nk = (ke - kb + BK - 1) / BK;

  // each thread stages 2 A chunks and 2 B chunks per K-step
  u32x4_t ra[2], rb[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, r = c / CPR, p = c % CPR;
      ra[i] = load_a_chunk<BF>(g, m0 + r, kb + kt * BK + p * EL);
      rb[i] = load_b_chunk<BF>(g, n0 + r, kb + kt * BK + p * EL);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, r = c / CPR, p = c % CPR;
      As[buf][r * LDR + p] = ra[i];
      Bs[buf][r * LDR + p] = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const int ar = wm * 64 + (l & 15), br = wn * 64 + (l & 15), ch = l >> 4;
    if constexpr (BF) {
      // 16x16x32: lane holds A[row][8*ch .. +8], B[8*ch .. +8][col]
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const u32x4_t x = As[buf][(ar + 16 * a) * LDR + ch];
        fa[a] = __builtin_bit_cast(bf16x8, x);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const u32x4_t x = Bs[buf][(br + 16 * b) * LDR + ch];
        fb[b] = __builtin_bit_cast(bf16x8, x);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    } else {
      // 16x16x4 f32: lane reads k = 4*ch .. +4 and feeds MFMA j with k = 4*ch + j
      u32x4_t fa[4], fb[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) fa[a] = As[buf][(ar + 16 * a) * LDR + ch];
#pragma unroll
      for (int b = 0; b < 4; ++b) fb[b] = Bs[buf][(br + 16 * b) * LDR + ch];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                __uint_as_float(fa[a][j]), __uint_as_float(fb[b][j]), acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C/D layout col = l&15, row = 4*(l>>4) + r ----
  const int col_l = l & 15, rq = (l >> 4) * 4;
  if constexpr (EPI == 0) {
    const int64_t cz = (int64_t)blockIdx.z * g.cz_stride;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int n = n0 + wn * 64 + 16 * b + col_l;
      const float bn = (g.bias && n < g.N) ? g.bias[n] : 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t m = m0 + wm * 64 + 16 * a + rq + r;
          if (m < g.M && n < g.ldc) {
            float v = acc[a][b][r] + bn;
            if (g.rowbias) v += g.rowbias[m];
            if (g.relu) v = fmaxf(v, 0.f);
            if (n >= g.N) v = 0.f;  // zero pad columns: next layer's K padding
            const int nn = g.c_perm32 ? dfm_proj_pos(n) : n;
            if (g.c_bf16)
              reinterpret_cast<uint16_t*>(g.C)[cz + m * g.ldc + nn] = f2bf(v);
            else
              reinterpret_cast<float*>(g.C)[cz + m * g.ldc + nn] = v;
          }
        }
    }
  } else if constexpr (EPI == 2) {
    // grouped dot: every G consecutive columns (G = 16, 32 or 64) form one
    // group; partial[m][n/G] = Σ_{n in group} relu(acc + bias[n%mod]) · v[n%mod]
    const int G = g.G;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gs[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int n = n0 + wn * 64 + 16 * b + col_l;
          float v = 0.f;
          if (n < g.N) {
            const int nm = n % g.mod;
            v = acc[a][b][r] + (g.bias ? g.bias[nm] : 0.f);
            if (g.relu) v = fmaxf(v, 0.f);
            v *= g.dotv[nm];
          }
          gs[b] = group_sum<16>(v);
        }
        const int64_t m = m0 + wm * 64 + 16 * a + rq + r;
        if (col_l == 0 && m < g.M) {
          const int64_t gb = (n0 + wn * 64) / G;   // first group of this wave
          float* dst = g.partial + m * g.ldp + gb;
          const int ng = (g.N - (n0 + wn * 64) + G - 1) / G;  // groups with columns
          if (G == 64) {
            if (ng > 0) dst[0] = (gs[0] + gs[1]) + (gs[2] + gs[3]);
          } else if (G == 32) {
            if (ng > 0) dst[0] = gs[0] + gs[1];
            if (ng > 1) dst[1] = gs[2] + gs[3];
          } else {
            if (ng > 0) dst[0] = gs[0];
            if (ng > 1) dst[1] = gs[1];
            if (ng > 2) dst[2] = gs[2];
            if (ng > 3) dst[3] = gs[3];
          }
        }
      }
  } else {
    float part[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[a][r] = 0.f;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int n = n0 + wn * 64 + 16 * b + col_l;
      const bool ok = n < g.N;
      const float bn = (ok && g.bias) ? g.bias[n] : 0.f;
      const float vn = ok ? g.dotv[n] : 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[a][b][r] + bn;
          if (g.relu) v = fmaxf(v, 0.f);
          part[a][r] += ok ? v * vn : 0.f;
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = group_sum<16>(part[a][r]);
        if (col_l == 0) red[wn][wm * 64 + 16 * a + rq + r] = s;
      }
    __syncthreads();
    if (tid < GBM) {
      const int64_t m = m0 + tid;
      if (m < g.M) g.partial[m * gridDim.y + blockIdx.y] = red[0][tid] + red[1][tid];
    }
  }
}

static inline void launch_gemm(const GemmArgs& g, bool bf, int epi, hipStream_t st) {
  dim3 grid((unsigned)((g.M + GBM - 1) / GBM), (unsigned)((g.N + GBN - 1) / GBN),
            g.ksplit ? (unsigned)((g.K + g.ksplit - 1) / g.ksplit) : 1u);
  if (epi == 2) {  // grouped dot (AFM attention logits), f32 only
    hipLaunchKernelGGL((gemm_mfma<false, 2>), grid, dim3(256), 0, st, g);
    return;
  }
  if (bf) {
    if (epi) hipLaunchKernelGGL((gemm_mfma<true, 1>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((gemm_mfma<true, 0>), grid, dim3(256), 0, st, g);
  } else {
    if (epi) hipLaunchKernelGGL((gemm_mfma<false, 1>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((gemm_mfma<false, 0>), grid, dim3(256), 0, st, g);
  }
}


}  // namespace hhfm
