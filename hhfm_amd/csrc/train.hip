// H6 — training step (`partial_fit`) for FM, HHFM, DeepFM and AFM on gfx950.
//
//   hhfm_fm_train_step    replaces sess.run((loss, optimizer)) of FM
//                         (Newcode/FM.py:123-136, 168-171)
//   hhfm_hhfm_train_step  replaces the same for OUR
//                         (Newcode/OurModel7.py:172-193, 219-228)
//   hhfm_dfm_train_step   replaces the same for DeepFM
//                         (Newcode/DFM.py:139-155, 214-217)
//   hhfm_afm_train_step   replaces the same for AFM
//                         (Newcode/AFM.py:144-156, 205-207)
//
// One wave per batch row computes the forward score(s) and scatters the
// gradient of the row's loss into dense fp32 gradient buffers with float
// atomics (the embedding gradient is a scatter by nature; rows repeat).  The
// L2 term λ·Σ E²/2 (tf.contrib.layers.l2_regularizer) makes the embedding
// gradient dense, so — exactly like TF — the optimizer then updates the whole
// table: `optimizer_apply` applies TF's Adagrad (accumulators initialised to
// 0.1 by the caller), GradientDescent, Momentum or Adam (slots initialised to
// 0) with the sparse-gradient rules TF uses for IndexedSlices variables, and
// accumulates Σ var² of the pre-update table for the reported loss (TF
// evaluates `loss` and the update in the same run).
// Gradients of reduce_max split equally between tied maxima (TF _MaxGrad).
#include <cfloat>

#include "gemm_mfma.h"

namespace hhfm {

enum { OPT_ADAGRAD = 0, OPT_SGD = 1 };
constexpr int kMaxNeg = 16;   // negatives per row (the reference samples 10, OurModel7.py:371)

// scal[0] = Σ dL/d(w0)  scal[1] = data loss  scal[2] = Σ E² (pre-update)  scal[3] = Σ w² (unused)
// scal[8], scal[9] = Adam's β1^t, β2^t (kept between steps); scal[10] != 0 once
// Adam has taken a step (a separate flag: β1^t underflows to exactly 0 after
// 828 steps (TF's flush-to-zero), and TF then keeps using 0, so 0 cannot also
// mean "not started")
__global__ __launch_bounds__(256) void fm_train_rows(
    const int32_t* __restrict__ idx, const float* __restrict__ y, int64_t B, int F,
    const float* __restrict__ E, const float* __restrict__ w, const float* __restrict__ w0,
    int64_t M, int k, float* __restrict__ dE, float* __restrict__ dw, float* __restrict__ scal) {
  const int l = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t b = wave; b < B; b += nwave) {
    const int32_t* x = idx + b * F;
    float t = 0.f;
    for (int c = l; c < k; c += kWave) {
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const float v = E[(int64_t)clamp_id(x[f], M) * k + c];
        s += v;
        q += v * v;
      }
      t += 0.5f * (s * s - q);
    }
    t = group_sum<kWave>(t);
    float fb = 0.f;
    for (int f = 0; f < F; ++f) fb += w[clamp_id(x[f], M)];
    const float out = (t + fb) + w0[0];
    const float r = y[b] - out;        // l2_loss(y - out) = r²/2   FM.py:124
    const float g = -r;                // d/d out
    for (int c = l; c < k; c += kWave) {
      float s = 0.f;
      for (int f = 0; f < F; ++f) s += E[(int64_t)clamp_id(x[f], M) * k + c];
      for (int f = 0; f < F; ++f) {
        const int64_t id = clamp_id(x[f], M);
        atomicAdd(dE + id * k + c, g * (s - E[id * k + c]));   // ∂out/∂e_f = Σe − e_f
      }
    }
    if (l < F) atomicAdd(dw + clamp_id(x[l], M), g);
    if (l == 0) {
      atomicAdd(scal + 0, g);
      atomicAdd(scal + 1, 0.5f * r * r);
    }
  }
}

// HHFM: loss_b = -log σ(pos - max_j neg_j); h = u + Σctx (+ Σtime)
__global__ __launch_bounds__(256) void hhfm_train_rows(
    const int32_t* __restrict__ X, const int32_t* __restrict__ Neg, int64_t B, int ncols,
    int c0, int c1, int t0, int t1, int NG, const float* __restrict__ E, int64_t M, int k,
    float* __restrict__ dE, float* __restrict__ scal) {
  const int l = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t b = wave; b < B; b += nwave) {
    const int32_t* x = X + b * ncols;
    const int32_t* ng = Neg + b * NG;
    const int64_t iu = clamp_id(x[0], M), ii = clamp_id(x[1], M);
    auto hval = [&](int c) {
      float h = E[iu * k + c];
      if (c1 > c0) {
        float s = 0.f;
        for (int j = c0; j < c1; ++j) s += E[(int64_t)clamp_id(x[j], M) * k + c];
        h = h + s;
      }
      if (t1 > t0) {
        float s = 0.f;
        for (int j = t0; j < t1; ++j) s += E[(int64_t)clamp_id(x[j], M) * k + c];
        h = h + s;
      }
      return h;
    };
    float pos = 0.f;
    for (int c = l; c < k; c += kWave) pos += hval(c) * E[ii * k + c];
    pos = group_sum<kWave>(pos);                        // PositiveFeadback  :171
    // NegativeFeadback (:172) for up to kMaxNeg negatives, kept in registers
    float negv[kMaxNeg];
    float mx = -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < kMaxNeg; ++j) {
      negv[j] = -__builtin_huge_valf();
      if (j < NG) {
        float v = 0.f;
        const int64_t in = clamp_id(ng[j], M);
        for (int c = l; c < k; c += kWave) v += hval(c) * E[in * k + c];
        v = group_sum<kWave>(v);
        negv[j] = v;
        mx = fmaxf(mx, v);
      }
    }
    // ties of the max share its gradient (reduce_max, :174)
    int nt = 0;
#pragma unroll
    for (int j = 0; j < kMaxNeg; ++j) nt += (j < NG && negv[j] == mx);
    const float z = pos - mx;
    const float sg = 1.f / (1.f + expf(-z));
    const float g = sg - 1.f;                           // d(-log σ(z))/dz      :178
    const float gt = g / (float)nt;
    for (int c = l; c < k; c += kWave) {
      const float h = hval(c);
      const float it = E[ii * k + c];
      float nsum = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxNeg; ++j)
        if (j < NG && negv[j] == mx) nsum += E[(int64_t)clamp_id(ng[j], M) * k + c];
      const float dh = g * it - gt * nsum;
      atomicAdd(dE + ii * k + c, g * h);
#pragma unroll
      for (int j = 0; j < kMaxNeg; ++j)
        if (j < NG && negv[j] == mx) atomicAdd(dE + (int64_t)clamp_id(ng[j], M) * k + c, -gt * h);
      atomicAdd(dE + iu * k + c, dh);
      for (int j = c0; j < c1; ++j) atomicAdd(dE + (int64_t)clamp_id(x[j], M) * k + c, dh);
      for (int j = t0; j < t1; ++j) atomicAdd(dE + (int64_t)clamp_id(x[j], M) * k + c, dh);
    }
    if (l == 0) atomicAdd(scal + 1, -logf(sg));
  }
}

// One TF-1.x optimizer step on a variable (training_ops.cc semantics, fp32):
//   Adagrad   accum += g²; var -= lr·g·rsqrt(accum)           (ApplyAdagrad)
//   SGD       var -= lr·g                                      (ApplyGradientDescent)
//   Momentum  accum = accum·0.95 + g; var -= accum·lr           (ApplyMomentum,
//             momentum 0.95 as FM.py:136); a SPARSE variable (its gradient an
//             IndexedSlices: embedding_lookup without a dense l2 term) updates
//             only the rows the batch touched (SparseApplyMomentum)
//   Adam      β1 0.9, β2 0.999, ε 1e-8 (FM.py:130), α = lr·√(1−β2^t)/(1−β1^t):
//             dense  m += (g−m)(1−β1); v += (g²−v)(1−β2); var -= m·α/(√v+ε)
//             (ApplyAdam); sparse (AdamOptimizer._apply_sparse_shared)
//             m = m·β1 + g(1−β1); v = v·β2 + g²(1−β2) on every row, the same
//             var update — the two differ only in rounding
// g = grad + λ·var; Σ var² (pre-update) accumulated into *sumsq when given.
// state: Adagrad / Momentum n floats, Adam 2n (m, then v).  pw: the step's
// β1^t, β2^t (TF's beta1_power / beta2_power) and the started flag pw[2]
// (0 = the first step, whose powers are β1, β2).
enum { OPT_MOMENTUM = 2, OPT_ADAM = 3 };
constexpr float kMomentum = 0.95f, kBeta1 = 0.9f, kBeta2 = 0.999f, kAdamEps = 1e-8f;

struct OptStep {
  int opt;
  float lr;
  const float* pw;         // Adam: [β1^t, β2^t, started] (device)
  const uint8_t* touched;  // sparse Momentum: rows the batch touched (else null)
  int rowlen;              // elements per row of the variable (touched index = i / rowlen)
  int sparse;              // the variable's TF gradient is an IndexedSlices
};

__global__ __launch_bounds__(256) void optimizer_apply(float* __restrict__ var,
                                                       float* __restrict__ grad,
                                                       float* __restrict__ state, int64_t n,
                                                       float lam, OptStep o,
                                                       float* __restrict__ sumsq) {
  float alpha = 0.f;
  if (o.opt == OPT_ADAM) {
    const bool started = o.pw[2] != 0.f;
    const float b1p = started ? o.pw[0] : kBeta1;
    const float b2p = started ? o.pw[1] : kBeta2;
    alpha = o.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  float ss = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = var[i];
    ss += v * v;
    const float g = grad[i] + lam * v;
    if (o.opt == OPT_ADAGRAD) {
      const float a = state[i] + g * g;
      state[i] = a;
      var[i] = v - o.lr * g * rsqrtf(a);
    } else if (o.opt == OPT_SGD) {
      var[i] = v - o.lr * g;
    } else if (o.opt == OPT_MOMENTUM) {
      if (!o.sparse || o.touched[i / o.rowlen]) {
        const float a = state[i] * kMomentum + g;
        state[i] = a;
        var[i] = v - a * o.lr;
      }
    } else {
      float m = state[i], vv = state[n + i];
      if (o.sparse) {
        m = m * kBeta1 + g * (1.f - kBeta1);
        vv = vv * kBeta2 + (g * g) * (1.f - kBeta2);
      } else {
        m += (g - m) * (1.f - kBeta1);
        vv += (g * g - vv) * (1.f - kBeta2);
      }
      state[i] = m;
      state[n + i] = vv;
      var[i] = v - (m * alpha) / (sqrtf(vv) + kAdamEps);
    }
    grad[i] = 0.f;   // leave the gradient buffer zeroed for the next step
  }
  if (sumsq) {
    ss = group_sum<kWave>(ss);
    if ((threadIdx.x & 63) == 0) atomicAdd(sumsq, ss);
  }
}

// after every variable's update: β1^t, β2^t -> β1^(t+1), β2^(t+1) (AdamOptimizer._finish).
// TF runs the product with flush-to-zero set (its CPU thread pools set FTZ/DAZ,
// core/lib/core/threadpool.cc), so β1^t reaches exactly 0 at t = 829 and stays
// there; the flush is explicit here, whatever the kernel's denormal mode.
__device__ __forceinline__ float ftz(float x) { return fabsf(x) < FLT_MIN ? 0.f : x; }

__global__ void adam_advance(float* pw) {
  const bool started = pw[2] != 0.f;
  pw[0] = ftz((started ? pw[0] : kBeta1) * kBeta1);
  pw[1] = ftz((started ? pw[1] : kBeta2) * kBeta2);
  pw[2] = 1.f;
}

// touched[x] = val for every id of the batch (rows of a sparse variable the
// step updates under Momentum); plain byte stores, equal values
__global__ __launch_bounds__(256) void mark_rows(const int32_t* __restrict__ idx, int64_t n,
                                                 int64_t M, uint8_t* __restrict__ touched,
                                                 uint8_t val) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    touched[clamp_id(idx[i], M)] = val;
}

__global__ void finish_loss(float* scal, float lam, float* loss) {
  loss[0] = scal[1] + lam * 0.5f * scal[2];   // + l2_regularizer(λ)(E) = λ·ΣE²/2
  scal[0] = scal[1] = scal[2] = scal[3] = 0.f;
}

static int grid_for_n(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

static bool opt_ok(int opt) {
  return opt == OPT_ADAGRAD || opt == OPT_SGD || opt == OPT_MOMENTUM || opt == OPT_ADAM;
}

// one optimizer_apply launch; `sparse` variables under Momentum need the
// touched mask (`mark_rows` before, cleared after by the caller)
static void apply_opt(float* var, float* grad, float* state, int64_t n, float lam, int opt,
                      float lr, const float* pw, const uint8_t* touched, int rowlen, bool sparse,
                      float* sumsq, hipStream_t st) {
  OptStep o{opt, lr, pw, touched, rowlen > 0 ? rowlen : 1, sparse ? 1 : 0};
  hipLaunchKernelGGL(optimizer_apply, dim3(grid_for_n(n)), dim3(256), 0, st, var, grad, state, n,
                     lam, o, sumsq);
}

// ---------------------------------------------------------------------------
// DeepFM training (fp32, the reference numerics).  Forward: the MLP as
// exact-fp32 MFMA GEMMs (gemm_mfma.h, layer 0 gathering its A rows from the
// table), activations kept for the backward pass.  Backward: a row kernel for
// the concat projection (out, d = out − y, dWp, dbp, dw, the last layer's
// delta), per layer dW = Hᵀ·G and G_prev = (G·Wᵀ) ⊙ relu' as GEMMs on
// transposed / zero-padded copies, and a scatter of the embedding gradient
// (deep part + FM part ∂y2/∂e_f = Σe − e_f).  Every activation row is padded
// to a multiple of 8 floats and every transposed copy to Bp = pad8(B) columns,
// zero-filled, so the GEMM's 16-byte K chunks never read past a row.
// ---------------------------------------------------------------------------
constexpr int kDfmTrainMaxLayers = 4;
constexpr int kDfmHeadMaxCols = 1024;   // F + k + d_L per concat row

static int64_t pad8(int64_t x) { return (x + 7) & ~int64_t(7); }

// dst[c][r] = src[r][c] (r < R, c < C; zero for R <= r < Rp) and, with a mask
// H, both the masked src (written back in place) and its transpose use
// src ⊙ (H > 0).  32x32 tiles through LDS.
__global__ __launch_bounds__(256) void tr_pad(float* __restrict__ src, int64_t R, int C,
                                              int64_t lds, const float* __restrict__ H,
                                              int64_t ldh, float* __restrict__ dst,
                                              int64_t ldd, int64_t Rp) {
  __shared__ float t[32][33];
  const int64_t r0 = (int64_t)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int64_t r = r0 + i;
    const int c = c0 + tx;
    float v = 0.f;
    if (r < R && c < C) {
      v = src[r * lds + c];
      if (H) {
        v = H[r * ldh + c] > 0.f ? v : 0.f;
        src[r * lds + c] = v;
      }
    }
    t[i][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i;
    const int64_t r = r0 + tx;
    if (c < C && r < Rp) dst[c * ldd + r] = t[tx][i];
  }
}

// dst[r][c] = src[r][c] for c < C, 0 for C <= c < ldd (row-major zero pad)
__global__ __launch_bounds__(256) void copy_pad(const float* __restrict__ src, int64_t R, int C,
                                                float* __restrict__ dst, int ldd) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R * ldd;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ldd;
    const int c = (int)(i - r * ldd);
    dst[i] = c < C ? src[r * C + c] : 0.f;
  }
}

// X0ᵀ[c][m] = E[x_m, c/k][c%k] (m < B), 0 for B <= m < Bp
__global__ __launch_bounds__(256) void gather_tr(const int32_t* __restrict__ idx, int64_t B,
                                                 int F, const float* __restrict__ E, int64_t M,
                                                 int k, float* __restrict__ dst, int64_t Bp) {
  __shared__ float t[32][33];
  const int64_t m0 = (int64_t)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int D = F * k;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int64_t m = m0 + i;
    const int c = c0 + tx;
    float v = 0.f;
    if (m < B && c < D) {
      const int f = c / k;
      v = E[(int64_t)clamp_id(idx[m * F + f], M) * k + (c - f * k)];
    }
    t[i][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i;
    const int64_t m = m0 + tx;
    if (c < D && m < Bp) dst[c * Bp + m] = t[tx][i];
  }
}

// db[n] = Σ_m G_T[n][m]  (wave per output)
__global__ __launch_bounds__(256) void row_sums(const float* __restrict__ GT, int N, int64_t ld,
                                                int64_t cols, float* __restrict__ out) {
  const int l = threadIdx.x & 63;
  const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t m = l; m < cols; m += kWave) s += GT[n * ld + m];
  s = group_sum<kWave>(s);
  if (l == 0) out[n] = s;
}

// Concat projection, forward and backward (DFM.py:109-137, l2_loss), wave
// per row; each lane keeps its columns' dWp partials over the block's rows.
// scal[0] += dbp  scal[1] += (out − y)²/2
__global__ __launch_bounds__(256) void dfm_train_head(
    const int32_t* __restrict__ idx, const float* __restrict__ y, int64_t B, int F,
    const float* __restrict__ E, const float* __restrict__ w, int64_t M, int k,
    const float* __restrict__ HL, int dL, int64_t ldh, const float* __restrict__ Wp,
    const float* __restrict__ bp, float* __restrict__ GL, float* __restrict__ gvec,
    float* __restrict__ dWp, float* __restrict__ dw, float* __restrict__ scal) {
  constexpr int NJ = kDfmHeadMaxCols / kWave;
  const int l = threadIdx.x & 63;
  const int D = F + k + dL;
  float part[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) part[j] = 0.f;
  float sb = 0.f, sl = 0.f;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* x = idx + m * F;
    // this lane's concat columns c = l + 64 j: [y1 (F) | y2 (k) | h_L (dL)]
    float cv[NJ];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = l + kWave * j;
      float v = 0.f;
      if (c < F) {
        v = w[clamp_id(x[c], M)];
      } else if (c < F + k) {
        const int cc = c - F;
        float s = 0.f, q = 0.f;
        for (int f = 0; f < F; ++f) {
          const float e = E[(int64_t)clamp_id(x[f], M) * k + cc];
          s += e;
          q += e * e;
        }
        v = 0.5f * (s * s - q);
      } else if (c < D) {
        v = HL[m * ldh + (c - F - k)];
      }
      cv[j] = v;
      if (c < D) dot = fmaf(v, Wp[c], dot);
    }
    const float out = group_sum<kWave>(dot) + bp[0];
    const float g = out - y[m];                    // d l2_loss(y − out) / d out
    sb += g;
    sl += 0.5f * g * g;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = l + kWave * j;
      if (c < D) part[j] = fmaf(g, cv[j], part[j]);
      if (c < F) atomicAdd(&dw[clamp_id(x[c], M)], g * Wp[c]);
      if (c >= F + k && c < D) {
        const int n = c - F - k;
        GL[m * ldh + n] = cv[j] > 0.f ? g * Wp[c] : 0.f;   // relu' of the last layer
      }
    }
    if (l == 0) gvec[m] = g;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = l + kWave * j;
    if (c < D && part[j] != 0.f) atomicAdd(&dWp[c], part[j]);
  }
  if (l == 0) {   // (g is wave-uniform: every lane holds the same sums)
    atomicAdd(&scal[0], sb);
    atomicAdd(&scal[1], sl);
  }
}

// dE[x_f][c] += dX0[m][f·k + c] + g_m·Wp[F+c]·(Σ_f' e_f'c − e_fc)   (wave per row)
__global__ __launch_bounds__(256) void dfm_train_scatter(
    const int32_t* __restrict__ idx, int64_t B, int F, const float* __restrict__ E, int64_t M,
    int k, const float* __restrict__ dX0, const float* __restrict__ gvec,
    const float* __restrict__ Wp, float* __restrict__ dE) {
  const int l = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* x = idx + m * F;
    const float g = gvec[m];
    for (int c = l; c < k; c += kWave) {
      float s = 0.f;
      for (int f = 0; f < F; ++f) s += E[(int64_t)clamp_id(x[f], M) * k + c];
      const float gy2 = g * Wp[F + c];
      for (int f = 0; f < F; ++f) {
        const int64_t id = clamp_id(x[f], M);
        const float e = E[id * k + c];
        atomicAdd(&dE[id * k + c], dX0[m * (int64_t)(F * k) + f * k + c] + gy2 * (s - e));
      }
    }
  }
}

struct DfmTrainPlan {
  int64_t Bp;
  int L, D0;
  int d[kDfmTrainMaxLayers + 1];     // d[0] = F·k, d[l+1] = layer l width
  int64_t off_WtP[kDfmTrainMaxLayers], off_WP[kDfmTrainMaxLayers];
  int64_t off_dW[kDfmTrainMaxLayers], off_db[kDfmTrainMaxLayers];
  int64_t off_H[kDfmTrainMaxLayers + 1], off_HT[kDfmTrainMaxLayers];
  int64_t off_G[kDfmTrainMaxLayers + 1], off_GT[kDfmTrainMaxLayers + 1];
  int64_t off_dX0, off_g, off_dWp, off_dE, off_dw, off_scal, off_touch;
  int64_t total;   // floats
};

static bool dfm_train_plan(int64_t B, int F, int k, int64_t M, int L, const int32_t* dims,
                           DfmTrainPlan& p) {
  if (L < 1 || L > kDfmTrainMaxLayers || F < 1 || k < 4 || k % 4) return false;
  p = DfmTrainPlan{};
  p.L = L;
  p.D0 = F * k;
  p.d[0] = p.D0;
  for (int i = 0; i < L; ++i) {
    if (dims[i] < 1) return false;
    p.d[i + 1] = dims[i];
  }
  if (F + k + p.d[L] > kDfmHeadMaxCols) return false;
  p.Bp = pad8(B > 0 ? B : 1);
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  // zero-initialised, kept zeroed by the step (scalars incl. Adam's β powers,
  // dE, dw, touched mask): first, at B-independent offsets, so a workspace
  // grown for a larger batch keeps its state by copying the old one's bytes
  p.off_scal = take(16);
  p.off_dE = take(M * k);
  p.off_dw = take(M);
  p.off_touch = take((M + 3) / 4);   // touched-row mask, M bytes
  for (int i = 0; i < L; ++i) {
    p.off_WtP[i] = take((int64_t)p.d[i + 1] * pad8(p.d[i]));
    p.off_WP[i] = take((int64_t)p.d[i] * pad8(p.d[i + 1]));
    p.off_dW[i] = take((int64_t)p.d[i] * p.d[i + 1]);
    p.off_db[i] = take(p.d[i + 1]);
    p.off_HT[i] = take((int64_t)p.d[i] * p.Bp);
  }
  for (int i = 1; i <= L; ++i) {
    p.off_H[i] = take(p.Bp * pad8(p.d[i]));
    p.off_G[i] = take(p.Bp * pad8(p.d[i]));
    p.off_GT[i] = take((int64_t)p.d[i] * p.Bp);
  }
  p.off_dX0 = take(p.Bp * p.D0);
  p.off_g = take(p.Bp);
  p.off_dWp = take(F + k + p.d[L]);
  p.total = o;
  return true;
}


// ---------------------------------------------------------------------------
// AFM training (fp32, AFM.py:103-156): the two pair-shaped products run as
// exact-fp32 MFMA GEMMs (gemm_mfma.h) over the B·np (row, pair) "combos":
//   R   = relu(pairs · W + b)           pair-mode A operand (e_i ⊙ e_j formed
//                                        in the loader), [B·np][A]
//   DP  = dZ · Wᵀ                       ∂L/∂pairs through the attention MLP
//   dW  = pairsᵀ · dZ                   split-K over the B·np combos, then a
//                                        fixed-order sum of the splits
// and two wave-per-row kernels do the rest: `afm_train_head` (logits,
// softmax over the row's pairs, out, d = out − y, the softmax backward
// dlogit = a ⊙ (da − Σ a·da), dZ = dlogit·p ⊙ relu', db, dp, dP, dw; writes
// dZ and the pair products transposed for the dW GEMM) and `afm_train_scatter`
// (∂L/∂e_i += dpair ⊙ e_j, ∂L/∂e_j += dpair ⊙ e_i, float atomics into dE).
// ---------------------------------------------------------------------------
constexpr int kAfmTrainMaxF = 16;                          // np <= 120
constexpr int kAfmTrainMaxNp = kAfmTrainMaxF * (kAfmTrainMaxF - 1) / 2;
constexpr int kAfmTrainMaxKA = 256;                        // k, A <= 256
constexpr int kAfmSplitK = 512;                            // combos per dW split

__global__ __launch_bounds__(256) void afm_train_head(
    const int32_t* __restrict__ idx, const float* __restrict__ y, int64_t B, int F,
    const float* __restrict__ E, const float* __restrict__ w, const float* __restrict__ w0,
    int64_t M, int k, int A, const float* __restrict__ R, const float* __restrict__ pvec,
    const float* __restrict__ P, float* __restrict__ Gz, float* __restrict__ PT,
    float* __restrict__ GzT, int64_t Kp, float* __restrict__ att, float* __restrict__ gvec,
    float* __restrict__ dP, float* __restrict__ dpv, float* __restrict__ db,
    float* __restrict__ dw, float* __restrict__ scal) {
  constexpr int NC = kAfmTrainMaxKA / kWave;
  __shared__ float sp_all[4][kAfmTrainMaxNp], lg_all[4][kAfmTrainMaxNp];
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sp = sp_all[wv];
  float* lg = lg_all[wv];
  const int np = F * (F - 1) / 2;
  float accP[NC], accV[NC], accB[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) accP[j] = accV[j] = accB[j] = 0.f;
  float sg = 0.f, sl = 0.f;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* x = idx + m * F;
    const int64_t c0 = m * np;   // first combo of this row
    // s_p = P·(e_i ⊙ e_j)   (lanes over k; one wave sum per pair and chunk)
    for (int p = l; p < np; p += kWave) sp[p] = 0.f;
#pragma unroll
    for (int kc = 0; kc < NC; ++kc) {
      const int c = l + kWave * kc;
      if (kc * kWave >= k) break;
      float ev[kAfmTrainMaxF];
#pragma unroll
      for (int f = 0; f < kAfmTrainMaxF; ++f)
        ev[f] = (f < F && c < k) ? E[(int64_t)clamp_id(x[f], M) * k + c] : 0.f;
      const float pc = c < k ? P[c] : 0.f;
      int p = 0;
#pragma unroll
      for (int i = 0; i < kAfmTrainMaxF; ++i)
#pragma unroll
        for (int j = i + 1; j < kAfmTrainMaxF; ++j)
          if (j < F) {
            const float s = group_sum<kWave>(ev[i] * ev[j] * pc);
            if (l == 0) sp[p] += s;
            ++p;
          }
    }
    __builtin_amdgcn_wave_barrier();
    // logit_p = Σ_a pvec_a · R[p][a]   (lanes over A)
    for (int p = 0; p < np; ++p) {
      float t = 0.f;
      for (int a = l; a < A; a += kWave) t = fmaf(pvec[a], R[(c0 + p) * A + a], t);
      t = group_sum<kWave>(t);
      if (l == 0) lg[p] = t;
    }
    __builtin_amdgcn_wave_barrier();
    // softmax over the row's pairs (AFM.py:125, max subtracted), out, d
    float mx = -__builtin_huge_valf();
    for (int p = l; p < np; p += kWave) mx = fmaxf(mx, lg[p]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, kWave));
    float se = 0.f;
    for (int p = l; p < np; p += kWave) se += expf(lg[p] - mx);
    se = group_sum<kWave>(se);
    float os = 0.f;
    for (int p = l; p < np; p += kWave) os += expf(lg[p] - mx) / se * sp[p];
    os = group_sum<kWave>(os);
    float fb = 0.f;
    for (int f = l; f < F; f += kWave) fb += w[clamp_id(x[f], M)];
    fb = group_sum<kWave>(fb);
    const float out = (os + fb) + w0[0];
    const float g = out - y[m];                      // d l2_loss(y − out) / d out
    sg += g;
    sl += 0.5f * g * g;
    // da_p = g·s_p, dlogit_p = a_p (da_p − Σ a·da)
    float t = 0.f;
    for (int p = l; p < np; p += kWave) t += expf(lg[p] - mx) / se * (g * sp[p]);
    t = group_sum<kWave>(t);
    for (int p = l; p < np; p += kWave) {
      const float a = expf(lg[p] - mx) / se;
      att[c0 + p] = a;
      lg[p] = a * (g * sp[p] - t);                   // lg now holds dlogit
      sp[p] = a;                                     // sp now holds att
    }
    if (l == 0) gvec[m] = g;
    __builtin_amdgcn_wave_barrier();
    // dZ = dlogit·p ⊙ relu'(z)  (lanes over A), written row-major and transposed
#pragma unroll
    for (int ac = 0; ac < NC; ++ac) {
      const int a = l + kWave * ac;
      if (ac * kWave >= A) break;
      if (a < A) {
        const float pa = pvec[a];
        for (int p = 0; p < np; ++p) {
          const float r = R[(c0 + p) * A + a];
          const float dl = lg[p];
          accV[ac] = fmaf(dl, r, accV[ac]);
          const float dz = r > 0.f ? dl * pa : 0.f;
          accB[ac] += dz;
          Gz[(c0 + p) * A + a] = dz;
          GzT[a * Kp + c0 + p] = dz;
        }
      }
    }
    // afm = Σ a_p (e_i ⊙ e_j) -> dP; pair products transposed for the dW GEMM
#pragma unroll
    for (int kc = 0; kc < NC; ++kc) {
      const int c = l + kWave * kc;
      if (kc * kWave >= k) break;
      if (c < k) {
        float ev[kAfmTrainMaxF];
#pragma unroll
        for (int f = 0; f < kAfmTrainMaxF; ++f)
          ev[f] = f < F ? E[(int64_t)clamp_id(x[f], M) * k + c] : 0.f;
        float afm = 0.f;
        int p = 0;
#pragma unroll
        for (int i = 0; i < kAfmTrainMaxF; ++i)
#pragma unroll
          for (int j = i + 1; j < kAfmTrainMaxF; ++j)
            if (j < F) {
              const float pr = ev[i] * ev[j];
              afm = fmaf(sp[p], pr, afm);
              PT[c * Kp + c0 + p] = pr;
              ++p;
            }
        accP[kc] = fmaf(g, afm, accP[kc]);
      }
    }
    for (int f = l; f < F; f += kWave) atomicAdd(&dw[clamp_id(x[f], M)], g);
    __builtin_amdgcn_wave_barrier();   // sp / lg are rewritten by the next row
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = l + kWave * j;
    if (c < k && accP[j] != 0.f) atomicAdd(&dP[c], accP[j]);
    if (c < A && accV[j] != 0.f) atomicAdd(&dpv[c], accV[j]);
    if (c < A && accB[j] != 0.f) atomicAdd(&db[c], accB[j]);
  }
  if (l == 0) {   // g is wave-uniform
    atomicAdd(&scal[0], sg);
    atomicAdd(&scal[1], sl);
  }
}

// dE[x_f][c] += Σ_{pairs ∋ f} (DP + a_p·d·P_c) ⊙ e_other   (wave per row, lanes over k)
__global__ __launch_bounds__(256) void afm_train_scatter(
    const int32_t* __restrict__ idx, int64_t B, int F, const float* __restrict__ E, int64_t M,
    int k, const float* __restrict__ DP, const float* __restrict__ att,
    const float* __restrict__ gvec, const float* __restrict__ P, float* __restrict__ dE) {
  const int l = threadIdx.x & 63;
  const int np = F * (F - 1) / 2;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* x = idx + m * F;
    const int64_t c0 = m * np;
    const float g = gvec[m];
    for (int c = l; c < k; c += kWave) {
      float ev[kAfmTrainMaxF], de[kAfmTrainMaxF];
#pragma unroll
      for (int f = 0; f < kAfmTrainMaxF; ++f) {
        ev[f] = f < F ? E[(int64_t)clamp_id(x[f], M) * k + c] : 0.f;
        de[f] = 0.f;
      }
      const float gp = g * P[c];
      int p = 0;
#pragma unroll
      for (int i = 0; i < kAfmTrainMaxF; ++i)
#pragma unroll
        for (int j = i + 1; j < kAfmTrainMaxF; ++j)
          if (j < F) {
            const float d = fmaf(att[c0 + p], gp, DP[(c0 + p) * k + c]);
            de[i] = fmaf(d, ev[j], de[i]);
            de[j] = fmaf(d, ev[i], de[j]);
            ++p;
          }
#pragma unroll
      for (int f = 0; f < kAfmTrainMaxF; ++f)
        if (f < F) atomicAdd(&dE[(int64_t)clamp_id(x[f], M) * k + c], de[f]);
    }
  }
}

// zero the K padding [n, Kp) of `rows` transposed rows of stride Kp
__global__ __launch_bounds__(256) void zero_cols(float* __restrict__ T, int rows, int64_t Kp,
                                                 int64_t n) {
  const int pad = (int)(Kp - n);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)rows * pad;
       i += (int64_t)gridDim.x * blockDim.x)
    T[(i / pad) * Kp + n + i % pad] = 0.f;
}

// dW[i] = Σ_s part[s][i] in split order (deterministic)
__global__ __launch_bounds__(256) void sum_splits(const float* __restrict__ part, int S,
                                                  int64_t n, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += part[z * n + i];
    out[i] = s;
  }
}

struct AfmTrainPlan {
  int np;
  int64_t n, Kp;
  int S;
  int64_t off_Wt, off_R, off_Gz, off_T, off_DP, off_att, off_g, off_part;
  int64_t off_dE, off_dw, off_dW, off_db, off_dpv, off_dP, off_scal, off_touch;
  int64_t total;   // floats
};

static bool afm_train_plan(int64_t B, int F, int k, int A, int64_t M, AfmTrainPlan& p) {
  if (F < 2 || F > kAfmTrainMaxF || k < 4 || k % 4 || k > kAfmTrainMaxKA || A < 4 || A % 4 ||
      A > kAfmTrainMaxKA || B < 0 || M < 1)
    return false;
  p = AfmTrainPlan{};
  p.np = F * (F - 1) / 2;
  p.n = B * p.np;
  if (p.n > (int64_t)1 << 30) return false;
  p.Kp = pad8(p.n > 0 ? p.n : 1);
  p.S = (int)((p.Kp + kAfmSplitK - 1) / kAfmSplitK);
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  // zero-initialised, kept zeroed by the step; first, at B-independent
  // offsets (see dfm_train_plan)
  p.off_scal = take(16);
  p.off_dE = take(M * k);
  p.off_dw = take(M);
  p.off_dW = take((int64_t)k * A);
  p.off_db = take(A);
  p.off_dpv = take(A);
  p.off_dP = take(k);
  p.off_touch = take((M + 3) / 4);   // touched-row mask, M bytes
  p.off_Wt = take((int64_t)A * k);
  p.off_R = take(p.n * A);
  p.off_Gz = take(p.n * A);
  p.off_T = take((int64_t)(k + A) * p.Kp);   // PT [k][Kp] then GzT [A][Kp]
  p.off_DP = take(p.n * k);
  p.off_att = take(p.n);
  p.off_g = take(B);
  p.off_part = take((int64_t)p.S * k * A);
  p.total = o;
  return true;
}

}  // namespace hhfm

using namespace hhfm;

extern "C" size_t hhfm_train_workspace(int64_t features_M, int32_t k) {
  // dE [M*k] + dw [M] + 16 scalars + the touched-row mask [M] bytes; must be
  // zero-filled once by the caller
  return (size_t)features_M * k * 4 + (size_t)features_M * 4 + 64 +
         (((size_t)features_M + 255) & ~size_t(255));
}

extern "C" int hhfm_fm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F,
                                  float* E, float* w, float* w0, int64_t features_M, int32_t k,
                                  float lr, float lam, int32_t optimizer, float* accE,
                                  float* accw, float* accw0, void* workspace, size_t ws_bytes,
                                  float* loss, void* stream) {
  if (B < 0 || F < 1 || k < 1 || features_M < 1) return HHFM_EINVAL;
  if (!opt_ok(optimizer)) return HHFM_EUNSUPPORTED;
  if (!idx || !y || !E || !w || !w0 || !loss || !workspace) return HHFM_EINVAL;
  if (optimizer != OPT_SGD && (!accE || !accw || !accw0)) return HHFM_EINVAL;
  if (ws_bytes < hhfm_train_workspace(features_M, k)) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dE = reinterpret_cast<float*>(workspace);
  float* dw = dE + features_M * k;
  float* scal = dw + features_M;
  uint8_t* touched = reinterpret_cast<uint8_t*>(scal + 16);
  if (B > 0)
    hipLaunchKernelGGL(fm_train_rows, dim3(grid_for_n(B * 64)), dim3(256), 0, st, idx, y, B, F,
                       E, w, w0, features_M, k, dE, dw, scal);
  // sparse gradients (FM.py:123-126): w's always (embedding_lookup only), E's
  // when λ = 0 (no dense l2 term); w0 and the λ > 0 table are dense
  const bool mark = optimizer == OPT_MOMENTUM && B > 0;
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)1);
  const int64_t nE = features_M * k;
  apply_opt(E, dE, accE, nE, lam, optimizer, lr, scal + 8, touched, k, lam == 0.f, scal + 2, st);
  apply_opt(w, dw, accw, features_M, 0.f, optimizer, lr, scal + 8, touched, 1, true, nullptr, st);
  apply_opt(w0, scal, accw0, 1, 0.f, optimizer, lr, scal + 8, nullptr, 1, false, nullptr, st);
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)0);
  if (optimizer == OPT_ADAM) hipLaunchKernelGGL(adam_advance, dim3(1), dim3(1), 0, st, scal + 8);
  hipLaunchKernelGGL(finish_loss, dim3(1), dim3(1), 0, st, scal, lam, loss);
  return (int)hipGetLastError();
}

extern "C" int hhfm_hhfm_train_step(const int32_t* X, const int32_t* Neg, int64_t B,
                                    int32_t ncols, int32_t ctx_begin, int32_t ctx_end,
                                    int32_t time_begin, int32_t time_end, int32_t NG, float* E,
                                    int64_t features_M, int32_t k, float lr, float lam,
                                    int32_t optimizer, float* accE, void* workspace,
                                    size_t ws_bytes, float* loss, void* stream) {
  if (B < 0 || ncols < 2 || NG < 1 || k < 1 || features_M < 1) return HHFM_EINVAL;
  if (NG > kMaxNeg) return HHFM_EUNSUPPORTED;
  if (!opt_ok(optimizer)) return HHFM_EUNSUPPORTED;
  if (!X || !Neg || !E || !loss || !workspace) return HHFM_EINVAL;
  if (optimizer != OPT_SGD && !accE) return HHFM_EINVAL;
  if (ws_bytes < hhfm_train_workspace(features_M, k)) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dE = reinterpret_cast<float*>(workspace);
  float* scal = dE + features_M * k + features_M;
  uint8_t* touched = reinterpret_cast<uint8_t*>(scal + 16);
  if (B > 0)
    hipLaunchKernelGGL(hhfm_train_rows, dim3(grid_for_n(B * 64)), dim3(256), 0, st, X, Neg, B,
                       ncols, ctx_begin, ctx_end, time_begin, time_end, NG, E, features_M, k,
                       dE, scal);
  // E's gradient is dense through λ·l2(E) (OurModel7.py:180-184), sparse at λ = 0
  const bool sparseE = lam == 0.f;
  const bool mark = optimizer == OPT_MOMENTUM && sparseE && B > 0;
  if (mark) {
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * ncols)), dim3(256), 0, st, X, B * ncols,
                       features_M, touched, (uint8_t)1);
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * NG)), dim3(256), 0, st, Neg, B * NG,
                       features_M, touched, (uint8_t)1);
  }
  const int64_t nE = features_M * k;
  apply_opt(E, dE, accE, nE, lam, optimizer, lr, scal + 8, touched, k, sparseE, scal + 2, st);
  if (mark) {
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * ncols)), dim3(256), 0, st, X, B * ncols,
                       features_M, touched, (uint8_t)0);
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * NG)), dim3(256), 0, st, Neg, B * NG,
                       features_M, touched, (uint8_t)0);
  }
  if (optimizer == OPT_ADAM) hipLaunchKernelGGL(adam_advance, dim3(1), dim3(1), 0, st, scal + 8);
  hipLaunchKernelGGL(finish_loss, dim3(1), dim3(1), 0, st, scal, lam, loss);
  return (int)hipGetLastError();
}

extern "C" int hhfm_dfm_train_workspace(int64_t B, int32_t F, int32_t k, int64_t features_M,
                                        int32_t nlayers, const int32_t* layer_dims,
                                        size_t* ws_bytes) {
  DfmTrainPlan p;
  if (!ws_bytes || !layer_dims || B < 0 || features_M < 1 ||
      !dfm_train_plan(B, F, k, features_M, nlayers, layer_dims, p))
    return HHFM_EINVAL;
  *ws_bytes = (size_t)p.total * 4;
  return HHFM_OK;
}

// bytes at the front of the DeepFM workspace that carry state between steps
// (scalars incl. Adam's β powers, dE, dw, the touched mask); B-independent
extern "C" int hhfm_dfm_train_state_bytes(int32_t F, int32_t k, int64_t features_M,
                                          int32_t nlayers, const int32_t* layer_dims,
                                          size_t* state_bytes) {
  DfmTrainPlan p;
  if (!state_bytes || !layer_dims || features_M < 1 ||
      !dfm_train_plan(1, F, k, features_M, nlayers, layer_dims, p))
    return HHFM_EINVAL;
  *state_bytes = (size_t)p.off_WtP[0] * 4;
  return HHFM_OK;
}

extern "C" int hhfm_dfm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F,
                                   float* E, float* w, int64_t features_M, int32_t k,
                                   int32_t nlayers, const int32_t* layer_dims, float* const* W,
                                   float* const* bias, float* Wp, float* bp, float lr,
                                   float lambda_l2, int32_t optimizer, float* const* acc,
                                   void* workspace, size_t ws_bytes, float* loss,
                                   void* stream) {
  DfmTrainPlan p;
  if (B < 0 || features_M < 1 || !layer_dims ||
      !dfm_train_plan(B, F, k, features_M, nlayers, layer_dims, p))
    return HHFM_EINVAL;
  if (!opt_ok(optimizer)) return HHFM_EUNSUPPORTED;
  if (!idx || !y || !E || !w || !W || !bias || !Wp || !bp || !loss || !workspace)
    return HHFM_EINVAL;
  const int L = p.L;
  for (int i = 0; i < L; ++i)
    if (!W[i] || !bias[i]) return HHFM_EINVAL;
  if (optimizer != OPT_SGD) {   // acc: E, w, W_0..W_{L-1}, b_0..b_{L-1}, Wp, bp
    if (!acc) return HHFM_EINVAL;
    for (int i = 0; i < 2 * L + 4; ++i)
      if (!acc[i]) return HHFM_EINVAL;
  }
  if (ws_bytes < (size_t)p.total * 4) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  auto at = [&](int64_t off) { return ws + off; };
  float* scal = at(p.off_scal);
  const int64_t Bp = p.Bp;
  const int64_t nE = features_M * k;
  auto acc_of = [&](int i) { return optimizer != OPT_SGD ? acc[i] : (float*)nullptr; };
  uint8_t* touched = reinterpret_cast<uint8_t*>(at(p.off_touch));

  if (B > 0) {
    // weights: Wᵀ zero-padded (forward Bt) and W zero-padded (backward Bt)
    for (int i = 0; i < L; ++i) {
      const int din = p.d[i], dout = p.d[i + 1];
      hipLaunchKernelGGL(tr_pad, dim3((unsigned)((din + 31) / 32), (unsigned)((dout + 31) / 32)),
                         dim3(256), 0, st, W[i], (int64_t)din, dout, (int64_t)dout,
                         (const float*)nullptr, (int64_t)0, at(p.off_WtP[i]), pad8(din),
                         pad8(din));
      hipLaunchKernelGGL(copy_pad, dim3(grid_for_n((int64_t)din * pad8(dout))), dim3(256), 0, st,
                         W[i], (int64_t)din, dout, at(p.off_WP[i]), (int)pad8(dout));
    }
    // forward: H_{i+1} = relu(H_i · W_i + b_i), H_0 gathered from the table
    for (int i = 0; i < L; ++i) {
      GemmArgs g{};
      g.M = B;
      g.N = p.d[i + 1];
      g.K = p.d[i];
      if (i == 0) {
        g.gidx = idx;
        g.T = E;
        g.Mtab = features_M;
        g.F = F;
        g.kf = k;
      } else {
        g.A = at(p.off_H[i]);
        g.lda = pad8(p.d[i]);
      }
      g.Bt = at(p.off_WtP[i]);
      g.ldb = pad8(p.d[i]);
      g.bias = bias[i];
      g.relu = 1;
      g.C = at(p.off_H[i + 1]);
      g.ldc = pad8(p.d[i + 1]);
      launch_gemm(g, false, 0, st);
    }
    // head: out, d = out − y, dWp, dbp, dw, last layer's delta
    const int64_t ldL = pad8(p.d[L]);
    (void)hipMemsetAsync(at(p.off_G[L]), 0, (size_t)(B * ldL) * 4, st);
    hipLaunchKernelGGL(dfm_train_head, dim3(grid_for_n(B * 64 / 8)), dim3(256), 0, st, idx, y, B,
                       F, E, w, features_M, k, at(p.off_H[L]), p.d[L], ldL, Wp, bp, at(p.off_G[L]),
                       at(p.off_g), at(p.off_dWp), at(p.off_dw), scal);
    hipLaunchKernelGGL(tr_pad, dim3((unsigned)((Bp + 31) / 32), (unsigned)((p.d[L] + 31) / 32)),
                       dim3(256), 0, st, at(p.off_G[L]), B, p.d[L], ldL, (const float*)nullptr,
                       (int64_t)0, at(p.off_GT[L]), Bp, Bp);
    // backward through the layers
    for (int i = L - 1; i >= 0; --i) {
      const int din = p.d[i], dout = p.d[i + 1];
      // H_iᵀ (transposed activations; the gathered table rows for i = 0)
      if (i == 0)
        hipLaunchKernelGGL(gather_tr, dim3((unsigned)((Bp + 31) / 32), (unsigned)((din + 31) / 32)),
                           dim3(256), 0, st, idx, B, F, E, features_M, k, at(p.off_HT[0]), Bp);
      else
        hipLaunchKernelGGL(tr_pad, dim3((unsigned)((Bp + 31) / 32), (unsigned)((din + 31) / 32)),
                           dim3(256), 0, st, at(p.off_H[i]), B, din, pad8(din),
                           (const float*)nullptr, (int64_t)0, at(p.off_HT[i]), Bp, Bp);
      {   // dW_i = H_iᵀ · G_{i+1}
        GemmArgs g{};
        g.M = din;
        g.N = dout;
        g.K = (int)Bp;
        g.A = at(p.off_HT[i]);
        g.lda = Bp;
        g.Bt = at(p.off_GT[i + 1]);
        g.ldb = Bp;
        g.C = at(p.off_dW[i]);
        g.ldc = dout;
        launch_gemm(g, false, 0, st);
      }
      hipLaunchKernelGGL(row_sums, dim3((unsigned)((dout + 3) / 4)), dim3(256), 0, st,
                         at(p.off_GT[i + 1]), dout, Bp, Bp, at(p.off_db[i]));
      {   // G_i = (G_{i+1} · W_iᵀ) ⊙ relu'(H_i), or dX0 = G_1 · W_0ᵀ
        GemmArgs g{};
        g.M = B;
        g.N = din;
        g.K = dout;
        g.A = at(p.off_G[i + 1]);
        g.lda = pad8(dout);
        g.Bt = at(p.off_WP[i]);
        g.ldb = pad8(dout);
        g.C = i == 0 ? at(p.off_dX0) : at(p.off_G[i]);
        g.ldc = i == 0 ? p.D0 : pad8(din);
        launch_gemm(g, false, 0, st);
      }
      if (i > 0)
        hipLaunchKernelGGL(tr_pad, dim3((unsigned)((Bp + 31) / 32), (unsigned)((din + 31) / 32)),
                           dim3(256), 0, st, at(p.off_G[i]), B, din, pad8(din),
                           (const float*)at(p.off_H[i]), pad8(din), at(p.off_GT[i]), Bp, Bp);
    }
    hipLaunchKernelGGL(dfm_train_scatter, dim3(grid_for_n(B * 64)), dim3(256), 0, st, idx, B, F,
                       E, features_M, k, at(p.off_dX0), at(p.off_g), Wp, at(p.off_dE));
  }
  // optimizer: λ only on the layer weights and the concat projection
  // (DFM.py:146-152); the table and w have IndexedSlices gradients (sparse)
  const bool mark = optimizer == OPT_MOMENTUM && B > 0;
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)1);
  const float* pw = scal + 8;
  apply_opt(E, at(p.off_dE), acc_of(0), nE, 0.f, optimizer, lr, pw, touched, k, true, nullptr,
            st);
  apply_opt(w, at(p.off_dw), acc_of(1), features_M, 0.f, optimizer, lr, pw, touched, 1, true,
            nullptr, st);
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)0);
  for (int i = 0; i < L; ++i) {
    const int64_t n = (int64_t)p.d[i] * p.d[i + 1];
    if (B == 0) {
      (void)hipMemsetAsync(at(p.off_dW[i]), 0, n * 4, st);
      (void)hipMemsetAsync(at(p.off_db[i]), 0, p.d[i + 1] * 4, st);
    }
    apply_opt(W[i], at(p.off_dW[i]), acc_of(2 + i), n, lambda_l2, optimizer, lr, pw, nullptr, 1,
              false, scal + 2, st);
    apply_opt(bias[i], at(p.off_db[i]), acc_of(2 + L + i), (int64_t)p.d[i + 1], 0.f, optimizer,
              lr, pw, nullptr, 1, false, nullptr, st);
  }
  const int64_t nWp = F + k + p.d[L];
  apply_opt(Wp, at(p.off_dWp), acc_of(2 + 2 * L), nWp, lambda_l2, optimizer, lr, pw, nullptr, 1,
            false, scal + 2, st);
  apply_opt(bp, scal, acc_of(3 + 2 * L), 1, 0.f, optimizer, lr, pw, nullptr, 1, false, nullptr,
            st);
  if (optimizer == OPT_ADAM) hipLaunchKernelGGL(adam_advance, dim3(1), dim3(1), 0, st, scal + 8);
  hipLaunchKernelGGL(finish_loss, dim3(1), dim3(1), 0, st, scal, lambda_l2, loss);
  return (int)hipGetLastError();
}

extern "C" int hhfm_afm_train_workspace(int64_t B, int32_t F, int32_t k, int32_t A,
                                        int64_t features_M, size_t* ws_bytes) {
  AfmTrainPlan p;
  if (!ws_bytes || !afm_train_plan(B, F, k, A, features_M, p)) return HHFM_EINVAL;
  *ws_bytes = (size_t)p.total * 4;
  return HHFM_OK;
}

// the AFM workspace's persistent prefix (as hhfm_dfm_train_state_bytes)
extern "C" int hhfm_afm_train_state_bytes(int32_t F, int32_t k, int32_t A, int64_t features_M,
                                          size_t* state_bytes) {
  AfmTrainPlan p;
  if (!state_bytes || !afm_train_plan(1, F, k, A, features_M, p)) return HHFM_EINVAL;
  *state_bytes = (size_t)p.off_Wt * 4;
  return HHFM_OK;
}

extern "C" int hhfm_afm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F,
                                   float* E, float* w, float* w0, int64_t features_M, int32_t k,
                                   int32_t A, float* W, float* b, float* pvec, float* P,
                                   float lr, float lambda_att, int32_t optimizer,
                                   float* const* acc, void* workspace, size_t ws_bytes,
                                   float* loss, void* stream) {
  AfmTrainPlan p;
  if (!afm_train_plan(B, F, k, A, features_M, p)) return HHFM_EINVAL;
  if (!opt_ok(optimizer)) return HHFM_EUNSUPPORTED;
  if (!idx || !y || !E || !w || !w0 || !W || !b || !pvec || !P || !loss || !workspace)
    return HHFM_EINVAL;
  if (optimizer != OPT_SGD) {   // acc: E, w, w0, W, b, pvec, P
    if (!acc) return HHFM_EINVAL;
    for (int i = 0; i < 7; ++i)
      if (!acc[i]) return HHFM_EINVAL;
  }
  if (ws_bytes < (size_t)p.total * 4) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* ws = reinterpret_cast<float*>(workspace);
  auto at = [&](int64_t off) { return ws + off; };
  float* scal = at(p.off_scal);
  float* PT = at(p.off_T);
  float* GzT = PT + (int64_t)k * p.Kp;
  auto acc_of = [&](int i) { return optimizer != OPT_SGD ? acc[i] : (float*)nullptr; };
  uint8_t* touched = reinterpret_cast<uint8_t*>(at(p.off_touch));

  if (B > 0) {
    // Wᵀ [A][k] for the forward GEMM
    hipLaunchKernelGGL(tr_pad, dim3((unsigned)((k + 31) / 32), (unsigned)((A + 31) / 32)),
                       dim3(256), 0, st, W, (int64_t)k, A, (int64_t)A, (const float*)nullptr,
                       (int64_t)0, at(p.off_Wt), (int64_t)k, (int64_t)k);
    {   // R = relu(pairs · W + b)   (AFM.py:117-121)
      GemmArgs g{};
      g.M = p.n;
      g.N = A;
      g.K = k;
      g.pair_mode = 1;
      g.P = p.np;
      g.gidx = idx;
      g.T = E;
      g.Mtab = features_M;
      g.F = F;
      g.kf = k;
      g.Bt = at(p.off_Wt);
      g.ldb = k;
      g.bias = b;
      g.relu = 1;
      g.C = at(p.off_R);
      g.ldc = A;
      launch_gemm(g, false, 0, st);
    }
    // a few rows per wave: the per-wave dP / dp / db flush is k + 2A same-address atomics
    const unsigned hb = (unsigned)std::min<int64_t>(256, (B + 3) / 4);
    hipLaunchKernelGGL(afm_train_head, dim3(hb), dim3(256), 0, st, idx, y,
                       B, F, E, w, w0, features_M, k, A, at(p.off_R), pvec, P, at(p.off_Gz), PT,
                       GzT, p.Kp, at(p.off_att), at(p.off_g), at(p.off_dP), at(p.off_dpv),
                       at(p.off_db), at(p.off_dw), scal);
    if (p.Kp > p.n)
      hipLaunchKernelGGL(zero_cols, dim3(grid_for_n((int64_t)(k + A) * (p.Kp - p.n))),
                         dim3(256), 0, st, PT, k + A, p.Kp, p.n);
    {   // DP = dZ · Wᵀ   (Bt = W [k][A])
      GemmArgs g{};
      g.M = p.n;
      g.N = k;
      g.K = A;
      g.A = at(p.off_Gz);
      g.lda = A;
      g.Bt = W;
      g.ldb = A;
      g.C = at(p.off_DP);
      g.ldc = k;
      launch_gemm(g, false, 0, st);
    }
    {   // dW = pairsᵀ · dZ, split over the combos
      GemmArgs g{};
      g.M = k;
      g.N = A;
      g.K = (int)p.Kp;
      g.A = PT;
      g.lda = p.Kp;
      g.Bt = GzT;
      g.ldb = p.Kp;
      g.C = at(p.off_part);
      g.ldc = A;
      g.ksplit = kAfmSplitK;
      g.cz_stride = (int64_t)k * A;
      launch_gemm(g, false, 0, st);
      hipLaunchKernelGGL(sum_splits, dim3(grid_for_n((int64_t)k * A)), dim3(256), 0, st,
                         (const float*)at(p.off_part), p.S, (int64_t)k * A, at(p.off_dW));
    }
    hipLaunchKernelGGL(afm_train_scatter, dim3(grid_for_n(B * 64)), dim3(256), 0, st, idx, B, F,
                       E, features_M, k, at(p.off_DP), at(p.off_att), at(p.off_g), P,
                       at(p.off_dE));
  }
  // the table and w have IndexedSlices gradients (sparse); l2_regularizer(λ)
  // on attention_W only (AFM.py:146)
  const bool mark = optimizer == OPT_MOMENTUM && B > 0;
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)1);
  const float* pw = scal + 8;
  const int64_t nE = features_M * k;
  apply_opt(E, at(p.off_dE), acc_of(0), nE, 0.f, optimizer, lr, pw, touched, k, true, nullptr,
            st);
  apply_opt(w, at(p.off_dw), acc_of(1), features_M, 0.f, optimizer, lr, pw, touched, 1, true,
            nullptr, st);
  if (mark)
    hipLaunchKernelGGL(mark_rows, dim3(grid_for_n(B * F)), dim3(256), 0, st, idx, B * F,
                       features_M, touched, (uint8_t)0);
  apply_opt(w0, scal, acc_of(2), 1, 0.f, optimizer, lr, pw, nullptr, 1, false, nullptr, st);
  apply_opt(W, at(p.off_dW), acc_of(3), (int64_t)k * A, lambda_att, optimizer, lr, pw, nullptr, 1,
            false, scal + 2, st);
  apply_opt(b, at(p.off_db), acc_of(4), (int64_t)A, 0.f, optimizer, lr, pw, nullptr, 1, false,
            nullptr, st);
  apply_opt(pvec, at(p.off_dpv), acc_of(5), (int64_t)A, 0.f, optimizer, lr, pw, nullptr, 1, false,
            nullptr, st);
  apply_opt(P, at(p.off_dP), acc_of(6), (int64_t)k, 0.f, optimizer, lr, pw, nullptr, 1, false,
            nullptr, st);
  if (optimizer == OPT_ADAM) hipLaunchKernelGGL(adam_advance, dim3(1), dim3(1), 0, st, scal + 8);
  hipLaunchKernelGGL(finish_loss, dim3(1), dim3(1), 0, st, scal, lambda_att, loss);
  return (int)hipGetLastError();
}
