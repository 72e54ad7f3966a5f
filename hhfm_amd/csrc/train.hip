// H6 — training step (`partial_fit`) for FM and HHFM on gfx950.
//
//   hhfm_fm_train_step    replaces sess.run((loss, optimizer)) of FM
//                         (Newcode/FM.py:123-136, 168-171)
//   hhfm_hhfm_train_step  replaces the same for OUR
//                         (Newcode/OurModel7.py:172-193, 219-228)
//
// One wave per batch row computes the forward score(s) and scatters the
// gradient of the row's loss into dense fp32 gradient buffers with float
// atomics (the embedding gradient is a scatter by nature; rows repeat).  The
// L2 term λ·Σ E²/2 (tf.contrib.layers.l2_regularizer) makes the embedding
// gradient dense, so — exactly like TF — the optimizer then updates the whole
// table: `optimizer_dense` applies TF's ApplyAdagrad (accum += g², var -= lr·
// g·rsqrt(accum), accumulators initialised to 0.1 by the caller) or plain
// gradient descent, and accumulates Σ var² of the pre-update table for the
// reported loss (TF evaluates `loss` and the update in the same run).
// Gradients of reduce_max split equally between tied maxima (TF _MaxGrad).
#include "hhfm_common.h"

namespace hhfm {

enum { OPT_ADAGRAD = 0, OPT_SGD = 1 };
constexpr int kMaxNeg = 16;   // negatives per row (the reference samples 10, OurModel7.py:371)

// scal[0] = Σ dL/d(w0)  scal[1] = data loss  scal[2] = Σ E² (pre-update)  scal[3] = Σ w² (unused)
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

// var -= lr·g·rsqrt(accum += g²) (Adagrad) or var -= lr·g (SGD);
// g = grad + λ·var; Σ var² (pre-update) accumulated into *sumsq when given.
__global__ __launch_bounds__(256) void optimizer_dense(float* __restrict__ var,
                                                       float* __restrict__ grad,
                                                       float* __restrict__ accum, int64_t n,
                                                       float lr, float lam, int opt,
                                                       float* __restrict__ sumsq) {
  float ss = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = var[i];
    ss += v * v;
    const float g = grad[i] + lam * v;
    if (opt == OPT_ADAGRAD) {
      const float a = accum[i] + g * g;
      accum[i] = a;
      var[i] = v - lr * g * rsqrtf(a);
    } else {
      var[i] = v - lr * g;
    }
    grad[i] = 0.f;   // leave the gradient buffer zeroed for the next step
  }
  if (sumsq) {
    ss = group_sum<kWave>(ss);
    if ((threadIdx.x & 63) == 0) atomicAdd(sumsq, ss);
  }
}

__global__ void fm_bias_update(float* w0, float* acc0, float* scal, float lr, int opt) {
  const float g = scal[0];
  if (opt == OPT_ADAGRAD) {
    const float a = acc0[0] + g * g;
    acc0[0] = a;
    w0[0] = w0[0] - lr * g * rsqrtf(a);
  } else {
    w0[0] = w0[0] - lr * g;
  }
}

__global__ void finish_loss(float* scal, float lam, float* loss) {
  loss[0] = scal[1] + lam * 0.5f * scal[2];   // + l2_regularizer(λ)(E) = λ·ΣE²/2
  scal[0] = scal[1] = scal[2] = scal[3] = 0.f;
}

static int grid_for_n(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace hhfm

using namespace hhfm;

extern "C" size_t hhfm_train_workspace(int64_t features_M, int32_t k) {
  // dE [M*k] + dw [M] + 4 scalars; must be zero-filled once by the caller
  return (size_t)features_M * k * 4 + (size_t)features_M * 4 + 64;
}

extern "C" int hhfm_fm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F,
                                  float* E, float* w, float* w0, int64_t features_M, int32_t k,
                                  float lr, float lam, int32_t optimizer, float* accE,
                                  float* accw, float* accw0, void* workspace, size_t ws_bytes,
                                  float* loss, void* stream) {
  if (B < 0 || F < 1 || k < 1 || features_M < 1) return HHFM_EINVAL;
  if (optimizer != OPT_ADAGRAD && optimizer != OPT_SGD) return HHFM_EUNSUPPORTED;
  if (!idx || !y || !E || !w || !w0 || !loss || !workspace) return HHFM_EINVAL;
  if (optimizer == OPT_ADAGRAD && (!accE || !accw || !accw0)) return HHFM_EINVAL;
  if (ws_bytes < hhfm_train_workspace(features_M, k)) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dE = reinterpret_cast<float*>(workspace);
  float* dw = dE + features_M * k;
  float* scal = dw + features_M;
  if (B > 0)
    hipLaunchKernelGGL(fm_train_rows, dim3(grid_for_n(B * 64)), dim3(256), 0, st, idx, y, B, F,
                       E, w, w0, features_M, k, dE, dw, scal);
  const int64_t nE = features_M * k;
  hipLaunchKernelGGL(optimizer_dense, dim3(grid_for_n(nE)), dim3(256), 0, st, E, dE, accE, nE,
                     lr, lam, optimizer, scal + 2);
  hipLaunchKernelGGL(optimizer_dense, dim3(grid_for_n(features_M)), dim3(256), 0, st, w, dw,
                     accw, features_M, lr, 0.f, optimizer, (float*)nullptr);
  hipLaunchKernelGGL(fm_bias_update, dim3(1), dim3(1), 0, st, w0, accw0, scal, lr, optimizer);
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
  if (optimizer != OPT_ADAGRAD && optimizer != OPT_SGD) return HHFM_EUNSUPPORTED;
  if (!X || !Neg || !E || !loss || !workspace) return HHFM_EINVAL;
  if (optimizer == OPT_ADAGRAD && !accE) return HHFM_EINVAL;
  if (ws_bytes < hhfm_train_workspace(features_M, k)) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dE = reinterpret_cast<float*>(workspace);
  float* scal = dE + features_M * k + features_M;
  if (B > 0)
    hipLaunchKernelGGL(hhfm_train_rows, dim3(grid_for_n(B * 64)), dim3(256), 0, st, X, Neg, B,
                       ncols, ctx_begin, ctx_end, time_begin, time_end, NG, E, features_M, k,
                       dE, scal);
  const int64_t nE = features_M * k;
  hipLaunchKernelGGL(optimizer_dense, dim3(grid_for_n(nE)), dim3(256), 0, st, E, dE, accE, nE,
                     lr, lam, optimizer, scal + 2);
  hipLaunchKernelGGL(finish_loss, dim3(1), dim3(1), 0, st, scal, lam, loss);
  return (int)hipGetLastError();
}
