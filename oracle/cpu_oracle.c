/*
 * cpu_oracle.c — TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).
 *
 * Plain-C restatement of the reference's TensorFlow-1.x scoring graphs
 * (data-man-34/HHFM), the same arithmetic as oracle/fm_oracle.py written as
 * sequential fp32 loops, parallelised over rows/queries with OpenMP.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 *   oracle_fm_out        FM.out            Newcode/FM.py:99-120
 *   oracle_hhfm_rows     OUR.PositiveFeadback Newcode/OurModel7.py:105-171
 *   oracle_catalog_topk  FM.topk  FM.py:172-185 (mode 0)
 *                        OUR.topk OurModel7.py:232-295 (mode 1)
 *                        + tf.nn.top_k order (score desc, index asc)
 * Tables are fp32 [M][k] (bf16 tables are upcast exactly by the caller).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}

int oracle_max_threads(void) { return omp_get_max_threads(); }

/* FM.py:99-120: Σ_k ½[(Σ_f e)² − Σ_f e²] + Σ_f w + w0 */
int oracle_fm_out(const int32_t* X, int64_t B, int F, const float* E, int k,
                  const float* w, float w0, float* out, int nthreads) {
  set_threads(nthreads);
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    const int32_t* x = X + b * F;
    float bil = 0.f;
    for (int e = 0; e < k; ++e) {
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const float v = E[(int64_t)x[f] * k + e];
        s += v;          /* reduce_sum(nonzero_embeddings, 1)   :100 */
        q += v * v;      /* reduce_sum(square(...), 1)          :105-106 */
      }
      bil += 0.5f * (s * s - q); /* 0.5*(summed² − squared_sum), Σ_k :109-117 */
    }
    float fb = 0.f;
    if (w)
      for (int f = 0; f < F; ++f) fb += w[x[f]]; /* Feature_bias :118 */
    out[b] = (bil + fb) + w0;                    /* add_n        :120 */
  }
  return 0;
}

/* OurModel7.py:122-171: h = u + Σctx (+ Σtime); out = Σ_k h·item */
int oracle_hhfm_rows(const int32_t* X, int64_t B, int ncols, int c0, int c1,
                     int t0, int t1, const float* E, int k, float* out,
                     int nthreads) {
  set_threads(nthreads);
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    const int32_t* x = X + b * ncols;
    float acc = 0.f;
    for (int e = 0; e < k; ++e) {
      float h = E[(int64_t)x[0] * k + e];
      if (c1 > c0) {
        float s = 0.f;
        for (int c = c0; c < c1; ++c) s += E[(int64_t)x[c] * k + e];
        h = h + s;
      }
      if (t1 > t0) {
        float s = 0.f;
        for (int c = t0; c < t1; ++c) s += E[(int64_t)x[c] * k + e];
        h = h + s;
      }
      acc += h * E[(int64_t)x[1] * k + e];
    }
    out[b] = acc;
  }
  return 0;
}

static int better(float as, int32_t ai, float bs, int32_t bi) {
  return as > bs || (as == bs && ai < bi);
}

/* Full-catalog score + top-K for queries A[B][ncols] over items
 * [item_begin, item_begin+N) of E; indices reported as offsets in [0, N). */
int oracle_catalog_topk(const int32_t* A, int64_t B, int ncols, int mode,
                        int c0, int c1, int t0, int t1, const float* E, int k,
                        const float* w, int64_t item_begin, int32_t N, int K,
                        float* top_s, int32_t* top_i, int nthreads) {
  if (K < 1 || K > N) return -1;
  set_threads(nthreads);
#pragma omp parallel
  {
    float* h = (float*)malloc(sizeof(float) * k);
    float* f = (float*)malloc(sizeof(float) * k);
    float* ls = (float*)malloc(sizeof(float) * K);
    int32_t* li = (int32_t*)malloc(sizeof(int32_t) * K);
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      const int32_t* a = A + b * ncols;
      for (int e = 0; e < k; ++e) {
        const float u = E[(int64_t)a[0] * k + e];
        float ctx = 0.f, tim = 0.f;
        for (int c = c0; c < c1; ++c) ctx += E[(int64_t)a[c] * k + e];
        for (int c = t0; c < t1; ++c) tim += E[(int64_t)a[c] * k + e];
        if (mode == 0) {            /* FM.py:176-177 */
          f[e] = ctx;
          h[e] = u + ctx;
        } else {                    /* OurModel7.py:270-292 */
          float x = u;
          if (c1 > c0) x = x + ctx;
          if (t1 > t0) x = x + tim;
          h[e] = x;
        }
      }
      int n = 0;
      /* Eight items per pass: each item keeps its own k-ordered fp32 chain
       * (the arithmetic of :178-185 / :294 unchanged); the eight independent
       * chains only give the CPU instruction-level parallelism. */
      for (int32_t it0 = 0; it0 < N; it0 += 8) {
        const int nb = N - it0 < 8 ? N - it0 : 8;
        float sc[8];
        const float* rows[8];
        for (int j = 0; j < 8; ++j) {
          sc[j] = 0.f;
          rows[j] = E + (item_begin + it0 + (j < nb ? j : 0)) * (int64_t)k;
        }
        if (mode == 0) {
          for (int e = 0; e < k; ++e)
            for (int j = 0; j < 8; ++j) sc[j] += h[e] * (rows[j][e] + f[e]); /* :178-183 */
        } else {
          for (int e = 0; e < k; ++e)
            for (int j = 0; j < 8; ++j) sc[j] += h[e] * rows[j][e];          /* :294 */
        }
        for (int j = 0; j < nb; ++j) {
          const int32_t it = it0 + j;
          float s = sc[j];
          if (mode == 0 && w) s = w[item_begin + it] + s;                    /* :184-185 */
          if (n == K && !better(s, it, ls[K - 1], li[K - 1])) continue;
          int p = n < K ? n : K - 1;
          while (p > 0 && better(s, it, ls[p - 1], li[p - 1])) {
            ls[p] = ls[p - 1];
            li[p] = li[p - 1];
            --p;
          }
          ls[p] = s;
          li[p] = it;
          if (n < K) ++n;
        }
      }
      memcpy(top_s + b * K, ls, sizeof(float) * K);
      memcpy(top_i + b * K, li, sizeof(int32_t) * K);
    }
    free(h); free(f); free(ls); free(li);
  }
  return 0;
}
