/*
 * tt_oracle.c -- CPU restatement of the reference's hot-path arithmetic (TEST INFRASTRUCTURE).
 *
 * This file is the CHECKER, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path (libtwotower_hip.so) never
 * links or calls it.
 *
 * Each function restates one reference computation in plain C float32, in the canonical
 * evaluation order that the HIP kernels implement (DESIGN.md "Canonical numerics"), so GPU
 * and oracle agree bit-for-bit where the doc says so.  The orders were chosen to be the
 * reference's own where the reference's order is observable on CPU:
 *   - numpy float32 pairwise sum (numpy loops_utils.h pairwise_sum) for np.linalg.norm as
 *     used by VectorDatabase (src/inference/vector_db.py:44, 152, 189): pinned bit-exact
 *     against numpy by tests/test_oracle.py.
 *   - faiss IndexFlatIP scores (vector_db.py:160,197; faiss-cpu >= 1.7.4, requirements.txt:26,
 *     3rd-party, absent offline): exact float32 inner product, results sorted descending.
 *     FAISS's own summation order (BLAS sgemm / SIMD fvec_inner_product) is build-dependent;
 *     ours is the MFMA fma chain below.  Pinned against an fp64 restatement within 1e-5.
 *   - torch reductions in BuyerTower (src/models/buyer_tower.py:43-101): torch's CPU
 *     summation order is vectorised and not reproduced; pinned within tolerance against
 *     golden outputs of the reference module itself (tests/golden/).
 * Compile: oracle/Makefile  ->  oracle/_build/libtt_oracle.so (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- numpy pairwise sum */
/* numpy/_core/src/umath/loops_utils.h.src  FLOAT_pairwise_sum, applied to x*x (the
 * float32 squares are rounded before summation: np.linalg.norm computes (x.conj()*x).real
 * then add.reduce). */
static float pw_sumsq(const float* a, int64_t n) {
  if (n < 8) {
    float res = 0.0f;
    for (int64_t i = 0; i < n; i++) {
      float p = a[i] * a[i];
      res = res + p;
    }
    return res;
  } else if (n <= 128) {
    float r[8];
    int64_t i;
    for (int j = 0; j < 8; j++) r[j] = a[j] * a[j];
    for (i = 8; i < n - (n % 8); i += 8) {
      for (int j = 0; j < 8; j++) {
        float p = a[i + j] * a[i + j];
        r[j] = r[j] + p;
      }
    }
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) {
      float p = a[i] * a[i];
      res = res + p;
    }
    return res;
  } else {
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pw_sumsq(a, n2) + pw_sumsq(a + n2, n - n2);
  }
}

float tto_norm(const float* x, int64_t d) { return sqrtf(pw_sumsq(x, d)); }

/* mode 0: x/(||x||+1e-8)  (vector_db.py:44-45)   mode 1: x/max(||x||,1e-12) (F.normalize) */
void tto_l2norm_rows(const float* x, int64_t n, int32_t d, int64_t ld_x, float* y, int64_t ld_y,
                     int32_t mode) {
  for (int64_t r = 0; r < n; r++) {
    const float* xr = x + r * ld_x;
    float nrm = tto_norm(xr, d);
    float den = mode == 0 ? nrm + 1e-8f : (nrm > 1e-12f ? nrm : 1e-12f);
    for (int32_t i = 0; i < d; i++) y[r * ld_y + i] = xr[i] / den;
    for (int64_t i = d; i < ld_y; i++) y[r * ld_y + i] = 0.0f;
  }
}

/* ---------------------------------------------------------------- canonical dot */
/* d is zero-padded to a multiple of 16 (padding contributes fmaf(0,0,acc) == acc).
 * Order: for t: for i in 0..3: for g in 0..3: acc = fmaf(x[16t+4g+i], q[16t+4g+i], acc)
 * == a chain of v_mfma_f32_16x16x4_f32 with lane-group g holding dims 16t+4g..+3. */
float tto_dot(const float* x, const float* q, int32_t d) {
  const int32_t dp = (d + 15) / 16 * 16;
  float acc = 0.0f;
  for (int32_t t = 0; t < dp / 16; t++)
    for (int i = 0; i < 4; i++)
      for (int g = 0; g < 4; g++) {
        const int32_t e = 16 * t + 4 * g + i;
        const float xv = e < d ? x[e] : 0.0f;
        const float qv = e < d ? q[e] : 0.0f;
        acc = fmaf(xv, qv, acc);
      }
  return acc;
}

/* ---------------------------------------------------------------- top-k */
typedef struct {
  float s;
  int64_t i;
} tto_pair;

static int better(const tto_pair* a, const tto_pair* b) { /* a ranks before b */
  const int an = a->s != a->s, bn = b->s != b->s;
  if (an != bn) return bn; /* NaN ranks last */
  if (!an && a->s != b->s) return a->s > b->s;
  return a->i < b->i;
}
static int cmp_pair(const void* pa, const void* pb) {
  const tto_pair* a = (const tto_pair*)pa;
  const tto_pair* b = (const tto_pair*)pb;
  if (better(a, b)) return -1;
  if (better(b, a)) return 1;
  return 0;
}

/* tto_dot for ROWS consecutive rows at once: the same per-row fmaf chain (order unchanged),
 * ROWS independent chains interleaved so the fma latency is hidden.  Columns >= d read as 0
 * (the padded tail block takes the branchy path). */
#define ROWS 8
static void dot_rows(const float* db, int64_t ld_db, int nr, const float* q, int32_t d,
                     float* out) {
  float acc[ROWS] = {0};
  const int32_t full = d / 16, dp = (d + 15) / 16 * 16;
  for (int32_t t = 0; t < full; t++)
    for (int i = 0; i < 4; i++)
      for (int g = 0; g < 4; g++) {
        const int32_t e = 16 * t + 4 * g + i;
        const float qv = q[e];
        if (nr == ROWS)
          for (int r = 0; r < ROWS; r++) acc[r] = fmaf(db[r * ld_db + e], qv, acc[r]);
        else
          for (int r = 0; r < nr; r++) acc[r] = fmaf(db[r * ld_db + e], qv, acc[r]);
      }
  for (int32_t t = full; t < dp / 16; t++)
    for (int i = 0; i < 4; i++)
      for (int g = 0; g < 4; g++) {
        const int32_t e = 16 * t + 4 * g + i;
        const float qv = e < d ? q[e] : 0.0f;
        for (int r = 0; r < nr; r++) acc[r] = fmaf(e < d ? db[r * ld_db + e] : 0.0f, qv, acc[r]);
      }
  for (int r = 0; r < nr; r++) out[r] = acc[r];
}

/* bounded heap of the k best pairs; heap[0] = the worst kept (better() is a strict total
 * order over distinct rows, so the kept set is exactly the sorted prefix of all pairs) */
static void heap_sift(tto_pair* h, int32_t m, int32_t j) {
  for (;;) {
    int32_t c = 2 * j + 1, w = j;
    if (c < m && better(&h[w], &h[c])) w = c;
    if (c + 1 < m && better(&h[w], &h[c + 1])) w = c + 1;
    if (w == j) return;
    tto_pair t = h[j];
    h[j] = h[w];
    h[w] = t;
    j = w;
  }
}
static void heap_push(tto_pair* h, int32_t* m, int32_t k, tto_pair p) {
  if (*m < k) {
    int32_t j = (*m)++;
    h[j] = p;
    while (j > 0) { /* sift up: parent must be worse than (better than) child */
      int32_t par = (j - 1) / 2;
      if (!better(&h[par], &h[j])) break;
      tto_pair t = h[par];
      h[par] = h[j];
      h[j] = t;
      j = par;
    }
  } else if (better(&p, &h[0])) {
    h[0] = p;
    heap_sift(h, *m, 0);
  }
}

/* Exact top-k (faiss IndexFlatIP.search semantics, vector_db.py:159-160): scores by
 * tto_dot, sorted descending, ties -> lower row; NaN never returned; tail (-inf, -1). */
void tto_scan_topk(const float* db, int64_t n, int32_t d, int64_t ld_db, int64_t row_base,
                   const float* q, int32_t nq, int64_t ld_q, int32_t k, float* out_s,
                   int64_t* out_i) {
  tto_pair* buf = (tto_pair*)malloc(sizeof(tto_pair) * (size_t)(k > 0 ? k : 1));
  float sc[ROWS];
  for (int32_t qi = 0; qi < nq; qi++) {
    int32_t m = 0;
    for (int64_t r0 = 0; r0 < n; r0 += ROWS) {
      const int nr = n - r0 < ROWS ? (int)(n - r0) : ROWS;
      dot_rows(db + r0 * ld_db, ld_db, nr, q + qi * ld_q, d, sc);
      for (int r = 0; r < nr; r++) {
        const float s = sc[r];
        if (s != s) continue;
        tto_pair p = {s + 0.0f, row_base + r0 + r};
        heap_push(buf, &m, k, p);
      }
    }
    qsort(buf, (size_t)m, sizeof(tto_pair), cmp_pair);
    for (int32_t j = 0; j < k; j++) {
      out_s[(int64_t)qi * k + j] = j < m ? buf[j].s : -INFINITY;
      out_i[(int64_t)qi * k + j] = j < m ? buf[j].i : -1;
    }
  }
  free(buf);
}

/* ---------------------------------------------------------------- buyer tower */
static void fnormalize(float* v, int32_t d) {
  float nrm = tto_norm(v, d);
  float den = nrm > 1e-12f ? nrm : 1e-12f;
  for (int32_t e = 0; e < d; e++) v[e] = v[e] / den;
}

/* BuyerTower.weighted_average (buyer_tower.py:58-66). items [b][s][d] (or gathered rows
 * from table by hist when table != NULL; hist < 0 -> zero row). */
void tto_weighted_avg_l2(const float* items, const float* table, int64_t ld_table,
                         const int64_t* hist, int64_t b, int32_t s, int32_t d, const float* w,
                         float* out, int64_t ld_out) {
  for (int64_t bi = 0; bi < b; bi++) {
    const float* wb = w + bi * s;
    float wsum = 0.0f;
    for (int32_t j = 0; j < s; j++) wsum = wsum + wb[j];
    wsum = wsum + 1e-8f;
    float* o = out + bi * ld_out;
    for (int32_t e = 0; e < d; e++) {
      float acc = 0.0f;
      for (int32_t j = 0; j < s; j++) {
        float nw = wb[j] / wsum;
        float x;
        if (table) {
          int64_t r = hist[bi * s + j];
          x = r >= 0 ? table[r * ld_table + e] : 0.0f;
        } else {
          x = items[(bi * s + j) * (int64_t)d + e];
        }
        float p = x * nw;
        acc = acc + p;
      }
      o[e] = acc;
    }
    fnormalize(o, d);
    for (int64_t e = d; e < ld_out; e++) o[e] = 0.0f;
  }
}

/* BuyerTower.attention_aggregation (buyer_tower.py:84-99), MLP Linear(d,h)-ReLU-Linear(h,1)
 * (buyer_tower.py:32-36).  W1 [h][d], b1 [h], W2 [h], b2 [1]. */
void tto_attn_agg_l2(const float* items, int64_t b, int32_t s, int32_t d, const float* w,
                     const float* W1, const float* b1, int32_t h, const float* W2,
                     const float* b2, float* out, int64_t ld_out) {
  float* c = (float*)malloc(sizeof(float) * (size_t)s);
  float* hs = (float*)malloc(sizeof(float) * (size_t)h);
  for (int64_t bi = 0; bi < b; bi++) {
    const float* xb = items + bi * (int64_t)s * d;
    for (int32_t j = 0; j < s; j++) {
      for (int32_t u = 0; u < h; u++) {
        float a = 0.0f;
        for (int32_t e = 0; e < d; e++) a = fmaf(W1[(int64_t)u * d + e], xb[(int64_t)j * d + e], a);
        a = a + b1[u];
        hs[u] = a > 0.0f ? a : 0.0f;
      }
      float a = 0.0f;
      for (int32_t u = 0; u < h; u++) a = fmaf(W2[u], hs[u], a);
      a = a + b2[0];
      c[j] = a * w[bi * s + j];
    }
    float m = -INFINITY;
    for (int32_t j = 0; j < s; j++) m = fmaxf(m, c[j]);
    float z = 0.0f;
    for (int32_t j = 0; j < s; j++) z = z + expf(c[j] - m);
    float* o = out + bi * ld_out;
    for (int32_t e = 0; e < d; e++) {
      float acc = 0.0f;
      for (int32_t j = 0; j < s; j++) {
        float alpha = expf(c[j] - m) / z;
        float p = xb[(int64_t)j * d + e] * alpha;
        acc = acc + p;
      }
      o[e] = acc;
    }
    fnormalize(o, d);
    for (int64_t e = d; e < ld_out; e++) o[e] = 0.0f;
  }
  free(c);
  free(hs);
}
