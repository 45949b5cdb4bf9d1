/*
 * lpa_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference hot path:
 *   GraphFrames 0.6.0 `labelPropagation(maxIter)` as called at
 *   /root/reference/CommunityDetection/Graphframes.py:81, whose arithmetic lives
 *   in Spark 2.4.5 GraphX (third-party, NOT vendored in /root/reference):
 *     graphx/lib/LabelPropagation.scala  sendMessage / mergeMessage / vertexProgram
 *     graphx/Pregel.scala                synchronous BSP loop (exactly maxIter updates)
 *   restated with the deterministic smallest-label tie-break of SURVEY.md App. A
 *   (GraphX breaks ties by Scala Map iteration order, which is not reproducible).
 * and the outlier stage of Graphframes.py:92-137 as SURVEY.md App. B defines it.
 *
 * Parity status: UNPINNED by the reference itself (the reference ships no tests
 * and no LPA outputs; GraphX/GraphFrames/Spark are absent here).  The oracle is
 * pinned to the upstream LabelPropagationSuite shape (two cliques + bridge) and
 * to the survey-time facts about the R9 sample (see tests/test_oracle.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  Built by oracle/Makefile into oracle/liboracle.so.
 */
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------- */
/* Counter-based RNG shared with the GPU generators (csrc/lpa_gen.hip).       */
/* splitmix64 finaliser; every draw is a pure function of (seed, edge, slot). */
/* ------------------------------------------------------------------------- */
static inline uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline uint64_t draw(uint64_t seed, uint64_t e, uint32_t slot) {
  return sm64(sm64(seed) + e * 32ull + slot);
}
/* uniform in [0, n) from a 32-bit draw (multiply-shift, no rejection) */
static inline uint32_t below(uint32_t r, uint32_t n) {
  return (uint32_t)(((uint64_t)r * n) >> 32);
}

/* Graph500 R-MAT quadrant thresholds A=.57 B=.19 C=.19 (D=.05) over 2^32. */
#define RMAT_TA 2448131358u  /* floor(0.57 * 2^32) */
#define RMAT_TB 3264175144u  /* floor(0.76 * 2^32) */
#define RMAT_TC 4080218931u  /* floor(0.95 * 2^32) */

/* bijective scramble of [0, 2^scale) (seeded vertex permutation) */
static inline uint64_t scramble(uint64_t x, int scale, uint64_t m1, uint64_t m2, uint64_t c1) {
  uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1ull);
  int sh = scale / 2 + 1;
  x = (x * m1 + c1) & mask;
  x ^= x >> sh;
  x = (x * m2) & mask;
  x ^= x >> sh;
  x = (x * m1 + c1) & mask;
  return x;
}

void oracle_gen_rmat(int32_t scale, int64_t m, uint64_t seed, int32_t scramble_ids,
                     int32_t* src, int32_t* dst) {
  uint64_t m1 = sm64(seed ^ 0x1234567ull) | 1ull;
  uint64_t m2 = sm64(seed ^ 0x89abcdefull) | 1ull;
  uint64_t c1 = sm64(seed ^ 0x5555ull);
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
    uint64_t u = 0, v = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 1) == 0) r = draw(seed, (uint64_t)e, (uint32_t)(l >> 1));
      uint32_t r32 = (l & 1) ? (uint32_t)r : (uint32_t)(r >> 32);
      uint64_t bu = 0, bv = 0;
      if (r32 < RMAT_TA) { bu = 0; bv = 0; }
      else if (r32 < RMAT_TB) { bu = 0; bv = 1; }
      else if (r32 < RMAT_TC) { bu = 1; bv = 0; }
      else { bu = 1; bv = 1; }
      u = (u << 1) | bu;
      v = (v << 1) | bv;
    }
    if (scramble_ids) { u = scramble(u, scale, m1, m2, c1); v = scramble(v, scale, m1, m2, c1); }
    src[e] = (int32_t)u;
    dst[e] = (int32_t)v;
  }
}

/* Chung-Lu power-law (config C5): P(i) ~ (i + i0)^(-1/(gamma-1))
 * over weight ranks, i0 by bisection so that the expected maximum degree is max_deg,
 * a quantized cumulative table Q[0..V] (Q[V] = 2^62), one 62-bit draw per endpoint,
 * rank -> id by the seeded affine permutation (mul * i + add) mod V.  Restates the
 * generator of csrc/lpa_gen.hip with the same double arithmetic in the same order. */
static uint64_t gcd_u64(uint64_t x, uint64_t y) {
  while (y) { uint64_t t = x % y; x = y; y = t; }
  return x;
}
static double cl_expmax(double x, int32_t V, int64_t m, double a) {
  double S = (pow((double)V + x, 1.0 - a) - pow(x, 1.0 - a)) / (1.0 - a) + 0.5 * pow(x, -a);
  return 2.0 * (double)m * pow(x, -a) / S;
}
int oracle_gen_chunglu(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed,
                       int32_t* src, int32_t* dst) {
  double a = 1.0 / (gamma - 1.0), i0 = 1.0;
  if (max_deg > 0.0) {
    double lo = log(1e-3), hi = log((double)V);
    for (int it = 0; it < 200; ++it) {
      double mid = 0.5 * (lo + hi);
      if (cl_expmax(exp(mid), V, m, a) > max_deg) lo = mid; else hi = mid;
    }
    i0 = exp(0.5 * (lo + hi));
  }
  uint64_t* Q = (uint64_t*)malloc(((size_t)V + 1) * sizeof(uint64_t));
  if (!Q) return -1;
  double W = 0.0, c = 0.0;
  for (int32_t i = 0; i < V; ++i) W += pow((double)i + i0, -a);
  for (int32_t i = 0; i < V; ++i) {
    Q[i] = (uint64_t)(c / W * 4611686018427387904.0);
    c += pow((double)i + i0, -a);
  }
  Q[V] = 1ull << 62;
  uint64_t mul = V > 1 ? sm64(seed ^ 0xC0FFEEull) % (uint64_t)V : 1ull;
  if (mul == 0) mul = 1;
  while (V > 1 && gcd_u64(mul, (uint64_t)V) != 1) mul = (mul + 1 == (uint64_t)V) ? 1 : mul + 1;
  uint64_t add = V > 1 ? sm64(seed ^ 0xADDull) % (uint64_t)V : 0ull;
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
    for (int k = 0; k < 2; ++k) {
      uint64_t r = draw(seed, (uint64_t)e, (uint32_t)k) >> 2;
      uint32_t lo = 0, hi = (uint32_t)V;
      while (hi - lo > 1) {
        uint32_t mid = lo + ((hi - lo) >> 1);
        if (Q[mid] <= r) lo = mid; else hi = mid;
      }
      int32_t id = (int32_t)((mul * (uint64_t)lo + add) % (uint64_t)V);
      if (k == 0) src[e] = id; else dst[e] = id;
    }
  }
  free(Q);
  return 0;
}

/* planted-partition SBM: u uniform; with p_in v uniform inside u's block,
 * otherwise uniform outside it. */
void oracle_gen_sbm(int32_t V, int32_t blocks, int64_t m, uint32_t p_in_q32, uint64_t seed,
                    int32_t* src, int32_t* dst) {
  uint32_t bs = (uint32_t)V / (uint32_t)blocks;
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
    uint64_t r0 = draw(seed, (uint64_t)e, 0);
    uint64_t r1 = draw(seed, (uint64_t)e, 1);
    uint32_t u = below((uint32_t)(r0 >> 32), (uint32_t)V);
    uint32_t b = u / bs;
    if (b >= (uint32_t)blocks) b = (uint32_t)blocks - 1;
    uint32_t lo = b * bs;
    uint32_t hi = (b == (uint32_t)blocks - 1) ? (uint32_t)V : lo + bs;
    uint32_t v;
    if ((uint32_t)(r0) < p_in_q32) {
      v = lo + below((uint32_t)(r1 >> 32), hi - lo);
    } else {
      uint32_t w = below((uint32_t)(r1 >> 32), (uint32_t)V - (hi - lo));
      v = (w < lo) ? w : w + (hi - lo);
    }
    src[e] = (int32_t)u;
    dst[e] = (int32_t)v;
  }
}

/* ------------------------------------------------------------------------- */
/* Symmetrised CSR (each directed edge (s,d) = one vote each way, App. A).     */
/* ------------------------------------------------------------------------- */
static int build_csr(int32_t V, int64_t m, const int32_t* src, const int32_t* dst,
                     int64_t** rp_out, int32_t** col_out) {
  int64_t* rp = (int64_t*)calloc((size_t)V + 1, sizeof(int64_t));
  int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * m > 0 ? 2 * m : 1));
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * ((size_t)V + 1));
  if (!rp || !col || !cur) { free(rp); free(col); free(cur); return -1; }
  /* parallel counting + scatter (full-size test configs have up to 2.8 B arcs); the
   * order of the neighbours inside a row is unspecified -- the mode does not depend
   * on it (mode_min_tie sorts) */
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
#pragma omp atomic
    rp[src[e] + 1]++;
#pragma omp atomic
    rp[dst[e] + 1]++;
  }
  for (int32_t v = 0; v < V; ++v) rp[v + 1] += rp[v];
  memcpy(cur, rp, sizeof(int64_t) * (size_t)V);
#pragma omp parallel for schedule(static)
  for (int64_t e = 0; e < m; ++e) {
    int64_t a, b;
#pragma omp atomic capture
    a = cur[src[e]]++;
#pragma omp atomic capture
    b = cur[dst[e]]++;
    col[a] = dst[e];
    col[b] = src[e];
  }
  free(cur);
  *rp_out = rp;
  *col_out = col;
  return 0;
}

/* LSD radix sort of uint32 keys (tmp = scratch of the same length). */
static void sort_u32(uint32_t* a, uint32_t* tmp, int64_t n) {
  if (n < 48) {
    for (int64_t i = 1; i < n; ++i) {
      uint32_t x = a[i];
      int64_t j = i - 1;
      while (j >= 0 && a[j] > x) { a[j + 1] = a[j]; --j; }
      a[j + 1] = x;
    }
    return;
  }
  uint32_t *in = a, *out = tmp;
  for (int sh = 0; sh < 32; sh += 8) {
    int64_t cnt[257];
    memset(cnt, 0, sizeof(cnt));
    for (int64_t i = 0; i < n; ++i) cnt[((in[i] >> sh) & 255u) + 1]++;
    for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
    for (int64_t i = 0; i < n; ++i) out[cnt[(in[i] >> sh) & 255u]++] = in[i];
    uint32_t* t = in; in = out; out = t;
  }
  /* 4 passes: result is back in `a` */
}

/* Mode of the multiset buf[0..d) with smallest-label tie-break (App. A step 2).
 * Returns the label; *is_tie = 1 when more than one label reaches the maximum. */
static uint32_t mode_min_tie(uint32_t* buf, uint32_t* tmp, int64_t d, int* is_tie) {
  sort_u32(buf, tmp, d);
  uint32_t best = buf[0];
  int64_t best_c = 0, nbest = 0;
  int64_t i = 0;
  while (i < d) {
    int64_t j = i + 1;
    while (j < d && buf[j] == buf[i]) ++j;
    int64_t c = j - i;
    if (c > best_c) { best_c = c; best = buf[i]; nbest = 1; }   /* ascending scan: first max = min label */
    else if (c == best_c) { nbest++; }
    i = j;
  }
  *is_tie = nbest > 1;
  return best;
}

/*
 * LPA-DET:
 *   L0[v] = v                                  (LabelPropagation.run mapVertices(vid => vid))
 *   exactly max_iter synchronous supersteps     (Pregel.apply loop)
 *   votes: each (s,d) votes L[d] at s and L[s] at d (sendMessage), counted with
 *   multiplicity (mergeMessage); isolated vertices keep their label (no message);
 *   new label = most frequent, smallest label on ties (vertexProgram, made deterministic).
 * iter_labels (nullable): max_iter x V labels after each superstep.
 * ties (nullable): per superstep number of vertices whose maximum is tied.
 * Returns 0, or -22 when max_iter <= 0 (GraphX require(maxSteps > 0)), -12 on OOM.
 */
int oracle_lpa(int32_t V, int64_t m, const int32_t* src, const int32_t* dst, int32_t max_iter,
               int32_t* labels_out, int32_t* iter_labels, int64_t* ties) {
  if (max_iter <= 0) return -22;
  if (V < 0 || m < 0) return -22;
  int64_t* rp;
  int32_t* col;
  if (build_csr(V, m, src, dst, &rp, &col)) return -12;
  int32_t* cur = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V > 0 ? V : 1));
  int32_t* nxt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V > 0 ? V : 1));
  if (!cur || !nxt) { free(rp); free(col); free(cur); free(nxt); return -12; }
  for (int32_t v = 0; v < V; ++v) cur[v] = v;
  int64_t maxd = 0;
  for (int32_t v = 0; v < V; ++v) if (rp[v + 1] - rp[v] > maxd) maxd = rp[v + 1] - rp[v];

  for (int32_t t = 0; t < max_iter; ++t) {
    int64_t nties = 0;
#pragma omp parallel reduction(+ : nties)
    {
      uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(maxd > 0 ? maxd : 1));
      uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(maxd > 0 ? maxd : 1));
#pragma omp for schedule(dynamic, 256)
      for (int32_t v = 0; v < V; ++v) {
        int64_t b = rp[v], e = rp[v + 1];
        if (e == b) { nxt[v] = cur[v]; continue; }
        for (int64_t k = b; k < e; ++k) buf[k - b] = (uint32_t)cur[col[k]];
        int tie = 0;
        nxt[v] = (int32_t)mode_min_tie(buf, tmp, e - b, &tie);
        nties += tie;
      }
      free(buf);
      free(tmp);
    }
    if (ties) ties[t] = nties;
    if (iter_labels) memcpy(iter_labels + (int64_t)t * V, nxt, sizeof(int32_t) * (size_t)V);
    int32_t* s = cur; cur = nxt; nxt = s;
  }
  memcpy(labels_out, cur, sizeof(int32_t) * (size_t)V);
  free(rp); free(col); free(cur); free(nxt);
  return 0;
}

/*
 * One superstep on a caller-built CSR (for the bench's CPU baseline: the timed
 * region excludes CSR construction exactly as the GPU timing does).
 */
int oracle_superstep_csr(int32_t V, const int64_t* rp, const int32_t* col, const int32_t* cur,
                         int32_t* nxt) {
  int64_t maxd = 0;
  for (int32_t v = 0; v < V; ++v) if (rp[v + 1] - rp[v] > maxd) maxd = rp[v + 1] - rp[v];
#pragma omp parallel
  {
    uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(maxd > 0 ? maxd : 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(maxd > 0 ? maxd : 1));
#pragma omp for schedule(dynamic, 256)
    for (int32_t v = 0; v < V; ++v) {
      int64_t b = rp[v], e = rp[v + 1];
      if (e == b) { nxt[v] = cur[v]; continue; }
      for (int64_t k = b; k < e; ++k) buf[k - b] = (uint32_t)cur[col[k]];
      int tie = 0;
      nxt[v] = (int32_t)mode_min_tie(buf, tmp, e - b, &tie);
    }
    free(buf);
    free(tmp);
  }
  return 0;
}

int oracle_build_csr(int32_t V, int64_t m, const int32_t* src, const int32_t* dst, int64_t* rp,
                     int32_t* col) {
  int64_t* r;
  int32_t* c;
  if (build_csr(V, m, src, dst, &r, &c)) return -12;
  memcpy(rp, r, sizeof(int64_t) * ((size_t)V + 1));
  memcpy(col, c, sizeof(int32_t) * (size_t)(2 * m));
  free(r);
  free(c);
  return 0;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------------- */
/* Outlier stage (Graphframes.py:92-137).               */
/* ------------------------------------------------------------------------- */

/* k-th smallest of vals[0..n) for k >= 1 (counting on a copy). */
static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

/* Threshold rule (App. B, a13): sort groups by (size desc, label asc);
 * k = n // 10; thr = sorted[-k].size if k > 0 else sorted[0].size
 * (Python's lst[-0] == lst[0], Graphframes.py:136).  sorted[-k] in descending
 * order is the k-th smallest size. */
static int64_t threshold_rule(int64_t* sizes, int64_t n) {
  if (n <= 0) return 0;
  qsort(sizes, (size_t)n, sizeof(int64_t), cmp_i64); /* ascending */
  int64_t k = n / 10;
  return k > 0 ? sizes[k - 1] : sizes[n - 1];
}

static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return (x > y) - (x < y);
}

/* distinct directed (s,d) pairs of E, as sorted uint64 keys (s<<32|d); returns count */
static int64_t distinct_edges(int64_t m, const int32_t* src, const int32_t* dst, uint64_t** out) {
  uint64_t* k = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(m > 0 ? m : 1));
  for (int64_t e = 0; e < m; ++e) k[e] = ((uint64_t)(uint32_t)src[e] << 32) | (uint32_t)dst[e];
  qsort(k, (size_t)m, sizeof(uint64_t), cmp_u64);
  int64_t n = 0;
  for (int64_t e = 0; e < m; ++e)
    if (n == 0 || k[n - 1] != k[e]) k[n++] = k[e];
  *out = k;
  return n;
}

/*
 * Mode L1 (App. B): size[l] = |{v : L[v]=l}| (Graphframes.py:100-104, :120);
 * inc[l] = |{distinct (s,d) : L[s]=l or L[d]=l}| (Graphframes.py:107-118);
 * threshold rule over the community sizes; flags[v] = size[L[v]] < thr.
 * summary = {n_groups, k, thr, n_flagged}.
 */
int oracle_outlier_l1(int32_t V, int64_t m, const int32_t* src, const int32_t* dst,
                      const int32_t* labels, int64_t* size_out, int64_t* inc_out,
                      uint8_t* flags_out, int64_t* summary) {
  memset(size_out, 0, sizeof(int64_t) * (size_t)V);
  memset(inc_out, 0, sizeof(int64_t) * (size_t)V);
  for (int32_t v = 0; v < V; ++v) size_out[labels[v]]++;
  uint64_t* de;
  int64_t nd = distinct_edges(m, src, dst, &de);
  for (int64_t i = 0; i < nd; ++i) {
    int32_t s = (int32_t)(de[i] >> 32), d = (int32_t)(uint32_t)de[i];
    int32_t ls = labels[s], ld = labels[d];
    inc_out[ls]++;
    if (ld != ls) inc_out[ld]++;
  }
  free(de);
  int64_t n = 0;
  for (int32_t l = 0; l < V; ++l) n += size_out[l] > 0;
  int64_t* sizes = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t j = 0;
  for (int32_t l = 0; l < V; ++l) if (size_out[l] > 0) sizes[j++] = size_out[l];
  int64_t thr = threshold_rule(sizes, n);
  free(sizes);
  int64_t nf = 0;
  for (int32_t v = 0; v < V; ++v) {
    flags_out[v] = (uint8_t)(size_out[labels[v]] < thr);
    nf += flags_out[v];
  }
  summary[0] = n;
  summary[1] = n / 10;
  summary[2] = thr;
  summary[3] = nf;
  return 0;
}

/*
 * Mode L2 (App. B; the commented Steps 5-6, Graphframes.py:121-137):
 *   E' = distinct (s,d) with L[s] = L[d]; L' = LPA-DET(V, E', sub_iter);
 *   per community l: threshold rule over the sizes of the sub-labels among l's
 *   members; flag members of sub-communities below it.
 * sub_labels_out (nullable): L'.  summary = {n_communities, n_subgroups, n_flagged,
 * n_communities_with_flags}.
 */
int oracle_outlier_l2(int32_t V, int64_t m, const int32_t* src, const int32_t* dst,
                      const int32_t* labels, int32_t sub_iter, int32_t* sub_labels_out,
                      uint8_t* flags_out, int64_t* summary) {
  uint64_t* de;
  int64_t nd = distinct_edges(m, src, dst, &de);
  int32_t* s2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nd > 0 ? nd : 1));
  int32_t* d2 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nd > 0 ? nd : 1));
  int64_t m2 = 0;
  for (int64_t i = 0; i < nd; ++i) {
    int32_t s = (int32_t)(de[i] >> 32), d = (int32_t)(uint32_t)de[i];
    if (labels[s] == labels[d]) { s2[m2] = s; d2[m2] = d; m2++; }
  }
  free(de);
  int32_t* sub = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V > 0 ? V : 1));
  int rc = oracle_lpa(V, m2, s2, d2, sub_iter, sub, NULL, NULL);
  free(s2);
  free(d2);
  if (rc) { free(sub); return rc; }
  if (sub_labels_out) memcpy(sub_labels_out, sub, sizeof(int32_t) * (size_t)V);
  /* groups = distinct (L, L') pairs with their member counts */
  uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(V > 0 ? V : 1));
  for (int32_t v = 0; v < V; ++v) key[v] = ((uint64_t)(uint32_t)labels[v] << 32) | (uint32_t)sub[v];
  qsort(key, (size_t)V, sizeof(uint64_t), cmp_u64);
  /* run-length over sorted pairs; per community l the counts of its sub-groups */
  int64_t* gcount = (int64_t*)malloc(sizeof(int64_t) * (size_t)(V > 0 ? V : 1));
  uint64_t* gkey = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(V > 0 ? V : 1));
  int64_t ng = 0;
  for (int32_t i = 0; i < V;) {
    int32_t j = i + 1;
    while (j < V && key[j] == key[i]) ++j;
    gkey[ng] = key[i];
    gcount[ng] = j - i;
    ng++;
    i = j;
  }
  free(key);
  /* thresholds per community; flagged (l,l') pairs marked in gflag */
  uint8_t* gflag = (uint8_t*)calloc((size_t)(ng > 0 ? ng : 1), 1);
  int64_t ncomm = 0, ncomm_flag = 0;
  int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ng > 0 ? ng : 1));
  for (int64_t i = 0; i < ng;) {
    int64_t j = i + 1;
    while (j < ng && (gkey[j] >> 32) == (gkey[i] >> 32)) ++j;
    int64_t n = j - i;
    for (int64_t q = 0; q < n; ++q) tmp[q] = gcount[i + q];
    int64_t thr = threshold_rule(tmp, n);
    int any = 0;
    for (int64_t q = i; q < j; ++q) if (gcount[q] < thr) { gflag[q] = 1; any = 1; }
    ncomm++;
    ncomm_flag += any;
    i = j;
  }
  free(tmp);
  int64_t nf = 0;
  for (int32_t v = 0; v < V; ++v) {
    uint64_t k = ((uint64_t)(uint32_t)labels[v] << 32) | (uint32_t)sub[v];
    int64_t lo = 0, hi = ng - 1;
    while (lo < hi) {
      int64_t mid = (lo + hi) / 2;
      if (gkey[mid] < k) lo = mid + 1; else hi = mid;
    }
    flags_out[v] = gflag[lo];
    nf += gflag[lo];
  }
  summary[0] = ncomm;
  summary[1] = ng;
  summary[2] = nf;
  summary[3] = ncomm_flag;
  free(gflag); free(gcount); free(gkey); free(sub);
  return 0;
}
