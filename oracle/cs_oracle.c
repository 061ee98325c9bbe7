/*
 * cs_oracle.c — CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.  The product
 * path (the package's C-ABI library) never calls it.
 *
 * A plain-C, fp64 restatement of the reference's scoring arithmetic, function by
 * function (citations relative to the reference root):
 *
 *   oracle_logsoftmax_gather  core.py:64-68 log_softmax_rows (S = M - max;
 *                             S - log(sum(exp(S)))), gathered at target ids as in
 *                             core.py:89-90 (ls[:, a_t]) and as the remote
 *                             echo=True prompt log-probs read by
 *                             src/utils.py:262-263.  Gemma-2 soft-capping
 *                             cap*tanh(x/cap) is applied first when cap > 0.
 *   oracle_segment_reduce     Python left-to-right folds: sum(valid)/len(valid)
 *                             (src/methods/best_of_n.py:303-305), np.mean of the
 *                             last len(path) log-probs (finite_lookahead.py:520),
 *                             mean(exp(lp)) (src/evaluation.py:211-212),
 *                             full_logprobs[-1:] (beam_search.py:389-390).
 *   oracle_welfare            min / sum / sum(log(max(u, eps))) / max over agents
 *                             in agent order (src/evaluation.py:337-381,
 *                             beam_search.py:558-560, best_of_n.py:384-408,
 *                             core.py:108-113, 374).
 *   oracle_topk               stable descending order, ties by index
 *                             (Python sorted(reverse=True) stability,
 *                             beam_search.py:558-560; np.argmax first max,
 *                             best_of_n.py:198).
 *
 * Row loops are OpenMP-parallel when built with -fopenmp (used only for the timed
 * CPU baseline; results do not depend on the thread count).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

enum { OR_F32 = 0, OR_BF16 = 1, OR_F16 = 2 };
enum { OR_MIN = 0, OR_SUM = 1, OR_SUMLOG = 2, OR_MAX = 3 };

static double f16_to_double(uint16_t h) {
  const int sign = (h >> 15) & 1;
  const int ex = (h >> 10) & 0x1f;
  const int man = h & 0x3ff;
  double v;
  if (ex == 0)
    v = ldexp((double)man, -24);
  else if (ex == 31)
    v = man ? NAN : INFINITY;
  else
    v = ldexp((double)(man | 0x400), ex - 25);
  return sign ? -v : v;
}

static double load_elem(const void* base, int dtype, int64_t i) {
  if (dtype == OR_F32) return (double)((const float*)base)[i];
  if (dtype == OR_BF16) {
    uint32_t u = (uint32_t)((const uint16_t*)base)[i] << 16;
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
  }
  return f16_to_double(((const uint16_t*)base)[i]);
}

static size_t elem_size(int dtype) { return dtype == OR_F32 ? 4 : 2; }

static double cap_fn(double x, double cap) { return cap > 0.0 ? cap * tanh(x / cap) : x; }

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void oracle_set_num_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* out_tok_lp[rows*k] (NaN for out-of-range targets), out_lse[rows] (nullable) */
void oracle_logsoftmax_gather(const void* logits, int dtype, int64_t rows, int64_t vocab,
                              int64_t ld, const int32_t* target_ids, int32_t k, double softcap,
                              double* out_tok_lp, double* out_lse) {
  const size_t es = elem_size(dtype);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t r = 0; r < rows; ++r) {
    const char* row = (const char*)logits + (size_t)r * (size_t)ld * es;
    double mx = -INFINITY;
    for (int64_t v = 0; v < vocab; ++v) {
      const double x = cap_fn(load_elem(row, dtype, v), softcap);
      if (x > mx) mx = x;
    }
    double sum = 0.0;
    for (int64_t v = 0; v < vocab; ++v) sum += exp(cap_fn(load_elem(row, dtype, v), softcap) - mx);
    const double lse = mx + log(sum);
    if (out_lse) out_lse[r] = lse;
    for (int32_t j = 0; j < k; ++j) {
      const int32_t t = target_ids[(size_t)r * k + j];
      out_tok_lp[(size_t)r * k + j] =
          (t >= 0 && t < vocab) ? (cap_fn(load_elem(row, dtype, t), softcap) - mx) - log(sum) : NAN;
    }
  }
}

void oracle_segment_reduce(const double* tok_lp, const int32_t* seg_offsets, int64_t n_seg,
                           double* out_sum_lp, double* out_sum_p, int32_t* out_count,
                           double* out_last) {
  for (int64_t s = 0; s < n_seg; ++s) {
    const int64_t b = seg_offsets[s], e = seg_offsets[s + 1];
    double a = 0.0, p = 0.0;
    int32_t c = 0;
    for (int64_t i = b; i < e; ++i) {
      const double v = tok_lp[i];
      if (isnan(v)) continue;
      a += v;
      p += exp(v);
      ++c;
    }
    if (out_sum_lp) out_sum_lp[s] = a;
    if (out_sum_p) out_sum_p[s] = p;
    if (out_count) out_count[s] = c;
    if (out_last) out_last[s] = (e > b) ? tok_lp[e - 1] : NAN;
  }
}

/* nonfinite: 0 = skip, 1 = replace with (nan_val, posinf_val, neginf_val) */
void oracle_welfare(const double* U, int32_t A, int32_t C, int64_t ldu, int kind, double eps,
                    int nonfinite, double nan_val, double posinf_val, double neginf_val,
                    double* W) {
  for (int32_t c = 0; c < C; ++c) {
    double acc = 0.0;
    int any = 0;
    for (int32_t a = 0; a < A; ++a) {
      double u = U[(size_t)a * ldu + c];
      if (!isfinite(u)) {
        if (nonfinite == 0) continue;
        u = isnan(u) ? nan_val : (u > 0 ? posinf_val : neginf_val);
      }
      switch (kind) {
        case OR_MIN: acc = any ? (u < acc ? u : acc) : u; break;
        case OR_MAX: acc = any ? (u > acc ? u : acc) : u; break;
        case OR_SUM: acc += u; break;
        default: acc += log(u > eps ? u : eps); break;
      }
      any = 1;
    }
    W[c] = any ? acc : NAN;
  }
}

/* greater-than in the selection order: value desc (NaN last), index asc */
static int ranks_before(double vj, int64_t j, double vi, int64_t i) {
  const int nj = isnan(vj), ni = isnan(vi);
  if (nj || ni) {
    if (nj && ni) return j < i;
    return ni; /* a number ranks before a NaN */
  }
  if (vj > vi) return 1;
  if (vj < vi) return 0;
  return j < i;
}

static const double* g_sort_vals;
static int cmp_rank(const void* pa, const void* pb) {
  const int32_t a = *(const int32_t*)pa, b = *(const int32_t*)pb;
  if (a == b) return 0;
  return ranks_before(g_sort_vals[a], a, g_sort_vals[b], b) ? -1 : 1;
}

void oracle_topk(const double* W, int32_t n_seg, int32_t seg_len, int64_t ld, int32_t k,
                 int32_t* out_idx) {
  int32_t* ord = (int32_t*)malloc(sizeof(int32_t) * (seg_len > 0 ? seg_len : 1));
  for (int32_t s = 0; s < n_seg; ++s) {
    for (int32_t i = 0; i < seg_len; ++i) ord[i] = i;
    g_sort_vals = W + (size_t)s * ld;
    qsort(ord, (size_t)seg_len, sizeof(int32_t), cmp_rank);
    for (int32_t r = 0; r < k; ++r) out_idx[(size_t)s * k + r] = ord[r];
  }
  free(ord);
}
