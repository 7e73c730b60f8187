/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of kamerkaya/SUPerman's Ryser / Gray-code exact permanent
 * algorithms, written from the reference's behaviour (file:line cited per
 * function).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the
 * reported CPU baseline.  The product (superman_amd/) never links or calls it.
 *
 * Pinning: the orc_ref_* functions are checked against golden vectors produced
 * by the reference's own CPU code compiled from /root/reference sources
 * (oracle/Makefile target `ref`, outputs in oracle/_ref/, vectors committed in
 * tests/golden/ by tests/golden/make_golden.py) and against exact big-integer
 * Ryser for small n (tests/exact.py).
 *
 * Deviations from the reference, all deliberate:
 *   - per-thread / per-chunk partials are combined in thread (chunk) order, not
 *     in `omp critical` completion order, so results are deterministic;
 *   - X is fp64 everywhere (v1's float X, algo.h:664, is wrong on reals);
 *   - sparse structure uses `!= 0` (v1 util.h:537 keeps only `> 0`).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAXN 64

/* gpu_exact_dense.cu:642-652 / cpu_algos.hpp:801-808 */
void orc_nw_start(const double* a, int n, double* x0, double* p0) {
  double p = 1.0;
  for (int j = 0; j < n; ++j) {
    double rs = 0.0;
    for (int k = 0; k < n; ++k) rs += a[j * n + k];
    x0[j] = a[j * n + (n - 1)] - rs / 2;
    p *= x0[j];
  }
  *p0 = p;
}

static void transpose(const double* a, int n, double* t) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) t[i * n + j] = a[j * n + i];
}

/* One thread's share of the dense Gray walk over [my_start, my_end):
 * gpu_exact_dense.cu:26-62 (cpu_perman64 body) == cpu_algos.hpp:831-866. */
static double dense_range(const double* mat_t, const double* x0, int n, long long my_start, long long my_end) {
  double x[ORC_MAXN];
  memcpy(x, x0, sizeof(double) * n);
  long long i = my_start;
  long long gray = (i - 1) ^ ((i - 1) >> 1);
  for (int k = 0; k < n - 1; ++k)
    if ((gray >> k) & 1LL)
      for (int j = 0; j < n; ++j) x[j] += mat_t[k * n + j];
  double my_p = 0;
  int prodSign = (i & 1LL) ? -1 : 1;
  while (i < my_end) {
    int k = __builtin_ctzll(i);
    gray ^= (1LL << k);
    double s = ((1LL << k) & gray) ? 1.0 : -1.0;
    double prod = 1.0;
    for (int j = 0; j < n; ++j) {
      x[j] += s * mat_t[k * n + j];
      prod *= x[j];
    }
    my_p += prodSign * prod;
    prodSign *= -1;
    i++;
  }
  return my_p;
}

/* cpu_algos.hpp:761-873 parallel_perman64<double,double>:
 * chunk_size = end/threads + 1, thread t walks [1 + t*cs, min(1+(t+1)*cs, end)). */
double orc_ref_dense(const double* a, int n, int threads) {
  double x0[ORC_MAXN], p;
  orc_nw_start(a, n, x0, &p);
  double* mat_t = (double*)malloc(sizeof(double) * n * n);
  transpose(a, n, mat_t);
  const long long start = 1, end = 1LL << (n - 1);
  const long long cs = end / threads + 1;
  double* part = (double*)calloc(threads, sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(static, 1)
  for (int tid = 0; tid < threads; ++tid) {
    long long ms = start + tid * cs;
    long long me = start + (tid + 1) * cs;
    if (me > end) me = end;
    part[tid] = dense_range(mat_t, x0, n, ms, me);
  }
  for (int tid = 0; tid < threads; ++tid) p += part[tid];
  free(part);
  free(mat_t);
  return (4 * (n & 1) - 2) * p;
}

/* gpu_exact_dense.cu:6-69 cpu_perman64: partial over [start, end) with
 * chunk_size = (end-start)/threads + 1 (no p0, no final factor). */
double orc_ref_dense_partial(const double* a, int n, long long start, long long end, int threads) {
  double x0[ORC_MAXN], p0;
  orc_nw_start(a, n, x0, &p0);
  double* mat_t = (double*)malloc(sizeof(double) * n * n);
  transpose(a, n, mat_t);
  const long long cs = (end - start) / threads + 1;
  double* part = (double*)calloc(threads, sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(static, 1)
  for (int tid = 0; tid < threads; ++tid) {
    long long ms = start + tid * cs;
    long long me = start + (tid + 1) * cs;
    if (me > end) me = end;
    part[tid] = dense_range(mat_t, x0, n, ms, me);
  }
  double p = 0.0;
  for (int tid = 0; tid < threads; ++tid) p += part[tid];
  free(part);
  free(mat_t);
  return p;
}

/* ------------------------------------------------------------------ sparse */
typedef struct {
  int n, nnz;
  int cptrs[ORC_MAXN + 1], rptrs[ORC_MAXN + 1];
  int rows[ORC_MAXN * ORC_MAXN], cols[ORC_MAXN * ORC_MAXN];
  double cvals[ORC_MAXN * ORC_MAXN], rvals[ORC_MAXN * ORC_MAXN];
} csx;

/* util.h:522-551 matrix2compressed (!= 0) */
static void compress(const double* a, int n, csx* s) {
  int er = 0, ec = 0;
  s->n = n;
  for (int i = 0; i < n; ++i) {
    s->rptrs[i] = er;
    s->cptrs[i] = ec;
    for (int j = 0; j < n; ++j) {
      if (a[i * n + j] != 0) {
        s->cols[er] = j;
        s->rvals[er++] = a[i * n + j];
      }
      if (a[j * n + i] != 0) {
        s->rows[ec] = j;
        s->cvals[ec++] = a[j * n + i];
      }
    }
  }
  s->rptrs[n] = er;
  s->cptrs[n] = ec;
  s->nnz = er;
}

/* cpu_algos.hpp:682-749 (per-thread body) == gpu_exact_sparse.cu:14-80 */
static double sparse_range(const csx* s, const double* x0, int n, long long my_start, long long my_end) {
  double x[ORC_MAXN];
  memcpy(x, x0, sizeof(double) * n);
  long long i = my_start;
  long long gray = (i - 1) ^ ((i - 1) >> 1);
  for (int k = 0; k < n - 1; ++k)
    if ((gray >> k) & 1LL)
      for (int j = s->cptrs[k]; j < s->cptrs[k + 1]; ++j) x[s->rows[j]] += s->cvals[j];
  double prod = 1.0;
  int zero_num = 0;
  for (int j = 0; j < n; ++j) {
    if (x[j] == 0) zero_num++;
    else prod *= x[j];
  }
  double my_p = 0;
  int prodSign = (i & 1LL) ? -1 : 1;
  while (i < my_end) {
    int k = __builtin_ctzll(i);
    gray ^= (1LL << k);
    double sg = ((1LL << k) & gray) ? 1.0 : -1.0;
    for (int j = s->cptrs[k]; j < s->cptrs[k + 1]; ++j) {
      const int r = s->rows[j];
      if (x[r] == 0) {
        zero_num--;
        x[r] += sg * s->cvals[j];
        prod *= x[r];
      } else {
        prod /= x[r];
        x[r] += sg * s->cvals[j];
        if (x[r] == 0) zero_num++;
        else prod *= x[r];
      }
    }
    if (zero_num == 0) my_p += prodSign * prod;
    prodSign *= -1;
    i++;
  }
  return my_p;
}

/* cpu_algos.hpp:635-757 parallel_perman64_sparse<double,double> */
double orc_ref_sparse(const double* a, int n, int threads) {
  csx* S = (csx*)malloc(sizeof(csx));
  compress(a, n, S);
  double x0[ORC_MAXN], p;
  orc_nw_start(a, n, x0, &p);
  const long long start = 1, end = 1LL << (n - 1);
  const long long cs = end / threads + 1;
  double* part = (double*)calloc(threads, sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(static, 1)
  for (int tid = 0; tid < threads; ++tid) {
    long long ms = start + tid * cs;
    long long me = start + (tid + 1) * cs;
    if (me > end) me = end;
    part[tid] = sparse_range(S, x0, n, ms, me);
  }
  for (int tid = 0; tid < threads; ++tid) p += part[tid];
  free(part);
  free(S);
  return (4 * (n & 1) - 2) * p;
}

/* gpu_exact_sparse.cu:6-87 cpu_perman64_sparse (partial, no p0) */
double orc_ref_sparse_partial(const double* a, int n, long long start, long long end, int threads) {
  csx* S = (csx*)malloc(sizeof(csx));
  compress(a, n, S);
  double x0[ORC_MAXN], p0;
  orc_nw_start(a, n, x0, &p0);
  const long long cs = (end - start) / threads + 1;
  double* part = (double*)calloc(threads, sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(static, 1)
  for (int tid = 0; tid < threads; ++tid) {
    long long ms = start + tid * cs;
    long long me = start + (tid + 1) * cs;
    if (me > end) me = end;
    part[tid] = sparse_range(S, x0, n, ms, me);
  }
  double p = 0.0;
  for (int tid = 0; tid < threads; ++tid) p += part[tid];
  free(part);
  free(S);
  return p;
}

/* One SkipPer chunk [my_start, my_end) starting from x (copied):
 * cpu_algos.hpp:1122-1196 == gpu_exact_sparse.cu:110-186.  Returns the partial
 * and adds the number of evaluated products to *visited. */
static double skip_range(const csx* s, const double* xin, int n, unsigned long long my_start,
                         unsigned long long my_end, unsigned long long* visited) {
  double my_x[ORC_MAXN];
  memcpy(my_x, xin, sizeof(double) * n);
  double my_p = 0;
  unsigned long long my_prev_gray = 0, i = my_start, vis = 0;
  while (i < my_end) {
    unsigned long long my_gray = i ^ (i >> 1);
    unsigned long long gray_diff = my_prev_gray ^ my_gray;
    int j = 0;
    while (gray_diff > 0) {
      unsigned long long onej = 1ULL << j;
      if (gray_diff & onej) {
        gray_diff ^= onej;
        if (my_gray & onej) {
          for (int ptr = s->cptrs[j]; ptr < s->cptrs[j + 1]; ptr++) my_x[s->rows[ptr]] += s->cvals[ptr];
        } else {
          for (int ptr = s->cptrs[j]; ptr < s->cptrs[j + 1]; ptr++) my_x[s->rows[ptr]] -= s->cvals[ptr];
        }
      }
      j++;
    }
    my_prev_gray = my_gray;
    int last_zero = -1;
    double my_prod = 1;
    for (j = n - 1; j >= 0; j--) {
      my_prod *= my_x[j];
      if (my_x[j] == 0) {
        last_zero = j;
        break;
      }
    }
    vis++;
    if (my_prod != 0 || last_zero < 0) {  /* last_zero < 0: underflow, no zero row (ref reads rptrs[-1]) */
      my_p += ((i & 1ULL) ? -1.0 : 1.0) * my_prod;
      i++;
    } else {
      unsigned long long change_j = ~0ULL;
      for (int ptr = s->rptrs[last_zero]; ptr < s->rptrs[last_zero + 1]; ptr++) {
        unsigned long long step_start = 1ULL << s->cols[ptr];
        unsigned long long period = step_start << 1;
        unsigned long long ci = step_start;
        if (i >= step_start) {
          unsigned long long steps = (i - step_start) / period;
          ci = step_start + ((steps + 1) * period);
        }
        if (ci < change_j) change_j = ci;
      }
      i++;
      if (change_j > i) i = change_j;
    }
  }
  *visited += vis;
  return my_p;
}

/* cpu_algos.hpp:1035-1213 parallel_skip_perman64_w_balanced<double,double>
 * (512 chunks; chunk partials summed in chunk order). */
double orc_ref_skip(const double* a, int n, int threads, unsigned long long* visited) {
  csx* S = (csx*)malloc(sizeof(csx));
  compress(a, n, S);
  double x[ORC_MAXN];
  for (int j = 0; j < n; j++) {
    double rs = 0.0;
    for (int ptr = S->rptrs[j]; ptr < S->rptrs[j + 1]; ptr++) rs += S->rvals[ptr];
    x[j] = -rs / (2.0f);
  }
  for (int ptr = S->cptrs[n - 1]; ptr < S->cptrs[n]; ptr++) x[S->rows[ptr]] += S->cvals[ptr];
  double prod = 1;
  for (int j = 0; j < n; j++) prod *= x[j];
  double p = prod;
  unsigned long long start = 1;
  for (int j = 0; j < n; j++) {
    if (x[j] == 0) {
      unsigned long long change_j = ~0ULL;
      for (int ptr = S->rptrs[j]; ptr < S->rptrs[j + 1]; ptr++) {
        unsigned long long ci = 1ULL << S->cols[ptr];
        if (ci < change_j) change_j = ci;
      }
      if (change_j > start) start = change_j;
    }
  }
  const unsigned long long end = 1ULL << (n - 1);
  const int no_chunks = 512;
  const unsigned long long cs = (end - start + 1) / no_chunks + 1;
  double* part = (double*)calloc(no_chunks, sizeof(double));
  unsigned long long* vis = (unsigned long long*)calloc(no_chunks, sizeof(unsigned long long));
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (int cid = 0; cid < no_chunks; cid++) {
    unsigned long long ms = start + cid * cs;
    unsigned long long me = start + (cid + 1) * cs;
    if (me > end) me = end;
    part[cid] = (ms < me) ? skip_range(S, x, n, ms, me, &vis[cid]) : 0.0;
  }
  unsigned long long tv = 0;
  for (int cid = 0; cid < no_chunks; cid++) {
    p += part[cid];
    tv += vis[cid];
  }
  if (visited) *visited = tv;
  free(part);
  free(vis);
  free(S);
  return (4 * (n & 1) - 2) * p;
}

/* gpu_exact_sparse.cu:89-191 cpu_perman64_skipper (partial over [start,end), x0 from the dense
 * prologue as in the wrapper gpu_exact_sparse.cu:1207-1218, 512 chunks). */
double orc_ref_skip_partial(const double* a, int n, long long start, long long end, int threads) {
  csx* S = (csx*)malloc(sizeof(csx));
  compress(a, n, S);
  double x0[ORC_MAXN], p0;
  orc_nw_start(a, n, x0, &p0);
  const int no_chunks = 512;
  const unsigned long long cs = (unsigned long long)(end - start + 1) / no_chunks + 1;
  double* part = (double*)calloc(no_chunks, sizeof(double));
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (int cid = 0; cid < no_chunks; cid++) {
    unsigned long long ms = start + cid * cs;
    unsigned long long me = start + (cid + 1) * cs;
    if (me > (unsigned long long)end) me = end;
    unsigned long long v = 0;
    part[cid] = (ms < me) ? skip_range(S, x0, n, ms, me, &v) : 0.0;
  }
  double p = 0.0;
  for (int cid = 0; cid < no_chunks; cid++) p += part[cid];
  free(part);
  free(S);
  return p;
}

/* ====================================================================== *
 * Engine-schedule mirror: the same Ryser sum, enumerated exactly as the
 * gfx950 kernels do, so the GPU result can be checked
 * bit-for-bit.  Independent restatement of the engine's spec:
 *   Gray bits: [0,L) lanes, [L,L+m) walk, [L+m,n-1) wave-chunk index a;
 *   lane state  x = x0 + sum_{b in gray(a)} A[:,L+m+b] (ascending b)
 *                    + sum_{e<L, lane bit e} A[:,e] via fma(sel, c, x);
 *   walk t=1..2^m-1 flips walk bit k=ctz(t), neg=(t>>(k+1))&1;
 *   term(t) = (-1)^t * prod, lane result negated if (a ^ popcount(lane)) & 1;
 *   wave value = pairwise tree over the 64 lanes (lanes >= 2^L give 0);
 *   range value = pairwise tree over wave-chunks, 64-way zero padded.
 * ====================================================================== */
typedef struct {
  int n, NP, kind, L, m, h;
  int rowperm[ORC_MAXN], colmap[ORC_MAXN], nblk[ORC_MAXN];
  unsigned long long rowmask[ORC_MAXN], umask;
  double x0[ORC_MAXN];
  double col[2 * ORC_MAXN][ORC_MAXN]; /* [2e+neg][j] */
  /* segmented walk (kind 3): segment i = rows [seg[i], seg[i+1]), rest = [seg[nseg], n) */
  int nseg, seg[ORC_MAXN + 1], segb, len0, cc; /* cc: cached walk bits 1..cc */
  int nsub, sub[ORC_MAXN + 1];    /* sub-segments of segment 0 */
  char dyn[ORC_MAXN];             /* rows some walk bit > segb touches */
} eplan;

/* Layout: L = min(6, n-1); m = max(min(rest, 10), rest - 20), shortened for small n (rest - m < 13)
   to max(min(rest, 6), rest - 13) so that there are 2^13 wave-chunks; h = rest - m. */
void orc_engine_layout(int n, int* L, int* m, int* h) {
  int nb = n - 1;
  int l = nb < 6 ? nb : 6;
  int rest = nb - l;
  int mm = rest < 10 ? rest : 10;
  if (rest - mm < 13) {  /* small n: shorter walks, 2^13 wave-chunks */
    int lo = rest < 6 ? rest : 6;
    mm = rest - 13 > lo ? rest - 13 : lo;
  }
  if (rest - 20 > mm) mm = rest - 20;
  if (mm > 31) mm = 31;
  *L = l;
  *m = mm;
  *h = rest - mm;
}

static void engine_plan(const double* a, int n, int kind, const int* colmap, int L, int m, int cc, int segb,
                        eplan* P) {
  memset(P, 0, sizeof(*P));
  P->cc = cc;
  P->n = n;
  P->NP = (n + 7) & ~7;
  P->kind = kind;
  P->L = L;
  P->m = m;
  P->h = n - 1 - L - m;
  int nb = n - 1;
  for (int e = 0; e < nb; ++e) P->colmap[e] = colmap ? colmap[e] : e;
  for (int j = 0; j < n; ++j) P->rowperm[j] = j;
  if (kind != 0) {
    char placed[ORC_MAXN] = {0};
    int cnt = 0;
    for (int k = 0; k < m; ++k) {
      int c = P->colmap[L + k];
      for (int i = 0; i < n; ++i)
        if (!placed[i] && a[i * n + c] != 0.0) {
          placed[i] = 1;
          P->rowperm[cnt++] = i;
        }
      P->nblk[L + k] = (cnt + 7) / 8;
    }
    for (int i = 0; i < n; ++i)
      if (!placed[i]) P->rowperm[cnt++] = i;
    if (kind == 3) {
      /* segmented walk: the rows of walk column 0 first, ordered by first
       * touch among walk columns 1.., the ones no other walk column touches
       * last; then the other rows in first-touch order (jit.cpp seg_row_order) */
      char pl[ORC_MAXN] = {0}, in0[ORC_MAXN] = {0};
      int c0 = P->colmap[L];
      cnt = 0;
      for (int i = 0; i < n; ++i) in0[i] = a[i * n + c0] != 0.0;
      for (int k = 1; k < m; ++k)
        for (int i = 0; i < n; ++i)
          if (in0[i] && !pl[i] && a[i * n + P->colmap[L + k]] != 0.0) pl[i] = 1, P->rowperm[cnt++] = i;
      for (int i = 0; i < n; ++i)
        if (in0[i] && !pl[i]) pl[i] = 1, P->rowperm[cnt++] = i;
      for (int k = 1; k < m; ++k)
        for (int i = 0; i < n; ++i)
          if (!pl[i] && a[i * n + P->colmap[L + k]] != 0.0) pl[i] = 1, P->rowperm[cnt++] = i;
      for (int i = 0; i < n; ++i)
        if (!pl[i]) P->rowperm[cnt++] = i;
    }
  }
  for (int e = 0; e < nb; ++e)
    if (e < L || e >= L + m) P->nblk[e] = (n + 7) / 8;
  for (int e = 0; e < nb; ++e)
    for (int j = 0; j < n; ++j) {
      double v = a[P->rowperm[j] * n + P->colmap[e]];
      P->col[2 * e][j] = v;
      P->col[2 * e + 1][j] = -v;
    }
  double x0[ORC_MAXN], p0;
  orc_nw_start(a, n, x0, &p0);
  for (int j = 0; j < n; ++j) P->x0[j] = x0[P->rowperm[j]];
  P->umask = 0;
  for (int j = 0; j < n; ++j) {
    int i = P->rowperm[j], touched = 0;
    for (int e = 0; e < L; ++e)
      if (a[i * n + P->colmap[e]] != 0.0) touched = 1;
    if (!touched) P->umask |= 1ULL << j;
    unsigned long long rm = 0;
    for (int k = 0; k < m; ++k)
      if (a[i * n + P->colmap[L + k]] != 0.0) rm |= 1ULL << k;
    P->rowmask[j] = rm;
  }
  if (kind == 3) {
    /* segments: the rows each walk bit touches first (rows are in first-touch order) */
    int R = 0;
    char seen[ORC_MAXN] = {0};
    P->nseg = 0;
    P->seg[0] = 0;
    for (int k = 0; k < m; ++k) {
      for (int j = 0; j < n; ++j)
        if (P->col[2 * (L + k)][j] != 0.0 && !seen[j]) seen[j] = 1, ++R;
      if (R > P->seg[P->nseg]) P->seg[++P->nseg] = R;
    }
    P->len0 = P->seg[1];
    /* sub-segments of segment 0: first touch by walk bits 1.. */
    char got[ORC_MAXN] = {0};
    int c = 0;
    P->nsub = 0;
    P->sub[0] = 0;
    for (int k = 1; k < m; ++k) {
      for (int j = 0; j < P->len0; ++j)
        if (P->col[2 * (L + k)][j] != 0.0 && !got[j]) got[j] = 1, ++c;
      if (c > P->sub[P->nsub]) P->sub[++P->nsub] = c;
    }
    /* pair steps flip walk bits k >= 1; bits k <= segb (the plan's choice,
     * sup_plan_info pair_bits; 0 = the default min(m-1, 5)) get their own
     * step (touched rows), bits > segb share one step over the union of
     * their rows (jit.cpp) */
    P->segb = segb > 0 ? segb : 5;
    if (P->segb > m - 1) P->segb = m - 1;
    for (int k = P->segb + 1; k < m; ++k)
      for (int j = 0; j < n; ++j)
        if (P->col[2 * (L + k)][j] != 0.0) P->dyn[j] = 1;
  }
}

static double e_prod4(const double* x, int n) {
  double p0 = x[0], p1 = n > 1 ? x[1] : 1.0, p2 = n > 2 ? x[2] : 1.0, p3 = n > 3 ? x[3] : 1.0;
  for (int j = 4; j < n; j += 4) {
    p0 *= x[j];
    if (j + 1 < n) p1 *= x[j + 1];
    if (j + 2 < n) p2 *= x[j + 2];
    if (j + 3 < n) p3 *= x[j + 3];
  }
  return (p0 * p1) * (p2 * p3);
}

static double e_bprod8(const double* x, int n, int b) {
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = (8 * b + i < n) ? x[8 * b + i] : 1.0;
  return ((v[0] * v[1]) * (v[2] * v[3])) * ((v[4] * v[5]) * (v[6] * v[7]));
}

static void e_suffix(const double* x, int n, double* U) {
  int NB = (n + 7) / 8;
  U[NB] = 1.0;
  for (int b = NB - 1; b >= 0; --b) U[b] = e_bprod8(x, n, b) * U[b + 1];
}

static void e_sparse_step(double* x, double* U, int n, const double* col, int nb) {
  int NB = (n + 7) / 8;
  for (int b = 0; b < NB && b < nb; ++b)
    for (int j = 8 * b; j < 8 * b + 8 && j < n; ++j) x[j] += col[j];
  for (int b = NB - 1; b >= 0; --b)
    if (b < nb) U[b] = e_bprod8(x, n, b) * U[b + 1];
}

static void e_start(const eplan* P, unsigned long long ga, unsigned lane, double* x) {
  int n = P->n;
  for (int j = 0; j < n; ++j) x[j] = P->x0[j];
  unsigned long long h = ga ^ (ga >> 1);
  for (int b = 0; h; ++b, h >>= 1)
    if (h & 1)
      for (int j = 0; j < n; ++j) x[j] += P->col[2 * (P->L + P->m + b)][j];
  for (int e = 0; e < P->L; ++e) {
    double sel = ((lane >> e) & 1u) ? 1.0 : 0.0;
    for (int j = 0; j < n; ++j) x[j] = fma(sel, P->col[2 * e][j], x[j]);
  }
}

/* segmented walk: segment product = recursive halving tree (jit.cpp tree()) */
static double e_tree(const double* x, int lo, int hi) {
  if (hi - lo == 1) return x[lo];
  int mid = lo + (hi - lo + 1) / 2;
  return e_tree(x, lo, mid) * e_tree(x, mid, hi);
}

/* segmented walk products: a binary product tree per row group.  Items are
 * the group's rows [lo, tlo) (each with the set of step classes touching it:
 * class k-1 for walk bit k <= segb, class segb for any walk bit > segb) and,
 * if rows [tlo, thi) exist, one constant item = e_tree over them.  Built
 * greedily: join the two clusters (in list order, first pair i < j on ties)
 * whose union of classes has the least weight, weight(class c < segb) =
 * 2^(segb-1-c), weight(class segb) = 1, cached classes (c < cc) weigh 0 and
 * double the weight of the rest; the joined cluster is appended.  A
 * step of class c re-forms the nodes whose class set holds c, in creation
 * order (jit.cpp make_tree). */
typedef struct {
  int ni, K, tlo, thi;
  int row[ORC_MAXN + 1];             /* item -> row, -1 = constant item */
  unsigned isig[ORC_MAXN + 1];
  int a[2 * ORC_MAXN], b[2 * ORC_MAXN];
  unsigned sig[2 * ORC_MAXN];
} etree;
typedef struct {
  double N[2 * ORC_MAXN], T;
} etv;

static unsigned long long e_weight(unsigned s, int segb, int cc) {
  unsigned long long w = 0;
  for (int c = cc; c <= segb; ++c)
    if ((s >> c) & 1u) w += c < segb ? (1ULL << (segb - 1 - c)) : 1ULL;
  return w << __builtin_popcount(s & ((1u << cc) - 1u)); /* one copy per cached state it depends on */
}

static void e_tree_build(etree* t, const unsigned* rsig, int lo, int tlo, int thi, int segb, int cc) {
  int id[ORC_MAXN + 1], cnt = 0;
  unsigned sg[ORC_MAXN + 1];
  t->ni = 0, t->K = 0, t->tlo = tlo, t->thi = thi;
  for (int r = lo; r < tlo; ++r) t->row[t->ni] = r, t->isig[t->ni++] = rsig[r];
  if (thi > tlo) t->row[t->ni] = -1, t->isig[t->ni++] = 0;
  for (int i = 0; i < t->ni; ++i) id[cnt] = i, sg[cnt++] = t->isig[i];
  while (cnt > 1) {
    int bi = 0, bj = 1;
    unsigned long long bw = ~0ULL;
    for (int i = 0; i < cnt; ++i)
      for (int j = i + 1; j < cnt; ++j) {
        unsigned long long w = e_weight(sg[i] | sg[j], segb, cc);
        if (w < bw) bw = w, bi = i, bj = j;
      }
    unsigned ns = sg[bi] | sg[bj];
    t->a[t->K] = id[bi], t->b[t->K] = id[bj], t->sig[t->K] = ns;
    ++t->K;
    /* drop positions bi < bj, keep the order of the rest, append the join */
    int w = 0;
    for (int i = 0; i < cnt; ++i)
      if (i != bi && i != bj) id[w] = id[i], sg[w++] = sg[i];
    id[w] = t->ni + t->K - 1, sg[w++] = ns;
    cnt = w;
  }
}

static double e_tv_id(const etree* t, const double* a, const etv* v, int id) {
  if (id < t->ni) return t->row[id] < 0 ? v->T : a[t->row[id]];
  return v->N[id - t->ni];
}
static void e_tree_init(const etree* t, const double* a, etv* v) {
  v->T = t->thi > t->tlo ? e_tree(a, t->tlo, t->thi) : 1.0;
  for (int i = 0; i < t->K; ++i) v->N[i] = e_tv_id(t, a, v, t->a[i]) * e_tv_id(t, a, v, t->b[i]);
}
static int e_root(const etree* t) { return t->K ? t->ni + t->K - 1 : (t->ni ? 0 : -1); }
static unsigned e_root_sig(const etree* t) { return t->K ? t->sig[t->K - 1] : (t->ni ? t->isig[0] : 0u); }
static double e_tree_top(const etree* t, const double* a, const etv* v) {
  int r = e_root(t);
  return r < 0 ? 1.0 : e_tv_id(t, a, v, r);
}
static void e_tree_update(const etree* t, const double* a, etv* v, int c) {
  for (int i = 0; i < t->K; ++i)
    if ((t->sig[i] >> c) & 1u) v->N[i] = e_tv_id(t, a, v, t->a[i]) * e_tv_id(t, a, v, t->b[i]);
}

/* D = top_x - top_y of segment 0's tree; a root node's product fuses with the
 * subtraction into one fma (the kernel's __builtin_fma, one rounding) */
static double e_seg_D(const etree* t, const double* x, const etv* vx, const double* y, const etv* vy) {
  if (t->K == 0) return e_tree_top(t, x, vx) - e_tree_top(t, y, vy);
  int i = t->K - 1;
  return fma(e_tv_id(t, x, vx, t->a[i]), e_tv_id(t, x, vx, t->b[i]), -vy->N[i]);
}

/* the outer tree (rows outside segment 0) and segment 0's tree */
static void e_seg_trees(const eplan* P, etree* outer, etree* inner) {
  unsigned rsig[ORC_MAXN] = {0};
  for (int k = 1; k < P->m; ++k) {
    int c = k <= P->segb ? k - 1 : P->segb;
    for (int j = 0; j < P->n; ++j)
      if (P->col[2 * (P->L + k)][j] != 0.0) rsig[j] |= 1u << c;
  }
  e_tree_build(outer, rsig, P->len0, P->seg[P->nseg], P->n, P->segb, P->cc);
  e_tree_build(inner, rsig, 0, P->sub[P->nsub], P->len0, P->segb, P->cc);
}

/* Row copies of the segmented walk: only x0 (walk bits 0..cc clear) is
 * walked; the value of row r in cached state S is x0_r + cx_r(S & rs_r)
 * (x0_r when S & rs_r = 0) and its walk-bit-0 twin x0_r + cy_r(S & rs_r),
 * rs_r = the cached walk bits 1..cc touching row r (bit k-1 for walk bit k),
 * cx_r(S) = a_k(r) (+ cx_r(S minus its lowest bit)) for the lowest set bit of
 * S (walk bit k), cy_r(S) = a_0(r) (+ cx_r(S) when S != 0), a_k = the +
 * column of walk bit k (jit.cpp seg_cx / seg_cy). */
static double e_cx(const eplan* P, int r, unsigned S) {
  unsigned low = S & (0u - S), rest = S ^ low;
  double a = P->col[2 * (P->L + __builtin_ctz(low) + 1)][r];
  return rest ? e_cx(P, r, rest) + a : a;
}
static unsigned e_rs(const eplan* P, int r) {
  unsigned s = 0;
  for (int k = 1; k <= P->cc && k < P->m; ++k)
    if (P->col[2 * (P->L + k)][r] != 0.0) s |= 1u << (k - 1);
  return s;
}
/* every state's copies of row r from x0 */
static void e_derive(const eplan* P, const double* x0, double xs[][ORC_MAXN], double ys[][ORC_MAXN], int r) {
  unsigned rs = e_rs(P, r);
  for (int S = 0; S < (1 << P->cc); ++S) {
    unsigned s = (unsigned)S & rs;
    xs[S][r] = s ? x0[r] + e_cx(P, r, s) : x0[r];
    if (r < P->len0) ys[S][r] = x0[r] + (s ? P->col[2 * P->L][r] + e_cx(P, r, s) : P->col[2 * P->L][r]);
  }
}

/* one pair step flipping walk bit k >= 1: its rows of x0 (and their copies in
 * every cached state), then in every state the outer tree and segment 0's
 * trees over x and y with D = top_x - top_y (e_seg_D) */
static void e_seg_step(const eplan* P, const etree* outer, const etree* inner, double* x0, double xs[][ORC_MAXN],
                       double ys[][ORC_MAXN], etv* vo, etv* vx, etv* vy, double* D, int k, int neg) {
  const double* c = P->col[2 * (P->L + k) + neg];
  int any = 0;
  int cl = k <= P->segb ? k - 1 : P->segb;
  if (cl < P->cc) return; /* cached walk bit: every state already held */
  for (int j = 0; j < P->n; ++j)
    if (k <= P->segb ? c[j] != 0.0 : P->dyn[j]) {
      x0[j] += c[j];
      e_derive(P, x0, xs, ys, j);
      any = 1;
    }
  if (!any) return;
  for (int S = 0; S < (1 << P->cc); ++S) {
    e_tree_update(outer, xs[S], &vo[S], cl);
    if ((e_root_sig(inner) >> cl) & 1u) {
      e_tree_update(inner, xs[S], &vx[S], cl);
      e_tree_update(inner, ys[S], &vy[S], cl);
      D[S] = e_seg_D(inner, xs[S], &vx[S], ys[S], &vy[S]);
    }
  }
}

static double pair64(double* v) {
  for (int w = 64; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) v[i] = v[2 * i] + v[2 * i + 1];
  return v[0];
}

/* walk_skip.hip / superman_amd/csrc/kernels.hpp kSkipSegBits */
#define SKIP_SEG_BITS 4
#define SKIP_SEG_MASK ((1u << SKIP_SEG_BITS) - 1u)

static unsigned next_toggle(unsigned t, unsigned k) {
  unsigned c = ((t >> (k + 1)) << (k + 1)) + (1u << k);
  if (c <= t) c += 2u << k;
  return c;
}

static double e_chunk(const eplan* P, unsigned long long ga, unsigned long long* visited) {
  int n = P->n, L = P->L, m = P->m, NB = (n + 7) / 8;
  unsigned T = 1u << m;
  double lv[64];
  if (P->kind == 1) {
    /* walk_sparse.hip's chunk end (round 5): a lane-uniform row that no walk
     * column touches is constant over the chunk; exactly zero at its first
     * state, every term is zero and the chunk's part is +0 */
    double x[ORC_MAXN];
    e_start(P, ga, 0, x);
    for (int r = 0; r < n; ++r)
      if (((P->umask >> r) & 1ULL) && P->rowmask[r] == 0 && x[r] == 0.0) {
        if (visited) *visited += (unsigned long long)T << L;
        return 0.0;
      }
  }
  if (P->kind != 2) {
    for (unsigned l = 0; l < 64; ++l) {
      if (l >= (1u << L)) {
        lv[l] = 0.0;
        continue;
      }
      double x[ORC_MAXN], U[ORC_MAXN / 8 + 2], acc;
      e_start(P, ga, l, x);
      if (P->kind == 3) {
        /* cached walk bits 1..cc: one full state per assignment S of them,
         * its rows derived from x0 (e_derive) */
        static __thread etv vo[16], vx[16], vy[16]; /* cc <= 4 */
        static __thread etree outer, inner;
        static __thread double xs[16][ORC_MAXN], ys[16][ORC_MAXN];
        double D[16];
        int NS = 1 << P->cc;
        e_seg_trees(P, &outer, &inner);
        for (int r = 0; r < n; ++r) e_derive(P, x, xs, ys, r);
        for (int S = 0; S < NS; ++S) {
          e_tree_init(&outer, xs[S], &vo[S]);
          e_tree_init(&inner, xs[S], &vx[S]);
          e_tree_init(&inner, ys[S], &vy[S]);
          D[S] = e_seg_D(&inner, xs[S], &vx[S], ys[S], &vy[S]);
        }
        acc = D[0] * e_tree_top(&outer, xs[0], &vo[0]);
        double tot = 0.0; /* two-level lane sum: acc folds into tot after pair j = 2^segb (q + 1) */
        /* pair j = Gray steps 2j, 2j+1: contributes (-1)^j D U1, in the
         * state of its Gray bits 1..cc */
        for (unsigned j = 1; j < T / 2; ++j) {
          unsigned pb = __builtin_ctz(j), neg = (j >> (pb + 1)) & 1u;
          int S = 0;
          e_seg_step(P, &outer, &inner, x, xs, ys, vo, vx, vy, D, (int)pb + 1, (int)neg);
          for (int i = 0; i < P->cc; ++i) S |= (int)(((j >> i) ^ (j >> (i + 1))) & 1u) << i;
          acc = fma((j & 1u) ? -D[S] : D[S], e_tree_top(&outer, xs[S], &vo[S]), acc);
          if ((j & ((1u << P->segb) - 1u)) == 0u) tot += acc, acc = 0.0;
        }
        acc = tot + acc;
      } else if (P->kind == 0) {
        acc = e_prod4(x, n);
        for (unsigned t = 1; t < T; ++t) {
          unsigned k = __builtin_ctz(t), neg = (t >> (k + 1)) & 1u;
          for (int j = 0; j < n; ++j) x[j] += P->col[2 * (L + k) + neg][j];
          double pr = e_prod4(x, n);
          acc = (t & 1u) ? acc - pr : acc + pr;
        }
      } else {
        e_suffix(x, n, U);
        acc = U[0];
        for (unsigned t = 1; t < T; ++t) {
          unsigned k = __builtin_ctz(t), neg = (t >> (k + 1)) & 1u;
          e_sparse_step(x, U, n, P->col[2 * (L + k) + neg], P->nblk[L + k]);
          acc = (t & 1u) ? acc - U[0] : acc + U[0];
        }
      }
      if ((((unsigned)ga) ^ (unsigned)__builtin_popcount(l)) & 1u) acc = -acc;
      lv[l] = acc;
    }
    if (visited) *visited += (unsigned long long)T << L;
    return pair64(lv);
  }
  /* skipper: 64 lanes in lock-step with wave-uniform jumps at the starts of
   * aligned segments of 2^SKIP_SEG_BITS Gray steps (walk_skip.hip, round 5):
   * at a segment start t with every lane's term zero, the lane-uniform rows
   * that are exactly zero and that no walk bit below SKIP_SEG_BITS touches
   * stay zero until one of their walk columns toggles; the wave moves to the
   * last such toggle.  Every other segment is walked state by state. */
  static __thread double X[64][ORC_MAXN], UU[64][ORC_MAXN / 8 + 2];
  double acc[64];
  (void)NB;
  for (unsigned l = 0; l < 64; ++l) {
    e_start(P, ga, l, X[l]);
    e_suffix(X[l], n, UU[l]);
    acc[l] = UU[l][0]; /* state 0 */
  }
  unsigned long long vis = 1;
  unsigned u = 1;
  int check = 1;
  for (; T > 1;) { /* T = 1: state 0 is the chunk */
    int all_zero = 1;
    for (unsigned l = 0; l < 64 && all_zero; ++l)
      if (UU[l][0] != 0.0) all_zero = 0;
    if (check && all_zero) {
      unsigned t = u - 1, nx = t;
      unsigned long long zm = 0;
      for (int r = 0; r < n; ++r)
        if (X[0][r] == 0.0) zm |= 1ULL << r;
      zm &= P->umask;
      while (zm) {
        int r = __builtin_ctzll(zm);
        zm &= zm - 1;
        unsigned long long mm = P->rowmask[r];
        if (mm & SKIP_SEG_MASK) continue;
        unsigned tr = T;
        while (mm) {
          unsigned k = __builtin_ctzll(mm);
          mm &= mm - 1;
          unsigned c = next_toggle(t, k);
          if (c < tr) tr = c;
        }
        if (tr > nx) nx = tr;
      }
      if (nx >= T) break;
      if (nx > t) {
        unsigned gn = nx ^ (nx >> 1), diff = (t ^ (t >> 1)) ^ gn;
        do {
          unsigned k = __builtin_ctz(diff);
          diff &= diff - 1;
          unsigned neg = ((gn >> k) & 1u) ^ 1u;
          for (unsigned l = 0; l < 64; ++l) e_sparse_step(X[l], UU[l], n, P->col[2 * (L + k) + neg], P->nblk[L + k]);
        } while (diff);
        for (unsigned l = 0; l < 64; ++l) acc[l] += UU[l][0]; /* nx: a segment start, even */
        vis++;
        u = nx + 1;
        continue;
      }
    }
    for (unsigned l = 0; l < 64; ++l) {
      e_sparse_step(X[l], UU[l], n, P->col[2 * L + ((u >> 1) & 1u)], P->nblk[L]);
      acc[l] -= UU[l][0];
    }
    vis++;
    if (u + 1 >= T) break;
    {
      unsigned v = u + 1, k = __builtin_ctz(v), neg = (v >> (k + 1)) & 1u;
      for (unsigned l = 0; l < 64; ++l) {
        e_sparse_step(X[l], UU[l], n, P->col[2 * (L + k) + neg], P->nblk[L + k]);
        acc[l] += UU[l][0];
      }
      vis++;
      check = (v & SKIP_SEG_MASK) == 0;
    }
    u += 2;
  }
  if (visited) *visited += vis << L;
  for (unsigned l = 0; l < 64; ++l) {
    double v = acc[l];
    if ((((unsigned)ga) ^ (unsigned)__builtin_popcount(l)) & 1u) v = -v;
    lv[l] = (l < (1u << L)) ? v : 0.0;
  }
  return pair64(lv);
}

/* Engine-mirror partial over wave-chunks [c0, c1) with layout (L, m).
 * kind: 0 dense, 1 SpaRyser (prefix blocks), 2 SkipPer, 3 segmented walk
 * (jit.cpp's generated kernel).  colmap: engine bit e
 * -> matrix column (n-1 entries; NULL = identity).  cc (kind 3): walk bits
 * 1..cc held in every state and segb specialised pair bits (the engine
 * plan's choices, sup_plan_info; segb 0 = default). */
double orc_engine_range(const double* a, int n, int kind, const int* colmap, int cc, int segb, int L, int m,
                        unsigned long long c0, unsigned long long c1, int threads, unsigned long long* visited) {
  eplan* P = (eplan*)malloc(sizeof(eplan));
  engine_plan(a, n, kind, colmap, L, m, cc, segb, P);
  unsigned long long count = c1 > c0 ? c1 - c0 : 0;
  if (count == 0) {
    free(P);
    return 0.0;
  }
  double* part = (double*)malloc(sizeof(double) * count);
  unsigned long long tv = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : tv)
  for (long long i = 0; i < (long long)count; ++i) {
    unsigned long long v = 0;
    part[i] = e_chunk(P, c0 + i, &v);
    tv += v;
  }
  while (count > 1) {
    unsigned long long groups = (count + 63) / 64;
    for (unsigned long long g = 0; g < groups; ++g) {
      double v[64];
      for (int l = 0; l < 64; ++l) {
        unsigned long long i = g * 64 + l;
        v[l] = i < count ? part[i] : 0.0;
      }
      part[g] = pair64(v);
    }
    count = groups;
  }
  double r = part[0];
  free(part);
  free(P);
  if (visited) *visited = tv;
  return r;
}

/* Full permanent with the engine's default layout and the given column map. */
double orc_engine_perman(const double* a, int n, int kind, const int* colmap, int cc, int segb, int threads) {
  int L, m, h;
  orc_engine_layout(n, &L, &m, &h);
  double s = orc_engine_range(a, n, kind, colmap, cc, segb, L, m, 0, 1ULL << h, threads, 0);
  return (4 * (n & 1) - 2) * s;
}

/* ======================================================================
 * Exact permanent, independent of the engine's exact path (test checker for
 * sup_perman_exact): plain Ryser (not Nijenhuis-Wilf),
 *   perm = (-1)^n sum_{S subset of columns} (-1)^|S| prod_i sum_{j in S} a_ij,
 * over all 2^n column subsets in Gray order, integer row sums in int64 and
 * the products modulo p with 128-bit multiplies.  The caller (oracle/
 * __init__.py exact_perman_crt) picks its own primes and joins them by CRT.
 * ====================================================================== */
static uint64_t e_mulmod(uint64_t a, uint64_t b, uint64_t p) { return (uint64_t)((unsigned __int128)a * b % p); }

unsigned long long orc_exact_mod(const long long* a, int n, unsigned long long p, int threads) {
  if (n <= 0) return 1 % p;
  int hb = n > 12 ? 8 : 0; /* 2^hb blocks of the subset space, one Gray walk each */
  unsigned long long nblk = 1ULL << hb, per = 1ULL << (n - hb), total = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : total)
  for (long long b = 0; b < (long long)nblk; ++b) {
    long long s[ORC_MAXN];
    unsigned long long base = (unsigned long long)b * per, acc = 0;
    unsigned long long g0 = base ^ (base >> 1);
    for (int i = 0; i < n; ++i) {
      s[i] = 0;
      for (int j = 0; j < n; ++j)
        if ((g0 >> j) & 1ULL) s[i] += a[i * n + j];
    }
    for (unsigned long long t = 0; t < per; ++t) {
      unsigned long long idx = base + t, g = idx ^ (idx >> 1);
      if (t > 0) {
        unsigned long long gp = (idx - 1) ^ ((idx - 1) >> 1);
        int k = __builtin_ctzll(g ^ gp);
        long long sg = ((g >> k) & 1ULL) ? 1 : -1;
        for (int i = 0; i < n; ++i) s[i] += sg * a[i * n + k];
      }
      unsigned long long pr = 1 % p;
      for (int i = 0; i < n && pr; ++i) {
        long long v = s[i] % (long long)p;
        pr = e_mulmod(pr, (unsigned long long)(v < 0 ? v + (long long)p : v), p);
      }
      int odd = __builtin_popcountll(g) & 1;
      acc = (acc + (odd ? (p - pr) % p : pr)) % p;
    }
    total = (total + acc) % p;
  }
  /* the reduction sums < nblk * p, fine below 2^63 for p < 2^55 */
  total %= p;
  return (n & 1) ? (p - total) % p : total;
}
