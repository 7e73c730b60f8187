#include <stdio.h>
#include <stdlib.h>
/* SkipPer policy simulator (round 5, test infrastructure): how many states
 * the wave-uniform SkipPer walk visits on sampled wave-chunks when zero checks
 * and jumps happen only at the starts of aligned 2^s-step segments (s = 0 is
 * round 4's per-state policy).  It restates the walk with the oracle's own
 * engine-mirror helpers (oracle.c is included, not linked).
 *   build: gcc -O2 -I oracle -o /tmp/skip_sim tools/probes/skip_sim.c -lm -fopenmp
 *   input: plan.txt = "n L m", the column map, the n x n matrix (SkipOrder
 *          applied), e.g. from superman_amd.plan_info(a, "skip", jit=-1)
 *   run:   /tmp/skip_sim <sampled chunks>  (config 5: profiles/r5/skip_sim.log) */
#include "oracle.c"
int main(int argc, char** argv) {
  FILE* f = fopen("plan.txt", "r");
  int n, L, m; if (fscanf(f, "%d %d %d", &n, &L, &m) != 3) return 1;
  int colmap[64]; for (int e = 0; e < n - 1; ++e) if (fscanf(f, "%d", &colmap[e]) != 1) return 1;
  static double a[64 * 64]; for (int i = 0; i < n * n; ++i) if (fscanf(f, "%lf", &a[i]) != 1) return 1;
  fclose(f);
  eplan* P = (eplan*)malloc(sizeof(eplan));
  engine_plan(a, n, 2, colmap, L, m, 0, 0, P);
  int h = n - 1 - L - m; unsigned T = 1u << m;
  int samples = atoi(argv[1]);
  for (int s = 0; s <= 12; s += (s < 4 ? 1 : 2)) {
    unsigned lowmask = (1u << s) - 1u;
    static double X[64][ORC_MAXN], UU[64][ORC_MAXN / 8 + 2];
    unsigned long long vis = 0, scans = 0, jumps = 0, segs = 0;
    for (int sidx = 0; sidx < samples; ++sidx) {
      unsigned long long ga = ((unsigned long long)sidx * 2 + 1) * (1ull << h) / (2ull * samples);
      for (unsigned l = 0; l < 64; ++l) { e_start(P, ga, l, X[l]); e_suffix(X[l], n, UU[l]); }
      unsigned t = 0;
      while (t < T) {
        int all_zero = 1;
        for (unsigned l = 0; l < 64; ++l) if (UU[l][0] != 0.0) all_zero = 0;
        unsigned next = t + (1u << s);   /* walk the segment */
        if (all_zero) {
          scans++;
          unsigned long long zm = 0;
          for (int r = 0; r < n; ++r) if (X[0][r] == 0.0 && !(P->rowmask[r] & lowmask)) zm |= 1ULL << r;
          zm &= P->umask;
          if (zm) {
            unsigned target = t;
            while (zm) {
              int r = __builtin_ctzll(zm); zm &= zm - 1;
              unsigned long long mm = P->rowmask[r]; unsigned tr = T;
              while (mm) { unsigned k = __builtin_ctzll(mm); mm &= mm - 1; unsigned c = next_toggle(t, k); if (c < tr) tr = c; }
              if (tr > target) target = tr;
            }
            jumps++;
            next = target;
          } else { vis += 1u << s; segs++; }
        } else { vis += 1u << s; segs++; }
        if (next >= T) break;
        unsigned gn = next ^ (next >> 1), diff = (t ^ (t >> 1)) ^ gn;
        do {
          unsigned k = __builtin_ctz(diff); diff &= diff - 1;
          unsigned neg = ((gn >> k) & 1u) ^ 1u;
          for (unsigned l = 0; l < 64; ++l) e_sparse_step(X[l], UU[l], n, P->col[2 * (L + k) + neg], P->nblk[L + k]);
        } while (diff);
        t = next;
      }
    }
    double tot = (double)samples * T;
    printf("s %2d: visited %.4f  scans/state %.5f jumps/state %.5f segments walked/state %.5f\n", s, vis / tot,
           scans / tot, jumps / tot, segs / tot);
  }
  return 0;
}
