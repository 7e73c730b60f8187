// approx_core.hpp — per-sample permanent estimators, shared verbatim by the
// gfx950 kernel (approx.hip) and the host threads (approx_host.cpp), so a
// sample computes the same bits on either side.
//
// Replaces the reference's randomized path:
//   * Rasmussen: gpu_approximation_dense.cu:155-229 kernel_rasmussen,
//     gpu_approximation_sparse.cu:198-290, algo.h:172-366 (CPU);
//   * scaling-based importance sampling: gpu_approximation_dense.cu:231-371
//     kernel_approximation, gpu_approximation_sparse.cu:292-453,
//     algo.h:366-560 (CPU).
// Both estimate the permanent of the 0/1 nonzero pattern (the reference's
// estimators multiply by row degrees / divide by sampling probabilities and
// never by the entry values).  Each step takes the remaining row with the
// fewest remaining nonzeros (first such row), as the reference kernels do.
//
// Differences from the reference, on purpose:
//   * randomness: Philox4x32-10 keyed by the seed with counter (sample,
//     step), instead of curand XORWOW seeded with rand()*tid — a sample's
//     estimate depends only on (seed, sample index), so results are
//     reproducible and independent of the grid, device count and CPU/GPU;
//   * the column pick in Rasmussen uses a multiply-shift of a 32-bit draw
//     (the reference scales a float curand_uniform and clamps);
//   * `is_break` is initialised (kernel_approximation leaves it undefined);
//   * patterns are bitsets of W 64-bit words, so n is up to 64·W (the
//     reference: 64 dense, 672 sparse).
#pragma once
#include <stdint.h>

#ifdef __HIP__
#define SUP_HD __host__ __device__ __forceinline__
#else
#define SUP_HD inline
#endif

namespace sup {

struct Philox4 {
  uint32_t v[4];
};

// Philox4x32-10 (Salmon et al., SC'11), counter (c0..c3), key (k0, k1).
SUP_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return Philox4{{c0, c1, c2, c3}};
}

SUP_HD Philox4 draw(uint64_t seed, uint64_t sample, uint32_t step) {
  return philox4x32_10((uint32_t)sample, (uint32_t)(sample >> 32), step, 0x5AB1Eu, (uint32_t)seed,
                       (uint32_t)(seed >> 32));
}

SUP_HD int popc64(uint64_t x) { return __builtin_popcountll(x); }

// Position of the k-th (0-based) set bit of x (k < popcount(x)).
SUP_HD int kth_bit(uint64_t x, int k) {
  int pos = 0;
  for (int h = 32; h >= 1; h >>= 1) {
    const uint64_t low = x & ((1ull << h) - 1ull);
    const int c = popc64(low);
    if (k >= c) {
      k -= c;
      x >>= h;
      pos += h;
    } else {
      x = low;
    }
  }
  return pos;
}

// Remaining row with the fewest remaining nonzeros (first one on ties):
// returns its count (n+1 if no row remains) and sets row / its live columns.
template <int W>
SUP_HD int pick_row(const uint64_t* rowpat, int n, const uint64_t (&rows)[W], const uint64_t (&cols)[W], int& row,
                    uint64_t (&live)[W]) {
  int best = n + 1;
  row = 0;
  for (int w = 0; w < W; ++w) live[w] = 0;
  for (int rw = 0; rw < W; ++rw) {
    const int hi = (n - 64 * rw) < 64 ? n - 64 * rw : 64;
    for (int b = 0; b < hi; ++b) {
      const int r = 64 * rw + b;
      const uint64_t* pr = rowpat + (size_t)r * W;
      int cnt = 0;
      uint64_t m[W];
      for (int w = 0; w < W; ++w) {
        m[w] = pr[w] & cols[w];
        cnt += popc64(m[w]);
      }
      if (((rows[rw] >> b) & 1ull) && cnt < best) {
        best = cnt;
        row = r;
        for (int w = 0; w < W; ++w) live[w] = m[w];
      }
    }
  }
  return best;
}

template <int W>
SUP_HD void clear_bit(uint64_t (&m)[W], int i) {
  for (int w = 0; w < W; ++w)
    if (w == (i >> 6)) m[w] &= ~(1ull << (i & 63));
}

template <int W>
SUP_HD void all_bits(uint64_t (&m)[W], int n) {
  for (int w = 0; w < W; ++w) {
    const int k = n - 64 * w;
    m[w] = k >= 64 ? ~0ull : (k <= 0 ? 0ull : ((1ull << k) - 1ull));
  }
}

// One Rasmussen sample (kernel_rasmussen, gpu_approximation_dense.cu:155-229):
// X = prod over steps of the chosen row's remaining degree, 0 if a row runs out.
template <int W>
SUP_HD double rasmussen_sample(const uint64_t* rowpat, int n, uint64_t seed, uint64_t sample, bool& zero) {
  uint64_t rows[W], cols[W], live[W];
  all_bits<W>(rows, n);
  all_bits<W>(cols, n);
  double est = 1.0;
  zero = false;
  for (int it = 0; it < n; ++it) {
    int row;
    const int best = pick_row<W>(rowpat, n, rows, cols, row, live);
    if (best == 0) {
      zero = true;
      return 0.0;
    }
    est *= (double)best;
    const uint32_t u = draw(seed, sample, (uint32_t)it).v[0];
    int k = (int)(((uint64_t)u * (uint32_t)best) >> 32);
    int col = 0;
    bool found = false;
    for (int w = 0; w < W; ++w) {
      const int c = popc64(live[w]);
      if (!found && k < c) {
        col = 64 * w + kth_bit(live[w], k);
        found = true;
      }
      if (!found) k -= c;
    }
    clear_bit<W>(cols, col);
    clear_bit<W>(rows, row);
  }
  return est;
}

// One scaling-guided sample (kernel_approximation, gpu_approximation_dense.cu:
// 231-371): every `intervals` steps, `times` Sinkhorn passes over the remaining
// submatrix (column sums of d_r, then row sums of d_c; fp32 factors, fp64 sums);
// the column is drawn with probability d_r[row]·d_c[j] / S over the row's
// remaining nonzeros and X /= p.  dr/dc: n floats each at stride `st`.
template <int W>
SUP_HD double scaling_sample(const uint64_t* rowpat, const uint64_t* colpat, int n, int intervals, int times,
                             uint64_t seed, uint64_t sample, float* dr, float* dc, uint32_t st, bool& zero) {
  uint64_t rows[W], cols[W], live[W];
  all_bits<W>(rows, n);
  all_bits<W>(cols, n);
  for (int i = 0; i < n; ++i) {
    dr[(size_t)i * st] = 1.0f;
    dc[(size_t)i * st] = 1.0f;
  }
  double est = 1.0;
  zero = false;
  for (int it = 0; it < n; ++it) {
    int row;
    pick_row<W>(rowpat, n, rows, cols, row, live);
    if (intervals > 0 && it % intervals == 0) {
      for (int k = 0; k < times; ++k) {
        for (int jw = 0; jw < W; ++jw) {  // (word, bit) loops: static register indices
          uint64_t jm = cols[jw];
          while (jm) {
          const int j = 64 * jw + __builtin_ctzll(jm);
          jm &= jm - 1;
          const uint64_t* cp = colpat + (size_t)j * W;
          double s = 0.0;
          for (int w = 0; w < W; ++w) {
            uint64_t m = cp[w] & rows[w];
            while (m) {
              const int i = 64 * w + __builtin_ctzll(m);
              m &= m - 1;
              s += (double)dr[(size_t)i * st];
            }
          }
          if (s == 0.0) {
            zero = true;
            return 0.0;
          }
          dc[(size_t)j * st] = (float)(1.0 / s);
          }
        }
        for (int iw = 0; iw < W; ++iw) {
          uint64_t im = rows[iw];
          while (im) {
          const int i = 64 * iw + __builtin_ctzll(im);
          im &= im - 1;
          const uint64_t* rp = rowpat + (size_t)i * W;
          double s = 0.0;
          for (int w = 0; w < W; ++w) {
            uint64_t m = rp[w] & cols[w];
            while (m) {
              const int j = 64 * w + __builtin_ctzll(m);
              m &= m - 1;
              s += (double)dc[(size_t)j * st];
            }
          }
          if (s == 0.0) {
            zero = true;
            return 0.0;
          }
          dr[(size_t)i * st] = (float)(1.0 / s);
          }
        }
      }
    }
    const double rr = (double)dr[(size_t)row * st];
    double S = 0.0;
    for (int w = 0; w < W; ++w) {
      uint64_t m = live[w];
      while (m) {
        const int j = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        S += rr * (double)dc[(size_t)j * st];
      }
    }
    if (S == 0.0) {
      zero = true;
      return 0.0;
    }
    const Philox4 d = draw(seed, sample, (uint32_t)it);
    const uint64_t bits = ((uint64_t)d.v[0] << 21) ^ (uint64_t)(d.v[1] >> 11);  // 53 random bits
    const double target = (double)(bits + 1ull) * (1.0 / 9007199254740992.0) * S;  // (0, 1] * S
    double acc = 0.0, pj = 0.0;
    int col = 0;
    bool done = false;
    for (int w = 0; w < W && !done; ++w) {
      uint64_t m = live[w];
      while (m) {
        const int j = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        const double s = rr * (double)dc[(size_t)j * st];
        acc += s;
        col = j;  // if rounding leaves target > acc, the last column is taken
        pj = s / S;
        if (target <= acc) {
          done = true;
          break;
        }
      }
    }
    est /= pj;
    clear_bit<W>(cols, col);
    clear_bit<W>(rows, row);
  }
  return est;
}

}  // namespace sup
