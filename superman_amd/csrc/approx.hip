// approx.hip — gfx950 kernels of the randomized permanent estimators
// (reference gpu_approximation_dense.cu:155-371,
// gpu_approximation_sparse.cu:198-453).
//
// One sample per lane, one 64-sample block per wave at a time, blocks taken
// from an atomic queue.  The per-sample code (approx_core.hpp) is integer
// bitset work — popcounts over the row patterns, a Philox draw per step — plus,
// for the scaling estimator, fp64 sums over fp32 factors kept in an HBM
// scratch laid out [index][lane] so a wave's accesses coalesce.  A block's 64
// estimates leave as three pairwise sums (value, square, zero count), written
// by block index: the result depends only on (seed, sample count), never on
// the grid, the device count or which wave took a block.
#include "approx.hpp"
#include "approx_core.hpp"
#include "walk_common.hpp"

namespace sup {

template <int W, int M>
__global__ __launch_bounds__(kBlock) void approx_blocks(ApproxParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gl = blockIdx.x * kBlock + threadIdx.x;
  float* dr = p.scratch ? p.scratch + gl : nullptr;
  float* dc = p.scratch ? p.scratch + (size_t)p.n * p.lanes_total + gl : nullptr;
  for (uint32_t b = next_chunk(p.counter); b < p.nblocks; b = next_chunk(p.counter)) {
    const uint64_t sample = (p.block0 + b) * 64u + lane;
    bool zero = false;
    double e;
    if constexpr (M == 0) {
      e = rasmussen_sample<W>(p.rowpat, p.n, p.seed, sample, zero);
    } else {
      e = scaling_sample<W>(p.rowpat, p.colpat, p.n, p.intervals, p.times, p.seed, sample, dr, dc, p.lanes_total,
                            zero);
    }
    const double s = wave_sum(e);
    const double q = wave_sum(e * e);
    const double z = wave_sum(zero ? 1.0 : 0.0);
    if (lane == 0) {
      p.part[b] = s;
      p.part[p.nblocks + b] = q;
      p.part[2 * p.nblocks + b] = z;
    }
  }
}

// ---- cooperative form: one wave per sample (large n) ----------------------
// The per-lane form keeps a sample per lane and, for the scaling estimator, its
// n + n fp32 factors in an HBM scratch: at n = 648 (the reference's default
// 36 x 36 grid) every Sinkhorn sum is a chain of dependent scratch loads.
// Here the 64 lanes share one sample: its factors live in LDS (2n floats per
// wave), the row pick is a wave min over the lanes' rows, and a Sinkhorn pass
// gives each lane the columns (rows) j = lane (mod 64), each summed in
// ascending order exactly as the per-lane code sums it — so every sample, and
// hence every block sum, is bit-identical to the per-lane kernel and to the
// host threads (approx_core.hpp).  Lane s keeps sample s of the block; the
// block leaves through the same wave_sum.

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// pick_row over the lanes: the remaining row with the fewest remaining
// nonzeros, the first (smallest index) on ties.
template <int W>
__device__ __forceinline__ int coop_pick_row(const uint64_t* rowpat, int n, const uint64_t (&rows)[W],
                                             const uint64_t (&cols)[W], uint32_t lane, int& row,
                                             uint64_t (&live)[W]) {
  uint32_t key = 0xFFFFFFFFu;
#pragma unroll
  for (int rw = 0; rw < W; ++rw) {  // rows r = 64 rw + lane (static word index: no scratch)
    const int r = 64 * rw + (int)lane;
    if (r >= n || !((rows[rw] >> lane) & 1ull)) continue;
    const uint64_t* pr = rowpat + (size_t)r * W;
    int cnt = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) cnt += popc64(pr[w] & cols[w]);
    const uint32_t k = ((uint32_t)cnt << 12) | (uint32_t)r;
    key = k < key ? k : key;
  }
#pragma unroll
  for (int off = 1; off <= 32; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)key, off, 64);
    key = o < key ? o : key;
  }
  row = (int)(key & 4095u);
  const uint64_t* pr = rowpat + (size_t)row * W;
#pragma unroll
  for (int w = 0; w < W; ++w) live[w] = pr[w] & cols[w];
  return (int)(key >> 12);
}

template <int W>
__device__ double coop_rasmussen(const uint64_t* rowpat, int n, uint64_t seed, uint64_t sample, uint32_t lane,
                                 bool& zero) {
  uint64_t rows[W], cols[W], live[W];
  all_bits<W>(rows, n);
  all_bits<W>(cols, n);
  double est = 1.0;
  zero = false;
  for (int it = 0; it < n; ++it) {
    int row;
    const int best = coop_pick_row<W>(rowpat, n, rows, cols, lane, row, live);
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

template <int W>
__device__ double coop_scaling(const uint64_t* rowpat, const uint64_t* colpat, int n, int intervals, int times,
                               uint64_t seed, uint64_t sample, float* dr, float* dc, uint32_t lane, bool& zero) {
  uint64_t rows[W], cols[W], live[W];
  all_bits<W>(rows, n);
  all_bits<W>(cols, n);
  for (int i = (int)lane; i < n; i += 64) dr[i] = 1.0f, dc[i] = 1.0f;
  wave_lds_sync();
  double est = 1.0;
  zero = false;
  for (int it = 0; it < n; ++it) {
    int row;
    coop_pick_row<W>(rowpat, n, rows, cols, lane, row, live);
    if (intervals > 0 && it % intervals == 0) {
      for (int k = 0; k < times; ++k) {
        bool z = false;
#pragma unroll
        for (int jw = 0; jw < W; ++jw) {  // columns j = 64 jw + lane
          const int j = 64 * jw + (int)lane;
          if (j >= n || !((cols[jw] >> lane) & 1ull)) continue;
          const uint64_t* cp = colpat + (size_t)j * W;
          double s = 0.0;
          for (int w = 0; w < W; ++w) {
            uint64_t m = cp[w] & rows[w];
            while (m) {
              const int i = 64 * w + __builtin_ctzll(m);
              m &= m - 1;
              s += (double)dr[i];
            }
          }
          if (s == 0.0) z = true;
          else dc[j] = (float)(1.0 / s);
        }
        if (__any(z)) {
          zero = true;
          return 0.0;
        }
        wave_lds_sync();
#pragma unroll
        for (int iw = 0; iw < W; ++iw) {  // rows i = 64 iw + lane
          const int i = 64 * iw + (int)lane;
          if (i >= n || !((rows[iw] >> lane) & 1ull)) continue;
          const uint64_t* rp = rowpat + (size_t)i * W;
          double s = 0.0;
          for (int w = 0; w < W; ++w) {
            uint64_t m = rp[w] & cols[w];
            while (m) {
              const int j = 64 * w + __builtin_ctzll(m);
              m &= m - 1;
              s += (double)dc[j];
            }
          }
          if (s == 0.0) z = true;
          else dr[i] = (float)(1.0 / s);
        }
        if (__any(z)) {
          zero = true;
          return 0.0;
        }
        wave_lds_sync();
      }
    }
    // the draw: every lane the same sequence (uniform LDS reads)
    const double rr = (double)dr[row];
    double S = 0.0;
    for (int w = 0; w < W; ++w) {
      uint64_t m = live[w];
      while (m) {
        const int j = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        S += rr * (double)dc[j];
      }
    }
    if (S == 0.0) {
      zero = true;
      return 0.0;
    }
    const Philox4 d = draw(seed, sample, (uint32_t)it);
    const uint64_t bits = ((uint64_t)d.v[0] << 21) ^ (uint64_t)(d.v[1] >> 11);
    const double target = (double)(bits + 1ull) * (1.0 / 9007199254740992.0) * S;
    double acc = 0.0, pj = 0.0;
    int col = 0;
    bool done = false;
    for (int w = 0; w < W && !done; ++w) {
      uint64_t m = live[w];
      while (m) {
        const int j = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        const double sv = rr * (double)dc[j];
        acc += sv;
        col = j;
        pj = sv / S;
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

// Dynamic LDS: 4 waves x 2n floats (scaling).
template <int W, int M>
__global__ __launch_bounds__(kBlock) void approx_coop(ApproxParams p) {
  extern __shared__ float lds[];
  const uint32_t lane = threadIdx.x & 63u;
  float* dr = lds + (size_t)(threadIdx.x >> 6) * 2u * (uint32_t)p.n;
  float* dc = dr + p.n;
  for (uint32_t b = next_chunk(p.counter); b < p.nblocks; b = next_chunk(p.counter)) {
    double mine = 0.0;
    bool mine_zero = false;
    for (uint32_t s = 0; s < 64; ++s) {
      const uint64_t sample = (p.block0 + b) * 64u + s;
      bool zero = false;
      double e;
      if constexpr (M == 0) e = coop_rasmussen<W>(p.rowpat, p.n, p.seed, sample, lane, zero);
      else e = coop_scaling<W>(p.rowpat, p.colpat, p.n, p.intervals, p.times, p.seed, sample, dr, dc, lane, zero);
      if (lane == s) mine = e, mine_zero = zero;
      wave_lds_sync();  // the next sample re-initialises the factors
    }
    const double sm = wave_sum(mine);
    const double q = wave_sum(mine * mine);
    const double z = wave_sum(mine_zero ? 1.0 : 0.0);
    if (lane == 0) {
      p.part[b] = sm;
      p.part[p.nblocks + b] = q;
      p.part[2 * p.nblocks + b] = z;
    }
  }
}

template <int W>
static hipError_t launch_coop_w(const ApproxParams& p, int grid, hipStream_t s) {
  const size_t lds = (p.method == 1 ? 2u * kWavesPerBlock * (size_t)p.n : 1u) * sizeof(float);
  if (p.method == 0) hipLaunchKernelGGL((approx_coop<W, 0>), dim3(grid), dim3(kBlock), lds, s, p);
  else hipLaunchKernelGGL((approx_coop<W, 1>), dim3(grid), dim3(kBlock), lds, s, p);
  return hipGetLastError();
}

template <int W>
static hipError_t occ_coop_w(int method, int n, int* b) {
  const size_t lds = (method == 1 ? 2u * kWavesPerBlock * (size_t)n : 1u) * sizeof(float);
  return method == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_coop<W, 0>, kBlock, lds)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_coop<W, 1>, kBlock, lds);
}

hipError_t launch_approx_coop(int words, const ApproxParams& p, int grid, hipStream_t s) {
  switch (words) {
    case 1: return launch_coop_w<1>(p, grid, s);
    case 2: return launch_coop_w<2>(p, grid, s);
    case 4: return launch_coop_w<4>(p, grid, s);
    case 8: return launch_coop_w<8>(p, grid, s);
    case 16: return launch_coop_w<16>(p, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t approx_coop_occupancy(int words, int method, int n, int* blocks_per_cu) {
  switch (words) {
    case 1: return occ_coop_w<1>(method, n, blocks_per_cu);
    case 2: return occ_coop_w<2>(method, n, blocks_per_cu);
    case 4: return occ_coop_w<4>(method, n, blocks_per_cu);
    case 8: return occ_coop_w<8>(method, n, blocks_per_cu);
    case 16: return occ_coop_w<16>(method, n, blocks_per_cu);
  }
  return hipErrorInvalidValue;
}

template <int W>
static hipError_t launch_w(const ApproxParams& p, int grid, hipStream_t s) {
  if (p.method == 0) hipLaunchKernelGGL((approx_blocks<W, 0>), dim3(grid), dim3(kBlock), 0, s, p);
  else hipLaunchKernelGGL((approx_blocks<W, 1>), dim3(grid), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

template <int W>
static hipError_t occ_w(int method, int* b) {
  return method == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_blocks<W, 0>, kBlock, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(b, approx_blocks<W, 1>, kBlock, 0);
}

hipError_t launch_approx(int words, const ApproxParams& p, int grid, hipStream_t s) {
  switch (words) {
    case 1: return launch_w<1>(p, grid, s);
    case 2: return launch_w<2>(p, grid, s);
    case 4: return launch_w<4>(p, grid, s);
    case 8: return launch_w<8>(p, grid, s);
    case 16: return launch_w<16>(p, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t approx_occupancy(int words, int method, int* blocks_per_cu) {
  switch (words) {
    case 1: return occ_w<1>(method, blocks_per_cu);
    case 2: return occ_w<2>(method, blocks_per_cu);
    case 4: return occ_w<4>(method, blocks_per_cu);
    case 8: return occ_w<8>(method, blocks_per_cu);
    case 16: return occ_w<16>(method, blocks_per_cu);
  }
  return hipErrorInvalidValue;
}

}  // namespace sup
