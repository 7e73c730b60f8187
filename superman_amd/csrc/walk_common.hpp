// walk_common.hpp — device-side building blocks of the gfx950 Ryser walk kernels.
//
// Work decomposition.  The reference walks the Gray index
// space i in [1, 2^(n-1)) with one contiguous range per GPU thread
// (gpu_exact_dense.cu:350-396).  Here the n-1 Gray bits are split into
//   engine bits [0, L)        -> the 64 lanes of a wave (lane l owns pattern l),
//   engine bits [L, L+m)      -> a Gray walk of 2^m steps that every lane of the
//                                wave performs in lock-step (flipped column is
//                                wave-uniform: k = ctz(t), computed on the SALU),
//   engine bits [L+m, n-1)    -> the wave-chunk index a; subset part = gray(a).
// A wave-chunk a therefore covers exactly the subsets {gray(i)} of the aligned
// reference index block [a*2^(L+m), (a+1)*2^(L+m)) — so chunk partial sums
// are comparable with the reference chunk helpers (gpu_exact_dense.cu:6-69).
//
// Because the flipped column is wave-uniform, the column is read with scalar
// loads (s_load_dwordx16 into SGPRs) and consumed as the SGPR operand of
// v_add_f64: no LDS traffic and no VALU address work on the hot loop.  X lives
// in VGPRs (n fp64 values per lane).
#pragma once
// Also compiled by hiprtc for the pattern-specialised walk (jit.cpp), where
// the HIP runtime header is implicit and <stdint.h> is not available.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "walk_params.hpp"

namespace sup {

template <int V>
struct Int {
  static constexpr int value = V;
};

// Constant address space pointer: uniform loads through it become s_load.
typedef const __attribute__((address_space(4))) double cdbl;
typedef const __attribute__((address_space(4))) int cint;

// Hide a uniform address from LLVM's loop-invariant code motion: otherwise the
// k = 0 columns (constant addresses) are hoisted out of the walk and pinned in
// SGPRs, which spills.  "+s" keeps the value wave-uniform and in SGPRs.  The
// base goes through the asm and the offset is added after it, so neither the
// load nor its address can leave the loop (an address formed before the asm
// was hoisted: one SGPR pair per constant, live for the whole kernel), and a
// constant offset folds into the s_load immediate.
__device__ __forceinline__ cdbl* opaque_c(const double* base, uint32_t byte_off) {
#ifdef SUP_OPAQUE_BEFORE_OFFSET  // the round-2 form (experiments: SUP_JIT_OPAQUE_R2=1)
  uint64_t a = (uint64_t)base + byte_off;
  asm volatile("" : "+s"(a));
  return (cdbl*)a;
#else
  uint64_t a = (uint64_t)base;
  asm volatile("" : "+s"(a));
  return (cdbl*)(a + byte_off);
#endif
}
__device__ __forceinline__ cint* opaque_i(const int* base, uint32_t byte_off) {
  uint64_t a = (uint64_t)base;
  asm volatile("" : "+s"(a));
  return (cint*)(a + byte_off);
}

// x[LO..HI) += col[LO..HI)   (col wave-uniform -> SGPR operands)
template <int N, int LO, int HI>
__device__ __forceinline__ void add_rows(double (&x)[N], cdbl* col) {
#pragma unroll
  for (int j = LO; j < HI; ++j) x[j] += col[j];
}

// Full-column update.  Columns longer than 32 doubles are consumed in two
// pieces with a scheduling fence between them so at most 64 SGPRs of column
// data are live (SGPR budget is 102 per wave).
template <int N>
__device__ __forceinline__ void add_col(double (&x)[N], cdbl* col) {
  if constexpr (N <= 32) {
    add_rows<N, 0, N>(x, col);
  } else {
    add_rows<N, 0, 32>(x, col);
    __builtin_amdgcn_sched_barrier(0);
    add_rows<N, 32, N>(x, col);
  }
}

// Canonical dense product (mirrored bit-for-bit by oracle/oracle.c
// orc_engine_prod): four strided partial products p_r = x_r * x_{r+4} * ...,
// combined as (p0*p1)*(p2*p3).  Missing partials are 1.0 (folded away).
template <int N>
__device__ __forceinline__ double prod4(const double (&x)[N]) {
  double p0 = x[0];
  double p1 = N > 1 ? x[1 < N ? 1 : 0] : 1.0;
  double p2 = N > 2 ? x[2 < N ? 2 : 0] : 1.0;
  double p3 = N > 3 ? x[3 < N ? 3 : 0] : 1.0;
#pragma unroll
  for (int j = 4; j < N; j += 4) {
    p0 *= x[j];
    if (j + 1 < N) p1 *= x[j + 1 < N ? j + 1 : 0];
    if (j + 2 < N) p2 *= x[j + 2 < N ? j + 2 : 0];
    if (j + 3 < N) p3 *= x[j + 3 < N ? j + 3 : 0];
  }
  return (p0 * p1) * (p2 * p3);
}

// Product of the rows of 8-row block b (rows [8b, min(8b+8, N))):
// ((x0*x1)*(x2*x3)) * ((x4*x5)*(x6*x7)), missing rows = 1.0.
template <int N, int B>
__device__ __forceinline__ double bprod8(const double (&x)[N]) {
  constexpr int r0 = 8 * B;
  auto v = [&](int i) -> double { return (r0 + i < N) ? x[(r0 + i < N) ? r0 + i : 0] : 1.0; };
  return ((v(0) * v(1)) * (v(2) * v(3))) * ((v(4) * v(5)) * (v(6) * v(7)));
}

// 64-lane pairwise sum.  Offsets ascend (xor 1, 2, ..., 32), so lane 0 ends
// with the pairwise tree ((v0+v1)+(v2+v3))+... ; every lane holds the same
// value (IEEE addition is commutative).  Mirrored by oracle/oracle.c
// orc_pairwise64.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 1; off <= 32; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// nblk of walk bit k (sparse kernels), unpacked on the SALU.
__device__ __forceinline__ int nb_of(const WalkParams& p, uint32_t k) {
  const uint64_t w = k < 16 ? p.nb_lo : p.nb_hi;
  return (int)((w >> ((k & 15u) * 4u)) & 15u);
}

// Column rows [LO, HI) (LO a multiple of 8) fetched with scalar loads into
// `c`, all issued before any use.  The empty asm pins every 8-double piece at
// this point, so the loads are not sunk into the (uniform) branches that
// consume them — one s_waitcnt per step instead of one per row block.
typedef double dbl8 __attribute__((ext_vector_type(8)));
template <int N, int LO, int HI>
__device__ __forceinline__ void fetch_rows(cdbl* col, double (&c)[N]) {
  typedef const __attribute__((address_space(4))) dbl8 cdbl8;
  constexpr int B0 = LO / 8, P = (HI - LO + 7) / 8;  // P <= 4 pieces of 8 doubles
  static_assert(P >= 1 && P <= 4, "fetch_rows handles 1..4 pieces");
  cdbl8* v = (cdbl8*)col;
  dbl8 t0 = v[B0], t1, t2, t3;
  if constexpr (P > 1) t1 = v[B0 + 1];
  if constexpr (P > 2) t2 = v[B0 + 2];
  if constexpr (P > 3) t3 = v[B0 + 3];
  // one pin for all pieces -> a single s_waitcnt
  if constexpr (P == 1) asm volatile("" : "+s"(t0));
  if constexpr (P == 2) asm volatile("" : "+s"(t0), "+s"(t1));
  if constexpr (P == 3) asm volatile("" : "+s"(t0), "+s"(t1), "+s"(t2));
  if constexpr (P == 4) asm volatile("" : "+s"(t0), "+s"(t1), "+s"(t2), "+s"(t3));
  auto put = [&](int piece, const dbl8& t) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 8 * (B0 + piece) + i;
      if (r < HI) c[(r < N) ? r : 0] = t[i];
    }
  };
  put(0, t0);
  if constexpr (P > 1) put(1, t1);
  if constexpr (P > 2) put(2, t2);
  if constexpr (P > 3) put(3, t3);
}

// ---- prefix-blocked rows (SpaRyser / SkipPer kernels) --------------------
// Rows are kept in 8-row blocks with suffix products U[b] = prod_{rows >= 8b}
// (U[NB] = 1).  Mirrored by oracle/oracle.c e_sparse_step / e_suffix.
template <int N>
struct Blocks {
  static constexpr int NB = (N + 7) / 8;
};

template <int N, int B>
__device__ __forceinline__ void blk_add(double (&x)[N], const double (&c)[N]) {
  constexpr int lo = 8 * B, hi = (8 * B + 8 < N) ? 8 * B + 8 : N;
#pragma unroll
  for (int j = lo; j < hi; ++j) x[j] += c[j];
}
template <int N, int B>
__device__ __forceinline__ void blk_prod(const double (&x)[N], double (&U)[Blocks<N>::NB + 1]) {
  U[B] = bprod8<N, B>(x) * U[B + 1];
}

template <int N>
__device__ __forceinline__ void suffix_all(const double (&x)[N], double (&U)[Blocks<N>::NB + 1]) {
  U[Blocks<N>::NB] = 1.0;
#pragma unroll
  for (int b = Blocks<N>::NB - 1; b >= 0; --b) {
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (8 * b + i < N) ? x[(8 * b + i < N) ? 8 * b + i : 0] : 1.0;
    U[b] = (((v[0] * v[1]) * (v[2] * v[3])) * ((v[4] * v[5]) * (v[6] * v[7]))) * U[b + 1];
  }
}

// One walk step: add column `col` to the leading nb row blocks and refresh
// their suffix products, top block first (U[b+1] is current when U[b] is
// formed).  A fall-through switch = one uniform jump per half, and the column
// rows are fetched up front (fetch_rows) so each half waits once.
template <int B, int LO, class F>
__device__ __forceinline__ void for_down(F&& f) {
  if constexpr (B >= LO) {
    f(Int<B>{});
    for_down<B - 1, LO>(f);
  }
}

// Nested form: `if (nb > B) { deeper blocks; block B }`, so a step touching
// nb blocks pays ~nb uniform branches (not NB), blocks still run top-down,
// and the control flow stays structured (x/U updated in place, no phi
// copies).  Rows 0-15 are fetched before the first branch, rows 16-31 and
// (N <= 40, N > 48) 32-63 inside the branch that first needs them; for
// 40 < N <= 48 each block from 4 on fetches its own rows right before use.
template <int N, int B>
__device__ __forceinline__ void sparse_nest(double (&x)[N], double (&U)[Blocks<N>::NB + 1], cdbl* col, int nb,
                                            double (&c)[N]) {
  constexpr int NB = Blocks<N>::NB;
  if constexpr (B < NB) {
    if (nb > B) {
      if constexpr (B == 2) fetch_rows<N, 16, (N < 32 ? N : 32)>(col, c);
      if constexpr (B == 4 && (N <= 40 || N > 48)) fetch_rows<N, 32, N>(col, c);
      sparse_nest<N, B + 1>(x, U, col, nb, c);
      // 40 < N <= 48: blocks 4.. fetch their own 8 rows after the deeper blocks
      // are done, so at most rows 0-31 + one block are live in SGPRs (no spills
      // in the walk loop; for N > 48 this form costs occupancy instead)
      if constexpr (B >= 4 && N > 40 && N <= 48) fetch_rows<N, 8 * B, (8 * B + 8 < N ? 8 * B + 8 : N)>(col, c);
      blk_add<N, B>(x, c);
      blk_prod<N, B>(x, U);
    }
  }
}

template <int N>
__device__ __forceinline__ void sparse_step(double (&x)[N], double (&U)[Blocks<N>::NB + 1], cdbl* col, int nb) {
  double c[N];
  fetch_rows<N, 0, (N < 16 ? N : 16)>(col, c);
  sparse_nest<N, 1>(x, U, col, nb, c);
  // block 0 always: nb == 0 only for an all-zero walk prefix, where adding the
  // (zero) column leaves x and U unchanged
  blk_add<N, 0>(x, c);
  blk_prod<N, 0>(x, U);
}

// Same step with a compile-time block count (walk bit 0, the odd steps: half
// of all steps) — straight-line code, only the rows it needs are fetched.
template <int N, int NBS>
__device__ __forceinline__ void sparse_step_static(double (&x)[N], double (&U)[Blocks<N>::NB + 1], cdbl* col) {
  static_assert(NBS >= 0 && NBS <= Blocks<N>::NB, "block count out of range");
  if constexpr (NBS > 0) {  // NBS == 0: all-zero walk column, x and U unchanged
    double c[N];
    constexpr int ROWS = (8 * NBS < N) ? 8 * NBS : N;
    auto blk = [&](auto Bc) {
      constexpr int b = decltype(Bc)::value;
      blk_add<N, b>(x, c);
      blk_prod<N, b>(x, U);
    };
    if constexpr (ROWS > 32) {
      fetch_rows<N, 32, ROWS>(col, c);
      for_down<NBS - 1, 4>(blk);
    }
    fetch_rows<N, 0, (ROWS < 32 ? ROWS : 32)>(col, c);
    for_down<(NBS < 4 ? NBS : 4) - 1, 0>(blk);
  }
}

// Dynamic wave-chunk queue: lane 0 takes the next chunk, the wave shares it.
// Which wave computes a chunk does not affect the result: every chunk writes
// its own slot of chunk_out, reduced afterwards in a fixed pairwise order.
__device__ __forceinline__ uint32_t next_chunk(unsigned int* counter) {
  uint32_t a = 0;
  if ((threadIdx.x & 63) == 0) a = atomicAdd(counter, 1u);
  return __builtin_amdgcn_readfirstlane(a);
}

// Lane-bit initialisation: x += col(e) on the lanes whose bit e is set.
// The column is wave-uniform (SGPR operands).  fma(sel, c, x) with sel in
// {0.0, 1.0} rounds exactly like x + (sel ? c : 0.0) for finite c — one VALU
// op per element and no divergent control flow.
template <int N>
__device__ __forceinline__ void add_col_masked(double (&x)[N], cdbl* col, bool on) {
  const double sel = on ? 1.0 : 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = __builtin_fma(sel, col[j], x[j]);
}

// Start state of lane `lane` in wave-chunk `ga`:
//   x = x0 + sum_{b in gray(ga)} col(L+m+b) + sum_{e in lane, e < L} col(e)
// applied in exactly this order (ascending b, then ascending e); mirrored by
// oracle/oracle.c orc_engine_start.
template <int N>
__device__ __forceinline__ void chunk_start(double (&x)[N], const WalkParams& p, uint64_t ga,
                                            uint32_t lane) {
  constexpr int NP = pad8(N);
  cdbl* x0 = opaque_c(p.x0, 0);
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = x0[j];
  uint64_t h = ga ^ (ga >> 1);
  const uint32_t hb = (uint32_t)(p.L + p.m);
  while (h) {
    const uint32_t b = (uint32_t)__builtin_ctzll(h);
    h &= h - 1;
    add_col<N>(x, opaque_c(p.cols, (2u * (hb + b)) * NP * 8u));
  }
  for (int e = 0; e < p.L; ++e)
    add_col_masked<N>(x, opaque_c(p.cols, (2u * e) * NP * 8u), (lane >> e) & 1u);
}

// A kernel argument read where it is used: a scalar load from the kernarg
// segment through an opaque base, so the value is not held in SGPRs across the
// walk (the register allocator spilled such values to VGPR lanes and reloaded
// them with v_readlane on every visited state).  Kernels whose first argument
// is their WalkParams only.
template <class T>
__device__ __forceinline__ T karg_at(uint32_t offset) {
  uint64_t a = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(a));
  return *(const __attribute__((address_space(4))) T*)(a + offset);
}
#define SUP_KARG(field) karg_at<decltype(WalkParams::field)>((uint32_t)__builtin_offsetof(WalkParams, field))

// chunk_start with the chunk bits' part read from the plan's start table
// (Plan::start_tab: x0 + those columns, added on the host in chunk_start's
// order, so the same values): one scalar-loaded row instead of popcount(gray
// ga) column adds; the lane columns are added here as chunk_start adds them.
template <int N>
__device__ __forceinline__ void chunk_start_tab(double (&x)[N], const WalkParams& p, uint64_t ga, uint32_t lane) {
  constexpr int NP = pad8(N);
  cdbl* t = opaque_c(SUP_KARG(start_tab), (uint32_t)ga * (uint32_t)(NP * 8));
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = t[j];
  for (int e = 0; e < p.L; ++e)
    add_col_masked<N>(x, opaque_c(p.cols, (2u * e) * NP * 8u), (lane >> e) & 1u);
}

// ------------------------------------------------------------ the fused fold --
// A value handed to another wave (any CU, any XCD: the XCDs' L2s are not
// coherent) goes through 8-byte agent-scope atomics on both sides, which are
// performed at the memory side (MI355X_MICROARCH.md, inter-workgroup
// visibility: "8-B agent atomics both sides"), and the publishing wave waits
// for them (vmcnt(0)) before its arrival is counted.
__device__ __forceinline__ void fold_publish(double* a, double v) {
  (void)__hip_atomic_exchange((unsigned long long*)a, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double fold_fetch(double* a) {
  return __builtin_bit_cast(double, __hip_atomic_fetch_or((unsigned long long*)a, 0ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void fold_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The wave's chunk group [a0, a0 + len) leaves the wave: lane l < len holds
// chunk a0 + l's partial (keep) and walked states (vkeep).  Called by the
// whole wave.  Without fold_cnt the partials are stored for
// launch_pairwise_reduce.  With it (round 6) the walk folds them itself into
// exactly that tree — 64-way levels over the chunk index, zero padded, one
// wave butterfly per group — each group formed by the wave whose arrival
// completes it (one counter per group: the last arriver, told by the value
// its atomic add returns, reads the group's values and publishes their sum
// one level up); the wave completing the root writes the result, the visited
// sum and the host's sequence flag, and zeroes the next launch's queue head.
// No reduction launch follows the walk.  A group may be completed by any
// wave; its sum is the same bits either way.
__device__ __forceinline__ void chunk_store(uint64_t a0, uint32_t len, double keep, uint32_t vkeep) {
  const uint32_t lane = __lane_id();
  const uint64_t count = SUP_KARG(chunk_count);
  const uint32_t nominal = len;  // the group's size (a power of two, a0 a multiple of it)
  if (a0 + len > count) len = (uint32_t)(count - a0);
  unsigned int* cnt = SUP_KARG(fold_cnt);
  if (!cnt) {
    if (lane < len) {
      SUP_KARG(chunk_out)[a0 + lane] = keep;
      unsigned int* vis = SUP_KARG(visited);
      if (vis) vis[a0 + lane] = vkeep;
    }
    return;
  }
  double* src = SUP_KARG(chunk_out);
  // The group's lowest tree levels inside the wave: it publishes one value,
  // the subtree sum of its `nominal` chunks (zero past the end) — the same
  // butterfly steps a 64-lane fold takes over them: the same bits — at
  // src[a0 / nominal].  A 64-group holds groups of one size (the host starts
  // the tail phase on a multiple of 64), so its level-1 fold reads 64 / size
  // values: the groups', or the tail groups' from tail_begin on.
  {
    double v = lane < len ? keep : 0.0;
    for (uint32_t o = 1; o < nominal; o <<= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) fold_publish(src + a0 / nominal, v);
  }
  unsigned long long* vacc = SUP_KARG(fold_vis);
  if (vacc) {  // walked states: an exact integer sum, any order
    unsigned long long v = lane < len ? (unsigned long long)vkeep : 0ull;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) (void)__hip_atomic_fetch_add(vacc, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  fold_drain();  // every value above performed before this wave's arrival counts
  double s = __shfl(keep, 0, 64);  // one chunk: the partial itself (no level)
  if (count > 1) {
    double* lv = SUP_KARG(fold_lv);
    uint64_t cv = count, idx = a0;
    uint32_t arrive = len;
    uint32_t sub = (idx & ~63ull) >= SUP_KARG(tail_begin) ? SUP_KARG(tail_group) : SUP_KARG(group);
    for (;;) {  // wave-uniform throughout
      const uint64_t g = idx >> 6, groups = (cv + 63u) >> 6;
      const uint64_t rest = cv - 64u * g;
      const uint32_t target = rest < 64u ? (uint32_t)rest : 64u;
      uint32_t old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(cnt + g, arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old + arrive != target) return;  // another wave completes this group
      if (lane == 0) __hip_atomic_store(cnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      // the rest of the group's tree: 64 / sub values (zero past the level's end)
      const uint32_t nsub = 64u / sub, real = (target + sub - 1u) / sub;
      double x = lane < real ? fold_fetch(src + (64u * g) / sub + lane) : 0.0;
      for (uint32_t o = 1; o < nsub; o <<= 1) x += __shfl_xor(x, o, 64);
      s = __shfl(x, 0, 64);
      if (groups == 1) break;  // the root
      if (lane == 0) fold_publish(lv + g, s);
      fold_drain();
      if (cv == count && groups <= 1024u) {
        // Up to 1024 level-1 groups: one counter for all of them, and the wave
        // completing the last one forms every upper level itself (level 2:
        // 64-groups of the level-1 values, zero past their end; level 3: the
        // <= 16 level-2 values) — the same tree in three memory round trips
        // instead of six at the walk's very end.
        unsigned int* top = cnt + groups;  // (where the level-2 counters would be)
        uint32_t o2 = 0;
        if (lane == 0) o2 = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        o2 = __builtin_amdgcn_readfirstlane(o2);
        if (o2 + 1u != (uint32_t)groups) return;
        if (lane == 0) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t g2 = (uint32_t)((groups + 63u) >> 6);  // <= 16
        double v[16];
#pragma unroll
        for (uint32_t k = 0; k < 16u; ++k) {  // every fetch first
          const uint64_t i = 64u * k + lane;
          v[k] = (k < g2 && i < groups) ? fold_fetch(lv + i) : 0.0;
        }
        double y = 0.0;
#pragma unroll
        for (uint32_t k = 0; k < 16u; ++k)
          if (k < g2) {
            double x2 = v[k];
            for (uint32_t o = 1; o < 64u; o <<= 1) x2 += __shfl_xor(x2, o, 64);
            y = lane == k ? x2 : y;
          }
        if (g2 > 1u)
          for (uint32_t o = 1; o < 64u; o <<= 1) y += __shfl_xor(y, o, 64);
        s = __shfl(y, 0, 64);
        break;
      }
      src = lv;
      lv += groups;
      cnt += groups;
      cv = groups;
      idx = g;
      arrive = 1;
      sub = 1;
    }
  }
  if (lane == 0) {
    double* res = SUP_KARG(fold_out);
    unsigned long long* res64 = (unsigned long long*)res;
    const unsigned long long vis_total =
        vacc ? __hip_atomic_exchange(vacc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    unsigned int* reset = SUP_KARG(fold_reset);
    if (reset) __hip_atomic_store(reset, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (SUP_KARG(fold_sys)) {  // the result is the signal: visited sum first, drained, then the value
      if (vacc) {
        __hip_atomic_store(res64 + 2, vis_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        fold_drain();
      }
      __hip_atomic_store(res64, __builtin_bit_cast(unsigned long long, s), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    res[0] = s;
    if (vacc) res64[2] = vis_total;
    unsigned int* flag = SUP_KARG(fold_flag);
    if (flag) {
      __threadfence_system();
      fold_drain();  // (the compiler may drop the fence's own wait: MI355X_MICROARCH.md, compiler hazard)
      __hip_atomic_store(flag, SUP_KARG(fold_seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace sup
