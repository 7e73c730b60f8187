/*
 * superman.h — C ABI of the MI355X-native Ryser / Gray-code permanent engine.
 *
 * This is the drop-in boundary for the reference's GPU exact-permanent path
 * (kamerkaya/SUPerman, v1 top level).  Every entry point below names the
 * reference symbol it replaces (file:line in the reference tree).  The
 * reference's wrappers are C++ templates over the storage type T in
 * {int, float, double}; here T travels as a `sup_dtype` tag next to a
 * `const void*`, so the ABI is plain C (pointers, sizes, an error code).
 *
 * Conventions (reference behaviour kept, reference defects fixed):
 *   - Host arrays are borrowed read-only; the caller owns them
 *     (reference: main.cu:501-528 new[]/delete[] around RunAlgo).
 *   - Device memory is owned by the library (per-device context, created on
 *     first use, reused across calls).
 *   - Every function returns 0 (SUP_OK) or a negative SUP_E* code; the
 *     message is available from sup_last_error() (thread-local).  The
 *     reference reports nothing (no cudaGetLastError anywhere).
 *   - The permanent is written through `out` as a double
 *     (reference returns it by value; interface_connector.c:22 truncated it
 *     to int — not reproduced).
 *   - X is always fp64 (the reference v1 float-X path, algo.h:664 /
 *     gpu_exact_dense.cu:336, is numerically wrong on real matrices and is
 *     not reproduced).
 *   - Device 0 is the default device (the reference hard-codes
 *     cudaSetDevice(1), gpu_exact_dense.cu:664); `sup_opts.device_id`
 *     selects another one (v2 flag -l, revised_perman/main.cpp:1443).
 */
#ifndef SUPERMAN_H
#define SUPERMAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUP_ABI_VERSION 10  /* 10: sup_opts.timing, sup_kernel_time (round 6); 9: sup_device_warmup, sup_opts.use_rccl = -1 (round 6); 8: sup_device_checks (round 5); 7: sup_rccl_devices, sup_stats.seg_cached_bits / seg_pair_bits */

/* ---- error codes ------------------------------------------------------ */
#define SUP_OK            0
#define SUP_EINVAL      (-1)   /* bad argument (n out of range, null pointer, bad range) */
#define SUP_ENODEV      (-2)   /* no HIP device / device id out of range                 */
#define SUP_EHIP        (-3)   /* a HIP runtime call failed                              */
#define SUP_ERCCL       (-4)   /* an RCCL call failed                                    */
#define SUP_ENOMEM      (-5)   /* host or device allocation failed                       */
#define SUP_EIO         (-6)   /* matrix file could not be read                          */
#define SUP_EUNSUPPORTED (-7)  /* algorithm id / option combination not provided         */

#define SUP_MAX_N 64           /* 64-bit Gray index: reference limit algo.h:752,781      */
#define SUP_MAX_READ_N 4096    /* MatrixMarket input and sup_decompose: larger matrices
                                  are accepted when the -o reductions shrink every leaf
                                  to <= SUP_MAX_N                                       */

/* ---- storage type of the input matrix (reference template parameter T) -- */
typedef enum {
  SUP_INT32 = 0,    /* file header "int"    (main.cu:494) */
  SUP_FLOAT32 = 1,  /* file header "float"  (main.cu:530) */
  SUP_FLOAT64 = 2   /* file header "double" (main.cu:563) */
} sup_dtype;

/* ---- kernel family ------------------------------------------------------ */
typedef enum {
  SUP_KERNEL_DENSE = 0,       /* kernel_xshared_coalescing_mshared          gpu_exact_dense.cu:329-399.
                                 The engine runs the plain dense walk, or the prefix-blocked walk when
                                 its cost model says the matrix's zeros make that cheaper (same sum) */
  SUP_KERNEL_SPARYSER = 1,    /* kernel_xshared_coalescing_mshared_sparse   gpu_exact_sparse.cu:455-552 */
  SUP_KERNEL_SKIPPER = 2,     /* kernel_xshared_coalescing_mshared_skipper  gpu_exact_sparse.cu:555-670 */
  SUP_KERNEL_DENSE_PLAIN = 3, /* always the plain dense walk (2n fp64 ops per Gray step)                */
  SUP_KERNEL_SEGMENTED = 4,   /* always the segmented walk specialised for the matrix pattern (n >= 10;
                                 the GPU entry points compile it with hiprtc, sup_perman_cpu runs the
                                 same operations on host threads)                                       */
  SUP_KERNEL_DENSE_LDS = 5    /* the plain dense walk with X and the walk columns staged in LDS, as the
                                 reference kernel (gpu_exact_dense.cu:329-399); bit-identical to
                                 SUP_KERNEL_DENSE_PLAIN, kept to measure the layout    */
} sup_kernel;

/* ---- multi-device scheduling policy -------------------------------------- */
typedef enum {
  SUP_SCHED_SINGLE = 0,   /* one device           (-p4; gpu_exact_dense.cu:640-699)            */
  SUP_SCHED_STATIC = 1,   /* static split         (-p5; gpu_exact_dense.cu:701-774)            */
  SUP_SCHED_CHUNKS = 2,   /* dynamic chunk queue  (-p6/-p8; gpu_exact_dense.cu:776-904,
                                                   gpu_exact_sparse.cu:1192-1324)            */
  SUP_SCHED_MANUAL = 3    /* manual distribution  (-p66; gpu_exact_dense.cu:913-990,
                             gpu_exact_sparse.cu:1328-1400): 3/8, 3/8, 1/8, 1/8 of the space
                             on devices 0-3 (gpu_num 4, as main.cu:71 passes; with fewer
                             devices the pieces wrap round modulo gpu_num)             */
} sup_sched;

typedef struct {
  int gpu_num;        /* devices to use (-d); default 1                                      */
  int device_id;      /* first device (v2 -l); default 0                                     */
  int threads;        /* host threads for the CPU worker (-t); default 16 (main.cu:333)      */
  int cpu_worker;     /* -c together with -g: a CPU thread also takes chunks                 */
  int grid_dim;       /* 0 = auto (resident-wave sized); reference default 2048              */
  int block_dim;      /* 0 = auto (256); the engine only supports 256                         */
  int walk_log2;      /* 0 = auto (the segmented walk lengthens its wave-chunks where its    */
                      /*  steps are cheap); else each lane walks 2^walk_log2 Gray steps per  */
                      /*  wave-chunk (sup_perman, sup_perman_shard, sup_plan_info)           */
  int chunk_log2;     /* 0 = auto; for SUP_SCHED_CHUNKS: wave-chunks per queue item = 2^x    */
  int use_rccl;       /* 1: multi-device partials combined by one RCCL all-reduce (bit-     */
                      /*    identical to the host combine); 2: also with a single device;   */
                      /*    -1: RCCL when the devices are distinct physical GPUs, else the  */
                      /*    host pairwise tree (the perman CLI's default); 0: host tree     */
  int verbose;        /* print per-device / per-chunk timing lines like the reference        */
  int jit;            /* segmented walk specialised for the matrix pattern (hiprtc, gfx950):  */
                      /*  -1 never; 0 auto: when its cost model wins and the predicted walk  */
                      /*  time saved exceeds what the plan costs (3 s, or twice this host's  */
                      /*  last cold plan; 0.1 s with the matrix's choices on disk; the first */
                      /*  decision for a matrix holds for the process); 1 whenever its cost  */
                      /*  model wins                                                         */
  const char* checkpoint; /* SUP_SCHED_CHUNKS (-p6/-p8) only, NULL = none: file recording every */
                      /*  finished queue item's partial (appended and flushed as items finish;*/
                      /*  header: plan fingerprint, chunk range, item size).  A call given a  */
                      /*  file with a matching header takes the items it lists instead of    */
                      /*  walking them, so an interrupted run resumes; the result is bit-    */
                      /*  identical to an uninterrupted one.  A mismatching header is         */
                      /*  SUP_EINVAL.  (ABI version 6)                                        */
  int timing;         /* sup_perman_shard: 1 (default) sup_stats.kernel_ms of the call (it waits */
                      /*  for the walk's end event); 0: the walk's HIP events are recorded but */
                      /*  read later by sup_kernel_time (kernel_ms 0) — the call returns as   */
                      /*  soon as its result is there (~8 us sooner on a 0.5 ms walk).        */
                      /*  (ABI version 10)                                                    */
} sup_opts;

typedef struct {
  double   kernel_ms;       /* device time of the walk kernels (max over devices, hipEvents)   */
  double   wall_ms;         /* host wall time of the call (upload + launch + reduce)           */
  uint64_t gray_steps;      /* nominal Gray steps = 2^(n-1)                                    */
  uint64_t visited_steps;   /* steps whose product was actually evaluated (sparse/skipper)     */
  int      devices_used;
  int      lane_bits;       /* L: Gray bits spread over the 64 lanes of a wave                  */
  int      walk_bits;       /* m: Gray bits walked by every wave-chunk                          */
  int      grid;            /* blocks per launch (256 threads each) on each device             */
  int      chunks_done_cpu; /* queue items taken by the CPU worker                              */
  double   partials[16];    /* per-device partial sums (before the final combine)              */
  int      walk_kind;       /* walk actually run: 0 dense, 1 prefix-blocked (SpaRyser), 2 SkipPer,
                               3 segmented (pattern-specialised, sup_opts.jit), 4 dense with X
                               in LDS (SUP_KERNEL_DENSE_LDS)                                     */
  int      leaves;          /* permanents computed: 1, or the leaf count of sup_perman_reduced   */
  double   est_ops_per_step;/* cost model: fp64 VALU ops per Gray step and lane                 */
  double   jit_ms;          /* hiprtc compile time spent by this call (0 when cached / unused)   */
  int      items_resumed;   /* queue items taken from sup_opts.checkpoint instead of walked      */
  int16_t  seg_cached_bits; /* segmented walk (walk_kind 3): cached walk bits of the plan run    */
  int16_t  seg_pair_bits;   /* segmented walk: specialised pair bits (0 for other walks)          */
} sup_stats;

/* Fill `o` with defaults. */
void sup_opts_init(sup_opts* o);

/* Library metadata. */
int         sup_abi_version(void);
const char* sup_last_error(void);     /* thread-local message of the last failing call */
int         sup_device_count(int* count);
/* The physical HIP device of logical devices 0..ndev-1 as the -R RCCL combine
 * uses them (its communicators, slot buffers and streams); SUP_DEVICE_MAP may
 * permute or repeat physical ids, and SUP_ERCCL is returned when two logical
 * devices share one GPU (RCCL needs distinct devices).  No HIP call. */
int         sup_rccl_devices(int ndev, int* phys);
/* Device-placement assertions passed so far in this process.  With
 * SUP_CHECK_DEVICE=1 in the environment, every allocation, module load and
 * launch of a device thread first checks that the thread's HIP device is the
 * physical device behind the logical device whose context it uses, and that
 * this logical device is the one the thread last selected (a mismatch fails
 * the call with SUP_EHIP); 0 when the mode is off.  Tests and diagnostics. */
uint64_t    sup_device_checks(void);
/* Initialise the HIP runtime, the contexts of devices [device_id, device_id +
 * gpu_num) and the ahead-of-time walk code objects of order n (0: none), so a
 * caller can run it on a thread beside its planning (the perman CLI does).
 * Thread-safe; a later call on the same devices returns at once. */
int         sup_device_warmup(int device_id, int gpu_num, int n);
/* The walk-kernel times (HIP events on the walk's stream) of this thread's
 * sup_perman_shard calls on logical device `device_id` made with
 * sup_opts.timing = 0 since the last sup_kernel_time: waits for them, returns
 * their sum (*total_ms) and count (*launches), and starts a new tally.  Any
 * pointer may be NULL (the tally is still reset). */
int         sup_kernel_time(int device_id, double* total_ms, uint64_t* launches);

/* ------------------------------------------------------------------------ *
 * Generic entry point.  `mat` is n x n row-major of type `t` (already
 * preprocessed by the caller when the reference would have rewritten it:
 * SortOrder / SkipOrder, util.h:553-684).  `kernel` picks the Gray walk,
 * `sched` the device policy.  Result: the permanent, fp64.
 * Replaces RunAlgo<T>'s GPU exact branch (main.cu:30-143).
 * ------------------------------------------------------------------------ */
int sup_perman(const void* mat, sup_dtype t, int n, sup_kernel kernel, sup_sched sched,
               const sup_opts* o, double* out, sup_stats* st);

/* Partial Ryser sum over reference Gray indices [start, end):
 *   sum_{i in [start,end)} (-1)^i * prod_j x_j(gray(i))
 * with x(0) = Nijenhuis-Wilf start vector (gpu_exact_dense.cu:642-652).
 * This is exactly what the reference chunk helpers return
 * (cpu_perman64 gpu_exact_dense.cu:6-69; cpu_perman64_sparse
 * gpu_exact_sparse.cu:6-87; cpu_perman64_skipper :89-191) except that index
 * 0 (the p0 term) is included when start == 0.  start and end must be
 * multiples of 2^(lane_bits + walk_bits) reported by the engine for this n
 * (any power-of-two aligned chunk boundary >= 64 works), or end == 2^(n-1). */
int sup_partial(const void* mat, sup_dtype t, int n, sup_kernel kernel,
                uint64_t start, uint64_t end, const sup_opts* o, double* out, sup_stats* st);

/* Shard `shard` of `nshards` of the engine's own enumeration of the full sum
 * (same plan as sup_perman): the shards' partials add up to
 * perm / (4(n&1)-2).  For one process per GPU (torch.distributed / MPI):
 * each rank computes its shard on `o->device_id`, then one all-reduce. */
int sup_perman_shard(const void* mat, sup_dtype t, int n, sup_kernel kernel, int shard, int nshards,
                     const sup_opts* o, double* out_partial, sup_stats* st);

/* The plan sup_perman would run with options `o` (NULL = defaults; o->jit and
 * o->gpu_num matter): walk kind (0 dense, 1 prefix/SpaRyser, 2 SkipPer,
 * 3 segmented), engine-bit -> column map (n-1 entries), lane and walk bits,
 * and (segmented walk) the walk bits held in every state (*cached_bits, 0-3)
 * and the pair bits with a specialised step (*pair_bits, 3-8; the walk loop is
 * unrolled by 2^pair_bits pair steps); *est_ops_per_step = the walk's cost
 * model (sup_stats.est_ops_per_step); any pointer may be NULL.  For the test
 * harness's bit-exact mirror of the enumeration. */
int sup_plan_info(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o, int* walk_kind,
                  int* colmap, int* lane_bits, int* walk_bits, int* cached_bits, int* pair_bits,
                  double* est_ops_per_step);

/* 64-bit fingerprint of the plan sup_perman / sup_perman_shard would run
 * with options `o` (walk kind, layout, engine column map, signed column
 * table, start vector, the segmented walk's cached / pair bits, budget and
 * kernel source).  One process per GPU: every rank plans on its own, and the
 * shards add up to the permanent only if all ranks walk the same plan —
 * all-gather the keys before summing (bench.py does, and aborts on a
 * mismatch). */
int sup_plan_key(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o, uint64_t* key);

/* Build the plan sup_perman would run and, if it is the segmented walk,
 * compile its kernel now (hiprtc; no device needed) into the in-memory and
 * disk caches, so a later sup_perman does not pay the compile.  (A SkipPer
 * request on an integer matrix measures SkipPer's visited fraction on a
 * sample of its chunks when a device is visible, here and in sup_plan_info.)  *walk_kind =
 * the plan's walk kind; *compile_ms = hiprtc time spent (0 when cached). */
int sup_prepare(const void* mat, sup_dtype t, int n, sup_kernel kernel, const sup_opts* o, int* walk_kind,
                double* compile_ms);
/* Explicit CPU algorithm for the CLI's `-c` mode (reference RunAlgo cpu
 * branch, main.cu:186-238): the same wave-chunk walk on `threads` host
 * threads, bit-identical to the GPU kernels.  Never used as a fallback by the
 * GPU entry points above, which fail with SUP_ENODEV without a device. */
int sup_perman_cpu(const void* mat, sup_dtype t, int n, sup_kernel kernel, int threads,
                   double* out, sup_stats* st);

/* Exact permanent of an integer matrix (int32, or float/double holding
 * integers; |a| < 2^31, row sums of |a| < 2^31).  The reference computes int
 * and -b (binary) inputs in fp64 (rounded beyond 2^53); here the same Ryser /
 * Gray-code walk runs on 2A in residue arithmetic modulo primes < 2^42 and
 * the residues are joined by CRT (walk_exact.hip, exact.cpp), with a built-in
 * divisibility self-check.  *out receives the signed decimal integer,
 * NUL-terminated (520 bytes always suffice).  o->gpu_num devices from
 * o->device_id take power-of-two items of wave-chunks from a queue
 * (o->chunk_log2 wave-chunks each, 0 = ~16 items per taker; one device alone
 * walks its whole range), and with o->cpu_worker a CPU thread (o->threads
 * host threads) takes items too; on_cpu = 1 runs o->threads host threads
 * instead.  The result never depends on who took which item (residue sums).
 * st (optional): kernel_ms (max over devices), wall_ms, devices_used,
 * gray_steps, chunks_done_cpu. */
int sup_perman_exact(const void* mat, sup_dtype t, int n, const sup_opts* o, int on_cpu, char* out,
                     size_t out_len, sup_stats* st);

/* The permanent in double-double (~106-bit significand): the MI355X form of
 * the reference's quad-precision calculation (v2 `-q`,
 * revised_perman/main.cpp:141-142 -> parallel_perman64<__float128,S>,
 * cpu_algos.hpp:761-873, CPU only).  The dense Ryser / Gray walk of
 * sup_perman (default layout, same wave-chunks) with every value a
 * double-double (walk_dd.hip); perm = *out_hi + *out_lo (out_lo may be NULL).
 * o->gpu_num devices from o->device_id split the wave-chunks statically;
 * on_cpu = 1 runs the same operations on o->threads host threads.  Chunk
 * partials are combined in one fixed pairwise order, so the result is
 * bit-identical for any device or thread count.  ~8x the fp64 walk's work
 * (16n + 13 fp64 ops per Gray step). */
int sup_perman_quad(const void* mat, sup_dtype t, int n, const sup_opts* o, int on_cpu, double* out_hi,
                    double* out_lo, sup_stats* st);

/* Nijenhuis-Wilf prologue (gpu_exact_dense.cu:642-652): x0[j] = a[j][n-1] - rowsum_j/2,
 * p0 = prod x0.  Host-only helper, exported for the test harness. */
int sup_nw_start(const void* mat, sup_dtype t, int n, double* x0, double* p0);

/* ------------------------------------------------------------------------ *
 * Reference-signature wrappers: one per GPU exact wrapper of the v1 tree.
 * Arguments keep the reference meaning; grid_dim/block_dim are accepted for
 * signature compatibility (the engine sizes its own launch when they are <= 0
 * or when they do not match its 256-thread wave-chunk layout).
 * ------------------------------------------------------------------------ */

/* gpu_exact_dense.cu:641 gpu_perman64_xshared_coalescing_mshared (-p4) */
int sup_gpu_perman64_xshared_coalescing_mshared(const void* mat, sup_dtype t, int nov,
    int grid_dim, int block_dim, double* out);
/* gpu_exact_dense.cu:702 ..._multigpu (-p5) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu(const void* mat, sup_dtype t, int nov,
    int gpu_num, int grid_dim, int block_dim, double* out);
/* gpu_exact_dense.cu:777 ..._multigpucpu_chunks (-p6) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks(const void* mat, sup_dtype t,
    int nov, int gpu_num, int cpu, int threads, int grid_dim, int block_dim, double* out);
/* gpu_exact_sparse.cu:854 ..._sparse (-p4 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_sparse(const void* mat, const int* cptrs,
    const int* rows, const void* cvals, sup_dtype t, int nov, int grid_dim, int block_dim,
    double* out);
/* gpu_exact_sparse.cu:917 ..._multigpu_sparse (-p5 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse(const void* mat, const int* cptrs,
    const int* rows, const void* cvals, sup_dtype t, int nov, int gpu_num, int grid_dim,
    int block_dim, double* out);
/* gpu_exact_sparse.cu:996 ..._multigpucpu_chunks_sparse (-p6 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse(const void* mat,
    const int* cptrs, const int* rows, const void* cvals, sup_dtype t, int nov, int gpu_num,
    int cpu, int threads, int grid_dim, int block_dim, double* out);
/* gpu_exact_dense.cu:914 ..._multigpu_manual_distribution (-p66): 3/8, 3/8, 1/8, 1/8 on 4 devices */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution(const void* mat, sup_dtype t,
    int nov, int gpu_num, int grid_dim, int block_dim, double* out);
/* gpu_exact_sparse.cu:1328 ..._multigpu_sparse_manual_distribution (-p66 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution(const void* mat,
    const int* cptrs, const int* rows, const void* cvals, sup_dtype t, int nov, int gpu_num, int grid_dim,
    int block_dim, double* out);
/* gpu_exact_sparse.cu:1124 ..._skipper (-p7 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_skipper(const void* mat, const int* rptrs,
    const int* cols, const int* cptrs, const int* rows, const void* cvals, sup_dtype t, int nov,
    int grid_dim, int block_dim, double* out);
/* gpu_exact_sparse.cu:1193 ..._multigpucpu_chunks_skipper (-p8 -s) */
int sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper(const void* mat,
    const int* rptrs, const int* cols, const int* cptrs, const int* rows, const void* cvals,
    sup_dtype t, int nov, int gpu_num, int cpu, int threads, int grid_dim, int block_dim,
    double* out);

/* ------------------------------------------------------------------------ *
 * Host preprocessing (hot-path inputs).
 * ------------------------------------------------------------------------ */

/* v1 matrix file: header "n nnz type", then 0-based "i j v" lines; malformed
 * lines skipped; binary => every listed entry is 1 (util.h:343-358,
 * main.cu:494-498).  *mat is allocated with malloc (free with sup_free). */
int sup_read_matrix(const char* path, int binary, void** mat, sup_dtype* t, int* n, int* nnz_header);
void sup_free(void* p);

/* CSR + CSC of a dense row-major matrix; nonzero test is != 0 (the reference
 * uses > 0 at util.h:537,542 and silently drops negative entries).  Arrays
 * are caller-allocated: cptrs/rptrs n+1, rows/cols/vals nnz (query nnz with
 * sup_count_nnz).  (util.h:522-551) */
int sup_count_nnz(const void* mat, sup_dtype t, int n, int* nnz);
int sup_compress(const void* mat, sup_dtype t, int n, int* cptrs, int* rows, void* cvals,
                 int* rptrs, int* cols, void* rvals);
/* SortOrder: stable ascending column nnz; rewrites mat in place and fills
 * colperm (new column c = old column colperm[c]).  (util.h:553-619) */
int sup_sort_order(void* mat, sup_dtype t, int n, int* colperm);
/* SkipOrder: greedy min-degree column order, rows in first-touch order;
 * rewrites mat in place.  (util.h:621-684) */
int sup_skip_order(void* mat, sup_dtype t, int n, int* rowperm, int* colperm);

/* MatrixMarket coordinate file (revised_perman/read_matrix.hpp:11-157 and
 * main.cpp:1515-1580): banner "%%MatrixMarket matrix coordinate <type>
 * <symmetry>", '%' comments, "M N nz", 1-based "i j [v]" entries.  real ->
 * SUP_FLOAT64; integer / pattern (or binary) -> SUP_INT32; pattern or binary
 * entries are 1; symmetric and skew-symmetric files mirror every off-diagonal
 * entry with the SAME value (as the reference does); complex, array format
 * and non-square matrices are rejected (SUP_EIO).  nnz_lines = nz from the
 * size line.  n may be up to SUP_MAX_READ_N (for sup_perman_reduced).
 * sup_read_matrix also accepts MatrixMarket files (detected by the banner),
 * so the CLI's -f takes either format. */
int sup_read_mtx(const char* path, int binary, void** mat, sup_dtype* t, int* n, int* nnz_lines);

/* ------------------------------------------------------------------------ *
 * Reductions in front of the engine (reference v2
 * -o / -u, revised_perman/main.cpp:993-1264, util.h:1138-1593).
 * ------------------------------------------------------------------------ */
typedef struct {
  int compress;           /* -o: remove degree-1/2 rows+columns, then expand rows/columns of
                             degree < max_deg while n > min_n (d1/d2/d34 recursion)            */
  double scale_threshold; /* -u <t>: scale rows/columns to sums t before each permanent and
                             divide the factors out afterwards; <= 0 = off                      */
  int min_n;              /* recursion stops at n <= min_n (reference: 30)                      */
  int max_deg;            /* expand only while the minimum degree < max_deg (reference: 5)      */
  int preprocessing;      /* -r applied to every leaf: 0 none, 1 SortOrder, 2 SkipOrder         */
} sup_reduce_opts;
void sup_reduce_opts_init(sup_reduce_opts* r);

/* Leaf permanent callback: perm of the n x n fp64 row-major matrix a. */
typedef int (*sup_leaf_fn)(const double* a, int n, void* user, double* out_perm);

/* Reduce `mat` and combine fn(leaf) over the expansion tree (left + right,
 * scale factors divided out).  No device work of its own: fn decides how each
 * leaf is computed.  *n_leaves = number of fn calls.  n <= SUP_MAX_READ_N;
 * a leaf larger than SUP_MAX_N fails with SUP_EUNSUPPORTED. */
int sup_decompose(const void* mat, sup_dtype t, int n, const sup_reduce_opts* r, sup_leaf_fn fn, void* user,
                  double* out, int* n_leaves);

/* sup_decompose with every leaf computed by the engine: sup_perman (on_cpu =
 * 0) or sup_perman_cpu (on_cpu = 1, o->threads threads) after r->preprocessing.
 * st accumulates over the leaves (kernel_ms, wall_ms, gray_steps, visited_steps,
 * leaves); the other fields describe the last leaf. */
int sup_perman_reduced(const void* mat, sup_dtype t, int n, sup_kernel kernel, sup_sched sched, const sup_opts* o,
                       int on_cpu, const sup_reduce_opts* r, double* out, sup_stats* st);

/* sup_perman_exact after the -o reductions (d1/d2/d34, as sup_perman_reduced
 * with r->compress; scaling is refused: not exact).  The tree folds every
 * coefficient into its leaves, so the permanent is the exact sum of the exact
 * leaf permanents (a big integer; up to 4096 x 4096 input, leaves <= 64).
 * st (optional): kernel_ms summed over leaves, leaves, wall_ms. */
int sup_perman_reduced_exact(const void* mat, sup_dtype t, int n, const sup_opts* o, int on_cpu,
                             const sup_reduce_opts* r, char* out, size_t out_len, sup_stats* st);

/* sup_perman_quad after the -o / -u reductions (as sup_perman_reduced):
 * every leaf by the double-double walk, the tree combined (sums, and the
 * scaling factors divided out) in double-double.  The leaf matrices are
 * formed in fp64 as in the reference; the fp64 walk's cancellation, which
 * costs the reduced sum its digits (HISTORY.md §7), is gone.  st->leaves = the
 * leaf count. */
int sup_perman_reduced_quad(const void* mat, sup_dtype t, int n, const sup_opts* o, int on_cpu,
                            const sup_reduce_opts* r, double* out_hi, double* out_lo, sup_stats* st);



/* ------------------------------------------------------------------------ *
 * Randomized estimators (reference -a, main.cu:77-103,
 * 156-183, 193-243).  Both estimate the permanent of the 0/1 nonzero pattern,
 * as the reference's do.  method 0: Rasmussen (kernel_rasmussen,
 * gpu_approximation_dense.cu:155-229; CPU algo.h:270-366); method 1:
 * scaling-guided importance sampling (kernel_approximation,
 * gpu_approximation_dense.cu:231-371; CPU algo.h:472-560) with Sinkhorn
 * passes every scale_intervals steps (-y, default 4), scale_times passes each
 * (-z, default 5).  `samples` (-x, default 100000) is rounded up to a multiple
 * of 64.  Randomness is Philox4x32-10 keyed by `seed`, counter (sample, step):
 * the estimate is a function of (matrix, method, samples, seed) only — the same
 * on the CPU (on_cpu = 1, o->threads threads), on one GPU or on o->gpu_num
 * GPUs (+ o->cpu_worker), which is how the reference's _multigpucpu_chunks
 * forms (gpu_approximation_dense.cu:411-525, 573-700) map here.  n <= 1024.
 * ------------------------------------------------------------------------ */
typedef struct {
  double   mean;           /* the estimate                                      */
  double   std_error;      /* sample standard deviation / sqrt(samples)         */
  double   zero_fraction;  /* samples that hit a dead end (estimate 0)          */
  uint64_t samples;        /* samples drawn (multiple of 64)                    */
  double   kernel_ms;      /* device time (max over devices)                    */
  double   wall_ms;
  int      devices;
  int      reserved_;
  int64_t  cpu_blocks;     /* 64-sample blocks computed on host threads         */
} sup_approx_result;

int sup_approx(const void* mat, sup_dtype t, int n, int method, uint64_t samples, int scale_intervals,
               int scale_times, uint64_t seed, const sup_opts* o, int on_cpu, sup_approx_result* res);

/* Grid graph of the -i mode (util.h:403-520 gridGraph2compressed): the
 * bipartite adjacency (nov = m*n/2, one of m, n even) whose permanent is the
 * number of domino tilings of the m x n board; *mat from malloc (sup_free). */
int sup_grid_graph(int m, int n, int** mat, int* nov);

#ifdef __cplusplus
}
#endif
#endif /* SUPERMAN_H */
