/*
 * runalgo_gpu.c — the reference's GPU exact dispatch (RunAlgo<T>,
 * main.cu:30-155) retargeted to the drop-in C ABI, as a maintainer would
 * rewire it: the caller reads the matrix (sup_read_matrix, util.h:343-358),
 * applies -r1 SortOrder / -r2 SkipOrder (util.h:553-684), builds CSR + CSC
 * (sup_compress, util.h:522-551) and calls the reference-named wrapper for the
 * algorithm id (the sup_gpu_perman64_* entry points, include/superman.h).
 * Every result is printed next to sup_perman with the same kernel family and
 * device policy, so the test (tests/test_gpu_capi_runalgo.py) can assert that
 * the wrappers are the engine bit for bit.
 *
 *   runalgo_gpu <matrix file> <algo id> <sparse 0|1> <-r 0|1|2> [gpu_num]
 *   runalgo_gpu --bad-csc <matrix file>   (a CSC without the negative entries)
 *
 * Output: "Result: <name> <perm %.17e>" and "Check: <perm %.17e>", or
 * "Error: <code> <message>".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/superman.h"

static size_t esize(sup_dtype t) { return t == SUP_FLOAT64 ? 8 : 4; }

static int fail(int rc) {
  printf("Error: %d %s\n", rc, sup_last_error());
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && strcmp(argv[1], "--bad-csc") == 0) {
    void* mat = NULL;
    sup_dtype t;
    int n = 0, nnz_h = 0, nnz = 0, rc;
    if ((rc = sup_read_matrix(argv[2], 0, &mat, &t, &n, &nnz_h))) return fail(rc);
    if ((rc = sup_count_nnz(mat, t, n, &nnz))) return fail(rc);
    int *cptrs = calloc(n + 1, sizeof(int)), *rows = calloc(nnz + 1, sizeof(int));
    void* cvals = calloc(nnz + 1, esize(t));
    /* the reference's `> 0` test (util.h:537): negative entries dropped */
    int k = 0;
    for (int c = 0; c < n; ++c) {
      cptrs[c] = k;
      for (int r = 0; r < n; ++r) {
        double v = t == SUP_FLOAT64 ? ((double*)mat)[r * n + c] : t == SUP_FLOAT32 ? ((float*)mat)[r * n + c]
                                                                               : ((int*)mat)[r * n + c];
        if (v > 0) {
          rows[k] = r;
          memcpy((char*)cvals + k * esize(t), (char*)mat + ((size_t)r * n + c) * esize(t), esize(t));
          ++k;
        }
      }
    }
    cptrs[n] = k;
    double perm = 0.0;
    rc = sup_gpu_perman64_xshared_coalescing_mshared_sparse(mat, cptrs, rows, cvals, t, n, 2048, 256, &perm);
    if (rc) return fail(rc);
    printf("Result: accepted %.17e\n", perm);
    return 0;
  }
  if (argc < 5) {
    fprintf(stderr, "usage: runalgo_gpu <file> <algo> <sparse> <r> [gpu_num]\n");
    return 2;
  }
  const int algo = atoi(argv[2]), dense = !atoi(argv[3]), prep = atoi(argv[4]);
  const int gpu_num = argc > 5 ? atoi(argv[5]) : 1;
  const int grid_dim = 2048, cpu = 0, threads = 16;
  void* mat = NULL;
  sup_dtype t;
  int n = 0, nnz_h = 0, nnz = 0, rc;
  if ((rc = sup_read_matrix(argv[1], 0, &mat, &t, &n, &nnz_h))) return fail(rc);
  const int block_dim = t == SUP_FLOAT64 ? 128 : 256; /* main.cu:24-28 */
  int* perm_r = malloc(sizeof(int) * n);
  int* perm_c = malloc(sizeof(int) * n);
  if (prep == 1 && (rc = sup_sort_order(mat, t, n, perm_c))) return fail(rc);
  if (prep == 2 && (rc = sup_skip_order(mat, t, n, perm_r, perm_c))) return fail(rc);
  if ((rc = sup_count_nnz(mat, t, n, &nnz))) return fail(rc);
  int *cptrs = malloc(sizeof(int) * (n + 1)), *rows = malloc(sizeof(int) * (nnz + 1));
  int *rptrs = malloc(sizeof(int) * (n + 1)), *cols = malloc(sizeof(int) * (nnz + 1));
  void *cvals = malloc(esize(t) * (nnz + 1)), *rvals = malloc(esize(t) * (nnz + 1));
  if ((rc = sup_compress(mat, t, n, cptrs, rows, cvals, rptrs, cols, rvals))) return fail(rc);

  const char* name = NULL;
  sup_kernel kern = SUP_KERNEL_DENSE;
  sup_sched sched = SUP_SCHED_SINGLE;
  double perm = 0.0;
  int g = 1;
  if (dense) {
    switch (algo) {
      case 4:
        name = "gpu_perman64_xshared_coalescing_mshared";
        rc = sup_gpu_perman64_xshared_coalescing_mshared(mat, t, n, grid_dim, block_dim, &perm);
        break;
      case 5:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu";
        sched = SUP_SCHED_STATIC, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpu(mat, t, n, gpu_num, grid_dim, block_dim, &perm);
        break;
      case 6:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks";
        sched = SUP_SCHED_CHUNKS, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks(mat, t, n, gpu_num, cpu, threads,
                                                                            grid_dim, block_dim, &perm);
        break;
      case 66:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution";
        sched = SUP_SCHED_MANUAL, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution(mat, t, n, gpu_num, grid_dim,
                                                                                      block_dim, &perm);
        break;
      default: printf("Unknown Algorithm ID\n"); return 0;
    }
  } else {
    kern = SUP_KERNEL_SPARYSER;
    switch (algo) {
      case 4:
        name = "gpu_perman64_xshared_coalescing_mshared_sparse";
        rc = sup_gpu_perman64_xshared_coalescing_mshared_sparse(mat, cptrs, rows, cvals, t, n, grid_dim, block_dim,
                                                                &perm);
        break;
      case 5:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_sparse";
        sched = SUP_SCHED_STATIC, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse(mat, cptrs, rows, cvals, t, n, gpu_num,
                                                                         grid_dim, block_dim, &perm);
        break;
      case 6:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse";
        sched = SUP_SCHED_CHUNKS, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse(
            mat, cptrs, rows, cvals, t, n, gpu_num, cpu, threads, grid_dim, block_dim, &perm);
        break;
      case 7:
        name = "gpu_perman64_xshared_coalescing_mshared_skipper";
        kern = SUP_KERNEL_SKIPPER;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_skipper(mat, rptrs, cols, cptrs, rows, cvals, t, n, grid_dim,
                                                                 block_dim, &perm);
        break;
      case 8:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper";
        kern = SUP_KERNEL_SKIPPER, sched = SUP_SCHED_CHUNKS, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper(
            mat, rptrs, cols, cptrs, rows, cvals, t, n, gpu_num, cpu, threads, grid_dim, block_dim, &perm);
        break;
      case 66:
        name = "gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution";
        sched = SUP_SCHED_MANUAL, g = gpu_num;
        rc = sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution(
            mat, cptrs, rows, cvals, t, n, gpu_num, grid_dim, block_dim, &perm);
        break;
      default: printf("Unknown Algorithm ID\n"); return 0;
    }
  }
  if (rc) return fail(rc);
  printf("Result: %s %.17e\n", name, perm);
  sup_opts o;
  sup_opts_init(&o);
  o.gpu_num = g;
  double check = 0.0;
  if ((rc = sup_perman(mat, t, n, kern, sched, &o, &check, NULL))) return fail(rc);
  printf("Check: %.17e\n", check);
  sup_free(mat);
  free(perm_r), free(perm_c), free(cptrs), free(rows), free(rptrs), free(cols), free(cvals), free(rvals);
  return 0;
}
