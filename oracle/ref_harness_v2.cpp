// ref_harness_v2.cpp — TEST INFRASTRUCTURE ONLY.
// Drives the reference's own v2 CPU algorithms, compiled unmodified from
// /root/reference/revised_perman (flags.h, cpu_algos.hpp, util.h) by
// oracle/Makefile into oracle/_ref/ref_v2.  Used only to generate the golden
// vectors in tests/golden/ (tests/golden/make_golden.py); never shipped.
//
// usage: ref_v2 <v1 matrix file> <algo> <threads> [binary 0|1] [preprocessing 0|1|2]
//   algo: dense    parallel_perman64<double,double>          cpu_algos.hpp:761
//         dense_q  parallel_perman64<__float128,double>      (reference -q mode)
//         sparse   parallel_perman64_sparse<double,double>   cpu_algos.hpp:635
//         skip     parallel_skip_perman64_w_balanced<double,double> cpu_algos.hpp:1035
//         order    print the preprocessed dense matrix (SortOrder/SkipOrder check)
#include "flags.h"
#include "cpu_algos.hpp"

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s file algo threads [binary] [prep]\n", argv[0]);
    return 2;
  }
  const std::string algo = argv[2];
  const int threads = std::atoi(argv[3]);
  const bool binary = argc > 4 && std::atoi(argv[4]) != 0;
  const int prep = argc > 5 ? std::atoi(argv[5]) : 0;
  std::ifstream in(argv[1]);
  std::string line, type;
  int n = 0, nnz = 0;
  std::getline(in, line);
  {
    std::istringstream iss(line);
    iss >> n >> nnz >> type;
  }
  DenseMatrix<double>* d = new DenseMatrix<double>();
  d->nov = n;
  d->mat = new double[n * n]();
  int cnt = 0;
  while (std::getline(in, line)) {
    std::istringstream iss(line);
    int i, j;
    double v;
    if (!(iss >> i >> j >> v)) continue;
    if (type == "int") v = (double)(int)v;
    if (type == "float") v = (double)(float)v;
    d->mat[i * n + j] = binary ? 1.0 : v;
  }
  for (int k = 0; k < n * n; ++k) cnt += d->mat[k] != 0;
  d->nnz = cnt;
  SparseMatrix<double>* s = new SparseMatrix<double>();
  s->nov = n;
  s->nnz = cnt;
  s->cptrs = new int[n + 1];
  s->rptrs = new int[n + 1];
  s->rows = new int[cnt];
  s->cols = new int[cnt];
  s->cvals = new double[cnt];
  s->rvals = new double[cnt];
  if (prep == 1) matrix2compressed_sortOrder_o(d, s);
  else if (prep == 2) matrix2compressed_skipOrder_o(d, s);
  else matrix2compressed_o(d, s);

  flags f;
  f.threads = threads;
  Result r;
  if (algo == "dense") r = parallel_perman64<double, double>(d, f);
  else if (algo == "dense_q") r = parallel_perman64<__float128, double>(d, f);
  else if (algo == "sparse") r = parallel_perman64_sparse<double, double>(d, s, f);
  else if (algo == "skip") r = parallel_skip_perman64_w_balanced<double, double>(s, f);
  else if (algo == "order") {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) std::printf("%.17g%c", d->mat[i * n + j], j + 1 == n ? '\n' : ' ');
    return 0;
  } else {
    std::fprintf(stderr, "unknown algo %s\n", algo.c_str());
    return 2;
  }
  std::printf("%.17e %f\n", r.permanent, r.time);
  return 0;
}
