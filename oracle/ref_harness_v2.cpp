// ref_harness_v2.cpp — TEST INFRASTRUCTURE ONLY.
// Drives the reference's own v2 CPU algorithms, compiled unmodified from
// /root/reference/revised_perman (flags.h, cpu_algos.hpp, util.h) by
// oracle/Makefile into oracle/_ref/ref_v2.  Used only to generate the golden
// vectors in tests/golden/ (tests/golden/make_golden.py); never shipped.
//
// usage: ref_v2 <matrix file> <algo> <threads> [binary 0|1] [preprocessing 0|1|2] [min_n] [scale]
//   matrix file: v1 format, or MatrixMarket (*.mtx, read by the reference's own
//         mmio.c banner parser + read_matrix.hpp readDenseMatrix /
//         readSymmetricDenseMatrix, as revised_perman/main.cpp:1515-1615)
//   algo: dense    parallel_perman64<double,double>          cpu_algos.hpp:761
//         dense_q  parallel_perman64<__float128,double>      (reference -q mode)
//         sparse   parallel_perman64_sparse<double,double>   cpu_algos.hpp:635
//         skip     parallel_skip_perman64_w_balanced<double,double> cpu_algos.hpp:1035
//         order    print the preprocessed dense matrix (SortOrder/SkipOrder check)
//         read     print the matrix as read (reader check)
//         reduce   -o / -u driver (main.cpp:993-1100, 1127-1259 restated below,
//                  dense leaves) over the reference's own d1compress /
//                  d2compress / d34compress / scalesk / scaleMatrix (util.h);
//                  prints "perm leaves"
//         leaves   the same, printing every leaf matrix instead of computing it
#include "flags.h"
#include "cpu_algos.hpp"
#include "read_matrix.hpp"
extern "C" {
#include "mmio.h"
}

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

// main.cpp:945-954 getNnz (lives in main.cpp, which does not build here)
int getNnz(const double* m, int n) {
  int c = 0;
  for (int i = 0; i < n * n; ++i) c += m[i] > 0.0;
  return c;
}

struct Reducer {
  flags f;
  int min_n = 30;
  double thr = -1.0;
  bool dump = false;
  int leaves = 0;

  void print(const double* m, int n) {
    std::printf("leaf %d\n", n);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) std::printf("%.17g%c", m[i * n + j], j + 1 == n ? '\n' : ' ');
  }
  // RunAlgo with the dense CPU algorithm on one matrix
  double run(double* m, int n) {
    ++leaves;
    if (dump) {  // leaves mode: the matrices only, no permanents
      print(m, n);
      return 0.0;
    }
    DenseMatrix<double> d;
    d.nov = n;
    d.mat = m;
    d.nnz = getNnz(m, n);
    Result r = parallel_perman64<double, double>(&d, f);
    d.mat = nullptr;
    return r.permanent;
  }
  // main.cpp:1229-1257 scale_and_calculate (double branch)
  double scaled(double* m, int n, bool compressing) {
    DenseMatrix<double> d;
    d.nov = n;
    d.mat = m;
    d.nnz = getNnz(m, n);
    SparseMatrix<double> s;
    s.nov = n;
    s.nnz = d.nnz;
    s.cptrs = new int[n + 1];
    s.rptrs = new int[n + 1];
    s.rows = new int[d.nnz];
    s.cols = new int[d.nnz];
    s.cvals = new double[d.nnz];
    s.rvals = new double[d.nnz];
    matrix2compressed_o(&d, &s);
    flags g = f;
    g.scaling_threshold = thr;
    ScaleCompanion<double>* sc = scalesk(&s, g);
    scaleMatrix(&d, sc);
    d.mat = nullptr;
    double v = compressing ? run(m, n) : singletons(m, n);
    for (int i = 0; i < n; ++i) v /= sc->c_v[i];
    for (int i = 0; i < n; ++i) v /= sc->r_v[i];
    return v;
  }
  // main.cpp:993-1063 compress_and_calculate_recursive
  double recurse(double* m, int n) {
    const int md = getMinNnz(m, n);
    if (md < 5 && n > min_n) {
      if (md == 1) {
        d1compress(m, n);
        return recurse(m, n);
      }
      if (md == 2) {
        d2compress(m, n);
        return recurse(m, n);
      }
      if (md == 3 || md == 4) {
        double* m2 = nullptr;
        int n2 = 0;
        d34compress(m, n, m2, n2, md);
        const double left = recurse(m, n);
        const double v = left + recurse(m2, n2);
        delete[] m2;
        return v;
      }
      return 0.0;
    }
    return thr > 0 ? scaled(m, n, true) : run(m, n);
  }
  // main.cpp:1065-1100 compress_singleton_and_then_recurse
  double singletons(double* m, int n) {
    bool comp = true;
    while (comp && n > 1) {
      comp = d1compress(m, n);
      if (!comp) comp = d2compress(m, n);
      if (comp && checkEmpty(m, n)) return 0.0;
    }
    return recurse(m, n);
  }
};

// main.cpp:1515-1615: mmio banner + readDenseMatrix / readSymmetricDenseMatrix
bool read_mtx(const char* path, bool binary, DenseMatrix<double>* d) {
  FILE* fp = std::fopen(path, "r");
  if (!fp) return false;
  MM_typecode code;
  int M, N, nz;
  if (mm_read_banner(fp, &code) != 0 || !mm_is_matrix(code) || !mm_is_coordinate(code) ||
      mm_read_mtx_crd_size(fp, &M, &N, &nz) != 0 || M != N || mm_is_complex(code)) {
    std::fclose(fp);
    return false;
  }
  std::fclose(fp);
  const bool pattern = mm_is_pattern(code), sym = mm_is_symmetric(code) || mm_is_skew(code);
  d->nov = M;
  if (sym) readSymmetricDenseMatrix(d, path, pattern, binary);
  else readDenseMatrix(d, path, pattern, binary);
  // integer / pattern files are DenseMatrix<int> in the reference (main.cpp:1821)
  if (!mm_is_real(code) || pattern || binary)
    for (int k = 0; k < M * M; ++k) d->mat[k] = (double)(int)d->mat[k];
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s file algo threads [binary] [prep]\n", argv[0]);
    return 2;
  }
  const std::string algo = argv[2];
  const int threads = std::atoi(argv[3]);
  const bool binary = argc > 4 && std::atoi(argv[4]) != 0;
  const int prep = argc > 5 ? std::atoi(argv[5]) : 0;
  const std::string path = argv[1];
  DenseMatrix<double>* d = new DenseMatrix<double>();
  int n = 0, cnt = 0;
  if (path.size() > 4 && path.compare(path.size() - 4, 4, ".mtx") == 0) {
    if (!read_mtx(argv[1], binary, d)) {
      std::fprintf(stderr, "cannot read MatrixMarket file %s\n", argv[1]);
      return 2;
    }
    n = d->nov;
  } else {
    std::ifstream in(argv[1]);
    std::string line, type;
    int nnz = 0;
    std::getline(in, line);
    {
      std::istringstream iss(line);
      iss >> n >> nnz >> type;
    }
    d->nov = n;
    d->mat = new double[n * n]();
    while (std::getline(in, line)) {
      std::istringstream iss(line);
      int i, j;
      double v;
      if (!(iss >> i >> j >> v)) continue;
      if (type == "int") v = (double)(int)v;
      if (type == "float") v = (double)(float)v;
      d->mat[i * n + j] = binary ? 1.0 : v;
    }
  }
  if (algo == "read") {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) std::printf("%.17g%c", d->mat[i * n + j], j + 1 == n ? '\n' : ' ');
    return 0;
  }
  if (algo == "reduce" || algo == "leaves") {
    Reducer R;
    R.f.threads = threads;
    R.min_n = argc > 6 ? std::atoi(argv[6]) : 30;
    R.thr = argc > 7 ? std::atof(argv[7]) : -1.0;
    R.dump = algo == "leaves";
    std::vector<double> m(d->mat, d->mat + n * n);
    // main.cpp:1640-1660: -u scales first (then -o), -o alone compresses
    const double v = R.thr > 0 ? R.scaled(m.data(), n, false) : R.singletons(m.data(), n);
    std::printf("%.17e %d\n", v, R.leaves);
    return 0;
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
