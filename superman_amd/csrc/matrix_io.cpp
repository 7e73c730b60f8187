// matrix_io.cpp — host preprocessing on the hot path:
// v1 matrix reader, CSR/CSC, SortOrder, SkipOrder.
#include <algorithm>
#include <cctype>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <sstream>
#include <string>
#include <vector>

#include "engine.hpp"

namespace sup {

template <class T>
static T& at(void* m, int n, int i, int j) {
  return ((T*)m)[(size_t)i * n + j];
}

static double get(const void* m, sup_dtype t, int n, int i, int j) {
  switch (t) {
    case SUP_INT32: return (double)((const int32_t*)m)[(size_t)i * n + j];
    case SUP_FLOAT32: return (double)((const float*)m)[(size_t)i * n + j];
    default: return ((const double*)m)[(size_t)i * n + j];
  }
}

static size_t esize(sup_dtype t) { return t == SUP_FLOAT64 ? 8 : 4; }

}  // namespace sup

using namespace sup;

extern "C" {

// MatrixMarket coordinate reader: mmio banner checks as revised_perman/
// main.cpp:1522-1575, entries as read_matrix.hpp:11-157 (1-based, '%' lines
// skipped, symmetric / skew files mirrored with the same value, pattern or -b
// entries = 1, later duplicates overwrite earlier ones).
int sup_read_mtx(const char* path, int binary, void** mat, sup_dtype* t, int* n, int* nnz_lines) {
  if (!path || !mat || !t || !n) {
    set_error("null argument");
    return SUP_EINVAL;
  }
  std::ifstream in(path);
  if (!in) {
    set_error(std::string("cannot open matrix file ") + path);
    return SUP_EIO;
  }
  std::string line;
  if (!std::getline(in, line)) {
    set_error("empty matrix file");
    return SUP_EIO;
  }
  std::istringstream ban(line);
  std::string tag, object, format, field, symmetry;
  ban >> tag >> object >> format >> field >> symmetry;
  auto lower = [](std::string v) {
    for (auto& ch : v) ch = (char)std::tolower((unsigned char)ch);
    return v;
  };
  object = lower(object), format = lower(format), field = lower(field), symmetry = lower(symmetry);
  if (tag != "%%MatrixMarket") {
    set_error("Could not process Matrix Market Banner");
    return SUP_EIO;
  }
  if (object != "matrix") {
    set_error("SUPerman only supports matrices");
    return SUP_EIO;
  }
  if (format != "coordinate") {
    set_error("SUPerman only supports mtx (coordinate) format");
    return SUP_EIO;
  }
  if (field == "complex" || (field != "real" && field != "integer" && field != "pattern")) {
    set_error("unsupported MatrixMarket field '" + field + "' (real, integer or pattern)");
    return SUP_EIO;
  }
  const bool sym = symmetry == "symmetric" || symmetry == "skew-symmetric";
  if (!sym && symmetry != "general") {
    set_error("unsupported MatrixMarket symmetry '" + symmetry + "'");
    return SUP_EIO;
  }
  const bool pattern = field == "pattern";
  while (in.peek() == '%') std::getline(in, line);  // read_matrix.hpp:23
  long M = 0, N = 0, nz = 0;
  if (!(in >> M >> N >> nz)) {
    set_error("Matrix size cannot be read");
    return SUP_EIO;
  }
  if (M != N) {
    set_error("SUPerman only works with nxn matrices");
    return SUP_EIO;
  }
  if (M < 1 || M > SUP_MAX_READ_N || nz < 0) {
    set_error("matrix order " + std::to_string(M) + " outside [1, " + std::to_string(SUP_MAX_READ_N) + "]");
    return SUP_EIO;
  }
  const int nov = (int)M;
  const sup_dtype dt = (field == "real" && !binary) ? SUP_FLOAT64 : SUP_INT32;  // main.cpp:1589,1821
  void* m = std::calloc((size_t)nov * nov, esize(dt));
  if (!m) {
    set_error("out of host memory");
    return SUP_ENOMEM;
  }
  auto put = [&](int i, int j, double v) {
    if (dt == SUP_INT32) at<int32_t>(m, nov, i, j) = (int32_t)v;
    else at<double>(m, nov, i, j) = v;
  };
  for (long e = 0; e < nz; ++e) {
    long x, y;
    double v = 1.0;
    bool ok = (bool)(in >> x >> y);
    if (ok && !pattern) ok = (bool)(in >> v);
    if (!ok) {
      std::free(m);
      set_error("MatrixMarket file ends after " + std::to_string(e) + " of " + std::to_string(nz) + " entries");
      return SUP_EIO;
    }
    if (x < 1 || x > nov || y < 1 || y > nov) {
      std::free(m);
      set_error("entry (" + std::to_string(x) + "," + std::to_string(y) + ") outside the " + std::to_string(nov) +
                "x" + std::to_string(nov) + " matrix (1-based)");
      return SUP_EIO;
    }
    if (pattern || binary) v = 1.0;
    put((int)x - 1, (int)y - 1, v);
    if (sym && x != y) put((int)y - 1, (int)x - 1, v);
  }
  *mat = m;
  *t = dt;
  *n = nov;
  if (nnz_lines) *nnz_lines = (int)nz;
  return SUP_OK;
}

// util.h:343-358 ReadMatrix + main.cu:494-498 header parse.
int sup_read_matrix(const char* path, int binary, void** mat, sup_dtype* t, int* n, int* nnz_header) {
  if (!path || !mat || !t || !n) {
    set_error("null argument");
    return SUP_EINVAL;
  }
  std::ifstream in(path);
  if (!in) {
    set_error(std::string("cannot open matrix file ") + path);
    return SUP_EIO;
  }
  std::string line, type;
  int nov = 0, nnz = 0;
  if (!std::getline(in, line)) {
    set_error("empty matrix file");
    return SUP_EIO;
  }
  if (line.rfind("%%MatrixMarket", 0) == 0) {
    in.close();
    return sup_read_mtx(path, binary, mat, t, n, nnz_header);
  }
  {
    std::istringstream iss(line);
    iss >> nov >> nnz >> type;
  }
  if (nov < 1 || nov > SUP_MAX_N) {
    set_error("matrix order " + std::to_string(nov) + " outside [1, 64]");
    return SUP_EIO;
  }
  sup_dtype dt;
  if (type == "int") dt = SUP_INT32;
  else if (type == "float") dt = SUP_FLOAT32;
  else if (type == "double") dt = SUP_FLOAT64;
  else {
    set_error("unknown matrix type '" + type + "' (expected int, float or double)");
    return SUP_EIO;
  }
  void* m = std::calloc((size_t)nov * nov, esize(dt));
  if (!m) {
    set_error("out of host memory");
    return SUP_ENOMEM;
  }
  while (std::getline(in, line)) {
    std::istringstream iss(line);
    int i, j;
    bool ok;
    if (dt == SUP_INT32) {
      int v;
      ok = (bool)(iss >> i >> j >> v);
      if (ok && i >= 0 && i < nov && j >= 0 && j < nov) at<int32_t>(m, nov, i, j) = binary ? 1 : v;
    } else if (dt == SUP_FLOAT32) {
      float v;
      ok = (bool)(iss >> i >> j >> v);
      if (ok && i >= 0 && i < nov && j >= 0 && j < nov) at<float>(m, nov, i, j) = binary ? 1.0f : v;
    } else {
      double v;
      ok = (bool)(iss >> i >> j >> v);
      if (ok && i >= 0 && i < nov && j >= 0 && j < nov) at<double>(m, nov, i, j) = binary ? 1.0 : v;
    }
    if (!ok) continue;  // erroneous line (util.h:351)
    if (i < 0 || i >= nov || j < 0 || j >= nov) {
      std::free(m);
      set_error("entry (" + std::to_string(i) + "," + std::to_string(j) + ") outside the " + std::to_string(nov) +
                "x" + std::to_string(nov) + " matrix");
      return SUP_EIO;
    }
  }
  *mat = m;
  *t = dt;
  *n = nov;
  if (nnz_header) *nnz_header = nnz;
  return SUP_OK;
}

void sup_free(void* p) { std::free(p); }

int sup_count_nnz(const void* mat, sup_dtype t, int n, int* nnz) {
  if (!mat || !nnz || n < 1 || n > SUP_MAX_N) {
    set_error("bad argument");
    return SUP_EINVAL;
  }
  int c = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) c += get(mat, t, n, i, j) != 0.0;
  *nnz = c;
  return SUP_OK;
}

// util.h:522-551 (nonzero test != 0 instead of > 0).
int sup_compress(const void* mat, sup_dtype t, int n, int* cptrs, int* rows, void* cvals, int* rptrs, int* cols,
                 void* rvals) {
  if (!mat || !cptrs || !rows || !rptrs || !cols || n < 1 || n > SUP_MAX_N) {
    set_error("bad argument");
    return SUP_EINVAL;
  }
  const size_t es = esize(t);
  const char* base = (const char*)mat;
  int er = 0, ec = 0;
  for (int i = 0; i < n; ++i) {
    rptrs[i] = er;
    cptrs[i] = ec;
    for (int j = 0; j < n; ++j) {
      if (get(mat, t, n, i, j) != 0.0) {
        cols[er] = j;
        if (rvals) std::memcpy((char*)rvals + (size_t)er * es, base + ((size_t)i * n + j) * es, es);
        ++er;
      }
      if (get(mat, t, n, j, i) != 0.0) {
        rows[ec] = j;
        if (cvals) std::memcpy((char*)cvals + (size_t)ec * es, base + ((size_t)j * n + i) * es, es);
        ++ec;
      }
    }
  }
  rptrs[n] = er;
  cptrs[n] = ec;
  return SUP_OK;
}

static void permute(void* mat, sup_dtype t, int n, const int* rowperm, const int* colperm) {
  const size_t es = esize(t);
  std::vector<char> old((size_t)n * n * es);
  std::memcpy(old.data(), mat, old.size());
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c)
      std::memcpy((char*)mat + ((size_t)r * n + c) * es,
                  old.data() + ((size_t)(rowperm ? rowperm[r] : r) * n + colperm[c]) * es, es);
}

// util.h:553-619.  The reference sorts with qsort and the comparator
// `left.second > right.second`, which glibc's merge sort turns into a stable
// ascending sort; ties keep the original column order here by construction.
int sup_sort_order(void* mat, sup_dtype t, int n, int* colperm) {
  if (!mat || !colperm || n < 1 || n > SUP_MAX_N) {
    set_error("bad argument");
    return SUP_EINVAL;
  }
  std::vector<int> cnt(n, 0);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) cnt[j] += get(mat, t, n, i, j) != 0.0;
  std::vector<int> perm(n);
  std::iota(perm.begin(), perm.end(), 0);
  std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return cnt[a] < cnt[b]; });
  permute(mat, t, n, nullptr, perm.data());
  std::copy(perm.begin(), perm.end(), colperm);
  return SUP_OK;
}

// util.h:621-684.  Greedy: take the remaining column of minimum current degree
// (lowest index on ties), append its not-yet-visited rows in increasing order,
// decrement the degrees of every column those rows touch.  Rows never visited
// (empty rows — the reference leaves rowPerm uninitialised there) are appended
// in increasing order.
int sup_skip_order(void* mat, sup_dtype t, int n, int* rowperm, int* colperm) {
  if (!mat || !rowperm || !colperm || n < 1 || n > SUP_MAX_N) {
    set_error("bad argument");
    return SUP_EINVAL;
  }
  std::vector<int> degs(n, 0);
  std::vector<char> used(n, 0), visited(n, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) degs[j] += get(mat, t, n, i, j) != 0.0;
  int ri = 0;
  for (int j = 0; j < n; ++j) {
    int cur = -1, best = INT_MAX;
    for (int l = 0; l < n; ++l)
      if (!used[l] && degs[l] < best) {
        best = degs[l];
        cur = l;
      }
    used[cur] = 1;
    colperm[j] = cur;
    for (int l = 0; l < n; ++l) {
      if (get(mat, t, n, l, cur) != 0.0 && !visited[l]) {
        visited[l] = 1;
        rowperm[ri++] = l;
        for (int k = 0; k < n; ++k)
          if (get(mat, t, n, l, k) != 0.0 && !used[k]) degs[k]--;
      }
    }
  }
  for (int l = 0; l < n; ++l)
    if (!visited[l]) rowperm[ri++] = l;
  permute(mat, t, n, rowperm, colperm);
  return SUP_OK;
}

}  // extern "C"
