// Thread-count independence of the host runtime's threaded setup pieces (tests/test_host_threads.py):
// spd_inverse (pipelined Cholesky, cyclic triangular stages) against the serial column-by-column
// restatement, and the centroid grid's counting sort against a sequential one.  Prints one line per
// check; the test runs it under several PUCFEM_HOST_THREADS values and compares the lines.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "pucfem_host.hpp"

using namespace pucfem;

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// the serial inverse: Cholesky by columns, L^-1 by columns, W^T W by rows (the operation order the
// threaded version keeps)
static bool serial_inverse(std::vector<double>& A, i64 n) {
  for (i64 j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (i64 k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0)) return false;
    d = std::sqrt(d);
    A[j * n + j] = d;
    for (i64 i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (i64 k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / d;
    }
  }
  std::vector<double> Wt(n * n, 0.0);
  for (i64 j = 0; j < n; ++j) {
    double* w = Wt.data() + j * n;
    w[j] = 1.0 / A[j * n + j];
    for (i64 i = j + 1; i < n; ++i) {
      double s = 0.0;
      for (i64 k = j; k < i; ++k) s -= A[i * n + k] * w[k];
      w[i] = s / A[i * n + i];
    }
  }
  for (i64 i = 0; i < n; ++i)
    for (i64 j = 0; j <= i; ++j) {
      double s = 0.0;
      for (i64 k = i; k < n; ++k) s += Wt[i * n + k] * Wt[j * n + k];
      A[i * n + j] = s;
    }
  for (i64 i = 0; i < n; ++i)
    for (i64 j = 0; j < i; ++j) A[j * n + i] = A[i * n + j];
  return true;
}

int main() {
  for (i64 n : {1, 5, 64, 130, 700}) {
    std::mt19937_64 r(n);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::vector<double> B(n * n), A(n * n);
    for (auto& x : B) x = u(r);
    for (i64 i = 0; i < n; ++i)
      for (i64 j = 0; j < n; ++j) {
        double s = 0.0;
        for (i64 k = 0; k < n; ++k) s += B[i * n + k] * B[j * n + k];
        A[i * n + j] = s + (i == j ? 0.1 * n : 0.0);
      }
    std::vector<double> S = A;
    const bool ok = spd_inverse(A, n), oks = serial_inverse(S, n);
    std::printf("spd n=%ld ok=%d serial_equal=%d hash=%016llx\n", (long)n, ok ? 1 : 0,
                ok == oks && std::memcmp(A.data(), S.data(), sizeof(double) * n * n) == 0 ? 1 : 0,
                (unsigned long long)fnv(A.data(), sizeof(double) * n * n));
  }
  {
    std::vector<double> N = {1.0, 2.0, 2.0, 1.0};  // indefinite
    std::printf("spd indefinite ok=%d\n", spd_inverse(N, 2) ? 1 : 0);
  }
  for (i64 T : {1000, 300000}) {
    std::mt19937_64 r(T);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::vector<double> cx(T), cy(T);
    for (i64 t = 0; t < T; ++t) {
      cx[t] = u(r);
      cy[t] = 0.3 * u(r);
    }
    Grid G;
    build_centroid_grid(cx, cy, 2.0, G);
    // sequential counting sort of the same cells
    const i64 nc = (i64)G.nx * G.ny;
    std::vector<i32> start(nc + 1, 0), item(T);
    std::vector<i32> cell(T);
    for (i64 t = 0; t < T; ++t) {
      auto co = [](double v, double v0, double h, i32 m) {
        const double f = std::floor((v - v0) / h);
        return !(f >= 0) ? 0 : (f >= m ? m - 1 : (i32)f);
      };
      cell[t] = co(cy[t], G.y0, G.hy, G.ny) * G.nx + co(cx[t], G.x0, G.hx, G.nx);
      start[cell[t] + 1]++;
    }
    for (i64 c = 0; c < nc; ++c) start[c + 1] += start[c];
    std::vector<i32> fill(start.begin(), start.end() - 1);
    for (i64 t = 0; t < T; ++t) item[fill[cell[t]]++] = (i32)t;
    bool same = start == G.cell_start && item == G.item;
    for (i64 k = 0; k < T && same; ++k) same = G.px[k] == cx[G.item[k]] && G.py[k] == cy[G.item[k]];
    std::printf("grid T=%ld cells=%ld sequential_equal=%d hash=%016llx\n", (long)T, (long)nc, same ? 1 : 0,
                (unsigned long long)fnv(G.item.data(), sizeof(i32) * T, fnv(G.cell_start.data(), sizeof(i32) * (nc + 1))));
  }
  for (i64 nr : {50, 200000}) {  // transpose (the restriction of every level): against a sequential counting sort
    std::mt19937_64 r(nr);
    const i64 nc = nr / 3 + 1;
    Csr A;
    A.nrows = nr;
    A.rowptr.assign(nr + 1, 0);
    for (i64 i = 0; i < nr; ++i) {
      const int len = (int)(r() % 3);
      for (int k = 0; k < len; ++k) {
        A.col.push_back((i32)(r() % nc));
        A.val.push_back((double)(r() % 1000) / 7.0);
      }
      A.rowptr[i + 1] = (i64)A.col.size();
    }
    Csr T;
    transpose(A, nc, T);
    std::vector<i64> rp(nc + 1, 0);
    for (i32 c : A.col) rp[c + 1]++;
    for (i64 c = 0; c < nc; ++c) rp[c + 1] += rp[c];
    std::vector<i32> col(A.col.size());
    std::vector<double> val(A.col.size());
    std::vector<i64> fill(rp.begin(), rp.end() - 1);
    for (i64 i = 0; i < nr; ++i)
      for (i64 k = A.rowptr[i]; k < A.rowptr[i + 1]; ++k) {
        const i64 d = fill[A.col[k]]++;
        col[d] = (i32)i;
        val[d] = A.val[k];
      }
    const bool same = T.nrows == nc && T.rowptr == rp && T.col == col && T.val == val;
    std::printf("transpose rows=%ld nnz=%ld sequential_equal=%d\n", (long)nr, (long)A.col.size(), same ? 1 : 0);
  }
  return 0;
}
