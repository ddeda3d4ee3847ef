// Host-side runtime of libpucfem (see pucfem_host.hpp).  Built with -ffp-contract=off so the
// assembly arithmetic is the reference's, operation for operation.
#include "pucfem_host.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <numeric>
#include <stdexcept>
#include <mutex>
#include <thread>

namespace pucfem {

// ----------------------------------------------------------------------------- refinement
void red_refine(const HostMesh& in, HostMesh& out, std::vector<i32>* edge_a, std::vector<i32>* edge_b) {
  const i64 N = in.N, T = in.T;
  // bucket every edge (a<b) under a, with multiplicity
  std::vector<i64> bptr(N + 1, 0);
  for (i64 t = 0; t < T; ++t)
    for (int e = 0; e < 3; ++e) {
      i32 a = in.tri[3 * t + e], b = in.tri[3 * t + (e + 1) % 3];
      bptr[std::min(a, b) + 1]++;
    }
  for (i64 i = 0; i < N; ++i) bptr[i + 1] += bptr[i];
  std::vector<i32> bval(bptr[N]);
  {
    std::vector<i64> fill(bptr.begin(), bptr.end() - 1);
    for (i64 t = 0; t < T; ++t)
      for (int e = 0; e < 3; ++e) {
        i32 a = in.tri[3 * t + e], b = in.tri[3 * t + (e + 1) % 3];
        bval[fill[std::min(a, b)]++] = std::max(a, b);
      }
  }
  // unique edges per bucket, with their multiplicity (buckets are independent: sort and count in
  // parallel, then a prefix sum gives every bucket its edge ids)
  std::vector<i64> eptr(N + 1, 0);
  parallel_for(N, [&](i64 a0, i64 a1) {
    for (i64 a = a0; a < a1; ++a) {
      auto s = bval.begin() + bptr[a], e = bval.begin() + bptr[a + 1];
      std::sort(s, e);  // duplicates stay: their count is the edge's multiplicity
      i64 d = 0;
      for (auto it = s; it != e; ++it)
        if (it == s || *it != *(it - 1)) ++d;
      eptr[a + 1] = d;
    }
  });
  for (i64 a = 0; a < N; ++a) eptr[a + 1] += eptr[a];
  const i64 E = eptr[N];
  std::vector<i32> eb(E);
  std::vector<uint8_t> emult(E);
  parallel_for(N, [&](i64 a0, i64 a1) {
    for (i64 a = a0; a < a1; ++a) {
      auto s = bval.begin() + bptr[a], e = bval.begin() + bptr[a + 1];
      i64 k = eptr[a];
      for (auto it = s; it != e;) {
        auto j = it;
        while (j != e && *j == *it) ++j;
        eb[k] = *it;
        emult[k] = (uint8_t)std::min<i64>(255, j - it);
        ++k;
        it = j;
      }
    }
  });
  auto edge_id = [&](i32 a, i32 b) -> i64 {
    if (a > b) std::swap(a, b);
    auto s = eb.begin() + eptr[a], e = eb.begin() + eptr[a + 1];
    auto it = std::lower_bound(s, e, b);
    return it - eb.begin();
  };
  out.N = N + E;
  out.T = 4 * T;
  out.fp32 = in.fp32;
  out.x.resize(out.N);
  out.y.resize(out.N);
  out.mk.resize(out.N);
  std::copy(in.x.begin(), in.x.end(), out.x.begin());
  std::copy(in.y.begin(), in.y.end(), out.y.begin());
  std::copy(in.mk.begin(), in.mk.end(), out.mk.begin());
  parallel_for(N, [&](i64 a0, i64 a1) {
    for (i64 a = a0; a < a1; ++a)
      for (i64 k = eptr[a]; k < eptr[a + 1]; ++k) {
        i32 b = eb[k];
        i64 n = N + k;
        out.x[n] = (in.x[a] + in.x[b]) * 0.5;
        out.y[n] = (in.y[a] + in.y[b]) * 0.5;
        if (emult[k] == 1)  // boundary edge: midpoint stays on the boundary segment
          out.mk[n] = (in.mk[a] == 2 && in.mk[b] == 2) ? 2 : 1;
        else
          out.mk[n] = 0;
      }
  });
  if (edge_a && edge_b) {
    edge_a->resize(E);
    edge_b->resize(E);
    parallel_for(N, [&](i64 a0, i64 a1) {
      for (i64 a = a0; a < a1; ++a)
        for (i64 k = eptr[a]; k < eptr[a + 1]; ++k) {
          (*edge_a)[k] = (i32)a;
          (*edge_b)[k] = eb[k];
        }
    });
  }
  out.tri.resize(3 * out.T);
  parallel_for(T, [&](i64 t0, i64 t1) {
    for (i64 t = t0; t < t1; ++t) {
      i32 a = in.tri[3 * t], b = in.tri[3 * t + 1], c = in.tri[3 * t + 2];
      i32 ab = (i32)(N + edge_id(a, b)), bc = (i32)(N + edge_id(b, c)), ca = (i32)(N + edge_id(c, a));
      const i32 ch[12] = {a, ab, ca, ab, b, bc, ca, bc, c, ab, bc, ca};
      std::copy(ch, ch + 12, out.tri.begin() + 12 * t);
    }
  });
}

// ----------------------------------------------------------------------------- ordering
// sqrt(N)/2 strips of equal node count: a strip is ~2 node spacings high and 2 sqrt(N) nodes long,
// so a stiffness neighbour lies within one strip of its row and a periodic master's columns (its
// slave's neighbours, at the far end of the same or the next strip) within two -- a band of
// ~4 sqrt(N) that fits int16 column deltas up to the ~10M-node meshes (L7: ~15k)
int auto_strips(i64 N) { return (int)std::max<i64>(1, std::llround(std::sqrt((double)N) / 2.0)); }

void make_ordering(const HostMesh& m, int nstrips, Ordering& ord) {
  const i64 N = m.N;
  const int S = nstrips > 0 ? nstrips : auto_strips(N);
  std::vector<double> ys(m.y.begin(), m.y.end());
  std::sort(ys.begin(), ys.end());
  std::vector<double> cuts;
  for (int s = 1; s < S; ++s) {
    // first distinct-value boundary at or after the equal-count target
    i64 k = std::max<i64>(1, (i64)((double)N * s / S));
    while (k < N && ys[k] == ys[k - 1]) ++k;
    if (k >= N) break;
    const double c = 0.5 * (ys[k - 1] + ys[k]);
    if (cuts.empty() || c > cuts.back()) cuts.push_back(c);
  }
  make_ordering_cuts(m, cuts, ord);
}

void make_ordering_cuts(const HostMesh& m, const std::vector<double>& cuts, Ordering& ord) {
  const i64 N = m.N;
  const int S = (int)cuts.size() + 1;
  ord.cuts = cuts;
  std::vector<i32> strip(N);
  for (i64 i = 0; i < N; ++i) strip[i] = (i32)(std::upper_bound(cuts.begin(), cuts.end(), m.y[i]) - cuts.begin());
  ord.new2old.resize(N);
  std::iota(ord.new2old.begin(), ord.new2old.end(), 0);
  std::sort(ord.new2old.begin(), ord.new2old.end(), [&](i32 a, i32 b) {
    if (strip[a] != strip[b]) return strip[a] < strip[b];
    if (m.x[a] != m.x[b]) return m.x[a] < m.x[b];
    if (m.y[a] != m.y[b]) return m.y[a] < m.y[b];
    return a < b;
  });
  ord.old2new.assign(N, 0);
  for (i64 i = 0; i < N; ++i) ord.old2new[ord.new2old[i]] = (i32)i;
  ord.strip_ptr.assign(S + 1, 0);
  for (i64 i = 0; i < N; ++i) ord.strip_ptr[strip[i] + 1]++;
  for (int s = 0; s < S; ++s) ord.strip_ptr[s + 1] += ord.strip_ptr[s];
}

// ----------------------------------------------------------------------------- pattern
// node -> incident triangles (internal node ids), triangles in ascending order per node
void build_incidence(const HostMesh& m, const Ordering& ord, Incidence& I) {
  std::vector<i64>& ptr = I.ptr;
  std::vector<i32>& tri = I.tri;
  const i64 N = m.N, T = m.T;
  ptr.assign(N + 1, 0);
  for (i64 q = 0; q < 3 * T; ++q) ++ptr[ord.old2new[m.tri[q]] + 1];
  for (i64 i = 0; i < N; ++i) ptr[i + 1] += ptr[i];
  tri.resize(ptr[N]);
  // fill with atomic cursors (any order), then sort every node's list: ascending triangle ids
  std::vector<std::atomic<i64>> cur(N);
  parallel_for(N, [&](i64 a, i64 b) {
    for (i64 i = a; i < b; ++i) cur[i].store(ptr[i], std::memory_order_relaxed);
  });
  parallel_for(T, [&](i64 t0, i64 t1) {
    for (i64 t = t0; t < t1; ++t)
      for (int i = 0; i < 3; ++i) tri[cur[ord.old2new[m.tri[3 * t + i]]].fetch_add(1, std::memory_order_relaxed)] = (i32)t;
  });
  parallel_for(N, [&](i64 a, i64 b) {
    for (i64 i = a; i < b; ++i) std::sort(tri.begin() + ptr[i], tri.begin() + ptr[i + 1]);
  });
}

void build_pattern(const HostMesh& m, const Ordering& ord, Csr& P, const Incidence* inc) {
  const i64 N = m.N;
  Incidence own;
  if (!inc) {
    build_incidence(m, ord, own);
    inc = &own;
  }
  const std::vector<i64>& iptr = inc->ptr;
  const std::vector<i32>& itri = inc->tri;
  // rows are independent: each chunk gathers, sorts and dedups its rows, then the chunks are
  // concatenated in row order
  std::vector<std::vector<i32>> ccol(PAR_CHUNKS);
  std::vector<std::vector<i64>> clen(PAR_CHUNKS);
  parallel_chunks(N, [&](int ch, i64 r0, i64 r1) {
    std::vector<i32>& out = ccol[ch];
    std::vector<i64>& len = clen[ch];
    std::vector<i32> tmp;
    for (i64 r = r0; r < r1; ++r) {
      tmp.clear();
      for (i64 e = iptr[r]; e < iptr[r + 1]; ++e) {
        const i64 t = itri[e];
        for (int j = 0; j < 3; ++j) tmp.push_back(ord.old2new[m.tri[3 * t + j]]);
      }
      std::sort(tmp.begin(), tmp.end());
      tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
      if (tmp.empty()) tmp.push_back((i32)r);  // isolated node: keep a diagonal entry
      out.insert(out.end(), tmp.begin(), tmp.end());
      len.push_back((i64)tmp.size());
    }
  });
  P.nrows = N;
  P.rowptr.assign(N + 1, 0);
  i64 r = 0;
  for (int ch = 0; ch < PAR_CHUNKS; ++ch)
    for (i64 l : clen[ch]) {
      P.rowptr[r + 1] = P.rowptr[r] + l;
      ++r;
    }
  host_alloc_fresh(P.col, P.rowptr[N]);
  std::vector<i64> cstart(PAR_CHUNKS + 1, 0);
  for (int ch = 0; ch < PAR_CHUNKS; ++ch) cstart[ch + 1] = cstart[ch] + (i64)ccol[ch].size();
  parallel_for(PAR_CHUNKS, [&](i64 c0, i64 c1) {
    for (i64 ch = c0; ch < c1; ++ch) std::copy(ccol[ch].begin(), ccol[ch].end(), P.col.begin() + cstart[ch]);
  }, 1);
}

// ----------------------------------------------------------------------------- assembly
// Row-parallel: every row gathers the contributions of its incident triangles in ascending triangle
// order, which is the order the reference's scatter loop (StokesColor.py:98-128, :224-284) adds them
// to each entry -- the values are the sequential scatter's, bit for bit.
void assemble_stokes(const HostMesh& m, const Ordering& ord, const Csr& P, Assembly& A, const Incidence* inc) {
  const i64 N = m.N, nnz = P.nnz();
  A.K.assign(nnz, 0.0);
  A.Gx.assign(nnz, 0.0);
  A.Gy.assign(nnz, 0.0);
  A.M.assign(N, 0.0);
  A.asum.assign(N, 0.0);
  Incidence own;
  if (!inc) {
    build_incidence(m, ord, own);
    inc = &own;
  }
  const std::vector<i64>& iptr = inc->ptr;
  const std::vector<i32>& itri = inc->tri;
  parallel_for(N, [&](i64 r0, i64 r1) {
    for (i64 r = r0; r < r1; ++r) {
      const i64 b = P.rowptr[r], e = P.rowptr[r + 1];
      auto pos = [&](i32 col) {
        const auto it = std::lower_bound(P.col.begin() + b, P.col.begin() + e, col);
        return (i64)(it - P.col.begin());
      };
      for (i64 q = iptr[r]; q < iptr[r + 1]; ++q) {
        const i64 t = itri[q];
        const i32 o[3] = {m.tri[3 * t], m.tri[3 * t + 1], m.tri[3 * t + 2]};
        const i32 n[3] = {ord.old2new[o[0]], ord.old2new[o[1]], ord.old2new[o[2]]};
        const double x1 = m.x[o[0]], y1 = m.y[o[0]], x2 = m.x[o[1]], y2 = m.y[o[1]], x3 = m.x[o[2]],
                     y3 = m.y[o[2]];
        // StokesColor.py:277-283 (buildLumpedMassMatrix): no degenerate skip
        const double det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2);
        const double area = 0.5 * std::fabs(det);
        for (int i = 0; i < 3; ++i)
          if (n[i] == r) A.M[r] += area / 3.0;
        if (std::fabs(det) < 1e-14) continue;  // StokesColor.py:113, :146, :239
        const double yd[3] = {y2 - y3, y3 - y1, y1 - y2};
        const double xd[3] = {x3 - x2, x1 - x3, x2 - x1};
        const double den = 2 * std::fabs(det);
        const double inv2A = 1.0 / det;  // StokesColor.py:149 / :241
        const double a3 = area / 3.0;
        for (int i = 0; i < 3; ++i) {
          if (n[i] != r) continue;
          A.asum[r] += a3;
          for (int j = 0; j < 3; ++j) {
            const i64 k = pos(n[j]);
            A.K[k] += (yd[i] * yd[j] + xd[i] * xd[j]) / den;  // StokesColor.py:120-126
            A.Gx[k] += (yd[j] * inv2A) * a3;
            A.Gy[k] += (xd[j] * inv2A) * a3;
          }
        }
      }
    }
  });
}

namespace {
using Row = std::vector<std::pair<i32, double>>;
void row_add(Row& dst, const Row& src) {  // dst[c] = dst[c] + src[c] (poisson.py:204)
  Row out;
  out.reserve(dst.size() + src.size());
  size_t i = 0, j = 0;
  while (i < dst.size() || j < src.size()) {
    if (j == src.size() || (i < dst.size() && dst[i].first < src[j].first)) out.push_back(dst[i++]);
    else if (i == dst.size() || src[j].first < dst[i].first) out.push_back(src[j++]);
    else {
      out.push_back({dst[i].first, dst[i].second + src[j].second});
      ++i, ++j;
    }
  }
  dst.swap(out);
}
}  // namespace

void assemble_literal(const HostMesh& m, const Ordering& ord, const std::vector<float>& g_tri,
                      const std::vector<std::pair<i64, i64>>& op_pairs_old,
                      const std::vector<i32>& dir_nodes_old, const std::vector<double>& dir_vals,
                      double heat_dt, Csr& out, std::vector<double>& b) {
  const i64 N = m.N, T = m.T;
  std::vector<Row> rows(N);
  b.assign(N, 0.0);
  std::vector<std::map<i32, double>> acc(N);
  // poisson.py:105-144 -- fp32 element arithmetic, fp64 accumulation in triangle order
  for (i64 t = 0; t < T; ++t) {
    const i32 o[3] = {m.tri[3 * t], m.tri[3 * t + 1], m.tri[3 * t + 2]};
    const float x1 = (float)m.x[o[0]], y1 = (float)m.y[o[0]], x2 = (float)m.x[o[1]],
                y2 = (float)m.y[o[1]], x3 = (float)m.x[o[2]], y3 = (float)m.y[o[2]];
    const float ADet = x1 * y2 - x1 * y3 - x2 * y1 + x2 * y3 + x3 * y1 - x3 * y2;
    if (ADet == 0.0f) continue;
    const float yd[3] = {y2 - y3, y3 - y1, y1 - y2};
    const float xd[3] = {x3 - x2, x1 - x3, x2 - x1};
    const float den = 2.0f * ADet;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const float v = (yd[i] * yd[j] + xd[i] * xd[j]) / den;
        acc[ord.old2new[o[i]]][ord.old2new[o[j]]] += (double)v;
      }
    const float area = 0.5f * ADet;
    const float s = (g_tri.empty() ? 0.0f : g_tri[t]) * (area / 3.0f);
    for (int i = 0; i < 3; ++i) b[ord.old2new[o[i]]] += (double)s;
  }
  for (i64 r = 0; r < N; ++r) {
    rows[r].assign(acc[r].begin(), acc[r].end());
    b[r] = -b[r];  // poisson.py:146 returns -BVector
  }
  acc.clear();
  // poisson.py:202-213 periodic row merge, sequential
  for (auto& pr : op_pairs_old) {
    const i32 mi = ord.old2new[pr.first], si = ord.old2new[pr.second];
    row_add(rows[mi], rows[si]);
    b[mi] += b[si];
    rows[si].clear();
    if (si < mi) rows[si] = {{si, 1.0}, {mi, -1.0}};
    else rows[si] = {{mi, -1.0}, {si, 1.0}};
    b[si] = 0.0;
  }
  // poisson.py:258-278 Dirichlet rows (columns kept)
  for (size_t k = 0; k < dir_nodes_old.size(); ++k) {
    const i32 i = ord.old2new[dir_nodes_old[k]];
    rows[i] = {{i, 1.0}};
    b[i] = dir_vals[k];
  }
  if (heat_dt > 0) {  // heatEq.py:305  A <- I + DT*A
    for (i64 r = 0; r < N; ++r) {
      bool diag = false;
      for (auto& e : rows[r]) {
        e.second = heat_dt * e.second;
        if (e.first == r) {
          e.second = 1.0 + e.second;
          diag = true;
        }
      }
      if (!diag) {
        rows[r].push_back({(i32)r, 1.0});
        std::sort(rows[r].begin(), rows[r].end());
      }
    }
  }
  out.nrows = N;
  out.rowptr.assign(N + 1, 0);
  out.col.clear();
  out.val.clear();
  for (i64 r = 0; r < N; ++r) {
    for (auto& e : rows[r]) {
      out.col.push_back(e.first);
      out.val.push_back(e.second);
    }
    out.rowptr[r + 1] = (i64)out.col.size();
  }
}

void build_pressure(const Csr& P, const std::vector<double>& K, const std::vector<i32>& dof,
                    const std::vector<i32>& slave_of, Csr& Pp) {
  const i64 N = P.nrows;
  // row r of the merged operator: a slave's identity row, or the master row plus its slave's row with the
  // columns mapped to their dofs, stably sorted by column and duplicates combined in insertion order.
  // Rows are independent: one pass counts them, the second writes them in place (parallel both).
  auto merge_row = [&](i64 r, std::vector<std::pair<i32, double>>& tmp) {
    tmp.clear();
    if (dof[r] != r) {  // slave: identity row, decoupled
      tmp.push_back({(i32)r, 1.0});
      return;
    }
    auto add_row = [&](i64 src) {
      for (i64 k = P.rowptr[src]; k < P.rowptr[src + 1]; ++k) tmp.push_back({dof[P.col[k]], K[k]});
    };
    add_row(r);
    if (slave_of[r] >= 0) add_row(slave_of[r]);
    std::stable_sort(tmp.begin(), tmp.end(),
                     [](const std::pair<i32, double>& a, const std::pair<i32, double>& b) { return a.first < b.first; });
    size_t w = 0;
    for (size_t k = 0; k < tmp.size(); ++k) {
      if (w > 0 && tmp[w - 1].first == tmp[k].first) tmp[w - 1].second += tmp[k].second;
      else tmp[w++] = tmp[k];
    }
    tmp.resize(w);
  };
  Pp.nrows = N;
  Pp.rowptr.assign(N + 1, 0);
  parallel_for(N, [&](i64 r0, i64 r1) {
    std::vector<std::pair<i32, double>> tmp;
    for (i64 r = r0; r < r1; ++r) {
      merge_row(r, tmp);
      Pp.rowptr[r + 1] = (i64)tmp.size();
    }
  });
  for (i64 r = 0; r < N; ++r) Pp.rowptr[r + 1] += Pp.rowptr[r];
  host_alloc_fresh(Pp.col, Pp.rowptr[N]);
  host_alloc_fresh(Pp.val, Pp.rowptr[N]);
  parallel_for(N, [&](i64 r0, i64 r1) {
    std::vector<std::pair<i32, double>> tmp;
    for (i64 r = r0; r < r1; ++r) {
      merge_row(r, tmp);
      i64 o = Pp.rowptr[r];
      for (const auto& e : tmp) {
        Pp.col[o] = e.first;
        Pp.val[o] = e.second;
        ++o;
      }
    }
  });
}

// ----------------------------------------------------------------------------- partition
void partition_rows(const Csr& P, const Ordering& ord, int world, std::vector<i64>& row_start) {
  const i64 S = (i64)ord.strip_ptr.size() - 1;
  if (world < 1 || world > S) throw std::runtime_error("world size exceeds the number of y-strips");
  row_start.assign(world + 1, 0);
  row_start[world] = P.nrows;
  const double total = (double)P.nnz();
  i64 prev = 0;  // previous cut, as a strip index
  for (int r = 1; r < world; ++r) {
    const double target = total * r / world;
    // first strip boundary past `prev` whose prefix nnz reaches the target, leaving at
    // least one strip for every remaining rank
    i64 c = prev + 1;
    while (c < S - (world - r) && (double)P.rowptr[ord.strip_ptr[c]] < target) ++c;
    if (c > prev + 1 && (double)P.rowptr[ord.strip_ptr[c]] - target >
                            target - (double)P.rowptr[ord.strip_ptr[c - 1]])
      --c;  // the boundary just before is closer to the target
    row_start[r] = ord.strip_ptr[c];
    prev = c;
  }
}

i32 to_local(const LocalPlan& lp, i32 g) {
  if (g >= lp.r0 && g < lp.r1) return (i32)(g - lp.r0);
  auto it = std::lower_bound(lp.ghost_global.begin(), lp.ghost_global.end(), g);
  if (it == lp.ghost_global.end() || *it != g) throw std::runtime_error("column not in ghost set");
  return (i32)(lp.n_own + (it - lp.ghost_global.begin()));
}

void make_local_plan(const std::vector<const Csr*>& pats, const std::vector<i64>& row_start, int rank,
                     LocalPlan& lp) {
  const int world = (int)row_start.size() - 1;
  lp.r0 = row_start[rank];
  lp.r1 = row_start[rank + 1];
  lp.n_own = lp.r1 - lp.r0;
  auto owner = [&](i64 g) {
    return (i32)(std::upper_bound(row_start.begin(), row_start.end(), g) - row_start.begin() - 1);
  };
  std::vector<i32> gh;
  for (auto* P : pats)
    for (i64 r = lp.r0; r < lp.r1; ++r)
      for (i64 k = P->rowptr[r]; k < P->rowptr[r + 1]; ++k)
        if (P->col[k] < lp.r0 || P->col[k] >= lp.r1) gh.push_back(P->col[k]);
  std::sort(gh.begin(), gh.end());
  gh.erase(std::unique(gh.begin(), gh.end()), gh.end());
  lp.ghost_global = gh;
  lp.n_ghost = (i64)gh.size();
  lp.ghost_owner.resize(gh.size());
  for (size_t k = 0; k < gh.size(); ++k) lp.ghost_owner[k] = owner(gh[k]);
  lp.recv_peer.clear();
  lp.recv_off.clear();
  lp.recv_cnt.clear();
  for (size_t k = 0; k < gh.size(); ++k) {
    if (lp.recv_peer.empty() || lp.recv_peer.back() != lp.ghost_owner[k]) {
      lp.recv_peer.push_back(lp.ghost_owner[k]);
      lp.recv_off.push_back((i64)k);
      lp.recv_cnt.push_back(0);
    }
    lp.recv_cnt.back()++;
  }
  // send lists: what every other rank q needs from my rows (its ghosts inside [r0, r1))
  lp.send_peer.clear();
  lp.send_off.clear();
  lp.send_cnt.clear();
  lp.send_local.clear();
  for (int q = 0; q < world; ++q) {
    if (q == rank) continue;
    std::vector<i32> need;
    for (auto* P : pats)
      for (i64 r = row_start[q]; r < row_start[q + 1]; ++r)
        for (i64 k = P->rowptr[r]; k < P->rowptr[r + 1]; ++k)
          if (P->col[k] >= lp.r0 && P->col[k] < lp.r1) need.push_back(P->col[k]);
    if (need.empty()) continue;
    std::sort(need.begin(), need.end());
    need.erase(std::unique(need.begin(), need.end()), need.end());
    lp.send_peer.push_back(q);
    lp.send_off.push_back((i64)lp.send_local.size());
    lp.send_cnt.push_back((i64)need.size());
    for (i32 g : need) lp.send_local.push_back((i32)(g - lp.r0));
  }
}

// ----------------------------------------------------------------------------- SELL-64
void build_sell(const Csr& A, const LocalPlan& lp, Sell& S) {
  const i64 n = lp.n_own;
  S.nrows = n;
  S.nslices = (n + 63) / 64;
  S.slice_off.assign(S.nslices + 1, 0);
  S.slice_w.assign(S.nslices, 0);
  for (i64 s = 0; s < S.nslices; ++s) {
    i64 w = 0;
    for (i64 l = 0; l < 64; ++l) {
      i64 r = s * 64 + l;
      if (r < n) w = std::max(w, A.rowptr[lp.r0 + r + 1] - A.rowptr[lp.r0 + r]);
    }
    S.slice_w[s] = (i32)w;
    S.slice_off[s + 1] = S.slice_off[s] + w * 64;
  }
  S.padded = S.slice_off[S.nslices];
  S.col.assign(S.padded, 0);
  for (i64 s = 0; s < S.nslices; ++s)
    for (i64 l = 0; l < 64; ++l) {
      i64 r = s * 64 + l;
      i64 len = r < n ? A.rowptr[lp.r0 + r + 1] - A.rowptr[lp.r0 + r] : 0;
      for (i64 k = 0; k < S.slice_w[s]; ++k) {
        i32 c = r < n ? (k < len ? to_local(lp, A.col[A.rowptr[lp.r0 + r] + k]) : (i32)r) : 0;
        S.col[S.slice_off[s] + k * 64 + l] = c;
      }
    }
}

bool sell_col16(const Sell& S, i64 nloc, std::vector<int16_t>& out) {
  std::vector<int16_t> o(S.padded, 0);
  for (i64 s = 0; s < S.nslices; ++s)
    for (i64 l = 0; l < 64; ++l) {
      if (s * 64 + l >= S.nrows) continue;
      for (i64 k = 0; k < S.slice_w[s]; ++k) {
        const i64 e = S.slice_off[s] + k * 64 + l;
        i64 d = (i64)S.col[e] - s * 64;
        if (d > INT16_MAX) d -= nloc;  // decoded as base + d + nloc (base + d < 0)
        if (d < INT16_MIN || d > INT16_MAX) return false;
        o[e] = (int16_t)d;
      }
    }
  out.swap(o);
  return true;
}

void sell_values(const Csr& A, const LocalPlan& lp, const Sell& S, const std::vector<double>& val,
                 std::vector<double>& out) {
  if (!S.rows.empty()) return sell_values_rows(A, lp.r0, S, val, out);
  out.assign(S.padded, 0.0);
  parallel_for(S.nslices, [&](i64 s0, i64 s1) {
    for (i64 s = s0; s < s1; ++s)
      for (i64 l = 0; l < 64; ++l) {
        i64 r = s * 64 + l;
        if (r >= S.nrows) continue;
        i64 b = A.rowptr[lp.r0 + r], len = A.rowptr[lp.r0 + r + 1] - b;
        for (i64 k = 0; k < len; ++k) out[S.slice_off[s] + k * 64 + l] = val[b + k];
      }
  }, 64);
}

// ----------------------------------------------------------------------------- grids
static void grid_dims(double xmin, double xmax, double ymin, double ymax, i64 nitems, double per_cell, Grid& G) {
  double w = std::max(xmax - xmin, 1e-300), h = std::max(ymax - ymin, 1e-300);
  double ncell = std::max(1.0, (double)nitems / per_cell);
  double cs = std::sqrt(w * h / ncell);
  G.nx = (i32)std::max(1.0, std::min(32768.0, std::ceil(w / cs)));
  G.ny = (i32)std::max(1.0, std::min(32768.0, std::ceil(h / cs)));
  G.x0 = xmin;
  G.y0 = ymin;
  G.hx = w / G.nx;
  G.hy = h / G.ny;
}

static inline i32 cell_of(double v, double v0, double hv, i32 n) {
  double f = std::floor((v - v0) / hv);
  if (!(f >= 0)) return 0;
  if (f >= n) return n - 1;
  return (i32)f;
}

void build_centroid_grid(const std::vector<double>& cx, const std::vector<double>& cy, double per_cell, Grid& G) {
  const i64 T = (i64)cx.size();
  grid_dims(*std::min_element(cx.begin(), cx.end()), *std::max_element(cx.begin(), cx.end()),
            *std::min_element(cy.begin(), cy.end()), *std::max_element(cy.begin(), cy.end()), T, per_cell, G);
  const i64 nc = (i64)G.nx * G.ny;
  std::vector<i32> cell;
  host_alloc_fresh(cell, T);
  parallel_for(T, [&](i64 t0, i64 t1) {
    for (i64 t = t0; t < t1; ++t) cell[t] = cell_of(cy[t], G.y0, G.hy, G.ny) * G.nx + cell_of(cx[t], G.x0, G.hx, G.nx);
  });
  // counting sort by cell, ascending triangle id inside each cell.  Each thread owns a contiguous range of
  // cells and scans every triangle (two passes over the 4 B cell ids) for those in its range: the same
  // order as one sequential pass, no per-thread histograms of all cells.
  G.cell_start.assign(nc + 1, 0);
  host_alloc_fresh(G.item, T);
  host_alloc_fresh(G.px, T);
  host_alloc_fresh(G.py, T);
  const int nt = (int)std::max<i64>(1, std::min<i64>((i64)host_threads(), T / 65536 + 1));
  auto range = [&](int w, i64& c0, i64& c1) {
    c0 = nc * w / nt;
    c1 = nc * (w + 1) / nt;
  };
  auto run = [&](auto&& f) {
    if (nt == 1) {
      f(0);
      return;
    }
    ThreadGroup g;
    for (int w = 0; w < nt; ++w) g.spawn([&f, w] { f(w); });
    g.join();
  };
  run([&](int w) {  // counts
    i64 c0, c1;
    range(w, c0, c1);
    for (i64 t = 0; t < T; ++t) {
      const i64 c = cell[t];
      if (c >= c0 && c < c1) G.cell_start[c + 1]++;
    }
  });
  for (i64 c = 0; c < nc; ++c) G.cell_start[c + 1] += G.cell_start[c];
  run([&](int w) {  // the fill
    i64 c0, c1;
    range(w, c0, c1);
    std::vector<i32> fill(G.cell_start.begin() + c0, G.cell_start.begin() + c1);
    for (i64 t = 0; t < T; ++t) {
      const i64 c = cell[t];
      if (c < c0 || c >= c1) continue;
      const i32 k = fill[c - c0]++;
      G.item[k] = (i32)t;
      G.px[k] = cx[t];
      G.py[k] = cy[t];
    }
  });
}

std::vector<float> centroid_knn_radius2(const Grid& G, const std::vector<double>& cx, const std::vector<double>& cy,
                                        int k) {
  return knn_radius2(G, cx, cy, k, true);
}

std::vector<float> knn_radius2(const Grid& G, const std::vector<double>& cx, const std::vector<double>& cy, int k,
                               bool self) {
  const i64 ncent = (i64)G.item.size();
  const i64 T = (i64)cx.size();
  std::vector<float> out(T, INFINITY);
  if (ncent - (self ? 1 : 0) < k) return out;
  auto work = [&](i64 t0, i64 t1) {
    std::vector<double> best(k);
    for (i64 t = t0; t < t1; ++t) {
      const double qx = cx[t], qy = cy[t];
      std::fill(best.begin(), best.end(), INFINITY);  // ascending k smallest squared distances
      const i32 ci = cell_of(qx, G.x0, G.hx, G.nx), cj = cell_of(qy, G.y0, G.hy, G.ny);
      for (i32 r = 0;; ++r) {
        const i32 jlo = std::max(cj - r, 0), jhi = std::min(cj + r, G.ny - 1);
        for (i32 j = jlo; j <= jhi; ++j) {
          const bool edge = j == cj - r || j == cj + r;
          for (i32 i = ci - r; i <= ci + r; i += (edge || r == 0) ? 1 : 2 * r) {
            if (i < 0 || i >= G.nx) continue;
            const i64 c = (i64)j * G.nx + i;
            for (i32 e = G.cell_start[c]; e < G.cell_start[c + 1]; ++e) {
              if (self && G.item[e] == (i32)t) continue;
              const double dx = G.px[e] - qx, dy = G.py[e] - qy, d = dx * dx + dy * dy;
              if (d >= best[k - 1]) continue;
              int p = k - 1;
              while (p > 0 && best[p - 1] > d) {
                best[p] = best[p - 1];
                --p;
              }
              best[p] = d;
            }
          }
        }
        // every unvisited cell is at least this far from q
        double dmin = INFINITY;
        if (ci - r > 0) dmin = std::min(dmin, qx - (G.x0 + (ci - r) * G.hx));
        if (ci + r < G.nx - 1) dmin = std::min(dmin, G.x0 + (ci + r + 1) * G.hx - qx);
        if (cj - r > 0) dmin = std::min(dmin, qy - (G.y0 + (cj - r) * G.hy));
        if (cj + r < G.ny - 1) dmin = std::min(dmin, G.y0 + (cj + r + 1) * G.hy - qy);
        if (dmin == INFINITY || (dmin > 0 && best[k - 1] < dmin * dmin * (1.0 - 1e-9))) break;
      }
      // round down: the device's acceptance test must never see a larger radius than the true one
      float f = (float)best[k - 1];
      if ((double)f > best[k - 1]) f = std::nextafter(f, 0.0f);
      out[t] = f;
    }
  };
  const int nt = host_threads();
  ThreadGroup g;
  for (int w = 0; w < nt; ++w) g.spawn([&work, w, nt, T] { work(T * w / nt, T * (w + 1) / nt); });
  g.join();
  return out;
}

void build_tri_grid(const std::vector<double>& x, const std::vector<double>& y, const std::vector<i32>& tri,
                    double per_cell, Grid& G, double inflate) {
  const i64 T = (i64)tri.size() / 3;
  grid_dims(*std::min_element(x.begin(), x.end()), *std::max_element(x.begin(), x.end()),
            *std::min_element(y.begin(), y.end()), *std::max_element(y.begin(), y.end()), T, per_cell, G);
  const i64 nc = (i64)G.nx * G.ny;
  G.cell_start.assign(nc + 1, 0);
  auto bbox = [&](i64 t, i32& cx0, i32& cx1, i32& cy0, i32& cy1) {
    double xa = std::min({x[tri[3 * t]], x[tri[3 * t + 1]], x[tri[3 * t + 2]]});
    double xb = std::max({x[tri[3 * t]], x[tri[3 * t + 1]], x[tri[3 * t + 2]]});
    double ya = std::min({y[tri[3 * t]], y[tri[3 * t + 1]], y[tri[3 * t + 2]]});
    double yb = std::max({y[tri[3 * t]], y[tri[3 * t + 1]], y[tri[3 * t + 2]]});
    if (inflate > 0) {  // relative to the triangle's extent, plus an absolute floor
      const double m = inflate * std::max(xb - xa, yb - ya) + 1e-14;
      xa -= m;
      xb += m;
      ya -= m;
      yb += m;
    }
    cx0 = cell_of(xa, G.x0, G.hx, G.nx);
    cx1 = cell_of(xb, G.x0, G.hx, G.nx);
    cy0 = cell_of(ya, G.y0, G.hy, G.ny);
    cy1 = cell_of(yb, G.y0, G.hy, G.ny);
  };
  for (i64 t = 0; t < T; ++t) {
    i32 a, b, c, d;
    bbox(t, a, b, c, d);
    for (i32 j = c; j <= d; ++j)
      for (i32 i = a; i <= b; ++i) G.cell_start[(i64)j * G.nx + i + 1]++;
  }
  for (i64 c = 0; c < nc; ++c) G.cell_start[c + 1] += G.cell_start[c];
  G.item.assign(G.cell_start[nc], 0);
  std::vector<i32> fill(G.cell_start.begin(), G.cell_start.end() - 1);
  for (i64 t = 0; t < T; ++t) {
    i32 a, b, c, d;
    bbox(t, a, b, c, d);
    for (i32 j = c; j <= d; ++j)
      for (i32 i = a; i <= b; ++i) G.item[fill[(i64)j * G.nx + i]++] = (i32)t;
  }
}

// ----------------------------------------------------------------------------- multigrid helpers
std::vector<std::pair<i64, i64>> level_pairs(const HostMesh& m, double L, double tol, double H) {
  std::vector<i64> left, right;
  for (i64 i = 0; i < m.N; ++i) {
    if (std::fabs(m.x[i]) < tol) left.push_back(i);
    if (std::fabs(m.x[i] - L) < tol) right.push_back(i);
  }
  std::vector<std::pair<i64, i64>> out;
  if (left.empty() || right.empty()) return out;
  std::vector<i64> rs = right;
  std::sort(rs.begin(), rs.end(), [&](i64 a, i64 b) { return m.y[a] != m.y[b] ? m.y[a] < m.y[b] : a < b; });
  for (i64 l : left) {
    const double y = m.y[l];
    if (std::fabs(y - 0.0) < tol || std::fabs(y - H) < tol) continue;
    auto it = std::lower_bound(rs.begin(), rs.end(), y, [&](i64 a, double v) { return m.y[a] < v; });
    i64 best = -1;
    double bd = INFINITY;
    for (auto jt : {it - 1, it}) {
      if (jt < rs.begin() || jt >= rs.end()) continue;
      const double d = std::fabs(m.y[*jt] - y);
      if (d < bd || (d == bd && *jt < best)) {
        bd = d;
        best = *jt;
      }
    }
    out.push_back({l, best});
  }
  return out;
}

void build_prolongation(i64 Nc, const std::vector<i32>& ea, const std::vector<i32>& eb, const Ordering& of,
                        const Ordering& oc, const std::vector<i32>& dof_c, const std::vector<i32>& master_of_f,
                        Csr& P) {
  const i64 Nf = (i64)of.new2old.size();
  P.nrows = Nf;
  // row g: nothing (a periodic slave), its coarse node, or the two coarse ends of its midpoint edge
  // (one entry when both ends merge); two threaded passes, lengths then entries
  auto row = [&](i64 g, i32* col, double* val) -> int {
    if (master_of_f[g] >= 0) return 0;
    const i64 o = of.new2old[g];
    if (o < Nc) {
      col[0] = dof_c[oc.old2new[o]];
      val[0] = 1.0;
      return 1;
    }
    i32 a = dof_c[oc.old2new[ea[o - Nc]]], b = dof_c[oc.old2new[eb[o - Nc]]];
    if (a == b) {
      col[0] = a;
      val[0] = 1.0;
      return 1;
    }
    if (b < a) std::swap(a, b);
    col[0] = a;
    val[0] = 0.5;
    col[1] = b;
    val[1] = 0.5;
    return 2;
  };
  host_alloc_fresh(P.rowptr, Nf + 1);
  P.rowptr[0] = 0;
  parallel_for(Nf, [&](i64 g0, i64 g1) {
    i32 c[2];
    double v[2];
    for (i64 g = g0; g < g1; ++g) P.rowptr[g + 1] = row(g, c, v);
  });
  for (i64 g = 0; g < Nf; ++g) P.rowptr[g + 1] += P.rowptr[g];
  host_alloc_fresh(P.col, P.rowptr[Nf]);
  host_alloc_fresh(P.val, P.rowptr[Nf]);
  parallel_for(Nf, [&](i64 g0, i64 g1) {
    for (i64 g = g0; g < g1; ++g) row(g, P.col.data() + P.rowptr[g], P.val.data() + P.rowptr[g]);
  });
}

// counting sort by column; each thread owns a contiguous range of columns and scans every entry (rows in
// ascending order inside every column, as one sequential pass)
void transpose(const Csr& A, i64 ncols, Csr& At) {
  At.nrows = ncols;
  At.rowptr.assign(ncols + 1, 0);
  const i64 nnz = A.nnz();
  const int nt = (int)std::max<i64>(1, std::min<i64>((i64)host_threads(), nnz / 65536 + 1));
  auto run = [&](auto&& f) {
    if (nt == 1) {
      f(0);
      return;
    }
    ThreadGroup g;
    for (int w = 0; w < nt; ++w) g.spawn([&f, w] { f(w); });
    g.join();
  };
  run([&](int w) {
    const i64 c0 = ncols * w / nt, c1 = ncols * (w + 1) / nt;
    for (i64 k = 0; k < nnz; ++k) {
      const i64 c = A.col[k];
      if (c >= c0 && c < c1) At.rowptr[c + 1]++;
    }
  });
  for (i64 c = 0; c < ncols; ++c) At.rowptr[c + 1] += At.rowptr[c];
  host_alloc_fresh(At.col, nnz);
  host_alloc_fresh(At.val, nnz);
  run([&](int w) {
    const i64 c0 = ncols * w / nt, c1 = ncols * (w + 1) / nt;
    std::vector<i64> fill(At.rowptr.begin() + c0, At.rowptr.begin() + c1);
    for (i64 r = 0; r < A.nrows; ++r)
      for (i64 k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) {
        const i64 c = A.col[k];
        if (c < c0 || c >= c1) continue;
        const i64 d = fill[c - c0]++;
        At.col[d] = (i32)r;
        At.val[d] = A.val[k];
      }
  });
}

bool lu_inverse(std::vector<double>& A, i64 n) {
  // LU with partial pivoting (row-major, in place: P A = L U, unit lower L), then the inverse column by
  // column: L y = P e_j, U x = y.  The columns are independent -> threads.
  std::vector<i64> piv(n);
  for (i64 k = 0; k < n; ++k) {
    i64 p = k;
    double best = std::fabs(A[k * n + k]);
    for (i64 i = k + 1; i < n; ++i)
      if (std::fabs(A[i * n + k]) > best) best = std::fabs(A[i * n + k]), p = i;
    if (!(best > 0.0) || !std::isfinite(best)) return false;
    piv[k] = p;
    if (p != k)
      for (i64 j = 0; j < n; ++j) std::swap(A[k * n + j], A[p * n + j]);
    const double inv = 1.0 / A[k * n + k];
    const double* rk = A.data() + k * n;
    parallel_for(n - k - 1, [&](i64 a, i64 b) {
      for (i64 i = k + 1 + a; i < k + 1 + b; ++i) {
        double* ri = A.data() + i * n;
        const double l = ri[k] * inv;
        ri[k] = l;
        if (l != 0.0)
          for (i64 j = k + 1; j < n; ++j) ri[j] -= l * rk[j];
      }
    });
  }
  // row permutation of the identity: e_j lands in row perm^-1(j)
  std::vector<i64> perm(n);
  std::iota(perm.begin(), perm.end(), (i64)0);
  for (i64 k = 0; k < n; ++k) std::swap(perm[k], perm[piv[k]]);
  std::vector<double> inv(n * n, 0.0);  // inverse, transposed (column j in row j)
  parallel_for(n, [&](i64 j0, i64 j1) {
    std::vector<double> x(n);
    for (i64 j = j0; j < j1; ++j) {
      for (i64 i = 0; i < n; ++i) x[i] = perm[i] == j ? 1.0 : 0.0;
      for (i64 i = 0; i < n; ++i) {  // L (unit diagonal)
        double s = x[i];
        const double* ri = A.data() + i * n;
        for (i64 k = 0; k < i; ++k) s -= ri[k] * x[k];
        x[i] = s;
      }
      for (i64 i = n - 1; i >= 0; --i) {  // U
        double s = x[i];
        const double* ri = A.data() + i * n;
        for (i64 k = i + 1; k < n; ++k) s -= ri[k] * x[k];
        x[i] = s / ri[i];
      }
      std::copy(x.begin(), x.end(), inv.begin() + j * n);
    }
  });
  for (i64 i = 0; i < n; ++i)
    for (i64 j = 0; j < n; ++j) A[i * n + j] = inv[j * n + i];
  return true;
}

bool spd_inverse(std::vector<double>& A, i64 n) {
  // Cholesky A = L L^T (lower, in place), then inv = L^-T L^-1.
  // Left-looking by rows, rows dealt cyclically to the threads: row i's entry in column j needs only row i
  // (its own thread's) and row j up to its diagonal, so the owner of row j publishes its diagonal (`ready`)
  // and the other threads go on with column j without a barrier.  Same operations in the same order as
  // the serial loop: bit-identical factor.
  const int nt = (int)std::max<i64>(1, std::min<i64>((i64)host_threads(), n / 64));
  {
    std::atomic<i64> ready{0};  // rows [0, ready) final up to and including their diagonal
    std::atomic<bool> bad{false};
    auto work = [&](int t) {
      for (i64 j = 0; j < n; ++j) {
        if (j % nt == t) {
          double d = A[j * n + j];
          for (i64 k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
          if (!(d > 0)) {
            bad.store(true, std::memory_order_release);
            ready.store(n, std::memory_order_release);
            return;
          }
          A[j * n + j] = std::sqrt(d);
          ready.store(j + 1, std::memory_order_release);
        } else {
          for (int spin = 0; ready.load(std::memory_order_acquire) <= j; ++spin)
            if (spin > 64) std::this_thread::yield();
        }
        if (bad.load(std::memory_order_acquire)) return;
        const double d = A[j * n + j];
        const double* aj = A.data() + j * n;
        i64 i = j + 1 + ((t - (j + 1) % nt) % nt + nt) % nt;  // first row > j of thread t
        for (; i < n; i += nt) {
          double* ai = A.data() + i * n;
          double s = ai[j];
          for (i64 k = 0; k < j; ++k) s -= ai[k] * aj[k];
          ai[j] = s / d;
        }
      }
    };
    if (nt == 1) {
      work(0);
    } else {
      ThreadGroup g;
      for (int t = 0; t < nt; ++t) g.spawn([&work, t] { work(t); });
      g.join();
    }
    if (bad.load()) return false;
  }
  // Linv (lower): column j of W = L^-1 by forward substitution, columns independent -> threads; stored
  // transposed (Wt[j][i] = W[i][j]) so both loops below read contiguous rows.  Same operations in the
  // same order as the column-by-column loop: the inverse is bit-identical to the serial one.
  // (triangular work per row: rows dealt cyclically to the threads, not parallel_for's contiguous ranges)
  auto cyclic = [nt](i64 n_, auto&& f) {
    if (nt == 1) {
      for (i64 i = 0; i < n_; ++i) f(i);
      return;
    }
    ThreadGroup g;
    for (int t = 0; t < nt; ++t)
      g.spawn([&f, t, nt, n_] {
        for (i64 i = t; i < n_; i += nt) f(i);
      });
    g.join();
  };
  std::vector<double> Wt(n * n, 0.0);
  cyclic(n, [&](i64 j) {
    {
      double* w = Wt.data() + j * n;
      w[j] = 1.0 / A[j * n + j];
      for (i64 i = j + 1; i < n; ++i) {
        double s = 0.0;
        for (i64 k = j; k < i; ++k) s -= A[i * n + k] * w[k];
        w[i] = s / A[i * n + i];
      }
    }
  });
  // inv = W^T W: inv[i][j] = sum_{k >= i} W[k][i] W[k][j] (j <= i), rows independent -> threads
  cyclic(n, [&](i64 i) {
    {
      const double* wi = Wt.data() + i * n;
      for (i64 j = 0; j <= i; ++j) {
        const double* wj = Wt.data() + j * n;
        double s = 0.0;
        for (i64 k = i; k < n; ++k) s += wi[k] * wj[k];
        A[i * n + j] = s;
      }
    }
  });
  for (i64 i = 0; i < n; ++i)
    for (i64 j = 0; j < i; ++j) A[j * n + i] = A[i * n + j];
  return true;
}

void make_local_plan2(const std::vector<PatRows>& pats, const std::vector<i64>& row_start, int rank, LocalPlan& lp,
                      const std::vector<const Csr*>* deep, std::vector<i32>* g1_out) {
  const int world = (int)row_start.size() - 1;
  lp.r0 = row_start[rank];
  lp.r1 = row_start[rank + 1];
  lp.n_own = lp.r1 - lp.r0;
  auto owner = [&](i64 g) {
    return (i32)(std::upper_bound(row_start.begin(), row_start.end(), g) - row_start.begin() - 1);
  };
  auto cols_of = [&](int q, std::vector<i32>& out, i64 lo, i64 hi, bool inside) {
    for (auto& pr : pats) {
      const Csr& A = *pr.A;
      const std::vector<i64>& rs = *pr.rows;
      for (i64 r = rs[q]; r < rs[q + 1]; ++r)
        for (i64 k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) {
          const i32 c = A.col[k];
          const bool in = c >= lo && c < hi;
          if (in == inside) out.push_back(c);
        }
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
  };
  // deep halos: rank q's ghost rows one layer out (G1) and their columns (G2)
  auto deep_of = [&](int q, std::vector<i32>& g1, std::vector<i32>& g2) {
    g1.clear();
    g2.clear();
    if (!deep) return;
    const i64 lo = row_start[q], hi = row_start[q + 1];
    for (const Csr* A : *deep)
      for (i64 r = lo; r < hi; ++r)
        for (i64 k = A->rowptr[r]; k < A->rowptr[r + 1]; ++k)
          if (A->col[k] < lo || A->col[k] >= hi) g1.push_back(A->col[k]);
    std::sort(g1.begin(), g1.end());
    g1.erase(std::unique(g1.begin(), g1.end()), g1.end());
    for (const Csr* A : *deep)
      for (i32 r : g1)
        for (i64 k = A->rowptr[r]; k < A->rowptr[r + 1]; ++k)
          if (A->col[k] < lo || A->col[k] >= hi) g2.push_back(A->col[k]);
  };
  // every ghost of rank q: the patterns' off-range columns and (deep) G1 and G2
  auto ghosts_of = [&](int q, std::vector<i32>& out) {
    cols_of(q, out, row_start[q], row_start[q + 1], false);
    if (!deep) return;
    std::vector<i32> g1, g2;
    deep_of(q, g1, g2);
    out.insert(out.end(), g1.begin(), g1.end());
    out.insert(out.end(), g2.begin(), g2.end());
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
  };
  std::vector<i32> gh;
  ghosts_of(rank, gh);
  if (g1_out) {
    std::vector<i32> g2;
    deep_of(rank, *g1_out, g2);
  }
  lp.ghost_global = gh;
  lp.n_ghost = (i64)gh.size();
  lp.ghost_owner.resize(gh.size());
  for (size_t k = 0; k < gh.size(); ++k) lp.ghost_owner[k] = owner(gh[k]);
  lp.recv_peer.clear();
  lp.recv_off.clear();
  lp.recv_cnt.clear();
  for (size_t k = 0; k < gh.size(); ++k) {
    if (lp.recv_peer.empty() || lp.recv_peer.back() != lp.ghost_owner[k]) {
      lp.recv_peer.push_back(lp.ghost_owner[k]);
      lp.recv_off.push_back((i64)k);
      lp.recv_cnt.push_back(0);
    }
    lp.recv_cnt.back()++;
  }
  lp.send_peer.clear();
  lp.send_off.clear();
  lp.send_cnt.clear();
  lp.send_local.clear();
  for (int q = 0; q < world; ++q) {
    if (q == rank) continue;
    std::vector<i32> need;
    if (deep) {  // q's ghosts inside my range
      std::vector<i32> gq;
      ghosts_of(q, gq);
      for (i32 g : gq)
        if (g >= lp.r0 && g < lp.r1) need.push_back(g);
    } else {
      cols_of(q, need, lp.r0, lp.r1, true);
    }
    // q only needs those of my rows that are not its own (q's rows are outside my range anyway)
    if (need.empty()) continue;
    lp.send_peer.push_back(q);
    lp.send_off.push_back((i64)lp.send_local.size());
    lp.send_cnt.push_back((i64)need.size());
    for (i32 g : need) lp.send_local.push_back((i32)(g - lp.r0));
  }
}

void build_sell_x(const Csr& A, i64 r0, i64 n, const LocalPlan& cols, Sell& S, bool pad_self) {
  S.nrows = n;
  S.nslices = (n + 63) / 64;
  S.slice_off.assign(S.nslices + 1, 0);
  S.slice_w.assign(S.nslices, 0);
  for (i64 s = 0; s < S.nslices; ++s) {
    i64 w = 0;
    for (i64 l = 0; l < 64; ++l) {
      const i64 r = s * 64 + l;
      if (r < n) w = std::max(w, A.rowptr[r0 + r + 1] - A.rowptr[r0 + r]);
    }
    S.slice_w[s] = (i32)w;
    S.slice_off[s + 1] = S.slice_off[s] + w * 64;
  }
  S.padded = S.slice_off[S.nslices];
  S.col.assign(S.padded, 0);
  for (i64 s = 0; s < S.nslices; ++s)
    for (i64 l = 0; l < 64; ++l) {
      const i64 r = s * 64 + l;
      const i64 len = r < n ? A.rowptr[r0 + r + 1] - A.rowptr[r0 + r] : 0;
      for (i64 k = 0; k < S.slice_w[s]; ++k)
        S.col[S.slice_off[s] + k * 64 + l] =
            k < len ? to_local(cols, A.col[A.rowptr[r0 + r] + k]) : (pad_self && r < n ? (i32)r : 0);
    }
}

void sell_values_x(const Csr& A, i64 r0, const Sell& S, const std::vector<double>& val, std::vector<double>& out) {
  if (!S.rows.empty()) return sell_values_rows(A, r0, S, val, out);
  out.assign(S.padded, 0.0);
  parallel_for(S.nslices, [&](i64 s0, i64 s1) {
    for (i64 s = s0; s < s1; ++s)
      for (i64 l = 0; l < 64; ++l) {
        const i64 r = s * 64 + l;
        if (r >= S.nrows) continue;
        const i64 b = A.rowptr[r0 + r], len = A.rowptr[r0 + r + 1] - b;
        for (i64 k = 0; k < len; ++k) out[S.slice_off[s] + k * 64 + l] = val[b + k];
      }
  }, 64);
}

}  // namespace pucfem

// ============================================================================= lattice layout
namespace pucfem {

void build_sell_rows(const Csr& A, i64 r0, const std::vector<i32>& rows, const LocalPlan& cols, Sell& S) {
  const i64 n = (i64)rows.size();
  S.nrows = n;
  S.nslices = (n + 63) / 64;
  S.slice_off.assign(S.nslices + 1, 0);
  S.slice_w.assign(S.nslices, 0);
  S.rows.assign(S.nslices * 64, -1);
  for (i64 s = 0; s < S.nslices; ++s) {
    i64 w = 0;
    for (i64 l = 0; l < 64; ++l) {
      const i64 k = s * 64 + l;
      if (k < n) {
        const i64 r = r0 + rows[k];
        w = std::max(w, A.rowptr[r + 1] - A.rowptr[r]);
        S.rows[k] = rows[k];
      }
    }
    S.slice_w[s] = (i32)w;
    S.slice_off[s + 1] = S.slice_off[s] + w * 64;
  }
  S.padded = S.slice_off[S.nslices];
  S.nnz = 0;
  for (i64 k = 0; k < n; ++k) S.nnz += A.rowptr[r0 + rows[k] + 1] - A.rowptr[r0 + rows[k]];
  S.col.assign(S.padded, 0);
  for (i64 s = 0; s < S.nslices; ++s)
    for (i64 l = 0; l < 64; ++l) {
      const i64 k = s * 64 + l;
      const i64 r = k < n ? r0 + rows[k] : -1;
      const i64 len = k < n ? A.rowptr[r + 1] - A.rowptr[r] : 0;
      // padding entries of a listed row gather the row's first column again (value 0, in cache)
      const i32 first = len > 0 ? to_local(cols, A.col[A.rowptr[r]]) : 0;
      for (i64 e = 0; e < S.slice_w[s]; ++e)
        S.col[S.slice_off[s] + e * 64 + l] = e < len ? to_local(cols, A.col[A.rowptr[r] + e]) : first;
    }
}

void sell_values_rows(const Csr& A, i64 r0, const Sell& S, const std::vector<double>& val, std::vector<double>& out) {
  out.assign(S.padded, 0.0);
  for (i64 s = 0; s < S.nslices; ++s)
    for (i64 l = 0; l < 64; ++l) {
      const i64 k = s * 64 + l;
      if (S.rows[k] < 0) continue;  // (a padding lane: the own rows' last slice is padded before any ghost rows)
      if (!S.gval.empty() && k >= S.gk0) {  // (ghost rows with their own entries: the values stored with them)
        const i64 p0 = S.slice_off[S.nslices_own];
        for (i64 e = 0; e < S.slice_w[s]; ++e) {
          const i64 q = S.slice_off[s] + e * 64 + l;
          out[q] = S.gval[q - p0];
        }
        continue;
      }
      const i64 r = S.global_row(r0, k);
      const i64 b = A.rowptr[r], len = A.rowptr[r + 1] - b;
      for (i64 e = 0; e < len; ++e) out[S.slice_off[s] + e * 64 + l] = val[b + e];
    }
}

void sell_append_ghost_rows(const Csr& A, const std::vector<i32>& grows, const LocalPlan& cols, Sell& S,
                            const LocalPlan* rows_plan, const GhostRowFn* custom) {
  const LocalPlan& rp = rows_plan ? *rows_plan : cols;
  // every ghost row's entries: A's row, or the custom one
  const i64 ng = (i64)grows.size();
  std::vector<std::vector<i32>> ccols(custom ? ng : 0);
  std::vector<std::vector<double>> cvals(custom ? ng : 0);
  std::vector<char> is_custom(ng, 0);
  if (custom)
    for (i64 k = 0; k < ng; ++k) is_custom[k] = (*custom)(grows[k], ccols[k], cvals[k]) ? 1 : 0;
  auto row_len = [&](i64 k) -> i64 {
    return is_custom[k] ? (i64)ccols[k].size() : A.rowptr[grows[k] + 1] - A.rowptr[grows[k]];
  };
  auto row_col = [&](i64 k, i64 e) -> i32 { return is_custom[k] ? ccols[k][e] : A.col[A.rowptr[grows[k]] + e]; };
  auto row_val = [&](i64 k, i64 e) -> double { return is_custom[k] ? cvals[k][e] : A.val[A.rowptr[grows[k]] + e]; };
  bool any_custom = false;
  for (char c : is_custom) any_custom = any_custom || c;
  if (S.gk0 >= 0) throw std::runtime_error("SELL already has ghost rows");
  if (S.rows.empty() && S.nrows > 0) throw std::runtime_error("ghost rows need a row-listed SELL");
  S.nslices_own = S.nslices;
  S.gk0 = S.nslices * 64;
  S.grow = grows;
  const i64 n = (i64)grows.size(), ns = (n + 63) / 64;
  S.rows.resize((S.nslices + ns) * 64, -1);
  S.slice_w.resize(S.nslices + ns, 0);
  S.slice_off.resize(S.nslices + ns + 1, S.slice_off[S.nslices]);
  for (i64 s = 0; s < ns; ++s) {
    i64 w = 0;
    for (i64 l = 0; l < 64 && s * 64 + l < n; ++l) {
      const i64 g = grows[s * 64 + l];
      w = std::max(w, row_len(s * 64 + l));
      S.rows[S.gk0 + s * 64 + l] = to_local(rp, (i32)g);
      if (S.rows[S.gk0 + s * 64 + l] < rp.n_own) throw std::runtime_error("ghost row list holds an owned row");
    }
    S.slice_w[S.nslices + s] = (i32)w;
    S.slice_off[S.nslices + s + 1] = S.slice_off[S.nslices + s] + w * 64;
  }
  const i64 p0 = S.padded;
  S.padded = S.slice_off[S.nslices + ns];
  S.col.resize(S.padded, 0);
  if (any_custom) S.gval.assign(S.padded - p0, 0.0);
  for (i64 s = 0; s < ns; ++s)
    for (i64 l = 0; l < 64; ++l) {
      const i64 k = s * 64 + l;
      const i64 len = k < n ? row_len(k) : 0;
      const i32 first = len > 0 ? to_local(cols, row_col(k, 0)) : 0;
      for (i64 e = 0; e < S.slice_w[S.nslices + s]; ++e) {
        const i64 q = S.slice_off[S.nslices + s] + e * 64 + l;
        S.col[q] = e < len ? to_local(cols, row_col(k, e)) : first;
        if (any_custom && e < len) S.gval[q - p0] = row_val(k, e);
      }
      S.nnz += len;
    }
  S.nslices += ns;
  S.nrows += n;
}


void build_macro(const HostMesh& c, int strips, int lw, Macro& M) {
  M.nv = c.N;
  M.nf = c.T;
  M.x = c.x;
  M.y = c.y;
  M.tri = c.tri;
  std::vector<std::pair<i32, i32>> es;
  es.reserve(3 * c.T);
  for (i64 t = 0; t < c.T; ++t)
    for (int e = 0; e < 3; ++e) {
      const i32 a = c.tri[3 * t + e], b = c.tri[3 * t + (e + 1) % 3];
      es.push_back({std::min(a, b), std::max(a, b)});
    }
  std::sort(es.begin(), es.end());
  es.erase(std::unique(es.begin(), es.end()), es.end());
  M.ne = (i64)es.size();
  M.ev.resize(2 * M.ne);
  for (i64 e = 0; e < M.ne; ++e) {
    M.ev[2 * e] = es[e].first;
    M.ev[2 * e + 1] = es[e].second;
  }
  auto eid = [&](i32 a, i32 b) {
    const std::pair<i32, i32> k{std::min(a, b), std::max(a, b)};
    return (i32)(std::lower_bound(es.begin(), es.end(), k) - es.begin());
  };
  M.fe.resize(3 * M.nf);
  for (i64 f = 0; f < M.nf; ++f) {
    const i32 A = c.tri[3 * f], B = c.tri[3 * f + 1], C = c.tri[3 * f + 2];
    M.fe[3 * f] = eid(A, B);
    M.fe[3 * f + 1] = eid(A, C);
    M.fe[3 * f + 2] = eid(B, C);
  }
  // strip keys (y) and x keys of every primitive; weights = nodes at level lw
  const i32 n = 1 << lw;
  const double wF = lat::interior_count(n), wE = std::max(0, n - 1), wV = 1.0;
  struct Item {
    double ky, kx, w;
    int kind;
    i32 id;
  };
  std::vector<Item> it;
  it.reserve(M.nf + M.ne + M.nv);
  for (i64 f = 0; f < M.nf; ++f) {
    const i32 A = c.tri[3 * f], B = c.tri[3 * f + 1], C = c.tri[3 * f + 2];
    it.push_back({(c.y[A] + c.y[B] + c.y[C]) / 3.0, (c.x[A] + c.x[B] + c.x[C]) / 3.0, wF, 0, (i32)f});
  }
  for (i64 e = 0; e < M.ne; ++e) {
    const i32 a = M.ev[2 * e], b = M.ev[2 * e + 1];
    it.push_back({(c.y[a] + c.y[b]) * 0.5, (c.x[a] + c.x[b]) * 0.5, wE, 1, (i32)e});
  }
  for (i64 v = 0; v < M.nv; ++v) it.push_back({c.y[v], c.x[v], wV, 2, (i32)v});
  std::vector<Item> byy = it;
  std::stable_sort(byy.begin(), byy.end(), [](const Item& a, const Item& b) { return a.ky < b.ky; });
  double W = 0.0;
  for (auto& q : byy) W += q.w;
  // auto: strips of about 16 faces (the rank partition's granularity), at most 64
  const int S = strips > 0 ? strips : (int)std::max<i64>(1, std::min<i64>(64, M.nf / 16));
  M.cuts.clear();
  double acc = 0.0;
  size_t k = 0;
  for (int s = 1; s < S; ++s) {
    const double target = W * s / S;
    while (k < byy.size() && acc + byy[k].w <= target) acc += byy[k++].w;
    // move to a key boundary (equal keys -- periodic partners -- share a strip)
    while (k > 0 && k < byy.size() && byy[k].ky == byy[k - 1].ky) acc += byy[k++].w;
    if (k == 0 || k >= byy.size()) continue;
    const double cut = 0.5 * (byy[k - 1].ky + byy[k].ky);
    if (M.cuts.empty() || cut > M.cuts.back()) M.cuts.push_back(cut);
  }
  M.S = (int)M.cuts.size() + 1;
  auto strip_of = [&](double ky) { return (i32)(std::upper_bound(M.cuts.begin(), M.cuts.end(), ky) - M.cuts.begin()); };
  for (int kind = 0; kind < 3; ++kind) {
    std::vector<Item> v;
    for (auto& q : it)
      if (q.kind == kind) v.push_back(q);
    std::sort(v.begin(), v.end(), [&](const Item& a, const Item& b) {
      const i32 sa = strip_of(a.ky), sb = strip_of(b.ky);
      if (sa != sb) return sa < sb;
      if (a.kx != b.kx) return a.kx < b.kx;
      return a.id < b.id;
    });
    std::vector<i32>& ord = kind == 0 ? M.order_f : kind == 1 ? M.order_e : M.order_v;
    std::vector<i32>& sp = kind == 0 ? M.strip_f : kind == 1 ? M.strip_e : M.strip_v;
    ord.resize(v.size());
    sp.assign(M.S + 1, 0);
    for (size_t q = 0; q < v.size(); ++q) {
      ord[q] = v[q].id;
      sp[strip_of(v[q].ky) + 1]++;
    }
    for (int s = 0; s < M.S; ++s) sp[s + 1] += sp[s];
  }
}

void lattice_ordering(const HostMesh& ml, const Macro& M, int l, Ordering& ord, LatticeLevel& LL) {
  const i32 n = 1 << l;
  LL.l = l;
  LL.n = n;
  LL.F = lat::interior_count(n);
  LL.face_start.assign(M.nf, -1);
  LL.edge_start.assign(M.ne, -1);
  LL.vert_start.assign(M.nv, -1);
  ord.strip_ptr.assign(M.S + 1, 0);
  i64 pos = 0;
  for (int s = 0; s < M.S; ++s) {
    for (i32 q = M.strip_f[s]; q < M.strip_f[s + 1]; ++q) {
      LL.face_start[M.order_f[q]] = pos;
      pos += LL.F;
    }
    for (i32 q = M.strip_e[s]; q < M.strip_e[s + 1]; ++q) {
      LL.edge_start[M.order_e[q]] = pos;
      pos += n - 1;
    }
    for (i32 q = M.strip_v[s]; q < M.strip_v[s + 1]; ++q) LL.vert_start[M.order_v[q]] = pos++;
    ord.strip_ptr[s + 1] = pos;
  }
  if (pos != ml.N || ml.T != M.nf * ((i64)1 << (2 * l)))
    throw std::runtime_error("lattice ordering: the mesh is not the coarse mesh refined " + std::to_string(l) + " times");
  // a triangle containing each node (the first one), then the node's lattice position in that
  // triangle's ancestor face (ancestor of fine triangle t = t >> 2l: red_refine numbers the children
  // of t as 4t .. 4t+3)
  std::vector<i64> n2t(ml.N, -1);
  for (i64 t = 0; t < ml.T; ++t)
    for (int v = 0; v < 3; ++v)
      if (n2t[ml.tri[3 * t + v]] < 0) n2t[ml.tri[3 * t + v]] = t;
  ord.new2old.assign(ml.N, -1);
  ord.old2new.assign(ml.N, -1);
  LL.type.assign(ml.N, 0);
  std::vector<int> bad(1, 0);
  std::mutex mx;
  parallel_for(ml.N, [&](i64 v0, i64 v1) {
    for (i64 v = v0; v < v1; ++v) {
      const i64 t = n2t[v];
      if (t < 0) {
        std::lock_guard<std::mutex> lk(mx);
        bad[0] = 1;
        continue;
      }
      const i64 f = t >> (2 * l);
      const i32 A = M.tri[3 * f], B = M.tri[3 * f + 1], C = M.tri[3 * f + 2];
      const double xa = M.x[A], ya = M.y[A];
      const double ex = M.x[B] - xa, ey = M.y[B] - ya, fx = M.x[C] - xa, fy = M.y[C] - ya;
      const double det = ex * fy - fx * ey;
      const double px = ml.x[v] - xa, py = ml.y[v] - ya;
      const double li = n * ((px * fy - fx * py) / det), lj = n * ((ex * py - px * ey) / det);
      const i64 i = std::llround(li), j = std::llround(lj);
      if (std::fabs(li - i) > 1e-4 || std::fabs(lj - j) > 1e-4 || i < 0 || j < 0 || i + j > n) {
        std::lock_guard<std::mutex> lk(mx);
        bad[0] = 2;
        continue;
      }
      i64 id;
      uint8_t ty;
      if (i >= 1 && j >= 1 && i + j <= n - 1) {
        id = LL.face_start[f] + lat::rowbase((i32)j - 1, n) + (i - 1);
        ty = 0;
      } else if ((i == 0 && j == 0) || (i == n && j == 0) || (i == 0 && j == n)) {
        id = LL.vert_start[i == n ? B : (j == n ? C : A)];
        ty = 2;
      } else {
        i32 e, from;
        i64 p;
        if (j == 0) {
          e = M.fe[3 * f], from = A, p = i;
        } else if (i == 0) {
          e = M.fe[3 * f + 1], from = A, p = j;
        } else {
          e = M.fe[3 * f + 2], from = B, p = j;
        }
        const i64 kk = M.ev[2 * e] == from ? p : n - p;
        id = LL.edge_node(e, (i32)kk);
        ty = 1;
      }
      ord.old2new[v] = (i32)id;
      LL.type[id] = ty;
    }
  });
  if (bad[0]) throw std::runtime_error("lattice ordering: a node is not on its macro face's lattice");
  for (i64 v = 0; v < ml.N; ++v) {
    const i32 g = ord.old2new[v];
    if (g < 0 || ord.new2old[g] >= 0) throw std::runtime_error("lattice ordering is not a bijection");
    ord.new2old[g] = (i32)v;
  }
  ord.cuts = M.cuts;
}

std::vector<i32> lattice_faces(const Macro& M, const LatticeLevel& LL, i64 r0, i64 nrows) {
  std::vector<std::pair<i64, i32>> v;
  if (LL.F > 0)
    for (i64 f = 0; f < M.nf; ++f)
      if (LL.face_start[f] >= r0 && LL.face_start[f] < r0 + nrows) v.push_back({LL.face_start[f], (i32)f});
  std::sort(v.begin(), v.end());
  std::vector<i32> out;
  for (auto& p : v) out.push_back(p.second);
  return out;
}

void lattice_tabs(const Macro& M, const LatticeLevel& LL, const std::vector<i32>& faces, i64 row0,
                  const LocalPlan& lp, const std::vector<i32>* dof, std::vector<lat::FaceTab>& out) {
  const i32 n = LL.n;
  out.resize(faces.size());
  auto loc = [&](i64 g) -> i32 { return to_local(lp, dof ? (*dof)[g] : (i32)g); };
  for (size_t q = 0; q < faces.size(); ++q) {
    const i32 f = faces[q];
    const i32 A = M.tri[3 * f], B = M.tri[3 * f + 1];
    lat::FaceTab& T = out[q];
    T.base = row0 >= 0 ? (i32)(LL.face_start[f] - row0) : to_local(lp, (i32)LL.face_start[f]);
    T.rec = (i32)q;
    const i32 es[3] = {M.fe[3 * f], M.fe[3 * f + 1], M.fe[3 * f + 2]};
    const i32 from[3] = {A, A, B};
    int32_t* dst[3][2] = {{&T.ab0, &T.abs}, {&T.ac0, &T.acs}, {&T.bc0, &T.bcs}};
    for (int k = 0; k < 3; ++k) {
      const i32 e = es[k];
      auto node = [&](i32 p) { return LL.edge_node(e, M.ev[2 * e] == from[k] ? p : n - p); };
      const i32 a1 = loc(node(1)), a2 = n >= 3 ? loc(node(2)) : a1 + 1;
      const i32 st = a2 - a1;
      if (st != 1 && st != -1) throw std::runtime_error("lattice table: edge nodes are not contiguous");
      for (i32 p = 1; p <= n - 1; ++p)
        if (loc(node(p)) != a1 + st * (p - 1)) throw std::runtime_error("lattice table: edge nodes are not contiguous");
      *dst[k][0] = a1 - st;
      *dst[k][1] = st;
    }
  }
}

void lattice_coefs(const Macro& M, const std::vector<i32>& faces, int l, double dtnu, std::vector<double>& out) {
  out.assign(faces.size() * (size_t)lat::NCOEF, 0.0);
  for (size_t q = 0; q < faces.size(); ++q) {
    const i32 f = faces[q];
    const i32 o[3] = {M.tri[3 * f], M.tri[3 * f + 1], M.tri[3 * f + 2]};
    const double x1 = M.x[o[0]], y1 = M.y[o[0]], x2 = M.x[o[1]], y2 = M.y[o[1]], x3 = M.x[o[2]], y3 = M.y[o[2]];
    // the reference's element formulas (StokesColor.py:98-128, :130-165): K_T is scale-invariant,
    // so every small triangle of the face has the macro triangle's element matrix
    const double det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2);
    const double yd[3] = {y2 - y3, y3 - y1, y1 - y2};
    const double xd[3] = {x3 - x2, x1 - x3, x2 - x1};
    const double den = 2 * std::fabs(det);
    auto KT = [&](int p, int r) { return (yd[p] * yd[r] + xd[p] * xd[r]) / den; };
    double* c = out.data() + q * lat::NCOEF;
    // each lattice edge is shared by an "up" triangle (the face's orientation) and a "down" one (its
    // point reflection), both contributing the same element entry
    c[lat::C_KAB] = 2.0 * KT(0, 1);
    c[lat::C_KAC] = 2.0 * KT(0, 2);
    c[lat::C_KBC] = 2.0 * KT(1, 2);
    c[lat::C_KD] = 2.0 * (KT(0, 0) + KT(1, 1) + KT(2, 2));
    // level-l small triangle: det / 4^l, hat gradients 2^l (yd, xd) / det, area / 3 = |det| / (6 4^l)
    const double s4 = std::ldexp(1.0, -2 * l), s2 = std::ldexp(1.0, l);
    const double a3 = 0.5 * std::fabs(det) * s4 / 3.0;
    double gx[3], gy[3];
    for (int p = 0; p < 3; ++p) {
      gx[p] = yd[p] * s2 / det;
      gy[p] = xd[p] * s2 / det;
    }
    // G row of an interior node: a3 (g_col(up) - g_col(down)) per direction (the down triangle's
    // hat gradients are the up triangle's, negated)
    c[lat::C_G1X] = a3 * (gx[1] - gx[0]);
    c[lat::C_G1Y] = a3 * (gy[1] - gy[0]);
    c[lat::C_G2X] = a3 * (gx[2] - gx[0]);
    c[lat::C_G2Y] = a3 * (gy[2] - gy[0]);
    c[lat::C_G3X] = a3 * (gx[2] - gx[1]);
    c[lat::C_G3Y] = a3 * (gy[2] - gy[1]);
    c[lat::C_AS1] = 6.0 * a3 + 1e-12;
    c[lat::C_VD] = 1.0 + dtnu * c[lat::C_KD];
    c[lat::C_VS] = 1.0 / std::sqrt(c[lat::C_VD]);
    c[lat::C_DTNU] = dtnu;
    c[lat::C_DINV] = 1.0 / c[lat::C_KD];
  }
}

void build_dye(const HostMesh& m, const Ordering& ord, const Csr& P, const Csr& Pp, const std::vector<i32>& dof,
               DyeOp& D) {
  const i64 T = m.T, nnz = P.nnz();
  // P position of every (triangle, i, j) pair; -1 for skipped (degenerate) triangles
  std::vector<i64> tpos(9 * (size_t)T, -1);
  std::vector<double> area(T, 0.0);
  std::vector<int> bad(1, 0);
  std::mutex mx;
  parallel_for(T, [&](i64 t0, i64 t1) {
    for (i64 t = t0; t < t1; ++t) {
      const i32 o0 = m.tri[3 * t], o1 = m.tri[3 * t + 1], o2 = m.tri[3 * t + 2];
      const double x1 = m.x[o0], y1 = m.y[o0], x2 = m.x[o1], y2 = m.y[o1], x3 = m.x[o2], y3 = m.y[o2];
      const double det = x1 * (y2 - y3) + x2 * (y3 - y1) + x3 * (y1 - y2);
      if (!(std::fabs(det) >= 1e-14)) continue;
      area[t] = 0.5 * std::fabs(det);
      const i32 a[3] = {ord.old2new[o0], ord.old2new[o1], ord.old2new[o2]};
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          const i64 k = P.find(a[i], a[j]);
          if (k < 0) {
            std::lock_guard<std::mutex> lk(mx);
            bad[0] = 1;
          }
          tpos[9 * t + 3 * i + j] = k;
        }
    }
  });
  if (bad[0]) throw std::runtime_error("dye operator: a triangle pair is missing from the stiffness pattern");
  // per P entry, the contributing weights in triangle order (counting sort, stable in t)
  D.cptr.assign(nnz + 1, 0);
  for (i64 q = 0; q < 9 * T; ++q)
    if (tpos[q] >= 0) ++D.cptr[tpos[q] + 1];
  for (i64 k = 0; k < nnz; ++k) D.cptr[k + 1] += D.cptr[k];
  D.cw.assign(D.cptr[nnz], 0);
  D.mc.assign(nnz, 0.0);
  {
    std::vector<i64> fill(D.cptr.begin(), D.cptr.end() - 1);
    for (i64 t = 0; t < T; ++t)
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          const i64 k = tpos[9 * t + 3 * i + j];
          if (k < 0) continue;
          D.cw[fill[k]++] = (i32)(3 * t + j);
          D.mc[k] += (area[t] / 12.0) * (i != j ? 1.0 : 2.0);
        }
  }
  D.diag_row.assign(nnz, -1);
  for (i64 r = 0; r < P.nrows; ++r)
    for (i64 k = P.rowptr[r]; k < P.rowptr[r + 1]; ++k)
      if (P.col[k] == r) D.diag_row[k] = (i32)r;
  // merged entries: P entry k (row r, column c) -> Pp entry of (dof[r], dof[c])
  const i64 nnzp = Pp.nnz();
  std::vector<i64> e_of(nnz);
  parallel_for(P.nrows, [&](i64 r0, i64 r1) {
    for (i64 r = r0; r < r1; ++r)
      for (i64 k = P.rowptr[r]; k < P.rowptr[r + 1]; ++k) e_of[k] = Pp.find(dof[r], dof[P.col[k]]);
  });
  D.eptr.assign(nnzp + 1, 0);
  for (i64 k = 0; k < nnz; ++k) {
    if (e_of[k] < 0) throw std::runtime_error("dye operator: a merged entry is missing from the pressure pattern");
    ++D.eptr[e_of[k] + 1];
  }
  for (i64 e = 0; e < nnzp; ++e) D.eptr[e + 1] += D.eptr[e];
  D.ek.assign(nnz, 0);
  std::vector<i64> fill(D.eptr.begin(), D.eptr.end() - 1);
  for (i64 k = 0; k < nnz; ++k) D.ek[fill[e_of[k]]++] = (i32)k;
  // entries in slave columns, grouped by merged row (rows in ascending order, entries by k)
  std::vector<std::vector<std::pair<i32, i32>>> byrow;
  std::vector<i32> rowid;
  std::vector<i32> slot(P.nrows, -1);
  for (i64 r = 0; r < P.nrows; ++r)
    for (i64 k = P.rowptr[r]; k < P.rowptr[r + 1]; ++k) {
      const i32 cc = P.col[k];
      if (dof[cc] == cc) continue;
      const i32 R = dof[r];
      if (slot[R] < 0) {
        slot[R] = (i32)rowid.size();
        rowid.push_back(R);
        byrow.emplace_back();
      }
      byrow[slot[R]].push_back({(i32)k, cc});
    }
  std::vector<i32> order(rowid.size());
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](i32 a, i32 b) { return rowid[a] < rowid[b]; });
  D.srow.clear();
  D.sptr.assign(1, 0);
  D.sk.clear();
  D.sc.clear();
  for (i32 o : order) {
    auto& v = byrow[o];
    std::sort(v.begin(), v.end());
    D.srow.push_back(rowid[o]);
    for (auto& e : v) {
      D.sk.push_back(e.first);
      D.sc.push_back(e.second);
    }
    D.sptr.push_back((i64)D.sk.size());
  }
}

void lattice_locator(const Macro& M, const LatticeLevel& LL, const HostMesh& m, const Ordering& ord,
                     std::vector<lat::SlFace>& faces, std::vector<uint32_t>& cells) {
  const int l = LL.l;
  const i32 n = LL.n;
  const i64 per = (i64)1 << (2 * l);  // fine triangles per face
  if (n < 4 || m.T != M.nf * per) throw std::runtime_error("lattice locator: needs >= 2 refinement levels");
  LocalPlan gp;  // identity plan: global internal ids
  gp.r0 = 0;
  gp.r1 = m.N;
  gp.n_own = m.N;
  std::vector<i32> all(M.nf);
  std::iota(all.begin(), all.end(), 0);
  std::vector<lat::FaceTab> tabs;
  lattice_tabs(M, LL, all, -1, gp, nullptr, tabs);
  faces.assign(M.nf, lat::SlFace{});
  for (i64 f = 0; f < M.nf; ++f) {
    const i32 A = M.tri[3 * f], B = M.tri[3 * f + 1], C = M.tri[3 * f + 2];
    const double ex = M.x[B] - M.x[A], ey = M.y[B] - M.y[A], fx = M.x[C] - M.x[A], fy = M.y[C] - M.y[A];
    const double det = ex * fy - fx * ey;
    lat::SlFace& S = faces[f];
    S.ax = M.x[A];
    S.ay = M.y[A];
    S.m00 = fy / det;
    S.m01 = -fx / det;
    S.m10 = -ey / det;
    S.m11 = ex / det;
    S.tab = tabs[f];
    S.va = (i32)LL.vert_start[A];
    S.vb = (i32)LL.vert_start[B];
    S.vc = (i32)LL.vert_start[C];
    S.t0 = f * per;
  }
  // cell table from face 0: lattice coordinates of the stored vertices of its fine triangles
  cells.assign((size_t)2 * n * n, 0xffffffffu);
  const lat::SlFace& S0 = faces[0];
  auto latpt = [&](i32 v, i32& i, i32& j) {
    const double dx = m.x[v] - S0.ax, dy = m.y[v] - S0.ay;
    const double u = n * (S0.m00 * dx + S0.m01 * dy), w = n * (S0.m10 * dx + S0.m11 * dy);
    i = (i32)std::llround(u);
    j = (i32)std::llround(w);
    if (std::fabs(u - i) > 1e-4 || std::fabs(w - j) > 1e-4) throw std::runtime_error("lattice locator: off-lattice vertex");
  };
  for (i64 t = 0; t < per; ++t) {
    i32 pi[3], pj[3];
    for (int k = 0; k < 3; ++k) latpt(m.tri[3 * t + k], pi[k], pj[k]);
    const i32 i = std::min({pi[0], pi[1], pi[2]}), j = std::min({pj[0], pj[1], pj[2]});
    bool has00 = false;
    for (int k = 0; k < 3; ++k) has00 = has00 || (pi[k] == i && pj[k] == j);
    const i32 sflag = has00 ? 0 : 1;
    i32 ci[3], cj[3];
    lat::cell_vertices(i, j, sflag, ci, cj);
    int rot = -1;
    for (int r = 0; r < 3; ++r) {
      bool ok = true;
      for (int k = 0; k < 3; ++k) ok = ok && ci[(r + k) % 3] == pi[k] && cj[(r + k) % 3] == pj[k];
      if (ok) rot = r;
    }
    if (rot < 0) throw std::runtime_error("lattice locator: a fine triangle is not a rotation of its cell");
    const i64 ce = lat::cell_index(n, i, j, sflag);
    if (cells[ce] != 0xffffffffu) throw std::runtime_error("lattice locator: two triangles in one cell");
    cells[ce] = ((uint32_t)t << 2) | (uint32_t)rot;
  }
  // every face: the same local numbering (red_refine's recursion is the same for every face)
  struct Ent {
    i32 i, j, s;
    uint32_t e;
  };
  std::vector<Ent> ents;
  for (i32 j = 0; j < n; ++j)
    for (i32 i = 0; i + j <= n - 1; ++i)
      for (i32 sflag = 0; sflag < 2; ++sflag) {
        if (i + j > n - 1 - sflag) continue;
        const uint32_t e = cells[lat::cell_index(n, i, j, sflag)];
        if (e == 0xffffffffu) throw std::runtime_error("lattice locator: empty cell");
        ents.push_back({i, j, sflag, e});
      }
  if ((i64)ents.size() != per) throw std::runtime_error("lattice locator: cell count");
  std::vector<int> bad(1, 0);
  std::mutex mx;
  parallel_for(M.nf, [&](i64 f0, i64 f1) {
    for (i64 f = f0; f < f1; ++f) {
      const lat::SlFace& S = faces[f];
      for (const Ent& E : ents) {
        i32 ci[3], cj[3];
        lat::cell_vertices(E.i, E.j, E.s, ci, cj);
        const int rot = (int)(E.e & 3);
        const i64 t = S.t0 + (i64)(E.e >> 2);
        for (int k = 0; k < 3; ++k) {
          const i32 want = lat::vertex(S.tab, S.va, S.vb, S.vc, n, ci[(rot + k) % 3], cj[(rot + k) % 3]);
          if (ord.old2new[m.tri[3 * t + k]] != want) {
            std::lock_guard<std::mutex> lk(mx);
            bad[0] = 1;
          }
        }
      }
    }
  }, 1);
  if (bad[0]) throw std::runtime_error("lattice locator: a face's fine triangles do not follow face 0's numbering");
}

void lattice_apply_host(int kind, int n, const std::vector<lat::FaceTab>& tab, const std::vector<double>& coef,
                        const double* x0, const double* x1, const double* wsk, double* y,
                        const std::vector<lat::FaceTab>* tab2, int n2) {
  const i32 F = lat::interior_count(n);
  const float rinv = 1.0f / (float)(n - 1);
  for (size_t q = 0; q < tab.size(); ++q) {
    const lat::FaceTab& T = tab[q];
    if (kind >= 3) {  // transfers (pucfem_kernels_impl.hpp k_transfer)
      const lat::FaceTab& G = (*tab2)[q];
      for (i32 t = 0; t < F; ++t) {
        int32_t i, j;
        lat::coords(t, n, rinv, i, j);
        double v;
        if (kind == 3) {
          const i32 i0 = i >> 1, i1 = (i + 1) >> 1, j0 = j >> 1, j1 = (j + 1) >> 1;
          if (!(i & 1) && !(j & 1)) v = x0[lat::point(G, n2, i0, j0)];
          else if (!(j & 1)) v = 0.5 * (x0[lat::point(G, n2, i0, j0)] + x0[lat::point(G, n2, i1, j0)]);
          else if (!(i & 1)) v = 0.5 * (x0[lat::point(G, n2, i0, j0)] + x0[lat::point(G, n2, i0, j1)]);
          else v = 0.5 * (x0[lat::point(G, n2, i0, j1)] + x0[lat::point(G, n2, i1, j0)]);
        } else {
          const i32 I = 2 * i, J = 2 * j;
          v = x0[lat::point(G, n2, I, J)] +
              0.5 * (x0[lat::point(G, n2, I - 1, J)] + x0[lat::point(G, n2, I + 1, J)] + x0[lat::point(G, n2, I, J - 1)] +
                     x0[lat::point(G, n2, I, J + 1)] + x0[lat::point(G, n2, I + 1, J - 1)] +
                     x0[lat::point(G, n2, I - 1, J + 1)]);
        }
        y[T.base + t] = v;
      }
      continue;
    }
    const double* c = coef.data() + (size_t)T.rec * lat::NCOEF;
    for (i32 t = 0; t < F; ++t) {
      int32_t i, j, nb[6];
      bool in[6];
      lat::coords(t, n, rinv, i, j);
      lat::neighbours(T, n, t, i, j, nb, in);
      const i32 r = T.base + t;
      if (kind == 0) {
        y[r] = c[lat::C_KD] * x0[r] + c[lat::C_KAB] * (x0[nb[0]] + x0[nb[1]]) + c[lat::C_KAC] * (x0[nb[2]] + x0[nb[3]]) +
               c[lat::C_KBC] * (x0[nb[4]] + x0[nb[5]]);
      } else if (kind == 1) {
        y[r] = c[lat::C_G1X] * (x0[nb[1]] - x0[nb[0]]) + c[lat::C_G2X] * (x0[nb[2]] - x0[nb[3]]) +
               c[lat::C_G3X] * (x0[nb[4]] - x0[nb[5]]) + c[lat::C_G1Y] * (x1[nb[1]] - x1[nb[0]]) +
               c[lat::C_G2Y] * (x1[nb[2]] - x1[nb[3]]) + c[lat::C_G3Y] * (x1[nb[4]] - x1[nb[5]]);
      } else {
        const double vs = c[lat::C_VS];
        double w[6];
        for (int k = 0; k < 6; ++k) w[k] = (in[k] ? vs : wsk[nb[k]]) * x0[nb[k]];
        y[r] = vs * (c[lat::C_VD] * vs * x0[r] +
                     c[lat::C_DTNU] * (c[lat::C_KAB] * (w[0] + w[1]) + c[lat::C_KAC] * (w[2] + w[3]) +
                                       c[lat::C_KBC] * (w[4] + w[5])));
      }
    }
  }
}

}  // namespace pucfem
