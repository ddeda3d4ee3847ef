// Lattice face-stencil lab: variants of the fp32 Chebyshev smoothing step on the interior rows of
// synthetic macro faces (the finest level's shape: 1734 faces of n = 128), against a pure streaming
// kernel with the same bytes.  Prints us per launch and GB/s on the algorithmic bytes (x, b, d read;
// d, x written: 20 B per row).
//   hipcc -O3 --offload-arch=gfx950 -I../include tools/face_lab.hip -o face_lab && ./face_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../puc-fluidsimulation-project_amd/csrc/pucfem_lattice.hpp"

using namespace pucfem;
#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr int BS = 256;

struct Coef {
  float kd, kab, kac, kbc, dinv;
};

// V0: one row per thread per iteration, RPT rows per thread (rolled), like the library's face_rows
template <int RPT>
__global__ __launch_bounds__(BS) void v0(const lat::FaceTab* tab, const Coef* cf, int nf, int n, int F, int cpf,
                                         float rinv, const float* __restrict__ xin, const float* __restrict__ b,
                                         float* __restrict__ d, float* __restrict__ xout, float c1, float c2) {
  const int items = nf * cpf;
  int it = blockIdx.x;
  {
    const int x = it & 7, q = items >> 3, rem = items & 7;
    it = x * q + (x < rem ? x : rem) + (it >> 3);
  }
  const int lf = it / cpf;
  const int t0 = (it - lf * cpf) * (BS * RPT) + threadIdx.x;
  const lat::FaceTab T = tab[lf];
  const Coef c = cf[lf];
  for (int r = 0; r < RPT; ++r) {
    const int t = t0 + r * BS;
    if (t >= F) break;
    int i, j, nb[6];
    bool in[6];
    lat::coords(t, n, rinv, i, j);
    lat::neighbours(T, n, t, i, j, nb, in);
    const int row = T.base + t;
    const float ax = c.kd * xin[row] + c.kab * (xin[nb[0]] + xin[nb[1]]) + c.kac * (xin[nb[2]] + xin[nb[3]]) +
                     c.kbc * (xin[nb[4]] + xin[nb[5]]);
    const float dn = c1 * d[row] + c2 * c.dinv * (b[row] - ax);
    d[row] = dn;
    xout[row] = xin[row] + dn;
  }
}

// V1: RPT rows per thread, every load of all RPT rows issued before the arithmetic
template <int RPT>
__global__ __launch_bounds__(BS) void v1(const lat::FaceTab* tab, const Coef* cf, int nf, int n, int F, int cpf,
                                         float rinv, const float* __restrict__ xin, const float* __restrict__ b,
                                         float* __restrict__ d, float* __restrict__ xout, float c1, float c2) {
  const int items = nf * cpf;
  int it = blockIdx.x;
  {
    const int x = it & 7, q = items >> 3, rem = items & 7;
    it = x * q + (x < rem ? x : rem) + (it >> 3);
  }
  const int lf = it / cpf;
  const int t0 = (it - lf * cpf) * (BS * RPT) + threadIdx.x;
  const lat::FaceTab T = tab[lf];
  const Coef c = cf[lf];
  float v[RPT][7], bb[RPT], dd[RPT];
  int rows[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    int t = t0 + r * BS;
    const bool ok = t < F;
    if (!ok) t = F - 1;
    int i, j, nb[6];
    bool in[6];
    lat::coords(t, n, rinv, i, j);
    lat::neighbours(T, n, t, i, j, nb, in);
    rows[r] = ok ? T.base + t : -1;
    const int row = T.base + t;
    v[r][0] = xin[row];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[r][1 + k] = xin[nb[k]];
    bb[r] = b[row];
    dd[r] = d[row];
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    if (rows[r] < 0) continue;
    const float ax = c.kd * v[r][0] + c.kab * (v[r][1] + v[r][2]) + c.kac * (v[r][3] + v[r][4]) + c.kbc * (v[r][5] + v[r][6]);
    const float dn = c1 * dd[r] + c2 * c.dinv * (bb[r] - ax);
    d[rows[r]] = dn;
    xout[rows[r]] = v[r][0] + dn;
  }
}

// fp64 CG direction (k_cg_dir face rows): p = r + beta po gathered at the 7 points, q = A p,
// pn = p, partial <p, q>.  A: rolled RPT loop; B: RPT rows with every load issued first
template <int RPT, bool LOADS_FIRST>
__global__ __launch_bounds__(BS) void cgdir(const lat::FaceTab* tab, const Coef* cf, int nf, int n, int F, int cpf,
                                            float rinv, const double* __restrict__ r, const double* __restrict__ po,
                                            double* __restrict__ pn, double* __restrict__ q, double beta, double* part) {
  __shared__ double sh[4];
  const int items = nf * cpf;
  double acc = 0.0;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int lf = it / cpf;
    const int t0 = (it - lf * cpf) * (BS * RPT) + threadIdx.x;
    const lat::FaceTab T = tab[lf];
    const Coef c = cf[lf];
    if constexpr (!LOADS_FIRST) {
      for (int rr = 0; rr < RPT; ++rr) {
        const int t = t0 + rr * BS;
        if (t >= F) break;
        int i, j, nb[6];
        bool in[6];
        lat::coords(t, n, rinv, i, j);
        lat::neighbours(T, n, t, i, j, nb, in);
        const int row = T.base + t;
        double g[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[k] = r[nb[k]] + beta * po[nb[k]];
        const double p = r[row] + beta * po[row];
        const double qq = c.kd * p + c.kab * (g[0] + g[1]) + c.kac * (g[2] + g[3]) + c.kbc * (g[4] + g[5]);
        pn[row] = p;
        q[row] = qq;
        acc += p * qq;
      }
    } else {
      double g[RPT][7];
      int rows[RPT];
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        int t = t0 + rr * BS;
        const bool ok = t < F;
        if (!ok) t = F - 1;
        int i, j, nb[6];
        bool in[6];
        lat::coords(t, n, rinv, i, j);
        lat::neighbours(T, n, t, i, j, nb, in);
        rows[rr] = ok ? T.base + t : -1;
        const int row = T.base + t;
        g[rr][0] = r[row] + beta * po[row];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[rr][1 + k] = r[nb[k]] + beta * po[nb[k]];
      }
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        if (rows[rr] < 0) continue;
        const double p = g[rr][0];
        const double qq = c.kd * p + c.kab * (g[rr][1] + g[rr][2]) + c.kac * (g[rr][3] + g[rr][4]) +
                          c.kbc * (g[rr][5] + g[rr][6]);
        pn[rows[rr]] = p;
        q[rows[rr]] = qq;
        acc += p * qq;
      }
    }
  }
  double v = acc;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// variants of the gather: MODE 0 one fp64 array (p precomputed); 1 AoS {r, po} pairs (one 16-B load
// per point); 2 two fp32 arrays
template <int MODE>
__global__ __launch_bounds__(BS) void cgdir2(const lat::FaceTab* tab, const Coef* cf, int nf, int n, int F, int cpf,
                                             float rinv, const double* __restrict__ r, const double2* __restrict__ rp,
                                             const float* __restrict__ rf, const float* __restrict__ pf,
                                             double* __restrict__ pn, double* __restrict__ q, double beta, double* part) {
  __shared__ double sh[4];
  const int items = nf * cpf;
  double acc = 0.0;
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int lf = it / cpf;
    const int t0 = (it - lf * cpf) * (BS * 4) + threadIdx.x;
    const lat::FaceTab T = tab[lf];
    const Coef c = cf[lf];
    for (int rr = 0; rr < 4; ++rr) {
      const int t = t0 + rr * BS;
      if (t >= F) break;
      int i, j, nb[6];
      bool in[6];
      lat::coords(t, n, rinv, i, j);
      lat::neighbours(T, n, t, i, j, nb, in);
      const int row = T.base + t;
      double g[7];
      if (MODE == 0) {
        g[0] = r[row];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[1 + k] = r[nb[k]];
      } else if (MODE == 1) {
        const double2 a = rp[row];
        g[0] = a.x + beta * a.y;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const double2 b2 = rp[nb[k]];
          g[1 + k] = b2.x + beta * b2.y;
        }
      } else {
        g[0] = rf[row] + beta * pf[row];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[1 + k] = rf[nb[k]] + beta * pf[nb[k]];
      }
      const double qq = c.kd * g[0] + c.kab * (g[1] + g[2]) + c.kac * (g[3] + g[4]) + c.kbc * (g[5] + g[6]);
      pn[row] = g[0];
      q[row] = qq;
      acc += g[0] * qq;
    }
  }
  double v = acc;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// isolate the fp64 direction kernel's cost: FLAGS bit 0 = partial reduction, 1 = pn store, 2 = q store,
// 3 = swizzled one-item-per-block grid (else grid-stride over a 4096-block grid), 4 = fp32 output
template <int FLAGS>
__global__ __launch_bounds__(BS) void cgx(const lat::FaceTab* tab, const Coef* cf, int nf, int n, int F, int cpf,
                                          float rinv, const double* __restrict__ r, double* __restrict__ pn,
                                          double* __restrict__ q, float* __restrict__ qf, double* part) {
  __shared__ double sh[4];
  const int items = nf * cpf;
  double acc = 0.0;
  int it0 = blockIdx.x, stride = gridDim.x;
  if (FLAGS & 8) {
    const int x = it0 & 7, qq = items >> 3, rem = items & 7;
    it0 = x * qq + (x < rem ? x : rem) + (it0 >> 3);
    stride = items + 1;
  }
  if (FLAGS & 64) stride = items + 1;  // natural order: one item per block, block b = item b
  for (int it = it0; it < items; it += stride) {
    const int lf = it / cpf;
    const int t0 = (it - lf * cpf) * (BS * 4) + threadIdx.x;
    const lat::FaceTab T = tab[lf];
    const Coef c = cf[lf];
    for (int rr = 0; rr < 4; ++rr) {
      const int t = t0 + rr * BS;
      if (t >= F) break;
      int i, j, nb[6];
      bool in[6];
      lat::coords(t, n, rinv, i, j);
      lat::neighbours(T, n, t, i, j, nb, in);
      const int row = T.base + t;
      double g[7];
      g[0] = r[row];
#pragma unroll
      for (int k = 0; k < 6; ++k) g[1 + k] = r[nb[k]];
      const double v = c.kd * g[0] + c.kab * (g[1] + g[2]) + c.kac * (g[3] + g[4]) + c.kbc * (g[5] + g[6]);
      if (FLAGS & 32) {
        reinterpret_cast<double2*>(pn)[row] = make_double2(g[0], v);
        continue;
      }
      if (FLAGS & 128) {
        __builtin_nontemporal_store(g[0], pn + row);
        __builtin_nontemporal_store(v, q + row);
      } else {
        if (FLAGS & 2) pn[row] = g[0];
        if (FLAGS & 4) {
          if (FLAGS & 16) qf[row] = (float)v;
          else q[row] = v;
        }
      }
      if (FLAGS & 1) acc += g[0] * v;
    }
  }
  if (FLAGS & 1) {
    double v = acc;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  }
}

__global__ __launch_bounds__(BS) void stream64(int64_t n, const double* __restrict__ r, double* __restrict__ pn,
                                               double* __restrict__ q) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
    const double v = r[i];
    pn[i] = v;
    q[i] = 2.0 * v;
  }
}

// streaming reference: the same bytes, no gathers
__global__ __launch_bounds__(BS) void stream(int64_t n, const float* __restrict__ xin, const float* __restrict__ b,
                                             float* __restrict__ d, float* __restrict__ xout, float c1, float c2) {
  for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < n; r += (int64_t)gridDim.x * BS) {
    const float dn = c1 * d[r] + c2 * (b[r] - xin[r]);
    d[r] = dn;
    xout[r] = xin[r] + dn;
  }
}

int main() {
  const int nf = 1734, n = 128, F = lat::interior_count(n);
  const int64_t rows = (int64_t)nf * F;
  const int64_t skel = 400000;  // edge nodes after the faces
  const int64_t N = rows + skel;
  std::vector<lat::FaceTab> tab(nf);
  for (int f = 0; f < nf; ++f) {
    tab[f].base = f * F;
    // three edges of this face: distinct skeleton slots (reads only)
    const int64_t e0 = rows + (int64_t)(f % 1000) * 3 * (n - 1);
    tab[f].ab0 = (int32_t)(e0 - 1);
    tab[f].abs = 1;
    tab[f].ac0 = (int32_t)(e0 + (n - 1) - 1);
    tab[f].acs = 1;
    tab[f].bc0 = (int32_t)(e0 + 2 * (n - 1) + n - 1);
    tab[f].bcs = -1;
    tab[f].rec = f;
  }
  std::vector<Coef> cf(nf, Coef{6.0f, -1.0f, -1.0f, -1.0f, 1.0f / 6.0f});
  lat::FaceTab* dtab;
  Coef* dcf;
  float *x, *b, *d, *xo;
  CK(hipMalloc(&dtab, nf * sizeof(lat::FaceTab)));
  CK(hipMalloc(&dcf, nf * sizeof(Coef)));
  CK(hipMemcpy(dtab, tab.data(), nf * sizeof(lat::FaceTab), hipMemcpyHostToDevice));
  CK(hipMemcpy(dcf, cf.data(), nf * sizeof(Coef), hipMemcpyHostToDevice));
  for (float** p : {&x, &b, &d, &xo}) {
    CK(hipMalloc(p, N * sizeof(float)));
    CK(hipMemset(*p, 0, N * sizeof(float)));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 20.0 * (double)rows;
  const float rinv = 1.0f / (float)(n - 1);
  auto timeit = [&](const char* name, auto&& launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    const int it = 50;
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / it;
    std::printf("%-28s %8.1f us  %7.0f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  timeit("stream (same bytes)", [&] { hipLaunchKernelGGL(stream, dim3(8192), dim3(BS), 0, 0, rows, x, b, d, xo, 0.3f, 0.7f); });
  auto run0 = [&](auto rpt, const char* nm) {
    constexpr int R = decltype(rpt)::value;
    const int cpf = (F + BS * R - 1) / (BS * R);
    timeit(nm, [&] {
      hipLaunchKernelGGL(v0<R>, dim3(nf * cpf), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf, rinv, x, b, d, xo, 0.3f, 0.7f);
    });
  };
  auto run1 = [&](auto rpt, const char* nm) {
    constexpr int R = decltype(rpt)::value;
    const int cpf = (F + BS * R - 1) / (BS * R);
    timeit(nm, [&] {
      hipLaunchKernelGGL(v1<R>, dim3(nf * cpf), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf, rinv, x, b, d, xo, 0.3f, 0.7f);
    });
  };
  run0(std::integral_constant<int, 1>{}, "v0 rolled RPT=1");
  run0(std::integral_constant<int, 4>{}, "v0 rolled RPT=4");
  run0(std::integral_constant<int, 8>{}, "v0 rolled RPT=8");
  run1(std::integral_constant<int, 2>{}, "v1 loads-first RPT=2");
  run1(std::integral_constant<int, 4>{}, "v1 loads-first RPT=4");
  run1(std::integral_constant<int, 8>{}, "v1 loads-first RPT=8");
  // fp64 direction kernel: r, po read, pn, q written (32 B per row)
  double *r, *po, *pn, *q, *part;
  for (double** p : {&r, &po, &pn, &q}) {
    CK(hipMalloc(p, N * sizeof(double)));
    CK(hipMemset(*p, 0, N * sizeof(double)));
  }
  CK(hipMalloc(&part, 65536 * sizeof(double)));
  const double bytes64 = 32.0 * (double)rows;
  auto timed = [&](const char* name, double by, auto&& launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    const int it = 50;
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1e3 * ms / it;
    std::printf("%-28s %8.1f us  %7.0f GB/s\n", name, us, by / (us * 1e-6) / 1e9);
  };
  auto rundir = [&](auto rpt, auto lf, int grid_cap, const char* nm) {
    constexpr int R = decltype(rpt)::value;
    constexpr bool LF = decltype(lf)::value;
    const int cpf = (F + BS * R - 1) / (BS * R);
    const int grid = std::min(nf * cpf, grid_cap);
    timed(nm, bytes64, [&] {
      hipLaunchKernelGGL((cgdir<R, LF>), dim3(grid), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf, rinv, r, po, pn, q, 0.5,
                         part);
    });
  };
  using I1 = std::integral_constant<int, 1>;
  using I4 = std::integral_constant<int, 4>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  rundir(I4{}, F_{}, 4096, "cgdir rolled RPT4 cap4096");
  rundir(I4{}, F_{}, 1 << 30, "cgdir rolled RPT4 full");
  rundir(I1{}, F_{}, 1 << 30, "cgdir rolled RPT1 full");
  rundir(I4{}, T_{}, 4096, "cgdir loads-first RPT4 cap");
  rundir(I4{}, T_{}, 1 << 30, "cgdir loads-first RPT4 full");
  double2* rp;
  float *rf, *pf;
  CK(hipMalloc(&rp, N * sizeof(double2)));
  CK(hipMemset(rp, 0, N * sizeof(double2)));
  CK(hipMalloc(&rf, N * sizeof(float)));
  CK(hipMalloc(&pf, N * sizeof(float)));
  CK(hipMemset(rf, 0, N * sizeof(float)));
  CK(hipMemset(pf, 0, N * sizeof(float)));
  const int cpf4 = (F + BS * 4 - 1) / (BS * 4);
  const int g4 = std::min(nf * cpf4, 4096);
  timed("cgdir one fp64 array", 24.0 * (double)rows, [&] {
    hipLaunchKernelGGL(cgdir2<0>, dim3(g4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, rp, rf, pf, pn, q, 0.5, part);
  });
  timed("cgdir AoS {r,po}", 32.0 * (double)rows, [&] {
    hipLaunchKernelGGL(cgdir2<1>, dim3(g4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, rp, rf, pf, pn, q, 0.5, part);
  });
  timed("cgdir two fp32 arrays", 24.0 * (double)rows, [&] {
    hipLaunchKernelGGL(cgdir2<2>, dim3(g4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, rp, rf, pf, pn, q, 0.5, part);
  });
  auto runx = [&](auto fl, const char* nm, double by) {
    constexpr int FL = decltype(fl)::value;
    const int grid = (FL & (8 | 64)) ? nf * cpf4 : g4;
    timed(nm, by, [&] {
      hipLaunchKernelGGL(cgx<FL>, dim3(grid), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, pn, q, rf, part);
    });
  };
  runx(std::integral_constant<int, 7>{}, "cgx part+pn+q (=cgdir2<0>)", 24.0 * rows);
  runx(std::integral_constant<int, 6>{}, "cgx pn+q, no partial", 24.0 * rows);
  runx(std::integral_constant<int, 4>{}, "cgx q only", 16.0 * rows);
  runx(std::integral_constant<int, 14>{}, "cgx pn+q swizzled full grid", 24.0 * rows);
  runx(std::integral_constant<int, 12>{}, "cgx q only swizzled full", 16.0 * rows);
  runx(std::integral_constant<int, 28>{}, "cgx fp32 q swizzled full", 12.0 * rows);
  runx(std::integral_constant<int, 0>{}, "cgx loads only (no stores)", 8.0 * rows);
  runx(std::integral_constant<int, 64 + 6>{}, "cgx pn+q natural full", 24.0 * rows);
  runx(std::integral_constant<int, 64 + 128>{}, "cgx pn+q nt stores natural", 24.0 * rows);
  runx(std::integral_constant<int, 128>{}, "cgx pn+q nt stores cap4096", 24.0 * rows);
  runx(std::integral_constant<int, 64 + 4>{}, "cgx q only natural full", 16.0 * rows);
  {  // AoS output {pn, q}: one 16-B store per row (pn has room for 2N doubles: q's allocation follows)
    double* big;
    CK(hipMalloc(&big, 2 * N * sizeof(double)));
    CK(hipMemset(big, 0, 2 * N * sizeof(double)));
    timed("cgx AoS {pn,q} store", 24.0 * rows, [&] {
      hipLaunchKernelGGL(cgx<32 + 8>, dim3(nf * cpf4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, big, q, rf, part);
    });
    // two arrays in one allocation, q offset by N + 8 KiB (channel-conflict check)
    double* big2;
    CK(hipMalloc(&big2, (2 * N + 4096) * sizeof(double)));
    timed("cgx pn+q one allocation +8K", 24.0 * rows, [&] {
      hipLaunchKernelGGL(cgx<14>, dim3(nf * cpf4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, big2,
                         big2 + N + 1024, rf, part);
    });
    timed("cgx pn+q one allocation +N", 24.0 * rows, [&] {
      hipLaunchKernelGGL(cgx<14>, dim3(nf * cpf4), dim3(BS), 0, 0, dtab, dcf, nf, n, F, cpf4, rinv, r, big2, big2 + N,
                         rf, part);
    });
  }
  timed("stream fp64 r -> pn, q", 24.0 * (double)rows, [&] {
    hipLaunchKernelGGL(stream64, dim3(8192), dim3(BS), 0, 0, rows, r, pn, q);
  });
  CK(hipDeviceSynchronize());
  return 0;
}
