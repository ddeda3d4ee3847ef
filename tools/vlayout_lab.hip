// Two-component layout lab (standalone, gfx950): the viscous Chebyshev step of the library's face rows
// (k_vcheb: r = b - A x, d = c1 d + c2 r, x_out = x + d, for the x and y components of u) on a synthetic
// triangular lattice of the L7 size, with the two components stored
//   SoA: x0[], x1[] (two 8-B gathers per neighbour; the library's layout), or
//   AoS: x[] of double2 (one 16-B gather per neighbour).
// The same algorithmic bytes either way (x gathered once, b read, d read + written in fp32, x_out written).
// Rows are processed as in face_rows_k: 1,024-row items, 4 rows per thread (K rows loaded together).
// Timed back to back (warm MALL) and after a 1 GB buffer write (cold).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off tools/vlayout_lab.hip -o tools/_bin/vlayout_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int BS = 256, RPT = 4;
constexpr int W = 127;  // lattice row length (a face's rectangle width at L7)
struct d2 {
  double x, y;
};
template <class T>
__device__ __forceinline__ void stnt(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void nbrs(int64_t t, int64_t n, int64_t (&nb)[6]) {
  // triangular lattice: (i +- 1, j), (i, j +- 1), (i + 1, j - 1), (i - 1, j + 1), clamped at the ends
  const int64_t c[6] = {t - 1, t + 1, t - W, t + W, t - W + 1, t + W - 1};
#pragma unroll
  for (int k = 0; k < 6; ++k) nb[k] = c[k] < 0 ? 0 : (c[k] >= n ? n - 1 : c[k]);
}

template <int K>
__global__ __launch_bounds__(BS) void k_soa(int64_t n, const double* __restrict__ x0, const double* __restrict__ x1,
                                            const double* __restrict__ b0, const double* __restrict__ b1,
                                            float* __restrict__ d0, float* __restrict__ d1, double* __restrict__ o0,
                                            double* __restrict__ o1, double a0, double a1, double c1, double c2) {
  const int64_t t0 = (int64_t)blockIdx.x * BS * RPT + threadIdx.x;
#pragma unroll
  for (int g = 0; g < RPT; g += K) {
    double v0[K][7], v1[K][7], bb0[K], bb1[K];
    float dd0[K], dd1[K];
    int64_t t[K];
#pragma unroll
    for (int r = 0; r < K; ++r) {
      t[r] = t0 + (g + r) * BS;
      const int64_t tt = t[r] < n ? t[r] : n - 1;
      int64_t nb[6];
      nbrs(tt, n, nb);
      v0[r][0] = x0[tt];
      v1[r][0] = x1[tt];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        v0[r][1 + k] = x0[nb[k]];
        v1[r][1 + k] = x1[nb[k]];
      }
      bb0[r] = b0[tt];
      bb1[r] = b1[tt];
      dd0[r] = d0[tt];
      dd1[r] = d1[tt];
    }
#pragma unroll
    for (int r = 0; r < K; ++r) {
      if (t[r] >= n) continue;
      double s0 = a0 * v0[r][0], s1 = a0 * v1[r][0];
#pragma unroll
      for (int k = 1; k < 7; ++k) {
        s0 += a1 * v0[r][k];
        s1 += a1 * v1[r][k];
      }
      const float e0 = (float)(c1 * (double)dd0[r] + c2 * (bb0[r] - s0));
      const float e1 = (float)(c1 * (double)dd1[r] + c2 * (bb1[r] - s1));
      stnt(d0 + t[r], e0);
      stnt(d1 + t[r], e1);
      stnt(o0 + t[r], v0[r][0] + (double)e0);
      stnt(o1 + t[r], v1[r][0] + (double)e1);
    }
  }
}

template <int K>
__global__ __launch_bounds__(BS) void k_aos(int64_t n, const d2* __restrict__ x, const d2* __restrict__ b,
                                            float2* __restrict__ d, d2* __restrict__ o, double a0, double a1,
                                            double c1, double c2) {
  const int64_t t0 = (int64_t)blockIdx.x * BS * RPT + threadIdx.x;
#pragma unroll
  for (int g = 0; g < RPT; g += K) {
    d2 v[K][7], bb[K];
    float2 dd[K];
    int64_t t[K];
#pragma unroll
    for (int r = 0; r < K; ++r) {
      t[r] = t0 + (g + r) * BS;
      const int64_t tt = t[r] < n ? t[r] : n - 1;
      int64_t nb[6];
      nbrs(tt, n, nb);
      v[r][0] = x[tt];
#pragma unroll
      for (int k = 0; k < 6; ++k) v[r][1 + k] = x[nb[k]];
      bb[r] = b[tt];
      dd[r] = d[tt];
    }
#pragma unroll
    for (int r = 0; r < K; ++r) {
      if (t[r] >= n) continue;
      double s0 = a0 * v[r][0].x, s1 = a0 * v[r][0].y;
#pragma unroll
      for (int k = 1; k < 7; ++k) {
        s0 += a1 * v[r][k].x;
        s1 += a1 * v[r][k].y;
      }
      const float e0 = (float)(c1 * (double)dd[r].x + c2 * (bb[r].x - s0));
      const float e1 = (float)(c1 * (double)dd[r].y + c2 * (bb[r].y - s1));
      typedef float v2f __attribute__((ext_vector_type(2)));
      typedef double v2d __attribute__((ext_vector_type(2)));
      v2f de = {e0, e1};
      __builtin_nontemporal_store(de, reinterpret_cast<v2f*>(d + t[r]));
      v2d w = {v[r][0].x + (double)e0, v[r][0].y + (double)e1};
      __builtin_nontemporal_store(w, reinterpret_cast<v2d*>(o + t[r]));
    }
  }
}

__global__ void k_fill(int64_t n, double* p, double s) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
    p[i] = s * (double)(i % 1013);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 14230528;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  double *x0, *x1, *b0, *b1, *o0, *o1, *junk;
  float *d0, *d1;
  CK(hipMalloc(&x0, 16 * n));  // (AoS reuses x0 as 2n doubles)
  CK(hipMalloc(&x1, 8 * n));
  CK(hipMalloc(&b0, 16 * n));
  CK(hipMalloc(&b1, 8 * n));
  CK(hipMalloc(&o0, 16 * n));
  CK(hipMalloc(&o1, 8 * n));
  CK(hipMalloc(&d0, 8 * n));
  CK(hipMalloc(&d1, 4 * n));
  const int64_t nj = (int64_t)1 << 27;  // 1 GB
  CK(hipMalloc(&junk, 8 * nj));
  for (double* p : {x0, b0, o0}) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(BS), 0, 0, 2 * n, p, 1e-3);
  for (double* p : {x1, b1, o1}) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(BS), 0, 0, n, p, 2e-3);
  CK(hipMemset(d0, 0, 8 * n));
  CK(hipMemset(d1, 0, 4 * n));
  CK(hipDeviceSynchronize());
  const int nb = (int)((n + BS * RPT - 1) / (BS * RPT));
  const double bytes = 56.0 * (double)n;  // x gathered once (16), b (16), d read + written (8 + 8), x_out (16)
  hipEvent_t a, e;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&e));
  auto run = [&](const char* name, auto&& launch) {
    for (int cold = 0; cold < 2; ++cold) {
      float tot = 0.0f;
      for (int it = 0; it < iters; ++it) {
        if (cold) hipLaunchKernelGGL(k_fill, dim3(8192), dim3(BS), 0, 0, nj, junk, 1.0);
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(e, 0));
        CK(hipEventSynchronize(e));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, e));
        if (it > 0) tot += ms;
      }
      const double ms = tot / (iters - 1);
      printf("%-28s %-5s %8.1f us  %6.0f GB/s\n", name, cold ? "cold" : "warm", 1e3 * ms, bytes / (ms * 1e-3) / 1e9);
    }
  };
  run("SoA K=1", [&] {
    hipLaunchKernelGGL(k_soa<1>, dim3(nb), dim3(BS), 0, 0, n, x0, x1, b0, b1, d0, d1, o0, o1, 4.0, -0.5, 0.3, 0.9);
  });
  run("SoA K=2", [&] {
    hipLaunchKernelGGL(k_soa<2>, dim3(nb), dim3(BS), 0, 0, n, x0, x1, b0, b1, d0, d1, o0, o1, 4.0, -0.5, 0.3, 0.9);
  });
  run("AoS K=1", [&] {
    hipLaunchKernelGGL(k_aos<1>, dim3(nb), dim3(BS), 0, 0, n, (const d2*)x0, (const d2*)b0, (float2*)d0, (d2*)o0, 4.0,
                       -0.5, 0.3, 0.9);
  });
  run("AoS K=2", [&] {
    hipLaunchKernelGGL(k_aos<2>, dim3(nb), dim3(BS), 0, 0, n, (const d2*)x0, (const d2*)b0, (float2*)d0, (d2*)o0, 4.0,
                       -0.5, 0.3, 0.9);
  });
  return 0;
}
