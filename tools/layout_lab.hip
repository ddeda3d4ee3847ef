// Vector-layout lab (standalone, gfx950) on the library's L7 pattern (PUCFEM_DUMP_SELL image):
// does interleaving the fields a kernel gathers together (x/y components, or the two vectors of a
// CG direction update) into one 16-byte gather pay?
//   dir<NR, AOS>: q_c = A (r_c + beta p_c), pn_c = r_c + beta p_c   (the CG direction kernel, NR RHS)
//   div<MODE>:    out = Gx ux + Gy uy  (MODE 0: all separate, 1: (gx, gy) interleaved, 2: and (ux, uy))
// fp64 values, int16 column deltas, SELL-64, one wave per slice, contiguous slices per block.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/layout_lab.hip -o tools/_bin/layout_lab
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

constexpr int BS = 256;
typedef double v2d __attribute__((ext_vector_type(2)));
template <class T>
__device__ __forceinline__ T ldnt(const T* p) {
  return __builtin_nontemporal_load(p);
}
template <int N>
struct Wn {
  static constexpr int value = N;
};
template <class F>
__device__ __forceinline__ void by_width(int w, F&& f) {
  switch (w) {
    case 6: f(Wn<6>{}); break;
    case 7: f(Wn<7>{}); break;
    case 8: f(Wn<8>{}); break;
    case 9: f(Wn<9>{}); break;
    case 10: f(Wn<10>{}); break;
    default: f(Wn<0>{}); break;
  }
}
struct Sl {
  const int64_t* off;
  const int32_t* w;
  const int16_t* c;
  int64_t ns, nr;
};
#define SLICE_LOOP                                                                              \
  const int64_t nb = gridDim.x, lb = blockIdx.x;                                                \
  const int64_t s0 = A.ns * lb / nb, s1 = A.ns * (lb + 1) / nb;                                 \
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);     \
  for (int64_t s = s0 + wv; s < s1; s += 4)

// SoA: r, p, pn, q are NR separate arrays each (stride ld); AoS (NR = 2): double2 arrays
template <int NR, bool AOS>
__global__ __launch_bounds__(BS) void k_dir(Sl A, const double* __restrict__ val, const double* __restrict__ r,
                                            const double* __restrict__ p, double* __restrict__ pn,
                                            double* __restrict__ q, int64_t ld, double beta) {
  SLICE_LOOP {
    const int64_t off = A.off[s], row = s * 64 + lane;
    const int32_t base = (int32_t)(s * 64);
    double acc[NR] = {};
    by_width(A.w[s], [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        double a[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = base + (int32_t)ldnt(A.c + e);
          a[k] = ldnt(val + e);
        }
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          if constexpr (AOS && NR == 2) {
            const double2 rj = reinterpret_cast<const double2*>(r)[cj[k]];
            const double2 pj = reinterpret_cast<const double2*>(p)[cj[k]];
            acc[0] += a[k] * (rj.x + beta * pj.x);
            acc[1] += a[k] * (rj.y + beta * pj.y);
          } else if constexpr (AOS && NR == 1) {  // r and p interleaved: (r, p) pairs
            const double2 rp = reinterpret_cast<const double2*>(r)[cj[k]];
            acc[0] += a[k] * (rp.x + beta * rp.y);
          } else {
#pragma unroll
            for (int c = 0; c < NR; ++c) acc[c] += a[k] * (r[c * ld + cj[k]] + beta * p[c * ld + cj[k]]);
          }
        }
      }
    });
    if (row < A.nr) {
      if constexpr (AOS && NR == 2) {
        const double2 rr = reinterpret_cast<const double2*>(r)[row];
        const double2 pp = reinterpret_cast<const double2*>(p)[row];
        reinterpret_cast<double2*>(pn)[row] = double2{rr.x + beta * pp.x, rr.y + beta * pp.y};
        reinterpret_cast<double2*>(q)[row] = double2{acc[0], acc[1]};
      } else if constexpr (AOS && NR == 1) {
        const double2 rp = reinterpret_cast<const double2*>(r)[row];
        pn[row] = rp.x + beta * rp.y;
        q[row] = acc[0];
      } else {
#pragma unroll
        for (int c = 0; c < NR; ++c) {
          pn[c * ld + row] = r[c * ld + row] + beta * p[c * ld + row];
          q[c * ld + row] = acc[c];
        }
      }
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(BS) void k_div(Sl A, const double* __restrict__ gx, const double* __restrict__ gy,
                                            const double* __restrict__ ux, const double* __restrict__ uy,
                                            double* __restrict__ out) {
  SLICE_LOOP {
    const int64_t off = A.off[s], row = s * 64 + lane;
    const int32_t base = (int32_t)(s * 64);
    double acc = 0.0;
    by_width(A.w[s], [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        double ax[WN], ay[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = base + (int32_t)ldnt(A.c + e);
          if constexpr (MODE == 0) {
            ax[k] = ldnt(gx + e);
            ay[k] = ldnt(gy + e);
          } else {
            const v2d g = ldnt(reinterpret_cast<const v2d*>(gx) + e);
            ax[k] = g.x;
            ay[k] = g.y;
          }
        }
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          if constexpr (MODE == 2) {
            const double2 u = reinterpret_cast<const double2*>(ux)[cj[k]];
            acc += ax[k] * u.x + ay[k] * u.y;
          } else {
            acc += ax[k] * ux[cj[k]] + ay[k] * uy[cj[k]];
          }
        }
      }
    });
    if (row < A.nr) out[row] = acc;
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  const int iters = argc > 2 ? atoi(argv[2]) : 30;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  int64_t h[3];
  if (fread(h, sizeof(h), 1, f) != 1) return 1;
  const int64_t ns = h[0], nr = h[1], pad = h[2];
  std::vector<int64_t> so(ns + 1);
  std::vector<int32_t> sw(ns), col(pad);
  std::vector<double> val(pad);
  if (fread(so.data(), 8, ns + 1, f) != (size_t)(ns + 1) || fread(sw.data(), 4, ns, f) != (size_t)ns ||
      fread(col.data(), 4, pad, f) != (size_t)pad || fread(val.data(), 8, pad, f) != (size_t)pad)
    return 1;
  fclose(f);
  std::vector<int16_t> c16(pad);
  int64_t nnz = 0;
  for (int64_t s = 0; s < ns; ++s)
    for (int64_t e = so[s]; e < so[s + 1]; ++e) {
      const int64_t l = (e - so[s]) % 64, r = s * 64 + l;
      c16[e] = r < nr ? (int16_t)(col[e] - s * 64) : 0;
      nnz += r < nr;
    }
  printf("pattern: slices %ld rows %ld entries %ld (nnz %ld)\n", (long)ns, (long)nr, (long)pad, (long)nnz);
  Sl A{};
  int64_t* dso;
  int32_t* dsw;
  int16_t* dc;
  double *dv, *dv2;
  CK(hipMalloc(&dso, 8 * (ns + 1)));
  CK(hipMalloc(&dsw, 4 * ns));
  CK(hipMalloc(&dc, 2 * pad));
  CK(hipMalloc(&dv, 8 * pad));
  CK(hipMalloc(&dv2, 16 * pad));
  CK(hipMemcpy(dso, so.data(), 8 * (ns + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsw, sw.data(), 4 * ns, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c16.data(), 2 * pad, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, val.data(), 8 * pad, hipMemcpyHostToDevice));
  std::vector<double> v2(2 * pad);
  for (int64_t e = 0; e < pad; ++e) v2[2 * e] = val[e], v2[2 * e + 1] = -val[e];
  CK(hipMemcpy(dv2, v2.data(), 16 * pad, hipMemcpyHostToDevice));
  A.off = dso;
  A.w = dsw;
  A.c = dc;
  A.ns = ns;
  A.nr = nr;
  const int64_t ld = ns * 64;
  double* vec[4];
  for (auto& p : vec) CK(hipMalloc(&p, 16 * ld));
  std::vector<double> hx(2 * ld);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  for (auto p : vec) CK(hipMemcpy(p, hx.data(), 16 * ld, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-34s %8.1f us  %7.0f GB/s  %7.1f MB\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / 1e6);
    fflush(stdout);
  };
  for (int nb : {2048, 8192}) {
    printf("-- %d blocks\n", nb);
    const double b1 = 10.0 * nnz + 32.0 * nr, b2 = 10.0 * nnz + 64.0 * nr, bd = 18.0 * nnz + 24.0 * nr;
    timeit("dir NR=1 SoA", b1, [&] {
      hipLaunchKernelGGL((k_dir<1, false>), dim3(nb), dim3(BS), 0, 0, A, dv, vec[0], vec[1], vec[2], vec[3], ld, 0.5);
    });
    timeit("dir NR=1 (r,p) interleaved", b1, [&] {
      hipLaunchKernelGGL((k_dir<1, true>), dim3(nb), dim3(BS), 0, 0, A, dv, vec[0], vec[1], vec[2], vec[3], ld, 0.5);
    });
    timeit("dir NR=2 SoA", b2, [&] {
      hipLaunchKernelGGL((k_dir<2, false>), dim3(nb), dim3(BS), 0, 0, A, dv, vec[0], vec[1], vec[2], vec[3], ld, 0.5);
    });
    timeit("dir NR=2 AoS", b2, [&] {
      hipLaunchKernelGGL((k_dir<2, true>), dim3(nb), dim3(BS), 0, 0, A, dv, vec[0], vec[1], vec[2], vec[3], ld, 0.5);
    });
    timeit("div separate", bd, [&] {
      hipLaunchKernelGGL((k_div<0>), dim3(nb), dim3(BS), 0, 0, A, dv, dv2, vec[0], vec[1], vec[2]);
    });
    timeit("div (gx,gy) interleaved", bd, [&] {
      hipLaunchKernelGGL((k_div<1>), dim3(nb), dim3(BS), 0, 0, A, dv2, dv2, vec[0], vec[1], vec[2]);
    });
    timeit("div (gx,gy) + (ux,uy) interleaved", bd, [&] {
      hipLaunchKernelGGL((k_div<2>), dim3(nb), dim3(BS), 0, 0, A, dv2, dv2, vec[0], vec[1], vec[2]);
    });
  }
  return 0;
}
