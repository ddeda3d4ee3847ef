// SpMV storage-format lab (standalone, gfx950): the multigrid smoother's access pattern
//   res[row] = b[row] - sum_k a[row,k] * x[col[row,k]]      (fp32 vectors)
// on a 7-point triangular-lattice operator of n x n nodes in strip (row-major) order -- the same
// nnz/row (7) and band (one strip) as the red-refined meshes' pressure operator.  Variants differ
// only in how the SELL-64 index / value streams are stored and loaded:
//   classic-<I><V>: entry k of lane l at off + k*64 + l (one 4/2-byte load per entry and stream)
//   pack<P>-<I><V>: P consecutive entries of a lane in one vector load (layout [k/P][lane][P])
// and in the block -> slice mapping (contiguous per block, or contiguous per XCD).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/spmv_lab.hip -o /tmp/spmv_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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
constexpr int W = 8;  // padded slice width (7 entries + 1 pad)

template <class T>
__device__ __forceinline__ T ldnt(const T* p) {
  return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ int64_t map_block(int xcd) {
  const int64_t nb = gridDim.x, b = blockIdx.x;
  if (!xcd) return b;
  return (b % 8) * (nb / 8) + b / 8;  // blocks of one XCD (b % 8) take one contiguous range
}

// classic layout; IT = int32 (absolute) or int16 (delta from the slice's first row); VT = float / half
template <typename IT, typename VT, bool NT>
__global__ __launch_bounds__(BS) void k_classic(int64_t nslices, const IT* __restrict__ col, const VT* __restrict__ val,
                                                const float* __restrict__ x, const float* __restrict__ b,
                                                float* __restrict__ res, int xcd) {
  const int64_t lb = map_block(xcd), nb = gridDim.x;
  const int64_t s0 = nslices * lb / nb, s1 = nslices * (lb + 1) / nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t off = s * W * 64;
    const int32_t base = (int32_t)(s * 64);
    int32_t cj[W];
    VT a[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int64_t e = off + k * 64 + lane;
      const IT c = NT ? ldnt(col + e) : col[e];
      cj[k] = sizeof(IT) == 2 ? base + (int32_t)c : (int32_t)c;
      a[k] = NT ? ldnt(val + e) : val[e];
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) acc += (float)a[k] * x[cj[k]];
    const int64_t row = s * 64 + lane;
    res[row] = b[row] - acc;
  }
}

// packed: P entries of one lane per vector load.  16-bit streams: P = 4 (8 B) or 8 (16 B);
// 32-bit streams: P = 4 (16 B).
template <typename IT, typename VT, int P, bool NT>
__global__ __launch_bounds__(BS) void k_packed(int64_t nslices, const IT* __restrict__ col, const VT* __restrict__ val,
                                               const float* __restrict__ x, const float* __restrict__ b,
                                               float* __restrict__ res, int xcd) {
  using IV = IT __attribute__((ext_vector_type(P)));
  using VV = VT __attribute__((ext_vector_type(P)));
  const int64_t lb = map_block(xcd), nb = gridDim.x;
  const int64_t s0 = nslices * lb / nb, s1 = nslices * (lb + 1) / nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const IV* colv = reinterpret_cast<const IV*>(col);
  const VV* valv = reinterpret_cast<const VV*>(val);
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int64_t offv = s * (W / P) * 64;
    const int32_t base = (int32_t)(s * 64);
    int32_t cj[W];
    float a[W];
#pragma unroll
    for (int g = 0; g < W / P; ++g) {
      const int64_t e = offv + g * 64 + lane;
      const IV c = NT ? ldnt(colv + e) : colv[e];
      const VV v = NT ? ldnt(valv + e) : valv[e];
#pragma unroll
      for (int q = 0; q < P; ++q) {
        cj[g * P + q] = sizeof(IT) == 2 ? base + (int32_t)c[q] : (int32_t)c[q];
        a[g * P + q] = (float)v[q];
      }
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) acc += a[k] * x[cj[k]];
    const int64_t row = s * 64 + lane;
    res[row] = b[row] - acc;
  }
}

// int16 column deltas packed 8 per lane (one 16-B load), fp32 values packed 4 (two 16-B loads)
__global__ __launch_bounds__(BS) void k_mixed(int64_t nslices, const int16_t* __restrict__ col,
                                              const float* __restrict__ val, const float* __restrict__ x,
                                              const float* __restrict__ b, float* __restrict__ res, int xcd) {
  using IV = int16_t __attribute__((ext_vector_type(8)));
  using VV = float __attribute__((ext_vector_type(4)));
  const int64_t lb = map_block(xcd), nb = gridDim.x;
  const int64_t s0 = nslices * lb / nb, s1 = nslices * (lb + 1) / nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const IV* colv = reinterpret_cast<const IV*>(col);
  const VV* valv = reinterpret_cast<const VV*>(val);
  for (int64_t s = s0 + wv; s < s1; s += 4) {
    const int32_t base = (int32_t)(s * 64);
    const IV c = ldnt(colv + s * 64 + lane);
    const VV v0 = ldnt(valv + s * 128 + lane), v1 = ldnt(valv + s * 128 + 64 + lane);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v0[k] * x[base + (int32_t)c[k]];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v1[k] * x[base + (int32_t)c[4 + k]];
    const int64_t row = s * 64 + lane;
    res[row] = b[row] - acc;
  }
}

// Chebyshev-step-like kernel as in the library (mode 1): per-slice offset / width loads (scalar),
// width-dispatched straight-line body, row streams x_in, d, dinv, b read and d, x_out written.
// PF: prefetch the next slice's (off, w) and issue the row-stream loads before the gathers.
template <int N>
struct Wn {
  static constexpr int value = N;
};
template <class F>
__device__ __forceinline__ void by_width(int w, F&& f) {
  switch (w) {
    case 7: f(Wn<7>{}); break;
    case 8: f(Wn<8>{}); break;
    default: f(Wn<0>{}); break;
  }
}
template <bool PF>
__global__ __launch_bounds__(BS) void k_chebl(int64_t nslices, const int64_t* __restrict__ soff,
                                              const int32_t* __restrict__ sw, const int16_t* __restrict__ col,
                                              const _Float16* __restrict__ val, const float* __restrict__ xin,
                                              const float* __restrict__ dinv, const float* __restrict__ b,
                                              float* __restrict__ d, float* __restrict__ xout, float c1, float c2) {
  const int64_t nb = gridDim.x, lb = blockIdx.x;
  const int64_t s0 = nslices * lb / nb, s1 = nslices * (lb + 1) / nb;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t s = s0 + wv;
  int64_t off = s < s1 ? soff[s] : 0;
  int w = s < s1 ? sw[s] : 0;
  for (; s < s1; s += 4) {
    int64_t off_n = 0;
    int w_n = 0;
    if (PF && s + 4 < s1) {
      off_n = soff[s + 4];
      w_n = sw[s + 4];
    }
    const int64_t row = s * 64 + lane;
    const int32_t base = (int32_t)(s * 64);
    float xr = 0.f, dr = 0.f, di = 0.f, br = 0.f;
    if (PF) {
      xr = xin[row];
      dr = d[row];
      di = dinv[row];
      br = b[row];
    }
    float acc = 0.f;
    by_width(w, [&](auto wc) {
      constexpr int WN = decltype(wc)::value;
      if constexpr (WN > 0) {
        int32_t cj[WN];
        _Float16 a[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          cj[k] = base + (int32_t)ldnt(col + e);
          a[k] = ldnt(val + e);
        }
#pragma unroll
        for (int k = 0; k < WN; ++k) acc += (float)a[k] * xin[cj[k]];
      } else {
        for (int k = 0; k < w; ++k) {
          const int64_t e = off + (int64_t)k * 64 + lane;
          acc += (float)ldnt(val + e) * xin[base + (int32_t)ldnt(col + e)];
        }
      }
    });
    if (!PF) {
      xr = xin[row];
      dr = d[row];
      di = dinv[row];
      br = b[row];
    }
    const float dn = c1 * dr + c2 * di * (br - acc);
    d[row] = dn;
    xout[row] = xr + dn;
    if (PF) {
      off = off_n;
      w = w_n;
    } else if (s + 4 < s1) {
      off = soff[s + 4];
      w = sw[s + 4];
    }
  }
}

struct Mat {
  int64_t nrows, nslices;
  std::vector<int32_t> col;  // [row][W] absolute
  std::vector<float> val;
};

// 7-point triangular lattice (neighbours (+-1,0), (0,+-1), (+1,-1), (-1,+1)), Neumann-like stencil
Mat lattice(int n) {
  Mat m;
  m.nrows = (int64_t)n * n;
  m.nslices = (m.nrows + 63) / 64;
  m.col.assign(m.nslices * 64 * W, 0);
  m.val.assign(m.nslices * 64 * W, 0.f);
  const int di[6] = {1, -1, 0, 0, 1, -1}, dj[6] = {0, 0, 1, -1, -1, 1};
  for (int64_t r = 0; r < m.nslices * 64; ++r) {
    int32_t* c = &m.col[r * W];
    float* v = &m.val[r * W];
    for (int k = 0; k < W; ++k) c[k] = (int32_t)std::min<int64_t>(r, m.nrows - 1);
    if (r >= m.nrows) continue;
    const int i = (int)(r % n), j = (int)(r / n);
    int k = 0;
    float diag = 0.f;
    for (int q = 0; q < 6; ++q) {
      const int ii = i + di[q], jj = j + dj[q];
      if (ii < 0 || ii >= n || jj < 0 || jj >= n) continue;
      c[k] = jj * n + ii;
      v[k] = -1.f;
      diag += 1.f;
      ++k;
    }
    c[k] = (int32_t)r;
    v[k] = diag + 0.01f;
  }
  return m;
}

template <typename IT, typename VT>
void layout(const Mat& m, int P, std::vector<IT>& col, std::vector<VT>& val) {
  col.assign(m.col.size(), 0);
  val.assign(m.val.size(), 0);
  for (int64_t s = 0; s < m.nslices; ++s)
    for (int l = 0; l < 64; ++l)
      for (int k = 0; k < W; ++k) {
        const int64_t r = s * 64 + l;
        int64_t e;
        if (P == 1) e = s * W * 64 + (int64_t)k * 64 + l;
        else e = (s * (W / P) * 64 + (int64_t)(k / P) * 64 + l) * P + (k % P);
        const int32_t c = m.col[r * W + k];
        col[e] = sizeof(IT) == 2 ? (IT)(c - s * 64) : (IT)c;
        val[e] = (VT)m.val[r * W + k];
      }
}

// --real FILE: the library's pressure operator (PUCFEM_DUMP_SELL image) in the Chebyshev-like kernel
int run_real(const char* path, int iters) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    return 1;
  }
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
  std::vector<_Float16> v16(pad);
  for (int64_t s = 0; s < ns; ++s)
    for (int64_t e = so[s]; e < so[s + 1]; ++e) {
      const int64_t l = (e - so[s]) % 64, r = s * 64 + l;
      c16[e] = r < nr ? (int16_t)(col[e] - s * 64) : 0;
      v16[e] = (_Float16)val[e];
    }
  printf("real: slices %ld rows %ld entries %ld\n", (long)ns, (long)nr, (long)pad);
  int64_t* dso;
  int32_t* dsw;
  int16_t* dc;
  _Float16* dv;
  float *x, *dinv, *b, *d, *xo;
  CK(hipMalloc(&dso, 8 * (ns + 1)));
  CK(hipMalloc(&dsw, 4 * ns));
  CK(hipMalloc(&dc, 2 * pad));
  CK(hipMalloc(&dv, 2 * pad));
  for (float** p : {&x, &dinv, &b, &d, &xo}) CK(hipMalloc(p, 4 * ns * 64));
  CK(hipMemcpy(dso, so.data(), 8 * (ns + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsw, sw.data(), 4 * ns, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c16.data(), 2 * pad, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, v16.data(), 2 * pad, hipMemcpyHostToDevice));
  std::vector<float> hx(ns * 64);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  for (float* p : {x, dinv, b, d}) CK(hipMemcpy(p, hx.data(), 4 * hx.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int pf = 0; pf < 2; ++pf)
    for (int nb : {1024, 2048, 4096, 8192}) {
      auto launch = [&] {
        if (pf)
          hipLaunchKernelGGL((k_chebl<true>), dim3(nb), dim3(BS), 0, 0, ns, dso, dsw, dc, dv, x, dinv, b, d, xo, 0.3f,
                             0.7f);
        else
          hipLaunchKernelGGL((k_chebl<false>), dim3(nb), dim3(BS), 0, 0, ns, dso, dsw, dc, dv, x, dinv, b, d, xo, 0.3f,
                             0.7f);
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      const double bytes = 4.0 * pad + 28.0 * nr;
      printf("real cheb-like i16f16 pf%d nb%-5d %8.1f us  %7.0f GB/s  %7.1f MB\n", pf, nb, ms * 1e3,
             bytes / (ms * 1e-3) / 1e9, bytes / 1e6);
      fflush(stdout);
    }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && !strcmp(argv[1], "--real")) return run_real(argv[2], argc > 3 ? atoi(argv[3]) : 50);
  const int n = argc > 1 ? atoi(argv[1]) : 3772;  // 3772^2 = 14.2M rows (L7)
  const int iters = argc > 2 ? atoi(argv[2]) : 50;
  Mat m = lattice(n);
  const int64_t N = m.nrows, E = m.nslices * 64 * W;
  printf("rows %ld slices %ld entries %ld\n", (long)N, (long)m.nslices, (long)E);
  float *x, *b, *res;
  CK(hipMalloc(&x, 4 * m.nslices * 64));
  CK(hipMalloc(&b, 4 * m.nslices * 64));
  CK(hipMalloc(&res, 4 * m.nslices * 64));
  std::vector<float> hx(m.nslices * 64);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  CK(hipMemcpy(x, hx.data(), 4 * hx.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(b, hx.data(), 4 * hx.size(), hipMemcpyHostToDevice));
  // reference result (classic int32 / fp32) for a correctness check of every variant
  std::vector<float> ref(m.nslices * 64), got(m.nslices * 64);
  void *dc = nullptr, *dv = nullptr;
  CK(hipMalloc(&dc, 4 * E));
  CK(hipMalloc(&dv, 4 * E));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double mat_bytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    CK(hipMemcpy(got.data(), res, 4 * got.size(), hipMemcpyDeviceToHost));
    double err = 0;
    for (int64_t i = 0; i < N; ++i) err = std::max(err, (double)std::fabs(got[i] - ref[i]));
    const double bytes = mat_bytes * E + 12.0 * N;  // matrix + x, b, res
    printf("%-34s %8.1f us  %7.0f GB/s  %7.1f MB  maxerr %.1e\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / 1e6,
           err);
    fflush(stdout);
  };
  auto launch_timed = [&](const char* name, double bytes, auto launch) {
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
  const int nbs[3] = {1024, 2048, 4096};
  // int32 / fp32 classic (also the reference)
  {
    std::vector<int32_t> c;
    std::vector<float> v;
    layout(m, 1, c, v);
    CK(hipMemcpy(dc, c.data(), 4 * E, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, v.data(), 4 * E, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((k_classic<int32_t, float, true>), dim3(1024), dim3(BS), 0, 0, m.nslices, (const int32_t*)dc,
                       (const float*)dv, x, b, res, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), res, 4 * ref.size(), hipMemcpyDeviceToHost));
    for (int nb : nbs)
      for (int xcd = 0; xcd < 2; ++xcd)
        for (int nt = 0; nt < 2; ++nt) {
          char nm[96];
          snprintf(nm, sizeof nm, "classic-i32f32 nb%d xcd%d nt%d", nb, xcd, nt);
          run(nm, 8.0, [&] {
            if (nt)
              hipLaunchKernelGGL((k_classic<int32_t, float, true>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                                 (const int32_t*)dc, (const float*)dv, x, b, res, xcd);
            else
              hipLaunchKernelGGL((k_classic<int32_t, float, false>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                                 (const int32_t*)dc, (const float*)dv, x, b, res, xcd);
          });
        }
    layout(m, 4, c, v);
    CK(hipMemcpy(dc, c.data(), 4 * E, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, v.data(), 4 * E, hipMemcpyHostToDevice));
    for (int nb : nbs)
      for (int xcd = 0; xcd < 2; ++xcd) {
        char nm[96];
        snprintf(nm, sizeof nm, "pack4-i32f32 nb%d xcd%d", nb, xcd);
        run(nm, 8.0, [&] {
          hipLaunchKernelGGL((k_packed<int32_t, float, 4, true>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                             (const int32_t*)dc, (const float*)dv, x, b, res, xcd);
        });
      }
  }
  // int16 / fp16
  {
    std::vector<int16_t> c;
    std::vector<_Float16> v;
    layout(m, 1, c, v);
    CK(hipMemcpy(dc, c.data(), 2 * E, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, v.data(), 2 * E, hipMemcpyHostToDevice));
    for (int nb : nbs)
      for (int xcd = 0; xcd < 2; ++xcd) {
        char nm[96];
        snprintf(nm, sizeof nm, "classic-i16f16 nb%d xcd%d", nb, xcd);
        run(nm, 4.0, [&] {
          hipLaunchKernelGGL((k_classic<int16_t, _Float16, true>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                             (const int16_t*)dc, (const _Float16*)dv, x, b, res, xcd);
        });
      }
    for (int P : {4, 8}) {
      layout(m, P, c, v);
      CK(hipMemcpy(dc, c.data(), 2 * E, hipMemcpyHostToDevice));
      CK(hipMemcpy(dv, v.data(), 2 * E, hipMemcpyHostToDevice));
      for (int nb : nbs)
        for (int xcd = 0; xcd < 2; ++xcd) {
          char nm[96];
          snprintf(nm, sizeof nm, "pack%d-i16f16 nb%d xcd%d", P, nb, xcd);
          run(nm, 4.0, [&] {
            if (P == 4)
              hipLaunchKernelGGL((k_packed<int16_t, _Float16, 4, true>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                                 (const int16_t*)dc, (const _Float16*)dv, x, b, res, xcd);
            else
              hipLaunchKernelGGL((k_packed<int16_t, _Float16, 8, true>), dim3(nb), dim3(BS), 0, 0, m.nslices,
                                 (const int16_t*)dc, (const _Float16*)dv, x, b, res, xcd);
          });
        }
    }
    // Chebyshev-like step on a width-7 SELL (the real operator's slice width), 7 entries per row
    {
      std::vector<int64_t> so(m.nslices + 1);
      std::vector<int32_t> swv(m.nslices, 7);
      std::vector<int16_t> c7(m.nslices * 64 * 7);
      std::vector<_Float16> v7(m.nslices * 64 * 7);
      for (int64_t q = 0; q <= m.nslices; ++q) so[q] = q * 7 * 64;
      for (int64_t q = 0; q < m.nslices; ++q)
        for (int l = 0; l < 64; ++l)
          for (int k = 0; k < 7; ++k) {
            const int64_t r = q * 64 + l;
            c7[q * 7 * 64 + k * 64 + l] = (int16_t)(m.col[r * W + k] - q * 64);
            v7[q * 7 * 64 + k * 64 + l] = (_Float16)m.val[r * W + k];
          }
      int64_t *dso;
      int32_t *dsw;
      float *dd, *dxo, *ddi;
      CK(hipMalloc(&dso, 8 * so.size()));
      CK(hipMalloc(&dsw, 4 * swv.size()));
      CK(hipMalloc(&dd, 4 * m.nslices * 64));
      CK(hipMalloc(&dxo, 4 * m.nslices * 64));
      CK(hipMalloc(&ddi, 4 * m.nslices * 64));
      CK(hipMemcpy(dso, so.data(), 8 * so.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dsw, swv.data(), 4 * swv.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dc, c7.data(), 2 * c7.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dv, v7.data(), 2 * v7.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(ddi, hx.data(), 4 * hx.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dd, hx.data(), 4 * hx.size(), hipMemcpyHostToDevice));
      const double E7 = (double)m.nslices * 64 * 7;
      for (int pf = 0; pf < 2; ++pf)
        for (int nb : nbs) {
          char nm[96];
          snprintf(nm, sizeof nm, "cheb-like w7 i16f16 pf%d nb%d", pf, nb);
          // bytes: 4 per entry + rows: x gathered 4, x_in 4, d 4 + 4, dinv 4, b 4, x_out 4
          const double bytes = 4.0 * E7 + 28.0 * N;
          launch_timed(nm, bytes, [&] {
            if (pf)
              hipLaunchKernelGGL((k_chebl<true>), dim3(nb), dim3(BS), 0, 0, m.nslices, dso, dsw, (const int16_t*)dc,
                                 (const _Float16*)dv, x, ddi, b, dd, dxo, 0.3f, 0.7f);
            else
              hipLaunchKernelGGL((k_chebl<false>), dim3(nb), dim3(BS), 0, 0, m.nslices, dso, dsw, (const int16_t*)dc,
                                 (const _Float16*)dv, x, ddi, b, dd, dxo, 0.3f, 0.7f);
          });
        }
    }
    // int16 columns, fp32 values (packed 8 / 4)
    std::vector<float> vf;
    layout(m, 8, c, vf);
    std::vector<float> vf4;
    std::vector<int16_t> c8 = c;
    layout(m, 4, c, vf4);
    CK(hipMemcpy(dc, c8.data(), 2 * E, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, vf4.data(), 4 * E, hipMemcpyHostToDevice));
    for (int nb : nbs) {
      char nm[96];
      snprintf(nm, sizeof nm, "pack8i16-pack4f32 nb%d xcd1", nb);
      run(nm, 6.0, [&] {
        hipLaunchKernelGGL((k_mixed), dim3(nb), dim3(BS), 0, 0, m.nslices, (const int16_t*)dc, (const float*)dv, x, b,
                           res, 1);
      });
    }
  }
  return 0;
}
