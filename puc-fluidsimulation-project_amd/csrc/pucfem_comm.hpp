// Communication backends of libpucfem.
//
//  * NcclComm  -- RCCL over xGMI, one process per GPU (the production path).
//  * LocalComm -- W ranks inside ONE process (one host thread per context, all on the same or
//                 different devices).  Same semantics (grouped send/recv/broadcast, all-reduce),
//                 implemented with host barriers, cross-stream events and device-to-device
//                 copies.  It exists so the multi-rank code path (partition, halos, replicated
//                 pieces, reductions) can be tested bit-for-bit against the single-rank path on a
//                 one-GPU box, where RCCL refuses two ranks on one device.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace pucfem {

// element type of a point-to-point / broadcast transfer (the mixed-precision V-cycle moves fp32)
enum class Dt { F64, F32 };
inline size_t dt_size(Dt t) { return t == Dt::F64 ? 8 : 4; }
template <typename T> constexpr Dt dt_of();
template <> constexpr Dt dt_of<double>() { return Dt::F64; }
template <> constexpr Dt dt_of<float>() { return Dt::F32; }

struct Comm {
  // traffic counters of this rank (pucfem_comm_counters): all-reduce calls and values, point-to-point
  // sends / broadcasts (messages) and their bytes, grouped launches
  int64_t n_allreduce = 0, v_allreduce = 0, n_msg = 0, b_msg = 0, n_group = 0, n_bcast = 0;
  void count_ar(size_t n) { ++n_allreduce; v_allreduce += (int64_t)n; }
  void count_msg(size_t bytes) { ++n_msg; b_msg += (int64_t)bytes; }
  virtual ~Comm() {}
  virtual void allreduce(double* buf, size_t n, bool is_max, hipStream_t st) = 0;
  virtual void group_start() = 0;
  virtual void send(const void* p, size_t n, Dt t, int peer, hipStream_t st) = 0;
  virtual void recv(void* p, size_t n, Dt t, int peer, hipStream_t st) = 0;
  virtual void bcast(void* p, size_t n, Dt t, int root, hipStream_t st) = 0;  // in place
  virtual void group_end(hipStream_t st) = 0;
  template <typename T> void send(const T* p, size_t n, int peer, hipStream_t st) { send(p, n, dt_of<T>(), peer, st); }
  template <typename T> void recv(T* p, size_t n, int peer, hipStream_t st) { recv(p, n, dt_of<T>(), peer, st); }
  template <typename T> void bcast(T* p, size_t n, int root, hipStream_t st) { bcast(p, n, dt_of<T>(), root, st); }
};

inline void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

struct NcclComm : Comm {
  ncclComm_t c = nullptr;
  NcclComm(int world, const ncclUniqueId& id, int rank) { nccl_check(ncclCommInitRank(&c, world, id, rank), "init"); }
  ~NcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  void allreduce(double* buf, size_t n, bool is_max, hipStream_t st) override {
    count_ar(n);
    nccl_check(ncclAllReduce(buf, buf, n, ncclDouble, is_max ? ncclMax : ncclSum, c, st), "allreduce");
  }
  void group_start() override {
    ++n_group;
    nccl_check(ncclGroupStart(), "group start");
  }
  static ncclDataType_t nt(Dt t) { return t == Dt::F64 ? ncclDouble : ncclFloat; }
  void send(const void* p, size_t n, Dt t, int peer, hipStream_t st) override {
    count_msg(n * dt_size(t));
    nccl_check(ncclSend(p, n, nt(t), peer, c, st), "send");
  }
  void recv(void* p, size_t n, Dt t, int peer, hipStream_t st) override {
    nccl_check(ncclRecv(p, n, nt(t), peer, c, st), "recv");
  }
  void bcast(void* p, size_t n, Dt t, int root, hipStream_t st) override {
    ++n_bcast;
    nccl_check(ncclBroadcast(p, p, n, nt(t), root, c, st), "broadcast");
  }
  void group_end(hipStream_t) override { nccl_check(ncclGroupEnd(), "group end"); }
};

// ------------------------------------------------------------------------------------------------
__global__ void k_comm_reduce(int world, int is_max, size_t n, const double* const* bufs, double* out);

struct LocalShared {
  explicit LocalShared(int w) : world(w), ops(w), red(w), ready(w), done(w) {}
  int world;
  std::mutex m;
  std::condition_variable cv;
  int count = 0;
  long gen = 0;
  struct Op {
    int kind;  // 0 send, 1 recv, 2 bcast
    void* p;
    size_t n;  // bytes
    int peer;  // send/recv partner, bcast root
  };
  std::vector<std::vector<Op>> ops;
  std::vector<double*> red;
  std::vector<hipEvent_t> ready, done;
  double** dev_ptrs = nullptr;  // device copy of red[] for the reduction kernel

  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long g = gen;
    if (++count == world) {
      count = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(600), [&] { return gen != g; }))
      throw std::runtime_error("LocalComm barrier timed out (a rank stopped participating)");
  }
};

inline std::map<std::string, std::weak_ptr<LocalShared>>& local_registry() {
  static std::map<std::string, std::weak_ptr<LocalShared>> r;
  return r;
}
inline std::mutex& local_registry_mutex() {
  static std::mutex m;
  return m;
}

struct LocalComm : Comm {
  std::shared_ptr<LocalShared> S;
  int rank, world;
  std::vector<LocalShared::Op> pending;
  size_t cap = 128;       // >= 2 * PROJ_MAX + 4 (the projection's multi-dot); grows on demand (tracers)
  double* tmp = nullptr;  // reduction output, up to cap values
  double** dptrs = nullptr;

  LocalComm(const std::string& key, int w, int r) : rank(r), world(w) {
    {
      std::lock_guard<std::mutex> lk(local_registry_mutex());
      auto& wp = local_registry()[key];
      S = wp.lock();
      if (!S) {
        S = std::make_shared<LocalShared>(w);
        wp = S;
      }
    }
    if (S->world != w) throw std::runtime_error("LocalComm world mismatch");
    if (hipEventCreateWithFlags(&S->ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S->done[r], hipEventDisableTiming) != hipSuccess ||
        hipMalloc(&tmp, cap * sizeof(double)) != hipSuccess || hipMalloc(&dptrs, 64 * sizeof(double*)) != hipSuccess)
      throw std::runtime_error("LocalComm: HIP allocation failed");
    S->barrier();  // every rank has created its events
  }
  ~LocalComm() override {
    (void)hipFree(tmp);
    (void)hipFree(dptrs);
  }
  static void chk(hipError_t e) {
    if (e != hipSuccess) throw std::runtime_error(std::string("LocalComm HIP: ") + hipGetErrorString(e));
  }
  void allreduce(double* buf, size_t n, bool is_max, hipStream_t st) override {
    count_ar(n);
    if (world > 64) throw std::runtime_error("LocalComm supports <= 64 ranks");
    if (n > cap) {  // this rank's output buffer only: no other rank touches it
      chk(hipStreamSynchronize(st));
      chk(hipFree(tmp));
      cap = n;
      chk(hipMalloc(&tmp, cap * sizeof(double)));
    }
    chk(hipEventRecord(S->ready[rank], st));
    S->red[rank] = buf;
    S->barrier();
    for (int p = 0; p < world; ++p)
      if (p != rank) chk(hipStreamWaitEvent(st, S->ready[p], 0));
    chk(hipMemcpyAsync(dptrs, S->red.data(), world * sizeof(double*), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_comm_reduce, dim3(1), dim3(64), 0, st, world, is_max ? 1 : 0, n, (const double* const*)dptrs,
                       tmp);
    chk(hipGetLastError());
    chk(hipEventRecord(S->done[rank], st));
    // the host staging of dptrs must not be overwritten before the copy above executed
    chk(hipStreamSynchronize(st));
    S->barrier();
    for (int p = 0; p < world; ++p)
      if (p != rank) chk(hipStreamWaitEvent(st, S->done[p], 0));
    chk(hipMemcpyAsync(buf, tmp, n * sizeof(double), hipMemcpyDeviceToDevice, st));
    S->barrier();
  }
  void group_start() override {
    ++n_group;
    pending.clear();
  }
  void send(const void* p, size_t n, Dt t, int peer, hipStream_t) override {
    count_msg(n * dt_size(t));
    pending.push_back({0, const_cast<void*>(p), n * dt_size(t), peer});
  }
  void recv(void* p, size_t n, Dt t, int peer, hipStream_t) override {
    pending.push_back({1, p, n * dt_size(t), peer});
  }
  void bcast(void* p, size_t n, Dt t, int root, hipStream_t) override {
    ++n_bcast;
    pending.push_back({2, p, n * dt_size(t), root});
  }
  void group_end(hipStream_t st) override {
    chk(hipEventRecord(S->ready[rank], st));
    S->ops[rank] = pending;
    S->barrier();
    // recv: k-th recv from p matches p's k-th send to me; bcast: ops are issued in the same order
    std::vector<int> nrecv(world, 0);
    int nb = 0;
    for (auto& op : pending) {
      if (op.kind == 1) {
        const int p = op.peer;
        int k = nrecv[p]++, seen = 0;
        const LocalShared::Op* src = nullptr;
        for (auto& o : S->ops[p])
          if (o.kind == 0 && o.peer == rank && seen++ == k) {
            src = &o;
            break;
          }
        if (!src || src->n != op.n) throw std::runtime_error("LocalComm: unmatched send/recv");
        chk(hipStreamWaitEvent(st, S->ready[p], 0));
        chk(hipMemcpyAsync(op.p, src->p, op.n, hipMemcpyDeviceToDevice, st));
      } else if (op.kind == 2) {
        const int q = op.peer;
        int k = nb++, seen = 0;
        if (q != rank) {
          const LocalShared::Op* src = nullptr;
          for (auto& o : S->ops[q])
            if (o.kind == 2 && seen++ == k) {
              src = &o;
              break;
            }
          if (!src || src->n != op.n || src->peer != q) throw std::runtime_error("LocalComm: unmatched broadcast");
          chk(hipStreamWaitEvent(st, S->ready[q], 0));
          chk(hipMemcpyAsync(op.p, src->p, op.n, hipMemcpyDeviceToDevice, st));
        }
      }
    }
    chk(hipEventRecord(S->done[rank], st));
    S->barrier();
    for (int p = 0; p < world; ++p)
      if (p != rank) chk(hipStreamWaitEvent(st, S->done[p], 0));
    S->barrier();
    pending.clear();
  }
};

}  // namespace pucfem
