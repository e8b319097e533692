// sph_comm.cpp — RCCL and in-process transports of the slab decomposition.
#include "sph_comm.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "sph_solver.hpp"

namespace sphx {

static void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw SphError(SPH_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

void rccl_unique_id(unsigned char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  check_nccl(ncclGetUniqueId(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, 128);
}

class RcclTransport final : public SlabTransport {
 public:
  RcclTransport(const unsigned char id[128], int r, int n) {
    rank = r;
    nranks = n;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    check_nccl(ncclCommInitRank(&comm_, n, u, r), "ncclCommInitRank");
  }
  ~RcclTransport() override {
    if (comm_) (aborted_ ? ncclCommAbort(comm_) : ncclCommDestroy(comm_));
    if (gather_) (void)hipFree(gather_);
  }
  void group_begin() override { check_nccl(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() override { check_nccl(ncclGroupEnd(), "ncclGroupEnd"); }
  void check_async() override {
    if (!comm_) throw SphError(SPH_ERR_COMM, "RCCL communicator aborted");
    ncclResult_t st = ncclSuccess;
    check_nccl(ncclCommGetAsyncError(comm_, &st), "ncclCommGetAsyncError");
    if (st != ncclSuccess && st != ncclInProgress)
      throw SphError(SPH_ERR_COMM, std::string("RCCL asynchronous error: ") + ncclGetErrorString(st));
  }
  void abort() override {
    if (comm_ && !aborted_) {
      aborted_ = true;
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  void exchange(const void* sl, size_t nsl, const void* sr, size_t nsr, void* rl, size_t nrl, void* rr, size_t nrr,
                hipStream_t s) override {
    // Point-to-point to the two x-neighbours, fused into one group (xGMI links are
    // point to point, so both faces move concurrently).
    check_nccl(ncclGroupStart(), "ncclGroupStart");
    if (has_left()) {
      if (nsl) check_nccl(ncclSend(sl, nsl, ncclChar, rank - 1, comm_, s), "ncclSend left");
      if (nrl) check_nccl(ncclRecv(rl, nrl, ncclChar, rank - 1, comm_, s), "ncclRecv left");
    }
    if (has_right()) {
      if (nsr) check_nccl(ncclSend(sr, nsr, ncclChar, rank + 1, comm_, s), "ncclSend right");
      if (nrr) check_nccl(ncclRecv(rr, nrr, ncclChar, rank + 1, comm_, s), "ncclRecv right");
    }
    check_nccl(ncclGroupEnd(), "ncclGroupEnd");
  }
  void allreduce_max_u32(unsigned* d, int n, hipStream_t s) override {
    check_nccl(ncclAllReduce(d, d, size_t(n), ncclUint32, ncclMax, comm_, s), "ncclAllReduce");
  }
  // All-gather + a rank-ordered sum on the device: the same additions, in the same order,
  // as LocalTransport's host sum (ncclAllReduce's reduction order is the library's).
  void allreduce_sum_f32(float* d, int n, hipStream_t s) override {
    const size_t need = size_t(n) * size_t(nranks);
    if (need > gathercap_) {
      check_hip(hipStreamSynchronize(s), "allreduce: sync");
      if (gather_) check_hip(hipFree(gather_), "hipFree");
      gathercap_ = need;
      check_hip(hipMalloc((void**)&gather_, sizeof(float) * gathercap_), "hipMalloc allreduce scratch");
    }
    check_nccl(ncclAllGather(d, gather_, size_t(n), ncclFloat, comm_, s), "ncclAllGather");
    launch_rank_ordered_sum(s, gather_, n, nranks, d);
  }

 private:
  ncclComm_t comm_ = nullptr;
  bool aborted_ = false;
  float* gather_ = nullptr;
  size_t gathercap_ = 0;
};

std::unique_ptr<SlabTransport> make_rccl_transport(const unsigned char id[128], int rank, int nranks) {
  return std::unique_ptr<SlabTransport>(new RcclTransport(id, rank, nranks));
}

// ---------------------------------------------------------------------------------
LocalHub::LocalHub(int nslabs) : slots(size_t(nslabs)), n(nslabs) {}

void LocalHub::barrier() {
  std::unique_lock<std::mutex> lk(m_);
  if (aborted_) throw SphError(SPH_ERR_COMM, "slab group aborted by another slab");
  const unsigned long long g = gen_;
  if (++waiting_ == n) {
    waiting_ = 0;
    gen_++;
    cv_.notify_all();
    return;
  }
  cv_.wait(lk, [&] { return gen_ != g || aborted_; });
  if (gen_ == g) throw SphError(SPH_ERR_COMM, "slab group aborted by another slab");
}

void LocalHub::abort() {
  std::lock_guard<std::mutex> lk(m_);
  aborted_ = true;
  cv_.notify_all();
}

class LocalTransport final : public SlabTransport {
 public:
  LocalTransport(std::shared_ptr<LocalHub> hub, int r) : hub_(std::move(hub)) {
    rank = r;
    nranks = hub_->n;
  }
  void exchange(const void* sl, size_t nsl, const void* sr, size_t nsr, void* rl, size_t nrl, void* rr, size_t nrr,
                hipStream_t s) override {
    check_hip(hipStreamSynchronize(s), "exchange: send buffers");
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    me.sl = sl;
    me.nsl = nsl;
    me.sr = sr;
    me.nsr = nsr;
    hub_->barrier();
    if (has_left() && nrl) {
      const LocalHub::Slot& L = hub_->slots[size_t(rank - 1)];
      if (L.nsr != nrl) throw SphError(SPH_ERR_COMM, "exchange: size mismatch with the left slab");
      check_hip(hipMemcpyAsync(rl, L.sr, nrl, hipMemcpyDeviceToDevice, s), "exchange: copy from left");
    }
    if (has_right() && nrr) {
      const LocalHub::Slot& R = hub_->slots[size_t(rank + 1)];
      if (R.nsl != nrr) throw SphError(SPH_ERR_COMM, "exchange: size mismatch with the right slab");
      check_hip(hipMemcpyAsync(rr, R.sl, nrr, hipMemcpyDeviceToDevice, s), "exchange: copy from right");
    }
    check_hip(hipStreamSynchronize(s), "exchange: copies");
    hub_->barrier();  // nobody reuses a send buffer before its copies are done
  }
  void allreduce_max_u32(unsigned* d, int n, hipStream_t s) override {
    if (n > 8) throw SphError(SPH_ERR_ARG, "allreduce: at most 8 values");
    unsigned v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    check_hip(hipMemcpyAsync(v, d, 4 * size_t(n), hipMemcpyDeviceToHost, s), "allreduce: read");
    check_hip(hipStreamSynchronize(s), "allreduce: read");
    std::memcpy(hub_->slots[size_t(rank)].vals, v, 4 * size_t(n));
    hub_->barrier();
    for (int r = 0; r < nranks; r++)
      for (int i = 0; i < n; i++) v[i] = std::max(v[i], hub_->slots[size_t(r)].vals[i]);
    hub_->barrier();
    check_hip(hipMemcpyAsync(d, v, 4 * size_t(n), hipMemcpyHostToDevice, s), "allreduce: write");
    check_hip(hipStreamSynchronize(s), "allreduce: write");
  }
  // Summed in rank order (deterministic).
  void allreduce_sum_f32(float* d, int n, hipStream_t s) override {
    std::vector<float>& mine = hub_->slots[size_t(rank)].fvals;
    mine.resize(size_t(n));
    check_hip(hipMemcpyAsync(mine.data(), d, 4 * size_t(n), hipMemcpyDeviceToHost, s), "allreduce: read");
    check_hip(hipStreamSynchronize(s), "allreduce: read");
    hub_->barrier();
    std::vector<float> v(size_t(n), 0.f);
    for (int r = 0; r < nranks; r++)
      for (int i = 0; i < n; i++) v[size_t(i)] += hub_->slots[size_t(r)].fvals[size_t(i)];
    hub_->barrier();
    check_hip(hipMemcpyAsync(d, v.data(), 4 * size_t(n), hipMemcpyHostToDevice, s), "allreduce: write");
    check_hip(hipStreamSynchronize(s), "allreduce: write");
  }

 private:
  std::shared_ptr<LocalHub> hub_;
};

std::unique_ptr<SlabTransport> make_local_transport(std::shared_ptr<LocalHub> hub, int rank) {
  return std::unique_ptr<SlabTransport>(new LocalTransport(std::move(hub), rank));
}

}  // namespace sphx
