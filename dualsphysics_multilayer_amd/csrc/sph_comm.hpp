// sph_comm.hpp — transports of the slab decomposition.
//
// A slab talks only to its two x-neighbours (rank-1, rank+1) plus one 4-value
// max-allreduce per dt.  Three implementations behind one interface:
//   * RcclTransport: one process per GPU, RCCL (ncclSend/ncclRecv in a group, point to
//     point over xGMI; ncclAllReduce max) on the solver's stream — the product path;
//   * ShmTransport: separate processes of one node through a shared-memory segment,
//     host-staged (the multi-process path where RCCL cannot run, e.g. 2 ranks on 1 GPU);
//   * LocalTransport: several slabs driven by host threads of ONE process (any
//     devices, including several slabs on one GPU), device-to-device copies through
//     a shared hub.  Used by SphSlabGroup: it runs the exact same pack / divide /
//     reduce code on a one-GPU machine, where RCCL refuses two ranks per device.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <memory>
#include <mutex>
#include <vector>

namespace sphx {

class SlabTransport {
 public:
  virtual ~SlabTransport() = default;
  // Send sl (nsl bytes) to rank-1 and sr to rank+1; receive nrl bytes from rank-1
  // into rl and nrr bytes from rank+1 into rr.  All pointers are device memory.
  // Sizes must pair up (my nsl == left's nrr).  Missing neighbours are skipped.
  virtual void exchange(const void* sl, size_t nsl, const void* sr, size_t nsr, void* rl, size_t nrl, void* rr,
                        size_t nrr, hipStream_t s) = 0;
  // In-place max over ranks of n uint32 values in device memory.
  virtual void allreduce_max_u32(unsigned* d, int n, hipStream_t s) = 0;
  // In-place sum over ranks of n floats in device memory (floating-body force sums,
  // column counts of the re-partition), added in rank order from 0.f so that both
  // transports give the same bits.
  virtual void allreduce_sum_f32(float* d, int n, hipStream_t s) = 0;
  // The same exchange in two halves: post() when the send buffers are complete on stream s
  // (nothing waits), collect() later on the same stream or one ordered after it.  RCCL and
  // the shared-memory transport move the data in collect (one send/receive group); the
  // in-process transport lets the neighbours copy from the posted buffers at once.  The
  // send buffers stay untouched until the next post of the same transport.
  virtual void post(const void* sl, size_t nsl, const void* sr, size_t nsr, hipStream_t s) {
    (void)s;
    posted_ = Posted{sl, nsl, sr, nsr};
  }
  virtual void collect(void* rl, size_t nrl, void* rr, size_t nrr, hipStream_t s) {
    exchange(posted_.sl, posted_.nsl, posted_.sr, posted_.nsr, rl, nrl, rr, nrr, s);
  }
  // Before a send buffer is freed or reallocated: the neighbours' reads of every buffer this
  // rank has sent are complete (RCCL / shm: the transfers are ordered on this rank's stream).
  virtual void drain_sends() {}
  // Stream s waits until the neighbours have read the buffers of the last post, before it
  // writes them again (RCCL / shm: a send completes in this rank's stream order already).
  virtual void wait_sends(hipStream_t s) { (void)s; }
  // Measurement mode of the in-process transport (SPH_SLAB_TURNS, SphSlabGroup): slab r's
  // interaction (kind TURN_INTERACTION) and the kernels of its divide after the exchange
  // (TURN_DIVIDE) start on the GPU after slab r-1's of the same step have ended, so one GPU
  // runs one slab's interaction (interior items + ghost transfer + face items) or divide at a
  // time, as each rank does on its own GPU.  SPH_SLAB_TURNS=2 adds the update kernels
  // (TURN_UPDATE) and the exchange's pack (TURN_PACK) to the chain (kinds in the step's cycle
  // interaction -> update -> pack -> divide): every kernel of a slab's step then runs alone on
  // the GPU but the few-us face-message / migrant copies and the unpack.  turn_wait() gates
  // the streams a and b (either may be null), turn_done() ends the turn on stream s.  No-ops
  // elsewhere.
  enum { TURN_INTERACTION = 0, TURN_UPDATE = 1, TURN_PACK = 2, TURN_DIVIDE = 3, TURN_KINDS = 4 };
  virtual bool turns() const { return false; }
  virtual void turn_wait(int kind, hipStream_t a, hipStream_t b) { (void)kind; (void)a; (void)b; }
  virtual void turn_done(int kind, hipStream_t s) { (void)kind; (void)s; }
  // Several exchanges fused into one transfer group (RCCL: ncclGroupStart/End).
  virtual void group_begin() {}
  virtual void group_end() {}
  // Raise SphError if the transport failed asynchronously (RCCL: ncclCommGetAsyncError).
  virtual void check_async() {}
  // Tear the transport down after an error (RCCL: ncclCommAbort); later calls fail.
  virtual void abort() {}
  int rank = 0, nranks = 1;
  bool has_left() const { return rank > 0; }
  bool has_right() const { return rank + 1 < nranks; }

 protected:
  struct Posted {
    const void* sl = nullptr;
    size_t nsl = 0;
    const void* sr = nullptr;
    size_t nsr = 0;
  } posted_;
};

// RCCL bootstrap: 128-byte ncclUniqueId created by rank 0 and broadcast by the host.
void rccl_unique_id(unsigned char id[128]);
std::unique_ptr<SlabTransport> make_rccl_transport(const unsigned char id[128], int rank, int nranks);

// Shared state of the in-process slabs: a generation barrier that can be aborted
// (a failing slab wakes the others instead of leaving them blocked), one mailbox per
// slab, and the point-to-point exchange state: the host threads only publish pointers,
// events and generation counters (no host thread waits for the GPU), the copies wait for
// the posting stream's event on the GPU.
class LocalHub {
 public:
  explicit LocalHub(int n);
  ~LocalHub();
  void barrier();  // throws if aborted
  void abort();
  // Block until pred() holds (evaluated under the hub lock); throws if aborted.
  template <class P>
  void wait_until(P pred) {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return aborted_ || pred(); });
    if (aborted_) throw_aborted();
  }
  template <class F>
  void publish(F f) {
    {
      std::lock_guard<std::mutex> lk(m_);
      f();
    }
    cv_.notify_all();
  }
  struct Slot {
    // exchange generation g: the buffers posted (posted >= g), the neighbours' copies of
    // them issued (consumed >= g: this slot's own copies of ITS neighbours' buffers)
    const void* sl = nullptr;
    size_t nsl = 0;
    const void* sr = nullptr;
    size_t nsr = 0;
    unsigned long long posted = 0, consumed = 0;
    hipEvent_t ready = nullptr;   // the posted buffers are complete
    hipEvent_t copied = nullptr;  // this slot's copies of the neighbours' buffers are done
    // turns (measurement mode), per kind: turns ended and the event of the last one
    unsigned long long turn[4] = {0, 0, 0, 0};
    hipEvent_t idone[4] = {nullptr, nullptr, nullptr, nullptr};
    unsigned vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<float> fvals;
    // device reductions (slabs of one GPU): this slab's values of generation parity k in
    // arbuf[k] (arcap bytes each), complete at arev[k]
    void* arbuf[2] = {nullptr, nullptr};
    size_t arcap = 0;
    hipEvent_t arev[2] = {nullptr, nullptr};
  };
  std::vector<Slot> slots;
  int n;
  int turns = 0;  // SPH_SLAB_TURNS: 1 interactions and divides, 2 every kernel of the step
  // every slab on one GPU (SphSlabGroup): the reductions stay on the device (each stream waits
  // for the other slabs' values and folds them), as RCCL's all-reduce does; else host-staged
  bool onedev = false;
  // the kind whose chain ends before a chain of `kind` starts (the step's cycle of kinds)
  int turn_prev(int kind) const {
    if (turns == 1) return kind == TURN_KIND_I ? TURN_KIND_D : TURN_KIND_I;
    return (kind + 3) % 4;
  }
  static constexpr int TURN_KIND_I = 0, TURN_KIND_D = 3;

 private:
  [[noreturn]] static void throw_aborted();
  std::mutex m_;
  std::condition_variable cv_;
  int waiting_ = 0;
  unsigned long long gen_ = 0;
  bool aborted_ = false;
};

std::unique_ptr<SlabTransport> make_local_transport(std::shared_ptr<LocalHub> hub, int rank);

// Host-staged ranks of one node over POSIX shared memory `name` (separate processes, e.g.
// several ranks on one GPU, where RCCL refuses duplicate devices): two mailboxes of
// slot_bytes per rank; rank 0 creates the segment, the others attach.
std::unique_ptr<SlabTransport> make_shm_transport(const char* name, int rank, int nranks, uint64_t slot_bytes);

}  // namespace sphx
