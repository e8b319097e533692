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
};

// RCCL bootstrap: 128-byte ncclUniqueId created by rank 0 and broadcast by the host.
void rccl_unique_id(unsigned char id[128]);
std::unique_ptr<SlabTransport> make_rccl_transport(const unsigned char id[128], int rank, int nranks);

// Shared state of the in-process slabs: a generation barrier that can be aborted
// (a failing slab wakes the others instead of leaving them blocked) and one mailbox
// per slab.
class LocalHub {
 public:
  explicit LocalHub(int n);
  void barrier();  // throws if aborted
  void abort();
  struct Slot {
    const void* sl = nullptr;
    size_t nsl = 0;
    const void* sr = nullptr;
    size_t nsr = 0;
    unsigned vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<float> fvals;
  };
  std::vector<Slot> slots;
  int n;

 private:
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
