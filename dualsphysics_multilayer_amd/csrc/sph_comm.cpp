// sph_comm.cpp — RCCL and in-process transports of the slab decomposition.
#include "sph_comm.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

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
LocalHub::LocalHub(int nslabs) : slots(size_t(nslabs)), n(nslabs) {
  if (const char* e = std::getenv("SPH_SLAB_TURNS")) turns = std::max(0, std::min(2, std::atoi(e)));
  if (turns) test_hook_notice("SPH_SLAB_TURNS");
}

LocalHub::~LocalHub() {
  for (Slot& sl : slots) {
    for (hipEvent_t e : {sl.ready, sl.copied, sl.idone[0], sl.idone[1], sl.idone[2], sl.idone[3], sl.arev[0], sl.arev[1]})
      if (e) (void)hipEventDestroy(e);
    for (void* b : sl.arbuf)
      if (b) (void)hipFree(b);
  }
}

void LocalHub::throw_aborted() { throw SphError(SPH_ERR_COMM, "slab group aborted by another slab"); }

void LocalHub::barrier() {
  std::unique_lock<std::mutex> lk(m_);
  if (aborted_) throw_aborted();
  const unsigned long long g = gen_;
  if (++waiting_ == n) {
    waiting_ = 0;
    gen_++;
    cv_.notify_all();
    return;
  }
  cv_.wait(lk, [&] { return gen_ != g || aborted_; });
  if (gen_ == g) throw_aborted();
}

void LocalHub::abort() {
  std::lock_guard<std::mutex> lk(m_);
  aborted_ = true;
  cv_.notify_all();
}

// In-process slabs, point to point as RCCL's send/receive: post() records an event where the
// send buffers are complete and publishes them; collect() makes the stream wait for the
// neighbours' events and copies their buffers (blit kernels: on one GPU they run in the block
// slots the interior interaction leaves free, sph_solver.cpp, at ~1 TB/s; the DMA engines,
// hipMemcpyDeviceToDeviceNoCU, moved the ghost messages at ~50 GB/s).  No host thread waits
// for the GPU: the host waits only for a neighbour's thread to have posted (or consumed), and
// a rank's next post first makes its stream wait until the neighbours' copies of its
// previous buffers are done.
class LocalTransport final : public SlabTransport {
  static constexpr hipMemcpyKind kCopyKind = hipMemcpyDeviceToDevice;

 public:
  LocalTransport(std::shared_ptr<LocalHub> hub, int r) : hub_(std::move(hub)) {
    rank = r;
    nranks = hub_->n;
  }
  void exchange(const void* sl, size_t nsl, const void* sr, size_t nsr, void* rl, size_t nrl, void* rr, size_t nrr,
                hipStream_t s) override {
    post(sl, nsl, sr, nsr, s);
    collect(rl, nrl, rr, nrr, s);
  }
  void post(const void* sl, size_t nsl, const void* sr, size_t nsr, hipStream_t s) override {
    events(s);
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    const unsigned long long g = gen_ + 1;
    // the neighbours have issued their copies of this rank's previous buffers: the stream
    // waits for them before anything is written again (the caller writes the new buffers
    // before posting them; drain_sends() covers buffers it frees or reallocates)
    reuse_guard(s);
    const hipError_t e = hipEventRecord(me.ready, s);
    check_hip(e, "exchange: post");
    hub_->publish([&] {
      me.sl = sl;
      me.nsl = has_left() ? nsl : 0;
      me.sr = sr;
      me.nsr = has_right() ? nsr : 0;
      me.posted = g;
    });
    gen_ = g;
  }
  void collect(void* rl, size_t nrl, void* rr, size_t nrr, hipStream_t s) override {
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    const unsigned long long g = gen_;
    const LocalHub::Slot* L = has_left() ? &hub_->slots[size_t(rank - 1)] : nullptr;
    const LocalHub::Slot* R = has_right() ? &hub_->slots[size_t(rank + 1)] : nullptr;
    hub_->wait_until([&] { return (!L || L->posted >= g) && (!R || R->posted >= g); });
    const bool cl = L && nrl, cr = R && nrr;
    if (cl) {
      if (L->nsr != nrl) throw SphError(SPH_ERR_COMM, "exchange: size mismatch with the left slab");
      check_hip(hipStreamWaitEvent(s, L->ready, 0), "exchange: wait left");
    }
    if (cr) {
      if (R->nsl != nrr) throw SphError(SPH_ERR_COMM, "exchange: size mismatch with the right slab");
      check_hip(hipStreamWaitEvent(s, R->ready, 0), "exchange: wait right");
    }
    if (hub_->onedev && cl && cr) {
      // both faces in one kernel, as RCCL moves a send/receive group (slabs of one GPU)
      launch_copy_pair(s, rl, L->sr, nrl, rr, R->sl, nrr);
    } else {
      if (cl) check_hip(hipMemcpyAsync(rl, L->sr, nrl, kCopyKind, s), "exchange: copy from left");
      if (cr) check_hip(hipMemcpyAsync(rr, R->sl, nrr, kCopyKind, s), "exchange: copy from right");
    }
    check_hip(hipEventRecord(me.copied, s), "exchange: copies");
    hub_->publish([&] { me.consumed = g; });
  }
  void drain_sends() override {
    if (!gen_) return;
    const unsigned long long g = gen_;
    const LocalHub::Slot* L = has_left() ? &hub_->slots[size_t(rank - 1)] : nullptr;
    const LocalHub::Slot* R = has_right() ? &hub_->slots[size_t(rank + 1)] : nullptr;
    // Each neighbour records one `copied` event per generation, so the wait below covers
    // generation g only while neither has consumed g+1 (it cannot before this rank posts g+1);
    // checked inside the hub lock, so that a change of the calling pattern fails loudly.
    bool ahead = false;
    hub_->wait_until([&] {
      const bool done = (!L || L->consumed >= g) && (!R || R->consumed >= g);
      if (done) ahead = (L && L->consumed != g) || (R && R->consumed != g);
      return done;
    });
    if (ahead) throw SphError(SPH_ERR_COMM, "exchange: a neighbour consumed a later generation before this drain");
    if (L) check_hip(hipEventSynchronize(L->copied), "exchange: drain left");
    if (R) check_hip(hipEventSynchronize(R->copied), "exchange: drain right");
  }
  void wait_sends(hipStream_t s) override {
    if (!gen_) return;
    reuse_guard(s);
  }
  bool turns() const override { return hub_->turns != 0; }
  void turn_wait(int kind, hipStream_t a, hipStream_t b) override {
    if (!active(kind)) return;
    if (has_left()) {
      const LocalHub::Slot& L = hub_->slots[size_t(rank - 1)];
      const unsigned long long t = turn_[kind] + 1;
      hub_->wait_until([&] { return L.turn[kind] >= t; });
      if (a) check_hip(hipStreamWaitEvent(a, L.idone[kind], 0), "turn: wait");
      if (b) check_hip(hipStreamWaitEvent(b, L.idone[kind], 0), "turn: wait");
    } else if (nranks > 1) {
      // the chain of one kind starts after the last slab's turn of the kind before it in the
      // step's cycle (the divides of a step all end before its first interaction, ...)
      const int other = hub_->turn_prev(kind);
      const LocalHub::Slot& Z = hub_->slots[size_t(nranks - 1)];
      const unsigned long long t = turn_[other];
      if (t) {
        hub_->wait_until([&] { return Z.turn[other] >= t; });
        if (a) check_hip(hipStreamWaitEvent(a, Z.idone[other], 0), "turn: wait");
        if (b) check_hip(hipStreamWaitEvent(b, Z.idone[other], 0), "turn: wait");
      }
    }
  }
  void turn_done(int kind, hipStream_t s) override {
    if (!active(kind)) return;
    events(s);
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    const unsigned long long t = turn_[kind] + 1;
    // the right neighbour has issued its wait for this slab's previous turn
    if (has_right()) {
      const LocalHub::Slot& R = hub_->slots[size_t(rank + 1)];
      hub_->wait_until([&] { return R.turn[kind] >= turn_[kind]; });
    }
    check_hip(hipEventRecord(me.idone[kind], s), "turn: record");
    hub_->publish([&] { me.turn[kind] = t; });
    turn_[kind] = t;
  }
  void allreduce_max_u32(unsigned* d, int n, hipStream_t s) override {
    if (n > 8) throw SphError(SPH_ERR_ARG, "allreduce: at most 8 values");
    if (device_reduce()) {
      const RankPtrs p = gather_device(d, 4 * size_t(n), s);
      launch_rank_max_u32(s, p, n, nranks, d);
      return;
    }
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
    if (device_reduce()) {
      const RankPtrs p = gather_device(d, 4 * size_t(n), s);
      launch_rank_ordered_sum(s, p, n, nranks, d);
      return;
    }
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
  // This slab's events, created on the device of its stream.
  void events(hipStream_t s) {
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    if (me.ready) return;
    int dev = 0, cur = 0;
    check_hip(hipStreamGetDevice(s, &dev), "hipStreamGetDevice");
    check_hip(hipGetDevice(&cur), "hipGetDevice");
    check_hip(hipSetDevice(dev), "hipSetDevice");
    for (hipEvent_t* e : {&me.ready, &me.copied, &me.idone[0], &me.idone[1], &me.idone[2], &me.idone[3], &me.arev[0],
                          &me.arev[1]})
      check_hip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
    check_hip(hipSetDevice(cur), "hipSetDevice");
  }
  // Before generation gen_ + 1 is posted: the neighbours consumed generation gen_ (their
  // threads issued the copies) and the stream waits until those copies are done.
  void reuse_guard(hipStream_t s) {
    if (!gen_) return;
    const unsigned long long g = gen_;
    const LocalHub::Slot* L = has_left() ? &hub_->slots[size_t(rank - 1)] : nullptr;
    const LocalHub::Slot* R = has_right() ? &hub_->slots[size_t(rank + 1)] : nullptr;
    hub_->wait_until([&] { return (!L || L->consumed >= g) && (!R || R->consumed >= g); });
    if (L) check_hip(hipStreamWaitEvent(s, L->copied, 0), "exchange: reuse left");
    if (R) check_hip(hipStreamWaitEvent(s, R->copied, 0), "exchange: reuse right");
  }
  // the kinds of the chain: interactions and divides (SPH_SLAB_TURNS=1), or all four (2)
  bool active(int kind) const {
    return hub_->turns == 2 || (hub_->turns == 1 && (kind == TURN_INTERACTION || kind == TURN_DIVIDE));
  }
  bool device_reduce() const { return hub_->onedev && nranks <= RankPtrs::MAXR; }
  // A reduction's inputs on the device, as RCCL's all-reduce keeps them: this slab's `bytes`
  // of d are copied into its buffer of the generation's parity and the event recorded; after
  // the host barrier (every slab's buffer and event of the generation published) stream s
  // waits for the other slabs' events and gets their buffers to fold.  Two parities: a slab
  // writes parity k again (generation g + 2) only after its stream has waited for every
  // slab's copy of generation g + 1, which each slab's stream issued after its fold of g; and
  // it records arev[k] again only after the barrier of g + 1, which every slab reaches after
  // issuing its waits on arev[k] of g.  A larger reduction (the same sizes on every slab, as
  // the calls are collective) first drains every slab's stream, then reallocates.
  RankPtrs gather_device(const void* d, size_t bytes, hipStream_t s) {
    events(s);
    LocalHub::Slot& me = hub_->slots[size_t(rank)];
    const int par = int(argen_ & 1ull);
    argen_++;
    if (bytes > me.arcap) {
      check_hip(hipStreamSynchronize(s), "allreduce: grow");
      hub_->barrier();  // no slab reads the old buffers any more
      for (void*& b : me.arbuf) {
        if (b) check_hip(hipFree(b), "hipFree");
        b = nullptr;
      }
      const size_t cap = std::max<size_t>(256, bytes + bytes / 2);
      for (void*& b : me.arbuf) check_hip(hipMalloc(&b, cap), "hipMalloc allreduce buffer");
      me.arcap = cap;
    }
    check_hip(hipMemcpyAsync(me.arbuf[par], d, bytes, hipMemcpyDeviceToDevice, s), "allreduce: stage");
    check_hip(hipEventRecord(me.arev[par], s), "allreduce: event");
    hub_->barrier();
    RankPtrs p{};
    for (int q = 0; q < nranks; q++) {
      const LocalHub::Slot& o = hub_->slots[size_t(q)];
      p.p[q] = o.arbuf[par];
      if (q != rank) check_hip(hipStreamWaitEvent(s, o.arev[par], 0), "allreduce: wait");
    }
    return p;
  }
  std::shared_ptr<LocalHub> hub_;
  unsigned long long gen_ = 0, turn_[4] = {0, 0, 0, 0}, argen_ = 0;
};

std::unique_ptr<SlabTransport> make_local_transport(std::shared_ptr<LocalHub> hub, int rank) {
  return std::unique_ptr<SlabTransport>(new LocalTransport(std::move(hub), rank));
}

// ---------------------------------------------------------------------------------
// Host-staged transport over a POSIX shared-memory segment: ranks of one node (separate
// processes, any devices, several ranks on one GPU included) without RCCL.  Layout: a
// 4 KiB head (generation counters, message sizes, abort flag) and per rank two mailboxes
// of `slot` bytes (data for the left / right neighbour; the left one also carries the
// values of a reduction).  Every call is synchronous: device -> mailbox, barrier, the
// neighbours' mailboxes -> device, barrier (nobody refills a mailbox before it was read).
// A barrier that waits past the deadline or sees the abort flag raises SPH_ERR_COMM
// after setting the flag, so every rank ends instead of hanging.
//
// Conformance (the precondition of the RCCL transport, whose ncclSend / ncclRecv pairs hang
// rather than fail when their sizes or order differ): every call publishes its kind, element
// count and sequence number, and after the first barrier each rank checks that its
// neighbours (an exchange) or all ranks (a reduction) are in the same call, and that every
// message a neighbour sends it has exactly the size it receives — zero-size sides included,
// which this transport could otherwise pass over silently.  SPH_COMM_LOG=<dir> (a test hook)
// also appends every call of rank r to <dir>/rank<r>.log ("seq kind nsl nsr nrl nrr" or
// "seq kind n") for an offline check of the same pairing (tests/test_gpu_slab_mp.py).
namespace {
constexpr int SHM_MAXRANKS = 64;
constexpr uint64_t SHM_MAGIC = 0x53504853484d3031ull;  // "SPHSHM01"
struct ShmHead {
  std::atomic<uint64_t> magic;
  int32_t nranks, pad;
  uint64_t slot;
  std::atomic<uint64_t> abort;
  std::atomic<uint64_t> arrive[SHM_MAXRANKS];
  uint64_t nsl[SHM_MAXRANKS], nsr[SHM_MAXRANKS];
  // conformance: every rank's current collective (kind, element count) and its sequence number
  uint64_t opkind[SHM_MAXRANKS], opseq[SHM_MAXRANKS];
};
static_assert(sizeof(ShmHead) <= 4096, "shm head");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free atomics in shared memory");
}  // namespace

class ShmTransport final : public SlabTransport {
 public:
  ShmTransport(const std::string& name, int r, int n, uint64_t slot) : name_(name) {
    rank = r;
    nranks = n;
    if (n < 1 || n > SHM_MAXRANKS || r < 0 || r >= n) throw SphError(SPH_ERR_ARG, "shm transport: invalid rank");
    if (name.empty() || name[0] != '/') throw SphError(SPH_ERR_ARG, "shm transport: the name must start with '/'");
    if (const char* e = std::getenv("SPH_COMM_TIMEOUT_S")) timeout_s_ = std::max(1.0, std::atof(e));
    bytes_ = 4096 + uint64_t(n) * 2 * slot;
    const auto t0 = std::chrono::steady_clock::now();
    if (r == 0) {
      (void)shm_unlink(name.c_str());
      const int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw SphError(SPH_ERR_COMM, "shm_open(create) " + name);
      if (ftruncate(fd, off_t(bytes_)) != 0) {
        ::close(fd);
        throw SphError(SPH_ERR_NOMEM, "shm transport: ftruncate");
      }
      map(fd);
      head_->nranks = n;
      head_->slot = slot;
      head_->abort.store(0);
      for (int k = 0; k < SHM_MAXRANKS; k++) head_->arrive[k].store(0);
      head_->magic.store(SHM_MAGIC);
    } else {
      for (;;) {  // wait for rank 0's segment
        const int fd = shm_open(name.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (fstat(fd, &st) == 0 && uint64_t(st.st_size) == bytes_) {
            map(fd);
            if (head_->magic.load() == SHM_MAGIC) break;
            unmap();
          } else {
            ::close(fd);
          }
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_)
          throw SphError(SPH_ERR_COMM, "shm transport: rank 0's segment " + name + " did not appear");
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
      if (head_->nranks != n || head_->slot != slot) throw SphError(SPH_ERR_ARG, "shm transport: layout mismatch");
    }
    slot_ = slot;
    if (const char* e = std::getenv("SPH_COMM_LOG")) {
      test_hook_notice("SPH_COMM_LOG");
      const std::string path = std::string(e) + "/rank" + std::to_string(r) + ".log";
      log_ = std::fopen(path.c_str(), "w");
      if (!log_) throw SphError(SPH_ERR_ARG, "SPH_COMM_LOG: cannot write " + path);
    }
  }
  ~ShmTransport() override {
    if (log_) std::fclose(log_);
    unmap();
    if (rank == 0) (void)shm_unlink(name_.c_str());
  }
  void check_async() override {
    if (head_->abort.load()) throw SphError(SPH_ERR_COMM, "shm transport aborted by another rank");
  }
  void abort() override { head_->abort.store(1); }
  void exchange(const void* sl, size_t nsl, const void* sr, size_t nsr, void* rl, size_t nrl, void* rr, size_t nrr,
                hipStream_t s) override {
    if (nsl > slot_ || nsr > slot_ || nrl > slot_ || nrr > slot_)
      throw SphError(SPH_ERR_NOMEM, "shm transport: message larger than the mailbox");
    check_hip(hipStreamSynchronize(s), "exchange: send buffers");
    if (has_left() && nsl) check_hip(hipMemcpy(box(rank, 0), sl, nsl, hipMemcpyDeviceToHost), "exchange: to mailbox");
    if (has_right() && nsr) check_hip(hipMemcpy(box(rank, 1), sr, nsr, hipMemcpyDeviceToHost), "exchange: to mailbox");
    head_->nsl[rank] = has_left() ? nsl : 0;
    head_->nsr[rank] = has_right() ? nsr : 0;
    announce(OP_EXCHANGE, 0);
    if (log_)
      std::fprintf(log_, "%llu X %zu %zu %zu %zu\n", (unsigned long long)seq_, has_left() ? nsl : 0,
                   has_right() ? nsr : 0, has_left() ? nrl : 0, has_right() ? nrr : 0);
    barrier();
    if (has_left()) conform(rank - 1, OP_EXCHANGE, 0, head_->nsr[rank - 1], nrl, "left");
    if (has_right()) conform(rank + 1, OP_EXCHANGE, 0, head_->nsl[rank + 1], nrr, "right");
    if (has_left() && nrl) check_hip(hipMemcpy(rl, box(rank - 1, 1), nrl, hipMemcpyHostToDevice), "exchange: from left");
    if (has_right() && nrr) check_hip(hipMemcpy(rr, box(rank + 1, 0), nrr, hipMemcpyHostToDevice), "exchange: from right");
    barrier();
  }
  void allreduce_max_u32(unsigned* d, int n, hipStream_t s) override {
    std::vector<unsigned> v(size_t(n), 0u);
    reduce_in(d, 4 * size_t(n), s, OP_MAX_U32, n);
    for (int r = 0; r < nranks; r++) {
      const unsigned* x = (const unsigned*)box(r, 0);
      for (int i = 0; i < n; i++) v[size_t(i)] = std::max(v[size_t(i)], x[i]);
    }
    reduce_out(d, v.data(), 4 * size_t(n), s);
  }
  // Summed in rank order from 0.f, as LocalTransport and launch_rank_ordered_sum do.
  void allreduce_sum_f32(float* d, int n, hipStream_t s) override {
    std::vector<float> v(size_t(n), 0.f);
    reduce_in(d, 4 * size_t(n), s, OP_SUM_F32, n);
    for (int r = 0; r < nranks; r++) {
      const float* x = (const float*)box(r, 0);
      for (int i = 0; i < n; i++) v[size_t(i)] += x[i];
    }
    reduce_out(d, v.data(), 4 * size_t(n), s);
  }

 private:
  void map(int fd) {
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw SphError(SPH_ERR_COMM, "shm transport: mmap");
    base_ = (char*)p;
    head_ = (ShmHead*)p;
  }
  void unmap() {
    if (base_) munmap(base_, bytes_);
    base_ = nullptr;
    head_ = nullptr;
  }
  char* box(int r, int side) { return base_ + 4096 + (uint64_t(r) * 2 + uint64_t(side)) * slot_; }
  void barrier() {
    const uint64_t g = ++gen_;
    head_->arrive[rank].store(g);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; spin++) {
      bool all = true;
      for (int r = 0; r < nranks && all; r++) all = head_->arrive[r].load() >= g;
      if (all) return;
      if (head_->abort.load()) throw SphError(SPH_ERR_COMM, "shm transport aborted by another rank");
      if ((spin & 255u) == 255u) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_) {
          abort();
          throw SphError(SPH_ERR_COMM, "shm transport: a rank is gone or stalled (no progress for " +
                                           std::to_string(int(timeout_s_)) + " s)");
        }
        std::this_thread::yield();
      }
    }
  }
  void reduce_in(const void* d, size_t bytes, hipStream_t s, unsigned kind, int n) {
    if (bytes > slot_) throw SphError(SPH_ERR_NOMEM, "shm transport: reduction larger than the mailbox");
    check_hip(hipStreamSynchronize(s), "allreduce: values");
    check_hip(hipMemcpy(box(rank, 0), d, bytes, hipMemcpyDeviceToHost), "allreduce: read");
    announce(kind, unsigned(n));
    if (log_) std::fprintf(log_, "%llu %c %d\n", (unsigned long long)seq_, kind == OP_MAX_U32 ? 'M' : 'S', n);
    barrier();
    for (int r = 0; r < nranks; r++)
      if (r != rank) conform(r, kind, unsigned(n), 0, 0, "reduction");
  }
  // conformance (above): this rank's call, then the check of a peer's after the barrier
  enum : unsigned { OP_EXCHANGE = 1, OP_MAX_U32 = 2, OP_SUM_F32 = 3 };
  void announce(unsigned kind, unsigned n) {
    seq_++;
    head_->opkind[rank] = (uint64_t(kind) << 32) | n;
    head_->opseq[rank] = seq_;
  }
  void conform(int peer, unsigned kind, unsigned n, uint64_t peer_sends, uint64_t i_receive, const char* side) {
    const uint64_t k = head_->opkind[peer], q = head_->opseq[peer];
    if (q != seq_ || k != ((uint64_t(kind) << 32) | n)) {
      abort();
      throw SphError(SPH_ERR_COMM, std::string("slab transport conformance: rank ") + std::to_string(peer) +
                                       " is in another collective (call " + std::to_string(q) + " kind " +
                                       std::to_string(k >> 32) + ") than rank " + std::to_string(rank) +
                                       " (call " + std::to_string(seq_) + " kind " + std::to_string(kind) + ")");
    }
    if (kind == OP_EXCHANGE && peer_sends != i_receive) {
      abort();
      throw SphError(SPH_ERR_COMM, std::string("slab transport conformance: the ") + side + " rank sends " +
                                       std::to_string(peer_sends) + " bytes where rank " + std::to_string(rank) +
                                       " receives " + std::to_string(i_receive) + " (call " + std::to_string(seq_) +
                                       ")");
    }
  }
  void reduce_out(void* d, const void* v, size_t bytes, hipStream_t s) {
    barrier();  // every rank has read every mailbox
    check_hip(hipMemcpyAsync(d, v, bytes, hipMemcpyHostToDevice, s), "allreduce: write");
    check_hip(hipStreamSynchronize(s), "allreduce: write");
  }
  std::string name_;
  char* base_ = nullptr;
  ShmHead* head_ = nullptr;
  uint64_t bytes_ = 0, slot_ = 0, gen_ = 0, seq_ = 0;
  double timeout_s_ = 120.0;
  std::FILE* log_ = nullptr;
};

std::unique_ptr<SlabTransport> make_shm_transport(const char* name, int rank, int nranks, uint64_t slot_bytes) {
  return std::unique_ptr<SlabTransport>(new ShmTransport(name ? name : "", rank, nranks, slot_bytes));
}

}  // namespace sphx
