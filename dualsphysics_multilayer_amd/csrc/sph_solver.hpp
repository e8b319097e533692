// sph_solver.hpp — C++ host orchestration of the MI355X SPH core.
//
// SphGpuSingle mirrors JSphGpuSingle (JSphGpuSingle.h:35; .cpp:331-596,808-880):
// RunCellDivide -> Interaction_Forces -> DtVariable -> ComputeVerlet /
// ComputeSymplecticPre/Corr, with the same step order.  Differences by design:
//   * dt, VelMax/AceMax/ViscDtMax and the particle counts stay on the device
//     (DevScalars); the host never blocks inside a step;
//   * the cell domain is the full map (CellDomFixed), see sph_divide.hip;
//   * buffers are owned here (one allocation per array, two sets for the sort
//     gather), the role of JArraysGpu's pools (JArraysGpu.h:134-145).
// Errors throw SphError; the C-ABI (sph_capi.cpp) turns them into SphStatus.
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sphcore.h"
#include "sph_kernels.hpp"

namespace sphx {

struct SphError : std::runtime_error {
  int status;
  SphError(int st, const std::string& m) : std::runtime_error(m), status(st) {}
};

void check_hip(hipError_t e, const char* what);
void derive_constants(const SphCaseDef& c, SphConstants& k);

class SphGpuSingle {
 public:
  SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& init, int device);
  ~SphGpuSingle();

  // Phases (JSphGpuSingle::RunCellDivide / Interaction_Forces / DtVariable / ComputeVerlet ...).
  void RunCellDivide();
  void Interaction_Forces(int interstep);
  void DtVariable(int mode);
  void ComputeVerlet();
  void ComputeSymplecticPre();
  void ComputeSymplecticCorr();
  // Whole steps: ComputeStep_Ver / ComputeStep_Sym + RunCellDivide (JSphGpuSingle.cpp:548-596,853-880).
  void ComputeStep();
  void Run(unsigned nsteps);

  void Sync();
  SphRunStats Stats();
  unsigned DtTrace(double* out, unsigned cap);
  void Download(SphParticlesHost& out);
  void DownloadInteraction(SphInterOut& out);
  void CountPairs(uint64_t out[6]);
  void SetTiming(bool on);
  void Timing(double out_ms[4], uint64_t* launches);
  void CheckErrors();

  SphConstants C{};
  KConst K{};
  DivGrid G{};
  int device = 0;
  hipStream_t stream = nullptr;

 private:
  void Alloc();
  void Free();
  void Upload(const SphParticlesHost& init);
  void TimedBegin(int phase);
  void TimedEnd(int phase);

  unsigned cap_ = 0, npb0_ = 0, keybits_ = 0;
  int step_algorithm_ = SPH_STEP_VERLET;
  int verletstep_ = 0;
  bool havepre_ = false;
  PartArrays cur_, alt_;
  float4* poscell_ = nullptr;
  float* press_ = nullptr;
  float4* arace_ = nullptr;
  unsigned* begincell_ = nullptr;
  uint4* items_ = nullptr;        // tiled-interaction work items (per divide)
  unsigned* rowtmp_ = nullptr;    // per-row item counts/offsets
  unsigned* qctr_ = nullptr;      // per-XCD-group work counters
  unsigned nblocks_tiled_ = 2048;
  bool tiled_ = true;             // SPH_INTERACTION=simple selects the one-lane-per-particle kernel
  SortScratch sort_;
  DevScalars* sc_ = nullptr;
  DevScalars* sc_host_ = nullptr;  // pinned mirror for readback
  double* dttrace_ = nullptr;
  unsigned tracecap_ = 1u << 16;
  unsigned long long* pairs_ = nullptr;
  std::vector<void*> allocs_;
  // timing (hipEvents on the solver stream)
  bool timing_ = false;
  struct Ev { hipEvent_t a, b; int phase; };
  std::vector<Ev> pending_;
  std::vector<hipEvent_t> evpool_;
  double phase_ms_[4] = {0, 0, 0, 0};
  uint64_t phase_n_[4] = {0, 0, 0, 0};
  hipEvent_t cur_a_ = nullptr;
};

}  // namespace sphx
