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
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sphcore.h"
#include "sph_comm.hpp"
#include "sph_kernels.hpp"

namespace sphx {

struct SphError : std::runtime_error {
  int status;
  SphError(int st, const std::string& m) : std::runtime_error(m), status(st) {}
};

void check_hip(hipError_t e, const char* what);
void test_hook_notice(const char* name);
void derive_constants(const SphCaseDef& c, SphConstants& k);
// Ghost columns per slab face (scelldiv, +1 with mDBC).
int ghost_width(const SphConstants& c);
// Narrowest slab between two neighbours (2 x ghost width).
int min_slab_width(const SphConstants& c);
// Cell bounds along `axis` (0 x, 1 y) of a particle-count-balanced slab split (sph_slab_partition).
void slab_partition(const SphCaseDef& c, const SphParticlesHost& all, int nranks, double bound_weight, int* bounds,
                    int axis = 0);
void partition_from_prefix(const std::vector<double>& prefix, int nranks, int* bounds, int minw = 1);
// PART / case files (sph_bi4.cpp)
void part_read(const std::string& path, SphPartHeader& h, SphParticlesHost* out);
void part_write(const std::string& path, const SphPartHeader& h, const SphParticlesHost& p);
void part_head_write(const std::string& path, const SphPartHeader& h);
void bi4_rewrite(const std::string& src, const std::string& dst);
void partfloat_write(const std::string& path, const char* app, uint32_t mkboundfirst, uint32_t nft,
                     const uint16_t* mkbound, const uint32_t* begin, const uint32_t* count, const float* mass,
                     const float* massp, const float* radius, uint32_t nparts, const uint32_t* cpart,
                     const uint32_t* step, const double* timestep, const double* center, const float* fvel,
                     const float* fomega, const float* facelin, const float* faceang);
uint32_t normals_read(const std::string& path, uint32_t cap, double* out);
void partfloat_read(const std::string& path, uint32_t cpart, uint32_t nft, double* center, float* fvel,
                    float* fomega, double* timestep);
uint32_t extra_normals_read(const std::string& path, uint32_t casenbound, uint32_t casenfloat, uint32_t cap,
                            float* normals, int32_t* usenormalsft);
void extra_normals_write(const std::string& path, const char* app, uint32_t cpart, uint32_t step, double timestep,
                         uint32_t casenbound, uint32_t casenfloat, int32_t usenormalsft, uint32_t nsize,
                         const float* normals);
void normals_write(const std::string& path, const char* case_name, double dp, double h, double dist, uint32_t nbound,
                   const double* nor);

// This rank's slab: owned global x-cell columns [c0, c1) of nranks.
struct SlabConfig {
  int rank = 0, nranks = 1, c0 = 0, c1 = 0;  // owned global cells [c0, c1) along the slab axis
  int axis = 0;                              // 0: x-slabs, 1: y-slabs
};

class SphGpuSingle {
 public:
  SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& init, int device);
  // Slab of a decomposed domain: `all` is the full initial particle set; this rank
  // keeps its owned + ghost columns and talks to its neighbours through `transport`.
  SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& all, int device, const SlabConfig& slab,
               std::unique_ptr<SlabTransport> transport);
  ~SphGpuSingle();
  bool slab() const { return transport_ != nullptr; }

  // Phases (JSphGpuSingle::RunCellDivide / Interaction_Forces / DtVariable / ComputeVerlet ...).
  void RunCellDivide();
  void Interaction_Forces(int interstep);
  void DtVariable(int mode);
  void UpdateTurn(bool begin);
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
  // mDBC: the current vectors particle -> ghost node by idp (the extra data of a PART)
  unsigned DownloadNormals(float* out, unsigned cap, int* usenormalsft);
  void DownloadInteraction(SphInterOut& out);
  void CountPairs(uint64_t out[6]);
  void SetTiming(bool on);
  void SetTimingPhases(unsigned mask);
  void SetTime(double time, double symdtpre);
  void Timing(double out_ms[4], uint64_t* launches);
  void CheckErrors();
  std::string HaloDiag();
  // Moving boundaries / floating bodies (sph_bodies.hip), configured before the first step.
  void SetMotion(unsigned nobj, unsigned nmov, const SphMotionMov* movs, unsigned nevt, const SphMotionEvent* evts);
  void SetMotionTree(unsigned nnode, const SphMotionObj* nodes, unsigned nmov, const SphMotionMov* movs, unsigned nevt,
                     const SphMotionEvent* evts, unsigned nrows, const double* rows);
  void SetFloatings(unsigned nft, const SphFloatingDef* defs, double ftpause);
  // Imposed velocity / external force table of one body (SPH_FTTAB_*), before the first step.
  void SetFloatingTable(unsigned body, int kind, unsigned n, const double* times, const double* values);
  // DtFixedFile / ViscoTime tables (SPH_TTAB_*); n = 0 removes one.
  void SetTimeTable(int kind, unsigned n, const double* times, const double* values);
  // Slabs: re-balance the column bounds every `every` steps (0: never) when the most loaded
  // slab exceeds the mean by more than `tolerance`; collective (all ranks the same values).
  void SetRepartition(unsigned every, double bound_weight, double tolerance);
  // Slabs: run the interaction of the items that reach no ghost column while the ghost
  // records of the divide are in flight (default on; off = ghosts in place before it).
  // never on for a slab that shares its GPU with another slab of the run (ShareDeviceCheck,
  // the in-process group constructor): the ghost overlap only pays with a GPU of its own
  void SetOverlap(bool on) { overlap_ = on && !shared_device_; }
  void MarkSharedDevice() {
    shared_device_ = true;
    overlap_ = false;
  }
  // Collective over the slab's ranks (creation of separate-process ranks): the overlap off
  // when another rank runs on this rank's GPU (the shared-device rule of SphSlabGroup).
  void ShareDeviceCheck();
  SlabConfig Slab() const { return slabcfg_; }
  unsigned RepartitionCount() const { return repart_count_; }
  double LastImbalance() const { return repart_last_imbalance_; }
  unsigned Floatings(SphFloatingState* out, unsigned cap);

  SphConstants C{};
  KConst K{};
  DivGrid G{};
  int device = 0;
  hipStream_t stream = nullptr;

 private:
  void Init(const SphCaseDef& cdef, const SphParticlesHost& init);
  void AllocFixed();
  void AllocParticles(unsigned cap);
  void FreeParticles();
  void Free();
  void Grow(unsigned np_live, unsigned newcap);
  void PresizeExchange(const SphParticlesHost& h);
  void Upload(const SphParticlesHost& init, const std::vector<unsigned>& sel, unsigned nown);
  void UploadNormals(const SphCaseDef& cdef, const SphParticlesHost& init);
  void UploadPhases(const SphCaseDef& cdef);
  void Exchange();
  void GhostCollect(hipStream_t s);   // the posted ghost records of the last divide into their slots
  void GhostFinish();                 // ... joined to the solver stream, if still pending
  bool OverlapEligible() const;       // nothing between the divide and the interaction reads a ghost
  bool OverlapGhosts() const;         // the interaction can start before the ghosts are in
  void ExchangeStream();              // xstream_ and its events
  void WaitEvent(hipEvent_t ev, const char* what);
  void Repartition();
  void RunMotion();                 // JSphCpu::RunMotion after ComputeStep (JSphCpuSingle.cpp:1096)
  void RunFloating(bool predictor); // JSphCpuSingle::RunFloating
  void TimedBegin(int phase);
  void TimedEnd(int phase);

  unsigned cap_ = 0, npb0_ = 0, keybits_ = 0;
  int step_algorithm_ = SPH_STEP_VERLET;
  int verletstep_ = 0;
  bool havepre_ = false;
  PartArrays cur_, alt_;
  float4* poscell_ = nullptr;
  float* press_ = nullptr;
  float4* normal_ = nullptr;      // mDBC: particle -> ghost node, by idp [nnormal_]
  unsigned nnormal_ = 0;          // CaseNpb, or past the floating normals (mDBC on floating bodies)
  bool ftnormals_ = false;        // UseNormalsFt: the floating bodies have normals (JSph.cpp:1301-1306)
  bool mdbc_corrector_ = false;   // MDBCCorrector: mDBC before the Symplectic corrector too
  unsigned* mdbclist_ = nullptr;  // mDBC: wet boundary particles of this interaction [npb] + count
  void* mdbcsums_ = nullptr;      // mDBC: reduced sums per listed particle (pass 2 -> solve)
  MdbcFaceRec* mdbcface_ = nullptr;  // slabs + mDBC: send left, send right, recv left, recv right (face sizes + 1)
  unsigned long long mdbcfacecap_ = 0;
  // SPH_SLAB_MINCAP test hook: every slab buffer starts at (or grows to) its minimum, so each
  // grow-and-redo path runs (tests/test_gpu_slab.py checks the runs stay bitwise the same)
  bool slab_mincap_ = false;
  bool cut_items_ = false;  // SPH_SLAB_CUT test hook: in-place ghosts with the overlap's cut items
  unsigned* bidx_ = nullptr;         // slabs + mDBC: boundary idp -> index [CaseNpb]
  float4* arace_ = nullptr;
  // NN multiphase (v5.0 solver) and shifting
  bool nn_ = false, shift_ = false;
  float4* phasek_ = nullptr;    // interaction constants, 2 float4 per phase
  float4* phaseeos_ = nullptr;  // {rho0, cteb, gamma, integer gamma} per phase
  float phase_rho_[SPH_MAXPHASES] = {};
  float4* shiftpos_ = nullptr;  // shifting sums of the last interaction [cap]
  // NN with SPH velocity gradients (VelocityGradientType 2): the first pass's effective
  // viscosity [cap] and stress tensor (ConstEq) [2 cap], read by the second pass
  bool nnsph_ = false;
  // single phase with Laminar+SPS and/or shifting: k_fluid_ext (sph_ext.hip); sps_: the SPS
  // stress tensor is particle state (PartArrays::tau, sorted by the divide), the interaction
  // writes the new one to taunew_ (swapped after it)
  bool ext_ = false, sps_ = false;
  float4* taunew_ = nullptr;
  bool facex_ = false;  // slab face exchange of per-particle values before the interaction
  float* viscoeta_ = nullptr;
  float4* tau_ = nullptr;
  // slabs: face records of eta / tau for the neighbours' ghosts; sizes (records) of the
  // send-left, send-right, receive-left, receive-right regions, known to both sides of a face
  NNFaceRec* nnface_ = nullptr;
  unsigned long long nnfacecap_ = 0;
  unsigned face_sl_ = 0, face_sr_ = 0, face_rl_ = 0, face_rr_ = 0;
  unsigned* idxmap_ = nullptr;  // idp -> local index [CaseNp]
  unsigned casenp_ = 0;
  void NNFaceExchange();
  unsigned* begincell_ = nullptr;
  uint4* items_ = nullptr;        // tiled-interaction work items (per divide)
  unsigned* rowtmp_ = nullptr;    // per-row item counts/offsets
  uint4* rowitems_ = nullptr;     // per-row staged items of the count pass
  unsigned ricap_ = 0;
  unsigned* qctr_ = nullptr;      // per-XCD-group work counters + the list's item counts
  // slabs: the list of the items whose p1 reach a ghost column (after the interior list in
  // items_; the ghost exchange after the divide runs beside the interaction of the others)
  unsigned* qctrf_ = nullptr;
  bool ghost_split_ = false;      // the last item build made two lists
  unsigned nblocks_tiled_ = 2048;
  unsigned qpass_ = 0;  // interactions run on the current item list (the build zeroed QCTR_COPIES)
  // The offset of the counter-block copy the next interaction on the item list runs on.
  unsigned NextQueueCopy();
  bool tiled_ = true;             // SPH_INTERACTION=simple selects the one-lane-per-particle kernel
  SortScratch sort_;
  // incremental divide (single domain, after the first divide; SPH_DIVIDE=full disables it)
  IncDivScratch inc_;
  unsigned* begincell_alt_ = nullptr;
  bool inc_ok_ = false;     // usable for this grid/domain
  bool inc_valid_ = false;  // inc_.skeys holds the keys of the current particle order
  DevScalars* sc_ = nullptr;
  DevScalars* sc_host_ = nullptr;  // pinned mirror for readback
  double* dttrace_ = nullptr;
  unsigned tracecap_ = 1u << 16;
  unsigned long long* pairs_ = nullptr;
  // moving boundaries (device motion program) and floating bodies
  MotionDev* motion_ = nullptr;
  MotMov* motmovs_ = nullptr;
  MotEvt* motevts_ = nullptr;
  double* motdata_ = nullptr;  // rows of the file movements' tables (4 doubles each)
  bool classified_ = false;     // the last update classified the particles for the divide
  bool packcounted_ = false;    // ... and ran the slab exchange's count pass
  PackArgs pack_args_;
  struct UpdateFuse {
    const IncDivScratch* cls = nullptr;
    const PackArgs* pk = nullptr;
  };
  UpdateFuse FuseUpdate(bool pre_at_divide);
  unsigned nmotobj_ = 0;
  FtBody* ftbodies_ = nullptr;
  unsigned* ftridp_ = nullptr;   // floating particle (idp - CaseNpb) -> position, per divide
  float* ftmassp_ = nullptr;     // particle mass per body (interaction)
  float* ftpart_ = nullptr;      // partial force sums [body][FT_NBLK][6]
  double4* fttab_ = nullptr;     // JLinearValue rows (time, x, y, z) of every body's tables
  FtTabDesc* fttabdesc_ = nullptr;  // [body][SPH_FTTAB_*] = {first row, rows, lookup state}
  void UploadFloatingTables();    // (again at a restart: the lookups start over, as new JLinearValues)
  std::vector<std::vector<double4>> fttabs_;  // host copy, [body * 4 + kind]
  int nftbodies_ = 0;
  void* dttab_ = nullptr;        // DtFixedFile rows: times [n], dt in ms [n] (double)
  void* viscotab_ = nullptr;     // ViscoTime rows: times [n], Visco [n] (float)
  unsigned nftp_ = 0;            // floating particles of the case (CaseNfloat)
  unsigned casenpb_ = 0;         // CaseNpb: first floating idp
  bool stepped_ = false;         // a step was issued (bodies are configured before it)
  // turns measurement mode: the dt maxima of the next DtVariable are folded at the end of the
  // interaction's turn (fold_turn_: its clear flag, -1 none), so that k_fold runs alone on the
  // GPU as on a rank's own; folded_ready_: DtVariable finds them folded
  int fold_turn_ = -1;
  bool folded_ready_ = false;
  std::vector<void*> allocs_;   // fixed-size allocations
  std::vector<void*> pallocs_;  // capacity-sized (per-particle) allocations
  // slab decomposition
  std::unique_ptr<SlabTransport> transport_;
  SlabConfig slabcfg_;
  bool exchange_armed_ = false;  // the initial divide has no exchange (ghosts come with the case)
  double comm_timeout_s_ = 120.0;  // SPH_COMM_TIMEOUT_S: deadline of a slab host wait
  unsigned nctmax_ = 0;            // cells of the widest grid (grid-sized buffers)
  int gmax_ncx_ = 0, gmax_ncy_ = 0;  // its x / y extents
  float* colcnt_ = nullptr;        // re-partition: column counts + bounds (device)
  unsigned repart_every_ = 0, repart_count_ = 0;
  double repart_bw_ = 0.3, repart_tol_ = 0.05, repart_last_imbalance_ = 1.0;
  unsigned long long stepsdone_ = 0;
  unsigned* folded_ = nullptr;   // 4 maxima + fatal error flags for the allreduce
  SlabCounts* slabcnt_ = nullptr;
  SlabCounts* slabcnt_host_ = nullptr;
  unsigned* packtiles_ = nullptr;
  SlabSendBufs send_{nullptr, nullptr, nullptr, nullptr, 0, 0};
  SlabGhost* recvg_ = nullptr;
  SlabRec* recvm_ = nullptr;
  unsigned long long recvgcap_ = 0, recvmcap_ = 0;
  void* sendgbuf_ = nullptr;
  void* sendmbuf_ = nullptr;
  // the ghost exchange after the divide (sph_kernels.hpp SlabFaces)
  SlabFaces faces_{};
  unsigned long long xg_sl_ = 0, xg_sr_ = 0, xg_rl_ = 0, xg_rr_ = 0;  // ghost records of this exchange
  unsigned xg_nm_ = 0;            // migrants it appended (apppos[xg_nm_ + e] = slot of ghost e)
  unsigned xg_np_ = 0;            // particles held after the migrants were appended
  bool ghost_pending_ = false;    // the last divide's ghost records have not been sent yet
  bool overlap_ = false;          // sph_slab_set_overlap (default off: DESIGN.md §6)
  bool shared_device_ = false;    // another slab of the run uses the same GPU
  bool in_run_ = false;           // inside Run(): the next phase after a divide is the interaction
  hipStream_t xstream_ = nullptr; // ghost transfer + scatter + face items beside the interior items
  hipEvent_t ev_div_ = nullptr, ev_ghost_ = nullptr;

  // timing (hipEvents on the solver stream)
  bool timing_ = false;
  unsigned timing_mask_ = 0xfu;  // phases timed (SetTimingPhases, sph_solver_set_timing_phases)
  struct Ev { hipEvent_t a, b; int phase; };
  std::vector<Ev> pending_;
  std::vector<hipEvent_t> evpool_;
  hipEvent_t xev_ = nullptr;  // exchange: counts arrived on the host (spin-waited)
  double phase_ms_[4] = {0, 0, 0, 0};
  uint64_t phase_n_[4] = {0, 0, 0, 0};
  hipEvent_t cur_a_ = nullptr;
};

// Several slabs of one domain driven by host threads of one process (LocalTransport).
class SphSlabGroup {
 public:
  SphSlabGroup(const SphCaseDef& cdef, const SphParticlesHost& all, int nslabs, const int* devices,
               const int* bounds, int axis = 0);
  void Run(unsigned nsteps);
  std::vector<std::unique_ptr<SphGpuSingle>> slabs;

 private:
  std::shared_ptr<LocalHub> hub_;
};

}  // namespace sphx
