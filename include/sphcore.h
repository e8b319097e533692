/*
 * sphcore.h — C-ABI of the MI355X-native SPH particle-interaction core.
 *
 * This is the drop-in boundary for the DualSPHysics v5.2 hot path
 * (SURVEY.md §8(b)): cell-linked-list divide → Interaction_Forces →
 * dt → Verlet/Symplectic update, as driven by JSphGpuSingle/JSphCpuSingle.
 * Plain C types, device pointers as void*, sizes as unsigned; no torch, no
 * C++ in the signatures.  Every function returns SphStatus (0 = ok); the text
 * of the last error of the calling thread is in sph_last_error().  The C++
 * host wrapper (csrc/sph_solver.hpp) turns a non-zero status back into an
 * exception, preserving the reference's fail-fast behaviour
 * (RunExceptionGpuDef.h:27, JSphGpu.cpp:118-125).
 *
 * Entry points and the reference interfaces they replace:
 *   sph_case_derive ............ JSph::ConfigConstants1/2 (JSph.cpp:1392-1457),
 *                                JSph::ConfigCellDivision (JSph.cpp:1772-1788),
 *                                JSph::SelecDomain (JSph.cpp:1794-1829)
 *   sph_solver_create .......... JSphGpuSingle::ConfigDomain + InitRunGpu
 *                                (JSphGpuSingle.cpp; CPU twin JSphCpuSingle.cpp:107-167)
 *   sph_divide ................. JSphGpuSingle::RunCellDivide (JSphGpuSingle.cpp:331-430):
 *                                cudiv::LimitsCell/PreSortFull/Sort/CalcBeginEndCell/
 *                                SortDataParticles (JCellDivGpu_ker.h:36-59,
 *                                JCellDivGpuSingle_ker.h:26-29), cusphs::UpdatePosCell
 *   sph_interaction_forces ..... JSphGpuSingle::Interaction_Forces (JSphGpuSingle.cpp:435-486):
 *                                cusph::Interaction_Forces(StInterParmsg) (JSphGpu_ker.h:200)
 *                                + ComputeVelMod/ReduMaxFloat/ComputeAceMod/AddDelta,
 *                                CPU twin JSphCpu::Interaction_Forces_ct (JSphCpu.cpp:1012)
 *   sph_compute_dt ............. JSph*::DtVariable (JSphGpu.cpp:984, JSphCpu.cpp:1614)
 *   sph_step_verlet ............ JSphGpu::ComputeVerlet (JSphGpu.cpp:874) =
 *                                cusphs::ComputeStepVerlet + cusph::ComputeStepPos
 *   sph_step_symplectic_pre/cor  JSphGpu::ComputeSymplecticPre/Corr (JSphGpu.cpp:900-983)
 *   sph_solver_run ............. JSphGpuSingle::Run main loop (JSphGpuSingle.cpp:853-880):
 *                                ComputeStep_Ver/_Sym + RunCellDivide, device-resident dt
 *   sph_download_particles ..... JSphGpuSingle::ParticlesDataDown (feeds SaveData)
 *   sph_partfloat_read, sph_extra_normals_read/write, sph_download_normals: restart of floating
 *     bodies and mDBC (JSphCpu::InitFloating, JSph::ConfigBoundNormals, JDsExtraData)
 *   sph_normals_read/write ..... JSph::LoadBoundNormals (JSph.cpp:1265-1295) over
 *                                JPartNormalData::LoadFile/SaveFile (JPartNormalData.cpp:178-257)
 *   sph_count_pairs ............ JDsPips::ComputeGpu (JDsPips.cpp:187-262) — work counter
 *   sph_slab_* ................. new: slab decomposition across GPUs; the
 *                                reference fork runs one domain per process (JSphGpuSingle)
 *   sph_comm_unique_id ......... RCCL bootstrap id (ncclGetUniqueId) for sph_slab_create
 *   sph_part_read/write ........ JPartDataBi4::LoadFilePart/LoadFileCase and AddPartInfo +
 *                                AddPartData + SaveFilePart (JPartDataBi4.cpp:304-440,
 *                                492-516) over the .bi4 container of JBinaryData
 *                                (JBinaryData.cpp:700-1160,1467-1545): PART and case files
 *   sph_solver_set_motion ...... JDsMotion::Init + JSph::CalcMotion/JSphCpu::RunMotion
 *     (+ _tree)                  (JDsMotion.cpp:94-137, JSph.cpp:2308, JSphCpu.cpp:1692-1789;
 *                                nested objects, circular / file / flash movements:
 *                                JMotion.cpp:96-317,556-700, JMotionObj.cpp:40-580)
 *   sph_solver_set_floatings ... JSph::LoadCaseConfig floating objects (JSph.cpp:1046-1100) +
 *                                JSphCpuSingle::RunFloating (JSphCpuSingle.cpp:897-1010)
 *   sph_solver_set_floating_table  FtLinearVel/FtAngularVel/FtLinearForce/FtAngularForce
 *                                (JSph.cpp:1060-1082; JSphCpuSingle.cpp:874-914)
 *   sph_solver_floatings ....... FtObjs[] (feeds PartFloat.fbi4, JPartFloatBi4)
 */
#ifndef SPHCORE_H
#define SPHCORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPH_ABI_VERSION 12

typedef enum {
  SPH_OK = 0,
  SPH_ERR_ARG = 1,        /* invalid argument / configuration            */
  SPH_ERR_HIP = 2,        /* HIP runtime error                           */
  SPH_ERR_STATE = 3,      /* call out of order / object in a bad state   */
  SPH_ERR_DT = 4,         /* dt NaN or infinite (JSphCpu.cpp:1622)       */
  SPH_ERR_BOUNDOUT = 5,   /* boundary particle excluded (JSphCpuSingle.cpp:507-518) */
  SPH_ERR_NOMEM = 6,      /* allocation failed                           */
  SPH_ERR_UNSUPPORTED = 7,/* feature outside the implemented scope       */
  SPH_ERR_COMM = 8        /* RCCL / slab exchange failure                */
} SphStatus;

/* TpStep (DualSphDef.h:316-319). */
enum { SPH_STEP_VERLET = 1, SPH_STEP_SYMPLECTIC = 2 };
/* TpDensity (DualSphDef.h:358-364). */
enum { SPH_DDT_NONE = 0, SPH_DDT_DDT = 1, SPH_DDT_DDT2 = 2, SPH_DDT_DDT2FULL = 3 };
/* TpCellMode (DualSphDef.h:477-481). */
enum { SPH_CELLMODE_FULL = 1, SPH_CELLMODE_HALF = 2 };
/* TpBoundary (DualSphDef.h:336-340) and TpSlipMode (DualSphDef.h:343-348); this fork
 * allows only SLIP_Vel0 with mDBC (JSph.cpp:788). */
enum { SPH_BOUND_DBC = 1, SPH_BOUND_MDBC = 2 };
enum { SPH_SLIP_VEL0 = 1, SPH_SLIP_NOSLIP = 2, SPH_SLIP_FREESLIP = 3 };
/* TpKernel (DualSphDef.h:355-359): Cubic spline (with its tensile correction) and
 * quintic Wendland (the default). */
enum { SPH_KERNEL_CUBIC = 1, SPH_KERNEL_WENDLAND = 2 };
/* v5.0 NN multiphase solver (src_mphase/DSPH_v5.0_NNewtonian):
 * RheologyTreatment (JSph.cpp:608-614), VelocityGradientType (:616-621), TpVisco
 * (DualSphDef.h:374-378) and TpShifting (JSphShifting.h). */
enum { SPH_RHEOLOGY_SINGLE = 1, SPH_RHEOLOGY_NN = 2 };
enum { SPH_VELGRAD_FDA = 1, SPH_VELGRAD_SPH = 2 };
enum { SPH_VISCO_ARTIFICIAL = 1, SPH_VISCO_LAMINARSPS = 2, SPH_VISCO_CONSTEQ = 3 };
enum { SPH_SHIFT_NONE = 0, SPH_SHIFT_NOBOUND = 1, SPH_SHIFT_NOFIXED = 2, SPH_SHIFT_FULL = 3 };
#define SPH_MAXPHASES 8

/* One <nnphases><phase> (JSph::InitMultiPhase, JSph.cpp:3137-3215 -> StPhaseArray +
 * StPhaseCte, DualSphDef.h:304-331), values as the XML gives them. */
typedef struct SphPhaseDef {
  int32_t mkfluid;          /* phase of the fluid block with this mkfluid              */
  int32_t phasetype;        /* <phasetype> (0 non-Newtonian: the only one in v5.0)      */
  double rho;               /* <rhop>                                                  */
  double cs0;               /* <csound> (0: not given -> CteB from the case's Cs0)     */
  double gamma;             /* <gamma> (0: the case's gamma)                           */
  double visco;             /* <visco> kinematic viscosity / consistency index         */
  double tau_yield;         /* <tau_yield>                                             */
  double tau_max;           /* <tau_max> (0: none)                                     */
  double bi_multi;          /* <Bi_multi> (with tau_max)                               */
  double hbp_m, hbp_n;      /* <HBP_m>, <HBP_n>                                        */
} SphPhaseDef;

/* Particle code bits, identical to the 16-bit `typecode` of DualSphDef.h:161-221. */
#define SPH_CODE_MASKSPECIAL 0xe000u
#define SPH_CODE_NORMAL 0x0u
#define SPH_CODE_PERIODIC 0x2000u
#define SPH_CODE_OUTIGNORE 0x4000u
#define SPH_CODE_OUTMOVE 0x6000u
#define SPH_CODE_OUTPOS 0x8000u
#define SPH_CODE_OUTRHOP 0xA000u
#define SPH_CODE_MASKTYPE 0x1800u
#define SPH_CODE_TYPE_FIXED 0x0u
#define SPH_CODE_TYPE_MOVING 0x800u
#define SPH_CODE_TYPE_FLOATING 0x1000u
#define SPH_CODE_TYPE_FLUID 0x1800u

/*
 * Case definition: what JSph::LoadCaseConfig and JSph::LoadCaseParticles read
 * from <case>.xml/<case>.bi4 (JSph.cpp:567-583 constants, :588-760 parameters,
 * :2051-2076 map limits).  Floating-point members are given as the XML text
 * parses them (double); sph_case_derive narrows them exactly as JSph does.
 */
typedef struct SphCaseDef {
  double dp;                /* <dp>                                        */
  double h;                 /* <h>   -> KernelH (float)                    */
  double cteb;              /* <b>   -> CteB (float)                       */
  double rhop0;             /* <rhop0>                                     */
  double gamma;             /* <gamma>                                     */
  double massbound, massfluid;
  double gravity[3];
  double cflnumber;
  int step_algorithm;       /* SPH_STEP_*                                  */
  int verlet_steps;         /* VerletSteps (40)                            */
  int kernel;               /* SPH_KERNEL_CUBIC / SPH_KERNEL_WENDLAND      */
  int tdensity;             /* SPH_DDT_*                                   */
  double visco;             /* artificial viscosity alpha                  */
  double viscoboundfactor;
  double ddtvalue;
  double coefdtmin;         /* CoefDtMin (0.05)                            */
  double dtini, dtmin;      /* 0 => derived (JSph.cpp:1448-1449)           */
  double rhopoutmin, rhopoutmax;
  double map_realposmin[3]; /* MapRealPosMin (after border + domain config)*/
  double map_realposmax[3]; /* MapRealPosMax                               */
  int cellmode;             /* SPH_CELLMODE_FULL / _HALF                   */
  int celldomfixed;         /* 1: cell domain = whole map (-cellfixed:1)   */
  uint32_t npb;             /* boundary particles are the first npb        */
  uint32_t np;              /* total particles                             */
  int32_t tboundary;        /* SPH_BOUND_* (<parameter Boundary>; 0 = DBC) */
  int32_t slipmode;         /* SPH_SLIP_* (<parameter SlipMode>)           */
  double mdbc_threshold;    /* MdbcThreshold (-mdbc_threshold, default 0)  */
  /* v5.0 NN multiphase (RheologyTreatment=2).  Phases are sorted by mkfluid (JSph.cpp:
   * 3187-3195); a fluid particle's phase is its code value (the fluid block index).  */
  int32_t rheology;         /* SPH_RHEOLOGY_* (0 = single)                 */
  int32_t velgrad;          /* SPH_VELGRAD_* (0 = FDA)                     */
  int32_t tvisco;           /* SPH_VISCO_* (0 = artificial)                */
  uint32_t nphases;
  double relaxation_dt;     /* RelaxationDt, lamda of the viscous dt       */
  /* shifting (JSphShifting::ConfigBasic; <parameter Shifting/ShiftCoef/ShiftTFS>) */
  int32_t shift_mode;       /* SPH_SHIFT_*                                 */
  int32_t mdbc_corrector;   /* <parameter MDBCCorrector>: mDBC also before the Symplectic
                               corrector's interaction (JSph.cpp:639,783; JSphCpuSingle.cpp:525) */
  double shift_coef, shift_tfs;
  SphPhaseDef phases[SPH_MAXPHASES];
  /* 2-D simulation (<data2d>, JSph::LoadConfigCtes JSph.cpp:571-572): particles in the
   * plane y = data2d_posy, 2-D Wendland constants (FunSphKernel.h:193-196), ace.y = 0 */
  int32_t data2d;
  int32_t pad2d;
  double data2d_posy;
  /* dt options (JSph::LoadConfigParameters, JSph.cpp:697-707): DtAllParticles = VelMax
   * over every particle, not only the fluid (JSphCpu.cpp:475); dtfixed > 0 = <parameter
   * DtFixed>, the dt of every step (JDsFixedDt; a DtFixedFile table goes through
   * sph_solver_set_time_table) */
  int32_t dtallparticles;
  /* <parameter Symmetry> (JSph.cpp:714): the plane y = 0 mirrors the particles; their
   * images near it are neighbours (JSphCpu.cpp:566-613, 671-796), MapRealPosMin.y = 0
   * (JSph.cpp:1386), a particle crossing y = 0 is reflected (JSphCpu.cpp:1247) */
  int32_t symmetry;
  double dtfixed;
} SphCaseDef;

/*
 * Derived constants (StCteSph, DualSphDef.h:374-402, plus the interaction and
 * divide constants of JSph/JSphCpu), in the precision the reference holds them.
 */
typedef struct SphConstants {
  float kernelh, kernelsize, kernelsize2;
  float awen, bwen;                 /* Wendland (FunSphKernel.h:191-202) */
  float cteb, gamma, rhopzero, ovrhopzero;
  float massfluid, massbound;
  float gravity[3];
  float eta2, ddtkh, ddtgz;
  float visco, viscoboundfactor;
  float rhopoutmin, rhopoutmax;
  float scell, movlimit;
  float pad0;
  double cs0, cflnumber, dtini, dtmin, dp;
  int tdensity, step_algorithm, verlet_steps, scelldiv;
  double map_realposmin[3], map_realsize[3];
  double dom_posmin[3];             /* DomPosMin = Map_PosMin (single domain) */
  uint32_t dom_cells[3];            /* Map_Cells = DomCells                   */
  uint32_t dom_cellcode;            /* DomCellCode (JDsDcell.cpp:64-69)       */
  int32_t tboundary, slipmode;      /* TBoundary, SlipMode (JSph.cpp:626-640) */
  float mdbc_threshold;             /* MdbcThreshold                          */
  uint32_t pad1;
  /* NN multiphase and shifting (JSph::ConfigConstantsMP, JSph.cpp:3220-3242) */
  int32_t rheology, velgrad, tvisco, shift_mode;
  uint32_t nphases;
  float relaxation_dt, shift_coef, shift_tfs;
  float phase_mass[SPH_MAXPHASES];  /* StPhaseArray.mass = rho dp^3               */
  float phase_cteb[SPH_MAXPHASES];  /* StPhaseArray.CteB                          */
  int32_t data2d, pad3;
  float spssmag, spsblin;           /* Laminar+SPS SpsSmag, SpsBlin (JSph.cpp:1438-1443) */
  /* kernel (TKernel) and the Cubic spline constants StKCubicCte (FunSphKernel.h:51-84) */
  int32_t kernel;
  float cub_a1, cub_a2, cub_aa, cub_a24, cub_c1, cub_d1, cub_c2, cub_od_wdeltap;
  int32_t pad4;
  int32_t dtallparticles, symmetry; /* DtAllParticles, Symmetry            */
  double dtfixed;                   /* DtFixed (0: variable dt)             */
} SphConstants;

/* Step statistics kept on the device and read back on demand. */
typedef struct SphRunStats {
  double time;            /* simulated time TimeStep                        */
  double last_dt;         /* last dt                                        */
  double sym_dtpre;       /* SymplecticDtPre                                */
  uint64_t nstep;         /* steps done                                     */
  uint32_t np, npb, npbok;/* current counts after the last divide           */
  uint32_t nout;          /* fluid particles excluded so far                */
  uint32_t dtmodif;       /* dt clamped to DtMin (JSphCpu.cpp:1623-1629)    */
  uint32_t error_flags;   /* bit0: NaN/inf dt, bit1: boundary out           */
  float velmax, acemax, viscdtmax; /* of the last interaction              */
  float viscetadtmax;     /* NN: max effective viscosity (ViscEtaDtMax)     */
} SphRunStats;

/* Host particle view (SaveData layout: JSph::SaveData, JSph.cpp:2717). */
typedef struct SphParticlesHost {
  uint32_t n;
  uint32_t* idp;        /* [n]    */
  double* pos;          /* [n][3] */
  float* vel;           /* [n][3] */
  float* rhop;          /* [n]    */
  uint16_t* code;       /* [n] (may be NULL on download) */
  float* boundnormal;   /* [n][3] mDBC only: normal from the particle to the boundary
                           limit, as the case's _Normals.nbi4 holds it (JSph::
                           LoadBoundNormals, JSph.cpp:1265); NULL otherwise and on download */
} SphParticlesHost;

/* Interaction outputs for kernel-level parity checks (StInterResultc + arrays). */
typedef struct SphInterOut {
  float* ar;      /* host [np]    density derivative (incl. DDT)            */
  float* ace;     /* host [np][3] acceleration (without gravity)            */
  float viscdtmax, velmax, acemax;
} SphInterOut;

typedef struct SphSolver SphSolver;

/* ---- library ----------------------------------------------------------- */
int sph_abi_version(void);
const char* sph_last_error(void);

/* ---- configuration ----------------------------------------------------- */
int sph_case_derive(const SphCaseDef* cdef, SphConstants* out);

/* ---- solver lifetime (device id = HIP device ordinal) ------------------- */
int sph_solver_create(const SphCaseDef* cdef, const SphParticlesHost* init, int device, SphSolver** out);
int sph_solver_destroy(SphSolver* s);

/* ---- hot path: individual phases (all async on the solver stream) -------- */
int sph_divide(SphSolver* s);                       /* RunCellDivide(true)        */
int sph_interaction_forces(SphSolver* s, int interstep); /* 1 Verlet, 2 SymPre, 3 SymCor */
int sph_compute_dt(SphSolver* s, int final_);       /* DtVariable(final)          */
int sph_step_verlet(SphSolver* s);                  /* ComputeVerlet(dt)          */
int sph_step_symplectic_pre(SphSolver* s);          /* ComputeSymplecticPre(dt)   */
int sph_step_symplectic_cor(SphSolver* s);          /* ComputeSymplecticCorr(dt)  */

/* ---- hot path: whole steps (ComputeStep + RunCellDivide), device-resident -- */
int sph_solver_run(SphSolver* s, uint32_t nsteps);
int sph_solver_sync(SphSolver* s);
int sph_solver_stats(SphSolver* s, SphRunStats* out);
/* Per-step dt trace (host array of length >= nsteps done); returns count.   */
int sph_solver_dt_trace(SphSolver* s, double* out, uint32_t cap, uint32_t* count);

/* ---- data out ------------------------------------------------------------ */
int sph_download_particles(SphSolver* s, SphParticlesHost* out);
int sph_download_interaction(SphSolver* s, SphInterOut* out);

/* ---- measurement ----------------------------------------------------------- */
/* Pair counts of one interaction pass (JDsPips): checked & real pairs for
 * fluid-fluid, fluid-bound and bound-fluid.  out[6] = {ff_chk, ff_real,
 * fb_chk, fb_real, bf_chk, bf_real}. */
int sph_count_pairs(SphSolver* s, uint64_t out[6]);
/* Average device time (ms) of the last timed region's kernels, by phase:
 * out[0]=interaction, [1]=update, [2]=divide, [3]=mDBC boundary correction. */
/* Restart from a PART (JSph::InitRun with PartBegin, JSph.cpp:2087-2106): simulated
 * time TimeStep of the loaded PART, and SymplecticDtPre if > 0 (else DtIni stays).
 * VelrhopM1 = Velrhop and VerletStep = 0 hold from creation, as in the reference. */
int sph_solver_set_time(SphSolver* s, double time, double symplectic_dtpre);
int sph_solver_set_timing(SphSolver* s, int enabled);
/* Which phases the timed region records (bit i = phase i of sph_solver_timing's out_ms;
 * sph_solver_set_timing(s, 1) times all four).  Each timed phase puts two event markers
 * in the solver stream; timing the interaction alone (mask 1) keeps the other launches
 * back to back, ~18 us per Verlet step at 1M particles.  Replaces no reference call: the
 * reference's JSphGpuSingle timers (TmgStart/TmgStop, JSphGpuSingle.cpp) sync per phase. */
int sph_solver_set_timing_phases(SphSolver* s, unsigned mask);
int sph_solver_timing(SphSolver* s, double out_ms[4], uint64_t* launches);

/* ---- slab decomposition over x or y --------------------------
 * Rank r owns the global cells [cx_begin, cx_end) of the slab axis (axis 0: x-cell
 * columns, axis 1: y-cell rows; the full extent of the other axes) and holds ghost copies
 * of the neighbours' particles in the W cells either side (one cell = 2h, the support
 * radius).  y-slabs keep every x row of cells whole on one rank (no rows cut at the faces,
 * whole-row items), for a domain whose load is spread along y (the dam breaks).  Every divide exchanges migrants and ghosts with rank-1 / rank+1, every
 * dt max-reduces VelMax/AceMax/ViscDtMax over all ranks, so every rank steps with the
 * single-domain dt and each particle sees its single-domain neighbour set.
 * On a slab solver: sph_solver_run and the phase calls are COLLECTIVE (all ranks
 * call them in the same order); stats.np is the number of OWNED particles;
 * sph_download_particles returns the owned particles only. */
typedef struct SphSlabDef {
  int32_t rank, nranks;
  int32_t cx_begin, cx_end;       /* owned global cells [begin, end) of the slab axis  */
  int32_t axis;                   /* 0: x-slabs (default), 1: y-slabs (3-D cases)       */
  int32_t pad;
  unsigned char comm_id[128];     /* sph_comm_unique_id() of rank 0, same on all ranks */
} SphSlabDef;

/* Column bounds balancing sum(fluid) + bound_weight*sum(bound) particles per rank,
 * from the full initial particle set; cx_bounds[nranks+1] (first 0, last = cells).
 * Every slab gets at least 2W columns (W = ghost width: scelldiv, +1 with mDBC), the
 * narrowest slab sph_slab_create accepts between two neighbours (W at a map end). */
int sph_slab_partition(const SphCaseDef* cdef, const SphParticlesHost* all, int nranks, double bound_weight,
                       int32_t* cx_bounds);
/* The same along `axis` (0 x, 1 y): bounds[nranks+1] in cells of that axis. */
int sph_slab_partition_axis(const SphCaseDef* cdef, const SphParticlesHost* all, int nranks, double bound_weight,
                            int axis, int32_t* bounds);
int sph_comm_unique_id(unsigned char id[128]);
/* One process per GPU over RCCL: every rank passes the FULL initial particle set
 * and keeps its owned + ghost columns. */
int sph_slab_create(const SphCaseDef* cdef, const SphParticlesHost* all, int device, const SphSlabDef* slab,
                    SphSolver** out);
/* The same slab with a host-staged transport over the POSIX shared-memory segment
 * `shm_name` ("/..."; two mailboxes of slot_bytes per rank; comm_id unused): separate
 * processes of ONE node without RCCL, e.g. several ranks on one GPU, where RCCL refuses
 * duplicate devices.  Rank 0 creates the segment, the others attach.  Same collective
 * calls and failure semantics (deadline SPH_COMM_TIMEOUT_S, abort flag -> SPH_ERR_COMM). */
int sph_slab_create_shm(const SphCaseDef* cdef, const SphParticlesHost* all, int device, const SphSlabDef* slab,
                        const char* shm_name, uint64_t slot_bytes, SphSolver** out);

/* Several slabs in ONE process (host threads, device-to-device copies; devices may
 * repeat).  The member handles are borrowed (no destroy); members accept the data-out
 * calls (stats, download, dt trace, timing) but not run/phase calls — run the group. */
typedef struct SphSlabGroup SphSlabGroup;
int sph_slab_group_create(const SphCaseDef* cdef, const SphParticlesHost* all, int nslabs, const int32_t* devices,
                          const int32_t* cx_bounds, SphSlabGroup** out);
int sph_slab_group_create_axis(const SphCaseDef* cdef, const SphParticlesHost* all, int nslabs,
                               const int32_t* devices, int axis, const int32_t* bounds, SphSlabGroup** out);
int sph_slab_group_destroy(SphSlabGroup* g);
int sph_slab_group_run(SphSlabGroup* g, uint32_t nsteps);
int sph_slab_group_member(SphSlabGroup* g, int i, SphSolver** out);
/* Periodic re-balancing of the column bounds: every `every` steps (0:
 * never) the owned particles per column (fluid + bound_weight x boundary) are summed over
 * the ranks and, when the most loaded slab exceeds the mean by more than `tolerance`
 * (relative), every rank moves to the same new bounds (each strictly inside the two slabs
 * it separates); the next exchange hands the columns over.  Collective: every rank (or
 * the group) with the same values, before or between runs. */
int sph_slab_set_repartition(SphSolver* s, uint32_t every, double bound_weight, double tolerance);
int sph_slab_group_set_repartition(SphSlabGroup* g, uint32_t every, double bound_weight, double tolerance);
/* Ghost exchange beside the interaction (default off): the ghost records of a divide travel
 * while the items whose stencil reaches no ghost column interact; the face items follow (the
 * rows are cut at the face columns for that).  Off: the ghosts are in place before the
 * interaction, over uncut rows.  Results are bitwise the same.  Off by default since round 5:
 * each slab's interaction measured alone on the GPU (the turns measurement mode of the
 * in-process transport) took 1.03-1.13 ms with the overlap against 0.85-0.92 ms
 * in place at the BASELINE cfg3 8-slab split — the cut rows' extra items cost more than the
 * transfer the overlap hides.  Always off for slabs that share a GPU with another slab of the
 * run (groups: same device id; sph_slab_create / _shm: same PCI bus id, checked collectively
 * at creation).
 * (No reference counterpart: the fork runs one domain per process, JSphGpuSingle.) */
int sph_slab_set_overlap(SphSolver* s, int on);
int sph_slab_group_set_overlap(SphSlabGroup* g, int on);
typedef struct SphSlabInfo {
  int32_t rank, nranks, cx_begin, cx_end;  /* current owned cells of the slab axis           */
  uint32_t repartitions;                   /* bounds changes so far                          */
  int32_t axis;                            /* the slab axis (0 x, 1 y)                       */
  double last_imbalance;                   /* max slab load / mean at the last check (1 = even) */
} SphSlabInfo;
int sph_slab_info(SphSolver* s, SphSlabInfo* out);

/* ---- PART / case files (.bi4), SURVEY.md §8(f) row 2 ------------------------------
 * Root values of JPartDataBi4 (case) + the values of its PART_%04u item, in the
 * reference's own names and types.  Positions are double on this interface; files
 * store them as Posd (double3, pos_double=1) or Pos (float3). */
typedef struct SphPartHeader {
  char app_name[64], case_name[64];
  uint32_t cpart, npok, nout, step;   /* Cpart, Npok, Nout, Step                          */
  double timestep, runtime;           /* TimeStep, RunTime                                */
  double domain_min[3], domain_max[3];/* DomainMin, DomainMax                             */
  double symplectic_dtpre;            /* SymplecticDtPre (written if > 0; read on restart) */
  uint64_t np_total;                  /* NpTotal (written if > 0)                         */
  uint64_t case_np, case_nfixed, case_nmoving, case_nfloat, case_nfluid;
  double dp, h, b, rhop0, gamma, massbound, massfluid;
  double map_posmin[3], map_posmax[3], case_posmin[3], case_posmax[3];
  double peri_xinc[3], peri_yinc[3], peri_zinc[3];
  double data2d_posy;
  int32_t data2d, peri_mode, axis_div, np_dynamic, reuse_ids, symmetry, splitting, pos_double;
  /* run header (Part_Head.ibi4, JPartDataHead) */
  int32_t visco_type;                 /* ViscoType (1 artificial)                         */
  float visco, viscoboundfactor;      /* ViscoValue, ViscoBoundFactor                     */
  float gravity[3];                   /* Gravity                                          */
  uint32_t mkbound, mkfluid;          /* Mk of the fixed and the fluid block              */
} SphPartHeader;

/* Read a PART or case file.  With out == NULL (or out->n < Npok) only *hdr is filled;
 * call again with arrays of hdr->npok entries (code may be NULL). */
int sph_part_read(const char* path, SphPartHeader* hdr, SphParticlesHost* out);
/* Write a PART file as the reference's SaveFilePart does (no solver statistics values). */
int sph_part_write(const char* path, const SphPartHeader* hdr, const SphParticlesHost* parts);
/* Write the run header Part_Head.ibi4 (JPartDataHead) that the reference's restart
 * (-partbegin) reads beside the PART files: case values + one Fixed and one Fluid MK block. */
int sph_part_head_write(const char* path, const SphPartHeader* hdr);
/* Boundary normals file <case>_Normals.nbi4 (PartNormals, double3[Nbound]): *nbound is
 * set; the normals are copied when out != NULL and cap >= Nbound. */
int sph_normals_read(const char* path, uint32_t cap, double* out, uint32_t* nbound);
int sph_normals_write(const char* path, const char* case_name, double dp, double h, double dist, uint32_t nbound,
                      const double* normals);
/* Parse any .bi4 container and write it back (format round trip; byte-identical for
 * files written by the reference). */
int sph_bi4_rewrite(const char* src, const char* dst);

/* ---- moving boundaries and floating bodies -------------------
 * Particle codes: sph_solver_create takes SphParticlesHost.code when it is not NULL (the
 * codes of JSphMk::Config, JSphMk.cpp:86-123: moving = SPH_CODE_TYPE_MOVING | moving-block
 * index, floating = SPH_CODE_TYPE_FLOATING | floating-block index); boundary (fixed and
 * moving) particles are the first npb, floating particles sit among the fluid ones. */

/* Movements of the JMotion program (JMotion::ReadXml, JMotion.cpp:556-700), in the units
 * JMotion holds them: lengths m, times s (durations/starts as JXml::GetAttributeFloat
 * reads them, i.e. float values), rotation speeds/accelerations/amplitudes in degrees,
 * phases in radians, frequencies in Hz. */
enum {
  SPH_MOV_WAIT = 1,      /* <wait>                                                   */
  SPH_MOV_RECT = 2,      /* <mvrect>      vec = vel                                  */
  SPH_MOV_RECTACE = 3,   /* <mvrectace>   vec = ace, vec2 = velini (prev: no velini) */
  SPH_MOV_ROT = 4,       /* <mvrot>       ang = vel, axis                            */
  SPH_MOV_ROTACE = 5,    /* <mvrotace>    ang = ace, ang2 = velini (prev)            */
  SPH_MOV_RECTSINU = 6,  /* <mvrectsinu>  vec = freq, vec2 = ampl, phase (prev)      */
  SPH_MOV_ROTSINU = 7,   /* <mvrotsinu>   ang = freq, ang2 = ampl, ang3 = phase (prev), axis */
  SPH_MOV_CIR = 8,       /* <mvcir>       ang = vel, axis, ref                       */
  SPH_MOV_CIRACE = 9,    /* <mvcirace>    ang = ace, ang2 = velini (prev), axis, ref */
  SPH_MOV_CIRSINU = 10,  /* <mvcirsinu>   ang = freq, ang2 = ampl, ang3 = phase (prev), axis, ref */
  SPH_MOV_RECTFILE = 11, /* <mvrectfile> (<mvfile>, <mvpredef>): positions of a table  */
  SPH_MOV_ROTFILE = 12,  /* <mvrotfile>   angles (degrees) of a table, axis          */
  SPH_MOV_NULL = 13      /* <mvnull>                                                 */
};
typedef struct SphMotionMov {
  int32_t obj;         /* motion object: its index in the nodes of sph_solver_set_motion_tree
                          (sph_solver_set_motion: the objreal ref = moving-block index)    */
  int32_t id;          /* movement id inside the object                                 */
  int32_t next;        /* id of the next movement of the object (0: none)               */
  int32_t type;        /* SPH_MOV_*                                                     */
  int32_t prev;        /* velprev / phaseprev: take the value of the previous movement   */
  int32_t fields;      /* RECTFILE: bit k set when coordinate k is in the file (fieldx/y/z >= 0) */
  uint32_t data_first; /* RECTFILE / ROTFILE: its first row of the tree call's table rows */
  uint32_t data_n;     /* ... and its rows (>= 2)                                        */
  double duration;     /* < 0: a flash movement (applied whole at its start)            */
  double vec[3], vec2[3], phase[3];
  double axisp1[3], axisp2[3], ref[3];
  double ang, ang2, ang3;
} SphMotionMov;
/* <begin mov start finish>: movement `mov` (id) of object `obj` starts at `start`
 * (finish < 0: no forced finish). */
typedef struct SphMotionEvent {
  int32_t obj, mov;
  double start, finish;
} SphMotionEvent;
/* Motion program of the case's moving objects (JDsMotion::Init, JDsMotion.cpp:94-106);
 * call once after sph_solver_create (or sph_slab_create, on every rank) and before the
 * first step; a restart calls sph_solver_set_time first (the program is advanced to it).  Evaluated on the device
 * every step (no host round trip), applied as JSphCpu::RunMotion (JSphCpu.cpp:1758-1789). */
int sph_solver_set_motion(SphSolver* s, uint32_t nobj, uint32_t nmov, const SphMotionMov* movs, uint32_t nevt,
                          const SphMotionEvent* evts);
/* A motion object of the program's tree (<obj> / <objreal> nested in each other,
 * JMotion::ReadXml + ObjAdd, JMotion.cpp:96-114,556-565): listed depth first, a parent
 * before its children and every subtree contiguous.  ref = the objreal ref (moving-block
 * index; the refs are 0..n-1), -1 for a virtual <obj> (its motion moves its children). */
typedef struct SphMotionObj {
  int32_t parent;  /* index of the parent node, -1 at the top level */
  int32_t ref;
} SphMotionObj;
/* The motion program as a tree of objects, with the tables of its file movements: rows of
 * four doubles {time, x, y, z} (RECTFILE) or {time, angle in degrees, 0, 0} (ROTFILE), as
 * JMotionDataFile loads them (JMotionMov.cpp:252-300).  sph_solver_set_motion is this call
 * with one top-level node per ref and no tables. */
int sph_solver_set_motion_tree(SphSolver* s, uint32_t nnode, const SphMotionObj* nodes, uint32_t nmov,
                               const SphMotionMov* movs, uint32_t nevt, const SphMotionEvent* evts, uint32_t nrows,
                               const double* rows);

/* Floating body (JCasePartBlock_Floating, JCaseParts.cpp:248-290 -> StFloatingData,
 * JSph.cpp:1046-1100), RigidAlgorithm=1 (SPH forces). */
typedef struct SphFloatingDef {
  uint32_t idbegin, count;     /* idp range of its particles                        */
  double massbody, masspart;   /* <massbody>, <masspart> (narrowed to float)        */
  double center[3];            /* <center>                                          */
  double inertia[9];           /* <inertia> row major (narrowed to float)           */
  double linvelini[3], angvelini[3];
  int32_t translationfree[3], rotationfree[3];
} SphFloatingDef;
/* Floating body state (StFloatingData members; PartFloat.fbi4 contents). */
typedef struct SphFloatingState {
  double center[3];
  float fvel[3], fomega[3], angles[3], facelin[3], faceang[3];
  float pad;
} SphFloatingState;
/* Configure the floating bodies (call once, before the first step); ftpause = FtPause.
 * On slabs every rank passes all bodies; their force sums are added over the ranks. */
int sph_solver_set_floatings(SphSolver* s, uint32_t nft, const SphFloatingDef* defs, double ftpause);
/* Imposed velocities and external forces of floating body `body` (JCasePartBlock_Floating
 * <linearvel> <angularvel> <linearforce> <angularforce>, JCaseParts.cpp:270-285 -> FtLinearVel,
 * FtAngularVel, FtLinearForce, FtAngularForce, JSph.cpp:1060-1082): a JLinearValue table of n
 * rows, times[n] nondecreasing and values[n][3], evaluated at the step's TimeStep by linear
 * interpolation (JLinearValue::GetValue3f, JLinearValue.cpp:209-390) inside RunFloating
 * (JSphCpuSingle.cpp:897-924): forces are added to the particle force sums before FtCalcForces;
 * velocities replace the integrated fvel/fomega components that are not "none" (DBL_MAX,
 * FtApplyImposedVel, :874-891), before the constraints.  Call after sph_solver_set_floatings,
 * before the first step (again for another table); on slabs on every rank. */
enum { SPH_FTTAB_LINVEL = 0, SPH_FTTAB_ANGVEL = 1, SPH_FTTAB_LINFORCE = 2, SPH_FTTAB_ANGFORCE = 3 };
int sph_solver_set_floating_table(SphSolver* s, uint32_t body, int32_t kind, uint32_t n, const double* times,
                                  const double* values);
int sph_solver_floatings(SphSolver* s, uint32_t cap, SphFloatingState* out, uint32_t* nft);
/* Time tables of the step (call before the first step, or after sph_solver_set_time; on
 * slabs on every rank; n >= 2 rows in any order, walked forward from the row of the last
 * lookup as the reference walks them (Position), n = 0 removes the table):
 *   SPH_TTAB_DTFIXED  <parameter DtFixedFile>: dt(t) of every step, values in ms as in the
 *                     file (JDsFixedDt::LoadFile/GetDt, JDsFixedDt.cpp; applied in DtVariable
 *                     before the NaN check and the DtMin floor, JSphCpu.cpp:1621);
 *   SPH_TTAB_VISCO    <parameter ViscoTime>: Visco(t) (JDsViscoInput, float rows), set at the
 *                     start of every step from its TimeStep (JSphCpuSingle.cpp:1092); the
 *                     boundary viscosity is Visco x ViscoBoundFactor. */
enum { SPH_TTAB_DTFIXED = 0, SPH_TTAB_VISCO = 1 };
int sph_solver_set_time_table(SphSolver* s, int32_t kind, uint32_t n, const double* times, const double* values);
/* PartFloat.fbi4 (JPartFloatBi4Save::SaveInitial + AddPartFloat/SavePartFloat,
 * JPartFloatBi4.cpp:243-346): per-body head arrays [nft] and, per saved PART k, its
 * Cpart/Step/TimeStep and the body states center[k][nft][3], fvel, fomega, facelin,
 * faceang [k][nft][3]; readable by the reference's JPartFloatBi4Load (FloatingInfo). */
int sph_partfloat_write(const char* path, const char* app, uint32_t mkboundfirst, uint32_t nft,
                        const uint16_t* mkbound, const uint32_t* begin, const uint32_t* count, const float* mass,
                        const float* massp, const float* radius, uint32_t nparts, const uint32_t* cpart,
                        const uint32_t* step, const double* timestep, const double* center, const float* fvel,
                        const float* fomega, const float* facelin, const float* faceang);
/* Restart of floating bodies (JSphCpu::InitFloating, JSphCpu.cpp:1885-1905): the state of
 * PART cpart in PartFloat.fbi4 (JPartFloatBi4Load::LoadPart) — center[nft][3], fvel, fomega
 * (any pointer may be NULL) and its TimeStep.  The reference restarts a body with these and
 * its angles at 0; a run driver passes them as the body's center / initial velocities. */
int sph_partfloat_read(const char* path, uint32_t cpart, uint32_t nft, double* center, float* fvel, float* fomega,
                       double* timestep);
/* mDBC extra data of a PART, PartExtra_%04u.bi4 (JDsExtraDataSave / JDsExtraDataLoad,
 * JDsExtraData.cpp; written every SaveExtraParts-th PART, -svextraparts): the Normals
 * float3[nsize] by idp, each the boundary particle's vector to its ghost node (twice the case
 * file's normal; turned with moving and floating bodies) and UseNormalsFt.  A restart with mDBC
 * reloads them (JSph::ConfigBoundNormals, JSph.cpp:1308-1316).  read: normals may be NULL
 * (nsize only); the case's CaseNbound / CaseNfloat must match the file's. */
int sph_extra_normals_read(const char* path, uint32_t casenbound, uint32_t casenfloat, uint32_t cap, float* normals,
                           uint32_t* nsize, int32_t* usenormalsft);
int sph_extra_normals_write(const char* path, const char* app, uint32_t cpart, uint32_t step, double timestep,
                            uint32_t casenbound, uint32_t casenfloat, int32_t usenormalsft, uint32_t nsize,
                            const float* normals);
/* The solver's current mDBC vectors particle -> ghost node by idp ([n][3]; normals NULL: n
 * only) and whether the floating bodies have them (UseNormalsFt) — JSphGpuSingle::SaveExtraData
 * (JSphGpuSingle.cpp:946-968). */
int sph_download_normals(SphSolver* s, uint32_t cap, float* normals, uint32_t* n, int32_t* usenormalsft);

#ifdef __cplusplus
}
#endif
#endif /* SPHCORE_H */
