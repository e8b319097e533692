// sph_device.hpp — device-side data layout and helpers of the MI355X SPH core.
//
// Layout in HBM (all arrays in cell-sorted order, SoA, 16-B aligned):
//   idp      u32     particle id                     (Idpg)
//   code     u16     type/special bits (DualSphDef.h:161-221)
//   dcell    u32     DCEL cell code (JDsDcellDef.h:24-43)
//   posxy    double2 x,y   } positions in double (JSphGpu posxy/posz)
//   posz     double  z     }
//   velrhop  float4  vx,vy,vz,rho
//   poscell  float4  position relative to the origin of its cell (float), w = dcell bits
//   press    float   EOS pressure (FunSphEos.h:37-47), computed once per divide
//   arace    float4  ace.x, ace.y, ace.z, ar  — interaction output (fused ar+ace)
// Time-integration extras: velrhopm1 (Verlet), posxypre/poszpre/velrhoppre (Symplectic).
// Device scalars (counts, maxima, dt, time) live in DevScalars so a whole step runs
// without a host round trip (the reference does >=6 blocking DtoH copies per step,
// SURVEY.md §3.2).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sphx {

typedef uint16_t typecode;

constexpr typecode CODE_MASKSPECIAL = 0xe000, CODE_OUTIGNORE = 0x4000, CODE_OUTMOVE = 0x6000,
                   CODE_OUTPOS = 0x8000, CODE_OUTRHOP = 0xA000, CODE_MASKTYPE = 0x1800,
                   CODE_TYPE_MOVING = 0x800, CODE_TYPE_FLOATING = 0x1000, CODE_TYPE_FLUID = 0x1800,
                   CODE_MASKVALUE = 0x7ff;
constexpr float ALMOSTZERO = 1e-18f;  // DualSphDef.h:132

__host__ __device__ inline typecode CodeSpecial(typecode c) { return c & CODE_MASKSPECIAL; }
__host__ __device__ inline typecode CodeType(typecode c) { return c & CODE_MASKTYPE; }
__host__ __device__ inline typecode CodeSetNormal(typecode c) { return c & typecode(~CODE_MASKSPECIAL); }
__host__ __device__ inline bool CodeIsNormal(typecode c) { return CodeSpecial(c) == 0; }
__host__ __device__ inline bool CodeIsFluid(typecode c) { return CodeType(c) == CODE_TYPE_FLUID; }
__host__ __device__ inline bool CodeIsOutRhop(typecode c) { return CodeSpecial(c) == CODE_OUTRHOP; }

// DCEL decoding (JDsDcellDef.h:36-39).
__host__ __device__ inline unsigned DcelCellx(unsigned dcc, unsigned cel) { return cel >> ((dcc >> 10) & 31); }
__host__ __device__ inline unsigned DcelCelly(unsigned dcc, unsigned cel) { return (cel << (dcc >> 25)) >> ((dcc >> 5) & 31); }
__host__ __device__ inline unsigned DcelCellz(unsigned dcc, unsigned cel) { return (cel << (dcc & 31)) >> (dcc & 31); }
__host__ __device__ inline unsigned DcelCell(unsigned dcc, unsigned cx, unsigned cy, unsigned cz) {
  return (cx << ((dcc >> 10) & 31)) | (cy << ((dcc >> 15) & 31)) | cz;
}

// Constants passed by value to every kernel (the reference's __constant__ CTE,
// JSphGpu_ker.cu:180-182, uploaded by cudaMemcpyToSymbol; here kernarg-resident).
struct KConst {
  float kernelh, kernelsize2, bwen, ovkernelh;
  float cteb, gamma, rhopzero, ovrhopzero;
  float massfluid, massbound, eta2, ddtkh;
  float ddtgz, cs0f, visco, viscobound;
  float scell, movlimit, rhopoutmin, rhopoutmax;
  float gravx, gravy, gravz, ovgamma;
  double gravxd, gravyd, gravzd;
  double map_realposmin_x, map_realposmin_y, map_realposmin_z;
  double map_realsize_x, map_realsize_y, map_realsize_z;
  double scelld;
  unsigned domcellcode;
  int tdensity;
  // derived for the tiled kernel
  float mhalfovh, bwenovh, ddtkhcs, ddtc1, ddtc2, ddtc3, ddtc4;
  int ddtseries;  // 1: |ddtgz*drz| <= 2h*ddtgz < 0.05 for every pair -> DDT2 hydrostatic term by series
  float ddte1, ddte2, ddte3, ddte4;  // the series in drz: rho0*((1+ddtgz*drz)^(1/gamma)-1) = drz*(e1+drz*(e2+...))
  float awen;  // Wendland W normalisation (mDBC)
  int mdbc;    // TBoundary == BC_MDBC: DDT (Molteni) keeps bound neighbours (JSphCpu.cpp:730)
  int scelldiv;  // 1 CellMode=full (cells of 2h), 2 half (cells of h): neighbour rows +-scelldiv
  // v5.0 NN multiphase (sph_nn.hip) and shifting (JSphShifting::RunCpu, JSphShifting.cpp:388-418)
  int nn;          // RheologyTreatment == 2
  int nntvisco;    // TpVisco of the NN interaction: 1 artificial, 2 laminar, 3 constitutive eq.
  int nnvelgrad;   // VelocityGradientType: 1 FDA, 2 SPH (two passes: k_nn_tiled, then k_nn_visc)
  int tvisco;      // single phase: 1 artificial, 2 Laminar+SPS (sph_ext.hip)
  float spssmag, spsblin;  // Laminar+SPS constants SpsSmag, SpsBlin (JSph.cpp:1438-1443)
  int shiftmode;   // TpShifting: 0 none, 1 NoBound, 2 NoFixed, 3 Full
  int sim2d;       // Simulate2D: ace.y = 0 after the interaction
  float lamda;     // RelaxationDt of the viscous dt (JSphCpu.cpp:1687)
  float shifttfs;  // ShiftTFS (0: no free-surface detection)
  float shiftmaxdist;   // float(Dp*0.1)
  float shiftcoef;      // ShiftCoef
  double coeftfs;       // (Simulate2D ? 2 : 3) - ShiftTFS
  int nnbi;             // NN: some phase has a bi-viscosity region (tau_max != 0)
  // kernel: 0 Wendland, 1 Cubic spline (StKCubicCte, FunSphKernel.h:51-84); kfold = the
  // per-pass kernel factor folded out of the tiled sums (bwen/h, or 1 for the Cubic)
  int cubic;
  float kfold, cub_a2, cub_a24, cub_c1, cub_d1, cub_c2, cub_odw;
  // time-dependent step options (JSph::LoadConfigParameters, JSph.cpp:619-622,697-707):
  // DtAllParticles (VelMax over every particle, JSphCpu.cpp:475), DtFixed / DtFixedFile
  // (JDsFixedDt: a constant dt, or dt(t) from rows of (time [s], dt [ms])) and ViscoTime
  // (JDsViscoInput: Visco(t), evaluated at every step's TimeStep, JSphCpuSingle.cpp:1092)
  int dtallp;
  int symmetry;  // Symmetry: images across y = 0 of the p2 near it (JSphCpu.cpp:566-613, 671-796)
  int nftbodies; // floating bodies (their particle masses: the NN kernel's fourth phase-table row)
  int dtfix_n;
  double dtfix_val;
  const double* dtfix_t;
  const double* dtfix_v;
  int visco_n;
  float viscobf;  // ViscoBoundFactor: the boundary's visco from the current Visco
  const float* visco_t;
  const float* visco_v;
};

// JDsFixedDt::GetDt (JDsFixedDt.cpp:103-125) at TimeStep t: the constant, or the table's
// row interval found by the reference's forward walk, which continues from the row the last
// call stopped at (Position, kept in DevScalars::dtfix_pos; rows in any order, as the
// reference's LoadFile accepts them), dt in ms -> s.
__device__ __forceinline__ double fixed_dt(const KConst& K, double t, int& pos) {
  if (K.dtfix_val > 0) return K.dtfix_val;
  const double* T = K.dtfix_t;
  const double* V = K.dtfix_v;
  const int n = K.dtfix_n;
  double tini = T[pos], tnext = (pos + 1 < n ? T[pos + 1] : tini);
  for (; tnext < t && pos + 2 < n; pos++) {
    tini = tnext;
    tnext = T[pos + 2];
  }
  if (t <= tini) return V[pos] / 1000;
  if (t >= tnext) return V[pos + 1] / 1000;
  const double f = (t - tini) / (tnext - tini);
  return (f * (V[pos + 1] - V[pos]) + V[pos]) / 1000;
}
// JDsViscoInput::GetVisco (JDsViscoInput.cpp:103-127) at float(TimeStep), in its float/double
// mix, walking on from the row of the last call (DevScalars::visco_pos).
__device__ __forceinline__ float visco_at(const KConst& K, float t, int& pos) {
  const float* T = K.visco_t;
  const float* V = K.visco_v;
  const int n = K.visco_n;
  float tini = T[pos], tnext = (pos + 1 < n ? T[pos + 1] : tini);
  for (; tnext < t && pos + 2 < n; pos++) {
    tini = tnext;
    tnext = T[pos + 2];
  }
  if (t <= tini) return V[pos];
  if (t >= tnext) return V[pos + 1];
  const double f = double(t - tini) / double(tnext - tini);
  const float vini = V[pos], vnext = V[pos + 1];
  return float(f * (vnext - vini) + vini);
}

// NN phase constants on the device, two float4 per phase (sph_nn.hip loads them to LDS):
//   [2k]   = {mass, cs0, visco, tau_yield}
//   [2k+1] = {HBP_m, HBP_n, tau_max, Bi_multi}
// and the EOS of each phase for the divide's press: {rho0, 1/rho0, cteb, gamma}.
constexpr int NN_MAXPH = 8;

// Cell grid of the (fixed) divide domain — StDivDataGpu (JCellDivDataGpu.h:26-79).
// Slab decomposition (sph_slab.hip) along the SLAB AXIS (axis 0: x, axis 1: y): a rank's grid
// covers the global cells [soff, soff + extent) of that axis (the full extent of the other
// two); the ones it owns are the local [sown0, sown1) and the W cells either side of them
// (the ghost rim, W = the ghost width) hold read-only ghost copies of the neighbours'
// particles.  dcell stays GLOBAL (same cell code as a single domain); poscell.w carries the
// LOCAL cell (the global one shifted by soff along the axis).  Single domain: axis 0, soff
// 0, own [0, ncx).  x-slabs cut the cell rows at the faces; y-slabs keep every x row whole
// (a row is all owned or all ghost), so their items and the ghost overlap's interior / face
// lists are whole rows.
struct DivGrid {
  int ncx, ncy, ncz;
  unsigned nsheet, nct;
  unsigned boxboundignore, boxfluid, boxboundout, boxfluidout, boxboundoutignore, boxfluidoutignore;
  unsigned nctt;        // size of begincell = 2*nct + 6
  unsigned boxdiscard;  // ghosts of the previous divide and particles handed to a neighbour
  int axis;             // slab axis (0 x, 1 y)
  int soff, sown0, sown1;
  __host__ __device__ int extent() const { return axis ? ncy : ncx; }  // local cells along the axis
  __host__ __device__ int offx() const { return axis ? 0 : soff; }
  __host__ __device__ int offy() const { return axis ? soff : 0; }
  __host__ __device__ bool split() const { return sown0 != 0 || sown1 != extent(); }  // a slab grid
};

// Local coordinate along the slab axis of a GLOBAL dcell.
__host__ __device__ __forceinline__ int slab_local(const DivGrid& g, unsigned dcc, unsigned dc) {
  return int(g.axis ? DcelCelly(dcc, dc) : DcelCellx(dcc, dc)) - g.soff;
}
__host__ __device__ __forceinline__ bool slab_owned(const DivGrid& g, int l) { return l >= g.sown0 && l < g.sown1; }

// Slab faces: a slab has sown0 (= extent - sown1) ghost cells per face along the axis, the
// support radius 2h in cells (1 with full cells, 2 with half cells; +1 with mDBC).  The owned
// cells a neighbour needs as its ghosts are the first / last sown0 owned ones.
__host__ __device__ __forceinline__ bool in_left_face(const DivGrid& g, int l) {
  return l >= g.sown0 && l < 2 * g.sown0;
}
__host__ __device__ __forceinline__ bool in_right_face(const DivGrid& g, int l) {
  return l < g.sown1 && l >= g.sown1 - (g.extent() - g.sown1);
}

// dcell markers: excluded particle (JSphCpu::UpdatePos, JSphCpu.cpp:1262) and a
// particle this rank drops at the next divide (slab ghosts).
constexpr unsigned DCELL_OUT = 0xFFFFFFFFu, DCELL_DISCARD = 0xFFFFFFFEu;

// Device-resident step scalars.
struct DevScalars {
  unsigned np, npb, npbok, nout;          // counts after the last divide
  unsigned nitems, nitems_bound, nown;    // (unused); owned particles (slab)
  float visco;                            // Visco of the step (ViscoTime; else K.visco)
  unsigned dtmodif, error_flags, npbout, ndiv;  // ndiv: particle count entering the divide
  unsigned long long nstep;
  double dt;        // dt of the step in flight
  double time;      // simulated time TimeStep
  double symdtpre;  // SymplecticDtPre
  double ddt_p;     // predictor dt (Symplectic)
  double last_dt;
  double tstep0;    // TimeStep at the start of the step in flight (motion, FtPause)
  float last_velmax, last_acemax, last_viscdt, last_visceta;
  int dtfix_pos, visco_pos;  // the DtFixedFile / ViscoTime tables' rows of the last lookup
  // Max-reductions (float bits of values >= 0) spread over RED_SLOTS slots so that
  // thousands of waves do not serialise on one address; k_dt folds and clears them.
  unsigned red[4][64];
};
// RED_VISCETA: NN max effective viscosity (ViscEtaDtMax, JSphCpuSingle.cpp:633 in the v5.0 solver)
constexpr int RED_VELMAX2 = 0, RED_ACEMAX2 = 1, RED_VISCDT = 2, RED_VISCETA = 3, RED_SLOTS = 64;

constexpr unsigned ERR_DT_NAN = 1u, ERR_BOUNDOUT = 2u;
// slab halo errors, by site: an mDBC ghost node whose support leaves the slab's grid, a face
// record that does not fit its buffer, a face record with no ghost copy to land in, a ghost
// record the divide cannot fill
constexpr unsigned ERR_HALO_NODE = 4u, ERR_HALO_FACE = 8u, ERR_HALO_MISS = 16u, ERR_HALO_GHOST = 32u;
constexpr unsigned ERR_HALO = ERR_HALO_NODE | ERR_HALO_FACE | ERR_HALO_MISS | ERR_HALO_GHOST;
// Errors the reference throws on (DtVariable, JSphCpu.cpp:1622; AbortBoundOut in
// RunCellDivide): once one is flagged, a batched run stops stepping ON THE DEVICE — k_dt
// no longer advances time/nstep and the update, motion and floating kernels leave the
// state as it was, so the run ends at the failing step and sph_solver_sync reports it.
// ERR_HALO (slabs: a ghost record the divide cannot fill, a face re-send record with no
// ghost copy to land in, an mDBC ghost node reaching past the ghost columns) halts too: it
// is folded into the dt all-reduce (folded[4]), so every slab stops at the same step rather
// than stepping on with incomplete face data.
constexpr unsigned ERR_FATAL = ERR_DT_NAN | ERR_BOUNDOUT | ERR_HALO;
__device__ __forceinline__ bool halted(const DevScalars* sc) { return (sc->error_flags & ERR_FATAL) != 0u; }

// Wave-level max of a non-negative float, then one atomicMax per wave into a slot
// chosen by the wave's global index (64 slots).
// A NaN is carried as the canonical quiet NaN, whose bits exceed every finite value and
// +inf: it wins the integer max and reaches k_dt, which then stops the run (ERR_DT_NAN).
__device__ inline void wave_max_atomic(DevScalars* sc, int which, float v) {
  unsigned b = (v != v) ? 0x7fc00000u : __float_as_uint(fmaxf(v, 0.f));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b = max(b, (unsigned)__shfl_xor((int)b, off, 64));
  const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && b) atomicMax(&sc->red[which][wave & (RED_SLOTS - 1)], b);
}
// max that keeps a NaN (fmaxf drops it): per-thread VelMax accumulation, so that a NaN
// velocity reaches the dt (the reference's DtVariable check, JSphCpu.cpp:1622)
__device__ __forceinline__ float nanmax(float a, float x) { return (x != x || a != a) ? __builtin_nanf("") : fmaxf(a, x); }

}  // namespace sphx
