// sph_solver.cpp — host orchestration (see sph_solver.hpp).
#include "sph_solver.hpp"
#include "sph_items.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <exception>
#include <thread>

namespace sphx {

// SPH_TRACE_SLAB=1: one stderr line per slab phase (rank, step, phase) -- a diagnostic of the
// slab protocol's host side (which rank waits where)
static bool trace_slab() {
  static const bool on = [] {
    const char* e = std::getenv("SPH_TRACE_SLAB");
    return e && *e == '1';
  }();
  return on;
}
#define SLAB_TRACE(what)                                                                                     \
  do {                                                                                                      \
    if (trace_slab() && slab())                                                                             \
      std::fprintf(stderr, "slabtrace rank %d step %llu %s\n", slabcfg_.rank, stepsdone_, what);          \
  } while (0)

// Test hooks read from the environment (buffer sizing, item cutting, slab turns) change how a
// run is executed, never its results; a production run must not pick one up silently, so the
// first one met is reported once on stderr.
void test_hook_notice(const char* name) {
  static bool said = false;
  if (said) return;
  said = true;
  std::fprintf(stderr, "libsphcore: test hook %s is set in the environment (measurement / test mode)\n", name);
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw SphError(SPH_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// ---- JSph::ConfigConstants1/2 (JSph.cpp:1392-1457), ConfigCellDivision (:1772-1788),
//      map limits (:2062-2076), SelecDomain/CalcCellCode (:1794-1829, JDsDcell.cpp:30-69) ----
static unsigned bits_for(unsigned v, unsigned minbits) {
  unsigned n = minbits;
  for (; v >> n; n++) {}
  return n;
}
static unsigned cell_code(unsigned nx, unsigned ny, unsigned nz) {
  unsigned sx = bits_for(nx, 2), sy = bits_for(ny, 2), sz = bits_for(nz, 2);
  const unsigned smin = sx + sy + sz;
  if (smin > 31) return 0;
  for (unsigned rest = 31 - smin; rest;) {
    if (rest) { sx++; rest--; }
    if (rest) { sy++; rest--; }
    if (rest) { sz++; rest--; }
  }
  return ((sx + 1) << 25) | (sy << 20) | (sz << 15) | ((sy + sz) << 10) | ((sx + 1 + sz) << 5) | (sx + 1 + sy);
}

void derive_constants(const SphCaseDef& c, SphConstants& k) {
  if (c.kernel != SPH_KERNEL_WENDLAND && c.kernel != SPH_KERNEL_CUBIC)
    throw SphError(SPH_ERR_ARG, "Kernel choice is not valid.");
  if (c.cellmode != SPH_CELLMODE_FULL && c.cellmode != SPH_CELLMODE_HALF) throw SphError(SPH_ERR_ARG, "invalid cellmode");
  if (c.step_algorithm != SPH_STEP_VERLET && c.step_algorithm != SPH_STEP_SYMPLECTIC)
    throw SphError(SPH_ERR_ARG, "invalid step algorithm");
  if (c.tdensity < 0 || c.tdensity > 3) throw SphError(SPH_ERR_ARG, "invalid DDT mode");
  if (c.npb > c.np) throw SphError(SPH_ERR_ARG, "npb > np");
  std::memset(&k, 0, sizeof(k));
  k.kernelh = float(c.h);
  k.cteb = float(c.cteb);
  k.gamma = float(c.gamma);
  k.rhopzero = float(c.rhop0);
  k.massfluid = float(c.massfluid);
  k.massbound = float(c.massbound);
  for (int i = 0; i < 3; i++) k.gravity[i] = float(c.gravity[i]);
  k.cflnumber = c.cflnumber;
  k.dp = c.dp;
  k.visco = float(c.visco);
  k.viscoboundfactor = float(c.viscoboundfactor);
  k.rhopoutmin = float(c.rhopoutmin);
  k.rhopoutmax = float(c.rhopoutmax);
  k.tdensity = c.tdensity;
  k.step_algorithm = c.step_algorithm;
  k.verlet_steps = c.verlet_steps;
  const double h = k.kernelh;
  k.kernelsize = float(h * 2.0f);  // Wendland factor 2 (FunSphKernel.h:190)
  k.kernelsize2 = k.kernelsize * k.kernelsize;
  k.data2d = c.data2d ? 1 : 0;
  if (k.data2d) {  // GetKernelWendland_Ctes(sim2d) (FunSphKernel.h:193-196)
    k.awen = float(0.557 / (h * h));
    k.bwen = float(-2.7852 / (h * h * h));
  } else {
    k.awen = float(0.41778 / (h * h * h));
    k.bwen = float(-2.08891 / (h * h * h * h));
  }
  k.kernel = c.kernel;
  if (k.kernel == SPH_KERNEL_CUBIC) {  // GetKernelCubic_Ctes (FunSphKernel.h:51-84)
    const double pi = 3.14159265358979323846;  // TypesDef.h:24
    const double a1 = k.data2d ? 10. / (pi * 7.) : 1. / pi;
    const double a2 = k.data2d ? a1 / (h * h) : a1 / (h * h * h);
    const double aa = k.data2d ? a1 / (h * h * h) : a1 / (h * h * h * h);
    const double deltap = 1. / 1.5;
    const double wdeltap = a2 * (1. - 1.5 * deltap * deltap + 0.75 * deltap * deltap * deltap);
    k.cub_od_wdeltap = float(1. / wdeltap);
    k.cub_a1 = float(a1);
    k.cub_a2 = float(a2);
    k.cub_aa = float(aa);
    k.cub_a24 = float(0.25 * a2);
    k.cub_c1 = float(-3. * aa);
    k.cub_d1 = float(9. * aa / 4.);
    k.cub_c2 = float(-3. * aa / 4.);
  }
  k.cs0 = std::sqrt(double(k.gamma) * double(k.cteb) / double(k.rhopzero));
  k.eta2 = float((h * 0.1) * (h * 0.1));
  k.ovrhopzero = 1.0f / k.rhopzero;
  k.ddtkh = k.kernelsize * float(c.ddtvalue);
  k.ddtgz = float(double(k.rhopzero) * double(std::fabs(k.gravity[2])) / double(k.cteb));
  k.dtini = c.dtini ? c.dtini : k.kernelh / k.cs0;
  k.dtmin = c.dtmin ? c.dtmin : (k.kernelh / k.cs0) * float(c.coefdtmin);
  k.scelldiv = (c.cellmode == SPH_CELLMODE_HALF ? 2 : 1);  // cells of 2h (full) or h (half)
  k.scell = k.kernelsize / k.scelldiv;
  k.movlimit = k.scell * 0.9f;
  for (int i = 0; i < 3; i++) {
    k.map_realposmin[i] = c.map_realposmin[i];
    k.map_realsize[i] = c.map_realposmax[i] - c.map_realposmin[i];
    k.dom_posmin[i] = c.map_realposmin[i];
    if (!(k.map_realsize[i] > 0)) throw SphError(SPH_ERR_ARG, "invalid map limits");
    k.dom_cells[i] = unsigned(std::ceil(k.map_realsize[i] / k.scell));
  }
  k.dom_cellcode = cell_code(k.dom_cells[0] + 1, k.dom_cells[1] + 1, k.dom_cells[2] + 1);
  if (!k.dom_cellcode) throw SphError(SPH_ERR_ARG, "failed to select a valid CellCode");
  // Boundary configuration (JSph.cpp:626-640, 785-790).
  k.tboundary = (c.tboundary == 0 ? SPH_BOUND_DBC : c.tboundary);
  if (k.tboundary != SPH_BOUND_DBC && k.tboundary != SPH_BOUND_MDBC)
    throw SphError(SPH_ERR_ARG, "Boundary Condition method is not valid.");
  k.slipmode = (k.tboundary == SPH_BOUND_MDBC ? (c.slipmode == 0 ? SPH_SLIP_VEL0 : c.slipmode) : SPH_SLIP_VEL0);
  if (k.slipmode != SPH_SLIP_VEL0)
    throw SphError(SPH_ERR_UNSUPPORTED, "Only the slip mode velocity=0 is allowed with mDBC conditions.");
  k.mdbc_threshold = (k.tboundary == SPH_BOUND_MDBC ? float(c.mdbc_threshold) : 0.f);
  // Rheology, viscosity and shifting options (JSph::LoadConfigParameters, JSph.cpp:608-700 of
  // the v5.0 solver; JSph.cpp:620-700 of v5.2).
  k.rheology = (c.rheology == 0 ? SPH_RHEOLOGY_SINGLE : c.rheology);
  k.velgrad = (c.velgrad == 0 ? SPH_VELGRAD_FDA : c.velgrad);
  k.tvisco = (c.tvisco == 0 ? SPH_VISCO_ARTIFICIAL : c.tvisco);
  k.shift_mode = c.shift_mode;
  k.shift_coef = float(c.shift_coef);
  k.shift_tfs = float(c.shift_tfs);
  k.relaxation_dt = float(c.relaxation_dt);
  if (k.rheology != SPH_RHEOLOGY_SINGLE && k.rheology != SPH_RHEOLOGY_NN)
    throw SphError(SPH_ERR_ARG, "Rheology treatment is not valid.");
  if (k.velgrad != SPH_VELGRAD_FDA && k.velgrad != SPH_VELGRAD_SPH)
    throw SphError(SPH_ERR_ARG, "Velocity gradient treatment is not valid.");
  if (k.tvisco < SPH_VISCO_ARTIFICIAL || k.tvisco > SPH_VISCO_CONSTEQ)
    throw SphError(SPH_ERR_ARG, "Viscosity treatment is not valid.");
  if (k.shift_mode < SPH_SHIFT_NONE || k.shift_mode > SPH_SHIFT_FULL)
    throw SphError(SPH_ERR_ARG, "Shifting mode is not valid.");
  k.dtallparticles = c.dtallparticles ? 1 : 0;  // JSph.cpp:697
  // Symmetry (JSph.cpp:714; its checks :1174-1179, MapRealPosMin.y = 0 :1386)
  k.symmetry = c.symmetry ? 1 : 0;
  if (k.symmetry) {
    if (k.data2d) throw SphError(SPH_ERR_ARG, "Symmetry is not allowed with 2-D simulations.");
    if (k.tvisco != SPH_VISCO_ARTIFICIAL) throw SphError(SPH_ERR_ARG, "Symmetry is only allowed with Artificial viscosity.");
    if (c.map_realposmin[1] != 0.0) throw SphError(SPH_ERR_ARG, "Symmetry needs MapRealPosMin.y = 0 (JSph.cpp:1386)");
    if (k.rheology != SPH_RHEOLOGY_SINGLE)
      throw SphError(SPH_ERR_UNSUPPORTED, "Symmetry is implemented for the single-phase interaction");
  }
  if (!(c.dtfixed >= 0)) throw SphError(SPH_ERR_ARG, "DtFixed must not be negative");
  k.dtfixed = c.dtfixed;  // max(0, DtFixed), JSph.cpp:699
  if (k.rheology == SPH_RHEOLOGY_SINGLE) {
    if (k.tvisco == SPH_VISCO_CONSTEQ)
      throw SphError(SPH_ERR_ARG, "ViscoTreatment 'Constitutive  eq.' not valid for Single-phase classic formulation.");
    if (k.tvisco == SPH_VISCO_LAMINARSPS) {  // JSph::ConfigConstants2 (JSph.cpp:1438-1443)
      const double dp_sps = (k.data2d ? std::sqrt(c.dp * c.dp * 2.) / 2. : std::sqrt(c.dp * c.dp * 3.) / 3.);
      k.spssmag = float(std::pow(0.12 * dp_sps, 2));
      k.spsblin = float((2. / 3.) * 0.0066 * dp_sps * dp_sps);
    }
    return;
  }
  // NN multiphase: JSph::InitMultiPhase + ConfigConstantsMP (JSph.cpp:3137-3242, v5.0 solver)
  if (k.tboundary == SPH_BOUND_MDBC)
    throw SphError(SPH_ERR_ARG, "Multiphase formulations are not supported with BC_mDBC.");
  if (c.nphases < 1 || c.nphases > SPH_MAXPHASES) throw SphError(SPH_ERR_ARG, "The number of phases is invalid.");
  k.nphases = c.nphases;
  bool cs0_present = true;
  for (unsigned p = 0; p < c.nphases; p++) {
    if (c.phases[p].phasetype != 0) throw SphError(SPH_ERR_UNSUPPORTED, "only phasetype 0 (non-Newtonian) exists in v5.0");
    if (p && c.phases[p].mkfluid <= c.phases[p - 1].mkfluid)
      throw SphError(SPH_ERR_ARG, "phases must be sorted by mkfluid");
    if (!float(c.phases[p].cs0)) cs0_present = false;
  }
  for (unsigned p = 0; p < c.nphases; p++) {
    const SphPhaseDef& ph = c.phases[p];
    const float rho = float(ph.rho), gam = (float(ph.gamma) ? float(ph.gamma) : k.gamma), cs = float(ph.cs0);
    k.phase_mass[p] = float(double(rho) * (k.data2d ? c.dp * c.dp : c.dp * c.dp * c.dp));
    // with a <csound> for every phase: CteB of InitMultiPhase (float arithmetic), else from
    // the case's Cs0 (ConfigConstantsMP, double arithmetic)
    k.phase_cteb[p] = cs0_present ? cs * cs * rho / gam : float(k.cs0 * k.cs0 * double(rho) / double(gam));
  }
  // DtMin is set here whatever the XML gives (ConfigConstantsMP runs after the parameters
  // are read, and ConfigConstants2 keeps a non-zero DtMin)
  const float coefdtmin = float(c.coefdtmin) * 1.0e-5f;  // CoefDtMin*=1.0e-5f
  k.dtmin = (double(k.kernelh) / k.cs0) * double(coefdtmin);
}

static KConst make_kconst(const SphConstants& c) {
  KConst K;
  std::memset(&K, 0, sizeof(K));
  K.kernelh = c.kernelh;
  K.kernelsize2 = c.kernelsize2;
  K.bwen = c.bwen;
  K.ovkernelh = 1.0f / c.kernelh;
  K.cteb = c.cteb;
  K.gamma = c.gamma;
  K.rhopzero = c.rhopzero;
  K.ovrhopzero = c.ovrhopzero;
  K.massfluid = c.massfluid;
  K.massbound = c.massbound;
  K.eta2 = c.eta2;
  K.ddtkh = c.ddtkh;
  K.ddtgz = c.ddtgz;
  K.cs0f = float(c.cs0);
  K.visco = c.visco;
  K.viscobound = c.visco * c.viscoboundfactor;
  K.scell = c.scell;
  K.movlimit = c.movlimit;
  K.rhopoutmin = c.rhopoutmin;
  K.rhopoutmax = c.rhopoutmax;
  K.gravx = c.gravity[0];
  K.gravy = c.gravity[1];
  K.gravz = c.gravity[2];
  K.ovgamma = 1.f / c.gamma;
  K.gravxd = c.gravity[0];
  K.gravyd = c.gravity[1];
  K.gravzd = c.gravity[2];
  K.map_realposmin_x = c.map_realposmin[0];
  K.map_realposmin_y = c.map_realposmin[1];
  K.map_realposmin_z = c.map_realposmin[2];
  K.map_realsize_x = c.map_realsize[0];
  K.map_realsize_y = c.map_realsize[1];
  K.map_realsize_z = c.map_realsize[2];
  K.scelld = double(c.scell);
  K.domcellcode = c.dom_cellcode;
  K.tdensity = c.tdensity;
  K.mhalfovh = -0.5f * K.ovkernelh;
  K.bwenovh = c.bwen * K.ovkernelh;
  // Cubic spline (FunSphKernel.h:38-175): the tiled kernels evaluate its fac directly, so
  // the per-pass factor the Wendland (bwen/h) takes is 1
  K.cubic = (c.kernel == SPH_KERNEL_CUBIC) ? 1 : 0;
  K.kfold = K.cubic ? 1.f : K.bwenovh;
  K.cub_a2 = c.cub_a2;
  K.cub_a24 = c.cub_a24;
  K.cub_c1 = c.cub_c1;
  K.cub_d1 = c.cub_d1;
  K.cub_c2 = c.cub_c2;
  K.cub_odw = c.cub_od_wdeltap;
  K.ddtkhcs = c.ddtkh * K.cs0f;
  K.awen = c.awen;
  K.mdbc = (c.tboundary == SPH_BOUND_MDBC) ? 1 : 0;
  K.scelldiv = c.scelldiv;
  K.nn = (c.rheology == SPH_RHEOLOGY_NN) ? 1 : 0;
  K.nntvisco = c.tvisco;
  K.nnvelgrad = c.velgrad;
  K.tvisco = c.tvisco;
  K.spssmag = c.spssmag;
  K.spsblin = c.spsblin;
  K.shiftmode = c.shift_mode;
  K.sim2d = c.data2d;
  K.lamda = c.relaxation_dt;
  K.shifttfs = c.shift_tfs;
  K.shiftcoef = c.shift_coef;
  K.shiftmaxdist = float(c.dp * 0.1);
  K.coeftfs = (c.data2d ? 2.0 : 3.0) - double(c.shift_tfs);
  K.dtallp = c.dtallparticles;
  K.symmetry = c.symmetry;
  K.dtfix_val = c.dtfixed;
  K.viscobf = c.viscoboundfactor;
  {  // binomial coefficients of (1+x)^(1/gamma) - 1
    const double a = 1.0 / double(c.gamma);
    K.ddtc1 = float(a);
    K.ddtc2 = float(a * (a - 1) / 2);
    K.ddtc3 = float(a * (a - 1) * (a - 2) / 6);
    K.ddtc4 = float(a * (a - 1) * (a - 2) * (a - 3) / 24);
    // |drz| <= 2h for every pair, so the series applies to all pairs of the case when
    // 2h*ddtgz is small (dam break: ~1e-3); decided once here, uniform in the kernel.
    // three terms: the x^4 term is 0.19 x^3 of the first, < 2e-6 for x < 0.02 (sph_interaction_tiled.hip)
    K.ddtseries = (double(c.kernelsize) * double(c.ddtgz) < 0.02) ? 1 : 0;
    const double gz = double(c.ddtgz), r0 = double(c.rhopzero);
    K.ddte1 = float(r0 * a * gz);
    K.ddte2 = float(r0 * a * (a - 1) / 2 * gz * gz);
    K.ddte3 = float(r0 * a * (a - 1) * (a - 2) / 6 * gz * gz * gz);
    K.ddte4 = float(r0 * a * (a - 1) * (a - 2) * (a - 3) / 24 * gz * gz * gz * gz);
  }
  return K;
}

// Ghost columns per slab face: the support radius 2h is one full cell or two half cells
// (scelldiv); with mDBC one column more, because a boundary particle's ghost node lies up
// to |2 normal| (about dp, less than a cell) from it and its search reaches 2h around the
// node (JSphCpu.cpp:1040-1047): a slab owning such a particle in its face column needs the
// fluid one column beyond.
int ghost_width(const SphConstants& c) { return int(c.scelldiv) + (c.tboundary == SPH_BOUND_MDBC ? 1 : 0); }

// Narrowest slab with neighbours on both sides: 2W columns, so that its two face column
// sets are disjoint.  A particle arriving from a neighbour (< one cell of movement) then
// lands in the face towards that neighbour, which keeps it as a ghost itself; in a narrower
// slab it could land in the opposite face and be missing from the other neighbour's ghosts
// until the next exchange.  A slab at the end of the map (one neighbour) needs W.
int min_slab_width(const SphConstants& c) { return 2 * ghost_width(c); }

// Full-map cell grid (JCellDivCpuSingle::PrepareNct, JCellDivCpuSingle.cpp:105-121, with CellDomFixed).
// A slab keeps the global extent of the other two axes and the cells [c0-W, c1+W) of its
// slab axis (owned + W ghost cells per face, W = ghost_width).
static DivGrid make_grid(const SphConstants& c, const SlabConfig* slab) {
  DivGrid g;
  g.ncx = int(c.dom_cells[0]);
  g.ncy = int(c.dom_cells[1]);
  g.ncz = int(c.dom_cells[2]);
  g.axis = 0;
  g.soff = 0;
  g.sown0 = 0;
  g.sown1 = g.ncx;
  if (slab) {
    const int W = ghost_width(c);
    const bool both = slab->rank > 0 && slab->rank + 1 < slab->nranks;
    if (slab->axis != 0 && slab->axis != 1) throw SphError(SPH_ERR_ARG, "slab axis must be 0 (x) or 1 (y)");
    const int ext = slab->axis ? g.ncy : g.ncx;
    if (slab->nranks < 1 || slab->rank < 0 || slab->rank >= slab->nranks || slab->c0 < 0 ||
        slab->c1 < slab->c0 + (both ? min_slab_width(c) : W) || slab->c1 > ext)
      throw SphError(SPH_ERR_ARG,
                     "invalid slab cells (a slab owns at least 2W cells of its axis, W at a map end; W = the ghost "
                     "width: scelldiv cells, +1 with mDBC)");
    g.axis = slab->axis;
    g.soff = slab->c0 - W;
    (slab->axis ? g.ncy : g.ncx) = slab->c1 - slab->c0 + 2 * W;
    g.sown0 = W;
    g.sown1 = W + slab->c1 - slab->c0;
  }
  g.nsheet = unsigned(g.ncx) * unsigned(g.ncy);
  const unsigned long long nct = (unsigned long long)g.nsheet * unsigned(g.ncz);
  if (nct * 2 + 7 >= (1ull << 31)) throw SphError(SPH_ERR_ARG, "the number of cells is too big");
  g.nct = unsigned(nct);
  g.boxboundignore = g.nct;
  g.boxfluid = g.boxboundignore + 1;
  g.boxboundout = g.boxfluid + g.nct;
  g.boxfluidout = g.boxboundout + 1;
  g.boxboundoutignore = g.boxfluidout + 1;
  g.boxfluidoutignore = g.boxboundoutignore + 1;
  g.boxdiscard = g.boxfluidoutignore + 1;
  g.nctt = g.nct * 2 + 6;
  return g;
}

// Global cell of every initial particle along `axis` (JSph::LoadDcellParticles, JSph.cpp:1690-1711).
static std::vector<unsigned> initial_columns(const SphConstants& C, const SphParticlesHost& h, int axis) {
  std::vector<unsigned> cx(h.n);
  for (unsigned p = 0; p < h.n; p++) {
    const double dx = h.pos[3 * p + axis] - C.dom_posmin[axis];
    cx[p] = dx >= 0 ? unsigned(dx / double(C.scell)) : 0u;
  }
  return cx;
}

// Contiguous split of the columns into nranks slabs of at least minw columns that
// minimises the heaviest slab (the step time of the slowest rank): bisection on the load
// bound L, each bound probed greedily (every slab takes columns while it stays <= L and
// leaves minw columns for each slab after it).  Falls back to the prefix quantiles when no
// bound is feasible (a slab of minw columns already exceeds every L tried).  cfg3 on 8
// ranks: heaviest slab 1.33M -> 1.21M particles (quantile cuts at whole columns of 143k /
// 190k particles had given one rank an extra column).
static bool greedy_split(const std::vector<double>& pre, int nranks, int minw, double L, int* b) {
  const int ncx = int(pre.size()) - 1;
  b[0] = 0;
  for (int r = 0; r < nranks - 1; r++) {
    const int lo = b[r] + minw, hi = ncx - (nranks - 1 - r) * minw;
    if (lo > hi || pre[size_t(lo)] - pre[size_t(b[r])] > L) return false;
    int e = lo;
    while (e < hi && pre[size_t(e) + 1] - pre[size_t(b[r])] <= L) e++;
    b[r + 1] = e;
  }
  b[nranks] = ncx;
  return pre[size_t(ncx)] - pre[size_t(b[nranks - 1])] <= L && ncx - b[nranks - 1] >= minw;
}

void partition_from_prefix(const std::vector<double>& pre, int nranks, int* b, int minw) {
  const int ncx = int(pre.size()) - 1;
  const double total = pre[size_t(ncx)];
  double lo = total / double(nranks), hi = total;
  std::vector<int> best(size_t(nranks) + 1, -1), t(size_t(nranks) + 1);
  if (greedy_split(pre, nranks, minw, hi, t.data())) best = t;
  for (int it = 0; it < 60 && best[0] == 0; it++) {
    const double mid = 0.5 * (lo + hi);
    if (greedy_split(pre, nranks, minw, mid, t.data())) {
      best = t;
      hi = mid;
    } else {
      lo = mid;
    }
  }
  if (best[0] == 0) {
    for (int r = 0; r <= nranks; r++) b[r] = best[size_t(r)];
    return;
  }
  // no feasible bound: the prefix quantiles, clamped to the minimum width
  b[0] = 0;
  b[nranks] = ncx;
  int c = 0;
  for (int r = 1; r < nranks; r++) {
    const double target = total * double(r) / double(nranks);
    while (c < ncx && pre[size_t(c)] < target) c++;
    int cut = c;
    if (cut > 0 && target - pre[size_t(cut) - 1] < pre[size_t(cut)] - target) cut--;
    cut = std::max(cut, b[r - 1] + minw);
    cut = std::min(cut, ncx - (nranks - r) * minw);
    b[r] = cut;
  }
}

void slab_partition(const SphCaseDef& cdef, const SphParticlesHost& all, int nranks, double bound_weight, int* b,
                    int axis) {
  SphConstants C;
  derive_constants(cdef, C);
  if (axis != 0 && axis != 1) throw SphError(SPH_ERR_ARG, "slab axis must be 0 (x) or 1 (y)");
  const int ncx = int(C.dom_cells[axis]), W = min_slab_width(C);
  if (nranks < 1 || (nranks > 1 && nranks * W > ncx))
    throw SphError(SPH_ERR_ARG, "nranks must be in [1, cells of the slab axis / (2 x ghost width)]");
  if (all.n != cdef.np) throw SphError(SPH_ERR_ARG, "particle count does not match the case");
  std::vector<double> w(size_t(ncx), 0.0);
  const std::vector<unsigned> cx = initial_columns(C, all, axis);
  for (unsigned p = 0; p < all.n; p++) w[std::min<unsigned>(cx[p], unsigned(ncx - 1))] += (p < cdef.npb ? bound_weight : 1.0);
  std::vector<double> pre(size_t(ncx) + 1, 0.0);
  for (int c = 0; c < ncx; c++) pre[size_t(c) + 1] = pre[size_t(c)] + w[size_t(c)];
  partition_from_prefix(pre, nranks, b, W);
}

SphGpuSingle::SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& init, int dev) : device(dev) {
  Init(cdef, init);
}

SphGpuSingle::SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& all, int dev, const SlabConfig& slab,
                           std::unique_ptr<SlabTransport> transport)
    : device(dev), transport_(std::move(transport)), slabcfg_(slab) {
  if (!transport_) throw SphError(SPH_ERR_ARG, "slab without a transport");
  if (transport_->rank != slab.rank || transport_->nranks != slab.nranks)
    throw SphError(SPH_ERR_ARG, "slab rank does not match the transport");
  Init(cdef, all);
}

void SphGpuSingle::Init(const SphCaseDef& cdef, const SphParticlesHost& init) {
  derive_constants(cdef, C);
  K = make_kconst(C);
  G = make_grid(C, slab() ? &slabcfg_ : nullptr);
  step_algorithm_ = cdef.step_algorithm;
  if (init.n != cdef.np) throw SphError(SPH_ERR_ARG, "particle count does not match the case");
  if (!init.n) throw SphError(SPH_ERR_ARG, "no particles");
  // Particles this solver holds: all (single domain) or owned + ghost columns (slab).
  std::vector<unsigned> sel;
  unsigned nown = init.n;
  if (slab()) {
    const std::vector<unsigned> cx = initial_columns(C, init, slabcfg_.axis);
    const int W = ghost_width(C);
    const int lo = slabcfg_.c0 - (slabcfg_.rank > 0 ? W : 0);
    const int hi = slabcfg_.c1 + (slabcfg_.rank + 1 < slabcfg_.nranks ? W : 0);
    nown = 0;
    for (unsigned p = 0; p < init.n; p++) {
      const int c = int(cx[p]);
      if (c >= lo && c < hi) sel.push_back(p);
      if (c >= slabcfg_.c0 && c < slabcfg_.c1) nown++;
    }
    if (sel.empty()) throw SphError(SPH_ERR_ARG, "slab without particles");
  } else {
    sel.resize(init.n);
    for (unsigned p = 0; p < init.n; p++) sel[p] = p;
  }
  npb0_ = 0;
  for (unsigned p : sel) npb0_ += (p < cdef.npb ? 1u : 0u);
  casenpb_ = cdef.npb;
  const unsigned n = unsigned(sel.size());
  if (const char* e = std::getenv("SPH_SLAB_MINCAP")) slab_mincap_ = slab() && std::atoi(e) != 0;
  if (const char* e = std::getenv("SPH_SLAB_CUT")) cut_items_ = slab() && std::atoi(e) != 0;
  if (slab_mincap_ || cut_items_) test_hook_notice(slab_mincap_ ? "SPH_SLAB_MINCAP" : "SPH_SLAB_CUT");
  cap_ = slab() ? n + (slab_mincap_ ? 16u : std::max(n / 2, 65536u)) : n;
  keybits_ = bits_for(G.boxdiscard, 1);
  // grid-sized buffers hold the widest grid a slab can get from a re-partition (all cells
  // of the slab axis + W = ghost_width ghost cells per face), so they never move
  gmax_ncx_ = int(C.dom_cells[0]) + (slab() && slabcfg_.axis == 0 ? 2 * ghost_width(C) : 0);
  gmax_ncy_ = int(C.dom_cells[1]) + (slab() && slabcfg_.axis == 1 ? 2 * ghost_width(C) : 0);
  nctmax_ = slab() ? unsigned(gmax_ncx_) * unsigned(gmax_ncy_) * unsigned(G.ncz) : G.nct;
  if (slab() && slabcfg_.axis == 1) {
    if (C.dom_cells[1] < 2u) throw SphError(SPH_ERR_UNSUPPORTED, "y-slabs of a 2-D case (one y row)");
    if (C.symmetry) throw SphError(SPH_ERR_UNSUPPORTED, "Symmetry (the y = 0 mirror) on y-slabs");
  }
  if (const char* e = std::getenv("SPH_INTERACTION")) tiled_ = std::string(e) != "simple";
  if (const char* e = std::getenv("SPH_COMM_TIMEOUT_S")) comm_timeout_s_ = std::max(1.0, std::atof(e));
  // incremental divide: distinct key offsets of the 27 neighbour cells (ncx >= 3, checked
  // again per divide for a re-partitioned slab; ncy >= 3 or a single y row), 30-bit counts
  inc_ok_ = G.ncx >= 3 && (G.ncy >= 3 || G.ncy == 1) && n < (1u << 29);
  if (const char* e = std::getenv("SPH_DIVIDE")) inc_ok_ = inc_ok_ && std::string(e) != "full";
  // The tiled kernel stages the 3x3 rows of 3 cells of CellMode=full, or the 5x5 rows of
  // 5 half-cells of CellMode=half (run_pass_half).
  nn_ = (C.rheology == SPH_RHEOLOGY_NN);
  nnsph_ = nn_ && C.velgrad == SPH_VELGRAD_SPH;
  casenp_ = cdef.np;
  shift_ = (C.shift_mode != SPH_SHIFT_NONE);
  sps_ = !nn_ && C.tvisco == SPH_VISCO_LAMINARSPS;
  ext_ = !nn_ && (sps_ || shift_);
  facex_ = slab() && (nnsph_ || sps_);
  mdbc_corrector_ = cdef.tboundary == SPH_BOUND_MDBC && cdef.mdbc_corrector != 0;
  if (ext_) tiled_ = true;
  if (C.kernel == SPH_KERNEL_CUBIC && nn_)
    throw SphError(SPH_ERR_UNSUPPORTED, "the Cubic spline kernel with NN multiphase is not implemented");
  if (C.kernel == SPH_KERNEL_CUBIC && !tiled_)
    throw SphError(SPH_ERR_UNSUPPORTED, "the Cubic spline kernel runs on the tiled interaction only");
  if (C.symmetry && !tiled_) throw SphError(SPH_ERR_UNSUPPORTED, "Symmetry runs on the tiled interaction only");
  if (slab()) {
    // the first interaction's face records (NN / SPS / mDBC face re-sends): the initial
    // particles of the face and ghost columns (both sides of a face count the same
    // particles); later from each exchange
    const std::vector<unsigned> cx = initial_columns(C, init, slabcfg_.axis);
    const bool hl = slabcfg_.rank > 0, hr = slabcfg_.rank + 1 < slabcfg_.nranks;
    const int W = ghost_width(C), c0 = slabcfg_.c0, c1 = slabcfg_.c1;
    for (unsigned p : sel) {
      const int c = int(cx[p]);
      face_sl_ += (hl && c >= c0 && c < c0 + W) ? 1u : 0u;
      face_sr_ += (hr && c >= c1 - W && c < c1) ? 1u : 0u;
      face_rl_ += (hl && c >= c0 - W && c < c0) ? 1u : 0u;
      face_rr_ += (hr && c >= c1 && c < c1 + W) ? 1u : 0u;
    }
  }
  if (nn_) {
    // the NN interaction is the tiled kernel of sph_nn.hip only (full or half cells)
    tiled_ = true;
  }
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
  try {
    AllocFixed();
    if (nn_) UploadPhases(cdef);
    AllocParticles(cap_);
    if (slab()) PresizeExchange(init);
    Upload(init, sel, nown);
    if (C.tboundary == SPH_BOUND_MDBC) UploadNormals(cdef, init);
    // ConfigDomain: RunCellDivide(true) (JSphCpuSingle.cpp:165-166), then InitRunGpu.
    RunCellDivide();
    exchange_armed_ = true;
    if (step_algorithm_ == SPH_STEP_VERLET)
      check_hip(hipMemcpyAsync(cur_.velrhopm1, cur_.velrhop, sizeof(float4) * cap_, hipMemcpyDeviceToDevice, stream),
                "init VelrhopM1");
    Sync();
    CheckErrors();
  } catch (...) {
    Free();
    (void)hipStreamDestroy(stream);
    stream = nullptr;
    throw;
  }
}

SphGpuSingle::~SphGpuSingle() {
  if (xstream_) (void)hipStreamSynchronize(xstream_);
  if (stream) (void)hipStreamSynchronize(stream);
  Free();
  for (auto& e : pending_) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  for (auto e : evpool_) (void)hipEventDestroy(e);
  if (xev_) (void)hipEventDestroy(xev_);
  if (ev_div_) (void)hipEventDestroy(ev_div_);
  if (ev_ghost_) (void)hipEventDestroy(ev_ghost_);
  if (xstream_) {
    (void)hipStreamSynchronize(xstream_);
    (void)hipStreamDestroy(xstream_);
  }
  if (stream) (void)hipStreamDestroy(stream);
}

void SphGpuSingle::AllocFixed() {
  auto dmalloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    check_hip(hipMalloc(&p, std::max<size_t>(bytes, 256)), "hipMalloc");
    allocs_.push_back(p);
    return p;
  };
  begincell_ = (unsigned*)dmalloc(4 * (2 * size_t(nctmax_) + 6));
  if (slab()) {  // re-partition: column counts [2 ncx] + the ranks' bounds [nranks + 1]
    colcnt_ = (float*)dmalloc(4 * (2 * size_t(C.dom_cells[slabcfg_.axis]) + size_t(slabcfg_.nranks) + 1));
  }
  // two lists x (fluid, bound) rows of item counts, for the widest grid of the run
  rowtmp_ = (unsigned*)dmalloc(4 * ITEMS_ROWTMP(std::max(G.ncy, gmax_ncy_), G.ncz));
  // the count pass's staged items (sph_items.hpp), sized for the widest grid of the run
  ricap_ = ITEMS_RICAP(std::max(G.ncx, gmax_ncx_));
  // test hook: smaller slots send more rows down the place pass's second walk
  // (tests/test_gpu_items.py checks the run is bitwise the same)
  if (const char* e = std::getenv("SPH_ITEMS_RICAP")) ricap_ = std::max(1u, std::min(ricap_, unsigned(std::atoi(e))));
  rowitems_ = (uint4*)dmalloc(sizeof(uint4) * (ITEMS_ROWTMP(std::max(G.ncy, gmax_ncy_), G.ncz) - 1) * ricap_);
  qctr_ = (unsigned*)dmalloc(QCTR_BYTES);
  check_hip(hipMemset(qctr_, 0, QCTR_BYTES), "zero work counters");
  sort_.digtot = (unsigned*)dmalloc(4 * (1u << RS_MAXBITS));
  if (inc_ok_) {
    begincell_alt_ = (unsigned*)dmalloc(4 * (2 * size_t(nctmax_) + 6));
    inc_.stayoff = (unsigned*)dmalloc(4 * (2 * size_t(nctmax_) + 6));
    inc_.nb2 = inc_blocks_boxes(G.nctt);
    if (const char* e = std::getenv("SPH_INC_DBG")) inc_.dbg = std::atoi(e);
    inc_.ctr = (unsigned*)dmalloc(4 * QSTRIDE);
    check_hip(hipMemset(inc_.ctr, 0, 4 * QSTRIDE), "zero far count");
  }
  if (facex_) idxmap_ = (unsigned*)dmalloc(4 * size_t(std::max(casenp_, 1u)));
  sc_ = (DevScalars*)dmalloc(sizeof(DevScalars));
  dttrace_ = (double*)dmalloc(8 * size_t(tracecap_));
  pairs_ = (unsigned long long*)dmalloc(8 * 6);
  folded_ = (unsigned*)dmalloc(4 * 8);
  slabcnt_ = (SlabCounts*)dmalloc(sizeof(SlabCounts));
  // the accumulated counts (nkeep, ghosts) start at zero; k_unpack_finish zeroes them again
  // at the end of every exchange
  check_hip(hipMemset(slabcnt_, 0, sizeof(SlabCounts)), "zero slab counts");
  if (slab()) {
    // face messages and their prefixes (the ghost exchange after the divide); the second
    // item list and its counters
    faces_.W = ghost_width(C);
    faces_.nfb = 2u * face_boxes_per_type(G, faces_.W);  // the full extent of the other axes: fixed
    for (int k = 0; k < 4; k++) {
      // the send messages' face-box counts accumulate in k_pack_count from zero; k_face_scan
      // zeroes them again once it has their prefixes
      faces_.msg[k] = (unsigned*)dmalloc(4 * (size_t(FMSG_HDR) + faces_.nfb));
      check_hip(hipMemset(faces_.msg[k], 0, 4 * (size_t(FMSG_HDR) + faces_.nfb)), "zero face messages");
      faces_.pre[k] = (unsigned*)dmalloc(4 * (size_t(faces_.nfb) + 1));
    }
    qctrf_ = (unsigned*)dmalloc(QCTR_BYTES);
    check_hip(hipMemset(qctrf_, 0, QCTR_BYTES), "zero work counters");
  }
  check_hip(hipHostMalloc((void**)&sc_host_, sizeof(DevScalars), hipHostMallocDefault), "hipHostMalloc");
  check_hip(hipHostMalloc((void**)&slabcnt_host_, sizeof(SlabCounts), hipHostMallocDefault), "hipHostMalloc");
}

// NN phase tables (JSph::InitMultiPhase + ConfigConstantsMP): the interaction's constants
// (sph_device.hpp layout) and the EOS of every phase for the divide's pressure.
void SphGpuSingle::UploadPhases(const SphCaseDef& cdef) {
  // rows [0, 2 NN_MAXPH): {mass, cs0, visco, tau_yield}, {m, n, tau_max, bi_multi} per phase;
  // rows [2 NN_MAXPH, 3 NN_MAXPH): per-phase products of the pair bodies, in float as the
  // kernels formed them per pair: {m tau_yield, -m log2(e), n - 1, DDTkh cs0}
  std::vector<float4> tab(3 * NN_MAXPH, make_float4(0.f, 0.f, 0.f, 0.f)), eos(NN_MAXPH, make_float4(1.f, 0.f, 1.f, 0.f));
  for (unsigned p = 0; p < C.nphases; p++) {
    const SphPhaseDef& ph = cdef.phases[p];
    tab[2 * p] = make_float4(C.phase_mass[p], float(ph.cs0), float(ph.visco), float(ph.tau_yield));
    tab[2 * p + 1] = make_float4(float(ph.hbp_m), float(ph.hbp_n), float(ph.tau_max), float(ph.bi_multi));
    if (float(ph.tau_max) != 0.f) K.nnbi = 1;  // the pair bodies take the bi-viscosity branch
    const float m = float(ph.hbp_m);
    tab[2 * NN_MAXPH + p] = make_float4(m * float(ph.tau_yield), -m * 1.4426950408889634f, float(ph.hbp_n) - 1.f,
                                        K.ddtkh * float(ph.cs0));
    const float gam = float(ph.gamma) ? float(ph.gamma) : C.gamma;
    const int ig = (gam == float(int(gam)) && gam >= 1.f && gam <= 16.f) ? int(gam) : 0;
    eos[p] = make_float4(float(ph.rho), C.phase_cteb[p], gam, float(ig));
    phase_rho_[p] = float(ph.rho);
  }
  for (float4** dst : {&phasek_, &phaseeos_}) {
    check_hip(hipMalloc((void**)dst, sizeof(float4) * 3 * NN_MAXPH), "hipMalloc phases");
    allocs_.push_back(*dst);
  }
  check_hip(hipMemcpy(phasek_, tab.data(), sizeof(float4) * tab.size(), hipMemcpyHostToDevice), "upload phases");
  check_hip(hipMemcpy(phaseeos_, eos.data(), sizeof(float4) * eos.size(), hipMemcpyHostToDevice), "upload phases");
}

// Everything sized by the particle capacity (both gather sets, sort scratch, slab tiles).
void SphGpuSingle::AllocParticles(unsigned cap) {
  auto dmalloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    check_hip(hipMalloc(&p, std::max<size_t>(bytes, 256)), "hipMalloc");
    pallocs_.push_back(p);
    return p;
  };
  const size_t n = cap;
  for (PartArrays* a : {&cur_, &alt_}) {
    *a = PartArrays();
    a->idp = (unsigned*)dmalloc(4 * n);
    a->code = (typecode*)dmalloc(2 * n);
    a->dcell = (unsigned*)dmalloc(4 * n);
    a->posxy = (double2*)dmalloc(16 * n);
    a->posz = (double*)dmalloc(8 * n);
    a->velrhop = (float4*)dmalloc(16 * n);
    if (sps_) a->tau = (float4*)dmalloc(32 * n);
    if (step_algorithm_ == SPH_STEP_VERLET) {
      a->velrhopm1 = (float4*)dmalloc(16 * n);
    } else {
      a->posxypre = (double2*)dmalloc(16 * n);
      a->poszpre = (double*)dmalloc(8 * n);
      a->velrhoppre = (float4*)dmalloc(16 * n);
    }
  }
  poscell_ = (float4*)dmalloc(16 * n);
  press_ = (float*)dmalloc(4 * n);
  // Interaction items (launch_items): an item holds TB particles unless it ends a row
  // (<= 2 per row: fluid and bound) or reaches TMAXCELLS = 4 cells (<= 1 per 4 cells).
  // (slabs: up to three column ranges per row)
  items_ = (uint4*)dmalloc(16 * (n / 128 + 6 * size_t(G.ncy) * size_t(G.ncz) + size_t(nctmax_) / 2 + 2));
  arace_ = (float4*)dmalloc(16 * n);
  if (shift_) shiftpos_ = (float4*)dmalloc(16 * n);  // the interaction's shifting sums
  if (sps_) taunew_ = (float4*)dmalloc(32 * n);
  if (nnsph_) {
    viscoeta_ = (float*)dmalloc(4 * n);
    if (C.tvisco == SPH_VISCO_CONSTEQ) tau_ = (float4*)dmalloc(32 * n);
  }
  for (int i = 0; i < 2; i++) {
    sort_.keys[i] = (unsigned*)dmalloc(4 * n);
    sort_.vals[i] = (unsigned*)dmalloc(4 * n);
  }
  if (inc_ok_) {
    inc_.nb1 = inc_blocks_classify(n);
    const size_t ns = size_t(inc_.nb1) * INC_TILE_SIZE;  // tile-major mover slots
    inc_.skeys = (unsigned*)dmalloc(4 * n);
    inc_.newkey = (unsigned*)dmalloc(4 * n);
    inc_.cw = (unsigned*)dmalloc(4 * n);
    inc_.fidx = (unsigned*)dmalloc(4 * n);
    inc_.mkey = (unsigned*)dmalloc(4 * ns);
    inc_.mposnear = (unsigned*)dmalloc(4 * ns);
    inc_.mfar = (uint2*)dmalloc(8 * n);
    inc_.mposfar = (unsigned*)dmalloc(4 * n);
    inc_.tagg = (uint2*)dmalloc(8 * size_t(inc_.nb1));
    inc_.tpg = (unsigned*)dmalloc(4 * size_t(inc_.nb1));
    const size_t nsup = (size_t(inc_.nb1) + 63) / 64;
    inc_.tsup = (unsigned long long*)dmalloc(8 * TSUP_STRIDE * nsup);
    check_hip(hipMemset(inc_.tsup, 0, 8 * TSUP_STRIDE * nsup), "zero super tiles");
    inc_valid_ = false;  // new scratch: the next divide is a full one
  }
  if (slab()) {
    // new positions of the appended particles and reserved ghost slots (either divide)
    inc_.apppos = (unsigned*)dmalloc(4 * n);
  }
  sort_.ntiles = unsigned((n + RS_TILE - 1) / RS_TILE);
  sort_.hist = (unsigned*)dmalloc(4 * size_t(sort_.ntiles) * (1u << RS_MAXBITS));
  // slab pack tile counts: tilecnt[7][ntiles] (ghost L/R, migrant L/R, staying, face ghosts L/R; sph_slab.hip)
  packtiles_ = (unsigned*)dmalloc(PK_TILECNT_BYTES(n));
  cap_ = cap;
}

void SphGpuSingle::FreeParticles() {
  for (void* p : pallocs_) (void)hipFree(p);
  pallocs_.clear();
}

void SphGpuSingle::Free() {
  FreeParticles();
  for (void* p : allocs_) (void)hipFree(p);
  allocs_.clear();
  for (void* p : {sendgbuf_, sendmbuf_, (void*)recvg_, (void*)recvm_, (void*)nnface_, (void*)mdbcface_})
    if (p) (void)hipFree(p);
  nnface_ = nullptr;
  mdbcface_ = nullptr;
  sendgbuf_ = sendmbuf_ = nullptr;
  recvg_ = nullptr;
  recvm_ = nullptr;
  if (sc_host_) (void)hipHostFree(sc_host_);
  if (slabcnt_host_) (void)hipHostFree(slabcnt_host_);
  sc_host_ = nullptr;
  slabcnt_host_ = nullptr;
}

// Slab exchange buffers sized once from the case, from its densest cell slice along the
// slab axis: W face slices of ghosts per face (+50 %), a quarter of that in migrants.  The face messages then
// need no hipMalloc (and no stream synchronisation) mid-run; the grow paths of Exchange()
// stay as the fallback for a flow that piles particles into a face column or a re-partition
// that hands over many columns at once.
void SphGpuSingle::PresizeExchange(const SphParticlesHost& h) {
  const int ax = slabcfg_.axis;
  std::vector<unsigned> cnt(size_t(C.dom_cells[ax]) + 1, 0u);
  unsigned mx = 0;
  for (unsigned p = 0; p < h.n; p++) {
    const double x = (h.pos[3 * p + ax] - C.dom_posmin[ax]) / double(C.scell);
    if (!(x >= 0.0)) continue;
    const size_t cx = size_t(x);
    if (cx < cnt.size()) mx = std::max(mx, ++cnt[cx]);
  }
  const unsigned long long g = (unsigned long long)mx * unsigned(ghost_width(C));
  send_.gcap = slab_mincap_ ? 1 : g + g / 2 + 4096;
  send_.mcap = slab_mincap_ ? 1 : g / 4 + 1024;
  check_hip(hipMalloc(&sendgbuf_, 2 * sizeof(SlabGhost) * send_.gcap), "hipMalloc ghost send buffers");
  send_.gl = (SlabGhost*)sendgbuf_;
  send_.gr = send_.gl + send_.gcap;
  check_hip(hipMalloc(&sendmbuf_, 2 * sizeof(SlabRec) * send_.mcap), "hipMalloc migrant send buffers");
  send_.ml = (SlabRec*)sendmbuf_;
  send_.mr = send_.ml + send_.mcap;
  recvgcap_ = 2 * send_.gcap;
  recvmcap_ = 2 * send_.mcap;
  check_hip(hipMalloc((void**)&recvg_, sizeof(SlabGhost) * recvgcap_), "hipMalloc ghost receive buffer");
  check_hip(hipMalloc((void**)&recvm_, sizeof(SlabRec) * recvmcap_), "hipMalloc migrant receive buffer");
}

// Slab capacity growth (a slab gains particles as the fluid moves across it): new
// arrays, the live [0, np_live) of the current set copied over, the old set freed.
void SphGpuSingle::Grow(unsigned np_live, unsigned newcap) {
  check_hip(hipStreamSynchronize(stream), "grow: sync");
  const PartArrays old = cur_;
  std::vector<void*> oldallocs;
  oldallocs.swap(pallocs_);
  AllocParticles(newcap);
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (src && dst && bytes) check_hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream), "grow: copy");
  };
  const size_t n = np_live;
  cp(cur_.idp, old.idp, 4 * n);
  cp(cur_.code, old.code, 2 * n);
  cp(cur_.dcell, old.dcell, 4 * n);
  cp(cur_.posxy, old.posxy, 16 * n);
  cp(cur_.posz, old.posz, 8 * n);
  cp(cur_.velrhop, old.velrhop, 16 * n);
  cp(cur_.velrhopm1, old.velrhopm1, 16 * n);
  cp(cur_.posxypre, old.posxypre, 16 * n);
  cp(cur_.poszpre, old.poszpre, 8 * n);
  cp(cur_.velrhoppre, old.velrhoppre, 16 * n);
  cp(cur_.tau, old.tau, 32 * n);
  check_hip(hipStreamSynchronize(stream), "grow: copy");
  for (void* p : oldallocs) (void)hipFree(p);
}

void SphGpuSingle::Upload(const SphParticlesHost& h, const std::vector<unsigned>& sel, unsigned nown) {
  const unsigned n = unsigned(sel.size());
  std::vector<unsigned> dcell(n), idp(n);
  std::vector<typecode> code(n);
  std::vector<double2> pxy(n);
  std::vector<double> pz(n);
  std::vector<float4> vr(n);
  for (unsigned i = 0; i < n; i++) {
    const unsigned p = sel[i];
    idp[i] = h.idp[p];
    const double x = h.pos[3 * p], y = h.pos[3 * p + 1], z = h.pos[3 * p + 2];
    pxy[i] = make_double2(x, y);
    pz[i] = z;
    vr[i] = make_float4(h.vel[3 * p], h.vel[3 * p + 1], h.vel[3 * p + 2], h.rhop[p]);
    // LoadCodeParticles (JSph.cpp:1257): the codes of the case's MK blocks when given,
    // else one fixed and one fluid block.
    if (h.code) {
      code[i] = h.code[p];
      const typecode t = CodeType(code[i]);
      if (!CodeIsNormal(code[i]) || (i < npb0_) != (t < CODE_TYPE_FLOATING))
        throw SphError(SPH_ERR_ARG, "particle codes: boundary (fixed/moving) particles must be the first npb");
    } else {
      code[i] = (i < npb0_ ? typecode(0) : CODE_TYPE_FLUID);
    }
    // JSph::LoadMultiphaseData (JSph.cpp:3248-3263 of the v5.0 solver): a fluid particle's
    // density starts at its phase's rho; its code value must name a phase.
    if (nn_ && CodeIsFluid(code[i])) {
      const unsigned ph = code[i] & CODE_MASKVALUE;
      if (ph >= C.nphases) throw SphError(SPH_ERR_ARG, "Fluid particle without phase information...");
      vr[i].w = phase_rho_[ph];
    }
    // JSph::CheckRhopLimits (JSph.cpp:2021-2030).
    if (i >= npb0_ && (vr[i].w < C.rhopoutmin || C.rhopoutmax < vr[i].w))
      throw SphError(SPH_ERR_ARG, "Initial fluid density is out of limits.");
    // JSph::LoadDcellParticles (JSph.cpp:1690-1711).
    const double dx = x - C.dom_posmin[0], dy = y - C.dom_posmin[1], dz = z - C.dom_posmin[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0 && dx < C.map_realsize[0] && dy < C.map_realsize[1] && dz < C.map_realsize[2]))
      throw SphError(SPH_ERR_ARG, "Found new particles out.");
    dcell[i] = DcelCell(C.dom_cellcode, unsigned(dx / double(C.scell)), unsigned(dy / double(C.scell)),
                        unsigned(dz / double(C.scell)));
  }
  check_hip(hipMemcpy(cur_.idp, idp.data(), 4 * size_t(n), hipMemcpyHostToDevice), "upload idp");
  check_hip(hipMemcpy(cur_.code, code.data(), 2 * size_t(n), hipMemcpyHostToDevice), "upload code");
  check_hip(hipMemcpy(cur_.dcell, dcell.data(), 4 * size_t(n), hipMemcpyHostToDevice), "upload dcell");
  check_hip(hipMemcpy(cur_.posxy, pxy.data(), 16 * size_t(n), hipMemcpyHostToDevice), "upload posxy");
  check_hip(hipMemcpy(cur_.posz, pz.data(), 8 * size_t(n), hipMemcpyHostToDevice), "upload posz");
  check_hip(hipMemcpy(cur_.velrhop, vr.data(), 16 * size_t(n), hipMemcpyHostToDevice), "upload velrhop");
  // InitRunCpu: SpsTauc = 0 (JSphCpu.cpp:423)
  if (cur_.tau) check_hip(hipMemset(cur_.tau, 0, 32 * size_t(cap_)), "zero tau");
  DevScalars s;
  std::memset(&s, 0, sizeof(s));
  s.np = n;
  s.npb = npb0_;
  s.npbok = npb0_;
  s.nown = nown;
  s.symdtpre = C.dtini;  // InitRun (JSph.cpp:2090)
  check_hip(hipMemcpy(sc_, &s, sizeof(s), hipMemcpyHostToDevice), "upload scalars");
  verletstep_ = 0;
}

// JSph::LoadBoundNormals + ConfigBoundNormals (JSph.cpp:1265-1340): the case's normals
// (particle -> boundary limit) as float, doubled (particle -> ghost node), kept by idp.
void SphGpuSingle::UploadNormals(const SphCaseDef& cdef, const SphParticlesHost& h) {
  if (!h.boundnormal) throw SphError(SPH_ERR_ARG, "mDBC needs the boundary normals (<case>_Normals.nbi4)");
  // normals by idp: the boundary's [0, CaseNpb) and, when the floating bodies have normals
  // (UseNormalsFt, JSph.cpp:1301-1306: mDBC on them too), theirs up to the last one given
  unsigned nnor = cdef.npb, nftnor = 0;
  for (unsigned p = 0; p < h.n; p++) {
    const unsigned id = h.idp[p];
    if (id < cdef.npb) continue;
    const float x = h.boundnormal[3 * p], y = h.boundnormal[3 * p + 1], z = h.boundnormal[3 * p + 2];
    if (x != 0.f || y != 0.f || z != 0.f) {
      nnor = std::max(nnor, id + 1);
      nftnor++;
    }
  }
  ftnormals_ = nftnor > 0;
  nnormal_ = nnor;
  std::vector<float4> nor(std::max(nnor, 1u), make_float4(0.f, 0.f, 0.f, 0.f));
  unsigned nerr = 0;
  for (unsigned p = 0; p < h.n; p++) {
    const unsigned id = h.idp[p];
    if (id >= nnor) continue;
    const float x = h.boundnormal[3 * p], y = h.boundnormal[3 * p + 1], z = h.boundnormal[3 * p + 2];
    if (id < cdef.npb && x == 0.f && y == 0.f && z == 0.f) nerr++;
    nor[id] = make_float4(x * 2.f, y * 2.f, z * 2.f, 0.f);
  }
  if (nerr == cdef.npb && !ftnormals_) throw SphError(SPH_ERR_ARG, "No valid normal vectors for using mDBC.");
  check_hip(hipMalloc((void**)&normal_, sizeof(float4) * nor.size()), "hipMalloc normals");
  allocs_.push_back(normal_);
  check_hip(hipMemcpy(normal_, nor.data(), sizeof(float4) * nor.size(), hipMemcpyHostToDevice), "upload normals");
  if (slab()) {
    // face-column boundary (and floating) records: sized per interaction from the exchange's
    // face sizes (Interaction_Forces); the idp -> index map of those particles
    check_hip(hipMalloc((void**)&bidx_, sizeof(unsigned) * std::max(nnor, 1u)), "hipMalloc mDBC faces");
    allocs_.push_back(bidx_);
  }
  // boundary particles migrate between slabs, but a slab never holds more boundary
  // particles (owned + ghost) than the case has: CaseNpb bounds every slab's npbok, so
  // the list and sums keep their size when Grow() raises the particle capacity (and the
  // floating particles with normals bound the floating part of the list)
  const size_t nlist = size_t(slab() ? cdef.npb : npb0_) + nftnor + 1;
  check_hip(hipMalloc((void**)&mdbclist_, sizeof(unsigned) * nlist), "hipMalloc mDBC list");
  allocs_.push_back(mdbclist_);
  check_hip(hipMalloc(&mdbcsums_, MDBC_SUM_BYTES * nlist), "hipMalloc mDBC sums");
  allocs_.push_back(mdbcsums_);
}

// Restart: TimeStep and SymplecticDtPre of the loaded PART (JSph::InitRun, JSph.cpp:2094-2106).
void SphGpuSingle::SetTime(double time, double symdtpre) {
  if (motion_) throw SphError(SPH_ERR_STATE, "set the restart time before the motion (it is advanced to that time)");
  UploadFloatingTables();  // the floating tables' lookups start over (a restart's new JLinearValues)
  Sync();
  check_hip(hipMemcpy(&sc_->time, &time, sizeof(double), hipMemcpyHostToDevice), "set time");
  // the tables' walks start again from their first rows (a restarted reference run loads them anew)
  check_hip(hipMemset(&sc_->dtfix_pos, 0, 2 * sizeof(int)), "reset table rows");
  if (symdtpre > 0)
    check_hip(hipMemcpy(&sc_->symdtpre, &symdtpre, sizeof(double), hipMemcpyHostToDevice), "set SymplecticDtPre");
  if (K.visco_n) {  // ViscoTime at the restart time
    launch_visco_init(stream, sc_, K);
    Sync();
  }
}

// ---- timing -----------------------------------------------------------------------
void SphGpuSingle::SetTiming(bool on) {
  Sync();
  timing_ = on;
  for (int i = 0; i < 4; i++) { phase_ms_[i] = 0; phase_n_[i] = 0; }
}
// Phases timed (bit i: phase i of phase_ms_; all by default).  Every event pair is a marker
// in the stream, so a run timing only the interaction keeps the other launches back to back.
void SphGpuSingle::SetTimingPhases(unsigned mask) {
  Sync();
  timing_mask_ = mask & 0xfu;
}
void SphGpuSingle::TimedBegin(int phase) {
  if (!timing_ || !((timing_mask_ >> phase) & 1u)) return;
  hipEvent_t a;
  if (!evpool_.empty()) { a = evpool_.back(); evpool_.pop_back(); }
  else check_hip(hipEventCreate(&a), "hipEventCreate");
  check_hip(hipEventRecord(a, stream), "hipEventRecord");
  cur_a_ = a;
}
void SphGpuSingle::TimedEnd(int phase) {
  if (!timing_ || !((timing_mask_ >> phase) & 1u)) return;
  hipEvent_t b;
  if (!evpool_.empty()) { b = evpool_.back(); evpool_.pop_back(); }
  else check_hip(hipEventCreate(&b), "hipEventCreate");
  check_hip(hipEventRecord(b, stream), "hipEventRecord");
  pending_.push_back(Ev{cur_a_, b, phase});
}
void SphGpuSingle::Timing(double out_ms[4], uint64_t* launches) {
  Sync();
  for (auto& e : pending_) {
    float ms = 0;
    check_hip(hipEventElapsedTime(&ms, e.a, e.b), "hipEventElapsedTime");
    phase_ms_[e.phase] += ms;
    phase_n_[e.phase]++;
    evpool_.push_back(e.a);
    evpool_.push_back(e.b);
  }
  pending_.clear();
  for (int i = 0; i < 4; i++) out_ms[i] = phase_n_[i] ? phase_ms_[i] / double(phase_n_[i]) : 0.0;
  if (launches) *launches = phase_n_[0];
}

// ---- phases ------------------------------------------------------------------------
// Slab exchange before the divide: pack the migrants and count the ghosts per face box
// (device), swap the face messages (migrant count, ghost count per face box) with both
// neighbours device to device, then ONE host wait to size the transfers; move the migrants
// (96-112 B records) and append them.  The divide reserves the ghosts' slots; their
// records follow it (launch_ghost_pack -> post; GhostCollect), beside the interaction of the
// items that need no ghost when the step allows it (OverlapGhosts).
void SphGpuSingle::Exchange() {
  const bool withm1 = (step_algorithm_ == SPH_STEP_VERLET), withpre = havepre_;
  const bool hl = transport_->has_left(), hr = transport_->has_right();
  if (!hl && !hr) return;  // a slab alone holds the whole domain: no ghosts, no migrants
  SLAB_TRACE("exchange: pack");
  // (the first pack's count pass may have run in the update kernel, FuseUpdate)
  auto pack = [&] {
    launch_slab_pack(stream, cap_, sc_, cur_, G, K, C.dom_posmin, hl, hr, withm1, withpre, packtiles_, slabcnt_,
                     send_, normal_, nnormal_, &faces_, packcounted_);
    packcounted_ = false;
  };
  // the pack rewrites the migrant and face-message send buffers: the neighbours' copies of
  // the last messages (in-process slabs copy asynchronously) are done first
  transport_->wait_sends(stream);
  // turns measurement mode 2: the pack kernels are a turn of their own
  const bool pturn = in_run_ && transport_->turns();
  if (pturn) transport_->turn_wait(SlabTransport::TURN_PACK, stream, nullptr);
  pack();  // (its accumulated counts were zeroed by the last exchange's kernels: no memset launches)
  if (pturn) transport_->turn_done(SlabTransport::TURN_PACK, stream);
  const size_t mb = 4 * (size_t(FMSG_HDR) + faces_.nfb);
  transport_->exchange(faces_.msg[0], hl ? mb : 0, faces_.msg[1], hr ? mb : 0, faces_.msg[2], hl ? mb : 0,
                       faces_.msg[3], hr ? mb : 0, stream);
  // received headers -> the counts the host reads; the prefixes of all four messages' counts
  // (slots of the received ghosts, records of the sent ones) in the same launch
  launch_face_scan(stream, faces_, slabcnt_, hl, hr);
  check_hip(hipMemcpyAsync(slabcnt_host_, slabcnt_, sizeof(SlabCounts), hipMemcpyDeviceToHost, stream),
            "exchange: read counts");
  // The transfer sizes must be on the host before the transfers are posted: the one host
  // wait of a divide.  Spin on an event (a blocking synchronise wakes up tens of us later);
  // the GPU idles from the counts copy until the next launches arrive.
  if (!xev_) check_hip(hipEventCreateWithFlags(&xev_, hipEventDisableTiming), "hipEventCreate");
  check_hip(hipEventRecord(xev_, stream), "exchange: event");
  WaitEvent(xev_, "exchange: wait counts");
  const SlabCounts c = *slabcnt_host_;
  SLAB_TRACE("exchange: counts");
  {
    // the neighbour's ghosts of this slab: the ghosts sent now + the migrants it sent here
    // (it keeps them as ghosts); the neighbour derives the same sizes from its counts.  They
    // size the face re-sends after the divide (NN eta / tau, SPS tau, mDBC densities) exactly
    face_sl_ = hl ? unsigned(c.sendl[0] + c.recvl[1]) : 0u;
    face_sr_ = hr ? unsigned(c.sendr[0] + c.recvr[1]) : 0u;
    face_rl_ = hl ? unsigned(c.recvl[0] + c.sendl[1]) : 0u;
    face_rr_ = hr ? unsigned(c.recvr[0] + c.sendr[1]) : 0u;
  }
  const unsigned long long gneed = std::max(c.sendl[0], c.sendr[0]), mneed = std::max(c.sendl[1], c.sendr[1]);
  if (gneed > send_.gcap) {  // the ghost records are packed after the divide: room for them
    transport_->drain_sends();  // the neighbours' reads of the old buffer are done
    check_hip(hipStreamSynchronize(stream), "exchange: sync");
    if (sendgbuf_) check_hip(hipFree(sendgbuf_), "hipFree");
    send_.gcap = slab_mincap_ ? gneed : gneed + gneed / 2 + 4096;
    check_hip(hipMalloc(&sendgbuf_, 2 * sizeof(SlabGhost) * send_.gcap), "hipMalloc ghost send buffers");
    send_.gl = (SlabGhost*)sendgbuf_;
    send_.gr = send_.gl + send_.gcap;
  }
  if (mneed > send_.mcap) {  // migrant records past the capacity were not written: grow, pack again
    transport_->drain_sends();  // ... and the face messages are rewritten: their reads are done
    check_hip(hipStreamSynchronize(stream), "exchange: sync");
    if (sendmbuf_) check_hip(hipFree(sendmbuf_), "hipFree");
    send_.mcap = slab_mincap_ ? mneed : mneed + mneed / 2 + 1024;
    check_hip(hipMalloc(&sendmbuf_, 2 * sizeof(SlabRec) * send_.mcap), "hipMalloc migrant send buffers");
    send_.ml = (SlabRec*)sendmbuf_;
    send_.mr = send_.ml + send_.mcap;
    // the counts accumulate again: start them over (the face messages already sent are unchanged)
    check_hip(hipMemsetAsync(&slabcnt_->nkeep, 0, sizeof(unsigned) * 3, stream), "exchange: reset nkeep, ghosts");
    for (int k = 0; k < 2; k++)
      check_hip(hipMemsetAsync(faces_.msg[k] + FMSG_HDR, 0, 4 * size_t(faces_.nfb), stream), "exchange: reset faces");
    pack();
  }
  const unsigned long long rgl = hl ? c.recvl[0] : 0, rgr = hr ? c.recvr[0] : 0;
  const unsigned long long rml = hl ? c.recvl[1] : 0, rmr = hr ? c.recvr[1] : 0;
  if (rgl + rgr > recvgcap_) {
    check_hip(hipStreamSynchronize(stream), "exchange: sync");
    if (recvg_) check_hip(hipFree(recvg_), "hipFree");
    recvgcap_ = slab_mincap_ ? rgl + rgr : rgl + rgr + (rgl + rgr) / 2 + 4096;
    check_hip(hipMalloc((void**)&recvg_, sizeof(SlabGhost) * recvgcap_), "hipMalloc ghost receive buffer");
  }
  if (rml + rmr > recvmcap_) {
    check_hip(hipStreamSynchronize(stream), "exchange: sync");
    if (recvm_) check_hip(hipFree(recvm_), "hipFree");
    recvmcap_ = slab_mincap_ ? rml + rmr : rml + rmr + (rml + rmr) / 2 + 1024;
    check_hip(hipMalloc((void**)&recvm_, sizeof(SlabRec) * recvmcap_), "hipMalloc migrant receive buffer");
  }
  const unsigned long long nin = rgl + rgr + rml + rmr;  // the ghosts' slots are reserved by the divide
  if (c.np + nin > cap_) {
    const unsigned long long want = (c.np + nin) + (slab_mincap_ ? 16 : (c.np + nin) / 2);
    if (want >= (1ull << 31)) throw SphError(SPH_ERR_NOMEM, "slab particle capacity overflow");
    Grow(c.np, unsigned(want));
  }
  // k_unpack zeroes the face counts of the messages just sent: the neighbours have read them
  transport_->wait_sends(stream);
  // the migrants of both faces (two concurrent streams over the two xGMI links)
  transport_->exchange(send_.ml, sizeof(SlabRec) * c.sendl[1], send_.mr, sizeof(SlabRec) * c.sendr[1], recvm_,
                       sizeof(SlabRec) * rml, recvm_ + rml, sizeof(SlabRec) * rmr, stream);
  launch_slab_unpack(stream, sc_, recvm_, unsigned(rml + rmr), recvg_, 0u, c.np, cur_, K, C.dom_posmin, withm1,
                     withpre, slabcnt_, normal_, nnormal_, &faces_, hl, hr);
  SLAB_TRACE("exchange: done");
  xg_sl_ = hl ? c.sendl[0] : 0;
  xg_sr_ = hr ? c.sendr[0] : 0;
  xg_rl_ = rgl;
  xg_rr_ = rgr;
  xg_nm_ = unsigned(rml + rmr);
  xg_np_ = unsigned(c.np + rml + rmr);
  inc_.nold = unsigned(c.np);  // the incremental divide places the appended [np, np + nm) apart
  inc_.napp = xg_nm_;
}

// The ghost records of the last divide: packed from the sorted face columns and posted by
// the divide (launch_ghost_pack -> SlabTransport::post), received from both neighbours on
// stream s, written into the slots the divide reserved.
void SphGpuSingle::GhostCollect(hipStream_t s) {
  SLAB_TRACE("ghosts: collect");
  transport_->collect(recvg_, sizeof(SlabGhost) * xg_rl_, recvg_ + xg_rl_, sizeof(SlabGhost) * xg_rr_, s);
  launch_ghost_scatter(s, sc_, recvg_, unsigned(xg_rl_ + xg_rr_), inc_.apppos + xg_nm_, cur_, K, C.dom_posmin,
                       poscell_, press_, G, inc_ok_ ? inc_.skeys : nullptr, nn_ ? phaseeos_ : nullptr);
}

// The ghosts of the last divide still in flight (end of a run): in place on the solver stream.
void SphGpuSingle::GhostFinish() {
  if (!ghost_pending_) return;
  if (ghost_split_) {  // packed and posted on the exchange stream
    GhostCollect(xstream_);
    check_hip(hipEventRecord(ev_ghost_, xstream_), "ghosts: event");
    check_hip(hipStreamWaitEvent(stream, ev_ghost_, 0), "ghosts: join");
  } else {
    GhostCollect(stream);
  }
  ghost_pending_ = false;
}

// The interaction of the items that reach no ghost column can run while the ghosts are in
// flight when nothing between the divide and it reads a ghost: the headline tiled kernel
// inside Run(), without mDBC (its correction reads ghosts first), bodies (their particle map
// is built after the divide) or the NN / Laminar+SPS / shifting kernels (face exchanges of
// per-particle values first).
bool SphGpuSingle::OverlapEligible() const {
  return slab() && in_run_ && tiled_ && !nn_ && !ext_ && !normal_ && !nftp_ && !nmotobj_ &&
         (transport_->has_left() || transport_->has_right());
}
bool SphGpuSingle::OverlapGhosts() const { return overlap_ && OverlapEligible(); }

// The one host wait of a slab divide: spin on the event (a blocking synchronise wakes up
// tens of us later) with a deadline, polling the transport's asynchronous error state.  A
// dead or failed peer ends this rank with SPH_ERR_COMM instead of a hang (the transport is
// aborted first, so the other ranks' pending transfers fail or time out too).
void SphGpuSingle::WaitEvent(hipEvent_t ev, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; spin++) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) check_hip(q, what);
    if ((spin & 1023u) == 1023u) {
      try {
        transport_->check_async();
      } catch (...) {
        transport_->abort();
        throw;
      }
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (sec > comm_timeout_s_) {
        transport_->abort();
        throw SphError(SPH_ERR_COMM, std::string(what) + ": no progress for " + std::to_string(int(sec)) +
                                         " s (a neighbour slab is gone or stalled)");
      }
    }
  }
}

// Periodic re-balancing of the x-slabs ("re-balanced every K steps"): the
// owned particles per global column (fluid + bound_weight x bound, the weights of
// sph_slab_partition) are summed over the ranks, every rank derives the same new column
// bounds from them, and the next exchange hands over whole columns as migrants.  Each
// bound stays strictly inside the two slabs it separates, so a particle moves at most
// one rank, and the copies a rank keeps of its outgoing migrants in its new ghost column
// (the usual pack rule) give the neighbours their ghost columns during the hand-over.
// Called between an update and the divide (all ranks, same step).
void SphGpuSingle::Repartition() {
  // (FuseUpdate leaves the count pass to the exchange at a re-partitioning divide)
  if (packcounted_) throw SphError(SPH_ERR_STATE, "internal: the update counted the pack of a re-partitioning divide");
  const int ncxg = int(C.dom_cells[slabcfg_.axis]), nr = slabcfg_.nranks;
  launch_column_counts(stream, cap_, sc_, cur_, G, K, ncxg, colcnt_);
  std::vector<float> bnd(size_t(nr) + 1, 0.f);
  bnd[size_t(slabcfg_.rank)] = float(slabcfg_.c0);  // each rank contributes its own bound
  if (slabcfg_.rank == nr - 1) bnd[size_t(nr)] = float(slabcfg_.c1);
  check_hip(hipMemcpyAsync(colcnt_ + 2 * ncxg, bnd.data(), 4 * bnd.size(), hipMemcpyHostToDevice, stream),
            "repartition: bounds");
  transport_->allreduce_sum_f32(colcnt_, 2 * ncxg + nr + 1, stream);
  std::vector<float> h(2 * size_t(ncxg) + size_t(nr) + 1);
  check_hip(hipMemcpyAsync(h.data(), colcnt_, 4 * h.size(), hipMemcpyDeviceToHost, stream), "repartition: read");
  if (!xev_) check_hip(hipEventCreateWithFlags(&xev_, hipEventDisableTiming), "hipEventCreate");
  check_hip(hipEventRecord(xev_, stream), "repartition: event");
  WaitEvent(xev_, "repartition: column counts");
  std::vector<int> old(size_t(nr) + 1);
  for (int r = 0; r <= nr; r++) old[size_t(r)] = int(h[2 * size_t(ncxg) + size_t(r)]);
  std::vector<double> w(static_cast<size_t>(ncxg));
  double total = 0;
  for (int c = 0; c < ncxg; c++) {
    w[size_t(c)] = double(h[size_t(c)]) + repart_bw_ * double(h[size_t(ncxg + c)]);
    total += w[size_t(c)];
  }
  std::vector<double> pre(size_t(ncxg) + 1, 0.0);
  for (int c = 0; c < ncxg; c++) pre[size_t(c) + 1] = pre[size_t(c)] + w[size_t(c)];
  double maxload = 0;
  for (int r = 0; r < nr; r++) maxload = std::max(maxload, pre[size_t(old[size_t(r) + 1])] - pre[size_t(old[size_t(r)])]);
  repart_last_imbalance_ = total > 0 ? maxload / (total / nr) : 1.0;
  if (!(repart_last_imbalance_ > 1.0 + repart_tol_)) return;
  std::vector<int> nb(old);
  const int W = min_slab_width(C);  // every slab keeps its two disjoint face column sets
  partition_from_prefix(pre, nr, nb.data(), W);
  for (int r = 1; r < nr; r++) {  // inside the two slabs it separates, and increasing
    nb[size_t(r)] = std::min(std::max(nb[size_t(r)], old[size_t(r) - 1] + W), old[size_t(r) + 1] - W);
    nb[size_t(r)] = std::max(nb[size_t(r)], nb[size_t(r) - 1] + W);
  }
  bool changed = false;
  for (int r = 1; r < nr; r++) {
    if (nb[size_t(r)] + W > nb[size_t(r) + 1]) return;  // the clamps left no valid split: keep the old one
    changed |= nb[size_t(r)] != old[size_t(r)];
  }
  if (!changed) return;
  slabcfg_.c0 = nb[size_t(slabcfg_.rank)];
  slabcfg_.c1 = nb[size_t(slabcfg_.rank) + 1];
  G = make_grid(C, &slabcfg_);
  keybits_ = bits_for(G.boxdiscard, 1);
  inc_valid_ = false;  // the box keys changed: the next divide sorts from scratch
  repart_count_++;
}

void SphGpuSingle::ShareDeviceCheck() {
  if (!slab() || transport_->nranks < 2) return;
  char bus[64] = {0};
  check_hip(hipDeviceGetPCIBusId(bus, int(sizeof(bus)) - 1, device), "hipDeviceGetPCIBusId");
  unsigned h = 2166136261u;  // FNV-1a of the bus id, kept below 2^23: exact as a float sum term
  for (const char* c = bus; *c; c++) h = (h ^ unsigned((unsigned char)*c)) * 16777619u;
  const float mine = float((h & 0x7fffffu) + 1u);
  const int nr = transport_->nranks;
  std::vector<float> v(size_t(nr), 0.f);
  v[size_t(slabcfg_.rank)] = mine;
  float* d = nullptr;
  check_hip(hipMalloc((void**)&d, sizeof(float) * size_t(nr)), "hipMalloc device check");
  check_hip(hipMemcpy(d, v.data(), sizeof(float) * v.size(), hipMemcpyHostToDevice), "device check");
  transport_->allreduce_sum_f32(d, nr, stream);
  check_hip(hipMemcpyAsync(v.data(), d, sizeof(float) * v.size(), hipMemcpyDeviceToHost, stream), "device check");
  check_hip(hipStreamSynchronize(stream), "device check");
  (void)hipFree(d);
  for (int r = 0; r < nr; r++)
    if (r != slabcfg_.rank && v[size_t(r)] == mine) MarkSharedDevice();
}

void SphGpuSingle::SetRepartition(unsigned every, double bound_weight, double tolerance) {
  if (!slab()) throw SphError(SPH_ERR_STATE, "re-partitioning applies to slab solvers only");
  if (!(bound_weight >= 0) || !(tolerance >= 0)) throw SphError(SPH_ERR_ARG, "invalid re-partition weights");
  repart_every_ = every;
  repart_bw_ = bound_weight;
  repart_tol_ = tolerance;
}

void SphGpuSingle::RunCellDivide() {
  // turns measurement mode: the divide's kernels after the exchange are a turn of their own
  // and the timed divide phase is those kernels alone (the exchange waits for neighbours)
  const bool turn = slab() && exchange_armed_ && in_run_ && transport_->turns();
  if (!turn) TimedBegin(2);
  if (slab() && exchange_armed_ && repart_every_ && (stepsdone_ % repart_every_) == 0 && transport_->nranks > 1 &&
      !havepre_)
    Repartition();
  // the exchange of this divide: ghosts in reserved slots, their records after the sort
  const bool ghosts = slab() && exchange_armed_ && (transport_->has_left() || transport_->has_right());
  if (slab() && exchange_armed_) Exchange();
  if (turn) {
    transport_->turn_wait(SlabTransport::TURN_DIVIDE, stream, nullptr);
    TimedBegin(2);
  }
  const unsigned ngl = ghosts ? unsigned(xg_rl_) : 0u, ngr = ghosts ? unsigned(xg_rr_) : 0u;
  const bool withm1 = (step_algorithm_ == SPH_STEP_VERLET);
  // Items (each build also zeroes its queues).  With the overlap a slab cuts its rows where
  // the stencil (scelldiv columns) stops reaching a ghost column: the interior list runs
  // while the ghost records are in flight, the face list (items of <= scelldiv columns) after
  // them.  With the ghosts in place the rows are not cut (full items); SPH_SLAB_CUT=1 cuts
  // them there too, which makes the two modes bitwise the same (a test hook).
  const bool overlap = ghosts && OverlapGhosts();
  ghost_split_ = false;
  ItemBuild ib;
  if (tiled_) {
    const int S = int(C.scelldiv), hl = slab() && transport_->has_left(), hr = slab() && transport_->has_right();
    // the owned cells along the slab axis whose stencil (scelldiv cells) reaches no ghost
    int ib0 = G.sown0 + (hl ? S : 0), ie0 = G.sown1 - (hr ? S : 0);
    if (ib0 >= ie0) ib0 = ie0 = G.sown0;  // a narrow slab: every item reaches a ghost cell
    const bool inc = inc_ok_ && inc_valid_ && G.ncx >= 3 && (G.ncy >= 3 || G.ncy == 1);
    const unsigned* bcnew = inc ? begincell_alt_ : begincell_;  // the begincell this divide writes
    if (overlap) {  // the interior list (qctr_), then the face list (qctrf_) after it
      const int xr[6] = {ib0, ie0, G.sown0, ib0, ie0, G.sown1};
      ib = make_item_build(bcnew, G, rowtmp_, items_, qctr_, C.scelldiv, xr, qctrf_, rowitems_, ricap_);
      ghost_split_ = true;
    } else if (cut_items_) {  // the overlap's items in one list (SPH_SLAB_CUT test hook)
      const int xa[6] = {G.sown0, ib0, ib0, ie0, ie0, G.sown1};
      ib = make_item_build(bcnew, G, rowtmp_, items_, qctr_, C.scelldiv, xa, nullptr, rowitems_, ricap_);
    } else {
      // ghosts in place: the rows' items over all owned columns, as in one domain (a row cut
      // at the face columns leaves items of one cell there, ~1/3 of the block's lanes)
      ib = make_item_build(bcnew, G, rowtmp_, items_, qctr_, C.scelldiv, nullptr, nullptr, rowitems_, ricap_);
    }
  }
  if (inc_ok_ && inc_valid_ && G.ncx >= 3 && (G.ncy >= 3 || G.ncy == 1)) {
    // the previous order merged with the particles whose box changed and, on a slab, the
    // particles the exchange appended and the ghosts' slots (sph_divide.hip); the item
    // count runs in the push launch, the item write right after it
    inc_.nb2 = inc_blocks_boxes(G.nctt);
    launch_divide_inc(stream, cap_, sc_, cur_, alt_, withm1, havepre_, K, C.dom_posmin, poscell_, press_, G, begincell_,
                      begincell_alt_, inc_, sort_, keybits_, nn_ ? phaseeos_ : nullptr, ghosts ? &faces_ : nullptr, ngl,
                      ngr, tiled_ ? &ib : nullptr, classified_);
    std::swap(begincell_, begincell_alt_);
  } else {
    // the ghosts' slots sort as entries [np, np + ngl + ngr) after the particles
    launch_presort(stream, cap_, sc_, cur_.dcell, cur_.code, G, C.dom_cellcode, sort_.keys[0], sort_.vals[0], ngl + ngr);
    if (ngl + ngr)
      launch_ghost_keys(stream, faces_, G, ngl, ngr, sort_.keys[0] + xg_np_, sort_.vals[0] + xg_np_, xg_np_);
    const int res = launch_radix_sort(stream, cap_, sc_, sort_, keybits_);
    launch_begincell(stream, cap_, sc_, sort_.keys[res], G, begincell_);
    launch_gather(stream, cap_, sc_, sort_.vals[res], cur_, alt_, withm1, havepre_, K, C.dom_posmin, poscell_, press_,
                  G.offx(), G.offy(), nn_ ? phaseeos_ : nullptr, ghosts ? xg_np_ : ~0u, xg_np_ - xg_nm_, inc_.apppos);
    if (inc_ok_)
      check_hip(hipMemcpyAsync(inc_.skeys, sort_.keys[res], 4 * size_t(cap_), hipMemcpyDeviceToDevice, stream),
                "keep sorted keys");
    if (tiled_) launch_items(stream, ib);
  }
  inc_valid_ = inc_ok_;
  classified_ = false;
  inc_.napp = 0;
  inc_.nvl = inc_.nvr = 0;
  std::swap(cur_, alt_);
  qpass_ = 0;
  if (ghosts) {
    // this slab's ghost records for the neighbours, from its sorted face columns, posted at
    // once.  With the overlap they are packed on the exchange stream, so the interaction's
    // interior items follow the divide directly on the solver stream; the transfer and the
    // scatter follow in the interaction (also, in the turns measurement mode, the in-place
    // transfer: it is then part of the slab's own interaction turn).
    hipStream_t gs = stream;
    if (overlap) {
      ExchangeStream();
      check_hip(hipEventRecord(ev_div_, stream), "divide: event");
      check_hip(hipStreamWaitEvent(xstream_, ev_div_, 0), "ghosts: wait divide");
      gs = xstream_;
    }
    launch_ghost_pack(gs, sc_, faces_, G, begincell_, cur_, poscell_, send_, unsigned(xg_sl_), unsigned(xg_sr_));
    transport_->post(send_.gl, sizeof(SlabGhost) * xg_sl_, send_.gr, sizeof(SlabGhost) * xg_sr_, gs);
    if (overlap || (transport_->turns() && OverlapEligible())) {
      ghost_pending_ = true;
    } else {
      GhostCollect(stream);
    }
  }
  if (nftp_) launch_ft_ridp(stream, cap_, sc_, cur_, casenpb_, nftp_, ftridp_, K, G);
  TimedEnd(2);
  if (turn) transport_->turn_done(SlabTransport::TURN_DIVIDE, stream);
}

unsigned SphGpuSingle::NextQueueCopy() {
  const unsigned c = qpass_ % QCTR_COPIES;
  if (++qpass_ > unsigned(QCTR_COPIES)) {  // beyond the copies the item build zeroed
    check_hip(hipMemsetAsync(qctr_ + c * QCTR_WORDS, 0, QCTR_QUEUE_BYTES, stream), "zero work counters");
    if (ghost_split_)
      check_hip(hipMemsetAsync(qctrf_ + c * QCTR_WORDS, 0, QCTR_QUEUE_BYTES, stream), "zero work counters");
  }
  return c * QCTR_WORDS;
}

void SphGpuSingle::Interaction_Forces(int interstep) {
  bool t0 = false;  // the interaction's timed interval has begun
  auto begin0 = [&] {
    if (!t0) TimedBegin(0);
    t0 = true;
  };
  // turns measurement mode (SPH_SLAB_TURNS, in-process slabs): this slab's interaction starts
  // on the GPU after the previous slab's has ended
  const bool turn = slab() && transport_->turns();
  if (turn) {
    ExchangeStream();
    transport_->turn_wait(SlabTransport::TURN_INTERACTION, stream, xstream_);
  }
  if (ghost_pending_ && !ghost_split_) {  // deferred in-place ghosts: the transfer is timed with it
    begin0();
    GhostCollect(stream);
    ghost_pending_ = false;
  }
  // mDBC boundary correction first, except in the Symplectic corrector unless MDBCCorrector
  // (JSphCpuSingle.cpp:525); with floating normals the floating particles too (JSphCpu.cpp:1199).
  if (normal_ && (mdbc_corrector_ || interstep != 3)) {
    TimedBegin(3);
    launch_mdbc(stream, slab() ? cap_ : npb0_, sc_, cur_, press_, normal_, begincell_, G, K, C.dom_posmin, C.mdbc_threshold,
                mdbclist_ + 1, mdbclist_, mdbcsums_, ftnormals_ ? ftridp_ : nullptr, ftnormals_ ? nftp_ : 0u);
    if (slab() && (transport_->has_left() || transport_->has_right())) {
      // records per side = the face's particles at the last exchange + the count slot: both
      // sides of a face derive the same size, and no face record can be dropped
      const bool hl = transport_->has_left(), hr = transport_->has_right();
      const unsigned nsl = hl ? face_sl_ + 1u : 0u, nsr = hr ? face_sr_ + 1u : 0u;
      const unsigned nrl = hl ? face_rl_ + 1u : 0u, nrr = hr ? face_rr_ + 1u : 0u;
      const unsigned long long need = 0ull + nsl + nsr + nrl + nrr;
      if (need > mdbcfacecap_) {
        transport_->drain_sends();
        check_hip(hipStreamSynchronize(stream), "mDBC faces: sync");
        if (mdbcface_) check_hip(hipFree(mdbcface_), "hipFree");
        mdbcface_ = nullptr;
        const unsigned long long want = slab_mincap_ ? need : need + need / 2 + 1024;
        check_hip(hipMalloc((void**)&mdbcface_, sizeof(MdbcFaceRec) * want), "hipMalloc mDBC faces");
        mdbcfacecap_ = want;
      }
      MdbcFaceRec *sl = mdbcface_, *sr = sl + nsl, *rl = sr + nsr, *rr = rl + nrl;
      // the neighbours' copies of the last message out of these buffers are done before the
      // pack rewrites them (in-process slabs copy asynchronously); an end slab's grid keeps
      // ghost columns on its outer side too: no records for that side
      transport_->wait_sends(stream);
      launch_mdbc_face_pack(stream, cap_, sc_, cur_, press_, K, G, hl ? sl : nullptr, hr ? sr : nullptr, nsl, nsr, bidx_,
                            nnormal_, ftnormals_);
      transport_->exchange(sl, sizeof(MdbcFaceRec) * nsl, sr, sizeof(MdbcFaceRec) * nsr, rl, sizeof(MdbcFaceRec) * nrl,
                           rr, sizeof(MdbcFaceRec) * nrr, stream);
      launch_mdbc_face_apply(stream, sc_, hl ? rl : nullptr, hr ? rr : nullptr, nrl, nrr, bidx_, nnormal_, cur_.idp,
                             cur_.velrhop, press_);
    }
    TimedEnd(3);
  }
  const unsigned qc = tiled_ ? NextQueueCopy() : 0u;
  unsigned *qa = qctr_ + qc, *qf = qctrf_ ? qctrf_ + qc : nullptr;
  if (nn_) {
    // NN multiphase (sph_nn.hip); the shifting sums only where they are applied: the
    // corrector (the predictor's RunShifting result is never used, shift=false in
    // ComputeSymplecticPre) and Verlet
    begin0();
    launch_nn_tiled(stream, nblocks_tiled_, sc_, items_, qa, poscell_, cur_.velrhop, press_, cur_.code, begincell_,
                    G, K, phasek_, arace_, shiftpos_, shift_ && interstep != 2, viscoeta_, tau_, ftmassp_);
    if (nnsph_) {
      // SPH velocity gradients: the viscous force is a second pass over the neighbours,
      // reading their effective viscosities / stress tensors (JSphCpu_NN_SPH.cpp:671-696)
      if (slab() && C.tvisco != SPH_VISCO_ARTIFICIAL && (transport_->has_left() || transport_->has_right()))
        NNFaceExchange();
      launch_nn_visc(stream, nblocks_tiled_, sc_, items_, qctr_ + NextQueueCopy(), poscell_, cur_.velrhop, cur_.code, viscoeta_, tau_,
                     begincell_, G, K, phasek_, arace_, ftmassp_);
    }
  } else if (ext_) {
    // Laminar+SPS and/or shifting (sph_ext.hip).  Slabs with SPS: the ghosts' tau (the
    // owners' from the last interaction) first
    if (sps_ && slab() && (transport_->has_left() || transport_->has_right())) NNFaceExchange();
    begin0();
    launch_fluid_ext(stream, nblocks_tiled_, sc_, items_, qa, poscell_, cur_.velrhop, press_, cur_.code, ftmassp_,
                     cur_.tau, begincell_, G, K, arace_, shiftpos_, taunew_, interstep != 2);
    if (sps_) std::swap(cur_.tau, taunew_);
  } else if (tiled_) {
    // The tiled kernel writes the arace of every owned particle (skipped boundary items
    // get ar = 0); its work queues are the copy NextQueueCopy picked.
    begin0();  // the timed interval is the interaction kernel alone (rocprof's per-kernel average)
    if (ghost_pending_) {
      // Slab: the interior items now, the ghost records in flight on the exchange stream
      // (packed and posted there after the divide); there the face items follow their
      // arrival.  The interior kernel leaves a few block slots free so that the transfer and
      // scatter kernels start at once.
      launch_fluid_tiled(stream, nblocks_tiled_, sc_, items_, qa, poscell_, cur_.velrhop, press_, begincell_, G, K,
                         arace_, cur_.code, ftmassp_, 64);
      GhostCollect(xstream_);
      launch_fluid_tiled(xstream_, nblocks_tiled_, sc_, items_, qf, poscell_, cur_.velrhop, press_, begincell_, G,
                         K, arace_, cur_.code, ftmassp_);
      check_hip(hipEventRecord(ev_ghost_, xstream_), "ghosts: event");
      check_hip(hipStreamWaitEvent(stream, ev_ghost_, 0), "ghosts: join");
      ghost_pending_ = false;
    } else {
      launch_fluid_tiled(stream, nblocks_tiled_, sc_, items_, qa, poscell_, cur_.velrhop, press_, begincell_, G, K,
                         arace_, cur_.code, ftmassp_);
      if (ghost_split_)  // the ghosts are in: the face items right after
        launch_fluid_tiled(stream, nblocks_tiled_, sc_, items_, qf, poscell_, cur_.velrhop, press_, begincell_,
                           G, K, arace_, cur_.code, ftmassp_);
    }
  } else {
    begin0();
    launch_interaction(stream, cap_, sc_, poscell_, cur_.velrhop, press_, begincell_, G, K, arace_, cur_.code,
                       ftmassp_);
  }
  TimedEnd(0);
  if (turn && fold_turn_ >= 0) {  // the next DtVariable's fold, inside this slab's turn
    launch_fold_maxima(stream, sc_, folded_, fold_turn_ != 0);
    folded_ready_ = true;
  }
  fold_turn_ = -1;
  if (turn) transport_->turn_done(SlabTransport::TURN_INTERACTION, stream);
}

// The exchange stream and its events (created on first use).
void SphGpuSingle::ExchangeStream() {
  if (!xstream_) check_hip(hipStreamCreateWithFlags(&xstream_, hipStreamNonBlocking), "hipStreamCreate");
  if (!ev_div_) check_hip(hipEventCreateWithFlags(&ev_div_, hipEventDisableTiming), "hipEventCreate");
  if (!ev_ghost_) check_hip(hipEventCreateWithFlags(&ev_ghost_, hipEventDisableTiming), "hipEventCreate");
}

// Slabs, SPH velocity gradients: the owned face-column fluid particles' eta (and tau) to the
// neighbours, written into their ghost copies by idp before the second pass.  Fixed-size
// records (count in slot 0) sized from the last exchange, so no host wait.
void SphGpuSingle::NNFaceExchange() {
  const bool hl = transport_->has_left(), hr = transport_->has_right();
  const unsigned long long nsl = hl ? face_sl_ + 1ull : 0, nsr = hr ? face_sr_ + 1ull : 0;
  const unsigned long long nrl = hl ? face_rl_ + 1ull : 0, nrr = hr ? face_rr_ + 1ull : 0;
  const unsigned long long need = nsl + nsr + nrl + nrr;
  if (need > nnfacecap_) {
    transport_->drain_sends();
    check_hip(hipStreamSynchronize(stream), "nn faces: sync");
    if (nnface_) check_hip(hipFree(nnface_), "hipFree");
    nnfacecap_ = slab_mincap_ ? need : need + need / 2 + 1024;
    check_hip(hipMalloc((void**)&nnface_, sizeof(NNFaceRec) * nnfacecap_), "hipMalloc NN face records");
  }
  NNFaceRec *sl = nnface_, *sr = sl + nsl, *rl = sr + nsr, *rr = rl + nrl;
  // NN: the first pass's eta (+ ConstEq tau); single phase Laminar+SPS: the particles' SPS tau
  float* veta = sps_ ? nullptr : viscoeta_;
  float4* tau = sps_ ? cur_.tau : tau_;
  transport_->wait_sends(stream);  // the neighbours copied the last message out of these buffers
  launch_nn_face_pack(stream, cap_, sc_, cur_, K, G, veta, tau, hl ? sl : nullptr, hr ? sr : nullptr, unsigned(nsl),
                      unsigned(nsr), idxmap_, casenp_);
  transport_->exchange(sl, sizeof(NNFaceRec) * nsl, sr, sizeof(NNFaceRec) * nsr, rl, sizeof(NNFaceRec) * nrl, rr,
                       sizeof(NNFaceRec) * nrr, stream);
  launch_nn_face_apply(stream, sc_, hl ? rl : nullptr, hr ? rr : nullptr, unsigned(nrl), unsigned(nrr), idxmap_,
                       casenp_, cur_.idp, veta, tau, tau != nullptr);
}

void SphGpuSingle::DtVariable(int mode) {
  if (slab() && transport_->nranks > 1) {  // one rank: its own maxima are the domain's
    SLAB_TRACE("dt allreduce");
    // The three maxima span the whole domain: fold locally, max over all slabs.
    if (!folded_ready_) launch_fold_maxima(stream, sc_, folded_, mode != DT_PEEK);
    folded_ready_ = false;
    transport_->allreduce_max_u32(folded_, 5, stream);  // 4 maxima + the fatal error flags
    launch_dt(stream, sc_, K, C.cflnumber, C.dtmin, C.cs0, mode, dttrace_, tracecap_, folded_);
  } else {
    launch_dt(stream, sc_, K, C.cflnumber, C.dtmin, C.cs0, mode, dttrace_, tracecap_);
  }
}

// Turns measurement mode 2 (SPH_SLAB_TURNS=2, in-process slabs): the update kernels are a
// turn of their own.
void SphGpuSingle::UpdateTurn(bool begin) {
  if (!(slab() && in_run_ && transport_->turns())) return;
  if (begin) transport_->turn_wait(SlabTransport::TURN_UPDATE, stream, nullptr);
  else transport_->turn_done(SlabTransport::TURN_UPDATE, stream);
}

// The next divide's classification (sph_incdiv.hpp) and, on a slab with neighbours, its
// exchange's count pass (sph_slabpack.hpp) in the update kernel: the next divide is
// incremental and nothing moves a particle between the update and the divide (no floating
// bodies, no moving boundaries; no re-partition at that divide, which changes the slab's
// columns and hence every key).  pre_at_divide: whether the Symplectic pre-state is held at
// the divide (the re-partition's condition).  SPH_CLS_SPLIT=1 (test hook) keeps the separate
// k_inc_classify and k_pack_count launches.
SphGpuSingle::UpdateFuse SphGpuSingle::FuseUpdate(bool pre_at_divide) {
  static const bool split = [] {
    const bool on = std::getenv("SPH_CLS_SPLIT") && std::atoi(std::getenv("SPH_CLS_SPLIT"));
    if (on) test_hook_notice("SPH_CLS_SPLIT");
    return on;
  }();
  classified_ = packcounted_ = false;
  UpdateFuse f;
  const bool repart = slab() && exchange_armed_ && repart_every_ && (stepsdone_ % repart_every_) == 0 &&
                      transport_->nranks > 1 && !pre_at_divide;
  if (split || repart || !inc_ok_ || !inc_valid_ || !(G.ncx >= 3 && (G.ncy >= 3 || G.ncy == 1)) || nftbodies_ ||
      nmotobj_ || inc_.napp != 0)
    return f;
  classified_ = true;
  f.cls = &inc_;
  const bool hl = slab() && transport_->has_left(), hr = slab() && transport_->has_right();
  if (slab() && exchange_armed_ && (hl || hr)) {
    pack_args_ = make_pack_args(cap_, cur_, G, K, C.dom_posmin, hl, hr, step_algorithm_ == SPH_STEP_VERLET,
                                pre_at_divide, packtiles_, slabcnt_, send_, normal_, nnormal_, &faces_);
    packcounted_ = true;
    f.pk = &pack_args_;
  }
  return f;
}

void SphGpuSingle::ComputeVerlet() {
  UpdateTurn(true);
  TimedBegin(1);
  verletstep_++;
  const bool euler = !(verletstep_ < C.verlet_steps);
  const UpdateFuse fu = FuseUpdate(false);
  launch_verlet(stream, cap_, sc_, K, euler, arace_, cur_, G, shift_ ? shiftpos_ : nullptr, fu.cls, fu.pk);
  if (euler) verletstep_ = 0;
  std::swap(cur_.velrhop, cur_.velrhopm1);
  TimedEnd(1);
  UpdateTurn(false);
}

void SphGpuSingle::ComputeSymplecticPre() {
  UpdateTurn(true);
  TimedBegin(1);
  std::swap(cur_.posxy, cur_.posxypre);
  std::swap(cur_.posz, cur_.poszpre);
  std::swap(cur_.velrhop, cur_.velrhoppre);
  havepre_ = true;
  const UpdateFuse fu = FuseUpdate(true);
  launch_sym_pre(stream, cap_, sc_, K, arace_, cur_, G, fu.cls, fu.pk);
  TimedEnd(1);
  UpdateTurn(false);
}

void SphGpuSingle::ComputeSymplecticCorr() {
  UpdateTurn(true);
  TimedBegin(1);
  const UpdateFuse fu = FuseUpdate(false);
  launch_sym_cor(stream, cap_, sc_, K, arace_, cur_, G, shift_ ? shiftpos_ : nullptr, fu.cls, fu.pk);
  havepre_ = false;
  TimedEnd(1);
  UpdateTurn(false);
}

void SphGpuSingle::ComputeStep() {
  stepped_ = true;
  stepsdone_++;
  // (turns mode: each interaction's turn ends with the fold of the DtVariable after it)
  const bool foldturn = slab() && transport_->nranks > 1 && transport_->turns();
  if (step_algorithm_ == SPH_STEP_VERLET) {
    if (foldturn) fold_turn_ = 1;
    Interaction_Forces(1);
    DtVariable(DT_VERLET);
    ComputeVerlet();
    if (nftbodies_) RunFloating(false);
  } else {
    if (foldturn) fold_turn_ = 1;
    Interaction_Forces(2);
    DtVariable(DT_SYM_PRE);
    ComputeSymplecticPre();
    if (nftbodies_) RunFloating(true);
    RunCellDivide();
    if (foldturn) fold_turn_ = 1;
    Interaction_Forces(3);
    DtVariable(DT_SYM_COR);
    ComputeSymplecticCorr();
    if (nftbodies_) RunFloating(false);
  }
  if (nmotobj_) RunMotion();
  RunCellDivide();
}

// ---- moving boundaries and floating bodies ------------------------------------------------
void SphGpuSingle::RunMotion() {
  TimedBegin(1);
  launch_motion(stream, slab() ? cap_ : npb0_, sc_, K, motion_, motmovs_, motevts_, motdata_, cur_, normal_, G);
  TimedEnd(1);
}

void SphGpuSingle::RunFloating(bool predictor) {
  TimedBegin(1);
  SLAB_TRACE("floating allreduce");
  // the body sums span the whole domain: each slab sums its owned particles, the
  // partial sums are added over the slabs, every slab integrates the same body
  launch_ft_partial(stream, sc_, ftbodies_, nftbodies_, ftridp_, arace_, cur_, ftpart_);
  if (slab() && transport_->nranks > 1) transport_->allreduce_sum_f32(ftpart_, nftbodies_ * FT_NBLK * 6, stream);
  launch_ft_body(stream, sc_, K, ftbodies_, nftbodies_, ftridp_, nftp_, cur_, predictor, ftpart_, fttab_,
                 fttabdesc_, ftnormals_ ? normal_ : nullptr);
  TimedEnd(1);
}

// The flat program: one top-level object per ref (sph_solver_set_motion).
void SphGpuSingle::SetMotion(unsigned nobj, unsigned nmov, const SphMotionMov* movs, unsigned nevt,
                             const SphMotionEvent* evts) {
  if (!nobj || nobj > unsigned(MOT_MAXOBJ)) throw SphError(SPH_ERR_UNSUPPORTED, "number of moving objects out of range");
  std::vector<SphMotionObj> nodes(nobj);
  for (unsigned k = 0; k < nobj; k++) nodes[k] = SphMotionObj{-1, int32_t(k)};
  SetMotionTree(nobj, nodes.data(), nmov, movs, nevt, evts, 0, nullptr);
}

// JDsMotion::Init (JDsMotion.cpp:94-106) + JMotion::ReadXml / ObjAdd / AxisAdd / MovAdd* /
// EventAdd / Prepare (JMotion.cpp:96-317,556-700): the program uploaded once; k_motion runs
// it every step.
void SphGpuSingle::SetMotionTree(unsigned nnode, const SphMotionObj* nodes, unsigned nmov, const SphMotionMov* movs,
                                 unsigned nevt, const SphMotionEvent* evts, unsigned nrows, const double* rows) {
  if (stepped_ || motion_) throw SphError(SPH_ERR_STATE, "the motion is configured once, before the first step");
  if (!nnode || nnode > unsigned(MOT_MAXOBJ)) throw SphError(SPH_ERR_UNSUPPORTED, "number of motion objects out of range");
  if ((nmov && !movs) || (nevt && !evts) || (nrows && !rows)) throw SphError(SPH_ERR_ARG, "motion arrays missing");
  MotionDev md;
  std::memset(&md, 0, sizeof(md));
  md.nobj = int(nnode);
  // the tree: depth first, a parent before its children, every subtree contiguous (the
  // parent of a node is the previous node or one of its ancestors)
  std::vector<int> seen(MOT_MAXOBJ, 0);
  int nref = 0;
  for (unsigned i = 0; i < nnode; i++) {
    const int p = nodes[i].parent;
    bool ok = p < 0 || (p < int(i) && p >= 0);
    if (ok && p >= 0) {
      ok = false;
      for (int q = int(i) - 1; q >= 0 && !ok; q = md.obj[q].parent) ok = (q == p);
    }
    if (!ok) throw SphError(SPH_ERR_ARG, "motion objects: not in depth-first order");
    const int r = nodes[i].ref;
    if (r >= MOT_MAXOBJ || r < -1) throw SphError(SPH_ERR_ARG, "motion objects: ref out of range");
    if (r >= 0) {
      if (seen[r]++) throw SphError(SPH_ERR_ARG, "motion objects: a ref is used twice");
      nref = std::max(nref, r + 1);
    }
    md.obj[i].parent = p;
    md.obj[i].ref = r;
  }
  for (int r = 0; r < nref; r++)  // JMotion::CreateMotList
    if (!seen[r]) throw SphError(SPH_ERR_ARG, "Motion references are no consecutives.");
  md.nref = nref;
  std::vector<MotMov> mv(std::max(nmov, 1u));
  auto find = [&](int obj, int id) -> int {
    for (unsigned k = 0; k < nmov; k++)
      if (movs[k].obj == obj && movs[k].id == id) return int(k);
    return -1;
  };
  // JMotion::AxisAdd: an axis of two distinct points is shared by the object's movements that
  // name the same points; a circular movement's reference point (p1 == p2) is its own
  auto axis_add = [&](int obj, const double* p1, const double* p2) -> int {
    const bool same = p1[0] == p2[0] && p1[1] == p2[1] && p1[2] == p2[2];
    if (!same)
      for (int k = 0; k < md.naxis; k++) {
        const MotAxis& a = md.axis[k];
        if (a.obj == obj && a.p1[0] == p1[0] && a.p1[1] == p1[1] && a.p1[2] == p1[2] && a.p2[0] == p2[0] &&
            a.p2[1] == p2[1] && a.p2[2] == p2[2])
          return k;
      }
    if (md.naxis >= MOT_MAXAXIS) throw SphError(SPH_ERR_UNSUPPORTED, "too many motion axes");
    MotAxis& a = md.axis[md.naxis];
    for (int c = 0; c < 3; c++) {
      a.p1[c] = p1[c];
      a.p2[c] = p2[c];
    }
    a.obj = obj;
    return md.naxis++;
  };
  for (unsigned k = 0; k < nmov; k++) {
    const SphMotionMov& m = movs[k];
    if (m.obj < 0 || unsigned(m.obj) >= nnode) throw SphError(SPH_ERR_ARG, "movement of an unknown object");
    if (m.type < SPH_MOV_WAIT || m.type > SPH_MOV_NULL) throw SphError(SPH_ERR_UNSUPPORTED, "movement type");
    if (m.type == SPH_MOV_WAIT && m.duration < 0)
      throw SphError(SPH_ERR_ARG, "Wating times lenght lower than zero are not allowed.");
    if (find(m.obj, m.id) != int(k)) throw SphError(SPH_ERR_ARG, "Cannot add a movement with a existing id inside the object.");
    MotMov& d = mv[k];
    std::memset(&d, 0, sizeof(d));
    d.type = m.type;
    d.prev = m.prev;
    d.fields = m.fields;
    d.time = m.duration;
    d.nextidx = -1;
    d.ax = d.rax = -1;
    if (m.next) {
      d.nextidx = find(m.obj, m.next);
      if (d.nextidx < 0) throw SphError(SPH_ERR_ARG, "movement `next` is not defined in its object");
    }
    for (int c = 0; c < 3; c++) {
      d.v[c] = m.vec[c];
      d.v2[c] = m.vec2[c];
      d.phase[c] = m.phase[c];
    }
    d.ang = m.ang;
    d.ang2 = m.ang2;
    d.ang3 = m.ang3;
    const bool rot = m.type == SPH_MOV_ROT || m.type == SPH_MOV_ROTACE || m.type == SPH_MOV_ROTSINU ||
                     m.type == SPH_MOV_ROTFILE;
    const bool cir = m.type == SPH_MOV_CIR || m.type == SPH_MOV_CIRACE || m.type == SPH_MOV_CIRSINU;
    if (rot || cir) d.ax = axis_add(m.obj, m.axisp1, m.axisp2);
    if (cir) d.rax = axis_add(m.obj, m.ref, m.ref);
    if (m.type == SPH_MOV_RECTFILE || m.type == SPH_MOV_ROTFILE) {
      if (m.data_n < 2 || size_t(m.data_first) + m.data_n > nrows)
        throw SphError(SPH_ERR_ARG, "file movement: its table rows are out of range (at least two)");
      if (m.type == SPH_MOV_RECTFILE && !(m.fields & 7)) throw SphError(SPH_ERR_ARG, "You need at least one position field.");
      d.dfirst = int(m.data_first);
      d.dn = int(m.data_n);
    }
  }
  // events ordered from last to first start, with the reference's exchange sort
  std::vector<MotEvt> ev(nevt);
  for (unsigned k = 0; k < nevt; k++) {
    if (evts[k].obj < 0 || unsigned(evts[k].obj) >= nnode) throw SphError(SPH_ERR_ARG, "event of an unknown object");
    ev[k].obj = evts[k].obj;
    ev[k].mov = find(evts[k].obj, evts[k].mov);
    if (ev[k].mov < 0) throw SphError(SPH_ERR_ARG, "event of an undefined movement");
    ev[k].start = evts[k].start;
    ev[k].finish = evts[k].finish;
  }
  for (unsigned c = 0; c + 1 < nevt; c++)
    for (unsigned c2 = c + 1; c2 < nevt; c2++)
      if (ev[c].start < ev[c2].start) std::swap(ev[c], ev[c2]);
  md.eventnext = int(nevt) - 1;
  check_hip(hipMalloc((void**)&motion_, sizeof(MotionDev)), "hipMalloc motion");
  allocs_.push_back(motion_);
  check_hip(hipMalloc((void**)&motmovs_, sizeof(MotMov) * mv.size()), "hipMalloc motion");
  allocs_.push_back(motmovs_);
  check_hip(hipMalloc((void**)&motevts_, sizeof(MotEvt) * std::max(nevt, 1u)), "hipMalloc motion");
  allocs_.push_back(motevts_);
  check_hip(hipMalloc((void**)&motdata_, sizeof(double) * 4 * std::max(nrows, 1u)), "hipMalloc motion");
  allocs_.push_back(motdata_);
  check_hip(hipMemcpy(motion_, &md, sizeof(md), hipMemcpyHostToDevice), "upload motion");
  check_hip(hipMemcpy(motmovs_, mv.data(), sizeof(MotMov) * mv.size(), hipMemcpyHostToDevice), "upload motion");
  if (nevt) check_hip(hipMemcpy(motevts_, ev.data(), sizeof(MotEvt) * nevt, hipMemcpyHostToDevice), "upload motion");
  if (nrows)
    check_hip(hipMemcpy(motdata_, rows, sizeof(double) * 4 * nrows, hipMemcpyHostToDevice), "upload motion tables");
  nmotobj_ = unsigned(nref);
  // restart: JDsMotion::SetTimeMod/ResetTime run the program from 0 to the PART time
  double t0 = 0;
  check_hip(hipMemcpy(&t0, &sc_->time, sizeof(double), hipMemcpyDeviceToHost), "read time");
  if (t0 > 0) launch_motion_advance(stream, sc_, motion_, motmovs_, motevts_, motdata_, 0.0, t0);
  Sync();
}

// JSph::LoadCaseConfig floating objects (JSph.cpp:1046-1100).
void SphGpuSingle::SetFloatings(unsigned nft, const SphFloatingDef* defs, double ftpause) {
  if (stepped_ || ftbodies_) throw SphError(SPH_ERR_STATE, "the floating bodies are configured once, before the first step");
  if (!nft || !defs) throw SphError(SPH_ERR_ARG, "no floating bodies");
  if (nn_) {
    // the v5.0 NN solver indexes its phase constants with a floating particle's code value,
    // its body index (JSphCpu_NN_FDA.cpp:199-200, 231, 267): bodies beyond the phases would
    // read past the phase table there
    if (nft > C.nphases) throw SphError(SPH_ERR_UNSUPPORTED, "NN multiphase: more floating bodies than phases");
  }
  if (C.symmetry) throw SphError(SPH_ERR_ARG, "Symmetry is not allowed with floating bodies.");  // JSph.cpp:1177
  std::vector<FtBody> b(nft);
  std::vector<float> massp(nft);
  unsigned begin = casenpb_;
  for (unsigned c = 0; c < nft; c++) {
    const SphFloatingDef& d = defs[c];
    if (d.idbegin != begin || !d.count) throw SphError(SPH_ERR_ARG, "floating blocks must follow the boundary in idp");
    FtBody& f = b[c];
    std::memset(&f, 0, sizeof(f));
    f.begin = d.idbegin - casenpb_;
    f.count = d.count;
    f.mass = float(d.massbody);
    f.massp = float(d.masspart);
    f.ftpause = float(ftpause);  // GetValueFloat (JSph.cpp:688)
    for (int k = 0; k < 9; k++) f.inertia[k] = float(d.inertia[k]);
    for (int k = 0; k < 3; k++) {
      f.center[k] = d.center[k];
      f.fvel[k] = float(d.linvelini[k]);
      f.fomega[k] = float(d.angvelini[k]);
    }
    // ComputeConstraintsValue (DualSphDef.h:456-464)
    f.constraints = (d.translationfree[0] ? 0u : 1u) | (d.translationfree[1] ? 0u : 2u) |
                    (d.translationfree[2] ? 0u : 4u) | (d.rotationfree[0] ? 0u : 8u) |
                    (d.rotationfree[1] ? 0u : 16u) | (d.rotationfree[2] ? 0u : 32u);
    massp[c] = f.massp;
    begin += d.count;
  }
  const unsigned nftp = begin - casenpb_;
  check_hip(hipMalloc((void**)&ftbodies_, sizeof(FtBody) * nft), "hipMalloc floatings");
  allocs_.push_back(ftbodies_);
  check_hip(hipMalloc((void**)&ftmassp_, sizeof(float) * nft), "hipMalloc floatings");
  allocs_.push_back(ftmassp_);
  check_hip(hipMalloc((void**)&ftridp_, sizeof(unsigned) * nftp), "hipMalloc floatings");
  allocs_.push_back(ftridp_);
  check_hip(hipMalloc((void**)&ftpart_, sizeof(float) * 6 * FT_NBLK * nft), "hipMalloc floatings");
  allocs_.push_back(ftpart_);
  check_hip(hipMemcpy(ftbodies_, b.data(), sizeof(FtBody) * nft, hipMemcpyHostToDevice), "upload floatings");
  check_hip(hipMemcpy(ftmassp_, massp.data(), sizeof(float) * nft, hipMemcpyHostToDevice), "upload floatings");
  nftbodies_ = int(nft);
  nftp_ = nftp;
  K.nftbodies = int(nft);
  // floating p2 carry their own mass: the FT instantiation of the tiled kernel (or the
  // per-particle kernel under SPH_INTERACTION=simple / CellMode=half)
  launch_ft_ridp(stream, cap_, sc_, cur_, casenpb_, nftp_, ftridp_, K, G);
  Sync();
}

// FtLinearVel / FtAngularVel / FtLinearForce / FtAngularForce of one body (JSph.cpp:1060-1082):
// the rows are re-uploaded as one buffer with a {first row, rows} descriptor per table.
void SphGpuSingle::SetFloatingTable(unsigned body, int kind, unsigned n, const double* times, const double* values) {
  if (stepped_) throw SphError(SPH_ERR_STATE, "floating tables are configured before the first step");
  if (!ftbodies_ || body >= unsigned(nftbodies_)) throw SphError(SPH_ERR_ARG, "floating table of an unknown body");
  if (kind < SPH_FTTAB_LINVEL || kind > SPH_FTTAB_ANGFORCE) throw SphError(SPH_ERR_ARG, "invalid floating table kind");
  // External forces: v5.2 adds them to FtoForces before FtCalcForces adds the particle sums
  // (sum + (0 + ext)); the v5.0 NN solver adds them inside FtCalcForces after the sums
  // (FtSumExternalForces, JSphCpuSingle.cpp:849 of that solver): the same float additions, so
  // both run k_ft_forces's (sph_bodies.hip).
  if (!n || !times || !values) throw SphError(SPH_ERR_ARG, "There are not times.");
  std::vector<double4> rows(n);
  for (unsigned i = 0; i < n; i++) {  // rows in the order given (any time order, as the reference)
    const double* v = values + 3 * size_t(i);
    if (kind >= SPH_FTTAB_LINFORCE && (v[0] == DBL_MAX || v[1] == DBL_MAX || v[2] == DBL_MAX))
      throw SphError(SPH_ERR_ARG, "external forces have no 'none' components");
    rows[i] = make_double4(times[i], v[0], v[1], v[2]);
  }
  fttabs_.resize(size_t(nftbodies_) * 4);
  fttabs_[size_t(body) * 4 + size_t(kind)] = rows;
  UploadFloatingTables();
}

void SphGpuSingle::UploadFloatingTables() {
  if (fttabs_.empty()) return;
  std::vector<double4> all;
  std::vector<FtTabDesc> desc(fttabs_.size());
  for (size_t t = 0; t < fttabs_.size(); t++) {
    desc[t] = FtTabDesc{int(all.size()), int(fttabs_[t].size()), -1, -1, 0.0};
    all.insert(all.end(), fttabs_[t].begin(), fttabs_[t].end());
  }
  Sync();
  for (void* p : {(void*)fttab_, (void*)fttabdesc_}) {
    if (!p) continue;
    (void)hipFree(p);
    allocs_.erase(std::remove(allocs_.begin(), allocs_.end(), p), allocs_.end());
  }
  check_hip(hipMalloc((void**)&fttab_, sizeof(double4) * std::max<size_t>(all.size(), 1)), "hipMalloc floating tables");
  allocs_.push_back(fttab_);
  check_hip(hipMalloc((void**)&fttabdesc_, sizeof(FtTabDesc) * desc.size()), "hipMalloc floating tables");
  allocs_.push_back(fttabdesc_);
  if (!all.empty())
    check_hip(hipMemcpy(fttab_, all.data(), sizeof(double4) * all.size(), hipMemcpyHostToDevice), "upload tables");
  check_hip(hipMemcpy(fttabdesc_, desc.data(), sizeof(FtTabDesc) * desc.size(), hipMemcpyHostToDevice),
            "upload tables");
}

// DtFixedFile (JDsFixedDt) and ViscoTime (JDsViscoInput) tables on the device; k_dt reads
// them at every DtVariable (fixed dt) and at every step's end (the next step's Visco).
void SphGpuSingle::SetTimeTable(int kind, unsigned n, const double* times, const double* values) {
  if (kind != SPH_TTAB_DTFIXED && kind != SPH_TTAB_VISCO) throw SphError(SPH_ERR_ARG, "invalid time table kind");
  if (n == 1 || (n && (!times || !values))) throw SphError(SPH_ERR_ARG, "Cannot be less than two values.");
  if (kind == SPH_TTAB_DTFIXED && n && C.dtfixed > 0)
    throw SphError(SPH_ERR_ARG, "The parameters 'DtFixed' and 'DtFixedFile' cannot be used at the same time.");
  // NN multiphase: ViscoTime sets Visco every step (JSphCpuSingle.cpp:1128 of the v5.0 solver),
  // which no NN interaction reads (they take the phases' viscosities, JSphCpu_NN_FDA.cpp:267,
  // JSphCpu_NN_SPH.cpp:202,413): the table is kept and, as there, changes nothing.
  Sync();
  void*& buf = (kind == SPH_TTAB_DTFIXED ? dttab_ : viscotab_);
  check_hip(hipMemset(kind == SPH_TTAB_DTFIXED ? &sc_->dtfix_pos : &sc_->visco_pos, 0, sizeof(int)), "reset table row");
  if (buf) {
    (void)hipFree(buf);
    allocs_.erase(std::remove(allocs_.begin(), allocs_.end(), buf), allocs_.end());
    buf = nullptr;
  }
  if (kind == SPH_TTAB_DTFIXED) {
    K.dtfix_n = int(n);
    K.dtfix_t = K.dtfix_v = nullptr;
    if (n) {
      std::vector<double> h(times, times + n);
      h.insert(h.end(), values, values + n);
      check_hip(hipMalloc(&buf, sizeof(double) * h.size()), "hipMalloc dt table");
      allocs_.push_back(buf);
      check_hip(hipMemcpy(buf, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice), "upload dt table");
      K.dtfix_t = (const double*)buf;
      K.dtfix_v = K.dtfix_t + n;
    }
  } else {
    K.visco_n = int(n);
    K.visco_t = K.visco_v = nullptr;
    if (n) {  // JDsViscoInput reads float rows (ReadNextFloat)
      std::vector<float> h(2 * size_t(n));
      for (unsigned i = 0; i < n; i++) {
        h[i] = float(times[i]);
        h[n + i] = float(values[i]);
      }
      check_hip(hipMalloc(&buf, sizeof(float) * h.size()), "hipMalloc visco table");
      allocs_.push_back(buf);
      check_hip(hipMemcpy(buf, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice), "upload visco table");
      K.visco_t = (const float*)buf;
      K.visco_v = K.visco_t + n;
    }
    launch_visco_init(stream, sc_, K);
    Sync();
  }
}

unsigned SphGpuSingle::Floatings(SphFloatingState* out, unsigned cap) {
  if (!nftbodies_) return 0;
  std::vector<FtBody> b(nftbodies_);
  Sync();
  check_hip(hipMemcpy(b.data(), ftbodies_, sizeof(FtBody) * b.size(), hipMemcpyDeviceToHost), "read floatings");
  for (unsigned c = 0; c < unsigned(nftbodies_) && c < cap && out; c++) {
    SphFloatingState& o = out[c];
    std::memset(&o, 0, sizeof(o));
    for (int k = 0; k < 3; k++) {
      o.center[k] = b[c].center[k];
      o.fvel[k] = b[c].fvel[k];
      o.fomega[k] = b[c].fomega[k];
      o.angles[k] = b[c].angles[k];
      o.facelin[k] = b[c].facelin[k];
      o.faceang[k] = b[c].faceang[k];
    }
  }
  return unsigned(nftbodies_);
}

void SphGpuSingle::Run(unsigned nsteps) {
  check_hip(hipSetDevice(device), "hipSetDevice");
  in_run_ = true;
  try {
    for (unsigned s = 0; s < nsteps; s++) ComputeStep();
    GhostFinish();  // the state between runs is whole (ghosts in place)
  } catch (...) {
    in_run_ = false;
    throw;
  }
  in_run_ = false;
  check_hip(hipGetLastError(), "kernel launch");
}

void SphGpuSingle::Sync() { check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize"); }

SphRunStats SphGpuSingle::Stats() {
  check_hip(hipMemcpyAsync(sc_host_, sc_, sizeof(DevScalars), hipMemcpyDeviceToHost, stream), "read scalars");
  Sync();
  const DevScalars& s = *sc_host_;
  SphRunStats r;
  std::memset(&r, 0, sizeof(r));
  r.time = s.time;
  r.last_dt = s.last_dt;
  r.sym_dtpre = s.symdtpre;
  r.nstep = s.nstep;
  // a slab reports the particles it owns (no ghosts); alone it holds exactly those
  r.np = (slab() && (transport_->has_left() || transport_->has_right())) ? s.nown : s.np;
  r.npb = s.npb;
  r.npbok = s.npbok;
  r.nout = s.nout;
  r.dtmodif = s.dtmodif;
  r.error_flags = s.error_flags;
  r.velmax = s.last_velmax;
  r.acemax = s.last_acemax;
  r.viscdtmax = s.last_viscdt;
  r.viscetadtmax = s.last_visceta;
  return r;
}

// The face sizes of the last exchange and the records the last mDBC face pack counted.
std::string SphGpuSingle::HaloDiag() {
  unsigned cnt[2] = {0u, 0u};
  if (mdbcface_ && slab()) {
    const bool hl = transport_->has_left(), hr = transport_->has_right();
    if (hl) check_hip(hipMemcpy(&cnt[0], &mdbcface_[0].idp, 4, hipMemcpyDeviceToHost), "read face count");
    if (hr)
      check_hip(hipMemcpy(&cnt[1], &mdbcface_[hl ? face_sl_ + 1u : 0u].idp, 4, hipMemcpyDeviceToHost),
                "read face count");
  }
  return "slab " + std::to_string(slabcfg_.rank) + " face sizes sl " + std::to_string(face_sl_) + " sr " +
         std::to_string(face_sr_) + " rl " + std::to_string(face_rl_) + " rr " + std::to_string(face_rr_) +
         ", mDBC records counted " + std::to_string(cnt[0]) + " / " + std::to_string(cnt[1]);
}

void SphGpuSingle::CheckErrors() {
  const SphRunStats s = Stats();
  if (s.error_flags & ERR_BOUNDOUT) throw SphError(SPH_ERR_BOUNDOUT, "boundary particles were excluded (AbortBoundOut)");
  if (s.error_flags & ERR_DT_NAN) throw SphError(SPH_ERR_DT, "The computed Dt is NaN or infinity");
  if (s.error_flags & ERR_HALO_NODE)
    throw SphError(SPH_ERR_UNSUPPORTED, "slab halo: an mDBC ghost node needs particles beyond the slab's ghost columns");
  if (s.error_flags & ERR_HALO_FACE)
    throw SphError(SPH_ERR_STATE, "slab halo: a face record did not fit its buffer (step " + std::to_string(s.nstep) +
                                      ", " + HaloDiag() + ")");
  if (s.error_flags & ERR_HALO_MISS)
    throw SphError(SPH_ERR_STATE, "slab halo: a face record found no ghost copy of its particle");
  if (s.error_flags & ERR_HALO_GHOST)
    throw SphError(SPH_ERR_STATE, "slab halo: a ghost record the divide did not place (face counts disagree)");
}

unsigned SphGpuSingle::DtTrace(double* out, unsigned cap) {
  const SphRunStats s = Stats();
  const unsigned n = unsigned(std::min<unsigned long long>(s.nstep, tracecap_));
  if (out && cap) {
    std::vector<double> all(tracecap_);
    check_hip(hipMemcpy(all.data(), dttrace_, 8 * size_t(tracecap_), hipMemcpyDeviceToHost), "read dt trace");
    const unsigned long long first = s.nstep - n;
    for (unsigned i = 0; i < n && i < cap; i++) out[i] = all[(first + i) % tracecap_];
  }
  return n;
}

void SphGpuSingle::Download(SphParticlesHost& out) {
  const SphRunStats s = Stats();
  const unsigned n = sc_host_->np;  // held particles (a slab also holds ghosts)
  if (out.n < s.np) throw SphError(SPH_ERR_ARG, "output buffer too small");
  std::vector<double2> pxy(n);
  std::vector<double> pz(n);
  std::vector<float4> vr(n);
  std::vector<unsigned> idp(n), dcell(n);
  std::vector<typecode> code(n);
  check_hip(hipMemcpy(pxy.data(), cur_.posxy, 16 * size_t(n), hipMemcpyDeviceToHost), "download posxy");
  check_hip(hipMemcpy(pz.data(), cur_.posz, 8 * size_t(n), hipMemcpyDeviceToHost), "download posz");
  check_hip(hipMemcpy(vr.data(), cur_.velrhop, 16 * size_t(n), hipMemcpyDeviceToHost), "download velrhop");
  check_hip(hipMemcpy(idp.data(), cur_.idp, 4 * size_t(n), hipMemcpyDeviceToHost), "download idp");
  check_hip(hipMemcpy(code.data(), cur_.code, 2 * size_t(n), hipMemcpyDeviceToHost), "download code");
  if (slab()) check_hip(hipMemcpy(dcell.data(), cur_.dcell, 4 * size_t(n), hipMemcpyDeviceToHost), "download dcell");
  unsigned k = 0;
  for (unsigned p = 0; p < n; p++) {
    if (slab()) {  // owned particles only
      if (!slab_owned(G, slab_local(G, C.dom_cellcode, dcell[p]))) continue;
    }
    if (out.idp) out.idp[k] = idp[p];
    if (out.code) out.code[k] = code[p];
    if (out.pos) { out.pos[3 * k] = pxy[p].x; out.pos[3 * k + 1] = pxy[p].y; out.pos[3 * k + 2] = pz[p]; }
    if (out.vel) { out.vel[3 * k] = vr[p].x; out.vel[3 * k + 1] = vr[p].y; out.vel[3 * k + 2] = vr[p].z; }
    if (out.rhop) out.rhop[k] = vr[p].w;
    k++;
  }
  if (k != s.np) throw SphError(SPH_ERR_STATE, "owned particle count mismatch");
  out.n = k;
}

void SphGpuSingle::DownloadInteraction(SphInterOut& out) {
  if (slab()) throw SphError(SPH_ERR_UNSUPPORTED, "interaction download is single-domain only");
  // Runs one interaction on the current state (like or_interaction) and reads ar/ace back.
  // Maxima accumulated so far (VelMax from the last divide) are kept for this call.
  Interaction_Forces(1);
  // an inspection: the SPS stress tensor of the state stays the one the next step starts from
  if (sps_) std::swap(cur_.tau, taunew_);
  DtVariable(DT_PEEK);
  const SphRunStats s = Stats();
  std::vector<float4> a(s.np);
  check_hip(hipMemcpy(a.data(), arace_, 16 * size_t(s.np), hipMemcpyDeviceToHost), "download arace");
  for (unsigned p = 0; p < s.np; p++) {
    if (out.ar) out.ar[p] = a[p].w;
    if (out.ace) { out.ace[3 * p] = a[p].x; out.ace[3 * p + 1] = a[p].y; out.ace[3 * p + 2] = a[p].z; }
  }
  out.velmax = s.velmax;
  out.acemax = s.acemax;
  out.viscdtmax = s.viscdtmax;
  // Leave the device maxima as a fresh interaction would find them (VelMax stays:
  // it belongs to the last divide).
  check_hip(hipMemsetAsync(&sc_->red[RED_ACEMAX2][0], 0, 4 * RED_SLOTS, stream), "reset acemax");
  check_hip(hipMemsetAsync(&sc_->red[RED_VISCDT][0], 0, 4 * RED_SLOTS, stream), "reset viscdt");
  Sync();
}

unsigned SphGpuSingle::DownloadNormals(float* out, unsigned cap, int* usenormalsft) {
  if (!normal_) throw SphError(SPH_ERR_STATE, "the case has no mDBC normals");
  if (usenormalsft) *usenormalsft = ftnormals_ ? 1 : 0;
  if (!out) return nnormal_;
  if (cap < nnormal_) throw SphError(SPH_ERR_ARG, "normals buffer too small");
  Sync();
  std::vector<float4> v(nnormal_);
  check_hip(hipMemcpy(v.data(), normal_, sizeof(float4) * nnormal_, hipMemcpyDeviceToHost), "download normals");
  for (unsigned i = 0; i < nnormal_; i++) {
    out[3 * i] = v[i].x;
    out[3 * i + 1] = v[i].y;
    out[3 * i + 2] = v[i].z;
  }
  return nnormal_;
}

void SphGpuSingle::CountPairs(uint64_t out[6]) {
  check_hip(hipMemsetAsync(pairs_, 0, 8 * 6, stream), "memset pairs");
  launch_count_pairs(stream, cap_, sc_, poscell_, begincell_, G, K, pairs_);
  unsigned long long h[6];
  check_hip(hipMemcpyAsync(h, pairs_, 8 * 6, hipMemcpyDeviceToHost, stream), "read pairs");
  Sync();
  for (int i = 0; i < 6; i++) out[i] = h[i];
}

// ---- in-process slab group -----------------------------------------------------------
SphSlabGroup::SphSlabGroup(const SphCaseDef& cdef, const SphParticlesHost& all, int nslabs, const int* devices,
                           const int* bounds, int axis)
    : hub_(std::make_shared<LocalHub>(nslabs)) {
  if (nslabs < 1) throw SphError(SPH_ERR_ARG, "nslabs < 1");
  for (int i = 0; i < nslabs; i++) {
    SlabConfig sc;
    sc.rank = i;
    sc.nranks = nslabs;
    sc.c0 = bounds[i];
    sc.c1 = bounds[i + 1];
    sc.axis = axis;
    slabs.emplace_back(new SphGpuSingle(cdef, all, devices[i], sc, make_local_transport(hub_, i)));
  }
  // Slabs sharing a GPU: the ghosts go before the interaction (one item list).  There the
  // face launch of the overlap waits for the CU slots of the interior launch and of the
  // other slabs' work, and the in-process copies use the same GPU's engines: measured on the
  // cfg3 two-slab split, 13.72 ms/step without overlap vs 13.84-13.95 with it.
  // Slabs on their own GPUs keep the overlap (sph_slab_group_set_overlap changes either).
  for (int i = 0; i < nslabs; i++)
    for (int j = 0; j < nslabs; j++)
      if (i != j && devices[i] == devices[j]) slabs[i]->MarkSharedDevice();
  // one GPU: the dt maxima and the floating / re-partition sums reduce on the device
  hub_->onedev = std::all_of(devices, devices + nslabs, [&](int d) { return d == devices[0]; });
}

void SphSlabGroup::Run(unsigned nsteps) {
  const size_t n = slabs.size();
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> err(n);
  std::vector<int> primary(n, 0);
  for (size_t i = 0; i < n; i++)
    th.emplace_back([&, i] {
      try {
        slabs[i]->Run(nsteps);
        slabs[i]->Sync();
        slabs[i]->CheckErrors();  // a fatal error halts every slab at the same step (DtVariable)
      } catch (const SphError& e) {
        err[i] = std::current_exception();
        primary[i] = std::string(e.what()).find("aborted by another slab") == std::string::npos;
        hub_->abort();
      } catch (...) {
        err[i] = std::current_exception();
        primary[i] = 1;
        hub_->abort();
      }
    });
  for (auto& t : th) t.join();
  for (size_t i = 0; i < n; i++)
    if (err[i] && primary[i]) {
      try {
        std::rethrow_exception(err[i]);
      } catch (const SphError& e) {
        // a face overflow is seen on every slab (folded): say where each slab stood
        if (std::string(e.what()).find("did not fit") == std::string::npos) throw;
        std::string m = e.what();
        for (size_t j = 0; j < n; j++) {
          try {
            m += "; " + slabs[j]->HaloDiag();
          } catch (...) {
          }
        }
        throw SphError(e.status, m);
      }
    }
  for (size_t i = 0; i < n; i++)
    if (err[i]) std::rethrow_exception(err[i]);
}

}  // namespace sphx
