// sph_oracle.cpp — CPU ORACLE for the SPH hot path (TEST INFRASTRUCTURE ONLY).
//
// Restatement of the reference CPU path of DualSPHysics v5.2 for the dam-break
// feature set.  Every function names the reference file:line it follows.  The
// arithmetic keeps the reference's precision choices (double positions, float
// velocity/density/accumulators, double time integration intermediates) and the
// reference's summation order (fluid-fluid pass, then fluid-bound pass, each with
// its own accumulators, combined exactly as JSphCpu.cpp:800-818 does).
//
// Parity pin: tests/test_oracle_golden.py checks this oracle against PART files
// written by the reference solver itself (built from /root/reference sources by
// oracle/Makefile) — fixtures in tests/golden/, generator tests/golden/make_golden.py.
//
// Build (done by __graft_entry__.build()):
//   g++ -O3 -fopenmp -ffast-math -shared -fPIC sph_oracle.cpp -o build/libsph_oracle.so
// (same optimisation flags as the reference's Makefile_cpu:19-28).
#include "sph_oracle.h"

#include <omp.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

struct d3 { double x, y, z; };
struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };
struct u3 { unsigned x, y, z; };
typedef unsigned short typecode;

// ---- DualSphDef.h:161-221 (16-bit typecode) ----------------------------------
constexpr typecode CODE_MASKSPECIAL = 0xe000, CODE_OUTIGNORE = 0x4000, CODE_OUTMOVE = 0x6000,
                   CODE_OUTPOS = 0x8000, CODE_OUTRHOP = 0xA000, CODE_MASKTYPE = 0x1800,
                   CODE_TYPE_FLOATING = 0x1000, CODE_TYPE_FLUID = 0x1800;
inline typecode CodeSpecial(typecode c) { return c & CODE_MASKSPECIAL; }
inline typecode CodeType(typecode c) { return c & CODE_MASKTYPE; }
inline typecode CodeSetNormal(typecode c) { return c & typecode(~CODE_MASKSPECIAL); }
inline bool CodeIsNormal(typecode c) { return CodeSpecial(c) == 0; }
inline bool CodeIsFluid(typecode c) { return CodeType(c) == CODE_TYPE_FLUID; }
inline bool CodeIsOutRhop(typecode c) { return CodeSpecial(c) == CODE_OUTRHOP; }

// ---- JDsDcellDef.h:24-43 (DCEL cell code) -------------------------------------
inline unsigned DcelGetCode(unsigned sx, unsigned sy, unsigned sz) {
  return ((sx + 1) << 25) | (sy << 20) | (sz << 15) | ((sy + sz) << 10) | ((sx + 1 + sz) << 5) | (sx + 1 + sy);
}
inline unsigned DcelCellx(unsigned dcc, unsigned cel) { return cel >> ((dcc >> 10) & 31); }
inline unsigned DcelCelly(unsigned dcc, unsigned cel) { return (cel << (dcc >> 25)) >> ((dcc >> 5) & 31); }
inline unsigned DcelCellz(unsigned dcc, unsigned cel) { return (cel << (dcc & 31)) >> (dcc & 31); }
inline unsigned DcelCell(unsigned dcc, unsigned cx, unsigned cy, unsigned cz) {
  return (cx << ((dcc >> 10) & 31)) | (cy << ((dcc >> 15) & 31)) | cz;
}
// JDsDcell.cpp:41-62 (CalcCellDistribution) + :64-69 (CalcCellCode).
unsigned CalcBitsValue(unsigned v, unsigned minbits) {
  // Functions.cpp: number of bits to store v (at least minbits).
  unsigned nbits = 1;
  for (; v >> nbits; nbits++) {}
  return std::max(nbits, minbits);
}
unsigned CalcCellCode(u3 ncells) {
  unsigned sx = CalcBitsValue(ncells.x, 2), sy = CalcBitsValue(ncells.y, 2), sz = CalcBitsValue(ncells.z, 2);
  const unsigned smin = sx + sy + sz, maxbits = 31;
  if (smin > maxbits) return 0;
  unsigned rest = maxbits - smin;
  while (rest) {
    if (rest) { sx++; rest--; }
    if (rest) { sy++; rest--; }
    if (rest) { sz++; rest--; }
  }
  return DcelGetCode(sx, sy, sz);
}

// ---- JSph::ConfigConstants1/2 (JSph.cpp:1392-1457), ConfigCellDivision (:1772-1788),
//      LoadCaseParticles map limits (:2056-2076), SelecDomain (:1794-1829) -------------
void Derive(const SphCaseDef& c, SphConstants& k) {
  if (c.kernel != SPH_KERNEL_WENDLAND && c.kernel != SPH_KERNEL_CUBIC) throw std::runtime_error("Kernel choice is not valid.");
  if (c.cellmode != SPH_CELLMODE_FULL && c.cellmode != SPH_CELLMODE_HALF) throw std::runtime_error("invalid cellmode");
  memset(&k, 0, sizeof(k));
  // JSph::LoadConfigCtes (JSph.cpp:567-583): values narrowed to float.
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
  // ConfigConstants1 (JSph.cpp:1394-1412).
  const float kernelk = 2.0f;  // GetKernelWendland_Factor (FunSphKernel.h:190)
  const double h = k.kernelh;
  k.kernelsize = float(h * kernelk);
  k.kernelsize2 = k.kernelsize * k.kernelsize;
  k.data2d = c.data2d ? 1 : 0;
  if (k.data2d) {  // FunSphKernel.h:193-196 (2D)
    k.awen = float(0.557 / (h * h));
    k.bwen = float(-2.7852 / (h * h * h));
  } else {
    k.awen = float(0.41778 / (h * h * h));  // FunSphKernel.h:198-199 (3D)
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
  // ConfigConstants2 (JSph.cpp:1445-1449).
  const float ddtvalue = float(c.ddtvalue);
  k.ddtkh = k.kernelsize * ddtvalue;
  k.ddtgz = float(double(k.rhopzero) * double(std::fabs(k.gravity[2])) / double(k.cteb));
  k.dtini = c.dtini;
  k.dtmin = c.dtmin;
  const float coefdtmin = float(c.coefdtmin);
  if (!k.dtini) k.dtini = k.kernelh / k.cs0;
  if (!k.dtmin) k.dtmin = (k.kernelh / k.cs0) * coefdtmin;
  // ConfigCellDivision (JSph.cpp:1772-1788).
  k.scelldiv = (c.cellmode == SPH_CELLMODE_FULL ? 1 : 2);
  k.scell = k.kernelsize / k.scelldiv;
  k.movlimit = k.scell * 0.9f;
  // Map (no periodic): Map_PosMin = MapRealPosMin (JSph.cpp:2062-2076).
  double msize[3];
  for (int i = 0; i < 3; i++) {
    k.map_realposmin[i] = c.map_realposmin[i];
    k.map_realsize[i] = c.map_realposmax[i] - c.map_realposmin[i];
    k.dom_posmin[i] = c.map_realposmin[i];
    msize[i] = c.map_realposmax[i] - c.map_realposmin[i];
    k.dom_cells[i] = unsigned(std::ceil(msize[i] / k.scell));
  }
  // SelecDomain(TUint3(0),Map_Cells) (JSph.cpp:1794-1829).
  k.dom_cellcode = CalcCellCode(u3{k.dom_cells[0] + 1, k.dom_cells[1] + 1, k.dom_cells[2] + 1});
  if (!k.dom_cellcode) throw std::runtime_error("failed to select a valid CellCode");
  // Boundary configuration (JSph.cpp:626-640, 785-790).
  k.tboundary = (c.tboundary == 0 ? SPH_BOUND_DBC : c.tboundary);
  if (k.tboundary != SPH_BOUND_DBC && k.tboundary != SPH_BOUND_MDBC)
    throw std::runtime_error("Boundary Condition method is not valid.");
  k.slipmode = (k.tboundary == SPH_BOUND_MDBC ? (c.slipmode == 0 ? SPH_SLIP_VEL0 : c.slipmode) : SPH_SLIP_VEL0);
  if (k.slipmode != SPH_SLIP_VEL0) throw std::runtime_error("Only the slip mode velocity=0 is allowed with mDBC conditions.");
  k.mdbc_threshold = (k.tboundary == SPH_BOUND_MDBC ? float(c.mdbc_threshold) : 0.f);
  // Single-phase classic formulation, artificial viscosity, no shifting: the only options
  // this restatement covers (the v5.0 NN solver is pinned to its own binary's PARTs).
  k.rheology = (c.rheology == 0 ? SPH_RHEOLOGY_SINGLE : c.rheology);
  k.velgrad = (c.velgrad == 0 ? SPH_VELGRAD_FDA : c.velgrad);
  k.tvisco = (c.tvisco == 0 ? SPH_VISCO_ARTIFICIAL : c.tvisco);
  k.shift_mode = c.shift_mode;
  k.shift_coef = float(c.shift_coef);
  k.shift_tfs = float(c.shift_tfs);
  k.relaxation_dt = float(c.relaxation_dt);
  if (k.rheology != SPH_RHEOLOGY_SINGLE || k.tvisco != SPH_VISCO_ARTIFICIAL || k.shift_mode != SPH_SHIFT_NONE)
    throw std::runtime_error("the oracle restates the single-phase artificial-viscosity path only");
  // Symmetry (JSph.cpp:714, checks :1174-1179; MapRealPosMin.y = 0, :1386, set by the case)
  k.symmetry = c.symmetry ? 1 : 0;
  if (k.symmetry && k.data2d) throw std::runtime_error("Symmetry is not allowed with 2-D simulations.");
}

// EOS as the reference binary evaluates it: FunSphEos.h:37-39 calls the unqualified
// `pow` inside namespace fsph, which resolves to the C ::pow(double,double), and
// -ffast-math turns rhop/rhop0 into rhop*(1/rhop0); so Press =
// float(double(b)*(pow(double(rhop*(1/rhop0)),gamma)-1)).  With this the oracle is
// BIT-IDENTICAL to the reference after the first step of the DDT-free case.  The pow
// is kept out of line: if GCC vectorised the loop with libmvec, results would depend
// on the OpenMP chunking (i.e. on the thread count).
__attribute__((noinline)) double scalar_pow(double x, double y) { return std::pow(x, y); }

// ---- Wendland kernel (FunSphKernel.h:217-224) and EOS (FunSphEos.h:37-47) -----------
inline float WendlandFac(const SphConstants& k, float rr2) {
  const float rad = std::sqrt(rr2);
  const float qq = rad / k.kernelh;
  const float wqq1 = 1.f - 0.5f * qq;
  return k.bwen * qq * wqq1 * wqq1 * wqq1 / rad;
}
// GetKernelWendland_WabFac (FunSphKernel.h:226-234).
inline float WendlandWabFac(const SphConstants& k, float rr2, float& fac) {
  const float rad = std::sqrt(rr2);
  const float qq = rad / k.kernelh;
  const float wqq1 = 1.f - 0.5f * qq;
  const float wqq2 = wqq1 * wqq1;
  fac = k.bwen * qq * wqq2 * wqq1 / rad;
  const float wqq = qq + qq + 1.f;
  return k.awen * wqq * wqq2 * wqq2;
}
// Cubic spline (FunSphKernel.h:89-149): GetKernelCubic_Wab / _Fac / _WabFac / _Tensil.
inline float CubicWab(const SphConstants& k, float rr2) {
  const float rad = std::sqrt(rr2);
  const float qq = rad / k.kernelh;
  if (rad > k.kernelh) {
    const float wqq1 = 2.0f - qq;
    const float wqq2 = wqq1 * wqq1;
    return k.cub_a24 * (wqq2 * wqq1);
  }
  const float wqq2 = qq * qq;
  return k.cub_a2 * (1.0f + (0.75f * qq - 1.5f) * wqq2);
}
inline float CubicFac(const SphConstants& k, float rr2) {
  const float rad = std::sqrt(rr2);
  const float qq = rad / k.kernelh;
  if (rad > k.kernelh) {
    const float wqq1 = 2.0f - qq;
    const float wqq2 = wqq1 * wqq1;
    return k.cub_c2 * wqq2 / rad;
  }
  const float wqq2 = qq * qq;
  return (k.cub_c1 * qq + k.cub_d1 * wqq2) / rad;
}
inline float CubicWabFac(const SphConstants& k, float rr2, float& fac) {
  fac = CubicFac(k, rr2);
  return CubicWab(k, rr2);
}
inline float CubicTensil(const SphConstants& k, float rr2, float rhopp1, float pressp1, float rhopp2, float pressp2) {
  const float wab = CubicWab(k, rr2);
  float fab = wab * k.cub_od_wdeltap;
  fab *= fab;
  fab *= fab;
  const float tensilp1 = (pressp1 / (rhopp1 * rhopp1)) * (pressp1 > 0 ? 0.01f : -0.2f);
  const float tensilp2 = (pressp2 / (rhopp2 * rhopp2)) * (pressp2 > 0 ? 0.01f : -0.2f);
  return fab * (tensilp1 + tensilp2);
}
// GetKernel_Fac / GetKernel_WabFac<tker> (FunSphKernel.h:284-296), tker = TKernel.
inline float KernelFac(const SphConstants& k, float rr2) {
  return k.kernel == SPH_KERNEL_CUBIC ? CubicFac(k, rr2) : WendlandFac(k, rr2);
}
inline float KernelWabFac(const SphConstants& k, float rr2, float& fac) {
  return k.kernel == SPH_KERNEL_CUBIC ? CubicWabFac(k, rr2, fac) : WendlandWabFac(k, rr2, fac);
}
inline float ComputePress(float rhop, const SphConstants& k) {
  return float(double(k.cteb) * (scalar_pow(double(rhop * k.ovrhopzero), double(k.gamma)) - 1.0f));
}

constexpr float ALMOSTZERO = 1e-18f;  // DualSphDef.h:132

// Divide data for the neighbour search (StDivDataCpu, JCellDivDataCpu.h:26-71).
struct DivData {
  int scelldiv;
  int ncx, ncy, ncz, nsheet;
  u3 cellzero;
  unsigned cellfluid;
  const unsigned* begincell;
  unsigned domcellcode;
  float scell;
  d3 domposmin;
};
// nsearch::Init / ParticleRange (JCellSearch_inline.h:33-82).
struct NgSearch { int cellinit, cxini, cxfin, yini, yfin, zini, zfin; };
inline NgSearch NgInit(unsigned rcell, bool boundp2, const DivData& d) {
  const int cx = int(DcelCellx(d.domcellcode, rcell)) - int(d.cellzero.x);
  const int cy = int(DcelCelly(d.domcellcode, rcell)) - int(d.cellzero.y);
  const int cz = int(DcelCellz(d.domcellcode, rcell)) - int(d.cellzero.z);
  NgSearch r;
  r.cellinit = (boundp2 ? 0 : int(d.cellfluid));
  r.cxini = cx - (cx < d.scelldiv ? cx : d.scelldiv);
  r.cxfin = cx + (d.ncx - cx - 1 < d.scelldiv ? d.ncx - cx - 1 : d.scelldiv) + 1;
  r.yini = cy - (cy < d.scelldiv ? cy : d.scelldiv);
  r.yfin = cy + (d.ncy - cy - 1 < d.scelldiv ? d.ncy - cy - 1 : d.scelldiv) + 1;
  r.zini = cz - (cz < d.scelldiv ? cz : d.scelldiv);
  r.zfin = cz + (d.ncz - cz - 1 < d.scelldiv ? d.ncz - cz - 1 : d.scelldiv) + 1;
  return r;
}
// nsearch::Init by position (JCellSearch_inline.h:52-67).
inline NgSearch NgInitPos(const d3& ps, bool boundp2, const DivData& d) {
  const int cx = int((ps.x - d.domposmin.x) / d.scell) - int(d.cellzero.x);
  const int cy = int((ps.y - d.domposmin.y) / d.scell) - int(d.cellzero.y);
  const int cz = int((ps.z - d.domposmin.z) / d.scell) - int(d.cellzero.z);
  NgSearch r;
  r.cellinit = (boundp2 ? 0 : int(d.cellfluid));
  r.cxini = cx - (cx < d.scelldiv ? cx : d.scelldiv);
  r.cxfin = cx + (d.ncx - cx - 1 < d.scelldiv ? d.ncx - cx - 1 : d.scelldiv) + 1;
  r.yini = cy - (cy < d.scelldiv ? cy : d.scelldiv);
  r.yfin = cy + (d.ncy - cy - 1 < d.scelldiv ? d.ncy - cy - 1 : d.scelldiv) + 1;
  r.zini = cz - (cz < d.scelldiv ? cz : d.scelldiv);
  r.zfin = cz + (d.ncz - cz - 1 < d.scelldiv ? d.ncz - cz - 1 : d.scelldiv) + 1;
  return r;
}
// tmatrix4d (TypesDef.h) and fmath::Determinant4x4 / InverseMatrix4x4 for doubles
// (FunctionsMath.h:186-199, 260-282).
struct m4d { double a11, a12, a13, a14, a21, a22, a23, a24, a31, a32, a33, a34, a41, a42, a43, a44; };
inline double Determinant4x4(const m4d& d) {
  return (d.a14 * d.a23 * d.a32 * d.a41 - d.a13 * d.a24 * d.a32 * d.a41 -
          d.a14 * d.a22 * d.a33 * d.a41 + d.a12 * d.a24 * d.a33 * d.a41 +
          d.a13 * d.a22 * d.a34 * d.a41 - d.a12 * d.a23 * d.a34 * d.a41 -
          d.a14 * d.a23 * d.a31 * d.a42 + d.a13 * d.a24 * d.a31 * d.a42 +
          d.a14 * d.a21 * d.a33 * d.a42 - d.a11 * d.a24 * d.a33 * d.a42 -
          d.a13 * d.a21 * d.a34 * d.a42 + d.a11 * d.a23 * d.a34 * d.a42 +
          d.a14 * d.a22 * d.a31 * d.a43 - d.a12 * d.a24 * d.a31 * d.a43 -
          d.a14 * d.a21 * d.a32 * d.a43 + d.a11 * d.a24 * d.a32 * d.a43 +
          d.a12 * d.a21 * d.a34 * d.a43 - d.a11 * d.a22 * d.a34 * d.a43 -
          d.a13 * d.a22 * d.a31 * d.a44 + d.a12 * d.a23 * d.a31 * d.a44 +
          d.a13 * d.a21 * d.a32 * d.a44 - d.a11 * d.a23 * d.a32 * d.a44 -
          d.a12 * d.a21 * d.a33 * d.a44 + d.a11 * d.a22 * d.a33 * d.a44);
}
// The rows of the inverse that the density extrapolation reads (a11..a14, a21..a24,
// a31..a34, a41..a44), each the cofactor expression of FunctionsMath.h:263-278 / det.
inline m4d InverseMatrix4x4(const m4d& d, double det) {
  m4d inv{};
  if (det) {
    inv.a11 = (d.a22 * (d.a33 * d.a44 - d.a34 * d.a43) + d.a23 * (d.a34 * d.a42 - d.a32 * d.a44) + d.a24 * (d.a32 * d.a43 - d.a33 * d.a42)) / det;
    inv.a21 = (d.a21 * (d.a34 * d.a43 - d.a33 * d.a44) + d.a23 * (d.a31 * d.a44 - d.a34 * d.a41) + d.a24 * (d.a33 * d.a41 - d.a31 * d.a43)) / det;
    inv.a31 = (d.a21 * (d.a32 * d.a44 - d.a34 * d.a42) + d.a22 * (d.a34 * d.a41 - d.a31 * d.a44) + d.a24 * (d.a31 * d.a42 - d.a32 * d.a41)) / det;
    inv.a41 = (d.a21 * (d.a33 * d.a42 - d.a32 * d.a43) + d.a22 * (d.a31 * d.a43 - d.a33 * d.a41) + d.a23 * (d.a32 * d.a41 - d.a31 * d.a42)) / det;
    inv.a12 = (d.a12 * (d.a34 * d.a43 - d.a33 * d.a44) + d.a13 * (d.a32 * d.a44 - d.a34 * d.a42) + d.a14 * (d.a33 * d.a42 - d.a32 * d.a43)) / det;
    inv.a22 = (d.a11 * (d.a33 * d.a44 - d.a34 * d.a43) + d.a13 * (d.a34 * d.a41 - d.a31 * d.a44) + d.a14 * (d.a31 * d.a43 - d.a33 * d.a41)) / det;
    inv.a32 = (d.a11 * (d.a34 * d.a42 - d.a32 * d.a44) + d.a12 * (d.a31 * d.a44 - d.a34 * d.a41) + d.a14 * (d.a32 * d.a41 - d.a31 * d.a42)) / det;
    inv.a42 = (d.a11 * (d.a32 * d.a43 - d.a33 * d.a42) + d.a12 * (d.a33 * d.a41 - d.a31 * d.a43) + d.a13 * (d.a31 * d.a42 - d.a32 * d.a41)) / det;
    inv.a13 = (d.a12 * (d.a23 * d.a44 - d.a24 * d.a43) + d.a13 * (d.a24 * d.a42 - d.a22 * d.a44) + d.a14 * (d.a22 * d.a43 - d.a23 * d.a42)) / det;
    inv.a23 = (d.a11 * (d.a24 * d.a43 - d.a23 * d.a44) + d.a13 * (d.a21 * d.a44 - d.a24 * d.a41) + d.a14 * (d.a23 * d.a41 - d.a21 * d.a43)) / det;
    inv.a33 = (d.a11 * (d.a22 * d.a44 - d.a24 * d.a42) + d.a12 * (d.a24 * d.a41 - d.a21 * d.a44) + d.a14 * (d.a21 * d.a42 - d.a22 * d.a41)) / det;
    inv.a43 = (d.a11 * (d.a23 * d.a42 - d.a22 * d.a43) + d.a12 * (d.a21 * d.a43 - d.a23 * d.a41) + d.a13 * (d.a22 * d.a41 - d.a21 * d.a42)) / det;
    inv.a14 = (d.a12 * (d.a24 * d.a33 - d.a23 * d.a34) + d.a13 * (d.a22 * d.a34 - d.a24 * d.a32) + d.a14 * (d.a23 * d.a32 - d.a22 * d.a33)) / det;
    inv.a24 = (d.a11 * (d.a23 * d.a34 - d.a24 * d.a33) + d.a13 * (d.a24 * d.a31 - d.a21 * d.a34) + d.a14 * (d.a21 * d.a33 - d.a23 * d.a31)) / det;
    inv.a34 = (d.a11 * (d.a24 * d.a32 - d.a22 * d.a34) + d.a12 * (d.a21 * d.a34 - d.a24 * d.a31) + d.a14 * (d.a22 * d.a31 - d.a21 * d.a32)) / det;
    inv.a44 = (d.a11 * (d.a22 * d.a33 - d.a23 * d.a32) + d.a12 * (d.a23 * d.a31 - d.a21 * d.a33) + d.a13 * (d.a21 * d.a32 - d.a22 * d.a31)) / det;
  }
  return inv;
}
inline void NgRange(int y, int z, const NgSearch& g, const DivData& d, unsigned& pini, unsigned& pfin) {
  const int v = d.nsheet * z + d.ncx * y + g.cellinit;
  pini = d.begincell[v + g.cxini];
  pfin = d.begincell[v + g.cxfin];
}

class Solver {
 public:
  SphConstants K;
  bool celldomfixed = false;
  int nthreads = 1;
  // particle state (JSphCpu: Idpc, Codec, Dcellc, Posc, Velrhopc, VelrhopM1c, PosPrec, VelrhopPrec)
  unsigned np = 0, npb = 0, npbok = 0, capacity = 0;
  std::vector<unsigned> idp, dcell;
  std::vector<typecode> code;
  std::vector<d3> pos, pospre;
  std::vector<f4> velrhop, velrhopm1, velrhoppre;
  std::vector<f3> boundnormal;  // BoundNormalc (mDBC): particle -> ghost node after ConfigBoundNormals
  bool mdbc = false;
  bool havepre = false;
  // interaction scratch
  std::vector<float> ar, delta, press;
  std::vector<f3> ace;
  double velmax = 0, acemax = 0;
  float viscdtmax = 0;
  // stepping
  int verletstep = 0;
  double symdtpre = 0, timestep = 0, lastdt = 0;
  uint64_t nstep = 0;
  unsigned dtmodif = 0, nout = 0;
  std::vector<double> dttrace;
  double runseconds = 0;
  // ---- JCellDivCpuSingle state ----
  u3 domcells{};
  bool boundlimitok = false, bounddivideok = false;
  u3 boundlimitmin{}, boundlimitmax{}, bounddividemin{}, bounddividemax{};
  u3 celldomainmin{}, celldomainmax{};
  unsigned ncx = 0, ncy = 0, ncz = 0, nsheet = 0, nct = 0;
  size_t nctt = 0;
  unsigned boxboundignore = 0, boxfluid = 0, boxboundout = 0, boxfluidout = 0, boxboundoutignore = 0, boxfluidoutignore = 0;
  bool dividefull = false;
  bool boundchanged = true;  // JSph::BoundChanged: true at ConfigDomain, false after each divide
  unsigned npbfinal = 0, npfinal = 0, nptot = 0;
  std::vector<unsigned> begincell, partsincell, cellpart, sortpart;

  void Init(const SphCaseDef& c, const SphParticlesHost& h, int nth) {
    Derive(c, K);
    celldomfixed = c.celldomfixed != 0;
    nthreads = nth > 0 ? nth : std::max(1, std::min(omp_get_num_procs(), 64));  // OMP_MAXTHREADS=64 (OmpDefs.h:39)
    np = h.n;
    npb = c.npb;
    npbok = npb;
    capacity = np;
    idp.assign(h.idp, h.idp + np);
    pos.resize(np);
    velrhop.resize(np);
    code.resize(np);
    dcell.resize(np);
    for (unsigned p = 0; p < np; p++) {
      pos[p] = d3{h.pos[3 * p], h.pos[3 * p + 1], h.pos[3 * p + 2]};
      velrhop[p] = f4{h.vel[3 * p], h.vel[3 * p + 1], h.vel[3 * p + 2], h.rhop[p]};
      // LoadCodeParticles (JSph.cpp:1257): fixed boundary mk block -> type fixed, fluid -> type fluid.
      code[p] = (p < npb ? typecode(0) : CODE_TYPE_FLUID);
    }
    domcells = u3{K.dom_cells[0], K.dom_cells[1], K.dom_cells[2]};
    // JSph::CheckRhopLimits (JSph.cpp:2021-2030).
    for (unsigned p = npb; p < np; p++)
      if (velrhop[p].w < K.rhopoutmin || K.rhopoutmax < velrhop[p].w)
        throw std::runtime_error("Initial fluid density is out of limits.");
    // JSph::LoadBoundNormals + ConfigBoundNormals (JSph.cpp:1265-1340): the file's
    // normals (boundary -> boundary limit) as float, doubled (boundary -> ghost node).
    mdbc = (K.tboundary == SPH_BOUND_MDBC);
    if (mdbc) {
      if (!h.boundnormal) throw std::runtime_error("mDBC needs the boundary normals (<case>_Normals.nbi4)");
      boundnormal.assign(np, f3{0, 0, 0});
      unsigned nerr = 0;
      for (unsigned p = 0; p < np; p++)
        if (idp[p] < c.npb) {
          const f3 n{h.boundnormal[3 * p], h.boundnormal[3 * p + 1], h.boundnormal[3 * p + 2]};
          if (n.x == 0 && n.y == 0 && n.z == 0) nerr++;
          boundnormal[p] = f3{n.x * 2.f, n.y * 2.f, n.z * 2.f};
        }
      if (nerr == c.npb) throw std::runtime_error("No valid normal vectors for using mDBC.");
    }
    // JSph::LoadDcellParticles (JSph.cpp:1690-1711), DomRealPos = MapRealPos (single domain).
    for (unsigned p = 0; p < np; p++) {
      const d3 ps = pos[p];
      const double dx = ps.x - K.dom_posmin[0], dy = ps.y - K.dom_posmin[1], dz = ps.z - K.dom_posmin[2];
      if (dx >= 0 && dy >= 0 && dz >= 0 && dx < K.map_realsize[0] && dy < K.map_realsize[1] && dz < K.map_realsize[2]) {
        dcell[p] = DcelCell(K.dom_cellcode, unsigned(dx / K.scell), unsigned(dy / K.scell), unsigned(dz / K.scell));
      } else {
        throw std::runtime_error("Found new particles out.");
      }
    }
    omp_set_num_threads(nthreads);
    // ConfigDomain: BoundChanged=true; RunCellDivide(true) (JSphCpuSingle.cpp:165-166).
    boundchanged = true;
    RunCellDivide();
    // InitRunCpu (JSphCpu.cpp:419-426) + InitRun (JSph.cpp:2087-2091).
    verletstep = 0;
    if (K.step_algorithm == SPH_STEP_VERLET) velrhopm1 = velrhop;
    if (K.step_algorithm == SPH_STEP_SYMPLECTIC) symdtpre = K.dtini;
  }

  // ======================= JCellDivCpuSingle =====================================
  DivData GetDivData() const {
    DivData d;
    d.scelldiv = K.scelldiv;
    d.ncx = int(ncx); d.ncy = int(ncy); d.ncz = int(ncz); d.nsheet = int(nsheet);
    d.cellzero = celldomainmin;
    d.cellfluid = boxfluid;
    d.begincell = begincell.data();
    d.domcellcode = K.dom_cellcode;
    d.scell = K.scell;
    d.domposmin = d3{K.dom_posmin[0], K.dom_posmin[1], K.dom_posmin[2]};
    return d;
  }
  // JCellDivCpu::LimitsCellBound/LimitsCellFluid (JCellDivCpu.cpp:246-352).
  void LimitsCell(unsigned n, unsigned pini, u3& cmin, u3& cmax) const {
    cmin = u3{UINT_MAX, UINT_MAX, UINT_MAX};
    cmax = u3{0, 0, 0};
    for (unsigned p = pini; p < pini + n; p++) {
      const unsigned rcell = dcell[p];
      const unsigned cx = DcelCellx(K.dom_cellcode, rcell), cy = DcelCelly(K.dom_cellcode, rcell), cz = DcelCellz(K.dom_cellcode, rcell);
      if (CodeSpecial(code[p]) < CODE_OUTIGNORE) {
        cmin.x = std::min(cmin.x, cx); cmin.y = std::min(cmin.y, cy); cmin.z = std::min(cmin.z, cz);
        cmax.x = std::max(cmax.x, cx); cmax.y = std::max(cmax.y, cy); cmax.z = std::max(cmax.z, cz);
      }
    }
    if (cmin.x > cmax.x) { cmin = domcells; cmax = u3{0, 0, 0}; }
  }
  // JCellDivCpuSingle::CalcCellDomain + MergeMapCellBoundFluid (JCellDivCpuSingle.cpp:45-96).
  void CalcCellDomain(unsigned npb1, unsigned npf1) {
    if (celldomfixed) {
      celldomainmin = u3{0, 0, 0};
      celldomainmax = u3{domcells.x - 1, domcells.y - 1, domcells.z - 1};
      if (!boundlimitok) { boundlimitok = true; boundlimitmin = celldomainmin; boundlimitmax = celldomainmax; }
      return;
    }
    u3 bmin, bmax;
    if (!boundlimitok) {
      LimitsCell(npb1, 0, bmin, bmax);
      boundlimitok = true; boundlimitmin = bmin; boundlimitmax = bmax;
    } else { bmin = boundlimitmin; bmax = boundlimitmax; }
    u3 fmin, fmax;
    LimitsCell(npf1, npb1, fmin, fmax);
    const unsigned sd = unsigned(K.scelldiv);
    auto lo = [&](unsigned b, unsigned f) { return std::max(std::min(b, f), (f >= sd ? f - sd : 0u)); };
    auto hi = [&](unsigned b, unsigned f) { return std::min(std::max(b, f), f + sd); };
    u3 cmin{lo(bmin.x, fmin.x), lo(bmin.y, fmin.y), lo(bmin.z, fmin.z)};
    u3 cmax{hi(bmax.x, fmax.x), hi(bmax.y, fmax.y), hi(bmax.z, fmax.z)};
    if (cmax.x >= domcells.x) cmax.x = domcells.x - 1;
    if (cmax.y >= domcells.y) cmax.y = domcells.y - 1;
    if (cmax.z >= domcells.z) cmax.z = domcells.z - 1;
    if (cmin.x > cmax.x || cmin.y > cmax.y || cmin.z > cmax.z) cmin = cmax = u3{0, 0, 0};
    celldomainmin = cmin;
    celldomainmax = cmax;
  }
  // JCellDivCpuSingle::PrepareNct (JCellDivCpuSingle.cpp:105-121).
  void PrepareNct() {
    ncx = celldomainmax.x - celldomainmin.x + 1;
    ncy = celldomainmax.y - celldomainmin.y + 1;
    ncz = celldomainmax.z - celldomainmin.z + 1;
    nsheet = ncx * ncy;
    nct = nsheet * ncz;
    nctt = size_t(nct) * 2 + 5 + 1;  // SizeBeginCell (JCellDivCpu.h:141)
    boxboundignore = nct;
    boxfluid = boxboundignore + 1;
    boxboundout = boxfluid + nct;
    boxfluidout = boxboundout + 1;
    boxboundoutignore = boxfluidout + 1;
    boxfluidoutignore = boxboundoutignore + 1;
    if (begincell.size() < nctt) { begincell.assign(nctt, 0); bounddivideok = false; }
    if (partsincell.size() < nctt) partsincell.assign(nctt, 0);
  }
  unsigned CellOf(unsigned p, unsigned& cx, unsigned& cy, unsigned& cz) const {
    const unsigned rcell = dcell[p];
    cx = DcelCellx(K.dom_cellcode, rcell) - celldomainmin.x;
    cy = DcelCelly(K.dom_cellcode, rcell) - celldomainmin.y;
    cz = DcelCellz(K.dom_cellcode, rcell) - celldomainmin.z;
    return cx + cy * ncx + cz * nsheet;
  }
  // JCellDivCpuSingle::PreSortFull / MakeSortFull (JCellDivCpuSingle.cpp:134-160, 203-214).
  void PreSortFull() {
    memset(partsincell.data(), 0, sizeof(unsigned) * (nctt - 1));
    for (unsigned p = 0; p < nptot; p++) {
      unsigned cx, cy, cz;
      const unsigned cellsort = CellOf(p, cx, cy, cz);
      const typecode rcode = code[p], codetype = CodeType(rcode), codeout = CodeSpecial(rcode);
      unsigned box;
      if (codetype < CODE_TYPE_FLOATING) {
        box = (codeout < CODE_OUTIGNORE ? ((cx < ncx && cy < ncy && cz < ncz) ? cellsort : boxboundignore)
                                        : (codeout == CODE_OUTIGNORE ? boxboundoutignore : boxboundout));
      } else {
        box = (codeout <= CODE_OUTIGNORE ? (codeout < CODE_OUTIGNORE ? boxfluid + cellsort : boxfluidoutignore)
                                         : (codetype == CODE_TYPE_FLOATING ? boxboundout : boxfluidout));
      }
      cellpart[p] = box;
      partsincell[box]++;
    }
    begincell[0] = 0;
    for (size_t box = 0; box < nctt - 1; box++) begincell[box + 1] = begincell[box] + partsincell[box];
    memset(partsincell.data(), 0, sizeof(unsigned) * (nctt - 1));
    for (unsigned p = 0; p < nptot; p++) {
      const unsigned box = cellpart[p];
      sortpart[begincell[box] + partsincell[box]] = p;
      partsincell[box]++;
    }
  }
  // JCellDivCpuSingle::PreSortFluid / MakeSortFluid (JCellDivCpuSingle.cpp:173-194, 223-234).
  void PreSortFluid(unsigned npf1, unsigned pini) {
    memset(partsincell.data() + boxfluid, 0, sizeof(unsigned) * (nctt - 1 - boxfluid));
    for (unsigned p = pini; p < pini + npf1; p++) {
      unsigned cx, cy, cz;
      const unsigned cellsortfluid = boxfluid + CellOf(p, cx, cy, cz);
      const typecode rcode = code[p], codetype = CodeType(rcode), codeout = CodeSpecial(rcode);
      const unsigned box = (codeout <= CODE_OUTIGNORE ? (codeout < CODE_OUTIGNORE ? cellsortfluid : boxfluidoutignore)
                                                      : (codetype == CODE_TYPE_FLOATING ? boxboundout : boxfluidout));
      cellpart[p] = box;
      partsincell[box]++;
    }
    for (size_t box = boxfluid; box < nctt - 1; box++) begincell[box + 1] = begincell[box] + partsincell[box];
    memset(partsincell.data() + boxfluid, 0, sizeof(unsigned) * (nctt - 1 - boxfluid));
    for (unsigned p = pini; p < pini + npf1; p++) {
      const unsigned box = cellpart[p];
      sortpart[begincell[box] + partsincell[box]] = p;
      partsincell[box]++;
    }
  }
  // JCellDivCpu::SortArray (JCellDivCpu.cpp:356-452).
  template <class T> void SortArray(std::vector<T>& v) {
    std::vector<T> v2(v.size());
    const unsigned ini = (dividefull ? 0 : npbfinal);
    if (ini) std::copy(v.begin(), v.begin() + ini, v2.begin());
#pragma omp parallel for schedule(static)
    for (int p = int(ini); p < int(nptot); p++) v2[p] = v[sortpart[p]];
    v.swap(v2);
  }
  // JCellDivCpuSingle::Divide (JCellDivCpuSingle.cpp:276-344) + RunCellDivide (JSphCpuSingle.cpp:437-501).
  void RunCellDivide() {
    const unsigned npb1 = npb, npf1 = np - npb;
    nptot = npb1 + npf1;
    if (cellpart.size() < nptot) { cellpart.resize(nptot); sortpart.resize(nptot); }
    if (boundchanged) {
      boundlimitok = bounddivideok = false;
      boundlimitmin = boundlimitmax = bounddividemin = bounddividemax = u3{0, 0, 0};
    }
    CalcCellDomain(npb1, npf1);
    PrepareNct();
    auto eq = [](u3 a, u3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; };
    if (!bounddivideok || !eq(bounddividemin, celldomainmin) || !eq(bounddividemax, celldomainmax)) {
      dividefull = true;
      bounddivideok = true; bounddividemin = celldomainmin; bounddividemax = celldomainmax;
    } else dividefull = false;
    if (dividefull) PreSortFull();
    else PreSortFluid(npf1, npb1);
    auto cellsize = [&](unsigned box) { return begincell[box + 1] - begincell[box]; };
    const unsigned npbignore = cellsize(boxboundignore);
    const unsigned npbout = cellsize(boxboundout), npfout = cellsize(boxfluidout);
    const unsigned npboutignore = cellsize(boxboundoutignore), npfoutignore = cellsize(boxfluidoutignore);
    npfinal = nptot - npbout - npfout - npboutignore - npfoutignore;
    npbfinal = npb1 - npboutignore;
    if (npbout != 0) throw std::runtime_error("boundary particles were excluded (AbortBoundOut)");
    // Sort particle data (JSphCpuSingle.cpp:449-462).
    SortArray(idp);
    SortArray(code);
    SortArray(dcell);
    SortArray(pos);
    SortArray(velrhop);
    if (mdbc) SortArray(boundnormal);  // JSphCpuSingle.cpp:464-467
    if (K.step_algorithm == SPH_STEP_VERLET && !velrhopm1.empty()) SortArray(velrhopm1);
    else if (K.step_algorithm == SPH_STEP_SYMPLECTIC && havepre) { SortArray(pospre); SortArray(velrhoppre); }
    np = npfinal;
    npb = npbfinal;
    npbok = npb - npbignore;
    nout += npfout;  // excluded fluid particles go to PartsOut (JSphCpuSingle.cpp:484-496)
    boundchanged = false;  // JSphCpuSingle.cpp:500
  }

  // ======================= JSphCpu interaction ==================================
  // PreInteractionVars_Forces + PreInteraction_Forces (JSphCpu.cpp:432-479).
  void PreInteraction() {
    ar.assign(np, 0.f);
    ace.assign(np, f3{0, 0, 0});
    delta.assign(np, 0.f);  // DDTArray=(TDensity!=DDT_None && Cpu) (JSph.cpp:814)
    press.resize(np);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < int(np); p++) press[p] = ComputePress(velrhop[p].w, K);
    // CalcVelMaxOmp (JSphCpu.cpp:499-528) over fluid particles (DtAllParticles=false).
    float vmax = 0;
    for (unsigned p = npb; p < np; p++) {
      const f4 v = velrhop[p];
      const float v2 = v.x * v.x + v.y * v.y + v.z * v.z;
      if (vmax < v2) vmax = v2;
    }
    velmax = std::sqrt(vmax);
    viscdtmax = 0;
  }

  // InteractionForcesFluid<Wendland,FTMODE_None,VISCO_Artificial,tdensity,false> (JSphCpu.cpp:631-822).
  template <int tdensity>
  void InteractionForcesFluid(bool boundp2, float visco, const DivData& dv, float& viscdt) {
    float viscth[64 * 16] = {0};
    const int pini = int(npb), pfin = int(np);
    const float massp2 = (boundp2 ? K.massbound : K.massfluid);
    const float cbar = float(K.cs0);
#pragma omp parallel for schedule(guided)
    for (int p1 = pini; p1 < pfin; p1++) {
      float visc = 0, arp1 = 0, deltap1 = 0;
      f3 acep1{0, 0, 0};
      const d3 posp1 = pos[p1];
      const f3 velp1{velrhop[p1].x, velrhop[p1].y, velrhop[p1].z};
      const float rhopp1 = velrhop[p1].w;
      const float pressp1 = press[p1];
      const bool rsymp1 = (K.symmetry && posp1.y <= K.kernelsize);  // JSphCpu.cpp:671
      const NgSearch g = NgInit(dcell[p1], boundp2, dv);
      for (int z = g.zini; z < g.zfin; z++)
        for (int y = g.yini; y < g.yfin; y++) {
          unsigned pif, pfi;
          NgRange(y, z, g, dv, pif, pfi);
          // Symmetry (JSphCpu.cpp:680-684, 709, 793-796): a p2 within the support radius
          // whose y is within it too is visited a second time as its image across y = 0
          bool rsym = false;
          for (unsigned p2 = pif; p2 < pfi; p2++) {
            const float drx = float(posp1.x - pos[p2].x);
            float dry = float(posp1.y - pos[p2].y);
            if (rsym) dry = float(posp1.y + pos[p2].y);
            const float drz = float(posp1.z - pos[p2].z);
            const float rr2 = drx * drx + dry * dry + drz * drz;
            if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) {
              const float fac = KernelFac(K, rr2);
              const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
              f4 velrhop2 = velrhop[p2];
              if (rsym) velrhop2.y = -velrhop2.y;
              {  // Momentum (JSphCpu.cpp:712-716).
                const float prs = (pressp1 + press[p2]) / (rhopp1 * velrhop2.w) +
                                  (K.kernel == SPH_KERNEL_CUBIC
                                       ? CubicTensil(K, rr2, rhopp1, pressp1, velrhop2.w, press[p2])
                                       : 0);
                const float p_vpm = -prs * massp2;
                acep1.x += p_vpm * frx; acep1.y += p_vpm * fry; acep1.z += p_vpm * frz;
              }
              // Continuity (JSphCpu.cpp:719-720).
              const float dvx = velp1.x - velrhop2.x, dvy = velp1.y - velrhop2.y, dvz = velp1.z - velrhop2.z;
              arp1 += massp2 * (dvx * frx + dvy * fry + dvz * frz) * (rhopp1 / velrhop2.w);
              // DDT Molteni & Colagrossi (JSphCpu.cpp:724-731).
              if (tdensity == SPH_DDT_DDT && deltap1 != FLT_MAX) {
                const float rhop1over2 = rhopp1 / velrhop2.w;
                const float visc_densi = K.ddtkh * cbar * (rhop1over2 - 1.f) / (rr2 + K.eta2);
                const float dot3 = (drx * frx + dry * fry + drz * frz);
                const float delta_ = visc_densi * dot3 * massp2;
                deltap1 = (boundp2 && !mdbc ? FLT_MAX : deltap1 + delta_);  // TBoundary==BC_DBC
              }
              // DDT Fourtakas (JSphCpu.cpp:733-740).
              if ((tdensity == SPH_DDT_DDT2 || (tdensity == SPH_DDT_DDT2FULL && !boundp2)) && deltap1 != FLT_MAX) {
                const float rh = 1.f + K.ddtgz * drz;
                const float drhop = K.rhopzero * std::pow(rh, 1.f / K.gamma) - K.rhopzero;
                const float visc_densi = K.ddtkh * cbar * ((velrhop2.w - rhopp1) - drhop) / (rr2 + K.eta2);
                const float dot3 = (drx * frx + dry * fry + drz * frz);
                const float delta_ = visc_densi * dot3 * massp2 / velrhop2.w;
                deltap1 = (boundp2 ? FLT_MAX : deltap1 - delta_);
              }
              // Artificial viscosity (JSphCpu.cpp:753-764).
              {
                const float dot = drx * dvx + dry * dvy + drz * dvz;
                const float dot_rr2 = dot / (rr2 + K.eta2);
                visc = std::max(dot_rr2, visc);
                if (dot < 0) {
                  const float amubar = K.kernelh * dot_rr2;
                  const float robar = (rhopp1 + velrhop2.w) * 0.5f;
                  const float pi_visc = (-visco * cbar * amubar / robar) * massp2;
                  acep1.x -= pi_visc * frx; acep1.y -= pi_visc * fry; acep1.z -= pi_visc * frz;
                }
              }
              rsym = (rsymp1 && !rsym && float(posp1.y - dry) <= K.kernelsize);
              if (rsym) p2--;
            } else {
              rsym = false;
            }
          }
        }
      // Store (JSphCpu.cpp:800-818), DDTArray path.
      if (arp1 || acep1.x || acep1.y || acep1.z || visc) {
        if (tdensity != SPH_DDT_NONE) {
          delta[p1] = (delta[p1] == FLT_MAX || deltap1 == FLT_MAX ? FLT_MAX : delta[p1] + deltap1);
        }
        ar[p1] += arp1;
        ace[p1] = f3{ace[p1].x + acep1.x, ace[p1].y + acep1.y, ace[p1].z + acep1.z};
        const int th = omp_get_thread_num();
        if (visc > viscth[th * 16]) viscth[th * 16] = visc;
      }
    }
    for (int th = 0; th < 64; th++) if (viscdt < viscth[th * 16]) viscdt = viscth[th * 16];
  }

  // InteractionForcesBound<Wendland,FTMODE_None> (JSphCpu.cpp:548-625).
  void InteractionForcesBound(const DivData& dv, float& viscdt) {
    float viscth[64 * 16] = {0};
    const int pfin = int(npbok);
    const float massp2 = K.massfluid;
#pragma omp parallel for schedule(guided)
    for (int p1 = 0; p1 < pfin; p1++) {
      float visc = 0, arp1 = 0;
      const d3 posp1 = pos[p1];
      const f4 velrhop1 = velrhop[p1];
      const bool rsymp1 = (K.symmetry && posp1.y <= K.kernelsize);  // JSphCpu.cpp:566
      const NgSearch g = NgInit(dcell[p1], false, dv);
      for (int z = g.zini; z < g.zfin; z++)
        for (int y = g.yini; y < g.yfin; y++) {
          unsigned pif, pfi;
          NgRange(y, z, g, dv, pif, pfi);
          bool rsym = false;  // Symmetry (JSphCpu.cpp:576-580, 600, 610-613)
          for (unsigned p2 = pif; p2 < pfi; p2++) {
            const float drx = float(posp1.x - pos[p2].x);
            float dry = float(posp1.y - pos[p2].y);
            if (rsym) dry = float(posp1.y + pos[p2].y);
            const float drz = float(posp1.z - pos[p2].z);
            const float rr2 = drx * drx + dry * dry + drz * drz;
            if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) {
              const float fac = KernelFac(K, rr2);
              const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
              f4 velrhop2 = velrhop[p2];
              if (rsym) velrhop2.y = -velrhop2.y;
              const float dvx = velrhop1.x - velrhop2.x, dvy = velrhop1.y - velrhop2.y, dvz = velrhop1.z - velrhop2.z;
              arp1 += massp2 * (dvx * frx + dvy * fry + dvz * frz) * (velrhop1.w / velrhop2.w);
              const float dot = drx * dvx + dry * dvy + drz * dvz;
              const float dot_rr2 = dot / (rr2 + K.eta2);
              visc = std::max(dot_rr2, visc);
              rsym = (rsymp1 && !rsym && float(posp1.y - dry) <= K.kernelsize);
              if (rsym) p2--;
            } else {
              rsym = false;
            }
          }
        }
      if (arp1 || visc) {
        ar[p1] += arp1;
        const int th = omp_get_thread_num();
        if (visc > viscth[th * 16]) viscth[th * 16] = visc;
      }
    }
    for (int th = 0; th < 64; th++) if (viscdt < viscth[th * 16]) viscdt = viscth[th * 16];
  }

  // JSphCpuSingle::Interaction_Forces (JSphCpuSingle.cpp:524-567) + Interaction_ForcesCpuT (JSphCpu.cpp:960-987).
  template <int tdensity> void InteractionT(float& viscdt) {
    const DivData dv = GetDivData();
    if (np > npb) {
      InteractionForcesFluid<tdensity>(false, K.visco, dv, viscdt);
      InteractionForcesFluid<tdensity>(true, K.visco * K.viscoboundfactor, dv, viscdt);
    }
    if (npbok) InteractionForcesBound(dv, viscdt);
    // For 2-D simulations zero the 2nd component (JSphCpuSingle.cpp:544-549).
    if (K.data2d)
      for (unsigned p = npb; p < np; p++) ace[p].y = 0;
  }
  // JSphCpu::InteractionMdbcCorrectionT2<Wendland,sim2d,SLIP_Vel0> (JSphCpu.cpp:1020-1187)
  // over n = NpbOk boundary particles (UseNormalsFt=false; JSphCpu.cpp:1193-1210).
  void MdbcCorrection() {
    const DivData dv = GetDivData();
    const float determlimit = 1e-3f;
    const float mdbcthreshold = K.mdbc_threshold;
    const int nn = int(npbok);
#pragma omp parallel for schedule(guided)
    for (int p1 = 0; p1 < nn; p1++) {
      const f3 bn = boundnormal[p1];
      if (bn.x == 0 && bn.y == 0 && bn.z == 0) continue;
      float rhopfinal = FLT_MAX;
      float sumwab = 0;
      const d3 gposp1{pos[p1].x + double(bn.x), pos[p1].y + double(bn.y), pos[p1].z + double(bn.z)};
      float rhopp1 = 0;
      f3 gradrhopp1{0, 0, 0};
      m4d a{};
      const NgSearch g = NgInitPos(gposp1, false, dv);
      for (int z = g.zini; z < g.zfin; z++)
        for (int y = g.yini; y < g.yfin; y++) {
          unsigned pif, pfi;
          NgRange(y, z, g, dv, pif, pfi);
          for (unsigned p2 = pif; p2 < pfi; p2++) {
            const float drx = float(gposp1.x - pos[p2].x);
            const float dry = float(gposp1.y - pos[p2].y);
            const float drz = float(gposp1.z - pos[p2].z);
            const float rr2 = (drx * drx + dry * dry + drz * drz);
            if (rr2 <= K.kernelsize2 && CodeIsFluid(code[p2])) {
              float fac;
              const float wab = KernelWabFac(K, rr2, fac);
              const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
              const f4 velrhopp2 = velrhop[p2];
              const float massp2 = K.massfluid;
              const float volp2 = massp2 / velrhopp2.w;
              rhopp1 += massp2 * wab;
              gradrhopp1.x += massp2 * frx;
              gradrhopp1.y += massp2 * fry;
              gradrhopp1.z += massp2 * frz;
              const float vwab = wab * volp2;
              sumwab += vwab;
              const float vfrx = frx * volp2, vfry = fry * volp2, vfrz = frz * volp2;
              if (K.data2d) {  // a_corr2 (JSphCpu.cpp:1087-1091), kept in the a11..a33 slots
                a.a11 += vwab;  a.a12 += drx * vwab;  a.a13 += drz * vwab;
                a.a21 += vfrx;  a.a22 += drx * vfrx;  a.a23 += drz * vfrx;
                a.a31 += vfrz;  a.a32 += drx * vfrz;  a.a33 += drz * vfrz;
              } else {
                a.a11 += vwab;  a.a12 += drx * vwab;  a.a13 += dry * vwab;  a.a14 += drz * vwab;
                a.a21 += vfrx;  a.a22 += drx * vfrx;  a.a23 += dry * vfrx;  a.a24 += drz * vfrx;
                a.a31 += vfry;  a.a32 += drx * vfry;  a.a33 += dry * vfry;  a.a34 += drz * vfry;
                a.a41 += vfrz;  a.a42 += drx * vfrz;  a.a43 += dry * vfrz;  a.a44 += drz * vfrz;
              }
            }
          }
        }
      if (sumwab >= mdbcthreshold || (mdbcthreshold >= 2 && sumwab + 2 >= mdbcthreshold)) {
        const f3 dpos{bn.x * (-1.f), bn.y * (-1.f), bn.z * (-1.f)};
        if (K.data2d) {  // JSphCpu.cpp:1094-1110 (fmath::Determinant3x3 / InverseMatrix3x3)
          const double d3 = a.a11 * a.a22 * a.a33 + a.a12 * a.a23 * a.a31 + a.a13 * a.a21 * a.a32 -
                            a.a31 * a.a22 * a.a13 - a.a32 * a.a23 * a.a11 - a.a33 * a.a21 * a.a12;
          if (std::fabs(d3) >= determlimit) {
            const double i11 = (a.a22 * a.a33 - a.a23 * a.a32) / d3, i12 = -(a.a12 * a.a33 - a.a13 * a.a32) / d3;
            const double i13 = (a.a12 * a.a23 - a.a13 * a.a22) / d3, i21 = -(a.a21 * a.a33 - a.a23 * a.a31) / d3;
            const double i22 = (a.a11 * a.a33 - a.a13 * a.a31) / d3, i23 = -(a.a11 * a.a23 - a.a13 * a.a21) / d3;
            const double i31 = (a.a21 * a.a32 - a.a22 * a.a31) / d3, i32 = -(a.a11 * a.a32 - a.a12 * a.a31) / d3;
            const double i33 = (a.a11 * a.a22 - a.a12 * a.a21) / d3;
            const float rhoghost = float(i11 * rhopp1 + i12 * gradrhopp1.x + i13 * gradrhopp1.z);
            const float grx = -float(i21 * rhopp1 + i22 * gradrhopp1.x + i23 * gradrhopp1.z);
            const float grz = -float(i31 * rhopp1 + i32 * gradrhopp1.x + i33 * gradrhopp1.z);
            rhopfinal = (rhoghost + grx * dpos.x + grz * dpos.z);
          } else if (a.a11 > 0) {
            rhopfinal = float(rhopp1 / a.a11);
          }
          rhopfinal = (rhopfinal != FLT_MAX ? rhopfinal : K.rhopzero);
          velrhop[p1].w = rhopfinal;
          continue;
        }
        const double determ = Determinant4x4(a);
        if (std::fabs(determ) >= determlimit) {
          const m4d inv = InverseMatrix4x4(a, determ);
          const float rhoghost = float(inv.a11 * rhopp1 + inv.a12 * gradrhopp1.x + inv.a13 * gradrhopp1.y + inv.a14 * gradrhopp1.z);
          const float grx = -float(inv.a21 * rhopp1 + inv.a22 * gradrhopp1.x + inv.a23 * gradrhopp1.y + inv.a24 * gradrhopp1.z);
          const float gry = -float(inv.a31 * rhopp1 + inv.a32 * gradrhopp1.x + inv.a33 * gradrhopp1.y + inv.a34 * gradrhopp1.z);
          const float grz = -float(inv.a41 * rhopp1 + inv.a42 * gradrhopp1.x + inv.a43 * gradrhopp1.y + inv.a44 * gradrhopp1.z);
          rhopfinal = (rhoghost + grx * dpos.x + gry * dpos.y + grz * dpos.z);
        } else if (a.a11 > 0) {
          rhopfinal = float(rhopp1 / a.a11);
        }
        rhopfinal = (rhopfinal != FLT_MAX ? rhopfinal : K.rhopzero);
        velrhop[p1].w = rhopfinal;  // SLIP_Vel0
      }
    }
  }

  // JSphCpuSingle::Interaction_Forces (JSphCpuSingle.cpp:524-567): mDBC correction first,
  // except in the Symplectic corrector (MDBCCorrector=0).
  void Interaction_Forces(int interstep = 1) {
    if (mdbc && interstep != 3) MdbcCorrection();
    PreInteraction();
    float viscdt = 0;
    switch (K.tdensity) {
      case SPH_DDT_NONE: InteractionT<SPH_DDT_NONE>(viscdt); break;
      case SPH_DDT_DDT: InteractionT<SPH_DDT_DDT>(viscdt); break;
      case SPH_DDT_DDT2: InteractionT<SPH_DDT_DDT2>(viscdt); break;
      case SPH_DDT_DDT2FULL: InteractionT<SPH_DDT_DDT2FULL>(viscdt); break;
      default: throw std::runtime_error("invalid tdensity");
    }
    // Delta-SPH correction added to Ar (JSphCpuSingle.cpp:553-559).
    if (K.tdensity != SPH_DDT_NONE)
      for (unsigned p = npb; p < np; p++) if (delta[p] != FLT_MAX) ar[p] += delta[p];
    viscdtmax = viscdt;
    // ComputeAceMaxOmp<false> (JSphCpuSingle.cpp:612-644).
    float amax = 0;
    for (unsigned p = npb; p < np; p++) {
      const f3 a = ace[p];
      const float a2 = a.x * a.x + a.y * a.y + a.z * a.z;
      if (amax < a2) amax = a2;
    }
    acemax = std::sqrt(double(amax));
  }

  // JSphCpu::DtVariable (JSphCpu.cpp:1614-1639).
  double DtVariable(bool final_) {
    const double dt1 = (acemax ? std::sqrt(double(K.kernelh) / acemax) : DBL_MAX);
    const double dt2 = double(K.kernelh) / (std::max(K.cs0, velmax * 10.) + double(K.kernelh) * viscdtmax);
    double dt = K.cflnumber * std::min(dt1, dt2);
    if (std::isnan(dt) || std::isinf(dt)) throw std::runtime_error("The computed Dt is NaN or infinity");
    if (dt < double(K.dtmin)) { dt = double(K.dtmin); dtmodif++; }
    (void)final_;
    return dt;
  }

  // JSphCpu::UpdatePos (JSphCpu.cpp:1240-1293), no periodic.
  void UpdatePos(d3 rpos, double movx, double movy, double movz, bool outrhop, unsigned p, std::vector<d3>& posv) {
    const bool outmove = (std::fabs(float(movx)) > K.movlimit || std::fabs(float(movy)) > K.movlimit || std::fabs(float(movz)) > K.movlimit);
    rpos.x += movx; rpos.y += movy; rpos.z += movz;
    if (K.symmetry && rpos.y < 0) rpos.y = -rpos.y;  // JSphCpu.cpp:1247
    const double dx = rpos.x - K.map_realposmin[0], dy = rpos.y - K.map_realposmin[1], dz = rpos.z - K.map_realposmin[2];
    const bool out = (dx != dx || dy != dy || dz != dz || dx < 0 || dy < 0 || dz < 0 ||
                      dx >= K.map_realsize[0] || dy >= K.map_realsize[1] || dz >= K.map_realsize[2]);
    posv[p] = rpos;
    if (outrhop || outmove || out) {
      typecode rcode = code[p];
      if (out) rcode = CodeSetNormal(rcode) | CODE_OUTPOS;
      else if (outrhop) rcode = CodeSetNormal(rcode) | CODE_OUTRHOP;
      else rcode = CodeSetNormal(rcode) | CODE_OUTMOVE;
      code[p] = rcode;
      dcell[p] = 0xFFFFFFFFu;
    } else {
      const unsigned cx = unsigned(dx / K.scell), cy = unsigned(dy / K.scell), cz = unsigned(dz / K.scell);
      dcell[p] = DcelCell(K.dom_cellcode, cx, cy, cz);
    }
  }

  // JSphCpu::ComputeVerletVarsFluid (JSphCpu.cpp:1300-1357).
  void ComputeVerletVarsFluid(const std::vector<f4>& vr1, const std::vector<f4>& vr2, double dt, double dt2, std::vector<f4>& vrnew) {
    const double dt205 = 0.5 * dt * dt;
    const double gx = K.gravity[0], gy = K.gravity[1], gz = K.gravity[2];
#pragma omp parallel for schedule(static)
    for (int p = int(npb); p < int(np); p++) {
      const float rhopnew = float(double(vr2[p].w) + dt2 * ar[p]);
      const double ax = double(ace[p].x) + gx, ay = double(ace[p].y) + gy, az = double(ace[p].z) + gz;
      const double dx = double(vr1[p].x) * dt + ax * dt205;
      const double dy = double(vr1[p].y) * dt + ay * dt205;
      const double dz = double(vr1[p].z) * dt + az * dt205;
      const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
      const f4 nv{float(double(vr2[p].x) + ax * dt2), float(double(vr2[p].y) + ay * dt2), float(double(vr2[p].z) + az * dt2), rhopnew};
      UpdatePos(pos[p], dx, dy, dz, outrhop, unsigned(p), pos);
      vrnew[p] = nv;
    }
  }
  // JSphCpu::ComputeVelrhopBound (JSphCpu.cpp:1366-1375).
  void ComputeVelrhopBound(const std::vector<f4>& vrold, double armul, std::vector<f4>& vrnew) {
#pragma omp parallel for schedule(static)
    for (int p = 0; p < int(npb); p++) {
      const float rhopnew = float(double(vrold[p].w) + armul * ar[p]);
      vrnew[p] = f4{0, 0, 0, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew)};
    }
  }
  // JSphCpu::ComputeVerlet (JSphCpu.cpp:1381-1399).
  void ComputeVerlet(double dt) {
    verletstep++;
    if (verletstep < K.verlet_steps) {
      const double twodt = dt + dt;
      ComputeVerletVarsFluid(velrhop, velrhopm1, dt, twodt, velrhopm1);
      ComputeVelrhopBound(velrhopm1, twodt, velrhopm1);
    } else {
      ComputeVerletVarsFluid(velrhop, velrhop, dt, dt, velrhopm1);
      ComputeVelrhopBound(velrhop, dt, velrhopm1);
      verletstep = 0;
    }
    velrhop.swap(velrhopm1);
  }
  // JSphCpu::ComputeSymplecticPre (JSphCpu.cpp:1406-1504).
  void ComputeSymplecticPre(double dt) {
    const double dt05 = dt * .5;
    pospre = pos;          // swap(PosPrec,Posc): PosPre <= Pos
    velrhoppre = velrhop;  // VelrhopPre <= Velrhop
    havepre = true;
    const double gx = K.gravity[0], gy = K.gravity[1], gz = K.gravity[2];
    for (unsigned p = 0; p < npb; p++) {
      const f4 vr = velrhoppre[p];
      const float rhopnew = float(double(vr.w) + dt05 * ar[p]);
      velrhop[p] = f4{vr.x, vr.y, vr.z, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew)};
    }
    std::vector<d3> mov(np);
#pragma omp parallel for schedule(static)
    for (int p = int(npb); p < int(np); p++) {
      const typecode rcode = code[p];
      const float rhopnew = float(double(velrhoppre[p].w) + dt05 * ar[p]);
      const double dx = double(velrhoppre[p].x) * dt05, dy = double(velrhoppre[p].y) * dt05, dz = double(velrhoppre[p].z) * dt05;
      const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
      const f4 nv{float(double(velrhoppre[p].x) + (double(ace[p].x) + gx) * dt05),
                  float(double(velrhoppre[p].y) + (double(ace[p].y) + gy) * dt05),
                  float(double(velrhoppre[p].z) + (double(ace[p].z) + gz) * dt05), rhopnew};
      mov[p] = d3{dx, dy, dz};
      velrhop[p] = nv;
      if (outrhop && CodeIsNormal(rcode)) code[p] = CodeSetNormal(rcode) | CODE_OUTRHOP;
    }
#pragma omp parallel for schedule(static)
    for (int p = int(npb); p < int(np); p++) {
      const typecode rcode = code[p];
      const bool outrhop = CodeIsOutRhop(rcode);
      if (CodeIsFluid(rcode)) UpdatePos(pospre[p], mov[p].x, mov[p].y, mov[p].z, outrhop, unsigned(p), pos);
      else pos[p] = pospre[p];
    }
    for (unsigned p = 0; p < npb; p++) pos[p] = pospre[p];
  }
  // JSphCpu::ComputeSymplecticCorr (JSphCpu.cpp:1510-1606).
  void ComputeSymplecticCorr(double dt) {
    const double dt05 = dt * .5;
    const double gx = K.gravity[0], gy = K.gravity[1], gz = K.gravity[2];
    for (unsigned p = 0; p < npb; p++) {
      const double epsilon_rdot = (-double(ar[p]) / double(velrhop[p].w)) * dt;
      const float rhopnew = float(double(velrhoppre[p].w) * (2. - epsilon_rdot) / (2. + epsilon_rdot));
      velrhop[p] = f4{0, 0, 0, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew)};
    }
    std::vector<d3> mov(np);
#pragma omp parallel for schedule(static)
    for (int p = int(npb); p < int(np); p++) {
      const typecode rcode = code[p];
      const double epsilon_rdot = (-double(ar[p]) / double(velrhop[p].w)) * dt;
      const float rhopnew = float(double(velrhoppre[p].w) * (2. - epsilon_rdot) / (2. + epsilon_rdot));
      const f4 nv{float(double(velrhoppre[p].x) + (double(ace[p].x) + gx) * dt),
                  float(double(velrhoppre[p].y) + (double(ace[p].y) + gy) * dt),
                  float(double(velrhoppre[p].z) + (double(ace[p].z) + gz) * dt), rhopnew};
      const double dx = (double(velrhoppre[p].x) + double(nv.x)) * dt05;
      const double dy = (double(velrhoppre[p].y) + double(nv.y)) * dt05;
      const double dz = (double(velrhoppre[p].z) + double(nv.z)) * dt05;
      const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
      mov[p] = d3{dx, dy, dz};
      if (outrhop && CodeIsNormal(rcode)) code[p] = CodeSetNormal(rcode) | CODE_OUTRHOP;
      velrhop[p] = nv;
    }
#pragma omp parallel for schedule(static)
    for (int p = int(npb); p < int(np); p++) {
      const typecode rcode = code[p];
      const bool outrhop = CodeIsOutRhop(rcode);
      if (CodeIsFluid(rcode)) UpdatePos(pospre[p], mov[p].x, mov[p].y, mov[p].z, outrhop, unsigned(p), pos);
      else pos[p] = pospre[p];
    }
    pospre.clear();
    velrhoppre.clear();
    havepre = false;
  }

  // JSphCpuSingle::ComputeStep_Ver (JSphCpuSingle.cpp:674-686).
  double ComputeStep_Ver() {
    Interaction_Forces();
    const double dt = DtVariable(true);
    ComputeVerlet(dt);
    return dt;
  }
  // JSphCpuSingle::ComputeStep_Sym (JSphCpuSingle.cpp:695-721).
  double ComputeStep_Sym() {
    const double dt = symdtpre;
    Interaction_Forces(2);
    const double ddt_p = DtVariable(false);
    ComputeSymplecticPre(dt);
    RunCellDivide();
    Interaction_Forces(3);
    const double ddt_c = DtVariable(true);
    ComputeSymplecticCorr(dt);
    symdtpre = std::min(ddt_p, ddt_c);
    return dt;
  }
  // Main loop body (JSphCpuSingle.cpp:1090-1100).
  void Run(unsigned nsteps) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned s = 0; s < nsteps; s++) {
      const double stepdt = (K.step_algorithm == SPH_STEP_SYMPLECTIC ? ComputeStep_Sym() : ComputeStep_Ver());
      RunCellDivide();
      timestep += stepdt;
      lastdt = stepdt;
      dttrace.push_back(stepdt);
      nstep++;
    }
    runseconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  // JDsPips::ComputeCpu-style pair counting (JDsPips.cpp:187-262).
  void CountPairs(uint64_t out[6]) const {
    const DivData dv = GetDivData();
    uint64_t c[6] = {0, 0, 0, 0, 0, 0};
    auto count = [&](unsigned p1, bool boundp2, uint64_t& chk, uint64_t& real) {
      const NgSearch g = NgInit(dcell[p1], boundp2, dv);
      for (int z = g.zini; z < g.zfin; z++)
        for (int y = g.yini; y < g.yfin; y++) {
          unsigned a, b;
          NgRange(y, z, g, dv, a, b);
          for (unsigned p2 = a; p2 < b; p2++) {
            chk++;
            const float drx = float(pos[p1].x - pos[p2].x), dry = float(pos[p1].y - pos[p2].y), drz = float(pos[p1].z - pos[p2].z);
            const float rr2 = drx * drx + dry * dry + drz * drz;
            if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) real++;
          }
        }
    };
    for (unsigned p1 = npb; p1 < np; p1++) { count(p1, false, c[0], c[1]); count(p1, true, c[2], c[3]); }
    for (unsigned p1 = 0; p1 < npbok; p1++) count(p1, false, c[4], c[5]);
    for (int i = 0; i < 6; i++) out[i] = c[i];
  }
};

template <class F> int Guard(F&& f) {
  try {
    f();
    return SPH_OK;
  } catch (const std::exception& e) {
    g_err = e.what();
    return SPH_ERR_STATE;
  }
}

}  // namespace

struct OrSolver { Solver s; };

extern "C" {

const char* or_last_error(void) { return g_err.c_str(); }

int or_case_derive(const SphCaseDef* cdef, SphConstants* out) {
  if (!cdef || !out) return SPH_ERR_ARG;
  return Guard([&] { Derive(*cdef, *out); });
}

int or_create(const SphCaseDef* cdef, const SphParticlesHost* init, int nthreads, OrSolver** out) {
  if (!cdef || !init || !out) return SPH_ERR_ARG;
  OrSolver* o = new OrSolver();
  const int r = Guard([&] { o->s.Init(*cdef, *init, nthreads); });
  if (r) { delete o; return r; }
  *out = o;
  return SPH_OK;
}

int or_destroy(OrSolver* s) { delete s; return SPH_OK; }

int or_run(OrSolver* s, uint32_t nsteps) {
  if (!s) return SPH_ERR_ARG;
  return Guard([&] { omp_set_num_threads(s->s.nthreads); s->s.Run(nsteps); });
}

int or_stats(OrSolver* o, SphRunStats* out) {
  if (!o || !out) return SPH_ERR_ARG;
  const Solver& s = o->s;
  memset(out, 0, sizeof(*out));
  out->time = s.timestep;
  out->last_dt = s.lastdt;
  out->sym_dtpre = s.symdtpre;
  out->nstep = s.nstep;
  out->np = s.np; out->npb = s.npb; out->npbok = s.npbok; out->nout = s.nout;
  out->dtmodif = s.dtmodif;
  out->velmax = float(s.velmax); out->acemax = float(s.acemax); out->viscdtmax = s.viscdtmax;
  return SPH_OK;
}

int or_dt_trace(OrSolver* o, double* out, uint32_t cap, uint32_t* count) {
  if (!o || !count) return SPH_ERR_ARG;
  const auto& t = o->s.dttrace;
  const uint32_t n = uint32_t(std::min<size_t>(cap, t.size()));
  if (out) std::copy(t.begin(), t.begin() + n, out);
  *count = uint32_t(t.size());
  return SPH_OK;
}

int or_download(OrSolver* o, SphParticlesHost* out) {
  if (!o || !out) return SPH_ERR_ARG;
  const Solver& s = o->s;
  if (out->n < s.np) { g_err = "output buffer too small"; return SPH_ERR_ARG; }
  for (unsigned p = 0; p < s.np; p++) {
    if (out->idp) out->idp[p] = s.idp[p];
    if (out->pos) { out->pos[3 * p] = s.pos[p].x; out->pos[3 * p + 1] = s.pos[p].y; out->pos[3 * p + 2] = s.pos[p].z; }
    if (out->vel) { out->vel[3 * p] = s.velrhop[p].x; out->vel[3 * p + 1] = s.velrhop[p].y; out->vel[3 * p + 2] = s.velrhop[p].z; }
    if (out->rhop) out->rhop[p] = s.velrhop[p].w;
    if (out->code) out->code[p] = s.code[p];
  }
  out->n = s.np;
  return SPH_OK;
}

int or_interaction(OrSolver* o, int interstep, SphInterOut* out) {
  if (!o || !out) return SPH_ERR_ARG;
  return Guard([&] {
    Solver& s = o->s;
    omp_set_num_threads(s.nthreads);
    s.Interaction_Forces(interstep);
    for (unsigned p = 0; p < s.np; p++) {
      if (out->ar) out->ar[p] = s.ar[p];
      if (out->ace) { out->ace[3 * p] = s.ace[p].x; out->ace[3 * p + 1] = s.ace[p].y; out->ace[3 * p + 2] = s.ace[p].z; }
    }
    out->viscdtmax = s.viscdtmax;
    out->velmax = float(s.velmax);
    out->acemax = float(s.acemax);
  });
}

int or_count_pairs(OrSolver* o, uint64_t out[6]) {
  if (!o || !out) return SPH_ERR_ARG;
  o->s.CountPairs(out);
  return SPH_OK;
}

double or_run_seconds(OrSolver* o) { return o ? o->s.runseconds : 0.0; }
int or_threads(OrSolver* o) { return o ? o->s.nthreads : 0; }

}  // extern "C"
