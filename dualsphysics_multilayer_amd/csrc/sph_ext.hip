// sph_ext.hip — single-phase Interaction_Forces with Laminar+SPS viscosity and/or shifting
// (SURVEY.md §8(f) row 4, v5.2 solver) as an LDS-tiled CDNA4 kernel.
//
// Reference: JSphCpu::InteractionForcesFluid<tker,ftmode,tvisco,tdensity,shift>
// (src/source/JSphCpu.cpp:631-822) with tvisco = VISCO_LaminarSPS (:765-791) or shift =
// true (:743-750), InteractionForcesBound (:548-625), ComputeSpsTau (:929-954) and
// Interaction_ForcesCpuT (:960-987); GPU twins KerInteractionForcesFluidBox /
// KerComputeSpsTau (JSphGpu_ker.cu:512-745, 1516).  The headline k_fluid_tiled keeps its
// algebra-folded body for artificial viscosity without shifting; this kernel evaluates the
// reference's per-pair terms as written, on the same items, LDS staging and mirrored
// drain units (sph_tiled.hpp), for the options that need more per-pair state:
//   * Laminar+SPS: the laminar term 4 visco (dr.fr)/((r^2+eta^2)(rho1+rho2)) m2 dv, the SPS
//     stress divergence m2 (tau1 + tau2).fr with the sub-particle stress tensor of the
//     PREVIOUS interaction (tau2 = 0 for a bound or floating p2), and the velocity
//     gradients of p1; at the end of each fluid p1 its new tau (ComputeSpsTau) goes to a
//     second buffer (the neighbours still read the old one), swapped by the solver;
//   * shifting: the sums shiftposfs = {sum m2/rho2 frx, ..fry, ..frz, -sum m2/rho2 dr.fr},
//     x = FLT_MAX (and every later pair skipped) next to a boundary particle under
//     ShiftMode NoBound / NoFixed or a floating particle under NoBound; those passes are
//     order-dependent and are then drained in the reference's row order.
// Floating bodies: a floating p2 carries its body's particle mass, switches the DDT off as
// in the reference (DELTA_HEAVYFLOATING), and has no SPS stress; a floating p1 gets no DDT,
// no shifting and no velocity gradient.
#include <cfloat>

#include "sph_tiled.hpp"

namespace sphx {

// Records: sA {x, y, z, |A|^2}, sB velrhop, sC {press, +-m2, tau_yz, tau_zz},
// sD {tau_xx, tau_xy, tau_xz, tau_yy} (Laminar+SPS only).  m2 < 0 flags a floating p2 in
// fluid rows and a fixed p2 in bound rows (ShiftMode NoFixed).
template <int TVISCO> struct ExtCap { static constexpr int v = 416; };   // 48-B records
template <> struct ExtCap<2> { static constexpr int v = 312; };          // 64-B records

struct ExtP1 {
  float x, y, z;
  float4 vr;
  float press;
  bool ftp1;
  float t[6];  // tau of p1 (previous interaction)
};

struct ExtAcc {
  float ax, ay, az, ar, delta, visc;
  float sx, sy, sz, sw;
  float gxx, gxy, gxz, gyy, gyz, gzz;
};

struct ExtArgs {
  const float4* poscell;
  const float4* velrhop;
  const float* press;
  const typecode* code;
  const float* ftmassp;  // particle mass per floating body (nullptr: no floating bodies)
  const float4* tau;     // Laminar+SPS: tau of the previous interaction [2 np]
};

// mir (Symmetry): the records' images across the plane y = 0 (JSphCpu.cpp:684,709): y and
// the y velocity negated; the item's frame starts at y = cy scell, so the image of a record
// at frame y is at -(y) - 2 cy scell (mirc = cy).  inl (Symmetry in a pass drained in the
// reference's order): each record followed by its image, at dst + 2 i and dst + 2 i + 1 —
// the reference visits an image right after its original (JSphCpu.cpp:793-796).
__device__ __forceinline__ void ext_stage(const KConst& K, const ExtArgs& E, unsigned rs, unsigned n, unsigned dst,
                                          int xo, int dy, int dz, bool boundrow, bool withtau,
                                          float4* __restrict__ sA, float4* __restrict__ sB, float4* __restrict__ sC,
                                          float4* __restrict__ sD, bool mir = false, int mirc = 0, bool inl = false) {
  const float oy = float(dy) * K.scell, oz = float(dz) * K.scell, my = float(2 * mirc) * K.scell;
  for (unsigned i = threadIdx.x; i < n; i += TB) {
    const unsigned q = rs + i;
    const float4 pc = E.poscell[q];
    const int cx2 = int(DcelCellx(K.domcellcode, __float_as_uint(pc.w)));
    const float x2 = pc.x + float(cx2 - xo) * K.scell;
    const float y2 = mir ? -(pc.y + oy) - my : pc.y + oy, z2 = pc.z + oz;
    const unsigned d = inl ? dst + 2 * i : dst + i;
    sA[d] = make_float4(x2, y2, z2, x2 * x2 + y2 * y2 + z2 * z2);
    float4 vr = E.velrhop[q];
    if (mir) vr.y = -vr.y;
    sB[d] = vr;
    const typecode c = E.code[q];
    float m2 = boundrow ? K.massbound : K.massfluid;
    bool flag = false, withtau2 = withtau && !boundrow;
    if (boundrow) {
      flag = CodeType(c) == 0;  // fixed
    } else if (E.ftmassp && CodeType(c) == CODE_TYPE_FLOATING) {
      m2 = E.ftmassp[c & CODE_MASKVALUE];
      flag = true;
      withtau2 = false;
    }
    float4 ta = make_float4(0.f, 0.f, 0.f, 0.f), tb = ta;
    if (withtau2) {
      ta = E.tau[2 * q];
      tb = E.tau[2 * q + 1];
    }
    sC[d] = make_float4(E.press[q], flag ? -m2 : m2, tb.x, tb.y);
    if (withtau) sD[d] = ta;
    if (inl) {  // the image right after it
      const float yi = -(pc.y + oy) - my;
      sA[d + 1] = make_float4(x2, yi, z2, x2 * x2 + yi * yi + z2 * z2);
      sB[d + 1] = make_float4(vr.x, -vr.y, vr.z, vr.w);
      sC[d + 1] = sC[d];
      if (withtau) sD[d + 1] = ta;
    }
  }
}

// Kernel factor fac (GetKernel_Fac<tker>, FunSphKernel.h:217-224 Wendland, :105-117 Cubic)
// and, for the Cubic spline, its Wab (the tensile correction's, :122-136).  Beyond the support
// (the masked pairs' rr2 = 1e30) both are 0.  The Cubic is a uniform runtime branch (K.cubic).
__device__ __forceinline__ float ext_fac(const KConst& K, float rr2, float& wab) {
  const float rad = fsqrt_(rr2);
  if (K.cubic) {
    const float qc = rad * K.ovkernelh;
    const float wqc = fmaxf(2.f - qc, 0.f);
    const bool far = rad > K.kernelh;
    // beyond h: c2 (2-q)^2 / r; within it (c1 q + d1 q^2) / r = (c1 + d1 q) / h (finite at r = 0)
    wab = far ? K.cub_a24 * (wqc * wqc * wqc) : K.cub_a2 * fmaf(fmaf(0.75f, qc, -1.5f), qc * qc, 1.f);
    return far ? K.cub_c2 * wqc * wqc * frcp(rad) : fmaf(K.cub_d1, qc, K.cub_c1) * K.ovkernelh;
  }
  wab = 0.f;
  const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
  return K.bwenovh * (wq * wq * wq);
}

// GetKernelCubic_Tensil (FunSphKernel.h:141-149) from the pair's Wab.
__device__ __forceinline__ float ext_tensil(const KConst& K, float wab, float rho1, float p1, float rho2, float p2) {
  float fab = wab * K.cub_odw;
  fab *= fab;
  fab *= fab;
  const float t1 = (p1 * frcp(rho1 * rho1)) * (p1 > 0.f ? 0.01f : -0.2f);
  const float t2 = (p2 * frcp(rho2 * rho2)) * (p2 > 0.f ? 0.01f : -0.2f);
  return fab * (t1 + t2);
}

// Fluid p1 pair (JSphCpu.cpp:682-797).  `ok` is the reference's pair test; a pair that fails
// it arrives with dr = 0 and rr2 = 1e30 (kernel factor 0, every sum +0) and its switches
// (DDT / shifting cut-offs, maxima) are masked.
template <int TVISCO, int TD, bool SHIFT, bool FT, bool BOUNDP2>
__device__ __forceinline__ void ext_pair(const KConst& K, const ExtP1& p, float drx, float dry, float drz, float rr2,
                                         bool ok, const float4& B, const float4& C, const float4& D, float visco,
                                         ExtAcc& a) {
  float wab;
  const float fac = ext_fac(K, rr2, wab);
  const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
  const bool flag2 = C.y < 0.f;
  const bool ftp2 = FT && !BOUNDP2 && flag2;
  const float massp2 = fabsf(C.y);
  if (FT && ok && ftp2) {
    if (TD == 1 && massp2 <= K.massfluid * 1.2f) a.delta = FLT_MAX;  // DELTA_HEAVYFLOATING (:699-703)
    if (SHIFT && K.shiftmode == 1) a.sx = FLT_MAX;
  }
  const float rho1 = p.vr.w, rho2 = B.w;
  const float inv_rho2 = frcp(rho2);
  // momentum: -m2 ((p1 + p2)/(rho1 rho2) + Cubic tensile correction) fr
  float prs = (p.press + C.x) * frcp(rho1 * rho2);
  if (K.cubic) prs += ext_tensil(K, wab, rho1, p.press, rho2, C.x);
  const float p_vpm = -prs * massp2;
  a.ax = fmaf(p_vpm, frx, a.ax);
  a.ay = fmaf(p_vpm, fry, a.ay);
  a.az = fmaf(p_vpm, frz, a.az);
  // continuity: m2 (dv.fr) rho1/rho2
  const float dvx = p.vr.x - B.x, dvy = p.vr.y - B.y, dvz = p.vr.z - B.z;
  const float dot = drx * dvx + dry * dvy + drz * dvz;
  a.ar = fmaf(massp2 * (fac * dot), rho1 * inv_rho2, a.ar);
  const float dot3 = fac * rr2;  // dr.fr
  const float inv_re = frcp(rr2 + K.eta2);
  if (TD == 1 && a.delta != FLT_MAX) {  // Molteni & Colagrossi (:724-731); rho1/rho2 - 1 as (rho1 - rho2)/rho2
    const float visc_densi = K.ddtkh * K.cs0f * ((rho1 - rho2) * inv_rho2) * inv_re;
    const float delta = visc_densi * dot3 * massp2;
    a.delta = (BOUNDP2 && !K.mdbc && ok) ? FLT_MAX : a.delta + delta;
  }
  if ((TD == 2 || (TD == 3 && !BOUNDP2)) && a.delta != FLT_MAX && !ftp2) {  // Fourtakas (:733-740)
    const float drhop = K.ddtseries ? drz * fmaf(drz, fmaf(drz, K.ddte3, K.ddte2), K.ddte1)
                                    : K.rhopzero * fexp2(K.ovgamma * flog2(1.f + K.ddtgz * drz)) - K.rhopzero;
    const float visc_densi = K.ddtkh * K.cs0f * ((rho2 - rho1) - drhop) * inv_re;
    const float delta = visc_densi * dot3 * massp2 * inv_rho2;
    a.delta = (BOUNDP2 && ok) ? FLT_MAX : a.delta - delta;
  }
  if (SHIFT && a.sx != FLT_MAX) {  // (:743-750)
    const float massrhop = massp2 * inv_rho2;
    const bool noshift = ok && BOUNDP2 && (K.shiftmode == 1 || (K.shiftmode == 2 && flag2));
    a.sx = noshift ? FLT_MAX : a.sx + massrhop * frx;
    a.sy += massrhop * fry;
    a.sz += massrhop * frz;
    a.sw -= massrhop * dot3;
  }
  const float dot_rr2 = dot * inv_re;
  a.visc = fmaxf(ok ? dot_rr2 : 0.f, a.visc);
  if constexpr (TVISCO == 1) {  // artificial (:757-764)
    if (dot < 0.f) {
      const float amubar = K.kernelh * dot_rr2;
      const float robar = (rho1 + rho2) * 0.5f;
      const float pi_visc = (-visco * K.cs0f * amubar * frcp(robar)) * massp2;
      a.ax = fmaf(-pi_visc, frx, a.ax);
      a.ay = fmaf(-pi_visc, fry, a.ay);
      a.az = fmaf(-pi_visc, frz, a.az);
    }
  } else {  // Laminar + SPS (:765-791)
    const float temp = 4.f * visco * frcp((rr2 + K.eta2) * (rho1 + rho2));
    const float vtemp = massp2 * temp * dot3;
    a.ax = fmaf(vtemp, dvx, a.ax);
    a.ay = fmaf(vtemp, dvy, a.ay);
    a.az = fmaf(vtemp, dvz, a.az);
    // tau1 + tau2 (the staged tau2 is 0 for a bound or floating p2: tau1 + 0 = tau1)
    const float txx = p.t[0] + D.x, txy = p.t[1] + D.y, txz = p.t[2] + D.z, tyy = p.t[3] + D.w;
    const float tyz = p.t[4] + C.z, tzz = p.t[5] + C.w;
    a.ax = fmaf(massp2, txx * frx + txy * fry + txz * frz, a.ax);
    a.ay = fmaf(massp2, txy * frx + tyy * fry + tyz * frz, a.ay);
    a.az = fmaf(massp2, txz * frx + tyz * fry + tzz * frz, a.az);
    if (!p.ftp1) {  // velocity gradients (xy = du/dy + dv/dx ...)
      const float volp2 = -massp2 * inv_rho2;
      float dv = dvx * volp2;
      a.gxx = fmaf(dv, frx, a.gxx);
      a.gxy = fmaf(dv, fry, a.gxy);
      a.gxz = fmaf(dv, frz, a.gxz);
      dv = dvy * volp2;
      a.gxy = fmaf(dv, frx, a.gxy);
      a.gyy = fmaf(dv, fry, a.gyy);
      a.gyz = fmaf(dv, frz, a.gyz);
      dv = dvz * volp2;
      a.gxz = fmaf(dv, frx, a.gxz);
      a.gyz = fmaf(dv, fry, a.gyz);
      a.gzz = fmaf(dv, frz, a.gzz);
    }
  }
}

// Bound p1 over fluid p2 (InteractionForcesBound, :577-608): continuity and visc-dt.
__device__ __forceinline__ void ext_bound_pair(const KConst& K, const ExtP1& p, float drx, float dry, float drz,
                                               float rr2, bool ok, const float4& B, const float4& C, ExtAcc& a) {
  float wab;
  const float fac = ext_fac(K, rr2, wab);
  const float dvx = p.vr.x - B.x, dvy = p.vr.y - B.y, dvz = p.vr.z - B.z;
  const float dot = drx * dvx + dry * dvy + drz * dvz;
  a.ar = fmaf(fabsf(C.y) * (fac * dot), p.vr.w * frcp(B.w), a.ar);
  a.visc = fmaxf(ok ? dot * frcp(rr2 + K.eta2) : 0.f, a.visc);
}

// KIND 0: fluid p1 / fluid p2, 1: fluid p1 / bound p2, 2: bound p1 / fluid p2.
template <int TVISCO, int TD, bool SHIFT, bool FT, int KIND>
__device__ __forceinline__ void ext_pairs(const KConst& K, const ExtP1& p, int j1, int j2, bool two,
                                          const float4* __restrict__ sA, const float4* __restrict__ sB,
                                          const float4* __restrict__ sC, const float4* __restrict__ sD, float visco,
                                          ExtAcc& a) {
  const float4 A1 = sA[j1], A2 = sA[j2];
  const float4 B1 = sB[j1], B2 = sB[j2];
  const float4 C1 = sC[j1], C2 = sC[j2];
  float4 D1 = make_float4(0.f, 0.f, 0.f, 0.f), D2 = D1;
  if constexpr (TVISCO == 2 && KIND != 2) {
    D1 = sD[j1];
    D2 = sD[j2];
  }
  float drx1 = p.x - A1.x, dry1 = p.y - A1.y, drz1 = p.z - A1.z;
  float drx2 = p.x - A2.x, dry2 = p.y - A2.y, drz2 = p.z - A2.z;
  float rr21 = drx1 * drx1 + dry1 * dry1 + drz1 * drz1;
  float rr22 = drx2 * drx2 + dry2 * dry2 + drz2 * drz2;
  const bool ok1 = rr21 <= K.kernelsize2 && rr21 >= ALMOSTZERO;
  const bool ok2 = two && rr22 <= K.kernelsize2 && rr22 >= ALMOSTZERO;
  drx1 = ok1 ? drx1 : 0.f;
  dry1 = ok1 ? dry1 : 0.f;
  drz1 = ok1 ? drz1 : 0.f;
  rr21 = ok1 ? rr21 : 1e30f;
  drx2 = ok2 ? drx2 : 0.f;
  dry2 = ok2 ? dry2 : 0.f;
  drz2 = ok2 ? drz2 : 0.f;
  rr22 = ok2 ? rr22 : 1e30f;
  if constexpr (KIND == 2) {
    ext_bound_pair(K, p, drx1, dry1, drz1, rr21, ok1, B1, C1, a);
    ext_bound_pair(K, p, drx2, dry2, drz2, rr22, ok2, B2, C2, a);
  } else {
    ext_pair<TVISCO, TD, SHIFT, FT, KIND == 1>(K, p, drx1, dry1, drz1, rr21, ok1, B1, C1, D1, visco, a);
    ext_pair<TVISCO, TD, SHIFT, FT, KIND == 1>(K, p, drx2, dry2, drz2, rr22, ok2, B2, C2, D2, visco, a);
  }
}

// Four 64-bit words of accepted candidates (bases b0..b3), popped two pairs per iteration
// in word order (ascending staged index within a word).
template <int TVISCO, int TD, bool SHIFT, bool FT, int KIND>
__device__ __forceinline__ void ext_drain4(const KConst& K, const ExtP1& p, unsigned long long c0,
                                           unsigned long long c1, unsigned long long c2, unsigned long long c3, int b0,
                                           int b1, int b2, int b3, const float4* __restrict__ sA,
                                           const float4* __restrict__ sB, const float4* __restrict__ sC,
                                           const float4* __restrict__ sD, float visco, ExtAcc& a) {
#pragma unroll
  for (int pass = 0; pass < 3; pass++) {  // drop empty words, keep the order
    const bool e2 = c2 == 0ull;
    c2 = e2 ? c3 : c2;
    b2 = e2 ? b3 : b2;
    c3 = e2 ? 0ull : c3;
    const bool e1 = c1 == 0ull;
    c1 = e1 ? c2 : c1;
    b1 = e1 ? b2 : b1;
    c2 = e1 ? c3 : c2;
    b2 = e1 ? b3 : b2;
    c3 = e1 ? 0ull : c3;
    const bool e0 = c0 == 0ull;
    c0 = e0 ? c1 : c0;
    b0 = e0 ? b1 : b0;
    c1 = e0 ? c2 : c1;
    b1 = e0 ? b2 : b1;
    c2 = e0 ? c3 : c2;
    b2 = e0 ? b3 : b2;
    c3 = e0 ? 0ull : c3;
  }
  auto pop = [&](void) -> int {
    const int j = b0 + int(__builtin_ctzll(c0 | (1ull << 63)));
    c0 &= c0 - 1ull;
    const bool e = c0 == 0ull;
    c0 = e ? c1 : c0;
    b0 = e ? b1 : b0;
    c1 = e ? c2 : c1;
    b1 = e ? b2 : b1;
    c2 = e ? c3 : c2;
    b2 = e ? b3 : b2;
    c3 = e ? 0ull : c3;
    return j;
  };
  while (c0) {
    const int j1 = pop();
    const bool two = c0 != 0ull;
    const int j2p = pop();
    ext_pairs<TVISCO, TD, SHIFT, FT, KIND>(K, p, j1, two ? j2p : j1, two, sA, sB, sC, sD, visco, a);
  }
}

// The (2S+1)^2 rows of one kind (S = scelldiv: 3x3 rows of cells of 2h, or 5x5 rows of
// half-cells, JCellSearch_inline.h:38-44): MIRRORED drains point-mirrored row pairs as one
// set (order-free sums), else rows in the reference's order (z-major, y, p2 ascending) for
// the passes whose shifting cut-off makes the sums order-dependent.
template <int TVISCO, int TD, bool SHIFT, bool FT, int KIND, int S>
__device__ __forceinline__ void ext_pass(const KConst& K, const ExtArgs& E, const DivGrid& g, const RowCtx& rc,
                                         const ExtP1& p, float thr, const unsigned* __restrict__ bc, bool mirrored,
                                         float visco, float4* __restrict__ sA, float4* __restrict__ sB,
                                         float4* __restrict__ sC, float4* __restrict__ sD, ExtAcc& a) {
  constexpr int TCAPX = ExtCap<TVISCO>::v;
  constexpr bool WT = TVISCO == 2 && KIND != 2;
  constexpr int NR = 2 * S + 1;           // rows per axis
  constexpr int NPAIR = (NR * NR - 1) / 2;  // mirrored row pairs; the own row after them
  const unsigned cellinit = (KIND == 1 ? 0u : g.boxfluid);
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  const int nunits = mirrored ? NPAIR + 1 : NR * NR;
  // Symmetry: a p1 within 2h of y = 0 (the first S rows) also meets the images of the p2 of
  // those rows (all within 2h of the plane), after its own rows: units of a mirrored z pair /
  // the z = 0 row per image row (S == 1: the row itself; S == 2: rows 0 and 1), its own image
  // skipped.  The reference visits an image right after its original when the original is
  // within the support radius (JSphCpu.cpp:793-796); an image is never nearer than its
  // original for y >= 0, so the images within the radius are exactly those.  Their order
  // matters only for a shifting cut-off: the passes drained in the reference's order
  // (NoBound's / NoFixed's bound rows — under NoFixed a moving boundary's image counts until
  // the first fixed pair) take each image right after its original (inline, its records
  // staged as [record, image] pairs); the order-free passes take the images after the rows,
  // in units of their own.
  const bool sym = K.symmetry && rc.cy < S;
  const bool inl = sym && !mirrored;
  const int nimg = (sym && !inl) ? S * (S + 1) : 0;  // image rows x (S mirrored z pairs + the z = 0 row)
  for (int u = 0; u < nunits + nimg; u++) {
    int dza = 0, dya = 0;
    bool paired = false, mir = false, selfrow = false;
    if (u >= nunits) {  // image unit: row ir of the first S rows, z unit iz
      const int v = u - nunits, ir = v / (S + 1), iz = v % (S + 1);
      mir = true;
      dya = ir - rc.cy;
      dza = iz < S ? -(iz + 1) : 0;
      paired = iz < S;
      selfrow = !paired && dya == 0;
    } else if (mirrored) {
      paired = u < NPAIR;
      if (S == 1) {
        dza = (u == 0 || u == 1 || u == 2) ? -1 : 0;
        dya = (u == 0) ? -1 : (u == 1) ? 1 : (u == 2) ? 0 : (u == 3) ? -1 : 0;
      } else if (paired) {
        half_row(u, dya, dza);
      }
    } else {
      dza = u / NR - S;
      dya = u % NR - S;
    }
    unsigned rs[2] = {0, 0}, re[2] = {0, 0}, ls[2] = {0, 0}, le[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !paired) break;
      const int dz = k ? -dza : dza, dy = (k && !mir) ? -dya : dya;  // an image pair mirrors z only
      const int z = rc.cz + dz, y = rc.cy + dy;
      if (z < 0 || z >= g.ncz || y < 0 || y >= g.ncy) continue;
      const unsigned rowbase = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
      rs[k] = bc[rowbase + rc.xa];
      re[k] = bc[rowbase + rc.xb + 1];
      ls[k] = bc[rowbase + rc.lxa];
      le[k] = bc[rowbase + rc.lxb + 1];
    }
    const unsigned n0 = re[0] - rs[0], n1 = re[1] - rs[1];
    if (n0 + n1 == 0u) continue;  // block-uniform
    // inline images (an ordered pass's row of the first S y rows: one row, not paired): the
    // row staged as [record, image] pairs, m = 2 staged records per particle
    const bool rowinl = inl && rc.cy + dya < S;
    const unsigned m = rowinl ? 2u : 1u;
    if (m * n0 + n1 <= unsigned(TCAPX)) {
      __syncthreads();
      if (n0) ext_stage(K, E, rs[0], n0, 0u, rc.xo, dya, dza, KIND == 1, WT, sA, sB, sC, sD, mir, rc.cy, rowinl);
      if (n1) ext_stage(K, E, rs[1], n1, n0, rc.xo, mir ? dya : -dya, -dza, KIND == 1, WT, sA, sB, sC, sD, mir, rc.cy);
      __syncthreads();
      const int wa0 = int(m * (ls[0] - rs[0])), wa1 = rc.act && n0 ? int(m * (le[0] - rs[0])) : wa0;
      const int wb0 = int(n0 + ls[1] - rs[1]), wb1 = rc.act && n1 ? int(n0 + le[1] - rs[1]) : wb0;
      // the own image (the lane's p1 in its own row's images) is no neighbour
      const bool own = rc.act && rc.p1 >= rs[0] && rc.p1 < re[0];
      const int self = (selfrow && own) ? int(rc.p1 - rs[0]) : ((rowinl && own) ? int(2 * (rc.p1 - rs[0]) + 1) : -1);
      for (int off = 0;; off += 128) {
        const int na = wa1 - wa0 - off, nb = wb1 - wb0 - off;
        if (na <= 0 && nb <= 0) break;
        unsigned long long c0, c1, c2, c3;
        test128(sA, wa0 + off, min(na, 128), px2, py2, pz2, thr, c0, c1);
        test128(sA, wb0 + off, min(nb, 128), px2, py2, pz2, thr, c2, c3);
        if (self >= 0) {
          const int ks = self - (wa0 + off);
          if (ks >= 0 && ks < 64) c0 &= ~(1ull << ks);
          else if (ks >= 64 && ks < 128) c1 &= ~(1ull << (ks - 64));
        }
        ext_drain4<TVISCO, TD, SHIFT, FT, KIND>(K, p, c0, c1, c2, c3, wa0 + off, wa0 + off + 64, wb0 + off,
                                                wb0 + off + 64, sA, sB, sC, sD, visco, a);
      }
    } else {
      for (int k = 0; k < (paired ? 2 : 1); k++) {
        const int dz = k ? -dza : dza, dy = (k && !mir) ? -dya : dya;
        for (unsigned seg = rs[k]; seg < re[k]; seg += unsigned(TCAPX) / m) {
          const unsigned segn = min(unsigned(TCAPX) / m, re[k] - seg);
          __syncthreads();
          ext_stage(K, E, seg, segn, 0u, rc.xo, dy, dz, KIND == 1, WT, sA, sB, sC, sD, mir, rc.cy, rowinl);
          __syncthreads();
          const int w0 = int(m * (max(ls[k], seg) - seg));
          const int w1 = rc.act ? max(w0, int(m) * (int(min(le[k], seg + segn)) - int(seg))) : w0;
          const bool own = rc.act && rc.p1 >= seg && rc.p1 < seg + segn;
          const int self = (selfrow && own) ? int(rc.p1 - seg) : ((rowinl && own) ? int(2 * (rc.p1 - seg) + 1) : -1);
          for (int off = w0; off < w1; off += 128) {
            unsigned long long c0, c1;
            test128(sA, off, min(w1 - off, 128), px2, py2, pz2, thr, c0, c1);
            if (self >= 0) {
              const int ks = self - off;
              if (ks >= 0 && ks < 64) c0 &= ~(1ull << ks);
              else if (ks >= 64 && ks < 128) c1 &= ~(1ull << (ks - 64));
            }
            ext_drain4<TVISCO, TD, SHIFT, FT, KIND>(K, p, c0, c1, 0ull, 0ull, off, off + 64, 0, 0, sA, sB, sC, sD,
                                                    visco, a);
          }
        }
      }
    }
  }
}

template <int TVISCO, int TD, bool SHIFT, bool FT, int S>
__global__ __launch_bounds__(TB) void k_fluid_ext(DevScalars* __restrict__ sc, const uint4* __restrict__ items,
                                                  unsigned* __restrict__ qctr, ExtArgs E,
                                                  const unsigned* __restrict__ bc, DivGrid g, KConst K,
                                                  float4* __restrict__ arace, float4* __restrict__ shiftpos,
                                                  float4* __restrict__ taunew, int shiftstore) {
  constexpr int TCAPX = ExtCap<TVISCO>::v;
  __shared__ float4 sABC[3 * TCAPX];  // sA, sB, sC: the candidate test's over-read stays inside
  float4* const sA = sABC;
  float4* const sB = sABC + TCAPX;
  float4* const sC = sABC + 2 * TCAPX;
  __shared__ float4 sD[TVISCO == 2 ? TCAPX : 1];
  __shared__ unsigned s_item;
  __shared__ unsigned char s_perm[TB];
  __shared__ unsigned s_nwave[4];
  float viscmax = 0.f, ace2max = 0.f;
  // passes whose shifting cut-off depends on the pair order: the fluid rows with floating
  // bodies under NoBound, the bound rows under NoBound / NoFixed
  const bool ordf = SHIFT && FT && K.shiftmode == 1;
  const bool ordb = SHIFT && (K.shiftmode == 1 || K.shiftmode == 2);
  ItemCursor<false> cur(qctr);
  for (;;) {
    const unsigned it = cur.next(&s_item);
    if (it == ITEM_NONE) break;
    const uint4 item = items[it];
    const bool bitem = (item.x & ITEM_BOUND) != 0u;
    const int cy = int(item.x & 0xffffu), cz = int((item.x >> 16) & 0x7fffu);
    const int ia = int(item.y & 0xffffu), ib = int(item.y >> 16);
    const int xo = (ia + ib + 1) >> 1;
    const int xa = max(ia - S, 0), xb = min(ib + S, g.ncx - 1);
    if (bitem) {  // no fluid within reach: ar = 0 (PreInteraction reset), nothing else
      bool any = false;
      for (int z = max(cz - S, 0); z <= min(cz + S, g.ncz - 1); z++)
        for (int y = max(cy - S, 0); y <= min(cy + S, g.ncy - 1); y++) {
          const unsigned rowbase = g.boxfluid + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
          any |= bc[rowbase + xa] != bc[rowbase + xb + 1];
        }
      if (!any) {
        for (unsigned p1 = item.z + threadIdx.x; p1 < item.w; p1 += TB) arace[p1] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
    }
    const unsigned p1 = item.z + lane_order(E.poscell, item.z, item.w - item.z, 0.5f * K.scell, s_perm, s_nwave);
    const bool act = threadIdx.x < item.w - item.z;
    ExtP1 p;
    int cx1 = ia;
    p.ftp1 = false;
    for (int k = 0; k < 6; k++) p.t[k] = 0.f;
    if (act) {
      const float4 pc1 = E.poscell[p1];
      cx1 = int(DcelCellx(K.domcellcode, __float_as_uint(pc1.w)));
      p.x = pc1.x + float(cx1 - xo) * K.scell;
      p.y = pc1.y;
      p.z = pc1.z;
      p.vr = E.velrhop[p1];
      p.press = bitem ? 0.f : E.press[p1];
      p.ftp1 = FT && !bitem && CodeType(E.code[p1]) == CODE_TYPE_FLOATING;
      if (TVISCO == 2 && !bitem && !p.ftp1) {  // taup1: zero for a floating p1 (not fluid)
        const float4 ta = E.tau[2 * p1], tb = E.tau[2 * p1 + 1];
        p.t[0] = ta.x;
        p.t[1] = ta.y;
        p.t[2] = ta.z;
        p.t[3] = ta.w;
        p.t[4] = tb.x;
        p.t[5] = tb.y;
      }
    } else {
      p.x = p.y = p.z = 1e30f;
      p.vr = make_float4(0.f, 0.f, 0.f, 1.f);
      p.press = 0.f;
    }
    const int lxa = max(cx1 - S, 0), lxb = min(cx1 + S, g.ncx - 1);
    const float thr = K.kernelsize2 * 1.0001f - (p.x * p.x + p.y * p.y + p.z * p.z);
    const RowCtx rc{cy, cz, xa, xb, lxa, lxb, xo, act, p1};
    if (bitem) {
      ExtAcc f = {};
      ext_pass<TVISCO, TD, SHIFT, FT, 2, S>(K, E, g, rc, p, thr, bc, true, 0.f, sA, sB, sC, sD, f);
      if (act) {
        arace[p1] = make_float4(0.f, 0.f, 0.f, (f.ar != 0.f || f.visc != 0.f) ? 0.f + f.ar : 0.f);
        viscmax = fmaxf(viscmax, f.visc);
      }
      continue;
    }
    // fluid p1: the fluid pass, then the bound pass; the shifting sums carry over
    // (shiftposfs[p1] is stored by the first pass and loaded by the second), a floating
    // p1 starts with x = FLT_MAX (:662); DDT is off for a floating p1 (:661)
    ExtAcc f = {}, b = {};
    if (p.ftp1) {
      f.sx = FLT_MAX;
      if (TD) f.delta = FLT_MAX;
    }
    const float visco = K.visco_n ? sc->visco : K.visco;  // ViscoTime (k_dt) or the case's
    ext_pass<TVISCO, TD, SHIFT, FT, 0, S>(K, E, g, rc, p, thr, bc, !ordf, visco, sA, sB, sC, sD, f);
    b.sx = f.sx;
    b.sy = f.sy;
    b.sz = f.sz;
    b.sw = f.sw;
    if (p.ftp1 && TD) b.delta = FLT_MAX;
    ext_pass<TVISCO, TD, SHIFT, FT, 1, S>(K, E, g, rc, p, thr, bc, !ordb, K.visco_n ? visco * K.viscobf : K.viscobound,
                                       sA, sB, sC, sD, b);
    if (act) {
      // the two passes' stores (:800-818); with shifting both always store
      float ar = 0.f, ax = 0.f, ay = 0.f, az = 0.f, delta = 0.f;
      float gxx = 0.f, gxy = 0.f, gxz = 0.f, gyy = 0.f, gyz = 0.f, gzz = 0.f;
      if (SHIFT || f.ar != 0.f || f.ax != 0.f || f.ay != 0.f || f.az != 0.f || f.visc != 0.f) {
        if (TD) delta = (f.delta == FLT_MAX ? FLT_MAX : 0.f + f.delta);
        ar = f.ar;
        ax = f.ax;
        ay = f.ay;
        az = f.az;
        gxx = f.gxx, gxy = f.gxy, gxz = f.gxz, gyy = f.gyy, gyz = f.gyz, gzz = f.gzz;
      }
      if (SHIFT || b.ar != 0.f || b.ax != 0.f || b.ay != 0.f || b.az != 0.f || b.visc != 0.f) {
        if (TD) delta = (delta == FLT_MAX || b.delta == FLT_MAX ? FLT_MAX : delta + b.delta);
        ar += b.ar;
        ax += b.ax;
        ay += b.ay;
        az += b.az;
        gxx += b.gxx, gxy += b.gxy, gxz += b.gxz, gyy += b.gyy, gyz += b.gyz, gzz += b.gzz;
      }
      if (TD && delta != FLT_MAX) ar += delta;
      if (K.sim2d) ay = 0.f;  // Simulate2D: Acec[].y = 0 (JSphCpuSingle.cpp:544-549)
      arace[p1] = make_float4(ax, ay, az, ar);
      if (SHIFT && shiftstore) shiftpos[p1] = make_float4(b.sx, b.sy, b.sz, b.sw);
      viscmax = fmaxf(viscmax, fmaxf(f.visc, b.visc));
      ace2max = nanmax(ace2max, ax * ax + ay * ay + az * az);
      if constexpr (TVISCO == 2) {
        // ComputeSpsTau (:929-954) of p1 from this interaction's gradients
        const float pow1 = gxx * gxx + gyy * gyy + gzz * gzz;
        const float prr = pow1 + pow1 + gxy * gxy + gxz * gxz + gyz * gyz;
        const float visc_sps = K.spssmag * sqrtf(prr);
        const float div_u = gxx + gyy + gzz;
        const float sps_k = (2.0f / 3.0f) * visc_sps * div_u;
        const float sps_blin = K.spsblin * prr;
        const float sumsps = -(sps_k + sps_blin);
        const float twovisc_sps = visc_sps + visc_sps;
        const float one_rho2 = 1.0f / p.vr.w;
        taunew[2 * p1] = make_float4(one_rho2 * (twovisc_sps * gxx + sumsps), one_rho2 * (visc_sps * gxy),
                                     one_rho2 * (visc_sps * gxz), one_rho2 * (twovisc_sps * gyy + sumsps));
        taunew[2 * p1 + 1] = make_float4(one_rho2 * (visc_sps * gyz), one_rho2 * (twovisc_sps * gzz + sumsps), 0.f,
                                         0.f);
      }
    }
  }
  wave_max_atomic(sc, RED_VISCDT, viscmax);
  wave_max_atomic(sc, RED_ACEMAX2, ace2max);
}

void launch_fluid_ext(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                      const float4* poscell, const float4* velrhop, const float* press, const typecode* code,
                      const float* ftmassp, const float4* tau, const unsigned* begincell, DivGrid g, const KConst& K,
                      float4* arace, float4* shiftpos, float4* taunew, bool shiftstore) {
  const ExtArgs E{poscell, velrhop, press, code, ftmassp, tau};
  const bool shift = K.shiftmode != 0, ft = ftmassp != nullptr;
  // CellMode: cells of 2h (S = 1) or of h (S = 2)
#define SPH_EXT(TV, TD, SH, FT)                                                                                  \
  if (K.scelldiv == 2)                                                                                           \
    hipLaunchKernelGGL((k_fluid_ext<TV, TD, SH, FT, 2>), dim3(fit_grid((const void*)&k_fluid_ext<TV, TD, SH, FT, 2>, nblocks)), dim3(TB), 0, stm, sc, items, qctr, E,     \
                       begincell, g, K, arace, shiftpos, taunew, int(shiftstore));                               \
  else                                                                                                           \
    hipLaunchKernelGGL((k_fluid_ext<TV, TD, SH, FT, 1>), dim3(fit_grid((const void*)&k_fluid_ext<TV, TD, SH, FT, 1>, nblocks)), dim3(TB), 0, stm, sc, items, qctr, E,     \
                       begincell, g, K, arace, shiftpos, taunew, int(shiftstore))
#define SPH_EXT_TD(TV, SH, FT)             \
  switch (K.tdensity) {                    \
    case 0: SPH_EXT(TV, 0, SH, FT); break; \
    case 1: SPH_EXT(TV, 1, SH, FT); break; \
    case 2: SPH_EXT(TV, 2, SH, FT); break; \
    default: SPH_EXT(TV, 3, SH, FT); break; \
  }
#define SPH_EXT_SH(TV, FT)                       \
  if (shift) { SPH_EXT_TD(TV, true, FT) }        \
  else { SPH_EXT_TD(TV, false, FT) }
#define SPH_EXT_FT(TV)               \
  if (ft) { SPH_EXT_SH(TV, true) }   \
  else { SPH_EXT_SH(TV, false) }
  if (K.tvisco == 2) {
    SPH_EXT_FT(2)
  } else {
    SPH_EXT_FT(1)
  }
#undef SPH_EXT_FT
#undef SPH_EXT_SH
#undef SPH_EXT_TD
#undef SPH_EXT
}

}  // namespace sphx
