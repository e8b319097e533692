// sph_nn.hip — non-Newtonian multiphase Interaction_Forces (the v5.0 NNewtonian solver,
// SURVEY.md §8(f) row 4) as an LDS-tiled CDNA4 kernel.
//
// Reference: JSphCpu::InteractionForcesFluid_NN_FDA_All / InteractionForcesBound_NN_FDA
// (src_mphase/DSPH_v5.0_NNewtonian/source/JSphCpu_NN_FDA.cpp:45-332), the tensor helpers
// GetVelocityGradients_FDA / GetStrainRateTensor / GetEta_Effective / GetStressTensor
// (JSphCpu_Tensors.cpp:40-139), GPU twin KerInteractionForcesFluid_NN_FDA
// (JSphGpu_NN_ker.cu:421-1555).  Per fluid p1 and pair: per-phase mass and sound speed of
// p2, momentum, continuity, DDT (only between particles of the same phase), multiphase
// shifting sums, and the viscous term with the effective viscosity of the Herschel-
// Bulkley-Papanastasiou law evaluated from the pair's FDA velocity gradient
// (Laminar: Morris operator; ConstEq: the stress tensor 2 eta D).
//
// Work decomposition: the items, LDS staging and mirrored drain units of
// sph_interaction_tiled.hip (sph_tiled.hpp), with one order-dependent sum handled apart:
// the shifting x sum of the reference is RESET by every pair with a heavier-phase
// neighbour (`heavyphase ? 0 : x + ...`, JSphCpu_NN_FDA.cpp:206), so its value depends on
// the pair order.  The reference visits the 3x3 rows z-major, y, then p2 ascending in the
// row — i.e. p2 in ascending cell-sorted index.  The fluid pass drains point-mirrored row
// pairs as one set (lanes with alike loop lengths; every other sum is order-free up to
// rounding) and flags a heavier-phase neighbour; a block with a flagged lane then re-sweeps
// its rows in the reference order for sx alone (nn_sx_sweep: phase interfaces only).  The
// bound-p2 pass keeps the reference order when its first no-shift pair can freeze every
// shifting sum (ShiftMode NoBound/NoFixed), else it is drained in mirrored units too.  cfg5: 1.85 -> 1.55 ms per interaction (SPH_NN_MIRROR=0: the
// row-ordered drain of every pass).
#include <algorithm>
#include <stdexcept>

#include "sph_tiled.hpp"

namespace sphx {

// Staged records per row segment: 41 B each (position, velrhop, {press, 1/rho}, tag); 480
// records + the 8-record pad + the phase table keep the block at 20472 B of LDS (8 blocks =
// 4 waves per SIMD), and a mirrored row pair mostly fits one segment (cfg5: 1.554 ms at
// 410 records of 48 B, 1.515 ms at 480 of 41 B).
#ifndef SPH_NN_TCAP
#define SPH_NN_TCAP 476  // 476 x 41 B + pad + the 3-row phase table: 20436 B (8 blocks/CU)
#endif
constexpr int NN_TCAP = SPH_NN_TCAP;

// Phase table in LDS: two float4 per phase.
//   a = {mass, cs0, visco, tau_yield}, b = {m (HBP_m), n (HBP_n), tau_max, bi_multi}
struct NNAcc {
  float ax, ay, az, ar, delta, visc, visceta;
  float sx, sy, sz, sw;  // shifting sums (shiftposfsp1)
  bool hv;               // mirrored drain: a heavier-phase neighbour was seen (sx needs the ordered sweep)
  bool ftsx;             // a floating p2 under ShiftMode NoBound (or a floating p1): sx = FLT_MAX, final
  float gxx, gxy, gxz, gyy, gyz, gzz;  // SPH velocity gradients (TVISCO 4; gradvelp1, xy = du/dy + dv/dx)
};

// Interaction modes of k_nn_tiled (TVISCO template parameter):
//   1, 2, 3  FDA velocity gradients (VelocityGradientType 1) with artificial, Laminar
//            (Morris) or constitutive-equation viscosity, all in the pair loop
//            (InteractionForcesFluid_NN_FDA_All, JSphCpu_NN_FDA.cpp:141-275);
//   4        SPH velocity gradients (VelocityGradientType 2), Laminar or ConstEq: the pair
//            loop of InteractionForcesFluid_NN_SPH_PressGrad (JSphCpu_NN_SPH.cpp:452-621)
//            accumulates gradvel, and each p1 then gets its strain rate, effective viscosity
//            and (ConstEq) stress tensor (_Visco_eta / _Visco_Stress_tensor, :128-222);
//            the viscous force is the second pass k_nn_visc (Morris / ConsEq, :228-446);
//   5        SPH gradients with artificial viscosity: PressGrad without a viscous term; the
//            artificial term is k_nn_visc's (the Morris pass, whose bound-p2 velocity
//            difference is 2 v1, JSphCpu_NN_SPH.cpp:403-405).
constexpr int NN_SPH_GRAD = 4, NN_SPH_ART = 5;

// Third part of a staged record: {press, 1/rho} (8 B) + the tag (1 B) — 41 B records in all.
struct NNSC {
  float2* c;
  unsigned char* t;
  // as the float4 {press, tag, 1/rho, 0} of the pair bodies: tag = phase index bits (fluid
  // rows) or 1.0 for a fixed boundary particle (bound rows)
  __device__ __forceinline__ float4 ld(int j, bool boundrow) const {
    const float2 v = c[j];
    const unsigned tg = t[j];
    return make_float4(v.x, boundrow ? float(tg) : __uint_as_float(tg), v.y, 0.f);
  }
};

struct NNP1 {
  float x, y, z;   // item-relative position
  float4 vr;       // velocity, rho
  float press;
  int ph;          // phase of p1
  float inv_rho;   // 1/rho1
  float mph;       // mass of p1's phase (the heavier-phase test of the shifting)
  float taumax, bimulti;  // bi-viscosity constants of p1's phase
  int uph;         // the item's phase (that of its first particle; -1: none): see NNUni
  bool p1uni;      // this lane's p1 is a fluid particle of phase uph (or the lane is idle)
};

// A single-phase drain unit (the bulk of every phase): every staged record of the unit and
// every p1 of the block are fluid particles of one phase k (a block vote after the staging).
// Its pairs then take that phase's constants from SGPRs, read once per item, instead of the
// dependent LDS chain record -> phase tag -> the phase table's two rows of every pair, and
// the same-phase / heavier-phase tests of the pair body are known (DDT on, no shifting reset).
// The values are those the table gives, so the result is bitwise the general path's.
struct NNUni {
  float4 a, c;  // sph[2 k] = {mass, cs0, visco, tau_yield}, sph[2 SPH_MAXPHASES + k]
  int k;
};

// GetEta_Effective (JSphCpu_Tensors.cpp:116-142): Herschel-Bulkley-Papanastasiou effective
// viscosity with the optional bi-viscosity region of p1's phase (tau_max, Bi_multi).  `bi`
// (K.nnbi, uniform over the launch): some phase has tau_max != 0; without one the
// bi-viscosity terms drop out (tau_max 0 selects tau_yield and no bi region), so that
// branch computes the same values with fewer operations.
__device__ __forceinline__ float nn_eta(bool bi, float dmag, float tau_yield, float visco, const float4& c,
                                        float taumax1, float bimulti1) {
  // c: the phase's {m tau_yield, -m log2(e), n - 1, .} (the solver's third table row)
  const float mtau = c.x;
  if (dmag <= ALMOSTZERO) dmag = ALMOSTZERO;
  // visco * D^(n-1), exactly visco for n = 1 (a per-wave skip for n = 1 / m = 0 measured
  // neutral-to-slower at cfg5)
  const float miou_hb = visco * fexp2(c.z * flog2(dmag));
  const float e = 1.f - fexp2(c.y * dmag);  // 1 - exp(-m D)
  if (!bi) {
    const float miou_pap = tau_yield * frcp(2.f * dmag) * e;
    const bool cap = (miou_pap > mtau || dmag == ALMOSTZERO);
    return (cap ? mtau : miou_pap) + (cap ? visco : miou_hb);
  }
  float miou_yield = (taumax1 != 0.f ? taumax1 : tau_yield) * frcp(2.f * dmag);
  // dmag <= taumax1 / (2 bimulti1 visco), without a second reciprocal (all factors > 0)
  const bool bi_region = taumax1 != 0.f && dmag * (2.f * bimulti1 * visco) <= taumax1;
  if (bi_region) miou_yield = bimulti1 * visco;
  const float miou_pap = miou_yield * e;
  const bool cap = (miou_pap > mtau || dmag == ALMOSTZERO);
  const float term1 = (taumax1 != 0.f ? miou_yield : (cap ? mtau : miou_pap));
  const float term2 = (bi_region ? visco : (cap ? visco : miou_hb));
  return term1 + term2;
}

// GetStrainRateTensor_tsym (JSphCpu_Tensors.cpp:185-208) of the SPH gradient (off-diagonal
// entries hold du/dy + dv/dx): D = {xx, xy, xz, yy, yz, zz} and |D| = sqrt(II_D) with the
// reference's expanded invariant.  II_D is a sum of squares up to rounding; where rounding
// leaves it below 0 the reference takes the square root of a negative number (NaN viscosity,
// with a printed warning) — here it is clamped to 0, i.e. |D| = 0.
__device__ __forceinline__ float nn_strain_rate(float gxx, float gxy, float gxz, float gyy, float gyz, float gzz,
                                                float d[6]) {
  const float div_vel = (gxx + gyy + gzz) / 3.f;
  d[0] = gxx - div_vel;
  d[1] = 0.5f * gxy;
  d[2] = 0.5f * gxz;
  d[3] = gyy - div_vel;
  d[4] = 0.5f * gyz;
  d[5] = gzz - div_vel;
  const float ii1 = d[0] * d[3] + d[3] * d[5] + d[0] * d[5];
  const float ii2 = d[1] * d[1] + d[4] * d[4] + d[2] * d[2];
  return sqrtf(fmaxf(-ii1 + ii2, 0.f));
}

// Maximum of a running maximum m >= 0 and x, as one integer max of the bit patterns
// (non-negative floats order like their bits; a negative x loses to m; a NaN x with the
// sign clear sticks): fmaxf costs two v_max here, the first canonicalising its input.
__device__ __forceinline__ float max_nonneg(float x, float m) {
  return __int_as_float(max(__float_as_int(x), __float_as_int(m)));
}

// One pair of the fluid p1 (InteractionForcesFluid_NN_FDA_All, JSphCpu_NN_FDA.cpp:141-275).
// BOUNDP2: p2 is a boundary particle (mass MassBound, phase = p1's phase).
// `ok`: the reference's pair test (rr2 <= KernelSize2 and rr2 >= ALMOSTZERO).  A pair that
// fails it comes in with rr2 = 1e30 (its dr unchanged): its kernel factor is 0, so fr and
// dot3 = fac r^2 are 0 and every sum gets +0 (each term carries fr or dot3; the FDA terms are
// finite with 1/r^2 = 1e-30), and the maxima, the DDT/shifting switches and the shifting
// reset are masked by ok — branch-free, so two pairs can be interleaved.
// ORDERED: pairs arrive in the reference's order (the shifting x sum is reset by a
// heavier-phase p2); else in mirrored-unit order: sx skips the heavy pair and a.hv records
// it, and the caller recomputes sx in the reference order (nn_sx_sweep) when any lane saw one.
// FT (floating bodies, JSphCpu_NN_FDA.cpp:203-215): a floating p2 (tag bit 7; the low bits
// its body index, which the reference also uses as the phase index of its phase constants)
// carries its body's particle mass (the fourth phase-table row), switches the Molteni DDT of
// p1 off when it is not heavier than 1.2 MassFluid (DELTA_HEAVYFLOATING), takes no part in
// the Fourtakas DDT, and under ShiftMode NoBound cancels p1's shifting.
template <int TVISCO, int TDENSITY, bool SHIFT, bool BOUNDP2, bool ORDERED = true, bool FT = false, bool UNI = false>
__device__ __forceinline__ void nn_pair(const KConst& K, const float4* __restrict__ sph, const NNP1& p, float drx,
                                        float dry, float drz, float rr2, bool ok, const float4& B, const float4& C,
                                        NNAcc& a, const NNUni& u = NNUni{}) {
  static_assert(!UNI || (!BOUNDP2 && !ORDERED), "single-phase units: fluid p2 in mirrored order only");
  // kernel (Wendland fac = bwen q (1-q/2)^3 / r = (bwen/h) (1-q/2)^3), 0 beyond 2h.  With the
  // FDA gradient (which needs 1/r^2 too) one v_rsq gives both: r = r^2 rsq, 1/r^2 = rsq^2
  // (one transcendental instead of v_sqrt + v_rcp; ulp-level differences)
  constexpr bool FDA = (TVISCO == 2 || TVISCO == 3);
  const float rsq = FDA ? __builtin_amdgcn_rsqf(rr2) : 0.f;
  const float rad = FDA ? rr2 * rsq : fsqrt_(rr2);
  const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
  const float fac = K.bwenovh * (wq * wq * wq);
  const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
  const unsigned tg = (BOUNDP2 || UNI) ? 0u : __float_as_uint(C.y);
  const bool ftp2 = FT && !BOUNDP2 && !UNI && (tg & 0x80u) != 0u;
  const int pp2 = UNI ? u.k : BOUNDP2 ? p.ph : int(FT ? (tg & 0x7fu) : tg);
  const bool samephase = UNI || p.ph == pp2;
  const float4 ph2 = UNI ? u.a : sph[2 * pp2];
  const float4 ph2c = UNI ? u.c : sph[2 * SPH_MAXPHASES + pp2];  // {m tau_yield, -m log2 e, n - 1, DDTkh cs0}
  const float massp2 = BOUNDP2 ? K.massbound : (ftp2 ? sph[3 * SPH_MAXPHASES + pp2].x : ph2.x);
  const float rho1 = p.vr.w, rho2 = B.w;
  const float inv_rho2 = C.z;  // staged 1/rho2
  // m2/rho2: every per-pair use of 1/rho2 below comes with the mass of p2 (the reference's
  // products re-associated, rounding-level differences)
  const float massrhop = massp2 * inv_rho2;
  // momentum (pressure): -(p1 + p2)/(rho1 rho2) m2
  {
    const float p_vpm = (p.press + C.x) * (p.inv_rho * -massrhop);
    a.ax = fmaf(p_vpm, frx, a.ax);
    a.ay = fmaf(p_vpm, fry, a.ay);
    a.az = fmaf(p_vpm, frz, a.az);
  }
  // continuity
  const float rhop1over2 = rho1 * inv_rho2;
  float dvx = p.vr.x - B.x, dvy = p.vr.y - B.y, dvz = p.vr.z - B.z;
  const float dot = drx * dvx + dry * dvy + drz * dvz;  // dv.fr = fac (dr.dv)
  a.ar = fmaf(fac * dot, massrhop, a.ar);  // m2 fac (dr.dv) / rho2; x rho1 after the pass
  const float cbar = ph2.y;  // max(Cs0[pp2], Cs0[pp2])
  const float dot3 = fac * rr2;  // drx*frx+dry*fry+drz*frz
  const float inv_re = frcp(rr2 + K.eta2);
  // m2/rho2 dot3/(r^2+eta^2): the common factor of the DDT (Fourtakas) and Morris terms
  const float xdm = inv_re * massrhop * dot3;
  // density diffusion, only between particles of the same phase (JSphCpu_NN_FDA.cpp:181-199)
  // (branch-free: once the sum is FLT_MAX it stays FLT_MAX, since FLT_MAX +- a finite
  // pair term rounds back to FLT_MAX; a per-lane `if (a.delta != FLT_MAX)` costs exec-mask
  // branches in every pair)
  if (TDENSITY == 1) {
    const float visc_densi = ph2c.w * (rhop1over2 - 1.f) * inv_re;  // DDTkh cbar (...) / (r^2+eta^2)
    const float delta = (samephase ? visc_densi * dot3 * massp2 : 0.f);
    a.delta = (BOUNDP2 && !K.mdbc && ok) ? FLT_MAX : a.delta + delta;
    if (FT && ftp2 && ok && massp2 <= K.massfluid * 1.2f) a.delta = FLT_MAX;
  }
  if (TDENSITY == 2 || (TDENSITY == 3 && !BOUNDP2)) {
    // rho0 (1 + ddtgz drz)^(1/gamma) - rho0 as the reference evaluates it in float: the
    // three-term series of k_fluid_tiled (exact to 2e-6 of the term) removes the float
    // cancellation of the reference, which the NN parity bar (10x the reference's own
    // rounding floor) does not absorb: step-1 velocities moved 5.7e-7 against 2e-8
    const float rh = 1.f + K.ddtgz * drz;
    const float drhop = K.rhopzero * fexp2(K.ovgamma * flog2(rh)) - K.rhopzero;
    const float delta = (samephase && !ftp2 ? ph2c.w * ((rho2 - rho1) - drhop) * xdm : 0.f);
    a.delta = (BOUNDP2 && ok) ? FLT_MAX : a.delta - delta;
  }
  // multiphase shifting (JSphCpu_NN_FDA.cpp:202-209): a heavier-phase neighbour resets x
  // (ORDERED: a no-shift pair sets sx = FLT_MAX and every later pair leaves the sums alone)
  if (FT && SHIFT && ftp2 && ok && K.shiftmode == 1) {
    a.sx = FLT_MAX;  // every later pair leaves the sums alone (the reference's x != FLT_MAX test)
    a.ftsx = true;
  }
  if (SHIFT && (!ORDERED || a.sx != FLT_MAX)) {
    // (a heavier p1 phase differs from p2's: the phase test of the reference is implied)
    const bool heavy = !UNI && ok && !BOUNDP2 && (p.mph > ph2.x);
    const bool noshift = ok && BOUNDP2 && (K.shiftmode == 1 || (K.shiftmode == 2 && C.y != 0.f));
    const float mr = heavy ? 0.f : massrhop;  // a heavier-phase pair adds nothing (fma by 0)
    if (ORDERED) {
      a.sx = noshift ? FLT_MAX : (heavy ? 0.f : fmaf(massrhop, frx, a.sx));
    } else {  // fluid p2 only (noshift needs a bound p2)
      a.sx = fmaf(mr, frx, a.sx);
      a.hv = heavy ? true : a.hv;
    }
    a.sy = fmaf(mr, fry, a.sy);
    a.sz = fmaf(mr, frz, a.sz);
    a.sw = fmaf(-mr, dot3, a.sw);
  }
  // viscosity
  const float dot_rr2 = dot * inv_re;
  a.visc = max_nonneg(ok ? dot_rr2 : 0.f, a.visc);
  const float visco_nn = ph2.z;
  if (TVISCO == 1) {  // artificial
    if (dot < 0.f) {
      const float amubar = K.kernelh * dot_rr2;
      const float robar = (rho1 + rho2) * 0.5f;
      const float pi_visc = (-visco_nn * cbar * amubar * frcp(robar)) * massp2;
      a.ax = fmaf(-pi_visc, frx, a.ax);
      a.ay = fmaf(-pi_visc, fry, a.ay);
      a.az = fmaf(-pi_visc, frz, a.az);
    }
  } else if (TVISCO == NN_SPH_GRAD) {
    // GetVelocityGradients_SPH_tsym (JSphCpu_Tensors.cpp:173-181), no slip on the tensor at a
    // boundary p2 (u_g = 2 u_b - u_f, JSphCpu_NN_SPH.cpp:585-587); pairs outside the test
    // have fr = 0
    if (BOUNDP2) {
      dvx = 2.f * p.vr.x;
      dvy = 2.f * p.vr.y;
      dvz = 2.f * p.vr.z;
    }
    const float volp2 = -massrhop;
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
  } else if (TVISCO == 2 || TVISCO == 3) {  // Laminar (2) or constitutive equation (3) with the FDA velocity gradient
    if (BOUNDP2) {  // no slip on the tensor: u_g = 2 u_b - u_f with u_b = 0
      dvx = 2.f * p.vr.x;
      dvy = 2.f * p.vr.y;
      dvz = 2.f * p.vr.z;
    }
    // GetVelocityGradients_FDA + GetStrainRateTensor (JSphCpu_Tensors.cpp:40-82), in the
    // reference's operation order: the effective viscosity divides by the invariant, whose
    // explicit form cancels, so its rounding is part of the result (a closed form of the
    // rank-one gradient's invariant moved step-1 velocities 30x past the noise floor)
    const float irr2 = FDA ? rsq * rsq : frcp(rr2);
    const float tx = dvx * irr2, ty = dvy * irr2, tz = dvz * irr2;
    const float a11 = tx * drx, a12 = tx * dry, a13 = tx * drz;
    const float a21 = ty * drx, a22 = ty * dry, a23 = ty * drz;
    const float a31 = tz * drx, a32 = tz * dry, a33 = tz * drz;
    const float div_vel = (a11 + a22 + a33) * (1.f / 3.f);
    const float d11 = a11 - div_vel, d22 = a22 - div_vel, d33 = a33 - div_vel;
    const float s12 = a12 + a21, s13 = a13 + a31, s23 = a23 + a32;  // 2 d12, 2 d13, 2 d23
    const float ii1 = d11 * d22 + d22 * d33 + d11 * d33;
    // d_ij^2 = s_ij^2 / 4 exactly (powers of two scale without rounding)
    const float ii2 = 0.25f * (s12 * s12 + s23 * s23 + s13 * s13);
    const float ii_d = ii1 - ii2;
    const float dmag = fabsf(ii_d);  // sqrt(II_D * II_D)
    const float eta = nn_eta(K.nnbi != 0, dmag, ph2.w, visco_nn, ph2c, p.taumax, p.bimulti);
    a.visceta = max_nonneg(ok ? eta : 0.f, a.visceta);
    if constexpr (TVISCO == 2) {  // Morris operator: m2 2 eta dot3 / ((r^2+eta^2) rho2)
      const float vtemp = (2.f * eta) * xdm;
      a.ax = fmaf(vtemp, dvx, a.ax);
      a.ay = fmaf(vtemp, dvy, a.ay);
      a.az = fmaf(vtemp, dvz, a.az);
    } else {  // GetStressTensor: tau = 2 eta D
      const float e2 = 2.f * eta;
      const float d12 = 0.5f * s12, d13 = 0.5f * s13, d23 = 0.5f * s23;
      const float t11 = e2 * d11, t12 = e2 * d12, t13 = e2 * d13, t22 = e2 * d22, t23 = e2 * d23, t33 = e2 * d33;
      a.ax = fmaf(t11 * frx + t12 * fry + t13 * frz, massrhop, a.ax);
      a.ay = fmaf(t12 * frx + t22 * fry + t23 * frz, massrhop, a.ay);
      a.az = fmaf(t13 * frx + t23 * fry + t33 * frz, massrhop, a.az);
    }
  }
}

// Boundary p1 over fluid p2 (InteractionForcesBound_NN_FDA, JSphCpu_NN_FDA.cpp:48-113):
// continuity with MassFluid and the visc-dt maximum.
// FT: a floating p2 with its body's particle mass (JSphCpu_NN_FDA.cpp:89-93).
template <bool FT = false>
__device__ __forceinline__ void nn_bound_pair(const KConst& K, const NNP1& p, float drx, float dry, float drz,
                                              float rr2, bool ok, const float4& B, const float4& C, NNAcc& a,
                                              const float4* __restrict__ sph) {
  const float rad = fsqrt_(rr2);
  const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
  const float fac = K.bwenovh * (wq * wq * wq);
  const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
  const float dvx = p.vr.x - B.x, dvy = p.vr.y - B.y, dvz = p.vr.z - B.z;
  float m2 = K.massfluid;
  if (FT) {
    const unsigned tg = __float_as_uint(C.y);
    if (tg & 0x80u) m2 = sph[3 * SPH_MAXPHASES + (tg & 0x7fu)].x;
  }
  a.ar = fmaf(m2 * (dvx * frx + dvy * fry + dvz * frz), p.vr.w * C.z, a.ar);
  const float dot = drx * dvx + dry * dvy + drz * dvz;
  a.visc = fmaxf(ok ? dot * frcp(rr2 + K.eta2) : 0.f, a.visc);
}

// Staging of one row segment: positions relative to the item (sA + |A|^2), velrhop (sB),
// {press, tag} (sC): tag = phase index (fluid rows) or 1 for a fixed boundary particle.
// `same`: cleared when a record this thread stages is not a fluid particle of phase `uph`.
__device__ __forceinline__ void nn_stage(const KConst& K, unsigned rs, unsigned n, int xo, int dy, int dz,
                                         bool boundrow, const float4* __restrict__ poscell,
                                         const float4* __restrict__ velrhop, const float* __restrict__ press,
                                         const typecode* __restrict__ code, float4* __restrict__ sA,
                                         float4* __restrict__ sB, NNSC sC, unsigned dst = 0u, bool* same = nullptr,
                                         int uph = -1) {
  const float oy = float(dy) * K.scell, oz = float(dz) * K.scell;
  sA += dst;
  sB += dst;
  sC.c += dst;
  sC.t += dst;
  for (unsigned i = threadIdx.x; i < n; i += TB) {
    const float4 pc = poscell[rs + i];
    const int cx2 = int(DcelCellx(K.domcellcode, __float_as_uint(pc.w)));
    const float x2 = pc.x + float(cx2 - xo) * K.scell;
    const float y2 = pc.y + oy, z2 = pc.z + oz;
    sA[i] = make_float4(x2, y2, z2, x2 * x2 + y2 * y2 + z2 * z2);
    const float4 vr = velrhop[rs + i];
    sB[i] = vr;
    const typecode c = code[rs + i];
    // fluid rows: the phase (fluid) or, bit 7 set, the body index (floating)
    const unsigned tag = boundrow ? (CodeType(c) == 0 ? 1u : 0u)
                                  : (unsigned(c & CODE_MASKVALUE) | (CodeType(c) == CODE_TYPE_FLOATING ? 0x80u : 0u));
    sC.c[i] = make_float2(press[rs + i], frcp(vr.w));
    sC.t[i] = (unsigned char)tag;
    if (same) *same = *same && int(tag) == uph;
  }
}

// One pass of a p1 over its (2S+1)^2 rows of one kind (S = scelldiv), z-major then y, p2
// ascending.  KIND 0: fluid p1 / fluid p2, 1: fluid p1 / bound p2, 2: bound p1 / fluid p2.
template <int TVISCO, int TDENSITY, bool SHIFT, int KIND, int S, bool FT>
__device__ __forceinline__ void nn_pass(const KConst& K, const DivGrid& g, const RowCtx& rc, const NNP1& p, float thr,
                                        const unsigned* __restrict__ bc, const float4* __restrict__ poscell,
                                        const float4* __restrict__ velrhop, const float* __restrict__ press,
                                        const typecode* __restrict__ code, float4* __restrict__ sA,
                                        float4* __restrict__ sB, NNSC sC,
                                        const float4* __restrict__ sph, NNAcc& a) {
  const unsigned cellinit = (KIND == 1 ? 0u : g.boxfluid);
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  for (int dz = -S; dz <= S; dz++) {
    for (int dy = -S; dy <= S; dy++) {
      const int z = rc.cz + dz, y = rc.cy + dy;
      if (z < 0 || z >= g.ncz || y < 0 || y >= g.ncy) continue;  // block-uniform
      const unsigned rowbase = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
      const unsigned rs = bc[rowbase + rc.xa], re = bc[rowbase + rc.xb + 1];
      const unsigned ls = bc[rowbase + rc.lxa], le = bc[rowbase + rc.lxb + 1];
      for (unsigned seg = rs; seg < re; seg += NN_TCAP) {
        const unsigned segn = min(unsigned(NN_TCAP), re - seg);
        __syncthreads();
        nn_stage(K, seg, segn, rc.xo, dy, dz, KIND == 1, poscell, velrhop, press, code, sA, sB, sC);
        __syncthreads();
        const int w0 = int(max(ls, seg) - seg);
        const int w1 = rc.act ? max(w0, int(min(le, seg + segn)) - int(seg)) : w0;
        for (int off = w0; off < w1; off += 128) {
          unsigned long long c0, c1;
          test128(sA, off, min(w1 - off, 128), px2, py2, pz2, thr, c0, c1);
          int b0 = off;
          if (!c0) {
            c0 = c1;
            c1 = 0ull;
            b0 += 64;
          }
          // ascending p2, two per iteration (the first pair's sums are updated first)
          auto pop = [&]() -> int {
            const int j = b0 + int(__builtin_ctzll(c0 | (1ull << 63)));
            c0 &= c0 - 1ull;
            const bool e = c0 == 0ull;
            c0 = e ? c1 : c0;
            b0 = e ? b0 + 64 : b0;
            c1 = e ? 0ull : c1;
            return j;
          };
          while (c0) {
            const int j1 = pop();
            const bool two = c0 != 0ull;
            const int j2p = pop();
            const int j2 = two ? j2p : j1;
            const float4 A1 = sA[j1], A2 = sA[j2];
            const float4 B1 = sB[j1], B2 = sB[j2];
            float drx1 = p.x - A1.x, dry1 = p.y - A1.y, drz1 = p.z - A1.z;
            float drx2 = p.x - A2.x, dry2 = p.y - A2.y, drz2 = p.z - A2.z;
            float rr21 = drx1 * drx1 + dry1 * dry1 + drz1 * drz1;
            float rr22 = drx2 * drx2 + dry2 * dry2 + drz2 * drz2;
            const bool ok1 = rr21 <= K.kernelsize2 && rr21 >= ALMOSTZERO;
            const bool ok2 = two && rr22 <= K.kernelsize2 && rr22 >= ALMOSTZERO;
            // a pair outside the test: rr2 = 1e30 (kernel factor 0, finite terms)
            rr21 = ok1 ? rr21 : 1e30f;
            rr22 = ok2 ? rr22 : 1e30f;
            const float4 C1 = sC.ld(j1, KIND == 1), C2 = sC.ld(j2, KIND == 1);
            if (KIND == 2) {
              nn_bound_pair<FT>(K, p, drx1, dry1, drz1, rr21, ok1, B1, C1, a, sph);
              nn_bound_pair<FT>(K, p, drx2, dry2, drz2, rr22, ok2, B2, C2, a, sph);
            } else {
              nn_pair<TVISCO, TDENSITY, SHIFT, KIND == 1, true, FT>(K, sph, p, drx1, dry1, drz1, rr21, ok1, B1, C1, a);
              nn_pair<TVISCO, TDENSITY, SHIFT, KIND == 1, true, FT>(K, sph, p, drx2, dry2, drz2, rr22, ok2, B2, C2, a);
            }
          }
        }
      }
    }
  }
}

// Drain of one round of a mirrored unit's accepted candidates: four 64-bit words c0..c3 of
// staged records from bases b0..b3, compacted into one chain and popped two pairs per
// iteration with value selects only (the chain of drain_words, sph_interaction_tiled.hip).
// KIND 0: fluid p1 / fluid p2 (sx in mirrored order, see nn_pair), 2: bound p1 / fluid p2.
template <int TVISCO, int TDENSITY, bool SHIFT, int KIND, bool FT, bool UNI = false>
__device__ __forceinline__ void nn_drain4(const KConst& K, const float4* __restrict__ sph, const NNP1& p,
                                          unsigned long long c0, unsigned long long c1, unsigned long long c2,
                                          unsigned long long c3, int b0, int b1, int b2, int b3,
                                          const float4* __restrict__ sA, const float4* __restrict__ sB,
                                          const NNSC sC, NNAcc& a, const NNUni& u = NNUni{}) {
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
    const float4 A1 = sA[j1], B1 = sB[j1];
    float drx1 = p.x - A1.x, dry1 = p.y - A1.y, drz1 = p.z - A1.z;
    float rr21 = drx1 * drx1 + dry1 * dry1 + drz1 * drz1;
    const bool ok1 = rr21 <= K.kernelsize2 && rr21 >= ALMOSTZERO;
    rr21 = ok1 ? rr21 : 1e30f;
    float4 C1;
    if (UNI) {  // no phase tag: the unit's phase is known
      const float2 v = sC.c[j1];
      C1 = make_float4(v.x, 0.f, v.y, 0.f);
    } else {
      C1 = sC.ld(j1, KIND == 1);
    }
    if (KIND == 2) nn_bound_pair<FT>(K, p, drx1, dry1, drz1, rr21, ok1, B1, C1, a, sph);
    else nn_pair<TVISCO, TDENSITY, SHIFT, KIND == 1, false, FT, UNI>(K, sph, p, drx1, dry1, drz1, rr21, ok1, B1, C1,
                                                                    a, u);
    keep_w(A1, B1);  // 16-B LDS reads (sph_tiled.hpp)
  }
}

// A pass over the 9 fluid rows (KIND 0: fluid p1, 2: bound p1) in drain units of two
// point-mirrored rows ((dy,dz) with (-dy,-dz)) staged as one segment and drained as one
// set, then the item's own row (run_pass of sph_interaction_tiled.hip): a particle's
// candidate counts in mirrored rows complement each other, so the lanes' loop lengths are
// alike.  Every sum but the shifting x sum is order-free (up to rounding); a heavier-phase
// neighbour is flagged in a.hv and the caller redoes sx in the reference order.
template <int TVISCO, int TDENSITY, bool SHIFT, int KIND, int S, bool FT>
__device__ __forceinline__ void nn_pass_mirrored(const KConst& K, const DivGrid& g, const RowCtx& rc, const NNP1& p,
                                                 float thr, const unsigned* __restrict__ bc,
                                                 const float4* __restrict__ poscell,
                                                 const float4* __restrict__ velrhop, const float* __restrict__ press,
                                                 const typecode* __restrict__ code, float4* __restrict__ sA,
                                                 float4* __restrict__ sB, NNSC sC,
                                                 const float4* __restrict__ sph, NNAcc& a,
                                                 const NNUni& unph = NNUni{}) {
  // KIND 1 (bound p2) only where no pair can freeze the shifting sums (no shifting, or
  // ShiftMode Full): the caller keeps the reference order otherwise
  const unsigned cellinit = KIND == 1 ? 0u : g.boxfluid;
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  constexpr int NPAIR = ((2 * S + 1) * (2 * S + 1) - 1) / 2;  // mirrored row pairs, then the own row
  for (int u = 0; u <= NPAIR; u++) {
    int dza = 0, dya = 0;
    const bool paired = u < NPAIR;
    if (S == 1) {
      dza = (u == 0 || u == 1 || u == 2) ? -1 : 0;
      dya = (u == 0) ? -1 : (u == 1) ? 1 : (u == 2) ? 0 : (u == 3) ? -1 : 0;
    } else if (paired) {
      half_row(u, dya, dza);  // the 12 lower rows of the 5x5 half-cell stencil (sph_tiled.hpp)
    }
    unsigned rs[2] = {0, 0}, re[2] = {0, 0}, ls[2] = {0, 0}, le[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !paired) break;
      const int dz = k ? -dza : dza, dy = k ? -dya : dya;
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
    if (n0 + n1 <= unsigned(NN_TCAP)) {
      __syncthreads();
      bool same = KIND == 0 && unph.k >= 0 && p.p1uni;
      if (n0) nn_stage(K, rs[0], n0, rc.xo, dya, dza, KIND == 1, poscell, velrhop, press, code, sA, sB, sC, 0u, &same, unph.k);
      if (n1)
        nn_stage(K, rs[1], n1, rc.xo, -dya, -dza, KIND == 1, poscell, velrhop, press, code, sA, sB, sC, n0, &same, unph.k);
      // the block's vote (and the barrier after the staging): a single-phase unit (NNUni)
      const bool uni = KIND == 0 ? __syncthreads_and(int(same)) != 0 : (__syncthreads(), false);
      const int wa0 = int(ls[0] - rs[0]), wa1 = rc.act && n0 ? int(le[0] - rs[0]) : wa0;
      const int wb0 = int(n0 + ls[1] - rs[1]), wb1 = rc.act && n1 ? int(n0 + le[1] - rs[1]) : wb0;
      for (int off = 0;; off += 128) {  // a second round only for windows of > 128 candidates
        const int na = wa1 - wa0 - off, nb = wb1 - wb0 - off;
        if (na <= 0 && nb <= 0) break;
        unsigned long long c0, c1, c2, c3;
        test128(sA, wa0 + off, min(na, 128), px2, py2, pz2, thr, c0, c1);
        test128(sA, wb0 + off, min(nb, 128), px2, py2, pz2, thr, c2, c3);
        if (KIND == 0 && uni)
          nn_drain4<TVISCO, TDENSITY, SHIFT, KIND, FT, KIND == 0>(K, sph, p, c0, c1, c2, c3, wa0 + off, wa0 + off + 64,
                                                                  wb0 + off, wb0 + off + 64, sA, sB, sC, a, unph);
        else
          nn_drain4<TVISCO, TDENSITY, SHIFT, KIND, FT>(K, sph, p, c0, c1, c2, c3, wa0 + off, wa0 + off + 64, wb0 + off,
                                                   wb0 + off + 64, sA, sB, sC, a);
      }
    } else {  // too long for one segment: each row on its own, in TCAP segments
      for (int k = 0; k < 2; k++) {
        const int dz = k ? -dza : dza, dy = k ? -dya : dya;
        for (unsigned seg = rs[k]; seg < re[k]; seg += NN_TCAP) {
          const unsigned segn = min(unsigned(NN_TCAP), re[k] - seg);
          __syncthreads();
          nn_stage(K, seg, segn, rc.xo, dy, dz, KIND == 1, poscell, velrhop, press, code, sA, sB, sC, 0u);
          __syncthreads();
          const int w0 = int(max(ls[k], seg) - seg);
          const int w1 = rc.act ? max(w0, int(min(le[k], seg + segn)) - int(seg)) : w0;
          for (int off = w0; off < w1; off += 128) {
            unsigned long long c0, c1;
            test128(sA, off, min(w1 - off, 128), px2, py2, pz2, thr, c0, c1);
            nn_drain4<TVISCO, TDENSITY, SHIFT, KIND, FT>(K, sph, p, c0, c1, 0ull, 0ull, off, off + 64, 0, 0, sA, sB,
                                                     sC, a);
          }
        }
      }
    }
  }
}

// The shifting x sum of a fluid p1 over its fluid rows with the reference's reset: the
// reference visits z-major rows, p2 ascending, and a heavier-phase neighbour sets the sum to
// 0 (JSphCpu_NN_FDA.cpp:202-209), so the result is the sum of the terms AFTER the last
// heavier-phase pair in that order.  This sweep walks the same pairs BACKWARDS (rows from
// the last, p2 descending) and a lane stops at its first heavier-phase pair: the terms it
// added are exactly the reference's, summed in the reverse order (rounding only), and rows
// before that pair are never staged once every lane has stopped.  At a layer interface the
// heavier p1 meets the lighter phase in the rows above it, the last ones of the order, so a
// sweep typically stages 3 of the 9 rows.  Run for a block when any of its lanes met a
// heavier-phase neighbour in the mirrored pass (phase interfaces only); `need`: this lane did
// (the others keep their mirrored-order sum, which no reset touched).
template <int S, bool FT>
__device__ __forceinline__ float nn_sx_sweep(const KConst& K, const DivGrid& g, const RowCtx& rc, const NNP1& p,
                                             float thr, const unsigned* __restrict__ bc,
                                             const float4* __restrict__ poscell,
                                             const float4* __restrict__ velrhop, const float* __restrict__ press,
                                             const typecode* __restrict__ code, float4* __restrict__ sA,
                                             float4* __restrict__ sB, NNSC sC,
                                             const float4* __restrict__ sph, bool need, float sx_mirrored) {
  float sx = 0.f;
  bool live = rc.act && need;  // still summing (no heavier-phase pair met yet, backwards)
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  for (int dz = S; dz >= -S; dz--) {
    for (int dy = S; dy >= -S; dy--) {
      if (!__syncthreads_or(int(live))) return need ? sx : sx_mirrored;  // block-uniform exit
      const int z = rc.cz + dz, y = rc.cy + dy;
      if (z < 0 || z >= g.ncz || y < 0 || y >= g.ncy) continue;  // block-uniform
      const unsigned rowbase = g.boxfluid + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
      const unsigned rs = bc[rowbase + rc.xa], re = bc[rowbase + rc.xb + 1];
      const unsigned ls = bc[rowbase + rc.lxa], le = bc[rowbase + rc.lxb + 1];
      if (re == rs) continue;
      // segments from the row's end
      for (unsigned segn0 = (re - rs - 1u) % unsigned(NN_TCAP) + 1u, seg = re - segn0, segn = segn0;;) {
        __syncthreads();
        nn_stage(K, seg, segn, rc.xo, dy, dz, false, poscell, velrhop, press, code, sA, sB, sC, 0u);
        __syncthreads();
        const int w0 = int(max(ls, seg) - seg);
        const int w1 = live ? max(w0, int(min(le, seg + segn)) - int(seg)) : w0;
        // chunks of 128 from the window's end, each drained highest candidate first
        for (int off = w0 + ((w1 - w0 - 1) / 128) * 128; live && off >= w0 && w1 > w0; off -= 128) {
          unsigned long long c0, c1;
          test128(sA, off, min(w1 - off, 128), px2, py2, pz2, thr, c0, c1);
          int b1 = off + 64;
          if (!c1) {
            c1 = c0;
            c0 = 0ull;
            b1 = off;
          }
          while (live && c1) {  // descending p2
            const int k = 63 - int(__builtin_clzll(c1));
            const int j = b1 + k;
            c1 &= ~(1ull << k);
            const bool e = c1 == 0ull;
            c1 = e ? c0 : c1;
            b1 = e ? off : b1;
            c0 = e ? 0ull : c0;
            const float4 A = sA[j], C = sC.ld(j, false);
            float drx = p.x - A.x;
            const float dry = p.y - A.y, drz = p.z - A.z;
            float rr2 = drx * drx + dry * dry + drz * drz;
            const bool ok = rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO;
            drx = ok ? drx : 0.f;
            rr2 = ok ? rr2 : 1e30f;
            const float rad = fsqrt_(rr2);
            const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
            const float fac = K.bwenovh * (wq * wq * wq);
            const float frx = fac * drx;
            const unsigned tg = __float_as_uint(C.y);
            const int pp2 = int(FT ? (tg & 0x7fu) : tg);
            const float mph2 = sph[2 * pp2].x;  // the heavier-phase test: phase constants (a body's index too)
            const float massp2 = (FT && (tg & 0x80u)) ? sph[3 * SPH_MAXPHASES + pp2].x : mph2;
            const bool heavy = ok && (p.mph > mph2);
            if (heavy) live = false;  // the reference's reset: nothing before this pair counts
            else sx += (massp2 * C.z) * frx;
          }
        }
        if (seg == rs) break;
        seg -= unsigned(NN_TCAP);
        segn = unsigned(NN_TCAP);
      }
    }
  }
  return need ? sx : sx_mirrored;
}

#ifndef SPH_NN_WAVES
#define SPH_NN_WAVES 4  // register budget for 4 waves per SIMD (<= 128 VGPRs)
#endif
#if SPH_NN_WAVES
#define SPH_NN_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(SPH_NN_WAVES, SPH_NN_WAVES)))
#else
#define SPH_NN_WAVES_ATTR
#endif

template <int TVISCO, int TDENSITY, bool SHIFT, int S, bool FT>
__global__ __launch_bounds__(TB) SPH_NN_WAVES_ATTR void k_nn_tiled(DevScalars* __restrict__ sc, const uint4* __restrict__ items,
                                                 unsigned* __restrict__ qctr, const float4* __restrict__ poscell,
                                                 const float4* __restrict__ velrhop, const float* __restrict__ press,
                                                 const typecode* __restrict__ code, const unsigned* __restrict__ bc,
                                                 DivGrid g, KConst K, const float4* __restrict__ phases,
                                                 float4* __restrict__ arace, float4* __restrict__ shiftpos,
                                                 float* __restrict__ viscoeta, float4* __restrict__ tau,
                                                 const float* __restrict__ ftmassp) {
  __shared__ float4 sAB[2 * NN_TCAP];  // sA then sB: the candidate test's over-read stays inside
  float4* const sA = sAB;
  float4* const sB = sAB + NN_TCAP;
  __shared__ float2 sC2[NN_TCAP];  // {press, 1/rho}
  __shared__ unsigned char sT[NN_TCAP];  // tag
  const NNSC sC = {sC2, sT};
  // phase table (+ FT: a fourth row, the particle mass of every floating body)
  __shared__ float4 sph[(FT ? 4 : 3) * SPH_MAXPHASES];
  __shared__ unsigned s_item;
  __shared__ unsigned char s_perm[TB];
  __shared__ unsigned s_nwave[4];
  if (threadIdx.x < 3 * SPH_MAXPHASES) sph[threadIdx.x] = phases[threadIdx.x];
  if (FT && threadIdx.x < SPH_MAXPHASES)
    sph[3 * SPH_MAXPHASES + threadIdx.x] =
        make_float4(threadIdx.x < unsigned(K.nftbodies) ? ftmassp[threadIdx.x] : 0.f, 0.f, 0.f, 0.f);
  float viscmax = 0.f, ace2max = 0.f, etamax = 0.f;
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
    const unsigned p1 = item.z + lane_order(poscell, item.z, item.w - item.z, 0.5f * K.scell, s_perm, s_nwave);
    const bool act = threadIdx.x < item.w - item.z;
    NNP1 p;
    int cx1 = ia;
    if (act) {
      const float4 pc1 = poscell[p1];
      cx1 = int(DcelCellx(K.domcellcode, __float_as_uint(pc1.w)));
      p.x = pc1.x + float(cx1 - xo) * K.scell;
      p.y = pc1.y;
      p.z = pc1.z;
      p.vr = velrhop[p1];
      p.press = press[p1];
      // a floating p1's code value is its body index, which the reference uses as its phase
      p.ph = bitem ? 0 : int(code[p1] & CODE_MASKVALUE);
    } else {
      p.x = p.y = p.z = 1e30f;
      p.vr = make_float4(0.f, 0.f, 0.f, 1.f);
      p.press = 0.f;
      p.ph = 0;
    }
    p.inv_rho = frcp(p.vr.w);
    p.mph = sph[2 * p.ph].x;
    p.taumax = sph[2 * p.ph + 1].z;
    p.bimulti = sph[2 * p.ph + 1].w;
    // the item's phase: that of its first particle when it is a fluid particle (NNUni)
    NNUni u;
    {
      const typecode c0 = code[item.z];
      u.k = (bitem || CodeType(c0) != CODE_TYPE_FLUID) ? -1 : int(c0 & CODE_MASKVALUE);
      u.k = __builtin_amdgcn_readfirstlane(u.k);
      const int kk = u.k < 0 ? 0 : u.k;
      const float4 ta = sph[2 * kk], tc = sph[2 * SPH_MAXPHASES + kk];
      u.a = make_float4(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ta.x))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ta.y))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ta.z))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ta.w))));
      u.c = make_float4(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(tc.x))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(tc.y))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(tc.z))),
                        __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(tc.w))));
    }
    p.uph = u.k;
    p.p1uni = !act || (int(code[p1] & CODE_MASKVALUE) == u.k && CodeType(code[p1]) == CODE_TYPE_FLUID);
    const int lxa = max(cx1 - S, 0), lxb = min(cx1 + S, g.ncx - 1);
    const float thr = K.kernelsize2 * 1.0001f - (p.x * p.x + p.y * p.y + p.z * p.z);
    const RowCtx rc{cy, cz, xa, xb, lxa, lxb, xo, act, p1};
    if (bitem) {
      NNAcc f = {};
      nn_pass_mirrored<TVISCO, TDENSITY, SHIFT, 2, S, FT>(K, g, rc, p, thr, bc, poscell, velrhop, press, code, sA, sB, sC,
                                                   sph, f);
      if (act) {
        arace[p1] = make_float4(0.f, 0.f, 0.f, (f.ar != 0.f || f.visc != 0.f) ? 0.f + f.ar : 0.f);
        viscmax = fmaxf(viscmax, f.visc);
      }
      continue;
    }
    // fluid p1: the fluid pass, then the bound pass; the shifting sums carry over
    // (shiftposfs[p1] is stored by the first pass and loaded by the second)
    NNAcc f = {}, b = {};
    // a floating p1 gets no DDT and no shifting (JSphCpu_NN_FDA.cpp:159-164)
    const bool ftp1 = FT && act && CodeType(code[p1]) == CODE_TYPE_FLOATING;
    if (ftp1) {
      if (TDENSITY) f.delta = FLT_MAX;
      if (SHIFT) {
        f.sx = FLT_MAX;
        f.ftsx = true;
      }
    }
    nn_pass_mirrored<TVISCO, TDENSITY, SHIFT, 0, S, FT>(K, g, rc, p, thr, bc, poscell, velrhop, press, code, sA, sB,
                                                     sC, sph, f, u);
    if (SHIFT && __syncthreads_or(int(f.hv)))
      f.sx = nn_sx_sweep<S, FT>(K, g, rc, p, thr, bc, poscell, velrhop, press, code, sA, sB, sC, sph, f.hv, f.sx);
    if (FT && f.ftsx) f.sx = FLT_MAX;  // x stays FLT_MAX once set (no reset after it)
    b.sx = f.sx;
    b.sy = f.sy;
    b.sz = f.sz;
    b.sw = f.sw;
    if (FT) {  // the bound-row call starts over for a floating p1 too (deltap1, shiftposfsp1.x)
      b.ftsx = f.ftsx;
      if (ftp1 && TDENSITY) b.delta = FLT_MAX;
    }
    // the first no-shift bound pair (ShiftMode NoBound/NoFixed) freezes every shifting sum:
    // only then is the bound pass order-dependent (uniform branch)
    if (SHIFT && (K.shiftmode == 1 || K.shiftmode == 2))
      nn_pass<TVISCO, TDENSITY, SHIFT, 1, S, FT>(K, g, rc, p, thr, bc, poscell, velrhop, press, code, sA, sB, sC, sph, b);
    else
      nn_pass_mirrored<TVISCO, TDENSITY, SHIFT, 1, S, FT>(K, g, rc, p, thr, bc, poscell, velrhop, press, code, sA, sB, sC,
                                                   sph, b);
    if (FT && b.ftsx) b.sx = FLT_MAX;
    f.ar *= p.vr.w;  // the continuity sums' common rho1 (nn_pair)
    b.ar *= p.vr.w;
    if (act) {
      // the two CPU passes' stores (JSphCpu_NN_FDA.cpp:278-296).  With shifting configured
      // the reference instantiates every interaction with shift=true (the predictor's too,
      // whose sums ComputeSymplecticPre then ignores), so both passes always store.
      const bool store = SHIFT || K.shiftmode != 0;
      float ar = 0.f, ax = 0.f, ay = 0.f, az = 0.f, delta = 0.f;
      if (store || f.ar != 0.f || f.ax != 0.f || f.ay != 0.f || f.az != 0.f || f.visc != 0.f) {
        if (TDENSITY) delta = (f.delta == FLT_MAX ? FLT_MAX : 0.f + f.delta);
        ar = f.ar;
        ax = f.ax;
        ay = f.ay;
        az = f.az;
      }
      if (store || b.ar != 0.f || b.ax != 0.f || b.ay != 0.f || b.az != 0.f || b.visc != 0.f) {
        if (TDENSITY) delta = (delta == FLT_MAX || b.delta == FLT_MAX ? FLT_MAX : delta + b.delta);
        ar += b.ar;
        ax += b.ax;
        ay += b.ay;
        az += b.az;
      }
      if (TDENSITY && delta != FLT_MAX) ar += delta;
      if (K.sim2d) ay = 0.f;  // Simulate2D: Acec[].y = 0 (JSphCpuSingle.cpp:614-620)
      arace[p1] = make_float4(ax, ay, az, ar);
      if (SHIFT) shiftpos[p1] = make_float4(b.sx, b.sy, b.sz, b.sw);
      viscmax = fmaxf(viscmax, fmaxf(f.visc, b.visc));
      etamax = fmaxf(etamax, fmaxf(f.visceta, b.visceta));
      // SPH gradients: the viscous force and so AceMax come from the second pass (k_nn_visc)
      if (TVISCO != NN_SPH_GRAD && TVISCO != NN_SPH_ART) ace2max = fmaxf(ace2max, ax * ax + ay * ay + az * az);
      if constexpr (TVISCO == NN_SPH_GRAD) {
        // gradvel[p1] += fluid sums, += bound sums (JSphCpu_NN_SPH.cpp:608-615), then
        // _Visco_eta (strain rate tensor + effective viscosity of p1's phase, :171-222)
        // and for ConstEq _Visco_Stress_tensor (tau = 2 eta D, :128-166)
        const float gxx = f.gxx + b.gxx, gxy = f.gxy + b.gxy, gxz = f.gxz + b.gxz;
        const float gyy = f.gyy + b.gyy, gyz = f.gyz + b.gyz, gzz = f.gzz + b.gzz;
        float d[6];
        const float dmag = nn_strain_rate(gxx, gxy, gxz, gyy, gyz, gzz, d);
        const float4 pa = sph[2 * p.ph], pc = sph[2 * SPH_MAXPHASES + p.ph];
        const float eta = nn_eta(K.nnbi != 0, dmag, pa.w, pa.z, pc, p.taumax, p.bimulti);
        viscoeta[p1] = eta;
        etamax = fmaxf(etamax, eta);
        if (K.nntvisco == 3) {
          const float e2 = 2.f * eta;
          tau[2 * p1] = make_float4(e2 * d[0], e2 * d[1], e2 * d[2], e2 * d[3]);
          tau[2 * p1 + 1] = make_float4(e2 * d[4], e2 * d[5], 0.f, 0.f);
        }
      }
    }
  }
  wave_max_atomic(sc, RED_VISCDT, viscmax);
  wave_max_atomic(sc, RED_ACEMAX2, ace2max);
  wave_max_atomic(sc, RED_VISCETA, etamax);
  // (the queue counters are zeroed by k_items_place, or by the solver before an interaction
  // without a new item list)
}

void launch_nn_tiled(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                     const float4* poscell, const float4* velrhop, const float* press, const typecode* code,
                     const unsigned* begincell, DivGrid g, const KConst& K, const float4* phases, float4* arace,
                     float4* shiftpos, bool shift, float* viscoeta, float4* tau, const float* ftmassp) {
  // CellMode: cells of 2h (S = 1) or of h (S = 2); floating bodies (FT)
#define SPH_NN(TV, TD, SH)                                                                                         \
  if (ftmassp && K.scelldiv == 2)                                                                                  \
    hipLaunchKernelGGL((k_nn_tiled<TV, TD, SH, 2, true>), dim3(fit_grid((const void*)&k_nn_tiled<TV, TD, SH, 2, true>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,         \
                       poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,    \
                       ftmassp);                                                                                   \
  else if (ftmassp)                                                                                                \
    hipLaunchKernelGGL((k_nn_tiled<TV, TD, SH, 1, true>), dim3(fit_grid((const void*)&k_nn_tiled<TV, TD, SH, 1, true>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,         \
                       poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,    \
                       ftmassp);                                                                                   \
  else if (K.scelldiv == 2)                                                                                        \
    hipLaunchKernelGGL((k_nn_tiled<TV, TD, SH, 2, false>), dim3(fit_grid((const void*)&k_nn_tiled<TV, TD, SH, 2, false>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,        \
                       poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,    \
                       ftmassp);                                                                                   \
  else                                                                                                             \
    hipLaunchKernelGGL((k_nn_tiled<TV, TD, SH, 1, false>), dim3(fit_grid((const void*)&k_nn_tiled<TV, TD, SH, 1, false>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,        \
                       poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,    \
                       ftmassp)
#define SPH_NN_TD(TV, SH)          \
  switch (K.tdensity) {            \
    case 0: SPH_NN(TV, 0, SH); break; \
    case 1: SPH_NN(TV, 1, SH); break; \
    case 2: SPH_NN(TV, 2, SH); break; \
    default: SPH_NN(TV, 3, SH); break; \
  }
#define SPH_NN_TV(SH)                                                          \
  if (K.nnvelgrad == 2) {                                                      \
    if (K.nntvisco == 1) SPH_NN_TD(NN_SPH_ART, SH) else SPH_NN_TD(NN_SPH_GRAD, SH) \
  } else if (K.nntvisco == 1) SPH_NN_TD(1, SH)                                 \
  else if (K.nntvisco == 2) SPH_NN_TD(2, SH)                                   \
  else SPH_NN_TD(3, SH)
#ifdef SPH_DIAG_HEADLINE_ONLY
  // diagnostic builds (kernel A/B at cfg5 only): the one instantiation pair of BASELINE cfg5
  if (K.nnvelgrad == 2 || K.nntvisco != 2 || K.tdensity != 3 || ftmassp || K.scelldiv != 1)
    throw std::runtime_error("SPH_DIAG_HEADLINE_ONLY build: cfg2 / cfg5 kernels only");
  if (shift) hipLaunchKernelGGL((k_nn_tiled<2, 3, true, 1, false>), dim3(fit_grid((const void*)&k_nn_tiled<2, 3, true, 1, false>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,
                                poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,
                                ftmassp);
  else hipLaunchKernelGGL((k_nn_tiled<2, 3, false, 1, false>), dim3(fit_grid((const void*)&k_nn_tiled<2, 3, false, 1, false>, nblocks)), dim3(TB), 0, stm, sc, items, qctr,
                          poscell, velrhop, press, code, begincell, g, K, phases, arace, shiftpos, viscoeta, tau,
                          ftmassp);
#else
  if (shift) {
    SPH_NN_TV(true)
  } else {
    SPH_NN_TV(false)
  }
#endif
#undef SPH_NN_TV
#undef SPH_NN_TD
#undef SPH_NN
}

// ---------------------------------------------------------------------------------------
// Second pass of the SPH velocity gradients: the viscous force of each fluid p1 over its
// fluid rows, then its bound rows (InteractionForcesFluid_NN_SPH_Morris / _ConsEq,
// JSphCpu_NN_SPH.cpp:228-446; GPU twins JSphGpu_NN_ker.cu:935-1120).  Every sum is
// order-free, so all rows are drained in point-mirrored units.  Records of 48 B:
//   sA {x, y, z, |A|^2} (item-relative position), and per mode
//   VM_ART    sB {v, rho}     sC {m2, visco(pp2), cs0(pp2), 0}
//   VM_MORRIS sB {v, rho}     sC {m2, eta2, 0, 0}
//   VM_CONSEQ sB {txx, txy, txz, tyy} sC {tyz, tzz, rho2, m2}
// A bound p2 takes p1's phase, MassBound, and p1's eta / stress tensor (:305, :426); its
// velocity difference is 2 v1 (no slip, :403-405).
constexpr int VM_ART = 1, VM_MORRIS = 2, VM_CONSEQ = 3;
#ifndef SPH_NNV_TCAP
#define SPH_NNV_TCAP 408  // 48-B records: 408 + pad + tables keep 8 blocks per CU (<= 20 KB)
#endif
constexpr int NNV_TCAP = SPH_NNV_TCAP;

struct NNVP1 {
  float x, y, z;
  float4 vr;                // velocity, rho
  float eta;                // Morris: visco_eta[p1]
  float4 ta, tb;            // ConsEq: tau[p1] {xx, xy, xz, yy}, {yz, zz}
  float visco, cs0;         // artificial: p1's phase (bound p2)
};

template <int VM>
__device__ __forceinline__ void nnv_stage(const KConst& K, unsigned rs, unsigned n, unsigned dst, int xo, int dy,
                                          int dz, bool boundrow, const float4* __restrict__ poscell,
                                          const float4* __restrict__ velrhop, const typecode* __restrict__ code,
                                          const float* __restrict__ viscoeta, const float4* __restrict__ tau,
                                          const float4* __restrict__ sph, float4* __restrict__ sA,
                                          float4* __restrict__ sB, float4* __restrict__ sC,
                                          const float* __restrict__ ftmassp) {
  const float oy = float(dy) * K.scell, oz = float(dz) * K.scell;
  for (unsigned i = threadIdx.x; i < n; i += TB) {
    const unsigned q = rs + i;
    const float4 pc = poscell[q];
    const int cx2 = int(DcelCellx(K.domcellcode, __float_as_uint(pc.w)));
    const float x2 = pc.x + float(cx2 - xo) * K.scell;
    const float y2 = pc.y + oy, z2 = pc.z + oz;
    sA[dst + i] = make_float4(x2, y2, z2, x2 * x2 + y2 * y2 + z2 * z2);
    const typecode cq = code[q];
    const unsigned ph = boundrow ? 0u : unsigned(cq & CODE_MASKVALUE);
    // a floating p2: its body's particle mass (JSphCpu_NN_SPH.cpp:283-288, 391-396); its
    // body index doubles as the phase index of the phase constants, as in the reference
    const float m2 = boundrow ? K.massbound
                              : ((ftmassp && CodeType(cq) == CODE_TYPE_FLOATING) ? ftmassp[ph] : sph[2 * ph].x);
    if constexpr (VM == VM_CONSEQ) {
      const float rho2 = velrhop[q].w;
      if (boundrow) {  // tau of p1 is used for a bound p2
        sB[dst + i] = make_float4(0.f, 0.f, 0.f, 0.f);
        sC[dst + i] = make_float4(0.f, 0.f, rho2, m2);
      } else {
        const float4 ta = tau[2 * q], tb = tau[2 * q + 1];
        sB[dst + i] = ta;
        sC[dst + i] = make_float4(tb.x, tb.y, rho2, m2);
      }
    } else {
      sB[dst + i] = velrhop[q];
      if constexpr (VM == VM_MORRIS)
        sC[dst + i] = make_float4(m2, boundrow ? 0.f : viscoeta[q], 0.f, 0.f);
      else
        sC[dst + i] = make_float4(m2, sph[2 * ph].z, sph[2 * ph].y, 0.f);
    }
  }
}

// One pair (the reference's pair test rr2 <= KernelSize2 && rr2 >= ALMOSTZERO; a pair that
// fails it comes in with dr = 0, rr2 = 1e30: fr = 0, and every term adds +0).
template <int VM, bool BOUNDP2>
__device__ __forceinline__ void nnv_pair(const KConst& K, const NNVP1& p, float drx, float dry, float drz, float rr2,
                                         const float4& B, const float4& C, float3& acc) {
  const float rad = fsqrt_(rr2);
  const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
  const float fac = K.bwenovh * (wq * wq * wq);
  const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
  if constexpr (VM == VM_CONSEQ) {
    // tau_sum = tau1 + tau2 (tau2 = tau1 for a bound p2); (tau_sum . fr) / rho2 * m2
    const float sxx = p.ta.x + (BOUNDP2 ? p.ta.x : B.x), sxy = p.ta.y + (BOUNDP2 ? p.ta.y : B.y);
    const float sxz = p.ta.z + (BOUNDP2 ? p.ta.z : B.z), syy = p.ta.w + (BOUNDP2 ? p.ta.w : B.w);
    const float syz = p.tb.x + (BOUNDP2 ? p.tb.x : C.x), szz = p.tb.y + (BOUNDP2 ? p.tb.y : C.y);
    const float ir2 = frcp(C.z);
    const float m2 = C.w;
    acc.x = fmaf((sxx * frx + sxy * fry + sxz * frz) * ir2, m2, acc.x);
    acc.y = fmaf((sxy * frx + syy * fry + syz * frz) * ir2, m2, acc.y);
    acc.z = fmaf((sxz * frx + syz * fry + szz * frz) * ir2, m2, acc.z);
  } else {
    const float dvx = BOUNDP2 ? 2.f * p.vr.x : p.vr.x - B.x;
    const float dvy = BOUNDP2 ? 2.f * p.vr.y : p.vr.y - B.y;
    const float dvz = BOUNDP2 ? 2.f * p.vr.z : p.vr.z - B.z;
    const float m2 = C.x;
    const float rho2 = B.w;
    if constexpr (VM == VM_MORRIS) {
      // temp = (eta1 + eta2) / ((r2 + eta^2) rho2); vtemp = m2 temp (dr . fr)
      const float eta2 = BOUNDP2 ? p.eta : C.y;
      const float temp = (p.eta + eta2) * frcp((rr2 + K.eta2) * rho2);
      const float vtemp = m2 * temp * (fac * rr2);
      acc.x = fmaf(vtemp, dvx, acc.x);
      acc.y = fmaf(vtemp, dvy, acc.y);
      acc.z = fmaf(vtemp, dvz, acc.z);
    } else {  // artificial, with the phase of p2 (p1's for a bound p2)
      const float dot = drx * dvx + dry * dvy + drz * dvz;
      if (dot < 0.f) {
        const float visco = BOUNDP2 ? p.visco : C.y, cbar = BOUNDP2 ? p.cs0 : C.z;
        const float dot_rr2 = dot * frcp(rr2 + K.eta2);
        const float amubar = K.kernelh * dot_rr2;
        const float robar = (p.vr.w + rho2) * 0.5f;
        const float pi_visc = (-visco * cbar * amubar * frcp(robar)) * m2;
        acc.x = fmaf(-pi_visc, frx, acc.x);
        acc.y = fmaf(-pi_visc, fry, acc.y);
        acc.z = fmaf(-pi_visc, frz, acc.z);
      }
    }
  }
}

// The accepted candidates of one round (four 64-bit words), two pairs per iteration.
template <int VM, bool BOUNDP2>
__device__ __forceinline__ void nnv_drain4(const KConst& K, const NNVP1& p, unsigned long long c0,
                                           unsigned long long c1, unsigned long long c2, unsigned long long c3, int b0,
                                           int b1, int b2, int b3, const float4* __restrict__ sA,
                                           const float4* __restrict__ sB, const float4* __restrict__ sC,
                                           float3& acc) {
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
    const int j2 = two ? j2p : j1;
    const float4 A1 = sA[j1], A2 = sA[j2];
    const float4 B1 = sB[j1], B2 = sB[j2];
    const float4 C1 = sC[j1], C2 = sC[j2];
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
    nnv_pair<VM, BOUNDP2>(K, p, drx1, dry1, drz1, rr21, B1, C1, acc);
    nnv_pair<VM, BOUNDP2>(K, p, drx2, dry2, drz2, rr22, B2, C2, acc);
  }
}

// A pass of the p1 over its (2S+1)^2 rows of one kind in point-mirrored drain units (the
// units of nn_pass_mirrored), rows too long for one segment row by row in NNV_TCAP segments.
template <int VM, bool BOUNDP2, int S>
__device__ __forceinline__ float3 nnv_pass(const KConst& K, const DivGrid& g, const RowCtx& rc, const NNVP1& p,
                                           float thr, const unsigned* __restrict__ bc,
                                           const float4* __restrict__ poscell, const float4* __restrict__ velrhop,
                                           const typecode* __restrict__ code, const float* __restrict__ viscoeta,
                                           const float4* __restrict__ tau, const float4* __restrict__ sph,
                                           float4* __restrict__ sA, float4* __restrict__ sB,
                                           float4* __restrict__ sC, const float* __restrict__ ftmassp) {
  float3 acc = make_float3(0.f, 0.f, 0.f);
  const unsigned cellinit = BOUNDP2 ? 0u : g.boxfluid;
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  constexpr int NPAIR = ((2 * S + 1) * (2 * S + 1) - 1) / 2;
  for (int u = 0; u <= NPAIR; u++) {
    int dza = 0, dya = 0;
    const bool paired = u < NPAIR;
    if (S == 1) {
      dza = (u == 0 || u == 1 || u == 2) ? -1 : 0;
      dya = (u == 0) ? -1 : (u == 1) ? 1 : (u == 2) ? 0 : (u == 3) ? -1 : 0;
    } else if (paired) {
      half_row(u, dya, dza);
    }
    unsigned rs[2] = {0, 0}, re[2] = {0, 0}, ls[2] = {0, 0}, le[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !paired) break;
      const int dz = k ? -dza : dza, dy = k ? -dya : dya;
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
    if (n0 + n1 <= unsigned(NNV_TCAP)) {
      __syncthreads();
      if (n0)
        nnv_stage<VM>(K, rs[0], n0, 0u, rc.xo, dya, dza, BOUNDP2, poscell, velrhop, code, viscoeta, tau, sph, sA, sB,
                      sC, ftmassp);
      if (n1)
        nnv_stage<VM>(K, rs[1], n1, n0, rc.xo, -dya, -dza, BOUNDP2, poscell, velrhop, code, viscoeta, tau, sph, sA,
                      sB, sC, ftmassp);
      __syncthreads();
      const int wa0 = int(ls[0] - rs[0]), wa1 = rc.act && n0 ? int(le[0] - rs[0]) : wa0;
      const int wb0 = int(n0 + ls[1] - rs[1]), wb1 = rc.act && n1 ? int(n0 + le[1] - rs[1]) : wb0;
      for (int off = 0;; off += 128) {
        const int na = wa1 - wa0 - off, nb = wb1 - wb0 - off;
        if (na <= 0 && nb <= 0) break;
        unsigned long long c0, c1, c2, c3;
        test128(sA, wa0 + off, min(na, 128), px2, py2, pz2, thr, c0, c1);
        test128(sA, wb0 + off, min(nb, 128), px2, py2, pz2, thr, c2, c3);
        nnv_drain4<VM, BOUNDP2>(K, p, c0, c1, c2, c3, wa0 + off, wa0 + off + 64, wb0 + off, wb0 + off + 64, sA, sB,
                                sC, acc);
      }
    } else {
      for (int k = 0; k < 2; k++) {
        const int dz = k ? -dza : dza, dy = k ? -dya : dya;
        for (unsigned seg = rs[k]; seg < re[k]; seg += NNV_TCAP) {
          const unsigned segn = min(unsigned(NNV_TCAP), re[k] - seg);
          __syncthreads();
          nnv_stage<VM>(K, seg, segn, 0u, rc.xo, dy, dz, BOUNDP2, poscell, velrhop, code, viscoeta, tau, sph, sA, sB,
                        sC, ftmassp);
          __syncthreads();
          const int w0 = int(max(ls[k], seg) - seg);
          const int w1 = rc.act ? max(w0, int(min(le[k], seg + segn)) - int(seg)) : w0;
          for (int off = w0; off < w1; off += 128) {
            unsigned long long c0, c1;
            test128(sA, off, min(w1 - off, 128), px2, py2, pz2, thr, c0, c1);
            nnv_drain4<VM, BOUNDP2>(K, p, c0, c1, 0ull, 0ull, off, off + 64, 0, 0, sA, sB, sC, acc);
          }
        }
      }
    }
  }
  return acc;
}

template <int VM, int S>
__global__ __launch_bounds__(TB) void k_nn_visc(DevScalars* __restrict__ sc, const uint4* __restrict__ items,
                                                unsigned* __restrict__ qctr, const float4* __restrict__ poscell,
                                                const float4* __restrict__ velrhop, const typecode* __restrict__ code,
                                                const float* __restrict__ viscoeta, const float4* __restrict__ tau,
                                                const unsigned* __restrict__ bc, DivGrid g, KConst K,
                                                const float4* __restrict__ phases, float4* __restrict__ arace,
                                                const float* __restrict__ ftmassp) {
  __shared__ float4 sABC[3 * NNV_TCAP];  // sA, sB, sC: the candidate test's over-read stays inside
  float4* const sA = sABC;
  float4* const sB = sABC + NNV_TCAP;
  float4* const sC = sABC + 2 * NNV_TCAP;
  __shared__ float4 sph[2 * SPH_MAXPHASES];
  __shared__ unsigned s_item;
  __shared__ unsigned char s_perm[TB];
  __shared__ unsigned s_nwave[4];
  if (threadIdx.x < 2 * SPH_MAXPHASES) sph[threadIdx.x] = phases[threadIdx.x];
  float ace2max = 0.f;
  ItemCursor<true> cur(qctr);
  for (;;) {
    const unsigned it = cur.next(&s_item);
    if (it == ITEM_NONE) break;
    const uint4 item = items[it];
    const int cy = int(item.x & 0xffffu), cz = int((item.x >> 16) & 0x7fffu);
    const int ia = int(item.y & 0xffffu), ib = int(item.y >> 16);
    const int xo = (ia + ib + 1) >> 1;
    const int xa = max(ia - S, 0), xb = min(ib + S, g.ncx - 1);
    const unsigned p1 = item.z + lane_order(poscell, item.z, item.w - item.z, 0.5f * K.scell, s_perm, s_nwave);
    const bool act = threadIdx.x < item.w - item.z;
    NNVP1 p;
    int cx1 = ia;
    p.eta = 0.f;
    p.ta = p.tb = make_float4(0.f, 0.f, 0.f, 0.f);
    p.visco = p.cs0 = 0.f;
    if (act) {
      const float4 pc1 = poscell[p1];
      cx1 = int(DcelCellx(K.domcellcode, __float_as_uint(pc1.w)));
      p.x = pc1.x + float(cx1 - xo) * K.scell;
      p.y = pc1.y;
      p.z = pc1.z;
      p.vr = velrhop[p1];
      const int ph = int(code[p1] & CODE_MASKVALUE);
      if constexpr (VM == VM_MORRIS) p.eta = viscoeta[p1];
      if constexpr (VM == VM_CONSEQ) {
        p.ta = tau[2 * p1];
        p.tb = tau[2 * p1 + 1];
      }
      if constexpr (VM == VM_ART) {
        p.visco = sph[2 * ph].z;
        p.cs0 = sph[2 * ph].y;
      }
    } else {
      p.x = p.y = p.z = 1e30f;
      p.vr = make_float4(0.f, 0.f, 0.f, 1.f);
    }
    const int lxa = max(cx1 - S, 0), lxb = min(cx1 + S, g.ncx - 1);
    const float thr = K.kernelsize2 * 1.0001f - (p.x * p.x + p.y * p.y + p.z * p.z);
    const RowCtx rc{cy, cz, xa, xb, lxa, lxb, xo, act, p1};
    const float3 f = nnv_pass<VM, false, S>(K, g, rc, p, thr, bc, poscell, velrhop, code, viscoeta, tau, sph, sA, sB,
                                            sC, ftmassp);
    const float3 b = nnv_pass<VM, true, S>(K, g, rc, p, thr, bc, poscell, velrhop, code, viscoeta, tau, sph, sA, sB,
                                           sC, ftmassp);
    if (act) {
      // ace[p1] = ace[p1] + acep1 per pass when non-zero (JSphCpu_NN_SPH.cpp:442-444)
      float4 r = arace[p1];
      if (f.x != 0.f || f.y != 0.f || f.z != 0.f) {
        r.x += f.x;
        r.y += f.y;
        r.z += f.z;
      }
      if (b.x != 0.f || b.y != 0.f || b.z != 0.f) {
        r.x += b.x;
        r.y += b.y;
        r.z += b.z;
      }
      if (K.sim2d) r.y = 0.f;  // Simulate2D: Acec[].y = 0 after the whole interaction
      arace[p1] = r;
      ace2max = nanmax(ace2max, r.x * r.x + r.y * r.y + r.z * r.z);
    }
  }
  wave_max_atomic(sc, RED_ACEMAX2, ace2max);
}

void launch_nn_visc(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                    const float4* poscell, const float4* velrhop, const typecode* code, const float* viscoeta,
                    const float4* tau, const unsigned* begincell, DivGrid g, const KConst& K, const float4* phases,
                    float4* arace, const float* ftmassp) {
#define SPH_NNV(VM)                                                                                             \
  if (K.scelldiv == 2)                                                                                          \
    hipLaunchKernelGGL((k_nn_visc<VM, 2>), dim3(fit_grid((const void*)&k_nn_visc<VM, 2>, nblocks)), dim3(TB), 0, stm, sc, items, qctr, poscell, velrhop,   \
                       code, viscoeta, tau, begincell, g, K, phases, arace, ftmassp);                                    \
  else                                                                                                          \
    hipLaunchKernelGGL((k_nn_visc<VM, 1>), dim3(fit_grid((const void*)&k_nn_visc<VM, 1>, nblocks)), dim3(TB), 0, stm, sc, items, qctr, poscell, velrhop,   \
                       code, viscoeta, tau, begincell, g, K, phases, arace, ftmassp)
  if (K.nntvisco == 1) SPH_NNV(VM_ART);
  else if (K.nntvisco == 2) SPH_NNV(VM_MORRIS);
  else SPH_NNV(VM_CONSEQ);
#undef SPH_NNV
}

// ---- slabs: the first pass's eta / tau of the face columns for the neighbours' ghosts ----
__global__ __launch_bounds__(256) void k_nn_face_pack(DevScalars* __restrict__ sc, PartArrays a, KConst K,
                                                      DivGrid g, const float* __restrict__ viscoeta,
                                                      const float4* __restrict__ tau, NNFaceRec* __restrict__ sl,
                                                      NNFaceRec* __restrict__ sr, unsigned capl, unsigned capr,
                                                      unsigned* __restrict__ idxmap, unsigned nidx) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= sc->np) return;
  const unsigned id = a.idp[p];
  if (id < nidx) idxmap[id] = p;
  if (p < sc->npb) return;  // fluid only (bound p2 use p1's values)
  const unsigned dc = a.dcell[p];
  if (dc >= DCELL_DISCARD) return;
  const int lcx = slab_local(g, K.domcellcode, dc);
  for (int side = 0; side < 2; side++) {  // a slab of one owned column sends a particle both ways
    NNFaceRec* dst = nullptr;
    unsigned cap = 0;
    if (side == 0 && in_left_face(g, lcx) && g.sown0 > 0) { dst = sl; cap = capl; }
    if (side == 1 && in_right_face(g, lcx) && g.sown1 < g.extent()) { dst = sr; cap = capr; }
    if (!dst) continue;
    const unsigned k = atomicAdd(&dst[0].idp, 1u);
    if (k + 1 >= cap) {  // the buffers hold every ghost sent at the divide; if not, say so
      atomicOr(&sc->error_flags, ERR_HALO_FACE);
      continue;
    }
    NNFaceRec r;
    r.idp = id;
    r.v[0] = viscoeta ? viscoeta[p] : 0.f;
    const float4 ta = tau ? tau[2 * p] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 tb = tau ? tau[2 * p + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    r.v[1] = ta.x;
    r.v[2] = ta.y;
    r.v[3] = ta.z;
    r.v[4] = ta.w;
    r.v[5] = tb.x;
    r.v[6] = tb.y;
    dst[k + 1] = r;
  }
}

__global__ __launch_bounds__(256) void k_nn_face_apply(DevScalars* __restrict__ sc, const NNFaceRec* __restrict__ rl,
                                                       const NNFaceRec* __restrict__ rr, unsigned capl,
                                                       unsigned capr, const unsigned* __restrict__ idxmap,
                                                       unsigned nidx, const unsigned* __restrict__ idp,
                                                       float* __restrict__ viscoeta, float4* __restrict__ tau,
                                                       int withtau) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const NNFaceRec* r = (blockIdx.y == 0 ? rl : rr);
  const unsigned cap = (blockIdx.y == 0 ? capl : capr);
  if (!r || i + 1 >= cap || i >= r[0].idp) return;
  const NNFaceRec q = r[i + 1];
  const unsigned p = q.idp < nidx ? idxmap[q.idp] : 0xffffffffu;
  if (p >= sc->np || idp[p] != q.idp) {  // every face particle arrived as a ghost at the divide
    atomicOr(&sc->error_flags, ERR_HALO_MISS);
    return;
  }
  if (viscoeta) viscoeta[p] = q.v[0];
  if (withtau) {
    tau[2 * p] = make_float4(q.v[1], q.v[2], q.v[3], q.v[4]);
    tau[2 * p + 1] = make_float4(q.v[5], q.v[6], 0.f, 0.f);
  }
}

void launch_nn_face_pack(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, const KConst& K,
                         const DivGrid& g, const float* viscoeta, const float4* tau, NNFaceRec* sl, NNFaceRec* sr,
                         unsigned capl, unsigned capr, unsigned* idxmap, unsigned nidx) {
  if (sl) hipMemsetAsync(sl, 0, sizeof(NNFaceRec), stm);
  if (sr) hipMemsetAsync(sr, 0, sizeof(NNFaceRec), stm);
  hipLaunchKernelGGL(k_nn_face_pack, dim3((cap + 255) / 256), dim3(256), 0, stm, sc, a, K, g, viscoeta, tau, sl, sr,
                     capl, capr, idxmap, nidx);
}

void launch_nn_face_apply(hipStream_t stm, DevScalars* sc, const NNFaceRec* rl, const NNFaceRec* rr, unsigned capl,
                          unsigned capr, const unsigned* idxmap, unsigned nidx, const unsigned* idp, float* viscoeta,
                          float4* tau, bool withtau) {
  const unsigned n = std::max(capl, capr);
  if (!n) return;
  hipLaunchKernelGGL(k_nn_face_apply, dim3((n + 255) / 256, 2), dim3(256), 0, stm, sc, rl, rr, capl, capr, idxmap,
                     nidx, idp, viscoeta, tau, int(withtau));
}

}  // namespace sphx
