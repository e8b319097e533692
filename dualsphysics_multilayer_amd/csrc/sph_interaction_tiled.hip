// sph_interaction_tiled.hip — LDS-tiled fluid Interaction_Forces for CDNA4.
//
// Same semantics as k_interaction (sph_interaction.hip; reference JSphCpu.cpp:631-822 /
// JSphGpu_ker.cu:512-745) for fluid p1, restructured for the MI355X:
//
//  * Work items: runs of TB consecutive fluid particles inside ONE (y,z) row of cells
//    (fewer at a row end), spanning <= TMAXCELLS x-cells [a,b], free to start and end
//    inside a cell (built per divide by k_items_*).  All
//    p1 of an item share their 3x3 neighbour rows, and each neighbour row is ONE
//    contiguous particle range (cells are x-fastest), so a block stages each of the
//    9 fluid + 9 bound row ranges once into LDS (coalesced 16-B loads) and every lane
//    reads its candidates from LDS.
//  * Candidate test and pair body are split: a lane first tests 128 candidates and
//    records the accepted ones as bits (two 64-bit masks, no LDS traffic), then walks
//    the set bits.  The heavy body then runs only for real pairs (~16% of candidates)
//    instead of for every candidate any lane of the wave accepted.
//  * Persistent blocks (as many as are co-resident, fit_grid) claiming items from work
//    queues per XCD group (blockIdx % 8): chunks of consecutive items dealt round-robin to
//    the groups, all groups' fluid-row items before any bound-row item (ItemCursor,
//    sph_tiled.hpp).
//  * Fast f32 transcendentals: v_rcp/v_sqrt/v_exp/v_log (<= 1 ulp) instead of the
//    IEEE division/sqrt/pow expansions; Wendland fac rewritten without the 1/rad
//    (fac = bwen*q*(1-q/2)^3/rad = (bwen/h)*(1-q/2)^3).  Rounding-level differences
//    only; parity tests hold it to the reference's noise floor.
#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "sph_items.hpp"
#include "sph_tiled.hpp"

namespace sphx {

// ------------------------------------------------------------------------------------
// Item list (per divide): the passes of sph_items.hpp as kernels.
__global__ __launch_bounds__(64 * IR_WAVES) void k_items_count(ItemBuild b) {
  extern __shared__ unsigned char items_smem[];
  items_count_block(b, blockIdx.x, items_smem);
}

__global__ __launch_bounds__(IP_BS) void k_items_place(ItemBuild b) {
  extern __shared__ unsigned char items_smem[];
  items_place_block(b, items_smem);
}

ItemBuild make_item_build(const unsigned* begincell, DivGrid g, unsigned* rowtmp, uint4* items, unsigned* qctr,
                          int scelldiv, const int* xr, unsigned* qctr2, uint4* rowitems, unsigned ricap) {
  ItemBuild b;
  b.bc = begincell;
  b.g = g;
  b.tmaxc = scelldiv == 1 ? TMAXCELLS : TMAXCELLS_HALF;
  b.xr = {{g.sown0, g.sown1, 0, 0, 0, 0}, qctr2 ? 2 : 1};
  if (xr)
    for (int k = 0; k < 6; k++) b.xr.x[k] = xr[k];
  b.nrows2 = 2u * unsigned(g.ncy) * unsigned(g.ncz);
  b.counts = rowtmp;
  b.items = items;
  b.rowitems = rowitems;
  b.ricap = ricap;
  b.qa = qctr;
  b.qb = qctr2;
  b.nblocks = (b.nrows2 + IR_WAVES - 1) / IR_WAVES;
  const unsigned L = b.rowlds();
  b.lds = ((IR_WAVES * L * unsigned(sizeof(unsigned) + sizeof(unsigned short)) + 15u) / 16u) * 16u;
  return b;
}

void launch_items_place(hipStream_t stm, const ItemBuild& b) {
  const unsigned n = unsigned(b.xr.nl) * b.nrows2;
  const unsigned lds = (((IP_BS / 64) * b.rowlds() * unsigned(sizeof(unsigned) + sizeof(unsigned short)) + 15u) / 16u) * 16u;
  hipLaunchKernelGGL(k_items_place, dim3(items_place_blocks(n)), dim3(IP_BS), lds, stm, b);
}

void launch_items(hipStream_t stm, const ItemBuild& b) {
  hipLaunchKernelGGL(k_items_count, dim3(b.nblocks), dim3(64 * IR_WAVES), b.lds, stm, b);
  launch_items_place(stm, b);
}

// ------------------------------------------------------------------------------------
struct TAcc {
  float ax, ay, az, ar, delta, visc;
  bool dstop;  // FT: the DDT of p1 is off (floating p1, or a light floating p2 under DDT1)
};

// Third record of a staged p2: float2 {press/rho, 1/rho}, or with floating bodies (FT)
// float4 {r press/rho, r/rho, r, kind} with r = m2/MassFluid and kind 0 fluid/bound,
// 1 heavy floating, 2 light floating (massp <= 1.2 MassFluid, DELTA_HEAVYFLOATING,
// JSphCpu.cpp:697-703).
template <bool FT> struct CRecT { typedef float2 type; };
template <> struct CRecT<true> { typedef float4 type; };
__device__ __forceinline__ float crec_r(const float2&) { return 1.f; }
__device__ __forceinline__ float crec_r(const float4& c) { return c.z; }
__device__ __forceinline__ float crec_kind(const float2&) { return 0.f; }
__device__ __forceinline__ float crec_kind(const float4& c) { return c.w; }

struct P1 {
  float x, y, z;        // x relative to the item's x origin, y/z cell-relative
  float4 vr;            // velocity, rho
  float press, inv_rho; // pressure (0 for a boundary p1), 1/rho
};

// Per-pass constants.  The pair body accumulates sums with the per-pass factors
// taken out; finish() applies them once per particle:
//   ar    = ar1 * sum w3 (dr.dv)/rho2
//   ace   = -(bm/rho1) * sum w3 [(p1/rho2 + p2/rho2) + pv'] dr,  pv' = cvp (dr.dv) rr  (dr.dv < 0)
//           with rr = 1/((r2+eta2)(rho1+rho2)): the reference's (p1+p2)/(rho1 rho2) and
//           Pi = cvisc (dr.dv)/(r2+eta2) / robar with the masses and 1/rho1 folded out
//   delta = kd * sum ...  (DDT: Molteni + , Fourtakas -)
struct PassK {
  float ar1;  // bwen/h * m2 * rho1   (continuity)
  float bm;   // bwen/h * m2          (momentum)
  float cvp;  // 2 * cvisc * rho1 / m2 (artificial viscosity; cvisc = -alpha*cs0*h*m2)
  float kd;   // ddtkh*cs0 * bwen/h * m2 (density diffusion)
};

// The Molteni DDT factor r (rho1/rho2 - 1) (JSphCpu.cpp:725-726) with the reference's
// rounding: rho1/rho2 correctly rounded (the v_rcp estimate refined by one fma residual
// step, exact for equal densities), then - 1 (exact: the quotient is within [0.5, 2]).
// The float cancellation of that subtraction is part of the reference's result: the exact
// (rho1 - rho2)/rho2 moved ar by 1.3e-5 of its maximum on the 1M state, 50x the
// reference's own fast-math/strict floor there.  r = the p2 mass ratio (FT records).
__device__ __forceinline__ float molteni(float rho1, float rho2, const float2& c) {
  const float q0 = rho1 * c.y;  // c.y = 1/rho2 (v_rcp)
  const float q = fmaf(fmaf(-rho2, q0, rho1), c.y, q0);
  return q - 1.f;
}
__device__ __forceinline__ float molteni(float rho1, float rho2, const float4& c) {
  const float ir = frcp(rho2);
  const float q0 = rho1 * ir;
  const float q = fmaf(fmaf(-rho2, q0, rho1), ir, q0);
  return (q - 1.f) * c.z;  // c.z = r
}

// One pair body (JSphCpu.cpp:682-797 semantics, fast f32 intrinsics).
// MODE 0: fluid p1 / fluid p2, 1: fluid p1 / bound p2, 2: bound p1 / fluid p2
// (InteractionForcesBound, JSphCpu.cpp:577-612: continuity + visc-dt only).
// `ok` = rr2 <= KernelSize2, the reference's pair test (JSphCpu.cpp:679); a pair beyond it
// contributes exactly +0 (kernel factor clamped to 0, visc term masked), which keeps the
// body branch-free so two pairs can be interleaved.  The test's lower bound rr2 >=
// ALMOSTZERO only removes p1 itself (and exactly coincident particles), whose terms all
// carry a factor dr = 0 or dr.dv = 0 and add +0 here.
// Algebra used (same quantities, fewer operations; constants folded into PassK):
//   fac = bwen*q*(1-q/2)^3/rad = (bwen/h)*w3,  w3 = (1-rad/(2h))^3   (FunSphKernel.h:217-224)
//   dv.fr = fac*(dr.dv), dr.fr = fac*rr2
//   continuity: ar += fac*m2*(dr.dv)*rho1/rho2
//   momentum + artificial viscosity: ace += fac*(-m2*(p1+p2)/(rho1*rho2) - pi_visc)*dr with
//     (p1+p2)/(rho1*rho2) = (p1/rho1)/rho2 + (p2/rho2)/rho1 and
//     pi_visc = cvisc*(dr.dv)/(r^2+eta^2)/robar; one reciprocal 1/((r^2+eta^2)*(rho1+rho2))
//     gives both 1/(r^2+eta^2) and 1/(rho1+rho2)
//   DDT2: rho0*(1+x)^(1/gamma) - rho0, x = ddtgz*drz, as the binomial series in drz up to
//         x^3 (|x| <= 2h*ddtgz < 0.02, decided per case on the host: the x^4 term is < 2e-6
//         of the first, < 1e-8 at the dam break's 1e-3), evaluated by Horner with rho1 as the
//         constant term; this also avoids the float cancellation of the reference's
//         rho0*powf(rh,1/gamma)-rho0.
template <int TDENSITY, int MODE, bool FT = false, typename CR = float2>
__device__ __forceinline__ void pair_body(const KConst& K, const P1& p, float drx, float dry, float drz, float rr2,
                                          bool ok, const float4& B, const CR& C, const PassK& Q, TAcc& a) {
  constexpr int TD = TDENSITY & 7;  // DDT mode; bit 3: the Fourtakas term as its series (K.ddtseries)
  constexpr bool CUB = (TDENSITY & 16) != 0;  // bit 4: the Cubic spline kernel
  const float rad = fsqrt_(rr2);
  float w3, wqc = 0.f, qc = 0.f;
  if (CUB) {
    // GetKernelCubic_Fac (FunSphKernel.h:105-117) with its constants not folded (PassK
    // carries kfold = 1): c2 (2-q)^2 / r beyond h, (c1 q + d1 q^2) / r = (c1 + d1 q) / h
    // within it (finite at r = 0); 2 - q clamped at 0, so nothing beyond the support
    qc = rad * K.ovkernelh;
    wqc = fmaxf(2.f - qc, 0.f);
    const float ffar = K.cub_c2 * wqc * wqc * frcp(rad);
    const float fnear = fmaf(K.cub_d1, qc, K.cub_c1) * K.ovkernelh;
    w3 = rad > K.kernelh ? ffar : fnear;
  } else {
    // 1 - rad/2h clamped to [0, 1] (the fma's clamp modifier): 0 beyond the support radius,
    // so the kernel factor needs no pair test
    const float wq = __builtin_amdgcn_fmed3f(fmaf(K.mhalfovh, rad, 1.f), 0.f, 1.f);
    w3 = wq * wq * wq;
  }
  const float dvx = p.vr.x - B.x, dvy = p.vr.y - B.y, dvz = p.vr.z - B.z;
  const float dot = drx * dvx + dry * dvy + drz * dvz;
  const float re = rr2 + K.eta2;
  float inv_re, rr = 0.f;
  if (MODE == 2) {
    inv_re = frcp(re);
  } else {
    const float rs = p.vr.w + B.w;  // 2*robar
    rr = frcp(re * rs);
    inv_re = rr * rs;
  }
  const float dot_rr2 = ok ? dot * inv_re : 0.f;
  a.visc = fmaxf(dot_rr2, a.visc);
  const float wc = w3 * C.y;  // w3/rho2
  a.ar = fmaf(wc, dot, a.ar);
  if (MODE == 2) return;
  float S = fmaf(C.y, p.press, C.x);  // (p1+p2)/rho2
  if (CUB) {
    // tensile correction GetKernelCubic_Tensil (FunSphKernel.h:141-149) added to
    // (p1+p2)/(rho1 rho2) (JSphCpu.cpp:713), here times rho1 (and the mass ratio r):
    // fab (p1/rho1^2 k1 + p2/rho2^2 k2), fab = (Wab / Wab(dp))^4, k = 0.01 (p > 0) or -0.2
    const float wab = rad > K.kernelh ? K.cub_a24 * (wqc * wqc * wqc)
                                      : K.cub_a2 * fmaf(fmaf(0.75f, qc, -1.5f), qc * qc, 1.f);
    float fab = wab * K.cub_odw;
    fab *= fab;
    fab *= fab;
    const float r = crec_r(C);
    const float t1 = p.press * p.inv_rho * p.inv_rho * (p.press > 0.f ? 0.01f : -0.2f);
    const float t2 = C.x * C.y * (C.x > 0.f ? 0.01f : -0.2f) * frcp(r);  // r^2 p2/rho2^2 / r
    S = fmaf(fab * p.vr.w, fmaf(r, t1, t2), S);
  }
  float pv = Q.cvp * fminf(dot, 0.f) * rr;  // artificial viscosity only for approaching pairs
  if (FT) pv *= crec_r(C);  // viscosity with the p2 mass
  const float c = w3 * (S + pv);
  a.ax = fmaf(c, drx, a.ax);
  a.ay = fmaf(c, dry, a.ay);
  a.az = fmaf(c, drz, a.az);
  if (MODE == 1) {
    if (TD == 1 && K.mdbc) {  // mDBC: Molteni DDT over bound neighbours too (JSphCpu.cpp:730)
      const float t = w3 * rr2 * inv_re;
      a.delta = fmaf(t, molteni(p.vr.w, B.w, C), a.delta);
    } else if ((TD == 1 || TD == 2) && ok) {
      a.delta = FLT_MAX;  // DBC: no DDT next to the boundary
    }
    return;
  }
  if (TD == 1) {
    const float t = w3 * rr2 * inv_re;
    a.delta = fmaf(t, molteni(p.vr.w, B.w, C), a.delta);
    if (FT && ok && crec_kind(C) == 2.f) a.dstop = true;  // light floating p2
  } else if (TD == 2 || TD == 3) {
    float rho1h;  // rho1 + drhop
    if (TDENSITY & 8)  // K.ddtseries (a template flag: no per-pair branch), Horner with rho1
      rho1h = fmaf(drz, fmaf(drz, fmaf(drz, K.ddte3, K.ddte2), K.ddte1), p.vr.w);
    else
      rho1h = p.vr.w + (K.rhopzero * fexp2(K.ovgamma * flog2(1.f + K.ddtgz * drz)) - K.rhopzero);
    float t = wc * rr2 * inv_re;
    if (FT && crec_kind(C) != 0.f) t = 0.f;  // no Fourtakas term with a floating p2 (JSphCpu.cpp:743)
    a.delta = fmaf(t, B.w - rho1h, a.delta);
  }
}

// The per-pass factors of the sums (PassK) applied once per particle.
template <int TDENSITY, int MODE, bool FT = false>
__device__ __forceinline__ TAcc finish(const KConst& K, TAcc a, const P1& p, const PassK& Q) {
  constexpr int TD = TDENSITY & 7;
  a.ar *= Q.ar1;
  if (MODE != 2) {
    const float s = -Q.bm * p.inv_rho;
    a.ax *= s;
    a.ay *= s;
    a.az *= s;
  }
  if (MODE == 0 || (MODE == 1 && TD == 1 && K.mdbc)) {
    if (TD == 1) a.delta *= Q.kd;
    else if (TD == 2 || TD == 3) a.delta *= -Q.kd;
  }
  if (FT && TD && a.dstop) a.delta = FLT_MAX;
  return a;
}

template <int TDENSITY, int MODE, bool FT>
__device__ __forceinline__ void drain_words(const KConst& K, const P1& p, unsigned long long c0,
                                            unsigned long long c1, unsigned long long c2, unsigned long long c3,
                                            int b0, int b1, int b2, int b3, const float4* __restrict__ sA,
                                            const float4* __restrict__ sB,
                                            const typename CRecT<FT>::type* __restrict__ sC, const PassK& Q,
                                            TAcc& a);

// One drain unit: the lane's candidates in up to two staged windows [wa0,wa1) and
// [wb0,wb1) (two point-mirrored neighbour rows, or one row), all positions relative to
// the item, drained as ONE set.  How many real neighbours a particle has in one row
// depends on where it sits inside its cell; in a mirrored pair of rows the two counts
// complement each other, so the loop length (the busiest lane's count / 2) is far closer
// to the average lane's than with one row at a time.
// The accepted candidates of a round (<= 128 per window) are four 64-bit words,
// compacted once into a chain (empty words dropped): `cur` is popped, and when it runs
// dry the next word shifts in.  Value selects only (a word picked by reference puts the
// masks in scratch), no divergent branch in the loop (the second pop of an iteration is
// unconditional; an empty pop's pair is masked off).
// SELF (the Symmetry image of the own row): staged record `self` of window a is the lane's
// own p1, whose image is no neighbour (the reference visits an image only after its
// original passed the rr2 >= ALMOSTZERO test, JSphCpu.cpp:687,793-796).
template <int TDENSITY, int MODE, bool FT = false, bool SELF = false>
__device__ __forceinline__ void tile_unit(const KConst& K, const P1& p, float thr, int wa0, int wa1, int wb0, int wb1,
                                          const float4* __restrict__ sA, const float4* __restrict__ sB,
                                          const typename CRecT<FT>::type* __restrict__ sC, const PassK& Q, TAcc& a,
                                          int self = -1) {
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  for (int off = 0;; off += 128) {  // a second round only for windows of > 128 candidates
    const int na = wa1 - wa0 - off, nb = wb1 - wb0 - off;
    if (na <= 0 && nb <= 0) break;
    unsigned long long c0, c1, c2, c3;
    test128(sA, wa0 + off, min(na, 128), px2, py2, pz2, thr, c0, c1);
    test128(sA, wb0 + off, min(nb, 128), px2, py2, pz2, thr, c2, c3);
    if (SELF) {
      const int k = self - (wa0 + off);
      if (k >= 0 && k < 64) c0 &= ~(1ull << k);
      else if (k >= 64 && k < 128) c1 &= ~(1ull << (k - 64));
    }
    drain_words<TDENSITY, MODE, FT>(K, p, c0, c1, c2, c3, wa0 + off, wa0 + off + 64, wb0 + off, wb0 + off + 64, sA,
                                    sB, sC, Q, a);
  }
}

// CellMode=half drain unit: four windows (two mirrored row pairs) of 5 half-cells each,
// <= 64 candidates per window and round (one word each), drained as ONE set.
template <int TDENSITY, int MODE, bool FT = false>
__device__ __forceinline__ void tile_unit4(const KConst& K, const P1& p, float thr, int4 w0, int4 w1,
                                           const float4* __restrict__ sA, const float4* __restrict__ sB,
                                           const typename CRecT<FT>::type* __restrict__ sC, const PassK& Q,
                                           TAcc& a) {
  const float px2 = -2.f * p.x, py2 = -2.f * p.y, pz2 = -2.f * p.z;
  for (int off = 0;; off += 64) {  // a second round only for windows of > 64 candidates
    const int n0 = w1.x - w0.x - off, n1 = w1.y - w0.y - off, n2 = w1.z - w0.z - off, n3 = w1.w - w0.w - off;
    if (n0 <= 0 && n1 <= 0 && n2 <= 0 && n3 <= 0) break;
    const unsigned long long c0 = test64(sA, w0.x + off, min(n0, 64), px2, py2, pz2, thr);
    const unsigned long long c1 = test64(sA, w0.y + off, min(n1, 64), px2, py2, pz2, thr);
    const unsigned long long c2 = test64(sA, w0.z + off, min(n2, 64), px2, py2, pz2, thr);
    const unsigned long long c3 = test64(sA, w0.w + off, min(n3, 64), px2, py2, pz2, thr);
    drain_words<TDENSITY, MODE, FT>(K, p, c0, c1, c2, c3, w0.x + off, w0.y + off, w0.z + off, w0.w + off, sA, sB,
                                    sC, Q, a);
  }
}

// Drain of one round of accepted candidates: four 64-bit words c0..c3 of staged records
// from bases b0..b3 (see tile_unit).
// Records addressed by byte offset j16 = 16 j of their index j.
__device__ __forceinline__ const float4* at16(const float4* __restrict__ base, int j16) {
  return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + j16);
}
__device__ __forceinline__ float2 at_rec(const float2* __restrict__ base, int j16) {
  return *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(base) + (j16 >> 1));
}
__device__ __forceinline__ float4 at_rec(const float4* __restrict__ base, int j16) { return *at16(base, j16); }

template <int TDENSITY, int MODE, bool FT>
__device__ __forceinline__ void drain_words(const KConst& K, const P1& p, unsigned long long c0,
                                            unsigned long long c1, unsigned long long c2, unsigned long long c3,
                                            int b0, int b1, int b2, int b3, const float4* __restrict__ sA,
                                            const float4* __restrict__ sB,
                                            const typename CRecT<FT>::type* __restrict__ sC, const PassK& Q,
                                            TAcc& a) {
  {
    // compact: drop empty words, keep the order (three bubble passes)
#pragma unroll
    for (int pass = 0; pass < 3; pass++) {
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
    // bases in bytes of a 16-B record (j16 = 16 j): one shift-add per pop gives the sA/sB
    // address, a shift right the 8-B sC one
    b0 <<= 4;
    b1 <<= 4;
    b2 <<= 4;
    b3 <<= 4;
    auto pop = [&](void) -> int {
      const int j = b0 + (int(__builtin_ctzll(c0 | (1ull << 63))) << 4);
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
      const float4 A1 = *at16(sA, j1), A2 = *at16(sA, j2);
      const float4 B1 = *at16(sB, j1), B2 = *at16(sB, j2);
      const typename CRecT<FT>::type C1 = at_rec(sC, j1), C2 = at_rec(sC, j2);
      const float drx1 = p.x - A1.x, dry1 = p.y - A1.y, drz1 = p.z - A1.z;
      const float drx2 = p.x - A2.x, dry2 = p.y - A2.y, drz2 = p.z - A2.z;
      const float rr21 = drx1 * drx1 + dry1 * dry1 + drz1 * drz1;
      const float rr22 = drx2 * drx2 + dry2 * dry2 + drz2 * drz2;
      // a missing second pair (j2 = j1) is moved beyond the support radius: factor 0
      const float rr22m = two ? rr22 : 1e30f;
      const bool ok1 = rr21 <= K.kernelsize2, ok2 = rr22m <= K.kernelsize2;
      pair_body<TDENSITY, MODE, FT>(K, p, drx1, dry1, drz1, rr21, ok1, B1, C1, Q, a);
      pair_body<TDENSITY, MODE, FT>(K, p, drx2, dry2, drz2, rr22m, ok2, B2, C2, Q, a);
      keep_w(A1, A2);  // 16-B reads (ds_read_b128) for the position records, see keep_w
    }
  }
}

// Stage the records [rs, re) of the row at (dy, dz) from the item's row into sA/sB/sC at
// dst: positions relative to the item (x to its x origin xo, y/z to its cell row), |A|^2,
// velrhop, press/rho, 1/rho.
struct FtRec {
  const typecode* code;
  const float* massp;  // particle mass per floating body
};
__device__ __forceinline__ void put_c(float2* sC, unsigned i, float pr, float ir, const KConst&, const FtRec&,
                                      unsigned) {
  sC[i] = make_float2(pr * ir, ir);
}
__device__ __forceinline__ void put_c(float4* sC, unsigned i, float pr, float ir, const KConst& K, const FtRec& ft,
                                      unsigned p2) {
  const typecode c = ft.code[p2];
  float r = 1.f, kind = 0.f;
  if (CodeType(c) == CODE_TYPE_FLOATING) {
    const float m = ft.massp[c & CODE_MASKVALUE];
    r = m / K.massfluid;
    kind = (m <= K.massfluid * 1.2f) ? 2.f : 1.f;
  }
  const float rir = r * ir;
  sC[i] = make_float4(pr * rir, rir, r, kind);
}
// mir (Symmetry, rows of the first y rows of a p1 in them): the records' images across y = 0,
// position y and velocity y negated (JSphCpu.cpp:684,709); the item's frame starts at
// y = mirc scell (its row), so the image of a record at frame y is at -y - 2 mirc scell.
template <typename CR>
__device__ __forceinline__ void stage_row(const KConst& K, unsigned rs, unsigned re, unsigned dst, int xo, int dy,
                                          int dz, const float4* __restrict__ poscell,
                                          const float4* __restrict__ velrhop, const float* __restrict__ press,
                                          float4* __restrict__ sA, float4* __restrict__ sB, CR* __restrict__ sC,
                                          const FtRec& ft, bool mir = false, int mirc = 0) {
  const float oy = float(dy) * K.scell, oz = float(dz) * K.scell, my = float(2 * mirc) * K.scell;
  for (unsigned i = threadIdx.x; i < re - rs; i += TB) {
    const float4 pc = poscell[rs + i];
    const int cx2 = int(DcelCellx(K.domcellcode, __float_as_uint(pc.w)));
    const float x2 = pc.x + float(cx2 - xo) * K.scell;
    const float y2 = mir ? -(pc.y + oy) - my : pc.y + oy, z2 = pc.z + oz;
    sA[dst + i] = make_float4(x2, y2, z2, x2 * x2 + y2 * y2 + z2 * z2);
    float4 vr = velrhop[rs + i];
    if (mir) vr.y = -vr.y;
    sB[dst + i] = vr;
    const float ir = frcp(vr.w);
    put_c(sC, dst + i, press[rs + i], ir, K, ft, rs + i);
  }
}

// Per-pass constants of the pair body for p2 of mass m2 (the Wendland bwen/h folded in).
__device__ __forceinline__ PassK pass_k(const KConst& K, float cvisc, float m2, float rho1) {
  PassK q;
  q.bm = K.kfold * m2;
  q.ar1 = q.bm * rho1;
  q.cvp = 2.f * cvisc * rho1 / m2;
  q.kd = K.ddtkhcs * q.bm;
  return q;
}

// Staged index of the lane's own p1 in the records [rs, re) staged from 0, or -1.
__device__ __forceinline__ int self_in(const RowCtx& rc, unsigned rs, unsigned re) {
  return (rc.act && rc.p1 >= rs && rc.p1 < re) ? int(rc.p1 - rs) : -1;
}

// One interaction pass of the item's p1 over the 3x3 neighbour rows of one particle
// kind: MODE 0/2 the fluid rows (fluid / bound p1), MODE 1 the bound rows (fluid p1).
// Drain units: point-mirrored row pairs, then the item's own row; a pair of rows is
// staged as one segment [row a][row b] when it fits TCAP, else row by row in segments.
template <int TDENSITY, int MODE, bool FT = false>
__device__ __forceinline__ TAcc run_pass(const KConst& K, const DivGrid& g, const RowCtx& rc, const P1& p, float thr,
                                         const PassK Q, const unsigned* __restrict__ bc,
                                         const float4* __restrict__ poscell, const float4* __restrict__ velrhop,
                                         const float* __restrict__ press, float4* __restrict__ sA,
                                         float4* __restrict__ sB, typename CRecT<FT>::type* __restrict__ sC,
                                         const FtRec& ft, bool dstop0 = false) {
  TAcc acc = {};
  acc.dstop = dstop0;
  const unsigned cellinit = (MODE == 1 ? 0u : g.boxfluid);
  // Symmetry: an item of the first y row (its p1 within 2h of y = 0; with cells of 2h that
  // is every p1 of the row) also meets the images of that row's p2 (all within 2h of the
  // plane): units 5 (rows dz = -1 / +1) and 6 (the own row, without the p1's own image).
  // The reference visits an image right after its original when the original is within the
  // support radius (JSphCpu.cpp:793-796); an image is never nearer than its original for
  // y >= 0, so the images within the radius are exactly those.
  const int nu = (K.symmetry && rc.cy == 0) ? 7 : 5;
  for (int u = 0; u < nu; u++) {
    const bool mir = u >= 5;
    const int dza = (u == 0 || u == 1 || u == 2 || u == 5) ? -1 : 0;
    const int dya = (u == 0) ? -1 : (u == 1) ? 1 : (u == 2) ? 0 : (u == 3) ? -1 : 0;
    const bool paired = u < 4 || u == 5;
    // rows (dya, dza) and (-dya, -dza); an out-of-grid row is empty
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
    if (n0 + n1 == 0u) continue;
    constexpr int tcap = TcapT<FT>::v;
    // unit 6 (the own row's images): the lane's own record is skipped when it is in the
    // staged rows (fluid p1, fluid rows)
    if (n0 + n1 <= unsigned(tcap)) {
      // both rows in one segment: [row a][row b]
      __syncthreads();
      if (n0) stage_row(K, rs[0], re[0], 0u, rc.xo, dya, dza, poscell, velrhop, press, sA, sB, sC, ft, mir);
      if (n1) stage_row(K, rs[1], re[1], n0, rc.xo, -dya, -dza, poscell, velrhop, press, sA, sB, sC, ft, mir);
      __syncthreads();
      const int wa0 = int(ls[0] - rs[0]), wa1 = rc.act && n0 ? int(le[0] - rs[0]) : wa0;
      const int wb0 = int(n0 + ls[1] - rs[1]), wb1 = rc.act && n1 ? int(n0 + le[1] - rs[1]) : wb0;
      if (u == 6)
        tile_unit<TDENSITY, MODE, FT, true>(K, p, thr, wa0, wa1, wb0, wb1, sA, sB, sC, Q, acc,
                                            self_in(rc, rs[0], re[0]));
      else
        tile_unit<TDENSITY, MODE, FT>(K, p, thr, wa0, wa1, wb0, wb1, sA, sB, sC, Q, acc);
    } else {
      // too long for one segment: each row on its own, in TCAP segments
      for (int k = 0; k < 2; k++) {
        const int dz = k ? -dza : dza, dy = k ? -dya : dya;
        for (unsigned seg = rs[k]; seg < re[k]; seg += tcap) {
          const unsigned segn = min(unsigned(tcap), re[k] - seg);
          __syncthreads();
          stage_row(K, seg, seg + segn, 0u, rc.xo, dy, dz, poscell, velrhop, press, sA, sB, sC, ft, mir);
          __syncthreads();
          const int w0 = int(max(ls[k], seg) - seg);
          const int w1 = rc.act ? max(w0, int(min(le[k], seg + segn)) - int(seg)) : w0;
          if (u == 6)
            tile_unit<TDENSITY, MODE, FT, true>(K, p, thr, w0, w1, 0, 0, sA, sB, sC, Q, acc,
                                                self_in(rc, seg, seg + segn));
          else
            tile_unit<TDENSITY, MODE, FT>(K, p, thr, w0, w1, 0, 0, sA, sB, sC, Q, acc);
        }
      }
    }
  }
  return finish<TDENSITY, MODE, FT>(K, acc, p, Q);
}

// CellMode=half pass: units of HALF_LPU lower rows + their mirrors (2 or 4 rows staged as
// one segment when they fit TCAP, drained as one set by tile_unit4), then the own row; a
// unit too long for one segment goes row by row in TCAP segments.
#ifndef SPH_HALF_LPU
#define SPH_HALF_LPU 1
#endif
constexpr int HALF_LPU = SPH_HALF_LPU;
static_assert(HALF_LPU == 1 || HALF_LPU == 2, "1 or 2 lower rows per unit");
template <int TDENSITY, int MODE, bool FT = false>
__device__ __forceinline__ TAcc run_pass_half(const KConst& K, const DivGrid& g, const RowCtx& rc, const P1& p,
                                              float thr, const PassK Q, const unsigned* __restrict__ bc,
                                              const float4* __restrict__ poscell,
                                              const float4* __restrict__ velrhop, const float* __restrict__ press,
                                              float4* __restrict__ sA, float4* __restrict__ sB,
                                              typename CRecT<FT>::type* __restrict__ sC, const FtRec& ft,
                                              bool dstop0 = false) {
  TAcc acc = {};
  acc.dstop = dstop0;
  const unsigned cellinit = (MODE == 1 ? 0u : g.boxfluid);
  constexpr int tcap = TcapT<FT>::v;
  constexpr int NU = 12 / HALF_LPU;  // units of lower rows; unit NU is the own row
  for (int u = 0; u <= NU; u++) {
    int dyr[4], dzr[4];
    unsigned rs[4], re[4], ls[4], le[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int dy = 0, dz = 0;
      if (u < NU) half_row(HALF_LPU * u + (k >> 1), dy, dz);
      if (k & 1) {
        dy = -dy;
        dz = -dz;
      }
      dyr[k] = dy;
      dzr[k] = dz;
      rs[k] = re[k] = ls[k] = le[k] = 0u;
      const int z = rc.cz + dz, y = rc.cy + dy;
      if ((u == NU && k) || (k >> 1) >= HALF_LPU || z < 0 || z >= g.ncz || y < 0 || y >= g.ncy) continue;
      const unsigned rowbase = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
      rs[k] = bc[rowbase + rc.xa];
      re[k] = bc[rowbase + rc.xb + 1];
      ls[k] = bc[rowbase + rc.lxa];
      le[k] = bc[rowbase + rc.lxb + 1];
    }
    const unsigned n0 = re[0] - rs[0], n1 = re[1] - rs[1], n2 = re[2] - rs[2], n3 = re[3] - rs[3];
    const unsigned ntot = n0 + n1 + n2 + n3;
    if (ntot == 0u) continue;
    if (ntot <= unsigned(tcap)) {
      const unsigned o1 = n0, o2 = o1 + n1, o3 = o2 + n2;
      __syncthreads();
      if (n0) stage_row(K, rs[0], re[0], 0u, rc.xo, dyr[0], dzr[0], poscell, velrhop, press, sA, sB, sC, ft);
      if (n1) stage_row(K, rs[1], re[1], o1, rc.xo, dyr[1], dzr[1], poscell, velrhop, press, sA, sB, sC, ft);
      if (n2) stage_row(K, rs[2], re[2], o2, rc.xo, dyr[2], dzr[2], poscell, velrhop, press, sA, sB, sC, ft);
      if (n3) stage_row(K, rs[3], re[3], o3, rc.xo, dyr[3], dzr[3], poscell, velrhop, press, sA, sB, sC, ft);
      __syncthreads();
      int4 w0, w1;
      w0.x = int(ls[0] - rs[0]);
      w1.x = rc.act && n0 ? int(le[0] - rs[0]) : w0.x;
      w0.y = int(o1 + ls[1] - rs[1]);
      w1.y = rc.act && n1 ? int(o1 + le[1] - rs[1]) : w0.y;
      w0.z = int(o2 + ls[2] - rs[2]);
      w1.z = rc.act && n2 ? int(o2 + le[2] - rs[2]) : w0.z;
      w0.w = int(o3 + ls[3] - rs[3]);
      w1.w = rc.act && n3 ? int(o3 + le[3] - rs[3]) : w0.w;
      tile_unit4<TDENSITY, MODE, FT>(K, p, thr, w0, w1, sA, sB, sC, Q, acc);
    } else {
      // too long for one segment: each row on its own, in TCAP segments (values picked
      // by selects: a runtime index into the row arrays would put them in scratch)
      for (int k = 0; k < 4; k++) {
        auto pick = [&](const unsigned* v) { return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3]; };
        const unsigned rsk = pick(rs), rek = pick(re), lsk = pick(ls), lek = pick(le);
        const int dy = k == 0 ? dyr[0] : k == 1 ? dyr[1] : k == 2 ? dyr[2] : dyr[3];
        const int dz = k == 0 ? dzr[0] : k == 1 ? dzr[1] : k == 2 ? dzr[2] : dzr[3];
        for (unsigned seg = rsk; seg < rek; seg += tcap) {
          const unsigned segn = min(unsigned(tcap), rek - seg);
          __syncthreads();
          stage_row(K, seg, seg + segn, 0u, rc.xo, dy, dz, poscell, velrhop, press, sA, sB, sC, ft);
          __syncthreads();
          const int w0 = int(max(lsk, seg) - seg);
          const int w1 = rc.act ? max(w0, int(min(lek, seg + segn)) - int(seg)) : w0;
          tile_unit<TDENSITY, MODE, FT>(K, p, thr, w0, w1, 0, 0, sA, sB, sC, Q, acc);
        }
      }
    }
  }
  // Symmetry with half cells: a p1 of the first two rows (within 2h of y = 0) also meets the
  // images of the p2 of rows 0 and 1 (all within 2h of the plane), as in run_pass: per image
  // row a unit of each mirrored z pair (dz = -+1, -+2) and the z = 0 row, its own image
  // skipped (JSphCpu.cpp:671-796).
  if (K.symmetry && rc.cy < 2) {
    for (int v = 0; v < 6; v++) {
      const int dya = v / 3 - rc.cy, iz = v % 3;
      const int dza = iz < 2 ? -(iz + 1) : 0;
      const bool paired = iz < 2, selfrow = !paired && dya == 0;
      unsigned rs[2] = {0, 0}, re[2] = {0, 0}, ls[2] = {0, 0}, le[2] = {0, 0};
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k == 1 && !paired) break;
        const int dz = k ? -dza : dza;
        const int z = rc.cz + dz, y = rc.cy + dya;
        if (z < 0 || z >= g.ncz || y < 0 || y >= g.ncy) continue;
        const unsigned rowbase = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
        rs[k] = bc[rowbase + rc.xa];
        re[k] = bc[rowbase + rc.xb + 1];
        ls[k] = bc[rowbase + rc.lxa];
        le[k] = bc[rowbase + rc.lxb + 1];
      }
      const unsigned n0 = re[0] - rs[0], n1 = re[1] - rs[1];
      if (n0 + n1 == 0u) continue;
      if (n0 + n1 <= unsigned(tcap)) {
        __syncthreads();
        if (n0) stage_row(K, rs[0], re[0], 0u, rc.xo, dya, dza, poscell, velrhop, press, sA, sB, sC, ft, true, rc.cy);
        if (n1) stage_row(K, rs[1], re[1], n0, rc.xo, dya, -dza, poscell, velrhop, press, sA, sB, sC, ft, true, rc.cy);
        __syncthreads();
        const int wa0 = int(ls[0] - rs[0]), wa1 = rc.act && n0 ? int(le[0] - rs[0]) : wa0;
        const int wb0 = int(n0 + ls[1] - rs[1]), wb1 = rc.act && n1 ? int(n0 + le[1] - rs[1]) : wb0;
        if (selfrow)
          tile_unit<TDENSITY, MODE, FT, true>(K, p, thr, wa0, wa1, wb0, wb1, sA, sB, sC, Q, acc,
                                              self_in(rc, rs[0], re[0]));
        else
          tile_unit<TDENSITY, MODE, FT>(K, p, thr, wa0, wa1, wb0, wb1, sA, sB, sC, Q, acc);
      } else {
        for (int k = 0; k < 2; k++) {
          const int dz = k ? -dza : dza;
          const unsigned rsk = k ? rs[1] : rs[0], rek = k ? re[1] : re[0], lsk = k ? ls[1] : ls[0],
                         lek = k ? le[1] : le[0];
          for (unsigned seg = rsk; seg < rek; seg += tcap) {
            const unsigned segn = min(unsigned(tcap), rek - seg);
            __syncthreads();
            stage_row(K, seg, seg + segn, 0u, rc.xo, dya, dz, poscell, velrhop, press, sA, sB, sC, ft, true, rc.cy);
            __syncthreads();
            const int w0 = int(max(lsk, seg) - seg);
            const int w1 = rc.act ? max(w0, int(min(lek, seg + segn)) - int(seg)) : w0;
            if (selfrow)
              tile_unit<TDENSITY, MODE, FT, true>(K, p, thr, w0, w1, 0, 0, sA, sB, sC, Q, acc,
                                                  self_in(rc, seg, seg + segn));
            else
              tile_unit<TDENSITY, MODE, FT>(K, p, thr, w0, w1, 0, 0, sA, sB, sC, Q, acc);
          }
        }
      }
    }
  }
  return finish<TDENSITY, MODE, FT>(K, acc, p, Q);
}

// The pass of the cell mode: S = scelldiv (1 full, 2 half).
template <int TDENSITY, int MODE, bool FT, int S>
__device__ __forceinline__ TAcc pass_s(const KConst& K, const DivGrid& g, const RowCtx& rc, const P1& p, float thr,
                                       const PassK Q, const unsigned* __restrict__ bc,
                                       const float4* __restrict__ poscell, const float4* __restrict__ velrhop,
                                       const float* __restrict__ press, float4* __restrict__ sA,
                                       float4* __restrict__ sB, typename CRecT<FT>::type* __restrict__ sC,
                                       const FtRec& ft, bool dstop0 = false) {
  if constexpr (S == 1)
    return run_pass<TDENSITY, MODE, FT>(K, g, rc, p, thr, Q, bc, poscell, velrhop, press, sA, sB, sC, ft, dstop0);
  else
    return run_pass_half<TDENSITY, MODE, FT>(K, g, rc, p, thr, Q, bc, poscell, velrhop, press, sA, sB, sC, ft,
                                             dstop0);
}


// The kernel body (k_fluid_tiled / k_fluid_tiled_w4 below).
template <int TDENSITY, bool FT, int S>
__device__ __forceinline__ void fluid_tiled(DevScalars* __restrict__ sc, const uint4* __restrict__ items,
                                            unsigned* __restrict__ qctr, const float4* __restrict__ poscell,
                                            const float4* __restrict__ velrhop, const float* __restrict__ press,
                                            const unsigned* __restrict__ bc, const DivGrid& g, const KConst& K,
                                            float4* __restrict__ arace, const FtRec& ft) {
  constexpr int tcap = TcapT<FT>::v;
  constexpr int TD = TDENSITY & 7;
  // position records then velrhop records in ONE array: the candidate test's last group of
  // 32 may read up to 31 records past a window that ends at tcap, which stays inside it
  __shared__ float4 sAB[2 * tcap];
  float4* const sA = sAB;
  float4* const sB = sAB + tcap;
  __shared__ typename CRecT<FT>::type sC[tcap];  // press/rho, 1/rho (FT: mass-scaled + kind)
  __shared__ unsigned s_item;
  __shared__ unsigned char s_perm[TB];  // lane -> p1 of the item (see lane_order)
  __shared__ unsigned s_nwave[4];
  float viscmax = 0.f, ace2max = 0.f;
  // Visco of the step: ViscoTime's value (device-resident, k_dt) or the case's
  const float visco = K.visco_n ? sc->visco : K.visco, viscob = K.visco_n ? visco * K.viscobf : K.viscobound;
  const float cvisc_f = -visco * K.cs0f * K.kernelh * K.massfluid;
  const float cvisc_b = -viscob * K.cs0f * K.kernelh * K.massbound;

  ItemCursor<false> cur(qctr);
  for (;;) {
    const unsigned it = cur.next(&s_item);
    if (it == ITEM_NONE) break;
    const uint4 item = items[it];
    const bool bitem = (item.x & ITEM_BOUND) != 0u;
    const int cy = int(item.x & 0xffffu), cz = int((item.x >> 16) & 0x7fffu);
    const int a = int(item.y & 0xffffu), b = int(item.y >> 16);
    const int xo = (a + b + 1) >> 1;
    const int xa = max(a - S, 0), xb = min(b + S, g.ncx - 1);
    if (bitem) {
      // Bound item: nothing to compute unless a fluid cell is in its neighbourhood;
      // then its particles get ar = 0 (PreInteraction's reset).
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
    {  // items hold <= TB particles: one p1 per lane
      const unsigned p1 = item.z + lane_order(poscell, item.z, item.w - item.z, 0.5f * K.scell, s_perm, s_nwave);
      const bool act = threadIdx.x < item.w - item.z;
      P1 p;
      int cx1 = a;
      if (act) {
        const float4 pc1 = poscell[p1];
        cx1 = int(DcelCellx(K.domcellcode, __float_as_uint(pc1.w)));
        p.x = pc1.x + float(cx1 - xo) * K.scell;
        p.y = pc1.y;
        p.z = pc1.z;
        p.vr = velrhop[p1];
        p.press = bitem ? 0.f : press[p1];
      } else {
        p.x = p.y = p.z = 1e30f;  // never within the support radius
        p.vr = make_float4(0.f, 0.f, 0.f, 1.f);
        p.press = 0.f;
      }
      p.inv_rho = frcp(p.vr.w);
      const int lxa = max(cx1 - S, 0), lxb = min(cx1 + S, g.ncx - 1);
      const float thr = K.kernelsize2 * 1.0001f - (p.x * p.x + p.y * p.y + p.z * p.z);
      const RowCtx rc{cy, cz, xa, xb, lxa, lxb, xo, act, p1};
      // pass 0: fluid p2 (fluid p1: momentum/continuity/DDT; bound p1: continuity),
      // pass 1: bound p2 of fluid p1.  Each pass holds only its own accumulator.
      TAcc f, bnd = {0, 0, 0, 0, 0, 0, false};
      if (bitem) {
        f = pass_s<TDENSITY, 2, FT, S>(K, g, rc, p, thr, pass_k(K, cvisc_f, K.massfluid, p.vr.w), bc, poscell,
                                       velrhop, press, sA, sB, sC, ft);
      } else {
        // a floating p1 gets no DDT (JSphCpu.cpp:659-662)
        const bool ftp1 = FT && act && CodeType(ft.code[p1]) == CODE_TYPE_FLOATING;
        f = pass_s<TDENSITY, 0, FT, S>(K, g, rc, p, thr, pass_k(K, cvisc_f, K.massfluid, p.vr.w), bc, poscell,
                                       velrhop, press, sA, sB, sC, ft, ftp1);
        bnd = pass_s<TDENSITY, 1, FT, S>(K, g, rc, p, thr, pass_k(K, cvisc_b, K.massbound, p.vr.w), bc, poscell,
                                         velrhop, press, sA, sB, sC, ft, ftp1);
      }
      if (act && bitem) {
        // InteractionForcesBound store (JSphCpu.cpp:617-621) onto the reset ar = 0.
        arace[p1] = make_float4(0.f, 0.f, 0.f, (f.ar != 0.f || f.visc != 0.f) ? 0.f + f.ar : 0.f);
        viscmax = fmaxf(viscmax, f.visc);
      } else if (act) {
        // Combine exactly as the two CPU passes store (JSphCpu.cpp:800-818).
        float ar = 0.f, ax = 0.f, ay = 0.f, az = 0.f, delta = 0.f;
        if (f.ar != 0.f || f.ax != 0.f || f.ay != 0.f || f.az != 0.f || f.visc != 0.f) {
          if (TD) delta = (f.delta == FLT_MAX ? FLT_MAX : 0.f + f.delta);
          ar = f.ar;
          ax = f.ax;
          ay = f.ay;
          az = f.az;
        }
        if (bnd.ar != 0.f || bnd.ax != 0.f || bnd.ay != 0.f || bnd.az != 0.f || bnd.visc != 0.f) {
          if (TD) delta = (delta == FLT_MAX || bnd.delta == FLT_MAX ? FLT_MAX : delta + bnd.delta);
          ar += bnd.ar;
          ax += bnd.ax;
          ay += bnd.ay;
          az += bnd.az;
        }
        if (TD && delta != FLT_MAX) ar += delta;
        if (K.sim2d) ay = 0.f;  // Simulate2D: Acec[].y = 0 (JSphCpuSingle.cpp:544-549)
        arace[p1] = make_float4(ax, ay, az, ar);
        viscmax = fmaxf(viscmax, fmaxf(f.visc, bnd.visc));
        ace2max = fmaxf(ace2max, ax * ax + ay * ay + az * az);
      }
    }
  }
  wave_max_atomic(sc, RED_VISCDT, viscmax);
  wave_max_atomic(sc, RED_ACEMAX2, ace2max);
  // (the queue counters are zeroed by k_items_place, or by the solver before an interaction
  // without a new item list)
}

// The kernel.  A register budget of 4 waves per SIMD (<= 128 VGPRs; 8 blocks per CU) for the
// instantiations whose natural allocation exceeds it (DDT1, the Cubic DDT 1/2 forms, with
// floating bodies Cubic DDT2 series: 129-135 VGPRs, 3 waves per SIMD): cfg3 (DDT1) 5.84 ->
// 5.49 ms per interaction; the others keep the compiler's allocation (cfg2's DDT2 series at
// 113 VGPRs under the budget ran 0.609-0.618 ms against 0.585-0.593 at its own 125).
template <int TD, bool FT>
constexpr bool tiled_w4() {
  return (TD & 7) == 1 || TD == 18 || TD == 26 || (FT && (TD == 19 || TD == 27));
}
template <int TDENSITY, bool FT = false, int S = 1>
__global__ __launch_bounds__(TB) void k_fluid_tiled(DevScalars* __restrict__ sc, const uint4* __restrict__ items,
                                                    unsigned* __restrict__ qctr, const float4* __restrict__ poscell,
                                                    const float4* __restrict__ velrhop,
                                                    const float* __restrict__ press,
                                                    const unsigned* __restrict__ bc, DivGrid g, KConst K,
                                                    float4* __restrict__ arace, FtRec ft) {
  fluid_tiled<TDENSITY, FT, S>(sc, items, qctr, poscell, velrhop, press, bc, g, K, arace, ft);
}
template <int TDENSITY, bool FT = false, int S = 1>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_fluid_tiled_w4(
    DevScalars* __restrict__ sc, const uint4* __restrict__ items, unsigned* __restrict__ qctr,
    const float4* __restrict__ poscell, const float4* __restrict__ velrhop, const float* __restrict__ press,
    const unsigned* __restrict__ bc, DivGrid g, KConst K, float4* __restrict__ arace, FtRec ft) {
  fluid_tiled<TDENSITY, FT, S>(sc, items, qctr, poscell, velrhop, press, bc, g, K, arace, ft);
}


template <int S>
static void launch_fluid_tiled_s(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items,
                                 unsigned* qctr, const float4* poscell, const float4* velrhop, const float* press,
                                 const unsigned* begincell, DivGrid g, const KConst& K, float4* arace,
                                 const FtRec& ft, unsigned reserve) {
#define SPH_TILED(TD, FTB)                                                                                     \
  do {                                                                                                         \
    if constexpr (tiled_w4<TD, FTB>())                                                                          \
      hipLaunchKernelGGL((k_fluid_tiled_w4<TD, FTB, S>),                                                       \
                         dim3(fit_grid((const void*)&k_fluid_tiled_w4<TD, FTB, S>, nblocks, TB, reserve)), dim3(TB), 0, stm, \
                         sc, items, qctr, poscell, velrhop, press, begincell, g, K, arace, ft);                \
    else                                                                                                       \
      hipLaunchKernelGGL((k_fluid_tiled<TD, FTB, S>), dim3(fit_grid((const void*)&k_fluid_tiled<TD, FTB, S>, nblocks, TB, reserve)), \
                         dim3(TB), 0, stm, sc, items, qctr, poscell, velrhop, press, begincell, g, K, arace, ft); \
  } while (0)
  // DDT 2/3 with the binomial series of the hydrostatic term (K.ddtseries) as TDENSITY | 8
  // and the Cubic spline kernel as TDENSITY | 16
  const int td = ((K.tdensity >= 2 && K.ddtseries) ? K.tdensity | 8 : K.tdensity) | (K.cubic ? 16 : 0);
  if (ft.massp) {
    switch (td) {
      case 0: SPH_TILED(0, true); break;
      case 1: SPH_TILED(1, true); break;
      case 2: SPH_TILED(2, true); break;
      case 3: SPH_TILED(3, true); break;
      case 10: SPH_TILED(10, true); break;
      case 11: SPH_TILED(11, true); break;
      case 16: SPH_TILED(16, true); break;
      case 17: SPH_TILED(17, true); break;
      case 18: SPH_TILED(18, true); break;
      case 19: SPH_TILED(19, true); break;
      case 26: SPH_TILED(26, true); break;
      default: SPH_TILED(27, true); break;
    }
  } else {
    switch (td) {
      case 0: SPH_TILED(0, false); break;
      case 1: SPH_TILED(1, false); break;
      case 2: SPH_TILED(2, false); break;
      case 3: SPH_TILED(3, false); break;
      case 10: SPH_TILED(10, false); break;
      case 11: SPH_TILED(11, false); break;
      case 16: SPH_TILED(16, false); break;
      case 17: SPH_TILED(17, false); break;
      case 18: SPH_TILED(18, false); break;
      case 19: SPH_TILED(19, false); break;
      case 26: SPH_TILED(26, false); break;
      default: SPH_TILED(27, false); break;
    }
  }
#undef SPH_TILED
}

void launch_fluid_tiled(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                        const float4* poscell, const float4* velrhop, const float* press, const unsigned* begincell,
                        DivGrid g, const KConst& K, float4* arace, const typecode* code, const float* ftmassp,
                        unsigned reserve) {
  const FtRec ft = {code, ftmassp};
#ifdef SPH_DIAG_HEADLINE_ONLY
  // diagnostic builds (kernel A/B at cfg2 only): the one instantiation of BASELINE cfg2
  if (K.scelldiv != 1 || ftmassp || !(K.tdensity == 2 && K.ddtseries) || K.cubic)
    throw std::runtime_error("SPH_DIAG_HEADLINE_ONLY build: cfg2 / cfg5 kernels only");
  hipLaunchKernelGGL((k_fluid_tiled<10, false, 1>), dim3(fit_grid((const void*)&k_fluid_tiled<10, false, 1>, nblocks, TB, reserve)),
                     dim3(TB), 0, stm, sc, items, qctr, poscell, velrhop, press, begincell, g, K, arace, ft);
#else
  if (K.scelldiv == 2)
    launch_fluid_tiled_s<2>(stm, nblocks, sc, items, qctr, poscell, velrhop, press, begincell, g, K, arace, ft, reserve);
  else
    launch_fluid_tiled_s<1>(stm, nblocks, sc, items, qctr, poscell, velrhop, press, begincell, g, K, arace, ft,
                            reserve);
#endif
}

}  // namespace sphx
