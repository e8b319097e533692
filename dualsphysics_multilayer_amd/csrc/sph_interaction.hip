// sph_interaction.hip — Interaction_Forces on CDNA4 (Wendland kernel, artificial
// viscosity, DDT none / Molteni / Fourtakas, DBC boundaries).
//
// Reference semantics (the parity contract):
//   fluid p1 (JSphCpu::InteractionForcesFluid, JSphCpu.cpp:631-822; GPU
//   KerInteractionForcesFluid, JSphGpu_ker.cu:512-745): neighbours in the 3x3x3
//   cells around p1, first the fluid cells (mass MassFluid, Visco) then the bound
//   cells (mass MassBound, Visco*ViscoBoundFactor), momentum + continuity + DDT +
//   artificial viscosity + visc-dt;
//   bound p1 < npbok (JSphCpu::InteractionForcesBound, JSphCpu.cpp:548-625):
//   continuity from fluid neighbours + visc-dt.
// The two fluid passes keep their own accumulators and are combined exactly as the
// CPU stores them (JSphCpu.cpp:800-818) including the sticky FLT_MAX of the DDT
// array and the final Ar += Delta (JSphCpuSingle.cpp:553-559), so the summation
// order per particle is the reference CPU's.
//
// Work decomposition: one lane per particle p1 (cell-sorted order => the lanes of a
// wave share neighbour cells, so candidate loads are wave-broadcast from L1/L2);
// neighbour cells are walked one cell at a time with p1 re-expressed relative to
// the neighbour cell's origin, so a candidate costs 3 subtractions + |r|^2 with no
// cell-code decoding.  ar and ace are written as one float4 (arace), visc-dt and
// |ace|^2 maxima are wave-reduced and folded with one atomicMax per wave.
#include <cfloat>

#include "sph_kernels.hpp"

namespace sphx {

struct Acc {
  float ax, ay, az, ar, delta, visc;
};

// Wendland fac (FunSphKernel.h:217-224).
__device__ __forceinline__ float wendland_fac(const KConst& K, float rr2) {
  const float rad = sqrtf(rr2);
  const float qq = rad / K.kernelh;
  const float wqq1 = 1.f - 0.5f * qq;
  return K.bwen * qq * wqq1 * wqq1 * wqq1 / rad;
}

// One fluid p1 against the particles of one neighbour cell [pini,pfin).
// Floating bodies present (FT): a floating p2 carries its body's particle mass, switches
// DDT off for p1 (Molteni: unless the body is heavy, DELTA_HEAVYFLOATING; Fourtakas: the
// term is skipped) (JSphCpu.cpp:692-703,743).
struct FtView {
  const typecode* code;
  const float* massp;  // per floating body
};

template <int TDENSITY, bool BOUNDP2, bool FT = false>
__device__ __forceinline__ void fluid_cell(const KConst& K, float rx, float ry, float rz, float4 vr1, float pr1,
                                           unsigned pini, unsigned pfin, const float4* __restrict__ poscell,
                                           const float4* __restrict__ velrhop, const float* __restrict__ press,
                                           float massp2c, float visco, Acc& a, FtView ft = {}) {
  for (unsigned p2 = pini; p2 < pfin; p2++) {
    const float4 pc2 = poscell[p2];
    const float drx = rx - pc2.x, dry = ry - pc2.y, drz = rz - pc2.z;
    const float rr2 = drx * drx + dry * dry + drz * drz;
    if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) {
      float massp2 = massp2c;
      bool ftp2 = false;
      if (FT && !BOUNDP2) {
        const typecode c2 = ft.code[p2];
        ftp2 = CodeType(c2) == CODE_TYPE_FLOATING;
        if (ftp2) {
          massp2 = ft.massp[c2 & CODE_MASKVALUE];
          if (TDENSITY == 1 && massp2 <= K.massfluid * 1.2f) a.delta = FLT_MAX;
        }
      }
      const float fac = wendland_fac(K, rr2);
      const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
      const float4 vr2 = velrhop[p2];
      const float pr2 = press[p2];
      {  // Momentum (JSphCpu.cpp:712-716).
        const float prs = (pr1 + pr2) / (vr1.w * vr2.w);
        const float p_vpm = -prs * massp2;
        a.ax += p_vpm * frx;
        a.ay += p_vpm * fry;
        a.az += p_vpm * frz;
      }
      // Continuity (JSphCpu.cpp:719-720).
      const float dvx = vr1.x - vr2.x, dvy = vr1.y - vr2.y, dvz = vr1.z - vr2.z;
      a.ar += massp2 * (dvx * frx + dvy * fry + dvz * frz) * (vr1.w / vr2.w);
      // Density diffusion (JSphCpu.cpp:724-740).
      if (TDENSITY == 1 && a.delta != FLT_MAX) {
        if (BOUNDP2 && !K.mdbc) a.delta = FLT_MAX;  // DBC: DDT off next to the boundary
        else {
          const float rhop1over2 = vr1.w / vr2.w;
          const float visc_densi = K.ddtkh * K.cs0f * (rhop1over2 - 1.f) / (rr2 + K.eta2);
          const float dot3 = (drx * frx + dry * fry + drz * frz);
          a.delta += visc_densi * dot3 * massp2;
        }
      }
      if ((TDENSITY == 2 || (TDENSITY == 3 && !BOUNDP2)) && a.delta != FLT_MAX && !ftp2) {
        if (BOUNDP2) a.delta = FLT_MAX;
        else {
          const float rh = 1.f + K.ddtgz * drz;
          const float drhop = K.rhopzero * powf(rh, K.ovgamma) - K.rhopzero;
          const float visc_densi = K.ddtkh * K.cs0f * ((vr2.w - vr1.w) - drhop) / (rr2 + K.eta2);
          const float dot3 = (drx * frx + dry * fry + drz * frz);
          a.delta -= visc_densi * dot3 * massp2 / vr2.w;
        }
      }
      {  // Artificial viscosity (JSphCpu.cpp:753-764).
        const float dot = drx * dvx + dry * dvy + drz * dvz;
        const float dot_rr2 = dot / (rr2 + K.eta2);
        a.visc = fmaxf(dot_rr2, a.visc);
        if (dot < 0) {
          const float amubar = K.kernelh * dot_rr2;
          const float robar = (vr1.w + vr2.w) * 0.5f;
          const float pi_visc = (-visco * K.cs0f * amubar / robar) * massp2;
          a.ax -= pi_visc * frx;
          a.ay -= pi_visc * fry;
          a.az -= pi_visc * frz;
        }
      }
    }
  }
}

// Neighbour-cell range of p1's cell, clamped to the grid (nsearch::Init, JCellSearch_inline.h:33-47):
// +-scelldiv cells (1 full, 2 half).
struct Range3 {
  int xi, xf, yi, yf, zi, zf;
};
__device__ __forceinline__ Range3 ngs_range(int cx, int cy, int cz, const DivGrid& g, int sd) {
  Range3 r;
  r.xi = cx - (cx < sd ? cx : sd);
  r.xf = cx + (g.ncx - cx - 1 < sd ? g.ncx - cx - 1 : sd) + 1;
  r.yi = cy - (cy < sd ? cy : sd);
  r.yf = cy + (g.ncy - cy - 1 < sd ? g.ncy - cy - 1 : sd) + 1;
  r.zi = cz - (cz < sd ? cz : sd);
  r.zf = cz + (g.ncz - cz - 1 < sd ? g.ncz - cz - 1 : sd) + 1;
  return r;
}

template <int TDENSITY, bool BOUNDP2, bool FT = false>
__device__ __forceinline__ void fluid_pass(const KConst& K, const DivGrid& g, const unsigned* __restrict__ begincell,
                                           const float4 pc1, int cx, int cy, int cz, const Range3& rg, float4 vr1,
                                           float pr1, const float4* __restrict__ poscell,
                                           const float4* __restrict__ velrhop, const float* __restrict__ press, Acc& a,
                                           FtView ft = {}) {
  const unsigned cellinit = (BOUNDP2 ? 0u : g.boxfluid);
  const float massp2 = (BOUNDP2 ? K.massbound : K.massfluid);
  const float visco = (BOUNDP2 ? K.viscobound : K.visco);
  for (int z = rg.zi; z < rg.zf; z++) {
    const float rz = pc1.z + float(cz - z) * K.scell;
    for (int y = rg.yi; y < rg.yf; y++) {
      const float ry = pc1.y + float(cy - y) * K.scell;
      const unsigned row = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
      unsigned pini = begincell[row + rg.xi];
      for (int x = rg.xi; x < rg.xf; x++) {
        const unsigned pfin = begincell[row + x + 1];
        const float rx = pc1.x + float(cx - x) * K.scell;
        fluid_cell<TDENSITY, BOUNDP2, FT>(K, rx, ry, rz, vr1, pr1, pini, pfin, poscell, velrhop, press, massp2, visco, a,
                                          ft);
        pini = pfin;
      }
    }
  }
}

template <int TDENSITY, bool ONLYBOUND = false, bool FT = false>
__global__ __launch_bounds__(256) void k_interaction(DevScalars* __restrict__ sc, const float4* __restrict__ poscell,
                                                     const float4* __restrict__ velrhop,
                                                     const float* __restrict__ press,
                                                     const unsigned* __restrict__ begincell, DivGrid g, KConst K,
                                                     float4* __restrict__ arace, FtView ft = {}) {
  if (K.visco_n) {  // ViscoTime: the step's Visco (k_dt)
    K.visco = sc->visco;
    K.viscobound = K.visco * K.viscobf;
  }
  const unsigned np = sc->np, npb = sc->npb, npbok = sc->npbok;
  const unsigned p1 = blockIdx.x * blockDim.x + threadIdx.x;
  float viscmax = 0.f, ace2 = 0.f;
  if (p1 < np) {
    const float4 pc1 = poscell[p1];
    const float4 vr1 = velrhop[p1];
    const unsigned dc = __float_as_uint(pc1.w);
    const int cx = int(DcelCellx(K.domcellcode, dc)), cy = int(DcelCelly(K.domcellcode, dc)),
              cz = int(DcelCellz(K.domcellcode, dc));
    const Range3 rg = ngs_range(cx, cy, cz, g, K.scelldiv);
    const bool own = slab_owned(g, g.axis ? cy : cx);  // slab ghosts are not p1
    if (!own) {
    } else if (!ONLYBOUND && p1 >= npb) {
      // ---- fluid p1 ----
      const float pr1 = press[p1];
      Acc f = {0, 0, 0, 0, 0, 0};
      Acc b = {0, 0, 0, 0, 0, 0};
      // a floating p1 gets no DDT (JSphCpu.cpp:659-662): both passes start sticky
      if (FT && TDENSITY && CodeType(ft.code[p1]) == CODE_TYPE_FLOATING) f.delta = b.delta = FLT_MAX;
      fluid_pass<TDENSITY, false, FT>(K, g, begincell, pc1, cx, cy, cz, rg, vr1, pr1, poscell, velrhop, press, f, ft);
      fluid_pass<TDENSITY, true, FT>(K, g, begincell, pc1, cx, cy, cz, rg, vr1, pr1, poscell, velrhop, press, b, ft);
      // Store exactly as the two CPU passes do (JSphCpu.cpp:800-818).
      float ar = 0.f, ax = 0.f, ay = 0.f, az = 0.f, delta = 0.f;
      if (f.ar != 0.f || f.ax != 0.f || f.ay != 0.f || f.az != 0.f || f.visc != 0.f) {
        if (TDENSITY) delta = (f.delta == FLT_MAX ? FLT_MAX : 0.f + f.delta);
        ar = 0.f + f.ar;
        ax = 0.f + f.ax;
        ay = 0.f + f.ay;
        az = 0.f + f.az;
      }
      if (b.ar != 0.f || b.ax != 0.f || b.ay != 0.f || b.az != 0.f || b.visc != 0.f) {
        if (TDENSITY) delta = (delta == FLT_MAX || b.delta == FLT_MAX ? FLT_MAX : delta + b.delta);
        ar += b.ar;
        ax += b.ax;
        ay += b.ay;
        az += b.az;
      }
      if (TDENSITY && delta != FLT_MAX) ar += delta;  // JSphCpuSingle.cpp:553-559
      if (K.sim2d) ay = 0.f;  // Simulate2D: Acec[].y = 0 (JSphCpuSingle.cpp:544-549)
      arace[p1] = make_float4(ax, ay, az, ar);
      viscmax = fmaxf(f.visc, b.visc);
      ace2 = ax * ax + ay * ay + az * az;  // ComputeAceMaxOmp (JSphCpuSingle.cpp:612-644)
    } else if (p1 < npb) {
      // ---- bound p1 (DBC) ----
      float arp1 = 0.f, visc = 0.f;
      if (p1 < npbok) {
        for (int z = rg.zi; z < rg.zf; z++) {
          const float rz = pc1.z + float(cz - z) * K.scell;
          for (int y = rg.yi; y < rg.yf; y++) {
            const float ry = pc1.y + float(cy - y) * K.scell;
            const unsigned row = g.boxfluid + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
            unsigned pini = begincell[row + rg.xi];
            for (int x = rg.xi; x < rg.xf; x++) {
              const unsigned pfin = begincell[row + x + 1];
              const float rx = pc1.x + float(cx - x) * K.scell;
              for (unsigned p2 = pini; p2 < pfin; p2++) {
                const float4 pc2 = poscell[p2];
                const float drx = rx - pc2.x, dry = ry - pc2.y, drz = rz - pc2.z;
                const float rr2 = drx * drx + dry * dry + drz * drz;
                if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) {
                  const float fac = wendland_fac(K, rr2);
                  const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
                  const float4 vr2 = velrhop[p2];
                  const float dvx = vr1.x - vr2.x, dvy = vr1.y - vr2.y, dvz = vr1.z - vr2.z;
                  float massp2 = K.massfluid;  // JSphCpu.cpp:589-594
                  if (FT) {
                    const typecode c2 = ft.code[p2];
                    if (CodeType(c2) == CODE_TYPE_FLOATING) massp2 = ft.massp[c2 & CODE_MASKVALUE];
                  }
                  arp1 += massp2 * (dvx * frx + dvy * fry + dvz * frz) * (vr1.w / vr2.w);
                  const float dot = drx * dvx + dry * dvy + drz * dvz;
                  const float dot_rr2 = dot / (rr2 + K.eta2);
                  visc = fmaxf(dot_rr2, visc);
                }
              }
              pini = pfin;
            }
          }
        }
      }
      arace[p1] = make_float4(0.f, 0.f, 0.f, (arp1 != 0.f || visc != 0.f) ? 0.f + arp1 : 0.f);
      viscmax = visc;
    }
  }
  wave_max_atomic(sc, RED_VISCDT, viscmax);
  wave_max_atomic(sc, RED_ACEMAX2, ace2);
}

void launch_interaction(hipStream_t stm, unsigned cap, DevScalars* sc, const float4* poscell, const float4* velrhop,
                        const float* press, const unsigned* begincell, DivGrid g, const KConst& K, float4* arace,
                        const typecode* code, const float* ftmassp) {
  const unsigned nb = (cap + 255) / 256;
  if (ftmassp) {
    const FtView ft = {code, ftmassp};
    switch (K.tdensity) {
      case 0: hipLaunchKernelGGL((k_interaction<0, false, true>), dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace, ft); break;
      case 1: hipLaunchKernelGGL((k_interaction<1, false, true>), dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace, ft); break;
      case 2: hipLaunchKernelGGL((k_interaction<2, false, true>), dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace, ft); break;
      default: hipLaunchKernelGGL((k_interaction<3, false, true>), dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace, ft); break;
    }
    return;
  }
  switch (K.tdensity) {
    case 0: hipLaunchKernelGGL(k_interaction<0>, dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace); break;
    case 1: hipLaunchKernelGGL(k_interaction<1>, dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace); break;
    case 2: hipLaunchKernelGGL(k_interaction<2>, dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace); break;
    default: hipLaunchKernelGGL(k_interaction<3>, dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, press, begincell, g, K, arace); break;
  }
}

void launch_interaction_bound(hipStream_t stm, unsigned npbcap, DevScalars* sc, const float4* poscell,
                              const float4* velrhop, const unsigned* begincell, DivGrid g, const KConst& K,
                              float4* arace) {
  const unsigned nb = (npbcap + 255) / 256;
  if (nb) hipLaunchKernelGGL((k_interaction<0, true>), dim3(nb), dim3(256), 0, stm, sc, poscell, velrhop, nullptr,
                             begincell, g, K, arace);
}

// ---------------------------------------------------------------------------------
// JDsPips-style pair counters: checked candidates and real (r <= 2h) pairs for the
// three passes, accumulated with one 64-bit atomic per wave.
__global__ __launch_bounds__(256) void k_count_pairs(const DevScalars* __restrict__ sc,
                                                     const float4* __restrict__ poscell,
                                                     const unsigned* __restrict__ begincell, DivGrid g, KConst K,
                                                     unsigned long long* __restrict__ out) {
  const unsigned np = sc->np, npb = sc->npb, npbok = sc->npbok;
  const unsigned p1 = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
  const float4 pc1 = p1 < np ? poscell[p1] : make_float4(0.f, 0.f, 0.f, 0.f);
  const int cx = int(DcelCellx(K.domcellcode, __float_as_uint(pc1.w)));
  const int cy = int(DcelCelly(K.domcellcode, __float_as_uint(pc1.w)));
  if (p1 < np && (p1 >= npb || p1 < npbok) && slab_owned(g, g.axis ? cy : cx)) {
    const unsigned dc = __float_as_uint(pc1.w);
    const int cz = int(DcelCellz(K.domcellcode, dc));
    const Range3 rg = ngs_range(cx, cy, cz, g, K.scelldiv);
    const bool fluid = p1 >= npb;
    for (int pass = 0; pass < (fluid ? 2 : 1); pass++) {
      const unsigned cellinit = (fluid && pass == 1) ? 0u : g.boxfluid;
      const int slot = fluid ? 2 * pass : 4;
      for (int z = rg.zi; z < rg.zf; z++)
        for (int y = rg.yi; y < rg.yf; y++) {
          const unsigned row = cellinit + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
          for (int x = rg.xi; x < rg.xf; x++) {
            const float rx = pc1.x + float(cx - x) * K.scell, ry = pc1.y + float(cy - y) * K.scell,
                        rz = pc1.z + float(cz - z) * K.scell;
            for (unsigned p2 = begincell[row + x]; p2 < begincell[row + x + 1]; p2++) {
              const float4 pc2 = poscell[p2];
              const float drx = rx - pc2.x, dry = ry - pc2.y, drz = rz - pc2.z;
              const float rr2 = drx * drx + dry * dry + drz * drz;
              c[slot]++;
              if (rr2 <= K.kernelsize2 && rr2 >= ALMOSTZERO) c[slot + 1]++;
            }
          }
        }
    }
  }
  for (int k = 0; k < 6; k++) {
    unsigned long long v = c[k];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&out[k], v);
  }
}

void launch_count_pairs(hipStream_t stm, unsigned cap, const DevScalars* sc, const float4* poscell,
                        const unsigned* begincell, DivGrid g, const KConst& K, unsigned long long* out6) {
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_count_pairs, dim3(nb), dim3(256), 0, stm, sc, poscell, begincell, g, K, out6);
}

}  // namespace sphx
