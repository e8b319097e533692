// sph_mdbc.hip — modified Dynamic Boundary Conditions (mDBC) on gfx950, SURVEY.md §8(f) row 1.
//
// Reference: JSphCpu::InteractionMdbcCorrectionT2<tker,sim2d,SLIP_Vel0>
// (JSphCpu.cpp:1020-1187; the sim2d branch with its 3x3 system in x, z: :1087-1110), called once per interaction before PreInteraction_Forces
// except in the Symplectic corrector (JSphCpuSingle.cpp:525, MDBCCorrector=0); the GPU
// twin is KerInteractionMdbcCorrection_Dbl (JSphGpu_ker.cu:1088-1250, the MDBCFastSingle=0
// path: the 4x4 correction matrix accumulated and inverted in double, as the CPU does).
//
// For every boundary particle p1 < NpbOk with a normal, the ghost node sits at
// pos + normal (normals already doubled by ConfigBoundNormals: particle -> ghost node).
// Over the fluid particles within the support of the ghost node:
//   rho_g     = sum m W,   grad rho_g = sum m gradW
//   A (4x4)   = sum V [W, dx W, dy W, dz W; gradW, dx gradW, ...]   (V = m / rho2)
// (2-D: A is 3x3 over (1, x, z), JSphCpu.cpp:1087-1110, Determinant3x3 / InverseMatrix3x3
// of FunctionsMath.h:91-93,157-172.)
// If |det A| >= 1e-3: the first-order extrapolation (A^-1 [rho_g, grad rho_g]) mirrored
// back to the particle; else if A11 > 0 the Shepard value rho_g / A11; with no fluid the
// density is RhopZero.  Vel0 keeps the boundary velocity (zero for fixed walls).
//
// Layout/parallelism: one wave per boundary particle, its lanes splitting the candidates
// (see k_mdbc); the summation order therefore differs from the CPU's sequential sums by
// rounding only.  Positions are read in double (posxy/posz) so the
// distances are the reference's float(gpos - pos2) bit for bit.  The normals are kept
// in case (idp) order — boundary ids are < CaseNbound and fixed boundaries never move —
// so the divide never has to reorder them.  The corrected density also refreshes the
// boundary particle's EOS pressure (PreInteraction recomputes it on the CPU).
#include <algorithm>
#include <cfloat>

#include "sph_kernels.hpp"

namespace sphx {

struct MdbcSum;

struct MdbcArgs {
  MdbcSum* sums;  // per listed particle: the wave-reduced sums (pass 2 -> pass 3)
  const unsigned* idp;
  const typecode* code;
  const double2* posxy;
  const double* posz;
  float4* velrhop;
  float* press;
  const float4* normal;  // [CaseNbound], by idp
  const unsigned* dcell;
  unsigned domcellcode;
  const unsigned* bc;
  double posminx, posminy, posminz, scelld;
  float kernelsize2, ovh, awen, bwenovh, massfluid, rhopzero, threshold, determlimit;
  float kernelsize;
  float cteb, ovrhopzero, gamma;
  int igamma;
  int scelldiv;
  int cubic;  // TKernel Cubic spline: GetKernelCubic_WabFac (FunSphKernel.h:122-136)
  float kh, cub_a2, cub_a24, cub_c1, cub_d1, cub_c2;
};

// fmath::Determinant4x4 (FunctionsMath.h:186-199), double.
struct M4 { double a11, a12, a13, a14, a21, a22, a23, a24, a31, a32, a33, a34, a41, a42, a43, a44; };
struct MdbcSum {
  M4 m;
  float r, gx, gy, gz, sumwab;
  unsigned p1;
};
static_assert(sizeof(MdbcSum) == MDBC_SUM_BYTES, "MdbcSum layout");
__device__ inline double det4(const M4& d) {
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

// EOS of the corrected density, as the gather evaluates it (sph_divide.hip gather_one).
__device__ inline float eos_press(const MdbcArgs& a, float rho) {
  const double xr = double(rho * a.ovrhopzero);
  double xg;
  if (a.igamma > 0) {
    double r = 1.0, b = xr;
    for (int e = a.igamma; e; e >>= 1) {
      if (e & 1) r *= b;
      b *= b;
    }
    xg = r;
  } else {
    xg = pow(xr, double(a.gamma));
  }
  return float(double(a.cteb) * (xg - 1.0));
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Ghost node of p1 and its neighbour-cell box: nsearch::Init by position
// (JCellSearch_inline.h:52-67) on the full-map grid, clamped to the grid (equal to the
// reference's ranges for a ghost node inside it).
struct GhostBox {
  double gx, gy, gz;
  int xini, xfin, yini, yfin, zini, zfin;
  int cxu;  // unclamped local x cell of the ghost node
};
template <int SD>
__device__ __forceinline__ GhostBox ghost_box(const MdbcArgs& a, const DivGrid& g, unsigned p1, float4 bn) {
  GhostBox b;
  const double2 pxy = a.posxy[p1];
  b.gx = pxy.x + double(bn.x);
  b.gy = pxy.y + double(bn.y);
  b.gz = a.posz[p1] + double(bn.z);
  const int cx = int((b.gx - a.posminx) / a.scelld) - g.offx();
  b.cxu = cx;
  const int cy = int((b.gy - a.posminy) / a.scelld) - g.offy();
  const int cz = int((b.gz - a.posminz) / a.scelld);
  b.xini = max(cx - SD, 0);
  b.xfin = min(cx + SD + 1, g.ncx);
  b.yini = max(cy - SD, 0);
  b.yfin = min(cy + SD + 1, g.ncy);
  b.zini = max(cz - SD, 0);
  b.zfin = min(cz + SD + 1, g.ncz);
  return b;
}

// Pass 1, one lane per boundary particle p1 < NpbOk: list the particles that have a
// normal and fluid in the cells around their ghost node; a dry one gets what the
// reference's correction gives it with empty sums (RhopZero when 0 >= threshold, else
// unchanged).  Most of the tank's walls are dry, so pass 2 runs over a short list.
// Threads [0, npbcap) take the boundary particles p1 < NpbOk, threads [npbcap, npbcap + nft)
// the floating particles of ftridp (mDBC on floating bodies, JSphCpu.cpp:1199: n = Np).
template <int SD>
__global__ __launch_bounds__(256) void k_mdbc_list(const DevScalars* __restrict__ sc, MdbcArgs a, DivGrid g,
                                                   unsigned* __restrict__ list, unsigned* __restrict__ nlist,
                                                   unsigned npbcap, const unsigned* __restrict__ ftridp,
                                                   unsigned nft) {
  const unsigned t = blockIdx.x * 256u + threadIdx.x;
  unsigned p1 = 0xffffffffu;
  if (t < npbcap) {
    if (t < sc->npbok) p1 = t;
  } else if (t - npbcap < nft) {
    p1 = ftridp[t - npbcap];  // owned floating particle, or none
  }
  const bool valid = p1 != 0xffffffffu;
  bool keep = false;
  bool own = true;
  if (valid && g.split()) own = slab_owned(g, slab_local(g, a.domcellcode, a.dcell[p1]));  // slab: owned p1 only
  if (valid && own) {
    const float4 bn = a.normal[a.idp[p1]];
    if (bn.x != 0.f || bn.y != 0.f || bn.z != 0.f) {
      const GhostBox b = ghost_box<SD>(a, g, p1, bn);
      // slab: every particle within the support of the ghost node must lie inside this
      // slab's grid where a neighbour holds the rest of the domain (the grid edge of the
      // whole map clamps, as the reference's search does); a ghost node in a ghost column
      // is fine while its support stays off the grid edge
      {
        const double pmin = g.axis ? a.posminy : a.posminx, gs = g.axis ? b.gy : b.gx;
        const double edge0 = pmin + double(g.soff) * a.scelld, edge1 = edge0 + double(g.extent()) * a.scelld;
        const double ks = double(a.kernelsize) * (1.0 + 1e-6);
        if ((gs - ks < edge0 && g.sown0 > 0) || (gs + ks >= edge1 && g.sown1 < g.extent()))
          atomicOr(&const_cast<DevScalars*>(sc)->error_flags, ERR_HALO_NODE);
      }
      unsigned tot = 0;
      if (b.xini < b.xfin)
        for (int z = b.zini; z < b.zfin; z++)
          for (int y = b.yini; y < b.yfin; y++) {
            const unsigned rowbase = g.boxfluid + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
            tot += a.bc[rowbase + b.xfin] - a.bc[rowbase + b.xini];
          }
      keep = tot > 0u;
      if (!keep && a.threshold <= 0.f) {
        // no fluid around: all sums 0 >= threshold, det 0 and A11 0 -> rhopfinal = RhopZero
        a.velrhop[p1].w = a.rhopzero;
        a.press[p1] = eos_press(a, a.rhopzero);
      }
    }
  }
  const unsigned long long bal = __ballot(keep);
  const unsigned lane = threadIdx.x & 63u;
  unsigned base = 0;
  if (lane == 0 && bal) base = atomicAdd(nlist, unsigned(__popcll(bal)));
  base = __shfl(base, 0, 64);
  if (keep) list[base + unsigned(__popcll(bal & ((1ull << lane) - 1ull)))] = p1;
}

// Pass 2, one WAVE per listed boundary particle: lanes 0..MAXR-1 read the fluid range of
// one neighbour row each (all row lookups in flight at once), a wave scan flattens the
// non-empty rows into one candidate index space k in [0, total) (row r holds
// [o_r, o_r + n_r), p2 = k + d_r), and the lanes split the candidates, four per lane per
// round with all loads issued before the arithmetic (the kernel is bound by the latency
// of these L2 reads, not by its FP work).  The 5 float and 16 double partial sums are
// reduced across the wave in a fixed butterfly order (deterministic) and lane 0 solves.
template <int SD, bool D2>
__global__ __launch_bounds__(256) void k_mdbc(
    const DevScalars* __restrict__ sc, MdbcArgs a, DivGrid g,
                                              const unsigned* __restrict__ list, const unsigned* __restrict__ nlist) {
  constexpr int W = 2 * SD + 1, MAXR = W * W;
  __shared__ float4 s_acc[4][256];  // accepted pairs of a round, per wave
  const unsigned lane = threadIdx.x & 63u;
  const unsigned nwaves = gridDim.x * 4u;
  const unsigned n = *nlist;
  for (unsigned it = blockIdx.x * 4u + (threadIdx.x >> 6); it < n; it += nwaves) {
    const unsigned p1 = list[it];
    const float4 bn = a.normal[a.idp[p1]];
    const GhostBox b = ghost_box<SD>(a, g, p1, bn);
    const double gx = b.gx, gy = b.gy, gz = b.gz;
    float rhopp1 = 0.f, gx_ = 0.f, gy_ = 0.f, gz_ = 0.f, sumwab = 0.f;
    M4 m = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned rini = 0, rlen = 0;
    if (int(lane) < MAXR && b.xini < b.xfin) {
      const int z = b.zini + int(lane) / W, y = b.yini + int(lane) % W;
      if (z < b.zfin && y < b.yfin) {
        const unsigned rowbase = g.boxfluid + unsigned(z) * g.nsheet + unsigned(y) * unsigned(g.ncx);
        rini = a.bc[rowbase + b.xini];
        rlen = a.bc[rowbase + b.xfin] - rini;
      }
    }
    // exclusive scan of the row lengths over the first MAXR lanes (row order = the
    // reference's z, y loop order)
    unsigned incl = rlen;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
      const unsigned t = __shfl_up(incl, off, 64);
      if (int(lane) >= off) incl += t;
    }
    const unsigned total = __builtin_amdgcn_readfirstlane(__shfl(incl, MAXR - 1, 64));
    const unsigned ofs = incl - rlen;
    unsigned o[MAXR], d[MAXR];
#pragma unroll
    for (int r = 0; r < MAXR; r++) {  // wave-uniform: scalar registers
      o[r] = __builtin_amdgcn_readfirstlane(__shfl(ofs, r, 64));
      d[r] = __builtin_amdgcn_readfirstlane(__shfl(rini, r, 64)) - o[r];
    }
    const bool any = total > 0u;
    // Rounds of 256 candidates (four per lane, all loads issued before the arithmetic):
    // each lane tests its four, the accepted pairs of the round are compacted into the
    // wave's LDS slab (ballot ranks: the reference's candidate order is not needed, the
    // sums are reduced in a fixed order below) and the pair body then runs once per 64
    // ACCEPTED pairs instead of once per candidate slot (only ~1 in 6 candidates lies
    // inside the support, and a divergent body costs the whole wave).
    float4* acc = s_acc[threadIdx.x >> 6];
    for (unsigned k0 = lane; k0 < total; k0 += 256u) {
      unsigned p2[4];
      bool v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const unsigned k = k0 + 64u * unsigned(u);
        v[u] = k < total;
        // the row holding k: the last one starting at or before k (an empty row shares
        // its offset with the next one, which then wins)
        unsigned dd = d[0];
#pragma unroll
        for (int r = 1; r < MAXR; r++)
          if (k >= o[r]) dd = d[r];
        p2[u] = v[u] ? k + dd : p1;
      }
      double2 q[4];
      double qz[4];
      typecode c2[4];
      float rho2[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        q[u] = a.posxy[p2[u]];
        qz[u] = a.posz[p2[u]];
        c2[u] = a.code[p2[u]];
        rho2[u] = a.velrhop[p2[u]].w;
      }
      unsigned nacc = 0;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const float drx = float(gx - q[u].x);
        const float dry = float(gy - q[u].y);
        const float drz = float(gz - qz[u]);
        const float rr2 = drx * drx + dry * dry + drz * drz;
        const bool ok = v[u] && rr2 <= a.kernelsize2 && CodeIsFluid(c2[u]);
        const unsigned long long bal = __ballot(ok);
        if (ok) acc[nacc + unsigned(__popcll(bal & ((1ull << lane) - 1ull)))] = make_float4(drx, dry, drz, rho2[u]);
        nacc += unsigned(__popcll(bal));
      }
      __builtin_amdgcn_wave_barrier();
      for (unsigned j = lane; j < ((nacc + 63u) & ~63u); j += 64u) {
        if (j < nacc) {
          const float4 e = acc[j];
          const float drx = e.x, dry = e.y, drz = e.z;
          const float rr2 = drx * drx + dry * dry + drz * drz;
          // GetKernelWendland_WabFac (FunSphKernel.h:226-234); fac in its r -> 0
          // form (bwen/h)(1-q/2)^3, finite when a fluid particle sits on the ghost node.
          const float rad = sqrtf(rr2);
          const float qq = rad * a.ovh;
          float fac, wab;
          if (a.cubic) {  // wave-uniform; fac within h as (c1 + d1 q) / h (finite at r = 0)
            if (rad > a.kh) {
              const float w1 = 2.f - qq, w2 = w1 * w1;
              fac = a.cub_c2 * w2 / rad;
              wab = a.cub_a24 * (w2 * w1);
            } else {
              fac = (a.cub_c1 + a.cub_d1 * qq) * a.ovh;
              wab = a.cub_a2 * (1.f + (0.75f * qq - 1.5f) * (qq * qq));
            }
          } else {
            const float wqq1 = 1.f - 0.5f * qq;
            const float wqq2 = wqq1 * wqq1;
            fac = a.bwenovh * wqq2 * wqq1;
            const float wqq = qq + qq + 1.f;
            wab = a.awen * wqq * wqq2 * wqq2;
          }
          const float frx = fac * drx, fry = fac * dry, frz = fac * drz;
          const float volp2 = a.massfluid / e.w;
          rhopp1 += a.massfluid * wab;
          gx_ += a.massfluid * frx;
          gy_ += a.massfluid * fry;
          gz_ += a.massfluid * frz;
          const float vwab = wab * volp2;
          sumwab += vwab;
          const float vfrx = frx * volp2, vfry = fry * volp2, vfrz = frz * volp2;
          if (D2) {  // a_corr2 (JSphCpu.cpp:1088-1091) in the a11..a33 slots
            m.a11 += vwab;  m.a12 += drx * vwab;  m.a13 += drz * vwab;
            m.a21 += vfrx;  m.a22 += drx * vfrx;  m.a23 += drz * vfrx;
            m.a31 += vfrz;  m.a32 += drx * vfrz;  m.a33 += drz * vfrz;
          } else {
            m.a11 += vwab;  m.a12 += drx * vwab;  m.a13 += dry * vwab;  m.a14 += drz * vwab;
            m.a21 += vfrx;  m.a22 += drx * vfrx;  m.a23 += dry * vfrx;  m.a24 += drz * vfrx;
            m.a31 += vfry;  m.a32 += drx * vfry;  m.a33 += dry * vfry;  m.a34 += drz * vfry;
            m.a41 += vfrz;  m.a42 += drx * vfrz;  m.a43 += dry * vfrz;  m.a44 += drz * vfrz;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (any) {  // wave-uniform
      rhopp1 = wsum(rhopp1); gx_ = wsum(gx_); gy_ = wsum(gy_); gz_ = wsum(gz_); sumwab = wsum(sumwab);
      m.a11 = wsum(m.a11); m.a12 = wsum(m.a12); m.a13 = wsum(m.a13); m.a14 = wsum(m.a14);
      m.a21 = wsum(m.a21); m.a22 = wsum(m.a22); m.a23 = wsum(m.a23); m.a24 = wsum(m.a24);
      m.a31 = wsum(m.a31); m.a32 = wsum(m.a32); m.a33 = wsum(m.a33); m.a34 = wsum(m.a34);
      m.a41 = wsum(m.a41); m.a42 = wsum(m.a42); m.a43 = wsum(m.a43); m.a44 = wsum(m.a44);
    }
    if (lane != 0u) continue;
    MdbcSum& res = a.sums[it];
    res.m = m;
    res.r = rhopp1;
    res.gx = gx_;
    res.gy = gy_;
    res.gz = gz_;
    res.sumwab = sumwab;
    res.p1 = p1;
  }
}

// Pass 3, one lane per listed particle: the reference's solve of the summed system
// (kept out of pass 2, whose registers then hold only the accumulation).
template <bool D2>
__global__ __launch_bounds__(256) void k_mdbc_solve(MdbcArgs a, const unsigned* __restrict__ nlist) {
  const unsigned it = blockIdx.x * blockDim.x + threadIdx.x;
  if (it >= *nlist) return;
  const MdbcSum& s = a.sums[it];
  const M4 m = s.m;
  const float rhopp1 = s.r, gx_ = s.gx, gy_ = s.gy, gz_ = s.gz, sumwab = s.sumwab;
  const unsigned p1 = s.p1;
  {
    const float4 bn = a.normal[a.idp[p1]];
    const float thr = a.threshold;
    if (!(sumwab >= thr || (thr >= 2.f && sumwab + 2.f >= thr))) return;
    float rhopfinal = FLT_MAX;
    if (D2) {
      // fmath::Determinant3x3 / InverseMatrix3x3 (FunctionsMath.h:91-93,157-172), double
      const M4& d = m;
      const double determ = d.a11 * d.a22 * d.a33 + d.a12 * d.a23 * d.a31 + d.a13 * d.a21 * d.a32 -
                            d.a31 * d.a22 * d.a13 - d.a32 * d.a23 * d.a11 - d.a33 * d.a21 * d.a12;
      if (fabs(determ) >= double(a.determlimit)) {
        const double i11 = (d.a22 * d.a33 - d.a23 * d.a32) / determ;
        const double i12 = -(d.a12 * d.a33 - d.a13 * d.a32) / determ;
        const double i13 = (d.a12 * d.a23 - d.a13 * d.a22) / determ;
        const double i21 = -(d.a21 * d.a33 - d.a23 * d.a31) / determ;
        const double i22 = (d.a11 * d.a33 - d.a13 * d.a31) / determ;
        const double i23 = -(d.a11 * d.a23 - d.a13 * d.a21) / determ;
        const double i31 = (d.a21 * d.a32 - d.a22 * d.a31) / determ;
        const double i32 = -(d.a11 * d.a32 - d.a12 * d.a31) / determ;
        const double i33 = (d.a11 * d.a22 - d.a12 * d.a21) / determ;
        const float rhoghost = float(i11 * rhopp1 + i12 * gx_ + i13 * gz_);
        const float grx = -float(i21 * rhopp1 + i22 * gx_ + i23 * gz_);
        const float grz = -float(i31 * rhopp1 + i32 * gx_ + i33 * gz_);
        rhopfinal = (rhoghost + grx * (-bn.x) + grz * (-bn.z));  // JSphCpu.cpp:1099
      } else if (m.a11 > 0) {
        rhopfinal = float(rhopp1 / m.a11);
      }
      rhopfinal = (rhopfinal != FLT_MAX ? rhopfinal : a.rhopzero);
      a.velrhop[p1].w = rhopfinal;
      a.press[p1] = eos_press(a, rhopfinal);
      return;
    }
    const double determ = det4(m);
    if (fabs(determ) >= double(a.determlimit)) {
      // Rows of fmath::InverseMatrix4x4 (FunctionsMath.h:260-282) that the extrapolation reads.
      const M4& d = m;
      const double i11 = (d.a22 * (d.a33 * d.a44 - d.a34 * d.a43) + d.a23 * (d.a34 * d.a42 - d.a32 * d.a44) + d.a24 * (d.a32 * d.a43 - d.a33 * d.a42)) / determ;
      const double i21 = (d.a21 * (d.a34 * d.a43 - d.a33 * d.a44) + d.a23 * (d.a31 * d.a44 - d.a34 * d.a41) + d.a24 * (d.a33 * d.a41 - d.a31 * d.a43)) / determ;
      const double i31 = (d.a21 * (d.a32 * d.a44 - d.a34 * d.a42) + d.a22 * (d.a34 * d.a41 - d.a31 * d.a44) + d.a24 * (d.a31 * d.a42 - d.a32 * d.a41)) / determ;
      const double i41 = (d.a21 * (d.a33 * d.a42 - d.a32 * d.a43) + d.a22 * (d.a31 * d.a43 - d.a33 * d.a41) + d.a23 * (d.a32 * d.a41 - d.a31 * d.a42)) / determ;
      const double i12 = (d.a12 * (d.a34 * d.a43 - d.a33 * d.a44) + d.a13 * (d.a32 * d.a44 - d.a34 * d.a42) + d.a14 * (d.a33 * d.a42 - d.a32 * d.a43)) / determ;
      const double i22 = (d.a11 * (d.a33 * d.a44 - d.a34 * d.a43) + d.a13 * (d.a34 * d.a41 - d.a31 * d.a44) + d.a14 * (d.a31 * d.a43 - d.a33 * d.a41)) / determ;
      const double i32 = (d.a11 * (d.a34 * d.a42 - d.a32 * d.a44) + d.a12 * (d.a31 * d.a44 - d.a34 * d.a41) + d.a14 * (d.a32 * d.a41 - d.a31 * d.a42)) / determ;
      const double i42 = (d.a11 * (d.a32 * d.a43 - d.a33 * d.a42) + d.a12 * (d.a33 * d.a41 - d.a31 * d.a43) + d.a13 * (d.a31 * d.a42 - d.a32 * d.a41)) / determ;
      const double i13 = (d.a12 * (d.a23 * d.a44 - d.a24 * d.a43) + d.a13 * (d.a24 * d.a42 - d.a22 * d.a44) + d.a14 * (d.a22 * d.a43 - d.a23 * d.a42)) / determ;
      const double i23 = (d.a11 * (d.a24 * d.a43 - d.a23 * d.a44) + d.a13 * (d.a21 * d.a44 - d.a24 * d.a41) + d.a14 * (d.a23 * d.a41 - d.a21 * d.a43)) / determ;
      const double i33 = (d.a11 * (d.a22 * d.a44 - d.a24 * d.a42) + d.a12 * (d.a24 * d.a41 - d.a21 * d.a44) + d.a14 * (d.a21 * d.a42 - d.a22 * d.a41)) / determ;
      const double i43 = (d.a11 * (d.a23 * d.a42 - d.a22 * d.a43) + d.a12 * (d.a21 * d.a43 - d.a23 * d.a41) + d.a13 * (d.a22 * d.a41 - d.a21 * d.a42)) / determ;
      const double i14 = (d.a12 * (d.a24 * d.a33 - d.a23 * d.a34) + d.a13 * (d.a22 * d.a34 - d.a24 * d.a32) + d.a14 * (d.a23 * d.a32 - d.a22 * d.a33)) / determ;
      const double i24 = (d.a11 * (d.a23 * d.a34 - d.a24 * d.a33) + d.a13 * (d.a24 * d.a31 - d.a21 * d.a34) + d.a14 * (d.a21 * d.a33 - d.a23 * d.a31)) / determ;
      const double i34 = (d.a11 * (d.a24 * d.a32 - d.a22 * d.a34) + d.a12 * (d.a21 * d.a34 - d.a24 * d.a31) + d.a14 * (d.a22 * d.a31 - d.a21 * d.a32)) / determ;
      const double i44 = (d.a11 * (d.a22 * d.a33 - d.a23 * d.a32) + d.a12 * (d.a23 * d.a31 - d.a21 * d.a33) + d.a13 * (d.a21 * d.a32 - d.a22 * d.a31)) / determ;
      const float rhoghost = float(i11 * rhopp1 + i12 * gx_ + i13 * gy_ + i14 * gz_);
      const float grx = -float(i21 * rhopp1 + i22 * gx_ + i23 * gy_ + i24 * gz_);
      const float gry = -float(i31 * rhopp1 + i32 * gx_ + i33 * gy_ + i34 * gz_);
      const float grz = -float(i41 * rhopp1 + i42 * gx_ + i43 * gy_ + i44 * gz_);
      // dpos = boundary particle - ghost node = -normal
      rhopfinal = (rhoghost + grx * (-bn.x) + gry * (-bn.y) + grz * (-bn.z));
    } else if (m.a11 > 0) {
      rhopfinal = float(rhopp1 / m.a11);
    }
    rhopfinal = (rhopfinal != FLT_MAX ? rhopfinal : a.rhopzero);
    a.velrhop[p1].w = rhopfinal;  // SLIP_Vel0: density only
    a.press[p1] = eos_press(a, rhopfinal);
  }
}

void launch_mdbc(hipStream_t stm, unsigned npbcap, const DevScalars* sc, const PartArrays& cur, float* press,
                 const float4* normal, const unsigned* begincell, DivGrid g, const KConst& K,
                 const double dom_posmin[3], float threshold, unsigned* list, unsigned* nlist, void* sums,
                 const unsigned* ftridp, unsigned nft) {
  if (!npbcap && !nft) return;
  if (!ftridp) nft = 0;
  MdbcArgs a;
  a.sums = static_cast<MdbcSum*>(sums);
  a.idp = cur.idp;
  a.code = cur.code;
  a.dcell = cur.dcell;
  a.domcellcode = K.domcellcode;
  a.posxy = cur.posxy;
  a.posz = cur.posz;
  a.velrhop = cur.velrhop;
  a.press = press;
  a.normal = normal;
  a.bc = begincell;
  a.posminx = dom_posmin[0];
  a.posminy = dom_posmin[1];
  a.posminz = dom_posmin[2];
  a.scelld = K.scelld;
  a.kernelsize2 = K.kernelsize2;
  a.kernelsize = sqrtf(K.kernelsize2);
  a.ovh = K.ovkernelh;
  a.awen = K.awen;
  a.bwenovh = K.bwenovh;
  a.massfluid = K.massfluid;
  a.rhopzero = K.rhopzero;
  a.threshold = threshold;
  a.determlimit = 1e-3f;  // JSphCpu.cpp:1197
  a.cteb = K.cteb;
  a.ovrhopzero = K.ovrhopzero;
  a.gamma = K.gamma;
  a.igamma = (K.gamma == float(int(K.gamma)) && K.gamma >= 1.f && K.gamma <= 16.f) ? int(K.gamma) : 0;
  a.scelldiv = K.scelldiv;
  a.cubic = K.cubic;
  a.kh = K.kernelh;
  a.cub_a2 = K.cub_a2;
  a.cub_a24 = K.cub_a24;
  a.cub_c1 = K.cub_c1;
  a.cub_d1 = K.cub_d1;
  a.cub_c2 = K.cub_c2;
  (void)hipMemsetAsync(nlist, 0, sizeof(unsigned), stm);
  const unsigned nlistmax = npbcap + nft;
  const unsigned nb1 = (nlistmax + 255u) / 256u;
  // 4 waves per block, one listed particle per wave at a time: enough blocks that the
  // latency-bound waves fill the CUs (2048 blocks left 2 waves per SIMD: 0.76 ms at 4M)
  const unsigned nb2 = std::min((nlistmax + 3u) / 4u, 32768u);
  const dim3 g3((nlistmax + 255u) / 256u);
  if (K.scelldiv == 1) {
    hipLaunchKernelGGL(k_mdbc_list<1>, dim3(nb1), dim3(256), 0, stm, sc, a, g, list, nlist, npbcap, ftridp, nft);
    if (K.sim2d) hipLaunchKernelGGL((k_mdbc<1, true>), dim3(nb2), dim3(256), 0, stm, sc, a, g, list, nlist);
    else hipLaunchKernelGGL((k_mdbc<1, false>), dim3(nb2), dim3(256), 0, stm, sc, a, g, list, nlist);
  } else {
    hipLaunchKernelGGL(k_mdbc_list<2>, dim3(nb1), dim3(256), 0, stm, sc, a, g, list, nlist, npbcap, ftridp, nft);
    if (K.sim2d) hipLaunchKernelGGL((k_mdbc<2, true>), dim3(nb2), dim3(256), 0, stm, sc, a, g, list, nlist);
    else hipLaunchKernelGGL((k_mdbc<2, false>), dim3(nb2), dim3(256), 0, stm, sc, a, g, list, nlist);
  }
  if (K.sim2d) hipLaunchKernelGGL(k_mdbc_solve<true>, g3, dim3(256), 0, stm, a, nlist);
  else hipLaunchKernelGGL(k_mdbc_solve<false>, g3, dim3(256), 0, stm, a, nlist);
}

}  // namespace sphx

// ---- slabs: corrected densities of the face-column boundary particles ------------------------
// mDBC corrects the OWNED boundary particles at the start of an interaction, after the
// divide's exchange sent their (uncorrected) copies to the neighbours as ghosts.  Each
// slab therefore re-sends (idp, rho, press) of its owned boundary particles in its first /
// last owned column (exactly the set the neighbour holds as ghosts, nothing moves in
// between) in a fixed-size buffer (count in slot 0: no host round trip), and the receiver
// writes them into its ghosts located by idp (bidx, rebuilt here).
namespace sphx {

__global__ __launch_bounds__(256) void k_mdbc_face_pack(const DevScalars* __restrict__ sc, PartArrays a,
                                                        const float* __restrict__ press, KConst K, DivGrid g,
                                                        MdbcFaceRec* __restrict__ sl, MdbcFaceRec* __restrict__ sr,
                                                        unsigned capl, unsigned capr, unsigned* __restrict__ bidx, unsigned nbidx,
                                                        int floating) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (floating ? sc->np : sc->npb)) return;
  // floating normals: the floating particles (held owned or as ghosts) are mapped and sent too
  if (p >= sc->npb && CodeType(a.code[p]) != CODE_TYPE_FLOATING) return;
  const unsigned id = a.idp[p];
  if (id < nbidx) bidx[id] = p;
  const int lcx = slab_local(g, K.domcellcode, a.dcell[p]);
  // a slab of one owned column sends the same particle both ways
  for (int side = 0; side < 2; side++) {
    MdbcFaceRec* dst = nullptr;
    unsigned cap = 0;
    if (side == 0 && in_left_face(g, lcx)) { dst = sl; cap = capl; }
    if (side == 1 && in_right_face(g, lcx)) { dst = sr; cap = capr; }
    if (!dst) continue;  // no neighbour on that side
    const unsigned k = atomicAdd(&dst[0].idp, 1u);
    if (k + 1 < cap) dst[k + 1] = MdbcFaceRec{id, a.velrhop[p].w, press[p]};
    else atomicOr(&const_cast<DevScalars*>(sc)->error_flags, ERR_HALO_FACE);
  }
}

__global__ __launch_bounds__(256) void k_mdbc_face_apply(DevScalars* __restrict__ sc,
                                                         const MdbcFaceRec* __restrict__ rl,
                                                         const MdbcFaceRec* __restrict__ rr, unsigned capl,
                                                         unsigned capr, const unsigned* __restrict__ bidx, unsigned nbidx,
                                                         const unsigned* __restrict__ idp,
                                                         float4* __restrict__ velrhop, float* __restrict__ press) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const MdbcFaceRec* r = (blockIdx.y == 0 ? rl : rr);
  const unsigned cap = (blockIdx.y == 0 ? capl : capr);
  if (!r || i + 1 >= cap || i >= r[0].idp) return;
  const MdbcFaceRec q = r[i + 1];
  // bidx was rebuilt by this divide's face pack for the boundary (and floating) particles
  // held now; a stale entry (the particle left this slab) would point at another particle
  const unsigned p = (q.idp < nbidx ? bidx[q.idp] : 0xffffffffu);
  if (p >= sc->np || idp[p] != q.idp) {
    atomicOr(&sc->error_flags, ERR_HALO_MISS);
    return;
  }
  velrhop[p].w = q.rho;
  press[p] = q.press;
}

void launch_mdbc_face_pack(hipStream_t stm, unsigned cap, const DevScalars* sc, const PartArrays& a,
                           const float* press, const KConst& K, const DivGrid& g, MdbcFaceRec* sl, MdbcFaceRec* sr,
                           unsigned capl, unsigned capr, unsigned* bidx, unsigned nbidx, bool floating) {
  if (sl) (void)hipMemsetAsync(sl, 0, sizeof(MdbcFaceRec), stm);
  if (sr) (void)hipMemsetAsync(sr, 0, sizeof(MdbcFaceRec), stm);
  if (cap)
    hipLaunchKernelGGL(k_mdbc_face_pack, dim3((cap + 255) / 256), dim3(256), 0, stm, sc, a, press, K, g, sl, sr,
                       capl, capr, bidx, nbidx, int(floating));
}

void launch_mdbc_face_apply(hipStream_t stm, DevScalars* sc, const MdbcFaceRec* rl, const MdbcFaceRec* rr,
                            unsigned capl, unsigned capr, const unsigned* bidx, unsigned nbidx, const unsigned* idp,
                            float4* velrhop, float* press) {
  const unsigned n = std::max(capl, capr);
  if (!n) return;
  hipLaunchKernelGGL(k_mdbc_face_apply, dim3((n + 255) / 256, 2), dim3(256), 0, stm, sc, rl, rr, capl, capr, bidx,
                     nbidx, idp, velrhop, press);
}

}  // namespace sphx
