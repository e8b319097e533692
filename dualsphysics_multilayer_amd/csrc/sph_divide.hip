// sph_divide.hip — DivideGpu on CDNA4: cell keys, stable LSD radix sort, begincell,
// fused gather + poscell + EOS pressure + VelMax.
//
// Reference behaviour (JCellDivGpuSingle::Divide, JCellDivGpuSingle.cpp:152-235;
// CPU parity source JCellDivCpuSingle.cpp:134-344):
//   * box key: bound cells [0,nct), BoundIgnore nct, fluid cells [nct+1, 2nct+1),
//     then BoundOut, FluidOut, BoundOutIgnore, FluidOutIgnore (KerPreSortFull,
//     JCellDivGpuSingle_ker.cu:41-102), cell index cx + cy*ncx + cz*nsheet (x fastest);
//   * the order inside a box is the previous order (the CPU counting sort is stable,
//     JCellDivCpuSingle.cpp:203-234), which fixes the neighbour summation order —
//     so the sort here is a STABLE radix sort (the reference GPU leaves stability to
//     thrust; -stable selects stable_sort_by_key, JCellDivGpu_ker.cu:116-124);
//   * the cell domain is the whole map (CellDomFixed, -cellfixed:1): the box order is
//     lexicographic in (z,y,x) either way, and bound particles outside a dynamic
//     domain are never neighbours of fluid, so the interaction order is unchanged
//     (checked on the oracle: tests/test_oracle_celldomfixed.py).  This removes the
//     per-step DtoH read of the cell limits (cudiv::LimitsCell, 2 syncs per divide).
#include <cstring>

#include "sph_items.hpp"
#include "sph_kernels.hpp"
#include "sph_incdiv.hpp"

namespace sphx {

// PreSort — one thread per particle, bounded by the live count.
__global__ __launch_bounds__(256) void k_presort(const DevScalars* __restrict__ sc, const unsigned* __restrict__ dcell,
                                                 const typecode* __restrict__ code, DivGrid g, unsigned dcc,
                                                 unsigned* __restrict__ keys, unsigned* __restrict__ vals,
                                                 unsigned extra) {
  const unsigned n = sc->np;
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) const_cast<DevScalars*>(sc)->ndiv = n + extra;
  if (p >= n) return;
  vals[p] = p;
  keys[p] = box_key(dcell[p], code[p], g, dcc);
}

void launch_presort(hipStream_t stm, unsigned cap, const DevScalars* sc, const unsigned* dcell, const typecode* code,
                    DivGrid g, unsigned domcellcode, unsigned* keys, unsigned* vals, unsigned extra) {
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_presort, dim3(nb), dim3(256), 0, stm, sc, dcell, code, g, domcellcode, keys, vals, extra);
}

// ---------------------------------------------------------------------------------
// Stable LSD radix sort.  Per pass: tile histograms (tile-major) -> per-digit scans over
// the tiles (digit totals) -> stable scatter (digit totals scanned in each block's
// prologue; wave match via ballots + tagged LDS wave counts).
__global__ __launch_bounds__(RS_BS) void k_rs_hist(const DevScalars* __restrict__ sc, const unsigned* __restrict__ keys,
                                                   unsigned shift, unsigned rbits, unsigned ntiles,
                                                   unsigned* __restrict__ hist, unsigned nfix) {
  __shared__ unsigned cnt[1 << RS_MAXBITS];
  const unsigned radix = 1u << rbits, mask = radix - 1;
  for (unsigned d = threadIdx.x; d < radix; d += RS_BS) cnt[d] = 0;
  __syncthreads();
  const unsigned n = nfix != ~0u ? nfix : sc->ndiv;
  const unsigned base = blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int it = 0; it < RS_ITEMS; it++) {
    const unsigned idx = base + it * RS_BS + threadIdx.x;
    if (idx < n) atomicAdd(&cnt[(keys[idx] >> shift) & mask], 1u);
  }
  __syncthreads();
  for (unsigned d = threadIdx.x; d < radix; d += RS_BS) hist[blockIdx.x * radix + d] = cnt[d];
}

// Per digit, the exclusive scan over the tiles of hist[tile*radix + d] (tile-major, so
// the histogram and scatter kernels read and write whole rows); the digit total to
// digtot[d].  A block takes SCAN_D consecutive digits x SCAN_C tile chunks: a lane
// (digit j, chunk c) walks its chunk, the lanes of a digit group read consecutive words.
constexpr int SCAN_D = 4, SCAN_C = 64;
__global__ __launch_bounds__(256) void k_rs_scan_tiles(unsigned* __restrict__ hist, unsigned ntiles, unsigned radix,
                                                       unsigned* __restrict__ digtot) {
  __shared__ unsigned s_sum[SCAN_C][SCAN_D];
  const unsigned j = threadIdx.x % SCAN_D, c = threadIdx.x / SCAN_D;
  const unsigned d = blockIdx.x * SCAN_D + j;
  const unsigned per = (ntiles + SCAN_C - 1) / SCAN_C, b0 = c * per;
  const unsigned b1 = d < radix ? min(b0 + per, ntiles) : b0;  // radix < SCAN_D: idle lanes
  // chunks of <= CH tiles stay in registers (one round of independent loads)
  constexpr unsigned CH = 8;
  const bool inreg = per <= CH;
  unsigned v[CH];
  unsigned sum = 0;
  if (inreg) {
#pragma unroll
    for (unsigned k = 0; k < CH; k++) {
      v[k] = (b0 + k < b1) ? hist[size_t(b0 + k) * radix + d] : 0u;
      sum += v[k];
    }
  } else {
    for (unsigned b = b0; b < b1; b++) sum += hist[size_t(b) * radix + d];
  }
  s_sum[c][j] = sum;
  __syncthreads();
  unsigned run = 0;
  for (unsigned cc = 0; cc < c; cc++) run += s_sum[cc][j];
  if (inreg) {
#pragma unroll
    for (unsigned k = 0; k < CH; k++) {
      if (b0 + k < b1) hist[size_t(b0 + k) * radix + d] = run;
      run += v[k];
    }
  } else {
    for (unsigned b = b0; b < b1; b++) {
      const size_t k = size_t(b) * radix + d;
      const unsigned x = hist[k];
      hist[k] = run;
      run += x;
    }
  }
  if (c == SCAN_C - 1 && d < radix) digtot[d] = run;
}

__global__ __launch_bounds__(RS_BS) void k_rs_scatter(const DevScalars* __restrict__ sc,
                                                      const unsigned* __restrict__ kin, const unsigned* __restrict__ vin,
                                                      unsigned* __restrict__ kout, unsigned* __restrict__ vout,
                                                      unsigned shift, unsigned rbits, unsigned ntiles,
                                                      const unsigned* __restrict__ hist,
                                                      const unsigned* __restrict__ digtot, unsigned nfix) {
  constexpr int NW = RS_BS / 64;
  __shared__ unsigned s_off[1 << RS_MAXBITS];
  __shared__ unsigned s_wc[NW][1 << RS_MAXBITS];
  __shared__ unsigned s_part[RS_BS];
  const unsigned radix = 1u << rbits, mask = radix - 1;
  const unsigned n = nfix != ~0u ? nfix : sc->ndiv;
  const unsigned base = blockIdx.x * RS_TILE;
  if (base >= n) return;  // whole block uniform
  // exclusive scan of the digit totals (<= 2048, contiguous per thread) in LDS
  const unsigned per = (radix + RS_BS - 1) / RS_BS, d0 = threadIdx.x * per, d1 = min(d0 + per, radix);
  unsigned run = 0;
  for (unsigned d = d0; d < d1; d++) {
    const unsigned v = digtot[d];
    s_off[d] = run;
    run += v;
  }
  s_part[threadIdx.x] = run;
  __syncthreads();
  for (int off = 1; off < RS_BS; off <<= 1) {
    const unsigned v = threadIdx.x >= unsigned(off) ? s_part[threadIdx.x - off] : 0u;
    __syncthreads();
    s_part[threadIdx.x] += v;
    __syncthreads();
  }
  const unsigned pre = threadIdx.x ? s_part[threadIdx.x - 1] : 0u;
  for (unsigned d = d0; d < d1; d++) s_off[d] += pre;
  __syncthreads();
  for (unsigned d = threadIdx.x; d < radix; d += RS_BS) {
    s_off[d] += hist[size_t(blockIdx.x) * radix + d];
#pragma unroll
    for (int w = 0; w < NW; w++) s_wc[w][d] = 0;
  }
  __syncthreads();
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lanemask_lt = (1ull << lane) - 1ull;
  for (int it = 0; it < RS_ITEMS; it++) {
    const unsigned idx = base + it * RS_BS + threadIdx.x;
    const bool valid = idx < n;
    const unsigned key = valid ? kin[idx] : 0u;
    const unsigned val = valid ? vin[idx] : 0u;
    const unsigned d = (key >> shift) & mask;
    unsigned long long peers = __ballot(valid);
    for (unsigned b = 0; b < rbits; b++) {
      const bool bit = (d >> b) & 1u;
      const unsigned long long bb = __ballot(bit);
      peers &= (bit ? bb : ~bb);
    }
    const unsigned rank = __popcll(peers & lanemask_lt);
    const unsigned cnt = __popcll(peers);
    const bool leader = valid && (peers & lanemask_lt) == 0ull;
    const unsigned tag = unsigned(it + 1) << 16;
    if (leader) s_wc[w][d] = tag | cnt;
    __syncthreads();
    if (valid) {
      unsigned pre = 0;
      for (unsigned ww = 0; ww < w; ww++) {
        const unsigned v = s_wc[ww][d];
        if ((v & 0xffff0000u) == tag) pre += v & 0xffffu;
      }
      const unsigned pos = s_off[d] + pre + rank;
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    if (leader) {
      bool last = true;
      unsigned total = 0;
      for (unsigned ww = 0; ww < NW; ww++) {
        const unsigned v = s_wc[ww][d];
        if ((v & 0xffff0000u) == tag) {
          total += v & 0xffffu;
          if (ww > w) last = false;
        }
      }
      if (last) s_off[d] += total;
    }
    __syncthreads();
  }
}

int launch_radix_sort(hipStream_t stm, unsigned cap, const DevScalars* sc, SortScratch& s, unsigned keybits,
                      unsigned nfix) {
  const unsigned passes = (keybits + RS_MAXBITS - 1) / RS_MAXBITS;
  const unsigned rbits = (keybits + passes - 1) / passes;
  const unsigned ntiles = ((nfix != ~0u && nfix < cap ? nfix : cap) + RS_TILE - 1) / RS_TILE;
  if (ntiles == 0) return 0;
  int cur = 0;
  for (unsigned p = 0; p < passes; p++) {
    const unsigned shift = p * rbits;
    const unsigned radix = 1u << rbits;
    hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(RS_BS), 0, stm, sc, s.keys[cur], shift, rbits, ntiles, s.hist,
                       nfix);
    hipLaunchKernelGGL(k_rs_scan_tiles, dim3((radix + SCAN_D - 1) / SCAN_D), dim3(256), 0, stm, s.hist, ntiles, radix, s.digtot);
    hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(RS_BS), 0, stm, sc, s.keys[cur], s.vals[cur],
                       s.keys[cur ^ 1], s.vals[cur ^ 1], shift, rbits, ntiles, s.hist, s.digtot, nfix);
    cur ^= 1;
  }
  return cur;
}

// ---------------------------------------------------------------------------------
// begincell[c] = first sorted index with key >= c (lower bound) for every box c.
// Particles move less than a cell per step, so the previous divide's begincell[c] is
// close to the new one: a galloping search from it (1-3 probes typically, any guess
// is correct, just slower) instead of a 20-probe binary search.
__device__ inline unsigned lower_bound_u32(const unsigned* __restrict__ a, unsigned lo, unsigned hi, unsigned v) {
  while (lo < hi) {
    const unsigned mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ inline unsigned gallop_lb(const unsigned* __restrict__ a, unsigned n, unsigned v, unsigned g) {
  g = min(g, n);
  if (g > 0 && a[g - 1] >= v) {  // answer in [0, g-1]: step left
    unsigned hi = g - 1, step = 1;
    while (hi >= step && a[hi - step] >= v) {
      hi -= step;
      step <<= 1;
    }
    const unsigned lo = hi >= step ? hi - step + 1 : 0u;
    return lower_bound_u32(a, lo, hi, v);
  }
  if (g < n && a[g] < v) {  // answer in [g+1, n]: step right
    unsigned lo = g + 1, step = 1;
    while (lo + step - 1 < n && a[lo + step - 1] < v) {
      lo += step;
      step <<= 1;
    }
    const unsigned hi = min(lo + step - 1, n);
    return lower_bound_u32(a, lo, hi, v);
  }
  return g;
}

__global__ __launch_bounds__(256) void k_begincell(DevScalars* __restrict__ sc, const unsigned* __restrict__ skeys,
                                                   DivGrid g, unsigned* __restrict__ begincell) {
  const unsigned n = sc->ndiv;
  const unsigned c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.nctt) return;
  const unsigned b = gallop_lb(skeys, n, c, begincell[c]);
  begincell[c] = b;
  // JCellDivCpuSingle::Divide counts (JCellDivCpuSingle.cpp:330-339) + RunCellDivide
  // (JSphCpuSingle.cpp:470-472), each from the thread of its box.
  if (c == g.boxboundignore) sc->npbok = b;
  if (c == g.boxfluid) sc->npb = b;
  if (c == g.boxboundout) sc->np = b;
  if (c == g.boxfluidout) {
    const unsigned b1 = lower_bound_u32(skeys, b, n, c + 1);
    sc->nout += b1 - b;
    const unsigned npbout = b - lower_bound_u32(skeys, 0, b, g.boxboundout);
    if (npbout) {
      sc->npbout = npbout;
      sc->error_flags |= ERR_BOUNDOUT;
    }
  }
}

void launch_begincell(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* skeys, DivGrid g,
                      unsigned* begincell) {
  (void)cap;
  const unsigned nb = (g.nctt + 255) / 256;
  hipLaunchKernelGGL(k_begincell, dim3(nb), dim3(256), 0, stm, sc, skeys, g, begincell);
}

// ---------------------------------------------------------------------------------
// Gather of every particle array + poscell + press + VelMax (fluid only).
struct GatherArgs {
  PartArrays src, dst;
  const unsigned* sortpart;
  float4* poscell;
  float* press;
  double posminx, posminy, posminz, scelld;
  float cteb, ovrhopzero, gamma, rhopzero;
  int igamma;  // gamma as a small positive integer, else 0
  unsigned dcc;
  int withm1, withpre;
  int xoff, yoff;  // slab: the local grid's offset (the slab axis only)
  // NN multiphase: per-phase EOS {rho0, cteb, gamma, integer gamma or 0} (nullptr: single phase)
  const float4* phase_eos;
  // slab: sorted values >= vfirst are reserved ghost slots -> apppos[value - appbase]
  unsigned vfirst, appbase;
  unsigned* apppos;
  int allp;  // DtAllParticles: VelMax over every particle (JSphCpu.cpp:475), else fluid only
};

// WITHM1 / WITHPRE are template parameters so every load of a particle is issued before
// the first store (as runtime flags the compiler kept the optional arrays in separate
// load -> wait -> store round trips).  GP particles per thread (i, i + 256, ...): the
// kernel is bound by two dependent memory latencies (sortpart, then the particle), so
// more bytes in flight per wave shorten it.
#ifndef SPH_GP
#define SPH_GP 4
#endif
constexpr int GP = SPH_GP;

// One particle's state, loaded from its source index (all loads issued before any store).
template <bool WITHM1, bool WITHPRE, bool WITHTAU = false> struct GatherRec {
  unsigned dc, idp;
  double2 pxy, pxypre;
  double pz, pzpre;
  float4 vr, m1, vpre;
  float4 ta, tb;  // Laminar+SPS tau (src.tau set: JSphCpuSingle.cpp:463 sorts SpsTauc too)
  typecode code;
  __device__ __forceinline__ void load(const PartArrays& src, unsigned s) {
    dc = src.dcell[s];
    pxy = src.posxy[s];
    pz = src.posz[s];
    vr = src.velrhop[s];
    idp = src.idp[s];
    code = src.code[s];
    if (WITHM1) m1 = src.velrhopm1[s];
    if (WITHPRE) {
      pxypre = src.posxypre[s];
      pzpre = src.poszpre[s];
      vpre = src.velrhoppre[s];
    }
    if constexpr (WITHTAU) {
      ta = src.tau[2 * s];
      tb = src.tau[2 * s + 1];
    }
  }
};

// Stores a loaded particle at its sorted index i with its poscell and press.
template <bool WITHM1, bool WITHPRE, bool WITHTAU>
__device__ __forceinline__ void gather_store(const GatherArgs& a, unsigned i,
                                             const GatherRec<WITHM1, WITHPRE, WITHTAU>& q) {
  const unsigned dc = q.dc;
  const double2 pxy = q.pxy;
  const double pz = q.pz;
  const float4 vr = q.vr;
  const typecode code = q.code;
  a.dst.idp[i] = q.idp;
  a.dst.code[i] = code;
  a.dst.dcell[i] = dc;
  a.dst.posxy[i] = pxy;
  a.dst.posz[i] = pz;
  a.dst.velrhop[i] = vr;
  if (WITHM1) a.dst.velrhopm1[i] = q.m1;
  if (WITHPRE) {
    a.dst.posxypre[i] = q.pxypre;
    a.dst.poszpre[i] = q.pzpre;
    a.dst.velrhoppre[i] = q.vpre;
  }
  if constexpr (WITHTAU) {
    a.dst.tau[2 * i] = q.ta;
    a.dst.tau[2 * i + 1] = q.tb;
  }
  // PosCell (KerUpdatePosCell): position relative to the origin of its divide cell
  // (global cell -> the same floats on every slab); w = the local cell.
  const unsigned cx = DcelCellx(a.dcc, dc), cy = DcelCelly(a.dcc, dc), cz = DcelCellz(a.dcc, dc);
  const double ox = a.posminx + double(cx) * a.scelld;
  const double oy = a.posminy + double(cy) * a.scelld;
  const double oz = a.posminz + double(cz) * a.scelld;
  const unsigned ldc = (a.xoff | a.yoff) ? DcelCell(a.dcc, cx - unsigned(a.xoff), cy - unsigned(a.yoff), cz) : dc;
  a.poscell[i] = make_float4(float(pxy.x - ox), float(pxy.y - oy), float(pz - oz), __uint_as_float(ldc));
  // Press (PreInteractionVars_Forces, JSphCpu.cpp:451-453; FunSphEos.h:37-47) as the
  // reference binary evaluates it: the unqualified pow in namespace fsph is the C
  // double pow, and -ffast-math makes rhop/rhop0 a product with 1/rhop0.  For an
  // integer gamma the double power is formed by squaring (<= 4 roundings at 1e-16,
  // far below the float rounding of the result).
  auto powg = [](double x, int ig, double g) -> double {
    if (ig > 0) {  // integer gamma (7 in every case here): exact squaring in double
      double r = 1.0, b = x;
      for (int e = ig; e; e >>= 1) {
        if (e & 1) r *= b;
        b *= b;
      }
      return r;
    }
    return pow(x, g);
  };
  if (a.phase_eos) {
    // ComputePress_NN (JSphCpu_Tensors.cpp:40-62 of the v5.0 solver): the phase's rho0, CteB
    // and gamma for fluid particles, the case's for the boundary, in float arithmetic
    // (cteb*(powf(rhop/rho0,gamma)-1)); the power is rounded once from double.
    float rho0 = a.rhopzero, cteb = a.cteb, gam = a.gamma;
    int ig = a.igamma;
    if (CodeIsFluid(code)) {
      const float4 e = a.phase_eos[code & CODE_MASKVALUE];
      rho0 = e.x;
      cteb = e.y;
      gam = e.z;
      ig = int(e.w);
    }
    const float r = vr.w / rho0;
    a.press[i] = cteb * (float(powg(double(r), ig, double(gam))) - 1.0f);
  } else {
    const double xr = double(vr.w * a.ovrhopzero);
    a.press[i] = float(double(a.cteb) * (powg(xr, a.igamma, double(a.gamma)) - 1.0));
  }
}


template <bool WITHM1, bool WITHPRE, bool WITHTAU>
__device__ __forceinline__ void gather_one(const GatherArgs& a, unsigned i, unsigned s, float4& vr_out, bool& fluid,
                                           unsigned npb) {
  GatherRec<WITHM1, WITHPRE, WITHTAU> q;
  q.load(a.src, s);
  gather_store<WITHM1, WITHPRE, WITHTAU>(a, i, q);
  vr_out = q.vr;
  fluid = i >= npb;
}

template <bool WITHM1, bool WITHPRE, bool WITHTAU>
__global__ __launch_bounds__(256) void k_gather(DevScalars* __restrict__ sc, GatherArgs a) {
  const unsigned n = sc->np, npb = sc->npb;
  const unsigned i0 = blockIdx.x * (256 * GP) + threadIdx.x;
  unsigned sp[GP];
#pragma unroll
  for (int k = 0; k < GP; k++) sp[k] = (i0 + 256 * k < n) ? a.sortpart[i0 + 256 * k] : 0u;
  float v2 = 0.f;
#pragma unroll
  for (int k = 0; k < GP; k++) {
    const unsigned i = i0 + 256 * k;
    if (i < n && sp[k] >= a.vfirst) {  // a reserved ghost slot: filled by launch_ghost_scatter
      a.apppos[sp[k] - a.appbase] = i;
    } else if (i < n) {
      float4 vr;
      bool fluid;
      gather_one<WITHM1, WITHPRE, WITHTAU>(a, i, sp[k], vr, fluid, npb);
      if (fluid || a.allp) v2 = nanmax(v2, vr.x * vr.x + vr.y * vr.y + vr.z * vr.z);  // CalcVelMaxOmp
    }
  }
  wave_max_atomic(sc, RED_VELMAX2, v2);
}

void launch_gather(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* sortpart, const PartArrays& src,
                   const PartArrays& dst, bool withm1, bool withpre, const KConst& K, const double dom_posmin[3],
                   float4* poscell, float* press, int xoff, int yoff, const float4* phase_eos, unsigned vfirst,
                   unsigned appbase, unsigned* apppos) {
  GatherArgs a;
  a.phase_eos = phase_eos;
  a.vfirst = vfirst;
  a.appbase = appbase;
  a.apppos = apppos;
  a.allp = K.dtallp;
  a.xoff = xoff;
  a.yoff = yoff;
  a.src = src;
  a.dst = dst;
  a.sortpart = sortpart;
  a.poscell = poscell;
  a.press = press;
  a.posminx = dom_posmin[0];
  a.posminy = dom_posmin[1];
  a.posminz = dom_posmin[2];
  a.scelld = K.scelld;
  a.cteb = K.cteb;
  a.ovrhopzero = K.ovrhopzero;
  a.rhopzero = K.rhopzero;
  a.gamma = K.gamma;
  a.igamma = (K.gamma == float(int(K.gamma)) && K.gamma >= 1.f && K.gamma <= 16.f) ? int(K.gamma) : 0;
  a.dcc = K.domcellcode;
  a.withm1 = withm1;
  a.withpre = withpre;
  const unsigned nb = (cap + 256 * GP - 1) / (256 * GP);
#define SPH_K_GATHER(M1, PRE, TAU) hipLaunchKernelGGL((k_gather<M1, PRE, TAU>), dim3(nb), dim3(256), 0, stm, sc, a)
#define SPH_K_GATHER_T(M1, PRE) \
  if (a.src.tau) SPH_K_GATHER(M1, PRE, true); \
  else SPH_K_GATHER(M1, PRE, false)
  if (withm1 && withpre) { SPH_K_GATHER_T(true, true); }
  else if (withm1) { SPH_K_GATHER_T(true, false); }
  else if (withpre) { SPH_K_GATHER_T(false, true); }
  else { SPH_K_GATHER_T(false, false); }
#undef SPH_K_GATHER_T
#undef SPH_K_GATHER
}

// ---------------------------------------------------------------------------------
// Incremental divide (single domain, every divide after the first).
//
// Particles move less than one cell per step (UpdatePos excludes a particle that moves
// more than MovLimit < Scell; it goes to an out box), so the previous divide's order is
// almost the new one.  The stable sort by box key is then a MERGE of two sequences that
// are both already ordered by (new key, previous index): the STAYERS (key unchanged;
// they keep their relative order) and the MOVERS (a few percent).  A mover is NEAR when
// its key moved by one of the 27 (dx,dy,dz) cell offsets, else FAR (an exclusion to an
// out box; anything else), kept in a short list.  Three kernels replace presort + the two
// radix passes + begincell, with no scan across blocks (a chained scan's look-back costs
// ~2 us per probe here: the status words cross the XCDs):
//   k_inc_classify  per tile of INC_TILE particles: new key, near/far flags and their
//                   tile-local prefixes, the tile's counts (+ one atomic into its super
//                   tile of 64), near movers' keys at tile-major slots, far movers
//                   appended to a list;
//   k_inc_boxes     per IB_BOX boxes: the mover prefixes of the tiles it reads (super +
//                   tile counts), the new begincell and every arrival's position from the
//                   window of previous keys that can reach its boxes, the stayers' offset;
//                   np / npb / npbok / nout as k_begincell;
//   k_inc_push      every particle pushed to its new position (gather_store: poscell,
//                   press, VelMax) with its key for the next divide.
// The result is the stable radix sort's, bit for bit (tests/test_divide_inc.py).
static_assert(INC_IPT == GP, "k_inc_push covers one classify tile per block");
#ifndef SPH_IB_BPT
#define SPH_IB_BPT 2
#endif
constexpr int IB_BS = 256, IB_BPT = SPH_IB_BPT, IB_BOX = IB_BS * IB_BPT;  // boxes per k_inc_boxes block
// Phase timestamps of the incremental-divide kernels (SPH_INC_DBG & 8: printed for every
// 16th block of the 12th incremental divide; the 100 MHz device clock).
#define TSDECL unsigned long long tsv[8]
#define TSTAMP(k) \
  do { \
    if (s.dbg & 8) tsv[k] = wall_clock64(); \
  } while (0)
#define TSPRINT(name, nk) \
  do { \
    if ((s.dbg & 8) && threadIdx.x == 0 && s.gen == 12 && (blockIdx.x % 16 == 0 || blockIdx.x + 1 == gridDim.x)) { \
      printf("TS %s %u %llu %llu %llu %llu %llu %llu\n", name, blockIdx.x, tsv[0], tsv[1], tsv[2], tsv[3], \
             tsv[(nk) > 4 ? 4 : 3], tsv[(nk) > 5 ? 5 : 3]); \
    } \
  } while (0)

__global__ __launch_bounds__(INC_BS) void k_inc_classify(DevScalars* __restrict__ sc, const unsigned* __restrict__ dcell,
                                                         const typecode* __restrict__ code, DivGrid g, unsigned dcc,
                                                         IncDivScratch s, int usey, int usez) {
  inc_classify_tile(sc, dcell, code, g, dcc, s, usey, usez, blockIdx.x);
}

// After an update that classified its particles (sph_incdiv.hpp), a slab's exchange appended
// s.napp migrants at [nold, np): their keys (the input of their own sort) and class, and the
// divide's particle count — the part of inc_classify_tile that concerns them.
__global__ __launch_bounds__(256) void k_inc_classify_app(DevScalars* __restrict__ sc,
                                                          const unsigned* __restrict__ dcell,
                                                          const typecode* __restrict__ code, DivGrid g, unsigned dcc,
                                                          IncDivScratch s) {
  const unsigned n = sc->np, nold = n - s.napp;
  if (blockIdx.x == 0 && threadIdx.x == 0) sc->ndiv = n;
  const unsigned e = blockIdx.x * 256 + threadIdx.x;
  if (e >= s.napp) return;
  const unsigned i = nold + e;
  const unsigned key = box_key(dcell[i], code[i], g, dcc);
  s.newkey[i] = key;
  s.cw[i] = CW_APP;
  s.akin[e] = key;
  s.avin[e] = e;
}

// One block per IB_BOX consecutive boxes [c0, c0 + IB_BOX).
// Mover prefixes: Ln(x) / Lf(x) = near / far movers before index x = the tile prefix
// (super-tile sums + the tile counts of the super tile) + the tile-local prefix of x.
// A near mover changes its key by at most omax = 1 + ncx + nsheet, so every near mover
// with a previous key below c0 - omax lands below c0 and none from c0 + IB_BOX + omax or
// above lands in the block: the block reads the near movers of that WINDOW of previous
// keys (list indices [Ln(obx(c0 - omax)), Ln(obx(c0 + IB_BOX + omax))), previous-index
// order) and
//   begin[c] = #stayers below c       = S(obx(c))
//            + #near movers below c   = Ln(obx(c0 - omax)) + #window keys < c0 + arrivals in [c0, c)
//            + #far movers below c    = #far keys < c0 + far arrivals in [c0, c)
// (S(x) = x - Ln(x) - Lf(x): stayers before index x).  Within a box the members are
// ordered by previous index: near arrivals in list order (a stable rank per box, wave
// match on the 9-bit box offset), the stayers after the near arrivals whose list index is
// at least Ln(obx(c)), far arrivals (a short list) by their previous index.  Two passes
// over the window: counts, then (after the per-box scan) ranks -> positions.
// LDS: 52 KB per block, so 3 blocks (12 waves) share a CU: the kernel is a chain of dependent
// global-memory latencies per block, and a 1M (cfg2) divide has ~700 blocks, a 1.25M y-slab
// of cfg3 ~1050.  (At 77 KB, 2 blocks per CU: the launch ran in 1.4-2 rounds of blocks.)  The
// window's near-mover keys are held as 16-bit codes relative to the block (below / box / above),
// the arrivals as packed words, and arrays whose lifetimes do not overlap share their storage.
constexpr int IB_FCAP = 128;  // far arrivals of a block held in LDS (more: read from global memory)
constexpr int IB_TPCAP = 1024;  // window tiles with LDS prefixes (more: computed from global memory)
constexpr int IB_WCAP = 4096;   // window near movers staged in LDS (more: read from global memory)
constexpr int IB_ACAP = 1024;   // near arrivals ranked through LDS buckets (more: chunked wave-match pass)
static_assert(IB_BOX <= 512 && IB_ACAP <= 2 * IB_BOX, "packed arrivals (9-bit box offset); buckets in s_nfbef");
// window code of a previous-key window entry: 0 below the block's boxes, 1 + the box offset
// inside them, WC_ABOVE above
constexpr unsigned WC_ABOVE = 0xffffu;
__global__ __launch_bounds__(IB_BS) void k_inc_boxes(DevScalars* __restrict__ sc, DivGrid g,
                                                     const unsigned* __restrict__ ob, unsigned* __restrict__ nbc,
                                                     IncDivScratch s, unsigned omax) {
  constexpr int NW = IB_BS / 64;
  __shared__ unsigned s_obx[IB_BOX + 1], s_ln[IB_BOX + 1], s_lf[IB_BOX + 1];
  __shared__ unsigned s_narr[IB_BOX], s_farr[IB_BOX], s_run[IB_BOX];
  // near / far arrivals of each box ahead of its stayers (up to the per-box scan), then the
  // buckets of pass 2
  __shared__ unsigned s_nfbef[2][IB_BOX];
  unsigned* const s_nbef = s_nfbef[0];
  unsigned* const s_fbef = s_nfbef[1];
  unsigned* const s_bkt = &s_nfbef[0][0];  // near arrivals' window indices bucketed by box
  // slab: the appended entries below each box (s_ab, up to the per-box scan); then the wave
  // counts of the unbucketed pass 2 (s_wc)
  constexpr int ABWC = NW * IB_BOX > 3 * (IB_BOX + 1) ? NW * IB_BOX : 3 * (IB_BOX + 1);
  __shared__ unsigned s_abwc[ABWC];
  unsigned(*const s_ab)[IB_BOX + 1] = reinterpret_cast<unsigned(*)[IB_BOX + 1]>(s_abwc);
  unsigned(*const s_wc)[IB_BOX] = reinterpret_cast<unsigned(*)[IB_BOX]>(s_abwc);
  __shared__ unsigned s_begin[IB_BOX];
  __shared__ uint2 s_tp[IB_TPCAP];      // (near, far) movers before tile tA + k
  __shared__ uint4 s_far[IB_FCAP];      // (f, previous index, key, Ln(previous index) clamped to the window)
  __shared__ unsigned s_fnb[IB_FCAP];   // near arrivals of its box before a far arrival
  __shared__ unsigned s_wsum[IB_BPT][NW];
  __shared__ unsigned long long s_red[2][NW];
  __shared__ unsigned s_xw[2], s_jw[2], s_below, s_farbelow, s_nfar;
  __shared__ unsigned short s_wcode[IB_WCAP];  // the window's near-mover key codes (when they fit)
  __shared__ unsigned s_arr[IB_ACAP];  // near arrivals (window index << 9 | box offset), unordered
  __shared__ unsigned s_boff[IB_BOX];   // bucket offsets (exclusive scan of s_narr)
  __shared__ unsigned s_nwsum[IB_BPT][IB_BS / 64];
  __shared__ unsigned s_nar;
  const unsigned b = blockIdx.x;
  TSDECL;
  TSTAMP(0);
  const unsigned n = sc->ndiv - s.napp;  // the previous divide's particles (all but the appended)
  const unsigned totf = s.ctr[0];
  const long nctt = long(g.nctt);
  const long c0 = long(b) * IB_BOX;
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned nsup = (s.nb1 + INC_SUP - 1) / INC_SUP;
  auto obxg = [&](long x) -> unsigned { return x <= 0 ? 0u : (x >= nctt ? n : min(ob[x], n)); };
  // ---- 1. obx of the block's box bounds and of the window ends
  unsigned xo[IB_BPT + 1];
#pragma unroll
  for (int m = 0; m <= IB_BPT; m++) {
    long c = c0 + int(threadIdx.x) + m * IB_BS;
    if (m == IB_BPT) c = threadIdx.x == 0 ? c0 + IB_BOX : (threadIdx.x == 1 ? c0 - long(omax) : c0 + IB_BOX + long(omax));
    xo[m] = obxg(c);
  }
#pragma unroll
  for (int m = 0; m < IB_BPT; m++) s_obx[int(threadIdx.x) + m * IB_BS] = xo[m];
  if (threadIdx.x == 0) s_obx[IB_BOX] = xo[IB_BPT];
  if (threadIdx.x == 1 || threadIdx.x == 2) s_xw[threadIdx.x - 1] = xo[IB_BPT];
  for (int k = int(threadIdx.x); k < IB_BOX; k += IB_BS) {
    s_narr[k] = 0;
    s_nbef[k] = 0;
    s_farr[k] = 0;
    s_fbef[k] = 0;
    s_run[k] = 0;
  }
  if (threadIdx.x == 0) {
    s_below = 0;
    s_farbelow = 0;
    s_nfar = 0;
    s_nar = 0;
  }
  __syncthreads();
  // ---- 2. the window's tiles [tA, tB]: their counts, the movers before tA, the totals;
  // the tile-local prefixes of the block's box bounds (one batch of loads)
  const unsigned xa = s_xw[0], xb = s_xw[1];
  const unsigned tA = (xa < n ? xa : (n ? n - 1 : 0u)) / INC_TILE;
  const unsigned tB = (xb < n ? xb : (n ? n - 1 : 0u)) / INC_TILE;
  const unsigned ntp = tB - tA + 1;
  const bool tplds = ntp <= unsigned(IB_TPCAP) && !(s.dbg & 16);
  unsigned cwo[IB_BPT + 1];
#pragma unroll
  for (int m = 0; m <= IB_BPT; m++) cwo[m] = s.cw[xo[m] < n ? xo[m] : 0u];
  uint2 ta[IB_TPCAP / IB_BS];
#pragma unroll
  for (int m = 0; m < IB_TPCAP / IB_BS; m++) {
    const unsigned k = threadIdx.x + m * IB_BS;
    ta[m] = (tplds && k < ntp) ? s.tagg[tA + k] : make_uint2(0u, 0u);
  }
  unsigned long long pre = 0, tot = 0;  // (near << 32 | far) before tA, and over all tiles
  for (unsigned q = threadIdx.x; q < nsup; q += IB_BS) {
    const unsigned long long v = s.tsup[q * TSUP_STRIDE];
    tot += v;
    if (q < tA / INC_SUP) pre += v;
  }
  for (unsigned t = (tA / INC_SUP) * INC_SUP + threadIdx.x; t < tA; t += IB_BS) {
    const uint2 v = s.tagg[t];
    pre += (static_cast<unsigned long long>(v.x) << 32) | v.y;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    pre += __shfl_xor(pre, off, 64);
    tot += __shfl_xor(tot, off, 64);
  }
  if (lane == 0) {
    s_red[0][w] = pre;
    s_red[1][w] = tot;
  }
  // tile counts -> LDS (exclusive scan below, by wave 0)
#pragma unroll
  for (int m = 0; m < IB_TPCAP / IB_BS; m++) s_tp[threadIdx.x + m * IB_BS] = ta[m];
  __syncthreads();
  pre = 0;
  tot = 0;
#pragma unroll
  for (int q = 0; q < NW; q++) {
    pre += s_red[0][q];
    tot += s_red[1][q];
  }
  const unsigned totn = unsigned(tot >> 32), totfc = unsigned(tot);  // far class: far list + drops
  if (w == 0 && tplds) {  // exclusive scan of the window's tile counts, 16 tiles per lane
    constexpr int PL = IB_TPCAP / 64;
    uint2 v[PL];
    unsigned sn = 0, sf = 0;
#pragma unroll
    for (int q = 0; q < PL; q++) {
      v[q] = s_tp[lane * PL + q];
      sn += v[q].x;
      sf += v[q].y;
    }
    unsigned xn = sn, xf = sf;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned yn = __shfl_up(xn, off, 64), yf = __shfl_up(xf, off, 64);
      if (lane >= unsigned(off)) {
        xn += yn;
        xf += yf;
      }
    }
    unsigned rn = unsigned(pre >> 32) + xn - sn, rf = unsigned(pre) + xf - sf;
#pragma unroll
    for (int q = 0; q < PL; q++) {
      s_tp[lane * PL + q] = make_uint2(rn, rf);
      rn += v[q].x;
      rf += v[q].y;
    }
  }
  __syncthreads();
  // movers before tile t: LDS for the window's tiles, else from the super/tile counts
  auto tp_of = [&](unsigned t) -> uint2 {
    if (tplds && t >= tA && t - tA < ntp) return s_tp[t - tA];
    unsigned long long p = 0;
    for (unsigned q = 0; q < t / INC_SUP; q++) p += s.tsup[q * TSUP_STRIDE];
    for (unsigned u = (t / INC_SUP) * INC_SUP; u < t; u++) {
      const uint2 v = s.tagg[u];
      p += (static_cast<unsigned long long>(v.x) << 32) | v.y;
    }
    return make_uint2(unsigned(p >> 32), unsigned(p));
  };
  auto lnlf = [&](unsigned x, unsigned cw) -> uint2 {  // (Ln(x), Lf(x))
    if (x >= n) return make_uint2(totn, totfc);
    const uint2 p = tp_of(x / INC_TILE);
    return make_uint2(p.x + (cw & CW_LOC), p.y + ((cw >> 11) & CW_LOC));
  };
  // the tile holding near mover j of the window (largest t with Ln(t * INC_TILE) <= j)
  auto slot_of = [&](unsigned j) -> unsigned {
    unsigned lo = tA, hi = tB;
    while (lo < hi) {
      const unsigned mid = (lo + hi + 1) >> 1;
      if (tp_of(mid).x <= j) lo = mid;
      else hi = mid - 1;
    }
    return lo * INC_TILE + (j - tp_of(lo).x);
  };
#pragma unroll
  for (int m = 0; m < IB_BPT; m++) {
    const uint2 l = lnlf(xo[m], cwo[m]);
    s_ln[int(threadIdx.x) + m * IB_BS] = l.x;
    s_lf[int(threadIdx.x) + m * IB_BS] = l.y;
  }
  {
    const uint2 l = lnlf(xo[IB_BPT], cwo[IB_BPT]);
    if (threadIdx.x == 0) {
      s_ln[IB_BOX] = l.x;
      s_lf[IB_BOX] = l.y;
    }
    if (threadIdx.x == 1 || threadIdx.x == 2) s_jw[threadIdx.x - 1] = l.x;
  }
  // movers before each tile that starts in this block's index range, for k_inc_push
  for (unsigned t = tA + threadIdx.x; t <= tB; t += IB_BS) {
    const unsigned x = t * INC_TILE;
    if (x >= s_obx[0] && x < s_obx[IB_BOX] && x < n) {
      const uint2 p = tp_of(t);
      s.tpg[t] = p.x + p.y;
    }
  }
  __syncthreads();
  TSTAMP(1);
  const unsigned jlo = s_jw[0], jhi = s_jw[1];
  const unsigned cend = unsigned(min(c0 + IB_BOX, nctt));
  auto wcode_of = [&](unsigned key) -> unsigned {
    return key < unsigned(c0) ? 0u : (key < cend ? key - unsigned(c0) + 1u : WC_ABOVE);
  };
  auto ln_clamped = [&](unsigned x) -> unsigned {  // Ln(x) of a far mover, clamped to the window
    if (x < xa) return jlo;
    if (x >= xb) return jhi;
    return lnlf(x, s.cw[x]).x;
  };
  // ---- far movers (a short list; usually empty): below the block, or arrivals
  for (unsigned f = threadIdx.x; f < totf; f += IB_BS) {
    const uint2 e = s.mfar[f];
    if (e.y < unsigned(c0)) {
      atomicAdd(&s_farbelow, 1u);
    } else if (e.y < cend) {
      const unsigned lc = e.y - unsigned(c0);
      atomicAdd(&s_farr[lc], 1u);
      if (e.x < s_obx[lc]) atomicAdd(&s_fbef[lc], 1u);
      const unsigned k = atomicAdd(&s_nfar, 1u);
      if (k < unsigned(IB_FCAP)) {
        s_far[k] = make_uint4(f, e.x, e.y, ln_clamped(e.x));
        s_fnb[k] = 0;
      }
    }
  }
  __syncthreads();
  const unsigned nfar = s_nfar;
  const bool farlds = nfar <= unsigned(IB_FCAP) && !(s.dbg & 32);
  // the window's keys into LDS: all loads of a round issued before the stores (one latency)
  const bool wlds = jhi - jlo <= unsigned(IB_WCAP) && !(s.dbg & 16);
  if (wlds) {
    constexpr int WR = 8;
    for (unsigned r0 = 0; r0 < jhi - jlo; r0 += WR * IB_BS) {
      unsigned kk[WR];
#pragma unroll
      for (int m = 0; m < WR; m++) {
        const unsigned e = r0 + threadIdx.x + m * IB_BS;
        kk[m] = e < jhi - jlo ? s.mkey[slot_of(jlo + e)] : 0u;
      }
#pragma unroll
      for (int m = 0; m < WR; m++) {
        const unsigned e = r0 + threadIdx.x + m * IB_BS;
        if (e < jhi - jlo) s_wcode[e] = (unsigned short)wcode_of(kk[m]);
      }
    }
    __syncthreads();
  }
  auto wcode = [&](unsigned j) -> unsigned { return wlds ? s_wcode[j - jlo] : wcode_of(s.mkey[slot_of(j)]); };
  // ---- pass 1: near arrivals per box, and the window's near movers below the block
  {
    unsigned below = 0;
    for (unsigned base = jlo; base < jhi; base += IB_BS) {
      const unsigned j = base + threadIdx.x;
      const unsigned wc = j < jhi ? wcode(j) : WC_ABOVE;
      below += unsigned(__popcll(__ballot(wc == 0u)));
      if (wc != 0u && wc != WC_ABOVE) {
        const unsigned lc = wc - 1u, key = unsigned(c0) + lc;
        atomicAdd(&s_narr[lc], 1u);
        if (j < s_ln[lc]) atomicAdd(&s_nbef[lc], 1u);
        const unsigned a = atomicAdd(&s_nar, 1u);
        if (a < unsigned(IB_ACAP)) s_arr[a] = ((j - jlo) << 9) | lc;
        if (s_farr[lc] && farlds) {  // near arrivals ahead of a far arrival of the same box
          for (unsigned k = 0; k < nfar; k++) {
            const uint4 fe = s_far[k];
            if (fe.z == key && j < fe.w) atomicAdd(&s_fnb[k], 1u);
          }
        }
      }
    }
    if (lane == 0 && below) atomicAdd(&s_below, below);
  }
  __syncthreads();
  TSTAMP(2);
  // ---- slab: the appended particles (sorted by key) below each box of the block; they
  // follow the old members of their box (larger previous index), in appended order
  // Appended entries, three lists sorted by key: the migrants (sorted apart), the left and
  // the right face's reserved ghost slots (generated in key order).  A box holds entries of
  // one list at most (migrants land in owned columns, ghosts in ghost columns).
  const unsigned napt = s.napp + s.nvl + s.nvr;
  if (napt) {
    // migrants: the block's range of their sorted keys (two searches of a short list), then
    // every box's bound inside it; ghost slots: the prefix of the face-box counts at the
    // first face box at or after the box (O(1))
    if (threadIdx.x < 2)
      s_ab[0][threadIdx.x ? IB_BOX : 0] =
          lower_bound_u32(s.akeys, 0u, s.napp, unsigned(min(c0 + (threadIdx.x ? IB_BOX : 0), nctt)));
    __syncthreads();
    const unsigned a0 = s_ab[0][0], a1 = s_ab[0][IB_BOX];
    for (int k = int(threadIdx.x); k <= IB_BOX; k += IB_BS) {
      const unsigned key = unsigned(min(c0 + k, nctt));
      if (k > 0 && k < IB_BOX) s_ab[0][k] = a0 == a1 ? a0 : lower_bound_u32(s.akeys, a0, a1, key);
      s_ab[1][k] = s.nvl ? s.vpre[0][face_lower(g, s.vW, key, 0)] : 0u;
      s_ab[2][k] = s.nvr ? s.vpre[1][face_lower(g, s.vW, key, g.sown1)] : 0u;
    }
    __syncthreads();
  }
  auto ab = [&](int k) -> unsigned { return napt ? s_ab[0][k] + s_ab[1][k] + s_ab[2][k] : 0u; };
  // ---- per-box scan: begin, stayer offset, counts
  const unsigned base0 = jlo + s_below + s_farbelow;
  unsigned cnt[IB_BPT], xs[IB_BPT], xsn[IB_BPT];
#pragma unroll
  for (int h = 0; h < IB_BPT; h++) {
    const int k = h * IB_BS + int(threadIdx.x);
    cnt[h] = s_narr[k] + s_farr[k];
    unsigned x = cnt[h], xn = s_narr[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned y = __shfl_up(x, off, 64), yn = __shfl_up(xn, off, 64);
      if (lane >= unsigned(off)) {
        x += y;
        xn += yn;
      }
    }
    xs[h] = x;
    xsn[h] = xn;
    if (lane == 63) {
      s_wsum[h][w] = x;
      s_nwsum[h][w] = xn;
    }
  }
  __syncthreads();
  unsigned hpre = 0, hpren = 0;
#pragma unroll
  for (int h = 0; h < IB_BPT; h++) {
    unsigned wpre = 0, hsum = 0, wpren = 0, hsumn = 0;
#pragma unroll
    for (int q = 0; q < NW; q++) {
      wpre += unsigned(q) < w ? s_wsum[h][q] : 0u;
      hsum += s_wsum[h][q];
      wpren += unsigned(q) < w ? s_nwsum[h][q] : 0u;
      hsumn += s_nwsum[h][q];
    }
    const int k = h * IB_BS + int(threadIdx.x);
    s_boff[k] = hpren + wpren + xsn[h] - s_narr[k];
    s_run[k] = 0;  // bucket fill counters
    hpren += hsumn;
    const unsigned S = s_obx[k] - s_ln[k] - s_lf[k];
    const unsigned stay = (s_obx[k + 1] - s_obx[k]) - (s_ln[k + 1] - s_ln[k]) - (s_lf[k + 1] - s_lf[k]);
    const unsigned begin = S + base0 + hpre + wpre + xs[h] - cnt[h] + ab(k);
    hpre += hsum;
    s_begin[k] = begin;
    const long c = c0 + k;
    if (c >= nctt) continue;
    const unsigned cu = unsigned(c);
    nbc[cu] = begin;
    s.stayoff[cu] = begin + s_nbef[k] + s_fbef[k] - S;
    const unsigned total = cnt[h] + stay + (ab(k + 1) - ab(k));
    if (napt) {  // the box's appended entries after its old members
      unsigned pos = begin + cnt[h] + stay;
      for (unsigned e = s_ab[0][k]; e < s_ab[0][k + 1]; e++) s.apppos[s.avals[e]] = pos++;
      for (unsigned j = s_ab[1][k]; j < s_ab[1][k + 1]; j++) s.apppos[s.napp + j] = pos++;
      for (unsigned j = s_ab[2][k]; j < s_ab[2][k + 1]; j++) s.apppos[s.napp + s.nvl + j] = pos++;
    }
    // JCellDivCpuSingle::Divide counts + RunCellDivide, as k_begincell
    if (cu == g.boxboundignore) sc->npbok = begin;
    if (cu == g.boxfluid) sc->npb = begin;
    if (cu == g.boxboundout) {
      sc->np = begin;
      if (total) {
        sc->npbout = total;
        sc->error_flags |= ERR_BOUNDOUT;
      }
    }
    if (cu == g.boxfluidout) sc->nout += total;
  }
  __syncthreads();
  TSTAMP(3);
  // ---- pass 2: stable rank of every near arrival in its box -> its new position.
  // Usually through LDS buckets (arrivals of one box, any order; rank = arrivals of the box
  // with a smaller list index), else one wave-matched chunk of the window at a time.
  const unsigned nar = s_nar;
  const bool bucketed = nar <= unsigned(IB_ACAP) && jhi - jlo < (1u << 23) && !(s.dbg & 64);
  auto near_pos = [&](unsigned j, unsigned lc, unsigned r) -> unsigned {
    const unsigned key = unsigned(c0) + lc;
    if (s_farr[lc]) {  // far arrivals of this box ahead of it (previous index below this mover's)
      if (farlds) {
        for (unsigned k = 0; k < nfar; k++)
          if (s_far[k].z == key && s_far[k].w <= j) r++;
      } else {
        for (unsigned f = 0; f < totf; f++) {
          const uint2 e = s.mfar[f];
          if (e.y == key && ln_clamped(e.x) <= j) r++;
        }
      }
    }
    const unsigned stay = (s_obx[lc + 1] - s_obx[lc]) - (s_ln[lc + 1] - s_ln[lc]) - (s_lf[lc + 1] - s_lf[lc]);
    return s_begin[lc] + r + (j >= s_ln[lc] ? stay : 0u);
  };
  if (bucketed) {
    for (unsigned a = threadIdx.x; a < nar; a += IB_BS) {
      const unsigned e = s_arr[a], lc = e & 511u;
      s_bkt[s_boff[lc] + atomicAdd(&s_run[lc], 1u)] = e >> 9;
    }
    __syncthreads();
    for (unsigned a = threadIdx.x; a < nar; a += IB_BS) {
      const unsigned e = s_arr[a], lc = e & 511u, jr = e >> 9;
      const unsigned b0 = s_boff[lc], b1 = b0 + s_narr[lc];
      unsigned r = 0;
      for (unsigned q = b0; q < b1; q++) r += s_bkt[q] < jr ? 1u : 0u;
      s.mposnear[slot_of(jlo + jr)] = near_pos(jlo + jr, lc, r);
    }
  } else {  // the wave counts (storage of the slab's s_ab, dead since the per-box scan)
    for (int k = int(threadIdx.x); k < NW * IB_BOX; k += IB_BS) s_abwc[k] = 0u;
    __syncthreads();
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (unsigned base = jlo; base < (bucketed ? jlo : jhi); base += IB_BS) {
    const unsigned j = base + threadIdx.x;
    const unsigned wc = j < jhi ? wcode(j) : WC_ABOVE;
    const bool valid = wc != 0u && wc != WC_ABOVE;
    if (__syncthreads_or(valid) == 0) continue;  // block-uniform
    const unsigned lc = valid ? wc - 1u : 0u;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 9; bit++) {
      const bool on = (lc >> bit) & 1u;
      const unsigned long long bb = __ballot(on);
      peers &= on ? bb : ~bb;
    }
    const unsigned rank = unsigned(__popcll(peers & lt)), pc = unsigned(__popcll(peers));
    const bool leader = valid && (peers & lt) == 0ull;
    if (leader) s_wc[w][lc] = pc;
    __syncthreads();
    if (valid) {
      unsigned r = s_run[lc] + rank;
      for (unsigned q = 0; q < w; q++) r += s_wc[q][lc];
      s.mposnear[slot_of(j)] = near_pos(j, lc, r);
    }
    __syncthreads();
    if (leader) {
      atomicAdd(&s_run[lc], pc);
      s_wc[w][lc] = 0;
    }
  }
  // ---- far arrivals: near arrivals before them + far arrivals before them + stayers
  for (unsigned k = threadIdx.x; k < nfar; k += IB_BS) {
    uint4 fe;
    unsigned nb = 0;
    if (farlds) {
      fe = s_far[k];
      nb = s_fnb[k];
    } else {  // the k-th far arrival of the block in list order, counted from global memory
      unsigned seen = 0, f = 0;
      for (; f < totf; f++) {
        const uint2 e = s.mfar[f];
        if (e.y >= unsigned(c0) && e.y < cend && seen++ == k) break;
      }
      const uint2 e = s.mfar[f];
      fe = make_uint4(f, e.x, e.y, ln_clamped(e.x));
      for (unsigned j = jlo; j < fe.w; j++) nb += (wcode(j) == fe.z - unsigned(c0) + 1u) ? 1u : 0u;
    }
    const unsigned lc = fe.z - unsigned(c0);
    unsigned r = nb;
    for (unsigned f = 0; f < totf; f++) {
      const uint2 e = s.mfar[f];
      if (e.y == fe.z && e.x < fe.y) r++;
    }
    const unsigned stay = (s_obx[lc + 1] - s_obx[lc]) - (s_ln[lc + 1] - s_ln[lc]) - (s_lf[lc + 1] - s_lf[lc]);
    s.mposfar[fe.x] = s_begin[lc] + r + (fe.y >= s_obx[lc] ? stay : 0u);
  }
  TSTAMP(4);
  TSTAMP(5);
  TSPRINT("boxes", 6);
}

// One tile per block.  Loads in three batches (one memory latency each): the particle
// states and the classification words, the new positions, then the stores.  Block 0
// also clears the super-tile sums and the far count for the next divide.
// With an item build (ib.nblocks > 0) the launch has ib.nblocks more blocks BEFORE the tiles
// (dispatched first, so their latency-bound row walks start with the push instead of
// trailing it): they run the item COUNT pass (sph_items.hpp) on the new begincell beside
// the HBM-bound push, and the place pass follows the launch (launch_items_place).  cfg2 1M
// divide phase: see DESIGN.md §4.
template <bool WITHM1, bool WITHPRE, bool WITHTAU>
__global__ __launch_bounds__(256) void k_inc_push(DevScalars* __restrict__ sc, GatherArgs a, IncDivScratch s,
                                                  ItemBuild ib) {
  if (blockIdx.x < ib.nblocks) {
    extern __shared__ unsigned char push_items_smem[];
    items_count_block(ib, blockIdx.x, push_items_smem);
    return;
  }
  const unsigned nd = sc->ndiv, n = sc->np, npb = sc->npb, nold = nd - s.napp;
  const unsigned t = blockIdx.x - ib.nblocks;
  const unsigned i0 = t * INC_TILE + threadIdx.x;
  GatherRec<WITHM1, WITHPRE, WITHTAU> q[GP];
  unsigned key[GP], cw[GP], fx[GP], pos[GP];
  const unsigned tpg = i0 < nd ? s.tpg[t] : 0u;
#pragma unroll
  for (int k = 0; k < GP; k++) {
    const unsigned i = i0 + 256 * k;
    const unsigned ii = i < nd ? i : 0u;
    key[k] = s.newkey[ii];
    // a tail lane (i >= nd) gets a zero classification word: it is neither a near nor a far
    // mover, so it never indexes fidx / mposfar with particle 0's word
    cw[k] = i < nd ? s.cw[ii] : 0u;
    q[k].load(a.src, ii);
  }
#pragma unroll
  for (int k = 0; k < GP; k++) {
    const bool far = (cw[k] & CW_FAR) != 0, app = (cw[k] & CW_APP) != 0;
    fx[k] = far ? s.fidx[i0 + 256 * k] : (app ? s.apppos[i0 + 256 * k - nold] : 0u);
  }
#pragma unroll
  for (int k = 0; k < GP; k++) {
    const bool near = (cw[k] & CW_NEAR) != 0, far = (cw[k] & CW_FAR) != 0;
    const unsigned ln = cw[k] & CW_LOC, lf = (cw[k] >> 11) & CW_LOC;
    const unsigned* tab = near ? s.mposnear : (far ? s.mposfar : s.stayoff);
    const unsigned x = tab[near ? t * INC_TILE + ln : (far ? fx[k] : key[k])];
    pos[k] = (near || far) ? x : x + (i0 + 256 * k) - tpg - ln - lf;
    if (cw[k] & CW_APP) pos[k] = fx[k];
    if (cw[k] & CW_DROP) pos[k] = ~0u;
  }
  float v2 = 0.f;
#pragma unroll
  for (int k = 0; k < GP; k++) {
    // particles of the out boxes leave the arrays, as in the pull gather
    if (i0 + 256 * k < nd && pos[k] < n) {
      gather_store<WITHM1, WITHPRE, WITHTAU>(a, pos[k], q[k]);
      s.skeys[pos[k]] = key[k];
      if (pos[k] >= npb || a.allp)
        v2 = nanmax(v2, q[k].vr.x * q[k].vr.x + q[k].vr.y * q[k].vr.y + q[k].vr.z * q[k].vr.z);
    }
  }
  wave_max_atomic(sc, RED_VELMAX2, v2);
  if (t == 0) {
    const unsigned nsup = (s.nb1 + INC_SUP - 1) / INC_SUP;
    for (unsigned u = threadIdx.x; u < nsup; u += 256) s.tsup[u * TSUP_STRIDE] = 0ull;
    if (threadIdx.x == 0) s.ctr[0] = 0u;
  }
}

// A short list (the migrants of an exchange) sorted stably by key in one block: bitonic
// sort of (key << 32 | index) in LDS (the indices are distinct, so the order is stable).
__global__ __launch_bounds__(1024) void k_small_sort(const unsigned* __restrict__ kin, const unsigned* __restrict__ vin,
                                                     unsigned n, unsigned* __restrict__ kout,
                                                     unsigned* __restrict__ vout) {
  __shared__ unsigned long long v[SMALLSORT_MAX];
  for (unsigned i = threadIdx.x; i < SMALLSORT_MAX; i += 1024)
    v[i] = i < n ? ((static_cast<unsigned long long>(kin[i]) << 32) | vin[i]) : ~0ull;
  __syncthreads();
  for (unsigned k = 2; k <= SMALLSORT_MAX; k <<= 1) {
    for (unsigned j = k >> 1; j > 0; j >>= 1) {
      for (unsigned i = threadIdx.x; i < SMALLSORT_MAX; i += 1024) {
        const unsigned l = i ^ j;
        if (l > i) {
          const unsigned long long a = v[i], b = v[l];
          if (((i & k) == 0) == (a > b)) {
            v[i] = b;
            v[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (unsigned i = threadIdx.x; i < n; i += 1024) {
    kout[i] = unsigned(v[i] >> 32);
    vout[i] = unsigned(v[i]);
  }
}

void launch_small_sort(hipStream_t stm, const unsigned* kin, const unsigned* vin, unsigned n, unsigned* kout,
                       unsigned* vout) {
  if (n) hipLaunchKernelGGL(k_small_sort, dim3(1), dim3(1024), 0, stm, kin, vin, n, kout, vout);
}

void launch_divide_inc(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& src, const PartArrays& dst,
                       bool withm1, bool withpre, const KConst& K, const double dom_posmin[3], float4* poscell,
                       float* press, DivGrid g, const unsigned* begincell_old, unsigned* begincell_new,
                       IncDivScratch& s, SortScratch& srt, unsigned keybits, const float4* phase_eos,
                       const SlabFaces* faces, unsigned ngl, unsigned ngr, const ItemBuild* items, bool classified) {
  s.gen++;
  const int usey = g.ncy > 1, usez = g.ncz > 1;
  const unsigned omax = 1u + (usey ? unsigned(g.ncx) : 0u) + (usez ? g.nsheet : 0u);
  s.akin = srt.keys[0];
  s.avin = srt.vals[0];
  s.nvl = faces ? ngl : 0u;
  s.nvr = faces ? ngr : 0u;
  // (classified: the update kernel classified its own tiles, sph_incdiv.hpp; the particles a
  // slab's exchange appended since are classified here)
  if (!classified)
    hipLaunchKernelGGL(k_inc_classify, dim3(s.nb1), dim3(INC_BS), 0, stm, sc, src.dcell, src.code, g, K.domcellcode,
                       s, usey, usez);
  else if (s.napp)
    hipLaunchKernelGGL(k_inc_classify_app, dim3((s.napp + 255) / 256), dim3(256), 0, stm, sc, src.dcell, src.code, g,
                       K.domcellcode, s);
  // slab: the reserved ghost slots are counted per face box (faces->pre: the received
  // counts' prefixes); k_inc_boxes reads their bounds from the prefixes, no keys needed
  if (faces) {
    s.vpre[0] = faces->pre[2];
    s.vpre[1] = faces->pre[3];
    s.vW = faces->W;
  }
  if (s.napp) {  // slab: the appended migrants, sorted by key apart (stable: appended order)
    if (s.napp <= SMALLSORT_MAX) {
      launch_small_sort(stm, srt.keys[0], srt.vals[0], s.napp, srt.keys[1], srt.vals[1]);
      s.akeys = srt.keys[1];
      s.avals = srt.vals[1];
    } else {
      const int res = launch_radix_sort(stm, cap, sc, srt, keybits, s.napp);
      s.akeys = srt.keys[res];
      s.avals = srt.vals[res];
    }
  }
  hipLaunchKernelGGL(k_inc_boxes, dim3(s.nb2), dim3(IB_BS), 0, stm, sc, g, begincell_old, begincell_new, s, omax);
  GatherArgs a;
  a.phase_eos = phase_eos;
  a.vfirst = ~0u;
  a.appbase = 0;
  a.apppos = nullptr;
  a.allp = K.dtallp;
  a.xoff = g.offx();
  a.yoff = g.offy();
  a.src = src;
  a.dst = dst;
  a.sortpart = nullptr;
  a.poscell = poscell;
  a.press = press;
  a.posminx = dom_posmin[0];
  a.posminy = dom_posmin[1];
  a.posminz = dom_posmin[2];
  a.scelld = K.scelld;
  a.cteb = K.cteb;
  a.ovrhopzero = K.ovrhopzero;
  a.rhopzero = K.rhopzero;
  a.gamma = K.gamma;
  a.igamma = (K.gamma == float(int(K.gamma)) && K.gamma >= 1.f && K.gamma <= 16.f) ? int(K.gamma) : 0;
  a.dcc = K.domcellcode;
  a.withm1 = withm1;
  a.withpre = withpre;
  // one tile per block, then the item count blocks (if any)
  ItemBuild ib;
  std::memset(&ib, 0, sizeof(ib));
  if (items) ib = *items;
  const unsigned nb = s.nb1 + (items ? ib.nblocks : 0u);
  const unsigned lds = items ? ib.lds : 0u;
#define SPH_K_INC_PUSH(M1, PRE, TAU) \
  hipLaunchKernelGGL((k_inc_push<M1, PRE, TAU>), dim3(nb), dim3(256), lds, stm, sc, a, s, ib)
#define SPH_K_INC_PUSH_T(M1, PRE) \
  if (a.src.tau) SPH_K_INC_PUSH(M1, PRE, true); \
  else SPH_K_INC_PUSH(M1, PRE, false)
  if (withm1 && withpre) { SPH_K_INC_PUSH_T(true, true); }
  else if (withm1) { SPH_K_INC_PUSH_T(true, false); }
  else if (withpre) { SPH_K_INC_PUSH_T(false, true); }
  else { SPH_K_INC_PUSH_T(false, false); }
#undef SPH_K_INC_PUSH_T
#undef SPH_K_INC_PUSH
  if (items) launch_items_place(stm, ib);
}

// ---------------------------------------------------------------------------------
// Slab ghosts into their reserved slots (the exchange after the divide, sph_slab.hip): the
// double position rebuilt as cell origin + offset and stored with its poscell and EOS
// pressure exactly as the gather stores a particle (gather_store); the key for the next
// divide (which drops the ghost: the update marks it DCELL_DISCARD).
__global__ __launch_bounds__(256) void k_ghost_scatter(const SlabGhost* __restrict__ rec, unsigned ng,
                                                       const unsigned* __restrict__ apppos, GatherArgs a, DivGrid g,
                                                       unsigned* __restrict__ skeys) {
  const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ng) return;
  const SlabGhost r = rec[e];
  const unsigned slot = apppos[e];
  GatherRec<false, false, false> q;
  const double ox = a.posminx + double(DcelCellx(a.dcc, r.dcell)) * a.scelld;
  const double oy = a.posminy + double(DcelCelly(a.dcc, r.dcell)) * a.scelld;
  const double oz = a.posminz + double(DcelCellz(a.dcc, r.dcell)) * a.scelld;
  q.dc = r.dcell;
  q.idp = r.idp;
  q.code = r.code;
  q.pxy = make_double2(ox + double(r.rx), oy + double(r.ry));
  q.pz = oz + double(r.rz);
  q.vr = r.velrhop;
  gather_store<false, false, false>(a, slot, q);
  if (skeys) skeys[slot] = box_key(r.dcell, r.code, g, a.dcc);
}

void launch_ghost_scatter(hipStream_t stm, DevScalars* sc, const SlabGhost* rec, unsigned ng, const unsigned* apppos,
                          const PartArrays& dst, const KConst& K, const double dom_posmin[3], float4* poscell,
                          float* press, DivGrid g, unsigned* skeys, const float4* phase_eos) {
  (void)sc;
  if (!ng) return;
  GatherArgs a;
  a.phase_eos = phase_eos;
  a.vfirst = ~0u;
  a.appbase = 0;
  a.apppos = nullptr;
  a.allp = K.dtallp;
  a.xoff = g.offx();
  a.yoff = g.offy();
  a.src = dst;
  a.dst = dst;
  a.sortpart = nullptr;
  a.poscell = poscell;
  a.press = press;
  a.posminx = dom_posmin[0];
  a.posminy = dom_posmin[1];
  a.posminz = dom_posmin[2];
  a.scelld = K.scelld;
  a.cteb = K.cteb;
  a.ovrhopzero = K.ovrhopzero;
  a.rhopzero = K.rhopzero;
  a.gamma = K.gamma;
  a.igamma = (K.gamma == float(int(K.gamma)) && K.gamma >= 1.f && K.gamma <= 16.f) ? int(K.gamma) : 0;
  a.dcc = K.domcellcode;
  a.withm1 = 0;
  a.withpre = 0;
  hipLaunchKernelGGL(k_ghost_scatter, dim3((ng + 255) / 256), dim3(256), 0, stm, rec, ng, apppos, a, g, skeys);
}

unsigned inc_blocks_classify(unsigned cap) { return (cap + INC_TILE - 1) / INC_TILE; }
unsigned inc_blocks_boxes(unsigned nctt) { return (nctt + IB_BOX - 1) / IB_BOX; }

}  // namespace sphx
