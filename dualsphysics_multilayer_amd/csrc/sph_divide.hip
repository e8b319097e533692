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
#include "sph_kernels.hpp"

namespace sphx {

// ---------------------------------------------------------------------------------
// PreSort (KerPreSortFull) — one thread per particle, bounded by the live count.
__global__ __launch_bounds__(256) void k_presort(const DevScalars* __restrict__ sc, const unsigned* __restrict__ dcell,
                                                 const typecode* __restrict__ code, DivGrid g, unsigned dcc,
                                                 unsigned* __restrict__ keys, unsigned* __restrict__ vals) {
  const unsigned n = sc->np;
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) const_cast<DevScalars*>(sc)->ndiv = n;
  if (p >= n) return;
  const unsigned rcell = dcell[p];
  vals[p] = p;
  if (rcell == DCELL_DISCARD) {  // slab: stale ghost / particle handed to a neighbour
    keys[p] = g.boxdiscard;
    return;
  }
  const unsigned cx = DcelCellx(dcc, rcell) - unsigned(g.xoff), cy = DcelCelly(dcc, rcell), cz = DcelCellz(dcc, rcell);
  if (rcell != DCELL_OUT && (g.xown0 != 0 || g.xown1 != g.ncx) && cx >= unsigned(g.ncx)) {
    keys[p] = g.boxdiscard;  // slab: a migrant handed over beyond this slab's ghost columns (re-partition)
    return;
  }
  const unsigned cellsort = cx + cy * unsigned(g.ncx) + cz * g.nsheet;
  const typecode rcode = code[p];
  const typecode codetype = CodeType(rcode), codeout = CodeSpecial(rcode);
  unsigned box;
  if (codetype < CODE_TYPE_FLOATING) {
    box = (codeout < CODE_OUTIGNORE
               ? ((cx < unsigned(g.ncx) && cy < unsigned(g.ncy) && cz < unsigned(g.ncz)) ? cellsort : g.boxboundignore)
               : (codeout == CODE_OUTIGNORE ? g.boxboundoutignore : g.boxboundout));
  } else {
    box = (codeout <= CODE_OUTIGNORE ? (codeout < CODE_OUTIGNORE ? g.boxfluid + cellsort : g.boxfluidoutignore)
                                     : (codetype == CODE_TYPE_FLOATING ? g.boxboundout : g.boxfluidout));
  }
  keys[p] = box;
}

void launch_presort(hipStream_t stm, unsigned cap, const DevScalars* sc, const unsigned* dcell, const typecode* code,
                    DivGrid g, unsigned domcellcode, unsigned* keys, unsigned* vals) {
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_presort, dim3(nb), dim3(256), 0, stm, sc, dcell, code, g, domcellcode, keys, vals);
}

// ---------------------------------------------------------------------------------
// Stable LSD radix sort.  Per pass: tile histograms (tile-major) -> per-digit scans over
// the tiles (digit totals) -> stable scatter (digit totals scanned in each block's
// prologue; wave match via ballots + tagged LDS wave counts).
__global__ __launch_bounds__(RS_BS) void k_rs_hist(const DevScalars* __restrict__ sc, const unsigned* __restrict__ keys,
                                                   unsigned shift, unsigned rbits, unsigned ntiles,
                                                   unsigned* __restrict__ hist) {
  __shared__ unsigned cnt[1 << RS_MAXBITS];
  const unsigned radix = 1u << rbits, mask = radix - 1;
  for (unsigned d = threadIdx.x; d < radix; d += RS_BS) cnt[d] = 0;
  __syncthreads();
  const unsigned n = sc->ndiv;
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
                                                      const unsigned* __restrict__ digtot) {
  constexpr int NW = RS_BS / 64;
  __shared__ unsigned s_off[1 << RS_MAXBITS];
  __shared__ unsigned s_wc[NW][1 << RS_MAXBITS];
  __shared__ unsigned s_part[RS_BS];
  const unsigned radix = 1u << rbits, mask = radix - 1;
  const unsigned n = sc->ndiv;
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

int launch_radix_sort(hipStream_t stm, unsigned cap, const DevScalars* sc, SortScratch& s, unsigned keybits) {
  const unsigned passes = (keybits + RS_MAXBITS - 1) / RS_MAXBITS;
  const unsigned rbits = (keybits + passes - 1) / passes;
  const unsigned ntiles = (cap + RS_TILE - 1) / RS_TILE;
  int cur = 0;
  for (unsigned p = 0; p < passes; p++) {
    const unsigned shift = p * rbits;
    const unsigned radix = 1u << rbits;
    hipLaunchKernelGGL(k_rs_hist, dim3(ntiles), dim3(RS_BS), 0, stm, sc, s.keys[cur], shift, rbits, ntiles, s.hist);
    hipLaunchKernelGGL(k_rs_scan_tiles, dim3((radix + SCAN_D - 1) / SCAN_D), dim3(256), 0, stm, s.hist, ntiles, radix, s.digtot);
    hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(RS_BS), 0, stm, sc, s.keys[cur], s.vals[cur],
                       s.keys[cur ^ 1], s.vals[cur ^ 1], shift, rbits, ntiles, s.hist, s.digtot);
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
  int xoff;
  // NN multiphase: per-phase EOS {rho0, cteb, gamma, integer gamma or 0} (nullptr: single phase)
  const float4* phase_eos;
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

template <bool WITHM1, bool WITHPRE>
__device__ __forceinline__ void gather_one(const GatherArgs& a, unsigned i, unsigned s, float4& vr_out, bool& fluid,
                                           unsigned npb) {
  const unsigned dc = a.src.dcell[s];
  const double2 pxy = a.src.posxy[s];
  const double pz = a.src.posz[s];
  const float4 vr = a.src.velrhop[s];
  const unsigned idp = a.src.idp[s];
  const typecode code = a.src.code[s];
  float4 m1, vpre;
  double2 pxypre;
  double pzpre;
  if (WITHM1) m1 = a.src.velrhopm1[s];
  if (WITHPRE) {
    pxypre = a.src.posxypre[s];
    pzpre = a.src.poszpre[s];
    vpre = a.src.velrhoppre[s];
  }
  a.dst.idp[i] = idp;
  a.dst.code[i] = code;
  a.dst.dcell[i] = dc;
  a.dst.posxy[i] = pxy;
  a.dst.posz[i] = pz;
  a.dst.velrhop[i] = vr;
  if (WITHM1) a.dst.velrhopm1[i] = m1;
  if (WITHPRE) {
    a.dst.posxypre[i] = pxypre;
    a.dst.poszpre[i] = pzpre;
    a.dst.velrhoppre[i] = vpre;
  }
  // PosCell (KerUpdatePosCell): position relative to the origin of its divide cell
  // (global cell -> the same floats on every slab); w = the local cell.
  const unsigned cx = DcelCellx(a.dcc, dc), cy = DcelCelly(a.dcc, dc), cz = DcelCellz(a.dcc, dc);
  const double ox = a.posminx + double(cx) * a.scelld;
  const double oy = a.posminy + double(cy) * a.scelld;
  const double oz = a.posminz + double(cz) * a.scelld;
  const unsigned ldc = a.xoff ? DcelCell(a.dcc, cx - unsigned(a.xoff), cy, cz) : dc;
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
  vr_out = vr;
  fluid = i >= npb;
}

template <bool WITHM1, bool WITHPRE>
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
    if (i < n) {
      float4 vr;
      bool fluid;
      gather_one<WITHM1, WITHPRE>(a, i, sp[k], vr, fluid, npb);
      if (fluid) v2 = fmaxf(v2, vr.x * vr.x + vr.y * vr.y + vr.z * vr.z);  // CalcVelMaxOmp over fluid
    }
  }
  wave_max_atomic(sc, RED_VELMAX2, v2);
}

void launch_gather(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* sortpart, const PartArrays& src,
                   const PartArrays& dst, bool withm1, bool withpre, const KConst& K, const double dom_posmin[3],
                   float4* poscell, float* press, int xoff, const float4* phase_eos) {
  GatherArgs a;
  a.phase_eos = phase_eos;
  a.xoff = xoff;
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
  if (withm1 && withpre) hipLaunchKernelGGL((k_gather<true, true>), dim3(nb), dim3(256), 0, stm, sc, a);
  else if (withm1) hipLaunchKernelGGL((k_gather<true, false>), dim3(nb), dim3(256), 0, stm, sc, a);
  else if (withpre) hipLaunchKernelGGL((k_gather<false, true>), dim3(nb), dim3(256), 0, stm, sc, a);
  else hipLaunchKernelGGL((k_gather<false, false>), dim3(nb), dim3(256), 0, stm, sc, a);
}

}  // namespace sphx
