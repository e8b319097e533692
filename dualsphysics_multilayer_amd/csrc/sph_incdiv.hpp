// sph_incdiv.hpp — the classification pass of the incremental divide (sph_divide.hip), as a
// block-level device function: k_inc_classify runs it over the particles after the update,
// and the single-domain update kernels (sph_step.hip) run it on the tile they have just
// updated, so a divide without bodies or slabs needs no classify launch (one pass over the
// particles' dcell / code / previous key less).  See sph_divide.hip for the three kernels of
// the incremental divide and what the classification words mean.
#pragma once
#include "sph_kernels.hpp"

namespace sphx {

constexpr int INC_BS = 256, INC_IPT = 4, INC_TILE = INC_BS * INC_IPT;  // = one k_inc_push block (GP = 4)
static_assert(INC_TILE == int(INC_TILE_SIZE), "tile size of the host allocations");
static_assert(INC_TILE <= 2048, "tile-local prefixes are 11 bits");
constexpr int INC_SUP = 64;  // tiles per super tile
constexpr unsigned CW_NEAR = 0x80000000u, CW_FAR = 0x40000000u, CW_LOC = 0x7ffu;
// slab: DROP = an old particle whose key became the discard box (a stale ghost): counted
// with the far movers in the prefixes (it is not a stayer) but kept out of the far list
// and never pushed; APP = a particle the exchange appended (no previous key)
constexpr unsigned CW_DROP = 0x20000000u, CW_APP = 0x10000000u;

// A key change by one of the 27 cell offsets dx + dy ncx + dz nsheet (distinct offsets:
// ncx >= 3 and ncy >= 3, or no y offsets when ncy = 1; checked on the host).
__device__ __forceinline__ bool inc_near(int d, int ncx, int nsheet, bool usey, bool usez) {
#pragma unroll
  for (int dz = -1; dz <= 1; dz++) {
#pragma unroll
    for (int dy = -1; dy <= 1; dy++) {
      if ((!usez && dz) || (!usey && dy)) continue;
      const int r = d - dz * nsheet - dy * ncx;
      if (r >= -1 && r <= 1) return true;
    }
  }
  return false;
}

// Tile b (INC_TILE particles, INC_IPT per thread at stride INC_BS; blocks of INC_BS threads,
// every thread of the block calls it): new key, near/far flags and their tile-local prefixes,
// the tile's counts (+ one atomic into its super tile of 64), near movers' keys at
// tile-major slots, far movers appended to a list.
__device__ __forceinline__ void inc_classify_tile(DevScalars* __restrict__ sc, const unsigned* __restrict__ dcell,
                                                  const typecode* __restrict__ code, const DivGrid& g, unsigned dcc,
                                                  const IncDivScratch& s, int usey, int usez, unsigned b) {
  __shared__ unsigned s_cn[INC_IPT * 4], s_cf[INC_IPT * 4];
  const unsigned n = sc->np;
  const unsigned nold = n - s.napp;  // the previous divide's particles; [nold, n) were appended
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (b == 0 && threadIdx.x == 0) sc->ndiv = n;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned key[INC_IPT], rn[INC_IPT], rf[INC_IPT], fpos[INC_IPT];
  bool nr[INC_IPT], fr[INC_IPT], dr[INC_IPT];
  // every load of the tile first (one memory latency), then the classification
  unsigned dc[INC_IPT], old[INC_IPT];
  typecode cd[INC_IPT];
#pragma unroll
  for (int k = 0; k < INC_IPT; k++) {
    const unsigned i = b * INC_TILE + k * INC_BS + threadIdx.x;
    const unsigned ii = i < n ? i : 0u;
    dc[k] = dcell[ii];
    cd[k] = code[ii];
    old[k] = s.skeys[ii];
  }
#pragma unroll
  for (int k = 0; k < INC_IPT; k++) {
    const unsigned i = b * INC_TILE + k * INC_BS + threadIdx.x;
    const bool valid = i < nold;
    key[k] = box_key(dc[k], cd[k], g, dcc);
    const int d = int(key[k] - old[k]);
    dr[k] = valid && d != 0 && key[k] == g.boxdiscard;
    nr[k] = valid && d != 0 && !dr[k] && inc_near(d, g.ncx, int(g.nsheet), usey != 0, usez != 0);
    fr[k] = valid && d != 0 && !nr[k] && !dr[k];
    const unsigned long long bn = __ballot(nr[k]), bf = __ballot(fr[k]), bfd = __ballot(fr[k] || dr[k]);
    rn[k] = unsigned(__popcll(bn & lt));
    rf[k] = unsigned(__popcll(bfd & lt));
    fpos[k] = 0;
    if (bf) {  // far movers (rare): appended to the list, one atomic per wave
      const unsigned lead = unsigned(__ffsll(static_cast<long long>(bf))) - 1u;
      unsigned base = 0;
      if (lane == lead) base = atomicAdd(&s.ctr[0], unsigned(__popcll(bf)));
      fpos[k] = __shfl(base, int(lead), 64) + unsigned(__popcll(bf & lt));
    }
    if (lane == 0) {
      s_cn[k * 4 + w] = unsigned(__popcll(bn));
      s_cf[k * 4 + w] = unsigned(__popcll(bfd));
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < INC_IPT; k++) {
    const unsigned i = b * INC_TILE + k * INC_BS + threadIdx.x;
    if (i >= n) continue;
    unsigned pn = 0, pf = 0;
    for (unsigned q = 0; q < unsigned(k * 4) + w; q++) {
      pn += s_cn[q];
      pf += s_cf[q];
    }
    s.newkey[i] = key[k];
    if (i >= nold) {  // appended: the input of their own sort
      s.cw[i] = CW_APP;
      s.akin[i - nold] = key[k];
      s.avin[i - nold] = i - nold;
      continue;
    }
    const unsigned ln = pn + rn[k], lf = pf + rf[k];  // tile-local exclusive prefixes
    s.cw[i] = ln | (lf << 11) | (nr[k] ? CW_NEAR : 0u) | (fr[k] ? CW_FAR : 0u) | (dr[k] ? CW_DROP : 0u);
    if (nr[k]) s.mkey[b * INC_TILE + ln] = key[k];
    if (fr[k]) {
      s.mfar[fpos[k]] = make_uint2(i, key[k]);
      s.fidx[i] = fpos[k];
    }
  }
  if (threadIdx.x == 0) {
    unsigned an = 0, af = 0;
#pragma unroll
    for (int q = 0; q < INC_IPT * 4; q++) {
      an += s_cn[q];
      af += s_cf[q];
    }
    s.tagg[b] = make_uint2(an, af);
    if (an | af) atomicAdd(&s.tsup[(b / INC_SUP) * TSUP_STRIDE], (static_cast<unsigned long long>(an) << 32) | af);
  }
}

}  // namespace sphx
