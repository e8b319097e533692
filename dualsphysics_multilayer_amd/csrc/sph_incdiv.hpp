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

// The tile's particle i = b INC_TILE + k INC_BS + t of a block of BS threads (BS a multiple of
// INC_BS dividing INC_TILE): a thread's e-th particle is e BS + its index, so k = e BS / INC_BS
// + index / INC_BS and t = index % INC_BS — the same order of waves (k, t / 64) for every BS.
template <int BS>
struct TileMap {
  static_assert(BS % INC_BS == 0 && INC_TILE % BS == 0, "blocks of INC_BS .. INC_TILE threads");
  static constexpr int IPT = INC_TILE / BS;
  __device__ __forceinline__ static int k(int e) { return e * (BS / INC_BS) + int(threadIdx.x) / INC_BS; }
  __device__ __forceinline__ static unsigned t() { return threadIdx.x % unsigned(INC_BS); }
};

// A particle's classification inputs held in registers by the update kernel that has just
// written them (one particle per thread): its new dcell and code, its previous divide's key.
struct ClsVals {
  unsigned dc;
  typecode cd;
  unsigned old;
};

// Tile b (INC_TILE particles; every thread of the block calls it): new key, near/far flags and
// their tile-local prefixes, the tile's counts (+ one atomic into its super tile of 64), near
// movers' keys at tile-major slots, far movers appended to a list.  vals: the inputs of the
// thread's IPT particles in registers, instead of loads of dcell / code / skeys.
template <int BS = INC_BS>
__device__ __forceinline__ void inc_classify_tile(DevScalars* __restrict__ sc, const unsigned* __restrict__ dcell,
                                                  const typecode* __restrict__ code, const DivGrid& g, unsigned dcc,
                                                  const IncDivScratch& s, int usey, int usez, unsigned b,
                                                  const ClsVals* vals = nullptr) {
  using M = TileMap<BS>;
  constexpr int IPT = M::IPT;
  __shared__ unsigned s_cn[INC_IPT * 4], s_cf[INC_IPT * 4];
  const unsigned n = sc->np;
  const unsigned nold = n - s.napp;  // the previous divide's particles; [nold, n) were appended
  const unsigned lane = threadIdx.x & 63, w = M::t() >> 6;
  if (b == 0 && threadIdx.x == 0) sc->ndiv = n;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned key[IPT], rn[IPT], rf[IPT], fpos[IPT];
  bool nr[IPT], fr[IPT], dr[IPT];
  // every load of the tile first (one memory latency), then the classification
  unsigned dc[IPT], old[IPT];
  typecode cd[IPT];
#pragma unroll
  for (int e = 0; e < IPT; e++) {
    if (vals) {
      dc[e] = vals[e].dc;
      cd[e] = vals[e].cd;
      old[e] = vals[e].old;
      continue;
    }
    const unsigned i = b * INC_TILE + M::k(e) * INC_BS + M::t();
    const unsigned ii = i < n ? i : 0u;
    dc[e] = dcell[ii];
    cd[e] = code[ii];
    old[e] = s.skeys[ii];
  }
#pragma unroll
  for (int e = 0; e < IPT; e++) {
    const int k = M::k(e);
    const unsigned i = b * INC_TILE + k * INC_BS + M::t();
    const bool valid = i < nold;
    key[e] = box_key(dc[e], cd[e], g, dcc);
    const int d = int(key[e] - old[e]);
    dr[e] = valid && d != 0 && key[e] == g.boxdiscard;
    nr[e] = valid && d != 0 && !dr[e] && inc_near(d, g.ncx, int(g.nsheet), usey != 0, usez != 0);
    fr[e] = valid && d != 0 && !nr[e] && !dr[e];
    const unsigned long long bn = __ballot(nr[e]), bf = __ballot(fr[e]), bfd = __ballot(fr[e] || dr[e]);
    rn[e] = unsigned(__popcll(bn & lt));
    rf[e] = unsigned(__popcll(bfd & lt));
    fpos[e] = 0;
    if (bf) {  // far movers (rare): appended to the list, one atomic per wave
      const unsigned lead = unsigned(__ffsll(static_cast<long long>(bf))) - 1u;
      unsigned base = 0;
      if (lane == lead) base = atomicAdd(&s.ctr[0], unsigned(__popcll(bf)));
      fpos[e] = __shfl(base, int(lead), 64) + unsigned(__popcll(bf & lt));
    }
    if (lane == 0) {
      s_cn[k * 4 + w] = unsigned(__popcll(bn));
      s_cf[k * 4 + w] = unsigned(__popcll(bfd));
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < IPT; e++) {
    const int k = M::k(e);
    const unsigned i = b * INC_TILE + k * INC_BS + M::t();
    if (i >= n) continue;
    unsigned pn = 0, pf = 0;
    for (unsigned q = 0; q < unsigned(k * 4) + w; q++) {
      pn += s_cn[q];
      pf += s_cf[q];
    }
    s.newkey[i] = key[e];
    if (i >= nold) {  // appended: the input of their own sort
      s.cw[i] = CW_APP;
      s.akin[i - nold] = key[e];
      s.avin[i - nold] = i - nold;
      continue;
    }
    const unsigned ln = pn + rn[e], lf = pf + rf[e];  // tile-local exclusive prefixes
    s.cw[i] = ln | (lf << 11) | (nr[e] ? CW_NEAR : 0u) | (fr[e] ? CW_FAR : 0u) | (dr[e] ? CW_DROP : 0u);
    if (nr[e]) s.mkey[b * INC_TILE + ln] = key[e];
    if (fr[e]) {
      s.mfar[fpos[e]] = make_uint2(i, key[e]);
      s.fidx[i] = fpos[e];
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
