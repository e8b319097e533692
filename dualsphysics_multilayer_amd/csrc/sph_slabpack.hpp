// sph_slabpack.hpp — the slab exchange's classification and count pass (sph_slab.hip) as
// device functions: k_pack_count runs the count pass, and the slab update kernels
// (sph_step.hip) run it on the tile they have just updated, so the exchange after an update
// starts with its scan (one pass over the particles' dcell / code less per divide).
#pragma once
#include "sph_incdiv.hpp"
#include "sph_kernels.hpp"

namespace sphx {


// bit 0: record for the left neighbour, bit 1: record for the right, bit 2: stays owned
// (so a record with bit 2 is a ghost copy, without it a migrant).
__device__ __forceinline__ unsigned pack_class_dc(const PackArgs& q, unsigned dc) {
  if (dc == DCELL_DISCARD || dc == DCELL_OUT) return 0u;
  const int lcx = slab_local(q.g, q.dcc, dc);
  if (lcx < q.g.sown0) return q.has_left ? 1u : 0u;
  if (lcx >= q.g.sown1) return q.has_right ? 2u : 0u;
  unsigned c = 4u;
  if (in_left_face(q.g, lcx) && q.has_left) c |= 1u;
  if (in_right_face(q.g, lcx) && q.has_right) c |= 2u;
  return c;
}

// The dcell words of a thread's PK_ITEMS particles, loaded before any of them is classified:
// the per-particle work (ballots, face atomics, LDS ranks) would otherwise serialise the
// loads, one memory latency per item.
__device__ __forceinline__ void load_dcells(const PackArgs& q, unsigned base, unsigned n, unsigned (&dcs)[PK_ITEMS]) {
#pragma unroll
  for (int it = 0; it < PK_ITEMS; it++) {
    const unsigned p = base + it * PK_BS + threadIdx.x;
    dcs[it] = p < n ? q.a.dcell[p] : DCELL_DISCARD;
  }
}

// the four stream flags of a class
__device__ __forceinline__ void streams(unsigned c, bool f[4]) {
  const bool stay = (c & 4u) != 0u;
  f[0] = (c & 1u) && stay;   // ghost -> left
  f[1] = (c & 2u) && stay;   // ghost -> right
  f[2] = (c & 1u) && !stay;  // migrant -> left
  f[3] = (c & 2u) && !stay;  // migrant -> right
}

// The count pass of one tile (PK_TILE particles; BS threads with PK_TILE / BS particles each at
// stride BS).  vals: the dcell and code of the thread's particles in registers.
template <int BS = PK_BS>
__device__ __forceinline__ void pack_count_tile(const DevScalars* __restrict__ sc, const PackArgs& q, unsigned tile,
                                                const ClsVals* vals = nullptr) {
  static_assert(BS % 64 == 0 && PK_TILE % BS == 0, "whole waves, whole tiles");
  constexpr int IPT = PK_TILE / BS;
  __shared__ unsigned s[7][BS / 64];
  const unsigned n = sc->np;
  const unsigned base = tile * PK_TILE;
  unsigned c4[7] = {0, 0, 0, 0, 0, 0, 0};  // 4 streams, staying, ghosts per face (face boxes)
  unsigned dcs[IPT];
#pragma unroll
  for (int it = 0; it < IPT; it++) {
    const unsigned p = base + it * BS + threadIdx.x;
    dcs[it] = p < n ? (vals ? vals[it].dc : q.a.dcell[p]) : DCELL_DISCARD;
  }
#pragma unroll
  for (int it = 0; it < IPT; it++) {
    const unsigned p = base + it * BS + threadIdx.x;
    int fi[2] = {-1, -1};  // face box of an owned face particle, per face
    if (p < n) {
      const unsigned c = pack_class_dc(q, dcs[it]);
      bool f[4];
      streams(c, f);
#pragma unroll
      for (int k = 0; k < 4; k++) c4[k] += f[k] ? 1u : 0u;
      c4[4] += (c >> 2) & 1u;
      if (q.fcnt[0] && (c & 4u) && (c & 3u)) {
        const unsigned key = box_key(dcs[it], vals ? vals[it].cd : q.a.code[p], q.g, q.dcc);
        if (c & 1u) fi[0] = face_idx(q.g, q.W, key, q.g.sown0);
        if (c & 2u) fi[1] = face_idx(q.g, q.W, key, q.g.sown1 - q.W);
      }
    }
    if (q.fcnt[0]) {
      // count per face box with one atomic per distinct box of the wave (the particles are
      // in the previous divide's cell order: a wave spans a few boxes)
#pragma unroll
      for (int side = 0; side < 2; side++) {
        c4[5 + side] += fi[side] >= 0 ? 1u : 0u;
        unsigned long long act = __ballot(fi[side] >= 0);
        while (act) {
          const int lead = __ffsll(static_cast<long long>(act)) - 1;
          const int b = __shfl(fi[side], lead, 64);
          const unsigned long long same = __ballot(fi[side] == b);
          if (int(threadIdx.x & 63) == lead) atomicAdd(&q.fcnt[side][b], unsigned(__popcll(same)));
          act &= ~same;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 7; k++)
    for (int off = 32; off > 0; off >>= 1) c4[k] += __shfl_xor(c4[k], off, 64);
  const unsigned w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 7; k++) s[k][w] = c4[k];
  __syncthreads();
  if (threadIdx.x < 7) {  // per tile; k_pack_scan sums them (no same-line atomics per block)
    const unsigned k = threadIdx.x;
    unsigned t = 0;
    for (int i = 0; i < BS / 64; i++) t += s[k][i];
    q.tilecnt[k * q.ntiles + tile] = t;
  }
}

}  // namespace sphx
