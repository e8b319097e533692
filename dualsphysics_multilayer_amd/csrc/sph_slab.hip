// sph_slab.hip — slab decomposition over x: pack / unpack of the particles that cross
// a slab face.
//
// Each rank owns the global x-cell columns [c0, c1) and keeps read-only ghost copies
// of the neighbours' particles in columns c0-1 and c1 (one column = 2h = the support
// radius, full-cell mode).  After every update (the only place positions change):
//   * stale ghosts were marked DCELL_DISCARD by the update kernels (sph_step.hip);
//   * an owned particle whose new column is < c0 (>= c1) MIGRATES: its full state goes
//     to the left (right) neighbour, and it stays here as a ghost (movement is bounded
//     by MovLimit = 0.9*Scell < one column, so it lands exactly in the ghost column);
//   * an owned particle in column c0 (c1-1) is copied to the left (right) neighbour
//     as a ghost.
// Records are written in particle order (tile counts -> scan -> ballot-ranked
// scatter), so the receive order and hence the in-cell summation order of the next
// interaction are deterministic.  The reference has no multi-GPU path in this fork
// (JSphGpuSingle only); this follows the single-domain semantics exactly: the
// owner of a particle computes it with the same neighbour set it would have in one
// domain.
#include "sph_kernels.hpp"

namespace sphx {

struct PackArgs {
  PartArrays a;
  DivGrid g;
  unsigned dcc;
  int has_left, has_right, withm1, withpre;
  unsigned* tilecnt;  // [2][ntiles]
  unsigned ntiles;
  SlabCounts* cnt;
  SlabRec* sendl;
  SlabRec* sendr;
  unsigned long long sendcap;
};

// bit 0: record for the left neighbour, bit 1: record for the right, bit 2: stays owned.
__device__ __forceinline__ unsigned pack_class(const PackArgs& q, unsigned p) {
  const unsigned dc = q.a.dcell[p];
  if (dc == DCELL_DISCARD || dc == DCELL_OUT) return 0u;
  const int lcx = int(DcelCellx(q.dcc, dc)) - q.g.xoff;
  if (lcx < q.g.xown0) return q.has_left ? 1u : 0u;
  if (lcx >= q.g.xown1) return q.has_right ? 2u : 0u;
  unsigned c = 4u;
  if (lcx == q.g.xown0 && q.has_left) c |= 1u;
  if (lcx == q.g.xown1 - 1 && q.has_right) c |= 2u;
  return c;
}

__global__ __launch_bounds__(PK_BS) void k_pack_count(const DevScalars* __restrict__ sc, PackArgs q) {
  __shared__ unsigned s[3][PK_BS / 64];
  const unsigned n = sc->np;
  const unsigned base = blockIdx.x * PK_TILE;
  unsigned cl = 0, cr = 0, ck = 0;
  for (int it = 0; it < PK_ITEMS; it++) {
    const unsigned p = base + it * PK_BS + threadIdx.x;
    if (p < n) {
      const unsigned c = pack_class(q, p);
      cl += c & 1u;
      cr += (c >> 1) & 1u;
      ck += (c >> 2) & 1u;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    cl += __shfl_xor(cl, off, 64);
    cr += __shfl_xor(cr, off, 64);
    ck += __shfl_xor(ck, off, 64);
  }
  const unsigned w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s[0][w] = cl;
    s[1][w] = cr;
    s[2][w] = ck;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned tl = 0, tr = 0, tk = 0;
    for (int i = 0; i < PK_BS / 64; i++) {
      tl += s[0][i];
      tr += s[1][i];
      tk += s[2][i];
    }
    q.tilecnt[blockIdx.x] = tl;
    q.tilecnt[q.ntiles + blockIdx.x] = tr;
    if (tk) atomicAdd(&q.cnt->nkeep, tk);
  }
}

// Exclusive scan of the tile counts (both directions), totals -> cnt->send.
__global__ __launch_bounds__(1024) void k_pack_scan(const DevScalars* __restrict__ sc, PackArgs q) {
  __shared__ unsigned part[2][1024];
  const unsigned nt = q.ntiles;
  const unsigned per = (nt + 1023) / 1024;
  const unsigned b0 = threadIdx.x * per, b1 = min(b0 + per, nt);
  for (int d = 0; d < 2; d++) {
    unsigned s = 0;
    for (unsigned i = b0; i < b1; i++) s += q.tilecnt[d * nt + i];
    part[d][threadIdx.x] = s;
  }
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const unsigned v0 = threadIdx.x >= unsigned(off) ? part[0][threadIdx.x - off] : 0u;
    const unsigned v1 = threadIdx.x >= unsigned(off) ? part[1][threadIdx.x - off] : 0u;
    __syncthreads();
    part[0][threadIdx.x] += v0;
    part[1][threadIdx.x] += v1;
    __syncthreads();
  }
  for (int d = 0; d < 2; d++) {
    unsigned run = threadIdx.x ? part[d][threadIdx.x - 1] : 0u;
    for (unsigned i = b0; i < b1; i++) {
      const unsigned v = q.tilecnt[d * nt + i];
      q.tilecnt[d * nt + i] = run;
      run += v;
    }
  }
  if (threadIdx.x == 1023) {
    q.cnt->send[0] = part[0][1023];
    q.cnt->send[1] = part[1][1023];
    q.cnt->np = sc->np;
  }
}

__device__ __forceinline__ void write_rec(const PackArgs& q, unsigned p, SlabRec* dst, bool migrant) {
  SlabRec r;
  r.posxy = q.a.posxy[p];
  r.posz = q.a.posz[p];
  r.idp = q.a.idp[p];
  r.dcell = q.a.dcell[p];
  r.velrhop = q.a.velrhop[p];
  r.vr2 = make_float4(0.f, 0.f, 0.f, 0.f);
  r.posxypre = make_double2(0., 0.);
  r.poszpre = 0.;
  if (migrant) {
    if (q.withm1) r.vr2 = q.a.velrhopm1[p];
    if (q.withpre) {
      r.vr2 = q.a.velrhoppre[p];
      r.posxypre = q.a.posxypre[p];
      r.poszpre = q.a.poszpre[p];
    }
  }
  r.code = q.a.code[p];
  r.flags = migrant ? SLABREC_MIGRANT : 0;
  r.pad = 0;
  *dst = r;
}

__global__ __launch_bounds__(PK_BS) void k_pack_write(const DevScalars* __restrict__ sc, PackArgs q) {
  constexpr int NW = PK_BS / 64;
  __shared__ unsigned s_w[2][NW];
  const unsigned n = sc->np;
  const unsigned base = blockIdx.x * PK_TILE;
  unsigned offl = q.tilecnt[blockIdx.x], offr = q.tilecnt[q.ntiles + blockIdx.x];
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int it = 0; it < PK_ITEMS; it++) {
    if (base + it * PK_BS >= n) break;  // uniform over the block
    const unsigned p = base + it * PK_BS + threadIdx.x;
    const unsigned c = p < n ? pack_class(q, p) : 0u;
    const unsigned long long bl = __ballot(c & 1u), br = __ballot((c >> 1) & 1u);
    if (lane == 0) {
      s_w[0][w] = __popcll(bl);
      s_w[1][w] = __popcll(br);
    }
    __syncthreads();
    unsigned prel = 0, prer = 0, totl = 0, totr = 0;
    for (int i = 0; i < NW; i++) {
      if (i < int(w)) {
        prel += s_w[0][i];
        prer += s_w[1][i];
      }
      totl += s_w[0][i];
      totr += s_w[1][i];
    }
    const bool migrant = (c & 4u) == 0u;
    if (c & 1u) {
      const unsigned long long k = offl + prel + __popcll(bl & lt);
      if (k < q.sendcap) write_rec(q, p, q.sendl + k, migrant);
    }
    if (c & 2u) {
      const unsigned long long k = offr + prer + __popcll(br & lt);
      if (k < q.sendcap) write_rec(q, p, q.sendr + k, migrant);
    }
    offl += totl;
    offr += totr;
    __syncthreads();
  }
}

void launch_slab_pack(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, DivGrid g, const KConst& K,
                      bool has_left, bool has_right, bool withm1, bool withpre, unsigned* tilecnt, SlabCounts* cnt,
                      SlabRec* sendl, SlabRec* sendr, unsigned long long sendcap) {
  PackArgs q;
  q.a = a;
  q.g = g;
  q.dcc = K.domcellcode;
  q.has_left = has_left;
  q.has_right = has_right;
  q.withm1 = withm1;
  q.withpre = withpre;
  q.tilecnt = tilecnt;
  q.ntiles = (cap + PK_TILE - 1) / PK_TILE;
  q.cnt = cnt;
  q.sendl = sendl;
  q.sendr = sendr;
  q.sendcap = sendcap;
  hipLaunchKernelGGL(k_pack_count, dim3(q.ntiles), dim3(PK_BS), 0, stm, sc, q);
  hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, stm, sc, q);
  hipLaunchKernelGGL(k_pack_write, dim3(q.ntiles), dim3(PK_BS), 0, stm, sc, q);
}

// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_unpack(const SlabRec* __restrict__ recv, unsigned np, unsigned nrecv,
                                                PartArrays a, int withm1, int withpre, SlabCounts* __restrict__ cnt) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned mig = 0;
  if (i < nrecv) {
    const SlabRec r = recv[i];
    const unsigned p = np + i;
    a.posxy[p] = r.posxy;
    a.posz[p] = r.posz;
    a.idp[p] = r.idp;
    a.dcell[p] = r.dcell;
    a.velrhop[p] = r.velrhop;
    a.code[p] = r.code;
    if (withm1) a.velrhopm1[p] = r.vr2;
    if (withpre) {
      a.velrhoppre[p] = r.vr2;
      a.posxypre[p] = r.posxypre;
      a.poszpre[p] = r.poszpre;
    }
    mig = (r.flags & SLABREC_MIGRANT) ? 1u : 0u;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mig += __shfl_xor(mig, off, 64);
  if ((threadIdx.x & 63) == 0 && mig) atomicAdd(&cnt->nkeep, mig);
}

__global__ void k_unpack_finish(DevScalars* __restrict__ sc, const SlabCounts* __restrict__ cnt, unsigned np,
                                unsigned nrecv) {
  sc->np = np + nrecv;
  sc->nown = cnt->nkeep;
}

void launch_slab_unpack(hipStream_t stm, DevScalars* sc, const SlabRec* recv, unsigned np, unsigned nrecv,
                        const PartArrays& a, bool withm1, bool withpre, SlabCounts* cnt) {
  if (nrecv)
    hipLaunchKernelGGL(k_unpack, dim3((nrecv + 255) / 256), dim3(256), 0, stm, recv, np, nrecv, a, int(withm1),
                       int(withpre), cnt);
  hipLaunchKernelGGL(k_unpack_finish, dim3(1), dim3(1), 0, stm, sc, cnt, np, nrecv);
}

}  // namespace sphx
