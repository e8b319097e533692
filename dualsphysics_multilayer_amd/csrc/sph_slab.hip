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
// Migrants travel as full 96-B records, ghosts as 40-B records (cell-relative float
// position, dcell, velrhop, idp, code).  Records are written in particle order (tile
// counts -> scan -> ballot-ranked scatter), so the receive order and hence the in-cell
// summation order of the next interaction are deterministic.  The reference has no
// multi-GPU path in this fork (JSphGpuSingle only); this follows the single-domain
// semantics exactly: the owner of a particle computes it with the same neighbour set
// it would have in one domain.
#include <algorithm>

#include "sph_kernels.hpp"
#include "sph_slabpack.hpp"

namespace sphx {

__global__ __launch_bounds__(PK_BS) void k_pack_count(const DevScalars* __restrict__ sc, PackArgs q) {
  pack_count_tile(sc, q, blockIdx.x);
}

// Exclusive scan of the tile counts (four streams), totals -> cnt; the tiles' staying
// particles and face ghosts summed (the face messages' ghost totals).
__global__ __launch_bounds__(1024) void k_pack_scan(const DevScalars* __restrict__ sc, PackArgs q) {
  __shared__ unsigned part[4][1024];
  __shared__ unsigned s_tot[3][16], s_fin[3];
  const unsigned nt = q.ntiles;
  const unsigned per = (nt + 1023) / 1024;
  const unsigned b0 = threadIdx.x * per, b1 = min(b0 + per, nt);
  // a thread's tiles of all seven count arrays loaded at once (one memory latency) when they
  // fit the registers (<= PS_MAX tiles per thread: capacities up to 4M particles), else in loops
  constexpr unsigned PS_MAX = 4;
  unsigned v[7][PS_MAX];
  const bool inreg = per <= PS_MAX;
  unsigned t[3] = {0u, 0u, 0u};
  if (inreg) {
#pragma unroll
    for (int d = 0; d < 7; d++)
#pragma unroll
      for (unsigned k = 0; k < PS_MAX; k++) v[d][k] = b0 + k < b1 ? q.tilecnt[d * nt + b0 + k] : 0u;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      unsigned s = 0;
#pragma unroll
      for (unsigned k = 0; k < PS_MAX; k++) s += v[d][k];
      part[d][threadIdx.x] = s;
    }
#pragma unroll
    for (int d = 0; d < 3; d++)
#pragma unroll
      for (unsigned k = 0; k < PS_MAX; k++) t[d] += v[4 + d][k];
  } else {
    for (int d = 0; d < 4; d++) {
      unsigned s = 0;
      for (unsigned i = b0; i < b1; i++) s += q.tilecnt[d * nt + i];
      part[d][threadIdx.x] = s;
    }
    for (unsigned i = b0; i < b1; i++)
      for (int d = 0; d < 3; d++) t[d] += q.tilecnt[(4 + d) * nt + i];
  }
  for (int d = 0; d < 3; d++)
    for (int off = 32; off > 0; off >>= 1) t[d] += __shfl_xor(t[d], off, 64);
  if ((threadIdx.x & 63) == 0)
    for (int d = 0; d < 3; d++) s_tot[d][threadIdx.x >> 6] = t[d];
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned u[3] = {0u, 0u, 0u};
    for (int w = 0; w < 16; w++)
      for (int d = 0; d < 3; d++) u[d] += s_tot[d][w];
    q.cnt->nkeep = u[0];
    q.cnt->ghosts[0] = u[1];
    q.cnt->ghosts[1] = u[2];
    for (int d = 0; d < 3; d++) s_fin[d] = u[d];
  }
  for (int off = 1; off < 1024; off <<= 1) {
    unsigned v[4];
    for (int d = 0; d < 4; d++) v[d] = threadIdx.x >= unsigned(off) ? part[d][threadIdx.x - off] : 0u;
    __syncthreads();
    for (int d = 0; d < 4; d++) part[d][threadIdx.x] += v[d];
    __syncthreads();
  }
  for (int d = 0; d < 4; d++) {
    unsigned run = threadIdx.x ? part[d][threadIdx.x - 1] : 0u;
    if (inreg) {
#pragma unroll
      for (unsigned k = 0; k < PS_MAX; k++)
        if (b0 + k < b1) {
          q.tilecnt[d * nt + b0 + k] = run;
          run += v[d][k];
        }
    } else {
      for (unsigned i = b0; i < b1; i++) {
        const unsigned x = q.tilecnt[d * nt + i];
        q.tilecnt[d * nt + i] = run;
        run += x;
      }
    }
  }
  if (threadIdx.x == 1023) {
    // ghosts: the face-box totals of k_pack_count (exchange after the divide), else records
    q.cnt->sendl[0] = q.fcnt[0] ? s_fin[1] : part[0][1023];
    q.cnt->sendr[0] = q.fcnt[0] ? s_fin[2] : part[1][1023];
    q.cnt->sendl[1] = part[2][1023];
    q.cnt->sendr[1] = part[3][1023];
    q.cnt->np = sc->np;
    if (q.fcnt[0])  // the face messages' headers {ghosts, migrants}
      for (int side = 0; side < 2; side++) {
        unsigned long long* h = reinterpret_cast<unsigned long long*>(q.fcnt[side] - FMSG_HDR);
        h[0] = side ? q.cnt->sendr[0] : q.cnt->sendl[0];
        h[1] = side ? q.cnt->sendr[1] : q.cnt->sendl[1];
      }
  }
}

__device__ __forceinline__ void write_ghost(const PackArgs& q, unsigned p, SlabGhost* dst) {
  const unsigned dc = q.a.dcell[p];
  const double2 pxy = q.a.posxy[p];
  const double pz = q.a.posz[p];
  // the owner's poscell of this particle (KerUpdatePosCell, global cell origin)
  const double ox = q.posminx + double(DcelCellx(q.dcc, dc)) * q.scelld;
  const double oy = q.posminy + double(DcelCelly(q.dcc, dc)) * q.scelld;
  const double oz = q.posminz + double(DcelCellz(q.dcc, dc)) * q.scelld;
  SlabGhost r;
  r.rx = float(pxy.x - ox);
  r.ry = float(pxy.y - oy);
  r.rz = float(pz - oz);
  r.dcell = dc;
  r.velrhop = q.a.velrhop[p];
  r.idp = q.a.idp[p];
  r.code = q.a.code[p];
  r.pad = 0;
  *dst = r;
}

__device__ __forceinline__ void write_migrant(const PackArgs& q, unsigned p, SlabRec* dst) {
  SlabRec r;
  r.posxy = q.a.posxy[p];
  r.posz = q.a.posz[p];
  r.idp = q.a.idp[p];
  r.dcell = q.a.dcell[p];
  r.velrhop = q.a.velrhop[p];
  r.vr2 = make_float4(0.f, 0.f, 0.f, 0.f);
  r.posxypre = make_double2(0., 0.);
  r.poszpre = 0.;
  if (q.withm1) r.vr2 = q.a.velrhopm1[p];
  if (q.withpre) {
    r.vr2 = q.a.velrhoppre[p];
    r.posxypre = q.a.posxypre[p];
    r.poszpre = q.a.poszpre[p];
  }
  r.code = q.a.code[p];
  r.flags = 0;
  r.pad = 0;
  r.normal = (q.normal && r.idp < q.nbound) ? q.normal[r.idp] : make_float4(0.f, 0.f, 0.f, 0.f);
  r.taua = q.a.tau ? q.a.tau[2 * p] : make_float4(0.f, 0.f, 0.f, 0.f);
  r.taub = q.a.tau ? q.a.tau[2 * p + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
  *dst = r;
}

__global__ __launch_bounds__(PK_BS) void k_pack_write(const DevScalars* __restrict__ sc, PackArgs q) {
  constexpr int NW = PK_BS / 64;
  __shared__ unsigned s_w[4][NW];
  const unsigned n = sc->np;
  const unsigned base = blockIdx.x * PK_TILE;
  unsigned off[4];
  for (int k = 0; k < 4; k++) off[k] = q.tilecnt[k * q.ntiles + blockIdx.x];
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned dcs[PK_ITEMS];
  load_dcells(q, base, n, dcs);
#pragma unroll
  for (int it = 0; it < PK_ITEMS; it++) {
    if (base + it * PK_BS >= n) break;  // uniform over the block
    const unsigned p = base + it * PK_BS + threadIdx.x;
    const unsigned c = p < n ? pack_class_dc(q, dcs[it]) : 0u;
    bool f[4];
    streams(c, f);
    unsigned long long bal[4];
#pragma unroll
    for (int k = 0; k < 4; k++) bal[k] = __ballot(f[k]);
    if (lane == 0)
      for (int k = 0; k < 4; k++) s_w[k][w] = __popcll(bal[k]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      unsigned pre = 0, tot = 0;
      for (int i = 0; i < NW; i++) {
        if (i < int(w)) pre += s_w[k][i];
        tot += s_w[k][i];
      }
      if (f[k] && !(k < 2 && q.fcnt[0])) {  // ghost records come after the divide (launch_ghost_pack)
        const unsigned long long slot = off[k] + pre + __popcll(bal[k] & lt);
        if (k < 2) {
          if (slot < q.b.gcap) write_ghost(q, p, (k == 0 ? q.b.gl : q.b.gr) + slot);
        } else {
          if (slot < q.b.mcap) write_migrant(q, p, (k == 2 ? q.b.ml : q.b.mr) + slot);
        }
      }
      off[k] += tot;
    }
    __syncthreads();
  }
}

PackArgs make_pack_args(unsigned cap, const PartArrays& a, DivGrid g, const KConst& K, const double dom_posmin[3],
                        bool has_left, bool has_right, bool withm1, bool withpre, unsigned* tilecnt, SlabCounts* cnt,
                        SlabSendBufs bufs, const float4* normal, unsigned nbound, const SlabFaces* faces) {
  PackArgs q;
  q.fcnt[0] = q.fcnt[1] = nullptr;
  q.W = g.sown0;
  if (faces) {  // zero on entry: k_unpack of the last exchange reset them
    q.fcnt[0] = faces->msg[0] + FMSG_HDR;
    q.fcnt[1] = faces->msg[1] + FMSG_HDR;
  }
  q.a = a;
  q.g = g;
  q.dcc = K.domcellcode;
  q.posminx = dom_posmin[0];
  q.posminy = dom_posmin[1];
  q.posminz = dom_posmin[2];
  q.scelld = K.scelld;
  q.has_left = has_left;
  q.has_right = has_right;
  q.withm1 = withm1;
  q.withpre = withpre;
  q.tilecnt = tilecnt;
  q.ntiles = (cap + PK_TILE - 1) / PK_TILE;
  q.cnt = cnt;
  q.b = bufs;
  q.normal = normal;
  q.nbound = nbound;
  return q;
}

void launch_slab_pack(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, DivGrid g, const KConst& K,
                      const double dom_posmin[3], bool has_left, bool has_right, bool withm1, bool withpre,
                      unsigned* tilecnt, SlabCounts* cnt, SlabSendBufs bufs, const float4* normal,
                      unsigned nbound, const SlabFaces* faces, bool counted) {
  const PackArgs q = make_pack_args(cap, a, g, K, dom_posmin, has_left, has_right, withm1, withpre, tilecnt, cnt, bufs,
                                    normal, nbound, faces);
  // (counted: the update kernel ran the count pass on its tiles, sph_slabpack.hpp)
  if (!counted) hipLaunchKernelGGL(k_pack_count, dim3(q.ntiles), dim3(PK_BS), 0, stm, sc, q);
  hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, stm, sc, q);
  hipLaunchKernelGGL(k_pack_write, dim3(q.ntiles), dim3(PK_BS), 0, stm, sc, q);
}

// ---------------------------------------------------------------------------------
// Face messages.  After their exchange one launch (before the host reads the counts): the
// received headers go to cnt->recvl / recvr (for the host's one read of the counts), and the
// exclusive prefixes of all four messages' nfb counts, one block per (message, tile of 8192):
// a block adds the counts of its message's earlier tiles (a block reduction; no inter-block
// ordering) to the scan of its own tile (coalesced loads into LDS, 8 consecutive per thread,
// wave + block scans).  The send messages' counts are zeroed for the next exchange by the
// exchange's unpack (k_unpack), once the neighbours have copied them.  (One block per message
// walking its tiles in turn took 16-38 us per exchange at the cfg3 y-slab face size, 25k
// boxes per message; one launch for the header and another for the scan, 6 + that.)
constexpr int FS_BS = 1024, FS_PT = 8, FS_TILE = FS_BS * FS_PT;
__global__ __launch_bounds__(FS_BS) void k_face_scan(SlabFaces f, SlabCounts* __restrict__ cnt, int hl, int hr) {
  __shared__ unsigned v[FS_TILE];
  __shared__ unsigned wsum[FS_BS / 64];
  const int m = int(blockIdx.y);  // send L, send R, receive L, receive R
  if ((m & 1) ? !hr : !hl) return;
  const unsigned t0 = blockIdx.x * unsigned(FS_TILE);
  const unsigned* __restrict__ c = f.msg[m] + FMSG_HDR;
  unsigned* __restrict__ pre = f.pre[m];
  const unsigned n = f.nfb, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (m >= 2 && blockIdx.x == 0 && threadIdx.x == 0) {  // the received header {ghosts, migrants}
    const unsigned long long* h = reinterpret_cast<const unsigned long long*>(f.msg[m]);
    unsigned long long* rv = m == 2 ? cnt->recvl : cnt->recvr;
    rv[0] = h[0];
    rv[1] = h[1];
  }
  // this tile's counts (loads in flight) and the sum of the earlier tiles' counts
#pragma unroll
  for (int k = 0; k < FS_PT; k++) {
    const unsigned i = t0 + k * FS_BS + threadIdx.x;
    v[k * FS_BS + threadIdx.x] = i < n ? c[i] : 0u;
  }
  unsigned below = 0;  // the earlier tiles: FS_PT loads per thread in flight at once
  for (unsigned i0 = 0; i0 < t0; i0 += FS_TILE) {
    unsigned e[FS_PT];
#pragma unroll
    for (int k = 0; k < FS_PT; k++) e[k] = c[i0 + k * FS_BS + threadIdx.x];  // whole tiles: in range
#pragma unroll
    for (int k = 0; k < FS_PT; k++) below += e[k];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) below += __shfl_xor(below, off, 64);
  if (lane == 0) wsum[w] = below;
  __syncthreads();
  unsigned base = 0;
  for (unsigned q = 0; q < FS_BS / 64; q++) base += wsum[q];
  __syncthreads();  // wsum is reused below
  unsigned x[FS_PT], sum = 0;
#pragma unroll
  for (int k = 0; k < FS_PT; k++) {
    x[k] = sum;
    sum += v[threadIdx.x * FS_PT + k];
  }
  unsigned inc = sum;  // inclusive wave scan of the thread sums
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(inc, off, 64);
    if (lane >= unsigned(off)) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  unsigned before = base;
  for (unsigned q = 0; q < w; q++) before += wsum[q];
  before += inc - sum;
#pragma unroll
  for (int k = 0; k < FS_PT; k++) v[threadIdx.x * FS_PT + k] = before + x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FS_PT; k++) {
    const unsigned i = t0 + k * FS_BS + threadIdx.x;
    if (i < n) pre[i] = v[k * FS_BS + threadIdx.x];
  }
  if (threadIdx.x == FS_BS - 1 && t0 + FS_TILE >= n) pre[n] = before + sum;
}

void launch_face_scan(hipStream_t stm, const SlabFaces& f, SlabCounts* cnt, bool has_left, bool has_right) {
  const unsigned nt = (f.nfb + FS_TILE - 1) / FS_TILE;
  hipLaunchKernelGGL(k_face_scan, dim3(nt ? nt : 1u, 4), dim3(FS_BS), 0, stm, f, cnt, int(has_left), int(has_right));
}

// Reserved ghost slots of the divide: one thread per face box (left face first) writes the
// box key of its count[idx] entries at pre[idx] (left: entries [0, ngl), right: after them).
__global__ __launch_bounds__(256) void k_ghost_keys(SlabFaces f, DivGrid g, unsigned ngl, unsigned* __restrict__ keys,
                                                    unsigned* __restrict__ vals, unsigned vbase, int hl, int hr) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const int side = t < f.nfb ? 0 : 1;
  const unsigned idx = side ? t - f.nfb : t;
  if (idx >= f.nfb || (side ? !hr : !hl)) return;
  const unsigned n = f.msg[2 + side][FMSG_HDR + idx];
  if (!n) return;
  const unsigned e0 = (side ? ngl : 0u) + f.pre[2 + side][idx];
  // the left ghost rim is [0, W), the right one [sown1, sown1 + W)
  const unsigned key = face_key(g, f.W, idx, side ? g.sown1 : 0);
  for (unsigned j = 0; j < n; j++) {
    keys[e0 + j] = key;
    if (vals) vals[e0 + j] = vbase + e0 + j;
  }
}

void launch_ghost_keys(hipStream_t stm, const SlabFaces& f, DivGrid g, unsigned ngl, unsigned ngr, unsigned* keys,
                       unsigned* vals, unsigned vbase) {
  if (ngl + ngr)
    hipLaunchKernelGGL(k_ghost_keys, dim3((2 * f.nfb + 255) / 256), dim3(256), 0, stm, f, g, ngl, keys, vals, vbase,
                       int(ngl > 0), int(ngr > 0));
}

// Ghost records from the sorted arrays, one thread per record (left face's records first):
// record r of a face belongs to the face box idx with pre[idx] <= r < pre[idx + 1] (binary
// search of the face's prefixes) and is that box's (r - pre[idx])-th member (the old members
// come first, in previous-index order — the order the pre-divide pack counted them in).
// Writes are contiguous per wave; a thread per box instead serialised the largest boxes
// (135-200 us per cfg3 slab divide, against ~5 us for this form).
__global__ __launch_bounds__(256) void k_ghost_pack(DevScalars* __restrict__ sc, SlabFaces f, DivGrid g,
                                                    const unsigned* __restrict__ bc, PartArrays a,
                                                    const float4* __restrict__ poscell, SlabSendBufs b, unsigned ngl,
                                                    unsigned ngr) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ngl + ngr) return;
  const int side = t < ngl ? 0 : 1;
  const unsigned r = side ? t - ngl : t;
  const unsigned* __restrict__ pre = f.pre[side];
  unsigned lo = 0, hi = f.nfb;  // pre[lo] <= r < pre[hi]
  while (hi - lo > 1u) {
    const unsigned mid = (lo + hi) >> 1;
    if (pre[mid] <= r) lo = mid;
    else hi = mid;
  }
  const unsigned key = face_key(g, f.W, lo, side ? g.sown1 - f.W : g.sown0);
  const unsigned i = bc[key] + (r - pre[lo]);
  if (i >= bc[key + 1]) {  // the divide placed fewer particles in the box than were counted
    atomicOr(&sc->error_flags, ERR_HALO_GHOST);
    return;
  }
  const float4 pc = poscell[i];
  SlabGhost rec;
  rec.rx = pc.x;
  rec.ry = pc.y;
  rec.rz = pc.z;
  rec.dcell = a.dcell[i];
  rec.velrhop = a.velrhop[i];
  rec.idp = a.idp[i];
  rec.code = a.code[i];
  rec.pad = 0;
  (side ? b.gr : b.gl)[r] = rec;
}

void launch_ghost_pack(hipStream_t stm, DevScalars* sc, const SlabFaces& f, DivGrid g, const unsigned* begincell,
                       const PartArrays& a, const float4* poscell, SlabSendBufs b, unsigned ngl, unsigned ngr) {
  if (ngl + ngr)
    hipLaunchKernelGGL(k_ghost_pack, dim3((ngl + ngr + 255) / 256), dim3(256), 0, stm, sc, f, g, begincell, a,
                       poscell, b, ngl, ngr);
}

// ---------------------------------------------------------------------------------
struct UnpackArgs {
  PartArrays a;
  const SlabRec* mig;
  const SlabGhost* gh;
  unsigned nm, ng, np;
  unsigned dcc;
  double posminx, posminy, posminz, scelld;
  int withm1, withpre;
  SlabCounts* cnt;
  DevScalars* sc;
  float4* normal;
  unsigned nbound;
  unsigned nfb;
  unsigned* fmsg[2];  // the send face messages' counts (zeroed here), or nullptr
};

// The exchange's last kernel: the migrants appended after the np particles; thread 0 sets the
// new counts and zeroes the accumulated pack counts, the threads from nm + ng on zero the send
// face messages' counts (k_pack_count accumulates them from zero), in place of memset launches.
__global__ __launch_bounds__(256) void k_unpack(UnpackArgs u) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    u.sc->np = u.np + u.nm + u.ng;
    u.sc->nown = u.cnt->nkeep + u.nm;
    u.cnt->nkeep = 0u;
    u.cnt->ghosts[0] = u.cnt->ghosts[1] = 0u;
  }
  if (i >= u.nm + u.ng) {
    const unsigned z = i - (u.nm + u.ng);
    if (z < 2u * u.nfb) {
      unsigned* c = u.fmsg[z < u.nfb ? 0 : 1];
      if (c) c[z < u.nfb ? z : z - u.nfb] = 0u;
    }
    return;
  }
  const unsigned p = u.np + i;
  PartArrays& a = u.a;
  if (i < u.nm) {
    const SlabRec r = u.mig[i];
    a.posxy[p] = r.posxy;
    a.posz[p] = r.posz;
    a.idp[p] = r.idp;
    a.dcell[p] = r.dcell;
    a.velrhop[p] = r.velrhop;
    a.code[p] = r.code;
    if (u.withm1) a.velrhopm1[p] = r.vr2;
    if (u.withpre) {
      a.velrhoppre[p] = r.vr2;
      a.posxypre[p] = r.posxypre;
      a.poszpre[p] = r.poszpre;
    }
    if (u.normal && r.idp < u.nbound) u.normal[r.idp] = r.normal;  // the owner's turned normal
    if (a.tau) {
      a.tau[2 * p] = r.taua;
      a.tau[2 * p + 1] = r.taub;
    }
  } else {
    const SlabGhost r = u.gh[i - u.nm];
    const double ox = u.posminx + double(DcelCellx(u.dcc, r.dcell)) * u.scelld;
    const double oy = u.posminy + double(DcelCelly(u.dcc, r.dcell)) * u.scelld;
    const double oz = u.posminz + double(DcelCellz(u.dcc, r.dcell)) * u.scelld;
    a.posxy[p] = make_double2(ox + double(r.rx), oy + double(r.ry));
    a.posz[p] = oz + double(r.rz);
    a.idp[p] = r.idp;
    a.dcell[p] = r.dcell;
    a.velrhop[p] = r.velrhop;
    a.code[p] = r.code;
  }
}

void launch_slab_unpack(hipStream_t stm, DevScalars* sc, const SlabRec* mig, unsigned nm, const SlabGhost* gh,
                        unsigned ng, unsigned np, const PartArrays& a, const KConst& K, const double dom_posmin[3],
                        bool withm1, bool withpre, SlabCounts* cnt, float4* normal, unsigned nbound,
                        const SlabFaces* faces, bool has_left, bool has_right) {
  UnpackArgs u;
  u.normal = normal;
  u.nbound = nbound;
  u.a = a;
  u.mig = mig;
  u.gh = gh;
  u.nm = nm;
  u.ng = ng;
  u.np = np;
  u.dcc = K.domcellcode;
  u.posminx = dom_posmin[0];
  u.posminy = dom_posmin[1];
  u.posminz = dom_posmin[2];
  u.scelld = K.scelld;
  u.withm1 = withm1;
  u.withpre = withpre;
  u.cnt = cnt;
  u.sc = sc;
  u.nfb = faces ? faces->nfb : 0u;
  u.fmsg[0] = faces && has_left ? faces->msg[0] + FMSG_HDR : nullptr;
  u.fmsg[1] = faces && has_right ? faces->msg[1] + FMSG_HDR : nullptr;
  const unsigned nthr = nm + ng + 2u * u.nfb;
  hipLaunchKernelGGL(k_unpack, dim3(nthr ? (nthr + 255) / 256 : 1u), dim3(256), 0, stm, u);
}

// ---------------------------------------------------------------------------------
__global__ void k_rank_ordered_sum(const float* __restrict__ g, int n, int nranks, float* __restrict__ out) {
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  float v = 0.f;
  for (int r = 0; r < nranks; r++) v = __fadd_rn(v, g[size_t(r) * size_t(n) + size_t(i)]);
  out[i] = v;
}

void launch_rank_ordered_sum(hipStream_t stm, const float* gathered, int n, int nranks, float* out) {
  if (n > 0) hipLaunchKernelGGL(k_rank_ordered_sum, dim3((n + 255) / 256), dim3(256), 0, stm, gathered, n, nranks, out);
}

__global__ void k_rank_ordered_sum_p(RankPtrs rp, int n, int nranks, float* __restrict__ out) {
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  float v = 0.f;
  for (int r = 0; r < nranks; r++) v = __fadd_rn(v, static_cast<const float*>(rp.p[r])[i]);
  out[i] = v;
}

void launch_rank_ordered_sum(hipStream_t stm, const RankPtrs& rp, int n, int nranks, float* out) {
  if (n > 0) hipLaunchKernelGGL(k_rank_ordered_sum_p, dim3((n + 255) / 256), dim3(256), 0, stm, rp, n, nranks, out);
}

__global__ void k_rank_max_u32(RankPtrs rp, int n, int nranks, unsigned* __restrict__ out) {
  const int i = int(threadIdx.x);
  if (i >= n) return;
  unsigned v = 0u;
  for (int r = 0; r < nranks; r++) v = max(v, static_cast<const unsigned*>(rp.p[r])[i]);
  out[i] = v;
}

// blockIdx.y: which copy; 16-B words when both pointers and the size allow, else 4-B, else bytes.
__global__ __launch_bounds__(256) void k_copy_pair(unsigned char* __restrict__ d0, const unsigned char* __restrict__ s0,
                                                   size_t n0, unsigned char* __restrict__ d1,
                                                   const unsigned char* __restrict__ s1, size_t n1) {
  unsigned char* d = blockIdx.y ? d1 : d0;
  const unsigned char* src = blockIdx.y ? s1 : s0;
  const size_t n = blockIdx.y ? n1 : n0;
  const size_t stride = size_t(gridDim.x) * blockDim.x, t0 = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t al = (reinterpret_cast<size_t>(d) | reinterpret_cast<size_t>(src) | n);
  if ((al & 15u) == 0) {
    for (size_t i = t0; i < n / 16; i += stride)
      reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(src)[i];
  } else if ((al & 3u) == 0) {
    for (size_t i = t0; i < n / 4; i += stride)
      reinterpret_cast<unsigned*>(d)[i] = reinterpret_cast<const unsigned*>(src)[i];
  } else {
    for (size_t i = t0; i < n; i += stride) d[i] = src[i];
  }
}

void launch_copy_pair(hipStream_t stm, void* d0, const void* s0, size_t n0, void* d1, const void* s1, size_t n1) {
  const size_t words = (std::max(n0, n1) + 15) / 16;
  const unsigned nb = unsigned(std::min<size_t>(std::max<size_t>((words + 255) / 256, 1), 1024));
  hipLaunchKernelGGL(k_copy_pair, dim3(nb, 2), dim3(256), 0, stm, static_cast<unsigned char*>(d0),
                     static_cast<const unsigned char*>(s0), n0, static_cast<unsigned char*>(d1),
                     static_cast<const unsigned char*>(s1), n1);
}

// (nranks <= RankPtrs::MAXR and n <= 64: LocalTransport's device_reduce and its 8-value limit)
void launch_rank_max_u32(hipStream_t stm, const RankPtrs& rp, int n, int nranks, unsigned* out) {
  if (n > 0) hipLaunchKernelGGL(k_rank_max_u32, dim3(1), dim3(64), 0, stm, rp, n, nranks, out);
}

// Owned particles per global column (u32 atomics in LDS-free global memory: integer counts
// are order independent, so every run and every rank sees the same numbers).
__global__ __launch_bounds__(256) void k_column_counts(const DevScalars* __restrict__ sc, PartArrays a, DivGrid g,
                                                       unsigned dcc, int ncxg, unsigned* __restrict__ cnt) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= sc->np) return;
  const unsigned dc = a.dcell[p];
  if (dc == DCELL_DISCARD || dc == DCELL_OUT) return;
  const int lcx = slab_local(g, dcc, dc), gcx = lcx + g.soff;
  if (!slab_owned(g, lcx) || gcx >= ncxg) return;  // ghosts are counted by their owner
  const bool fluid = CodeType(a.code[p]) >= CODE_TYPE_FLOATING;
  atomicAdd(&cnt[(fluid ? 0 : ncxg) + gcx], 1u);
}

__global__ void k_counts_to_float(unsigned* __restrict__ c, int n) {
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) reinterpret_cast<float*>(c)[i] = float(c[i]);
}

void launch_column_counts(hipStream_t stm, unsigned cap, const DevScalars* sc, const PartArrays& a, DivGrid g,
                          const KConst& K, int ncxg, float* counts) {
  unsigned* c = reinterpret_cast<unsigned*>(counts);
  (void)hipMemsetAsync(c, 0, sizeof(unsigned) * 2 * size_t(ncxg), stm);
  hipLaunchKernelGGL(k_column_counts, dim3((cap + 255) / 256), dim3(256), 0, stm, sc, a, g, K.domcellcode, ncxg, c);
  hipLaunchKernelGGL(k_counts_to_float, dim3((2 * ncxg + 255) / 256), dim3(256), 0, stm, c, 2 * ncxg);
}

}  // namespace sphx
