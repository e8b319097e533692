// sph_kernels.hpp — host-side launchers of the HIP kernels (one per hot-path phase).
//
// All launchers are asynchronous on `stm`, never allocate and never synchronise,
// so a whole step can be captured into a hipGraph.  Grids are sized from the
// particle capacity; the live counts (np, npb, npbok) are read on the device from
// DevScalars, so no host round trip is needed between phases.
#pragma once
#include "../../include/sphcore.h"
#include "sph_device.hpp"

namespace sphx {

// One set of per-particle arrays (cell-sorted order).
struct PartArrays {
  unsigned* idp = nullptr;
  typecode* code = nullptr;
  unsigned* dcell = nullptr;
  double2* posxy = nullptr;
  double* posz = nullptr;
  float4* velrhop = nullptr;
  float4* velrhopm1 = nullptr;   // Verlet
  double2* posxypre = nullptr;   // Symplectic
  double* poszpre = nullptr;
  float4* velrhoppre = nullptr;
  float4* tau = nullptr;         // Laminar+SPS: sub-particle stress tensor, [2i] {xx,xy,xz,yy}, [2i+1] {yz,zz}
};

// A double product that is not fused into a following add (an opaque use of the rounded
// product): the update's arithmetic as the reference's plain multiplies and adds, whatever the
// surrounding code shape (sph_step.hip).
__device__ __forceinline__ double nc(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

// JSphCpu::UpdatePos (JSphCpu.cpp:1240-1293), single domain, no periodic.
// Returns the new dcell; rcode (optional): the particle's code held in registers, updated in
// place (else read from a.code when the particle leaves).
__device__ __forceinline__ unsigned update_pos(const KConst& K, double rx, double ry, double rz, double movx,
                                               double movy, double movz, bool outrhop, unsigned p, const PartArrays& a,
                                               typecode* rcode_in = nullptr) {
  const bool outmove = (fabsf(float(movx)) > K.movlimit || fabsf(float(movy)) > K.movlimit ||
                        fabsf(float(movz)) > K.movlimit);
  rx += movx;
  ry += movy;
  rz += movz;
  if (K.symmetry && ry < 0) ry = -ry;  // Symmetry: reflected across y = 0 (JSphCpu.cpp:1247)
  const double dx = rx - K.map_realposmin_x, dy = ry - K.map_realposmin_y, dz = rz - K.map_realposmin_z;
  const bool out = (dx != dx || dy != dy || dz != dz || dx < 0 || dy < 0 || dz < 0 || dx >= K.map_realsize_x ||
                    dy >= K.map_realsize_y || dz >= K.map_realsize_z);
  a.posxy[p] = make_double2(rx, ry);
  a.posz[p] = rz;
  if (outrhop || outmove || out) {
    typecode rcode = rcode_in ? *rcode_in : a.code[p];
    if (out) rcode = CodeSetNormal(rcode) | CODE_OUTPOS;
    else if (outrhop) rcode = CodeSetNormal(rcode) | CODE_OUTRHOP;
    else rcode = CodeSetNormal(rcode) | CODE_OUTMOVE;
    a.code[p] = rcode;
    if (rcode_in) *rcode_in = rcode;
    a.dcell[p] = DCELL_OUT;
    return DCELL_OUT;
  }
  const unsigned cx = unsigned(dx / K.scelld), cy = unsigned(dy / K.scelld), cz = unsigned(dz / K.scelld);
  const unsigned dc = DcelCell(K.domcellcode, cx, cy, cz);
  a.dcell[p] = dc;
  return dc;
}
// Boundary and floating particles: UpdatePos with outrhop=false (MoveLinBound/MoveMatBound,
// JSphCpu.cpp:1699,1721; RunFloating, JSphCpuSingle.cpp:969).
__device__ __forceinline__ void update_pos_bound(const KConst& K, double rx, double ry, double rz, double movx,
                                                 double movy, double movz, unsigned p, const PartArrays& a,
                                                 DevScalars* sc) {
  (void)sc;
  update_pos(K, rx, ry, rz, movx, movy, movz, false, p, a);
}

// JSphShifting::RunCpu (JSphShifting.cpp:388-418) for one fluid particle, added to its
// displacement as ComputeSymplecticCorr / ComputeVerletVarsFluid do: rs = the interaction's
// shifting sums (x = FLT_MAX: cancelled next to the boundary), v = the velocity RunShifting
// reads, dt = the step's dt.
__device__ __forceinline__ void shift_displacement(const KConst& K, float4 rs, float4 v, double dt, double& dx,
                                                   double& dy, double& dz) {
  if (rs.x == 3.402823466e+38f) return;
  const double coefumagn = dt * double(K.shiftcoef) * double(K.kernelh);
  const double vx = double(v.x), vy = double(v.y), vz = double(v.z);
  double umagn = coefumagn * sqrt(nc(vx * vx) + nc(vy * vy) + nc(vz * vz));
  if (K.shifttfs != 0.f) {
    if (rs.w < K.shifttfs) umagn = 0;
    else umagn *= (double(rs.w) - double(K.shifttfs)) / K.coeftfs;
  }
  const float sx = float(double(rs.x) * umagn), sy = float(double(rs.y) * umagn), sz = float(double(rs.z) * umagn);
  const float md = K.shiftmaxdist;
  if (K.nn) {  // v5.0: clamped from above only (JSphShifting.cpp:412-414 of the NN solver)
    dx += double(sx < md ? sx : md);
    dy += double(sy < md ? sy : md);
    dz += double(sz < md ? sz : md);
  } else {  // v5.2: |shift| clamped to maxdist with its sign (JSphShifting.cpp:412-414)
    dx += double(fabsf(sx) < md ? sx : (sx >= 0 ? md : -md));
    dy += double(fabsf(sy) < md ? sy : (sy >= 0 ? md : -md));
    dz += double(fabsf(sz) < md ? sz : (sz >= 0 ? md : -md));
  }
}

// Box key of one particle (KerPreSortFull, JCellDivGpuSingle_ker.cu:41-102).
__device__ __forceinline__ unsigned box_key(unsigned rcell, typecode rcode, const DivGrid& g, unsigned dcc) {
  if (rcell == DCELL_DISCARD) return g.boxdiscard;  // slab: stale ghost / particle handed to a neighbour
  const unsigned cx = DcelCellx(dcc, rcell) - unsigned(g.offx()), cy = DcelCelly(dcc, rcell) - unsigned(g.offy()),
                 cz = DcelCellz(dcc, rcell);
  if (rcell != DCELL_OUT && g.split() && (g.axis ? cy >= unsigned(g.ncy) : cx >= unsigned(g.ncx)))
    return g.boxdiscard;  // slab: a migrant handed over beyond this slab's ghost rim (re-partition)
  const unsigned cellsort = cx + cy * unsigned(g.ncx) + cz * g.nsheet;
  const typecode codetype = CodeType(rcode), codeout = CodeSpecial(rcode);
  if (codetype < CODE_TYPE_FLOATING)
    return codeout < CODE_OUTIGNORE
               ? ((cx < unsigned(g.ncx) && cy < unsigned(g.ncy) && cz < unsigned(g.ncz)) ? cellsort : g.boxboundignore)
               : (codeout == CODE_OUTIGNORE ? g.boxboundoutignore : g.boxboundout);
  return codeout <= CODE_OUTIGNORE ? (codeout < CODE_OUTIGNORE ? g.boxfluid + cellsort : g.boxfluidoutignore)
                                   : (codetype == CODE_TYPE_FLOATING ? g.boxboundout : g.boxfluidout);
}

// ---- slab face boxes (the ghost exchange; sph_slab.hip, the incremental divide) ----
// The W cells of a face along the slab axis, from the local axis cell s0, as (type, z, y, x)
// boxes enumerated in box-key order: x-slabs ((type ncz + z) ncy + y) W + (x - s0), y-slabs
// ((type ncz + z) W + (y - s0)) ncx + x.  The sender's face (its first / last owned cells)
// and the receiver's ghost rim number the same global boxes alike.
__host__ __device__ __forceinline__ unsigned face_boxes_per_type(const DivGrid& g, int W) {
  return unsigned(g.ncz) * unsigned(W) * unsigned(g.axis ? g.ncx : g.ncy);
}
// Box key of face box idx.
__device__ __forceinline__ unsigned face_key(const DivGrid& g, int W, unsigned idx, int s0) {
  if (g.axis == 0) {
    const unsigned xrel = idx % unsigned(W);
    unsigned t = idx / unsigned(W);
    const unsigned y = t % unsigned(g.ncy);
    t /= unsigned(g.ncy);
    const unsigned z = t % unsigned(g.ncz), type = t / unsigned(g.ncz);
    return (type ? g.boxfluid : 0u) + unsigned(s0) + xrel + y * unsigned(g.ncx) + z * g.nsheet;
  }
  const unsigned x = idx % unsigned(g.ncx);
  unsigned t = idx / unsigned(g.ncx);
  const unsigned yrel = t % unsigned(W);
  t /= unsigned(W);
  const unsigned z = t % unsigned(g.ncz), type = t / unsigned(g.ncz);
  return (type ? g.boxfluid : 0u) + x + (unsigned(s0) + yrel) * unsigned(g.ncx) + z * g.nsheet;
}
// Face box of a box key (-1: not a cell box of the face's W cells from s0).
__device__ __forceinline__ int face_idx(const DivGrid& g, int W, unsigned key, int s0) {
  unsigned type, cs;
  if (key < g.nct) {
    type = 0u;
    cs = key;
  } else if (key >= g.boxfluid && key < g.boxfluid + g.nct) {
    type = 1u;
    cs = key - g.boxfluid;
  } else {
    return -1;
  }
  const int x = int(cs % unsigned(g.ncx));
  const unsigned r = cs / unsigned(g.ncx);  // z ncy + y
  const int y = int(r % unsigned(g.ncy));
  const unsigned tz = type * unsigned(g.ncz) + r / unsigned(g.ncy);
  if (g.axis == 0) {
    const int xr = x - s0;
    if (xr < 0 || xr >= W) return -1;
    return int((tz * unsigned(g.ncy) + unsigned(y)) * unsigned(W) + unsigned(xr));
  }
  const int yr = y - s0;
  if (yr < 0 || yr >= W) return -1;
  return int((tz * unsigned(W) + unsigned(yr)) * unsigned(g.ncx) + unsigned(x));
}
// Index of the first face box whose key is >= key (the prefix of the face's counts there =
// its entries below key).
__device__ __forceinline__ unsigned face_lower(const DivGrid& g, int W, unsigned key, int s0) {
  const unsigned nfb1 = face_boxes_per_type(g, W);  // face boxes of one type
  unsigned type, cs;
  if (key < g.nct) {
    type = 0u;
    cs = key;
  } else if (key < g.boxfluid) {
    return nfb1;  // BoundIgnore: after every bound face box
  } else if (key < g.boxfluid + g.nct) {
    type = 1u;
    cs = key - g.boxfluid;
  } else {
    return 2u * nfb1;  // out and discard boxes: after every face box
  }
  const int x = int(cs % unsigned(g.ncx));
  const unsigned r = cs / unsigned(g.ncx);  // z ncy + y
  if (g.axis == 0) return type * nfb1 + r * unsigned(W) + unsigned(min(max(x - s0, 0), W));
  const int y = int(r % unsigned(g.ncy)), z = int(r / unsigned(g.ncy));
  const unsigned zb = type * nfb1 + unsigned(z) * unsigned(W) * unsigned(g.ncx);  // the first box of this z
  const int yr = y - s0;
  if (yr < 0) return zb;
  if (yr >= W) return zb + unsigned(W) * unsigned(g.ncx);
  return zb + unsigned(yr) * unsigned(g.ncx) + unsigned(x);
}

struct SlabFaces;  // the ghost exchange after the divide (below)
struct ItemBuild;  // the per-divide item list of the tiled interactions (sph_items.hpp)

// Scratch of the cell sort (DivideGpu).
struct SortScratch {
  unsigned* keys[2] = {nullptr, nullptr};
  unsigned* vals[2] = {nullptr, nullptr};
  unsigned* hist = nullptr;     // [radix * ntiles]
  unsigned* digtot = nullptr;   // [radix]
  unsigned ntiles = 0;
};

constexpr int RS_BS = 256;        // threads per radix block
#ifndef SPH_RS_ITEMS
#define SPH_RS_ITEMS 8
#endif
constexpr int RS_ITEMS = SPH_RS_ITEMS;  // keys per thread per tile
constexpr int RS_TILE = RS_BS * RS_ITEMS;
constexpr int RS_MAXBITS = 11;    // widest digit (2048 buckets)

// ---- divide (JCellDivGpuSingle::Divide + JSphGpuSingle::RunCellDivide) ----
// PreSort: box key per particle (KerPreSortFull, JCellDivGpuSingle_ker.cu:41-102).
// `extra` reserved entries follow the particles (slab ghost slots, launch_ghost_keys): the
// sort covers np + extra keys.
void launch_presort(hipStream_t stm, unsigned cap, const DevScalars* sc, const unsigned* dcell, const typecode* code,
                    DivGrid g, unsigned domcellcode, unsigned* keys, unsigned* vals, unsigned extra = 0);
// Stable LSD radix sort of (keys, vals) for the first sc->ndiv entries (or the first `nfix`
// when given: a count the host knows); result in keys[res]/vals[res].
int launch_radix_sort(hipStream_t stm, unsigned cap, const DevScalars* sc, SortScratch& s, unsigned keybits,
                      unsigned nfix = ~0u);
// begincell by lower-bound search + new counts (KerCalcBeginEndCell, JCellDivGpu_ker.cu:512-546).
void launch_begincell(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* skeys, DivGrid g, unsigned* begincell);
// Gather + poscell + press + VelMax (KerSortDataParticles, JCellDivGpu_ker.cu:553-720; KerUpdatePosCell,
// JSphGpuSimple_ker.cu:41-69; PreInteraction press/VelMax, JSphGpu.cpp:831-870).
// Sorted entries with a value >= vfirst are reserved slots (no particle yet): their sorted
// index goes to apppos[value - appbase] instead.
void launch_gather(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* sortpart, const PartArrays& src,
                   const PartArrays& dst, bool withm1, bool withpre, const KConst& K, const double dom_posmin[3],
                   float4* poscell, float* press, int xoff, int yoff, const float4* phase_eos = nullptr, unsigned vfirst = ~0u,
                   unsigned appbase = 0, unsigned* apppos = nullptr);

constexpr unsigned TSUP_STRIDE = 16;  // u64 entries per super-tile line
// Incremental divide (sph_divide.hip): the stable order of the previous divide merged with
// the particles whose box changed, every divide after the first.  On a slab the exchange
// appended `napp` particles (migrants + ghosts) after the `nold` of the previous divide:
// they are sorted apart (a small radix sort) and placed after the old members of their box.
struct IncDivScratch {
  unsigned* skeys = nullptr;      // [cap] box key of the particle at each index (last divide)
  unsigned* newkey = nullptr;     // [cap] box key of this divide
  unsigned* cw = nullptr;         // [cap] tile-local near / far prefixes (11 bits each) | near, far flags
  unsigned* fidx = nullptr;       // [cap] far-list index of a far mover
  uint2* tagg = nullptr;          // [tiles] (near, far) movers of each tile
  // [tiles / 64] (near << 32 | far) per super tile, each on its own 128-B line (TSUP_STRIDE:
  // device-scope atomics serialise per line), cleared by k_inc_push
  unsigned long long* tsup = nullptr;
  unsigned* tpg = nullptr;        // [tiles] movers before each tile (k_inc_boxes -> k_inc_push)
  unsigned* mkey = nullptr;       // [cap] new keys of the near movers, at tile * INC_TILE + local rank
  uint2* mfar = nullptr;          // [cap] (previous index, new key) of the far movers (appended)
  unsigned* mposnear = nullptr;   // [cap] new positions of the near movers (same slots as mkey)
  unsigned* mposfar = nullptr;    // [cap] new positions of the far movers
  unsigned* stayoff = nullptr;    // [nctt] new index of a stayer = stayoff[key] + i - movers before i
  unsigned* ctr = nullptr;        // [0]: far movers (cleared by k_inc_push)
  // slab: the appended particles [nold, nold + napp): keys / indices for their sort (written
  // by k_inc_classify), the sorted result, and their new positions (k_inc_boxes)
  unsigned* akin = nullptr;
  unsigned* avin = nullptr;
  const unsigned* akeys = nullptr;
  const unsigned* avals = nullptr;
  unsigned* apppos = nullptr;     // [cap]
  unsigned nold = 0, napp = 0;
  // slab: reserved ghost slots after the old members of their boxes, like the appended
  // particles: nvl of the left face, nvr of the right, counted per face box (vpre: the
  // prefixes of the received counts, SlabFaces order, vW ghost columns), positions
  // apppos[napp + e]; no particle data until launch_ghost_scatter
  const unsigned* vpre[2] = {nullptr, nullptr};
  int vW = 0;
  unsigned nvl = 0, nvr = 0;
  unsigned nb1 = 0, nb2 = 0, gen = 0;
  // SPH_INC_DBG: 8 phase timestamps of the divide kernels (printf); 16 / 32 force the
  // global-memory paths of the tile prefixes / far arrivals (tests)
  int dbg = 0;
};
constexpr unsigned INC_TILE_SIZE = 1024;  // particles per classify tile (sph_divide.hip INC_TILE)
// Stable sort of <= SMALLSORT_MAX (key, index) pairs in one block (the migrants of a divide).
constexpr unsigned SMALLSORT_MAX = 4096;
void launch_small_sort(hipStream_t stm, const unsigned* kin, const unsigned* vin, unsigned n, unsigned* kout,
                       unsigned* vout);
unsigned inc_blocks_classify(unsigned cap);
unsigned inc_blocks_boxes(unsigned nctt);
void launch_divide_inc(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& src, const PartArrays& dst,
                       bool withm1, bool withpre, const KConst& K, const double dom_posmin[3], float4* poscell,
                       float* press, DivGrid g, const unsigned* begincell_old, unsigned* begincell_new,
                       IncDivScratch& s, SortScratch& srt, unsigned keybits, const float4* phase_eos = nullptr,
                       const SlabFaces* faces = nullptr, unsigned ngl = 0, unsigned ngr = 0,
                       const ItemBuild* items = nullptr, bool classified = false);

// ---- interaction (cusph::Interaction_Forces, JSphGpu_ker.cu:788-885) ----
// With floating bodies (ftmassp != nullptr: particle mass per body, `code` of the
// sorted particles) the kernel reads the p2 codes (JSphCpu.cpp:692-703).
void launch_interaction(hipStream_t stm, unsigned cap, DevScalars* sc, const float4* poscell, const float4* velrhop,
                        const float* press, const unsigned* begincell, DivGrid g, const KConst& K, float4* arace,
                        const typecode* code = nullptr, const float* ftmassp = nullptr);
// Bound p1 only (grid over the bound capacity) — used beside the tiled fluid kernel.
void launch_interaction_bound(hipStream_t stm, unsigned npbcap, DevScalars* sc, const float4* poscell,
                              const float4* velrhop, const unsigned* begincell, DivGrid g, const KConst& K,
                              float4* arace);
// Work counters of the persistent tiled kernels (qctr): per XCD group g an item queue of its
// fluid-row items (line g) and one of its bound-row items (line QCTR_BQ + g), each on its own
// 128-B line (device-scope atomics serialize per line; line 8 is unused).
constexpr int QSTRIDE = 32;
constexpr int QCTR_BQ = 9;
// Line 17 holds the list's item counts {all, bound, first item, chunk log2} (k_items_place;
// ItemGroups reads them), so one counter block describes one item list.
constexpr size_t QCTR_QUEUE_BYTES = 17 * QSTRIDE * sizeof(unsigned);  // what a re-run zeroes
constexpr int QCTR_WORDS = 18 * QSTRIDE;
constexpr int QCTR_NITEMS = 17 * QSTRIDE;
// A list's counter blocks come in QCTR_COPIES copies (QCTR_WORDS apart), all set up by the
// item build, so that the interactions on one item list (NN's force and viscous passes; an
// interaction without a divide before it, e.g. sph_download_interaction) each start on
// fresh queues without a memset launch.
constexpr int QCTR_COPIES = 2;
constexpr size_t QCTR_BYTES = size_t(QCTR_COPIES) * QCTR_WORDS * sizeof(unsigned);
// Tiled fluid interaction (sph_interaction_tiled.hip); its per-divide item list is built
// by sph_items.hpp (launch_items, or the incremental divide's push launch + launch_items_write).
// With floating bodies (ftmassp != nullptr) the staged p2 records carry their mass ratio
// and kind (the FT instantiation; one more float2 of LDS per record).
void launch_fluid_tiled(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                        const float4* poscell, const float4* velrhop, const float* press, const unsigned* begincell,
                        DivGrid g, const KConst& K, float4* arace, const typecode* code = nullptr,
                        const float* ftmassp = nullptr, unsigned reserve = 0);
// mDBC boundary correction (sph_mdbc.hip; JSphCpu.cpp:1020-1187): density of every
// boundary particle p1 < npbok with a normal extrapolated from its ghost node; press
// refreshed.  `normal` is indexed by idp; list[npbcap] + nlist: scratch of the
// wet-particle list.
// With floating normals (UseNormalsFt, JSphCpu.cpp:1199) the floating particles of ftridp[nft]
// (owned, by idp - CaseNpb) are corrected too.
void launch_mdbc(hipStream_t stm, unsigned npbcap, const DevScalars* sc, const PartArrays& cur, float* press,
                 const float4* normal, const unsigned* begincell, DivGrid g, const KConst& K,
                 const double dom_posmin[3], float threshold, unsigned* list, unsigned* nlist, void* sums,
                 const unsigned* ftridp = nullptr, unsigned nft = 0);
constexpr size_t MDBC_SUM_BYTES = 152;  // sizeof(MdbcSum): 16 doubles + 5 floats + index
// Slabs: (idp, rho, press) of the owned face-column boundary particles after mDBC, for
// the neighbours' ghost copies (slot 0 holds the count).  Capacities capl / capr (records,
// count slot included) are the exchange's face sizes + 1: both sides of a face derive the
// same size, and it bounds the face's boundary particles, so no record is ever dropped.
struct MdbcFaceRec {
  unsigned idp;
  float rho, press;
};
// floating: the floating particles (floating normals) are sent and mapped too (cap = the
// particle capacity; else the boundary part only).
void launch_mdbc_face_pack(hipStream_t stm, unsigned cap, const DevScalars* sc, const PartArrays& a,
                           const float* press, const KConst& K, const DivGrid& g, MdbcFaceRec* sl, MdbcFaceRec* sr,
                           unsigned capl, unsigned capr, unsigned* bidx, unsigned nbidx, bool floating = false);
// A record whose idp this slab does not hold as a boundary particle this step (bidx
// stale or missing) raises ERR_HALO (fatal: every slab halts at this step) instead of writing.
void launch_mdbc_face_apply(hipStream_t stm, DevScalars* sc, const MdbcFaceRec* rl, const MdbcFaceRec* rr,
                            unsigned capl, unsigned capr, const unsigned* bidx, unsigned nbidx, const unsigned* idp, float4* velrhop,
                            float* press);
// NN multiphase interaction (sph_nn.hip; JSphCpu_NN_FDA.cpp of the v5.0 solver): all items
// (fluid and bound p1) of the tiled item list; phases = the device phase table (2 float4
// per phase, sph_device.hpp); shiftpos written when `shift` (the corrector's interaction).
void launch_nn_tiled(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                     const float4* poscell, const float4* velrhop, const float* press, const typecode* code,
                     const unsigned* begincell, DivGrid g, const KConst& K, const float4* phases, float4* arace,
                     float4* shiftpos, bool shift, float* viscoeta, float4* tau, const float* ftmassp = nullptr);
// Single-phase interaction with Laminar+SPS viscosity and/or shifting (sph_ext.hip):
// arace, shiftpos (when shiftstore), the new SPS tau into taunew (Laminar+SPS; `tau` holds
// the previous interaction's), ViscDtMax / AceMax.
void launch_fluid_ext(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                      const float4* poscell, const float4* velrhop, const float* press, const typecode* code,
                      const float* ftmassp, const float4* tau, const unsigned* begincell, DivGrid g, const KConst& K,
                      float4* arace, float4* shiftpos, float4* taunew, bool shiftstore);
// NN with SPH velocity gradients, second pass: the Morris / constitutive-equation /
// artificial viscous force of every fluid p1 from the first pass's effective viscosities or
// stress tensors (JSphCpu_NN_SPH.cpp:228-446), added onto arace; AceMax.
void launch_nn_visc(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                    const float4* poscell, const float4* velrhop, const typecode* code, const float* viscoeta,
                    const float4* tau, const unsigned* begincell, DivGrid g, const KConst& K, const float4* phases,
                    float4* arace, const float* ftmassp = nullptr);
// Slabs, SPH velocity gradients: the first pass's effective viscosity (Laminar) or stress
// tensor (ConstEq) of the owned face-column fluid particles, for the neighbours' ghosts
// (the second pass reads them for every p2).  Records {idp, v[7]}; count in slot 0 of
// each buffer.  idxmap: idp -> local index of every held particle (apply side).
struct NNFaceRec {
  unsigned idp;
  float v[7];
};
void launch_nn_face_pack(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, const KConst& K,
                         const DivGrid& g, const float* viscoeta, const float4* tau, NNFaceRec* sl, NNFaceRec* sr,
                         unsigned capl, unsigned capr, unsigned* idxmap, unsigned nidx);
void launch_nn_face_apply(hipStream_t stm, DevScalars* sc, const NNFaceRec* rl, const NNFaceRec* rr, unsigned capl,
                          unsigned capr, const unsigned* idxmap, unsigned nidx, const unsigned* idp, float* viscoeta,
                          float4* tau, bool withtau);
// Pair counters (JDsPips).
void launch_count_pairs(hipStream_t stm, unsigned cap, const DevScalars* sc, const float4* poscell,
                        const unsigned* begincell, DivGrid g, const KConst& K, unsigned long long* out6);

// ---- dt and time integration ----
enum DtMode { DT_VERLET = 0, DT_SYM_PRE = 1, DT_SYM_COR = 2, DT_PEEK = 3 };
// `folded` (slab mode): the three maxima already folded and max-reduced over ranks
// (launch_fold_maxima + SlabTransport::allreduce_max_u32); nullptr = fold the slots here.
void launch_dt(hipStream_t stm, DevScalars* sc, const KConst& K, double cfl, double dtmin, double cs0, int mode,
               double* dttrace, unsigned tracecap, const unsigned* folded = nullptr);
// sc->visco = Visco at the current TimeStep (ViscoTime table, else the case's).
void launch_visco_init(hipStream_t stm, DevScalars* sc, const KConst& K);
// folded[5]: VelMax^2, AceMax^2, ViscDtMax, ViscEtaDtMax, this slab's fatal error flags
void launch_fold_maxima(hipStream_t stm, DevScalars* sc, unsigned* folded, bool clear);
// Update kernels skip slab ghosts (local cell along the slab axis outside [g.sown0, g.sown1)) and mark
// them DCELL_DISCARD for the next divide.
// shiftpos (nullptr: no shifting): the interaction's shifting sums, turned into the
// displacement of JSphShifting::RunCpu inside the update.
// cls (not null): the incremental divide's classification rides on the update (sph_incdiv.hpp);
// pk (not null, with cls): the slab exchange's count pass too (sph_slabpack.hpp)
struct PackArgs;
void launch_verlet(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, bool euler, const float4* arace,
                   PartArrays a, DivGrid g, const float4* shiftpos = nullptr, const IncDivScratch* cls = nullptr,
                   const PackArgs* pk = nullptr);
void launch_sym_pre(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a,
                    DivGrid g, const IncDivScratch* cls = nullptr, const PackArgs* pk = nullptr);
void launch_sym_cor(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a,
                    DivGrid g, const float4* shiftpos = nullptr, const IncDivScratch* cls = nullptr,
                    const PackArgs* pk = nullptr);

// ---- moving boundaries and floating bodies (sph_bodies.hip) ----
constexpr int MOT_MAXOBJ = 32, MOT_MAXACT = 4, MOT_MAXAXIS = 64;
struct MotMov {     // one movement of the program (JMotionMov*), units as SphMotionMov
  int type, nextidx, prev, fields;
  int ax, rax;      // its axis and (circular) reference point in MotionDev::axis, or -1
  int dfirst, dn;   // file movements: rows [dfirst, dfirst + dn) of the table rows
  double time;      // duration (< 0: flash)
  double v[3], v2[3], phase[3];
  double ang, ang2, ang3;
};
struct MotEvt {     // JMotionEvent
  int obj, mov;
  double start, finish;
};
struct MotAct {     // JMotionMovActive
  int mov, del, flash, dfindex;
  double start, finish, eventfinish;
  double vel[3], velang, phase[3], phaseuni;
  double dflast[3], dflastang;  // the file movements' last position / angle
};
struct M4d {        // JMatrix4d, row major a[4*r+c]
  double a[16];
};
struct MPos {       // JMotionPos: accumulated motion of one object in one step
  int simple, pad;
  double s[3];
  M4d m;
};
struct MotObj {     // JMotionObj run state; nodes depth first (a parent before its children)
  int active, moving, na, parent, ref, pad;
  MotAct act[MOT_MAXACT];
  MPos modpos;      // its motion of the current step (read by its children)
};
struct MotAxis {    // JMotionAxis: moved with the parent object; a circular reference point is
  double p1[3], p2[3];  // moved by its movement
  int obj, pad;
};
struct MotOut {     // JMotionListData of one object for the step: 0 none, 1 linear, 2 matrix
  int type, pad;
  double mov[3], vel[3];
  double m[12];
};
struct MotionDev {
  int nobj, nref, eventnext, objsactive, overflow, naxis;
  MotObj obj[MOT_MAXOBJ];
  MotOut out[MOT_MAXOBJ];  // by ref
  MotAxis axis[MOT_MAXAXIS];
};
// Floating body (StFloatingData + StFtoForces/StFtoForcesRes), device resident.
// One JLinearValue table of a floating body on the device: its rows [first, first + n) of
// the table buffer and the lookup state the reference keeps between calls (FindTime's
// Position / PositionNext for the TimeStep of the last call; pos < 0: none yet).
struct FtTabDesc {
  int first, n;
  int pos, posnext;
  double t;
};

struct FtBody {
  unsigned begin, count;   // floating-particle index range (idp - CaseNpb)
  unsigned constraints;    // FTCON_* bits (DualSphDef.h:445-453)
  int skip;                // TimeStep < FtPause in this call
  float mass, massp, ftpause, pad;
  float inertia[9];
  double center[3];
  float angles[3], fvel[3], fomega[3], facelin[3], faceang[3];
  // per call
  float face[3], fomegaace[3], fvelres[3], fomegares[3];
  double fcenterres[3];
  // mDBC on the body (floating normals): the rotation of its normals this step (the 3x3 part
  // of Move(center) Rotate(dang) Move(-center0), JSphCpuSingle.cpp:988-999), row major
  double nrot[9];
};
// k_motion over [sc->tstep0, +sc->last_dt) (or [t0, t0+dt) when t0 >= 0: restart
// catch-up, no particle update), then the boundary particles.
void launch_motion(hipStream_t stm, unsigned npbcap, DevScalars* sc, const KConst& K, MotionDev* md,
                   const MotMov* movs, const MotEvt* evts, const double* data, const PartArrays& a, float4* normal,
                   const DivGrid& g);
void launch_motion_advance(hipStream_t stm, DevScalars* sc, MotionDev* md, const MotMov* movs, const MotEvt* evts,
                           const double* data, double t0, double dt);
// Owned floating particles only (slab ghosts are summed by their owner).
void launch_ft_ridp(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, unsigned casenpb,
                    unsigned nftp, unsigned* ftridp, const KConst& K, const DivGrid& g);
constexpr int FT_NBLK = 32;  // partial-sum blocks per body; part = float[nbodies][FT_NBLK][6]
// RunFloating in two halves: partial force sums (a slab adds them over the slabs in
// between), then body integration + particle update + body state.
void launch_ft_partial(hipStream_t stm, DevScalars* sc, const FtBody* bodies, int nbodies, const unsigned* ftridp,
                       const float4* arace, const PartArrays& a, float* part);
// fttab/ftdesc: the bodies' imposed-velocity / external-force tables (SPH_FTTAB_*), or nullptr.
// normal (mDBC on floating bodies, by idp): turned with the body after a full step.
void launch_ft_body(hipStream_t stm, DevScalars* sc, const KConst& K, FtBody* bodies, int nbodies,
                    const unsigned* ftridp, unsigned nftp, const PartArrays& a, bool predictor, const float* part,
                    const double4* fttab = nullptr, FtTabDesc* ftdesc = nullptr, float4* normal = nullptr);

// ---- slab decomposition (sph_slab.hip) ----
// A particle MIGRATING to a neighbour: its full state, 112 B.  A boundary particle also
// carries its mDBC normal (kept by idp, turned with moving objects by its owner), so the
// new owner continues with the turned normal (JSphCpu.cpp:1724-1728).
struct SlabRec {
  double2 posxy;
  double posz;
  unsigned idp, dcell;
  float4 velrhop;
  float4 vr2;  // velrhopm1 (Verlet) or velrhoppre (Symplectic, inside a step)
  double2 posxypre;
  double poszpre;
  unsigned short code, flags;
  unsigned pad;
  float4 normal;  // mDBC normal of a boundary particle (idp < nbound), else 0
  float4 taua, taub;  // Laminar+SPS: the migrant's SPS stress tensor (PartArrays::tau)
};
// A GHOST copy for a neighbour: what a neighbour of the interaction needs, 40 B.  The
// position travels as the float offset from its (global) cell origin, i.e. exactly the
// poscell the owner computes; the receiver rebuilds the double position as origin +
// offset (exact: < 31 significant bits), so its poscell is bit-identical.
struct SlabGhost {
  float rx, ry, rz;
  unsigned dcell;
  float4 velrhop;
  unsigned idp;
  unsigned short code, pad;
};
constexpr int PK_BS = 256, PK_ITEMS = 4, PK_TILE = PK_BS * PK_ITEMS;
// Bytes of the pack kernels' tile counters for a capacity of n particles: [4][ntiles] u32.
// per tile: the four record streams, the particles staying owned, the ghosts per face (k_pack_count)
constexpr size_t PK_TILECNT_BYTES(size_t n) { return 7 * sizeof(unsigned) * ((n + PK_TILE - 1) / PK_TILE); }
// Device counters of one exchange: [0] ghosts, [1] migrants, per neighbour.
struct SlabCounts {
  unsigned long long sendl[2], sendr[2];  // records for the left / right neighbour
  unsigned long long recvl[2], recvr[2];  // records from the left / right neighbour
  unsigned np;                            // particles before the exchange (sc->np)
  unsigned nkeep;                         // particles staying owned (not migrating, not dropped)
  unsigned ghosts[2];                     // ghosts counted per face box for the left / right neighbour
};
struct SlabSendBufs {
  SlabGhost* gl;
  SlabGhost* gr;
  SlabRec* ml;
  SlabRec* mr;
  unsigned long long gcap, mcap;  // records beyond the capacity are counted, not written
};
// The pack's arguments (sph_slab.hip; the count pass also in the slab update, sph_slabpack.hpp).
struct PackArgs {
  PartArrays a;
  DivGrid g;
  unsigned dcc;
  double posminx, posminy, posminz, scelld;
  int has_left, has_right, withm1, withpre;
  unsigned* tilecnt;  // [4][ntiles]: ghost L, ghost R, migrant L, migrant R
  unsigned ntiles;
  SlabCounts* cnt;
  SlabSendBufs b;
  const float4* normal;  // mDBC normals by idp (nullptr without mDBC)
  unsigned nbound;
  unsigned* fcnt[2];     // ghost counts per face box (the exchange after the divide), or nullptr
  int W;
};
PackArgs make_pack_args(unsigned cap, const PartArrays& a, DivGrid g, const KConst& K, const double dom_posmin[3],
                        bool has_left, bool has_right, bool withm1, bool withpre, unsigned* tilecnt, SlabCounts* cnt,
                        SlabSendBufs bufs, const float4* normal, unsigned nbound, const SlabFaces* faces);
// Classify every particle after an update (stable order) and write the records for
// the two neighbours: tile counts -> scan -> scatter, four streams (ghost/migrant x
// left/right).  has_left/has_right: the neighbour exists.
// faces != nullptr (the ghost exchange after the divide): ghosts are counted per face box
// into faces->msg[0/1] (zeroed here) instead of written as records.
void launch_slab_pack(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, DivGrid g, const KConst& K,
                      const double dom_posmin[3], bool has_left, bool has_right, bool withm1, bool withpre,
                      unsigned* tilecnt, SlabCounts* cnt, SlabSendBufs bufs, const float4* normal = nullptr,
                      unsigned nbound = 0, const SlabFaces* faces = nullptr, bool counted = false);
// ---- the ghost exchange after the divide (sph_slab.hip, sph_divide.hip) ----
// Before the divide a slab sends each neighbour only the NUMBER of its ghosts per face box
// (with the migrants); the receiver's divide reserves their slots (they follow the old
// members of their box, as appended particles do) and the ghost records travel after the
// divide, packed from the sender's sorted arrays in box order, while the interaction of
// the items that reach no ghost column runs.  Face boxes: the boxes of the W face columns,
// in key order — type (bound, fluid) major, then z, y, x: idx = ((type ncz + z) ncy + y) W
// + xrel, nfb = 2 ncz ncy W (the sender's face columns and the receiver's ghost columns are
// the same global columns).  A face message is {u64 ghosts, u64 migrants} + u32 count[nfb].
constexpr unsigned FMSG_HDR = 4;  // u32 words of a face message's header
struct SlabFaces {
  unsigned* msg[4];  // send left, send right, receive left, receive right: [FMSG_HDR + nfb]
  unsigned* pre[4];  // exclusive prefixes of their counts: [nfb + 1]
  unsigned nfb = 0;
  int W = 0;
};
// (The pack writes the send messages' counts and headers.)  After the message exchange:
// cnt->recvl / recvr from the received headers; then the prefixes of all four messages'
// counts (off the host wait's path).
void launch_face_scan(hipStream_t stm, const SlabFaces& f, SlabCounts* cnt, bool has_left, bool has_right);
// The divide's virtual keys of the ngl + ngr reserved ghost slots (left face first):
// keys[e] = the receiver's box key, vals[e] = vbase + e.
void launch_ghost_keys(hipStream_t stm, const SlabFaces& f, DivGrid g, unsigned ngl, unsigned ngr, unsigned* keys,
                       unsigned* vals, unsigned vbase);
// After the sender's divide: the ghost records of both faces from the sorted arrays, in face
// box order (the old members of each box: its first count[idx] particles).
void launch_ghost_pack(hipStream_t stm, DevScalars* sc, const SlabFaces& f, DivGrid g, const unsigned* begincell,
                       const PartArrays& a, const float4* poscell, SlabSendBufs b, unsigned ngl, unsigned ngr);
// The receiver: record e -> its reserved slot apppos[e] (position, poscell, EOS pressure as
// the gather forms them; key for the next divide into skeys when given).
void launch_ghost_scatter(hipStream_t stm, DevScalars* sc, const SlabGhost* rec, unsigned ng, const unsigned* apppos,
                          const PartArrays& dst, const KConst& K, const double dom_posmin[3], float4* poscell,
                          float* press, DivGrid g, unsigned* skeys, const float4* phase_eos = nullptr);
// out[i] = (((0 + g[0][i]) + g[1][i]) + ...) over nranks rows of n floats (rank order).
void launch_rank_ordered_sum(hipStream_t stm, const float* gathered, int n, int nranks, float* out);
// The same over the ranks' own buffers (in-process slabs of one GPU, LocalTransport), and the
// max of n uint32 values over them.
struct RankPtrs {
  static constexpr int MAXR = 16;
  const void* p[MAXR];
};
void launch_rank_ordered_sum(hipStream_t stm, const RankPtrs& rp, int n, int nranks, float* out);
void launch_rank_max_u32(hipStream_t stm, const RankPtrs& rp, int n, int nranks, unsigned* out);
// Two device-to-device copies in one launch (the in-process transport's two faces, on one GPU).
void launch_copy_pair(hipStream_t stm, void* d0, const void* s0, size_t n0, void* d1, const void* s1, size_t n1);
// Owned particles per GLOBAL x-column: counts[c] fluid (incl. floating), counts[ncxg + c]
// boundary (the re-partition's weights), as floats (exact integers).
void launch_column_counts(hipStream_t stm, unsigned cap, const DevScalars* sc, const PartArrays& a, DivGrid g,
                          const KConst& K, int ncxg, float* counts);
// Append nm received migrants at [np, np+nm) and ng ghosts after them; set sc->np, sc->nown.
void launch_slab_unpack(hipStream_t stm, DevScalars* sc, const SlabRec* mig, unsigned nm, const SlabGhost* gh,
                        unsigned ng, unsigned np, const PartArrays& a, const KConst& K, const double dom_posmin[3],
                        bool withm1, bool withpre, SlabCounts* cnt, float4* normal = nullptr, unsigned nbound = 0,
                        const SlabFaces* faces = nullptr, bool has_left = false, bool has_right = false);

}  // namespace sphx
