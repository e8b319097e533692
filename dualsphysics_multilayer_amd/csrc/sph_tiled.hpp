// sph_tiled.hpp — pieces shared by the LDS-tiled interaction kernels (the single-phase
// k_fluid_tiled of sph_interaction_tiled.hip and the NN multiphase k_nn_tiled of
// sph_nn.hip): block shape and LDS capacities, fast f32 intrinsics, the item flag, the
// expanded-form candidate test and the lane order of an item's particles.
#pragma once
#include <cfloat>
#include <mutex>
#include <unordered_map>

#include "sph_kernels.hpp"

namespace sphx {

constexpr int TB = 128;        // threads per block = max p1 per item (2 waves)
#ifndef SPH_TCAP
#define SPH_TCAP 504
#endif
// staged neighbour records per segment.  504 puts the block at 20.3 KB of LDS, the most
// that keeps 8 blocks = 4 waves per SIMD.  Measured at 1M: 0.806 ms vs 0.838 at 416 (a
// mirrored row pair fits one segment for 94% of the units instead of 81%); 0.936 at 580
// (7 blocks/CU), 1.02 at 672 (6 blocks/CU).  The position records (sA) are followed by
// the velrhop records (sB) in ONE LDS array in every tiled kernel, so the candidate
// test's last group of 32 (up to 31 records past a window ending at the capacity) reads
// inside that array; its bits are masked off.
constexpr int TCAP = SPH_TCAP;
// With floating bodies a record is 48 B (the third part a float4): 416 records keep the
// block at <= 20 KB of LDS, i.e. the same 8 blocks (4 waves/SIMD) per CU.
#ifndef SPH_TCAP_FT
#define SPH_TCAP_FT 416
#endif
template <bool FT> struct TcapT { static constexpr int v = TCAP; };
template <> struct TcapT<true> { static constexpr int v = SPH_TCAP_FT; };
constexpr int TMAXCELLS = 4;   // max x-cells per item (CellMode=full: cells of 2h)
// CellMode=half (cells of h, +-2-cell stencil): an item spans <= 32 half-cells (at the
// lattice density, ~5.2 particles per half-cell, TB particles take ~25), so its staged
// rows [a-2, b+2] hold ~150 records and a mirrored row pair fits one TCAP segment.
// Measured at 1M (interaction ms): 12 cells 1.13, 16: 0.95, 20: 0.87 with units of two
// mirrored pairs; 24: 0.84, 32: 0.77 with units of one pair (SPH_HALF_LPU=1).
#ifndef SPH_TMAXCELLS_HALF
#define SPH_TMAXCELLS_HALF 32
#endif
constexpr int TMAXCELLS_HALF = SPH_TMAXCELLS_HALF;

// Staged position records read whole: the drain uses x, y, z only, and a 12-B LDS read
// (ds_read_b96) is serviced in 8 lane groups of 8 = 8 LDS cycles per wave-instruction,
// against 4 for the 16-B ds_read_b128 (MI355X_MICROARCH.md §LDS).  An empty asm at the end
// of the drain iteration takes the records' .w as operands, so the compiler keeps the full
// 16-B loads without waiting for them earlier than their other uses.
__device__ __forceinline__ void keep_w(const float4& a, const float4& b) {
  asm volatile("" ::"v"(a.w), "v"(b.w));
}

__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt_(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }

constexpr unsigned ITEM_BOUND = 0x80000000u;  // flag in item.x: p1 are boundary particles

// Candidate test with the expanded form |p-A|^2 = |p|^2 + |A|^2 - 2 p.A (3 FMAs + 1
// compare per candidate on one ds_read_b128) against a threshold inflated by 1e-4 (the
// expanded form rounds to ~1e-6 relative); the body recomputes |p-A|^2 exactly and applies
// the reference's test, so no pair is lost or added.
// 32 candidates b[0..31] -> bits (bit k = candidate k): the compare lands in VCC and
// v_addc_co_u32 shifts it in (bits = 2 bits + vcc), two VALU per candidate besides the 3
// FMAs instead of compare + select + or.  Candidates in descending order so candidate k
// ends at bit k.  (VCC only: no memory access.)
__device__ __forceinline__ unsigned test32(const float4* __restrict__ b, float px2, float py2, float pz2,
                                           float thr) {
  unsigned bits = 0u;
#pragma unroll 8
  for (int ji = 31; ji >= 0; ji--) {
    const float4 A = b[ji];
    const float q = fmaf(px2, A.x, fmaf(py2, A.y, fmaf(pz2, A.z, A.w)));
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(bits) : "v"(thr), "v"(q) : "vcc");
  }
  return bits;
}

// One window of n (<= 32 * NG) staged records from sA + s0 in groups of 32 -> words w[NG]
// (a group past the window's end reads up to 31 records beyond it, inside the staging
// array, and its bits are masked off).  n <= 0 gives empty words.
template <int NG>
__device__ __forceinline__ void test_groups(const float4* __restrict__ sA, int s0, int n, float px2, float py2,
                                            float pz2, float thr, unsigned (&w)[NG]) {
  const float4* __restrict__ b = sA + s0;
#pragma unroll
  for (int g = 0; g < NG; g++) w[g] = 0u;
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int left = n - g * 32;
    if (left <= 0) break;
    w[g] = test32(b + g * 32, px2, py2, pz2, thr) & (left >= 32 ? ~0u : ((1u << left) - 1u));
  }
}

// A window of <= 64 candidates -> one 64-bit mask (the short 5-cell windows of CellMode=half).
__device__ __forceinline__ unsigned long long test64(const float4* __restrict__ sA, int s0, int n, float px2,
                                                     float py2, float pz2, float thr) {
  unsigned w[2];
  test_groups<2>(sA, s0, n, px2, py2, pz2, thr, w);
  return (static_cast<unsigned long long>(w[1]) << 32) | w[0];
}

// A window of <= 128 candidates -> two 64-bit masks.
__device__ __forceinline__ void test128(const float4* __restrict__ sA, int s0, int n, float px2, float py2,
                                        float pz2, float thr, unsigned long long& m0, unsigned long long& m1) {
  unsigned w[4];
  test_groups<4>(sA, s0, n, px2, py2, pz2, thr, w);
  m0 = (static_cast<unsigned long long>(w[1]) << 32) | w[0];
  m1 = (static_cast<unsigned long long>(w[3]) << 32) | w[2];
}

// Which p1 of the item each lane computes.  A lane's drain loops run as long as the
// busiest lane of its wave, and a particle's candidate counts per mirrored row pair
// depend mostly on how far it sits from its cell's centre in y and z; so the n (<= TB)
// particles are split between the two waves by that distance (|dy| + |dz| below or
// above half a cell, stable ballot ranks): simulated on the 1M lattice, drain
// utilisation 0.68 -> 0.74.  Results do not depend on the assignment: every p1 is
// summed by one lane over the same candidates in the same order.
__device__ __forceinline__ unsigned lane_order(const float4* __restrict__ poscell, unsigned first, unsigned n,
                                               float hs, unsigned char* s_perm, unsigned* s_nwave) {
  const unsigned me = threadIdx.x, wv = me >> 6, ln = me & 63u;
  const bool valid = me < n;
  bool low = false;
  if (valid) {
    const float4 pc = poscell[first + me];
    low = fabsf(pc.y - hs) + fabsf(pc.z - hs) < hs;
  }
  const unsigned long long bl = __ballot(low), bh = __ballot(valid && !low);
  const unsigned long long lt = (1ull << ln) - 1ull;
  if (ln == 0) {
    s_nwave[wv] = unsigned(__popcll(bl));
    s_nwave[2 + wv] = unsigned(__popcll(bh));
  }
  __syncthreads();
  const unsigned nl0 = s_nwave[0], nl = nl0 + s_nwave[1], nh0 = s_nwave[2];
  if (valid) {
    const unsigned pos = low ? (wv ? nl0 : 0u) + unsigned(__popcll(bl & lt))
                             : nl + (wv ? nh0 : 0u) + unsigned(__popcll(bh & lt));
    s_perm[pos] = (unsigned char)me;
  }
  __syncthreads();
  return valid ? s_perm[me] : me;
}

// The per-XCD-group work of a tiled interaction: the item list is [fluid-row items | bound-row
// items] in spatial order; group g takes every 8th chunk of SPH_ITEM_CHUNK fluid items from
// chunk g, then likewise of the bound items (most of them cheap: no fluid in reach, or
// continuity only), its own first item statically (k_fluid_tiled / k_nn_tiled).  The groups'
// loads are then alike and every group ends on short items, so the blocks' last items
// finish close together.  Measured (three alternating A/B runs each): contiguous eighths of
// the whole list (the bound items all in the last groups) -> eighths of the fluid, then of
// the bound items: cfg5 1.502 -> 1.446 ms, cfg2 0.671 -> 0.665; -> round-robin: cfg2
// 0.666 -> 0.638 ms, cfg5 unchanged.  The XCD-local spatial contiguity of a group's items
// was worth less than the balance (neighbour rows are MALL hits either way).  Dealt in
// chunks of 16 consecutive items (chunks of 1, 4, 16: same time) the L2-miss traffic of
// the cfg2 interaction is 228 MB per launch instead of 397 MB.  Lists of >= ITEM_CHUNK_BIG_N
// items (cfg3's 10M, cfg4's 4M) are dealt in chunks of 64: a group's neighbour rows stay in
// its XCD's L2 longer (cfg3: 3.9 -> 2.2 GB of HBM traffic per launch at the same time,
// DESIGN.md §9), while a list of a few thousand items keeps enough chunks per group.  The
// item build writes the chunk's log2 beside the list's counts (QCTR_NITEMS + 3).
constexpr unsigned ITEM_CHUNK_LOG2 = 4, ITEM_CHUNK_BIG_LOG2 = 6, ITEM_CHUNK_BIG_N = 32768;
// Items of one kind (fluid or bound) dealt to the 8 groups round-robin in chunks of 2^sh.
struct ItemDeal {
  unsigned lo, n, sh;  // the kind's list range [lo, lo + n), chunk log2
  __device__ __forceinline__ unsigned count(unsigned g) const {
    const unsigned CH = 1u << sh;
    const unsigned nch = (n + CH - 1u) >> sh;
    if (g >= nch) return 0u;
    unsigned c = ((nch - g + 7u) / 8u) << sh;
    if ((nch - 1u) % 8u == g) c -= (nch << sh) - n;  // the kind's last chunk is short
    return c;
  }
  __device__ __forceinline__ unsigned item(unsigned g, unsigned c) const {
    return lo + ((g + 8u * (c >> sh)) << sh) + (c & ((1u << sh) - 1u));
  }
};
struct ItemGroups {
  ItemDeal f, b;  // the fluid-row and bound-row items
  // the list's counts {all, bound, first item, chunk log2}, written by k_items_place beside
  // the work queues
  __device__ __forceinline__ explicit ItemGroups(const unsigned* qctr) {
    const unsigned n = qctr[QCTR_NITEMS];
    const unsigned nb = min(qctr[QCTR_NITEMS + 1], n), nf = n - nb, lo = qctr[QCTR_NITEMS + 2];
    const unsigned sh = min(qctr[QCTR_NITEMS + 3], 10u);
    f = {lo, nf, sh};
    b = {lo + nf, nb, sh};
  }
};

// The items of a block, claimed in two phases: the fluid-row items of its own group g, then
// of the groups g+1, ..., g+7 (work stealing), and only then the bound-row items in the same
// group order.  So the fluid work (~100 us per item at cfg2) of the whole launch is claimed
// before any block takes a bound-row item (mostly cheap: no fluid in reach, or continuity
// only), and the last items of the launch are bound-row ones wherever they can be.  (One
// queue per group over [fluid | bound] let a block that had drained its group steal a heavy
// fluid item late: cfg2 blocks ended over ~60 us, 9 % of the block slots idle.)  A block's
// first fluid item of its own group is static (no start-up burst of ~256 same-line atomics
// per counter); a group known to be exhausted costs no atomic (counters only grow).
// FLUID_ONLY: the bound-row items are not claimed (NN's viscous pass).
constexpr unsigned ITEM_NONE = 0xffffffffu;
template <bool FLUID_ONLY = false>
struct ItemCursor {
  ItemGroups IG;
  unsigned* qctr;
  unsigned grp, ph = 0, q = 0;
  bool first = true;
  __device__ __forceinline__ explicit ItemCursor(unsigned* qc) : IG(qc), qctr(qc), grp(blockIdx.x & 7u) {}
  // the next item of this block (block-uniform; ITEM_NONE at the end).  s_item: LDS word.
  __device__ __forceinline__ unsigned next(unsigned* s_item) {
    for (;;) {
      if (q == 8u) {
        if (FLUID_ONLY || ph) return ITEM_NONE;
        ph = 1u;
        q = 0u;
      }
      const unsigned xg = (grp + q) & 7u;
      const ItemDeal& d = ph ? IG.b : IG.f;
      const unsigned n = d.count(xg);
      const unsigned nst = ph ? 0u : (gridDim.x - xg + 7u) / 8u;  // the group's static items
      unsigned* ctr = &qctr[(ph ? QCTR_BQ + xg : xg) * QSTRIDE];
      if (threadIdx.x == 0)
        *s_item = first ? (blockIdx.x >> 3)
                  : (nst + __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n)
                      ? n
                      : nst + atomicAdd(ctr, 1u);
      first = false;
      __syncthreads();
      const unsigned c = *s_item;
      __syncthreads();
      if (c < n) return d.item(xg, c);
      q++;
    }
  }
};

// Grid of a persistent tiled kernel: no more blocks than can be resident at once.  A block
// that is not resident at the start begins only when a resident one exits — after the queues
// ran dry — and then still runs its static first item (ItemGroups): at cfg3 (DDT1, 129 VGPRs,
// 3 waves per SIMD = 6 blocks per CU) 512 of 2048 blocks started 5.7 ms into a 5.8 ms launch,
// and 26 % of the launch's block slots idled.  The occupancy of each kernel on the current
// device is looked up once.  `reserve` block slots are left free (the ghost overlap's
// interior launch, so that the transfer and scatter kernels start at once): the cap by
// residency comes first, then the reserve is taken off it (at least one block stays).
inline unsigned fit_grid(const void* kernel, unsigned want, int threads = TB, unsigned reserve = 0) {
  static std::mutex m;
  static std::unordered_map<unsigned long long, unsigned> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const unsigned long long key = reinterpret_cast<unsigned long long>(kernel) ^ (unsigned long long)(dev) << 56;
  std::lock_guard<std::mutex> lk(m);
  auto it = cache.find(key);
  if (it == cache.end()) {
    int perc = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perc, kernel, threads, 0) != hipSuccess || perc <= 0) perc = 1;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 1;
    it = cache.emplace(key, unsigned(perc) * unsigned(ncu)).first;
  }
  const unsigned cap = it->second > reserve ? it->second - reserve : 1u;
  return want < cap ? want : cap;
}

// i-th of the 12 "lower" rows of the 5x5 CellMode=half stencil (dz < 0, or dz = 0 and
// dy < 0); the other 12 are their point mirrors, the 25th the item's own row.
__device__ __forceinline__ void half_row(int i, int& dy, int& dz) {
  if (i < 10) {
    dz = -2 + i / 5;
    dy = -2 + i % 5;
  } else {
    dz = 0;
    dy = i - 12;
  }
}

// Item geometry shared by the passes of one p1.
struct RowCtx {
  int cy, cz;     // the item's cell row
  int xa, xb;     // x-cell range staged for the item
  int lxa, lxb;   // this lane's own 3-cell x range
  int xo;         // x origin of item-relative positions
  bool act;       // lane holds a p1
  unsigned p1;    // the lane's p1 (Symmetry: its own image is not a neighbour)
};

}  // namespace sphx
