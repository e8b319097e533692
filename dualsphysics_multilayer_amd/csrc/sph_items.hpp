// sph_items.hpp — the per-divide item list of the tiled interactions (k_fluid_tiled,
// k_fluid_ext, k_nn_tiled), built from the new begincell in two passes over the (y,z)
// rows: a COUNT pass (items per row and list), a one-block SCAN of the counts into item
// offsets, then a WRITE pass (the same walk, writing the items at the offsets).  The count
// pass is a device function so that it can run in the blocks the incremental divide's push
// launch adds after its own (sph_divide.hip): the push is HBM-bound, the walk latency-bound,
// and the two need only the new begincell.  (A last-block ticket in place of the scan
// launch cost more than the launch: one device-scope atomic per count block on one line,
// ~4000 of them at 1M, serialise across the XCDs — the divide phase went 0.085 -> 0.105 ms.)
//
// The count pass also stages each row's items in a slot of `ricap` items per (list, row)
// (rowitems); the write pass then copies the staged items to their offsets (one wave per
// row, a coalesced copy) and walks again only a row whose items overflowed its slot.  cfg2
// 1M: the write pass 14.4 -> see DESIGN.md §4.
//
// Rows [0,nrows) are fluid rows (fluid p1), rows [nrows,2*nrows) bound rows (bound p1,
// DBC).  An item is a run of <= TB consecutive particles of one row, cut earlier only where
// it would span more than tmaxc x-cells; items may start and end inside a cell.  One wave per
// row copies the row's cell begin offsets to LDS, then lane 0 walks the items; the count and
// write passes run the same walk, so the list is deterministic and in spatial (z, y, x)
// order, fluid items first.
#pragma once
#include <algorithm>

#include "sph_kernels.hpp"
#include "sph_tiled.hpp"

namespace sphx {

constexpr int IR_WAVES = 4;            // rows per block: one wave each (blocks of 256 threads)
constexpr int ROWCELLS_LDS = 1024;     // longest row (cells) walked from LDS; longer: global memory

struct ItemRanges {
  int x[6];  // column ranges [x[2k], x[2k+1]) of p1 (empty when equal): list A = range 0 (and
             // 1, 2 with one list), list B = ranges 1, 2
  int nl;    // lists: 1 or 2
};

// One item build: what both passes and the scan read.
struct ItemBuild {
  const unsigned* bc;   // the new begincell
  DivGrid g;
  int tmaxc;            // max x-cells per item (TMAXCELLS / TMAXCELLS_HALF)
  ItemRanges xr;
  unsigned* counts;     // [nl][nrows2] row counts, scanned in place into offsets (+ the total)
  uint4* items;
  uint4* rowitems;      // [nl][nrows2][ricap] the count pass's items of each row
  unsigned ricap;       // staged items per (list, row)
  unsigned* qa;         // counter block of list A (its item counts + work queues)
  unsigned* qb;         // list B (nl == 2)
  unsigned nrows2;      // 2 ncy ncz
  unsigned nblocks;     // blocks of one pass (IR_WAVES rows each)
  unsigned lds;         // dynamic LDS bytes of a pass block
  __host__ __device__ unsigned rowlds() const { return unsigned(min(g.ncx, ROWCELLS_LDS)) + 1u; }
};

// One wave walks row r of one kind (fluid or bound p1): its cell begin offsets to LDS
// (pre / nzfrom: this wave's rowlds() entries), then lane 0 emits the items of each column
// range of each list.  WRITE = false counts them (counts[list][row]), true writes them at the
// scanned offsets.
template <bool WRITE>
__device__ __forceinline__ void items_row(const ItemBuild& b, unsigned r, unsigned* pre, unsigned short* nzfrom) {
  const DivGrid& g = b.g;
  const ItemRanges& xr = b.xr;
  const unsigned nrows = unsigned(g.ncy) * unsigned(g.ncz), nrows2 = 2u * nrows;
  const unsigned lane = threadIdx.x & 63;
  const bool bound = r >= nrows;
  const unsigned rr = bound ? r - nrows : r;
  const unsigned y = rr % unsigned(g.ncy), z = rr / unsigned(g.ncy);
  const unsigned rowbase = (bound ? 0u : g.boxfluid) + z * g.nsheet + y * unsigned(g.ncx);
  const int ncx = g.ncx;
  const unsigned* __restrict__ bc = b.bc;
  {  // a row without particles in its ranges (most rows of the air above the water and of
     // the boundary): no items, no staging
    int xlo = ncx, xhi = 0;
    for (int k = 0; k < 3; k++)
      if (xr.x[2 * k] < xr.x[2 * k + 1]) {
        xlo = min(xlo, xr.x[2 * k]);
        xhi = max(xhi, xr.x[2 * k + 1]);
      }
    if (xlo >= xhi || bc[rowbase + xlo] == bc[rowbase + xhi]) {
      if (!WRITE && lane == 0)
        for (int list = 0; list < xr.nl; list++) b.counts[list * nrows2 + r] = 0u;
      return;
    }
  }
  const bool lds = ncx <= ROWCELLS_LDS;
  if (lds) {
    for (int x = int(lane); x <= ncx; x += 64) pre[x] = bc[rowbase + x];
    __builtin_amdgcn_wave_barrier();
  }
  for (int list = 0; list < xr.nl; list++) {
    uint4* out = WRITE ? b.items + b.counts[list * nrows2 + r] : nullptr;
    unsigned nitems = 0;
    uint4* stage = WRITE ? nullptr : b.rowitems + size_t(list * nrows2 + r) * b.ricap;
    auto emit = [&](int a, int e, unsigned p, unsigned q) {
      const uint4 it = make_uint4((y | (z << 16)) | (bound ? ITEM_BOUND : 0u), unsigned(a) | (unsigned(e) << 16), p, q);
      if (WRITE)
        out[nitems] = it;
      else if (nitems < b.ricap)
        stage[nitems] = it;
      nitems++;
    };
    // p1 only in owned columns (slab ghosts are neighbours, never p1); each range walked on
    // its own, so no item crosses from one to the next
    for (int rg = (list ? 1 : 0); rg < (xr.nl == 2 && list == 0 ? 1 : 3); rg++) {
      const int xbeg = xr.x[2 * rg], xend = xr.x[2 * rg + 1];  // uniform over the wave
      if (xbeg >= xend) continue;
      if (!lds) {  // very long rows: the same walk on global memory, cell by cell
        if (lane == 0) {
          auto PRE = [&](int x) -> unsigned { return bc[rowbase + x]; };
          unsigned p = PRE(xbeg);
          const unsigned pend = PRE(xend);
          int c = xbeg;
          while (p < pend) {
            while (PRE(c + 1) <= p) c++;
            const unsigned q = min(min(p + unsigned(TB), pend), PRE(min(c + b.tmaxc, xend)));
            int e = c;
            while (PRE(e + 1) < q) e++;
            emit(c, e, p, q);
            p = q;
            c = e;
          }
        }
        continue;
      }
      // first non-empty cell of the range at or after x: lane-local blocks, then a wave suffix-min
      const int per = (ncx + 63) / 64, x0 = int(lane) * per, x1 = min(x0 + per, ncx);
      int nz = xend;
      for (int x = x1 - 1; x >= x0; x--) {
        if (x >= xbeg && x < xend && pre[x + 1] > pre[x]) nz = x;
        nzfrom[x] = (unsigned short)nz;
      }
      int suf = nz;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_down(suf, off, 64);
        if (int(lane) + off < 64) suf = min(suf, v);
      }
      const int later = __shfl_down(suf, 1, 64);
      const int carry = int(lane) < 63 ? later : xend;
      for (int x = x0; x < x1; x++)
        if (int(nzfrom[x]) == xend) nzfrom[x] = (unsigned short)carry;
      if (lane == 63) nzfrom[ncx] = (unsigned short)xend;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        // Walk the items: the cell holding p is known (c), the cell holding q-1 is at most
        // TMAXCELLS-1 cells further, an item ending at a cell end jumps to the next non-empty.
        // The five offsets pre[c..c+4] of an item are independent LDS reads (one latency);
        // the cell holding q-1 is c + #{k = 1..3 : pre[c+k] <= q-1}.
        static_assert(TMAXCELLS == 4, "the walk reads pre[c..c+4]");
        const unsigned pend = pre[xend];
        int c = nzfrom[xbeg];
        unsigned p = c < xend ? pre[c] : pend;
        if (b.tmaxc != TMAXCELLS) {  // CellMode=half: longer items, the cell holding q-1 by a short scan
          while (p < pend) {
            const unsigned q = min(min(p + unsigned(TB), pend), pre[min(c + b.tmaxc, xend)]);
            int e = c;
            while (pre[e + 1] <= q - 1) e++;
            emit(c, e, p, q);
            p = q;
            c = pre[e + 1] == q ? int(nzfrom[e + 1]) : e;
          }
        } else {
          while (p < pend) {
            const unsigned p1 = pre[min(c + 1, xend)], p2 = pre[min(c + 2, xend)], p3 = pre[min(c + 3, xend)];
            const unsigned p4 = pre[min(c + 4, xend)];
            const unsigned q = min(min(p + unsigned(TB), pend), p4);
            const int e = c + int(p1 <= q - 1) + int(p2 <= q - 1) + int(p3 <= q - 1);
            emit(c, e, p, q);
            p = q;
            const unsigned pe1 = e + 1 - c == 1 ? p1 : e + 1 - c == 2 ? p2 : e + 1 - c == 3 ? p3 : p4;
            c = pe1 == q ? int(nzfrom[e + 1]) : e;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // nzfrom is rebuilt for the next range
    }
    if (!WRITE && lane == 0) b.counts[list * nrows2 + r] = nitems;
  }
}

// Exclusive scan of the row counts of the lists by ONE block (blockDim a multiple of 64,
// <= 1024), in place -> item offsets; each list's counts {all, bound, first item} into its
// counter block (qctr[QCTR_NITEMS...]) and its per-XCD work queues zeroed for the next
// interaction.  s: >= blockDim/64 + 4 words of LDS.  (Chunks of contiguous counts per
// thread: a few thousand rows at 1M, ~16k at 10M.)
__device__ __forceinline__ void items_scan(const ItemBuild& b, unsigned* s) {
  unsigned* __restrict__ counts = b.counts;
  const unsigned nrows2 = b.nrows2, nrows = nrows2 / 2, nl = unsigned(b.xr.nl), n = nl * nrows2;
  const unsigned nt = blockDim.x, nw = nt / 64, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned* wsum = s;
  unsigned* mark = s + nw;  // offsets where list A's bound rows, list B and its bound rows begin
  if (threadIdx.x < 8 * QCTR_COPIES) {  // the interactions' item queues (every copy) start over
    const unsigned q = (threadIdx.x >> 3) * QCTR_WORDS + (threadIdx.x & 7) * QSTRIDE;
    b.qa[q] = 0u;
    if (nl == 2) b.qb[q] = 0u;
  }
  // thread t scans the contiguous chunk [t per, (t+1) per)
  const unsigned per = (n + nt - 1) / nt, i0 = threadIdx.x * per, i1 = min(i0 + per, n);
  unsigned sum = 0;
  for (unsigned i = i0; i < i1; i++) sum += counts[i];
  unsigned inc = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned v = __shfl_up(inc, off, 64);
    if (lane >= unsigned(off)) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  unsigned run = inc - sum;
  for (unsigned q = 0; q < w; q++) run += wsum[q];
  for (unsigned i = i0; i < i1; i++) {
    if (i == nrows) mark[0] = run;
    if (i == nrows2) mark[1] = run;
    if (i == nrows2 + nrows) mark[2] = run;
    const unsigned v = counts[i];
    counts[i] = run;
    run += v;
  }
  if (threadIdx.x == nt - 1) {
    mark[3] = run;  // the total
    counts[n] = run;  // so that every row's count is the next offset minus its own
  }
  __syncthreads();
  if (threadIdx.x < QCTR_COPIES) {
    const unsigned tot = mark[3], na = nl == 2 ? mark[1] : tot, c = threadIdx.x * QCTR_WORDS + QCTR_NITEMS;
    b.qa[c] = na;
    b.qa[c + 1] = na - mark[0];  // the bound rows' items: the list's tail (ItemGroups)
    b.qa[c + 2] = 0u;
    if (nl == 2) {
      b.qb[c] = tot - na;
      b.qb[c + 1] = tot - mark[2];
      b.qb[c + 2] = na;  // the second list follows the first in the item array
    }
  }
}

// The write pass of row r: its staged items copied to their offsets by the wave, or, when
// a list's items overflowed the row's slot, the walk again.
__device__ __forceinline__ void items_copy_row(const ItemBuild& b, unsigned r, unsigned* pre, unsigned short* nz) {
  const unsigned lane = threadIdx.x & 63, nl = unsigned(b.xr.nl);
  unsigned off[2], cnt[2];
  bool fits = true;
  for (unsigned list = 0; list < nl; list++) {
    const unsigned i = list * b.nrows2 + r;
    off[list] = b.counts[i];
    cnt[list] = b.counts[i + 1] - off[list];
    fits &= cnt[list] <= b.ricap;
  }
  if (!fits) {
    items_row<true>(b, r, pre, nz);
    return;
  }
  for (unsigned list = 0; list < nl; list++) {
    const uint4* __restrict__ src = b.rowitems + size_t(list * b.nrows2 + r) * b.ricap;
    for (unsigned k = lane; k < cnt[list]; k += 64) b.items[off[list] + k] = src[k];
  }
}

// Block `blk` of a pass (IR_WAVES rows; dynamic LDS `smem` of b.lds bytes).
template <bool WRITE>
__device__ __forceinline__ void items_pass_block(const ItemBuild& b, unsigned blk, unsigned char* smem) {
  const unsigned L = b.rowlds(), w = threadIdx.x >> 6;
  unsigned* pre = reinterpret_cast<unsigned*>(smem) + w * L;
  unsigned short* nz = reinterpret_cast<unsigned short*>(smem + IR_WAVES * L * sizeof(unsigned)) + w * L;
  const unsigned r = blk * IR_WAVES + w;
  if (r >= b.nrows2) return;
  if (WRITE)
    items_copy_row(b, r, pre, nz);
  else
    items_row<false>(b, r, pre, nz);
}

// Host side (sph_interaction_tiled.hip).  scelldiv 1 (CellMode=full): items of <= 4 cells;
// 2 (half): <= TMAXCELLS_HALF half-cells.  p1 in the local columns [xr[0], xr[1]),
// [xr[2], xr[3]), [xr[4], xr[5]), each range's items on their own (nullptr: the owned
// columns).  With qctr2: two lists in `items`, the first of range 0 (counter block qctr),
// the second of ranges 1 and 2 after it (qctr2).  rowtmp holds 2 x 2 ncy ncz counts + 1;
// rowitems 2 x 2 ncy ncz x ricap items.
inline size_t ITEMS_ROWTMP(int ncy, int ncz) { return 4 * size_t(ncy) * size_t(ncz) + 1; }
// Staged items per row: a row of ncx full cells holds ~ncx/4 items of 4 cells or, dense,
// one item per 128 particles (~40 per cell of 2h) — ~ncx/3; longer rows walk again.
inline unsigned ITEMS_RICAP(int ncx) { return unsigned(std::min(128, ncx / 2 + 8)); }
ItemBuild make_item_build(const unsigned* begincell, DivGrid g, unsigned* rowtmp, uint4* items, unsigned* qctr,
                          int scelldiv, const int* xr, unsigned* qctr2, uint4* rowitems, unsigned ricap);
void launch_items(hipStream_t stm, const ItemBuild& b);             // count, scan, write
void launch_items_scan_write(hipStream_t stm, const ItemBuild& b);  // after a count done elsewhere

}  // namespace sphx
