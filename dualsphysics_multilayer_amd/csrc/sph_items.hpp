// sph_items.hpp — the per-divide item list of the tiled interactions (k_fluid_tiled,
// k_fluid_ext, k_nn_tiled), built from the new begincell in two launches over the (y,z)
// rows: a COUNT pass (one wave per row walks its items, counts them per list and stages them
// in the row's slot of `ricap` items, rowitems), then a PLACE pass (each block sums the counts
// below its rows, scans its own, and copies the staged items to their offsets; a row whose
// items overflowed its slot is walked again).  The count pass is a device function so that
// it can run in the blocks the incremental divide's push launch adds after its own
// (sph_divide.hip): the push is HBM-bound, the walk latency-bound, and the two need only the
// new begincell.  cfg2 1M (rocprof): a one-block scan + a second walk took 4.8 + 14.4 us, the
// place pass takes DESIGN.md §4's figure.  (A last-block ticket in place of a scan launch cost
// more than the launch: one device-scope atomic per count block on one line, ~4000 of them at
// 1M, serialise across the XCDs — the divide phase went 0.085 -> 0.105 ms.)
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
  int x[6];  // ranges [x[2k], x[2k+1]) of p1 along the slab axis (empty when equal): list A =
             // range 0 (and 1, 2 with one list), list B = ranges 1, 2.  x-slabs: column ranges
             // of every row; y-slabs: the rows whose y is in a range, each over all its columns
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
// range of each list.  WRITE = false counts them (counts[list][row]) and stages them,
// true writes the items of list `onelist` at item offset `outoff`.
template <bool WRITE>
__device__ __forceinline__ void items_row(const ItemBuild& b, unsigned r, unsigned* pre, unsigned short* nzfrom,
                                          int onelist = -1, unsigned outoff = 0) {
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
  // the column range [rx0, rx1) of range k in this row (y-slabs: the whole row or nothing)
  auto range_x = [&](int k, int& rx0, int& rx1) {
    if (g.axis == 0) {
      rx0 = xr.x[2 * k];
      rx1 = xr.x[2 * k + 1];
    } else {
      const bool in = int(y) >= xr.x[2 * k] && int(y) < xr.x[2 * k + 1];
      rx0 = 0;
      rx1 = in ? ncx : 0;
    }
  };
  {  // a row without particles in its ranges (most rows of the air above the water and of
     // the boundary): no items, no staging
    int xlo = ncx, xhi = 0;
    for (int k = 0; k < 3; k++) {
      int rx0, rx1;
      range_x(k, rx0, rx1);
      if (rx0 < rx1) {
        xlo = min(xlo, rx0);
        xhi = max(xhi, rx1);
      }
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
  for (int list = onelist < 0 ? 0 : onelist; list < (onelist < 0 ? xr.nl : onelist + 1); list++) {
    uint4* out = WRITE ? b.items + outoff : nullptr;  // (WRITE: one list, at its offset)
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
      int xbeg, xend;  // uniform over the wave
      range_x(rg, xbeg, xend);
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

// The PLACE pass (k_items_place: scan + write in one launch).  Block k takes the (list, row)
// entries [i0, i1) of the flattened counts: the items below i0 are one block reduction over
// the counts before it (every block reads its own prefix of the raw counts: no scan kernel,
// no cross-block ordering), its own entries an in-block exclusive scan, then its threads copy
// the staged items to their offsets (a row whose items overflowed its slot is walked again).  One more block writes each list's counts {all, bound, first item} into its
// counter blocks (QCTR_COPIES copies) and zeroes their work queues for the next interactions.
constexpr int IP_BS = 512;        // threads of a place block (8 waves)
constexpr int IP_MAXROWS = 1024;  // entries per place block (2 per thread)
inline unsigned items_place_blocks(unsigned n) {
  const unsigned want = std::min(128u, std::max(1u, n / 64u));
  return std::max(want, (n + IP_MAXROWS - 1) / IP_MAXROWS) + 1u;  // + the counts block
}

__device__ __forceinline__ unsigned block_sum(unsigned v, unsigned* s_w) {
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  unsigned t = 0;
  for (unsigned q = 0; q < blockDim.x / 64; q++) t += s_w[q];
  return t;
}

// This thread's part of the sum of counts[lo, hi): 16-B loads, several in flight (a strided
// scalar loop waits one memory latency per element it reads).
__device__ __forceinline__ unsigned partial_sum(const unsigned* __restrict__ counts, unsigned lo, unsigned hi) {
  if (lo >= hi) return 0u;
  unsigned s = 0;
  const unsigned a = min((lo + 3u) & ~3u, hi), nv = (hi - a) / 4u, t = a + 4u * nv;
  if (threadIdx.x < a - lo) s += counts[lo + threadIdx.x];
  if (threadIdx.x < hi - t) s += counts[t + threadIdx.x];
  const uint4* __restrict__ v = reinterpret_cast<const uint4*>(counts + a);
#pragma unroll 4
  for (unsigned k = threadIdx.x; k < nv; k += blockDim.x) {
    const uint4 x = v[k];
    s += (x.x + x.y) + (x.z + x.w);
  }
  return s;
}

__device__ __forceinline__ void items_place_block(const ItemBuild& b, unsigned char* smem) {
  __shared__ unsigned s_w[IP_BS / 64], s_off[IP_MAXROWS], s_cnt[IP_MAXROWS], s_tot;
  const unsigned* __restrict__ counts = b.counts;
  const unsigned nrows2 = b.nrows2, nrows = nrows2 / 2, nl = unsigned(b.xr.nl), n = nl * nrows2;
  const unsigned nb = gridDim.x - 1;  // the last block: the lists' counts
  const unsigned per = (n + nb - 1) / nb, i0 = blockIdx.x * per, i1 = min(i0 + per, n);
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (blockIdx.x == nb) {  // the lists' counts and fresh work queues
    // items below nrows, nrows2, nrows2 + nrows, n (the segments' sums, loads of all four
    // issued before the first block reduction, then prefixes)
    const unsigned p0 = partial_sum(counts, 0u, nrows), p1 = partial_sum(counts, nrows, nrows2);
    const unsigned p2 = partial_sum(counts, nrows2, min(nrows2 + nrows, n));
    const unsigned p3 = partial_sum(counts, min(nrows2 + nrows, n), n);
    const unsigned m0 = block_sum(p0, s_w);
    const unsigned m1 = m0 + block_sum(p1, s_w);
    const unsigned m2 = m1 + block_sum(p2, s_w);
    const unsigned m3 = m2 + block_sum(p3, s_w);
    if (threadIdx.x < 16 * QCTR_COPIES) {  // the fluid and bound queues of the 8 groups
      const unsigned k = threadIdx.x & 15;
      const unsigned q = (threadIdx.x >> 4) * QCTR_WORDS + (k < 8 ? k : QCTR_BQ + k - 8) * QSTRIDE;
      b.qa[q] = 0u;
      if (nl == 2) b.qb[q] = 0u;
    }
    if (threadIdx.x < QCTR_COPIES) {
      const unsigned na = nl == 2 ? m1 : m3, c = threadIdx.x * QCTR_WORDS + QCTR_NITEMS;
      // the deal's chunk (ItemDeal): 64 items for the lists of the large cases, else 16
      const unsigned sh = m3 >= ITEM_CHUNK_BIG_N ? ITEM_CHUNK_BIG_LOG2 : ITEM_CHUNK_LOG2;
      b.qa[c] = na;
      b.qa[c + 1] = na - m0;  // the bound rows' items: the list's tail (ItemGroups)
      b.qa[c + 2] = 0u;
      b.qa[c + 3] = sh;
      if (nl == 2) {
        b.qb[c] = m3 - na;
        b.qb[c + 1] = m3 - m2;
        b.qb[c + 2] = na;  // the second list follows the first in the item array
        b.qb[c + 3] = sh;
      }
    }
    return;
  }
  if (i0 >= n) return;
  const unsigned below = block_sum(partial_sum(counts, 0u, i0), s_w);
  // own entries: two per thread, an exclusive scan
  const unsigned e0 = i0 + 2 * threadIdx.x;
  const unsigned v0 = e0 < i1 ? counts[e0] : 0u, v1 = e0 + 1 < i1 ? counts[e0 + 1] : 0u;
  unsigned inc = v0 + v1;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned t = __shfl_up(inc, off, 64);
    if (lane >= unsigned(off)) inc += t;
  }
  __syncthreads();
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  unsigned run = below + inc - v0 - v1;
  for (unsigned q = 0; q < w; q++) run += s_w[q];
  if (e0 < i1) {
    s_off[e0 - i0] = run;
    s_cnt[e0 - i0] = v0;
  }
  if (e0 + 1 < i1) {
    s_off[e0 + 1 - i0] = run + v0;
    s_cnt[e0 + 1 - i0] = v1;
  }
  if (threadIdx.x == blockDim.x - 1) s_tot = run + v0 + v1 - below;  // the block's items
  __syncthreads();
  // The block's items are contiguous in the list: thread t copies items t, t + IP_BS, ... from
  // their rows' slots (the row by a binary search of the offsets), all loads independent.
  const unsigned nr = i1 - i0, tot = s_tot;
  for (unsigned k = threadIdx.x; k < tot; k += blockDim.x) {
    const unsigned o = below + k;
    unsigned lo = 0, hi = nr - 1;  // the last row whose offset is <= o (empty rows before it share it)
    while (lo < hi) {
      const unsigned mid = (lo + hi + 1) >> 1;
      if (s_off[mid] <= o) lo = mid;
      else hi = mid - 1;
    }
    if (s_cnt[lo] <= b.ricap) b.items[o] = b.rowitems[size_t(i0 + lo) * b.ricap + (o - s_off[lo])];
  }
  // a row whose items overflowed its slot: walked again by one wave
  const unsigned L = b.rowlds();
  unsigned* pre = reinterpret_cast<unsigned*>(smem) + w * L;
  unsigned short* nz = reinterpret_cast<unsigned short*>(smem + (IP_BS / 64) * L * sizeof(unsigned)) + w * L;
  for (unsigned j = w; j < nr; j += IP_BS / 64)
    if (s_cnt[j] > b.ricap) {
      const unsigned i = i0 + j, list = i / nrows2;
      items_row<true>(b, i - list * nrows2, pre, nz, int(list), s_off[j]);
    }
}

// Block `blk` of the count pass (IR_WAVES rows; dynamic LDS `smem` of b.lds bytes).
__device__ __forceinline__ void items_count_block(const ItemBuild& b, unsigned blk, unsigned char* smem) {
  const unsigned L = b.rowlds(), w = threadIdx.x >> 6;
  unsigned* pre = reinterpret_cast<unsigned*>(smem) + w * L;
  unsigned short* nz = reinterpret_cast<unsigned short*>(smem + IR_WAVES * L * sizeof(unsigned)) + w * L;
  const unsigned r = blk * IR_WAVES + w;
  if (r < b.nrows2) items_row<false>(b, r, pre, nz);
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
void launch_items(hipStream_t stm, const ItemBuild& b);        // count, place
void launch_items_place(hipStream_t stm, const ItemBuild& b);  // after a count done elsewhere

}  // namespace sphx
