// sph_kernels.hpp — host-side launchers of the HIP kernels (one per hot-path phase).
//
// All launchers are asynchronous on `stm`, never allocate and never synchronise,
// so a whole step can be captured into a hipGraph.  Grids are sized from the
// particle capacity; the live counts (np, npb, npbok) are read on the device from
// DevScalars, so no host round trip is needed between phases.
#pragma once
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
};

// Scratch of the cell sort (DivideGpu).
struct SortScratch {
  unsigned* keys[2] = {nullptr, nullptr};
  unsigned* vals[2] = {nullptr, nullptr};
  unsigned* hist = nullptr;     // [radix * ntiles]
  unsigned* digtot = nullptr;   // [radix]
  unsigned ntiles = 0;
};

constexpr int RS_BS = 256;        // threads per radix block
constexpr int RS_ITEMS = 16;      // keys per thread per tile
constexpr int RS_TILE = RS_BS * RS_ITEMS;
constexpr int RS_MAXBITS = 11;    // widest digit (2048 buckets)

// ---- divide (JCellDivGpuSingle::Divide + JSphGpuSingle::RunCellDivide) ----
// PreSort: box key per particle (KerPreSortFull, JCellDivGpuSingle_ker.cu:41-102).
void launch_presort(hipStream_t stm, unsigned cap, const DevScalars* sc, const unsigned* dcell, const typecode* code,
                    DivGrid g, unsigned domcellcode, unsigned* keys, unsigned* vals);
// Stable LSD radix sort of (keys, vals) for the first sc->np entries; result in keys[res]/vals[res].
int launch_radix_sort(hipStream_t stm, unsigned cap, const DevScalars* sc, SortScratch& s, unsigned keybits);
// begincell by lower-bound search + new counts (KerCalcBeginEndCell, JCellDivGpu_ker.cu:512-546).
void launch_begincell(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* skeys, DivGrid g, unsigned* begincell);
// Gather + poscell + press + VelMax (KerSortDataParticles, JCellDivGpu_ker.cu:553-720; KerUpdatePosCell,
// JSphGpuSimple_ker.cu:41-69; PreInteraction press/VelMax, JSphGpu.cpp:831-870).
void launch_gather(hipStream_t stm, unsigned cap, DevScalars* sc, const unsigned* sortpart, const PartArrays& src,
                   const PartArrays& dst, bool withm1, bool withpre, const KConst& K, const double dom_posmin[3],
                   float4* poscell, float* press);

// ---- interaction (cusph::Interaction_Forces, JSphGpu_ker.cu:788-885) ----
void launch_interaction(hipStream_t stm, unsigned cap, DevScalars* sc, const float4* poscell, const float4* velrhop,
                        const float* press, const unsigned* begincell, DivGrid g, const KConst& K, float4* arace);
// Bound p1 only (grid over the bound capacity) — used beside the tiled fluid kernel.
void launch_interaction_bound(hipStream_t stm, unsigned npbcap, DevScalars* sc, const float4* poscell,
                              const float4* velrhop, const unsigned* begincell, DivGrid g, const KConst& K,
                              float4* arace);
// Tiled fluid interaction (sph_interaction_tiled.hip) and its per-divide item list.
void launch_items(hipStream_t stm, DevScalars* sc, const unsigned* begincell, DivGrid g, unsigned* rowtmp,
                  uint4* items, unsigned* qctr);
void launch_fluid_tiled(hipStream_t stm, unsigned nblocks, DevScalars* sc, const uint4* items, unsigned* qctr,
                        const float4* poscell, const float4* velrhop, const float* press, const unsigned* begincell,
                        DivGrid g, const KConst& K, float4* arace);
// Pair counters (JDsPips).
void launch_count_pairs(hipStream_t stm, unsigned cap, const DevScalars* sc, const float4* poscell,
                        const unsigned* begincell, DivGrid g, const KConst& K, unsigned long long* out6);

// ---- dt and time integration ----
enum DtMode { DT_VERLET = 0, DT_SYM_PRE = 1, DT_SYM_COR = 2, DT_PEEK = 3 };
void launch_dt(hipStream_t stm, DevScalars* sc, const KConst& K, double cfl, double dtmin, double cs0, int mode,
               double* dttrace, unsigned tracecap);
void launch_verlet(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, bool euler, const float4* arace,
                   PartArrays a);
void launch_sym_pre(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a);
void launch_sym_cor(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a);

}  // namespace sphx
