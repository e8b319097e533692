// sph_step.hip — dt control and time integration (Verlet, Symplectic) on CDNA4.
//
// dt (JSphCpu::DtVariable, JSphCpu.cpp:1614-1639; GPU JSphGpu.cpp:984-1013) is
// computed ON THE DEVICE by one wave from the max-reduced VelMax, AceMax and
// ViscDtMax, so the step needs none of the reference's blocking DtoH copies.
// Update kernels follow JSphCpu.cpp:1240-1606 (double intermediates, float storage,
// UpdatePos out-of-map / MovLimit / RhopOut exclusion) — GPU twins
// KerComputeStepVerlet / KerComputeStepSymplecticPre/Cor / KerComputeStepPos
// (JSphGpuSimple_ker.cu:129-450, JSphGpu_ker.cu:320-378,1598-1690).
#include <cfloat>

#include "sph_kernels.hpp"
#include "sph_incdiv.hpp"
#include "sph_slabpack.hpp"

namespace sphx {

// One wave folds the reduction slots (max of non-negative floats as uint bits):
// m[0] VelMax^2, m[1] AceMax^2, m[2] ViscDtMax, m[3] ViscEtaDtMax (NN).
__device__ __forceinline__ void fold_slots(DevScalars* __restrict__ sc, bool clear, unsigned m[4]) {
  const unsigned l = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; k++) m[k] = sc->red[k][l];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < 4; k++) m[k] = max(m[k], (unsigned)__shfl_xor((int)m[k], off, 64));
  if (clear)
#pragma unroll
    for (int k = 0; k < 4; k++) sc->red[k][l] = 0u;
}

// Slab mode: fold the local slots into folded[0..3] for the max-allreduce over ranks
// (the reference's single-domain CalcVelMaxOmp/ComputeAceMaxOmp/ViscDtMax reductions
// span the whole domain, so the slabs must agree on the same maxima).
__global__ void k_fold(DevScalars* __restrict__ sc, unsigned* __restrict__ folded, int clear) {
  unsigned m[4];
  fold_slots(sc, clear != 0, m);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 4; k++) folded[k] = m[k];
    // a fatal error of this slab (e.g. ERR_BOUNDOUT from its divide) rides the same max
    // all-reduce, so every slab halts at the same step, as the one reference domain does
    folded[4] = sc->error_flags & ERR_FATAL;
  }
}

void launch_fold_maxima(hipStream_t stm, DevScalars* sc, unsigned* folded, bool clear) {
  hipLaunchKernelGGL(k_fold, dim3(1), dim3(64), 0, stm, sc, folded, int(clear));
}

__global__ void k_dt(DevScalars* __restrict__ sc, KConst K, double cfl, double dtmin, double cs0, int mode,
                     double* __restrict__ dttrace, unsigned tracecap, const unsigned* __restrict__ folded) {
  const unsigned l = threadIdx.x;
  unsigned m[4];
  if (folded) {
    for (int k = 0; k < 4; k++) m[k] = folded[k];
    if (l == 0) sc->error_flags |= folded[4];
  } else {
    fold_slots(sc, mode != DT_PEEK, m);
  }
  if (l != 0) return;
  const float velmaxf = sqrtf(__uint_as_float(m[0]));  // CalcVelMaxOmp returns float sqrt
  const double velmax = double(velmaxf);
  const double acemax = sqrt(double(__uint_as_float(m[1])));
  const float viscdt = __uint_as_float(m[2]);
  const float visceta = __uint_as_float(m[3]);
  sc->last_velmax = velmaxf;
  sc->last_acemax = float(acemax);
  sc->last_viscdt = viscdt;
  sc->last_visceta = visceta;
  if (mode == DT_PEEK) return;
  if (halted(sc)) return;  // an earlier fatal error: the run no longer advances
  const double kh = double(K.kernelh);
  const double dt1 = (acemax ? sqrt(kh / acemax) : DBL_MAX);
  const double dt2 = kh / (fmax(cs0, velmax * 10.) + kh * double(viscdt));
  // NN: viscous time step h^2/(ViscEtaDtMax*RelaxationDt), float products as the v5.0
  // solver forms them (JSphCpu.cpp:1687 of src_mphase/DSPH_v5.0_NNewtonian)
  const double dt3 = (K.nn ? double(K.kernelh * K.kernelh) / double(visceta * K.lamda) : DBL_MAX);
  double dt = cfl * fmin(dt3, fmin(dt1, dt2));
  // DtFixed / DtFixedFile at the step's TimeStep (the corrector's DtVariable sees the same
  // TimeStep as the predictor's: the time advanced in between)
  if (K.dtfix_n || K.dtfix_val > 0) dt = fixed_dt(K, mode == DT_SYM_COR ? sc->tstep0 : sc->time, sc->dtfix_pos);
  // a NaN maximum (a NaN velocity, acceleration or viscosity anywhere) also stops the run:
  // fmin/fmax above would drop it, and the state it came from is already lost
  if (isnan(dt) || isinf(dt) || isnan(velmax) || isnan(acemax) || isnan(viscdt) || isnan(visceta)) {
    // the reference throws here (JSphCpu.cpp:1622): this step is not taken, and every
    // later kernel of a batched run sees the flag (halted) and leaves the state alone
    sc->error_flags |= ERR_DT_NAN;
    return;
  }
  if (dt < dtmin) {
    dt = dtmin;
    sc->dtmodif++;
  }
  if (mode == DT_VERLET) {
    sc->dt = dt;
  } else if (mode == DT_SYM_PRE) {
    sc->ddt_p = dt;
    sc->dt = sc->symdtpre;  // the step runs with SymplecticDtPre (JSphCpuSingle.cpp:696)
  } else {                  // DT_SYM_COR
    sc->symdtpre = fmin(sc->ddt_p, dt);  // JSphCpuSingle.cpp:719
  }
  if (mode != DT_SYM_COR) {
    // Step bookkeeping: TimeStep+=stepdt (JSphCpuSingle.cpp:1099).
    const double stepdt = sc->dt;
    sc->tstep0 = sc->time;
    if (dttrace && tracecap) dttrace[sc->nstep % tracecap] = stepdt;
    sc->time += stepdt;
    sc->last_dt = stepdt;
    sc->nstep++;
  }
  // ViscoTime: Visco of the next step, at its TimeStep (JSphCpuSingle.cpp:1092), once the
  // step in flight is done (the Symplectic corrector keeps the predictor's Visco)
  if (K.visco_n && mode != DT_SYM_PRE) sc->visco = visco_at(K, float(sc->time), sc->visco_pos);
}

// Visco at the current TimeStep (a new ViscoTime table, a restart time).
__global__ void k_visco_init(DevScalars* __restrict__ sc, KConst K) {
  if (threadIdx.x == 0) sc->visco = K.visco_n ? visco_at(K, float(sc->time), sc->visco_pos) : K.visco;
}

void launch_visco_init(hipStream_t stm, DevScalars* sc, const KConst& K) {
  hipLaunchKernelGGL(k_visco_init, dim3(1), dim3(64), 0, stm, sc, K);
}

void launch_dt(hipStream_t stm, DevScalars* sc, const KConst& K, double cfl, double dtmin, double cs0, int mode,
               double* dttrace, unsigned tracecap, const unsigned* folded) {
  hipLaunchKernelGGL(k_dt, dim3(1), dim3(64), 0, stm, sc, K, cfl, dtmin, cs0, mode, dttrace, tracecap, folded);
}

// Slab ghost: its local column is outside the owned range.  The owner updates it; here
// it is only dropped at the next divide (fresh copies arrive with the exchange).
__device__ __forceinline__ bool slab_ghost(const KConst& K, const DivGrid& g, unsigned dc) {
  return g.split() && !slab_owned(g, slab_local(g, K.domcellcode, dc));
}

enum { UPD_VERLET = 0, UPD_SYM_PRE = 1, UPD_SYM_COR = 2 };

// The update's products are kept out of multiply-add fusion (nc, sph_kernels.hpp): the
// reference's doubles are plain multiplies and adds, and without it -ffp-contract=fast (which
// fuses across statements and ignores `#pragma clang fp contract`) chose per code shape which
// product to fuse — one-ulp position differences between the fused update at 512 x 2 and the
// per-particle kernel (profiles/r06_ab/dbg18_upd512_stirred.log).

// One particle's update inputs, all loaded before any of its stores: one memory latency per
// particle instead of a chain of them (the stores to the particle arrays would otherwise keep
// each later load behind the branch that needs it).  Per kind:
//   Verlet: v1 = velrhop, v2 = velrhop (Euler) or velrhopm1, pos = posxy / posz (fluid)
//   SymPre: v1 = velrhoppre, pos = posxypre / poszpre (every particle: copied when halted)
//   SymCor: v1 = velrhop, v2 = velrhoppre, pos = posxypre / poszpre (fluid, floating)
struct UpdIn {
  float4 ra, v1, v2, sh;
  double2 pxy;
  double pz;
  unsigned dcell;
  typecode code;
};
// The particle's dcell and code after its update: the next divide's classification inputs.
struct UpdOut {
  unsigned dcell;
  typecode code;
};

template <int KIND>
__device__ __forceinline__ UpdIn upd_load(int euler, const float4* __restrict__ arace, const PartArrays& a,
                                          const float4* __restrict__ shiftpos, unsigned p, unsigned npb) {
  UpdIn in;
  in.dcell = a.dcell[p];
  in.code = a.code[p];
  in.ra = arace[p];
  if (KIND == UPD_SYM_PRE) {
    in.v1 = a.velrhoppre[p];
    in.v2 = in.v1;
  } else {
    in.v1 = a.velrhop[p];
    // (velrhopm1 read on Euler steps too: a select between it and v1 as pointers put `in` in
    // scratch memory)
    in.v2 = (KIND == UPD_SYM_COR ? a.velrhoppre[p] : a.velrhopm1[p]);
    if (KIND == UPD_VERLET && euler) in.v2 = in.v1;
  }
  in.pxy = make_double2(0., 0.);
  in.pz = 0.;
  in.sh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (KIND == UPD_SYM_PRE || p >= npb) {
    in.pxy = (KIND == UPD_VERLET ? a.posxy : a.posxypre)[p];
    in.pz = (KIND == UPD_VERLET ? a.posz : a.poszpre)[p];
  }
  if (KIND != UPD_SYM_PRE && shiftpos && p >= npb) in.sh = shiftpos[p];
  return in;
}
// After the loads of a thread's particles, before the first store: every load issued (without
// this use the compiler sinks the loads only one branch needs — code, position, shifting —
// into it, behind the stores before it).
__device__ __forceinline__ void upd_keep(const UpdIn& in) {
  asm volatile("" ::"v"(unsigned(in.code)), "v"(in.pxy.x), "v"(in.pxy.y), "v"(in.pz), "v"(in.sh.x));
}

// ComputeVerlet (JSphCpu.cpp:1381-1399): bound -> ComputeVelrhopBound, fluid -> ComputeVerletVarsFluid.
// New values are written in velrhopm1 (the caller swaps velrhop/velrhopm1 afterwards).
__device__ __forceinline__ UpdOut verlet_part(const DevScalars* __restrict__ sc, const KConst& K, int euler,
                                              const PartArrays& a, const DivGrid& g, bool shift, unsigned p,
                                              unsigned npb, const UpdIn& in) {
  UpdOut o{in.dcell, in.code};
  const bool ghost = slab_ghost(K, g, in.dcell);
  if (ghost) {
    a.dcell[p] = DCELL_DISCARD;
    o.dcell = DCELL_DISCARD;
  }
  if (halted(sc)) {  // keep the state: the caller's velrhop/velrhopm1 swap then restores it
    a.velrhopm1[p] = in.v1;
    // a slab still drops its ghosts (above): the next exchange sends fresh copies (without
    // this the stale ones piled up, a duplicate set per halted step)
    return o;
  }
  if (ghost) return o;
  const double dt = sc->dt;
  const double dt2 = (euler ? dt : dt + dt);
  const float4 ra = in.ra;
  const float4 vr2 = in.v2;
  const float rhopnew = float(double(vr2.w) + nc(dt2 * double(ra.w)));
  if (p < npb) {
    a.velrhopm1[p] = make_float4(0.f, 0.f, 0.f, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    return o;
  }
  const float4 vr1 = in.v1;
  if (CodeType(in.code) == CODE_TYPE_FLOATING) {  // JSphCpu.cpp:1352-1355: RunFloating moves it
    a.velrhopm1[p] = make_float4(vr1.x, vr1.y, vr1.z, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    return o;
  }
  const double dt205 = 0.5 * dt * dt;
  const double agx = double(ra.x) + K.gravxd, agy = double(ra.y) + K.gravyd, agz = double(ra.z) + K.gravzd;
  double dx = nc(double(vr1.x) * dt) + nc(agx * dt205);
  double dy = nc(double(vr1.y) * dt) + nc(agy * dt205);
  double dz = nc(double(vr1.z) * dt) + nc(agz * dt205);
  if (shift) shift_displacement(K, in.sh, vr1, dt, dx, dy, dz);  // RunShifting(dt) before ComputeVerlet
  const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
  const float4 nv = make_float4(float(double(vr2.x) + nc(agx * dt2)), float(double(vr2.y) + nc(agy * dt2)),
                                float(double(vr2.z) + nc(agz * dt2)), rhopnew);
  typecode rcode = in.code;
  o.dcell = update_pos(K, in.pxy.x, in.pxy.y, in.pz, dx, dy, dz, outrhop, p, a, &rcode);
  o.code = rcode;
  a.velrhopm1[p] = nv;
  return o;
}

// ComputeSymplecticPre (JSphCpu.cpp:1406-1504).  The caller has already moved the
// current pos/velrhop into the *pre arrays (pointer swap); new values go to pos/velrhop.
__device__ __forceinline__ UpdOut sym_pre_part(const DevScalars* __restrict__ sc, const KConst& K,
                                               const PartArrays& a, const DivGrid& g, unsigned p, unsigned npb,
                                               const UpdIn& in) {
  UpdOut o{in.dcell, in.code};
  const bool ghost = slab_ghost(K, g, in.dcell);
  if (ghost) {  // ghosts are dropped all the same, halted or not (verlet_part)
    a.dcell[p] = DCELL_DISCARD;
    o.dcell = DCELL_DISCARD;
  }
  const double2 pxy = in.pxy;
  const double pz = in.pz;
  if (halted(sc)) {  // keep the state (the caller moved it into the pre arrays)
    a.velrhop[p] = in.v1;
    a.posxy[p] = pxy;
    a.posz[p] = pz;
    return o;
  }
  if (ghost) return o;
  const double dt = sc->dt, dt05 = dt * .5;
  const float4 ra = in.ra;
  const float4 vp = in.v1;
  const float rhopnew = float(double(vp.w) + nc(dt05 * double(ra.w)));
  if (p < npb) {
    a.velrhop[p] = make_float4(vp.x, vp.y, vp.z, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    a.posxy[p] = pxy;
    a.posz[p] = pz;
    return o;
  }
  typecode rcode = in.code;
  if (CodeType(rcode) == CODE_TYPE_FLOATING) {  // JSphCpu.cpp:1475-1478 (+ position copied, :1498)
    a.velrhop[p] = make_float4(vp.x, vp.y, vp.z, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    a.posxy[p] = pxy;
    a.posz[p] = pz;
    return o;
  }
  const double dx = nc(double(vp.x) * dt05), dy = nc(double(vp.y) * dt05), dz = nc(double(vp.z) * dt05);
  const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
  a.velrhop[p] = make_float4(float(double(vp.x) + nc((double(ra.x) + K.gravxd) * dt05)),
                             float(double(vp.y) + nc((double(ra.y) + K.gravyd) * dt05)),
                             float(double(vp.z) + nc((double(ra.z) + K.gravzd) * dt05)), rhopnew);
  if (outrhop && CodeIsNormal(rcode)) {
    rcode = CodeSetNormal(rcode) | CODE_OUTRHOP;
    a.code[p] = rcode;
  }
  if (CodeIsFluid(rcode)) {
    o.dcell = update_pos(K, pxy.x, pxy.y, pz, dx, dy, dz, CodeIsOutRhop(rcode), p, a, &rcode);
  } else {
    a.posxy[p] = pxy;
    a.posz[p] = pz;
  }
  o.code = rcode;
  return o;
}

// ComputeSymplecticCorr (JSphCpu.cpp:1510-1606).
__device__ __forceinline__ UpdOut sym_cor_part(const DevScalars* __restrict__ sc, const KConst& K,
                                               const PartArrays& a, const DivGrid& g, bool shift, unsigned p,
                                               unsigned npb, const UpdIn& in) {
  UpdOut o{in.dcell, in.code};
  if (slab_ghost(K, g, in.dcell)) {  // ghosts dropped even when halted
    a.dcell[p] = DCELL_DISCARD;
    o.dcell = DCELL_DISCARD;
    return o;
  }
  if (halted(sc)) return o;
  const double dt = sc->dt, dt05 = dt * .5;
  const float4 ra = in.ra;
  const float4 vr = in.v1;
  const float4 vp = in.v2;
  const double epsilon_rdot = nc((-double(ra.w) / double(vr.w)) * dt);
  const float rhopnew = float(nc(double(vp.w) * (2. - epsilon_rdot)) / (2. + epsilon_rdot));
  if (p < npb) {
    a.velrhop[p] = make_float4(0.f, 0.f, 0.f, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    return o;  // boundary keeps its position (already restored by the predictor)
  }
  typecode rcode = in.code;
  if (CodeType(rcode) == CODE_TYPE_FLOATING) {  // JSphCpu.cpp:1577-1580, 1595
    a.velrhop[p] = make_float4(vp.x, vp.y, vp.z, (rhopnew < K.rhopzero ? K.rhopzero : rhopnew));
    a.posxy[p] = in.pxy;
    a.posz[p] = in.pz;
    return o;
  }
  const float4 nv = make_float4(float(double(vp.x) + nc((double(ra.x) + K.gravxd) * dt)),
                                float(double(vp.y) + nc((double(ra.y) + K.gravyd) * dt)),
                                float(double(vp.z) + nc((double(ra.z) + K.gravzd) * dt)), rhopnew);
  double dx = nc((double(vp.x) + double(nv.x)) * dt05);
  double dy = nc((double(vp.y) + double(nv.y)) * dt05);
  double dz = nc((double(vp.z) + double(nv.z)) * dt05);
  // RunShifting(dt) after the corrector's interaction, with the predicted velocity
  // (JSphCpuSingle.cpp:764 of the v5.0 solver, JSphShifting.cpp:388-418)
  if (shift) shift_displacement(K, in.sh, vr, dt, dx, dy, dz);
  const bool outrhop = (rhopnew < K.rhopoutmin || rhopnew > K.rhopoutmax);
  if (outrhop && CodeIsNormal(rcode)) {
    rcode = CodeSetNormal(rcode) | CODE_OUTRHOP;
    a.code[p] = rcode;
  }
  a.velrhop[p] = nv;
  if (CodeIsFluid(rcode)) {
    o.dcell = update_pos(K, in.pxy.x, in.pxy.y, in.pz, dx, dy, dz, CodeIsOutRhop(rcode), p, a, &rcode);
  } else {
    a.posxy[p] = in.pxy;
    a.posz[p] = in.pz;
  }
  o.code = rcode;
  return o;
}

// One particle's update of kind KIND from its loaded inputs (the kind's arithmetic and stores).
template <int KIND>
__device__ __forceinline__ UpdOut upd_compute(const DevScalars* __restrict__ sc, const KConst& K, int euler,
                                              const PartArrays& a, const DivGrid& g, bool shift, unsigned p,
                                              unsigned npb, const UpdIn& in) {
  if (KIND == UPD_VERLET) return verlet_part(sc, K, euler, a, g, shift, p, npb, in);
  if (KIND == UPD_SYM_PRE) return sym_pre_part(sc, K, a, g, p, npb, in);
  return sym_cor_part(sc, K, a, g, shift, p, npb, in);
}

template <int KIND>
__global__ __launch_bounds__(256) void k_update(const DevScalars* __restrict__ sc, KConst K, int euler,
                                                const float4* __restrict__ arace, PartArrays a, DivGrid g,
                                                const float4* __restrict__ shiftpos) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= sc->np) return;
  const unsigned npb = sc->npb;
  const UpdIn in = upd_load<KIND>(euler, arace, a, shiftpos, p, npb);
  upd_keep(in);
  upd_compute<KIND>(sc, K, euler, a, g, shiftpos != nullptr, p, npb, in);
}

// The update with the incremental divide's classification of the same particles (sph_incdiv.hpp):
// one block of UPD_BS threads per classify tile updates its INC_TILE particles (INC_TILE /
// UPD_BS per thread at stride UPD_BS: every input of all of them loaded first, one memory
// latency) and classifies them from the dcell and code it has just computed, in registers
// (with the previous keys, loaded with the update's inputs).  A step without bodies: nothing
// moves a particle between the update and the divide.  PACK (a slab with neighbours): also the
// exchange's count pass over the same tile (sph_slabpack.hpp, PK_TILE = INC_TILE).
// 512 threads x 2 particles (98 VGPRs, 5 waves/SIMD): at a cfg3 y-slab 47 vs 60 us per call
// for 1024 x 1 (profiles/r06_turns8/turns14_*.log).  Bitwise the per-particle kernels since
// the update's products are kept out of multiply-add fusion (nc, above; before that the
// unrolled pair fused other products: profiles/r06_ab/test16_*.log, dbg18_upd512_stirred.log).
constexpr int UPD_BS = 512, UPD_IPT = INC_TILE / UPD_BS;
static_assert(PK_TILE == INC_TILE, "the pack's tiles are the classify tiles");
template <int KIND, bool PACK>
__global__ __launch_bounds__(UPD_BS) void k_update_cls(DevScalars* __restrict__ sc, KConst K, int euler,
                                                       const float4* __restrict__ arace, PartArrays a, DivGrid g,
                                                       const float4* __restrict__ shiftpos, IncDivScratch s,
                                                       int usey, int usez, PackArgs q) {
  const unsigned np = sc->np, npb = sc->npb;
  const unsigned base = blockIdx.x * INC_TILE + threadIdx.x;
  ClsVals v[UPD_IPT];
  UpdIn in[UPD_IPT];
#pragma unroll
  for (int e = 0; e < UPD_IPT; e++) {
    const unsigned p = base + e * UPD_BS;
    v[e] = ClsVals{DCELL_DISCARD, 0, 0u};
    if (p < np) {
      v[e].old = s.skeys[p];
      in[e] = upd_load<KIND>(euler, arace, a, shiftpos, p, npb);
    }
  }
#pragma unroll
  for (int e = 0; e < UPD_IPT; e++)
    if (base + e * UPD_BS < np) upd_keep(in[e]);
#pragma unroll
  for (int e = 0; e < UPD_IPT; e++) {
    const unsigned p = base + e * UPD_BS;
    if (p < np) {
      const UpdOut o = upd_compute<KIND>(sc, K, euler, a, g, shiftpos != nullptr, p, npb, in[e]);
      v[e].dc = o.dcell;
      v[e].cd = o.code;
    }
  }
  inc_classify_tile<UPD_BS>(sc, a.dcell, a.code, g, K.domcellcode, s, usey, usez, blockIdx.x, v);
  if (PACK) pack_count_tile<UPD_BS>(sc, q, blockIdx.x, v);
}
template <int KIND>
static void launch_update_cls(hipStream_t stm, DevScalars* sc, const KConst& K, int euler, const float4* arace,
                              const PartArrays& a, const DivGrid& g, const float4* shiftpos, const IncDivScratch& s,
                              const PackArgs* pk) {
  const int usey = g.ncy > 1, usez = g.ncz > 1;
  if (pk)
    hipLaunchKernelGGL((k_update_cls<KIND, true>), dim3(s.nb1), dim3(UPD_BS), 0, stm, sc, K, euler, arace, a, g,
                       shiftpos, s, usey, usez, *pk);
  else
    hipLaunchKernelGGL((k_update_cls<KIND, false>), dim3(s.nb1), dim3(UPD_BS), 0, stm, sc, K, euler, arace, a, g,
                       shiftpos, s, usey, usez, PackArgs{});
}

// cls: the divide's scratch when the classification rides on the update (nullptr: the
// per-particle kernel, the divide classifies).
void launch_verlet(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, bool euler, const float4* arace,
                   PartArrays a, DivGrid g, const float4* shiftpos, const IncDivScratch* cls, const PackArgs* pk) {
  if (cls) {
    launch_update_cls<UPD_VERLET>(stm, sc, K, int(euler), arace, a, g, shiftpos, *cls, pk);
    return;
  }
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_update<UPD_VERLET>, dim3(nb), dim3(256), 0, stm, sc, K, int(euler), arace, a, g, shiftpos);
}
void launch_sym_pre(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a,
                    DivGrid g, const IncDivScratch* cls, const PackArgs* pk) {
  if (cls) {
    launch_update_cls<UPD_SYM_PRE>(stm, sc, K, 0, arace, a, g, nullptr, *cls, pk);
    return;
  }
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_update<UPD_SYM_PRE>, dim3(nb), dim3(256), 0, stm, sc, K, 0, arace, a, g, nullptr);
}
void launch_sym_cor(hipStream_t stm, unsigned cap, DevScalars* sc, const KConst& K, const float4* arace, PartArrays a,
                    DivGrid g, const float4* shiftpos, const IncDivScratch* cls, const PackArgs* pk) {
  if (cls) {
    launch_update_cls<UPD_SYM_COR>(stm, sc, K, 0, arace, a, g, shiftpos, *cls, pk);
    return;
  }
  const unsigned nb = (cap + 255) / 256;
  hipLaunchKernelGGL(k_update<UPD_SYM_COR>, dim3(nb), dim3(256), 0, stm, sc, K, 0, arace, a, g, shiftpos);
}

}  // namespace sphx
