// sph_bodies.hip — moving boundaries and floating rigid bodies on gfx950, SURVEY.md §8(f) row 3.
//
// Both run ON THE DEVICE, so a step keeps the core's no-host-round-trip property even
// though the motion of a step depends on its dt (computed on the device by k_dt):
//
// * Moving boundaries.  The reference evaluates its motion program on the host
//   (JSph::CalcMotion -> JDsMotion::ProcesTime -> JMotion::ProcesTimeSimple,
//   JSph.cpp:2308, JDsMotion.cpp:121-137, JMotion.cpp:347-366, JMotionObj.cpp:368-580)
//   and applies it with JSphCpu::RunMotion / MoveLinBound / MoveMatBound
//   (JSphCpu.cpp:1692-1790; GPU cusph::MoveLinBound/MoveMatBound, JSphGpu_ker.cu:2032+).
//   Here one wave restates the event/active-movement machinery (k_motion) over a
//   program uploaded once, then a grid over the boundary particles applies the
//   per-object displacement (k_move_bound).  Supported movements: wait, mvrect,
//   mvrectace, mvrot, mvrotace, mvrectsinu, mvrotsinu, chained by `next`, started by
//   <begin> events (finish optional); nested objects and file-driven movements are
//   refused by the loader.
// * Floating bodies (RigidAlgorithm=1, SPH).  JSphCpuSingle::RunFloating
//   (JSphCpuSingle.cpp:897-1010): FtCalcForcesSum (:748-768), FtCalcForces (:775-815),
//   FtCalcForcesRes (:822-858), constraints (:863-873), then the particle update and the
//   body state.  GPU twins: cusph::FtCalcForcesSum/FtCalcForces/FtUpdate
//   (JSphGpu_ker.cu:1749-2030).  k_ft_partial: FT_NBLK blocks per body sum the particle
//   forces (fixed-order LDS trees), k_ft_forces: one lane per body adds the partials in
//   order (deterministic) and integrates the body;
//   k_ft_update moves the particles and stores the body state.
//
// Matrix algebra follows JMatrix4 (JMatrix4.h:131-366) operation for operation and the
// float 3x3 helpers of FunctionsMath.h:91-329; contraction into FMA is disabled here so
// the double motion matrices round like the reference's x86 build.
#include <cfloat>

#include "sph_kernels.hpp"

#pragma clang fp contract(off)

namespace sphx {

// ---- 4x4 double matrices (JMatrix4d) --------------------------------------------------
struct M4d {
  double a[16];  // row major, a[4*r+c]
};
__device__ inline void m4_identity(M4d& m) {
  for (int i = 0; i < 16; i++) m.a[i] = (i % 5 == 0 ? 1.0 : 0.0);
}
// this = this * m2 (JMatrix4::Mul, JMatrix4.h:131-149)
__device__ inline void m4_mul(M4d& m1, const M4d& m2) {
  M4d r;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      r.a[4 * i + j] = m1.a[4 * i] * m2.a[j] + m1.a[4 * i + 1] * m2.a[4 + j] + m1.a[4 * i + 2] * m2.a[8 + j] +
                       m1.a[4 * i + 3] * m2.a[12 + j];
  m1 = r;
}
__device__ inline void m4_mov(M4d& m, double x, double y, double z) {  // MatrixMov
  m4_identity(m);
  m.a[3] = x;
  m.a[7] = y;
  m.a[11] = z;
}
// JMatrix4::MatrixRot(ang [degrees], axisp1, axisp2) (JMatrix4.h:332-366)
__device__ inline M4d m4_rot(double ang, const double* p1, const double* p2) {
  const double rad = ang * 0.017453292519943295769;
  const double vx = p2[0] - p1[0], vy = p2[1] - p1[1], vz = p2[2] - p1[2];
  const double L = sqrt(vx * vx + vy * vy + vz * vz);
  const double L1 = sqrt(vy * vy + vz * vz);
  M4d t, tm1, rx, rxm1, ry, rym1, rz;
  m4_mov(t, p1[0], p1[1], p1[2]);
  m4_mov(tm1, -p1[0], -p1[1], -p1[2]);
  m4_identity(rx);
  m4_identity(rxm1);
  if (L1 == 0) {
    rx.a[5] = 0; rx.a[6] = 1; rx.a[9] = -1; rx.a[10] = 0;
    rxm1.a[5] = 0; rxm1.a[6] = -1; rxm1.a[9] = 1; rxm1.a[10] = 0;
  } else {
    rx.a[5] = vz / L1; rx.a[6] = vy / L1; rx.a[9] = -vy / L1; rx.a[10] = vz / L1;
    rxm1.a[5] = vz / L1; rxm1.a[6] = -vy / L1; rxm1.a[9] = vy / L1; rxm1.a[10] = vz / L1;
  }
  m4_identity(ry);
  ry.a[0] = L1 / L; ry.a[2] = vx / L; ry.a[8] = -vx / L; ry.a[10] = L1 / L;
  m4_identity(rym1);
  rym1.a[0] = L1 / L; rym1.a[2] = -vx / L; rym1.a[8] = vx / L; rym1.a[10] = L1 / L;
  const double cs = cos(rad), sn = sin(rad);
  m4_identity(rz);
  rz.a[0] = cs; rz.a[1] = sn; rz.a[4] = -sn; rz.a[5] = cs;
  m4_mul(t, rx);
  m4_mul(t, ry);
  m4_mul(t, rz);
  m4_mul(t, rym1);
  m4_mul(t, rxm1);
  m4_mul(t, tm1);
  return t;
}

// JMotionPos (JMotionPos.cpp:29-107): accumulated motion of one object in one step.
struct MPos {
  bool simple;
  double s[3];
  M4d m;
};
__device__ inline void mpos_reset(MPos& p) {
  p.simple = true;
  p.s[0] = p.s[1] = p.s[2] = 0;
  m4_identity(p.m);
}
__device__ inline void mpos_move(MPos& p, double x, double y, double z) {
  if (p.simple) {
    p.s[0] = p.s[0] + x;
    p.s[1] = p.s[1] + y;
    p.s[2] = p.s[2] + z;
  } else {
    M4d mv;
    m4_mov(mv, x, y, z);
    m4_mul(p.m, mv);
  }
}
__device__ inline void mpos_rotate(MPos& p, double ang, const double* p1, const double* p2) {
  if (p.simple) {
    m4_mov(p.m, p.s[0], p.s[1], p.s[2]);
    p.simple = false;
  }
  const M4d r = m4_rot(ang, p1, p2);
  m4_mul(p.m, r);
}

// ---- motion program ----------------------------------------------------------------------
// JMotionMovActive (JMotionObj.cpp:40-208): ConfigData of a (next) movement.
__device__ inline void act_config(MotAct& a, const MotMov& mv) {
  a.vel[0] = a.vel[1] = a.vel[2] = 0;
  a.velang = 0;
  a.phase[0] = a.phase[1] = a.phase[2] = 0;
  a.phaseuni = 0;
  switch (mv.type) {
    case SPH_MOV_RECT: a.vel[0] = mv.v[0]; a.vel[1] = mv.v[1]; a.vel[2] = mv.v[2]; break;
    case SPH_MOV_RECTACE: a.vel[0] = mv.v2[0]; a.vel[1] = mv.v2[1]; a.vel[2] = mv.v2[2]; break;
    case SPH_MOV_ROT: a.velang = mv.ang; break;
    case SPH_MOV_ROTACE: a.velang = mv.ang2; break;
    case SPH_MOV_RECTSINU:
      a.phase[0] = mv.phase[0]; a.phase[1] = mv.phase[1]; a.phase[2] = mv.phase[2];
      break;
    case SPH_MOV_ROTSINU: a.phaseuni = mv.ang3; break;
    default: break;
  }
}

// One object: JMotionObj::ProcesTime (JMotionObj.cpp:368-580) without parents/children.
// Returns true when the object moved (modif) in [timestep, timestep+dt).
__device__ bool obj_proces_time(MotionDev& md, MotObj& o, const MotMov* movs, double timestep, double dt,
                                MPos& modpos) {
  bool modif = false;
  int na = o.na;
  if (na) {
    const double tstepfin = timestep + dt;
    mpos_reset(modpos);
    for (int ca = 0; ca < na; ca++) {
      MotAct& amov = o.act[ca];
      if (amov.del) {  // erase the active movement marked in the previous step
        for (int k = ca; k + 1 < na; k++) o.act[k] = o.act[k + 1];
        ca--;
        na--;
        continue;
      }
      bool rep;
      double dt2 = dt, timestep2 = timestep;
      do {
        rep = false;
        const MotMov& mv = movs[amov.mov];
        double dtmov = (tstepfin > amov.finish ? amov.finish - timestep2 : dt2);
        const double dtover = dt2 - dtmov;
        if (timestep2 < amov.start) dtmov -= (amov.start - timestep2);
        if (dtmov > 0) {
          const double t = dtmov;
          switch (mv.type) {
            case SPH_MOV_RECT:
              mpos_move(modpos, mv.v[0] * t, mv.v[1] * t, mv.v[2] * t);
              modif = true;
              break;
            case SPH_MOV_RECTACE: {
              const double atx = mv.v[0] * t, aty = mv.v[1] * t, atz = mv.v[2] * t;
              // 0.5f*at*t in the reference: the float literal promotes to double exactly
              mpos_move(modpos, amov.vel[0] * t + 0.5 * atx * t, amov.vel[1] * t + 0.5 * aty * t,
                        amov.vel[2] * t + 0.5 * atz * t);
              amov.vel[0] = amov.vel[0] + atx;
              amov.vel[1] = amov.vel[1] + aty;
              amov.vel[2] = amov.vel[2] + atz;
              modif = true;
            } break;
            case SPH_MOV_ROT:
              mpos_rotate(modpos, mv.ang * t, mv.p1, mv.p2);
              modif = true;
              break;
            case SPH_MOV_ROTACE: {
              const double at = mv.ang * t;
              mpos_rotate(modpos, amov.velang * t + 0.5 * at * t, mv.p1, mv.p2);
              amov.velang += at;
              modif = true;
            } break;
            case SPH_MOV_RECTSINU: {
              double ph[3] = {amov.phase[0], amov.phase[1], amov.phase[2]};
              double q1[3] = {0, 0, 0}, q2[3] = {0, 0, 0};
              for (int k = 0; k < 3; k++)
                if (mv.v2[k] != 0) {
                  q1[k] = mv.v2[k] * sin(ph[k]);
                  ph[k] += double(mv.v[k] * 6.28318530717958647692 * t);
                  q2[k] = mv.v2[k] * sin(ph[k]);
                }
              mpos_move(modpos, q2[0] - q1[0], q2[1] - q1[1], q2[2] - q1[2]);
              amov.phase[0] = ph[0];
              amov.phase[1] = ph[1];
              amov.phase[2] = ph[2];
              modif = true;
            } break;
            case SPH_MOV_ROTSINU: {
              double ph = amov.phaseuni;
              double ang = mv.ang2 * sin(ph);
              ph += double(mv.ang * (3.14159265358979323846 + 3.14159265358979323846) * t);
              ang = mv.ang2 * sin(ph) - ang;
              mpos_rotate(modpos, ang, mv.p1, mv.p2);
              amov.phaseuni = ph;
              modif = true;
            } break;
            default: break;  // wait
          }
        }
        // chain to the next movement to consume the rest of dt
        if ((dtover > 0 || dtmov == 0) && mv.nextidx >= 0) {
          const MotMov& nm = movs[mv.nextidx];
          amov.start += mv.time;
          const double velp[3] = {amov.vel[0], amov.vel[1], amov.vel[2]};
          const double php[3] = {amov.phase[0], amov.phase[1], amov.phase[2]};
          const double velangp = amov.velang, phaseunip = amov.phaseuni;
          amov.mov = mv.nextidx;
          amov.finish = amov.start + nm.time;
          if (amov.eventfinish >= 0 && amov.eventfinish < amov.finish) amov.finish = amov.eventfinish;
          act_config(amov, nm);
          if (nm.prev) {
            if (nm.type == SPH_MOV_RECTACE) { amov.vel[0] = velp[0]; amov.vel[1] = velp[1]; amov.vel[2] = velp[2]; }
            if (nm.type == SPH_MOV_ROTACE) amov.velang = velangp;
            if (nm.type == SPH_MOV_RECTSINU) { amov.phase[0] = php[0]; amov.phase[1] = php[1]; amov.phase[2] = php[2]; }
            if (nm.type == SPH_MOV_ROTSINU) amov.phaseuni = phaseunip;
          }
          dt2 = dtover;
          timestep2 = amov.start;
          if (timestep2 <= amov.finish) rep = true;
        }
      } while (rep);
      if (tstepfin > amov.finish) amov.del = 1;
    }
    o.na = na;
  }
  if (modif) {
    o.moving = 1;
  } else if (o.moving) {
    o.moving = 0;
  } else if (!na) {
    o.active = 0;
  }
  return modif;
}

// JSph::CalcMotion + JMotion::ProcesTimeSimple for [sc->tstep0, sc->tstep0 + stepdt),
// results in md->out[obj] (JMotionListData::Sp_Movedt, JMotionList.cpp:43-61).
__global__ void k_motion(const DevScalars* __restrict__ sc, MotionDev* __restrict__ md,
                         const MotMov* __restrict__ movs, const MotEvt* __restrict__ evts, double t0, double dt0) {
  if (threadIdx.x != 0) return;
  const double timestep = (t0 >= 0 ? t0 : sc->tstep0), dt = (t0 >= 0 ? dt0 : sc->last_dt);
  for (int o = 0; o < md->nobj; o++) md->out[o].type = 0;  // PreMotion
  if (t0 < 0 && halted(sc)) return;  // a fatal error stopped the run: nothing moves
  // JMotion::ProcesTime (JMotion.cpp:446-468): start the events that begin before t+dt
  bool looking = true;
  for (int c = md->eventnext; c >= 0 && looking; c--) {
    const MotEvt& e = evts[c];
    if (e.start < timestep + dt) {
      MotObj& o = md->obj[e.obj];
      if (o.na < MOT_MAXACT) {
        MotAct& a = o.act[o.na++];
        const MotMov& mv = movs[e.mov];
        a.mov = e.mov;
        a.start = e.start;
        a.eventfinish = e.finish;
        a.finish = a.start + mv.time;
        if (e.finish >= 0 && e.finish < a.finish) a.finish = e.finish;
        a.del = 0;
        act_config(a, mv);
      } else {
        md->overflow = 1;
      }
      o.active = 1;
      md->eventnext--;
      md->objsactive = 1;
    } else {
      looking = false;
    }
  }
  if (md->objsactive) {
    md->objsactive = 0;
    for (int oi = 0; oi < md->nobj; oi++) {
      MotObj& o = md->obj[oi];
      if (!o.active) continue;
      MPos mp;
      mpos_reset(mp);
      const bool modif = obj_proces_time(*md, o, movs, timestep, dt, mp);
      md->objsactive |= o.active;
      if (modif) {
        MotOut& r = md->out[oi];
        if (mp.simple) {
          r.type = 1;
          for (int k = 0; k < 3; k++) {
            r.mov[k] = mp.s[k];
            r.vel[k] = mp.s[k] / dt;
          }
        } else {
          r.type = 2;
          for (int k = 0; k < 12; k++) r.m[k] = mp.m.a[k];
        }
      }
    }
    // ProcesTimeSimple records the movements only when ProcesTime reports active objects
    if (!md->objsactive)
      for (int o = 0; o < md->nobj; o++) md->out[o].type = 0;
  }
}

// MoveLinBound / MoveMatBound (JSphCpu.cpp:1692-1731) over the boundary particles:
// the object is the moving block index in the code (JSphMk::Config, JSphMk.cpp:110).
__global__ __launch_bounds__(256) void k_move_bound(const DevScalars* __restrict__ sc, KConst K,
                                                    const MotionDev* __restrict__ md, PartArrays a,
                                                    float4* __restrict__ normal) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= sc->npb) return;
  if (a.dcell[p] == DCELL_DISCARD) return;  // slab ghost (marked by the update): its owner moves it
  const typecode c = a.code[p];
  if (CodeType(c) != CODE_TYPE_MOVING || !CodeIsNormal(c)) return;
  const unsigned obj = c & CODE_MASKVALUE;
  if (obj >= unsigned(md->nobj)) return;
  const MotOut& r = md->out[obj];
  if (r.type == 0) return;
  const double2 pxy = a.posxy[p];
  const double pz = a.posz[p];
  float4 v = a.velrhop[p];
  double mx, my, mz;
  if (r.type == 1) {
    mx = r.mov[0];
    my = r.mov[1];
    mz = r.mov[2];
    v.x = float(r.vel[0]);
    v.y = float(r.vel[1]);
    v.z = float(r.vel[2]);
  } else {
    const double* m = r.m;
    const double x2 = m[0] * pxy.x + m[1] * pxy.y + m[2] * pz + m[3];
    const double y2 = m[4] * pxy.x + m[5] * pxy.y + m[6] * pz + m[7];
    const double z2 = m[8] * pxy.x + m[9] * pxy.y + m[10] * pz + m[11];
    mx = x2 - pxy.x;
    my = y2 - pxy.y;
    mz = z2 - pz;
    const double dt = sc->last_dt;
    v.x = float(mx / dt);
    v.y = float(my / dt);
    v.z = float(mz / dt);
    if (normal) {  // the normal turns with the body (JSphCpu.cpp:1724-1728)
      const unsigned id = a.idp[p];
      const float4 n = normal[id];
      const double gx = pxy.x + double(n.x), gy = pxy.y + double(n.y), gz = pz + double(n.z);
      const double g2x = m[0] * gx + m[1] * gy + m[2] * gz + m[3];
      const double g2y = m[4] * gx + m[5] * gy + m[6] * gz + m[7];
      const double g2z = m[8] * gx + m[9] * gy + m[10] * gz + m[11];
      normal[id] = make_float4(float(g2x - x2), float(g2y - y2), float(g2z - z2), 0.f);
    }
  }
  a.velrhop[p] = v;
  update_pos_bound(K, pxy.x, pxy.y, pz, mx, my, mz, p, a, const_cast<DevScalars*>(sc));
}

void launch_motion(hipStream_t stm, unsigned npbcap, DevScalars* sc, const KConst& K, MotionDev* md,
                   const MotMov* movs, const MotEvt* evts, const PartArrays& a, float4* normal, const DivGrid&) {
  hipLaunchKernelGGL(k_motion, dim3(1), dim3(64), 0, stm, sc, md, movs, evts, -1.0, 0.0);
  const unsigned nb = (npbcap + 255) / 256;
  if (nb) hipLaunchKernelGGL(k_move_bound, dim3(nb), dim3(256), 0, stm, sc, K, md, a, normal);
}

void launch_motion_advance(hipStream_t stm, DevScalars* sc, MotionDev* md, const MotMov* movs, const MotEvt* evts,
                           double t0, double dt) {
  hipLaunchKernelGGL(k_motion, dim3(1), dim3(64), 0, stm, sc, md, movs, evts, t0, dt);
}

// ---- floating bodies ------------------------------------------------------------------------
// CalcRidp (JSphCpu.cpp CalcRidp; JSphCpuSingle.cpp:478): position of each floating
// particle after a divide, by idp - CaseNpb.
__global__ __launch_bounds__(256) void k_ft_ridp(const DevScalars* __restrict__ sc, const typecode* __restrict__ code,
                                                 const unsigned* __restrict__ idp, const unsigned* __restrict__ dcell,
                                                 unsigned casenpb, unsigned nftp, unsigned* __restrict__ ftridp,
                                                 KConst K, DivGrid g) {
  const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < sc->npb || p >= sc->np) return;
  if (CodeType(code[p]) != CODE_TYPE_FLOATING) return;
  if (!slab_owned(g, slab_local(g, K.domcellcode, dcell[p]))) return;  // slab ghost
  const unsigned k = idp[p] - casenpb;
  if (k < nftp) ftridp[k] = p;
}

void launch_ft_ridp(hipStream_t stm, unsigned cap, DevScalars* sc, const PartArrays& a, unsigned casenpb,
                    unsigned nftp, unsigned* ftridp, const KConst& K, const DivGrid& g) {
  (void)hipMemsetAsync(ftridp, 0xff, sizeof(unsigned) * nftp, stm);
  hipLaunchKernelGGL(k_ft_ridp, dim3((cap + 255) / 256), dim3(256), 0, stm, sc, a.code, a.idp, a.dcell, casenpb, nftp,
                     ftridp, K, g);
}

// float 3x3 helpers (FunctionsMath.h:91-329)
struct M3f {
  float a11, a12, a13, a21, a22, a23, a31, a32, a33;
};
__device__ inline M3f m3_mul(const M3f& a, const M3f& b) {
  return {a.a11 * b.a11 + a.a12 * b.a21 + a.a13 * b.a31, a.a11 * b.a12 + a.a12 * b.a22 + a.a13 * b.a32,
          a.a11 * b.a13 + a.a12 * b.a23 + a.a13 * b.a33, a.a21 * b.a11 + a.a22 * b.a21 + a.a23 * b.a31,
          a.a21 * b.a12 + a.a22 * b.a22 + a.a23 * b.a32, a.a21 * b.a13 + a.a22 * b.a23 + a.a23 * b.a33,
          a.a31 * b.a11 + a.a32 * b.a21 + a.a33 * b.a31, a.a31 * b.a12 + a.a32 * b.a22 + a.a33 * b.a32,
          a.a31 * b.a13 + a.a32 * b.a23 + a.a33 * b.a33};
}
__device__ inline M3f m3_tras(const M3f& a) { return {a.a11, a.a21, a.a31, a.a12, a.a22, a.a32, a.a13, a.a23, a.a33}; }
__device__ inline M3f m3_rot(float ax, float ay, float az) {
  const float cosx = cosf(ax), cosy = cosf(ay), cosz = cosf(az);
  const float sinx = sinf(ax), siny = sinf(ay), sinz = sinf(az);
  return {cosy * cosz, -cosy * sinz, siny,
          sinx * siny * cosz + cosx * sinz, -sinx * siny * sinz + cosx * cosz, -sinx * cosy,
          -cosx * siny * cosz + sinx * sinz, cosx * siny * sinz + sinx * cosz, cosx * cosy};
}
__device__ inline M3f m3_inv(const M3f& d) {
  const float det = d.a11 * d.a22 * d.a33 + d.a12 * d.a23 * d.a31 + d.a13 * d.a21 * d.a32 - d.a31 * d.a22 * d.a13 -
                    d.a32 * d.a23 * d.a11 - d.a33 * d.a21 * d.a12;
  if (!det) return {0, 0, 0, 0, 0, 0, 0, 0, 0};
  return {(d.a22 * d.a33 - d.a23 * d.a32) / det, -(d.a12 * d.a33 - d.a13 * d.a32) / det,
          (d.a12 * d.a23 - d.a13 * d.a22) / det, -(d.a21 * d.a33 - d.a23 * d.a31) / det,
          (d.a11 * d.a33 - d.a13 * d.a31) / det, -(d.a11 * d.a23 - d.a13 * d.a21) / det,
          (d.a21 * d.a32 - d.a22 * d.a31) / det, -(d.a11 * d.a32 - d.a12 * d.a31) / det,
          (d.a11 * d.a22 - d.a12 * d.a21) / det};
}

constexpr int FT_BS = 256;

// FtCalcForcesSum, stage 1: block (j, cf) sums force = ace*massp and torque = r x force
// over the particles fp = j*FT_BS + t (+ FT_NBLK*FT_BS strides) of body cf with a
// fixed-order LDS tree -> part[cf][j][6].
__global__ __launch_bounds__(FT_BS) void k_ft_partial(const DevScalars* __restrict__ sc,
                                                      const FtBody* __restrict__ bodies,
                                                      const unsigned* __restrict__ ftridp,
                                                      const float4* __restrict__ arace,
                                                      const double2* __restrict__ posxy,
                                                      const double* __restrict__ posz, float* __restrict__ part) {
  __shared__ float red[6][FT_BS];
  const int cf = blockIdx.y, j = blockIdx.x;
  const FtBody& b = bodies[cf];
  const double cx = b.center[0], cy = b.center[1], cz = b.center[2];
  const float massp = b.massp;
  float s[6] = {0, 0, 0, 0, 0, 0};
  for (unsigned fp = unsigned(j) * FT_BS + threadIdx.x; fp < b.count; fp += FT_NBLK * FT_BS) {
    const unsigned p = ftridp[b.begin + fp];
    if (p == 0xffffffffu) continue;
    const float4 ra = arace[p];
    const float fx = ra.x * massp, fy = ra.y * massp, fz = ra.z * massp;
    const double2 pxy = posxy[p];
    const float dx = float(pxy.x - cx), dy = float(pxy.y - cy), dz = float(posz[p] - cz);
    s[0] += fx;
    s[1] += fy;
    s[2] += fz;
    s[3] += fz * dy - fy * dz;
    s[4] += fx * dz - fz * dx;
    s[5] += fy * dx - fx * dy;
  }
  for (int k = 0; k < 6; k++) red[k][threadIdx.x] = s[k];
  __syncthreads();
  for (int w = FT_BS / 2; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w)
      for (int k = 0; k < 6; k++) red[k][threadIdx.x] += red[k][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 6) part[(size_t(cf) * FT_NBLK + j) * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// JLinearValue::GetValue3f at time t (JLinearValue.cpp:209-247 FindTime, :301-329
// GetValue3d, :387-390) of one table of n (time, x, y, z) rows, in any row order as the
// reference reads them (<vel> elements or a file): FindTime walks from the row of its last
// call (back while the row's time is >= t, then forward to the first later row whose time is
// >= t, the row before it as the lower one), and a call at the TimeStep of the last one keeps
// that interval (the Symplectic predictor and corrector of one step); the factor
// (t - tpre)/(tnext - tpre) clamped to [0,1] (0 for equal times), linear interpolation in
// double without contraction; DBL_MAX ("none") propagates from the earlier row, an interval
// ending in "none" keeps the earlier value; DBL_MAX -> FLT_MAX.
__device__ void ft_table_eval(const double4* __restrict__ tab, FtTabDesc& d, double t, float out[3]) {
  const double4* T = tab + d.first;
  const int n = d.n;
  if (d.pos < 0 || t != d.t) {
    int pos = d.pos < 0 ? 0 : d.pos, posnext = pos;
    double tpre = T[pos].x, tnext = tpre;
    if (n > 1) {
      while (tpre >= t && pos > 0) tpre = T[--pos].x;  // back
      posnext = pos + 1 < n ? pos + 1 : pos;
      tnext = T[posnext].x;
      while (tnext < t && posnext + 1 < n) tnext = T[++posnext].x;  // forward
      if (posnext - pos > 1) pos = posnext - 1;
    }
    d.pos = pos;
    d.posnext = posnext;
    d.t = t;
  }
  const int pos = d.pos, posnext = d.posnext;
  const double tpre = T[pos].x, tnext = T[posnext].x, tdif = tnext - tpre;
  double f = tdif != 0.0 ? (t - tpre) / tdif : 0.0;
  if (f < 0.) f = 0.;
  if (f > 1.) f = 1.;
  const double vi[3] = {T[pos].y, T[pos].z, T[pos].w}, vn[3] = {T[posnext].y, T[posnext].z, T[posnext].w};
  for (int k = 0; k < 3; k++) {
    double v;
    if (f == 0.) v = vi[k];
    else if (f >= 1.) v = vn[k];
    else {
      v = __dadd_rn(__dmul_rn(__dsub_rn(vn[k], vi[k]), f), vi[k]);
      if (vi[k] == DBL_MAX) v = DBL_MAX;
      else if (vn[k] == DBL_MAX) v = vi[k];
    }
    out[k] = (v == DBL_MAX ? FLT_MAX : float(v));
  }
}

// Stage 2, one lane per body: the partial sums in order, then FtCalcForces +
// FtCalcForcesRes + imposed velocities + constraints.  tab/desc: the bodies' JLinearValue
// tables (desc[body*4 + kind] = {first row, rows}, kinds SPH_FTTAB_*; nullptr: none).
__global__ void k_ft_forces(const DevScalars* __restrict__ sc, KConst K, FtBody* __restrict__ bodies, int nbodies,
                            const float* __restrict__ part, int predictor, const double4* __restrict__ tab,
                            FtTabDesc* __restrict__ desc) {
  const int cf = blockIdx.x * blockDim.x + threadIdx.x;
  if (cf >= nbodies || halted(sc)) return;
  FtBody& b = bodies[cf];
  const double dt = (predictor ? sc->dt * .5 : sc->dt);
  if (!(sc->tstep0 >= double(b.ftpause))) {
    b.skip = 1;
    return;
  }
  float red[6] = {0, 0, 0, 0, 0, 0};
  for (int j = 0; j < FT_NBLK; j++)
    for (int k = 0; k < 6; k++) red[k] += part[(size_t(cf) * FT_NBLK + j) * 6 + k];
  b.skip = 0;
  // FtCalcForces: inertia rotated to the current orientation, I^-1 * torque, + gravity.
  const M3f frot = m3_rot(b.angles[0], b.angles[1], b.angles[2]);
  const M3f ini = {b.inertia[0], b.inertia[1], b.inertia[2], b.inertia[3], b.inertia[4],
                   b.inertia[5], b.inertia[6], b.inertia[7], b.inertia[8]};
  const M3f inert = m3_mul(m3_mul(frot, ini), m3_tras(frot));
  const M3f inv = m3_inv(inert);
  float face[3] = {red[0], red[1], red[2]};
  float fo[3] = {red[3], red[4], red[5]};
  // external forces (RunFloating, JSphCpuSingle.cpp:904-914; added in FtCalcForces :797-798)
  const double tstep = sc->tstep0;
  if (desc && desc[cf * 4 + 2].n) {
    float e[3];
    ft_table_eval(tab, desc[cf * 4 + 2], tstep, e);
    for (int k = 0; k < 3; k++) face[k] = face[k] + e[k];
  }
  if (desc && desc[cf * 4 + 3].n) {
    float e[3];
    ft_table_eval(tab, desc[cf * 4 + 3], tstep, e);
    for (int k = 0; k < 3; k++) fo[k] = fo[k] + e[k];
  }
  float omegaace[3] = {fo[0] * inv.a11 + fo[1] * inv.a12 + fo[2] * inv.a13,
                       fo[0] * inv.a21 + fo[1] * inv.a22 + fo[2] * inv.a23,
                       fo[0] * inv.a31 + fo[1] * inv.a32 + fo[2] * inv.a33};
  const float fmass = b.mass;
  face[0] = (face[0] + fmass * K.gravx) / fmass;
  face[1] = (face[1] + fmass * K.gravy) / fmass;
  face[2] = (face[2] + fmass * K.gravz) / fmass;
  // FtCalcForcesRes
  float fomega[3], fvel[3], fvel0[3] = {b.fvel[0], b.fvel[1], b.fvel[2]};
  for (int k = 0; k < 3; k++) fomega[k] = float(dt * omegaace[k] + b.fomega[k]);
  if (K.sim2d) {  // Simulate2D (JSphCpuSingle.cpp:839)
    face[1] = 0;
    fomega[0] = 0;
    fomega[2] = 0;
    fvel0[1] = 0;
  }
  double fcenter[3];
  for (int k = 0; k < 3; k++) fcenter[k] = b.center[k] + dt * fvel0[k];
  for (int k = 0; k < 3; k++) fvel[k] = float(dt * face[k] + fvel0[k]);
  // FtApplyImposedVel (JSphCpuSingle.cpp:874-891): components given by the tables
  if (desc && desc[cf * 4 + 0].n) {
    float v[3];
    ft_table_eval(tab, desc[cf * 4 + 0], tstep, v);
    for (int k = 0; k < 3; k++)
      if (v[k] != FLT_MAX) fvel[k] = v[k];
  }
  if (desc && desc[cf * 4 + 1].n) {
    float v[3];
    ft_table_eval(tab, desc[cf * 4 + 1], tstep, v);
    for (int k = 0; k < 3; k++)
      if (v[k] != FLT_MAX) fomega[k] = v[k];
  }
  // FtApplyConstraints (DualSphDef.h:466-473)
  const unsigned con = b.constraints;
  if (con) {
    for (int k = 0; k < 3; k++) {
      if (con & (1u << k)) { face[k] = 0; fvel[k] = 0; }
      if (con & (8u << k)) { omegaace[k] = 0; fomega[k] = 0; }
    }
  }
  for (int k = 0; k < 3; k++) {
    b.face[k] = face[k];
    b.fomegaace[k] = omegaace[k];
    b.fvelres[k] = fvel[k];
    b.fomegares[k] = fomega[k];
    b.fcenterres[k] = fcenter[k];
  }
  if (!predictor) {
    // mDBC on the body: its normals turn by the step's change of the (float) angles, in
    // degrees (JSphCpuSingle.cpp:988-999: Move(center) Rotate(dang) Move(-center0), of
    // which MulNormal uses the 3x3 part, JMatrix4::MatrixRot = RotZ RotX RotY of the
    // nonzero angles, JMatrix4.h:270-324)
    double dang[3];
    for (int k = 0; k < 3; k++) {
      const float na = float(double(b.angles[k]) + double(fomega[k]) * dt);  // as k_ft_update
      dang[k] = double(na - b.angles[k]) * 57.29577951308232087684;
    }
    M4d r;
    m4_identity(r);
    const int ax[3] = {2, 0, 1};
    for (int q = 0; q < 3; q++) {
      const int k = ax[q];
      if (!dang[k]) continue;
      const double rad = dang[k] * 0.017453292519943295769;
      const double cs = cos(rad), sn = sin(rad);
      M4d m;
      m4_identity(m);
      if (k == 0) { m.a[5] = cs; m.a[6] = -sn; m.a[9] = sn; m.a[10] = cs; }        // MatrixRotX
      else if (k == 1) { m.a[0] = cs; m.a[2] = sn; m.a[8] = -sn; m.a[10] = cs; }   // MatrixRotY
      else { m.a[0] = cs; m.a[1] = -sn; m.a[4] = sn; m.a[5] = cs; }                // MatrixRotZ
      m4_mul(r, m);
    }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) b.nrot[3 * i + j] = r.a[4 * i + j];
  }
}

// Particle update + body state (RunFloating, JSphCpuSingle.cpp:950-1003).
__global__ __launch_bounds__(256) void k_ft_update(DevScalars* __restrict__ sc, KConst K, FtBody* __restrict__ bodies,
                                                   int nbodies, const unsigned* __restrict__ ftridp, unsigned nftp,
                                                   PartArrays a, int predictor, float4* __restrict__ normal) {
  const unsigned fp = blockIdx.x * blockDim.x + threadIdx.x;
  const double dt = (predictor ? sc->dt * .5 : sc->dt);
  if (fp < nftp && !halted(sc)) {
    int cf = 0;
    while (cf + 1 < nbodies && fp >= bodies[cf + 1].begin) cf++;
    const FtBody& b = bodies[cf];
    const unsigned p = ftridp[fp];
    if (!b.skip && p != 0xffffffffu) {
      float4 v = a.velrhop[p];
      const double2 pxy = a.posxy[p];
      const double pz = a.posz[p];
      update_pos_bound(K, pxy.x, pxy.y, pz, dt * double(v.x), dt * double(v.y), dt * double(v.z), p, a, sc);
      const double2 nxy = a.posxy[p];
      const float dx = float(nxy.x - b.fcenterres[0]), dy = float(nxy.y - b.fcenterres[1]),
                  dz = float(a.posz[p] - b.fcenterres[2]);
      const float* w = b.fomegares;
      v.x = b.fvelres[0] + (w[1] * dz - w[2] * dy);
      v.y = b.fvelres[1] + (w[2] * dx - w[0] * dz);
      v.z = b.fvelres[2] + (w[0] * dy - w[1] * dx);
      a.velrhop[p] = v;
      if (normal && !predictor) {  // BoundNormalc[p] = float3(mat.MulNormal(double3(normal)))
        const unsigned id = a.idp[p];
        const float4 n = normal[id];
        if (n.x != 0.f || n.y != 0.f || n.z != 0.f) {
          const double nx = n.x, ny = n.y, nz = n.z;
          const double* m = b.nrot;
          normal[id] = make_float4(float(m[0] * nx + m[1] * ny + m[2] * nz), float(m[3] * nx + m[4] * ny + m[5] * nz),
                                   float(m[6] * nx + m[7] * ny + m[8] * nz), 0.f);
        }
      }
    }
  }
  if (fp == 0 && !predictor && !halted(sc)) {
    const float fdt = float(dt);
    for (int cf = 0; cf < nbodies; cf++) {
      FtBody& b = bodies[cf];
      if (b.skip) continue;
      for (int k = 0; k < 3; k++) {
        b.center[k] = b.fcenterres[k];
        b.angles[k] = float(double(b.angles[k]) + double(b.fomegares[k]) * dt);
        b.facelin[k] = (b.fvelres[k] - b.fvel[k]) / fdt;
        b.faceang[k] = (b.fomegares[k] - b.fomega[k]) / fdt;
        b.fvel[k] = b.fvelres[k];
        b.fomega[k] = b.fomegares[k];
      }
    }
  }
}

void launch_ft_partial(hipStream_t stm, DevScalars* sc, const FtBody* bodies, int nbodies, const unsigned* ftridp,
                       const float4* arace, const PartArrays& a, float* part) {
  hipLaunchKernelGGL(k_ft_partial, dim3(FT_NBLK, nbodies), dim3(FT_BS), 0, stm, sc, bodies, ftridp, arace, a.posxy,
                     a.posz, part);
}

void launch_ft_body(hipStream_t stm, DevScalars* sc, const KConst& K, FtBody* bodies, int nbodies,
                    const unsigned* ftridp, unsigned nftp, const PartArrays& a, bool predictor, const float* part,
                    const double4* fttab, FtTabDesc* ftdesc, float4* normal) {
  hipLaunchKernelGGL(k_ft_forces, dim3((nbodies + 63) / 64), dim3(64), 0, stm, sc, K, bodies, nbodies, part,
                     int(predictor), fttab, ftdesc);
  hipLaunchKernelGGL(k_ft_update, dim3((nftp + 255) / 256), dim3(256), 0, stm, sc, K, bodies, nbodies, ftridp, nftp,
                     a, int(predictor), normal);
}

}  // namespace sphx
