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
//   per-object displacement (k_move_bound).  Every movement of JMotion::ReadXml: wait,
//   mvrect, mvrectace, mvrot, mvrotace, mvcir, mvcirace, mvrectsinu, mvrotsinu, mvcirsinu,
//   mvrectfile (mvfile, mvpredef), mvrotfile, mvnull, flash movements (negative duration),
//   chained by `next`, started by <begin> events (finish optional), in a tree of nested
//   <obj> / <objreal> objects (a parent's motion moves its children and their axes).
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
// JMatrix4::MulPoint
__device__ inline void m4_point(const M4d& m, const double* p, double* q) {
  const double x = m.a[0] * p[0] + m.a[1] * p[1] + m.a[2] * p[2] + m.a[3];
  const double y = m.a[4] * p[0] + m.a[5] * p[1] + m.a[6] * p[2] + m.a[7];
  const double z = m.a[8] * p[0] + m.a[9] * p[1] + m.a[10] * p[2] + m.a[11];
  q[0] = x;
  q[1] = y;
  q[2] = z;
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

// JMotionPos (JMotionPos.cpp:29-107, JMotionPos.h:52).
__device__ inline void mpos_reset(MPos& p) {
  p.simple = 1;
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
__device__ inline void mpos_tomatrix(MPos& p) {
  if (p.simple) {
    m4_mov(p.m, p.s[0], p.s[1], p.s[2]);
    p.simple = 0;
  }
}
__device__ inline void mpos_rotate(MPos& p, double ang, const double* p1, const double* p2) {
  mpos_tomatrix(p);
  const M4d r = m4_rot(ang, p1, p2);
  m4_mul(p.m, r);
}
__device__ inline void mpos_movemix(MPos& p, const MPos& q) {
  if (p.simple && !q.simple) mpos_tomatrix(p);
  if (q.simple) mpos_move(p, q.s[0], q.s[1], q.s[2]);
  else m4_mul(p.m, q.m);
}
__device__ inline void mpos_point(const MPos& p, double* x) {  // PointMove, in place
  if (p.simple) {
    x[0] = x[0] + p.s[0];
    x[1] = x[1] + p.s[1];
    x[2] = x[2] + p.s[2];
  } else {
    m4_point(p.m, x, x);
  }
}

// ---- motion program ----------------------------------------------------------------------
// JMotionMovActive (JMotionObj.cpp:40-208): ConfigData of a (next) movement.
__device__ inline void act_config(MotAct& a, const MotMov& mv, const double* __restrict__ data) {
  a.vel[0] = a.vel[1] = a.vel[2] = 0;
  a.velang = 0;
  a.phase[0] = a.phase[1] = a.phase[2] = 0;
  a.phaseuni = 0;
  a.dfindex = 0;
  a.dflast[0] = a.dflast[1] = a.dflast[2] = 0;
  a.dflastang = 0;
  switch (mv.type) {
    case SPH_MOV_RECT: a.vel[0] = mv.v[0]; a.vel[1] = mv.v[1]; a.vel[2] = mv.v[2]; break;
    case SPH_MOV_RECTACE: a.vel[0] = mv.v2[0]; a.vel[1] = mv.v2[1]; a.vel[2] = mv.v2[2]; break;
    case SPH_MOV_ROT: case SPH_MOV_CIR: a.velang = mv.ang; break;
    case SPH_MOV_ROTACE: case SPH_MOV_CIRACE: a.velang = mv.ang2; break;
    case SPH_MOV_RECTSINU:
      a.phase[0] = mv.phase[0]; a.phase[1] = mv.phase[1]; a.phase[2] = mv.phase[2];
      break;
    case SPH_MOV_ROTSINU: case SPH_MOV_CIRSINU: a.phaseuni = mv.ang3; break;
    case SPH_MOV_RECTFILE: {  // DfConfig(true): the table's first position
      const double* r = data + 4 * mv.dfirst;
      a.dflast[0] = r[1]; a.dflast[1] = r[2]; a.dflast[2] = r[3];
    } break;
    case SPH_MOV_ROTFILE: a.dflastang = data[4 * mv.dfirst + 1]; break;
    default: break;
  }
}
// JMotionMovActive constructor / NextMov: the flash flag and the finish of a movement that
// starts at a.start.
__device__ inline void act_span(MotAct& a, const MotMov& mv) {
  a.flash = mv.time < 0;
  a.finish = a.flash ? a.start : a.start + mv.time;
  if (a.eventfinish >= 0 && a.eventfinish < a.finish) a.finish = a.eventfinish;
}

// JMotionMovActive::BinarySearch (JMotionObj.cpp:112-139) over the times of a table.
__device__ unsigned df_search(unsigned size, const double* __restrict__ d, double t) {
  unsigned ret = 0;
  if (size > 1) {
    int ccen = 0, cmin = 0, cmax = int(size) - 1;
    while (cmin <= cmax) {
      ccen = ((cmax - cmin) / 2) + cmin;
      const double tc = d[4 * ccen];
      if (tc == t) cmin = cmax + 1;
      else if (t < tc) cmax = ccen - 1;
      else cmin = ccen + 1;
    }
    if (ccen && ccen < int(size) && t < d[4 * ccen]) ccen--;
    ret = unsigned(ccen);
    while (ret && t == d[4 * (ret - 1)]) ret--;
  }
  return ret;
}
// DfGetNewPos / DfGetNewAng (JMotionObj.cpp:144-178): the table interpolated at t, from the
// persistent index; k = 1 (x, y, z) or the angle column.
__device__ void df_value(MotAct& a, const MotMov& mv, const double* __restrict__ data, double t, double* out, int nk) {
  const double* d = data + 4 * mv.dfirst;
  const unsigned n = unsigned(mv.dn);
  unsigned idx = unsigned(a.dfindex);
  if (idx == 0) idx = df_search(n, d, t);
  while (idx < n && t > d[4 * idx]) idx++;
  a.dfindex = int(idx);
  if (idx >= n) {  // beyond the last instant: the last value
    for (int k = 0; k < nk; k++) out[k] = d[4 * (n - 1) + 1 + k];
  } else {
    const unsigned i0 = idx ? idx - 1 : 0;  // (the reference reads row -1 at t <= the first time)
    const double tfactor = (t - d[4 * i0]) / (d[4 * idx] - d[4 * i0]);
    for (int k = 0; k < nk; k++) {
      const double v0 = d[4 * i0 + 1 + k], v1 = d[4 * idx + 1 + k];
      out[k] = (nk == 1 || ((mv.fields >> k) & 1)) ? v0 + tfactor * (v1 - v0) : 0.0;
    }
  }
}

// One node: JMotionObj::ProcesTime (JMotionObj.cpp:368-580) for this object; its children
// follow it in the node order.  Returns modif (the object moved in [timestep, +dt)).
__device__ bool obj_proces_time(MotionDev& md, int oi, const MotMov* movs, const double* __restrict__ data,
                                double timestep, double dt) {
  MotObj& o = md.obj[oi];
  o.active = 1;
  const MotObj* par = o.parent >= 0 ? &md.obj[o.parent] : nullptr;
  if (par && par->moving)  // the parent's motion of this step moves every axis of the object
    for (int k = 0; k < md.naxis; k++)
      if (md.axis[k].obj == oi) {
        mpos_point(par->modpos, md.axis[k].p1);
        mpos_point(par->modpos, md.axis[k].p2);
      }
  bool modif = false;
  int na = o.na;
  if (na) {
    const double tstepfin = timestep + dt;
    mpos_reset(o.modpos);
    MPos& modpos = o.modpos;
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
        if (dtmov > 0 || amov.flash) {
          const double t = amov.flash ? -mv.time : dtmov;
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
              mpos_rotate(modpos, mv.ang * t, md.axis[mv.ax].p1, md.axis[mv.ax].p2);
              modif = true;
              break;
            case SPH_MOV_ROTACE: {
              const double at = mv.ang * t;
              mpos_rotate(modpos, amov.velang * t + 0.5 * at * t, md.axis[mv.ax].p1, md.axis[mv.ax].p2);
              amov.velang += at;
              modif = true;
            } break;
            case SPH_MOV_CIR:
            case SPH_MOV_CIRACE:
            case SPH_MOV_CIRSINU: {  // the reference point turns about the axis; the object follows it
              double ang;
              if (mv.type == SPH_MOV_CIR) {
                ang = mv.ang * t;
              } else if (mv.type == SPH_MOV_CIRACE) {
                const double at = mv.ang * t;
                ang = amov.velang * t + 0.5 * at * t;
                amov.velang += at;
              } else {
                double ph = amov.phaseuni;
                ang = mv.ang2 * sin(ph);
                ph += double(mv.ang * (3.14159265358979323846 + 3.14159265358979323846) * t);
                ang = mv.ang2 * sin(ph) - ang;
                amov.phaseuni = ph;
              }
              const M4d m = m4_rot(ang, md.axis[mv.ax].p1, md.axis[mv.ax].p2);
              MotAxis& r = md.axis[mv.rax];
              m4_point(m, r.p1, r.p2);
              mpos_move(modpos, r.p2[0] - r.p1[0], r.p2[1] - r.p1[1], r.p2[2] - r.p1[2]);
              r.p1[0] = r.p2[0];
              r.p1[1] = r.p2[1];
              r.p1[2] = r.p2[2];
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
              mpos_rotate(modpos, ang, md.axis[mv.ax].p1, md.axis[mv.ax].p2);
              amov.phaseuni = ph;
              modif = true;
            } break;
            case SPH_MOV_RECTFILE:
            case SPH_MOV_ROTFILE: {  // the table at the time since the movement began
              double tt = timestep - amov.start;
              if (tt < 0) tt = 0;
              tt += data[4 * mv.dfirst];
              tt += t;
              if (mv.type == SPH_MOV_RECTFILE) {
                double np[3];
                df_value(amov, mv, data, tt, np, 3);
                mpos_move(modpos, np[0] - amov.dflast[0], np[1] - amov.dflast[1], np[2] - amov.dflast[2]);
                amov.dflast[0] = np[0];
                amov.dflast[1] = np[1];
                amov.dflast[2] = np[2];
              } else {
                double na1;
                df_value(amov, mv, data, tt, &na1, 1);
                mpos_rotate(modpos, na1 - amov.dflastang, md.axis[mv.ax].p1, md.axis[mv.ax].p2);
                amov.dflastang = na1;
              }
              modif = true;
            } break;
            default: break;  // wait, null
          }
        }
        // chain to the next movement to consume the rest of dt (JMotionMovActive::NextMov)
        if ((dtover > 0 || dtmov == 0) && mv.nextidx >= 0) {
          const MotMov& nm = movs[mv.nextidx];
          if (!amov.flash) amov.start += mv.time;
          const double velp[3] = {amov.vel[0], amov.vel[1], amov.vel[2]};
          const double php[3] = {amov.phase[0], amov.phase[1], amov.phase[2]};
          const double velangp = amov.velang, phaseunip = amov.phaseuni;
          amov.mov = mv.nextidx;
          act_span(amov, nm);
          act_config(amov, nm, data);
          if (nm.prev) {
            if (nm.type == SPH_MOV_RECTACE) { amov.vel[0] = velp[0]; amov.vel[1] = velp[1]; amov.vel[2] = velp[2]; }
            if (nm.type == SPH_MOV_ROTACE || nm.type == SPH_MOV_CIRACE) amov.velang = velangp;
            if (nm.type == SPH_MOV_RECTSINU) { amov.phase[0] = php[0]; amov.phase[1] = php[1]; amov.phase[2] = php[2]; }
            if (nm.type == SPH_MOV_ROTSINU || nm.type == SPH_MOV_CIRSINU) amov.phaseuni = phaseunip;
          }
          dt2 = dtover;
          timestep2 = amov.start;
          if (timestep2 <= amov.finish || amov.flash) rep = true;
        }
      } while (rep);
      if (tstepfin > amov.finish) amov.del = 1;
    }
    o.na = na;
  }
  if (par && par->moving) {  // the parent's motion on top of the object's own
    if (modif) mpos_movemix(o.modpos, par->modpos);
    else o.modpos = par->modpos;
    modif = true;
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
// results in md->out[ref] (JMotionListData::Sp_Movedt, JMotionList.cpp:43-61).
__global__ void k_motion(const DevScalars* __restrict__ sc, MotionDev* __restrict__ md,
                         const MotMov* __restrict__ movs, const MotEvt* __restrict__ evts,
                         const double* __restrict__ data, double t0, double dt0) {
  if (threadIdx.x != 0) return;
  const double timestep = (t0 >= 0 ? t0 : sc->tstep0), dt = (t0 >= 0 ? dt0 : sc->last_dt);
  for (int r = 0; r < md->nref; r++) md->out[r].type = 0;  // PreMotion
  if (t0 < 0 && halted(sc)) return;  // a fatal error stopped the run: nothing moves
  // JMotion::ProcesTime (JMotion.cpp:446-468): start the events that begin before t+dt
  bool looking = true;
  for (int c = md->eventnext; c >= 0 && looking; c--) {
    const MotEvt& e = evts[c];
    if (e.start < timestep + dt) {
      MotObj& o = md->obj[e.obj];
      if (o.na < MOT_MAXACT) {  // JMotionObj::BeginEvent
        MotAct& a = o.act[o.na++];
        const MotMov& mv = movs[e.mov];
        a.mov = e.mov;
        a.start = e.start;
        a.eventfinish = e.finish;
        act_span(a, mv);
        a.del = 0;
        act_config(a, mv, data);
      } else {
        md->overflow = 1;
      }
      for (int q = e.obj; q >= 0 && !md->obj[q].active; q = md->obj[q].parent) md->obj[q].active = 1;
      md->eventnext--;
      md->objsactive = 1;
    } else {
      looking = false;
    }
  }
  if (md->objsactive) {
    md->objsactive = 0;
    // the top-level objects that are active, each followed by its whole subtree
    bool proc[MOT_MAXOBJ], modif[MOT_MAXOBJ];
    for (int i = 0; i < md->nobj; i++) {
      const int p = md->obj[i].parent;
      proc[i] = p < 0 ? md->obj[i].active != 0 : proc[p];
      modif[i] = proc[i] && obj_proces_time(*md, i, movs, data, timestep, dt);
    }
    // Active |= the children's (after each child's own subtree)
    for (int i = md->nobj - 1; i >= 0; i--) {
      const int p = md->obj[i].parent;
      if (proc[i] && p >= 0) md->obj[p].active |= md->obj[i].active;
    }
    for (int i = 0; i < md->nobj; i++)
      if (proc[i] && md->obj[i].parent < 0) md->objsactive |= md->obj[i].active;
    for (int i = 0; i < md->nobj; i++) {
      const MotObj& o = md->obj[i];
      if (!modif[i] || o.ref < 0) continue;
      MotOut& r = md->out[o.ref];
      if (o.modpos.simple) {
        r.type = 1;
        for (int k = 0; k < 3; k++) {
          r.mov[k] = o.modpos.s[k];
          r.vel[k] = o.modpos.s[k] / dt;
        }
      } else {
        r.type = 2;
        for (int k = 0; k < 12; k++) r.m[k] = o.modpos.m.a[k];
      }
    }
    // ProcesTimeSimple records the movements only when ProcesTime reports active objects
    if (!md->objsactive)
      for (int r = 0; r < md->nref; r++) md->out[r].type = 0;
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
  if (obj >= unsigned(md->nref)) return;
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
                   const MotMov* movs, const MotEvt* evts, const double* data, const PartArrays& a, float4* normal,
                   const DivGrid&) {
  hipLaunchKernelGGL(k_motion, dim3(1), dim3(64), 0, stm, sc, md, movs, evts, data, -1.0, 0.0);
  const unsigned nb = (npbcap + 255) / 256;
  if (nb) hipLaunchKernelGGL(k_move_bound, dim3(nb), dim3(256), 0, stm, sc, K, md, a, normal);
}

void launch_motion_advance(hipStream_t stm, DevScalars* sc, MotionDev* md, const MotMov* movs, const MotEvt* evts,
                           const double* data, double t0, double dt) {
  hipLaunchKernelGGL(k_motion, dim3(1), dim3(64), 0, stm, sc, md, movs, evts, data, t0, dt);
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
