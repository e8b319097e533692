// sph_capi.cpp — extern "C" boundary (include/sphcore.h) over sphx::SphGpuSingle.
#include <cstring>
#include <string>
#include <vector>

#include "sph_solver.hpp"

struct SphSolver {
  sphx::SphGpuSingle* impl;
  bool member;  // borrowed from a SphSlabGroup: data-out calls only
};

struct SphSlabGroup {
  sphx::SphSlabGroup* impl;
  std::vector<SphSolver> members;
};

namespace {
thread_local std::string g_last_error;

template <class F>
int guard(F&& f) {
  try {
    f();
    return SPH_OK;
  } catch (const sphx::SphError& e) {
    g_last_error = e.what();
    return e.status;
  } catch (const std::bad_alloc&) {
    g_last_error = "out of host memory";
    return SPH_ERR_NOMEM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return SPH_ERR_STATE;
  }
}
#define NOT_MEMBER(s)                                                               \
  do {                                                                              \
    if ((s)->member) {                                                              \
      g_last_error = "slab group member: step the group (sph_slab_group_run)";     \
      return SPH_ERR_STATE;                                                         \
    }                                                                               \
  } while (0)
#define NEED(x)                                   \
  do {                                            \
    if (!(x)) {                                   \
      g_last_error = "invalid argument: " #x;     \
      return SPH_ERR_ARG;                         \
    }                                             \
  } while (0)
}  // namespace

extern "C" {

int sph_abi_version(void) { return SPH_ABI_VERSION; }
const char* sph_last_error(void) { return g_last_error.c_str(); }

int sph_case_derive(const SphCaseDef* cdef, SphConstants* out) {
  NEED(cdef && out);
  return guard([&] { sphx::derive_constants(*cdef, *out); });
}

int sph_solver_create(const SphCaseDef* cdef, const SphParticlesHost* init, int device, SphSolver** out) {
  NEED(cdef && init && out);
  NEED(init->idp && init->pos && init->vel && init->rhop);
  return guard([&] {
    auto* impl = new sphx::SphGpuSingle(*cdef, *init, device);
    *out = new SphSolver{impl, false};
  });
}

int sph_solver_destroy(SphSolver* s) {
  if (!s) return SPH_OK;
  NOT_MEMBER(s);
  const int r = guard([&] { delete s->impl; });
  delete s;
  return r;
}

int sph_divide(SphSolver* s) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->RunCellDivide(); });
}
int sph_interaction_forces(SphSolver* s, int interstep) {
  NEED(s && interstep >= 1 && interstep <= 3);
  NOT_MEMBER(s);
  return guard([&] { s->impl->Interaction_Forces(interstep); });
}
int sph_compute_dt(SphSolver* s, int final_) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->DtVariable(final_ ? sphx::DT_VERLET : sphx::DT_PEEK); });
}
int sph_step_verlet(SphSolver* s) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->ComputeVerlet(); });
}
int sph_step_symplectic_pre(SphSolver* s) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->ComputeSymplecticPre(); });
}
int sph_step_symplectic_cor(SphSolver* s) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->ComputeSymplecticCorr(); });
}
int sph_solver_run(SphSolver* s, uint32_t nsteps) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->Run(nsteps); });
}
int sph_solver_sync(SphSolver* s) {
  NEED(s);
  return guard([&] {
    s->impl->Sync();
    s->impl->CheckErrors();
  });
}
int sph_solver_stats(SphSolver* s, SphRunStats* out) {
  NEED(s && out);
  return guard([&] { *out = s->impl->Stats(); });
}
int sph_solver_dt_trace(SphSolver* s, double* out, uint32_t cap, uint32_t* count) {
  NEED(s && count);
  return guard([&] { *count = s->impl->DtTrace(out, cap); });
}
int sph_download_particles(SphSolver* s, SphParticlesHost* out) {
  NEED(s && out);
  return guard([&] { s->impl->Download(*out); });
}
int sph_download_interaction(SphSolver* s, SphInterOut* out) {
  NEED(s && out);
  NOT_MEMBER(s);
  return guard([&] { s->impl->DownloadInteraction(*out); });
}
int sph_count_pairs(SphSolver* s, uint64_t out[6]) {
  NEED(s && out);
  return guard([&] { s->impl->CountPairs(out); });
}
int sph_solver_set_time(SphSolver* s, double time, double symplectic_dtpre) {
  NEED(s);
  return guard([&] { s->impl->SetTime(time, symplectic_dtpre); });
}
int sph_solver_set_motion(SphSolver* s, uint32_t nobj, uint32_t nmov, const SphMotionMov* movs, uint32_t nevt,
                          const SphMotionEvent* evts) {
  NEED(s);
  return guard([&] { s->impl->SetMotion(nobj, nmov, movs, nevt, evts); });
}
int sph_solver_set_motion_tree(SphSolver* s, uint32_t nnode, const SphMotionObj* nodes, uint32_t nmov,
                               const SphMotionMov* movs, uint32_t nevt, const SphMotionEvent* evts, uint32_t nrows,
                               const double* rows) {
  NEED(s && nodes && (rows || !nrows));
  return guard([&] { s->impl->SetMotionTree(nnode, nodes, nmov, movs, nevt, evts, nrows, rows); });
}
int sph_solver_set_floatings(SphSolver* s, uint32_t nft, const SphFloatingDef* defs, double ftpause) {
  NEED(s && defs);
  return guard([&] { s->impl->SetFloatings(nft, defs, ftpause); });
}
int sph_solver_set_floating_table(SphSolver* s, uint32_t body, int32_t kind, uint32_t n, const double* times,
                                  const double* values) {
  NEED(s && times && values);
  return guard([&] { s->impl->SetFloatingTable(body, kind, n, times, values); });
}
int sph_solver_floatings(SphSolver* s, uint32_t cap, SphFloatingState* out, uint32_t* nft) {
  NEED(s);
  return guard([&] {
    const unsigned n = s->impl->Floatings(out, cap);
    if (nft) *nft = n;
  });
}
int sph_partfloat_write(const char* path, const char* app, uint32_t mkboundfirst, uint32_t nft,
                        const uint16_t* mkbound, const uint32_t* begin, const uint32_t* count, const float* mass,
                        const float* massp, const float* radius, uint32_t nparts, const uint32_t* cpart,
                        const uint32_t* step, const double* timestep, const double* center, const float* fvel,
                        const float* fomega, const float* facelin, const float* faceang) {
  NEED(path && nft && mkbound && begin && count && mass && massp && radius && (!nparts || (cpart && step &&
       timestep && center && fvel && fomega && facelin && faceang)));
  return guard([&] {
    sphx::partfloat_write(path, app, mkboundfirst, nft, mkbound, begin, count, mass, massp, radius, nparts, cpart,
                          step, timestep, center, fvel, fomega, facelin, faceang);
  });
}
int sph_partfloat_read(const char* path, uint32_t cpart, uint32_t nft, double* center, float* fvel, float* fomega,
                       double* timestep) {
  NEED(path && nft);
  return guard([&] { sphx::partfloat_read(path, cpart, nft, center, fvel, fomega, timestep); });
}
int sph_extra_normals_read(const char* path, uint32_t casenbound, uint32_t casenfloat, uint32_t cap, float* normals,
                           uint32_t* nsize, int32_t* usenormalsft) {
  NEED(path && nsize);
  return guard([&] { *nsize = sphx::extra_normals_read(path, casenbound, casenfloat, cap, normals, usenormalsft); });
}
int sph_extra_normals_write(const char* path, const char* app, uint32_t cpart, uint32_t step, double timestep,
                            uint32_t casenbound, uint32_t casenfloat, int32_t usenormalsft, uint32_t nsize,
                            const float* normals) {
  NEED(path && (normals || !nsize));
  return guard([&] {
    sphx::extra_normals_write(path, app, cpart, step, timestep, casenbound, casenfloat, usenormalsft, nsize, normals);
  });
}
int sph_download_normals(SphSolver* s, uint32_t cap, float* normals, uint32_t* n, int32_t* usenormalsft) {
  NEED(s && n);
  return guard([&] {
    int ft = 0;
    *n = s->impl->DownloadNormals(normals, cap, &ft);
    if (usenormalsft) *usenormalsft = ft;
  });
}
int sph_solver_set_timing(SphSolver* s, int enabled) {
  NEED(s);
  return guard([&] { s->impl->SetTiming(enabled != 0); });
}
int sph_solver_set_timing_phases(SphSolver* s, unsigned mask) {
  NEED(s);
  return guard([&] { s->impl->SetTimingPhases(mask); });
}
int sph_solver_timing(SphSolver* s, double out_ms[4], uint64_t* launches) {
  NEED(s && out_ms);
  return guard([&] { s->impl->Timing(out_ms, launches); });
}

int sph_slab_partition(const SphCaseDef* cdef, const SphParticlesHost* all, int nranks, double bound_weight,
                       int32_t* cx_bounds) {
  return sph_slab_partition_axis(cdef, all, nranks, bound_weight, 0, cx_bounds);
}
int sph_slab_partition_axis(const SphCaseDef* cdef, const SphParticlesHost* all, int nranks, double bound_weight,
                            int axis, int32_t* bounds) {
  NEED(cdef && all && all->pos && bounds && nranks >= 1);
  return guard([&] { sphx::slab_partition(*cdef, *all, nranks, bound_weight, bounds, axis); });
}

int sph_comm_unique_id(unsigned char id[128]) {
  NEED(id);
  return guard([&] { sphx::rccl_unique_id(id); });
}

int sph_slab_create(const SphCaseDef* cdef, const SphParticlesHost* all, int device, const SphSlabDef* slab,
                    SphSolver** out) {
  NEED(cdef && all && slab && out);
  NEED(all->idp && all->pos && all->vel && all->rhop);
  return guard([&] {
    sphx::check_hip(hipSetDevice(device), "hipSetDevice");
    sphx::SlabConfig sc;
    sc.rank = slab->rank;
    sc.nranks = slab->nranks;
    sc.c0 = slab->cx_begin;
    sc.c1 = slab->cx_end;
    sc.axis = slab->axis;
    auto tr = sphx::make_rccl_transport(slab->comm_id, slab->rank, slab->nranks);
    auto* impl = new sphx::SphGpuSingle(*cdef, *all, device, sc, std::move(tr));
    try {
      impl->ShareDeviceCheck();  // overlap off for ranks that share a GPU (collective)
    } catch (...) {
      delete impl;
      throw;
    }
    *out = new SphSolver{impl, false};
  });
}

int sph_slab_create_shm(const SphCaseDef* cdef, const SphParticlesHost* all, int device, const SphSlabDef* slab,
                        const char* shm_name, uint64_t slot_bytes, SphSolver** out) {
  NEED(cdef && all && slab && out && shm_name && slot_bytes);
  NEED(all->idp && all->pos && all->vel && all->rhop);
  return guard([&] {
    sphx::check_hip(hipSetDevice(device), "hipSetDevice");
    sphx::SlabConfig sc;
    sc.rank = slab->rank;
    sc.nranks = slab->nranks;
    sc.c0 = slab->cx_begin;
    sc.c1 = slab->cx_end;
    sc.axis = slab->axis;
    auto tr = sphx::make_shm_transport(shm_name, slab->rank, slab->nranks, slot_bytes);
    auto* impl = new sphx::SphGpuSingle(*cdef, *all, device, sc, std::move(tr));
    try {
      impl->ShareDeviceCheck();  // overlap off for ranks that share a GPU (collective)
    } catch (...) {
      delete impl;
      throw;
    }
    *out = new SphSolver{impl, false};
  });
}

int sph_slab_group_create(const SphCaseDef* cdef, const SphParticlesHost* all, int nslabs, const int32_t* devices,
                          const int32_t* cx_bounds, SphSlabGroup** out) {
  return sph_slab_group_create_axis(cdef, all, nslabs, devices, 0, cx_bounds, out);
}
int sph_slab_group_create_axis(const SphCaseDef* cdef, const SphParticlesHost* all, int nslabs,
                               const int32_t* devices, int axis, const int32_t* bounds, SphSlabGroup** out) {
  NEED(cdef && all && devices && bounds && out && nslabs >= 1);
  NEED(all->idp && all->pos && all->vel && all->rhop);
  return guard([&] {
    std::vector<int> dev(devices, devices + nslabs), b(bounds, bounds + nslabs + 1);
    auto* impl = new sphx::SphSlabGroup(*cdef, *all, nslabs, dev.data(), b.data(), axis);
    auto* g = new SphSlabGroup{impl, {}};
    for (auto& sl : impl->slabs) g->members.push_back(SphSolver{sl.get(), true});
    *out = g;
  });
}

int sph_slab_group_destroy(SphSlabGroup* g) {
  if (!g) return SPH_OK;
  const int r = guard([&] { delete g->impl; });
  delete g;
  return r;
}

int sph_slab_group_run(SphSlabGroup* g, uint32_t nsteps) {
  NEED(g);
  return guard([&] { g->impl->Run(nsteps); });
}

int sph_slab_set_repartition(SphSolver* s, uint32_t every, double bound_weight, double tolerance) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->SetRepartition(every, bound_weight, tolerance); });
}

int sph_slab_group_set_repartition(SphSlabGroup* g, uint32_t every, double bound_weight, double tolerance) {
  NEED(g);
  return guard([&] {
    for (auto& m : g->impl->slabs) m->SetRepartition(every, bound_weight, tolerance);
  });
}

int sph_solver_set_time_table(SphSolver* s, int32_t kind, uint32_t n, const double* times, const double* values) {
  NEED(s);
  return guard([&] { s->impl->SetTimeTable(kind, n, times, values); });
}

int sph_slab_set_overlap(SphSolver* s, int on) {
  NEED(s);
  NOT_MEMBER(s);
  return guard([&] { s->impl->SetOverlap(on != 0); });
}

int sph_slab_group_set_overlap(SphSlabGroup* g, int on) {
  NEED(g);
  return guard([&] {
    for (auto& m : g->impl->slabs) m->SetOverlap(on != 0);
  });
}

int sph_slab_info(SphSolver* s, SphSlabInfo* out) {
  NEED(s && out);
  return guard([&] {
    const sphx::SlabConfig c = s->impl->Slab();
    std::memset(out, 0, sizeof(*out));
    out->rank = c.rank;
    out->nranks = c.nranks;
    out->cx_begin = c.c0;
    out->cx_end = c.c1;
    out->axis = c.axis;
    out->repartitions = s->impl->RepartitionCount();
    out->last_imbalance = s->impl->LastImbalance();
  });
}

int sph_slab_group_member(SphSlabGroup* g, int i, SphSolver** out) {
  NEED(g && out && i >= 0 && size_t(i) < g->members.size());
  *out = &g->members[size_t(i)];
  return SPH_OK;
}

int sph_part_read(const char* path, SphPartHeader* hdr, SphParticlesHost* out) {
  NEED(path && hdr);
  return guard([&] { sphx::part_read(path, *hdr, out); });
}

int sph_part_write(const char* path, const SphPartHeader* hdr, const SphParticlesHost* parts) {
  NEED(path && hdr && parts);
  return guard([&] { sphx::part_write(path, *hdr, *parts); });
}

int sph_part_head_write(const char* path, const SphPartHeader* hdr) {
  NEED(path && hdr);
  return guard([&] { sphx::part_head_write(path, *hdr); });
}

int sph_normals_read(const char* path, uint32_t cap, double* out, uint32_t* nbound) {
  NEED(path && nbound);
  return guard([&] { *nbound = sphx::normals_read(path, cap, out); });
}

int sph_normals_write(const char* path, const char* case_name, double dp, double h, double dist, uint32_t nbound,
                      const double* normals) {
  NEED(path && (normals || !nbound));
  return guard([&] { sphx::normals_write(path, case_name, dp, h, dist, nbound, normals); });
}

int sph_bi4_rewrite(const char* src, const char* dst) {
  NEED(src && dst);
  return guard([&] { sphx::bi4_rewrite(src, dst); });
}

}  // extern "C"
