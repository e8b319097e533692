// sph_capi.cpp — extern "C" boundary (include/sphcore.h) over sphx::SphGpuSingle.
#include <cstring>
#include <string>

#include "sph_solver.hpp"

struct SphSolver {
  sphx::SphGpuSingle* impl;
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
    *out = new SphSolver{impl};
  });
}

int sph_solver_destroy(SphSolver* s) {
  if (!s) return SPH_OK;
  const int r = guard([&] { delete s->impl; });
  delete s;
  return r;
}

int sph_divide(SphSolver* s) {
  NEED(s);
  return guard([&] { s->impl->RunCellDivide(); });
}
int sph_interaction_forces(SphSolver* s, int interstep) {
  NEED(s && interstep >= 1 && interstep <= 3);
  return guard([&] { s->impl->Interaction_Forces(interstep); });
}
int sph_compute_dt(SphSolver* s, int final_) {
  NEED(s);
  return guard([&] { s->impl->DtVariable(final_ ? sphx::DT_VERLET : sphx::DT_PEEK); });
}
int sph_step_verlet(SphSolver* s) {
  NEED(s);
  return guard([&] { s->impl->ComputeVerlet(); });
}
int sph_step_symplectic_pre(SphSolver* s) {
  NEED(s);
  return guard([&] { s->impl->ComputeSymplecticPre(); });
}
int sph_step_symplectic_cor(SphSolver* s) {
  NEED(s);
  return guard([&] { s->impl->ComputeSymplecticCorr(); });
}
int sph_solver_run(SphSolver* s, uint32_t nsteps) {
  NEED(s);
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
  return guard([&] { s->impl->DownloadInteraction(*out); });
}
int sph_count_pairs(SphSolver* s, uint64_t out[6]) {
  NEED(s && out);
  return guard([&] { s->impl->CountPairs(out); });
}
int sph_solver_set_timing(SphSolver* s, int enabled) {
  NEED(s);
  return guard([&] { s->impl->SetTiming(enabled != 0); });
}
int sph_solver_timing(SphSolver* s, double out_ms[4], uint64_t* launches) {
  NEED(s && out_ms);
  return guard([&] { s->impl->Timing(out_ms, launches); });
}

}  // extern "C"
