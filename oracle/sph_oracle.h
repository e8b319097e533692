/*
 * sph_oracle.h — C API of the CPU ORACLE (test infrastructure only).
 *
 * A restatement of the reference CPU path (JSphCpu / JSphCpuSingle /
 * JCellDivCpuSingle of DualSPHysics v5.2) for the dam-break feature set:
 * Wendland kernel, artificial viscosity, DDT none/Molteni/Fourtakas, DBC,
 * Verlet and Symplectic, no floating/periodic/shifting/inout.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline — never as the
 * product path.  It shares the SphCaseDef/SphParticlesHost/SphRunStats/
 * SphInterOut PODs of include/sphcore.h so the two read the same inputs.
 */
#ifndef SPH_ORACLE_H
#define SPH_ORACLE_H
#include "../include/sphcore.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrSolver OrSolver;

const char* or_last_error(void);
int or_case_derive(const SphCaseDef* cdef, SphConstants* out);
int or_create(const SphCaseDef* cdef, const SphParticlesHost* init, int nthreads, OrSolver** out);
int or_destroy(OrSolver* s);
/* nsteps x (ComputeStep + RunCellDivide), JSphCpuSingle::Run (JSphCpuSingle.cpp:1090-1120). */
int or_run(OrSolver* s, uint32_t nsteps);
int or_stats(OrSolver* s, SphRunStats* out);
int or_dt_trace(OrSolver* s, double* out, uint32_t cap, uint32_t* count);
/* Current particle state, in the solver's (cell-sorted) order. */
int or_download(OrSolver* s, SphParticlesHost* out);
/* PreInteraction_Forces + Interaction_Forces on the current state; the state
 * itself is not advanced.  interstep: 1 Verlet, 2 SymPredictor, 3 SymCorrector. */
int or_interaction(OrSolver* s, int interstep, SphInterOut* out);
/* JDsPips-style pair counts on the current state: {ff_chk, ff_real, fb_chk, fb_real, bf_chk, bf_real}. */
int or_count_pairs(OrSolver* s, uint64_t out[6]);
/* Wall seconds spent inside or_run's step loop (for the CPU baseline). */
double or_run_seconds(OrSolver* s);
int or_threads(OrSolver* s);

#ifdef __cplusplus
}
#endif
#endif
