// sph_solver.cpp — host orchestration (see sph_solver.hpp).
#include "sph_solver.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace sphx {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw SphError(SPH_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// ---- JSph::ConfigConstants1/2 (JSph.cpp:1392-1457), ConfigCellDivision (:1772-1788),
//      map limits (:2062-2076), SelecDomain/CalcCellCode (:1794-1829, JDsDcell.cpp:30-69) ----
static unsigned bits_for(unsigned v, unsigned minbits) {
  unsigned n = minbits;
  for (; v >> n; n++) {}
  return n;
}
static unsigned cell_code(unsigned nx, unsigned ny, unsigned nz) {
  unsigned sx = bits_for(nx, 2), sy = bits_for(ny, 2), sz = bits_for(nz, 2);
  const unsigned smin = sx + sy + sz;
  if (smin > 31) return 0;
  for (unsigned rest = 31 - smin; rest;) {
    if (rest) { sx++; rest--; }
    if (rest) { sy++; rest--; }
    if (rest) { sz++; rest--; }
  }
  return ((sx + 1) << 25) | (sy << 20) | (sz << 15) | ((sy + sz) << 10) | ((sx + 1 + sz) << 5) | (sx + 1 + sy);
}

void derive_constants(const SphCaseDef& c, SphConstants& k) {
  if (c.kernel != SPH_KERNEL_WENDLAND) throw SphError(SPH_ERR_UNSUPPORTED, "only the Wendland kernel is implemented");
  if (c.cellmode != SPH_CELLMODE_FULL)
    throw SphError(SPH_ERR_UNSUPPORTED, "only CellMode=Full is implemented on the GPU path");
  if (c.step_algorithm != SPH_STEP_VERLET && c.step_algorithm != SPH_STEP_SYMPLECTIC)
    throw SphError(SPH_ERR_ARG, "invalid step algorithm");
  if (c.tdensity < 0 || c.tdensity > 3) throw SphError(SPH_ERR_ARG, "invalid DDT mode");
  if (c.npb > c.np) throw SphError(SPH_ERR_ARG, "npb > np");
  std::memset(&k, 0, sizeof(k));
  k.kernelh = float(c.h);
  k.cteb = float(c.cteb);
  k.gamma = float(c.gamma);
  k.rhopzero = float(c.rhop0);
  k.massfluid = float(c.massfluid);
  k.massbound = float(c.massbound);
  for (int i = 0; i < 3; i++) k.gravity[i] = float(c.gravity[i]);
  k.cflnumber = c.cflnumber;
  k.dp = c.dp;
  k.visco = float(c.visco);
  k.viscoboundfactor = float(c.viscoboundfactor);
  k.rhopoutmin = float(c.rhopoutmin);
  k.rhopoutmax = float(c.rhopoutmax);
  k.tdensity = c.tdensity;
  k.step_algorithm = c.step_algorithm;
  k.verlet_steps = c.verlet_steps;
  const double h = k.kernelh;
  k.kernelsize = float(h * 2.0f);  // Wendland factor 2 (FunSphKernel.h:190)
  k.kernelsize2 = k.kernelsize * k.kernelsize;
  k.awen = float(0.41778 / (h * h * h));
  k.bwen = float(-2.08891 / (h * h * h * h));
  k.cs0 = std::sqrt(double(k.gamma) * double(k.cteb) / double(k.rhopzero));
  k.eta2 = float((h * 0.1) * (h * 0.1));
  k.ovrhopzero = 1.0f / k.rhopzero;
  k.ddtkh = k.kernelsize * float(c.ddtvalue);
  k.ddtgz = float(double(k.rhopzero) * double(std::fabs(k.gravity[2])) / double(k.cteb));
  k.dtini = c.dtini ? c.dtini : k.kernelh / k.cs0;
  k.dtmin = c.dtmin ? c.dtmin : (k.kernelh / k.cs0) * float(c.coefdtmin);
  k.scelldiv = 1;
  k.scell = k.kernelsize / k.scelldiv;
  k.movlimit = k.scell * 0.9f;
  for (int i = 0; i < 3; i++) {
    k.map_realposmin[i] = c.map_realposmin[i];
    k.map_realsize[i] = c.map_realposmax[i] - c.map_realposmin[i];
    k.dom_posmin[i] = c.map_realposmin[i];
    if (!(k.map_realsize[i] > 0)) throw SphError(SPH_ERR_ARG, "invalid map limits");
    k.dom_cells[i] = unsigned(std::ceil(k.map_realsize[i] / k.scell));
  }
  k.dom_cellcode = cell_code(k.dom_cells[0] + 1, k.dom_cells[1] + 1, k.dom_cells[2] + 1);
  if (!k.dom_cellcode) throw SphError(SPH_ERR_ARG, "failed to select a valid CellCode");
}

static KConst make_kconst(const SphConstants& c) {
  KConst K;
  std::memset(&K, 0, sizeof(K));
  K.kernelh = c.kernelh;
  K.kernelsize2 = c.kernelsize2;
  K.bwen = c.bwen;
  K.ovkernelh = 1.0f / c.kernelh;
  K.cteb = c.cteb;
  K.gamma = c.gamma;
  K.rhopzero = c.rhopzero;
  K.ovrhopzero = c.ovrhopzero;
  K.massfluid = c.massfluid;
  K.massbound = c.massbound;
  K.eta2 = c.eta2;
  K.ddtkh = c.ddtkh;
  K.ddtgz = c.ddtgz;
  K.cs0f = float(c.cs0);
  K.visco = c.visco;
  K.viscobound = c.visco * c.viscoboundfactor;
  K.scell = c.scell;
  K.movlimit = c.movlimit;
  K.rhopoutmin = c.rhopoutmin;
  K.rhopoutmax = c.rhopoutmax;
  K.gravx = c.gravity[0];
  K.gravy = c.gravity[1];
  K.gravz = c.gravity[2];
  K.ovgamma = 1.f / c.gamma;
  K.gravxd = c.gravity[0];
  K.gravyd = c.gravity[1];
  K.gravzd = c.gravity[2];
  K.map_realposmin_x = c.map_realposmin[0];
  K.map_realposmin_y = c.map_realposmin[1];
  K.map_realposmin_z = c.map_realposmin[2];
  K.map_realsize_x = c.map_realsize[0];
  K.map_realsize_y = c.map_realsize[1];
  K.map_realsize_z = c.map_realsize[2];
  K.scelld = double(c.scell);
  K.domcellcode = c.dom_cellcode;
  K.tdensity = c.tdensity;
  K.mhalfovh = -0.5f * K.ovkernelh;
  K.bwenovh = c.bwen * K.ovkernelh;
  K.ddtkhcs = c.ddtkh * K.cs0f;
  {  // binomial coefficients of (1+x)^(1/gamma) - 1
    const double a = 1.0 / double(c.gamma);
    K.ddtc1 = float(a);
    K.ddtc2 = float(a * (a - 1) / 2);
    K.ddtc3 = float(a * (a - 1) * (a - 2) / 6);
    K.ddtc4 = float(a * (a - 1) * (a - 2) * (a - 3) / 24);
  }
  return K;
}

// Full-map cell grid (JCellDivCpuSingle::PrepareNct, JCellDivCpuSingle.cpp:105-121, with CellDomFixed).
static DivGrid make_grid(const SphConstants& c) {
  DivGrid g;
  g.ncx = int(c.dom_cells[0]);
  g.ncy = int(c.dom_cells[1]);
  g.ncz = int(c.dom_cells[2]);
  g.nsheet = unsigned(g.ncx) * unsigned(g.ncy);
  const unsigned long long nct = (unsigned long long)g.nsheet * unsigned(g.ncz);
  if (nct * 2 + 6 >= (1ull << 31)) throw SphError(SPH_ERR_ARG, "the number of cells is too big");
  g.nct = unsigned(nct);
  g.boxboundignore = g.nct;
  g.boxfluid = g.boxboundignore + 1;
  g.boxboundout = g.boxfluid + g.nct;
  g.boxfluidout = g.boxboundout + 1;
  g.boxboundoutignore = g.boxfluidout + 1;
  g.boxfluidoutignore = g.boxboundoutignore + 1;
  g.nctt = g.nct * 2 + 6;
  return g;
}

SphGpuSingle::SphGpuSingle(const SphCaseDef& cdef, const SphParticlesHost& init, int dev) : device(dev) {
  derive_constants(cdef, C);
  K = make_kconst(C);
  G = make_grid(C);
  step_algorithm_ = cdef.step_algorithm;
  if (init.n != cdef.np) throw SphError(SPH_ERR_ARG, "particle count does not match the case");
  if (!init.n) throw SphError(SPH_ERR_ARG, "no particles");
  cap_ = init.n;
  npb0_ = cdef.npb;
  keybits_ = bits_for(G.boxfluidoutignore, 1);
  if (const char* e = std::getenv("SPH_INTERACTION")) tiled_ = std::string(e) != "simple";
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
  try {
    Alloc();
    Upload(init);
    // ConfigDomain: RunCellDivide(true) (JSphCpuSingle.cpp:165-166), then InitRunGpu.
    RunCellDivide();
    if (step_algorithm_ == SPH_STEP_VERLET)
      check_hip(hipMemcpyAsync(cur_.velrhopm1, cur_.velrhop, sizeof(float4) * cap_, hipMemcpyDeviceToDevice, stream),
                "init VelrhopM1");
    Sync();
    CheckErrors();
  } catch (...) {
    Free();
    hipStreamDestroy(stream);
    throw;
  }
}

SphGpuSingle::~SphGpuSingle() {
  if (stream) hipStreamSynchronize(stream);
  Free();
  for (auto& e : pending_) { hipEventDestroy(e.a); hipEventDestroy(e.b); }
  for (auto e : evpool_) hipEventDestroy(e);
  if (stream) hipStreamDestroy(stream);
}

void SphGpuSingle::Alloc() {
  auto dmalloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    check_hip(hipMalloc(&p, std::max<size_t>(bytes, 256)), "hipMalloc");
    allocs_.push_back(p);
    return p;
  };
  const size_t n = cap_;
  for (PartArrays* a : {&cur_, &alt_}) {
    a->idp = (unsigned*)dmalloc(4 * n);
    a->code = (typecode*)dmalloc(2 * n);
    a->dcell = (unsigned*)dmalloc(4 * n);
    a->posxy = (double2*)dmalloc(16 * n);
    a->posz = (double*)dmalloc(8 * n);
    a->velrhop = (float4*)dmalloc(16 * n);
    if (step_algorithm_ == SPH_STEP_VERLET) {
      a->velrhopm1 = (float4*)dmalloc(16 * n);
    } else {
      a->posxypre = (double2*)dmalloc(16 * n);
      a->poszpre = (double*)dmalloc(8 * n);
      a->velrhoppre = (float4*)dmalloc(16 * n);
    }
  }
  poscell_ = (float4*)dmalloc(16 * n);
  press_ = (float*)dmalloc(4 * n);
  arace_ = (float4*)dmalloc(16 * n);
  begincell_ = (unsigned*)dmalloc(4 * size_t(G.nctt));
  items_ = (uint4*)dmalloc(16 * (2 * size_t(G.nct) + 1));
  rowtmp_ = (unsigned*)dmalloc(4 * 2 * size_t(G.ncy) * size_t(G.ncz));
  qctr_ = (unsigned*)dmalloc(4 * 8);
  for (int i = 0; i < 2; i++) {
    sort_.keys[i] = (unsigned*)dmalloc(4 * n);
    sort_.vals[i] = (unsigned*)dmalloc(4 * n);
  }
  sort_.ntiles = unsigned((n + RS_TILE - 1) / RS_TILE);
  sort_.hist = (unsigned*)dmalloc(4 * size_t(sort_.ntiles) * (1u << RS_MAXBITS));
  sort_.digtot = (unsigned*)dmalloc(4 * (1u << RS_MAXBITS));
  sc_ = (DevScalars*)dmalloc(sizeof(DevScalars));
  dttrace_ = (double*)dmalloc(8 * size_t(tracecap_));
  pairs_ = (unsigned long long*)dmalloc(8 * 6);
  check_hip(hipHostMalloc((void**)&sc_host_, sizeof(DevScalars), hipHostMallocDefault), "hipHostMalloc");
}

void SphGpuSingle::Free() {
  for (void* p : allocs_) hipFree(p);
  allocs_.clear();
  if (sc_host_) hipHostFree(sc_host_);
  sc_host_ = nullptr;
}

void SphGpuSingle::Upload(const SphParticlesHost& h) {
  const unsigned n = h.n;
  std::vector<unsigned> dcell(n);
  std::vector<typecode> code(n);
  std::vector<double2> pxy(n);
  std::vector<double> pz(n);
  std::vector<float4> vr(n);
  for (unsigned p = 0; p < n; p++) {
    const double x = h.pos[3 * p], y = h.pos[3 * p + 1], z = h.pos[3 * p + 2];
    pxy[p] = make_double2(x, y);
    pz[p] = z;
    vr[p] = make_float4(h.vel[3 * p], h.vel[3 * p + 1], h.vel[3 * p + 2], h.rhop[p]);
    // LoadCodeParticles (JSph.cpp:1257): the case has one fixed and one fluid MK block.
    code[p] = (p < npb0_ ? typecode(0) : CODE_TYPE_FLUID);
    // JSph::CheckRhopLimits (JSph.cpp:2021-2030).
    if (p >= npb0_ && (vr[p].w < C.rhopoutmin || C.rhopoutmax < vr[p].w))
      throw SphError(SPH_ERR_ARG, "Initial fluid density is out of limits.");
    // JSph::LoadDcellParticles (JSph.cpp:1690-1711).
    const double dx = x - C.dom_posmin[0], dy = y - C.dom_posmin[1], dz = z - C.dom_posmin[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0 && dx < C.map_realsize[0] && dy < C.map_realsize[1] && dz < C.map_realsize[2]))
      throw SphError(SPH_ERR_ARG, "Found new particles out.");
    dcell[p] = DcelCell(C.dom_cellcode, unsigned(dx / double(C.scell)), unsigned(dy / double(C.scell)),
                        unsigned(dz / double(C.scell)));
  }
  check_hip(hipMemcpy(cur_.idp, h.idp, 4 * size_t(n), hipMemcpyHostToDevice), "upload idp");
  check_hip(hipMemcpy(cur_.code, code.data(), 2 * size_t(n), hipMemcpyHostToDevice), "upload code");
  check_hip(hipMemcpy(cur_.dcell, dcell.data(), 4 * size_t(n), hipMemcpyHostToDevice), "upload dcell");
  check_hip(hipMemcpy(cur_.posxy, pxy.data(), 16 * size_t(n), hipMemcpyHostToDevice), "upload posxy");
  check_hip(hipMemcpy(cur_.posz, pz.data(), 8 * size_t(n), hipMemcpyHostToDevice), "upload posz");
  check_hip(hipMemcpy(cur_.velrhop, vr.data(), 16 * size_t(n), hipMemcpyHostToDevice), "upload velrhop");
  DevScalars s;
  std::memset(&s, 0, sizeof(s));
  s.np = n;
  s.npb = npb0_;
  s.npbok = npb0_;
  s.symdtpre = C.dtini;  // InitRun (JSph.cpp:2090)
  check_hip(hipMemcpy(sc_, &s, sizeof(s), hipMemcpyHostToDevice), "upload scalars");
  verletstep_ = 0;
}

// ---- timing -----------------------------------------------------------------------
void SphGpuSingle::SetTiming(bool on) {
  Sync();
  timing_ = on;
  for (int i = 0; i < 4; i++) { phase_ms_[i] = 0; phase_n_[i] = 0; }
}
void SphGpuSingle::TimedBegin(int phase) {
  (void)phase;
  if (!timing_) return;
  hipEvent_t a;
  if (!evpool_.empty()) { a = evpool_.back(); evpool_.pop_back(); }
  else check_hip(hipEventCreate(&a), "hipEventCreate");
  check_hip(hipEventRecord(a, stream), "hipEventRecord");
  cur_a_ = a;
}
void SphGpuSingle::TimedEnd(int phase) {
  if (!timing_) return;
  hipEvent_t b;
  if (!evpool_.empty()) { b = evpool_.back(); evpool_.pop_back(); }
  else check_hip(hipEventCreate(&b), "hipEventCreate");
  check_hip(hipEventRecord(b, stream), "hipEventRecord");
  pending_.push_back(Ev{cur_a_, b, phase});
}
void SphGpuSingle::Timing(double out_ms[4], uint64_t* launches) {
  Sync();
  for (auto& e : pending_) {
    float ms = 0;
    check_hip(hipEventElapsedTime(&ms, e.a, e.b), "hipEventElapsedTime");
    phase_ms_[e.phase] += ms;
    phase_n_[e.phase]++;
    evpool_.push_back(e.a);
    evpool_.push_back(e.b);
  }
  pending_.clear();
  for (int i = 0; i < 4; i++) out_ms[i] = phase_n_[i] ? phase_ms_[i] / double(phase_n_[i]) : 0.0;
  if (launches) *launches = phase_n_[0];
}

// ---- phases ------------------------------------------------------------------------
void SphGpuSingle::RunCellDivide() {
  TimedBegin(2);
  launch_presort(stream, cap_, sc_, cur_.dcell, cur_.code, G, C.dom_cellcode, sort_.keys[0], sort_.vals[0]);
  const int res = launch_radix_sort(stream, cap_, sc_, sort_, keybits_);
  launch_begincell(stream, cap_, sc_, sort_.keys[res], G, begincell_);
  const bool withm1 = (step_algorithm_ == SPH_STEP_VERLET);
  launch_gather(stream, cap_, sc_, sort_.vals[res], cur_, alt_, withm1, havepre_, K, C.dom_posmin, poscell_, press_);
  std::swap(cur_, alt_);
  if (tiled_) launch_items(stream, sc_, begincell_, G, rowtmp_, items_, qctr_);
  TimedEnd(2);
}

void SphGpuSingle::Interaction_Forces(int interstep) {
  (void)interstep;  // mDBC / shifting are not on this path
  TimedBegin(0);
  if (tiled_) {
    check_hip(hipMemsetAsync(qctr_, 0, 4 * 8, stream), "reset work counters");
    // Boundary rows without fluid neighbours are skipped by the tiled kernel: their ar=0.
    check_hip(hipMemsetAsync(arace_, 0, sizeof(float4) * npb0_, stream), "zero boundary arace");
    launch_fluid_tiled(stream, nblocks_tiled_, sc_, items_, qctr_, poscell_, cur_.velrhop, press_, begincell_, G, K,
                       arace_);
  } else {
    launch_interaction(stream, cap_, sc_, poscell_, cur_.velrhop, press_, begincell_, G, K, arace_);
  }
  TimedEnd(0);
}

void SphGpuSingle::DtVariable(int mode) {
  launch_dt(stream, sc_, K, C.cflnumber, C.dtmin, C.cs0, mode, dttrace_, tracecap_);
}

void SphGpuSingle::ComputeVerlet() {
  TimedBegin(1);
  verletstep_++;
  const bool euler = !(verletstep_ < C.verlet_steps);
  launch_verlet(stream, cap_, sc_, K, euler, arace_, cur_);
  if (euler) verletstep_ = 0;
  std::swap(cur_.velrhop, cur_.velrhopm1);
  TimedEnd(1);
}

void SphGpuSingle::ComputeSymplecticPre() {
  TimedBegin(1);
  std::swap(cur_.posxy, cur_.posxypre);
  std::swap(cur_.posz, cur_.poszpre);
  std::swap(cur_.velrhop, cur_.velrhoppre);
  havepre_ = true;
  launch_sym_pre(stream, cap_, sc_, K, arace_, cur_);
  TimedEnd(1);
}

void SphGpuSingle::ComputeSymplecticCorr() {
  TimedBegin(1);
  launch_sym_cor(stream, cap_, sc_, K, arace_, cur_);
  havepre_ = false;
  TimedEnd(1);
}

void SphGpuSingle::ComputeStep() {
  if (step_algorithm_ == SPH_STEP_VERLET) {
    Interaction_Forces(1);
    DtVariable(DT_VERLET);
    ComputeVerlet();
  } else {
    Interaction_Forces(2);
    DtVariable(DT_SYM_PRE);
    ComputeSymplecticPre();
    RunCellDivide();
    Interaction_Forces(3);
    DtVariable(DT_SYM_COR);
    ComputeSymplecticCorr();
  }
  RunCellDivide();
}

void SphGpuSingle::Run(unsigned nsteps) {
  for (unsigned s = 0; s < nsteps; s++) ComputeStep();
  check_hip(hipGetLastError(), "kernel launch");
}

void SphGpuSingle::Sync() { check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize"); }

SphRunStats SphGpuSingle::Stats() {
  check_hip(hipMemcpyAsync(sc_host_, sc_, sizeof(DevScalars), hipMemcpyDeviceToHost, stream), "read scalars");
  Sync();
  const DevScalars& s = *sc_host_;
  SphRunStats r;
  std::memset(&r, 0, sizeof(r));
  r.time = s.time;
  r.last_dt = s.last_dt;
  r.sym_dtpre = s.symdtpre;
  r.nstep = s.nstep;
  r.np = s.np;
  r.npb = s.npb;
  r.npbok = s.npbok;
  r.nout = s.nout;
  r.dtmodif = s.dtmodif;
  r.error_flags = s.error_flags;
  r.velmax = s.last_velmax;
  r.acemax = s.last_acemax;
  r.viscdtmax = s.last_viscdt;
  return r;
}

void SphGpuSingle::CheckErrors() {
  const SphRunStats s = Stats();
  if (s.error_flags & ERR_BOUNDOUT) throw SphError(SPH_ERR_BOUNDOUT, "boundary particles were excluded (AbortBoundOut)");
  if (s.error_flags & ERR_DT_NAN) throw SphError(SPH_ERR_DT, "The computed Dt is NaN or infinity");
}

unsigned SphGpuSingle::DtTrace(double* out, unsigned cap) {
  const SphRunStats s = Stats();
  const unsigned n = unsigned(std::min<unsigned long long>(s.nstep, tracecap_));
  if (out && cap) {
    std::vector<double> all(tracecap_);
    check_hip(hipMemcpy(all.data(), dttrace_, 8 * size_t(tracecap_), hipMemcpyDeviceToHost), "read dt trace");
    const unsigned long long first = s.nstep - n;
    for (unsigned i = 0; i < n && i < cap; i++) out[i] = all[(first + i) % tracecap_];
  }
  return n;
}

void SphGpuSingle::Download(SphParticlesHost& out) {
  const SphRunStats s = Stats();
  const unsigned n = s.np;
  if (out.n < n) throw SphError(SPH_ERR_ARG, "output buffer too small");
  std::vector<double2> pxy(n);
  std::vector<double> pz(n);
  std::vector<float4> vr(n);
  check_hip(hipMemcpy(pxy.data(), cur_.posxy, 16 * size_t(n), hipMemcpyDeviceToHost), "download posxy");
  check_hip(hipMemcpy(pz.data(), cur_.posz, 8 * size_t(n), hipMemcpyDeviceToHost), "download posz");
  check_hip(hipMemcpy(vr.data(), cur_.velrhop, 16 * size_t(n), hipMemcpyDeviceToHost), "download velrhop");
  if (out.idp) check_hip(hipMemcpy(out.idp, cur_.idp, 4 * size_t(n), hipMemcpyDeviceToHost), "download idp");
  if (out.code) check_hip(hipMemcpy(out.code, cur_.code, 2 * size_t(n), hipMemcpyDeviceToHost), "download code");
  for (unsigned p = 0; p < n; p++) {
    if (out.pos) { out.pos[3 * p] = pxy[p].x; out.pos[3 * p + 1] = pxy[p].y; out.pos[3 * p + 2] = pz[p]; }
    if (out.vel) { out.vel[3 * p] = vr[p].x; out.vel[3 * p + 1] = vr[p].y; out.vel[3 * p + 2] = vr[p].z; }
    if (out.rhop) out.rhop[p] = vr[p].w;
  }
  out.n = n;
}

void SphGpuSingle::DownloadInteraction(SphInterOut& out) {
  // Runs one interaction on the current state (like or_interaction) and reads ar/ace back.
  // Maxima accumulated so far (VelMax from the last divide) are kept for this call.
  Interaction_Forces(1);
  DtVariable(DT_PEEK);
  const SphRunStats s = Stats();
  std::vector<float4> a(s.np);
  check_hip(hipMemcpy(a.data(), arace_, 16 * size_t(s.np), hipMemcpyDeviceToHost), "download arace");
  for (unsigned p = 0; p < s.np; p++) {
    if (out.ar) out.ar[p] = a[p].w;
    if (out.ace) { out.ace[3 * p] = a[p].x; out.ace[3 * p + 1] = a[p].y; out.ace[3 * p + 2] = a[p].z; }
  }
  out.velmax = s.velmax;
  out.acemax = s.acemax;
  out.viscdtmax = s.viscdtmax;
  // Leave the device maxima as a fresh interaction would find them (VelMax stays:
  // it belongs to the last divide).
  check_hip(hipMemsetAsync(&sc_->red[RED_ACEMAX2][0], 0, 4 * RED_SLOTS, stream), "reset acemax");
  check_hip(hipMemsetAsync(&sc_->red[RED_VISCDT][0], 0, 4 * RED_SLOTS, stream), "reset viscdt");
  Sync();
}

void SphGpuSingle::CountPairs(uint64_t out[6]) {
  check_hip(hipMemsetAsync(pairs_, 0, 8 * 6, stream), "memset pairs");
  launch_count_pairs(stream, cap_, sc_, poscell_, begincell_, G, K, pairs_);
  unsigned long long h[6];
  check_hip(hipMemcpyAsync(h, pairs_, 8 * 6, hipMemcpyDeviceToHost, stream), "read pairs");
  Sync();
  for (int i = 0; i < 6; i++) out[i] = h[i];
}

}  // namespace sphx
