// host_loop.cpp — a compiled C++ host on the C-ABI of the MI355X core.
//
// What a JSphAmdSingle : JSph would do around libsphcore.so, as a standalone program:
// load a dam-break case (<case>.xml + <case>.bi4, the files oracle/tools/gencase_ref writes
// for the reference), derive SphCaseDef as JSph::LoadCaseConfig / LoadCaseParticles do,
// run the JSphGpuSingle::Run loop through sph_solver_create / sph_solver_run /
// sph_download_particles, and write the state as reference PART files (sph_part_write),
// which tests/test_cpp_host.py compares with the reference's own PARTs.
//
//   host_loop <case path without extension> <outdir> <step1> [<step2> ...]
//   -> <outdir>/Part_0001.bi4 after step1 steps, Part_0002.bi4 after step2, ...
//
// Build: g++ -O2 -std=c++17 -I<repo>/include host_loop.cpp -L<repo>/dualsphysics_multilayer_amd/lib
//        -lsphcore -Wl,-rpath,<repo>/dualsphysics_multilayer_amd/lib -o host_loop
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "sphcore.h"

static void Check(int st, const char* where) {  // RunExceptionGpuDef.h:27 analogue
  if (st != SPH_OK) throw std::runtime_error(std::string(where) + ": " + sph_last_error());
}

// Minimal XML value lookup for the case files gencase_ref writes (JXml's role).
struct CaseXml {
  std::string text;
  explicit CaseXml(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    text = ss.str();
  }
  std::string attr_after(size_t pos, const char* attr) const {
    const std::string key = std::string(attr) + "=\"";
    const size_t a = text.find(key, pos);
    if (a == std::string::npos) throw std::runtime_error(std::string("missing attribute ") + attr);
    const size_t b = text.find('"', a + key.size());
    return text.substr(a + key.size(), b - a - key.size());
  }
  double constant(const char* name) const {  // <constants><name value="..."/>
    const size_t p = text.find(std::string("<") + name + " ");
    if (p == std::string::npos) throw std::runtime_error(std::string("missing constant ") + name);
    return std::atof(attr_after(p, "value").c_str());
  }
  double gravity(const char* axis) const { return std::atof(attr_after(text.find("<gravity "), axis).c_str()); }
  double parameter(const char* key, double def) const {  // <parameter key="..." value="..."/>
    const size_t p = text.find(std::string("<parameter key=\"") + key + "\"");
    return p == std::string::npos ? def : std::atof(attr_after(p, "value").c_str());
  }
};

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <case> <outdir> <step1> [step2 ...]\n", argv[0]);
    return 2;
  }
  try {
    const std::string casepath = argv[1], outdir = argv[2];
    if (sph_abi_version() != SPH_ABI_VERSION) throw std::runtime_error("libsphcore ABI version mismatch");
    // ---- JSph::LoadCaseParticles: the particles of <case>.bi4 (JPartsLoad4) ----
    SphPartHeader hdr;
    std::memset(&hdr, 0, sizeof(hdr));
    Check(sph_part_read((casepath + ".bi4").c_str(), &hdr, nullptr), "read case header");
    const uint32_t np = hdr.npok;
    std::vector<uint32_t> idp(np);
    std::vector<double> pos(3 * size_t(np));
    std::vector<float> vel(3 * size_t(np)), rhop(np);
    SphParticlesHost parts = {np, idp.data(), pos.data(), vel.data(), rhop.data(), nullptr, nullptr};
    Check(sph_part_read((casepath + ".bi4").c_str(), &hdr, &parts), "read case particles");
    // ---- JSph::LoadCaseConfig: constants and parameters (JSph.cpp:567-760) ----
    const CaseXml xml(casepath + ".xml");
    SphCaseDef cd;
    std::memset(&cd, 0, sizeof(cd));
    cd.dp = xml.constant("dp");
    cd.h = xml.constant("h");
    cd.cteb = xml.constant("b");
    cd.rhop0 = xml.constant("rhop0");
    cd.gamma = xml.constant("gamma");
    cd.massbound = xml.constant("massbound");
    cd.massfluid = xml.constant("massfluid");
    cd.gravity[0] = xml.gravity("x");
    cd.gravity[1] = xml.gravity("y");
    cd.gravity[2] = xml.gravity("z");
    cd.cflnumber = xml.constant("cflnumber");
    cd.step_algorithm = int(xml.parameter("StepAlgorithm", 1));
    cd.verlet_steps = int(xml.parameter("VerletSteps", 40));
    cd.kernel = int(xml.parameter("Kernel", 2));
    cd.tdensity = int(xml.parameter("DensityDT", 0));
    cd.visco = xml.parameter("Visco", 0);
    cd.viscoboundfactor = xml.parameter("ViscoBoundFactor", 1);
    cd.ddtvalue = xml.parameter("DensityDTvalue", 0.1);
    cd.coefdtmin = xml.parameter("CoefDtMin", 0.05);
    cd.dtini = xml.parameter("DtIni", 0);
    cd.dtmin = xml.parameter("DtMin", 0);
    cd.rhopoutmin = xml.parameter("RhopOutMin", 700);
    cd.rhopoutmax = xml.parameter("RhopOutMax", 1300);
    cd.cellmode = SPH_CELLMODE_FULL;
    cd.tboundary = SPH_BOUND_DBC;
    cd.npb = uint32_t(hdr.case_nfixed);
    cd.np = np;
    // map limits: JPartsLoad4::CalculeLimits with border double(float(h))*BORDER_MAP, then
    // JSph::ResizeMapLimits with the case's <posmax z="default + 50%"> (JSph.cpp:2056-2059)
    const double border = double(float(cd.h)) * 0.05;
    for (int i = 0; i < 3; i++) {
      cd.map_realposmin[i] = hdr.case_posmin[i] - border;
      cd.map_realposmax[i] = hdr.case_posmax[i] + border;
    }
    cd.map_realposmax[2] += (cd.map_realposmax[2] - cd.map_realposmin[2]) * 0.5;
    // ---- JSphGpuSingle::Run: the step loop stays on the device ----
    SphSolver* s = nullptr;
    Check(sph_solver_create(&cd, &parts, /*device*/ 0, &s), "create");
    uint32_t done = 0;
    for (int a = 3; a < argc; a++) {
      const uint32_t target = uint32_t(std::atoi(argv[a]));
      if (target > done) Check(sph_solver_run(s, target - done), "run");
      done = target;
      SphRunStats st;
      Check(sph_solver_stats(s, &st), "stats");  // synchronises
      SphParticlesHost out = {st.np, idp.data(), pos.data(), vel.data(), rhop.data(), nullptr, nullptr};
      Check(sph_download_particles(s, &out), "download");  // ParticlesDataDown -> SaveData
      SphPartHeader ph = hdr;
      std::snprintf(ph.app_name, sizeof(ph.app_name), "host_loop (libsphcore C-ABI)");
      ph.cpart = uint32_t(a - 2);
      ph.npok = out.n;
      ph.nout = st.nout;
      ph.step = uint32_t(st.nstep);
      ph.timestep = st.time;
      ph.pos_double = 1;
      char fn[64];
      std::snprintf(fn, sizeof(fn), "/Part_%04u.bi4", ph.cpart);
      Check(sph_part_write((outdir + fn).c_str(), &ph, &out), "write PART");
      std::printf("Part_%04u step=%u time=%.9g np=%u nout=%u\n", ph.cpart, ph.step, ph.timestep, out.n, st.nout);
    }
    Check(sph_solver_destroy(s), "destroy");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "host_loop: %s\n", e.what());
    return 1;
  }
  return 0;
}
