// gencase_ref — dam-break case writer for the REFERENCE solver (test infrastructure).
//
// GenCase is a missing blob in the reference, so this tool writes
// the <case>.xml + <case>.bi4 pair that JSphCpuSingle loads (JSph::LoadCaseConfig,
// JSph.cpp:923; JPartsLoad4::LoadParticles, JPartsLoad4.cpp:151-252).  The .bi4 is
// written through the reference's own JPartDataBi4 (JPartDataBi4.cpp:183-237,305-378,429).
//
// The lattice/constants are the SURVEY §8(c) recipe, restated independently in
// dualsphysics_multilayer_amd/case_dambreak.py (the product-side generator); a CPU
// test checks that both produce the same particles bit for bit.
//
// usage: gencase_ref <dp> <outdir> <step:1=Verlet|2=Symplectic> <ddt:0..3> [timemax] [casename]
//                    [boundary:1=DBC|2=mDBC] [dim:3|2] [viscotreatment] [visco] [shifting] [shiftcoef]
//                    [shifttfs] [kernel] [sym:0|1]
//
// With boundary=2 the case also gets <casename>_Normals.nbi4, written through the
// reference's own JPartNormalData (JPartNormalData.cpp:178-207), as GenCase would: the
// final normal of each boundary particle points from the particle to the boundary limit,
// dp/2 beyond the wall layer towards the fluid (the sum of those vectors on edges and
// corners).  JSph::LoadBoundNormals/ConfigBoundNormals (JSph.cpp:1265-1340) read it.
#include "JPartDataBi4.h"
#include "JPartNormalData.h"
#include "Functions.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s dp outdir step ddt [timemax] [casename] [boundary] [dim] [viscotreatment] [visco] "
                    "[shifting] [shiftcoef] [shifttfs] [kernel] [sym]\n", argv[0]);
    return 1;
  }
  const double dp = atof(argv[1]);
  const std::string dir = argv[2];
  const int step = atoi(argv[3]);
  const int ddt = atoi(argv[4]);
  const double tmax = (argc > 5 ? atof(argv[5]) : 1.5);
  const std::string name = (argc > 6 ? argv[6] : "CaseDambreak");
  const int boundary = (argc > 7 ? atoi(argv[7]) : 1);
  // dim 2: the 2-D dam break of examples/main/01_DamBreak/CaseDambreakVal2D_Def.xml (tank
  // 4 x 3 in x-z with bottom, left and right walls, water column 1 x 2, y = 0, Visco 0.02)
  const int dim = (argc > 8 ? atoi(argv[8]) : 3);
  const bool d2 = (dim == 2);
  // viscosity and shifting (<parameters> ViscoTreatment/Visco, Shifting/ShiftCoef/ShiftTFS,
  // JSph.cpp:620-700): 1 artificial (default, Visco 0.1 / 0.02 in 2-D) or 2 Laminar+SPS
  const int tvisco = (argc > 9 ? atoi(argv[9]) : 1);
  const std::string visco = (argc > 10 ? argv[10] : (d2 ? "0.02" : "0.1"));
  const int shifting = (argc > 11 ? atoi(argv[11]) : 0);
  const std::string shiftcoef = (argc > 12 ? argv[12] : "-2");
  const std::string shifttfs = (argc > 13 ? argv[13] : "0");
  const int kernel = (argc > 14 ? atoi(argv[14]) : 2);  // 1 Cubic spline, 2 Wendland
  // sym 1: <parameter Symmetry> (JSph.cpp:714) on the half tank y >= 0: no y = 0 wall, the
  // fluid from y = 0 (the plane y = 0 mirrors the particles)
  const bool sym = (argc > 15 ? atoi(argv[15]) : 0) != 0;

  // 3-D: tank 1.6 x 0.67 x 0.4 (walls: bottom, x=0, x=L, y=0, y=W); water 0.4 x 0.67 x 0.3.
  const int nx = int(std::round((d2 ? 4.0 : 1.6) / dp)), ny = d2 ? 0 : int(std::round(0.67 / dp));
  const int nz = int(std::round((d2 ? 3.0 : 0.4) / dp));
  const int mx = int(std::round((d2 ? 1.0 : 0.4) / dp)), my = d2 ? 0 : int(std::round(0.67 / dp));
  const int mz = int(std::round((d2 ? 2.0 : 0.3) / dp));
  std::vector<tdouble3> pos, nor;
  for (int k = 0; k <= nz; k++)
    for (int j = 0; j <= ny; j++)
      for (int i = 0; i <= nx; i++)
        if (k == 0 || i == 0 || i == nx || (!d2 && ((j == 0 && !sym) || j == ny))) {
          pos.push_back(TDouble3(i * dp, j * dp, k * dp));
          const double hd = dp * 0.5;
          // 2-D: the particles sit at y = 0 and have no y walls (no y normal)
          const double ny_ = d2 ? 0. : (j == 0 ? (sym ? 0. : hd) : (j == ny ? -hd : 0.));
          nor.push_back(TDouble3(i == 0 ? hd : (i == nx ? -hd : 0.), ny_, k == 0 ? hd : 0.));
        }
  const unsigned nb = unsigned(pos.size());
  for (int k = 1; k <= mz; k++)
    for (int j = (d2 || sym ? 0 : 1); j < (d2 ? 1 : my); j++)
      for (int i = 1; i <= mx; i++) pos.push_back(TDouble3(i * dp, j * dp, k * dp));
  const unsigned np = unsigned(pos.size()), nf = np - nb;

  const double g = 9.81, rho0 = 1000., gamma = 7., coefsound = 20., coefh = 1.0;
  const double hswl = mz * dp;
  const double cs0 = coefsound * std::sqrt(g * hswl);
  const double b = cs0 * cs0 * rho0 / gamma;
  const double h = coefh * std::sqrt((d2 ? 2. : 3.) * dp * dp);  // JCaseCtes::ComputeFinalH
  const double mass = rho0 * dp * dp * (d2 ? 1.0 : dp);

  std::vector<unsigned> idp(np);
  std::vector<tfloat3> vel(np, TFloat3(0));
  std::vector<float> rhop(np);
  tdouble3 pmin = TDouble3(DBL_MAX), pmax = TDouble3(-DBL_MAX);
  for (unsigned p = 0; p < np; p++) {
    idp[p] = p;
    rhop[p] = (p < nb ? float(rho0) : float(rho0 * std::pow(1. + rho0 * g * (hswl - pos[p].z) / b, 1. / gamma)));
    pmin = MinValues(pmin, pos[p]);
    pmax = MaxValues(pmax, pos[p]);
  }

  JPartDataBi4 pd;
  pd.ConfigBasic(0, 1, "gencase_ref", "gencase_ref", name, d2, 0, dir);
  pd.ConfigParticles(np, nb, 0, 0, nf, pmin, pmax, false, false);
  pd.ConfigCtes(dp, h, b, rho0, gamma, mass, mass);
  pd.AddPartInfo(0, 0, np, 0, 0, 0, pmin, pmax, 0, 0);
  pd.AddPartData(np, idp.data(), pos.data(), vel.data(), rhop.data());
  pd.SaveFileCase(name);
  if (boundary == 2) {
    JPartNormalData nd;
    nd.ConfigBasic("gencase_ref", name, false, 0, dp, h, 2. * h);
    nd.AddNormalData("Plane", nb, nor.data());
    nd.SaveFile(dir);
  }

  FILE* f = fopen((dir + "/" + name + ".xml").c_str(), "w");
  if (!f) { perror("xml"); return 2; }
  fprintf(f, "<?xml version=\"1.0\" encoding=\"UTF-8\" ?>\n<case app=\"gencase_ref\">\n<execution>\n<constants>\n");
  fprintf(f, "%s\n<gravity x=\"0\" y=\"0\" z=\"%g\"/>\n<cflnumber value=\"0.2\"/>\n",
          d2 ? "<data2d value=\"true\"/>\n<data2dposy value=\"0\"/>" : "<data2d value=\"false\"/>", -g);
  fprintf(f, "<gamma value=\"%g\"/>\n<rhop0 value=\"%g\"/>\n<dp value=\"%.10g\"/>\n", gamma, rho0, dp);
  fprintf(f, "<h value=\"%.10E\"/>\n<b value=\"%.10E\"/>\n<massbound value=\"%.10E\"/>\n<massfluid value=\"%.10E\"/>\n", h, b, mass, mass);
  fprintf(f, "</constants>\n<particles np=\"%u\" nb=\"%u\" nbf=\"%u\" mkboundfirst=\"10\" mkfluidfirst=\"0\">\n", np, nb, nb);
  fprintf(f, "<fixed mkbound=\"0\" mk=\"10\" begin=\"0\" count=\"%u\"/>\n<fluid mkfluid=\"0\" mk=\"0\" begin=\"%u\" count=\"%u\"/>\n</particles>\n", nb, nb, nf);
  fprintf(f, "<parameters>\n");
  auto par = [&](const char* k, const std::string& v) { fprintf(f, "<parameter key=\"%s\" value=\"%s\"/>\n", k, v.c_str()); };
  par("StepAlgorithm", std::to_string(step));
  par("VerletSteps", "40");
  par("Kernel", std::to_string(kernel));
  par("ViscoTreatment", std::to_string(tvisco));
  par("Visco", visco);
  par("ViscoBoundFactor", "1");
  par("DensityDT", std::to_string(ddt));
  par("DensityDTvalue", "0.1");
  par("Shifting", std::to_string(shifting));
  if (shifting) {
    par("ShiftCoef", shiftcoef);
    par("ShiftTFS", shifttfs);
  }
  par("Boundary", std::to_string(boundary));
  if (boundary == 2) par("SlipMode", "1");
  if (sym) par("Symmetry", "1");
  par("RigidAlgorithm", "1");
  par("CoefDtMin", "0.05");
  par("DtIni", "0");
  par("DtMin", "0");
  par("TimeMax", fun::DoubleStr(tmax));
  par("TimeOut", "0.01");
  par("PartsOutMax", "1");
  par("RhopOutMin", "700");
  par("RhopOutMax", "1300");
  fprintf(f, "<simulationdomain><posmin x=\"default\" y=\"default\" z=\"default\"/>"
             "<posmax x=\"default\" y=\"default\" z=\"default + 50%%\"/></simulationdomain>\n");
  fprintf(f, "</parameters>\n</execution>\n</case>\n");
  fclose(f);
  printf("np=%u nb=%u nf=%u h=%.10g b=%.10g cs0=%.10g mass=%.10g\n", np, nb, nf, h, b, cs0, mass);
  return 0;
}
