// genflume_ref — wave-flume case writer for the REFERENCE solver (test infrastructure).
//
// The BASELINE cfg4 case: a flume with a piston wavemaker, a flap at
// the far end and a floating box.  GenCase is a missing blob, so like gencase_ref this
// tool writes the <case>.xml + <case>.bi4 pair that JSph::LoadCaseConfig (JSph.cpp:923)
// and JPartsLoad4 (JPartsLoad4.cpp:151-252) read, the .bi4 through the reference's own
// JPartDataBi4 (JPartDataBi4.cpp:183-237,305-378,429).
//
// Blocks, in the order JSphMk::Config (JSphMk.cpp:86-123) and JCaseParts require:
//   fixed   mkbound 0  bottom + the two side walls
//   moving  mkbound 1  piston (x = 2dp), <motion> ref 0: mvrectsinu along x
//   moving  mkbound 2  flap (x = L), <motion> ref 1: wait, then mvrotsinu about the
//                      hinge line (L, y, 0)   (JMotion::ReadXml, JMotion.cpp:556-700)
//   floating mkbound 3 a box of rhopbody 500 at the free surface (JCasePartBlock_Floating,
//                      JCaseParts.cpp:248-290: massbody, masspart, center, inertia)
//   fluid   mkfluid 0  still water of depth d, minus the box
// With boundary=2 (mDBC) the fixed/moving walls get normals (<case>_Normals.nbi4,
// JPartNormalData.cpp:178-207) pointing to the boundary limit dp/2 towards the fluid; with
// ftnormals=1 the floating box's outer layer gets them too (from the particle to the nearest
// point of the box's boundary limit, dp/2 outside it: a face, edge or corner point), which
// makes the reference apply mDBC to the floating body (UseNormalsFt, JSph.cpp:1301-1306).
//
// usage: genflume_ref <dp> <outdir> <step:1|2> <ddt:0..3> [timemax] [casename] [boundary:1|2]
//                     [L W H depth] [flapwait flapfreq flapampl] [ftnormals:0|1] [nofloat:0|1]
// nofloat=1: no floating box (the water fills its place), e.g. for Symmetry, which the
// reference refuses with floating bodies.
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
    fprintf(stderr, "usage: %s dp outdir step ddt [timemax] [casename] [boundary] [L W H depth] [flapwait flapfreq flapampl]\n",
            argv[0]);
    return 1;
  }
  const double dp = atof(argv[1]);
  const std::string dir = argv[2];
  const int step = atoi(argv[3]);
  const int ddt = atoi(argv[4]);
  const double tmax = (argc > 5 ? atof(argv[5]) : 1.0);
  const std::string name = (argc > 6 ? argv[6] : "CaseFlume");
  const int boundary = (argc > 7 ? atoi(argv[7]) : 1);
  const double L = (argc > 8 ? atof(argv[8]) : 1.2), W = (argc > 9 ? atof(argv[9]) : 0.3);
  const double H = (argc > 10 ? atof(argv[10]) : 0.4), D = (argc > 11 ? atof(argv[11]) : 0.2);
  // flap motion: wait, then mvrotsinu of this frequency (Hz) and amplitude (degrees)
  const std::string fwait = (argc > 12 ? argv[12] : "0.004"), ffreq = (argc > 13 ? argv[13] : "2"),
                    fampl = (argc > 14 ? argv[14] : "3");
  const bool ftnormals = (argc > 15 ? atoi(argv[15]) != 0 : false);
  const bool nofloat = (argc > 16 ? atoi(argv[16]) != 0 : false);

  const int nx = int(std::round(L / dp)), ny = int(std::round(W / dp)), nz = int(std::round(H / dp));
  const int kd = int(std::round(D / dp));
  const int ip = 2;  // piston plane
  // floating box: half-size nbh lattice spacings, centred at x = 0.55 L, mid-width,
  // its centre one spacing below the free surface
  const int nbh = std::max(2, int(std::round(0.03 / dp)));
  const int bic = int(std::round(0.55 * L / dp)), bjc = ny / 2, bkc = kd - 1;
  auto inbox = [&](int i, int j, int k) {
    return !nofloat && std::abs(i - bic) <= nbh && std::abs(j - bjc) <= nbh && std::abs(k - bkc) <= nbh;
  };
  const double hd = dp * 0.5;
  std::vector<tdouble3> pos, nor;
  // fixed: bottom (k=0) and side walls (j=0, j=ny), x from 0 to L
  for (int k = 0; k <= nz; k++)
    for (int j = 0; j <= ny; j++)
      for (int i = 0; i <= nx; i++)
        if (k == 0 || j == 0 || j == ny) {
          pos.push_back(TDouble3(i * dp, j * dp, k * dp));
          nor.push_back(TDouble3(0., j == 0 ? hd : (j == ny ? -hd : 0.), k == 0 ? hd : 0.));
        }
  const unsigned nfixed = unsigned(pos.size());
  // piston
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j < ny; j++) {
      pos.push_back(TDouble3(ip * dp, j * dp, k * dp));
      nor.push_back(TDouble3(hd, 0., 0.));
    }
  const unsigned npiston = unsigned(pos.size()) - nfixed;
  // flap
  for (int k = 1; k <= nz; k++)
    for (int j = 1; j < ny; j++) {
      pos.push_back(TDouble3(nx * dp, j * dp, k * dp));
      nor.push_back(TDouble3(-hd, 0., 0.));
    }
  const unsigned nflap = unsigned(pos.size()) - nfixed - npiston;
  const unsigned npb = unsigned(pos.size());
  // floating box
  tdouble3 bcen = TDouble3(0);
  for (int k = bkc - nbh; k <= bkc + nbh && !nofloat; k++)
    for (int j = bjc - nbh; j <= bjc + nbh; j++)
      for (int i = bic - nbh; i <= bic + nbh; i++) {
        pos.push_back(TDouble3(i * dp, j * dp, k * dp));
        tdouble3 n = TDouble3(0);
        if (ftnormals && boundary == 2) {  // outer layer: towards the nearest limit point
          n.x = (i - bic == nbh ? hd : (bic - i == nbh ? -hd : 0.));
          n.y = (j - bjc == nbh ? hd : (bjc - j == nbh ? -hd : 0.));
          n.z = (k - bkc == nbh ? hd : (bkc - k == nbh ? -hd : 0.));
        }
        nor.push_back(n);
        bcen = bcen + pos.back();
      }
  const unsigned nfloat = unsigned(pos.size()) - npb;
  if (nfloat) bcen = bcen / double(nfloat);
  const unsigned nbound = unsigned(pos.size());
  // fluid
  for (int k = 1; k <= kd; k++)
    for (int j = 1; j < ny; j++)
      for (int i = ip + 1; i < nx; i++)
        if (!inbox(i, j, k)) pos.push_back(TDouble3(i * dp, j * dp, k * dp));
  const unsigned np = unsigned(pos.size()), nf = np - nbound;

  const double g = 9.81, rho0 = 1000., gamma = 7., coefsound = 20., coefh = 1.0;
  const double hswl = kd * dp;
  const double cs0 = coefsound * std::sqrt(g * hswl);
  const double b = cs0 * cs0 * rho0 / gamma;
  const double h = coefh * std::sqrt(3. * dp * dp);
  const double mass = rho0 * dp * dp * dp;
  const double rhopbody = 500.;
  const double massp = rhopbody * dp * dp * dp, massbody = massp * nfloat;
  double ixx = 0, iyy = 0, izz = 0;
  for (unsigned p = npb; p < nbound; p++) {
    const tdouble3 r = pos[p] - bcen;
    ixx += massp * (r.y * r.y + r.z * r.z);
    iyy += massp * (r.x * r.x + r.z * r.z);
    izz += massp * (r.x * r.x + r.y * r.y);
  }

  std::vector<unsigned> idp(np);
  std::vector<tfloat3> vel(np, TFloat3(0));
  std::vector<float> rhop(np);
  tdouble3 pmin = TDouble3(DBL_MAX), pmax = TDouble3(-DBL_MAX);
  for (unsigned p = 0; p < np; p++) {
    idp[p] = p;
    rhop[p] = (p < nbound ? float(rho0) : float(rho0 * std::pow(1. + rho0 * g * (hswl - pos[p].z) / b, 1. / gamma)));
    pmin = MinValues(pmin, pos[p]);
    pmax = MaxValues(pmax, pos[p]);
  }

  JPartDataBi4 pd;
  pd.ConfigBasic(0, 1, "genflume_ref", "genflume_ref", name, false, 0, dir);
  pd.ConfigParticles(np, nfixed, npiston + nflap, nfloat, nf, pmin, pmax, false, false);
  pd.ConfigCtes(dp, h, b, rho0, gamma, mass, mass);
  pd.AddPartInfo(0, 0, np, 0, 0, 0, pmin, pmax, 0, 0);
  pd.AddPartData(np, idp.data(), pos.data(), vel.data(), rhop.data());
  pd.SaveFileCase(name);
  if (boundary == 2) {
    JPartNormalData nd;
    nd.ConfigBasic("genflume_ref", name, false, 0, dp, h, 2. * h);
    nd.AddNormalData("Plane", nbound, nor.data());
    nd.SaveFile(dir);
  }

  FILE* f = fopen((dir + "/" + name + ".xml").c_str(), "w");
  if (!f) { perror("xml"); return 2; }
  fprintf(f, "<?xml version=\"1.0\" encoding=\"UTF-8\" ?>\n<case app=\"genflume_ref\">\n<execution>\n<constants>\n");
  fprintf(f, "<data2d value=\"false\"/>\n<gravity x=\"0\" y=\"0\" z=\"%g\"/>\n<cflnumber value=\"0.2\"/>\n", -g);
  fprintf(f, "<gamma value=\"%g\"/>\n<rhop0 value=\"%g\"/>\n<dp value=\"%.10g\"/>\n", gamma, rho0, dp);
  fprintf(f, "<h value=\"%.10E\"/>\n<b value=\"%.10E\"/>\n<massbound value=\"%.10E\"/>\n<massfluid value=\"%.10E\"/>\n", h, b, mass, mass);
  fprintf(f, "</constants>\n");
  // JMotion::ReadXml (JMotion.cpp:556-700); objreal ref k drives the k-th moving block.
  fprintf(f, "<motion>\n");
  fprintf(f, "<objreal ref=\"0\"><begin mov=\"1\" start=\"0\"/>\n"
             "<mvrectsinu id=\"1\" duration=\"100\" anglesunits=\"degrees\"><freq x=\"1.5\" y=\"0\" z=\"0\"/>"
             "<ampl x=\"0.02\" y=\"0\" z=\"0\"/><phase x=\"0\" y=\"0\" z=\"0\"/></mvrectsinu>\n</objreal>\n");
  fprintf(f, "<objreal ref=\"1\"><begin mov=\"1\" start=\"0\"/>\n<wait id=\"1\" duration=\"%s\" next=\"2\"/>\n"
             "<mvrotsinu id=\"2\" duration=\"100\" anglesunits=\"degrees\"><axisp1 x=\"%.10g\" y=\"0\" z=\"0\"/>"
             "<axisp2 x=\"%.10g\" y=\"1\" z=\"0\"/><freq v=\"%s\"/><ampl v=\"%s\"/><phase v=\"0\"/></mvrotsinu>\n"
             "</objreal>\n", fwait.c_str(), nx * dp, nx * dp, ffreq.c_str(), fampl.c_str());
  fprintf(f, "</motion>\n");
  fprintf(f, "<particles np=\"%u\" nb=\"%u\" nbf=\"%u\" mkboundfirst=\"10\" mkfluidfirst=\"0\">\n", np, nbound, nfixed);
  fprintf(f, "<fixed mkbound=\"0\" mk=\"10\" begin=\"0\" count=\"%u\"/>\n", nfixed);
  fprintf(f, "<moving mkbound=\"1\" mk=\"11\" begin=\"%u\" count=\"%u\" refmotion=\"0\"/>\n", nfixed, npiston);
  fprintf(f, "<moving mkbound=\"2\" mk=\"12\" begin=\"%u\" count=\"%u\" refmotion=\"1\"/>\n", nfixed + npiston, nflap);
  if (nfloat) {
    fprintf(f, "<floating mkbound=\"3\" mk=\"13\" begin=\"%u\" count=\"%u\">\n", npb, nfloat);
    fprintf(f, "<massbody value=\"%.17g\"/>\n<masspart value=\"%.17g\"/>\n", massbody, massp);
    fprintf(f, "<center x=\"%.17g\" y=\"%.17g\" z=\"%.17g\"/>\n", bcen.x, bcen.y, bcen.z);
    fprintf(f, "<inertia x=\"%.17g\" y=\"%.17g\" z=\"%.17g\"/>\n</floating>\n", ixx, iyy, izz);
  }
  fprintf(f, "<fluid mkfluid=\"0\" mk=\"0\" begin=\"%u\" count=\"%u\"/>\n</particles>\n", nbound, nf);
  fprintf(f, "<parameters>\n");
  auto par = [&](const char* k, const std::string& v) { fprintf(f, "<parameter key=\"%s\" value=\"%s\"/>\n", k, v.c_str()); };
  par("StepAlgorithm", std::to_string(step));
  par("VerletSteps", "40");
  par("Kernel", "2");
  par("ViscoTreatment", "1");
  par("Visco", "0.1");
  par("ViscoBoundFactor", "1");
  par("DensityDT", std::to_string(ddt));
  par("DensityDTvalue", "0.1");
  par("Shifting", "0");
  par("Boundary", std::to_string(boundary));
  if (boundary == 2) par("SlipMode", "1");
  par("RigidAlgorithm", "1");
  par("FtPause", "0");
  par("CoefDtMin", "0.05");
  par("DtIni", "0");
  par("DtMin", "0");
  par("TimeMax", fun::DoubleStr(tmax));
  par("TimeOut", "0.01");
  par("PartsOutMax", "1");
  par("RhopOutMin", "700");
  par("RhopOutMax", "1300");
  fprintf(f, "<simulationdomain><posmin x=\"default - 10%%\" y=\"default\" z=\"default\"/>"
             "<posmax x=\"default + 10%%\" y=\"default\" z=\"default + 50%%\"/></simulationdomain>\n");
  fprintf(f, "</parameters>\n</execution>\n</case>\n");
  fclose(f);
  printf("np=%u nfixed=%u npiston=%u nflap=%u nfloat=%u nf=%u h=%.10g b=%.10g cs0=%.10g mass=%.10g\n", np, nfixed,
         npiston, nflap, nfloat, nf, h, b, cs0, mass);
  return 0;
}
