// partdump_ref — converts reference PART files (Part_XXXX.bi4) into flat
// little-endian fixtures (test infrastructure; reads through the reference's own
// JPartDataBi4::LoadFilePart, JPartDataBi4.cpp:162-520).
//
// Output layout (one file per part):
//   u32 magic 'SPHG'  u32 np  f64 timestep  u32 nstep-field(0)  u32 pad
//   u32 idp[np]  f64 pos[np][3]  f32 vel[np][3]  f32 rhop[np]
// Particles are sorted by idp so fixtures compare by particle identity.
//
// usage: partdump_ref <dir> <part> <outfile>
#include "JPartDataBi4.h"
#include "Functions.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s dir part outfile\n", argv[0]); return 1; }
  const std::string dir = argv[1];
  const unsigned part = unsigned(atoi(argv[2]));
  JPartDataBi4 pd;
  pd.LoadFilePart(dir, part, 0, 1);
  const unsigned n = pd.Get_Npok();
  std::vector<unsigned> id(n);
  std::vector<tdouble3> pos(n);
  std::vector<tfloat3> vel(n);
  std::vector<float> rho(n);
  pd.Get_Idp(n, id.data());
  if (pd.Get_PosSimple()) {
    std::vector<tfloat3> pf(n);
    pd.Get_Pos(n, pf.data());
    for (unsigned i = 0; i < n; i++) pos[i] = ToTDouble3(pf[i]);
  } else {
    pd.Get_Posd(n, pos.data());
  }
  pd.Get_Vel(n, vel.data());
  pd.Get_Rhop(n, rho.data());
  const double t = pd.Get_TimeStep();

  std::vector<unsigned> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::sort(order.begin(), order.end(), [&](unsigned a, unsigned b) { return id[a] < id[b]; });

  FILE* f = fopen(argv[3], "wb");
  if (!f) { perror("out"); return 2; }
  const unsigned hdr[2] = {0x47485053u, n};
  const unsigned tail[2] = {0u, 0u};
  fwrite(hdr, 4, 2, f);
  fwrite(&t, 8, 1, f);
  fwrite(tail, 4, 2, f);
  for (unsigned i : order) fwrite(&id[i], 4, 1, f);
  for (unsigned i : order) fwrite(&pos[i], 8, 3, f);
  for (unsigned i : order) fwrite(&vel[i], 4, 3, f);
  for (unsigned i : order) fwrite(&rho[i], 4, 1, f);
  fclose(f);
  printf("part=%u np=%u t=%.17g\n", part, n, t);
  return 0;
}
