// ftdump_ref — converts the reference's floating-body PART data (PartFloat.fbi4) into a
// flat little-endian fixture (test infrastructure; reads through the reference's own
// JPartFloatBi4Load, JPartFloatBi4.cpp).
//
// Output: u32 magic 'SPHF'  u32 ftcount  u32 nparts  u32 pad
//         per part: f64 timestep, per floating: f64 center[3], f32 fvel[3], f32 fomega[3]
//
// usage: ftdump_ref <dir> <outfile>
#include "JPartFloatBi4.h"
#include "Functions.h"
#include <cstdio>
#include <string>

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s dir outfile\n", argv[0]); return 1; }
  JPartFloatBi4Load ft;
  ft.LoadFile(argv[1]);
  const unsigned nft = ft.GetFtCount(), nparts = ft.GetCount();
  FILE* f = fopen(argv[2], "wb");
  if (!f) { perror("out"); return 2; }
  const unsigned hdr[4] = {0x46485053u, nft, nparts, 0u};
  fwrite(hdr, 4, 4, f);
  for (unsigned cp = 0; cp < nparts; cp++) {
    ft.LoadPartItem(cp);
    const double t = ft.GetPartTimeStep();
    fwrite(&t, 8, 1, f);
    for (unsigned cf = 0; cf < nft; cf++) {
      const tdouble3 c = ft.GetPartCenter(cf);
      const tfloat3 v = ft.GetPartVelLin(cf), w = ft.GetPartVelAng(cf);
      fwrite(&c, 8, 3, f);
      fwrite(&v, 4, 3, f);
      fwrite(&w, 4, 3, f);
    }
  }
  fclose(f);
  printf("ftcount=%u parts=%u\n", nft, nparts);
  return 0;
}
