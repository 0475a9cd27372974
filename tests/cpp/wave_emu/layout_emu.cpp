// Prints csrc/pool_sizes.h's snapshot offsets for n dofs (host build against
// the emulation header; checked against _native.snapshot_layout).
#include <cstdio>
#include <cstdlib>
#include "../../../nimblephysics_amd/csrc/pool_sizes.h"
int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 33;
  std::printf("%d %d %d %d %d %d %d %d %d %d %d\n", SN_CONTACTS, SN_ROWS, SN_FC, SN_VF, snYf(n), snAc(n), snAcubE(n),
              snPT(n), snQ(n), snEdge(n), snapWorkspaceOffset(n));
  return 0;
}
