// ORACLE / TEST INFRASTRUCTURE ONLY.  extern "C" entry to the reference's own
// ODE Dantzig solver (dart/external/odelcpsolver/lcp.h:60 dSolveLCP), compiled
// from /root/reference by oracle/Makefile into oracle/_ref/ (git-ignored).
#include "dart/external/odelcpsolver/lcp.h"
extern "C" int ref_dSolveLCP(int n, double* A, double* x, double* b, double* w, int nub, double* lo,
                             double* hi, int* findex, int earlyTermination) {
  return dSolveLCP(n, A, x, b, w, nub, lo, hi, findex, earlyTermination != 0) ? 1 : 0;
}
