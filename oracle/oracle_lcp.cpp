// ORACLE / TEST INFRASTRUCTURE ONLY -- placeholder, filled in below.
#include "oracle_lcp.hpp"
namespace oracle {
void pinvSolve(const double*, const double*, double*, int, double*) {}
}
