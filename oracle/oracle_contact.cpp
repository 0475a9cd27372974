// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
// Collision detection + contact LCP (filled in incrementally).
#include <cstdio>
#include <cstdlib>

#include "oracle_lcp.hpp"

namespace oracle {

void collide(const World& w, const Kin<double>& k, std::vector<Contact>& out) {
  out.clear();
  (void)w; (void)k;
}

void solveContacts(const World& w, const Kin<double>& k, const double* q, const double* v, const double* tau,
                   std::vector<double>& v1, const std::vector<Contact>& contacts,
                   std::vector<double>& lcpCache, Snapshot& snap) {
  (void)w; (void)k; (void)q; (void)v; (void)tau; (void)v1; (void)lcpCache;
  snap.numRows = 0;
  snap.numClamping = 0;
  snap.numUpperBound = 0;
  if (!contacts.empty()) { std::fprintf(stderr, "oracle: contacts not implemented\n"); std::abort(); }
}

void buildClampingMatrices(const World& w, const Snapshot& snap, std::vector<double>& Ac,
                           std::vector<double>& Aub, std::vector<double>& AcubE) {
  (void)w; (void)snap; Ac.clear(); Aub.clear(); AcubE.clear();
}

void constrainedJacobians(const World&, const Kin<double>&, const Snapshot&, const std::vector<double>&,
                          const std::vector<double>&, const std::vector<double>&, const std::vector<double>&,
                          const std::vector<double>&, const std::vector<double>&, const std::vector<double>&,
                          const std::vector<double>&, const std::vector<double>&, std::vector<double>&,
                          std::vector<double>&, std::vector<double>&) {
  std::abort();
}

}  // namespace oracle
