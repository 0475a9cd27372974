// ORACLE / TEST INFRASTRUCTURE ONLY -- see nimble_oracle.cpp header.
#pragma once
#include <vector>

#include "oracle.hpp"

namespace oracle {

// dart/neural/ConstraintMapping (NeuralConstants.hpp): mapping >= 0 means
// UPPER_BOUND pointing at that row.
enum { CM_CLAMPING = -1, CM_NOT_CLAMPING = -2, CM_IRRELEVANT = -3, CM_ILLEGAL = -4 };

// ConstraintSolver::solve -> BoxedLcpConstraintSolver::solveConstrainedGroup ->
// applyConstraintImpulses -> Skeleton::computeImpulseForwardDynamics.
// Updates v1 in place and fills the snapshot's constraint fields.
void solveContacts(const World& w, const Kin<double>& k, const double* q, const double* v, const double* tau,
                   std::vector<double>& v1, const std::vector<Contact>& contacts,
                   std::vector<double>& lcpCache, Snapshot& snap);

void buildClampingMatrices(const World& w, const Snapshot& snap, std::vector<double>& Ac,
                           std::vector<double>& Aub, std::vector<double>& AcubE);

void constrainedJacobians(const World& w, const Kin<double>& k, const Snapshot& snap,
                          const std::vector<double>& M, const std::vector<double>& Minv,
                          const std::vector<double>& C, const std::vector<double>& dCq,
                          const std::vector<double>& dCv, const std::vector<double>& dM,
                          const std::vector<double>& Ac, const std::vector<double>& Aub,
                          const std::vector<double>& AcubE, std::vector<double>& posVel,
                          std::vector<double>& velVel, std::vector<double>& forceVel,
                          std::vector<double>* dFcOut = nullptr);

// dart/external/odelcpsolver/lcp.cpp:780 dSolveLCP (Dantzig), restated.
bool dantzigSolveLCP(int n, double* A, double* x, double* b, double* w, int nub, double* lo, double* hi,
                     int* findex, bool earlyTermination);

}  // namespace oracle
