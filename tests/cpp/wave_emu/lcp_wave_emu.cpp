// Host driver for the wave LCP kernels under the wavefront emulation
// (hip/hip_runtime.h next to this file; test infrastructure only): reads LCP
// problems from stdin, runs the one-row-per-lane (R = 1, m <= 64) and the
// two-rows-per-lane (R = 2) instances of waveDantzigR, wavePgsR,
// waveLcpValidR, waveReduceR and the COD factor / min-norm solve, with every
// buffer a separate heap allocation (AddressSanitizer bounds), and prints
// the results for tests/test_wave_emu.py to check against the oracle.
//
// input:  count, then per problem: m, A (m*m row-major), b, lo, hi, findex, x0
// output: per problem and R: "R m okD xD... okP xP... validD reduceAlive codRank xCod... packedSame"
// (packedSame: the packed-factor Dantzig, kPL, gave the same flag and x bit
// for bit, its factor in a buffer of exactly dantzigLDoubles(m, true))
// With LCP_EMU_DANTZIG_ONLY=1 in the environment only waveDantzigR and its
// validity check run, R = 1 only for m <= 64: "R m okD xD... validD".
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "../../../nimblephysics_amd/csrc/lcp_wave.cuh"

struct Problem {
  int m;
  std::vector<double> A, b, lo, hi, x0;
  std::vector<int> fi;
};

static void runWave(const std::function<void(int)>& f) {
  std::barrier<> bar(64);
  wave_emu::waveBar[0] = &bar;
  std::vector<std::thread> ths;
  for (int l = 0; l < 64; l++)
    ths.emplace_back([&f, l] {
      wave_emu::tl_lane = l;
      wave_emu::tl_wave = 0;
      wave_emu::tl_seq = 0;
      f(l);
    });
  for (auto& t : ths) t.join();
}

template <int R>
static void solveDantzig(const Problem& P) {
  const int m = P.m;
  std::vector<double> L((size_t)m * (m | 1) + 8), scr((size_t)m + 8), xD((size_t)64 * R);
  int okD = 0, validD = 0;
  runWave([&](int lane) {
    double b[R], lo[R], hi[R], x[R];
    int fi[R];
    for (int s = 0; s < R; s++) {
      const int r = lane + 64 * s;
      b[s] = r < m ? P.b[r] : 0.0;
      lo[s] = r < m ? P.lo[r] : 0.0;
      hi[s] = r < m ? P.hi[r] : 0.0;
      fi[s] = r < m ? P.fi[r] : -1;
    }
    const bool d = waveDantzigR<false, R>(m, P.A.data(), L.data(), scr.data(), x, b, lo, hi, fi, lane);
    const bool v = d && waveLcpValidR<false, R>(m, P.A.data(), 0.0, x, b, hi, lo, fi, false, lane);
    for (int s = 0; s < R; s++) {
      const int r = lane + 64 * s;
      if (r < 64 * R) xD[r] = x[s];
    }
    if (lane == 0) { okD = d; validD = v; }
  });
  std::printf("%d %d %d", R, m, okD);
  for (int i = 0; i < m; i++) std::printf(" %.17g", xD[i]);
  std::printf(" %d\n", validD);
}

template <int R>
static void solve(const Problem& P) {
  const int m = P.m;
  std::vector<double> L((size_t)m * (m | 1) + 8), scr((size_t)m + 8), M1((size_t)m * m + 8);
  // (codFactor stages a 24-double column in v: the pool reserves it)
  std::vector<double> codWs((size_t)12 * m + 64), codV((size_t)(m > 24 ? m : 24) + 8), codScr((size_t)m + 8), Acopy(P.A);
  std::vector<double> xD((size_t)64 * R), xP((size_t)64 * R), xC((size_t)64 * R);
  std::vector<double> Lp((size_t)dantzigLDoubles(m, true)), scrP((size_t)m), xDp((size_t)64 * R);
  int okD = 0, okP = 0, validD = 0, alive = 0, rank = 0, okDp = 0;
  runWave([&](int lane) {
    double b[R], lo[R], hi[R], x[R], xp[R], xo[R];
    int fi[R];
    for (int s = 0; s < R; s++) {
      const int r = lane + 64 * s;
      b[s] = r < m ? P.b[r] : 0.0;
      lo[s] = r < m ? P.lo[r] : 0.0;
      hi[s] = r < m ? P.hi[r] : 0.0;
      fi[s] = r < m ? P.fi[r] : -1;
      xp[s] = r < m ? P.x0[r] : 0.0;
    }
    const bool d = waveDantzigR<false, R>(m, P.A.data(), L.data(), scr.data(), x, b, lo, hi, fi, lane);
    const bool v = d && waveLcpValidR<false, R>(m, P.A.data(), 0.0, x, b, hi, lo, fi, false, lane);
    // (the packed factor is the wide kernel's: R = 2 only, which the R = 1
    // results equal bit for bit anyway)
    double xpk[R];
    bool dp = d;
    for (int s = 0; s < R; s++) xpk[s] = x[s];
    if constexpr (R == 2)
      dp = waveDantzigR<false, R, false, false, true>(m, P.A.data(), Lp.data(), scrP.data(), xpk, b, lo, hi, fi, lane);
    const bool p = wavePgsR<false, false, R>(m, P.A.data(), xp, b, lo, hi, fi, lane, nullptr, 1e-4);
    double scl[R];
    int rep[R];
    unsigned long long al[R];
    waveReduceR<false, R>(m, P.A.data(), 0.0, b, lo, hi, fi, lane, scl, rep, al);
    // COD of A and the min-norm solve of A x = b
    for (size_t t = lane; t < (size_t)m * m; t += 64) M1[t] = P.A[t];
    WSYNC();
    codFactorR<false, R>(M1.data(), codWs.data(), m, m, m, codV.data(), lane);
    codSolveWaveR<false, R>(M1.data(), codWs.data(), m, m, m, b, codScr.data(), lane, xo);
    Cod c;
    carveCod(codWs.data(), M1.data(), m, m, m, c);
    for (int s = 0; s < R; s++) {
      const int r = lane + 64 * s;
      if (r < 64 * R) { xD[r] = x[s]; xP[r] = xp[s]; xC[r] = xo[s]; xDp[r] = xpk[s]; }
    }
    if (lane == 0) {
      okD = d; okP = p; validD = v; alive = popR(al); rank = *c.rank; okDp = dp;
    }
  });
  std::printf("%d %d %d", R, m, okD);
  for (int i = 0; i < m; i++) std::printf(" %.17g", xD[i]);
  std::printf(" %d", okP);
  for (int i = 0; i < m; i++) std::printf(" %.17g", xP[i]);
  std::printf(" %d %d %d", validD, alive, rank);
  for (int i = 0; i < m; i++) std::printf(" %.17g", xC[i]);
  bool same = okDp == okD;
  for (int i = 0; i < m; i++) same = same && std::memcmp(&xDp[i], &xD[i], sizeof(double)) == 0;
  std::printf(" %d\n", same ? 1 : 0);
}

int main() {
  int count = 0;
  if (std::scanf("%d", &count) != 1) return 2;
  for (int k = 0; k < count; k++) {
    Problem P;
    if (std::scanf("%d", &P.m) != 1) return 2;
    const int m = P.m;
    P.A.resize((size_t)m * m); P.b.resize(m); P.lo.resize(m); P.hi.resize(m); P.x0.resize(m); P.fi.resize(m);
    for (auto& v : P.A) std::scanf("%lf", &v);
    for (auto& v : P.b) std::scanf("%lf", &v);
    for (auto& v : P.lo) std::scanf("%lf", &v);
    for (auto& v : P.hi) std::scanf("%lf", &v);
    for (auto& v : P.fi) std::scanf("%d", &v);
    for (auto& v : P.x0) std::scanf("%lf", &v);
    const char* only = std::getenv("LCP_EMU_DANTZIG_ONLY");
    if (only && only[0] == '1') {
      if (m <= 64) solveDantzig<1>(P);
      else solveDantzig<2>(P);
      continue;
    }
    if (m <= 64) solve<1>(P);
    solve<2>(P);
  }
  return 0;
}
