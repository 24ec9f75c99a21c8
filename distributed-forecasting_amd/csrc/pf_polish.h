// pf_polish.h — exact-MAP proximal-Newton polish (stub; filled in next)
#pragma once
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ void polish_run(const FitKArgs &a, FitSmem<NW, KMAX> &sm, double &x, double &f,
                           double &g, int &n_eval) {
  (void)a; (void)sm; (void)x; (void)f; (void)g; (void)n_eval;
}
