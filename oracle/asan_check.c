/*
 * asan_check.c — host sanitizer run of the C oracle (TEST INFRASTRUCTURE
 * ONLY; SURVEY.md §5 "race / memory checking" for native code): the oracle
 * translation unit compiled with -fsanitize=address,undefined and driven
 * through its entry points (objective, Stan L-BFGS, analytic and
 * finite-difference Hessians, damped polish) for linear, logistic and flat
 * growth on a small synthetic problem.  Built and run by `make -C oracle
 * asan` (tests/test_oracle.py::test_oracle_sanitizers).
 */
#include "stan_lbfgs.c"

#include <stdio.h>

#define T_ 400
#define K_ 8
#define S_ 10

static int run(int growth) {
    static double t[T_], y[T_], cap[T_], X[T_ * K_], tc[S_], sig[K_], sa[K_], sm[K_];
    for (int i = 0; i < T_; ++i) {
        t[i] = (double)i / (T_ - 1);
        const double d = (double)i;
        for (int k = 0; k < K_ / 2; ++k) {
            X[i * K_ + 2 * k] = sin(2.0 * M_PI * (k + 1) * d / 7.0);
            X[i * K_ + 2 * k + 1] = cos(2.0 * M_PI * (k + 1) * d / 7.0);
        }
        cap[i] = 1.5;
        y[i] = 0.4 + 0.3 * t[i] + 0.05 * sin(2.0 * M_PI * d / 7.0) + 0.01 * sin(12.9898 * d);
    }
    for (int j = 0; j < S_; ++j) tc[j] = 0.8 * (j + 1) / (S_ + 1);
    for (int k = 0; k < K_; ++k) { sig[k] = 10.0; sa[k] = 0.0; sm[k] = 1.0; }
    orc_problem pb = {T_, K_, S_, growth, t, y, growth == 1 ? cap : NULL, X, tc, sig, sa, sm, 0.05};
    const int P = 3 + S_ + K_;
    double th[3 + S_ + K_], g[3 + S_ + K_], f;
    memset(th, 0, sizeof th);
    th[0] = growth == 1 ? 1.0 : 0.3;
    th[1] = growth == 1 ? 0.3 : 0.4;
    if (orc_objective(&pb, th, &f, g)) return 1;
    orc_opts o;
    orc_default_opts(&o);
    int it = 0, ne = 0;
    const int st = orc_lbfgs_fit(&pb, &o, th, &f, &it, &ne);
    double *H = malloc(sizeof(double) * P * P), *Hf = malloc(sizeof(double) * P * P), rr = 0.0;
    const int rh = orc_hessian(&pb, th, H, &rr);
    const int rf = orc_hessian_fd(&pb, th, 1e-5, Hf);
    int nn = 0, ne2 = 0, ns = 0, cert = 0;
    double f2 = f;
    const int rp = orc_polish_ex(&pb, th, 50, 1, &f2, &nn, &ne2, &ns, &cert);
    printf("growth %d: stan status %d (%d it, %d evals) f %.12g -> polish f %.12g cert %d "
           "(hessian rc %d/%d, polish rc %d)\n", growth, st, it, ne, f, f2, cert, rh, rf, rp);
    free(H);
    free(Hf);
    return !(isfinite(f2) && f2 <= f + 1e-9 * fabs(f));
}

int main(void) {
    int bad = 0;
    for (int growth = 0; growth < 3; ++growth) bad |= run(growth);
    return bad;
}
