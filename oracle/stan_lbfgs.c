/*
 * stan_lbfgs.c — CPU oracle: Prophet's Stan log-posterior + Stan's L-BFGS.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/prophet_oracle.py header): used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
 * the product path.
 *
 * Restates UPSTREAM code that the reference calls but does not contain
 * (reference call site: notebooks/prophet/02_training.py:172 `model.fit`,
 * pinned by requirements.txt:3-4 pystan==2.19.1.1 / fbprophet==0.7.1):
 *   - prophet.stan  model block (linear / logistic / flat trend, priors,
 *     normal likelihood), evaluated with Stan's `log_prob_propto<false>`
 *     (data-only constants dropped, no Jacobian for sigma_obs' lower=0
 *     log transform) — the ModelAdaptor Stan's optimizer wraps.
 *   - Stan 2.19 optimization/bfgs.hpp (BFGSMinimizer::step),
 *     bfgs_linesearch.hpp (WolfeLineSearch, WolfLSZoom, CubicInterp),
 *     lbfgs_update.hpp (two-loop recursion, history 5) with PyStan's
 *     optimizing() defaults: init_alpha 1e-3, tol_obj 1e-12,
 *     tol_rel_obj 1e4, tol_grad 1e-8, tol_rel_grad 1e7, tol_param 1e-8,
 *     iter 1e4 (Prophet passes iter=1e4).
 * PARITY UNPINNED at the iteration level (no Stan here); the optimum is
 * certified against scipy L-BFGS-B in tests/test_oracle.py
 * (test_map_certified).
 *
 * Parameter vector (Stan unconstrained order):
 *   theta = [k, m, delta[S], log(sigma_obs), beta[K]],  P = 3 + S + K.
 * f(theta) = -log_posterior (minimised), g = grad f.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

typedef struct {
    int T, K, S, growth;           /* growth: 0 linear, 1 logistic, 2 flat */
    const double *t, *y, *cap;     /* [T] (cap may be NULL unless logistic) */
    const double *X;               /* [T*K] row-major */
    const double *t_change;        /* [S] sorted */
    const double *sigmas, *s_a, *s_m; /* [K] */
    double tau;
} orc_problem;

typedef struct {
    double init_alpha, tol_obj, tol_rel_obj, tol_grad, tol_rel_grad, tol_param;
    int max_iter, history;
    double c1, c2, min_alpha;
    int max_ls_its, max_ls_restarts;
} orc_opts;

void orc_default_opts(orc_opts *o) {
    o->init_alpha = 1e-3;
    o->tol_obj = 1e-12;
    o->tol_rel_obj = 1e4;
    o->tol_grad = 1e-8;
    o->tol_rel_grad = 1e7;
    o->tol_param = 1e-8;
    o->max_iter = 10000;
    o->history = 5;
    o->c1 = 1e-4;
    o->c2 = 0.9;
    o->min_alpha = 1e-12;
    o->max_ls_its = 20;
    o->max_ls_restarts = 10;
}

/* status codes (Stan TERM_*), shared with include/prophet_hip.h */
enum { ST_SUCCESS = 0, ST_ABSX = 10, ST_ABSF = 20, ST_RELF = 21,
       ST_ABSGRAD = 30, ST_RELGRAD = 31, ST_MAXIT = 40, ST_LSFAIL = -1,
       ST_CONSTANT = 50, ST_BADINIT = -2 };

static double sgn(double x) { return (x > 0) - (x < 0); }

/* -log posterior and its gradient. returns nonzero if not finite. */
int orc_objective(const orc_problem *pb, const double *theta, double *f_out, double *g) {
    const int T = pb->T, K = pb->K, S = pb->S;
    const double k = theta[0], m = theta[1];
    const double *delta = theta + 2;
    const double ls = theta[2 + S];
    const double *beta = theta + 3 + S;
    const double sigma = exp(ls);
    double *gamma = NULL, *k_s = NULL, *PK = NULL, *PM = NULL;
    if (pb->growth == 1) {
        gamma = (double *)calloc(S, sizeof(double));
        k_s = (double *)calloc(S + 1, sizeof(double));
        PK = (double *)calloc(S + 1, sizeof(double));
        PM = (double *)calloc(S + 1, sizeof(double));
        k_s[0] = k;
        for (int i = 0; i < S; ++i) k_s[i + 1] = k_s[i] + delta[i];
        double m_pr = m;
        for (int i = 0; i < S; ++i) {
            gamma[i] = (pb->t_change[i] - m_pr) * (1 - k_s[i] / k_s[i + 1]);
            m_pr += gamma[i];
        }
    }
    double L = -k * k / 50.0 - m * m / 50.0 - 2.0 * sigma * sigma - T * ls;
    for (int j = 0; j < S; ++j) L -= fabs(delta[j]) / pb->tau;
    for (int f = 0; f < K; ++f) L -= beta[f] * beta[f] / (2.0 * pb->sigmas[f] * pb->sigmas[f]);

    const int P = 3 + S + K;
    for (int p = 0; p < P; ++p) g[p] = 0.0;
    double *gd = g + 2, *gb = g + 3 + S;
    const double inv_s2 = 1.0 / (sigma * sigma);
    double rr = 0.0, gk = 0.0, gm = 0.0;
    for (int i = 0; i < T; ++i) {
        const double *x = pb->X + (size_t)i * K;
        double xbm = 0.0, xba = 0.0;
        for (int f = 0; f < K; ++f) {
            xbm += x[f] * beta[f] * pb->s_m[f];
            xba += x[f] * beta[f] * pb->s_a[f];
        }
        const double ti = pb->t[i];
        double tr, Kt = k, Mt = m, sg = 0.0;
        int seg = 0;
        if (pb->growth == 0) {
            double ad = 0.0, atd = 0.0;
            for (int j = 0; j < S; ++j)
                if (ti >= pb->t_change[j]) { ad += delta[j]; atd += -pb->t_change[j] * delta[j]; seg = j + 1; }
            tr = (k + ad) * ti + (m + atd);
        } else if (pb->growth == 1) {
            for (int j = 0; j < S; ++j)
                if (ti >= pb->t_change[j]) { Kt += delta[j]; Mt += gamma[j]; seg = j + 1; }
            double z = Kt * (ti - Mt);
            sg = 1.0 / (1.0 + exp(-z));
            tr = pb->cap[i] * sg;
        } else {
            tr = m;
        }
        const double mu = tr * (1.0 + xbm) + xba;
        const double r = pb->y[i] - mu;
        rr += r * r;
        const double w = r * inv_s2;
        const double G = w * (1.0 + xbm);
        for (int f = 0; f < K; ++f) gb[f] += x[f] * (w * tr * pb->s_m[f] + w * pb->s_a[f]);
        if (pb->growth == 0) {
            gk += G * ti;
            gm += G;
            for (int j = 0; j < S; ++j)
                if (ti >= pb->t_change[j]) gd[j] += G * (ti - pb->t_change[j]);
        } else if (pb->growth == 1) {
            double a = G * pb->cap[i] * sg * (1.0 - sg);
            PK[seg] += a * (ti - Mt);
            PM[seg] += -a * Kt;
        } else {
            gm += G;
        }
    }
    if (pb->growth == 1) {
        /* reverse-mode through logistic_gamma's recursion */
        double m_pr_arr_last = m;
        double *m_pr = (double *)calloc(S + 1, sizeof(double));
        m_pr[0] = m;
        for (int i = 0; i < S; ++i) m_pr[i + 1] = m_pr[i] + gamma[i];
        (void)m_pr_arr_last;
        for (int i = S - 1; i >= 0; --i) {
            double bar_g = PM[i + 1];
            PM[i] += PM[i + 1];
            double ki = k_s[i], ki1 = k_s[i + 1];
            PM[i] += bar_g * (-(1 - ki / ki1));
            PK[i] += bar_g * (-(pb->t_change[i] - m_pr[i]) / ki1);
            PK[i + 1] += bar_g * ((pb->t_change[i] - m_pr[i]) * ki / (ki1 * ki1));
        }
        double sk = 0.0;
        for (int s = S; s >= 1; --s) { sk += PK[s]; gd[s - 1] = sk; }
        gk = sk + PK[0];
        gm = PM[0];
        free(m_pr);
    }
    L -= rr * inv_s2 / 2.0;
    g[0] = gk - k / 25.0;
    g[1] = gm - m / 25.0;
    for (int j = 0; j < S; ++j) gd[j] -= sgn(delta[j]) / pb->tau;
    g[2 + S] = -T + rr * inv_s2 - 4.0 * sigma * sigma;
    for (int f = 0; f < K; ++f) gb[f] -= beta[f] / (pb->sigmas[f] * pb->sigmas[f]);
    /* minimise -L */
    *f_out = -L;
    int bad = !isfinite(L);
    for (int p = 0; p < P; ++p) { g[p] = -g[p]; if (!isfinite(g[p])) bad = 1; }
    if (gamma) { free(gamma); free(k_s); free(PK); free(PM); }
    return bad;
}

/* ---------------- Stan bfgs_linesearch.hpp restatement ---------------- */
static double cubic_interp0(double df0, double x1, double f1, double df1, double loX, double hiX) {
    const double c3 = (-12 * f1 + 6 * x1 * (df0 + df1)) / (x1 * x1 * x1);
    const double c2 = -(4 * df0 + 2 * df1) / x1 + 6 * f1 / (x1 * x1);
    const double c1 = df0;
    const double t_s = sqrt(c2 * c2 - 2.0 * c1 * c3);
    const double s1 = -(c2 + t_s) / c3;
    const double s2 = -(c2 - t_s) / c3;
    double tmpF, minF, minX;
    minF = loX * (loX * (loX * c3 / 3.0 + c2) / 2.0 + c1);
    minX = loX;
    tmpF = hiX * (hiX * (hiX * c3 / 3.0 + c2) / 2.0 + c1);
    if (tmpF < minF) { minF = tmpF; minX = hiX; }
    if (loX < s1 && s1 < hiX) {
        tmpF = s1 * (s1 * (s1 * c3 / 3.0 + c2) / 2.0 + c1);
        if (tmpF < minF) { minF = tmpF; minX = s1; }
    }
    if (loX < s2 && s2 < hiX) {
        tmpF = s2 * (s2 * (s2 * c3 / 3.0 + c2) / 2.0 + c1);
        if (tmpF < minF) { minF = tmpF; minX = s2; }
    }
    return minX;
}

static double cubic_interp(double x0, double f0, double df0, double x1, double f1, double df1,
                           double loX, double hiX) {
    return x0 + cubic_interp0(df0, x1 - x0, f1 - f0, df1, loX - x0, hiX - x0);
}

typedef struct {
    const orc_problem *pb;
    int n_eval;
} evaluator;

static int feval(evaluator *ev, const double *x, double *f, double *g) {
    ev->n_eval++;
    return orc_objective(ev->pb, x, f, g);
}

static double dot(const double *a, const double *b, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

static double norm2(const double *a, int n) { return sqrt(dot(a, a, n)); }

/* WolfLSZoom */
static int wolf_zoom(evaluator *ev, int n, double *alpha, double *newX, double *newF, double *newDF,
                     const double *x, double f, const double *p, double c1dfp, double c2dfp,
                     double alo, double aloF, double aloDFp, double ahi, double ahiF, double ahiDFp,
                     double min_range) {
    int itNum = 0;
    while (1) {
        itNum++;
        if (fabs(alo - ahi) < min_range) return 1;
        if (itNum % 5 == 0) {
            *alpha = 0.5 * (alo + ahi);
        } else {
            double lo = fmin(alo, ahi), hi = fmax(alo, ahi);
            *alpha = cubic_interp(alo, aloF, aloDFp, ahi, ahiF, ahiDFp, lo, hi);
            if (*alpha < lo + 0.01 * (hi - lo) || *alpha > hi - 0.01 * (hi - lo))
                *alpha = 0.5 * (alo + ahi);
        }
        for (int i = 0; i < n; ++i) newX[i] = x[i] + *alpha * p[i];
        while (feval(ev, newX, newF, newDF)) {
            *alpha = 0.5 * (*alpha + fmin(alo, ahi));
            if (fabs(fmin(alo, ahi) - *alpha) < min_range) return 1;
            for (int i = 0; i < n; ++i) newX[i] = x[i] + *alpha * p[i];
        }
        double newDFp = dot(newDF, p, n);
        if (*newF > (f + *alpha * c1dfp) || *newF >= aloF) {
            ahi = *alpha; ahiF = *newF; ahiDFp = newDFp;
        } else {
            if (fabs(newDFp) <= -c2dfp) break;
            if (newDFp * (ahi - alo) >= 0) { ahi = alo; ahiF = aloF; ahiDFp = aloDFp; }
            alo = *alpha; aloF = *newF; aloDFp = newDFp;
        }
    }
    return 0;
}

/* WolfeLineSearch: on success x1,f1,g1 hold the accepted point, alpha the step */
static int wolfe_ls(evaluator *ev, int n, double *alpha, double *x1, double *f1, double *g1,
                    const double *p, const double *x0, double f0, const double *g0,
                    const orc_opts *o, double *scratch_g) {
    const double dfp = dot(g0, p, n);
    const double c1dfp = o->c1 * dfp, c2dfp = o->c2 * dfp;
    double alpha0 = o->min_alpha, alpha1 = *alpha;
    double prevF = f0, prevDFp = dfp, newDFp;
    int nits = 0, lsRestarts = 0, ret = 0;
    (void)scratch_g;
    while (1) {
        if (nits >= o->max_ls_its) { ret = 1; break; }
        for (int i = 0; i < n; ++i) x1[i] = x0[i] + alpha1 * p[i];
        if (feval(ev, x1, f1, g1)) {
            if (lsRestarts >= o->max_ls_restarts) { ret = 1; break; }
            alpha1 = 0.5 * (alpha0 + alpha1);
            lsRestarts++;
            continue;
        }
        lsRestarts = 0;
        newDFp = dot(g1, p, n);
        if ((*f1 > f0 + alpha1 * c1dfp) || (*f1 >= prevF && nits > 0)) {
            ret = wolf_zoom(ev, n, alpha, x1, f1, g1, x0, f0, p, c1dfp, c2dfp,
                            alpha0, prevF, prevDFp, alpha1, *f1, newDFp, 1e-16);
            break;
        }
        if (fabs(newDFp) <= -c2dfp) { *alpha = alpha1; break; }
        if (newDFp >= 0) {
            ret = wolf_zoom(ev, n, alpha, x1, f1, g1, x0, f0, p, c1dfp, c2dfp,
                            alpha1, *f1, newDFp, alpha0, prevF, prevDFp, 1e-16);
            break;
        }
        alpha0 = alpha1;
        prevF = *f1;
        prevDFp = newDFp;
        alpha1 *= 10.0;
        nits++;
    }
    return ret;
}

/* ---------------- Stan bfgs.hpp + lbfgs_update.hpp restatement ---------------- */
#define MAXP 512
#define MAXH 32

int orc_lbfgs_fit(const orc_problem *pb, const orc_opts *o, double *theta,
                  double *f_out, int *n_iter_out, int *n_eval_out) {
    const int n = 3 + pb->S + pb->K;
    if (n > MAXP || o->history > MAXH) return ST_BADINIT;
    evaluator ev = {pb, 0};
    static __thread double xk[MAXP], gk[MAXP], pk[MAXP], xk1[MAXP], gk1[MAXP], pk1[MAXP];
    static __thread double sk[MAXP], yk[MAXP];
    static __thread double hs[MAXH][MAXP], hy[MAXH][MAXP], hrho[MAXH];
    int hcount = 0, hhead = 0; /* circular buffer: oldest at hhead */
    double gammak = 1.0;
    double fk, fk1 = 0.0, alpha = 0.0, alphak_1 = 0.0;
    memcpy(xk, theta, n * sizeof(double));
    if (feval(&ev, xk, &fk, gk)) { *n_eval_out = ev.n_eval; *n_iter_out = 0; *f_out = fk; return ST_BADINIT; }
    for (int i = 0; i < n; ++i) pk[i] = -gk[i];
    int itNum = 0, retCode = 0;
    while (retCode == 0) {
        itNum++;
        int resetB = (itNum == 1) ? 1 : 0;
        while (1) {
            if (resetB) {
                for (int i = 0; i < n; ++i) pk[i] = -gk[i];
            }
            if (itNum > 1 && resetB != 2) {
                alpha = fmin(1.0, 1.01 * cubic_interp0(dot(gk1, pk1, n), alphak_1, fk - fk1,
                                                       dot(gk, pk1, n), o->min_alpha, 1.0));
            } else {
                alpha = o->init_alpha;
            }
            int ls = wolfe_ls(&ev, n, &alpha, xk1, &fk1, gk1, pk, xk, fk, gk, o, NULL);
            if (ls) {
                if (resetB) { retCode = ST_LSFAIL; break; }
                resetB = 2;
                continue;
            }
            break;
        }
        if (retCode == ST_LSFAIL) break;
        /* swap so that k is the most recent iterate */
        { double tf = fk; fk = fk1; fk1 = tf; }
        for (int i = 0; i < n; ++i) {
            double t;
            t = xk[i]; xk[i] = xk1[i]; xk1[i] = t;
            t = gk[i]; gk[i] = gk1[i]; gk1[i] = t;
            t = pk[i]; pk[i] = pk1[i]; pk1[i] = t;
            sk[i] = xk[i] - xk1[i];
            yk[i] = gk[i] - gk1[i];
        }
        alphak_1 = alpha;
        if (fabs(fk1 - fk) < o->tol_obj) {
            retCode = ST_ABSF;
        } else if (norm2(gk, n) < o->tol_grad) {
            retCode = ST_ABSGRAD;
        } else if (norm2(sk, n) < o->tol_param) {
            retCode = ST_ABSX;
        } else if (itNum >= o->max_iter) {
            retCode = ST_MAXIT;
        } else if (((fk1 - fk) / fmax(fabs(fk1), fmax(fabs(fk), 1.0))) < o->tol_rel_obj * DBL_EPSILON) {
            retCode = ST_RELF;
        } else {
            /* LBFGSUpdate::update */
            double skyk = dot(yk, sk, n);
            if (resetB) { hcount = 0; hhead = 0; }
            double yy = dot(yk, yk, n);
            gammak = skyk / yy;
            int slot;
            if (hcount < o->history) { slot = (hhead + hcount) % o->history; hcount++; }
            else { slot = hhead; hhead = (hhead + 1) % o->history; }
            memcpy(hs[slot], sk, n * sizeof(double));
            memcpy(hy[slot], yk, n * sizeof(double));
            hrho[slot] = 1.0 / skyk;
            /* LBFGSUpdate::search_direction (two-loop) */
            double al[MAXH];
            for (int i = 0; i < n; ++i) pk[i] = -gk[i];
            for (int c = hcount - 1; c >= 0; --c) {
                int s = (hhead + c) % o->history;
                al[c] = hrho[s] * dot(hs[s], pk, n);
                for (int i = 0; i < n; ++i) pk[i] -= al[c] * hy[s][i];
            }
            for (int i = 0; i < n; ++i) pk[i] *= gammak;
            for (int c = 0; c < hcount; ++c) {
                int s = (hhead + c) % o->history;
                double b = hrho[s] * dot(hy[s], pk, n);
                for (int i = 0; i < n; ++i) pk[i] += (al[c] - b) * hs[s][i];
            }
            if (-dot(pk, gk, n) / fmax(fabs(fk), 1.0) < o->tol_rel_grad * DBL_EPSILON)
                retCode = ST_RELGRAD;
            else
                retCode = ST_SUCCESS;
        }
    }
    memcpy(theta, xk, n * sizeof(double));
    *f_out = fk;
    *n_iter_out = itNum;
    *n_eval_out = ev.n_eval;
    return retCode;
}

/* Batch helper used by the CPU baseline: fit S series sharing t/X/t_change.
 * Y is [S*T] series-major (already y_scaled), theta [S*P] in/out. */
int orc_lbfgs_fit_batch(int S_series, const orc_problem *proto, const double *Y,
                        const orc_opts *o, double *theta, double *f_out,
                        int *status, int *n_iter, int *n_eval) {
    const int P = 3 + proto->S + proto->K;
    for (int s = 0; s < S_series; ++s) {
        orc_problem pb = *proto;
        pb.y = Y + (size_t)s * proto->T;
        status[s] = orc_lbfgs_fit(&pb, o, theta + (size_t)s * P, f_out + s, n_iter + s, n_eval + s);
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * OWL-QN (orthant-wise L-BFGS, Andrew & Gao 2007) on the same objective.
 * NOT part of Stan: this is the engine's optional "polish" that finishes the
 * L1 (double_exponential on delta) problem exactly where Stan's smooth
 * L-BFGS stalls at the kink.  f = h + c*sum|delta|, c = 1/tau.
 * ------------------------------------------------------------------------- */
static void owl_pseudo_grad(int n, int S, double c, const double *x, const double *gh, double *pg) {
    for (int i = 0; i < n; ++i) pg[i] = gh[i];
    for (int j = 0; j < S; ++j) {
        int i = 2 + j;
        if (x[i] > 0) pg[i] = gh[i] + c;
        else if (x[i] < 0) pg[i] = gh[i] - c;
        else if (gh[i] + c < 0) pg[i] = gh[i] + c;
        else if (gh[i] - c > 0) pg[i] = gh[i] - c;
        else pg[i] = 0.0;
    }
}

/* smooth-part gradient from the full gradient: gh = g - c*sign(delta) */
static void owl_smooth_grad(int n, int S, double c, const double *x, const double *g, double *gh) {
    for (int i = 0; i < n; ++i) gh[i] = g[i];
    for (int j = 0; j < S; ++j) gh[2 + j] = g[2 + j] - c * sgn(x[2 + j]);
}

int orc_owlqn_fit2(const orc_problem *pb, int max_iter, double tol_rel_f, double tol_pg, int H, double *theta,
                  double *f_out, int *n_iter_out, int *n_eval_out);
int orc_owlqn_fit(const orc_problem *pb, int max_iter, double tol_rel_f, double *theta,
                  double *f_out, int *n_iter_out, int *n_eval_out) {
    return orc_owlqn_fit2(pb, max_iter, tol_rel_f, 0.0, 5, theta, f_out, n_iter_out, n_eval_out);
}

int orc_owlqn_fit2(const orc_problem *pb, int max_iter, double tol_rel_f, double tol_pg, int H, double *theta,
                  double *f_out, int *n_iter_out, int *n_eval_out) {
    const int n = 3 + pb->S + pb->K, S = pb->S;
    const double c = 1.0 / pb->tau;
    evaluator ev = {pb, 0};
    double x[MAXP], g[MAXP], gh[MAXP], pg[MAXP], d[MAXP], xn[MAXP], gn[MAXP], ghn[MAXP], xi[MAXP];
    double hs[MAXH][MAXP], hy[MAXH][MAXP], hrho[MAXH], al[MAXH];
    int hcount = 0, hhead = 0;
    double f, fn = 0.0;
    memcpy(x, theta, n * sizeof(double));
    if (feval(&ev, x, &f, g)) return ST_BADINIT;
    owl_smooth_grad(n, S, c, x, g, gh);
    int it, ret = ST_MAXIT;
    for (it = 1; it <= max_iter; ++it) {
        owl_pseudo_grad(n, S, c, x, gh, pg);
        double pgn = norm2(pg, n);
        if (pgn < 1e-10 || pgn < tol_pg) { ret = ST_ABSGRAD; break; }
        /* two-loop on pseudo-gradient */
        for (int i = 0; i < n; ++i) d[i] = -pg[i];
        for (int q = hcount - 1; q >= 0; --q) {
            int s = (hhead + q) % H;
            al[q] = hrho[s] * dot(hs[s], d, n);
            for (int i = 0; i < n; ++i) d[i] -= al[q] * hy[s][i];
        }
        if (hcount > 0) {
            int s = (hhead + hcount - 1) % H;
            double gam = dot(hs[s], hy[s], n) / dot(hy[s], hy[s], n);
            for (int i = 0; i < n; ++i) d[i] *= gam;
        }
        for (int q = 0; q < hcount; ++q) {
            int s = (hhead + q) % H;
            double b = hrho[s] * dot(hy[s], d, n);
            for (int i = 0; i < n; ++i) d[i] += (al[q] - b) * hs[s][i];
        }
        /* constrain direction to the descent orthant of -pg */
        for (int i = 0; i < n; ++i) if (d[i] * pg[i] >= 0) d[i] = 0.0;
        for (int i = 0; i < n; ++i) xi[i] = (x[i] != 0) ? sgn(x[i]) : sgn(-pg[i]);
        double alpha = (hcount == 0) ? fmin(1.0, 1.0 / pgn) : 1.0;
        int ok = 0;
        for (int ls = 0; ls < 60; ++ls) {
            for (int i = 0; i < n; ++i) xn[i] = x[i] + alpha * d[i];
            for (int j = 0; j < S; ++j) { int i = 2 + j; if (xn[i] * xi[i] <= 0) xn[i] = 0.0; }
            if (!feval(&ev, xn, &fn, gn)) {
                double dec = 0.0;
                for (int i = 0; i < n; ++i) dec += pg[i] * (xn[i] - x[i]);
                if (fn <= f + 1e-4 * dec) { ok = 1; break; }
            }
            alpha *= 0.5;
        }
        if (!ok) { ret = ST_LSFAIL; break; }
        owl_smooth_grad(n, S, c, xn, gn, ghn);
        double sy = 0.0, yy = 0.0;
        int slot;
        if (hcount < H) { slot = (hhead + hcount) % H; } else { slot = hhead; }
        for (int i = 0; i < n; ++i) {
            hs[slot][i] = xn[i] - x[i];
            hy[slot][i] = ghn[i] - gh[i];
            sy += hs[slot][i] * hy[slot][i];
            yy += hy[slot][i] * hy[slot][i];
        }
        if (sy > 1e-16 * yy && yy > 0) {
            hrho[slot] = 1.0 / sy;
            if (hcount < H) hcount++; else hhead = (hhead + 1) % H;
        }
        double rel = (f - fn) / fmax(fabs(f), 1.0);
        memcpy(x, xn, n * sizeof(double));
        memcpy(gh, ghn, n * sizeof(double));
        f = fn;
        if (rel < tol_rel_f) { ret = ST_RELF; break; }
    }
    memcpy(theta, x, n * sizeof(double));
    *f_out = f;
    *n_iter_out = it;
    *n_eval_out = ev.n_eval;
    return ret;
}

/* ---------------------------------------------------------------------------
 * Exact-MAP polish (engine extension, NOT Stan): proximal Newton on
 * f = h + c*||delta||_1 (c = 1/tau) from the point where Stan's L-BFGS stopped.
 * Each iteration: exact Hessian of the smooth part h, the lasso-QP subproblem
 *   min_z gh.(z-x) + 1/2 (z-x)' H (z-x) + c ||z_delta||_1
 * solved exactly by an active-set method (Cholesky solves on the free set),
 * then Armijo backtracking on the true objective.  Linear, flat and logistic growth.
 * The HIP kernel (pf_polish.h) implements the same algorithm.
 * ------------------------------------------------------------------------- */
#define PMAX 128

/* Hessian of h (smooth part of -log posterior) at theta: linear, flat and
 * logistic growth.  With r = y - mu and sigma^2 = exp(2 l):
 *   H = (1/sigma^2) sum_i [dmu_i dmu_i' - r_i d2mu_i] + prior Hessian,
 * plus the l row/column.  Trend parameters (k, m, delta) enter mu through
 *   linear:   tr = k_s t + m_s              dmu/dth_t = u D_t
 *   logistic: tr = cap sigmoid(z), z = k_s (t - m_s) with m_s from
 *             UPSTREAM logistic_gamma;      dmu/dth_t = u cap s' dz
 * where dz = (t - m_s) E_s - k_s M_s, E_s = dk_s/dth_t, M_s = dm_s/dth_t
 * (recursion through logistic_gamma), and the second derivative adds
 *   - r u cap [s'' dz dz' + s' d2z],  d2z = -(E_s M_s' + M_s E_s') - k_s D2M_s.
 * The per-row terms are the rank-one updates below; the d2z terms collapse
 * to per-segment sums rho_s = sum_{i in s} r_i u_i cap_i s'_i.  Same
 * formulas as the HIP kernel's Hessian (pf_polish.h), checked against
 * central differences of orc_objective's gradient in tests/test_oracle.py. */
#define HMAXS 64
int orc_hessian(const orc_problem *pb, const double *theta, double *H /*P*P*/, double *rr_out) {
    const int T = pb->T, K = pb->K, S = pb->S, P = 3 + S + K, nt = 2 + S, il = 2 + S;
    const int g = pb->growth;
    if (P > PMAX || S + 1 > HMAXS) return -1;
    const double k = theta[0], m = theta[1];
    const double *delta = theta + 2, *beta = theta + 3 + S;
    const double sig2 = exp(2.0 * theta[il]);
    static __thread double ks[HMAXS], ms[HMAXS], Mt[HMAXS][HMAXS], rho[HMAXS];
    double dz[PMAX], Jb[PMAX], Wb[PMAX], Jr[PMAX];
    for (int a = 0; a < P * P; ++a) H[a] = 0.0;
    for (int p = 0; p < P; ++p) Jr[p] = 0.0;
    /* segment rates / offsets and (logistic) dm_s/dth_t */
    ks[0] = k;
    for (int j = 0; j < S; ++j) ks[j + 1] = ks[j] + delta[j];
    ms[0] = m;
    for (int s = 0; s <= S; ++s) { rho[s] = 0.0; for (int c = 0; c < nt; ++c) Mt[s][c] = 0.0; }
    Mt[0][1] = 1.0;
    if (g == 1) {
        for (int s = 0; s < S; ++s) {
            const double q = ks[s] / ks[s + 1], b = ks[s + 1];
            ms[s + 1] = ms[s] + (pb->t_change[s] - ms[s]) * (1 - q);
            for (int c = 0; c < nt; ++c) {
                const double Es = (c == 0 || (c >= 2 && c - 2 < s)) ? 1.0 : 0.0;
                const double Es1 = (c == 0 || (c >= 2 && c - 2 < s + 1)) ? 1.0 : 0.0;
                const double dq = Es / b - ks[s] * Es1 / (b * b);
                Mt[s + 1][c] = q * Mt[s][c] + (ms[s] - pb->t_change[s]) * dq;
            }
        }
    }
    double rr = 0.0;
    for (int i = 0; i < T; ++i) {
        const double *x = pb->X + (size_t)i * K;
        const double ti = pb->t[i];
        double xbm = 0.0, xba = 0.0;
        for (int f = 0; f < K; ++f) { xbm += x[f] * beta[f] * pb->s_m[f]; xba += x[f] * beta[f] * pb->s_a[f]; }
        int s = 0;
        for (int j = 0; j < S; ++j) if (ti >= pb->t_change[j]) s = j + 1;
        const double u = 1.0 + xbm;
        double tr, wt, gf = 1.0, sp = 0.0, sg = 0.0, capi = 0.0;
        for (int c = 0; c < nt; ++c) dz[c] = 0.0;
        if (g == 0) {
            double ad = 0.0, atd = 0.0;
            for (int j = 0; j < S; ++j)
                if (ti >= pb->t_change[j]) { ad += delta[j]; atd -= pb->t_change[j] * delta[j]; dz[2 + j] = ti - pb->t_change[j]; }
            tr = (k + ad) * ti + (m + atd);
            dz[0] = ti;
            dz[1] = 1.0;
        } else if (g == 1) {
            capi = pb->cap[i];
            const double z = ks[s] * (ti - ms[s]);
            sg = 1.0 / (1.0 + exp(-z));
            sp = sg * (1.0 - sg);
            tr = capi * sg;
            for (int c = 0; c < nt; ++c) {
                const double Es = (c == 0 || (c >= 2 && c - 2 < s)) ? 1.0 : 0.0;
                dz[c] = (ti - ms[s]) * Es - ks[s] * Mt[s][c];
            }
            gf = capi * sp;
        } else {
            tr = m;
            dz[1] = 1.0;
        }
        const double r = pb->y[i] - (tr * u + xba);
        rr += r * r;
        if (g == 1) {
            const double spp = sp * (1.0 - 2.0 * sg);
            const double a = u * capi * sp;
            wt = a * a - r * u * capi * spp;
            rho[s] += r * u * capi * sp;
        } else {
            wt = u * u;
        }
        for (int f = 0; f < K; ++f) {
            const double kf = tr * pb->s_m[f] + pb->s_a[f];
            Jb[f] = x[f] * kf;
            Wb[f] = x[f] * (u * kf - r * pb->s_m[f]);
        }
        for (int c = 0; c < nt; ++c) Jr[c] += r * u * gf * dz[c];
        for (int f = 0; f < K; ++f) Jr[nt + 1 + f] += r * Jb[f];
        for (int a = 0; a < nt; ++a) {
            for (int b = 0; b <= a; ++b) H[a * P + b] += wt * dz[a] * dz[b];
            for (int f = 0; f < K; ++f) H[(nt + 1 + f) * P + a] += gf * dz[a] * Wb[f];
        }
        for (int f = 0; f < K; ++f)
            for (int f2 = 0; f2 <= f; ++f2) H[(nt + 1 + f) * P + nt + 1 + f2] += Jb[f] * Jb[f2];
    }
    if (g == 1) {
        /* sum_s rho_s [E_s M_s' + M_s E_s' + k_s D2M_s], D2M by recursion */
        static __thread double D2[HMAXS][HMAXS];
        for (int a = 0; a < nt; ++a) for (int b = 0; b < nt; ++b) D2[a][b] = 0.0;
        for (int s = 0; s <= S; ++s) {
            if (s > 0) {
                const int sp_ = s - 1;
                const double q = ks[sp_] / ks[s], b = ks[s];
                for (int a = 0; a < nt; ++a)
                    for (int c = 0; c < nt; ++c) {
                        const double Ea = (a == 0 || (a >= 2 && a - 2 < sp_)) ? 1.0 : 0.0;
                        const double Ea1 = (a == 0 || (a >= 2 && a - 2 < s)) ? 1.0 : 0.0;
                        const double Ec = (c == 0 || (c >= 2 && c - 2 < sp_)) ? 1.0 : 0.0;
                        const double Ec1 = (c == 0 || (c >= 2 && c - 2 < s)) ? 1.0 : 0.0;
                        const double dqa = Ea / b - ks[sp_] * Ea1 / (b * b);
                        const double dqc = Ec / b - ks[sp_] * Ec1 / (b * b);
                        const double d2q = -(Ea * Ec1 + Ea1 * Ec) / (b * b) + 2.0 * ks[sp_] * Ea1 * Ec1 / (b * b * b);
                        D2[a][c] = q * D2[a][c] + dqa * Mt[sp_][c] + Mt[sp_][a] * dqc +
                                   (ms[sp_] - pb->t_change[sp_]) * d2q;
                    }
            }
            for (int a = 0; a < nt; ++a) {
                const double Ea = (a == 0 || (a >= 2 && a - 2 < s)) ? 1.0 : 0.0;
                for (int b = 0; b <= a; ++b) {
                    const double Eb = (b == 0 || (b >= 2 && b - 2 < s)) ? 1.0 : 0.0;
                    H[a * P + b] += rho[s] * (Ea * Mt[s][b] + Mt[s][a] * Eb + ks[s] * D2[a][b]);
                }
            }
        }
    }
    /* symmetrize, scale by 1/sigma^2 (l row excluded: set below) */
    for (int a = 0; a < P; ++a)
        for (int b = 0; b < a; ++b) { H[a * P + b] /= sig2; H[b * P + a] = H[a * P + b]; }
    for (int a = 0; a < P; ++a) H[a * P + a] /= sig2;
    /* priors */
    H[0] += 1.0 / 25.0;
    H[1 * P + 1] += 1.0 / 25.0;
    for (int f = 0; f < K; ++f) H[(3 + S + f) * P + 3 + S + f] += 1.0 / (pb->sigmas[f] * pb->sigmas[f]);
    /* l row/col: d2h/dl2 = 8 sigma^2 + 2 Q / sigma^2 ; d2h/dl dp = (2/sigma^2) sum r dmu/dp */
    H[il * P + il] = 8.0 * sig2 + 2.0 * rr / sig2;
    for (int p = 0; p < P; ++p) {
        if (p == il) continue;
        const double v = 2.0 * Jr[p] / sig2;
        H[il * P + p] = v;
        H[p * P + il] = v;
    }
    if (rr_out) *rr_out = rr;
    return 0;
}

/* Central-difference Hessian of the smooth gradient (check for orc_hessian;
 * relative step h per coordinate, L1 term's gradient removed by its sign at
 * the perturbed point). */
int orc_hessian_fd(const orc_problem *pb, const double *theta, double h, double *H) {
    const int S = pb->S, P = 3 + S + pb->K;
    if (P > PMAX) return -1;
    double xp[PMAX], gp[PMAX], gm[PMAX], f;
    for (int q = 0; q < P; ++q) {
        const double e = h * fmax(1.0, fabs(theta[q]));
        memcpy(xp, theta, P * sizeof(double));
        xp[q] = theta[q] + e;
        if (orc_objective(pb, xp, &f, gp)) return -2;
        for (int j = 0; j < S; ++j) gp[2 + j] -= sgn(xp[2 + j]) / pb->tau;
        xp[q] = theta[q] - e;
        if (orc_objective(pb, xp, &f, gm)) return -2;
        for (int j = 0; j < S; ++j) gm[2 + j] -= sgn(xp[2 + j]) / pb->tau;
        for (int p = 0; p < P; ++p) H[p * P + q] = (gp[p] - gm[p]) / (2.0 * e);
    }
    return 0;
}

/* Cholesky solve of M x = b (M n*n SPD, row-major, overwritten). 0 on success. */
static int chol_solve(double *M, int n, double *b) {
    for (int kk = 0; kk < n; ++kk) {
        double d = M[kk * n + kk];
        for (int j = 0; j < kk; ++j) d -= M[kk * n + j] * M[kk * n + j];
        if (!(d > 0)) return -1;
        d = sqrt(d);
        M[kk * n + kk] = d;
        for (int i = kk + 1; i < n; ++i) {
            double v = M[i * n + kk];
            for (int j = 0; j < kk; ++j) v -= M[i * n + j] * M[kk * n + j];
            M[i * n + kk] = v / d;
        }
    }
    for (int i = 0; i < n; ++i) {
        double v = b[i];
        for (int j = 0; j < i; ++j) v -= M[i * n + j] * b[j];
        b[i] = v / M[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int j = i + 1; j < n; ++j) v -= M[j * n + i] * b[j];
        b[i] = v / M[i * n + i];
    }
    return 0;
}

/* Active-set solution of the lasso-QP subproblem.  Returns #solves, z out. */
int orc_qp_active(const double *H, const double *gh, const double *x, int P, int d0, int S,
                  double c, double *z, int max_as) {
    static __thread double M[PMAX * PMAX], rhs[PMAX], zn[PMAX], gq[PMAX];
    int zero[PMAX], idx[PMAX];
    double s[PMAX];
    for (int p = 0; p < P; ++p) { zero[p] = 0; s[p] = 0.0; z[p] = x[p]; }
    for (int j = 0; j < S; ++j) {
        const int p = d0 + j;
        if (fabs(gh[p]) <= c) zero[p] = 1;
        else if (x[p] != 0 && sgn(x[p]) == -sgn(gh[p])) s[p] = sgn(x[p]);
        else s[p] = -sgn(gh[p]);
    }
    int nsolve = 0;
    for (int it = 0; it < max_as; ++it) {
        int n = 0;
        for (int p = 0; p < P; ++p) if (!zero[p]) idx[n++] = p;
        for (int a = 0; a < n; ++a) {
            const int pa = idx[a];
            double v = -(gh[pa] + c * s[pa]);
            for (int p = 0; p < P; ++p) if (zero[p]) v += H[pa * P + p] * x[p];
            rhs[a] = v;
            for (int b = 0; b < n; ++b) M[a * n + b] = H[pa * P + idx[b]];
        }
        if (chol_solve(M, n, rhs)) return -1;
        nsolve++;
        for (int p = 0; p < P; ++p) zn[p] = 0.0;
        for (int a = 0; a < n; ++a) zn[idx[a]] = x[idx[a]] + rhs[a];
        /* first sign crossing along z -> zn among free delta coords */
        int jmin = -1;
        double tmin = 2.0;
        for (int j = 0; j < S; ++j) {
            const int p = d0 + j;
            if (!zero[p] && zn[p] * s[p] < 0) {
                const double tt = (z[p] != zn[p]) ? z[p] / (z[p] - zn[p]) : 0.0;
                if (tt < tmin) { tmin = tt; jmin = p; }
            }
        }
        if (jmin >= 0) {
            for (int p = 0; p < P; ++p) z[p] = z[p] + tmin * (zn[p] - z[p]);
            z[jmin] = 0.0;
            zero[jmin] = 1;
            s[jmin] = 0.0;
            continue;
        }
        for (int p = 0; p < P; ++p) z[p] = zn[p];
        /* KKT for zero coords */
        int add = -1;
        double best = 0.0;
        for (int j = 0; j < S; ++j) {
            const int p = d0 + j;
            if (!zero[p]) continue;
            double v = gh[p];
            for (int q = 0; q < P; ++q) v += H[p * P + q] * (z[q] - x[q]);
            gq[p] = v;
            if (fabs(v) > c * (1 + 1e-12) && fabs(v) > best) { best = fabs(v); add = p; }
        }
        if (add < 0) break;
        zero[add] = 0;
        s[add] = -sgn(gq[add]);
    }
    return nsolve;
}

/* Proximal Newton with Levenberg-Marquardt damping: when the QP under the
 * exact Hessian hits a non-positive pivot (the objective is not convex away
 * from the optimum: multiplicative seasonality, logistic trend), the model is
 * H + lam * dmax * I with lam raised x10 until the active-set QP solves; lam
 * is relaxed /10 after every accepted step.  Any positive-definite model
 * predicts zero decrease exactly at a KKT point, so the certificate
 * (dec >= -1e-15 |f| after a QP solved to KKT) is unchanged.  cert_out = 1
 * when the loop ended on that certificate. */
int orc_polish_cfg2(const orc_problem *pb, double *theta, int max_it, int damp, double lam0,
                    double lam_decay, double alpha_first,
                    double *f_out, int *n_newton, int *n_eval, int *n_solve, int *cert_out) {
    const int S = pb->S, P = 3 + S + pb->K;
    const double c = 1.0 / pb->tau;
    if (P > PMAX) return -1;
    static __thread double H[PMAX * PMAX], Hd[PMAX * PMAX];
    double g[PMAX], gh[PMAX], z[PMAX], d[PMAX], xn[PMAX], gn[PMAX], f, fn = 0.0;
    evaluator ev = {pb, 0};
    if (feval(&ev, theta, &f, g)) return -2;
    int it, ns = 0, cert = 0, nn = 0;
    double lam = lam0;
    for (it = 0; it < max_it; ++it) {
        for (int p = 0; p < P; ++p) gh[p] = g[p];
        for (int j = 0; j < S; ++j) gh[2 + j] -= c * sgn(theta[2 + j]);
        if (orc_hessian(pb, theta, H, NULL)) break;
        double dmax = 0.0;
        for (int p = 0; p < P; ++p) dmax = fmax(dmax, fabs(H[p * P + p]));
        int r = -1;
        for (int tr = 0; tr < 16; ++tr) {
            memcpy(Hd, H, (size_t)P * P * sizeof(double));
            for (int p = 0; p < P; ++p) Hd[p * P + p] += lam * dmax;
            r = orc_qp_active(Hd, gh, theta, P, 2, S, c, z, 200);
            if (r >= 0 || !damp) break;
            lam = (lam == 0.0) ? 1e-10 : lam * 10.0;
        }
        if (r < 0) break;
        ns += r;
        double l1z = 0.0, l1x = 0.0, dec = 0.0;
        for (int p = 0; p < P; ++p) { d[p] = z[p] - theta[p]; dec += gh[p] * d[p]; }
        for (int j = 0; j < S; ++j) { l1z += fabs(z[2 + j]); l1x += fabs(theta[2 + j]); }
        dec += c * (l1z - l1x);
        if (dec > -1e-15 * fabs(f)) { cert = 1; break; }
        double alpha = (nn == 0) ? alpha_first : 1.0;
        int ok = 0;
        for (int ls = 0; ls < 30; ++ls) {
            for (int p = 0; p < P; ++p) xn[p] = theta[p] + alpha * d[p];
            if (!feval(&ev, xn, &fn, gn) && fn <= f + 1e-4 * alpha * dec) { ok = 1; break; }
            alpha *= 0.5;
        }
        if (!ok) break;
        ++nn;
        memcpy(theta, xn, P * sizeof(double));
        memcpy(g, gn, P * sizeof(double));
        f = fn;
        /* the first step's damping (lam0) ends with it; damping raised by a
         * non-positive pivot relaxes x lam_decay per accepted step */
        if (nn == 1 && lam <= lam0) lam = 0.0;
        else lam = (lam < 1e-9) ? 0.0 : lam * lam_decay;
    }
    *f_out = f;
    *n_newton = nn;
    *n_eval = ev.n_eval;
    *n_solve = ns;
    if (cert_out) *cert_out = cert;
    return 0;
}

int orc_polish_cfg(const orc_problem *pb, double *theta, int max_it, int damp, double lam0,
                   double *f_out, int *n_newton, int *n_eval, int *n_solve, int *cert_out) {
    return orc_polish_cfg2(pb, theta, max_it, damp, lam0, 0.1, 1.0, f_out, n_newton, n_eval, n_solve,
                           cert_out);
}

/* The engine's default: the first QP's model is damped by ORC_POLISH_LAM0 *
 * max|diag H| (pf_fit_opts.polish_lam0).  An undamped first Newton step from
 * a warm-up iterate can jump into a neighbouring, worse local optimum of the
 * non-convex MAP objective (tools/diag_basin_commit.py: the polish from Stan
 * iteration 60 lands 3e-5 .. 5e-4 above the MAP that the polish from
 * iterations 50 or 70 reaches); one damped step keeps it in the basin. */
#define ORC_POLISH_LAM0 1e-2
int orc_polish_ex(const orc_problem *pb, double *theta, int max_it, int damp, double *f_out,
                  int *n_newton, int *n_eval, int *n_solve, int *cert_out) {
    return orc_polish_cfg(pb, theta, max_it, damp, damp ? ORC_POLISH_LAM0 : 0.0, f_out, n_newton, n_eval,
                          n_solve, cert_out);
}

int orc_polish(const orc_problem *pb, double *theta, int max_it, double *f_out,
               int *n_newton, int *n_eval, int *n_solve) {
    return orc_polish_ex(pb, theta, max_it, 0, f_out, n_newton, n_eval, n_solve, NULL);
}
