/*
 * ic_oracle.c — CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of one reference cleaning run
 * (/root/reference/iterative_cleaner.py:65-146) under the repo's archive
 * stand-in semantics (iterative_cleaner_amd/archive.py).  It is the checker
 * for the HIP path; it is never linked into libicgpu.so.
 *
 *   orc_lmdif1        scipy 1.15.3 leastsq(err,[1.0]) for n = 1
 *                     (scipy/optimize/_minpack_py.py:291-506 -> MINPACK lmdif,
 *                      fdjac2, qrfac, lmpar, qrsolv, enorm), used at
 *                     iterative_cleaner.py:277-279
 *   orc_template      template build, iterative_cleaner.py:88-94
 *   orc_fit_cube      fit-cube prep, iterative_cleaner.py:96-100
 *   orc_fit_residual  remove_profile_inplace / remove_profile1d, :259-288
 *   orc_diagnostics   comprehensive_stats diagnostics, :206-217
 *   orc_test          scalers + combine, :219-256
 *   orc_rotate        fractional dedispersion (psrchive's FFT phase rotation,
 *                     dedisperse / dededisperse at iterative_cleaner.py:91,
 *                     :100, :104) in the written order of
 *                     iterative_cleaner_amd/phase_rotation.py; parity with real
 *                     psrchive UNPINNED (psrchive absent), pinned to numpy's
 *                     irfft(rfft(x) * phasor) within one f32 ulp
 *   orc_clean_loop    the while loop, :83-146
 *
 * Build: gcc -O2 -fPIC -shared -ffp-contract=off -fno-fast-math -fopenmp (oracle/Makefile)
 * Pinned against the tests/golden npz fixtures (reference outputs) and live scipy.
 *
 * Threads (OpenMP, OMP_NUM_THREADS): the loops over profiles, subints and
 * median lines are split over threads.  Every item is computed by one thread
 * with the same operations in the same order as the serial loop, so the bits
 * do not depend on the thread count; only the order in which independent
 * items finish does.  The whole-archive checks at BASELINE.json's sizes
 * (tests/test_wholearchive_gpu.py) need that parallelism to run in seconds.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SUPER_BLOCK 256

/* Canonical combine of super-block partials p[lo*stride], .. p[(hi-1)*stride]
 * (archive.py sb_tree): halving tree, mid = lo + (hi - lo) / 2. */
static double sb_tree1(const double *p, size_t stride, int lo, int hi)
{
    if (hi - lo == 1) return p[(size_t)lo * stride];
    int mid = lo + (hi - lo) / 2;
    double a = sb_tree1(p, stride, lo, mid);
    double b = sb_tree1(p, stride, mid, hi);
    return a + b;
}

/* ------------------------------------------------------------------ enorm */
/* MINPACK enorm (sequential, three-accumulator scaled sum of squares).      */
static double enorm_d(int n, const double *x)
{
    const double rdwarf = 3.834e-20, rgiant = 1.304e19;
    double s1 = 0.0, s2 = 0.0, s3 = 0.0, x1max = 0.0, x3max = 0.0;
    double agiant = rgiant / (double)n;
    for (int i = 0; i < n; ++i) {
        double xabs = fabs(x[i]);
        if (xabs > rdwarf && xabs < agiant) {
            s2 += xabs * xabs;
        } else if (xabs <= rdwarf) {
            if (xabs > x3max) {
                double t = x3max / xabs;
                s3 = 1.0 + s3 * (t * t);
                x3max = xabs;
            } else if (xabs != 0.0) {
                double t = xabs / x3max;
                s3 += t * t;
            }
        } else {
            if (xabs > x1max) {
                double t = x1max / xabs;
                s1 = 1.0 + s1 * (t * t);
                x1max = xabs;
            } else {
                double t = xabs / x1max;
                s1 += t * t;
            }
        }
    }
    if (s1 != 0.0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
    if (s2 != 0.0) {
        if (s2 >= x3max) return sqrt(s2 * (1.0 + (x3max / s2) * (x3max * s3)));
        return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
    }
    return x3max * sqrt(s3);
}

static double enorm1(double v) { return enorm_d(1, &v); }
static double dmax(double a, double b) { return a >= b ? a : b; }
static double dmin(double a, double b) { return a <= b ? a : b; }

/* err(a) = a*T - p  (iterative_cleaner.py:277), f64, no contraction */
static void fcn(int m, double a, const float *T, const float *p, double *out)
{
    for (int i = 0; i < m; ++i) {
        double t = a * (double)T[i];
        out[i] = t - (double)p[i];
    }
}

/* MINPACK qrsolv for n = 1. r: R(0,0); w = sqrt(par)*diag; qtb = qtf.
 * returns x, writes sdiag. */
static double qrsolv1(double r, double w, double qtb, double *sdiag)
{
    double rr = r, wa = qtb, sd;
    if (w != 0.0) {
        sd = w;
        double qtbpj = 0.0;
        if (sd != 0.0) {
            double cs, sn;
            if (fabs(rr) >= fabs(sd)) {
                double tn = sd / rr;
                cs = 0.5 / sqrt(0.25 + 0.25 * (tn * tn));
                sn = cs * tn;
            } else {
                double ct = rr / sd;
                sn = 0.5 / sqrt(0.25 + 0.25 * (ct * ct));
                cs = sn * ct;
            }
            rr = cs * rr + sn * sd;
            double temp = cs * wa + sn * qtbpj;
            wa = temp;
        }
    }
    sd = rr;
    double x;
    if (sd == 0.0) {
        x = 0.0;
    } else {
        double sum = 0.0;
        x = (wa - sum) / sd;
    }
    *sdiag = sd;
    return x;
}

/* MINPACK lmpar for n = 1; returns the step x, updates *par. */
static double lmpar1(double r, double diag, double qtb, double delta, double *par_io)
{
    const double p1 = 0.1, p001 = 0.001, dwarf = DBL_MIN;
    double par = *par_io;
    int nsing = (r == 0.0) ? 0 : 1;
    double wa1 = qtb;
    if (nsing < 1) wa1 = 0.0;
    if (nsing >= 1) wa1 = wa1 / r;
    double x = wa1;
    int iter = 0;
    double wa2 = diag * x;
    double dxnorm = enorm1(wa2);
    double fp = dxnorm - delta;
    if (!(fp <= p1 * delta)) {
        double parl = 0.0;
        if (nsing >= 1) {
            double t = diag * (wa2 / dxnorm);
            double sum = 0.0;
            t = (t - sum) / r;
            double temp = enorm1(t);
            parl = ((fp / delta) / temp) / temp;
        }
        double sum = 0.0;
        sum += r * qtb;
        double g = sum / diag;
        double gnorm = enorm1(g);
        double paru = gnorm / delta;
        if (paru == 0.0) paru = dwarf / dmin(delta, p1);
        par = dmax(par, parl);
        par = dmin(par, paru);
        if (par == 0.0) par = gnorm / dxnorm;
        for (;;) {
            ++iter;
            if (par == 0.0) par = dmax(dwarf, p001 * paru);
            double temp = sqrt(par);
            double w = temp * diag;
            double sdiag;
            x = qrsolv1(r, w, qtb, &sdiag);
            wa2 = diag * x;
            dxnorm = enorm1(wa2);
            temp = fp;
            fp = dxnorm - delta;
            if (fabs(fp) <= p1 * delta || (parl == 0.0 && fp <= temp && temp < 0.0) || iter == 10)
                break;
            double t = diag * (wa2 / dxnorm);
            t = t / sdiag;
            double tn = enorm1(t);
            double parc = ((fp / delta) / tn) / tn;
            if (fp > 0.0) parl = dmax(parl, par);
            if (fp < 0.0) paru = dmin(paru, par);
            par = dmax(parl, par + parc);
        }
    }
    if (iter == 0) par = 0.0;
    *par_io = par;
    return x;
}

/* scipy.optimize.leastsq(err, [1.0]) with err(a) = a*T - p.
 * Returns info; *x_out = solution; *nfev_out = evaluations inside lmdif.
 * work: 3*m doubles (or NULL). */
int orc_lmdif1(int m, const float *T, const float *p, double *x_out, int *nfev_out, double *work)
{
    const double ftol = 1.49012e-8, xtol = 1.49012e-8, gtol = 0.0;
    const double epsfcn = DBL_EPSILON, epsmch = DBL_EPSILON, factor = 100.0;
    const int maxfev = 400;
    double *own = NULL;
    if (!work) work = own = (double *)malloc(sizeof(double) * 3 * (size_t)(m > 0 ? m : 1));
    double *fvec = work, *wa4 = work + m, *fjac = work + 2 * m;
    int info = 0, nfev = 0;
    double x = 1.0;

    fcn(m, x, T, p, fvec);
    nfev = 1;
    double fnorm = enorm_d(m, fvec);
    double par = 0.0, xnorm = 0.0, delta = 0.0, diag = 0.0;
    int iter = 1;
    for (;;) {
        /* fdjac2 */
        double eps = sqrt(dmax(epsfcn, epsmch));
        double temp = x;
        double h = eps * fabs(temp);
        if (h == 0.0) h = eps;
        double xh = temp + h;
        fcn(m, xh, T, p, wa4);
        for (int i = 0; i < m; ++i) fjac[i] = (wa4[i] - fvec[i]) / h;
        nfev += 1;
        /* qrfac, n = 1, pivoting */
        double acnorm = enorm_d(m, fjac);
        double ajnorm = enorm_d(m, fjac);
        if (ajnorm != 0.0) {
            if (fjac[0] < 0.0) ajnorm = -ajnorm;
            for (int i = 0; i < m; ++i) fjac[i] = fjac[i] / ajnorm;
            fjac[0] = fjac[0] + 1.0;
        }
        double rdiag = -ajnorm;
        if (iter == 1) {
            diag = acnorm;
            if (diag == 0.0) diag = 1.0;
            xnorm = enorm1(diag * x);
            delta = factor * xnorm;
            if (delta == 0.0) delta = factor;
        }
        /* qtf = (Q^T fvec)[0] */
        double qtf = fvec[0];
        if (fjac[0] != 0.0) {
            double sum = 0.0;
            for (int i = 0; i < m; ++i) sum += fjac[i] * fvec[i];
            double t = -sum / fjac[0];
            qtf = fvec[0] + fjac[0] * t;
        }
        double r = rdiag;
        double gnorm = 0.0;
        if (fnorm != 0.0 && acnorm != 0.0) {
            double sum = 0.0;
            sum += r * (qtf / fnorm);
            /* scipy keeps gnorm = 0 when this term is NaN (non-finite profile):
             * info 4 at once with x = 1 (tests/golden/leastsq_nonfinite.npz) */
            double g = fabs(sum / acnorm);
            if (g > gnorm) gnorm = g;
        }
        if (gnorm <= gtol) info = 4;
        if (info != 0) break;
        diag = dmax(diag, acnorm);
        for (;;) {
            double step = lmpar1(r, diag, qtf, delta, &par);
            double wa1 = -step;
            double x2 = x + wa1;
            double pnorm = enorm1(diag * wa1);
            if (iter == 1) delta = dmin(delta, pnorm);
            fcn(m, x2, T, p, wa4);
            nfev += 1;
            double fnorm1 = enorm_d(m, wa4);
            double actred = -1.0;
            if (0.1 * fnorm1 < fnorm) {
                double t = fnorm1 / fnorm;
                actred = 1.0 - t * t;
            }
            double w3 = 0.0;
            w3 += r * wa1;
            double temp1 = enorm1(w3) / fnorm;
            double temp2 = (sqrt(par) * pnorm) / fnorm;
            double prered = temp1 * temp1 + temp2 * temp2 / 0.5;
            double dirder = -(temp1 * temp1 + temp2 * temp2);
            double ratio = 0.0;
            if (prered != 0.0) ratio = actred / prered;
            if (ratio <= 0.25) {
                double tt = 0.0;
                if (actred >= 0.0) tt = 0.5;
                if (actred < 0.0) tt = 0.5 * dirder / (dirder + 0.5 * actred);
                if (0.1 * fnorm1 >= fnorm || tt < 0.1) tt = 0.1;
                delta = tt * dmin(delta, pnorm / 0.1);
                par = par / tt;
            } else if (par == 0.0 || ratio >= 0.75) {
                delta = pnorm / 0.5;
                par = 0.5 * par;
            }
            if (ratio >= 1e-4) {
                x = x2;
                double w2 = diag * x;
                memcpy(fvec, wa4, sizeof(double) * (size_t)m);
                xnorm = enorm1(w2);
                fnorm = fnorm1;
                iter += 1;
            }
            if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0) info = 1;
            if (delta <= xtol * xnorm) info = 2;
            if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0 && info == 2) info = 3;
            if (info != 0) goto done;
            if (nfev >= maxfev) info = 5;
            if (fabs(actred) <= epsmch && prered <= epsmch && 0.5 * ratio <= 1.0) info = 6;
            if (delta <= epsmch * xnorm) info = 7;
            if (gnorm <= epsmch) info = 8;
            if (info != 0) goto done;
            if (ratio >= 1e-4) break;
        }
    }
done:
    *x_out = x;
    if (nfev_out) *nfev_out = nfev;
    free(own);
    return info;
}

/* ---------------------------------------------------------- fit + residual */
/* remove_profile1d (iterative_cleaner.py:275-288) + f32 store (:272).
 * D: fit cube (P, m) dedispersed; R out (P, m) f32 dedispersed frame. */
void orc_fit_residual(int P, int m, const float *T, const float *D,
                      int pr_on, double pr_factor, int pr_start, int pr_end,
                      double *amp, int32_t *info, float *R)
{
#pragma omp parallel
    {
    double *work = (double *)malloc(sizeof(double) * 3 * (size_t)m);
#pragma omp for schedule(dynamic, 64)
    for (int k = 0; k < P; ++k) {
        const float *p = D + (size_t)k * m;
        double x;
        int st = orc_lmdif1(m, T, p, &x, NULL, work);
        amp[k] = x;
        info[k] = st;
        float *o = R + (size_t)k * m;
        if (st < 1 || st > 4) {
            for (int i = 0; i < m; ++i) o[i] = 0.0f;
            continue;
        }
        for (int i = 0; i < m; ++i) {
            double t = x * (double)T[i];
            double e = t - (double)p[i];
            if (pr_on && i >= pr_start && i < pr_end) e = e * pr_factor;
            o[i] = (float)e;
        }
    }
    free(work);
    }
}

/* ------------------------------------------------------- archive stand-in */
static inline float ded_at(const float *prof, int n, int shift, int i)
{
    int j = i + shift;
    if (j >= n) j -= n;
    return prof[j];
}

/* remove_baseline (archive.py): per subint window from the weighted total.
 * raw (nsub, nchan, n) dispersed frame; W weights; writes base (nsub*nchan). */
void orc_baseline(int nsub, int nchan, int n, const float *raw, const float *W,
                  const int32_t *shift, double duty, float *base, int32_t *win_out)
{
    int width = (int)(duty * (double)n);
    if (width < 1) width = 1;
    const int nsb = (nchan + SUPER_BLOCK - 1) / SUPER_BLOCK;
#pragma omp parallel
    {
    double *tot = (double *)malloc(sizeof(double) * (size_t)n);
    double *part = (double *)malloc(sizeof(double) * (size_t)n * nsb);
#pragma omp for schedule(dynamic, 1)
    for (int s = 0; s < nsub; ++s) {
        for (int b0 = 0; b0 < nchan; b0 += SUPER_BLOCK) {
            double *pb = part + (size_t)(b0 / SUPER_BLOCK) * n;
            for (int i = 0; i < n; ++i) pb[i] = 0.0;
            int b1 = b0 + SUPER_BLOCK < nchan ? b0 + SUPER_BLOCK : nchan;
            for (int c = b0; c < b1; ++c) {
                const float *prof = raw + ((size_t)s * nchan + c) * n;
                double w = (double)W[(size_t)s * nchan + c];
                for (int i = 0; i < n; ++i) pb[i] = pb[i] + w * (double)ded_at(prof, n, shift[c], i);
            }
        }
        for (int i = 0; i < n; ++i) tot[i] = sb_tree1(part + i, (size_t)n, 0, nsb);
        /* first argmin of circular window sums, numpy NaN semantics */
        int best = 0;
        double bestv = 0.0;
        for (int j = 0; j < n; ++j) {
            double msum = 0.0;
            for (int k = 0; k < width; ++k) {
                int q = j + k;
                q %= n;
                msum = msum + tot[q];
            }
            if (j == 0) { best = 0; bestv = msum; continue; }
            if (isnan(bestv)) continue;
            if (isnan(msum) || msum < bestv) { best = j; bestv = msum; }
        }
        if (win_out) win_out[s] = best;
        for (int c = 0; c < nchan; ++c) {
            const float *prof = raw + ((size_t)s * nchan + c) * n;
            double acc = 0.0;
            for (int k = 0; k < width; ++k) acc = acc + (double)ded_at(prof, n, shift[c], (best + k) % n);
            base[(size_t)s * nchan + c] = (float)(acc / (double)width);
        }
    }
    free(tot);
    free(part);
    }
}

/* fit cube (iterative_cleaner.py:96-100): D = f32(ded - base(w0)). */
void orc_fit_cube(int nsub, int nchan, int n, const float *raw, const float *w0,
                  const int32_t *shift, double duty, float *D)
{
    float *base = (float *)malloc(sizeof(float) * (size_t)nsub * nchan);
    orc_baseline(nsub, nchan, n, raw, w0, shift, duty, base, NULL);
#pragma omp parallel for schedule(static)
    for (int s = 0; s < nsub; ++s)
        for (int c = 0; c < nchan; ++c) {
            const float *prof = raw + ((size_t)s * nchan + c) * n;
            float b = base[(size_t)s * nchan + c];
            float *o = D + ((size_t)s * nchan + c) * n;
            for (int i = 0; i < n; ++i) o[i] = ded_at(prof, n, shift[c], i) - b;
        }
    free(base);
}

/* template (iterative_cleaner.py:88-94): remove_baseline(W), dedisperse,
 * fscrunch, tscrunch, amps * 10000 (f32). */
static void orc_scrunch(int nsub, int nchan, int n, const float *raw, const float *W,
                        const int32_t *shift, const float *base, float *T);

void orc_template(int nsub, int nchan, int n, const float *raw, const float *W,
                  const int32_t *shift, double duty, float *T)
{
    float *base = (float *)malloc(sizeof(float) * (size_t)nsub * nchan);
    orc_baseline(nsub, nchan, n, raw, W, shift, duty, base, NULL);
    orc_scrunch(nsub, nchan, n, raw, W, shift, base, T);
    free(base);
}

/* dedisperse (integer shifts), fscrunch, tscrunch of f32(raw - base), amps * 10000 */
static void orc_scrunch(int nsub, int nchan, int n, const float *raw, const float *W,
                        const int32_t *shift, const float *base, float *T)
{
    const int nsb = (nchan + SUPER_BLOCK - 1) / SUPER_BLOCK;
    double *num = (double *)malloc(sizeof(double) * (size_t)n);
    float *F = (float *)malloc(sizeof(float) * (size_t)nsub * n);
    float *wf = (float *)malloc(sizeof(float) * (size_t)nsub);
#pragma omp parallel
    {
    double *num = (double *)malloc(sizeof(double) * (size_t)n);
    double *part = (double *)malloc(sizeof(double) * (size_t)n * nsb);
    double *wpart = (double *)malloc(sizeof(double) * (size_t)nsb);
#pragma omp for schedule(dynamic, 1)
    for (int s = 0; s < nsub; ++s) {
        for (int b0 = 0; b0 < nchan; b0 += SUPER_BLOCK) {
            int b1 = b0 + SUPER_BLOCK < nchan ? b0 + SUPER_BLOCK : nchan;
            double *pb = part + (size_t)(b0 / SUPER_BLOCK) * n;
            double wp = 0.0;
            for (int i = 0; i < n; ++i) pb[i] = 0.0;
            for (int c = b0; c < b1; ++c) {
                const float *prof = raw + ((size_t)s * nchan + c) * n;
                double w = (double)W[(size_t)s * nchan + c];
                float b = base[(size_t)s * nchan + c];
                wp = wp + w;
                for (int i = 0; i < n; ++i) {
                    float y = ded_at(prof, n, shift[c], i) - b;
                    pb[i] = pb[i] + w * (double)y;
                }
            }
            wpart[b0 / SUPER_BLOCK] = wp;
        }
        const double wsum = sb_tree1(wpart, 1, 0, nsb);
        for (int i = 0; i < n; ++i) num[i] = sb_tree1(part + i, (size_t)n, 0, nsb);
        for (int i = 0; i < n; ++i) F[(size_t)s * n + i] = (wsum != 0.0) ? (float)(num[i] / wsum) : 0.0f;
        wf[s] = (float)wsum;
    }
    free(num); free(part); free(wpart);
    }
    double wt = 0.0;
    for (int i = 0; i < n; ++i) num[i] = 0.0;
    for (int s = 0; s < nsub; ++s) {
        double w = (double)wf[s];
        wt = wt + w;
        for (int i = 0; i < n; ++i) num[i] = num[i] + w * (double)F[(size_t)s * n + i];
    }
    for (int i = 0; i < n; ++i) {
        float t = (wt != 0.0) ? (float)(num[i] / wt) : 0.0f;
        T[i] = t * 10000.0f;
    }
    free(num); free(F); free(wf);
}

/* ------------------------------------------- fractional dedispersion (FFT) */
/* tw[2q], tw[2q+1] = cos, sin of -2 pi q / n (x87 long double, rounded to f64) */
void orc_twiddles(int n, double *tw)
{
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int q = 0; q < n; ++q) {
        const long double ang = -2.0L * pi * (long double)q / (long double)n;
        tw[2 * q] = (double)cosl(ang);
        tw[2 * q + 1] = (double)sinl(ang);
    }
}

/* o[0], o[1] = cos, sin of 2 pi k d / n, harmonic k of a delay of d bins (n a
 * power of two), in the written f64 order of phase_rotation.py phasors (the
 * GPU's ic_phasor):
 *   Veltkamp split d = dh + dl with dh of 40 bits (c = d * 8193), so that
 *   k dh and k dl are exact; t = k dh - n rint(k dh / n) (exact, |t| <= n/2);
 *   y = (t + k dl) * (4/n) quarter turns; q = rint(y), z = y - q;
 *   sin / cos of (pi/2) z by Horner in w = z^2 on the Taylor coefficients
 *   (-1)^j (pi/2)^(2j+1)/(2j+1)!, j <= 8, and (-1)^j (pi/2)^(2j)/(2j)!, j <= 8;
 *   then the quadrant q mod 4. */
static const double PH_S[9] = {0x1.921fb54442d18p+0,  -0x1.4abbce625be53p-1, 0x1.466bc6775aae2p-4,
                               -0x1.32d2cce62bd86p-8, 0x1.50783487ee782p-13, -0x1.e3074fde8871fp-19,
                               0x1.e8f434d018d63p-25, -0x1.6fadb9f155744p-31, 0x1.aaec32af93359p-38};
static const double PH_C[9] = {1.0,                   -0x1.3bd3cc9be45dep+0, 0x1.03c1f081b5ac4p-2,
                               -0x1.55d3c7e3cbffap-6, 0x1.e1f506891babbp-11, -0x1.a6d1f2a204a8cp-16,
                               0x1.f9d38a3763cc3p-22, -0x1.b6e24f44b128fp-28, 0x1.20c62c2f2d7f5p-34};
static void orc_phasor0(int k, double d, int n, double *o)
{
    const double c = d * 8193.0;
    const double dh = c - (c - d), dl = d - dh;
    const double nn = (double)n;
    const double xh = (double)k * dh, xl = (double)k * dl;
    const double t = xh - nn * rint(xh * (1.0 / nn));
    const double y = (t + xl) * (4.0 / nn);
    const double q = rint(y);
    const double z = y - q, w = z * z;
    double sp = PH_S[8], cp = PH_C[8];
    for (int j = 7; j >= 0; --j) {
        sp = PH_S[j] + w * sp;
        cp = PH_C[j] + w * cp;
    }
    const double sn = z * sp;
    switch ((int)q & 3) {
    case 0: o[0] = cp;  o[1] = sn;  break;
    case 1: o[0] = -sn; o[1] = cp;  break;
    case 2: o[0] = -cp; o[1] = -sn; break;
    default: o[0] = sn; o[1] = -cp; break;
    }
}

/* The phasor of harmonic k (ic_phasor): orc_phasor0 for k < 64 and multiples
 * of 64, else the product P0(k mod 64) P0(k - k mod 64) of separately rounded
 * operations (re = a.re b.re - a.im b.im, im = a.re b.im + a.im b.re). */
static void orc_phasor(int k, double d, int n, double *o)
{
    const int lo = k & 63, hi = k - lo;
    if (lo == 0 || hi == 0) {
        orc_phasor0(k, d, n, o);
        return;
    }
    double a[2], b[2];
    orc_phasor0(lo, d, n, a);
    orc_phasor0(hi, d, n, b);
    const double re1 = a[0] * b[0], re2 = a[1] * b[1];
    const double im1 = a[0] * b[1], im2 = a[1] * b[0];
    o[0] = re1 - re2;
    o[1] = im1 + im2;
}

/* ph[(c*(n/2+1) + k)*2 + {0,1}] = orc_phasor(k, delay[c], n) */
void orc_phasors(int n, int nchan, const double *delay, double *ph)
{
    const int m = n / 2;
    for (int c = 0; c < nchan; ++c)
        for (int k = 0; k <= m; ++k) orc_phasor(k, delay[c], n, ph + ((size_t)c * (m + 1) + k) * 2);
}

/* FFT of m complex points (re/im interleaved) through `tmp`, in IEEE f32 (psrchive's
 * precision): Stockham stages of radix 8 while three or more of the log2 m levels
 * remain, then one of radix 4 or 2 (phase_rotation.py _stockham, the GPU's
 * rot_pass).  Stage (R, ns), butterfly j < m/R: k = j mod ns, a_q = v[j + q m/R];
 * for ns > 1, b_q = a_q times tw[q k n/(R ns)] (q >= 1); y = DFT_R(b) in the
 * written order below; out[(j - k) R + k + p ns] = y_p.  tw: the f32 table. */
#define ROT_S8 ((float)0x1.6a09e667f3bcdp-1)   /* f32(f64(sqrt(2)/2)) = Re exp(-i pi/4) */
static void dft4(float *r, float *i)   /* in place, 4 points */
{
    const float c0r = r[0] + r[2], c0i = i[0] + i[2];
    const float c1r = r[0] - r[2], c1i = i[0] - i[2];
    const float c2r = r[1] + r[3], c2i = i[1] + i[3];
    const float dr = r[1] - r[3], di = i[1] - i[3];
    const float c3r = di, c3i = -dr;
    r[0] = c0r + c2r; i[0] = c0i + c2i;
    r[1] = c1r + c3r; i[1] = c1i + c3i;
    r[2] = c0r - c2r; i[2] = c0i - c2i;
    r[3] = c1r - c3r; i[3] = c1i - c3i;
}
static void dft8(float *r, float *i)   /* in place, 8 points, natural output order */
{
    float cr[8], ci[8];
    for (int q = 0; q < 4; ++q) {
        cr[q] = r[q] + r[q + 4]; ci[q] = i[q] + i[q + 4];
        cr[q + 4] = r[q] - r[q + 4]; ci[q + 4] = i[q] - i[q + 4];
    }
    float t1 = cr[5] + ci[5], t2 = ci[5] - cr[5];
    cr[5] = t1 * ROT_S8; ci[5] = t2 * ROT_S8;
    t1 = ci[6]; ci[6] = -cr[6]; cr[6] = t1;
    t1 = ci[7] - cr[7]; t2 = cr[7] + ci[7];
    cr[7] = t1 * ROT_S8; ci[7] = -(t2 * ROT_S8);
    dft4(cr, ci);
    dft4(cr + 4, ci + 4);
    for (int p = 0; p < 4; ++p) {
        r[2 * p] = cr[p]; i[2 * p] = ci[p];
        r[2 * p + 1] = cr[p + 4]; i[2 * p + 1] = ci[p + 4];
    }
}
static void stockham(int m, float *v, float *tmp, const float *tw)
{
    const int n = 2 * m;
    int lg = 0;
    while ((1 << lg) < m) ++lg;
    for (int ns = 1, done = 0; done < lg;) {
        const int rem = lg - done, R = rem >= 3 ? 8 : (rem == 2 ? 4 : 2);
        const int g = m / R;
        for (int j = 0; j < g; ++j) {
            const int k = j & (ns - 1);
            float br[8], bi[8];
            for (int q = 0; q < R; ++q) {
                const float ar = v[2 * (j + q * g)], ai = v[2 * (j + q * g) + 1];
                if (ns > 1 && q > 0) {
                    const float *w = tw + 2 * (size_t)(q * k * (n / (R * ns)));
                    const float p1 = ar * w[0], p2 = ai * w[1];
                    const float p3 = ar * w[1], p4 = ai * w[0];
                    br[q] = p1 - p2;
                    bi[q] = p3 + p4;
                } else {
                    br[q] = ar;
                    bi[q] = ai;
                }
            }
            if (R == 8) {
                dft8(br, bi);
            } else if (R == 4) {
                dft4(br, bi);
            } else {
                const float y0r = br[0] + br[1], y0i = bi[0] + bi[1];
                const float y1r = br[0] - br[1], y1i = bi[0] - bi[1];
                br[0] = y0r; bi[0] = y0i; br[1] = y1r; bi[1] = y1i;
            }
            const int o = (j - k) * R + k;
            for (int p = 0; p < R; ++p) {
                tmp[2 * (o + p * ns)] = br[p];
                tmp[2 * (o + p * ns) + 1] = bi[p];
            }
        }
        memcpy(v, tmp, sizeof(float) * 2 * (size_t)m);
        ns *= R;
        done += R == 8 ? 3 : (R == 4 ? 2 : 1);
    }
}

/* The inverse's half-length inputs conj(Z'_k), conj(Z'_q) (q = M - k), what it
 * stores, from Z_k, Z_q in one linear map (phase_rotation.py _pair), f32: w_k =
 * (c, sn), phasors pk, pq (their imaginary parts signed for the direction); the
 * conjugate's imaginary part is (-a) + (-b) of the two terms'. */
static void rot_pair(const float *zk, const float *zq, float c, float sn, const float *pk, const float *pq,
                     float *ok, float *oq)
{
    const float h1 = (1.0f + sn) * 0.5f, h2 = (1.0f - sn) * 0.5f, hc = c * 0.5f;
    const float akr = h1 * pk[0] + h2 * pq[0], aki = h1 * pk[1] - h2 * pq[1];
    const float aqr = h1 * pq[0] + h2 * pk[0], aqi = h1 * pq[1] - h2 * pk[1];
    const float bkr = -(hc * (pk[1] + pq[1])), bki = hc * (pk[0] - pq[0]);
    ok[0] = (akr * zk[0] - aki * zk[1]) + (bkr * zq[0] + bki * zq[1]);
    ok[1] = (-(akr * zk[1] + aki * zk[0])) + (-(bki * zq[0] - bkr * zq[1]));
    oq[0] = (aqr * zq[0] - aqi * zq[1]) + (bki * zk[1] - bkr * zk[0]);
    oq[1] = (-(aqr * zq[1] + aqi * zq[0])) + (-(bki * zk[0] + bkr * zk[1]));
}

/* One profile: out = rotation of f32(x - b) by the phasors p (f64, rounded to f32
 * here; sign +1: dedisperse, y[j] = x[j + s]; -1: dededisperse).  tw: the f32
 * table.  work: 4n floats. */
static void rotate1(int n, const float *x, float b, const double *p, int sign, const float *tw,
                    float *work, float *out)
{
    const int m = n / 2;
    float *v = work, *tmp = work + 2 * (size_t)m;
    for (int j = 0; j < m; ++j) {
        v[2 * j] = x[2 * j] - b;
        v[2 * j + 1] = x[2 * j + 1] - b;
    }
    stockham(m, v, tmp, tw);
    const double sg = sign > 0 ? 1.0 : -1.0;
    {
        const float X0 = v[0] + v[1], XM = v[0] - v[1];
        const float Y0 = X0 * (float)p[0], YM = XM * (float)p[2 * m];
        v[0] = (Y0 + YM) * 0.5f;
        v[1] = -((Y0 - YM) * 0.5f);
    }
    for (int k = 1; k <= m / 2; ++k) {
        const int q = m - k;
        float zk[2] = {v[2 * k], v[2 * k + 1]}, zq[2] = {v[2 * q], v[2 * q + 1]};
        float Zk[2], Zq[2];
        const float pk[2] = {(float)p[2 * k], (float)(sg * p[2 * k + 1])};
        const float pq[2] = {(float)p[2 * q], (float)(sg * p[2 * q + 1])};
        rot_pair(zk, zq, tw[2 * k], tw[2 * k + 1], pk, pq, Zk, Zq);
        v[2 * q] = Zq[0];   /* conjugated by rot_pair */
        v[2 * q + 1] = Zq[1];
        v[2 * k] = Zk[0];   /* k = M/2 pairs with itself: k's values last */
        v[2 * k + 1] = Zk[1];
    }
    stockham(m, v, tmp, tw);
    const float inv = (float)(1.0 / (double)m);
    for (int j = 0; j < m; ++j) {
        out[2 * j] = v[2 * j] * inv;
        out[2 * j + 1] = (-v[2 * j + 1]) * inv;
    }
}

/* Rotate every profile of a (nsub, nchan, n) cube by its delay:
 * out = rot(f32(in - base)) (base may be NULL = 0).  n a power of two >= 4.
 * per_profile 0: delay [nchan] (a channel's delay for every subint);
 * 1: delay [nsub*nchan], profile k's own (psrchive's per-Integration period).
 * identity: the rotation of an archive stored dedispersed, whose dedisperse is
 * a no-op: out = f32(in - base). */
void orc_rotate_ex(int nsub, int nchan, int n, const float *in, const float *base, const double *delay,
                   int per_profile, int identity, int sign, float *out)
{
    const int m = n / 2;
    const size_t P = (size_t)nsub * nchan;
    if (identity) {
        for (size_t k = 0; k < P; ++k) {
            const float b = base ? base[k] : 0.0f;
            for (int j = 0; j < n; ++j) out[k * n + j] = in[k * n + j] - b;
        }
        return;
    }
    double *tw64 = (double *)malloc(sizeof(double) * 2 * (size_t)n);
    float *tw = (float *)malloc(sizeof(float) * 2 * (size_t)n);
    double *ph = (double *)malloc(sizeof(double) * 2 * (per_profile ? P : (size_t)nchan) * (m + 1));
    orc_twiddles(n, tw64);
    for (int q = 0; q < 2 * n; ++q) tw[q] = (float)tw64[q];
    free(tw64);
    orc_phasors(n, per_profile ? (int)P : nchan, delay, ph);
#pragma omp parallel
    {
    float *work = (float *)malloc(sizeof(float) * 4 * (size_t)n);
#pragma omp for schedule(dynamic, 64)
    for (long k = 0; k < (long)P; ++k) {
        const size_t row = per_profile ? (size_t)k : (size_t)(k % nchan);
        rotate1(n, in + (size_t)k * n, base ? base[k] : 0.0f, ph + row * (m + 1) * 2, sign, tw, work,
                out + (size_t)k * n);
    }
    free(work);
    }
    free(tw); free(ph);
}

void orc_rotate(int nsub, int nchan, int n, const float *in, const float *base, const double *delay,
                int sign, float *out)
{
    orc_rotate_ex(nsub, nchan, n, in, base, delay, 0, 0, sign, out);
}

/* ------------------------------------------------------ pairwise sums */
static float pw_f32(const float *a, int n, int stride)
{
    if (n < 8) {
        float res = 0.0f;
        for (int i = 0; i < n; ++i) res += a[(size_t)i * stride];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[(size_t)j * stride];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[(size_t)(i + j) * stride];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[(size_t)i * stride];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_f32(a, n2, stride) + pw_f32(a + (size_t)n2 * stride, n - n2, stride);
}

static double pw_f64(const double *a, int n)
{
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_f64(a, n2) + pw_f64(a + n2, n - n2);
}

float orc_sum_f32(const float *a, int n) { return 0.0f + pw_f32(a, n, 1); }
double orc_sum_f64(const double *a, int n) { return 0.0 + pw_f64(a, n); }

/* ------------------------------------------------- closed-form fit (fast mode) */
/* fit_mode 1 (IC_FIT_CLOSED, include/iterative_cleaner.h): NOT the reference's
 * arithmetic (which is leastsq, iterative_cleaner.py:277-278) but its closed-form
 * least-squares solution, stated in numpy terms as
 *     TT = np.sum(T64 * T64);  a = np.sum(np.roll(T64 * p64, sh)) / TT   (pairwise f64 sums)
 * the products summed in the archive's stored (dispersed) sample order, sample j
 * pairing with the dedispersed bin (j - sh) mod m (round 6; the dedispersed order
 * before), with a = 0 when TT == 0 and status 1 (5 when a is not finite: residual
 * zeroed, like a failed leastsq, :284-286).  The residual follows :279-283 as in
 * the exact mode.  D: fit cube (P, m), dedispersed; shift: [nchan] channel shifts
 * of the rows (row k is channel k % nchan), or NULL (0). */
void orc_fit_closed(int P, int m, const float *T, const float *D,
                    int pr_on, double pr_factor, int pr_start, int pr_end,
                    double *amp, int32_t *info, float *R, const int32_t *shift, int nchan)
{
    double *prod = (double *)malloc(sizeof(double) * (size_t)m);
    for (int i = 0; i < m; ++i) prod[i] = (double)T[i] * (double)T[i];
    const double TT = orc_sum_f64(prod, m);
    for (int k = 0; k < P; ++k) {
        const float *p = D + (size_t)k * m;
        const int sh = shift ? (int)(((shift[k % nchan] % m) + m) % m) : 0;
        for (int j = 0; j < m; ++j) {
            int i = j - sh;
            if (i < 0) i += m;
            prod[j] = (double)T[i] * (double)p[i];
        }
        const double dot = orc_sum_f64(prod, m);
        const double x = TT != 0.0 ? dot / TT : 0.0;
        const int st = isfinite(x) ? 1 : 5;
        amp[k] = x;
        info[k] = st;
        float *o = R + (size_t)k * m;
        for (int i = 0; i < m; ++i) {
            if (st != 1) { o[i] = 0.0f; continue; }
            double t = x * (double)T[i];
            double e = t - (double)p[i];
            if (pr_on && i >= pr_start && i < pr_end) e = e * pr_factor;
            o[i] = (float)e;
        }
    }
    free(prod);
}

/* ------------------------------------------------------------ fft max */
/* max_k |DFT(x)_k| for k = 0..n/2 (np.fft.rfft magnitude; tolerance-level
 * agreement with pocketfft).  Radix-2 iterative for powers of two, direct
 * DFT otherwise.  work: 4*n doubles. */
/* the radix-2 twiddles cos / -sin(2 pi idx / n), idx < n/2, exactly as the
 * butterflies below computed them per use: [2 * idx] = c, [2 * idx + 1] = s */
static double *fft_table(int n)
{
    if (n < 2 || (n & (n - 1))) return NULL;
    double *t = (double *)malloc(sizeof(double) * (size_t)n);
    for (int idx = 0; idx < n / 2; ++idx) {
        t[2 * idx] = cos(2.0 * M_PI * (double)idx / (double)n);
        t[2 * idx + 1] = -sin(2.0 * M_PI * (double)idx / (double)n);
    }
    return t;
}

static double fftmax(const double *x, int n, double *work, const double *tab)
{
    double best = 0.0;
    int pow2 = n > 0 && (n & (n - 1)) == 0;
    if (n == 1) return fabs(x[0]);
    if (pow2) {
        double *re = work, *im = work + n;
        int lg = 0;
        while ((1 << lg) < n) ++lg;
        for (int i = 0; i < n; ++i) {
            int rv = 0;
            for (int b = 0; b < lg; ++b) rv |= ((i >> b) & 1) << (lg - 1 - b);
            re[rv] = x[i];
            im[rv] = 0.0;
        }
        for (int len = 2; len <= n; len <<= 1) {
            int half = len >> 1;
            int step = n / len;
            for (int st = 0; st < n; st += len)
                for (int k = 0; k < half; ++k) {
                    /* twiddle exp(-2 pi i k/len) = exp(-2 pi i (k*step)/n) */
                    int idx = k * step;
                    double c = tab[2 * idx];
                    double s = tab[2 * idx + 1];
                    double ur = re[st + k], ui = im[st + k];
                    double vr = re[st + k + half] * c - im[st + k + half] * s;
                    double vi = re[st + k + half] * s + im[st + k + half] * c;
                    re[st + k] = ur + vr; im[st + k] = ui + vi;
                    re[st + k + half] = ur - vr; im[st + k + half] = ui - vi;
                }
        }
        for (int k = 0; k <= n / 2; ++k) {
            double a = hypot(re[k], im[k]);
            if (isnan(a)) return a;
            if (a > best) best = a;
        }
        return best;
    }
    for (int k = 0; k <= n / 2; ++k) {
        double sr = 0.0, si = 0.0;
        for (int j = 0; j < n; ++j) {
            long q = ((long)k * j) % n;
            double ang = 2.0 * M_PI * (double)q / (double)n;
            sr += x[j] * cos(ang);
            si -= x[j] * sin(ang);
        }
        double a = hypot(sr, si);
        if (isnan(a)) return a;
        if (a > best) best = a;
    }
    return best;
}

/* ----------------------------------------------------- diagnostics */
/* X: weighted cube (P, n) f32, dispersed frame; valid (P).
 * std/mean/fft f64, ptp f32, with numpy.ma data conventions. */
void orc_diagnostics(int P, int n, const float *X, const uint8_t *valid,
                     double *std_o, double *mean_o, float *ptp_o, double *fft_o)
{
    double *tab = fft_table(n);
#pragma omp parallel
    {
    double *d = (double *)malloc(sizeof(double) * (size_t)n);
    double *sq = (double *)malloc(sizeof(double) * (size_t)n);
    double *work = (double *)malloc(sizeof(double) * 4 * (size_t)n);
#pragma omp for schedule(dynamic, 256)
    for (int k = 0; k < P; ++k) {
        const float *x = X + (size_t)k * n;
        if (!valid[k]) {
            std_o[k] = 0.0;
            mean_o[k] = 0.0;
            ptp_o[k] = 1e20f;
            for (int i = 0; i < n; ++i) d[i] = (double)x[i];
            fft_o[k] = fftmax(d, n, work, tab);
            continue;
        }
        float s32 = orc_sum_f32(x, n);
        double mean = (double)s32 / (double)n;
        for (int i = 0; i < n; ++i) {
            d[i] = (double)x[i] - mean;
            sq[i] = d[i] * d[i];
        }
        double var = orc_sum_f64(sq, n) / (double)n;
        float mx = x[0], mn = x[0];
        int nan = 0;
        for (int i = 0; i < n; ++i) {
            if (isnan(x[i])) nan = 1;
            if (x[i] > mx) mx = x[i];
            if (x[i] < mn) mn = x[i];
        }
        /* numpy.ma masks a non-finite mean (the domained divide of ma.mean), so
         * every anomaly of ma.var is masked and its sum is 0: std 0 */
        std_o[k] = isfinite(mean) ? sqrt(var) : 0.0;
        mean_o[k] = mean;
        ptp_o[k] = nan ? NAN : (mx - mn);
        fft_o[k] = fftmax(d, n, work, tab);
    }
    free(d); free(sq); free(work);
    }
    free(tab);
}

/* f64 data (psrchive get_data returning f64; ic_params.data_f64): X is the f64
 * product f64(R) * f64(w), and numpy.ma sums, ptp and scales in f64
 * (iterative_cleaner.py:111-112, :206-209). */
void orc_diagnostics_f64(int P, int n, const double *X, const uint8_t *valid,
                         double *std_o, double *mean_o, double *ptp_o, double *fft_o)
{
    double *tab = fft_table(n);
#pragma omp parallel
    {
    double *d = (double *)malloc(sizeof(double) * (size_t)n);
    double *sq = (double *)malloc(sizeof(double) * (size_t)n);
    double *work = (double *)malloc(sizeof(double) * 4 * (size_t)n);
#pragma omp for schedule(dynamic, 256)
    for (int k = 0; k < P; ++k) {
        const double *x = X + (size_t)k * n;
        if (!valid[k]) {
            std_o[k] = 0.0;
            mean_o[k] = 0.0;
            ptp_o[k] = 1e20;    /* numpy.ma's f64 fill value (f32 data: f32(1e20)) */
            for (int i = 0; i < n; ++i) d[i] = x[i];
            fft_o[k] = fftmax(d, n, work, tab);
            continue;
        }
        double mean = orc_sum_f64(x, n) / (double)n;
        for (int i = 0; i < n; ++i) {
            d[i] = x[i] - mean;
            sq[i] = d[i] * d[i];
        }
        double var = orc_sum_f64(sq, n) / (double)n;
        double mx = x[0], mn = x[0];
        int nan = 0;
        for (int i = 0; i < n; ++i) {
            if (isnan(x[i])) nan = 1;
            if (x[i] > mx) mx = x[i];
            if (x[i] < mn) mn = x[i];
        }
        /* numpy.ma masks a non-finite mean (the domained divide of ma.mean), so
         * every anomaly of ma.var is masked and its sum is 0: std 0 */
        std_o[k] = isfinite(mean) ? sqrt(var) : 0.0;
        mean_o[k] = mean;
        ptp_o[k] = nan ? NAN : (mx - mn);
        fft_o[k] = fftmax(d, n, work, tab);
    }
    free(d); free(sq); free(work);
    }
    free(tab);
}

/* ------------------------------------------------------ medians + scalers */
static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}
static int cmp_f(const void *a, const void *b)
{
    float x = *(const float *)a, y = *(const float *)b;
    return (x > y) - (x < y);
}

/* median of cnt values (no NaN) already sorted, numpy arithmetic in dtype */
static double mid_median_d(const double *s, int cnt)
{
    int idx = cnt / 2;
    if (cnt % 2) return 0.0 + s[idx];
    double t = (0.0 + s[idx - 1]) + s[idx];
    return t / 2.0;
}
static float mid_median_f(const float *s, int cnt)
{
    int idx = cnt / 2;
    if (cnt % 2) return 0.0f + s[idx];
    float t = (0.0f + s[idx - 1]) + s[idx];
    return t / 2.0f;
}

/* One line of a masked f64 diagnostic: out[i] = final scaled value. */
static void scale_line_masked_d(int len, const double *d, const uint8_t *valid, int vstride,
                                int dstride, double thr, double *out, int ostride, double *buf)
{
    const double tiny = DBL_MIN;
    int cnt = 0, nan = 0;
    for (int i = 0; i < len; ++i)
        if (valid[(size_t)i * vstride]) {
            double v = d[(size_t)i * dstride];
            if (isnan(v)) nan = 1;
            buf[cnt++] = v;
        }
    double med = NAN, mad = NAN;
    if (cnt > 0) {
        if (!nan) {
            qsort(buf, (size_t)cnt, sizeof(double), cmp_d);
            med = mid_median_d(buf, cnt);
        }
        int c2 = 0, nan2 = 0;
        for (int i = 0; i < len; ++i)
            if (valid[(size_t)i * vstride]) {
                double r = d[(size_t)i * dstride] - med;
                double a = fabs(r);
                if (isnan(a)) nan2 = 1;
                buf[c2++] = a;
            }
        if (!nan2) {
            qsort(buf, (size_t)c2, sizeof(double), cmp_d);
            mad = mid_median_d(buf, c2);
        }
    }
    for (int i = 0; i < len; ++i) {
        double dv = d[(size_t)i * dstride];
        double v;
        if (!valid[(size_t)i * vstride]) {
            v = 0.0 + fabs(dv);
        } else {
            double r = dv - med;
            double q = r / mad;
            int dom = !isfinite(q) || (fabs(r) * tiny >= fabs(mad));
            if (dom) {
                v = 0.0 + fabs(0.0 + r);
            } else {
                double a = fabs(q);
                double res = a / thr;
                if (!isfinite(res) || a * tiny >= fabs(thr)) v = 0.0 + a;
                else v = res;
            }
        }
        out[(size_t)i * ostride] = v;
    }
}

static void scale_line_masked_f(int len, const float *d, const uint8_t *valid, int vstride,
                                int dstride, double thr, double *out, int ostride, float *buf)
{
    const double tiny = DBL_MIN;
    int cnt = 0, nan = 0;
    for (int i = 0; i < len; ++i)
        if (valid[(size_t)i * vstride]) {
            float v = d[(size_t)i * dstride];
            if (isnan(v)) nan = 1;
            buf[cnt++] = v;
        }
    float med = NAN, mad = NAN;
    if (cnt > 0) {
        if (!nan) {
            qsort(buf, (size_t)cnt, sizeof(float), cmp_f);
            med = mid_median_f(buf, cnt);
        }
        int c2 = 0, nan2 = 0;
        for (int i = 0; i < len; ++i)
            if (valid[(size_t)i * vstride]) {
                float r = d[(size_t)i * dstride] - med;
                float a = fabsf(r);
                if (isnan(a)) nan2 = 1;
                buf[c2++] = a;
            }
        if (!nan2) {
            qsort(buf, (size_t)c2, sizeof(float), cmp_f);
            mad = mid_median_f(buf, c2);
        }
    }
    for (int i = 0; i < len; ++i) {
        float dv = d[(size_t)i * dstride];
        double v;
        if (!valid[(size_t)i * vstride]) {
            v = 0.0 + (double)fabsf(dv);
        } else {
            float r = dv - med;
            float q = r / mad;
            int dom = !isfinite(q) || ((double)fabsf(r) * tiny >= (double)fabsf(mad));
            if (dom) {
                v = 0.0 + (double)fabsf(0.0f + r);
            } else {
                float a = fabsf(q);
                double res = (double)a / thr;
                if (!isfinite(res) || (double)a * tiny >= fabs(thr)) v = 0.0 + (double)a;
                else v = res;
            }
        }
        out[(size_t)i * ostride] = v;
    }
}

static void scale_line_plain(int len, const double *d, int dstride, double thr,
                             double *out, int ostride, double *buf)
{
    int nan = 0;
    for (int i = 0; i < len; ++i) {
        buf[i] = d[(size_t)i * dstride];
        if (isnan(buf[i])) nan = 1;
    }
    double med = NAN, mad = NAN;
    if (!nan) {
        qsort(buf, (size_t)len, sizeof(double), cmp_d);
        med = mid_median_d(buf, len);
    }
    int nan2 = 0;
    for (int i = 0; i < len; ++i) {
        buf[i] = fabs(d[(size_t)i * dstride] - med);
        if (isnan(buf[i])) nan2 = 1;
    }
    if (!nan2) {
        qsort(buf, (size_t)len, sizeof(double), cmp_d);
        mad = mid_median_d(buf, len);
    }
    for (int i = 0; i < len; ++i) {
        double r = d[(size_t)i * dstride] - med;
        double q = r / mad;
        out[(size_t)i * ostride] = fabs(q) / thr;
    }
}

static double nanmax2(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    return a > b ? a : b;
}

static void test_impl(int nsub, int nchan, const uint8_t *valid, const double *std_d, const double *mean_d,
                      const float *ptp_d, const double *ptp64, const double *fft_d, double chanthresh,
                      double subintthresh, double *test);

/* scalers + combine: test (nsub*nchan) from the 4 diagnostics. */
void orc_test(int nsub, int nchan, const uint8_t *valid, const double *std_d,
              const double *mean_d, const float *ptp_d, const double *fft_d,
              double chanthresh, double subintthresh, double *test)
{
    test_impl(nsub, nchan, valid, std_d, mean_d, ptp_d, NULL, fft_d, chanthresh, subintthresh, test);
}

/* the same for f64 data: ptp is f64 and scaled in f64 */
void orc_test_f64(int nsub, int nchan, const uint8_t *valid, const double *std_d,
                  const double *mean_d, const double *ptp_d, const double *fft_d,
                  double chanthresh, double subintthresh, double *test)
{
    test_impl(nsub, nchan, valid, std_d, mean_d, NULL, ptp_d, fft_d, chanthresh, subintthresh, test);
}

static void test_impl(int nsub, int nchan, const uint8_t *valid, const double *std_d, const double *mean_d,
                      const float *ptp_d, const double *ptp64, const double *fft_d, double chanthresh,
                      double subintthresh, double *test)
{
    size_t P = (size_t)nsub * nchan;
    int L = nsub > nchan ? nsub : nchan;
    double *ch = (double *)malloc(sizeof(double) * P);
    double *sb = (double *)malloc(sizeof(double) * P);
    double *S = (double *)malloc(sizeof(double) * 4 * P);
    for (int which = 0; which < 4; ++which) {
#pragma omp parallel
        {
        double *bufd = (double *)malloc(sizeof(double) * (size_t)L);
        float *buff = (float *)malloc(sizeof(float) * (size_t)L);
#pragma omp for schedule(dynamic, 8)
        for (int c = 0; c < nchan; ++c) {
            if (which == 0) scale_line_masked_d(nsub, std_d + c, valid + c, nchan, nchan, chanthresh, ch + c, nchan, bufd);
            if (which == 1) scale_line_masked_d(nsub, mean_d + c, valid + c, nchan, nchan, chanthresh, ch + c, nchan, bufd);
            if (which == 2 && ptp64) scale_line_masked_d(nsub, ptp64 + c, valid + c, nchan, nchan, chanthresh, ch + c, nchan, bufd);
            if (which == 2 && !ptp64) scale_line_masked_f(nsub, ptp_d + c, valid + c, nchan, nchan, chanthresh, ch + c, nchan, buff);
            if (which == 3) scale_line_plain(nsub, fft_d + c, nchan, chanthresh, ch + c, nchan, bufd);
        }
#pragma omp for schedule(dynamic, 1)
        for (int s = 0; s < nsub; ++s) {
            size_t o = (size_t)s * nchan;
            if (which == 0) scale_line_masked_d(nchan, std_d + o, valid + o, 1, 1, subintthresh, sb + o, 1, bufd);
            if (which == 1) scale_line_masked_d(nchan, mean_d + o, valid + o, 1, 1, subintthresh, sb + o, 1, bufd);
            if (which == 2 && ptp64) scale_line_masked_d(nchan, ptp64 + o, valid + o, 1, 1, subintthresh, sb + o, 1, bufd);
            if (which == 2 && !ptp64) scale_line_masked_f(nchan, ptp_d + o, valid + o, 1, 1, subintthresh, sb + o, 1, buff);
            if (which == 3) scale_line_plain(nchan, fft_d + o, 1, subintthresh, sb + o, 1, bufd);
        }
        free(bufd); free(buff);
        }
        for (size_t k = 0; k < P; ++k) S[which * P + k] = nanmax2(ch[k], sb[k]);
    }
    for (size_t k = 0; k < P; ++k) {
        double v[4] = {S[k], S[P + k], S[2 * P + k], S[3 * P + k]};
        if (isnan(v[0]) || isnan(v[1]) || isnan(v[2]) || isnan(v[3])) { test[k] = NAN; continue; }
        qsort(v, 4, sizeof(double), cmp_d);
        test[k] = ((0.0 + v[1]) + v[2]) / 2.0;
    }
    free(ch); free(sb); free(S);
}

/* --------------------------------------------------------- the loop */
typedef struct {
    int32_t nsub, nchan, nbin, max_iter;
    double chanthresh, subintthresh;
    int32_t pr_on;
    double pr_factor;
    int32_t pr_start, pr_end;
    double baseline_duty;
    int32_t fit_mode;   /* 0: exact leastsq (orc_fit_residual), 1: closed form (orc_fit_closed) */
    int32_t data_f64;   /* 1: get_data returns f64 (orc_diagnostics_f64 / orc_test_f64) */
    int32_t dedisp_mode; /* 0: integer shifts; 1: FFT phase rotation by `delay` (orc_rotate) */
    int32_t input_dedispersed; /* 1 (dedisp_mode 1): raw is stored dedispersed, its dedisperse a no-op */
    int32_t delay_per_profile; /* 1 (dedisp_mode 1): `delay` is [nsub*nchan] */
} orc_params;

/* One full clean loop (iterative_cleaner.py:83-146).
 * raw: pscrunched cube (nsub,nchan,nbin) dispersed frame; w0 weights.
 * Outputs: test (P), weights (P), loops, changed[max_iter], nzero[max_iter];
 * optional (may be NULL): R_last (P*nbin, dispersed frame, unweighted),
 * T_all (max_iter*nbin), amp_last/info_last (P),
 * diag_last: std, mean (P f64), ptp (P, f64 storage: f32 values unless data_f64), fft (P f64).
 * dedisp_mode 1: `delay` [nchan] f64 bins ([nsub*nchan] with delay_per_profile);
 * every dedisperse / dededisperse of the reference is the FFT phase rotation
 * (archive.py with dm_delay), `shift` unused; with input_dedispersed the raw
 * cube is stored dedispersed, so only the dededisperse (:104) rotates. */
int orc_clean_loop(const orc_params *pp, const float *raw, const float *w0, const int32_t *shift,
                   double *test, float *weights, int32_t *loops_out, int32_t *changed,
                   int32_t *nzero, float *R_last, float *T_all, double *amp_last,
                   int32_t *info_last, double *std_l, double *mean_l, double *ptp_l, double *fft_l,
                   const double *delay)
{
    const int nsub = pp->nsub, nchan = pp->nchan, n = pp->nbin;
    const size_t P = (size_t)nsub * nchan, N = P * (size_t)n;
    float *D = (float *)malloc(sizeof(float) * N);
    float *Rd = (float *)malloc(sizeof(float) * N);
    float *X = (float *)malloc(sizeof(float) * N);
    float *T = (float *)malloc(sizeof(float) * (size_t)n);
    double *amp = (double *)malloc(sizeof(double) * P);
    int32_t *info = (int32_t *)malloc(sizeof(int32_t) * P);
    double *sd = (double *)malloc(sizeof(double) * P), *mn = (double *)malloc(sizeof(double) * P);
    float *pt = (float *)malloc(sizeof(float) * P);
    double *pt64 = (double *)malloc(sizeof(double) * P);
    double *X64 = pp->data_f64 ? (double *)malloc(sizeof(double) * N) : NULL;
    double *ff = (double *)malloc(sizeof(double) * P);
    uint8_t *valid = (uint8_t *)malloc(P);
    int maxit = pp->max_iter;
    float *hist = (float *)malloc(sizeof(float) * P * (size_t)(maxit + 1));
    float *Wcur = (float *)malloc(sizeof(float) * P);
    for (size_t k = 0; k < P; ++k) valid[k] = (w0[k] != 0.0f);
    memcpy(hist, w0, sizeof(float) * P);
    memcpy(Wcur, w0, sizeof(float) * P);
    int nhist = 1;
    const int fftded = pp->dedisp_mode == 1;
    const int ppd = fftded && pp->delay_per_profile, ided = fftded && pp->input_dedispersed;
    int32_t *zsh = fftded ? (int32_t *)calloc((size_t)nchan, sizeof(int32_t)) : NULL;
    float *dr = NULL, *Tc = NULL, *bs = NULL, *Rx = NULL;
    if (fftded) {
        /* remove_baseline reads the dedispersed view rot(raw); the data it
         * leaves, f32(raw - base), is then rotated (dedisperse) */
        dr = (float *)malloc(sizeof(float) * N);
        Tc = (float *)malloc(sizeof(float) * N);
        Rx = (float *)malloc(sizeof(float) * N);
        bs = (float *)malloc(sizeof(float) * P);
        orc_rotate_ex(nsub, nchan, n, raw, NULL, delay, ppd, ided, 1, dr);
        orc_baseline(nsub, nchan, n, dr, w0, zsh, pp->baseline_duty, bs, NULL);
        orc_rotate_ex(nsub, nchan, n, raw, bs, delay, ppd, ided, 1, D);
    } else {
        orc_fit_cube(nsub, nchan, n, raw, w0, shift, pp->baseline_duty, D);
    }
    int x = 0, loops = -1;
    while (x < maxit) {
        x += 1;
        if (fftded) {
            orc_baseline(nsub, nchan, n, dr, Wcur, zsh, pp->baseline_duty, bs, NULL);
            orc_rotate_ex(nsub, nchan, n, raw, bs, delay, ppd, ided, 1, Tc);
            for (size_t k = 0; k < P; ++k) bs[k] = 0.0f;
            orc_scrunch(nsub, nchan, n, Tc, Wcur, zsh, bs, T);
        } else {
            orc_template(nsub, nchan, n, raw, Wcur, shift, pp->baseline_duty, T);
        }
        if (T_all) memcpy(T_all + (size_t)(x - 1) * n, T, sizeof(float) * (size_t)n);
        if (pp->fit_mode == 1)
            orc_fit_closed((int)P, n, T, D, pp->pr_on, pp->pr_factor, pp->pr_start, pp->pr_end, amp, info, Rd,
                           fftded ? NULL : shift, nchan);
        else
            orc_fit_residual((int)P, n, T, D, pp->pr_on, pp->pr_factor, pp->pr_start, pp->pr_end, amp, info, Rd);
        /* dededisperse + apply_weights */
        if (fftded) orc_rotate_ex(nsub, nchan, n, Rd, NULL, delay, ppd, 0, -1, Rx);
#pragma omp parallel for schedule(static)
        for (int s = 0; s < nsub; ++s)
            for (int c = 0; c < nchan; ++c) {
                size_t k = (size_t)s * nchan + c;
                const float *r = fftded ? Rx + k * n : Rd + k * n;
                float *o = X + k * n;
                float w = w0[k];
                int sh = fftded ? 0 : shift[c];
                for (int j = 0; j < n; ++j) {
                    int i = j - sh;
                    if (i < 0) i += n;
                    if (X64) X64[k * n + j] = (double)r[i] * (double)w;
                    else o[j] = r[i] * w;
                }
            }
        if (X64) {
            orc_diagnostics_f64((int)P, n, X64, valid, sd, mn, pt64, ff);
            orc_test_f64(nsub, nchan, valid, sd, mn, pt64, ff, pp->chanthresh, pp->subintthresh, test);
        } else {
            orc_diagnostics((int)P, n, X, valid, sd, mn, pt, ff);
            orc_test(nsub, nchan, valid, sd, mn, pt, ff, pp->chanthresh, pp->subintthresh, test);
            for (size_t k = 0; k < P; ++k) pt64[k] = (double)pt[k];
        }
        int ndiff = 0, nz = 0;
        for (size_t k = 0; k < P; ++k) {
            float w = (test[k] >= 1.0) ? 0.0f : w0[k];
            if (w != hist[(size_t)(nhist - 1) * P + k]) ++ndiff;
            if (w == 0.0f) ++nz;
            Wcur[k] = w;
        }
        changed[x - 1] = ndiff;
        nzero[x - 1] = nz;
        for (int h = 0; h < nhist; ++h) {
            int eq = 1;
            for (size_t k = 0; k < P && eq; ++k) if (!(Wcur[k] == hist[(size_t)h * P + k])) eq = 0;
            if (eq) { loops = x; x = 1000000; }
        }
        memcpy(hist + (size_t)nhist * P, Wcur, sizeof(float) * P);
        ++nhist;
    }
    if (x == maxit) loops = maxit;
    memcpy(weights, Wcur, sizeof(float) * P);
    if (R_last) {
        /* dededispersed residual, unweighted (ic.py:104-108) */
        for (int s = 0; s < nsub; ++s)
            for (int c = 0; c < nchan; ++c) {
                size_t k = (size_t)s * nchan + c;
                for (int j = 0; j < n; ++j) {
                    int i = j - (fftded ? 0 : shift[c]);
                    if (i < 0) i += n;
                    R_last[k * n + j] = fftded ? Rx[k * n + i] : Rd[k * n + i];
                }
            }
    }
    if (amp_last) memcpy(amp_last, amp, sizeof(double) * P);
    if (info_last) memcpy(info_last, info, sizeof(int32_t) * P);
    if (std_l) memcpy(std_l, sd, sizeof(double) * P);
    if (mean_l) memcpy(mean_l, mn, sizeof(double) * P);
    if (ptp_l) memcpy(ptp_l, pt64, sizeof(double) * P);
    if (fft_l) memcpy(fft_l, ff, sizeof(double) * P);
    *loops_out = loops;
    free(D); free(Rd); free(X); free(T); free(amp); free(info); free(sd); free(mn);
    free(pt); free(pt64); free(X64); free(ff); free(valid); free(hist); free(Wcur);
    free(zsh); free(dr); free(Tc); free(bs); free(Rx);
    return 0;
}
