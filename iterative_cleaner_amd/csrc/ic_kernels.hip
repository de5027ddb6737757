// ic_kernels.hip — gfx950 kernels of the surgical-cleaning loop
// (/root/reference/iterative_cleaner.py:83-146).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see Makefile).
// -ffp-contract=off is load-bearing: every f64/f32 operation below must be an
// individually rounded IEEE op in the order written, so that results equal
// numpy / scipy (MINPACK) bit-for-bit.  Explicit fma() is never used on an
// exact path.
//
// Kernels (per cleaning iteration, in launch order):
//   k_chan_partials  canonical-order channel sums (archive.py chan_sum) of
//                    W*ded (baseline total) or W*f32(ded-base) (fscrunch)
//   k_window         per-subint off-pulse window: first argmin of circular
//                    window sums (archive.py window_argmin)
//   k_base           per-profile window mean -> f32 baseline
//   k_fscrunch       combine super-block partials -> F[s][i], wf[s]
//   k_tscrunch       weighted mean over subints, *10000 -> T (ic.py:94)
//   k_fit            exact scipy leastsq(a*T-p, [1.0]) per profile (ic.py:278)
//   k_diag           residual (ic.py:279-288), f32 store (:272), dededisperse
//                    (:104), apply_weights (:296), diagnostics (:206-217)
//   k_linestats      per channel / subint median & MAD (ic.py:229-256)
//   k_combine        scale, max, median-of-4, threshold, new weights,
//                    convergence counters (ic.py:221-225, :303-305, :127-141)
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "ic_internal.h"

namespace icgpu {

__device__ constexpr double kRdwarf = 3.834e-20;
__device__ constexpr double kRgiant = 1.304e19;

// ============================================================ template stage

// part[s][sb][i] = sum_{c in sb, ascending} W[s,c] * x[s,c,i]   (f64, from 0.0)
// x = ded (base == nullptr) or f32(ded - base[s,c]);  wpart[s][sb] = sum W.
// One lane per bin; lanes of a wave read 64 consecutive (rotated) bins.
__global__ __launch_bounds__(256) void k_chan_partials(
    const float *__restrict__ raw, const float *__restrict__ W, const int32_t *__restrict__ shift,
    const float *__restrict__ base, int nsub, int nchan, int nbin, int nsb,
    double *__restrict__ part, double *__restrict__ wpart)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int sb = blockIdx.y;
    const int s = blockIdx.z;
    const int c0 = sb * kSuperBlock;
    const int c1 = min(c0 + kSuperBlock, nchan);
    if (i < nbin) {
        double acc = 0.0;
        const size_t krow = (size_t)s * nchan;
#pragma unroll 4
        for (int c = c0; c < c1; ++c) {
            const size_t k = krow + c;
            const double w = (double)W[k];
            int j = i + shift[c];
            if (j >= nbin) j -= nbin;
            float x = raw[k * nbin + j];
            if (base) x = x - base[k];
            const double t = w * (double)x;
            acc = acc + t;
        }
        part[((size_t)s * nsb + sb) * nbin + i] = acc;
    }
    if (wpart && blockIdx.x == 0 && threadIdx.x == 0) {
        double a = 0.0;
        for (int c = c0; c < c1; ++c) a = a + (double)W[(size_t)s * nchan + c];
        wpart[(size_t)s * nsb + sb] = a;
    }
}

// numpy argmin combine: first NaN wins; otherwise smaller value, then lower index.
__device__ __forceinline__ bool argmin_better(double va, int ia, double vb, int ib)
{
    const bool na = isnan(va), nb = isnan(vb);
    if (na || nb) {
        if (na && nb) return ia < ib;
        return na;
    }
    if (va < vb) return true;
    if (vb < va) return false;
    return ia < ib;
}

// One block per subint: tot[i] = sum_sb part; m[j] = sum_{k<width} tot[(j+k)%n];
// win[s] = first argmin.
__global__ __launch_bounds__(256) void k_window(const double *__restrict__ part, int nsb, int nbin,
                                                int width, int32_t *__restrict__ win)
{
    extern __shared__ double sh[];
    double *tot = sh;                       // nbin
    double *bv = sh + nbin;                 // 256
    int *bi = (int *)(bv + 256);            // 256
    const int s = blockIdx.x;
    for (int i = threadIdx.x; i < nbin; i += blockDim.x) {
        double t = 0.0;
        for (int sb = 0; sb < nsb; ++sb) t = t + part[((size_t)s * nsb + sb) * nbin + i];
        tot[i] = t;
    }
    __syncthreads();
    double best = 0.0;
    int besti = -1;
    for (int j = threadIdx.x; j < nbin; j += blockDim.x) {
        double m = 0.0;
        int q = j;
        for (int k = 0; k < width; ++k) {
            m = m + tot[q];
            if (++q == nbin) q = 0;
        }
        if (besti < 0 || argmin_better(m, j, best, besti)) {
            best = m;
            besti = j;
        }
    }
    bv[threadIdx.x] = best;
    bi[threadIdx.x] = besti;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            const int o = threadIdx.x + off;
            if (bi[o] >= 0 && (bi[threadIdx.x] < 0 ||
                               argmin_better(bv[o], bi[o], bv[threadIdx.x], bi[threadIdx.x]))) {
                bv[threadIdx.x] = bv[o];
                bi[threadIdx.x] = bi[o];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) win[s] = bi[0];
}

// base[k] = f32( (sum_{k<width} f64(ded[(win+k)%n])) / width ), one lane per profile.
__global__ __launch_bounds__(256) void k_base(const float *__restrict__ raw, const int32_t *__restrict__ shift,
                                              const int32_t *__restrict__ win, int nsub, int nchan,
                                              int nbin, int width, float *__restrict__ base)
{
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= (size_t)nsub * nchan) return;
    const int s = (int)(k / nchan);
    const int c = (int)(k % nchan);
    int q = win[s] + shift[c];
    if (q >= nbin) q -= nbin;
    const float *prof = raw + k * nbin;
    double acc = 0.0;
    for (int t = 0; t < width; ++t) {
        acc = acc + (double)prof[q];
        if (++q == nbin) q = 0;
    }
    base[k] = (float)(acc / (double)width);
}

// D[k][i] = f32(ded[k][i] - base0[k])  (fit cube, dedispersed frame); grid-stride over N
__global__ __launch_bounds__(256) void k_fitcube(const float *__restrict__ raw, const int32_t *__restrict__ shift,
                                                 const float *__restrict__ base, int nsub, int nchan,
                                                 int nbin, float *__restrict__ D)
{
    const size_t N = (size_t)nsub * nchan * nbin;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (size_t)gridDim.x * blockDim.x) {
        const size_t k = e / nbin;
        const int i = (int)(e - k * nbin);
        const int c = (int)(k % nchan);
        int j = i + shift[c];
        if (j >= nbin) j -= nbin;
        D[e] = raw[k * nbin + j] - base[k];
    }
}

// F[s][i] = f32(num/wsum) (0 if wsum == 0); wf[s] = f32(wsum)
__global__ __launch_bounds__(256) void k_fscrunch(const double *__restrict__ part, const double *__restrict__ wpart,
                                                  int nsb, int nbin, float *__restrict__ F,
                                                  float *__restrict__ wf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (i >= nbin) return;
    double num = 0.0, wsum = 0.0;
    for (int sb = 0; sb < nsb; ++sb) {
        num = num + part[((size_t)s * nsb + sb) * nbin + i];
        wsum = wsum + wpart[(size_t)s * nsb + sb];
    }
    F[(size_t)s * nbin + i] = (wsum != 0.0) ? (float)(num / wsum) : 0.0f;
    if (i == 0) wf[s] = (float)wsum;
}

// T[i] = f32( f32(sum_s wf*F / sum_s wf) * 10000 )
__global__ __launch_bounds__(256) void k_tscrunch(const float *__restrict__ F, const float *__restrict__ wf,
                                                  int nsub, int nbin, float *__restrict__ T,
                                                  double *__restrict__ T64)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nbin) return;
    double wt = 0.0, num = 0.0;
    for (int s = 0; s < nsub; ++s) {
        const double w = (double)wf[s];
        wt = wt + w;
        const double t = w * (double)F[(size_t)s * nbin + i];
        num = num + t;
    }
    const float t = (wt != 0.0) ? (float)(num / wt) : 0.0f;
    const float tt = t * 10000.0f;
    T[i] = tt;
    T64[i] = (double)tt;
}

// ============================================================ exact lmdif

struct Enorm {
    double s1, s2, s3, x1max, x3max;
};

__device__ __forceinline__ void en_zero(Enorm &e) { e.s1 = e.s2 = e.s3 = e.x1max = e.x3max = 0.0; }

// MINPACK enorm, one component (rare branches kept exactly).
__device__ __forceinline__ void en_add(Enorm &e, double v, double agiant)
{
    const double xabs = fabs(v);
    if (xabs > kRdwarf && xabs < agiant) {
        e.s2 += xabs * xabs;
    } else if (xabs <= kRdwarf) {
        if (xabs > e.x3max) {
            const double t = e.x3max / xabs;
            e.s3 = 1.0 + e.s3 * (t * t);
            e.x3max = xabs;
        } else if (xabs != 0.0) {
            const double t = xabs / e.x3max;
            e.s3 += t * t;
        }
    } else {
        if (xabs > e.x1max) {
            const double t = e.x1max / xabs;
            e.s1 = 1.0 + e.s1 * (t * t);
            e.x1max = xabs;
        } else {
            const double t = xabs / e.x1max;
            e.s1 += t * t;
        }
    }
}

__device__ __forceinline__ double en_fin(const Enorm &e)
{
    if (e.s1 != 0.0) return e.x1max * sqrt(e.s1 + (e.s2 / e.x1max) / e.x1max);
    if (e.s2 != 0.0) {
        if (e.s2 >= e.x3max) return sqrt(e.s2 * (1.0 + (e.x3max / e.s2) * (e.x3max * e.s3)));
        return sqrt(e.x3max * ((e.s2 / e.x3max) + (e.x3max * e.s3)));
    }
    return e.x3max * sqrt(e.s3);
}

__device__ __forceinline__ double enorm1(double v)
{
    Enorm e;
    en_zero(e);
    en_add(e, v, kRgiant);
    return en_fin(e);
}

__device__ __forceinline__ double dmax_(double a, double b) { return a >= b ? a : b; }
__device__ __forceinline__ double dmin_(double a, double b) { return a <= b ? a : b; }

// MINPACK qrsolv, n = 1
__device__ double qrsolv1(double r, double w, double qtb, double *sdiag)
{
    double rr = r, wa = qtb;
    if (w != 0.0) {
        const double sd = w;
        const double qtbpj = 0.0;
        double cs, sn;
        if (fabs(rr) >= fabs(sd)) {
            const double tn = sd / rr;
            cs = 0.5 / sqrt(0.25 + 0.25 * (tn * tn));
            sn = cs * tn;
        } else {
            const double ct = rr / sd;
            sn = 0.5 / sqrt(0.25 + 0.25 * (ct * ct));
            cs = sn * ct;
        }
        rr = cs * rr + sn * sd;
        const double t1 = cs * wa;
        const double t2 = sn * qtbpj;
        wa = t1 + t2;
    }
    *sdiag = rr;
    if (rr == 0.0) return 0.0;
    const double sum = 0.0;
    return (wa - sum) / rr;
}

// MINPACK lmpar, n = 1
__device__ double lmpar1(double r, double diag, double qtb, double delta, double *par_io)
{
    const double p1 = 0.1, p001 = 0.001, dwarf = DBL_MIN;
    double par = *par_io;
    const int nsing = (r == 0.0) ? 0 : 1;
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
            const double sum = 0.0;
            t = (t - sum) / r;
            const double temp = enorm1(t);
            parl = ((fp / delta) / temp) / temp;
        }
        double sum = 0.0;
        sum += r * qtb;
        const double g = sum / diag;
        const double gnorm = enorm1(g);
        double paru = gnorm / delta;
        if (paru == 0.0) paru = dwarf / dmin_(delta, p1);
        par = dmax_(par, parl);
        par = dmin_(par, paru);
        if (par == 0.0) par = gnorm / dxnorm;
        for (;;) {
            ++iter;
            if (par == 0.0) par = dmax_(dwarf, p001 * paru);
            double temp = sqrt(par);
            const double w = temp * diag;
            double sdiag;
            x = qrsolv1(r, w, qtb, &sdiag);
            wa2 = diag * x;
            dxnorm = enorm1(wa2);
            temp = fp;
            fp = dxnorm - delta;
            if (fabs(fp) <= p1 * delta || (parl == 0.0 && fp <= temp && temp < 0.0) || iter == 10) break;
            double t = diag * (wa2 / dxnorm);
            t = t / sdiag;
            const double tn = enorm1(t);
            const double parc = ((fp / delta) / tn) / tn;
            if (fp > 0.0) parl = dmax_(parl, par);
            if (fp < 0.0) paru = dmin_(paru, par);
            par = dmax_(parl, par + parc);
        }
    }
    if (iter == 0) par = 0.0;
    *par_io = par;
    return x;
}

enum FitState { ST_A0 = 0, ST_A2 = 1, ST_B = 2, ST_DONE = 3 };

// Per-lane lmdif state (scipy leastsq, n = 1, m = nbin).
struct LmState {
    double x, fnorm, par, delta, diag, xnorm;
    double acnorm, J0, f0;       // Jacobian norm, J[0], fvec[0] at x
    double acn2, J02, f02;       // the same at x2 (speculative Jacobian)
    double aj, r, Jn0, qtf;
    double gnorm, x2, pnorm, wa1;
    int iter, nfev, info;
};

__device__ int lm_start_inner(LmState &L)
{
    const double step = lmpar1(L.r, L.diag, L.qtf, L.delta, &L.par);
    L.wa1 = -step;
    L.x2 = L.x + L.wa1;
    L.pnorm = enorm1(L.diag * L.wa1);
    if (L.iter == 1) L.delta = dmin_(L.delta, L.pnorm);
    return ST_A2;
}

__device__ int lm_after_qtf(LmState &L)
{
    L.gnorm = 0.0;
    if (L.fnorm != 0.0 && L.acnorm != 0.0) {
        double sum = 0.0;
        sum += L.r * (L.qtf / L.fnorm);
        L.gnorm = dmax_(L.gnorm, fabs(sum / L.acnorm));
    }
    if (L.gnorm <= 0.0) {  // gtol = 0
        L.info = 4;
        return ST_DONE;
    }
    L.diag = dmax_(L.diag, L.acnorm);
    return lm_start_inner(L);
}

// start of an outer iteration: fdjac2 done (acnorm, J0, f0 at x); qrfac + qtf setup
__device__ int lm_outer(LmState &L)
{
    L.nfev += 1;
    double ajnorm = L.acnorm;
    L.Jn0 = L.J0;
    if (ajnorm != 0.0) {
        if (L.J0 < 0.0) ajnorm = -ajnorm;
        L.Jn0 = L.J0 / ajnorm;
        L.Jn0 = L.Jn0 + 1.0;
    }
    L.aj = ajnorm;
    L.r = -ajnorm;
    if (L.iter == 1) {
        L.diag = L.acnorm;
        if (L.diag == 0.0) L.diag = 1.0;
        L.xnorm = enorm1(L.diag * L.x);
        L.delta = 100.0 * L.xnorm;
        if (L.delta == 0.0) L.delta = 100.0;
    }
    if (L.Jn0 != 0.0) return ST_B;  // needs sum_i Jn_i * fvec_i
    L.qtf = L.f0;
    return lm_after_qtf(L);
}

__device__ int lm_after_b(LmState &L, double sum)
{
    const double t = -sum / L.Jn0;
    L.qtf = L.f0 + L.Jn0 * t;
    return lm_after_qtf(L);
}

__device__ int lm_after_a2(LmState &L, double fnorm1)
{
    const double ftol = 1.49012e-8, xtol = 1.49012e-8, epsmch = DBL_EPSILON;
    L.nfev += 1;
    double actred = -1.0;
    if (0.1 * fnorm1 < L.fnorm) {
        const double t = fnorm1 / L.fnorm;
        actred = 1.0 - t * t;
    }
    double w3 = 0.0;
    w3 += L.r * L.wa1;
    const double temp1 = enorm1(w3) / L.fnorm;
    const double temp2 = (sqrt(L.par) * L.pnorm) / L.fnorm;
    const double prered = temp1 * temp1 + temp2 * temp2 / 0.5;
    const double dirder = -(temp1 * temp1 + temp2 * temp2);
    double ratio = 0.0;
    if (prered != 0.0) ratio = actred / prered;
    if (ratio <= 0.25) {
        double tt = 0.0;
        if (actred >= 0.0) tt = 0.5;
        if (actred < 0.0) tt = 0.5 * dirder / (dirder + 0.5 * actred);
        if (0.1 * fnorm1 >= L.fnorm || tt < 0.1) tt = 0.1;
        L.delta = tt * dmin_(L.delta, L.pnorm / 0.1);
        L.par = L.par / tt;
    } else if (L.par == 0.0 || ratio >= 0.75) {
        L.delta = L.pnorm / 0.5;
        L.par = 0.5 * L.par;
    }
    if (ratio >= 1e-4) {
        L.x = L.x2;
        L.xnorm = enorm1(L.diag * L.x);
        L.fnorm = fnorm1;
        L.iter += 1;
        L.acnorm = L.acn2;
        L.J0 = L.J02;
        L.f0 = L.f02;
    }
    int info = 0;
    if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0) info = 1;
    if (L.delta <= xtol * L.xnorm) info = 2;
    if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0 && info == 2) info = 3;
    if (info == 0) {
        if (L.nfev >= 400) info = 5;
        if (fabs(actred) <= epsmch && prered <= epsmch && 0.5 * ratio <= 1.0) info = 6;
        if (L.delta <= epsmch * L.xnorm) info = 7;
        if (L.gnorm <= epsmch) info = 8;
    }
    if (info != 0) {
        L.info = info;
        return ST_DONE;
    }
    if (ratio < 1e-4) return lm_start_inner(L);
    return lm_outer(L);
}

#define FIT_TB 64

// One lane per profile, 64 profiles per block (one wave).  Each lane runs the
// MINPACK lmdif state machine; the data passes it needs (A: f(xa) norm +
// Jacobian norm at xa; B: sum_i Jn_i*fvec_i) are served by wave-wide sweeps
// over the profiles' samples, staged through an LDS tile (transposed so
// lane l reads column l conflict-free).
__global__ __launch_bounds__(64) void k_fit(const float *__restrict__ D, const double *__restrict__ T64,
                                            long P, int nbin, double *__restrict__ amp_o,
                                            int32_t *__restrict__ info_o)
{
    __shared__ float tile[FIT_TB][65];
    const int lane = threadIdx.x;
    const long k0 = (long)blockIdx.x * 64;
    const long k = k0 + lane;
    const bool live = k < P;
    const double agiant = kRgiant / (double)nbin;
    const double eps = sqrt(DBL_EPSILON);  // sqrt(max(epsfcn, epsmch))

    LmState L;
    L.x = 1.0; L.fnorm = 0.0; L.par = 0.0; L.delta = 0.0; L.diag = 0.0; L.xnorm = 0.0;
    L.acnorm = 0.0; L.J0 = 0.0; L.f0 = 0.0; L.acn2 = 0.0; L.J02 = 0.0; L.f02 = 0.0;
    L.aj = 0.0; L.r = 0.0; L.Jn0 = 0.0; L.qtf = 0.0; L.gnorm = 0.0; L.x2 = 0.0; L.pnorm = 0.0;
    L.wa1 = 0.0; L.iter = 1; L.nfev = 0; L.info = 0;
    int st = live ? ST_A0 : ST_DONE;

    for (;;) {
        const bool reqA = (st == ST_A0) || (st == ST_A2);
        const bool reqB = (st == ST_B);
        const bool anyA = __any(reqA);
        const bool anyB = __any(reqB);
        if (!anyA && !anyB) break;
        const double xa = (st == ST_A0) ? L.x : L.x2;
        double ha = eps * fabs(xa);
        if (ha == 0.0) ha = eps;
        const double xha = xa + ha;
        double hb = eps * fabs(L.x);
        if (hb == 0.0) hb = eps;
        const double xhb = L.x + hb;
        const double xb = L.x;
        const double ajb = L.aj;
        Enorm eF, eJ;
        en_zero(eF);
        en_zero(eJ);
        double fa0 = 0.0, Ja0 = 0.0, sum = 0.0;
        for (int b0 = 0; b0 < nbin; b0 += FIT_TB) {
            const int tb = min(FIT_TB, nbin - b0);
            __syncthreads();
            for (int m = 0; m < 64; ++m) {
                const long kk = k0 + m;
                float v = 0.0f;
                if (lane < tb && kk < P) v = D[kk * nbin + b0 + lane];
                tile[lane][m] = v;
            }
            __syncthreads();
            for (int ii = 0; ii < tb; ++ii) {
                const int i = b0 + ii;
                const double t = T64[i];
                const double pv = (double)tile[ii][lane];
                if (anyA && reqA) {
                    const double u = xa * t;
                    const double f = u - pv;
                    en_add(eF, f, agiant);
                    const double uh = xha * t;
                    const double wa = uh - pv;
                    const double d = wa - f;
                    const double J = d / ha;
                    en_add(eJ, J, agiant);
                    if (i == 0) {
                        fa0 = f;
                        Ja0 = J;
                    }
                }
                if (anyB && reqB) {
                    const double u = xb * t;
                    const double f = u - pv;
                    const double uh = xhb * t;
                    const double wa = uh - pv;
                    const double d = wa - f;
                    const double J = d / hb;
                    double Jn = J / ajb;
                    if (i == 0) Jn = Jn + 1.0;
                    const double pr = Jn * f;
                    sum = sum + pr;
                }
            }
        }
        if (st == ST_A0) {
            L.fnorm = en_fin(eF);
            L.nfev = 1;
            L.acnorm = en_fin(eJ);
            L.f0 = fa0;
            L.J0 = Ja0;
            st = lm_outer(L);
        } else if (st == ST_A2) {
            L.acn2 = en_fin(eJ);
            L.f02 = fa0;
            L.J02 = Ja0;
            st = lm_after_a2(L, en_fin(eF));
        } else if (st == ST_B) {
            st = lm_after_b(L, sum);
        }
    }
    if (live) {
        amp_o[k] = L.x;
        info_o[k] = L.info;
    }
}

// ============================================================ diagnostics

// numpy pairwise sum of n values produced by get(i), in dtype Tp (one wave).
// scratch: >= 8*nleaf + nleaf + nops slots of Tp in LDS.
template <typename Tp, typename Get>
__device__ Tp wave_pairwise(const PwPlan &pl, Get get, Tp *scratch, int lane)
{
    const int nl = pl.nleaf;
    Tp *acc = scratch;             // [nl*8]
    Tp *slot = scratch + nl * 8;   // [nl + nops]
    for (int task = lane; task < nl * 8; task += 64) {
        const int Lf = task >> 3, j = task & 7;
        const int st = pl.leaf_start[Lf], len = pl.leaf_len[Lf];
        if (len < 8) {
            if (j == 0) {
                Tp res = (Tp)0;
                for (int q = 0; q < len; ++q) res = res + get(st + q);
                acc[task] = res;
            }
            continue;
        }
        const int main = len - len % 8;
        Tp r = get(st + j);
        for (int q = 8; q < main; q += 8) r = r + get(st + q + j);
        acc[task] = r;
    }
    __syncthreads();
    for (int Lf = lane; Lf < nl; Lf += 64) {
        const int st = pl.leaf_start[Lf], len = pl.leaf_len[Lf];
        const Tp *r = acc + Lf * 8;
        Tp res;
        if (len < 8) {
            res = r[0];
        } else {
            const Tp a01 = r[0] + r[1], a23 = r[2] + r[3], a45 = r[4] + r[5], a67 = r[6] + r[7];
            const Tp lo = a01 + a23, hi = a45 + a67;
            res = lo + hi;
            for (int q = len - len % 8; q < len; ++q) res = res + get(st + q);
        }
        slot[Lf] = res;
    }
    __syncthreads();
    Tp out = (Tp)0;
    if (lane == 0) {
        for (int o = 0; o < pl.nops; ++o) slot[nl + o] = slot[pl.op_a[o]] + slot[pl.op_b[o]];
        out = (Tp)0 + slot[pl.root];
        acc[0] = out;
    }
    __syncthreads();
    out = acc[0];
    __syncthreads();
    return out;
}

// One wave per profile.  LDS: X f32 [nbin] | complex f64 work [nbin/2 or nbin] |
// pairwise scratch.  Computes the f32 residual (iterative_cleaner.py:279-288,
// :272), dededisperses it (:104), applies the ORIGINAL weight (:296) and
// the four diagnostics (:206-217) with numpy.ma data conventions.
__global__ __launch_bounds__(64) void k_diag(
    const float *__restrict__ D, const double *__restrict__ T64, const double *__restrict__ amp,
    const int32_t *__restrict__ info, const float *__restrict__ w0, const int32_t *__restrict__ shift,
    const double2 *__restrict__ tw, const PwPlan *__restrict__ plan_g, int nsub, int nchan, int nbin,
    int pr_on, double pr_factor, int pr_start, int pr_end, double *__restrict__ std_o,
    double *__restrict__ mean_o, float *__restrict__ ptp_o, double *__restrict__ fft_o)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ PwPlan pl;
    const int n = nbin;
    const int lane = threadIdx.x;
    const size_t k = blockIdx.x;
    const int c = (int)(k % nchan);
    // plan -> LDS
    {
        const int32_t *src = (const int32_t *)plan_g;
        int32_t *dst = (int32_t *)&pl;
        for (int q = lane; q < (int)(sizeof(PwPlan) / 4); q += 64) dst[q] = src[q];
    }
    const bool pow2 = (n & (n - 1)) == 0 && n >= 4;
    double2 *cw = (double2 *)smem;                                  // n/2 (pow2) or unused
    float *X = (float *)(smem + (size_t)(pow2 ? n / 2 : 1) * 16);     // n
    const size_t xoff = (size_t)(pow2 ? n / 2 : 1) * 16 + (((size_t)n * 4 + 15) & ~(size_t)15);
    double *scr = (double *)(smem + xoff);

    const double x = amp[k];
    const int stt = info[k];
    const bool ok = stt >= 1 && stt <= 4;
    const float w = w0[k];
    const bool valid = (w != 0.0f);
    const int sh = shift[c];
    const float *p = D + k * (size_t)n;
    // residual -> X (dispersed frame): X[j] = f32(f32(r[i]) * w), i = (j - sh) mod n
    for (int i = lane; i < n; i += 64) {
        float R = 0.0f;
        if (ok) {
            const double u = x * T64[i];
            double e = u - (double)p[i];
            if (pr_on && i >= pr_start && i < pr_end) e = e * pr_factor;
            R = (float)e;
        }
        int j = i + sh;
        if (j >= n) j -= n;
        X[j] = R * w;
    }
    __syncthreads();
    double mean = 0.0, var = 0.0;
    float ptp = 1e20f;
    double sd = 0.0;
    if (valid) {
        const float s32 = wave_pairwise<float>(pl, [&](int q) { return X[q]; }, (float *)scr, lane);
        mean = (double)s32 / (double)n;
        const double mu = mean;
        const double ss = wave_pairwise<double>(
            pl,
            [&](int q) {
                const double d = (double)X[q] - mu;
                return d * d;
            },
            scr, lane);
        var = ss / (double)n;
        sd = sqrt(var);
        // ptp (NaN-propagating like ndarray.max/min)
        float mx = -INFINITY, mn = INFINITY;
        int nan = 0;
        for (int q = lane; q < n; q += 64) {
            const float v = X[q];
            if (isnan(v)) nan = 1;
            mx = fmaxf(mx, v);
            mn = fminf(mn, v);
        }
        for (int off = 32; off > 0; off >>= 1) {
            mx = fmaxf(mx, __shfl_xor(mx, off));
            mn = fminf(mn, __shfl_xor(mn, off));
            nan |= __shfl_xor(nan, off);
        }
        ptp = nan ? NAN : (mx - mn);
    }
    // fftmax: max_k |rfft(v)_k|, v = f64(X) - mean (valid) or f64(X) (invalid)
    const double mu = valid ? mean : 0.0;
    double best = 0.0;
    int nanf = 0;
    if (pow2) {
        const int m = n / 2;
        int lg = 0;
        while ((1 << lg) < m) ++lg;
        // z_j = v_{2j} + i v_{2j+1}, bit-reversed into cw
        for (int j = lane; j < m; j += 64) {
            const int rv = lg ? (int)(__builtin_bitreverse32((unsigned)j) >> (32 - lg)) : 0;
            const double re = valid ? (double)X[2 * j] - mu : (double)X[2 * j];
            const double im = valid ? (double)X[2 * j + 1] - mu : (double)X[2 * j + 1];
            cw[rv] = make_double2(re, im);
        }
        __syncthreads();
        for (int len = 2; len <= m; len <<= 1) {
            const int half = len >> 1;
            const int tstep = (n / len);  // twiddle exp(-2 pi i k/len) = tw[k * n/len]
            for (int b = lane; b < m / 2; b += 64) {
                const int grp = b / half, kk = b % half;
                const int i0 = grp * len + kk, i1 = i0 + half;
                const double2 wv = tw[kk * tstep];
                const double2 a = cw[i0], bb = cw[i1];
                const double vr = bb.x * wv.x - bb.y * wv.y;
                const double vi = bb.x * wv.y + bb.y * wv.x;
                cw[i0] = make_double2(a.x + vr, a.y + vi);
                cw[i1] = make_double2(a.x - vr, a.y - vi);
            }
            __syncthreads();
        }
        // split: X_k = (Z_k + conj(Z_{m-k}))/2 - i/2 * W^k (Z_k - conj(Z_{m-k})), W = exp(-2 pi i/n)
        for (int kk = lane; kk <= m; kk += 64) {
            const double2 zk = cw[kk == m ? 0 : kk];
            const double2 zm = cw[(m - kk) % m];
            const double er = 0.5 * (zk.x + zm.x), ei = 0.5 * (zk.y - zm.y);
            const double orr = 0.5 * (zk.y + zm.y), oi = -0.5 * (zk.x - zm.x);
            const double2 wv = tw[kk == m ? 0 : kk];
            double wr = wv.x, wi = wv.y;
            if (kk == m) { wr = -1.0; wi = 0.0; }
            const double re = er + (orr * wr - oi * wi);
            const double im = ei + (orr * wi + oi * wr);
            const double a = hypot(re, im);
            if (isnan(a)) nanf = 1;
            best = fmax(best, a);
        }
    } else {
        for (int kk = lane; kk <= n / 2; kk += 64) {
            double sr = 0.0, si = 0.0;
            long q = 0;
            for (int j = 0; j < n; ++j) {
                const double v = valid ? (double)X[j] - mu : (double)X[j];
                const double2 wv = tw[q];
                sr += v * wv.x;
                si += v * wv.y;
                q += kk;
                if (q >= n) q -= n;
            }
            const double a = hypot(sr, si);
            if (isnan(a)) nanf = 1;
            best = fmax(best, a);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        best = fmax(best, __shfl_xor(best, off));
        nanf |= __shfl_xor(nanf, off);
    }
    if (lane == 0) {
        std_o[k] = valid ? sd : 0.0;
        mean_o[k] = valid ? mean : 0.0;
        ptp_o[k] = valid ? ptp : 1e20f;
        fft_o[k] = nanf ? NAN : best;
    }
}

// residual cube on request (ic_get_residual): R (dispersed frame, unweighted); grid-stride
__global__ __launch_bounds__(256) void k_residual(const float *__restrict__ D, const double *__restrict__ T64,
                                                  const double *__restrict__ amp, const int32_t *__restrict__ info,
                                                  const int32_t *__restrict__ shift, size_t N, int nchan, int nbin,
                                                  int pr_on, double pr_factor, int pr_start, int pr_end,
                                                  float *__restrict__ R)
{
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (size_t)gridDim.x * blockDim.x) {
        const size_t k = e / nbin;
        const int i = (int)(e - k * nbin);
        const int c = (int)(k % nchan);
        const int st = info[k];
        float v = 0.0f;
        if (st >= 1 && st <= 4) {
            const double u = amp[k] * T64[i];
            double ee = u - (double)D[e];
            if (pr_on && i >= pr_start && i < pr_end) ee = ee * pr_factor;
            v = (float)ee;
        }
        int j = i + shift[c];
        if (j >= nbin) j -= nbin;
        R[k * nbin + j] = v;
    }
}

// ============================================================ medians

__device__ __forceinline__ unsigned long long key64(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey64(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

__device__ void bitonic_sort(unsigned long long *a, int N)
{
    for (int kk = 2; kk <= N; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < N; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const bool up = (i & kk) == 0;
                    const unsigned long long x = a[i], y = a[ixj];
                    if ((x > y) == up) {
                        a[i] = y;
                        a[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// median of the cnt smallest keys (sorted ascending), numpy arithmetic in dtype
__device__ double sorted_median(const unsigned long long *a, int cnt, bool f32)
{
    const int idx = cnt / 2;
    if (f32) {
        const float hi = (float)unkey64(a[idx]);
        if (cnt % 2) return (double)(0.0f + hi);
        const float lo = (float)unkey64(a[idx - 1]);
        const float t = (0.0f + lo) + hi;
        return (double)(t / 2.0f);
    }
    const double hi = unkey64(a[idx]);
    if (cnt % 2) return 0.0 + hi;
    const double lo = unkey64(a[idx - 1]);
    const double t = (0.0 + lo) + hi;
    return t / 2.0;
}

// One block per line: lines [0, 4*nchan) are columns (diag = line / nchan),
// lines [4*nchan, 4*nchan + 4*nsub) rows.  diag 0 std, 1 mean, 2 ptp (f32), 3 fft (plain).
__global__ __launch_bounds__(256) void k_linestats(LineStatsArgs a)
{
    extern __shared__ unsigned long long keys[];
    __shared__ int cnt_s, nan_s;
    const int line = blockIdx.x;
    const bool col = line < 4 * a.nchan;
    const int diag = col ? line / a.nchan : (line - 4 * a.nchan) / a.nsub;
    const int idx = col ? line % a.nchan : (line - 4 * a.nchan) % a.nsub;
    const int len = col ? a.nsub : a.nchan;
    const bool f32 = diag == 2;
    const bool plain = diag == 3;
    int Npad = 1;
    while (Npad < len) Npad <<= 1;
    auto at = [&](int q, bool &v) -> double {
        const size_t kk = col ? (size_t)q * a.nchan + idx : (size_t)idx * a.nchan + q;
        v = plain ? true : (a.valid[kk] != 0);
        if (diag == 0) return a.std_d[kk];
        if (diag == 1) return a.mean_d[kk];
        if (diag == 2) return (double)a.ptp_d[kk];
        return a.fft_d[kk];
    };
    // pass 1: valid values
    if (threadIdx.x == 0) { cnt_s = 0; nan_s = 0; }
    __syncthreads();
    for (int q = threadIdx.x; q < Npad; q += blockDim.x) keys[q] = ~0ull;
    __syncthreads();
    for (int q = threadIdx.x; q < len; q += blockDim.x) {
        bool v;
        const double d = at(q, v);
        if (v) {
            const int pos = atomicAdd(&cnt_s, 1);
            keys[pos] = key64(d);
            if (isnan(d)) atomicOr(&nan_s, 1);
        }
    }
    __syncthreads();
    const int cnt = cnt_s;
    double med = NAN, mad = NAN;
    if (cnt > 0 && !nan_s) {
        bitonic_sort(keys, Npad);
        med = sorted_median(keys, cnt, f32);
        __syncthreads();
        // pass 2: |d - med| over valid entries (in dtype)
        if (threadIdx.x == 0) { cnt_s = 0; nan_s = 0; }
        __syncthreads();
        for (int q = threadIdx.x; q < Npad; q += blockDim.x) keys[q] = ~0ull;
        __syncthreads();
        for (int q = threadIdx.x; q < len; q += blockDim.x) {
            bool v;
            const double d = at(q, v);
            if (v) {
                double r;
                if (f32) r = (double)fabsf((float)d - (float)med);
                else r = fabs(d - med);
                const int pos = atomicAdd(&cnt_s, 1);
                keys[pos] = key64(r);
                if (isnan(r)) atomicOr(&nan_s, 1);
            }
        }
        __syncthreads();
        if (!nan_s) {
            bitonic_sort(keys, Npad);
            mad = sorted_median(keys, cnt, f32);
        }
    }
    if (threadIdx.x == 0) {
        if (col) {
            a.col_med[diag * a.nchan + idx] = med;
            a.col_mad[diag * a.nchan + idx] = mad;
        } else {
            a.row_med[diag * a.nsub + idx] = med;
            a.row_mad[diag * a.nsub + idx] = mad;
        }
    }
}

// ============================================================ combine

__device__ __forceinline__ double scale_masked_d(double dv, bool valid, double med, double mad, double thr)
{
    if (!valid) return 0.0 + fabs(dv);
    const double r = dv - med;
    const double q = r / mad;
    const bool dom = !isfinite(q) || (fabs(r) * DBL_MIN >= fabs(mad));
    if (dom) return 0.0 + fabs(0.0 + r);
    const double aq = fabs(q);
    const double res = aq / thr;
    if (!isfinite(res) || aq * DBL_MIN >= fabs(thr)) return 0.0 + aq;
    return res;
}

__device__ __forceinline__ double scale_masked_f(float dv, bool valid, float med, float mad, double thr)
{
    if (!valid) return 0.0 + (double)fabsf(dv);
    const float r = dv - med;
    const float q = r / mad;
    const bool dom = !isfinite(q) || ((double)fabsf(r) * DBL_MIN >= (double)fabsf(mad));
    if (dom) return 0.0 + (double)fabsf(0.0f + r);
    const float aq = fabsf(q);
    const double res = (double)aq / thr;
    if (!isfinite(res) || (double)aq * DBL_MIN >= fabs(thr)) return 0.0 + (double)aq;
    return res;
}

__device__ __forceinline__ double scale_plain(double dv, double med, double mad, double thr)
{
    const double r = dv - med;
    const double q = r / mad;
    return fabs(q) / thr;
}

__device__ __forceinline__ double nanmax2(double a, double b)
{
    if (isnan(a) || isnan(b)) return NAN;
    return a > b ? a : b;
}

// counters: [0] changed vs hist[iter-1], [1] zero weights, [2+h] != hist[h]
__global__ __launch_bounds__(256) void k_combine(
    int nsub, int nchan, const uint8_t *__restrict__ valid, const float *__restrict__ w0,
    const double *__restrict__ std_d, const double *__restrict__ mean_d, const float *__restrict__ ptp_d,
    const double *__restrict__ fft_d, const double *__restrict__ col_med, const double *__restrict__ col_mad,
    const double *__restrict__ row_med, const double *__restrict__ row_mad, double cth, double sth,
    double *__restrict__ test, float *__restrict__ W, float *__restrict__ hist, int iter,
    int32_t *__restrict__ counters)
{
    const size_t P = (size_t)nsub * nchan;
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    int changed = 0, zero = 0;
    if (k < P) {
        const int s = (int)(k / nchan), c = (int)(k % nchan);
        const bool v = valid[k] != 0;
        double S[4];
        S[0] = nanmax2(scale_masked_d(std_d[k], v, col_med[c], col_mad[c], cth),
                       scale_masked_d(std_d[k], v, row_med[s], row_mad[s], sth));
        S[1] = nanmax2(scale_masked_d(mean_d[k], v, col_med[nchan + c], col_mad[nchan + c], cth),
                       scale_masked_d(mean_d[k], v, row_med[nsub + s], row_mad[nsub + s], sth));
        S[2] = nanmax2(scale_masked_f(ptp_d[k], v, (float)col_med[2 * nchan + c], (float)col_mad[2 * nchan + c], cth),
                       scale_masked_f(ptp_d[k], v, (float)row_med[2 * nsub + s], (float)row_mad[2 * nsub + s], sth));
        S[3] = nanmax2(scale_plain(fft_d[k], col_med[3 * nchan + c], col_mad[3 * nchan + c], cth),
                       scale_plain(fft_d[k], row_med[3 * nsub + s], row_mad[3 * nsub + s], sth));
        double t;
        if (isnan(S[0]) || isnan(S[1]) || isnan(S[2]) || isnan(S[3])) {
            t = NAN;
        } else {
            // sort 4
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3 - a; ++b)
                    if (S[b] > S[b + 1]) {
                        const double tmp = S[b];
                        S[b] = S[b + 1];
                        S[b + 1] = tmp;
                    }
            t = ((0.0 + S[1]) + S[2]) / 2.0;
        }
        test[k] = t;
        const float wn = (t >= 1.0) ? 0.0f : w0[k];
        W[k] = wn;
        hist[(size_t)iter * P + k] = wn;
        changed = !(wn == hist[(size_t)(iter - 1) * P + k]);
        zero = (wn == 0.0f);
    }
    // wave reduce then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        changed += __shfl_xor(changed, off);
        zero += __shfl_xor(zero, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (changed) atomicAdd(&counters[0], changed);
        if (zero) atomicAdd(&counters[1], zero);
    }
    // history equality (iterative_cleaner.py:135-136): counters[2+h] |= any(W != hist[h])
    for (int h = 0; h < iter; ++h) {
        int d = 0;
        if (k < P) d = !(W[k] == hist[(size_t)h * P + k]);
        if (__any(d) && (threadIdx.x & 63) == 0) atomicOr(&counters[2 + h], 1);
    }
}

// ============================================================ launchers

static inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_chan_partials(hipStream_t st, const float *raw, const float *W, const int32_t *shift,
                                const float *base, int nsub, int nchan, int nbin, double *part,
                                double *wpart)
{
    const int nsb = (nchan + kSuperBlock - 1) / kSuperBlock;
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    dim3 grid(cdiv(nbin, bs), nsb, nsub);
    hipLaunchKernelGGL(k_chan_partials, grid, dim3(bs), 0, st, raw, W, shift, base, nsub, nchan, nbin,
                       nsb, part, wpart);
    return hipGetLastError();
}

hipError_t launch_window(hipStream_t st, const double *part, int nsub, int nsb, int nbin, int width,
                         int32_t *win)
{
    const size_t shm = (size_t)nbin * 8 + 256 * 8 + 256 * 4;
    hipLaunchKernelGGL(k_window, dim3(nsub), dim3(256), shm, st, part, nsb, nbin, width, win);
    return hipGetLastError();
}

hipError_t launch_base(hipStream_t st, const float *raw, const int32_t *shift, const int32_t *win,
                       int nsub, int nchan, int nbin, int width, float *base)
{
    const size_t P = (size_t)nsub * nchan;
    hipLaunchKernelGGL(k_base, dim3(cdiv(P, 256)), dim3(256), 0, st, raw, shift, win, nsub, nchan, nbin,
                       width, base);
    return hipGetLastError();
}

hipError_t launch_fitcube(hipStream_t st, const float *raw, const int32_t *shift, const float *base,
                          int nsub, int nchan, int nbin, float *D)
{
    const size_t N = (size_t)nsub * nchan * nbin;
    const unsigned grid = (unsigned)(cdiv(N, 256) < 65536u * 8 ? cdiv(N, 256) : 65536u * 8);
    hipLaunchKernelGGL(k_fitcube, dim3(grid), dim3(256), 0, st, raw, shift, base, nsub, nchan, nbin, D);
    return hipGetLastError();
}

hipError_t launch_fscrunch(hipStream_t st, const double *part, const double *wpart, int nsub, int nsb,
                           int nbin, float *F, float *wf)
{
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    hipLaunchKernelGGL(k_fscrunch, dim3(cdiv(nbin, bs), nsub), dim3(bs), 0, st, part, wpart, nsb, nbin, F,
                       wf);
    return hipGetLastError();
}

hipError_t launch_tscrunch(hipStream_t st, const float *F, const float *wf, int nsub, int nbin, float *T,
                           double *T64)
{
    hipLaunchKernelGGL(k_tscrunch, dim3(cdiv(nbin, 64)), dim3(64), 0, st, F, wf, nsub, nbin, T, T64);
    return hipGetLastError();
}

hipError_t launch_fit(hipStream_t st, const float *D, const double *T64, long P, int nbin, double *amp,
                      int32_t *info)
{
    hipLaunchKernelGGL(k_fit, dim3(cdiv(P, 64)), dim3(64), 0, st, D, T64, P, nbin, amp, info);
    return hipGetLastError();
}

size_t diag_lds_bytes(int nbin, int nleaf, int nops)
{
    const bool pow2 = (nbin & (nbin - 1)) == 0 && nbin >= 4;
    size_t b = (size_t)(pow2 ? nbin / 2 : 1) * 16;
    b += ((size_t)nbin * 4 + 15) & ~(size_t)15;
    b += (size_t)(nleaf * 9 + nops + 8) * 8;
    return b;
}

hipError_t launch_diag(hipStream_t st, const float *D, const double *T64, const double *amp,
                       const int32_t *info, const float *w0, const int32_t *shift, const double2 *tw,
                       const PwPlan *plan, int nsub, int nchan, int nbin, int pr_on, double pr_factor,
                       int pr_start, int pr_end, double *std_o, double *mean_o, float *ptp_o,
                       double *fft_o)
{
    (void)nsub;
    // nleaf/nops upper bound from nbin: leaves >= 64 samples except tiny n
    const int nleaf_ub = nbin <= 128 ? 1 : (nbin / 64 + 1);
    const size_t shm = diag_lds_bytes(nbin, nleaf_ub, nleaf_ub);
    const size_t P = (size_t)nsub * nchan;
    hipLaunchKernelGGL(k_diag, dim3((unsigned)P), dim3(64), shm, st, D, T64, amp, info, w0, shift, tw, plan,
                       nsub, nchan, nbin, pr_on, pr_factor, pr_start, pr_end, std_o, mean_o, ptp_o, fft_o);
    return hipGetLastError();
}

static int next_pow2(int v)
{
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

hipError_t launch_linestats(hipStream_t st, const LineStatsArgs &a)
{
    const int Npad = next_pow2(a.nsub > a.nchan ? a.nsub : a.nchan);
    const size_t shm = (size_t)Npad * 8;
    const unsigned lines = 4u * (unsigned)(a.nchan + a.nsub);
    hipLaunchKernelGGL(k_linestats, dim3(lines), dim3(256), shm, st, a);
    return hipGetLastError();
}

hipError_t launch_combine(hipStream_t st, int nsub, int nchan, const uint8_t *valid, const float *w0,
                          const double *std_d, const double *mean_d, const float *ptp_d,
                          const double *fft_d, const double *col_med, const double *col_mad,
                          const double *row_med, const double *row_mad, double chanthresh,
                          double subintthresh, double *test, float *W, float *hist, int iter,
                          int32_t *counters)
{
    const size_t P = (size_t)nsub * nchan;
    hipLaunchKernelGGL(k_combine, dim3(cdiv(P, 256)), dim3(256), 0, st, nsub, nchan, valid, w0, std_d,
                       mean_d, ptp_d, fft_d, col_med, col_mad, row_med, row_mad, chanthresh, subintthresh,
                       test, W, hist, iter, counters);
    return hipGetLastError();
}

hipError_t launch_residual(hipStream_t st, const float *D, const double *T64, const double *amp,
                           const int32_t *info, const int32_t *shift, int nsub, int nchan, int nbin,
                           int pr_on, double pr_factor, int pr_start, int pr_end, float *R)
{
    const size_t N = (size_t)nsub * nchan * nbin;
    const unsigned grid = (unsigned)(cdiv(N, 256) < 65536u * 8 ? cdiv(N, 256) : 65536u * 8);
    hipLaunchKernelGGL(k_residual, dim3(grid), dim3(256), 0, st, D, T64, amp, info, shift, N, nchan, nbin,
                       pr_on, pr_factor, pr_start, pr_end, R);
    return hipGetLastError();
}

}  // namespace icgpu
