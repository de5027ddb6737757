// ic_internal.h — shared declarations between the host session (ic_session.hip)
// and the gfx950 kernels (ic_kernels.hip).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace icgpu {

constexpr int kSuperBlock = 256;    // canonical channel super-block (archive.py SUPER_BLOCK)
constexpr int kMaxLeaves = 256;     // pairwise-sum leaves (nbin <= 32768)
constexpr int kFitTile = 32;        // bins per k_fit_pass LDS tile (fit cube row padding)

// numpy pairwise-summation plan for one nbin (numpy loops_utils.h.src order):
// leaves in address order, then a post-order list of internal adds.
struct PwPlan {
    int32_t n;
    int32_t nleaf;
    int32_t nops;
    int32_t root;                   // slot of the final value
    int32_t leaf_start[kMaxLeaves];
    int32_t leaf_len[kMaxLeaves];
    int32_t op_a[kMaxLeaves];       // slot ids; slot nleaf+o is the o-th op result
    int32_t op_b[kMaxLeaves];
};

enum KernelId {
    K_CHAN_PARTIALS = 0,
    K_WINDOW,
    K_BASE,
    K_FITCUBE,
    K_FSCRUNCH,
    K_TSCRUNCH,
    K_FIT_PASS,
    K_FIT_STATE,
    K_DIAG,
    K_LINESTATS,
    K_COMBINE,
    K_RESIDUAL,
    K_FIT_TAIL,
    K_COUNT
};

// lmdif per-profile state (structure of arrays, device memory)
struct FitStateArrays {
    double *x, *fnorm, *par, *delta, *diag, *xnorm, *acnorm, *J0, *f0, *aj, *r, *Jn0, *qtf, *gnorm,
        *x2, *pnorm, *wa1, *xa;
    int32_t *iter, *nfev, *mode, *slow;
    double *o_fnorm, *o_acnorm, *o_f0, *o_J0, *o_sum;
    int32_t *o_exact;
};

struct LineStatsArgs {
    int nsub, nchan;
    const uint8_t *valid;
    const double *std_d, *mean_d, *fft_d;
    const float *ptp_d;
    double *col_med, *col_mad;      // [4][nchan]
    double *row_med, *row_mad;      // [4][nsub]
};

// ---- launch wrappers (ic_kernels.hip); all asynchronous on `st` ----
// mode 0: part = sum W*ded; 1: part2 = sum W*f32(ded-base) + wpart; 2: both.
// flags: only subints with flags[s] != 0 (nullptr: all)
hipError_t launch_chan_partials(hipStream_t st, int mode, const float *raw, const float *W, const int32_t *shift,
                                const float *base, const int32_t *flags, int nsub, int nchan, int nbin,
                                double *part, double *part2, double *wpart);
// flags != nullptr: flags[s] = window of subint s moved (win updated in place)
hipError_t launch_window(hipStream_t st, const double *part, int nsub, int nsb, int nbin, int width,
                         int32_t *win, int32_t *flags);
// flags != nullptr: only subints with flags[s] != 0
hipError_t launch_base(hipStream_t st, const float *raw, const int32_t *shift, const int32_t *win,
                       const int32_t *flags, int nsub, int nchan, int nbin, int width, float *base);
hipError_t launch_fitcube(hipStream_t st, const float *raw, const int32_t *shift, const float *base,
                          int nsub, int nchan, int nbin, int ldD, float *D);
hipError_t launch_fscrunch(hipStream_t st, const double *part, const double *wpart, int nsub, int nsb,
                           int nbin, float *F, float *wf);
hipError_t launch_tscrunch(hipStream_t st, const float *F, const float *wf, int nsub, int nbin, float *T,
                           double *T64);
hipError_t launch_fit_init(hipStream_t st, const FitStateArrays &S, long P);
// list == nullptr: all P profiles; else list[0 .. *nlist) with *nlist <= bound
// (the host sizes grids from a count it already knows: counts only shrink).
hipError_t launch_fit_pass(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           const int32_t *list, const int32_t *nlist, long bound, const FitStateArrays &S);
hipError_t launch_fit_state(hipStream_t st, const FitStateArrays &S, long P, const int32_t *list,
                            const int32_t *nlist, long bound, double *amp, int32_t *info, int32_t *next_list,
                            int32_t *next_n);
hipError_t launch_fit_tail(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           const int32_t *list, const int32_t *nlist, long bound, const FitStateArrays &S,
                           double *amp, int32_t *info, unsigned long long *sweeps);
// tw: exp(-2 pi i q/nbin), q < nbin; tw_p2 (power-of-two nbin only): see p2_twiddles()
hipError_t launch_diag(hipStream_t st, const float *D, const double *T64, const double *amp,
                       const int32_t *info, const float *w0, const int32_t *shift, const double2 *tw,
                       const double2 *tw_p2, const PwPlan *plan, int nsub, int nchan, int nbin, int ldD, int pr_on, double pr_factor,
                       int pr_start, int pr_end, double *std_o, double *mean_o, float *ptp_o,
                       double *fft_o);
hipError_t launch_linestats(hipStream_t st, const LineStatsArgs &a);
hipError_t launch_combine(hipStream_t st, int nsub, int nchan, const uint8_t *valid, const float *w0,
                          const double *std_d, const double *mean_d, const float *ptp_d,
                          const double *fft_d, const double *col_med, const double *col_mad,
                          const double *row_med, const double *row_mad, double chanthresh,
                          double subintthresh, double *test, float *W, float *hist, int iter,
                          int32_t *counters);
hipError_t launch_residual(hipStream_t st, const float *D, const double *T64, const double *amp,
                           const int32_t *info, const int32_t *shift, int nsub, int nchan, int nbin, int ldD,
                           int pr_on, double pr_factor, int pr_start, int pr_end, float *R);

}  // namespace icgpu
