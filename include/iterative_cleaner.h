/*
 * iterative_cleaner.h — C-ABI of libicgpu.so, the MI355X (gfx950) surgical
 * RFI-cleaning loop.
 *
 * The reference has no FFI layer; its drop-in boundary is the Python function
 * clean(ar, args, arch) (/root/reference/iterative_cleaner.py:65).  The
 * entry points below replace the body of its cleaning loop,
 * iterative_cleaner.py:83-146 (template :88-94, fit-cube prep :96-100,
 * remove_profile_inplace :101/:259-288, dededisperse :104, apply_weights
 * :111-117/:291-297, comprehensive_stats :120/:181-256, set_weights_archive
 * :122-125/:300-305, convergence :127-146).  The Python host
 * (iterative_cleaner_amd/cleaner.py) keeps the reference's CLI, clean()
 * signature, prints, log and file side effects, and binds these symbols with
 * ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - plain pointers and sizes only; host arrays are caller-owned and copied;
 *   - return 0 on success, a negative IC_E* code on error; the message of the
 *     last error on the calling thread is ic_last_error();
 *   - one session per host thread; sessions on different devices may run
 *     concurrently (every call is synchronous on the session's HIP stream).
 *
 * Layouts: cube[s][c][b] float32 (nsub, nchan, nbin), profile-contiguous, in
 * the DISPERSED frame, already pscrunched (total intensity); weights[s][c]
 * float32; shift[c] = dedispersion delay in bins (ded[i] = raw[(i+shift)%nbin]).
 */
#ifndef ITERATIVE_CLEANER_H
#define ITERATIVE_CLEANER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IC_ABI_VERSION 2

#define IC_OK 0
#define IC_EINVAL -1   /* bad argument / shape                         */
#define IC_EHIP -2     /* HIP runtime error                            */
#define IC_ENOMEM -3   /* device or host allocation failed             */
#define IC_ESTATE -4   /* call out of order (e.g. run before upload)   */

/* Loop parameters: args Namespace of iterative_cleaner.py:16-42. */
typedef struct {
    int32_t nsub, nchan, nbin;
    int32_t max_iter;          /* -m                                          */
    double chanthresh;         /* -c  (iterative_cleaner.py:19, default 5)     */
    double subintthresh;       /* -s  (:23, default 5)                         */
    int32_t pr_on;             /* pulse_region != [0,0,1] (:280)               */
    double pr_factor;          /* pulse_region[0] (:283)                       */
    int32_t pr_start, pr_end;  /* slice(int(pr[1]), int(pr[2])).indices(nbin) */
    double baseline_duty;      /* archive stand-in remove_baseline duty (0.15) */
    int32_t fit_mode;          /* 0 = exact scipy leastsq emulation (default)  */
} ic_params;

/* Library / device info. */
int ic_abi_version(void);
int ic_device_count(void);

/* Session lifetime.  device: HIP ordinal. */
int ic_session_create(const ic_params *params, int device, void **session);
void ic_session_destroy(void *session);

/* Upload the cube (host pointers; one H2D copy).  Replaces the archive data
 * read by iterative_cleaner.py:97-100 (fit cube) and :88-93 (template). */
int ic_upload(void *session, const float *cube, const float *w0, const int32_t *shift);

/* Same from device pointers already resident in HBM on the session's device
 * (e.g. torch-ROCm tensors): a device-to-device copy, no PCIe. */
int ic_upload_device(void *session, const float *d_cube, const float *d_w0,
                     const int32_t *d_shift);

/* Run the cleaning loop to convergence or max_iter (iterative_cleaner.py:83-146).
 * Outputs (host, any may be NULL):
 *   test_out        [nsub*nchan] f64 : avg_test_results of the last loop (:120)
 *   weights_out     [nsub*nchan] f32 : weights of the last loop (:125, :128)
 *   loops_out       [1]              : `loops` (:139, :146)
 *   changed_out     [max_iter]       : "Differences to previous weights" (:129)
 *   nzero_out       [max_iter]       : zero-weight count -> "RFI fraction" (:130)
 *   n_iter_out      [1]              : loop iterations executed
 *   converged_out   [1]              : 1 if the loop stopped on a repeated mask
 *                                      (:135-140), 0 if it hit max_iter (:143) */
int ic_run(void *session, double *test_out, float *weights_out, int32_t *loops_out,
           int32_t *changed_out, int32_t *nzero_out, int32_t *n_iter_out, int32_t *converged_out);

/* The last iteration's residual cube (:101-108), dispersed frame, unweighted,
 * f32 [nsub][nchan][nbin] — what --unload_res writes (:161-162). */
int ic_get_residual(void *session, float *out);

/* Last iteration's internals for parity checks (any may be NULL):
 * template T [nbin], fit amplitude/status [P] (:278), diagnostics [P] (:206-217). */
int ic_get_template(void *session, float *T);
int ic_get_fit(void *session, double *amp, int32_t *info);
int ic_get_diagnostics(void *session, double *std_o, double *mean_o, float *ptp_o,
                       double *fftmax_o);

/* Per-launch timing of the last ic_run (HIP events on the session stream):
 * fills up to n entries of {kernel id, milliseconds summed over the run,
 * launches}; returns the number of kernel ids. */
typedef struct {
    int32_t kernel;
    int32_t launches;
    double ms;
} ic_kernel_time;
int ic_get_kernel_times(void *session, ic_kernel_time *out, int n);
const char *ic_kernel_name(int kernel);
int ic_set_timing(void *session, int enabled);

/* Statistics of the last ic_run (measurement; see DESIGN.md roofline). */
typedef struct {
    int32_t iterations;          /* cleaning loops executed                        */
    int32_t fit_rounds;          /* k_fit_pass launches, summed over iterations    */
    int64_t fit_profile_sweeps;  /* profiles swept by k_fit_pass, summed (x nbin x 4 B = fit bytes) */
    int64_t fit_tail_sweeps;     /* profile sweeps done by k_fit_tail (the last few thousand profiles) */
    int32_t window_moves;        /* subint baseline windows that moved between iterations */
    int32_t reserved;
} ic_run_stats;
int ic_get_run_stats(void *session, ic_run_stats *out);

/* Scheduling knob of the exact fit: when at most `threshold` profiles still
 * need data sweeps, k_fit_tail finishes them in one launch (one wave per
 * profile) instead of further sweep/state rounds.  Results are identical either
 * way (both paths are bit-exact).  0 = never; default 8192. */
int ic_set_fit_tail(void *session, int64_t threshold);

const char *ic_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ITERATIVE_CLEANER_H */
