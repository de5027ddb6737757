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

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IC_ABI_VERSION 8

#define IC_OK 0
#define IC_EINVAL -1   /* bad argument / shape                         */
#define IC_EHIP -2     /* HIP runtime error                            */
#define IC_ENOMEM -3   /* device or host allocation failed             */
#define IC_ESTATE -4   /* call out of order (e.g. run before upload)   */
#define IC_ECOMM -5    /* a shard exchange failed (or a peer aborted)  */

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
    int32_t fit_mode;          /* IC_FIT_EXACT (default) or IC_FIT_CLOSED       */
    int32_t data_f64;          /* psrchive get_data dtype: 0 = f32
                                  (default), 1 = f64: apply_weights and the masked
                                  statistics then run in f64 (iterative_cleaner.py:
                                  111-112, 206-209): X = f64(R) * f64(w), f64 mean
                                  sum and ptp, ptp scaled in f64.  The samples must
                                  still be f32 values (the archive's amplitudes).  */
    int32_t dedisp_mode;       /* IC_DEDISP_SHIFT (default) or IC_DEDISP_FFT       */
    int32_t input_dedispersed; /* 1: the uploaded cube is the archive as stored
                                  DEDISPERSED (psrchive get_dedispersed()): the
                                  reference's dedisperse (:91, :100) is then a
                                  no-op and only the residual's dededisperse (:104)
                                  rotates.  IC_DEDISP_FFT only (with integer shifts
                                  the host rolls the cube back to the dispersed
                                  frame, which is exact); 0 otherwise.            */
} ic_params;

/* ic_params.fit_mode.
 *   IC_FIT_EXACT   scipy.optimize.leastsq(a*T - p, [1.0]) emulated bit for bit
 *                  (MINPACK lmdif, n = 1; iterative_cleaner.py:277-278): the
 *                  reference's arithmetic, zap masks identical to it.
 *   IC_FIT_CLOSED  the closed-form least-squares amplitude
 *                  a = sum_i T_i p_i / sum_i T_i^2 (f64 numpy pairwise sums; the
 *                  products T_i p_i of the dedispersed profile summed in the
 *                  stored, dispersed sample order j = (i + shift) mod nbin
 *                  since round 6; a = 0 when the template is all zero;
 *                  info = 1, or 5 (residual zeroed) when a is not finite), fused
 *                  with the residual and the diagnostics in one sweep of the raw
 *                  cube: the HBM-bound fast mode of the north star.  It is NOT
 *                  the reference's arithmetic: amplitudes differ from leastsq in
 *                  the last bits, and rarely a profile's zap decision flips. */
#define IC_FIT_EXACT 0
#define IC_FIT_CLOSED 1

/* ic_params.dedisp_mode: how dedisperse / dededisperse (iterative_cleaner.py:91,
 * :100, :104) move a channel's samples.
 *   IC_DEDISP_SHIFT  integer rotation by shift[c] bins (ded[i] = raw[(i+shift)%nbin]),
 *                    the archive stand-in's default.
 *   IC_DEDISP_FFT    psrchive's FFT phase rotation by a fractional delay
 *                    (ic_set_delays: delay[c] bins per channel; ic_set_delays2:
 *                    delay[s][c] per profile, psrchive's per-Integration folding
 *                    period): forward real FFT, harmonic k times
 *                    exp(+-2 pi i k delay / nbin), inverse real FFT, in IEEE
 *                    f32 (psrchive's precision) and the arithmetic order
 *                    written in iterative_cleaner_amd/phase_rotation.py
 *                    (bit-identical to it and to the C oracle; within 4 f32
 *                    epsilons of the profile's largest |sample| of numpy's f64
 *                    irfft(rfft(x) * phasor); parity with real psrchive
 *                    unpinned).  nbin must be a power of
 *                    two in 64..4096 (either fit_mode); the shift arrays of the
 *                    uploads are then unused (pass zeros). */
#define IC_DEDISP_SHIFT 0
#define IC_DEDISP_FFT 1

/* Library / device info. */
int ic_abi_version(void);
int ic_device_count(void);

/* Session lifetime.  device: HIP ordinal. */
int ic_session_create(const ic_params *params, int device, void **session);
void ic_session_destroy(void *session);

/* Upload the cube (host pointers; one H2D copy).  Replaces the archive data
 * read by iterative_cleaner.py:97-100 (fit cube) and :88-93 (template). */
int ic_upload(void *session, const float *cube, const float *w0, const int32_t *shift);

/* Full-polarisation upload: data [nsub][npol][nchan][nbin] f32 as the archive
 * holds it (psrchive get_data), pscrunched ON THE DEVICE to the total intensity
 * f32(pol0 + pol1) (npol >= 2; npol == 1: pol0), the pscrunch of
 * iterative_cleaner.py:70/:89/:100 (archive.py pscrunch).  The host then never
 * pscrunches a copy of the archive. */
int ic_upload_pols(void *session, const float *data, int npol, const float *w0, const int32_t *shift);

/* Same from device pointers already resident in HBM on the session's device
 * (e.g. torch-ROCm tensors): a device-to-device copy, no PCIe. */
int ic_upload_device(void *session, const float *d_cube, const float *d_w0,
                     const int32_t *d_shift);

/* Batch pipelining (config C4: many archives of one shape per GPU).  Queue the
 * host->device copy of the NEXT archive on the session's copy stream and return
 * at once; the next ic_run waits for the copy and cleans that archive.  Two input
 * slots: at most two uploads may be pending, so the pattern
 *     ic_upload_async(a0); for k: { ic_upload_async(a[k+1]); ic_run(); }
 * overlaps every archive's copy with the previous archive's cleaning.  The host
 * arrays of an upload must stay untouched until the ic_run that consumes it
 * returns, and must be page-locked (ic_host_alloc) for the copy to overlap.
 * ic_upload / ic_upload_device fail with IC_ESTATE while uploads are pending.
 * Replaces the per-archive reload of iterative_cleaner.py:60 (main loop). */
int ic_upload_async(void *session, const float *cube, const float *w0, const int32_t *shift);
int ic_host_alloc(size_t bytes, void **ptr);
void ic_host_free(void *ptr);

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

/* Fractional delays of the session's channels (dedisp_mode IC_DEDISP_FFT):
 * delay_bins [nchan] f64 (a shard: its nchan_loc channels), in bins, finite;
 * dedisperse moves sample j + delay to j.  Required before ic_run; kept until
 * changed. */
int ic_set_delays(void *session, const double *delay_bins);
/* The same with one delay per profile: delay_bins [nsub*nchan] f64 (a shard:
 * [nsub][nchan_loc]), profile (s, c) at s*nchan + c — psrchive dedisperses each
 * Integration with its own folding period (delay_s,c = DM delay of channel c /
 * period_s * nbin).  The phasors exp(2 pi i k delay / nbin) are then evaluated
 * per profile on the device by the same f64 formula the channel table uses, so
 * rows that are all equal give exactly ic_set_delays' results (and take its
 * table). */
int ic_set_delays2(void *session, const double *delay_bins);

/* dedisperse (sign +1) or dededisperse (sign -1) a cube [nsub][nchan][nbin] f32
 * by the FFT phase rotation on the GPU (the operation IC_DEDISP_FFT applies at
 * iterative_cleaner.py:91/:100/:104).  Synchronous; in and out may alias. */
int ic_rotate_profiles(int device, int nsub, int nchan, int nbin, const float *in, const double *delay_bins,
                       int sign, float *out);
/* The same with per-profile delays delay_bins [nsub*nchan] (ic_set_delays2). */
int ic_rotate_profiles2(int device, int nsub, int nchan, int nbin, const float *in, const double *delay_bins,
                        int sign, float *out);

/* The last iteration's residual cube (:101-108), dispersed frame, unweighted,
 * f32 [nsub][nchan][nbin] — what --unload_res writes (:161-162). */
int ic_get_residual(void *session, float *out);

/* Profiles whose fit status was not 1-4 in each iteration of the last ic_run
 * (the reference prints "Bad status for least squares fit when removing
 * profile." once per such profile and loop, iterative_cleaner.py:284-285, and
 * zeroes its residual).  Fills up to n entries; returns the iteration count. */
int ic_get_bad_fits(void *session, int32_t *per_iter, int n);

/* Last iteration's internals for parity checks (any may be NULL):
 * template T [nbin], fit amplitude/status [P] (:278), diagnostics [P] (:206-217). */
int ic_get_template(void *session, float *T);
int ic_get_fit(void *session, double *amp, int32_t *info);
int ic_get_diagnostics(void *session, double *std_o, double *mean_o, float *ptp_o,
                       double *fftmax_o);
/* The same with ptp in f64 (the data_f64 loop's ptp is an f64 value). */
int ic_get_diagnostics_f64(void *session, double *std_o, double *mean_o, double *ptp_o,
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
/* Restrict the timing to one kernel id (ic_kernel_name ids; -1 = every kernel,
 * the default): two HIP events per launch cost ~5 us, so a timed region that
 * must stay representative times only the kernel it prices. */
int ic_set_timing_kernel(void *session, int kernel);

/* Statistics of the last ic_run (measurement; see DESIGN.md roofline). */
typedef struct {
    int32_t iterations;          /* cleaning loops executed                        */
    int32_t fit_rounds;          /* k_fit_pass launches, summed over iterations    */
    int64_t fit_profile_sweeps;  /* profiles swept by k_fit_pass, summed (x nbin x 4 B = fit bytes) */
    int64_t fit_tail_sweeps;     /* profile sweeps done by k_fit_tail (the last few thousand profiles) */
    int32_t window_moves;        /* subint baseline windows that moved between iterations */
    int32_t near_threshold;      /* last iteration: profiles whose test value lies within 1e-9 of
                                    the zap threshold 1.0, where fftmax's last bits (not
                                    bit-identical to numpy's pocketfft) could decide the zap */
    int64_t reserved0;           /* 0 (round 4's persistent-lanes counters; that schedule was
                                    removed in round 5) */
    int64_t reserved1;           /* 0 */
} ic_run_stats;
int ic_get_run_stats(void *session, ic_run_stats *out);

/* Schedule options of a session.  They choose how the work of the loop is
 * scheduled, never its arithmetic: every setting gives the same bits (the GPU
 * tests hold each schedule equal to the default and to the oracle).  Set after
 * ic_session_create; read by the following ic_run calls.  The library reads
 * no environment variables.  ic_set_option fails with IC_EINVAL for an unknown
 * option or a value out of range (given below), and on a session the option
 * cannot serve.
 *   IC_OPT_FIT_TAIL        profiles left when k_fit_tail takes over the exact
 *                          fit (one wave per profile), >= 0, 0 = never; 8192
 *                          (4096 for sessions of >= 2^20 profiles, else 12288
 *                          for nbin >= 2048)
 *   IC_OPT_DIAG_FORK       fit round after which the diagnostics of the fitted
 *                          profiles run on a second stream, 0..64, 0 = no fork;
 *                          3 (4 for nbin >= 2048 with integer dedispersion)
 *                          (exact fit only)
 *   IC_OPT_FORK_DELAY      rounds between that round and the forked pass, 0..8;
 *                          1 (2 for nbin >= 2048)
 *   IC_OPT_TEMPLATE_INCR   1 = incremental template stage (integer
 *                          dedispersion), 0 = full template passes; 1
 *   IC_OPT_FIT_TILED       1 = tiled fit cube (integer dedispersion),
 *                          0 = row-major; 1
 *   IC_OPT_ROWSTAT_WAVES   waves per row median/MAD line: 0 (one wave), 4 or 8; 8
 *   IC_OPT_ROWSTAT_MINLEN  shortest row that takes them, 1..16384; 1024
 *   IC_OPT_DIAG_CHAIN      1 = chain-layout diagnostics kernel at nbin 1024,
 *                          2048, 4096; 0 = the row-layout kernel; 1
 *   IC_OPT_FIT_SCHEDULE    how the exact fit is scheduled: IC_FIT_ROUNDS (the
 *                          only value since round 5) = rounds of a sweep kernel
 *                          over every profile with a pending data request and a
 *                          state kernel, k_fit_tail for the last profiles
 *   IC_OPT_TAIL_SPLIT      with the fork: at the hand-over to k_fit_tail the
 *                          fork round's survivors already fitted are measured
 *                          on the second stream beside the tail, only the
 *                          tail's profiles after it: IC_TAIL_SPLIT_OFF, _ON, or
 *                          _AUTO (on for nbin >= 2048); IC_TAIL_SPLIT_AUTO
 *   IC_OPT_ROT_STATS       FFT dedispersion at nbin 1024 (f32 data): 1 = the
 *                          residual's inverse rotation measures its rows in the
 *                          same kernel (the rotated residual never goes to
 *                          HBM), 0 = it writes them and a statistics pass reads
 *                          them back; 1
 *   IC_OPT_SYNC_TIMEOUT_MS longest host wait for the GPU, >= 1 ms; 600000.  A
 *                          wait that runs out fails its call with IC_EHIP and
 *                          marks the session failed: every later call on it
 *                          but ic_session_destroy fails with IC_ESTATE, and
 *                          destroy then leaks its device memory (its kernels may
 *                          still be running) instead of freeing it. */
#define IC_OPT_FIT_TAIL 1
#define IC_OPT_DIAG_FORK 2
#define IC_OPT_FORK_DELAY 3
#define IC_OPT_TEMPLATE_INCR 4
#define IC_OPT_FIT_TILED 5
#define IC_OPT_ROWSTAT_WAVES 6
#define IC_OPT_ROWSTAT_MINLEN 7
#define IC_OPT_DIAG_CHAIN 8
#define IC_OPT_SYNC_TIMEOUT_MS 9
#define IC_OPT_FIT_SCHEDULE 10
/* 11, 12: IC_OPT_FIT_LANE_WAVES, IC_OPT_FIT_LATE_LANES until round 4 (removed
 * with the lanes schedule) */
#define IC_OPT_TAIL_SPLIT 13
#define IC_OPT_ROT_STATS 14
#define IC_TAIL_SPLIT_OFF 0
#define IC_TAIL_SPLIT_ON 1
#define IC_TAIL_SPLIT_AUTO 2
#define IC_FIT_ROUNDS 0
int ic_set_option(void *session, int option, int64_t value);
int ic_get_option(void *session, int option, int64_t *value);
/* = ic_set_option(session, IC_OPT_FIT_TAIL, threshold) */
int ic_set_fit_tail(void *session, int64_t threshold);

const char *ic_last_error(void);

/* remove_profile1d (iterative_cleaner.py:275-288) on the GPU for nprof given
 * profiles [nprof][nbin] f32 against the template T [nbin] f32: the amplitude
 * (:278; fit_mode as ic_params.fit_mode) and status per profile, and the f32
 * residual a*T - p (zeros for a status outside 1-4, :284-286).  Outputs may be
 * NULL (not all).  Synchronous. */
int ic_fit_profiles(int device, int nprof, int nbin, const float *T, const float *profiles, int fit_mode,
                    double *amp_out, int32_t *info_out, float *resid_out);

/* comprehensive_stats (iterative_cleaner.py:181-226) alone, on the GPU, for
 * the data the reference hands it (:111-117): data [nsub][nchan][nbin] f32 and
 * weights [nsub][nchan] f32; the kernel forms X = f32(data * w), masked where
 * w == 0, computes the four diagnostics (:206-217), their channel / subint
 * median-MAD scaling (:219-224) and test [nsub*nchan] f64 = the median of the
 * four (:225).  std/mean/ptp/fftmax outputs may be NULL.  Synchronous. */
int ic_comprehensive_stats(int device, int nsub, int nchan, int nbin, const float *data, const float *weights,
                           double chanthresh, double subintthresh, double *test_out, double *std_out,
                           double *mean_out, float *ptp_out, double *fftmax_out);
/* The same with the row-median form of IC_OPT_ROWSTAT_WAVES / _MINLEN. */
int ic_comprehensive_stats_rowstat(int device, int nsub, int nchan, int nbin, const float *data,
                                   const float *weights, double chanthresh, double subintthresh, double *test_out,
                                   double *std_out, double *mean_out, float *ptp_out, double *fftmax_out,
                                   int rowstat_waves, int rowstat_minlen);

/* ------------------------------------------------------------------------
 * Channel-sharded cleaning of ONE archive across `world` shards (config C3,
 * SURVEY.md §8(e)).  The reference cleans an archive in one process
 * (iterative_cleaner.py:83-146); these entry points split the same loop by
 * channel blocks.  Rank r owns the channels of one node of the canonical
 * super-block tree (archive.py sb_tree / shards.py channel_shards) and the
 * subint rows [r*nsub/world, (r+1)*nsub/world) of the row medians.  Per
 * iteration a shard exchanges: the template's per-subint channel-sum roots,
 * each row sent to its row owner (two all-to-alls, nsub*nbin f64 out per rank),
 * the owners' windows and fscrunch rows (two small all-gathers), its
 * diagnostics rows with the row owners (one all-to-all), the row medians/MADs
 * (one all-gather of 8*rows doubles) and the convergence counters (one
 * all-reduce).  Results are bit-identical to an
 * unsharded session.  world must be a power of two <= the number of 256-channel
 * super-blocks.
 *
 * A shard session takes the GLOBAL shape in ic_params; ic_upload /
 * ic_upload_device take the shard's channel slice: cube [nsub][nchan_loc][nbin],
 * w0 [nsub][nchan_loc], shift [nchan_loc]; per-profile outputs of ic_run and
 * the ic_get_* calls are the shard's [nsub][nchan_loc] slice, while loops,
 * changed and nzero are global.  Every shard of a group must call ic_run
 * together (collectives inside).
 * ------------------------------------------------------------------------ */

/* Channel ranges [chan_ranges[2r], chan_ranges[2r+1]) and row ranges of every
 * rank (arrays of 2*world int32). */
int ic_shard_layout(int nsub, int nchan, int world, int32_t *chan_ranges, int32_t *row_ranges);

/* Host-provided transport (one process per GPU; e.g. torch.distributed over
 * RCCL/xGMI).  All exchange buffers are obtained through alloc() so that the
 * host owns them.  Collectives are issued in stream order on `stream` (the
 * session's hipStream_t) and return 0 on success.
 *   allgather:  recv[r*bytes .. (r+1)*bytes) = rank r's send, every r
 *   alltoallv:  send = blocks for ranks 0..world-1 (send_bytes[r] each, back to
 *               back); recv = blocks from ranks 0..world-1 (recv_bytes[r])
 *   allreduce_sum_i32: in place */
typedef struct {
    void *ctx;
    int (*alloc)(void *ctx, size_t bytes, void **dev_ptr);
    int (*release)(void *ctx, void *dev_ptr);
    int (*allgather)(void *ctx, const void *send, void *recv, size_t bytes, void *stream);
    int (*alltoallv)(void *ctx, const void *send, const size_t *send_bytes, void *recv,
                     const size_t *recv_bytes, void *stream);
    int (*allreduce_sum_i32)(void *ctx, int32_t *buf, size_t n, void *stream);
} ic_comm_ops;

/* Shard `rank` of `world` on HIP device `device`, exchanging through `ops`
 * (copied; ops->ctx must outlive the session). */
int ic_session_create_shard(const ic_params *params, int device, int rank, int world, const ic_comm_ops *ops,
                            void **session);

/* Native RCCL transport (one process per GPU, RCCL over xGMI): rank 0 calls
 * ic_rccl_unique_id and the host hands the 128 id bytes to every rank once
 * (e.g. through the torch.distributed store); each rank then creates its shard
 * with them on its own device.  Every exchange is an RCCL collective (all-to-all
 * as grouped sends / receives) issued by the library on the session stream: no
 * host callback per exchange.  A failing shard aborts its communicator and
 * returns its error; a peer learns of it from RCCL (an error from its own
 * collective, or RCCL's asynchronous error while the library waits on the
 * GPU: IC_ECOMM), or at worst from IC_OPT_SYNC_TIMEOUT_MS (IC_EHIP).
 * The communicator is created non-blocking and polled: a rank that never
 * joins (it failed before ic_session_create_rccl) makes its peers' creation
 * fail with IC_ECOMM after the init timeout instead of blocking them forever.
 * librccl is loaded on first use (/opt/rocm/lib/librccl.so.1); IC_ECOMM if it
 * is missing. */
int ic_rccl_unique_id(void *id_out /* 128 bytes */);
int ic_session_create_rccl(const ic_params *params, int device, int rank, int world, const void *unique_id,
                           void **session);
/* The librccl file to load instead of the ROCm install's (another RCCL build,
 * or a test stub exporting the same nccl* symbols); NULL restores the
 * default.  Process-wide; must precede the first RCCL use of the process
 * (IC_ESTATE after it, unless the path is the one already loaded). */
int ic_rccl_set_library(const char *path);
/* How long ic_session_create_rccl waits for every rank to join, in ms (>= 1;
 * process-wide; default 600000). */
int ic_rccl_set_init_timeout(int64_t ms);

/* In-process shard group: `world` shards driven by `world` host threads of one
 * process (one or several devices), exchanging by device-to-device / peer
 * copies.  Destroy the group after all its sessions. */
int ic_group_create(int world, void **group);
void ic_group_destroy(void *group);
int ic_session_create_grouped(const ic_params *params, int device, void *group, int rank, void **session);

#ifdef __cplusplus
}
#endif
#endif /* ITERATIVE_CLEANER_H */
