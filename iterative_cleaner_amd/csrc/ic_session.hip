// ic_session.hip — host side of libicgpu.so: the C-ABI declared in
// include/iterative_cleaner.h.  Owns device buffers and the HIP stream of a
// session, prepares the fit cube at the start of every run, and drives the cleaning
// loop of iterative_cleaner.py:83-146 (one launch sequence per iteration and
// one small device->host read of the convergence counters).  A channel shard
// (ic_session_create_shard / _grouped) runs the same sequence on its channel
// slice with four exchanges per iteration through a Comm (ic_comm.h).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <sched.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/iterative_cleaner.h"
#include "ic_comm.h"
#include "ic_internal.h"

using namespace icgpu;

namespace icgpu {
thread_local PendingTiming g_timing;
}

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// calls on a session whose host wait timed out (Session::failed)
int failed_session()
{
    return fail(IC_ESTATE, "session failed: a host wait timed out with its kernels possibly still running; destroy it");
}

#define CK(call)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(IC_EHIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                \
    } while (0)

const char *kKernelNames[K_COUNT] = {"k_chan_partials", "k_window",    "k_base",
                                     "k_fscrunch",      "k_tscrunch",  "k_fit_pass", "k_fit_state",
                                     "k_diag",          "k_linestats", "k_combine",  "k_residual",
                                     "k_fit_tail",      "k_sb_tree",   "k_shard_pack", "exchange",
                                     "k_tnorm",         "k_rotate"};

constexpr long kTailProfiles = 8192;  // default: hand the remaining profiles to k_fit_tail below this
constexpr long kTailProfilesLarge = 4096;   // the same for sessions of >= 2^20 profiles
constexpr long kTailProfilesLong = 12288;   // smaller sessions of >= 2048-bin profiles

struct Timed {
    int kid;
    hipEvent_t a, b;
};

struct Session {
    ic_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    size_t P = 0, N = 0, Ppad = 0;
    int ldD = 0;                // fit-cube row stride (bins, padded to kFitTile)
    int nsb = 0, width = 0;
    bool uploaded = false, ran = false;
    int last_iter = 0;
    // channel shard (unsharded: world == 1, comm == nullptr, nchan == p.nchan)
    int rank = 0, world = 1;
    Comm *comm = nullptr;
    int nchan = 0;                  // channels of this session (local slice)
    int c0 = 0;                     // its first global channel
    ShardGeom geom{};
    SbPlan plan_sb{};               // the session's super-blocks
    SbPlan plan_top{};              // the shard roots (world leaves)
    int rows_own = 0, rows_pad = 0;
    double *xw_send = nullptr, *xw_recv = nullptr;          // window-total roots -> row owners
    double *xf_send = nullptr, *xf_recv = nullptr;          // fscrunch + weight roots -> row owners
    int32_t *xwg_send = nullptr, *xwg_recv = nullptr;       // owners' windows, all-gathered
    float *xfg_send = nullptr, *xfg_recv = nullptr;         // owners' fscrunch rows, all-gathered
    int wg_blk = 0;                                          // ints per rank in xwg (rows_pad, even)
    long fg_blk = 0;                                         // floats per rank in xfg (even)
    std::vector<size_t> wsb, wrb, fsb, frb;                 // block bytes: window / fscrunch roots
    unsigned char *xd_send = nullptr, *xd_recv = nullptr;   // diagnostics / valid rows
    double *xr_send = nullptr, *xr_recv = nullptr;          // row medians / MADs
    std::vector<size_t> dsb, drb, vsb, vrb;                 // block bytes: diag, valid
    double *std_r = nullptr, *mean_r = nullptr, *fft_r = nullptr;   // owned rows [rows_own][nchan_g]
    double *ptp_r = nullptr;
    uint8_t *valid_r = nullptr;
    // device buffers
    float *raw = nullptr, *D = nullptr, *w0 = nullptr, *W = nullptr, *base = nullptr, *base0 = nullptr;
    // input slots (raw/w0/shift alias slot `cur`); slot 1 is allocated by the first
    // ic_upload_async that needs it.  Pending async uploads queue in `fifo`.
    float *slot_raw[2] = {nullptr, nullptr}, *slot_w0[2] = {nullptr, nullptr};
    int32_t *slot_shift[2] = {nullptr, nullptr};
    hipEvent_t slot_ev[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr;
    int cur = 0, fifo[2] = {0, 0}, fifo_n = 0;
    bool ever_uploaded = false;
    float *F = nullptr, *wf = nullptr, *T = nullptr, *hist = nullptr;
    double *ptp = nullptr;      // f64 storage; f32 values unless p.data_f64
    uint8_t *valid = nullptr;
    int32_t *shift = nullptr, *win = nullptr, *wflag = nullptr, *info = nullptr, *counters = nullptr;
    double *part = nullptr, *part2 = nullptr, *wpart = nullptr, *T64 = nullptr, *amp = nullptr, *std_ = nullptr,
           *mean = nullptr, *fft = nullptr, *test = nullptr, *lstat = nullptr, *TT = nullptr,
           *T2 = nullptr;   // [2 nbin]: the template twice (k_diag_cl)
    double2 *tw = nullptr, *tw_p2 = nullptr;
    PwPlan *plan = nullptr;
    FitStateArrays fs{};
    int32_t *lists = nullptr;   // two active-profile lists of P entries
    int32_t *rcount = nullptr;  // round counters (ic_internal.h kRoundWords) + the tail's sweep counter
    int32_t *h_rcount = nullptr;  // host-mapped mirror, written by k_fit_state's last block
    int32_t *h_small = nullptr;   // pinned readback of the per-iteration counters and run stats
                                  // (a pageable D2H copy is staged synchronously, ~30 us each)
    int32_t *d_h_rcount = nullptr;  // its device address
    void *fs_block = nullptr;   // one allocation backing fs
    int fit_rounds = 0;
    int plan_ub = 0;            // max(leaves, ops) of the pairwise plan (k_tnorm scratch)
    LineStatsArgs ls_knobs;     // row-median form (IC_OPT_ROWSTAT_*)
    long tail_threshold = kTailProfiles;   // IC_OPT_FIT_TAIL
    bool diag_chain = true;     // IC_OPT_DIAG_CHAIN: k_diag_cl at nbin 1024/2048/4096
    double sync_timeout_s = 600.0;   // IC_OPT_SYNC_TIMEOUT_MS
    // a host wait timed out with kernels of this session possibly still in
    // flight: every later call but ic_session_destroy fails (IC_ESTATE), and
    // destroy leaks the device buffers instead of freeing memory in use
    bool failed = false;
    bool comm_lost = false;   // ... because the transport reported a lost peer
    // diagnostics forked onto a second stream (exact fit): the state kernel
    // of round diag_fork (0 = off) flags the profiles still fitting; from
    // round diag_fork + fork_delay on the others are measured on dstream while
    // the fit's latency-bound late rounds and tail run, the flagged ones on
    // the main stream once the fit is done.  C2, one MI355X, same box (ms per
    // clean): no fork 28.70-28.77, fork 3 / delay 1 27.99-28.06, 3 / 0
    // 28.53-28.61, 3 / 2 28.41-28.46, 4 / 0 28.01-28.19, 4 / 1 28.45-28.52
    int diag_fork = 3;
    int pr_lo = 0, pr_hi = 0;   // this run's clamped pulse region (the FFT mode's forked residual rotation)
    // incremental template stage (integer dedispersion, iteration >= 2):
    // column exactness flags [nsub][nsb][nbin] of part (exA, set once per run
    // by prepare) and part2 (exF, set by every full fscrunch pass);
    // k_chan_delta then moves the sums through the changed channels only
    bool incr = true;
    uint8_t *exA = nullptr, *exF = nullptr;
    hipStream_t dstream = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    uint8_t *late = nullptr;       // [P] 1: still fitting after round diag_fork (pass A skips them)
    int fork_round = -1;           // this iteration's fork round (-1: none)
    // the second fork (run_fit): the tail's list, marked in tmark, measured after the fit
    bool tail_split = false;
    // FFT mode: the residual's rotation measures its rows itself (k_rotate's
    // statistics epilogue, nbin 1024) instead of a k_diag STATS pass over R
    // (IC_OPT_ROT_STATS)
    bool rot_stats = true;
    int tail_split_mode = IC_TAIL_SPLIT_AUTO;   // IC_OPT_TAIL_SPLIT
    const int32_t *tail_list = nullptr;
    const unsigned long long *tail_cin = nullptr;
    long tail_bound = 0;
    uint8_t *tmark = nullptr;
    hipEvent_t fork2_ev = nullptr;
    int fork_delay = 1;            // rounds between the flags and pass A (IC_OPT_FORK_DELAY)
    ic_run_stats stats{};
    std::vector<int32_t> bad_fits;   // per iteration of the last run: fit statuses outside 1-4
    // fractional dedispersion (dedisp_mode IC_DEDISP_FFT): the dedispersed raw
    // cube rot(raw), the template stage's rot(f32(raw - base)) (carried rows),
    // the residual scratch, zero shifts/levels for the shift-indexed kernels,
    // and the phasor table [nchan][nbin/2 + 1] of ic_set_delays
    bool fftded = false, delays_set = false;
    int dtiled = 0;                  // fit cube D in the tiled layout (dt_ofs)
    float *dr = nullptr, *Tc = nullptr, *R = nullptr, *zbase = nullptr;
    int32_t *zshift = nullptr;
    float *ph = nullptr;   // f32 pairs
    double *delay2 = nullptr;        // [P] per-profile delays (ic_set_delays2), else nullptr
    // timing
    bool timing = false;
    int timing_only = -1;            // >= 0: time only this kernel id
    std::vector<Timed> events;
    std::vector<hipEvent_t> epool;   // reused across runs: no hipEventCreate in the timed region
    hipEvent_t sev = nullptr;        // spin_sync's marker
    size_t enext = 0;
    double kms[K_COUNT] = {0};
    int klaunch[K_COUNT] = {0};
};

template <typename T>
hipError_t dalloc(T **p, size_t n)
{
    return hipMalloc((void **)p, n * sizeof(T) + 16);
}

// numpy pairwise plan (loops_utils.h.src): leaves <= 128 in address order
int plan_build(std::vector<int> &ls, std::vector<int> &ll, std::vector<int> &oa, std::vector<int> &ob,
               int start, int n)
{
    if (n <= 128) {
        ls.push_back(start);
        ll.push_back(n);
        return (int)ls.size() - 1;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    const int a = plan_build(ls, ll, oa, ob, start, n2);
    const int b = plan_build(ls, ll, oa, ob, start + n2, n - n2);
    oa.push_back(a);
    ob.push_back(b);
    return -(int)oa.size();  // op o encoded as -(o+1)
}

int make_plan(int n, PwPlan *pl)
{
    std::vector<int> ls, ll, oa, ob;
    const int root = plan_build(ls, ll, oa, ob, 0, n);
    if ((int)ls.size() > kMaxLeaves || (int)oa.size() > kMaxLeaves) return -1;
    memset(pl, 0, sizeof *pl);
    pl->n = n;
    pl->nleaf = (int)ls.size();
    pl->nops = (int)oa.size();
    auto slot = [&](int id) { return id >= 0 ? id : pl->nleaf + (-id - 1); };
    for (int q = 0; q < pl->nleaf; ++q) {
        pl->leaf_start[q] = ls[q];
        pl->leaf_len[q] = ll[q];
    }
    for (int q = 0; q < pl->nops; ++q) {
        pl->op_a[q] = slot(oa[q]);
        pl->op_b[q] = slot(ob[q]);
    }
    pl->root = slot(root);
    return 0;
}

// timing events come from a per-session pool (created on first use, reused
// once collect_timing has read them)
static hipError_t take_event(Session *s, hipEvent_t *e)
{
    if (s->enext == s->epool.size()) {
        hipEvent_t n = nullptr;
        const hipError_t rc = hipEventCreate(&n);
        if (rc != hipSuccess) return rc;
        s->epool.push_back(n);
    }
    *e = s->epool[s->enext++];
    return hipSuccess;
}

// Wait for an event by polling it (the blocking wait's wake-up cost ~0.1 ms
// per iteration boundary on the MI355X hosts): a busy poll for the first
// 200 us (the common case: the GPU is a few kernels behind), then polls with
// sched_yield between them, so a long wait does not hold a host core; after
// the session's sync timeout (IC_OPT_SYNC_TIMEOUT_MS, default 600 s) it gives
// up with hipErrorLaunchTimeOut and marks the session failed, so a kernel
// that never finishes fails the run instead of hanging its caller, and no
// later call reuses buffers its kernels may still be using.
static const auto kBusyPoll = std::chrono::microseconds(200);
static hipError_t poll_event(Session *s, hipEvent_t ev)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto spin = kBusyPoll;
    const auto limit = std::chrono::duration<double>(s->sync_timeout_s);
    hipError_t e;
    unsigned n = 0;
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
        const auto dt = clk::now() - t0;
        if (dt > limit) {
            s->failed = true;
            return hipErrorLaunchTimeOut;
        }
        if (dt > spin) {
            sched_yield();
            // a peer lost by the transport (RCCL's asynchronous error): the
            // kernels queued behind its collective may never run
            if (s->comm && (++n & 255) == 0 && s->comm->remote_error()) {
                s->failed = true;
                s->comm_lost = true;
                return hipErrorLaunchTimeOut;
            }
        }
    }
    return e;
}

// Wait for a round's survivor count, which k_fit_state's last block publishes
// into host-mapped memory (a system-scope release store): the same polling as
// poll_event, on the value itself, so the round needs no event (a marker packet
// between the state kernel and the next sweep costs ~7 us per round boundary)
static hipError_t poll_count(Session *s, const int32_t *cnt)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto spin = kBusyPoll;
    const auto limit = std::chrono::duration<double>(s->sync_timeout_s);
    unsigned n = 0;
    while (__atomic_load_n(cnt, __ATOMIC_ACQUIRE) < 0) {
        const auto dt = clk::now() - t0;
        if (dt > limit) {
            s->failed = true;
            return hipErrorLaunchTimeOut;
        }
        if (dt > spin) {
            sched_yield();
            if (s->comm && (++n & 255) == 0 && s->comm->remote_error()) {
                s->failed = true;
                s->comm_lost = true;
                return hipErrorLaunchTimeOut;
            }
        }
    }
    return hipSuccess;
}

static hipError_t spin_sync(Session *s)
{
    hipError_t e = hipEventRecord(s->sev, s->stream);
    if (e != hipSuccess) return e;
    return poll_event(s, s->sev);
}

// Timed launches go through the dispatch packet (g_timing, ic_internal.h):
// no marker packets around them.  A wrapper that launched nothing drops its
// events; one that launched several kernels ends the interval with a marker.
#define LAUNCH(S, KID, CALL) LAUNCH_ON(S, KID, (S)->stream, CALL)
#define LAUNCH_ON(S, KID, ST, CALL)                                            \
    do {                                                                       \
        Timed t_{KID, nullptr, nullptr};                                       \
        const bool tm_ = (S)->timing && ((S)->timing_only < 0 || (S)->timing_only == (KID)); \
        if (tm_) {                                                             \
            CK(take_event((S), &t_.a));                                        \
            CK(take_event((S), &t_.b));                                        \
            g_timing = PendingTiming{t_.a, t_.b, 0, 0};                        \
        }                                                                      \
        const hipError_t lc_ = (CALL);                                         \
        const PendingTiming pt_ = g_timing;                                    \
        g_timing = PendingTiming{};                                            \
        CK(lc_);                                                               \
        if (tm_ && pt_.used) {                                                 \
            if (pt_.extra) CK(hipEventRecord(t_.b, (ST)));                     \
            (S)->events.push_back(t_);                                         \
        } else if (tm_) {                                                      \
            (S)->enext -= 2;   /* nothing launched: the pair goes back */      \
        }                                                                      \
    } while (0)

// Twiddles of k_diag_p2 for nbin = N = 2^k: [M = N/2] exp(-2 pi i q/N) for the
// real-FFT post-processing, then for every Stockham stage after the first (radix
// R = 8 while >= 3 levels remain, then 4 or 2; Ns = product of earlier radices)
// the table w^(r k), w = exp(-2 pi i/(R Ns)), k < Ns, r = 1..R-1, as [k][r-1].
// Total <= N entries.
std::vector<double2> p2_twiddles(int N)
{
    std::vector<double2> t;
    if (N < 4 || (N & (N - 1))) return t;
    const long double pi = 3.141592653589793238462643383279502884L;
    auto w = [&](long double num, long double den) {
        const long double a = -2.0L * pi * num / den;
        return make_double2((double)cosl(a), (double)sinl(a));
    };
    const int M = N / 2;
    for (int q = 0; q < M; ++q) t.push_back(w(q, N));
    int lg = 0;
    while ((1 << lg) < M) ++lg;
    for (int done = 0, Ns = 1; done < lg;) {
        const int rem = lg - done, R = rem >= 3 ? 8 : (rem == 2 ? 4 : 2);
        if (Ns > 1)
            for (int k = 0; k < Ns; ++k)
                for (int r = 1; r < R; ++r) t.push_back(w((long double)r * k, (long double)R * Ns));
        Ns *= R;
        done += R == 8 ? 3 : (R == 4 ? 2 : 1);
    }
    return t;
}

int collect_timing(Session *s)
{
    if (s->events.empty()) return 0;
    CK(hipStreamSynchronize(s->stream));
    for (auto &e : s->events) {
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e.a, e.b));
        s->kms[e.kid] += ms;
        s->klaunch[e.kid] += 1;
    }
    s->events.clear();
    s->enext = 0;
    return 0;
}

void free_all(Session *s)
{
    for (int q = 0; q < 2; ++q) {
        void *sb[] = {s->slot_raw[q], s->slot_w0[q], s->slot_shift[q]};
        for (void *b : sb)
            if (b) (void)hipFree(b);
        if (s->slot_ev[q]) (void)hipEventDestroy(s->slot_ev[q]);
    }
    if (s->copy_stream) (void)hipStreamDestroy(s->copy_stream);
    if (s->dstream) (void)hipStreamDestroy(s->dstream);
    if (s->fork_ev) (void)hipEventDestroy(s->fork_ev);
    if (s->join_ev) (void)hipEventDestroy(s->join_ev);
    if (s->fork2_ev) (void)hipEventDestroy(s->fork2_ev);
    void *bufs[] = {s->late, s->exA, s->exF, s->D,     s->W,   s->base, s->base0, s->F,   s->wf,
                    s->T,    s->ptp,   s->hist, s->valid, s->win, s->info, s->comm ? nullptr : s->counters,
                    s->part, s->wpart, s->T64,  s->amp, s->std_, s->mean, s->fft,  s->test,
                    s->lstat, s->tw,   s->plan, s->fs_block, s->lists, s->rcount, s->tw_p2, s->part2,
                    s->wflag, s->TT, s->dr, s->Tc, s->R, s->zbase, s->zshift, s->ph, s->T2, s->fs.U, s->tmark,
                    s->delay2};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    void *rbufs[] = {s->std_r, s->mean_r, s->fft_r, s->ptp_r, s->valid_r};
    for (void *b : rbufs)
        if (b) (void)hipFree(b);
    if (s->comm) {
        void *xbufs[] = {s->xw_send, s->xw_recv, s->xf_send, s->xf_recv, s->xwg_send, s->xwg_recv, s->xfg_send,
                         s->xfg_recv, s->xd_send, s->xd_recv, s->xr_send, s->xr_recv, s->counters};
        for (void *b : xbufs)
            if (b) s->comm->release(b);
        s->counters = nullptr;
        delete s->comm;
        s->comm = nullptr;
    }
    if (s->h_rcount) (void)hipHostFree(s->h_rcount);
    if (s->h_small) (void)hipHostFree(s->h_small);
    if (s->sev) (void)hipEventDestroy(s->sev);
    for (auto &e : s->epool) (void)hipEventDestroy(e);
    s->epool.clear();
    s->events.clear();
    if (s->stream) (void)hipStreamDestroy(s->stream);
}

__global__ void k_valid(const float *w0, uint8_t *valid, float *W, float *hist0, size_t P)
{
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < P) {
        const float w = w0[k];
        valid[k] = (w != 0.0f);
        W[k] = w;
        hist0[k] = w;
    }
}

#define CM(S, call, what)                                                                         \
    do {                                                                                          \
        Timed t_{K_EXCHANGE, nullptr, nullptr};                                                   \
        const bool tm_ = (S)->timing && ((S)->timing_only < 0 || (S)->timing_only == K_EXCHANGE); \
        if (tm_) {                                                                                \
            CK(take_event((S), &t_.a));                                                           \
            CK(take_event((S), &t_.b));                                                           \
            CK(hipEventRecord(t_.a, (S)->stream));                                                \
        }                                                                                         \
        const int rc_ = (call);                                                                   \
        if (tm_) {                                                                                \
            CK(hipEventRecord(t_.b, (S)->stream));                                                \
            (S)->events.push_back(t_);                                                            \
        }                                                                                         \
        if (rc_ != 0) {                                                                           \
            (S)->comm->abort();                                                                   \
            return fail(IC_ECOMM, "shard %d/%d: %s exchange failed (%d)", (S)->rank, (S)->world,  \
                        what, rc_);                                                               \
        }                                                                                         \
    } while (0)

// Halving-tree plan (archive.py sb_tree) as a post-order stack program.
void sb_plan_rec(int lo, int hi, uint8_t *merges)
{
    if (hi - lo == 1) return;
    const int mid = lo + (hi - lo) / 2;
    sb_plan_rec(lo, mid, merges);
    sb_plan_rec(mid, hi, merges);
    merges[hi - 1]++;
}

SbPlan make_sb_plan(int n)
{
    SbPlan pl;
    memset(&pl, 0, sizeof pl);
    pl.n = n;
    if (n >= 1 && n <= kMaxSbLeaves) sb_plan_rec(0, n, pl.merges);
    return pl;
}

// shards.py channel_shards / row_owners; 0 or an error message
const char *shard_layout(int nsub, int nchan, int world, int32_t *chan0, int32_t *row0)
{
    if (world < 1 || (world & (world - 1))) return "world size must be a power of two";
    if (world > kMaxShards) return "world size too large";
    const int nsb = (nchan + kSuperBlock - 1) / kSuperBlock;
    if (nsb < world) return "fewer 256-channel super-blocks than shards";
    int depth = 0;
    while ((1 << depth) < world) ++depth;
    for (int r = 0; r < world; ++r) {
        int lo = 0, hi = nsb;
        for (int d = depth - 1; d >= 0; --d) {
            const int mid = lo + (hi - lo) / 2;
            if ((r >> d) & 1)
                lo = mid;
            else
                hi = mid;
        }
        chan0[2 * r] = lo * kSuperBlock;
        chan0[2 * r + 1] = std::min(hi * kSuperBlock, nchan);
        row0[2 * r] = (int)((long)r * nsub / world);
        row0[2 * r + 1] = (int)((long)(r + 1) * nsub / world);
    }
    return nullptr;
}

// Window stage: per-subint window from the W-weighted total of `part`
// (unsharded: combine the super-blocks).  Sharded: reduce the local
// super-blocks to this shard's root, send each subint's root row to the rank
// that owns the row (all-to-all), the owner combines the world's roots in
// canonical order and searches the window, and the owners' windows are
// all-gathered (4 B per subint) - each root crosses the fabric once.
int window_stage(Session *s, int32_t *flags)
{
    const int nsub = s->p.nsub, nbin = s->p.nbin;
    if (!s->comm) {
        LAUNCH(s, K_WINDOW, launch_window(s->stream, s->part, (long)s->nsb * nbin, nbin, s->plan_sb, nsub, nbin,
                                          s->width, s->win, flags));
        return 0;
    }
    LAUNCH(s, K_SB_TREE, launch_sb_tree(s->stream, s->part, nullptr, s->plan_sb, nsub, nbin, nbin, s->xw_send));
    CM(s, s->comm->alltoallv(s->xw_send, s->wsb.data(), s->xw_recv, s->wrb.data(), s->stream), "window roots");
    if (s->rows_own > 0)
        LAUNCH(s, K_WINDOW, launch_window(s->stream, s->xw_recv, nbin, (long)s->rows_own * nbin, s->plan_top,
                                          s->rows_own, nbin, s->width, s->xwg_send, nullptr));
    CM(s, s->comm->allgather(s->xwg_send, s->xwg_recv, sizeof(int32_t) * s->wg_blk, s->stream), "windows");
    LAUNCH(s, K_SHARD_PACK, launch_unpack_windows(s->stream, s->geom, s->wg_blk, s->xwg_recv, s->win, flags));
    return 0;
}

// fscrunch + tscrunch from part2/wpart (sharded as window_stage: root rows of
// nbin + 1 doubles to the row owners, owners' F rows + wf all-gathered)
int scrunch_stage(Session *s)
{
    const int nsub = s->p.nsub, nbin = s->p.nbin;
    if (!s->comm) {
        LAUNCH(s, K_FSCRUNCH, launch_fscrunch(s->stream, s->part2, (long)s->nsb * nbin, nbin, s->wpart, s->nsb, 1,
                                              s->plan_sb, nsub, nbin, s->F, s->wf));
    } else {
        const long row = nbin + 1, own = (long)s->rows_own * row;
        LAUNCH(s, K_SB_TREE, launch_sb_tree(s->stream, s->part2, s->wpart, s->plan_sb, nsub, nbin, row, s->xf_send));
        CM(s, s->comm->alltoallv(s->xf_send, s->fsb.data(), s->xf_recv, s->frb.data(), s->stream), "fscrunch roots");
        if (s->rows_own > 0)
            LAUNCH(s, K_FSCRUNCH, launch_fscrunch(s->stream, s->xf_recv, row, own, s->xf_recv + nbin, row, own,
                                                  s->plan_top, s->rows_own, nbin, s->xfg_send,
                                                  s->xfg_send + (size_t)s->rows_pad * nbin));
        CM(s, s->comm->allgather(s->xfg_send, s->xfg_recv, sizeof(float) * s->fg_blk, s->stream), "fscrunch rows");
        LAUNCH(s, K_SHARD_PACK, launch_unpack_fscrunch(s->stream, s->geom, s->rows_pad, s->fg_blk, nbin, s->xfg_recv,
                                                       s->F, s->wf));
    }
    LAUNCH(s, K_TSCRUNCH, launch_tscrunch(s->stream, s->F, s->wf, nsub, nbin, s->T, s->T64, s->T2));
    return 0;
}

// phasor table f32(ic_phasor(k, delay[c], nbin)), k <= nbin/2, as f32 pairs
// (phase_rotation.py phasors; oracle orc_phasors; the rotation computes in
// f32): the same function the per-profile kernel evaluates on the device and
// rounds, so a table row and a profile with that delay agree
std::vector<float> make_phasors(int nbin, int nchan, const double *delay)
{
    const int m = nbin / 2;
    std::vector<float> ph(2 * (size_t)nchan * (m + 1));
    for (int c = 0; c < nchan; ++c)
        for (int k = 0; k <= m; ++k) {
            const double2 v = ic_phasor(k, delay[c], nbin);
            ph[2 * ((size_t)c * (m + 1) + k)] = (float)v.x;
            ph[2 * ((size_t)c * (m + 1) + k) + 1] = (float)v.y;
        }
    return ph;
}

RotateArgs rotate_args(Session *s, const float *in, const float *base, int sign, const int32_t *flags, float *out,
                       long ldo)
{
    RotateArgs a{};
    a.in = in;
    a.ld_in = s->p.nbin;
    a.base = base;
    a.ph = s->ph;
    a.delay2 = s->delay2;
    // an archive stored dedispersed: its dedisperse is a no-op (archive.py),
    // only the residual's dededisperse rotates
    a.identity = sign > 0 && s->p.input_dedispersed;
    a.sign = sign;
    a.tw = s->tw;
    a.tw_p2 = s->tw_p2;
    a.flags = flags;
    a.nsub = s->p.nsub;
    a.nchan = s->nchan;
    a.nbin = s->p.nbin;
    a.out = out;
    a.ldo = ldo;
    return a;
}

// the iteration's residual rows f32(a T - D) (remove_profile1d, ic.py:277-288),
// rotated back to the dispersed frame (dededisperse, ic.py:104) -> s->R
RotateArgs residual_rotate_args(Session *s, int pr_start, int pr_end)
{
    RotateArgs a = rotate_args(s, s->D, nullptr, -1, nullptr, s->R, s->p.nbin);
    a.ld_in = s->ldD;
    a.T64 = s->T64;
    a.amp = s->amp;
    a.info = s->info;
    a.pr_on = s->p.pr_on;
    a.pr_factor = s->p.pr_factor;
    a.pr_start = pr_start;
    a.pr_end = pr_end;
    a.in_tiled = s->dtiled;
    return a;
}

// the FFT mode's residual rotation also computes comprehensive_stats of its rows
// (no R, no DIAG_STATS pass): when the option is on and the kernel serves nbin
bool rot_stats_on(const Session *s)
{
    return s->fftded && s->rot_stats && rotate_stats_supported(s->p.nbin, s->p.data_f64 != 0);
}
void with_stats(Session *s, RotateArgs &a)
{
    a.out = nullptr;
    a.w0 = s->w0;
    a.tw_p2 = s->tw_p2;
    a.std_o = s->std_;
    a.mean_o = s->mean;
    a.ptp_o = s->ptp;
    a.fft_o = s->fft;
}

// fit-cube preparation (iterative_cleaner.py:96-100): baseline with w0, dedisperse.
// The w0 baseline (window + per-profile levels) is also the template stage's
// baseline of the first iteration (W == w0).  A shard also hands the validity
// of its profiles to the row owners (static for the whole run).
int prepare(Session *s)
{
    const int nsub = s->p.nsub, nchan = s->nchan, nbin = s->p.nbin;
    IC_GGL(k_valid, dim3((unsigned)((s->P + 255) / 256)), dim3(256), 0, s->stream, s->w0,
                       s->valid, s->W, s->hist, s->P);
    CK(hipGetLastError());
    if (s->comm) {
        LAUNCH(s, K_SHARD_PACK,
               launch_pack_rows(s->stream, s->geom, nchan, nullptr, nullptr, nullptr, nullptr, s->valid, s->xd_send));
        CM(s, s->comm->alltoallv(s->xd_send, s->vsb.data(), s->xd_recv, s->vrb.data(), s->stream), "valid rows");
        LAUNCH(s, K_SHARD_PACK,
               launch_assemble_rows(s->stream, s->geom, s->xd_recv, nullptr, nullptr, nullptr, nullptr, s->valid_r));
    }
    if (s->fftded) {
        // remove_baseline reads the dedispersed view rot(raw) (archive.py
        // _ded_view); dedisperse then rotates the data it leaves, f32(raw - base0):
        // that is the fit cube D and iteration 1's template rows Tc (W == w0)
        LAUNCH(s, K_ROTATE, launch_rotate(s->stream, rotate_args(s, s->raw, nullptr, +1, nullptr, s->dr, nbin)));
        LAUNCH(s, K_CHAN_PARTIALS,
               launch_chan_partials(s->stream, 0, s->dr, s->w0, s->zshift, nullptr, nullptr, nsub, nchan, nbin,
                                    s->part, nullptr, nullptr, nullptr, 0, 0, s->exA, nullptr));
        if (int rc = window_stage(s, nullptr)) return rc;
        LAUNCH(s, K_BASE,
               launch_base(s->stream, s->dr, s->zshift, s->win, nullptr, nsub, nchan, nbin, s->width, s->base0));
        RotateArgs ra = rotate_args(s, s->raw, s->base0, +1, nullptr, s->Tc, nbin);
        ra.out2 = s->D;
        ra.ldo2 = s->ldD;
        ra.out2_tiled = s->dtiled;
        LAUNCH(s, K_ROTATE, launch_rotate(s->stream, ra));
        CK(hipMemcpyAsync(s->base, s->base0, sizeof(float) * s->P, hipMemcpyDeviceToDevice, s->stream));
        CK(hipMemsetAsync(s->wflag + nsub, 0, sizeof(int32_t), s->stream));
        return 0;
    }
    LAUNCH(s, K_CHAN_PARTIALS,
           launch_chan_partials(s->stream, 0, s->raw, s->w0, s->shift, nullptr, nullptr, nsub, nchan, nbin, s->part,
                                nullptr, nullptr, nullptr, 0, 0, s->exA, nullptr));
    if (int rc = window_stage(s, nullptr)) return rc;
    LAUNCH(s, K_BASE,
           launch_base(s->stream, s->raw, s->shift, s->win, nullptr, nsub, nchan, nbin, s->width, s->base0));
    // the fit cube D = f32(ded - base0) is written by iteration 1's template
    // pass (chan_partials mode 3), which reads the same values
    CK(hipMemcpyAsync(s->base, s->base0, sizeof(float) * s->P, hipMemcpyDeviceToDevice, s->stream));
    CK(hipMemsetAsync(s->wflag + nsub, 0, sizeof(int32_t), s->stream));
    return 0;
}

// Template of iteration `iter` (iterative_cleaner.py:88-94): remove_baseline
// with the current weights W, dedisperse, fscrunch, tscrunch.  The baseline
// level of a profile depends on W only through its subint's window (the window
// position is the argmin over the W-weighted total; the level is the raw
// window mean), so s->base/s->win carry over between iterations: one read of
// the cube computes the W-weighted total AND the fscrunch partials with the
// carried baseline; subints whose window moved get their levels and partials
// recomputed (flagged launches that are empty when nothing moved).
int iteration_template(Session *s, int iter)
{
    const int nsub = s->p.nsub, nchan = s->nchan, nbin = s->p.nbin;
    if (s->fftded) {
        // FFT dedispersion: the window totals and levels read rot(raw); the rows
        // rot(f32(raw - base)) of subints whose window moved are re-rotated, and
        // the fscrunch partials are taken over those rows (no shift, no level).
        // Incremental (IC_OPT_TEMPLATE_INCR): both sums move through the changed
        // channels (k_chan_delta, part from rot(raw), part2 from the rows), the
        // subints whose window moved are summed again after their re-rotation.
        const bool incr = iter > 1 && s->incr;
        if (iter > 1) {
            if (incr) {
                const float *Wo = s->hist + (size_t)(iter - 2) * s->P;
                LAUNCH(s, K_CHAN_PARTIALS,
                       launch_chan_delta(s->stream, s->dr, s->zshift, s->zbase, s->W, Wo, nsub, nchan, nbin, s->part,
                                         s->part2, s->wpart, s->exA, s->exF, s->Tc));
            } else {
                LAUNCH(s, K_CHAN_PARTIALS,
                       launch_chan_partials(s->stream, 0, s->dr, s->W, s->zshift, nullptr, nullptr, nsub, nchan, nbin,
                                            s->part, nullptr, nullptr, nullptr, 0, 0, s->exA, nullptr));
            }
            if (int rc = window_stage(s, s->wflag)) return rc;
            LAUNCH(s, K_BASE,
                   launch_base(s->stream, s->dr, s->zshift, s->win, s->wflag, nsub, nchan, nbin, s->width, s->base));
            LAUNCH(s, K_ROTATE,
                   launch_rotate(s->stream, rotate_args(s, s->raw, s->base, +1, s->wflag, s->Tc, nbin)));
        }
        LAUNCH(s, K_CHAN_PARTIALS,
               launch_chan_partials(s->stream, 1, s->Tc, s->W, s->zshift, s->zbase, incr ? s->wflag : nullptr, nsub,
                                    nchan, nbin, nullptr, s->part2, s->wpart, nullptr, 0, 0, nullptr, s->exF));
        return scrunch_stage(s);
    }
    if (iter == 1) {   // W == w0: the carried baseline is exactly prepare()'s; also writes D (exact fit)
        LAUNCH(s, K_CHAN_PARTIALS,
               launch_chan_partials(s->stream, s->D ? 3 : 1, s->raw, s->W, s->shift, s->base, nullptr, nsub, nchan,
                                    nbin, nullptr, s->part2, s->wpart, s->D, s->ldD, s->dtiled, nullptr, s->exF));
    } else {
        if (s->incr) {
            // the sums of the previous iteration moved through the changed channels
            const float *Wo = s->hist + (size_t)(iter - 2) * s->P;
            LAUNCH(s, K_CHAN_PARTIALS,
                   launch_chan_delta(s->stream, s->raw, s->shift, s->base, s->W, Wo, nsub, nchan, nbin, s->part,
                                     s->part2, s->wpart, s->exA, s->exF));
        } else {
            LAUNCH(s, K_CHAN_PARTIALS,
                   launch_chan_partials(s->stream, 2, s->raw, s->W, s->shift, s->base, nullptr, nsub, nchan, nbin,
                                        s->part, s->part2, s->wpart));
        }
        if (int rc = window_stage(s, s->wflag)) return rc;
        LAUNCH(s, K_BASE,
               launch_base(s->stream, s->raw, s->shift, s->win, s->wflag, nsub, nchan, nbin, s->width, s->base));
        LAUNCH(s, K_CHAN_PARTIALS,
               launch_chan_partials(s->stream, 1, s->raw, s->W, s->shift, s->base, s->wflag, nsub, nchan, nbin,
                                    nullptr, s->part2, s->wpart, nullptr, 0, 0, nullptr, s->exF));
    }
    return scrunch_stage(s);
}

// Row medians/MADs of a shard: the diagnostics rows go to their owners
// (all-to-all), each owner runs the row selections over whole rows, and the
// results are all-gathered into row_med/row_mad [4][nsub].
int shard_rowstats(Session *s, const LineStatsArgs &la)
{
    LAUNCH(s, K_SHARD_PACK,
           launch_pack_rows(s->stream, s->geom, s->nchan, s->std_, s->mean, s->fft, s->ptp, nullptr, s->xd_send));
    CM(s, s->comm->alltoallv(s->xd_send, s->dsb.data(), s->xd_recv, s->drb.data(), s->stream), "diagnostics rows");
    LAUNCH(s, K_SHARD_PACK,
           launch_assemble_rows(s->stream, s->geom, s->xd_recv, s->std_r, s->mean_r, s->fft_r, s->ptp_r, nullptr));
    LineStatsArgs lr;
    lr.nsub = s->rows_own;
    lr.nchan = s->geom.nchan_g;
    lr.valid = s->valid_r;
    lr.std_d = s->std_r;
    lr.mean_d = s->mean_r;
    lr.fft_d = s->fft_r;
    lr.ptp_d = s->ptp_r;
    lr.ptp_f32 = la.ptp_f32;
    lr.grp_waves = la.grp_waves;
    lr.grp_minlen = la.grp_minlen;
    lr.col_med = lr.col_mad = nullptr;
    lr.row_med = s->xr_send;
    lr.row_mad = s->xr_send + 4 * s->rows_own;
    LAUNCH(s, K_LINESTATS, launch_linestats(s->stream, lr, 2));
    CM(s, s->comm->allgather(s->xr_send, s->xr_recv, sizeof(double) * 8 * s->rows_pad, s->stream), "row statistics");
    LAUNCH(s, K_SHARD_PACK, launch_unpack_rowstats(s->stream, s->geom, s->rows_pad, s->xr_recv, la.row_med, la.row_mad));
    return 0;
}

// exact scipy leastsq for every profile (ic.py:266-272).
// Rounds of k_fit_pass + k_fit_state over a compacted list of the profiles
// that still need a data sweep.  Each round's survivor count lands in
// the low word of ctr[r] on the device; kernels read their list length there, so the
// host only needs an UPPER bound to size grids (counts never grow) and reads
// the counts one round behind: the stream always has the next round queued.
// Once the bound drops to tail_threshold (default kTailProfiles; 0 = never),
// k_fit_tail finishes the rest in one launch (one wave per profile).
// fork != nullptr: after round s->diag_fork the diagnostics of the profiles
// already fitted run on s->dstream (fork_diag); the survivors of that round
// are kept in the third list buffer for the main stream's second pass.
int fork_diag(Session *s, const DiagArgs &da, int r);
// after the round counters (and two spare words): the tail's sweep counter
// (u64, accumulating over a run: zeroed and read once per run by ic_run)
unsigned long long *tail_counter(Session *s) { return (unsigned long long *)(s->rcount + kRoundWords + 2); }

int run_fit(Session *s, const DiagArgs *fork)
{
    s->fork_round = -1;
    s->tail_split = false;
    const long P = (long)s->P;
    const int nbin = s->p.nbin;
    // zeroes too: per round, blocks done << 32 | survivors (the tail's sweep
    // counter after them accumulates over the run: zeroed and read once per
    // run by ic_run), and the late flags the fork round's state kernel sets
    CK(launch_fit_init(s->stream, s->fs, P, s->rcount, kRoundWords + 2, fork ? s->late : nullptr));
    CK(launch_fit_prep(s->stream, s->fs, s->T64, nbin));
    unsigned long long *ctr = (unsigned long long *)s->rcount;
    unsigned *done = (unsigned *)(s->rcount + 2 * kMaxRounds);
    unsigned long long *tail_sweeps = tail_counter(s);
    int32_t *bufs[3] = {s->lists, s->lists + P, s->lists + 2 * P};
    const int32_t *cur = nullptr;                    // round 0: all profiles
    const unsigned long long *cin = nullptr;         // the round's packed list counts (RoundList)
    long bound = P;                                 // >= the active count of the next round
    int rounds = 0;
    bool tail = false;
    int flagged = -1;   // the fork round, once its survivors are flagged and pass A not yet queued
    for (int r = 0;; ++r) {
        if (r >= kMaxRounds) return fail(IC_EHIP, "lmdif did not terminate after %d rounds", r);
        if (bound <= s->tail_threshold) {
            if (flagged >= 0) {
                if (int rc = fork_diag(s, *fork, flagged)) return rc;
                flagged = -1;
            }
            // (auto: profiles of >= 2048 bins, whose tail and statistics are long
            // enough to share the chip: C5 48.9-49.3 ms split against 50.7-50.8;
            // at 1024 bins the statistics' 8-wave blocks beside the tail stretch
            // its critical path, C2 26.0 against 25.5-25.6, C3 173.0 against
            // 171.7; C1 1.29-1.31 against 1.26-1.27; C4 2.91-2.93 against 2.94-2.96)
            const bool split = fork && (s->tail_split_mode == IC_TAIL_SPLIT_ON ||
                                        (s->tail_split_mode == IC_TAIL_SPLIT_AUTO && nbin >= 2048));
            if (split && s->fork_round >= 0 && cur && !s->fftded) {
                // the second fork: the fork round's survivors fitted by now (not in
                // the tail's list, marked here) are measured on dstream beside the tail
                CK(launch_mark_list(s->stream, cur, cin, P, bound, s->tmark, 1));
                CK(hipEventRecord(s->fork2_ev, s->stream));
                CK(hipStreamWaitEvent(s->dstream, s->fork2_ev, 0));
                DiagArgs b1 = *fork;
                b1.list = s->lists + 2 * P;
                b1.nctr = ctr + s->fork_round;
                b1.skip = s->tmark;
                LAUNCH_ON(s, K_DIAG, s->dstream, launch_diag(s->dstream, b1));
                CK(hipEventRecord(s->join_ev, s->dstream));
                s->tail_split = true;
                s->tail_list = cur;
                s->tail_cin = cin;
                s->tail_bound = bound;
            }
            LAUNCH(s, K_FIT_TAIL, launch_fit_tail(s->stream, s->D, s->T64, P, nbin, s->ldD, s->dtiled, cur, cin, bound,
                                                  s->fs, s->amp, s->info, tail_sweeps));
            tail = true;
            break;
        }
        const bool fork_here = fork && r == s->diag_fork;
        int32_t *next = fork_here ? bufs[2] : bufs[r & 1];
        LAUNCH(s, K_FIT_PASS, launch_fit_pass(s->stream, s->D, s->T64, P, nbin, s->ldD, s->dtiled, cur, cin, bound,
                                                s->fs, r == 0));
        __atomic_store_n(s->h_rcount + r, -1, __ATOMIC_RELAXED);
        LAUNCH(s, K_FIT_STATE, launch_fit_state(s->stream, s->fs, P, cur, cin, bound, s->amp, s->info, next,
                                                ctr + r, done + r, s->d_h_rcount + r, fork_here ? s->late : nullptr));
        if (fork_here) flagged = r;
        // pass A is queued fork_delay rounds after the flags: the first late
        // rounds are the largest and run alone
        if (flagged >= 0 && r >= flagged + s->fork_delay) {
            if (int rc = fork_diag(s, *fork, flagged)) return rc;
            flagged = -1;
        }
        ++rounds;
        cur = next;
        cin = ctr + r;   // packed A / B counts of the next round's list
        if (r >= 1) {
            // count after round r-1 (= input of round r) bounds the count after round r
            CK(poll_count(s, s->h_rcount + (r - 1)));
            const long c = s->h_rcount[r - 1];
            if (c == 0) break;   // round r had nothing to do
            bound = c;
        }
    }
    if (flagged >= 0)
        if (int rc = fork_diag(s, *fork, flagged)) return rc;
    // no stream synchronisation: the counts below were all read by the loop
    // (after the event of their round), so the diagnostics queue right behind
    // the last fit kernel
    int64_t swept = rounds > 0 ? P : 0;   // round 0 input
    for (int r = 0; r + 1 < rounds; ++r) swept += s->h_rcount[r];
    int effective = rounds;
    if (!tail) {
        // trailing rounds that had an empty input list
        while (effective > 1 && s->h_rcount[effective - 2] == 0) --effective;
    }
    s->fit_rounds = effective;
    s->stats.fit_rounds += effective;
    s->stats.fit_profile_sweeps += swept;
    return 0;
}

// The fork (run_fit, round r): the profiles that round r's state kernel did
// not flag in s->late have their final amp / info, so their diagnostics
// (pass A: k_diag_cl skipping the flagged ones) run on dstream, ordered after
// round r only, while the main stream goes on with the late rounds and the
// tail (latency-bound: a few thousand waves).  The flagged profiles, round r's
// survivor list in the third list buffer, get pass B on the main stream after
// the fit (run_impl), which then joins dstream.
int fork_diag(Session *s, const DiagArgs &da, int r)
{
    CK(hipEventRecord(s->fork_ev, s->stream));
    CK(hipStreamWaitEvent(s->dstream, s->fork_ev, 0));
    if (s->fftded) {   // their residual rows, rotated back (run_impl: the rest after the fit)
        RotateArgs ra = residual_rotate_args(s, s->pr_lo, s->pr_hi);
        ra.late = s->late;
        ra.late_sel = 0;
        if (rot_stats_on(s)) with_stats(s, ra);
        LAUNCH_ON(s, K_ROTATE, s->dstream, launch_rotate(s->dstream, ra));
    }
    if (!rot_stats_on(s)) {
        DiagArgs a = da;
        a.skip = s->late;
        LAUNCH_ON(s, K_DIAG, s->dstream, launch_diag(s->dstream, a));
    }
    CK(hipEventRecord(s->join_ev, s->dstream));
    s->fork_round = r;
    return 0;
}

}  // namespace

extern "C" {

int ic_abi_version(void) { return IC_ABI_VERSION; }

int ic_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *ic_last_error(void) { return g_err.c_str(); }

const char *ic_kernel_name(int kernel)
{
    if (kernel < 0 || kernel >= K_COUNT) return "";
    return kKernelNames[kernel];
}

}  // extern "C"

namespace {

// Shared by every create entry point.  sharded: this session is channel shard
// `rank` of `world` (world may be 1: the exchanges then run over a one-rank
// transport, which tests it end to end); make_comm() builds the transport
// after the device is current.
template <typename MakeComm>
int create_session(const ic_params *params, int device, int rank, int world, bool sharded, MakeComm make_comm,
                   void **out)
{
    if (!params || !out) return fail(IC_EINVAL, "null argument");
    *out = nullptr;
    const ic_params &p = *params;
    if (p.nsub <= 0 || p.nchan <= 0 || p.nbin <= 0)
        return fail(IC_EINVAL, "bad shape nsub=%d nchan=%d nbin=%d", p.nsub, p.nchan, p.nbin);
    if (p.nbin > 32768) return fail(IC_EINVAL, "nbin=%d > 32768 unsupported", p.nbin);
    if (p.nsub > 16384 || p.nchan > 16384)
        return fail(IC_EINVAL, "line length > 16384 unsupported (nsub=%d nchan=%d)", p.nsub, p.nchan);
    if (p.max_iter < 0) return fail(IC_EINVAL, "max_iter < 0");
    if (p.fit_mode != IC_FIT_EXACT && p.fit_mode != IC_FIT_CLOSED)
        return fail(IC_EINVAL, "fit_mode %d unsupported", p.fit_mode);
    if (p.dedisp_mode != IC_DEDISP_SHIFT && p.dedisp_mode != IC_DEDISP_FFT)
        return fail(IC_EINVAL, "dedisp_mode %d unsupported", p.dedisp_mode);
    if (p.input_dedispersed != 0 && (p.input_dedispersed != 1 || p.dedisp_mode != IC_DEDISP_FFT))
        return fail(IC_EINVAL, "input_dedispersed=%d needs dedisp_mode IC_DEDISP_FFT (0 or 1)", p.input_dedispersed);
    if (p.dedisp_mode == IC_DEDISP_FFT && !rotate_supported(p.nbin))
        return fail(IC_EINVAL, "fractional dedispersion needs a power-of-two nbin in 64..4096 (nbin=%d)", p.nbin);
    if (diag_lds_bytes(p.nbin) > 160 * 1024)
        return fail(IC_EINVAL, "nbin=%d needs %zu bytes of LDS for the diagnostics (> 160 KiB)", p.nbin,
                    diag_lds_bytes(p.nbin));
    if (window_lds_bytes(p.nbin) > 160 * 1024)
        return fail(IC_EINVAL, "nbin=%d needs %zu bytes of LDS for the baseline window (> 160 KiB)", p.nbin,
                    window_lds_bytes(p.nbin));
    if (world < 1 || rank < 0 || rank >= world) return fail(IC_EINVAL, "bad rank %d / world %d", rank, world);
    std::vector<int32_t> cr(2 * world), rr(2 * world);
    if (const char *e = shard_layout(p.nsub, p.nchan, world, cr.data(), rr.data()))
        return fail(IC_EINVAL, "cannot shard nchan=%d over %d: %s", p.nchan, world, e);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(IC_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(IC_EINVAL, "device %d out of range (%d devices)", device, ndev);
    Session *s = new Session();
    s->p = p;
    s->device = device;
    s->rank = rank;
    s->world = world;
    s->c0 = cr[2 * rank];
    s->nchan = cr[2 * rank + 1] - cr[2 * rank];
    s->P = (size_t)p.nsub * s->nchan;
    s->N = s->P * (size_t)p.nbin;
    s->nsb = (s->nchan + kSuperBlock - 1) / kSuperBlock;
    s->plan_sb = make_sb_plan(s->nsb);
    s->plan_top = make_sb_plan(world);
    s->geom.world = world;
    s->geom.rank = rank;
    s->geom.nsub = p.nsub;
    s->geom.nchan_g = p.nchan;
    for (int r = 0; r < world; ++r) {
        s->geom.chan0[r] = cr[2 * r];
        s->geom.row0[r] = rr[2 * r];
    }
    s->geom.chan0[world] = p.nchan;
    s->geom.row0[world] = p.nsub;
    s->rows_own = rr[2 * rank + 1] - rr[2 * rank];
    s->rows_pad = (p.nsub + world - 1) / world;
    s->ldD = ((p.nbin + kFitTile - 1) / kFitTile) * kFitTile;
    s->Ppad = ((s->P + 63) / 64) * 64;
    s->width = (int)(p.baseline_duty * (double)p.nbin);
    if (s->width < 1) s->width = 1;
    int rc = 0;
    auto bail = [&](int code) {
        free_all(s);
        delete s;
        return code;
    };
#define AL(ptr, n)                                                                                  \
    do {                                                                                            \
        if (dalloc(&(ptr), (n)) != hipSuccess) {                                                    \
            rc = fail(IC_ENOMEM, "hipMalloc(%s, %zu elements) failed", #ptr, (size_t)(n));          \
            return bail(rc);                                                                        \
        }                                                                                           \
    } while (0)
    if (hipSetDevice(device) != hipSuccess) return bail(fail(IC_EHIP, "hipSetDevice(%d) failed", device));
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(IC_EHIP, "hipStreamCreate failed"));
    // the diagnostics fork's stream exists for every session it can serve
    // (IC_OPT_DIAG_FORK may switch it on or off before any run)
    if (p.fit_mode == IC_FIT_EXACT) {
        // (a higher priority for the fit's stream measured no different)
        if (hipStreamCreateWithFlags(&s->dstream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s->fork_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s->join_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s->fork2_ev, hipEventDisableTiming) != hipSuccess)
            return bail(fail(IC_EHIP, "diagnostics stream / events failed"));
    }
    const size_t P = s->P, N = s->N;
    const int nsub = p.nsub, nchan = s->nchan, nbin = p.nbin;
    const bool exact = p.fit_mode == IC_FIT_EXACT;
    // the fit's lists hold int32 profile indices, its round counts are 32-bit fields (RoundList)
    if (exact && P >= (1ull << 31))
        return bail(fail(IC_EINVAL, "the exact fit takes < 2^31 profiles per session or shard (%zu)", P));
    AL(s->slot_raw[0], N);
    s->raw = s->slot_raw[0];
    // the closed-form fit reads the raw cube (no fit cube, no lmdif state), unless
    // the dedispersion is the FFT rotation: then the rotated fit cube is kept
    if (exact || p.dedisp_mode == IC_DEDISP_FFT) {
        AL(s->D, s->Ppad * (size_t)s->ldD);
        if (hipMemset(s->D, 0, sizeof(float) * s->Ppad * (size_t)s->ldD) != hipSuccess)
            return bail(fail(IC_EHIP, "hipMemset(D) failed"));
    }
    AL(s->TT, 1);
    s->fftded = p.dedisp_mode == IC_DEDISP_FFT;
    // The FFT mode forks too (round 6): its forked pass is the residual rotation
    // that measures the rows, one kernel since the statistics moved into it, and
    // it now hides behind the late fit rounds (C2 --dedisp fft 45.51-45.70 ->
    // 45.03-45.06 ms per clean, per-profile delays 47.23-47.44 -> 47.04-47.19,
    // alternating on one box; round 4, with two kernels per forked pass and the
    // radix-2 rotation, it had lost: 55.4-55.5 unforked, 56.7-56.9 forked)
    // large sessions hand over later: C2 (1.15 M profiles) 26.49-26.56 ms per
    // clean at 8192, 26.19-26.23 at 4096 (2048: 26.23-26.28, 6144: 26.30-26.34),
    // C3 flat; C4 and C5 lose at 4096 (2.90 -> 3.02-3.04, 46.5 -> 46.9)
    if (P >= ((size_t)1 << 20)) s->tail_threshold = kTailProfilesLarge;
    // long profiles hand over earlier: C5 (4096 bins) 46.1-47.0 ms at 8192,
    // 45.5-46.2 at 12288 (C4 at 512 bins flat from 6144 to 12288)
    else if (nbin >= 2048) s->tail_threshold = kTailProfilesLong;
    // long profiles take more rounds before their late phase: C5 (4096 bins)
    // 49.7-49.9 ms per clean forked after round 3 / delay 1, 48.2 after
    // round 4 / delay 2 (round 5: 48.4-48.7, 6: 49.1)
    if (!s->fftded && nbin >= 2048) {
        s->diag_fork = 4;
        s->fork_delay = 2;
    }
    // the fit cube (written by k_chan_partials mode 3, or by k_rotate in the FFT
    // mode) is tiled; IC_OPT_FIT_TILED = 0: row-major.  The closed-form fit of
    // the FFT mode reads its rotated fit cube row by row (k_diag DIAG_FIT).
    s->dtiled = (s->fftded && !exact) ? 0 : 1;
    if (s->fftded) {
        AL(s->dr, N);
        AL(s->Tc, N);
        // R (the rotated residual rows) only when a run measures them in a
        // separate pass (run_impl: !rot_stats_on)
        AL(s->zbase, P);
        AL(s->zshift, (size_t)nchan);
        AL(s->ph, 2 * (size_t)nchan * (nbin / 2 + 1));
        if (hipMemset(s->zbase, 0, sizeof(float) * P) != hipSuccess ||
            hipMemset(s->zshift, 0, sizeof(int32_t) * nchan) != hipSuccess)
            return bail(fail(IC_EHIP, "hipMemset(zero levels / shifts) failed"));
    }
    AL(s->slot_w0[0], P);
    s->w0 = s->slot_w0[0];
    AL(s->W, P);
    AL(s->base, P);
    AL(s->base0, P);
    AL(s->valid, P);
    AL(s->slot_shift[0], (size_t)nchan);
    s->shift = s->slot_shift[0];
    AL(s->win, (size_t)nsub);
    AL(s->wflag, (size_t)nsub + 1);   // + window-moves counter
    AL(s->part, (size_t)nsub * s->nsb * nbin);
    // the incremental template stage's column flags (IC_OPT_TEMPLATE_INCR)
    AL(s->exA, (size_t)nsub * s->nsb * nbin);
    AL(s->exF, (size_t)nsub * s->nsb * nbin);
    AL(s->part2, (size_t)nsub * s->nsb * nbin);
    AL(s->wpart, (size_t)nsub * s->nsb);
    AL(s->F, (size_t)nsub * nbin);
    AL(s->wf, (size_t)nsub);
    AL(s->T, (size_t)nbin);
    AL(s->T64, (size_t)s->ldD);
    if (hipMemset(s->T64, 0, sizeof(double) * s->ldD) != hipSuccess)
        return bail(fail(IC_EHIP, "hipMemset(T64) failed"));   // zero tail: padded samples are no-ops
    AL(s->T2, (size_t)2 * nbin);
    AL(s->amp, P);
    AL(s->info, P);
    AL(s->std_, P);
    AL(s->mean, P);
    AL(s->ptp, P);
    AL(s->fft, P);
    AL(s->test, P);
    AL(s->hist, P * (size_t)(p.max_iter + 1));
    AL(s->lstat, (size_t)16 * (nchan + nsub));
    AL(s->tw, (size_t)nbin);
    AL(s->tw_p2, (size_t)nbin);
    AL(s->plan, 1);
    if (exact) AL(s->lists, 3 * P);   // two ping-pong round lists + the fork round's survivors
    AL(s->rcount, (size_t)kRoundWords + 4);   // + two spare words and the tail's sweep counter
    if (exact) AL(s->late, P);
    if (exact) {
        AL(s->tmark, P);
        if (hipMemset(s->tmark, 0, P) != hipSuccess) return bail(fail(IC_EHIP, "hipMemset(tail marks) failed"));
    }
    if (sharded) {
        std::string cerr;
        int ccode = IC_EINVAL;
        s->comm = make_comm(&cerr, &ccode);
        if (!s->comm) return bail(fail(ccode, "shard transport: %s", cerr.empty() ? "failed" : cerr.c_str()));
        s->comm->set_timeout_ms((long long)(s->sync_timeout_s * 1000.0 + 0.5));
        const size_t nchan_g = (size_t)p.nchan;
        AL(s->std_r, (size_t)s->rows_own * nchan_g);
        AL(s->mean_r, (size_t)s->rows_own * nchan_g);
        AL(s->fft_r, (size_t)s->rows_own * nchan_g);
        AL(s->ptp_r, (size_t)s->rows_own * nchan_g);
        AL(s->valid_r, (size_t)s->rows_own * nchan_g);
        size_t dsend = 0, drecv = 0;
        for (int r = 0; r < world; ++r) {
            const size_t rows_r = (size_t)(rr[2 * r + 1] - rr[2 * r]);
            const size_t nch_r = (size_t)(cr[2 * r + 1] - cr[2 * r]);
            s->dsb.push_back(shard_block_bytes(rows_r * nchan, 32));
            s->vsb.push_back(shard_block_bytes(rows_r * nchan, 1));
            s->drb.push_back(shard_block_bytes((size_t)s->rows_own * nch_r, 32));
            s->vrb.push_back(shard_block_bytes((size_t)s->rows_own * nch_r, 1));
            dsend += s->dsb.back();
            drecv += s->drb.back();
        }
        // root rows to their owners: rank r's block = its rows, contiguous in the send buffer
        for (int r = 0; r < world; ++r) {
            const size_t rows_r = (size_t)(rr[2 * r + 1] - rr[2 * r]);
            s->wsb.push_back(sizeof(double) * rows_r * nbin);
            s->wrb.push_back(sizeof(double) * s->rows_own * nbin);
            s->fsb.push_back(sizeof(double) * rows_r * (nbin + 1));
            s->frb.push_back(sizeof(double) * s->rows_own * (nbin + 1));
        }
        s->wg_blk = (s->rows_pad + 1) & ~1;
        s->fg_blk = ((long)s->rows_pad * (nbin + 1) + 1) & ~1L;
        struct {
            void **ptr;
            size_t bytes;
            const char *name;
        } xb[] = {{(void **)&s->xw_send, sizeof(double) * nsub * nbin, "window roots"},
                  {(void **)&s->xw_recv, sizeof(double) * world * s->rows_own * nbin, "owned window roots"},
                  {(void **)&s->xf_send, sizeof(double) * nsub * (nbin + 1), "fscrunch roots"},
                  {(void **)&s->xf_recv, sizeof(double) * world * s->rows_own * (nbin + 1), "owned fscrunch roots"},
                  {(void **)&s->xwg_send, sizeof(int32_t) * s->wg_blk, "owned windows"},
                  {(void **)&s->xwg_recv, sizeof(int32_t) * s->wg_blk * world, "gathered windows"},
                  {(void **)&s->xfg_send, sizeof(float) * s->fg_blk, "owned fscrunch rows"},
                  {(void **)&s->xfg_recv, sizeof(float) * s->fg_blk * world, "gathered fscrunch rows"},
                  {(void **)&s->xd_send, dsend, "diagnostics send"},
                  {(void **)&s->xd_recv, drecv, "diagnostics receive"},
                  {(void **)&s->xr_send, sizeof(double) * 8 * s->rows_pad, "row statistics"},
                  {(void **)&s->xr_recv, sizeof(double) * 8 * s->rows_pad * world, "gathered row statistics"},
                  {(void **)&s->counters, sizeof(int32_t) * (p.max_iter + 5), "counters"}};
        for (auto &b : xb)
            if (s->comm->alloc(b.ptr, b.bytes + 16) != 0 || !*b.ptr)
                return bail(fail(IC_ENOMEM, "exchange buffer (%s, %zu bytes) failed", b.name, b.bytes));
    } else {
        AL(s->counters, (size_t)(p.max_iter + 5));
    }
#undef AL
    if (hipHostMalloc((void **)&s->h_rcount, sizeof(int32_t) * kMaxRounds,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&s->d_h_rcount, s->h_rcount, 0) != hipSuccess)
        return bail(fail(IC_ENOMEM, "hipHostMalloc(round counts) failed"));
    if (hipEventCreateWithFlags(&s->sev, hipEventDisableTiming) != hipSuccess)
        return bail(fail(IC_EHIP, "hipEventCreate failed"));
    if (hipHostMalloc((void **)&s->h_small, sizeof(int32_t) * ((size_t)p.max_iter + 20)) != hipSuccess)
        return bail(fail(IC_ENOMEM, "hipHostMalloc(readback) failed"));
    if (exact) {
        // fit state: 21 double arrays + 5 four-byte arrays, each padded to 256 B
        const size_t dstride = ((P * 8 + 255) / 256) * 256, istride = ((P * 4 + 255) / 256) * 256;
        if (hipMalloc(&s->fs_block, 21 * dstride + 5 * istride) != hipSuccess)
            return bail(fail(IC_ENOMEM, "hipMalloc(fit state) failed"));
        char *b = (char *)s->fs_block;
        double **dp[] = {&s->fs.x,     &s->fs.fnorm, &s->fs.par,   &s->fs.delta,   &s->fs.diag, &s->fs.xnorm,
                         &s->fs.acnorm, &s->fs.J0,   &s->fs.f0,    &s->fs.aj,      &s->fs.r,    &s->fs.Jn0,
                         &s->fs.qtf,   &s->fs.gnorm, &s->fs.x2,    &s->fs.pnorm,   &s->fs.wa1,  &s->fs.xa,
                         &s->fs.o_fnorm, &s->fs.o_acnorm, &s->fs.o_sum};
        for (auto *q : dp) { *q = (double *)b; b += dstride; }
        int32_t **ip[] = {&s->fs.iter, &s->fs.nfev, &s->fs.mode, &s->fs.slow, (int32_t **)&s->fs.p0};
        for (auto *q : ip) { *q = (int32_t *)b; b += istride; }
        s->fs.T64 = s->T64;
        // k_fit_prep's 4 scalars
        if (dalloc(&s->fs.U, 8) != hipSuccess) return bail(fail(IC_ENOMEM, "hipMalloc(fit prep) failed"));
    }
    // twiddles exp(-2 pi i q / n) and the pairwise plan
    std::vector<double2> tw(nbin);
    for (int q = 0; q < nbin; ++q) {
        const long double ang = -2.0L * 3.141592653589793238462643383279502884L * (long double)q / (long double)nbin;
        tw[q] = make_double2((double)cosl(ang), (double)sinl(ang));
    }
    const std::vector<double2> tw2 = p2_twiddles(nbin);
    PwPlan plan;
    if (make_plan(nbin, &plan) != 0) return bail(fail(IC_EINVAL, "pairwise plan too large for nbin=%d", nbin));
    s->plan_ub = std::max(plan.nleaf, plan.nops);
    if (hipMemcpy(s->tw, tw.data(), sizeof(double2) * nbin, hipMemcpyHostToDevice) != hipSuccess ||
        (!tw2.empty() &&
         hipMemcpy(s->tw_p2, tw2.data(), sizeof(double2) * tw2.size(), hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(s->plan, &plan, sizeof plan, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(IC_EHIP, "upload of constants failed"));
    *out = s;
    return IC_OK;
}

}  // namespace

extern "C" {

int ic_session_create(const ic_params *params, int device, void **out)
{
    return create_session(params, device, 0, 1, false, [](std::string *, int *) -> Comm * { return nullptr; }, out);
}

int ic_shard_layout(int nsub, int nchan, int world, int32_t *chan_ranges, int32_t *row_ranges)
{
    if (!chan_ranges || !row_ranges || nsub <= 0 || nchan <= 0) return fail(IC_EINVAL, "bad argument");
    if (const char *e = shard_layout(nsub, nchan, world, chan_ranges, row_ranges))
        return fail(IC_EINVAL, "cannot shard nchan=%d over %d: %s", nchan, world, e);
    return IC_OK;
}

int ic_session_create_shard(const ic_params *params, int device, int rank, int world, const ic_comm_ops *ops,
                            void **out)
{
    if (!ops || !ops->alloc || !ops->release || !ops->allgather || !ops->alltoallv || !ops->allreduce_sum_i32)
        return fail(IC_EINVAL, "incomplete ic_comm_ops");
    const ic_comm_ops o = *ops;
    return create_session(params, device, rank, world, true,
                          [&](std::string *, int *) -> Comm * { return make_callback_comm(o, rank, world); }, out);
}

int ic_rccl_unique_id(void *id_out)
{
    if (!id_out) return fail(IC_EINVAL, "null argument");
    std::string err;
    if (rccl_unique_id(id_out, &err)) return fail(IC_ECOMM, "ncclGetUniqueId: %s", err.c_str());
    return IC_OK;
}

int ic_rccl_set_library(const char *path)
{
    const char *err = nullptr;
    if (rccl_set_library(path, &err)) return fail(IC_ESTATE, "%s", err);
    return IC_OK;
}

int ic_rccl_set_init_timeout(int64_t ms)
{
    const char *err = nullptr;
    if (rccl_set_init_timeout((long long)ms, &err)) return fail(IC_EINVAL, "%s", err);
    return IC_OK;
}

int ic_session_create_rccl(const ic_params *params, int device, int rank, int world, const void *unique_id,
                           void **out)
{
    if (!unique_id) return fail(IC_EINVAL, "null unique id");
    return create_session(params, device, rank, world, true,
                          [&](std::string *err, int *code) -> Comm * {
                              *code = IC_ECOMM;   // librccl missing, a rank that never joined, RCCL's own errors
                              return make_rccl_comm(unique_id, rank, world, err);
                          },
                          out);
}

int ic_group_create(int world, void **group)
{
    if (!group) return fail(IC_EINVAL, "null argument");
    *group = local_group_create(world);
    if (!*group) return fail(IC_EINVAL, "bad group size %d", world);
    return IC_OK;
}

void ic_group_destroy(void *group) { local_group_destroy((LocalGroup *)group); }

int ic_session_create_grouped(const ic_params *params, int device, void *group, int rank, void **out)
{
    LocalGroup *g = (LocalGroup *)group;
    if (!g) return fail(IC_EINVAL, "null group");
    return create_session(params, device, rank, local_group_world(g), true,
                          [&](std::string *err, int *) -> Comm * {
                              const char *e = nullptr;
                              Comm *c = make_local_comm(g, rank, device, &e);
                              if (e) *err = e;
                              return c;
                          }, out);
}

void ic_session_destroy(void *session)
{
    Session *s = (Session *)session;
    if (!s) return;
    if (s->failed) {
        // kernels of this session may still be running (a wait timed out):
        // freeing their buffers could hand memory in use to another
        // allocation, and a synchronising free could hang; leak them
        delete s;
        return;
    }
    (void)hipSetDevice(s->device);
    free_all(s);
    delete s;
}

int ic_upload(void *session, const float *cube, const float *w0, const int32_t *shift)
{
    Session *s = (Session *)session;
    if (!s || !cube || !w0 || !shift) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (s->fifo_n) return fail(IC_ESTATE, "ic_upload with %d asynchronous upload(s) pending", s->fifo_n);
    CK(hipSetDevice(s->device));
    for (int c = 0; c < s->nchan; ++c)
        if (shift[c] < 0 || shift[c] >= s->p.nbin) return fail(IC_EINVAL, "shift[%d]=%d out of [0,nbin)", c, shift[c]);
    s->ever_uploaded = true;
    CK(hipMemcpyAsync(s->raw, cube, sizeof(float) * s->N, hipMemcpyHostToDevice, s->stream));
    CK(hipMemcpyAsync(s->w0, w0, sizeof(float) * s->P, hipMemcpyHostToDevice, s->stream));
    CK(hipMemcpyAsync(s->shift, shift, sizeof(int32_t) * s->nchan, hipMemcpyHostToDevice, s->stream));
    CK(hipStreamSynchronize(s->stream));
    s->uploaded = true;
    s->ran = false;
    return IC_OK;
}

int ic_upload_pols(void *session, const float *data, int npol, const float *w0, const int32_t *shift)
{
    Session *s = (Session *)session;
    if (!s || !data || !w0 || !shift) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (npol < 1) return fail(IC_EINVAL, "npol=%d", npol);
    if (s->fifo_n) return fail(IC_ESTATE, "ic_upload_pols with %d asynchronous upload(s) pending", s->fifo_n);
    CK(hipSetDevice(s->device));
    for (int c = 0; c < s->nchan; ++c)
        if (shift[c] < 0 || shift[c] >= s->p.nbin) return fail(IC_EINVAL, "shift[%d]=%d out of [0,nbin)", c, shift[c]);
    s->ever_uploaded = true;
    const size_t row = sizeof(float) * (size_t)s->nchan * s->p.nbin;   // one subint of one polarisation
    // pol 0 -> raw; pol 1 -> the fit-cube buffer as scratch (rebuilt, and re-zeroed, below),
    // or a temporary buffer when the session keeps no fit cube (fit_mode 1)
    CK(hipMemcpy2DAsync(s->raw, row, data, row * npol, row, s->p.nsub, hipMemcpyHostToDevice, s->stream));
    if (npol >= 2) {
        float *pol1 = s->D;
        if (!pol1 && hipMalloc((void **)&pol1, sizeof(float) * s->N) != hipSuccess)
            return fail(IC_ENOMEM, "hipMalloc(pol1 scratch, %zu floats) failed", s->N);
        hipError_t e = hipMemcpy2DAsync(pol1, row, (const char *)data + row, row * npol, row, s->p.nsub,
                                        hipMemcpyHostToDevice, s->stream);
        if (e == hipSuccess) e = launch_pscrunch(s->stream, s->raw, pol1, s->N);
        if (e == hipSuccess && s->D)
            e = hipMemsetAsync(s->D, 0, sizeof(float) * s->Ppad * (size_t)s->ldD, s->stream);
        if (!s->D) {
            if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
            (void)hipFree(pol1);
        }
        if (e != hipSuccess) return fail(IC_EHIP, "ic_upload_pols: %s", hipGetErrorString(e));
    }
    CK(hipMemcpyAsync(s->w0, w0, sizeof(float) * s->P, hipMemcpyHostToDevice, s->stream));
    CK(hipMemcpyAsync(s->shift, shift, sizeof(int32_t) * s->nchan, hipMemcpyHostToDevice, s->stream));
    CK(hipStreamSynchronize(s->stream));
    s->uploaded = true;
    s->ran = false;
    return IC_OK;
}

int ic_upload_device(void *session, const float *d_cube, const float *d_w0, const int32_t *d_shift)
{
    Session *s = (Session *)session;
    if (!s || !d_cube || !d_w0 || !d_shift) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (s->fifo_n) return fail(IC_ESTATE, "ic_upload_device with %d asynchronous upload(s) pending", s->fifo_n);
    CK(hipSetDevice(s->device));
    s->ever_uploaded = true;
    CK(hipMemcpyAsync(s->raw, d_cube, sizeof(float) * s->N, hipMemcpyDeviceToDevice, s->stream));
    CK(hipMemcpyAsync(s->w0, d_w0, sizeof(float) * s->P, hipMemcpyDeviceToDevice, s->stream));
    CK(hipMemcpyAsync(s->shift, d_shift, sizeof(int32_t) * s->nchan, hipMemcpyDeviceToDevice, s->stream));
    CK(hipStreamSynchronize(s->stream));
    s->uploaded = true;
    s->ran = false;
    return IC_OK;
}

int ic_upload_async(void *session, const float *cube, const float *w0, const int32_t *shift)
{
    Session *s = (Session *)session;
    if (!s || !cube || !w0 || !shift) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (s->fifo_n == 2) return fail(IC_ESTATE, "two asynchronous uploads already pending (run one first)");
    for (int c = 0; c < s->nchan; ++c)
        if (shift[c] < 0 || shift[c] >= s->p.nbin) return fail(IC_EINVAL, "shift[%d]=%d out of [0,nbin)", c, shift[c]);
    CK(hipSetDevice(s->device));
    // the slot not holding the newest data: after the queued upload, else after the current archive
    const int target = s->fifo_n ? 1 - s->fifo[s->fifo_n - 1] : (s->ever_uploaded ? 1 - s->cur : s->cur);
    if (!s->slot_raw[target]) {
        if (dalloc(&s->slot_raw[target], s->N) != hipSuccess || dalloc(&s->slot_w0[target], s->P) != hipSuccess ||
            dalloc(&s->slot_shift[target], (size_t)s->nchan) != hipSuccess)
            return fail(IC_ENOMEM, "second input slot (%zu bytes) failed", sizeof(float) * (s->N + s->P));
    }
    if (!s->copy_stream) CK(hipStreamCreateWithFlags(&s->copy_stream, hipStreamNonBlocking));
    if (!s->slot_ev[target]) CK(hipEventCreateWithFlags(&s->slot_ev[target], hipEventDisableTiming));
    CK(hipMemcpyAsync(s->slot_raw[target], cube, sizeof(float) * s->N, hipMemcpyHostToDevice, s->copy_stream));
    CK(hipMemcpyAsync(s->slot_w0[target], w0, sizeof(float) * s->P, hipMemcpyHostToDevice, s->copy_stream));
    CK(hipMemcpyAsync(s->slot_shift[target], shift, sizeof(int32_t) * s->nchan, hipMemcpyHostToDevice,
                      s->copy_stream));
    CK(hipEventRecord(s->slot_ev[target], s->copy_stream));
    s->fifo[s->fifo_n++] = target;
    s->ever_uploaded = true;
    return IC_OK;
}

int ic_host_alloc(size_t bytes, void **ptr)
{
    if (!ptr) return fail(IC_EINVAL, "null argument");
    *ptr = nullptr;
    if (hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess || !*ptr)
        return fail(IC_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
    return IC_OK;
}

void ic_host_free(void *ptr)
{
    if (ptr) (void)hipHostFree(ptr);
}

int ic_set_timing_kernel(void *session, int kernel)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null session");
    if (s->failed) return failed_session();
    if (kernel >= K_COUNT) return fail(IC_EINVAL, "kernel id %d >= %d", kernel, (int)K_COUNT);
    s->timing_only = kernel < 0 ? -1 : kernel;
    return IC_OK;
}

int ic_set_timing(void *session, int enabled)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null session");
    if (s->failed) return failed_session();
    s->timing = enabled != 0;
    s->events.clear();   // events of earlier runs are discarded unread
    s->enext = 0;
    for (int q = 0; q < K_COUNT; ++q) {
        s->kms[q] = 0.0;
        s->klaunch[q] = 0;
    }
    return IC_OK;
}

int ic_get_kernel_times(void *session, ic_kernel_time *out, int n)
{
    Session *s = (Session *)session;
    if (!s || (!out && n > 0)) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (int rc = collect_timing(s)) return rc;
    int m = 0;
    for (int q = 0; q < K_COUNT && m < n; ++q) {
        out[m].kernel = q;
        out[m].launches = s->klaunch[q];
        out[m].ms = s->kms[q];
        ++m;
    }
    return m;
}

}  // extern "C"

namespace {

// the diagnostics launch of one iteration: exact fit (amp/info from run_fit,
// fit cube D) or closed form (k_diag computes amp/info from raw and base0)
DiagArgs diag_args(Session *s, int pr_start, int pr_end)
{
    const ic_params &p = s->p;
    DiagArgs a{};
    a.mode = p.fit_mode == IC_FIT_EXACT ? DIAG_EXACT : DIAG_CLOSED;
    a.D = s->D;
    a.ldD = s->ldD;
    a.dtiled = s->dtiled;
    a.raw = s->raw;
    a.base = s->base0;
    a.T64 = s->T64;
    a.T2 = s->T2;
    a.TT = s->TT;
    a.amp = s->amp;
    a.info = s->info;
    a.w0 = s->w0;
    a.shift = s->shift;
    a.tw = s->tw;
    a.tw_p2 = s->tw_p2;
    a.plan = s->plan;
    a.nsub = p.nsub;
    a.nchan = s->nchan;
    a.nbin = p.nbin;
    a.pr_on = p.pr_on;
    a.pr_factor = p.pr_factor;
    a.pr_start = pr_start;
    a.pr_end = pr_end;
    a.std_o = s->std_;
    a.mean_o = s->mean;
    a.fft_o = s->fft;
    a.ptp_o = s->ptp;
    a.data_f64 = p.data_f64 != 0;
    a.chain = s->diag_chain ? 1 : 0;
    return a;
}

int run_impl(Session *s, double *test_out, float *weights_out, int32_t *loops_out, int32_t *changed_out,
             int32_t *nzero_out, int32_t *n_iter_out, int32_t *converged_out)
{
    CK(hipSetDevice(s->device));
    if (s->fifo_n) {   // the oldest asynchronous upload becomes the current archive
        const int slot = s->fifo[0];
        s->fifo[0] = s->fifo[1];
        --s->fifo_n;
        CK(hipStreamWaitEvent(s->stream, s->slot_ev[slot], 0));
        s->cur = slot;
        s->raw = s->slot_raw[slot];
        s->w0 = s->slot_w0[slot];
        s->shift = s->slot_shift[slot];
        s->uploaded = true;
        s->ran = false;
    }
    if (!s->uploaded) return fail(IC_ESTATE, "ic_run before ic_upload");
    // timed launches of earlier runs: fold them into the totals so the event
    // pool stays at one run's worth (the previous run ended synchronised)
    if (s->events.size() > 4096)
        if (int rc = collect_timing(s)) return rc;
    if (s->fftded && !s->delays_set) return fail(IC_ESTATE, "ic_run before ic_set_delays (dedisp_mode FFT)");
    if (s->fftded && !rot_stats_on(s) && !s->R && dalloc(&s->R, s->N) != hipSuccess) {
        s->R = nullptr;
        return fail(IC_ENOMEM, "hipMalloc(R: %zu floats) failed", s->N);
    }
    // the second fork's tail marks are cleared at the end of each iteration; a
    // run that failed in between may have left some set
    if (s->tmark) CK(hipMemsetAsync(s->tmark, 0, s->P, s->stream));
    const ic_params &p = s->p;
    const int nsub = p.nsub, nchan = s->nchan, nbin = p.nbin;
    int pr_start = p.pr_start < 0 ? 0 : (p.pr_start > nbin ? nbin : p.pr_start);
    int pr_end = p.pr_end < 0 ? 0 : (p.pr_end > nbin ? nbin : p.pr_end);
    // fit cube (ic.py:96-100) + initial weights/history; a session can be re-run
    s->stats = ic_run_stats{};
    if (int rc = prepare(s)) return rc;
    LineStatsArgs la;
    la.nsub = nsub;
    la.nchan = nchan;
    la.valid = s->valid;
    la.std_d = s->std_;
    la.mean_d = s->mean;
    la.fft_d = s->fft;
    la.ptp_d = s->ptp;
    la.ptp_f32 = !p.data_f64;
    la.grp_waves = s->ls_knobs.grp_waves;
    la.grp_minlen = s->ls_knobs.grp_minlen;
    la.col_med = s->lstat;
    la.col_mad = s->lstat + 4 * nchan;
    la.row_med = s->lstat + 8 * nchan;
    la.row_mad = s->lstat + 8 * nchan + 4 * nsub;
    int32_t *cnt = s->h_small;   // [max_iter + 5] counters, then the run stats (pinned)
    s->bad_fits.clear();
    int x = 0, loops = -1, n_iter = 0, converged = 0;
    // k_fit_tail's sweep counter (after the per-round counters): one run's total
    CK(hipMemsetAsync(tail_counter(s), 0, sizeof(unsigned long long), s->stream));
    while (x < p.max_iter) {
        x += 1;
        ++n_iter;
        if (int rc = iteration_template(s, n_iter)) return rc;
        DiagArgs da = diag_args(s, pr_start, pr_end);
        // the statistics pass: FFT dedispersion measures the residual rows
        // rotated back to the dispersed frame (R), written by k_rotate
        DiagArgs ds = da;
        if (s->fftded) {
            ds.mode = DIAG_STATS;
            ds.D = s->R;
            ds.ldD = nbin;
            ds.dtiled = 0;
        }
        s->pr_lo = pr_start;
        s->pr_hi = pr_end;
        if (p.fit_mode == IC_FIT_EXACT) {
            const bool fork = s->diag_fork > 0 && s->dstream && s->late && diag_list_supported(ds);
            if (int rc = run_fit(s, fork ? &ds : nullptr)) return rc;
        } else {
            LAUNCH(s, K_TNORM, launch_tnorm(s->stream, s->T64, s->plan, s->plan_ub, s->TT));
        }
        if (s->fftded) {
            if (p.fit_mode == IC_FIT_CLOSED) {   // the closed-form amplitudes of the rotated fit cube
                DiagArgs fa = da;
                fa.mode = DIAG_FIT;
                LAUNCH(s, K_DIAG, launch_diag(s->stream, fa));
            }
            // residual in the dedispersed frame, dededispersed by the inverse
            // rotation (ic.py:101-104), then comprehensive_stats of those rows
            // (after a fork: the profiles still fitting at it, the others were
            // rotated on dstream)
            RotateArgs ra = residual_rotate_args(s, pr_start, pr_end);
            if (s->fork_round >= 0) {
                // pass B: the profiles still fitting at the fork round.  With
                // per-profile delays from the round's survivor list (C2 fft_pp
                // 47.64-47.80 -> 47.24-47.34 ms per clean); with a channel's
                // phasor table by the late flags over the channel-major items,
                // whose profiles share the table row (the list: 45.44-45.57 ->
                // 45.77-45.88)
                if (s->delay2) {
                    ra.list = s->lists + 2 * s->P;
                    ra.nctr = (const unsigned long long *)s->rcount + s->fork_round;
                } else {
                    ra.late = s->late;
                    ra.late_sel = 1;
                }
            }
            if (rot_stats_on(s)) with_stats(s, ra);
            LAUNCH(s, K_ROTATE, launch_rotate(s->stream, ra));
            da = ds;
        }
        if (rot_stats_on(s)) {
            // the rotation measured its rows (after a fork: pass A's on dstream)
            if (s->fork_round >= 0) CK(hipStreamWaitEvent(s->stream, s->join_ev, 0));
        } else if (s->tail_split) {
            // the tail's profiles (the rest of pass B ran beside the tail), then
            // join dstream and clear the marks for the next iteration
            DiagArgs b = da;
            b.list = s->tail_list;
            b.nctr = s->tail_cin;
            LAUNCH(s, K_DIAG, launch_diag(s->stream, b));
            CK(hipStreamWaitEvent(s->stream, s->join_ev, 0));
            CK(launch_mark_list(s->stream, s->tail_list, s->tail_cin, (long)s->P, s->tail_bound, s->tmark, 0));
        } else if (s->fork_round >= 0) {
            // pass B: the profiles still fitting at the fork, then join pass A
            DiagArgs b = da;
            b.list = s->lists + 2 * s->P;
            b.nctr = (const unsigned long long *)s->rcount + s->fork_round;
            LAUNCH(s, K_DIAG, launch_diag(s->stream, b));
            CK(hipStreamWaitEvent(s->stream, s->join_ev, 0));
        } else {
            LAUNCH(s, K_DIAG, launch_diag(s->stream, da));
        }
        // channel medians are local to a shard; row medians need whole rows
        LAUNCH(s, K_LINESTATS, launch_linestats(s->stream, la, s->comm ? 1 : 3));
        if (s->comm)
            if (int rc = shard_rowstats(s, la)) return rc;
        CK(hipMemsetAsync(s->counters, 0, sizeof(int32_t) * (p.max_iter + 5), s->stream));
        LAUNCH(s, K_COMBINE,
               launch_combine(s->stream, nsub, nchan, s->valid, s->info, s->w0, s->std_, s->mean, s->ptp, la.ptp_f32,
                              s->fft,
                              la.col_med, la.col_mad, la.row_med, la.row_mad, p.chanthresh, p.subintthresh,
                              s->test, s->W, s->hist, n_iter, s->counters));
        if (s->comm)
            CM(s, s->comm->allreduce_sum_i32(s->counters, (size_t)(n_iter + 4), s->stream), "convergence counters");
        CK(hipMemcpyAsync(cnt, s->counters, sizeof(int32_t) * (n_iter + 4), hipMemcpyDeviceToHost,
                          s->stream));
        CK(spin_sync(s));
        if (changed_out) changed_out[n_iter - 1] = cnt[0];
        if (nzero_out) nzero_out[n_iter - 1] = cnt[1];
        s->bad_fits.push_back(cnt[2]);
        s->stats.near_threshold = cnt[3];
        for (int h = 0; h < n_iter; ++h)
            if (cnt[4 + h] == 0) {
                loops = x;
                converged = 1;
                x = 1000000;
            }
    }
    if (x == p.max_iter) loops = p.max_iter;
    s->last_iter = n_iter;
    if (test_out && n_iter > 0)
        CK(hipMemcpyAsync(test_out, s->test, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    if (weights_out)
        CK(hipMemcpyAsync(weights_out, s->W, sizeof(float) * s->P, hipMemcpyDeviceToHost, s->stream));
    {
        int32_t *moves = s->h_small + p.max_iter + 6;                               // pinned
        unsigned long long *tsw = (unsigned long long *)(s->h_small + ((p.max_iter + 9) & ~1));   // 8-B aligned
        CK(hipMemcpyAsync(moves, s->wflag + nsub, sizeof *moves, hipMemcpyDeviceToHost, s->stream));
        CK(hipMemcpyAsync(tsw, tail_counter(s), sizeof *tsw, hipMemcpyDeviceToHost, s->stream));
        CK(spin_sync(s));
        s->stats.window_moves = *moves;
        s->stats.fit_tail_sweeps += (int64_t)tsw[0];
    }
    // timing events are read when asked for (ic_get_kernel_times), not here
    if (loops_out) *loops_out = loops;
    if (n_iter_out) *n_iter_out = n_iter;
    s->stats.iterations = n_iter;
    if (converged_out) *converged_out = converged;
    s->ran = n_iter > 0;
    return IC_OK;
}

}  // namespace

extern "C" {

int ic_run(void *session, double *test_out, float *weights_out, int32_t *loops_out, int32_t *changed_out,
           int32_t *nzero_out, int32_t *n_iter_out, int32_t *converged_out)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null session");
    if (s->failed) return failed_session();
    int rc = run_impl(s, test_out, weights_out, loops_out, changed_out, nzero_out, n_iter_out, converged_out);
    if (rc && s->comm_lost) rc = fail(IC_ECOMM, "the shard transport lost a peer (RCCL asynchronous error)");
    if (rc && s->comm) s->comm->abort();   // peers must not wait for this shard
    return rc;
}

int ic_get_residual(void *session, float *out)
{
    Session *s = (Session *)session;
    if (!s || !out) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->ran) return fail(IC_ESTATE, "no completed iteration");
    CK(hipSetDevice(s->device));
    const ic_params &p = s->p;
    int pr_start = p.pr_start < 0 ? 0 : (p.pr_start > p.nbin ? p.nbin : p.pr_start);
    int pr_end = p.pr_end < 0 ? 0 : (p.pr_end > p.nbin ? p.nbin : p.pr_end);
    // temporary output buffer
    float *R = nullptr;
    CK(hipMalloc((void **)&R, sizeof(float) * s->N));
    hipError_t e;
    if (s->fftded) {   // residual + dededisperse (the inverse rotation) in one pass
        RotateArgs ra = residual_rotate_args(s, pr_start, pr_end);
        ra.out = R;
        e = launch_rotate(s->stream, ra);
    } else {
        e = launch_residual(s->stream, s->D, s->raw, s->base0, s->T64, s->amp, s->info, s->shift, p.nsub, s->nchan,
                            p.nbin, s->ldD, s->dtiled, p.pr_on, p.pr_factor, pr_start, pr_end, R);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, R, sizeof(float) * s->N, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(R);
    if (e != hipSuccess) return fail(IC_EHIP, "residual: %s", hipGetErrorString(e));
    return IC_OK;
}

int ic_set_delays(void *session, const double *delay_bins)
{
    Session *s = (Session *)session;
    if (!s || !delay_bins) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->fftded) return fail(IC_ESTATE, "ic_set_delays on a session with dedisp_mode %d", s->p.dedisp_mode);
    for (int c = 0; c < s->nchan; ++c)
        if (!isfinite(delay_bins[c])) return fail(IC_EINVAL, "delay[%d] is not finite", c);
    CK(hipSetDevice(s->device));
    const std::vector<float> ph = make_phasors(s->p.nbin, s->nchan, delay_bins);
    CK(hipMemcpyAsync(s->ph, ph.data(), sizeof(float) * ph.size(), hipMemcpyHostToDevice, s->stream));
    CK(hipStreamSynchronize(s->stream));
    if (s->delay2) {
        CK(hipFree(s->delay2));
        s->delay2 = nullptr;
    }
    s->delays_set = true;
    return IC_OK;
}

int ic_set_delays2(void *session, const double *delay_bins)
{
    Session *s = (Session *)session;
    if (!s || !delay_bins) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->fftded) return fail(IC_ESTATE, "ic_set_delays2 on a session with dedisp_mode %d", s->p.dedisp_mode);
    const int nsub = s->p.nsub, nchan = s->nchan;
    for (size_t k = 0; k < (size_t)nsub * nchan; ++k)
        if (!isfinite(delay_bins[k])) return fail(IC_EINVAL, "delay[%zu] is not finite", k);
    // one delay row for every subint: the channel table (the same phasors)
    bool rows_equal = true;
    for (int sb = 1; sb < nsub && rows_equal; ++sb)
        rows_equal = memcmp(delay_bins, delay_bins + (size_t)sb * nchan, sizeof(double) * nchan) == 0;
    if (rows_equal) return ic_set_delays(session, delay_bins);
    CK(hipSetDevice(s->device));
    if (!s->delay2 && hipMalloc((void **)&s->delay2, sizeof(double) * s->P) != hipSuccess) {
        s->delay2 = nullptr;
        return fail(IC_ENOMEM, "hipMalloc(per-profile delays) failed");
    }
    CK(hipMemcpyAsync(s->delay2, delay_bins, sizeof(double) * s->P, hipMemcpyHostToDevice, s->stream));
    CK(hipStreamSynchronize(s->stream));
    s->delays_set = true;
    return IC_OK;
}

namespace {
// ic_rotate_profiles(2): per_profile = 0: delay_bins [nchan] (the phasor
// table), 1: [nsub*nchan] (phasors evaluated per profile in the kernel)
int rotate_profiles(int device, int nsub, int nchan, int nbin, const float *in, const double *delay_bins,
                    int per_profile, int sign, float *out)
{
    if (!in || !delay_bins || !out || nsub <= 0 || nchan <= 0) return fail(IC_EINVAL, "bad argument");
    if (!rotate_supported(nbin))
        return fail(IC_EINVAL, "fractional dedispersion needs a power-of-two nbin in 64..4096 (nbin=%d)", nbin);
    if (sign != 1 && sign != -1) return fail(IC_EINVAL, "sign must be +1 or -1");
    const size_t nd = per_profile ? (size_t)nsub * nchan : (size_t)nchan;
    for (size_t c = 0; c < nd; ++c)
        if (!isfinite(delay_bins[c])) return fail(IC_EINVAL, "delay[%zu] is not finite", c);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(IC_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(IC_EINVAL, "device %d out of range (%d devices)", device, ndev);
    CK(hipSetDevice(device));
    const size_t N = (size_t)nsub * nchan * nbin;
    const std::vector<float> ph = per_profile ? std::vector<float>(2) : make_phasors(nbin, nchan, delay_bins);
    std::vector<double2> tw(nbin);
    for (int q = 0; q < nbin; ++q) {
        const long double ang = -2.0L * 3.141592653589793238462643383279502884L * (long double)q / (long double)nbin;
        tw[q] = make_double2((double)cosl(ang), (double)sinl(ang));
    }
    const std::vector<double2> tw2 = p2_twiddles(nbin);   // the rotation's stage tables
    float *d = nullptr;
    float *dph = nullptr;
    double2 *dtw = nullptr, *dtw2 = nullptr;
    double *ddl = nullptr;
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc((void **)&d, sizeof(float) * N);
    if (e == hipSuccess && per_profile) e = hipMalloc((void **)&ddl, sizeof(double) * nd);
    if (e == hipSuccess && per_profile)
        e = hipMemcpyAsync(ddl, delay_bins, sizeof(double) * nd, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMalloc((void **)&dph, sizeof(float) * ph.size());
    if (e == hipSuccess) e = hipMalloc((void **)&dtw, sizeof(double2) * tw.size());
    if (e == hipSuccess) e = hipMemcpyAsync(d, in, sizeof(float) * N, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dph, ph.data(), sizeof(float) * ph.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(dtw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMalloc((void **)&dtw2, sizeof(double2) * tw2.size());
    if (e == hipSuccess) e = hipMemcpyAsync(dtw2, tw2.data(), sizeof(double2) * tw2.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        RotateArgs a{};
        a.in = d;
        a.ld_in = nbin;
        a.ph = per_profile ? nullptr : dph;
        a.delay2 = ddl;
        a.sign = sign;
        a.tw = dtw;
        a.tw_p2 = dtw2;
        a.nsub = nsub;
        a.nchan = nchan;
        a.nbin = nbin;
        a.out = d;
        a.ldo = nbin;
        e = launch_rotate(st, a);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(float) * N, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (d) (void)hipFree(d);
    if (dph) (void)hipFree(dph);
    if (dtw) (void)hipFree(dtw);
    if (dtw2) (void)hipFree(dtw2);
    if (ddl) (void)hipFree(ddl);
    if (st) (void)hipStreamDestroy(st);
    if (e != hipSuccess) return fail(IC_EHIP, "ic_rotate_profiles: %s", hipGetErrorString(e));
    return IC_OK;
}
}  // namespace

int ic_rotate_profiles(int device, int nsub, int nchan, int nbin, const float *in, const double *delay_bins,
                       int sign, float *out)
{
    return rotate_profiles(device, nsub, nchan, nbin, in, delay_bins, 0, sign, out);
}

int ic_rotate_profiles2(int device, int nsub, int nchan, int nbin, const float *in, const double *delay_bins,
                        int sign, float *out)
{
    return rotate_profiles(device, nsub, nchan, nbin, in, delay_bins, 1, sign, out);
}

int ic_get_bad_fits(void *session, int32_t *per_iter, int n)
{
    Session *s = (Session *)session;
    if (!s || (!per_iter && n > 0)) return fail(IC_EINVAL, "null argument");
    const int m = (int)s->bad_fits.size();
    for (int q = 0; q < m && q < n; ++q) per_iter[q] = s->bad_fits[q];
    return m;
}

int ic_set_fit_tail(void *session, int64_t threshold) { return ic_set_option(session, IC_OPT_FIT_TAIL, threshold); }

// Schedule options (include/iterative_cleaner.h): validated here, read by the
// next ic_run; every setting gives the same bits.
int ic_set_option(void *session, int option, int64_t v)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null session");
    if (s->failed) return fail(IC_ESTATE, "session failed (a host wait timed out); destroy it");
    switch (option) {
    case IC_OPT_FIT_TAIL:
        if (v < 0) return fail(IC_EINVAL, "IC_OPT_FIT_TAIL=%lld < 0", (long long)v);
        s->tail_threshold = (long)v;
        return IC_OK;
    case IC_OPT_DIAG_FORK:
        if (v < 0 || v > 64) return fail(IC_EINVAL, "IC_OPT_DIAG_FORK=%lld outside 0..64", (long long)v);
        if (v > 0 && s->p.fit_mode != IC_FIT_EXACT) return fail(IC_EINVAL, "IC_OPT_DIAG_FORK needs the exact fit");
        s->diag_fork = (int)v;
        return IC_OK;
    case IC_OPT_FORK_DELAY:
        if (v < 0 || v > 8) return fail(IC_EINVAL, "IC_OPT_FORK_DELAY=%lld outside 0..8", (long long)v);
        s->fork_delay = (int)v;
        return IC_OK;
    case IC_OPT_TEMPLATE_INCR:
        if (v != 0 && v != 1) return fail(IC_EINVAL, "IC_OPT_TEMPLATE_INCR=%lld (0 or 1)", (long long)v);
        s->incr = v != 0;
        return IC_OK;
    case IC_OPT_FIT_TILED:
        if (v != 0 && v != 1) return fail(IC_EINVAL, "IC_OPT_FIT_TILED=%lld (0 or 1)", (long long)v);
        if (v && s->fftded && s->p.fit_mode != IC_FIT_EXACT)
            return fail(IC_EINVAL, "IC_OPT_FIT_TILED: the closed-form fit of the FFT mode reads a row-major cube");
        // the fit cube of the last run is in the old layout: its residual
        // (ic_get_residual, the FFT mode's rotation) waits for the next run
        if ((int)v != s->dtiled) s->ran = false;
        s->dtiled = (int)v;
        return IC_OK;
    case IC_OPT_ROWSTAT_WAVES:
        if (v != 0 && v != 4 && v != 8) return fail(IC_EINVAL, "IC_OPT_ROWSTAT_WAVES=%lld (0, 4 or 8)", (long long)v);
        s->ls_knobs.grp_waves = (int)v;
        return IC_OK;
    case IC_OPT_ROWSTAT_MINLEN:
        if (v < 1 || v > 16384) return fail(IC_EINVAL, "IC_OPT_ROWSTAT_MINLEN=%lld outside 1..16384", (long long)v);
        s->ls_knobs.grp_minlen = (int)v;
        return IC_OK;
    case IC_OPT_DIAG_CHAIN:
        if (v != 0 && v != 1) return fail(IC_EINVAL, "IC_OPT_DIAG_CHAIN=%lld (0 or 1)", (long long)v);
        s->diag_chain = v != 0;
        return IC_OK;
    case IC_OPT_SYNC_TIMEOUT_MS:
        if (v < 1) return fail(IC_EINVAL, "IC_OPT_SYNC_TIMEOUT_MS=%lld < 1", (long long)v);
        s->sync_timeout_s = (double)v / 1000.0;
        if (s->comm) s->comm->set_timeout_ms((long long)v);
        return IC_OK;
    case IC_OPT_FIT_SCHEDULE:
        // the persistent lanes schedule (round 4, measured slower than the
        // rounds) was removed in round 5: only the rounds remain
        if (v != IC_FIT_ROUNDS) return fail(IC_EINVAL, "IC_OPT_FIT_SCHEDULE=%lld (only IC_FIT_ROUNDS)", (long long)v);
        return IC_OK;
    case IC_OPT_TAIL_SPLIT:
        if (v < 0 || v > 2) return fail(IC_EINVAL, "IC_OPT_TAIL_SPLIT=%lld (0, 1 or 2)", (long long)v);
        s->tail_split_mode = (int)v;
        return IC_OK;
    case IC_OPT_ROT_STATS:
        if (v != 0 && v != 1) return fail(IC_EINVAL, "IC_OPT_ROT_STATS=%lld (0 or 1)", (long long)v);
        s->rot_stats = v != 0;
        return IC_OK;
    default:
        return fail(IC_EINVAL, "unknown option %d", option);
    }
}

int ic_get_option(void *session, int option, int64_t *out)
{
    Session *s = (Session *)session;
    if (!s || !out) return fail(IC_EINVAL, "null argument");
    switch (option) {
    case IC_OPT_FIT_TAIL: *out = s->tail_threshold; return IC_OK;
    case IC_OPT_DIAG_FORK: *out = s->diag_fork; return IC_OK;
    case IC_OPT_FORK_DELAY: *out = s->fork_delay; return IC_OK;
    case IC_OPT_TEMPLATE_INCR: *out = s->incr ? 1 : 0; return IC_OK;
    case IC_OPT_FIT_TILED: *out = s->dtiled; return IC_OK;
    case IC_OPT_ROWSTAT_WAVES: *out = s->ls_knobs.grp_waves; return IC_OK;
    case IC_OPT_ROWSTAT_MINLEN: *out = s->ls_knobs.grp_minlen; return IC_OK;
    case IC_OPT_DIAG_CHAIN: *out = s->diag_chain ? 1 : 0; return IC_OK;
    case IC_OPT_SYNC_TIMEOUT_MS: *out = (int64_t)(s->sync_timeout_s * 1000.0 + 0.5); return IC_OK;
    case IC_OPT_FIT_SCHEDULE: *out = IC_FIT_ROUNDS; return IC_OK;
    case IC_OPT_TAIL_SPLIT: *out = s->tail_split_mode; return IC_OK;
    case IC_OPT_ROT_STATS: *out = s->rot_stats ? 1 : 0; return IC_OK;
    default: return fail(IC_EINVAL, "unknown option %d", option);
    }
}

int ic_get_run_stats(void *session, ic_run_stats *out)
{
    Session *s = (Session *)session;
    if (!s || !out) return fail(IC_EINVAL, "null argument");
    *out = s->stats;
    return IC_OK;
}

int ic_get_template(void *session, float *T)
{
    Session *s = (Session *)session;
    if (!s || !T) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->ran) return fail(IC_ESTATE, "no completed iteration");
    CK(hipMemcpyAsync(T, s->T, sizeof(float) * s->p.nbin, hipMemcpyDeviceToHost, s->stream));
    CK(hipStreamSynchronize(s->stream));
    return IC_OK;
}

int ic_get_fit(void *session, double *amp, int32_t *info)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->ran) return fail(IC_ESTATE, "no completed iteration");
    if (amp) CK(hipMemcpyAsync(amp, s->amp, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    if (info) CK(hipMemcpyAsync(info, s->info, sizeof(int32_t) * s->P, hipMemcpyDeviceToHost, s->stream));
    CK(hipStreamSynchronize(s->stream));
    return IC_OK;
}

int ic_get_diagnostics_f64(void *session, double *std_o, double *mean_o, double *ptp_o, double *fftmax_o)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null argument");
    if (s->failed) return failed_session();
    if (!s->ran) return fail(IC_ESTATE, "no completed iteration");
    if (std_o) CK(hipMemcpyAsync(std_o, s->std_, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    if (mean_o) CK(hipMemcpyAsync(mean_o, s->mean, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    if (ptp_o) CK(hipMemcpyAsync(ptp_o, s->ptp, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    if (fftmax_o) CK(hipMemcpyAsync(fftmax_o, s->fft, sizeof(double) * s->P, hipMemcpyDeviceToHost, s->stream));
    CK(hipStreamSynchronize(s->stream));
    return IC_OK;
}

int ic_get_diagnostics(void *session, double *std_o, double *mean_o, float *ptp_o, double *fftmax_o)
{
    Session *s = (Session *)session;
    if (!s) return fail(IC_EINVAL, "null argument");
    std::vector<double> ptp(ptp_o ? s->P : 0);
    if (int rc = ic_get_diagnostics_f64(session, std_o, mean_o, ptp_o ? ptp.data() : nullptr, fftmax_o)) return rc;
    for (size_t k = 0; k < ptp.size(); ++k) ptp_o[k] = (float)ptp[k];   // exact unless data_f64
    return IC_OK;
}

// comprehensive_stats alone (iterative_cleaner.py:181-226 on the data of
// :111-117): one-shot device buffers, the diagnostics kernel in DIAG_STATS mode,
// the line medians and the combine of one "iteration" (weights/history unused).
int ic_comprehensive_stats(int device, int nsub, int nchan, int nbin, const float *data, const float *weights,
                           double chanthresh, double subintthresh, double *test_out, double *std_o, double *mean_o,
                           float *ptp_o, double *fftmax_o)
{
    return ic_comprehensive_stats_rowstat(device, nsub, nchan, nbin, data, weights, chanthresh, subintthresh,
                                          test_out, std_o, mean_o, ptp_o, fftmax_o, 8, 1024);
}

int ic_comprehensive_stats_rowstat(int device, int nsub, int nchan, int nbin, const float *data,
                                   const float *weights, double chanthresh, double subintthresh, double *test_out,
                                   double *std_o, double *mean_o, float *ptp_o, double *fftmax_o, int rowstat_waves,
                                   int rowstat_minlen)
{
    if (!data || !weights || !test_out) return fail(IC_EINVAL, "null argument");
    if (rowstat_waves != 0 && rowstat_waves != 4 && rowstat_waves != 8)
        return fail(IC_EINVAL, "rowstat_waves=%d (0, 4 or 8)", rowstat_waves);
    if (rowstat_minlen < 1) return fail(IC_EINVAL, "rowstat_minlen=%d < 1", rowstat_minlen);
    if (nsub <= 0 || nchan <= 0 || nbin <= 0 || nsub > 16384 || nchan > 16384 || nbin > 32768)
        return fail(IC_EINVAL, "bad shape nsub=%d nchan=%d nbin=%d", nsub, nchan, nbin);
    if (diag_lds_bytes(nbin) > 160 * 1024) return fail(IC_EINVAL, "nbin=%d unsupported", nbin);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(IC_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(IC_EINVAL, "device %d out of range (%d devices)", device, ndev);
    CK(hipSetDevice(device));
    const size_t P = (size_t)nsub * nchan, N = P * (size_t)nbin;
    PwPlan plan;
    if (make_plan(nbin, &plan) != 0) return fail(IC_EINVAL, "pairwise plan too large for nbin=%d", nbin);
    std::vector<double2> tw(nbin);
    for (int q = 0; q < nbin; ++q) {
        const long double ang = -2.0L * 3.141592653589793238462643383279502884L * (long double)q / (long double)nbin;
        tw[q] = make_double2((double)cosl(ang), (double)sinl(ang));
    }
    const std::vector<double2> tw2 = p2_twiddles(nbin);
    struct Buf {
        void *p = nullptr;
        ~Buf() { if (p) (void)hipFree(p); }
    } bD, bw, bvalid, bW, bhist, bstd, bmean, bfft, bptp, btest, blstat, bcnt, btw, btw2, bplan;
    hipStream_t st = nullptr;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{st};
    struct {
        Buf *b;
        size_t bytes;
    } al[] = {{&bD, 4 * N},       {&bw, 4 * P},      {&bvalid, P},      {&bW, 4 * P},
              {&bhist, 8 * P},    {&bstd, 8 * P},    {&bmean, 8 * P},   {&bfft, 8 * P},
              {&bptp, 8 * P},     {&btest, 8 * P},   {&blstat, 8 * 16 * ((size_t)nsub + nchan)},
              {&bcnt, 4 * 8},     {&btw, 16 * (size_t)nbin}, {&btw2, 16 * (size_t)nbin + 16}, {&bplan, sizeof plan}};
    for (auto &x : al)
        if (hipMalloc(&x.b->p, x.bytes + 16) != hipSuccess) return fail(IC_ENOMEM, "hipMalloc(%zu) failed", x.bytes);
    float *D = (float *)bD.p, *w0 = (float *)bw.p, *W = (float *)bW.p, *hist = (float *)bhist.p;
    uint8_t *valid = (uint8_t *)bvalid.p;
    double *sd = (double *)bstd.p, *mn = (double *)bmean.p, *ff = (double *)bfft.p, *test = (double *)btest.p;
    double *pt = (double *)bptp.p;
    double *lstat = (double *)blstat.p;
    int32_t *cnt = (int32_t *)bcnt.p;
    CK(hipMemcpyAsync(D, data, 4 * N, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(w0, weights, 4 * P, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(btw.p, tw.data(), 16 * (size_t)nbin, hipMemcpyHostToDevice, st));
    if (!tw2.empty()) CK(hipMemcpyAsync(btw2.p, tw2.data(), 16 * tw2.size(), hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(bplan.p, &plan, sizeof plan, hipMemcpyHostToDevice, st));
    CK(hipMemsetAsync(cnt, 0, 4 * 8, st));
    IC_GGL(k_valid, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, w0, valid, W, hist, P);
    CK(hipGetLastError());
    DiagArgs a{};
    a.mode = DIAG_STATS;
    a.D = D;
    a.ldD = nbin;
    a.w0 = w0;
    a.tw = (const double2 *)btw.p;
    a.tw_p2 = (const double2 *)btw2.p;
    a.plan = (const PwPlan *)bplan.p;
    a.nsub = nsub;
    a.nchan = nchan;
    a.nbin = nbin;
    a.std_o = sd;
    a.mean_o = mn;
    a.fft_o = ff;
    a.ptp_o = pt;
    CK(launch_diag(st, a));
    LineStatsArgs la;
    la.nsub = nsub;
    la.nchan = nchan;
    la.valid = valid;
    la.std_d = sd;
    la.mean_d = mn;
    la.fft_d = ff;
    la.ptp_d = pt;
    la.ptp_f32 = 1;
    la.grp_waves = rowstat_waves;
    la.grp_minlen = rowstat_minlen;
    la.col_med = lstat;
    la.col_mad = lstat + 4 * nchan;
    la.row_med = lstat + 8 * nchan;
    la.row_mad = lstat + 8 * nchan + 4 * nsub;
    CK(launch_linestats(st, la, 3));
    CK(launch_combine(st, nsub, nchan, valid, nullptr, w0, sd, mn, pt, 1, ff, la.col_med, la.col_mad, la.row_med, la.row_mad,
                      chanthresh, subintthresh, test, W, hist, 1, cnt));
    CK(hipMemcpyAsync(test_out, test, 8 * P, hipMemcpyDeviceToHost, st));
    if (std_o) CK(hipMemcpyAsync(std_o, sd, 8 * P, hipMemcpyDeviceToHost, st));
    if (mean_o) CK(hipMemcpyAsync(mean_o, mn, 8 * P, hipMemcpyDeviceToHost, st));
    std::vector<double> ptp64(ptp_o ? P : 0);
    if (ptp_o) CK(hipMemcpyAsync(ptp64.data(), pt, 8 * P, hipMemcpyDeviceToHost, st));
    if (fftmax_o) CK(hipMemcpyAsync(fftmax_o, ff, 8 * P, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    for (size_t k = 0; k < ptp64.size(); ++k) ptp_o[k] = (float)ptp64[k];
    return IC_OK;
}

// remove_profile1d (iterative_cleaner.py:275-288) over caller-given profiles:
// a one-shot session of nsub x nchan >= nprof profiles (zero rows pad the last
// subint) whose fit cube is the profiles themselves, then the session's fit
// (exact: run_fit; closed form: the fused kernel on raw rows with a zero
// baseline) and k_residual with no dispersion shift.
int ic_fit_profiles(int device, int nprof, int nbin, const float *T, const float *profiles, int fit_mode,
                    double *amp_out, int32_t *info_out, float *resid_out)
{
    if (!T || !profiles || (!amp_out && !info_out && !resid_out)) return fail(IC_EINVAL, "null argument");
    if (nprof <= 0 || nbin <= 0) return fail(IC_EINVAL, "bad shape nprof=%d nbin=%d", nprof, nbin);
    ic_params p{};
    p.nchan = nprof < 4096 ? nprof : 4096;
    p.nsub = (nprof + p.nchan - 1) / p.nchan;
    p.nbin = nbin;
    p.max_iter = 1;
    p.chanthresh = p.subintthresh = 5.0;
    p.baseline_duty = 0.15;
    p.fit_mode = fit_mode;
    void *h = nullptr;
    int rc = create_session(&p, device, 0, 1, false, [](std::string *, int *) -> Comm * { return nullptr; }, &h);
    if (rc) return rc;
    Session *s = (Session *)h;
    struct Guard {
        Session *s;
        ~Guard() { ic_session_destroy(s); }
    } guard{s};
    s->dtiled = 0;   // D is filled row by row below
    const size_t P = s->P, row = sizeof(float) * (size_t)nbin;
    std::vector<double> t64(s->ldD, 0.0);
    for (int i = 0; i < nbin; ++i) t64[i] = (double)T[i];
    CK(hipMemcpyAsync(s->T64, t64.data(), sizeof(double) * s->ldD, hipMemcpyHostToDevice, s->stream));
    CK(hipMemcpyAsync(s->T2, t64.data(), sizeof(double) * nbin, hipMemcpyHostToDevice, s->stream));
    CK(hipMemcpyAsync(s->T2 + nbin, t64.data(), sizeof(double) * nbin, hipMemcpyHostToDevice, s->stream));
    CK(hipMemsetAsync(s->shift, 0, sizeof(int32_t) * s->nchan, s->stream));
    CK(hipMemsetAsync(s->base0, 0, sizeof(float) * P, s->stream));
    {
        std::vector<float> ones(P, 1.0f);
        CK(hipMemcpyAsync(s->w0, ones.data(), sizeof(float) * P, hipMemcpyHostToDevice, s->stream));
        CK(hipStreamSynchronize(s->stream));
    }
    CK(hipMemsetAsync(s->raw, 0, sizeof(float) * s->N, s->stream));
    CK(hipMemcpyAsync(s->raw, profiles, row * nprof, hipMemcpyHostToDevice, s->stream));
    if (fit_mode == IC_FIT_EXACT) {
        CK(hipMemcpy2DAsync(s->D, sizeof(float) * s->ldD, s->raw, row, row, P, hipMemcpyDeviceToDevice, s->stream));
        if (int r = run_fit(s, nullptr)) return r;
    } else {
        CK(launch_tnorm(s->stream, s->T64, s->plan, s->plan_ub, s->TT));
        DiagArgs da = diag_args(s, 0, 0);
        CK(launch_diag(s->stream, da));
    }
    if (amp_out) CK(hipMemcpyAsync(amp_out, s->amp, sizeof(double) * nprof, hipMemcpyDeviceToHost, s->stream));
    if (info_out) CK(hipMemcpyAsync(info_out, s->info, sizeof(int32_t) * nprof, hipMemcpyDeviceToHost, s->stream));
    if (resid_out) {
        float *R = nullptr;
        CK(hipMalloc((void **)&R, sizeof(float) * s->N));
        hipError_t e = launch_residual(s->stream, s->D, s->raw, s->base0, s->T64, s->amp, s->info, s->shift, p.nsub,
                                       s->nchan, nbin, s->ldD, s->dtiled, 0, 1.0, 0, 0, R);
        if (e == hipSuccess) e = hipMemcpyAsync(resid_out, R, row * nprof, hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        (void)hipFree(R);
        if (e != hipSuccess) return fail(IC_EHIP, "ic_fit_profiles residual: %s", hipGetErrorString(e));
    }
    CK(hipStreamSynchronize(s->stream));
    return IC_OK;
}

}  // extern "C"
