// ic_internal.h — shared declarations between the host session (ic_session.hip)
// and the gfx950 kernels (ic_kernels.hip).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace icgpu {

// Kernel timing on the dispatch packet itself.  The session's LAUNCH macro
// parks a start/stop event pair here; the first IC_GGL of the launch wrapper
// it calls dispatches through hipExtLaunchKernelGGL, whose packet records
// both timestamps, so a timed kernel costs no extra marker packets (C2, the
// bench's timed region with k_fit_pass timed: 27.74 ms per clean with a
// hipEventRecord pair around each launch, 27.62 with the packet's own).
// Further kernels of the same wrapper are counted in `extra`; the session
// then ends the interval with a marker after the wrapper.
struct PendingTiming {
    hipEvent_t a = nullptr, b = nullptr;
    int used = 0, extra = 0;
};
extern thread_local PendingTiming g_timing;
#define IC_GGL(K, GRID, BLOCK, SHM, ST, ...)                                                                 \
    do {                                                                                                    \
        if (::icgpu::g_timing.a && !::icgpu::g_timing.used) {                                               \
            ::icgpu::g_timing.used = 1;                                                                     \
            hipExtLaunchKernelGGL(K, GRID, BLOCK, SHM, ST, ::icgpu::g_timing.a, ::icgpu::g_timing.b, 0,      \
                                  __VA_ARGS__);                                                             \
        } else {                                                                                            \
            if (::icgpu::g_timing.a) ++::icgpu::g_timing.extra;                                             \
            hipLaunchKernelGGL(K, GRID, BLOCK, SHM, ST, __VA_ARGS__);                                       \
        }                                                                                                   \
    } while (0)

constexpr int kSuperBlock = 256;    // canonical channel super-block (archive.py SUPER_BLOCK)
constexpr int kMaxLeaves = 256;     // pairwise-sum leaves (nbin <= 32768)
constexpr int kFitTile = 32;        // bins per k_fit_pass LDS tile (fit cube row padding)

// Tiled fit cube (dtiled): profiles in groups of 64 (one k_fit_pass wave),
// each group stored as ldD/32 tiles of [64 profiles][32 bins] (8 KiB), so a
// wave's 32-bin step of its 64 rows is one contiguous 8-KiB block instead of
// 64 lines 4 KiB apart.  Element (k, i) of a cube with row length ldD
// (a multiple of 32, profiles padded to a multiple of 64):
__host__ __device__ inline size_t dt_ofs(size_t k, int i, int ldD)
{
    return (((k >> 6) * (size_t)(ldD >> 5) + (size_t)(i >> 5)) << 11) + ((k & 63) << 5) + (size_t)(i & 31);
}
// element (k, i) of the fit cube in either layout
__host__ __device__ inline size_t d_ofs(size_t k, int i, int ldD, int dtiled)
{
    return dtiled ? dt_ofs(k, i, ldD) : k * (size_t)ldD + (size_t)i;
}

// Canonical combine of super-block partials (archive.py sb_tree): the halving
// tree over n leaves, evaluated as a post-order stack program: push leaf j,
// then merge the two top entries merges[j] times.  n <= kMaxSbLeaves (nchan <=
// 16384); the stack never holds more than 1 + log2(n) <= 7 entries.
constexpr int kMaxSbLeaves = 64;
struct SbPlan {
    int32_t n;
    uint8_t merges[kMaxSbLeaves];
};

// Row/column geometry of a channel shard's exchanges (world <= kMaxShards):
// rank r owns channels [chan0[r], chan0[r+1]) and subint rows [row0[r], row0[r+1]).
constexpr int kMaxShards = 64;
struct ShardGeom {
    int32_t world, rank, nsub, nchan_g;
    int32_t chan0[kMaxShards + 1];
    int32_t row0[kMaxShards + 1];
};

// bytes of one exchange block of n elements of esz bytes (32 = std+mean+fft+ptp),
// padded so that every block, and the f64 fields inside it, start 8-aligned
__host__ __device__ inline size_t shard_block_bytes(size_t n, size_t esz) { return ((n * esz + 7) / 8) * 8; }

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
    K_FSCRUNCH,
    K_TSCRUNCH,
    K_FIT_PASS,
    K_FIT_STATE,
    K_DIAG,
    K_LINESTATS,
    K_COMBINE,
    K_RESIDUAL,
    K_FIT_TAIL,
    K_SB_TREE,
    K_SHARD_PACK,     // pack / assemble / unpack of shard exchanges
    K_EXCHANGE,       // the collectives themselves (host transport or peer copies)
    K_TNORM,          // fit_mode 1: sum(T*T)
    K_ROTATE,         // fractional dedispersion (FFT phase rotation)
    K_COUNT
};

// lmdif per-profile state (structure of arrays, device memory)
struct FitStateArrays {
    double *x, *fnorm, *par, *delta, *diag, *xnorm, *acnorm, *J0, *f0, *aj, *r, *Jn0, *qtf, *gnorm,
        *x2, *pnorm, *wa1, *xa;
    int32_t *iter, *nfev, *mode, *slow;
    // sweep outputs (k_fit_pass -> k_fit_state): the norms carry the flags in
    // their sign bits (fnorm: the A sweep took the exact path; acnorm: J(1) ==
    // T in round 0), o_sum the dot of a B sweep (or round 0's fused one).
    // The two norms are stored as one double2 (fnorm, acnorm) per profile,
    // ((double2 *)o_fnorm)[k], over the o_fnorm and o_acnorm arrays (adjacent,
    // 2 x 8P bytes): one 16-B store per A sweep
    double *o_fnorm, *o_acnorm, *o_sum;
    float *p0;            // first sample of every profile's fit-cube row (round 0)
    const double *T64;    // the iteration's template (k_fit_state recomputes f0 / J0 from it)
    // the first outer iteration's profile-independent qrfac (k_fit_prep): U = {valid, acnorm, aj, Jn0}
    double *U;
};

struct LineStatsArgs {
    int nsub, nchan;
    const uint8_t *valid;
    const double *std_d, *mean_d, *fft_d;
    const double *ptp_d;            // ptp (f32 values unless data_f64)
    int ptp_f32;                    // 1: ptp lines use f32 arithmetic (numpy.ma on f32 data)
    double *col_med, *col_mad;      // [4][nchan]
    double *row_med, *row_mad;      // [4][nsub]
    // row-median form (session options IC_OPT_ROWSTAT_WAVES / _MINLEN, checked
    // when set): grp_waves waves per line (0 = one wave per line, 4 or 8) for
    // rows of >= grp_minlen values
    int grp_waves = 8, grp_minlen = 1024;
};

// ---- launch wrappers (ic_kernels.hip); all asynchronous on `st` ----
// mode 0: part = sum W*ded; 1: part2 = sum W*f32(ded-base) + wpart; 2: both;
// 3: mode 1 + the fit cube D[k][i] = f32(ded-base) (row stride ldD).
// flags: only subints with flags[s] != 0 (nullptr: all)
hipError_t launch_chan_partials(hipStream_t st, int mode, const float *raw, const float *W, const int32_t *shift,
                                const float *base, const int32_t *flags, int nsub, int nchan, int nbin,
                                double *part, double *part2, double *wpart, float *D = nullptr, int ldD = 0,
                                int dtiled = 0, uint8_t *exA = nullptr, uint8_t *exF = nullptr);
// exA / exF (optional): per column [s][sb][i] 1 = its part / part2 sum is
// exact in any order with weights 0 / 1 (k_chan_partials' ExTrack), the
// condition for launch_chan_delta.  Iteration >= 2 (Wn = this iteration's weights, Wo = the
// previous one's): part, part2 (carried levels) and wpart moved from Wo to Wn
// through the changed channels only; inexact columns summed again in full.
// rawF (FFT dedispersion): part2's terms are f32(rawF - base) instead of
// f32(raw - base) (part's stay raw's).
hipError_t launch_chan_delta(hipStream_t st, const float *raw, const int32_t *shift, const float *base,
                             const float *Wn, const float *Wo, int nsub, int nchan, int nbin, double *part,
                             double *part2, double *wpart, const uint8_t *exA, const uint8_t *exF,
                             const float *rawF = nullptr);
// flags != nullptr: flags[s] = window of subint s moved (win updated in place)
// element (s, leaf, i) of `part` is part[s*ss + leaf*sl + i]; the leaves are
// combined with `plan` (single device: the nsb super-blocks; sharded: the
// gathered shard roots)
hipError_t launch_window(hipStream_t st, const double *part, long ss, long sl, const SbPlan &plan, int nsub,
                         int nbin, int width, int32_t *win, int32_t *flags);
// dynamic LDS of k_window (nbin doubles + per-thread partials)
size_t window_lds_bytes(int nbin);
// flags != nullptr: only subints with flags[s] != 0
hipError_t launch_base(hipStream_t st, const float *raw, const int32_t *shift, const int32_t *win,
                       const int32_t *flags, int nsub, int nchan, int nbin, int width, float *base);
// total intensity in place: raw[i] = f32(raw[i] + pol1[i])  (archive.py pscrunch)
hipError_t launch_pscrunch(hipStream_t st, float *raw, const float *pol1, size_t n);
// num (s, leaf, i) = part[s*ss + leaf*sl + i], weight (s, leaf) = wpart[s*wss + leaf*wsl]
hipError_t launch_fscrunch(hipStream_t st, const double *part, long ss, long sl, const double *wpart, long wss,
                           long wsl, const SbPlan &plan, int nsub, int nbin, float *F, float *wf);
// shard root of the local super-block partials, one row of ostr doubles per
// subint: out[s*ostr + i] = tree(part[s][*][i]), out[s*ostr + nbin] =
// tree(wpart[s][*]) (wpart may be null)
hipError_t launch_sb_tree(hipStream_t st, const double *part, const double *wpart, const SbPlan &plan, int nsub,
                          int nbin, long ostr, double *out);
// windows / fscrunch rows all-gathered from the row owners -> full arrays
hipError_t launch_unpack_windows(hipStream_t st, const ShardGeom &g, int blk, const int32_t *recv, int32_t *win,
                                 int32_t *flags);
hipError_t launch_unpack_fscrunch(hipStream_t st, const ShardGeom &g, int rows_pad, long blk, int nbin,
                                  const float *recv, float *F, float *wf);
// diagnostics rows -> per-destination blocks [std|mean|fft|ptp (f64)] x rows_d x nchan_loc
// (valid == true: the single u8 field `valid` instead)
hipError_t launch_pack_rows(hipStream_t st, const ShardGeom &g, int nchan_loc, const double *std_d,
                            const double *mean_d, const double *fft_d, const double *ptp_d, const uint8_t *valid,
                            unsigned char *send);
// per-source blocks -> owned rows [rows_own][nchan_g] of each field
hipError_t launch_assemble_rows(hipStream_t st, const ShardGeom &g, const unsigned char *recv, double *std_r,
                                double *mean_r, double *fft_r, double *ptp_r, uint8_t *valid_r);
// gathered [world][8 * rows_pad] (rank p: med [4][rows_p], mad [4][rows_p]) -> row_med/row_mad [4][nsub]
hipError_t launch_unpack_rowstats(hipStream_t st, const ShardGeom &g, int rows_pad, const double *recv,
                                  double *row_med, double *row_mad);
// buf[i] = sum_r gathered[r][i]
hipError_t launch_sum_i32(hipStream_t st, const int32_t *gathered, int world, int n, int32_t *buf);
// T2 (optional): [2 nbin] receives T64[0..nbin) twice
hipError_t launch_tscrunch(hipStream_t st, const float *F, const float *wf, int nsub, int nbin, float *T,
                           double *T64, double *T2 = nullptr);
hipError_t launch_fit_init(hipStream_t st, const FitStateArrays &S, long P, int32_t *z32 = nullptr,
                           int nz32 = 0, uint8_t *late = nullptr);
// S.U from the template (one block; before round 0 of every fit)
hipError_t launch_fit_prep(hipStream_t st, const FitStateArrays &S, const double *T64, int nbin);
// Round counters of the exact fit (Session::rcount, int32 words): [0, 2K) the
// packed list counts of every round (u64: [63:32] B requests at the list's
// end, [31:0] A requests at its front), [2K, 3K) the blocks of each round's
// k_fit_state that finished (u32), then the tail's sweep counter (u64, zeroed
// once per run).  k_fit_init zeroes the first 3K words every iteration.
constexpr int kMaxRounds = 1024;   // lmdif rounds per fit (maxfev = 400 bounds it far below)
constexpr int kRoundWords = 3 * kMaxRounds;
// list == nullptr: all P profiles (round 0); else the list written by the
// previous round's k_fit_state, partitioned by request: nctr -> its packed
// counts (above), their sum <= bound (the host sizes grids from a count it
// already knows: counts only shrink).
// m[k] = v for the profiles of a round list (at most `bound` entries)
hipError_t launch_mark_list(hipStream_t st, const int32_t *list, const unsigned long long *nctr, long P, long bound,
                            uint8_t *m, uint8_t v);
hipError_t launch_fit_pass(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           int dtiled, const int32_t *list, const unsigned long long *nctr, long bound,
                           const FitStateArrays &S, bool round0);
// ctr: zeroed device word, packed [63:32] B survivors, [31:0] A survivors
// (the next round's nctr); done: zeroed word counting the finished blocks;
// host_n: host-mapped int the last block writes the survivor total to.
// round0 (launch_fit_pass): the first round (list == nullptr: every profile
// at x = 1, the fused first B sweep).
hipError_t launch_fit_state(hipStream_t st, const FitStateArrays &S, long P, const int32_t *list,
                            const unsigned long long *nctr, long bound, double *amp, int32_t *info,
                            int32_t *next_list, unsigned long long *ctr, unsigned *done, int32_t *host_n,
                            uint8_t *late = nullptr);
hipError_t launch_fit_tail(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           int dtiled, const int32_t *list, const unsigned long long *nctr, long bound,
                           const FitStateArrays &S, double *amp, int32_t *info, unsigned long long *sweeps);
// Diagnostics kernels (k_diag_p2<N> for power-of-two nbin 64..4096, k_diag
// otherwise).  mode: DIAG_EXACT = residual from the exact fit's amp/info and
// the fit cube D (row stride ldD); DIAG_CLOSED = fit_mode 1, the closed-form
// amplitude sum(T*p)/TT from raw + base (written to amp/info), then the same
// residual; DIAG_STATS = comprehensive_stats of the rows of D alone (no shift).
// tw: exp(-2 pi i q/nbin), q < nbin; tw_p2 (power-of-two nbin only): see p2_twiddles()
// DIAG_FIT = the closed-form amplitude alone (amp/info) of the rows of D (no
// shift, no level): fit_mode 1 with fractional dedispersion, whose residual is
// then rotated back and measured in DIAG_STATS.
enum DiagMode { DIAG_EXACT = 0, DIAG_CLOSED = 1, DIAG_STATS = 2, DIAG_FIT = 3 };
struct DiagArgs {
    int mode;
    const float *D;
    int ldD;
    const float *raw, *base;
    const double *T64, *TT;
    const double *T2;   // [2 nbin]: T64[0..nbin) twice (k_diag_cl's wrap-free gather), or null
    double *amp;
    int32_t *info;
    const float *w0;
    const int32_t *shift;
    const double2 *tw, *tw_p2;
    const PwPlan *plan;
    int nsub, nchan, nbin;
    int pr_on;
    double pr_factor;
    int pr_start, pr_end;
    double *std_o, *mean_o, *fft_o, *ptp_o;
    int data_f64;      // psrchive get_data returns f64: X = f64(R) * f64(w), f64 mean and ptp
    int dtiled;        // D is the tiled fit cube (dt_ofs); DIAG_STATS inputs are row-major
    // only the profiles of a list (the fork of the exact fit's diagnostics):
    // list + packed count as the fit rounds' (RoundList); nullptr = all
    const int32_t *list = nullptr;
    const unsigned long long *nctr = nullptr;
    const uint8_t *skip = nullptr;   // != nullptr: profiles with skip[k] != 0 are left out
    int chain = 1;   // 0: the row-layout k_diag_p2 at nbin 1024/2048/4096 too (IC_OPT_DIAG_CHAIN)
};
hipError_t launch_diag(hipStream_t st, const DiagArgs &a);
// the diagnostics kernel launch_diag picks for `a` takes a profile list
bool diag_list_supported(const DiagArgs &a);
// late != nullptr (launch_fit_state): late[k] = 1 for every survivor of the
// round (the fork round; the flags were zeroed before it)
// dynamic LDS the generic k_diag needs for one wave (0 for the power-of-two kernels)
size_t diag_lds_bytes(int nbin);
// *TT = numpy pairwise sum of T64[i]^2 over nbin (plan), nleaf_ub >= plan leaves/ops
hipError_t launch_tnorm(hipStream_t st, const double *T64, const PwPlan *plan, int nleaf_ub, double *TT);
// which: bit 0 = column lines (length nsub), bit 1 = row lines (length nchan)
hipError_t launch_linestats(hipStream_t st, const LineStatsArgs &a, int which = 3);
// counters: [0] changed, [1] zero weights, [2] fit statuses outside 1-4 (info
// may be null), [3] test values within 1e-9 of 1.0, [4+h] new weights !=
// history h (iterative_cleaner.py:127-141)
hipError_t launch_combine(hipStream_t st, int nsub, int nchan, const uint8_t *valid, const int32_t *info,
                          const float *w0,
                          const double *std_d, const double *mean_d, const double *ptp_d, int ptp_f32,
                          const double *fft_d, const double *col_med, const double *col_mad,
                          const double *row_med, const double *row_mad, double chanthresh,
                          double subintthresh, double *test, float *W, float *hist, int iter,
                          int32_t *counters);
// Phasor exp(+2 pi i k d / n) of harmonic k (0 <= k <= n/2) for a delay of d
// bins, n a power of two (<= 8192): the phase rotation's multiplier
// (phase_rotation.py phasors; oracle orc_phasor).  One fixed sequence of
// separately rounded f64 operations, so that the host's per-channel table
// (ic_set_delays), the device's per-profile evaluation (ic_set_delays2) and
// the two restatements agree bit for bit:
//   the delay is split (Veltkamp, 2^13 + 1) into dh (40 significant bits) and
//   dl, so k dh and k dl are exact; t = k dh - n rint(k dh / n) is exact and
//   |t| <= n/2; y = (t + k dl) 4/n counts quarter turns (one rounding); with
//   q = rint(y), z = y - q (exact, |z| <= 1/2), the angle is (pi/2)(q + z):
//   sin and cos of (pi/2) z by their Taylor polynomials in z^2 (through z^17
//   and z^16, Horner; truncation < 1e-17), then the quadrant q mod 4.
// ic_phasor0 is within 2.3e-16 of the exact phasor (measured against x87 long
// double); ic_phasor, the definition, takes it directly for k < 64 and for
// multiples of 64, and otherwise forms it as the product of its two parts,
// P(k) = P0(k mod 64) P0(k - k mod 64), one complex multiply of separately
// rounded operations ((a.x b.x - a.y b.y), (a.x b.y + a.y b.x)): a profile's
// n/2 + 1 phasors then need 64 + n/128 polynomial evaluations instead of one
// each (k_rotate's per-profile delays), within 7e-16 of the exact phasor.
__host__ __device__ inline double2 ic_phasor0(int k, double d, int n)
{
    const double c = d * 8193.0;
    const double dh = c - (c - d);
    const double dl = d - dh;
    const double kk = (double)k, nn = (double)n;
    const double xh = kk * dh, xl = kk * dl;
    const double t = xh - nn * rint(xh * (1.0 / nn));
    const double y = (t + xl) * (4.0 / nn);
    const double q = rint(y);
    const double z = y - q;
    const double w = z * z;
    // (-1)^j (pi/2)^(2j+1) / (2j+1)!  and  (-1)^j (pi/2)^(2j) / (2j)!
    double sp = 0x1.aaec32af93359p-38;
    sp = -0x1.6fadb9f155744p-31 + w * sp;
    sp = 0x1.e8f434d018d63p-25 + w * sp;
    sp = -0x1.e3074fde8871fp-19 + w * sp;
    sp = 0x1.50783487ee782p-13 + w * sp;
    sp = -0x1.32d2cce62bd86p-8 + w * sp;
    sp = 0x1.466bc6775aae2p-4 + w * sp;
    sp = -0x1.4abbce625be53p-1 + w * sp;
    sp = 0x1.921fb54442d18p+0 + w * sp;
    const double sn = z * sp;
    double cp = 0x1.20c62c2f2d7f5p-34;
    cp = -0x1.b6e24f44b128fp-28 + w * cp;
    cp = 0x1.f9d38a3763cc3p-22 + w * cp;
    cp = -0x1.a6d1f2a204a8cp-16 + w * cp;
    cp = 0x1.e1f506891babbp-11 + w * cp;
    cp = -0x1.55d3c7e3cbffap-6 + w * cp;
    cp = 0x1.03c1f081b5ac4p-2 + w * cp;
    cp = -0x1.3bd3cc9be45dep+0 + w * cp;
    cp = 1.0 + w * cp;
    switch ((int)q & 3) {
    case 0: return make_double2(cp, sn);
    case 1: return make_double2(-sn, cp);
    case 2: return make_double2(-cp, -sn);
    default: return make_double2(sn, -cp);
    }
}
__host__ __device__ inline double2 ic_phasor_mul(double2 a, double2 b)
{
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__host__ __device__ inline double2 ic_phasor(int k, double d, int n)
{
    const int lo = k & 63, hi = k - lo;
    if (lo == 0 || hi == 0) return ic_phasor0(k, d, n);
    return ic_phasor_mul(ic_phasor0(lo, d, n), ic_phasor0(hi, d, n));
}

// Fractional dedispersion (dedisp_mode IC_DEDISP_FFT; phase_rotation.py):
// out[p] = rot(f32(in[p] - base[p])) by the channel's phasors, sign +1 =
// dedisperse, -1 = dededisperse.  Rows p = s*nchan + c of ld_in / ldo floats;
// out2 (optional) receives a second copy (row strides multiples of 4:
// 16-byte row accesses); in and out2 may be fit cubes in the tiled layout
// (in_tiled / out2_tiled: d_ofs, strides multiples of 32); flags: only subints
// with flags[s] != 0; late: only profiles with (late[p] != 0) == late_sel (the
// diagnostics fork's two passes).  in may equal out (each row is read whole
// before it is written).  nbin a power of two, 64 .. 4096.
struct RotateArgs {
    const float *in;
    long ld_in;
    const float *base;          // [P] or nullptr (0)
    const float *ph;            // [nchan][nbin/2 + 1][2]: f32(ic_phasor(k, delay[c], nbin))
    const double *delay2;       // [P] per-profile delays (ic_set_delays2): phasors
                                // ic_phasor(k, delay2[p], nbin) evaluated in the kernel, ph unused
    int identity;               // the rotation is the identity (an archive stored
                                // dedispersed, sign +1): out = f32(in - base), no FFT
    int sign;
    const double2 *tw;          // [nbin]: exp(-2 pi i q / nbin)
    const int32_t *flags;       // [nsub] or nullptr (all)
    int nsub, nchan, nbin;
    float *out;
    long ldo;
    float *out2;
    long ldo2;
    // residual input (amp != nullptr): row p is f32(amp[p] * T64[i] - in[i])
    // (x pr_factor on [pr_start, pr_end)), or 0 when info[p] is outside 1-4
    // (k_residual's arithmetic); base is then unused
    const double *T64, *amp;
    const int32_t *info;
    int pr_on;
    double pr_factor;
    int pr_start, pr_end;
    int in_tiled, out2_tiled;
    const uint8_t *late;
    int late_sel;
    // list (optional): rotate only the profiles of this round list (RoundList:
    // A requests from the front, B from the end, counts packed in *nctr)
    const int32_t *list;
    const unsigned long long *nctr;
    // statistics of the rotated rows (std_o != nullptr; residual input, sign
    // -1, rotate_stats_supported): instead of writing row p to out, the kernel
    // measures X = f32(row * w0[p]) as k_diag's DIAG_STATS pass would (ic.py:
    // 111-117, :206-212) and writes std / mean / ptp / fftmax of p; out unused
    const float *w0;
    const double2 *tw_p2;       // k_diag_p2's twiddle table (p2_twiddles)
    double *std_o, *mean_o, *ptp_o, *fft_o;
};
hipError_t launch_rotate(hipStream_t st, const RotateArgs &a);
bool rotate_supported(int nbin);
// the residual rotation can carry the statistics (RotateArgs.std_o): f32 rows
// whose rotation keeps a profile in one wave's registers (nbin 1024)
bool rotate_stats_supported(int nbin, bool data_f64);
// D == nullptr: fit-cube rows formed from raw and base (fit_mode 1)
hipError_t launch_residual(hipStream_t st, const float *D, const float *raw, const float *base, const double *T64,
                           const double *amp, const int32_t *info, const int32_t *shift, int nsub, int nchan,
                           int nbin, int ldD, int dtiled, int pr_on, double pr_factor, int pr_start, int pr_end,
                           float *R);

}  // namespace icgpu
