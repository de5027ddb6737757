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
//   k_sb_tree        (channel shards) local super-block partials -> shard root
//   k_tscrunch       weighted mean over subints, *10000 -> T (ic.py:94)
//   k_fit            exact scipy leastsq(a*T-p, [1.0]) per profile (ic.py:278)
//   k_diag           residual (ic.py:279-288), f32 store (:272), dededisperse
//                    (:104), apply_weights (:296), diagnostics (:206-217)
//   k_linestats      per channel / subint median & MAD (ic.py:229-256)
//   k_combine        scale, max, median-of-4, threshold, new weights,
//                    convergence counters (ic.py:221-225, :303-305, :127-141)
#include <algorithm>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "ic_internal.h"

namespace icgpu {

__device__ constexpr double kRdwarf = 3.834e-20;
__device__ constexpr double kRgiant = 1.304e19;

// LDS ordering between lanes of ONE wave: DS instructions of a wave execute in
// order, so only compiler reordering must be prevented (no s_barrier).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- cross-lane trees on DPP + readlane (VALU latency, no LDS crossbar) ----
// Level m of an xor-butterfly pairs lane groups [0,m) and [m,2m).  Within a
// row of 16 that is quad_perm (m = 1, 2), row_half_mirror (m = 4) and
// row_mirror (m = 8): after level m every lane of a group of m holds the same
// value, so a mirror delivers the partner group's value.  The last two levels
// combine lanes 0, 16, 32, 48 read into scalars, in tree order.  The result is
// wave-uniform.  (IEEE add/max/min are commutative: a lane adding its partner's
// value gets the same bits as the partner adding its own.)
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ int dpp(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true);
}
// (every lane reads an in-range lane for these controls, so the f64 form needs
// no `old` operand: mov_dpp saves the two zeroing moves per level)
template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ float lane_read(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ int lane_read(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double lane_read(double v, int l)
{
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

// tree over lanes [0, ACT) (ACT a power of two <= 64), uniform result
template <int ACT, typename T, typename Op>
__device__ __forceinline__ T wave_tree(T v, Op op)
{
    if (ACT >= 2) v = op(v, dpp<kDppXor1>(v));
    if (ACT >= 4) v = op(v, dpp<kDppXor2>(v));
    if (ACT >= 8) v = op(v, dpp<kDppHalfMirror>(v));
    if (ACT >= 16) v = op(v, dpp<kDppMirror>(v));
    if (ACT == 64) return op(op(lane_read(v, 0), lane_read(v, 16)), op(lane_read(v, 32), lane_read(v, 48)));
    if (ACT == 32) return op(lane_read(v, 0), lane_read(v, 16));
    return lane_read(v, 0);
}

struct OpAdd {
    template <typename T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
struct OpMaxF {
    __device__ __forceinline__ float operator()(float a, float b) const { return fmaxf(a, b); }
    __device__ __forceinline__ double operator()(double a, double b) const { return fmax(a, b); }
};
struct OpMinF {
    __device__ __forceinline__ float operator()(float a, float b) const { return fminf(a, b); }
    __device__ __forceinline__ double operator()(double a, double b) const { return fmin(a, b); }
};
struct OpOr {
    __device__ __forceinline__ int operator()(int a, int b) const { return a | b; }
};


// ============================================================ template stage

// part[s][sb][i] = sum_{c in sb, ascending} W[s,c] * x[s,c,i]   (f64, from 0.0)
// x = ded (base == nullptr) or f32(ded - base[s,c]);  wpart[s][sb] = sum W.
// One lane per bin; lanes of a wave read 64 consecutive (rotated) bins.
// Canonical-order channel partial sums over one super-block, lane per bin:
//   MODE 0: part  = sum_c W*ded                     (baseline window total)
//   MODE 1: part2 = sum_c W*f32(ded - base), wpart  (fscrunch)
//   MODE 2: both, in one read of the cube (base = the previous iteration's)
//   MODE 3: MODE 1 that also writes the fit cube D[k][i] = f32(ded - base)
//           (iteration 1: base = base0, W = w0: the fit cube of ic.py:96-100 comes
//           out of the same read of the cube)
// flags != nullptr: only subints with flags[s] != 0 (a moved window) run.
// the fit cube is written once and read by the next kernels' sweeps, not by
// this one: non-temporal stores keep the write stream out of the way (C2
// -0.14 ms per clean; non-temporal raw loads here cost +0.5 ms)
__device__ __forceinline__ void st_fitcube(float *p, float v)
{
    __builtin_nontemporal_store(v, p);
}

// Exactness of a super-block column (the incremental template stage,
// k_chan_delta), for archives whose weights are 0 or 1: the column's terms
// are its values v_c (f64 from f32) over EVERY channel c of the super-block,
// whatever its current weight.  With biased f32 exponents emin / emax of the
// nonzero ones (subnormals as 1), every v_c is an integer multiple of
// 2^(emin - 150) and 256 |v_c| < 2^(emax - 118); if emax - emin <= 21 every
// partial sum of any subset of them, in any order and with any signs, is an
// f64 integer multiple of 2^(emin - 150) below 2^(53 + emin - 150): exact.
// The canonical sequential sum then equals the exact sum, and so does an old
// sum plus the terms that entered minus those that left.  ExTrack keeps the
// largest and smallest nonzero magnitude as bit patterns (4 VALU ops per
// value; an Inf / NaN value is a larger pattern than any finite one and fails
// the test).  Fractional weights: k_chan_delta ignores the flags.
struct ExTrack {
    unsigned mx = 0u, mn = 0xffffffffu;   // max |v| bits, min (|v| bits - 1): zero -> 0xffffffff
    __device__ __forceinline__ void add(float v)
    {
        const unsigned a = __float_as_uint(v) & 0x7fffffffu;
        mx = max(mx, a);
        mn = min(mn, a - 1u);
    }
    __device__ __forceinline__ uint8_t exact() const
    {
        if (mx >= 0x7f800000u) return 0;   // Inf / NaN
        if (mn == 0xffffffffu) return 1;   // all zero
        const int emax = max((int)(mx >> 23), 1), emin = max((int)((mn + 1u) >> 23), 1);
        return emax - emin <= 21 ? 1 : 0;
    }
};

template <int MODE>
__global__ __launch_bounds__(256) void k_chan_partials(
    const float *__restrict__ raw, const float *__restrict__ W, const int32_t *__restrict__ shift,
    const float *__restrict__ base, const int32_t *__restrict__ flags, int nsub, int nchan, int nbin, int nsb,
    double *__restrict__ part, double *__restrict__ part2, double *__restrict__ wpart, float *__restrict__ D,
    int ldD, int dtiled, uint8_t *__restrict__ exA, uint8_t *__restrict__ exF)
{
    constexpr bool A = MODE == 0 || MODE == 2, F = MODE != 0, WD = MODE == 3;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int sb = blockIdx.y;
    const int s = blockIdx.z;
    if (flags && flags[s] == 0) return;
    const int c0 = sb * kSuperBlock;
    const int c1 = min(c0 + kSuperBlock, nchan);
    // column exactness (ExTrack) of this pass's sums (A: exA, F: exF)
    const bool tA = A && exA, tF = F && exF;
    ExTrack xa, xf;
    if (i < nbin) {
        double acc = 0.0, acc2 = 0.0;
        const size_t krow = (size_t)s * nchan;
        // batches of 16 channels: all 16 row loads are issued before the
        // (sequential, canonical-order) accumulation consumes them
        constexpr int B = 16;
        int c = c0;
        for (; c + B <= c1; c += B) {
            float xv[B], wv[B], bv[B];
#pragma unroll
            for (int q = 0; q < B; ++q) {
                int j = i + shift[c + q];
                if (j >= nbin) j -= nbin;
                xv[q] = raw[(krow + c + q) * nbin + j];
                wv[q] = W[krow + c + q];
                bv[q] = F ? base[krow + c + q] : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < B; ++q) {
                const double w = (double)wv[q];
                const float d = xv[q] - bv[q];
                if (A) acc = acc + w * (double)xv[q];
                if (F) acc2 = acc2 + w * (double)d;
                if (WD) st_fitcube(D + d_ofs(krow + c + q, i, ldD, dtiled), d);
                if (tA) xa.add(xv[q]);
                if (tF) xf.add(d);
            }
        }
        for (; c < c1; ++c) {
            const size_t k = krow + c;
            int j = i + shift[c];
            if (j >= nbin) j -= nbin;
            const float x = raw[k * nbin + j];
            const double w = (double)W[k];
            const float d = F ? x - base[k] : 0.0f;
            if (A) acc = acc + w * (double)x;
            if (F) acc2 = acc2 + w * (double)d;
            if (WD) st_fitcube(D + d_ofs(k, i, ldD, dtiled), d);
            if (tA) xa.add(x);
            if (tF) xf.add(d);
        }
        const size_t col = ((size_t)s * nsb + sb) * nbin + i;
        if (A) part[col] = acc;
        if (F) part2[col] = acc2;
        if (tA) exA[col] = xa.exact();
        if (tF) exF[col] = xf.exact();
    }
    if (F && blockIdx.x == 0 && threadIdx.x == 0) {
        double a = 0.0;
        for (int c = c0; c < c1; ++c) a = a + (double)W[(size_t)s * nchan + c];
        wpart[(size_t)s * nsb + sb] = a;
    }
}

// Incremental template stage (iteration >= 2, integer dedispersion): the
// window totals `part` and the fscrunch partials `part2` of every super-block
// column move from the previous weights Wo to the current Wn by the terms of
// the channels whose weight changed: old + (sum of Wn v - Wo v over them),
// exact for columns whose flag (ExTrack, set by the last full pass) holds;
// the other columns, and every column of a super-block with a weight other
// than 0 or 1, are summed again in canonical order over all channels.  part2
// uses the carried levels: subints whose window moves are summed again
// afterwards (k_chan_partials mode 1, flagged).  wpart is summed again (256
// weights).  One block per (bin range, super-block, subint); a block whose
// super-block has no changed channel does nothing.
// BPT bins per thread (bin i0 + 256 b, b < BPT): the change list and the
// block's fixed costs serve BPT times the columns, and BPT times the loads are
// in flight per batch of channels.
// SPLIT (FFT dedispersion): part's terms come from raw (the rotated raw cube)
// and part2's from rawF (the rotated baselined rows Tc, base = 0); otherwise
// both from raw, part2's as f32(raw - base).
template <int BPT, bool SPLIT>
__global__ __launch_bounds__(256) void k_chan_delta(const float *__restrict__ raw, const float *__restrict__ rawF,
                                                    const int32_t *__restrict__ shift,
                                                    const float *__restrict__ base, const float *__restrict__ Wn,
                                                    const float *__restrict__ Wo, int nchan, int nbin, int nsb,
                                                    double *__restrict__ part, double *__restrict__ part2,
                                                    double *__restrict__ wpart, const uint8_t *__restrict__ exA,
                                                    const uint8_t *__restrict__ exF)
{
    __shared__ int chg[kSuperBlock];
    __shared__ int fix[256 * BPT];           // columns summed again: bin | 1 << 16 (part) | 1 << 17 (part2)
    __shared__ double tA[kSuperBlock], tF[kSuperBlock];
    __shared__ int wcnt[4], wfrac[4], wfix[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i0 = blockIdx.x * 256 * BPT + threadIdx.x;
    const int sb = blockIdx.y, s = blockIdx.z;
    const int c0 = sb * kSuperBlock, c1 = min(c0 + kSuperBlock, nchan);
    const size_t krow = (size_t)s * nchan;
    const size_t col0 = ((size_t)s * nsb + sb) * nbin;
    // the changed channels of the super-block, in ascending order
    int n, frac, nones;
    {
        const int c = c0 + (int)threadIdx.x;
        const float wn = c < c1 ? Wn[krow + c] : 0.0f, wo = c < c1 ? Wo[krow + c] : 0.0f;
        const bool ch = __float_as_uint(wn) != __float_as_uint(wo);
        const bool fr = !(wn == 0.0f || wn == 1.0f) || !(wo == 0.0f || wo == 1.0f);
        const unsigned long long m = __ballot(ch);
        const unsigned long long m1 = __ballot(wn == 1.0f);
        const bool fw = __any(fr);
        if (lane == 0) {
            wcnt[wave] = __popcll(m);
            wfrac[wave] = fw ? 1 : 0;
            wfix[wave] = __popcll(m1);
        }
        __syncthreads();
        int off = 0;
        for (int w = 0; w < wave; ++w) off += wcnt[w];
        if (ch) chg[off + __popcll(m & ((1ull << lane) - 1ull))] = c;
        n = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        frac = wfrac[0] | wfrac[1] | wfrac[2] | wfrac[3];
        nones = wfix[0] + wfix[1] + wfix[2] + wfix[3];
        __syncthreads();
    }
    if (n == 0) return;
    constexpr int B = 16 / BPT;   // channels per batch: 16 loads in flight per thread
    if (frac) {
        // a weight other than 0 / 1: every column in canonical order (k_chan_partials' sums)
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int i = i0 + 256 * b;
            if (i >= nbin) continue;
            double acc = 0.0, acc2 = 0.0;
            int c = c0;
            for (; c + 16 <= c1; c += 16) {
                float xv[16], wv[16], bv[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    int j = i + shift[c + q];
                    if (j >= nbin) j -= nbin;
                    xv[q] = raw[(krow + c + q) * nbin + j];
                    wv[q] = Wn[krow + c + q];
                    bv[q] = SPLIT ? rawF[(krow + c + q) * nbin + j] - base[krow + c + q] : base[krow + c + q];
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const double w = (double)wv[q];
                    const float d = SPLIT ? bv[q] : xv[q] - bv[q];
                    acc = acc + w * (double)xv[q];
                    acc2 = acc2 + w * (double)d;
                }
            }
            for (; c < c1; ++c) {
                int j = i + shift[c];
                if (j >= nbin) j -= nbin;
                const float x = raw[(krow + c) * nbin + j];
                const double w = (double)Wn[krow + c];
                const float d = (SPLIT ? rawF[(krow + c) * nbin + j] : x) - base[krow + c];
                acc = acc + w * (double)x;
                acc2 = acc2 + w * (double)d;
            }
            part[col0 + i] = acc;
            part2[col0 + i] = acc2;
        }
    } else {
        bool okA[BPT], okF[BPT];
        double dA[BPT], dF[BPT];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int i = i0 + 256 * b;
            okA[b] = i < nbin && exA[col0 + i];
            okF[b] = i < nbin && exF[col0 + i];
            dA[b] = dF[b] = 0.0;
        }
        for (int q0 = 0; q0 < n; q0 += B) {
            float xv[B][BPT], fv[SPLIT ? B : 1][BPT], bv[B], wnv[B], wov[B];
#pragma unroll
            for (int q = 0; q < B; ++q) {
                const int c = chg[min(q0 + q, n - 1)];
                bv[q] = base[krow + c];
                wnv[q] = Wn[krow + c];
                wov[q] = Wo[krow + c];
                const float *row = raw + (krow + c) * nbin;
                const int sc = shift[c];
#pragma unroll
                for (int b = 0; b < BPT; ++b) {
                    const int i = min(i0 + 256 * b, nbin - 1);
                    int j = i + sc;
                    if (j >= nbin) j -= nbin;
                    xv[q][b] = row[j];
                    if (SPLIT) fv[SPLIT ? q : 0][b] = rawF[(krow + c) * nbin + j];
                }
            }
#pragma unroll
            for (int q = 0; q < B; ++q) {
                if (q0 + q < n) {
                    const double wn = (double)wnv[q], wo = (double)wov[q];
#pragma unroll
                    for (int b = 0; b < BPT; ++b) {
                        const float d = (SPLIT ? fv[SPLIT ? q : 0][b] : xv[q][b]) - bv[q];
                        dA[b] = dA[b] + (wn * (double)xv[q][b] - wo * (double)xv[q][b]);
                        dF[b] = dF[b] + (wn * (double)d - wo * (double)d);
                    }
                }
            }
        }
        int need[BPT];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const int i = i0 + 256 * b;
            need[b] = 0;
            if (i < nbin) {
                if (okA[b]) part[col0 + i] = part[col0 + i] + dA[b];
                if (okF[b]) part2[col0 + i] = part2[col0 + i] + dF[b];
                need[b] = (okA[b] ? 0 : 1 << 16) | (okF[b] ? 0 : 1 << 17);
            }
        }
        // inexact columns: the whole block sums each again, one channel per
        // thread, then one thread adds the 256 terms in canonical order
        int nfix = 0;
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
            const unsigned long long m = __ballot(need[b] != 0);
            if (lane == 0) wfix[wave] = __popcll(m);
            __syncthreads();
            int off = nfix;
            for (int w = 0; w < wave; ++w) off += wfix[w];
            if (need[b]) fix[off + __popcll(m & ((1ull << lane) - 1ull))] = need[b] | (i0 + 256 * b);
            nfix += wfix[0] + wfix[1] + wfix[2] + wfix[3];
            __syncthreads();
        }
        for (int f = 0; f < nfix; ++f) {
            const int e = fix[f], ib = e & 0xffff;
            const int c = c0 + (int)threadIdx.x;
            if (c < c1) {
                int j = ib + shift[c];
                if (j >= nbin) j -= nbin;
                const float x = raw[(krow + c) * nbin + j];
                const double w = (double)Wn[krow + c];
                const float d = (SPLIT ? rawF[(krow + c) * nbin + j] : x) - base[krow + c];
                tA[threadIdx.x] = w * (double)x;
                tF[threadIdx.x] = w * (double)d;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                double acc = 0.0, acc2 = 0.0;
                for (int q = 0; q < c1 - c0; ++q) {
                    acc = acc + tA[q];
                    acc2 = acc2 + tF[q];
                }
                if (e & (1 << 16)) part[col0 + ib] = acc;
                if (e & (1 << 17)) part2[col0 + ib] = acc2;
            }
            __syncthreads();
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // weights 0 / 1 only: the sequential sum is the count of ones, exactly
        double a = (double)nones;
        if (frac) {
            a = 0.0;
            for (int c = c0; c < c1; ++c) a = a + (double)Wn[krow + c];
        }
        wpart[(size_t)s * nsb + sb] = a;
    }
}

// Canonical super-block combine (archive.py sb_tree) as a post-order stack
// program (SbPlan): the stack lives in registers (static indices only), top
// at st[0].
template <typename Get>
__device__ __forceinline__ double sb_eval(const SbPlan &pl, Get get)
{
    double st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = 0.0;
    for (int j = 0; j < pl.n; ++j) {
#pragma unroll
        for (int k = 7; k > 0; --k) st[k] = st[k - 1];
        st[0] = get(j);
        for (int m = 0; m < (int)pl.merges[j]; ++m) {
            st[0] = st[1] + st[0];   // left subtree + right subtree
#pragma unroll
            for (int k = 1; k < 7; ++k) st[k] = st[k + 1];
        }
    }
    return st[0];
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

// One block per subint: tot[i] = sb_tree over the leaves of part; m[j] =
// sum_{k<width} tot[(j+k)%n]; win[s] = first argmin.
// flags != nullptr: flags[s] = (window moved), win[s] updated in place.
// kWindowThreads threads, so each window sum (a width-long in-order chain) has
// its own thread up to nbin = 1024.  The argmin order (NaN first, then value,
// then index) is total, so the result does not depend on the block size.
constexpr int kWindowThreads = 1024;
__global__ __launch_bounds__(kWindowThreads) void k_window(const double *__restrict__ part, long ss, long sl, SbPlan plan,
                                                int nbin, int width, int32_t *__restrict__ win,
                                                int32_t *__restrict__ flags)
{
    extern __shared__ double sh[];
    double *tot = sh;                       // nbin
    double *bv = sh + nbin;                 // blockDim
    int *bi = (int *)(bv + blockDim.x);     // blockDim
    const int s = blockIdx.x;
    for (int i = threadIdx.x; i < nbin; i += blockDim.x) {
        const double *src = part + (size_t)s * ss + i;
        tot[i] = sb_eval(plan, [&](int j) { return src[(size_t)j * sl]; });
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
    if (threadIdx.x == 0) {
        if (flags) {
            const int moved = win[s] != bi[0];
            flags[s] = moved;
            if (moved) atomicAdd(&flags[gridDim.x], 1);   // flags[nsub]: moves counter
        }
        win[s] = bi[0];
    }
}

// base[k] = f32( (sum_{t<width} f64(ded[(win+t)%n])) / width ), sequential in t.
// Per-profile baseline level: f32(sum_seq f64(x_j) / width) over the subint's
// window, in the dedispersed frame (Appendix C stand-in; oracle orc_baseline).
// Four profiles per wave, 16 lanes each: a lane issues its window loads in
// batches of 8 before adding them, so one memory latency serves four profiles
// (one profile per wave left the kernel bound by a full latency per profile).
// The sequential f64 sum of f32 values is computed in parallel when that is
// provably exact: every x_j is an integer multiple of 2^(emin-150) and
// |sum| < width * 2^(emax-126), so when ceil(log2 width) + emax - emin + 24 <=
// 53 every partial sum, in any order, is representable and the result equals
// the sequential one bit for bit.  Otherwise (rare: values spanning > 2^21, or
// Inf/NaN) the profile's 16 lanes walk the window in order.
// V4 (nbin % 4 == 0, 16-B aligned rows): the lanes read the aligned float4s
// that cover the window (which wraps on a float4 boundary) and keep the
// elements inside it; the exact path does not depend on the order of the adds.
template <bool V4>
__global__ __launch_bounds__(256) void k_base(const float *__restrict__ raw, const int32_t *__restrict__ shift,
                                              const int32_t *__restrict__ win, const int32_t *__restrict__ flags,
                                              int nsub, int nchan, int nbin, int width, float *__restrict__ base)
{
    constexpr int GL = 16, BATCH = 8;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = lane / GL, gl = lane % GL;
    const long P = (long)nsub * nchan;
    const int lgw = 32 - __clz(max(width - 1, 1));   // ceil(log2(width)), >= 1
    for (long k0 = ((long)blockIdx.x * 4 + wave) * 4; k0 < P; k0 += (long)gridDim.x * 16) {
        const long k = k0 + grp;
        // window unchanged: base unchanged
        const bool act = k < P && !(flags && flags[k / nchan] == 0);
        double acc = 0.0;
        int emax = 0, emin = 255, q0 = 0;
        const float *row = raw + (size_t)(act ? k : 0) * nbin;
        if (act) {
            q0 = win[k / nchan] + shift[k % nchan];
            if (q0 >= nbin) q0 -= nbin;
            if constexpr (V4) {
                const float4 *row4 = (const float4 *)row;
                const int nq = nbin >> 2, a = q0 >> 2, off = q0 & 3;
                const int nf = (off + width + 3) >> 2;   // float4s covering the window
                constexpr int B4 = 4;
                for (int m0 = gl; m0 < nf; m0 += GL * B4) {
                    float4 xv[B4];
#pragma unroll
                    for (int u = 0; u < B4; ++u) {
                        const int m = m0 + GL * u;
                        int qi = a + m;
                        if (qi >= nq) qi -= nq;
                        xv[u] = m < nf ? row4[qi] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    }
#pragma unroll
                    for (int u = 0; u < B4; ++u) {
                        const int e0 = 4 * (m0 + GL * u) - off;   // window offset of the first element
                        const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const float x = (e0 + c >= 0 && e0 + c < width) ? xs[c] : 0.0f;
                            acc = acc + (double)x;
                            const int be = max((int)((__float_as_uint(x) >> 23) & 0xffu), 1);
                            if (x != 0.0f) {
                                emax = max(emax, be);
                                emin = min(emin, be);
                            }
                        }
                    }
                }
            } else
            for (int j0 = gl; j0 < width; j0 += GL * BATCH) {
                float xv[BATCH];
#pragma unroll
                for (int u = 0; u < BATCH; ++u) {
                    const int j = j0 + GL * u;
                    int q = q0 + j;
                    if (q >= nbin) q -= nbin;
                    xv[u] = j < width ? row[q] : 0.0f;
                }
#pragma unroll
                for (int u = 0; u < BATCH; ++u) {
                    const float x = xv[u];
                    acc = acc + (double)x;
                    const int be = max((int)((__float_as_uint(x) >> 23) & 0xffu), 1);
                    if (x != 0.0f) {
                        emax = max(emax, be);
                        emin = min(emin, be);
                    }
                }
            }
        }
        for (int off = GL / 2; off > 0; off >>= 1) {   // within the 16-lane group
            acc = acc + __shfl_xor(acc, off);
            emax = max(emax, __shfl_xor(emax, off));
            emin = min(emin, __shfl_xor(emin, off));
        }
        if (act && emax != 0 && lgw + emax - emin + 24 > 53) {
            acc = 0.0;   // in order (every lane of the group walks the same values)
            for (int j = 0; j < width; ++j) {
                int q = q0 + j;
                if (q >= nbin) q -= nbin;
                acc = acc + (double)row[q];
            }
        }
        if (act && gl == 0) base[k] = (float)(acc / (double)width);
    }
}

// pscrunch on the device: raw = f32(pol0 + pol1), float4 grid-stride
__global__ __launch_bounds__(256) void k_pscrunch(float *__restrict__ raw, const float *__restrict__ pol1, size_t n)
{
    const size_t n4 = n / 4;
    float4 *r4 = (float4 *)raw;
    const float4 *p4 = (const float4 *)pol1;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 a = r4[i];
        const float4 b = p4[i];
        a.x = a.x + b.x;
        a.y = a.y + b.y;
        a.z = a.z + b.z;
        a.w = a.w + b.w;
        r4[i] = a;
    }
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        raw[i] = raw[i] + pol1[i];
}

// F[s][i] = f32(num/wsum) (0 if wsum == 0); wf[s] = f32(wsum); num and wsum
// are the canonical trees over the leaves
__global__ __launch_bounds__(256) void k_fscrunch(const double *__restrict__ part, long ss, long sl,
                                                  const double *__restrict__ wpart, long wss, long wsl, SbPlan plan,
                                                  int nbin, float *__restrict__ F, float *__restrict__ wf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (i >= nbin) return;
    const double *src = part + (size_t)s * ss + i;
    const double *wsrc = wpart + (size_t)s * wss;
    const double num = sb_eval(plan, [&](int j) { return src[(size_t)j * sl]; });
    const double wsum = sb_eval(plan, [&](int j) { return wsrc[(size_t)j * wsl]; });
    F[(size_t)s * nbin + i] = (wsum != 0.0) ? (float)(num / wsum) : 0.0f;
    if (i == 0) wf[s] = (float)wsum;
}

// Shard root of local super-block partials [s][nsb_loc][nbin] (channel shards):
// out[s*ostr + i] = sb_tree(part[s][*][i]); out[s*ostr + nbin] = sb_tree(wpart[s][*])
// (wpart optional; ostr >= nbin + 1 then): one row per subint, so the rows a
// rank owns are one contiguous all-to-all block.
__global__ __launch_bounds__(256) void k_sb_tree(const double *__restrict__ part, const double *__restrict__ wpart,
                                                 SbPlan plan, int nbin, long ostr, double *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    const int n = plan.n;
    if (i < nbin) {
        const double *src = part + (size_t)s * n * nbin + i;
        out[(size_t)s * ostr + i] = sb_eval(plan, [&](int j) { return src[(size_t)j * nbin]; });
    }
    if (wpart && i == 0) {
        const double *w = wpart + (size_t)s * n;
        out[(size_t)s * ostr + nbin] = sb_eval(plan, [&](int j) { return w[j]; });
    }
}

// T[i] = f32( f32(sum_s wf*F / sum_s wf) * 10000 )
__global__ __launch_bounds__(256) void k_tscrunch(const float *__restrict__ F, const float *__restrict__ wf,
                                                  int nsub, int nbin, float *__restrict__ T,
                                                  double *__restrict__ T64, double *__restrict__ T2)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nbin) return;
    double wt = 0.0, num = 0.0;
    // batches of 16 subints: the 16 loads are in flight together, then the
    // sums run in subint order (the chain is latency-bound with 16 blocks)
    constexpr int B = 16;
    int s = 0;
    for (; s + B <= nsub; s += B) {
        float fv[B], wv[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            wv[q] = wf[s + q];
            fv[q] = F[(size_t)(s + q) * nbin + i];
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const double w = (double)wv[q];
            wt = wt + w;
            const double t = w * (double)fv[q];
            num = num + t;
        }
    }
    for (; s < nsub; ++s) {
        const double w = (double)wf[s];
        wt = wt + w;
        const double t = w * (double)F[(size_t)s * nbin + i];
        num = num + t;
    }
    const float t = (wt != 0.0) ? (float)(num / wt) : 0.0f;
    const float tt = t * 10000.0f;
    T[i] = tt;
    T64[i] = (double)tt;
    if (T2) {
        T2[i] = (double)tt;
        T2[i + nbin] = (double)tt;
    }
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
        // scipy's MINPACK keeps gnorm = 0 when the term is NaN (a non-finite
        // profile): info 4 at once, x = 1 (probed against scipy 1.15.3;
        // tests/golden/leastsq_nonfinite.npz)
        const double g = fabs(sum / L.acnorm);
        if (g > L.gnorm) L.gnorm = g;
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

__device__ int lm_after_a2(LmState &L, double fnorm1, bool *accepted = nullptr)
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
    if (accepted) *accepted = ratio >= 1e-4;
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

// Exact fast path.  enorm: while every component is 0 or inside
// (RDWARF, agiant) MINPACK's enorm reduces to sqrt(sum_seq a*a).  The range is
// verified per lane without per-sample work after the first 32 samples:
//  * upper: the sequential sum of the nonnegative squares bounds every square
//    (RN is monotone), so hi(RN(s2)) < hi(RN(agiant^2)) at the end implies
//    |a| < agiant for every component (NaN/Inf fail the compare);
//  * lower: over the first 32 samples (the peeled first tile pair) every
//    nonzero square is checked, hi(RN(a^2)) > hi(RN(RDWARF^2)) implies
//    |a| > RDWARF (equal high words count as out of range); after them the
//    running sum must be >= 2^-40.  A later component with |a| <= RDWARF then
//    adds RN(a^2) <= 2^-129 < ulp(s2)/2 to s2, a no-op, exactly as MINPACK
//    leaves it out of s2; MINPACK's final factor 1 + (x3max/s2)(x3max s3) <=
//    1 + n RDWARF^2 / 2^-40 rounds to 1 for any n < 2^50, and s2 >= x3max, so
//    its result is sqrt(s2) as well.
// A nonzero a whose square underflowed to 0 would slip through the first-tile
// check, so the A sweep takes this path only for |x| in [2^-100, 2^100]:
// there every nonzero f = RN(RN(x t) - p) (t, p from f32) is >= 2^-301 and
// every nonzero J >= 2^-427 in magnitude, |J| <= 2^355, and all squares are
// normal.  Division q = RN(a/b): y = RN(1/b) and ylo = RN((1 - b y) y) (1 - b y
// is exact) approximate 1/b to 2^-105 relative, so q0 = RN(a y + RN(a ylo)) is
// within 2^-104 |a/b| + ulp/2, i.e. faithful, and one Markstein correction
// q = RN(q0 + RN(a - b q0) y) (the remainder exact) is RN(a/b), barring
// over/underflow — which would push J out of the verified enorm range and send
// the lane to the exact pass.
struct FastAcc {
    double s2;
    uint32_t minhm1;
};

__device__ __forceinline__ void fa_zero(FastAcc &a)
{
    a.s2 = 0.0;
    a.minhm1 = 0xffffffffu;
}

template <bool CHK>
__device__ __forceinline__ void fa_add(FastAcc &a, double v)
{
    const double sq = v * v;   // == RN(|v| * |v|)
    a.s2 = a.s2 + sq;
    if (CHK) {
        const uint32_t hi = (uint32_t)((unsigned long long)__double_as_longlong(sq) >> 32);
        a.minhm1 = min(a.minhm1, hi - 1u);   // zero -> 0xffffffff
    }
}

// after the checked samples: no nonzero square at or below RDWARF^2, and the
// running sum large enough to absorb any later one
__device__ __forceinline__ bool fa_lo_ok(const FastAcc &a, uint32_t hr1)
{
    return ((a.minhm1 == 0xffffffffu) || (a.minhm1 + 1u >= hr1)) && a.s2 >= 0x1p-40;
}

__device__ __forceinline__ bool fa_hi_ok(const FastAcc &a, uint32_t hg)
{
    return (uint32_t)((unsigned long long)__double_as_longlong(a.s2) >> 32) < hg;
}

__device__ __forceinline__ double fa_fin(const FastAcc &a) { return a.s2 != 0.0 ? sqrt(a.s2) : 0.0; }

// low part of 1/b given y = RN(1/b)
__device__ __forceinline__ double recip_lo(double b, double y) { return fma(-b, y, 1.0) * y; }

__device__ __forceinline__ double mdiv(double a, double b, double y, double ylo)
{
    const double q0 = fma(a, y, a * ylo);
    const double r0 = fma(-b, q0, a);
    return fma(r0, y, q0);
}

__device__ __forceinline__ bool x_in_fast_range(double x)
{
    const double ax = fabs(x);
    return ax >= 0x1p-500 && ax <= 0x1p500;
}

// the A sweep's squared-high-word range check (see fa_add) needs the tighter range
__device__ __forceinline__ bool x_in_sq_range(double x)
{
    const double ax = fabs(x);
    return ax >= 0x1p-100 && ax <= 0x1p100;
}

// ---- data movement of a sweep: LDS-DMA, double buffered ----------------------
// A wave owns 64 profiles (one per lane) and streams their rows of D through
// two 4-KiB LDS buffers, 16 bins per tile, with global_load_lds_dwordx4: the
// next tile is in flight while the current one is consumed, and no VGPRs hold
// it on the way.  A DMA writes 1 KiB lane-linearly (slot = lane), so the
// transpose to "lane p reads its own profile" is done on the SOURCE side:
// instruction m, lane l fetches chunk c = (l&3) ^ ((l>>4)&3) (4 bins) of
// profile 16m + l/4.  Profile p's chunk c then sits in slot
// 64(p>>4) + 4(p&15) + (c ^ ((p>>2)&3)), and the ds_read_b128 of one chunk by
// all 64 lanes hits 16 distinct 16-B slots in each 16-lane bank group.
// D is padded to [roundup(P,64)][ldD], ldD a multiple of 32: no guards.
#define FIT_TB 16
#define FIT_BUF 4096

typedef float fv4 __attribute__((ext_vector_type(4)));

struct DmaTiles {
    const float *src[4];   // this lane's DMA source for instruction m at bin 0
    int tiled;             // fit cube layout (dt_ofs): bin b0 of a row is at + (b0/32) 2048 + b0 % 32
    uint32_t rd[4];        // LDS byte address of this lane's chunk c in buffer 0
    char *lds;             // buffer 0 (buffer 1 at +FIT_BUF)
};

__device__ __forceinline__ uint32_t lds_u32(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

__device__ __forceinline__ void dma_tile(const DmaTiles &d, char *buf, int b0)
{
    const int off = d.tiled ? ((b0 >> 5) << 11) + (b0 & 31) : b0;
#pragma unroll
    for (int m = 0; m < 4; ++m)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(d.src[m] + off),
                                         (__attribute__((address_space(3))) void *)(buf + m * 1024), 16, 0,
                                         0);   // default cache policy (nt: 15.7 -> 18.8 ms per C2 clean)
}

// ds_read in asm: the compiler would otherwise order every LDS read behind a
// vmcnt(0) for the DMAs, draining the prefetch.  Ordering against the DMA is
// the explicit counted vmcnt in sweep_dma; the lgkmcnt wait ties the values.
template <int OFF>
__device__ __forceinline__ void read_tile(const DmaTiles &d, fv4 (&v)[4])
{
#pragma unroll
    for (int c = 0; c < 4; ++c) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[c]) : "v"(d.rd[c]), "i"(OFF));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}

// one pair of tiles (t, t + 1) = one 128-B line of each of the wave's 64 rows;
// CHK: the body runs its per-sample range checks.  Both halves of the next line
// are requested together, right after tile t + 1 has been read into registers
// (a half line requested alone is refetched when the L2 drops the line in
// between: measured 1.2 % faster than refilling each buffer as soon as it is
// read).  The ds_reads complete before the DMA that overwrites their buffer is
// issued (read_tile waits on lgkmcnt, and the memory clobber keeps the compiler
// from hoisting the DMA above them).
template <bool CHK, typename Body>
__device__ __forceinline__ void sweep_pair(const DmaTiles &d, int t, int nt, Body &body)
{
    fv4 v[4];
    body.load_T(t * FIT_TB);   // scalar loads issued ahead of the waits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tiles t and t + 1 landed
    read_tile<0>(d, v);
    body.template run<CHK>(t * FIT_TB, v);
    body.fence();   // keep tile t's arithmetic ahead of the DMA issue below
    body.load_T((t + 1) * FIT_TB);
    read_tile<FIT_BUF>(d, v);
    asm volatile("" ::: "memory");
    if (t + 2 < nt) {
        dma_tile(d, d.lds, (t + 2) * FIT_TB);
        dma_tile(d, d.lds + FIT_BUF, (t + 3) * FIT_TB);
    }
    body.template run<CHK>((t + 1) * FIT_TB, v);
    body.fence();
}

// Body::kPeel: the first pair (32 samples) is peeled with the checks on, then
// body.checked().  issued: the first tile pair's DMA is already in flight
// (k_fit_pass issues it before it loads the lanes' lmdif state)
template <typename Body>
__device__ __forceinline__ void sweep_dma(const DmaTiles &d, int ldD, Body &body, bool issued = false)
{
    const int nt = ldD / FIT_TB;   // even, >= 2
    if (!issued) {
        dma_tile(d, d.lds, 0);
        dma_tile(d, d.lds + FIT_BUF, FIT_TB);
    }
    int t = 0;
    if constexpr (Body::kPeel) {
        sweep_pair<true>(d, 0, nt, body);
        body.checked();
        t = 2;
    }
    for (; t < nt; t += 2) sweep_pair<false>(d, t, nt, body);
}

struct PassIn {
    bool A, B;                   // lane takes part in pass A / B
    double xa, xha, ha, yha, yla;  // A: f(xa) and J(xa)
    double xb, xhb, hb, yhb, ylb, ajb, yaj, ylj;  // B: sum Jn*f at xb
};

struct PassOut {
    double fnorm, acnorm, sum;
    float p0;                    // the profile's first sample (round 0: k_fit_state's f0 / J0)
    bool bad;                    // fast path left its verified range
    bool jt;                     // FUSE: J(1) == T, sum is qtf's dot
};

// Fast sweep body: straight-line over a 16-bin tile, wave-uniform predicates
// only (lanes that did not request the sweep compute on defaults; their
// results are discarded).  Zero-padded samples (p = 0, T = 0) are exact
// no-ops: f = J = 0 adds nothing to either norm, and Jn*f = 0 to the dot.
// FUSE (round 0: DA at x = 1 for every lane, k_fit_init): the A sweep at
// x = 1 specialised (1 t = t; h = 2^-26, so J = RN(d / h) = d 2^26 exactly,
// which is what mdiv gives), plus the dot of the B sweep that would follow,
// sum_i RN(Jn_i f_i) with Jn_i = RN(J_i / aj) (+1 at i = 0) and the shared aj
// of k_fit_prep, and jt = (J_i == T_i for every i): when that holds, and the
// profile's own qrfac is k_fit_prep's, the dot is the B sweep's own.
template <bool DA, bool DB, bool FUSE = false>
struct FastBody {
    static constexpr bool kPeel = true;
    const PassIn &in;
    const double *__restrict__ T64;
    FastAcc fF, fJ;
    double sum, fsum;
    float p00;   // FUSE: the first sample
    int lo_ok;
    bool jt;

    __device__ __forceinline__ FastBody(const PassIn &i, const double *T) : in(i), T64(T)
    {
        fa_zero(fF);
        fa_zero(fJ);
        sum = fsum = 0.0;
        p00 = 0.0f;
        lo_ok = 1;
        jt = true;
    }

    // the flag is materialised here (empty asm): otherwise the compiler sinks
    // the per-sample minima below the sweep loop and keeps the squares live
    __device__ __forceinline__ void checked()
    {
        if (DA) {
            const uint32_t hr1 = (uint32_t)((unsigned long long)__double_as_longlong(kRdwarf * kRdwarf) >> 32) + 1u;
            lo_ok = (fa_lo_ok(fF, hr1) && fa_lo_ok(fJ, hr1)) ? 1 : 0;
            asm volatile("" : "+v"(lo_ok));
        }
    }

    // empty asm on the accumulators: the compiler may not sink a tile's
    // arithmetic below the following s_waitcnt (asm statements keep their order)
    __device__ __forceinline__ void fence()
    {
        asm volatile("" : "+v"(fF.s2), "+v"(fJ.s2), "+v"(sum), "+v"(fF.minhm1), "+v"(fJ.minhm1));
        if (FUSE) asm volatile("" : "+v"(fsum));
    }

    double tv[FIT_TB];   // the tile's template values (wave-uniform: SGPRs)
    __device__ __forceinline__ void load_T(int b0)
    {
#pragma unroll
        for (int i = 0; i < FIT_TB; ++i) tv[i] = T64[b0 + i];
    }

    // Four samples at a time, stage by stage: the four dependent chains (the
    // products, the differences, the four-step divisions) are interleaved so
    // that every f64 op has independent neighbours to hide its latency behind;
    // the accumulations still run in sample order.  Per sample: A = f(x),
    // f(x + h), J = RN((f(x + h) - f(x))/h), f^2 and J^2 summed; B = the same f
    // and J, Jn = RN(J/ajnorm) (+1 on sample 0), sum += Jn f.
    template <bool CHK>
    __device__ __forceinline__ void group4(const double (&t)[4], const fv4 &pv4, bool first)
    {
        const float pf[4] = {pv4.x, pv4.y, pv4.z, pv4.w};
        double p[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = (double)pf[k];
        if (DA && FUSE) {
            // x = 1: f = RN(t - p), d = RN(RN((1 + 2^-26) t) - p) - f, J = d 2^26
            constexpr double xh1 = 1.0 + 0x1p-26;
            double f[4], d[4], q[4], r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = xh1 * t[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = t[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - f[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = d[k] * 0x1p26;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fa_add<CHK>(fF, f[k]);
                fa_add<CHK>(fJ, q[k]);
            }
            if (first) p00 = pf[0];
            // Jn = mdiv(J, aj, yaj, ylj) (the B sweep's), dot in sample order
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = q[k] * in.ylj;
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = fma(q[k], in.yaj, d[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = fma(-in.ajb, d[k], q[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = fma(r[k], in.yaj, d[k]);
            if (first) d[0] = d[0] + 1.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                jt = jt && (q[k] == t[k]);
                d[k] = d[k] * f[k];
                fsum = fsum + d[k];
            }
        } else if (DA) {
            double f[4], d[4], q[4], r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = in.xa * t[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = in.xha * t[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = f[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - f[k];
            // J = mdiv(d, ha, yha, yla), stage-interleaved
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = d[k] * in.yla;
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = fma(d[k], in.yha, q[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = fma(-in.ha, q[k], d[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = fma(r[k], in.yha, q[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fa_add<CHK>(fF, f[k]);
                fa_add<CHK>(fJ, q[k]);
            }
        }
        if (DB) {
            double f[4], d[4], q[4], r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = in.xb * t[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = in.xhb * t[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) f[k] = f[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - p[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] - f[k];
            // J = mdiv(d, hb, yhb, ylb)
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = d[k] * in.ylb;
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = fma(d[k], in.yhb, q[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = fma(-in.hb, q[k], d[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = fma(r[k], in.yhb, q[k]);
            // Jn = mdiv(J, ajb, yaj, ylj)
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = q[k] * in.ylj;
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = fma(q[k], in.yaj, d[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = fma(-in.ajb, d[k], q[k]);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = fma(r[k], in.yaj, d[k]);
            if (first) d[0] = d[0] + 1.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = d[k] * f[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) sum = sum + d[k];
        }
    }

    template <bool CHK>
    __device__ __forceinline__ void run(int b0, const fv4 (&v)[4])
    {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double t4[4] = {tv[4 * c], tv[4 * c + 1], tv[4 * c + 2], tv[4 * c + 3]};
            group4<CHK>(t4, v[c], CHK && c == 0 && b0 == 0);
        }
    }
};

// Exact sweep body: MINPACK's branchy enorm and true divisions, per lane.
struct ExactBody {
    static constexpr bool kPeel = false;
    const PassIn &in;
    const double *__restrict__ T64;
    double agiant;
    Enorm eF, eJ;
    double sum;
    float p00;   // the first sample

    __device__ __forceinline__ ExactBody(const PassIn &i, const double *T, double ag) : in(i), T64(T), agiant(ag)
    {
        en_zero(eF);
        en_zero(eJ);
        sum = 0.0;
        p00 = 0.0f;
    }

    __device__ void sample(double t, double pv, bool first)
    {
        if (in.A) {
            const double u = in.xa * t;
            const double f = u - pv;
            const double uh = in.xha * t;
            const double wa = uh - pv;
            const double d = wa - f;
            en_add(eF, f, agiant);
            const double J = d / in.ha;
            en_add(eJ, J, agiant);
            if (first) p00 = (float)pv;
        }
        if (in.B) {
            const double u = in.xb * t;
            const double f = u - pv;
            const double uh = in.xhb * t;
            const double wa = uh - pv;
            const double d = wa - f;
            const double J = d / in.hb;
            double Jn = J / in.ajb;
            if (first) Jn = Jn + 1.0;
            const double pr = Jn * f;
            sum = sum + pr;
        }
    }

    __device__ __forceinline__ void fence() {}
    __device__ __forceinline__ void load_T(int) {}
    template <bool CHK>
    __device__ void run(int b0, const fv4 (&v)[4])
    {
        for (int c = 0; c < 4; ++c) {
            const int i = b0 + 4 * c;
            sample(T64[i], (double)v[c].x, i == 0);
            sample(T64[i + 1], (double)v[c].y, false);
            sample(T64[i + 2], (double)v[c].z, false);
            sample(T64[i + 3], (double)v[c].w, false);
        }
    }
};

template <bool DA, bool DB, bool FUSE = false>
__device__ __forceinline__ void fast_sweep(const DmaTiles &d, int ldD, const PassIn &in,
                                           const double *__restrict__ T64, double agiant, PassOut &out,
                                           bool issued = false)
{
    FastBody<DA, DB, FUSE> body(in, T64);
    sweep_dma(d, ldD, body, issued);
    const uint32_t hg = (uint32_t)((unsigned long long)__double_as_longlong(agiant * agiant) >> 32);
    out.p0 = body.p00;
    out.sum = FUSE ? body.fsum : body.sum;
    out.fnorm = fa_fin(body.fF);
    out.acnorm = fa_fin(body.fJ);
    out.bad = DA && in.A && !(body.lo_ok && fa_hi_ok(body.fF, hg) && fa_hi_ok(body.fJ, hg));
    // the dot counts only where J stayed in the fast path's verified range (mdiv = RN division)
    out.jt = FUSE && body.jt && !out.bad;
}

// ---- split lmdif: state machine (k_fit_state) <-> data sweeps (k_fit_pass) ----
// Per-profile state lives in HBM as structure-of-arrays (FitState below);
// a round is one k_fit_pass (every profile with a pending request reads its
// samples once) followed by one k_fit_state (each lane consumes its sweep
// result and runs MINPACK's scalar logic up to its next data request).

__device__ __forceinline__ void lm_load(LmState &L, const FitStateArrays &S, long k)
{
    L.x = S.x[k]; L.fnorm = S.fnorm[k]; L.par = S.par[k]; L.delta = S.delta[k]; L.diag = S.diag[k];
    L.xnorm = S.xnorm[k]; L.acnorm = S.acnorm[k]; L.J0 = S.J0[k]; L.f0 = S.f0[k];
    L.aj = S.aj[k]; L.r = S.r[k]; L.Jn0 = S.Jn0[k]; L.qtf = S.qtf[k]; L.gnorm = S.gnorm[k];
    L.x2 = S.x2[k]; L.pnorm = S.pnorm[k]; L.wa1 = S.wa1[k];
    L.iter = S.iter[k]; L.nfev = S.nfev[k]; L.info = 0;
    L.acn2 = 0.0; L.J02 = 0.0; L.f02 = 0.0;
}

__device__ __forceinline__ void lm_store(const LmState &L, const FitStateArrays &S, long k)
{
    S.x[k] = L.x; S.fnorm[k] = L.fnorm; S.par[k] = L.par; S.delta[k] = L.delta; S.diag[k] = L.diag;
    S.xnorm[k] = L.xnorm; S.acnorm[k] = L.acnorm; S.J0[k] = L.J0; S.f0[k] = L.f0;
    S.aj[k] = L.aj; S.r[k] = L.r; S.Jn0[k] = L.Jn0; S.qtf[k] = L.qtf; S.gnorm[k] = L.gnorm;
    S.x2[k] = L.x2; S.pnorm[k] = L.pnorm; S.wa1[k] = L.wa1;
    S.iter[k] = L.iter; S.nfev[k] = L.nfev;
}

// A round's input list.  k_fit_state writes the survivors of a round into the
// P-entry list buffer partitioned by request: A requests from the front
// (list[0 .. nA)), B requests from the end down (list[P - 1 - j], j < nB), so
// that the next round's waves hold one kind each (a wave with both runs both
// sweep bodies; round 0's unanswered B requests and the profiles one stage
// behind after them would otherwise spread over most waves).  Both counts
// share one 64-bit word, [63:32] nB and [31:0] nA, so that one atomic per
// block returns both list offsets; the blocks that finished are counted in a
// word of their own (k_fit_state).
__host__ __device__ constexpr unsigned long long rl_pack(unsigned long long nB, unsigned long long nA)
{
    return (nB << 32) | nA;
}
struct RoundList {
    const int32_t *list;
    long nA, nB, P;
    __device__ __forceinline__ RoundList(const int32_t *l, const unsigned long long *ctr, long P_) : list(l), P(P_)
    {
        if (!l) {
            nA = P_;
            nB = 0;
        } else {
            const unsigned long long v = *ctr;
            nA = (long)(v & 0xffffffffull);
            nB = (long)(v >> 32);
        }
    }
    __device__ __forceinline__ long n() const { return nA + nB; }
    __device__ __forceinline__ long at(long s) const
    {
        if (!list) return s;
        return s < nA ? (long)list[s] : (long)list[P - 1 - (s - nA)];
    }
};

// m[k] = v for every profile k of a round list (the second fork: the profiles
// handed to k_fit_tail)
__global__ __launch_bounds__(256) void k_mark_list(const int32_t *__restrict__ list,
                                                   const unsigned long long *__restrict__ nctr, long P,
                                                   uint8_t *__restrict__ m, uint8_t v)
{
    const RoundList rl(list, nctr, P);
    const long slot = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot < rl.n()) m[rl.at(slot)] = v;
}

// request encoding in S.mode: ST_A0 / ST_A2 -> sweep A at S.xa; ST_B -> sweep B
// at (S.x, S.aj); ST_DONE -> nothing.  S.slow: J at x came from an exact sweep.
// also zeroes the round counters (nz32 words) and the late flags (P bytes, optional)
__global__ __launch_bounds__(256) void k_fit_init(FitStateArrays S, long P, int32_t *__restrict__ z32, int nz32,
                                                  uint8_t *__restrict__ late)
{
    const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nz32) z32[k] = 0;
    if (k >= P) return;
    if (late) late[k] = 0;
    S.mode[k] = ST_A0;
    S.xa[k] = 1.0;
    S.x[k] = 1.0; S.par[k] = 0.0; S.iter[k] = 1; S.nfev[k] = 0; S.slow[k] = 0;
}

// The first outer iteration, at x = 1 for every profile, has a Jacobian that is
// the template itself: h = eps |x| = 2^-26 exactly, (1 + 2^-26) t is exact for
// an f32 t, and whenever RN(t - p) and RN(RN((1 + 2^-26) t) - p) are exact (t
// and p within ~2^29 of each other, or p = 0) the forward difference is
// (2^-26 t) / 2^-26 = t exactly.  Then enorm(J) (= acnorm = ajnorm), the sign,
// Jn_0 and qtf's weights Jn_i = RN(J_i / aj) are the same for every profile
// (lm_outer, MINPACK qrfac with n = 1), and the B sweep's dot
// sum_i RN(Jn_i f_i) can be summed in round 0 together with the A sweep, which
// has the same f_i: one full sweep of the fit cube less per iteration.  A
// profile whose J differs anywhere (k_fit_pass checks J_i == T_i), or whose
// own acnorm / aj / Jn0 differ, sends its B request as before.
// R0: the round-0 form (list == nullptr, every request A at x = 1), which sums
// the first B sweep's dot in the same sweep (k_fit_prep's U); a kernel of its
// own so that the other rounds keep their register allocation (and occupancy)
template <bool R0>
__global__ __launch_bounds__(64) void k_fit_pass(const float *__restrict__ D, const double *__restrict__ T64,
                                                 long P, int nbin, int ldD, int nsw, int dtiled,
                                                 const int32_t *__restrict__ list,
                                                 const unsigned long long *__restrict__ nctr, FitStateArrays S,
                                                 const double *__restrict__ U)
{
    __shared__ __attribute__((aligned(16))) char lbuf[2 * FIT_BUF];
    const int lane = threadIdx.x;
    const long slot = (long)blockIdx.x * 64 + lane;
    const RoundList rl(list, nctr, P);
    const long nact = rl.n();   // the grid is only an upper bound
    if ((long)blockIdx.x * 64 >= nact) return;
    DmaTiles dt;
    dt.lds = lbuf;
    dt.tiled = dtiled;
    {
        const int c = (lane & 3) ^ ((lane >> 4) & 3);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const long sl = (long)blockIdx.x * 64 + m * 16 + (lane >> 2);
            long kr = 0;   // empty slots read row 0 (valid: D is padded)
            if (sl < nact) kr = rl.at(sl);
            dt.src[m] = D + d_ofs(kr, 4 * c, ldD, dtiled);
        }
        const uint32_t base = lds_u32(lbuf) + 16u * (uint32_t)(64 * (lane >> 4) + 4 * (lane & 15));
        const int g = (lane >> 2) & 3;
#pragma unroll
        for (int c2 = 0; c2 < 4; ++c2) dt.rd[c2] = base + 16u * (uint32_t)(c2 ^ g);
    }
    // the first tile pair is requested from the list alone, before the lanes'
    // lmdif state is read: the state's dependent loads (list -> mode -> x, aj)
    // then overlap the pair's memory latency instead of preceding it
    dma_tile(dt, dt.lds, 0);
    dma_tile(dt, dt.lds + FIT_BUF, FIT_TB);
    const bool in_range = slot < nact;
    const long k = in_range ? rl.at(slot) : 0;
    const int st = in_range ? S.mode[k] : ST_DONE;
    const bool reqA = (st == ST_A0) || (st == ST_A2);
    const bool reqB = (st == ST_B);
    if (!__any(reqA || reqB)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA may outlive the block's LDS
        return;
    }
    const double agiant = kRgiant / (double)nbin;
    const double eps = sqrt(DBL_EPSILON);
    PassIn in;
    in.xa = reqA ? S.xa[k] : 1.0;
    in.ha = eps * fabs(in.xa);
    if (in.ha == 0.0) in.ha = eps;
    in.xha = in.xa + in.ha;
    in.yha = 1.0 / in.ha;
    in.yla = recip_lo(in.ha, in.yha);
    in.xb = reqB ? S.x[k] : 1.0;
    in.hb = eps * fabs(in.xb);
    if (in.hb == 0.0) in.hb = eps;
    in.xhb = in.xb + in.hb;
    in.yhb = 1.0 / in.hb;
    in.ylb = recip_lo(in.hb, in.yhb);
    in.ajb = reqB ? S.aj[k] : 1.0;
    in.yaj = 1.0 / in.ajb;
    in.ylj = recip_lo(in.ajb, in.yaj);
    const bool slow = reqB && S.slow[k];
    const bool fastA = reqA && x_in_sq_range(in.xa);
    const bool fastB = reqB && !slow && x_in_fast_range(in.xb) && x_in_fast_range(in.ajb);
    in.A = fastA;
    in.B = fastB;
    PassOut o;
    o.bad = o.jt = false;
    o.fnorm = o.acnorm = o.sum = 0.0;
    o.p0 = 0.0f;
    const bool anyA = __any(fastA), anyB = __any(fastB);
    if constexpr (R0) {
        // every profile at x = 1: the first B sweep's dot rides along (k_fit_prep)
        // (the dot is summed even when k_fit_prep found no shared qrfac, U[0] == 0:
        // k_fit_state then ignores it)
        in.ajb = U[2];
        in.yaj = 1.0 / in.ajb;
        in.ylj = recip_lo(in.ajb, in.yaj);
        // uniform, but held in VGPRs: the sweep's scalars (a tile of template
        // values) already fill the SGPR file
        asm volatile("" : "+v"(in.ajb), "+v"(in.yaj), "+v"(in.ylj));
        if (anyA) fast_sweep<true, false, true>(dt, nsw, in, T64, agiant, o, true);
    } else {
        if (anyA && anyB)
            fast_sweep<true, true>(dt, nsw, in, T64, agiant, o, true);
        else if (anyA)
            fast_sweep<true, false>(dt, nsw, in, T64, agiant, o, true);
        else if (anyB)
            fast_sweep<false, true>(dt, nsw, in, T64, agiant, o, true);
    }
    const bool exA = reqA && (!fastA || o.bad);
    const bool exB = reqB && !fastB;
    if (__any(exA || exB)) {
        PassIn ie = in;
        ie.A = exA;
        ie.B = exB;
        ExactBody body(ie, T64, agiant);
        // the early tile pair is still pending when no fast sweep consumed it
        const bool fast_ran = R0 ? anyA : (anyA || anyB);
        sweep_dma(dt, nsw, body, !fast_ran);
        if (exA || exB) {
            if (exA) o.p0 = body.p00;
            o.sum = body.sum;
            o.fnorm = en_fin(body.eF);
            o.acnorm = en_fin(body.eJ);
        }
    }
    // The outputs, as few bytes as possible: written into the sweep's read
    // stream, a DRAM write costs ~10x its size (tools/ubench_sweep: five 8-B
    // fields per profile +90 us per 4.7-GB round, one +20 us).  The two norms
    // carry the flags in their sign bits (both are >= 0 or NaN, whose sign
    // nothing reads): exA on fnorm, jt on acnorm.  f0 and J0, the residual and
    // the Jacobian at sample 0, are recomputed by k_fit_state from the first
    // sample, which round 0 stores once (OutS::f0J0).
    if (reqA) {
        // both norms in one 16-B store (o_fnorm's and o_acnorm's arrays are
        // adjacent: read as one double2 array of P entries)
        ((double2 *)S.o_fnorm)[k] = make_double2(exA ? -fabs(o.fnorm) : fabs(o.fnorm),
                                                 o.jt ? -fabs(o.acnorm) : fabs(o.acnorm));
        if (o.jt) S.o_sum[k] = o.sum;
        if (R0) S.p0[k] = o.p0;
    }
    if (reqB) S.o_sum[k] = o.sum;
}

// One profile's MINPACK transition after its sweep (k_fit_state): request
// st, the sweep's results from o (OutS: k_fit_pass's o_* fields), the lmdif
// state read from and written to S; returns the next request (ST_DONE: amp /
// info written).
struct OutS {
    const FitStateArrays &S;
    long k;
    __device__ __forceinline__ double fnorm() const { return fabs(((const double2 *)S.o_fnorm)[k].x); }
    __device__ __forceinline__ double acnorm() const { return fabs(((const double2 *)S.o_fnorm)[k].y); }
    __device__ __forceinline__ double sum() const { return S.o_sum[k]; }
    // bit 0: the A sweep took the exact path; bit 1: J(1) == T (round 0)
    __device__ __forceinline__ int exact() const
    {
        const double2 n = ((const double2 *)S.o_fnorm)[k];
        return (signbit(n.x) ? 1 : 0) | (signbit(n.y) ? 2 : 0);
    }
    // the residual f0 and the Jacobian J0 at sample 0 of the A sweep at x: the
    // sweep's own operations on its first sample (ExactBody::sample; the fast
    // bodies' four-op division is RN(d / h) wherever their result is used, and
    // at x = 1 d 2^26 = d / 2^-26), from the first sample round 0 stored
    __device__ __forceinline__ void f0J0(double x, double &f0, double &J0) const
    {
        const double eps = sqrt(DBL_EPSILON);
        double h = eps * fabs(x);
        if (h == 0.0) h = eps;
        const double xh = x + h;
        const double t = S.T64[0], pv = (double)S.p0[k];
        const double u = x * t;
        const double f = u - pv;
        const double uh = xh * t;
        const double wa = uh - pv;
        const double d = wa - f;
        f0 = f;
        J0 = d / h;
    }
};
template <typename Out>
__device__ __forceinline__ int fit_transition(const FitStateArrays &S, long k, int st, const Out &o,
                                              double *__restrict__ amp_o, int32_t *__restrict__ info_o)
{
    LmState L;
    if (st == ST_B) {
        // after a B sweep only qtf and the inner-loop start change: read the
        // fields lm_after_b / lm_after_qtf / lm_start_inner use, write the
        // ones they set (half the state traffic of a full load/store)
        L.Jn0 = S.Jn0[k]; L.f0 = S.f0[k]; L.fnorm = S.fnorm[k]; L.acnorm = S.acnorm[k]; L.r = S.r[k];
        L.diag = S.diag[k]; L.delta = S.delta[k]; L.par = S.par[k]; L.x = S.x[k]; L.iter = S.iter[k];
        L.info = 0;
        st = lm_after_b(L, o.sum());
        S.qtf[k] = L.qtf; S.gnorm[k] = L.gnorm; S.diag[k] = L.diag; S.par[k] = L.par;
        S.delta[k] = L.delta; S.wa1[k] = L.wa1; S.x2[k] = L.x2; S.pnorm[k] = L.pnorm;
    } else if (st == ST_A0) {
        // the first transition: the state is k_fit_init's (x = 1, par = 0,
        // iter = 1) and lm_outer reads nothing else; on the usual way out (a B
        // request) only the fields it set are written
        L.x = 1.0; L.par = 0.0; L.iter = 1; L.info = 0;
        L.acn2 = 0.0; L.J02 = 0.0; L.f02 = 0.0;
        L.fnorm = o.fnorm();
        L.nfev = 1;
        L.acnorm = o.acnorm();
        o.f0J0(1.0, L.f0, L.J0);
        const int oe = o.exact();
        S.slow[k] = oe & 1;
        st = lm_outer(L);
        // J(1) == T and the same qrfac as k_fit_prep's: the round-0 sweep
        // already summed qtf's dot, so the B request is answered here
        if (st == ST_B && (oe & 2) && S.U[0] != 0.0 && L.acnorm == S.U[1] && L.aj == S.U[2] &&
            L.Jn0 == S.U[3]) {
            st = lm_after_b(L, o.sum());
            lm_store(L, S, k);
        } else if (st == ST_B) {
            S.fnorm[k] = L.fnorm; S.nfev[k] = L.nfev; S.acnorm[k] = L.acnorm; S.f0[k] = L.f0;
            S.J0[k] = L.J0; S.Jn0[k] = L.Jn0; S.aj[k] = L.aj; S.r[k] = L.r; S.diag[k] = L.diag;
            S.xnorm[k] = L.xnorm; S.delta[k] = L.delta;
        } else {
            lm_store(L, S, k);
        }
    } else if (st == ST_A2) {
        // lm_after_a2 and what follows it read 14 of the 19 fields (acnorm, J0,
        // f0, aj and Jn0 are set anew on the way that uses them), and write: on
        // a rejected step, the inner loop's 6 (nfev, par, delta, wa1, x2,
        // pnorm); on an accepted one those and the outer iteration's 13; on
        // ST_DONE, nothing but amp / info (most profiles end here)
        L.x = S.x[k]; L.fnorm = S.fnorm[k]; L.par = S.par[k]; L.delta = S.delta[k]; L.diag = S.diag[k];
        L.xnorm = S.xnorm[k]; L.r = S.r[k]; L.qtf = S.qtf[k]; L.gnorm = S.gnorm[k]; L.x2 = S.x2[k];
        L.pnorm = S.pnorm[k]; L.wa1 = S.wa1[k]; L.iter = S.iter[k]; L.nfev = S.nfev[k]; L.info = 0;
        L.acnorm = L.J0 = L.f0 = L.aj = L.Jn0 = 0.0;   // not read before they are set
        L.acn2 = o.acnorm();
        o.f0J0(L.x2, L.f02, L.J02);   // the A request was at the trial point x2
        bool accepted = false;
        st = lm_after_a2(L, o.fnorm(), &accepted);
        if (st != ST_DONE) {
            S.nfev[k] = L.nfev; S.par[k] = L.par; S.delta[k] = L.delta; S.wa1[k] = L.wa1; S.x2[k] = L.x2;
            S.pnorm[k] = L.pnorm;
            if (accepted) {
                S.x[k] = L.x; S.xnorm[k] = L.xnorm; S.fnorm[k] = L.fnorm; S.iter[k] = L.iter;
                S.acnorm[k] = L.acnorm; S.J0[k] = L.J0; S.f0[k] = L.f0; S.aj[k] = L.aj; S.r[k] = L.r;
                S.Jn0[k] = L.Jn0; S.qtf[k] = L.qtf; S.gnorm[k] = L.gnorm; S.diag[k] = L.diag;
                S.slow[k] = o.exact() & 1;   // J at the new x came from this sweep
            }
        }
    } else if (st != ST_DONE) {
        return st;   // (no other request exists)
    } else {
        return ST_DONE;
    }
    S.mode[k] = st;
    if (st == ST_A2) S.xa[k] = L.x2;
    if (st == ST_DONE) {
        amp_o[k] = L.x;
        info_o[k] = L.info;
    }
    return st;
}

// Consume the sweep result, run lmdif's scalar logic to the next request.
// Survivors (profiles still needing a sweep) are appended to next_list;
// *next_n counts them (order within the list is irrelevant: profiles are
// independent).  The append is aggregated per block (one atomic per 512
// profiles), and the last block to finish publishes the final count to
// host-mapped memory (host_n), so the host needs no copy dispatch to learn it.
// BS threads per block: 512 for rounds of kStateSmallP profiles or more,
// 256 below (twice the blocks: C5 47.8 -> 45.6-46.3 ms per clean; C2's late
// rounds 25.41-25.43 -> 25.29-25.31; 256 for C2's full rounds too: 26.55
// against 26.44-26.49)
constexpr long kStateSmallP = 524288;
template <int BS>
__global__ __launch_bounds__(BS) void k_fit_state(FitStateArrays S, long P, const int32_t *__restrict__ list,
                                                            const unsigned long long *__restrict__ nctr,
                                                            double *__restrict__ amp_o, int32_t *__restrict__ info_o,
                                                            int32_t *__restrict__ next_list,
                                                            unsigned long long *__restrict__ ctr,
                                                            unsigned *__restrict__ done, int32_t *host_n,
                                                            uint8_t *__restrict__ late)
{
    __shared__ int wcnt[BS / 64];
    __shared__ int woff[BS / 64];
    __shared__ int wcntB[BS / 64];
    __shared__ int woffB[BS / 64];
    const long slot = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const RoundList rl(list, nctr, P);
    const long nact = rl.n();
    // the grid is sized from an upper bound: blocks past the list return at
    // once, and only the nblk blocks with work take part in the append (a
    // same-address atomic each, ~12 ns apiece, serialised)
    const long nblk = (nact + blockDim.x - 1) / blockDim.x;
    if ((long)blockIdx.x >= nblk) {
        if (nblk == 0 && blockIdx.x == 0 && threadIdx.x == 0)   // empty list: the count is 0
            __hip_atomic_store(host_n, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    int still = 0, stillB = 0;
    long k = 0;
    if (slot < nact) {
        k = rl.at(slot);
        const int st = fit_transition(S, k, S.mode[k], OutS{S, k}, amp_o, info_o);
        if (st != ST_DONE) still = st == ST_B ? 2 : 1;   // B requests go to the list's end
    }
    if (late && still) late[k] = 1;   // the fork round: still fitting after it
    // block-aggregated append, partitioned by request (RoundList)
    stillB = still == 2;
    still = still == 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(still), mB = __ballot(stillB);
    if (lane == 0) {
        wcnt[wave] = __popcll(m);
        wcntB[wave] = __popcll(mB);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0, totB = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            tot += wcnt[w];
            totB += wcntB[w];
        }
        // one atomic per block for both list offsets (B count, A count)
        const unsigned long long old = atomicAdd(ctr, rl_pack((unsigned)totB, (unsigned)tot));
        long base = (long)(old & 0xffffffffull), baseB = (long)(old >> 32);
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            woff[w] = (int)base;
            base += wcnt[w];
            woffB[w] = (int)baseB;
            baseB += wcntB[w];
        }
        // then the finished-block count.  Both atomics are performed where
        // device-scope atomics are (coherent across XCDs) and return only once
        // performed; the wait below keeps a block's count behind its offset
        // atomic's return, so when the last block's count returns nblk - 1
        // every block's offsets were performed, and its load of ctr sees the
        // final counts of the round.  (An acq_rel count instead - an L2
        // write-back and invalidate per block - cost 1.4 ms per C2 clean.)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned fin = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fin == (unsigned)nblk - 1) {
            // (the last block only.  What makes its load of ctr see every
            // block's offset atomic is the hardware order above: each block's
            // returning offset atomic, then its vmcnt(0), then its count.  The
            // counts are relaxed - no release pairs with this acquire - so the
            // acquire fence only keeps the compiler and the L1 from serving the
            // load early; it is not a memory-model synchronisation.)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            const unsigned long long v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(host_n, (int32_t)((v & 0xffffffffull) + (v >> 32)), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    __syncthreads();
    if (still) next_list[woff[wave] + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)k;
    if (stillB) next_list[P - 1 - (woffB[wave] + __popcll(mB & ((1ull << lane) - 1ull)))] = (int32_t)k;
}

// ---- tail: the last few thousand profiles, one wave each, to completion ----
// Rounds over a small active list are latency-bound (a lone wave sweeping 64
// profiles).  Here one wave owns ONE profile: lanes compute the per-sample
// terms of a chunk in parallel (exact divisions), then every lane runs the
// sequential MINPACK accumulation over the chunk in LDS (same values in all
// lanes: uniform control flow), and the lmdif state machine runs in registers
// between sweeps — no host round trips, no state traffic.  All arithmetic is
// the exact path (true divisions, branchy enorm), so it matches k_fit_pass
// bit for bit whatever the lane's range.
#define TAIL_CH 256
#define TAIL_WAVES 2   // waves (profiles) per block: C4 2.88-2.92 -> 2.85-2.90 ms against 4; C2, C5 the same

// s += a[0], s += a[1], ... in order (and t over b, a second chain interleaved
// with it).  The terms are read from LDS in register blocks of SB, the next
// block's reads issued before the current block's adds, so the dependent f64
// adds, not the LDS latency, set the pace of the sequential MINPACK sums.
template <int SB, bool TWO>
__device__ __forceinline__ void seq_sums(const double *a, const double *b, int n, double &s, double &t)
{
    int q = 0;
    if (n >= SB) {
        double ca[SB], cb[SB];
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            ca[i] = a[i];
            if (TWO) cb[i] = b[i];
        }
        for (q = SB; q + SB <= n; q += SB) {
            double na[SB], nb[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                na[i] = a[q + i];
                if (TWO) nb[i] = b[q + i];
            }
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                s = s + ca[i];
                if (TWO) t = t + cb[i];
            }
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                ca[i] = na[i];
                if (TWO) cb[i] = nb[i];
            }
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            s = s + ca[i];
            if (TWO) t = t + cb[i];
        }
    }
    for (; q < n; ++q) {
        s = s + a[q];
        if (TWO) t = t + b[q];
    }
}

// One block: U = {valid, acnorm, aj, Jn0} (k_fit_pass's round-0 form computes
// Jn_i = RN(J_i / aj) itself, as the B sweep does).  MINPACK's enorm is a
// sequential sum: every thread squares its samples into LDS and checks the
// range, then one thread adds the squares in order (register blocks, the
// next block's reads ahead of the adds) - sqrt(sum_seq t^2) is MINPACK's enorm
// while every component is 0 or inside (RDWARF, agiant) (fa_add's argument);
// MINPACK's branchy enorm otherwise.
__global__ __launch_bounds__(256) void k_fit_prep(const double *__restrict__ T64, int nbin, int nsw,
                                                  double *__restrict__ U)
{
    extern __shared__ double sq[];   // [nsw]
    const double agiant = kRgiant / (double)nbin;
    int ok = 1;
    for (int i = threadIdx.x; i < nsw; i += blockDim.x) {
        const double a = fabs(T64[i]);
        ok &= (a == 0.0 || (a > kRdwarf && a < agiant)) ? 1 : 0;
        sq[i] = a * a;
    }
    const bool in_range = __syncthreads_and(ok) != 0;
    if (threadIdx.x != 0) return;
    double acn;
    if (in_range) {
        double s2 = 0.0, unused = 0.0;
        seq_sums<16, false>(sq, nullptr, nsw, s2, unused);
        acn = s2 != 0.0 ? sqrt(s2) : 0.0;   // MINPACK: sqrt(s2 (1 + 0)) with no small / large components
    } else {
        Enorm e;
        en_zero(e);
        for (int i = 0; i < nsw; ++i) en_add(e, T64[i], agiant);
        acn = en_fin(e);
    }
    const double J0 = T64[0];
    double ajnorm = acn, Jn0 = J0;   // lm_outer
    if (ajnorm != 0.0) {
        if (J0 < 0.0) ajnorm = -ajnorm;
        Jn0 = J0 / ajnorm;
        Jn0 = Jn0 + 1.0;
    }
    // the fast B sweep's conditions on aj as well (x = 1 is in range)
    const bool valid = acn != 0.0 && Jn0 != 0.0 && x_in_fast_range(ajnorm);
    U[0] = valid ? 1.0 : 0.0;
    U[1] = acn;
    U[2] = valid ? ajnorm : 1.0;
    U[3] = Jn0;
}

// one fit-cube row in either layout (d_ofs)
struct RowRef {
    const float *D;
    size_t k;
    int ldD, tiled;
    __device__ __forceinline__ float operator[](int i) const { return D[d_ofs(k, i, ldD, tiled)]; }
};

__device__ __forceinline__ void tail_sweep_a(const RowRef &p, const double *__restrict__ T64, int nbin,
                                             double xa, double agiant, double (*buf)[TAIL_CH], int lane,
                                             double &fnorm, double &acnorm, double &f0, double &J0)
{
    const double eps = sqrt(DBL_EPSILON);
    double h = eps * fabs(xa);
    if (h == 0.0) h = eps;
    const double xh = xa + h;
    Enorm eF, eJ;
    en_zero(eF);
    en_zero(eJ);
    for (int c0 = 0; c0 < nbin; c0 += TAIL_CH) {
        const int n = min(TAIL_CH, nbin - c0);
        bool okF = true, okJ = true;   // every component 0 or inside (RDWARF, agiant)
        for (int q = lane; q < n; q += 64) {
            const double t = T64[c0 + q];
            const double pv = (double)p[c0 + q];
            const double u = xa * t;
            const double f = u - pv;
            const double uh = xh * t;
            const double wa = uh - pv;
            const double d = wa - f;
            const double J = d / h;
            buf[0][q] = f;
            buf[1][q] = J;
            const double af = fabs(f), aJ = fabs(J);
            okF = okF && (af == 0.0 || (af > kRdwarf && af < agiant));
            okJ = okJ && (aJ == 0.0 || (aJ > kRdwarf && aJ < agiant));
            buf[2][q] = af * af;
            buf[3][q] = aJ * aJ;
        }
        okF = __all(okF);
        okJ = __all(okJ);
        wave_sync();
        if (c0 == 0) {
            f0 = buf[0][0];
            J0 = buf[1][0];
        }
        // in range, en_add is exactly s2 += x*x, in order (the squares were
        // formed above, off the dependency chain)
        if (okF && okJ) {   // the usual case: both chains interleaved
            double sF = eF.s2, sJ = eJ.s2;
            seq_sums<8, true>(buf[2], buf[3], n, sF, sJ);
            eF.s2 = sF;
            eJ.s2 = sJ;
        } else {
            if (okF) {
                double dummy = 0.0;
                seq_sums<16, false>(buf[2], nullptr, n, eF.s2, dummy);
            } else {
                for (int q = 0; q < n; ++q) en_add(eF, buf[0][q], agiant);
            }
            if (okJ) {
                double dummy = 0.0;
                seq_sums<16, false>(buf[3], nullptr, n, eJ.s2, dummy);
            } else {
                for (int q = 0; q < n; ++q) en_add(eJ, buf[1][q], agiant);
            }
        }
        wave_sync();
    }
    fnorm = en_fin(eF);
    acnorm = en_fin(eJ);
}

__device__ __forceinline__ double tail_sweep_b(const RowRef &p, const double *__restrict__ T64, int nbin,
                                               double x, double aj, double (*buf)[TAIL_CH], int lane)
{
    const double eps = sqrt(DBL_EPSILON);
    double h = eps * fabs(x);
    if (h == 0.0) h = eps;
    const double xh = x + h;
    double sum = 0.0;
    for (int c0 = 0; c0 < nbin; c0 += TAIL_CH) {
        const int n = min(TAIL_CH, nbin - c0);
        for (int q = lane; q < n; q += 64) {
            const double t = T64[c0 + q];
            const double pv = (double)p[c0 + q];
            const double u = x * t;
            const double f = u - pv;
            const double uh = xh * t;
            const double wa = uh - pv;
            const double d = wa - f;
            const double J = d / h;
            double Jn = J / aj;
            if (c0 + q == 0) Jn = Jn + 1.0;
            buf[0][q] = Jn * f;
        }
        wave_sync();
        double dummy = 0.0;
        seq_sums<16, false>(buf[0], nullptr, n, sum, dummy);
        wave_sync();
    }
    return sum;
}

// 3 waves per SIMD for the register allocation (2 waves: 0.1 ms per C2 clean slower)
__global__ __launch_bounds__(64 * TAIL_WAVES, 3) void k_fit_tail(const float *__restrict__ D,
                                                              const double *__restrict__ T64, long P, int nbin,
                                                              int ldD, int dtiled, const int32_t *__restrict__ list,
                                                              const unsigned long long *__restrict__ nctr,
                                                              FitStateArrays S,
                                                              double *__restrict__ amp_o,
                                                              int32_t *__restrict__ info_o,
                                                              unsigned long long *__restrict__ sweeps)
{
    __shared__ double sbuf[TAIL_WAVES][4][TAIL_CH];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double(*buf)[TAIL_CH] = sbuf[wave];
    const RoundList rl(list, nctr, P);
    const long nact = rl.n();
    const double agiant = kRgiant / (double)nbin;
    unsigned long long nsw = 0;
    for (long slot = (long)blockIdx.x * TAIL_WAVES + wave; slot < nact; slot += (long)gridDim.x * TAIL_WAVES) {
        const long k = rl.at(slot);
        int st = S.mode[k];
        if (st == ST_DONE) continue;
        LmState L;
        lm_load(L, S, k);
        double xa = S.xa[k];
        // the row's samples are contiguous in runs of 32 (tiled) or whole
        const RowRef p{D, (size_t)k, ldD, dtiled};
        while (st != ST_DONE) {
            ++nsw;
            if (st == ST_B) {
                const double sum = tail_sweep_b(p, T64, nbin, L.x, L.aj, buf, lane);
                st = lm_after_b(L, sum);
            } else {
                double fnorm, acnorm, f0 = 0.0, J0 = 0.0;
                tail_sweep_a(p, T64, nbin, xa, agiant, buf, lane, fnorm, acnorm, f0, J0);
                if (st == ST_A0) {
                    L.fnorm = fnorm;
                    L.nfev = 1;
                    L.acnorm = acnorm;
                    L.f0 = f0;
                    L.J0 = J0;
                    st = lm_outer(L);
                } else {
                    L.acn2 = acnorm;
                    L.f02 = f0;
                    L.J02 = J0;
                    st = lm_after_a2(L, fnorm);
                }
            }
            if (st == ST_A2) xa = L.x2;
        }
        if (lane == 0) {
            S.mode[k] = ST_DONE;
            amp_o[k] = L.x;
            info_o[k] = L.info;
        }
    }
    if (lane == 0 && nsw) atomicAdd(sweeps, nsw);
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
    wave_sync();
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
    wave_sync();
    Tp out = (Tp)0;
    if (lane == 0) {
        for (int o = 0; o < pl.nops; ++o) slot[nl + o] = slot[pl.op_a[o]] + slot[pl.op_b[o]];
        out = (Tp)0 + slot[pl.root];
        acc[0] = out;
    }
    wave_sync();
    out = acc[0];
    wave_sync();
    return out;
}

// Persistent blocks of `wpb` independent waves; each wave cleans profiles
// k = blockIdx.x*wpb + wave, += gridDim.x*wpb.  LDS: plan + twiddles (block-shared,
// loaded once) | per wave: complex work [n/2] (pow2) | X f32 [n] | pairwise scratch.
// Per profile: the f32 residual (iterative_cleaner.py:279-288, :272), dededispersion
// (:104), the ORIGINAL weight (:296) and the four diagnostics (:206-217) with
// numpy.ma data conventions.
// ---- mixed-radix (8/4/2) Stockham FFT helpers (forward, exp(-2 pi i jk/N)) ----
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 w)
{
    return make_double2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
// fused form for the power-of-two path (the FFT diagnostic is compared within
// a tolerance, never bit-for-bit: pocketfft's own rounding is not reproduced)
__device__ __forceinline__ double2 cmul_f(double2 a, double2 w)
{
    return make_double2(__builtin_fma(a.x, w.x, -(a.y * w.y)), __builtin_fma(a.x, w.y, a.y * w.x));
}
__device__ __forceinline__ double2 mul_mi(double2 a) { return make_double2(a.y, -a.x); }   // * (-i)

template <int R>
__device__ __forceinline__ void dft_small(double2 (&v)[R]);

template <>
__device__ __forceinline__ void dft_small<2>(double2 (&v)[2])
{
    const double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}

template <>
__device__ __forceinline__ void dft_small<4>(double2 (&v)[4])
{
    const double2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    const double2 s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    v[1] = cadd(d02, d13);
    v[3] = csub(d02, d13);
}

template <>
__device__ __forceinline__ void dft_small<8>(double2 (&v)[8])
{
    double2 e[4] = {v[0], v[2], v[4], v[6]};
    double2 o[4] = {v[1], v[3], v[5], v[7]};
    dft_small<4>(e);
    dft_small<4>(o);
    const double h = 0.70710678118654752440;   // sqrt(1/2)
    // o_k * exp(-2 pi i k/8), k = 0..3
    const double2 o1 = make_double2(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));
    const double2 o2 = mul_mi(o[2]);
    const double2 o3 = make_double2(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));
    v[0] = cadd(e[0], o[0]);
    v[4] = csub(e[0], o[0]);
    v[1] = cadd(e[1], o1);
    v[5] = csub(e[1], o1);
    v[2] = cadd(e[2], o2);
    v[6] = csub(e[2], o2);
    v[3] = cadd(e[3], o3);
    v[7] = csub(e[3], o3);
}

// exp(-2 pi i q/n) for 0 <= q < n from the half table tw[0..n/2)
__device__ __forceinline__ double2 twid(const double2 *tw, int q, int half)
{
    if (q < half) return tw[q];
    const double2 t = tw[q - half];
    return make_double2(-t.x, -t.y);
}

// One radix-R Stockham stage over m points (src -> dst), Ns = product of earlier radices.
// get(q) supplies src point q (lets the first stage read the real input directly).
template <int R, typename Get>
__device__ __forceinline__ void stockham_stage(Get get, double2 *dst, int m, int Ns, const double2 *tw, int n,
                                               int lane)
{
    const int nb = m / R;
    const int tmul = n / (R * Ns);
    for (int b = lane; b < nb; b += 64) {
        const int k = b & (Ns - 1);
        double2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = get(b + r * nb);
        if (Ns > 1) {
#pragma unroll
            for (int r = 1; r < R; ++r) v[r] = cmul(v[r], twid(tw, r * k * tmul, n / 2));
        }
        dft_small<R>(v);
        const int idx = (b - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) dst[idx + r * Ns] = v[r];
    }
}

struct DiagLayout {
    int ntw;          // twiddles in LDS
    size_t cw_off, x_off, p_off, scr_off, per_wave;
};

__host__ __device__ inline DiagLayout diag_layout(int n, int nleaf, int nops)
{
    DiagLayout L;
    const bool pow2 = (n & (n - 1)) == 0 && n >= 4;
    L.ntw = pow2 ? n / 2 : n;
    L.cw_off = 0;                                            // buffer A: n/2 complex
    const size_t cwb = (size_t)(pow2 ? n / 2 : 1) * 16;
    L.x_off = cwb;                                           // buffer B (n/2 complex) aliases X (n f64)
    const size_t xb = ((size_t)n * 8 + 15) & ~(size_t)15;
    const size_t pb = ((size_t)n * 4 + 15) & ~(size_t)15;
    L.p_off = L.x_off + (pow2 ? (cwb > xb ? cwb : xb) : xb);  // DIAG_CLOSED: the fit-cube row
    L.scr_off = L.p_off + pb;
    L.per_wave = L.scr_off + (size_t)(nleaf * 9 + nops + 8) * 8;
    L.per_wave = (L.per_wave + 15) & ~(size_t)15;
    return L;
}

__global__ __launch_bounds__(256) void k_diag(DiagArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ PwPlan pl;
    const int n = a.nbin;
    const int wpb = blockDim.x >> 6;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    {
        const int32_t *src = (const int32_t *)a.plan;
        int32_t *dst = (int32_t *)&pl;
        for (int q = threadIdx.x; q < (int)(sizeof(PwPlan) / 4); q += blockDim.x) dst[q] = src[q];
    }
    const DiagLayout lay = diag_layout(n, a.plan->nleaf, a.plan->nops);
    double2 *tw = (double2 *)smem;
    for (int q = threadIdx.x; q < lay.ntw; q += blockDim.x) tw[q] = a.tw[q];
    __syncthreads();
    unsigned char *wb = smem + (size_t)lay.ntw * 16 + (size_t)wave * lay.per_wave;
    double2 *cw = (double2 *)(wb + lay.cw_off);
    double *X = (double *)(wb + lay.x_off);   // f32 values unless data_f64
    float *Pr = (float *)(wb + lay.p_off);
    double *scr = (double *)(wb + lay.scr_off);
    const bool pow2 = (n & (n - 1)) == 0 && n >= 4;
    const size_t P = (size_t)a.nsub * a.nchan;
    const double *T64 = a.T64;
    const int mode = a.mode;

    for (size_t k = (size_t)blockIdx.x * wpb + wave; k < P; k += (size_t)gridDim.x * wpb) {
        const int c = (int)((unsigned)k % (unsigned)a.nchan);
        const float w = a.w0[k];
        const bool valid = (w != 0.0f);
        const int sh = mode == DIAG_STATS ? 0 : a.shift[c];
        wave_sync();   // previous profile's LDS reads are done
        double x = 0.0;
        int stt = 0;
        const float *p;
        if (mode == DIAG_CLOSED) {
            // the fit-cube row f32(ded - base0), dedispersed order, then the
            // closed-form amplitude from numpy pairwise sums
            const float *row = a.raw + k * (size_t)n;
            const float b = a.base[k];
            for (int j = lane; j < n; j += 64) {
                int i = j - sh;
                if (i < 0) i += n;
                Pr[i] = row[j] - b;
            }
            wave_sync();
            // the products in the stored (dispersed) order j: bin i = (j - sh) mod n
            const double dot = wave_pairwise<double>(pl, [&](int q) {
                int i = q - sh;
                if (i < 0) i += n;
                return T64[i] * (double)Pr[i];
            }, scr, lane);
            const double TT = *a.TT;
            x = TT != 0.0 ? dot / TT : 0.0;
            stt = isfinite(x) ? 1 : 5;
            if (lane == 0) {
                a.amp[k] = x;
                a.info[k] = stt;
            }
            p = Pr;
        } else {
            if (mode == DIAG_EXACT) {
                x = a.amp[k];
                stt = a.info[k];
            }
            p = a.D + k * (size_t)a.ldD;
        }
        const bool tr = a.dtiled && mode == DIAG_EXACT;   // the tiled fit cube (dt_ofs)
        auto prow = [&](int i) -> float { return tr ? a.D[dt_ofs(k, i, a.ldD)] : p[i]; };
        const bool ok = stt >= 1 && stt <= 4;
        // residual -> X (dispersed frame): X[j] = f32(f32(r[i]) * w), j = (i + sh) mod n
        // (f64(f32(r[i])) * f64(w) for f64 data)
        for (int i = lane; i < n; i += 64) {
            float R = 0.0f;
            if (mode == DIAG_STATS) {
                R = p[i];
            } else if (ok) {
                const double u = x * T64[i];
                double e = u - (double)prow(i);
                if (a.pr_on && i >= a.pr_start && i < a.pr_end) e = e * a.pr_factor;
                R = (float)e;
            }
            int j = i + sh;
            if (j >= n) j -= n;
            X[j] = a.data_f64 ? (double)R * (double)w : (double)(R * w);
        }
        wave_sync();
        double mean = 0.0, sd = 0.0, ptp = a.data_f64 ? 1e20 : (double)1e20f;   // numpy.ma fill value
        if (valid) {
            if (a.data_f64)
                mean = wave_pairwise<double>(pl, [&](int q) { return X[q]; }, scr, lane) / (double)n;
            else
                mean = (double)wave_pairwise<float>(pl, [&](int q) { return (float)X[q]; }, (float *)scr, lane) /
                       (double)n;
            const double mu = mean;
            const double ss = wave_pairwise<double>(
                pl,
                [&](int q) {
                    const double d = (double)X[q] - mu;
                    return d * d;
                },
                scr, lane);
            sd = sqrt(ss / (double)n);
            double mx = -INFINITY, mn = INFINITY;
            int nan = 0;
            for (int q = lane; q < n; q += 64) {
                const double v = X[q];
                if (isnan(v)) nan = 1;
                mx = fmax(mx, v);
                mn = fmin(mn, v);
            }
            mx = wave_tree<64>(mx, OpMaxF());
            mn = wave_tree<64>(mn, OpMinF());
            nan = wave_tree<64>(nan, OpOr());
            // max - min in the data dtype (exact widening of f32 values)
            ptp = nan ? (double)NAN : (a.data_f64 ? mx - mn : (double)((float)mx - (float)mn));
        }
        // fftmax: max_k |rfft(v)_k|, v = f64(X) - mean (valid) or f64(X) (invalid)
        const double mu = valid ? mean : 0.0;
        double best = 0.0;
        int nanf = 0;
        if (pow2) {
            const int m = n / 2;
            double2 *bufA = cw;
            double2 *bufB = (double2 *)X;    // X is dead once the first stage has read it
            int lg = 0;
            while ((1 << lg) < m) ++lg;
            // stage radices: as many 8s as possible, then one 4 or 2
            int Ns = 1, done = 0;
            double2 *src = nullptr, *dst = bufA;
            auto first = [&](int q) {
                return valid ? make_double2((double)X[2 * q] - mu, (double)X[2 * q + 1] - mu)
                             : make_double2((double)X[2 * q], (double)X[2 * q + 1]);
            };
            auto from = [&](int q) { return src[q]; };
            while (done < lg) {
                const int rem = lg - done;
                const int rl = rem >= 3 ? 3 : rem;
                if (Ns == 1) {
                    if (rl == 3) stockham_stage<8>(first, dst, m, Ns, tw, n, lane);
                    else if (rl == 2) stockham_stage<4>(first, dst, m, Ns, tw, n, lane);
                    else stockham_stage<2>(first, dst, m, Ns, tw, n, lane);
                } else {
                    if (rl == 3) stockham_stage<8>(from, dst, m, Ns, tw, n, lane);
                    else if (rl == 2) stockham_stage<4>(from, dst, m, Ns, tw, n, lane);
                    else stockham_stage<2>(from, dst, m, Ns, tw, n, lane);
                }
                wave_sync();
                Ns <<= rl;
                done += rl;
                src = dst;
                dst = (dst == bufA) ? bufB : bufA;
            }
            const double2 *Z = (lg == 0) ? nullptr : src;
            // X_k = (Z_k + conj(Z_{m-k}))/2 - i/2 W^k (Z_k - conj(Z_{m-k})), W = exp(-2 pi i/n)
            for (int kk = lane; kk <= m; kk += 64) {
                const double2 zk = Z[kk == m ? 0 : kk];
                const double2 zm = Z[kk == 0 ? 0 : m - kk];
                const double er = 0.5 * (zk.x + zm.x), ei = 0.5 * (zk.y - zm.y);
                const double orr = 0.5 * (zk.y + zm.y), oi = -0.5 * (zk.x - zm.x);
                double wr = -1.0, wi = 0.0;
                if (kk < m) {
                    const double2 wv = tw[kk];
                    wr = wv.x;
                    wi = wv.y;
                }
                const double re = er + (orr * wr - oi * wi);
                const double im = ei + (orr * wi + oi * wr);
                const double mag = hypot(re, im);
                if (isnan(mag)) nanf = 1;
                best = fmax(best, mag);
            }
        } else {
            for (int kk = lane; kk <= n / 2; kk += 64) {
                double sr = 0.0, si = 0.0;
                int q = 0;
                for (int j = 0; j < n; ++j) {
                    const double v = valid ? (double)X[j] - mu : (double)X[j];
                    const double2 wv = tw[q];
                    sr += v * wv.x;
                    si += v * wv.y;
                    q += kk;
                    if (q >= n) q -= n;
                }
                const double mag = hypot(sr, si);
                if (isnan(mag)) nanf = 1;
                best = fmax(best, mag);
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            best = fmax(best, __shfl_xor(best, off));
            nanf |= __shfl_xor(nanf, off);
        }
        if (lane == 0) {
            a.std_o[k] = valid && isfinite(mean) ? sd : 0.0;   // numpy.ma: a non-finite mean is masked -> std 0
            a.mean_o[k] = valid ? mean : 0.0;
            a.ptp_o[k] = ptp;
            a.fft_o[k] = nanf ? NAN : best;
        }
    }
}

// ---------------------------------------------------------------------------
// k_diag_p2<N>: the same diagnostics for power-of-two nbin = N (64..4096).
// A profile group of TPP = 64*WPP threads cleans one profile: one wave for
// N <= 1024, N/1024 waves for N = 2048/4096, so every thread holds the same
// 16 samples and one pairwise chain at every N >= 1024 (at N = 4096 one wave
// per profile needed a 32-KiB work array per wave: 1.25 waves/SIMD).
// numpy's pairwise sum for N = 2^k is a balanced tree over leaves of
// min(N,128) samples, each leaf 8 strided chains of min(N,128)/8 samples:
// chain c = (leaf c/8, accumulator c%8) lives in thread c%TPP, slot c/TPP, and
// the tree is reproduced exactly by xor-shuffles within a wave (IEEE add is
// commutative), a balanced add of the group's waves and a balanced in-register
// add of the slots.  X sits in LDS at idx + 8*(idx>>7) so the chain reads are
// bank-conflict free.  The rFFT is an in-place mixed-radix Stockham FFT of
// N/2 complex points (all of a stage's inputs are in registers before it
// writes).
// Modes (DiagArgs.mode):
//   DIAG_EXACT   residual from the exact fit's amplitude / status (ic.py:279-288)
//   DIAG_CLOSED  fit_mode 1: closed-form amplitude a = sum(T*p) / sum(T*T)
//                (numpy pairwise f64 sums over the dedispersed profile, the
//                fit cube row p = f32(ded - base0) formed from the raw cube),
//                then the same residual; writes amp / info
//   DIAG_STATS   comprehensive_stats alone (ic.py:181-226): X = f32(row * w)
template <int N, bool D64 = false>
struct P2 {
    static constexpr int WPP = N >= 2048 ? N / 1024 : 1;   // waves per profile
    static constexpr int TPP = 64 * WPP;                    // threads per profile
    static constexpr int M = N / 2;
    static constexpr int LEAF = N < 128 ? N : 128;
    static constexpr int NL = N / LEAF;
    static constexpr int CL = LEAF / 8;
    static constexpr int CH = 8 * NL;
    static constexpr int CPL = CH > TPP ? CH / TPP : 1;     // chains per thread
    static constexpr int ACT = CH < TPP ? CH : TPP;         // threads holding a chain
    static constexpr int WACT = ACT < 64 ? ACT : 64;        // ... per wave
    static constexpr int NPT = N / TPP;                     // samples per thread
    static constexpr int XPAD = N + 8 * NL;
    static constexpr int XBYTES = ((XPAD * (D64 ? 8 : 4) + 15) / 16) * 16;   // X: f32, or f64 (data_f64)
    static constexpr int CBYTES = M * 16;   // complex points at cidx(q)
    static constexpr int WORK_BYTES = XBYTES > CBYTES ? XBYTES : CBYTES;
    static constexpr int RED_BYTES = WPP > 1 ? 512 : 0;     // cross-wave partials
    static constexpr int GROUP_BYTES = WORK_BYTES + RED_BYTES;
    static constexpr int LG = __builtin_ctz(M);
    static constexpr int TW = 2 * M;   // twiddle entries: M post-processing + <= M stage tables
    // multi-wave groups: the table (up to 64 KiB) would cost blocks; it is read
    // through L1/L2 and the LDS holds only the groups' work arrays
    static constexpr bool TWG = WPP > 1;
    static constexpr int TW_LDS = TWG ? 0 : TW;
};

__device__ __forceinline__ int xaddr(int idx) { return idx + 8 * (idx >> 7); }

// xaddr((j0 + TPP u) mod N) for 0 <= j0 < N, in 3 VALU ops per u: the
// unwrapped address has compile-time offsets from one base (two for TPP = 64:
// xaddr(j0 + 64 u) = xaddr(j0) + 64 u + 8 ((u + bit6(j0)) >> 1)), and
// xaddr(j + N) = xaddr(j) + xaddr(N), so the wrap is an unsigned min
template <int N, int TPP>
struct XWrap {
    int a0, a1;
    __device__ __forceinline__ explicit XWrap(int j0) : a0(xaddr(j0)), a1(TPP == 64 ? xaddr(j0) + ((j0 >> 3) & 8) : 0) {}
    __device__ __forceinline__ int operator()(int u) const
    {
        constexpr int XN = N + 8 * (N >> 7);
        const int off = TPP % 128 == 0 ? u * (TPP + TPP / 16) : 64 * u + 8 * (u >> 1);
        const int au = ((TPP == 64 && (u & 1)) ? a1 : a0) + off;
        return (int)min((unsigned)au, (unsigned)(au - XN));
    }
};
// complex work array slot of point q: XOR swizzle of the low 3 bits with bits
// 3-5.  Conflict-free for every access of the kernel: the radix-8 scatters
// (ds_write_b128, 8-lane groups over 32 banks: low bits (b&7)^r or r^(b&7)) and
// the contiguous / reversed gathers (ds_read_b128, 16-lane groups over 64 banks).
__device__ __forceinline__ int cidx(int q) { return q ^ ((q >> 3) & 7); }
// Address forms with compile-time offsets (the thread index is opaque to the
// compiler, so it cannot split these itself):
//   cidx(x + 64 m) = cidx(x) + 64 m                 (the XOR reads bits 3-5 only)
//   xaddr(x + 8 q) = xaddr(x) + 8 q                 if x % 128 + 8 q < 128
//   xaddr(x + 128 m) = xaddr(x) + 136 m

// barrier of a profile group: one wave needs only ordering of its LDS ops
template <int WPP>
__device__ __forceinline__ void gsync()
{
    if constexpr (WPP > 1) __syncthreads();
    else wave_sync();
}

template <typename T, int CPL>
__device__ __forceinline__ T tree_slots(const T (&v)[CPL])
{
    if constexpr (CPL == 1) return v[0];
    else if constexpr (CPL == 2) return v[0] + v[1];
    else if constexpr (CPL == 4) return (v[0] + v[1]) + (v[2] + v[3]);
    else return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));   // CPL == 8
}

// Group-uniform reduction of a per-thread value: the wave tree over its WACT
// active lanes, then (WPP > 1) a balanced tree over the group's waves through
// `red` (WPP slots of 8 B, one slot array per call site; both barriers keep the
// slots reusable on the next profile).
template <int WPP, int WACT, typename T, typename Op>
__device__ __forceinline__ T group_tree(T v, Op op, T *red, int wave, int lane)
{
    T w = wave_tree<WACT>(v, op);
    if constexpr (WPP == 1) {
        return w;
    } else {
        if (lane == 0) red[wave] = w;
        __syncthreads();
        T r;
        if constexpr (WPP == 2) r = op(red[0], red[1]);
        else r = op(op(red[0], red[1]), op(red[2], red[3]));   // WPP == 4
        __syncthreads();
        return r;
    }
}

// chain sums (one per slot) -> the pairwise total over the group, balanced
// over threads, then over slots
template <int N, typename T>
__device__ __forceinline__ T chain_total(const T (&cs)[P2<N>::CPL], T *red, int wave, int lane)
{
    using C = P2<N>;
    T fs[C::CPL];
#pragma unroll
    for (int sl = 0; sl < C::CPL; ++sl) fs[sl] = group_tree<C::WPP, C::WACT>(cs[sl], OpAdd(), red + 8 * sl, wave, lane);
    return tree_slots<T, C::CPL>(fs);
}

// One radix-R Stockham stage (compile-time R, NS = product of earlier radices),
// in place: every input of the stage is in registers before it writes.
// stw: this stage's twiddles w^(r k), w = exp(-2 pi i/(R NS)), as [k][r-1]
// (host-built in long double; no recurrences).  FIRST: the input is the real
// signal X (f32, padded addresses) minus mu, read as complex pairs.
// DER: only each butterfly's base twiddle w = stw[k][0] is read; w^2 .. w^(R-1)
// come from repeated complex products (a few ulp off the table's correctly
// rounded values: the FFT diagnostic is compared within 1e-9, and this trades
// R - 2 LDS reads for 4 (R - 2) VALU ops per butterfly)
template <int R, int NS, bool FIRST, int M, int TPP, typename XT, bool DER = false>
__device__ __forceinline__ void p2_stage(double2 *C, const XT *X, double mu, const double2 *stw, int t)
{
    constexpr int NB = M / R;
    constexpr int BPL = (NB + TPP - 1) / TPP;
    double2 v[BPL][R];
#pragma unroll
    for (int u = 0; u < BPL; ++u) {
        const int b = t + TPP * u;
        if (NB % TPP == 0 || b < NB) {
            // 2 q = 2 b + 2 r NB: a multiple of 128 apart when NB % 64 == 0
            const XT *xb = X + xaddr(2 * b);
            const double2 *cb = C + cidx(b);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int q = b + r * NB;
                if (FIRST) {
                    const XT *xq = NB % 64 == 0 ? xb + r * (2 * NB + NB / 8) : X + xaddr(2 * q);
                    if constexpr (sizeof(XT) == 8) {
                        const double2 xv = *(const double2 *)xq;
                        v[u][r] = make_double2(xv.x - mu, xv.y - mu);
                    } else {
                        const float2 xv = *(const float2 *)xq;
                        v[u][r] = make_double2((double)xv.x - mu, (double)xv.y - mu);
                    }
                } else {
                    v[u][r] = NB % 64 == 0 ? cb[r * NB] : C[cidx(q)];
                }
            }
        }
    }
    gsync<TPP / 64>();
#pragma unroll
    for (int u = 0; u < BPL; ++u) {
        const int b = t + TPP * u;
        if (NB % TPP == 0 || b < NB) {
            const int k = b & (NS - 1);
            if (NS > 1) {
                const double2 *tk = stw + k * (R - 1);
                if constexpr (DER) {
                    const double2 w1 = tk[0];
                    double2 wr = w1;
#pragma unroll
                    for (int r = 1; r < R; ++r) {
                        if (r > 1) wr = cmul_f(wr, w1);
                        v[u][r] = cmul_f(v[u][r], wr);
                    }
                } else {
#pragma unroll
                    for (int r = 1; r < R; ++r) v[u][r] = cmul_f(v[u][r], tk[r - 1]);
                }
            }
            dft_small<R>(v[u]);
            const int idx = (b - k) * R + k;
            if constexpr (NS % 64 == 0) {
                double2 *cw = C + cidx(idx);
#pragma unroll
                for (int r = 0; r < R; ++r) cw[r * NS] = v[u][r];
            } else if constexpr (NS == 8 && R == 8) {
                // idx = 64 m + k (k < 8): cidx(idx + 8 r) = 64 m + 8 r + (k ^ r)
#pragma unroll
                for (int r = 0; r < R; ++r) C[(idx ^ r) + 8 * r] = v[u][r];
            } else if constexpr (NS == 1 && R == 8) {
                // idx = 8 b: cidx(idx + r) = idx + (r ^ (b & 7)) = (idx + (b & 7)) ^ r
                const int A = idx + (b & 7);
#pragma unroll
                for (int r = 0; r < R; ++r) C[A ^ r] = v[u][r];
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) C[cidx(idx + r * NS)] = v[u][r];
            }
        }
    }
    gsync<TPP / 64>();
}

// the whole N/2-point FFT as a compile-time chain of stages (radix 8 while >= 3
// levels remain, then 4 or 2); OFF = offset of the next stage table in tw
template <int M, int TPP, int LG, int DONE, int NS, int OFF, typename XT, bool DER = false>
__device__ __forceinline__ void p2_fft(double2 *C, const XT *X, double mu, const double2 *tw, int t)
{
    if constexpr (DONE < LG) {
        constexpr int REM = LG - DONE;
        constexpr int R = REM >= 3 ? 8 : (REM == 2 ? 4 : 2);
        constexpr int LR = R == 8 ? 3 : (R == 4 ? 2 : 1);
        p2_stage<R, NS, DONE == 0, M, TPP, XT, DER>(C, X, mu, tw + OFF, t);
        p2_fft<M, TPP, LG, DONE + LR, NS * R, (NS > 1 ? OFF + NS * (R - 1) : OFF), XT, DER>(C, X, mu, tw, t);
    }
}

// occupancy floors (waves per SIMD, <= 128 VGPRs): 4 for the multi-wave groups
// (the LDS allows 4 blocks of 4096 per CU) and for N = 1024 (the LDS allows 4
// waves/SIMD with 8-wave blocks), where the template is then read from L1
// instead of being held in 32 VGPRs.  Measured on C2 (k_diag ms per clean):
// 3 waves + template in registers 8.63, 4 waves + registers 8.10 (spills),
// 4 waves + L1 template 7.95 (profiles/r02_c2_diag_ab.txt).
template <int N>
constexpr int p2_min_waves() { return N >= 2048 ? 4 : (N == 1024 ? 4 : 1); }

// D64 (data_f64): psrchive's get_data returns f64, so apply_weights and the
// masked statistics run in f64 (iterative_cleaner.py:111-112, :206-209): X =
// f64(R) * f64(w), the mean's pairwise sum and ptp in f64.
template <int N, int MODE, bool D64>
__global__ __launch_bounds__(N >= 2048 ? P2<N>::TPP : 512, p2_min_waves<N>()) void k_diag_p2(DiagArgs a)
{
    using C = P2<N, D64>;
    using XT = typename std::conditional<D64, double, float>::type;
    constexpr int WPP = C::WPP, TPP = C::TPP, NPT = C::NPT;
    // one-wave groups keep the template and the next row in registers; the
    // multi-wave groups (N >= 2048) read both when needed and rely on occupancy
    constexpr bool TREG = WPP == 1 && N != 1024, PREFETCH = WPP == 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // [M] post-processing twiddles, then the stage tables (LDS copy unless TWG)
    const double2 *tw = C::TWG ? a.tw_p2 : (const double2 *)smem;
    const double *T = a.T64;          // L1/L2-resident, read coalesced
    constexpr int mode = MODE;
    const int lane = threadIdx.x & 63;
    // WPP == 1: independent waves (groups) per block; WPP > 1: the block is one group
    const int group = WPP == 1 ? (int)(threadIdx.x >> 6) : 0;
    const int gpb = WPP == 1 ? (int)(blockDim.x >> 6) : 1;
    const int wave = WPP == 1 ? 0 : (int)(threadIdx.x >> 6);   // wave within the group
    int t = WPP == 1 ? lane : (int)threadIdx.x;               // thread within the group
    if (!C::TWG) {
        for (int q = threadIdx.x; q < C::TW; q += blockDim.x) ((double2 *)smem)[q] = a.tw_p2[q];
        __syncthreads();
    }
    unsigned char *gb = smem + (size_t)C::TW_LDS * 16 + (size_t)group * C::GROUP_BYTES;
    XT *X = (XT *)gb;
    double2 *Cb = (double2 *)gb;   // aliases X after the first FFT stage has read it
    double *red = (double *)(gb + C::WORK_BYTES);   // 64 slots of 8 B (WPP > 1)
    const unsigned P = (unsigned)a.nsub * (unsigned)a.nchan;
    const unsigned stride = gridDim.x * gpb;
    const int nchan = a.nchan;
    // the template stays in registers, and each group loads the next profile's
    // row while it works on the current one: every global load of the loop is
    // issued ahead of its use (software pipelining)
    double tv[TREG ? NPT : 1];
    if (TREG) {
#pragma unroll
        for (int u = 0; u < NPT; ++u) tv[u] = T[t + TPP * u];
    }
    constexpr bool closed = mode == DIAG_CLOSED || mode == DIAG_FIT;
    const double TT = closed ? *a.TT : 0.0;
    // DIAG_EXACT reads the raw row, not the fit cube: the cube's value is
    // D_i = f32(raw_j - base0), j = (i + sh) mod N (k_chan_partials mode 3), and
    // the raw rows are contiguous whatever the cube's layout (dt_ofs)
    constexpr bool fromraw = mode == DIAG_CLOSED || mode == DIAG_EXACT;
    const float *rows = fromraw ? a.raw : a.D;
    const size_t ld = fromraw ? (size_t)N : (size_t)a.ldD;
    float pv[NPT];
    auto loadrow = [&](unsigned kk) {
        const float *pn = rows + (size_t)kk * ld;
#pragma unroll
        for (int u = 0; u < NPT; ++u) pv[u] = pn[t + TPP * u];
    };
    // profiles: all P, or the slots of a list, minus those with skip[k] != 0
    // (the two passes of the exact fit's forked diagnostics)
    const RoundList rl(a.list, a.nctr, (long)P);
    const unsigned nslot = (unsigned)rl.n();
    const uint8_t *skip = a.skip;
    auto next_slot = [&](unsigned sl) {   // the first slot >= sl this group measures (uniform)
        if (skip)
            while (sl < nslot && skip[rl.at(sl)]) sl += stride;
        return sl;
    };
    unsigned slot = next_slot(__builtin_amdgcn_readfirstlane(blockIdx.x * gpb + group));
    unsigned k = slot < nslot ? (unsigned)rl.at(slot) : 0u;
    // per-profile scalars, loaded one profile ahead as well
    double nx = 0.0;
    int nst = 0, nsh = 0;
    float nw = 0.0f, nb = 0.0f;
    if (slot < nslot) {
        if (PREFETCH) {
            loadrow(k);
        }
        if (mode == DIAG_EXACT) {
            nx = a.amp[k];
            nst = a.info[k];
        }
        if (fromraw) nb = a.base[k];
        nw = a.w0[k];
        nsh = (mode == DIAG_STATS || mode == DIAG_FIT) ? 0 : a.shift[k % (unsigned)nchan];
    }
    for (unsigned snext = 0; slot < nslot; slot = snext, k = slot < nslot ? (unsigned)rl.at(slot) : 0u) {
        snext = next_slot(slot + stride);
        // opaque to the optimiser: the LDS addresses of the FFT stages derive
        // from t, and hoisting all of them out of the loop costs ~100 VGPRs
        // (spills at N >= 2048); recomputing them is a few VALU ops each
        asm volatile("" : "+v"(t));
        double x = nx;
        int st = nst;
        const float w = nw;
        const bool valid = (w != 0.0f);
        const int sh = nsh;
        const float bk = nb;
        if (!PREFETCH) {
            loadrow(k);
        }
        gsync<WPP>();
        if (closed) {
            // fit cube row p_i = f32(ded_i - base0), i = (j - sh) mod N: to LDS in
            // the dedispersed order, then a = sum(T*p)/sum(T*T) over the chains
            // of the stored order (the products T_i p_i of j = i + sh)
            const XWrap<N, TPP> xw((t - sh) & (N - 1));
#pragma unroll
            for (int u = 0; u < NPT; ++u) X[xw(u)] = (XT)(pv[u] - bk);
            gsync<WPP>();
            double cs[C::CPL];
            const bool act = C::ACT >= TPP || t < C::ACT;   // every thread holds a chain at N >= 512
#pragma unroll
            for (int sl = 0; sl < C::CPL; ++sl) {
                const int ch = t + TPP * sl;
                const int base = (ch >> 3) * C::LEAF + (ch & 7);
                double r = 0.0;
                if (act) {
                    // the chain's stored (dispersed) samples j = base + 8 q pair
                    // with the dedispersed bins i = (j - sh) mod N
                    auto term = [&](int j) {
                        const int i = (j - sh) & (N - 1);
                        return T[i] * (double)X[xaddr(i)];
                    };
                    r = term(base);
#pragma unroll
                    for (int q = 1; q < C::CL; ++q) {
                        const double pr = term(base + 8 * q);
                        r = r + pr;
                    }
                }
                cs[sl] = r;
            }
            const double dot = 0.0 + chain_total<N, double>(cs, red, wave, lane);
            x = TT != 0.0 ? dot / TT : 0.0;
            st = isfinite(x) ? 1 : 5;
#pragma unroll
            for (int u = 0; u < NPT; ++u) pv[u] = (float)X[TPP % 128 == 0 ? xaddr(t) + u * (TPP + TPP / 16) : xaddr(t + TPP * u)];
            if (t == 0) {
                a.amp[k] = x;
                a.info[k] = st;
            }
            gsync<WPP>();
        }
        if constexpr (mode == DIAG_FIT) {   // the amplitude is all this mode produces
            if (PREFETCH && snext < nslot) loadrow((unsigned)rl.at(snext));
            continue;
        }
        const bool ok = st >= 1 && st <= 4;
        // residual -> X (dispersed frame, padded addresses)
        // X = apply_weights(R, w0): f32(R * w), or f64(R) * f64(w) for f64 data
        auto weigh = [&](float R) -> XT {
            if constexpr (D64) return (double)R * (double)w;
            else return R * w;
        };
        if (mode == DIAG_STATS) {
#pragma unroll
            for (int u = 0; u < NPT; ++u) X[TPP % 128 == 0 ? xaddr(t) + u * (TPP + TPP / 16) : xaddr(t + TPP * u)] = weigh(pv[u]);
        } else if (mode == DIAG_EXACT) {
            // sample j = t + TPP u of the raw row (dispersed frame) is the
            // dedispersed sample i = (j - sh) mod N: residual f32(x T_i - D_i)
            // with D_i = f32(raw_j - base0), written to X[j]
            const int i0 = (t - sh) & (N - 1);
            double tg[NPT];   // the template gathered at i: all loads issued before the first use
            {
                // byte offsets (8 i0 + 8 TPP u) mod 8N through a buffer descriptor: two VALU per load
                const __amdgpu_buffer_rsrc_t tr =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(T), 0, 8 * N, 0x00020000);
                const unsigned b0 = 8u * (unsigned)i0;
#pragma unroll
                for (int u = 0; u < NPT; ++u)
                    tg[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                           tr, (b0 + 8u * TPP * u) & (8u * N - 1u), 0, 0));
            }
            if (a.pr_on) {
#pragma unroll
                for (int u = 0; u < NPT; ++u) {
                    const int i = (i0 + TPP * u) & (N - 1);
                    const float pj = pv[u] - bk;
                    double e = x * tg[u] - (double)pj;
                    if (i >= a.pr_start && i < a.pr_end) e = e * a.pr_factor;
                    const float R = ok ? (float)e : 0.0f;
                    X[TPP % 128 == 0 ? xaddr(t) + u * (TPP + TPP / 16) : xaddr(t + TPP * u)] = weigh(R);
                }
            } else {
#pragma unroll
                for (int u = 0; u < NPT; ++u) {
                    const float pj = pv[u] - bk;
                    const double e = x * tg[u] - (double)pj;
                    const float R = ok ? (float)e : 0.0f;
                    X[TPP % 128 == 0 ? xaddr(t) + u * (TPP + TPP / 16) : xaddr(t + TPP * u)] = weigh(R);
                }
            }
        } else if (a.pr_on) {
            const XWrap<N, TPP> xw((t + sh) & (N - 1));
#pragma unroll
            for (int u = 0; u < NPT; ++u) {
                const int i = t + TPP * u;
                const double uu = x * (TREG ? tv[u] : T[i]);
                double e = uu - (double)pv[u];
                if (i >= a.pr_start && i < a.pr_end) e = e * a.pr_factor;
                const float R = ok ? (float)e : 0.0f;
                X[xw(u)] = weigh(R);
            }
        } else {
            const XWrap<N, TPP> xw((t + sh) & (N - 1));
#pragma unroll
            for (int u = 0; u < NPT; ++u) {
                const int i = t + TPP * u;
                const double uu = x * (TREG ? tv[u] : T[i]);
                const double e = uu - (double)pv[u];
                const float R = ok ? (float)e : 0.0f;
                X[xw(u)] = weigh(R);
            }
        }
        if (snext < nslot) {
            const unsigned kn = (unsigned)rl.at(snext);
            if (PREFETCH) loadrow(kn);
            if (mode == DIAG_EXACT) {
                nx = a.amp[kn];
                nst = a.info[kn];
            }
            if (fromraw) nb = a.base[kn];
            nw = a.w0[kn];
            nsh = mode == DIAG_STATS ? 0 : a.shift[kn % (unsigned)nchan];
        }
        gsync<WPP>();
        // masked ptp data is numpy.ma's fill value of the dtype: 1e20 (f64) / f32(1e20)
        double mean = 0.0, sd = 0.0, fftv = 0.0, ptp = D64 ? 1e20 : (double)1e20f;
        if (valid) {
            // chain values -> registers
            XT v[C::CPL][C::CL];
            const bool act = C::ACT >= TPP || t < C::ACT;   // every thread holds a chain at N >= 512
#pragma unroll
            for (int sl = 0; sl < C::CPL; ++sl) {
                const int ch = t + TPP * sl;
                const int base = (ch >> 3) * C::LEAF + (ch & 7);
#pragma unroll
                for (int q = 0; q < C::CL; ++q) v[sl][q] = act ? X[xaddr(base) + 8 * q] : (XT)0;
            }
            // mean: pairwise sum in the data dtype (f32, or f64 for f64 data)
            XT fs[C::CPL];
#pragma unroll
            for (int sl = 0; sl < C::CPL; ++sl) {
                XT r = v[sl][0];
#pragma unroll
                for (int q = 1; q < C::CL; ++q) r = r + v[sl][q];
                fs[sl] = r;
            }
            const XT s32 = (XT)0 + chain_total<N, XT>(fs, (XT *)(red + 16), wave, lane);
            mean = (double)s32 / (double)N;
            // var: f64 pairwise sum of (f64(X) - mean)^2
            double ds[C::CPL];
#pragma unroll
            for (int sl = 0; sl < C::CPL; ++sl) {
                double d0 = (double)v[sl][0] - mean;
                double r = d0 * d0;
#pragma unroll
                for (int q = 1; q < C::CL; ++q) {
                    const double d = (double)v[sl][q] - mean;
                    const double sq = d * d;
                    r = r + sq;
                }
                ds[sl] = r;
            }
            const double ss = 0.0 + chain_total<N, double>(ds, red + 24, wave, lane);
            sd = sqrt(ss / (double)N);
            // ptp (NaN-propagating), in the data dtype
            XT mx = -INFINITY, mn = INFINITY;
            if (act) {
#pragma unroll
                for (int sl = 0; sl < C::CPL; ++sl)
#pragma unroll
                    for (int q = 0; q < C::CL; ++q) {
                        mx = OpMaxF()(mx, v[sl][q]);
                        mn = OpMinF()(mn, v[sl][q]);
                    }
            }
            mx = group_tree<WPP, 64>(mx, OpMaxF(), (XT *)(red + 32), wave, lane);
            mn = group_tree<WPP, 64>(mn, OpMinF(), (XT *)(red + 36), wave, lane);
            // a NaN sample makes the pairwise sum s32 NaN; a NaN s32 without one
            // (inf - inf) is rare, and only then are the samples checked one by one
            int nan = 0;
            if (isnan(s32)) {   // group-uniform
                if (act) {
#pragma unroll
                    for (int sl = 0; sl < C::CPL; ++sl)
#pragma unroll
                        for (int q = 0; q < C::CL; ++q) nan |= isnan(v[sl][q]);
                }
                nan = group_tree<WPP, 64>(nan, OpOr(), (int *)(red + 40), wave, lane);
            }
            ptp = nan ? (double)NAN : (double)(XT)(mx - mn);
            // rFFT of f64(X) - mean: N/2-point complex Stockham, in place
            p2_fft<C::M, TPP, C::LG, 0, 1, C::M, XT>(Cb, X, mean, tw, t);
            // X_k = E_k + w^k O_k, computed as 2 X_k (the 1/2 factors are exact
            // powers of two, applied once to the maximum).  Bins pair up: with
            // E_k, O_k from Z_k and Z_(M-k), E_(M-k) = conj E_k, O_(M-k) = conj O_k
            // and w^(M-k) = -conj w^k, so X_(M-k) = conj(E_k - w^k O_k): one
            // product t = w^k O_k serves X_k = E + t and X_(M-k).  Pairs k = 0 ..
            // M/2 cover every bin: k = 0 gives DC (E + O) and Nyquist (E - O), k = M/2
            // pairs with itself.  NaN: the a2 are >= 0 or NaN, so their sum is NaN
            // iff one of them is.
            constexpr int H = C::M / 2;
            constexpr int JF = H / TPP;   // pair tasks every thread holds
            double best2 = 0.0, nsum = 0.0;
            auto post = [&](const double2 zk, const double2 zm, const double2 wv) {
                const double er = zk.x + zm.x, ei = zk.y - zm.y;
                const double orr = zk.y + zm.y, oi = zm.x - zk.x;
                const double tr = __builtin_fma(orr, wv.x, -(oi * wv.y));
                const double ti = __builtin_fma(orr, wv.y, oi * wv.x);
                const double re = er + tr, im = ei + ti;
                const double rm = er - tr, imm = ti - ei;
                const double a2 = __builtin_fma(re, re, im * im);
                const double b2 = __builtin_fma(rm, rm, imm * imm);
                nsum = nsum + a2;
                nsum = nsum + b2;
                best2 = fmax(best2, fmax(a2, b2));
            };
#pragma unroll
            for (int j = 0; j < JF; ++j) {
                // kk = t + TPP j, M - kk = (TPP - t) + (M - TPP (j + 1)): 64-multiples apart
                const int kk = t + TPP * j;
                const double2 zk = Cb[cidx(t) + TPP * j];
                const double2 zm = Cb[kk == 0 ? 0 : cidx(TPP - t) + (C::M - TPP * (j + 1))];
                post(zk, zm, tw[kk]);
            }
            {
                const int kk = t + TPP * JF;   // the rest: kk <= M/2 (one thread at N >= 256)
                if (kk <= H) post(Cb[cidx(kk)], Cb[cidx(kk == 0 ? 0 : C::M - kk)], tw[kk]);
            }
            int nanf = isnan(nsum);
            best2 = group_tree<WPP, 64>(best2, OpMaxF(), red + 44, wave, lane);
            nanf = group_tree<WPP, 64>(nanf, OpOr(), (int *)(red + 48), wave, lane);
            fftv = nanf ? NAN : 0.5 * sqrt(best2);
        } else {
            // invalid: rfft of f64(X) = +-0 -> 0, unless R was non-finite (X NaN)
            int nanx = 0;
            for (int i = t; i < N; i += TPP) nanx |= isnan(X[xaddr(i)]);
            nanx = group_tree<WPP, 64>(nanx, OpOr(), (int *)(red + 52), wave, lane);
            fftv = nanx ? NAN : 0.0;
        }
        if (t == 0) {
            a.std_o[k] = valid && isfinite(mean) ? sd : 0.0;   // numpy.ma: a non-finite mean is masked -> std 0
            a.mean_o[k] = valid ? mean : 0.0;
            a.ptp_o[k] = ptp;
            a.fft_o[k] = fftv;
        }
    }
}

// ---------------------------------------------------------------------------
// k_diag_cl<N, MODE>: DIAG_EXACT / DIAG_CLOSED diagnostics for N >= 1024 (f32
// data, no pulse region), chain layout.  Same arithmetic and the same bits as
// k_diag_p2 (ic.py:206-217, :272-288, :296); what changes is where the data
// lives:
// - Thread t of a profile group (L = N/16 threads: one wave at N = 1024) owns
//   pairwise chain t = (leaf t/8, accumulator t%8), the dispersed-frame samples
//   j = 128(t/8) + t%8 + 8q, q < 16, and loads them straight from the raw row
//   (one 64-bit address per profile, immediate offsets 32q).
// - The template is gathered at i = (j - sh) mod N from T2 = [T, T] (2N f64),
//   so the wrap costs nothing: one address, immediate offsets 64q.
// - mean / var / ptp run on the residual in registers (no LDS round trip), and
//   the var pass stores d = f64(X) - mean, which IS the FFT's input, as f64
//   into the complex work array in the first stage's gather order, so the FFT
//   starts without conversions or subtractions.  The work array's input image
//   is swizzled slot(p) = p ^ (((p >> 6) & 3) << 2): the chain stores (32
//   lanes x 8 B per half-wave) and the stage-1 gathers (16-B points) are both
//   bank-conflict free, and all addresses are per-thread bases + immediates.
// - Profile-uniform conditions (fit status, w0 == 0 / 1) are scalar branches.
// DIAG_CLOSED first forms the closed-form amplitude over the same chains (the
// stored order: the products T_i p_i of the lane's samples j, i = (j - sh) mod
// N, with the template gathered for the residual).
constexpr int p2_tw_entries(int N)
{
    const int M = N / 2;
    int lg = 0;
    while ((1 << lg) < M) ++lg;
    int n = M;
    for (int done = 0, ns = 1; done < lg;) {
        const int rem = lg - done, R = rem >= 3 ? 8 : (rem == 2 ? 4 : 2);
        if (ns > 1) n += ns * (R - 1);
        ns *= R;
        done += R == 8 ? 3 : (R == 4 ? 2 : 1);
    }
    return n;
}

// The one-wave (N = 1024) form: twiddles from an LDS copy (through L1/L2:
// 2.59 ms per pass against 2.00), 4 waves per SIMD, 8 profile groups per
// block.  Closed mode takes the dedispersed-order samples of the row by a
// second global read, not from an LDS copy of the registers' dispersed-order
// ones: the read misses L2 often enough to add 15 % to the pass's HBM traffic,
// but the copy costs LDS bandwidth, which binds at N = 1024 (C2 fast mode
// 2.48 -> 2.62 ms per pass with the copy).  Stage and spectrum twiddles are
// derived from one base twiddle per butterfly / lane (p2_stage DER; tw[t + L j]
// = tw[t] exp(-2 pi i j / 16)) instead of read one each for the multi-wave
// groups (N >= 2048), whose table is read through L1/L2 (C5 k_diag 2.81 ->
// 2.68 ms per launch); at N = 1024, whose table is in LDS, that measured no
// faster (2.005 -> 2.03).
template <int N>
struct CLay {
    static constexpr int L = N / 16;     // threads per profile = chains of 16 samples
    static constexpr int WPP = L / 64;   // waves per profile
    static constexpr int M = N / 2;
    static constexpr int LG = __builtin_ctz(M);
    static constexpr int GPB = WPP > 1 ? 1 : 8;   // profile groups per block
    static constexpr bool TWG = WPP > 1;   // multi-wave groups read the table through L1/L2
    static constexpr int TW_LDS = TWG ? 0 : p2_tw_entries(N);
    static constexpr int CBYTES = M * 16;
    static constexpr int RED_BYTES = WPP > 1 ? 512 : 0;
    static constexpr int GROUP_BYTES = CBYTES + RED_BYTES;
    static_assert(N >= 1024 && L % 64 == 0, "chain layout: one chain of 16 samples per thread");
};

__device__ __forceinline__ float ufirst(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ int ufirst(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double ufirst(double v)
{
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}

template <int N, int MODE>
__global__ __launch_bounds__(CLay<N>::L * CLay<N>::GPB, 4) void k_diag_cl(DiagArgs a)
{
    using C = CLay<N>;
    constexpr int L = C::L, WPP = C::WPP, M = C::M;
    constexpr bool closed = MODE == DIAG_CLOSED;
    constexpr bool stats = MODE == DIAG_STATS;   // X = f32(D_row * w): the rows are the residual
    constexpr bool twder = WPP > 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double2 *tw = C::TWG ? a.tw_p2 : (const double2 *)smem;
    const int lane = threadIdx.x & 63;
    const int group = WPP == 1 ? (int)(threadIdx.x >> 6) : 0;
    const int gpb = WPP == 1 ? (int)(blockDim.x >> 6) : 1;
    const int wave = WPP == 1 ? 0 : (int)(threadIdx.x >> 6);
    int t = WPP == 1 ? lane : (int)threadIdx.x;
    if (!C::TWG) {
        for (int q = threadIdx.x; q < C::TW_LDS; q += blockDim.x) ((double2 *)smem)[q] = a.tw_p2[q];
        __syncthreads();
    }
    unsigned char *gb = smem + (size_t)C::TW_LDS * 16 + (size_t)group * C::GROUP_BYTES;
    double2 *Cb = (double2 *)gb;
    double *red = (double *)(gb + C::CBYTES);
    const unsigned P = (unsigned)a.nsub * (unsigned)a.nchan;
    const unsigned stride = gridDim.x * gpb;
    const unsigned nchan = (unsigned)a.nchan;
    // profiles: all P, or the slots of a list, minus those with skip[k] != 0
    // (the two passes of the fit's forked diagnostics)
    const RoundList rl(a.list, a.nctr, (long)P);
    const unsigned nslot = (unsigned)rl.n();
    const uint8_t *skip = a.skip;
    // The group's upcoming slots, 64 at a time: lane j of each wave holds the
    // profile of slot wb0 + j stride (-1: past the end, or skipped), so the next
    // profile is a ballot bit away and the list and skip reads are one batch per
    // 64 profiles, where a dependent pair of reads per profile stalled the
    // prefetch of the next row (list and skip passes of the fork).
    unsigned wb0 = 0;
    int wkk = -1;
    unsigned long long wmask = 0;
    auto fill = [&](unsigned b) {
        wb0 = b;
        const unsigned sl = b + (unsigned)lane * stride;
        int kk = -1;
        if (sl < nslot && sl >= b) {
            kk = (int)rl.at(sl);
            if (skip && skip[kk]) kk = -1;
        }
        wkk = kk;
        wmask = __ballot(kk >= 0);
    };
    auto take = [&]() -> int {   // the next profile of the group (uniform), -1 when done
        while (wmask == 0) {
            const unsigned nb = wb0 + 64u * stride;
            if (nb >= nslot || nb < wb0) return -1;
            fill(nb);
        }
        const int j = __builtin_ctzll(wmask);
        wmask &= wmask - 1;
        return __builtin_amdgcn_readlane(wkk, j);
    };
    // a VGPR zero: the per-profile scalars of the next profile are read by
    // vector loads (counted on vmcnt), not scalar ones, whose lgkmcnt would be
    // waited on by the FFT's LDS waits
    int zv;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
    const int ca = t >> 3, cc = t & 7;
    const int jb = 128 * ca + cc;   // first sample of the thread's chain
    // byte offsets in the work array: d of chain sample q at wb[q & 3] + 64 (q & ~3)
    // (point p = jb/2 + 4q, part cc & 1); stage-1 point t + L r at rb[r & 3] + 16 L r
    int wb[4], rb[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        wb[m] = 16 * (64 * ca + ((4 * m + (cc >> 1)) ^ (4 * (ca & 3)))) + 8 * (cc & 1);
        rb[m] = 16 * (t ^ ((((t >> 6) + (L / 64) * m) & 3) << 2));
    }
    float pv[16];
    auto loadrow = [&](unsigned kk) {
        const float *pn = (stats ? a.D : a.raw) + (size_t)kk * N + jb;
#pragma unroll
        for (int q = 0; q < 16; ++q) pv[q] = pn[8 * q];
    };
    fill(__builtin_amdgcn_readfirstlane(blockIdx.x * gpb + group));
    int kq = take();
    unsigned k = kq >= 0 ? (unsigned)kq : 0u;
    double nx = 0.0;
    int nst = 0, nsh = 0;
    float nw = 0.0f, nb = 0.0f;
    auto prefetch = [&](unsigned kk) {
        loadrow(kk);
        const unsigned kv = kk + (unsigned)zv;
        if (!closed && !stats) {
            nx = a.amp[kv];
            nst = a.info[kv];
        }
        if (!stats) {
            nb = a.base[kv];
            nsh = a.shift[kk % nchan + (unsigned)zv];
        }
        nw = a.w0[kv];
    };
    if (kq >= 0) prefetch(k);
    for (; kq >= 0;) {
        // multi-wave groups: keep the FFT's LDS addresses inside the loop (hoisted,
        // they spill at N >= 2048; k_diag_p2); one wave: hoisted, 118 VGPRs
        if (WPP > 1) asm volatile("" : "+v"(t));
        double x = ufirst(nx);
        int st = ufirst(nst);
        const float w = ufirst(nw);
        const float bk = nb;
        const int sh = ufirst(nsh);
        // template at the dedispersed index of every chain sample
        double tg[16];
        if constexpr (!stats) {
            const double *tb = a.T2 + ((unsigned)(jb - sh) & (unsigned)(N - 1));
#pragma unroll
            for (int q = 0; q < 16; ++q) tg[q] = tb[8 * q];
        }
        if constexpr (closed) {
            // a = sum(T*p)/sum(T*T) over the chains of the stored (dispersed)
            // order: the lane's samples j = jb + 8q with p = f32(raw_j - base),
            // the dedispersed bin i = (j - sh) mod N, T_i = tg[q] (the
            // residual's gather): no second read of the row (round 6; before,
            // the dot ran over the dedispersed chains and gathered raw at
            // (i + sh) mod N again)
            double r = tg[0] * (double)(pv[0] - bk);
#pragma unroll
            for (int q = 1; q < 16; ++q) {
                const double pr = tg[q] * (double)(pv[q] - bk);
                r = r + pr;
            }
            double cs[1] = {r};
            const double dot = 0.0 + chain_total<N, double>(cs, red, wave, lane);
            const double TT = *a.TT;
            x = ufirst(TT != 0.0 ? dot / TT : 0.0);
            st = isfinite(x) ? 1 : 5;
            if (t == 0) {
                a.amp[k] = x;
                a.info[k] = st;
            }
        }
        // residual (ic.py:279-288) of the dispersed-frame sample j, f32 store
        // (:272), apply_weights (:296): X_j = f32(f32(x T_i - D_i) * w), D_i = f32(raw_j - base0)
        const bool ok = stats || (st >= 1 && st <= 4);
        const bool valid = w != 0.0f;
        float X[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if constexpr (stats) {
                X[q] = pv[q];
            } else {
                const float pj = pv[q] - bk;
                const double e = x * tg[q] - (double)pj;
                X[q] = (float)e;
            }
        }
        if (w != 1.0f) {   // fractional weights (w * 1 = w exactly: skipped)
#pragma unroll
            for (int q = 0; q < 16; ++q) X[q] = X[q] * w;
        }
        if (!ok) {   // a bad leastsq status zeroes the residual (ic.py:284-286)
            asm volatile("");   // a rare branch, not 16 selects on every profile
#pragma unroll
            for (int q = 0; q < 16; ++q) X[q] = 0.0f * w;
        }
        const unsigned kc = k;   // this profile (the prefetch below moves k on)
        kq = take();
        if (kq >= 0) {
            k = (unsigned)kq;
            prefetch(k);
        }
        double mean = 0.0, sd = 0.0, fftv = 0.0, ptp = (double)1e20f;
        if (valid) {
            // mean: f32 chain, then the pairwise tree (ic.py:207)
            float s = X[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) s = s + X[q];
            float fs[1] = {s};
            const float s32 = 0.0f + chain_total<N, float>(fs, (float *)(red + 16), wave, lane);
            mean = (double)s32 / (double)N;
            // the previous profile's spectrum reads are done before d overwrites the array
            gsync<WPP>();
            // var (ic.py:206): f64 pairwise sum of (f64(X) - mean)^2; d -> FFT input
            double r = 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const double d = (double)X[q] - mean;
                const double sq = d * d;
                r = q == 0 ? sq : r + sq;
                *(double *)(gb + wb[q & 3] + 64 * (q & ~3)) = d;
            }
            double rs[1] = {r};
            const double ss = 0.0 + chain_total<N, double>(rs, red + 24, wave, lane);
            sd = sqrt(ss / (double)N);
            // ptp (ic.py:208), NaN-propagating
            float mx = -INFINITY, mn = INFINITY;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                mx = OpMaxF()(mx, X[q]);
                mn = OpMinF()(mn, X[q]);
            }
            mx = group_tree<WPP, 64>(mx, OpMaxF(), (float *)(red + 32), wave, lane);
            mn = group_tree<WPP, 64>(mn, OpMinF(), (float *)(red + 36), wave, lane);
            int nan = 0;
            if (isnan(s32)) {
#pragma unroll
                for (int q = 0; q < 16; ++q) nan |= isnan(X[q]);
                nan = group_tree<WPP, 64>(nan, OpOr(), (int *)(red + 40), wave, lane);
            }
            ptp = nan ? (double)NAN : (double)(float)(mx - mn);
            // rFFT of d (ic.py:210-212): stage 1 (radix 8, no twiddles) from the
            // swizzled input image, then k_diag_p2's stages
            gsync<WPP>();
            double2 v[8];
#pragma unroll
            for (int r8 = 0; r8 < 8; ++r8) v[r8] = *(const double2 *)(gb + rb[r8 & 3] + 16 * L * r8);
            gsync<WPP>();
            dft_small<8>(v);
            {
                const int A = 8 * t + (t & 7);   // cidx(8t + r) = A ^ r
#pragma unroll
                for (int r8 = 0; r8 < 8; ++r8) Cb[A ^ r8] = v[r8];
            }
            gsync<WPP>();
            p2_fft<M, L, C::LG, 3, 8, M, float, twder>(Cb, (const float *)nullptr, 0.0, tw, t);
            // spectrum in conjugate bin pairs (k_diag_p2).  No NaN bookkeeping:
            // a finite f32 sum s32 means every X is finite, and then every d,
            // Z and |X_k|^2 is finite (|X_k|^2 < 1e85); a non-finite s32 (a NaN or
            // Inf sample, or an f32 overflow: d = -Inf) makes some bin NaN in
            // any FFT order, so numpy's max|rfft| is NaN (ic.py:210-212)
            constexpr int H = M / 2;
            constexpr int JF = H / L;
            double best2 = 0.0;
            auto post = [&](const double2 zk, const double2 zm, const double2 wv) {
                const double er = zk.x + zm.x, ei = zk.y - zm.y;
                const double orr = zk.y + zm.y, oi = zm.x - zk.x;
                const double tr = __builtin_fma(orr, wv.x, -(oi * wv.y));
                const double ti = __builtin_fma(orr, wv.y, oi * wv.x);
                const double re = er + tr, im = ei + ti;
                const double rm = er - tr, imm = ti - ei;
                const double a2 = __builtin_fma(re, re, im * im);
                const double b2 = __builtin_fma(rm, rm, imm * imm);
                best2 = fmax(best2, fmax(a2, b2));
            };
            static_assert(JF == 4 && 16 * L == N, "tw[t + L j] = tw[t] exp(-2 pi i j / 16)");
            const double2 wt = tw[t];
#pragma unroll
            for (int j = 0; j < JF; ++j) {
                const int kk = t + L * j;
                const double2 zk = Cb[cidx(t) + L * j];
                const double2 zm = Cb[kk == 0 ? 0 : cidx(L - t) + (M - L * (j + 1))];
                if (twder) {
                    // exp(-2 pi i j / 16), j = 0..3
                    constexpr double c16[4] = {1.0, 0.92387953251128675613, 0.70710678118654752440,
                                               0.38268343236508977173};
                    constexpr double s16[4] = {0.0, 0.38268343236508977173, 0.70710678118654752440,
                                               0.92387953251128675613};
                    const double2 wj = make_double2(c16[j], -s16[j]);
                    post(zk, zm, j == 0 ? wt : cmul_f(wt, wj));
                } else {
                    post(zk, zm, tw[kk]);
                }
            }
            {
                // the self-paired bin k = M/2 (one task): post(Z, Z, w) with the
                // exact zeros ei = oi = 0 of a finite Z folded in, on every lane
                const double2 z = Cb[cidx(H)], wv = tw[H];
                const double er = z.x + z.x, orr = z.y + z.y;
                const double tr = orr * wv.x, ti = orr * wv.y;
                const double re = er + tr, rm = er - tr, q2 = ti * ti;
                best2 = fmax(best2, fmax(__builtin_fma(re, re, q2), __builtin_fma(rm, rm, q2)));
            }
            best2 = group_tree<WPP, 64>(best2, OpMaxF(), red + 44, wave, lane);
            fftv = isfinite(s32) ? 0.5 * sqrt(best2) : (double)NAN;
        } else {
            // invalid: rfft of f64(X) = +-0 -> 0, unless R was non-finite (X NaN)
            int nanx = 0;
#pragma unroll
            for (int q = 0; q < 16; ++q) nanx |= isnan(X[q]);
            nanx = group_tree<WPP, 64>(nanx, OpOr(), (int *)(red + 52), wave, lane);
            fftv = nanx ? NAN : 0.0;
        }
        if (t == 0) {
            a.std_o[kc] = valid && isfinite(mean) ? sd : 0.0;   // numpy.ma: a non-finite mean is masked -> std 0
            a.mean_o[kc] = valid ? mean : 0.0;
            a.ptp_o[kc] = ptp;
            a.fft_o[kc] = fftv;
        }
    }
}

// residual cube on request (ic_get_residual): R (dispersed frame, unweighted).
// D == nullptr (fit_mode 1 keeps no fit cube): the fit-cube row is formed from
// raw and the w0 baseline as in k_chan_partials mode 3, f32(ded - base).
__global__ __launch_bounds__(256) void k_residual(const float *__restrict__ D, const float *__restrict__ raw,
                                                  const float *__restrict__ base, const double *__restrict__ T64,
                                                  const double *__restrict__ amp, const int32_t *__restrict__ info,
                                                  const int32_t *__restrict__ shift, size_t P, int nchan, int nbin,
                                                  int ldD, int dtiled, int pr_on, double pr_factor, int pr_start,
                                                  int pr_end, float *__restrict__ R)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (size_t k = (size_t)blockIdx.x * 4 + wave; k < P; k += (size_t)gridDim.x * 4) {
        const int sh = shift[k % nchan];
        const int st = info[k];
        const bool ok = st >= 1 && st <= 4;
        const double a = amp[k];
        const float b = D ? 0.0f : base[k];
        for (int i = lane; i < nbin; i += 64) {
            int j = i + sh;
            if (j >= nbin) j -= nbin;
            float v = 0.0f;
            if (ok) {
                const float p = D ? D[d_ofs(k, i, ldD, dtiled)] : raw[k * nbin + j] - b;
                const double u = a * T64[i];
                double e = u - (double)p;
                if (pr_on && i >= pr_start && i < pr_end) e = e * pr_factor;
                v = (float)e;
            }
            R[k * nbin + j] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// Fractional dedispersion: psrchive's FFT phase rotation in the stand-in's
// written order (phase_rotation.py; oracle orc_rotate), in IEEE f32 as
// psrchive's.  A profile per wave (N <= 1024: four to a block, sharing the
// twiddle tables staged in LDS) or per block (N >= 2048); grid-stride over
// channel-major items so that the profiles in flight share a channel's phasor
// row in L2; the N/2 complex points live in LDS between the passes.
//   1. z[j] = (f32(x[2j] - b), f32(x[2j+1] - b))
//   2. Z = FFT_{N/2}(z): Stockham stages of radix 8 (then 4 or 2), one LDS
//      round trip per stage
//   3. pairs (k, N/2 - k): real spectrum, x phasor, inverse half-spectrum
//      (conj) in one linear map (rot_pair)
//   4. r = FFT_{N/2}(that); out = r.re / M, -r.im / M
// A complex point is an f32 pair (rc2) and every complex operation one packed
// VOP3P instruction (v_pk_add_f32 / v_pk_mul_f32 with op_sel / neg modifiers
// for the swaps and the one-sided signs), each half an IEEE f32 operation of
// the definition: the same bits as the oracle's scalar f32 code
// (-ffp-contract=off), at half the f64 instruction count.
typedef float rc2 __attribute__((ext_vector_type(2)));

template <int N>
struct RotCfg {
    static constexpr int M = N / 2, H = M / 2;
    static constexpr int LG = N == 64 ? 5 : N == 128 ? 6 : N == 256 ? 7 : N == 512 ? 8 : N == 1024 ? 9
                                                                              : N == 2048 ? 10 : 11;   // log2 M
    static constexpr int TB = M / 8 < 64 ? 64 : (M / 8 > 256 ? 256 : M / 8);
    // one-wave profiles run four to a block, which stages the twiddle table in
    // LDS once for all four; the one-block profiles of N >= 2048 stage it too,
    // once per block of the grid-stride loop (16 profiles per block at C5:
    // 62.7-63.1 -> 58.0-58.2 ms per C5 clean in the FFT mode, against f64
    // entries through L1/L2 rounded at each use)
    static constexpr int WPB = TB == 64 ? 4 : 1;
    static constexpr bool TW_LDS = true;
};

// LDS slot of complex point i: one pad slot after every 8 points.  With 8-byte
// points ds_write_b64 banks 16 contiguous lanes on (slot mod 16) and ds_read_b64
// 32 lanes on (slot mod 32) (MI355X_MICROARCH.md): the stage stores (lane t ->
// points 8 t + q, and 64 (t / 8) + t % 8 + 8 q) are conflict-free, the
// contiguous reads (t + 64 q) 2-way on 3 of 32 banks.  A XOR swizzle cannot
// make the stores conflict-free without per-q address arithmetic on the reads
// (bits 6+ of the slot change with q).  All offsets are per-lane bases plus
// immediates: rsl(i + 8 c) = rsl(i) + 9 c.
__device__ __forceinline__ constexpr int rsl(int i) { return i + (i >> 3); }
template <int M> constexpr int rot_slots() { return M + M / 8; }

// packed complex arithmetic (each half one IEEE f32 operation)
__device__ __forceinline__ rc2 pk_nlo(rc2 a, rc2 b)   // (a.x - b.x, a.y + b.y)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 pk_nhi(rc2 a, rc2 b)   // (a.x + b.x, a.y - b.y)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 pk_mi(rc2 a, rc2 b)   // a + (-i) b = (a.x + b.y, a.y - b.x)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 pk_pi(rc2 a, rc2 b)   // a + i b = (a.x - b.y, a.y + b.x)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 pk_c7(rc2 c)   // (c.y - c.x, c.x + c.y)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1]" : "=v"(r) : "v"(c));
    return r;
}
__device__ __forceinline__ rc2 pk_cross(rc2 a, rc2 b)   // (a.y + b.y, a.x - b.x)
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 pk_addc(rc2 a, rc2 b)   // (a.x + b.x, (-a.y) + (-b.y))
{
    rc2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ rc2 rc2_of(double2 d) { return (rc2){(float)d.x, (float)d.y}; }

// 8-byte loads of the phasor table / 16-byte loads of the f64 twiddle table
// through a buffer descriptor: a 32-bit per-lane offset plus an immediate,
// instead of a 64-bit address register per table entry kept live across the
// profile loop
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rot_rsrc(const void *p, unsigned bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double2 rot_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ rc2 rot_ld2(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff)
{
    return __builtin_bit_cast(rc2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// Twiddle sources: k_diag_p2's table (p2_twiddles: M plain entries tw[i] =
// exp(-2 pi i i / N), then for every Stockham stage after the first, of radix
// R and span ns, the entries w^(q k), w = exp(-2 pi i / (R ns)), as [k][q - 1]
// at M + ns - 8: the spans are 8, 64, 512, so the earlier tables fill ns - 8
// slots), the same long-double values rounded to f64; the rotation uses them
// rounded to f32.  Staged in LDS as f32 (TwLds32; with the statistics, whose
// FFT needs the f64 table in LDS too, the f32 stage tables only: TwLdsSt), or
// read as f64 through L1/L2 and rounded at the use (TwGlobal, one-block
// profiles N >= 2048).
template <int N>
struct TwGlobal {
    static constexpr bool ASM_ROWS = false;
    __amdgpu_buffer_rsrc_t r;
    template <int NS, int R>
    __device__ __forceinline__ rc2 stage(unsigned k, int q) const
    {
        return rc2_of(rot_ld(r, 16u * (unsigned)(k * (R - 1)), 16u * (unsigned)(N / 2 + NS - 8 + q - 1)));
    }
    __device__ __forceinline__ rc2 post(unsigned i) const { return rc2_of(rot_ld(r, 16u * i, 0)); }
};
template <int N>
struct TwLds32 {
    static constexpr bool ASM_ROWS = true;   // rot_pass reads the stage rows with ds_read_b64
    const rc2 *t;
    template <int NS, int R>
    __device__ __forceinline__ rc2 stage(unsigned k, int q) const
    {
        return t[N / 2 + NS - 8 + q - 1 + k * (R - 1)];
    }
    // LDS byte address of entry [k][0] of the stage table of span NS
    template <int NS, int R>
    __device__ __forceinline__ uint32_t row(unsigned k) const
    {
        return lds_u32(t + (N / 2 + NS - 8 + k * (R - 1)));
    }
    __device__ __forceinline__ rc2 post(unsigned i) const { return t[i]; }
};
// with the statistics: the f32 stage tables alone (s: the entries from M on)
// beside the f64 table the statistics FFT reads, whose plain part serves the
// post step (rounded at the use); 53 KB of LDS per four-wave block, three
// blocks per CU
template <int N>
struct TwLdsSt {
    static constexpr bool ASM_ROWS = true;
    const rc2 *s;
    const double2 *t;
    template <int NS, int R>
    __device__ __forceinline__ rc2 stage(unsigned k, int q) const
    {
        return s[NS - 8 + q - 1 + k * (R - 1)];
    }
    template <int NS, int R>
    __device__ __forceinline__ uint32_t row(unsigned k) const
    {
        return lds_u32(s + (NS - 8 + k * (R - 1)));
    }
    __device__ __forceinline__ rc2 post(unsigned i) const { return rc2_of(t[i]); }
};

// the rotation's complex product (a.r w.r - a.i w.i, a.r w.i + a.i w.r):
// (a.r w.r, a.r w.i) and (a.i w.i, a.i w.r), then one add with the low half
// subtracted
__device__ __forceinline__ rc2 rot_cmul(rc2 a, rc2 w)
{
    return pk_nlo(a.xx * w, a.yy * w.yx);
}
// DFT of 4 / 8 points in place, natural output order, in the written order of
// phase_rotation.py (_dft4, _dft8) and the oracle (dft4, dft8): c3 = -i d is
// folded into y1 = c1 + c3 = pk_mi(c1, d) and y3 = c1 - c3 = pk_pi(c1, d)
// (x + (-y) is x - y bit for bit), and c6 = -i c6 into the odd DFT_4's first
// level the same way
__device__ __forceinline__ void rot_dft4(rc2 *b)
{
    const rc2 c0 = b[0] + b[2], c1 = b[0] - b[2], c2 = b[1] + b[3], d = b[1] - b[3];
    b[0] = c0 + c2;
    b[1] = pk_mi(c1, d);
    b[2] = c0 - c2;
    b[3] = pk_pi(c1, d);
}
__device__ __forceinline__ void rot_dft8(rc2 *b)
{
    constexpr float s = (float)0x1.6a09e667f3bcdp-1;   // f32(f64(sqrt(2)/2))
    rc2 c[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        c[q] = b[q] + b[q + 4];
        c[q + 4] = b[q] - b[q + 4];
    }
    c[5] = pk_mi(c[5], c[5]) * (rc2){s, s};    // ((c.r + c.i) s, (c.i - c.r) s)
    c[7] = pk_c7(c[7]) * (rc2){s, -s};         // ((c.i - c.r) s, -((c.r + c.i) s))
    rot_dft4(c);
    // odd DFT_4 of (c4, c5, -i c6, c7)
    const rc2 e0 = pk_mi(c[4], c[6]), e1 = pk_pi(c[4], c[6]), e2 = c[5] + c[7], d = c[5] - c[7];
    b[0] = c[0];
    b[2] = c[1];
    b[4] = c[2];
    b[6] = c[3];
    b[1] = e0 + e2;
    b[3] = pk_mi(e1, d);
    b[5] = e0 - e2;
    b[7] = pk_pi(e1, d);
}

// One Stockham stage of radix Q = 2^R and span ns = 2^LGS (phase_rotation.py
// _stockham): group ja < G = M/Q holds the points v[ja + q G]; from the second
// stage on they are multiplied by the stage's twiddles w^(q k), k = ja mod ns,
// then transformed by DFT_Q, and y_p lands at v[(ja - k) Q + k + p ns].  One LDS
// round trip per stage (8 points per lane at N = 1024, three stages per FFT).
// IN_REG: the pass's input is z (one group per thread, G == TB) instead of
// LDS; OUT_REG: its output stays in z.  The last pass's group ja holds points
// ja + q G, the distribution the first pass reads, so a profile can enter and
// leave the FFT in registers (k_rotate's direct layout).
template <int N, int R, int LGS, bool IN_REG = false, bool OUT_REG = false, typename TW>
__device__ __forceinline__ void rot_pass(rc2 *v, const TW &tw, int t, rc2 *z = nullptr)
{
    using C = RotCfg<N>;
    constexpr int M = C::M, TB = C::TB, G = M >> R, Q = 1 << R;
    constexpr int GPT = (G + TB - 1) / TB;
    constexpr int ns = 1 << LGS;
    static_assert(!(IN_REG || OUT_REG) || G == TB, "register passes hold one group per thread");
    static_assert(ns == 1 || ns >= 8, "stage spans are 1, 8, 64, 512");
    rc2 u[GPT][Q];
    // the stage's twiddles first (their latency overlaps the LDS reads and the barrier)
    rc2 w[GPT][Q - 1];
    // one-group-per-lane passes read their points (and the f32 twiddle rows)
    // as separate ds_read_b64 in asm: the compiler pairs adjacent 8-byte LDS
    // loads into ds_read2_b64, which serves 16-lane groups on 32 banks at 4x
    // the LDS cycles per byte (MI355X_MICROARCH.md); one lgkmcnt wait ties
    // the values
    constexpr bool ASM = GPT == 1 && G == TB && G % 8 == 0 && !IN_REG;
    if constexpr (ASM) {
        const int ja = t, k = ja & (ns - 1);
        if constexpr (ns > 1 && TW::ASM_ROWS) {
            const uint32_t wa = tw.template row<ns, Q>((unsigned)k);
#pragma unroll
            for (int q = 1; q < Q; ++q)
                asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(w[0][q - 1]) : "v"(wa), "i"(8 * (q - 1)));
        } else if constexpr (ns > 1) {
#pragma unroll
            for (int q = 1; q < Q; ++q) w[0][q - 1] = tw.template stage<ns, Q>((unsigned)k, q);
        }
        const uint32_t va = lds_u32(v + rsl(ja));   // rsl(ja + q G) = rsl(ja) + q (G + G/8)
#pragma unroll
        for (int q = 0; q < Q; ++q)
            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(u[0][q]) : "v"(va), "i"(8 * q * (G + G / 8)));
        if constexpr (Q == 8) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(u[0][0]), "+v"(u[0][1]), "+v"(u[0][2]), "+v"(u[0][3]), "+v"(u[0][4]), "+v"(u[0][5]),
                           "+v"(u[0][6]), "+v"(u[0][7]));
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < Q; ++q) asm volatile("" : "+v"(u[0][q]));
        }
        if constexpr (ns > 1 && TW::ASM_ROWS) {
#pragma unroll
            for (int q = 0; q < Q - 1; ++q) asm volatile("" : "+v"(w[0][q]));
        }
    }
#pragma unroll
    for (int gi = 0; gi < GPT && !ASM; ++gi) {
        const int ja = t + TB * gi;
        const int k = ja & (ns - 1);
        if (G % TB == 0 || ja < G) {
            if constexpr (ns > 1) {
#pragma unroll
                for (int q = 1; q < Q; ++q) w[gi][q - 1] = tw.template stage<ns, Q>((unsigned)k, q);
            }
            if constexpr (IN_REG) {
#pragma unroll
                for (int q = 0; q < Q; ++q) u[gi][q] = z[q];
            } else if constexpr (G % 8 == 0) {
                const rc2 *vj = v + rsl(ja);    // rsl(ja + q G) = rsl(ja) + q (G + G/8)
#pragma unroll
                for (int q = 0; q < Q; ++q) u[gi][q] = vj[q * (G + G / 8)];
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) u[gi][q] = v[rsl(ja + q * G)];
            }
        }
    }
    gsync<C::TB / 64>();
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
        const int ja = t + TB * gi;
        if (G % TB == 0 || ja < G) {
            const int k = ja & (ns - 1);
            if constexpr (ns > 1) {
#pragma unroll
                for (int q = 1; q < Q; ++q) u[gi][q] = rot_cmul(u[gi][q], w[gi][q - 1]);
            }
            if constexpr (Q == 8) {
                rot_dft8(u[gi]);
            } else if constexpr (Q == 4) {
                rot_dft4(u[gi]);
            } else {
                const rc2 a = u[gi][0], b = u[gi][1];
                u[gi][0] = a + b;
                u[gi][1] = a - b;
            }
            const int base = ((ja >> LGS) << (LGS + R)) + k;
            if constexpr (OUT_REG) {
                static_assert(ns * Q == M, "only the last pass keeps its output");
#pragma unroll
                for (int q = 0; q < Q; ++q) z[q] = u[gi][q];
            } else if constexpr (ns % 8 == 0) {
                rc2 *vb = v + rsl(base);   // rsl(base + q ns) = rsl(base) + q (ns + ns/8)
#pragma unroll
                for (int q = 0; q < Q; ++q) vb[q * (ns + ns / 8)] = u[gi][q];
            } else {
                // ns = 1: base = Q ja, a multiple of 8 for Q = 8 (rsl(base + q) = rsl(base) + q)
                rc2 *vb = v + rsl(base);
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    if constexpr (Q == 8) vb[q] = u[gi][q];
                    else v[rsl(base + q)] = u[gi][q];
                }
            }
        }
    }
    gsync<C::TB / 64>();
}

// the full N/2-point FFT: passes of 3 stages (the last one shorter); IN_REG /
// OUT_REG: the first pass reads z / the last pass leaves its output in z
template <int N, int LG0 = 0, bool IN_REG = false, bool OUT_REG = false, typename TW>
__device__ __forceinline__ void rot_fft(rc2 *v, const TW &tw, int t, rc2 *z = nullptr)
{
    constexpr int LG = RotCfg<N>::LG;
    if constexpr (LG0 < LG) {
        constexpr int R = LG - LG0 >= 3 ? 3 : LG - LG0;
        constexpr bool LAST = LG0 + R >= LG;
        rot_pass<N, R, LG0, IN_REG && LG0 == 0, OUT_REG && LAST>(v, tw, t, z);
        rot_fft<N, LG0 + R, false, OUT_REG>(v, tw, t, z);
    }
}

// The inverse's half-length inputs Z'_k, Z'_q (q = M - k) from the transform's
// Z_k, Z_q in one linear map (phase_rotation.py _pair, oracle rot_pair): the
// real spectrum X_k = E_k + w O_k, the phasors and the inverse's packing
// composed, Z'_k = A_k Z_k + B_k conj(Z_q), Z'_q = A_q Z_q - conj(B_k) conj(Z_k),
// with w = exp(-2 pi i k / N) = (c, sn) and the signed phasors pk, pq.  Returns
// conj(Z'_k), conj(Z'_q) (what the inverse stores; the imaginary part as (-a) +
// (-b) of the two terms', the definition's order).  Packed: (h1, h2) = ((1 +
// sn), (1 - sn)) * 0.5; A_k = (h1 pk.r + h2 pq.r, h1 pk.i - h2 pq.i), A_q
// likewise; B_k = (pk.i + pq.i, pk.r - pq.r) * (-c/2, c/2) (-(x y) = (-x) y);
// A Z is rot_cmul; B_k conj(Z_q) = (b.r zq.r + b.i zq.i, b.i zq.r - b.r zq.i);
// -conj(B_k) conj(Z_k) = (b.i zk.i - b.r zk.r, b.i zk.r + b.r zk.i).
__device__ __forceinline__ void rot_pair(rc2 zk, rc2 zq, rc2 w, rc2 pk, rc2 pq, rc2 &ok, rc2 &oq)
{
    rc2 hh;
    const rc2 one = {1.0f, 1.0f};
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(hh) : "v"(one), "v"(w));
    hh = hh * (rc2){0.5f, 0.5f};
    const rc2 hcv = w.xx * (rc2){-0.5f, 0.5f};
    const rc2 ak = pk_nhi(hh.xx * pk, hh.yy * pq);
    const rc2 aq = pk_nhi(hh.xx * pq, hh.yy * pk);
    const rc2 b = pk_cross(pk, pq) * hcv;
    ok = pk_addc(rot_cmul(ak, zk), pk_nhi(b * zq.xx, b.yx * zq.yy));
    oq = pk_addc(rot_cmul(aq, zq), pk_nlo(b.yy * zk.yx, b.xx * zk));
}

// comprehensive_stats (ic.py:206-212) of the rotated residual row held by one
// wave in the direct layout: z[q] = point j = t + TB q, i.e. R[2j] = f32(z.re /
// M), R[2j + 1] = f32(-z.im / M) (k_rotate's store), X = f32(R w) (apply_weights,
// ic.py:111-117, 296).  Every value is k_diag_cl<N, DIAG_STATS>'s, bit for bit:
// - mean / var / ptp: X goes through the wave's LDS slots once (the padded
//   xaddr image) and each lane reads its pairwise chain (leaf t/8, accumulator
//   t%8: samples 128(t/8) + t%8 + 8q); the trees are chain_total's;
// - fftmax: k_diag_cl's first radix-8 stage reads the points t + 64 r of d =
//   f64(X) - mean, which is exactly the direct layout this lane holds, so the
//   rFFT starts from registers; the later stages are p2_fft's with its f64
//   table (tw_p2, which k_rotate stages in LDS: tw64), the spectrum's post
//   twiddles tw[k < M] from the same table's plain part.  v: the wave's LDS
//   work array (M f64 complex points).
template <int N>
__device__ __forceinline__ void rot_stats(const RotateArgs &a, size_t p, double2 *v, const double2 *tw64, int t,
                                          rc2 (&z)[8], float inv, float w)
{
    constexpr int M = RotCfg<N>::M, H = M / 2, TB = RotCfg<N>::TB, L = TB;
    static_assert(N == 1024 && TB == 64 && CLay<N>::L == 64, "one wave per profile, 16 samples per lane");
    static_assert(RotCfg<N>::TW_LDS, "the statistics FFT reads k_diag's table from the rotation's LDS copy (tw64)");
    float xr[16];   // sample 2(t + 64 q) + e at xr[2q + e]
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        xr[2 * q] = z[q].x * inv;
        xr[2 * q + 1] = (-z[q].y) * inv;
    }
    if (w != 1.0f) {   // fractional weights (w * 1 = w exactly: skipped)
#pragma unroll
        for (int e = 0; e < 16; ++e) xr[e] = xr[e] * w;
    }
    const bool valid = w != 0.0f;
    double mean = 0.0, sd = 0.0, fftv = 0.0, ptp = (double)1e20f;
    if (valid) {
        // the row into LDS (the last pass's reads of v are done: rot_pass ends
        // with gsync), float pairs at xaddr(2j) = 2t + 136 q
        float *xs = (float *)v;
#pragma unroll
        for (int q = 0; q < 8; ++q) *(float2 *)(xs + 2 * t + 136 * q) = make_float2(xr[2 * q], xr[2 * q + 1]);
        wave_sync();
        float X[16];
        {
            const float *xc = xs + 136 * (t >> 3) + (t & 7);
#pragma unroll
            for (int q = 0; q < 16; ++q) X[q] = xc[8 * q];
        }
        float s = X[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) s = s + X[q];
        float fs[1] = {s};
        const float s32 = 0.0f + chain_total<N, float>(fs, (float *)nullptr, 0, t);
        mean = (double)s32 / (double)N;
        double r = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const double d = (double)X[q] - mean;
            const double sq = d * d;
            r = q == 0 ? sq : r + sq;
        }
        double rs[1] = {r};
        const double ss = 0.0 + chain_total<N, double>(rs, (double *)nullptr, 0, t);
        sd = sqrt(ss / (double)N);
        float mx = -INFINITY, mn = INFINITY;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            mx = OpMaxF()(mx, X[q]);
            mn = OpMinF()(mn, X[q]);
        }
        mx = group_tree<1, 64>(mx, OpMaxF(), (float *)nullptr, 0, t);
        mn = group_tree<1, 64>(mn, OpMinF(), (float *)nullptr, 0, t);
        int nan = 0;
        if (isnan(s32)) {
#pragma unroll
            for (int q = 0; q < 16; ++q) nan |= isnan(X[q]);
            nan = group_tree<1, 64>(nan, OpOr(), (int *)nullptr, 0, t);
        }
        ptp = nan ? (double)NAN : (double)(float)(mx - mn);
        // rfft of d (ic.py:210-212): stage 1 (radix 8, no twiddles) on the
        // lane's points t + 64 r, then k_diag_p2's stages in the complex work
        // array Cb = v (cidx slots, M entries: inside the rotation's padded
        // array).  The chain reads above precede the stores (one wave: its LDS
        // operations stay in order)
        double2 c8[8];
#pragma unroll
        for (int r8 = 0; r8 < 8; ++r8) c8[r8] = make_double2((double)xr[2 * r8] - mean, (double)xr[2 * r8 + 1] - mean);
        dft_small<8>(c8);
        double2 *Cb = v;
        {
            const int A = 8 * t + (t & 7);   // cidx(8t + r) = A ^ r
#pragma unroll
            for (int r8 = 0; r8 < 8; ++r8) Cb[A ^ r8] = c8[r8];
        }
        wave_sync();
        p2_fft<M, L, CLay<N>::LG, 3, 8, M, float, false>(Cb, (const float *)nullptr, 0.0, tw64, t);
        // the spectrum in conjugate bin pairs (k_diag_cl's post, 2 X_k)
        constexpr int JF = H / L;
        double best2 = 0.0;
        auto post = [&](const double2 zk, const double2 zm, const double2 wv) {
            const double er = zk.x + zm.x, ei = zk.y - zm.y;
            const double orr = zk.y + zm.y, oi = zm.x - zk.x;
            const double tr = __builtin_fma(orr, wv.x, -(oi * wv.y));
            const double ti = __builtin_fma(orr, wv.y, oi * wv.x);
            const double re = er + tr, im = ei + ti;
            const double rm = er - tr, imm = ti - ei;
            const double a2 = __builtin_fma(re, re, im * im);
            const double b2 = __builtin_fma(rm, rm, imm * imm);
            best2 = fmax(best2, fmax(a2, b2));
        };
#pragma unroll
        for (int j = 0; j < JF; ++j) {
            const int kk = t + L * j;
            const double2 zk = Cb[cidx(t) + L * j];
            const double2 zm = Cb[kk == 0 ? 0 : cidx(L - t) + (M - L * (j + 1))];
            post(zk, zm, tw64[kk]);
        }
        {
            // the self-paired bin k = M/2 (k_diag_cl)
            const double2 zc = Cb[cidx(H)], wv = tw64[H];
            const double er = zc.x + zc.x, orr = zc.y + zc.y;
            const double tr = orr * wv.x, ti = orr * wv.y;
            const double re = er + tr, rm = er - tr, q2 = ti * ti;
            best2 = fmax(best2, fmax(__builtin_fma(re, re, q2), __builtin_fma(rm, rm, q2)));
        }
        best2 = group_tree<1, 64>(best2, OpMaxF(), (double *)nullptr, 0, t);
        // a non-finite f32 sum means a NaN / Inf sample: some bin is NaN (k_diag_cl)
        fftv = isfinite(s32) ? 0.5 * sqrt(best2) : (double)NAN;
    } else {
        // w = 0: rfft of f64(X) = +-0 -> 0, unless R was non-finite (X NaN)
        int nanx = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) nanx |= isnan(xr[e]);
        nanx = group_tree<1, 64>(nanx, OpOr(), (int *)nullptr, 0, t);
        fftv = nanx ? NAN : 0.0;
    }
    if (t == 0) {
        a.std_o[p] = valid && isfinite(mean) ? sd : 0.0;   // numpy.ma: a non-finite mean is masked -> std 0
        a.mean_o[p] = valid ? mean : 0.0;
        a.ptp_o[p] = ptp;
        a.fft_o[p] = fftv;
    }
}

// PP: per-profile delays (a.delay2, ic_set_delays2): each lane evaluates its
// phasors with ic_phasor instead of loading the channel's table row.
// ST: the residual's rotation measures its rows instead of storing them
// (RotateArgs.std_o; the direct layout only): the rotated row R, still in the
// lane's registers, becomes X = f32(R w0), whose mean / var / ptp run on the
// numpy pairwise chains (one LDS transposition into k_diag_cl's chain layout,
// the same trees: the same bits) and whose real spectrum comes from a third
// pass of the rotation's own FFT (max |rfft|, within 1e-9 of numpy like every
// diagnostics kernel's).  R never goes to HBM: the residual's 4N write and the
// statistics pass's 4N read are gone, and so is the R buffer.
template <int N, bool PP, bool ST = false>
// 3 waves per SIMD (137-167 VGPRs at N = 1024; 4 waves spill 2-13 VGPRs without
// the statistics: C2 fft 40.7 either way, fft_pp 40.9 -> 41.3 ms)
__global__ __launch_bounds__(RotCfg<N>::TB * RotCfg<N>::WPB, N <= 1024 ? 3 : 2) void k_rotate(RotateArgs a)
{
    using C = RotCfg<N>;
    constexpr int M = C::M, H = C::H, TB = C::TB, WPB = C::WPB;
    constexpr int NJ = (M / 2 + TB - 1) / TB;    // float4 rows per lane (4 samples = 2 points)
    constexpr int NK = H / TB + 1;               // spectrum pairs (k, M - k) per lane, k <= H
    // direct layout (every pass radix 8, one group per lane: N = 1024): lane t
    // loads points t + TB q (q < 8) straight into the first pass's registers and
    // stores the last pass's registers, which are the same points; two LDS round
    // trips per profile fewer
    constexpr bool DIRECT = C::LG % 3 == 0 && (M >> 3) == TB;
    // the wave's points (rot_slots f32 pairs); with the statistics the same
    // array holds their f64 FFT's M complex points
    constexpr int VS = ST ? 2 * M : rot_slots<M>();
    static_assert(rot_slots<M>() <= VS, "the rotation's slots fit");
    __shared__ __attribute__((aligned(16))) rc2 vv[WPB][VS];
    constexpr int TWE = p2_tw_entries(N);   // k_diag_p2's table: M plain + the stage tables
    // the twiddle table: f32 for the rotation, or f64 when the statistics FFT
    // needs it (the rotation then rounds each entry at its use)
    __shared__ rc2 tws32[C::TW_LDS ? (ST ? TWE - M : TWE) : 1];
    __shared__ double2 tws64[C::TW_LDS && ST ? TWE : 1];
    const int t = threadIdx.x % TB, wv = threadIdx.x / TB;
    rc2 *v = vv[wv];
    const unsigned nsub = (unsigned)a.nsub, nchan = (unsigned)a.nchan;
    const size_t P = (size_t)nsub * nchan;
    const float sg = a.sign > 0 ? 1.0f : -1.0f;
    const float inv = (float)(1.0 / (double)M);
    const __amdgpu_buffer_rsrc_t twr = rot_rsrc(a.tw_p2, 16u * TWE);
    const auto tw = [&]() {
        if constexpr (!C::TW_LDS) return TwGlobal<N>{twr};
        else if constexpr (ST) return TwLdsSt<N>{tws32, tws64};
        else return TwLds32<N>{tws32};
    }();
    if constexpr (C::TW_LDS) {
        for (int i = threadIdx.x; i < TWE; i += TB * WPB) {
            if constexpr (ST) {
                tws64[i] = a.tw_p2[i];
                if (i >= M) tws32[i - M] = rc2_of(a.tw_p2[i]);
            } else {
                tws32[i] = rc2_of(a.tw_p2[i]);
            }
        }
        __syncthreads();
    }
    // every global load of a profile in flight at once: one memory latency
    // per profile, not one per row (or per flag / fit lookup)
    auto load_rows = [&](size_t k, float4 (&xr)[NJ]) {
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
            const int j2 = t + u * TB;
            if ((M / 2) % TB == 0 || j2 < M / 2)
            {
                // non-temporal, as the direct layout's (C5 fft 58.8 -> 57.4-57.9 ms,
                // C4 fft 3.90 -> 3.76 ms with the stores below)
                const fv4 xv = __builtin_nontemporal_load((const fv4 *)(a.in + d_ofs(k, 4 * j2, (int)a.ld_in, a.in_tiled)));
                xr[u] = make_float4(xv.x, xv.y, xv.z, xv.w);
            }
        }
    };
    // the profile is left out (uniform over the block): its subint's flag is 0,
    // or its late flag is not the one selected
    auto skip = [&](size_t p, unsigned s) {
        return (a.flags && a.flags[s] == 0) || (a.late && ((a.late[p] != 0) != (a.late_sel != 0)));
    };
    // a block's profiles are consecutive items (channel-major): they share a
    // channel's phasor row
    // items: channel-major over every profile, or the profiles of a round list
    // (RotateArgs.list: the diagnostics fork's second pass, the profiles still
    // fitting at its round - a scan of every profile for their late flags cost
    // that pass 2.7-3.4 ms per iteration on C2 for a tenth of the profiles)
    const RoundList rl(a.list, a.nctr, (long)P);
    const size_t nitems = a.list ? (size_t)rl.n() : P;
    for (size_t item = (size_t)blockIdx.x * WPB + wv; item < nitems; item += (size_t)gridDim.x * WPB) {
        unsigned c, s;
        size_t p;
        if (a.list) {
            p = (size_t)rl.at((long)item);
            c = (unsigned)(p % nchan);
            s = (unsigned)(p / nchan);
        } else {
            c = (unsigned)(item / nsub);
            s = (unsigned)(item % nsub);
            p = (size_t)s * nchan + c;
        }
        if (skip(p, s)) continue;
        // the channel's f32 phasor row (8 bytes per harmonic)
        const __amdgpu_buffer_rsrc_t phr = rot_rsrc(PP ? (const void *)a.tw : (const void *)(a.ph + 2 * (size_t)c * (M + 1)),
                                                    8u * (M + 1));
        const double dly = PP ? a.delay2[p] : 0.0;
        // PP, N >= 256 (M a multiple of 64): the lane's harmonics k = t + u TB
        // and M - k have the low parts lo1 = t mod 64 and lo2 = -t mod 64 in
        // every round, and high parts that are the same across the wave: w0 + u
        // TB for k, and M - 64 - w0 - u TB for M - k (M - w0 - u TB where lo1 =
        // 0), w0 = t - lo1.  So a lane evaluates P0(lo1), P0(lo2) and one of
        // the wave's 3 NK high parts (lane j), and every round reads its high
        // parts from lanes u, NK + u, 2 NK + u (ic_phasor's product form: 3
        // polynomials per lane instead of 2 NK)
        constexpr bool PPX = PP && N >= 256;
        const int lo1 = t & 63, w0 = t - lo1;
        double2 A1{}, A2{}, Bh{};
        if constexpr (PPX) {
            const int lo2 = (64 - lo1) & 63, j = lo1;
            int hv = j < NK ? w0 + j * TB : (j < 2 * NK ? M - 64 - w0 - (j - NK) * TB : M - w0 - (j - 2 * NK) * TB);
            if (j >= 3 * NK || hv < 0) hv = 0;
            A1 = ic_phasor0(lo1, dly, N);
            A2 = ic_phasor0(lo2, dly, N);
            Bh = ic_phasor0(hv, dly, N);
        }
        auto bcast = [&](int lane) {
            return make_double2(__hiloint2double(__builtin_amdgcn_readlane(__double2hiint(Bh.x), lane),
                                                 __builtin_amdgcn_readlane(__double2loint(Bh.x), lane)),
                                __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(Bh.y), lane),
                                                 __builtin_amdgcn_readlane(__double2loint(Bh.y), lane)));
        };
        // the post step's phasors one round ahead: the first round's are
        // requested with the rows, each later round's before the round before it
        // RM (N >= 256): the last round would hold k = H alone, in lane 0.  Lane
        // 0 takes it in round 0 instead of the DC / Nyquist bins, which it
        // finishes after the rounds: no round with one active lane and no
        // divergent branch in round 0 (the schedule only: the same operations).
        // Per-channel C2 46.8 -> 46.4 ms (f64 rotation); with per-profile
        // delays it spilled in f64 (48.1 -> 48.6), in f32 it gains (39.8 -> 39.6)
        constexpr bool RM = H % TB == 0;
        constexpr int NR = RM ? NK - 1 : NK;
        auto kof = [&](int u) { return (RM && u == 0 && t == 0) ? H : t + u * TB; };
        // the phasors (f64, ic_phasor) rounded to f32 at the use; the table's are f32
        auto ldph = [&](int u, rc2 (&pp)[2]) {
            const int k = kof(u);
            if constexpr (PPX) {
                const double2 b1 = bcast(u), b2 = bcast(NK + u), b3 = bcast(2 * NK + u);
                if (k <= H) {
                    pp[0] = rc2_of(lo1 == 0 ? b1 : (w0 + u * TB == 0 ? A1 : ic_phasor_mul(A1, b1)));
                    pp[1] = rc2_of(lo1 == 0 ? b3 : (M - 64 - w0 - u * TB == 0 ? A2 : ic_phasor_mul(A2, b2)));
                }
                if (RM && u == 0) {   // lane 0's k = H: P0(H) from the round NK - 1 parts
                    const double2 bh = bcast(NK - 1), bh3 = bcast(3 * NK - 1);
                    if (t == 0) {
                        pp[0] = rc2_of(bh);
                        pp[1] = rc2_of(bh3);
                    }
                }
            } else if (k <= H) {
                if constexpr (PP) {
                    pp[0] = rc2_of(ic_phasor(k, dly, N));
                    pp[1] = rc2_of(ic_phasor(M - k, dly, N));
                } else {
                    pp[0] = rot_ld2(phr, 8u * (unsigned)k, 0);
                    pp[1] = rot_ld2(phr, 8u * (unsigned)(M - k), 0);
                }
            }
        };
        rc2 phn[2];
        ldph(0, phn);
        rc2 z[8];
        static_assert(!ST || DIRECT, "the statistics epilogue needs the direct layout");
        float wst = 1.0f;   // ST: the profile's weight, requested with the rows
        if constexpr (ST) wst = a.w0[p];
        if constexpr (DIRECT) {
            const size_t k = p;
            float2 x2[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
            {
                // read once per rotation (non-temporal: C2 fft 39.25-39.42 -> 39.05-39.25 ms)
                const rc2 xv =
                    __builtin_nontemporal_load((const rc2 *)(a.in + d_ofs(k, 2 * (t + TB * q), (int)a.ld_in, a.in_tiled)));
                x2[q] = make_float2(xv.x, xv.y);
            }
            if (a.amp) {
                const __amdgpu_buffer_rsrc_t t64r = rot_rsrc(a.T64, 16u * M);
                double2 tt[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) tt[q] = rot_ld(t64r, 16u * (unsigned)t, 16u * (unsigned)(TB * q));
                const int st = a.info[p];
                const bool ok = st >= 1 && st <= 4;
                const double am = a.amp[p];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    float r[2] = {0.0f, 0.0f};
                    if (ok) {
                        const float pv[2] = {x2[q].x, x2[q].y};
                        const double tv[2] = {tt[q].x, tt[q].y};
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const int i = 2 * (t + TB * q) + e;
                            const double uu = am * tv[e];
                            double d = uu - (double)pv[e];
                            if (a.pr_on && i >= a.pr_start && i < a.pr_end) d = d * a.pr_factor;
                            r[e] = (float)d;
                        }
                    }
                    z[q] = (rc2){r[0], r[1]};
                }
            } else {
                const float b = a.base ? a.base[p] : 0.0f;
#pragma unroll
                for (int q = 0; q < 8; ++q) z[q] = (rc2){x2[q].x, x2[q].y} - (rc2){b, b};
            }
            rot_fft<N, 0, true, false>(v, tw, t, z);
        } else {
        float4 xin[NJ];
        load_rows(p, xin);
        if (a.amp) {
            // the residual of the exact fit (k_residual's arithmetic), formed on the fly;
            // the template is requested with the rows, before the status is known
            // (behind the scattered amp / info loads it was a second latency)
            const __amdgpu_buffer_rsrc_t t64r = rot_rsrc(a.T64, 16u * M);
            double2 tt[NJ][2];
#pragma unroll
            for (int u = 0; u < NJ; ++u) {
                const int j2 = t + u * TB;
                if ((M / 2) % TB != 0 && j2 >= M / 2) break;
                tt[u][0] = rot_ld(t64r, 32u * (unsigned)t, 32u * (unsigned)(u * TB));
                tt[u][1] = rot_ld(t64r, 32u * (unsigned)t, 32u * (unsigned)(u * TB) + 16u);
            }
            const int st = a.info[p];
            const bool ok = st >= 1 && st <= 4;
            const double am = a.amp[p];
#pragma unroll
            for (int u = 0; u < NJ; ++u) {
                const int j2 = t + u * TB;
                if ((M / 2) % TB != 0 && j2 >= M / 2) break;
                float r[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                if (ok) {
                    const float pv[4] = {xin[u].x, xin[u].y, xin[u].z, xin[u].w};
                    const double tv[4] = {tt[u][0].x, tt[u][0].y, tt[u][1].x, tt[u][1].y};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int i = 4 * j2 + e;
                        const double uu = am * tv[e];
                        double d = uu - (double)pv[e];
                        if (a.pr_on && i >= a.pr_start && i < a.pr_end) d = d * a.pr_factor;
                        r[e] = (float)d;
                    }
                }
                v[rsl(2 * j2)] = (rc2){r[0], r[1]};
                v[rsl(2 * j2 + 1)] = (rc2){r[2], r[3]};
            }
        } else {
            const float b = a.base ? a.base[p] : 0.0f;
#pragma unroll
            for (int u = 0; u < NJ; ++u) {
                const int j2 = t + u * TB;
                if ((M / 2) % TB != 0 && j2 >= M / 2) break;
                v[rsl(2 * j2)] = (rc2){xin[u].x, xin[u].y} - (rc2){b, b};
                v[rsl(2 * j2 + 1)] = (rc2){xin[u].z, xin[u].w} - (rc2){b, b};
            }
        }
        gsync<TB / 64>();
        rot_fft<N>(v, tw, t);
        }
        // the post step's twiddles, at their use
        // Re P(M) for the DC / Nyquist step after the rounds (RM); P(0) = (1, 0)
        // exactly for every delay, so Y_0 = X_0 * 1 = X_0
        float pmr = 0.0f;
        if constexpr (RM) {
            if constexpr (PPX) pmr = (float)bcast(2 * NK).x;   // P0(M), lane 2 NK of the wave's high parts
            else pmr = rot_ld2(phr, 8u * (unsigned)M, 0).x;
        }
        const rc2 sgv = {1.0f, sg};
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            const int k = kof(u);
            const rc2 wk = k <= H ? tw.post((unsigned)(k & (M - 1))) : (rc2){0.0f, 0.0f};
            const rc2 pk = phn[0], pq = phn[1];
            if (u + 1 < NR) ldph(u + 1, phn);
            if (k <= H) {
                if (!RM && k == 0) {
                    const rc2 z0 = v[rsl(0)];
                    const float X0 = z0.x + z0.y, XM = z0.x - z0.y;
                    const float Y0 = X0 * pk.x, YM = XM * pq.x;
                    v[rsl(0)] = (rc2){(Y0 + YM) * 0.5f, -((Y0 - YM) * 0.5f)};
                } else {
                    const int q = M - k;
                    const rc2 zk = v[rsl(k)], zq = v[rsl(q)];
                    rc2 Zk, Zq;   // conjugated
                    rot_pair(zk, zq, wk, pk * sgv, pq * sgv, Zk, Zq);
                    v[rsl(q)] = Zq;
                    v[rsl(k)] = Zk;
                }
            }
        }
        if constexpr (RM) {
            if (t == 0) {   // DC and Nyquist: X_0 = Z_0.r + Z_0.i, X_M = Z_0.r - Z_0.i
                const rc2 z0 = v[rsl(0)];
                const float X0 = z0.x + z0.y, XM = z0.x - z0.y;
                const float Y0 = X0, YM = XM * pmr;
                v[rsl(0)] = (rc2){(Y0 + YM) * 0.5f, -((Y0 - YM) * 0.5f)};
            }
        }
        gsync<TB / 64>();
        float *o = a.out + p * (size_t)a.ldo;
        const rc2 scl = {inv, -inv};   // (r.re / M, -r.im / M): x (-1/M) = -(x) (1/M)
        if constexpr (ST) {
            rot_fft<N, 0, false, true>(v, tw, t, z);
            rot_stats<N>(a, p, (double2 *)v, tws64, t, z, inv, wst);
        } else if constexpr (DIRECT) {
            rot_fft<N, 0, false, true>(v, tw, t, z);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int j = t + TB * q;
                // written once, read by later kernels: non-temporal stores
                // (C2 fft 39.71-39.95 -> 39.43-39.53 ms; only out2's: 39.56-39.75)
                const rc2 yv = z[q] * scl;
                __builtin_nontemporal_store(yv, (rc2 *)(o + 2 * j));
                if (a.out2) __builtin_nontemporal_store(yv, (rc2 *)(a.out2 + d_ofs(p, 2 * j, (int)a.ldo2, a.out2_tiled)));
            }
        } else {
            rot_fft<N>(v, tw, t);
#pragma unroll
            for (int u = 0; u < NJ; ++u) {
                const int j2 = t + u * TB;
                if ((M / 2) % TB != 0 && j2 >= M / 2) break;
                const rc2 r0 = v[rsl(2 * j2)] * scl, r1 = v[rsl(2 * j2 + 1)] * scl;
                const float4 y = make_float4(r0.x, r0.y, r1.x, r1.y);
                const fv4 yv = {y.x, y.y, y.z, y.w};
                __builtin_nontemporal_store(yv, (fv4 *)(o + 4 * j2));
                if (a.out2) __builtin_nontemporal_store(yv, (fv4 *)(a.out2 + d_ofs(p, 4 * j2, (int)a.ldo2, a.out2_tiled)));
            }
        }
        gsync<TB / 64>();   // v is reused by the block's next profile
    }
}

// TT = numpy pairwise sum of T64[i]^2 (fit_mode 1's denominator), one wave
__global__ __launch_bounds__(64) void k_tnorm(const double *__restrict__ T64, const PwPlan *__restrict__ plan,
                                              double *__restrict__ TT)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char tsm[];
    const int lane = threadIdx.x & 63;
    const double v = wave_pairwise<double>(*plan, [&](int q) { return T64[q] * T64[q]; }, (double *)tsm, lane);
    if (lane == 0) *TT = v;
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

// ---- per-line median / MAD: one wave per line, radix select ------------------
// Lines: columns (length nsub) of each diagnostic, or rows (length nchan);
// diag 0 std, 1 mean, 2 ptp (f32 arithmetic), 3 fft (plain: every entry valid).
// The valid values of the line go to wave-private LDS as order-preserving
// 64-bit keys (key64), compacted with a ballot.  Order statistics come from a
// most-significant-digit radix select: 8-bit digits from the highest bit where min and max differ,
// a 256-bin LDS histogram per digit, the target bin found by a DPP prefix scan.
// Once the chosen bin holds a single key, one compare-only scan returns it.
// numpy.ma median arithmetic: odd -> 0+mid, even -> ((0+lo)+hi)/2 in the
// dtype; any NaN -> NaN.

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v)
{
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v)
{
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v)
{
    return wave_tree<64>(v, OpAdd());
}

// inclusive prefix sum over the 64 lanes (DPP row shifts + row broadcasts)
__device__ __forceinline__ int wave_incl_scan(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// r-th smallest (0-based) of keys[0, n): uniform result
__device__ unsigned long long wave_select(const unsigned long long *keys, int n, int r, unsigned *hist, int lane)
{
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int j = lane; j < n; j += 64) {
        const unsigned long long k = keys[j];
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
    lo = wave_min_u64(lo);
    hi = wave_max_u64(hi);
    if (lo == hi) return lo;
    const int top = 63 - __clzll((long long)(lo ^ hi));
    int shift = (top / 8) * 8;
    unsigned long long prefix = shift + 8 >= 64 ? 0ull : (lo & (~0ull << (shift + 8)));
    for (; shift >= 0; shift -= 8) {
        const unsigned long long hmask = shift + 8 >= 64 ? 0ull : (~0ull << (shift + 8));
#pragma unroll
        for (int q = 0; q < 4; ++q) hist[lane * 4 + q] = 0u;
        wave_sync();
        for (int j = lane; j < n; j += 64) {
            const unsigned long long k = keys[j];
            if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        wave_sync();
        const uint4 c4 = *(const uint4 *)&hist[lane * 4];
        const int sl = (int)(c4.x + c4.y + c4.z + c4.w);
        const int incl = wave_incl_scan(sl);
        const unsigned long long over = __ballot(incl > r);
        const int L = __ffsll((long long)over) - 1;   // lane holding the target bin
        int below = __shfl(incl - sl, L);
        const uint4 cl = *(const uint4 *)&hist[L * 4];
        int bin = L * 4;
        unsigned cb = cl.x;   // keys in the chosen bin
        if (r - below >= (int)cl.x) {
            below += cl.x;
            ++bin;
            cb = cl.y;
            if (r - below >= (int)cl.y) {
                below += cl.y;
                ++bin;
                cb = cl.z;
                if (r - below >= (int)cl.z) {
                    below += cl.z;
                    ++bin;
                    cb = cl.w;
                }
            }
        }
        r -= below;
        prefix |= (unsigned long long)bin << shift;
        if (cb == 1u && shift > 0) {   // a single key holds the prefix: one compare-only scan
            // one key left under the prefix: it is the answer, found in one
            // compare-only scan instead of the remaining digit passes
            const unsigned long long m = ~0ull << shift;
            unsigned long long f = 0ull;
            for (int j = lane; j < n; j += 64) {
                const unsigned long long k = keys[j];
                if ((k & m) == prefix) f = k;
            }
            return wave_max_u64(f);
        }
        wave_sync();
    }
    return prefix;
}

// median of keys[0, n) (n > 0, no NaN), dtype arithmetic
__device__ double wave_median(const unsigned long long *keys, int n, bool f32, unsigned *hist, int lane)
{
    const int idx = n / 2;
    if (n % 2) {
        const double m = unkey64(wave_select(keys, n, idx, hist, lane));
        return f32 ? (double)(0.0f + (float)m) : 0.0 + m;
    }
    const unsigned long long klo = wave_select(keys, n, idx - 1, hist, lane);
    // hi = rank idx: klo again if it is repeated, else the next larger key
    int le = 0;
    unsigned long long nxt = ~0ull;
    for (int j = lane; j < n; j += 64) {
        const unsigned long long k = keys[j];
        le += k <= klo;
        if (k > klo && k < nxt) nxt = k;
    }
    le = wave_sum_i(le);
    nxt = wave_min_u64(nxt);
    const unsigned long long khi = le > idx ? klo : nxt;
    const double lo = unkey64(klo), hi = unkey64(khi);
    if (f32) {
        const float t = (0.0f + (float)lo) + (float)hi;
        return (double)(t / 2.0f);
    }
    const double t = (0.0 + lo) + hi;
    return t / 2.0;
}

__global__ __launch_bounds__(256) void k_linestats(LineStatsArgs a, int rows, int len, int wpb, int per_wave)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lsm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int line = blockIdx.x * wpb + wave;
    const int nl = 4 * (rows ? a.nsub : a.nchan);
    if (line >= nl || wave >= wpb) return;
    unsigned *hist = (unsigned *)(lsm + (size_t)wave * per_wave);
    unsigned long long *keys = (unsigned long long *)(lsm + (size_t)wave * per_wave + 1024);
    const int nline = rows ? a.nsub : a.nchan;
    const int diag = line / nline, idx = line % nline;
    const bool f32 = diag == 2 && a.ptp_f32, plain = diag == 3;
    // gather the valid values (ballot compaction keeps no particular order: the
    // selection does not need one)
    int cnt = 0, nan = 0;
    for (int q0 = 0; q0 < len; q0 += 64) {
        const int q = q0 + lane;
        double d = 0.0;
        bool v = false;
        if (q < len) {
            const size_t kk = rows ? (size_t)idx * a.nchan + q : (size_t)q * a.nchan + idx;
            v = plain ? true : (a.valid[kk] != 0);
            d = diag == 0 ? a.std_d[kk] : diag == 1 ? a.mean_d[kk] : diag == 2 ? a.ptp_d[kk] : a.fft_d[kk];
        }
        const unsigned long long m = __ballot(v);
        if (v) keys[cnt + __popcll(m & ((1ull << lane) - 1ull))] = key64(d);
        nan |= v && isnan(d);
        cnt += __popcll(m);
    }
    nan = __any(nan);
    wave_sync();
    double med = NAN, mad = NAN;
    if (cnt > 0 && !nan) {
        med = wave_median(keys, cnt, f32, hist, lane);
        // |d - med| in the dtype, in place
        int rnan = 0;
        for (int j = lane; j < cnt; j += 64) {
            const double d = unkey64(keys[j]);
            const double r = f32 ? (double)fabsf((float)d - (float)med) : fabs(d - med);
            rnan |= isnan(r);
            keys[j] = key64(r);
        }
        rnan = __any(rnan);
        wave_sync();
        if (!rnan) mad = wave_median(keys, cnt, f32, hist, lane);
    }
    if (lane == 0) {
        if (!rows) {
            a.col_med[diag * a.nchan + idx] = med;
            a.col_mad[diag * a.nchan + idx] = mad;
        } else {
            a.row_med[diag * a.nsub + idx] = med;
            a.row_mad[diag * a.nsub + idx] = mad;
        }
    }
}

// ---- long lines: W waves per line -------------------------------------------
// The rows (length nchan, a few thousand) are too few for one wave each to fill
// the chip (4*nsub waves), and early radix digits put most keys of a wave in
// one bin, so the LDS atomics serialise.  Here a block of W waves owns a line:
// wave w gathers its own slice of the line into its own key segment, the 256
// bins are shared by the block, and min/max/count/NaN flags are block
// reductions.  Order statistics do not depend on where a key sits, so the
// result is the one k_linestats computes.

template <int W> struct GrpRed {
    unsigned long long *s;   // 2*W slots
    int wave, lane;
    __device__ unsigned long long min_u64(unsigned long long v)
    {
        v = wave_min_u64(v);
        if (lane == 0) s[wave] = v;
        __syncthreads();
        unsigned long long r = s[0];
#pragma unroll
        for (int i = 1; i < W; ++i) r = s[i] < r ? s[i] : r;
        __syncthreads();
        return r;
    }
    __device__ unsigned long long max_u64(unsigned long long v)
    {
        v = wave_max_u64(v);
        if (lane == 0) s[wave] = v;
        __syncthreads();
        unsigned long long r = s[0];
#pragma unroll
        for (int i = 1; i < W; ++i) r = s[i] > r ? s[i] : r;
        __syncthreads();
        return r;
    }
    // min and max in one round trip
    __device__ void minmax_u64(unsigned long long &lo, unsigned long long &hi)
    {
        lo = wave_min_u64(lo);
        hi = wave_max_u64(hi);
        if (lane == 0) {
            s[wave] = lo;
            s[W + wave] = hi;
        }
        __syncthreads();
        lo = s[0];
        hi = s[W];
#pragma unroll
        for (int i = 1; i < W; ++i) {
            lo = s[i] < lo ? s[i] : lo;
            hi = s[W + i] > hi ? s[W + i] : hi;
        }
        __syncthreads();
    }
    __device__ int sum_i(int v) { return sum_uniform(wave_sum_i(v)); }
    // v already uniform across the wave
    __device__ int sum_uniform(int v)
    {
        if (lane == 0) s[wave] = (unsigned long long)(unsigned)v;
        __syncthreads();
        int r = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) r += (int)(unsigned)s[i];
        __syncthreads();
        return r;
    }
};

// r-th smallest (0-based) over every wave's segment keys[0, n): uniform result
template <int W>
__device__ unsigned long long grp_select(GrpRed<W> &g, const unsigned long long *keys, int n, int r, unsigned *hist)
{
    const int lane = g.lane;
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int j = lane; j < n; j += 64) {
        const unsigned long long k = keys[j];
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
    g.minmax_u64(lo, hi);
    if (lo == hi) return lo;
    const int top = 63 - __clzll((long long)(lo ^ hi));
    int shift = (top / 8) * 8;
    unsigned long long prefix = shift + 8 >= 64 ? 0ull : (lo & (~0ull << (shift + 8)));
    for (; shift >= 0; shift -= 8) {
        const unsigned long long hmask = shift + 8 >= 64 ? 0ull : (~0ull << (shift + 8));
        for (int t = threadIdx.x; t < 256; t += 64 * W) hist[t] = 0u;
        __syncthreads();
        for (int j = lane; j < n; j += 64) {
            const unsigned long long k = keys[j];
            if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        const uint4 c4 = *(const uint4 *)&hist[lane * 4];
        const int sl = (int)(c4.x + c4.y + c4.z + c4.w);
        const int incl = wave_incl_scan(sl);
        const unsigned long long over = __ballot(incl > r);
        const int L = __ffsll((long long)over) - 1;
        int below = __shfl(incl - sl, L);
        const uint4 cl = *(const uint4 *)&hist[L * 4];
        int bin = L * 4;
        unsigned cb = cl.x;   // keys in the chosen bin
        if (r - below >= (int)cl.x) {
            below += cl.x;
            ++bin;
            cb = cl.y;
            if (r - below >= (int)cl.y) {
                below += cl.y;
                ++bin;
                cb = cl.z;
                if (r - below >= (int)cl.z) {
                    below += cl.z;
                    ++bin;
                    cb = cl.w;
                }
            }
        }
        r -= below;
        prefix |= (unsigned long long)bin << shift;
        if (cb == 1u && shift > 0) {   // uniform: every wave read the same bins
            const unsigned long long m = ~0ull << shift;
            unsigned long long f = 0ull;
            for (int j = lane; j < n; j += 64) {
                const unsigned long long k = keys[j];
                if ((k & m) == prefix) f = k;
            }
            return g.max_u64(f);   // its barriers also order the bin reads before any re-zeroing
        }
        __syncthreads();   // every wave has read the bins before the next zeroing
    }
    return prefix;
}

// median over the block's keys (ntot > 0 in total, no NaN), dtype arithmetic
template <int W>
__device__ double grp_median(GrpRed<W> &g, const unsigned long long *keys, int n, int ntot, bool f32, unsigned *hist)
{
    const int idx = ntot / 2;
    if (ntot % 2) {
        const double m = unkey64(grp_select<W>(g, keys, n, idx, hist));
        return f32 ? (double)(0.0f + (float)m) : 0.0 + m;
    }
    const unsigned long long klo = grp_select<W>(g, keys, n, idx - 1, hist);
    int le = 0;
    unsigned long long nxt = ~0ull;
    for (int j = g.lane; j < n; j += 64) {
        const unsigned long long k = keys[j];
        le += k <= klo;
        if (k > klo && k < nxt) nxt = k;
    }
    le = g.sum_i(le);
    nxt = g.min_u64(nxt);
    const unsigned long long khi = le > idx ? klo : nxt;
    const double lo = unkey64(klo), hi = unkey64(khi);
    if (f32) {
        const float t = (0.0f + (float)lo) + (float)hi;
        return (double)(t / 2.0f);
    }
    const double t = (0.0 + lo) + hi;
    return t / 2.0;
}

// one block of W waves per line; LDS: 256 bins, 2*W reduction slots, len keys
template <int W> __global__ __launch_bounds__(64 * W) void k_linestats_grp(LineStatsArgs a, int rows, int len)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lsm[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned *hist = (unsigned *)lsm;
    GrpRed<W> g{(unsigned long long *)(lsm + 1024), wave, lane};
    const int nline = rows ? a.nsub : a.nchan;
    const int line = blockIdx.x;
    const int diag = line / nline, idx = line % nline;
    const bool f32 = diag == 2 && a.ptp_f32, plain = diag == 3;
    const int seg = (((len + W - 1) / W) + 63) & ~63;
    const int q0w = wave * seg, q1w = min(len, q0w + seg);
    unsigned long long *keys = (unsigned long long *)(lsm + 1024 + 16 * W) + q0w;
    int cnt = 0, nan = 0;
    for (int q0 = q0w; q0 < q1w; q0 += 64) {
        const int q = q0 + lane;
        double d = 0.0;
        bool v = false;
        if (q < q1w) {
            const size_t kk = rows ? (size_t)idx * a.nchan + q : (size_t)q * a.nchan + idx;
            v = plain ? true : (a.valid[kk] != 0);
            d = diag == 0 ? a.std_d[kk] : diag == 1 ? a.mean_d[kk] : diag == 2 ? a.ptp_d[kk] : a.fft_d[kk];
        }
        const unsigned long long m = __ballot(v);
        if (v) keys[cnt + __popcll(m & ((1ull << lane) - 1ull))] = key64(d);
        nan |= v && isnan(d);
        cnt += __popcll(m);
    }
    nan = g.sum_uniform(__any(nan) ? 1 : 0);   // the barrier also publishes the keys
    const int ntot = g.sum_uniform(cnt);
    double med = NAN, mad = NAN;
    if (ntot > 0 && !nan) {
        med = grp_median<W>(g, keys, cnt, ntot, f32, hist);
        int rnan = 0;
        for (int j = lane; j < cnt; j += 64) {
            const double d = unkey64(keys[j]);
            const double r = f32 ? (double)fabsf((float)d - (float)med) : fabs(d - med);
            rnan |= isnan(r);
            keys[j] = key64(r);
        }
        rnan = g.sum_uniform(__any(rnan) ? 1 : 0);
        if (!rnan) mad = grp_median<W>(g, keys, cnt, ntot, f32, hist);
    }
    if (threadIdx.x == 0) {
        if (!rows) {
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

// |test - 1| at or below this counts as a near tie (the fftmax tolerance of
// the parity tests, DESIGN.md "Numerical semantics")
constexpr double kNearTie = 1e-9;

// counters: [0] changed vs hist[iter-1], [1] zero weights, [2] profiles whose
// fit status is not 1-4 (info may be null: 0), [3] profiles whose test value
// lies within kNearTie of the zap threshold 1.0 (where the last bits of fftmax,
// not bit-identical to pocketfft, could decide), [4+h] != hist[h]

__global__ __launch_bounds__(256) void k_combine(
    int nsub, int nchan, const uint8_t *__restrict__ valid, const int32_t *__restrict__ info,
    const float *__restrict__ w0,
    const double *__restrict__ std_d, const double *__restrict__ mean_d, const double *__restrict__ ptp_d, int ptp_f32,
    const double *__restrict__ fft_d, const double *__restrict__ col_med, const double *__restrict__ col_mad,
    const double *__restrict__ row_med, const double *__restrict__ row_mad, double cth, double sth,
    double *__restrict__ test, float *__restrict__ W, float *__restrict__ hist, int iter,
    int32_t *__restrict__ counters)
{
    // grid-stride; the convergence counters are reduced per block (one atomic
    // per counter per block: same-address atomics serialise at the memory side)
    __shared__ int red[4][4];
    __shared__ unsigned long long dred[4];
    const size_t P = (size_t)nsub * nchan;
    int changed = 0, zero = 0, bad = 0, near = 0;
    unsigned long long diff = 0ull;   // bit h: W != hist[h] somewhere (h < 64)
    const int hmax = iter < 64 ? iter : 64;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < P; k += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(k / nchan), c = (int)(k % nchan);
        const bool v = valid[k] != 0;
        double S[4];
        S[0] = nanmax2(scale_masked_d(std_d[k], v, col_med[c], col_mad[c], cth),
                       scale_masked_d(std_d[k], v, row_med[s], row_mad[s], sth));
        S[1] = nanmax2(scale_masked_d(mean_d[k], v, col_med[nchan + c], col_mad[nchan + c], cth),
                       scale_masked_d(mean_d[k], v, row_med[nsub + s], row_mad[nsub + s], sth));
        // ptp: numpy.ma in f32 for f32 data (Appendix A.5), f64 for f64 data
        S[2] = ptp_f32 ? nanmax2(scale_masked_f((float)ptp_d[k], v, (float)col_med[2 * nchan + c],
                                                (float)col_mad[2 * nchan + c], cth),
                                 scale_masked_f((float)ptp_d[k], v, (float)row_med[2 * nsub + s],
                                                (float)row_mad[2 * nsub + s], sth))
                       : nanmax2(scale_masked_d(ptp_d[k], v, col_med[2 * nchan + c], col_mad[2 * nchan + c], cth),
                                 scale_masked_d(ptp_d[k], v, row_med[2 * nsub + s], row_mad[2 * nsub + s], sth));
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
        near += fabs(t - 1.0) <= kNearTie;   // false for NaN
        const float wn = (t >= 1.0) ? 0.0f : w0[k];
        W[k] = wn;
        hist[(size_t)iter * P + k] = wn;
        changed += !(wn == hist[(size_t)(iter - 1) * P + k]);
        zero += (wn == 0.0f);
        if (info) {   // "Bad status for least squares fit" (iterative_cleaner.py:284-285)
            const int st = info[k];
            bad += (st < 1 || st > 4);
        }
        // history equality (iterative_cleaner.py:135-136)
        for (int h = 0; h < hmax; ++h)
            if (!(wn == hist[(size_t)h * P + k])) diff |= 1ull << h;
        for (int h = 64; h < iter; ++h)
            if (!(wn == hist[(size_t)h * P + k])) atomicOr(&counters[4 + h], 1);
    }
    for (int off = 32; off > 0; off >>= 1) {
        changed += __shfl_xor(changed, off);
        zero += __shfl_xor(zero, off);
        bad += __shfl_xor(bad, off);
        near += __shfl_xor(near, off);
        diff |= __shfl_xor(diff, off);
    }
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wave] = changed;
        red[1][wave] = zero;
        red[2][wave] = bad;
        red[3][wave] = near;
        dred[wave] = diff;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int ch = 0, ze = 0, bd = 0, nt = 0;
        unsigned long long df = 0ull;
        for (int w = 0; w < nw; ++w) {
            ch += red[0][w];
            ze += red[1][w];
            bd += red[2][w];
            nt += red[3][w];
            df |= dred[w];
        }
        // counters[0..1] (changed, zero) as one u64 add: both < 2^32, no carry
        if (ch || ze)
            atomicAdd((unsigned long long *)counters, ((unsigned long long)(unsigned)ze << 32) | (unsigned)ch);
        if (bd) atomicAdd(&counters[2], bd);
        if (nt) atomicAdd(&counters[3], nt);
        for (int h = 0; h < hmax; ++h)
            if ((df >> h) & 1ull) atomicOr(&counters[4 + h], 1);
    }
}

// ============================================================ shard exchanges

// owner rank of subint row s / channel c (world <= 64: linear scan)
__device__ __forceinline__ int geom_row_owner(const ShardGeom &g, int s)
{
    int r = 0;
    while (r + 1 < g.world && s >= g.row0[r + 1]) ++r;
    return r;
}
__device__ __forceinline__ int geom_chan_owner(const ShardGeom &g, int c)
{
    int r = 0;
    while (r + 1 < g.world && c >= g.chan0[r + 1]) ++r;
    return r;
}

// Send blocks to row owners.  Destination d receives, for its rows
// [row0[d], row0[d+1]) x my nchan_loc channels, the fields back to back:
// std, mean, fft (f64), ptp (f32)  — or, in valid mode, valid (u8).
// Blocks are padded to 8 bytes (shard_block_bytes); d's block starts after
// the blocks of d' < d.
__global__ __launch_bounds__(256) void k_pack_rows(ShardGeom g, int nchan_loc, const double *__restrict__ std_d,
                                                   const double *__restrict__ mean_d, const double *__restrict__ fft_d,
                                                   const double *__restrict__ ptp_d, const uint8_t *__restrict__ valid,
                                                   unsigned char *__restrict__ send)
{
    const size_t P = (size_t)g.nsub * nchan_loc;
    const size_t esz = valid ? 1 : 32;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < P; k += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(k / nchan_loc);
        const int d = geom_row_owner(g, s);
        const size_t n_d = (size_t)(g.row0[d + 1] - g.row0[d]) * nchan_loc;   // elements in d's block
        const size_t e = k - (size_t)g.row0[d] * nchan_loc;                   // element within it
        size_t off = 0;
        for (int q = 0; q < d; ++q) off += shard_block_bytes((size_t)(g.row0[q + 1] - g.row0[q]) * nchan_loc, esz);
        unsigned char *blk = send + off;
        if (valid) {
            blk[e] = valid[k];
        } else {
            ((double *)blk)[e] = std_d[k];
            ((double *)blk)[n_d + e] = mean_d[k];
            ((double *)blk)[2 * n_d + e] = fft_d[k];
            ((double *)blk)[3 * n_d + e] = ptp_d[k];
        }
    }
}

// Owned rows from the per-source blocks (source p sent rows_own x nchan_p
// elements per field, after the padded blocks of sources p' < p).
__global__ __launch_bounds__(256) void k_assemble_rows(ShardGeom g, const unsigned char *__restrict__ recv,
                                                       double *__restrict__ std_r, double *__restrict__ mean_r,
                                                       double *__restrict__ fft_r, double *__restrict__ ptp_r,
                                                       uint8_t *__restrict__ valid_r)
{
    const int rows = g.row0[g.rank + 1] - g.row0[g.rank];
    const size_t n = (size_t)rows * g.nchan_g;
    const size_t esz = valid_r ? 1 : 32;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(k / g.nchan_g), c = (int)(k % g.nchan_g);
        const int p = geom_chan_owner(g, c);
        const int np = g.chan0[p + 1] - g.chan0[p];
        const size_t n_p = (size_t)rows * np;
        const size_t e = (size_t)r * np + (c - g.chan0[p]);
        size_t off = 0;
        for (int q = 0; q < p; ++q) off += shard_block_bytes((size_t)rows * (g.chan0[q + 1] - g.chan0[q]), esz);
        const unsigned char *blk = recv + off;
        if (valid_r) {
            valid_r[k] = blk[e];
        } else {
            std_r[k] = ((const double *)blk)[e];
            mean_r[k] = ((const double *)blk)[n_p + e];
            fft_r[k] = ((const double *)blk)[2 * n_p + e];
            ptp_r[k] = ((const double *)blk)[3 * n_p + e];
        }
    }
}

// gathered row statistics: rank p's slot (8 * rows_pad doubles) holds med
// [4][rows_p] then mad [4][rows_p] of its rows_p owned rows
__global__ __launch_bounds__(256) void k_unpack_rowstats(ShardGeom g, int rows_pad, const double *__restrict__ recv,
                                                         double *__restrict__ row_med, double *__restrict__ row_mad)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;   // q * nsub + s
    if (k >= 4 * g.nsub) return;
    const int q = k / g.nsub, s = k % g.nsub;
    const int p = geom_row_owner(g, s);
    const int rows_p = g.row0[p + 1] - g.row0[p];
    const int r = s - g.row0[p];
    const double *slot = recv + (size_t)p * 8 * rows_pad;
    row_med[k] = slot[q * rows_p + r];
    row_mad[k] = slot[4 * rows_p + q * rows_p + r];
}

// Window positions gathered from the row owners (blocks of `blk` ints per
// rank) -> win[nsub] on every rank; flags (optional): moved per subint and the
// moves counter flags[nsub], as k_window does unsharded.
__global__ __launch_bounds__(256) void k_unpack_windows(ShardGeom g, int blk, const int32_t *__restrict__ recv,
                                                        int32_t *__restrict__ win, int32_t *__restrict__ flags)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= g.nsub) return;
    const int p = geom_row_owner(g, s);
    const int w = recv[(size_t)p * blk + (s - g.row0[p])];
    if (flags) {
        const int moved = win[s] != w;
        flags[s] = moved;
        if (moved) atomicAdd(&flags[g.nsub], 1);
    }
    win[s] = w;
}

// fscrunch rows gathered from the row owners: rank p's block (blk floats) holds
// F rows [rows_pad][nbin] then wf [rows_pad] -> F[nsub][nbin], wf[nsub]
__global__ __launch_bounds__(256) void k_unpack_fscrunch(ShardGeom g, int rows_pad, long blk, int nbin,
                                                         const float *__restrict__ recv, float *__restrict__ F,
                                                         float *__restrict__ wf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = blockIdx.y;
    if (i >= nbin) return;
    const int p = geom_row_owner(g, s);
    const float *b = recv + (size_t)p * blk;
    const int t = s - g.row0[p];
    F[(size_t)s * nbin + i] = b[(size_t)t * nbin + i];
    if (i == 0) wf[s] = b[(size_t)rows_pad * nbin + t];
}

__global__ void k_sum_i32(const int32_t *__restrict__ gathered, int world, int n, int32_t *__restrict__ buf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t a = 0;
    for (int r = 0; r < world; ++r) a += gathered[(size_t)r * n + i];
    buf[i] = a;
}

// ============================================================ launchers

static inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

hipError_t launch_chan_partials(hipStream_t st, int mode, const float *raw, const float *W, const int32_t *shift,
                                const float *base, const int32_t *flags, int nsub, int nchan, int nbin,
                                double *part, double *part2, double *wpart, float *D, int ldD, int dtiled,
                                uint8_t *exA, uint8_t *exF)
{
    const int nsb = (nchan + kSuperBlock - 1) / kSuperBlock;
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    dim3 grid(cdiv(nbin, bs), nsb, nsub);
    if (mode == 3 && (!D || ldD < nbin || (dtiled && ldD % 32 != 0))) return hipErrorInvalidValue;
#define IC_CP(M)                                                                                                  \
    IC_GGL(k_chan_partials<M>, grid, dim3(bs), 0, st, raw, W, shift, base, flags, nsub, nchan, nbin, \
                       nsb, part, part2, wpart, D, ldD, dtiled, exA, exF)
    if (mode == 0)
        IC_CP(0);
    else if (mode == 1)
        IC_CP(1);
    else if (mode == 2)
        IC_CP(2);
    else
        IC_CP(3);
#undef IC_CP
    return hipGetLastError();
}

size_t window_lds_bytes(int nbin) { return (size_t)nbin * 8 + kWindowThreads * (8 + 4); }

hipError_t launch_chan_delta(hipStream_t st, const float *raw, const int32_t *shift, const float *base,
                             const float *Wn, const float *Wo, int nsub, int nchan, int nbin, double *part,
                             double *part2, double *wpart, const uint8_t *exA, const uint8_t *exF,
                             const float *rawF)
{
    const int nsb = (nchan + kSuperBlock - 1) / kSuperBlock;
    if (!exA || !exF) return hipErrorInvalidValue;
    // 256 threads: one per channel of the super-block (the change list), then one per bin
    // bins per thread by nbin (C5 template stage 4.55 -> 4.32 ms per clean against 1)
    const int bpt = nbin >= 1024 ? 4 : (nbin >= 512 ? 2 : 1);
#define IC_CD(BP, SP)                                                                                   \
    IC_GGL((k_chan_delta<BP, SP>), dim3(cdiv(nbin, 256 * BP), nsb, nsub), dim3(256), 0, st, raw, rawF, shift, \
           base, Wn, Wo, nchan, nbin, nsb, part, part2, wpart, exA, exF)
    if (rawF) {
        if (bpt == 4) IC_CD(4, true);
        else if (bpt == 2) IC_CD(2, true);
        else IC_CD(1, true);
    } else {
        if (bpt == 4) IC_CD(4, false);
        else if (bpt == 2) IC_CD(2, false);
        else IC_CD(1, false);
    }
#undef IC_CD
    return hipGetLastError();
}

hipError_t launch_window(hipStream_t st, const double *part, long ss, long sl, const SbPlan &plan, int nsub,
                         int nbin, int width, int32_t *win, int32_t *flags)
{
    if (plan.n < 1 || plan.n > kMaxSbLeaves) return hipErrorInvalidValue;
    const size_t shm = window_lds_bytes(nbin);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    IC_GGL(k_window, dim3(nsub), dim3(kWindowThreads), shm, st, part, ss, sl, plan, nbin, width, win, flags);
    return hipGetLastError();
}

hipError_t launch_base(hipStream_t st, const float *raw, const int32_t *shift, const int32_t *win, const int32_t *flags,
                       int nsub, int nchan, int nbin, int width, float *base)
{
    const size_t P = (size_t)nsub * nchan;
    const unsigned grid = (unsigned)std::min<size_t>(cdiv(P, 16), 16384);
    if (nbin % 4 == 0 && ((uintptr_t)raw & 15) == 0 && width <= nbin)
        IC_GGL(k_base<true>, dim3(grid), dim3(256), 0, st, raw, shift, win, flags, nsub, nchan, nbin, width, base);
    else
        IC_GGL(k_base<false>, dim3(grid), dim3(256), 0, st, raw, shift, win, flags, nsub, nchan, nbin, width, base);
    return hipGetLastError();
}

hipError_t launch_pscrunch(hipStream_t st, float *raw, const float *pol1, size_t n)
{
    IC_GGL(k_pscrunch, dim3(std::min<unsigned>(cdiv(n / 4 + 1, 256), 8192)), dim3(256), 0, st, raw, pol1, n);
    return hipGetLastError();
}

hipError_t launch_fscrunch(hipStream_t st, const double *part, long ss, long sl, const double *wpart, long wss,
                           long wsl, const SbPlan &plan, int nsub, int nbin, float *F, float *wf)
{
    if (plan.n < 1 || plan.n > kMaxSbLeaves) return hipErrorInvalidValue;
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    IC_GGL(k_fscrunch, dim3(cdiv(nbin, bs), nsub), dim3(bs), 0, st, part, ss, sl, wpart, wss, wsl, plan,
                       nbin, F, wf);
    return hipGetLastError();
}

hipError_t launch_sb_tree(hipStream_t st, const double *part, const double *wpart, const SbPlan &plan, int nsub,
                          int nbin, long ostr, double *out)
{
    if (plan.n < 1 || plan.n > kMaxSbLeaves) return hipErrorInvalidValue;
    if (ostr < nbin + (wpart ? 1 : 0)) return hipErrorInvalidValue;
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    IC_GGL(k_sb_tree, dim3(cdiv(nbin, bs), nsub), dim3(bs), 0, st, part, wpart, plan, nbin, ostr, out);
    return hipGetLastError();
}

hipError_t launch_unpack_windows(hipStream_t st, const ShardGeom &g, int blk, const int32_t *recv, int32_t *win,
                                 int32_t *flags)
{
    IC_GGL(k_unpack_windows, dim3(cdiv(g.nsub, 256)), dim3(256), 0, st, g, blk, recv, win, flags);
    return hipGetLastError();
}

hipError_t launch_unpack_fscrunch(hipStream_t st, const ShardGeom &g, int rows_pad, long blk, int nbin,
                                  const float *recv, float *F, float *wf)
{
    const int bs = nbin >= 256 ? 256 : ((nbin + 63) / 64) * 64;
    IC_GGL(k_unpack_fscrunch, dim3(cdiv(nbin, bs), g.nsub), dim3(bs), 0, st, g, rows_pad, blk, nbin,
                       recv, F, wf);
    return hipGetLastError();
}

hipError_t launch_pack_rows(hipStream_t st, const ShardGeom &g, int nchan_loc, const double *std_d,
                            const double *mean_d, const double *fft_d, const double *ptp_d, const uint8_t *valid,
                            unsigned char *send)
{
    const size_t P = (size_t)g.nsub * nchan_loc;
    if (P == 0) return hipSuccess;
    IC_GGL(k_pack_rows, dim3(std::min<unsigned>(cdiv(P, 256), 4096)), dim3(256), 0, st, g, nchan_loc,
                       std_d, mean_d, fft_d, ptp_d, valid, send);
    return hipGetLastError();
}

hipError_t launch_assemble_rows(hipStream_t st, const ShardGeom &g, const unsigned char *recv, double *std_r,
                                double *mean_r, double *fft_r, double *ptp_r, uint8_t *valid_r)
{
    const size_t n = (size_t)(g.row0[g.rank + 1] - g.row0[g.rank]) * g.nchan_g;
    if (n == 0) return hipSuccess;
    IC_GGL(k_assemble_rows, dim3(std::min<unsigned>(cdiv(n, 256), 4096)), dim3(256), 0, st, g, recv,
                       std_r, mean_r, fft_r, ptp_r, valid_r);
    return hipGetLastError();
}

hipError_t launch_unpack_rowstats(hipStream_t st, const ShardGeom &g, int rows_pad, const double *recv,
                                  double *row_med, double *row_mad)
{
    IC_GGL(k_unpack_rowstats, dim3(cdiv(4 * (size_t)g.nsub, 256)), dim3(256), 0, st, g, rows_pad, recv,
                       row_med, row_mad);
    return hipGetLastError();
}

hipError_t launch_sum_i32(hipStream_t st, const int32_t *gathered, int world, int n, int32_t *buf)
{
    IC_GGL(k_sum_i32, dim3(cdiv(n, 64)), dim3(64), 0, st, gathered, world, n, buf);
    return hipGetLastError();
}

hipError_t launch_tscrunch(hipStream_t st, const float *F, const float *wf, int nsub, int nbin, float *T,
                           double *T64, double *T2)
{
    IC_GGL(k_tscrunch, dim3(cdiv(nbin, 64)), dim3(64), 0, st, F, wf, nsub, nbin, T, T64, T2);
    return hipGetLastError();
}

hipError_t launch_fit_init(hipStream_t st, const FitStateArrays &S, long P, int32_t *z32, int nz32, uint8_t *late)
{
    IC_GGL(k_fit_init, dim3(cdiv(max(P, (long)nz32), 256)), dim3(256), 0, st, S, P, z32, nz32, late);
    return hipGetLastError();
}

hipError_t launch_fit_prep(hipStream_t st, const FitStateArrays &S, const double *T64, int nbin)
{
    const int nsw = ((nbin + 2 * FIT_TB - 1) / (2 * FIT_TB)) * (2 * FIT_TB);
    IC_GGL(k_fit_prep, dim3(1), dim3(256), sizeof(double) * nsw, st, T64, nbin, nsw, S.U);
    return hipGetLastError();
}

hipError_t launch_fit_pass(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           int dtiled, const int32_t *list, const unsigned long long *nctr, long bound,
                           const FitStateArrays &S, bool round0)
{
    const long n = list ? bound : P;
    if (n <= 0) return hipSuccess;
    // sweep length: nbin rounded up to whole tile pairs (sweep_dma); the row
    // stride ldD may be longer (padding off the power-of-two stride)
    const int nsw = ((nbin + 2 * FIT_TB - 1) / (2 * FIT_TB)) * (2 * FIT_TB);
    if (ldD % 4 != 0 || ldD < nsw || (dtiled && ldD % 32 != 0)) return hipErrorInvalidValue;
    if (round0 && list) return hipErrorInvalidValue;
    if (round0)
        IC_GGL(k_fit_pass<true>, dim3(cdiv(n, 64)), dim3(64), 0, st, D, T64, P, nbin, ldD, nsw, dtiled,
                           list, nctr, S, (const double *)S.U);
    else
        IC_GGL(k_fit_pass<false>, dim3(cdiv(n, 64)), dim3(64), 0, st, D, T64, P, nbin, ldD, nsw,
                           dtiled, list, nctr, S, (const double *)nullptr);
    return hipGetLastError();
}

hipError_t launch_mark_list(hipStream_t st, const int32_t *list, const unsigned long long *nctr, long P, long bound,
                            uint8_t *m, uint8_t v)
{
    if (!list || !nctr || !m) return hipErrorInvalidValue;
    if (bound <= 0) return hipSuccess;
    IC_GGL(k_mark_list, dim3(cdiv(std::min(bound, P), 256)), dim3(256), 0, st, list, nctr, P, m, v);
    return hipGetLastError();
}

hipError_t launch_fit_state(hipStream_t st, const FitStateArrays &S, long P, const int32_t *list,
                            const unsigned long long *nctr, long bound, double *amp, int32_t *info,
                            int32_t *next_list, unsigned long long *ctr, unsigned *done, int32_t *host_n,
                            uint8_t *late)
{
    const long n = list ? bound : P;
    if (n <= 0) return hipSuccess;
    if (n < kStateSmallP)
        IC_GGL(k_fit_state<256>, dim3(cdiv(n, 256)), dim3(256), 0, st, S, P, list, nctr, amp, info, next_list, ctr,
               done, host_n, late);
    else
        IC_GGL(k_fit_state<512>, dim3(cdiv(n, 512)), dim3(512), 0, st, S, P, list, nctr, amp, info, next_list, ctr,
               done, host_n, late);
    return hipGetLastError();
}

hipError_t launch_fit_tail(hipStream_t st, const float *D, const double *T64, long P, int nbin, int ldD,
                           int dtiled, const int32_t *list, const unsigned long long *nctr, long bound,
                           const FitStateArrays &S, double *amp, int32_t *info, unsigned long long *sweeps)
{
    const long n = list ? bound : P;
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<long>(cdiv(n, TAIL_WAVES), 65536);
    IC_GGL(k_fit_tail, dim3(grid), dim3(64 * TAIL_WAVES), 0, st, D, T64, P, nbin, ldD, dtiled, list, nctr,
                       S, amp, info, sweeps);
    return hipGetLastError();
}

template <int NN, bool D64>
static hipError_t launch_p2(hipStream_t st, const DiagArgs &a, size_t P)
{
    using C = P2<NN, D64>;
    const size_t fixed = (size_t)C::TW_LDS * 16;
    int gpb = C::WPP > 1 ? 1 : 8;
    while (gpb > 1 && fixed + gpb * (size_t)C::GROUP_BYTES > 150 * 1024) --gpb;
    const size_t shm = fixed + gpb * (size_t)C::GROUP_BYTES;
    const unsigned grid = (unsigned)std::min<size_t>((P + gpb - 1) / gpb, 4096);
    if (a.mode == DIAG_EXACT)
        IC_GGL((k_diag_p2<NN, DIAG_EXACT, D64>), dim3(grid), dim3(C::TPP * gpb), shm, st, a);
    else if (a.mode == DIAG_CLOSED)
        IC_GGL((k_diag_p2<NN, DIAG_CLOSED, D64>), dim3(grid), dim3(C::TPP * gpb), shm, st, a);
    else if (a.mode == DIAG_FIT)   // f32 rows either way (launch_diag passes D64 = false)
        IC_GGL((k_diag_p2<NN, DIAG_FIT, false>), dim3(grid), dim3(C::TPP * gpb), shm, st, a);
    else   // comprehensive_stats of given rows (f64 data: the fractional-dedispersion loop)
        IC_GGL((k_diag_p2<NN, DIAG_STATS, D64>), dim3(grid), dim3(C::TPP * gpb), shm, st, a);
    return hipGetLastError();
}

template <int NN>
static hipError_t launch_cl(hipStream_t st, const DiagArgs &a, size_t P)
{
    using C = CLay<NN>;
    const int gpb = C::GPB;
    const size_t shm = (size_t)C::TW_LDS * 16 + gpb * (size_t)C::GROUP_BYTES;
    const unsigned grid = (unsigned)std::min<size_t>((P + gpb - 1) / gpb, 4096);
    if (a.mode == DIAG_EXACT)
        IC_GGL((k_diag_cl<NN, DIAG_EXACT>), dim3(grid), dim3(C::L * gpb), shm, st, a);
    else if (a.mode == DIAG_STATS)
        IC_GGL((k_diag_cl<NN, DIAG_STATS>), dim3(grid), dim3(C::L * gpb), shm, st, a);
    else
        IC_GGL((k_diag_cl<NN, DIAG_CLOSED>), dim3(grid), dim3(C::L * gpb), shm, st, a);
    return hipGetLastError();
}

static bool uses_cl(const DiagArgs &a)
{
    if (!a.chain || a.data_f64 || !(a.nbin == 1024 || a.nbin == 2048 || a.nbin == 4096)) return false;
    // STATS: row-major residual rows (the FFT mode's rotated residual; the
    // pulse region was applied when they were formed)
    if (a.mode == DIAG_STATS) return a.D && a.ldD == a.nbin && !a.dtiled;
    return (a.mode == DIAG_EXACT || a.mode == DIAG_CLOSED) && a.T2 && a.raw && a.base && !a.pr_on;
}

// profile lists / skips: k_diag_cl, and k_diag_p2 in the exact mode and on
// given rows (the FFT mode's rotated residuals)
bool diag_list_supported(const DiagArgs &a)
{
    const int n = a.nbin;
    return uses_cl(a) ||
           ((a.mode == DIAG_EXACT || a.mode == DIAG_STATS) && n >= 64 && n <= 4096 && (n & (n - 1)) == 0);
}

hipError_t launch_diag(hipStream_t st, const DiagArgs &a)
{
    const int nbin = a.nbin;
    const size_t P = (size_t)a.nsub * a.nchan;
    if (P == 0) return hipSuccess;
    if (a.mode == DIAG_CLOSED ? (!a.raw || !a.base || !a.TT || !a.amp || !a.info)
                              : (!a.D || a.ldD < nbin || (a.mode != DIAG_STATS && (!a.amp || !a.info)) ||
                                 (a.mode == DIAG_FIT && !a.TT)))
        return hipErrorInvalidValue;
    // the chain-layout kernel: exact / closed modes from the raw cube, f32 data, no pulse region
    if (uses_cl(a)) {
        if (nbin == 1024) return launch_cl<1024>(st, a, P);
        if (nbin == 2048) return launch_cl<2048>(st, a, P);
        if (nbin == 4096) return launch_cl<4096>(st, a, P);
    }
    if ((a.list || a.skip) && !diag_list_supported(a)) return hipErrorInvalidValue;
#define IC_P2(NN)                                                                                  \
    if (nbin == NN) {                                                                              \
        if (a.data_f64 && a.mode != DIAG_FIT) return launch_p2<NN, true>(st, a, P);                \
        return launch_p2<NN, false>(st, a, P);                                                     \
    }
    IC_P2(64) IC_P2(128) IC_P2(256) IC_P2(512) IC_P2(1024) IC_P2(2048) IC_P2(4096)
#undef IC_P2
    if (a.mode == DIAG_FIT) return hipErrorInvalidValue;   // power-of-two nbin only
    // nleaf/nops upper bound from nbin: leaves >= 64 samples except tiny n
    const int nleaf_ub = nbin <= 128 ? 1 : (nbin / 64 + 1);
    const DiagLayout lay = diag_layout(nbin, nleaf_ub, nleaf_ub);
    const size_t fixed = (size_t)lay.ntw * 16;
    int wpb = 4;
    while (wpb > 1 && fixed + wpb * lay.per_wave > 150 * 1024) --wpb;
    const size_t shm = fixed + wpb * lay.per_wave;
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<size_t>((P + wpb - 1) / wpb, 8192);
    IC_GGL(k_diag, dim3(grid), dim3(64 * wpb), shm, st, a);
    return hipGetLastError();
}

size_t diag_lds_bytes(int nbin)
{
    switch (nbin) {
    case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: return 0;
    default: break;
    }
    const int nleaf_ub = nbin <= 128 ? 1 : (nbin / 64 + 1);
    const DiagLayout lay = diag_layout(nbin, nleaf_ub, nleaf_ub);
    return (size_t)lay.ntw * 16 + lay.per_wave;
}

hipError_t launch_tnorm(hipStream_t st, const double *T64, const PwPlan *plan, int nleaf_ub, double *TT)
{
    const size_t shm = (size_t)(nleaf_ub * 9 + nleaf_ub + 8) * 8;
    IC_GGL(k_tnorm, dim3(1), dim3(64), shm, st, T64, plan, TT);
    return hipGetLastError();
}

hipError_t launch_linestats(hipStream_t st, const LineStatsArgs &a, int which)
{
    // columns (length nsub), then rows (length nchan); wave-private LDS:
    // 256-bin histogram + the line's keys
    for (int rows = 0; rows < 2; ++rows) {
        if (!((which >> rows) & 1)) continue;
        const int len = rows ? a.nchan : a.nsub;
        const int lines = 4 * (rows ? a.nsub : a.nchan);
        if (lines == 0 || len == 0) continue;
        // few long lines (the rows): W waves per line (a.grp_waves = W in {0, 4, 8},
        // 0 = one wave per line; a.grp_minlen = the shortest line it takes)
        if (lines < 8192 && len >= a.grp_minlen) {
            const int W = a.grp_waves;
            if (W == 4 || W == 8) {
                const int seg = (((len + W - 1) / W) + 63) & ~63;
                const size_t gshm = 1024 + 16 * (size_t)W + (size_t)W * seg * 8;
                if (gshm <= 160 * 1024) {
                    if (W == 4)
                        IC_GGL(k_linestats_grp<4>, dim3(lines), dim3(256), gshm, st, a, rows, len);
                    else
                        IC_GGL(k_linestats_grp<8>, dim3(lines), dim3(512), gshm, st, a, rows, len);
                    const hipError_t e = hipGetLastError();
                    if (e != hipSuccess) return e;
                    continue;
                }
            }
        }
        const int per_wave = 1024 + ((len * 8 + 15) / 16) * 16;
        int wpb = 4;
        while (wpb > 1 && (size_t)wpb * per_wave > 64 * 1024) --wpb;
        const size_t shm = (size_t)wpb * per_wave;
        if (shm > 160 * 1024) return hipErrorInvalidValue;
        IC_GGL(k_linestats, dim3(cdiv(lines, wpb)), dim3(64 * wpb), shm, st, a, rows, len, wpb,
                           per_wave);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_combine(hipStream_t st, int nsub, int nchan, const uint8_t *valid, const int32_t *info,
                          const float *w0,
                          const double *std_d, const double *mean_d, const double *ptp_d, int ptp_f32,
                          const double *fft_d, const double *col_med, const double *col_mad,
                          const double *row_med, const double *row_mad, double chanthresh,
                          double subintthresh, double *test, float *W, float *hist, int iter,
                          int32_t *counters)
{
    const size_t P = (size_t)nsub * nchan;
    const unsigned grid = (unsigned)std::min<size_t>(cdiv(P, 256), 1024);
    IC_GGL(k_combine, dim3(grid), dim3(256), 0, st, nsub, nchan, valid, info, w0, std_d,
                       mean_d, ptp_d, ptp_f32, fft_d, col_med, col_mad, row_med, row_mad, chanthresh, subintthresh,
                       test, W, hist, iter, counters);
    return hipGetLastError();
}

hipError_t launch_residual(hipStream_t st, const float *D, const float *raw, const float *base, const double *T64,
                           const double *amp, const int32_t *info, const int32_t *shift, int nsub, int nchan,
                           int nbin, int ldD, int dtiled, int pr_on, double pr_factor, int pr_start, int pr_end,
                           float *R)
{
    const size_t P = (size_t)nsub * nchan;
    if (!D && (!raw || !base)) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<size_t>(cdiv(P, 4), 16384);
    IC_GGL(k_residual, dim3(grid), dim3(256), 0, st, D, raw, base, T64, amp, info, shift, P, nchan, nbin,
                       ldD, dtiled, pr_on, pr_factor, pr_start, pr_end, R);
    return hipGetLastError();
}

bool rotate_supported(int nbin)
{
    switch (nbin) {
    case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: return true;
    default: return false;
    }
}

bool rotate_stats_supported(int nbin, bool data_f64) { return nbin == 1024 && !data_f64; }

// The identity "rotation" of an archive stored dedispersed (its dedisperse is a
// no-op, archive.py dedisperse): out[p] = f32(in[p] - base[p]) (and out2), for
// the subints flags selects; a wave per profile, 16-byte rows.
__global__ __launch_bounds__(256) void k_rotate_identity(RotateArgs a)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t P = (size_t)a.nsub * a.nchan;
    for (size_t p = (size_t)blockIdx.x * 4 + wave; p < P; p += (size_t)gridDim.x * 4) {
        if (a.flags && a.flags[p / (unsigned)a.nchan] == 0) continue;
        const float b = a.base ? a.base[p] : 0.0f;
        for (int j = 4 * lane; j < a.nbin; j += 256) {
            const float4 x = *(const float4 *)(a.in + d_ofs(p, j, (int)a.ld_in, a.in_tiled));
            const float4 y = make_float4(x.x - b, x.y - b, x.z - b, x.w - b);
            *(float4 *)(a.out + p * (size_t)a.ldo + j) = y;
            if (a.out2) *(float4 *)(a.out2 + d_ofs(p, j, (int)a.ldo2, a.out2_tiled)) = y;
        }
    }
}

hipError_t launch_rotate(hipStream_t st, const RotateArgs &a)
{
    const size_t P = (size_t)a.nsub * a.nchan;
    if (P == 0) return hipSuccess;
    const bool stats = a.std_o != nullptr;
    if (stats && (!rotate_stats_supported(a.nbin, false) || !a.amp || a.sign > 0 || a.out2 || !a.w0 || !a.mean_o ||
                  !a.ptp_o || !a.fft_o))
        return hipErrorInvalidValue;
    if (!rotate_supported(a.nbin) || !a.in || (!a.out && !stats) || !a.tw || !a.tw_p2 || a.ld_in < a.nbin ||
        (!stats && a.ldo < a.nbin) ||
        (!a.ph && !a.delay2 && !a.identity) ||
        (a.ld_in & 3) || (a.ldo & 3) || (a.out2 && (a.ldo2 < a.nbin || (a.ldo2 & 3))) ||
        (a.amp && (!a.T64 || !a.info)) || (a.in_tiled && (a.ld_in & 31)) || (a.out2_tiled && (a.ldo2 & 31)) ||
        (a.identity && (a.amp || a.late || a.list)) || (a.list && !a.nctr))
        return hipErrorInvalidValue;
    if (a.identity) {
        IC_GGL(k_rotate_identity, dim3((unsigned)std::min<size_t>(cdiv(P, 4), 16384)), dim3(256), 0, st, a);
        return hipGetLastError();
    }
#define IC_ROT(NN)                                                                                 \
    case NN:                                                                                       \
        if (a.delay2)                                                                              \
            IC_GGL((k_rotate<NN, true>),                                                           \
                   dim3((unsigned)std::min<size_t>(cdiv(P, RotCfg<NN>::WPB), 16384 / RotCfg<NN>::WPB)), \
                   dim3(RotCfg<NN>::TB * RotCfg<NN>::WPB), 0, st, a);                              \
        else                                                                                       \
            IC_GGL((k_rotate<NN, false>),                                                          \
                   dim3((unsigned)std::min<size_t>(cdiv(P, RotCfg<NN>::WPB), 16384 / RotCfg<NN>::WPB)), \
                   dim3(RotCfg<NN>::TB * RotCfg<NN>::WPB), 0, st, a);                              \
        break;
    if (stats) {   // nbin 1024 (rotate_stats_supported)
        const dim3 grid((unsigned)std::min<size_t>(cdiv(P, RotCfg<1024>::WPB), 16384 / RotCfg<1024>::WPB));
        const dim3 block(RotCfg<1024>::TB * RotCfg<1024>::WPB);
        if (a.delay2) IC_GGL((k_rotate<1024, true, true>), grid, block, 0, st, a);
        else IC_GGL((k_rotate<1024, false, true>), grid, block, 0, st, a);
        return hipGetLastError();
    }
    switch (a.nbin) {
        IC_ROT(64) IC_ROT(128) IC_ROT(256) IC_ROT(512) IC_ROT(1024) IC_ROT(2048) IC_ROT(4096)
    default: return hipErrorInvalidValue;
    }
#undef IC_ROT
    return hipGetLastError();
}

}  // namespace icgpu
