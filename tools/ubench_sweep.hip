// ubench_sweep.hip — where does a full round of k_fit_pass go?  One A sweep
// (f = RN(RN(x t) - p), J = RN(d / h) by the four-op division, sum f^2 and J^2
// in sample order: FastBody<true, false>'s arithmetic) of every profile of a
// C2-sized fit cube (1 152 000 profiles x 1024 bins, 4.7 GB), one wave per 64
// profiles, 16-bin LDS-DMA tiles double-buffered as in ic_kernels.hip.
// Variants (times per full round, hipEvents, best of 5):
//   dma     the sweep's data movement alone (tiles read from LDS, xor-folded)
//   alu     the arithmetic alone on LDS tiles that are never refilled
//   both    the real sweep (= a full round of k_fit_pass's A body)
// each with the fit cube's tiled layout (t32: [64 profiles][32 bins] blocks,
// the source-side transposed DMA, 16 half lines per instruction) and with a
// [bins/4][64 profiles][4 bins] layout (l4: every DMA instruction 1 KiB
// contiguous, lane-linear, no transpose).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/ubench_sweep.hip -o tools/ubench_sweep
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef float fv4 __attribute__((ext_vector_type(4)));
constexpr int TB = 16;     // bins per tile
constexpr int BUF = 4096;  // bytes per tile buffer (64 profiles x 16 bins x 4 B)

enum { LAY_T32 = 0, LAY_L4 = 1 };
enum { DO_DMA = 1, DO_ALU = 2, DO_PRO = 4, DO_EPI = 8, DO_PRE = 16, EPI_NT = 32, EPI_PACK = 64, PERS = 128,
       EPI_ONE = 256, EPI_HOT = 512 };
// EPI_ONE: one 8-B output per lane; EPI_HOT: the five outputs into the same
// 2.5 KiB for every wave (cache-resident: no DRAM writes)
// PERS: a persistent grid (the resident waves), groups taken from a queue
// (one atomic per group): a wave's output stores of one group are in flight
// while it sweeps the next, instead of holding its slot at s_endpgm
// DO_PRO: k_fit_pass's prologue, a dependent chain before the sweep (a list
// entry, the profile's request, its trial point), DO_PRE: the same chain with
// the first tile pair requested before it; DO_EPI: the five per-lane outputs

__device__ __forceinline__ uint32_t lds_u32(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

struct Acc {
    double sf, sj, xa, xha, ha, yha, yla;
    uint32_t x;
};

template <int OFF>
__device__ __forceinline__ void read_tile(const uint32_t (&rd)[4], fv4 (&v)[4])
{
#pragma unroll
    for (int c = 0; c < 4; ++c) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[c]) : "v"(rd[c]), "i"(OFF));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}

template <int WHAT>
__device__ __forceinline__ void body(Acc &a, const double *__restrict__ T, int b0, const fv4 (&v)[4])
{
    if (!(WHAT & DO_ALU)) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
            a.x ^= __float_as_uint(v[c].x) ^ __float_as_uint(v[c].y) ^ __float_as_uint(v[c].z) ^ __float_as_uint(v[c].w);
        return;
    }
    double t[TB];
#pragma unroll
    for (int i = 0; i < TB; ++i) t[i] = T[b0 + i];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float pf[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
        double p[4], f[4], d[4], q[4], r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = (double)pf[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = a.xa * t[4 * c + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = a.xha * t[4 * c + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = f[k] - p[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = d[k] - p[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = d[k] - f[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = d[k] * a.yla;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = fma(d[k], a.yha, q[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = fma(-a.ha, q[k], d[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = fma(r[k], a.yha, q[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a.sf = a.sf + f[k] * f[k];
            a.sj = a.sj + q[k] * q[k];
        }
    }
    asm volatile("" : "+v"(a.sf), "+v"(a.sj));
}

template <int LAY>
__device__ __forceinline__ void dma(const float *const (&src)[4], char *buf, int b0)
{
    const int off = LAY == LAY_T32 ? ((b0 >> 5) << 11) + (b0 & 31) : (b0 >> 2) * 256;
#pragma unroll
    for (int m = 0; m < 4; ++m)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src[m] + off),
                                         (__attribute__((address_space(3))) void *)(buf + m * 1024), 16, 0, 0);
}

struct Side {
    const int *list, *mode;
    const double *xa;
    double *o;
};

template <int LAY, int WHAT>
__device__ __forceinline__ void do_group(char *lbuf, const float *__restrict__ D, const double *__restrict__ T, long G,
                                         int ld, double *__restrict__ out, const Side &sd, long g)
{
    const int lane = threadIdx.x;
    const float *src[4];
    uint32_t rd[4];
    if (LAY == LAY_T32) {
        // instruction m, lane l: chunk (l & 3) ^ ((l >> 4) & 3) of profile 16 m + l / 4
        const int c = (lane & 3) ^ ((lane >> 4) & 3);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const long k = 64 * g + 16 * m + (lane >> 2);
            src[m] = D + (((k >> 6) * (long)(ld >> 5)) << 11) + ((k & 63) << 5) + 4 * c;
        }
        const uint32_t base = lds_u32(lbuf) + 16u * (uint32_t)(64 * (lane >> 4) + 4 * (lane & 15));
        const int gq = (lane >> 2) & 3;
#pragma unroll
        for (int c2 = 0; c2 < 4; ++c2) rd[c2] = base + 16u * (uint32_t)(c2 ^ gq);
    } else {
        // instruction m: bins 4 m .. 4 m + 3 of all 64 profiles, 1 KiB contiguous, lane-linear
#pragma unroll
        for (int m = 0; m < 4; ++m) src[m] = D + g * 64L * ld + m * 256 + lane * 4;
#pragma unroll
        for (int c2 = 0; c2 < 4; ++c2) rd[c2] = lds_u32(lbuf) + 1024u * c2 + 16u * lane;
    }
    Acc a;
    a.sf = a.sj = 0.0;
    a.x = 0;
    a.xa = 1.0 + 1e-3 * lane;
    a.ha = 0x1p-26 * a.xa;
    a.xha = a.xa + a.ha;
    a.yha = 1.0 / a.ha;
    a.yla = fma(-a.ha, a.yha, 1.0) * a.yha;
    const int nt = ld / TB;
    long kk = 0;
    if (WHAT & DO_PRE) {
        dma<LAY>(src, lbuf, 0);
        dma<LAY>(src, lbuf + BUF, TB);
    }
    if (WHAT & (DO_PRO | DO_PRE)) {
        kk = sd.list[64 * g + lane];
        const int st = sd.mode[kk];
        if (!__any(st != 3)) return;   // (never: every request is 1 here)
        a.xa = st == 1 ? sd.xa[kk] : 1.0;
        a.ha = 0x1p-26 * a.xa;
        a.xha = a.xa + a.ha;
        a.yha = 1.0 / a.ha;
        a.yla = fma(-a.ha, a.yha, 1.0) * a.yha;
    }
    if (WHAT & DO_PRE) {
    } else if (WHAT & DO_DMA) {
        dma<LAY>(src, lbuf, 0);
        dma<LAY>(src, lbuf + BUF, TB);
    } else {
        dma<LAY>(src, lbuf, 0);
        dma<LAY>(src, lbuf + BUF, TB);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (int t = 0; t < nt; t += 2) {
        fv4 v[4];
        if (WHAT & DO_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        read_tile<0>(rd, v);
        body<WHAT>(a, T, t * TB, v);
        asm volatile("" : "+v"(a.sf), "+v"(a.sj), "+v"(a.x));
        read_tile<BUF>(rd, v);
        asm volatile("" ::: "memory");
        if ((WHAT & DO_DMA) && t + 2 < nt) {
            dma<LAY>(src, lbuf, (t + 2) * TB);
            dma<LAY>(src, lbuf + BUF, (t + 3) * TB);
        }
        body<WHAT>(a, T, (t + 1) * TB, v);
        asm volatile("" : "+v"(a.sf), "+v"(a.sj), "+v"(a.x));
    }
    if (WHAT & EPI_ONE) {
        sd.o[kk] = a.sf + a.sj;
    } else if (WHAT & EPI_HOT) {
        sd.o[lane] = a.sf;
        sd.o[lane + 64] = a.sj;
        sd.o[lane + 128] = a.sf * 2.0;
        sd.o[lane + 192] = a.sj * 2.0;
        sd.o[lane + 256] = a.sf + a.sj;
    } else if (WHAT & EPI_NT) {
        __builtin_nontemporal_store(a.sf, &sd.o[kk]);
        __builtin_nontemporal_store(a.sj, &sd.o[kk + 64 * G]);
        __builtin_nontemporal_store(a.sf * 2.0, &sd.o[kk + 128 * G]);
        __builtin_nontemporal_store(a.sj * 2.0, &sd.o[kk + 192 * G]);
        __builtin_nontemporal_store(a.sf + a.sj, &sd.o[kk + 256 * G]);
    } else if (WHAT & EPI_PACK) {
        double4 *o4 = (double4 *)sd.o;
        o4[kk] = make_double4(a.sf, a.sj, a.sf * 2.0, a.sj * 2.0);
        sd.o[kk + 256 * G] = a.sf + a.sj;
    } else if (WHAT & DO_EPI) {
        sd.o[kk] = a.sf;
        sd.o[kk + 64 * G] = a.sj;
        sd.o[kk + 128 * G] = a.sf * 2.0;
        sd.o[kk + 192 * G] = a.sj * 2.0;
        sd.o[kk + 256 * G] = a.sf + a.sj;
    }
    if (a.sf + a.sj + (double)a.x == 1.2345) out[0] = 1.0;   // keep the work
}

template <int LAY, int WHAT>
__global__ __launch_bounds__(64) void k_sweep(const float *__restrict__ D, const double *__restrict__ T, long G,
                                             int ld, double *__restrict__ out, Side sd, unsigned *q)
{
    __shared__ __attribute__((aligned(16))) char lbuf[2 * BUF];
    if (WHAT & PERS) {
        for (;;) {
            unsigned g = 0;
            if (threadIdx.x == 0) g = atomicAdd(q, 1u);
            g = __builtin_amdgcn_readfirstlane(g);
            if (g >= G) break;
            do_group<LAY, WHAT>(lbuf, D, T, G, ld, out, sd, g);
        }
    } else {
        if ((long)blockIdx.x < G) do_group<LAY, WHAT>(lbuf, D, T, G, ld, out, sd, blockIdx.x);
    }
}

Side g_side;
unsigned *g_q;
int g_resident;

template <int LAY, int WHAT>
float run(const float *D, const double *T, long G, int ld, double *out, hipEvent_t e0, hipEvent_t e1)
{
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipMemsetAsync(g_q, 0, 4));
        const unsigned grid = (WHAT & PERS) ? (unsigned)g_resident : (unsigned)G;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_sweep<LAY, WHAT>), dim3(grid), dim3(64), 0, 0, D, T, G, ld, out, g_side, g_q);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

__global__ void k_fill(float *D, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        D[i] = (float)((i * 2654435761u) & 1023) * 0.01f - 5.0f;
}

int main(int argc, char **argv)
{
    const long P = argc > 1 ? atol(argv[1]) : 1152000;
    const int ld = 1024;
    const long G = P / 64;
    const size_t n = (size_t)G * 64 * ld;
    float *D;
    double *T, *out;
    CK(hipMalloc(&D, n * sizeof(float)));
    CK(hipMalloc(&T, ld * sizeof(double)));
    CK(hipMalloc(&out, sizeof(double)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, D, n);
    std::vector<double> th(ld);
    for (int i = 0; i < ld; ++i) th[i] = (double)(float)(0.5 + 0.001 * i);
    CK(hipMemcpy(T, th.data(), ld * sizeof(double), hipMemcpyHostToDevice));
    {
        std::vector<int> li(G * 64), mo(G * 64, 1);
        std::vector<double> xa(G * 64, 1.0009765625);
        for (long i = 0; i < G * 64; ++i) li[i] = (int)i;   // a full round's list: every profile in order
        int *dl, *dm;
        double *dx, *dout;
        CK(hipMalloc(&dl, li.size() * 4));
        CK(hipMalloc(&dm, mo.size() * 4));
        CK(hipMalloc(&dx, xa.size() * 8));
        CK(hipMalloc(&dout, xa.size() * 8 * 5));
        CK(hipMemcpy(dl, li.data(), li.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dm, mo.data(), mo.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dx, xa.data(), xa.size() * 8, hipMemcpyHostToDevice));
        g_side = Side{dl, dm, dx, dout};
        CK(hipMalloc(&g_q, 4));
        int nb = 0, ncu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sweep<LAY_T32, DO_DMA | DO_ALU | DO_PRO | DO_EPI | PERS>, 64, 0));
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
        g_resident = nb * ncu;
        printf("persistent grid: %d waves (%d per CU)\n", g_resident, nb);
    }
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double gb = n * 4.0 / 1e9;
    struct R { const char *name; float ms; } r[] = {
        {"t32 dma ", run<LAY_T32, DO_DMA>(D, T, G, ld, out, e0, e1)},
        {"t32 alu ", run<LAY_T32, DO_ALU>(D, T, G, ld, out, e0, e1)},
        {"t32 both", run<LAY_T32, DO_DMA | DO_ALU>(D, T, G, ld, out, e0, e1)},
        {"l4  dma ", run<LAY_L4, DO_DMA>(D, T, G, ld, out, e0, e1)},
        {"l4  alu ", run<LAY_L4, DO_ALU>(D, T, G, ld, out, e0, e1)},
        {"l4  both", run<LAY_L4, DO_DMA | DO_ALU>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | DO_EPI>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pre+epi", run<LAY_T32, DO_DMA | DO_ALU | DO_PRE | DO_EPI>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi_nt", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | EPI_NT>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi_pack", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | EPI_PACK>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi (again)", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | DO_EPI>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi_one", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | EPI_ONE>(D, T, G, ld, out, e0, e1)},
        {"t32 both+pro+epi_hot", run<LAY_T32, DO_DMA | DO_ALU | DO_PRO | EPI_HOT>(D, T, G, ld, out, e0, e1)},
        {"t32 both+epi_hot", run<LAY_T32, DO_DMA | DO_ALU | EPI_HOT>(D, T, G, ld, out, e0, e1)},
    };
    printf("fit cube %.2f GB (%ld profiles x %d bins), one A sweep per profile, best of 5\n", gb, G * 64, ld);
    for (auto &x : r) printf("%s %8.3f ms  %7.1f GB/s\n", x.name, x.ms, gb / (x.ms / 1e3));
    return 0;
}
