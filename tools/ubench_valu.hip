// Micro-benchmark: issue rate of f64 / f32 / int VALU ops on gfx950 (wave64),
// to decide whether the fit sweep is VALU-bound.  8 independent chains per
// lane, many waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ __launch_bounds__(256) void k(double *out, float *outf, int *outi, int iters, double a, double b)
{
    double x[8];
    float y[8];
    int z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        x[j] = threadIdx.x * 1e-3 + j;
        y[j] = (float)x[j];
        z[j] = threadIdx.x + j;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) x[j] = __builtin_fma(x[j], a, b);
            if (OP == 1) x[j] = x[j] * a;
            if (OP == 2) x[j] = x[j] + b;
            if (OP == 3) y[j] = __builtin_fmaf(y[j], (float)a, (float)b);
            if (OP == 4) z[j] = z[j] + i;
        }
    }
    double s = 0;
    float sf = 0;
    int si = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        s += x[j];
        sf += y[j];
        si += z[j];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    outf[blockIdx.x * blockDim.x + threadIdx.x] = sf;
    outi[blockIdx.x * blockDim.x + threadIdx.x] = si;
}

template <int OP>
void run(const char *name, int blocks, int iters)
{
    double *o;
    float *of;
    int *oi;
    hipMalloc(&o, sizeof(double) * blocks * 256);
    hipMalloc(&of, sizeof(float) * blocks * 256);
    hipMalloc(&oi, sizeof(int) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, of, oi, iters, 0.999999, 1e-9);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, of, oi, iters, 0.999999, 1e-9);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waveinstr = (double)blocks * 4 * iters * 8;   // wave64 instructions
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    const double cycles = ms * 1e-3 * clk * 1e3 * 1024;   // SIMD-cycles at the max clock
    printf("%-10s %8.3f ms  %.3g wave-instr/s  %.2f SIMD-cycles/instr at %d MHz\n", name, ms,
           waveinstr / (ms * 1e-3), cycles / waveinstr, clk / 1000);
    hipFree(o);
    hipFree(of);
    hipFree(oi);
}

int main()
{
    const int blocks = 256 * 8 * 2;   // 16 waves per CU... x2 generations
    run<0>("fma_f64", blocks, 4096);
    run<1>("mul_f64", blocks, 4096);
    run<2>("add_f64", blocks, 4096);
    run<3>("fma_f32", blocks, 4096);
    run<4>("add_u32", blocks, 4096);
    return 0;
}
