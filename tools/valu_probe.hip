// FP64 VALU throughput probe (timing only; not part of the product).
//
// Table mode's sweeps issue one v_mul_f64 and one v_add_f64 per cell-tap (no FMA: the
// reference rounds every product). This measures what gfx950 sustains for exactly that mix:
// every lane runs C independent accumulator chains acc += b * x (mul, then add), with b from
// SGPRs. Prints wave-instructions per second and per CU-cycle for the given clock.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/valu_probe.hip -o tools/valu_probe
//   tools/valu_probe [waves_per_cu=8] [iters=4096]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int C>
__global__ __launch_bounds__(256) void chains(double *out, const double *coef, int iters)
{
    double acc[C], x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        acc[c] = 0.0;
        x[c] = 1.0 + 1e-9 * (threadIdx.x + c);
    }
    for (int it = 0; it < iters; ++it) {
        const double b = coef[it & 63]; // uniform: s_load
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += b * x[c];
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += acc[c];
    if (s == 12345.678) out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int C> static void run(int blocks, int iters, double *out, const double *coef)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(chains<C>, dim3(blocks), dim3(256), 0, 0, out, coef, iters);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(chains<C>, dim3(blocks), dim3(256), 0, 0, out, coef, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double winstr = (double)blocks * 4 * iters * C * 2; // mul + add per chain per iteration
    const double per_s = winstr / (ms * 1e-3);
    // 256 CUs x 4 SIMDs; a 4-cycle instruction => 1 wave-instruction per SIMD per 4 cycles
    printf("{\"chains\": %d, \"blocks\": %d, \"ms\": %.4f, \"wave_instr_per_s\": %.4e, "
           "\"simd_cycles_per_instr_at_2400MHz\": %.3f}\n",
           C, blocks, ms, per_s, 1024.0 * 2.4e9 / per_s);
}

int main(int argc, char **argv)
{
    const int wpc = argc > 1 ? atoi(argv[1]) : 8;
    const int iters = argc > 2 ? atoi(argv[2]) : 4096;
    const int blocks = 256 * wpc / 4;
    double *out, *coef;
    hipMalloc(&out, (size_t)blocks * 256 * sizeof(double));
    hipMalloc(&coef, 64 * sizeof(double));
    double h[64];
    for (int i = 0; i < 64; ++i) h[i] = 0.5 + i * 1e-3;
    hipMemcpy(coef, h, sizeof(h), hipMemcpyHostToDevice);
    run<2>(blocks, iters, out, coef);
    run<4>(blocks, iters, out, coef);
    run<8>(blocks, iters, out, coef);
    run<16>(blocks, iters, out, coef);
    hipFree(out);
    hipFree(coef);
    return 0;
}
