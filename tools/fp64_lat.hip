// FP64 VALU latency / throughput probe (timing only): K independent chains of `acc = acc + x * y` (v_mul_f64
// then v_add_f64, the sweeps' pair; no FMA) per lane, W waves per SIMD. Prints ns per chained step, and the
// implied cycles per step per wave at the measured clock-free basis (ns). Build: make -C tools fp64_lat
#include <chrono>
#include <cstdio>
#include <hip/hip_runtime.h>

template <int K>
__global__ __launch_bounds__(256) void chains(double *out, double x, int iters)
{
    double acc[K], y[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        acc[k] = threadIdx.x * 1e-9 + k;
        y[k] = 1.0 + k * 1e-7 + threadIdx.x * 1e-12;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = acc[k] + y[k] * x;
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += acc[k];
    if (s == 12345.678) out[threadIdx.x] = s;
}

template <int K> void run(double *d, int waves_per_simd)
{
    const int cus = 256, iters = 20000;
    const dim3 grid(cus * waves_per_simd), block(256); // 4 waves per block = one per SIMD
    hipLaunchKernelGGL(chains<K>, grid, block, 0, 0, d, 0.999999, 100);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(chains<K>, grid, block, 0, 0, d, 0.999999, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double steps = (double)iters; // per chain, per wave
    const double ns_per_step = ms * 1e6 / steps;
    // VALU instructions per SIMD: waves_per_simd * K * 2 * iters
    const double instr_per_ns = (double)waves_per_simd * K * 2 * iters / (ms * 1e6);
    std::printf("{\"chains\": %d, \"waves_per_simd\": %d, \"ns_per_chained_step\": %.3f, \"valu_instr_per_ns_per_simd\": %.3f}\n",
                K, waves_per_simd, ns_per_step, instr_per_ns);
}

int main()
{
    double *d;
    hipMalloc(&d, 4096 * sizeof(double));
    for (int w : {1, 2, 4, 8}) {
        run<1>(d, w);
        run<2>(d, w);
        run<4>(d, w);
        run<8>(d, w);
    }
    hipFree(d);
    return 0;
}
