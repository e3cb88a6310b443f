// Read-bandwidth probe for the sweeps' access pattern (not part of the product).
//
//   chunk : every wave streams its own contiguous chunk of S KiB (1 KiB per step,
//           16 B per lane, U steps in flight) - the current strip-tap-major layout,
//           where a (strip, row) tile's (2N+1) taps are contiguous;
//   ilv G : groups of G consecutive waves interleave their chunks step by step, so
//           step s of the G waves is one contiguous G KiB run (a tap-interleaved layout);
//   front : grid-stride over the whole buffer (tools/hbm_probe's pattern).
// Prints one JSON line of GB/s per pattern. Usage: pattern_probe [GiB] [S]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <algorithm>

typedef double dvec2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// chunk c of S steps; step s of chunk c lives at (G == 0) c*S*64 + s*64, else
// group (c / G), member g = c % G: (c/G)*S*G*64 + (s*G + g)*64.
template <int U>
__global__ __launch_bounds__(256) void chunk_kernel(const dvec2 *__restrict__ p, int nchunks, int S, int G,
                                                    double *sink)
{
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    dvec2 acc = {0, 0};
    for (int c = wave; c < nchunks; c += nw) {
        size_t base;
        size_t step;
        if (G == 0) {
            base = (size_t)c * S * 64;
            step = 64;
        } else {
            base = (size_t)(c / G) * S * G * 64 + (size_t)(c % G) * 64;
            step = (size_t)G * 64;
        }
        const dvec2 *q = p + base + lane;
        int s = 0;
        for (; s + U <= S; s += U) {
            dvec2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(q + (size_t)(s + u) * step);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
        for (; s < S; ++s) acc += __builtin_nontemporal_load(q + (size_t)s * step);
    }
    if (acc.x == 123.456 && acc.y == 654.321) *sink = acc.x;
}

// chunk pattern (G = 0, U = 4) plus Wk 1-KiB writes per wave after its chunk (output runs
// contiguous in chunk order), to price a small write fraction inside a read stream.
__global__ __launch_bounds__(256) void chunk_write_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out,
                                                          int nchunks, int S, int Wk, int nt_store)
{
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    for (int c = wave; c < nchunks; c += nw) {
        const dvec2 *q = p + (size_t)c * S * 64 + lane;
        dvec2 acc = {0, 0};
        int s = 0;
        for (; s + 4 <= S; s += 4) {
            dvec2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(q + (size_t)(s + u) * 64);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += v[u];
        }
        for (; s < S; ++s) acc += __builtin_nontemporal_load(q + (size_t)s * 64);
        dvec2 *o = out + (size_t)c * Wk * 64 + lane;
        for (int w = 0; w < Wk; ++w) {
            if (nt_store) __builtin_nontemporal_store(acc, o + (size_t)w * 64);
            else o[(size_t)w * 64] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void front_kernel(const dvec2 *__restrict__ p, size_t n, double *sink)
{
    dvec2 acc = {0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride * 4) {
        dvec2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t k = i + u * stride;
            v[u] = k < n ? __builtin_nontemporal_load(p + k) : dvec2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    if (acc.x == 123.456 && acc.y == 654.321) *sink = acc.x;
}

int main(int argc, char **argv)
{
    const size_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 8;
    const int S = argc > 2 ? atoi(argv[2]) : 103; // c3's mean 2N+1
    const size_t bytes = gib << 30;
    // whole groups only (G <= 64): the last chunk's last step ends at nchunks*S KiB <= bytes
    const int nchunks = (int)(bytes / ((size_t)S * 1024)) / 64 * 64;
    if (nchunks < 64 || (size_t)nchunks * S * 1024 > bytes) { fprintf(stderr, "bad sizes\n"); return 1; }
    dvec2 *a;
    double *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(a, 0x3f, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return (double)nchunks * S * 1024 / (ts[2] * 1e-3) / 1e9;
    };
    const int blocks = (nchunks + 3) / 4;
    printf("{\"gib\": %zu, \"S_kib\": %d", gib, S);
    printf(", \"front\": %.1f", timeit([&] {
        hipLaunchKernelGGL(front_kernel, dim3(8192), dim3(256), 0, 0, a, (size_t)nchunks * S * 64, sink);
    }));
    for (int U : {2, 4, 8}) {
        for (int G : {0, 4, 16, 64}) {
            auto go = [&] {
                if (U == 2) hipLaunchKernelGGL(chunk_kernel<2>, dim3(blocks), dim3(256), 0, 0, a, nchunks, S, G, sink);
                if (U == 4) hipLaunchKernelGGL(chunk_kernel<4>, dim3(blocks), dim3(256), 0, 0, a, nchunks, S, G, sink);
                if (U == 8) hipLaunchKernelGGL(chunk_kernel<8>, dim3(blocks), dim3(256), 0, 0, a, nchunks, S, G, sink);
            };
            printf(", \"U%d_G%d\": %.1f", U, G, timeit(go));
        }
    }
    // small write fractions inside the read stream (per wave: S KiB read, Wk KiB written)
    dvec2 *wout;
    CK(hipMalloc(&wout, (size_t)nchunks * 4 * 1024));
    for (int Wk : {0, 1, 2, 4}) {
        for (int nt : {0, 1}) {
            if (Wk == 0 && nt) continue;
            auto go = [&] {
                hipLaunchKernelGGL(chunk_write_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, nt);
            };
            const double rd = timeit(go); // GB/s of the read bytes alone
            printf(", \"W%d%s_read_GBps\": %.1f", Wk, nt ? "nt" : "", rd);
        }
    }
    printf("}\n");
    return 0;
}
