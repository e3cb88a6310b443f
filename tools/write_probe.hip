// Where does a small write fraction inside a saturating read stream cost its ~13%?
// (not part of the product; DESIGN.md section 4 "The ceiling is set by the writes").
//
// Every wave reads S KiB contiguous (1 KiB per step, 16 B per lane, nt loads, 4 in flight)
// per chunk and writes Wk KiB per chunk. Modes:
//   after  : store after the chunk, value depends on every load (the sweeps' epilogue)
//   first  : store before the chunk's loads, value independent of them
//   defer  : P chunks per wave; chunk c's store is issued after chunk c+1's first loads
//   lds    : like after, but each wave's result goes through LDS and the block's 4 waves
//            store 4 KiB contiguous (one wave) after a barrier
// Usage: write_probe [GiB] [S] [Wk]; one JSON line of read GB/s per mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef double dvec2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ dvec2 read_chunk(const dvec2 *q, int S)
{
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
    return acc;
}

// mode 0 after, 1 first, 3 none; P chunks per wave (contiguous chunk indices)
__global__ __launch_bounds__(256) void wk_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out, int nchunks,
                                                 int S, int Wk, int mode, int P, double *sink)
{
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    dvec2 keep = {0, 0};
    for (int i = 0; i < P; ++i) {
        const int c = wave * P + i;
        if (c >= nchunks) break;
        dvec2 *o = out + (size_t)c * Wk * 64 + lane;
        if (mode == 1)
            for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(dvec2{(double)lane, (double)w}, o + (size_t)w * 64);
        const dvec2 acc = read_chunk(p + (size_t)c * S * 64 + lane, S);
        if (mode == 0)
            for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(acc, o + (size_t)w * 64);
        keep += acc;
    }
    if (mode == 3 && keep.x == 123.456) *sink = keep.y;
}

// deferred: the store of chunk c goes out after chunk c+1 is read
__global__ __launch_bounds__(256) void defer_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out, int nchunks,
                                                    int S, int Wk, int P)
{
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    dvec2 pend = {0, 0};
    int pc = -1;
    for (int i = 0; i < P; ++i) {
        const int c = wave * P + i;
        if (c >= nchunks) break;
        const dvec2 acc = read_chunk(p + (size_t)c * S * 64 + lane, S);
        if (pc >= 0) {
            dvec2 *o = out + (size_t)pc * Wk * 64 + lane;
            for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(pend, o + (size_t)w * 64);
        }
        pend = acc;
        pc = c;
    }
    if (pc >= 0) {
        dvec2 *o = out + (size_t)pc * Wk * 64 + lane;
        for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(pend, o + (size_t)w * 64);
    }
}

// block-gathered: 4 waves' Wk KiB each go out as one block-contiguous 4*Wk KiB run, all lanes storing
__global__ __launch_bounds__(256) void lds_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out, int nchunks,
                                                  int S, int Wk)
{
    __shared__ dvec2 buf[4 * 64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int c = blockIdx.x * 4 + wv;
    dvec2 acc = {0, 0};
    if (c < nchunks) acc = read_chunk(p + (size_t)c * S * 64 + lane, S);
    buf[threadIdx.x] = acc;
    __syncthreads();
    dvec2 *o = out + (size_t)blockIdx.x * 4 * Wk * 64;
    for (int w = 0; w < Wk; ++w)
        __builtin_nontemporal_store(buf[threadIdx.x], o + (size_t)w * 256 + threadIdx.x);
}

// time-windowed: stores are held until the chip-wide clock (s_memrealtime, 100 MHz) is inside the
// first W ticks of every T-tick period, so all CUs write in the same short windows
__global__ __launch_bounds__(256) void window_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out,
                                                     int nchunks, int S, int Wk, int P, unsigned T, unsigned W)
{
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    dvec2 pend = {0, 0};
    int pc = -1;
    auto flush = [&]() {
        dvec2 *o = out + (size_t)pc * Wk * 64 + lane;
        for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(pend, o + (size_t)w * 64);
        pc = -1;
    };
    for (int i = 0; i < P; ++i) {
        const int c = wave * P + i;
        if (c >= nchunks) break;
        const dvec2 *q = p + (size_t)c * S * 64 + lane;
        dvec2 acc = {0, 0};
        int s = 0;
        for (; s + 4 <= S; s += 4) {
            dvec2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(q + (size_t)(s + u) * 64);
            if (pc >= 0 && (unsigned)(__builtin_amdgcn_s_memrealtime() % T) < W) flush();
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += v[u];
        }
        for (; s < S; ++s) acc += __builtin_nontemporal_load(q + (size_t)s * 64);
        if (pc >= 0) flush(); // a second result is ready: no queue, write the older one now
        pend = acc;
        pc = c;
    }
    if (pc >= 0) flush();
}

// P = 1 with waiting: a wave that has read its chunk sleeps until the next write window
__global__ __launch_bounds__(256) void wait_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out,
                                                   int nchunks, int S, int Wk, unsigned T, unsigned W)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const dvec2 acc = read_chunk(p + (size_t)c * S * 64 + lane, S);
    while ((unsigned)(__builtin_amdgcn_s_memrealtime() % T) >= W) __builtin_amdgcn_s_sleep(16);
    dvec2 *o = out + (size_t)c * Wk * 64 + lane;
    for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(acc, o + (size_t)w * 64);
}

// wait_kernel plus reads paused inside the windows: a wave about to issue a group of loads while
// the window is open sleeps until it closes, so windows carry (almost) only writes
__global__ __launch_bounds__(256) void pause_kernel(const dvec2 *__restrict__ p, dvec2 *__restrict__ out,
                                                    int nchunks, int S, int Wk, unsigned T, unsigned W)
{
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const dvec2 *q = p + (size_t)c * S * 64 + lane;
    dvec2 acc = {0, 0};
    for (int s = 0; s + 4 <= S; s += 4) {
        while ((unsigned)(__builtin_amdgcn_s_memrealtime() & (T - 1)) < W) __builtin_amdgcn_s_sleep(4);
        dvec2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(q + (size_t)(s + u) * 64);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    while ((unsigned)(__builtin_amdgcn_s_memrealtime() & (T - 1)) >= W) __builtin_amdgcn_s_sleep(16);
    dvec2 *o = out + (size_t)c * Wk * 64 + lane;
    for (int w = 0; w < Wk; ++w) __builtin_nontemporal_store(acc, o + (size_t)w * 64);
}

int main(int argc, char **argv)
{
    const size_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 8;
    const int S = argc > 2 ? atoi(argv[2]) : 129;
    const int Wk = argc > 3 ? atoi(argv[3]) : 1;
    const size_t bytes = gib << 30;
    const int nchunks = (int)(bytes / ((size_t)S * 1024)) / 64 * 64;
    dvec2 *a, *wout;
    double *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&wout, (size_t)nchunks * Wk * 1024 + 4096));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(a, 0x3f, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 7; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return (double)nchunks * S * 1024 / (ts[3] * 1e-3) / 1e9;
    };
    printf("{\"gib\": %zu, \"S_kib\": %d, \"Wk_kib\": %d", gib, S, Wk);
    for (int P : {1, 2, 4}) {
        const int waves = (nchunks + P - 1) / P;
        const int blocks = (waves + 3) / 4;
        printf(", \"none_P%d\": %.1f", P, timeit([&] {
            hipLaunchKernelGGL(wk_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, 3, P, sink);
        }));
        printf(", \"after_P%d\": %.1f", P, timeit([&] {
            hipLaunchKernelGGL(wk_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, 0, P, sink);
        }));
        printf(", \"first_P%d\": %.1f", P, timeit([&] {
            hipLaunchKernelGGL(wk_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, 1, P, sink);
        }));
        if (P > 1)
            printf(", \"defer_P%d\": %.1f", P, timeit([&] {
                hipLaunchKernelGGL(defer_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, P);
            }));
    }
    printf(", \"lds_block\": %.1f", timeit([&] {
        hipLaunchKernelGGL(lds_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, 0, a, wout, nchunks, S, Wk);
    }));
    // reads and writes as separate launches: the same bytes, no interleaving
    const int blocks1 = (nchunks + 3) / 4;
    printf(", \"split_launches\": %.1f", timeit([&] {
        hipLaunchKernelGGL(wk_kernel, dim3(blocks1), dim3(256), 0, 0, a, wout, nchunks, S, Wk, 3, 1, sink);
        hipLaunchKernelGGL(wk_kernel, dim3(blocks1), dim3(256), 0, 0, a, wout, nchunks, 0, Wk, 1, 1, sink);
    }));
    for (unsigned T : {2048u, 4096u})
        for (unsigned W : {32u, 64u, 128u}) {
            printf(", \"pause_T%u_W%u\": %.1f", T, W, timeit([&] {
                hipLaunchKernelGGL(pause_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, 0, a, wout, nchunks, S, Wk, T, W);
            }));
        }
    for (unsigned T : {2048u, 4096u, 8192u})
        for (unsigned W : {32u, 64u, 128u, 256u, 512u}) {
            printf(", \"wait_T%u_W%u\": %.1f", T, W, timeit([&] {
                hipLaunchKernelGGL(wait_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, 0, a, wout, nchunks, S, Wk, T, W);
            }));
        }
    for (int P : {2, 4}) {
        const int blocks = ((nchunks + P - 1) / P + 3) / 4;
        for (unsigned T : {8192u, 16384u, 32768u})
            for (unsigned W : {T / 16, T / 8}) {
                printf(", \"win_P%d_T%u_W%u\": %.1f", P, T, W, timeit([&] {
                    hipLaunchKernelGGL(window_kernel, dim3(blocks), dim3(256), 0, 0, a, wout, nchunks, S, Wk, P, T, W);
                }));
            }
    }
    printf("}\n");
    return 0;
}
