// HIP kernels (gfx950 / CDNA4) for DIGITAL_FILTER::filter(dt)
// (reference: digital-filtering-c++/df/df.cpp:332-485).
//
//   K0 expand_coeffs   per-N coefficient table -> strip-tap-major By/Bz   (setup)
//   K1 rng_count       pcg32 + polar accept flags, per-block accept counts
//   K2 rng_scan        exclusive scan of block counts (global accept ranks)
//   K3 rng_generate    normals in the reference's stream order -> ry, rz halo
//   K4 ypass           y-convolution (df.cpp:359-383), R rows per wave in registers
//   K5 zpass_epilogue  z-convolution (df.cpp:385-405) fused with correlate
//                      (408-417), RST scaling (419-447) and SRA T'/rho' (470-485)
//   K6 halo pack/unpack  z-halo columns for the multi-GPU strip exchange
//
// All FP64 and built with -ffp-contract=off: every product and sum rounds on its
// own, in the reference's order, so the sweeps are bit-exact given equal noise.
#include <type_traits>

#include "df_kernels.hpp"
#include "df_rng.hpp"

namespace dfamd {

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }


typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(3))) dvec2 *lds_pair_ptr; // LDS-staged noise (ds_read_b128)
__device__ __forceinline__ double2 ld_pair(const double2 *p) { return *p; }
__device__ __forceinline__ double2 ld_pair(lds_pair_ptr p)
{
    const dvec2 v = *p;
    return make_double2(v.x, v.y);
}

// Coefficient stream load: read once per call, so optionally non-temporal.
template <bool NT> __device__ __forceinline__ double2 ldB(const double *p)
{
    if (NT) {
        const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2 *>(p));
        return make_double2(v.x, v.y);
    }
    return *reinterpret_cast<const double2 *>(p);
}

// ------------------------------------------------------------------ K0 setup

// Zero taps keep the reference's sum bit for bit: before a cell's first tap the sum
// is +0 and +0 + (+-0) = +0; after its last tap x + (+-0) = x.
__global__ __launch_bounds__(256) void expand_coeffs_kernel(double *__restrict__ B,
                                                            const long long *__restrict__ off,
                                                            const int *__restrict__ N_st,
                                                            const int *__restrict__ N_cell,
                                                            const double *__restrict__ tab,
                                                            const int *__restrict__ tab_off, int Ny,
                                                            int Nz_loc)
{
    const int sj = blockIdx.x; // s * Ny + j
    const int s = sj / Ny, j = sj - s * Ny;
    const int N = N_st[sj];
    double *dst = B + off[sj];
    const int total = (2 * N + 1) * kStrip;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int t = e / kStrip, cell = e - t * kStrip;
        const int i = t - N, ai = i < 0 ? -i : i;
        const int k = s * kStrip + cell;
        double v = 0.0;
        if (k < Nz_loc) {
            const int Nc = N_cell ? N_cell[(size_t)j * Nz_loc + k] : N;
            if (ai <= Nc) v = tab[tab_off[Nc] + ai];
        }
        dst[e] = v;
    }
}

hipError_t launch_expand_coeffs(double *B, const long long *off, const int *N_st, const int *N_cell,
                                const double *tab, const int *tab_off, int Ny, int nstrips, int Nz_loc,
                                hipStream_t st)
{
    hipLaunchKernelGGL(expand_coeffs_kernel, dim3((unsigned)nstrips * Ny), dim3(256), 0, st, B, off, N_st,
                       N_cell, tab, tab_off, Ny, Nz_loc);
    return hipGetLastError();
}

// ---------------------------------------------------------------- K1-K3 RNG
//
// Attempt t (0-based within the call) consumes pcg32 outputs 4t..4t+3 of the
// stream that starts at the call's state S. Block b owns attempts
// [b*4096, (b+1)*4096); wave w of the block owns the contiguous run
// b*4096 + w*1024 + [0, 1024) and lane l handles b*4096 + w*1024 + m*64 + l,
// m = 0..15. Consecutive lanes hold consecutive attempts, so a wave's accepted
// attempts map to consecutive stream positions (coalesced stores), and a wave's
// whole run covers one contiguous stream range it can test once (K3).

// State at the thread's first attempt, advance(S, 4*(b*4096 + w*1024 + l)), as two
// affine steps from host-built jump tables (pcg_random.hpp:639-662 composed).
__device__ __forceinline__ uint64_t thread_first_state(const RngGeom &g, uint64_t S, int b, int tid)
{
    const PcgJumpDev jb = g.jump_block[b], jt = g.jump_thread[tid];
    return jt.mult * (jb.mult * S + jb.plus) + jt.plus;
}

// The accept flags of thread tid of attempt block gb (bit m: its attempt m), from the call's start state S.
// The screen reads outputs 1 and 3 of each attempt only: the lane walks the states one and three steps
// into its attempts directly, each with one 64-bit multiply-add per attempt (J s + P_k, the 256-step jump
// conjugated: J and the step commute), instead of the attempt start plus two steps.
__device__ __forceinline__ uint32_t lane_accept_bits(const RngGeom &g, uint64_t S, int gb, int tid)
{
    const uint64_t st0 = thread_first_state(g, S, gb, tid);
    uint64_t s1 = st0 * kPcgMult + kPcgInc;
    uint64_t s3 = s1 * kPcgMult2 + kPcgInc2;
    uint32_t bits = 0, unsure = 0;
#pragma unroll 4
    for (int m = 0; m < kRngPerThread; ++m) {
        const int v = polar_screen13(s1, s3);
        bits |= (v > 0 ? 1u : 0u) << m;
        unsure |= (v < 0 ? 1u : 0u) << m;
        s1 = g.next_mult * s1 + g.next_plus1; // the lane's next attempt, 64 attempts on
        s3 = g.next_mult * s3 + g.next_plus3;
    }
    // ~2e-5 of the attempts: the exact double test of polar_attempt (random.tcc:1822-1826)
    while (unsure) {
        const int m = __builtin_ctz(unsure);
        unsure &= unsure - 1;
        uint64_t s = st0;
        for (int k = 0; k < m; ++k) s = g.next_mult * s + g.next_plus;
        if (polar_attempt(s).accept) bits |= 1u << m;
    }
    return bits;
}

// Counts blocks [b0, b0 + gridDim.x) of the call; blocks >= nb_total (padding of
// the last z-strip rank's share) report zero.
// Blocks [b0, b0 + nb) of the call, one workgroup each (the loop strides only if a grid smaller than nb
// caps how many K1 waves are resident beside the sweeps; 0 = one block per attempt block).
__global__ __launch_bounds__(kRngThreads) void rng_count_kernel(RngGeom g, const RngStateDev *__restrict__ sin,
                                                               int *__restrict__ counts, int *__restrict__ wave_counts,
                                                               uint16_t *__restrict__ masks, int b0, int nb, int nb_total)
{
    __shared__ int wsum[kRngThreads / 64];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int gb = b0 + blockIdx.x; gb < b0 + nb; gb += gridDim.x) { // block-uniform trip count
        if (gb >= nb_total) {
            if (tid == 0) counts[gb] = 0;
            if (tid < kRngThreads / 64) wave_counts[(size_t)gb * (kRngThreads / 64) + tid] = 0;
            if (g.xbuf && tid < 64) {
                const int sh = gb / g.xchunk;
                g.xbuf[(size_t)sh * g.xstride + (size_t)(gb - sh * g.xchunk) * 64 + tid] = 0;
            }
            continue;
        }
        const uint32_t bits = lane_accept_bits(g, sin->state, gb, tid);
        int cnt = __builtin_popcount(bits);
        masks[(size_t)gb * kRngThreads + tid] = (uint16_t)bits; // accept flags for K3
        if (g.xbuf) { // accepted attempts per group of 64 (one ballot each) into the share's record (run form)
            const int lane = tid & 63;
            int mine = 0;
#pragma unroll
            for (int m = 0; m < kRngPerThread; ++m) {
                const int n = __popcll(__ballot((bits >> m) & 1u));
                mine = lane == m ? n : mine;
            }
            const int sh = gb / g.xchunk;
            if (lane < kRngPerThread)
                g.xbuf[(size_t)sh * g.xstride + (size_t)(gb - sh * g.xchunk) * 64 + w * kRngPerThread + lane] = (uint8_t)mine;
        }
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        if ((tid & 63) == 0) {
            wsum[w] = cnt;
            wave_counts[(size_t)gb * (kRngThreads / 64) + w] = cnt; // the wave's run of 1024 attempts
        }
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int ww = 0; ww < kRngThreads / 64; ++ww) t += wsum[ww];
            counts[gb] = t;
        }
        __syncthreads(); // wsum is rewritten by the next iteration
    }
}

// K2: exclusive scan of the per-block accept counts in two levels, so no thread walks a long
// serial run (a single-block scan took 58 us for the 33k blocks of an 8-GPU plane):
// K2a scans each run of 1024 counts (4 per thread, wave shuffles + one LDS pass) into
// offsets[] and writes the run's total to part[]; K2b scans part[] in one block. A block's
// global offset is offsets[b] + part[b >> 10] (read by K3).
__global__ __launch_bounds__(256) void rng_scan_local_kernel(const int *__restrict__ counts,
                                                             long long *__restrict__ offsets,
                                                             long long *__restrict__ part, int nblocks)
{
    __shared__ long long wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int b0 = blockIdx.x * 1024 + tid * 4;
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = b0 + i < nblocks ? counts[b0 + i] : 0;
    const long long t = (long long)v[0] + v[1] + v[2] + v[3];
    long long x = t; // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    long long excl = x - t;
    for (int ww = 0; ww < w; ++ww) excl += wsum[ww];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (b0 + i < nblocks) offsets[b0 + i] = excl;
        excl += v[i];
    }
    if (tid == 255) part[blockIdx.x] = excl; // run total
}

__global__ __launch_bounds__(1024) void rng_scan_parts_kernel(long long *__restrict__ part, int nparts,
                                                              const RngStateDev *__restrict__ sin, uint64_t Q,
                                                              int *__restrict__ err, int *__restrict__ ntasks)
{
    __shared__ long long p[1024];
    const int tid = threadIdx.x;
    if (tid == 0) *ntasks = 0; // K2c appends this call's wave tasks
    p[tid] = tid < nparts ? part[tid] : 0;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const long long v = tid >= o ? p[tid - o] : 0;
        __syncthreads();
        p[tid] += v;
        __syncthreads();
    }
    if (tid < nparts) part[tid] = tid ? p[tid - 1] : 0;
    if (tid == 1023) {
        const uint64_t f = (uint64_t)sin->saved_flag;
        const long long A = (long long)((Q - f + 1) / 2);
        if (p[1023] < A) *err = 1; // not enough attempts launched: host re-sizes
    }
}


// A stream position q as (array, row, column) of the reference's six arrays.
struct StreamPos {
    int sidx;
    uint32_t row, col;
};

template <class G> __device__ __forceinline__ StreamPos stream_pos(const G &g, uint64_t q)
{
    int sidx = 0;
#pragma unroll
    for (int s = 1; s < 6; ++s) sidx += (q >= g.seg[s]) ? 1 : 0;
    const uint32_t p = (uint32_t)(q - g.seg[sidx]);
    const uint32_t W = g.width[sidx];
    const uint32_t row = (W == 1) ? p : (uint32_t)__umul64hi((uint64_t)p, g.inv_width[sidx]);
    return {sidx, row, p - row * W};
}

// Position d normals further on (wave-uniform, SALU): at most two row steps when rows hold
// >= 128 normals and d <= 128; sidx == 6 means past the end of the call's stream.
template <class G> __device__ __forceinline__ StreamPos stream_advance(const G &g, StreamPos s, uint32_t d)
{
    while (d > 0 && s.sidx < 6) {
        const uint32_t room = g.width[s.sidx] - s.col;
        if (d < room) {
            s.col += d;
            break;
        }
        d -= room;
        s.col = 0;
        if (++s.row == g.rows[s.sidx]) {
            s.row = 0;
            ++s.sidx;
        }
    }
    return s;
}

template <class G> __device__ __forceinline__ StreamPos stream_next(const G &g, StreamPos s)
{
    if (++s.col == g.width[s.sidx]) {
        s.col = 0;
        if (++s.row == g.rows[s.sidx]) {
            s.row = 0;
            ++s.sidx;
        }
    }
    return s;
}

// Destination in this GPU's buffers, or nullptr if the reference draws that
// normal but this GPU never reads it (the r_zs interior, which df.cpp:377
// overwrites; columns owned by other GPUs).
template <class G> __device__ __forceinline__ double *stream_dest(const G &g, StreamPos s)
{
    const int c = s.sidx >> 1;
    const int col = (int)s.col;
    if ((s.sidx & 1) == 0) { // r_ys: Nz_g columns per row
        if (col < g.yz0 || col >= g.yz1) return nullptr;
        return g.ry[c] + (size_t)s.row * g.Pz + (col - g.yz0);
    }
    int lc;
    if (col < g.Nzp[c]) {
        if (!g.is_first) return nullptr;
        lc = col;
    } else if (col >= g.Nzp[c] + g.Nz_g) {
        if (!g.is_last) return nullptr;
        lc = col - g.z0;
    } else {
        return nullptr;
    }
    return g.rz[c] + (size_t)s.row * g.rz_pitch[c] + lc;
}

// Does [a, b) (offsets inside one row-major array of rows of width W) hit a
// column in [c0, c1)?
__device__ __forceinline__ bool span_hits_cols(uint32_t a, uint32_t b, uint32_t W, uint32_t c0, uint32_t c1)
{
    if (c0 >= c1 || a >= b) return false;
    const uint32_t ra = a / W, rb = (b - 1) / W;
    const uint32_t ca = a - ra * W, cb = (b - 1) - rb * W;
    if (rb > ra + 1) return true; // a full row in between
    if (rb == ra) return ca < c1 && cb >= c0;
    return ca < c1 || cb >= c0; // [ca, W) then [0, cb]
}

// Does the stream range [q0, q1) hold a normal this GPU stores? (z-strips:
// blocks of attempts that only feed other GPUs' columns skip their pass 2.)
template <class G> __device__ bool range_needed(const G &g, uint64_t q0, uint64_t q1)
{
    for (int sidx = 0; sidx < 6; ++sidx) {
        const uint64_t lo = q0 > g.seg[sidx] ? q0 : g.seg[sidx];
        const uint64_t hi = q1 < g.seg[sidx + 1] ? q1 : g.seg[sidx + 1];
        if (lo >= hi) continue;
        const uint32_t a = (uint32_t)(lo - g.seg[sidx]), b = (uint32_t)(hi - g.seg[sidx]);
        const uint32_t W = g.width[sidx];
        if ((sidx & 1) == 0) {
            if (span_hits_cols(a, b, W, (uint32_t)g.yz0, (uint32_t)g.yz1)) return true;
        } else {
            const uint32_t nzp = (uint32_t)g.Nzp[sidx >> 1];
            if (g.is_first && span_hits_cols(a, b, W, 0, nzp)) return true;
            if (g.is_last && span_hits_cols(a, b, W, nzp + (uint32_t)g.Nz_g, W)) return true;
        }
    }
    return false;
}

// log(r2) of the polar transform (random.tcc:1831): 2 glibc's own log (bit-identical normals, the
// default), 1 the table-driven log_r2 (within 1 ulp), 0 the device library's log.
__device__ __forceinline__ double polar_log(const RngGeom &g, double r2)
{
    if (g.fast_log == 2) return glibc_log(r2);
    return g.fast_log ? log_r2(r2, g.log_tab) : log(r2);
}

// K2c: one thread per wave of attempts (4 per block). A wave's accepted attempts hold ranks
// [r_lo, r_hi) = block offset + the preceding waves' counts, i.e. stream positions
// [f + 2 r_lo, f + 2 r_hi). Waves that store something on this GPU (or end the call) are
// appended to a task list, so K3 never runs a wave that only feeds other strips or the r_zs
// interior. Also stores the cached normal carried into the call (stream position 0).
__global__ __launch_bounds__(256) void rng_plan_kernel(RngGeom g, const RngStateDev *__restrict__ sin,
                                                       const long long *__restrict__ offsets,
                                                       const long long *__restrict__ part,
                                                       const int *__restrict__ wave_counts, int nb_total,
                                                       WaveTask *__restrict__ tasks, int *__restrict__ ntasks)
{
    constexpr int WPB = kRngThreads / 64; // waves per attempt block
    const int gw = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
    const uint64_t f = (uint64_t)sin->saved_flag;
    const long long A = (long long)((g.Q - f + 1) / 2);
    if (gw == 0 && f) {
        double *d = stream_dest(g, stream_pos(g, 0));
        if (d) *d = sin->saved * 1.0 + 0.0;
    }
    bool need = false;
    long long r_lo = 0;
    if (gw < nb_total * WPB) {
        const int b = gw / WPB, w = gw % WPB;
        r_lo = offsets[b] + part[b >> 10];
        for (int ww = 0; ww < w; ++ww) r_lo += wave_counts[(size_t)b * WPB + ww];
        const long long r_hi = r_lo + wave_counts[gw];
        if (r_lo < A) {
            const uint64_t q_lo = f + 2ull * (uint64_t)r_lo;
            const uint64_t q_hi = (f + 2ull * (uint64_t)r_hi) < g.Q ? (f + 2ull * (uint64_t)r_hi) : g.Q;
            const bool ends_call = A - 1 < r_hi;
            need = ends_call || (q_lo < q_hi && range_needed(g, q_lo, q_hi));
        }
    }
    const uint64_t m = __ballot(need);
    if (!m) return;
    int base = 0;
    if (lane == 0) base = atomicAdd(ntasks, __popcll(m)); // one atomic per plan wave
    base = __shfl(base, 0);
    if (need) {
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        tasks[base + below] = WaveTask{r_lo, gw, 0};
    }
}

// K3, compacted form (planes without the dense generation). A sequential form (round 1) ran the
// transform (4 draws, log, sqrt, divide) in every iteration with the ~21% rejected lanes idle, and
// walked the stream position per iteration in scalar code. Here a wave first appends the state of each
// accepted attempt to a wave-private LDS ring, in rank order (slot k = the wave's k-th accepted attempt,
// stream positions q0 + 2k and q0 + 2k + 1), and every 4 iterations turns each full run of 64 slots into
// one batch with all 64 lanes busy. A batch covers 128 consecutive stream positions, so whether it stores
// anything on this GPU is one scalar range test; the r_zs interior (df.cpp:377) and other strips' columns
// are skipped a batch at a time. Same draws, same arithmetic, same destinations: bit-identical.
constexpr int kGenRing = 512; // slots per wave: < 64 carried + 4 iterations x 64 appended between flushes

// Wave-uniform lookups into the kernel argument's per-array tables as select chains over registers
// loaded once, instead of one scalar load with a computed offset per use.
template <class T, int K> __device__ __forceinline__ T sel(const T (&v)[K], int i)
{
    T r = v[0];
#pragma unroll
    for (int k = 1; k < K; ++k) r = (i == k) ? v[k] : r;
    return r;
}

// Where a wave's accepted attempts store (uniform, computed once per wave): all of its stream
// positions lie in array `su` starting at (row, col) unless `generic` (the run crosses an array end or
// the rows are narrower than a batch: per-lane table lookups then). Columns this GPU stores: [lo1, hi1)
// at local column col + o1 and [lo2, W) at col + o2 (r_ys: this strip's columns; r_zs: the plane-edge
// pads, df.cpp:343-348; the r_zs interior, which df.cpp:377 overwrites, never).
struct WaveDest {
    double *base;
    size_t pitch;
    uint32_t W, row, col, lo1, hi1, lo2;
    int o1, o2;
    bool generic;
};

__device__ __forceinline__ WaveDest wave_dest(const RngGeom &g, uint64_t q_lo, uint64_t n_pos)
{
    WaveDest w{};
    const StreamPos P = stream_pos(g, q_lo);
    const int su = P.sidx < 6 ? P.sidx : 5;
    w.W = sel(g.width, su);
    const uint64_t left = (uint64_t)(sel(g.rows, su) - P.row) * w.W - P.col;
    w.generic = P.sidx >= 6 || w.W < 2 * 64 || n_pos > left;
    const int cmp = su >> 1;
    const bool odd = su & 1;
    const uint32_t nzp = (uint32_t)sel(g.Nzp, cmp);
    w.base = odd ? sel(g.rz, cmp) : sel(g.ry, cmp);
    w.pitch = odd ? (size_t)sel(g.rz_pitch, cmp) : (size_t)g.Pz;
    w.row = P.row;
    w.col = P.col;
    w.lo1 = odd ? 0u : (uint32_t)g.yz0;
    w.hi1 = odd ? (g.is_first ? nzp : 0u) : (uint32_t)g.yz1;
    w.lo2 = odd && g.is_last ? nzp + (uint32_t)g.Nz_g : w.W;
    w.o1 = odd ? 0 : -g.yz0;
    w.o2 = -g.z0;
    return w;
}

// One batch: ring slots [head, head + n) hold the states of the wave's accepted attempts of ranks
// rk + (0..n-1) (rk uniform), stream positions qw + 2 * (head + lane) from the wave's first one qw.
__device__ __forceinline__ void gen_batch(const RngGeom &g, const WaveDest &w, const uint64_t *ring, int head, int n,
                                          long long rk, uint64_t qw, uint64_t f, long long A,
                                          RngStateDev *__restrict__ sout, int lane)
{
    const long long rank = rk + lane;
    const bool live = lane < n && rank < A;
    double *d0 = nullptr, *d1 = nullptr;
    if (live) {
        if (!w.generic) { // a few row wraps at most: the wave's run spans < 2048 positions, rows >= 128
            uint32_t col = w.col + 2u * (uint32_t)(head + lane);
            double *r = w.base + (size_t)w.row * w.pitch;
            while (col >= w.W) {
                col -= w.W;
                r += w.pitch;
            }
            uint32_t col1 = col + 1;
            double *r1 = r;
            if (col1 == w.W) {
                col1 = 0;
                r1 += w.pitch;
            }
            auto dest = [&](double *rowp, uint32_t cc) -> double * {
                if (cc >= w.lo1 && cc < w.hi1) return rowp + ((int)cc + w.o1);
                if (cc >= w.lo2) return rowp + ((int)cc + w.o2);
                return nullptr;
            };
            d0 = dest(r, col);
            d1 = dest(r1, col1);
        } else {
            const uint64_t q0 = qw + 2ull * (uint64_t)(head + lane);
            const StreamPos p0 = stream_pos(g, q0); // rare: per-lane table lookups
            d0 = stream_dest(g, p0);
            d1 = (q0 + 1 < g.Q) ? stream_dest(g, stream_next(g, p0)) : nullptr;
        }
    }
    const bool last = live && rank == A - 1;
    if (!(d0 || d1 || last)) return; // the whole batch leaves at once where nothing is stored here
    const uint64_t st = ring[(head + lane) & (kGenRing - 1)];
    uint64_t s3 = st;
    PolarAttempt a;
    if (g.debug_flags & 4) {
        a.x = (double)(uint32_t)st * 1e-10;
        a.y = 0.5;
        a.r2 = 0.5;
        s3 = st + 3;
    } else {
        a = polar_draws(st, s3); // the draws K1 tested; the fourth step only for the call's last attempt
    }
    const double mult = (g.debug_flags & 1) ? a.r2 : sqrt(-2 * polar_log(g, a.r2) / a.r2);
    const double xm = a.x * mult;
    const double ym = a.y * mult;
    const double n0 = ym * 1.0 + 0.0, n1 = xm * 1.0 + 0.0;
    if (g.debug_flags & 2) {
        if (n0 == 1234.5) *d0 = n1; // keep the values alive
    } else if (d0 && d1 == d0 + 1 && ((uintptr_t)d0 & 15) == 0) {
        if (g.nt_stores) __builtin_nontemporal_store(dvec2{n0, n1}, reinterpret_cast<dvec2 *>(d0));
        else *reinterpret_cast<double2 *>(d0) = make_double2(n0, n1);
    } else {
        if (d0) *d0 = n0;
        if (d1) *d1 = n1;
    }
    if (last) {
        sout->state = s3 * kPcgMult + kPcgInc; // state after this attempt's 4th output
        sout->saved_flag = (int)((g.Q - f) & 1u);
        sout->saved = xm;
    }
}

__global__ __launch_bounds__(kRngThreads) void rng_generate_compact_kernel(RngGeom g,
                                                                          const RngStateDev *__restrict__ sin,
                                                                          RngStateDev *__restrict__ sout,
                                                                          const WaveTask *__restrict__ tasks,
                                                                          const int *__restrict__ ntasks,
                                                                          const uint16_t *__restrict__ masks,
                                                                          const int *__restrict__ counts_in,
                                                                          const int *__restrict__ wave_counts_in,
                                                                          int *__restrict__ err)
{
    __shared__ uint64_t ring_all[kRngThreads / 64][kGenRing];
    const int lane = threadIdx.x & 63;
    uint64_t *ring = ring_all[threadIdx.x >> 6];
    const int split = g.gen_split;
    const int vslot = uniform(blockIdx.x * (kRngThreads / 64) + (threadIdx.x >> 6));
    const int slot = vslot / split, sub = vslot - slot * split;
    const uint64_t f = (uint64_t)sin->saved_flag;
    const long long A = (long long)((g.Q - f + 1) / 2);
    int gw;
    long long rank_w; // uniform
    if (g.fused_plan) {
        // Small planes (g.fused_plan: one GPU, <= 1024 attempt blocks): no scan or plan launch. The wave
        // is attempt wave `slot`; it sums the accept counts before it (<= 1024 block counts, then its
        // block's earlier waves) for its first rank, and leaves if it stores nothing here - the same
        // ranks and the same test as K2 + K2c (rng_scan_plan_small_kernel), so the same bits.
        constexpr int WPB = kRngThreads / 64;
        const int nw = g.nb_plan * WPB;
        if (slot >= nw) return;
        gw = slot;
        const int b = gw / WPB, w = gw - b * WPB;
        long long v = 0;
        for (int i = lane; i < b; i += 64) v += counts_in[i];
        if (lane < w) v += wave_counts_in[(size_t)b * WPB + lane];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        rank_w = v;
        if (vslot == 0) { // once per call: the attempt-shortage check and the cached normal at position 0
            long long t = 0;
            for (int i = lane; i < g.nb_plan; i += 64) t += counts_in[i];
            for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
            if (lane == 0) {
                if (t < A) *err = 1; // not enough attempts launched (as K2)
                if (f) {
                    double *d = stream_dest(g, stream_pos(g, 0));
                    if (d) *d = sin->saved * 1.0 + 0.0;
                }
            }
        }
        const long long r_hi = rank_w + wave_counts_in[gw];
        if (rank_w >= A) return;
        const uint64_t q_lo = f + 2ull * (uint64_t)rank_w;
        const uint64_t q_hi = min(f + 2ull * (uint64_t)r_hi, (uint64_t)g.Q);
        const bool need = (A - 1 < r_hi) || (q_lo < q_hi && range_needed(g, q_lo, q_hi));
        if (!need) return;
    } else {
        if (slot >= *ntasks) return;
        gw = uniform(tasks[slot].gw);
        rank_w = tasks[slot].r_lo;
    }
    const int b = gw / (kRngThreads / 64), tid = (gw % (kRngThreads / 64)) * 64 + lane;
    // split counting: only counts were exchanged, so the flags of another rank's blocks are recomputed
    const uint32_t bits = g.recount ? lane_accept_bits(g, sin->state, b, tid) : masks[(size_t)b * kRngThreads + tid];
    uint64_t st = thread_first_state(g, sin->state, b, tid);
    const int per = kRngPerThread / split, m0 = sub * per, m1 = m0 + per;
    for (int m = 0; m < m0; ++m) {
        st = g.next_mult * st + g.next_plus;
        rank_w += __popcll(__ballot((bits >> m) & 1u));
    }
    const long long rank0 = rank_w; // rank of ring slot 0
    int tail = 0, head = 0;         // uniform
    // this wave's positions: [qw, qw + 2 * (accepted attempts in iterations m0..m1-1)), within the call
    const uint64_t qw = f + 2ull * (uint64_t)(rank0 < A ? rank0 : 0);
    uint32_t nacc = 0;
    for (int m = m0; m < m1; ++m) nacc += (uint32_t)__popcll(__ballot((bits >> m) & 1u));
    const uint64_t q_end = min(qw + 2ull * nacc, (uint64_t)g.Q);
    const WaveDest wd = wave_dest(g, qw, q_end > qw ? q_end - qw : 0);
    for (int m = m0; m < m1; ++m) {
        const bool acc = (bits >> m) & 1u;
        const uint64_t mask = __ballot(acc);
        if (acc) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            ring[(tail + below) & (kGenRing - 1)] = st;
        }
        tail += __popcll(mask);
        st = g.next_mult * st + g.next_plus;
        const bool fin = m == m1 - 1;
        if (fin || ((m - m0) & 3) == 3) {
            // the ring is wave-private and LDS ops of one wave complete in order: only the compiler
            // must not move the reads above the appends
            __asm__ volatile("" ::: "memory");
            while (tail - head >= 64 || (fin && tail > head)) {
                const int n = min(64, tail - head);
                const long long rk = rank0 + head;
                if (rk < A && !(g.debug_flags & 8)) gen_batch(g, wd, ring, head, n, rk, qw, f, A, sout, lane);
                head += n;
            }
            __asm__ volatile("" ::: "memory");
        }
    }
}

// ---------------------------------------------------------------- chunk generation (run generation)
//
// The compacted K3 above spends more time in its per-wave skeleton (ring appends, batch loop, per-lane
// destination walk, mostly scalar and branch work: 29M SALU against 37M VALU per c3 table call) than in
// the transform. The run generation (K3r below) generates by 64-rank chunks instead: lane l of chunk c holds
// rank 64c + l, draws its attempt's four outputs, transforms and stores the pair at a destination computed
// by arithmetic (consecutive lanes, consecutive 16-B pairs). glibc's near-1 band (6.25% of r2, so present in
// 98% of 64-lane batches) is not evaluated in the chunk's batch: those lanes push (x, y, destinations) on a
// wave-private LDS stack, popped 64 at a time into batches of their own (the near-1 half of glibc_log
// alone), the rest at the wave's end. Same draws, same arithmetic (x*x + y*y and the log's band test
// recomputed bit for bit), same destinations as K3: bit-identical noise. (Round 3's two-kernel form of it -
// Kc compacting accepted states into memory, K3a one wave per 8 chunks - was removed in round 5: no plane
// selected it once K3r existed.)

__device__ __forceinline__ void store_pair(const RngGeom &g, double *d0, double *d1, double n0, double n1)
{
    if (g.debug_flags & 2) {
        if (n0 == 1234.5) *d0 = n1; // keep the values alive
    } else if (d0 && d1 == d0 + 1 && ((uintptr_t)d0 & 15) == 0) {
        if (g.nt_stores) __builtin_nontemporal_store(dvec2{n0, n1}, reinterpret_cast<dvec2 *>(d0));
        else *reinterpret_cast<double2 *>(d0) = make_double2(n0, n1);
    } else {
        if (d0) *d0 = n0;
        if (d1) *d1 = n1;
    }
}

// A deferred near-1 lane: its uniforms and its two destinations (nullptr: not stored here).
struct Near1Slot {
    double x, y;
    double *d0, *d1;
};

// Pop n <= 64 deferred near-1 lanes from the top of the wave's stack and finish them: x*x + y*y is
// polar_draws' r2 bit for bit, and every argument is in glibc's near-1 band.
__device__ __forceinline__ void near1_batch(const RngGeom &g, const Near1Slot *q, int top, int n, int lane)
{
    if (lane >= n) return;
    const Near1Slot e = q[top - n + lane];
    const double xx = e.x * e.x;
    const double yy = e.y * e.y;
    const double r2 = xx + yy;
    const double mult = (g.debug_flags & 1) ? r2 : sqrt(-2 * glibc_log_band1(r2) / r2);
    const double xm = e.x * mult;
    const double ym = e.y * mult;
    store_pair(g, e.d0, e.d1, ym * 1.0 + 0.0, xm * 1.0 + 0.0);
}


// One needed 64-rank chunk c of the dense generation: lane l holds rank 64 c + l, whose attempt starts at
// state s (any value for ranks past the call's end). di: the chunk's index in the host list (chunk_dest).
// Near-1 lanes go on the wave's LDS stack (top: its uniform height), batches of 64 are finished here.
// The fast-chunk descriptor of list entry di (arr -1: the general path).
__device__ __forceinline__ ChunkDest chunk_dest_of(const RngGeom &g, uint64_t f, int di)
{
    return g.chunk_dest[f] && !g.debug_flags ? g.chunk_dest[f][di] : ChunkDest{0, 0, 0, -1, 0, 0};
}

// Lane k's descriptor (held one per lane, K3r) as a uniform value: four v_readlane, no memory access.
__device__ __forceinline__ ChunkDest chunk_dest_lane(const ChunkDest &mine, int k)
{
    static_assert(sizeof(ChunkDest) == 16, "ChunkDest is read as four dwords");
    int w[4];
    __builtin_memcpy(w, &mine, 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_readlane(w[i], k);
    ChunkDest cd;
    __builtin_memcpy(&cd, w, 16);
    return cd;
}

__device__ __forceinline__ void dense_chunk(const RngGeom &g, uint64_t f, long long A, long long c, const ChunkDest cd,
                                            uint64_t s, int lane, bool defer, Near1Slot *stk, int &top,
                                            RngStateDev *__restrict__ sout)
{
    if (cd.arr >= 0) { // uniform
        // fast chunk (host-built ChunkDest): no lane is past the call or its last attempt, the stored positions
        // are one run [lo, hi) in one stream array with at most one row wrap - no stream position search
        const int ca = cd.arr >> 1;
        double *const arr = (cd.arr & 1) ? (ca == 0 ? g.rz[0] : ca == 1 ? g.rz[1] : g.rz[2])
                                         : (ca == 0 ? g.ry[0] : ca == 1 ? g.ry[1] : g.ry[2]);
        double *const base = arr + cd.off;
        const int e0 = 2 * lane, e1 = e0 + 1;
        double *const p0 = e0 >= cd.lo && e0 < cd.hi ? base + e0 + (e0 >= cd.wr ? cd.jump : 0) : nullptr;
        double *const p1 = e1 >= cd.lo && e1 < cd.hi ? base + e1 + (e1 >= cd.wr ? cd.jump : 0) : nullptr;
        const bool livef = p0 || p1;
        uint64_t s3f;
        const PolarAttempt af = polar_draws(s, s3f);
        const bool nearf = defer && livef && glibc_log_near1(af.r2);
        const uint64_t nmf = __ballot(nearf);
        if (nmf) {
            if (nearf) {
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(nmf >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)nmf, 0u));
                stk[top + below] = Near1Slot{af.x, af.y, p0, p1};
            }
            top += __popcll(nmf);
        }
        if (!nearf && livef) {
            const double lg = defer ? glibc_log_main(af.r2) : polar_log(g, af.r2);
            const double mult = sqrt(-2 * lg / af.r2);
            const double xm = af.x * mult;
            const double ym = af.y * mult;
            store_pair(g, p0, p1, ym * 1.0 + 0.0, xm * 1.0 + 0.0);
        }
    } else {
        const long long rank = c * 64 + lane;
        const uint64_t q = f + 2ull * (uint64_t)rank;
        const uint64_t q0 = f + 128ull * (uint64_t)c; // uniform
        const StreamPos P0 = stream_pos(g, q0);
        const int su = P0.sidx < 6 ? P0.sidx : 5;
        const uint32_t W = g.width[su];
        const bool generic = P0.sidx >= 6 || W < 128 || q0 + 128 > g.seg[su + 1];
        double *d0 = nullptr, *d1 = nullptr;
        const bool live = rank < A;
        if (live) {
            if (!generic) { // one array, at most one row wrap
                uint32_t row = P0.row, col = P0.col + 2u * (uint32_t)lane;
                if (col >= W) {
                    col -= W;
                    ++row;
                }
                d0 = stream_dest(g, StreamPos{su, row, col});
                if (++col == W) {
                    col = 0;
                    ++row;
                }
                d1 = stream_dest(g, StreamPos{su, row, col}); // q + 1 < the array's end
            } else {
                const StreamPos p0 = stream_pos(g, q);
                d0 = stream_dest(g, p0);
                d1 = (q + 1 < g.Q) ? stream_dest(g, stream_next(g, p0)) : nullptr;
            }
        }
        const bool last = live && rank == A - 1;
        const bool active = d0 || d1 || last;
        PolarAttempt a{};
        uint64_t s3 = s;
        bool near = false;
        if (active) {
            if (g.debug_flags & 4) {
                a.x = (double)(uint32_t)s * 1e-10;
                a.y = 0.5;
                a.r2 = 0.5;
            } else {
                a = polar_draws(s, s3); // the draws K1 tested; s3 left at the fourth output's state
            }
            // the call's last attempt also sets the stream state: never deferred
            near = defer && !last && glibc_log_near1(a.r2);
        }
        const uint64_t nm = __ballot(near);
        if (nm) {
            if (near) {
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
                stk[top + below] = Near1Slot{a.x, a.y, d0, d1};
            }
            top += __popcll(nm);
        }
        if (active && !near) {
            double lg;
            if (defer) lg = __ballot(last && glibc_log_near1(a.r2)) ? glibc_log(a.r2) : glibc_log_main(a.r2);
            else lg = polar_log(g, a.r2);
            const double mult = (g.debug_flags & 1) ? a.r2 : sqrt(-2 * lg / a.r2);
            const double xm = a.x * mult;
            const double ym = a.y * mult;
            store_pair(g, d0, d1, ym * 1.0 + 0.0, xm * 1.0 + 0.0);
            if (last) {
                sout->state = s3 * kPcgMult + kPcgInc; // state after this attempt's 4th output
                sout->saved_flag = (int)((g.Q - f) & 1u);
                sout->saved = xm;
            }
        }
    }
    if (top >= 64) { // the stack is wave-private and a wave's LDS ops complete in order
        __asm__ volatile("" ::: "memory");
        near1_batch(g, stk, top, 64, lane);
        top -= 64;
        __asm__ volatile("" ::: "memory");
    }
}

// ---------------------------------------------------------------- run generation (gen_dense 2)
//
// Round 3's dense form needed every accepted attempt's state in memory: with split counting it recomputed
// the accept flags of every attempt wave that feeds a needed chunk (a whole wave of 1024 attempts for a few
// chunks: 40 us of a c4/8 table rank, profiles/r3/bl) behind a chain of scan kernels. The run form counts per
// 64-attempt group instead (K1, one ballot each; the split-counting exchange carries these bytes), scans them
// (K2g), and locates where each piece of consecutive needed chunks starts (K2l: group G and the accepts of G
// before the piece's first rank). One wave per piece (K3r) then walks the groups from there: each lane tests
// its attempt of the group (K1's mask on one GPU, the same float screen under split counting), accepted lanes
// of the piece append their state to a wave-private 128-slot LDS ring in rank order, and each completed chunk
// goes through dense_chunk (the chunk generation above: bit-identical noise). A piece of n chunks walks
// ~1.27 n + 1 groups; no round trip of states through memory, no per-wave pass over the whole stream.

// K2s: one share's block prefix. One 1024-thread block over the share's xchunk block counts (K1's per-block
// totals): the exclusive prefix of each block within the share (int32) and the share's total (int64), written
// to the share's record. Runs right after K1, before any exchange: with split counting it is each rank's own
// share, so the records the ranks exchange already carry their prefixes and nothing scans after the exchange.
__global__ __launch_bounds__(1024) void rng_share_scan_kernel(RngGeom g, const int *__restrict__ counts, int share)
{
    __shared__ long long wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = g.xchunk, per = (n + 1023) / 1024;
    const int b0 = share * n, i0 = min(tid * per, n), i1 = min(i0 + per, n);
    long long t = 0;
    for (int i = i0; i < i1; ++i) t += counts[b0 + i];
    long long x = t; // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    long long excl = x - t;
    for (int ww = 0; ww < w; ++ww) excl += wsum[ww];
    uint8_t *rec = g.xbuf + (size_t)share * g.xstride;
    int *lp = reinterpret_cast<int *>(rec + g.xlp_off);
    for (int i = i0; i < i1; ++i) {
        lp[i] = (int)excl;
        excl += counts[b0 + i];
    }
    if (tid == 1023) *reinterpret_cast<long long *>(rec + g.xtot_off) = excl;
}

// Where rank T of the call lies, from the share records: the group G (attempts [64 G, 64 G + 64)) whose
// accepted attempts hold ranks [T - skip, ...). Returns false if T is past every counted attempt. Uniform.
// Shares' totals -> the share; block prefixes in a 64-block window around the expected block (pi/4 of 4096
// attempts accepted per block: the window almost always brackets T at once) -> the block; its 64 group
// counts -> the group.
__device__ bool locate_rank(const RngGeom &g, long long T, int lane, long long &G, int &skip, long long &grand)
{
    const int W = g.xworld;
    int s = 0;
    long long Tl = T;
    if (W == 1) { // one share (one GPU): its total only bounds T, so the block search below need not wait for it
        grand = *reinterpret_cast<const long long *>(g.xbuf + g.xtot_off);
    } else {
        long long tot = 0;
        for (int sh = lane; sh < W; sh += 64)
            tot += *reinterpret_cast<const long long *>(g.xbuf + (size_t)sh * g.xstride + g.xtot_off);
        long long incl = tot; // shares in lane order (W <= 64: checked at create)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        grand = __shfl(incl, 63);
        if (T >= grand) return false;
        const uint64_t ms = __ballot(lane < W && T < incl && T >= incl - tot);
        s = __builtin_ctzll(ms);
        Tl = T - __shfl(incl - tot, s);
    }
    const uint8_t *rec = g.xbuf + (size_t)s * g.xstride;
    const int *lp = reinterpret_cast<const int *>(rec + g.xlp_off);
    const int n = g.xchunk;
    int lo = (int)((double)Tl * (1.0 / 3216.990877275948)) - 32; // 4096 * pi / 4 accepts per block
    lo = max(0, min(lo, n - 64));
    int b = -1;
    for (int it = 0; it < 1 << 16; ++it) { // bounded: each step moves the window towards T
        const int i = lo + lane;
        const bool le = i < n && (long long)lp[i] <= Tl; // lp is nondecreasing
        const uint64_t m = __ballot(le);
        if (m == 0) {
            if (lo == 0) break; // cannot happen (lp[0] = 0 <= Tl)
            lo = max(0, lo - 63);
            continue;
        }
        const int last = 63 - __builtin_clzll(m);
        if (last == 63 && lo + 64 < n) {
            lo += 63;
            continue;
        }
        b = lo + last;
        break;
    }
    if (b < 0 || T >= grand) return false;
    const long long Tb = Tl - __shfl(lp[min(lo + lane, n - 1)], b - lo);
    const int cnt = rec[(size_t)b * 64 + lane];
    int gin = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(gin, o);
        if (lane >= o) gin += y;
    }
    const uint64_t mg = __ballot((long long)gin > Tb);
    if (!mg) return false;
    const int gl = __builtin_ctzll(mg);
    skip = (int)(Tb - __shfl(gin - cnt, gl));
    G = ((long long)s * n + b) * 64 + gl;
    return true;
}

// K3r: one wave per piece (see above). RECOUNT (split counting): each lane screens its attempt of the group as
// K1 does; the walk keeps the states one and three steps into the attempt (s1, s3: one multiply-add each per
// group), the ring holds s1, and s0 = one step back when the chunk is generated. Otherwise (one GPU) the flags
// are K1's masks: the 16 groups of one (block, wave) share a 16-bit word per lane (word (G >> 4) * 64 + lane,
// bit G & 15), loaded once and the next one ahead; the walk keeps s0 alone.
template <bool RECOUNT>
__global__ __launch_bounds__(kRngThreads) void rng_run_generate_kernel(RngGeom g, const RngStateDev *__restrict__ sin,
                                                                      RngStateDev *__restrict__ sout,
                                                                      const uint16_t *__restrict__ masks,
                                                                      int *__restrict__ err)
{
    __shared__ Near1Slot stack_all[kRngThreads / 64][128];
    __shared__ uint64_t ring_all[kRngThreads / 64][128];
    const int lane = threadIdx.x & 63, wv = uniform(threadIdx.x >> 6);
    Near1Slot *stk = stack_all[wv];
    uint64_t *ring = ring_all[wv];
    const uint64_t f = (uint64_t)sin->saved_flag;
    const int p = blockIdx.x * (kRngThreads / 64) + wv;
    const long long A = (long long)((g.Q - f + 1) / 2);
    if (p == 0 && lane == 0 && f) { // the normal cached by the previous call is stream position 0
        double *d = stream_dest(g, stream_pos(g, 0));
        if (d) *d = sin->saved * 1.0 + 0.0;
    }
    if (p >= g.npieces[f]) return;
    const RunPiece pc = g.pieces[f][p];
    const bool defer = g.fast_log == 2;
    const long long c0 = uniform((int)pc.c0), cend = c0 + uniform((int)pc.n);
    long long G, grand;
    int skip;
    // the piece's (<= 12) chunk descriptors, one per lane, loaded once beside the locate
    const ChunkDest cds = lane < (int)pc.n ? chunk_dest_of(g, f, (int)pc.li0 + lane) : ChunkDest{0, 0, 0, -1, 0, 0};
    const bool found = locate_rank(g, c0 * 64, lane, G, skip, grand);
    if (p == g.npieces[f] - 1 && lane == 0 && grand < A) *err = 1; // not enough attempts launched: host re-sizes
    if (!found) return;
    G = uniform((int)G);
    long long R = c0 * 64 - uniform(skip); // rank of group G's first accepted attempt
    const long long r_lo = c0 * 64, r_end = min(cend * 64, A);
    const int span = (int)(r_end - r_lo);
    // lane's attempt 64 G + lane: its start state s0 (RECOUNT: s1, 1 step on, and s3, 3 steps on, instead)
    uint64_t st, s3 = 0;
    {
        const uint64_t S = sin->state;
        const PcgJumpDev jb = g.jump_block[G >> 6], jg = g.jump_gi[G & 63], jl = g.jump_lane[lane];
        st = jl.mult * (jg.mult * (jb.mult * S + jb.plus) + jg.plus) + jl.plus;
        if (RECOUNT) {
            st = st * kPcgMult + kPcgInc;
            s3 = st * kPcgMult2 + kPcgInc2;
        }
    }
    const long long nwords = g.nb_groups >> 4; // mask words per lane in the call
    uint32_t mw = 0, mw_next = 0;
    if (!RECOUNT) {
        mw = masks[(size_t)(G >> 4) * 64 + lane];
        mw_next = (G >> 4) + 1 < nwords ? masks[(size_t)((G >> 4) + 1) * 64 + lane] : 0u;
    }
    long long c = c0;
    int top = 0;
    while (c < cend && G < g.nb_groups) { // uniform; the group bound only matters after a shortage (err set)
        bool acc;
        if (RECOUNT) {
            const int v = polar_screen13(st, s3);
            acc = v > 0;
            if (v < 0) { // ~2e-5 of the attempts: the exact double test (random.tcc:1822-1826), as K1
                uint64_t s0 = (st - kPcgInc) * kPcgMultInv;
                acc = polar_attempt(s0).accept;
            }
        } else {
            acc = (mw >> (G & 15)) & 1u;
        }
        const uint64_t m = __ballot(acc);
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        // rank R + below, compared in 32 bits against the piece's span (R - r_lo is uniform, the span <= 768)
        if (acc && (unsigned)((int)(R - r_lo) + below) < (unsigned)span) ring[((int)R + below) & 127] = st;
        R += __popcll(m);
        ++G;
        if (RECOUNT) {
            st = g.next_mult * st + g.next_plus1;
            s3 = g.next_mult * s3 + g.next_plus3;
        } else {
            st = g.next_mult * st + g.next_plus;
            if ((G & 15) == 0) { // the next (block, wave) word; the one after it in flight
                mw = mw_next;
                mw_next = (G >> 4) + 1 < nwords ? masks[(size_t)((G >> 4) + 1) * 64 + lane] : 0u;
            }
        }
        __asm__ volatile("" ::: "memory"); // wave-private ring: only the compiler must keep the order
        while (c < cend && R >= min((c + 1) * 64, A)) { // every rank of chunk c is in the ring
            const uint64_t rs = ring[(c * 64 + lane) & 127];
            const uint64_t s = RECOUNT ? (rs - kPcgInc) * kPcgMultInv : rs;
            dense_chunk(g, f, A, c, chunk_dest_lane(cds, (int)(c - c0)), s, lane, defer, stk, top, sout);
            ++c;
        }
        __asm__ volatile("" ::: "memory");
    }
    if (top > 0) {
        __asm__ volatile("" ::: "memory");
        near1_batch(g, stk, top, top, lane);
    }
}

// K2 + K2c in one block for planes of at most 1024 attempt blocks (c1, c2, the reference's own
// grid): the scan of the block counts (one count per thread), the attempt-shortage check and the
// wave plan, with the offsets kept in LDS. One launch instead of three: small planes are bound by
// the host's launch rate. Same offsets, part[0] = 0 and task list as K2a/K2b/K2c (task order is
// free: K3 takes its ranks from each task).
__global__ __launch_bounds__(1024) void rng_scan_plan_small_kernel(RngGeom g, const RngStateDev *__restrict__ sin,
                                                                   const int *__restrict__ counts,
                                                                   long long *__restrict__ offsets,
                                                                   long long *__restrict__ part,
                                                                   const int *__restrict__ wave_counts, int nb_scan,
                                                                   int nb_total, WaveTask *__restrict__ tasks,
                                                                   int *__restrict__ ntasks, int *__restrict__ err)
{
    constexpr int WPB = kRngThreads / 64;
    __shared__ long long p[1024];
    __shared__ int base_sh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int v = tid < nb_scan ? counts[tid] : 0;
    p[tid] = v;
    if (tid == 0) base_sh = 0;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) { // inclusive scan
        const long long y = tid >= o ? p[tid - o] : 0;
        __syncthreads();
        p[tid] += y;
        __syncthreads();
    }
    const long long excl = p[tid] - v;
    if (tid < nb_scan) offsets[tid] = excl;
    __syncthreads();
    p[tid] = excl; // exclusive offsets for the plan below
    __syncthreads();
    const uint64_t f = (uint64_t)sin->saved_flag;
    const long long A = (long long)((g.Q - f + 1) / 2);
    if (tid == 0) {
        part[0] = 0;
        if (p[nb_scan - 1] + counts[nb_scan - 1] < A) *err = 1; // not enough attempts launched
        if (f) {
            double *d = stream_dest(g, stream_pos(g, 0));
            if (d) *d = sin->saved * 1.0 + 0.0;
        }
    }
    for (int gw0 = 0; gw0 < nb_total * WPB; gw0 += 1024) { // uniform trip count: every wave reaches the barriers
        const int gw = gw0 + tid;
        bool need = false;
        long long r_lo = 0;
        if (gw < nb_total * WPB) {
            const int b = gw / WPB, w = gw % WPB;
            r_lo = p[b];
            for (int ww = 0; ww < w; ++ww) r_lo += wave_counts[(size_t)b * WPB + ww];
            const long long r_hi = r_lo + wave_counts[gw];
            if (r_lo < A) {
                const uint64_t q_lo = f + 2ull * (uint64_t)r_lo;
                const uint64_t q_hi = (f + 2ull * (uint64_t)r_hi) < g.Q ? (f + 2ull * (uint64_t)r_hi) : g.Q;
                const bool ends_call = A - 1 < r_hi;
                need = ends_call || (q_lo < q_hi && range_needed(g, q_lo, q_hi));
            }
        }
        const uint64_t m = __ballot(need);
        int base = 0;
        if (m && lane == 0) base = atomicAdd(&base_sh, __popcll(m)); // LDS atomic: one block
        base = __shfl(base, 0);
        if (need) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            tasks[base + below] = WaveTask{r_lo, gw, 0};
        }
    }
    __syncthreads();
    if (tid == 0) *ntasks = base_sh;
}

__global__ void replicate_share_kernel(uint4 *__restrict__ buf, size_t n16, int rank)
{
    const int r = blockIdx.y; // destination record
    if (r == rank) return;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        buf[(size_t)r * n16 + i] = buf[(size_t)rank * n16 + i];
}

hipError_t launch_replicate_share(uint8_t *buf, size_t bytes, int world, int rank, hipStream_t st)
{
    hipLaunchKernelGGL(replicate_share_kernel, dim3(64, world), dim3(256), 0, st, reinterpret_cast<uint4 *>(buf),
                       bytes / 16, rank);
    return hipGetLastError();
}

hipError_t launch_rng_share_scan(const RngGeom &g, const int *counts, int share, hipStream_t st)
{
    hipLaunchKernelGGL(rng_share_scan_kernel, dim3(1), dim3(1024), 0, st, g, counts, share);
    return hipGetLastError();
}

hipError_t launch_rng_count(const RngGeom &g, const RngStateDev *st_in, int *counts, int *wave_counts,
                            uint16_t *masks, int b0, int nb, int nb_total, hipStream_t st)
{
    hipLaunchKernelGGL(rng_count_kernel, dim3(nb), dim3(kRngThreads), 0, st, g, st_in, counts, wave_counts, masks, b0,
                       nb, nb_total);
    return hipGetLastError();
}

hipError_t launch_rng_finish(const RngGeom &g, const RngStateDev *st_in, RngStateDev *st_out, int *counts,
                             const int *wave_counts, long long *offsets, long long *part, uint16_t *masks,
                             WaveTask *tasks, int *ntasks, int *err, int nb_total, int nb_scan, hipStream_t st)
{
    const int nparts = (nb_scan + 1023) / 1024; // <= 1024: checked at create
    if (g.gen_dense == 2) { // run generation: K3r alone (K2s ran with K1, before any exchange)
        const int np = g.npieces[0] > g.npieces[1] ? g.npieces[0] : g.npieces[1];
        if (g.recount)
            hipLaunchKernelGGL(rng_run_generate_kernel<true>, dim3((np + 3) / 4), dim3(kRngThreads), 0, st, g, st_in,
                               st_out, masks, err);
        else
            hipLaunchKernelGGL(rng_run_generate_kernel<false>, dim3((np + 3) / 4), dim3(kRngThreads), 0, st, g, st_in,
                               st_out, masks, err);
        return hipGetLastError();
    }
    if (g.fused_plan) {
        // the compacted K3 plans its own waves (small planes: one launch fewer per call)
    } else if (nb_scan <= 1024 && nb_total <= 1024) {
        hipLaunchKernelGGL(rng_scan_plan_small_kernel, dim3(1), dim3(1024), 0, st, g, st_in, counts, offsets, part,
                           wave_counts, nb_scan, nb_total, tasks, ntasks, err);
    } else {
        hipLaunchKernelGGL(rng_scan_local_kernel, dim3(nparts), dim3(256), 0, st, counts, offsets, part, nb_scan);
        hipLaunchKernelGGL(rng_scan_parts_kernel, dim3(1), dim3(1024), 0, st, part, nparts, st_in, g.Q, err, ntasks);
        const int nw = nb_total * (kRngThreads / 64);
        hipLaunchKernelGGL(rng_plan_kernel, dim3((nw + 255) / 256), dim3(256), 0, st, g, st_in, offsets, part,
                           wave_counts, nb_total, tasks, ntasks);
    }
    hipLaunchKernelGGL(rng_generate_compact_kernel, dim3(nb_total * g.gen_split), dim3(kRngThreads), 0, st, g,
                       st_in, st_out, tasks, ntasks, masks, counts, wave_counts, err);
    return hipGetLastError();
}


// Hold this wave's output stores until the next write window (SweepArgs::ywin_T/zwin_T).
__device__ __forceinline__ void write_window(int T, int W)
{
    if (T <= 0 || W <= 0) return; // W = 0 would never open: treated as off
    const uint64_t m = (uint64_t)T - 1;
    // bounded: a wave waits at most ~T ticks of the clock, and never more than 8192 sleeps (~1.7 ms)
    // whatever the counter does, so every wave reaches its stores and the grid drains
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < 8192; ++it) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if ((t & m) < (uint64_t)W || t - t0 > (uint64_t)T) break;
        __builtin_amdgcn_s_sleep(8);
    }
}

// ---------------------------------------------------------------- K4 y-pass
//
// One wave = one tile of R consecutive rows x one 128-cell strip; lane l owns
// cells 2l, 2l+1. Walking the noise rows t once, each noise row is loaded a
// single time and applied to every tile row r whose stencil covers it (tap
// i = t - r), so per cell the taps still accumulate in the reference's order
// i = -N..N. The coefficient stream is the only HBM-bound load: one 1 KiB
// coalesced dwordx4 per (row, tap).

template <int R, bool TABLE, bool NT, int YU, bool PC>
__global__ __launch_bounds__(256) void ypass_kernel(SweepArgs a, int nrowblk)
{
    const int c = blockIdx.y;
    if (!((a.comps_mask >> c) & 1)) return;
    const int lane = threadIdx.x & 63;
    // XCD-aware order (guide T1): blocks b and b+8 share an XCD, so hand each XCD
    // a contiguous run of blocks; with strip-major tiles the row blocks that
    // re-read the same noise rows then meet in one L2. gridDim.x % 8 == 0.
    const int per_xcd = gridDim.x >> 3;
    const int b = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    const int tile = uniform(b * 4 + (threadIdx.x >> 6));
    if (tile >= a.nstrips * nrowblk) return;
    const int s = tile / nrowblk;          // strip-major: neighbouring tiles share noise rows
    int rb = tile - s * nrowblk;
    rb = nrowblk - 1 - rb; // wide stencils (large j) start first: shorter tail
    const int j0 = rb * R;
    const int Ny = a.Ny;
    const int nr = min(R, Ny - j0);
    const int col = s * kStrip + 2 * lane;
    const int Pz = a.Pz;
    // Lanes wholly in the last strip's padding leave: every later load then fetches only the
    // live lanes' bytes (Nz = 400 on the reference's grid: 22% of a 512-wide stream)
    if (col >= a.Nz_loc) return;

    int N[R];
    const double *bp[R];
    const double *tb[R], *tb1[R]; // table mode: half-vector of cell col (and col+1 when PC)
    int Nlo = 1 << 30, Nhi = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        N[r] = 0;
        bp[r] = nullptr;
        tb[r] = tb1[r] = nullptr;
        if (r < nr) {
            N[r] = a.Ny_st[c][(size_t)s * Ny + j0 + r];
            Nlo = min(Nlo, N[r]);
            Nhi = max(Nhi, N[r]);
            if (TABLE && PC) { // per-lane N; the table is zero past each N (taps up to N_st)
                const int *nc = a.Ny_cell[c] + (size_t)(j0 + r) * a.Nz_loc;
                tb[r] = a.tab + a.tab_off[col < a.Nz_loc ? nc[col] : 0];
                tb1[r] = a.tab + a.tab_off[col + 1 < a.Nz_loc ? nc[col + 1] : 0];
            } else if (TABLE) {
                tb[r] = a.tabf + a.tabf_off[N[r]] + N[r]; // centre of the full vector: tap i at tb[i]
            } else {
                bp[r] = a.By[c] + a.byoff[c][(size_t)s * Ny + j0 + r] + (ptrdiff_t)(N[r] - r) * kStrip + 2 * lane;
            }
        }
    }
    const double *np = a.ry[c] + (size_t)(j0 + a.Nyp[c]) * Pz + col;

    double acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc0[r] = acc1[r] = 0.0;

    auto coef = [&](int r, int t) -> double2 {
        if (TABLE) {
            const int i = t - r;
            if (!PC) {
                const double b = tb[r][i];
                return make_double2(b, b);
            }
            const int ai = i < 0 ? -i : i;
            return make_double2(tb[r][ai], tb1[r][ai]);
        }
        return ldB<NT>(bp[r] + (ptrdiff_t)t * kStrip);
    };
    auto predicated = [&](int t) {
        const double2 n = ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)t * Pz));
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = t - r;
            if (r < nr && i >= -N[r] && i <= N[r]) {
                const double2 b = coef(r, t);
                acc0[r] += b.x * n.x;
                acc1[r] += b.y * n.y;
            }
        }
    };
    auto noise = [&](int t) { return ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)t * Pz)); };
    auto body = [&](int t) {
        const double2 n = ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)t * Pz));
        double2 b[R];
#pragma unroll
        for (int r = 0; r < R; ++r) b[r] = coef(r, t);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc0[r] += b[r].x * n.x;
            acc1[r] += b[r].y * n.y;
        }
    };

    const int tlo = -Nhi, thi = (nr - 1) + Nhi;
    const bool body_ok = (nr == R) && (R - 1 - Nlo <= Nlo);
    const int bl = body_ok ? R - 1 - Nlo : thi + 1;
    const int bh = body_ok ? Nlo : thi;
    int t = tlo;
    for (; t < bl; ++t) predicated(t);
    if (YU >= 8 && !PC && t + YU - 1 <= bh) {
        // Deep pipeline (yunroll 8): a ring of YU taps' noise and coefficients in registers;
        // slot u is refilled with tap t+u+YU right after it is consumed, so YU taps are always
        // in flight. For planes with few waves per SIMD and wide stencils (the reference's own
        // grid: N_y up to 212) a wave's serial load->use chain, not HBM bandwidth, sets the time.
        double2 nb[YU], cb[YU][R];
#pragma unroll
        for (int u = 0; u < YU; ++u) {
            nb[u] = noise(t + u);
#pragma unroll
            for (int r = 0; r < R; ++r) cb[u][r] = coef(r, t + u);
        }
        auto use = [&](const double2 n, const double2 *b) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc0[r] += b[r].x * n.x;
                acc1[r] += b[r].y * n.y;
            }
        };
        for (; t + 2 * YU - 1 <= bh; t += YU) {
#pragma unroll
            for (int u = 0; u < YU; ++u) {
                use(nb[u], cb[u]);
                nb[u] = noise(t + u + YU);
#pragma unroll
                for (int r = 0; r < R; ++r) cb[u][r] = coef(r, t + u + YU);
            }
        }
#pragma unroll
        for (int u = 0; u < YU; ++u) use(nb[u], cb[u]);
        t += YU;
    }
    if (YU >= 4) {
        for (; t + 3 <= bh; t += 4) {
            body(t);
            body(t + 1);
            body(t + 2);
            body(t + 3);
        }
    }
    for (; t + 1 <= bh; t += 2) {
        body(t);
        body(t + 1);
    }
    for (; t <= bh; ++t) body(t);
    for (; t <= thi; ++t) predicated(t);

    write_window(a.ywin_T, a.ywin_W);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r < nr) {
            double *o = a.rz[c] + (size_t)(j0 + r) * a.rz_pitch[c] + a.Nzp[c] + col;
            if (col + 1 < a.Nz_loc) {
                if (a.ynt_stores) __builtin_nontemporal_store(dvec2{acc0[r], acc1[r]}, reinterpret_cast<dvec2 *>(o));
                else *reinterpret_cast<double2 *>(o) = make_double2(acc0[r], acc1[r]);
            }
            else if (col < a.Nz_loc) o[0] = acc0[r];
        }
    }
}

// K4, table mode (row-uniform N per cell: every plane but per-cell grids): the per-wave tile of ypass_kernel with
// the coefficients from the full symmetric vectors (tabf) and only the paths table mode takes, so the kernel's
// register budget is set by its hot loop alone (the shared ypass_kernel carried every packed and table path:
// 105 VGPRs, 4 waves per SIMD, for a loop that needs ~60; round 4). Hot loop on tiles whose R rows share one N:
// taps in groups of 4 noise rows, the noise KYD groups ahead in a register ring, the group's R + 3
// coefficients one scalar window (b[t - R + 1 .. t + 3]) loaded one group ahead. Tiles where N steps between
// their rows take the per-row form with the next two noise rows in flight. Same products, same order as
// df.cpp:373-375: bit-identical.
template <int R, int KYD>
__global__ __launch_bounds__(256) void ypass_table_kernel(SweepArgs a, int nrowblk)
{
    const int c = blockIdx.y;
    if (!((a.comps_mask >> c) & 1)) return;
    const int lane = threadIdx.x & 63;
    const int per_xcd = gridDim.x >> 3; // XCD-aware order, as ypass_kernel
    const int b = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    const int tile = uniform(b * 4 + (threadIdx.x >> 6));
    if (tile >= a.nstrips * nrowblk) return;
    const int s = tile / nrowblk;
    const int rb = nrowblk - 1 - (tile - s * nrowblk); // wide stencils (large j) start first
    const int j0 = rb * R;
    const int Ny = a.Ny;
    const int nr = min(R, Ny - j0);
    const int col = s * kStrip + 2 * lane;
    const int Pz = a.Pz;
    if (col >= a.Nz_loc) return; // lanes wholly in the last strip's padding
    int N[R];
    const double *tb[R];
    int Nlo = 1 << 30, Nhi = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        N[r] = 0;
        tb[r] = a.tabf; // unused for r >= nr
        if (r < nr) {
            N[r] = a.Ny_st[c][(size_t)s * Ny + j0 + r];
            Nlo = min(Nlo, N[r]);
            Nhi = max(Nhi, N[r]);
            tb[r] = a.tabf + a.tabf_off[N[r]] + N[r]; // centre of the full vector: tap i at tb[i]
        }
    }
    const double *np = a.ry[c] + (size_t)(j0 + a.Nyp[c]) * Pz + col;
    double acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc0[r] = acc1[r] = 0.0;
    auto noise = [&](int t) { return ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)t * Pz)); };
    auto predicated = [&](int t) {
        const double2 n = noise(t);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = t - r;
            if (r < nr && i >= -N[r] && i <= N[r]) {
                const double bb = tb[r][i];
                acc0[r] += bb * n.x;
                acc1[r] += bb * n.y;
            }
        }
    };
    auto body_n = [&](int t, const double2 n) {
        double bb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) bb[r] = tb[r][t - r];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc0[r] += bb[r] * n.x;
            acc1[r] += bb[r] * n.y;
        }
    };
    const int tlo = -Nhi, thi = (nr - 1) + Nhi;
    const bool body_ok = (nr == R) && (R - 1 - Nlo <= Nlo);
    const int bl = body_ok ? R - 1 - Nlo : thi + 1;
    const int bh = body_ok ? Nlo : thi;
    int t = tlo;
    for (; t < bl; ++t) predicated(t);
    if (Nlo == Nhi && t + 4 * KYD - 1 <= bh) {
        constexpr int WN = (R + 3 + 7) / 8 * 8;
        const double *cb = tb[0] - (R - 1); // window base: b[t - R + 1 + k] = cb[t + k]
        double2 nq[KYD][4];
        const ptrdiff_t P1 = Pz, P2 = 2 * (ptrdiff_t)Pz, P3 = 3 * (ptrdiff_t)Pz, P4 = 4 * (ptrdiff_t)Pz;
        const double *nl = np + (ptrdiff_t)t * Pz; // next group to load
        auto ldn = [&](double2 (&nn)[4]) {
            nn[0] = ld_pair(reinterpret_cast<const double2 *>(nl));
            nn[1] = ld_pair(reinterpret_cast<const double2 *>(nl + P1));
            nn[2] = ld_pair(reinterpret_cast<const double2 *>(nl + P2));
            nn[3] = ld_pair(reinterpret_cast<const double2 *>(nl + P3));
            nl += P4;
        };
        auto taps = [&](const double2 (&nn)[4], const double (&ww)[WN]) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double bb = ww[u - r + R - 1];
                    acc0[r] += bb * nn[u].x;
                    acc1[r] += bb * nn[u].y;
                }
                __builtin_amdgcn_sched_barrier(0); // one tap's products at a time (register pressure)
            }
        };
        const double *wq = cb + t;
        double w[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) w[k] = wq[k];
#pragma unroll
        for (int g = 0; g < KYD; ++g) ldn(nq[g]);
        for (; t + 8 * KYD - 1 <= bh; t += 4 * KYD) { // the groups issued below stay within bh
#pragma unroll
            for (int g = 0; g < KYD; ++g) {
                double wn[WN];
#pragma unroll
                for (int k = 0; k < WN; ++k) wn[k] = wq[4 + k]; // the table is padded past its last vector
                __builtin_amdgcn_sched_barrier(0);
                taps(nq[g], w);
                ldn(nq[g]); // group t + 4 (g + KYD)
                __builtin_amdgcn_sched_barrier(0);
                wq += 4;
#pragma unroll
                for (int k = 0; k < WN; ++k) w[k] = wn[k];
            }
        }
#pragma unroll
        for (int g = 0; g < KYD; ++g) { // drain: groups t .. t + 4 KYD - 1, loaded, within bh
            double wn[WN];
#pragma unroll
            for (int k = 0; k < WN; ++k) wn[k] = wq[4 + k];
            taps(nq[g], w);
            wq += 4;
#pragma unroll
            for (int k = 0; k < WN; ++k) w[k] = wn[k];
        }
        t += 4 * KYD;
    }
    if (t + 1 <= bh) { // per-row coefficients, the next two noise rows in flight
        double2 n0 = noise(t), n1 = noise(t + 1);
        for (; t + 5 <= bh; t += 4) {
            const double2 m0 = noise(t + 2), m1 = noise(t + 3);
            body_n(t, n0);
            body_n(t + 1, n1);
            n0 = noise(t + 4);
            n1 = noise(t + 5);
            body_n(t + 2, m0);
            body_n(t + 3, m1);
        }
        if (t + 3 <= bh) {
            const double2 m0 = noise(t + 2), m1 = noise(t + 3);
            body_n(t, n0);
            body_n(t + 1, n1);
            body_n(t + 2, m0);
            body_n(t + 3, m1);
            t += 4;
        } else {
            body_n(t, n0);
            body_n(t + 1, n1);
            t += 2;
        }
    }
    for (; t <= bh; ++t) body_n(t, noise(t));
    for (; t <= thi; ++t) predicated(t);
    write_window(a.ywin_T, a.ywin_W);
    if (col < a.ylo[c]) return; // ylo even: the lane's pair is wholly in or out
    const int yhi = a.yhi[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r < nr) {
            double *o = a.rz[c] + (size_t)(j0 + r) * a.rz_pitch[c] + a.yout[c] + col;
            if (col + 1 < yhi) {
                if (a.ynt_stores) __builtin_nontemporal_store(dvec2{acc0[r], acc1[r]}, reinterpret_cast<dvec2 *>(o));
                else *reinterpret_cast<double2 *>(o) = make_double2(acc0[r], acc1[r]);
            } else if (col < yhi) o[0] = acc0[r];
        }
    }
}

// K4, block-cooperative form over a PAIR of rows (SweepArgs::ycoop 7, 8; 7 is the default for long
// chains): one block per (strip, rows j0, j0 + 1). The block walks the union of the two rows' noise
// ranges in chunks; wave w loads noise rows w, w+4, ... of the chunk once and both rows' coefficients
// for them, so each noise load serves two products (the one-row form re-reads every noise row once per
// output row: half its vector-memory bytes are noise). Threads 0-127 add row j0's products and threads
// 128-255 row j0 + 1's, each over its own row's taps in the order i = -N..N: bit-identical to the other
// forms. The next chunk's loads are in flight through the barrier and the sums (as PIPE).
// Measured on the reference's grid (profiles/r2/ab_ycoop2_native.jsonl): y-pass 0.178 (one row, PIPE)
// -> 0.157 ms; four rows per block, two chunks in flight and 8 noise rows per wave were slower.
// A strip with fewer live columns than 128 (the last strip of a plane whose width is not a multiple
// of 128: 16 of 128 on the reference's grid) folds G = 64 / P tap groups into the wave, P = live
// column pairs rounded up to a power of two: lane l loads column pair l % P of noise row l / P, so one
// load instruction covers G noise rows and the block walks its chain in 1/G of the chunks.
// Blocks x, x+8, ... (one XCD) run tiles [ycoop2_xcd[c][x], ycoop2_xcd[c][x+1]): contiguous runs of equal
// coefficient bytes (balance_ycoop2 in df_capi.cpp).
template <bool NT, int KPW>
__global__ __launch_bounds__(256) void ypass_coop2_kernel(SweepArgs a)
{
    constexpr int CH = 4 * KPW; // noise rows per chunk and tap group
    constexpr int RR = 2, RH = 1; // rows per block, rows summed per thread
    __shared__ double2 prod[RR * CH * 64];
    const int c = blockIdx.y;
    if (!((a.comps_mask >> c) & 1)) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int Ny = a.Ny, nrowblk = (Ny + RR - 1) / RR;
    const int x = blockIdx.x & 7;
    const int pos = a.ycoop2_xcd[c][x] + (int)(blockIdx.x >> 3);
    if (pos >= a.ycoop2_xcd[c][x + 1]) return; // block-uniform
    const int code = a.ycoop2_perm[c] ? a.ycoop2_perm[c][pos] : pos * 8; // tile * 8 + part (balance_ycoop2)
    const int tile = code >> 3, part = code & 7;
    const int s = tile / nrowblk;             // rows ascending within a strip (L2 reuse of noise rows)
    const int j0 = (tile - s * nrowblk) * RR;
    const int nr = min(RR, Ny - j0);
    // the item's columns: the whole strip (part 0), a 64-column half (1, 2) or a 32-column quarter (3-6)
    const int iw = part == 0 ? kStrip : part <= 2 ? 64 : 32;
    const int cb = part == 0 ? 0 : part <= 2 ? (part - 1) * 64 : (part - 3) * 32, c0 = s * kStrip + cb;
    // live column pairs of this item -> P lanes per tap group (power of two), G groups per wave
    const int pairs = min(iw / 2, (a.Nz_loc - c0 + 1) >> 1);
    int lp = 0;
    while ((1 << lp) < pairs) ++lp;
    const int P = 1 << lp, G = 64 >> lp, CHG = CH * G;
    const int q = lane >> lp, p = lane & (P - 1);
    int lo[RR], hi[RR]; // row r's noise rows [lo, hi] = j0 + r + [-N, N]
    const double *bp[RR];
    int mlo = 1 << 30, mhi = -(1 << 30);
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const int rr = r < nr ? r : 0; // a missing row mirrors the first and is never summed
        const int N = a.Ny_st[c][(size_t)s * Ny + j0 + rr];
        lo[r] = j0 + rr - N;
        hi[r] = j0 + rr + N;
        mlo = min(mlo, lo[r]);
        mhi = max(mhi, hi[r]);
        bp[r] = a.By[c] + a.byoff[c][(size_t)s * Ny + j0 + rr] + cb + 2 * p; // tap t at bp + t*128
    }
    const int M = mhi - mlo + 1;
    const int col = c0 + 2 * p;
    const bool live = col < a.Nz_loc;
    const double *np = a.ry[c] + (size_t)(mlo + a.Nyp[c]) * a.Pz + col; // noise row mlo + u at np + u*Pz
    double2 b[RR][KPW], n[KPW];
    auto load = [&](int u0) {
#pragma unroll
        for (int k = 0; k < KPW; ++k) {
            const int u = u0 + (w + 4 * k) * G + q, m = mlo + u;
            n[k] = (live && u < M) ? ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)u * a.Pz))
                                      : make_double2(0.0, 0.0);
#pragma unroll
            for (int r = 0; r < RR; ++r)
                b[r][k] = (live && u < M && m >= lo[r] && m <= hi[r])
                                 ? ldB<NT>(bp[r] + (ptrdiff_t)(m - lo[r]) * kStrip)
                                 : make_double2(0.0, 0.0);
        }
    };
    // row r, chunk slot v (noise row u0 + v), column pair p at prod[r*CH*64 + v*P + p]
    const int rs = threadIdx.x >> 7, cell = threadIdx.x & (kStrip - 1); // summing thread: rows rs + 2i, cell
    int lor[RH], hir[RH];
#pragma unroll
    for (int i = 0; i < RH; ++i) { // selects: no indexed register array
        lor[i] = rs ? lo[2 * i + 1] : lo[2 * i];
        hir[i] = rs ? hi[2 * i + 1] : hi[2 * i];
    }
    double acc[RH];
#pragma unroll
    for (int i = 0; i < RH; ++i) acc[i] = 0.0;
    load(0);
    for (int u0 = 0; u0 < M; u0 += CHG) {
#pragma unroll
        for (int k = 0; k < KPW; ++k)
#pragma unroll
            for (int r = 0; r < RR; ++r)
                prod[r * CH * 64 + ((w + 4 * k) * G + q) * P + p] =
                    make_double2(b[r][k].x * n[k].x, b[r][k].y * n[k].y);
        if (u0 + CHG < M) load(u0 + CHG); // block-uniform
        __syncthreads();
        if (cell < 2 * P) {
#pragma unroll
            for (int i = 0; i < RH; ++i) {
                // this chunk's noise rows of row 2i + rs: u in [ua, ub) (wave-uniform)
                const int ua = __builtin_amdgcn_readfirstlane(max(0, lor[i] - mlo - u0));
                const int ub = __builtin_amdgcn_readfirstlane(min(CHG, hir[i] - mlo - u0 + 1));
                const double *pc = reinterpret_cast<const double *>(prod + (2 * i + rs) * CH * 64) + cell;
                // LDS reads issued 8 at a time, then their adds in tap order: one add per LDS round trip made
                // the sum a serial chain of LDS latencies (CHG = 128 of them per chunk on a folded narrow strip).
                if (P == 64 && ua == 0 && ub == CHG) { // whole chunk of a full strip: immediate offsets
#pragma unroll
                    for (int g = 0; g < CH; g += 8) {
                        double v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = pc[(g + e) * 128];
#pragma unroll
                        for (int e = 0; e < 8; ++e) acc[i] += v[e];
                    }
                } else {
                    // slots past ub (clamped into the chunk) are read but never added: the same additions
                    for (int g = ua; g < ub; g += 8) {
                        double v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] = pc[min(g + e, CHG - 1) * 2 * P];
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            if (g + e < ub) acc[i] += v[e]; // wave-uniform condition
                    }
                }
            }
        }
        __syncthreads();
    }
    const int k = c0 + cell;
#pragma unroll
    for (int i = 0; i < RH; ++i) {
        const int r = 2 * i + rs;
        if (r < nr && cell < 2 * P && k < a.Nz_loc) {
            double *o = a.rz[c] + (size_t)(j0 + r) * a.rz_pitch[c] + a.Nzp[c] + k;
            if (a.ynt_stores) __builtin_nontemporal_store(acc[i], o);
            else *o = acc[i];
        }
    }
}

// K4 table mode, noise staged in LDS (SweepArgs::ylds): one block per (strip, 4R rows), wave w summing rows
// j0 + wR .. j0 + wR + R - 1 for the lane's column pair. The block walks the union of its rows' noise ranges
// in chunks of 16 noise rows: every noise row is read from global memory ONCE per block (each wave loads 4 of
// the chunk's rows, the next chunk's loads in flight through the current chunk's sums) and from LDS by every
// wave whose rows reach it. The per-wave forms load each noise row once per wave: on c3 their 2.6 GB of
// vector-memory reads per call hold the y-pass 0.05 ms above its FP64 floor (ablation, profiles/r3/an).
// Each row adds its taps in the order i = -N..N (noise rows ascending), so results are bit-identical.
template <int K> using ic_t = std::integral_constant<int, K>;
// f(ic_t<K>), f(ic_t<K + 1>), ..., f(ic_t<E - 1>): a loop over register sets unrolled at compile time
template <int K, int E, class F> __device__ __forceinline__ void unroll_to(F &&f)
{
    if constexpr (K < E) {
        f(ic_t<K>{});
        unroll_to<K + 1, E>(f);
    }
}

// PD: chunks of noise loads in flight (register sets; the loop is unrolled by PD so each set stays static)
// NW waves per block (one block = NW R rows), C noise rows per chunk (C / NW loaded per wave)
template <int R, int PD, int NW = 4, int C = 16>
__global__ __launch_bounds__(64 * NW) void ypass_tlds_kernel(SweepArgs a, int nrowblk)
{
    constexpr int LW = C / NW; // chunk rows each wave loads
    __shared__ double2 nbuf[2][C][64];
    const int c = blockIdx.y;
    if (!((a.comps_mask >> c) & 1)) return;
    const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
    const int per_xcd = gridDim.x >> 3; // XCD-aware: each XCD a contiguous run of strip-major tiles
    const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= a.nstrips * nrowblk) return; // block-uniform
    const int s = tile / nrowblk;
    const int rb = nrowblk - 1 - (tile - s * nrowblk); // wide stencils first
    const int Ny = a.Ny, RB = NW * R, j0 = rb * RB;
    const int *nst = a.Ny_st[c] + (size_t)s * Ny;
    int mlo = 1 << 30, mhi = -(1 << 30); // the block's noise rows
    for (int q = 0; q < RB && j0 + q < Ny; ++q) {
        const int N = nst[j0 + q];
        mlo = min(mlo, j0 + q - N);
        mhi = max(mhi, j0 + q + N);
    }
    const int jw = j0 + w * R;
    int lo[R], hi[R];
    const double *tb[R]; // row r's full tap vector: tap t = m - lo[r] at tb[r][t]
#pragma unroll
    for (int r = 0; r < R; ++r) {
        lo[r] = 1 << 30;
        hi[r] = -(1 << 30);
        tb[r] = a.tabf;
        if (jw + r < Ny) {
            const int N = nst[jw + r];
            lo[r] = jw + r - N;
            hi[r] = jw + r + N;
            tb[r] = a.tabf + a.tabf_off[N];
        }
    }
    const int col = s * kStrip + 2 * lane;
    const bool live = col < a.Nz_loc;
    const double *np = a.ry[c] + (size_t)a.Nyp[c] * a.Pz + col; // noise row m at np + m * Pz
    double2 pre[PD][LW];
    auto gload = [&](auto K, int u0) {
        constexpr int k0 = decltype(K)::value;
#pragma unroll
        for (int k = 0; k < LW; ++k) {
            const int m = u0 + w + NW * k;
            pre[k0][k] = live && m <= mhi ? ld_pair(reinterpret_cast<const double2 *>(np + (ptrdiff_t)m * a.Pz))
                                          : make_double2(0.0, 0.0);
        }
    };
    auto lstore = [&](auto K, int buf) {
        constexpr int k0 = decltype(K)::value;
#pragma unroll
        for (int k = 0; k < LW; ++k) nbuf[buf][w + NW * k][lane] = pre[k0][k];
    };
    double acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc0[r] = acc1[r] = 0.0;
    auto compute = [&](int u0, int buf) {
        const int mb = min(u0 + C - 1, mhi);
        bool full = mb == u0 + C - 1, any = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            full = full && lo[r] <= u0 && hi[r] >= mb;
            any = any || (lo[r] <= mb && hi[r] >= u0);
        }
        if (full) { // every row of the wave takes all 16 noise rows of the chunk
            const double *cb[R];
#pragma unroll
            for (int r = 0; r < R; ++r) cb[r] = tb[r] + (u0 - lo[r]);
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const double2 n = nbuf[buf][q][lane];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double b = cb[r][q];
                    acc0[r] += b * n.x;
                    acc1[r] += b * n.y;
                }
            }
        } else if (any) {
            for (int m = u0; m <= mb; ++m) {
                const double2 n = nbuf[buf][m - u0][lane];
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (m >= lo[r] && m <= hi[r]) { // wave-uniform
                        const double b = tb[r][m - lo[r]];
                        acc0[r] += b * n.x;
                        acc1[r] += b * n.y;
                    }
            }
        }
    };
    // chunk i: rows mlo + 16 i ..; its loads in register set i % PD, its sums from LDS buffer i % 2.
    // Step i: the loads of chunk i + PD go into the set chunk i vacated, chunk i is summed, chunk i + 1
    // (loaded PD - 1 steps earlier) is stored to the other buffer, barrier.
    const int nch = (mhi - mlo) / C + 1;
    gload(ic_t<0>{}, mlo);
    if constexpr (PD > 1) gload(ic_t<1 % PD>{}, mlo + C);
    if constexpr (PD > 2) gload(ic_t<2 % PD>{}, mlo + 2 * C);
    lstore(ic_t<0>{}, 0);
    __syncthreads();
    auto step = [&](auto K, int i) {
        constexpr int k = decltype(K)::value;
        if (i + PD < nch) gload(K, mlo + (i + PD) * C); // block-uniform
        compute(mlo + i * C, i & 1);
        if (i + 1 < nch) lstore(ic_t<(k + 1) % PD>{}, (i + 1) & 1);
        __syncthreads();
    };
    for (int i = 0; i < nch; i += PD) {
        step(ic_t<0>{}, i);
        if constexpr (PD > 1)
            if (i + 1 < nch) step(ic_t<1 % PD>{}, i + 1);
        if constexpr (PD > 2)
            if (i + 2 < nch) step(ic_t<2 % PD>{}, i + 2);
    }
    write_window(a.ywin_T, a.ywin_W);
    if (col < a.ylo[c]) return; // ylo even: the lane's pair is wholly in or out
    const int yhi = a.yhi[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (jw + r >= Ny) continue;
        double *o = a.rz[c] + (size_t)(jw + r) * a.rz_pitch[c] + a.yout[c] + col;
        if (col + 1 < yhi) {
            if (a.ynt_stores) __builtin_nontemporal_store(dvec2{acc0[r], acc1[r]}, reinterpret_cast<dvec2 *>(o));
            else *reinterpret_cast<double2 *>(o) = make_double2(acc0[r], acc1[r]);
        } else if (col < yhi) o[0] = acc0[r];
    }
}

// K4 table mode, long chains, round 5 (SweepArgs::ylds 3): the LDS-staged block of ypass_tlds_kernel cut finer
// for planes whose y-pass is a few hundred thousand cells of chains up to ~425 taps (the reference's own grid:
// 510 x 400, N_y 14-212). One cell per lane, so a block covers a 64-column tile (the grid's 400 columns are 7
// tiles with one 16-column tail instead of 4 strips with a 16-column tail that idled a quarter of the waves),
// and R rows per wave, so each noise value read from LDS serves R products (R = 1 makes the LDS array, not the
// FP64 pipe, the limit: profiles/r5). Blocks run in the host's order (SweepArgs::ylist): heaviest union of
// noise rows first, components and tiles interleaved, so the widest stencils (N_y 206-212 around j = 160-200)
// start first instead of wherever their rows fall.
// Waits: scalar loads return out of order, so while one is in flight every LDS wait is a full lgkmcnt(0). A
// chunk's R x C coefficients (uniform: one scalar window per row, zero taps where the window hangs past the
// row's range) are therefore loaded before the chunk's barrier, whose wait they share, and the chunk's sums
// then wait on LDS reads alone; no chunk takes a per-tap path (a scalar load and its wait per tap made a
// row's first and last chunk cost more than the rest of it). The noise loads of the chunks in flight are
// unconditional, so their vmcnt waits are counted, not zero.
// Round 6 (1.45 scalar instructions per vector one, the CU's one scalar unit busier than
// the FP64 pipe): the per-chunk bookkeeping is all increments. Each noise load has its own lane pointer advanced
// by one chunk per step (one VALU add, where a clamped row index cost four scalar instructions per load: r_ys
// now carries kYTailRows rows past its last so the loads need no clamp; rows past a block's range are summed
// with zero taps or never staged); each row's coefficient window is a scalar pointer advanced by C doubles, and
// whether the row has a tap in the chunk is a compare of the chunk index against a range fixed at the start.
// Each row adds its taps in the order i = -N..N (noise rows ascending) with df.cpp:373-375's products:
// bit-identical to every other form.
// DBG (timing ablations, wrong sums; DFAMD_YT_DEBUG): 1 no coefficient loads after chunk 0, 4 every row of a
// wave sums with row 0's window
template <int R, int NW, int C, int PD, int DBG = 0>
__global__ __launch_bounds__(64 * NW) void ypass_t64_kernel(SweepArgs a)
{
    constexpr int LP = C / (2 * NW); // pairs of chunk rows each wave loads
    static_assert(C % (2 * NW) == 0, "chunk row pairs split evenly over the waves");
    // noise rows 2p, 2p + 1 of a chunk side by side for each lane: one ds_read_b128 (4 LDS cycles for 1 KiB)
    // fetches two rows, where the compiler's ds_read2st64_b64 of two separate rows takes 8
    __shared__ dvec2 nbuf[2][C / 2][64];
    const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
    const int tile = a.ylist[blockIdx.x];
    const int nrb = a.ylist_nrb, ncol = a.ylist_ncol;
    const int rb = tile % nrb, ct = (tile / nrb) % ncol, c = tile / (nrb * ncol);
    if (!((a.comps_mask >> c) & 1)) return; // block-uniform
    const int Ny = a.Ny, RB = NW * R, j0 = rb * RB;
    const int *nst = a.Ny_st[c] + (size_t)(ct >> 1) * Ny; // tap ranges of the 128-cell strip holding the tile
    int mlo = 1 << 30, mhi = -(1 << 30);                    // the block's noise rows
    for (int q = 0; q < RB && j0 + q < Ny; ++q) {
        const int N = nst[j0 + q];
        mlo = min(mlo, j0 + q - N);
        mhi = max(mhi, j0 + q + N);
    }
    const int jw = j0 + w * R;
    // row r has a tap in chunk i (rows mlo + C i ..) for i - ilo[r] in [0, iw[r]] (unsigned: one compare); its
    // window there is cwin[r] + C i
    int ilo[R];
    unsigned iw[R];
    const double *cwin[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ilo[r] = 1 << 30; // no row: i - ilo is negative, far above iw as unsigned
        iw[r] = 0;
        cwin[r] = a.tabf;
        if (jw + r < Ny) {
            const int N = nst[jw + r], lo = jw + r - N;
            ilo[r] = (lo - mlo) / C; // lo >= mlo
            iw[r] = (unsigned)((jw + r + N - mlo) / C - ilo[r]);
            cwin[r] = a.tabf + a.tabf_off[N] + (mlo - lo); // tap t = m - lo of noise row m at tabf_off[N] + t
        }
    }
    const int col = ct * 64 + lane; // < Pz: a padding column is loaded and summed but never stored
    // The next chunk each of this wave's loads fetches: rows 2 (w + NW k) and + 1 of it, at byte offset vo[k] of
    // this lane's column from the uniform bases nb (even rows) and nb1 (odd rows): global loads with a scalar base
    // and a 32-bit vector offset (launch_ypass_t checks r_ys < 4 GiB), one vector add per pair and chunk.
    const unsigned Pz8 = (unsigned)a.Pz * 8u;
    const char *nb = reinterpret_cast<const char *>(a.ry[c]), *nb1 = nb + Pz8;
    unsigned vo[LP];
#pragma unroll
    for (int k = 0; k < LP; ++k) vo[k] = (unsigned)(a.Nyp[c] + mlo + 2 * (w + NW * k)) * Pz8 + (unsigned)col * 8u;
    dvec2 pre[PD][LP]; // wave w loads row pairs w + NW k of the chunk
    auto gload = [&](auto K) {
        constexpr int k0 = decltype(K)::value;
#pragma unroll
        for (int k = 0; k < LP; ++k) {
            pre[k0][k] = dvec2{*reinterpret_cast<const double *>(nb + vo[k]),
                               *reinterpret_cast<const double *>(nb1 + vo[k])};
            vo[k] += (unsigned)C * Pz8;
        }
    };
    auto lstore = [&](auto K, int buf) {
        constexpr int k0 = decltype(K)::value;
#pragma unroll
        for (int k = 0; k < LP; ++k) nbuf[buf][w + NW * k][lane] = pre[k0][k];
    };
    // Every live chunk takes the whole-window path: a row's window may hang past its first or last tap into the
    // table's zero guards (kTabGuard >= C, df_capi.cpp upload_tables); zero taps leave each sum bit for bit.
    bool liv[R];
    auto live = [&](int i) {
        bool f = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            liv[r] = (unsigned)(i - ilo[r]) <= iw[r];
            f = f || liv[r];
        }
        return f;
    };
    double cw[R][C]; // the chunk's coefficients (uniform), loaded whether or not the chunk is live (no branch)
    auto cload = [&](int i) {
#pragma unroll
        for (int r = 0; r < (DBG == 4 ? 1 : R); ++r) {
            const double *src = liv[r] ? cwin[r] + i * C : a.tabf; // a.tabf: kTabGuard zeros
#pragma unroll
            for (int q = 0; q < C; ++q) cw[r][q] = src[q];
        }
    };
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0;
    auto compute = [&](int buf, bool on) {
        if (!on) return;
#pragma unroll
        for (int p = 0; p < C / 2; ++p) {
            const dvec2 n = nbuf[buf][p][lane];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] += cw[DBG == 4 ? 0 : r][2 * p] * n.x;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] += cw[DBG == 4 ? 0 : r][2 * p + 1] * n.y;
        }
    };
    // chunk i: rows mlo + C i ..; its loads in register set i % PD, its sums from LDS buffer i % 2 (as
    // ypass_tlds_kernel); its coefficients (full chunks) loaded before the barrier that precedes it
    const int nch = (mhi - mlo) / C + 1;
    // prologue: chunks 0 .. PD - 1 in flight, chunk 0 staged
    unroll_to<0, PD>([&](auto K) { gload(K); });
    lstore(ic_t<0>{}, 0);
    bool on = live(0);
    cload(0);
    __syncthreads();
    // Steps run in whole groups of PD: a step past the last chunk stages rows no row has a tap in (on is false
    // from there: every ilo + iw < nch) and sums nothing. Its loads reach at most 2 PD C - 1 rows past the block's
    // last (<= 127 < kYTailRows).
    auto step = [&](auto K, int i) {
        constexpr int k = decltype(K)::value;
        // chunk i + PD into the set chunk i left - unconditionally, so the count of loads in flight is fixed and
        // the waits below are counted vmcnt(n), not vmcnt(0)
        gload(K);
        compute(i & 1, on);
        lstore(ic_t<(k + 1) % PD>{}, (i + 1) & 1);
        on = live(i + 1);
        if constexpr (DBG != 1) cload(i + 1);
        __syncthreads();
    };
    for (int i = 0; i < nch; i += PD) unroll_to<0, PD>([&](auto K) { step(K, i + decltype(K)::value); });
    if (col < a.ylo[c] || col >= a.yhi[c]) return;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (jw + r >= Ny) continue;
        double *o = a.rz[c] + (size_t)(jw + r) * a.rz_pitch[c] + a.yout[c] + col;
        if (a.ynt_stores) __builtin_nontemporal_store(acc[r], o);
        else *o = acc[r];
    }
}

template <int R, bool TABLE> static hipError_t launch_ypass_t(const SweepArgs &a, hipStream_t st)
{
    if constexpr (TABLE) {
        if (a.ylds == 3 && !a.per_cell) { // 64-column tiles, heaviest first; rows per wave from ylist_R
            const dim3 grid((unsigned)a.ylist_n);
            for (int c = 0; c < 3; ++c) // 32-bit byte offsets into r_ys (df_capi.cpp t64_fits)
                if ((double)(a.Ny + 2 * a.Nyp[c] + kYTailRows) * a.Pz * 8.0 >= 4294967296.0) return hipErrorInvalidValue;
            // R x C coefficients of a chunk held in SGPRs (24 doubles at most: more spill)
            // measured on the reference's grid (profiles/r5): 1 x 16 24.7-25.1 us, 1 x 24 26.6 (the call beside the
            // RNG -2%, profiles/r5/p), 2 x 16 26.6, 2 x 8 35-39, the round-4 ypass_tlds 40.4; 4 chunks in flight lose
            // (VGPRs 38 -> 114) except on a lone block
            if (a.ylist_dbg && a.ylist_C == 16 && a.ylist_PD == 2) { // timing ablations (DFAMD_YT_DEBUG)
                if (a.ylist_dbg == 1 && a.ylist_R == 1) hipLaunchKernelGGL((ypass_t64_kernel<1, 4, 16, 2, 1>), grid, dim3(256), 0, st, a);
                else if (a.ylist_dbg == 1 && a.ylist_R == 2) hipLaunchKernelGGL((ypass_t64_kernel<2, 4, 16, 2, 1>), grid, dim3(256), 0, st, a);
                else if (a.ylist_dbg == 4 && a.ylist_R == 2) hipLaunchKernelGGL((ypass_t64_kernel<2, 4, 16, 2, 4>), grid, dim3(256), 0, st, a);
                else return hipErrorInvalidValue;
                return hipGetLastError();
            }
            switch (a.ylist_R * 1000 + a.ylist_C * 10 + a.ylist_PD) {
            case 1162: hipLaunchKernelGGL((ypass_t64_kernel<1, 4, 16, 2>), grid, dim3(256), 0, st, a); break;
            case 1164: hipLaunchKernelGGL((ypass_t64_kernel<1, 4, 16, 4>), grid, dim3(256), 0, st, a); break;
            case 1242: hipLaunchKernelGGL((ypass_t64_kernel<1, 4, 24, 2>), grid, dim3(256), 0, st, a); break;
            case 2082: hipLaunchKernelGGL((ypass_t64_kernel<2, 4, 8, 2>), grid, dim3(256), 0, st, a); break;
            case 2162: hipLaunchKernelGGL((ypass_t64_kernel<2, 4, 16, 2>), grid, dim3(256), 0, st, a); break;
            default: return hipErrorInvalidValue; // df_set_tuning admits the pairs above only
            }
            return hipGetLastError();
        }
        if (a.ylds && !a.per_cell) {
            const int nrowblk = (a.Ny + 4 * R - 1) / (4 * R);
            const unsigned blocks = (unsigned)(((long long)a.nstrips * nrowblk + 7) / 8 * 8);
            // 4 and 8 rows per wave take one chunk in flight: with 2-3 the compiler puts their arrays in scratch
            if (R <= 2) hipLaunchKernelGGL((ypass_tlds_kernel<R <= 2 ? R : 1, 2>), dim3(blocks, 3), dim3(256), 0, st, a, nrowblk);
            else hipLaunchKernelGGL((ypass_tlds_kernel<R, 1>), dim3(blocks, 3), dim3(256), 0, st, a, nrowblk);
            return hipGetLastError();
        }
    }
    const int nrowblk = (a.Ny + R - 1) / R;
    const long long tiles = (long long)a.nstrips * nrowblk;
    const unsigned blocks = (unsigned)(((tiles + 3) / 4 + 7) / 8 * 8); // multiple of 8 for the XCD swizzle
    const dim3 grid(blocks, 3);
    if constexpr (TABLE) {
        if (a.per_cell) {
            hipLaunchKernelGGL((ypass_kernel<R, true, false, 2, true>), grid, dim3(256), 0, st, a, nrowblk);
        } else {
            constexpr int KYD = R <= 2 ? 4 : R == 4 ? 2 : 1;
            hipLaunchKernelGGL((ypass_table_kernel<R, KYD>), grid, dim3(256), 0, st, a, nrowblk);
        }
    } else if (a.yunroll >= 8) {
        hipLaunchKernelGGL((ypass_kernel<R, false, true, 8, false>), grid, dim3(256), 0, st, a, nrowblk);
    } else if (a.yunroll >= 4) {
        hipLaunchKernelGGL((ypass_kernel<R, false, true, 4, false>), grid, dim3(256), 0, st, a, nrowblk);
    } else {
        hipLaunchKernelGGL((ypass_kernel<R, false, true, 2, false>), grid, dim3(256), 0, st, a, nrowblk);
    }
    return hipGetLastError();
}

hipError_t launch_ypass(const SweepArgs &a, bool table, int rows_per_wave, hipStream_t st)
{
    if (!table && a.ycoop >= 7) { // row pairs, 4 noise rows per wave per chunk (32 KiB LDS)
        const dim3 grid((unsigned)(8 * a.ycoop2_run), 3);
        hipLaunchKernelGGL((ypass_coop2_kernel<true, 4>), grid, dim3(256), 0, st, a);
        return hipGetLastError();
    }
    switch (rows_per_wave) {
    case 1: return table ? launch_ypass_t<1, true>(a, st) : launch_ypass_t<1, false>(a, st);
    case 2: return table ? launch_ypass_t<2, true>(a, st) : launch_ypass_t<2, false>(a, st);
    case 4: return table ? launch_ypass_t<4, true>(a, st) : launch_ypass_t<4, false>(a, st);
    default: return table ? launch_ypass_t<8, true>(a, st) : launch_ypass_t<8, false>(a, st);
    }
}

// ------------------------------------------------------ K5 z-pass + epilogue

// Lane l owns cells col = 2l, 2l+1 of the strip; tap i needs x[col+i] and
// x[col+1+i]. With N even, pairs P_m = (x[col-N+2m], x[col-N+2m+1]) are 16-B
// aligned: even tap -N+2m uses P_m, odd tap -N+2m+1 uses (P_m.y, P_{m+1}.x), so
// one 16-B noise load serves two taps and the order i = -N..N is unchanged.
// SPLIT (packed planes with few tiles per SIMD; SweepArgs::zsplit): one 3-wave block per tile, wave c
// sums component c's taps, the three sums meet in LDS and wave 0 runs the epilogue - three times the
// waves in flight for the same bytes. Same sums, same epilogue: bit-identical.
// Table z-pass staging: row j's noise of strips [s0, s0 + ns) plus N columns either side, per
// component, into LDS regions of a.zstage_reg doubles. zstage 2: 16-B copies with each thread's loads
// (up to 3 per component) all issued before its LDS stores, so a block waits for one round trip
// instead of one per element; rows start 16-B aligned (pitch, Nzp and N even), checked per block.
__device__ __forceinline__ void zstage_copy(const SweepArgs &a, double *lds, int j, int s0, int ns, int nthr)
{
    const int tid = threadIdx.x;
    const double *src[3];
    int cnt[3];
    bool vec = a.zstage >= 2;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        cnt[c] = 0;
        src[c] = nullptr;
        if (!((a.comps_mask >> c) & 1)) continue;
        const int N = a.Nz_st[c][(size_t)s0 * a.Ny + j];
        src[c] = a.rz[c] + (size_t)j * a.rz_pitch[c] + a.Nzp[c] + s0 * kStrip - N;
        cnt[c] = ns * kStrip + 2 * N;
        vec = vec && ((uintptr_t)src[c] & 15) == 0 && (cnt[c] & 1) == 0;
    }
    if (!vec) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
            for (int e = tid; e < cnt[c]; e += nthr) lds[c * a.zstage_reg + e] = src[c][e];
        return;
    }
    double2 v[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int e = tid + k * nthr;
            if (e < cnt[c] / 2) v[c][k] = reinterpret_cast<const double2 *>(src[c])[e];
        }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        dvec2 *d = reinterpret_cast<dvec2 *>(lds + c * a.zstage_reg); // zstage_reg even: 16-B regions
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int e = tid + k * nthr;
            if (e < cnt[c] / 2) d[e] = dvec2{v[c][k].x, v[c][k].y};
        }
        for (int e = tid + 3 * nthr; e < cnt[c] / 2; e += nthr) { // wide stencils: the rest
            const double2 x = reinterpret_cast<const double2 *>(src[c])[e];
            d[e] = dvec2{x.x, x.y};
        }
    }
}

template <bool TABLE, bool NT, int ZU, bool PC, bool SPLIT = false>
__global__ __launch_bounds__(256) void zpass_kernel(SweepArgs a)
{
    extern __shared__ double zstage_lds[]; // 3 x zstage_reg doubles when a.zstage (table mode)
    const int lane = threadIdx.x & 63;
    const int Ny = a.Ny, nst = a.zs_n; // this launch's strips (SweepArgs::zs_lo ...)
    int j, s;
    bool staged = false;
    if (TABLE && !PC && a.zgroup) {
        // Table mode, launches without a strip gap: block = (row, group of <= 4 consecutive strips), wave w =
        // strip 4 g + w, so no block straddles two rows (a z-strip rank's 6 interior strips per row are groups
        // of 4 and 2, not blocks across rows). Where the group's strips share one tap range per component the
        // block stages that row's noise (128 ns + 2N columns per component) in LDS once and the waves read
        // their tap pairs from there (ds_read_b128) instead of overlapping (128 + 2N)-column windows through
        // L1. Block-uniform: the barrier is reached by all; waves past the group leave after the copy.
        const int ngrp = (nst + 3) >> 2;
        const int jj = (int)blockIdx.x / ngrp, g = (int)blockIdx.x - jj * ngrp;
        if (jj >= Ny) return; // block-uniform
        j = Ny - 1 - jj;      // wide stencils first
        const int s0 = a.zs_lo + 4 * g, ns = min(4, nst - 4 * g), w = uniform(threadIdx.x >> 6);
        s = s0 + w;
        staged = a.zstage != 0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (!staged || !((a.comps_mask >> c) & 1)) continue;
            const int *nz = a.Nz_st[c] + (size_t)s0 * Ny + j;
            for (int k = 1; k < ns; ++k) staged = staged && nz[(size_t)k * Ny] == nz[0];
        }
        if (staged) {
            zstage_copy(a, zstage_lds, j, s0, ns, 256);
            __syncthreads();
        }
        if (w >= ns) return;
    } else {
        const int tile = SPLIT ? (int)blockIdx.x : uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
        if (tile >= nst * Ny) return; // block-uniform when SPLIT
        const int jj = tile / nst;
        const int sl = tile - jj * nst;
        s = a.zs_lo + sl + (sl >= a.zs_gap_at ? a.zs_gap : 0);
        j = Ny - 1 - jj; // wide stencils first
    }
    const int col = s * kStrip + 2 * lane;
    // padding lanes leave (after their share of the staging copy); SPLIT keeps them to the barrier
    // (their loads stay inside the padded strip: B holds 128 cells per strip, r_zs Pz + 2 Nzp columns)
    if (!SPLIT && col >= a.Nz_loc) return;
    const int wv = uniform(threadIdx.x >> 6);

    double f0[3], f1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        f0[c] = f1[c] = 0.0;
        if (!((a.comps_mask >> c) & 1)) continue;
        if (SPLIT && c != wv) continue;
        const int N = a.Nz_st[c][(size_t)s * Ny + j];
        const double2 *gxp = reinterpret_cast<const double2 *>(a.rz[c] + (size_t)j * a.rz_pitch[c] + a.Nzp[c] + col - N);
        const double *bp = TABLE ? nullptr : a.Bz[c] + a.bzoff[c][(size_t)s * Ny + j] + 2 * lane; // tap t = i + N
        const double *tb = nullptr, *tb1 = nullptr;
        if (TABLE && PC) { // per-lane N; the table is zero past each N (taps up to N_st)
            const int *nc = a.Nz_cell[c] + (size_t)j * a.Nz_loc;
            tb = a.tab + a.tab_off[col < a.Nz_loc ? nc[col] : 0];
            tb1 = a.tab + a.tab_off[col + 1 < a.Nz_loc ? nc[col + 1] : 0];
        } else if (TABLE) {
            tb = a.tabf + a.tabf_off[N]; // full vector: tap t at tb[t]
        }
        auto coef = [&](int t) -> double2 {
            if (TABLE) {
                if (!PC) {
                    const double v = tb[t];
                    return make_double2(v, v);
                }
                const int i = t - N, ai = i < 0 ? -i : i;
                return make_double2(tb[ai], tb1[ai]);
            }
            return ldB<NT>(bp + (ptrdiff_t)t * kStrip);
        };
        // one instantiation per address space: global (plain loads) or LDS (ds_read_b128)
        auto taps = [&](auto xp, double &r0, double &r1) {
        double acc0 = 0.0, acc1 = 0.0;
        double2 P = ld_pair(xp);
        int m = 0;
        if (ZU >= 4) {
            for (; m + 4 <= N; m += 4) { // 8 taps: 8 coefficient loads + 4 noise pairs in flight
                const double2 P1 = ld_pair(xp + m + 1), P2 = ld_pair(xp + m + 2), P3 = ld_pair(xp + m + 3), P4 = ld_pair(xp + m + 4);
                double2 b[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) b[u] = coef(2 * m + u);
                acc0 += b[0].x * P.x;
                acc1 += b[0].y * P.y;
                acc0 += b[1].x * P.y;
                acc1 += b[1].y * P1.x;
                acc0 += b[2].x * P1.x;
                acc1 += b[2].y * P1.y;
                acc0 += b[3].x * P1.y;
                acc1 += b[3].y * P2.x;
                acc0 += b[4].x * P2.x;
                acc1 += b[4].y * P2.y;
                acc0 += b[5].x * P2.y;
                acc1 += b[5].y * P3.x;
                acc0 += b[6].x * P3.x;
                acc1 += b[6].y * P3.y;
                acc0 += b[7].x * P3.y;
                acc1 += b[7].y * P4.x;
                P = P4;
            }
        }
        for (; m + 2 <= N; m += 2) {
            const double2 P1 = ld_pair(xp + m + 1), P2 = ld_pair(xp + m + 2);
            const double2 b0 = coef(2 * m), b1 = coef(2 * m + 1), b2 = coef(2 * m + 2), b3 = coef(2 * m + 3);
            acc0 += b0.x * P.x;
            acc1 += b0.y * P.y;
            acc0 += b1.x * P.y;
            acc1 += b1.y * P1.x;
            acc0 += b2.x * P1.x;
            acc1 += b2.y * P1.y;
            acc0 += b3.x * P1.y;
            acc1 += b3.y * P2.x;
            P = P2;
        }
        for (; m < N; ++m) {
            const double2 P1 = ld_pair(xp + m + 1);
            const double2 b0 = coef(2 * m), b1 = coef(2 * m + 1);
            acc0 += b0.x * P.x;
            acc1 += b0.y * P.y;
            acc0 += b1.x * P.y;
            acc1 += b1.y * P1.x;
            P = P1;
        }
        const double2 bl = coef(2 * N);
        acc0 += bl.x * P.x;
        acc1 += bl.y * P.y;
        r0 = acc0;
        r1 = acc1;
        };
        if (TABLE && !PC && staged) {
            taps((lds_pair_ptr)(zstage_lds + c * a.zstage_reg + (threadIdx.x >> 6) * kStrip + 2 * lane), f0[c], f1[c]);
        } else {
            taps(gxp, f0[c], f1[c]);
        }
    }

    if constexpr (SPLIT) {
        __shared__ double2 zsplit_part[3][64];
        double2 mine = make_double2(0.0, 0.0);
#pragma unroll
        for (int c = 0; c < 3; ++c)
            if (c == wv) mine = make_double2(f0[c], f1[c]);
        zsplit_part[wv][lane] = mine;
        __syncthreads();
        if (wv != 0) return;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double2 v = zsplit_part[c][lane];
            f0[c] = v.x;
            f1[c] = v.y;
        }
    }

    if (a.write_filt) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (!((a.comps_mask >> c) & 1)) continue;
            const size_t idx = (size_t)j * a.Nz_loc + col;
            if (col < a.Nz_loc) a.filt[c][idx] = f0[c];
            if (col + 1 < a.Nz_loc) a.filt[c][idx + 1] = f1[c];
        }
        return;
    }
    if (col >= a.Nz_loc) return;
    const double *rc = a.rowc;
    const double sR11 = rc[j], bb = rc[Ny + j], sR22b = rc[2 * Ny + j], sR33 = rc[3 * Ny + j];
    const double t1 = rc[4 * Ny + j], Ts = rc[5 * Ny + j], rh = rc[6 * Ny + j];
    // The lane's two cells as one 16-B access per field when the row offset keeps them
    // aligned (every row when Nz_loc is even), else two 8-B accesses.
    const size_t idx = (size_t)j * a.Nz_loc + col;
    const bool has1 = col + 1 < a.Nz_loc, pair = has1 && (idx & 1) == 0;
    auto ld = [&](const double *p) -> double2 {
        if (pair) return *reinterpret_cast<const double2 *>(p + idx);
        return make_double2(p[idx], has1 ? p[idx + 1] : 0.0);
    };
    auto st = [&](double *p, double x, double y) {
        if (pair) {
            if (a.nt_stores) __builtin_nontemporal_store(dvec2{x, y}, reinterpret_cast<dvec2 *>(p + idx));
            else *reinterpret_cast<double2 *>(p + idx) = make_double2(x, y);
            return;
        }
        p[idx] = x;
        if (has1) p[idx + 1] = y;
    };
    double fu[2] = {f0[0], f1[0]}, fv[2] = {f0[1], f1[1]}, fw[2] = {f0[2], f1[2]};
    if (a.do_corr) { // df.cpp:415
        const double2 ou = ld(a.filt_old[0]), ov = ld(a.filt_old[1]), ow = ld(a.filt_old[2]);
        write_window(a.zwin_T, a.zwin_W); // the filt_old loads are in flight meanwhile
        const double o[3][2] = {{ou.x, ou.y}, {ov.x, ov.y}, {ow.x, ow.y}};
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            fu[e] = o[0][e] * a.sa[0] + fu[e] * a.s1a[0];
            fv[e] = o[1][e] * a.sa[1] + fv[e] * a.s1a[1];
            fw[e] = o[2][e] * a.sa[2] + fw[e] * a.s1a[2];
        }
    }
    else
        write_window(a.zwin_T, a.zwin_W);
    double up[2], vp[2], wp[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        up[e] = sR11 * fu[e];              // df.cpp:436
        vp[e] = bb * fu[e] + sR22b * fv[e]; // df.cpp:437
        wp[e] = sR33 * fw[e];              // df.cpp:438
    }
    st(a.fluc[0], up[0], up[1]);
    st(a.fluc[1], vp[0], vp[1]);
    st(a.fluc[2], wp[0], wp[1]);
    st(a.filt_old[0], fu[0], fu[1]); // df.cpp:440-442
    st(a.filt_old[1], fv[0], fv[1]);
    st(a.filt_old[2], fw[0], fw[1]);
    if (a.do_sra) { // df.cpp:474-481
        double T2[2], R2[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const double t2 = t1 * up[e];
            T2[e] = t2 * Ts;
            R2[e] = -t2 * rh;
        }
        st(a.T, T2[0], T2[1]);
        st(a.rho, R2[0], R2[1]);
    }
}

hipError_t launch_zpass(const SweepArgs &a, bool table, hipStream_t st)
{
    const long long tiles = (long long)a.zs_n * a.Ny;
    if (tiles <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)((tiles + 3) / 4);
    if (table && a.per_cell) {
        hipLaunchKernelGGL((zpass_kernel<true, false, 4, true>), dim3(blocks), dim3(256), 0, st, a);
    } else if (table) {
        const size_t lds = a.zstage && a.zgroup ? 3 * (size_t)a.zstage_reg * sizeof(double) : 0;
        const dim3 grid(a.zgroup ? (unsigned)(a.Ny * ((a.zs_n + 3) / 4)) : blocks);
        hipLaunchKernelGGL((zpass_kernel<true, false, 4, false>), grid, dim3(256), lds, st, a);
    } else if (a.zsplit) { // packed, one 3-wave block per tile
        hipLaunchKernelGGL((zpass_kernel<false, true, 4, false, true>), dim3((unsigned)tiles), dim3(192), 0, st, a);
    } else {
        hipLaunchKernelGGL((zpass_kernel<false, true, 4, false>), dim3(blocks), dim3(256), 0, st, a);
    }
    return hipGetLastError();
}

// ------------------------------------------------- stage API elementwise ops

__global__ void stage_kernel(SweepArgs a, int op, int comp)
{
    const size_t n = (size_t)a.Ny * a.Nz_loc;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x) {
        const int j = (int)(idx / a.Nz_loc);
        const double *rc = a.rowc;
        if (op == 0) {
            a.filt[comp][idx] = a.filt_old[comp][idx] * a.sa[comp] + a.filt[comp][idx] * a.s1a[comp];
        } else if (op == 1) {
            const double fu = a.filt[0][idx], fv = a.filt[1][idx], fw = a.filt[2][idx];
            a.fluc[0][idx] = rc[j] * fu;
            a.fluc[1][idx] = rc[a.Ny + j] * fu + rc[2 * a.Ny + j] * fv;
            a.fluc[2][idx] = rc[3 * a.Ny + j] * fw;
            a.filt_old[0][idx] = fu;
            a.filt_old[1][idx] = fv;
            a.filt_old[2][idx] = fw;
        } else {
            const double t2 = rc[4 * a.Ny + j] * a.fluc[0][idx];
            a.T[idx] = t2 * rc[5 * a.Ny + j];
            a.rho[idx] = -t2 * rc[6 * a.Ny + j];
        }
    }
}

hipError_t launch_stage(const SweepArgs &a, int op, int comp, hipStream_t st)
{
    hipLaunchKernelGGL(stage_kernel, dim3(1024), dim3(256), 0, st, a, op, comp);
    return hipGetLastError();
}

// ------------------------------------------------------------ statistics

__global__ void rms_add_kernel(SweepArgs a, double *__restrict__ acc)
{
    const size_t n = (size_t)a.Ny * a.Nz_loc;
    const double *src[5] = {a.fluc[0], a.fluc[1], a.fluc[2], a.T, a.rho};
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int f = 0; f < 5; ++f) {
            const double x = src[f][idx];
            acc[f * n + idx] += x * x;
        }
    }
}

__global__ void rms_finish_kernel(const double *__restrict__ acc, double *__restrict__ out, size_t n, double count)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = sqrt(acc[i] / count);
}

hipError_t launch_rms_add(const SweepArgs &a, double *acc, hipStream_t st)
{
    hipLaunchKernelGGL(rms_add_kernel, dim3(2048), dim3(256), 0, st, a, acc);
    return hipGetLastError();
}

hipError_t launch_rms_finish(const double *acc, double *out, size_t n, double count, hipStream_t st)
{
    hipLaunchKernelGGL(rms_finish_kernel, dim3(1024), dim3(256), 0, st, acc, out, n, count);
    return hipGetLastError();
}

// ------------------------------------------------------------ K6 z-halo

__global__ void halo_pack_kernel(SweepArgs a, double *__restrict__ sl, double *__restrict__ sr)
{
    size_t base = 0;
    for (int c = 0; c < 3; ++c) {
        const int W = a.Nzp[c];
        const size_t n = (size_t)a.Ny * W;
        for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
            const int j = (int)(e / W), kk = (int)(e - (size_t)j * W);
            const int w = a.halo_w[c] ? a.halo_w[c][j] : W;
            if (kk >= w) continue;
            const size_t o = base + (a.halo_w[c] ? (size_t)a.halo_off[c][j] : (size_t)j * W) + kk;
            const double *row = a.rz[c] + (size_t)j * a.rz_pitch[c] + a.Nzp[c];
            if (sl) sl[o] = row[kk];              // to rank - 1: this strip's first w columns
            if (sr) sr[o] = row[a.Nz_loc - w + kk]; // to rank + 1: its last w
        }
        base += a.halo_w[c] ? (size_t)a.halo_off[c][a.Ny] : n;
    }
}

__global__ void halo_unpack_kernel(SweepArgs a, const double *__restrict__ rl, const double *__restrict__ rr)
{
    size_t base = 0;
    for (int c = 0; c < 3; ++c) {
        const int W = a.Nzp[c];
        const size_t n = (size_t)a.Ny * W;
        for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
            const int j = (int)(e / W), kk = (int)(e - (size_t)j * W);
            const int w = a.halo_w[c] ? a.halo_w[c][j] : W;
            if (kk >= w) continue;
            const size_t o = base + (a.halo_w[c] ? (size_t)a.halo_off[c][j] : (size_t)j * W) + kk;
            double *row = a.rz[c] + (size_t)j * a.rz_pitch[c];
            if (rl) row[W - w + kk] = rl[o];              // left pad: the w columns just left of the strip
            if (rr) row[a.Nzp[c] + a.Nz_loc + kk] = rr[o]; // right pad: the w columns just right of it
        }
        base += a.halo_w[c] ? (size_t)a.halo_off[c][a.Ny] : n;
    }
}

// ------------------------------------------------------------ K7 coupling handoff

// dst[dst_cell[i]] = beta * dst[dst_cell[i]] + src[plane_cell[i]] (identity where an index array is null).
__global__ void gather_kernel(const double *__restrict__ src, long long nsrc, long long n,
                              const long long *__restrict__ pidx, double *__restrict__ dst,
                              const long long *__restrict__ didx, long long ndst, double beta, int *bad)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const long long p = pidx ? pidx[i] : i;
        const long long d = didx ? didx[i] : i;
        if (p < 0 || p >= nsrc || d < 0 || d >= ndst) {
            atomicAdd(bad, 1);
            continue;
        }
        const double v = src[p];
        dst[d] = beta == 0.0 ? v : beta * dst[d] + v;
    }
}

hipError_t launch_gather(const double *src, long long nsrc, long long n, const long long *pidx, double *dst,
                         const long long *didx, long long ndst, double beta, int *bad, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    const long long want = (n + 255) / 256;
    const int blocks = (int)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, st, src, nsrc, n, pidx, dst, didx, ndst, beta, bad);
    return hipGetLastError();
}

hipError_t launch_halo_pack(const SweepArgs &a, double *send_l, double *send_r, hipStream_t st)
{
    hipLaunchKernelGGL(halo_pack_kernel, dim3(512), dim3(256), 0, st, a, send_l, send_r);
    return hipGetLastError();
}

// One-rank RCCL loopback (tuning key halo_loopback): the halo columns a rank sent to itself must
// arrive unchanged; mismatches are counted into *bad. corrupt = 1 perturbs element 0 as received
// (a test of the check itself).
__global__ void halo_check_kernel(const double *__restrict__ sent, const double *__restrict__ got, size_t n, int corrupt,
                                  int *bad)
{
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const double g = got[e] + ((corrupt && e == 0) ? 1.0 : 0.0);
        if (g != sent[e] && !(g != g && sent[e] != sent[e])) atomicAdd(bad, 1);
    }
}

// Timing only (DFAMD_SOLO_XCHG_US): one wave that holds its stream for `ticks` of the 100 MHz real-time
// clock, standing in for the exchange of a solo-strip handle. Bounded: at most 2^20 sleeps (~60 ms).
__global__ void hold_kernel(unsigned long long ticks)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < (1 << 20); ++it) {
        if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
}

hipError_t launch_hold(double us, hipStream_t st)
{
    hold_kernel<<<1, 64, 0, st>>>((unsigned long long)(us * 100.0));
    return hipGetLastError();
}

hipError_t launch_halo_check(const double *sent, const double *got, size_t n, int corrupt, int *bad, hipStream_t st)
{
    hipLaunchKernelGGL(halo_check_kernel, dim3(256), dim3(256), 0, st, sent, got, n, corrupt, bad);
    return hipGetLastError();
}

hipError_t launch_halo_unpack(const SweepArgs &a, const double *recv_l, const double *recv_r, hipStream_t st)
{
    hipLaunchKernelGGL(halo_unpack_kernel, dim3(512), dim3(256), 0, st, a, recv_l, recv_r);
    return hipGetLastError();
}

} // namespace dfamd
