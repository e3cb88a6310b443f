// C ABI of libdfamd.so (include/df_c.h): host orchestration of the MI355X
// filter(dt) path. One handle = one GPU = one z-strip of the inflow plane.
//
// Per df_filter call (reference df.cpp:449-468), all on the handle's stream:
//   rng_count -> rng_scan -> rng_generate      generate_white_noise (332-349)
//   ypass (u,v,w in one launch)                filtering_sweeps y-part (359-383)
//   [halo pack -> RCCL send/recv -> unpack]    only when the plane is split
//   zpass_epilogue (u,v,w in one launch)       z-part (385-405) + correlate_fields
//                                              (408-417) + apply_RST_scaling
//                                              (419-447) + get_rho_T_fluc (470-485)
#include "df_c.h"
#include "df_kernels.hpp"
#include "df_rng.hpp"
#include "df_setup.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

using namespace dfamd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

// On failure the HIP error is also cleared from the thread's last-error slot, so that a later, healthy
// launch check (hipGetLastError) does not report it again.
#define HIP_OR(expr, code)                                                                                  \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess) {                                                                             \
            (void)hipGetLastError();                                                                        \
            return fail(code, std::string(#expr) + ": " + hipGetErrorString(e_));                          \
        }                                                                                                   \
    } while (0)

#define NCCL_OR(expr)                                                                                       \
    do {                                                                                                    \
        ncclResult_t r_ = (expr);                                                                           \
        if (r_ != ncclSuccess) return fail(DF_ECOMM, std::string(#expr) + ": " + ncclGetErrorString(r_));   \
    } while (0)

// Run generation share record (RngGeom::xbuf): 64 group counts per block, int32 block prefixes, int64 total.
void record_layout(long long chunk, long long *stride, long long *lp_off, long long *tot_off)
{
    *lp_off = chunk * 64;
    *tot_off = (*lp_off + chunk * 4 + 7) / 8 * 8;
    *stride = (*tot_off + 8 + 15) / 16 * 16;
}

struct CompDev {
    int Nyp = 0, Nzp = 0, rz_pitch = 0;
    int *halo_w = nullptr;          // z-strips: halo columns per row (alloc_halo)
    long long *halo_off = nullptr;  // and their offsets in the packed halo (Ny + 1)
    double *ry[kMaxNoiseSets] = {}, *rz[kMaxNoiseSets] = {}; // noise set g % nsets feeds generation g
    double *By = nullptr, *Bz = nullptr;
    long long *byoff = nullptr, *bzoff = nullptr;
    int *Ny_st = nullptr, *Nz_st = nullptr;     // tap range per (strip, row), [s*Ny + j]
    int *Ny_st_g = nullptr;                     // the same over the strip widened by its ghost columns
    int *Ny_cell = nullptr, *Nz_cell = nullptr; // per-cell N of this strip (grid planes only)
    double *filt_old = nullptr, *fluc = nullptr, *filt = nullptr;
    long long by_elems = 0, bz_elems = 0; // strip-tap-major element counts
    long long by_size = 0, bz_size = 0;   // reference offset-packed sizes (this strip's cells)
    int ycoop2_xcd[9] = {};               // row-pair y-pass tiles of XCD x: [ycoop2_xcd[x], ycoop2_xcd[x+1])
    int *ycoop2_perm = nullptr;           // row-pair y-pass: dispatch position -> item code (balance_ycoop2)
    double sa = 0, s1a = 0;
};

struct PhaseEvents {
    hipEvent_t e[6]; // main stream: start, after ypass, after halo, after zpass; RNG stream: start, end
    bool rng = false;
    bool ahead = false; // the call's y-pass ran ahead on ystream (timed by YEvents, not e[0] -> e[1])
    int gens = 0; // generations enqueued during the call: e[4] before the first, e[5] after the last
};

// An epoch's y-passes run ahead on ystream, timed as one span (profiling)
struct YEvents {
    hipEvent_t e[2];
    int n = 0; // y-passes between e[0] and e[1]
};

} // namespace

struct df_handle {
    Flow flow;
    PlaneSpec spec;
    Setup setup;
    int coeff_mode = DF_COEFF_PACKED;
    std::string csv_path;
    int device = 0;
    hipStream_t stream = nullptr;     // sweeps (memory-bound)
    hipStream_t rng_stream = nullptr; // noise generation for the NEXT call (compute-bound), overlapped
    hipEvent_t ev_rng[2] = {}, ev_release[kMaxNoiseSets] = {}; // release: one per epoch slot (epoch_slots)
    // Y-pass ahead (round 5): the y-pass reads only its generation's r_ys and writes only that set's r_zs
    // interior, and depends on nothing a call changes, so it runs on ystream as soon as its epoch's noise is
    // ready, calls ahead of the call that consumes it; the stream then waits for ev_swept instead of ev_rng and
    // runs the halo and the z-pass alone. ep_swept: the epoch (by parity) was swept ahead; cur_swept: the
    // current step's set was.
    int yahead = 0;
    hipStream_t ystream = nullptr;
    hipEvent_t ev_swept[2] = {};
    bool ep_swept[2] = {false, false};
    bool cur_swept = false;
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    int Nz_g = 0, z0 = 0, z1 = 0, Nz_loc = 0, nstrips = 0, Pz = 0, Ny = 0;
    int rows_per_wave = 8;
    int yunroll = 2, zunroll = 4; // z: 8 taps per step (-1..3% against 4; 16 taps +0..6%, profiles/r5/zu)
    int nt_stores = 1; // outputs streamed past the caches (same-handle A/B: -1.5% per call)
    int ynt_stores = 1; // the y-pass output likewise
    int ywin_T = 0, ywin_W = 0, zwin_T = 0, zwin_W = 0; // sweep write windows (SweepArgs)
    // table z-pass noise staged in LDS; 2 (default): 16-B copies, every load issued before the LDS stores
    // (c3 table z-pass 0.142 -> 0.129 ms, call -2.5%; profiles/r2/ab_zstage2_zquad_table.jsonl)
    int zstage = 2;
    int fuse_plan = 0; // small planes: K3 plans its own waves, no K2/K2c launch (RngGeom::fused_plan)
    // Dense generation (RngGeom::gen_dense: compaction through memory, one wave per needed 64-rank chunk,
    // near-1 log lanes deferred). Default in table mode (VALU-bound, where K3's skeleton costs); packed
    // keeps the compacted K3 (its RNG hides under the HBM-bound sweeps; the dense form adds 2 x 8 B per
    // stored pair of traffic). Never on planes that use fused_plan or gen_split > 1 (small planes).
    int gen_dense = 0;
    int ycoop = 0;     // packed y-pass, block-cooperative tiles (set for long tap chains in plan_strips)
    int zsplit = 0;    // packed z-pass, a wave per component (set for planes with few tiles in plan_strips)
    int ycoop_ovh = 0; // row-pair y-pass: per-tile cost in full-strip taps when balancing the XCD runs
    int ycoop_order = 0; // row-pair y-pass dispatch order within an XCD run: 0 ascending rows, g >= 1 groups of g
                         // consecutive tiles, heaviest group first (balance_ycoop2)
    int ycoop_split = 0; // row-pair y-pass: tiles whose widest row has N >= ycoop_split run as two 64-column halves
                         // (two blocks, each half the chunks of the tile's chain); 0 = never
    int ycoop_split4 = 0; // ... and those with N >= ycoop_split4 as four 32-column quarters; 0 = never
    std::vector<int> y_nst[3]; // host copy of Ny_st (tap range per strip and row) for balance_ycoop2
    std::vector<int> ycoop2_perm_host[3]; // balance_ycoop2's dispatch order (uploaded to CompDev::ycoop2_perm)
    // z-strips: 1 = every rank counts every attempt block, so the halo send/recv is the call's only
    // collective (SURVEY 8e option B, north star "single RCCL halo exchange"; the packed default).
    // 0 = split counting plus a per-call all-gather of block and wave counts (option A), ordered after
    // the halo; K3 recomputes the accept flags of the waves it runs (the table-mode default).
    int rng_replicate = 1;
    int halo_loopback = 0; // one-rank communicator: send the halo columns to itself and check them (2: corrupt one)
    int overlap = 1; // generate the next call's noise on rng_stream during this call's sweeps
    int solo_strip = 0; // timing only: one strip of a split plane, halo never exchanged (DFAMD_SOLO_STRIP)
    double solo_xchg_us = 0; // timing only: a solo strip's exchange held for this long (DFAMD_SOLO_XCHG_US)
    CompDev c[3];
    double *T = nullptr, *rho = nullptr, *rowc = nullptr, *tab = nullptr, *tabf = nullptr;
    int *tab_off = nullptr, *tabf_off = nullptr;
    // RNG
    RngStateDev *rstate = nullptr; // [2], ping-pong by call parity
    int *counts = nullptr;
    long long *offsets = nullptr;
    long long *part = nullptr; // K2a run totals -> run prefixes (K2b)
    uint16_t *masks = nullptr; // per-thread polar accept flags (K1 -> K3)
    int *wave_counts = nullptr; // accepted attempts per wave of each block (K1 -> K2c)
    uint8_t *xbuf = nullptr;    // run generation: the shares' records (group counts, block prefixes, totals)
    WaveTask *tasks = nullptr;  // waves K3 runs (K2c)
    int *ntasks = nullptr;
    int *err_dev = nullptr;   // mapped host memory: [0] RNG ran short, [1] gather indices skipped, [2] halo loopback mismatches
    int *err_host = nullptr;
    int rng_blocks = 0;       // attempt blocks per call (4096 attempts each), same on every rank
    int rng_chunk = 0;        // blocks counted by each z-strip rank (split counting, SURVEY 8e option A)
    bool split_count = false;
    ncclComm_t rng_comm = nullptr;           // second communicator: the count all-gather runs on rng_stream
    // Fused exchange (round 4; split counting with the run generation): the next generation's K1 goes on
    // rng_stream at the start of a call and its group counts travel inside the call's halo group - one grouped
    // RCCL operation per df_filter (north star) - and the rest of that generation runs after the group, beside
    // the z-pass. gen_pending: K1 enqueued, the exchange and gen_end not yet.
    int fused_x = 1;
    // Generations enqueued ahead of the step that consumes them (fused exchange): 2 = the share records of
    // generation k + 2 travel in call k's halo group and its K3r runs during call k + 1, so the RNG chain has a
    // whole call to finish instead of the z-pass beside it (4 noise sets). 1 = generation k + 1 in call k.
    int look = 1;
    bool gen_pending = false;
    RngGeom pend_g{};
    hipEvent_t ev_xchg = nullptr; // DFAMD_SOLO_STRIP: where the halo group would sit (after the pack)
    hipEvent_t ev_counted = nullptr;         // in-process groups: this handle's counts are ready
    hipEvent_t ev_halo = nullptr;            // split counting: the halo of the call just enqueued is done
    // RCCL z-strips (round 3): the halo send/recv, the unpack and the edge strips' z-pass run on comm_stream
    // (high priority) while the stream runs the z-pass of the strips whose stencils stay inside this rank's
    // columns (phase_halo_zpass). 0 = one serial chain (pack, send/recv, unpack, whole z-pass). -1 (default):
    // packed planes only. One rank of c4 over 8 timed alone without the exchange (profiles/r3/az): packed
    // 1.83-1.85 vs 1.85-1.92 ms (the split costs nothing, so the exchange time is the gain); table 0.296-0.308
    // vs 0.278-0.290 ms (+17 us: a row of 6 interior strips leaves half the 4-tile blocks unstaged and the
    // edge launch runs unstaged, against an exchange of a few tens of us).
    int halo_overlap = -1;
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_packed = nullptr, ev_unpacked = nullptr; // halo packed (stream); edge strips done (comm_stream)
    std::shared_ptr<std::vector<df_handle *>> group; // in-process strip group (df_create_group)
    long long gen_launched = 0; // generations enqueued (generation n reads state slot n%nsets, writes (n+1)%nsets)
    long long gen_used = 0;     // generations consumed by a visible step (ctor step 0, filter, stage API)
    // Hand-off batch (round 3): the two cross-stream hand-offs of a call (noise ready -> sweeps; sweeps done
    // -> noise set reusable) cost 5-15 us of queue packets per call on small planes (tools/handoff_ab.py,
    // profiles/r3/h). With hb > 1 the generations go in epochs of hb calls over 2*hb noise sets: one
    // noise-ready wait and one release record on the sweep stream per epoch instead of per call.
    int hb = 1;
    // the configured hand-off batch; a stream state loaded from outside (df_set_rng_state: checkpoints, the C++
    // objects of one process handing the reference's shared stream on) drops to one generation per epoch, so a
    // program that switches objects every call regenerates one generation per switch, not hb; after
    // kHbRestoreCalls calls without such a load the handle returns to hb_conf
    int hb_conf = 1;
    int calls_since_load = 0;
    int nsets = 2;
    long long gen_base = 0; // generation that starts epoch 0 (reset whenever the prefetched noise is discarded)
    int cur = 0;                // noise set of the current step
    int ylds = 0; // table y-pass with LDS-staged noise (SweepArgs::ylds): 2 ypass_tlds, 3 ypass_t64
    int yt_rows = 1, yt_chunk = 16, yt_pd = 2; // ypass_t64: rows per wave, noise rows per LDS chunk, chunks in flight
    int yt_limit = 0; // timing only (DFAMD_YT_LIMIT): ypass_t64 launches the first yt_limit blocks of its list alone
    int yt_dbg = 0;   // timing only (DFAMD_YT_DEBUG, wrong sums): ypass_t64 ablations of its coefficient loads
    int *ylist = nullptr;    // ypass_t64 dispatch order (build_ylist)
    int ylist_n = 0, ylist_nrb = 0, ylist_ncol = 0, ylist_cap = 0;
    // Ghost columns (round 5, table-mode z-strips with row-uniform N): each rank y-filters its strip widened by
    // Gl / Gr columns of its neighbours' (the widest z half-width, Nzp), straight into its z-halo, so the z-pass
    // needs no exchange; the RNG generates those columns' r_ys too. ghost_cap: the layout and tables exist
    // (ry pitch Pzy holds Wext columns); ghost: in use.
    int ghost_cap = 0, ghost = 0;
    int Gl = 0, Gr = 0, Wext = 0, nstrips_g = 0, Pzy = 0;
    int *ylist_g = nullptr;  // ypass_t64 order over the widened strip
    int ylist_g_n = 0, ylist_g_nrb = 0, ylist_g_ncol = 0, ylist_g_cap = 0;
    struct RunTables {
        const ChunkDest *chunk_dest[2] = {};
        const RunPiece *pieces[2] = {};
        int npieces[2] = {};
    } run_tab[2]; // run generation tables without (0) and with (1) the ghost columns
    bool dense_ready = false; // the run generation's chunk tables are built (alloc_dense)
    RngGeom geom{};
    // halo
    double *send_l = nullptr, *send_r = nullptr, *recv_l = nullptr, *recv_r = nullptr;
    size_t halo_elems = 0;
    // statistics (get_rms)
    double *rms_acc = nullptr, *rms_tmp = nullptr;
    long long rms_count = 0;
    // profiling
    bool profiling = false;
    int profile_every = 1;  // events on every profile_every-th df_filter only (df_set_profiling(h, n))
    long long prof_seq = 0; // df_filter calls since profiling was switched on
    bool prof_call = false; // this df_filter records its phase events
    std::vector<PhaseEvents> ev;
    size_t ev_used = 0;
    df_profile prof{};
    double prof_rng_span = 0; // RNG stream time of the profiled calls' generation bursts (ms)
    long long prof_rng_gens = 0; // generations in those bursts
    std::vector<YEvents> yev;   // ahead y-pass spans (every profile_every-th epoch)
    size_t yev_used = 0;
    long long yev_seq = 0;
    double prof_y_span = 0, prof_y_main = 0; // ms: ahead spans; y-passes on the stream
    long long prof_y_n = 0, prof_y_calls = 0; // y-passes in the spans; profiled calls whose y-pass ran ahead
    std::vector<void *> allocs;
    // Schedule trace (a handle created with device = DF_DEVICE_TRACE): the noise pipeline's host logic runs with
    // every HIP call it would make replaced by a record (trace_*), six int64 per record, read by df_trace
    bool tracing = false;
    std::vector<long long> tr;
};

namespace {

// Process-wide registry of every live device range the library allocated, all handles together.
// A new allocation that overlaps a live one fails loudly instead of aliasing another handle's buffer
// (round 2 saw one handle's T' change after a second handle was created while the coefficient pool
// was requested physically contiguous; the cause was not pinned down - DESIGN.md section 3).
struct AllocRegistry {
    std::mutex mu;
    std::map<uintptr_t, std::pair<uintptr_t, const void *>> live; // start -> (end, owner)
};
AllocRegistry &registry()
{
    static AllocRegistry r;
    return r;
}
std::string hex_range(uintptr_t a, uintptr_t b)
{
    char buf[64];
    std::snprintf(buf, sizeof buf, "[0x%llx, 0x%llx)", (unsigned long long)a, (unsigned long long)b);
    return buf;
}
// Claim [p, p + bytes) for owner; DF_EHIP naming both ranges if it overlaps a live range.
int registry_claim(const void *p, size_t bytes, const void *owner)
{
    const uintptr_t a = (uintptr_t)p, b = a + bytes;
    AllocRegistry &r = registry();
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.live.upper_bound(a); // first start > a; its predecessor may still cover a
    if (it != r.live.begin()) {
        auto prev = std::prev(it);
        if (prev->second.first > a)
            return fail(DF_EHIP, "device allocation " + hex_range(a, b) + " overlaps the live range " +
                                     hex_range(prev->first, prev->second.first) + (prev->second.second == owner ? " of the same handle" : " of another handle"));
    }
    if (it != r.live.end() && it->first < b)
        return fail(DF_EHIP, "device allocation " + hex_range(a, b) + " overlaps the live range " +
                                 hex_range(it->first, it->second.first) + (it->second.second == owner ? " of the same handle" : " of another handle"));
    r.live.emplace(a, std::make_pair(b, owner));
    return DF_OK;
}
void registry_release(const void *p)
{
    AllocRegistry &r = registry();
    std::lock_guard<std::mutex> lk(r.mu);
    r.live.erase((uintptr_t)p);
}

int dalloc(df_handle *h, void **p, size_t bytes)
{
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError(); // HIP keeps the failure as the thread's last error: the next launch check
                                 // (hipGetLastError after a kernel) would report it as its own
        return fail(e == hipErrorOutOfMemory ? DF_ENOMEM : DF_EHIP,
                    "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
    }
    if (int rc = registry_claim(*p, bytes, h)) {
        (void)hipFree(*p);
        *p = nullptr;
        return rc;
    }
    h->allocs.push_back(*p);
    HIP_OR(hipMemsetAsync(*p, 0, bytes, h->stream), DF_EHIP);
    return DF_OK;
}

template <class T> int dalloc_t(df_handle *h, T **p, size_t n) { return dalloc(h, (void **)p, n * sizeof(T)); }

template <class T> int upload(df_handle *h, T *dst, const T *src, size_t n)
{
    HIP_OR(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, h->stream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP); // src may be a temporary
    return DF_OK;
}

SweepArgs sweep_args(df_handle *h)
{
    SweepArgs a{};
    for (int c = 0; c < 3; ++c) {
        CompDev &d = h->c[c];
        a.ry[c] = d.ry[h->cur];
        a.rz[c] = d.rz[h->cur];
        a.By[c] = d.By;
        a.Bz[c] = d.Bz;
        a.byoff[c] = d.byoff;
        a.bzoff[c] = d.bzoff;
        a.Ny_st[c] = d.Ny_st;
        a.Nz_st[c] = d.Nz_st;
        a.Ny_cell[c] = d.Ny_cell;
        a.Nz_cell[c] = d.Nz_cell;
        a.Nyp[c] = d.Nyp;
        a.Nzp[c] = d.Nzp;
        a.rz_pitch[c] = d.rz_pitch;
        a.filt_old[c] = d.filt_old;
        a.fluc[c] = d.fluc;
        a.filt[c] = d.filt;
        a.sa[c] = d.sa;
        a.s1a[c] = d.s1a;
    }
    a.Ny = h->Ny;
    a.Nz_loc = h->Nz_loc;
    a.Pz = h->Pzy; // ry pitch (the y-pass's noise); the z-pass reads rz only
    a.nstrips = h->nstrips;
    a.zs_lo = 0;
    a.zs_n = a.zs_gap_at = h->nstrips;
    a.zs_gap = 0;
    for (int c = 0; c < 3; ++c) {
        a.halo_w[c] = h->c[c].halo_w;
        a.halo_off[c] = h->c[c].halo_off;
    }
    a.zgroup = 1;
    a.tab = h->tab;
    a.tab_off = h->tab_off;
    a.tabf = h->tabf;
    a.tabf_off = h->tabf_off;
    a.T = h->T;
    a.rho = h->rho;
    a.rowc = h->rowc;
    a.comps_mask = 7;
    a.yunroll = h->yunroll;
    a.ycoop = h->ycoop;
    a.ycoop2_run = 0;
    for (int c = 0; c < 3; ++c)
        for (int x = 0; x < 8; ++x) {
            a.ycoop2_xcd[c][x] = h->c[c].ycoop2_xcd[x];
            a.ycoop2_run = std::max(a.ycoop2_run, h->c[c].ycoop2_xcd[x + 1] - h->c[c].ycoop2_xcd[x]);
        }
    for (int c = 0; c < 3; ++c) {
        a.ycoop2_xcd[c][8] = h->c[c].ycoop2_xcd[8];
        a.ycoop2_perm[c] = h->ycoop_order || h->ycoop_split || h->ycoop_split4 ? h->c[c].ycoop2_perm : nullptr;
    }
    a.ylds = h->ylds;
    a.ylist = h->ylist;
    a.ylist_n = h->yt_limit > 0 ? std::min(h->ylist_n, h->yt_limit) : h->ylist_n;
    a.ylist_dbg = h->yt_dbg;
    a.ylist_nrb = h->ylist_nrb;
    a.ylist_ncol = h->ylist_ncol;
    a.ylist_R = h->yt_rows;
    a.ylist_C = h->yt_chunk;
    a.ylist_PD = h->yt_pd;
    for (int c = 0; c < 3; ++c) {
        a.yout[c] = h->c[c].Nzp;
        a.ylo[c] = 0;
        a.yhi[c] = h->Nz_loc;
    }
    a.zsplit = h->zsplit;
    a.zunroll = h->zunroll;
    a.nt_stores = h->nt_stores;
    a.ynt_stores = h->ynt_stores;
    a.ywin_T = h->ywin_T;
    a.ywin_W = h->ywin_W;
    a.zwin_T = h->zwin_T;
    a.zwin_W = h->zwin_W;
    a.per_cell = h->setup.per_cell;
    int nzp = 0;
    for (int c = 0; c < 3; ++c) nzp = std::max(nzp, a.Nzp[c]);
    a.zstage_reg = 4 * kStrip + 2 * nzp;
    a.zstage = 3 * a.zstage_reg * (int)sizeof(double) <= 64 * 1024 ? h->zstage : 0;
    return a;
}

// The z-halo of row j holds the plane's widest z half-width of that row (Setup::Nz_row, a property of the global
// row, so both neighbours size it alike) columns of each side, not Nzp: the z-pass of any strip reads no further
// (its tap range N_st is at most the row's maximum). c4 (N 4-64 over the rows): 1.6 MB per side, not 3.1 MB.
int alloc_halo(df_handle *h)
{
    h->halo_elems = 0;
    int rc;
    for (int c = 0; c < 3; ++c) {
        std::vector<int> w(h->Ny);
        std::vector<long long> off(h->Ny + 1, 0);
        for (int j = 0; j < h->Ny; ++j) {
            w[j] = std::min(h->setup.comp[c].Nz_row[j], h->c[c].Nzp);
            off[j + 1] = off[j] + w[j];
        }
        h->halo_elems += (size_t)off[h->Ny];
        if ((rc = dalloc_t(h, &h->c[c].halo_w, w.size()))) return rc;
        if ((rc = upload(h, h->c[c].halo_w, w.data(), w.size()))) return rc;
        if ((rc = dalloc_t(h, &h->c[c].halo_off, off.size()))) return rc;
        if ((rc = upload(h, h->c[c].halo_off, off.data(), off.size()))) return rc;
    }
    if ((rc = dalloc_t(h, &h->send_l, h->halo_elems))) return rc;
    if ((rc = dalloc_t(h, &h->send_r, h->halo_elems))) return rc;
    if ((rc = dalloc_t(h, &h->recv_l, h->halo_elems))) return rc;
    return dalloc_t(h, &h->recv_r, h->halo_elems);
}

int check_rng_error(df_handle *h)
{
    if (h->err_host && *(volatile int *)h->err_host)
        return fail(DF_ERNG, "device RNG ran short of polar attempts; stream state is invalid");
    if (h->err_host && ((volatile int *)h->err_host)[2]) {
        const int bad = ((volatile int *)h->err_host)[2];
        h->err_host[2] = 0;
        return fail(DF_ECOMM, "RCCL halo loopback: " + std::to_string(bad) + " values arrived changed");
    }
    return DF_OK;
}

bool prof_on(df_handle *h) { return h->profiling && h->prof_call && h->ev_used < h->ev.size(); }

// ---------------------------------------------------------------- schedule trace
// A DF_DEVICE_TRACE handle has no GPU: its streams and events are stand-in handles (kTrStream + i, kTrEvent + id) and
// each operation the pipeline would enqueue becomes one record {op, stream, a, b, c, d} (tests/test_schedule.py
// rebuilds the happens-before order from them and checks every noise set, stream state slot and event wait).
enum TraceOp {
    TR_RECORD = 1, // stream, event, tag: the event recorded (tag: the generation whose work it follows)
    TR_WAIT,       // stream, event, tag: the stream waits for the event's latest record (tag: the intended one)
    TR_K1,         // stream, gen, state slot read: attempt counts into the RNG scratch
    TR_K3,         // stream, gen, set, slot in, slot out: scratch + state in -> the set's r_ys and r_zs pads, state out
    TR_SHARE,      // stream, gen: the other ranks' share records into the scratch (solo-strip stand-in)
    TR_YPASS,      // stream, gen, set: r_ys of the set -> its r_zs interior
    TR_PACK,       // stream, gen, set: halo columns read from the set's r_zs interior
    TR_ZPASS,      // stream, gen, set: the set's r_zs -> the fields
    TR_SYNC,       // every stream drained by the host
    TR_STATE_R,    // -, slot, gen: the host reads the stream state before generation gen (df_rng_state)
    TR_STATE_W     // -, slot, gen: the host writes it (df_set_rng_state, the seed at create)
};
enum TraceEvent { TE_RNG = 0, TE_SWEPT = 2, TE_RELEASE = 4, TE_COUNTED = 4 + kMaxNoiseSets, TE_XCHG, TE_HALO, TE_N };
constexpr uintptr_t kTrStream = 0x10, kTrEvent = 0x100;
long long tr_stream(hipStream_t st) { return (long long)((uintptr_t)st - kTrStream); }
long long tr_event(hipEvent_t ev) { return (long long)((uintptr_t)ev - kTrEvent); }
void trace(df_handle *h, long long op, long long st = -1, long long a = 0, long long b = 0, long long c = 0,
           long long d = 0)
{
    h->tr.insert(h->tr.end(), {op, st, a, b, c, d});
}
// hipEventRecord / hipStreamWaitEvent of the pipeline; tag = the generation the record follows / the wait means
int q_record(df_handle *h, hipEvent_t ev, hipStream_t st, long long tag)
{
    if (h->tracing) {
        trace(h, TR_RECORD, tr_stream(st), tr_event(ev), tag);
        return DF_OK;
    }
    HIP_OR(hipEventRecord(ev, st), DF_EHIP);
    return DF_OK;
}
int q_wait(df_handle *h, hipStream_t st, hipEvent_t ev, long long tag)
{
    if (h->tracing) {
        trace(h, TR_WAIT, tr_stream(st), tr_event(ev), tag);
        return DF_OK;
    }
    HIP_OR(hipStreamWaitEvent(st, ev, 0), DF_EHIP);
    return DF_OK;
}
#define Q_OR(expr)                                                                                          \
    do {                                                                                                    \
        if (int rc_ = (expr)) return rc_;                                                                   \
    } while (0)

void ev_record(df_handle *h, int phase, hipStream_t st = nullptr)
{
    if (!prof_on(h)) return;
    (void)hipEventRecord(h->ev[h->ev_used].e[phase], st ? st : phase >= 4 && h->overlap ? h->rng_stream : h->stream);
}

int sync_all(df_handle *h)
{
    if (h->tracing) {
        trace(h, TR_SYNC);
        return DF_OK;
    }
    HIP_OR(hipStreamSynchronize(h->rng_stream), DF_EHIP);
    if (h->ystream) HIP_OR(hipStreamSynchronize(h->ystream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    if (h->comm_stream) HIP_OR(hipStreamSynchronize(h->comm_stream), DF_EHIP);
    return DF_OK;
}

int drain_profile(df_handle *h)
{
    if (!h->ev_used) return DF_OK;
    int rc = sync_all(h);
    if (rc) return rc;
    for (size_t i = 0; i < h->ev_used; ++i) {
        float t[3] = {0, 0, 0}, tot = 0, r = 0;
        for (int p = 0; p < 3; ++p) (void)hipEventElapsedTime(&t[p], h->ev[i].e[p], h->ev[i].e[p + 1]);
        (void)hipEventElapsedTime(&tot, h->ev[i].e[0], h->ev[i].e[3]);
        if (h->ev[i].rng) {
            (void)hipEventElapsedTime(&r, h->ev[i].e[4], h->ev[i].e[5]);
            h->prof_rng_span += r;
            h->prof_rng_gens += h->ev[i].gens;
        }
        if (h->ev[i].ahead) h->prof_y_calls++;
        else h->prof_y_main += t[0];
        h->prof.halo_ms += t[1];
        h->prof.zpass_ms += t[2];
        h->prof.total_ms += tot;
        h->prof.calls++;
        h->ev[i].rng = false;
        h->ev[i].gens = 0;
    }
    h->ev_used = 0;
    for (size_t i = 0; i < h->yev_used; ++i) {
        float y = 0;
        (void)hipEventElapsedTime(&y, h->yev[i].e[0], h->yev[i].e[1]);
        h->prof_y_span += y;
        h->prof_y_n += h->yev[i].n;
    }
    h->yev_used = 0;
    // an ahead call's y-pass time: the measured time per ahead y-pass (its epoch's span / its y-passes)
    h->prof.ypass_ms = h->prof_y_main + (h->prof_y_n ? h->prof_y_span / (double)h->prof_y_n * (double)h->prof_y_calls : 0.0);
    // Every call consumes one generation, but with hand-off batches (hb > 1) a call enqueues a burst of hb
    // generations at an epoch start and none mid-epoch, and sampled profiling may always land on the same
    // epoch position: rng_ms is therefore the measured time per generation times the calls profiled.
    h->prof.rng_ms = h->prof_rng_gens ? h->prof_rng_span / (double)h->prof_rng_gens * (double)h->prof.calls : 0.0;
    return DF_OK;
}

// ---------------------------------------------------------------- phases

// Epochs of the noise pipeline: with hb == 1 every generation is its own epoch (absolute index, so the
// event parity is the noise-set parity); with hb > 1, epochs of hb
// generations counted from gen_base.
constexpr int kHbRestoreCalls = 16;

long long gen_epoch(const df_handle *h, long long g) { return h->hb == 1 ? g : (g - h->gen_base) / h->hb; }
int gen_pos(const df_handle *h, long long g) { return h->hb == 1 ? 0 : (int)((g - h->gen_base) % h->hb); }
int gen_set(const df_handle *h, long long g) { return (int)(g % h->nsets); }
// Epochs whose noise sets the handle holds at once (nsets / hb): epoch e reuses epoch e - slots' sets, free once
// epoch e - slots + 1 has begun (ev_release[(e - slots) % slots], recorded then on the stream)
int epoch_slots(const df_handle *h) { return h->nsets / h->hb; }

// Noise pipeline. The reference draws all six noise arrays at the start of each
// call (df.cpp:453); the draws depend only on the stream state, so generation n+1
// is enqueued on rng_stream as soon as call n's sweeps are enqueued, into the
// other noise set, and runs (compute-bound) under call n's memory-bound sweeps.
bool run_form_ok(const df_handle *h)
{
    const bool fused_plan = h->fuse_plan && !h->split_count && h->rng_blocks <= 1024;
    return h->gen_dense == 2 && h->dense_ready && !fused_plan && h->geom.gen_split == 1;
}

// allow_run: the run generation may be used (an in-process group takes it only when every strip can, since the
// strips exchange its share records)
int gen_begin(df_handle *h, RngGeom &g, hipStream_t &rs, bool allow_run = true)
{
    const long long gi = h->gen_launched, e = gen_epoch(h, gi);
    const int set = gen_set(h, gi);
    rs = h->overlap ? h->rng_stream : h->stream;
    // the epoch's sets were last read by epoch e - K (K = epoch_slots), released when epoch e - K + 1 began
    const int K = epoch_slots(h);
    // (its last generation: gi - nsets + hb - 1)
    if (gen_pos(h, gi) == 0 && e >= K) Q_OR(q_wait(h, rs, h->ev_release[e % K], gi - h->nsets + h->hb - 1));
    g = h->geom;
    g.recount = h->split_count ? 1 : 0;
    // small single-plane calls: the compacted K3 computes its waves' ranks and plan itself
    g.nb_plan = h->rng_blocks;
    g.fused_plan = h->fuse_plan && !h->split_count && h->rng_blocks <= 1024 ? 1 : 0;
    g.gen_dense = allow_run && run_form_ok(h) ? 2 : 0;
    if (g.gen_dense == 2) { // K1 writes the group counts of its share's record, K2s the share's prefix
        g.xbuf = h->xbuf;
        g.xworld = h->split_count ? h->world : 1;
        g.xchunk = h->split_count ? h->rng_chunk : h->rng_blocks;
        record_layout(g.xchunk, &g.xstride, &g.xlp_off, &g.xtot_off);
    } else {
        g.xbuf = nullptr;
    }
    for (int c = 0; c < 3; ++c) {
        g.ry[c] = h->c[c].ry[set];
        g.rz[c] = h->c[c].rz[set];
    }
    if (prof_on(h) && h->ev[h->ev_used].gens++ == 0) { // a burst of hb generations is timed as one span
        ev_record(h, 4);
        h->ev[h->ev_used].rng = true;
    }
    if (h->tracing) {
        trace(h, TR_K1, tr_stream(rs), gi, gen_set(h, gi));
        return DF_OK;
    }
    const RngStateDev *in = h->rstate + gen_set(h, gi);
    if (!h->split_count)
        HIP_OR(launch_rng_count(g, in, h->counts, h->wave_counts, h->masks, 0, h->rng_blocks, h->rng_blocks, rs),
               DF_EHIP);
    else
        HIP_OR(launch_rng_count(g, in, h->counts, h->wave_counts, h->masks, h->rank * h->rng_chunk, h->rng_chunk,
                                h->rng_blocks, rs),
               DF_EHIP);
    if (g.gen_dense == 2) HIP_OR(launch_rng_share_scan(g, h->counts, h->split_count ? h->rank : 0, rs), DF_EHIP);
    return DF_OK;
}

int phase_ypass(df_handle *h, int comps_mask, int set = -1, hipStream_t st = nullptr, long long gen = -1);

// The last generation of epoch e (gen_epoch's inverse)
long long epoch_last(const df_handle *h, long long e) { return h->hb == 1 ? e : h->gen_base + e * h->hb + h->hb - 1; }

// The epoch just generated: its y-passes on ystream, ev_swept after them (df_handle::yahead)
int sweep_ahead(df_handle *h, long long e)
{
    const bool on = h->yahead && h->overlap && h->ystream;
    h->ep_swept[e & 1] = on;
    if (!on) return DF_OK;
    Q_OR(q_wait(h, h->ystream, h->ev_rng[e & 1], epoch_last(h, e)));
    const bool timed = h->profiling && (h->yev_seq++ % h->profile_every) == 0 && h->yev_used < h->yev.size();
    if (timed) HIP_OR(hipEventRecord(h->yev[h->yev_used].e[0], h->ystream), DF_EHIP);
    const long long g0 = h->hb == 1 ? e : h->gen_base + e * h->hb;
    for (long long g = g0; g < g0 + h->hb; ++g)
        if (int rc = phase_ypass(h, 7, gen_set(h, g), h->ystream, g)) return rc;
    if (timed) {
        HIP_OR(hipEventRecord(h->yev[h->yev_used].e[1], h->ystream), DF_EHIP);
        h->yev[h->yev_used++].n = h->hb;
    }
    return q_record(h, h->ev_swept[e & 1], h->ystream, epoch_last(h, e));
}

int gen_end(df_handle *h, const RngGeom &g, hipStream_t rs)
{
    const long long gi = h->gen_launched;
    const int nb_scan = h->split_count ? h->rng_chunk * h->world : h->rng_blocks;
    // split counting exchanges counts only: K3 recomputes the accept flags of the waves it runs
    // (g.recount), a sixth or less of all waves on an interior rank of 8
    if (h->tracing)
        trace(h, TR_K3, tr_stream(rs), gi, gen_set(h, gi), gen_set(h, gi), gen_set(h, gi + 1));
    else
        HIP_OR(launch_rng_finish(g, h->rstate + gen_set(h, gi), h->rstate + gen_set(h, gi + 1), h->counts,
                                 h->wave_counts, h->offsets, h->part, h->masks, h->tasks, h->ntasks, h->err_dev,
                                 h->rng_blocks, nb_scan, rs),
               DF_EHIP);
    if (prof_on(h)) ev_record(h, 5, rs);
    if (gen_pos(h, gi) == h->hb - 1) { // the epoch's noise is ready
        Q_OR(q_record(h, h->ev_rng[gen_epoch(h, gi) & 1], rs, gi));
        h->gen_launched++;
        return sweep_ahead(h, gen_epoch(h, gi));
    }
    h->gen_launched++;
    return DF_OK;
}

// In-process strip group: every member counts its share, the shares are copied
// device to device (the all-gather), then every member scans and generates.
int launch_gen_group(std::vector<df_handle *> &hs)
{
    const int n = (int)hs.size();
    std::vector<RngGeom> gs(n);
    std::vector<hipStream_t> rss(n);
    int rc;
    bool run = true; // one form for the whole group: strips set one by one may disagree for a while
    for (int r = 0; r < n; ++r) run = run && run_form_ok(hs[r]);
    for (int r = 0; r < n; ++r) {
        HIP_OR(hipSetDevice(hs[r]->device), DF_EHIP);
        if ((rc = gen_begin(hs[r], gs[r], rss[r], run))) return rc;
        HIP_OR(hipEventRecord(hs[r]->ev_counted, rss[r]), DF_EHIP);
    }
    for (int r = 0; r < n; ++r) {
        df_handle *h = hs[r];
        HIP_OR(hipSetDevice(h->device), DF_EHIP);
        for (int o = 0; o < n; ++o) {
            if (o == r) continue;
            const size_t at = (size_t)o * h->rng_chunk;
            HIP_OR(hipStreamWaitEvent(rss[r], hs[o]->ev_counted, 0), DF_EHIP);
            HIP_OR(hipMemcpyAsync(h->counts + at, hs[o]->counts + at, h->rng_chunk * sizeof(int), hipMemcpyDefault,
                                  rss[r]),
                   DF_EHIP);
            HIP_OR(hipMemcpyAsync(h->wave_counts + at * kWavesPerBlock, hs[o]->wave_counts + at * kWavesPerBlock,
                                  (size_t)h->rng_chunk * kWavesPerBlock * sizeof(int), hipMemcpyDefault, rss[r]),
                   DF_EHIP);
            if (gs[r].gen_dense == 2)
                HIP_OR(hipMemcpyAsync(gs[r].xbuf + (size_t)o * gs[r].xstride, gs[o].xbuf + (size_t)o * gs[r].xstride,
                                      (size_t)gs[r].xstride, hipMemcpyDefault, rss[r]),
                       DF_EHIP);
        }
        if ((rc = gen_end(h, gs[r], rss[r]))) return rc;
    }
    return DF_OK;
}

// Noise pipeline. The reference draws all six noise arrays at the start of each
// call (df.cpp:453); the draws depend only on the stream state, so generation n+1
// is enqueued on rng_stream as soon as call n's sweeps are enqueued, into the
// other noise set, and runs (compute-bound) under call n's memory-bound sweeps.
int launch_gen(df_handle *h)
{
    if (h->group) return launch_gen_group(*h->group);
    RngGeom g;
    hipStream_t rs;
    int rc = gen_begin(h, g, rs);
    if (rc) return rc;
    if (h->split_count) {
        int *mine = h->counts + (size_t)h->rank * h->rng_chunk;
        const size_t nwc = (size_t)h->rng_chunk * kWavesPerBlock;
        int *wmine = h->wave_counts + (size_t)h->rank * nwc;
        const size_t ngc = (size_t)g.xstride;
        uint8_t *gmine = g.xbuf + (size_t)h->rank * ngc;
        if (h->tracing && !h->rng_comm) {
            trace(h, TR_SHARE, tr_stream(rs), h->gen_launched);
        } else if (h->rng_comm) { // the RNG's one exchange: accept counts per block and per wave
            // Never concurrent with the halo send/recv of the other communicator: every rank issues
            // the all-gather only after its own halo group of the call just enqueued has completed,
            // so the two communicators' kernels run in the same order on every rank.
            if (h->ev_halo) HIP_OR(hipStreamWaitEvent(rs, h->ev_halo, 0), DF_EHIP);
            NCCL_OR(ncclGroupStart());
            if (g.gen_dense == 2) { // run form: the group counts alone (block counts are their sums)
                NCCL_OR(ncclAllGather(gmine, g.xbuf, ngc, ncclUint8, h->rng_comm, rs));
            } else {
                NCCL_OR(ncclAllGather(mine, h->counts, h->rng_chunk, ncclInt, h->rng_comm, rs));
                NCCL_OR(ncclAllGather(wmine, h->wave_counts, nwc, ncclInt, h->rng_comm, rs));
            }
            NCCL_OR(ncclGroupEnd());
        } else if (g.gen_dense == 2) { // DFAMD_SOLO_STRIP: this rank's group counts stand in for every share
            HIP_OR(launch_replicate_share(g.xbuf, ngc, h->world, h->rank, rs), DF_EHIP);
        } else { // DFAMD_SOLO_STRIP timing mode: stand-in shares for the other ranks
            for (int o = 0; o < h->world; ++o)
                if (o != h->rank) {
                    HIP_OR(hipMemcpyAsync(h->counts + (size_t)o * h->rng_chunk, mine, h->rng_chunk * sizeof(int),
                                          hipMemcpyDeviceToDevice, rs),
                           DF_EHIP);
                    HIP_OR(hipMemcpyAsync(h->wave_counts + (size_t)o * nwc, wmine, nwc * sizeof(int),
                                          hipMemcpyDeviceToDevice, rs),
                           DF_EHIP);
                }
        }
    }
    return gen_end(h, g, rs);
}

// Start a visible step on the next generation (reference: generate_white_noise()).
int consume_gen(df_handle *h)
{
    const long long gi = h->gen_used, e = gen_epoch(h, gi);
    const bool first = gen_pos(h, gi) == 0;
    int rc;
    if (first && gi > (h->hb == 1 ? 0 : h->gen_base))
        Q_OR(q_record(h, h->ev_release[(e - 1) % epoch_slots(h)], h->stream, gi - 1)); // the previous epoch's sets free
    const long long need = h->hb == 1 ? gi + 1 : h->gen_base + (e + 1) * h->hb; // this epoch, launched
    while (h->gen_launched < need)
        if ((rc = launch_gen(h))) return rc;
    h->cur_swept = h->ep_swept[e & 1];
    if (first) Q_OR(q_wait(h, h->stream, (h->cur_swept ? h->ev_swept : h->ev_rng)[e & 1], need - 1));
    h->cur = gen_set(h, gi);
    h->gen_used++;
    return DF_OK;
}

// After a visible step's sweeps are enqueued: generations up to hb steps ahead, under those sweeps.
// One generation is enqueued per step (an epoch enqueued as one burst measured no better, profiles/r3/m),
// so the last generation of epoch e + 1 goes
// under the last step of epoch e, just before epoch e + 1 waits for it.
int fused_gen_end(df_handle *h);
bool fused_active(const df_handle *h);
int prefetch_epochs(const df_handle *h);
int prefetch_gen(df_handle *h)
{
    if (int rc = fused_gen_end(h)) return rc;
    if (!h->overlap || h->gen_used == 0) return DF_OK;
    const long long gi = h->gen_used - 1; // the generation this step consumed
    (void)gi;
    const long long need = h->gen_used + (fused_active(h) ? h->look : prefetch_epochs(h) * h->hb);
    int rc;
    while (h->gen_launched < need)
        if ((rc = launch_gen(h))) return rc;
    return DF_OK;
}

// Epochs generated ahead of the one being consumed. Two where three epochs of sets are held (epoch_slots >= 3) and
// the handle batches or runs the y-pass ahead: ahead handles (consumed, swept, generating) so an epoch's y-passes
// never wait for its own generation to start behind the release of the epoch before; batched single-GPU table
// planes so their VALU-bound generation has a whole epoch of slack to fill the sweeps' gaps. Never more than
// epoch_slots - 1: generation of epoch e waits for the release of epoch e - epoch_slots, recorded when epoch
// e - epoch_slots + 1 begins (tests/test_schedule.py checks every schedule on the host).
int prefetch_epochs(const df_handle *h)
{
    return (h->hb > 1 || (h->yahead && (h->ystream || h->device < 0))) && epoch_slots(h) >= 3 ? 2 : 1;
}

// The fused exchange applies to split-counting z-strip handles of one process per GPU (RCCL, or the solo-strip
// timing stand-in) with the run generation and one generation per hand-off.
bool fused_active(const df_handle *h)
{
    return h->fused_x && h->split_count && h->world > 1 && (h->comm || h->solo_strip) && !h->group && h->overlap &&
           h->hb == 1 && h->gen_dense == 2 && h->dense_ready;
}

// Start of a visible step: the next generation's K1 (its group counts) on rng_stream, ev_counted after it.
int fused_gen_begin(df_handle *h)
{
    h->gen_pending = false; // a K1 left pending by a failed call is simply redone
    if (!fused_active(h) || h->gen_launched != h->gen_used + (h->look - 1)) return DF_OK;
    hipStream_t rs;
    int rc = gen_begin(h, h->pend_g, rs);
    if (rc) return rc;
    if (h->pend_g.gen_dense != 2) return DF_OK; // cannot happen with fused_active; the plain path then runs
    Q_OR(q_record(h, h->ev_counted, rs, h->gen_launched));
    h->gen_pending = true;
    if (h->ghost) { // no halo group to ride in: the records' all-gather follows the counts on the RNG stream, so
                    // the sweep stream never waits on a collective (the sweeps of calls k, k + 1 run beside it)
        if (h->comm && !h->solo_strip) {
            const size_t ngc = (size_t)h->pend_g.xstride;
            NCCL_OR(ncclAllGather(h->pend_g.xbuf + (size_t)h->rank * ngc, h->pend_g.xbuf, ngc, ncclUint8, h->rng_comm, rs));
            HIP_OR(hipEventRecord(h->ev_halo, rs), DF_EHIP);
        } else { // solo strip: the exchange's stand-in (and its held time) on the RNG stream
            if (h->solo_xchg_us > 0 && !h->tracing) HIP_OR(launch_hold(h->solo_xchg_us, rs), DF_EHIP);
            Q_OR(q_record(h, h->ev_xchg, rs, h->gen_launched));
        }
    }
    return DF_OK;
}

// After the halo group (which carried the group counts): scan, locate, generate on rng_stream.
int fused_gen_end(df_handle *h)
{
    if (!h->gen_pending) return DF_OK;
    h->gen_pending = false;
    hipStream_t rs = h->rng_stream;
    if (h->comm) {
        HIP_OR(hipStreamWaitEvent(rs, h->ev_halo, 0), DF_EHIP);
    } else { // solo strip: the same dependency on this call's halo position, the exchange by a stand-in copy
        Q_OR(q_wait(h, rs, h->ev_xchg, h->gen_launched));
        if (h->tracing) trace(h, TR_SHARE, tr_stream(rs), h->gen_launched);
        else HIP_OR(launch_replicate_share(h->pend_g.xbuf, (size_t)h->pend_g.xstride, h->world, h->rank, rs), DF_EHIP);
    }
    return gen_end(h, h->pend_g, rs);
}

int phase_ypass(df_handle *h, int comps_mask, int set, hipStream_t st, long long gen)
{
    if (h->tracing) {
        trace(h, TR_YPASS, tr_stream(st ? st : h->stream), gen >= 0 ? gen : h->gen_used - 1, set >= 0 ? set : h->cur);
        return DF_OK;
    }
    SweepArgs a = sweep_args(h);
    a.comps_mask = comps_mask;
    if (set >= 0)
        for (int c = 0; c < 3; ++c) {
            a.ry[c] = h->c[c].ry[set];
            a.rz[c] = h->c[c].rz[set];
        }
    if (h->ghost) { // the strip widened by its ghost columns; each component keeps the Nzp columns its halo holds
        a.Nz_loc = h->Wext;
        a.nstrips = h->nstrips_g;
        a.ylist = h->ylist_g;
        a.ylist_n = h->ylist_g_n;
        a.ylist_nrb = h->ylist_g_nrb;
        a.ylist_ncol = h->ylist_g_ncol;
        for (int c = 0; c < 3; ++c) {
            a.Ny_st[c] = h->c[c].Ny_st_g;
            a.yout[c] = h->c[c].Nzp - h->Gl;
            a.ylo[c] = h->Gl - h->c[c].Nzp > 0 ? h->Gl - h->c[c].Nzp : 0;
            a.yhi[c] = std::min(h->Wext, h->Gl + h->Nz_loc + (h->Gr ? h->c[c].Nzp : 0));
        }
    }
    HIP_OR(launch_ypass(a, h->coeff_mode == DF_COEFF_TABLE, h->rows_per_wave, st ? st : h->stream), DF_EHIP);
    return DF_OK;
}

int phase_halo_pack(df_handle *h)
{
    if (h->world == 1) return DF_OK;
    if (h->tracing) {
        trace(h, TR_PACK, tr_stream(h->stream), h->gen_used - 1, h->cur);
        return DF_OK;
    }
    SweepArgs a = sweep_args(h);
    HIP_OR(launch_halo_pack(a, h->rank > 0 ? h->send_l : nullptr, h->rank < h->world - 1 ? h->send_r : nullptr,
                            h->stream),
           DF_EHIP);
    return DF_OK;
}

int phase_halo_unpack(df_handle *h, hipStream_t st = nullptr)
{
    if (h->world == 1) return DF_OK;
    SweepArgs a = sweep_args(h);
    HIP_OR(launch_halo_unpack(a, h->rank > 0 ? h->recv_l : nullptr, h->rank < h->world - 1 ? h->recv_r : nullptr,
                              st ? st : h->stream),
           DF_EHIP);
    return DF_OK;
}

// One-rank communicator with halo_loopback set: the grouped ncclSend/ncclRecv of the z-strip path
// run with this rank as its own left and right neighbour (both plane edges packed, sent, received
// and compared on the device); the received columns are not unpacked, so results are unchanged.
int halo_loopback(df_handle *h)
{
    SweepArgs a = sweep_args(h);
    HIP_OR(launch_halo_pack(a, h->send_l, h->send_r, h->stream), DF_EHIP);
    NCCL_OR(ncclGroupStart());
    NCCL_OR(ncclSend(h->send_l, h->halo_elems, ncclDouble, 0, h->comm, h->stream));
    NCCL_OR(ncclRecv(h->recv_l, h->halo_elems, ncclDouble, 0, h->comm, h->stream));
    NCCL_OR(ncclSend(h->send_r, h->halo_elems, ncclDouble, 0, h->comm, h->stream));
    NCCL_OR(ncclRecv(h->recv_r, h->halo_elems, ncclDouble, 0, h->comm, h->stream));
    NCCL_OR(ncclGroupEnd());
    HIP_OR(launch_halo_check(h->send_l, h->recv_l, h->halo_elems, h->halo_loopback == 2, h->err_dev + 2, h->stream),
           DF_EHIP);
    HIP_OR(launch_halo_check(h->send_r, h->recv_r, h->halo_elems, 0, h->err_dev + 2, h->stream), DF_EHIP);
    if (h->ev_halo) HIP_OR(hipEventRecord(h->ev_halo, h->stream), DF_EHIP);
    return DF_OK;
}

// The grouped send/recv with rank +- 1 on stream st, then ev_halo there.
int halo_sendrecv(df_handle *h, hipStream_t st)
{
    if (h->gen_pending) HIP_OR(hipStreamWaitEvent(st, h->ev_counted, 0), DF_EHIP); // the next generation's counts
    NCCL_OR(ncclGroupStart());
    if (h->gen_pending) { // fused exchange: the next generation's share records, in place, in the same group
        const size_t ngc = (size_t)h->pend_g.xstride;
        NCCL_OR(ncclAllGather(h->pend_g.xbuf + (size_t)h->rank * ngc, h->pend_g.xbuf, ngc, ncclUint8, h->comm, st));
    }
    if (h->rank > 0) {
        NCCL_OR(ncclSend(h->send_l, h->halo_elems, ncclDouble, h->rank - 1, h->comm, st));
        NCCL_OR(ncclRecv(h->recv_l, h->halo_elems, ncclDouble, h->rank - 1, h->comm, st));
    }
    if (h->rank < h->world - 1) {
        NCCL_OR(ncclSend(h->send_r, h->halo_elems, ncclDouble, h->rank + 1, h->comm, st));
        NCCL_OR(ncclRecv(h->recv_r, h->halo_elems, ncclDouble, h->rank + 1, h->comm, st));
    }
    NCCL_OR(ncclGroupEnd());
    if (h->ev_halo) HIP_OR(hipEventRecord(h->ev_halo, st), DF_EHIP);
    return DF_OK;
}

int phase_halo_rccl(df_handle *h)
{
    if (h->world == 1) return h->halo_loopback && h->comm ? halo_loopback(h) : DF_OK;
    if (h->ghost) return DF_OK; // the y-pass filled the z-halo itself
    if (h->solo_strip) { // timing only: the pack, no exchange (or a hold of DFAMD_SOLO_XCHG_US in its place)
        int rc = phase_halo_pack(h);
        if (!rc && h->solo_xchg_us > 0 && !h->tracing) HIP_OR(launch_hold(h->solo_xchg_us, h->stream), DF_EHIP);
        if (!rc && h->gen_pending) Q_OR(q_record(h, h->ev_xchg, h->stream, h->gen_launched));
        return rc;
    }
    if (!h->comm) return fail(DF_EINVAL, "z-strip handle without an RCCL communicator: use df_filter_group");
    int rc = phase_halo_pack(h);
    if (rc || (rc = halo_sendrecv(h, h->stream))) return rc;
    return phase_halo_unpack(h);
}

// Strips [lo, hi) of a z-strip rank read no halo column: strip s spans columns [128 s, 128 s + 127] and its
// stencils reach Nzp further either side (Nzp = the widest component's Nz_max), so it is interior when
// 128 s >= Nzp and 128 (s + 1) + Nzp <= Nz_loc. The plane's own edges (rank 0's left, the last rank's right)
// read the generated raw-noise pads (df.cpp:385-405's quirk), not the halo, so they count as interior.
bool halo_interior(const df_handle *h, int *lo, int *hi)
{
    int w = 0;
    for (int c = 0; c < 3; ++c) w = std::max(w, h->c[c].Nzp);
    *lo = h->rank == 0 ? 0 : (w + kStrip - 1) / kStrip;
    *hi = h->rank == h->world - 1 ? h->nstrips : std::max(0, (h->Nz_loc - w) / kStrip);
    *hi = std::min(*hi, h->nstrips);
    return *hi > *lo;
}

int phase_zpass(df_handle *h, bool corr, bool sra, double dt, int part = 0, hipStream_t st = nullptr);

// Halo exchange, then the z-pass. RCCL z-strips with halo_overlap: the stream packs the halo and runs the
// z-pass of the interior strips; comm_stream (high priority) runs the send/recv, the unpack and the edge
// strips' z-pass beside it, and the stream waits for that before the call ends. The edge strips' blocks
// join the interior launch's as its slots free instead of running as a small launch on an idle chip (the
// round-1 form, which also split the y-pass, lost 80-190 us per call that way; profiles/r1/probe/
// halo_overlap_rejected.jsonl).
int phase_halo_zpass(df_handle *h, bool corr, bool sra, double dt)
{
    int lo = 0, hi = 0, rc;
    const bool peer = h->comm && !h->solo_strip; // DFAMD_SOLO_STRIP (timing only): the same streams, no exchange
    const bool ov = h->halo_overlap > 0 || (h->halo_overlap < 0 && h->coeff_mode == DF_COEFF_PACKED);
    if (h->world == 1 || h->ghost || !(peer || h->solo_strip) || !ov || !h->comm_stream || !halo_interior(h, &lo, &hi)) {
        if ((rc = phase_halo_rccl(h))) return rc;
        ev_record(h, 2);
        return phase_zpass(h, corr, sra, dt);
    }
    if ((rc = phase_halo_pack(h))) return rc;
    HIP_OR(hipEventRecord(h->ev_packed, h->stream), DF_EHIP);
    ev_record(h, 2); // halo_ms is the pack alone here; the exchange runs under zpass_ms
    HIP_OR(hipStreamWaitEvent(h->comm_stream, h->ev_packed, 0), DF_EHIP);
    if (!peer && h->solo_xchg_us > 0) HIP_OR(launch_hold(h->solo_xchg_us, h->comm_stream), DF_EHIP);
    if (!peer && h->gen_pending) HIP_OR(hipEventRecord(h->ev_xchg, h->comm_stream), DF_EHIP);
    // From here on comm_stream holds work that reads the send buffers: whatever fails below, the stream
    // joins comm_stream before returning, so the next call's pack cannot overwrite buffers still in flight.
    auto join = [h](int code) {
        if (hipEventRecord(h->ev_unpacked, h->comm_stream) == hipSuccess)
            (void)hipStreamWaitEvent(h->stream, h->ev_unpacked, 0);
        else
            (void)hipStreamSynchronize(h->comm_stream);
        return code;
    };
    if (peer && (rc = halo_sendrecv(h, h->comm_stream))) return join(rc);
    if (peer && (rc = phase_halo_unpack(h, h->comm_stream))) return join(rc);
    if ((rc = phase_zpass(h, corr, sra, dt, 2, h->comm_stream))) return join(rc); // edge strips
    rc = phase_zpass(h, corr, sra, dt, 1); // interior strips
    return join(rc);
}

// part 0: every strip; 1: the halo-interior strips; 2: the edge strips around them (halo_interior)
int phase_zpass(df_handle *h, bool corr, bool sra, double dt, int part, hipStream_t st)
{
    if (h->tracing) {
        trace(h, TR_ZPASS, tr_stream(st ? st : h->stream), h->gen_used - 1, h->cur);
        return DF_OK;
    }
    SweepArgs a = sweep_args(h);
    if (part) {
        int lo = 0, hi = 0;
        halo_interior(h, &lo, &hi);
        if (part == 1) {
            a.zs_lo = lo;
            a.zs_n = a.zs_gap_at = hi - lo;
        } else {
            a.zs_n = lo + (h->nstrips - hi);
            a.zs_gap_at = lo;
            a.zs_gap = hi - lo;
            a.zstage = 0; // a block's 4 tiles may straddle the gap
            a.zgroup = 0;
        }
    }
    if (corr) {
        const double pi = 3.141592654; // df.cpp:411
        for (int c = 0; c < 3; ++c) {
            const double alpha = std::exp(-pi * dt / h->setup.comp[c].Lt);
            a.sa[c] = std::sqrt(alpha);
            a.s1a[c] = std::sqrt(1.0 - alpha);
        }
    }
    a.do_corr = corr ? 1 : 0;
    a.do_sra = sra ? 1 : 0;
    HIP_OR(launch_zpass(a, h->coeff_mode == DF_COEFF_TABLE, st ? st : h->stream), DF_EHIP);
    return DF_OK;
}

int write_csv_if(df_handle *h)
{
    if (h->csv_path.empty()) return DF_OK;
    if (h->solo_strip) return fail(DF_EINVAL, "DFAMD_SOLO_STRIP handle: timing only, no CSV");
    const size_t n = (size_t)h->Ny * h->Nz_loc;
    std::vector<double> f[5];
    double *src[5] = {h->c[0].fluc, h->c[1].fluc, h->c[2].fluc, h->T, h->rho};
    for (int i = 0; i < 5; ++i) {
        f[i].resize(n);
        HIP_OR(hipMemcpyAsync(f[i].data(), src[i], n * 8, hipMemcpyDeviceToHost, h->stream), DF_EHIP);
    }
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    std::string path = h->csv_path;
    if (h->world > 1) path += ".rank" + std::to_string(h->rank);
    std::string err;
    if (!write_csv(h->setup, path, f[0].data(), f[1].data(), f[2].data(), f[3].data(), f[4].data(), h->z0,
                   h->Nz_loc, err))
        return fail(DF_EIO, err);
    return DF_OK;
}

// ---------------------------------------------------------------- create

// Config fields and the environment's tuning knobs (df.hpp:38-49 plus extensions).
int read_config(df_handle *h, const df_config_c *cfg)
{
    h->flow.d_i = cfg->d_i;
    h->flow.rho_e = cfg->rho_e;
    h->flow.U_e = cfg->U_e;
    h->flow.mu = cfg->mu_e;
    h->spec.kind = cfg->plane;
    h->spec.Ny = cfg->Ny;
    h->spec.Nz = cfg->Nz;
    h->spec.N_min = cfg->N_min;
    h->spec.N_max = cfg->N_max;
    if (cfg->plane == DF_PLANE_GRID) { // caller vertices, else the Tecplot grid_file (df.hpp:47)
        if (cfg->grid_y && cfg->grid_z) {
            if (cfg->Ny < 1 || cfg->Nz < 1) return fail(DF_EINVAL, "grid plane: Ny and Nz (cells) must be set with grid_y/grid_z");
            const size_t nv = (size_t)(cfg->Ny + 1) * (cfg->Nz + 1);
            h->spec.grid_y.assign(cfg->grid_y, cfg->grid_y + nv);
            h->spec.grid_z.assign(cfg->grid_z, cfg->grid_z + nv);
        } else if (cfg->grid_file) {
            h->spec.grid_file = cfg->grid_file;
        } else {
            return fail(DF_EINVAL, "grid plane needs grid_y/grid_z vertex arrays or a grid_file");
        }
    }
    if (!cfg->vel_fluc_file || !cfg->line_file)
        return fail(DF_EINVAL, "vel_fluc_file (RST profile) and line_file (mean profile) are required");
    h->spec.rst_file = cfg->vel_fluc_file;
    h->spec.line_file = cfg->line_file;
    h->coeff_mode = cfg->coeff_mode;
    if (h->coeff_mode != DF_COEFF_PACKED && h->coeff_mode != DF_COEFF_TABLE)
        return fail(DF_EINVAL, "coeff_mode must be DF_COEFF_PACKED or DF_COEFF_TABLE");
    if (cfg->csv_path) h->csv_path = cfg->csv_path;
    h->rank = cfg->rank;
    h->world = cfg->world < 1 ? 1 : cfg->world;
    if (h->rank < 0 || h->rank >= h->world) return fail(DF_EINVAL, "rank out of range");
    h->rows_per_wave = cfg->rows_per_wave; // 0: chosen from the plane's shape after setup (below)
    // Timing-only environment: DFAMD_RNG_OVERLAP=0 runs the noise on the sweep stream
    // (profilers), DFAMD_SOLO_STRIP one rank of a split plane alone, DFAMD_SOLO_XCHG_US its exchange held,
    // DFAMD_RNG_DEBUG the RNG ablations (wrong results by design). Launch shapes are df_set_tuning keys.
    if (const char *e = std::getenv("DFAMD_RNG_OVERLAP")) h->overlap = std::atoi(e);
    if (const char *e = std::getenv("DFAMD_SOLO_STRIP")) h->solo_strip = std::atoi(e) && cfg->world > 1 && !cfg->comm_id;
    if (const char *e = std::getenv("DFAMD_SOLO_XCHG_US")) h->solo_xchg_us = h->solo_strip ? std::atof(e) : 0;
    // Table mode splits the counting (one small all-gather of counts beside the halo): its sweeps are
    // VALU-bound like the RNG, so every rank counting the whole stream shows (one rank of a c4 split
    // in 8: 0.28-0.30 -> 0.24-0.27 ms per call). Packed keeps the halo as the call's only collective:
    // its sweeps are HBM-bound and hide the replicated count (equal within noise at N = 4, 8;
    // profiles/r2/strip_timing_c4_counts_only.jsonl).
    h->rng_replicate = h->coeff_mode == DF_COEFF_PACKED ? 1 : 0;
    if (h->solo_strip && !h->rng_replicate) h->split_count = true;
    if (const char *e = std::getenv("DFAMD_RNG_DEBUG")) h->geom.debug_flags = std::atoi(e); // timing ablation
    // timing ablation (wrong fields by design): ypass_t64 runs only the first n blocks of its heaviest-first list
    if (const char *e = std::getenv("DFAMD_YT_LIMIT")) h->yt_limit = std::atoi(e);
    if (const char *e = std::getenv("DFAMD_YT_DEBUG")) h->yt_dbg = std::atoi(e);
    if (h->rows_per_wave != 0 && h->rows_per_wave != 1 && h->rows_per_wave != 2 && h->rows_per_wave != 4 &&
        h->rows_per_wave != 8)
        return fail(DF_EINVAL, "rows_per_wave must be 1, 2, 4 or 8");
    return DF_OK;
}

// Row-pair y-pass tiles split into 8 contiguous runs of equal cost, one run per XCD (ypass_coop2_kernel):
// a plain 1/8 split of the tile list hands XCDs whole runs of narrow-stencil rows or of a narrow last
// strip (the reference's grid: N_y 28-212 along the rows, a 16-column last strip) and leaves them idle
// while the others stream. Cost of a tile = its coefficient taps x live columns + ycoop_ovh full-strip
// taps (a per-block fixed cost).
// Work items: a tile, or (ycoop_split) one 64-column half of a wide-stencil tile. A block's chunks are its chain
// of dependent round trips, and every resident block gets about the same share of HBM, so a 27-chunk tile of the
// reference's grid ends the launch long after the 4-chunk ones; its halves fold two tap groups into each wave
// (as the narrow last strip does), so each walks the chain in half the chunks, in parallel. Code = tile * 8 +
// part (0 whole, 1-2 the 64-column halves, 3-6 the 32-column quarters; ycoop_split4).
void balance_ycoop2(df_handle *h, int c)
{
    constexpr int RR = 2; // rows per block of the row-pair y-pass
    const int Ny = h->Ny, nrb = (Ny + RR - 1) / RR;
    const std::vector<int> &Nst = h->y_nst[c];
    // host-only handles (no device state) never built the tap ranges: nothing to balance
    if (Nst.size() < (size_t)h->nstrips * Ny) return;
    std::vector<double> wgt;
    std::vector<int> code;
    const double ovh = (double)h->ycoop_ovh * kStrip;
    double tot = 0;
    for (int st = 0; st < h->nstrips; ++st) {
        const int live = std::min(kStrip, h->Nz_loc - st * kStrip);
        for (int rb = 0; rb < nrb; ++rb) {
            double taps = 0;
            int nmax = 0;
            for (int j = rb * RR; j < std::min(Ny, rb * RR + RR); ++j) {
                taps += 2 * Nst[(size_t)st * Ny + j] + 1;
                nmax = std::max(nmax, Nst[(size_t)st * Ny + j]);
            }
            const int tile = st * nrb + rb;
            auto item = [&](double w, int part) {
                wgt.push_back(w);
                code.push_back(tile * 8 + part);
                tot += w;
            };
            if (h->ycoop_split4 > 0 && live == kStrip && nmax >= h->ycoop_split4)
                for (int part = 3; part <= 6; ++part) item(taps * 32 + ovh, part);
            else if (h->ycoop_split > 0 && live > 64 && nmax >= h->ycoop_split)
                for (int part = 1; part <= 2; ++part) item(taps * (part == 1 ? 64 : live - 64) + ovh, part);
            else
                item(taps * live + ovh, 0);
        }
    }
    int *xr = h->c[c].ycoop2_xcd;
    int x = 1;
    double acc = 0;
    xr[0] = 0;
    for (size_t t = 0; t < wgt.size() && x < 8; ++t) {
        acc += wgt[t];
        while (x < 8 && acc >= tot * x / 8) xr[x++] = (int)t + 1;
    }
    while (x <= 8) xr[x++] = (int)wgt.size();
    // Dispatch order inside each XCD run. Ascending rows (order 0) keeps neighbouring row pairs, which share
    // most noise rows, resident together; but where the widest stencils sit at the end of a run (the
    // reference's grid: N_y peaks at 212 around j = 170, N 28-60 elsewhere) they start last and the run
    // ends on a tail of 27-chunk blocks. Order g >= 1: groups of g consecutive items, heaviest group first.
    std::vector<int> &perm = h->ycoop2_perm_host[c];
    perm = code;
    const int gsz = h->ycoop_order;
    if (gsz > 0)
        for (int xx = 0; xx < 8; ++xx) {
            std::vector<std::pair<double, int>> grp; // (group weight, first item)
            for (int t = xr[xx]; t < xr[xx + 1]; t += gsz) {
                double w = 0;
                for (int u = t; u < std::min(t + gsz, xr[xx + 1]); ++u) w += wgt[u];
                grp.push_back({w, t});
            }
            std::stable_sort(grp.begin(), grp.end(), [](const auto &p, const auto &q) { return p.first > q.first; });
            int pos = xr[xx];
            for (const auto &gq : grp)
                for (int u = gq.second; u < std::min(gq.second + gsz, xr[xx + 1]); ++u) perm[pos++] = code[u];
        }
}

// Upload the dispatch order of the row-pair y-pass (alloc_components, df_set_tuning).
int upload_ycoop2_perm(df_handle *h, int c)
{
    if (!h->c[c].ycoop2_perm || h->ycoop2_perm_host[c].empty()) return DF_OK;
    return upload(h, h->c[c].ycoop2_perm, h->ycoop2_perm_host[c].data(), h->ycoop2_perm_host[c].size());
}

// Dispatch order of ypass_t64_kernel (ylds 3): blocks of 4 * yt_rows rows x 64 columns of every component, the
// largest union of noise rows (a block's chunk count, so its time) first; ties keep component, tile, row order.
// ghost: over the strip widened by its ghost columns (row-uniform N: every column of a row has the row's N).
int build_ylist(df_handle *h, bool ghost)
{
    const int Ny = h->Ny, RB = 4 * h->yt_rows;
    const int W = ghost ? h->Wext : h->Nz_loc;
    const int ncol = (W + 63) / 64, nrb = (Ny + RB - 1) / RB;
    const int n = 3 * ncol * nrb;
    if (n > (ghost ? h->ylist_g_cap : h->ylist_cap)) return fail(DF_EINVAL, "ypass_t64 tile list larger than its allocation");
    std::vector<std::pair<int, int>> cost(n); // (-noise rows, tile)
    for (int c = 0; c < 3; ++c)
        for (int ct = 0; ct < ncol; ++ct)
            for (int rb = 0; rb < nrb; ++rb) {
                const int *nst = ghost ? h->setup.comp[c].Ny_row.data() : h->y_nst[c].data() + (size_t)(ct >> 1) * Ny;
                int lo = 1 << 30, hi = -(1 << 30);
                for (int j = rb * RB; j < std::min(Ny, rb * RB + RB); ++j) {
                    lo = std::min(lo, j - nst[j]);
                    hi = std::max(hi, j + nst[j]);
                }
                const int t = (c * ncol + ct) * nrb + rb;
                cost[t] = {-(hi - lo + 1), t};
            }
    std::stable_sort(cost.begin(), cost.end(), [](const auto &p, const auto &q) { return p.first < q.first; });
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = cost[i].second;
    (ghost ? h->ylist_g_n : h->ylist_n) = n;
    (ghost ? h->ylist_g_nrb : h->ylist_nrb) = nrb;
    (ghost ? h->ylist_g_ncol : h->ylist_ncol) = ncol;
    return upload(h, ghost ? h->ylist_g : h->ylist, order.data(), order.size());
}

int build_ylists(df_handle *h)
{
    int rc = h->ylist ? build_ylist(h, false) : DF_OK;
    if (!rc && h->ylist_g) rc = build_ylist(h, true);
    return rc;
}

// The ypass_t64 shapes built (launch_ypass_t)
bool t64_shape_ok(int R, int C, int PD)
{
    if (PD == 4) return R == 1 && C == 16;
    return PD == 2 && ((R == 1 && (C == 16 || C == 24)) || (R == 2 && (C == 8 || C == 16)));
}

// ypass_t64 addresses each component's r_ys (with its kYTailRows) by 32-bit byte offsets
bool t64_fits(const df_handle *h)
{
    int nyp = 0;
    for (int c = 0; c < 3; ++c) nyp = std::max(nyp, h->setup.comp[c].Ny_max);
    return (double)(h->Ny + 2 * nyp + kYTailRows) * h->Pzy * 8.0 < 4294967296.0;
}

// This handle's z-strip of the plane, its launch shapes and its share of the coefficient stream.
int plan_strips(df_handle *h)
{
    const Setup &s = h->setup;
    // ---- partition (host)
    h->Ny = s.Ny;
    h->Nz_g = s.Nz;
    h->z0 = (int)((long long)h->rank * s.Nz / h->world);
    h->z1 = (int)((long long)(h->rank + 1) * s.Nz / h->world);
    h->Nz_loc = h->z1 - h->z0;
    if (h->Nz_loc < 1) return fail(DF_EINVAL, "more z-strips than plane columns");
    h->nstrips = (h->Nz_loc + kStrip - 1) / kStrip;
    h->Pz = h->nstrips * kStrip;
    for (int c = 0; c < 3; ++c)
        if (h->world > 1 && s.comp[c].Nz_max > h->Nz_loc)
            return fail(DF_EINVAL, "z-strip narrower than the z half-width: use fewer GPUs");
    // Default launch shapes, measured on MI355X (tools/tune_sweep.py, tools/ab.py; profiles/r1/probe/
    // tune_small_planes.jsonl): c3-class planes packed 2 rows per wave, table 4. Where a wave's serial tap chain
    // rather than bandwidth sets the time - y half-widths >= 128 (the reference's own grid: 212) or
    // under ~1 wave per SIMD - packed takes 1 row with the 8-deep load pipeline, table 1 row (round 3).
    if (h->rows_per_wave == 0) {
        int nymax = 0;
        for (int c = 0; c < 3; ++c) nymax = std::max(nymax, s.comp[c].Ny_max);
        const bool long_chain = nymax >= 128;
        const bool tiny = (long long)h->nstrips * ((s.Ny + 1) / 2) < 1024;
        // table mode, long chains: 1 row per wave with the noise 4 groups ahead (ydepth): the reference's grid
        // -4..-7% per call against 2 rows (profiles/r3/ao)
        if (h->coeff_mode == DF_COEFF_TABLE) h->rows_per_wave = long_chain ? 1 : 4;
        else if (long_chain || tiny) {
            h->rows_per_wave = 1;
            h->yunroll = 8;
        } else h->rows_per_wave = 2;
        // table mode, long chains: the noise staged in LDS per block of rows (ylds): round 3's ypass_tlds (the
        // reference's grid y-pass 0.051 -> 0.043 ms, call -9%, profiles/r3/bd), round 5's ypass_t64 (64-column
        // tiles, one cell and one row per lane, heaviest blocks first, whole-window chunks: 40.4 -> 24.7 us alone,
        // profiles/r5). c3 and c2 (short chains, FP64-issue-bound) lose with LDS staging.
        if (h->coeff_mode == DF_COEFF_TABLE && long_chain) h->ylds = s.per_cell ? 2 : 3;
        // ypass_t64 at 2 rows per wave (round 6): with the per-chunk bookkeeping down to increments, two rows' chains
        // per lane beat one on two boxes (kernel alone -9% and -11%, call -7%; profiles/r6/d, e); round 5's form
        // lost with 2 (its scalar bookkeeping, 1.45 scalar instructions per vector one, was the bottleneck)
        if (h->ylds == 3) h->yt_rows = 2;
        // Long chains, packed: one block per row pair, noise loads shared by both rows, the next chunk in
        // flight, XCD runs of equal bytes (the reference's grid: y-pass 0.209 (one wave per tile) -> 0.181
        // (one block per tile) -> 0.157 ms; profiles/r2/ab_ycoop_native.jsonl, ab_ycoop2_native.jsonl).
        // c3-class planes lose with it.
        // Inside each XCD run, groups of 4 tiles go heaviest first (ycoop_order 4): the widest stencils no
        // longer start last (reference's grid y-pass -2.5%; ascending order 0 and groups of 1/16/64 measured
        // alongside in profiles/r3/p).
        if (h->coeff_mode == DF_COEFF_PACKED && long_chain) {
            h->ycoop = 7;
            h->ycoop_order = 4;
            // tiles whose widest row has N >= 96 run as two 64-column halves, N >= 192 as four 32-column
            // quarters (balance_ycoop2): the reference's grid call -4.2% and another -0.8% (one-handle A/B,
            // 60-call windows, both orders; profiles/r5/m; halves at thresholds 64-160 within 1%, r5/g)
            h->ycoop_split = 96;
            h->ycoop_split4 = 192;
        }
        // Long chains, both modes: the y-pass runs ahead on its own stream (df_handle::yahead), so a call's
        // z-pass shares the chip with later calls' y-passes instead of idling beside its own latency-bound tail
        // (one-handle A/B with 60-call windows, both orders: the reference's grid packed -0.5%, table -1%; c3
        // table, c2 and c1 neutral or slower, so off there; profiles/r5/m, i)
        if (long_chain) h->yahead = 1;
        // Up to 2048 z tiles with short chains (c1: 128, c2: 2048), packed: a wave per component in the z-pass,
        // 3x the waves in flight (c1 z-pass 11.9 -> 9.0 us, profiles/r2/ab_zsplit.jsonl; c2 z-pass -2.5%, call
        // -1%, 60-call windows in both orders, profiles/r5/n; the reference grid's 2040 long-chain tiles gain
        // nothing)
        const long long ztiles = (long long)h->nstrips * s.Ny;
        if (h->coeff_mode == DF_COEFF_PACKED && (ztiles < 1024 || (!long_chain && ztiles <= 2048))) h->zsplit = 1;
    }
    // Planes of <= 1024 attempt blocks: K3 plans its own waves (one launch fewer: table mode the
    // reference's grid -5% per call, c1/c2 even; packed c2 -8..-10%, c1 -7%, profiles/r2/
    // ab_fuse_plan_packed.jsonl). Packed planes with long y chains keep
    // the scan-and-plan launch: the fused K3's extra waves beside the row-pair y-pass cost the
    // reference's grid 11% (profiles/r2/ab_fuse_plan.jsonl).
    h->fuse_plan = h->coeff_mode == DF_COEFF_TABLE || h->ycoop < 7 ? 1 : 0;
    // Table mode generates its noise through the run form (round 4: group counts, one wave per piece of needed
    // chunks): with split counting it needs no pass over the whole stream after the exchange and its counts
    // travel in the halo group (c4 over 8, one rank: 0.25-0.26 -> 0.24 ms per call, profiles/r4/d); on one GPU
    // it is even with Kc + K3a (c3 0.364 vs 0.366 ms, profiles/r4/e).
    h->gen_dense = h->coeff_mode == DF_COEFF_TABLE ? 2 : 0;
    const int Ny = s.Ny;
    for (int c = 0; c < 3; ++c) {
        CompDev &d = h->c[c];
        const ComponentSetup &F = s.comp[c];
        d.Nyp = F.Ny_max;
        d.Nzp = F.Nz_max;
        d.rz_pitch = h->Pz + 2 * d.Nzp;
        d.by_size = d.bz_size = 0; // |by|, |bz| of the reference (df.cpp:151, 191) over this strip's cells
        for (int j = 0; j < Ny; ++j) {
            if (!s.per_cell) {
                d.by_size += (long long)h->Nz_loc * (2 * F.Ny_row[j] + 1);
                d.bz_size += (long long)h->Nz_loc * (2 * F.Nz_row[j] + 1);
                continue;
            }
            for (int k = h->z0; k < h->z1; ++k) {
                d.by_size += 2 * F.Ny_at(j, k) + 1;
                d.bz_size += 2 * F.Nz_at(j, k) + 1;
            }
        }
    }

    // Ghost columns (table-mode z-strips, row-uniform N): the widest z half-width of the plane's components
    // (Nzp, which the z-halo holds) on each side that has a neighbour. The ry pitch Pzy holds the widened strip.
    h->Pzy = h->Pz;
    if (h->coeff_mode == DF_COEFF_TABLE && h->world > 1 && !s.per_cell) {
        int G = 0;
        for (int c = 0; c < 3; ++c) G = std::max(G, h->c[c].Nzp);
        G = (G + 1) / 2 * 2; // even: the y-pass's 16-B pairs stay aligned in rz
        h->ghost_cap = 1;
        h->Gl = h->rank > 0 ? G : 0;
        h->Gr = h->rank < h->world - 1 ? G : 0;
        h->Wext = h->Nz_loc + h->Gl + h->Gr;
        h->nstrips_g = (h->Wext + kStrip - 1) / kStrip;
        h->Pzy = std::max(h->Pz, h->nstrips_g * kStrip);
    }
    if (h->ylds == 3 && !t64_fits(h)) h->ylds = 2; // ypass_t64 addresses r_ys with 32-bit offsets

    // Write windows (SweepArgs::ywin_T): on planes whose sweeps stream >= 2 GB of packed coefficients per
    // pass the waves hold their stores for a chip-wide window of 2.56 us every 41 us; c3 -5.1% per call,
    // c5 -3.1% (profiles/r1/probe/win_*.json). Smaller planes (c2: +4.7%) and the VALU-bound table mode
    // (+40%) store at once.
    {
        long long by = 0, bz = 0;
        for (int c = 0; c < 3; ++c) {
            by += h->c[c].by_size;
            bz += h->c[c].bz_size;
        }
        if (h->coeff_mode != DF_COEFF_TABLE) {
            if (8 * by >= 2000000000LL) h->ywin_T = 4096, h->ywin_W = 256;
            if (8 * bz >= 2000000000LL) h->zwin_T = 4096, h->zwin_W = 256;
        }
    }

    return DF_OK;
}

// RNG stream geometry (df.cpp:343-348 order) and launch size.
int plan_rng(df_handle *h)
{
    const Setup &s = h->setup;
    const int Ny = s.Ny;
    RngGeom &g = h->geom;
    g.seg[0] = 0;
    for (int c = 0; c < 3; ++c) {
        const uint64_t Ly = (uint64_t)s.Nz * (Ny + 2 * h->c[c].Nyp);
        const uint64_t Lz = (uint64_t)Ny * (s.Nz + 2 * h->c[c].Nzp);
        if (Ly >= (1ull << 32) || Lz >= (1ull << 32)) return fail(DF_EINVAL, "noise array exceeds 2^32 normals");
        g.seg[2 * c + 1] = g.seg[2 * c] + Ly;
        g.seg[2 * c + 2] = g.seg[2 * c + 1] + Lz;
    }
    g.Q = g.seg[6];
    for (int sidx = 0; sidx < 6; ++sidx) {
        const int c = sidx >> 1;
        const uint32_t W = (sidx & 1) ? (uint32_t)(s.Nz + 2 * h->c[c].Nzp) : (uint32_t)s.Nz;
        g.width[sidx] = W;
        g.rows[sidx] = (sidx & 1) ? (uint32_t)Ny : (uint32_t)(Ny + 2 * h->c[c].Nyp);
        // ceil(2^64 / W): floor(p * inv / 2^64) == p / W for every p < 2^32
        g.inv_width[sidx] = (W == 1) ? 0 : (uint64_t)(~0ull / W) + 1;
    }
    g.fast_log = 2; // glibc's own log in the polar transform: normals bit-identical (tests/test_rng_log.py)
    g.nt_stores = 1; // noise written past the caches: it is read once, by the next call's sweeps (A/B -1.4%)
    const PcgJump next = pcg_jump(4ull * 64); // attempt start -> the lane's next attempt start
    g.next_mult = next.mult;
    g.next_plus = next.plus;
    { // s_k = A_k s0 + C_k (k steps): the next attempt's s_k = J s_k + (A_k C_J + C_k - J C_k)
        const PcgJump j1 = pcg_jump(1), j3 = pcg_jump(3);
        g.next_plus1 = j1.mult * next.plus + j1.plus - next.mult * j1.plus;
        g.next_plus3 = j3.mult * next.plus + j3.plus - next.mult * j3.plus;
    }
    g.Nz_g = s.Nz;
    g.Pz = h->Pzy;
    g.z0 = h->z0;
    g.z1 = h->z1;
    g.yz0 = h->z0; // ghost columns off (select_ghost switches)
    g.yz1 = h->z1;
    g.is_first = h->rank == 0;
    g.is_last = h->rank == h->world - 1;
    {
        const double A = std::ceil((double)g.Q / 2.0);
        const double p = 0.78539816339744830962; // pi/4 acceptance of the polar method
        const double T = A / p * 1.002 + 16.0 * std::sqrt(A) + 8192.0;
        h->rng_blocks = (int)std::ceil(T / kRngBlockAttempts);
    }
    // K3 splits each attempt wave over up to 16 waves while the plane has fewer than ~4 waves of
    // attempts per SIMD (c1: 140 waves; the reference's grid: ~750): a wave's 16 serial polar
    // iterations (log, sqrt, divide in FP64) otherwise set K3's time on small planes. Packed planes aim at
    // half of that (round 6): their K3 runs beside HBM-bound sweeps, whose bandwidth its extra waves take
    // (c2 packed -4..-5% per call with gen_split 2 against 4, both orders; c1, the reference's grid and the
    // table planes neutral; profiles/r6/k)
    const long long k3_waves = h->coeff_mode == DF_COEFF_PACKED ? 2048 : 4096;
    g.gen_split = 1;
    while (g.gen_split < kRngPerThread && (long long)h->rng_blocks * kWavesPerBlock * g.gen_split < k3_waves)
        g.gen_split *= 2;
    if (g.gen_split < 1 || g.gen_split > kRngPerThread || (g.gen_split & (g.gen_split - 1)))
        return fail(DF_EINVAL, "gen_split must be a power of two <= 16");
    return DF_OK;
}

// Device, streams and the noise-set events.
int open_device(df_handle *h, int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(DF_EHIP, "no HIP device visible");
    if (device >= ndev) return fail(DF_EINVAL, "device ordinal out of range");
    h->device = device;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    // Sweeps on the high-priority queue, noise for the next call on the low one:
    // the memory-bound sweeps keep their waves; the compute-bound RNG fills gaps.
    int prio_lo = 0, prio_hi = 0;
    HIP_OR(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi), DF_EHIP);
    const int use_prio = 0; // measured: priorities cost 1-2% wall time (in-process A/B, tools/ab.py)
    HIP_OR(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, use_prio ? prio_hi : 0), DF_EHIP);
    HIP_OR(hipStreamCreateWithPriority(&h->rng_stream, hipStreamNonBlocking, use_prio ? prio_lo : 0), DF_EHIP);
    // The two streams' per-call hand-offs (noise ready, noise set free) order kernels on this GPU and
    // are never waited on by the host (df_sync synchronizes the streams themselves), so they are
    // recorded without the system-scope fence: the reference's grid -2.2%, c2 -1.5% (packed) /
    // -3.6% (table) per call, c3 unchanged (profiles/r2/ab_event_scope.jsonl; a device-scope
    // release instead was neutral).
    const unsigned ev_flags = hipEventDisableTiming | hipEventDisableSystemFence;
    for (int set = 0; set < 2; ++set) {
        HIP_OR(hipEventCreateWithFlags(&h->ev_rng[set], ev_flags), DF_EHIP);
        HIP_OR(hipEventCreateWithFlags(&h->ev_swept[set], ev_flags), DF_EHIP);
    }
    for (int k = 0; k < kMaxNoiseSets; ++k) HIP_OR(hipEventCreateWithFlags(&h->ev_release[k], ev_flags), DF_EHIP);
    return DF_OK;
}

// ystream exists only on handles that run the y-pass ahead: a process's streams share the device's few hardware
// queues (GPU_MAX_HW_QUEUES, 4 here), and a third stream on every handle put the stream and rng_stream of a second
// live handle on one queue, serialising its noise generation with its sweeps (c3 table 0.341 -> 0.380 ms on the
// bench line, where the packed handle stays open beside it; profiles/r5/e)
// comm_stream (high priority) exists only where the halo overlap form can run: packed z-strips by default, table
// ones once halo_overlap is set to 1 - the streams of a process share the device's hardware queues (above)
int ensure_comm_stream(df_handle *h)
{
    const bool ov = h->halo_overlap > 0 || (h->halo_overlap < 0 && h->coeff_mode == DF_COEFF_PACKED);
    if (h->comm_stream || !ov || h->device < 0 || h->world < 2 || !(h->comm || h->solo_strip)) return DF_OK;
    int prio_lo = 0, prio_hi = 0;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi), DF_EHIP);
    HIP_OR(hipStreamCreateWithPriority(&h->comm_stream, hipStreamNonBlocking, prio_hi), DF_EHIP);
    return DF_OK;
}

int ensure_ystream(df_handle *h)
{
    if (!h->ystream && h->yahead && h->tracing) h->ystream = (hipStream_t)(kTrStream + 2);
    if (h->ystream || !h->yahead || h->device < 0) return DF_OK;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(hipStreamCreateWithFlags(&h->ystream, hipStreamNonBlocking), DF_EHIP);
    return DF_OK;
}

// Per-N coefficient tables (table mode, and the source K0 expands the packed stream from) and the
// per-row constants of apply_RST_scaling / get_rho_T_fluc.
int upload_tables(df_handle *h)
{
    const Setup &s = h->setup;
    const int Ny = s.Ny;
    std::vector<int> tab_off_h;
    std::vector<double> tab_h;
    int Nmax_all = 0;
    for (auto &kv : s.coeffs) Nmax_all = std::max(Nmax_all, kv.first);
    // Every N's half-vector padded with zeros to Nmax_all+1 entries, and a zero row at N = 0:
    // per-cell reads past a lane's own N (up to its strip's N) then add exact zeros.
    const size_t L = (size_t)Nmax_all + 1;
    tab_off_h.assign(Nmax_all + 1, 0);
    tab_h.assign(L, 0.0); // row 0: all zeros (padding lanes)
    for (auto &kv : s.coeffs) {
        tab_off_h[kv.first] = (int)tab_h.size();
        tab_h.insert(tab_h.end(), kv.second.begin(), kv.second.end());
        tab_h.resize(tab_h.size() + (L - kv.second.size()), 0.0);
    }
    // The same coefficients as full symmetric vectors b[|i|], i = -N..N, each starting on a
    // 64-B boundary: a wave-uniform run of 8 taps is then one aligned s_load_dwordx16 with
    // no |i| address arithmetic (row-uniform N: every non-grid plane).
    std::vector<int> tabf_off_h(Nmax_all + 1, 0);
    std::vector<double> tabf_h;
    // kTabGuard zeros before every vector and after the last: ypass_t64 reads a whole chunk's window of taps even
    // where it hangs past a row's first or last tap, and a zero tap leaves the sum bit for bit (+0 + (+-0) = +0
    // before the first tap, x + (+-0) = x after the last); the first kTabGuard entries are zeros for rows with
    // no tap in a chunk. Also the slack of the other sweeps' whole-window scalar loads.
    constexpr int kTabGuard = 24; // >= the longest ypass_t64 chunk (yt_chunk)
    for (auto &kv : s.coeffs) {
        tabf_h.resize((tabf_h.size() + kTabGuard + 7) / 8 * 8, 0.0);
        tabf_off_h[kv.first] = (int)tabf_h.size();
        const int n = kv.first;
        for (int i = -n; i <= n; ++i) tabf_h.push_back(kv.second[i < 0 ? -i : i]);
    }
    tabf_h.resize(tabf_h.size() + 2 * kTabGuard, 0.0);
    int rc;
    if ((rc = dalloc_t(h, &h->tab, tab_h.size()))) return rc;
    if ((rc = dalloc_t(h, &h->tab_off, tab_off_h.size()))) return rc;
    if ((rc = upload(h, h->tab, tab_h.data(), tab_h.size()))) return rc;
    if ((rc = upload(h, h->tab_off, tab_off_h.data(), tab_off_h.size()))) return rc;
    if ((rc = dalloc_t(h, &h->tabf, tabf_h.size()))) return rc;
    if ((rc = dalloc_t(h, &h->tabf_off, tabf_off_h.size()))) return rc;
    if ((rc = upload(h, h->tabf, tabf_h.data(), tabf_h.size()))) return rc;
    if ((rc = upload(h, h->tabf_off, tabf_off_h.data(), tabf_off_h.size()))) return rc;

    // ---- row constants of apply_RST_scaling / get_rho_T_fluc (df.cpp:425-438, 474)
    std::vector<double> rowc(7 * (size_t)Ny);
    for (int j = 0; j < Ny; ++j) {
        double b;
        if (s.R11[j] < 1e-10) b = 0.0;
        else b = s.R21[j] / std::sqrt(s.R11[j]);
        rowc[j] = std::sqrt(s.R11[j]);
        rowc[Ny + j] = b;
        rowc[2 * Ny + j] = std::sqrt(s.R22[j] - b * b);
        rowc[3 * Ny + j] = std::sqrt(s.R33[j]);
        rowc[4 * Ny + j] = -0.5 * (1.4 - 1) * s.Ms[j] * s.Ms[j] / s.Us[j];
        rowc[5 * Ny + j] = s.Ts[j];
        rowc[6 * Ny + j] = s.rhos[j];
    }
    if ((rc = dalloc_t(h, &h->rowc, rowc.size()))) return rc;
    return upload(h, h->rowc, rowc.data(), rowc.size());
}

// Noise sets, fields, tap ranges and (packed mode) the strip-tap-major coefficient stream.
int alloc_components(df_handle *h)
{
    const Setup &s = h->setup;
    // Packed mode: the six coefficient arrays (By0 Bz0 By1 Bz1 By2 Bz2, each 2 MiB aligned) share ONE
    // allocation instead of one each: c3 3.47-3.51 -> 3.37-3.41 ms per call, mean over 8 handles on each
    // of two boxes (profiles/r2/pool/; order By0 By1 By2 Bz0 Bz1 Bz2 = 2 gains a little less). Same
    // bytes, same kernels: where the 20 GB stream lands is all that changes (presumably larger physical
    // fragments for one large allocation, i.e. fewer address-translation misses; not measured).
    const int pool = 1;
    const int Ny = s.Ny;
    int rc;
    const size_t n_loc = (size_t)Ny * h->Nz_loc;
    for (int c = 0; c < 3; ++c) {
        CompDev &d = h->c[c];
        const ComponentSetup &F = s.comp[c];
        for (int set = 0; set < h->nsets; ++set) {
            if ((rc = dalloc_t(h, &d.ry[set], (size_t)(Ny + 2 * d.Nyp + kYTailRows) * h->Pzy))) return rc;
            if ((rc = dalloc_t(h, &d.rz[set], (size_t)Ny * d.rz_pitch))) return rc;
        }
        if ((rc = dalloc_t(h, &d.filt_old, n_loc))) return rc;
        if ((rc = dalloc_t(h, &d.fluc, n_loc))) return rc;
        // tap range of each (strip, row): the largest N among the strip's cells of that row
        std::vector<int> Nst[2];
        for (int dir = 0; dir < 2; ++dir) {
            Nst[dir].resize((size_t)h->nstrips * Ny);
            for (int st = 0; st < h->nstrips; ++st)
                for (int j = 0; j < Ny; ++j) {
                    int m = dir ? F.Nz_row[j] : F.Ny_row[j];
                    if (s.per_cell) {
                        m = 0;
                        const int k1 = std::min(h->z0 + (st + 1) * kStrip, h->z1);
                        for (int k = h->z0 + st * kStrip; k < k1; ++k) m = std::max(m, dir ? F.Nz_at(j, k) : F.Ny_at(j, k));
                    }
                    Nst[dir][(size_t)st * Ny + j] = m;
                }
        }
        h->y_nst[c] = Nst[0]; // host copy for the row-block y-pass's XCD balance
        if ((rc = dalloc_t(h, &d.ycoop2_perm, 4 * (size_t)h->nstrips * ((Ny + 1) / 2)))) return rc; // quarters
        balance_ycoop2(h, c);
        if ((rc = upload_ycoop2_perm(h, c))) return rc;
        if ((rc = dalloc_t(h, &d.Ny_st, Nst[0].size()))) return rc;
        if ((rc = dalloc_t(h, &d.Nz_st, Nst[1].size()))) return rc;
        if ((rc = upload(h, d.Ny_st, Nst[0].data(), Nst[0].size()))) return rc;
        if ((rc = upload(h, d.Nz_st, Nst[1].data(), Nst[1].size()))) return rc;
        if (h->ghost_cap) { // the widened strip's tap ranges: row-uniform, the same for each of its 128-column strips
            std::vector<int> ng((size_t)h->nstrips_g * Ny);
            for (int st = 0; st < h->nstrips_g; ++st)
                for (int j = 0; j < Ny; ++j) ng[(size_t)st * Ny + j] = F.Ny_row[j];
            if ((rc = dalloc_t(h, &d.Ny_st_g, ng.size()))) return rc;
            if ((rc = upload(h, d.Ny_st_g, ng.data(), ng.size()))) return rc;
        }
        if (c == 2 && h->coeff_mode == DF_COEFF_TABLE && !s.per_cell) { // ypass_t64's list, sized for 1 row per wave
            h->ylist_cap = 3 * ((h->Nz_loc + 63) / 64) * ((Ny + 3) / 4);
            if ((rc = dalloc_t(h, &h->ylist, h->ylist_cap))) return rc;
            if ((rc = build_ylist(h, false))) return rc;
            if (h->ghost_cap) {
                h->ylist_g_cap = 3 * ((h->Wext + 63) / 64) * ((Ny + 3) / 4);
                if ((rc = dalloc_t(h, &h->ylist_g, h->ylist_g_cap))) return rc;
                if ((rc = build_ylist(h, true))) return rc;
            }
        }
        if (s.per_cell) {
            std::vector<int> nc[2];
            for (int dir = 0; dir < 2; ++dir) {
                nc[dir].resize(n_loc);
                for (int j = 0; j < Ny; ++j)
                    for (int kl = 0; kl < h->Nz_loc; ++kl)
                        nc[dir][(size_t)j * h->Nz_loc + kl] = dir ? F.Nz_at(j, h->z0 + kl) : F.Ny_at(j, h->z0 + kl);
            }
            if ((rc = dalloc_t(h, &d.Ny_cell, n_loc))) return rc;
            if ((rc = dalloc_t(h, &d.Nz_cell, n_loc))) return rc;
            if ((rc = upload(h, d.Ny_cell, nc[0].data(), n_loc))) return rc;
            if ((rc = upload(h, d.Nz_cell, nc[1].data(), n_loc))) return rc;
        }
        if (h->coeff_mode == DF_COEFF_PACKED) {
            // strip-tap-major offsets, one block per (strip, row)
            for (int dir = 0; dir < 2; ++dir) {
                std::vector<long long> off((size_t)h->nstrips * Ny);
                long long run = 0;
                for (int st = 0; st < h->nstrips; ++st)
                    for (int j = 0; j < Ny; ++j) {
                        off[(size_t)st * Ny + j] = run;
                        run += (long long)(2 * Nst[dir][(size_t)st * Ny + j] + 1) * kStrip;
                    }
                long long **doff = dir ? &d.bzoff : &d.byoff;
                double **dB = dir ? &d.Bz : &d.By;
                (dir ? d.bz_elems : d.by_elems) = run;
                if ((rc = dalloc_t(h, doff, off.size()))) return rc;
                if ((rc = upload(h, *doff, off.data(), off.size()))) return rc;
                if (pool) continue; // one allocation for all six arrays, below
                if ((rc = dalloc_t(h, dB, (size_t)run))) return rc;
                HIP_OR(launch_expand_coeffs(*dB, *doff, dir ? d.Nz_st : d.Ny_st, dir ? d.Nz_cell : d.Ny_cell,
                                            h->tab, h->tab_off, Ny, h->nstrips, h->Nz_loc, h->stream),
                       DF_EHIP);
            }
        }
    }
    if (pool && h->coeff_mode == DF_COEFF_PACKED) {
        const size_t align = (2u << 20) / sizeof(double);
        size_t total = 0;
        for (int k = 0; k < 6; ++k) {
            const CompDev &d = h->c[pool == 1 ? k >> 1 : k % 3];
            const int dir = pool == 1 ? k & 1 : k / 3;
            total += ((size_t)(dir ? d.bz_elems : d.by_elems) + align - 1) / align * align;
        }
        double *base = nullptr;
        if ((rc = dalloc_t(h, &base, total))) return rc;
        for (int k = 0; k < 6; ++k) {
            CompDev &d = h->c[pool == 1 ? k >> 1 : k % 3];
            const int dir = pool == 1 ? k & 1 : k / 3;
            double *&B = dir ? d.Bz : d.By;
            B = base;
            base += ((size_t)(dir ? d.bz_elems : d.by_elems) + align - 1) / align * align;
            HIP_OR(launch_expand_coeffs(B, dir ? d.bzoff : d.byoff, dir ? d.Nz_st : d.Ny_st, dir ? d.Nz_cell : d.Ny_cell,
                                        h->tab, h->tab_off, Ny, h->nstrips, h->Nz_loc, h->stream),
                   DF_EHIP);
        }
    }
    if ((rc = dalloc_t(h, &h->T, n_loc))) return rc;
    return dalloc_t(h, &h->rho, n_loc);
}

// RNG buffers, Brown jump tables, the error flags and the stream's starting state.
int alloc_rng(df_handle *h, const df_config_c *cfg)
{
    RngGeom &g = h->geom;
    int rc;
    for (int c = 0; c < 3; ++c) {
        g.Nzp[c] = h->c[c].Nzp;
        g.rz_pitch[c] = h->c[c].rz_pitch;
    }
    if ((rc = dalloc_t(h, &h->rstate, h->nsets))) return rc;
    h->rng_chunk = (h->rng_blocks + h->world - 1) / h->world;
    const int nb_pad = h->rng_chunk * h->world;
    if ((rc = dalloc_t(h, &h->counts, nb_pad))) return rc;
    if ((rc = dalloc_t(h, &h->offsets, nb_pad))) return rc;
    if ((nb_pad + 1023) / 1024 > 1024) return fail(DF_EINVAL, "plane too large for the RNG scan (> 2^20 attempt blocks)");
    if ((rc = dalloc_t(h, &h->part, (nb_pad + 1023) / 1024))) return rc;
    if ((rc = dalloc_t(h, &h->masks, (size_t)nb_pad * kRngThreads))) return rc;
    if ((rc = dalloc_t(h, &h->wave_counts, (size_t)nb_pad * kWavesPerBlock))) return rc;
    {
        long long st1 = 0, stw = 0, lo, to;
        record_layout(h->rng_blocks, &st1, &lo, &to);
        record_layout(h->rng_chunk, &stw, &lo, &to);
        if ((rc = dalloc_t(h, &h->xbuf, (size_t)std::max(st1, stw * h->world)))) return rc;
        // the run generation's share lookup holds at most 64 shares: split counting with it needs <= 64 ranks
        if (h->world > 64 && h->gen_dense == 2 && !h->rng_replicate)
            return fail(DF_EINVAL, "more than 64 z-strip ranks with split counting (set rng_replicate 1)");
    }
    h->geom.nb_groups = (long long)h->rng_blocks * 64;
    if ((rc = dalloc_t(h, &h->tasks, (size_t)nb_pad * kWavesPerBlock))) return rc;
    if ((rc = dalloc_t(h, &h->ntasks, 1))) return rc;
    HIP_OR(hipEventCreateWithFlags(&h->ev_counted, hipEventDisableTiming), DF_EHIP);
    {
        // jump tables: block b starts 4*4096*b outputs in; thread tid = 64*w + l starts
        // 4*(1024*w + l) further (wave w owns attempts [1024*w, 1024*(w+1)) of the block)
        auto compose = [](PcgJumpDev a, PcgJump b) { // b after a
            return PcgJumpDev{b.mult * a.mult, b.mult * a.plus + b.plus};
        };
        std::vector<PcgJumpDev> jb(nb_pad), jt(kRngThreads);
        const PcgJump blk = pcg_jump(4ull * kRngBlockAttempts);
        jb[0] = PcgJumpDev{1, 0};
        for (int b = 1; b < nb_pad; ++b) jb[b] = compose(jb[b - 1], blk);
        for (int t = 0; t < kRngThreads; ++t) {
            const PcgJump j = pcg_jump(4ull * (uint64_t)((t >> 6) * (kRngBlockAttempts / 4) + (t & 63)));
            jt[t] = PcgJumpDev{j.mult, j.plus};
        }
        PcgJumpDev *djb = nullptr, *djt = nullptr;
        if ((rc = dalloc_t(h, &djb, jb.size()))) return rc;
        if ((rc = dalloc_t(h, &djt, jt.size()))) return rc;
        if ((rc = upload(h, djb, jb.data(), jb.size()))) return rc;
        if ((rc = upload(h, djt, jt.data(), jt.size()))) return rc;
        h->geom.jump_block = djb;
        h->geom.jump_thread = djt;
        // run generation: group gi of a block starts 4*64*gi outputs in, lane l of a group 4*l further
        std::vector<PcgJumpDev> jg(64), jl(64);
        for (int i = 0; i < 64; ++i) {
            const PcgJump a = pcg_jump(4ull * 64 * (uint64_t)i), b = pcg_jump(4ull * (uint64_t)i);
            jg[i] = PcgJumpDev{a.mult, a.plus};
            jl[i] = PcgJumpDev{b.mult, b.plus};
        }
        PcgJumpDev *djg = nullptr, *djl = nullptr;
        if ((rc = dalloc_t(h, &djg, 64))) return rc;
        if ((rc = dalloc_t(h, &djl, 64))) return rc;
        if ((rc = upload(h, djg, jg.data(), 64))) return rc;
        if ((rc = upload(h, djl, jl.data(), 64))) return rc;
        h->geom.jump_gi = djg;
        h->geom.jump_lane = djl;
    }
    {
        std::vector<LogTabEntry> lt(kLogTab);
        build_log_table(lt.data());
        LogTabEntry *dlt = nullptr;
        if ((rc = dalloc_t(h, &dlt, lt.size()))) return rc;
        if ((rc = upload(h, dlt, lt.data(), lt.size()))) return rc;
        h->geom.log_tab = dlt;
    }
    HIP_OR(hipHostMalloc((void **)&h->err_host, 3 * sizeof(int), hipHostMallocMapped), DF_EHIP);
    h->err_host[0] = h->err_host[1] = h->err_host[2] = 0;
    HIP_OR(hipHostGetDevicePointer((void **)&h->err_dev, h->err_host, 0), DF_EHIP);

    uint64_t seed = cfg->seed;
    if (cfg->seed_from_random_device) seed = (uint64_t)std::random_device{}(); // df.cpp:334
    RngStateDev st0{pcg_seed1(seed), 0, 0, 0.0};
    if (cfg->rng_resume) st0 = RngStateDev{cfg->rng_state, cfg->rng_saved_flag ? 1 : 0, 0, cfg->rng_saved};
    return upload(h, h->rstate, &st0, 1);
}

// Run generation tables (RngGeom::gen_dense 2): for each parity f of the incoming cached normal, the
// 64-rank chunks whose pairs (positions f + 2r, f + 2r + 1) store something on this GPU - the same
// columns as stream_dest: r_ys columns [z0, z1), r_zs pads on the plane's first/last strip - plus the
// chunk of the call's last rank A - 1 (it sets the stream state); their fast destinations and the pieces.
int build_run_tables(df_handle *h, int yz0, int yz1, df_handle::RunTables &out)
{
    RngGeom g = h->geom;
    g.yz0 = yz0;
    g.yz1 = yz1;
    const uint64_t A0 = (g.Q + 1) / 2; // A for f = 0 (f = 1: A0 or A0 - 1)
    const uint64_t nch = (A0 + 63) / 64;
    if (nch >= (1ull << 31)) return fail(DF_EINVAL, "plane too large for the dense generation tables");
    std::vector<uint32_t> bits[2], list[2];
    for (int f = 0; f < 2; ++f) {
        bits[f].assign((nch + 31) / 32 + 2, 0u); // host bitmap of the needed chunks, listed below
        const long long A = (long long)((g.Q - f + 1) / 2);
        auto mark = [&](uint64_t qa, uint64_t qb) { // positions [qa, qb)
            if (qb <= qa || qb < (uint64_t)f + 1) return;
            const long long r0 = qa > (uint64_t)f ? (long long)((qa - f) / 2) : 0;
            long long r1 = (long long)((qb - 1 - f) / 2); // inclusive
            if (r1 > A - 1) r1 = A - 1;
            for (long long c = r0 >> 6; c <= (r1 >> 6); ++c) bits[f][c >> 5] |= 1u << (c & 31);
        };
        for (int sidx = 0; sidx < 6; ++sidx) {
            const uint64_t base = g.seg[sidx], W = g.width[sidx], rows = g.rows[sidx];
            const int cmp = sidx >> 1;
            if ((sidx & 1) == 0) { // r_ys: this strip's columns of every row
                if (g.yz0 == 0 && (uint64_t)g.yz1 == W) mark(base, base + rows * W);
                else
                    for (uint64_t r = 0; r < rows; ++r) mark(base + r * W + g.yz0, base + r * W + g.yz1);
            } else { // r_zs: the raw-noise pads (df.cpp:343-348) on the plane's edge strips
                const uint64_t nzp = (uint64_t)g.Nzp[cmp];
                for (uint64_t r = 0; r < rows; ++r) {
                    if (g.is_first) mark(base + r * W, base + r * W + nzp);
                    if (g.is_last) mark(base + r * W + nzp + g.Nz_g, base + (r + 1) * W);
                }
            }
        }
        if (A > 0) bits[f][((A - 1) >> 6) >> 5] |= 1u << (((A - 1) >> 6) & 31);
        for (uint64_t c = 0; c < nch; ++c)
            if ((bits[f][c >> 5] >> (c & 31)) & 1u) list[f].push_back((uint32_t)c);
    }
    // K3r fast chunks: no rank past the call or the call's last (that one sets the stream state), all 128
    // positions in one stream array with at most one row wrap, and the positions this GPU stores (stream_dest:
    // r_ys columns [z0, z1), the r_zs pads of the plane's edge strips) one run [lo, hi) whose destinations are
    // affine in the position on either side of the wrap: destinations by arithmetic. Round 4: r_zs pads and
    // partial chunks (a strip's first and last of each row) too, not only whole r_ys chunks.
    auto dest_of = [&g](int su, uint64_t row, uint64_t col, long long &off) { // host mirror of stream_dest
        const int cmp = su >> 1;
        if ((su & 1) == 0) {
            if (col < (uint64_t)g.yz0 || col >= (uint64_t)g.yz1) return false;
            off = (long long)(row * (uint64_t)g.Pz + (col - (uint64_t)g.yz0));
            return true;
        }
        long long lc;
        if (col < (uint64_t)g.Nzp[cmp]) {
            if (!g.is_first) return false;
            lc = (long long)col;
        } else if (col >= (uint64_t)(g.Nzp[cmp] + g.Nz_g)) {
            if (!g.is_last) return false;
            lc = (long long)col - g.z0;
        } else {
            return false;
        }
        off = (long long)(row * (uint64_t)g.rz_pitch[cmp]) + lc;
        return true;
    };
    std::vector<ChunkDest> dest[2];
    for (int f = 0; f < 2; ++f) {
        const long long A = (long long)((g.Q - f + 1) / 2);
        dest[f].resize(std::max<size_t>(1, list[f].size()), ChunkDest{0, 0, 0, -1, 0, 0});
        for (size_t i = 0; i < list[f].size(); ++i) {
            const uint64_t c = list[f][i], q0 = f + 128 * c;
            if ((long long)(64 * c + 63) >= A - 1) continue;
            int su = 0;
            while (su < 5 && q0 >= g.seg[su + 1]) ++su;
            const uint64_t W = g.width[su];
            if (q0 + 128 > g.seg[su + 1] || W == 0) continue;
            uint64_t row = (q0 - g.seg[su]) / W, col = (q0 - g.seg[su]) % W;
            int lo = -1, hi = -1, wr = 128, wraps = 0;
            long long d0 = 0, d1 = 0;
            bool ok = true;
            for (int e = 0; e < 128 && ok; ++e) {
                long long off;
                if (dest_of(su, row, col, off)) {
                    const long long d = off - e;
                    if (lo < 0) {
                        lo = e;
                        d0 = d1 = d;
                    } else if (hi >= 0) {
                        ok = false; // a second run
                    } else if (d != d1) {
                        if (d1 != d0) ok = false; // a second change of the affine map
                        d1 = d;
                        wr = e;
                    }
                } else if (lo >= 0 && hi < 0) {
                    hi = e;
                }
                if (++col == W) {
                    col = 0;
                    ++row;
                    ++wraps;
                }
            }
            if (!ok || lo < 0 || wraps > 1) continue;
            if (hi < 0) hi = 128;
            ChunkDest d{};
            d.off = d0;
            d.jump = (int)(d1 - d0);
            d.wr = (uint8_t)wr;
            d.arr = (signed char)su;
            d.lo = (uint8_t)lo;
            d.hi = (uint8_t)hi;
            dest[f][i] = d;
        }
    }
    int rc;
    for (int f = 0; f < 2; ++f) {
        ChunkDest *dd = nullptr;
        if ((rc = dalloc_t(h, &dd, dest[f].size()))) return rc;
        if ((rc = upload(h, dd, dest[f].data(), dest[f].size()))) return rc;
        out.chunk_dest[f] = dd;
    }
    // Run generation (gen_dense 2): the list cut into pieces of consecutive chunks, at most kRunPiece each and
    // of near-equal length within a run (a 9-chunk row segment of a strip is one piece, not 8 + 1)
    const uint32_t kRunPiece = 12; // piece lengths 6 / 12 / 24 / 48 measured: 12 kept (profiles/r4/n)
    for (int f = 0; f < 2; ++f) {
        std::vector<RunPiece> pcs;
        const std::vector<uint32_t> &L = list[f];
        for (size_t i = 0; i < L.size();) {
            size_t j = i + 1;
            while (j < L.size() && L[j] == L[j - 1] + 1) ++j; // run [i, j)
            const uint32_t run = (uint32_t)(j - i), np = (run + kRunPiece - 1) / kRunPiece;
            for (uint32_t k = 0, at = 0; k < np; ++k) {
                const uint32_t n = (run - at) / (np - k) + ((run - at) % (np - k) ? 1 : 0);
                const uint32_t c0 = L[i + at];
                pcs.push_back(RunPiece{c0, (uint32_t)(i + at), n, 0});
                at += n;
            }
            i = j;
        }
        RunPiece *dp = nullptr;
        if ((rc = dalloc_t(h, &dp, std::max<size_t>(1, pcs.size())))) return rc;
        if (!pcs.empty() && (rc = upload(h, dp, pcs.data(), pcs.size()))) return rc;
        out.pieces[f] = dp;
        out.npieces[f] = (int)pcs.size();
    }
    return DF_OK;
}

// The r_ys columns the RNG stores and the run tables for the ghost mode in use.
void apply_ghost_geom(df_handle *h)
{
    const int m = h->ghost ? 1 : 0;
    h->geom.yz0 = h->ghost ? h->z0 - h->Gl : h->z0;
    h->geom.yz1 = h->ghost ? h->z1 + h->Gr : h->z1;
    if (!h->dense_ready && !h->run_tab[0].pieces[0]) return; // run tables not built (yet)
    for (int f = 0; f < 2; ++f) {
        h->geom.chunk_dest[f] = h->run_tab[m].chunk_dest[f];
        h->geom.pieces[f] = h->run_tab[m].pieces[f];
        h->geom.npieces[f] = h->run_tab[m].npieces[f];
    }
}

int alloc_dense(df_handle *h)
{
    int rc = build_run_tables(h, h->z0, h->z1, h->run_tab[0]);
    if (!rc && h->ghost_cap) rc = build_run_tables(h, h->z0 - h->Gl, h->z1 + h->Gr, h->run_tab[1]);
    if (rc) return rc;
    apply_ghost_geom(h);
    h->dense_ready = true;
    return DF_OK;
}

// Halo buffers and the RCCL communicators (cfg->comm_id).
int open_comm(df_handle *h, const df_config_c *cfg)
{
    int rc;
    if (h->world > 1 && (rc = alloc_halo(h))) return rc;
    // A communicator of one rank is accepted too: the same init, split and grouped all-gather then run on a
    // single GPU (tests/test_gpu_parity.py::test_rccl_single_rank_matches_plain), the halo being a no-op.
    if (cfg->comm_id) {
        ncclUniqueId id;
        std::memcpy(&id, cfg->comm_id, sizeof(id));
        NCCL_OR(ncclCommInitRank(&h->comm, h->world, id, h->rank));
        NCCL_OR(ncclCommSplit(h->comm, 0, h->rank, &h->rng_comm, nullptr)); // RNG all-gather, own stream
        HIP_OR(hipEventCreateWithFlags(&h->ev_halo, hipEventDisableTiming), DF_EHIP);
        HIP_OR(hipEventRecord(h->ev_halo, h->stream), DF_EHIP);
        h->split_count = !h->rng_replicate;
    }
    if (h->world > 1 && (cfg->comm_id || h->solo_strip)) {
        if (int rc2 = ensure_comm_stream(h)) return rc2;
        HIP_OR(hipEventCreateWithFlags(&h->ev_packed, hipEventDisableTiming), DF_EHIP);
        HIP_OR(hipEventCreateWithFlags(&h->ev_xchg, hipEventDisableTiming), DF_EHIP);
        HIP_OR(hipEventCreateWithFlags(&h->ev_unpacked, hipEventDisableTiming), DF_EHIP);
    }
    return DF_OK;
}

// DF_DEVICE_TRACE: no GPU; stand-in streams and events, the state the create path would leave (the seed in state
// slot 0, every release event recorded once on the stream)
int open_trace(df_handle *h)
{
    h->device = -1;
    h->tracing = true;
    h->stream = (hipStream_t)(kTrStream + 0);
    h->rng_stream = (hipStream_t)(kTrStream + 1);
    for (int i = 0; i < 2; ++i) {
        h->ev_rng[i] = (hipEvent_t)(kTrEvent + TE_RNG + i);
        h->ev_swept[i] = (hipEvent_t)(kTrEvent + TE_SWEPT + i);
    }
    for (int k = 0; k < kMaxNoiseSets; ++k) h->ev_release[k] = (hipEvent_t)(kTrEvent + TE_RELEASE + k);
    h->ev_counted = (hipEvent_t)(kTrEvent + TE_COUNTED);
    h->ev_xchg = (hipEvent_t)(kTrEvent + TE_XCHG);
    h->ev_halo = (hipEvent_t)(kTrEvent + TE_HALO);
    h->dense_ready = h->gen_dense == 2 && h->geom.gen_split == 1;
    if (int rc = ensure_ystream(h)) return rc;
    trace(h, TR_STATE_W, -1, 0, 0);
    for (int k = 0; k < kMaxNoiseSets; ++k) Q_OR(q_record(h, h->ev_release[k], h->stream, -(1ll << 40)));
    return DF_OK;
}

int build(df_handle *h, const df_config_c *cfg)
{
    int rc;
    if ((rc = read_config(h, cfg))) return rc;
    std::string err;
    if (!build_setup(h->flow, h->spec, h->setup, err)) return fail(DF_EIO, err);
    if ((rc = plan_strips(h))) return rc;
    if ((rc = plan_rng(h))) return rc;
    // Hand-off batch: small single-GPU planes, where the two per-call cross-stream hand-offs are 10-40% of
    // a call (c2 packed -17%, the reference's grid -9%, c1 -40% with both removed; profiles/r3/h), take
    // epochs of hb calls over 2*hb noise sets (a few MB each there): c1 (16k cells) 4, c2 (262k) 2
    // (c1 -23% packed / -15% table, c2 -6% / -9%; profiles/r3/i/hb_ab.jsonl). Planes with long y chains
    // (the reference's grid) ran slower with epochs in round 2 (+3% packed / +14% table: their latency-bound
    // y-pass read noise written calls earlier, no longer cache-warm); with round 3's y-passes (row-pair
    // dispatch order, table at 1 row per wave with a deep noise ring) epochs of 4 pay there too: -3..-4%
    // packed, -5..-6% table (profiles/r3/at; c2 keeps 2, c1 4: r3/au). Split planes and RCCL handles keep
    // one hand-off per call (their RNG exchanges stay in call order with the halo).
    {
        int nymax = 0;
        for (int c = 0; c < 3; ++c) nymax = std::max(nymax, h->setup.comp[c].Ny_max);
        const long long cells = (long long)h->Ny * h->Nz_loc;
        if (h->world == 1 && !cfg->comm_id)
            h->hb = cells <= (1ll << 16) || (nymax >= 128 && cells <= (1ll << 20)) ? 4 : cells <= (1ll << 20) ? 2 : 1;
        // Table mode on larger single-GPU planes (round 4): its RNG chain competes for the same VALU slots as the
        // sweeps and, with one generation per hand-off, ends up on the critical path; two generations per epoch
        // let it run a call further ahead (c3: 0.366 -> 0.352 ms per call median, profiles/r4/e).
        if (h->world == 1 && !cfg->comm_id && h->coeff_mode == DF_COEFF_TABLE && h->hb == 1) h->hb = 2;
    }
    if (h->hb != 1 && h->hb != 2 && h->hb != 4) return fail(DF_EINVAL, "handoff batch must be 1, 2 or 4");
    if (h->world > 1 || cfg->comm_id) h->hb = 1;
    // RCCL table z-strips run the y-pass ahead: the next call's y-pass fills the SIMDs while the stream waits on
    // the halo exchange (one c4/8 rank with a 40 us stand-in exchange: 0.244 / 0.238 -> 0.215 / 0.210 ms, ranks
    // 0 / 4; 0.196-0.198 either way without it; profiles/r5/d/strip.jsonl)
    if (h->world > 1 && h->coeff_mode == DF_COEFF_TABLE && (cfg->comm_id || h->solo_strip)) h->yahead = 1;
    // ahead handles hold three epochs of noise sets (consumed, swept ahead, generating), and so do batched
    // single-GPU table planes (consumed and two generating; prefetch_epochs): their RNG chain competes with the
    // sweeps for the same VALU slots, and a whole epoch of slack lets it fill the sweeps' gaps (same-box A/B of two
    // builds, 60-call windows: c3 table 0.334-0.338 -> 0.327 ms, c2 table -2%; profiles/r5/r)
    h->hb_conf = h->hb;
    h->nsets = h->hb > 1 ? 2 * h->hb : 2;
    if (h->yahead || (h->world == 1 && !cfg->comm_id && h->coeff_mode == DF_COEFF_TABLE && h->hb > 1))
        h->nsets = 3 * h->hb;
    // z-strip handles in table mode, one process per GPU (split counting, the fused exchange): generations two
    // calls ahead. look is consulted only by fused_active() handles (one generation per hand-off), so in-process
    // groups and batched handles keep look 1 and the noise sets their batch needs (a batched handle
    // with look 2 was cut to 4 sets where its epochs need 2 * hb).
    if (h->world > 1 && h->coeff_mode == DF_COEFF_TABLE && (cfg->comm_id || h->solo_strip)) h->look = 2;
    if (h->hb > 1) h->look = 1;
    if (h->look == 2) h->nsets = std::max(h->nsets, 4);
    if (cfg->device == DF_DEVICE_TRACE) return open_trace(h);
    if (cfg->device < 0) { // host-only handle: setup queries, no GPU
        h->device = -1;
        return DF_OK;
    }
    if ((rc = open_device(h, cfg->device))) return rc;
    if ((rc = ensure_ystream(h))) return rc;
    if ((rc = upload_tables(h))) return rc;
    if ((rc = alloc_components(h))) return rc;
    if ((rc = alloc_rng(h, cfg))) return rc;
    if (h->gen_dense == 2 && h->geom.gen_split == 1 && (rc = alloc_dense(h))) return rc;
    if ((rc = open_comm(h, cfg))) return rc;
    for (int k = 0; k < kMaxNoiseSets; ++k) HIP_OR(hipEventRecord(h->ev_release[k], h->stream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return DF_OK;
}

int step0(df_handle *h)
{
    // Constructor step 0 (df.cpp:57-62): noise, sweeps, RST; no correlation, no SRA.
    int rc;
    if ((rc = consume_gen(h))) return rc;
    if ((rc = fused_gen_begin(h))) return rc;
    if (!h->cur_swept && (rc = phase_ypass(h, 7))) return rc;
    if ((rc = phase_halo_zpass(h, false, false, 0.0))) return rc;
    if ((rc = prefetch_gen(h))) return rc;
    if ((rc = sync_all(h))) return rc;
    return check_rng_error(h);
}

void destroy(df_handle *h)
{
    if (!h) return;
    if (h->tracing) { // stand-in streams and events, nothing allocated
        delete h;
        return;
    }
    // Drain every stream before any buffer or communicator goes: comm_stream may still hold a send/recv,
    // an unpack or the edge z-pass when a call failed part-way (phase_halo_zpass's error returns).
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->rng_stream) (void)hipStreamSynchronize(h->rng_stream);
    if (h->ystream) (void)hipStreamSynchronize(h->ystream);
    if (h->comm_stream) (void)hipStreamSynchronize(h->comm_stream);
    for (auto &pe : h->ev)
        for (auto &e : pe.e) (void)hipEventDestroy(e);
    for (auto &ye : h->yev)
        for (auto &e : ye.e) (void)hipEventDestroy(e);
    for (void *p : h->allocs) {
        registry_release(p); // before the free: another thread's hipMalloc may get the address back at once
        (void)hipFree(p);
    }
    if (h->err_host) (void)hipHostFree(h->err_host);
    if (h->rng_comm) ncclCommDestroy(h->rng_comm);
    if (h->comm) ncclCommDestroy(h->comm);
    if (h->ev_counted) (void)hipEventDestroy(h->ev_counted);
    if (h->ev_halo) (void)hipEventDestroy(h->ev_halo);
    for (int set = 0; set < 2; ++set) {
        if (h->ev_rng[set]) (void)hipEventDestroy(h->ev_rng[set]);
        if (h->ev_swept[set]) (void)hipEventDestroy(h->ev_swept[set]);
    }
    for (int k = 0; k < kMaxNoiseSets; ++k)
        if (h->ev_release[k]) (void)hipEventDestroy(h->ev_release[k]);
    if (h->rng_stream) (void)hipStreamDestroy(h->rng_stream);
    if (h->ystream) (void)hipStreamDestroy(h->ystream);
    if (h->comm_stream) (void)hipStreamDestroy(h->comm_stream);
    if (h->ev_packed) (void)hipEventDestroy(h->ev_packed);
    if (h->ev_xchg) (void)hipEventDestroy(h->ev_xchg);
    if (h->ev_unpacked) (void)hipEventDestroy(h->ev_unpacked);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

// Strips of one plane held by handles of this process: each phase runs on every
// handle before the halo copies, then the z-pass. corr_sra = false is step 0.
int group_step(df_handle **hs, int n, bool corr_sra, double dt)
{
    if (!hs || n < 1) return fail(DF_EINVAL, "empty handle group");
    for (int r = 0; r < n; ++r) {
        if (!hs[r]) return fail(DF_EINVAL, "null handle in group");
        if (hs[r]->rank != r || hs[r]->world != n || hs[r]->comm)
            return fail(DF_EINVAL, "group handles must be ranks 0..n-1 of one plane, created without comm_id");
        // before any strip consumes a generation: a refused call leaves every stream state as it was
        if (hs[r]->ghost != hs[0]->ghost) return fail(DF_EINVAL, "halo_ghost differs between the strips of a group");
    }
    int rc;
    for (int r = 0; r < n; ++r) {
        df_handle *h = hs[r];
        HIP_OR(hipSetDevice(h->device), DF_EHIP);
        if ((rc = check_rng_error(h))) return rc;
        if ((rc = consume_gen(h))) return rc;
        if (!h->cur_swept && (rc = phase_ypass(h, 7))) return rc;
        if (!h->ghost && (rc = phase_halo_pack(h))) return rc;
    }
    const bool ghost = hs[0]->ghost != 0;
    if (!ghost)
        for (int r = 0; r < n; ++r) HIP_OR(hipStreamSynchronize(hs[r]->stream), DF_EHIP);
    for (int r = 0; r < n; ++r) {
        df_handle *h = hs[r];
        HIP_OR(hipSetDevice(h->device), DF_EHIP);
        const size_t bytes = h->halo_elems * sizeof(double);
        if (!ghost && r > 0) HIP_OR(hipMemcpyAsync(h->recv_l, hs[r - 1]->send_r, bytes, hipMemcpyDefault, h->stream), DF_EHIP);
        if (!ghost && r < n - 1) HIP_OR(hipMemcpyAsync(h->recv_r, hs[r + 1]->send_l, bytes, hipMemcpyDefault, h->stream), DF_EHIP);
        if (!ghost && (rc = phase_halo_unpack(h))) return rc;
        if ((rc = phase_zpass(h, corr_sra, corr_sra, dt))) return rc;
        if ((rc = prefetch_gen(h))) return rc;
    }
    for (int r = 0; r < n; ++r) {
        if ((rc = sync_all(hs[r]))) return rc;
        if ((rc = check_rng_error(hs[r]))) return rc;
        if (corr_sra && (rc = write_csv_if(hs[r]))) return rc;
    }
    return DF_OK;
}

bool valid(df_handle *h)
{
    if (!h) {
        g_err = "null handle";
        return false;
    }
    return true;
}

// Handles that own GPU state (not host-only).
bool valid_dev(df_handle *h)
{
    if (!valid(h)) return false;
    if (h->device < 0) {
        g_err = "host-only handle (created with device = -1) has no GPU state";
        return false;
    }
    return true;
}

// Handles the pipeline runs on: GPU handles and DF_DEVICE_TRACE handles (df_filter, the stream state, the hand-off
// batch and the y-pass-ahead setting)
bool valid_sched(df_handle *h) { return valid(h) && (h->tracing || valid_dev(h)); }

// Handles whose results may be read. A DFAMD_SOLO_STRIP handle (tools/strip_timing.py: one rank of
// a split plane timed alone, halo never exchanged) computes wrong fields by design.
bool valid_out(df_handle *h)
{
    if (!valid_dev(h)) return false;
    if (h->solo_strip) {
        g_err = "DFAMD_SOLO_STRIP handle: timing only, its fields and stream state are not results";
        return false;
    }
    return true;
}

} // namespace

// =================================================================== C ABI

extern "C" {

int df_abi_version(void) { return DF_ABI_VERSION; }

const char *df_last_error(void) { return g_err.c_str(); }

size_t df_config_sizeof(void) { return sizeof(df_config_c); }

const char *df_data_dir(void)
{
    static const std::string dir = [] {
        Dl_info info{};
        std::string lib = dladdr((void *)&df_data_dir, &info) && info.dli_fname ? info.dli_fname : "";
        const size_t slash = lib.find_last_of('/');
        return (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/data";
    }();
    return dir.c_str();
}

void df_config_default(df_config_c *cfg)
{
    std::memset(cfg, 0, sizeof(*cfg));
    Flow f;
    cfg->d_i = f.d_i;
    cfg->rho_e = f.rho_e;
    cfg->U_e = f.U_e;
    cfg->mu_e = f.mu;
    cfg->seed = 0;
    cfg->seed_from_random_device = 1;
    cfg->plane = DF_PLANE_NATIVE;
    cfg->coeff_mode = DF_COEFF_TABLE; // same fields bit for bit as DF_COEFF_PACKED, no B stream
    static const std::string rst = std::string(df_data_dir()) + "/RST.dat";
    static const std::string line = std::string(df_data_dir()) + "/line.dat";
    cfg->vel_fluc_file = rst.c_str();
    cfg->line_file = line.c_str();
    cfg->world = 1;
    cfg->rows_per_wave = 0;
}

df_handle *df_create(const df_config_c *cfg)
{
    if (!cfg) {
        g_err = "null config";
        return nullptr;
    }
    df_handle *h = new df_handle();
    int rc = DF_OK;
    if (cfg->device >= 0) (void)hipGetLastError(); // a stale error of earlier HIP work is not this handle's
    if (cfg->device < 0 && cfg->world > 1 && !cfg->comm_id) rc = DF_OK; // host-only strip planning
    else if (cfg->world > 1 && !cfg->comm_id && !(std::getenv("DFAMD_SOLO_STRIP") && std::atoi(std::getenv("DFAMD_SOLO_STRIP"))))
        rc = fail(DF_EINVAL, "world > 1 needs comm_id (RCCL) or df_create_group (in-process strips)");
    if (rc == DF_OK) rc = build(h, cfg);
    if (rc == DF_OK && (h->device >= 0 || h->tracing)) rc = step0(h);
    if (rc != DF_OK) {
        std::string keep = g_err;
        destroy(h);
        g_err = keep;
        return nullptr;
    }
    g_err.clear();
    return h;
}

static int restart_pipeline(df_handle *h, int hb_new);

int df_filter(df_handle *h, double dt)
{
    if (!valid_sched(h)) return DF_EINVAL;
    int rc = check_rng_error(h);
    if (rc) return rc;
    if (h->world > 1 && !h->comm && !h->solo_strip)
        return fail(DF_EINVAL, "z-strip handle without RCCL: use df_filter_group");
    if (!h->tracing) HIP_OR(hipSetDevice(h->device), DF_EHIP);
    if (h->hb != h->hb_conf && ++h->calls_since_load > kHbRestoreCalls) { // no state loads lately: batch again
        if ((rc = sync_all(h)) || (rc = restart_pipeline(h, h->hb_conf))) return rc;
    }
    // Sampled phase events: each hipEventRecord is a queue packet between this call's kernels, and on
    // short calls six of them cost up to 10% of the call (tools/event_cost.py; profiles/r3/d)
    h->prof_call = h->profiling && (h->prof_seq++ % h->profile_every) == 0;
    const bool prof = prof_on(h);
    if ((rc = consume_gen(h))) return rc;
    if ((rc = fused_gen_begin(h))) return rc;
    ev_record(h, 0);
    if (prof) h->ev[h->ev_used].ahead = h->cur_swept;
    if (!h->cur_swept && (rc = phase_ypass(h, 7))) return rc;
    ev_record(h, 1);
    if ((rc = phase_halo_zpass(h, true, true, dt))) return rc; // phase event 2 inside
    ev_record(h, 3);
    if ((rc = prefetch_gen(h))) return rc; // next call's noise, under this call's sweeps
    if (prof) h->ev_used++;
    h->prof_call = false;
    return write_csv_if(h);
}

int df_filter_group(df_handle **hs, int n, double dt) { return group_step(hs, n, true, dt); }

int df_create_group(const df_config_c *cfgs, int n, df_handle **out)
{
    if (!cfgs || !out || n < 1) return fail(DF_EINVAL, "bad group arguments");
    for (int r = 0; r < n; ++r) out[r] = nullptr;
    int rc = DF_OK;
    for (int r = 0; r < n && rc == DF_OK; ++r) {
        if (cfgs[r].comm_id || cfgs[r].rank != r || cfgs[r].world != n) {
            rc = fail(DF_EINVAL, "group configs must be ranks 0..n-1 of one plane without comm_id");
            break;
        }
        out[r] = new df_handle();
        rc = build(out[r], &cfgs[r]);
    }
    if (rc == DF_OK && n > 1) {
        auto grp = std::make_shared<std::vector<df_handle *>>(out, out + n);
        for (int r = 0; r < n; ++r) {
            out[r]->group = grp;
            out[r]->split_count = true; // each strip counts 1/n of the attempts (SURVEY 8e option A)
        }
    }
    if (rc == DF_OK) rc = group_step(out, n, false, 0.0); // the constructor's step 0
    if (rc != DF_OK) {
        std::string keep = g_err;
        for (int r = 0; r < n; ++r) {
            destroy(out[r]);
            out[r] = nullptr;
        }
        g_err = keep;
    }
    return rc;
}

int df_generate_white_noise(df_handle *h)
{
    if (!valid_dev(h)) return DF_EINVAL;
    int rc = consume_gen(h);
    return rc ? rc : prefetch_gen(h);
}

int df_filtering_sweeps(df_handle *h, int comp)
{
    if (!valid_dev(h)) return DF_EINVAL;
    if (comp < 0 || comp > 2) return fail(DF_EINVAL, "comp must be 0, 1 or 2");
    if (h->world > 1) return fail(DF_EINVAL, "stage API is single-strip only");
    int rc;
    if (!h->c[comp].filt && (rc = dalloc_t(h, &h->c[comp].filt, (size_t)h->Ny * h->Nz_loc))) return rc;
    if ((rc = phase_ypass(h, 1 << comp))) return rc;
    SweepArgs a = sweep_args(h);
    a.comps_mask = 1 << comp;
    a.write_filt = 1;
    HIP_OR(launch_zpass(a, h->coeff_mode == DF_COEFF_TABLE, h->stream), DF_EHIP);
    return DF_OK;
}

static int stage_elementwise(df_handle *h, int op, int comp, double dt)
{
    if (!valid_dev(h)) return DF_EINVAL;
    for (int c = 0; c < 3; ++c)
        if ((op == 1 || c == comp) && !h->c[c].filt && op != 2)
            return fail(DF_EINVAL, "df_filtering_sweeps must run before this stage");
    SweepArgs a = sweep_args(h);
    if (op == 0) {
        const double pi = 3.141592654; // df.cpp:411
        const double alpha = std::exp(-pi * dt / h->setup.comp[comp].Lt);
        a.sa[comp] = std::sqrt(alpha);
        a.s1a[comp] = std::sqrt(1.0 - alpha);
    }
    HIP_OR(launch_stage(a, op, comp, h->stream), DF_EHIP);
    return DF_OK;
}

int df_correlate_fields(df_handle *h, int comp, double dt)
{
    if (comp < 0 || comp > 2) return fail(DF_EINVAL, "comp must be 0, 1 or 2");
    return stage_elementwise(h, 0, comp, dt);
}

int df_apply_RST_scaling(df_handle *h) { return stage_elementwise(h, 1, 0, 0.0); }

int df_get_rho_T_fluc(df_handle *h) { return stage_elementwise(h, 2, 0, 0.0); }

int df_get_field(df_handle *h, int which, double *out)
{
    if (!valid_out(h) || !out) return DF_EINVAL;
    const double *src = df_device_field(h, which);
    if (!src) return DF_EINVAL;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(hipMemcpyAsync(out, src, (size_t)h->Ny * h->Nz_loc * 8, hipMemcpyDeviceToHost, h->stream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return check_rng_error(h);
}

int df_get_fields(df_handle *h, int n, const int *which, double *const *host_out)
{
    // The C++ mirrors' per-call refresh: every copy queued on the handle's stream, ONE synchronisation.
    // Into pinned memory (df_host_pin) the copies are DMA transfers that overlap each other's setup;
    // into pageable memory the runtime stages them (still one host wait at the end).
    if (!valid_out(h) || n < 0 || (n && (!which || !host_out))) return fail(DF_EINVAL, "df_get_fields: bad arguments");
    const size_t bytes = (size_t)h->Ny * h->Nz_loc * 8;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    for (int i = 0; i < n; ++i) {
        const double *src = df_device_field(h, which[i]);
        if (!src || !host_out[i]) return fail(DF_EINVAL, "df_get_fields: field " + std::to_string(i));
        HIP_OR(hipMemcpyAsync(host_out[i], src, bytes, hipMemcpyDeviceToHost, h->stream), DF_EHIP);
    }
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return check_rng_error(h);
}

int df_alloc_registry(const void *p, size_t bytes, int claim)
{
    if (!p || (claim && !bytes)) return fail(DF_EINVAL, "df_alloc_registry: null or empty range");
    if (claim) return registry_claim(p, bytes, nullptr);
    registry_release(p);
    return DF_OK;
}

long long df_alloc_registry_count(void)
{
    AllocRegistry &r = registry();
    std::lock_guard<std::mutex> lk(r.mu);
    return (long long)r.live.size();
}

int df_host_pin(void *p, size_t bytes)
{
    if (!p || !bytes) return fail(DF_EINVAL, "df_host_pin: null or empty range");
    HIP_OR(hipHostRegister(p, bytes, hipHostRegisterDefault), DF_EHIP);
    return DF_OK;
}

int df_host_unpin(void *p)
{
    if (!p) return fail(DF_EINVAL, "df_host_unpin: null pointer");
    HIP_OR(hipHostUnregister(p), DF_EHIP);
    return DF_OK;
}

int df_set_field(df_handle *h, int which, const double *host_in)
{
    if (!valid_dev(h) || !host_in) return DF_EINVAL;
    if (which < DF_U || which > DF_FILT_OLD_W) return fail(DF_EINVAL, "df_set_field: only u, v, w, T, rho and filt_old");
    double *dst = const_cast<double *>(df_device_field(h, which));
    if (!dst) return DF_EINVAL;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    int rc = sync_all(h); // a running call must not see half a field
    if (rc) return rc;
    HIP_OR(hipMemcpyAsync(dst, host_in, (size_t)h->Ny * h->Nz_loc * 8, hipMemcpyHostToDevice, h->stream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return DF_OK;
}

const double *df_device_field(df_handle *h, int which)
{
    if (!valid_out(h)) return nullptr;
    switch (which) {
    case DF_U: case DF_V: case DF_W: return h->c[which].fluc;
    case DF_T: return h->T;
    case DF_RHO: return h->rho;
    case DF_FILT_OLD_U: case DF_FILT_OLD_V: case DF_FILT_OLD_W: return h->c[which - DF_FILT_OLD_U].filt_old;
    case DF_FILT_U: case DF_FILT_V: case DF_FILT_W:
        if (h->c[which - DF_FILT_U].filt) return h->c[which - DF_FILT_U].filt;
        g_err = "filt is only materialized by the stage API (df_filtering_sweeps)";
        return nullptr;
    }
    g_err = "unknown field";
    return nullptr;
}

int df_dims(df_handle *h, int *Ny, int *Nz, int *z0, int *z1)
{
    if (!valid(h)) return DF_EINVAL;
    if (Ny) *Ny = h->Ny;
    if (Nz) *Nz = h->Nz_g;
    if (z0) *z0 = h->z0;
    if (z1) *z1 = h->z1;
    return DF_OK;
}

int df_get_row(df_handle *h, int which, double *out)
{
    if (!valid(h) || !out) return DF_EINVAL;
    const Setup &s = h->setup;
    const std::vector<double> *v = nullptr;
    switch (which) {
    case DF_ROW_R11: v = &s.R11; break;
    case DF_ROW_R21: v = &s.R21; break;
    case DF_ROW_R22: v = &s.R22; break;
    case DF_ROW_R33: v = &s.R33; break;
    case DF_ROW_US: v = &s.Us; break;
    case DF_ROW_TS: v = &s.Ts; break;
    case DF_ROW_RHOS: v = &s.rhos; break;
    case DF_ROW_MS: v = &s.Ms; break;
    case DF_ROW_PS: v = &s.Ps; break;
    case DF_ROW_YC: v = &s.yc; break;
    case DF_ROW_YC_D: v = &s.yc_d; break;
    default: return fail(DF_EINVAL, "unknown row");
    }
    std::copy(v->begin(), v->begin() + s.Ny, out);
    return DF_OK;
}

double df_get_scalar(df_handle *h, int which)
{
    if (!valid(h)) return NAN;
    switch (which) {
    case 0: return h->setup.u_tau;
    case 1: return h->setup.tau_w;
    case 2: return h->setup.d_v;
    }
    return NAN;
}

int df_get_halfwidths(df_handle *h, int comp, int dir, int *out)
{
    if (!valid(h) || !out || comp < 0 || comp > 2 || dir < 0 || dir > 1) return fail(DF_EINVAL, "bad argument");
    const ComponentSetup &F = h->setup.comp[comp];
    for (int j = 0; j < h->Ny; ++j)
        for (int k = 0; k < h->Nz_loc; ++k)
            out[(size_t)j * h->Nz_loc + k] = dir ? F.Nz_at(j, h->z0 + k) : F.Ny_at(j, h->z0 + k);
    return DF_OK;
}

int df_get_offsets(df_handle *h, int comp, int dir, int *out)
{
    if (!valid(h) || !out || comp < 0 || comp > 2 || dir < 0 || dir > 1) return fail(DF_EINVAL, "bad argument");
    const ComponentSetup &F = h->setup.comp[comp];
    long long b_size = 0; // df.cpp:151-152 / 191-192, over this strip's cells in row-major order
    for (int j = 0; j < h->Ny; ++j)
        for (int k = 0; k < h->Nz_loc; ++k) {
            const int N = dir ? F.Nz_at(j, h->z0 + k) : F.Ny_at(j, h->z0 + k);
            b_size += 2 * N + 1;
            out[(size_t)j * h->Nz_loc + k] = (int)(b_size - N - 1);
        }
    return DF_OK;
}

int df_get_comp_info(df_handle *h, int comp, int *Ny_max, int *Nz_max, long long *by_size, long long *bz_size)
{
    if (!valid(h) || comp < 0 || comp > 2) return fail(DF_EINVAL, "bad argument");
    if (Ny_max) *Ny_max = h->c[comp].Nyp;
    if (Nz_max) *Nz_max = h->c[comp].Nzp;
    if (by_size) *by_size = h->c[comp].by_size;
    if (bz_size) *bz_size = h->c[comp].bz_size;
    return DF_OK;
}

int df_get_coeffs(df_handle *h, int comp, int dir, double *out, long long n)
{
    if (!valid(h) || !out || comp < 0 || comp > 2 || dir < 0 || dir > 1) return fail(DF_EINVAL, "bad argument");
    const long long need = dir ? h->c[comp].bz_size : h->c[comp].by_size;
    if (n < need) return fail(DF_EINVAL, "output too small for the packed coefficient vector");
    const ComponentSetup &F = h->setup.comp[comp];
    long long pos = 0;
    for (int j = 0; j < h->Ny; ++j)
        for (int k = 0; k < h->Nz_loc; ++k) {
            const int N = dir ? F.Nz_at(j, h->z0 + k) : F.Ny_at(j, h->z0 + k);
            const std::vector<double> &half = h->setup.coeffs.at(N);
            for (int i = -N; i <= N; ++i) out[pos++] = half[i < 0 ? -i : i];
        }
    return DF_OK;
}

int df_rng_state(df_handle *h, uint64_t *state, int *saved_flag, double *saved)
{
    if (h && h->tracing) {
        trace(h, TR_SYNC);
        trace(h, TR_STATE_R, -1, gen_set(h, h->gen_used), h->gen_used);
        if (state) *state = 0;
        if (saved_flag) *saved_flag = 0;
        if (saved) *saved = 0;
        return DF_OK;
    }
    if (!valid_out(h)) return DF_EINVAL;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    int rc = sync_all(h);
    if (rc) return rc;
    RngStateDev st; // state after the last visible step: slot gen_used % 2 (a prefetched
                    // generation writes the other slot)
    HIP_OR(hipMemcpyAsync(&st, h->rstate + gen_set(h, h->gen_used), sizeof st, hipMemcpyDeviceToHost, h->stream),
           DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    if (state) *state = st.state;
    if (saved_flag) *saved_flag = st.saved_flag;
    if (saved) *saved = st.saved;
    return check_rng_error(h);
}

// Discard the prefetched generations (the caller has synchronized both streams) and start epoch 0 at
// the next visible step with hand-off batch hb_new; with overlap its generations are enqueued now.
static int restart_pipeline(df_handle *h, int hb_new)
{
    h->gen_launched = h->gen_used;
    h->gen_base = h->gen_used;
    h->hb = hb_new;
    if (!h->overlap) return DF_OK;
    const long long need = h->gen_used + h->hb;
    int rc;
    while (h->gen_launched < need)
        if ((rc = launch_gen(h))) return rc;
    return DF_OK;
}

int df_set_rng_state(df_handle *h, uint64_t state, int saved_flag, double saved)
{
    if (!valid_sched(h)) return DF_EINVAL;
    if (h->group) return fail(DF_EINVAL, "df_set_rng_state on a member of an in-process strip group");
    if (!h->tracing) HIP_OR(hipSetDevice(h->device), DF_EHIP);
    int rc = sync_all(h);
    if (rc) return rc;
    if (h->tracing) {
        trace(h, TR_STATE_W, -1, gen_set(h, h->gen_used), h->gen_used);
    } else {
        RngStateDev st{state, saved_flag ? 1 : 0, 0, saved};
        HIP_OR(hipMemcpyAsync(h->rstate + gen_set(h, h->gen_used), &st, sizeof st, hipMemcpyHostToDevice, h->stream),
               DF_EHIP);
        HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    }
    h->calls_since_load = 0;
    if (h->gen_launched > h->gen_used || h->hb != 1) // the prefetched noise came from the old state: redo it
        return restart_pipeline(h, 1);
    return DF_OK;
}

long long df_stream_length(df_handle *h) { return valid(h) ? (long long)h->geom.Q : -1; }

int df_get_tuning(df_handle *h, const char *key, int *value)
{
    if (!h || !key || !value) return fail(DF_EINVAL, "null handle, key or value");
    const std::string k(key);
    const std::pair<const char *, int> keys[] = {
        {"rows_per_wave", h->rows_per_wave}, {"yunroll", h->yunroll}, {"ycoop", h->ycoop},
        {"ycoop_order", h->ycoop_order}, {"ycoop_split", h->ycoop_split}, {"ycoop_split4", h->ycoop_split4}, {"ylds", h->ylds}, {"yt_rows", h->yt_rows}, {"yt_chunk", h->yt_chunk}, {"yt_pd", h->yt_pd}, {"zsplit", h->zsplit}, {"ypass_ahead", h->yahead},
        {"zstage", h->zstage}, {"nt_stores", h->nt_stores}, {"ywin_T", h->ywin_T}, {"ywin_W", h->ywin_W}, {"zwin_T", h->zwin_T},
        {"zwin_W", h->zwin_W}, {"gen_split", h->geom.gen_split}, {"fuse_plan", h->fuse_plan},
        {"handoff_batch", h->hb_conf}, {"gen_dense", h->gen_dense}, {"fast_log", h->geom.fast_log},
        {"rng_replicate", h->rng_replicate}, {"fused_exchange", h->fused_x}, {"halo_overlap", h->halo_overlap},
        {"halo_ghost", h->ghost},
        // read-only: noise sets allocated at create, epochs generated ahead of the one consumed (prefetch_epochs)
        {"noise_sets", h->nsets}, {"prefetch_epochs", prefetch_epochs(h)}};
    for (const auto &kv : keys)
        if (k == kv.first) {
            *value = kv.second;
            return DF_OK;
        }
    return fail(DF_EINVAL, "unknown tuning key for df_get_tuning: " + k);
}

int df_set_tuning(df_handle *h, const char *key, int value)
{
    // Launch-shape knobs only: every setting produces bit-identical fields (tests/test_gpu_parity.py).
    if (!h) return fail(DF_EINVAL, "null handle");
    if (!key) return fail(DF_EINVAL, "null tuning key");
    const std::string k(key);
    if (k == "rows_per_wave") {
        if (value != 1 && value != 2 && value != 4 && value != 8)
            return fail(DF_EINVAL, "rows_per_wave must be 1, 2, 4 or 8");
        h->rows_per_wave = value;
    }
    else if (k == "yunroll") h->yunroll = value >= 8 ? 8 : value >= 4 ? 4 : 2;
    else if (k == "nt_stores") h->nt_stores = h->ynt_stores = h->geom.nt_stores = value != 0;
    else if (k == "zsplit") h->zsplit = value != 0;
    else if (k == "ypass_ahead") { // from the next epoch generated on (ep_swept)
        h->yahead = value != 0;
        if (int rc = ensure_ystream(h)) return rc;
    }
    else if (k == "zstage") h->zstage = value ? 2 : 0; // 0: the unstaged table z-pass that large halos take (tests)
    else if (k == "fused_exchange") h->fused_x = value != 0; // from the next df_filter on; the same on every rank
    else if (k == "ylds") { // LDS-staged table y-pass (2: ypass_tlds; 3: ypass_t64, 64-column tiles; 0: off)
        // (host-only handles have no list; the plane decides, as alloc_components does)
        const bool t64_plane = h->device >= 0 ? h->ylist != nullptr
                                              : h->coeff_mode == DF_COEFF_TABLE && !h->setup.per_cell;
        if (value == 3 && !t64_plane) return fail(DF_EINVAL, "ylds 3 needs a table-mode plane with row-uniform N");
        if (value == 3 && !t64_fits(h)) return fail(DF_EINVAL, "ylds 3 needs r_ys under 4 GiB per component");
        h->ylds = value == 3 ? 3 : value ? 2 : 0;
    } else if (k == "yt_pd") {
        if (value != 2 && value != 4) return fail(DF_EINVAL, "yt_pd must be 2 or 4");
        if (!t64_shape_ok(h->yt_rows, h->yt_chunk, value))
            return fail(DF_EINVAL, "yt_pd 4 is built for yt_rows 1 x yt_chunk 16 only");
        h->yt_pd = value;
    } else if (k == "yt_rows" || k == "yt_chunk") { // ypass_t64 shapes (rows x chunk), t64_shape_ok
        const int R = k == "yt_rows" ? value : h->yt_rows, C = k == "yt_chunk" ? value : h->yt_chunk;
        const int Cu = k == "yt_rows" && !t64_shape_ok(R, C, 2) ? 16 : C; // a row count alone: chunks of 16
        if (!t64_shape_ok(R, Cu, 2)) return fail(DF_EINVAL, "yt_rows x yt_chunk must be 1 x 16, 1 x 24, 2 x 8 or 2 x 16");
        if (h->device >= 0)
            if (int rc = sync_all(h)) return rc; // a queued y-pass may still read the old order
        h->yt_rows = R;
        h->yt_chunk = Cu;
        if (R != 1 || Cu != 16) h->yt_pd = 2;
        if (int rc = build_ylists(h)) return rc;
    }
    else if (k == "halo_ghost") { // the same on every rank of a plane (it decides whether a halo exchange runs)
        if (value && !h->ghost_cap)
            return fail(DF_EINVAL, "halo_ghost needs a table-mode z-strip handle with row-uniform half-widths");
        if ((value != 0) != (h->ghost != 0)) {
            std::vector<df_handle *> mem = h->group ? *h->group : std::vector<df_handle *>{h};
            if (h->device >= 0 || h->tracing)
                for (df_handle *m : mem) // queued generations and sweeps keep the layout they had
                    if (int rc = sync_all(m)) return rc;
            h->ghost = value != 0;
            apply_ghost_geom(h);
            // prefetched noise has the other layout: redo it (an in-process group generates for every strip at
            // once, so once all its strips agree)
            bool agree = true;
            for (df_handle *m : mem) agree = agree && m->ghost == h->ghost;
            if ((h->device >= 0 || h->tracing) && agree && h->gen_launched > h->gen_used) {
                if (!h->group) {
                    if (int rc = restart_pipeline(h, h->hb)) return rc;
                } else {
                    for (df_handle *m : mem) m->gen_launched = m->gen_used; // hb 1: one generation each, redone
                    if (int rc = launch_gen(h)) return rc;
                }
            }
        }
    }
    else if (k == "halo_overlap") {
        if (h->device >= 0)
            if (int rc = sync_all(h)) return rc; // a call in flight keeps the form it was enqueued with
        h->halo_overlap = value < 0 ? -1 : value != 0;
        if (int rc = ensure_comm_stream(h)) return rc;
    }

    else if (k == "ycoop_order" || k == "ycoop_split" || k == "ycoop_split4") {
        if (value < 0) return fail(DF_EINVAL, k + " must be >= 0");
        (k == "ycoop_order" ? h->ycoop_order : k == "ycoop_split" ? h->ycoop_split : h->ycoop_split4) = value;
        if (valid_dev(h)) {
            if (int rc = sync_all(h)) return rc;
            for (int c = 0; c < 3; ++c) {
                balance_ycoop2(h, c);
                if (int rc = upload_ycoop2_perm(h, c)) return rc;
            }
        }
    }
    else if (k == "ycoop") {
        if (value != 0 && value != 7)
            return fail(DF_EINVAL, "ycoop must be 0 (a wave per tile) or 7 (a block per row pair, 4 noise rows per "
                                   "wave per chunk)");
        h->ycoop = value;
    }
    else if (k == "rng_replicate") { // collective form changes: set it alike on every rank before the first df_filter
        if (h->group) return fail(DF_EINVAL, "rng_replicate applies to RCCL or single handles, not in-process groups");
        if (!value && h->world > 64 && h->gen_dense == 2)
            return fail(DF_EINVAL, "the run generation's share lookup holds at most 64 split-counting ranks");
        h->rng_replicate = value != 0;
        h->split_count = (h->comm || h->solo_strip) && !h->rng_replicate;
    }
    else if (k == "halo_loopback") {
        if (!h->comm || h->world != 1 || value < 0 || value > 2)
            return fail(DF_EINVAL, "halo_loopback needs a one-rank RCCL handle (comm_id, world 1) and a value 0-2");
        int rc;
        if (value && !h->send_l && (rc = alloc_halo(h))) return rc;
        h->halo_loopback = value;
    }
    else if (k == "fuse_plan") h->fuse_plan = value != 0;
    else if (k == "handoff_batch") {
        if (value != 1 && value != 2 && value != 4) return fail(DF_EINVAL, "handoff_batch must be 1, 2 or 4");
        if (value > 1 && (2 * value > h->nsets || h->nsets % value))
            return fail(DF_EINVAL, "handoff_batch " + std::to_string(value) + " needs at least " +
                                       std::to_string(2 * value) + " noise sets, a multiple of it; this handle has " +
                                       std::to_string(h->nsets) + " (sized at create by the plane's own batch)");
        if (value > 1 && (h->world > 1 || h->comm || h->group))
            return fail(DF_EINVAL, "handoff_batch > 1 is for single-GPU handles");
        h->hb_conf = value;
        if ((h->device >= 0 || h->tracing) && value != h->hb) {
            int rc = sync_all(h);
            if (rc) return rc;
            if ((rc = restart_pipeline(h, value))) return rc;
        } else h->hb = value;
    }
    else if (k == "gen_dense") { // collective form changes on split-counting handles: the same on every rank
        if (value != 0 && value != 2)
            return fail(DF_EINVAL, "gen_dense must be 0 (compacted K3) or 2 (run generation)");
        if (value == 2 && h->world > 64 && h->split_count)
            return fail(DF_EINVAL, "the run generation's share lookup holds at most 64 split-counting ranks");
        if (value && h->device >= 0 && !h->dense_ready) {
            int rc = alloc_dense(h);
            if (rc) return rc;
        }
        h->gen_dense = value;
    }
    else if (k == "fast_log") {
        if (value < 0 || value > 2) return fail(DF_EINVAL, "fast_log must be 0 (device log), 1 (log_r2) or 2 (glibc_log)");
        h->geom.fast_log = value;
    }
    else if (k == "ywin_T" || k == "zwin_T") {
        if (value < 0 || value > (1 << 24) || (value & (value - 1)))
            return fail(DF_EINVAL, k + " must be 0 or a power of two <= 2^24 (ticks of the 100 MHz clock)");
        (k[0] == 'y' ? h->ywin_T : h->zwin_T) = value;
    } else if (k == "ywin_W" || k == "zwin_W") {
        if (value < 0) return fail(DF_EINVAL, k + " must be >= 0");
        (k[0] == 'y' ? h->ywin_W : h->zwin_W) = value;
    }
    else if (k == "gen_split") {
        if (value < 1 || value > kRngPerThread || (value & (value - 1)))
            return fail(DF_EINVAL, "gen_split must be 1, 2, 4, 8 or 16");
        h->geom.gen_split = value;
    }
    else return fail(DF_EINVAL, "unknown tuning key: " + k);
    return DF_OK;
}

int df_set_profiling(df_handle *h, int on)
{
    if (!valid_dev(h)) return DF_EINVAL;
    if (on && h->ev.empty()) {
        h->ev.resize(1024);
        for (auto &pe : h->ev)
            for (auto &e : pe.e) HIP_OR(hipEventCreate(&e), DF_EHIP);
        h->yev.resize(256);
        for (auto &ye : h->yev)
            for (auto &e : ye.e) HIP_OR(hipEventCreate(&e), DF_EHIP);
    }
    if (on < 0) return fail(DF_EINVAL, "df_set_profiling: on must be >= 0");
    int rc = drain_profile(h);
    h->profiling = on != 0;
    h->profile_every = on > 1 ? on : 1;
    h->prof_seq = 0;
    h->prof = df_profile{};
    h->prof_rng_span = 0;
    h->prof_rng_gens = 0;
    h->yev_seq = 0;
    h->prof_y_span = h->prof_y_main = 0;
    h->prof_y_n = h->prof_y_calls = 0;
    return rc;
}

int df_get_profile(df_handle *h, df_profile *out)
{
    if (!valid_dev(h) || !out) return DF_EINVAL;
    int rc = drain_profile(h);
    *out = h->prof;
    return rc;
}

static int sync_errors(df_handle *h)
{
    if (int rc = check_rng_error(h)) return rc;
    if (const int bad = ((volatile int *)h->err_host)[1]) {
        h->err_host[1] = 0;
        return fail(DF_EINVAL, "df_gather_field: " + std::to_string(bad) + " out-of-range indices were skipped");
    }
    return DF_OK;
}

int df_sync(df_handle *h)
{
    if (!valid_dev(h)) return DF_EINVAL;
    int rc = sync_all(h);
    return rc ? rc : sync_errors(h);
}

// Every result a caller can see (fields, statistics, gathers, the stage API) is written on the handle's stream;
// the RNG stream and ystream carry later calls' noise and y-passes (df_sync waited for those
// too, on every step of a synchronous caller). The noise this call consumed was ready before its sweeps ran
// (the stream waited for it), so its error flag is final here.
int df_wait(df_handle *h)
{
    if (!valid_dev(h)) return DF_EINVAL;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return sync_errors(h);
}

int df_gather_field(df_handle *h, int which, long long n, const long long *plane_cell, double *dst,
                    const long long *dst_cell, long long dst_len, double beta)
{
    if (!valid_dev(h)) return DF_EINVAL;
    const double *src = df_device_field(h, which);
    if (!src) return DF_EINVAL;
    const long long nsrc = (long long)h->Ny * h->Nz_loc;
    if (n < 0 || (n > 0 && !dst)) return fail(DF_EINVAL, "df_gather_field: bad count or null destination");
    if (!plane_cell && n > nsrc) return fail(DF_EINVAL, "df_gather_field: n exceeds the plane without plane_cell");
    if (!dst_cell && n > dst_len) return fail(DF_EINVAL, "df_gather_field: n exceeds dst_len without dst_cell");
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(launch_gather(src, nsrc, n, plane_cell, dst, dst_cell, dst_len, beta, h->err_dev + 1, h->stream), DF_EHIP);
    return DF_OK;
}

void *df_stream(df_handle *h) { return valid_dev(h) ? (void *)h->stream : nullptr; }

long long df_trace(df_handle *h, long long *out, long long cap)
{
    if (!valid(h) || !h->tracing) {
        fail(DF_EINVAL, "df_trace needs a handle created with device = DF_DEVICE_TRACE");
        return -1;
    }
    const long long n = (long long)h->tr.size() / 6;
    if (out) std::memcpy(out, h->tr.data(), (size_t)std::min(n, std::max(0ll, cap)) * 6 * sizeof(long long));
    return n;
}

int df_get_noise(df_handle *h, int comp, int dir, double *out, long long n)
{
    if (!valid_out(h) || !out || comp < 0 || comp > 2 || dir < 0 || dir > 1) return fail(DF_EINVAL, "bad argument");
    const CompDev &d = h->c[comp];
    const int width = dir ? h->Nz_loc + 2 * d.Nzp : h->Nz_loc;
    const int rows = dir ? h->Ny : h->Ny + 2 * d.Nyp;
    if (n < (long long)width * rows) return fail(DF_EINVAL, "output too small");
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    const double *src = dir ? d.rz[h->cur] : d.ry[h->cur] + (h->ghost ? h->Gl : 0); // ghost: the strip's own columns
    HIP_OR(hipMemcpy2DAsync(out, (size_t)width * 8, src, (size_t)(dir ? d.rz_pitch : h->Pzy) * 8,
                            (size_t)width * 8, rows, hipMemcpyDeviceToHost, h->stream),
           DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return DF_OK;
}

double df_algorithmic_bytes(df_handle *h, int kernel)
{
    // SURVEY 8d byte model: per component 8(|by|+|bz|) + 16n (N_ys, N_zs, by/bz offsets)
    // + 24n (filt_old read + write, fluc write); + 16n for T', rho'. The y-pass gets
    // 8|by| + 8n, the z-pass + epilogue the rest.
    if (!valid(h)) return -1.0;
    const double n = (double)h->Ny * h->Nz_loc;
    double y = 0, z = 0;
    for (int c = 0; c < 3; ++c) {
        y += 8.0 * h->c[c].by_size + 8.0 * n;
        z += 8.0 * h->c[c].bz_size + 8.0 * n + 24.0 * n;
    }
    z += 16.0 * n;
    return kernel == 0 ? y : kernel == 1 ? z : y + z;
}

int df_comm_unique_id(void *out, size_t len)
{
    if (!out || len < sizeof(ncclUniqueId)) return fail(DF_EINVAL, "need 128 bytes for the RCCL unique id");
    ncclUniqueId id;
    NCCL_OR(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof id);
    return DF_OK;
}

int df_comm_info(df_handle *h, df_comm_stats *out)
{
    if (!valid(h) || !out) return fail(DF_EINVAL, "bad argument");
    *out = df_comm_stats{};
    if (h->comm) {
        NCCL_OR(ncclCommCount(h->comm, &out->rccl_ranks));
        NCCL_OR(ncclCommUserRank(h->comm, &out->rccl_rank));
    }
    const bool split = h->world > 1 || h->halo_loopback;
    out->halo_peers = h->ghost ? 0 : h->world > 1 ? (h->rank > 0) + (h->rank < h->world - 1) : (h->halo_loopback ? 2 : 0);
    out->halo_bytes_sent = split ? (long long)out->halo_peers * (long long)h->halo_elems * 8 : 0;
    // 2: the records ride in the halo's ncclGroup (one grouped RCCL operation per call); 1: an all-gather of their own
    // (halo_ghost: no halo, the records travel alone on the RNG stream: 1)
    out->rng_collective = h->split_count && h->rng_comm ? (fused_active(h) && !h->ghost ? 2 : 1) : 0;
    const long long others = (long long)h->rng_chunk * (h->world - 1);
    long long rec = 0, lo = 0, to = 0;
    record_layout(h->rng_chunk, &rec, &lo, &to);
    out->rng_bytes_received = !out->rng_collective ? 0
                              : h->gen_dense == 2 ? rec * (h->world - 1)
                                                  : others * (long long)(sizeof(int) + kWavesPerBlock * sizeof(int));
    out->rng_blocks_counted = h->split_count ? h->rng_chunk : h->rng_blocks;
    out->rng_blocks_total = h->rng_blocks;
    return DF_OK;
}

int df_rms_reset(df_handle *h)
{
    if (!valid_dev(h)) return DF_EINVAL;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    const size_t n = (size_t)h->Ny * h->Nz_loc;
    int rc;
    if (!h->rms_acc && (rc = dalloc_t(h, &h->rms_acc, 5 * n))) return rc;
    if (!h->rms_tmp && (rc = dalloc_t(h, &h->rms_tmp, n))) return rc;
    HIP_OR(hipMemsetAsync(h->rms_acc, 0, 5 * n * sizeof(double), h->stream), DF_EHIP);
    h->rms_count = 0;
    return DF_OK;
}

int df_rms_add(df_handle *h)
{
    if (!valid_dev(h)) return DF_EINVAL;
    int rc;
    if (!h->rms_acc && (rc = df_rms_reset(h))) return rc;
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    HIP_OR(launch_rms_add(sweep_args(h), h->rms_acc, h->stream), DF_EHIP);
    h->rms_count++;
    return DF_OK;
}

int df_rms_get(df_handle *h, int which, double *out)
{
    if (!valid_out(h) || !out || which < DF_U || which > DF_RHO) return fail(DF_EINVAL, "bad argument");
    if (!h->rms_acc || h->rms_count == 0) return fail(DF_EINVAL, "no df_rms_add since df_rms_reset");
    HIP_OR(hipSetDevice(h->device), DF_EHIP);
    const size_t n = (size_t)h->Ny * h->Nz_loc;
    HIP_OR(launch_rms_finish(h->rms_acc + which * n, h->rms_tmp, n, (double)h->rms_count, h->stream), DF_EHIP);
    HIP_OR(hipMemcpyAsync(out, h->rms_tmp, n * sizeof(double), hipMemcpyDeviceToHost, h->stream), DF_EHIP);
    HIP_OR(hipStreamSynchronize(h->stream), DF_EHIP);
    return DF_OK;
}

long long df_rms_count(df_handle *h) { return valid(h) ? h->rms_count : -1; }

int df_get_vertices(df_handle *h, double *y, double *z)
{
    if (!valid(h)) return DF_EINVAL;
    if (y) std::copy(h->setup.y_vert.begin(), h->setup.y_vert.begin() + h->Ny + 1, y);
    if (z) std::copy(h->setup.z_vert.begin(), h->setup.z_vert.end(), z);
    return DF_OK;
}

int df_get_grid(df_handle *h, double *y, double *z)
{
    if (!valid(h)) return DF_EINVAL;
    const Setup &s = h->setup;
    const int W = s.Nz + 1;
    for (int j = 0; j <= s.Ny; ++j)
        for (int k = 0; k < W; ++k) {
            const size_t v = (size_t)j * W + k;
            if (y) y[v] = s.yv.empty() ? s.y_vert[j] : s.yv[v];
            if (z) z[v] = s.zv.empty() ? s.z_vert[k] : s.zv[v];
        }
    return DF_OK;
}

int df_plane_info(df_handle *h, int *plane, int *per_cell)
{
    if (!valid(h)) return DF_EINVAL;
    if (plane) *plane = h->spec.kind;
    if (per_cell) *per_cell = h->setup.per_cell ? 1 : 0;
    return DF_OK;
}

void df_destroy(df_handle *h) { destroy(h); }

} // extern "C"
