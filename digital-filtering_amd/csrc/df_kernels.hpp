// Device-side data contract and kernel launchers for the filter(dt) hot path.
//
// HBM layout (one handle = one GPU = one z-strip [z0, z1) of the plane):
//   ry[c]   noise for the y-pass, (Ny + 2*Nyp_c) rows x Pz columns, Pz = 128*nstrips
//           (reference r_ys, df.cpp:197, row stride padded from Nz to Pz).
//   rz[c]   Ny rows x rz_pitch_c, rz_pitch_c = Pz + 2*Nzp_c; local column Nzp_c + k
//           holds y-filtered cell k (reference r_zs interior, df.cpp:377); columns
//           [0,Nzp_c) and [Nzp_c+Nz_loc, ...) are the z-halo: raw noise at the
//           global plane edges (df.cpp:343-348 quirk) or the neighbour's y-filtered
//           columns when the plane is split over GPUs.
//   By/Bz   filter coefficients in "strip-tap-major" order: for strip s (128 cells
//           of one row) and row j, (2*N_sj+1) taps x 128 cells, cell fastest. The
//           values are the reference's offset-packed by/bz (df.cpp:151-216), moved
//           so that a wave reads tap i of 128 neighbouring cells as one 1 KiB load.
//   filt_old[c], fluc[c], T, rho: dense Ny x Nz_loc, row-major idx = j*Nz_loc + k
//           (reference FilterField::filt_old/fluc, df.hpp:24-34).
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

#include "df_rng.hpp"

namespace dfamd {

constexpr int kStrip = 128;           // cells per strip (one wave, 2 per lane)
constexpr int kMaxNoiseSets = 12;     // noise sets per handle (2 x the hand-off batch; 3 x with the y-pass ahead)
constexpr int kYTailRows = 128;       // r_ys rows allocated past the last noise row: ypass_t64 loads whole chunks
                                      // up to (yt_pd + 1) * yt_chunk <= 96 rows past a block's last row, unclamped
constexpr int kRngThreads = 256;      // threads per RNG block
constexpr int kRngPerThread = 16;     // polar attempts per thread
constexpr int kRngBlockAttempts = kRngThreads * kRngPerThread;
constexpr int kWavesPerBlock = kRngThreads / 64;
static_assert(kRngThreads == 256 && kRngPerThread * 64 == kRngBlockAttempts / 4,
              "RNG mapping: 4 waves per block, each owning a contiguous run of 64 * kRngPerThread attempts");

struct RngStateDev {
    uint64_t state;
    int saved_flag;
    int pad;
    double saved;
};

struct PcgJumpDev {
    uint64_t mult, plus;
};

// One wave of attempts whose normals this GPU stores (K2c -> K3): its first rank and its index
// gw = 4 * block + wave.
struct WaveTask {
    long long r_lo;
    int gw, pad;
};

// K3r destination of a 128-position chunk (host-built, RngGeom::chunk_dest): position i of the chunk, if
// lo <= i < hi, goes to buffer arr + off + i, plus jump once i >= wr (one row wrap: pitch - width); positions
// outside [lo, hi) are drawn but not stored here (other strips' columns, the r_zs interior).
struct ChunkDest {
    long long off;
    int jump;
    uint8_t wr;      // 0..128
    signed char arr; // stream array: even r_ys, odd r_zs of component arr >> 1; -1: general path
    uint8_t lo, hi;  // stored positions [lo, hi) of the chunk's 128
};

// Run generation (gen_dense 2): a wave generates a piece of consecutive needed 64-rank chunks [c0, c0 + n)
// (host list per parity f; li0 = the list index of c0, for chunk_dest).
struct RunPiece {
    uint32_t c0, li0, n, pad;
};

struct RngGeom {
    uint64_t seg[7];        // stream order u.r_ys,u.r_zs,v.r_ys,v.r_zs,w.r_ys,w.r_zs
    uint64_t Q;             // normals drawn per call
    uint64_t next_mult, next_plus; // jump over 64*4 outputs (attempt start to the lane's next one)
    uint64_t next_plus1, next_plus3; // the same jump for the states 1 and 3 steps into an attempt (K1)
    const PcgJumpDev *jump_block;  // [nblocks]: jump over 4*4096*b outputs
    const PcgJumpDev *jump_thread; // [kRngThreads]: jump over 4*(1024*(tid/64) + tid%64) outputs
    int Nz_g, Pz, z0, z1, is_first, is_last;
    int yz0, yz1;                  // r_ys columns stored here: [yz0, yz1) at ry column col - yz0 (pitch Pz); [z0, z1),
                                   // or the strip plus its ghost columns on z-strips that y-filter their own halo
    uint32_t width[6], rows[6];    // row length / row count of each of the six noise arrays
    int debug_flags;               // timing ablations only (wrong results): 1 no log/sqrt, 2 no stores, 4 no redraw,
                                   // 8 no batches (compacted K3: the append loop alone)
    int nt_stores;                 // noise pairs stored non-temporally
    int gen_split;                 // K3 waves per attempt wave (1, 2, 4, 8, 16): each runs kRngPerThread/gen_split
                                   // iterations, so few-wave planes get short serial chains
    int fused_plan;                // compacted K3 plans its own waves (one GPU, nb_plan <= 1024 blocks): no K2/K2c launch
    int nb_plan;                   // attempt blocks of the call (fused_plan)
    int recount;                   // split counting: K3 recomputes its waves' accept flags (masks are not exchanged)
    int fast_log;                  // log in the polar transform: 2 glibc_log (glibc's bits), 1 log_r2 (table-driven,
                                   // within 1 ulp), 0 the device library's log (df_rng.hpp)
    const LogTabEntry *log_tab;    // kLogTab entries (build_log_table)
    uint64_t inv_width[6];         // ceil(2^64 / width): row = umulhi(p, inv) for p < 2^32 (0 if width == 1)
    int Nzp[3], rz_pitch[3];
    double *ry[3], *rz[3];
    int gen_dense;                  // 0: compacted K3; 2: run generation (K2s, K3r)
    // K3r fast chunks: per listed needed chunk of the call's parity f, where its 128 positions land when they all
    // go to one stream array with at most one row wrap; arr < 0 marks a chunk for the general per-lane path.
    const struct ChunkDest *chunk_dest[2];
    // Run generation (gen_dense 2). The attempt blocks are cut into xworld shares of xchunk blocks (the z-strip
    // ranks' counting shares; one share on a single GPU); share s has a record of xstride bytes at xbuf +
    // s * xstride: the accepted attempts of each 64-attempt group of its blocks (uint8, 64 per block; K1), the
    // share-local exclusive prefix of its block counts (int32 at xlp_off; K2s) and its total (int64 at
    // xtot_off; K2s). Under split counting the records are what the ranks exchange. Also the pieces of each
    // parity's chunk list, and jumps to a group inside a block (4 * 64 * gi outputs) and to a lane in a group.
    uint8_t *xbuf;
    long long xstride, xlp_off, xtot_off;
    int xchunk, xworld;
    const RunPiece *pieces[2];
    int npieces[2];
    const PcgJumpDev *jump_gi, *jump_lane;
    long long nb_groups; // groups of the call's attempt blocks (64 per block)
};

struct SweepArgs {
    // y-pass
    const double *ry[3];
    double *rz[3];
    const double *By[3], *Bz[3];
    const long long *byoff[3], *bzoff[3]; // [s*Ny + j] element offsets
    const int *Ny_st[3], *Nz_st[3];       // tap range per (strip, row): [s*Ny + j], max N over the strip's cells
    const int *Ny_cell[3], *Nz_cell[3];   // per-cell N, [j*Nz_loc + k] (grid planes; table mode only)
    int per_cell;                         // N varies within a strip: table mode reads lane N
    int Nyp[3], Nzp[3], rz_pitch[3];
    int Ny, Nz_loc, Pz, nstrips;
    // coefficient table (DF_COEFF_TABLE mode): half-vector of N at tab + tab_off[N]
    const double *tab;
    const int *tab_off;
    // the same as full symmetric vectors (b[|i|], i = -N..N) at tabf + tabf_off[N], 64-B aligned
    const double *tabf;
    const int *tabf_off;
    // y-pass output: column col of the y-pass plane goes to rz column yout[c] + col when ylo[c] <= col < yhi[c]
    // (Nzp, 0, Nz_loc; ghost columns: the strip widened by its neighbours' halo columns, Nzp - Gl, ...)
    int yout[3], ylo[3], yhi[3];
    // z-pass epilogue
    double *filt_old[3], *fluc[3], *filt[3], *T, *rho;
    const double *rowc;     // 7 x Ny: sqrt(R11), b, sqrt(R22-b^2), sqrt(R33), SRA t1, Ts, rhos
    double sa[3], s1a[3];   // sqrt(alpha), sqrt(1-alpha) per component
    int do_corr, do_sra, comps_mask;
    int write_filt;         // stage API: z-pass stores filt[c] only (df.cpp:401)
    int yunroll, zunroll;   // taps per loop iteration: packed y 2, 4, 8 (deep ring); z pairs per step 4
    int nt_stores;          // z-pass outputs stored non-temporally
    int ynt_stores;         // y-pass output (r_zs) stored non-temporally
    int zstage;             // table z-pass: a block's 4 strips of one row read their noise from LDS (2: 16-B copy,
                            // all loads issued before the stores)
    int zsplit;             // packed z-pass: one 3-wave block per tile, a wave per component (few tiles per SIMD)
    int ycoop;              // packed y-pass: 7 = one block per row pair (long chains), 0 = a wave per tile
    int ycoop2_xcd[3][9];   // row-pair y-pass: XCD x runs tiles [ycoop2_xcd[c][x], ycoop2_xcd[c][x+1]) (equal bytes)
    int ycoop2_run;         // the longest such run (grid = 8 x this)
    const int *ycoop2_perm[3]; // dispatch position -> tile inside each run (nullptr: ascending)
    int ylds;                  // table y-pass with the noise staged in LDS per block of 4R rows (ypass_tlds_kernel)
    // ylds 3 (ypass_t64_kernel): blocks of 4 ylist_R rows x 64 columns, launched in the order ylist[0, ylist_n)
    // (tile = (c * ylist_ncol + column tile) * ylist_nrb + row block; heaviest union of noise rows first)
    const int *ylist;
    int ylist_n, ylist_nrb, ylist_ncol, ylist_R, ylist_C, ylist_PD; // R rows per wave, C noise rows per LDS chunk,
                                                                     // PD chunks of noise loads in flight
    int ylist_dbg; // timing only (DFAMD_YT_DEBUG, wrong sums): ypass_t64_kernel's DBG ablations, 0 = none
    // z-pass strip range of one launch: local strip sl in [0, zs_n) is strip zs_lo + sl, plus zs_gap past
    // zs_gap_at (a z-strip plane's edge strips, which read the halo, around the interior ones: the halo
    // exchange runs under the interior launch). Whole plane: 0, nstrips, nstrips, 0.
    int zs_lo, zs_n, zs_gap_at, zs_gap;
    // z-halo of row j, component c: the plane's widest z half-width of that row (Setup Nz_row, the same on every
    // rank) columns, packed row after row at halo_off[c][j] (nullptr: Nzp[c] columns for every row)
    const int *halo_w[3];
    const long long *halo_off[3];
    int zgroup;             // table z-pass: blocks of (row, <= 4 consecutive strips) (launches without a gap)
    int zstage_reg;         // doubles per component region of that LDS segment (512 + 2 * max Nzp)
    // Write windows: a wave holds its output stores until the chip-wide real-time clock (100 MHz) is
    // in the first W ticks of a T-tick period, so the CUs write together and the read stream runs
    // write-free in between (tools/write_probe). T a power of two; T or W = 0: store at once. Per pass.
    int ywin_T, ywin_W, zwin_T, zwin_W;
};

// Launchers (all asynchronous on `st`). Return hipSuccess or the launch error.
// K0: strip-tap-major coefficients of one component and direction; taps beyond a cell's
// own N (N_cell, or N_st when N_cell is null) are zero.
hipError_t launch_expand_coeffs(double *B, const long long *off, const int *N_st, const int *N_cell,
                                const double *tab, const int *tab_off, int Ny, int nstrips, int Nz_loc,
                                hipStream_t st);
// K1 for blocks [b0, b0+nb) of nb_total (a z-strip rank counts its share only).
hipError_t launch_rng_count(const RngGeom &g, const RngStateDev *st_in, int *counts, int *wave_counts,
                            uint16_t *masks, int b0, int nb, int nb_total, hipStream_t st);
// K2s (run generation): share `share`'s block prefix and total into its exchange record (after K1).
hipError_t launch_rng_share_scan(const RngGeom &g, const int *counts, int share, hipStream_t st);
hipError_t launch_rng_finish(const RngGeom &g, const RngStateDev *st_in, RngStateDev *st_out, int *counts,
                             const int *wave_counts, long long *offsets, long long *part, uint16_t *masks,
                             WaveTask *tasks, int *ntasks, int *err, int nb_total, int nb_scan, hipStream_t st);
// DFAMD_SOLO_STRIP stand-in for the split-counting all-gather: rank's record of `bytes` (a multiple of 16)
// copied over every other rank's record of buf (one launch, as one collective would be).
hipError_t launch_replicate_share(uint8_t *buf, size_t bytes, int world, int rank, hipStream_t st);
hipError_t launch_ypass(const SweepArgs &a, bool table, int rows_per_wave, hipStream_t st);
hipError_t launch_zpass(const SweepArgs &a, bool table, hipStream_t st);
// Stage API elementwise kernels: op 0 correlate_fields(comp) (df.cpp:408-417),
// op 1 apply_RST_scaling (419-447), op 2 get_rho_T_fluc (470-485).
hipError_t launch_stage(const SweepArgs &a, int op, int comp, hipStream_t st);
// rms_add (df.cpp:571-582): acc[f][idx] += x_f^2 for u', v', w', T', rho'.
hipError_t launch_rms_add(const SweepArgs &a, double *acc, hipStream_t st);
// plot_rms (df.cpp:615-621): out = sqrt(acc / count)
hipError_t launch_rms_finish(const double *acc, double *out, size_t n, double count, hipStream_t st);
hipError_t launch_gather(const double *src, long long nsrc, long long n, const long long *pidx, double *dst,
                         const long long *didx, long long ndst, double beta, int *bad, hipStream_t st);
hipError_t launch_halo_pack(const SweepArgs &a, double *send_l, double *send_r, hipStream_t st);
hipError_t launch_halo_unpack(const SweepArgs &a, const double *recv_l, const double *recv_r, hipStream_t st);
hipError_t launch_hold(double us, hipStream_t st); // timing only: a stand-in exchange of us microseconds
hipError_t launch_halo_check(const double *sent, const double *got, size_t n, int corrupt, int *bad, hipStream_t st);

} // namespace dfamd
