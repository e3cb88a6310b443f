/*
 * df_c.h — C ABI of the MI355X-native DIGITAL_FILTER (libdfamd.so).
 *
 * This is the drop-in boundary for connorswitala/digital-filtering's hot path.
 * Each entry point replaces one piece of the reference C++ API
 * (/root/reference/digital-filtering-c++/df/df.hpp); the C++ header df.hpp in
 * this directory rebuilds that API (DFConfig, FilterField, DIGITAL_FILTER) on
 * top of these functions, and INTEGRATION.md shows the Fortran / ctypes
 * bindings a maintainer would add.
 *
 * Plain pointers and sizes only. All functions return 0 (DF_OK) on success and
 * a negative DF_E* code on failure; df_last_error() describes the last failure
 * of the calling thread. A handle owns one GPU stream and is not thread-safe.
 */
#ifndef DF_C_H
#define DF_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DF_ABI_VERSION 1

enum df_status {
    DF_OK = 0,
    DF_EINVAL = -1,   /* bad argument / config                               */
    DF_EIO = -2,      /* input file missing or malformed (reference: cerr + continue, df.cpp:225-228) */
    DF_EHIP = -3,     /* HIP runtime / kernel launch failure, or no GPU       */
    DF_ENOMEM = -4,   /* device allocation failed                             */
    DF_ERNG = -5,     /* device RNG ran short of polar attempts (never expected) */
    DF_ECOMM = -6     /* RCCL failure (multi-GPU z-strips)                    */
};

enum df_plane {
    DF_PLANE_NATIVE = 0,    /* read_grid()'s built-in 560 x 400 grid (df.cpp:71-118) */
    DF_PLANE_SYNTHETIC = 1, /* SURVEY 8d benchmark planes (Ny, Nz, N_min, N_max) */
    DF_PLANE_GRID = 2       /* a real inflow grid: grid_y/grid_z vertices or grid_file */
};
enum df_coeff_mode {
    DF_COEFF_PACKED = 0, /* stream the per-cell coefficient vectors by/bz from HBM (reference data contract) */
    DF_COEFF_TABLE = 1   /* read b(N,i) from a per-N table: same values, no B stream */
};
enum df_field {
    DF_U = 0, DF_V = 1, DF_W = 2, DF_T = 3, DF_RHO = 4,
    DF_FILT_OLD_U = 5, DF_FILT_OLD_V = 6, DF_FILT_OLD_W = 7,
    DF_FILT_U = 8, DF_FILT_V = 9, DF_FILT_W = 10 /* stage API only (after df_filtering_sweeps) */
};
enum df_row {
    DF_ROW_R11 = 0, DF_ROW_R21, DF_ROW_R22, DF_ROW_R33, DF_ROW_US, DF_ROW_TS, DF_ROW_RHOS, DF_ROW_MS, DF_ROW_PS,
    DF_ROW_YC, DF_ROW_YC_D
};

/* Mirrors struct DFConfig (df.hpp:38-49) field for field, then extensions.
 * df_config_default() fills the values the reference constructor hard-codes
 * (df.cpp:7-16) so an untouched config behaves like the reference. */
typedef struct df_config_c {
    double d_i, rho_e, U_e, mu_e;          /* df.hpp:39-42 */
    int vel_file_offset, vel_file_N_values; /* df.hpp:44-45 (unused by the reference too) */
    const char *grid_file;                 /* df.hpp:47: DF_PLANE_GRID without grid_y/grid_z reads this
                                              Tecplot BLOCK file (write_tecplot's layout, df.cpp:712-762) */
    const char *vel_fluc_file;             /* df.hpp:48: RST profile (reference reads ../files/RST.dat, df.cpp:224) */
    /* ---- extensions ---- */
    const char *line_file;                 /* mean profile (reference ../line.dat, df.cpp:16) */
    uint64_t seed;                         /* pcg32 seed (reference: random_device, df.cpp:334) */
    int seed_from_random_device;           /* 1: draw the 32-bit seed from std::random_device like the reference */
    int plane;                             /* enum df_plane */
    int Ny, Nz;                            /* synthetic plane size */
    int N_min, N_max;                      /* synthetic half-width rule */
    int coeff_mode;                        /* enum df_coeff_mode */
    const char *csv_path;                  /* non-NULL: write the reference CSV after every df_filter (df.cpp:466-467) */
    int device;                            /* HIP device ordinal; -1 = host-only handle (setup
                                              queries only, no GPU: used by CPU tests); DF_DEVICE_TRACE
                                              = schedule trace (df_trace) */
    int rank, world;                       /* z-strip partition: this GPU is strip `rank` of `world` */
    const void *comm_id;                   /* 128-byte RCCL unique id, from df_comm_unique_id (world > 1;
                                              world 1 also accepted: exercises the same RCCL calls) */
    int rows_per_wave;                     /* y-pass register blocking (tuning knob, 0 = from the plane's shape) */
    int rng_resume;                        /* 1: start the stream at (rng_state, rng_saved_flag, rng_saved) */
    int rng_saved_flag;                    /*    instead of seeding (checkpoint/resume, and continuing */
    uint64_t rng_state;                    /*    the reference's process-wide stream across instances) */
    double rng_saved;
    /* DF_PLANE_GRID: (Ny+1)*(Nz+1) vertex coordinates, index j*(Nz+1)+k, row 0 at the wall,
     * Ny x Nz cells (the Ny/Nz fields above). Per-cell dy, dz, yc follow df.cpp:104-116 with
     * dz = z[j,k+1] - z[j,k]; half-widths are then per cell (df.cpp:144-195). Copied at create. */
    const double *grid_y, *grid_z;
} df_config_c;

typedef struct df_handle df_handle;

/* df_config_c.device of a schedule-trace handle: no GPU. df_create, df_filter, df_set_rng_state, df_rng_state and
 * df_set_tuning("handoff_batch" | "ypass_ahead") run the host logic of the noise pipeline - generations, hand-off
 * epochs, the y-pass ahead, releases, restarts - and record what each would enqueue instead of calling HIP;
 * df_trace copies the records out (tests/test_schedule.py checks them). */
#define DF_DEVICE_TRACE (-2)
/* Records of a DF_DEVICE_TRACE handle so far, six int64 each {op, stream, a, b, c, d} (df_capi.cpp TraceOp);
 * copies min(cap, n) of them into out (NULL: count only) and returns n, or -1. */
long long df_trace(df_handle *h, long long *out, long long cap);

typedef struct df_profile {
    long long calls;      /* df_filter calls timed since df_set_profiling(h, 1) */
    double rng_ms;        /* summed device time of each phase, milliseconds */
    double ypass_ms;
    double halo_ms;
    double zpass_ms;
    double total_ms;      /* first event to last event of each call, summed */
} df_profile;

/* Reference defaults (df.cpp:7-16) plus: coeff_mode DF_COEFF_TABLE (bit-identical to
 * DF_COEFF_PACKED, no coefficient stream), vel_fluc_file / line_file = the profiles in
 * df_data_dir(). (The Python test/bench mirror dfamd.make_config defaults to DF_COEFF_PACKED,
 * the reference's data contract; its docstring lists what the mode changes besides the bytes.) */
void df_config_default(df_config_c *cfg);
/* The data/ directory next to the loaded libdfamd.so (RST.dat, line.dat). */
const char *df_data_dir(void);

/* DIGITAL_FILTER::DIGITAL_FILTER(DFConfig) (df.hpp:89, df.cpp:4-66): setup plus
 * the constructor's step 0 (noise, sweeps, RST scaling; no correlation, no SRA).
 * Returns NULL on failure. */
df_handle *df_create(const df_config_c *cfg);

/* DIGITAL_FILTER::filter(double dt) (df.hpp:100, df.cpp:449-468): one timestep.
 * Asynchronous on the handle's stream unless csv_path is set. */
int df_filter(df_handle *h, double dt);

/* Several z-strips of one plane held by ONE process (one device each, or several
 * strips on one device): cfgs[r] has rank r, world n and no comm_id. Creation
 * runs step 0 for the whole plane; df_filter_group advances all strips by dt
 * with in-process halo copies instead of RCCL. */
int df_create_group(const df_config_c *cfgs, int n, df_handle **out);
int df_filter_group(df_handle **hs, int n, double dt);

/* The reference's public stage functions (df.hpp:96-101), run on the device. */
int df_generate_white_noise(df_handle *h);          /* df.cpp:332-349 */
int df_filtering_sweeps(df_handle *h, int comp);    /* df.cpp:351-406, writes filt of one component */
int df_correlate_fields(df_handle *h, int comp, double dt); /* df.cpp:408-417 */
int df_apply_RST_scaling(df_handle *h);             /* df.cpp:419-447 */
int df_get_rho_T_fluc(df_handle *h);                /* df.cpp:470-485 */

/* Host copy of a dense [Ny x Nz_local] field (u.fluc etc., df.hpp:24-34). Synchronizes. */
int df_get_field(df_handle *h, int which, double *host_out);
/* Several fields at once (the drop-in's per-call host mirrors): host_out[i] receives field which[i];
 * all copies are queued on the handle's stream and the call synchronizes ONCE. */
int df_get_fields(df_handle *h, int n, const int *which, double *const *host_out);
/* Process-wide registry of the library's live device allocations, every handle's. Each allocation is
 * checked against it: one that overlaps a live range fails (df_create returns NULL, DF_EHIP, the
 * message names both ranges) instead of silently aliasing another handle's buffer. Diagnostic entry:
 * claim (claim = 1) or release (claim = 0) a range by hand; df_alloc_registry_count = live ranges. */
int df_alloc_registry(const void *p, size_t bytes, int claim);
long long df_alloc_registry_count(void);
/* Page-lock caller memory (hipHostRegister) so df_get_field(s) into it run as DMA transfers;
 * df_host_unpin releases it (call before the memory is freed). */
int df_host_pin(void *p, size_t bytes);
int df_host_unpin(void *p);
/* Upload a dense [Ny x Nz_local] host field into which = DF_U..DF_FILT_OLD_W. Synchronizes.
 * Checkpoint/resume: the reference's resumable state is the stream (df_rng_state)
 * plus filt_old of u, v, w (df.cpp:440-442); df_set_rng_state + df_set_field(DF_FILT_OLD_*)
 * on any handle of the same plane makes its next df_filter continue the saved run bit for bit. */
int df_set_field(df_handle *h, int which, const double *host_in);
/* Device pointer of the same dense field (row-major, pitch Nz_local doubles). */
const double *df_device_field(df_handle *h, int which);
/* Ny, global Nz, and the [z0, z1) columns this handle owns. */
int df_dims(df_handle *h, int *Ny, int *Nz, int *z0, int *z1);
/* Per-row profiles (length Ny) and scalars (0 u_tau, 1 tau_w, 2 d_v). */
int df_get_row(df_handle *h, int which, double *out);
double df_get_scalar(df_handle *h, int which);
/* Per-cell half-widths / offsets of one component, reference layout (N_ys, N_zs,
 * by_offsets, bz_offsets, df.hpp:30-31): out has Ny*Nz_local ints. dir 0 = y, 1 = z. */
int df_get_halfwidths(df_handle *h, int comp, int dir, int *out);
int df_get_offsets(df_handle *h, int comp, int dir, int *out);
/* max half-widths (F.Ny_max, F.Nz_max) and the offset-packed coefficient count. */
int df_get_comp_info(df_handle *h, int comp, int *Ny_max, int *Nz_max, long long *by_size, long long *bz_size);
/* Offset-packed coefficients exactly as FilterField::by / bz (df.cpp:151-216). */
int df_get_coeffs(df_handle *h, int comp, int dir, double *out, long long n);

/* The reference's process-wide RNG stream (df.cpp:334-335) as each handle holds it: pcg32 state,
 * normal_distribution cached flag and value. Synchronizes. include/df.hpp hands one state on between
 * the objects of a process through these two calls (DFConfig::shared_stream). */
int df_rng_state(df_handle *h, uint64_t *state, int *saved_flag, double *saved);
int df_set_rng_state(df_handle *h, uint64_t state, int saved_flag, double saved);
/* Noise arrays as the reference holds them after the sweeps (FilterField r_ys /
 * r_zs, df.hpp:26): dir 0 -> r_ys, (Ny + 2*Ny_max) x Nz_local; dir 1 -> r_zs,
 * Ny x (Nz_local + 2*Nz_max) with the z-halo. `n` is the capacity of out. */
int df_get_noise(df_handle *h, int comp, int dir, double *out, long long n);
/* Normals drawn per df_filter (the six r_ys/r_zs arrays, df.cpp:343-348). */
long long df_stream_length(df_handle *h);

/* Statistics path of the reference's get_rms() (df.cpp:566-611): per-cell sums of
 * u'^2, v'^2, w'^2, T'^2, rho'^2 kept on the device. df_rms_add accumulates the
 * current fields (rms_add, df.cpp:571-582); df_rms_get returns
 * sqrt(sum / count) (plot_rms, df.cpp:615-621) for which = DF_U..DF_RHO. */
int df_rms_reset(df_handle *h);
int df_rms_add(df_handle *h);
int df_rms_get(df_handle *h, int which, double *out);
long long df_rms_count(df_handle *h);
/* Grid vertices used by the reference's writers: y per vertex row (Ny+1) and
 * z per vertex column (Nz+1, global); y/z do not vary along the other axis. */
int df_get_vertices(df_handle *h, double *y, double *z);
/* All grid vertices (the reference's y and z vectors, df.hpp:61): (Ny+1)*(Nz+1) each,
 * index j*(Nz+1)+k, global Nz. Exact on every plane kind (on a grid plane y and z vary
 * along both axes; df_get_vertices then returns column 0 of y and row 0 of z). */
int df_get_grid(df_handle *h, double *y, double *z);
/* Plane kind (enum df_plane) and whether any half-width varies along a row. */
int df_plane_info(df_handle *h, int *plane, int *per_cell);

/* Device-side coupling handoff (the CFD inflow hook us3d_user.f90:51-130
 * sets ghost-cell u = U + u'): for i < n, on the handle's stream after df_filter,
 *     dst[dst_cell[i]] = beta * dst[dst_cell[i]] + field[plane_cell[i]]
 * (beta == 0 assigns without reading dst). plane_cell / dst_cell are DEVICE int64
 * arrays or NULL (identity); dst is device memory of dst_len doubles. No host sync:
 * out-of-range indices are skipped and reported by the next df_sync. */
int df_gather_field(df_handle *h, int which, long long n, const long long *plane_cell, double *dst,
                    const long long *dst_cell, long long dst_len, double beta);

/* Launch-shape tuning (extension; results are bit-identical for every setting except "fast_log":
 * 2 (default) = glibc's own log algorithm in the polar transform (normals and fields bit-identical to
 * the reference's), 1 = a table-driven log within 1 ulp of it, 0 = the device math library's log;
 * 1 and 0 keep the normals within 2 ulp of the reference's). Every key is a default on some plane or a
 * documented use; variants measured neutral or slower were removed (rounds 4-5, DESIGN.md sections 8-9).
 * Sweeps:
 *   "rows_per_wave" (1,2,4,8; 0 at create = by plane), "yunroll" (packed per-wave y-pass: 2, 4; 8 = the
 *   8-deep load ring of long chains), "ycoop" (packed y-pass: 7 = a block per row pair, the long-chain
 *   default; 0 = a wave per tile), "ycoop_order" (row-pair dispatch inside each XCD run: 0 ascending,
 *   g >= 1 groups of g tiles heaviest first; 4 on long chains), "ycoop_split" (row-pair tiles whose widest
 *   row has N >= this run as two 64-column halves; 96 on long chains, 0 never), "ycoop_split4" (... as four
 *   32-column quarters; 192 on long chains), "ypass_ahead" (1: each
 *   epoch's y-passes run on a stream of their own as soon as its noise is generated and the call runs only
 *   the halo and z-pass; long-chain planes and RCCL table z-strips; it pays only with the three epochs of noise
 *   sets such handles allocate at create), "ylds" (table y-pass with LDS-staged noise:
 *   2 = a block per (strip, 4 rows), 3 = a block per (64 columns, 4 waves of "yt_rows" rows) walking the
 *   tap window in "yt_chunk"-row chunks through a double-buffered LDS ring, "yt_pd" chunks of noise loads
 *   in flight, heaviest first; 0 = a wave per tile), "yt_rows" x "yt_chunk" (1 x 16 default, 1 x 24: on
 *   the reference's grid the call -2% beside the RNG, the kernel alone +7%; 2 x 8, 2 x 16), "yt_pd" (2; 4 for yt_rows 1: deeper prefetch, more VGPRs), "zsplit" (packed z-pass, a wave
 *   per component: few-tile planes), "zstage" (table z-pass noise staged in LDS: 2 default, 0 the unstaged
 *   form large halos take), "nt_stores" (non-temporal output stores), "ywin_T" / "ywin_W" / "zwin_T" /
 *   "zwin_W" (sweep write windows: packed planes streaming >= 2 GB of coefficients).
 * Noise generation:
 *   "gen_split" (1-16: generation waves per wave of attempts, small planes), "fuse_plan" (the compacted K3
 *   plans its own waves on small planes), "handoff_batch" (1,2,4: generations per cross-stream hand-off;
 *   at most half the noise sets allocated at create), "gen_dense" (0 compacted K3; 2 run generation:
 *   group counts, one wave per piece of needed chunks), "fast_log" (above).
 * Z-strips (RCCL handles; "gen_dense", "fused_exchange" and "rng_replicate" change the collective sequence:
 * set them alike on every rank before the next df_filter):
 *   "rng_replicate" (1 every rank counts every attempt, 0 split counting), "fused_exchange" (split
 *   counting with gen_dense 2: the next generation's share records travel in the call's halo group, one
 *   grouped RCCL operation per call; 0 = an all-gather of their own), "halo_overlap" (1 = send/recv, unpack
 *   and edge-strip z-pass on a high-priority stream under the interior strips' z-pass; 0 = one serial
 *   chain; -1 default = 1 packed, 0 table), "halo_loopback" (one-rank RCCL handle: send the halo to itself
 *   and check it), "halo_ghost" (table mode, row-uniform planes, same on every rank: 1 = each strip
 *   y-filters its neighbours' halo columns itself from the same noise, no halo exchange; the share records'
 *   all-gather runs on the noise stream ahead of the call). */
int df_set_tuning(df_handle *h, const char *key, int value);

/* The launch shape the handle will use for a df_set_tuning key: the plane-dependent defaults chosen at
 * create time (host-only handles included) or the last setting. Every df_set_tuning key but
 * "halo_loopback", and two read-only keys of the noise pipeline: "noise_sets" (sets allocated at create) and
 * "prefetch_epochs" (hand-off epochs generated ahead of the one being consumed); DF_EINVAL for other keys. */
int df_get_tuning(df_handle *h, const char *key, int *value);

/* Timing (hipEvents on the handle's stream). on = 0 off, 1 events on every df_filter, n > 1 on every
 * n-th df_filter only (the first of each n; df_profile.calls counts the timed calls): the events are
 * queue packets between a call's kernels and cost up to 10% of a short call. */
int df_set_profiling(df_handle *h, int on);
int df_get_profile(df_handle *h, df_profile *out);
/* Wait for ALL queued work of the handle: its results AND the noise generation / y-passes already enqueued
 * for later calls (state loads, timing brackets, teardown). */
int df_sync(df_handle *h);
/* Wait for the results of the work enqueued so far - fields, T'/rho', statistics, gathers, the stage API -
 * and nothing else: later calls' noise and y-passes keep running (df.cpp:449-468's filter() returns when
 * its fields are done). The per-step wait of a synchronous caller (DIGITAL_FILTER::filter). Reports the
 * same errors as df_sync. */
int df_wait(df_handle *h);
/* The HIP stream (hipStream_t) every result is written on: a GPU-resident caller orders its own work after
 * df_filter with hipStreamWaitEvent / launches on this stream, no host wait at all. */
void *df_stream(df_handle *h);
/* Bytes of HBM the packed/table hot path must move per df_filter (SURVEY 8d model). */
double df_algorithmic_bytes(df_handle *h, int kernel /* -1 whole call, 0 ypass, 1 zpass */);

int df_comm_unique_id(void *out, size_t len); /* RCCL unique id, len >= 128 */

/* What one df_filter of a z-strip handle exchanges (bench and monitoring).
 * rccl_ranks comes from ncclCommCount on the handle's communicator (0: no RCCL). The collective
 * form follows coeff_mode: DF_COEFF_PACKED replicates the counting, so the halo send/recv is the
 * call's only collective (rng_collective 0); DF_COEFF_TABLE (the df_config_default mode) splits the
 * counting: each rank counts 1/N of the attempt blocks and the ranks exchange share records (per
 * 64-attempt accept counts, the share's block prefix and its total). With the run generation and
 * "fused_exchange" (the defaults) the records of a later generation travel inside the call's halo
 * ncclGroup, so a call issues ONE grouped RCCL operation (rng_collective 2); otherwise they are
 * all-gathered on a second communicator (rng_collective 1). df_set_tuning(h, "rng_replicate", 0 | 1)
 * overrides the counting form (alike on every rank, before the first df_filter). */
typedef struct df_comm_stats {
    int rccl_ranks, rccl_rank;    /* ncclCommCount / ncclCommUserRank; 0, 0 without RCCL */
    int halo_peers;               /* neighbours this strip exchanges z-halo columns with (0-2) */
    int rng_collective;           /* 2: records in the halo group; 1: an RNG all-gather; 0: none */
    long long halo_bytes_sent;    /* per df_filter, all three components */
    long long rng_bytes_received; /* per df_filter, RNG share records (0 when replicated) */
    long long rng_blocks_counted; /* attempt blocks of 4096 this rank tests per call (K1) */
    long long rng_blocks_total;   /* attempt blocks of the whole plane's call */
} df_comm_stats;
int df_comm_info(df_handle *h, df_comm_stats *out);

void df_destroy(df_handle *h);
const char *df_last_error(void);
int df_abi_version(void);
/* sizeof(df_config_c) as compiled into the library (FFI layout check, e.g. the Fortran module). */
size_t df_config_sizeof(void);

#ifdef __cplusplus
}
#endif
#endif /* DF_C_H */
