/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * Plain-C CPU restatement of the DIGITAL_FILTER::filter(dt) hot path of
 * connorswitala/digital-filtering (reference @ /root/reference, read-only) and
 * of the setup that feeds it. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as a checker.
 * The product (libdfamd.so) never links, loads or calls it.
 *
 * Pinning:
 *   - pcg32 core: the reference's own known-answer test
 *     digital-filtering-c++/pcg-cpp/test-high/expected/check-pcg32.out
 *     (two-arg seed (42,54), round 1 outputs + backstep/advance).
 *   - everything else (1-arg seeding, libstdc++ polar normals, setup rows,
 *     half-widths, fields): golden vectors produced by the reference's own
 *     df.cpp compiled unmodified in this container (oracle/ref/, outputs in
 *     oracle/_ref/), committed under tests/golden/ with gen_golden.py.
 *
 * All citations are path:line relative to /root/reference/digital-filtering-c++/.
 */
#ifndef DF_ORACLE_H
#define DF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- pcg32 = setseq_xsh_rr_64_32 (pcg-cpp/include/pcg_random.hpp:1663,1866) ---- */
uint64_t orc_pcg32_seed1(uint64_t seed);                 /* 1-arg ctor, pcg_random.hpp:484-487 */
void     orc_pcg32_seed2(uint64_t seed, uint64_t stream,  /* 2-arg ctor (set_stream), KAT only */
                         uint64_t *state, uint64_t *inc);
uint32_t orc_pcg32_next(uint64_t *state, uint64_t inc);  /* operator(), output_previous = true */
uint64_t orc_pcg32_advance(uint64_t state, uint64_t delta, uint64_t inc); /* pcg_random.hpp:639-662 */
void     orc_pcg32_fill(uint64_t *state, uint64_t inc, uint32_t *out, size_t n);

/* ---- libstdc++ 11 normal_distribution<double> over pcg32 (random.tcc:1800-1835) ---- */
typedef struct {
    uint64_t state;        /* pcg32 state (increment is the default stream) */
    int      saved_flag;   /* _M_saved_available */
    double   saved;        /* _M_saved */
    uint64_t attempts;     /* polar attempts consumed so far (diagnostic) */
    uint64_t accepted;     /* accepted attempts so far (diagnostic) */
} orc_rng;

void   orc_rng_seed(orc_rng *r, uint64_t seed);
double orc_normal(orc_rng *r);
void   orc_normals(orc_rng *r, double *out, size_t n);

/* ---- the DIGITAL_FILTER object ---- */
enum { ORC_PLANE_NATIVE = 0, ORC_PLANE_SYNTHETIC = 1, ORC_PLANE_GRID = 2 };

typedef struct {
    int plane;             /* ORC_PLANE_NATIVE: read_grid() df.cpp:71-118 */
    int Ny, Nz;            /* synthetic plane size */
    int N_min, N_max;      /* synthetic half-width rule */
    const char *rst_file;  /* df.cpp:224 "../files/RST.dat" */
    const char *line_file; /* df.cpp:16  "../line.dat"      */
    /* ORC_PLANE_GRID: the vertices read_grid() would read from grid_file (df.cpp:71-118 with
     * its placeholder replaced): (Ny+1)*(Nz+1) y and z values, index j*(Nz+1)+k. Cell geometry
     * follows df.cpp:104-116; dz is the cell's bottom edge z[j,k+1]-z[j,k] (the reference's
     * placeholder grid has the constant 0.000133 there, df.cpp:108). */
    const double *grid_y, *grid_z;
} orc_cfg;

typedef struct {
    double *by, *bz, *r_ys, *r_zs, *filt_old, *filt, *fluc;
    int *N_ys, *N_zs, *by_offsets, *bz_offsets;
    long long by_size, bz_size, r_ys_size, r_zs_size;
    double Iz_inn, Iz_out, Lt;
    int Nz_max, Ny_max;
} orc_field;

typedef struct {
    int Ny, Nz, n_cells;
    double d_i, d_v, rho_e, U_e, T_e, mu, T_w, gcon, P, rho_w;
    double u_tau, tau_w, dt;
    int N_in;
    double *y, *z;                 /* (Ny+1)*(Nz+1) vertices (CSV writer) */
    double *yc, *yc_d, *dy, *dz;   /* per cell */
    double *ydline, *yline;        /* per row */
    double *R11, *R21, *R22, *R33; /* per row */
    double *Us, *Ts, *Ps, *rhos, *Ms;
    double *T_fluc, *rho_fluc;
    orc_field F[3];                /* u, v, w */
    orc_rng *rng;                  /* borrowed: the reference's stream is a process-wide static */
} orc_df;

/* Constructor semantics (df.cpp:4-66): setup + step 0 (noise, sweeps, RST; no correlate/SRA).
 * Returns NULL on error (message via orc_last_error). */
orc_df *orc_df_create(const orc_cfg *cfg, orc_rng *rng);
void    orc_df_destroy(orc_df *df);
const char *orc_last_error(void);

/* Hot path stages (df.cpp:332-485), callable one by one as in the reference. */
void orc_generate_white_noise(orc_df *df);             /* df.cpp:332-349 */
void orc_filtering_sweeps(orc_df *df, int comp);       /* df.cpp:351-406 */
void orc_correlate_fields(orc_df *df, int comp);       /* df.cpp:408-417 */
void orc_apply_RST_scaling(orc_df *df);                /* df.cpp:419-447 */
void orc_get_rho_T_fluc(orc_df *df);                   /* df.cpp:470-485 */
void orc_filter(orc_df *df, double dt);                /* df.cpp:449-468 (no CSV) */

/* Accessors for ctypes. which: 0..2 = u,v,w fluc; 3 = T'; 4 = rho'. */
const double *orc_field_ptr(const orc_df *df, int which);
int orc_dims(const orc_df *df, int *Ny, int *Nz);
/* row: 0 R11, 1 R21, 2 R22, 3 R33, 4 Us, 5 Ts, 6 rhos, 7 Ms, 8 Ps, 9 yline, 10 ydline */
const double *orc_row_ptr(const orc_df *df, int row);
const orc_field *orc_field_struct(const orc_df *df, int comp);
double orc_scalar(const orc_df *df, int which); /* 0 u_tau, 1 tau_w, 2 d_v */

/* CSV writer restated from df.cpp:764-803 (15-digit fixed). Returns 0 on success. */
int orc_write_csv(const orc_df *df, const char *path);

/* Synthetic half-width rule (mirrors df.cpp:146-148). */
int orc_synthetic_N(int j, int Ny, int N_min, int N_max);

#ifdef __cplusplus
}
#endif
#endif
