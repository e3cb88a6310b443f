/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see df_oracle.h). Never part of the product.
 *
 * Plain-C restatement of connorswitala/digital-filtering's DIGITAL_FILTER
 * (digital-filtering-c++/df/df.cpp, df.hpp) plus the third-party arithmetic it
 * runs through: vendored pcg-cpp's pcg32 and GCC 11.4 libstdc++'s
 * normal_distribution<double> / generate_canonical<double,53>
 * (/usr/include/c++/11/bits/random.tcc:1800-1835, 3346-3378).
 *
 * Floating-point: every expression keeps the reference's evaluation order and is
 * compiled with -ffp-contract=off (x86-64 -O2 without -march, like the reference
 * Makefile, emits no FMA either), so this file reproduces the reference bit for
 * bit on the same libm.
 */
#define _GNU_SOURCE
#include "df_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PCG_MULT 6364136223846793005ULL /* pcg_random.hpp:158 */
#define PCG_INC  1442695040888963407ULL /* pcg_random.hpp:159 */

static char g_err[512];
const char *orc_last_error(void) { return g_err; }
static void set_err(const char *m, const char *a) { snprintf(g_err, sizeof g_err, "%s%s", m, a ? a : ""); }

/* ------------------------------------------------------------------ pcg32 */

static inline uint32_t pcg_output(uint64_t s)
{
    /* xsh_rr_mixin<uint32_t,uint64_t>::output (pcg_random.hpp:845-872):
     * opbits=5, xshift=18, bottomspare=27, rot from the top 5 bits. */
    uint32_t rot = (uint32_t)(s >> 59);
    s ^= s >> 18;
    uint32_t x = (uint32_t)(s >> 27);
    return (x >> rot) | (x << ((32u - rot) & 31u));
}

uint64_t orc_pcg32_seed1(uint64_t seed)
{
    /* engine(itype state): state_ = bump(state + increment()) (pcg_random.hpp:484-487) */
    return (seed + PCG_INC) * PCG_MULT + PCG_INC;
}

void orc_pcg32_seed2(uint64_t seed, uint64_t stream, uint64_t *state, uint64_t *inc)
{
    /* specific_stream: inc = (stream << 1) | 1; state_ = bump(state + inc) */
    *inc = (stream << 1) | 1u;
    *state = (seed + *inc) * PCG_MULT + *inc;
}

uint32_t orc_pcg32_next(uint64_t *state, uint64_t inc)
{
    /* output_previous == true for 64-bit state: output(old); state = bump(old)
     * (pcg_random.hpp:413-437) */
    uint64_t old = *state;
    *state = old * PCG_MULT + inc;
    return pcg_output(old);
}

uint64_t orc_pcg32_advance(uint64_t state, uint64_t delta, uint64_t inc)
{
    /* Brown's arbitrary-stride LCG jump (pcg_random.hpp:639-662). */
    uint64_t cur_mult = PCG_MULT, cur_plus = inc;
    uint64_t acc_mult = 1, acc_plus = 0;
    while (delta > 0) {
        if (delta & 1u) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta >>= 1;
    }
    return acc_mult * state + acc_plus;
}

void orc_pcg32_fill(uint64_t *state, uint64_t inc, uint32_t *out, size_t n)
{
    for (size_t i = 0; i < n; ++i) out[i] = orc_pcg32_next(state, inc);
}

/* -------------------------------------------------- libstdc++ polar normal */

static inline double canonical53(uint64_t *state)
{
    /* generate_canonical<double,53>(pcg32) (random.tcc:3346-3378): m = 2 draws,
     * sum = 0 + lo*1; sum += hi*2^32; ret = sum / 2^64; clamp ret>=1. */
    double sum = 0.0;
    sum += (double)orc_pcg32_next(state, PCG_INC) * 1.0;
    sum += (double)orc_pcg32_next(state, PCG_INC) * 4294967296.0;
    double ret = sum / 18446744073709551616.0;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

void orc_rng_seed(orc_rng *r, uint64_t seed)
{
    r->state = orc_pcg32_seed1(seed);
    r->saved_flag = 0;
    r->saved = 0.0;
    r->attempts = 0;
    r->accepted = 0;
}

double orc_normal(orc_rng *r)
{
    /* normal_distribution<double>::operator() — Marsaglia polar with a cached
     * second value (random.tcc:1800-1835). */
    double ret;
    if (r->saved_flag) {
        r->saved_flag = 0;
        ret = r->saved;
    } else {
        double x, y, r2;
        do {
            x = 2.0 * canonical53(&r->state) - 1.0;
            y = 2.0 * canonical53(&r->state) - 1.0;
            r2 = x * x + y * y;
            r->attempts++;
        } while (r2 > 1.0 || r2 == 0.0);
        r->accepted++;
        const double mult = sqrt(-2 * log(r2) / r2);
        r->saved = x * mult;
        r->saved_flag = 1;
        ret = y * mult;
    }
    /* ret * stddev() + mean() with (0, 1): maps -0.0 to +0.0 */
    return ret * 1.0 + 0.0;
}

void orc_normals(orc_rng *r, double *out, size_t n)
{
    for (size_t i = 0; i < n; ++i) out[i] = orc_normal(r);
}

/* ------------------------------------------------------------ file input */

/* Parse every whitespace-separated double in a line (istringstream >> double). */
static int parse_doubles(const char *line, double *vals, int maxv)
{
    int n = 0;
    const char *p = line;
    while (*p) {
        while (*p && isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        char *end;
        double v = strtod(p, &end);
        if (end == p) break; /* istream extraction stops at the first failure */
        if (n < maxv) vals[n] = v;
        ++n;
        p = end;
    }
    return n;
}

typedef struct { char **lines; int n; } lines_t;

static int read_lines(const char *path, lines_t *L)
{
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    L->lines = NULL; L->n = 0;
    int cap = 0;
    char *buf = NULL; size_t bcap = 0; ssize_t len;
    while ((len = getline(&buf, &bcap, f)) >= 0) {
        if (len > 0 && buf[len - 1] == '\n') buf[--len] = 0; /* std::getline drops '\n' only */
        if (L->n == cap) { cap = cap ? 2 * cap : 512; L->lines = realloc(L->lines, cap * sizeof(char *)); }
        L->lines[L->n++] = strdup(buf);
    }
    free(buf);
    fclose(f);
    return 0;
}

static void free_lines(lines_t *L)
{
    for (int i = 0; i < L->n; ++i) free(L->lines[i]);
    free(L->lines);
}

/* df.cpp:805-848 */
static void linear_interpolate(const double *yd, const double *fd, int nd,
                               const double *yn, double *fn, int nn)
{
    for (int j = 0; j < nn; ++j) {
        double y = yn[j];
        if (y <= yd[0]) { fn[j] = fd[0]; continue; }
        if (y >= yd[nd - 1]) { fn[j] = fd[nd - 1]; continue; }
        int i = 0;
        while (i + 1 < nd && y > yd[i + 1]) ++i;
        double x0 = yd[i], x1 = yd[i + 1], f0 = fd[i], f1 = fd[i + 1];
        fn[j] = f0 + (f1 - f0) * ((y - x0) / (x1 - x0));
    }
}

#define DALLOC(n) ((double *)calloc((size_t)(n) > 0 ? (size_t)(n) : 1, sizeof(double)))
#define IALLOC(n) ((int *)calloc((size_t)(n) > 0 ? (size_t)(n) : 1, sizeof(int)))

/* -------------------------------------------------------------- grids */

static void read_grid_native(orc_df *df)
{
    /* df.cpp:71-118 */
    int Nz = 400, Ny = 560;
    df->Nz = Nz; df->Ny = Ny; df->n_cells = Nz * Ny;
    df->y = DALLOC((Ny + 1) * (Nz + 1));
    df->z = DALLOC((Ny + 1) * (Nz + 1));
    df->yc = DALLOC(df->n_cells); df->yc_d = DALLOC(df->n_cells);
    df->dy = DALLOC(df->n_cells); df->dz = DALLOC(df->n_cells);
    df->ydline = DALLOC(Ny); df->yline = DALLOC(Ny);

    double y_max = 3 * df->d_i, eta, a = 2.0;
    for (int j = Ny; j >= 0; --j)
        for (int k = 0; k < Nz + 1; ++k) {
            eta = ((j) * y_max / (Ny + 1)) / y_max;
            df->y[abs(j - Ny) * (Nz + 1) + k] = y_max * (1 - tanh(a * eta) / tanh(a));
            df->z[j * (Nz + 1) + k] = k * 0.000133;
        }
    for (int j = 0; j < Ny; ++j) {
        for (int k = 0; k < Nz; ++k) {
            int idx = j * Nz + k;
            df->dy[idx] = df->y[(j + 1) * (Nz + 1) + k] - df->y[j * (Nz + 1) + k];
            df->dz[idx] = 0.000133;
            df->yc[idx] = 0.25 * (df->y[j * (Nz + 1) + k] + df->y[(j + 1) * (Nz + 1) + k]
                                  + df->y[j * (Nz + 1) + k + 1] + df->y[(j + 1) * (Nz + 1) + k + 1]);
            df->yc_d[idx] = df->yc[idx] / df->d_i;
        }
        df->ydline[j] = df->yc_d[j * Nz];
        df->yline[j] = df->yc[j * Nz];
    }
}

static void read_grid_synthetic(orc_df *df, int Ny, int Nz)
{
    /* SURVEY §8d synthetic plane: uniform wall-normal spacing 2.4*d_i/Ny, dz = 1.33e-4;
     * cell centres through the same 4-vertex average as df.cpp:109-112. */
    df->Nz = Nz; df->Ny = Ny; df->n_cells = Nz * Ny;
    df->y = DALLOC((Ny + 1) * (Nz + 1));
    df->z = DALLOC((Ny + 1) * (Nz + 1));
    df->yc = DALLOC(df->n_cells); df->yc_d = DALLOC(df->n_cells);
    df->dy = DALLOC(df->n_cells); df->dz = DALLOC(df->n_cells);
    df->ydline = DALLOC(Ny); df->yline = DALLOC(Ny);
    double hy = 2.4 * df->d_i / Ny;
    for (int j = 0; j <= Ny; ++j)
        for (int k = 0; k < Nz + 1; ++k) {
            df->y[j * (Nz + 1) + k] = j * hy;
            df->z[j * (Nz + 1) + k] = k * 0.000133;
        }
    for (int j = 0; j < Ny; ++j) {
        for (int k = 0; k < Nz; ++k) {
            int idx = j * Nz + k;
            df->dy[idx] = df->y[(j + 1) * (Nz + 1) + k] - df->y[j * (Nz + 1) + k];
            df->dz[idx] = 0.000133;
            df->yc[idx] = 0.25 * (df->y[j * (Nz + 1) + k] + df->y[(j + 1) * (Nz + 1) + k]
                                  + df->y[j * (Nz + 1) + k + 1] + df->y[(j + 1) * (Nz + 1) + k + 1]);
            df->yc_d[idx] = df->yc[idx] / df->d_i;
        }
        df->ydline[j] = df->yc_d[j * Nz];
        df->yline[j] = df->yc[j * Nz];
    }
}

static void read_grid_vertices(orc_df *df, int Ny, int Nz, const double *gy, const double *gz)
{
    /* read_grid() (df.cpp:71-118) on caller vertices instead of its placeholder grid */
    df->Nz = Nz; df->Ny = Ny; df->n_cells = Nz * Ny;
    size_t nv = (size_t)(Ny + 1) * (Nz + 1);
    df->y = DALLOC(nv);
    df->z = DALLOC(nv);
    memcpy(df->y, gy, nv * sizeof(double));
    memcpy(df->z, gz, nv * sizeof(double));
    df->yc = DALLOC(df->n_cells); df->yc_d = DALLOC(df->n_cells);
    df->dy = DALLOC(df->n_cells); df->dz = DALLOC(df->n_cells);
    df->ydline = DALLOC(Ny); df->yline = DALLOC(Ny);
    for (int j = 0; j < Ny; ++j) {
        for (int k = 0; k < Nz; ++k) {
            int idx = j * Nz + k;
            df->dy[idx] = df->y[(j + 1) * (Nz + 1) + k] - df->y[j * (Nz + 1) + k];
            df->dz[idx] = df->z[j * (Nz + 1) + k + 1] - df->z[j * (Nz + 1) + k];
            df->yc[idx] = 0.25 * (df->y[j * (Nz + 1) + k] + df->y[(j + 1) * (Nz + 1) + k]
                                  + df->y[j * (Nz + 1) + k + 1] + df->y[(j + 1) * (Nz + 1) + k + 1]);
            df->yc_d[idx] = df->yc[idx] / df->d_i;
        }
        df->ydline[j] = df->yc_d[j * Nz];
        df->yline[j] = df->yc[j * Nz];
    }
}

/* ------------------------------------------------------ RST + line file */

static int read_line_file(orc_df *df, const char *path)
{
    /* df.cpp:487-553 */
    lines_t L;
    if (read_lines(path, &L) != 0) { set_err("cannot open line file: ", path); return -1; }
    if (L.n < 2) { free_lines(&L); set_err("line file too short: ", path); return -1; }
    int N_line = 0;
    const char *pos = strstr(L.lines[1], "i=");
    if (pos) N_line = (int)strtol(pos + 2, NULL, 10);
    if (N_line < 2) { free_lines(&L); set_err("bad i= count in ", path); return -1; }
    double *u_f = DALLOC(N_line), *p_f = DALLOC(N_line), *rho_f = DALLOC(N_line),
           *T_f = DALLOC(N_line), *y_f = DALLOC(N_line);
    int count = 0;
    double v[32];
    for (int li = 2; li < L.n; ++li) {
        if (L.lines[li][0] == 0) continue;
        int nv = parse_doubles(L.lines[li], v, 32);
        if (count < N_line) {
            if (nv < 10) { set_err("short row in ", path); free_lines(&L); return -1; }
            y_f[count] = v[1]; rho_f[count] = v[4]; u_f[count] = v[5];
            T_f[count] = v[8]; p_f[count] = v[9];
        }
        count++;
    }
    free_lines(&L);
    int Ny = df->Ny;
    df->Us = DALLOC(Ny); df->Ts = DALLOC(Ny); df->Ps = DALLOC(Ny);
    df->rhos = DALLOC(Ny); df->Ms = DALLOC(Ny);
    linear_interpolate(y_f, u_f, N_line, df->yline, df->Us, Ny);
    linear_interpolate(y_f, p_f, N_line, df->yline, df->Ps, Ny);
    linear_interpolate(y_f, T_f, N_line, df->yline, df->Ts, Ny);
    linear_interpolate(y_f, rho_f, N_line, df->yline, df->rhos, Ny);
    for (int j = 0; j < Ny; ++j) df->Ms[j] = df->Us[j] / sqrt(1.4 * df->gcon * df->Ts[j]);
    double dyl = y_f[1] - y_f[0];
    double du = df->Us[1] - df->Us[0];
    df->tau_w = df->mu * du / dyl;
    df->u_tau = sqrt(df->tau_w / df->rhos[0]);
    free(u_f); free(p_f); free(rho_f); free(T_f); free(y_f);
    return 0;
}

static int get_RST_in(orc_df *df, const char *rst_path, const char *line_path)
{
    /* df.cpp:220-330 */
    lines_t L;
    if (read_lines(rst_path, &L) != 0) { set_err("cannot open RST file: ", rst_path); return -1; }
    if (L.n < 2) { free_lines(&L); set_err("RST file too short: ", rst_path); return -1; }
    double N_in_d = 0;
    const char *pos = strstr(L.lines[1], "i=");
    if (pos) N_in_d = strtod(pos + 2, NULL);
    int N_in = (int)N_in_d;
    if (N_in < 2) { free_lines(&L); set_err("bad i= count in ", rst_path); return -1; }
    df->N_in = N_in;
    double *y_in = DALLOC(N_in), *yin_d = DALLOC(N_in);
    double *urms = DALLOC(N_in), *vrms = DALLOC(N_in), *wrms = DALLOC(N_in), *uvrms = DALLOC(N_in);
    int count = 0;
    double v[32];
    for (int li = 2; li < L.n; ++li) {
        if (L.lines[li][0] == 0) continue;
        int nv = parse_doubles(L.lines[li], v, 32);
        if (count < N_in) {
            if (nv < 6) { set_err("short row in ", rst_path); free_lines(&L); return -1; }
            y_in[count] = v[0]; yin_d[count] = v[1]; urms[count] = v[2];
            vrms[count] = v[3]; wrms[count] = v[4]; uvrms[count] = v[5];
        }
        count++;
    }
    free_lines(&L);

    /* Truncate Ny to rows with yc/d_i <= last RST y/delta (df.cpp:282-288). */
    int new_Ny = 0, j = 0;
    while (j < df->Ny && df->yc_d[j * df->Nz] <= yin_d[N_in - 1]) { new_Ny++; j++; }
    df->Ny = new_Ny;
    df->n_cells = df->Ny * df->Nz;
    /* The resize calls of df.cpp:298-304 keep the leading rows (row-major). */

    if (read_line_file(df, line_path) != 0) return -1;

    int Ny = df->Ny;
    double *R11_in = DALLOC(N_in), *R21_in = DALLOC(N_in), *R22_in = DALLOC(N_in), *R33_in = DALLOC(N_in);
    double ut = df->u_tau;
    for (int i = 0; i < N_in; ++i) {
        R11_in[i] = urms[i] * urms[i] * ut * ut;
        R22_in[i] = vrms[i] * vrms[i] * ut * ut;
        R33_in[i] = wrms[i] * wrms[i] * ut * ut;
        R21_in[i] = uvrms[i] * ut * ut;
    }
    df->R11 = DALLOC(Ny); df->R21 = DALLOC(Ny); df->R22 = DALLOC(Ny); df->R33 = DALLOC(Ny);
    linear_interpolate(yin_d, R11_in, N_in, df->ydline, df->R11, Ny);
    linear_interpolate(yin_d, R22_in, N_in, df->ydline, df->R22, Ny);
    linear_interpolate(yin_d, R21_in, N_in, df->ydline, df->R21, Ny);
    linear_interpolate(yin_d, R33_in, N_in, df->ydline, df->R33, Ny);
    df->d_v = df->d_i / 4500;
    free(y_in); free(yin_d); free(urms); free(vrms); free(wrms); free(uvrms);
    free(R11_in); free(R21_in); free(R22_in); free(R33_in);
    return 0;
}

/* ------------------------------------------------- filter properties */

int orc_synthetic_N(int j, int Ny, int N_min, int N_max)
{
    double x = (Ny > 1) ? (double)j / (double)(Ny - 1) : 0.0;
    double h = N_min + (N_max - N_min) * 0.5 * (1.0 + tanh((x - 0.2) / 0.03));
    int N = 2 * (int)floor(h / 2.0);
    return N < 2 ? 2 : N;
}

/* Coefficients of one cell, df.cpp:166-177 / 206-216. */
static void cell_coeffs(int N, double *temp, double *dst /* points at centre */)
{
    const double pi_c = -2.0 * 3.14159265358979323846; /* df.hpp:16 */
    double sum = 0.0;
    for (int i = 0; i <= N; ++i) {
        temp[i] = exp(pi_c * abs(i) / N);
        sum += (i == 0 ? 1.0 : 2.0) * temp[i] * temp[i];
    }
    sum = sqrt(sum);
    for (int i = -N; i <= N; ++i) dst[i] = temp[abs(i)] / sum;
}

static void calculate_filter_properties(orc_df *df, orc_field *F, const orc_cfg *cfg)
{
    /* df.cpp:130-218 */
    int n = df->n_cells, Ny = df->Ny, Nz = df->Nz;
    double *Iz = DALLOC(n);
    long long b_size = 0;
    F->Nz_max = 0; F->Ny_max = 0;
    for (int idx = 0; idx < n; ++idx) {
        int n_val;
        if (cfg->plane != ORC_PLANE_SYNTHETIC) {
            Iz[idx] = F->Iz_inn + (F->Iz_out - F->Iz_inn) * 0.5 * (1 + tanh((df->yc[idx] / df->d_i - 0.2) / 0.03));
            double n_int = fmax(1.0, Iz[idx] / df->dz[idx]);
            n_val = 2 * (int)n_int;
        } else {
            n_val = orc_synthetic_N(idx / Nz, Ny, cfg->N_min, cfg->N_max);
        }
        F->N_zs[idx] = n_val;
        b_size += 2 * n_val + 1;
        F->bz_offsets[idx] = (int)(b_size - n_val - 1);
        if (n_val > F->Nz_max) F->Nz_max = n_val;
    }
    F->r_zs_size = (long long)(Nz + 2 * F->Nz_max) * Ny;
    F->r_zs = DALLOC(F->r_zs_size);
    F->bz_size = b_size;
    F->bz = DALLOC(b_size);
    double *temp = DALLOC(F->Nz_max + 1);
    for (int idx = 0; idx < n; ++idx) cell_coeffs(F->N_zs[idx], temp, F->bz + F->bz_offsets[idx]);
    free(temp);

    b_size = 0;
    for (int idx = 0; idx < n; ++idx) {
        int n_val;
        if (cfg->plane != ORC_PLANE_SYNTHETIC) {
            double Iy = 0.67 * Iz[idx];
            double n_int = fmax(1.0, Iy / df->dy[idx]);
            n_val = 2 * (int)n_int;
        } else {
            n_val = orc_synthetic_N(idx / Nz, Ny, cfg->N_min, cfg->N_max);
        }
        b_size += 2 * n_val + 1;
        F->by_offsets[idx] = (int)(b_size - n_val - 1);
        F->N_ys[idx] = n_val;
        if (n_val > F->Ny_max) F->Ny_max = n_val;
    }
    F->r_ys_size = (long long)Nz * (2 * F->Ny_max + Ny);
    F->r_ys = DALLOC(F->r_ys_size);
    F->by_size = b_size;
    F->by = DALLOC(b_size);
    temp = DALLOC(F->Ny_max + 1);
    for (int idx = 0; idx < n; ++idx) cell_coeffs(F->N_ys[idx], temp, F->by + F->by_offsets[idx]);
    free(temp);
    free(Iz);
}

/* ------------------------------------------------------------ hot path */

void orc_generate_white_noise(orc_df *df)
{
    /* df.cpp:332-349: u.r_ys, u.r_zs, v.r_ys, v.r_zs, w.r_ys, w.r_zs in that order */
    for (int c = 0; c < 3; ++c) {
        orc_normals(df->rng, df->F[c].r_ys, (size_t)df->F[c].r_ys_size);
        orc_normals(df->rng, df->F[c].r_zs, (size_t)df->F[c].r_zs_size);
    }
}

void orc_filtering_sweeps(orc_df *df, int comp)
{
    /* df.cpp:351-406 */
    orc_field *F = &df->F[comp];
    int Ny = df->Ny, Nz = df->Nz;
    int Nz_pad = F->Nz_max, Ny_pad = F->Ny_max;
    /* rows are independent and every cell keeps the reference's tap order, so the OpenMP build
       (liboracle_omp.so, bench.py's parallel CPU figure) returns the same bits */
#pragma omp parallel for schedule(dynamic, 8)
    for (int j = 0; j < Ny; ++j) {
        long long r_idy = (long long)(j + Ny_pad) * Nz;
        long long r_idz = (long long)j * (Nz + 2 * Nz_pad) + Nz_pad;
        int idx = j * Nz;
        for (int k = 0; k < Nz; ++k) {
            long long off = F->by_offsets[idx];
            int N = F->N_ys[idx];
            double sum = 0.0;
            for (int i = -N; i <= N; ++i) sum += F->by[off + i] * F->r_ys[r_idy + (long long)i * Nz];
            F->r_zs[r_idz] = sum;
            r_idy++; r_idz++; idx++;
        }
    }
#pragma omp parallel for schedule(dynamic, 8)
    for (int j = 0; j < Ny; ++j) {
        long long r_idz = (long long)j * (Nz + 2 * Nz_pad) + Nz_pad;
        int idx = j * Nz;
        for (int k = 0; k < Nz; ++k) {
            long long off = F->bz_offsets[idx];
            int N = F->N_zs[idx];
            double sum = 0.0;
            for (int i = -N; i <= N; ++i) sum += F->bz[off + i] * F->r_zs[r_idz + i];
            F->filt[idx] = sum;
            r_idz++; idx++;
        }
    }
}

void orc_correlate_fields(orc_df *df, int comp)
{
    /* df.cpp:408-417 (pi = 3.141592654 as written) */
    orc_field *F = &df->F[comp];
    double pi = 3.141592654;
    double alpha = exp(-pi * df->dt / F->Lt);
#pragma omp parallel for
    for (int idx = 0; idx < df->n_cells; ++idx)
        F->filt[idx] = F->filt_old[idx] * sqrt(alpha) + F->filt[idx] * sqrt(1.0 - alpha);
}

void orc_apply_RST_scaling(orc_df *df)
{
    /* df.cpp:419-447 */
    orc_field *u = &df->F[0], *v = &df->F[1], *w = &df->F[2];
#pragma omp parallel for
    for (int j = 0; j < df->Ny; ++j) {
        double b;
        if (df->R11[j] < 1e-10) b = 0.0;
        else b = df->R21[j] / sqrt(df->R11[j]);
        int idx = j * df->Nz;
        for (int k = 0; k < df->Nz; ++k) {
            u->fluc[idx] = sqrt(df->R11[j]) * u->filt[idx];
            v->fluc[idx] = b * u->filt[idx] + sqrt(df->R22[j] - b * b) * v->filt[idx];
            w->fluc[idx] = sqrt(df->R33[j]) * w->filt[idx];
            for (int c = 0; c < 3; ++c) df->F[c].filt_old[idx] = df->F[c].filt[idx];
            idx++;
        }
    }
}

void orc_get_rho_T_fluc(orc_df *df)
{
    /* df.cpp:470-485 */
#pragma omp parallel for
    for (int j = 0; j < df->Ny; ++j) {
        double temp1 = -0.5 * (1.4 - 1) * df->Ms[j] * df->Ms[j] / df->Us[j];
        for (int k = 0; k < df->Nz; ++k) {
            double temp2 = temp1 * df->F[0].fluc[j * df->Nz + k];
            df->T_fluc[j * df->Nz + k] = temp2 * df->Ts[j];
            df->rho_fluc[j * df->Nz + k] = -temp2 * df->rhos[j];
        }
    }
}

void orc_filter(orc_df *df, double dt)
{
    /* df.cpp:449-468 minus the stdout timer and the CSV side effect */
    df->dt = dt;
    orc_generate_white_noise(df);
    for (int c = 0; c < 3; ++c) {
        orc_filtering_sweeps(df, c);
        orc_correlate_fields(df, c);
    }
    orc_apply_RST_scaling(df);
    orc_get_rho_T_fluc(df);
}

/* ------------------------------------------------------- construction */

orc_df *orc_df_create(const orc_cfg *cfg, orc_rng *rng)
{
    orc_df *df = (orc_df *)calloc(1, sizeof(orc_df));
    /* Flow constants hard-coded in the ctor (df.cpp:7-16). */
    df->d_i = 0.0013; df->rho_e = 0.044; df->U_e = 869.1; df->mu = 7.1212e-6;
    df->T_w = 97.5; df->gcon = 287.0; df->T_e = 55.2;
    df->P = df->rho_e * 287.0 * df->T_e; df->rho_w = 0.0249;
    df->rng = rng;

    if (cfg->plane == ORC_PLANE_NATIVE) read_grid_native(df);
    else if (cfg->plane == ORC_PLANE_GRID) {
        if (cfg->Ny < 2 || cfg->Nz < 1 || !cfg->grid_y || !cfg->grid_z) {
            set_err("bad grid plane spec", NULL); free(df); return NULL;
        }
        read_grid_vertices(df, cfg->Ny, cfg->Nz, cfg->grid_y, cfg->grid_z);
    } else {
        if (cfg->Ny < 2 || cfg->Nz < 1 || cfg->N_min < 2 || cfg->N_max < cfg->N_min) {
            set_err("bad synthetic plane spec", NULL); free(df); return NULL;
        }
        read_grid_synthetic(df, cfg->Ny, cfg->Nz);
    }
    if (get_RST_in(df, cfg->rst_file, cfg->line_file) != 0) { orc_df_destroy(df); return NULL; }

    int n = df->n_cells;
    for (int c = 0; c < 3; ++c) { /* allocate_data_structures, df.cpp:120-128 */
        orc_field *F = &df->F[c];
        F->N_ys = IALLOC(n); F->N_zs = IALLOC(n);
        F->fluc = DALLOC(n); F->filt = DALLOC(n); F->filt_old = DALLOC(n);
        F->by_offsets = IALLOC(n); F->bz_offsets = IALLOC(n);
    }
    /* Integral length scales, df.cpp:35-45 */
    df->F[0].Iz_out = 0.4 * df->d_i; df->F[0].Iz_inn = 150 * df->d_v; df->F[0].Lt = 0.8 * df->d_i / df->U_e;
    df->F[1].Iz_out = 0.3 * df->d_i; df->F[1].Iz_inn = 75 * df->d_v;  df->F[1].Lt = 0.3 * df->d_i / df->U_e;
    df->F[2].Iz_out = 0.4 * df->d_i; df->F[2].Iz_inn = 150 * df->d_v; df->F[2].Lt = 0.3 * df->d_i / df->U_e;
    df->rho_fluc = DALLOC(n);
    df->T_fluc = DALLOC(n);
    for (int c = 0; c < 3; ++c) calculate_filter_properties(df, &df->F[c], cfg);

    /* Step 0 (df.cpp:57-62): noise, sweeps, RST — no correlation, no SRA. */
    orc_generate_white_noise(df);
    for (int c = 0; c < 3; ++c) orc_filtering_sweeps(df, c);
    orc_apply_RST_scaling(df);
    return df;
}

void orc_df_destroy(orc_df *df)
{
    if (!df) return;
    for (int c = 0; c < 3; ++c) {
        orc_field *F = &df->F[c];
        free(F->by); free(F->bz); free(F->r_ys); free(F->r_zs);
        free(F->filt_old); free(F->filt); free(F->fluc);
        free(F->N_ys); free(F->N_zs); free(F->by_offsets); free(F->bz_offsets);
    }
    free(df->y); free(df->z); free(df->yc); free(df->yc_d); free(df->dy); free(df->dz);
    free(df->ydline); free(df->yline);
    free(df->R11); free(df->R21); free(df->R22); free(df->R33);
    free(df->Us); free(df->Ts); free(df->Ps); free(df->rhos); free(df->Ms);
    free(df->T_fluc); free(df->rho_fluc);
    free(df);
}

/* ------------------------------------------------------------ accessors */

const double *orc_field_ptr(const orc_df *df, int which)
{
    if (which >= 0 && which < 3) return df->F[which].fluc;
    if (which == 3) return df->T_fluc;
    if (which == 4) return df->rho_fluc;
    return NULL;
}

int orc_dims(const orc_df *df, int *Ny, int *Nz) { *Ny = df->Ny; *Nz = df->Nz; return df->n_cells; }

const double *orc_row_ptr(const orc_df *df, int row)
{
    switch (row) {
    case 0: return df->R11; case 1: return df->R21; case 2: return df->R22; case 3: return df->R33;
    case 4: return df->Us; case 5: return df->Ts; case 6: return df->rhos; case 7: return df->Ms;
    case 8: return df->Ps; case 9: return df->yline; case 10: return df->ydline;
    }
    return NULL;
}

const orc_field *orc_field_struct(const orc_df *df, int comp) { return &df->F[comp]; }

double orc_scalar(const orc_df *df, int which)
{
    switch (which) { case 0: return df->u_tau; case 1: return df->tau_w; case 2: return df->d_v; }
    return 0.0;
}

int orc_write_csv(const orc_df *df, const char *path)
{
    /* df.cpp:764-803 */
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    int Ny = df->Ny, Nz = df->Nz;
    fputs("z,y,u_fluc,v_fluc,w_fluc,T_fluc,rho_fluc\n", f);
    for (int j = 0; j < Ny; ++j)
        for (int k = 0; k < Nz; ++k) {
            int n00 = j * (Nz + 1) + k, n01 = j * (Nz + 1) + (k + 1);
            int n10 = (j + 1) * (Nz + 1) + k, n11 = (j + 1) * (Nz + 1) + (k + 1);
            double yc = 0.25 * (df->y[n00] + df->y[n01] + df->y[n10] + df->y[n11]);
            double zc = 0.25 * (df->z[n00] + df->z[n01] + df->z[n10] + df->z[n11]);
            int c = j * Nz + k;
            fprintf(f, "%.15f,%.15f,%.15f,%.15f,%.15f,%.15f,%.15f\n", zc, yc,
                    df->F[0].fluc[c], df->F[1].fluc[c], df->F[2].fluc[c], df->T_fluc[c], df->rho_fluc[c]);
        }
    fclose(f);
    return 0;
}
