// ORACLE HARNESS — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own DIGITAL_FILTER (df.cpp compiled unmodified from
// /root/reference by oracle/ref/Makefile) to produce golden vectors and the
// "reference" CPU baseline. Nothing here is part of the product.
//
// Determinism: the reference seeds a function-local static pcg32 from
// std::random_device (df.cpp:334). This translation unit defines
// std::random_device::_M_getval(), which the executable's own inline
// random_device::operator() binds to instead of libstdc++'s, so the seed comes
// from $DF_SEED without touching the reference source.
//
// Synthetic planes reuse the reference's own setup code: after the
// native constructor has run, the harness installs a uniform grid, re-runs
// get_RST_in() for the rows, and chooses per-cell dy/dz with Iz_inn == Iz_out so
// that the reference's calculate_filter_properties() (df.cpp:130-218) itself
// produces the requested half-width N(j). The hot path is the reference's.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <unistd.h>
#include <vector>

#define private public
#include "df.hpp"
#undef private

extern std::vector<double> z; // ref_shim.hpp (global vertex array df.cpp uses)

static unsigned int g_seed = 42u;
unsigned int std::random_device::_M_getval() { return g_seed; }

static void write_bin(const std::string &path, const void *p, size_t bytes)
{
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(2); }
    if (bytes) fwrite(p, 1, bytes, f);
    fclose(f);
}

static int synthetic_N(int j, int Ny, int N_min, int N_max)
{
    double x = (Ny > 1) ? (double)j / (double)(Ny - 1) : 0.0;
    double h = N_min + (N_max - N_min) * 0.5 * (1.0 + tanh((x - 0.2) / 0.03));
    int N = 2 * (int)floor(h / 2.0);
    return N < 2 ? 2 : N;
}

static void dump_state(DIGITAL_FILTER &df, const std::string &out, const std::string &tag)
{
    size_t n = (size_t)df.n_cells;
    write_bin(out + "/" + tag + "_u.bin", df.u.fluc.data(), n * 8);
    write_bin(out + "/" + tag + "_v.bin", df.v.fluc.data(), n * 8);
    write_bin(out + "/" + tag + "_w.bin", df.w.fluc.data(), n * 8);
    write_bin(out + "/" + tag + "_T.bin", df.T_fluc.data(), n * 8);
    write_bin(out + "/" + tag + "_rho.bin", df.rho_fluc.data(), n * 8);
}

static void dump_setup(DIGITAL_FILTER &df, const std::string &out)
{
    size_t Ny = (size_t)df.Ny, n = (size_t)df.n_cells;
    write_bin(out + "/R11.bin", df.R11.data(), Ny * 8);
    write_bin(out + "/R21.bin", df.R21.data(), Ny * 8);
    write_bin(out + "/R22.bin", df.R22.data(), Ny * 8);
    write_bin(out + "/R33.bin", df.R33.data(), Ny * 8);
    write_bin(out + "/Us.bin", df.Us.data(), Ny * 8);
    write_bin(out + "/Ts.bin", df.Ts.data(), Ny * 8);
    write_bin(out + "/rhos.bin", df.rhos.data(), Ny * 8);
    write_bin(out + "/Ms.bin", df.Ms.data(), Ny * 8);
    const char *nm[3] = {"u", "v", "w"};
    FilterField *F[3] = {&df.u, &df.v, &df.w};
    for (int c = 0; c < 3; ++c) {
        write_bin(out + "/Nys_" + nm[c] + ".bin", F[c]->N_ys.data(), n * 4);
        write_bin(out + "/Nzs_" + nm[c] + ".bin", F[c]->N_zs.data(), n * 4);
    }
    std::ofstream js(out + "/meta.json");
    js << std::setprecision(17);
    js << "{\"Ny\": " << df.Ny << ", \"Nz\": " << df.Nz << ", \"u_tau\": " << df.u_tau
       << ", \"tau_w\": " << df.tau_w << ", \"d_v\": " << df.d_v
       << ", \"Ny_max\": [" << df.u.Ny_max << ", " << df.v.Ny_max << ", " << df.w.Ny_max << "]"
       << ", \"Nz_max\": [" << df.u.Nz_max << ", " << df.v.Nz_max << ", " << df.w.Nz_max << "]"
       << ", \"by_size\": [" << df.u.by.size() << ", " << df.v.by.size() << ", " << df.w.by.size() << "]"
       << ", \"bz_size\": [" << df.u.bz.size() << ", " << df.v.bz.size() << ", " << df.w.bz.size() << "]"
       << "}\n";
}

// Install a synthetic plane on an already-constructed object and run step 0 the
// way the constructor does (df.cpp:26-62).
static void make_synthetic(DIGITAL_FILTER &df, int Ny, int Nz, int N_min, int N_max)
{
    int n = Ny * Nz;
    df.Ny = Ny; df.Nz = Nz; df.n_cells = n;
    df.y = Vector((size_t)(Ny + 1) * (Nz + 1));
    z = Vector((size_t)(Ny + 1) * (Nz + 1));
    df.yc = Vector(n);
    df.yc_d = Vector((size_t)n + Nz, 1e300); // sentinel row: get_RST_in's loop reads yc_d[Ny*Nz]
    df.dy = Vector(n);
    df.dz = Vector(n);
    df.ydline = Vector(Ny);
    df.yline = Vector(Ny);
    double hy = 2.4 * df.d_i / Ny;
    for (int j = 0; j <= Ny; ++j)
        for (int k = 0; k < Nz + 1; ++k) {
            df.y[j * (Nz + 1) + k] = j * hy;
            z[j * (Nz + 1) + k] = k * 0.000133;
        }
    for (int j = 0; j < Ny; ++j) {
        for (int k = 0; k < Nz; ++k) {
            int idx = j * Nz + k;
            df.dy[idx] = df.y[(j + 1) * (Nz + 1) + k] - df.y[j * (Nz + 1) + k];
            df.dz[idx] = 0.000133;
            df.yc[idx] = 0.25 * (df.y[j * (Nz + 1) + k] + df.y[(j + 1) * (Nz + 1) + k]
                                 + df.y[j * (Nz + 1) + k + 1] + df.y[(j + 1) * (Nz + 1) + k + 1]);
            df.yc_d[idx] = df.yc[idx] / df.d_i;
        }
        df.ydline[j] = df.yc_d[j * Nz];
        df.yline[j] = df.yc[j * Nz];
    }
    df.get_RST_in(); // reference rows on the synthetic grid
    if (df.Ny != Ny) { fprintf(stderr, "unexpected truncation %d -> %d\n", Ny, df.Ny); exit(3); }
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.allocate_data_structures(*F);
    const double Iz0 = 0.4 * df.d_i;
    for (FilterField *F : {&df.u, &df.v, &df.w}) { F->Iz_inn = Iz0; F->Iz_out = Iz0; }
    df.dz.resize(n);
    for (int j = 0; j < Ny; ++j) {
        double q = synthetic_N(j, Ny, N_min, N_max) / 2 + 0.5; // Iz/dz = q -> N = 2*int(q)
        for (int k = 0; k < Nz; ++k) {
            df.dz[j * Nz + k] = Iz0 / q;
            df.dy[j * Nz + k] = 0.67 * Iz0 / q;
        }
    }
    df.rho_fluc = Vector(n);
    df.T_fluc = Vector(n);
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.calculate_filter_properties(*F);
    for (FilterField *F : {&df.u, &df.v, &df.w})
        for (int idx = 0; idx < n; ++idx) {
            int want = synthetic_N(idx / Nz, Ny, N_min, N_max);
            if (F->N_ys[idx] != want || F->N_zs[idx] != want) {
                fprintf(stderr, "half-width mismatch at %d: %d/%d vs %d\n", idx, F->N_ys[idx], F->N_zs[idx], want);
                exit(4);
            }
        }
    df.generate_white_noise();
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.filtering_sweeps(*F);
    df.apply_RST_scaling();
}

// Install caller vertices (a real inflow grid) in place of read_grid()'s placeholder
// (df.cpp:71-118): per-cell dy, dz, yc exactly as df.cpp:104-116 derives them, with
// dz taken from the vertices instead of the constant 0.000133 (df.cpp:108). Rows
// (get_RST_in), integral scales (ctor values), half-widths and coefficients
// (calculate_filter_properties) and step 0 are the reference's own code.
static void make_grid(DIGITAL_FILTER &df, int Ny, int Nz, const std::vector<double> &gy,
                      const std::vector<double> &gz)
{
    int n = Ny * Nz;
    df.Ny = Ny; df.Nz = Nz; df.n_cells = n;
    df.y = gy;
    z = gz;
    df.yc = Vector(n);
    df.yc_d = Vector((size_t)n + Nz, 1e300); // sentinel row: get_RST_in's loop reads yc_d[Ny*Nz]
    df.dy = Vector(n);
    df.dz = Vector(n);
    df.ydline = Vector(Ny);
    df.yline = Vector(Ny);
    for (int j = 0; j < Ny; ++j) {
        for (int k = 0; k < Nz; ++k) {
            int idx = j * Nz + k;
            df.dy[idx] = df.y[(j + 1) * (Nz + 1) + k] - df.y[j * (Nz + 1) + k];
            df.dz[idx] = z[j * (Nz + 1) + k + 1] - z[j * (Nz + 1) + k];
            df.yc[idx] = 0.25 * (df.y[j * (Nz + 1) + k] + df.y[(j + 1) * (Nz + 1) + k]
                                 + df.y[j * (Nz + 1) + k + 1] + df.y[(j + 1) * (Nz + 1) + k + 1]);
            df.yc_d[idx] = df.yc[idx] / df.d_i;
        }
        df.ydline[j] = df.yc_d[j * Nz];
        df.yline[j] = df.yc[j * Nz];
    }
    df.get_RST_in(); // truncates Ny to the RST profile's reach (df.cpp:280-304)
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.allocate_data_structures(*F);
    df.rho_fluc = Vector(df.n_cells);
    df.T_fluc = Vector(df.n_cells);
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.calculate_filter_properties(*F);
    df.generate_white_noise();
    for (FilterField *F : {&df.u, &df.v, &df.w}) df.filtering_sweeps(*F);
    df.apply_RST_scaling();
}

static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: ref_harness rng|native|synth|time ...\n");
        return 1;
    }
    std::string mode = argv[1];
    std::cout.setf(std::ios::unitbuf);

    if (mode == "rng") { // rng <seed> <n> <outdir>
        unsigned seed = (unsigned)strtoul(argv[2], 0, 10);
        size_t n = strtoull(argv[3], 0, 10);
        std::string out = argv[4];
        pcg32 r1(seed);
        std::vector<uint32_t> u(n);
        for (auto &x : u) x = r1();
        pcg32 r2(seed);
        std::normal_distribution<> dist(0.0, 1.0);
        std::vector<double> g(n);
        for (auto &x : g) x = dist(r2);
        write_bin(out + "/u32.bin", u.data(), n * 4);
        write_bin(out + "/normals.bin", g.data(), n * 8);
        return 0;
    }

    // Common: <root> <seed> ...  (root holds files/RST.dat, line.dat and run/)
    std::string root = argv[2];
    g_seed = (unsigned)strtoul(argv[3], 0, 10);
    if (chdir((root + "/run").c_str()) != 0) { perror("chdir"); return 2; }
    DFConfig cfg{};

    if (mode == "native") { // native <root> <seed> <dt> <nsteps> <outdir>
        double dt = strtod(argv[4], 0);
        int nsteps = atoi(argv[5]);
        std::string out = argv[6];
        DIGITAL_FILTER df(cfg);
        dump_setup(df, out);
        dump_state(df, out, "step0");
        for (int s = 1; s <= nsteps; ++s) {
            df.filter(dt);
            dump_state(df, out, "step" + std::to_string(s));
        }
        return 0;
    }
    if (mode == "synth") { // synth <root> <seed> <Ny> <Nz> <Nmin> <Nmax> <dt> <nsteps> <outdir> [dt2 nsteps2]
        int Ny = atoi(argv[4]), Nz = atoi(argv[5]), Nmin = atoi(argv[6]), Nmax = atoi(argv[7]);
        double dt = strtod(argv[8], 0);
        int nsteps = atoi(argv[9]);
        std::string out = argv[10];
        double dt2 = argc > 12 ? strtod(argv[11], 0) : 0.0;
        int nsteps2 = argc > 12 ? atoi(argv[12]) : 0;
        DIGITAL_FILTER df(cfg);
        make_synthetic(df, Ny, Nz, Nmin, Nmax);
        dump_setup(df, out);
        dump_state(df, out, "step0");
        int s = 1;
        for (; s <= nsteps; ++s) { df.filter(dt); dump_state(df, out, "step" + std::to_string(s)); }
        for (int t = 0; t < nsteps2; ++t, ++s) { df.filter(dt2); dump_state(df, out, "step" + std::to_string(s)); }
        return 0;
    }
    if (mode == "grid") { // grid <root> <seed> <vertfile> <dt> <nsteps> <outdir>
        FILE *f = fopen(argv[4], "rb");
        if (!f) { perror(argv[4]); return 2; }
        int dims[2];
        if (fread(dims, 4, 2, f) != 2) return 2;
        size_t nv = (size_t)(dims[0] + 1) * (dims[1] + 1);
        std::vector<double> gy(nv), gz(nv);
        if (fread(gy.data(), 8, nv, f) != nv || fread(gz.data(), 8, nv, f) != nv) return 2;
        fclose(f);
        double dt = strtod(argv[5], 0);
        int nsteps = atoi(argv[6]);
        std::string out = argv[7];
        DIGITAL_FILTER df(cfg);
        make_grid(df, dims[0], dims[1], gy, gz);
        dump_setup(df, out);
        dump_state(df, out, "step0");
        for (int s = 1; s <= nsteps; ++s) { df.filter(dt); dump_state(df, out, "step" + std::to_string(s)); }
        return 0;
    }
    if (mode == "writers") { // writers <root> <seed> <dt> <nsteps> <outdir>: the reference's file outputs
        // filter() writes ../files/cpp_vel_fluc.csv after every call (df.cpp:466-467); then
        // write_tecplot (df.cpp:712-762) and plot_RST_lerp (677-706, ../files/myRST.csv, duanRST.csv).
        double dt = strtod(argv[4], 0);
        int nsteps = atoi(argv[5]);
        std::string out = argv[6];
        DIGITAL_FILTER df(cfg);
        for (int s = 1; s <= nsteps; ++s) df.filter(dt);
        df.write_tecplot(out + "/tecplot.dat");
        df.plot_RST_lerp();
        dump_state(df, out, "final");
        return 0;
    }
    if (mode == "rms") { // rms <root> <seed> <outdir> [Ny Nz Nmin Nmax]: the reference driver's call (cpp-main.cpp:12-17)
        std::string out = argv[4];
        DIGITAL_FILTER df(cfg);
        if (argc > 8) make_synthetic(df, atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]));
        df.get_rms(); // 500 x {noise, sweeps, correlate, RST, SRA, rms_add} at dt = 1e-5, then plot_rms
        size_t n = (size_t)df.n_cells;
        write_bin(out + "/rms_u.bin", df.u.rms.data(), n * 8);
        write_bin(out + "/rms_v.bin", df.v.rms.data(), n * 8);
        write_bin(out + "/rms_w.bin", df.w.rms.data(), n * 8);
        write_bin(out + "/rms_T.bin", df.T_rms.data(), n * 8);
        write_bin(out + "/rms_rho.bin", df.rho_rms.data(), n * 8);
        std::ofstream js(out + "/meta.json");
        js << "{\"Ny\": " << df.Ny << ", \"Nz\": " << df.Nz << ", \"rms_counter\": " << df.rms_counter << "}\n";
        return 0;
    }
    if (mode == "time") { // time <root> <seed> <Ny> <Nz> <Nmin> <Nmax> <dt> <ncalls>
        int Ny = atoi(argv[4]), Nz = atoi(argv[5]), Nmin = atoi(argv[6]), Nmax = atoi(argv[7]);
        double dt = strtod(argv[8], 0);
        int ncalls = atoi(argv[9]);
        double t0 = now_s();
        DIGITAL_FILTER df(cfg);
        make_synthetic(df, Ny, Nz, Nmin, Nmax);
        double t_setup = now_s() - t0;
        // filter(dt) minus its CSV side effect (df.cpp:449-461), i.e. exactly the
        // region the reference's own "Filtering took" timer covers (df.cpp:452-462).
        double tn = 0, ts = 0, tc = 0, tr = 0, tt = 0, tot = 0;
        double best = 1e300;
        for (int c = 0; c < ncalls; ++c) {
            df.dt = dt;
            double a = now_s();
            df.generate_white_noise();
            double b = now_s();
            double sw = 0, co = 0;
            for (FilterField *F : {&df.u, &df.v, &df.w}) {
                double p = now_s(); df.filtering_sweeps(*F);
                double q = now_s(); df.correlate_fields(*F);
                double r = now_s(); sw += q - p; co += r - q;
            }
            double d = now_s();
            df.apply_RST_scaling();
            double e = now_s();
            df.get_rho_T_fluc();
            double f = now_s();
            tn += b - a; ts += sw; tc += co; tr += e - d; tt += f - e; tot += f - a;
            if (f - a < best) best = f - a;
        }
        double chk = 0;
        for (double x : df.u.fluc) chk += x * x;
        printf("{\"setup_s\": %.6f, \"calls\": %d, \"mean_s\": %.6f, \"best_s\": %.6f, "
               "\"noise_s\": %.6f, \"sweeps_s\": %.6f, \"correlate_s\": %.6f, \"rst_s\": %.6f, \"sra_s\": %.6f, "
               "\"cells\": %d, \"sum_u2\": %.17g}\n",
               t_setup, ncalls, tot / ncalls, best, tn / ncalls, ts / ncalls, tc / ncalls, tr / ncalls,
               tt / ncalls, df.n_cells, chk);
        return 0;
    }
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 1;
}
