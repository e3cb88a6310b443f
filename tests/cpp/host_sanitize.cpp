// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer on the host side of
// libdfamd: df_capi.cpp and df_setup.cpp). Every handle is host-only (device = -1), so no GPU is
// touched: setup of the reference's own grid, synthetic and ragged planes, caller-vertex grids,
// z-strip planning, every host accessor, and the error paths. Built and run by
// tests/test_host_sanitize.py; exits non-zero on the first failed check (the sanitizers abort on
// their own findings).
#include "df_c.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

static int fails = 0;
#define CHECK(cond)                                                                                \
    do {                                                                                           \
        if (!(cond)) {                                                                             \
            std::fprintf(stderr, "FAIL %s:%d %s (%s)\n", __FILE__, __LINE__, #cond, df_last_error()); \
            ++fails;                                                                               \
        }                                                                                          \
    } while (0)

static std::string g_rst, g_line;

static df_config_c base()
{
    df_config_c c;
    df_config_default(&c);
    c.vel_fluc_file = g_rst.c_str();
    c.line_file = g_line.c_str();
    c.device = -1;
    c.seed = 7;
    return c;
}

// Every host query of one handle, with buffers sized from the handle's own answers.
static void exercise(df_handle *h)
{
    int Ny = 0, Nz = 0, z0 = 0, z1 = 0;
    CHECK(df_dims(h, &Ny, &Nz, &z0, &z1) == DF_OK);
    CHECK(Ny > 0 && Nz > 0 && z1 > z0);
    const int nloc = z1 - z0;
    for (int r = DF_ROW_R11; r <= DF_ROW_YC_D; ++r) {
        std::vector<double> row(Ny);
        CHECK(df_get_row(h, r, row.data()) == DF_OK);
        for (double x : row) CHECK(!std::isnan(x) || r == DF_ROW_R22);
    }
    for (int comp = 0; comp < 3; ++comp) {
        int nyx = 0, nzx = 0;
        long long bys = 0, bzs = 0;
        CHECK(df_get_comp_info(h, comp, &nyx, &nzx, &bys, &bzs) == DF_OK);
        CHECK(nyx >= 2 && nzx >= 2 && bys > 0 && bzs > 0);
        for (int dir = 0; dir < 2; ++dir) {
            std::vector<int> hw((size_t)Ny * nloc), off((size_t)Ny * nloc);
            CHECK(df_get_halfwidths(h, comp, dir, hw.data()) == DF_OK);
            CHECK(df_get_offsets(h, comp, dir, off.data()) == DF_OK);
            long long total = 0;
            for (int N : hw) {
                CHECK(N >= 2 && N % 2 == 0 && N <= (dir ? nzx : nyx));
                total += 2 * N + 1;
            }
            CHECK(total == (dir ? bzs : bys));
            std::vector<double> cf((size_t)total);
            CHECK(df_get_coeffs(h, comp, dir, cf.data(), total) == DF_OK);
            CHECK(df_get_coeffs(h, comp, dir, cf.data(), total - 1) != DF_OK); // too small
        }
    }
    CHECK(df_stream_length(h) > 0);
    int plane = -1, per_cell = -1;
    CHECK(df_plane_info(h, &plane, &per_cell) == DF_OK);
    std::vector<double> y((size_t)(Ny + 1) * (Nz + 1)), z((size_t)(Ny + 1) * (Nz + 1));
    CHECK(df_get_grid(h, y.data(), z.data()) == DF_OK);
    CHECK(df_get_row(h, 99, y.data()) != DF_OK);
    CHECK(df_get_halfwidths(h, 3, 0, nullptr) != DF_OK);
    CHECK(df_filter(h, 1e-8) != DF_OK); // host-only
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s RST.dat line.dat\n", argv[0]);
        return 2;
    }
    g_rst = argv[1];
    g_line = argv[2];

    { // the reference's own plane (read_grid placeholder, df.cpp:71-118)
        df_config_c c = base();
        df_handle *h = df_create(&c);
        CHECK(h);
        if (h) exercise(h), df_destroy(h);
    }
    for (int mode = 0; mode < 2; ++mode) // synthetic planes, ragged ones included
        for (auto dims : {std::vector<int>{128, 128, 8, 8}, {37, 5, 2, 6}, {300, 3, 2, 40}, {16, 300, 2, 64},
                          {64, 129, 2, 2}}) {
            df_config_c c = base();
            c.plane = DF_PLANE_SYNTHETIC;
            c.Ny = dims[0], c.Nz = dims[1], c.N_min = dims[2], c.N_max = dims[3];
            c.coeff_mode = mode;
            df_handle *h = df_create(&c);
            CHECK(h);
            if (h) exercise(h), df_destroy(h);
        }
    { // caller vertices: a stretched wall-normal grid with a slight spanwise warp (per-cell N)
        const int Ny = 40, Nz = 24;
        std::vector<double> gy((Ny + 1) * (Nz + 1)), gz((Ny + 1) * (Nz + 1));
        for (int j = 0; j <= Ny; ++j)
            for (int k = 0; k <= Nz; ++k) {
                const double eta = (double)j / Ny;
                gy[j * (Nz + 1) + k] = 0.0013 * 2.4 * (1 - std::tanh(2.0 * (1 - eta)) / std::tanh(2.0)) * (1 + 0.05 * k / Nz);
                gz[j * (Nz + 1) + k] = 1.33e-4 * k * (1 + 0.3 * eta);
            }
        df_config_c c = base();
        c.plane = DF_PLANE_GRID;
        c.Ny = Ny, c.Nz = Nz;
        c.grid_y = gy.data(), c.grid_z = gz.data();
        df_handle *h = df_create(&c);
        CHECK(h);
        if (h) exercise(h), df_destroy(h);
    }
    for (int world : {2, 3, 4}) // z-strip planning (host-only strips of one synthetic plane)
        for (int r = 0; r < world; ++r) {
            df_config_c c = base();
            c.plane = DF_PLANE_SYNTHETIC;
            c.Ny = 48, c.Nz = 400, c.N_min = 2, c.N_max = 16;
            c.rank = r, c.world = world;
            df_handle *h = df_create(&c);
            CHECK(h);
            if (h) exercise(h), df_destroy(h);
        }
    { // error paths: each must fail with a message, not crash
        df_config_c c = base();
        c.vel_fluc_file = "/nonexistent/RST.dat";
        CHECK(df_create(&c) == nullptr && std::strlen(df_last_error()) > 0);
        c = base();
        c.plane = DF_PLANE_SYNTHETIC;
        c.Ny = 1, c.Nz = 4, c.N_min = 2, c.N_max = 4;
        CHECK(df_create(&c) == nullptr);
        c.Ny = 16, c.Nz = 20, c.N_max = 16, c.rank = 0, c.world = 4; // strips narrower than N
        CHECK(df_create(&c) == nullptr);
        CHECK(df_create(nullptr) == nullptr);
        CHECK(df_filter(nullptr, 1e-8) != DF_OK);
        df_destroy(nullptr);
    }
    std::printf("host sanitize: %s (%d failed checks)\n", fails ? "FAIL" : "ok", fails);
    return fails != 0;
}
