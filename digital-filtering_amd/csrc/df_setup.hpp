// Host-side setup for one DIGITAL_FILTER plane: grid, wall-normal profiles,
// Reynolds-stress rows, filter half-widths and the per-N coefficient table.
// Restates (from scratch, per row instead of per cell) the reference constructor
// inputs: read_grid (df.cpp:71-118), get_RST_in (220-330), read_line_file
// (487-553), linear_interpolate (805-848), calculate_filter_properties (130-218).
//
// On the reference's grid and the synthetic planes every input of
// calculate_filter_properties (yc, dy, dz) depends on the row j only, so the
// half-width N is a per-row quantity. A grid plane (caller vertices)
// has per-cell dy, dz and yc, hence per-cell N: those are kept per cell
// (ComponentSetup::Ny_cell / Nz_cell) next to the per-row maxima.
#pragma once
#include <map>
#include <string>
#include <vector>

namespace dfamd {

struct Flow {
    // DFConfig fields (df.hpp:38-49) with the values the reference hard-codes
    // in its constructor (df.cpp:7-16).
    double d_i = 0.0013, rho_e = 0.044, U_e = 869.1, mu = 7.1212e-6;
    double T_w = 97.5, gcon = 287.0, T_e = 55.2, rho_w = 0.0249;
};

enum PlaneKind { kPlaneNative = 0, kPlaneSynthetic = 1, kPlaneGrid = 2 };

struct PlaneSpec {
    int kind = kPlaneNative;
    int Ny = 0, Nz = 0;        // synthetic plane size
    int N_min = 0, N_max = 0;  // synthetic half-width rule
    std::string rst_file, line_file;
    // kPlaneGrid: vertices (Ny+1)*(Nz+1), index j*(Nz+1)+k, row 0 at the wall (Ny, Nz = cells),
    // or, when empty, grid_file in the reference's Tecplot BLOCK layout (write_tecplot, df.cpp:712-762).
    std::vector<double> grid_y, grid_z;
    std::string grid_file;
};

struct ComponentSetup {
    double Iz_inn = 0, Iz_out = 0, Lt = 0;
    std::vector<int> Ny_row, Nz_row;   // half-width per row (the row's maximum on a grid plane)
    std::vector<int> Ny_cell, Nz_cell; // per cell, Ny x Nz (global), only when Setup::per_cell
    int Ny_max = 0, Nz_max = 0;
    int Ny_at(int j, int k) const { return Ny_cell.empty() ? Ny_row[j] : Ny_cell[(size_t)j * Nz_cols + k]; }
    int Nz_at(int j, int k) const { return Nz_cell.empty() ? Nz_row[j] : Nz_cell[(size_t)j * Nz_cols + k]; }
    int Nz_cols = 0;
};

struct Setup {
    int Ny = 0, Nz = 0;                       // global plane (after RST truncation)
    std::vector<double> y_vert, z_vert;       // vertex y per row (Ny+1), z per column (Nz+1)
    std::vector<double> yv, zv;               // grid plane: all vertices (Ny+1)*(Nz+1) (writers)
    bool per_cell = false;                    // some half-width varies along a row
    std::vector<double> yc, yc_d, dy;         // cell-centre y, y/d_i, height per row
    double dz = 0.000133;                     // df.cpp:108
    std::vector<double> R11, R21, R22, R33;   // per row (df.cpp:292-323)
    std::vector<double> Us, Ts, Ps, rhos, Ms; // per row (df.cpp:509-545)
    double u_tau = 0, tau_w = 0, d_v = 0;
    ComponentSetup comp[3];                   // u, v, w
    std::map<int, std::vector<double>> coeffs; // N -> b[0..N] (df.cpp:166-177)
};

// Builds everything above. Returns false and fills `err` on bad input
// (the reference prints to cerr and continues with unset state; we fail fast).
bool build_setup(const Flow &flow, const PlaneSpec &spec, Setup &out, std::string &err);

// Synthetic half-width rule N(j) = max(2, 2*floor(h/2)),
// h = Nmin + (Nmax-Nmin)*0.5*(1+tanh((j/(Ny-1)-0.2)/0.03)) (mirrors df.cpp:146-148).
int synthetic_halfwidth(int j, int Ny, int N_min, int N_max);

// One cell's coefficient half-vector b[0..N] exactly as df.cpp:166-177 computes it.
void cell_coefficients(int N, double *half);

// Reference CSV (df.cpp:764-803) for a dense [Ny x Nz] block of rows starting at
// global column z0 (z0 = 0, nz = Nz for the whole plane).
bool write_csv(const Setup &s, const std::string &path, const double *u, const double *v, const double *w,
               const double *T, const double *rho, int z0, int nz, std::string &err);

} // namespace dfamd
