// Host setup for the filter(dt) hot path — see df_setup.hpp.
// Floating-point expressions keep the reference's evaluation order; the library
// is compiled with -ffp-contract=off so the results are bit-identical to the
// reference's x86-64 -O2 build on the same libm.
#include "df_setup.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace dfamd {

namespace {

// Clamped linear interpolation with a linear search (df.cpp:805-848).
std::vector<double> lerp(const std::vector<double> &yd, const std::vector<double> &fd,
                         const std::vector<double> &yn)
{
    std::vector<double> fn(yn.size());
    for (size_t j = 0; j < yn.size(); ++j) {
        const double y = yn[j];
        if (y <= yd.front()) { fn[j] = fd.front(); continue; }
        if (y >= yd.back()) { fn[j] = fd.back(); continue; }
        size_t i = 0;
        while (i + 1 < yd.size() && y > yd[i + 1]) ++i;
        const double x0 = yd[i], x1 = yd[i + 1], f0 = fd[i], f1 = fd[i + 1];
        fn[j] = f0 + (f1 - f0) * ((y - x0) / (x1 - x0));
    }
    return fn;
}

// Tecplot-style point file: header line, "ZONE ... i=<n>" line, then n rows.
bool read_table(const std::string &path, int min_cols, std::vector<std::vector<double>> &rows, std::string &err)
{
    std::ifstream fin(path);
    if (!fin) { err = "cannot open " + path; return false; }
    std::string line;
    std::getline(fin, line);
    std::getline(fin, line);
    const size_t pos = line.find("i=");
    double n_in = 0;
    if (pos != std::string::npos) {
        std::istringstream iss(line.substr(pos + 2));
        iss >> n_in;
    }
    const int n = (int)n_in;
    if (n < 2) { err = "missing or bad \"i=\" count in " + path; return false; }
    rows.clear();
    int count = 0;
    while (std::getline(fin, line)) {
        if (line.empty()) continue;
        std::istringstream iss(line);
        std::vector<double> v;
        double x;
        while (iss >> x) v.push_back(x);
        if (count < n) {
            if ((int)v.size() < min_cols) { err = "short row " + std::to_string(count) + " in " + path; return false; }
            rows.push_back(std::move(v));
        }
        count++;
    }
    if ((int)rows.size() < n) { err = path + ": fewer rows than its i= count"; return false; }
    return true;
}

void grid_native(const Flow &f, Setup &s)
{
    // df.cpp:71-118. y does not depend on k; vertex row jr = |j - Ny|.
    const int Nz = 400, Ny = 560;
    s.Ny = Ny;
    s.Nz = Nz;
    s.y_vert.assign(Ny + 1, 0.0);
    const double y_max = 3 * f.d_i, a = 2.0;
    for (int j = Ny; j >= 0; --j) {
        const double eta = ((j)*y_max / (Ny + 1)) / y_max;
        s.y_vert[std::abs(j - Ny)] = y_max * (1 - std::tanh(a * eta) / std::tanh(a));
    }
}

void grid_synthetic(const Flow &f, int Ny, int Nz, Setup &s)
{
    // uniform wall-normal spacing 2.4*d_i/Ny.
    s.Ny = Ny;
    s.Nz = Nz;
    s.y_vert.assign(Ny + 1, 0.0);
    const double hy = 2.4 * f.d_i / Ny;
    for (int j = 0; j <= Ny; ++j) s.y_vert[j] = j * hy;
}

// Tecplot BLOCK file as write_tecplot writes it (df.cpp:712-762): VARIABLES naming z and y
// first, ZONE with I = Nz+1 and J = Ny+1, then I*J values of each variable in that order.
bool read_tecplot_grid(const std::string &path, int &Ny, int &Nz, std::vector<double> &gy,
                       std::vector<double> &gz, std::string &err)
{
    std::ifstream in(path);
    if (!in) { err = "cannot open grid file " + path; return false; }
    std::string line;
    int I = -1, J = -1, yfirst = -1;
    while (std::getline(in, line)) {
        std::string up = line;
        for (char &ch : up) ch = (char)std::toupper((unsigned char)ch);
        if (up.find("VARIABLES") != std::string::npos) {
            const size_t py = up.find("\"Y\""), pz = up.find("\"Z\"");
            if (py == std::string::npos || pz == std::string::npos) { err = path + ": VARIABLES must name \"y\" and \"z\""; return false; }
            yfirst = py < pz;
        }
        if (up.find("ZONE") != std::string::npos) {
            auto num = [&](const char *key) {
                size_t p = up.find(key);
                return p == std::string::npos ? -1 : std::atoi(up.c_str() + p + std::strlen(key));
            };
            I = num("I=");
            J = num("J=");
            break;
        }
    }
    if (yfirst < 0 || I < 2 || J < 3) { err = path + ": needs VARIABLES and ZONE I=(Nz+1) J=(Ny+1) headers"; return false; }
    const size_t n = (size_t)I * J;
    std::vector<double> a(n), b(n);
    size_t got = 0;
    std::string tok;
    while (got < 2 * n && in >> tok) {
        char *end = nullptr;
        const double v = std::strtod(tok.c_str(), &end);
        if (end == tok.c_str()) continue; // VARLOCATION / DT lines
        (got < n ? a[got] : b[got - n]) = v;
        ++got;
    }
    if (got < 2 * n) { err = path + ": fewer values than 2*I*J"; return false; }
    Nz = I - 1;
    Ny = J - 1;
    gy = yfirst ? a : b;
    gz = yfirst ? b : a;
    return true;
}

void cell_geometry(const Flow &f, Setup &s)
{
    const int Ny = s.Ny, Nz = s.Nz;
    s.z_vert.resize(Nz + 1);
    for (int k = 0; k <= Nz; ++k) s.z_vert[k] = k * 0.000133; // df.cpp:100
    s.yc.resize(Ny);
    s.yc_d.resize(Ny);
    s.dy.resize(Ny);
    for (int j = 0; j < Ny; ++j) {
        const double y0 = s.y_vert[j], y1 = s.y_vert[j + 1];
        s.dy[j] = y1 - y0;                       // df.cpp:107
        s.yc[j] = 0.25 * (y0 + y1 + y0 + y1);    // df.cpp:109-112 vertex order
        s.yc_d[j] = s.yc[j] / f.d_i;             // df.cpp:113
    }
}

} // namespace

int synthetic_halfwidth(int j, int Ny, int N_min, int N_max)
{
    const double x = (Ny > 1) ? (double)j / (double)(Ny - 1) : 0.0;
    const double h = N_min + (N_max - N_min) * 0.5 * (1.0 + std::tanh((x - 0.2) / 0.03));
    const int N = 2 * (int)std::floor(h / 2.0);
    return N < 2 ? 2 : N;
}

void cell_coefficients(int N, double *half)
{
    constexpr double pi_c = -2.0 * 3.14159265358979323846; // df.hpp:16
    std::vector<double> temp(N + 1);
    double sum = 0.0;
    for (int i = 0; i <= N; ++i) {
        temp[i] = std::exp(pi_c * std::abs(i) / N);
        sum += (i == 0 ? 1.0 : 2.0) * temp[i] * temp[i];
    }
    sum = std::sqrt(sum);
    for (int i = 0; i <= N; ++i) half[i] = temp[i] / sum;
}

bool build_setup(const Flow &f, const PlaneSpec &spec, Setup &s, std::string &err)
{
    // per-cell geometry of a grid plane (df.cpp:104-116 on caller vertices)
    std::vector<double> cyc, cdy, cdz;
    if (spec.kind == kPlaneGrid) {
        int Ny = spec.Ny, Nz = spec.Nz;
        std::vector<double> gy = spec.grid_y, gz = spec.grid_z;
        if (gy.empty() && !spec.grid_file.empty()) {
            if (!read_tecplot_grid(spec.grid_file, Ny, Nz, gy, gz, err)) return false;
        }
        if (Ny < 2 || Nz < 1 || gy.size() != (size_t)(Ny + 1) * (Nz + 1) || gz.size() != gy.size()) {
            err = "grid plane needs Ny >= 2, Nz >= 1 and (Ny+1)*(Nz+1) y and z vertices (or a grid_file)";
            return false;
        }
        s.Ny = Ny;
        s.Nz = Nz;
        const size_t n = (size_t)Ny * Nz;
        cyc.resize(n);
        cdy.resize(n);
        cdz.resize(n);
        for (int j = 0; j < Ny; ++j)
            for (int k = 0; k < Nz; ++k) {
                const size_t idx = (size_t)j * Nz + k, v00 = (size_t)j * (Nz + 1) + k, v10 = v00 + Nz + 1;
                cdy[idx] = gy[v10] - gy[v00];                              // df.cpp:107
                cdz[idx] = gz[v00 + 1] - gz[v00];                          // bottom edge (df.cpp:108 placeholder)
                cyc[idx] = 0.25 * (gy[v00] + gy[v10] + gy[v00 + 1] + gy[v10 + 1]); // df.cpp:109-112
                if (!(cdy[idx] > 0) || !(cdz[idx] > 0)) {
                    err = "grid plane: vertices must increase in j (y) and k (z) at every cell";
                    return false;
                }
            }
        s.yv = std::move(gy);
        s.zv = std::move(gz);
        // rows (ydline, yline, dy per row) come from column 0 as in df.cpp:116
        s.y_vert.resize(Ny + 1);
        for (int j = 0; j <= Ny; ++j) s.y_vert[j] = s.yv[(size_t)j * (Nz + 1)];
        s.z_vert.assign(s.zv.begin(), s.zv.begin() + Nz + 1);
        s.yc.resize(Ny);
        s.yc_d.resize(Ny);
        s.dy.resize(Ny);
        for (int j = 0; j < Ny; ++j) {
            s.yc[j] = cyc[(size_t)j * Nz];
            s.yc_d[j] = s.yc[j] / f.d_i;
            s.dy[j] = cdy[(size_t)j * Nz];
        }
    } else if (spec.kind == kPlaneNative) {
        grid_native(f, s);
    } else if (spec.kind == kPlaneSynthetic) {
        if (spec.Ny < 2 || spec.Nz < 1 || spec.N_min < 2 || spec.N_max < spec.N_min) {
            err = "synthetic plane needs Ny >= 2, Nz >= 1, 2 <= N_min <= N_max";
            return false;
        }
        grid_synthetic(f, spec.Ny, spec.Nz, s);
    } else {
        err = "unknown plane kind";
        return false;
    }
    if (spec.kind != kPlaneGrid) cell_geometry(f, s);

    // ---- get_RST_in (df.cpp:220-330)
    std::vector<std::vector<double>> rst;
    if (!read_table(spec.rst_file, 6, rst, err)) return false;
    const int N_in = (int)rst.size();
    std::vector<double> yin_d(N_in), urms(N_in), vrms(N_in), wrms(N_in), uvrms(N_in);
    for (int i = 0; i < N_in; ++i) {
        yin_d[i] = rst[i][1];
        urms[i] = rst[i][2];
        vrms[i] = rst[i][3];
        wrms[i] = rst[i][4];
        uvrms[i] = rst[i][5];
    }
    // Keep only rows with yc/d_i <= last RST y/delta (df.cpp:282-288).
    int new_Ny = 0;
    while (new_Ny < s.Ny && s.yc_d[new_Ny] <= yin_d[N_in - 1]) new_Ny++;
    if (new_Ny < 2) { err = "RST profile covers fewer than two grid rows"; return false; }
    s.Ny = new_Ny;
    if (!s.yv.empty()) s.yv.resize((size_t)(s.Ny + 1) * (s.Nz + 1)); // df.cpp:297 keeps the first rows
    if (!s.zv.empty()) s.zv.resize((size_t)(s.Ny + 1) * (s.Nz + 1));
    s.y_vert.resize(s.Ny + 1);
    s.yc.resize(s.Ny);
    s.yc_d.resize(s.Ny);
    s.dy.resize(s.Ny);

    // ---- read_line_file (df.cpp:487-553)
    std::vector<std::vector<double>> ln;
    if (!read_table(spec.line_file, 10, ln, err)) return false;
    const int N_line = (int)ln.size();
    std::vector<double> y_f(N_line), rho_f(N_line), u_f(N_line), T_f(N_line), p_f(N_line);
    for (int i = 0; i < N_line; ++i) {
        y_f[i] = ln[i][1];
        rho_f[i] = ln[i][4];
        u_f[i] = ln[i][5];
        T_f[i] = ln[i][8];
        p_f[i] = ln[i][9];
    }
    const std::vector<double> &yline = s.yc; // yline[j] = yc[j*Nz] (df.cpp:116)
    s.Us = lerp(y_f, u_f, yline);
    s.Ps = lerp(y_f, p_f, yline);
    s.Ts = lerp(y_f, T_f, yline);
    s.rhos = lerp(y_f, rho_f, yline);
    s.Ms.resize(s.Ny);
    for (int j = 0; j < s.Ny; ++j) s.Ms[j] = s.Us[j] / std::sqrt(1.4 * f.gcon * s.Ts[j]);
    const double dyl = y_f[1] - y_f[0];
    const double du = s.Us[1] - s.Us[0];
    s.tau_w = f.mu * du / dyl;
    s.u_tau = std::sqrt(s.tau_w / s.rhos[0]);

    // ---- Reynolds-stress rows (df.cpp:312-323)
    const double ut = s.u_tau;
    std::vector<double> R11_in(N_in), R21_in(N_in), R22_in(N_in), R33_in(N_in);
    for (int i = 0; i < N_in; ++i) {
        R11_in[i] = urms[i] * urms[i] * ut * ut;
        R22_in[i] = vrms[i] * vrms[i] * ut * ut;
        R33_in[i] = wrms[i] * wrms[i] * ut * ut;
        R21_in[i] = uvrms[i] * ut * ut;
    }
    const std::vector<double> &ydline = s.yc_d;
    s.R11 = lerp(yin_d, R11_in, ydline);
    s.R22 = lerp(yin_d, R22_in, ydline);
    s.R21 = lerp(yin_d, R21_in, ydline);
    s.R33 = lerp(yin_d, R33_in, ydline);
    s.d_v = f.d_i / 4500; // df.cpp:326

    // ---- integral scales (df.cpp:35-45) and half-widths (df.cpp:144-195)
    ComponentSetup &u = s.comp[0], &v = s.comp[1], &w = s.comp[2];
    u.Iz_out = 0.4 * f.d_i; u.Iz_inn = 150 * s.d_v; u.Lt = 0.8 * f.d_i / f.U_e;
    v.Iz_out = 0.3 * f.d_i; v.Iz_inn = 75 * s.d_v;  v.Lt = 0.3 * f.d_i / f.U_e;
    w.Iz_out = 0.4 * f.d_i; w.Iz_inn = 150 * s.d_v; w.Lt = 0.3 * f.d_i / f.U_e;
    const bool grid = spec.kind == kPlaneGrid;
    s.per_cell = false;
    for (ComponentSetup &F : s.comp) {
        F.Ny_row.resize(s.Ny);
        F.Nz_row.resize(s.Ny);
        F.Nz_cols = s.Nz;
        F.Ny_max = F.Nz_max = 0;
        if (grid) { // df.cpp:144-149, 185-190 per cell
            const size_t n = (size_t)s.Ny * s.Nz;
            F.Ny_cell.resize(n);
            F.Nz_cell.resize(n);
            for (int j = 0; j < s.Ny; ++j) {
                int ry = 0, rz = 0;
                for (int k = 0; k < s.Nz; ++k) {
                    const size_t idx = (size_t)j * s.Nz + k;
                    const double Iz = F.Iz_inn + (F.Iz_out - F.Iz_inn) * 0.5 * (1 + std::tanh((cyc[idx] / f.d_i - 0.2) / 0.03));
                    const int nz = 2 * (int)std::max(1.0, Iz / cdz[idx]);
                    const double Iy = 0.67 * Iz;
                    const int ny = 2 * (int)std::max(1.0, Iy / cdy[idx]);
                    F.Nz_cell[idx] = nz;
                    F.Ny_cell[idx] = ny;
                    if (k && (nz != F.Nz_cell[idx - 1] || ny != F.Ny_cell[idx - 1])) s.per_cell = true;
                    ry = std::max(ry, ny);
                    rz = std::max(rz, nz);
                    if (!s.coeffs.count(ny)) {
                        std::vector<double> hv(ny + 1);
                        cell_coefficients(ny, hv.data());
                        s.coeffs.emplace(ny, std::move(hv));
                    }
                    if (!s.coeffs.count(nz)) {
                        std::vector<double> hv(nz + 1);
                        cell_coefficients(nz, hv.data());
                        s.coeffs.emplace(nz, std::move(hv));
                    }
                }
                F.Ny_row[j] = ry;
                F.Nz_row[j] = rz;
                F.Ny_max = std::max(F.Ny_max, ry);
                F.Nz_max = std::max(F.Nz_max, rz);
            }
            continue;
        }
        for (int j = 0; j < s.Ny; ++j) {
            int nz, ny;
            if (spec.kind == kPlaneNative) {
                const double Iz = F.Iz_inn + (F.Iz_out - F.Iz_inn) * 0.5 * (1 + std::tanh((s.yc[j] / f.d_i - 0.2) / 0.03));
                nz = 2 * (int)std::max(1.0, Iz / s.dz);
                const double Iy = 0.67 * Iz;
                ny = 2 * (int)std::max(1.0, Iy / s.dy[j]);
            } else {
                nz = ny = synthetic_halfwidth(j, s.Ny, spec.N_min, spec.N_max);
            }
            F.Nz_row[j] = nz;
            F.Ny_row[j] = ny;
            F.Nz_max = std::max(F.Nz_max, nz);
            F.Ny_max = std::max(F.Ny_max, ny);
        }
        for (int j = 0; j < s.Ny; ++j) {
            for (int N : {F.Ny_row[j], F.Nz_row[j]}) {
                if (!s.coeffs.count(N)) {
                    std::vector<double> h(N + 1);
                    cell_coefficients(N, h.data());
                    s.coeffs.emplace(N, std::move(h));
                }
            }
        }
    }
    if (grid && !s.per_cell) // row-uniform grid: the per-row representation is exact
        for (ComponentSetup &F : s.comp) {
            F.Ny_cell.clear();
            F.Nz_cell.clear();
        }
    return true;
}

bool write_csv(const Setup &s, const std::string &path, const double *u, const double *v, const double *w,
               const double *T, const double *rho, int z0, int nz, std::string &err)
{
    FILE *f = std::fopen(path.c_str(), "w");
    if (!f) { err = "cannot open " + path + " for writing"; return false; }
    std::fputs("z,y,u_fluc,v_fluc,w_fluc,T_fluc,rho_fluc\n", f);
    const int W = s.Nz + 1;
    for (int j = 0; j < s.Ny; ++j) {
        const double y0 = s.y_vert[j], y1 = s.y_vert[j + 1];
        double yc = 0.25 * (y0 + y0 + y1 + y1); // n00, n01, n10, n11 (df.cpp:779-785)
        for (int kl = 0; kl < nz; ++kl) {
            const int k = z0 + kl;
            double zc = 0.25 * (s.z_vert[k] + s.z_vert[k + 1] + s.z_vert[k] + s.z_vert[k + 1]);
            if (!s.yv.empty()) { // grid plane: the cell's own four vertices
                const size_t n00 = (size_t)j * W + k, n01 = n00 + 1, n10 = n00 + W, n11 = n10 + 1;
                yc = 0.25 * (s.yv[n00] + s.yv[n01] + s.yv[n10] + s.yv[n11]);
                zc = 0.25 * (s.zv[n00] + s.zv[n01] + s.zv[n10] + s.zv[n11]);
            }
            const size_t c = (size_t)j * nz + kl;
            std::fprintf(f, "%.15f,%.15f,%.15f,%.15f,%.15f,%.15f,%.15f\n", zc, yc, u[c], v[c], w[c], T[c], rho[c]);
        }
    }
    std::fclose(f);
    return true;
}

} // namespace dfamd
