// df.hpp — drop-in C++ API of the MI355X DIGITAL_FILTER.
//
// Same names, members and call sequence as the reference header
// connorswitala/digital-filtering digital-filtering-c++/df/df.hpp:
//   struct FilterField (df.hpp:24-34), struct DFConfig (df.hpp:38-49),
//   class DIGITAL_FILTER (df.hpp:52-125): ctor = setup + step 0, filter(dt),
//   the stage functions, get_rms / plot_rms, the CSV / Tecplot writers.
// Everything runs on the GPU through the C ABI in df_c.h (libdfamd.so); the
// public FilterField vectors are host mirrors refreshed after each call
// (DFConfig::host_mirror), the device copies are reachable zero-copy through
// device_field(). Default (host_mirror 1): u/v/w.fluc, T', rho' after every call with
// one synchronisation into page-locked vectors; filt_old/filt on request (sync_host(), checkpoint())
// or every call with host_mirror 2.
//
// Deliberate differences: DFConfig fields are honoured
// (the reference ignores them; their defaults here are its hard-coded values);
// input paths come from the config instead of "../files/RST.dat" / "../line.dat";
// filter() writes its CSV only when DFConfig::csv_path is set; errors throw
// std::runtime_error instead of printing to cerr and continuing. The RNG stream is
// the reference's: one process-wide stream shared by every object in call order
// (df.cpp:334-335's function-local statics; DFConfig::shared_stream, the default),
// or per object with shared_stream = false.
#pragma once

#include "df_c.h"

#include <chrono>
#include <cmath>
#include <cstdint>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#ifndef DF_NO_USING_STD
using namespace std; // as the reference header does (df.hpp:18)
#endif

#define NOW std::chrono::high_resolution_clock::now();            // df.hpp:15
constexpr double pi_c = -2.0 * 3.14159265358979323846;             // df.hpp:16
typedef std::vector<double> Vector;                                 // df.hpp:19

// Input profiles: DF_DATA_DIR if the build defines it, else the data/ directory installed next to
// libdfamd.so (df_data_dir(); independent of the working directory).
#ifdef DF_DATA_DIR
inline std::string df_default_data_dir() { return DF_DATA_DIR; }
#else
inline std::string df_default_data_dir() { return df_data_dir(); }
#endif

struct FilterField { // df.hpp:24-34
    Vector by, bz, r_ys, r_zs, rms_added, rms, filt_old, filt, fluc;
    std::vector<int> N_ys, N_zs, by_offsets, bz_offsets;
    double Iz_inn = 0, Iz_out = 0, Lt = 0;
    int Nz_max = 0, Ny_max = 0;
};

// The reference's resumable state: the process-wide stream (df.cpp:334-335) and
// filt_old of u, v, w (df.cpp:440-442). restore() on a handle of the same plane continues the
// saved run bit for bit.
struct DFCheckpoint {
    std::uint64_t rng_state = 0;
    int rng_saved_flag = 0;
    double rng_saved = 0.0;
    Vector filt_old_u, filt_old_v, filt_old_w;
};

// The reference draws every object's noise from ONE pcg32 + normal_distribution, function-local
// statics of generate_white_noise (df.cpp:334-335): the first object to draw seeds it, later objects
// continue it in call order (constructor step 0 included). Each handle here owns a device-side copy
// of the stream; with DFConfig::shared_stream the objects of a process hand this one state on: an
// object that draws after another first loads the shared state into its handle (df_set_rng_state).
// The state is read back from the device only when another object needs it (or the holder is
// destroyed), so a single object's filter() pays no per-call state copy.
// Cost and ordering: every switch between objects synchronizes both handles and regenerates the
// prefetched noise of the one that draws next (one noise generation, plus, on an RCCL handle with
// split counting - the table-mode default - its counts all-gather). Multi-rank programs must
// therefore construct their objects and call them in the same order on every rank.
struct DFSharedStream {
    bool seeded = false;
    bool stale = false;          // state/saved are older than the holder's device copy
    std::uint64_t state = 0;
    int saved_flag = 0;
    double saved = 0.0;
    const void *last = nullptr;  // the object whose handle holds the current state
    df_handle *last_h = nullptr; // its handle (read back from it when stale)
    void materialize()
    {
        if (stale && last_h) {
            if (df_rng_state(last_h, &state, &saved_flag, &saved) != DF_OK)
                throw std::runtime_error(std::string("libdfamd: ") + df_last_error());
            stale = false;
        }
    }
};
inline DFSharedStream &df_shared_stream()
{
    static DFSharedStream s; // one per process (inline function: one instance across translation units)
    return s;
}

struct DFConfig { // df.hpp:38-49; defaults = values hard-coded in df.cpp:7-16
    double d_i = 0.0013, rho_e = 0.044, U_e = 869.1, mu_e = 7.1212e-6;
    int vel_file_offset = 0, vel_file_N_values = 0;
    std::string grid_file;                                   // DF_PLANE_GRID: Tecplot BLOCK grid (write_tecplot layout)
    std::string vel_fluc_file = df_default_data_dir() + "/RST.dat"; // RST profile (reference: ../files/RST.dat)
    // ---- extensions
    std::string line_file = df_default_data_dir() + "/line.dat";    // mean profile (reference: ../line.dat)
    std::uint64_t seed = 0;
    bool seed_from_random_device = true;                     // df.cpp:334
    int plane = DF_PLANE_NATIVE;                             // DF_PLANE_SYNTHETIC: Ny x Nz, N in [N_min, N_max]
    int Ny = 0, Nz = 0, N_min = 0, N_max = 0;                // DF_PLANE_GRID: Ny x Nz cells of grid_y/grid_z
    Vector grid_y, grid_z;                                   // DF_PLANE_GRID vertices, (Ny+1)*(Nz+1), j*(Nz+1)+k
    // Drop-in default: the per-N table (bit-identical fields, ~8x faster at c3, no 20-85 GB
    // coefficient stream beside the solver); DF_COEFF_PACKED streams the reference's by/bz.
    int coeff_mode = DF_COEFF_TABLE;
    std::string csv_path;                                    // e.g. "../files/cpp_vel_fluc.csv" (df.cpp:466)
    std::string rms_csv_path = "../files/cpp_vel_fluc_rms.csv"; // df.cpp:623
    int device = 0;
    int rank = 0, world = 1;
    const void *comm_id = nullptr;
    // Host mirrors (the reference's public vectors, df.hpp:28, 59): 1 (default) refreshes u/v/w.fluc,
    // T', rho' after every call - one stream synchronisation, DMA into page-locked vectors; filt_old
    // and filt are refreshed on request (sync_host(), checkpoint()). 2: all of them after every call.
    // 0: never (a GPU-resident solver reads device_field()).
    int host_mirror = 1;
    // With host_mirror 0: filter() returns as soon as the call is enqueued, no host wait at all; the caller
    // orders its own work on stream() (df_stream: launch there, or hipStreamWaitEvent on an event recorded
    // there) - the GPU-resident coupling of us3d_user.f90:80-120. "Filtering took" then times the enqueue.
    bool stream_ordered = false;
    bool pin_mirrors = true;     // page-lock the mirror vectors (hipHostRegister via df_host_pin)
    int mirror_coefficients = -1; // by/bz host copies: 1 always, 0 never, -1 when <= 1 GiB
    bool verbose = true;         // print "Filtering took X seconds." (df.cpp:464)
    bool shared_stream = true;   // one stream for every object of the process, as the reference's statics
                                 // (see DFSharedStream: per-switch cost; same object order on every rank)
    bool resume = false;         // start the stream at (rng_state, rng_saved_flag, rng_saved)
    std::uint64_t rng_state = 0;
    int rng_saved_flag = 0;
    double rng_saved = 0.0;
};

class DIGITAL_FILTER {
  private:
    df_handle *h_ = nullptr;
    DFConfig cfg_;
    int Ny = 0, Nz = 0, n_cells = 0;
    Vector rho_fluc, T_fluc;
    Vector R11, R21, R22, R33;
    int rms_counter = 0;
    double dt = 0.0;
    Vector y, z;               // vertices of this strip, (Ny+1)*(Nz+1), index j*(Nz+1)+k (df.hpp:61)
    Vector Us, Ts, rhos, Ps, Ms;
    double d_i = 0, d_v = 0, u_tau = 0, tau_w = 0;
    Vector T_rms, rho_rms;

    static void check(int rc)
    {
        if (rc != DF_OK) throw std::runtime_error(std::string("libdfamd: ") + df_last_error());
    }
    int comp_of(const FilterField &F) const
    {
        if (&F == &u) return 0;
        if (&F == &v) return 1;
        if (&F == &w) return 2;
        throw std::invalid_argument("FilterField does not belong to this DIGITAL_FILTER");
    }
    Vector row(int which) const
    {
        Vector r(Ny);
        check(df_get_row(h_, which, r.data()));
        return r;
    }
    void pull(Vector &dst, int which)
    {
        dst.resize(n_cells);
        check(df_get_field(h_, which, dst.data()));
    }
    // Page-locked mirrors: each registered range, re-registered when a vector's buffer moved.
    struct Pin {
        const void *p = nullptr;
        size_t bytes = 0;
        const void *refused = nullptr; // the runtime refused this buffer: do not retry every call
    };
    Pin pins_[11];
    void pin(Vector &v, Pin &pn)
    {
        v.resize(n_cells);
        const size_t bytes = v.size() * sizeof(double);
        if (!cfg_.pin_mirrors || bytes == 0 || (pn.p == v.data() && pn.bytes == bytes) || pn.refused == v.data())
            return;
        if (pn.p) df_host_unpin(const_cast<void *>(pn.p));
        pn = Pin{};
        if (df_host_pin(v.data(), bytes) == DF_OK) pn = Pin{v.data(), bytes, nullptr};
        else pn.refused = v.data(); // pageable copies still work, at the runtime's staging rate
    }
    void unpin_all()
    {
        for (Pin &pn : pins_)
            if (pn.p) df_host_unpin(const_cast<void *>(pn.p));
        for (Pin &pn : pins_) pn = Pin{};
    }
    // Every mirror in one df_get_fields: one stream synchronisation per refresh. After apply_RST_scaling
    // the reference's filt equals filt_old (df.cpp:440-442): filt is a second DMA copy of the device
    // filt_old (at PCIe rate, ~2x faster than copying the host vector).
    void refresh_mirrors(bool with_filt_old)
    {
        Vector *dst[11] = {&u.fluc,     &v.fluc,     &w.fluc, &T_fluc, &rho_fluc, &u.filt_old,
                           &v.filt_old, &w.filt_old, &u.filt, &v.filt, &w.filt};
        const int which[11] = {DF_U,          DF_V,          DF_W,          DF_T,          DF_RHO,       DF_FILT_OLD_U,
                               DF_FILT_OLD_V, DF_FILT_OLD_W, DF_FILT_OLD_U, DF_FILT_OLD_V, DF_FILT_OLD_W};
        const int n = with_filt_old ? 11 : 5;
        double *out[11];
        for (int i = 0; i < n; ++i) {
            pin(*dst[i], pins_[i]);
            out[i] = dst[i]->data();
        }
        check(df_get_fields(h_, n, which, out));
    }
    void refresh() // after filter() / get_rms(): the per-call set
    {
        if (cfg_.host_mirror) refresh_mirrors(cfg_.host_mirror >= 2);
    }
    void refresh_full() // construction, stage API, restore: every mirror (not per call)
    {
        if (cfg_.host_mirror) refresh_mirrors(true);
    }
    void fill_field(FilterField &F, int c)
    {
        F.N_ys.resize(n_cells);
        F.N_zs.resize(n_cells);
        F.by_offsets.resize(n_cells);
        F.bz_offsets.resize(n_cells);
        check(df_get_halfwidths(h_, c, 0, F.N_ys.data()));
        check(df_get_halfwidths(h_, c, 1, F.N_zs.data()));
        check(df_get_offsets(h_, c, 0, F.by_offsets.data()));
        check(df_get_offsets(h_, c, 1, F.bz_offsets.data()));
        long long by_size = 0, bz_size = 0;
        check(df_get_comp_info(h_, c, &F.Ny_max, &F.Nz_max, &by_size, &bz_size));
        // integral scales (df.cpp:35-45)
        const double Lt[3] = {0.8, 0.3, 0.3}, Iout[3] = {0.4, 0.3, 0.4}, Iinn[3] = {150, 75, 150};
        F.Lt = Lt[c] * d_i / cfg_.U_e;
        F.Iz_out = Iout[c] * d_i;
        F.Iz_inn = Iinn[c] * d_v;
        const bool mirror = cfg_.mirror_coefficients > 0 ||
                            (cfg_.mirror_coefficients < 0 && 8.0 * (by_size + bz_size) <= 1073741824.0);
        if (mirror) load_coefficients(F);
    }

  public:
    FilterField u, v, w;

    explicit DIGITAL_FILTER(DFConfig config) : cfg_(config)
    {
        df_config_c c;
        df_config_default(&c);
        c.d_i = config.d_i;
        c.rho_e = config.rho_e;
        c.U_e = config.U_e;
        c.mu_e = config.mu_e;
        c.vel_file_offset = config.vel_file_offset;
        c.vel_file_N_values = config.vel_file_N_values;
        c.grid_file = config.grid_file.empty() ? nullptr : config.grid_file.c_str();
        c.grid_y = config.grid_y.empty() ? nullptr : config.grid_y.data();
        c.grid_z = config.grid_z.empty() ? nullptr : config.grid_z.data();
        c.vel_fluc_file = config.vel_fluc_file.c_str();
        c.line_file = config.line_file.c_str();
        c.seed = config.seed;
        c.seed_from_random_device = config.seed_from_random_device ? 1 : 0;
        c.plane = config.plane;
        c.Ny = config.Ny;
        c.Nz = config.Nz;
        c.N_min = config.N_min;
        c.N_max = config.N_max;
        c.coeff_mode = config.coeff_mode;
        c.csv_path = nullptr; // the wrapper writes the CSV itself (write_csv)
        c.device = config.device;
        c.rank = config.rank;
        c.world = config.world;
        c.comm_id = config.comm_id;
        c.rng_resume = config.resume ? 1 : 0;
        c.rng_state = config.rng_state;
        c.rng_saved_flag = config.rng_saved_flag;
        c.rng_saved = config.rng_saved;
        DFSharedStream &ss = df_shared_stream();
        if (config.shared_stream && !config.resume && ss.seeded) { // step 0 continues the process's stream
            ss.materialize();
            c.rng_resume = 1;
            c.rng_state = ss.state;
            c.rng_saved_flag = ss.saved_flag;
            c.rng_saved = ss.saved;
        }
        h_ = df_create(&c);
        if (!h_) throw std::runtime_error(std::string("DIGITAL_FILTER: ") + df_last_error());
        try {
            stream_out(); // step 0 drew from the stream
            mirror_setup();
        } catch (...) { // the destructor does not run for a half-built object
            df_destroy(h_);
            h_ = nullptr;
            throw;
        }
    }
    DIGITAL_FILTER(const DIGITAL_FILTER &) = delete;
    DIGITAL_FILTER &operator=(const DIGITAL_FILTER &) = delete;
    ~DIGITAL_FILTER()
    {
        DFSharedStream &ss = df_shared_stream();
        if (ss.last == this) { // publish the state before the handle that holds it goes
            try {
                ss.materialize();
            } catch (...) {
            }
            ss.last = nullptr;
            ss.last_h = nullptr;
        }
        unpin_all();
        df_destroy(h_);
    }

  private:
    // Shared stream (DFConfig::shared_stream): load the process's state before a draw unless this
    // handle already holds it, publish the state after.
    void stream_in()
    {
        DFSharedStream &ss = df_shared_stream();
        if (!cfg_.shared_stream || !ss.seeded || ss.last == this) return;
        ss.materialize();
        check(df_set_rng_state(h_, ss.state, ss.saved_flag, ss.saved));
        ss.last = this;
        ss.last_h = h_;
    }
    void stream_out() // this handle now holds the process's stream; read back lazily (materialize)
    {
        if (!cfg_.shared_stream) return;
        DFSharedStream &ss = df_shared_stream();
        ss.seeded = true;
        ss.stale = true;
        ss.last = this;
        ss.last_h = h_;
    }
    // Host mirrors of the setup (rows, scalars, vertices, half-widths) and of step 0's fields.
    void mirror_setup()
    {
        int ny, nz, z0, z1;
        check(df_dims(h_, &ny, &nz, &z0, &z1));
        Ny = ny;
        Nz = z1 - z0;
        n_cells = Ny * Nz;
        d_i = cfg_.d_i;
        d_v = df_get_scalar(h_, 2);
        u_tau = df_get_scalar(h_, 0);
        tau_w = df_get_scalar(h_, 1);
        R11 = row(DF_ROW_R11);
        R21 = row(DF_ROW_R21);
        R22 = row(DF_ROW_R22);
        R33 = row(DF_ROW_R33);
        Us = row(DF_ROW_US);
        Ts = row(DF_ROW_TS);
        rhos = row(DF_ROW_RHOS);
        Ps = row(DF_ROW_PS);
        Ms = row(DF_ROW_MS);
        {
            Vector gy((size_t)(Ny + 1) * (nz + 1)), gz(gy.size());
            check(df_get_grid(h_, gy.data(), gz.data()));
            y.resize((size_t)(Ny + 1) * (Nz + 1));
            z.resize(y.size());
            for (int j = 0; j <= Ny; ++j)
                for (int k = 0; k <= Nz; ++k) {
                    y[(size_t)j * (Nz + 1) + k] = gy[(size_t)j * (nz + 1) + z0 + k];
                    z[(size_t)j * (Nz + 1) + k] = gz[(size_t)j * (nz + 1) + z0 + k];
                }
        }
        fill_field(u, 0);
        fill_field(v, 1);
        fill_field(w, 2);
        rho_fluc.assign(n_cells, 0.0);
        T_fluc.assign(n_cells, 0.0);
        refresh_full();
    }

  public:
    // ====== setup steps: performed by the constructor (df.cpp:26-53); kept for API parity
    void read_grid() {}
    void allocate_data_structures(FilterField &F) { (void)comp_of(F); }
    void calculate_filter_properties(FilterField &F) { fill_field(F, comp_of(F)); }
    void get_RST_in() {}
    void read_line_file() {}

    // ====== hot path (df.cpp:332-485), on the GPU
    void generate_white_noise()
    {
        stream_in();
        check(df_generate_white_noise(h_));
        stream_out();
    }
    void filtering_sweeps(FilterField &F)
    {
        const int c = comp_of(F);
        check(df_filtering_sweeps(h_, c));
        if (cfg_.host_mirror) pull(F.filt, DF_FILT_U + c);
    }
    void correlate_fields(FilterField &F)
    {
        const int c = comp_of(F);
        check(df_correlate_fields(h_, c, dt));
        if (cfg_.host_mirror) pull(F.filt, DF_FILT_U + c);
    }
    void apply_RST_scaling()
    {
        check(df_apply_RST_scaling(h_));
        refresh_full();
    }
    void get_rho_T_fluc()
    {
        check(df_get_rho_T_fluc(h_));
        refresh_full();
    }
    void filter(double dt_input)
    {
        dt = dt_input;
        stream_in();
        auto start = NOW;
        check(df_filter(h_, dt));
        // the fields of this call, not the noise and y-passes already queued for later calls (df_wait)
        if (!(cfg_.stream_ordered && cfg_.host_mirror == 0)) check(df_wait(h_));
        auto end = NOW;
        stream_out();
        if (cfg_.verbose) {
            auto elapsed = std::chrono::duration<double>(end - start);
            std::cout << "Filtering took " << elapsed.count() << " seconds." << std::endl;
        }
        refresh();
        if (!cfg_.csv_path.empty()) write_csv(cfg_.csv_path);
    }

    // ====== debugging (df.cpp:557-561)
    void display_data(Vector &vec)
    {
        for (auto val : vec) std::cout << val << std::endl;
    }

    // ====== RMS (df.cpp:566-675), accumulated on the GPU
    void allocate_rms_structures(FilterField &F)
    {
        F.rms_added.assign(n_cells, 0.0);
        F.rms.assign(n_cells, 0.0);
    }
    void rms_add()
    {
        if (rms_counter == 0 && df_rms_count(h_) != 0) check(df_rms_reset(h_));
        check(df_rms_add(h_));
        rms_counter++;
    }
    void get_rms()
    {
        allocate_rms_structures(u);
        allocate_rms_structures(v);
        allocate_rms_structures(w);
        check(df_rms_reset(h_));
        rms_counter = 0;
        dt = 1e-5; // df.cpp:594
        stream_in();
        for (int i = 0; i < 500; ++i) {
            check(df_filter(h_, dt)); // noise, sweeps, correlate, RST, SRA (df.cpp:597-605)
            check(df_rms_add(h_));
            rms_counter++;
        }
        check(df_wait(h_));
        stream_out();
        refresh();
        plot_rms();
    }
    void plot_rms()
    {
        u.rms.resize(n_cells);
        v.rms.resize(n_cells);
        w.rms.resize(n_cells);
        T_rms.resize(n_cells);
        rho_rms.resize(n_cells);
        check(df_rms_get(h_, DF_U, u.rms.data()));
        check(df_rms_get(h_, DF_V, v.rms.data()));
        check(df_rms_get(h_, DF_W, w.rms.data()));
        check(df_rms_get(h_, DF_T, T_rms.data()));
        check(df_rms_get(h_, DF_RHO, rho_rms.data()));
        const std::string filename = cfg_.rms_csv_path;
        std::ofstream file(filename);
        file << "z, y, u'_rms, v'_rms, w'_rms, T'_rms, rho'_rms \n";
        for (int j = 0; j < Ny; ++j)
            for (int k = 0; k < Nz; ++k) {
                const int idx = j * Nz + k;
                const int iidx = j * (Nz + 1) + k; // df.cpp:634-636
                file << z[iidx] << ", " << y[iidx] << ", " << u.rms[idx] << ", " << v.rms[idx] << ", " << w.rms[idx]
                     << ", " << T_rms[idx] << ", " << rho_rms[idx] << std::endl;
            }
        file.close();
        std::cout << "Finished plotting to file: " << filename << std::endl;
    }

    // ====== writers (df.cpp:677-803)
    void write_tecplot(const std::string &filename)
    {
        std::ofstream file(filename);
        file << "VARIABLES = \"z\", \"y\", \"u_fluc\", \"v_fluc\", \"w_fluc\" \n";
        file << "ZONE T=\"Flow Field\", I=" << Nz + 1 << ", J=" << Ny + 1 << ", F=BLOCK\n";
        file << "VARLOCATION=([3-5]=CELLCENTERED)\n";
        for (int j = 0; j < Ny + 1; ++j)
            for (int k = 0; k < Nz + 1; ++k) file << z[j * (Nz + 1) + k] << std::endl;
        for (int j = 0; j < Ny + 1; ++j)
            for (int k = 0; k < Nz + 1; ++k) file << y[j * (Nz + 1) + k] << std::endl;
        for (const Vector *f : {&u.fluc, &v.fluc, &w.fluc})
            for (int idx = 0; idx < n_cells; ++idx) file << (*f)[idx] << std::endl;
        file.close();
        std::cout << "Finished plotting." << std::endl;
    }
    void plot_RST_lerp()
    {
        std::ofstream file("../files/myRST.csv");
        file << "y, R11, R21, R22, R33 \n";
        const Vector yc = row(DF_ROW_YC);
        for (int j = 0; j < Ny; ++j)
            file << yc[j] << ", " << ", " << R11[j] << ", " << R21[j] << ", " << R22[j] << ", " << R33[j] << std::endl;
        file.close();
        std::ifstream fin(cfg_.vel_fluc_file);
        std::ofstream file1("../files/duanRST.csv");
        file1 << "y_d, R11_in, R21_in, R22_in, R33_in \n";
        std::string line;
        std::getline(fin, line);
        std::getline(fin, line);
        while (std::getline(fin, line)) {
            if (line.empty()) continue;
            std::istringstream iss(line);
            std::vector<double> val;
            double x;
            while (iss >> x) val.push_back(x);
            if (val.size() < 6) continue;
            file1 << val[0] << ", " << val[2] * val[2] * u_tau * u_tau << ", " << val[5] * u_tau * u_tau << ", "
                  << val[3] * val[3] * u_tau * u_tau << ", " << val[4] * val[4] * u_tau * u_tau << std::endl;
        }
        std::cout << "Finished plotting RST to file. " << std::endl;
    }
    void write_csv(const std::string &filename)
    {
        std::ofstream file(filename, std::ios::trunc);
        if (!file) {
            std::cerr << "Error: cannot open " << filename << " for writing.\n";
            return;
        }
        file << "z,y,u_fluc,v_fluc,w_fluc,T_fluc,rho_fluc\n";
        file << std::setprecision(15) << std::fixed;
        for (int j = 0; j < Ny; ++j)
            for (int k = 0; k < Nz; ++k) {
                const int n00 = j * (Nz + 1) + k, n01 = n00 + 1, n10 = n00 + Nz + 1, n11 = n10 + 1; // df.cpp:775-785
                const double yc = 0.25 * (y[n00] + y[n01] + y[n10] + y[n11]);
                const double zc = 0.25 * (z[n00] + z[n01] + z[n10] + z[n11]);
                const int c = j * Nz + k;
                file << zc << "," << yc << "," << u.fluc[c] << "," << v.fluc[c] << "," << w.fluc[c] << ","
                     << T_fluc[c] << "," << rho_fluc[c] << "\n";
            }
        file.close();
        std::cout << "CSV written to " << filename << "\n";
    }

    Vector linear_interpolate(const std::vector<double> &y_data, const std::vector<double> &f_data,
                              const std::vector<double> &y_new)
    { // df.cpp:805-848
        if (y_data.size() != f_data.size()) throw std::invalid_argument("y_data and f_data must be the same size.");
        if (y_data.size() < 2) throw std::invalid_argument("Need at least two data points to interpolate.");
        std::vector<double> f_new(y_new.size());
        for (size_t j = 0; j < y_new.size(); ++j) {
            const double y = y_new[j];
            if (y <= y_data.front()) { f_new[j] = f_data.front(); continue; }
            if (y >= y_data.back()) { f_new[j] = f_data.back(); continue; }
            size_t i = 0;
            while (i + 1 < y_data.size() && y > y_data[i + 1]) ++i;
            f_new[j] = f_data[i] + (f_data[i + 1] - f_data[i]) * ((y - y_data[i]) / (y_data[i + 1] - y_data[i]));
        }
        return f_new;
    }

    // ====== MI355X extensions
    df_handle *handle() { return h_; }
    // The HIP stream (hipStream_t) every result is written on (DFConfig::stream_ordered), and the two waits:
    // wait() = this object's results so far (df_wait), sync() = every queued call's work (df_sync).
    void *stream() { return df_stream(h_); }
    void wait() { check(df_wait(h_)); }
    void sync() { check(df_sync(h_)); }
    void set_stream_ordered(bool on) { cfg_.stream_ordered = on; }
    // Refresh every host mirror now (filt_old and filt included), whatever host_mirror says.
    void sync_host() { refresh_mirrors(true); }
    void set_host_mirror(int level) { cfg_.host_mirror = level; }
    const double *device_field(int which) { return df_device_field(h_, which); } // zero-copy for a GPU CFD
    const Vector &T_fluc_host() const { return T_fluc; }
    const Vector &rho_fluc_host() const { return rho_fluc; }
    void load_coefficients(FilterField &F)
    {
        const int c = comp_of(F);
        long long by_size = 0, bz_size = 0;
        check(df_get_comp_info(h_, c, nullptr, nullptr, &by_size, &bz_size));
        F.by.resize(by_size);
        F.bz.resize(bz_size);
        check(df_get_coeffs(h_, c, 0, F.by.data(), by_size));
        check(df_get_coeffs(h_, c, 1, F.bz.data(), bz_size));
    }
    void load_noise(FilterField &F)
    {
        const int c = comp_of(F);
        F.r_ys.resize((size_t)(Ny + 2 * F.Ny_max) * Nz);
        F.r_zs.resize((size_t)Ny * (Nz + 2 * F.Nz_max));
        check(df_get_noise(h_, c, 0, F.r_ys.data(), (long long)F.r_ys.size()));
        check(df_get_noise(h_, c, 1, F.r_zs.data(), (long long)F.r_zs.size()));
    }
    void rng_state(std::uint64_t &state, int &saved_flag, double &saved)
    {
        check(df_rng_state(h_, &state, &saved_flag, &saved));
    }
    DFCheckpoint checkpoint()
    {
        DFCheckpoint ck;
        rng_state(ck.rng_state, ck.rng_saved_flag, ck.rng_saved);
        pull(ck.filt_old_u, DF_FILT_OLD_U);
        pull(ck.filt_old_v, DF_FILT_OLD_V);
        pull(ck.filt_old_w, DF_FILT_OLD_W);
        return ck;
    }
    void restore(const DFCheckpoint &ck)
    {
        for (const Vector *f : {&ck.filt_old_u, &ck.filt_old_v, &ck.filt_old_w})
            if ((int)f->size() != n_cells) throw std::invalid_argument("checkpoint is for another plane");
        check(df_set_rng_state(h_, ck.rng_state, ck.rng_saved_flag, ck.rng_saved));
        stream_out(); // the restored state is the process's stream from here on
        check(df_set_field(h_, DF_FILT_OLD_U, ck.filt_old_u.data()));
        check(df_set_field(h_, DF_FILT_OLD_V, ck.filt_old_v.data()));
        check(df_set_field(h_, DF_FILT_OLD_W, ck.filt_old_w.data()));
        refresh_full();
    }
};
