// Drop-in counterpart of the reference driver digital-filtering-c++/test/cpp-main.cpp:
// the same three lines (DFConfig, DIGITAL_FILTER df(config), df.get_rms()), built
// against include/df.hpp + libdfamd.so instead of df.cpp.
//
//   cpp-test                      native grid, like the reference (get_rms: 500 x filter(1e-5))
//   cpp-test filter N dt          N x filter(dt), prints sum(u'^2)
//   cpp-test synth Ny Nz Nmin Nmax seed steps [csv [ordered]]   synthetic plane, writes u'/v'/w'/T'/rho' CSV;
//                                 ordered: host_mirror 0 + stream_ordered (no host wait per call), one
//                                 wait() and mirror refresh before the CSV
//   cpp-test rms seed             native grid, seeded, get_rms() -> ../files/cpp_vel_fluc_rms.csv
//   cpp-test writers seed dt steps out   native grid, steps x filter(dt), then write_tecplot(out) and
//                                 plot_RST_lerp() -> ../files/myRST.csv, ../files/duanRST.csv
//   cpp-test twin Ny Nz Nmin Nmax seed steps csvA csvB   two objects on the process's one stream
//                                 (df.cpp:334-335): A then B constructed, filter calls alternating
//   cpp-test time native|synth Ny Nz Nmin Nmax packed|table calls   one JSON line: wall ms per call
//                                 of the C-ABI call (df_filter + df_wait: this call's fields; and + df_sync:
//                                 everything queued, later calls' noise included) and of
//                                 DIGITAL_FILTER::filter() with host_mirror 0, 1, 2 on the same object, and
//                                 the y-pass-ahead setting flipped (bench.py `dropin`)
#include "df.hpp"

#include <cstdlib>

static int time_dropin(char **argv)
{
    DFConfig config;
    config.plane = std::string(argv[2]) == "native" ? DF_PLANE_NATIVE : DF_PLANE_SYNTHETIC;
    config.Ny = std::atoi(argv[3]);
    config.Nz = std::atoi(argv[4]);
    config.N_min = std::atoi(argv[5]);
    config.N_max = std::atoi(argv[6]);
    config.coeff_mode = std::string(argv[7]) == "packed" ? DF_COEFF_PACKED : DF_COEFF_TABLE;
    const int calls = std::atoi(argv[8]);
    config.seed = 42;
    config.seed_from_random_device = false;
    config.verbose = false;
    config.mirror_coefficients = 0;
    DIGITAL_FILTER df(config);
    df_handle *h = df.handle();
    int ny, nz, z0, z1;
    df_dims(h, &ny, &nz, &z0, &z1);
    const double cells = (double)ny * (z1 - z0);
    auto wall = [&](auto &&call) {
        for (int i = 0; i < 5; ++i) call();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < calls; ++i) call();
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double, std::milli>(t1 - t0).count() / calls;
    };
    auto ok = [](int rc) {
        if (rc != DF_OK) throw std::runtime_error(df_last_error());
    };
    const double capi_async = wall([&] { ok(df_filter(h, 1e-8)); }) ; // queue only; the sync below drains
    ok(df_sync(h));
    const double capi_sync = wall([&] { ok(df_filter(h, 1e-8)); ok(df_sync(h)); });
    const double capi = wall([&] { ok(df_filter(h, 1e-8)); ok(df_wait(h)); });
    // the same per-call wait with the y-pass-ahead setting flipped (its default is decided on this figure)
    int ahead = 0;
    ok(df_get_tuning(h, "ypass_ahead", &ahead));
    ok(df_set_tuning(h, "ypass_ahead", !ahead));
    const double capi_flip = wall([&] { ok(df_filter(h, 1e-8)); ok(df_wait(h)); });
    ok(df_set_tuning(h, "ypass_ahead", ahead));
    ok(df_sync(h));
    double dropin[3];
    for (int m = 0; m < 3; ++m) {
        df.set_host_mirror(m);
        dropin[m] = wall([&] { df.filter(1e-8); });
    }
    df.set_host_mirror(0);
    df.set_stream_ordered(true); // no host wait: the caller orders its work on df.stream()
    const double ordered = wall([&] { df.filter(1e-8); });
    df.sync();
    df.set_stream_ordered(false);
    std::cout << std::setprecision(6) << "{\"plane\": \"" << argv[2] << "\", \"Ny\": " << ny << ", \"Nz\": " << nz
              << ", \"coeff_mode\": \"" << argv[7] << "\", \"calls\": " << calls
              << ", \"capi_ms\": " << capi << ", \"capi_sync_all_ms\": " << capi_sync << ", \"capi_async_ms\": " << capi_async
              << ", \"ypass_ahead\": " << ahead << ", \"capi_ms_ypass_ahead_flipped\": " << capi_flip
              << ", \"dropin_ms\": {\"mirror0\": " << dropin[0] << ", \"mirror1\": " << dropin[1]
              << ", \"mirror2\": " << dropin[2] << ", \"mirror0_stream_ordered\": " << ordered
              << "}, \"mirror_bytes\": {\"mirror1\": " << 5 * 8 * cells
              << ", \"mirror2\": " << 11 * 8 * cells << "}}" << std::endl;
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 9 && std::string(argv[1]) == "time") return time_dropin(argv);

    // Create configuration struct
    DFConfig config;
    if (argc > 1 && std::string(argv[1]) == "synth" && argc >= 8) {
        config.plane = DF_PLANE_SYNTHETIC;
        config.Ny = std::atoi(argv[2]);
        config.Nz = std::atoi(argv[3]);
        config.N_min = std::atoi(argv[4]);
        config.N_max = std::atoi(argv[5]);
        config.seed = std::strtoull(argv[6], nullptr, 10);
        config.seed_from_random_device = false;
        const bool ordered = argc > 9 && std::string(argv[9]) == "ordered";
        if (ordered) {
            config.host_mirror = 0;
            config.stream_ordered = true;
        }
        DIGITAL_FILTER df(config);
        const int steps = std::atoi(argv[7]);
        for (int s = 0; s < steps; ++s) df.filter(1e-8);
        if (ordered) {
            df.wait();
            df.sync_host();
        }
        df.write_csv(argc > 8 ? argv[8] : "cpp_vel_fluc.csv");
        return 0;
    }

    if (argc >= 2 && std::string(argv[1]) == "remirror") {
        // the host mirrors are the public vectors (df.hpp:28, 59), page-locked by the wrapper. A
        // caller may move, swap or re-allocate them between calls; every later refresh must land in the
        // vector the caller holds then. Checked against a fresh df_get_field copy after each call.
        config.plane = DF_PLANE_SYNTHETIC;
        config.Ny = 96;
        config.Nz = 300;
        config.N_min = 2;
        config.N_max = 12;
        config.seed = 5;
        config.seed_from_random_device = false;
        config.verbose = false;
        DIGITAL_FILTER df(config);
        const size_t n = df.u.fluc.size();
        int bad = 0;
        auto check = [&](int step) {
            const std::pair<Vector *, int> m[5] = {{&df.u.fluc, DF_U}, {&df.v.fluc, DF_V}, {&df.w.fluc, DF_W},
                                                   {nullptr, DF_T}, {nullptr, DF_RHO}};
            for (const auto &p : m) {
                if (!p.first) continue;
                Vector ref(n);
                if (df_get_field(df.handle(), p.second, ref.data()) != DF_OK || *p.first != ref) {
                    std::cerr << "mirror of field " << p.second << " stale after step " << step << std::endl;
                    ++bad;
                }
            }
        };
        df.filter(1e-8);
        check(0);
        for (int step = 1; step <= 6; ++step) {
            switch (step % 3) {
            case 1: df.u.fluc = Vector(n, 7.0); break; // move-assign: a new buffer, the pinned one freed
            case 2: {
                Vector other(n, -3.0);
                std::swap(df.v.fluc, other); // the pinned buffer now belongs to `other`, freed at scope end
                break;
            }
            default:
                df.w.fluc.clear(); // freed and re-allocated at the same size: often the same address
                df.w.fluc.shrink_to_fit();
                df.w.fluc.resize(n, 1.0);
            }
            df.filter(1e-8);
            check(step);
        }
        std::cout << "remirror " << (bad ? "FAILED" : "ok") << " (" << bad << " stale mirrors)" << std::endl;
        return bad ? 1 : 0;
    }

    if (argc >= 10 && std::string(argv[1]) == "twin") {
        config.plane = DF_PLANE_SYNTHETIC;
        config.Ny = std::atoi(argv[2]);
        config.Nz = std::atoi(argv[3]);
        config.N_min = std::atoi(argv[4]);
        config.N_max = std::atoi(argv[5]);
        config.seed = std::strtoull(argv[6], nullptr, 10);
        config.seed_from_random_device = false;
        DIGITAL_FILTER a(config);
        DIGITAL_FILTER b(config); // continues the stream a's step 0 left (the reference's statics)
        const int steps = std::atoi(argv[7]);
        for (int s = 0; s < steps; ++s) {
            a.filter(1e-8);
            b.filter(1e-8);
        }
        a.write_csv(argv[8]);
        b.write_csv(argv[9]);
        return 0;
    }

    if (argc > 5 && std::string(argv[1]) == "writers") {
        config.seed = std::strtoull(argv[2], nullptr, 10);
        config.seed_from_random_device = false;
        DIGITAL_FILTER df(config);
        const int steps = std::atoi(argv[4]);
        for (int s = 0; s < steps; ++s) df.filter(std::atof(argv[3]));
        df.write_tecplot(argv[5]);
        df.plot_RST_lerp();
        return 0;
    }

    if (argc > 2 && std::string(argv[1]) == "rms") {
        config.seed = std::strtoull(argv[2], nullptr, 10);
        config.seed_from_random_device = false;
    }

    // Constructor
    DIGITAL_FILTER df(config);

    if (argc > 1 && std::string(argv[1]) == "filter") {
        const int n = argc > 2 ? std::atoi(argv[2]) : 1;
        const double dt = argc > 3 ? std::atof(argv[3]) : 1e-5;
        for (int i = 0; i < n; ++i) df.filter(dt);
        double s = 0;
        for (double x : df.u.fluc) s += x * x;
        std::cout << "sum u'^2 = " << s << std::endl;
        return 0;
    }
    // Call filter procedure with timestep (as in the reference driver)
    double dt = 1e-5;
    (void)dt;
    df.get_rms();
    return 0;
}
