"""Python view of libdfamd.so (include/df_c.h) — the MI355X DIGITAL_FILTER.

Mirrors the reference C++ API (digital-filtering-c++/df/df.hpp): construct with a
DFConfig-like set of keyword arguments (the constructor runs setup + step 0,
df.cpp:4-66), call ``filter(dt)`` per timestep (df.cpp:449-468), read ``u.fluc``
etc. through ``field()``. Every call goes through the C ABI into HIP kernels;
there is no CPU fallback: a missing library or GPU raises.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# DFAMD_LIB: another build of the library, for same-box A/B timing (tools/lib_ab.sh)
LIB_PATH = os.environ.get("DFAMD_LIB") or os.path.join(HERE, "libdfamd.so")
DATA = os.path.join(HERE, "data")
HEADER = os.path.join(os.path.dirname(HERE), "include", "df_c.h")

PLANE = {"native": 0, "synthetic": 1, "grid": 2}
DEVICE_TRACE = -2  # df_c.h DF_DEVICE_TRACE: the noise pipeline's host logic, recorded instead of run (df_trace)
COEFF = {"packed": 0, "table": 1}
FIELDS = {"u": 0, "v": 1, "w": 2, "T": 3, "rho": 4, "filt_old_u": 5, "filt_old_v": 6, "filt_old_w": 7,
          "filt_u": 8, "filt_v": 9, "filt_w": 10}
ROWS = {"R11": 0, "R21": 1, "R22": 2, "R33": 3, "Us": 4, "Ts": 5, "rhos": 6, "Ms": 7, "Ps": 8, "yc": 9, "yc_d": 10}


class DFError(RuntimeError):
    pass


class _Cfg(C.Structure):
    _fields_ = [
        ("d_i", C.c_double), ("rho_e", C.c_double), ("U_e", C.c_double), ("mu_e", C.c_double),
        ("vel_file_offset", C.c_int), ("vel_file_N_values", C.c_int),
        ("grid_file", C.c_char_p), ("vel_fluc_file", C.c_char_p),
        ("line_file", C.c_char_p), ("seed", C.c_uint64), ("seed_from_random_device", C.c_int),
        ("plane", C.c_int), ("Ny", C.c_int), ("Nz", C.c_int), ("N_min", C.c_int), ("N_max", C.c_int),
        ("coeff_mode", C.c_int), ("csv_path", C.c_char_p), ("device", C.c_int),
        ("rank", C.c_int), ("world", C.c_int), ("comm_id", C.c_void_p), ("rows_per_wave", C.c_int),
        ("rng_resume", C.c_int), ("rng_saved_flag", C.c_int), ("rng_state", C.c_uint64), ("rng_saved", C.c_double),
        ("grid_y", C.c_void_p), ("grid_z", C.c_void_p),
    ]


class CommStats(C.Structure):
    _fields_ = [("rccl_ranks", C.c_int), ("rccl_rank", C.c_int), ("halo_peers", C.c_int), ("rng_collective", C.c_int),
                ("halo_bytes_sent", C.c_longlong), ("rng_bytes_received", C.c_longlong),
                ("rng_blocks_counted", C.c_longlong), ("rng_blocks_total", C.c_longlong)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Profile(C.Structure):
    _fields_ = [("calls", C.c_longlong), ("rng_ms", C.c_double), ("ypass_ms", C.c_double),
                ("halo_ms", C.c_double), ("zpass_ms", C.c_double), ("total_ms", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib():
    """Load libdfamd.so (fails loudly: the HIP path is the only path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DFError(f"{LIB_PATH} is not built; run `make -C digital-filtering_amd` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    H = C.c_void_p
    sig = {
        "df_abi_version": (C.c_int, []),
        "df_last_error": (C.c_char_p, []),
        "df_config_default": (None, [C.POINTER(_Cfg)]),
        "df_data_dir": (C.c_char_p, []),
        "df_create": (H, [C.POINTER(_Cfg)]),
        "df_create_group": (C.c_int, [C.POINTER(_Cfg), C.c_int, C.POINTER(H)]),
        "df_filter": (C.c_int, [H, C.c_double]),
        "df_filter_group": (C.c_int, [C.POINTER(H), C.c_int, C.c_double]),
        "df_generate_white_noise": (C.c_int, [H]),
        "df_filtering_sweeps": (C.c_int, [H, C.c_int]),
        "df_correlate_fields": (C.c_int, [H, C.c_int, C.c_double]),
        "df_apply_RST_scaling": (C.c_int, [H]),
        "df_get_rho_T_fluc": (C.c_int, [H]),
        "df_get_field": (C.c_int, [H, C.c_int, C.c_void_p]),
        "df_device_field": (C.c_void_p, [H, C.c_int]),
        "df_set_field": (C.c_int, [H, C.c_int, C.c_void_p]),
        "df_dims": (C.c_int, [H] + [C.POINTER(C.c_int)] * 4),
        "df_get_row": (C.c_int, [H, C.c_int, C.c_void_p]),
        "df_get_scalar": (C.c_double, [H, C.c_int]),
        "df_get_halfwidths": (C.c_int, [H, C.c_int, C.c_int, C.c_void_p]),
        "df_get_offsets": (C.c_int, [H, C.c_int, C.c_int, C.c_void_p]),
        "df_get_comp_info": (C.c_int, [H, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                       C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
        "df_get_coeffs": (C.c_int, [H, C.c_int, C.c_int, C.c_void_p, C.c_longlong]),
        "df_rng_state": (C.c_int, [H, C.POINTER(C.c_uint64), C.POINTER(C.c_int), C.POINTER(C.c_double)]),
        "df_set_rng_state": (C.c_int, [H, C.c_uint64, C.c_int, C.c_double]),
        "df_stream_length": (C.c_longlong, [H]),
        "df_get_noise": (C.c_int, [H, C.c_int, C.c_int, C.c_void_p, C.c_longlong]),
        "df_rms_reset": (C.c_int, [H]),
        "df_rms_add": (C.c_int, [H]),
        "df_rms_get": (C.c_int, [H, C.c_int, C.c_void_p]),
        "df_rms_count": (C.c_longlong, [H]),
        "df_get_vertices": (C.c_int, [H, C.c_void_p, C.c_void_p]),
        "df_get_grid": (C.c_int, [H, C.c_void_p, C.c_void_p]),
        "df_plane_info": (C.c_int, [H, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "df_set_profiling": (C.c_int, [H, C.c_int]),
        "df_set_tuning": (C.c_int, [H, C.c_char_p, C.c_int]),
        "df_get_tuning": (C.c_int, [H, C.c_char_p, C.POINTER(C.c_int)]),
        "df_gather_field": (C.c_int, [H, C.c_int, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p, C.c_longlong,
                                      C.c_double]),
        "df_get_profile": (C.c_int, [H, C.POINTER(Profile)]),
        "df_sync": (C.c_int, [H]),
        "df_wait": (C.c_int, [H]),
        "df_stream": (C.c_void_p, [H]),
        "df_algorithmic_bytes": (C.c_double, [H, C.c_int]),
        "df_comm_unique_id": (C.c_int, [C.c_void_p, C.c_size_t]),
        "df_comm_info": (C.c_int, [H, C.POINTER(CommStats)]),
        "df_trace": (C.c_longlong, [H, C.c_void_p, C.c_longlong]),
        "df_destroy": (None, [H]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def header_symbols():
    """Function names declared in include/df_c.h (for the export test)."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?[\s\*])(df_\w+)\s*\(", txt, re.M)))


def _check(rc):
    if rc != 0:
        raise DFError(f"libdfamd error {rc}: {lib().df_last_error().decode()}")


def comm_unique_id():
    buf = C.create_string_buffer(128)
    _check(lib().df_comm_unique_id(buf, 128))
    return buf.raw


def make_config(plane="native", Ny=0, Nz=0, N_min=0, N_max=0, seed=None, coeff_mode="packed", device=0,
                rank=0, world=1, comm_id=None, csv_path=None, rows_per_wave=0, rst_file=None, line_file=None,
                d_i=None, rho_e=None, U_e=None, mu_e=None, resume=None, grid_y=None, grid_z=None, grid_file=None):
    """resume = (pcg state, saved_flag, saved): start the stream there instead of seeding.
    plane="grid": grid_y / grid_z vertex arrays of shape (Ny+1, Nz+1) (Ny, Nz cells), or grid_file.

    coeff_mode defaults to "packed" here, NOT to df_config_default's DF_COEFF_TABLE: this mirror
    serves the tests and bench.py, which exercise the reference's offset-packed data contract (the
    HBM roofline point). The fields are bit-identical either way, but the launch plan follows the
    mode: packed replicates the RNG counting (halo = the only collective), allocates the 20-85 GB
    coefficient stream and uses the row-pair y-pass on long chains; table splits the counting (one
    all-gather of counts per call) and allocates no stream. Pass coeff_mode="table" to get the
    C/C++/Fortran drop-in default."""
    cfg = _Cfg()
    lib().df_config_default(C.byref(cfg))
    keep = []

    def cstr(s):
        b = s.encode()
        keep.append(b)
        return b

    for k, v in (("d_i", d_i), ("rho_e", rho_e), ("U_e", U_e), ("mu_e", mu_e)):
        if v is not None:
            setattr(cfg, k, v)
    cfg.vel_fluc_file = cstr(rst_file or os.path.join(DATA, "RST.dat"))
    cfg.line_file = cstr(line_file or os.path.join(DATA, "line.dat"))
    if seed is None:
        cfg.seed_from_random_device = 1
    else:
        cfg.seed_from_random_device = 0
        cfg.seed = seed
    cfg.plane = PLANE[plane]
    cfg.Ny, cfg.Nz, cfg.N_min, cfg.N_max = Ny, Nz, N_min, N_max
    if grid_y is not None:
        gy = np.ascontiguousarray(grid_y, dtype=np.float64)
        gz = np.ascontiguousarray(grid_z, dtype=np.float64)
        if gy.ndim == 2 and not (Ny or Nz):
            cfg.Ny, cfg.Nz = gy.shape[0] - 1, gy.shape[1] - 1
        if gy.size != (cfg.Ny + 1) * (cfg.Nz + 1) or gz.size != gy.size:
            raise DFError("grid_y/grid_z must hold (Ny+1)*(Nz+1) vertices")
        keep += [gy, gz]
        cfg.grid_y, cfg.grid_z = gy.ctypes.data, gz.ctypes.data
    if grid_file:
        cfg.grid_file = cstr(grid_file)
    cfg.coeff_mode = COEFF[coeff_mode]
    cfg.csv_path = cstr(csv_path) if csv_path else None
    cfg.device, cfg.rank, cfg.world = device, rank, world
    if comm_id is not None:
        idbuf = C.create_string_buffer(bytes(comm_id), 128)
        keep.append(idbuf)
        cfg.comm_id = C.cast(idbuf, C.c_void_p)
    cfg.rows_per_wave = rows_per_wave
    if resume is not None:
        cfg.rng_resume = 1
        cfg.rng_state, cfg.rng_saved_flag, cfg.rng_saved = int(resume[0]), int(resume[1]), float(resume[2])
    return cfg, keep


class DigitalFilter:
    """DIGITAL_FILTER(DFConfig): setup + constructor step 0 on the GPU."""

    # keys that change how the noise is generated: the generations prefetched at create are redrawn after them
    RNG_FORM_KEYS = ("gen_dense", "gen_split", "fuse_plan", "fast_log")

    def __init__(self, _handle=None, _keep=None, tuning=None, **kw):
        """tuning: df_set_tuning keys applied right after create (step 0 has run with the plane's defaults;
        noise already prefetched is redrawn when a generation-form key is among them)."""
        if _handle is not None:
            self._h, self._keep = _handle, _keep
        else:
            cfg, self._keep = make_config(**kw)
            self._cfg = cfg
            self._h = lib().df_create(C.byref(cfg))
            if not self._h:
                raise DFError("df_create failed: " + lib().df_last_error().decode())
        ny, nz, z0, z1 = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(lib().df_dims(self._h, C.byref(ny), C.byref(nz), C.byref(z0), C.byref(z1)))
        self.Ny, self.Nz, self.z0, self.z1 = ny.value, nz.value, z0.value, z1.value
        self.Nz_loc = self.z1 - self.z0
        if tuning:
            for k, v in tuning.items():
                self.set_tuning(k, v)
            if any(k in self.RNG_FORM_KEYS for k in tuning):
                self.set_rng_state(*self.rng_state())  # restart the noise pipeline with the new form

    def close(self):
        if getattr(self, "_h", None):
            lib().df_destroy(self._h)
            self._h = None

    def __del__(self):
        # At interpreter exit the HIP runtime may already be torn down: leave the handle to
        # process teardown then (call close() explicitly to release it earlier).
        if sys is None or sys.is_finalizing():
            return
        self.close()

    # --- hot path
    def filter(self, dt):
        _check(lib().df_filter(self._h, dt))

    def sync(self):
        _check(lib().df_sync(self._h))

    def wait(self):
        """This handle's results so far (df_wait), not the later calls' noise already queued."""
        _check(lib().df_wait(self._h))

    def trace(self):
        """Schedule records of a device=DEVICE_TRACE handle (df_trace): int64 array (n, 6) {op, stream, a, b, c, d}."""
        n = lib().df_trace(self._h, None, 0)
        if n < 0:
            raise DFError(lib().df_last_error().decode())
        out = np.zeros((n, 6), dtype=np.int64)
        if n:
            lib().df_trace(self._h, out.ctypes.data, n)
        return out

    # --- stage API (df.hpp:96-101)
    def generate_white_noise(self):
        _check(lib().df_generate_white_noise(self._h))

    def filtering_sweeps(self, comp):
        _check(lib().df_filtering_sweeps(self._h, comp))

    def correlate_fields(self, comp, dt):
        _check(lib().df_correlate_fields(self._h, comp, dt))

    def apply_RST_scaling(self):
        _check(lib().df_apply_RST_scaling(self._h))

    def get_rho_T_fluc(self):
        _check(lib().df_get_rho_T_fluc(self._h))

    # --- outputs
    def field(self, name):
        out = np.empty((self.Ny, self.Nz_loc), dtype=np.float64)
        _check(lib().df_get_field(self._h, FIELDS[name], out.ctypes.data))
        return out

    def fields(self):
        return {k: self.field(k) for k in ("u", "v", "w", "T", "rho")}

    def set_field(self, name, values):
        a = np.ascontiguousarray(values, dtype=np.float64)
        if a.size != self.Ny * self.Nz_loc:
            raise DFError(f"set_field: need {self.Ny} x {self.Nz_loc} values")
        _check(lib().df_set_field(self._h, FIELDS[name], a.ctypes.data))

    def checkpoint(self):
        """The resumable state: stream state and filt_old of u, v, w."""
        return {"rng": self.rng_state(), **{k: self.field(k) for k in ("filt_old_u", "filt_old_v", "filt_old_w")}}

    def restore(self, ck):
        self.set_rng_state(*ck["rng"])
        for k in ("filt_old_u", "filt_old_v", "filt_old_w"):
            self.set_field(k, ck[k])

    def device_ptr(self, name):
        return lib().df_device_field(self._h, FIELDS[name])

    def gather(self, name, dst, n, dst_len, plane_cell=None, dst_cell=None, beta=0.0):
        """df_gather_field: device pointers (ints, e.g. torch data_ptr()) in, async on the library stream."""
        _check(lib().df_gather_field(self._h, FIELDS[name], n, plane_cell, dst, dst_cell, dst_len, beta))

    def row(self, name):
        out = np.empty(self.Ny, dtype=np.float64)
        _check(lib().df_get_row(self._h, ROWS[name], out.ctypes.data))
        return out

    def scalar(self, name):
        return lib().df_get_scalar(self._h, ("u_tau", "tau_w", "d_v").index(name))

    def halfwidths(self, comp, direction):
        out = np.empty((self.Ny, self.Nz_loc), dtype=np.int32)
        _check(lib().df_get_halfwidths(self._h, comp, "yz".index(direction), out.ctypes.data))
        return out

    def offsets(self, comp, direction):
        out = np.empty((self.Ny, self.Nz_loc), dtype=np.int32)
        _check(lib().df_get_offsets(self._h, comp, "yz".index(direction), out.ctypes.data))
        return out

    def comp_info(self, comp):
        a, b, c, d = C.c_int(), C.c_int(), C.c_longlong(), C.c_longlong()
        _check(lib().df_get_comp_info(self._h, comp, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"Ny_max": a.value, "Nz_max": b.value, "by_size": c.value, "bz_size": d.value}

    def coeffs(self, comp, direction):
        info = self.comp_info(comp)
        n = info["by_size" if direction == "y" else "bz_size"]
        out = np.empty(n, dtype=np.float64)
        _check(lib().df_get_coeffs(self._h, comp, "yz".index(direction), out.ctypes.data, n))
        return out

    # --- RNG stream (df.cpp:334-335 state)
    def rng_state(self):
        s, f, v = C.c_uint64(), C.c_int(), C.c_double()
        _check(lib().df_rng_state(self._h, C.byref(s), C.byref(f), C.byref(v)))
        return (s.value, f.value, v.value)

    def set_rng_state(self, state, saved_flag, saved):
        _check(lib().df_set_rng_state(self._h, state, saved_flag, saved))

    def noise(self, comp, direction):
        """r_ys (direction 'y') or r_zs with its z-halo (direction 'z'), reference shapes."""
        info = self.comp_info(comp)
        if direction == "y":
            shape = (self.Ny + 2 * info["Ny_max"], self.Nz_loc)
        else:
            shape = (self.Ny, self.Nz_loc + 2 * info["Nz_max"])
        out = np.empty(shape, dtype=np.float64)
        _check(lib().df_get_noise(self._h, comp, "yz".index(direction), out.ctypes.data, out.size))
        return out

    def stream_length(self):
        return lib().df_stream_length(self._h)

    # --- statistics (get_rms, df.cpp:566-621)
    def rms_reset(self):
        _check(lib().df_rms_reset(self._h))

    def rms_add(self):
        _check(lib().df_rms_add(self._h))

    def rms(self, name):
        out = np.empty((self.Ny, self.Nz_loc), dtype=np.float64)
        _check(lib().df_rms_get(self._h, FIELDS[name], out.ctypes.data))
        return out

    def vertices(self):
        y = np.empty(self.Ny + 1)
        z = np.empty(self.Nz + 1)
        _check(lib().df_get_vertices(self._h, y.ctypes.data, z.ctypes.data))
        return y, z

    def grid(self):
        """All vertices: (y, z), each (Ny+1, Nz+1)."""
        y = np.empty((self.Ny + 1, self.Nz + 1))
        z = np.empty_like(y)
        _check(lib().df_get_grid(self._h, y.ctypes.data, z.ctypes.data))
        return y, z

    def plane_info(self):
        p, pc = C.c_int(), C.c_int()
        _check(lib().df_plane_info(self._h, C.byref(p), C.byref(pc)))
        return p.value, bool(pc.value)

    # --- measurement
    def set_tuning(self, key, value):
        _check(lib().df_set_tuning(self._h, key.encode(), int(value)))

    def get_tuning(self, key):
        """The launch shape in use for a tuning key (plane-dependent defaults or the last set_tuning)."""
        v = C.c_int(0)
        _check(lib().df_get_tuning(self._h, key.encode(), C.byref(v)))
        return v.value

    def set_profiling(self, on, every=1):
        """on: phase events on; every n > 1: only on every n-th filter() call (sampled)."""
        _check(lib().df_set_profiling(self._h, max(1, int(every)) if on else 0))

    def profile(self):
        p = Profile()
        _check(lib().df_get_profile(self._h, C.byref(p)))
        return p.as_dict()

    def comm_info(self):
        """df_comm_info: RCCL ranks, halo and RNG-collective bytes of one df_filter."""
        st = CommStats()
        _check(lib().df_comm_info(self._h, C.byref(st)))
        return st.as_dict()

    def algorithmic_bytes(self, kernel=-1):
        return lib().df_algorithmic_bytes(self._h, kernel)


def create_group(n, tuning=None, **kw):
    """n z-strips of one plane in this process (in-process halo copies). tuning: df_set_tuning keys for every
    strip, from the call after the generation prefetched at create on."""
    cfgs = (_Cfg * n)()
    keep = []
    for r in range(n):
        cfg, k = make_config(rank=r, world=n, **kw)
        cfgs[r] = cfg
        keep += k
    hs = (C.c_void_p * n)()
    _check(lib().df_create_group(cfgs, n, hs))
    out = [DigitalFilter(_handle=hs[r], _keep=keep) for r in range(n)]
    for f in out:
        for k, v in (tuning or {}).items():
            f.set_tuning(k, v)
    return out


def filter_group(filters, dt):
    hs = (C.c_void_p * len(filters))(*[f._h for f in filters])
    _check(lib().df_filter_group(hs, len(filters), dt))
