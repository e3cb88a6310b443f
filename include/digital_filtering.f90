! digital_filtering.f90 — Fortran binding of the MI355X-native DIGITAL_FILTER (libdfamd.so).
!
! Compile this file with the host CFD code and link -ldfamd (INTEGRATION.md):
!     amdflang -c digital_filtering.f90
!     amdflang my_code.f90 digital_filtering.o -L<dir> -ldfamd -Wl,-rpath,<dir>
!
! Two modules:
!   df_c_binding       bind(C) interfaces to include/df_c.h, one per C entry point;
!   DIGITAL_FILTERING  the API shape of the reference's Fortran module
!                      (digital-filtering-fortran/df/df.f90:1-138, 621-651 and
!                      test/fortran-main.f90): DFConfig, digital_filter_type,
!                      create_digital_filter(config), filter(DF, dt).
! The numerics are those of the reference's C++ path (df.cpp), which the library
! reproduces on the GPU; the reference's Fortran variant (random_number noise,
! its own correlation form, df.f90:470-588) is unfinished and is not followed.
!
! Field layout matches df.f90: DF%u%fluc(idx), idx = (j-1)*Nz + k, j = 1..Ny rows
! (wall-normal), k = 1..Nz columns (spanwise). The same array on the device is
! DF%device_fluc(DF_U); df_gather_field moves values into a CFD code's own device
! arrays without a host round trip (SURVEY 8f1, us3d_user.f90:51-130).

module df_c_binding
    use, intrinsic :: iso_c_binding
    implicit none
    public

    integer(c_int), parameter :: DF_OK = 0
    integer(c_int), parameter :: DF_U = 0, DF_V = 1, DF_W = 2, DF_T = 3, DF_RHO = 4
    integer(c_int), parameter :: DF_FILT_OLD_U = 5, DF_FILT_OLD_V = 6, DF_FILT_OLD_W = 7
    integer(c_int), parameter :: DF_PLANE_NATIVE = 0, DF_PLANE_SYNTHETIC = 1, DF_PLANE_GRID = 2
    integer(c_int), parameter :: DF_COEFF_PACKED = 0, DF_COEFF_TABLE = 1
    integer(c_int), parameter :: DF_ROW_R11 = 0, DF_ROW_R21 = 1, DF_ROW_R22 = 2, DF_ROW_R33 = 3, &
                                 DF_ROW_US = 4, DF_ROW_TS = 5, DF_ROW_RHOS = 6, DF_ROW_MS = 7, &
                                 DF_ROW_PS = 8, DF_ROW_YC = 9, DF_ROW_YC_D = 10

    ! struct df_config_c (df_c.h), member for member; bind(C) gives the C padding.
    type, bind(C) :: df_config_c
        real(c_double) :: d_i, rho_e, U_e, mu_e
        integer(c_int) :: vel_file_offset, vel_file_N_values
        type(c_ptr) :: grid_file, vel_fluc_file, line_file
        integer(c_int64_t) :: seed
        integer(c_int) :: seed_from_random_device, plane, Ny, Nz, N_min, N_max, coeff_mode
        type(c_ptr) :: csv_path
        integer(c_int) :: device, rank, world
        type(c_ptr) :: comm_id
        integer(c_int) :: rows_per_wave, rng_resume, rng_saved_flag
        integer(c_int64_t) :: rng_state
        real(c_double) :: rng_saved
        type(c_ptr) :: grid_y, grid_z
    end type df_config_c

    ! struct df_profile and struct df_comm_stats (df_c.h)
    type, bind(C) :: df_profile
        integer(c_long_long) :: calls
        real(c_double) :: rng_ms, ypass_ms, halo_ms, zpass_ms, total_ms
    end type df_profile
    type, bind(C) :: df_comm_stats
        integer(c_int) :: rccl_ranks, rccl_rank, halo_peers, rng_collective
        integer(c_long_long) :: halo_bytes_sent, rng_bytes_received, rng_blocks_counted, rng_blocks_total
    end type df_comm_stats

    interface
        subroutine df_config_default(cfg) bind(C, name="df_config_default")
            import :: df_config_c
            type(df_config_c), intent(out) :: cfg
        end subroutine
        integer(c_size_t) function df_config_sizeof() bind(C, name="df_config_sizeof")
            import :: c_size_t
        end function
        type(c_ptr) function df_create(cfg) bind(C, name="df_create")
            import :: c_ptr, df_config_c
            type(df_config_c), intent(in) :: cfg
        end function
        subroutine df_destroy(h) bind(C, name="df_destroy")
            import :: c_ptr
            type(c_ptr), value :: h
        end subroutine
        integer(c_int) function df_filter(h, dt) bind(C, name="df_filter")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            real(c_double), value :: dt
        end function
        integer(c_int) function df_get_field(h, which, out) bind(C, name="df_get_field")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
            real(c_double), intent(out) :: out(*)
        end function
        integer(c_int) function df_get_fields(h, n, which, host_out) bind(C, name="df_get_fields")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: n
            integer(c_int), intent(in) :: which(*)
            type(c_ptr), intent(in) :: host_out(*)
        end function
        integer(c_int) function df_host_pin(p, bytes) bind(C, name="df_host_pin")
            import :: c_ptr, c_int, c_size_t
            type(c_ptr), value :: p
            integer(c_size_t), value :: bytes
        end function
        integer(c_int) function df_host_unpin(p) bind(C, name="df_host_unpin")
            import :: c_ptr, c_int
            type(c_ptr), value :: p
        end function
        type(c_ptr) function df_device_field(h, which) bind(C, name="df_device_field")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: which
        end function
        integer(c_int) function df_dims(h, Ny, Nz, z0, z1) bind(C, name="df_dims")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), intent(out) :: Ny, Nz, z0, z1
        end function
        integer(c_int) function df_get_row(h, which, out) bind(C, name="df_get_row")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
            real(c_double), intent(out) :: out(*)
        end function
        real(c_double) function df_get_scalar(h, which) bind(C, name="df_get_scalar")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
        end function
        integer(c_int) function df_get_halfwidths(h, comp, dir, out) bind(C, name="df_get_halfwidths")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: comp, dir
            integer(c_int), intent(out) :: out(*)
        end function
        integer(c_int) function df_rng_state(h, state, saved_flag, saved) bind(C, name="df_rng_state")
            import :: c_ptr, c_int, c_int64_t, c_double
            type(c_ptr), value :: h
            integer(c_int64_t), intent(out) :: state
            integer(c_int), intent(out) :: saved_flag
            real(c_double), intent(out) :: saved
        end function
        integer(c_int) function df_rms_reset(h) bind(C, name="df_rms_reset")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_rms_add(h) bind(C, name="df_rms_add")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_rms_get(h, which, out) bind(C, name="df_rms_get")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
            real(c_double), intent(out) :: out(*)
        end function
        integer(c_int) function df_gather_field(h, which, n, plane_cell, dst, dst_cell, dst_len, beta) &
                bind(C, name="df_gather_field")
            import :: c_ptr, c_int, c_long_long, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
            integer(c_long_long), value :: n, dst_len
            type(c_ptr), value :: plane_cell, dst, dst_cell
            real(c_double), value :: beta
        end function
        integer(c_int) function df_sync(h) bind(C, name="df_sync")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_wait(h) bind(C, name="df_wait")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        type(c_ptr) function df_stream(h) bind(C, name="df_stream")
            import :: c_ptr
            type(c_ptr), value :: h
        end function
        integer(c_long_long) function df_stream_length(h) bind(C, name="df_stream_length")
            import :: c_ptr, c_long_long
            type(c_ptr), value :: h
        end function
        type(c_ptr) function df_last_error() bind(C, name="df_last_error")
            import :: c_ptr
        end function
        integer(c_int) function df_abi_version() bind(C, name="df_abi_version")
            import :: c_int
        end function
        ! ---- the rest of df_c.h: strip groups, the stage API, setup queries, tuning, profiling, diagnostics
        type(c_ptr) function df_data_dir() bind(C, name="df_data_dir")
            import :: c_ptr
        end function
        integer(c_int) function df_create_group(cfgs, n, out) bind(C, name="df_create_group")
            import :: c_int, c_ptr, df_config_c
            type(df_config_c), intent(in) :: cfgs(*)
            integer(c_int), value :: n
            type(c_ptr), intent(out) :: out(*)
        end function
        integer(c_int) function df_filter_group(hs, n, dt) bind(C, name="df_filter_group")
            import :: c_int, c_ptr, c_double
            type(c_ptr), intent(in) :: hs(*)
            integer(c_int), value :: n
            real(c_double), value :: dt
        end function
        integer(c_int) function df_generate_white_noise(h) bind(C, name="df_generate_white_noise")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_filtering_sweeps(h, comp) bind(C, name="df_filtering_sweeps")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: comp
        end function
        integer(c_int) function df_correlate_fields(h, comp, dt) bind(C, name="df_correlate_fields")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: comp
            real(c_double), value :: dt
        end function
        integer(c_int) function df_apply_RST_scaling(h) bind(C, name="df_apply_RST_scaling")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_get_rho_T_fluc(h) bind(C, name="df_get_rho_T_fluc")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_alloc_registry(p, bytes, claim) bind(C, name="df_alloc_registry")
            import :: c_ptr, c_size_t, c_int
            type(c_ptr), value :: p
            integer(c_size_t), value :: bytes
            integer(c_int), value :: claim
        end function
        integer(c_long_long) function df_alloc_registry_count() bind(C, name="df_alloc_registry_count")
            import :: c_long_long
        end function
        integer(c_int) function df_set_field(h, which, host_in) bind(C, name="df_set_field")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: which
            real(c_double), intent(in) :: host_in(*)
        end function
        integer(c_int) function df_get_offsets(h, comp, dir, out) bind(C, name="df_get_offsets")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: comp, dir
            integer(c_int), intent(out) :: out(*)
        end function
        integer(c_int) function df_get_comp_info(h, comp, Ny_max, Nz_max, by_size, bz_size) &
                bind(C, name="df_get_comp_info")
            import :: c_ptr, c_int, c_long_long
            type(c_ptr), value :: h
            integer(c_int), value :: comp
            integer(c_int), intent(out) :: Ny_max, Nz_max
            integer(c_long_long), intent(out) :: by_size, bz_size
        end function
        integer(c_int) function df_get_coeffs(h, comp, dir, out, n) bind(C, name="df_get_coeffs")
            import :: c_ptr, c_int, c_double, c_long_long
            type(c_ptr), value :: h
            integer(c_int), value :: comp, dir
            real(c_double), intent(out) :: out(*)
            integer(c_long_long), value :: n
        end function
        integer(c_int) function df_set_rng_state(h, state, saved_flag, saved) bind(C, name="df_set_rng_state")
            import :: c_ptr, c_int, c_int64_t, c_double
            type(c_ptr), value :: h
            integer(c_int64_t), value :: state
            integer(c_int), value :: saved_flag
            real(c_double), value :: saved
        end function
        integer(c_int) function df_get_noise(h, comp, dir, out, n) bind(C, name="df_get_noise")
            import :: c_ptr, c_int, c_double, c_long_long
            type(c_ptr), value :: h
            integer(c_int), value :: comp, dir
            real(c_double), intent(out) :: out(*)
            integer(c_long_long), value :: n
        end function
        integer(c_long_long) function df_rms_count(h) bind(C, name="df_rms_count")
            import :: c_ptr, c_long_long
            type(c_ptr), value :: h
        end function
        integer(c_int) function df_get_vertices(h, y, z) bind(C, name="df_get_vertices")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            real(c_double), intent(out) :: y(*), z(*)
        end function
        integer(c_int) function df_get_grid(h, y, z) bind(C, name="df_get_grid")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            real(c_double), intent(out) :: y(*), z(*)
        end function
        integer(c_int) function df_plane_info(h, plane, per_cell) bind(C, name="df_plane_info")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), intent(out) :: plane, per_cell
        end function
        integer(c_int) function df_set_tuning(h, key, value) bind(C, name="df_set_tuning")
            import :: c_ptr, c_int, c_char
            type(c_ptr), value :: h
            character(kind=c_char), intent(in) :: key(*) ! NUL-terminated: trim(k) // c_null_char
            integer(c_int), value :: value
        end function
        integer(c_int) function df_get_tuning(h, key, value) bind(C, name="df_get_tuning")
            import :: c_ptr, c_int, c_char
            type(c_ptr), value :: h
            character(kind=c_char), intent(in) :: key(*)
            integer(c_int), intent(out) :: value
        end function
        integer(c_int) function df_set_profiling(h, on) bind(C, name="df_set_profiling")
            import :: c_ptr, c_int
            type(c_ptr), value :: h
            integer(c_int), value :: on
        end function
        integer(c_int) function df_get_profile(h, out) bind(C, name="df_get_profile")
            import :: c_ptr, c_int, df_profile
            type(c_ptr), value :: h
            type(df_profile), intent(out) :: out
        end function
        real(c_double) function df_algorithmic_bytes(h, kernel) bind(C, name="df_algorithmic_bytes")
            import :: c_ptr, c_int, c_double
            type(c_ptr), value :: h
            integer(c_int), value :: kernel
        end function
        integer(c_int) function df_comm_unique_id(out, len) bind(C, name="df_comm_unique_id")
            import :: c_ptr, c_size_t, c_int
            type(c_ptr), value :: out
            integer(c_size_t), value :: len
        end function
        integer(c_int) function df_comm_info(h, out) bind(C, name="df_comm_info")
            import :: c_ptr, c_int, df_comm_stats
            type(c_ptr), value :: h
            type(df_comm_stats), intent(out) :: out
        end function
        integer(c_long_long) function df_trace(h, out, cap) bind(C, name="df_trace")
            import :: c_ptr, c_long_long
            type(c_ptr), value :: h
            integer(c_long_long), intent(out) :: out(*)
            integer(c_long_long), value :: cap
        end function
    end interface

contains

    ! df_last_error() as a Fortran string.
    function df_error_message() result(msg)
        character(len=:), allocatable :: msg
        character(kind=c_char), pointer :: s(:)
        type(c_ptr) :: p
        integer :: n
        interface
            integer(c_size_t) function c_strlen(str) bind(C, name="strlen")
                import :: c_ptr, c_size_t
                type(c_ptr), value :: str
            end function
        end interface
        p = df_last_error()
        if (.not. c_associated(p)) then
            msg = ""
            return
        end if
        n = int(c_strlen(p))
        call c_f_pointer(p, s, [n])
        allocate(character(len=n) :: msg)
        msg = transfer(s(1:n), msg)
    end function df_error_message

end module df_c_binding


module DIGITAL_FILTERING
    use, intrinsic :: iso_c_binding
    use df_c_binding
    implicit none
    private
    public :: digital_filter_type, create_digital_filter, filter, destroy_digital_filter, DFConfig, FilterField
    public :: get_rms, rng_state, device_fluc, gather_fluc
    public :: DF_U, DF_V, DF_W, DF_T, DF_RHO, DF_PLANE_NATIVE, DF_PLANE_SYNTHETIC, DF_PLANE_GRID
    public :: DF_COEFF_PACKED, DF_COEFF_TABLE

    integer, parameter :: dp = selected_real_kind(15)

    ! df.f90:100-104 fields first (same names and defaults as the C++ constructor,
    ! df.cpp:7-10), then the extensions of df_config_c.
    type :: DFConfig
        real(kind=dp) :: d_i = 0.0013_dp, rho_e = 0.044_dp, U_e = 869.1_dp, mu_e = 7.1212e-6_dp
        integer :: vel_file_offset = 0, vel_file_N_values = 0
        character(len=256) :: grid_file = '', vel_fluc_file = ''
        character(len=256) :: line_file = ''
        integer(c_int64_t) :: seed = -1_c_int64_t   ! < 0: seed from random_device like the reference
        integer :: plane = 0                         ! DF_PLANE_NATIVE / DF_PLANE_SYNTHETIC / DF_PLANE_GRID
        integer :: Ny = 0, Nz = 0, N_min = 0, N_max = 0
        ! DF_PLANE_GRID: the inflow grid's vertices, (Ny+1)*(Nz+1) each, index j*(Nz+1)+k+1
        ! (Ny x Nz cells, row 1 at the wall); unallocated -> grid_file (Tecplot BLOCK, write_tecplot layout)
        real(kind=dp), allocatable :: grid_y(:), grid_z(:)
        integer :: coeff_mode = 1                    ! DF_COEFF_TABLE (default: same fields, no B stream) / DF_COEFF_PACKED
        character(len=256) :: csv_file = ''          ! non-blank: reference CSV after every filter
        integer :: device = 0                        ! HIP device; -1 = host-only handle (setup queries)
        logical :: host_mirror = .true.              ! refresh DF%u%fluc ... after every filter
        ! checkpoint/resume: start the stream at (rng_state, rng_saved_flag, rng_saved) instead of seeding
        logical :: rng_resume = .false.
        integer(c_int64_t) :: rng_state = 0_c_int64_t  ! pcg32 state bits (two's complement of the uint64)
        integer :: rng_saved_flag = 0
        real(kind=dp) :: rng_saved = 0.0_dp
    end type DFConfig

    ! df.f90:84-98: per-component host view (the device holds the working arrays).
    type :: FilterField
        real(kind=dp), allocatable :: fluc(:), filt_old(:)
        integer, allocatable :: N_ys(:), N_zs(:)
        integer :: Ny_max = 0, Nz_max = 0
    end type FilterField

    type :: digital_filter_type
        type(c_ptr) :: handle = c_null_ptr
        integer :: Ny = 0, Nz = 0, z0 = 0, z1 = 0, n_cells = 0
        real(kind=dp) :: dt = 0.0_dp
        real(kind=dp) :: u_tau = 0.0_dp, tau_w = 0.0_dp
        logical :: host_mirror = .true., on_device = .true.
        type(c_ptr) :: pinned(8) = c_null_ptr       ! page-locked mirror buffers (df_host_pin), by address
        type(FilterField) :: u, v, w
        real(kind=dp), allocatable :: T_fluc(:), rho_fluc(:)
        real(kind=dp), allocatable :: R11(:), R21(:), R22(:), R33(:), yc(:)
    end type digital_filter_type

contains

    subroutine check(rc, what)
        integer(c_int), intent(in) :: rc
        character(len=*), intent(in) :: what
        if (rc /= DF_OK) then
            write(*, '(a)') 'DIGITAL_FILTERING: ' // what // ': ' // df_error_message()
            error stop 1
        end if
    end subroutine check

    ! NUL-terminated copy of a blank-padded Fortran string (kept alive by the caller).
    subroutine c_string(s, buf, p)
        character(len=*), intent(in) :: s
        character(kind=c_char), allocatable, target, intent(inout) :: buf(:)
        type(c_ptr), intent(out) :: p
        integer :: i, n
        n = len_trim(s)
        if (n == 0) then
            p = c_null_ptr
            return
        end if
        allocate(buf(n + 1))
        do i = 1, n
            buf(i) = s(i:i)
        end do
        buf(n + 1) = c_null_char
        p = c_loc(buf)
    end subroutine c_string

    ! Blank input path -> $DF_DATA_DIR/<name>, else digital-filtering_amd/data/<name>
    ! (the reference reads ../files/RST.dat and ../line.dat, df.cpp:16, 224).
    function data_path(given, name) result(path)
        character(len=*), intent(in) :: given, name
        character(len=512) :: path, dir
        integer :: n, st
        if (len_trim(given) > 0) then
            path = given
            return
        end if
        call get_environment_variable('DF_DATA_DIR', dir, n, st)
        path = ''  ! blank: keep df_config_default's path (df_data_dir(), next to libdfamd.so)
        if (st == 0 .and. n > 0) path = trim(dir) // '/' // name
    end function data_path

    ! DIGITAL_FILTER(DFConfig) (df.f90:74-138 shape; df.cpp:4-66 semantics): setup and
    ! the constructor's step 0 on the device.
    function create_digital_filter(config) result(DF)
        type(DFConfig), intent(in) :: config
        type(digital_filter_type) :: DF
        type(df_config_c) :: c
        character(kind=c_char), allocatable, target :: s_grid(:), s_rst(:), s_line(:), s_csv(:)
        real(c_double), allocatable, target :: gy(:), gz(:)
        integer(c_int) :: Ny, Nz, z0, z1
        integer :: comp

        if (df_config_sizeof() /= c_sizeof(c)) then
            write(*, '(a)') 'DIGITAL_FILTERING: df_config_c layout differs from libdfamd'
            error stop 1
        end if
        call df_config_default(c)
        c%d_i = config%d_i
        c%rho_e = config%rho_e
        c%U_e = config%U_e
        c%mu_e = config%mu_e
        c%vel_file_offset = config%vel_file_offset
        c%vel_file_N_values = config%vel_file_N_values
        call c_string(config%grid_file, s_grid, c%grid_file)
        if (len_trim(data_path(config%vel_fluc_file, 'RST.dat')) > 0) &
            call c_string(data_path(config%vel_fluc_file, 'RST.dat'), s_rst, c%vel_fluc_file)
        if (len_trim(data_path(config%line_file, 'line.dat')) > 0) &
            call c_string(data_path(config%line_file, 'line.dat'), s_line, c%line_file)
        call c_string(config%csv_file, s_csv, c%csv_path)
        if (config%seed >= 0) then
            c%seed = config%seed
            c%seed_from_random_device = 0
        end if
        c%plane = config%plane
        c%Ny = config%Ny
        c%Nz = config%Nz
        c%N_min = config%N_min
        c%N_max = config%N_max
        c%coeff_mode = config%coeff_mode
        c%device = config%device
        if (allocated(config%grid_y) .and. allocated(config%grid_z)) then
            gy = config%grid_y
            gz = config%grid_z
            c%grid_y = c_loc(gy)
            c%grid_z = c_loc(gz)
        end if
        if (config%rng_resume) then
            c%rng_resume = 1
            c%rng_state = config%rng_state
            c%rng_saved_flag = config%rng_saved_flag
            c%rng_saved = config%rng_saved
        end if

        DF%handle = df_create(c)
        if (.not. c_associated(DF%handle)) then
            write(*, '(a)') 'DIGITAL_FILTERING: create_digital_filter: ' // df_error_message()
            error stop 1
        end if
        call check(df_dims(DF%handle, Ny, Nz, z0, z1), 'df_dims')
        DF%Ny = Ny
        DF%Nz = z1 - z0
        DF%z0 = z0
        DF%z1 = z1
        DF%n_cells = DF%Ny * DF%Nz
        DF%on_device = config%device >= 0
        DF%host_mirror = config%host_mirror .and. DF%on_device
        DF%u_tau = df_get_scalar(DF%handle, 0_c_int)
        DF%tau_w = df_get_scalar(DF%handle, 1_c_int)
        allocate(DF%R11(Ny), DF%R21(Ny), DF%R22(Ny), DF%R33(Ny), DF%yc(Ny))
        call check(df_get_row(DF%handle, DF_ROW_R11, DF%R11), 'df_get_row')
        call check(df_get_row(DF%handle, DF_ROW_R21, DF%R21), 'df_get_row')
        call check(df_get_row(DF%handle, DF_ROW_R22, DF%R22), 'df_get_row')
        call check(df_get_row(DF%handle, DF_ROW_R33, DF%R33), 'df_get_row')
        call check(df_get_row(DF%handle, DF_ROW_YC, DF%yc), 'df_get_row')
        do comp = 0, 2
            call load_halfwidths(DF, comp)
        end do
        if (DF%host_mirror) call refresh(DF)
    end function create_digital_filter

    subroutine load_halfwidths(DF, comp)
        type(digital_filter_type), intent(inout), target :: DF
        integer, intent(in) :: comp
        type(FilterField), pointer :: F
        integer(c_int), allocatable :: tmp(:)
        F => field_of(DF, comp)
        allocate(tmp(DF%n_cells))
        call check(df_get_halfwidths(DF%handle, int(comp, c_int), 0_c_int, tmp), 'df_get_halfwidths')
        F%N_ys = tmp
        call check(df_get_halfwidths(DF%handle, int(comp, c_int), 1_c_int, tmp), 'df_get_halfwidths')
        F%N_zs = tmp
        F%Ny_max = maxval(F%N_ys)
        F%Nz_max = maxval(F%N_zs)
    end subroutine load_halfwidths

    function field_of(DF, comp) result(F)
        type(digital_filter_type), intent(inout), target :: DF
        integer, intent(in) :: comp
        type(FilterField), pointer :: F
        select case (comp)
        case (0)
            F => DF%u
        case (1)
            F => DF%v
        case default
            F => DF%w
        end select
    end function field_of

    ! Host mirrors of the current fields: the eight D2H copies queued together, one synchronisation
    ! (df_get_fields), into page-locked arrays (re-registered if an array moved, e.g. after the
    ! assignment df = create_digital_filter(...)); skipped when host_mirror = .false.
    subroutine refresh(DF)
        type(digital_filter_type), intent(inout), target :: DF
        integer :: comp, i
        type(FilterField), pointer :: F
        integer(c_int) :: which(8), rc
        type(c_ptr) :: outp(8)
        do comp = 0, 2
            F => field_of(DF, comp)
            if (.not. allocated(F%fluc)) allocate(F%fluc(DF%n_cells), F%filt_old(DF%n_cells))
            which(comp + 1) = int(comp, c_int)
            outp(comp + 1) = c_loc(F%fluc)
            which(comp + 4) = int(DF_FILT_OLD_U + comp, c_int)
            outp(comp + 4) = c_loc(F%filt_old)
        end do
        if (.not. allocated(DF%T_fluc)) allocate(DF%T_fluc(DF%n_cells), DF%rho_fluc(DF%n_cells))
        which(7) = DF_T
        outp(7) = c_loc(DF%T_fluc)
        which(8) = DF_RHO
        outp(8) = c_loc(DF%rho_fluc)
        do i = 1, 8
            if (.not. c_associated(outp(i), DF%pinned(i))) then
                if (c_associated(DF%pinned(i))) rc = df_host_unpin(DF%pinned(i))
                DF%pinned(i) = c_null_ptr
                ! a refused registration leaves a pageable copy (slower, same bytes)
                if (df_host_pin(outp(i), int(DF%n_cells, c_size_t) * 8_c_size_t) == DF_OK) DF%pinned(i) = outp(i)
            end if
        end do
        call check(df_get_fields(DF%handle, 8_c_int, which, outp), 'df_get_fields')
    end subroutine refresh

    ! filter(DF, dt) (df.f90:621-651 shape; df.cpp:449-468 semantics).
    subroutine filter(DF, dt_input)
        type(digital_filter_type), intent(inout) :: DF
        real(kind=dp), intent(in) :: dt_input
        DF%dt = dt_input
        call check(df_filter(DF%handle, real(dt_input, c_double)), 'filter')
        if (DF%host_mirror) call refresh(DF)
    end subroutine filter

    subroutine destroy_digital_filter(DF)
        type(digital_filter_type), intent(inout) :: DF
        integer :: i
        integer(c_int) :: rc
        do i = 1, 8
            if (c_associated(DF%pinned(i))) rc = df_host_unpin(DF%pinned(i))
            DF%pinned(i) = c_null_ptr
        end do
        if (c_associated(DF%handle)) call df_destroy(DF%handle)
        DF%handle = c_null_ptr
    end subroutine destroy_digital_filter

    ! get_rms (df.cpp:566-611) on the device: n_steps filter(dt) calls accumulated
    ! per cell; rms(:, 1..5) = u', v', w', T', rho' RMS per cell.
    subroutine get_rms(DF, dt, n_steps, rms)
        type(digital_filter_type), intent(inout) :: DF
        real(kind=dp), intent(in) :: dt
        integer, intent(in) :: n_steps
        real(kind=dp), intent(out) :: rms(:, :)
        integer :: i
        logical :: keep
        keep = DF%host_mirror
        DF%host_mirror = .false.
        call check(df_rms_reset(DF%handle), 'df_rms_reset')
        do i = 1, n_steps
            call filter(DF, dt)
            call check(df_rms_add(DF%handle), 'df_rms_add')
        end do
        do i = 1, 5
            call check(df_rms_get(DF%handle, int(i - 1, c_int), rms(:, i)), 'df_rms_get')
        end do
        DF%host_mirror = keep
        if (keep) call refresh(DF)
    end subroutine get_rms

    ! pcg32 state, cached-normal flag and value after the last call (bit-exact with the reference).
    subroutine rng_state(DF, state, saved_flag, saved)
        type(digital_filter_type), intent(inout) :: DF
        integer(c_int64_t), intent(out) :: state
        integer, intent(out) :: saved_flag
        real(kind=dp), intent(out) :: saved
        integer(c_int) :: f
        call check(df_rng_state(DF%handle, state, f, saved), 'df_rng_state')
        saved_flag = f
    end subroutine rng_state

    ! Device address of a dense field (row-major Ny x Nz, i.e. idx = (j-1)*Nz + k).
    type(c_ptr) function device_fluc(DF, which)
        type(digital_filter_type), intent(in) :: DF
        integer, intent(in) :: which
        device_fluc = df_device_field(DF%handle, int(which, c_int))
    end function device_fluc

    ! dst(dst_cell(i)) = beta*dst(dst_cell(i)) + field(plane_cell(i)) on the device, ordered
    ! after the last filter on the library stream (0-based int64 device index arrays, or
    ! c_null_ptr for identity). Errors in indices surface at the next df_sync.
    subroutine gather_fluc(DF, which, n, plane_cell, dst, dst_cell, dst_len, beta)
        type(digital_filter_type), intent(in) :: DF
        integer, intent(in) :: which
        integer(c_long_long), intent(in) :: n, dst_len
        type(c_ptr), intent(in) :: plane_cell, dst, dst_cell
        real(kind=dp), intent(in) :: beta
        call check(df_gather_field(DF%handle, int(which, c_int), n, plane_cell, dst, dst_cell, dst_len, &
                                   real(beta, c_double)), 'gather_fluc')
    end subroutine gather_fluc

end module DIGITAL_FILTERING
