! fortran_main.f90 — the reference's Fortran driver (digital-filtering-fortran/test/
! fortran-main.f90) on the MI355X library, plus the modes the tests use.
!
!   fortran-main                                   create + filter(1e-8) on the native plane
!   fortran-main host PLANE Ny Nz Nmin Nmax OUT     host-only setup dump (no GPU)
!   fortran-main run PLANE Ny Nz Nmin Nmax SEED STEPS DT OUT
!                                                   ctor + STEPS x filter(DT), fields dumped;
!                                                   optional STATE FLAG SAVED resume the stream
!   fortran-main gather PLANE Ny Nz Nmin Nmax SEED OUT
!                                                   device handoff: u' gathered into a
!                                                   hipMalloc'd array, reversed, beta = 1
! PLANE: 0 native grid (files/RST.dat), 1 synthetic (Ny, Nz, Nmin, Nmax used).
! OUT files are raw little-endian streams read by tests/test_fortran.py.
program fortran_main
    use, intrinsic :: iso_c_binding
    use DIGITAL_FILTERING
    use df_c_binding, only: df_sync
    implicit none
    integer, parameter :: dp = selected_real_kind(15)

    interface
        integer(c_int) function hipMalloc(p, n) bind(C, name="hipMalloc")
            import :: c_ptr, c_int, c_size_t
            type(c_ptr), intent(out) :: p
            integer(c_size_t), value :: n
        end function
        integer(c_int) function hipFree(p) bind(C, name="hipFree")
            import :: c_ptr, c_int
            type(c_ptr), value :: p
        end function
        integer(c_int) function hipMemcpy(dst, src, n, kind) bind(C, name="hipMemcpy")
            import :: c_ptr, c_int, c_size_t
            type(c_ptr), value :: dst, src
            integer(c_size_t), value :: n
            integer(c_int), value :: kind
        end function
    end interface
    integer(c_int), parameter :: H2D = 1, D2H = 2

    type(digital_filter_type) :: df
    type(DFConfig) :: config
    character(len=256) :: mode, arg, out
    real(kind=dp) :: dt

    if (command_argument_count() == 0) then
        ! fortran-main.f90: configure, construct, one filter(dt) call.
        config%d_i = 0.0013_dp
        config%rho_e = 0.044_dp
        config%U_e = 869.1_dp
        config%grid_file = 'grid.dat'
        df = create_digital_filter(config)
        dt = 1e-8_dp
        call filter(df, dt)
        write(*, '(a, i0, a, i0, a, es24.16)') 'plane ', df%Ny, ' x ', df%Nz, '  sum u''^2 = ', sum(df%u%fluc**2)
        call destroy_digital_filter(df)
        stop
    end if

    call get_command_argument(1, mode)
    call read_plane(config)
    select case (trim(mode))
    case ('host')
        call get_command_argument(7, out)
        config%device = -1
        config%seed = 1
        df = create_digital_filter(config)
        call dump_setup(df, out)
    case ('run')
        call get_command_argument(7, arg)
        read(arg, *) config%seed
        call run_mode(config)
    case ('gather')
        call get_command_argument(7, arg)
        read(arg, *) config%seed
        call get_command_argument(8, out)
        call gather_mode(config, out)
    case default
        write(*, '(a)') 'unknown mode ' // trim(mode)
        error stop 2
    end select
    call destroy_digital_filter(df)

contains

    subroutine read_plane(c)
        type(DFConfig), intent(inout) :: c
        character(len=64) :: a
        call get_command_argument(2, a)
        read(a, *) c%plane
        call get_command_argument(3, a)
        read(a, *) c%Ny
        call get_command_argument(4, a)
        read(a, *) c%Nz
        call get_command_argument(5, a)
        read(a, *) c%N_min
        call get_command_argument(6, a)
        read(a, *) c%N_max
    end subroutine read_plane

    subroutine dump_setup(d, path)
        type(digital_filter_type), intent(in) :: d
        character(len=*), intent(in) :: path
        integer :: u
        open(newunit=u, file=trim(path), access='stream', form='unformatted', status='replace')
        write(u) int(d%Ny, 4), int(d%Nz, 4), d%u_tau, d%tau_w
        write(u) d%R11, d%R21, d%R22, d%R33, d%yc
        write(u) int(d%u%N_ys, 4), int(d%u%N_zs, 4), int(d%v%N_ys, 4), int(d%v%N_zs, 4), &
                 int(d%w%N_ys, 4), int(d%w%N_zs, 4)
        close(u)
    end subroutine dump_setup

    subroutine run_mode(c)
        type(DFConfig), intent(inout) :: c
        integer :: steps, i, u, flag
        integer(c_int64_t) :: state
        real(kind=dp) :: saved, step_dt
        character(len=64) :: a
        call get_command_argument(8, a)
        read(a, *) steps
        call get_command_argument(9, a)
        read(a, *) step_dt
        call get_command_argument(10, out)
        if (command_argument_count() >= 13) then
            c%rng_resume = .true.
            call get_command_argument(11, a)
            read(a, *) c%rng_state
            call get_command_argument(12, a)
            read(a, *) c%rng_saved_flag
            call get_command_argument(13, a)
            read(a, *) c%rng_saved
        end if
        df = create_digital_filter(c)
        do i = 1, steps
            call filter(df, step_dt)
        end do
        call rng_state(df, state, flag, saved)
        open(newunit=u, file=trim(out), access='stream', form='unformatted', status='replace')
        write(u) int(df%Ny, 4), int(df%Nz, 4), state, int(flag, 4), saved
        write(u) df%u%fluc, df%v%fluc, df%w%fluc, df%T_fluc, df%rho_fluc, df%u%filt_old
        close(u)
    end subroutine run_mode

    ! A CFD code's ghost-cell array: dst(i) = base(i) + u'(plane cell n-1-i), filled on the
    ! device from the library's field without a host round trip (df_gather_field).
    subroutine gather_mode(c, path)
        type(DFConfig), intent(inout) :: c
        character(len=*), intent(in) :: path
        integer(c_long_long), allocatable, target :: idx(:)
        real(kind=dp), allocatable, target :: base(:), got(:)
        type(c_ptr) :: d_dst, d_idx
        integer(c_long_long) :: n, i
        integer :: u
        c%host_mirror = .true.
        df = create_digital_filter(c)
        call filter(df, 1e-8_dp)
        n = df%n_cells
        allocate(idx(n), base(n), got(n))
        do i = 1, n
            idx(i) = n - i
            base(i) = 1000.0_dp + real(i, dp)
        end do
        if (hipMalloc(d_dst, int(8 * n, c_size_t)) /= 0) error stop 3
        if (hipMalloc(d_idx, int(8 * n, c_size_t)) /= 0) error stop 3
        if (hipMemcpy(d_dst, c_loc(base), int(8 * n, c_size_t), H2D) /= 0) error stop 3
        if (hipMemcpy(d_idx, c_loc(idx), int(8 * n, c_size_t), H2D) /= 0) error stop 3
        call gather_fluc(df, DF_U, n, d_idx, d_dst, c_null_ptr, n, 1.0_dp)
        if (df_sync(df%handle) /= 0) error stop 4
        if (hipMemcpy(c_loc(got), d_dst, int(8 * n, c_size_t), D2H) /= 0) error stop 3
        open(newunit=u, file=trim(path), access='stream', form='unformatted', status='replace')
        write(u) int(df%Ny, 4), int(df%Nz, 4)
        write(u) df%u%fluc, base, got
        close(u)
        if (hipFree(d_dst) /= 0 .or. hipFree(d_idx) /= 0) error stop 3
    end subroutine gather_mode

end program fortran_main
