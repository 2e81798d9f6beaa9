! mitgcm_amd.F90 -- ISO_C_BINDING interface to the MI355X C-ABI (include/mitgcm_amd.h)
! for Fortran hosts.  The model-handle API (mgcm_*) is bound by name; the
! reference-signature drop-ins (CG2D_AMD, INI_CG2D_AMD) need no interface: they
! follow the amdflang/gfortran external naming (lower case + '_') and take every
! argument by reference, exactly as the reference's own CG2D (model/src/cg2d.F:13).
module mitgcm_amd
  use, intrinsic :: iso_c_binding
  implicit none
  interface
    function mgcm_create(sNx, sNy, OLx, OLy, Nr, nSx, nSy, device) bind(C, name="mgcm_create")
      import :: c_ptr, c_int
      integer(c_int), value :: sNx, sNy, OLx, OLy, Nr, nSx, nSy, device
      type(c_ptr) :: mgcm_create
    end function
    subroutine mgcm_destroy(m) bind(C, name="mgcm_destroy")
      import :: c_ptr
      type(c_ptr), value :: m
    end subroutine
    function mgcm_set_param(m, name, value) bind(C, name="mgcm_set_param")
      import :: c_ptr, c_int, c_char, c_double
      type(c_ptr), value :: m
      character(kind=c_char), dimension(*) :: name
      real(c_double), value :: value
      integer(c_int) :: mgcm_set_param
    end function
    function mgcm_put(m, name, host, count) bind(C, name="mgcm_put")
      import :: c_ptr, c_int, c_char, c_double, c_long
      type(c_ptr), value :: m
      character(kind=c_char), dimension(*) :: name
      real(c_double), dimension(*) :: host
      integer(c_long), value :: count
      integer(c_int) :: mgcm_put
    end function
    function mgcm_get(m, name, host, count) bind(C, name="mgcm_get")
      import :: c_ptr, c_int, c_char, c_double, c_long
      type(c_ptr), value :: m
      character(kind=c_char), dimension(*) :: name
      real(c_double), dimension(*) :: host
      integer(c_long), value :: count
      integer(c_int) :: mgcm_get
    end function
    function mgcm_init(m) bind(C, name="mgcm_init")
      import :: c_ptr, c_int
      type(c_ptr), value :: m
      integer(c_int) :: mgcm_init
    end function
    function mgcm_forward_step(m, nsteps) bind(C, name="mgcm_forward_step")
      import :: c_ptr, c_int
      type(c_ptr), value :: m
      integer(c_int), value :: nsteps
      integer(c_int) :: mgcm_forward_step
    end function
    function mgcm_sync(m) bind(C, name="mgcm_sync")
      import :: c_ptr, c_int
      type(c_ptr), value :: m
      integer(c_int) :: mgcm_sync
    end function
    function mgcm_last_error() bind(C, name="mgcm_last_error")
      import :: c_ptr
      type(c_ptr) :: mgcm_last_error
    end function
  end interface
end module mitgcm_amd
