! cg2d_host.F90 -- Fortran host exercising the reference-signature CG2D drop-in.
!
! Reads (stream, native endian) the operator and a right-hand side written by
! the test (tests/test_gpu_parity.py::test_fortran_cg2d_dropin), declares them exactly as the reference
! does -- (1-OLx:sNx+OLx, 1-OLy:sNy+OLy, nSx, nSy), model/src/cg2d.F:52-53 and
! model/inc/CG2D.h -- registers the operator with INI_CG2D_AMD and calls
! CG2D_AMD with CG2D's own argument list (model/src/cg2d.F:13-17).  Writes
! x, firstResidual, lastResidual, numIters back for the test to compare.
program cg2d_host
  implicit none
  integer :: sNx, sNy, OLx, OLy, nSx, nSy, maxIters, normRHS
  real(8) :: cg2dNorm, tolSq
  real(8), allocatable :: aW2d(:,:,:,:), aS2d(:,:,:,:), aC2d(:,:,:,:)
  real(8), allocatable :: pW(:,:,:,:), pS(:,:,:,:), pC(:,:,:,:)
  real(8), allocatable :: cg2d_b(:,:,:,:), cg2d_x(:,:,:,:)
  real(8) :: firstResidual, minResidualSq, lastResidual
  integer :: numIters, nIterMin, myThid, u
  character(len=512) :: dir
  call get_command_argument(1, dir)
  open(newunit=u, file=trim(dir)//'/cg2d_in.bin', access='stream', form='unformatted', status='old')
  read(u) sNx, sNy, OLx, OLy, nSx, nSy, maxIters, normRHS
  read(u) cg2dNorm, tolSq
  allocate(aW2d(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy), aS2d(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy))
  allocate(aC2d(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy), pW(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy))
  allocate(pS(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy), pC(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy))
  allocate(cg2d_b(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy), cg2d_x(1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy))
  read(u) aW2d, aS2d, aC2d, pW, pS, pC, cg2d_b, cg2d_x
  close(u)
  call INI_CG2D_AMD(sNx, sNy, OLx, OLy, nSx, nSy, aW2d, aS2d, aC2d, pW, pS, pC, cg2dNorm, tolSq, normRHS)
  numIters = maxIters
  nIterMin = -1
  myThid = 1
  call CG2D_AMD(cg2d_b, cg2d_x, firstResidual, minResidualSq, lastResidual, numIters, nIterMin, myThid)
  open(newunit=u, file=trim(dir)//'/cg2d_out.bin', access='stream', form='unformatted', status='replace')
  write(u) numIters, nIterMin
  write(u) firstResidual, minResidualSq, lastResidual
  write(u) cg2d_x
  close(u)
  print '(A,I6,A,1PE23.14,A,1PE23.14)', ' cg2d_host: iters=', numIters, ' init_res=', firstResidual, &
        ' last_res=', lastResidual
end program cg2d_host
