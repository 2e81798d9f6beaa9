"""Host-side initialisation (INITIALISE_FIXED subset), numpy, once per run.

These routines run once on the host in the reference too; the product keeps
them on the host and hands the results to the device mirror.  Arrays are
halo-inclusive, shaped (nTiles, ny, nx) for 2-D and (nTiles, Nr, ny, nx) for
3-D, where [t, j+OLy-1, i+OLx-1] is the reference's (i, j, bi, bj).

Restated from:
  INI_VERTICAL_GRID   model/src/ini_vertical_grid.F
  INI_LOCAL_GRID      model/src/ini_local_grid.F
  INI_CARTESIAN_GRID  model/src/ini_cartesian_grid.F
  INI_GRID reciprocals model/src/ini_grid.F
  INI_CORI            model/src/ini_cori.F
  INI_DEPTHS          model/src/ini_depths.F
  INI_MASKS_ETC       model/src/ini_masks_etc.F
  INI_LINEAR_PHISURF  model/src/ini_linear_phisurf.F:78-88
  INI_CG2D            model/src/ini_cg2d.F:61-237
"""
import numpy as np

from .topology import LatLonTopology


class Grid:
    def __init__(self, sNx, sNy, OLx, OLy, Nr, nSx=1, nSy=1, topology=None):
        self.sNx, self.sNy, self.OLx, self.OLy, self.Nr, self.nSx, self.nSy = sNx, sNy, OLx, OLy, Nr, nSx, nSy
        self.nTiles = nSx * nSy
        self.nx, self.ny = sNx + 2 * OLx, sNy + 2 * OLy
        self.topo = topology or LatLonTopology(sNx, sNy, OLx, OLy, nSx, nSy)
        self.f = {}   # name -> array (float64)
        self.i = {}   # integer arrays

    # ---- helpers ------------------------------------------------------------
    def z2(self):
        return np.zeros((self.nTiles, self.ny, self.nx))

    def z3(self):
        return np.zeros((self.nTiles, self.Nr, self.ny, self.nx))

    def sl(self, i0, i1, j0, j1):
        """Slice for Fortran ranges i0..i1, j0..j1 (inclusive) on the last two axes."""
        return (slice(j0 + self.OLy - 1, j1 + self.OLy), slice(i0 + self.OLx - 1, i1 + self.OLx))

    def exch(self, a):
        return self.topo.exchange(a)

    def exch_uv(self, u, v, withSigns=False):
        """EXCH_UV_XY(Z)_RS/RL of a C-grid vector pair (grid arrays: withSigns=.FALSE.)."""
        return self.topo.exchange_uv(u, v, withSigns)

    # ---- vertical grid --------------------------------------------------------
    def ini_vertical_grid(self, delR, rkSign=-1.0, Ro_SeaLevel=0.0):
        Nr = self.Nr
        drF = np.array(delR, dtype=np.float64)
        drC = np.zeros(Nr + 1)
        drC[0] = 0.5 * drF[0]
        for k in range(1, Nr):
            drC[k] = 0.5 * (drF[k - 1] + drF[k])
        drC[Nr] = 0.5 * drF[Nr - 1]
        rF = np.zeros(Nr + 1)
        rF[0] = Ro_SeaLevel               # p-coordinates: surface pressure (ini_vertical_grid.F)
        for k in range(Nr):
            rF[k + 1] = rF[k] + rkSign * drF[k]
        rC = np.zeros(Nr)
        rC[0] = rF[0] + rkSign * drC[0]
        for k in range(1, Nr):
            rC[k] = rC[k - 1] + rkSign * drC[k]
        self.f.update(drF=drF, drC=drC, rF=rF, rC=rC, recip_drF=1.0 / drF, recip_drC=1.0 / drC)

    # ---- horizontal grid ------------------------------------------------------
    def _local_grid(self, t, delX, delY, xgOrigin, ygOrigin):
        """INI_LOCAL_GRID (model/src/ini_local_grid.F): corner coordinates
        xGloc/yGloc (sNx+2OLx+1, sNy+2OLy+1) as sequential running sums, and
        delXloc(i) / delYloc(j) for i = -OLx..sNx+OLx (index i+OLx)."""
        sNx, sNy, OLx, OLy = self.sNx, self.sNy, self.OLx, self.OLy
        Nx, Ny = sNx * self.nSx, sNy * self.nSy
        bi, bj = t % self.nSx, t // self.nSx
        iG0, jG0 = bi * sNx, bj * sNy
        xG0 = xgOrigin
        for i in range(1, iG0 + 1):
            xG0 += delX[i - 1]
        for i in range(1, OLx + 1):
            xG0 -= delX[(iG0 - i + OLx * Nx) % Nx]
        yG0 = ygOrigin
        for j in range(1, jG0 + 1):
            yG0 += delY[j - 1]
        for j in range(1, OLy + 1):
            yG0 -= delY[(jG0 - j + OLy * Ny) % Ny]
        dXl = np.array([delX[(iG0 + i - 1 + OLx * Nx) % Nx] for i in range(-OLx, sNx + OLx + 1)])
        dYl = np.array([delY[(jG0 + j - 1 + OLy * Ny) % Ny] for j in range(-OLy, sNy + OLy + 1)])
        nxl, nyl = sNx + 2 * OLx + 1, sNy + 2 * OLy + 1
        xGl = np.zeros(nxl)
        xGl[0] = xG0
        for ii in range(1, nxl):
            xGl[ii] = xGl[ii - 1] + dXl[ii]
        yGl = np.zeros(nyl)
        yGl[0] = yG0
        for jj in range(1, nyl):
            yGl[jj] = yGl[jj - 1] + dYl[jj]
        XG = np.broadcast_to(xGl[None, :], (nyl, nxl))
        YG = np.broadcast_to(yGl[:, None], (nyl, nxl))
        return XG, YG, dXl, dYl

    _GRID_NAMES = ("xC", "yC", "xG", "yG", "dxF", "dyF", "dxG", "dyG", "dxC", "dyC", "dxV", "dyU",
                   "rA", "rAw", "rAs", "rAz")

    def ini_cartesian_grid(self, delX, delY, xgOrigin, ygOrigin):
        """INI_CARTESIAN_GRID (model/src/ini_cartesian_grid.F)."""
        delX = np.asarray(delX, dtype=np.float64)
        delY = np.asarray(delY, dtype=np.float64)
        for n in self._GRID_NAMES:
            self.f[n] = self.z2()
        self.usingSphericalPolarGrid = False
        for t in range(self.nTiles):
            XG, YG, dXl, dYl = self._local_grid(t, delX, delY, xgOrigin, ygOrigin)
            f = self.f
            f["xG"][t] = XG[:-1, :-1]
            f["yG"][t] = YG[:-1, :-1]
            f["xC"][t] = 0.25 * (XG[:-1, :-1] + XG[:-1, 1:] + XG[1:, :-1] + XG[1:, 1:])
            f["yC"][t] = 0.25 * (YG[:-1, :-1] + YG[:-1, 1:] + YG[1:, :-1] + YG[1:, 1:])
            dxl = dXl[1:]   # delXloc(i) for i = 1-OLx..sNx+OLx
            dyl = dYl[1:]
            f["dxF"][t] = dxl[None, :]
            f["dyF"][t] = dyl[:, None]
            f["dxG"][t] = dxl[None, :]
            f["dyG"][t] = dyl[:, None]
            f["dxC"][t, :, 1:] = 0.5 * (f["dxF"][t, :, 1:] + f["dxF"][t, :, :-1])
            f["dyC"][t, 1:, :] = 0.5 * (f["dyF"][t, 1:, :] + f["dyF"][t, :-1, :])
            f["dxV"][t, 1:, 1:] = 0.5 * (f["dxG"][t, 1:, 1:] + f["dxG"][t, 1:, :-1])
            f["dyU"][t, 1:, 1:] = 0.5 * (f["dyG"][t, 1:, 1:] + f["dyG"][t, :-1, 1:])
            f["rA"][t] = f["dxF"][t] * f["dyF"][t]
            f["rAw"][t] = f["dxC"][t] * f["dyG"][t]
            f["rAs"][t] = f["dxG"][t] * f["dyC"][t]
            f["rAz"][t] = f["dxV"][t] * f["dyU"][t]
        self._reciprocals()

    def ini_spherical_polar_grid(self, delX, delY, xgOrigin, ygOrigin, rSphere=6370.0e3):
        """INI_SPHERICAL_POLAR_GRID (model/src/ini_spherical_polar_grid.F:60-250),
        rotateGrid=F, cosPower=0.  Transcendentals go through the C library
        (math.sin/cos/tan) element by element, as the compiled reference does,
        not through numpy's vectorised kernels."""
        from math import cos, sin, tan
        deg2rad = 2.0 * np.pi / 360.0          # PARAMS.h:18, PI = 3.14159265358979323844D0
        delX = np.asarray(delX, dtype=np.float64)
        delY = np.asarray(delY, dtype=np.float64)
        for n in self._GRID_NAMES + ("tanPhiAtU", "tanPhiAtV"):
            self.f[n] = self.z2()
        self.usingSphericalPolarGrid = True
        self.rSphere = rSphere
        self.recip_rSphere = 1.0 / rSphere
        nx, ny = self.nx, self.ny
        for t in range(self.nTiles):
            XG, YG, dXl, dYl = self._local_grid(t, delX, delY, xgOrigin, ygOrigin)
            f = self.f
            f["xG"][t] = XG[:-1, :-1]
            f["yG"][t] = YG[:-1, :-1]
            f["xC"][t] = 0.25 * (XG[:-1, :-1] + XG[:-1, 1:] + XG[1:, :-1] + XG[1:, 1:])
            f["yC"][t] = 0.25 * (YG[:-1, :-1] + YG[:-1, 1:] + YG[1:, :-1] + YG[1:, 1:])
            dxl = dXl          # delXloc(i), i = -OLx.. ; Fortran i (1-OLx based) -> index I+1
            dyl = dYl
            dxF, dyF, dxG, dyG = f["dxF"][t], f["dyF"][t], f["dxG"][t], f["dyG"][t]
            rA, rAs, rAz = f["rA"][t], f["rAs"][t], f["rAz"][t]
            for J in range(ny):
                for I in range(nx):
                    lat = f["yC"][t, J, I]
                    dlon, dlat = dxl[I + 1], dyl[J + 1]
                    dxF[J, I] = rSphere * cos(lat * deg2rad) * dlon * deg2rad
                    dyF[J, I] = rSphere * dlat * deg2rad
                    lat = 0.5 * (YG[J, I] + YG[J, I + 1])
                    v = rSphere * cos(deg2rad * lat) * dlon * deg2rad
                    dxG[J, I] = 0.0 if v < 1.0 else v
                    dyG[J, I] = rSphere * dlat * deg2rad
                    # rA (ini_spherical_polar_grid.F:158-170)
                    rA[J, I] = rSphere * rSphere * dlon * deg2rad * abs(sin((lat + dlat) * deg2rad) - sin(lat * deg2rad))
                    # rAs (:183-197)
                    latc = f["yC"][t, J, I]
                    dlat2 = 0.5 * (dyl[J + 1] + dyl[J])
                    v = rSphere * rSphere * dlon * deg2rad * abs(sin(latc * deg2rad) - sin((latc - dlat2) * deg2rad))
                    rAs[J, I] = 0.0 if (abs(latc) > 90.0 or abs(latc - dlat2) > 90.0) else v
                    # rAz (:200-213)
                    latz = 0.5 * (YG[J, I] + YG[J + 1, I])
                    dlonz = 0.5 * (dxl[I + 1] + dxl[I])
                    v = rSphere * rSphere * dlonz * deg2rad * abs(sin(latz * deg2rad) - sin((latz - dlat2) * deg2rad))
                    rAz[J, I] = 0.0 if (abs(latz) > 90.0 or abs(latz - dlat2) > 90.0) else v
                    # tanPhiAtU/V (:216-223)
                    f["tanPhiAtU"][t, J, I] = tan(latz * deg2rad)
                    f["tanPhiAtV"][t, J, I] = tan(lat * deg2rad)
            f["dxC"][t, :, 1:] = 0.5 * (dxF[:, 1:] + dxF[:, :-1])
            f["dyC"][t, 1:, :] = 0.5 * (dyF[1:, :] + dyF[:-1, :])
            f["dxV"][t, 1:, 1:] = 0.5 * (dxG[1:, 1:] + dxG[1:, :-1])
            f["dyU"][t, 1:, 1:] = 0.5 * (dyG[1:, 1:] + dyG[:-1, 1:])
            f["rAw"][t, :, 1:] = 0.5 * (rA[:, 1:] + rA[:, :-1])
        self._reciprocals()

    def ini_curvilinear_grid(self, facet_records, radius_fromHorizGrid, rSphere, anglesFromFile):
        """INI_CURVILINEAR_GRID (model/src/ini_curvilinear_grid.F:238-340, OLD_GRID_IO
        undefined) + CALC_GRID_ANGLES (calc_grid_angles.F).  facet_records[f] is the
        (nrec, fNy+1, fNx+1) content of facet f's grid file (tileNNN.mitgrid or
        <horizGridFile>.faceNNN.bin): XC YC DXF DYF RA XG YG DXV DYU RAZ DXC DYC RAW RAS
        DXG DYG [AngleCS AngleSN].  MDS_FACEF_READ_RS (pkg/mdsio/mdsio_facef_read.F:83-99)
        puts rows tBy+1..tBy+sNy+1, columns tBx+1..tBx+sNx+1 at (1..sNx+1, 1..sNy+1)."""
        names = ("xC", "yC", "dxF", "dyF", "rA", "xG", "yG", "dxV", "dyU", "rAz", "dxC", "dyC", "rAw", "rAs",
                 "dxG", "dyG", "angleCosC", "angleSinC")
        topo = self.topo
        f = {n: self.z2() for n in names}           # INI_GRID zeroes every array first
        f["angleCosC"][:] = 1.0
        nrec = 18 if anglesFromFile else 16
        for t in range(self.nTiles):
            tid = t + 1
            rec = facet_records[topo.face[tid] - 1]
            tbx, tby = topo.tBx[tid], topo.tBy[tid]
            for r in range(nrec):
                f[names[r]][t, self.OLy:self.OLy + self.sNy + 1, self.OLx:self.OLx + self.sNx + 1] = \
                    rec[r, tby:tby + self.sNy + 1, tbx:tbx + self.sNx + 1]
        f["xC"] = topo.exchange(f["xC"])
        f["yC"] = topo.exchange(f["yC"])
        f["dxF"], f["dyF"] = topo.exchange_uv_agrid(f["dxF"], f["dyF"], False)
        f["rA"] = topo.exchange(f["rA"])
        f["xG"] = topo.exchange_z(f["xG"])
        f["yG"] = topo.exchange_z(f["yG"])
        f["dxV"], f["dyU"] = topo.exchange_uv_bgrid(f["dxV"], f["dyU"], False)
        f["rAz"] = topo.exchange_z(f["rAz"])
        f["dxC"], f["dyC"] = topo.exchange_uv(f["dxC"], f["dyC"], False)
        f["rAw"], f["rAs"] = topo.exchange_uv(f["rAw"], f["rAs"], False)
        f["dyG"], f["dxG"] = topo.exchange_uv(f["dyG"], f["dxG"], False)
        if rSphere != radius_fromHorizGrid:
            fac = rSphere / radius_fromHorizGrid
            fac2 = fac * fac
            for n in ("dxC", "dyC", "dxG", "dyG", "dxF", "dyF", "dxV", "dyU"):
                f[n] = f[n] * fac
            for n in ("rA", "rAz", "rAw", "rAs"):
                f[n] = f[n] * fac2
        self.rSphere = rSphere
        if not anglesFromFile:
            # CALC_GRID_ANGLES (calc_grid_angles.F:70-110)
            from math import sqrt
            deg2rad = 2.0 * np.pi / 360.0      # PI = 2*ASIN(1), ini_parms.F
            yG, dxG, dyG = f["yG"], f["dxG"], f["dyG"]
            uP, vP = self.z2(), self.z2()
            with np.errstate(divide="ignore", invalid="ignore"):
                uP[:, :-1, :] = np.where(dyG[:, :-1, :] > 0.0,
                                         -(yG[:, :-1, :] - yG[:, 1:, :]) * deg2rad / dyG[:, :-1, :], 0.0)
                vP[:, :, :-1] = np.where(dxG[:, :, :-1] > 0.0,
                                         (yG[:, :, :-1] - yG[:, :, 1:]) * deg2rad / dxG[:, :, :-1], 0.0)
            cs, sn = f["angleCosC"], f["angleSinC"]
            for t in range(self.nTiles):
                for J in range(self.ny - 1):
                    for I in range(self.nx - 1):
                        uC = 0.5 * (uP[t, J, I] + uP[t, J, I + 1])
                        vC = 0.5 * (vP[t, J, I] + vP[t, J + 1, I])
                        un = sqrt(uC * uC + vC * vC)
                        if un != 0.0:
                            un = 1.0 / un
                        cs[t, J, I] = uC * un
                        sn[t, J, I] = -vC * un
        f["angleSinC"], f["angleCosC"] = topo.exchange_uv_agrid(f["angleSinC"], f["angleCosC"], True)
        self.f.update(f)
        self._reciprocals()

    def _reciprocals(self):
        for n in ("dxG", "dyG", "dxC", "dyC", "dxF", "dyF", "dxV", "dyU", "rA", "rAs", "rAw", "rAz"):
            a = self.f[n]
            # 1/x, unlike x*(1/x) shortcuts: same as ini_grid.F:78-101
            r = np.zeros_like(a)
            nz = a != 0.0
            r[nz] = 1.0 / a[nz]
            self.f["recip_" + n] = r

    def ini_cori(self, f0=1e-4, beta=1e-11, selectCoriMap=1, omega=None):
        """INI_CORI (model/src/ini_cori.F:29-83)."""
        if selectCoriMap == 2:
            from math import cos, sin
            deg2rad = 2.0 * np.pi / 360.0
            if omega is None:
                omega = 2.0 * np.pi / 86164.0      # ini_parms.F:481-483, rotationPeriod default
            self.omega = omega
            sinv = np.vectorize(lambda x: sin(x * deg2rad), otypes=[np.float64])
            cosv = np.vectorize(lambda x: cos(x * deg2rad), otypes=[np.float64])
            self.f["fCori"] = 2.0 * omega * sinv(self.f["yC"])
            self.f["fCoriG"] = 2.0 * omega * sinv(self.f["yG"])
            self.f["fCoriCos"] = 2.0 * omega * cosv(self.f["yC"])
            return
        if selectCoriMap == 1:
            self.f["fCori"] = f0 + beta * self.f["yC"]
            self.f["fCoriG"] = f0 + beta * self.f["yG"]
        elif selectCoriMap == 0:
            self.f["fCori"] = np.full_like(self.f["yC"], f0)
            self.f["fCoriG"] = np.full_like(self.f["yC"], f0)
        else:
            raise NotImplementedError("selectCoriMap=%d" % selectCoriMap)

    # ---- depths and masks -----------------------------------------------------
    def ini_depths_masks(self, bathy, hFacMin=1.0, hFacMinDr=0.0, gBaro=9.81):
        """bathy: global (Ny, Nx) lat-lon array, or tile layout (nTiles, ny, nx) (interiors used);
        negative below sea level."""
        sNx, sNy, Nr = self.sNx, self.sNy, self.Nr
        rF, drF, recip_drF = self.f["rF"], self.f["drF"], self.f["recip_drF"]
        R_low, Ro_surf = self.z2(), self.z2()
        inner = self.sl(1, sNx, 1, sNy)
        for t in range(self.nTiles):
            bi, bj = t % self.nSx, t // self.nSx
            if bathy.ndim == 3:
                R_low[t][inner] = bathy[t][inner]
            else:
                R_low[t][inner] = bathy[bj * sNy:(bj + 1) * sNy, bi * sNx:(bi + 1) * sNx]
            Ro_surf[t][inner] = rF[0]
        R_low = self.exch(R_low)
        Ro_surf = self.exch(Ro_surf)
        rEmpty = rF[0]
        rLowW = self.z2(); rSurfW = self.z2(); rLowS = self.z2(); rSurfS = self.z2()
        rLowW[:, :, 0] = rEmpty; rSurfW[:, :, 0] = rEmpty
        rLowS[:, 0, :] = rEmpty; rSurfS[:, 0, :] = rEmpty
        rLowW[:, :, 1:] = np.maximum(R_low[:, :, :-1], R_low[:, :, 1:])
        rSurfW[:, :, 1:] = np.minimum(Ro_surf[:, :, :-1], Ro_surf[:, :, 1:])
        rLowS[:, 1:, :] = np.maximum(R_low[:, :-1, :], R_low[:, 1:, :])
        rSurfS[:, 1:, :] = np.minimum(Ro_surf[:, :-1, :], Ro_surf[:, 1:, :])
        hFacC = self.z3()
        for k in range(Nr):
            mn = max(hFacMin, min(hFacMinDr * recip_drF[k], 1.0))
            hl = (rF[k] - R_low) * recip_drF[k]
            hl = np.minimum(np.maximum(hl, 0.0), 1.0)
            hFacC[:, k] = np.where((hl < mn * 0.5) | (R_low >= Ro_surf), 0.0, np.maximum(hl, mn))
        tmp = np.zeros_like(R_low)
        for k in range(Nr):
            tmp = tmp + drF[k] * hFacC[:, k]
        R_low = rF[0] - tmp
        for k in range(Nr):
            mn = max(hFacMin, min(hFacMinDr * recip_drF[k], 1.0))
            hl = (rF[k] - Ro_surf) * recip_drF[k]
            hl = hFacC[:, k] - np.maximum(hl, 0.0)
            hl = np.maximum(hl, 0.0)
            hFacC[:, k] = np.where(hl < mn * 0.5, 0.0, np.maximum(hl, mn))
        tmp = np.zeros_like(R_low)
        kSurfC = np.full(R_low.shape, Nr + 1, dtype=np.int32)
        kLowC = np.zeros(R_low.shape, dtype=np.int32)
        for k in range(Nr):
            tmp = tmp + drF[k] * hFacC[:, k]
            kLowC[hFacC[:, k] != 0.0] = k + 1
        for k in range(Nr - 1, -1, -1):
            kSurfC[hFacC[:, k] != 0.0] = k + 1
        Ro_surf = R_low + tmp
        maskInC = np.where(kSurfC <= Nr, 1.0, 0.0)
        hFacW, hFacS = self.z3(), self.z3()
        for k in range(Nr):
            mn = max(hFacMin, min(hFacMinDr * recip_drF[k], 1.0))
            for rLow, rSurf, out in ((rLowW, rSurfW, hFacW), (rLowS, rSurfS, hFacS)):
                h1 = (rF[k] - rLow) * recip_drF[k]
                hl = np.minimum(h1, 1.0)
                h1 = np.where((hl < mn * 0.5) | (rLow >= rSurf), 0.0, np.maximum(hl, mn))
                h2 = (rF[k] - rSurf) * recip_drF[k]
                hl = h1 - np.maximum(h2, 0.0)
                out[:, k] = np.where(hl < mn * 0.5, 0.0, np.maximum(hl, mn))
        hFacW, hFacS = self.exch_uv(hFacW, hFacS)       # EXCH_UV_XYZ_RS(hFacW,hFacS,.FALSE.)
        kSurfW = np.full(R_low.shape, Nr + 1, dtype=np.int32)
        kSurfS = np.full(R_low.shape, Nr + 1, dtype=np.int32)
        for k in range(Nr - 1, -1, -1):
            kSurfW[hFacW[:, k] != 0.0] = k + 1
            kSurfS[hFacS[:, k] != 0.0] = k + 1
        # ini_masks_etc.F:218-231 recip_Rcol; :325-399 rLow/rSurf at U and V points from the
        # adjusted R_low / Ro_surf, rSurf = rLow + Sum_k drF*hFac (EXCH_UV_XY_RS afterwards)
        col = Ro_surf - R_low
        recip_Rcol = np.zeros_like(col)
        recip_Rcol[col > 0.0] = 1.0 / col[col > 0.0]
        rLowW, rLowS = self.z2(), self.z2()
        rLowW[:, :, 1:] = np.maximum(R_low[:, :, :-1], R_low[:, :, 1:])
        rLowS[:, 1:, :] = np.maximum(R_low[:, :-1, :], R_low[:, 1:, :])
        tW, tS = np.zeros_like(R_low), np.zeros_like(R_low)
        for k in range(Nr):
            tW = tW + drF[k] * hFacW[:, k]
            tS = tS + drF[k] * hFacS[:, k]
        rSurfW, rSurfS = rLowW + tW, rLowS + tS
        f = self.f
        rLowW, rLowS = self.exch_uv(rLowW, rLowS)       # ini_masks_etc.F: EXCH_UV_XY_RS(.FALSE.)
        rSurfW, rSurfS = self.exch_uv(rSurfW, rSurfS)
        f.update(recip_Rcol=recip_Rcol, rLowW=rLowW, rLowS=rLowS, rSurfW=rSurfW,
                 rSurfS=rSurfS, h0FacC=hFacC.copy(), h0FacW=hFacW.copy(), h0FacS=hFacS.copy())
        f.update(R_low=R_low, Ro_surf=Ro_surf, hFacC=hFacC, hFacW=hFacW, hFacS=hFacS, maskInC=maskInC,
                 maskInW=np.where(kSurfW <= Nr, 1.0, 0.0), maskInS=np.where(kSurfS <= Nr, 1.0, 0.0))
        self.i.update(kSurfC=kSurfC, kLowC=kLowC, kSurfW=kSurfW, kSurfS=kSurfS)
        for c in "CWS":
            h = f["hFac" + c]
            nz = h != 0.0
            r = np.zeros_like(h)
            r[nz] = 1.0 / h[nz]
            f["recip_hFac" + c] = r
            f["mask" + c] = np.where(nz, 1.0, 0.0)
        # INI_LINEAR_PHISURF, z-coordinates
        f["Bo_surf"] = np.full_like(R_low, gBaro)
        f["recip_Bo"] = np.full_like(R_low, 1.0 / gBaro)
        # globalArea: GLOBAL_SUM_TILE_RL of the tile sums of rA*maskInC (interior)
        ga = 0.0
        for t in range(self.nTiles):
            ta = 0.0
            a = (f["rA"][t] * maskInC[t])[inner]
            for v in a.ravel():
                ta = ta + v
            ga = ga + ta
        self.globalArea = ga

    # ---- elliptic operator ----------------------------------------------------
    def ini_cg2d(self, deltaTMom, deltaTFreeSurf, cg2dTargetResidual, cg2dTargetResWunit=-1.0,
                 cg2dpcOffDFac=0.51, freeSurfFac=1.0, implicSurfPress=1.0, implicDiv2DFlow=1.0):
        sNx, sNy, Nr = self.sNx, self.sNy, self.Nr
        f = self.f
        aW, aS = self.z2(), self.z2()
        inner = self.sl(1, sNx, 1, sNy)
        for k in range(Nr):
            fa = f["dyG"] * f["drF"][k] * f["hFacW"][:, k]
            aW[(slice(None),) + inner] = (aW + implicSurfPress * implicDiv2DFlow * fa * f["recip_dxC"])[(slice(None),) + inner]
            fa = f["dxG"] * f["drF"][k] * f["hFacS"][:, k]
            aS[(slice(None),) + inner] = (aS + implicSurfPress * implicDiv2DFlow * fa * f["recip_dyC"])[(slice(None),) + inner]
        myNorm = max(np.abs(aW[(slice(None),) + inner]).max(), np.abs(aS[(slice(None),) + inner]).max(), 0.0)
        myNorm = 1.0 / myNorm if myNorm != 0.0 else 1.0
        aW[(slice(None),) + inner] = aW[(slice(None),) + inner] * myNorm
        aS[(slice(None),) + inner] = aS[(slice(None),) + inner] * myNorm
        aW, aS = self.exch_uv(aW, aS)                   # ini_cg2d.F:138 EXCH_UV_XY_RS(.FALSE.)
        self.cg2dNorm = myNorm
        self.cg2dNormaliseRHS = cg2dTargetResWunit <= 0.0
        tol = cg2dTargetResidual if self.cg2dNormaliseRHS else \
            myNorm * cg2dTargetResWunit * self.globalArea / deltaTMom
        self.cg2dTolerance_sq = tol * tol
        aC = self.z2()
        s0 = self.sl(0, sNx, 0, sNy)
        aWe = np.roll(aW, -1, axis=2)
        aSn = np.roll(aS, -1, axis=1)
        val = -(aW + aWe + aS + aSn + freeSurfFac * myNorm * f["recip_Bo"] * f["rA"] / deltaTMom / deltaTFreeSurf)
        aC[(slice(None),) + s0] = val[(slice(None),) + s0]
        pC, pW, pS = self.z2(), self.z2(), self.z2()
        acw = np.roll(aC, 1, axis=2)
        acs = np.roll(aC, 1, axis=1)
        with np.errstate(divide="ignore", invalid="ignore"):
            pCv = np.where(aC == 0.0, 1.0, 1.0 / aC)
            dW = cg2dpcOffDFac * (acw + aC)
            pWv = np.where(aC + acw == 0.0, 0.0, -aW / (dW * dW))
            dS = cg2dpcOffDFac * (acs + aC)
            pSv = np.where(aC + acs == 0.0, 0.0, -aS / (dS * dS))
        for dst, src in ((pC, pCv), (pW, pWv), (pS, pSv)):
            dst[(slice(None),) + inner] = src[(slice(None),) + inner]
        pW, pS = self.exch_uv(pW, pS)                   # ini_cg2d.F:233-234
        f.update(aW2d=aW, aS2d=aS, aC2d=aC, pC=self.exch(pC), pW=pW, pS=pS)
