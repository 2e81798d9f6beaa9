"""Tile topologies: which interior point every halo point is a copy of.

LatLonTopology restates EXCH1 (eesupp/src/exch1_rx.template:8-276): periodic
in both directions over the nSx x nSy tile layout (the default when no OBCS /
EXCH2 topology is configured).  The same map drives the host exchange (numpy,
used at initialisation) and the device halo kernels (mgcm_set_halo_map).
"""
import numpy as np


class LatLonTopology:
    def __init__(self, sNx, sNy, OLx, OLy, nSx=1, nSy=1):
        self.sNx, self.sNy, self.OLx, self.OLy, self.nSx, self.nSy = sNx, sNy, OLx, OLy, nSx, nSy
        self.nx, self.ny = sNx + 2 * OLx, sNy + 2 * OLy
        self.nTiles = nSx * nSy
        self._src = None

    def src_of_point(self):
        """Flat (t, j, i) source offset of every halo-inclusive point (itself for interior)."""
        if self._src is not None:
            return self._src
        sNx, sNy, OLx, OLy = self.sNx, self.sNy, self.OLx, self.OLy
        Nx, Ny = sNx * self.nSx, sNy * self.nSy
        n2 = self.nx * self.ny
        src = np.arange(self.nTiles * n2, dtype=np.int64).reshape(self.nTiles, self.ny, self.nx)
        jj, ii = np.meshgrid(np.arange(1 - OLy, sNy + OLy + 1), np.arange(1 - OLx, sNx + OLx + 1), indexing="ij")
        for t in range(self.nTiles):
            bi, bj = t % self.nSx, t // self.nSx
            iG = (bi * sNx + ii - 1) % Nx
            jG = (bj * sNy + jj - 1) % Ny
            st = (jG // sNy) * self.nSx + iG // sNx
            si, sj = iG % sNx + 1, jG % sNy + 1
            s = st * n2 + (sj + OLy - 1) * self.nx + (si + OLx - 1)
            halo = (ii < 1) | (ii > sNx) | (jj < 1) | (jj > sNy)
            src[t][halo] = s[halo]
        self._src = src.ravel()
        return self._src

    def exchange(self, a):
        """Return a copy of `a` (nTiles, [nz,] ny, nx) with every halo point refreshed."""
        src = self.src_of_point()
        a = np.array(a, dtype=np.float64, copy=True)
        if a.ndim == 3:
            flat = a.reshape(-1)
            flat[:] = flat[src]
            return a
        nt, nz = a.shape[0], a.shape[1]
        b = np.moveaxis(a, 1, 0).reshape(nz, -1)   # (nz, nTiles*n2)
        b = b[:, src]
        return np.moveaxis(b.reshape(nz, nt, self.ny, self.nx), 0, 1).copy()

    # vector / staggered variants: on the lat-lon (EXCH1) topology every component is a
    # plain scalar copy (exch_uv_xy_rx.template:87-95, exch_z_3d_rx.template:71)
    def exchange_uv(self, u, v, withSigns=True):
        return self.exchange(u), self.exchange(v)

    exchange_uv_agrid = exchange_uv
    exchange_uv_bgrid = exchange_uv

    def exchange_z(self, a):
        return self.exchange(a)
