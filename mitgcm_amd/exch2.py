"""pkg/exch2 restated as halo maps: cube and LLC facet topologies.

Exch2Topology builds the tile-to-tile connectivity of pkg/exch2 from the facet
dimensions and the facet edge links (W2_SET_CS6_FACETS, W2_SET_MAP_TILES,
W2_SET_F2F_INDEX, W2_SET_TILE2TILES) and then derives, once, which value every
halo point ends up holding after each of the reference's exchange routines:

  scalar      EXCH2_3D_RX        (pkg/exch2/exch2_3d_rx.template)
  uv C-grid   EXCH2_UV_3D_RX     (exch2_uv_3d_rx.template -> EXCH2_RX2_CUBE 'Cg')
  uv A-grid   EXCH2_UV_AGRID_3D_RX (exch2_uv_agrid_3d_rx.template)
  z-point     EXCH2_Z_3D_RX      (exch2_z_3d_rx.template)

It does so by running the reference's sequence of copies (two EXCH2_RX1/RX2
passes, "ignore corners" then "update corners", each pass reading a snapshot
because every PUT precedes every GET, then the per-face corner fix-ups) on
arrays of source ids instead of values.  The result is a gather map: for every
halo point, the interior point it copies (and, for vectors, from which
component and with which sign).  The device applies the maps with one gather
kernel per exchange (mgcm_set_halo_map / mgcm_set_uv_map); the oracle applies
the same maps on the CPU.
"""
import numpy as np

EDGE_N, EDGE_S, EDGE_E, EDGE_W = 1, 2, 3, 4


def cs6_facet_links():
    """W2_SET_CS6_FACETS (pkg/exch2/w2_set_cs6_facets.F:77-99): facet_link(i,j) for
    edges i = N,S,E,W of the 6 cube faces, as (facet, edge) pairs (1-based)."""
    links = {}
    for j in range(1, 7):
        w = lambda jj: 1 + (jj + 5) % 6
        if j % 2 == 1:
            links[j] = [(w(j + 2), EDGE_W), (w(j - 1), EDGE_N), (w(j + 1), EDGE_W), (w(j - 2), EDGE_N)]
        else:
            links[j] = [(w(j + 1), EDGE_S), (w(j - 2), EDGE_E), (w(j + 2), EDGE_S), (w(j - 1), EDGE_E)]
    return links


class Exch2Topology:
    """facet_dims: [(nx, ny)] per facet; links: {facet: [(facet, edge)] for N,S,E,W}
    (edge 0 / facet 0 = disconnected).  Tiles of sNx x sNy, numbered facet by facet,
    x fastest within a facet (w2_set_map_tiles.F:150-175)."""

    def __init__(self, facet_dims, links, sNx, sNy, OLx, OLy):
        if OLx != OLy:
            raise ValueError("exch2: OLx != OLy not supported (exchange width is OLx, exch2_3d_rx.template)")
        self.sNx, self.sNy, self.OLx, self.OLy = sNx, sNy, OLx, OLy
        self.nx, self.ny = sNx + 2 * OLx, sNy + 2 * OLy
        self.n2 = self.nx * self.ny
        self.facet_dims = list(facet_dims)
        self.links = links
        self.nSy = 1
        self._f2f_index()
        self._map_tiles()
        self._tile2tiles()
        self.nTiles = self.nSx = self.nTiles_
        self._cache = {}

    # ---------------------------------------------------------------- set-up
    def _f2f_index(self):
        """W2_SET_F2F_INDEX (w2_set_f2f_index.F:120-213): index transform from the
        facet across edge i of facet j to facet j's own (extended) index space."""
        self.fpij, self.foi, self.foj = {}, {}, {}
        dims = self.facet_dims
        for j in range(1, len(dims) + 1):
            for i in range(1, 5):
                jj, ii = self.links[j][i - 1]
                if jj < 1:
                    continue
                # lo = facet_dims(2*(j-1)+(i+1)/2): x-size for N/S edges, y-size for E/W
                lo = dims[j - 1][0] if (i + 1) // 2 == 1 else dims[j - 1][1]
                p = [1, 0, 0, 1]
                if i == 1 and ii == 2:
                    oi, oj = 0, dims[j - 1][1]
                elif i == 2 and ii == 1:
                    oi, oj = 0, -dims[jj - 1][1]
                elif i == 3 and ii == 4:
                    oi, oj = dims[j - 1][0], 0
                elif i == 4 and ii == 3:
                    oi, oj = -dims[jj - 1][0], 0
                elif i == 1 and ii == 4:
                    p = [0, -1, 1, 0]
                    oi, oj = lo + 1, dims[j - 1][1]
                elif i == 2 and ii == 3:
                    p = [0, -1, 1, 0]
                    oi, oj = lo + 1, -dims[jj - 1][0]
                elif i == 3 and ii == 2:
                    p = [0, 1, -1, 0]
                    oi, oj = dims[j - 1][0], lo + 1
                elif i == 4 and ii == 1:
                    p = [0, 1, -1, 0]
                    oi, oj = -dims[jj - 1][1], lo + 1
                else:
                    raise ValueError("exch2: unsupported edge pairing %d.%d -> %d.%d" % (j, i, jj, ii))
                self.fpij[(i, j)] = p
                self.foi[(i, j)], self.foj[(i, j)] = oi, oj

    def _map_tiles(self):
        """W2_SET_MAP_TILES (w2_set_map_tiles.F:61-175), no blank tiles."""
        self.face, self.tBx, self.tBy, self.fNx, self.fNy = [None], [None], [None], [None], [None]
        self.facet_first = {}
        for j, (fNx, fNy) in enumerate(self.facet_dims, start=1):
            if fNx % self.sNx or fNy % self.sNy:
                raise ValueError("exch2: facet %d (%dx%d) not divisible into %dx%d tiles" %
                                 (j, fNx, fNy, self.sNx, self.sNy))
            self.facet_first[j] = len(self.face)
            for ty in range(fNy // self.sNy):
                for tx in range(fNx // self.sNx):
                    self.face.append(j)
                    self.tBx.append(tx * self.sNx)
                    self.tBy.append(ty * self.sNy)
                    self.fNx.append(fNx)
                    self.fNy.append(fNy)
        self.face = self.face      # 1-based tile ids: index 0 unused
        n = len(self.face) - 1
        self.face_of = np.array(self.face[1:])
        self.nTiles_ = n

    def _tile2tiles(self):
        """W2_SET_TILE2TILES (w2_set_tile2tiles.F:83-262): neighbours of every tile,
        their index transforms and halo ranges; edge flags; opposingSend."""
        sNx, sNy = self.sNx, self.sNy
        n = self.nTiles_
        self.nbr = {t: [] for t in range(1, n + 1)}   # (tile, pij, oi, oj, iLo, iHi, jLo, jHi, edge2edge)
        self.isN = [0] * (n + 1)
        self.isS = [0] * (n + 1)
        self.isE = [0] * (n + 1)
        self.isW = [0] * (n + 1)
        for is_ in range(1, n + 1):
            js = self.face[is_]
            iLo, iHi = self.tBx[is_] + 1, self.tBx[is_] + sNx
            jLo, jHi = self.tBy[is_] + 1, self.tBy[is_] + sNy
            for i in range(1, 5):
                ii1, ii2, jj1, jj2 = iLo, iHi, jLo, jHi
                if i == 1:
                    jj1 = jj2 = jHi + 1
                    intern = jHi < self.fNy[is_]
                    if not intern:
                        self.isN[is_] = 1
                elif i == 2:
                    jj1 = jj2 = jLo - 1
                    intern = jLo > 1
                    if not intern:
                        self.isS[is_] = 1
                elif i == 3:
                    ii1 = ii2 = iHi + 1
                    intern = iHi < self.fNx[is_]
                    if not intern:
                        self.isE[is_] = 1
                else:
                    ii1 = ii2 = iLo - 1
                    intern = iLo > 1
                    if not intern:
                        self.isW[is_] = 1
                ddi = min(ii2 - ii1, 1)
                ddj = min(jj2 - jj1, 1)
                if intern:
                    nbTx = self.facet_dims[js - 1][0] // sNx
                    ii = 1 + i % 2
                    it = 2 * ii - 3
                    if i <= 2:
                        it = is_ + it * nbTx
                    else:
                        it = is_ + it
                        ii = ii + 2
                    self.nbr[is_].append(dict(
                        tile=it, pij=[1, 0, 0, 1], oi=0, oj=0,
                        iLo=ii1 - ddi - self.tBx[is_], iHi=ii2 + ddi - self.tBx[is_],
                        jLo=jj1 - ddj - self.tBy[is_], jHi=jj2 + ddj - self.tBy[is_], e2e=10 * i + ii))
                else:
                    jt, ii = self.links[js][i - 1]
                    if jt <= 0:
                        continue
                    fp, fo_i, fo_j = self.fpij[(ii, jt)], self.foi[(ii, jt)], self.foj[(ii, jt)]
                    ib1 = fp[0] * ii1 + fp[1] * jj1 + fo_i
                    ib2 = fp[0] * ii2 + fp[1] * jj2 + fo_i
                    jb1 = fp[2] * ii1 + fp[3] * jj1 + fo_j
                    jb2 = fp[2] * ii2 + fp[3] * jj2 + fo_j
                    tx1, tx2 = sorted(((ib1 - 1) // sNx, (ib2 - 1) // sNx))
                    ty1, ty2 = sorted(((jb1 - 1) // sNy, (jb2 - 1) // sNy))
                    nbTx = self.facet_dims[jt - 1][0] // sNx
                    mp, mo_i, mo_j = self.fpij[(i, js)], self.foi[(i, js)], self.foj[(i, js)]
                    for ty in range(ty1, ty2 + 1):
                        for tx in range(tx1, tx2 + 1):
                            it = self.facet_first[jt] + tx + ty * nbTx
                            cl = lambda v, b, nn: min(max(v, b + 1), b + nn)
                            itb1 = cl(ib1, self.tBx[it], sNx)
                            itb2 = cl(ib2, self.tBx[it], sNx)
                            jtb1 = cl(jb1, self.tBy[it], sNy)
                            jtb2 = cl(jb2, self.tBy[it], sNy)
                            isb1 = mp[0] * itb1 + mp[1] * jtb1 + mo_i
                            isb2 = mp[0] * itb2 + mp[1] * jtb2 + mo_i
                            jsb1 = mp[2] * itb1 + mp[3] * jtb1 + mo_j
                            jsb2 = mp[2] * itb2 + mp[3] * jtb2 + mo_j
                            self.nbr[is_].append(dict(
                                tile=it, pij=list(mp), oi=mo_i, oj=mo_j,
                                iLo=isb1 - ddi - self.tBx[is_], iHi=isb2 + ddi - self.tBx[is_],
                                jLo=jsb1 - ddj - self.tBy[is_], jHi=jsb2 + ddj - self.tBy[is_], e2e=10 * i + ii))
        # exch2_opposingSend (w2_set_tile2tiles.F:285-315)
        for is_ in range(1, n + 1):
            for ns, nb in enumerate(self.nbr[is_]):
                i = nb["e2e"] // 10
                it = nb["tile"]
                opp = [nt for nt, nb2 in enumerate(self.nbr[it]) if nb2["tile"] == is_ and nb2["e2e"] % 10 == i]
                if len(opp) != 1:
                    raise ValueError("exch2: tile %d neighbour %d: %d opposing connections" % (is_, ns, len(opp)))
                nb["opp"] = opp[0]

    # ------------------------------------------------- W2_EXCH2_TOPOLOGY.h arrays
    def w2_arrays(self, ldNb=None, ldT=None):
        """The topology as the COMMON blocks of pkg/exch2/W2_EXCH2_TOPOLOGY.h hold it after
        W2_E2SETUP (w2_e2setup.F -> w2_set_map_tiles.F, w2_set_tile2tiles.F), Fortran layout
        (first index fastest): exch2_myFace, exch2_tBasex/y, exch2_is{N,S,E,W}edge,
        exch2_nNeighbours (nTiles); exch2_neighbourId, exch2_opposingSend, exch2_neighbourDir,
        exch2_oi/oj, exch2_iLo/iHi/jLo/jHi (ldNb, ldT); exch2_pij (4, ldNb, ldT) -- int32
        arrays, what a Fortran host passes to the device library (mgcm_exch2_maps)."""
        n = self.nTiles_
        maxNb = max(len(self.nbr[t]) for t in range(1, n + 1))
        ldNb = ldNb or maxNb
        ldT = ldT or n
        if maxNb > ldNb or n > ldT:
            raise ValueError("w2_arrays: %d tiles / %d neighbours exceed (%d, %d)" % (n, maxNb, ldT, ldNb))
        z = lambda *shape: np.zeros(shape, dtype=np.int32)
        a = {"exch2_myFace": z(ldT), "exch2_tBasex": z(ldT), "exch2_tBasey": z(ldT), "exch2_isNedge": z(ldT),
             "exch2_isSedge": z(ldT), "exch2_isEedge": z(ldT), "exch2_isWedge": z(ldT), "exch2_nNeighbours": z(ldT)}
        for k in ("neighbourId", "opposingSend", "neighbourDir", "oi", "oj", "iLo", "iHi", "jLo", "jHi"):
            a["exch2_" + k] = z(ldT, ldNb)
        a["exch2_pij"] = z(ldT, ldNb, 4)
        for t in range(1, n + 1):
            a["exch2_myFace"][t - 1] = self.face[t]
            a["exch2_tBasex"][t - 1], a["exch2_tBasey"][t - 1] = self.tBx[t], self.tBy[t]
            a["exch2_isNedge"][t - 1], a["exch2_isSedge"][t - 1] = self.isN[t], self.isS[t]
            a["exch2_isEedge"][t - 1], a["exch2_isWedge"][t - 1] = self.isE[t], self.isW[t]
            a["exch2_nNeighbours"][t - 1] = len(self.nbr[t])
            for q, nb in enumerate(self.nbr[t]):
                a["exch2_neighbourId"][t - 1, q] = nb["tile"]
                a["exch2_opposingSend"][t - 1, q] = nb["opp"] + 1
                a["exch2_neighbourDir"][t - 1, q] = nb["e2e"] // 10
                a["exch2_pij"][t - 1, q] = nb["pij"]
                for k in ("oi", "oj", "iLo", "iHi", "jLo", "jHi"):
                    a["exch2_" + k][t - 1, q] = nb[k]
        a["ldNb"], a["ldT"] = ldNb, ldT
        return a

    # ---------------------------------------------------------- index helpers
    def g(self, t, i, j):
        """flat offset of local point (i, j) (1-based, halo-inclusive) of 1-based tile t"""
        return (t - 1) * self.n2 + (j + self.OLy - 1) * self.nx + (i + self.OLx - 1)

    def is_interior(self, g):
        l = g % self.n2
        i, j = l % self.nx - self.OLx + 1, l // self.nx - self.OLy + 1
        return 1 <= i <= self.sNx and 1 <= j <= self.sNy

    # --------------------------------------------------- reference exchanges
    def _scal_bounds(self, t, nb, eW, upd):
        """EXCH2_GET_SCAL_BOUNDS (exch2_get_scal_bounds.F:56-133)"""
        iLo, iHi, jLo, jHi = nb["iLo"], nb["iHi"], nb["jLo"], nb["jHi"]
        si = sj = 1
        if iLo == iHi and iLo == 0:
            iLo = 1 - eW
            si = 1
            sj = 1 if jLo <= jHi else -1
            jLo, jHi = (jLo - sj * (eW - 1), jHi + sj * (eW - 1)) if upd else (jLo + sj, jHi - sj)
        if iLo == iHi and iLo > 1:
            iHi = iHi + eW - 1
            si = 1
            sj = 1 if jLo <= jHi else -1
            jLo, jHi = (jLo - sj * (eW - 1), jHi + sj * (eW - 1)) if upd else (jLo + sj, jHi - sj)
        if jLo == jHi and jLo == 0:
            jLo = 1 - eW
            sj = 1
            si = 1 if iLo <= iHi else -1
            iLo, iHi = (iLo - si * (eW - 1), iHi + si * (eW - 1)) if upd else (iLo + si, iHi - si)
        if jLo == jHi and jLo > 1:
            jHi = jHi + eW - 1
            sj = 1
            si = 1 if iLo <= iHi else -1
            iLo, iHi = (iLo - si * (eW - 1), iHi + si * (eW - 1)) if upd else (iLo + si, iHi - si)
        return iLo, iHi, jLo, jHi, si, sj

    @staticmethod
    def _rng(lo, hi, st):
        return range(lo, hi + st, st) if (hi - lo) * st >= 0 else range(0)

    def _rx1_pass(self, ids, sg, upd):
        """one EXCH2_RX1_CUBE pass (exch2_rx1_cube.template:92-258): all PUTs read the
        array (snapshot) before any GET writes; GETs in neighbour order."""
        src_ids, src_sg = ids.copy(), sg.copy()
        eW = self.OLx
        for t in range(1, self.nTiles_ + 1):
            for nb in self.nbr[t]:
                S = nb["tile"]
                snb = self.nbr[S][nb["opp"]]
                p, oi, oj = snb["pij"], snb["oi"], snb["oj"]
                iLo, iHi, jLo, jHi, si, sj = self._scal_bounds(t, nb, eW, upd)
                for jl in self._rng(jLo, jHi, sj):
                    for il in self._rng(iLo, iHi, si):
                        itc, jtc = il + self.tBx[t], jl + self.tBy[t]
                        isl = p[0] * itc + p[1] * jtc + oi - self.tBx[S]
                        jsl = p[2] * itc + p[3] * jtc + oj - self.tBy[S]
                        self._chk(S, isl, jsl)
                        d, s = self.g(t, il, jl), self.g(S, isl, jsl)
                        ids[d], sg[d] = src_ids[s], src_sg[s]

    def _chk(self, S, isl, jsl):
        if not (1 - self.OLx <= isl <= self.sNx + self.OLx and 1 - self.OLy <= jsl <= self.sNy + self.OLy):
            raise ValueError("exch2: source (%d,%d) of tile %d out of bounds" % (isl, jsl, S))

    def _uv_bounds(self, t, nb, eW, upd, cg):
        """EXCH2_GET_UV_BOUNDS (exch2_get_uv_bounds.F:84-262) for target tile t, neighbour nb"""
        tIlo, tIhi, tJlo, tJhi = nb["iLo"], nb["iHi"], nb["jLo"], nb["jHi"]
        S = nb["tile"]
        snb = self.nbr[S][nb["opp"]]
        p = snb["pij"]
        oi1 = oi2 = snb["oi"]
        oj1 = oj2 = snb["oj"]
        si = sj = 1
        I1 = J1 = None
        if tIlo == tIhi and tIlo == 0:
            i1, i1h = 1 - eW, 0
            si = 1
            sj = 1 if tJlo <= tJhi else -1
            j1, j1h = (tJlo - sj * (eW - 1), tJhi + sj * (eW - 1)) if upd else (tJlo + sj, tJhi - sj)
            I1 = (i1, i1h); J1 = (j1, j1h)
        if tIlo == tIhi and tIlo > 1:
            i1, i1h = tIlo, tIhi + eW - 1
            si = 1
            sj = 1 if tJlo <= tJhi else -1
            j1, j1h = (tJlo - sj * (eW - 1), tJhi + sj * (eW - 1)) if upd else (tJlo + sj, tJhi - sj)
            I1 = (i1, i1h); J1 = (j1, j1h)
        if tJlo == tJhi and tJlo == 0:
            j1, j1h = 1 - eW, 0
            sj = 1
            si = 1 if tIlo <= tIhi else -1
            i1, i1h = (tIlo - si * (eW - 1), tIhi + si * (eW - 1)) if upd else (tIlo + si, tIhi - si)
            I1 = (i1, i1h); J1 = (j1, j1h)
        if tJlo == tJhi and tJlo > 1:
            j1, j1h = tJlo, tJhi + eW - 1
            sj = 1
            si = 1 if tIlo <= tIhi else -1
            i1, i1h = (tIlo - si * (eW - 1), tIhi + si * (eW - 1)) if upd else (tIlo + si, tIhi - si)
            I1 = (i1, i1h); J1 = (j1, j1h)
        (i1, i1h), (j1, j1h) = I1, J1
        (i2, i2h), (j2, j2h) = I1, J1
        if cg:
            if p[0] == -1:
                oi1 += 1
            if p[2] == -1:
                oj1 += 1
            if p[1] == -1:
                oi2 += 1
            if p[3] == -1:
                oj2 += 1
            if upd:
                if p[0] == -1 or p[2] == -1:
                    i1 += 1
                if p[1] == -1 or p[3] == -1:
                    j2 += 1
                if tIlo == tIhi and tIlo > 1:
                    if self.isS[t]:
                        j1 = tJlo + 1
                        j2 = tJlo + 1
                    if self.isN[t]:
                        j1h = tJhi - 1
                        j2h = tJhi
                if tJlo == tJhi and tJlo > 1:
                    if self.isW[t]:
                        i1 = tIlo + 1
                        i2 = tIlo + 1
                    if self.isE[t]:
                        i1h = tIhi
                        i2h = tIhi - 1
            else:
                if p[0] == -1 or p[2] == -1:
                    i1 += 1
                    i1h += 1
                if p[1] == -1 or p[3] == -1:
                    j2 += 1
                    j2h += 1
        return (i1, i1h, j1, j1h), (i2, i2h, j2, j2h), si, sj, (oi1, oj1, oi2, oj2), p, S

    def _rx2_pass(self, u, us, v, vs, upd, withSigns, cg=True):
        """one EXCH2_RX2_CUBE pass (exch2_rx2_cube.template + exch2_put_rx2.template:98-225)"""
        su, sus, sv, svs = u.copy(), us.copy(), v.copy(), vs.copy()
        eW = self.OLx
        for t in range(1, self.nTiles_ + 1):
            for nb in self.nbr[t]:
                r1, r2, si, sj, (oi1, oj1, oi2, oj2), p, S = self._uv_bounds(t, nb, eW, upd, cg)
                for comp, (ilo, ihi, jlo, jhi), oi, oj, coef in (
                        (0, r1, oi1, oj1, (p[0], p[2])), (1, r2, oi2, oj2, (p[1], p[3]))):
                    sa1, sa2 = coef
                    if not withSigns:
                        sa1, sa2 = abs(sa1), abs(sa2)
                    dst_id, dst_sg = (u, us) if comp == 0 else (v, vs)
                    for jl in self._rng(jlo, jhi, sj):
                        for il in self._rng(ilo, ihi, si):
                            itc, jtc = il + self.tBx[t], jl + self.tBy[t]
                            isl = p[0] * itc + p[1] * jtc + oi - self.tBx[S]
                            jsl = p[2] * itc + p[3] * jtc + oj - self.tBy[S]
                            self._chk(S, isl, jsl)
                            d, s = self.g(t, il, jl), self.g(S, isl, jsl)
                            if sa1 != 0:
                                dst_id[d], dst_sg[d] = su[s], sus[s] * sa1
                            else:
                                dst_id[d], dst_sg[d] = sv[s], svs[s] * sa2

    def _identity(self, nfield=1):
        N = self.nTiles_ * self.n2
        return [np.arange(N, dtype=np.int64) + f * N for f in range(nfield)], [np.ones(N, dtype=np.int64)
                                                                              for _ in range(nfield)]

    def scalar_ids(self):
        """EXCH2_3D_RX (exch2_3d_rx.template:60-70): source id of every point."""
        if "T" not in self._cache:
            (ids,), (sg,) = self._identity(1)
            self._rx1_pass(ids, sg, False)
            self._rx1_pass(ids, sg, True)
            self._cache["T"] = ids
        return self._cache["T"]

    def uv_ids(self, withSigns=True):
        """EXCH2_UV_3D_RX (exch2_uv_3d_rx.template:60-226), W2_USE_R1_ONLY undefined:
        (uid, usg, vid, vsg); ids < N refer to u, >= N to v."""
        key = ("UV", bool(withSigns))
        if key in self._cache:
            return self._cache[key]
        (u, v), (us, vs) = self._identity(2)
        self._rx2_pass(u, us, v, vs, False, withSigns)
        self._rx2_pass(u, us, v, vs, True, withSigns)
        sN, sE, sW, sS = self.isN, self.isE, self.isW, self.isS
        nX, nY, OL = self.sNx, self.sNy, self.OLx
        neg = -1 if withSigns else 1

        def cp(dst, dsg, d, src, ssg, s, f=1):
            dst[d], dsg[d] = src[s], ssg[s] * f
        for t in range(1, self.nTiles_ + 1):
            G = lambda i, j: self.g(t, i, j)
            if OL >= 2 and sW[t] and sS[t]:
                cp(u, us, G(0, 0), v, vs, G(1, 0))
                cp(v, vs, G(0, 0), u, us, G(0, 1))
            if OL >= 2 and sW[t] and sN[t]:
                cp(u, us, G(0, nY + 1), v, vs, G(1, nY + 2), neg)
                cp(v, vs, G(0, nY + 2), u, us, G(0, nY), neg)
            if OL >= 2 and sE[t] and sS[t]:
                cp(u, us, G(nX + 2, 0), v, vs, G(nX, 0), neg)
                cp(v, vs, G(nX + 1, 0), u, us, G(nX + 2, 1), neg)
            if OL >= 2 and sE[t] and sN[t]:
                cp(u, us, G(nX + 2, nY + 1), v, vs, G(nX, nY + 2))
                cp(v, vs, G(nX + 1, nY + 2), u, us, G(nX + 2, nY))
        self._cache[key] = (u, us, v, vs)
        return self._cache[key]

    def agrid_ids(self, withSigns):
        """EXCH2_UV_AGRID_3D_RX (exch2_uv_agrid_3d_rx.template:60-150)."""
        key = ("AG", bool(withSigns))
        if key in self._cache:
            return self._cache[key]
        (u, v), (us, vs) = self._identity(2)
        for a, s in ((u, us), (v, vs)):
            self._rx1_pass(a, s, False)
            self._rx1_pass(a, s, True)
        neg = -1 if withSigns else 1
        nX, nY, OL = self.sNx, self.sNy, self.OLx
        for t in range(1, self.nTiles_ + 1):
            uL, uLs, vL, vLs = u.copy(), us.copy(), v.copy(), vs.copy()
            G = lambda i, j: self.g(t, i, j)
            pts = []
            if self.face[t] % 2 == 1:
                if self.isN[t]:
                    pts += [(G(i, nY + j), -1) for j in range(1, OL + 1) for i in range(1 - OL, nX + OL + 1)]
                if self.isW[t]:
                    pts += [(G(1 - i, j), +1) for j in range(1 - OL, nY + OL + 1) for i in range(1, OL + 1)]
            else:
                if self.isE[t]:
                    pts += [(G(nX + i, j), +1) for j in range(1 - OL, nY + OL + 1) for i in range(1, OL + 1)]
                if self.isS[t]:
                    pts += [(G(i, 1 - j), -1) for j in range(1, OL + 1) for i in range(1 - OL, nX + OL + 1)]
            for d, which in pts:
                # which=-1: u = -v, v = u ; which=+1: u = v, v = -u   (negOne applied per the template)
                if which == -1:
                    u[d], us[d] = vL[d], vLs[d] * neg
                    v[d], vs[d] = uL[d], uLs[d]
                else:
                    u[d], us[d] = vL[d], vLs[d]
                    v[d], vs[d] = uL[d], uLs[d] * neg
        self._cache[key] = (u, us, v, vs)
        return self._cache[key]

    def bgrid_ids(self, withSigns):
        """EXCH2_UV_BGRID_3D_RX (exch2_uv_bgrid_3d_rx.template:58-330), B-grid (corner)
        vectors, W2_FILL_NULL_REGIONS undefined."""
        key = ("BG", bool(withSigns))
        if key in self._cache:
            return self._cache[key]
        (u, v), (us, vs) = self._identity(2)
        nX, nY, OL = self.sNx, self.sNy, self.OLx
        neg = -1 if withSigns else 1
        save = {t: {n: (a[self.g(t, *ij)], s[self.g(t, *ij)])
                    for n, a, s, ij in (("uNW", u, us, (1, nY + 1)), ("vNW", v, vs, (1, nY + 1)),
                                        ("uSE", u, us, (nX + 1, 1)), ("vSE", v, vs, (nX + 1, 1)))}
                for t in range(1, self.nTiles_ + 1)}
        for a, s in ((u, us), (v, vs)):
            self._rx1_pass(a, s, False)
            self._rx1_pass(a, s, True)
        for t in range(1, self.nTiles_ + 1):
            G = lambda i, j: self.g(t, i, j)
            uL, uLs, vL, vLs = u.copy(), us.copy(), v.copy(), vs.copy()
            odd = self.face[t] % 2 == 1

            def setL(di, dj, si_, sj_, fu, fv):   # u(d) = fu * vLoc(s); v(d) = fv * uLoc(s)
                d, s_ = G(di, dj), G(si_, sj_)
                u[d], us[d] = vL[s_], vLs[s_] * fu
                v[d], vs[d] = uL[s_], uLs[s_] * fv
            if odd:
                if self.isN[t]:
                    for j in range(1, OL + 1):
                        for i in range(1 - OL, nX + OL):
                            setL(i + 1, nY + j, i, nY + j, neg, 1)
                if self.isW[t]:
                    for j in range(1 - OL, nY + OL):
                        for i in range(1, OL + 1):
                            setL(1 - i, j + 1, 1 - i, j, 1, neg)
            else:
                if self.isE[t]:
                    for j in range(1 - OL, nY + OL):
                        for i in range(1, OL + 1):
                            setL(nX + i, j + 1, nX + i, j, 1, neg)
                if self.isS[t]:
                    for j in range(1, OL + 1):
                        for i in range(1 - OL, nX + OL):
                            setL(i + 1, 1 - j, i, 1 - j, neg, 1)

            def cp(dst, dsg, d, src, ssg, s, f=1):
                dst[G(*d)], dsg[G(*d)] = src[G(*s)], ssg[G(*s)] * f
            if self.isW[t] and self.isS[t]:
                for i in range(1, OL + 1):
                    if odd:
                        cp(v, vs, (1 - i, 1), u, us, (1, 1 - i), neg)
                        cp(u, us, (1 - i, 1), v, vs, (1, 1 - i))
                    else:
                        cp(u, us, (1, 1 - i), v, vs, (1 - i, 1), neg)
                        cp(v, vs, (1, 1 - i), u, us, (1 - i, 1))
            if self.isE[t] and self.isS[t]:
                if odd:
                    for i in range(2, OL + 1):
                        cp(u, us, (nX + 1, 2 - i), v, vs, (nX + i, 1))
                        cp(v, vs, (nX + 1, 2 - i), u, us, (nX + i, 1), neg)
                else:
                    d = G(nX + 1, 1)
                    u[d], us[d] = save[t]["uSE"]
                    v[d], vs[d] = save[t]["vSE"]
                    for i in range(2, OL + 1):
                        cp(u, us, (nX + i, 1), v, vs, (nX + 1, 2 - i), neg)
                        cp(v, vs, (nX + i, 1), u, us, (nX + 1, 2 - i))
            if self.isE[t] and self.isN[t]:
                for i in range(2, OL + 1):
                    if odd:
                        cp(u, us, (nX + i, nY + 1), v, vs, (nX + 1, nY + i))
                        cp(v, vs, (nX + i, nY + 1), u, us, (nX + 1, nY + i), neg)
                    else:
                        cp(u, us, (nX + 1, nY + i), v, vs, (nX + i, nY + 1), neg)
                        cp(v, vs, (nX + 1, nY + i), u, us, (nX + i, nY + 1))
            if self.isW[t] and self.isN[t]:
                if odd:
                    d = G(1, nY + 1)
                    u[d], us[d] = save[t]["uNW"]
                    v[d], vs[d] = save[t]["vNW"]
                    for i in range(2, OL + 1):
                        cp(u, us, (1, nY + i), v, vs, (2 - i, nY + 1))
                        cp(v, vs, (1, nY + i), u, us, (2 - i, nY + 1), neg)
                else:
                    for i in range(2, OL + 1):
                        cp(u, us, (2 - i, nY + 1), v, vs, (1, nY + i), neg)
                        cp(v, vs, (2 - i, nY + 1), u, us, (1, nY + i))
        self._cache[key] = (u, us, v, vs)
        return self._cache[key]

    def exchange_uv_bgrid(self, u, v, withSigns):
        return self._apply2(u, v, self.bgrid_ids(withSigns))

    def z_ids(self):
        """EXCH2_Z_3D_RX (exch2_z_3d_rx.template:37-200), W2_FILL_NULL_REGIONS undefined."""
        if "Z" in self._cache:
            return self._cache["Z"]
        (a,), (s,) = self._identity(1)
        nX, nY, OL = self.sNx, self.sNy, self.OLx
        phiNW = {t: a[self.g(t, 1, nY + 1)] for t in range(1, self.nTiles_ + 1)}
        phiSE = {t: a[self.g(t, nX + 1, 1)] for t in range(1, self.nTiles_ + 1)}
        self._rx1_pass(a, s, False)
        self._rx1_pass(a, s, True)
        for t in range(1, self.nTiles_ + 1):
            G = lambda i, j: self.g(t, i, j)

            def cp(di, dj, si_, sj_):
                a[G(di, dj)] = a[G(si_, sj_)]
            if self.face[t] % 2 == 0:
                if self.isE[t]:
                    for j in range(nY + OL, 2 - OL - 1, -1):
                        for i in range(nX + 1, nX + OL + 1):
                            cp(i, j, i, j - 1)
                    if self.isN[t]:
                        for j in range(nY + 2, nY + OL + 1):
                            cp(nX + 1, j, nX - nY + j, nY + 1)
                if self.isS[t]:
                    for j in range(1 - OL, 1):
                        for i in range(nX + OL, 2 - OL - 1, -1):
                            cp(i, j, i - 1, j)
                    if self.isE[t]:
                        a[G(nX + 1, 1)] = phiSE[t]
                        for i in range(nX + 2, nX + OL + 1):
                            cp(i, 1, nX + 1, nX + 2 - i)
                    if self.isW[t]:
                        for j in range(1 - OL, 1):
                            cp(1, j, j, 1)
                if self.isW[t] and self.isN[t]:
                    for i in range(2 - OL, 1):
                        cp(i, nY + 1, 1, nY + 2 - i)
            else:
                if self.isN[t]:
                    for j in range(nY + 1, nY + OL + 1):
                        for i in range(nX + OL, 2 - OL - 1, -1):
                            cp(i, j, i - 1, j)
                    if self.isE[t]:
                        for i in range(nX + 2, nX + OL + 1):
                            cp(i, nY + 1, nX + 1, nY - nX + i)
                if self.isW[t]:
                    for j in range(nY + OL, 2 - OL - 1, -1):
                        for i in range(1 - OL, 1):
                            cp(i, j, i, j - 1)
                    if self.isN[t]:
                        a[G(1, nY + 1)] = phiNW[t]
                        for j in range(nY + 2, nY + OL + 1):
                            cp(1, j, nY + 2 - j, nY + 1)
                    if self.isS[t]:
                        for i in range(1 - OL, 1):
                            cp(i, 1, 1, i)
                if self.isE[t] and self.isS[t]:
                    for j in range(2 - OL, 1):
                        cp(nX + 1, j, nX + 2 - j, 1)
        self._cache["Z"] = a
        return a

    # ------------------------------------------------------ applying the maps
    def src_of_point(self):
        """Scalar map in the mgcm_set_halo_map convention: source offset, or the point
        itself when it is left untouched."""
        return self.scalar_ids().copy()

    def uv_codes(self, withSigns=True):
        """Vector maps for mgcm_set_uv_map: per point of u (then v), 0 = untouched,
        +(src+1) / -(src+1) with src indexing [u | v]."""
        u, us, v, vs = self.uv_ids(withSigns)
        N = self.nTiles_ * self.n2
        ar = np.arange(N, dtype=np.int64)
        cu = np.where(u == ar, 0, (u + 1) * us)
        cv = np.where(v == ar + N, 0, (v + 1) * vs)
        return cu.astype(np.int64), cv.astype(np.int64)

    def exchange(self, a):
        """EXCH_XY/XYZ on (nTiles, [nz,] ny, nx) arrays."""
        return self._apply1(a, self.scalar_ids())

    def exchange_z(self, a):
        return self._apply1(a, self.z_ids())

    def _apply1(self, a, ids):
        a = np.array(a, dtype=np.float64, copy=True)
        if a.ndim == 3:
            return a.reshape(-1)[ids].reshape(a.shape)
        nt, nz = a.shape[0], a.shape[1]
        b = np.moveaxis(a, 1, 0).reshape(nz, -1)[:, ids]
        return np.moveaxis(b.reshape(nz, nt, self.ny, self.nx), 0, 1).copy()

    def _apply2(self, u, v, maps):
        uid, us, vid, vs = maps
        u = np.array(u, dtype=np.float64, copy=True)
        v = np.array(v, dtype=np.float64, copy=True)
        shp = u.shape
        if u.ndim == 3:
            uv = np.concatenate([u.reshape(-1), v.reshape(-1)])
            return (uv[uid] * us).reshape(shp), (uv[vid] * vs).reshape(shp)
        nt, nz = shp[0], shp[1]
        U = np.moveaxis(u, 1, 0).reshape(nz, -1)
        V = np.moveaxis(v, 1, 0).reshape(nz, -1)
        uv = np.concatenate([U, V], axis=1)
        ru = uv[:, uid] * us
        rv = uv[:, vid] * vs
        f = lambda r: np.moveaxis(r.reshape(nz, nt, self.ny, self.nx), 0, 1).copy()
        return f(ru), f(rv)

    def exchange_uv(self, u, v, withSigns=True):
        """EXCH_UV_XY(Z)_RL (C-grid vectors)."""
        return self._apply2(u, v, self.uv_ids(withSigns))

    def exchange_uv_agrid(self, u, v, withSigns):
        return self._apply2(u, v, self.agrid_ids(withSigns))


def cube_topology(nCube, sNx, sNy, OL):
    """6-face cube of nCube x nCube facets (preDefTopol=3 / default cube)."""
    return Exch2Topology([(nCube, nCube)] * 6, cs6_facet_links(), sNx, sNy, OL, OL)


def llc5_facet_links():
    """The 5-facet lat-lon-cap connectivity of utils/exch2/input/data.exch2.llc_120_5f
    (preDefTopol = 0, facetEdgeLink(1:4, j) = N, S, E, W of facet j as face.edge, 0 = open):
    facets 1, 2 (n x 3n), the Arctic cap 3 (n x n), facets 4, 5 (3n x n); the southern
    edges of 1, 2 and the eastern edges of 4, 5 are disconnected (Antarctica)."""
    N, S, E, W = EDGE_N, EDGE_S, EDGE_E, EDGE_W
    return {1: [(3, W), (0, 0), (2, W), (5, N)],
            2: [(3, S), (0, 0), (4, S), (1, E)],
            3: [(5, W), (2, N), (4, W), (1, N)],
            4: [(5, S), (2, E), (0, 0), (3, E)],
            5: [(1, W), (4, N), (0, 0), (3, N)]}


def llc_topology(n, sNx, sNy, OL):
    """LLC facets of size n (LLC-n: 13 tiles of n x n when sNx = sNy = n)."""
    dims = [(n, 3 * n), (n, 3 * n), (n, n), (3 * n, n), (3 * n, n)]
    return Exch2Topology(dims, llc5_facet_links(), sNx, sNy, OL, OL)
