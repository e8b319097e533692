"""Dam-break case definition: lattice, constants and map limits.

GenCase is a missing blob in the reference, so cases are
generated here.  The lattice/constant recipe is the SURVEY §8(c) one; the
oracle-side writer ``oracle/tools/gencase_ref.cpp`` produces the same particles
through the reference's own .bi4 code, and ``tests/test_case.py`` checks the two
agree bit for bit.

What the reference derives while loading a case is mirrored here so that
``SphCaseDef`` carries exactly what ``JSph`` would hold:

* constants are the XML text values (``%.10E`` for h, b and masses, as the case
  XML stores them) parsed back to double — ``JSph::LoadConfigCtes``
  (JSph.cpp:567-583) then narrows them to float inside the core;
* map limits follow ``JSph::LoadCaseParticles`` (JSph.cpp:2051-2062):
  ``JPartsLoad4::CalculeLimits`` (JPartsLoad4.cpp:339-347) with border
  ``double(float(h))*BORDER_MAP`` (DualSphDef.h:130), then
  ``JSph::ResizeMapLimits`` (JSph.cpp:1354-1387) with the case's
  ``<simulationdomain>`` ``posmax z="default + 50%"``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

BORDER_MAP = 0.05  # DualSphDef.h:130

STEP_VERLET, STEP_SYMPLECTIC = 1, 2
DDT_NONE, DDT_DDT, DDT_DDT2, DDT_DDT2FULL = 0, 1, 2, 3
CELLMODE_FULL, CELLMODE_HALF = 1, 2
CODE_TYPE_FIXED, CODE_TYPE_FLUID = 0x0, 0x1800


def _cround(v: float) -> int:
    """std::round (half away from zero) for v >= 0, exact in double."""
    r = math.floor(v)
    return int(r + 1 if v - r >= 0.5 else r)


def _xml_e10(v: float) -> float:
    """Value as written by ``%.10E`` in the case XML and parsed back."""
    return float("%.10E" % v)


@dataclass
class DamBreakCase:
    """3D dam break: tank 1.6 x 0.67 x 0.4 m, water column 0.4 x 0.67 x 0.3 m.

    Walls: bottom, x=0, x=1.6, y=0, y=0.67.
    """

    dp: float
    step_algorithm: int = STEP_VERLET
    tdensity: int = DDT_DDT2
    ddtvalue: float = 0.1
    visco: float = 0.1
    viscoboundfactor: float = 1.0
    cflnumber: float = 0.2
    verlet_steps: int = 40
    coefdtmin: float = 0.05
    rhopoutmin: float = 700.0
    rhopoutmax: float = 1300.0
    cellmode: int = CELLMODE_FULL
    celldomfixed: bool = False
    gravity: tuple = (0.0, 0.0, -9.81)
    rhop0: float = 1000.0
    gamma: float = 7.0
    coefsound: float = 20.0
    coefh: float = 1.0
    tboundary: int = 1  # 1 DBC, 2 mDBC (<parameter Boundary>, JSph.cpp:626-640)
    slipmode: int = 1  # mDBC: only SLIP_Vel0 in this fork (JSph.cpp:788)
    mdbc_threshold: float = 0.0  # -mdbc_threshold (JSphCfgRun.cpp:124)
    mdbc_corrector: int = 0  # <parameter MDBCCorrector> (JSph.cpp:639)
    # ViscoTreatment 1 artificial / 2 Laminar+SPS (then `visco` is the kinematic viscosity,
    # e.g. 1e-6), shifting mode 0-3 with ShiftCoef / ShiftTFS (JSph.cpp:620-700)
    tvisco: int = 1
    shift_mode: int = 0
    shift_coef: float = -2.0
    shift_tfs: float = 0.0
    kernel: int = 2  # <parameter Kernel>: 1 Cubic spline, 2 Wendland (JSph.cpp:554-559)
    # <parameter Symmetry> (JSph.cpp:714): the half tank y >= 0 with the plane y = 0 as a
    # mirror — no y = 0 wall, the fluid from y = 0 (oracle/tools/gencase_ref sym 1)
    symmetry: bool = False
    # generated
    pos: np.ndarray = field(init=False, repr=False)
    vel: np.ndarray = field(init=False, repr=False)
    rhop: np.ndarray = field(init=False, repr=False)
    idp: np.ndarray = field(init=False, repr=False)
    npb: int = field(init=False)
    np: int = field(init=False)

    def __post_init__(self) -> None:
        dp = self.dp
        nx, ny, nz = _cround(1.6 / dp), _cround(0.67 / dp), _cround(0.4 / dp)
        mx, my, mz = _cround(0.4 / dp), _cround(0.67 / dp), _cround(0.3 / dp)
        # Boundary: loop order k, j, i over the full tank lattice, walls only.
        k, j, i = np.meshgrid(np.arange(nz + 1), np.arange(ny + 1), np.arange(nx + 1), indexing="ij")
        wall = (k == 0) | (i == 0) | (i == nx) | ((j == 0) & (not self.symmetry)) | (j == ny)
        bi, bj, bk = i[wall], j[wall], k[wall]
        self._wall_ijk = (bi, bj, bk, nx, ny)
        # Fluid: i in [1,mx], j in [1,my-1], k in [1,mz], loop order k, j, i.
        fk, fj, fi = np.meshgrid(np.arange(1, mz + 1), np.arange(0 if self.symmetry else 1, my),
                                 np.arange(1, mx + 1), indexing="ij")
        ii = np.concatenate([bi, fi.ravel()]).astype(np.float64)
        jj = np.concatenate([bj, fj.ravel()]).astype(np.float64)
        kk = np.concatenate([bk, fk.ravel()]).astype(np.float64)
        self.pos = np.stack([ii * dp, jj * dp, kk * dp], axis=1)
        self.npb = int(bi.size)
        self.np = int(self.pos.shape[0])
        self.idp = np.arange(self.np, dtype=np.uint32)
        self.vel = np.zeros((self.np, 3), dtype=np.float32)
        g, rho0, gamma = -self.gravity[2], self.rhop0, self.gamma
        hswl = mz * dp
        cs0 = self.coefsound * math.sqrt(g * hswl)
        b = cs0 * cs0 * rho0 / gamma
        h = self.coefh * math.sqrt(3.0 * dp * dp)
        mass = rho0 * dp * dp * dp
        self._h, self._b, self._mass = h, b, mass
        rhop = np.empty(self.np, dtype=np.float32)
        rhop[: self.npb] = np.float32(rho0)
        z = self.pos[self.npb :, 2]
        rhop[self.npb :] = (rho0 * np.power(1.0 + rho0 * g * (hswl - z) / b, 1.0 / gamma)).astype(np.float32)
        self.rhop = rhop

    def normals_double(self) -> np.ndarray:
        """Final normals of the boundary particles (double3[npb]), what GenCase stores in
        <case>_Normals.nbi4 (PartNormals, JPartNormalData.cpp:178-207) and what
        oracle/tools/gencase_ref writes: from the particle to the boundary limit, dp/2
        beyond the wall layer towards the fluid (summed over the walls of edges/corners)."""
        bi, bj, bk, nx, ny = self._wall_ijk
        hd = self.dp * 0.5
        nor = np.zeros((bi.size, 3))
        nor[:, 0] = np.where(bi == 0, hd, np.where(bi == nx, -hd, 0.0))
        if not getattr(self, "data2d", False):  # 2-D: no y walls, no y normal
            y0 = 0.0 if getattr(self, "symmetry", False) else hd  # Symmetry: no y = 0 wall
            nor[:, 1] = np.where(bj == 0, y0, np.where(bj == ny, -hd, 0.0))
        nor[:, 2] = np.where(bk == 0, hd, 0.0)
        return nor

    @property
    def boundnormal(self) -> np.ndarray | None:
        """Per-particle normals as JSph::LoadBoundNormals holds them (float3, zero for
        fluid), or None without mDBC."""
        if self.tboundary != 2:
            return None
        if getattr(self, "_boundnormal", None) is not None:
            return self._boundnormal
        out = np.zeros((self.np, 3), np.float32)
        out[: self.npb] = self.normals_double().astype(np.float32)
        return out

    @property
    def nf(self) -> int:
        return self.np - self.npb

    @property
    def code(self) -> np.ndarray:
        c = np.full(self.np, CODE_TYPE_FLUID, dtype=np.uint16)
        c[: self.npb] = CODE_TYPE_FIXED
        return c

    # -- constants as the case XML stores them ------------------------------
    @property
    def h(self) -> float:
        return _xml_e10(self._h)

    @property
    def cteb(self) -> float:
        return _xml_e10(self._b)

    @property
    def mass(self) -> float:
        return _xml_e10(self._mass)

    def restart_from(self, header: dict, particles: dict) -> "DamBreakCase":
        """This case continued from a loaded PART (JPartsLoad4 + JSph::InitRun with
        PartBegin): particles in file order, the map limits of the PART file
        (MapPosMin/Max), simulated time TimeStep (apply with solver.set_time)."""
        import copy

        if self.tboundary == 2:
            # JSph::ConfigBoundNormals needs the extra-data files of the run to restart
            # with mDBC (JSph.cpp:1308-1315), which this core does not write.
            raise NotImplementedError("restart with mDBC needs the reference's extra data files")
        c = copy.copy(self)
        c.idp = np.ascontiguousarray(particles["idp"], np.uint32)
        c.pos = np.ascontiguousarray(particles["pos"], np.float64)
        c.vel = np.ascontiguousarray(particles["vel"], np.float32)
        c.rhop = np.ascontiguousarray(particles["rhop"], np.float32)
        c.np = len(c.idp)
        c.npb = int(header["case_nfixed"])
        c._map = (np.array(header["map_posmin"]), np.array(header["map_posmax"]))
        c.time0 = float(header["timestep"])
        c.symdtpre0 = float(header.get("symplectic_dtpre", 0.0))
        return c

    def map_limits(self) -> tuple[np.ndarray, np.ndarray]:
        """MapRealPosMin/Max as JSph::LoadCaseParticles computes them."""
        if getattr(self, "_map", None) is not None:
            return self._map
        kernelh = float(np.float32(self.h))
        border = kernelh * BORDER_MAP
        pmin = self.pos.min(axis=0)
        pmax = self.pos.max(axis=0)
        dmin = pmin - border
        dmax = pmax + border
        dif = dmax - dmin
        prcmax = np.array([0.0, 0.0, 0.5])  # posmax z="default + 50%"
        dmax = dmax + dif * prcmax
        if getattr(self, "symmetry", False):
            dmin[1] = 0.0  # JSph::ResizeMapLimits with Symmetry (JSph.cpp:1386)
        return dmin, dmax

    def case_def(self) -> dict:
        """Fields of the C ``SphCaseDef`` (include/sphcore.h)."""
        pmin, pmax = self.map_limits()
        dpx = float("%.10g" % self.dp)
        return dict(
            dp=dpx,
            h=self.h,
            cteb=self.cteb,
            rhop0=self.rhop0,
            gamma=self.gamma,
            massbound=self.mass,
            massfluid=self.mass,
            gravity=tuple(self.gravity),
            cflnumber=self.cflnumber,
            step_algorithm=self.step_algorithm,
            verlet_steps=self.verlet_steps,
            kernel=getattr(self, "kernel", 2),
            tdensity=self.tdensity,
            visco=self.visco,
            viscoboundfactor=self.viscoboundfactor,
            ddtvalue=self.ddtvalue,
            coefdtmin=self.coefdtmin,
            dtini=0.0,
            dtmin=0.0,
            rhopoutmin=self.rhopoutmin,
            rhopoutmax=self.rhopoutmax,
            map_realposmin=tuple(pmin.tolist()),
            map_realposmax=tuple(pmax.tolist()),
            cellmode=self.cellmode,
            celldomfixed=int(self.celldomfixed),
            npb=self.npb,
            np=self.np,
            tboundary=self.tboundary,
            slipmode=self.slipmode,
            mdbc_threshold=self.mdbc_threshold,
            rheology=1, velgrad=1, tvisco=self.tvisco, nphases=0, phases=(), relaxation_dt=0.2,
            shift_mode=self.shift_mode, shift_coef=float(np.float32(self.shift_coef)),
            shift_tfs=float(np.float32(self.shift_tfs)),
            data2d=int(getattr(self, "data2d", False)),
            data2d_posy=0.0,
            dtallparticles=int(getattr(self, "dtallparticles", 0)),
            dtfixed=float(getattr(self, "dtfixed", 0.0)),
            symmetry=int(bool(getattr(self, "symmetry", False))),
            mdbc_corrector=int(getattr(self, "mdbc_corrector", 0)) if self.tboundary == 2 else 0,
        )


@dataclass
class DamBreak2DCase(DamBreakCase):
    """2-D dam break (Simulate2D) in the geometry of examples/main/01_DamBreak/
    CaseDambreakVal2D_Def.xml: tank 4 x 3 m (x, z) with bottom, left and right walls, water
    column 1 x 2 m, all particles at y = 0; h = coefh sqrt(2 dp^2), mass rho0 dp^2, Visco
    0.02 (the example's), Wendland, DDT2.  oracle/tools/gencase_ref (dim 2) writes the same
    case for the reference (tests/test_2d.py checks the two agree bit for bit)."""

    visco: float = 0.02
    data2d: bool = True

    def __post_init__(self) -> None:
        dp = self.dp
        nx, nz = _cround(4.0 / dp), _cround(3.0 / dp)
        mx, mz = _cround(1.0 / dp), _cround(2.0 / dp)
        k, i = np.meshgrid(np.arange(nz + 1), np.arange(nx + 1), indexing="ij")
        wall = (k == 0) | (i == 0) | (i == nx)
        bi, bk = i[wall], k[wall]
        self._wall_ijk = (bi, np.zeros_like(bi), bk, nx, 0)
        fk, fi = np.meshgrid(np.arange(1, mz + 1), np.arange(1, mx + 1), indexing="ij")
        ii = np.concatenate([bi, fi.ravel()]).astype(np.float64)
        kk = np.concatenate([bk, fk.ravel()]).astype(np.float64)
        self.pos = np.stack([ii * dp, np.zeros_like(ii), kk * dp], axis=1)
        self.npb = int(bi.size)
        self.np = int(self.pos.shape[0])
        self.idp = np.arange(self.np, dtype=np.uint32)
        self.vel = np.zeros((self.np, 3), dtype=np.float32)
        g, rho0, gamma = -self.gravity[2], self.rhop0, self.gamma
        hswl = mz * dp
        cs0 = self.coefsound * math.sqrt(g * hswl)
        b = cs0 * cs0 * rho0 / gamma
        self._h, self._b, self._mass = self.coefh * math.sqrt(2.0 * dp * dp), b, rho0 * dp * dp
        rhop = np.empty(self.np, dtype=np.float32)
        rhop[: self.npb] = np.float32(rho0)
        z = self.pos[self.npb:, 2]
        rhop[self.npb:] = (rho0 * np.power(1.0 + rho0 * g * (hswl - z) / b, 1.0 / gamma)).astype(np.float32)
        self.rhop = rhop


def dambreak_np(dp: float) -> int:
    """Particle count of the dam-break lattice without building it."""
    nx, ny, nz = _cround(1.6 / dp), _cround(0.67 / dp), _cround(0.4 / dp)
    mx, my, mz = _cround(0.4 / dp), _cround(0.67 / dp), _cround(0.3 / dp)
    total = (nx + 1) * (ny + 1) * (nz + 1)
    inner = (nx - 1) * (ny - 1) * nz  # k>=1, i in [1,nx-1], j in [1,ny-1]
    return (total - inner) + mx * (my - 1) * mz


@dataclass
class WaveFlumeCase:
    """Wave flume with a piston, a flap and a floating box (BASELINE cfg4):
    the lattice, blocks, motion program and floating body that oracle/tools/genflume_ref
    writes for the reference (tests/test_bodies.py checks the two agree bit for bit).

    Tank L x W x H (walls: bottom, y=0, y=W), still water of depth D from the piston
    (x = 2dp, mvrectsinu along x) to the flap (x = L, a 0.004 s wait then mvrotsinu about
    the hinge line (L, y, 0)); a box of rhopbody 500 floats at mid-length.  Block order and
    codes as JSphMk::Config: fixed, moving (piston, flap), floating, fluid."""

    dp: float
    step_algorithm: int = STEP_VERLET
    tdensity: int = DDT_DDT2
    tboundary: int = 1
    length: float = 1.2
    width: float = 0.3
    height: float = 0.4
    depth: float = 0.2
    ddtvalue: float = 0.1
    visco: float = 0.1
    viscoboundfactor: float = 1.0
    cflnumber: float = 0.2
    verlet_steps: int = 40
    coefdtmin: float = 0.05
    rhopoutmin: float = 700.0
    rhopoutmax: float = 1300.0
    cellmode: int = CELLMODE_FULL
    celldomfixed: bool = False
    gravity: tuple = (0.0, 0.0, -9.81)
    rhop0: float = 1000.0
    gamma: float = 7.0
    coefsound: float = 20.0
    coefh: float = 1.0
    rhopbody: float = 500.0
    slipmode: int = 1
    mdbc_threshold: float = 0.0
    ftpause: float = 0.0
    time0: float = 0.0
    symdtpre0: float = 0.0
    has_bodies: bool = True
    tvisco: int = 1
    shift_mode: int = 0
    shift_coef: float = -2.0
    shift_tfs: float = 0.0
    # mDBC on the floating box too (genflume_ref ftnormals=1): its outer layer gets normals
    ftnormals: bool = False
    mdbc_corrector: int = 0  # <parameter MDBCCorrector> (JSph.cpp:639)

    def __post_init__(self) -> None:
        dp = self.dp
        nx, ny, nz = _cround(self.length / dp), _cround(self.width / dp), _cround(self.height / dp)
        kd, ip = _cround(self.depth / dp), 2
        nbh = max(2, _cround(0.03 / dp))
        bic, bjc, bkc = _cround(0.55 * self.length / dp), ny // 2, kd - 1
        hd = dp * 0.5
        blocks, nor = [], []
        # fixed: bottom and side walls, loop order k, j, i
        k, j, i = np.meshgrid(np.arange(nz + 1), np.arange(ny + 1), np.arange(nx + 1), indexing="ij")
        wall = (k == 0) | (j == 0) | (j == ny)
        fi, fj, fk = i[wall], j[wall], k[wall]
        blocks.append((fi, fj, fk))
        nor.append(np.stack([np.zeros(fi.size), np.where(fj == 0, hd, np.where(fj == ny, -hd, 0.0)),
                             np.where(fk == 0, hd, 0.0)], axis=1))
        # piston (x = ip dp) and flap (x = nx dp): k = 1..nz, j = 1..ny-1
        pk, pj = np.meshgrid(np.arange(1, nz + 1), np.arange(1, ny), indexing="ij")
        pk, pj = pk.ravel(), pj.ravel()
        for xi, sgn in ((ip, 1.0), (nx, -1.0)):
            blocks.append((np.full(pk.size, xi), pj, pk))
            nor.append(np.stack([np.full(pk.size, sgn * hd), np.zeros(pk.size), np.zeros(pk.size)], axis=1))
        # floating box
        bk, bj, bi = np.meshgrid(np.arange(bkc - nbh, bkc + nbh + 1), np.arange(bjc - nbh, bjc + nbh + 1),
                                 np.arange(bic - nbh, bic + nbh + 1), indexing="ij")
        blocks.append((bi.ravel(), bj.ravel(), bk.ravel()))
        fnor = np.zeros((bi.size, 3))
        if self.ftnormals and self.tboundary == 2:  # outer layer -> the nearest limit point
            for ax, off in enumerate((bi.ravel() - bic, bj.ravel() - bjc, bk.ravel() - bkc)):
                fnor[:, ax] = np.where(off == nbh, hd, np.where(off == -nbh, -hd, 0.0))
        nor.append(fnor)
        # fluid minus the box
        wk, wj, wi = np.meshgrid(np.arange(1, kd + 1), np.arange(1, ny), np.arange(ip + 1, nx), indexing="ij")
        inbox = (np.abs(wi - bic) <= nbh) & (np.abs(wj - bjc) <= nbh) & (np.abs(wk - bkc) <= nbh)
        blocks.append((wi[~inbox], wj[~inbox], wk[~inbox]))
        counts = [b[0].size for b in blocks]
        ii = np.concatenate([b[0] for b in blocks]).astype(np.float64)
        jj = np.concatenate([b[1] for b in blocks]).astype(np.float64)
        kk = np.concatenate([b[2] for b in blocks]).astype(np.float64)
        self.pos = np.stack([ii * dp, jj * dp, kk * dp], axis=1)
        self.np = int(self.pos.shape[0])
        self.case_nfixed, npist, nflap, self.case_nfloat = counts[0], counts[1], counts[2], counts[3]
        self.case_nmoving = npist + nflap
        self.npb = self.case_npb = self.case_nfixed + self.case_nmoving
        self.case_nbound = self.case_npb + self.case_nfloat
        self.idp = np.arange(self.np, dtype=np.uint32)
        self.vel = np.zeros((self.np, 3), dtype=np.float32)
        code = np.empty(self.np, np.uint16)
        edges = np.cumsum([0] + counts)
        for c, v in zip(range(5), (CODE_TYPE_FIXED, 0x800, 0x801, 0x1000, CODE_TYPE_FLUID)):
            code[edges[c]:edges[c + 1]] = v
        self._code = code
        self._normals = np.concatenate(nor)
        g, rho0, gamma = -self.gravity[2], self.rhop0, self.gamma
        hswl = kd * dp
        cs0 = self.coefsound * math.sqrt(g * hswl)
        b = cs0 * cs0 * rho0 / gamma
        self._h, self._b, self._mass = self.coefh * math.sqrt(3.0 * dp * dp), b, rho0 * dp * dp * dp
        rhop = np.full(self.np, np.float32(rho0), dtype=np.float32)
        z = self.pos[self.case_nbound:, 2]
        rhop[self.case_nbound:] = (rho0 * np.power(1.0 + rho0 * g * (hswl - z) / b, 1.0 / gamma)).astype(np.float32)
        self.rhop = rhop
        # floating body: GenCase-style centre and diagonal inertia, summed in particle order
        fp = self.pos[self.case_npb:self.case_nbound]
        cen = [0.0, 0.0, 0.0]
        for p in fp:
            cen = [cen[0] + p[0], cen[1] + p[1], cen[2] + p[2]]
        cen = [c / len(fp) for c in cen]
        massp = self.rhopbody * dp * dp * dp
        ixx = iyy = izz = 0.0
        for p in fp:
            rx, ry, rz = p[0] - cen[0], p[1] - cen[1], p[2] - cen[2]
            ixx += massp * (ry * ry + rz * rz)
            iyy += massp * (rx * rx + rz * rz)
            izz += massp * (rx * rx + ry * ry)
        self.floatings = [dict(idbegin=self.case_npb, count=self.case_nfloat, massbody=massp * len(fp),
                               masspart=massp, center=tuple(cen), inertia=(ixx, 0.0, 0.0, 0.0, iyy, 0.0, 0.0, 0.0, izz),
                               translationfree=(1, 1, 1), rotationfree=(1, 1, 1), linvelini=(0.0,) * 3,
                               angvelini=(0.0,) * 3, mkbound=3)]
        f32 = lambda v: float(np.float32(v))  # noqa: E731  (JXml::GetAttributeFloat)
        hinge = float("%.10g" % (nx * dp))
        zero3 = (0.0, 0.0, 0.0)
        mov = lambda **kw: dict(dict(obj=0, id=1, next=0, type=1, prev=0, fields=0, data_first=0,  # noqa: E731
                                     data_n=0, duration=f32(100), vec=zero3, vec2=zero3, phase=zero3, axisp1=zero3,
                                     axisp2=zero3, ref=zero3, ang=0.0, ang2=0.0, ang3=0.0), **kw)
        # the tree form of XmlCase.motion: two top-level objreal nodes (refs 0, 1), no tables
        self.motion = dict(nobj=2, objs=[dict(parent=-1, ref=0), dict(parent=-1, ref=1)], rows=[], movs=[
            mov(obj=0, type=6, vec=(1.5, 0.0, 0.0), vec2=(0.02, 0.0, 0.0)),
            mov(obj=1, id=1, next=2, type=1, duration=f32(0.004)),
            mov(obj=1, id=2, type=7, axisp1=(hinge, 0.0, 0.0), axisp2=(hinge, 1.0, 0.0), ang=2.0, ang2=3.0),
        ], evts=[dict(obj=0, mov=1, start=0.0, finish=-1.0), dict(obj=1, mov=1, start=0.0, finish=-1.0)])

    @property
    def code(self) -> np.ndarray:
        return self._code

    @property
    def nf(self) -> int:
        return self.np - self.npb

    @property
    def h(self) -> float:
        return _xml_e10(self._h)

    @property
    def cteb(self) -> float:
        return _xml_e10(self._b)

    @property
    def mass(self) -> float:
        return _xml_e10(self._mass)

    def normals_double(self) -> np.ndarray:
        """<case>_Normals.nbi4 contents (double3[CaseNbound]; zero for the floating box unless
        ftnormals)."""
        return self._normals[: self.case_nbound]

    @property
    def boundnormal(self) -> np.ndarray | None:
        if self.tboundary != 2:
            return None
        out = np.zeros((self.np, 3), np.float32)
        out[: self.case_nbound] = self._normals.astype(np.float32)
        return out

    def map_limits(self) -> tuple[np.ndarray, np.ndarray]:
        """posmin x "default - 10%", posmax x "default + 10%", z "default + 50%"
        (JSph::ResizeMapLimits)."""
        border = float(np.float32(self.h)) * BORDER_MAP
        rmin = self.pos.min(axis=0) - border
        rmax = self.pos.max(axis=0) + border
        dif = rmax - rmin
        return rmin - dif * np.array([0.1, 0.0, 0.0]), rmax + dif * np.array([0.1, 0.0, 0.5])

    def case_def(self) -> dict:
        d = DamBreakCase.case_def(self)
        return d


# Example phases of examples/mphase_nnewtonian/01_WetDambreak/CaseWetDambreak2DNN_Def.xml:72-99
NN_EXAMPLE_PHASES = (
    dict(mkfluid=0, phasetype=0, rho=2000.0, cs0=0.0, gamma=0.0, visco=0.2, tau_yield=0.0001, tau_max=0.0,
         bi_multi=0.0, hbp_m=100.0, hbp_n=1.5),
    dict(mkfluid=1, phasetype=0, rho=1500.0, cs0=0.0, gamma=0.0, visco=0.1, tau_yield=0.001, tau_max=0.0,
         bi_multi=0.0, hbp_m=10.0, hbp_n=1.0),
    dict(mkfluid=2, phasetype=0, rho=1000.0, cs0=0.0, gamma=0.0, visco=0.05, tau_yield=0.0005, tau_max=0.0,
         bi_multi=0.0, hbp_m=0.0, hbp_n=1.0),
)


@dataclass
class WetDambreakNNCase:
    """Three-phase non-Newtonian wet dam break (BASELINE cfg5): the
    2-D reference example CaseWetDambreak2DNN_Def.xml extruded along y, as
    oracle/tools/gennn_ref writes it for the v5.0 NN solver (tests/test_nn.py checks the two
    agree bit for bit).

    Lattice (i, j, k)*dp; lengths scale with `scale` except the 0.04 m walls: tank x in
    [0, 4s], z in [0, 1.25s], y in [0, width]; walls bottom, x = 0, x = 4s, y = 0, y = width;
    phases drawn in the example's order (later replaces earlier, walls last): mkfluid 0
    x <= 4s, z <= 0.5s; mkfluid 1 x <= 1s, 0.5s <= z <= 0.75s; mkfluid 2 x <= 0.5s,
    0.75s <= z <= 1s.  Boundary first, then the phases, each in k, j, i order.  Constants:
    cs0 = 20 (speedsystem 1 x coefsound 20), b = cs0^2 rho0/gamma, h = 0.91924 sqrt(3) dp,
    Symplectic, Wendland, RheologyTreatment 2, FDA gradients, Laminar viscosity, DDT 3 (0.1),
    shifting Full (coef -10, TFS 2.75), CFL 0.1, RelaxationDt 0.2, RhopOut [500, 3000]."""

    dp: float
    width: float = 0.64
    scale: float = 1.0
    shift_tfs: float = 2.75
    tvisco: int = 2
    velgrad: int = 1  # VelocityGradientType: 1 FDA, 2 SPH (JSph.cpp:617-622 of the v5.0 solver)
    tdensity: int = DDT_DDT2FULL
    shift_mode: int = 3
    step_algorithm: int = STEP_SYMPLECTIC
    ddtvalue: float = 0.1
    visco: float = 0.05
    viscoboundfactor: float = 1.0
    cflnumber: float = 0.1
    verlet_steps: int = 40
    coefdtmin: float = 0.05
    rhopoutmin: float = 500.0
    rhopoutmax: float = 3000.0
    relaxation_dt: float = 0.2
    shift_coef: float = -10.0
    cellmode: int = CELLMODE_FULL
    celldomfixed: bool = False
    gravity: tuple = (0.0, 0.0, -9.81)
    rhop0: float = 1000.0
    gamma: float = 7.0
    coefh: float = 0.91924
    tboundary: int = 1
    slipmode: int = 1
    mdbc_threshold: float = 0.0
    phases: tuple = NN_EXAMPLE_PHASES
    csound: float = 0.0  # > 0: phase k gets <csound> csound*(1+0.1k) (gennn_ref's option)
    explicit_codes: bool = True  # the fluid codes carry the phase (fluid block index)

    def __post_init__(self) -> None:
        if self.csound > 0:
            self.phases = tuple(dict(ph, cs0=float("%.10g" % (self.csound * (1.0 + 0.1 * k))))
                                for k, ph in enumerate(self.phases))
        dp, s = self.dp, self.scale
        nx, nz, ny = _cround(4.0 * s / dp), _cround(1.25 * s / dp), _cround(self.width / dp)
        nw = _cround(0.04 / dp)
        x0, z0 = _cround(4.0 * s / dp), _cround(0.5 * s / dp)
        x1, z1b = _cround(1.0 * s / dp), _cround(0.75 * s / dp)
        x2, z2b = _cround(0.5 * s / dp), _cround(1.0 * s / dp)
        k, j, i = np.meshgrid(np.arange(nz + 1), np.arange(ny + 1), np.arange(nx + 1), indexing="ij")
        k, j, i = k.ravel(), j.ravel(), i.ravel()
        wall = (k <= nw) | (i <= nw) | (i >= nx - nw) | (j <= nw) | (j >= ny - nw)
        ph = np.full(k.size, -1, np.int64)
        ph[(i <= x0) & (k <= z0)] = 0
        ph[(i <= x1) & (k >= z0) & (k <= z1b)] = 1
        ph[(i <= x2) & (k >= z1b) & (k <= z2b)] = 2
        ph[wall] = -1
        sel = [wall] + [(~wall) & (ph == p) for p in range(3)]
        self.nph = [int(m.sum()) for m in sel[1:]]
        ii = np.concatenate([i[m] for m in sel]).astype(np.float64)
        jj = np.concatenate([j[m] for m in sel]).astype(np.float64)
        kk = np.concatenate([k[m] for m in sel]).astype(np.float64)
        self.pos = np.stack([ii * dp, jj * dp, kk * dp], axis=1)
        self.npb = int(wall.sum())
        self.np = int(self.pos.shape[0])
        self.idp = np.arange(self.np, dtype=np.uint32)
        self.vel = np.zeros((self.np, 3), dtype=np.float32)
        code = np.full(self.np, CODE_TYPE_FIXED, np.uint16)
        rhop = np.full(self.np, np.float32(self.rhop0), np.float32)
        o = self.npb
        for p, n in enumerate(self.nph):
            code[o:o + n] = CODE_TYPE_FLUID | p
            rhop[o:o + n] = np.float32(self.phases[p]["rho"])
            o += n
        self._code = code
        self.rhop = rhop
        cs0 = 20.0 * 1.0
        self._h = self.coefh * math.sqrt(3.0 * dp * dp)
        self._b = cs0 * cs0 * self.rhop0 / self.gamma
        self._mass = self.rhop0 * dp * dp * dp

    @property
    def code(self) -> np.ndarray:
        return self._code

    @property
    def nf(self) -> int:
        return self.np - self.npb

    @property
    def boundnormal(self):
        return None

    h = DamBreakCase.h
    cteb = DamBreakCase.cteb
    mass = DamBreakCase.mass
    map_limits = DamBreakCase.map_limits

    def case_def(self) -> dict:
        d = DamBreakCase.case_def(self)
        f32 = lambda v: float(np.float32(v))  # noqa: E731  (JXml ReadElementFloat / GetValueFloat)
        phases = tuple({k: (f32(v) if isinstance(v, float) else v) for k, v in ph.items()} for ph in self.phases)
        d.update(rheology=2, velgrad=self.velgrad, tvisco=self.tvisco, nphases=len(self.phases), phases=phases,
                 relaxation_dt=f32(self.relaxation_dt), shift_mode=self.shift_mode, shift_coef=f32(self.shift_coef),
                 shift_tfs=f32(self.shift_tfs))
        return d


def wetdambreak_nn_np(dp: float, width: float = 0.64, scale: float = 1.0) -> int:
    """Particle count of the NN wet dam break (lattice sizes only)."""
    return WetDambreakNNCase(dp, width=width, scale=scale).np
