"""The Yee leapfrog scheme: one class for the 1D, 2D (TMz/TEz) and 3D solvers.

Re-designs the reference's ``Scheme3D`` / ``SchemeTMz`` / ``SchemeTEz``
(``Source/Scheme/*.cpp``): fields are flat device tensors (z fastest, same
linear layout as ``Grid.cpp:127-139``), all geometry and material work happens
once in :meth:`YeeScheme.init_grids`, and the time loop is a fixed sequence of
backend operations (:mod:`fdtd3d_amd.ops`).  On the HIP backend each of those
is one HIP launch on the current stream, so a step can be captured in a HIP
graph.

Per time step ``t`` (reference ``Scheme3D::performNSteps``,
``Scheme3D.cpp:1900-2942``):

1. [TF/SF] 1D incident line, E half step.
2. E update -- plain ``E += Cb curl H`` or the UPML chain
   ``D' = CaD D + CbD curl H`` -> [Drude ``D1' = b0 D' + b1 D + b2 D_ - a1 D1 - a2 D1_``]
   -> ``E' = CaE E + CbE src' - CcE src``; TF/SF corrections folded in.
3. Hard source (point ``sin(2 pi f dt t)`` unless TF/SF is on).
4. [decomposed] E halo exchange.
5. [TF/SF] 1D incident line, H half step; H update (mirror of 2.).
6. [decomposed] H halo exchange.
7. Periodic hooks: NTFF, intermediate dumps, checkpoints, finite check.

Complex fields (reference ``COMPLEX_FIELD_VALUES``) are two real planes
stepped independently -- the update coefficients are real, so this is exact --
with the complex source ``sin + i cos`` split between them.
"""

from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..layout.approximation import (phase_velocity_incident_wave_2d, phase_velocity_incident_wave_3d)
from ..layout.materials import MaterialSampler, Scene, sigma_profile_1d
from ..layout.yee import (E_COMPONENTS, H_COMPONENTS, MATERIAL_STENCIL, MATERIAL_STENCIL_DOUBLE, UPML_AXES,
                          YeeLayout)
from ..layout.approximation import approximate_material
from ..ops.coef import Coef
from .regions import RegionLevel
from ..parallel.domain import Domain, box_empty, box_intersect, box_subtract
from ..utils.assertions import FdtdError, fdtd_assert
from ..utils.constants import ACCURACY, EPS0, MU0, PI, SPEED_OF_LIGHT

# steps per blocked amplitude pass (csrc/tb3d_mr.h AmpDev: T - 1 levels of
# running maxima in LDS, <= 3).  fp32, check every 32 steps: 256^3 T = 3 67.3k,
# T = 2 64.3k, per step 37.3k Mcells/s; 512^3 79.7k / 76.2k / 45.2k
# (profiles/amplitude_r4.md)
AMP_TB_STEPS = 3
from ..utils import logging as log
from .blocking import (F64_AUTO_STEPS, TB2D_AUTO_STEPS, TB2D_AUTO_STEPS_F64, TFSF_MAX_STEPS, BlockedStepping,
                       auto_time_block)
from .tfsf import build_tfsf_sets, build_tfsf_tables, incident_line_length


Box = Tuple[Tuple[int, int, int], Tuple[int, int, int]]

GRAPH_STEPS = 60  # steps per captured HIP graph (a multiple of 6: D/D1 level rotations return to the start)


@dataclass
class SchemeConfig:
    """Everything that defines a run (mirrors the relevant reference flags)."""

    scheme: str = "3d"                       # 3d | tmz | tez | 1d
    size: Tuple[int, int, int] = (100, 100, 100)
    time_steps: int = 100
    amplitude_steps: int = 10
    pml_size: Tuple[int, int, int] = (10, 10, 10)
    tfsf_size: Tuple[int, int, int] = (20, 20, 20)
    ntff_size: Tuple[int, int, int] = (15, 15, 15)
    theta: float = 90.0                      # degrees
    phi: float = 0.0
    psi: float = 90.0
    use_pml: bool = False
    pml_type: str = "upml"
    use_tfsf: bool = False
    use_ntff: bool = False
    use_metamaterials: bool = False
    use_amp_mode: bool = False
    use_point_source: bool = False
    double_material_precision: bool = False
    dx: float = 0.0005
    wavelength: float = 0.02
    courant: float = 0.5
    dtype: str = "f64"
    complex_values: bool = False
    scene: str = "reference"
    sphere_eps: float = 2.0
    sphere_radius: float = 20.0
    sphere_center: Tuple[float, float, float] = (40.5, 40.5, 40.5)
    source: str = "sine"                     # sine | gaussian
    gaussian_width: float = 30.0
    gaussian_delay: float = 120.0
    ntff_step: int = 100
    check_finite: bool = False
    finite_check_step: int = 100
    use_fused: bool = False
    cpml_kappa_max: float = 1.0
    cpml_alpha_max: float = 0.0
    time_block: int = 1                      # steps per HBM pass (temporal blocking, 3D vacuum/dielectric); 0 = auto
    hybrid_block: int = 0                    # PML / TF-SF / dispersive 3D runs: blocked core + stepped shell
    shell_streams: int = 0                   # hybrid shell: streams for the independent window launches (0 auto)
    hybrid_graph: str = "auto"               # 2D hybrid passes: auto (launch records) / graph (HIP graphs) / off
    hybrid_tfsf: str = "auto"                # hybrid + TF/SF: faces in the blocked core (auto / core) or the shell
    blocked_drude: str = "auto"              # Drude box inside the blocked passes: auto (HIP) / on / off
                                             # (0 = auto: 4 on the HIP fp32 path, 1 = off)
    profile_phases: bool = False             # per-phase HIP event timers (utils/profiler.py)
    use_hip_graph: bool = False              # replay captured HIP graphs of GRAPH_STEPS steps
    dispersion: str = "drude"                # drude | lorentz (metamaterial regions)
    lorentz_omega0_ratio: float = 0.5        # Lorentz resonance / source frequency
    amplitude_check_steps: int = 8           # amplitude mode: steps between host reads of the changed counts

    @classmethod
    def from_settings(cls, s) -> "SchemeConfig":
        dim = s.dimension
        if dim == 3:
            scheme = "3d"
            size = (s.sizeX, s.sizeY, s.sizeZ)
        elif dim == 2:
            scheme = s.mode2D
            size = (s.sizeX, s.sizeY, 1)
        else:
            scheme = "1d"
            size = (s.sizeX, 1, 1)
        return cls(
            scheme=scheme, size=size, time_steps=s.numTimeSteps, amplitude_steps=s.numAmplitudeTimeSteps,
            pml_size=(s.pmlSizeX, s.pmlSizeY, s.pmlSizeZ), tfsf_size=(s.tfsfSizeX, s.tfsfSizeY, s.tfsfSizeZ),
            ntff_size=(s.ntffSizeX, s.ntffSizeY, s.ntffSizeZ), theta=s.incidentWaveAngle1,
            phi=s.incidentWaveAngle2, psi=s.incidentWaveAngle3, use_pml=s.doUsePML, pml_type=s.pmlType,
            use_tfsf=s.doUseTFSF, use_ntff=s.doUseNTFF, use_metamaterials=s.doUseMetamaterials,
            use_amp_mode=s.doUseAmplitudeMode, use_point_source=s.doUsePointSource,
            double_material_precision=s.doUseDoubleMaterialPrecision, dx=s.gridStep,
            wavelength=s.sourceWaveLength, courant=s.courantNum, dtype=s.valueType,
            complex_values=s.doUseComplexFieldValues, scene=s.scene, sphere_eps=s.sphereEps,
            sphere_radius=s.sphereRadius, sphere_center=(s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ),
            source=s.sourceType, gaussian_width=s.gaussianWidth, gaussian_delay=s.gaussianDelay,
            ntff_step=s.ntffStep, check_finite=s.doCheckFinite, finite_check_step=s.finiteCheckStep,
            use_fused=not s.doUseSplitKernels, cpml_kappa_max=s.cpmlKappaMax, cpml_alpha_max=s.cpmlAlphaMax,
            dispersion=s.dispersion, lorentz_omega0_ratio=s.lorentzOmega0Ratio, time_block=s.timeBlock,
            amplitude_check_steps=s.amplitudeCheckSteps,
            hybrid_block=s.hybridBlock, shell_streams=s.shellStreams, hybrid_graph=s.hybridGraph,
            hybrid_tfsf=s.hybridTfsf, blocked_drude=s.blockedDrude,
            profile_phases=s.doProfilePhases, use_hip_graph=s.doUseHipGraph)


def _drude_coefs(dt: float, e0: float, eps, w, g, q: float):
    """(b0, b1, b2, ma1, ma2) of the second-order dispersive ADE D -> D1
    (reference Drude form, Kernels.h:103-107; Lorentz with w0 > 0 via ``q`` =
    dt^2 w0^2) -- elementwise over tensors / floats of eps, omega_p, gamma."""
    A = 4 * e0 * eps + 2 * dt * e0 * eps * g + e0 * (dt * dt * w * w + q * eps)
    b0 = (4 + 2 * dt * g + q) / A
    b1 = (-8.0 + 2 * q) / A
    b2 = (4 - 2 * dt * g + q) / A
    ma1 = -(2 * e0 * (dt * dt * w * w + q * eps) - 8 * e0 * eps) / A
    ma2 = -(4 * e0 * eps - 2 * dt * e0 * eps * g + e0 * (dt * dt * w * w + q * eps)) / A
    if not isinstance(b1, torch.Tensor):
        b1 = torch.full_like(A, b1)
    return b0, b1, b2, ma1, ma2


def _torch_dtype(name: str):
    return {"f32": torch.float32, "f64": torch.float64}[name]


class YeeScheme(BlockedStepping):
    """A Yee FDTD solver on one (possibly decomposed) domain."""

    # decomposed 3D hybrid shells with the folded CPML: the windows of a half step in one launch per row
    # layout (a rank's in-order window launches; 512^3 config 3 on 2x2x1: 37.5k vs 33.3k Mcells/s per GPU,
    # while one GPU keeps its per-window launches on the shell streams: 92.9k-94.9k vs 95.0k-95.6k,
    # profiles/decomp_r6.md).  FDTD3D_MULTI_CPML=0: per-window launches (A/B)
    multi_cpml = os.environ.get("FDTD3D_MULTI_CPML", "1") != "0"

    def __init__(self, cfg: SchemeConfig, ops, domain: Optional[Domain] = None, halo=None):
        self.cfg = cfg
        self.ops = ops
        self.device = ops.device
        self.dtype = _torch_dtype(cfg.dtype)
        fdtd_assert(ops.dtype == self.dtype, "backend dtype mismatch")
        self.domain = domain if domain is not None else Domain.serial(cfg.size)
        fdtd_assert(tuple(self.domain.global_size) == tuple(cfg.size), "domain does not match grid size")
        self.halo = halo
        scheme = cfg.scheme
        psi = cfg.psi
        if scheme == "tmz":
            psi = 90.0
        elif scheme == "tez":
            psi = 0.0
        self.layout = YeeLayout(cfg.size, scheme, tuple(cfg.pml_size) if cfg.use_pml else (0, 0, 0),
                                tuple(cfg.tfsf_size), math.radians(cfg.theta) if scheme == "3d" else PI / 2,
                                math.radians(cfg.phi), math.radians(psi), cfg.double_material_precision)
        if ops.layout is None:
            ops.layout = self.layout
        self.comps = self.layout.components
        self.e_comps = tuple(c for c in self.comps if c[0] == "E")
        self.h_comps = tuple(c for c in self.comps if c[0] == "H")
        self.planes = 2 if cfg.complex_values else 1
        self.use_upml_chain = (cfg.use_pml and cfg.pml_type == "upml") or cfg.use_metamaterials
        self.use_cpml = cfg.use_pml and cfg.pml_type == "cpml" and not cfg.use_metamaterials
        if cfg.use_pml and cfg.pml_type == "cpml" and cfg.use_metamaterials:
            log.log(0, "--pml-type cpml with --use-metamaterials: the absorbing layers run the UPML D/B form "
                       "(the dispersive chain carries D; reference Scheme3D.cpp:266-416)")
        self.t = 0
        self.sub_step = 0
        self.timers: Dict[str, float] = {}
        self.hooks: List[Callable[["YeeScheme", int], None]] = []
        # periodic work (NTFF, intermediate dumps, checkpoints): (period,
        # offset, fn) fires fn(scheme, t) after step t when (t - offset) %
        # period == 0.  Unlike per-step hooks these keep the blocked / hybrid
        # passes: advance() ends a pass at every firing step.
        self.periodic: List[Tuple[int, int, Callable[["YeeScheme", int], None]]] = []
        self.initialized = False
        from ..utils.profiler import PhaseProfiler
        self.prof = PhaseProfiler(self.device, cfg.profile_phases)

    # ================================================================ init
    def init_scheme(self, dx: Optional[float] = None, source_frequency: Optional[float] = None) -> None:
        """``Scheme3D::initScheme`` (Scheme3D.cpp:3388-3402): dt from the
        Courant number and the incident line's relative phase velocity."""
        cfg = self.cfg
        self.dx = cfg.dx if dx is None else dx
        self.source_frequency = SPEED_OF_LIGHT / cfg.wavelength if source_frequency is None else source_frequency
        self.wavelength = SPEED_OF_LIGHT / self.source_frequency
        self.courant = cfg.courant
        self.dt = self.dx * self.courant / SPEED_OF_LIGHT
        n_lambda = self.wavelength / self.dx
        if cfg.scheme == "3d":
            v0 = phase_velocity_incident_wave_3d(self.dx, self.wavelength, self.courant, n_lambda, PI / 2, 0.0)
            v = phase_velocity_incident_wave_3d(self.dx, self.wavelength, self.courant, n_lambda,
                                                self.layout.theta, self.layout.phi)
        else:
            v0 = phase_velocity_incident_wave_2d(self.dx, self.wavelength, self.courant, n_lambda, 0.0)
            v = phase_velocity_incident_wave_2d(self.dx, self.wavelength, self.courant, n_lambda, self.layout.phi)
        self.rel_phase_velocity = v0 / v

    # ------------------------------------------------------------------
    def _global_box(self, comp: str) -> Box:
        return self.layout.global_range(comp)

    def local_box(self, comp: str, window: Optional[Box] = None) -> Box:
        """Local box on which ``comp`` is updated (global range ∩ window ∩
        allocated region), in local indices."""
        g = self._global_box(comp)
        if window is None:
            window = self.domain.owned_global()
        b = box_intersect(box_intersect(g, window), self.domain.allocated_global())
        return self.domain.to_local(b)

    def _zeros(self):
        return torch.zeros(self.domain.shape, dtype=self.dtype, device=self.device)

    def init_grids(self) -> None:
        """Allocate fields, evaluate materials and build every static table
        (``Scheme3D::initGrids``, Scheme3D.cpp:3405-4067)."""
        if not hasattr(self, "dt"):
            self.init_scheme()
        cfg = self.cfg
        t0 = time.perf_counter()
        dom = self.domain
        shape = dom.shape
        self.mem_plan = self.capacity_plan()
        self._check_capacity(self.mem_plan)
        self.F: List[Dict[str, torch.Tensor]] = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]

        self.scene = Scene(cfg.scene, cfg.scheme, self.source_frequency, cfg.sphere_eps, cfg.sphere_radius,
                           tuple(cfg.sphere_center))
        vacuum = self.scene.is_vacuum(cfg.use_metamaterials)
        self.vacuum = vacuum
        sampler = MaterialSampler(self.layout, self.scene, dom.origin, shape, self.device)
        self.sampler = sampler
        dt, dx = self.dt, self.dx

        # ---- per-component material (relative eps / mu at the component)
        # (None = vacuum; a material the scene holds uniformly at 1 -- mu
        # everywhere, eps of a Drude sphere -- is never evaluated on the grid)
        self.mat: Dict[str, Optional[torch.Tensor]] = {}
        for c in self.comps:
            name = "eps" if c[0] == "E" else "mu"
            if vacuum or sampler.uniform(name) == 1.0:
                self.mat[c] = None
            else:
                self.mat[c] = sampler.averaged(c, name)

        # ---- plain-update coefficients Cb = dt / (eps eps0 dx), Db = dt / (mu mu0 dx)
        self.cb: Dict[str, Coef] = {}
        # uniform material of every component of a kind (e.g. mu = 1 in a
        # dielectric or dispersive scene): scalar coefficients keep the
        # kernels on their scalar fast path (the HIP ops need one form per kind)
        uni = {c: self.mat[c] is None or bool((self.mat[c] == self.mat[c].flatten()[0]).all()) for c in self.comps}
        for c in self.comps:
            base = EPS0 if c[0] == "E" else MU0
            m = self.mat[c]
            kind_uniform = all(uni[o] for o in self.comps if o[0] == c[0])
            if m is not None and kind_uniform:
                self.cb[c] = Coef(dt / (base * dx) / float(m.flatten()[0]))
            elif m is None:
                self.cb[c] = Coef(dt / (base * dx))
            else:
                self.cb[c] = Coef(dt / (base * dx), cell=(1.0 / m).to(self.dtype))

        if self.use_upml_chain:
            self._init_upml()
        if self.use_cpml:
            from .cpml import CPML
            self.cpml = CPML(self)
        if cfg.use_tfsf:
            self._init_tfsf()
        self._init_source()
        if cfg.use_amp_mode:
            # one [x][component][y][z] buffer per plane: the maxima of one x
            # plane of all components are contiguous, so the blocked amplitude
            # kernel reads them through ONE buffer descriptor per plane
            # (csrc/tb3d_mr.h AmpDev); each component is a strided view
            self.amp = []
            sh = tuple(self.domain.shape)
            for _ in range(self.planes):
                big = torch.zeros((sh[0], len(self.comps), sh[1], sh[2]), dtype=self.dtype, device=self.device)
                self.amp.append({c: big[:, n] for n, c in enumerate(self.comps)})
        # fused E+H kernel (ping-pong buffers): plain 3D updates with at most a
        # hard E point source
        self.fused = (cfg.use_fused and hasattr(self.ops, "fused_step") and cfg.scheme == "3d"
                      and not self.use_upml_chain and not self.use_cpml and not cfg.use_tfsf
                      and not cfg.use_amp_mode)
        # plain 3D runs with TF/SF injection: the fp32 blocked kernel applies
        # the corrections itself (models/tfsf.py TfsfSets), so such serial runs
        # take blocked passes like plain ones (single steps keep the tables)
        self.tfsf_blocked = (cfg.use_tfsf and getattr(self, "tfsf_sets", None) is not None and cfg.use_fused
                             and cfg.scheme == "3d" and not self.use_upml_chain and not self.use_cpml
                             and not cfg.use_amp_mode and self.halo is None)
        if self.fused or self.tfsf_blocked:
            self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
        # HIP graph mode (--use-hip-graph): serial HIP runs capture GRAPH_STEPS
        # steps once and replay them; sources read a device table, so the
        # split kernels (separate source launch) are used
        self.graph_mode = (cfg.use_hip_graph and self.device.type == "cuda" and self.ops.name == "hip"
                           and self.halo is None and not cfg.use_amp_mode and not cfg.check_finite
                           and not cfg.profile_phases)
        self._graph_src = None
        if self.graph_mode and self.fused:
            self.fused = False
        # temporal blocking: T fused steps per pass (yee3d_tb.hip); decomposed
        # runs exchange T-deep ghosts every T steps (buffer size == T)
        T = int(cfg.time_block)
        if T <= 0:  # automatic (models/blocking.py auto_time_block: one rule with the driver)
            percell = sum(any(getattr(self.cb.get(c), "cell", None) is not None for c in self.comps if c[0] == k)
                          for k in "EH")
            world = 1
            if self.halo is not None:
                t = self.domain.topology
                world = t[0] * t[1] * t[2]
            T = auto_time_block(cfg.scheme, cfg.dtype, self.ops.name, percell, world,
                                tfsf=bool(getattr(self, "tfsf_blocked", False)))
            if self.halo is not None and self.domain.buffer_size != T:
                T = 1
        if self.tfsf_blocked and T > TFSF_MAX_STEPS:
            # the in-kernel TF/SF variant of the blocked kernel exists for T <= 5
            # (yee3d_tb.hip TF_ENT); a longer request runs 5-step passes
            log.log(1, "--time-block %d with TF/SF: %d steps per pass" % (T, TFSF_MAX_STEPS))
            T = TFSF_MAX_STEPS
        self.tb = 1
        hip_ok = self.ops.name != "hip" or self.dtype == torch.float64 or self.domain.shape[2] % 4 == 0
        if (T > 1 and (self.fused or self.tfsf_blocked) and hasattr(self.ops, "tb_step") and hip_ok
                and T <= getattr(self.ops, "tb_max_steps", 6)
                and (self.halo is None or self.domain.buffer_size == T)):
            self.tb = T
        # 2D (TMz / TEz) plain runs: the blocked pass of yee2d_tb.hip (rows of
        # whole 16-byte lanes) or the generic oracle; F_alt is its ping-pong buffer
        if (cfg.scheme in ("tmz", "tez") and T > 1 and cfg.use_fused and hasattr(self.ops, "tb_step")
                and not self.use_upml_chain and not self.use_cpml and not cfg.use_tfsf and not cfg.use_amp_mode
                and not self.graph_mode
                and (self.ops.name != "hip" or self.domain.shape[1] % (16 // self.dtype.itemsize) == 0)
                and T <= getattr(self.ops, "tb2d_max_steps", 8)
                and (self.halo is None or self.domain.buffer_size == T)):
            self.tb = T
            self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
        # 1D plain serial HIP runs: a whole advance() in one launch of the
        # register-resident kernel (yee1d_res.hip) -- the per-step path is
        # launch-bound at these sizes, HIP graphs included
        # (the torch backend on the CPU runs the host library's native loop)
        self.res1d = (cfg.scheme == "1d" and (self.ops.name == "hip" or self.device.type == "cpu") and cfg.use_fused
                      and hasattr(self.ops, "resident_1d") and self.halo is None
                      and not self.use_upml_chain and not self.use_cpml and not cfg.use_tfsf
                      and not cfg.use_amp_mode and self.line_source is None
                      and self.domain.shape[0] <= self.ops.resident_1d_max_cells())
        if self.res1d:
            self.graph_mode = False
        self.hybrid = None
        self._drude_plan = self._plan_drude_blk()
        self._init_hybrid()
        if (self.hybrid is None and cfg.scheme == "3d" and self.ops.name == "hip"
                and getattr(self, "chain_regions", None) is not None and getattr(self, "_chain_prof", None) is not None):
            # stepped 3D runs: the z PML slabs' chain boxes widened to whole
            # 128-byte row segments (their 10-cell rows read a third of each
            # line; the widened cells have sigma = 0, where the chain is the
            # plain update algebraically).  Hybrid runs keep the exact slabs:
            # their core must stay clear of every chain box.
            self._init_chain_regions(self._chain_prof, z_align=128 // self.dtype.itemsize)
        if self.use_upml_chain:
            # after the chain boxes are final: region-local levels cover them
            self._alloc_upml_levels()
        dg = self._drude_glob  # every rank alike (decomposed: ranks the box misses have no local plan)
        if dg is not None:
            if ((self.hybrid is not None and self.hybrid.get("drude"))
                    or (self.hybrid is None and self.tb == dg[0])):
                if self._drude_plan is not None:
                    self._finish_drude_blk()
            else:
                self._drude_plan = self._drude_glob = None  # neither pass form took it: the stepped dispersive box
                self.__dict__.pop("_chain_plan_cache", None)
        # the eps-layout material grids (fp64, 8 B per cell and material) and
        # the averaged materials only feed the coefficients built above
        self.sampler.free()
        self.mat = {c: None for c in self.comps}
        self.initialized = True
        self.timers["init"] = time.perf_counter() - t0

    # -------------------------------------------------------------- capacity
    def capacity_plan(self) -> Dict[str, int]:
        """Bytes this rank's scheme will hold resident, by array family,
        estimated before anything is allocated (the layout rules of
        init_grids): field sets, UPML D levels (two; three for dispersive
        components), Drude D1 levels + uint8 index, CPML psi slabs, amplitude
        maxima -- and the transient peak of the material setup (a few fp64
        grids).  Per-cell figures at 1024^3 fp32: fields 24 B per set, a
        Drude + UPML run 150 B in all."""
        cfg = self.cfg
        n = self.domain.shape
        cells = n[0] * n[1] * n[2]  # this rank's allocated region (ghosts included)
        isz = 4 if cfg.dtype == "f32" else 8
        planes = self.planes
        plan = {"fields": 6 * isz * cells * planes}
        scene = Scene(cfg.scene, cfg.scheme)
        blocked = cfg.use_fused and cfg.scheme in ("3d", "tmz", "tez") and self.ops.name == "hip"
        if blocked or cfg.use_tfsf:
            plan["fields_pingpong"] = plan["fields"]
        if cfg.use_amp_mode:
            plan["amplitude"] = plan["fields"]
        if self.use_upml_chain:
            disp_e = cfg.use_metamaterials and scene.uniform("omega_pe") != 0.0
            disp_h = cfg.use_metamaterials and scene.uniform("omega_pm") != 0.0
            nd = 3 * (disp_e + disp_h)  # dispersive components
            aux = disp = cells
            if (cfg.scheme == "3d" and self.halo is None and getattr(self.ops, "region_aux", False)
                    and not (cfg.use_tfsf and cfg.use_pml and min(cfg.tfsf_size) <= max(self.layout.pml_size))):
                # region-local levels (models/regions.py): the PML slabs (one
                # cell of staggering slack per side) and the dispersive box
                inner = 1
                for a in range(3):
                    p_ = self.layout.pml_size[a] + 1 if cfg.use_pml and self.layout.active(a) else 0
                    inner *= max(0, n[a] - 2 * p_)
                slabs = cells - inner
                disp = 0
                if cfg.use_metamaterials:
                    if cfg.scene == "drude-sphere":
                        r = int(math.ceil(cfg.sphere_radius)) + 2
                        lo = [int(cfg.sphere_center[a]) - r for a in range(3)]
                        hi = [int(cfg.sphere_center[a]) + r + 1 for a in range(3)]
                        disp = 1
                        for a in range(3):
                            disp *= max(0, min(n[a], hi[a]) - max(0, lo[a]))
                        # D1 also lives in the PML slabs the dispersive box reaches
                        pml = [self.layout.pml_size[a] + 1 if cfg.use_pml else 0 for a in range(3)]
                        if any(lo[a] < pml[a] or hi[a] > n[a] - pml[a] for a in range(3)):
                            disp += slabs
                    else:
                        disp = cells  # (the reference scene's small boxes: bounded by the grid)
                aux = min(cells, slabs + disp)
                disp = min(cells, disp)
            plan["upml_D"] = isz * aux * planes * (3 * nd + 2 * (6 - nd))
            if nd:
                plan["drude_D1"] = 3 * isz * disp * planes * nd
                lean = self.ops.name == "hip" and cfg.scheme == "3d"
                plan["drude_coef"] = cells * nd * (2 if lean else 1 + 5 * isz)
        if self.use_cpml:
            pml = self.layout.pml_size
            slab = sum(2 * pml[a] * (cells // max(1, n[a])) for a in range(3) if self.layout.active(a))
            plan["cpml_psi"] = 2 * 4 * isz * slab * planes  # ~4 terms per slab cell, two copies
        plan["init_transient"] = 4 * 8 * cells if not scene.is_vacuum(cfg.use_metamaterials) else 0
        return plan

    def _check_capacity(self, plan: Dict[str, int]) -> None:
        """Fail before allocating when the plan cannot fit the device (a
        1024^3 run that would die half-initialised after minutes of setup)."""
        if self.device.type != "cuda":
            return
        free, total = torch.cuda.mem_get_info(self.device)
        need = sum(plan.values())
        log.info("capacity plan %.1f GB (%s) of %.1f GB free" % (
            need / 1e9, ", ".join("%s %.1f" % (k, v / 1e9) for k, v in plan.items() if v), free / 1e9))
        if need > 0.97 * free:
            raise FdtdError("grid %s needs about %.1f GB on this device (%s) but %.1f GB are free: use more ranks "
                            "(--manual-topology / torchrun) or a smaller grid"
                            % (tuple(self.domain.shape), need / 1e9,
                               ", ".join("%s %.1f GB" % (k, v / 1e9) for k, v in plan.items() if v), free / 1e9))

    # ------------------------------------------------------------------ UPML
    def _sigma_profiles(self) -> Dict[int, torch.Tensor]:
        """Global-eps-layout sigma profile along each axis, restricted to the
        local eps region (float64)."""
        dom = self.domain
        dbl = self.layout.double_material_precision
        prof = {}
        for a in range(3):
            n_glob = (self.cfg.size[a] + 1) * (2 if dbl else 1)
            pml = self.layout.pml_size[a] if (self.cfg.use_pml and self.layout.active(a)) else 0
            p = sigma_profile_1d(n_glob, pml, self.dx, dbl)
            lo = dom.origin[a] * (2 if dbl else 1)
            n_loc = (dom.shape[a] + 1) * (2 if dbl else 1)
            seg = np.zeros(n_loc)
            take = p[max(lo, 0):max(lo, 0) + n_loc]
            seg[:take.size] = take
            if not self.layout.active(a):
                seg[:] = 0.0
            prof[a] = torch.as_tensor(seg, dtype=torch.float64, device=self.device)
        return prof

    def _avg_profile(self, comp: str, axis: int, p: torch.Tensor) -> torch.Tensor:
        """sigma along ``axis`` averaged at ``comp`` positions (1D, local)."""
        n = self.domain.shape[axis]
        if not self.layout.active(axis):
            return torch.zeros(n, dtype=torch.float64, device=self.device)
        pts = []
        if not self.layout.double_material_precision:
            for off in MATERIAL_STENCIL[comp]:
                o = off[axis]
                pts.append(p[o:o + n])
        else:
            for base, sub in MATERIAL_STENCIL_DOUBLE[comp]:
                o = 2 * base[axis] + sub[axis]
                pts.append(p[o:o + 2 * n:2])
        return approximate_material(pts)

    def _init_upml(self) -> None:
        cfg = self.cfg
        dt, dx = self.dt, self.dx
        prof = self._sigma_profiles()
        dtp = self.dtype
        self.upml: Dict[str, dict] = {}
        for c in self.comps:
            aD, aCa, aCb = UPML_AXES[c]
            sD = self._avg_profile(c, aD, prof[aD])
            sCa = self._avg_profile(c, aCa, prof[aCa])
            sCb = self._avg_profile(c, aCb, prof[aCb])
            two = 2 * EPS0  # the reference normalises H-side sigma by eps0 too (Scheme3D.cpp:1198-1201)
            caD = (two - sD * dt) / (two + sD * dt)
            cbD = (two * dt / dx) / (two + sD * dt)
            caE = (two - sCa * dt) / (two + sCa * dt)
            cbE_a = (two + sCb * dt)
            ccE_a = -(two - sCb * dt)
            inv_ca = 1.0 / (two + sCa * dt)
            drude = cfg.use_metamaterials
            base = EPS0 if c[0] == "E" else MU0
            if drude:
                inv_mod = None
                inv_mod_s = 1.0
            elif self.mat[c] is None:
                inv_mod = None
                inv_mod_s = 1.0 / base
            else:
                inv_mod = (1.0 / (self.mat[c] * base))
                inv_mod_s = 1.0

            def prof_coef(scalar, axis_vals: Dict[int, torch.Tensor], cell=None) -> Coef:
                k = Coef(scalar)
                for a, v in axis_vals.items():
                    v = v.to(dtp)
                    if a == 0:
                        k.px = v if k.px is None else k.px * v
                    elif a == 1:
                        k.py = v if k.py is None else k.py * v
                    else:
                        k.pz = v if k.pz is None else k.pz * v
                if cell is not None:
                    k.cell = cell.to(dtp)
                return k

            st = {
                "caD": prof_coef(1.0, {aD: caD}),
                "cbD": prof_coef(1.0, {aD: cbD}),
                "caE": prof_coef(1.0, {aCa: caE}),
                "cbE": prof_coef(inv_mod_s, {aCb: cbE_a, aCa: inv_ca}, inv_mod),
                "ccE": prof_coef(inv_mod_s, {aCb: ccE_a, aCa: inv_ca}, inv_mod),
            }
            # the same coefficients in the factored form of the fused chain
            # kernel (chain_kernels.hip): 1D profiles along aD / aCa / aCb, the
            # scalar and the optional per-cell 1/(eps eps0) factor
            st["prof"] = {"caD": caD.to(dtp).contiguous(), "cbD": cbD.to(dtp).contiguous(),
                          "caE": caE.to(dtp).contiguous(), "ica": inv_ca.to(dtp).contiguous(),
                          "cbEa": cbE_a.to(dtp).contiguous(), "ccEa": ccE_a.to(dtp).contiguous(),
                          "s": float(inv_mod_s), "cell": None if inv_mod is None else inv_mod.to(dtp).contiguous(),
                          "axes": (aD, aCa, aCb)}
            # D (3 levels for a dispersive component) and D1 levels: allocated
            # once the time stepping is known (init_grids): full-grid arrays
            # for the chain kernels, region-local boxes for the single-pass
            # shell.  A component without any dispersive cell (H in an
            # electric Drude scene) keeps two D levels and no D1 at all: its
            # chain boxes all take the non-dispersive form.
            st["nlev"] = 2
            st["D"] = None
            if drude:
                name = "eps" if c[0] == "E" else "mu"
                ue = self.sampler.uniform(name)
                eps_c = ue if ue is not None else self.sampler.averaged(c, name)
                wname, gname = ("omega_pe", "gamma_e") if c[0] == "E" else ("omega_pm", "gamma_m")
                uw, ug = self.sampler.uniform(wname), self.sampler.uniform(gname)
                e0 = base
                # second-order ADE  D -> D1 (= E) of the dispersive permittivity,
                # bilinear in the non-derivative terms (reference Drude form,
                # Kernels.h:103-107):
                #   drude:   eps(w) = eps - wp^2 / (w^2 + i g w)
                #   lorentz: eps(w) = eps + wp^2 / (w0^2 - w^2 - i g w)
                # Lorentz multiplies both sides by (w0^2 + d_t^2 + g d_t); with
                # w0 = 0 it is exactly the Drude recurrence.
                w0 = 0.0
                if cfg.dispersion == "lorentz":
                    w0 = cfg.lorentz_omega0_ratio * 2 * PI * self.source_frequency
                q = dt * dt * w0 * w0
                lean = (ue is not None and ug is not None and cfg.scheme == "3d"
                        and getattr(self.ops, "drude_lut", False) and hasattr(self.ops, "_drude_lut"))
                lut = None
                if uw == 0.0 and ug == 0.0:
                    active = None
                elif lean:
                    # eps and gamma uniform: the coefficients are a function of
                    # omega_p alone -- the uint8 index + table built slab by
                    # slab (_drude_index), never a full-grid fp64 omega grid
                    active, lut = self._drude_index(c, dt, e0, eps_c, ug, q, dtp)
                    if lut is None:
                        lean = False  # more than 256 distinct tuples: per-cell arrays
                if uw == 0.0 and ug == 0.0:
                    pass
                elif not lean or lut is not None:
                    w = g = None
                    if lut is None:
                        w, g = self.sampler.averaged_drude(c, electric=(c[0] == "E"))
                        active = (w != 0) | (g != 0)
                    local = bool(active.any())
                    # decomposed: a rank without dispersive cells of c still
                    # keeps the dispersive state arrays when another rank has
                    # some (every rank must exchange the same message list)
                    if self.halo is not None:
                        local = self.halo.allreduce_max(1.0 if local else 0.0) > 0
                    if not local:
                        active = None
                    if active is not None:
                        st["nlev"] = 3
                        st["D1"] = None
                        st["drude_active"] = active
                        if lut is not None:
                            st["_drude_lut"] = lut
                            for n in ("b0", "b1", "b2", "ma1", "ma2"):
                                st[n] = Coef(1.0)  # cell: self._drude_cells(c) on demand
                        else:
                            if w is None:
                                w, g = self.sampler.averaged_drude(c, electric=(c[0] == "E"))
                            for n, v in zip(("b0", "b1", "b2", "ma1", "ma2"), _drude_coefs(dt, e0, eps_c, w, g, q)):
                                st[n] = Coef(1.0, cell=v.to(dtp))
                    del w, g
                # the non-dispersive chain (E from D through 1/(eps eps0)) for the
                # chain boxes with no dispersive cell (PML slabs away from the
                # metamaterial): with w = g = 0 the ADE gives D1 = D/(eps eps0)
                # exactly, so D1 and its five coefficient arrays are not needed
                if not isinstance(eps_c, torch.Tensor):
                    s_pl, cell_pl = 1.0 / (eps_c * base), None
                else:
                    inv_e = 1.0 / (eps_c * base)
                    uniform = bool((inv_e == inv_e.flatten()[0]).all())
                    s_pl, cell_pl = ((float(inv_e.flatten()[0]), None) if uniform
                                     else (1.0, inv_e.to(dtp).contiguous()))
                    del inv_e
                st["plain"] = {"cbE": prof_coef(s_pl, {aCb: cbE_a, aCa: inv_ca}, cell_pl),
                               "ccE": prof_coef(s_pl, {aCb: ccE_a, aCa: inv_ca}, cell_pl),
                               "prof": dict(st["prof"], s=s_pl, cell=cell_pl)}
            self.upml[c] = st
        self._init_chain_regions(prof)
        if cfg.use_metamaterials and getattr(self.ops, "chain_rows", False) and cfg.scheme == "3d":
            # row tables built now (host syncs), never under a HIP graph capture
            for kind in ("E", "H"):
                self._drude_rows(kind)
        if (cfg.use_metamaterials and cfg.scheme == "3d" and getattr(self.ops, "drude_lut", False)
                and hasattr(self.ops, "_drude_lut")):
            # the uint8 material index + coefficient table too (torch.unique
            # syncs the host): built here, not lazily inside a graph capture
            for c in self.comps:
                st = self.upml[c]
                if "D1" in st and "_drude_lut" not in st:
                    self.ops._drude_lut(st, [st[n].cell for n in ("b0", "b1", "b2", "ma1", "ma2")],
                                        self.domain.shape)

    def _drude_index(self, c: str, dt: float, e0: float, eps_c, ug: float, q: float, dtp,
                     slab_cells: int = 1 << 24):
        """(active mask, (uint8 index, coefficient table)) of the dispersive
        component ``c`` with uniform eps and gamma: omega_p is sampled and
        averaged over x slabs of the local region (MaterialSampler on each
        slab), so the transient is a slab of fp64 grids instead of several
        full ones (1024^3: ~35 GB).  Pass 1 collects the distinct omega
        values, pass 2 maps every cell to its table row.  (None for the
        table when there are more than 256 distinct values.)"""
        dom = self.domain
        shape = tuple(dom.shape)
        electric = c[0] == "E"
        cells = shape[1] * shape[2]
        xc = max(1, min(shape[0], slab_cells // max(1, cells)))  # ~16M cells per slab

        def slabs():
            for x0 in range(0, shape[0], xc):
                n = min(xc, shape[0] - x0)
                smp = MaterialSampler(self.layout, self.scene, (dom.origin[0] + x0, dom.origin[1], dom.origin[2]),
                                      (n, shape[1], shape[2]), self.device)
                w, _ = smp.averaged_drude(c, electric)
                yield x0, n, w
                del smp, w

        active = torch.zeros(shape, dtype=torch.bool, device=self.device)
        uniq = None
        for x0, n, w in slabs():
            # (a uniform non-zero gamma makes every cell dispersive, like
            # approximate_drude's (w != 0) | (g != 0))
            active[x0:x0 + n] = (w != 0) if ug == 0.0 else True
            u = torch.unique(w)
            uniq = u if uniq is None else torch.unique(torch.cat([uniq, u]))
            if uniq.numel() > 256:
                return active, None
        ids = torch.empty(shape, dtype=torch.uint8, device=self.device)
        for x0, n, w in slabs():
            ids[x0:x0 + n] = torch.searchsorted(uniq, w).to(torch.uint8)
        tab = torch.stack(_drude_coefs(dt, e0, eps_c, uniq, ug, q), 1).to(dtp).contiguous()
        return active, (ids.contiguous(), tab)

    def _drude_cells(self, c: str) -> None:
        """Per-cell Drude coefficient arrays of component ``c`` rebuilt from
        its uint8 index + table (the lean initialisation keeps only those) for
        the paths that take them per cell (generic D-form boxes, the
        single-pass shell's dispersive box)."""
        st = self.upml[c]
        if st["b0"].cell is not None or st.get("_drude_lut") is None:
            return
        ids, tab = st["_drude_lut"]
        for q, n in enumerate(("b0", "b1", "b2", "ma1", "ma2")):
            st[n] = Coef(1.0, cell=tab[:, q][ids.long()].contiguous())

    def _alloc_upml_levels(self) -> None:
        """D / D1 levels of the chain kernels: region-local (models/regions.py:
        D over each component's chain boxes -- the PML slabs and the
        dispersive box -- D1 over the chain boxes that hold dispersive cells)
        where every launch is a fused chain launch, full-grid otherwise (2D,
        the generic D-form path of TF/SF targets inside a chain box)."""
        reg = self._upml_region_boxes()
        self.upml_regional = reg is not None
        for c in self.comps:
            st = self.upml[c]
            if st["D"] is None:
                if reg is not None:
                    st["D"] = [[RegionLevel(reg[c][0], self.dtype, self.device) for _ in range(st["nlev"])]
                               for _ in range(self.planes)]
                else:
                    st["D"] = [[self._zeros() for _ in range(st["nlev"])] for _ in range(self.planes)]
            if "D1" in st and st["D1"] is None:
                if reg is not None:
                    st["D1"] = [[RegionLevel(reg[c][1], self.dtype, self.device) for _ in range(3)]
                                for _ in range(self.planes)]
                else:
                    st["D1"] = [[self._zeros() for _ in range(3)] for _ in range(self.planes)]

    def _upml_region_boxes(self):
        """Per component (D boxes, D1 boxes), local, for region-local levels;
        None when the run needs full-grid levels."""
        if (self.cfg.scheme != "3d" or getattr(self, "chain_regions", None) is None or self.halo is not None
                or not getattr(self.ops, "region_aux", False)):
            # (decomposed runs keep full-grid levels: their z-aligned chain
            # boxes differ per rank, the halo messages of boxed arrays assume
            # the same cover on both ends)
            return None
        dom = self.domain
        out = {c: ([], []) for c in self.comps}
        for kind, comps in (("E", self.e_comps), ("H", self.h_comps)):
            for r, dru in self.chain_regions[kind]["chain"]:
                for c in comps:
                    b = dom.to_local(r[c])
                    if box_empty(b):
                        continue
                    if self.cfg.use_tfsf:
                        tb = self.tfsf_bbox.get(c)
                        if tb is not None and not box_empty(box_intersect(b, tb)):
                            return None  # TF/SF targets in a chain box: the generic full-grid D form
                    out[c][0].append(b)
                    if dru[c]:
                        out[c][1].append(b)
        return out

    def _bbox_global(self, mask: torch.Tensor) -> Box:
        """Global bounding box of the True cells of a local mask (empty box
        when none)."""
        if mask is None or not bool(mask.any()):
            o = self.domain.origin
            return o, o
        lo, hi = [], []
        for a in range(3):
            other = tuple(d for d in range(3) if d != a)
            nzv = torch.nonzero(mask.any(dim=other[1]).any(dim=other[0])).flatten()
            lo.append(int(nzv.min()))
            hi.append(int(nzv.max()) + 1)
        return self.domain.to_global((tuple(lo), tuple(hi)))

    def _disp_box(self, c: str) -> Box:
        """Global bounding box of component ``c``'s dispersive cells over ALL
        ranks (serial: the local box).  A rank's region-local arrays over it
        (the dispersive chain box, the blocked Drude state) cover the box
        clipped to the rank's allocation, so two neighbours agree on the cells
        of every ghost message (a sphere's cap seen by one rank has a smaller
        local bounding box than the sphere clipped to that rank).  Collective
        on the first call per component (all ranks call it in init_grids),
        cached after."""
        cache = self.__dict__.setdefault("_disp_box_cache", {})
        if c in cache:
            return cache[c]
        b = self._bbox_global(self.upml[c].get("drude_active")) if c in getattr(self, "upml", {}) else None
        if b is None:
            o = self.domain.origin
            b = (o, o)
        if self.halo is not None:
            big = float(1 << 30)
            e = box_empty(b)
            vals = [-big if e else -float(b[0][d]) for d in range(3)] + [-big if e else float(b[1][d]) for d in range(3)]
            r = [self.halo.allreduce_max(v) for v in vals]
            lo, hi = tuple(int(-r[d]) for d in range(3)), tuple(int(r[3 + d]) for d in range(3))
            o = self.domain.origin
            b = (lo, hi) if all(hi[d] > lo[d] for d in range(3)) else (o, o)
        cache[c] = b
        return b

    def _init_chain_regions(self, prof, z_align: int = 1) -> None:
        """Region-local UPML/Drude chain (3D and 2D).  Where all sigma values
        of a component vanish and its Drude parameters are zero the chain is
        algebraically the plain Yee update (D' - D = (dt/dx) curl, E = D/(eps eps0)
        and, for Drude, D1 = D/(eps eps0) exactly), so each component's box is
        split into ``plain`` slabs (float4 Yee kernels) and ``chain`` boxes
        (fused chain kernel): 6 PML slabs + the dispersive bounding box.  D / D1
        are only ever read in the chain boxes, which are static."""
        self.chain_regions = None
        self._chain_prof = prof
        self.__dict__.pop("_chain_plan_cache", None)
        if self.cfg.scheme == "1d":
            return
        cfg = self.cfg
        dom = self.domain
        alloc = dom.allocated_global()
        per = {}
        sigma0 = {}  # per component: the box where every sigma vanishes (global)
        self._chain_sigma0 = sigma0
        self._disp_chain = {}
        for c in self.comps:
            C = box_intersect(self._global_box(c), alloc)
            lo, hi = list(C[0]), list(C[1])
            for a in range(3):
                if not (cfg.use_pml and self.layout.active(a)):
                    continue
                sv = self._avg_profile(c, a, prof[a]).cpu().numpy()
                zero = np.nonzero(sv == 0.0)[0]
                if zero.size == 0:
                    lo[a], hi[a] = C[0][a], C[0][a]
                    continue
                zl, zh = int(zero.min()), int(zero.max()) + 1
                fdtd_assert(bool((sv[zl:zh] == 0.0).all()), "sigma profile is not zero on one contiguous range")
                if a == 2 and z_align > 1:
                    # local z index rounded inward to whole row segments
                    zl = -(-zl // z_align) * z_align
                    zh = max(zl, zh // z_align * z_align)
                lo[a] = max(lo[a], zl + dom.origin[a])
                hi[a] = min(hi[a], zh + dom.origin[a])
            I = box_intersect(C, (tuple(lo), tuple(hi)))
            if box_empty(I):
                I = (C[0], C[0])
            sigma0[c] = I
            Dbox = box_intersect(self._disp_box(c), alloc)
            plain_core = I
            plain = box_subtract(plain_core, Dbox) if not box_empty(plain_core) else [(C[0], C[0])] * 6
            chain = box_subtract(C, plain_core) + [box_intersect(plain_core, Dbox)]
            # which chain boxes need the dispersive (D1) form
            drude = [cfg.use_metamaterials and (n == 6 or not box_empty(box_intersect(chain[n], Dbox)))
                     for n in range(7)]
            per[c] = (plain, chain, drude)
            self._disp_chain[c] = chain[6]  # the dispersive box's chain box (blocked Drude: never stepped)
        regions = {}
        for kind, comps in (("E", self.e_comps), ("H", self.h_comps)):
            plain = [{c: per[c][0][n] for c in comps} for n in range(6)]
            chain = [({c: per[c][1][n] for c in comps}, {c: per[c][2][n] for c in comps}) for n in range(7)]
            regions[kind] = {"plain": [r for r in plain if any(not box_empty(b) for b in r.values())],
                             "chain": [r for r in chain if any(not box_empty(b) for b in r[0].values())]}
        self.chain_regions = regions
        if getattr(self, "upml_regional", False):
            # region-local levels follow the (new) chain boxes
            for c in self.comps:
                self.upml[c]["D"] = None
                if "D1" in self.upml[c]:
                    self.upml[c]["D1"] = None
            self._alloc_upml_levels()

    # ----------------------------------------------------------------- TF/SF
    def _init_tfsf(self) -> None:
        n = incident_line_length(self.cfg.size, self.cfg.scheme)
        self.inc_len = n
        self.einc = [torch.zeros(n, dtype=self.dtype, device=self.device) for _ in range(self.planes)]
        self.hinc = [torch.zeros(n, dtype=self.dtype, device=self.device) for _ in range(self.planes)]
        self.inc_ce = self.dt / (self.rel_phase_velocity * EPS0 * self.dx)
        self.inc_ch = self.dt / (self.rel_phase_velocity * MU0 * self.dx)
        # tables on the full allocated region; each step filters by window
        alloc = self.domain.allocated_global()
        boxes = {c: self.local_box(c, alloc) for c in self.comps}
        # E-form tables (coefficient Cb, applied to E after a plain update) and,
        # with the UPML chain, D-form tables (coefficient CbD, applied to D)
        self.tfsf = build_tfsf_tables(self.layout, self.comps, self.domain.origin, self.domain.shape, boxes,
                                      dict(self.cb), self.device, self.dtype, n)
        self.tfsf_D = self.tfsf
        if self.use_upml_chain:
            self.tfsf_D = build_tfsf_tables(self.layout, self.comps, self.domain.origin, self.domain.shape, boxes,
                                            {c: self.upml[c]["cbD"] for c in self.comps}, self.device, self.dtype, n)
        # in-kernel form for the blocked passes (incident direction along x or
        # y; models/tfsf.py TfsfSets; fp32 and, from round 6, fp64 HIP kernels)
        self.tfsf_sets = None
        if self.cfg.scheme == "3d" and getattr(self.ops, "tfsf_sets_ok", False):
            self.tfsf_sets = build_tfsf_sets(self.layout, self.comps, self.domain.origin, self.domain.shape, boxes,
                                             self.device, self.dtype, n)
            if self.tfsf_sets is not None:
                self.tfsf_sets.tables = self.tfsf  # the torch oracle's blocked pass applies these
        # local bounding box of each component's TF/SF targets
        self.tfsf_bbox = {}
        for c in self.comps:
            ijk = [t.ijk for t in self.tfsf[c] if t.n > 0]
            if ijk:
                allv = torch.cat(ijk).view(-1, 3)
                self.tfsf_bbox[c] = (tuple(int(v) for v in allv.min(0).values),
                                     tuple(int(v) + 1 for v in allv.max(0).values))
            else:
                self.tfsf_bbox[c] = None

    # ---------------------------------------------------------------- source
    def _init_source(self) -> None:
        cfg = self.cfg
        size = cfg.size
        self.point_source = None
        self.line_source = None
        if cfg.use_tfsf and not cfg.use_point_source:
            return
        if cfg.scheme == "3d":
            comp, g = "Ez", (size[0] // 2, size[1] // 2, size[2] // 2)
        elif cfg.scheme == "tmz":
            # reference SchemeTMz.cpp:1345: Ez at (70, Ny/2)
            comp, g = "Ez", (70 if size[0] > 140 else size[0] // 2, size[1] // 2, 0)
        elif cfg.scheme == "tez":
            comp, g = "Hz", (size[0] // 2, size[1] // 2, 0)
        else:
            comp, g = "Ez", (size[0] // 2, 0, 0)
        li = self.domain.local_index(g)
        self.point_source = (comp, li, g)
        if cfg.use_amp_mode and cfg.scheme == "3d":
            # amplitude mode drives an Ez z-line at (Nx/8, Ny/2, k in the non-PML range)
            # (Scheme3D.cpp:2995-3013)
            lo = self.layout.pml_size[2] if cfg.use_pml else 0
            hi = size[2] - lo
            offs = []
            for k in range(lo, hi):
                li2 = self.domain.local_index((size[0] // 8, size[1] // 2, k))
                if li2 is not None:
                    s = self.domain.shape
                    offs.append((li2[0] * s[1] + li2[1]) * s[2] + li2[2])
            self.line_source = ("Ez", torch.as_tensor(offs, dtype=torch.int64, device=self.device))
            # the same line as (component, i, j, k0, k1) for the blocked
            # amplitude passes (serial runs: the whole line is local)
            self.line_box = None
            li0 = self.domain.local_index((size[0] // 8, size[1] // 2, lo))
            if self.halo is None and li0 is not None and hi > lo:
                self.line_box = ("Ez", li0[0], li0[1], li0[2], li0[2] + hi - lo)

    def source_value(self, t: int, plane: int) -> float:
        cfg = self.cfg
        if cfg.source == "gaussian":
            v = math.exp(-((t - cfg.gaussian_delay) / cfg.gaussian_width) ** 2)
            return v if plane == 0 else 0.0
        arg = self.dt * t * 2 * PI * self.source_frequency
        return math.sin(arg) if plane == 0 else math.cos(arg)

    def source_values(self, t0: int, n: int, plane: int) -> torch.Tensor:
        """``source_value(t0 + s, plane)`` for s < n as one float64 tensor."""
        cfg = self.cfg
        t = torch.arange(t0, t0 + n, dtype=torch.float64)
        if cfg.source == "gaussian":
            v = torch.exp(-((t - cfg.gaussian_delay) / cfg.gaussian_width) ** 2)
            return v if plane == 0 else torch.zeros_like(v)
        arg = self.dt * t * 2 * PI * self.source_frequency
        return torch.sin(arg) if plane == 0 else torch.cos(arg)

    # ================================================================ stepping
    def _window(self, kind: str) -> Box:
        return self.domain.window(kind, self.sub_step)

    def _boxes(self, comps, kind) -> Dict[str, Box]:
        w = self._window(kind)
        return {c: self.local_box(c, w) for c in comps}

    def _update(self, kind: str, p: int, windows: Optional[Sequence[Box]] = None, tfsf_once: bool = False) -> None:
        """Update all E (or H) components of plane ``p`` on the given global
        windows (default: this sub-step's window).  ``tfsf_once``: apply the
        E-form TF/SF corrections once over the whole grid after all windows
        instead of per window (the hybrid shell: every target cell lies in
        one of the windows, and per-window application costs a launch per
        window, component and face)."""
        comps = self.e_comps if kind == "E" else self.h_comps
        F = self.F[p]
        if windows is None:
            windows = [self._window(kind)]
        elif self.halo is not None:
            # hybrid shell of a decomposed run: clip to this sub-step's deep-halo window
            dw = self._window(kind)
            windows = [b for b in (box_intersect(w, dw) for w in windows) if not box_empty(b)]
        use_tfsf = self.cfg.use_tfsf
        tfsf_here = use_tfsf and not tfsf_once
        chain = self.use_upml_chain and getattr(self, "chain_regions", None) is not None
        if chain and self.hybrid is not None and len(windows) > 1:
            # hybrid shell: the chain boxes lie inside the shell, so each runs
            # once, whole; only the plain slabs are cut to the shell windows
            # (decomposed: clipped to this sub-step's deep-halo window)
            self._update_chain_regions(kind, p, None if self.halo is None else self._window(kind), tfsf_here,
                                       plain_windows=windows)
            windows = []
        fused_cpml = self.use_cpml and getattr(self.ops, "fused_cpml_ok", lambda *a: False)(self)
        # hybrid shell without the folded CPML kernels: the psi slabs lie inside
        # the shell, so their corrections run once per slab after all windows
        # (one launch per slab instead of one per slab and window)
        cpml_once = (self.use_cpml and not fused_cpml and self.hybrid is not None and len(windows) > 1
                     and self.halo is None)

        # built (first call: device tensors) on the current stream BEFORE the
        # window launches fork onto the shell streams, which would not wait for it
        ktab = self.cpml.kernel_table(kind, p) if fused_cpml else None

        def one(w):
            if chain:
                self._update_chain_regions(kind, p, w, tfsf_here)
                return
            boxes = {c: self.local_box(c, w) for c in comps}
            if self.use_upml_chain:
                for c in comps:
                    self._upml_region(kind, c, p, boxes[c])
                return
            if fused_cpml:
                # CPML folded into the update kernel (yee3d_cpml.hip)
                self.ops.curl_update_cpml(kind, boxes, F, F, self.cb, ktab)
            else:
                self.ops.curl_update(kind, boxes, F, F, self.cb)
                if self.use_cpml and not cpml_once:
                    self.cpml.apply(kind, p, boxes)
            if tfsf_here:
                inc = self.hinc[p] if kind == "E" else self.einc[p]
                for c in comps:
                    for tab in self.tfsf[c]:
                        self.ops.tfsf_apply(F[c], tab, inc, boxes[c])

        multi = (len(windows) > 1 and not tfsf_here and self.hybrid is not None and not chain
                 and not self.use_upml_chain and not fused_cpml and (not self.use_cpml or cpml_once)
                 and self.cfg.scheme in ("tmz", "tez") and getattr(self.ops, "multi2d", False))
        multi_cpml = (len(windows) > 1 and not tfsf_here and self.hybrid is not None and not chain and fused_cpml
                      and self.cfg.scheme == "3d" and self.multi_cpml and self.halo is not None
                      and hasattr(self.ops, "curl_update_cpml_multi"))
        if multi:
            # 2D hybrid shell: every window of the half step in one launch (its
            # passes replay from a HIP graph, where a step costs its launch count)
            self.ops.curl_update_multi(kind, [{c: self.local_box(c, w) for c in comps} for w in windows], F, F,
                                       self.cb)
        elif multi_cpml:
            # decomposed 3D hybrid shell with the folded CPML: the windows of the half step in one launch
            # per row layout (a rank's small windows were launch-bound, profiles/decomp_r6.md)
            self.ops.curl_update_cpml_multi(kind, [{c: self.local_box(c, w) for c in comps} for w in windows], F, F,
                                            self.cb, ktab)
        elif len(windows) > 1 and not tfsf_here and self.hybrid is not None:
            # the hybrid shell's windows are disjoint: their launches of a half
            # step are independent and run side by side on several streams
            self._par_launches([(lambda w=w: one(w)) for w in windows])
        else:
            for w in windows:
                one(w)
        if cpml_once:
            alloc = self.domain.allocated_global()
            self.cpml.apply(kind, p, {c: self.local_box(c, alloc) for c in comps})
        if use_tfsf and tfsf_once:
            inc = self.hinc[p] if kind == "E" else self.einc[p]
            alloc = self.domain.allocated_global()
            many = []
            for c in comps:
                whole = self.local_box(c, alloc)
                for tab in self.tfsf[c]:
                    bb = getattr(tab, "bbox", None)
                    if (hasattr(self.ops, "tfsf_apply_many") and bb is not None
                            and all(whole[0][d] <= bb[0][d] and bb[1][d] <= whole[1][d] for d in range(3))):
                        many.append((F[c], tab))  # every target inside the update range
                    else:
                        self.ops.tfsf_apply(F[c], tab, inc, whole)
            if many:
                # the rest of the half step's tables in one or two launches
                self.ops.tfsf_apply_many(many, inc)
        if self.use_upml_chain:
            for c in comps:
                self._upml_rotate(c, p)

    def _par_launches(self, fns) -> None:
        """Run independent launch callables round-robin on ``--shell-streams``
        HIP streams (the current one first), joined back into the current
        stream: the tail of one small window launch overlaps the next instead
        of idling CUs.  Serial runs on the HIP path only.  The side streams
        fork before the first launch, so a callable must not create device
        data others read (lazy tables): build those before the call."""
        n = int(getattr(self.cfg, "shell_streams", 0))
        if n <= 0:
            # two streams: 512^3 alternating runs (profiles/physics_r6.md, tools/gpu_r6_as.sh) -- CPML + TF/SF
            # 96.0k vs 94.2k with three, UPML + TF/SF 92.3k vs 91.5k, fp64 CPML + TF/SF 49.1k vs 48.6k, Drude
            # + UPML 83.7k vs 84.0k
            n = 2 if self.ops.name == "hip" else 1
        # decomposed runs in order: their deep-halo shell windows on three
        # streams measured slower (2x2x1 of 512^3 CPML + TF/SF: 30.6k vs
        # 35.3k Mcells/s per GPU, tools/gpu_r5_zi.sh)
        if (n <= 1 or len(fns) <= 1 or self.halo is not None or self.device.type != "cuda"
                or getattr(self, "_capturing", False)):
            for f in fns:
                f()
            return
        main = torch.cuda.current_stream(self.device)
        pool = self.__dict__.get("_shell_pool")
        if pool is None or len(pool) < n - 1:
            pool = self._shell_pool = [torch.cuda.Stream(device=self.device) for _ in range(n - 1)]
        pool = pool[:n - 1]
        used = range(1, min(n, len(fns)))
        for k in used:
            # fork before the first launch: a wait recorded after it would
            # hold the side streams until the main stream's launch has ended
            pool[k - 1].wait_stream(main)
        for q, f in enumerate(fns):
            k = q % n
            if k == 0:
                f()
                continue
            with torch.cuda.stream(pool[k - 1]):
                f()
        for k in used:
            main.wait_stream(pool[k - 1])

    def _update_chain_regions(self, kind: str, p: int, w: Optional[Box], tfsf_plain: bool = True,
                              plain_windows: Optional[Sequence[Box]] = None) -> None:
        """UPML/Drude step on window ``w``: plain float4 Yee kernels on the
        plain slabs, the fused chain kernel on the chain boxes (components whose
        chain box holds TF/SF targets take the generic D-form path there)."""
        comps = self.e_comps if kind == "E" else self.h_comps
        F = self.F[p]
        tfsf = self.cfg.use_tfsf
        inc = (self.hinc[p] if kind == "E" else self.einc[p]) if tfsf else None
        pws = tuple(plain_windows) if plain_windows is not None else None
        key = (kind, w, pws)
        cache = self.__dict__.setdefault("_chain_plan_cache", {})
        plan = cache.get(key)
        if plan is None:
            # the launch list of this (kind, window set) is static: built once
            # (the hybrid shell steps through T window sets every pass)
            plan = cache[key] = self._chain_plan(kind, w, pws)
        pfns = [(lambda boxes=boxes: self.ops.curl_update(kind, boxes, F, F, self.cb)) for boxes in plan["plain"]]
        fns = []
        slow_all = []
        for launches, slow in plan["chain"]:
            for sel, form, plain_form, fold, rows in launches:
                if rows is not None:
                    fns.append(lambda sel=sel, form=form, pf=plain_form, rows=rows: self.ops.chain_update(
                        kind, sel, F, self.upml, p, form, pf, cb=self.cb, rows=rows))
                elif fold is None:
                    fns.append(lambda sel=sel, form=form, pf=plain_form: self.ops.chain_update(
                        kind, sel, F, self.upml, p, form, pf))
                else:
                    fns.append(lambda sel=sel, form=form, pf=plain_form, fold=fold: self.ops.chain_update(
                        kind, sel, F, self.upml, p, form, pf, plain=fold, cb=self.cb))
            slow_all += slow
        if plain_windows is not None and self.hybrid is not None and not slow_all:
            # hybrid shell: plain slabs and chain boxes are disjoint -- their
            # launches run side by side on several streams (the float4 plain
            # kernels store only their own elements of a 4-cell group that
            # straddles an unaligned z border with a chain box: st4m)
            self._par_launches(pfns + fns)
        else:
            for f in pfns + fns:
                f()
        for c, b in slow_all:
            self._upml_region(kind, c, p, b)
        if tfsf and tfsf_plain:
            # corrections on every plain box (folded ones included), after all updates
            for boxes in plan["plain"] + plan["folded"]:
                for c in comps:
                    for tab in self.tfsf[c]:
                        self.ops.tfsf_apply(F[c], tab, inc, boxes[c])

    def _chain_plan(self, kind: str, w: Optional[Box], pws) -> dict:
        """Launches of one UPML/Drude step on window ``w`` (plain slabs cut to
        ``pws`` when given): local plain boxes per launch, and per chain box
        the fused chain launches (dispersive / non-dispersive form) plus the
        components that take the generic D-form path (TF/SF targets inside)."""
        comps = self.e_comps if kind == "E" else self.h_comps
        dom = self.domain
        tfsf = self.cfg.use_tfsf
        reg = self.chain_regions[kind]
        whole = dom.allocated_global()
        plain = []
        for r in reg["plain"]:
            for pw in (pws if pws is not None else [w]):
                boxes = {c: dom.to_local(box_intersect(r[c], pw)) for c in comps}
                if not all(box_empty(b) for b in boxes.values()):
                    plain.append(boxes)
        chain = []
        # (the hybrid shell's steps only: a whole-grid step runs the chain on the box's exported state)
        skip_disp = pws is not None and (self.drude_blk is not None or self._drude_plan is not None)
        for r, dru in reg["chain"]:
            if skip_disp and kind == "E" and all(r[c] == self._disp_chain.get(c) for c in comps):
                continue  # the Drude box runs inside the blocked passes (blocking.py _drude_pass)
            boxes = {c: dom.to_local(box_intersect(r[c], w if w is not None else whole)) for c in comps}
            if all(box_empty(b) for b in boxes.values()):
                continue
            fast, slow = {}, []
            for c in comps:
                b = boxes[c]
                tb = self.tfsf_bbox.get(c) if tfsf else None
                if tb is not None and not box_empty(b) and not box_empty(box_intersect(b, tb)):
                    slow.append((c, b))
                    fast[c] = (b[0], b[0])
                else:
                    fast[c] = b
            if self.cfg.scheme != "3d":
                # 2D: the chain boxes are the thin PML slabs (+ the dispersive
                # box); the factored per-component chain runs there
                chain.append(([], [(c, boxes[c]) for c in comps if not box_empty(boxes[c])]))
                continue
            # one launch per form: dispersive chain / non-dispersive chain
            launches = []
            for form in (True, False):
                sel = {c: (fast[c] if dru[c] == form else (fast[c][0], fast[c][0])) for c in comps}
                if any(not box_empty(b) for b in sel.values()):
                    rows = self._drude_rows(kind) if form and self._sigma0_launch(sel) else None
                    launches.append([sel, form, self.cfg.use_metamaterials and not form, None, rows])
            chain.append((launches, slow))
        folded = []
        if self.cfg.scheme == "3d" and getattr(self.ops, "chain_fold", False):
            # a thin plain box on the z side of a non-dispersive chain box with
            # the same or a narrower (x, y) footprint rides in that chain
            # launch: the rows a z PML slab shares with a shell window are
            # read once, whole
            def fits(pb, cbx):
                if box_empty(pb):
                    return True
                if box_empty(cbx) or pb[1][2] - pb[0][2] > 64:
                    return False
                if any(pb[0][d] < cbx[0][d] or pb[1][d] > cbx[1][d] for d in (0, 1)):
                    return False
                return pb[0][2] == cbx[1][2] or pb[1][2] == cbx[0][2]

            keep = []
            for boxes in plain:
                host = None
                for launches, _ in chain:
                    for L in launches:
                        if L[3] is None and not L[1] and all(fits(boxes[c], L[0][c]) for c in comps):
                            host = L
                            break
                    if host is not None:
                        break
                if host is None:
                    keep.append(boxes)
                else:
                    host[3] = {c: b for c, b in boxes.items() if not box_empty(b)}
                    folded.append(boxes)
            plain = keep
        chain = [([tuple(L) for L in launches], slow) for launches, slow in chain]
        return {"plain": plain, "chain": chain, "folded": folded}

    def _sigma0_launch(self, sel: Dict[str, Box]) -> bool:
        """True when every (local) box of a chain launch lies where all sigma
        vanish: there the chain collapses to the plain update away from the
        dispersive cells."""
        if not getattr(self.ops, "chain_rows", False) or not self.cfg.use_metamaterials:
            return False
        for c, b in sel.items():
            if box_empty(b):
                continue
            z = self.domain.to_local(self._chain_sigma0[c])
            if box_empty(z) or any(b[0][d] < z[0][d] or b[1][d] > z[1][d] for d in range(3)):
                return False
        return True

    def _drude_rows(self, kind: str):
        """Per local row (x, y): the z range [z0, z1) holding every dispersive
        cell of the kind's components (int32 ``(nx, ny, 2)`` over the rows'
        bounding box, plus its origin).  Dispersive chain launches on sigma = 0
        boxes run the chain inside the ranges only and the plain update on the
        rest of the box: ~half of a sphere's bounding box, whose D / D1 levels
        are then never touched (reference: every cell of the grid runs the
        ADE sweep, Scheme3D.cpp:326-364)."""
        cache = self.__dict__.setdefault("_drude_rows_cache", {})
        if kind in cache:
            return cache[kind]
        comps = self.e_comps if kind == "E" else self.h_comps
        m = None
        for c in comps:
            a = self.upml[c].get("drude_active")
            if a is not None:
                m = a.clone() if m is None else (m | a)
        if m is None or not bool(m.any()):
            cache[kind] = None
            return None
        rows_any = m.any(dim=2)
        xs = torch.nonzero(rows_any.any(dim=1)).flatten()
        ys = torch.nonzero(rows_any.any(dim=0)).flatten()
        x0, x1, y0, y1 = int(xs.min()), int(xs.max()) + 1, int(ys.min()), int(ys.max()) + 1
        sub = m[x0:x1, y0:y1, :].to(torch.int8)
        nz = sub.shape[2]
        has = sub.any(dim=2)
        first = torch.argmax(sub, dim=2)
        last = nz - 1 - torch.argmax(torch.flip(sub, dims=(2,)), dim=2)
        z0 = torch.where(has, first, torch.zeros_like(first))
        z1 = torch.where(has, last + 1, torch.zeros_like(last))
        tab = torch.stack([z0, z1], dim=-1).to(torch.int32).contiguous()
        cache[kind] = (tab, x0, y0)
        return cache[kind]

    def _upml_region(self, kind: str, c: str, p: int, box: Box) -> None:
        F = self.F[p]
        st = self.upml[c]
        D = st["D"][p]
        Dn = D[-1]
        Dc = D[0]
        self.ops.curl_general(kind, c, box, Dn, Dc, F, st["caD"], st["cbD"])
        if self.cfg.use_tfsf:
            inc = self.hinc[p] if kind == "E" else self.einc[p]
            for tab in self.tfsf_D[c]:
                self.ops.tfsf_apply(Dn, tab, inc, box)
        if st.get("D1") is not None:
            self._drude_cells(c)
            D1 = st["D1"][p]
            D1n, D1c, D1p = D1[2], D1[0], D1[1]
            Dp = D[1]
            self.ops.lincomb(D1n, box, [(st["b0"], Dn), (st["b1"], Dc), (st["b2"], Dp),
                                        (st["ma1"], D1c), (st["ma2"], D1p)])
            src_new, src_old = D1n, D1c
            cbE, ccE = st["cbE"], st["ccE"]
        else:
            src_new, src_old = Dn, Dc
            # a non-dispersive component of a metamaterial run: E from D
            # through 1/(eps eps0) (the plain form; D1 = D/(eps eps0) exactly)
            pl = st.get("plain")
            cbE, ccE = (pl["cbE"], pl["ccE"]) if pl is not None else (st["cbE"], st["ccE"])
        self.ops.lincomb(F[c], box, [(st["caE"], F[c]), (cbE, src_new), (ccE, src_old)])

    def _upml_rotate(self, c: str, p: int) -> None:
        """new -> cur -> prev (the reference's ``nextTimeStep`` shift)."""
        st = self.upml[c]
        D = st["D"][p]
        if len(D) == 3:
            D[0], D[1], D[2] = D[2], D[0], D[1]
            D1 = st["D1"][p]
            D1[0], D1[1], D1[2] = D1[2], D1[0], D1[1]
        else:
            D[0], D[1] = D[1], D[0]

    def named_state(self) -> Dict[str, torch.Tensor]:
        """Every array needed to resume the run, by stable name (checkpoints).
        The blocked Drude pass's state goes back into the chain levels first
        (the next pass re-reads them), so either path resumes the other's."""
        self._drude_blk_export()
        out: Dict[str, torch.Tensor] = {}
        for p in range(self.planes):
            sfx = "" if p == 0 else "-im"
            for c in self.comps:
                out[c + sfx] = self.F[p][c]
            if self.use_upml_chain:
                for c in self.comps:
                    lists = [("%s%s" % ("D" if c[0] == "E" else "B", c[1]), self.upml[c]["D"][p])]
                    if self.upml[c].get("D1") is not None:
                        lists.append(("%s1%s" % ("D" if c[0] == "E" else "B", c[1]), self.upml[c]["D1"][p]))
                    for base, levels in lists:
                        for lv, t in enumerate(levels):
                            if isinstance(t, RegionLevel):
                                for q, part in enumerate(t.data):
                                    out["%s-aux%d-r%d%s" % (base, lv, q, sfx)] = part
                            else:
                                out["%s-aux%d%s" % (base, lv, sfx)] = t
            if self.use_cpml:
                for c, slabs in self.cpml.slabs.items():
                    for n, sl in enumerate(slabs):
                        out["psi-%s-%s-a%d-s%d%s" % (c, sl.src, sl.axis, sl.side, sfx)] = sl.psi[p]
            if self.cfg.use_tfsf:
                out["EInc" + sfx] = self.einc[p]
                out["HInc" + sfx] = self.hinc[p]
            if self.cfg.use_amp_mode:
                for c in self.comps:
                    out["%sAmplitude%s" % (c, sfx)] = self.amp[p][c]
        return out

    def state_tensors(self) -> List[torch.Tensor]:
        """Every array that carries state between steps (for deep-halo
        exchanges and checkpoints)."""
        out = []
        for p in range(self.planes):
            out += [self.F[p][c] for c in self.comps]
            if self.use_upml_chain:
                for c in self.comps:
                    for levels in (self.upml[c]["D"][p], self.upml[c].get("D1") and self.upml[c]["D1"][p]):
                        for t in (levels or ()):
                            out += list(t.data) if isinstance(t, RegionLevel) else [t]
            if self.use_cpml:
                out += self.cpml.state_tensors(p)
        db = self.drude_blk
        if db is not None:
            # the blocked Drude pass's current state set (float4 per box cell, seen
            # as z x 4 floats; models/blocking.py _drude_pass)
            s0, s1 = db["state"][db["cur"]]
            out += [s0.view(s0.shape[0], s0.shape[1], -1), s1.view(s1.shape[0], s1.shape[1], -1)]
        return out

    def state_boxes(self) -> List[Optional[Tuple[Box, Tuple[int, int, int]]]]:
        """Per :meth:`state_tensors` entry: None for arrays of the local field
        shape, else (global box the array covers, local index of its first
        element) -- the CPML psi slabs, whose ghost parts a deep-halo exchange
        moves through the same messages."""
        out = []
        for p in range(self.planes):
            out += [None] * len(self.comps)
            if self.use_upml_chain:
                for c in self.comps:
                    for levels in (self.upml[c]["D"][p], self.upml[c].get("D1") and self.upml[c]["D1"][p]):
                        for t in (levels or ()):
                            if isinstance(t, RegionLevel):
                                out += [(self.domain.to_global(b), b[0]) for b in t.boxes]
                            else:
                                out.append(None)
            if self.use_cpml:
                out += self.cpml.state_boxes(p)
        db = self.drude_blk
        if db is not None:
            cover = self.domain.to_global(db["box"])
            out += [(cover, db["box"][0], 4)] * 2  # (global box, local first index, z cells x 4 floats)
        return out

    def _apply_sources(self, t: int, p: int) -> None:
        if self.line_source is not None and self.cfg.use_amp_mode and self.in_amplitude:
            comp, offs = self.line_source
            if offs.numel():
                self.ops.set_values(self.F[p][comp], offs, self.source_value(t, p))
            return
        if self.point_source is not None:
            comp, li, _ = self.point_source
            if li is not None:
                if self._graph_src is not None:
                    tab, counter, t0 = self._graph_src
                    self.ops.set_value_tab(self.F[p][comp], li, tab[p], counter, t - t0)
                else:
                    self.ops.set_value(self.F[p][comp], li, self.source_value(t, p))

    in_amplitude = False

    def step(self, windows: Optional[Sequence[Box]] = None) -> None:
        """Advance one full leapfrog step (serial runs: optionally only on the
        global ``windows``, disjoint boxes -- the stepped shell of a hybrid
        blocked pass)."""
        t = self.t
        cfg = self.cfg
        B = self.domain.buffer_size
        halo = self.halo
        if self.drude_blk is not None and windows is None:
            self._drude_blk_export()  # a whole-grid step runs the chain on the Drude box
        if self.fused:
            self._fused_step(t)
            return
        deep = halo is not None and B > 1
        if deep and self.sub_step == 0:
            if getattr(self, "_deep_fresh", False):
                self._deep_fresh = False  # a hybrid pass exchanged already
            else:
                with self.prof.phase("halo-deep"):
                    halo.exchange_all(self)
        ph = self.prof.phase
        use_tfsf = cfg.use_tfsf
        for p in range(self.planes):
            if use_tfsf:
                with ph("incident-E"):
                    if self._graph_src is not None:
                        tab, counter, t0 = self._graph_src
                        self.ops.inc_step_e_tab(self.einc[p], self.hinc[p], self.inc_ce, tab[p], counter, t - t0)
                    else:
                        self.ops.inc_step_e(self.einc[p], self.hinc[p], self.inc_ce, self.source_value(t, p))
            with ph("E"):
                if halo is not None and not deep:
                    halo.finish_and_update(self, "E", p)
                else:
                    self._update("E", p, windows, tfsf_once=windows is not None and self._tfsf_once)
            with ph("source"):
                self._apply_sources(t, p)
            if halo is not None and not deep:
                with ph("halo-post"):
                    halo.start(self, "E", p)
            if use_tfsf:
                with ph("incident-H"):
                    self.ops.inc_step_h(self.einc[p], self.hinc[p], self.inc_ch)
            with ph("H"):
                if halo is not None and not deep:
                    halo.finish_and_update(self, "H", p)
                else:
                    self._update("H", p, windows, tfsf_once=windows is not None and self._tfsf_once)
            if halo is not None and not deep:
                with ph("halo-post"):
                    halo.start(self, "H", p)
        self.t += 1
        if deep:
            self.sub_step = (self.sub_step + 1) % B
        for h in self.hooks:
            h(self, self.t)
        if cfg.check_finite and self.t % max(1, cfg.finite_check_step) == 0:
            self.check_finite()

    def _fused_step(self, t: int) -> None:
        """One step through the fused E+H kernel.  Decomposed runs use the
        deep-halo protocol for any buffer size (a full ghost exchange every
        ``B`` steps, redundant compute in between)."""
        B = self.domain.buffer_size
        if self.halo is not None and B == 1:
            self._fused_step_overlap(t)
            return
        if self.halo is not None and self.sub_step == 0:
            with self.prof.phase("halo-deep"):
                self.halo.exchange_all(self)
        wE = self.domain.window_fused("E", self.sub_step)
        wH = self.domain.window_fused("H", self.sub_step)
        boxes = {c: self.local_box(c, wE) for c in self.e_comps}
        boxes.update({c: self.local_box(c, wH) for c in self.h_comps})
        for p in range(self.planes):
            src = None
            if self.point_source is not None and self.point_source[1] is not None:
                comp, li, _ = self.point_source
                src = (comp, li, self.source_value(t, p))
            with self.prof.phase("fused-E+H"):
                self.ops.fused_step(self.F[p], self.F_alt[p], boxes, self.cb, src)
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]
        self.t += 1
        if self.halo is not None:
            self.sub_step = (self.sub_step + 1) % B
        for h in self.hooks:
            h(self, self.t)
        if self.cfg.check_finite and self.t % max(1, self.cfg.finite_check_step) == 0:
            self.check_finite()

    def _fused_regions(self):
        """(E box, H box) global pairs of the overlapped fused step: first the
        interior (needs no ghost), then the one-cell H shell slabs next to
        neighbours, each with the E cells its H update needs."""
        key = "_fused_regions_cache"
        cached = getattr(self, key, None)
        if cached is not None:
            return cached
        dom = self.domain
        wE = dom.window_fused("E", 0)
        wH = dom.window_fused("H", 0)
        hl = [dom.has_low(a) for a in range(3)]
        hh = [dom.has_high(a) for a in range(3)]
        hI = (tuple(dom.lo[a] + (1 if hl[a] else 0) for a in range(3)),
              tuple(dom.hi[a] - (1 if hh[a] else 0) for a in range(3)))
        eI = box_intersect(wE, (hI[0], tuple(hI[1][a] + 1 for a in range(3))))
        regions = [(eI, hI)]
        lo, hi = list(wH[0]), list(wH[1])
        for a in range(3):
            for side in (0, 1):
                if (side == 0 and hl[a]) or (side == 1 and hh[a]):
                    slo, shi = list(lo), list(hi)
                    if side == 0:
                        shi[a] = lo[a] + 1
                        lo[a] += 1
                    else:
                        slo[a] = hi[a] - 1
                        hi[a] -= 1
                    S = (tuple(slo), tuple(shi))
                    if box_empty(S):
                        continue
                    E = box_intersect(wE, (S[0], tuple(S[1][d] + 1 for d in range(3))))
                    regions.append((E, S))
        setattr(self, key, regions)
        return regions

    def _fused_step_overlap(self, t: int) -> None:
        """Decomposed fused step (``--buffer-size 1``): the interior update runs
        while the 1-deep ghost exchange (all axes, edges included) proceeds on
        a side stream; the boundary shell follows once the ghosts are in."""
        regions = self._fused_regions()

        def boxes_of(eb, hb):
            b = {c: self.local_box(c, eb) for c in self.e_comps}
            b.update({c: self.local_box(c, hb) for c in self.h_comps})
            return b

        srcs = []
        for p in range(self.planes):
            src = None
            if self.point_source is not None and self.point_source[1] is not None:
                comp, li, _ = self.point_source
                src = (comp, li, self.source_value(t, p))
            srcs.append(src)
        interior = boxes_of(*regions[0])
        side = self._fork_side_stream()
        for p in range(self.planes):
            self.ops.fused_step(self.F[p], self.F_alt[p], interior, self.cb, srcs[p])
        self.halo.exchange_all(self, stream=side)
        if side is not None:
            torch.cuda.current_stream(self.device).wait_stream(side)
        for eb, hb in regions[1:]:
            bx = boxes_of(eb, hb)
            for p in range(self.planes):
                self.ops.fused_step(self.F[p], self.F_alt[p], bx, self.cb, srcs[p])
        for p in range(self.planes):
            self.F[p], self.F_alt[p] = self.F_alt[p], self.F[p]
        self.t += 1
        for h in self.hooks:
            h(self, self.t)
        if self.cfg.check_finite and self.t % max(1, self.cfg.finite_check_step) == 0:
            self.check_finite()

    def add_periodic(self, period: int, offset: int, fn: Callable[["YeeScheme", int], None]) -> None:
        """Run ``fn(scheme, t)`` after every step ``t`` with ``(t - offset) %
        period == 0`` (see ``self.periodic``)."""
        self.periodic.append((max(1, int(period)), int(offset), fn))

    def _next_periodic(self, t0: int, t1: int) -> int:
        """First step in ``(t0, t1]`` at which periodic work fires (``t1`` if none)."""
        nxt = t1
        for period, off, _ in self.periodic:
            t = t0 + 1 + ((off - (t0 + 1)) % period)
            nxt = min(nxt, t)
        return nxt

    def advance(self, n: int) -> None:
        """``n`` leapfrog steps; blocked / hybrid passes end at every step at
        which periodic work fires, which then runs between passes."""
        end = self.t + n
        while self.t < end:
            nxt = self._next_periodic(self.t, end) if self.periodic else end
            self._advance(nxt - self.t)
            for period, off, fn in self.periodic:
                if (self.t - off) % period == 0:
                    fn(self, self.t)

    def _advance(self, n: int) -> None:
        """``n`` leapfrog steps, ``self.tb`` at a time through the temporally
        blocked kernel where possible (no per-step hooks; a tail shorter than
        ``self.tb`` is one shorter pass), single fused steps otherwise."""
        T = self.tb
        if getattr(self, "res1d", False) and not self.hooks and n > 0:
            self._resident_1d(n)
            return
        if self.hybrid is not None and not self.hooks:
            P = self._hybrid_graph_passes()
            if P and n >= (P + 2) * self.hybrid["T"]:
                n -= self._hybrid_graph(n, P)
            while n > 0:
                k = min(self.hybrid["T"], n)
                self._hybrid_step(k)
                n -= k
            return
        if self.graph_mode and not self.hooks and n >= GRAPH_STEPS:
            n -= self._advance_graph(n)
        while n > 0:
            if T > 1 and not self.hooks and self.sub_step == 0:
                # a short tail runs as one shorter blocked pass (its ghosts are
                # T deep anyway), so the next call starts on a pass boundary
                k = min(T, n)
                self._tb_step(k)
                n -= k
            else:
                self.step()
                n -= 1

    def _hybrid_graph_passes(self) -> int:
        """Hybrid passes per HIP graph (0: no graph).  A 2D pass's stepped
        shell is a few thin strips, so a step is ~30 small launches whose host
        cost (not the GPU) bounds the rate.  (3D passes are GPU-bound: graphs
        measured no faster with the capture done in the warm-up and 13-30%
        slower with it in the timed run, profiles/graph2d_r4.md.)  Needs: 2D,
        serial HIP run, no per-step hooks (periodic work runs between
        ``_advance`` calls; a replayed graph is reused only while
        :meth:`_state_order_key` matches its capture), no point source inside
        a core box (the core pass takes its values as launch arguments), and a
        pass count after which the field buffers (2) and the UPML / Drude
        level lists (2 or 3 levels) are back in place."""
        hp = self.hybrid
        if (hp is None or self.cfg.scheme not in ("tmz", "tez") or self.halo is not None or self.hooks
                or self.ops.name != "hip" or self.device.type != "cuda" or self.prof.enabled
                or not hasattr(self.ops, "inc_step_e_tab") or not hasattr(self.ops, "counter_add")
                or getattr(self.cfg, "hybrid_graph", "auto") == "off"):
            return 0
        if self.point_source is not None and self.point_source[1] is not None:
            li = self.point_source[1]
            if any(all(b[0][d] <= li[d] < b[1][d] for d in range(3)) for b in hp["core"]):
                return 0
        levels = {2}
        if self.use_upml_chain:
            levels |= {self.upml[c].get("nlev", 2) for c in self.comps}
        T = hp["T"]
        for P in range(2, 13, 2):
            if all((P * T) % L == 0 for L in levels):
                return P
        return 0

    def _state_order_key(self) -> tuple:
        """Identity of every rotating state buffer in its current role: the
        field buffer set of each plane and, with the UPML chain, the order of
        each component's D (and Drude D1) level list, which ``_upml_rotate``
        permutes every step.  A captured graph bakes these pointers in, so it
        may be replayed only while the key is unchanged (two calls of
        ``advance`` can leave the fields in the captured parity but the level
        lists rotated: an odd number of steps in an even number of passes)."""
        key = [self.F[p][self.comps[0]].data_ptr() for p in range(self.planes)]
        if self.use_upml_chain:
            for c in self.comps:
                st = self.upml[c]
                for name in ("D", "D1"):
                    lv = st.get(name)
                    if lv:
                        key += [id(x) for p in range(self.planes) for x in lv[p]]
        return tuple(key)

    def _hybrid_graph(self, n: int, P: int) -> int:
        """Replay ``P`` hybrid passes at a time from one HIP graph; the shell's
        sources (incident line, point source) read a device table through a
        step counter the graph advances (the ``_graph_src`` path of
        :meth:`step`).  The graph is captured once and kept while its buffers
        are the current ones (:meth:`_state_order_key`: field-buffer parity
        and UPML level order; table long enough); later calls refill the
        table and reset the counter.  Returns the steps taken."""
        T = self.hybrid["T"]
        taken = 0
        if not getattr(self, "_hybrid_warm", False):
            # one pass outside any graph first: first-use set-up (table
            # checks, compact TF/SF tables) may synchronise, which a capture
            # must not
            self._hybrid_step(T)
            self._hybrid_warm = True
            n -= T
            taken += T
        G = P * T
        reps = n // G
        if reps == 0:
            return taken
        t0 = self.t
        vals = torch.tensor([[self.source_value(t0 + i, p) for i in range(reps * G)] for p in range(self.planes)],
                            dtype=torch.float64)
        key = (P, T, self._state_order_key())
        if getattr(self.cfg, "hybrid_graph", "auto") != "graph" and hasattr(self.ops, "record"):
            return taken + self._hybrid_replay(reps, P, T, t0, vals, key)
        g = self.__dict__.get("_hgraph")
        if g is None or g["key"] != key or g["reps"] < reps:
            tab = torch.zeros((self.planes, reps * G), dtype=torch.float64, device=self.device)
            counter = torch.zeros(1, dtype=torch.int32, device=self.device)
            graph = torch.cuda.CUDAGraph()
            self._graph_src = (tab, counter, t0)
            # one stream inside the graph (cross-stream joins as graph nodes
            # measured slower than the plain chain of small kernels)
            self._capturing = True
            try:
                with torch.cuda.graph(graph):
                    for _ in range(P):
                        self._hybrid_step(T)
                    self.ops.counter_add(counter, G)
            finally:
                self._graph_src = None
                self._capturing = False
            self.t = t0  # capture records the kernels, it does not run them
            g = self._hgraph = {"key": key, "reps": reps, "graph": graph, "tab": tab, "counter": counter}
        g["tab"][:, :reps * G].copy_(vals)
        g["counter"].zero_()
        for _ in range(reps):
            g["graph"].replay()
        self.t = t0 + reps * G
        return taken + reps * G

    def _hybrid_replay(self, reps: int, P: int, T: int, t0: int, vals: torch.Tensor, key: tuple) -> int:
        """``reps`` times ``P`` hybrid passes from a launch record: the first
        ``P`` passes run with the ops recording their library calls (one
        stream, sources read from the device table through the counter, as a
        graph would), the other repetitions re-issue the recorded calls from
        a list (``HipOps.replay``) -- the kernels of a pass without the Python
        planning around them.  Direct launches on the stream pipeline better
        than a replayed HIP graph of the same ~80 small kernels a pass (2D
        8192^2 CPML + TF/SF: the graph's GPU idled ~40% between its nodes,
        profiles/graph2d_r6.md).  The record is kept while its buffers are
        the current ones (:meth:`_state_order_key`) and its table is long
        enough.  Returns the steps taken."""
        G = P * T
        r = self.__dict__.get("_hrec")
        done = 0
        if r is None or r["key"] != key or r["reps"] < reps:
            tab = torch.zeros((self.planes, reps * G), dtype=torch.float64, device=self.device)
            counter = torch.zeros(1, dtype=torch.int32, device=self.device)
            tab.copy_(vals)
            rec = []
            self._graph_src = (tab, counter, t0)
            self._capturing = True  # one stream: no shell-stream forks (torch stream waits are not recorded)
            self.ops.record(rec)
            try:
                for _ in range(P):
                    self._hybrid_step(T)
                self.ops.counter_add(counter, G)
            finally:
                self.ops.record(None)
                self._graph_src = None
                self._capturing = False
            r = self._hrec = {"key": key, "reps": reps, "rec": rec, "tab": tab, "counter": counter}
            done = 1
        else:
            r["tab"][:, :reps * G].copy_(vals)
            r["counter"].zero_()
        for _ in range(reps - done):
            self.ops.replay(r["rec"])
        self.t = t0 + reps * G
        return reps * G

    def _resident_1d(self, n: int) -> None:
        """``n`` 1D steps in one launch per plane (ops.resident_1d): per-step
        source values go to the device as one table."""
        boxes = {c: self.local_box(c, self._window(c[0])) for c in self.comps}
        for p in range(self.planes):
            vals, si = None, None
            if self.point_source is not None and self.point_source[1] is not None:
                comp, li, _ = self.point_source
                fdtd_assert(comp == "Ez", "1D point source must drive Ez")
                si = li[0]
                vals = self.source_values(self.t, n, p).to(self.device, self.dtype)
            with self.prof.phase("resident-1d"):
                self.ops.resident_1d(self.F[p], boxes, self.cb, n, si, vals)
        self.t += n
        if self.cfg.check_finite:
            self.check_finite()

    def _advance_graph(self, n: int) -> int:
        """Capture GRAPH_STEPS steps into one HIP graph and replay it
        ``n // GRAPH_STEPS`` times; returns the steps taken.  Sources read a
        device table through a device step counter that the graph advances,
        and GRAPH_STEPS is a multiple of 6, so the UPML / Drude level lists
        (rotated every step) are back in place at the end of each replay."""
        G = GRAPH_STEPS
        reps = n // G
        t0 = self.t
        tab = torch.tensor([[self.source_value(t0 + i, p) for i in range(reps * G)] for p in range(self.planes)],
                           dtype=torch.float64, device=self.device)
        counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        graph = torch.cuda.CUDAGraph()
        self._graph_src = (tab, counter, t0)
        try:
            with torch.cuda.graph(graph):
                for _ in range(G):
                    self.step()
                self.ops.counter_add(counter, G)
        finally:
            self._graph_src = None
        self.t = t0  # capture records the kernels, it does not run them
        for _ in range(reps):
            graph.replay()
        self.t = t0 + reps * G
        self._graph = (graph, tab, counter)  # keep alive until the stream has drained
        return reps * G

    def perform_steps(self, n: Optional[int] = None) -> None:
        """``Scheme3D::performSteps`` (Scheme3D.cpp:3336-3385)."""
        n = self.cfg.time_steps if n is None else n
        self.advance(n)
        if self.cfg.use_amp_mode:
            self.amplitude_taken = self.perform_amplitude_steps()

    # ------------------------------------------------------------ amplitude
    def amplitude_box(self, c: str) -> Box:
        """Computation box of ``c`` minus PML cells (Scheme3D.cpp:3016-3030)."""
        lo_g, hi_g = self._global_box(c)
        lay = self.layout
        left, right = lay.pml_borders()
        # first / one-past-last index along each axis whose real coordinate
        # lies outside the PML slabs (the reference's !isInPML per axis)
        m0 = lay.coord_fp(c, (0, 0, 0))
        lo, hi = list(lo_g), list(hi_g)
        for a in lay.axes:
            if left[a] != right[a]:
                lo[a] = max(lo[a], int(math.ceil(left[a] - m0.c[a])))
                hi[a] = min(hi[a], int(math.ceil(right[a] - m0.c[a])))
        b = box_intersect((tuple(lo), tuple(hi)), self.domain.owned_global())
        return self.domain.to_local(b)

    # the stop is exact (at the stable step, not at the end of its check
    # period) whenever the period before it ended with at most this share of
    # the amplitude cells changing: that period starts from a snapshot
    AMP_SNAPSHOT_SHARE = 0.02

    def perform_amplitude_steps(self) -> int:
        """Steady-state mode: keep stepping until no cell's running max |f|
        grows by more than ``ACCURACY`` (relative), or until
        ``amplitude_steps`` extra steps.  The reference loop never sets its
        stable flag (``Scheme3D.cpp:2945-3291``); this implements the
        documented intent.  Returns the number of steps taken.

        The changed-cell counts of ``--amplitude-check-steps`` K steps
        accumulate on the device and are read once per period.  Near
        convergence (the previous period's last count at most
        ``AMP_SNAPSHOT_SHARE`` of the amplitude cells) a period starts from a
        snapshot of the whole state; when one of its steps changes nothing,
        the state goes back to the snapshot and exactly the steps up to the
        stable one are replayed -- the run stops where K = 1 would.  A period
        that drops to zero without a snapshot ends the run at its end (logged)."""
        fdtd_assert(self.planes == 1, "amplitude mode needs real field values (reference asserts the same)")
        self.in_amplitude = True
        K = max(1, int(getattr(self.cfg, "amplitude_check_steps", 8)))
        boxes = [self.amplitude_box(c) for c in self.comps]
        counts = torch.zeros(K, dtype=torch.int32, device=self.device)
        self.amplitude_counts = []  # changed cells of every step taken
        cells = sum(max(0, b[1][0] - b[0][0]) * max(0, b[1][1] - b[0][1]) * max(0, b[1][2] - b[0][2]) for b in boxes)
        if self.halo is not None:
            cells = self.halo.allreduce_sum(cells)
        near = max(1, int(self.AMP_SNAPSHOT_SHARE * cells))
        taken = 0
        T = self._amp_blocked_steps()

        def period(n):
            counts.zero_()
            s_ = 0
            while s_ < n:
                if T > 1 and n - s_ >= 2:
                    # blocked pass with the amplitude update of every step
                    # folded in (csrc/tb3d_mr.h AmpDev)
                    k = min(T, n - s_)
                    self._amp_tb_step(k, boxes, counts[s_:s_ + k])
                    s_ += k
                    continue
                self.step()
                self.ops.amplitude_update_many([self.F[0][c] for c in self.comps],
                                               [self.amp[0][c] for c in self.comps], boxes, ACCURACY,
                                               counts[s_:s_ + 1])
                s_ += 1
            got = [int(v) for v in counts[:n].cpu()]
            if self.halo is not None:
                got = [self.halo.allreduce_sum(v) for v in got]
            return got

        try:
            last = None
            while taken < self.cfg.amplitude_steps:
                n = min(K, self.cfg.amplitude_steps - taken)
                snap = None
                if n > 1 and last is not None and last <= near:
                    snap = ({k: v.clone() for k, v in self.named_state().items()}, self.t, self.sub_step)
                got = period(n)
                first = next((s_ for s_ in range(n) if got[s_] == 0 and taken + s_ + 1 > 1), None)
                if first is None:
                    self.amplitude_counts += got
                    last = got[-1]
                    taken += n
                    continue
                self.amplitude_converged = True
                self.amplitude_stable_step = taken + first + 1
                if first + 1 < n:
                    if snap is None:
                        log.log(0, "amplitude mode: stable at step %d, the run ends with its check period (%d steps)"
                                % (taken + first + 1, taken + n))
                    else:
                        # back to the period's start, then exactly the steps up to the stable one
                        state, t0, sub0 = snap
                        for k, v in self.named_state().items():
                            v.copy_(state[k])
                        self.t, self.sub_step = t0, sub0
                        got = period(first + 1)
                        n = first + 1
                self.amplitude_counts += got
                return taken + n
            self.amplitude_converged = False
            log.log(0, "amplitude mode: stable state not reached after %d steps" % taken)
            return taken
        finally:
            self.in_amplitude = False

    def _amp_blocked_steps(self) -> int:
        """Steps per blocked amplitude pass (1: per-step stepping).  Serial
        3D runs of uniform media without PML, TF/SF, dispersive media or
        hooks, whose ops fold the amplitude update into the blocked kernel."""
        cfg = self.cfg
        if (cfg.scheme != "3d" or self.halo is not None or self.planes != 1 or cfg.use_pml or cfg.use_tfsf
                or cfg.use_metamaterials or self.hooks or not hasattr(self.ops, "tb_amp_step")
                or getattr(self, "line_box", None) is None or cfg.check_finite):
            return 1
        if any(getattr(self.cb.get(c), "cell", None) is not None for c in self.comps):
            return 1
        if self.ops.name == "hip" and (self.dtype != torch.float32 or self.domain.shape[2] % 4 != 0):
            return 1
        T = min(AMP_TB_STEPS, getattr(self.ops, "tb_amp_max_steps", 1))
        if T > 1 and not hasattr(self, "F_alt"):
            self.F_alt = [{c: self._zeros() for c in self.comps} for _ in range(self.planes)]
        return T

    def _amp_tb_step(self, T: int, aboxes, counts: torch.Tensor) -> None:
        upd, outs = self._tb_regions(T)
        vals = [self.source_value(self.t + l, 0) for l in range(T)]
        self.ops.tb_amp_step(self.F[0], self.F_alt[0], upd, outs[0], self.cb, T, self.line_box, vals,
                             [self.amp[0][c] for c in self.comps], aboxes, ACCURACY, counts)
        self.F[0], self.F_alt[0] = self.F_alt[0], self.F[0]
        self.t += T

    # -------------------------------------------------------------- checks
    def check_finite(self) -> None:
        for p in range(self.planes):
            for c in self.comps:
                m = self.ops.maxabs(self.F[p][c], ((0, 0, 0), tuple(self.domain.shape)))
                if not math.isfinite(m):
                    raise FdtdError("non-finite values in %s at step %d" % (c, self.t))

    # -------------------------------------------------------------- access
    def field(self, comp: str, plane: int = 0) -> torch.Tensor:
        return self.F[plane][comp]

    def owned_field(self, comp: str, plane: int = 0) -> torch.Tensor:
        """View of the owned (non-ghost) part of a field."""
        gl = self.domain.ghost_lo
        s = self.domain.owned_shape
        return self.F[plane][comp][gl[0]:gl[0] + s[0], gl[1]:gl[1] + s[1], gl[2]:gl[2] + s[2]]

    def cells(self) -> int:
        n = 1
        for v in self.cfg.size:
            n *= v
        return n

    # ------------------------------------------------------- synthetic data
    def randomize_fields(self, seed: int = 1) -> None:
        """Pseudo-random E / H in [-1, 1) keyed by global cell index
        (utils/synthetic.py): a decomposed run starts from the same fields as
        a serial one.  The ping-pong buffer gets the same values, so cells a
        pass never stores (PEC, padding) agree in both.  H is scaled by
        1/eta0 so that E and H carry comparable energy."""
        from ..utils.synthetic import hash_fill
        eta0 = math.sqrt(MU0 / EPS0)
        for p in range(self.planes):
            for n, c in enumerate(self.comps):
                hash_fill(self.F[p][c], self.domain.origin, self.cfg.size, seed * 64 + p * 8 + n)
                if c[0] == "H":
                    self.F[p][c].mul_(1.0 / eta0)
                # cells a component never updates (PEC walls) stay zero: a
                # frozen non-zero tangential E would drive H linearly forever
                ub = self.local_box(c, self.domain.allocated_global())
                keep = torch.zeros_like(self.F[p][c], dtype=torch.bool)
                keep[ub[0][0]:ub[1][0], ub[0][1]:ub[1][1], ub[0][2]:ub[1][2]] = True
                self.F[p][c].masked_fill_(~keep, 0.0)
                for alt in (getattr(self, "F_alt", None),):
                    if alt is not None:
                        alt[p][c].copy_(self.F[p][c])

    def field_energy(self) -> float:
        """Vacuum field energy over this rank's owned cells in units of
        eps0 * cell volume: sum of E^2 + eta0^2 H^2 (fp64) -- the bench
        checksum (all-reduced by the caller)."""
        from ..utils.synthetic import energy
        box = self.domain.to_local(self.domain.owned_global())
        eta2 = MU0 / EPS0
        return sum(energy(self.F[p][c], box) * (eta2 if c[0] == "H" else 1.0)
                   for p in range(self.planes) for c in self.comps)
