"""CPML inside the multi-row blocked kernel (csrc/yee3d_tb.hip, FX bit 8):
one T-step pass over the whole grid vs T stepped steps of the split CPML
kernels, from random fields (every slab live from the first step).  T > 1
hands psi from level to level through thread-private scratch."""
import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu


def _mk(cfg, gpu):
    s = YeeScheme(cfg, make_ops("hip", None, gpu, torch.float32))
    s.init_scheme()
    s.init_grids()
    s.randomize_fields(seed=5)
    return s


def _where(d):
    i = int(d.abs().argmax())
    return tuple(int(v) for v in torch.unravel_index(torch.tensor(i), d.shape))


PML = {"x": (6, 0, 0), "y": (0, 6, 0), "z": (0, 0, 6), "xyz": (5, 6, 7)}


@pytest.mark.parametrize("T", [1, 4])
@pytest.mark.parametrize("axes", ["x", "y", "z", "xyz"])
@pytest.mark.parametrize("tfsf", [False, True])
def test_cpml_pass_vs_stepped(gpu, T, axes, tfsf):
    if tfsf and axes != "xyz":
        pytest.skip("TF/SF with all slabs only")
    cfg = SchemeConfig(scheme="3d", size=(48, 40, 72), dtype="f32", pml_size=PML[axes], tfsf_size=(9, 10, 11),
                       scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=tfsf, hybrid_block=1, time_steps=T)
    a, b = _mk(cfg, gpu), _mk(cfg, gpu)
    assert a.use_cpml and a.hybrid is None
    for _ in range(T):
        a.step()
    alloc = b.domain.allocated_global()
    upd = {c: b.local_box(c, alloc) for c in b.comps}
    out = {c: torch.zeros_like(b.F[0][c]) for c in b.comps}
    tf = b._tfsf_pass(0, T) if tfsf else None
    srcs = b._pass_sources(b.t, T)[0]
    # the whole grid's cone reaches every slab: the class of the configured axes
    cax = sum(1 << a for a in range(3) if PML[axes][a] > 0)
    b.ops.tb_step(b.F[0], out, upd, ((0, 0, 0), cfg.size), b.cb, T, srcs, tfsf=tf, cpml=b.cpml.host_table(0),
                  cpml_axes=cax)
    b.cpml.flip(0)
    torch.cuda.synchronize()
    bad = []
    for c in a.comps:
        d = (a.F[0][c] - out[c]).double().cpu()
        scale = max(float(a.F[0][o].abs().max()) for o in a.comps if o[0] == c[0])
        if float(d.abs().max()) > 2e-5 * scale:
            bad.append(("field", c, float(d.abs().max()), _where(d), scale))
        src_scale = max(float(a.F[0][o].abs().max()) for o in a.comps if o[0] != c[0])
        for sa, sb in zip(a.cpml.slabs[c], b.cpml.slabs[c]):
            d = (sa.psi[0] - sb.psi[0]).double().cpu()
            if float(d.abs().max()) > 2e-5 * src_scale:
                bad.append(("psi", c, "axis", sa.axis, "side", sa.side, sa.lbox, float(d.abs().max()), _where(d),
                            float(sa.psi[0].abs().max())))
    assert not bad, bad
