"""Geometry of the blocked / mixed shell plans (models/blocking.py
_hybrid3_plan, _hybrid4_plan) on the CPU: the core and the shell pieces tile
the grid exactly once; a piece's class carries every CPML axis whose slab its
dependency cone (the piece grown by T + 1) reaches and the TF/SF bit when the
cone holds a TF/SF target; the mixed plan's stepped windows are disjoint,
cover the stepped pieces, and grow by one cell per remaining step."""
import pytest
import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.parallel.domain import box_empty, box_intersect, box_volume


def _scheme(tfsf):
    cfg = SchemeConfig(scheme="3d", size=(56, 48, 60), dtype="f32", pml_size=(5, 6, 7), tfsf_size=(9, 10, 11),
                       scene="vacuum", use_pml=True, pml_type="cpml", use_tfsf=tfsf, time_steps=1, hybrid_block=1)
    ops = make_ops("torch", None, "cpu", torch.float32)
    ops.tb_cpml_steps = (1, 4)  # the HIP backend's CPML pass lengths
    s = YeeScheme(cfg, ops)
    s.init_scheme()
    s.init_grids()
    return s


def _grow(b, n):
    return (tuple(b[0][d] - n for d in range(3)), tuple(b[1][d] + n for d in range(3)))


def _cover_count(boxes, shape):
    cnt = torch.zeros(shape, dtype=torch.int32)
    for b in boxes:
        cnt[b[0][0]:b[1][0], b[0][1]:b[1][1], b[0][2]:b[1][2]] += 1
    return cnt


@pytest.mark.parametrize("tfsf", [True, False])
def test_blocked_plan_tiles_grid_and_classes(tfsf):
    s = _scheme(tfsf)
    T = 4
    plan = s._hybrid3_plan(T)
    assert plan is not None and plan["v3"]
    shape = tuple(s.domain.shape)
    cnt = _cover_count(plan["core"] + [b for b, _ in plan["shell"]], shape)
    assert int(cnt.min()) == 1 and int(cnt.max()) == 1  # every cell in exactly one launch box
    slabs = [sl for c in s.comps for sl in s.cpml.slabs[c]]
    for b, cls in plan["shell"]:
        g = _grow(b, T + 1)
        need = 0
        for sl in slabs:
            if not box_empty(box_intersect(g, sl.gbox)):
                need |= 1 << sl.axis
        assert cls & 7 == need, (b, cls, need)
        assert bool(cls & 8) == bool(tfsf and s._tfsf_targets_in(g))
    # the core's cone holds no CPML cell and no TF/SF target
    for K in plan["core"]:
        g = _grow(K, T + 1)
        assert all(box_empty(box_intersect(g, sl.gbox)) for sl in slabs)
        assert not (tfsf and s._tfsf_targets_in(g))
    # face, edge and corner classes all occur
    assert {1, 2, 4} <= {cls & 7 for _, cls in plan["shell"]}
    assert {3, 5, 6, 7} <= {cls & 7 for _, cls in plan["shell"]}


def test_mixed_plan_windows():
    s = _scheme(True)
    T = 4
    p3 = s._hybrid3_plan(T)
    p4 = s._hybrid4_plan(p3)
    assert p4["v4"]
    shape = tuple(s.domain.shape)
    assert all((cls & 7) in (0, 1, 2) for _, cls in p4["shell"])
    stepped = p4["copy"]
    assert stepped and all(box_volume(b) > 0 for b in stepped)
    # blocked launches + stepped pieces still tile the grid once
    cnt = _cover_count(p4["core"] + [b for b, _ in p4["shell"]] + stepped, shape)
    assert int(cnt.min()) == 1 and int(cnt.max()) == 1
    full = _cover_count(stepped, shape) > 0
    for st, win in enumerate(p4["windows"]):
        wc = _cover_count(win, shape)
        assert int(wc.max()) == 1  # disjoint: no cell stepped twice in place
        d = T - st
        # exactly the stepped pieces grown by T - s (clipped to the grid)
        want = torch.zeros(shape, dtype=torch.bool)
        for b in stepped:
            g = _grow(b, d)
            want[max(0, g[0][0]):g[1][0], max(0, g[0][1]):g[1][1], max(0, g[0][2]):g[1][2]] = True
        assert torch.equal(wc > 0, want), st
        assert bool((wc > 0)[full].all())
    # psi copy-back only from x / y face pieces, inside their slabs
    for sl, sub in p4["psi_fix"]:
        assert sl.axis in (0, 1)
        assert all(sub[d].start >= 0 and sub[d].stop <= sl.psi[0].shape[d] for d in range(3))
