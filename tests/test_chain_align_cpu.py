"""Chain boxes widened into sigma = 0 cells (the stepped 3D HIP path rounds
the z PML slabs' chain boxes to whole 128-byte row segments) give the same
fields as the exact slabs: there the UPML / Drude chain is the plain update
algebraically.  CPU, torch backend, the region logic forced on."""

import torch

from fdtd3d_amd.models.scheme import SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops


def _run(cfg, z_align):
    s = YeeScheme(cfg, make_ops("torch", None, "cpu", torch.float64))
    s.init_scheme()
    s.init_grids()
    if z_align > 1:
        s._init_chain_regions(s._chain_prof, z_align=z_align)
        zl = min(b[0][2] for r in s.chain_regions["E"]["plain"] for b in r.values() if b[1][2] > b[0][2])
        assert zl % z_align == 0 and zl > cfg.pml_size[2], zl
    s.perform_steps()
    return s


def test_z_aligned_chain_boxes_match():
    for scene, meta in (("vacuum", False), ("drude-sphere", True)):
        cfg = SchemeConfig(scheme="3d", size=(24, 20, 72), time_steps=12, use_pml=True, use_metamaterials=meta,
                           pml_size=(4, 4, 5), scene=scene, sphere_radius=5, sphere_center=(12.0, 10.0, 36.0),
                           dtype="f64")
        a = _run(cfg, 1)
        b = _run(cfg, 16)
        for c in a.comps:
            x, y = a.F[0][c], b.F[0][c]
            scale = float(x.abs().max()) + 1e-300
            assert float((x - y).abs().max()) <= 1e-12 * scale, (scene, c)
