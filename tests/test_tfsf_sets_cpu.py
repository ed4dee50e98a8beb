"""TF/SF sets (the blocked kernels' in-kernel form, models/tfsf.py
TfsfSets) against the per-cell correction tables of the stepped path: for a
random incident line, the summed correction every target cell receives from
its sets equals the sum of its table entries."""
import numpy as np
import pytest
import torch

from fdtd3d_amd.layout.yee import YeeLayout
from fdtd3d_amd.models.tfsf import build_tfsf_sets, build_tfsf_tables, incident_line_length
from fdtd3d_amd.ops.coef import Coef

COMPS = ("Ex", "Ey", "Ez", "Hx", "Hy", "Hz")


def _layout(size, tfsf, theta, phi, psi):
    import math
    return YeeLayout(size=size, scheme="3d", pml_size=(0, 0, 0), tfsf_size=tfsf, theta=math.radians(theta),
                     phi=math.radians(phi), psi=math.radians(psi))


@pytest.mark.parametrize("theta,phi,psi", [(90, 0, 90), (90, 0, 20), (90, 90, 30), (90, 90, 90), (90, 0, 0)])
@pytest.mark.parametrize("origin,shape", [((0, 0, 0), (30, 34, 40)), ((7, 3, 11), (12, 20, 16))])
def test_sets_equal_tables(theta, phi, psi, origin, shape):
    size = (30, 34, 40)
    lay = _layout(size, (5, 6, 7), theta, phi, psi)
    n = incident_line_length(size, "3d")
    boxes = {c: ((0, 0, 0), tuple(shape)) for c in COMPS}
    tabs = build_tfsf_tables(lay, COMPS, origin, shape, boxes, {c: Coef(1.0) for c in COMPS}, "cpu",
                             torch.float64, n)
    sets = build_tfsf_sets(lay, COMPS, origin, shape, boxes, "cpu", torch.float64, n)
    assert sets is not None
    rng = np.random.default_rng(3)
    line = {"E": rng.standard_normal(n), "H": rng.standard_normal(n)}
    i0, w0, w1, cc = (t.numpy() for t in (sets.i0, sets.w0, sets.w1, sets.c))
    for ci, c in enumerate(COMPS):
        inc = line["H"] if c[0] == "E" else line["E"]  # E targets read the H line
        want = np.zeros(shape)
        for t in tabs[c]:
            ijk = t.ijk.numpy()
            v = t.coef.numpy() * (t.w0.numpy() * inc[t.i0.numpy()] + t.w1.numpy() * inc[t.i0.numpy() + 1])
            np.add.at(want, (ijk[:, 0], ijk[:, 1], ijk[:, 2]), v)
        got = np.zeros(shape)
        for s in sets.sets:
            if s["n"] != ci:
                continue
            lo, hi, va = s["lo"], s["hi"], s["va"]
            k = np.arange(hi[va] - lo[va])
            e = s["goff"] + k
            g = cc[e] * (w0[e] * inc[i0[e]] + w1[e] * inc[i0[e] + 1])
            sl = tuple(slice(lo[d], hi[d]) for d in range(3))
            bshape = [1, 1, 1]
            bshape[va] = g.size
            got[sl] += g.reshape(bshape)
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-12)


def test_sets_reject_oblique():
    lay = _layout((30, 34, 40), (5, 6, 7), 60, 20, 10)
    n = incident_line_length((30, 34, 40), "3d")
    boxes = {c: ((0, 0, 0), (30, 34, 40)) for c in COMPS}
    assert build_tfsf_sets(lay, COMPS, (0, 0, 0), (30, 34, 40), boxes, "cpu", torch.float64, n) is None


def test_sets_struct_layout():
    lay = _layout((30, 34, 40), (5, 6, 7), 90, 0, 90)
    n = incident_line_length((30, 34, 40), "3d")
    boxes = {c: ((0, 0, 0), (30, 34, 40)) for c in COMPS}
    sets = build_tfsf_sets(lay, COMPS, (0, 0, 0), (30, 34, 40), boxes, "cpu", torch.float64, n)
    v = sets.struct_ints()
    # TfDev: nsets, ld, xpl[2][2], 24 x TfSet(10 ints) == fdtd_tfdev_size() / 4
    assert v.size == 6 + 24 * 10
    assert v[0] == len(sets.sets) and v[1] == sets.ld == sets.n_e + sets.n_h
    assert all(s["kind"] == "E" for s in sets.sets[:sum(1 for s in sets.sets if s["kind"] == "E")])
