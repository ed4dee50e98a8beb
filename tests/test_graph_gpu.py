"""HIP graph mode (--use-hip-graph): captured-and-replayed steps must equal
eagerly launched ones bit for bit (sources from the device table, UPML / Drude
level rotations restored after every replay)."""
import dataclasses

import pytest
import torch

from fdtd3d_amd.models.scheme import GRAPH_STEPS, SchemeConfig, YeeScheme
from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu

CASES = {
    "1d": SchemeConfig(scheme="1d", size=(3000, 1, 1), scene="vacuum", source="gaussian", dtype="f64"),
    "tmz-pml": SchemeConfig(scheme="tmz", size=(120, 100, 1), scene="vacuum", use_pml=True, pml_size=(8, 8, 1),
                            dtype="f32"),
    "3d-split": SchemeConfig(scheme="3d", size=(40, 36, 44), scene="vacuum", dtype="f32"),
    "3d-upml-tfsf-drude": SchemeConfig(scheme="3d", size=(48, 48, 40), use_pml=True, use_tfsf=True,
                                       use_metamaterials=True, pml_size=(5, 5, 5), tfsf_size=(9, 9, 9),
                                       scene="drude-sphere", sphere_radius=6, sphere_center=(24.0, 24.0, 20.0),
                                       dtype="f32"),
    "3d-cpml-complex": SchemeConfig(scheme="3d", size=(36, 36, 36), use_pml=True, pml_type="cpml",
                                    pml_size=(6, 6, 6), scene="vacuum", complex_values=True, dtype="f32"),
}


@pytest.mark.parametrize("name", list(CASES))
def test_graph_replay_equals_eager(gpu, name):
    steps = 2 * GRAPH_STEPS + 7
    res = []
    for graph in (False, True):
        cfg = dataclasses.replace(CASES[name], use_hip_graph=graph, time_steps=steps)
        dt = torch.float32 if cfg.dtype == "f32" else torch.float64
        s = YeeScheme(cfg, make_ops("hip", None, gpu, dt))
        s.init_scheme()
        s.init_grids()
        assert s.graph_mode == graph
        s.perform_steps()
        torch.cuda.synchronize()
        assert s.t == steps
        res.append({(p, c): s.F[p][c].cpu() for p in range(s.planes) for c in s.comps})
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k
