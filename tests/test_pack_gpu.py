"""Halo pack / unpack kernels (aux_kernels.hip box_pack / box_unpack): the
16-byte vector path (aligned rows) and the element-wise fallback (unaligned
z start, odd z span, unaligned buffer) against torch slicing, fp32 and fp64."""
import pytest
import torch

from fdtd3d_amd.ops import make_ops

pytestmark = pytest.mark.gpu

SHAPE = (8, 10, 32)
BOXES = [
    ((1, 2, 0), (5, 9, 32)),     # whole aligned rows
    ((0, 0, 4), (6, 7, 28)),     # aligned start and span
    ((2, 1, 1), (7, 8, 30)),     # z start offset by one element
    ((0, 0, 0), (3, 4, 31)),     # odd z span
    ((3, 3, 5), (4, 4, 6)),      # one cell
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("box", BOXES)
@pytest.mark.parametrize("buf_off", [0, 1])
def test_pack_unpack_vs_torch(gpu, dtype, box, buf_off):
    ops = make_ops("hip", None, gpu, dtype)
    g = torch.Generator(device="cpu").manual_seed(7)
    ts = [torch.randn(SHAPE, generator=g, dtype=torch.float64).to(gpu, dtype) for _ in range(3)]
    sl = tuple(slice(box[0][d], box[1][d]) for d in range(3))
    n = 1
    for d in range(3):
        n *= box[1][d] - box[0][d]
    big = torch.full((3 * n + buf_off + 4,), float("nan"), dtype=dtype, device=gpu)
    out = big[buf_off:buf_off + 3 * n]
    ops.pack(ts, box, out)
    want = torch.cat([t[sl].reshape(-1) for t in ts])
    assert torch.equal(out, want)
    assert torch.isnan(big[:buf_off]).all() and torch.isnan(big[buf_off + 3 * n:]).all()  # nothing outside
    dst = [torch.zeros(SHAPE, dtype=dtype, device=gpu) for _ in range(3)]
    ops.unpack(dst, box, out)
    torch.cuda.synchronize()
    for t, d in zip(ts, dst):
        assert torch.equal(d[sl], t[sl])
        m = torch.ones(SHAPE, dtype=torch.bool, device=gpu)
        m[sl] = False
        assert float(d[m].abs().max()) == 0.0 if m.any() else True


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("box", [((1, 2, 0), (9, 11, 24)),      # aligned z: vector path
                                 ((0, 3, 5), (7, 12, 18)),      # unaligned both ends: masked vectors
                                 ((2, 0, 3), (5, 13, 4)),       # one cell in z
                                 ((0, 0, 1), (10, 13, 23))])
def test_copy_box_vs_torch(gpu, dtype, box):
    """ops.copy_box (k_box_xfer / k_box_xfer_m): only the box changes, every
    component pair."""
    ops = make_ops("hip", None, gpu, dtype)
    shape = (10, 13, 24)
    g = torch.Generator().manual_seed(3)
    src = [torch.rand(shape, generator=g, dtype=torch.float64).to(dtype).to(gpu) for _ in range(6)]
    dst = [torch.rand(shape, generator=g, dtype=torch.float64).to(dtype).to(gpu) for _ in range(6)]
    want = [d.clone() for d in dst]
    sl = tuple(slice(box[0][d], box[1][d]) for d in range(3))
    for a, b in zip(src, want):
        b[sl] = a[sl]
    ops.copy_box(src, dst, box)
    torch.cuda.synchronize()
    for a, b in zip(dst, want):
        assert torch.equal(a, b)
