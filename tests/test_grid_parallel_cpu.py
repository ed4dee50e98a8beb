"""The reference's only unit test, re-done on the new grid API
(``Tests/unit-test-parallel-grid.cpp``): every rank fills its chunk with its
rank id (levels rank, 16 rank, 256 rank), shares, gathers the full grid and
checks that every global cell carries its owner's id on every level.

Added on top (the reference never checks halo *contents*): after ``share()``
every ghost cell equals the owning neighbour's interior value, and a NaN
poisoning of all ghosts before the exchange leaves no NaN behind (a missed
direction -- edge or corner with deep halos -- would)."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fdtd3d_amd.grid import Grid, ParallelGrid
from fdtd3d_amd.ops import make_ops
from fdtd3d_amd.parallel.domain import Domain
from fdtd3d_amd.parallel.halo import HaloExchanger
from fdtd3d_amd.parallel.topology import ParallelGridCore

SIZE = (32, 32, 32)  # the reference asserts 32 % P == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, axes, buf, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        core = ParallelGridCore.create(SIZE, world, axes)
        dom = core.domain(rank, buf)
        g = ParallelGrid(dom, HaloExchanger(dom), make_ops("torch", None, "cpu", torch.float64), "Ez", 3)
        for lv, mul in enumerate((1.0, 16.0, 256.0)):
            g.levels[lv].fill_(float("nan"))          # poison every ghost
            g.owned(lv).fill_(rank * mul)
        g.share()
        bad = []
        for lv, mul in enumerate((1.0, 16.0, 256.0)):
            t = g.levels[lv]
            if bool(torch.isnan(t).any()):
                bad.append("nan left in level %d" % lv)
            # every allocated cell holds the owner's id (ghosts included)
            o = dom.origin
            for idx in [(0, 0, 0), tuple(s - 1 for s in dom.shape), tuple(s // 2 for s in dom.shape)]:
                gidx = tuple(idx[d] + o[d] for d in range(3))
                owner = next(r for r in range(core.used_procs) if core.domain(r, buf).owns(gidx))
                if float(t[idx]) != owner * mul:
                    bad.append("level %d cell %s: %s != owner %d" % (lv, gidx, float(t[idx]), owner))
            full = g.gather_full_grid(lv)
            for r in range(core.used_procs):
                dr = core.domain(r, buf)
                blk = full[dr.lo[0]:dr.hi[0], dr.lo[1]:dr.hi[1], dr.lo[2]:dr.hi[2]]
                if not bool((blk == r * mul).all()):
                    bad.append("gathered block of rank %d wrong on level %d" % (r, lv))
        torch.save({"bad": bad}, os.path.join(outdir, "r%d.pt" % rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,axes,buf", [(2, "x", 1), (4, "xy", 2), (4, "yz", 1), (8, "xyz", 2),
                                            (8, "xyz", 3)])
def test_parallel_grid_share_and_gather(world, axes, buf):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), axes, buf, d), nprocs=world, join=True)
        for r in range(world):
            res = torch.load(os.path.join(d, "r%d.pt" % r), weights_only=True)
            assert res["bad"] == [], (r, res["bad"][:5])


def test_grid_levels_and_ranges(tmp_path):
    dom = Domain.serial((6, 5, 4))
    g = Grid(dom, "Ex", 3)
    g.current.fill_(1.0)
    g.next_time_step()
    g.current.fill_(2.0)
    g.next_time_step()
    g.current.fill_(3.0)
    assert float(g.previous2[0, 0, 0]) == 1.0 and float(g.previous[0, 0, 0]) == 2.0
    assert g.computation_start((1, 1, 0)) == (1, 1, 0)
    assert g.computation_end((1, 0, 1)) == (5, 5, 3)
    assert g.total_position((2, 3, 1)) == (2, 3, 1)
    files = g.save(str(tmp_path))
    assert [os.path.basename(f) for f in files] == ["current[2]_rank-0_Ex.dat", "previous[2]_rank-0_Ex.dat",
                                                     "previous2[2]_rank-0_Ex.dat"]
    assert os.path.getsize(files[0]) == 6 * 5 * 4 * 8
