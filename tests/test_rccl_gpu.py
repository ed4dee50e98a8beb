"""The multi-GPU exchange through REAL RCCL on one MI355X (GPU only).

RCCL refuses two ranks on one device, and the round's GPU box has one GPU,
so the decomposed GPU tests (``test_parallel_gpu.py``) run their ranks as
threads over an in-process transport.  This test closes the gap between
those and an 8-GPU node: a fresh child process initialises a 1-rank ``nccl``
(= RCCL) group with the solver's ``nccl_init_kwargs`` and posts the exact op
list of one direct 26-neighbour deep exchange with every peer mapped to
self (``tests/rccl_self_child.py``).  RCCL matches point-to-point operations
per peer in posting order (tags are ignored), which the gloo tests cannot
see: the check pins that every send of the op list pairs with the receive of
the same size, that x-face slices go straight from / into the arrays, that
the packed edge / corner buffers unpack into the right ghost boxes, and that
the main stream reads them only after ``_join_side`` (negative control: an
unordered read sees stale ghosts).

Reference: ``Source/Grid/ParallelGrid.cpp:1535-1594`` (``SendReceiveRawBuffer``).
"""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_self_exchange():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_self_child.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RCCL_SELF ")]
    assert r.returncode == 0 and line, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    out = json.loads(line[-1][len("RCCL_SELF "):])
    assert out["backend"] == "nccl"
    for case in ("direct", "packed"):
        res = out[case]
        assert res["n_msgs"] == 26, res
        assert res["max_err"] == 0.0, (case, res)            # every ghost box: bit-exact
        assert res["owned_untouched"], (case, res)
        assert res["stale_err"] > 0.0, (case, res)           # the unordered read saw old ghosts
    # x faces straight from the arrays: 6 messages per x face instead of one packed buffer
    assert out["direct"]["messages"] == 24 + 2 * 6, out["direct"]
    assert out["packed"]["messages"] == 26, out["packed"]
