"""Rank-prefixed levelled logging honouring ``--log-level``.

The reference parses ``--log-level`` but never reads it;
here level 0 prints only results, 1 adds progress, 2 adds per-phase timings and
3 adds debug detail.
"""

import os
import sys
import time

_LEVEL = 0
_RANK = int(os.environ.get("RANK", "0"))


def set_level(level: int) -> None:
    global _LEVEL
    _LEVEL = int(level)


def get_level() -> int:
    return _LEVEL


def set_rank(rank: int) -> None:
    global _RANK
    _RANK = int(rank)


def log(level: int, msg: str, all_ranks: bool = False) -> None:
    if level > _LEVEL:
        return
    if not all_ranks and _RANK != 0:
        return
    sys.stdout.write("[%s r%d] %s\n" % (time.strftime("%H:%M:%S"), _RANK, msg))
    sys.stdout.flush()


def info(msg, all_ranks=False):
    log(1, msg, all_ranks)


def debug(msg, all_ranks=False):
    log(3, msg, all_ranks)
