"""Dump file naming (reference ``Source/File-Management/Commons.h:56-68``):

    current[<step>]_rank-<pid>_<name>
    previous[<step>]_rank-<pid>_<name>
    previous2[<step>]_rank-<pid>_<name>

followed by the format suffix (``.dat``, ``.txt``, ``-Re.bmp`` ...).
"""

import os
from enum import Enum


class GridFileType(Enum):
    CURRENT = 0
    PREVIOUS = 1
    PREVIOUS2 = 2
    ALL = 3


_PREFIX = {GridFileType.CURRENT: "current", GridFileType.PREVIOUS: "previous", GridFileType.PREVIOUS2: "previous2"}


def grid_file_name(step: int, level: GridFileType, rank: int, name: str, directory: str = ".") -> str:
    if level == GridFileType.ALL:
        raise ValueError("ALL is not a single file level")
    return os.path.join(directory, "%s[%d]_rank-%d_%s" % (_PREFIX[level], int(step), int(rank), name))


def levels(kind: GridFileType):
    """File levels written for a dump type."""
    if kind == GridFileType.ALL:
        return [GridFileType.CURRENT, GridFileType.PREVIOUS, GridFileType.PREVIOUS2]
    return [kind]
