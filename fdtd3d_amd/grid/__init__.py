"""Time-levelled grid API (reference ``Source/Grid``)."""

from .grid import Grid, ParallelGrid  # noqa: F401
