"""Integer and floating-point grid coordinates in 1, 2 and 3 dimensions.

Semantics follow the reference coordinate classes
(``Source/Coordinate/GridCoordinate{1D,2D,3D}.h``):

* arithmetic is component-wise; scalar ``*`` scales every component;
* ordering comparisons are **all-components** (``a > b`` iff every component of
  ``a`` is greater), exactly as ``GridCoordinate3D.h:120-160``;
* ``!=`` is the proper negation of ``==`` (reference bug
  ``GridCoordinate3D.h:111`` -- comparing z with ``==`` -- is fixed);
* ``convert_coord`` FP->int asserts that every component is integral
  (``GridCoordinate.cpp:4-12``); ``shrink_coord`` drops the last axis.

Unlike the reference's template chain, one class handles every dimension; the
integer/FP flavour is a flag so the Yee layout code can mirror the reference's
exact-integer checks.
"""

from __future__ import annotations

from typing import Iterable, Sequence, Tuple

from .assertions import fdtd_assert


class GridCoordinate:
    __slots__ = ("c", "fp")

    def __init__(self, *comps, fp: bool = False):
        if len(comps) == 1 and isinstance(comps[0], (tuple, list)):
            comps = tuple(comps[0])
        fdtd_assert(1 <= len(comps) <= 3, "coordinates have 1..3 components")
        self.fp = fp
        self.c: Tuple = tuple(float(v) for v in comps) if fp else tuple(int(v) for v in comps)

    # -- construction helpers --
    @classmethod
    def same(cls, value, dim: int, fp: bool = False) -> "GridCoordinate":
        return cls(*([value] * dim), fp=fp)

    @property
    def dim(self) -> int:
        return len(self.c)

    def get_x(self):
        return self.c[0]

    def get_y(self):
        fdtd_assert(self.dim >= 2, "no y component")
        return self.c[1]

    def get_z(self):
        fdtd_assert(self.dim >= 3, "no z component")
        return self.c[2]

    x = property(get_x)
    y = property(get_y)
    z = property(get_z)

    def calculate_total_coord(self) -> int:
        t = 1
        for v in self.c:
            t *= v
        return t

    def get_max(self):
        return max(self.c)

    def as_tuple(self) -> Tuple:
        return self.c

    # -- arithmetic --
    def _other(self, rhs) -> Sequence:
        if isinstance(rhs, GridCoordinate):
            fdtd_assert(rhs.dim == self.dim, "dimension mismatch")
            return rhs.c
        return (rhs,) * self.dim

    def _mk(self, vals: Iterable, fp=None) -> "GridCoordinate":
        return GridCoordinate(*vals, fp=self.fp if fp is None else fp)

    def __add__(self, rhs):
        o = self._other(rhs)
        fp = self.fp or (isinstance(rhs, GridCoordinate) and rhs.fp)
        return self._mk((a + b for a, b in zip(self.c, o)), fp)

    def __sub__(self, rhs):
        o = self._other(rhs)
        fp = self.fp or (isinstance(rhs, GridCoordinate) and rhs.fp)
        return self._mk((a - b for a, b in zip(self.c, o)), fp)

    def __neg__(self):
        return self._mk(-a for a in self.c)

    def __mul__(self, s):
        fp = self.fp or isinstance(s, float)
        return self._mk((a * s for a in self.c), fp)

    __rmul__ = __mul__

    # -- comparisons (all components) --
    def __eq__(self, rhs) -> bool:
        return isinstance(rhs, GridCoordinate) and self.c == rhs.c

    def __ne__(self, rhs) -> bool:
        return not self.__eq__(rhs)

    def __hash__(self):
        return hash(self.c)

    def __gt__(self, rhs) -> bool:
        return all(a > b for a, b in zip(self.c, self._other(rhs)))

    def __lt__(self, rhs) -> bool:
        return all(a < b for a, b in zip(self.c, self._other(rhs)))

    def __ge__(self, rhs) -> bool:
        return all(a >= b for a, b in zip(self.c, self._other(rhs)))

    def __le__(self, rhs) -> bool:
        return all(a <= b for a, b in zip(self.c, self._other(rhs)))

    def __repr__(self):
        return "GridCoordinate%s%dD%s" % ("FP" if self.fp else "", self.dim, self.c)


def GridCoordinate1D(x):
    return GridCoordinate(x)


def GridCoordinate2D(x, y):
    return GridCoordinate(x, y)


def GridCoordinate3D(x, y, z):
    return GridCoordinate(x, y, z)


def GridCoordinateFP1D(x):
    return GridCoordinate(x, fp=True)


def GridCoordinateFP2D(x, y):
    return GridCoordinate(x, y, fp=True)


def GridCoordinateFP3D(x, y, z):
    return GridCoordinate(x, y, z, fp=True)


def convert_coord(c: GridCoordinate) -> GridCoordinate:
    """FP -> integer (asserting exact integrality) or integer -> FP."""
    if c.fp:
        for v in c.c:
            fdtd_assert(float(int(v)) == v, "non-integral coordinate %r" % (c,))
        return GridCoordinate(*(int(v) for v in c.c))
    return GridCoordinate(*c.c, fp=True)


def shrink_coord(c: GridCoordinate) -> GridCoordinate:
    fdtd_assert(c.dim >= 2, "cannot shrink a 1D coordinate")
    return GridCoordinate(*c.c[:-1], fp=c.fp)
