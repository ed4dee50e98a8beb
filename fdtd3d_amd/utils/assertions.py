"""Diagnostics: assertions with context and a fatal-error path.

The reference prints a backtrace and exits on any failed ``ASSERT``
(``Source/Helpers/Assert.h:25-91``, ``Assert.cpp:5-30``).  Here a failed check
raises :class:`FdtdError`, which the CLI driver turns into a non-zero exit code
after printing the Python traceback, so library users can catch it.
"""

import traceback


class FdtdError(RuntimeError):
    pass


def fdtd_assert(cond, msg="assertion failed"):
    if not cond:
        raise FdtdError(msg)


def unreachable(msg="unreachable code reached"):
    raise FdtdError(msg)


def format_exception(e: BaseException) -> str:
    return "".join(traceback.format_exception(type(e), e, e.__traceback__))
