"""Version of fdtd3d-amd.  ``REFERENCE_VERSION`` is the version of the reference
solver whose feature set and CLI we implement (reference
``Source/Settings/Settings.h:8``)."""

__version__ = "0.3.0"
REFERENCE_VERSION = "0.2.2"
SOLVER_VERSION = "%s (fdtd3d-amd, compatible with fdtd3d %s)" % (__version__, REFERENCE_VERSION)
