"""Run-time configuration and command-line parsing.

Python mirror of the native parser in ``csrc/settings.cpp``.  Both read the same
option table, ``csrc/settings.inc``, so every flag accepted by the reference
(``Source/Settings/Settings.inc:28-125``) is accepted here with the same name,
argument kind and default.  Behaviour reproduced from the reference parser
(``Source/Settings/Settings.cpp:19-321``):

* ``--help`` / ``--version`` stop parsing (``EXIT_BREAK_ARG_PARSING``).
* ``--same-size*`` copy the x value to y and z *at the point they appear*.
  (Reference bug ``Settings.cpp:133-136`` -- ``--same-size-ntff`` clobbering the
  TF/SF sizes -- is fixed: it copies ntffSizeX.)
* ``--cmd-from-file FILE`` must be the only option; the file holds one token per
  line (whitespace separated tokens are accepted, as ``std::ifstream >>`` does).
  A file may not itself contain ``--cmd-from-file``.
* ``--save-cmd-to-file FILE`` writes every other token, one per line.
* Unknown options are an error (``EXIT_UNKNOWN_OPTION``).

Build-time switches of the reference (value type, complex values, grid
dimension, parallel buffer topology, CUDA) are ordinary run-time options here.
"""

from __future__ import annotations

import os
import re
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..version import SOLVER_VERSION

_INC_PATH = os.path.join(os.path.dirname(os.path.dirname(__file__)), "csrc", "settings.inc")

EXIT_OK = 0
EXIT_ERROR = 1
EXIT_UNKNOWN_OPTION = 2
EXIT_BREAK_ARG_PARSING = 3


@dataclass(frozen=True)
class OptionSpec:
    kind: str            # ACTION, ACTION_ARG, BOOL, INT, FLOAT, STRING
    cli: str
    help: str
    field: Optional[str] = None
    default: object = None

    @property
    def takes_arg(self) -> bool:
        return self.kind in ("ACTION_ARG", "INT", "FLOAT", "STRING")


_ROW_RE = re.compile(r'^\s*FDTD_(ACTION_ARG|ACTION|BOOL|INT|FLOAT|STRING)\s*\((.*)\)\s*$')
_TOKEN_RE = re.compile(r'"((?:[^"\\]|\\.)*)"|([^,\s][^,]*)')


def _split_args(body: str) -> List[str]:
    out = []
    for m in _TOKEN_RE.finditer(body):
        if m.group(1) is not None:
            out.append(m.group(1))
        else:
            out.append(m.group(2).strip())
    return out


def load_option_table(path: str = _INC_PATH) -> List[OptionSpec]:
    """Parse ``settings.inc`` into a list of :class:`OptionSpec`."""
    specs: List[OptionSpec] = []
    in_comment = False
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            s = line.strip()
            if in_comment:
                if "*/" in s:
                    in_comment = False
                continue
            if s.startswith("/*"):
                if "*/" not in s:
                    in_comment = True
                continue
            m = _ROW_RE.match(s)
            if not m:
                continue
            kind, args = m.group(1), _split_args(m.group(2))
            if kind in ("ACTION", "ACTION_ARG"):
                specs.append(OptionSpec(kind, args[0], args[1]))
            elif kind == "BOOL":
                specs.append(OptionSpec(kind, args[1], args[2], field=args[0], default=False))
            else:
                raw = args[2]
                if kind == "INT":
                    default = int(raw)
                elif kind == "FLOAT":
                    default = float(raw)
                else:
                    default = raw
                specs.append(OptionSpec(kind, args[1], args[3], field=args[0], default=default))
    return specs


OPTIONS: List[OptionSpec] = load_option_table()
OPTIONS_BY_CLI: Dict[str, OptionSpec] = {o.cli: o for o in OPTIONS}


class SettingsError(Exception):
    def __init__(self, msg: str, code: int = EXIT_ERROR):
        super().__init__(msg)
        self.code = code


class Settings:
    """All run-time options.  Attribute names equal the reference's field names
    (``sizeX``, ``doUsePML``, ...) and snake-case getters are provided through
    :meth:`get`.  ``dimension`` defaults to 3 (the reference default is 2 only
    because its build selects the dimension)."""

    def __init__(self) -> None:
        for o in OPTIONS:
            if o.field is not None:
                setattr(self, o.field, o.default)
        self.dimension = 3
        self.cmd_history: List[str] = []

    # -- reference-style getters (getSizeX, getDoUsePML, ...) --
    def __getattr__(self, name: str):
        if name.startswith("get") and len(name) > 3:
            fld = name[3].lower() + name[4:]
            alias = _GETTER_ALIASES.get(name)
            if alias:
                fld = alias
            d = self.__dict__
            if fld in d:
                return lambda: d[fld]
            # getDoUsePML -> doUsePML ; getPMLSizeX -> pmlSizeX
            for k in d:
                if k.lower() == fld.lower():
                    return lambda k=k: d[k]
        raise AttributeError(name)

    def as_dict(self) -> Dict[str, object]:
        out = {o.field: getattr(self, o.field) for o in OPTIONS if o.field}
        out["dimension"] = self.dimension
        return out

    # ---------------------------------------------------------------- parsing
    def parse_arg(self, argv: Sequence[str], index: int, is_cmd: bool, out=sys.stdout) -> Tuple[int, int]:
        """Parse the token at ``index``.  Returns ``(status, new_index)``."""
        a = argv[index]
        if a == "--help":
            out.write(help_text())
            return EXIT_BREAK_ARG_PARSING, index
        if a == "--version":
            out.write("Version: %s\n" % SOLVER_VERSION)
            return EXIT_BREAK_ARG_PARSING, index
        spec = OPTIONS_BY_CLI.get(a)
        if spec is None:
            out.write("Unknown option [%s]\n" % a)
            return EXIT_UNKNOWN_OPTION, index
        val = None
        if spec.takes_arg:
            index += 1
            if index >= len(argv):
                raise SettingsError("option %s needs an argument" % a)
            val = argv[index]
        if spec.kind == "BOOL":
            setattr(self, spec.field, True)
        elif spec.kind == "INT":
            try:
                setattr(self, spec.field, int(val))
            except ValueError:
                raise SettingsError("option %s expects an integer, got %r" % (a, val))
        elif spec.kind == "FLOAT":
            try:
                setattr(self, spec.field, float(val))
            except ValueError:
                raise SettingsError("option %s expects a number, got %r" % (a, val))
        elif spec.kind == "STRING":
            setattr(self, spec.field, val)
        elif a == "--same-size":
            self.sizeY = self.sizeZ = self.sizeX
        elif a == "--same-size-pml":
            self.pmlSizeY = self.pmlSizeZ = self.pmlSizeX
        elif a == "--same-size-tfsf":
            self.tfsfSizeY = self.tfsfSizeZ = self.tfsfSizeX
        elif a == "--same-size-ntff":
            self.ntffSizeY = self.ntffSizeZ = self.ntffSizeX
        elif a == "--same-size-topology":
            self.topologySizeY = self.topologySizeZ = self.topologySizeX
        elif a == "--1d":
            self.dimension = 1
        elif a == "--2d":
            self.dimension = 2
        elif a == "--3d":
            self.dimension = 3
        elif a == "--cmd-from-file":
            if not is_cmd:
                out.write("Command line files are not allowed in other command line files.\n")
                return EXIT_ERROR, index
            if len(argv) != 2:
                out.write("Command line files are allowed only without other options.\n")
                return EXIT_ERROR, index
            status = self.load_cmd_from_file(val, out=out)
            if status == EXIT_ERROR:
                out.write("ERROR: Incorrect command line file.\n")
            return status, index
        elif a == "--save-cmd-to-file":
            save_cmd_to_file(argv, val, out=out)
        return EXIT_OK, index

    def set_from_cmd(self, argv: Sequence[str], is_cmd: bool = True, out=sys.stdout) -> int:
        """Parse ``argv`` (without the program name)."""
        argv = list(argv)
        self.cmd_history.extend(argv)
        i = 0
        while i < len(argv):
            status, i = self.parse_arg(argv, i, is_cmd, out=out)
            if status != EXIT_OK:
                return status
            i += 1
        return EXIT_OK

    def load_cmd_from_file(self, path: str, out=sys.stdout) -> int:
        out.write("Loading command line from file %s\n" % path)
        try:
            with open(path, "r", encoding="utf-8") as f:
                tokens = f.read().split()
        except OSError:
            return EXIT_ERROR
        return self.set_from_cmd(tokens, is_cmd=False, out=out)

    def validate(self) -> None:
        """Sanity checks the reference performs with ASSERTs."""
        if self.valueType not in ("f32", "f64"):
            raise SettingsError("--dtype must be f32 or f64")
        if self.mode2D not in ("tmz", "tez"):
            raise SettingsError("--2d-mode must be tmz or tez")
        if self.parallelBufferDimension not in ("x", "y", "z", "xy", "yz", "xz", "xyz"):
            raise SettingsError("--topology must be one of x y z xy yz xz xyz")
        if self.pmlType not in ("upml", "cpml"):
            raise SettingsError("--pml-type must be upml or cpml")
        if self.backend not in ("auto", "hip", "torch"):
            raise SettingsError("--backend must be auto, hip or torch")
        if not (0.0 <= self.incidentWaveAngle1 <= 90.0 and 0.0 <= self.incidentWaveAngle2 <= 90.0):
            # reference YeeGridLayout.h:446-447 asserts theta, phi in [0, pi/2]
            raise SettingsError("--angle-teta and --angle-phi must be within [0, 90] degrees")
        if self.scene not in ("reference", "vacuum", "sphere", "drude-sphere"):
            raise SettingsError("--scene must be reference, vacuum, sphere or drude-sphere")
        if self.dispersion not in ("drude", "lorentz"):
            raise SettingsError("--dispersion must be drude or lorentz")
        if self.sourceType not in ("sine", "gaussian"):
            raise SettingsError("--source must be sine or gaussian")
        if self.bufferSize < 1:
            raise SettingsError("--buffer-size must be >= 1")
        for n in ("sizeX", "sizeY", "sizeZ"):
            if getattr(self, n) < 1:
                raise SettingsError("--%s must be positive" % n.lower())


_GETTER_ALIASES = {
    "getPMLSizeX": "pmlSizeX", "getPMLSizeY": "pmlSizeY", "getPMLSizeZ": "pmlSizeZ",
    "getTFSFSizeX": "tfsfSizeX", "getTFSFSizeY": "tfsfSizeY", "getTFSFSizeZ": "tfsfSizeZ",
    "getNTFFSizeX": "ntffSizeX", "getNTFFSizeY": "ntffSizeY", "getNTFFSizeZ": "ntffSizeZ",
    "getNumAmplitudeSteps": "numAmplitudeTimeSteps",
    "getIncidentWaveAngle1": "incidentWaveAngle1",
    "getIncidentWaveAngle2": "incidentWaveAngle2",
    "getIncidentWaveAngle3": "incidentWaveAngle3",
    "getDimension": "dimension",
}


def save_cmd_to_file(argv: Sequence[str], path: str, out=sys.stdout) -> int:
    out.write("Saving command line to file %s\n" % path)
    toks = []
    i = 0
    argv = list(argv)
    while i < len(argv):
        if argv[i] == "--save-cmd-to-file":
            i += 2
            continue
        toks.append(argv[i])
        i += 1
    with open(path, "w", encoding="utf-8") as f:
        for t in toks:
            f.write(t + "\n")
    return EXIT_OK


def help_text() -> str:
    lines = [
        "fdtd3d-amd: 1D, 2D and 3D FDTD electromagnetics solver for AMD Instinct MI355X "
        "(HIP kernels, RCCL domain decomposition).\n",
        "Usage: fdtd3d [options]\n\n",
        "Options:\n",
    ]
    for o in OPTIONS:
        if o.kind in ("ACTION", "BOOL"):
            lines.append("  %s\n\t%s\n" % (o.cli, o.help))
        elif o.kind == "ACTION_ARG":
            lines.append("  %s <string>\n\t%s\n" % (o.cli, o.help))
        elif o.kind == "INT":
            lines.append("  %s <int> (default: %d)\n\t%s\n" % (o.cli, o.default, o.help))
        elif o.kind == "FLOAT":
            lines.append("  %s <float> (default: %f)\n\t%s\n" % (o.cli, o.default, o.help))
        else:
            lines.append("  %s <string> (default: %s)\n\t%s\n" % (o.cli, o.default, o.help))
    lines.append("  --help\n\tPrint this help\n  --version\n\tPrint the version\n")
    return "".join(lines)


def setup_from_cmd(argv: Sequence[str], out=sys.stdout) -> Tuple[int, Settings]:
    """Equivalent of ``Settings::SetupFromCmd`` that returns instead of exiting."""
    s = Settings()
    try:
        status = s.set_from_cmd(argv, is_cmd=True, out=out)
    except SettingsError as e:
        out.write("ERROR: %s\n" % e)
        return e.code, s
    if status == EXIT_OK:
        try:
            s.validate()
        except SettingsError as e:
            out.write("ERROR: %s\n" % e)
            return e.code, s
    return status, s
