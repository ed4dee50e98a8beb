"""Per-phase timers of the time loop (``--profile-phases``).

The reference only wall-clocks ``performSteps`` (``Source/main.cpp:153-158``).
Here every phase of a step (E / H updates, sources, TF/SF incident line, halo
exchange, blocked passes ...) can be bracketed with a pair of HIP events on the
current stream -- no host synchronisation inside the loop; the events are
resolved once in :meth:`PhaseProfiler.summary`.  On the CPU backend phases are
host wall-clock intervals.  Disabled, ``phase()`` costs one attribute test.
"""

from __future__ import annotations

import time
from collections import OrderedDict
from contextlib import contextmanager
from typing import Dict

import torch


class PhaseProfiler:
    def __init__(self, device, enabled: bool = False):
        self.enabled = bool(enabled)
        self.cuda = torch.device(device).type == "cuda"
        self._events: "OrderedDict[str, list]" = OrderedDict()
        self._cpu: "OrderedDict[str, list]" = OrderedDict()

    def reset(self) -> None:
        self._events.clear()
        self._cpu.clear()

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._events.setdefault(name, []).append((s, e))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._cpu.setdefault(name, []).append(time.perf_counter() - t0)

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{phase: {"calls": n, "total_ms": t, "mean_ms": t/n}} (GPU time of the
        bracketed stream work, or host time on the CPU backend)."""
        out: Dict[str, Dict[str, float]] = OrderedDict()
        if self.cuda and self._events:
            torch.cuda.synchronize()
        for name, evs in self._events.items():
            tot = sum(s.elapsed_time(e) for s, e in evs)
            out[name] = {"calls": len(evs), "total_ms": tot, "mean_ms": tot / len(evs)}
        for name, ts in self._cpu.items():
            tot = sum(ts) * 1e3
            out[name] = {"calls": len(ts), "total_ms": tot, "mean_ms": tot / len(ts)}
        return out

    def report(self) -> str:
        s = self.summary()
        if not s:
            return ""
        total = sum(v["total_ms"] for v in s.values()) or 1.0
        lines = ["Phase timings (%s):" % ("GPU events" if self.cuda else "host clock")]
        for k, v in s.items():
            lines.append("  %-14s %7d calls %11.3f ms  %8.4f ms/call  %5.1f%%" % (
                k, v["calls"], v["total_ms"], v["mean_ms"], 100.0 * v["total_ms"] / total))
        return "\n".join(lines)
