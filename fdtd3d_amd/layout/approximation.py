"""Numerical approximations: material averaging, Drude parameter averaging,
numerical-dispersion-corrected phase velocity and sub-cell sphere smoothing.

Behavioural re-implementation of the reference ``Approximation`` statics
(``Source/Layout/Approximation.cpp``), vectorised over torch tensors where they
are applied per cell.  Deliberate fixes:

* #6 -- ``phaseVelocityIncidentWave3D`` used ``=`` instead of ``==`` in its
  special-case tests, so every call took the axis-aligned shortcut and clobbered
  theta.  Here the special cases trigger only for theta == pi/2 and the listed
  phi values; otherwise the Newton iteration runs.
* #7 -- the 4-point Drude average used chained ``==`` comparisons and never set
  its gamma divider.  Here the rule is the one the 2-point branch encodes:
  plasma frequency averages as ``sqrt(mean(omega^2))`` over the points, collision
  frequency as the mean over the *dispersive* points (points with omega == gamma
  == 0 are vacuum).  It agrees with the reference wherever the reference is
  well defined (2-point, and 4-point with 0 or 3 vacuum points).
"""

from __future__ import annotations

import math
from typing import Sequence

import torch

from ..utils.constants import PI, SPEED_OF_LIGHT

NEWTON_ACCURACY = 1e-7  # Approximation.cpp:7


def approximate_material(vals: Sequence[torch.Tensor]) -> torch.Tensor:
    """Pairwise-hierarchical mean of 2, 4 or 8 values (Approximation.cpp:15-32)."""
    n = len(vals)
    if n == 1:
        return vals[0]
    if n == 2:
        return (vals[0] + vals[1]) / 2.0
    if n == 4:
        return (approximate_material(vals[0:2]) + approximate_material(vals[2:4])) / 2.0
    if n == 8:
        return (approximate_material(vals[0:4]) + approximate_material(vals[4:8])) / 2.0
    raise ValueError("material averaging needs 1, 2, 4 or 8 points")


def approximate_drude(omegas: Sequence[torch.Tensor], gammas: Sequence[torch.Tensor]):
    """Effective (omega_p, gamma) of a cell mixing Drude and vacuum points."""
    n = len(omegas)
    sq = sum(w * w for w in omegas) / float(n)
    omega = torch.sqrt(sq)
    disp = sum(((w != 0) | (g != 0)).to(omegas[0].dtype) for w, g in zip(omegas, gammas))
    gsum = sum(gammas)
    gamma = torch.where(disp > 0, gsum / torch.clamp(disp, min=1.0), torch.zeros_like(gsum))
    return omega, gamma


def phase_velocity_incident_wave_3d(delta: float, wavelength: float, courant: float, n_lambda: float,
                                    theta: float, phi: float) -> float:
    """Numerical phase velocity of a plane wave on the Yee grid
    (Taflove; reference Approximation.cpp:212-269)."""
    half = PI / 2
    if theta == half and phi in (0.0, half, PI, 3 * half):
        return SPEED_OF_LIGHT * PI / (n_lambda * math.asin(math.sin(PI * courant / n_lambda) / courant))
    if theta == half and phi in (PI / 4, 3 * PI / 4, 5 * PI / 4, 7 * PI / 4):
        s2 = math.sqrt(2.0)
        return SPEED_OF_LIGHT * PI / (n_lambda * s2 * math.asin(math.sin(PI * courant / n_lambda) / (courant * s2)))
    k = 2 * PI
    k_prev = k + NEWTON_ACCURACY
    nd = delta / wavelength
    A = nd * math.sin(theta) * math.cos(phi) / 2
    B = nd * math.sin(theta) * math.sin(phi) / 2
    C = nd * math.cos(theta) / 2
    D = (math.sin(PI * courant / n_lambda) ** 2) / (courant ** 2)
    it = 0
    while (k_prev - k) ** 2 >= NEWTON_ACCURACY and it < 1000:
        k_prev = k
        f = math.sin(A * k) ** 2 + math.sin(B * k) ** 2 + math.sin(C * k) ** 2 - D
        df = A * math.sin(2 * A * k) + B * math.sin(2 * B * k) + C * math.sin(2 * C * k)
        k -= f / df
        it += 1
    return SPEED_OF_LIGHT * 2 * PI / k


def phase_velocity_incident_wave_2d(delta, wavelength, courant, n_lambda, phi) -> float:
    return phase_velocity_incident_wave_3d(delta, wavelength, courant, n_lambda, PI / 2, phi)


def approximate_sphere(x: torch.Tensor, y: torch.Tensor, z: torch.Tensor, center: Sequence[float],
                       radius: float, eps_in: float, eps_out: float = 1.0) -> torch.Tensor:
    """Linear sub-cell smoothing of a sphere boundary over one cell
    (Approximation.cpp:286-314): inside by more than half a cell -> eps_in,
    outside by more than half a cell -> eps_out, linear in between."""
    d = torch.sqrt((x - center[0]) ** 2 + (y - center[1]) ** 2 + (z - center[2]) ** 2)
    diff = d - radius
    prop = 0.5 - diff
    mid = prop * eps_in + (1 - prop) * eps_out
    out = torch.where(diff < -0.5, torch.full_like(d, eps_in), mid)
    return torch.where(diff > 0.5, torch.full_like(d, eps_out), out)


def approximate_sphere_volumetric(x: torch.Tensor, y: torch.Tensor, z: torch.Tensor, center: Sequence[float],
                                  radius: float, eps_in: float, eps_out: float = 1.0, samples: int = 4):
    """Volume-fraction smoothing by sub-cell sampling (the reference's
    ``approximateSphere_1`` integrates a plane cut with 1000x1000 quadrature,
    Approximation.cpp:316-689; here ``samples^3`` points per cell give the
    fill fraction directly)."""
    frac = torch.zeros_like(x)
    offs = [(s + 0.5) / samples - 0.5 for s in range(samples)]
    r2 = radius * radius
    for ox in offs:
        for oy in offs:
            for oz in offs:
                inside = ((x + ox - center[0]) ** 2 + (y + oy - center[1]) ** 2 + (z + oz - center[2]) ** 2) < r2
                frac = frac + inside.to(x.dtype)
    frac = frac / float(samples ** 3)
    return frac * eps_in + (1 - frac) * eps_out
