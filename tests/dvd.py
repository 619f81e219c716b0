"""de Vahl Davis differentially heated cavity, restating the reference's
tests/validation/test_natural_convection.c (constants :50-61, velocity BCs
:76-88, kinetic energy :94-102, Nusselt number :112-129, driver :140-293)."""
from __future__ import annotations

import math

import numpy as np

from cfd_amd import _abi as A
from cfd_amd import api

L, T_HOT, T_COLD, T_REF = 1.0, 310.0, 290.0, 300.0
DT_TEMP = T_HOT - T_COLD
BETA, G, PR = 0.003333, 9.81, 0.71
STEADY_TOL, MIN_STEPS = 1e-6, 200
# (u_max*, v_max*, Nu) of de Vahl Davis 1983 and the reference's 10 % gate (:303-306)
REF_RA1E3 = (3.649, 3.697, 1.117)
GATE = 0.10


def setup(n: int, Ra: float, dt: float):
    nu_alpha = G * BETA * DT_TEMP * (L * L * L) / Ra
    alpha = math.sqrt(nu_alpha / PR)
    nu = PR * alpha
    g = api.Grid(n, n, 1, 0.0, L, 0.0, L, 0.0, 0.0)
    f = api.FlowField(n, n, 1)
    f.u[...] = 0.0
    f.v[...] = 0.0
    f.w[...] = 0.0
    f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[0] = (T_HOT - DT_TEMP * (np.asarray(g.x) / L))[None, :] * np.ones((n, 1))
    p = api.params_default()
    p.dt = dt
    p.mu = nu
    p.alpha = alpha
    p.beta = BETA
    p.T_ref = T_REF
    p.gravity[0] = 0.0
    p.gravity[1] = -G
    p.gravity[2] = 0.0
    p.max_iter = 1
    p.source_amplitude_u = 0.0
    p.source_amplitude_v = 0.0
    tb = p.thermal_bc
    tb.left = tb.right = A.BC_TYPE_DIRICHLET
    tb.top = tb.bottom = A.BC_TYPE_NEUMANN
    tb.dirichlet_values.left = T_HOT
    tb.dirichlet_values.right = T_COLD
    return g, f, p, alpha


def velocity_bcs(f):
    for a in (f.u[0], f.v[0]):
        a[:, 0] = 0.0
        a[:, -1] = 0.0
        a[0, :] = 0.0
        a[-1, :] = 0.0


def kinetic_energy(f) -> float:
    ke = 0.0
    for a, b in zip(f.u.ravel().tolist(), f.v.ravel().tolist()):
        ke += a * a + b * b
    return 0.5 * ke


def nusselt(f, dx: float) -> float:
    T = f.T[0]
    n = T.shape[0]
    dy = L / (n - 1)
    integral = 0.0
    for j in range(n):
        T0 = (T[j, 0] - T_COLD) * (1.0 / DT_TEMP)
        T1 = (T[j, 1] - T_COLD) * (1.0 / DT_TEMP)
        T2 = (T[j, 2] - T_COLD) * (1.0 / DT_TEMP)
        d = (-3.0 * T0 + 4.0 * T1 - T2) / (2.0 * dx)
        w = 0.5 if j in (0, n - 1) else 1.0
        integral += w * (-d * L)
    return integral * dy / L


def run(step, g, f, p, alpha, max_steps: int):
    """March to steady state; step(f) advances one step and returns a status."""
    prev = kinetic_energy(f)
    steps, converged = 0, False
    for s in range(max_steps):
        velocity_bcs(f)
        st = step(f)
        if st != A.CFD_SUCCESS:
            raise RuntimeError(f"step {s} failed: {st}")
        velocity_bcs(f)
        ke = kinetic_energy(f)
        res = abs(ke - prev) / (prev + 1e-10)
        prev = ke
        steps = s + 1
        if s > MIN_STEPS and res < STEADY_TOL:
            converged = True
            break
    n = g.nx
    scale = L / alpha
    umax = float(np.max(np.abs(f.u[0][:, n // 2]))) * scale
    vmax = float(np.max(np.abs(f.v[0][n // 2, :]))) * scale
    return {"steps": steps, "converged": converged, "umax": umax, "vmax": vmax,
            "nu": nusselt(f, L / (n - 1))}
