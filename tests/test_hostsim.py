"""The device interpreter on the CPU (tests/hostsim: pdeval_kernels.h + pdeval_tier2.h built
by g++ for one lane) against the oracle: jets, residual, scale and the tier-2 noise bound.
This checks the device source's arithmetic without a GPU (the GPU parity tests check the
gfx950 build itself)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from pdeval import problem_defs as P

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, 'hostsim', '_build', 'libsim.so')
SRC = [os.path.join(ROOT, 'pde-engine_amd', 'csrc', f) for f in
       ('pdeval_kernels.h', 'pdeval_tier2.h', 'pdeval_point.h', 'jet.h', 'dd.h')] + \
      [os.path.join(HERE, 'hostsim', 'sim.cpp')]


@pytest.fixture(scope='module')
def sim():
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in SRC):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-DPD_HOST_SIM',
                               '-I' + os.path.join(HERE, 'hostsim'), '-o', SO,
                               os.path.join(HERE, 'hostsim', 'sim.cpp')])
    lib = C.CDLL(SO)
    vp = C.c_void_p
    lib.sim_point.argtypes = [C.c_int, vp, C.c_int, C.c_double, C.c_double, C.c_int, vp, vp, vp]
    lib.sim_set_omega2.argtypes = [C.c_double]
    lib.sim_point_tier.argtypes = [C.c_int, vp, C.c_int, C.c_int, C.c_int, vp]
    return lib


EXPRS = ['rho**2 + z**2', 'z*neg(rho/z + 1)', 'exp(z/(-rho**2 + z**2))',
         'exp_neg(square(rho/(-rho/z + 1)))', 'rho**2/(rho**2 + z**2)**(3/2)',
         'sqrt(z**2 + (rho - 1)**2) - sqrt(z**2 + (rho + 1)**2)', 'rho**3*z**2 - z**5/rho**2',
         'log(rho + z**2)*z', 'rho/Abs(z)', '1/(1 - 1/(-rho**2 + z**2 + 1))', 'z**4/(rho**3 + 2)']


@pytest.mark.parametrize('omega2', [0.0, 1.0, 0.25])
@pytest.mark.parametrize('s', EXPRS)
def test_device_source_matches_oracle(sim, s, omega2):
    """The device epilogue (jets; with Omega != 0 the rotation corrections ff_rotate_A / _B)
    against the oracle's closed-form partials, at Omega = 0 (the problem path) and for rotating
    field lines (validator.py:326-329)."""
    sim.sim_set_omega2(omega2)
    O.set_omega2(omega2)
    try:
        _device_source_matches_oracle(sim, s)
    finally:
        sim.sim_set_omega2(0.0)
        O.set_omega2(0.0)


def _device_source_matches_oracle(sim, s):
    pd_ = P.force_free()
    w = np.array(pd_.compile(pd_.parse(s)), dtype=np.int32)
    for pt in ((1.3, -0.55), (2.2, 1.1), (0.8, 6 / 7), (0.37, 1.9)):
        jet, err, res = np.zeros(15), np.zeros(15), np.zeros(4)
        rc = sim.sim_point(0, w.ctypes.data, len(w), pt[0], pt[1], 1, jet.ctypes.data,
                           err.ctypes.data, res.ctypes.data)
        assert rc == 0
        o = O.point(0, w, *pt)
        oj = O.jet(0, w, *pt)
        if not (o[3] and res[3]):
            assert not o[3] and not res[3]
            continue
        assert np.allclose(jet, oj, rtol=1e-12, atol=1e-12 * np.abs(oj).max()), (s, pt)
        assert abs(res[1] - o[1]) <= 1e-9 * o[1] + 1e-300
        # residuals agree to the noise bound, and the noise bounds to a factor 4
        assert abs(res[0] - o[0]) <= 4 * max(o[2], res[2]) + 1e-12 * o[1], (s, pt, res, o)
        assert res[2] <= 4 * o[2] + 1e-300 and o[2] <= 4 * res[2] + 1e-300, (s, pt, res[2], o[2])


def test_kerr_lean_epilogue_equals_kerr_epilogue(sim):
    """The lean grid passes' Kerr epilogue (doubled coefficient table, one maximum for the
    coefficient tests) gives the PointResult of kerr_epilogue bit for bit, on random jets and on
    every special value in every coefficient (NaN, +-inf, the 2^160 bound, zeros, subnormals)."""
    sim.sim_kerr_epi_pair.argtypes = [C.c_void_p] * 3
    rng = np.random.default_rng(7)
    specials = [np.nan, np.inf, -np.inf, 0.0, -0.0, 2.0 ** 160, -(2.0 ** 160), np.nextafter(2.0 ** 160, 0),
                5e-324, 1e308, -1e308, 1.0]
    cases = []
    for _ in range(2000):
        u = rng.standard_normal(6) * 10.0 ** rng.integers(-30, 30, 6)
        k = rng.standard_normal(4) * 10.0 ** rng.integers(-5, 5, 4)
        cases.append((u, k))
    for i in range(6):
        for v in specials:
            for base in (np.zeros(6), np.ones(6), rng.standard_normal(6)):
                u = base.copy()
                u[i] = v
                cases.append((u, rng.standard_normal(4)))
                cases.append((u, np.array([0.0, 1.0, 0.0, 1.0])))
    cases.append((np.zeros(6), np.zeros(4)))
    cases.append((np.array([0, 0, 0, 1e300, 0, 1e300]), np.array([1e10, 1e10, 1.0, 1.0])))
    out = np.zeros(10)
    bad = []
    for u, k in cases:
        u = np.ascontiguousarray(u, dtype=np.float64)
        k = np.ascontiguousarray(k, dtype=np.float64)
        sim.sim_kerr_epi_pair(u.ctypes.data, k.ctypes.data, out.ctypes.data)
        if out[:5].tobytes() != out[5:].tobytes():
            bad.append((u.tolist(), k.tolist(), out.tolist()))
    assert not bad, bad[:3]
