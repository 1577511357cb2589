"""ctypes loader for the CPU oracle (oracle/_build/libjetoracle.so) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'oracle', '_build', 'libjetoracle.so')
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
        _lib = C.CDLL(LIB)
        vp = C.c_void_p
        _lib.oracle_validate.argtypes = [C.c_int, vp, vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp,
                                         vp, C.c_int64, C.c_int64]
        _lib.oracle_jet.argtypes = [C.c_int, vp, C.c_int64, C.c_double, C.c_double, C.c_int, vp, vp]
        _lib.oracle_point.argtypes = [C.c_int, vp, C.c_int64, C.c_double, C.c_double, C.c_int, vp]
        _lib.oracle_set_omega2.argtypes = [C.c_double]
        _lib.oracle_set_omega2_lo.argtypes = [C.c_double]
        _lib.oracle_set_kerr_constants.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                                   C.c_double, C.c_double, C.c_int, C.c_int]
    return _lib


DEFAULT_KERR = (1, 1, 1, 10, 1.171875, 0.359375, 0, 0)   # pdeval_default_kerr_constants


def set_kerr_constants(k=DEFAULT_KERR):
    """The oracle's Kerr constants (a pdeval._lib.KerrConstants or the 8-tuple of its fields);
    process-wide: set it before validating, not while another thread validates."""
    if hasattr(k, 'key'):
        k = k.key()
    load().oracle_set_kerr_constants(*k)


class _Params(C.Structure):
    _fields_ = [('tau_point', C.c_double), ('tau_grid', C.c_double),
                ('kerr_abs_tol', C.c_double), ('full_grid', C.c_int32), ('max_bad', C.c_int32),
                ('strict_symbolic', C.c_int32), ('reserved', C.c_int32),
                ('noise_kappa', C.c_double), ('point_abs_tol', C.c_double),
                ('res_rel_acc', C.c_double), ('omega2', C.c_double),
                ('omega2_lo', C.c_double)]


def params(tau_point=1e-10, tau_grid=1e-7, kerr_abs_tol=1e-10, full_grid=1, max_bad=0,
           strict_symbolic=1, noise_kappa=16.0, point_abs_tol=1e-20, res_rel_acc=1e-11, omega2=0.0,
           omega2_lo=0.0):
    return _Params(tau_point, tau_grid, kerr_abs_tol, full_grid, max_bad, strict_symbolic, 0,
                   noise_kappa, point_abs_tol, res_rel_acc, omega2, omega2_lo)


def validate(problem_id, ops, offsets, prm=None, first=0, count=-1, n_ref=None):
    """Oracle verdicts for programs [first, first+count); returns dict of arrays (full length)."""
    lib = load()
    ops = np.ascontiguousarray(ops, dtype=np.int32)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    nref = n_ref if n_ref is not None else (1 if problem_id == 0 else 3)
    out = dict(status=np.full(n, 255, np.uint8), q_ref=np.zeros(n), res_ref=np.zeros(n * nref),
               q_grid=np.zeros(n), n_bad=np.zeros(n, np.int32), n_nonfinite=np.zeros(n, np.int32),
               fingerprint=np.zeros(n * 4))
    prm = prm or params()
    lib.oracle_validate(problem_id, ops.ctypes.data, offsets.ctypes.data, n, C.addressof(prm),
                        *[out[k].ctypes.data for k in ('status', 'q_ref', 'res_ref', 'q_grid',
                                                       'n_bad', 'n_nonfinite', 'fingerprint')],
                        first, count)
    out['res_ref'] = out['res_ref'].reshape(n, nref)
    out['fingerprint'] = out['fingerprint'].reshape(n, 4)
    return out


def jet(problem_id, words, x, y, cplx=False):
    lib = load()
    w = np.ascontiguousarray(words, dtype=np.int32)
    nc = 15 if problem_id == 0 else 6
    re, im = np.zeros(nc), np.zeros(nc)
    rc = lib.oracle_jet(problem_id, w.ctypes.data, w.size, x, y, int(cplx), re.ctypes.data, im.ctypes.data)
    if rc:
        raise ValueError(f'oracle_jet rc={rc}')
    return re + 1j * im if cplx else re


def set_omega2(w):
    """Force-free Omega^2 of the oracle's oracle_point / oracle_jet (oracle_validate takes it
    from its params)."""
    load().oracle_set_omega2(float(w))
    load().oracle_set_omega2_lo(0.0)


def point(problem_id, words, x, y, cplx=False):
    """(|residual|, S, noise bound, finite) at one point, with the tier-2 noise bound."""
    lib = load()
    w = np.ascontiguousarray(words, dtype=np.int32)
    out = np.zeros(4)
    rc = lib.oracle_point(problem_id, w.ctypes.data, w.size, x, y, int(cplx), out.ctypes.data)
    if rc:
        raise ValueError(f'oracle_point rc={rc}')
    return out


def validate_mt(problem_id, ops, offsets, prm=None, threads=None, chunk=64):
    """validate() over a thread pool (the C oracle keeps no global state and ctypes releases
    the GIL): chunks of `chunk` programs, results identical to the one-thread call."""
    from concurrent.futures import ThreadPoolExecutor
    lib = load()
    ops = np.ascontiguousarray(ops, dtype=np.int32)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    nref = 1 if problem_id == 0 else 3
    out = dict(status=np.full(n, 255, np.uint8), q_ref=np.zeros(n), res_ref=np.zeros(n * nref),
               q_grid=np.zeros(n), n_bad=np.zeros(n, np.int32), n_nonfinite=np.zeros(n, np.int32),
               fingerprint=np.zeros(n * 4))
    prm = prm or params()
    ptrs = [out[k].ctypes.data for k in ('status', 'q_ref', 'res_ref', 'q_grid', 'n_bad',
                                         'n_nonfinite', 'fingerprint')]

    def run(first):
        lib.oracle_validate(problem_id, ops.ctypes.data, offsets.ctypes.data, n, C.addressof(prm),
                            *ptrs, first, min(chunk, n - first))
    threads = threads or max(1, min(16, int(os.environ.get('OMP_NUM_THREADS') or 0) or os.cpu_count() or 1))
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(0, n, chunk)))
    out['res_ref'] = out['res_ref'].reshape(n, nref)
    out['fingerprint'] = out['fingerprint'].reshape(n, 4)
    return out
