"""ctypes binding of libpdeval.so (the C ABI declared in ``include/pdeval.h``).

This is the Python side of the drop-in boundary: the reference's validator plugins are
Python objects called once per candidate (``problems/__init__.py:52``); here one call
validates a whole batch through the C ABI.  There is deliberately no fallback: if the
library is missing or no GPU is present, :func:`load` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from .opcodes import FP_N

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PDEVAL_LIB', os.path.join(_HERE, '..', 'lib', 'libpdeval.so'))

EXPORTS = (
    'pdeval_create', 'pdeval_destroy', 'pdeval_last_error', 'pdeval_n_ref_points',
    'pdeval_n_points', 'pdeval_default_params', 'pdeval_validate_batch',
    'pdeval_validate_device', 'pdeval_program_depth', 'pdeval_program_flops', 'pdeval_program_hoist_flops',
    'pdeval_version',
    'pdeval_set_timing', 'pdeval_pass_times', 'pdeval_pass_counts', 'pdeval_eval_points',
    'pdeval_compile_batch', 'pdeval_canonical', 'pdeval_point_eval', 'pdeval_point_states',
    'pdeval_comm_unique_id', 'pdeval_comm_init', 'pdeval_gather_bits', 'pdeval_comm_destroy',
    'pdeval_default_kerr_constants', 'pdeval_set_kerr_constants', 'pdeval_compile_batch_mt',
    'pdeval_format_reasons', 'pdeval_device_error',
)
MAX_BATCH = 1 << 30          # PDEVAL_MAX_BATCH
UNIQUE_ID_BYTES = 128
LIST_NAMES = ('defer_stack3', 'complex', 'defer_stack8', 'tier2', 'tier2_stack3', 'tier2_complex',
              'complex_stack8', 'tier2_stack8', 'point_deep', 'point_dd', 'point_dd_complex',
              'point_dd_stack8', 'tier2_complex_stack8', 'grid_slow', 'grid_slow_stack3',
              'grid_slow_complex')
N_PASSES = 12


class Params(C.Structure):
    _fields_ = [('tau_point', C.c_double), ('tau_grid', C.c_double),
                ('kerr_abs_tol', C.c_double), ('full_grid', C.c_int32), ('max_bad', C.c_int32),
                ('strict_symbolic', C.c_int32), ('reserved', C.c_int32),
                ('noise_kappa', C.c_double), ('point_abs_tol', C.c_double),
                ('res_rel_acc', C.c_double), ('omega2', C.c_double),
                ('omega2_lo', C.c_double)]


class Outputs(C.Structure):
    _fields_ = [('verdict_bits', C.c_void_p), ('status', C.c_void_p), ('q_ref', C.c_void_p),
                ('res_ref', C.c_void_p), ('q_grid', C.c_void_p), ('n_bad', C.c_void_p),
                ('n_nonfinite', C.c_void_p), ('fingerprint', C.c_void_p)]


class KerrConstants(C.Structure):
    """pdeval_kerr_constants (include/pdeval.h): the validator's M_value, a_value (exact
    rationals, the point stage) and the stand-ins of the symbols M, a (constant test, grid)."""
    _fields_ = [('M_num', C.c_int64), ('M_den', C.c_int64), ('a_num', C.c_int64), ('a_den', C.c_int64),
                ('M_sym', C.c_double), ('a_sym', C.c_double), ('op_M_fixed', C.c_int32),
                ('op_a_fixed', C.c_int32)]

    def key(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class PdevalError(RuntimeError):
    pass


_lib: Optional[C.CDLL] = None


def load(path: Optional[str] = None) -> C.CDLL:
    """Load libpdeval.so and declare its signatures (raises if it is missing)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = os.path.abspath(path or LIB_PATH)
    if not os.path.exists(p):
        raise PdevalError(f'libpdeval.so not found at {p}: run __graft_entry__.build()')
    lib = C.CDLL(p)
    vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    lib.pdeval_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(vp)]
    lib.pdeval_destroy.argtypes = [vp]
    lib.pdeval_last_error.argtypes = [vp]
    lib.pdeval_last_error.restype = C.c_char_p
    lib.pdeval_n_ref_points.argtypes = [vp]
    lib.pdeval_n_points.argtypes = [vp]
    lib.pdeval_default_params.argtypes = [C.c_int, C.POINTER(Params)]
    lib.pdeval_validate_batch.argtypes = [vp, vp, i64, vp, i64, C.POINTER(Params), C.POINTER(Outputs)]
    lib.pdeval_validate_device.argtypes = [vp, vp, i64, vp, i64, C.POINTER(Params),
                                           C.POINTER(Outputs), vp, C.c_int]
    lib.pdeval_device_error.argtypes = [vp, C.POINTER(C.c_uint32)]
    lib.pdeval_program_depth.argtypes = [vp, i64]
    lib.pdeval_program_flops.argtypes = [C.c_int, vp, i64]
    lib.pdeval_program_flops.restype = dbl
    lib.pdeval_program_hoist_flops.argtypes = [C.c_int, vp, i64]
    lib.pdeval_program_hoist_flops.restype = dbl
    lib.pdeval_version.restype = C.c_char_p
    lib.pdeval_set_timing.argtypes = [vp, C.c_int]
    lib.pdeval_pass_times.argtypes = [vp, vp, C.c_int, vp]
    lib.pdeval_pass_counts.argtypes = [vp, vp, C.c_int]
    lib.pdeval_eval_points.argtypes = [vp, vp, i64, vp, vp, C.c_int, C.c_int, vp, vp]
    lib.pdeval_compile_batch.argtypes = [C.c_int, vp, vp, i64, vp, i64, vp, vp, vp]
    lib.pdeval_canonical.argtypes = [C.c_int, C.c_char_p, i64, C.c_char_p, i64]
    lib.pdeval_compile_batch_mt.argtypes = [C.c_int, vp, vp, i64, vp, i64, vp, vp, vp, C.c_int]
    lib.pdeval_format_reasons.argtypes = [C.c_int, i64, vp, vp, C.c_int, vp, vp, vp, vp, i64, vp]
    lib.pdeval_point_eval.argtypes = [vp, vp, i64, C.c_int, vp, vp]
    lib.pdeval_point_states.argtypes = [vp, vp, i64]
    lib.pdeval_comm_unique_id.argtypes = [vp]
    lib.pdeval_comm_init.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.pdeval_gather_bits.argtypes = [vp, vp, i64, vp, vp]
    lib.pdeval_comm_destroy.argtypes = [vp]
    lib.pdeval_default_kerr_constants.argtypes = [C.POINTER(KerrConstants)]
    lib.pdeval_set_kerr_constants.argtypes = [vp, C.POINTER(KerrConstants)]
    for name in EXPORTS:
        getattr(lib, name)   # every symbol of the header must resolve
    if path is None:
        _lib = lib
    return lib


def default_params(problem_id: int) -> Params:
    p = Params()
    _check(None, load().pdeval_default_params(problem_id, C.byref(p)))
    return p


def default_kerr_constants() -> KerrConstants:
    k = KerrConstants()
    _check(None, load().pdeval_default_kerr_constants(C.byref(k)))
    return k


def _check(ctx, rc: int):
    if rc != 0:
        msg = load().pdeval_last_error(ctx)
        raise PdevalError(f'pdeval error {rc}: {msg.decode() if msg else ""}')


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


CONTEXTS_CREATED = 0   # (pdeval.hostpool forks only before the first one: the GPU is then live)


class Context:
    """One libpdeval context = one GPU + one problem's sample grid."""

    def __init__(self, problem_id: int, device: int = 0, grid: Optional[np.ndarray] = None,
                 kerr: Optional[KerrConstants] = None):
        global CONTEXTS_CREATED
        CONTEXTS_CREATED += 1
        lib = load()
        h = C.c_void_p()
        gp = None
        ng = 0
        if grid is not None:
            g = np.ascontiguousarray(grid, dtype=np.float64)
            gp, ng = g.ctypes.data_as(C.POINTER(C.c_double)), g.size
        rc = lib.pdeval_create(device, problem_id, gp, ng, C.byref(h))
        if rc != 0:
            raise PdevalError(f'pdeval_create failed ({rc}): {lib.pdeval_last_error(None).decode()}')
        self.h = h
        self.lib = lib
        self.problem_id = problem_id
        self.device = device
        self.n_ref = lib.pdeval_n_ref_points(h)
        self.n_points = lib.pdeval_n_points(h)
        if kerr is not None:
            self.set_kerr_constants(kerr)

    def set_kerr_constants(self, k: KerrConstants):
        """The Kerr constants of this context (pdeval_set_kerr_constants)."""
        _check(self.h, self.lib.pdeval_set_kerr_constants(self.h, C.byref(k)))

    def close(self):
        if self.h:
            self.lib.pdeval_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def validate(self, ops: np.ndarray, offsets: np.ndarray, params: Optional[Params] = None):
        """Host arrays in, dict of per-candidate numpy outputs back (synchronous)."""
        ops = np.ascontiguousarray(ops, dtype=np.int32)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = len(offsets) - 1
        res = {
            'verdict_bits': np.zeros((n + 7) // 8, dtype=np.uint8),
            'status': np.zeros(n, dtype=np.uint8),
            'q_ref': np.zeros(n, dtype=np.float64),
            'res_ref': np.zeros(n * self.n_ref, dtype=np.float64),
            'q_grid': np.zeros(n, dtype=np.float64),
            'n_bad': np.zeros(n, dtype=np.int32),
            'n_nonfinite': np.zeros(n, dtype=np.int32),
            'fingerprint': np.zeros(n * FP_N, dtype=np.float64),
        }
        out = Outputs(*[_ptr(res[f]) for f, _ in Outputs._fields_])
        prm = params if params is not None else default_params(self.problem_id)
        rc = self.lib.pdeval_validate_batch(self.h, _ptr(ops), ops.size, _ptr(offsets), n,
                                            C.byref(prm), C.byref(out))
        _check(self.h, rc)
        res['res_ref'] = res['res_ref'].reshape(n, self.n_ref)
        res['fingerprint'] = res['fingerprint'].reshape(n, FP_N)
        res['verdict'] = np.unpackbits(res['verdict_bits'], bitorder='little')[:n].astype(bool)
        return res

    def set_timing(self, enable: bool = True):
        _check(self.h, self.lib.pdeval_set_timing(self.h, int(enable)))

    def pass_times(self):
        """{pass name: ms} of the most recent validate_device call (timing enabled)."""
        ms = (C.c_float * N_PASSES)()
        names = (C.c_char_p * N_PASSES)()
        _check(self.h, self.lib.pdeval_pass_times(self.h, ms, N_PASSES, names))
        return {names[k].decode(): float(ms[k]) for k in range(N_PASSES)}

    def eval_points(self, words, xs, ys, tier2: bool = True, jets: bool = False):
        """(n, 4) array {|residual|, S, noise, finite} of one program at the given points
        (and, with jets=True, an (n, 2, 15) array of u's coefficients and error bounds)."""
        w = np.ascontiguousarray(words, dtype=np.int32)
        x = np.ascontiguousarray(xs, dtype=np.float64)
        y = np.ascontiguousarray(ys, dtype=np.float64)
        out = np.zeros((len(x), 4))
        jt = np.zeros((len(x), 2, 15)) if jets else None
        _check(self.h, self.lib.pdeval_eval_points(self.h, _ptr(w), w.size, _ptr(x), _ptr(y), len(x),
                                                   int(tier2), _ptr(out), _ptr(jt)))
        return (out, jt) if jets else out

    def point_eval(self, words, tier: int):
        """(n_ref, 6) array {Re res, Im res, |res|, S, noise, finite} of one program at the
        reference points in precision tier 0 fp64 / 1 complex / 2 double-double / 3 complex dd,
        and the tier's point-stage decision (PDEVAL_PS_* bits)."""
        w = np.ascontiguousarray(words, dtype=np.int32)
        out = np.zeros((self.n_ref, 6))
        st = np.zeros(1, dtype=np.uint8)
        _check(self.h, self.lib.pdeval_point_eval(self.h, _ptr(w), w.size, tier, _ptr(out), _ptr(st)))
        return out, int(st[0])

    def point_states(self, n: int) -> np.ndarray:
        """Point-stage state (PDEVAL_PS_* bits) of every candidate of the most recent call."""
        out = np.zeros(n, dtype=np.uint8)
        _check(self.h, self.lib.pdeval_point_states(self.h, _ptr(out), n))
        return out

    # ---- multi-GPU exchange (RCCL through the C ABI)
    def comm_init(self, world: int, rank: int, unique_id: bytes):
        """Join the RCCL communicator of `world` ranks (collective; same id on every rank)."""
        buf = C.create_string_buffer(bytes(unique_id), UNIQUE_ID_BYTES)
        _check(self.h, self.lib.pdeval_comm_init(self.h, world, rank, buf))

    def gather_bits(self, d_local: int, nbytes: int, d_global: int, stream: int = 0):
        """All-gather nbytes of device memory from every rank into d_global (world * nbytes)."""
        _check(self.h, self.lib.pdeval_gather_bits(self.h, d_local, nbytes, d_global, stream or None))

    def comm_destroy(self):
        _check(self.h, self.lib.pdeval_comm_destroy(self.h))

    def pass_counts(self):
        """{work list: entries} of the most recent call (synchronizes)."""
        c = (C.c_int64 * len(LIST_NAMES))()
        _check(self.h, self.lib.pdeval_pass_counts(self.h, c, len(LIST_NAMES)))
        return {k: int(c[i]) for i, k in enumerate(LIST_NAMES)}

    def validate_device(self, d_ops: int, n_words: int, d_offsets: int, n: int, d_out: Outputs,
                        params: Optional[Params] = None, stream: int = 0, zero_bits: bool = True):
        """Device pointers in and out (inputs resident in HBM), asynchronous on `stream`."""
        prm = params if params is not None else default_params(self.problem_id)
        if not stream:
            raise PdevalError('validate_device needs an explicit (non-null) HIP stream handle')
        rc = self.lib.pdeval_validate_device(self.h, d_ops, n_words, d_offsets, n, C.byref(prm),
                                             C.byref(d_out), stream, int(zero_bits))
        _check(self.h, rc)

    def device_error(self) -> int:
        """The device error word of the most recent validate_device call (call after its stream
        is synchronized): 0, or PdevalError naming the kernel families whose work-list check met
        an entry outside the batch (pdeval_device_error)."""
        w = C.c_uint32(0)
        _check(self.h, self.lib.pdeval_device_error(self.h, C.byref(w)))
        return int(w.value)


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (on one rank; share it with the others)."""
    buf = C.create_string_buffer(UNIQUE_ID_BYTES)
    rc = load().pdeval_comm_unique_id(buf)
    if rc != 0:
        raise PdevalError(f'pdeval_comm_unique_id failed ({rc}): {load().pdeval_last_error(None).decode()}')
    return buf.raw


def program_depth(words: np.ndarray) -> int:
    w = np.ascontiguousarray(words, dtype=np.int32)
    return load().pdeval_program_depth(_ptr(w), w.size)


def program_flops(problem_id: int, words: np.ndarray) -> float:
    w = np.ascontiguousarray(words, dtype=np.int32)
    return load().pdeval_program_flops(problem_id, _ptr(w), w.size)
