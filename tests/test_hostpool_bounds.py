"""Every host SymPy step has a time bound: a check that hangs
returns within its bound and the device's class stands -- on the main thread (SIGALRM), on a
worker thread with no pool (helper thread), and in the pool when a child is stuck where
SIGALRM cannot reach it (the job's deadline)."""
import os
import signal
import subprocess
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _hang(x):
    if x == 'hang':
        time.sleep(60)
    return x


def _hang_unsignalled(x):
    """Sleeps with SIGALRM blocked: a child stuck in a C-level call the signal cannot interrupt."""
    if x == 'hang':
        signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGALRM})
        time.sleep(60)
    return x


def test_bounded_call_main_thread_restores_timer():
    from pdeval import hostpool
    signal.setitimer(signal.ITIMER_REAL, 100.0)      # an application's own timer
    try:
        t0 = time.time()
        assert hostpool.run(_hang, ['a', 'hang', 'b'], item_timeout=0.5, default='T') == ['a', 'T', 'b']
        assert time.time() - t0 < 5
        left, _ = signal.getitimer(signal.ITIMER_REAL)
        assert 90.0 < left <= 100.0                      # restored, not cancelled
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)


def test_bounded_call_worker_thread_without_pool():
    from pdeval import hostpool
    assert not hostpool.active()
    box = {}

    def body():
        t0 = time.time()
        box['got'] = hostpool.run(_hang, ['a', 'hang'], min_items=1, item_timeout=0.5, default='T')
        box['dt'] = time.time() - t0

    t = threading.Thread(target=body)
    t.start()
    t.join(20)
    assert box.get('got') == ['a', 'T'] and box['dt'] < 5, box


def _kerr_overflow_case():
    """A Kerr point reject of the fp64 range (exp(r**2/a**2) at r = 5) that the host's exact
    point check re-decides: the device's outputs for it, as the point stage writes them."""
    from pdeval import problem_defs as P
    from pdeval._lib import KerrConstants
    from pdeval.opcodes import CLS_REJECT_POINT
    pd_ = P.kerr()
    s = 'pow_neg_3_2(exp(r**2/a**2)*exp(a**2*x**2))'
    ops, off, _ = P.compile_strings(pd_, [s])
    out = {'status': np.array([CLS_REJECT_POINT], np.uint8), 'verdict': np.array([False]),
           'res_ref': np.array([[0.0, 0.0, np.nan]]), 'q_ref': np.array([np.nan]),
           'n_bad': np.array([0], np.int32), 'n_nonfinite': np.array([0], np.int32)}
    return pd_, KerrConstants(1, 1, 1, 10, 1.171875, 0.359375, 0, 0), [s], out, ops, off


def test_kerr_exact_point_check_hang_keeps_device_class(monkeypatch):
    from pdeval import batch
    from pdeval.opcodes import CLS_ACCEPT, CLS_REJECT_POINT
    pd_, kc, items, out, ops, off = _kerr_overflow_case()
    # the real check passes this candidate (the reference accepts it)
    r = {k: v.copy() for k, v in out.items()}
    assert batch.kerr_exact_point_check(pd_, kc, items, r, ops, off) == [0]
    assert r['status'][0] == CLS_ACCEPT
    # a check that hangs: back within the bound, the device's reject stands
    monkeypatch.setattr(batch, 'HOST_CHECK_TIMEOUT_S', 0.5)
    monkeypatch.setattr(batch, '_kerr_fast_point_check', lambda *a: time.sleep(60))
    for via_thread in (False, True):
        r = {k: v.copy() for k, v in out.items()}
        box = {}

        def body():
            t0 = time.time()
            box['rows'] = batch.kerr_exact_point_check(pd_, kc, items, r, ops, off)
            box['dt'] = time.time() - t0
        if via_thread:
            t = threading.Thread(target=body)
            t.start()
            t.join(20)
        else:
            body()
        assert box.get('rows') == [] and box['dt'] < 5, box
        assert r['status'][0] == CLS_REJECT_POINT


def test_zero_gradient_hang_keeps_device_class(monkeypatch):
    from pdeval import batch
    from pdeval import problem_defs as P
    from pdeval.opcodes import CLS_ACCEPT, CLS_ZERO_GRADIENT
    pd_ = P.force_free()
    items = ['exp_neg(rho**2 + z**2)*exp(rho**2)*exp(z**2)']
    out = {'status': np.array([CLS_ACCEPT], np.uint8), 'verdict': np.array([True]),
           'fingerprint': np.ones((1, 4))}
    r = {k: v.copy() for k, v in out.items()}
    assert batch.symbolic_zero_gradient(pd_, items, r) == [0] and r['status'][0] == CLS_ZERO_GRADIENT
    monkeypatch.setattr(batch, 'HOST_CHECK_TIMEOUT_S', 0.5)
    monkeypatch.setattr(batch, '_zero_gradient', lambda *a: time.sleep(60))
    r = {k: v.copy() for k, v in out.items()}
    t0 = time.time()
    assert batch.symbolic_zero_gradient(pd_, items, r) == []
    assert time.time() - t0 < 5 and r['status'][0] == CLS_ACCEPT and r['verdict'][0]


def _pool_deadline_body():
    from pdeval import hostpool
    hostpool.DEADLINE_MARGIN_S = 2.0
    assert hostpool.start(2) is not None
    try:
        t0 = time.time()
        got = hostpool.run(_hang_unsignalled, ['a', 'hang', 'b', 'c'], min_items=1, item_timeout=0.5, default='T')
        dt = time.time() - t0
        # the stuck chunk yields the default for its items; the others their values
        assert got[1] == 'T' and [g for g in got if g != 'T'] and dt < 15, (got, dt)
        assert hostpool._POOL.overdue == 1
        # the pool still serves jobs on its other child
        assert hostpool.run(_hang, ['x', 'y'], min_items=1) == ['x', 'y']
    finally:
        hostpool.stop()


def test_pool_job_deadline_stuck_child():
    code = (f"import sys; sys.path[:0] = [{HERE!r}, {os.path.join(os.path.dirname(HERE), 'pde-engine_amd')!r}]; "
            "import test_hostpool_bounds as t; t._pool_deadline_body(); print('BODY-OK')")
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and 'BODY-OK' in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


def _sleep_unsignalled(x):
    """'hang4' sleeps 4 s and 's1' 1 s, with SIGALRM blocked (no per-item bound reaches them)."""
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGALRM})
    try:
        time.sleep({'hang4': 4.0, 's1': 1.0}.get(x, 0.0))
    finally:
        signal.pthread_sigmask(signal.SIG_UNBLOCK, {signal.SIGALRM})
    return x


def _pool_cancel_body():
    from pdeval import hostpool
    hostpool.DEADLINE_MARGIN_S = 0.5
    assert hostpool.start(1) is not None
    try:
        got = hostpool.run(_sleep_unsignalled, ['hang4'] + ['s1'] * 5, min_items=1, item_timeout=0.2, default='T')
        assert got == ['T'] * 6 and hostpool._POOL.overdue == 1, got
        # the overdue job's items still queued are skipped once the child is free again: the
        # next job waits for the 4 s hang only, not for five more 1 s items
        t0 = time.time()
        assert hostpool.run(_sleep_unsignalled, ['y'], min_items=1) == ['y']
        assert time.time() - t0 < 3.5, time.time() - t0
    finally:
        hostpool.stop()


def test_pool_overdue_job_is_cancelled():
    """after a job's deadline its unfinished chunks no longer run ahead of the next
    jobs (a shared per-job cancel flag the children check before each item)."""
    code = (f"import sys; sys.path[:0] = [{HERE!r}, {os.path.join(os.path.dirname(HERE), 'pde-engine_amd')!r}]; "
            "import test_hostpool_bounds as t; t._pool_cancel_body(); print('BODY-OK')")
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and 'BODY-OK' in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
