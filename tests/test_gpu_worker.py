"""GPU: the batched validator worker speaks the reference's queue protocol
(general_method_paper_reproduction.py:1723-1816) and tags the paper's known solutions."""
import queue

import pytest

import golden_data as G

pytestmark = pytest.mark.gpu


def test_worker_queue_protocol_and_tags():
    from pdeval.worker import validator_worker
    rows = G.decided(G.ref_rows('ff_edge.jsonl', 'ff_d2.jsonl'))
    tq, rq = queue.Queue(), queue.Queue()
    for i, r in enumerate(rows):
        tq.put((i + 1, r['expr']))
    tq.put(None)
    n = validator_worker('run_test', None, None, 'force_free', tq, rq, batch_size=64)
    assert n == len(rows)
    msgs = []
    while not rq.empty():
        msgs.append(rq.get())
    ends = [m for m in msgs if m[2] == 'end']
    assert all(m[0] == 'run_test' and m[2] in ('start', 'end') for m in msgs)
    res = {t[5]: t for m in ends for t in m[3]}
    assert len(res) == len(rows)
    for i, r in enumerate(rows):
        status, ok, reason, is_paper, name, eid = res[i + 1]
        assert status == 'completed' and ok == r['ok'], (r['expr'], reason)
    tagged = {rows[eid - 1]['expr']: name for eid, t in res.items() for name in [t[4]] if t[3]}
    # the 6 paper solutions the reference decides, in original and stream forms
    for s in ('rho**2', 'rho**2*z', '1 - z/sqrt(rho**2 + z**2)', 'rho**2/(rho**2 + z**2)**(3/2)',
              'sqrt(rho**2 + z**2) - z', 'rho**2*exp(-2*z)', '-z/sqrt(rho**2 + z**2) + 1',
              'square(rho*exp_neg(z))'):
        assert s in tagged, (s, tagged)
