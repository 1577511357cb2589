"""CPU tests of the result persistence protocol (pdeval/persist.py): the worker's result tuples
applied to a run database with the reference's schema by the centralized writer
(general_method_paper_reproduction.py:1109-1220), and the rows --print-run-id reports
(_generate_report_from_db, :1826-1870)."""
import hashlib
import os
import queue
import sqlite3
import threading

import golden_data as G
from pdeval import persist


def _sig(s):
    return int(hashlib.sha256(s.encode()).hexdigest()[:12], 16)


def test_writer_applies_worker_tuples(tmp_path):
    db = os.path.join(tmp_path, 'run.db')
    run_id = 'paper_repro_test-1'
    table = persist.init_run_db(db, run_id, max_depth=2)
    assert table == 'expressions_paper_repro_test_1'
    rows = G.decided(G.ref_rows('ff_d1.jsonl', 'ff_d2.jsonl'))
    ids = persist.insert_candidates(db, table, [(r['expr'], r['expr'], _sig(r['expr']), r['depth']) for r in rows])
    assert len(ids) == len(rows)
    persist.register_worker(db, run_id, 4242)
    q = queue.Queue()
    t = threading.Thread(target=lambda: out.append(persist.result_writer(run_id, table, db, q, poll_s=0.05)))
    out = []
    t.start()
    known = {'rho**2': 'Vertical field', 'rho**2*z': 'X-point'}
    results = [('completed', bool(r['ok']), r['reason'], r['expr'] in known, known.get(r['expr']), i)
               for i, r in zip(ids, rows)]
    half = len(results) // 2
    q.put((run_id, 4242, 'start', ids[0], rows[0]['expr'][:120]))
    q.put((run_id, 4242, 'end', results[:half]))
    q.put((run_id, 4242, results[half:-2]))            # legacy (run_id, pid, results)
    q.put((run_id, results[-2:]))                      # legacy (run_id, results)
    q.put(('another-run', 1, 'end', results))          # other runs are ignored
    q.put(None)
    t.join(timeout=30)
    assert out == [len(results)]
    conn = sqlite3.connect(db)
    got = dict(conn.execute(f'SELECT id, is_valid FROM {table}').fetchall())
    assert all(got[i] == int(r['ok']) for i, r in zip(ids, rows))
    assert conn.execute(f"SELECT COUNT(*) FROM {table} WHERE validation_status = 'completed'").fetchone()[0] == len(rows)
    reasons = dict(conn.execute(f'SELECT id, validation_reason FROM {table}').fetchall())
    assert all(reasons[i] == r['reason'] for i, r in zip(ids, rows))
    assert conn.execute("SELECT validated FROM worker_progress WHERE pid = 4242").fetchone()[0] == len(results) - 2
    tg, tv = conn.execute('SELECT total_generated, total_validated FROM run_metadata WHERE run_id = ?',
                          (run_id,)).fetchone()
    assert (tg, tv) == (len(rows), len(rows))
    rep = persist.report(db, table)
    assert rep['total'] == len(rows) and rep['not_completed'] == 0
    assert rep['valid'] == sum(bool(r['ok']) for r in rows)
    want = sorted(known[r['expr']] for r in rows if r['expr'] in known)
    assert want and sorted(n for _, n in rep['paper_solutions']) == want
    assert rep['paper_distinct'] == len(want)
    assert dict(rep['by_depth']) == {d: sum(r['depth'] == d for r in rows) for d in (1, 2)}


def test_start_message_marks_in_progress(tmp_path):
    db = os.path.join(tmp_path, 'run.db')
    table = persist.init_run_db(db, 'r')
    ids = persist.insert_candidates(db, table, [('rho', 'rho', 1, 1), ('z', 'z', 2, 1)])
    q = queue.Queue()
    q.put(('r', 7, 'start', ids[1], 'z'))
    q.put(None)
    persist.result_writer('r', table, db, q, poll_s=0.05)
    st = dict(sqlite3.connect(db).execute(f'SELECT id, validation_status FROM {table}').fetchall())
    assert st == {ids[0]: 'pending', ids[1]: 'in_progress'}
