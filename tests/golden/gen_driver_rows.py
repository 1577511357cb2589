#!/usr/bin/env python3
"""Fixture generator (runs ONLY in the build container, never on the GPU box).

Runs the reference's own driver end to end -- ``general_method_paper_reproduction.py
--problem force_free|kerr_magnetosphere --max-depth 2 --validators 0`` (generate -> Lean-normalize -> inline
``validate`` -> SQLite, ``:1222-1669``) -- in a scratch copy of the reference, under a wall-clock
limit, and dumps the rows of its run table as data:

    tests/golden/ref/driver_ff_d2_rows.jsonl   one object per row, in id order:
        id, expression, normalized, signature, depth, validation_status, is_valid,
        validation_reason, is_paper_solution, paper_solution_name
    tests/golden/ref/driver_ff_d2_run.json     run facts (rows, wall time, whether it finished)

``--validators N > 0`` is not usable in this checkout: ``_parallel_validator_worker`` imports
``physics_agent.problems`` (absent), falls back to ``PreciseFoliationValidator`` and dies with
``NameError`` at ``:1701`` (never imported in that module), so no row is ever validated; the
inline path is the one that runs.  It has no per-candidate timeout: on this box its 51st row
did not return within 50 min, so the fixture holds the rows that completed before the limit.
``--db`` dumps an existing run database instead of running the driver.
"""
import argparse
import glob
import json
import os
import sqlite3
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_streams import make_scratch_copy  # noqa: E402

COLS = ('id', 'expression', 'normalized', 'signature', 'depth', 'validation_status', 'is_valid',
        'validation_reason', 'is_paper_solution', 'paper_solution_name')
# the inline path's describe() / last_evidence() columns (:1324-1365), dumped for Kerr
EVIDENCE_COLS = ('validator_method', 'validator_math', 'validator_evidence')


def dump(db, out_rows, evidence=False):
    c = sqlite3.connect(db)
    table = [r[0] for r in c.execute("select name from sqlite_master where type='table' "
                                     "and name like 'expressions_%'")][0]
    cols = COLS + (EVIDENCE_COLS if evidence else ())
    rows = c.execute(f"select {', '.join(cols)} from {table} order by id").fetchall()
    with open(out_rows, 'w') as f:
        for r in rows:
            f.write(json.dumps(dict(zip(cols, r))) + '\n')
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/tmp/refdrv')
    ap.add_argument('--max-depth', type=int, default=2)
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--limit-s', type=int, default=3000)
    ap.add_argument('--db', default=None, help='dump this run database instead of running the driver')
    ap.add_argument('--out', default=os.path.join(HERE, 'ref'))
    a = ap.parse_args()
    facts = {'command': f'general_method_paper_reproduction.py --problem {a.problem} '
                        f'--max-depth {a.max_depth} --validators 0'}
    if a.db is None:
        make_scratch_copy('/root/reference', a.ref)
        t0 = time.time()
        try:
            subprocess.run([sys.executable, 'general_method_paper_reproduction.py', '--problem', a.problem,
                            '--max-depth', str(a.max_depth), '--validators', '0'], cwd=a.ref,
                           timeout=a.limit_s, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            facts['finished'] = True
        except subprocess.TimeoutExpired:
            facts['finished'] = False
        facts['wall_s'] = round(time.time() - t0, 1)
        a.db = sorted(glob.glob(os.path.join(a.ref, f'problems/{a.problem}/outputs/parallel_runs_*.db')),
                      key=os.path.getmtime)[-1]
    tag = 'ff' if a.problem == 'force_free' else 'kerr'
    rows = dump(a.db, os.path.join(a.out, f'driver_{tag}_d{a.max_depth}_rows.jsonl'), evidence=tag != 'ff')
    facts['rows'] = len(rows)
    facts['completed'] = sum(r[5] == 'completed' for r in rows)
    facts['valid'] = sum(bool(r[6]) for r in rows)
    with open(os.path.join(a.out, f'driver_{tag}_d{a.max_depth}_run.json'), 'w') as f:
        json.dump(facts, f, indent=1)
    print(json.dumps(facts))


if __name__ == '__main__':
    main()
