"""Result persistence: the run database and the centralized result writer.

The reference's validator workers never touch the candidate table directly; they put result
tuples on a queue and one writer process applies them in bulk
(``general_method_paper_reproduction.py:1109-1220``):

* ``(run_id, pid, 'start', expr_id, snippet)``  -- the worker took a candidate: the row goes
  from 'pending' to 'in_progress' and ``worker_progress`` records it (:1137-1151);
* ``(run_id, pid, 'end', [(status, is_valid, reason, is_paper, paper_name, id), ...])`` and the
  legacy ``(run_id, pid, results)`` / ``(run_id, results)`` forms -- appended to a batch that is
  written with ONE ``executemany`` UPDATE per drain (:1178-1189), plus the per-worker counters
  (:1190-1199); ``run_metadata`` totals are refreshed at most once a second (:1206-1218);
* ``None`` stops the writer.

``pdeval/worker.py`` emits exactly these tuples, so the reference's own writer consumes them
unchanged.  This module restates the writer (and the schema of ``_init_parallel_database``,
:644-747) so the GPU worker pool can run standalone and so the protocol is tested here; its
:func:`report` runs the queries of ``_generate_report_from_db`` (:1826-1870), i.e. what
``--print-run-id`` prints.
"""
from __future__ import annotations

import queue as _queue
import sqlite3
import time
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

Result = Tuple[str, Optional[bool], str, Optional[bool], Optional[str], int]


def table_name_for(run_id: str) -> str:
    return f"expressions_{run_id.replace('-', '_')}"      # :646


def init_run_db(db_path: str, run_id: str, max_depth: int = 4) -> str:
    """Create the run's candidate table, indices and bookkeeping tables (the reference's
    schema, :655-742).  Returns the table name."""
    table = table_name_for(run_id)
    conn = sqlite3.connect(db_path, timeout=60)
    try:
        c = conn.cursor()
        c.execute('PRAGMA journal_mode=WAL')
        c.execute(f"""CREATE TABLE IF NOT EXISTS {table} (
            id INTEGER PRIMARY KEY AUTOINCREMENT,
            expression TEXT NOT NULL,
            normalized TEXT NOT NULL UNIQUE,
            signature INTEGER,
            depth INTEGER NOT NULL,
            validation_status TEXT DEFAULT 'pending',
            is_valid BOOLEAN,
            validation_reason TEXT,
            validator_method TEXT,
            validator_math TEXT,
            is_paper_solution BOOLEAN DEFAULT 0,
            paper_solution_name TEXT,
            created_at TIMESTAMP DEFAULT CURRENT_TIMESTAMP,
            validated_at TIMESTAMP,
            validator_evidence TEXT)""")
        for col in ('signature', 'validation_status', 'depth'):
            short = {'validation_status': 'status'}.get(col, col)
            c.execute(f'CREATE INDEX IF NOT EXISTS idx_{table}_{short} ON {table}({col})')
        c.execute("""CREATE TABLE IF NOT EXISTS run_metadata (
            run_id TEXT PRIMARY KEY, table_name TEXT NOT NULL,
            started_at TIMESTAMP DEFAULT CURRENT_TIMESTAMP, completed_at TIMESTAMP,
            max_depth INTEGER, total_generated INTEGER, total_validated INTEGER,
            valid_solutions INTEGER, status TEXT DEFAULT 'running')""")
        c.execute("""CREATE TABLE IF NOT EXISTS generator_progress (
            run_id TEXT PRIMARY KEY, state_json TEXT, updated_at TIMESTAMP DEFAULT CURRENT_TIMESTAMP)""")
        c.execute("""CREATE TABLE IF NOT EXISTS worker_progress (
            run_id TEXT NOT NULL, pid INTEGER NOT NULL, role TEXT, validated INTEGER DEFAULT 0,
            errors INTEGER DEFAULT 0, updated_at TIMESTAMP DEFAULT CURRENT_TIMESTAMP,
            current_expr_id INTEGER, current_started_at TIMESTAMP, current_expr_snippet TEXT,
            last_completed_id INTEGER, last_completed_at TIMESTAMP, PRIMARY KEY (run_id, pid))""")
        c.execute('INSERT OR IGNORE INTO run_metadata (run_id, table_name, max_depth) VALUES (?, ?, ?)',
                  (run_id, table, max_depth))
        conn.commit()
    finally:
        conn.close()
    return table


def insert_candidates(db_path: str, table: str, rows: Iterable[Tuple[str, str, int, int]]) -> List[int]:
    """INSERT (expression, normalized, signature, depth) rows as 'pending' (the generator's
    INSERT, :1277-1286 / :1367-1378); returns their ids."""
    conn = sqlite3.connect(db_path, timeout=60)
    ids = []
    try:
        for expr, norm, sig, depth in rows:
            cur = conn.execute(f'INSERT OR IGNORE INTO {table} (expression, normalized, signature, depth) '
                               f'VALUES (?, ?, ?, ?)', (expr, norm, sig, depth))
            if cur.rowcount == 1:
                ids.append(cur.lastrowid)
        conn.commit()
    finally:
        conn.close()
    return ids


def register_worker(db_path: str, run_id: str, pid: int, role: str = 'validator'):
    conn = sqlite3.connect(db_path, timeout=60)
    try:
        conn.execute('INSERT OR IGNORE INTO worker_progress (run_id, pid, role) VALUES (?, ?, ?)', (run_id, pid, role))
        conn.commit()
    finally:
        conn.close()


def result_writer(run_id: str, table: str, db_path: str, result_queue, poll_s: float = 0.5,
                  meta_every_s: float = 1.0) -> int:
    """The centralized writer (:1109-1220): drain `result_queue` until ``None``; returns the
    number of result rows written."""
    conn = sqlite3.connect(db_path)
    conn.execute('PRAGMA journal_mode=WAL')
    conn.execute('PRAGMA busy_timeout=5000')
    cur = conn.cursor()
    batch: List[Result] = []
    worker_counts: Dict[int, int] = {}
    written = 0
    last_meta = time.time()
    try:
        while True:
            try:
                item = result_queue.get(timeout=poll_s)
            except _queue.Empty:
                item = ()
            if item is None:
                break
            if item:
                if len(item) >= 3 and isinstance(item[2], str):
                    rid, wpid, kind = item[:3]
                    if rid == run_id and kind == 'start':
                        _, _, _, expr_id, snippet = item
                        try:
                            cur.execute('UPDATE worker_progress SET current_expr_id = ?, current_started_at = '
                                        'CURRENT_TIMESTAMP, current_expr_snippet = ?, updated_at = CURRENT_TIMESTAMP '
                                        'WHERE run_id = ? AND pid = ?', (expr_id, snippet, run_id, wpid))
                            cur.execute(f"UPDATE {table} SET validation_status = 'in_progress' "
                                        f"WHERE id = ? AND validation_status = 'pending'", (expr_id,))
                            conn.commit()
                        except sqlite3.Error:
                            pass
                    elif rid == run_id and kind == 'end':
                        results = item[3]
                        worker_counts[wpid] = worker_counts.get(wpid, 0) + len(results)
                        batch.extend(results)
                elif len(item) == 3:                       # legacy (run_id, pid, results)
                    rid, wpid, results = item
                    if rid == run_id:
                        worker_counts[wpid] = worker_counts.get(wpid, 0) + len(results)
                        batch.extend(results)
                elif len(item) == 2 and item[0] == run_id:  # legacy (run_id, results)
                    batch.extend(item[1])
            if batch:
                try:
                    cur.executemany(f"""UPDATE {table}
                        SET validation_status = ?, is_valid = ?, validation_reason = ?,
                            is_paper_solution = ?, paper_solution_name = ?, validated_at = CURRENT_TIMESTAMP
                        WHERE id = ?""", batch)
                    for wpid, cnt in list(worker_counts.items()):
                        cur.execute(f"UPDATE worker_progress SET validated = COALESCE(validated, 0) + ?, "
                                    f"last_completed_id = (SELECT MAX(id) FROM {table} WHERE validation_status = "
                                    f"'completed'), last_completed_at = CURRENT_TIMESTAMP, current_expr_id = NULL, "
                                    f"current_expr_snippet = NULL, updated_at = CURRENT_TIMESTAMP "
                                    f"WHERE run_id = ? AND pid = ?", (cnt, run_id, wpid))
                        del worker_counts[wpid]
                    conn.commit()
                    written += len(batch)
                    batch.clear()
                except sqlite3.OperationalError:        # locked: retry on the next drain
                    time.sleep(0.02)
            if time.time() - last_meta > meta_every_s:
                _refresh_meta(conn, table, run_id)
                last_meta = time.time()
        _refresh_meta(conn, table, run_id)
    finally:
        conn.close()
    return written


def _refresh_meta(conn, table: str, run_id: str):
    try:
        tg, tv = conn.execute(f"SELECT COUNT(*), COUNT(CASE WHEN validation_status != 'pending' THEN 1 END) "
                              f"FROM {table}").fetchone()
        conn.execute('UPDATE run_metadata SET total_generated = ?, total_validated = ? WHERE run_id = ?',
                     (tg, tv, run_id))
        conn.commit()
    except sqlite3.Error:
        pass


def report(db_path: str, table: str) -> dict:
    """What ``--print-run-id`` prints (_generate_report_from_db, :1833-1870)."""
    conn = sqlite3.connect(db_path)
    try:
        total, valid, paper_distinct = conn.execute(
            f"SELECT COUNT(*), SUM(CASE WHEN is_valid = 1 THEN 1 ELSE 0 END), "
            f"COUNT(DISTINCT CASE WHEN is_paper_solution = 1 THEN signature END) FROM {table}").fetchone()
        papers = conn.execute(f'SELECT expression, paper_solution_name FROM {table} '
                              f'WHERE is_paper_solution = 1 ORDER BY paper_solution_name').fetchall()
        by_depth = conn.execute(f'SELECT depth, COUNT(*) FROM {table} GROUP BY depth ORDER BY depth').fetchall()
        pending = conn.execute(f"SELECT COUNT(*) FROM {table} WHERE validation_status != 'completed'").fetchone()[0]
    finally:
        conn.close()
    return {'total': total, 'valid': valid or 0, 'paper_distinct': paper_distinct or 0,
            'paper_solutions': papers, 'by_depth': by_depth, 'not_completed': pending}
