#!/usr/bin/env python3
"""Summarize a rocprofv3 results database (kernel trace) into a per-kernel stats table."""
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                     "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(scratch_size), "
                     "max(grid_x), max(workgroup_x) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    lines = [f"# rocprofv3 --kernel-trace summary of {db}",
             "# name | calls | total_ns | avg_ns | min_ns | max_ns | pct | vgpr | agpr | sgpr | scratch | grid_x | wg_x"]
    for r in rows:
        lines.append(f"{r[0]} | {r[1]} | {r[2]:.0f} | {r[3]:.0f} | {r[4]:.0f} | {r[5]:.0f} | "
                     f"{100*r[2]/tot:.2f} | {r[6]} | {r[7]} | {r[8]} | {r[9]} | {r[10]} | {r[11]}")
    txt = '\n'.join(lines) + '\n'
    if out:
        open(out, 'w').write(txt)
    print(txt)


if __name__ == '__main__':
    main(*sys.argv[1:])
