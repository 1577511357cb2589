#!/usr/bin/env python3
"""Merge the parts of `bench.py --strict-full --part P --parts N` (one GPU call each) into the
whole-set record of the streaming strict mode: rows, seconds, candidates/s over the 142,004
validated d4 strings, suspects, replays, timeouts, verdict changes.  Parts may come from
different splits (thirds, sixths) as long as their row ranges tile the set exactly.
Usage: python scripts/strict_full_summary.py OUT.json PART.json [...]"""
import json
import sys


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    parts = []
    for p in paths:
        with open(p) as f:
            parts.append(json.loads(f.read().strip().split('\n')[-1]))
    parts.sort(key=lambda r: r['rows_range'][0])
    pos = 0
    for r in parts:
        assert r['rows_range'][0] == pos and r['complete'], (r['rows_range'], pos)
        pos = r['rows_range'][1]
    keys = ('strings', 'rows', 'grid_zero', 'sent', 'suspect', 'replayed', 'timeouts', 'verdicts_changed_vs_default')
    tot = {k: sum(r[k] for r in parts) for k in keys}
    sec = sum(r['seconds'] for r in parts)
    rec = {'metric': parts[0]['metric'], 'rows_covered': pos, 'complete': pos == 142004, **tot,
           'seconds': round(sec, 2), 'candidates_per_s': round(tot['strings'] / sec, 1),
           'suspect_fraction': round(tot['suspect'] / tot['strings'], 5),
           'suspect_fraction_of_grid_zeros': round(tot['suspect'] / max(1, tot['grid_zero']), 4),
           'timeout_s': parts[0]['timeout_s'], 'batch': parts[0]['batch'],
           'parts': [{'rows_range': r['rows_range'], 'seconds': r['seconds'], 'candidates_per_s': r['candidates_per_s'],
                      'suspect': r['suspect'], 'timeouts': r['timeouts']} for r in parts],
           'note': 'sum of the parts\' wall times (each part a separate GPU call, the SymPy pool started per part)'}
    with open(out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != 'parts'}))


if __name__ == '__main__':
    main()
