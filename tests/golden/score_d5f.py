#!/usr/bin/env python3
"""Score the product on the faithful depth-5 sample (build container; no reference import).

Input: the reference's verdicts on ``streams/force_free_d5_faithful.txt.gz`` (the sample that
``gen_d5_faithful.py`` draws by the reference's own enumerator rules), recorded by
``gen_reference_verdicts.py verdicts --timeout 20`` into ``ref/d5f_*.jsonl``.

For every DECIDED row (the reference finished within 20 s) it computes, without a GPU:
  * the default ('off') plugin verdict: the device's class -- the C oracle's, which the GPU
    parity tests hold equal to the device class for class -- through the host steps the product
    path applies to force-free rows (pdeval.batch.ff_range_point_check, symbolic_zero_gradient);
  * the 'strict' verdict: the same, and for grid zeros of a suspect shape
    (pdeval.symbolic.suspect, FROZEN: its source is the text of commit 5708cbc, from before this
    sample was drawn; the sha256 of that source is recorded in the summary) the product's replay of the reference's symbolic
    stage (pdeval.symbolic.strict_str, 60 s bound -- past it the device's verdict stands).
The replays are recorded in ``replay/d5f_replay.jsonl`` (strings and verdicts only), so the CPU
test re-scores without SymPy; the summary goes to ``ref/d5f_score.json``.

Usage: python tests/golden/score_d5f.py [--procs N]
"""
import argparse
import glob
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def _replay(s):
    from pdeval import symbolic as S
    from pdeval.hostpool import _call_bounded
    t0 = time.time()
    r = _call_bounded(S.strict_str, ('force_free', s), 60, 'timeout')
    rec = {'expr': s, 't': round(time.time() - t0, 3)}
    if r == 'timeout':
        rec.update(ok=None, reason=None, timeout=True)
    elif r is None or r == 'keep':
        rec.update(ok=None, reason=None, timeout=False, keep=r == 'keep')
    else:
        rec.update(ok=bool(r[0]), reason=r[1], timeout=False)
    return rec


def rows():
    out = []
    for p in sorted(glob.glob(os.path.join(HERE, 'ref', 'd5f_*_t20.jsonl'))):
        with open(p) as f:
            out.extend(json.loads(l) for l in f)
    out.sort(key=lambda r: r['idx'])
    return out


def score(rs, replays):
    """(summary, per-row records) of the decided rows rs with the replay records."""
    import numpy as np
    import oracle_lib as O
    from pdeval import problem_defs as P
    from pdeval import symbolic as S
    from pdeval.batch import ff_range_point_check, symbolic_zero_gradient
    from pdeval.opcodes import CLS_ACCEPT, CLS_REJECT_SYMBOLIC
    pd = P.force_free()
    dec = [r for r in rs if r['ok'] is not None]
    strs = [r['expr'] for r in dec]
    ops, off, _ = P.compile_strings(pd, strs)
    ora = O.validate_mt(0, ops, off)
    ff_range_point_check(pd, strs, ora, ops, off, 4096, True, 0)
    symbolic_zero_gradient(pd, strs, ora)
    zero = np.isin(ora['status'], (CLS_ACCEPT, CLS_REJECT_SYMBOLIC))
    susp = [bool(zero[i]) and S.suspect(pd.parse(s), pd.x, pd.y) for i, s in enumerate(strs)]
    per = []
    for i, r in enumerate(dec):
        dev = bool(ora['status'][i] == CLS_ACCEPT)
        strict = dev
        rep = replays.get(r['expr']) if susp[i] else None
        if susp[i] and rep is not None and rep.get('ok') is not None:
            strict = bool(rep['ok'])
        per.append({'expr': r['expr'], 'ref_ok': bool(r['ok']), 'ref_reason': r['reason'], 'class': int(ora['status'][i]),
                    'off': dev, 'strict': strict, 'grid_zero': bool(zero[i]), 'suspect': susp[i],
                    'replay_timeout': bool(susp[i] and (rep is None or rep.get('timeout')))})
    n = len(per)
    summ = {'rows': len(rs), 'decided': n, 'undecided_20s': len(rs) - n,
            'grid_zero': int(zero.sum()), 'suspect': int(sum(susp)),
            'replay_timeouts': sum(p['replay_timeout'] for p in per),
            'off_agree': sum(p['off'] == p['ref_ok'] for p in per),
            'strict_agree': sum(p['strict'] == p['ref_ok'] for p in per),
            'off_divergent': sorted(p['expr'] for p in per if p['off'] != p['ref_ok']),
            'strict_divergent': sorted(p['expr'] for p in per if p['strict'] != p['ref_ok'])}
    return summ, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=2)
    a = ap.parse_args()
    from pdeval import problem_defs as P
    from pdeval import symbolic as S
    import oracle_lib as O
    import numpy as np
    from pdeval.batch import ff_range_point_check, symbolic_zero_gradient
    from pdeval.opcodes import CLS_ACCEPT, CLS_REJECT_SYMBOLIC
    rs = rows()
    rp = os.path.join(HERE, 'replay', 'd5f_replay.jsonl')
    replays = {}
    if os.path.exists(rp):
        with open(rp) as f:
            replays = {r['expr']: r for r in map(json.loads, f)}
    # the suspects among the decided rows' grid zeros that have no replay record yet
    pd = P.force_free()
    dec = [r for r in rs if r['ok'] is not None]
    strs = [r['expr'] for r in dec]
    ops, off, _ = P.compile_strings(pd, strs)
    ora = O.validate_mt(0, ops, off)
    ff_range_point_check(pd, strs, ora, ops, off, 4096, True, 0)
    symbolic_zero_gradient(pd, strs, ora)
    zero = np.isin(ora['status'], (CLS_ACCEPT, CLS_REJECT_SYMBOLIC))
    need = [s for i, s in enumerate(strs) if zero[i] and s not in replays and S.suspect(pd.parse(s), pd.x, pd.y)]
    print(f'{len(rs)} rows, {len(dec)} decided, {int(zero.sum())} grid zeros, {len(need)} replays to run', flush=True)
    if need:
        with mp.get_context('fork').Pool(a.procs) as pool, open(rp, 'a') as f:
            for k, rec in enumerate(pool.imap_unordered(_replay, need)):
                replays[rec['expr']] = rec
                f.write(json.dumps(rec) + '\n')
                f.flush()
                if (k + 1) % 20 == 0:
                    print(f'[replay] {k + 1}/{len(need)}', flush=True)
    summ, _ = score(rs, replays)
    # the rule scored, frozen: the source of pdeval.symbolic.suspect, equal to its text at
    # commit 5708cbc (before the sample was drawn)
    import inspect
    summ['suspect_source_sha256'] = hashlib.sha256(inspect.getsource(S.suspect).encode()).hexdigest()
    with open(os.path.join(HERE, 'ref', 'd5f_score.json'), 'w') as f:
        json.dump(summ, f, indent=1)
    print(json.dumps({k: v for k, v in summ.items() if not isinstance(v, list)}))
    print('off divergent:', summ['off_divergent'])
    print('strict divergent:', summ['strict_divergent'])


if __name__ == '__main__':
    main()
