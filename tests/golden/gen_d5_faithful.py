#!/usr/bin/env python3
"""Depth-5 force-free parity sample built by the reference's own enumerator rules
(runs ONLY in the build container, never on the GPU box; imports the reference from a scratch
copy exactly as ``gen_streams.py`` / ``gen_reference_verdicts.py`` do).

configs[3] is ``--max-depth 5``.  Its stream (~12 M candidates to normalize) is not enumerated
here, so this script draws a seeded sample from the exact depth-5 CANDIDATE list and sends it
through the same stages the driver applies before ``validate``:

1. Candidate list (restated from ``lean_normalizer/lean_bridge_fixed.py:139-195``, fed with the
   committed depth-1..4 stream ``streams/force_free_d4.txt.gz``):
   * unary ops (``UNARY_OPS`` order, ``expression_operations.py:80-89``) on every depth-4 string,
     with the ``inv(inv(..))`` / constant-``1`` pruning of ``:142-153``;
   * binary ops over every additive depth split ``d1 + d2 = 5`` -- (1,4), (2,3), (3,2), (4,1)
     (``:155-158``) -- in ``ALL_BINARY_OPS`` order, the constant x constant pruning, the
     ``a > b`` swap for ``add`` / ``mul``, the a-a / x1 / /1 / a/a / 1-1 pruning and the
     UNPARENTHESISED splices ``({a} + {b})``, ``({a} - {b})``, ``({a} * {b})``,
     ``({a} / ({b}))``, ``({a} / (1 - {b}))`` (``:166-195``; the special ops of
     ``ALL_BINARY_OPS`` have no branch and emit nothing).
   The restatement is checked first: fed with the committed depth-1..3 stream it reproduces the
   reference's depth-2/3/4 candidate counts 128 / 5,924 / 258,285.
2. ``normalize_batch`` (``lean_bridge_fixed.py:42-68``): the reference's ``LeanNormalizer.normalize``
   (``lean_bridge.py:67-112``) on each sampled candidate; the 16-hex signature dedupe
   (``:204-210``) against every depth-2..4 normalized form of the committed stream (the
   enumerator's ``seen_signatures``; depth-1 primitives are never added to it, ``:129-137``) and
   within the sample in candidate order.
3. The driver's pre-validate filters (``general_method_paper_reproduction.py:1253-1294``, the
   same code path as ``gen_reference_verdicts.py filters``): degenerate denominators, the
   run-wide ``UNIQUE(str(simplify(expand(sympify(s)))))`` insert and the constant-only skip.
   The UNIQUE key of a depth-5 row is compared with the keys of the depth-1..4 rows that reach
   ``validate`` (``streams/force_free_d4_validated.txt.gz``) through a numeric pre-match: two
   rows with equal keys are the same function, so only depth-1..4 rows whose value at two fixed
   points agrees with the depth-5 row (rel. 1e-9) have their key computed and compared.
   Rows that the bounded normalize / key simplify could not finish keep their own string (as
   the reference does on an exception) and are counted.

The sample is uniform over CANDIDATES, so a normalized form is drawn with weight equal to the
number of candidate strings that produce it (the stream keeps it once); the counts of every
stage go to ``streams/force_free_d5_faithful.json``.

Output: ``streams/force_free_d5_faithful.txt.gz`` ("<candidate idx>\\t5\\t<expr>"), the input of
``gen_reference_verdicts.py verdicts --timeout 20`` (-> ``ref/ff_d5f_*.jsonl``).
"""
import argparse
import gzip
import json
import multiprocessing as mp
import os
import random
import signal
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

UNARY = ('neg', 'inv', 'sqrt', 'square', 'pow_3_2', 'pow_neg_3_2', 'exp', 'exp_neg')
BINARY = ('add', 'sub', 'mul', 'div', 'geom_sum',
          'sqrt_shift_neg', 'sqrt_shift_pos', 'exp_mul', 'log_mul')   # ALL_BINARY_OPS order


def _has_vars(s):
    return ('r' in s) or ('x' in s) or ('rho' in s) or ('z' in s)


def candidates(by_depth, depth):
    """Yield the depth-``depth`` candidate strings in the enumerator's order (prune=True)."""
    for e in by_depth[depth - 1]:
        if not _has_vars(e):
            continue
        for op in UNARY:
            if op == 'inv' and e.startswith('inv('):
                continue
            if op in ('sqrt', 'square', 'pow_3_2', 'pow_neg_3_2') and e == '1':
                continue
            yield f'{op}({e})'
    for d1 in range(1, depth):
        d2 = depth - d1
        if d2 < 1 or d2 >= depth:
            continue
        for e1 in by_depth[d1]:
            v1 = _has_vars(e1)
            for e2 in by_depth[d2]:
                if not v1 and not _has_vars(e2):
                    continue
                for op in BINARY:
                    a, b = e1, e2
                    if op in ('add', 'mul') and a > b:
                        a, b = b, a
                    if op == 'add':
                        yield f'({a} + {b})'
                    elif op == 'sub':
                        if a != b:
                            yield f'({a} - {b})'
                    elif op == 'mul':
                        if a != '1' and b != '1':
                            yield f'({a} * {b})'
                    elif op == 'div':
                        if b != '1' and a != b:
                            yield f'({a} / ({b}))'
                    elif op == 'geom_sum':
                        if b != '1':
                            yield f'({a} / (1 - {b}))'


class _Timeout(BaseException):
    pass


def _alarm(_s, _f):
    raise _Timeout()


_NORM = None
_D = None
_LIMIT = 60
PTS = (('0.731', '0.412'), ('1.37', '-0.583'))


def _init(ref):
    global _NORM, _D
    os.chdir(ref)
    sys.path.insert(0, ref)
    from lean_normalizer.lean_bridge import LeanNormalizer          # noqa: E402  (reference)
    from general_method_paper_reproduction import GeneralFoliationDiscovery  # noqa: E402
    _NORM = LeanNormalizer()
    _D = GeneralFoliationDiscovery(use_lean_normalizer=False, problem_name='force_free',
                                   mode='parallel')
    signal.signal(signal.SIGALRM, _alarm)


def _normalize(item):
    i, s = item
    signal.alarm(_LIMIT)
    try:
        return i, _NORM.normalize(s), False
    except _Timeout:
        return i, s, True
    finally:
        signal.alarm(0)


def _fingerprint(s):
    """Values at two fixed points (complex; None where not finite) of the locals parse."""
    import sympy as sp
    signal.alarm(_LIMIT)
    try:
        u = sp.sympify(s, locals=_D._sympify_locals)
        rho, z = _D.problem.symbols['rho'], _D.problem.symbols['z']
        out = []
        for pr, pz in PTS:
            try:
                v = complex(u.evalf(30, subs={rho: sp.Rational(pr), z: sp.Rational(pz)}))
                out.append(v if (v == v and abs(v) < 1e300) else None)
            except Exception:
                out.append(None)
        return out
    except _Timeout:
        return [None, None]
    except Exception:
        return [None, None]
    finally:
        signal.alarm(0)


def _fp_item(item):
    return item[0], _fingerprint(item[1])


def _key(item):
    """The driver's UNIQUE key str(simplify(expand(sympify(s)))) (``:1277-1280``), bounded."""
    import sympy as sp
    i, s = item
    signal.alarm(_LIMIT)
    try:
        return i, str(sp.simplify(sp.expand(sp.sympify(s)))), False
    except _Timeout:
        return i, s, True
    except Exception:
        return i, s, False
    finally:
        signal.alarm(0)


def check_counts(by_depth):
    got = {d: sum(1 for _ in candidates(by_depth, d)) for d in (2, 3, 4)}
    want = {2: 128, 3: 5924, 4: 258285}
    assert got == want, (got, want)
    return got


def main():
    global _LIMIT
    import numpy as np
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/tmp/refcopy')
    ap.add_argument('--sample', type=int, default=12000, help='depth-5 candidates drawn')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--procs', type=int, default=6)
    ap.add_argument('--limit', type=int, default=60, help='bound per normalize / key (s)')
    a = ap.parse_args()
    _LIMIT = a.limit
    from gen_streams import make_scratch_copy
    from gen_reference_verdicts import _filter_one, _init_worker
    make_scratch_copy('/root/reference', a.ref)
    t0 = time.time()
    by_depth = {d: [] for d in range(1, 5)}
    with gzip.open(os.path.join(HERE, 'streams', 'force_free_d4.txt.gz'), 'rt') as f:
        for line in f:
            d, e = line.rstrip('\n').split('\t', 1)
            by_depth[int(d)].append(e)
    stats = {'candidate_counts_d2_d4': check_counts(by_depth)}
    n5 = sum(1 for _ in candidates(by_depth, 5))
    stats['candidates_d5'] = n5
    pick = sorted(random.Random(a.seed).sample(range(n5), a.sample))
    want, sample = set(pick), []
    for i, s in enumerate(candidates(by_depth, 5)):
        if i in want:
            sample.append((i, s))
    print(f'[d5] {n5} candidates, sampled {len(sample)} ({time.time()-t0:.0f}s)', flush=True)

    ctx = mp.get_context('fork')
    with ctx.Pool(a.procs, _init, (a.ref,)) as pool:
        norm = dict((i, (n, to)) for i, n, to in pool.imap_unordered(_normalize, sample, chunksize=8))
    stats['normalize_timeouts'] = sum(1 for n, to in norm.values() if to)
    stream4 = set(e for d in (2, 3, 4) for e in by_depth[d])
    seen = set()
    streamed = []
    dup_d4 = dup_d5 = 0
    for i, _s in sample:                      # stream order within depth 5
        n = norm[i][0]
        if n in stream4:
            dup_d4 += 1
            continue
        if n in seen:
            dup_d5 += 1
            continue
        seen.add(n)
        streamed.append((i, n))
    stats.update(signature_dup_of_d2_d4=dup_d4, signature_dup_in_sample=dup_d5,
                 streamed=len(streamed))
    print(f'[d5] normalized: {len(streamed)} streamed ({time.time()-t0:.0f}s)', flush=True)

    with ctx.Pool(a.procs, _init_worker, (a.ref, 'force_free')) as pool:
        filt = list(pool.imap(_filter_one, [(i, 5, n) for i, n in streamed], chunksize=4))
    stats['degenerate'] = sum(1 for r in filt if r['degenerate'])
    stats['key_simplify_timeouts'] = sum(1 for r in filt if r.get('simplify_timeout'))
    print(f'[d5] filters done ({time.time()-t0:.0f}s)', flush=True)

    # run-wide UNIQUE key against the depth-1..4 rows that reach validate
    with gzip.open(os.path.join(HERE, 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        d4v = [l.rstrip('\n').split('\t')[2] for l in f]
    live = [r for r in filt if not r['degenerate']]
    with ctx.Pool(a.procs, _init, (a.ref,)) as pool:
        fp4 = [fp for _i, fp in pool.imap(_fp_item, list(enumerate(d4v)), chunksize=64)]
        fp5 = dict(pool.imap_unordered(_fp_item, [(r['idx'], r['expr']) for r in live], chunksize=4))
        print(f'[d5] fingerprints done ({time.time()-t0:.0f}s)', flush=True)
        arr = np.array([[(v if v is not None else complex('nan')) for v in fp] for fp in fp4])
        cand = {}
        for r in live:
            f5 = fp5[r['idx']]
            m = np.ones(len(d4v), bool)
            for k in range(2):
                col = arr[:, k]
                if f5[k] is None:
                    m &= np.isnan(col.real)
                else:
                    m &= np.abs(col - f5[k]) <= 1e-9 * np.maximum(1.0, np.maximum(np.abs(col), abs(f5[k])))
            hits = np.nonzero(m)[0]
            if len(hits):
                cand[r['idx']] = hits.tolist()
        need = sorted(set(j for h in cand.values() for j in h))
        stats['d4_rows_prematched'] = len(need)
        keys4 = {j: k for j, k, _to in pool.imap_unordered(_key, [(j, d4v[j]) for j in need],
                                                            chunksize=1)}
    kept, keyseen = [], set()
    dup4 = dup5 = const = 0
    for r in filt:                            # stream order
        if r['degenerate']:
            continue
        k = r['normalized']
        if k in keyseen:
            dup5 += 1
            continue
        if any(keys4.get(j) == k for j in cand.get(r['idx'], ())):
            dup4 += 1
            continue
        keyseen.add(k)
        if r['const_only']:
            const += 1
            continue
        kept.append(r)
    stats.update(unique_dup_of_d1_d4=dup4, unique_dup_in_sample=dup5, const_only=const,
                 reach_validate=len(kept), wall_s=round(time.time() - t0, 1),
                 sample=a.sample, seed=a.seed, limit_s=a.limit)
    out = os.path.join(HERE, 'streams', 'force_free_d5_faithful.txt.gz')
    with gzip.open(out, 'wt') as f:
        for r in kept:
            f.write(f"{r['idx']}\t5\t{r['expr']}\n")
    with open(os.path.join(HERE, 'streams', 'force_free_d5_faithful.json'), 'w') as f:
        json.dump(stats, f, indent=1)
    print(json.dumps(stats))


if __name__ == '__main__':
    main()
