#!/usr/bin/env python3
"""Seeded depth-5 force-free candidate strings for reference-verdict fixtures (no reference import).

The depth-5 stream (configs[3]) is not enumerable here (~12.4 M candidates to normalize, SURVEY
§8d), so the reference's symbolic stage beyond depth 4 is probed on candidates of the same
grammar instead: one more operation on top of the depth-4 candidates that reach ``validate``
(``streams/force_free_d4_validated.txt.gz``) --
  * a unary op of the problem (``expression_operations.UNARY_OPS``) on a depth-4 candidate;
  * a binary op (``BINARY_OPS``) of a depth-4 candidate and a "leaf" (``rho``, ``z``, and the
    unary ops applied to them).
This is a PROXY grammar, not the enumerator's: its binary depth is additive
(``lean_bridge_fixed.py:155-157``: ``for d1 in range(1, depth): d2 = depth - d1``, so depth 5
pairs (1,4), (2,3), (3,2), (4,1)), its depth-1 set is the five primitives
``rho, z, rho**2 + z**2, rho/z, 1`` (``problems/__init__.py:73-79``), its splices are
unparenthesised (``:166-195``), and its candidates go through ``normalize_batch``, the signature
dedupe and the pre-validate filters -- so part of this sample is depth 6 (a unary leaf is depth 2)
and the (2,3)/(3,2) pairs are absent.  The faithful sample is ``gen_d5_faithful.py``; this one
stays as a further stress set of the same vocabulary (``ref/ff_d5_s*.jsonl``).
Strings are written as the stream writes them: unary ops by name (``sqrt(<a>)``; the driver's
``sympify`` locals hold the unary ops, ``general_method_paper_reproduction.py:1703-1712``) and
binary ops as SymPy infix (``geom_sum(a, b)`` = ``a/(1 - b)``, ``expression_operations.py``).  Output: ``tests/golden/streams/force_free_d5_sample.txt.gz`` ("5\\t<expr>" per line),
the input of ``gen_reference_verdicts.py verdicts`` (-> ``ref/ff_d5_s<N>.jsonl``).
"""
import gzip
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
UNARY = ('neg', 'inv', 'sqrt', 'square', 'pow_3_2', 'pow_neg_3_2', 'exp', 'exp_neg')
INFIX = {'add': '({a}) + ({b})', 'sub': '({a}) - ({b})', 'mul': '({a})*({b})', 'div': '({a})/({b})',
         'geom_sum': '({a})/(1 - ({b}))'}


def main():
    with gzip.open(os.path.join(HERE, 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        d4 = [l.rstrip('\n').split('\t')[2] for l in f]
    leaves = ['rho', 'z'] + [f'{u}({v})' for u in UNARY for v in ('rho', 'z')]
    rng = random.Random(0)
    out, seen = [], set()
    while len(out) < N:
        a = rng.choice(d4)
        if rng.random() < 0.6:
            s = f'{rng.choice(UNARY)}({a})'
        else:
            op = rng.choice(sorted(INFIX))
            b = rng.choice(leaves)
            if rng.random() < 0.5:
                a, b = b, a
            s = INFIX[op].format(a=a, b=b)
        if s not in seen:
            seen.add(s)
            out.append(s)
    path = os.path.join(HERE, 'streams', 'force_free_d5_sample.txt.gz')
    with gzip.open(path, 'wt') as f:
        for s in out:
            f.write(f'5\t{s}\n')
    print(f'wrote {len(out)} depth-5 strings to {path}')


if __name__ == '__main__':
    main()
