#!/usr/bin/env python3
"""Fixture generator (runs ONLY in the build container, never on the GPU box).

Drives the reference's own enumerator
``lean_normalizer/lean_bridge_fixed.py:113-215`` (``FastExpressionGenerator.stream_generate``)
with the problem plugin's primitives / ops (``problems/__init__.py:66-108, 259-302``) exactly
as the driver does (``general_method_paper_reproduction.py:1413-1421``: ``batch_size=2000``,
``binary_ops=all_binary_ops``, ``prune=True``), and writes the streamed candidate strings, in
stream order, as data fixtures:

    tests/golden/streams/<problem>_d<D>.txt.gz      one line per candidate: "<depth>\t<expr>"

The only change to the reference's behaviour is speed: the per-string normalizer
(``lean_bridge.py:67-78``, a pure SymPy function) is mapped over a process pool instead of a
loop; ``normalize_batch``'s result layout (``lean_bridge_fixed.py:42-68``: normalized string +
``sha256(normalized)[:16]`` signature) is reproduced around it so the enumerator's dedupe is
unchanged.  The reference is imported from a scratch copy (``--ref``), because the mount is
read-only and its constructors open SQLite caches.  No reference code is copied into the repo.
"""
import argparse
import gzip
import hashlib
import multiprocessing as mp
import os
import shutil
import sys
import time

_NORM = None


def _norm(s):
    return _NORM.normalize(s)


def make_scratch_copy(ref_src, dst):
    if os.path.isdir(dst):
        return dst
    for root, _dirs, files in os.walk(ref_src):
        for f in files:
            if f.endswith('.py'):
                rel = os.path.relpath(os.path.join(root, f), ref_src)
                os.makedirs(os.path.join(dst, os.path.dirname(rel)), exist_ok=True)
                shutil.copy(os.path.join(root, f), os.path.join(dst, rel))
    for p in ('problems/force_free/outputs', 'problems/kerr_magnetosphere/outputs'):
        os.makedirs(os.path.join(dst, p), exist_ok=True)
    return dst


class PoolNormalizer:
    """normalize_batch() with the reference's result layout, normalize() mapped over a pool."""

    def __init__(self, pool):
        self.pool = pool

    def normalize_batch(self, batch):
        strs = [s for s, _ in batch]
        outs = self.pool.map(_norm, strs, chunksize=max(1, len(strs) // (8 * os.cpu_count())))
        res = []
        for (s, idx), n in zip(batch, outs):
            res.append({'normalized': n, 'index': idx,
                        'signature': hashlib.sha256(n.encode()).hexdigest()[:16]})
        return res


def main():
    global _NORM
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/tmp/refcopy')
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--max-depth', type=int, default=3)
    ap.add_argument('--procs', type=int, default=os.cpu_count())
    ap.add_argument('--out', default=os.path.join(os.path.dirname(__file__), 'streams'))
    a = ap.parse_args()
    make_scratch_copy('/root/reference', a.ref)
    os.chdir(a.ref)
    sys.path.insert(0, a.ref)
    from problems import load_problem                       # noqa: E402  (reference)
    from lean_normalizer.lean_bridge import LeanNormalizer  # noqa: E402  (reference)
    from lean_normalizer.lean_bridge_fixed import FastExpressionGenerator  # noqa: E402
    prob = load_problem(a.problem)
    _NORM = LeanNormalizer()
    out = []
    t0 = time.time()
    with mp.get_context('fork').Pool(a.procs) as pool:
        gen = FastExpressionGenerator(normalizer=PoolNormalizer(pool))

        def on_batch(depth, exprs):
            out.extend((depth, e) for e in exprs)
            print(f'[stream] depth {depth}: +{len(exprs)} (total {len(out)}) {time.time()-t0:.0f}s',
                  flush=True)
        gen.stream_generate(primitives=prob.primitives, unary_ops=prob.unary_ops,
                            binary_ops=prob.all_binary_ops, max_depth=a.max_depth,
                            batch_size=2000, on_batch=on_batch, prune=True)
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, f'{prob.slug}_d{a.max_depth}.txt.gz')
    with gzip.open(path, 'wt') as f:
        for d, e in out:
            f.write(f'{d}\t{e}\n')
    print(f'wrote {len(out)} candidates to {path} in {time.time()-t0:.0f}s')


if __name__ == '__main__':
    main()
