#!/usr/bin/env python3
"""Per-call split of the inline path (the reference's --validators 0 loop calls
validator.validate(sympify(s, locals), ...) once per candidate,
general_method_paper_reproduction.py:1288-1339): sympify, the plugin's canonical key, the
compile (flatten.py on the tree, or the native compiler on str(u)), the device call
(pdeval_validate_batch: upload, launch chain, download, sync) and the host steps + reason.

Usage (GPU box): python scripts/profile_inline.py [--n 2000] [--problem force_free]
Prints one JSON line.
"""
import argparse
import gzip
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=2000)
    ap.add_argument('--problem', default='force_free')
    a = ap.parse_args()
    import numpy as np
    import sympy as sp
    from problems import load_problem
    from pdeval.batch import get_validator
    from pdeval import problem_defs as P
    from pdeval import native
    prob = load_problem(a.problem)
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    name = 'force_free_d4_validated.txt.gz' if a.problem == 'force_free' else 'kerr_magnetosphere_d3_validated.txt.gz'
    with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'streams', name), 'rt') as f:
        strs = [l.rstrip('\n').split('\t')[-1] for l in f]
    sample = random.Random(0).sample(strs, min(a.n, len(strs)))
    bv = get_validator(prob.slug)
    pd = P.get(prob.slug)
    v = prob.validator
    kw = {'check_regularity': False, 'fast_point_only': False}
    # warm
    for s in sample[:20]:
        v.validate(sp.sympify(s, locals=locs), **kw)
    t = dict(sympify=0.0, key=0.0, compile_tree=0.0, compile_native_str=0.0, device=0.0, host=0.0)
    n_nat = 0
    for s in sample:
        t0 = time.perf_counter()
        u = sp.sympify(s, locals=locs)
        t1 = time.perf_counter()
        key = str(u)
        t2 = time.perf_counter()
        ops, off, notes = P.compile_exprs(pd, [u])
        t3 = time.perf_counter()
        n_ops, n_off, st = native.compile_native(pd.problem_id, [key])
        n_nat += int(st[0] == native.COMPILE_OK)
        t4 = time.perf_counter()
        r = bv.run(ops, off)
        t5 = time.perf_counter()
        r = bv.host_steps(r, ops, off, [u])
        bv.table(r, ops, off, notes)
        t6 = time.perf_counter()
        t['sympify'] += t1 - t0
        t['key'] += t2 - t1
        t['compile_tree'] += t3 - t2
        t['compile_native_str'] += t4 - t3
        t['device'] += t5 - t4
        t['host'] += t6 - t5
    n = len(sample)
    per = {k: round(1e6 * x / n, 1) for k, x in t.items()}
    t0 = time.perf_counter()
    for s in sample:
        v.validate(sp.sympify(s, locals=locs), **kw)
    dt = time.perf_counter() - t0
    print(json.dumps({'problem': prob.slug, 'n': n, 'us_per_call': per, 'native_ok_on_str_u': n_nat,
                      'plugin_validate_cand_per_s': round(n / dt), 'plugin_us_per_call': round(1e6 * dt / n, 1)}))


if __name__ == '__main__':
    main()
