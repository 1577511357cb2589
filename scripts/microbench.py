#!/usr/bin/env python3
"""Per-opcode cost model of the pass-1 kernel on the GPU: batches of one repeated program,
pass times from the library's events.
Usage: python scripts/microbench.py [--n N] [--problem force_free|kerr_magnetosphere]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))

PROGS = ['rho', 'rho*z', 'rho*z*z', 'rho**2*z', 'rho/z', 'rho + z**2', 'exp(rho*z)', 'sqrt(rho + z**2)',
         'rho**3*z**2', '(rho + z)*(rho - z)', '(rho + z)/(rho - z + 3)', 'exp(rho)*sqrt(z + 3)',
         'rho**2/(rho**2 + z**2)**(3/2)']
KERR_PROGS = ['r', 'x', 'r*x', 'r + x', 'r*x*x', 'r*x + r', '-r + 3', '3*r*x', 'r/x', 'x/(r + 3)', 'exp(r*x)',
              'exp(-r)*x', 'sqrt(r + x)', '(r + x)**(3/2)', '(r + x)**(-3/2)', 'log(r + x)', 'r**2*x', 'r**3*x',
              'exp(r)*exp(x)', '(r + 2)*(x + 3)', 'M*r + a*x']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 18)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--problem', default='force_free')
    a = ap.parse_args()
    import torch
    from pdeval import _lib, problem_defs as P
    from pdeval.opcodes import FP_N
    from pdeval.flatten import disasm
    pd_ = P.get(a.problem)
    ctx = _lib.Context(pd_.problem_id)
    dev = torch.device('cuda:0')
    stream = torch.cuda.Stream(dev)
    n = a.n
    outs = [torch.zeros(s, dtype=t, device=dev) for s, t in
            ((((n + 31) // 32) * 4, torch.uint8), (n, torch.uint8), (n, torch.float64), (n, torch.float64),
             (n * ctx.n_ref, torch.float64), (n, torch.int32), (n, torch.int32), (n * FP_N, torch.float64))]
    d_out = _lib.Outputs(*[o.data_ptr() for o in outs])
    prm = _lib.default_params(pd_.problem_id)
    ctx.set_timing(True)
    for s in (PROGS if pd_.problem_id == 0 else KERR_PROGS):
        w = np.array(pd_.compile(pd_.parse(s)), dtype=np.int32)
        ops = np.tile(w, n)
        off = np.arange(n + 1, dtype=np.int64) * len(w)
        d_ops = torch.from_numpy(ops).to(dev)
        d_off = torch.from_numpy(off).to(dev)
        torch.cuda.synchronize()
        best = None
        for _ in range(a.reps):
            ctx.validate_device(d_ops.data_ptr(), d_ops.numel(), d_off.data_ptr(), n, d_out, prm,
                                stream.cuda_stream, True)
            t = ctx.pass_times()
            best = t if best is None or t['pass1_stack2'] < best['pass1_stack2'] else best
        ops_s = ' '.join(l.split()[0] for l in disasm(w.tolist()).split('\n')[1:])
        ns = best['pass1_stack2'] * 1e6 / n
        print(f'{s:34s} pass1 {best["pass1_stack2"]:8.3f} ms  {ns:7.2f} ns/cand  [{ops_s}]', flush=True)


if __name__ == '__main__':
    main()
