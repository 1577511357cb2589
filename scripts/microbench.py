#!/usr/bin/env python3
"""Per-opcode cost model of the pass-1 kernel on the GPU: batches of one repeated program,
pass times from the library's events.
Usage: python scripts/microbench.py [--n N] [--problem force_free|kerr_magnetosphere] [--set calib]

--set calib: one program per opcode the FLOP model prices (scripts/flop_calib.py turns their
PMC FP64 counts, scripts/gpu_pmc_micro.sh, into the executed-flop table of the model)."""
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

# one opcode each on top of a base program of both coordinates (no hoisted prefix: the first
# opcodes already mix x and y); the base programs themselves come first
CALIB_FF = ['rho', 'z', 'rho*z', 'rho + z', 'rho - z', '3*rho*z', 'rho*z + 3', 'rho/z', 'z/rho',
            '(rho + z)*(rho - z)', '(rho + z)/(rho - z + 7)', '(rho + z) - (rho*z + 7)',
            'exp(rho*z)', 'sqrt(rho*z + 7)', 'log(rho*z + 7)', '(rho*z + 7)**(3/2)', '(rho*z + 7)**(-3/2)',
            '(rho*z + 7)**(1/4)', '(rho*z)**2', '(rho*z)**3', '(rho*z)**4', '(rho*z)**5', '(rho*z)**7',
            'rho**2*z', 'rho + z**2', 'rho*z + rho**2', 'rho*z - rho**3', 'rho*z/rho**2', 'rho**2/(rho*z + 7)',
            'rho**3*z**2', 'Abs(rho*z - 1)', '3/(rho*z + 7)', 'z*rho + z**2',
            '(rho*z + 7)**2', '(rho*z + 7)**3', '(rho*z + 7)**4', '(rho*z + 7)**5', '(rho*z + 7)**7',
            'z/(rho*z + 7)', 'rho**2*z + rho*z']
CALIB_KERR = ['r', 'x', 'r*x', 'r + x', 'r - x', '3*r*x', 'r*x + 3', 'r/x', 'x/r', '(r + x)*(r - x)',
              '(r + x)/(r - x + 7)', '(r + x) - (r*x + 7)', 'exp(r*x)', 'sqrt(r*x + 7)', 'log(r*x + 7)',
              '(r*x + 7)**(3/2)', '(r*x + 7)**(-3/2)', '(r*x + 7)**(1/4)', '(r*x)**2', '(r*x)**3', '(r*x)**4',
              '(r*x)**5', '(r*x)**7', 'r**2*x', 'r + x**2', 'r*x + r**2', 'r*x - r**3', 'r*x/r**2',
              'r**2/(r*x + 7)', 'r**3*x**2', 'Abs(r*x - 1)', '3/(r*x + 7)', 'x*r + x**2', 'M*r*x', 'a*r*x',
              '(r*x + 7)**2', '(r*x + 7)**3', '(r*x + 7)**4', '(r*x + 7)**5', '(r*x + 7)**7',
              'x/(r*x + 7)', 'r**2*x + r*x']


def programs(problem_id: int, which: str):
    if which == 'calib':
        return CALIB_FF if problem_id == 0 else CALIB_KERR
    return PROGS if problem_id == 0 else KERR_PROGS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1 << 18)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--set', default='default', choices=['default', 'calib'])
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
    # by field name (round 6: the positional list passed an n-double buffer as res_ref, which
    # holds n x n_ref -- Kerr's 3 reference points wrote past it and faulted the GPU)
    outs = {'verdict_bits': torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device=dev),
            'status': torch.zeros(n, dtype=torch.uint8, device=dev),
            'q_ref': torch.zeros(n, dtype=torch.float64, device=dev),
            'res_ref': torch.zeros(n * ctx.n_ref, dtype=torch.float64, device=dev),
            'q_grid': torch.zeros(n, dtype=torch.float64, device=dev),
            'n_bad': torch.zeros(n, dtype=torch.int32, device=dev),
            'n_nonfinite': torch.zeros(n, dtype=torch.int32, device=dev),
            'fingerprint': torch.zeros(n * FP_N, dtype=torch.float64, device=dev)}
    assert set(outs) == {f for f, _ in _lib.Outputs._fields_}
    d_out = _lib.Outputs(*[outs[f].data_ptr() for f, _ in _lib.Outputs._fields_])
    prm = _lib.default_params(pd_.problem_id)
    ctx.set_timing(True)
    for s in programs(pd_.problem_id, a.set):
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
