"""The decode pass's negation folding (csrc/pdeval_grid.h decode_kernel, PD_FOLD_NEG), restated
on the CPU and checked with the oracle's arithmetic.

The decoder drops NEG opcodes and tracks a sign per stack slot instead: ADDC c becomes ADDC -c
under a negative sign, ADD_X/SUB_X, ADD_Y/SUB_Y and ADD_P/SUB_P swap, a sum of two signed
operands becomes ADD, SUB or RSUB with a sign, products and quotients multiply the signs, an
even POWN or ABS clears it; programs whose folded sign would reach EXP, LOG, SQRT or POW keep
their NEGs.  The claims the device relies on are checked here on the depth-4 workload's
programs, bit for bit in the oracle's double arithmetic:
  * every jet coefficient of the folded program is the original's times the final sign;
  * the force-free residual and its scale are the same (the determinant is even in u).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from pdeval.opcodes import FLAG_COMPLEX, IMM_PRM, PDOP, op_len

_PUSH = {PDOP[k] for k in ('PUSH_X', 'PUSH_Y', 'PUSH_C', 'PUSH_P', 'PUSH_I')}
_BIN = {PDOP[k] for k in ('ADD', 'SUB', 'RSUB', 'MUL', 'DIV', 'RDIV')}
_NEEDS_VALUE = {PDOP[k] for k in ('EXP', 'LOG', 'SQRT', 'POW')}
_SWAP = {PDOP['ADD_X']: PDOP['SUB_X'], PDOP['SUB_X']: PDOP['ADD_X'], PDOP['ADD_Y']: PDOP['SUB_Y'],
         PDOP['SUB_Y']: PDOP['ADD_Y'], PDOP['ADD_P']: PDOP['SUB_P'], PDOP['SUB_P']: PDOP['ADD_P']}


def fold(words):
    """(folded words, final sign), or None when a folded sign would reach a composition."""
    w = [int(v) for v in words]
    out = [w[0]]
    sg = [1] * 5
    d = 0
    i = 1
    while i < len(w):
        word = w[i] & 0xffffffff
        op = word & 0xff
        n = op_len(word)
        body = w[i:i + n]
        if op in _PUSH:
            d += 1
            sg[d] = 1
        elif op in _BIN:
            d -= 1
            sl, sa = sg[d], sg[d + 1]
            if op in (PDOP['MUL'], PDOP['DIV'], PDOP['RDIV']):
                sg[d] = sl * sa
            elif sl == sa:
                sg[d] = sa
            elif op == PDOP['ADD']:
                body = [(word & ~0xff) | (PDOP['SUB'] if sl > 0 else PDOP['RSUB'])]
                sg[d] = 1
            elif op == PDOP['SUB']:
                body = [(word & ~0xff) | PDOP['ADD']]
                sg[d] = sl
            else:
                body = [(word & ~0xff) | PDOP['ADD']]
                sg[d] = sa
        elif op == PDOP['NEG']:
            sg[d] = -sg[d]
            i += n
            continue
        elif sg[d] < 0:
            if op == PDOP['ADDC']:
                if word & IMM_PRM:
                    return None
                imm = np.array(body[1:], dtype=np.int32).view(np.float64) * -1.0
                body = [word] + imm.view(np.int32).tolist()
            elif op in _SWAP:
                body = [(word & ~0xff) | _SWAP[op]]
            elif op == PDOP['ABS'] or (op == PDOP['POWN'] and not ((word >> 8) & 0xff) & 1):
                sg[d] = 1
            elif op in _NEEDS_VALUE:
                return None
        out.extend(int(np.int32(np.uint32(v & 0xffffffff))) for v in body)
        i += n
    return np.array(out, dtype=np.int32), sg[1]


def _programs(n, name='force_free_d4_validated'):
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'data', name + '.npz'))
    ops, off = d['ops'], d['offsets']
    rng = np.random.default_rng(1)
    idx = rng.choice(len(off) - 1, n, replace=False)
    return [ops[off[i]:off[i + 1]] for i in idx]


@pytest.mark.parametrize('pid,name,pts', [
    (0, 'force_free_d4_validated', ((0.8, 6 / 7), (1.37, -0.61))),
    (1, 'kerr_magnetosphere_d4_stream', ((3.1, 0.3), (5.7, -0.45)))])
def test_fold_keeps_every_coefficient_up_to_the_sign(pid, name, pts):
    """Kerr: the residual is linear in u, so |L[u]| and its scale are unchanged as well."""
    progs = [p for p in _programs(4000, name) if any((int(v) & 0xff) == PDOP['NEG'] for v in p[1:])]
    folded = 0
    for p in progs:
        f = fold(p)
        if f is None:
            continue
        words, s = f
        cx = bool(int(p[0]) & FLAG_COMPLEX)
        for (x, y) in pts:
            a = O.jet(pid, p, x, y, cx)
            b = O.jet(pid, words, x, y, cx)
            fin = np.isfinite(a)
            assert np.array_equal(b[fin], s * a[fin]), (p, words)
            ra, rb = O.point(pid, p, x, y, cx), O.point(pid, words, x, y, cx)
            if np.isfinite(ra[0]):
                assert ra[0] == rb[0] and ra[1] == rb[1]      # |residual| and scale, bit for bit
        folded += 1
    assert folded > 0.5 * len(progs) and folded > 100, (folded, len(progs))
