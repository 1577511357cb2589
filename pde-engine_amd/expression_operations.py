"""Operation vocabulary of the candidate generator (the input alphabet of the validator).

Same names and semantics as the reference's ``expression_operations.py:11-106`` (which the
driver maps into ``sympify``'s locals, ``general_method_paper_reproduction.py:84-93``, so that
strings such as ``exp_neg(z)`` or ``pow_3_2(rho)`` parse into real SymPy operations).  The
functions are module level so they pickle for ``multiprocessing``.
"""
import sympy as sp

_HALF3 = sp.Rational(3, 2)


def op_neg(a):
    return -a


def op_inv(a):
    return 1 / a


def op_sqrt(a):
    return sp.sqrt(a)


def op_square(a):
    return a ** 2


def op_pow_3_2(a):
    return a ** _HALF3


def op_pow_neg_3_2(a):
    return a ** (-_HALF3)


def op_exp(a):
    return sp.exp(a)


def op_exp_neg(a):
    return sp.exp(-a)


def op_add(a, b):
    return a + b


def op_sub(a, b):
    return a - b


def op_mul(a, b):
    return a * b


def op_div(a, b):
    return a / b


def op_geom_sum(a, b):
    return a / (1 - b)


def op_sqrt_shift_neg(a, b):
    return sp.sqrt((a - 1) ** 2 + b ** 2)


def op_sqrt_shift_pos(a, b):
    return sp.sqrt((a + 1) ** 2 + b ** 2)


def op_exp_mul(a, b):
    return a * sp.exp(b)


def op_log_mul(a, b):
    return a * sp.log(b)


UNARY_OPS = {name: globals()['op_' + name] for name in
             ('neg', 'inv', 'sqrt', 'square', 'pow_3_2', 'pow_neg_3_2', 'exp', 'exp_neg')}
BINARY_OPS = {name: globals()['op_' + name] for name in ('add', 'sub', 'mul', 'div', 'geom_sum')}
SPECIAL_OPS = {name: globals()['op_' + name] for name in
               ('sqrt_shift_neg', 'sqrt_shift_pos', 'exp_mul', 'log_mul')}
ALL_BINARY_OPS = {**BINARY_OPS, **SPECIAL_OPS}
