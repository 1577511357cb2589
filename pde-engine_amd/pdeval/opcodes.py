"""Opcode numbers of the candidate-program format; mirror of ``include/pdeval.h``.

``tests/test_abi.py`` parses the header and checks every value here against it.
"""

PDOP = dict(
    HEADER=0,
    PUSH_X=1, PUSH_Y=2, PUSH_C=3,
    ADD=4, SUB=5, RSUB=6, MUL=7, DIV=8, RDIV=9,
    ADDC=10, MULC=11, RDIVC=12, NEG=13,
    ADD_X=14, ADD_Y=15, MUL_X=16, MUL_Y=17, SUB_X=18, SUB_Y=19,
    POWN=20, POW=21, EXP=22, LOG=23, ABS=24, SQRT=25,
    DIV_X=26, DIV_Y=27, PUSH_I=28,
    PUSH_P=29, ADD_P=30, SUB_P=31, MUL_P=32, DIV_P=33, RDIV_P=34, UNSUPPORTED=254,
)
OP_NAME = {v: k for k, v in PDOP.items()}
HAS_IMM = {PDOP['PUSH_C'], PDOP['ADDC'], PDOP['MULC'], PDOP['RDIVC'], PDOP['POW']}
# bit 8 of an immediate-carrying opcode word: a double-double low part (2 more words) follows
IMM_DD = 1 << 8
# bit 9: the immediate is one of the problem's constants (Kerr M, a): descriptor word, then 0
IMM_PRM = 1 << 9
# descriptor: bits 0-2 {M, a, 1/M, 1/a, M^2, a^2, 1/M^2, 1/a^2} (index ^ 2: the reciprocal,
# index + 4: the square), bit 3: negated
PRM_M, PRM_A, PRM_INV_M, PRM_INV_A, PRM_M2, PRM_A2, PRM_NEG = 0, 1, 2, 3, 4, 5, 8
PRM_NAME = {0: 'M', 1: 'a', 2: '1/M', 3: '1/a', 4: 'M**2', 5: 'a**2', 6: '1/M**2', 7: '1/a**2'}


def op_len(word: int) -> int:
    """Words taken by the opcode `word` and its immediate(s)."""
    if (word & 0xff) in HAS_IMM:
        return 5 if word & IMM_DD else 3
    return 1
# opcodes whose operand (bits 8-23) is a coordinate power v**n: n in bits 8-15, axis in bit 16
P_OPS = {PDOP[k] for k in ('PUSH_P', 'ADD_P', 'SUB_P', 'MUL_P', 'DIV_P', 'RDIV_P')}

PROBLEM_FORCE_FREE = 0
PROBLEM_KERR = 1

# per-candidate classes (status[] output)
CLS_ACCEPT = 0
CLS_REJECT_POINT = 1
CLS_REJECT_GRID = 2
CLS_ZERO_GRADIENT = 3
CLS_NONFINITE_REF = 4
CLS_UNSUPPORTED = 5
CLS_BAD_PROGRAM = 6
CLS_REJECT_SYMBOLIC = 7
CLS_NAME = {0: 'accept', 1: 'reject_point', 2: 'reject_grid', 3: 'zero_gradient',
            4: 'nonfinite_ref', 5: 'unsupported', 6: 'bad_program', 7: 'reject_symbolic'}

MAX_STACK = 8
FP_N = 4
FLAG_COMPLEX = 1 << 16   # header flag: program pushes the imaginary unit
FLAG_NOCOORD = 1 << 17   # header flag: program references no coordinate
FLAG_RATIONAL = 1 << 18  # header flag: value is rational at rational points (exact det)
FLAG_NONSMOOTH2D = 1 << 19  # header flag: contains Abs and references both coordinates
FLAG_UNPROVABLE = 1 << 20   # header flag: u = c*exp(g)**(p/4), p > 0 (pdeval.h)
