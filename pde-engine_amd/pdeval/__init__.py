"""pdeval -- MI355X-native candidate validator for the pde-engine discovery pipeline.

Host side: flattener (SymPy -> postfix jet programs), ctypes binding of libpdeval.so,
batch validation with the reference's verdict semantics, worker pool and multi-GPU sharding.
"""
from .opcodes import *  # noqa: F401,F403
