import os
import sys

import pytest

# torch first: its bundled HIP runtime must be the one the process loads before libpdeval.so
# (which then binds to the already-loaded libamdhip64 of the same soname); the GPU tests that
# hand torch device buffers to the C ABI need torch to see the GPUs
import torch  # noqa: E402,F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'pde-engine_amd'), os.path.join(ROOT, 'tests'), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libpdeval.so)')
    config.addinivalue_line('markers', 'slow: long CPU test')
