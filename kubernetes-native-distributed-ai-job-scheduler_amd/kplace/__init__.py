"""kplace — Python binding of libkplace.so, the MI355X batch placement engine.

The product is the C-ABI library (include/kplace.h); this package only wraps
it for tests and bench.py and generates synthetic workloads.
"""
from . import _abi, synth  # noqa: F401
from ._abi import default_params  # noqa: F401
