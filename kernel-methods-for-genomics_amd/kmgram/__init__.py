"""kmgram — MI355X-native string-kernel Gram engine (host side).

Python host layer over libkmgram.so (hand-written HIP kernels for gfx950, C ABI in
include/kmgram.h).  ``kernels.py`` next to this package is the drop-in mirror of the
reference module; ``Kernel`` below is constructor/evaluate sugar over the same
method-string grammar.
"""
from . import _lib
from .engine import GramEngine, default_engine
from .params import beta, delta, mismatch_weights

__all__ = ["GramEngine", "default_engine", "Kernel", "beta", "delta", "mismatch_weights"]


class Kernel:
    """``Kernel('MM_k5_m1').evaluate(X)`` == ``kernels.select_method(X, 'MM_k5_m1')``."""

    def __init__(self, method):
        self.method = method

    def evaluate(self, X):
        import kernels  # the drop-in module (this directory on sys.path)
        return kernels.select_method(X, self.method)

    def __repr__(self):
        return f"Kernel({self.method!r})"
