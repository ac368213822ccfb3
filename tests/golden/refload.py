"""Import the reference's Python prototype (/root/reference/code) for fixture generation.

Runs ONLY in the build container (the reference is absent on the GPU box) and
only from gen_golden.py. The reference is Python 2 code; four ordinary import /
runtime errors are bridged here, nothing in the reference's arithmetic is
replaced:

1. ``code/utils.py:5`` imports ``cvxopt`` but never uses it: an empty module is
   registered under that name.
2. ``range``/``map`` return lists in Python 2 (``utils.py:33,47,68`` assign into
   or ``np.array`` them): list-returning versions are injected into the
   module's globals.
3. ``utils.py:99`` passes float COO indices to ``csc_matrix``; SciPy 1.15 rejects
   them, so the wrapper casts the index arrays to int64 first.
4. ``sys.dont_write_bytecode`` keeps the read-only reference tree untouched.
"""
from __future__ import annotations

import builtins
import sys
import types

import numpy as np
import scipy.sparse as sp

REF_CODE = "/root/reference/code"


def load_reference():
    sys.dont_write_bytecode = True
    if "cvxopt" not in sys.modules:
        sys.modules["cvxopt"] = types.ModuleType("cvxopt")
    if REF_CODE not in sys.path:
        sys.path.insert(0, REF_CODE)
    import utils as ref_utils  # noqa: E402  (the reference's code/utils.py)

    ref_utils.range = lambda *a: list(builtins.range(*a))
    ref_utils.map = lambda *a: list(builtins.map(*a))
    _csc = sp.csc_matrix

    def csc_int(arg, *a, **k):
        if isinstance(arg, tuple) and len(arg) == 2 and isinstance(arg[1], tuple):
            vals, (ri, ci) = arg
            arg = (vals, (np.asarray(ri).astype(np.int64), np.asarray(ci).astype(np.int64)))
        return _csc(arg, *a, **k)

    ref_utils.csc_matrix = csc_int
    import solvers as ref_solvers  # noqa: E402  (the reference's code/solvers.py)

    return ref_utils, ref_solvers
