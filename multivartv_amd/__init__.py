"""multivartv_amd — MI355X-native mesh-TV ADMM solver (the hot path of brayano/MultivarTV).

The numerical work runs in hand-written HIP kernels for gfx950 behind the C ABI
in include/mvtv/mvtv.h (libmvtv.so). This package is the host-side mirror of
the reference's Python interface (code/solvers.py, code/utils.py) over that ABI.
"""
from ._lib import (ORDER_CPP, ORDER_PY, SOLVER_AUTO, SOLVER_PCG, SOLVER_PCG_SPECTRAL, SOLVER_SPECTRAL,  # noqa: F401
                   VARIANT_CPP,
                   VARIANT_PY, VARIANT_RCPP, DimMismatchError, MaxIterError, MvtvError, Problem, device_count, lib)

from . import cv  # noqa: E402,F401  (CV / lambda-path driver, rcpp…/solvers.cpp:186-376)

__version__ = "0.1.0"
