"""Shared pytest setup: the ``gpu`` marker and golden-fixture loading."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, {k: z[k] for k in z.files if k != "meta"}


@pytest.fixture
def golden():
    return load_golden


def log_parity(case, **errs):
    """Record the achieved error of one parity check: a JSON line in $MVTV_PARITY_LOG (if set), so the
    errors the suite actually reached on the GPU box can be tabulated."""
    path = os.environ.get("MVTV_PARITY_LOG")
    if not path:
        return
    rec = {"case": case}
    rec.update({k: (float(v) if not isinstance(v, (int, str)) else v) for k, v in errs.items()})
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
