"""CPU-only checks of the C-ABI library: it loads, exports every symbol include/mvtv/mvtv.h declares,
and its host-side bindings agree with the header (no compute calls, no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import multivartv_amd as mv
from multivartv_amd import _lib
from multivartv_amd import slab  # noqa: F401  (registers the slab entry points in _lib.SIGNATURES)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mvtv", "mvtv.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mvtv_[A-Za-z_0-9]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared_functions()
    for n in ("mvtv_problem_create", "mvtv_admm", "mvtv_admm_run", "mvtv_apply_D", "mvtv_apply_Dt",
              "mvtv_apply_A", "mvtv_solve", "mvtv_state_set", "mvtv_state_get", "mvtv_timing_get"):
        assert n in names


def test_library_exports_every_declared_symbol():
    L = mv.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the ABI structs have the C compiler's sizes and field offsets."""
    structs = {"mvtv_problem_desc": _lib.ProblemDesc, "mvtv_admm_opts": _lib.AdmmOpts,
               "mvtv_admm_stats": _lib.AdmmStats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mvtv/mvtv.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_host_only_calls():
    L = mv.lib()
    assert L.mvtv_version().startswith(b"multivartv_amd")
    assert L.mvtv_status_string(3) == b"dimension mismatch (mixed-partial construction)"
    o = _lib.default_opts(mv.VARIANT_CPP, fixed_iters=3)
    assert o.variant == mv.VARIANT_CPP and o.fixed_iters == 3 and np.isnan(o.sigma)
    assert L.mvtv_kernel_name(8) == b"pcg_fused3d"
    assert [L.mvtv_kernel_name(k).decode() for k in range(len(_lib.KERNELS))] == _lib.KERNELS


def test_no_device_fails_loudly():
    if mv.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(mv.MvtvError):
        mv.Problem([4, 4], np.zeros(16))


def test_rccl_resolves_to_rocm_not_torch():
    """libmvtv's RCCL is ROCm's librccl (on libmvtv's HIP runtime) even after `import torch` has mapped
    torch's librccl: torch's links torch's own HIP runtime copy, on which libmvtv's streams are invalid (a
    GPU run of the NOLOAD reuse failed at ncclCommInitRank with "unhandled cuda error"). One RCCL *runs* per
    bench rank because torch.distributed is given gloo there. Child process: the resolution is per process."""
    code = ("import torch, multivartv_amd\n"
            "from multivartv_amd import slab\n"
            "print(slab.Comm.library())\n")
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    import torch
    torch_lib = os.path.realpath(os.path.join(os.path.dirname(torch.__file__), "lib"))
    path = os.path.realpath(out.stdout.strip().splitlines()[-1])
    assert path and not path.startswith(torch_lib)
    assert "rccl" in os.path.basename(path)
