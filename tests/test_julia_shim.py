"""CPU check of the (otherwise untested: no Julia in the image) Julia shim: its C-layout structs
must list the same fields, in the same order and with the same widths, as include/nkhip.h (whose
layout test_abi.py checks against gcc).  A drifting shim would corrupt every ccall."""
import ctypes as C
import os
import re

import pytest

import _nkpath  # noqa: F401
from ariadne_hip import _lib

SHIM = os.path.join(os.path.dirname(_lib.PKG_DIR), "newtonkrylov.jl_amd", "julia", "AriadneHIP.jl")
JL_SIZE = {"Int32": 4, "Int64": 8, "Float64": 8, "Bool": 1}
PAIRS = [("NkProblem", _lib.nk_problem), ("NkKrylovOpts", _lib.nk_krylov_opts),
         ("NkKrylovStats", _lib.nk_krylov_stats), ("NkUserOps", _lib.nk_user_ops), ("NkPrecond", _lib.nk_precond)]


def jl_fields(name):
    src = open(SHIM).read()
    body = re.search(rf"^struct {name}\n(.*?)^end", src, re.S | re.M).group(1)
    out = []
    for line in body.splitlines():
        m = re.match(r"\s*(\w+)::([\w{}]+)", line)
        if m:
            t = m.group(2)
            out.append((m.group(1), 8 if t.startswith("Ptr") else JL_SIZE[t]))
    return out


@pytest.mark.parametrize("jl,cstruct", PAIRS, ids=[p[0] for p in PAIRS])
def test_shim_struct_matches_header(jl, cstruct):
    got = jl_fields(jl)
    want = [("lambda" if f == "lam" else f, C.sizeof(t)) for f, t in cstruct._fields_]
    assert got == want
