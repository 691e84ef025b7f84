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
JL_SIZE = {"Int32": 4, "Int64": 8, "Float64": 8, "Bool": 1, "UInt8": 1}
PAIRS = [("NkProblem", _lib.nk_problem), ("NkKrylovOpts", _lib.nk_krylov_opts),
         ("NkKrylovStats", _lib.nk_krylov_stats), ("NkUserOps", _lib.nk_user_ops), ("NkPrecond", _lib.nk_precond),
         ("NkPathInfo", _lib.nk_path_info)]


def jl_fields(name):
    src = open(SHIM).read()
    body = re.search(rf"^struct {name}\n(.*?)^end", src, re.S | re.M).group(1)
    out = []
    for line in body.splitlines():
        m = re.match(r"\s*(\w+)::(NTuple\{\d+, ?\w+\}|[\w{}]+)", line)
        if m:
            t = m.group(2)
            tup = re.match(r"NTuple\{(\d+), ?(\w+)\}", t)
            size = int(tup.group(1)) * JL_SIZE[tup.group(2)] if tup else (8 if t.startswith("Ptr") else JL_SIZE[t])
            out.append((m.group(1), size))
    return out


@pytest.mark.parametrize("jl,cstruct", PAIRS, ids=[p[0] for p in PAIRS])
def test_shim_struct_matches_header(jl, cstruct):
    got = jl_fields(jl)
    want = [("lambda" if f == "lam" else f, C.sizeof(t)) for f, t in cstruct._fields_]
    assert got == want


# ---------------------------------------------------------------------------------------------------
# Every `ccall((:nk_*, libnkhip), Ret, (Args...), ...)` in the shim against the prototype in nkhip.h:
# the symbol exists, the argument count matches, and each argument / the return value has the same
# class (32-bit int, 64-bit int, double, pointer).  A wrong width here would corrupt the call.
HEADER = os.path.join(os.path.dirname(_lib.PKG_DIR), "include", "nkhip.h")


def _split_top(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _matching(s, i):
    """index of the parenthesis closing the one at s[i]"""
    depth = 0
    for j in range(i, len(s)):
        depth += s[j] == "("
        depth -= s[j] == ")"
        if depth == 0:
            return j
    raise ValueError("unbalanced")


JL_CLASS = {"Cint": "i32", "Int32": "i32", "Int64": "i64", "Float64": "f64", "Cdouble": "f64", "VP": "ptr",
            "Cstring": "ptr"}


def jl_class(t):
    t = t.strip()
    if t.startswith(("Ptr{", "Ref{")) or t == "Ptr":
        return "ptr"
    return JL_CLASS[t]


def c_class(decl):
    d = decl.strip()
    if "*" in d or "[" in d:
        return "ptr"
    d = d.replace("const", "").strip()
    typ = d.rsplit(None, 1)[0] if len(d.split()) > 1 else d
    return {"int": "i32", "int32_t": "i32", "int64_t": "i64", "double": "f64"}[typ]


def header_prototypes():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"([\w\s\*]+?)\b(nk_\w+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        if "typedef" in ret or "(*" in m.group(0):
            continue
        params = [] if args.strip() in ("", "void") else _split_top(args)
        protos[name] = (c_class(ret.strip() + " x"), [c_class(p) for p in params])
    return protos


def shim_ccalls():
    src = open(SHIM).read()
    calls = []
    for m in re.finditer(r"ccall\(\(:(nk_\w+),\s*libnkhip\),", src):
        rest = src[m.end():]
        ret_end = rest.index(",")
        ret = rest[:ret_end].strip()
        i = rest.index("(", ret_end)
        j = _matching(rest, i)
        calls.append((m.group(1), ret, _split_top(rest[i + 1:j])))
    return calls


def test_shim_ccalls_match_header():
    protos = header_prototypes()
    calls = shim_ccalls()
    assert len(calls) >= 30
    for name, ret, args in calls:
        assert name in protos, f"{name} is not declared in nkhip.h"
        cret, cargs = protos[name]
        got = [jl_class(a) for a in args]
        assert len(got) == len(cargs), f"{name}: {len(got)} ccall arguments, header has {len(cargs)}"
        assert got == cargs, f"{name}: argument classes {got} != header {cargs}"
        assert jl_class(ret) == cret, f"{name}: return {ret} vs header class {cret}"


def test_shim_binds_the_reference_operator_surface():
    """The shim's entry points for src/Ariadne.jl:48-162: mul! on J, transpose(J), the batched forms,
    collect(J) -- and the left preconditioner M is passed to the solve, not dropped (:327-329)."""
    names = {c[0] for c in shim_ccalls()}
    for sym in ("nk_jv", "nk_jtv", "nk_jv_batched", "nk_jtv_batched", "nk_jacobian_collect", "nk_krylov_solve"):
        assert sym in names
    src = open(SHIM).read()
    assert "isempty(kwargs) || error(" in src
    assert re.search(r"GC\.@preserve Nc N Mc M begin.*?NkKrylovOpts\(.*?, Np, Mp,.*?ccall\(\(:nk_krylov_solve",
                     src, re.S)
    for k in ("heat3d", "heat3d_midpoint", "heat3d_trapezoid"):
        assert f"{k} = NK_HEAT3D" in src
