"""CPU-only checks of the product boundary: libnkhip.so loads, exports every symbol the public
header declares, and the host mirror fails loudly without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import _nkpath  # noqa: F401
import ariadne_hip as ah
from ariadne_hip import _lib
from oracle import oracle as oc

HEADER = _lib.HEADER


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|double\*|void\*|const char\*)\s+(nk_\w+)\s*\(", src, re.M)))


def test_library_built_in_tree():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build()"
    assert _lib.LIB_PATH.startswith(os.path.dirname(os.path.dirname(__file__)))


KNOBS = ["NK_RES_NOXCHG", "NK_RES_JV", "NK_RES_STRIDED", "NK_RES_NTC", "NK_RES_PRE", "NK_F0R",
         "NK_ST_BLOCKS", "NK_MGS_VARIANT", "NK_RED_BLOCKS", "NK_UPD_U", "NK_RES_NWC",
         "NK_ALLOC_STAGGER", "NK_ALLOC_STAGGER_MOD"]


def test_product_library_has_no_kbench_hooks_or_knobs():
    """The product library (what the Julia shim and the Python mirror load) carries no timing hooks,
    no tuning knob and no wrong-answer probe (NK_RES_NOXCHG): those live in the kernel-variant bench
    build only, lib/libnkhip_kbench.so, which exports the nkb_* hooks and reads the knobs."""
    prod = open(_lib.PRODUCT_LIB, "rb").read()
    kb = open(_lib.KBENCH_LIB, "rb").read()
    for sym in (b"nkb_copy", b"nkb_stencil_kind", b"nkb_mgs_res", b"nkb_update_x", b"nkb_stream_jv"):
        assert sym not in prod, sym
        assert sym in kb, sym
    for k in KNOBS:
        assert k.encode() not in prod, k
        assert k.encode() in kb, k
    # the product is the smaller build: variant instantiations pruned
    assert len(prod) < 0.7 * len(kb)
    # operational configuration stays readable in the product (transport, timeouts, shared-GPU rigs, the
    # one-GPU exchange rigs of bench.py --block-of / tools/halo_self.py and the exchange-form switch)
    for k in (b"NK_DIST_MAILBOX", b"NK_MB_SPIN_LIMIT", b"NK_RES_SHARED", b"NK_MGS_RESIDENT", b"NK_HALO_CAP",
              b"NK_DIST_FORCE", b"NK_HALO_SELF", b"NK_HALO_SELF_AXES", b"NK_HALO_FUSE", b"NK_SHARED_FUSE_MAX"):
        assert k in prod, k


def test_every_header_symbol_exported_and_bound():
    lib = ah.load()
    names = header_functions()
    assert len(names) >= 30
    for name in names:
        assert hasattr(lib, name), f"{name} declared in include/nkhip.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(names)


def test_header_structs_match_ctypes():
    src = open(HEADER).read()
    body = re.search(r"typedef struct nk_problem \{(.*?)\} nk_problem;", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"\b(\w+);", body.replace(",", ";"))
    # names differ only where Python reserves the word (lambda -> lam)
    want = [f if f != "lambda" else "lam" for f in fields]
    got = [f[0] for f in _lib.nk_problem._fields_]
    assert got == want


def test_struct_layouts_match_c(tmp_path):
    """sizeof/offsetof of the public structs as gcc lays them out == the ctypes mirrors."""
    import subprocess

    structs = {"nk_problem": _lib.nk_problem, "nk_krylov_opts": _lib.nk_krylov_opts,
               "nk_krylov_stats": _lib.nk_krylov_stats, "nk_prof_entry": _lib.nk_prof_entry,
               "nk_user_ops": _lib.nk_user_ops, "nk_newton_opts": _lib.nk_newton_opts,
               "nk_newton_stats": _lib.nk_newton_stats, "nk_precond": _lib.nk_precond}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for sname, cls in structs.items():
        lines.append(f'printf("{sname} %zu\\n", sizeof({sname}));')
        for fname, _ in cls._fields_:
            cname = "lambda" if fname == "lam" else fname
            lines.append(f'printf("{sname}.{fname} %zu\\n", offsetof({sname}, {cname}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    for sname, cls in structs.items():
        assert int(got[sname]) == C.sizeof(cls), sname
        for fname, _ in cls._fields_:
            assert int(got[f"{sname}.{fname}"]) == getattr(cls, fname).offset, f"{sname}.{fname}"


def test_no_gpu_fails_loudly():
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(ah.NKError):
        ah.Context(0)


def test_forcing_mirror_matches_oracle():
    ew = ah.EisenstatWalker()
    rng = np.random.default_rng(7)
    for _ in range(100):
        eta, tol = rng.uniform(0, 1), 10 ** rng.uniform(-12, -2)
        prior = 10 ** rng.uniform(-6, 2)
        n = prior * rng.uniform(0.01, 1.2)
        assert ew(eta, tol, n, prior) == oc.ew_forcing(eta, tol, n, prior)
    assert ah.Fixed().initial() == 0.1 and ah.Fixed(0.3)(1, 2, 3, 4) == 0.3
    assert ew.initial() == 0.999


def test_stats_update():
    s = ah.Stats(0, 0, 1.0).update(7, 0.5).update(3, 0.25)
    assert s == ah.Stats(2, 10, 0.25)


def test_slab_partition():
    for n, r in [(4096, 8), (37, 4), (9, 3), (5, 5)]:
        grids = [ah.slab((16, n), k, r) for k in range(r)]
        assert sum(g.shape_xyz[-1] for g in grids) == n
        assert [g.offset for g in grids] == list(np.cumsum([0] + [g.shape_xyz[-1] for g in grids])[:-1])
        assert all(g.global_xyz == (16, n) for g in grids)
    with pytest.raises(ValueError):
        ah.slab((4, 2), 0, 3)


def test_block_partition():
    """3D blocks tile the global grid exactly once; rank = (iz py + iy) px + ix; blocks sharing a face
    share its extents (what k_faces_ipc relies on); pgrid (1, 1, n) is the slab split."""
    for gx, pg in [((40, 20, 24), (2, 2, 2)), ((33, 20, 17), (1, 3, 1)), ((130, 18, 20), (4, 2, 1)), ((9, 8, 7), (3, 2, 1))]:
        n = int(np.prod(pg))
        blocks = [ah.block(gx, r, pg) for r in range(n)]
        cover = np.zeros(gx[::-1], dtype=int)
        for b in blocks:
            (x0, y0, z0), (nx, ny, nz) = b.origin, b.shape_xyz
            cover[z0:z0 + nz, y0:y0 + ny, x0:x0 + nx] += 1
            assert b.offset == z0 and b.global_xyz == gx
        assert (cover == 1).all()
        px, py, _ = pg
        for r, b in enumerate(blocks):
            if r % px + 1 < px:  # x neighbour: same ny, nz
                assert blocks[r + 1].shape_xyz[1:] == b.shape_xyz[1:]
            if (r // px) % py + 1 < py:  # y neighbour: same nx, nz
                o = blocks[r + px].shape_xyz
                assert (o[0], o[2]) == (b.shape_xyz[0], b.shape_xyz[2])
    for r in range(3):
        s, b = ah.slab((8, 8, 9), r, 3), ah.block((8, 8, 9), r, (1, 1, 3))
        assert (s.shape_xyz, s.offset) == (b.shape_xyz, b.offset)
    with pytest.raises(ValueError):
        ah.block((4, 8, 8), 0, (5, 1, 1))
    with pytest.raises(ValueError):
        ah.block((8, 8), 0, (2, 1, 1))


def test_grid_shapes():
    g = ah.Grid.full(7, 5)
    assert g.np_shape == (5, 7) and g.n == 35 and g.nxyz == (7, 5, 1)
    g3 = ah.Grid.full(4, 3, 2)
    assert g3.np_shape == (2, 3, 4) and g3.dim == 3


def test_unsupported_algo_and_generic_residual_rejected():
    with pytest.raises(NotImplementedError):
        ah.krylov.KrylovWorkspace("bicgstab", ah.KrylovConstructor.__new__(ah.KrylovConstructor))
    with pytest.raises(TypeError):
        ah.JacobianOperator(lambda r, u, p: None, None, None)
    with pytest.raises(NotImplementedError):
        ah.G_Midpoint_.bind(lambda du, u, p, t: None)  # only diffusion! has a fused device residual
    with pytest.raises(TypeError):
        ah.G_Euler_(alpha=0.3)  # α is G_Midpoint!'s keyword
