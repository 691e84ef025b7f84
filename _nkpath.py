"""Put the in-tree host package (newtonkrylov.jl_amd/ariadne_hip) on sys.path.

The package directory name contains a dot, so it cannot be imported as a dotted module; its
Python host mirror lives in the sub-package `ariadne_hip` next to csrc/ and lib/libnkhip.so.
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "newtonkrylov.jl_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
