"""Feature / label / window file readers of the reference drivers.

Formats (TESTS/TEST1/foo.cpp:9-120, shared by TEST2-4):
  *.feature  "n d" header, then n*d whitespace-separated values, column-major (all of feature 0,
             then feature 1, ...), foo.cpp:9-46.
  *.label    "n" header, then n values, foo.cpp:48-81.
  *.window   "nwindows dwindows" header, then nwindows*dwindows ints read in file order, so
             row w of the file is window w; -1 pads a short last window, foo.cpp:83-117.
The reference prints and exit(1)s on a malformed file; these raise ValueError instead.
"""
from __future__ import annotations

import numpy as np


def _tokens(path):
    with open(path) as fh:
        return fh.read().split()


def read_features(path: str) -> np.ndarray:
    """n x d float64 array in Fortran (column-major, ldim = n) order, ready for the handle create."""
    tok = _tokens(path)
    if len(tok) < 2:
        raise ValueError(f"{path}: missing 'n d' header")
    n, d = int(tok[0]), int(tok[1])
    vals = np.array(tok[2:2 + n * d], dtype=np.float64)
    if vals.size != n * d:
        raise ValueError(f"{path}: expected {n * d} entries, found {vals.size}")
    return vals.reshape(d, n).T.copy(order="F")


def read_labels(path: str) -> np.ndarray:
    tok = _tokens(path)
    if not tok:
        raise ValueError(f"{path}: missing 'n' header")
    n = int(tok[0])
    vals = np.array(tok[1:1 + n], dtype=np.float64)
    if vals.size != n:
        raise ValueError(f"{path}: expected {n} labels, found {vals.size}")
    return vals


def read_windows(path: str):
    """(windows int32[nwindows*dwindows], nwindows, dwindows) as the ParamCreate calls take them."""
    tok = _tokens(path)
    if len(tok) < 2:
        raise ValueError(f"{path}: missing 'nwindows dwindows' header")
    nw, dw = int(tok[0]), int(tok[1])
    vals = np.array(tok[2:2 + nw * dw], dtype=np.int32)
    if vals.size != nw * dw:
        raise ValueError(f"{path}: expected {nw * dw} entries, found {vals.size}")
    return vals, nw, dw
