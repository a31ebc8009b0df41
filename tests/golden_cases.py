"""Rebuild the golden MUL_MAT / MUL_MAT_ID cases (tests/golden/manifest.json) as host buffers.

A case is described exactly as test-backend-ops builds it (tests/test-backend-ops.cpp:3127-3191,
3226-3246 of the reference): a physical tensor filled by the portable PRNG (weights quantized
row-wise with the `_ref` quantizer), then optionally permuted or viewed. This module produces the
physical byte buffers plus the (ne, nb) of the logical operands, so that both the CPU oracle and
the GPU backend can be run on byte-identical inputs.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import numpy as np

import qref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["records"]


def load_bin(name: str, dtype) -> np.ndarray:
    return np.fromfile(os.path.join(GOLDEN, name), dtype=dtype)


@dataclass
class Operand:
    type: int
    buf: np.ndarray          # physical bytes (uint8) or floats
    ne: list                 # logical ne[4]
    nb: list                 # logical nb[4] (bytes)
    offset: int = 0          # byte offset of the logical tensor inside buf


def _phys_nb(t: int, ne) -> list:
    return qref.contiguous_nb(t, ne)


def _permute(ne, nb, per):
    ne2, nb2 = [0] * 4, [0] * 4
    for i in range(4):
        ne2[per[i]] = ne[i]
        nb2[per[i]] = nb[i]
    return ne2, nb2


def weights_bytes(t: int, ne, seed: int) -> np.ndarray:
    nel = int(np.prod(ne))
    f = qref.fill_uniform(nel, seed)
    if t == qref.F32:
        return f.view(np.uint8).copy()
    return qref.quantize(t, f, n_per_row=ne[0])


def mul_mat_operands(r: dict):
    """(a, b, out_ne) for a manifest `mul_mat` record."""
    t = r["type_id"]
    a_ne, b_ne = r["a_ne"], r["b_ne"]
    abuf = weights_bytes(t, a_ne, r["seed_a"])
    bbuf = qref.fill_uniform(int(np.prod(b_ne)), r["seed_b"])
    a_nb, b_nb = _phys_nb(t, a_ne), _phys_nb(qref.F32, b_ne)
    per = r["per"]
    if per != [0, 1, 2, 3]:
        a_lne, a_lnb = _permute(a_ne, a_nb, per)
        b_lne, b_lnb = _permute(b_ne, b_nb, per)
    elif r["view"]:
        k = r["k"]
        a_lne, a_lnb = [k] + list(a_ne[1:]), a_nb
        b_lne, b_lnb = [k] + list(b_ne[1:]), b_nb
    else:
        a_lne, a_lnb, b_lne, b_lnb = list(a_ne), a_nb, list(b_ne), b_nb
    return Operand(t, abuf, a_lne, a_lnb), Operand(qref.F32, bbuf, b_lne, b_lnb), list(r["out_ne"])


def mul_mat_id_operands(r: dict):
    t = r["type_id"]
    k, m, n, E, U = r["k"], r["m"], r["n"], r["n_mats"], r["n_used"]
    a_ne = [k, m, E, 1]
    abuf = weights_bytes(t, a_ne, r["seed_a"])
    b_ne = [k, 1 if r["b"] else U, n, 1]
    bbuf = qref.fill_uniform(int(np.prod(b_ne)), r["seed_b"])
    ids_full = load_bin(r["name"] + ".ids.i32", np.int32)          # [n][E]
    ids = Operand(qref.I32, ids_full, [U, n, 1, 1], [4, 4 * E, 4 * E * n, 4 * E * n])
    a = Operand(t, abuf, a_ne, _phys_nb(t, a_ne))
    b = Operand(qref.F32, bbuf, b_ne, _phys_nb(qref.F32, b_ne))
    return a, b, ids, list(r["out_ne"])


def oracle_mul_mat(a: Operand, b: Operand, out_ne, threads=0) -> np.ndarray:
    out = np.zeros(int(np.prod(out_ne)), np.float32)
    A = qref.tensor(a.type, a.buf, a.ne, a.nb)
    B = qref.tensor(b.type, b.buf, b.ne, b.nb)
    D = qref.tensor(qref.F32, out, out_ne, _phys_nb(qref.F32, out_ne))
    qref.mul_mat(A, B, D, threads=threads)
    return out


def oracle_mul_mat_id(a: Operand, b: Operand, ids: Operand, out_ne, threads=0) -> np.ndarray:
    out = np.zeros(int(np.prod(out_ne)), np.float32)
    A = qref.tensor(a.type, a.buf, a.ne, a.nb)
    B = qref.tensor(b.type, b.buf, b.ne, b.nb)
    I = qref.tensor(qref.I32, ids.buf, ids.ne, ids.nb)
    D = qref.tensor(qref.F32, out, out_ne, _phys_nb(qref.F32, out_ne))
    qref.mul_mat_id(A, B, I, D, threads=threads)
    return out
