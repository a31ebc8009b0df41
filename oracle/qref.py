"""oracle/qref.py — ctypes front-end for oracle/liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the parity checker, never by the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

# ggml type ids (reference include/ggml.h:372-412)
F32, F16, Q4_0, Q8_0, Q8_1, Q4_K, Q5_K, Q6_K, Q8_K, I32 = 0, 1, 2, 8, 9, 12, 13, 14, 15, 26
NAMES = {Q4_0: "q4_0", Q8_0: "q8_0", Q4_K: "q4_K", Q5_K: "q5_K", Q6_K: "q6_K", F32: "f32"}
BY_NAME = {v: k for k, v in NAMES.items()}
HOT_TYPES = (Q4_0, Q8_0, Q4_K, Q5_K, Q6_K)
BLCK = {Q4_0: 32, Q8_0: 32, Q8_1: 32, Q4_K: 256, Q5_K: 256, Q6_K: 256, Q8_K: 256, F32: 1}
TSIZE = {Q4_0: 18, Q8_0: 34, Q8_1: 36, Q4_K: 144, Q5_K: 176, Q6_K: 210, Q8_K: 292, F32: 4}
ACT_REF, ACT_X86 = 0, 1


def row_size(t: int, ne0: int) -> int:
    return TSIZE[t] * (ne0 // BLCK[t])


class QTensor(C.Structure):
    _fields_ = [("type", C.c_int), ("data", C.c_void_p), ("ne", C.c_int64 * 4), ("nb", C.c_size_t * 4)]


def build() -> None:
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "qref.c")):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.qref_fill_uniform.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_float, C.c_float]
        L.qref_quantize_chunk.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p]
        L.qref_quantize_chunk.restype = C.c_size_t
        L.qref_dequantize_row.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64]
        L.qref_quantize_act.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int]
        L.qref_vec_dot.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.qref_vec_dot.restype = C.c_float
        L.qref_mul_mat.argtypes = [C.POINTER(QTensor)] * 3 + [C.c_int, C.c_int]
        L.qref_mul_mat_id.argtypes = [C.POINTER(QTensor)] * 4 + [C.c_int, C.c_int]
        L.qref_fp32_to_fp16.argtypes = [C.c_float]
        L.qref_fp32_to_fp16.restype = C.c_uint16
        L.qref_fp16_to_fp32.argtypes = [C.c_uint16]
        L.qref_fp16_to_fp32.restype = C.c_float
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def fill_uniform_c(n: int, seed: int, lo=-1.0, hi=1.0) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().qref_fill_uniform(_ptr(out), n, seed, lo, hi)
    return out


def fill_uniform(n: int, seed: int, lo=-1.0, hi=1.0) -> np.ndarray:
    """numpy restatement of qref_fill_uniform (splitmix64 counter mode); bit-identical."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return (np.float32(lo) + np.float32(hi - lo) * u).astype(np.float32)


def quantize(t: int, x: np.ndarray, n_per_row: int | None = None, imatrix: np.ndarray | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32).ravel()
    npr = n_per_row or x.size
    out = np.zeros(row_size(t, x.size), np.uint8)
    im = None if imatrix is None else np.ascontiguousarray(imatrix, np.float32)
    lib().qref_quantize_chunk(t, _ptr(x), _ptr(out), 0, x.size // npr, npr, None if im is None else _ptr(im))
    return out


def dequantize(t: int, q: np.ndarray, n: int) -> np.ndarray:
    q = np.ascontiguousarray(q, np.uint8)
    out = np.empty(n, np.float32)
    lib().qref_dequantize_row(t, _ptr(q), _ptr(out), n)
    return out


def quantize_act(t: int, x: np.ndarray, flavour: int = ACT_X86) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.zeros(row_size(t, x.size), np.uint8)
    lib().qref_quantize_act(t, _ptr(x), _ptr(out), x.size, flavour)
    return out


def vec_dot(t: int, n: int, w: np.ndarray, a: np.ndarray) -> float:
    return float(lib().qref_vec_dot(t, n, _ptr(np.ascontiguousarray(w)), _ptr(np.ascontiguousarray(a))))


def tensor(t: int, buf: np.ndarray, ne, nb) -> QTensor:
    T = QTensor()
    T.type = t
    T.data = buf.ctypes.data
    for i in range(4):
        T.ne[i] = int(ne[i]) if i < len(ne) else 1
        T.nb[i] = int(nb[i])
    return T


def contiguous_nb(t: int, ne) -> list:
    ne = list(ne) + [1] * (4 - len(ne))
    nb = [TSIZE[t], row_size(t, ne[0])]
    nb.append(nb[1] * ne[1])
    nb.append(nb[2] * ne[2])
    return nb


def mul_mat(a: QTensor, b: QTensor, c: QTensor, flavour: int = ACT_X86, threads: int = 0) -> None:
    rc = lib().qref_mul_mat(C.byref(a), C.byref(b), C.byref(c), flavour, threads)
    if rc != 0:
        raise ValueError(f"qref_mul_mat rejected shapes (rc={rc})")


def mul_mat_id(a: QTensor, b: QTensor, ids: QTensor, c: QTensor, flavour: int = ACT_X86, threads: int = 0) -> None:
    rc = lib().qref_mul_mat_id(C.byref(a), C.byref(b), C.byref(ids), C.byref(c), flavour, threads)
    if rc != 0:
        raise ValueError(f"qref_mul_mat_id rejected shapes (rc={rc})")


def mul_mat_simple(t: int, wq: np.ndarray, N: int, K: int, x: np.ndarray, M: int, threads: int = 0) -> np.ndarray:
    """dst[M, N] = W[N, K] (quantized rows) @ x[M, K]^T — contiguous 2-D case."""
    out = np.zeros((M, N), np.float32)
    x = np.ascontiguousarray(x, np.float32)
    A = tensor(t, wq, [K, N, 1, 1], contiguous_nb(t, [K, N, 1, 1]))
    B = tensor(F32, x, [K, M, 1, 1], contiguous_nb(F32, [K, M, 1, 1]))
    D = tensor(F32, out, [N, M, 1, 1], contiguous_nb(F32, [N, M, 1, 1]))
    mul_mat(A, B, D, threads=threads)
    return out


def nmse(out: np.ndarray, ref: np.ndarray) -> float:
    """test-backend-ops.cpp:180-193 — sum((a-b)^2) / sum(b^2), in double."""
    a = np.asarray(out, np.float64).ravel()
    b = np.asarray(ref, np.float64).ravel()
    den = float(np.sum(b * b))
    return float(np.sum((a - b) ** 2)) / den if den > 0 else float(np.sum((a - b) ** 2))
