"""mi355x_qmm.py — Python front-end (ctypes) of libggml-hip-mi355x.so.

Host-side mirror of the reference's MUL_MAT operator interface for the repo's harness and
bench: operands are described exactly like ggml tensors (type, ne[4], nb[4] in bytes) and
live in device memory that PyTorch-ROCm allocates (plumbing only). Every compute call goes
through the C ABI of include/ggml-mi355x.h; there is no fallback — if the HIP library is
missing or no gfx950 device is present the calls raise.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libggml-hip-mi355x.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
# diagnostics: A/B a variant build of the same library (scripts/*); unset in every product run
if os.environ.get("GGML_MI355X_LIB"):
    LIB_PATH = os.environ["GGML_MI355X_LIB"]
HEADER = os.path.join(os.path.dirname(HERE), "include", "ggml-mi355x.h")

F32, Q4_0, Q8_0, Q4_K, Q5_K, Q6_K, I32 = 0, 2, 8, 12, 13, 14, 26
BLCK = {Q4_0: 32, Q8_0: 32, Q4_K: 256, Q5_K: 256, Q6_K: 256, F32: 1, I32: 1}
TSIZE = {Q4_0: 18, Q8_0: 34, Q4_K: 144, Q5_K: 176, Q6_K: 210, F32: 4, I32: 4}
NAMES = {Q4_0: "q4_0", Q8_0: "q8_0", Q4_K: "q4_K", Q5_K: "q5_K", Q6_K: "q6_K"}


class MmTensor(C.Structure):
    """ggml_mi355x_tensor (include/ggml-mi355x.h)"""
    _fields_ = [("type", C.c_int32), ("data", C.c_void_p), ("ne", C.c_int64 * 4), ("nb", C.c_size_t * 4)]


class Mi355xError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile the HIP library in-tree (gfx950) if missing or stale."""
    srcs = [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))]
    if os.environ.get("GGML_MI355X_LIB"):
        return LIB_PATH
    stale = not os.path.exists(LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs)
    if force or stale:
        subprocess.check_call(["make", "-s", "-C", HERE, "-j8", LIB_NAME])
    return LIB_PATH


_lib = None


def lib():
    """Load the library (no compute call is made here, so this also works without a GPU)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Mi355xError(f"{LIB_PATH} missing: run `make -C ggml-gfx906_amd` (HIP extension not built)")
        # torch-ROCm ships its own libamdhip64.so.7 (same soname as /opt/rocm's). Import torch
        # first so the process holds ONE HIP runtime, torch's: loaded the other way round, our
        # library would pull in /opt/rocm's runtime and torch's HIP init then finds no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P = C.POINTER(MmTensor)
        L.ggml_mi355x_mul_mat.argtypes = [P, P, P, C.c_void_p]
        L.ggml_mi355x_mul_mat_id.argtypes = [P, P, P, P, C.c_void_p]
        L.ggml_mi355x_dequantize.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.ggml_mi355x_supports_mul_mat.argtypes = [P, P]
        L.ggml_mi355x_get_rows.argtypes = [P, P, P, C.c_void_p]
        L.ggml_mi355x_quantize.argtypes = [P, P, C.c_void_p]
        L.ggml_mi355x_cpy.argtypes = [P, P, C.c_void_p]
        L.ggml_mi355x_repack_size.argtypes = [P, C.POINTER(C.c_size_t)]
        L.ggml_mi355x_repack.argtypes = [P, C.c_void_p, C.c_size_t, C.c_void_p]
        L.ggml_mi355x_mul_mat_repacked.argtypes = [P, C.c_void_p, P, P, C.c_void_p]
        L.ggml_mi355x_supports_mul_mat_id.argtypes = [P, P, P]
        L.ggml_mi355x_mul_mat_plan.argtypes = [P, P, C.c_int, C.c_char_p, C.c_size_t]
        L.ggml_mi355x_reload_settings.restype = C.c_int
        L.ggml_mi355x_device_error.restype = C.c_int
        L.ggml_mi355x_strerror.restype = C.c_char_p
        L.ggml_mi355x_strerror.argtypes = [C.c_int]
        L.ggml_backend_init.restype = C.c_void_p
        L.ggml_backend_score.restype = C.c_int
        _lib = L
    return _lib


def exported_api() -> list:
    """Function names declared GGML_MI355X_API in include/ggml-mi355x.h."""
    import re
    txt = open(HEADER).read()
    txt = re.sub(r"#define GGML_MI355X_API[^\n]*", "", txt)
    return re.findall(r"GGML_MI355X_API\s+[\w\s\*]*?\b(\w+)\s*\(", txt)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise Mi355xError(f"{what}: {lib().ggml_mi355x_strerror(rc).decode()} (rc={rc})")


def row_size(t: int, ne0: int) -> int:
    return TSIZE[t] * (ne0 // BLCK[t])


def contiguous_nb(t: int, ne) -> list:
    ne = list(ne) + [1] * (4 - len(ne))
    nb = [TSIZE[t], row_size(t, ne[0])]
    nb.append(nb[1] * ne[1])
    nb.append(nb[2] * ne[2])
    return nb


def tensor(t: int, ptr: int, ne, nb) -> MmTensor:
    T = MmTensor()
    T.type = t
    T.data = ptr
    ne = list(ne) + [1] * (4 - len(ne))
    for i in range(4):
        T.ne[i] = int(ne[i])
        T.nb[i] = int(nb[i])
    return T


def _stream_ptr(stream) -> int | None:
    """hipStream_t for a call: None = torch's current stream; a torch Stream; or a raw handle"""
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def mul_mat(a: MmTensor, b: MmTensor, d: MmTensor, stream=None) -> None:
    _check(lib().ggml_mi355x_mul_mat(C.byref(a), C.byref(b), C.byref(d), _stream_ptr(stream)), "mul_mat")


def get_rows(a: MmTensor, rows: MmTensor, d: MmTensor, stream=None) -> None:
    """dst = get_rows(a, rows) (GGML_OP_GET_ROWS) on the device"""
    _check(lib().ggml_mi355x_get_rows(C.byref(a), C.byref(rows), C.byref(d), _stream_ptr(stream)), "get_rows")


def quantize(src: MmTensor, dst: MmTensor, stream=None) -> None:
    """dst (Q4_0 / Q8_0) = quantize_row_*_ref(src f32) on the device (GGML_OP_CPY f32 -> q)"""
    _check(lib().ggml_mi355x_quantize(C.byref(src), C.byref(dst), _stream_ptr(stream)), "quantize")


def repack_size(a: MmTensor) -> int:
    """bytes of the repacked (MFMA-fragment order) copy of quantized src0 `a`"""
    n = C.c_size_t(0)
    _check(lib().ggml_mi355x_repack_size(C.byref(a), C.byref(n)), "repack_size")
    return n.value


def repack(a: MmTensor, dst_ptr: int, nbytes: int, stream=None) -> None:
    _check(lib().ggml_mi355x_repack(C.byref(a), dst_ptr, nbytes, _stream_ptr(stream)), "repack")


def mul_mat_repacked(a: MmTensor, rp_ptr: int, b: MmTensor, d: MmTensor, stream=None) -> None:
    _check(lib().ggml_mi355x_mul_mat_repacked(C.byref(a), rp_ptr, C.byref(b), C.byref(d), _stream_ptr(stream)),
           "mul_mat_repacked")


def cpy(src: MmTensor, dst: MmTensor, stream=None) -> None:
    """dst = src (GGML_OP_CPY): f32 -> Q4_0/Q8_0, hot quant -> f32 (dup_q), hot -> same type"""
    _check(lib().ggml_mi355x_cpy(C.byref(src), C.byref(dst), _stream_ptr(stream)), "cpy")


def device_error() -> int:
    """returns and clears the device error word (call after synchronizing the stream)"""
    return lib().ggml_mi355x_device_error()


def mul_mat_id(a: MmTensor, b: MmTensor, ids: MmTensor, d: MmTensor, stream=None) -> None:
    _check(lib().ggml_mi355x_mul_mat_id(C.byref(a), C.byref(b), C.byref(ids), C.byref(d), _stream_ptr(stream)),
           "mul_mat_id")


def dequantize(t: int, src_ptr: int, dst_ptr: int, n: int, stream=None) -> None:
    _check(lib().ggml_mi355x_dequantize(t, src_ptr, dst_ptr, n, _stream_ptr(stream)), "dequantize")


def reload_settings() -> None:
    """re-read the GGML_MI355X_* knobs (the library reads them once otherwise)"""
    lib().ggml_mi355x_reload_settings()


@contextlib.contextmanager
def knobs(**env):
    """set GGML_MI355X_* knobs (None = unset) for the calls inside the block, then restore them"""
    saved = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        reload_settings()
        yield
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        reload_settings()


def mul_mat_plan(a: MmTensor, b: MmTensor, repacked: bool = False) -> str:
    """the kernel launches mul_mat would make for these operands (no launch, no GPU needed)"""
    buf = C.create_string_buffer(512)
    _check(lib().ggml_mi355x_mul_mat_plan(C.byref(a), C.byref(b), 1 if repacked else 0, buf, len(buf)), "mul_mat_plan")
    return buf.value.decode()


def supports_mul_mat_id(a: MmTensor, b: MmTensor, ids: MmTensor) -> bool:
    return bool(lib().ggml_mi355x_supports_mul_mat_id(C.byref(a), C.byref(b), C.byref(ids)))


def device_count() -> int:
    return lib().ggml_mi355x_device_count()
