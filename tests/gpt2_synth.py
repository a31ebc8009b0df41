"""tests/gpt2_synth.py — synthetic GPT-2 checkpoints in the reference's legacy ggml format.

Test infrastructure (it quantizes with the CPU oracle, oracle/qref.py). There is no network
for real GPT-2 weights, so checkpoints are random-init with the GPT-2
architecture and written in exactly the layout examples/gpt-2/main-sched.cpp:155-546 reads
(SURVEY Appendix D):

    u32 magic 0x67676d6c; i32 n_vocab, n_ctx, n_embd, n_head, n_layer, ftype (+ 1000*QNT_VERSION);
    i32 n_vocab; n_vocab x (u32 len, bytes);
    records until EOF: i32 n_dims, i32 name_len, i32 ttype, i32 ne[n_dims], name, data.

Only the 2-d weight matrices are quantized (examples/gpt-2/quantize.cpp:116-123: wte, lm_head
and the four per-layer "/w" matrices); lm_head is absent so the loader ties it to wte
(main-sched.cpp:503-510). Values come from the platform-independent counter-mode generator
qref.fill_uniform (splitmix64), so the same (hparams, seed) always yields the same bytes:
weights ~ U(-a, a) with a = 0.02*sqrt(3) (std 0.02), biases std 0.02, ln gains 1 +- 0.1.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

import qref

GPT2_117M = dict(n_vocab=50257, n_ctx=1024, n_embd=768, n_head=12, n_layer=12)
FTYPE = {qref.Q4_0: 2, qref.Q8_0: 7, qref.Q4_K: 12, qref.Q5_K: 13, qref.Q6_K: 14, qref.F32: 0}
QNT_VERSION = 2


def _tensors(hp: dict, seed: int):
    """(name, shape ne, f32 values, is_matrix) in the order the reference converter writes them."""
    E, V, C = hp["n_embd"], hp["n_vocab"], hp["n_ctx"]
    k = [seed * 1000]

    def u(n, scale, center=0.0):
        k[0] += 1
        a = scale * np.sqrt(3.0)
        return (qref.fill_uniform(n, k[0], -a, a) + np.float32(center)).astype(np.float32)

    yield "model/ln_f/g", [E], u(E, 0.1, 1.0), False
    yield "model/ln_f/b", [E], u(E, 0.02), False
    yield "model/wte", [E, V], u(E * V, 0.02), True
    yield "model/wpe", [E, C], u(E * C, 0.01), False
    for i in range(hp["n_layer"]):
        p = f"model/h{i}/"
        yield p + "ln_1/g", [E], u(E, 0.1, 1.0), False
        yield p + "ln_1/b", [E], u(E, 0.02), False
        yield p + "attn/c_attn/w", [E, 3 * E], u(3 * E * E, 0.02), True
        yield p + "attn/c_attn/b", [3 * E], u(3 * E, 0.02), False
        yield p + "attn/c_proj/w", [E, E], u(E * E, 0.02), True
        yield p + "attn/c_proj/b", [E], u(E, 0.02), False
        yield p + "ln_2/g", [E], u(E, 0.1, 1.0), False
        yield p + "ln_2/b", [E], u(E, 0.02), False
        yield p + "mlp/c_fc/w", [E, 4 * E], u(4 * E * E, 0.02), True
        yield p + "mlp/c_fc/b", [4 * E], u(4 * E, 0.02), False
        yield p + "mlp/c_proj/w", [4 * E, E], u(4 * E * E, 0.02), True
        yield p + "mlp/c_proj/b", [E], u(E, 0.02), False


def vocab(n_vocab: int) -> list:
    """ids 0..94 are the printable ASCII characters (so any prompt tokenizes), the rest dummies."""
    return [bytes([32 + i]) if i < 95 else f"<t{i}>".encode() for i in range(n_vocab)]


def write_model(path: str, hp: dict, wtype: int = qref.Q4_0, seed: int = 1234) -> str:
    """Write the checkpoint; returns its sha256."""
    h = hashlib.sha256()
    with open(path, "wb") as f:
        def w(b):
            f.write(b)
            h.update(b)

        w(struct.pack("<I", 0x67676D6C))
        ftype = FTYPE[wtype] + (1000 * QNT_VERSION if wtype != qref.F32 else 0)
        w(struct.pack("<6i", hp["n_vocab"], hp["n_ctx"], hp["n_embd"], hp["n_head"], hp["n_layer"], ftype))
        w(struct.pack("<i", hp["n_vocab"]))
        for word in vocab(hp["n_vocab"]):
            w(struct.pack("<I", len(word)) + word)
        for name, ne, vals, is_mat in _tensors(hp, seed):
            t = wtype if is_mat else qref.F32
            data = qref.quantize(t, vals, n_per_row=ne[0]).tobytes() if t != qref.F32 else vals.tobytes()
            nm = name.encode()
            w(struct.pack("<3i", len(ne), len(nm), t) + struct.pack(f"<{len(ne)}i", *ne) + nm)
            w(data)
    return h.hexdigest()
