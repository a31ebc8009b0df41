"""oracle/gpt2_np.py — TEST INFRASTRUCTURE: float64 GPT-2 forward on dequantized weights.

The exact-arithmetic companion of oracle/_ref/gpt2_ref: the same legacy checkpoint, the same
graph (examples/gpt-2/main-sched.cpp:553-858: norm -> *g + b, c_attn, causal softmax
attention with 1/sqrt(d) scaling, c_proj + residual, norm, c_fc, GELU (tanh form),
c_proj + residual, ln_f, lm_head tied to wte), but every weight is dequantized once with the
oracle's bit-exact dequantize_row_* and all arithmetic runs in float64 with unquantized
activations. It measures how far any quantized-activation implementation — the reference's
ggml-cpu (Q8_0 / Q8_K activation blocks) or ours (int8 per 32) — sits from the exact product.
"""
from __future__ import annotations

import struct

import numpy as np

import qref


def load(path: str):
    f = open(path, "rb")
    magic, = struct.unpack("<I", f.read(4))
    assert magic == 0x67676D6C
    n_vocab, n_ctx, n_embd, n_head, n_layer, ftype = struct.unpack("<6i", f.read(24))
    hp = dict(n_vocab=n_vocab, n_ctx=n_ctx, n_embd=n_embd, n_head=n_head, n_layer=n_layer, ftype=ftype % 1000)
    nv, = struct.unpack("<i", f.read(4))
    for _ in range(nv):
        ln, = struct.unpack("<I", f.read(4))
        f.read(ln)
    W = {}
    while True:
        h = f.read(12)
        if len(h) < 12:
            break
        nd, ln, tt = struct.unpack("<3i", h)
        ne = list(struct.unpack(f"<{nd}i", f.read(4 * nd))) + [1]
        name = f.read(ln).decode()
        n = ne[0] * ne[1]
        if tt == qref.F32:
            v = np.frombuffer(f.read(4 * n), np.float32).astype(np.float64)
        else:
            raw = np.frombuffer(f.read(qref.row_size(tt, ne[0]) * ne[1]), np.uint8)
            v = qref.dequantize(tt, raw, n).astype(np.float64)
        W[name] = v.reshape(ne[1], ne[0]) if nd == 2 else v
    W.setdefault("model/lm_head", W["model/wte"])
    return hp, W


def _norm(x, g, b, eps=1e-5):
    mu = x.mean()
    var = ((x - mu) ** 2).mean()
    return (x - mu) / np.sqrt(var + eps) * g + b


def _gelu(x):
    return 0.5 * x * (1.0 + np.tanh(0.7978845608028654 * x * (1.0 + 0.044715 * x * x)))


def logits(path: str, tokens) -> np.ndarray:
    """logits[pos][n_vocab] feeding `tokens` one at a time (float64)"""
    hp, W = load(path)
    E, H, L = hp["n_embd"], hp["n_head"], hp["n_layer"]
    D = E // H
    K = [np.zeros((0, E)) for _ in range(L)]
    V = [np.zeros((0, E)) for _ in range(L)]
    out = []
    for p, t in enumerate(tokens):
        x = W["model/wte"][t] + W["model/wpe"][p]
        for i in range(L):
            pf = f"model/h{i}/"
            h = _norm(x, W[pf + "ln_1/g"], W[pf + "ln_1/b"])
            qkv = W[pf + "attn/c_attn/w"] @ h + W[pf + "attn/c_attn/b"]
            q, k, v = qkv[:E], qkv[E:2 * E], qkv[2 * E:]
            K[i] = np.vstack([K[i], k])
            V[i] = np.vstack([V[i], v])
            a = np.empty(E)
            for hh in range(H):
                s = K[i][:, hh * D:(hh + 1) * D] @ q[hh * D:(hh + 1) * D] / np.sqrt(D)
                s = np.exp(s - s.max())
                s /= s.sum()
                a[hh * D:(hh + 1) * D] = s @ V[i][:, hh * D:(hh + 1) * D]
            x = x + W[pf + "attn/c_proj/w"] @ a + W[pf + "attn/c_proj/b"]
            h = _norm(x, W[pf + "ln_2/g"], W[pf + "ln_2/b"])
            h = _gelu(W[pf + "mlp/c_fc/w"] @ h + W[pf + "mlp/c_fc/b"])
            x = x + W[pf + "mlp/c_proj/w"] @ h + W[pf + "mlp/c_proj/b"]
        out.append(W["model/lm_head"] @ _norm(x, W["model/ln_f/g"], W["model/ln_f/b"]))
    return np.array(out)
