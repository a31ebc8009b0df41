"""gpt2.py — host driver of the MI355X GPT-2 decode engine (include/ggml-mi355x-gpt2.h).

The reference runs examples/gpt-2 as a ggml graph on one GPU + CPU (main-sched.cpp:109-152)
and, across devices, relies on ggml_backend_sched moving activations between backends
(cpy_tensor_async, src/ggml-backend.cpp:1383). Here every GPU runs one PIPELINE STAGE in its
own process (torch.distributed, RCCL over xGMI):

  * stage r owns a contiguous layer range (partition_layers); stage 0 also embeds the tokens,
    the last stage also runs ln_f + lm_head + greedy argmax;
  * n_micro micro-batches of n_seq sequences circulate round the ring: at tick k stage r works
    on micro-batch (k - r) mod n_micro, then ONE batched send/recv moves every stage's output
    to its successor (hidden state, n_seq x n_embd f32; from the last stage back to stage 0 the
    next token ids) — one RCCL exchange per tick, no other collective on the data path;
  * with n_micro = n_stages every stage is busy every tick once the ring is full.

Compute goes through the C ABI only (libggml-hip-mi355x.so); torch provides the device, the
stream and torch.distributed — plumbing, not compute. No CPU fallback: a missing library or
device raises.
"""
from __future__ import annotations

import ctypes as C
import os

import mi355x_qmm as Q

HEADER = os.path.join(os.path.dirname(Q.HERE), "include", "ggml-mi355x-gpt2.h")
FTYPE_OF = {Q.F32: 0, Q.Q4_0: 2, Q.Q8_0: 7, Q.Q4_K: 12, Q.Q5_K: 13, Q.Q6_K: 14}
GPT2_117M = dict(n_vocab=50257, n_ctx=1024, n_embd=768, n_head=12, n_layer=12)


class HParams(C.Structure):
    """ggml_mi355x_gpt2_hparams (main-sched.cpp:44-52)"""
    _fields_ = [(n, C.c_int32) for n in ("n_vocab", "n_ctx", "n_embd", "n_head", "n_layer", "ftype")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_bound = False


def lib():
    global _bound
    L = Q.lib()
    if not _bound:
        vp, i32 = C.c_void_p, C.c_int32
        L.ggml_mi355x_gpt2_read_hparams.argtypes = [C.c_char_p, C.POINTER(HParams)]
        L.ggml_mi355x_gpt2_model_init.argtypes = [C.POINTER(HParams), i32, i32, C.POINTER(vp)]
        L.ggml_mi355x_gpt2_model_load.argtypes = [vp, C.c_char_p]
        L.ggml_mi355x_gpt2_model_tensor.argtypes = [vp, C.c_char_p, C.POINTER(vp), C.POINTER(i32), C.POINTER(C.c_int64 * 2)]
        L.ggml_mi355x_gpt2_model_bytes.argtypes = [vp]
        L.ggml_mi355x_gpt2_model_bytes.restype = C.c_int64
        L.ggml_mi355x_gpt2_model_free.argtypes = [vp]
        L.ggml_mi355x_gpt2_model_free.restype = None
        L.ggml_mi355x_gpt2_ctx_init.argtypes = [vp, i32, C.POINTER(vp)]
        L.ggml_mi355x_gpt2_ctx_buffers.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]
        L.ggml_mi355x_gpt2_decode.argtypes = [vp, vp, i32]
        L.ggml_mi355x_gpt2_ctx_free.argtypes = [vp]
        L.ggml_mi355x_gpt2_ctx_free.restype = None
        L.ggml_mi355x_memcpy.argtypes = [vp, vp, C.c_size_t, vp]
        _bound = True
    return L


def exported_api() -> list:
    import re
    txt = open(HEADER).read()
    txt = re.sub(r"#define GGML_MI355X_API[^\n]*", "", txt)
    return re.findall(r"GGML_MI355X_API\s+[\w\s\*]*?\b(\w+)\s*\(", txt)


def read_hparams(path: str) -> dict:
    hp = HParams()
    Q._check(lib().ggml_mi355x_gpt2_read_hparams(path.encode(), C.byref(hp)), f"read_hparams({path})")
    return hp.as_dict()


def make_hparams(wtype: int = Q.Q4_0, **kw) -> dict:
    hp = dict(GPT2_117M)
    hp.update(kw)
    hp["ftype"] = FTYPE_OF[wtype]
    return hp


def partition_layers(n_layer: int, n_stages: int, head_cost: float = 1.0, embed_cost: float = 0.25) -> list:
    """Contiguous layer ranges [(l0, l1), ...], one per stage, minimizing the slowest stage
    (the pipeline's tick), where a layer costs 1, the last stage's ln_f + lm_head `head_cost`
    and the first stage's embedding `embed_cost` (decode is launch-bound: a layer is five
    launches, the head one wide mat-vec). Every stage gets at least one layer; exact DP over
    split points (n_layer is tens)."""
    if n_stages < 1 or n_stages > n_layer:
        raise ValueError(f"cannot split {n_layer} layers over {n_stages} stages")
    INF = float("inf")

    def cost(s, a, b):
        return (b - a) + (embed_cost if s == 0 else 0.0) + (head_cost if s == n_stages - 1 else 0.0)

    # best[s][b] = (max stage cost, split) for stages 0..s covering layers [0, b)
    best = [[(INF, None)] * (n_layer + 1) for _ in range(n_stages)]
    for b in range(1, n_layer + 1):
        best[0][b] = (cost(0, 0, b), [(0, b)])
    for s in range(1, n_stages):
        for b in range(s + 1, n_layer + 1):
            for a in range(s, b):
                prev, split = best[s - 1][a]
                if split is None:
                    continue
                c = max(prev, cost(s, a, b))
                if c < best[s][b][0] - 1e-9:
                    best[s][b] = (c, split + [(a, b)])
    return best[n_stages - 1][n_layer][1]


class Stage:
    """One pipeline stage: the weights of layers [l0, l1) on the current device."""

    def __init__(self, hp: dict, l0: int = 0, l1: int | None = None):
        self.hp = dict(hp)
        self.l0, self.l1 = l0, hp["n_layer"] if l1 is None else l1
        h = HParams(*[hp[n] for n, _ in HParams._fields_])
        out = C.c_void_p()
        Q._check(lib().ggml_mi355x_gpt2_model_init(C.byref(h), self.l0, self.l1, C.byref(out)), "gpt2_model_init")
        self.handle = out.value
        self.first, self.last = self.l0 == 0, self.l1 == hp["n_layer"]

    def load(self, path: str) -> None:
        Q._check(lib().ggml_mi355x_gpt2_model_load(self.handle, path.encode()), f"gpt2_model_load({path})")

    def tensor(self, name: str):
        """(device pointer, ggml type, [ne0, ne1]) or None when the tensor is not in this stage."""
        p, t, ne = C.c_void_p(), C.c_int32(), (C.c_int64 * 2)()
        if lib().ggml_mi355x_gpt2_model_tensor(self.handle, name.encode(), C.byref(p), C.byref(t), C.byref(ne)) != 0:
            return None
        return p.value, t.value, [ne[0], ne[1]]

    def tensor_names(self) -> list:
        names = []
        if self.first:
            names += ["model/wte", "model/wpe"]
        if self.last:
            names += ["model/ln_f/g", "model/ln_f/b", "model/lm_head"]
        for i in range(self.l0, self.l1):
            names += [f"model/h{i}/{s}" for s in ("ln_1/g", "ln_1/b", "ln_2/g", "ln_2/b", "attn/c_attn/w", "attn/c_attn/b",
                                                  "attn/c_proj/w", "attn/c_proj/b", "mlp/c_fc/w", "mlp/c_fc/b",
                                                  "mlp/c_proj/w", "mlp/c_proj/b")]
        return names

    def nbytes(self) -> int:
        return int(lib().ggml_mi355x_gpt2_model_bytes(self.handle))

    def fill_synthetic(self, seed: int = 1234) -> None:
        """Random-init weights generated ON THE DEVICE (torch RNG) and quantized by the
        library's own device quantizer (ggml_mi355x_quantize, bit-exact with
        quantize_row_q4_0_ref / q8_0_ref) — no host round trip for 100+ MB of weights. Same
        statistics as tests/gpt2_synth.py (weights std 0.02, gains 1 +- 0.1)."""
        import torch
        g = torch.Generator(device="cuda")
        for k, name in enumerate(self.tensor_names()):
            ptr, t, ne = self.tensor(name)
            g.manual_seed(seed * 1000 + k)
            n = ne[0] * ne[1]
            vals = (torch.rand(n, device="cuda", generator=g) * 2 - 1) * (0.02 * 3 ** 0.5)
            if name.endswith("/g"):
                vals = vals * 5 + 1.0
            if t == Q.F32:
                Q._check(lib().ggml_mi355x_memcpy(ptr, vals.data_ptr(), 4 * n, None), "memcpy")
            else:
                src = Q.tensor(Q.F32, vals.data_ptr(), [ne[0], ne[1], 1, 1], Q.contiguous_nb(Q.F32, ne))
                dst = Q.tensor(t, ptr, [ne[0], ne[1], 1, 1], Q.contiguous_nb(t, ne))
                Q.quantize(src, dst)
            torch.cuda.synchronize()

    def free(self) -> None:
        if self.handle:
            lib().ggml_mi355x_gpt2_model_free(self.handle)
            self.handle = None


class Context:
    """A decode context of a stage: n_seq sequences, their KV cache, positions and buffers."""

    def __init__(self, stage: Stage, n_seq: int = 1):
        self.stage, self.n_seq = stage, n_seq
        out = C.c_void_p()
        Q._check(lib().ggml_mi355x_gpt2_ctx_init(stage.handle, n_seq, C.byref(out)), "gpt2_ctx_init")
        self.handle = out.value
        t, p, h, lg = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        Q._check(lib().ggml_mi355x_gpt2_ctx_buffers(self.handle, C.byref(t), C.byref(p), C.byref(h), C.byref(lg)), "ctx_buffers")
        self.tokens_ptr, self.pos_ptr, self.hidden_ptr, self.logits_ptr = t.value, p.value, h.value, lg.value
        E = stage.hp["n_embd"]
        self.hidden_bytes = 4 * n_seq * E

    # stream-ordered copies in / out of the context (ptr: host or device address)
    def _copy(self, dst, src, nbytes, stream=None):
        Q._check(lib().ggml_mi355x_memcpy(dst, src, nbytes, stream), "memcpy")

    def set_tokens(self, ptr, stream=None):
        self._copy(self.tokens_ptr, ptr, 4 * self.n_seq, stream)

    def set_pos(self, ptr, stream=None):
        self._copy(self.pos_ptr, ptr, 4 * self.n_seq, stream)

    def decode(self, stream=None, graph: bool = True) -> None:
        """One step for all n_seq sequences (asynchronous on `stream`, a hipStream_t)."""
        if graph and not stream:
            graph = False   # the legacy default stream is not capturable
        Q._check(lib().ggml_mi355x_gpt2_decode(self.handle, stream, 1 if graph else 0), "gpt2_decode")

    def free(self) -> None:
        if self.handle:
            lib().ggml_mi355x_gpt2_ctx_free(self.handle)
            self.handle = None


def _stream_ptr():
    import torch
    return torch.cuda.current_stream().cuda_stream


def greedy_generate(ctx: Context, prompt, n_new: int, graph: bool = True):
    """Single-stage (whole model on this GPU) greedy decode for ctx.n_seq identical-length
    prompts (list of lists). Prompt tokens are fed one per step (decode path), then the
    engine's own argmax output feeds back on the device. Returns the generated ids per
    sequence."""
    import torch
    assert ctx.stage.first and ctx.stage.last
    S = ctx.n_seq
    P = len(prompt[0])
    toks = torch.tensor(prompt, dtype=torch.int32).t().contiguous().cuda()   # [P][S]
    st = _stream_ptr()
    zeros = torch.zeros(S, dtype=torch.int32, device="cuda")
    ctx.set_pos(zeros.data_ptr(), st)
    out = torch.empty((n_new, S), dtype=torch.int32, device="cuda")
    for i in range(P):
        ctx.set_tokens(toks[i].data_ptr(), st)
        ctx.decode(st, graph)
    for j in range(n_new):
        ctx._copy(out[j].data_ptr(), ctx.tokens_ptr, 4 * S, st)
        if j + 1 < n_new:
            ctx.decode(st, graph)
    torch.cuda.synchronize()
    return out.t().cpu().tolist()


class Pipeline:
    """Ring pipeline over torch.distributed (see module docstring). `stage_fn(mb, inbuf)` runs
    one decode step of this rank's stage for micro-batch mb whose input is `inbuf` and returns
    the output buffer to forward (a torch tensor of `msg_elems` f32). The protocol is
    independent of the compute, so it is tested on CPU with gloo and a numpy stage."""

    def __init__(self, rank: int, world: int, n_micro: int, msg_elems: int, device, group=None, comm_device=None):
        """device: where stage outputs live; comm_device: where the exchange happens (default
        = device; "cpu" stages every message through host memory, for process groups whose
        backend cannot move device tensors, e.g. gloo with two ranks sharing one GPU)"""
        import torch
        if n_micro != world:
            # the tick schedule below keeps exactly one micro-batch per stage in flight: with
            # fewer, stage 0 would read the ring before the last stage has produced a token; with
            # more, a token arriving on the ring would be dropped for the next prompt
            raise ValueError(f"Pipeline needs n_micro == world (got n_micro={n_micro}, world={world})")
        self.rank, self.world, self.n_micro = rank, world, n_micro
        self.next, self.prev = (rank + 1) % world, (rank - 1) % world
        self.comm_device = torch.device(comm_device if comm_device is not None else device)
        self.recv = [torch.zeros(msg_elems, dtype=torch.float32, device=self.comm_device) for _ in range(2)]
        self.group = group
        self.cur = 0
        self.k = 0

    def tick(self, k: int, stage_fn, first_input_fn) -> bool:
        """Tick k: this rank holds micro-batch m = (k - rank) mod n_micro, valid once k >= rank.
        Stage 0's input on its first visit of a micro-batch (k < n_micro) comes from
        first_input_fn(mb) (the prompt), afterwards from the ring (the last stage's tokens).
        Ends with the tick's one batched exchange. Returns whether a real step was computed."""
        import torch.distributed as dist
        mb = (k - self.rank) % self.n_micro
        valid = k >= self.rank
        if self.rank == 0 and k < self.n_micro:
            inbuf = first_input_fn(mb)
        else:
            inbuf = self.recv[self.cur]
        out = stage_fn(mb, inbuf, valid)
        if out.device != self.comm_device:
            out = out.to(self.comm_device)     # synchronizes the producing stream
        if self.world > 1:
            nxt = 1 - self.cur
            ops = [dist.P2POp(dist.isend, out, self.next, self.group),
                   dist.P2POp(dist.irecv, self.recv[nxt], self.prev, self.group)]
            for r in dist.batch_isend_irecv(ops):
                r.wait()
            self.cur = nxt
        else:
            self.recv[self.cur].copy_(out)
        return valid

    def run(self, n_ticks: int, stage_fn, first_input_fn) -> int:
        """n_ticks more ticks; returns how many real steps this rank computed"""
        done = 0
        for _ in range(n_ticks):
            done += self.tick(self.k, stage_fn, first_input_fn)
            self.k += 1
        return done


def pipeline_generate(stage: Stage, rank: int, world: int, prompts: list, n_new: int, comm_device=None, group=None,
                      graph: bool = True):
    """Greedy generation through the ring pipeline with real stages: micro-batch mb (one
    sequence, prompt prompts[mb]; n_micro = world) walks the stages every `world` ticks. Stage
    0 feeds the prompt one token per visit, then the token the last stage sent round the ring.
    Returns the n_new generated ids per micro-batch on rank 0 (None elsewhere). Collective:
    every rank calls it with its own stage."""
    import torch
    P = len(prompts[0])
    assert len(prompts) == world and all(len(p) == P for p in prompts)
    dev = torch.device("cuda", torch.cuda.current_device())
    st = torch.cuda.current_stream().cuda_stream
    E = stage.hp["n_embd"]
    ctxs = [Context(stage, 1) for _ in range(world)]
    zero = torch.zeros(1, dtype=torch.int32, device=dev)
    for c in ctxs:
        c.set_pos(zero.data_ptr(), st)
    send = [torch.zeros(E, dtype=torch.float32, device=dev) for _ in range(world)]
    steps = [0] * world
    gen = [[] for _ in range(world)]
    host_tok = torch.zeros(1, dtype=torch.int32)

    def stage_fn(mb, inbuf, valid):
        if valid and steps[mb] < P + n_new:
            c = ctxs[mb]
            k = steps[mb]
            if stage.first:
                if k < P:
                    tok = torch.tensor([prompts[mb][k]], dtype=torch.int32, device=dev)
                else:
                    host_tok.copy_(inbuf.view(torch.int32)[:1].cpu())
                    gen[mb].append(int(host_tok[0]))
                    tok = host_tok.to(dev)
                c.set_tokens(tok.data_ptr(), st)
            else:
                c._copy(c.hidden_ptr, inbuf.data_ptr(), c.hidden_bytes, st)
            c.decode(st, graph)
            steps[mb] += 1
            src = c.tokens_ptr if stage.last else c.hidden_ptr
            c._copy(send[mb].data_ptr(), src, 4 if stage.last else c.hidden_bytes, st)
        return send[mb]

    pipe = Pipeline(rank, world, world, E, dev, group=group, comm_device=comm_device)
    first = lambda mb: send[mb]  # noqa: E731  (stage 0 ignores its input while in the prompt)
    pipe.run(world * (P + n_new) + world, stage_fn, first)
    torch.cuda.synchronize()
    for c in ctxs:
        c.free()
    return gen if rank == 0 else None
