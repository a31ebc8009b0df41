"""GPT-2 decode engine (include/ggml-mi355x-gpt2.h, ggml-gfx906_amd/gpt2.py) vs the reference.

Oracle: the reference's own ggml-cpu graph of examples/gpt-2/main-sched.cpp:553-858, run by
oracle/_ref/gpt2_ref (built from /root/reference sources). Golden logits for small synthetic
checkpoints of every hot weight type are committed (tests/golden/gpt2_*.logits.f32, made by
oracle/gen_gpt2_golden.py); the checkpoints are regenerated bit-identically from their seed
(sha256 checked). At the full 117M shape the oracle binary runs live next to the engine.

Tolerances, per position (NMSE, the reference's own measure, tests/test-backend-ops.cpp:
3106-3108, whose per-op bar is 5e-4):
  * engine vs the EXACT forward (oracle/gpt2_np.py: float64 on the bit-exact dequantized
    weights, unquantized activations): <= 5e-4 — the engine is as close to the exact product
    as one reference op is allowed to be;
  * engine vs the reference's ggml-cpu logits: <= 1e-3. Both sides quantize activations
    (ggml-cpu: Q8_0 blocks for Q4_0/Q8_0 weights, coarser per-256 Q8_K for the K-quants,
    src/ggml-cpu/ggml-cpu.c:1264-1299; ours: int8 per 32), so each sits up to ~5e-4 from
    exact (measured: ggml-cpu 2e-4 for Q4_0/Q8_0, 4.3e-4 for the K-quants, pinned by
    test_reference_cpu_is_near_exact) and their difference is bounded by the sum.
"""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import gpt2 as G
import gpt2_synth
import qref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "gpt2_ref")
MANIFEST = json.load(open(os.path.join(GOLDEN, "gpt2_manifest.json")))
SMALL = MANIFEST["hparams"]
NMSE_MAX = 5e-4          # vs the exact forward
NMSE_VS_REF = 1e-3       # vs the reference ggml-cpu (two quantized-activation paths)


def nmse(a, b):
    return float(((a.astype(np.float64) - b) ** 2).sum() / max((b.astype(np.float64) ** 2).sum(), 1e-30))


_models = {}


def small_model(name: str) -> str:
    """the golden case's checkpoint, regenerated from its seed and pinned by sha256"""
    if name not in _models:
        path = os.path.join(tempfile.gettempdir(), f"gpt2_test_{name}_{os.getpid()}.bin")
        sha = gpt2_synth.write_model(path, SMALL, qref.BY_NAME[name], MANIFEST["seed"])
        assert sha == MANIFEST["cases"][name]["model_sha256"], "synthetic checkpoint generator drifted"
        _models[name] = path
    return _models[name]


def golden_logits(name: str) -> np.ndarray:
    c = MANIFEST["cases"][name]
    return np.fromfile(os.path.join(GOLDEN, c["logits"]), np.float32).reshape(len(c["tokens"]), SMALL["n_vocab"])


# ------------------------------------------------------------------------------------------
# CPU: layer partition, checkpoint generator, oracle pin, header / exports, ring protocol
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_layer,n_stages", [(12, 1), (12, 2), (12, 4), (12, 8), (12, 12), (3, 2), (24, 8), (48, 8)])
def test_partition_layers(n_layer, n_stages):
    parts = G.partition_layers(n_layer, n_stages)
    assert len(parts) == n_stages
    assert parts[0][0] == 0 and parts[-1][1] == n_layer
    for (a0, a1), (b0, b1) in zip(parts, parts[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in parts]
    assert min(sizes) >= 1
    # the last stage also runs the head: it never gets more layers than the others
    assert sizes[-1] <= min(sizes[:-1] or sizes) + 1
    assert max(sizes) - min(sizes) <= 2


def test_partition_rejects():
    with pytest.raises(ValueError):
        G.partition_layers(3, 4)


@pytest.mark.parametrize("name", sorted(MANIFEST["cases"]))
def test_synthetic_checkpoint_is_pinned(name):
    small_model(name)


def test_read_hparams_host_only():
    hp = G.read_hparams(small_model("q4_0"))
    assert hp == dict(SMALL, ftype=2)
    bad = os.path.join(tempfile.gettempdir(), f"not_gpt2_{os.getpid()}.bin")
    open(bad, "wb").write(b"\0" * 64)
    with pytest.raises(Exception):
        G.read_hparams(bad)


_exact = {}


def exact_logits(name: str, n: int) -> np.ndarray:
    import gpt2_np
    if (name, n) not in _exact:
        _exact[(name, n)] = gpt2_np.logits(small_model(name), MANIFEST["cases"][name]["tokens"][:n])
    return _exact[(name, n)]


@pytest.mark.parametrize("name", sorted(MANIFEST["cases"]))
def test_reference_cpu_is_near_exact(name):
    """pins the float64 forward to the reference: ggml-cpu's logits sit within its own
    per-op bar of the exact product on every position"""
    want = exact_logits(name, 12)
    got = golden_logits(name)[:12]
    errs = [nmse(got[i], want[i]) for i in range(12)]
    assert max(errs) <= NMSE_MAX, errs
    assert (got.argmax(1) == want.argmax(1)).mean() >= 0.9


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
@pytest.mark.parametrize("name", ["q4_0", "q4_K"])
def test_oracle_reproduces_golden(name):
    """the reference binary regenerates the committed logits bit for bit"""
    c = MANIFEST["cases"][name]
    out = os.path.join(tempfile.gettempdir(), f"gpt2_oracle_{name}_{os.getpid()}.f32")
    subprocess.run([REF_BIN, small_model(name), "--tokens", ",".join(map(str, c["tokens"])), "--out", out, "--threads", "1"],
                   check=True, capture_output=True)
    got = np.fromfile(out, np.float32).reshape(len(c["tokens"]), -1)
    assert np.array_equal(got, golden_logits(name))


def test_gpt2_header_exports():
    names = G.exported_api()
    for must in ("ggml_mi355x_gpt2_model_init", "ggml_mi355x_gpt2_model_load", "ggml_mi355x_gpt2_decode",
                 "ggml_mi355x_gpt2_ctx_init", "ggml_mi355x_memcpy"):
        assert must in names
    lib = G.lib()
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", G.Q.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported


def test_model_init_rejects_bad_hparams():
    for bad in (dict(n_head=5), dict(ftype=3), dict(n_embd=4096 + 64, n_head=65)):
        hp = dict(G.make_hparams(), **bad)
        with pytest.raises(G.Q.Mi355xError):
            G.Stage(hp)


def _ring_worker(rank, world, port, n_micro, n_ticks, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    E = 8
    pipe = G.Pipeline(rank, world, n_micro, E, "cpu")
    log = []

    # mock stage: stage r adds (r + 1) to a hidden vector; the last stage emits the "token"
    # = hidden[0] (bit-packed like the engine's int32 ids); stage 0 embeds token t as [t]*E
    def stage(mb, inbuf, valid):
        out = inbuf.clone()
        if rank == 0:
            tok = inbuf.view(torch.int32)[0].item()
            out = torch.full((E,), float(tok), dtype=torch.float32)
        out += rank + 1
        if rank == world - 1:
            t = torch.zeros(E, dtype=torch.int32)
            t[0] = int(out[0].item())
            out = t.view(torch.float32)
        if valid:
            log.append((mb, float(inbuf[0]) if rank else int(inbuf.view(torch.int32)[0])))
        return out

    def first(mb):
        t = torch.zeros(E, dtype=torch.int32)
        t[0] = 100 * mb
        return t.view(torch.float32)

    done = pipe.run(n_ticks, stage, first)
    q.put((rank, done, log))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_micro", [(2, 1), (2, 3), (3, 2)])
def test_pipeline_rejects_unsupported_micro_batching(world, n_micro):
    with pytest.raises(ValueError):
        G.Pipeline(0, world, n_micro, 8, "cpu")


@pytest.mark.parametrize("world,n_micro", [(2, 2), (3, 3), (4, 4), (8, 8)])
def test_pipeline_ring_gloo(world, n_micro):
    """ring protocol on CPU/gloo: every micro-batch's token advances by sum(r+1) per lap
    (world 8 = the driver's 8-GPU scaling run)"""
    import multiprocessing as mp
    import socket
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:   # a port the OS just handed out, not a random guess
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n_ticks = 4 * world + 3
    ps = [ctx.Process(target=_ring_worker, args=(r, world, port, n_micro, n_ticks, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, done, log = q.get(timeout=120)
        res[r] = (done, log)
    for p in ps:
        p.join(timeout=60)
    inc = sum(r + 1 for r in range(world))
    # stage 0 sees, for micro-batch mb, tokens 100 mb, 100 mb + inc, 100 mb + 2 inc, ...
    seen = {}
    for mb, tok in res[0][1]:
        seen.setdefault(mb, []).append(tok)
    assert sorted(seen) == list(range(n_micro))
    for mb, toks in seen.items():
        assert toks == [100 * mb + i * inc for i in range(len(toks))], (mb, toks)
    assert res[0][0] == n_ticks
    for r in range(world):
        assert res[r][0] == n_ticks - r


# ------------------------------------------------------------------------------------------
# GPU: engine vs reference logits
# ------------------------------------------------------------------------------------------
def _run_logits(path, tokens, n_seq=1, graph=True, split=None):
    """feed `tokens` one per step (teacher forcing) and return logits[pos][n_vocab] of seq 0.
    split=[(l0,l1),...] runs the stages in sequence on this GPU, handing the hidden state over
    with device copies (the same buffers the RCCL pipeline moves)."""
    import torch
    hp = G.read_hparams(path)
    parts = split or [(0, hp["n_layer"])]
    stages = [G.Stage(hp, a, b) for a, b in parts]
    for s in stages:
        s.load(path)
    ctxs = [G.Context(s, n_seq) for s in stages]
    st = torch.cuda.current_stream().cuda_stream
    zeros = torch.zeros(n_seq, dtype=torch.int32, device="cuda")
    for c in ctxs:
        c.set_pos(zeros.data_ptr(), st)
    V = hp["n_vocab"]
    out = []
    for t in tokens:
        tk = torch.full((n_seq,), t, dtype=torch.int32, device="cuda")
        ctxs[0].set_tokens(tk.data_ptr(), st)
        for i, c in enumerate(ctxs):
            if i:
                c._copy(c.hidden_ptr, ctxs[i - 1].hidden_ptr, c.hidden_bytes, st)
            c.decode(st, graph)
        lg = torch.empty((n_seq, V), dtype=torch.float32, device="cuda")
        ctxs[-1]._copy(lg.data_ptr(), ctxs[-1].logits_ptr, 4 * n_seq * V, st)
        out.append(lg.cpu().numpy())
    torch.cuda.synchronize()
    for c in ctxs:
        c.free()
    for s in stages:
        s.free()
    return np.stack(out)   # [pos][seq][vocab]


@pytest.mark.gpu
@pytest.mark.parametrize("block", ["1", "0"], ids=["two_launch_layer", "five_launch_layer"])
@pytest.mark.parametrize("name", sorted(MANIFEST["cases"]))
def test_engine_matches_reference_logits(name, block, monkeypatch):
    """both layer forms (csrc/gpt2_block.hip, and the five-launch fallback used above
    n_embd 1024) against the reference's logits and the exact forward"""
    monkeypatch.setenv("GGML_MI355X_GPT2_BLOCK", block)
    c = MANIFEST["cases"][name]
    got = _run_logits(small_model(name), c["tokens"])[:, 0]
    assert np.isfinite(got).all()
    want = golden_logits(name)
    errs = [nmse(got[i], want[i]) for i in range(len(want))]
    assert max(errs) <= NMSE_VS_REF, errs
    assert (got.argmax(1) == want.argmax(1)).mean() >= 0.9
    n = min(len(want), 24)
    ex = exact_logits(name, n)
    errs = [nmse(got[i], ex[i]) for i in range(n)]
    assert max(errs) <= NMSE_MAX, errs


@pytest.mark.gpu
def test_graph_replay_equals_eager():
    c = MANIFEST["cases"]["q4_0"]
    a = _run_logits(small_model("q4_0"), c["tokens"][:20], graph=True)
    b = _run_logits(small_model("q4_0"), c["tokens"][:20], graph=False)
    assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [[(0, 1), (1, 3)], [(0, 1), (1, 2), (2, 3)]])
def test_stage_split_equals_single_stage(split):
    c = MANIFEST["cases"]["q4_K"]
    a = _run_logits(small_model("q4_K"), c["tokens"])
    b = _run_logits(small_model("q4_K"), c["tokens"], split=split)
    assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("n_seq", [2, 3, 5, 8])
def test_batched_sequences_match_single(n_seq):
    """n_seq sequences decoded together (wider mat-vec column groups) give each sequence the
    single-sequence result"""
    c = MANIFEST["cases"]["q8_0"]
    one = _run_logits(small_model("q8_0"), c["tokens"])[:, 0]
    many = _run_logits(small_model("q8_0"), c["tokens"], n_seq=n_seq)
    for s in range(n_seq):
        assert np.allclose(many[:, s], one, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_greedy_generate_device_loop():
    """device-resident greedy loop (argmax feeds the next step) equals host-side argmax of the
    teacher-forced logits"""
    path = small_model("q4_0")
    hp = G.read_hparams(path)
    st = G.Stage(hp)
    st.load(path)
    ctx = G.Context(st, 2)
    prompt = [[40, 72, 73], [40, 72, 73]]
    gen = G.greedy_generate(ctx, prompt, 10)
    ctx.free()
    st.free()
    assert gen[0] == gen[1]
    seq = prompt[0] + gen[0]
    lg = _run_logits(path, seq[:-1])[:, 0]
    assert lg[2:].argmax(1).tolist() == gen[0]


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
def test_engine_117m_matches_reference_live():
    """full GPT-2 117M shape (Q4_0, synthetic weights): engine vs the reference ggml-cpu
    graph run live on this host, 80 positions (crosses the attention kernel's 64-key pass)"""
    path = os.path.join(tempfile.gettempdir(), f"gpt2_117m_q4_0_{os.getpid()}.bin")
    gpt2_synth.write_model(path, gpt2_synth.GPT2_117M, qref.Q4_0, 1234)
    toks = [(31 * i + 7) % 50257 for i in range(80)]
    out = path + ".logits"
    subprocess.run([REF_BIN, path, "--tokens", ",".join(map(str, toks)), "--out", out, "--threads", "16"], check=True,
                   capture_output=True, timeout=100)
    want = np.fromfile(out, np.float32).reshape(len(toks), -1)
    got = _run_logits(path, toks)[:, 0]
    errs = [nmse(got[i], want[i]) for i in range(len(toks))]
    os.remove(path)
    assert max(errs) <= NMSE_VS_REF, max(errs)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
def test_reference_scheduler_drives_plugin():
    """drop-in: the reference's ggml_backend_sched runs the GPT-2 graph with our plugin as the
    GPU backend (weights + KV on MI355X, ops split by supports_op); logits match ggml-cpu"""
    c = MANIFEST["cases"]["q4_0"]
    out = os.path.join(tempfile.gettempdir(), f"gpt2_plugin_{os.getpid()}.f32")
    r = subprocess.run([REF_BIN, small_model("q4_0"), "--tokens", ",".join(map(str, c["tokens"][:24])), "--out", out,
                        "--plugin", G.Q.LIB_PATH, "--devices", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.fromfile(out, np.float32).reshape(24, -1)
    want = golden_logits("q4_0")[:24]
    errs = [nmse(got[i], want[i]) for i in range(24)]
    assert max(errs) <= NMSE_VS_REF, errs


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_reference_scheduler_layer_fusion(name):
    """drop-in, whole-layer fusion (backend.cpp plan_layers): the reference scheduler's GPT-2 with
    the plugin runs every decode layer as the engine's two launches (the debug log names each
    fused layer, chained layers pass the residual on as partial slabs) and its logits match the
    golden ggml-cpu logits, as the node-by-node path (GGML_MI355X_LAYER_FUSION=0) does. Q4_0 / Q8_0
    read the c_proj / MLP-projection copies the plugin makes, K-quants read the ggml rows in place."""
    c = MANIFEST["cases"][name]
    n = min(24, len(c["tokens"]))
    want = golden_logits(name)[:n]
    got = {}
    for fuse in ("1", "0"):
        out = os.path.join(tempfile.gettempdir(), f"gpt2_plugin_lf{fuse}_{name}_{os.getpid()}.f32")
        env = dict(os.environ, GGML_MI355X_LAYER_FUSION=fuse, GGML_MI355X_DEBUG="1")
        r = subprocess.run([REF_BIN, small_model(name), "--tokens", ",".join(map(str, c["tokens"][:n])), "--out", out,
                            "--plugin", G.Q.LIB_PATH, "--devices", "1"], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        fused = [ln for ln in r.stderr.splitlines() if "layer fused" in ln]
        if fuse == "1":
            # every decode graph (positions 1 .. n-1) fuses all its layers, chained
            assert len(fused) >= (n - 1) * SMALL["n_layer"], (len(fused), [ln for ln in r.stderr.splitlines() if "not fused" in ln][:8])
            assert any("residual from the previous layer" in ln for ln in fused) or SMALL["n_layer"] == 1
            # the decode graphs differ only in their position, which the fused layers read from the
            # backend's position word: after the first decode step's capture every step replays it
            replays = [ln for ln in r.stderr.splitlines() if "hipGraph replayed" in ln and "position word" in ln]
            assert len(replays) >= n - 4, (len(replays), r.stderr[-1500:])
        else:
            assert not fused
        got[fuse] = np.fromfile(out, np.float32).reshape(n, -1)
        os.remove(out)
    for fuse, lg in got.items():
        errs = [nmse(lg[i], want[i]) for i in range(n)]
        assert max(errs) <= NMSE_VS_REF, (fuse, max(errs))
    assert max(nmse(got["1"][i], got["0"][i]) for i in range(n)) <= NMSE_VS_REF
