"""GPT-2 pipeline split with REAL stages (gpt2.pipeline_generate): two ranks, each holding a
layer range of the small golden checkpoint, run the ring protocol of the multi-GPU bench and must
generate exactly what one whole-model stage generates for every micro-batch.

* >= 2 gfx950 GPUs: rank r on GPU r, RCCL ("nccl") moves the hidden state / tokens over xGMI;
  plus the reference's own ggml_backend_sched splitting the graph over 2 plugin devices
  (oracle/_ref/gpt2_ref --plugin --devices 2, cross-device cpy_tensor_async) vs the golden logits.
* one GPU (the test box): both ranks share GPU 0 and exchange through host memory over gloo
  (RCCL refuses two ranks on one device) — the same stages, ring schedule and hand-offs.
"""
import os
import socket
import subprocess
import tempfile

import numpy as np
import pytest

import gpt2_synth
import qref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "gpt2_ref")
pytestmark = pytest.mark.gpu


def _n_gpus():
    import mi355x_qmm as M
    return M.device_count()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _small_model(name="q4_K"):
    import json
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "gpt2_manifest.json")))
    path = os.path.join(tempfile.gettempdir(), f"gpt2_pipe_{name}_{os.getpid()}.bin")
    sha = gpt2_synth.write_model(path, man["hparams"], qref.BY_NAME[name], man["seed"])
    assert sha == man["cases"][name]["model_sha256"]
    return path


PROMPTS = [[40, 72, 73, 83], [52, 72, 0, 9]]
N_NEW = 12


def _rank(rank, world, port, path, split, multi_gpu, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "ggml-gfx906_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist

    import gpt2 as G
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank if multi_gpu else 0)
    if multi_gpu:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    hp = G.read_hparams(path)
    st = G.Stage(hp, *split[rank])
    st.load(path)
    gen = G.pipeline_generate(st, rank, world, PROMPTS, N_NEW, comm_device=None if multi_gpu else "cpu")
    st.free()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, gen))


def test_pipeline_two_stages_match_single_stage():
    import torch
    import torch.multiprocessing as mp

    import gpt2 as G
    path = _small_model()
    hp = G.read_hparams(path)
    world = 2
    split = G.partition_layers(hp["n_layer"], world)
    multi = _n_gpus() >= 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, path, split, multi, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single stage, whole model, same prompts
    st = G.Stage(hp)
    st.load(path)
    want = []
    for pr in PROMPTS:
        c = G.Context(st, 1)
        want.append(G.greedy_generate(c, [pr], N_NEW)[0])
        c.free()
    st.free()
    torch.cuda.synchronize()
    assert res[0] == want, (res[0], want)


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
def test_reference_scheduler_splits_over_two_devices():
    """the reference's ggml_backend_sched places layers on two plugin devices and moves
    activations with our cross-device cpy_tensor_async (hipMemcpyPeerAsync over xGMI). On a
    one-GPU box both plugin devices are GPU 0 (GGML_MI355X_VIRTUAL_DEVICES=2): the graph split,
    the hand-off copies and the stream / event ordering run, with a same-GPU copy for the peer
    copy."""
    env = dict(os.environ)
    if _n_gpus() < 2:
        env["GGML_MI355X_VIRTUAL_DEVICES"] = "2"
    import json
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "gpt2_manifest.json")))
    c = man["cases"]["q4_0"]
    path = _small_model("q4_0")
    out = os.path.join(tempfile.gettempdir(), f"gpt2_plugin2_{os.getpid()}.f32")
    lib = os.path.join(ROOT, "ggml-gfx906_amd", "libggml-hip-mi355x.so")
    r = subprocess.run([REF_BIN, path, "--tokens", ",".join(map(str, c["tokens"][:24])), "--out", out, "--plugin", lib,
                        "--devices", "2"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    import re
    m = re.search(r"(\d+) backends, (\d+) splits", r.stderr)
    assert m and int(m.group(1)) == 3 and int(m.group(2)) >= 2, r.stderr[-500:]   # 2 plugin devices + CPU
    got = np.fromfile(out, np.float32).reshape(24, -1)
    want = np.fromfile(os.path.join(ROOT, "tests", "golden", c["logits"]), np.float32).reshape(len(c["tokens"]), -1)[:24]
    for i in range(24):
        e = float(((got[i].astype(np.float64) - want[i]) ** 2).sum() / (want[i].astype(np.float64) ** 2).sum())
        assert e <= 1e-3, (i, e)


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="oracle/_ref not built")
def test_reference_scheduler_eight_devices_pipelined():
    """configs[4]'s scheduler form at eight devices with sequences in flight: the reference's
    ggml_backend_sched over 8 plugin devices (virtual ones on GPU 0 when the box has fewer GPUs),
    created with parallel = true (GGML_SCHED_MAX_COPIES input copies, event-ordered hand-offs) and
    fed 4 sequences round-robin by ggml_backend_sched_graph_compute_async. Checks:
      * the serial pass (one graph at a time) of the golden prompt matches the golden logits;
      * the KV the pipelined pass wrote gives the serial pass's logits for every sequence
        (async_vs_serial_nmse, gpt2_ref --n-seq)."""
    env = dict(os.environ)
    if _n_gpus() < 8:
        env["GGML_MI355X_VIRTUAL_DEVICES"] = "8"
    import json
    import re
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "gpt2_manifest.json")))
    c = man["cases"]["q4_0"]
    path = _small_model("q4_0")
    out = os.path.join(tempfile.gettempdir(), f"gpt2_plugin8_{os.getpid()}.f32")
    lib = os.path.join(ROOT, "ggml-gfx906_amd", "libggml-hip-mi355x.so")
    r = subprocess.run([REF_BIN, path, "--tokens", ",".join(map(str, c["tokens"][:16])), "--out", out, "--plugin", lib,
                        "--devices", "8", "--parallel", "--n-seq", "4", "--time-tokens", "8"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    m = re.search(r"(\d+) backends, (\d+) splits", r.stderr)
    assert m and int(m.group(2)) >= 2, r.stderr[-500:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["n_seq"] == 4 and j["parallel"] == 1 and j["tokens"] == 32, j
    assert j["async_vs_serial_nmse"] <= 1e-10, j
    got = np.fromfile(out, np.float32).reshape(16, -1)
    want = np.fromfile(os.path.join(ROOT, "tests", "golden", c["logits"]), np.float32).reshape(len(c["tokens"]), -1)[:16]
    for i in range(16):
        e = float(((got[i].astype(np.float64) - want[i]) ** 2).sum() / (want[i].astype(np.float64) ** 2).sum())
        assert e <= 1e-3, (i, e)
