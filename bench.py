#!/usr/bin/env python3
"""bench.py — MI355X quantized MUL_MAT throughput (BASELINE.json metric) on 1..8 GPUs.

Headline workload (N=1, BASELINE.json configs[1]): Q4_0 mat-vec, K=4096, N=4096 rows, M=1
column, HBM-cold. One *step* = ONE GGML_OP_MUL_MAT over a stack of B=64 independent 4096x4096
Q4_0 matrices, each with its own activation column (ggml's batched mat-vec: src0 ne02=64,
src1 ne12=64) — 606 MB of weights per step, > 2x the 256 MB Infinity Cache, so every byte
streams from HBM. value = algorithmic bytes of all steps of all ranks / max-over-ranks wall
time of the timed steps (GB/s).

Why batched: a single 9.5 MB GEMV is bounded by the launch, not by HBM — on MI355X an empty
kernel already costs 1.4-1.6 us of device time and dependent launches on one stream issue
every ~2.8 us (scripts/hbm_probe.hip); the per-matrix numbers are reported beside it
(configs.*_single) so both regimes are visible.

Multi-GPU (one process per GPU over torch.distributed / RCCL): `python bench.py --gpus N`
starts the N ranks itself (a torch.distributed.run child process, before any GPU call) unless
it is already running under torchrun; a rank count different from --gpus is an error. The
headline: every rank runs the same per-GPU workload on its own weights (weak scaling, no
data-path collective — independent matrices partition with no exchange); barriers +
max-over-ranks timing go through torch.distributed. The row-sharded configs (configs.*_rowsplit,
rowsplit.py) split ONE matrix's rows over the N ranks and all-gather dst (RCCL) every call:
strong scaling of a single GEMM with its one exchange step.

Extra fields on the single JSON line:
  roofline      the mat-vec kernel: algorithmic bytes per launch / mean launch duration
                (HIP events around each launch on the launch stream)
  cpu_baseline  the reference's own ggml-cpu (oracle/_ref, built from the reference sources)
                on a bounded sample (Q4_0 4096x4096 mat-vec, rotated weights); falls back
                to the C oracle port
  configs       the other BASELINE.json kernel configs (Q4_K north star, Q4_K/Q5_K/Q6_K
                4096x11008, Q8_0 M=512): GB/s, TFLOP/s, roofline fractions; *_single rows
                are one matrix per launch
  gpt2          the metric's second half, BASELINE.json configs[4]: GPT-2 117M Q4_0 greedy
                decode tokens/s (random-init weights generated and quantized on the device),
                layers pipeline-split over the N ranks (gpt2.py: one stage per GPU, RCCL
                send/recv of the 3 KB/sequence hidden state per tick, N micro-batches in
                flight); at N=1 also the single-stream latency. The reference's ggml-cpu runs
                the same model shape on the host (cpu_baseline.gpt2, oracle/_ref/gpt2_ref).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ggml-gfx906_amd"))

import mi355x_qmm as M  # noqa: E402

MFMA_I8_PEAK_TOPS = 5000.0      # dense int8 MFMA peak (2x the bf16 rate, MI355X_MICROARCH.md MFMA table, no sparsity)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MEASURED_GBS = 6290.0      # float4 copy measured on MI355X (same guide)
# BENCH_ONE_GPU_REHEARSAL=1 with --gpus N: all N ranks share GPU 0 and exchange over gloo through
# host memory — the N > 1 code paths (rank plumbing, row-split all-gather, pipeline ring,
# timing reduction) on a one-GPU box. Its numbers are not scaling numbers.
REHEARSAL = os.environ.get("BENCH_ONE_GPU_REHEARSAL") == "1"


def synthetic_weights(t: int, N: int, K: int, seed: int) -> np.ndarray:
    """Random quant bits with realistic fp16 scales (no oracle involved)."""
    rng = np.random.default_rng(seed)
    nblk = K // M.BLCK[t]
    bs = M.TSIZE[t]
    w = rng.integers(0, 256, size=(N, nblk, bs), dtype=np.uint8)
    d = np.float16(0.01).view(np.uint16)
    dm = np.float16(0.002).view(np.uint16)
    lo, hi = np.uint8(d & 0xFF), np.uint8(d >> 8)
    if t in (M.Q4_0, M.Q8_0):
        w[:, :, 0], w[:, :, 1] = lo, hi
    elif t in (M.Q4_K, M.Q5_K):
        w[:, :, 0], w[:, :, 1] = lo, hi
        w[:, :, 2], w[:, :, 3] = np.uint8(dm & 0xFF), np.uint8(dm >> 8)
    elif t == M.Q6_K:
        w[:, :, 208], w[:, :, 209] = lo, hi
    return w.reshape(N, nblk * bs)


def alg_bytes(t: int, K: int, N: int, Mc: int) -> int:
    return M.row_size(t, K) * N + 4 * K * Mc + 4 * N * Mc


class MatVecSet:
    """`copies` device copies of a stacked weight tensor [K, N, batch] (quantized rows) plus
    activations [K, M, batch] and outputs [N, M, batch]: one launch = one MUL_MAT over the
    whole stack (ne02 = ne12 = batch), rotating over the copies."""

    def __init__(self, torch, t: int, K: int, N: int, Mc: int, batch: int, copies: int, seed: int = 1234,
                 repacked: bool = False):
        self.torch, self.t, self.K, self.N, self.Mc, self.batch, self.copies = torch, t, K, N, Mc, batch, copies
        host = synthetic_weights(t, N, K, seed)                       # one matrix, replicated on device
        one = torch.from_numpy(host.reshape(-1)).cuda()
        self.w = [one.repeat(batch) for _ in range(copies)]
        rng = np.random.default_rng(seed + 1)
        self.x = torch.from_numpy(rng.uniform(-1, 1, size=(batch, Mc, K)).astype(np.float32)).cuda()
        self.y = torch.zeros((batch, Mc, N), dtype=torch.float32, device="cuda")
        nb_a = M.contiguous_nb(t, [K, N, batch])
        self.A = [M.tensor(t, wi.data_ptr(), [K, N, batch, 1], nb_a) for wi in self.w]
        self.B = M.tensor(M.F32, self.x.data_ptr(), [K, Mc, batch, 1], M.contiguous_nb(M.F32, [K, Mc, batch]))
        self.D = M.tensor(M.F32, self.y.data_ptr(), [N, Mc, batch, 1], M.contiguous_nb(M.F32, [N, Mc, batch]))
        self.bytes = alg_bytes(t, K, N, Mc) * batch
        self.flops = 2.0 * K * N * Mc * batch
        # repacked: each weight copy also held in the int8 tile's fragment layout (made once, as a
        # repacked weight buffer does at upload), and the launches use it
        self.rp = None
        if repacked:
            n = M.repack_size(self.A[0])
            self.rp = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(copies)]
            for a, r in zip(self.A, self.rp):
                M.repack(a, r.data_ptr(), n)
            torch.cuda.synchronize()

    def launch(self, i: int, stream=None) -> None:
        if self.rp is not None:
            M.mul_mat_repacked(self.A[i % self.copies], self.rp[i % self.copies].data_ptr(), self.B, self.D, stream)
        else:
            M.mul_mat(self.A[i % self.copies], self.B, self.D, stream)

    def launch_us(self, reps: int) -> float:
        """mean device time per launch: HIP events on the launch stream around `reps` back-to-back
        launches (rotating weight copies, so every launch reads HBM-cold weights)"""
        torch = self.torch
        st = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.launch(0)
        a.record(st)
        for i in range(reps):
            self.launch(i)
        b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / reps

    def graph_period_us(self, n: int) -> float:
        """per-launch period of n back-to-back launches captured in one hipGraph"""
        torch = self.torch
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(n):
                self.launch(i)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):   # capture on the warmed-up stream: its scratch is sized
            for i in range(n):
                self.launch(i)
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / (5 * n)


def config_row(s: MatVecSet, us: float) -> dict:
    gbs = s.bytes / (us * 1e-6) / 1e9
    tf = s.flops / (us * 1e-6) / 1e12
    row = {"us": round(us, 3), "GB/s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
           "TFLOP/s": round(tf, 3)}
    if s.Mc > 8:   # mat-mat path: the int8 tile (v_mfma_i32_32x32x32_i8), priced
        # against the dense int8 peak
        row.update(bound="mfma", mfma_frac_i8=round(tf / MFMA_I8_PEAK_TOPS, 4),
                   graph_period_us=round(s.graph_period_us(16), 3))
    return row


def measured_traffic(key: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc FETCH_SIZE run (profiles/traffic.json),
    corrected as MI355X_MICROARCH.md prescribes; None when absent."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            return json.load(f)[key]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def measured_rocprof(key: str):
    """the headline kernel's rocprofv3 durations from the committed profile of the same command at
    the round's final HEAD (profiles/headline_rocprof.json, scripts/rocprof_headline.py); None
    when absent"""
    try:
        with open(os.path.join(ROOT, "profiles", "headline_rocprof.json")) as f:
            r = json.load(f)[key]
    except (OSError, KeyError, ValueError):
        return None
    return {k: r[k] for k in ("mean_us", "median_us", "launches", "frac_mean", "frac_median", "summary", "round") if k in r}


def rowsplit_configs(torch, world: int, rank: int, reps: int = 20) -> dict:
    """configs.*_rowsplit: ONE matrix row-sharded over the `world` ranks (rowsplit.py, the
    split-buffer partition) and dst all-gathered over RCCL every call — strong scaling of a
    single GEMM with its one exchange step. Collective: every rank calls it. Timed per call
    (barrier + sync around `reps` calls, slowest rank); GB/s counts the whole matrix's
    algorithmic bytes."""
    import rowsplit as RS
    import torch.distributed as dist
    out = {}
    dev = torch.device("cuda", torch.cuda.current_device())
    for name, t, K, N, Mc in (("q4_K_4096x11008_m1_rowsplit", M.Q4_K, 4096, 11008, 1),
                              ("q8_0_4096x4096_m512_rowsplit", M.Q8_0, 4096, 4096, 512)):
        lo, hi = RS.row_split(N, world)[rank]
        copies = 8                                 # rotated weight copies: HBM-cold per call
        w = [torch.from_numpy(synthetic_weights(t, max(hi - lo, 1), K, 1234 + rank).reshape(-1)).to(dev) for _ in range(copies)]
        x = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, (Mc, K)).astype(np.float32)).to(dev)
        y = torch.zeros((Mc, N), dtype=torch.float32, device=dev)
        mms = [RS.ShardedMatMul(torch, t, K, N, rank, world, wi, comm_device="cpu" if REHEARSAL else None) for wi in w]

        def sync():
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()

        for i in range(3):
            mms[i % copies].forward(x, y)
        sync()
        t0 = time.perf_counter()
        for i in range(reps):
            mms[i % copies].forward(x, y)
        sync()
        el = time.perf_counter() - t0
        t_max = max_over_ranks(el, torch.device("cpu") if REHEARSAL else dev) if world > 1 else el
        us = t_max / reps * 1e6
        gbytes = alg_bytes(t, K, N, Mc)
        out[name] = {"us": round(us, 3), "GB/s": round(gbytes / us / 1e3, 1), "TFLOP/s": round(2.0 * K * N * Mc / us / 1e6, 3),
                     "shards": world, "rows_per_shard": [b - a for a, b in RS.row_split(N, world)],
                     "allgather_bytes": 4 * N * Mc if world > 1 else 0, "scaling": "strong",
                     "timing": "host wall per call incl. the RCCL all-gather, slowest rank"}
        del w, mms, x, y
        torch.cuda.empty_cache()
    return out


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the CPU share the GPU box gives one GPU (its harness
    exports OMP_NUM_THREADS=16 and allows no more: 128 cores / 8 GPUs), else all cores here."""
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)


def cgroup_cpu_quota():
    """CPUs of time this job may use (cgroup v2 cpu.max quota / period), None if unlimited"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def ref_cpu_run(exe: str, threads: int, seconds: float, timeout: float):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    try:
        out = subprocess.run([exe, "q4_0", "4096", "4096", "1", str(threads), str(seconds), "32"],
                             capture_output=True, text=True, env=env, timeout=timeout)
    except subprocess.TimeoutExpired:
        return None
    return json.loads(out.stdout.strip().splitlines()[-1]) if out.returncode == 0 else None


def cpu_baseline(seconds: float) -> dict:
    """Reference ggml-cpu (oracle/_ref) on the host cores, bounded sample of the same config.
    The main value uses the job's CPU share (OMP_NUM_THREADS; on the GPU box the cgroup quota is
    16 CPUs of the 256 it shows); a short run with one thread per visible CPU is reported beside it."""
    threads = cpu_threads()
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_cpu_bench")
    sample = f"Q4_0 K=4096 N=4096 M=1 mat-vec, 32 rotated weight copies (302 MB), ~{seconds:.0f} s"
    if os.path.exists(exe):
        r = ref_cpu_run(exe, threads, seconds, 300)
        if r is not None:
            res = {"value": round(r["GBps"], 3), "unit": "GB/s", "cores": threads, "kind": "reference",
                   "sample": sample, "us_per_mul_mat": round(r["sec_per_mul_mat"] * 1e6, 2),
                   "host_cpus_visible": os.cpu_count(), "cgroup_cpu_quota": cgroup_cpu_quota()}
            nvis = os.cpu_count() or 1
            if nvis != threads:
                ra = ref_cpu_run(exe, nvis, min(seconds, 3.0), 60)
                res["all_visible_cpus"] = ({"value": round(ra["GBps"], 3), "unit": "GB/s", "threads": nvis,
                                            "us_per_mul_mat": round(ra["sec_per_mul_mat"] * 1e6, 2),
                                            "sample": "same config, ~3 s"} if ra else
                                           {"value": None, "threads": nvis, "note": "did not finish within 60 s"})
            return res
    # fallback: the C oracle restatement (scalar generic-order dots)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import qref
    K = N = 4096
    w = qref.quantize(qref.Q4_0, qref.fill_uniform(N * K, 1234), n_per_row=K)
    x = qref.fill_uniform(K, 5678).reshape(1, K)
    t0, runs = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        qref.mul_mat_simple(qref.Q4_0, w, N, K, x, 1, threads=threads)
        runs += 1
    per = (time.perf_counter() - t0) / runs
    return {"value": round(alg_bytes(M.Q4_0, K, N, 1) / per / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port", "sample": sample.replace("32 rotated weight copies (302 MB)", "1 weight copy"),
            "us_per_mul_mat": round(per * 1e6, 2)}


def gpt2_leg(torch, world: int, rank: int, n_seq: int, ticks: int, warm: int, cpu_group=None) -> dict:
    """GPT-2 117M Q4_0 decode through the pipeline ring (gpt2.Pipeline): stage `rank` of
    `world`, n_micro = world micro-batches of n_seq sequences. Returns this rank's timing.
    cpu_group: a gloo group for host-side waits (world > 1)."""
    import gpt2 as G
    import torch.distributed as dist
    hp = G.make_hparams(M.Q4_0)
    parts = G.partition_layers(hp["n_layer"], world)
    stage = G.Stage(hp, *parts[rank])
    stage.fill_synthetic(1234)
    n_micro = world
    ctxs = [G.Context(stage, n_seq) for _ in range(n_micro)]
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", torch.cuda.current_device())
    zeros = torch.zeros(n_seq, dtype=torch.int32, device=dev)
    for c in ctxs:
        c.set_pos(zeros.data_ptr(), st)
    E = hp["n_embd"]
    send = [torch.zeros(n_seq * E, dtype=torch.float32, device=dev) for _ in range(n_micro)]
    prompt = [torch.full((n_seq * E,), 0, dtype=torch.int32, device=dev) for _ in range(n_micro)]
    for mb in range(n_micro):
        prompt[mb][:n_seq] = torch.arange(n_seq, dtype=torch.int32, device=dev) + 40 + mb

    def stage_fn(mb, inbuf, valid):
        c = ctxs[mb]
        if valid:
            if stage.first:
                c.set_tokens(inbuf.data_ptr(), st)
            else:
                c._copy(c.hidden_ptr, inbuf.data_ptr(), c.hidden_bytes, st)
            c.decode(st, graph=True)
        src = c.tokens_ptr if stage.last else c.hidden_ptr
        c._copy(send[mb].data_ptr(), src, 4 * n_seq if stage.last else c.hidden_bytes, st)
        return send[mb]

    pipe = G.Pipeline(rank, world, n_micro, n_seq * E, dev, comm_device="cpu" if REHEARSAL else None)
    first = lambda mb: prompt[mb].view(torch.float32)  # noqa: E731

    def sync():
        if world > 1:
            # wait on the host: an RCCL barrier would leave a spinning kernel on the other GPUs
            # while rank 0's scheduler run uses them
            dist.barrier(group=cpu_group)
        torch.cuda.synchronize()

    # warm-up fills the ring (world - 1 ticks) and captures every context's hipGraph; the
    # timed ticks then each complete one micro-batch step at the last stage
    pipe.run(warm + world - 1, stage_fn, first)
    sync()
    t0 = time.perf_counter()
    pipe.run(ticks, stage_fn, first)
    sync()
    el = time.perf_counter() - t0
    out = {"elapsed": el, "ticks": ticks, "stages": parts, "stage_weight_bytes": stage.nbytes()}
    # single-stream latency at N=1: back-to-back graph replays with the device-side argmax loop
    if world == 1:
        c = G.Context(stage, 1)
        c.set_pos(zeros.data_ptr(), st)
        c.set_tokens(prompt[0].data_ptr(), st)
        for _ in range(4):
            c.decode(st, graph=True)
        sync()
        n = 256
        t1 = time.perf_counter()
        for _ in range(n):
            c.decode(st, graph=True)
        sync()
        out["latency_ms_per_token"] = (time.perf_counter() - t1) / n * 1e3
        c.free()
    for c in ctxs:
        c.free()
    stage.free()
    return out


def sched_plugin_gpt2(threads: int, tokens: int = 64, devices: int = 1, n_seq: int = 1) -> dict | None:
    """the drop-in path: the reference's own ggml_backend_sched GPT-2 graph (oracle/_ref/gpt2_ref,
    restating examples/gpt-2/main-sched.cpp) with our plugin loaded as its GPU backend, on the same
    synthetic 117M Q4_0 checkpoint; decode ms/token over `tokens` positions. devices > 1: the
    scheduler splits the layers over that many plugin devices (its pipeline form, hand-offs by
    our cross-device cpy_tensor_async); run by rank 0 while the other ranks wait.
    n_seq > 1: the scheduler's pipeline form (parallel = true: GGML_SCHED_MAX_COPIES copies of the
    split inputs, event-ordered hand-offs, reference ggml-backend.cpp:1460) with n_seq sequences
    decoded round-robin by ggml_backend_sched_graph_compute_async, so stages overlap"""
    exe = os.path.join(ROOT, "oracle", "_ref", "gpt2_ref")
    if not os.path.exists(exe):
        return None
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import tempfile

    import gpt2_synth
    import qref
    path = os.path.join(tempfile.gettempdir(), f"bench_gpt2_sched_{os.getpid()}.bin")
    gpt2_synth.write_model(path, gpt2_synth.GPT2_117M, qref.Q4_0, 1234)
    try:
        env = dict(os.environ)
        if REHEARSAL and devices > 1:
            env["GGML_MI355X_VIRTUAL_DEVICES"] = str(devices)   # plugin devices over GPU 0
        extra = ["--parallel", "--n-seq", str(n_seq)] if n_seq > 1 else []
        r = subprocess.run([exe, path, "--tokens", "40", "--threads", str(threads), "--plugin", M.LIB_PATH, "--devices",
                            str(devices), "--time-tokens", str(tokens)] + extra, capture_output=True, text=True,
                           timeout=300 if devices == 1 else 150, env=env)   # (the N > 1 ranks wait on it)
        if r.returncode != 0:
            return None
        j = json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.TimeoutExpired, ValueError, IndexError):
        return None
    finally:
        os.remove(path)
    row = {"value": round(j["tokens_per_s"], 2), "unit": "tokens/s", "ms_per_token": round(j["ms_per_token"], 3),
           "devices": devices, "splits": j.get("splits"),
           "path": f"reference ggml_backend_sched + libggml-hip-mi355x.so on {devices} device(s) (weights, KV and "
                   f"supported ops on MI355X, the rest on ggml-cpu with {threads} threads)",
           "sample": f"GPT-2 117M Q4_0 (synthetic), {n_seq} sequence(s), {tokens} decode positions each after a "
                     f"40-token prompt"}
    if n_seq > 1:
        row.update(n_seq=n_seq, parallel=True, async_vs_serial_nmse=j.get("async_vs_serial_nmse"))
    return row


def cpu_gpt2_baseline(threads: int, tokens: int = 128) -> dict | None:
    """the reference's ggml-cpu GPT-2 graph (oracle/_ref/gpt2_ref) on a synthetic 117M Q4_0
    checkpoint written by tests/gpt2_synth.py: decode ms/token over `tokens` positions"""
    exe = os.path.join(ROOT, "oracle", "_ref", "gpt2_ref")
    if not os.path.exists(exe):
        return None
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import tempfile

    import gpt2_synth
    import qref
    path = os.path.join(tempfile.gettempdir(), f"bench_gpt2_117m_{os.getpid()}.bin")
    gpt2_synth.write_model(path, gpt2_synth.GPT2_117M, qref.Q4_0, 1234)
    try:
        r = subprocess.run([exe, path, "--tokens", "40", "--threads", str(threads), "--time-tokens", str(tokens)],
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            return None
        j = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.remove(path)
    return {"value": round(j["tokens_per_s"], 2), "unit": "tokens/s", "cores": threads, "kind": "reference",
            "sample": f"GPT-2 117M Q4_0 (synthetic), 1 sequence, {tokens} decode positions after a 1-token prompt",
            "ms_per_token": round(j["ms_per_token"], 4)}


def cpu_gpt2_example_baseline(threads: int, n_predict: int = 128) -> dict | None:
    """the reference example itself (oracle/_ref/gpt-2-sched = examples/gpt-2/main-sched.cpp,
    unmodified, CPU backend) greedy-decoding the synthetic 117M Q4_0 checkpoint: its own
    'predict time ... ms per token' line"""
    exe = os.path.join(ROOT, "oracle", "_ref", "gpt-2-sched")
    if not os.path.exists(exe):
        return None
    sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import re
    import tempfile

    import gpt2_synth
    import qref
    path = os.path.join(tempfile.gettempdir(), f"bench_gpt2_example_{os.getpid()}.bin")
    gpt2_synth.write_model(path, gpt2_synth.GPT2_117M, qref.Q4_0, 1234)
    try:
        r = subprocess.run([exe, "-m", path, "-p", "This is an example", "-n", str(n_predict), "--top_k", "1", "-s", "1",
                            "-t", str(threads)], capture_output=True, text=True, timeout=600)
        m = re.search(r"predict time =\s*([\d.]+) ms / ([\d.]+) ms per token", r.stdout)
        if r.returncode != 0 or not m:
            return None
    finally:
        os.remove(path)
    ms = float(m.group(2))
    return {"value": round(1e3 / ms, 2), "unit": "tokens/s", "cores": threads, "kind": "reference",
            "sample": f"examples/gpt-2/main-sched.cpp itself, GPT-2 117M Q4_0 (synthetic), prompt 'This is an example' "
                      f"(18 tokens) + {n_predict} greedy tokens, its predict-time average", "ms_per_token": ms}


def launch_env():
    """(world, rank, local_rank) as torch.distributed.run exports them; 1 process by default"""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def spawn_ranks(n: int) -> int:
    """run this script under torch.distributed.run with n local ranks (127.0.0.1 rendezvous)"""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dry_run(args, world: int, rank: int) -> None:
    """--dry-run: the multi-rank plumbing on CPU (gloo) — launcher, barrier, slowest-rank
    timing and the JSON line's n_gpus — without any GPU work"""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t = 0.01 * (rank + 1)
    t_max = max_over_ranks(t, torch.device("cpu")) if world > 1 else t
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(t_max * 1e3, 4), "ranks_seen": world,
                          "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def max_over_ranks(seconds: float, device) -> float:
    """slowest rank's elapsed time (all ranks get it); `device` is cuda for RCCL, cpu for gloo"""
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_gbps(bytes_per_step_per_rank: int, steps: int, world: int, t_max: float) -> float:
    """whole-job throughput: every rank streams its own weight stacks (weak scaling, no data-path
    collective), so the job moves world x bytes per step in the slowest rank's time"""
    return bytes_per_step_per_rank * steps * world / t_max / 1e9


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # ~10 ms of timed launches: the start / stop synchronization is <0.5 % of it
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extra", action="store_true", help="skip the secondary configs")
    ap.add_argument("--no-gpt2", action="store_true", help="skip the GPT-2 decode leg")
    ap.add_argument("--gpt2-ticks", type=int, default=256, help="timed pipeline ticks of the GPT-2 leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo: only the launcher, rank plumbing and timing reduction (no GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks as a child torch.distributed.run (this process has
        # not touched the GPU) and return its exit status
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world, rank, local = launch_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_run:
        dry_run(args, world, rank)
        return
    builder = local == 0
    if REHEARSAL:
        local = 0                      # every rank on GPU 0; exchanges over gloo through host memory
    torch.cuda.set_device(local)
    cpu_group = None
    reduce_dev = torch.device("cpu") if REHEARSAL else torch.device("cuda", local)
    if world > 1 and REHEARSAL:
        dist.init_process_group("gloo")
        cpu_group = dist.group.WORLD
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        cpu_group = dist.new_group(backend="gloo")
    if builder:
        M.build()                      # one rank per node compiles (if stale); the others wait
    if world > 1:
        dist.barrier()
    if M.device_count() < 1:
        raise SystemExit("no gfx950 device visible: the MI355X backend cannot run")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ---------------- headline: one MUL_MAT over 64 stacked Q4_0 4096x4096 matrices ------------
    BATCH = args.batch
    g = MatVecSet(torch, M.Q4_0, 4096, 4096, 1, BATCH, 2)
    for i in range(2):
        g.launch(i)
    torch.cuda.synchronize()

    for i in range(args.warmup):
        g.launch(i)
    # one timed region for both numbers: `value` from its host wall time (slowest rank, barriers
    # and synchronize included), the roofline from HIP events recorded on the launch stream at
    # its two ends (device time of the same K launches)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    barrier()
    t0 = time.perf_counter()
    ev0.record(st)
    for i in range(args.steps):
        g.launch(i)
    ev1.record(st)
    barrier()
    elapsed = time.perf_counter() - t0
    t_max = max_over_ranks(elapsed, reduce_dev) if world > 1 else elapsed

    kernel_us = ev0.elapsed_time(ev1) * 1e3 / args.steps
    value = job_gbps(g.bytes, args.steps, world, t_max)
    achieved = g.bytes / (kernel_us * 1e-6) / 1e9

    extra = {}
    if not args.no_extra and rank == 0:
        # single-matrix launches (launch-bound regime), 64 copies rotated for HBM-cold reads
        single = MatVecSet(torch, M.Q4_0, 4096, 4096, 1, 1, 64)
        # single launches are host-submission-bound in eager mode: rate them by the period of
        # back-to-back launches inside one hipGraph, and show the eager event time beside it
        extra["q4_0_4096x4096_m1_single"] = dict(config_row(single, single.graph_period_us(64)),
                                                 eager_events_us=round(single.launch_us(64), 3))
        del single
        for name, t, K, N, Mc, batch in (
            ("q4_K_4096x4096_m1_b64", M.Q4_K, 4096, 4096, 1, 64),
            ("q4_K_4096x11008_m1_b24", M.Q4_K, 4096, 11008, 1, 24),
            ("q5_K_4096x11008_m1_b24", M.Q5_K, 4096, 11008, 1, 24),
            ("q6_K_4096x11008_m1_b24", M.Q6_K, 4096, 11008, 1, 24),
            ("q8_0_4096x4096_m512", M.Q8_0, 4096, 4096, 512, 1),
            ("q4_K_4096x4096_m512", M.Q4_K, 4096, 4096, 512, 1),
            # the same with the weights in the repacked layout (ggml_mi355x_repack, made once as a
            # repacked weight buffer does at upload)
            ("q8_0_4096x4096_m512_repacked", M.Q8_0, 4096, 4096, 512, 1),
            ("q4_K_4096x4096_m512_repacked", M.Q4_K, 4096, 4096, 512, 1),
        ):
            s2 = MatVecSet(torch, t, K, N, Mc, batch, 2 if batch > 1 else 24, repacked=name.endswith("_repacked"))
            s2.launch(0)
            torch.cuda.synchronize()
            extra[name] = config_row(s2, s2.launch_us(16))
            if batch > 1:
                one = MatVecSet(torch, t, K, N, Mc, 1, 64)
                one.launch(0)
                extra[name.rsplit("_b", 1)[0] + "_single"] = dict(config_row(one, one.graph_period_us(64)),
                                                                  eager_events_us=round(one.launch_us(64), 3))
                del one
            del s2
            torch.cuda.empty_cache()

    if not args.no_extra:
        extra.update(rowsplit_configs(torch, world, rank))

    cpu = cpu_baseline(args.cpu_seconds) if (rank == 0 and world == 1) else None

    # ---------------- GPT-2 117M Q4_0 decode, layers pipeline-split over the ranks ------------
    gpt2 = None
    if not args.no_gpt2:
        torch.cuda.empty_cache()
        runs = {}
        for n_seq in (1, 8):
            r = gpt2_leg(torch, world, rank, n_seq, args.gpt2_ticks, 8, cpu_group)
            t_g = max_over_ranks(r["elapsed"], reduce_dev) if world > 1 else r["elapsed"]
            runs[n_seq] = (r, t_g)
        r1, t1 = runs[1]
        gpt2 = {"metric": "GPT-2 117M Q4_0 greedy decode tokens/s", "unit": "tokens/s",
                "value": round(args.gpt2_ticks * 1 / t1, 1),
                "ms_per_tick": round(t1 / args.gpt2_ticks * 1e3, 4),
                "batched_n_seq8_tokens_per_s": round(args.gpt2_ticks * 8 / runs[8][1], 1),
                "parallelism": f"pp{world} (layer ranges {r1['stages']}), {world} micro-batch(es) in flight",
                "stage0_weight_bytes": r1["stage_weight_bytes"],
                "data": "synthetic random-init GPT-2 117M weights, quantized to Q4_0 on the device"}
        if "latency_ms_per_token" in r1:
            gpt2["single_stream_ms_per_token"] = round(r1["latency_ms_per_token"], 4)
            gpt2["single_stream_tokens_per_s"] = round(1e3 / r1["latency_ms_per_token"], 1)
        if cpu is not None:
            cpu["gpt2"] = cpu_gpt2_example_baseline(cpu["cores"]) or cpu_gpt2_baseline(cpu["cores"])
        if rank == 0:
            # configs[4]'s scheduler form: the reference's scheduler over all `world` devices
            thr = cpu["cores"] if cpu else cpu_threads()
            gpt2["reference_scheduler_with_plugin"] = sched_plugin_gpt2(thr, devices=world)
            # its pipeline form: 8 sequences in flight, stages overlapping across devices
            gpt2["reference_scheduler_with_plugin_pipelined"] = sched_plugin_gpt2(thr, devices=world, n_seq=8)
        if world > 1:
            dist.barrier(group=cpu_group)   # host wait: rank 0's scheduler run uses the other GPUs

    if rank == 0:
        line = {
            "metric": "quantized GEMM GB/s (Q4_0 mul_mat_vec 4096x4096, M=1, HBM-cold)",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "q4_0 weights x int8 activations (int32 block dots, fp32 scale accumulate)",
            "data": "synthetic (random quant bits, fp16 scales 0.01; x ~ U[-1,1])",
            "config": {"workload": f"configs[1]: Q4_0 mul_mat_vec K=4096 N=4096 M=1, {BATCH} independent "
                                   f"matrices per MUL_MAT (ne02=ne12={BATCH})",
                       "matrices_per_step": BATCH, "weight_bytes_per_step": g.bytes,
                       "parallelism": f"independent weight stacks per GPU x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": measured_traffic("q4_0_4096x4096_m1_b64") if BATCH == 64 else None,
                         "traffic_source": "profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE, x2 gfx950 correction)",
                         "launch_us": round(kernel_us, 3), "launch_us_basis": "HIP events around the timed region",
                         "rocprof": measured_rocprof("q4_0_4096x4096_m1_b64") if BATCH == 64 else None,
                         "alg_bytes_per_launch": g.bytes,
                         "frac_of_measured_copy_bw": round(achieved / HBM_MEASURED_GBS, 4)},
            "cpu_baseline": cpu,
            "configs": extra,
            "gpt2": gpt2,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
