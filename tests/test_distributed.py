"""Multi-process (gloo, world_size 2, CPU) coverage of bench.py's N>1 path: rank/world from the
torch.distributed.run environment, the slowest-rank timing reduction and the weak-scaling
aggregate. The GPU run uses the same functions over RCCL ("nccl")."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    w, r, l = bench.launch_env()
    dist.init_process_group("gloo", rank=r, world_size=w)
    elapsed = 0.5 + rank            # rank 1 is the slow one
    t_max = bench.max_over_ranks(elapsed, torch.device("cpu"))
    gbps = bench.job_gbps(606076928, 20, w, t_max)
    dist.barrier()
    dist.destroy_process_group()
    q.put((r, w, l, t_max, gbps))


def test_two_rank_timing_and_aggregate():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1] and all(r[1] == 2 and r[2] == r[0] for r in res)
    for r in res:
        assert r[3] == pytest.approx(1.5)                           # max over ranks
        assert r[4] == pytest.approx(606076928 * 20 * 2 / 1.5 / 1e9)  # both ranks' bytes / slowest time


def test_single_process_defaults(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.launch_env() == (1, 0, 0)
    assert bench.job_gbps(1e9, 10, 1, 2.0) == pytest.approx(5.0)


def _bench_json(args, env=None):
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(line[-1]) if line else None), r.stderr


@pytest.mark.parametrize("n", [2, 8])
def test_bench_gpus_n_starts_n_ranks(n):
    """`bench.py --gpus N` with no launcher starts its own torch.distributed.run child with N
    ranks (gloo dry run: rank plumbing only) and reports n_gpus = N from the slowest rank;
    N = 8 is the driver's scaling run"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc, line, err = _bench_json(["--gpus", str(n), "--dry-run"], env)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == n and line["ranks_seen"] == n
    assert line["ms_per_step"] == pytest.approx(10.0 * n)    # max over ranks (rank n-1: 10 n ms)


def test_bench_rejects_rank_count_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    rc, line, err = _bench_json(["--gpus", "2", "--dry-run"], env)
    assert rc != 0 and line is None and "--gpus 2" in err


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu_rehearsal():
    """bench.py's N > 1 legs end to end on the one-GPU test box: BENCH_ONE_GPU_REHEARSAL=1 puts
    both ranks on GPU 0 with gloo exchanges through host memory, so the row-split all-gather,
    the GPT-2 pipeline ring, the host-side waits and the slowest-rank reductions all run (the
    driver's 8-GPU run takes the same code with RCCL). Numbers are not checked, only that every
    leg produced one."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_ONE_GPU_REHEARSAL"] = "1"
    rc, line, err = _bench_json(["--gpus", "2", "--steps", "3", "--warmup", "1", "--gpt2-ticks", "16",
                                 "--cpu-seconds", "1"], env)
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 2 and line["value"] > 0
    for k in ("q4_K_4096x11008_m1_rowsplit", "q8_0_4096x4096_m512_rowsplit"):
        assert line["configs"][k]["shards"] == 2 and line["configs"][k]["us"] > 0
    assert line["gpt2"]["value"] > 0 and line["gpt2"]["batched_n_seq8_tokens_per_s"] > 0
    assert line["gpt2"]["parallelism"].startswith("pp2")
    sched = line["gpt2"]["reference_scheduler_with_plugin"]   # 2 plugin devices (virtual, GPU 0)
    assert sched is not None and sched["devices"] == 2 and sched["splits"] >= 2 and sched["value"] > 0
