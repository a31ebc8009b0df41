"""Row-sharded MUL_MAT (ggml-gfx906_amd/rowsplit.py): the partition rule, the all-gather
bookkeeping over a real 2-rank process group (gloo, CPU, oracle compute per shard), and on the
GPU the HIP shards of one matrix reassembled against the unsharded launch."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import qref  # noqa: E402
import rowsplit as R  # noqa: E402


def _ref_get_row_split(nrows, fr, n, i, rnd):
    """direct transcription of the reference's get_row_split arithmetic (ggml-cuda.cu:778-791)
    with tensor_split as ggml_backend_cuda_split_buffer_type normalizes it (:1066-1074)"""
    lo = 0 if i == 0 else int(nrows * fr[i])
    lo -= lo % rnd
    if i == n - 1:
        hi = nrows
    else:
        hi = int(nrows * fr[i + 1])
        hi -= hi % rnd
    return lo, hi


@pytest.mark.parametrize("nrows", [16, 100, 4096, 11008, 50257])
@pytest.mark.parametrize("n,fractions", [(1, None), (2, None), (3, None), (8, None), (2, [1, 3]), (4, [1, 0, 2, 1])])
def test_row_split_rule(nrows, n, fractions):
    sh = R.row_split(nrows, n, fractions)
    assert len(sh) == n and sh[0][0] == 0 and sh[-1][1] == nrows
    for (a0, a1), (b0, b1) in zip(sh, sh[1:]):
        assert a1 == b0 and a0 <= a1
    fr = fractions or [1] * n
    tot = sum(fr)
    cum = [sum(fr[:i]) / tot for i in range(n)]
    for i in range(n):
        assert sh[i] == _ref_get_row_split(nrows, cum, n, i, R.SPLIT_ROW_ROUND)
        if i < n - 1:
            assert sh[i][1] % R.SPLIT_ROW_ROUND == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t, K, N, M, fr = case
    w = qref.quantize(t, qref.fill_uniform(N * K, 1234), n_per_row=K)
    x = qref.fill_uniform(M * K, 5678).reshape(M, K)
    lo, hi = R.row_split(N, world, fr)[rank]
    rb = qref.row_size(t, K)
    w_local = torch.from_numpy(w.reshape(N, rb)[lo:hi].copy())

    def compute(xt, y):   # this rank's rows with the CPU oracle (stands in for the HIP kernel)
        if hi > lo:
            y[:, :hi - lo] = torch.from_numpy(qref.mul_mat_simple(t, w_local.numpy().reshape(-1), hi - lo, K, xt.numpy(), M))

    mm = R.ShardedMatMul(torch, t, K, N, rank, world, w_local, fractions=fr, compute=compute)
    out = torch.full((M, N), np.nan, dtype=torch.float32)
    mm.forward(torch.from_numpy(x.copy()), out)
    full = qref.mul_mat_simple(t, w, N, K, x, M)
    ok = bool(np.array_equal(out.numpy(), full))
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("case", [(qref.Q4_0, 256, 96, 1, None), (qref.Q4_K, 512, 100, 3, None),
                                  (qref.Q6_K, 256, 77, 2, [1, 3])])
def test_all_gather_bookkeeping_two_ranks(case):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, True), (1, True)]


@pytest.mark.gpu
@pytest.mark.parametrize("t,K,N,M,shards,fr", [(qref.Q4_K, 4096, 11008, 1, 2, None), (qref.Q4_0, 4096, 4096, 1, 3, None),
                                               (qref.Q8_0, 4096, 4096, 64, 2, [1, 3]), (qref.Q6_K, 1024, 1000, 5, 4, None)])
def test_hip_shards_reassemble_to_unsharded(t, K, N, M, shards, fr):
    """the HIP kernels run shard by shard on one GPU (virtual ranks) and reassembled equal the
    unsharded launch to fp32 rounding (the reduction order can differ with the launch shape: the
    few-token mat-mat picks its split-K count from the shard's workgroup count)"""
    import mi355x_qmm as Q
    rng = np.random.default_rng(7)
    rb = Q.row_size(t, K)
    w = qref.quantize(t, qref.fill_uniform(N * K, 99), n_per_row=K).reshape(N, rb)
    x = torch.from_numpy(rng.uniform(-1, 1, (M, K)).astype(np.float32)).cuda()
    full = torch.zeros((M, N), dtype=torch.float32, device="cuda")
    dw = torch.from_numpy(w.reshape(-1).copy()).cuda()
    Q.mul_mat(Q.tensor(t, dw.data_ptr(), [K, N, 1, 1], Q.contiguous_nb(t, [K, N])),
              Q.tensor(Q.F32, x.data_ptr(), [K, M, 1, 1], Q.contiguous_nb(Q.F32, [K, M])),
              Q.tensor(Q.F32, full.data_ptr(), [N, M, 1, 1], Q.contiguous_nb(Q.F32, [N, M])))
    parts = []
    for r in range(shards):
        lo, hi = R.row_split(N, shards, fr)[r]
        wl = torch.from_numpy(w[lo:hi].reshape(-1).copy()).cuda()
        mm = R.ShardedMatMul(torch, t, K, N, r, shards, wl, fractions=fr)
        local = torch.zeros((M, mm.width), dtype=torch.float32, device="cuda")
        mm.compute(x, local)
        parts.append(local)
    out = torch.full((M, N), float("nan"), dtype=torch.float32, device="cuda")
    R.assemble(parts, R.row_split(N, shards, fr), out)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert torch.allclose(out, full, rtol=1e-5, atol=1e-5 * float(full.abs().max()))
