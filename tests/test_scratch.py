"""Mat-mat scratch (csrc/dispatch.cpp Scratch / scratch_for): one grow-only buffer per
(device, stream), never grown inside a hipGraph capture. ADVICE r01: the old thread-local
buffer was shared by every stream of a thread, and its growth (sync + free) was illegal inside
a capture."""
import threading

import numpy as np
import pytest

import mi355x_qmm as M
import qref

pytestmark = pytest.mark.gpu


def _operands(torch, t=qref.Q8_0, K=1024, N=256, Mc=512, seed=1):
    w = qref.quantize(t, qref.fill_uniform(N * K, seed), n_per_row=K)
    x = qref.fill_uniform(Mc * K, seed + 1).reshape(Mc, K)
    dw = torch.from_numpy(w).cuda()
    dx = torch.from_numpy(x.copy()).cuda()
    dy = torch.zeros((Mc, N), dtype=torch.float32, device="cuda")
    A = M.tensor(t, dw.data_ptr(), [K, N, 1, 1], M.contiguous_nb(t, [K, N]))
    B = M.tensor(M.F32, dx.data_ptr(), [K, Mc, 1, 1], M.contiguous_nb(M.F32, [K, Mc]))
    D = M.tensor(M.F32, dy.data_ptr(), [N, Mc, 1, 1], M.contiguous_nb(M.F32, [N, Mc]))
    want = qref.mul_mat_simple(t, w, N, K, x, Mc)
    return (A, B, D), (dw, dx, dy), want


def test_capture_on_fresh_stream_fails_cleanly_then_works_after_eager_run():
    import torch
    (A, B, D), keep, want = _operands(torch)
    result = {}

    def body():
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, stream=s):
                M.mul_mat(A, B, D, s)
            result["first"] = "captured"
        except M.Mi355xError as e:
            result["first"] = str(e)
        torch.cuda.synchronize()
        M.mul_mat(A, B, D, s)          # eager: sizes this stream's scratch
        torch.cuda.synchronize()
        keep[2].zero_()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s):
            M.mul_mat(A, B, D, s)
        g2.replay()
        torch.cuda.synchronize()
        result["replay"] = keep[2].cpu().numpy()

    th = threading.Thread(target=body)    # a fresh host thread as well
    th.start()
    th.join(timeout=120)
    assert "first" in result and result["first"] != "captured" and "rc=-2" in result["first"], result.get("first")
    assert qref.nmse(result["replay"], want) <= 5e-4


def test_two_streams_one_thread_do_not_share_scratch():
    """two streams of one thread run mat-mats concurrently without racing on a shared buffer"""
    import torch
    (A1, B1, D1), k1, want1 = _operands(torch, seed=3)
    (A2, B2, D2), k2, want2 = _operands(torch, qref.Q4_K, 2048, 512, 300, seed=5)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(8):
        M.mul_mat(A1, B1, D1, s1)
        M.mul_mat(A2, B2, D2, s2)
    torch.cuda.synchronize()
    assert qref.nmse(k1[2].cpu().numpy(), want1) <= 5e-4
    assert qref.nmse(k2[2].cpu().numpy(), want2) <= 5e-4


def test_two_threads_default_stream_growth():
    """two host threads on the default stream (handle 0), the second needing a larger
    scratch. The per-scratch mutex in mul_mat keeps the first call's buffer alive until its
    kernels are queued; the grower synchronizes the stream behind them before freeing it."""
    import torch
    small = _operands(torch, qref.Q8_0, 1024, 256, 64, seed=11)
    big = _operands(torch, qref.Q4_K, 4096, 512, 1024, seed=13)
    errors = []

    def worker(ops, reps):
        (A, B, D), keep, want = ops
        try:
            for _ in range(reps):
                M.mul_mat(A, B, D, None)
            torch.cuda.synchronize()
            err = qref.nmse(keep[2].cpu().numpy(), want)
            if not err <= 5e-4:
                errors.append(err)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(small, 40)), threading.Thread(target=worker, args=(big, 6))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
