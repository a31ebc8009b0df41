"""rowsplit.py — row-sharded ("tensor parallel") quantized MUL_MAT across ranks, one process per
GPU over torch.distributed (RCCL over xGMI on the box, gloo in the CPU tests).

The reference shards a weight matrix by rows over the GPUs of one process (split buffer type,
src/ggml-cuda/ggml-cuda.cu:763-1094; partition get_row_split :778-791) and gathers the partial
dst rows onto the main device with peer copies (:1640-1700). The plugin implements exactly
that inside one process (csrc/backend.cpp, ggml_backend_split_buffer_type). This module is the
MI355X-native multi-process form of the same partition: rank r owns rows [lo_r, hi_r) of
every matrix, computes its rows of dst with the HIP mat-vec / mat-mat kernels (C ABI), and ONE
all-gather (RCCL) hands every rank the whole dst — the only data-path exchange.

Shard sizes follow the same rule as the plugin (cumulative fractions, rows rounded down to
SPLIT_ROW_ROUND except on the last shard), so a rank's rows are identical in both forms.
"""
from __future__ import annotations

import mi355x_qmm as Q

SPLIT_ROW_ROUND = 16   # csrc/backend.cpp SPLIT_ROW_ROUND


def row_split(nrows: int, n_shards: int, fractions=None) -> list:
    """[(lo, hi)] per shard; fractions = relative shares (None / all zero: equal shares)"""
    if n_shards < 1:
        raise ValueError("n_shards must be >= 1")
    fr = list(fractions or [])[:n_shards] + [0.0] * max(0, n_shards - len(fractions or []))
    if not any(fr):
        fr = [1.0] * n_shards
    tot = float(sum(fr))
    cum, s = [], 0.0
    for f in fr:
        cum.append(s / tot)
        s += f
    out = []
    for i in range(n_shards):
        lo = 0 if i == 0 else int(nrows * cum[i])
        lo -= lo % SPLIT_ROW_ROUND
        if i == n_shards - 1:
            hi = nrows
        else:
            hi = int(nrows * cum[i + 1])
            hi -= hi % SPLIT_ROW_ROUND
        out.append((lo, max(hi, lo)))
    return out


def assemble(parts: list, shards: list, out) -> None:
    """out[..., lo:hi] = parts[r][..., :hi-lo] for every shard r; parts[r] is [cols, >= hi-lo]
    (padded to a common width for the all-gather); out is [cols, N]"""
    for (lo, hi), p in zip(shards, parts):
        if hi > lo:
            out[:, lo:hi].copy_(p[:, :hi - lo])


class ShardedMatMul:
    """dst[M, N] = W[N, K] . x[M, K] with W row-sharded over `world` ranks.

    `w_local` holds this rank's rows (quantized, contiguous, device memory): rows
    [lo, hi) = row_split(N, world, fractions)[rank]. Call forward(x, out) on every rank."""

    def __init__(self, torch, t: int, K: int, N: int, rank: int, world: int, w_local, fractions=None, group=None,
                 compute=None, comm_device=None):
        """comm_device "cpu": the all-gather runs on host copies (process groups that cannot move
        device tensors, e.g. gloo with ranks sharing one GPU)"""
        self.torch, self.t, self.K, self.N, self.rank, self.world, self.group = torch, t, K, N, rank, world, group
        self.comm_device = comm_device
        self.shards = row_split(N, world, fractions)
        self.lo, self.hi = self.shards[rank]
        self.rows = self.hi - self.lo
        self.width = max(h - l for l, h in self.shards)       # all-gather needs equal pieces
        self.equal = all(h - l == self.width for l, h in self.shards)
        self.w_local = w_local
        self.compute = compute or self._hip_compute
        self._buf = {}

    def _hip_compute(self, x, y) -> None:
        """y[M, rows] = W_local . x on the current stream through the C ABI"""
        M = x.shape[0]
        if self.rows == 0:
            return
        A = Q.tensor(self.t, self.w_local.data_ptr(), [self.K, self.rows, 1, 1], Q.contiguous_nb(self.t, [self.K, self.rows]))
        B = Q.tensor(Q.F32, x.data_ptr(), [self.K, M, 1, 1], Q.contiguous_nb(Q.F32, [self.K, M]))
        D = Q.tensor(Q.F32, y.data_ptr(), [self.rows, M, 1, 1], [4, 4 * self.width, 4 * self.width * M, 4 * self.width * M])
        Q.mul_mat(A, B, D)

    def _buffers(self, M: int, device):
        key = (M, str(device))
        if key not in self._buf:
            torch = self.torch
            local = torch.zeros((M, self.width), dtype=torch.float32, device=device)
            gathered = torch.empty((self.world, M, self.width), dtype=torch.float32, device=device)
            self._buf[key] = (local, gathered)
        return self._buf[key]

    def forward(self, x, out) -> None:
        """x: [M, K] f32, out: [M, N] f32 (both on this rank's device). Collective."""
        import torch.distributed as dist
        M = x.shape[0]
        if self.world == 1:          # one shard = all rows: no exchange
            self.compute(x, out)
            return
        local, gathered = self._buffers(M, x.device)
        self.compute(x, local)
        if self.comm_device is not None and self.comm_device != str(x.device):
            host = [t.to(self.comm_device) for t in (local, gathered)]
            dist.all_gather_into_tensor(host[1].view(-1), host[0].view(-1), group=self.group)
            gathered.copy_(host[1])
            assemble(list(gathered), self.shards, out)
            return
        if M == 1 and self.equal:
            # dst rows of all ranks are contiguous and equal: gather straight into out
            dist.all_gather_into_tensor(out.view(-1), local.view(-1), group=self.group)
            return
        dist.all_gather_into_tensor(gathered.view(-1), local.view(-1), group=self.group)
        assemble(list(gathered), self.shards, out)
