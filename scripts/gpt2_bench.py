"""GPT-2 117M Q4_0 single-GPU decode timing (for rocprofv3 --kernel-trace --stats runs).
usage: python scripts/gpt2_bench.py [n_seq] [tokens] [graph 0/1]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-gfx906_amd"))
import torch  # noqa: E402

import gpt2 as G  # noqa: E402
import mi355x_qmm as M  # noqa: E402

n_seq = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n_tok = int(sys.argv[2]) if len(sys.argv) > 2 else 256
graph = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
torch.cuda.set_device(0)
hp = G.make_hparams(M.Q4_0)
st = G.Stage(hp)
st.fill_synthetic(1234)
c = G.Context(st, n_seq)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    sp = s.cuda_stream
    z = torch.zeros(n_seq, dtype=torch.int32, device="cuda")
    c.set_pos(z.data_ptr(), sp)
    c.set_tokens((z + 40).data_ptr(), sp)
    for _ in range(4):
        c.decode(sp, graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_tok):
        c.decode(sp, graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
print(f"n_seq={n_seq} graph={graph}: {dt / n_tok * 1e3:.4f} ms/step, {n_seq * n_tok / dt:.1f} tokens/s")
