"""Diagnostics: greedy stream of the engine on the small golden model (block layer vs the
five-launch layer) and, at the first position where the two streams differ, the top-2 logit
margin of each. Usage: python scripts/greedy_diag.py q4_K [n_new]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("ggml-gfx906_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gpt2 as G  # noqa: E402
import gpt2_synth  # noqa: E402
import qref  # noqa: E402
import json  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "q4_K"
n_new = int(sys.argv[2]) if len(sys.argv) > 2 else 24
import test_gpt2_example as TE  # noqa: E402

path, prompt, ref = TE.model_and_stream(name)
n_new = len(ref)


def run(block):
    os.environ["GGML_MI355X_GPT2_BLOCK"] = "1" if block else "0"
    hp = G.read_hparams(path)
    st = G.Stage(hp)
    st.load(path)
    ctx = G.Context(st, 1)
    gen = G.greedy_generate(ctx, [prompt], n_new)[0]
    ctx.free()
    st.free()
    return gen


torch.cuda.set_device(0)
a, b = run(True), run(False)
print("reference  ", ref)
print("block      ", a)
print("five-launch", b)
# teacher-forced logits on the reference stream: top-2 margin where block and reference differ
seq = prompt + ref
for block in (True, False):
    os.environ["GGML_MI355X_GPT2_BLOCK"] = "1" if block else "0"
    hp = G.read_hparams(path)
    st = G.Stage(hp)
    st.load(path)
    ctx = G.Context(st, 1)
    stream = torch.cuda.current_stream().cuda_stream
    z = torch.zeros(1, dtype=torch.int32, device="cuda")
    ctx.set_pos(z.data_ptr(), stream)
    out = []
    for t in seq[:-1]:
        tk = torch.full((1,), t, dtype=torch.int32, device="cuda")
        ctx.set_tokens(tk.data_ptr(), stream)
        ctx.decode(stream, True)
        lg = torch.empty((1, hp["n_vocab"]), dtype=torch.float32, device="cuda")
        ctx._copy(lg.data_ptr(), ctx.logits_ptr, 4 * hp["n_vocab"], stream)
        out.append(lg.cpu().numpy()[0])
    ctx.free()
    st.free()
    lg = np.stack(out)[len(prompt) - 1:]
    for i, r in enumerate(ref):
        top = np.argsort(lg[i])[::-1][:2]
        if top[0] != r:
            print(("block" if block else "five-launch"), "pos", i, "argmax", top[0], "ref", r,
                  "logit[argmax]-logit[ref]", float(lg[i][top[0]] - lg[i][r]))
            break
    else:
        print(("block" if block else "five-launch"), "teacher-forced argmax matches the reference at every position")
