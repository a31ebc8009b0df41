"""oracle/gen_gpt2_golden.py — TEST INFRASTRUCTURE: golden GPT-2 logits from the reference.

For each weight type, writes a small synthetic GPT-2 checkpoint (tests/gpt2_synth.py, legacy
ggml format), runs it through the REFERENCE ggml-cpu graph (oracle/_ref/gpt2_ref, built from
/root/reference by oracle/ref.mk) token by token, and stores the logits of every position as
tests/golden/gpt2_<type>.logits.f32 plus tests/golden/gpt2_manifest.json (hparams, seed, the
checkpoint's sha256, tokens, command). The checkpoint itself is not committed: the tests
regenerate it deterministically and check the sha256 first.

    python oracle/gen_gpt2_golden.py        # in the build container (needs oracle/_ref)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import gpt2_synth  # noqa: E402
import qref  # noqa: E402

SMALL = dict(n_vocab=1000, n_ctx=128, n_embd=256, n_head=4, n_layer=3)
# token streams: printable ids, then a long tail so positions cross the attention kernel's
# 64-key passes (q4_0 case)
TOKENS = {
    "q4_0": [(7 * i + 40) % 1000 for i in range(70)],
    "q8_0": [40, 72, 73, 83, 0, 73, 83, 0, 65, 78, 999, 500],
    "q4_K": [40, 72, 73, 83, 0, 73, 83, 0, 65, 78, 999, 500],
    "q5_K": [40, 72, 73, 83, 0, 73, 83, 0, 65, 78, 999, 500],
    "q6_K": [40, 72, 73, 83, 0, 73, 83, 0, 65, 78, 999, 500],
}
SEED = 1234
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "gpt2_ref")


def main():
    manifest = {"generator": "oracle/gen_gpt2_golden.py -> oracle/_ref/gpt2_ref (reference ggml-cpu, 1 thread)",
                "hparams": SMALL, "seed": SEED, "cases": {}}
    for name, toks in TOKENS.items():
        t = qref.BY_NAME[name]
        path = f"/tmp/gpt2_golden_{name}.bin"
        sha = gpt2_synth.write_model(path, SMALL, t, SEED)
        out = os.path.join(GOLDEN, f"gpt2_{name}.logits.f32")
        cmd = [REF, path, "--tokens", ",".join(map(str, toks)), "--out", out, "--threads", "1"]
        subprocess.check_call(cmd)
        lg = np.fromfile(out, np.float32).reshape(len(toks), SMALL["n_vocab"])
        manifest["cases"][name] = {"model_sha256": sha, "tokens": toks, "logits": os.path.basename(out),
                                   "argmax": lg.argmax(1).tolist()}
        print(name, sha[:16], lg.shape)
    with open(os.path.join(GOLDEN, "gpt2_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
