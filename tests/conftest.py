"""pytest configuration: `gpu` marker = needs a real MI355X (run with -m gpu on the GPU box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ggml-gfx906_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
