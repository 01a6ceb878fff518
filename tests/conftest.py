"""pytest config: `gpu` marker + import paths (repo root for `oracle`, acoss-1_amd/ for `acoss`)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "acoss-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


GOLDEN = os.path.join(ROOT, "tests", "golden", "reference_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU; run with -m gpu")
