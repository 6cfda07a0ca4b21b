import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")

# torch bundles its own libamdhip64.so.7; importing it before libsmore_hip.so
# makes the library bind to that same HIP runtime (same soname), so torch
# tensors/streams and the library's device pointers live in one runtime
# whatever order the tests run in (bench.py imports torch first too).
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
