import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "multi_gpu: needs two or more GPUs (RCCL between devices)")


def pytest_collection_modifyitems(config, items):
    # Two-GPU tests (the RCCL transport, not yet run on hardware: every box
    # this build ran on had one GPU) go last, so that under -x a failure
    # there cannot stop the one-GPU parity suite before it has run.
    multi = [it for it in items if it.get_closest_marker("multi_gpu")]
    if multi:
        items[:] = [it for it in items if not it.get_closest_marker("multi_gpu")] + multi


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


# Parity numbers the GPU tests measure (worst rel-L2, ulp distances, ...),
# written as JSON to $BMFR_PARITY_LOG at the end of the session when set --
# the source of the figures quoted in BASELINE.md / DESIGN.md.
_PARITY = {}


@pytest.fixture(scope="session")
def parity_log():
    def record(name: str, values: dict) -> None:
        _PARITY[name] = values
    return record


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("BMFR_PARITY_LOG")
    if path and _PARITY:
        import json
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        old.update(_PARITY)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)
