import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-drl-rmc_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_sessionfinish(session, exitstatus):
    """Put the parity exemption counts (tests/parity.py) on record."""
    try:
        import json
        from parity import EXEMPTIONS
    except Exception:
        return
    if not EXEMPTIONS:
        return
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_exemptions.json"), "w") as f:
        json.dump(EXEMPTIONS, f, indent=1)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """One line in the summary tail (which the driver's GPU test record keeps): how many oracle weight
    comparisons used compare_state's 2 lr exemption, and for how many entries (tests/parity.py)."""
    try:
        from parity import COMPARISONS, EXEMPTIONS
    except Exception:
        return
    if not COMPARISONS[0]:
        return
    per_test = {}
    for x in EXEMPTIONS:
        per_test[x["test"]] = per_test.get(x["test"], 0) + x["entries"]
    terminalreporter.write_line(
        f"parity exemptions (2 lr bound): {sum(per_test.values())} weight entries in {len(EXEMPTIONS)} tensors "
        f"of {len(per_test)} tests, max {max(per_test.values(), default=0)} entries per test, over "
        f"{COMPARISONS[0]} oracle weight comparisons (every other entry within 1e-5)")
