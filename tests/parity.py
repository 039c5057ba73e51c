"""Shared parity tolerances of the GPU tests (numbers stated once, here).

Gradients are fp32 sums of B per-sample products, formed in a different order than torch's
CPU kernels (split-K slabs summed in slice order).  Where a gradient entry is a near-cancelling
sum, its absolute error is set by the size of the terms, not by the entry, so the bound is
relative to the tensor's largest entry: |got - ref| <= 2e-6 + 1e-4 |ref| + 5e-4 max|ref|.
The 1e-5 bar of BASELINE.json applies to Q values, loss and the updated weights, which the
tests check separately."""
import numpy as np


def assert_grad_close(got, ref, what=""):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = float(np.abs(ref).max()) if ref.size else 0.0
    tol = 2e-6 + 1e-4 * np.abs(ref) + 5e-4 * scale
    d = np.abs(got - ref)
    bad = d > tol
    assert not bad.any(), (what, int(bad.sum()), float(d.max()), scale)


# Weight entries that used compare_state's 2 lr exemption (tests/test_gpu_engine.py), per test
# and tensor; conftest.py writes them to gpurun_out/parity_exemptions.json at session end so the
# count is on record for every run.
EXEMPTIONS = []
COMPARISONS = [0]   # compare_state calls (weights checked against the oracle) this session


def record_exemptions(counts, numels):
    import os
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    for k, n in counts.items():
        EXEMPTIONS.append({"test": test, "tensor": k, "entries": int(n), "numel": int(numels[k])})
