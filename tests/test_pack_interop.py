"""`.pack` checkpoints written by the drop-in load in the reference's own Network.load, and the
reference's load in the drop-in, bit for bit (VERDICT r4
missing #2).  Needs /root/reference (build container only; skipped on the GPU box, which has no
reference).  tests/golden/pack_interop.py does the work, one process per side."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(HERE, "golden", "pack_interop.py")


@pytest.mark.skipif(not os.path.isdir("/root/reference/dqn"), reason="reference not present (GPU box)")
def test_pack_interop_both_directions(tmp_path):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    for role in ("ours-save", "ref", "ours-load"):
        r = subprocess.run([sys.executable, SCRIPT, role, str(tmp_path)], capture_output=True, text=True,
                           timeout=300, env=env, cwd=str(tmp_path))
        assert r.returncode == 0, (role, r.stdout[-3000:], r.stderr[-3000:])
        if role == "ref":
            assert r.stdout.count("ok ref-load") == 3 and "bit-identical" in r.stdout, r.stdout
        if role == "ours-load":
            assert r.stdout.count("ok ours-load") == 3, r.stdout
