"""The fused kernels' untracked action-row loads (fs_kernels.hip row_load / settle_w): on the
gfx950 assembly of every kernel that has them, no instruction reads or overwrites a load's
register between the load and the wait that makes it resident (tools/check_async_loads.py).
Build-container test: hipcc cross-compiles, no GPU needed."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_register_touched_while_its_row_is_in_flight():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_async_loads.py")], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " 0 findings" in r.stdout and "8 kernels" in r.stdout, r.stdout
