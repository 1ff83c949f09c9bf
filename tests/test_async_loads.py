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
    # k_step_n (8 instances: 2 float modes x 4 P2 variants) and k_step_n_packed (8) read rows, and
    # k_step_n1 and k_step_n1_packed (6 each: no kActors variant), k_step_n_pf and k_step_n_packed_pf
    # (6 each: the request prefetch never runs per-arena actors)
    assert " 0 findings" in r.stdout and "40 kernels" in r.stdout, r.stdout


def test_wait_counts_are_proven_and_a_too_deep_wait_is_caught(tmp_path):
    """The same analysis proves every `s_waitcnt vmcnt(11)` row wait (vmcnt(3) in the packed-trajectory
    kernels): on every path at least that many vector memory instructions follow the row's load
    (advisor r02).  A copy of the kernel whose waits claim more than the stores of one tick plus a
    load (30, packed 4) must be reported."""
    src = os.path.join(ROOT, "footsies_gym_amd", "csrc", "fs_kernels.hip")
    text = open(src).read()
    assert text.count("constexpr int kRowWait = PK ? 3 : 11;") == 1
    bad = tmp_path / "fs_kernels.hip"
    # (per-field waits claim 30, packed ones 4: one more than the 2 stores and a load)
    bad.write_text(text.replace("constexpr int kRowWait = PK ? 3 : 11;", "constexpr int kRowWait = PK ? 4 : 30;"))
    # the one-lane kernels (fs_arena1.h, included from the same directory) wait with
    # vmcnt(12 (D - 1)), packed vmcnt(5 (D - 1)), D = 3 slots: 24 / 10 are exact, so 25 / 11 must
    # be reported
    one = open(os.path.join(ROOT, "footsies_gym_amd", "csrc", "fs_arena1.h")).read()
    assert "constexpr int W = (PK ? 5 : 12) * (D - 1);" in one and "#define FS_ROW_DEPTH 3" in one
    (tmp_path / "fs_arena1.h").write_text(one.replace("constexpr int W = (PK ? 5 : 12) * (D - 1);",
                                                      "constexpr int W = (PK ? 5 : 12) * (D - 1) + 1;"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_async_loads.py"), str(bad)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 1, r.stdout[-2000:] + r.stderr[-2000:]
    assert "vmcnt(30) copies" in r.stdout and "vmcnt(4) copies" in r.stdout, r.stdout[-2000:]
    assert "vmcnt(25) copies" in r.stdout and "vmcnt(11) copies" in r.stdout, r.stdout[-2000:]
