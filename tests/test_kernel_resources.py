"""Every kernel of libfootsies.so keeps its state in registers: no private (scratch) memory.

Compiles each HIP source for gfx950 with the library's own flags (footsies_gym_amd/build.py) and
-Rpass-analysis=kernel-resource-usage, and requires `ScratchSize [bytes/lane]: 0` for every
kernel the compiler reports (the per-arena-actor variants of k_step_n, k_step,
k_step_n_policy and k_reset spilled 48-64 B per lane, through a select between two uint4 RNG
states; fs_kernels.hip sel4).  Build-container test: hipcc cross-compiles, no GPU needed."""
import os
import re
import subprocess

import pytest

from footsies_gym_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_resources(src, extra=()):
    """{kernel symbol: {"VGPRs": .., "ScratchSize": .., "Occupancy": ..}} from the compiler's remarks."""
    cmd = [B._hipcc(), "--offload-arch=" + B.ARCH, *B.flags_for(src), *extra, "-I", os.path.join(ROOT, "include"),
           "--cuda-device-only", "-S", "-o", os.devnull, os.path.join(B.CSRC, src),
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    res, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = res.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark: +(VGPRs|ScratchSize|Occupancy)[^:]*: (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return res


@pytest.mark.parametrize("src", [s for s in B.SOURCES if s.endswith(".hip")])
def test_no_kernel_uses_scratch(src):
    res = kernel_resources(src)
    assert res, "no kernel resource remarks for %s" % src
    spills = {k: v for k, v in res.items() if v.get("ScratchSize", -1) != 0}
    assert not spills, spills
    if src == "fs_kernels.hip":
        # every template instance of the step kernels is present, the per-arena-actor ones included
        names = " ".join(res)
        for k in ("k_step_n", "k_step", "k_step_n_policy", "k_step_n_hashed", "k_step_n1", "k_step_n1_packed",
                  "k_step_n_packed", "k_reset"):
            assert re.search(r"\b_ZN3fsk\d+%sI" % k, names), k
        assert sum("ILi0ELi3EE" in n or "ILi1ELi3EE" in n for n in res) >= 8  # kActors = 3
