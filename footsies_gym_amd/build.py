"""Build libfootsies.so in-tree with hipcc for gfx950.

``python -m footsies_gym_amd.build`` (or ``__graft_entry__.build()``).  The
library is plain C-ABI (no torch types), compiled directly by hipcc; the built
``.so`` lives next to this file so it travels with the repository snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
LIB = os.path.join(HERE, "libfootsies.so")
ARCH = os.environ.get("FOOTSIES_OFFLOAD_ARCH", "gfx950")
SOURCES = ["fs_kernels.hip", "fs_delay.hip", "fs_gather.hip", "fs_learn.hip", "fs_api.cpp"]
HEADERS = ["fs_internal.h", "fs_tables.h", "fs_policy.h", "fs_arena1.h"]

# -ffp-contract=off: no a*b+c fusion -- every float op must round like the C# it restates.
# -simplifycfg-sink-common=false: SimplifyCFG otherwise sinks the per-branch field stores
#   of the action state machine into one store through a pointer phi, which blocks SROA and
#   leaves the whole per-lane arena (272 B) in scratch memory -- 400+ scratch ops per tick.
# -amdgpu-mfma-vgpr-form: the policy kernel's MFMA results land in VGPRs, where the tanh
#   epilogue reads them, instead of AGPRs plus one v_accvgpr_read per element.
# -fno-slp-vectorize: pairs of box-coordinate adds otherwise become v_pk_add_f32 plus the
#   v_mov_b32s that line their operands up in register pairs -- more VALU issues, not fewer.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off",
          "-fno-fast-math", "-Wall", "-Wno-unused-function", "-Wno-bitwise-instead-of-logical",
          "-fno-slp-vectorize",
          "-mllvm", "-simplifycfg-sink-common=false", "-mllvm", "-amdgpu-mfma-vgpr-form"]
# Per-source additions.  The simulation kernels are one wave's long dependent chain per tick
# (one or two waves per SIMD at C4 / C3): the max-ILP machine scheduler interleaves the tick's
# independent work between its LDS reads and DPP / VCC hazards (two-tick loop 1034 -> 1013
# instructions, s_nop 29 -> 6) instead of the default occupancy-first schedule:
# +9.3 % at 32 768 arenas, +3.5 % at 65 536 (profiles/r04l_sched_*.txt).
SOURCE_FLAGS = {"fs_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def flags_for(src):
    """The hipcc flags a source file of the library is compiled with (CFLAGS + SOURCE_FLAGS)."""
    return CFLAGS + SOURCE_FLAGS.get(os.path.basename(src), [])


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = ([os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "footsies.h")] +
            [os.path.abspath(__file__)])  # (the flags live here)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    hipcc = _hipcc()
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, "--offload-arch=" + ARCH, *flags_for(src), "-I", INCLUDE, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(obj)
    cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB, *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
