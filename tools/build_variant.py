#!/usr/bin/env python3
"""Build libfootsies.so from an alternative fs_kernels.hip (measurement only, never shipped).

  python tools/build_variant.py KERNEL_SOURCE OUT_DIR [EXTRA_HIPCC_FLAGS ...]

The other sources and headers come from footsies_gym_amd/csrc; the library lands at
OUT_DIR/libfootsies.so (time it with tools/ab_time.py).
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from footsies_gym_amd import build as B  # noqa: E402


def main(src, out, extra=()):
    os.makedirs(out, exist_ok=True)
    for f in os.listdir(B.CSRC):
        if f.endswith((".hip", ".cpp", ".h")):
            shutil.copy(os.path.join(B.CSRC, f), out)
    shutil.copy(src, os.path.join(out, "fs_kernels.hip"))
    objs = []
    for s in B.SOURCES:
        o = os.path.join(out, s + ".o")
        subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, *B.flags_for(s), *extra, "-I", os.path.join(ROOT, "include"),
                        "-c", os.path.join(out, s), "-o", o], check=True)
        objs.append(o)
    subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o",
                    os.path.join(out, "libfootsies.so"), *objs], check=True)
    for o in objs:
        os.remove(o)
    print("built", os.path.join(out, "libfootsies.so"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
