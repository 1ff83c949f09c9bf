#!/usr/bin/env python3
"""Build libfootsies.so from the csrc sources of a git revision (measurement only, never shipped):
the baseline side of an A/B against the working tree.

  python tools/build_head_lib.py REV OUT_DIR      (e.g. HEAD ab_libs/head)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from footsies_gym_amd import build as B  # noqa: E402


def main(rev, out):
    # the repository's layout (csrc includes ../../include/footsies.h), the revision's own header
    src = os.path.join(out, "footsies_gym_amd", "csrc")
    inc = os.path.join(out, "include")
    os.makedirs(src, exist_ok=True)
    os.makedirs(inc, exist_ok=True)
    with open(os.path.join(inc, "footsies.h"), "wb") as fh:
        fh.write(subprocess.run(["git", "-C", ROOT, "show", "%s:include/footsies.h" % rev], check=True,
                                capture_output=True).stdout)
    present = set()
    for f in os.listdir(B.CSRC):
        if f.endswith((".hip", ".cpp", ".h")):
            rel = os.path.relpath(os.path.join(B.CSRC, f), ROOT)
            r = subprocess.run(["git", "-C", ROOT, "show", "%s:%s" % (rev, rel)], capture_output=True)
            if r.returncode:  # (a file the revision does not have yet)
                continue
            present.add(f)
            with open(os.path.join(src, f), "wb") as fh:
                fh.write(r.stdout)
    objs = []
    for s in (s for s in B.SOURCES if s in present):
        o = os.path.join(out, s + ".o")
        subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, *B.flags_for(s), "-I", inc,
                        "-c", os.path.join(src, s), "-o", o], check=True)
        objs.append(o)
    subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o",
                    os.path.join(out, "libfootsies.so"), *objs], check=True)
    for o in objs:
        os.remove(o)
    print("built", os.path.join(out, "libfootsies.so"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
