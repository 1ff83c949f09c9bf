#!/bin/bash
# The trace and the FETCH_SIZE / WRITE_SIZE passes alone (one rocprofv3 run each) over
# tools/profile_driver.py in fused mode.  Usage (GPU box, repo root):
#   tools/prof_pmc_traffic.sh OUTDIR [profile_driver args...]
set -e
OUT=${1:?outdir}; shift; DARGS="$@"
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
run() { name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/$name" -o run "$@" -- python3 "$ROOT/tools/profile_driver.py" --mode fused $DARGS > "$ROOT/$OUT/$name.log" 2>&1
}
run trace
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo done
