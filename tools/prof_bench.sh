#!/bin/bash
# rocprofv3 passes over bench.py itself (the command whose numbers are reported):
# one kernel-trace/stats pass, then one pass per PMC group (no trace domains with --pmc).
# Usage, on the GPU box from the repo root: tools/prof_bench.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/prof_bench}; shift || true
ARGS=${@:-"--steps 400 --warmup 100 --no-cpu-baseline"}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
run() { name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/$name" -o run "$@" \
    -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/$name.log" 2>&1
}
run trace
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo done
