#!/bin/bash
# SQ issue counters of the one-lane and two-lane fused kernels at 131 072 arenas (1000-tick
# launches), per P2 kind, one rocprofv3 pass each (no trace domains with --pmc).
# Usage (GPU box, repo root): tools/prof_sq_lanes.sh OUTDIR
set -e
OUT=${1:-gpurun_out/sq_lanes}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
for lanes in 1 2; do
  for p2 in external bot; do
    FOOTSIES_FUSED_LANES=$lanes timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/$OUT/l${lanes}_$p2" -o run --pmc $SQ -- python3 "$ROOT/tools/profile_driver.py" --mode fused \
      --chunk 1000 --launches 3 --envs 131072 --p2 $p2 > "$ROOT/$OUT/l${lanes}_$p2.log" 2>&1
  done
done
echo done
