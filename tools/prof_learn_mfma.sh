#!/bin/bash
# SQ counters of the C5 learner's kernels (tools/learn_time.py --only hip): MFMA and VALU busy
# cycles beside the wave cycles, one rocprofv3 pass per group (no trace domains with --pmc).
# On the GPU box from the repo root: tools/prof_learn_mfma.sh OUTDIR
set -e
OUT=${1:-gpurun_out/lmfma}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
run() { name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" --output-format csv -d "$ROOT/$OUT/$name" -o run -- python3 "$ROOT/tools/learn_time.py" --only hip --reps 3 > "$ROOT/$OUT/$name.log" 2>&1
}
run trace --kernel-trace --stats
run mfma --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE
echo done
