#!/bin/bash
# rocprofv3 passes over tools/learn_time.py --only hip (fs_ppo_grad's kernels): one kernel
# trace, then SQ counter groups, each in its own run (no trace domains combined with --pmc).
set -e
OUT=${1:-gpurun_out/lprof}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
run() { name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/$name" -o run "$@" -- python3 "$ROOT/tools/learn_time.py" --only hip --reps 3 > "$ROOT/$OUT/$name.log" 2>&1
}
run trace
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
run sq3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT || true
echo done
