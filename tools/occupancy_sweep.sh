#!/bin/bash
# Throughput of the fused kernels against waves per SIMD (measurement only): the two-lane kernel at
# 65 536 / 131 072 / 262 144 arenas (2 / 4 / 8 waves per SIMD) and the one-lane kernel at 131 072 /
# 262 144 (2 / 4), 1000-tick launches.  Usage (GPU box, repo root): tools/occupancy_sweep.sh OUT.log
set -e
OUT=${1:-gpurun_out/occupancy.log}
L=footsies_gym_amd/libfootsies.so
: > $OUT
for n in 65536 131072 262144; do
  timeout -k 10 300 python3 tools/ab_time.py $L@FOOTSIES_FUSED_LANES=2 $L@FOOTSIES_FUSED_LANES=1 --envs $n --rounds 2 --launches 3 >> $OUT 2>&1
done
echo done >> $OUT
