#!/bin/bash
# A/B of the C5 learner's minibatch gradient (tools/learn_time.py) between library builds, rounds
# interleaved: tools/ab_learn.sh OUT LIB_A LIB_B ...   (measurement only)
set -e
out=$1; shift
for r in 1 2 3; do
  for lib in "$@"; do
    printf "round %d %-40s " $r "$lib" >> "$out"
    FOOTSIES_LIB=$(realpath "$lib") timeout -k 10 120 python tools/learn_time.py --only hip --reps 20 >> "$out"
  done
done
