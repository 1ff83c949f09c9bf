#!/bin/bash
# A/B of one PPO iteration's phases and per-kernel device times (tools/ppo_profile.py) between
# library builds, rounds interleaved: tools/ab_ppo.sh OUT LIB_A LIB_B ...   (measurement only)
set -e
out=$1; shift
for r in 1 2; do
  for lib in "$@"; do
    echo "== round $r $lib" >> "$out"
    FOOTSIES_LIB=$(realpath "$lib") timeout -k 10 200 python tools/ppo_profile.py 2>/dev/null | grep -E "^collect|k_ppo_grad" >> "$out"
  done
done
