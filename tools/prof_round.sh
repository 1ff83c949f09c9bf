#!/bin/bash
# One round's profiles of the C3 step kernel.  On the GPU box, from the repo root:
#   tools/prof_round.sh TAG
# (1) rocprofv3 kernel-trace/stats + FETCH_SIZE / WRITE_SIZE passes over the bench command whose
#     roofline block they back (tools/prof_bench.sh) -> gpurun_out/prof_TAG;
# (2) the SQ counter passes of the same kernel at 1000 ticks per launch (tools/prof_pmc.sh)
#     -> gpurun_out/pmc_TAG.
# Then, back in the build container, reduce them to the committed files:
#   python3 tools/summarize_profile.py gpurun_out/prof_TAG TAG --envs 65536 --chunk 1000 \
#       --command "python3 bench.py --no-cpu-baseline --no-extras --no-c4 --warmup 1000"
#   python3 tools/summarize_profile.py gpurun_out/pmc_TAG_c4 TAG_c4 --envs 262144 --chunk 1000 \
#       --command "python3 tools/profile_driver.py --mode fused --envs 262144 --chunk 1000 --launches 3 --layout packed"
#   python3 tools/pmc_table.py gpurun_out/pmc_TAG --ticks 1000 --waves 2048 --kernel k_step_n_packed \
#       --json profiles/TAG_sq.json --command "python3 tools/profile_driver.py --mode fused --chunk 1000 --launches 3 --layout packed"
# (the SQ passes profile the bench's own layout: packed trajectory records, k_step_n_packed)
set -e
TAG=${1:?tag}
timeout -k 10 900 bash tools/prof_bench.sh gpurun_out/prof_$TAG --no-cpu-baseline --no-extras --no-c4 --warmup 1000
timeout -k 10 900 bash tools/prof_pmc.sh gpurun_out/pmc_$TAG fused --chunk 1000 --launches 3 --layout packed
# (3) the c4_strong leg's one-GPU point: FETCH / WRITE at 262 144 arenas, 1000-tick packed launches
timeout -k 10 600 bash tools/prof_pmc_traffic.sh gpurun_out/pmc_${TAG}_c4 --envs 262144 --chunk 1000 --launches 3 --layout packed
echo prof_round done
