set -e
for rep in 1 2 3; do
 for v in none torch_launches sim_launches; do
  timeout -k 10 60 python tools/cold_region_probe.py $v >> gpurun_out/r03n_cold_region_probe.txt
 done
done
