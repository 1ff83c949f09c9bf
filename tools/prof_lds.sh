set -e
timeout -k 10 120 ./tools/valu_probe/valu_probe > gpurun_out/valu_probe3.json
R=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_lds/sq4 -o run --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -- python3 $R/tools/profile_driver.py --mode fused --chunk 1000 --launches 3 > $R/gpurun_out/pmc_lds_sq4.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_lds/sq5 -o run --pmc LdsLatency -- python3 $R/tools/profile_driver.py --mode fused --chunk 1000 --launches 3 > $R/gpurun_out/pmc_lds_sq5.log 2>&1
echo ok
