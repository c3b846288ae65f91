export TMPDIR=/tmp
K='k_subtree|k_partition2|k_scan'
python tools/gpu_steps.py \
  stamps 200 'PKD_SUBTREE_STAMPS=1 python tools/bench_build.py --n 100000000 --steps 1' \
  pmc_fetch 120 "timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex '$K' --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/bench_build.py --n 100000000 --steps 1" \
  pmc_write 120 "timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex '$K' --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/bench_build.py --n 100000000 --steps 1" \
  pmc_sq 120 "timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_SMEM --kernel-include-regex '$K' --output-format csv -d gpurun_out/pmc_sq -o run -- python3 tools/bench_build.py --n 100000000 --steps 1"
