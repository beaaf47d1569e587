source tools/gpu_run.sh
export TMPDIR=/tmp
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
step bench 400 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_c2 400 python bench.py --steps 1000 --warmup 100 --config c2 --no-cpu-baseline
step pmc_sq1 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc1 -o p -- python tools/prof_rollout.py --launches 3
step pmc_sq2 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2 -o p -- python tools/prof_rollout.py --launches 3
