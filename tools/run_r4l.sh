source tools/gpu_run.sh
export TMPDIR=/tmp
bash tools/final_bench.sh
