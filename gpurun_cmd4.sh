source tools/gpu_run.sh
export TMPDIR=/tmp
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
step bench 400 python bench.py --steps 1000 --warmup 100 --cpu-seconds 3
step bench_c2 400 python bench.py --steps 1000 --warmup 100 --config c2 --no-cpu-baseline
step bench_c4 400 python bench.py --steps 1000 --warmup 100 --config c4 --envs 262144 --no-cpu-baseline
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
