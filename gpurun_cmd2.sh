source tools/gpu_run.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q --maxfail=5
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 1000 --warmup 100 --cpu-seconds 5
step bench_step 400 python bench.py --steps 300 --warmup 30 --mode step --no-cpu-baseline
