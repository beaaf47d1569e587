source tools/gpu_run.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
P="python tools/prof_rollout.py --launches 5 --time"
step ab1 300 $P
step ab5 300 $P --config c2
step ab7 300 $P --envs 131072
step ab8 300 $P --envs 262144 --config c4
step bench 400 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
