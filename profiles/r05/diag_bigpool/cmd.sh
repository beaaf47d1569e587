source tools/gpu_run.sh
export SPARC_POOL_CACHE=/tmp/sparc_pools
for P in 4096 16384; do
  SPARC_POOL_WORKERS=8 timeout -k 10 300 python3 -c "import sys; sys.path[:0] = ['.', 'sparc-gym_amd']; import bench; bench.make_pool($P, *bench.CONFIGS['c3'][:2])" || exit 3
done
export SPARC_POOL_WORKERS=1
step diag_p1024 300 python tools/diag_split.py --config c3
step diag_p4096 300 python tools/diag_split.py --config c3 --puzzles 4096
step diag_p16384 300 python tools/diag_split.py --config c3 --puzzles 16384
