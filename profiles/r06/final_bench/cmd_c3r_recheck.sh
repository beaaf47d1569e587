#!/bin/bash
source tools/gpu_run.sh
step bigpool16k 300 python -u -m pytest tests/test_gpu_bigpool.py -k "16384" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_c3r 300 python bench.py --config c3r
step bench_c3 300 python bench.py
