#!/bin/bash
# End-of-round measurement, part 2: one bench line per config (roofline traffic from
# profiles/pmc_traffic.json) and rocprofv3 --kernel-trace --stats of the default bench command
# (without its CPU-baseline leg: under rocprofv3 the forked baseline workers stalled past the
# 180-s silence limit once; the kernel launches are the same).
source tools/gpu_run.sh
for cfg in ${BENCH_CONFIGS:-c3 c2 c3r c3g7 c4c c4}; do
  step bench_$cfg 300 python bench.py --config $cfg
done
# the headline config on pools past the LDS row budget (global rows, sparc_move1.hpp row slots)
for pz in ${BENCH_POOLS:-4096 16384}; do
  step bench_c3_p$pz 300 python bench.py --config c3 --puzzles $pz
done
export TMPDIR=/tmp
step bench_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_rocprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
