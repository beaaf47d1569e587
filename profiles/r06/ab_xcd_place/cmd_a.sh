#!/bin/bash
source tools/gpu_run.sh
for r in 1 2; do
  for v in head fbitop fbitop_u2 fu2 prio_audit; do
    step c3r_${v}_$r 180 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time --lib ab/lib_$v.so
  done
done
for r in 1 2; do
  step c3_p1024_$r 180 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time
  for P in 4096 16384; do
    for pl in hash xcd; do
      step c3_p${P}_${pl}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time --puzzles $P --placement $pl
    done
    step c3_p${P}_xcd_8b_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time --puzzles $P --placement xcd --variant 5:2
  done
done
