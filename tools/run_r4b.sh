source tools/gpu_run.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  for sh in 0 1 3 4 5 6; do
    step shape_c3r_s${sh}_$r 120 env SPARC_R1R_SHAPE=$sh python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time
  done
  for v in head notab noreload noflood noaudit; do
    step ab_c3r_s0_${v}_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time --lib ab/lib_$v.so
  done
  for v in head trienx; do
    step ab_c3_${v}_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 20 --time --lib ab/lib_$v.so
  done
done
step bench_c3r_2000 300 python bench.py --config c3r --env-steps 2000 --no-cpu-baseline
step prof_c2 420 bash tools/collect_profiles.sh gpurun_out/prof_c2 c2 4096 2000 5
step load_rules 600 python tools/prof_load_rules.py --puzzles 100000 --distinct 1000
