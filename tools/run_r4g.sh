source tools/gpu_run.sh
export TMPDIR=/tmp
step bench_rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_rocprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step load_rules 600 python tools/prof_load_rules.py --puzzles 100000 --distinct 1000
for r in 1 2; do
  step ab_c3_head_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head.so
  step ab_c3_notriecode_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_notriecode.so
done
