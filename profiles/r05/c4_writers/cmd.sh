source tools/gpu_run.sh
step obs_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "obs or c4" -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  step c4_stream_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time
  step c4_inline_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --variant 4
  step c4_lut4w6_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_lut4w6.so
  step c4_obsw6_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_obsw6.so
  step c4_obsw8_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_obsw8.so
  step c4_head_$r 300 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_head_HEAD.so
  step c4c_$r 300 python tools/prof_rollout.py --config c4c --envs 262144 --chunk 50 --launches 10 --time
done
step bench_c4 300 python bench.py --config c4 --steps 10 --warmup 2
step diag_c3 300 python tools/diag_split.py --config c3
step diag_c2 300 python tools/diag_split.py --config c2 --envs 4096
for P in 1024 4096 16384; do
  step c3_p$P 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles $P
done
step counters 60 rocprofv3 -L
