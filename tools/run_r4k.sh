source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2; do
  step ab_c3_base_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c3_triepin_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c2_base_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c2_triepin_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time
  step ab_c3g7_base_$r 120 python tools/prof_rollout.py --config c3g7 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c3g7_triepin_$r 120 python tools/prof_rollout.py --config c3g7 --envs 65536 --chunk 2000 --launches 10 --time
done
step tests 600 python -u -m pytest tests/test_gpu_iocodes.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
