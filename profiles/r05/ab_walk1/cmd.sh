source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in head_HEAD new; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
    step c2_${v}_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time $L
  done
done
step diag_c3 300 python tools/diag_split.py --config c3
R=XCD0_RDREQ,XCD1_RDREQ,XCD2_RDREQ,XCD3_RDREQ,XCD4_RDREQ,XCD5_RDREQ,XCD6_RDREQ,XCD7_RDREQ
R128=XCD0_RDREQ128,XCD1_RDREQ128,XCD2_RDREQ128,XCD3_RDREQ128,XCD4_RDREQ128,XCD5_RDREQ128,XCD6_RDREQ128,XCD7_RDREQ128
step xcd_c2 120 rocprofv3 -E tools/xcd_counters.yaml --pmc $R -f csv -d gpurun_out/pmc/xcd_c2 -o run -- python3 tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 4
step xcd128_c2 120 rocprofv3 -E tools/xcd_counters.yaml --pmc $R128 -f csv -d gpurun_out/pmc/xcd128_c2 -o run -- python3 tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 4
step xcd_c3 120 rocprofv3 -E tools/xcd_counters.yaml --pmc $R -f csv -d gpurun_out/pmc/xcd_c3 -o run -- python3 tools/prof_rollout.py --config c3 --chunk 2000 --launches 4
for P in 1024 4096 16384; do
  step l2_c3_p$P 180 rocprofv3 --pmc TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum -f csv -d gpurun_out/pmc/l2_c3_p$P -o run -- python3 tools/prof_rollout.py --config c3 --chunk 2000 --launches 4 --puzzles $P
done
du -sh gpurun_out/pmc
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
