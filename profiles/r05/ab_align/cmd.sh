source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in noalign new prio21 prio11; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
  done
  for v in noalign new prio21; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c2_${v}_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time $L
  done
done
for r in 1 2; do
  for P in 4096 16384; do
    for v in noalign new; do
      if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
      step c3p${P}_${v}_$r 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles $P $L
    done
  done
done
R=XCD0_RDREQ,XCD1_RDREQ,XCD2_RDREQ,XCD3_RDREQ,XCD4_RDREQ,XCD5_RDREQ,XCD6_RDREQ,XCD7_RDREQ
step xcd_c2_500 120 rocprofv3 -E tools/xcd_counters.yaml --pmc $R -f csv -d gpurun_out/pmc/xcd_c2_500 -o run -- python3 tools/prof_rollout.py --config c2 --envs 4096 --chunk 500 --launches 4
step xcd_c2_8000 180 rocprofv3 -E tools/xcd_counters.yaml --pmc $R -f csv -d gpurun_out/pmc/xcd_c2_8000 -o run -- python3 tools/prof_rollout.py --config c2 --envs 4096 --chunk 8000 --launches 4
step l2_c3_p16384 180 rocprofv3 --pmc TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum -f csv -d gpurun_out/pmc/l2_c3_p16384_align -o run -- python3 tools/prof_rollout.py --config c3 --chunk 2000 --launches 4 --puzzles 16384
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
