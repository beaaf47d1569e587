source tools/gpu_run.sh
P="python tools/prof_rollout.py --launches 5 --time"
step ab1 300 $P
step ab2 300 $P --rand
step ab3 300 $P --no-out
step ab4 300 $P --rand --no-out
step ab5 300 $P --config c2
step ab6 300 $P --config c2 --rand --no-out
