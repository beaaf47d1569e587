source tools/gpu_run.sh
P="python tools/prof_rollout.py --launches 5 --time"
step ab1 300 $P
step ab2 300 env SPARC_DIAG_LIB=sparc-gym_amd/build/libdiag_notrie.so $P
step ab3 300 $P --config c2
step ab4 300 env SPARC_DIAG_LIB=sparc-gym_amd/build/libdiag_notrie.so $P --config c2
