source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2; do
  step ab_c3_head_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c3_la_$r 120 env SPARC_TRIE_LA=1 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c2_head_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time
  step ab_c2_nola_$r 120 env SPARC_TRIE_LA=0 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time
done
