# round-4 measurement, part 2: bench lines of every config (roofline traffic from the committed
# profiles/pmc_traffic.json), rocprofv3 stats of the default bench command, the rule-table load time
source tools/gpu_run.sh
export TMPDIR=/tmp
bash tools/final_bench.sh
step load_rules 600 python tools/prof_load_rules.py --puzzles 100000 --distinct 1000
