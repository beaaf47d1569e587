# round-4 measurement, part 1: GPU suite, smoke, per-config kernel stats + PMC passes (folded on the box)
export SKIP_TESTS=0
bash tools/final_prof.sh
