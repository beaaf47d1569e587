SKIP_TESTS=1 bash tools/final_prof.sh
