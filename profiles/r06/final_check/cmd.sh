#!/bin/bash
source tools/gpu_run.sh
step gputests_final 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_final 120 python -c "import __graft_entry__ as g; g.smoke()"
