#!/bin/bash
# One rocprofv3 --pmc pass (counters in $1) over the C3 bench, k_long only.
set -u
TAG=${TAG:-s3pmc1}; R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $1 --kernel-include-regex k_long -d "$O/pmc" -o c3 --output-format csv -- \
  python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > "$O/pmc.log" 2>&1
