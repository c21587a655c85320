#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, within gfx950's per-block
# slot limits) for the dominant kernel of a config.
# Usage: tools/pmc_session.sh TAG CONFIG KERNEL_REGEX [DOCS]
set -u
TAG=$1; CFG=$2; KRE=$3; DOCS=${4:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
EXTRA=""
[ -n "$DOCS" ] && EXTRA="--docs $DOCS"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
  "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $p" | tee -a "$O/session.log"
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex "$KRE" -d "$O/pmc$i" -o $CFG --output-format csv -- \
      python3 "$R/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host $EXTRA > "$O/pmc$i.log" 2>&1
  rc=$?
  echo "[$(date +%T)] rc=$rc" | tee -a "$O/session.log"
  if [ $rc -ne 0 ]; then tail -30 "$O/pmc$i.log"; exit $rc; fi
done
echo "pmc done" | tee -a "$O/session.log"
