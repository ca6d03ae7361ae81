#!/bin/bash
# PMC passes for one bench workload.  Usage: TAG=x BENCH_ARGS="..." tools/pmc.sh
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/runtime
# traces beside --pmc, as the pool requires).
set -u
TAG=${TAG:-pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUTD="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUTD"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [[ -z "$counters" ]] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d "$OUTD/p$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-} > "$OUTD/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok: $counters"
done <<PASSES
${PASSES:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA}
PASSES
