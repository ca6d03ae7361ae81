#!/bin/bash
# Round-6 PMC evidence: instruction / activity counters per workload
# (tools/pmc.sh passes), summarised on the box by tools/pmc_summary.py into
# gpurun_out/r6pmc/<name>.txt; raw outputs dropped.
#   WORKLOADS="name|bench args;..."  EXTRA="third pass counters" (optional)
set -u
R=$GRAFT_REPO_ROOT
cd "$R"
mkdir -p gpurun_out/r6pmc
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA"
[[ -n "${EXTRA:-}" ]] && P="$P
$EXTRA"
IFS=';' read -ra WL <<< "${WORKLOADS:-trimmedmean|;trimmedmean_n512|--agg trimmedmean --clients 512 --d 1.25e7;median|--agg median}"
for w in "${WL[@]}"; do
  name=${w%%|*}; args=${w#*|}
  TAG=r6pmc/$name BENCH_ARGS="$args" PASSES="$P" bash tools/pmc.sh || exit 1
  python3 tools/pmc_summary.py gpurun_out/r6pmc/$name > gpurun_out/r6pmc/$name.txt
  find gpurun_out/r6pmc/$name -type f -delete
  echo "pmc $name ok"
done
