#!/bin/bash
# On the GPU box, after tools/profile_round.sh (TAG) / tools/gpu_pmcw.sh pmc steps:
# fold the PMC CSVs into profiles/traffic.json + summaries, copy what is to be
# kept to gpurun_out/keep/, and delete the per-dispatch CSVs (gpurun_out/ must
# stay under 64 MiB to come back).  usage: bash tools/gpu_pmc_pack.sh TAG [pmc_dir ...]
set -u
R=$GRAFT_REPO_ROOT
TAG=$1; shift
K=$R/gpurun_out/keep
mkdir -p "$K"
cd "$R"
[ -d "gpurun_out/$TAG" ] && python3 tools/pmc_traffic.py "gpurun_out/$TAG" "$TAG" > "$K/pmc_traffic_$TAG.txt" 2>&1
[ -d gpurun_out/pmcw ] && python3 tools/pmc_traffic.py gpurun_out/pmcw "${TAG}w" > "$K/pmc_traffic_${TAG}w.txt" 2>&1
for d in "$@"; do python3 tools/pmc_summary.py "$d" > "$K/$(basename "$d").txt" 2>&1; done
cp profiles/traffic.json "$K/traffic.json"
cp profiles/${TAG}* "$K/" 2>/dev/null
find gpurun_out -name "*counter_collection.csv" -delete
find gpurun_out -name "*kernel_trace.csv" -delete
du -sh gpurun_out
