#!/bin/bash
# Per-kernel stats of one bench line under several library variants (same box):
#   LIBS="libsra_base.so libsra.so" ARGS="--agg bulyantrimmedmean --d 1e7" TAG=x
# kernel_stats.csv per library under gpurun_out/$TAG/<lib>/; prints the sra:: rows.
set -u
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r6lp}
OUT=$R/gpurun_out/$TAG
PKG=$R/secure-robust-federated-learning_amd
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in ${LIBS:-libsra_base.so libsra.so}; do
  n=${L%.so}
  SRA_LIB=$PKG/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run \
    -- python3 "$R/bench.py" --steps ${STEPS:-3} --warmup 1 --no-cpu --no-host ${ARGS:-} > "$OUT/$n.log" 2>&1 || { echo "$L failed"; tail -5 "$OUT/$n.log"; exit 1; }
  f=$(find "$OUT/$n" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/${n}_kernel_stats.csv"
  find "$OUT/$n" -name "*kernel_trace.csv" -delete
  python3 - "$f" "$n" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "sra::" in r["Name"]:
        print("%-14s %-60s calls %6s avg %10.1f us" % (sys.argv[2], r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
