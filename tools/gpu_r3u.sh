#!/bin/bash
# Round 3, session u: same-box A/B of the session-start library (tools/ab) vs
# the current one on the Krum family (mom_krum's N > 128 Gram in particular).
# (tools/ab/libsra_r3start.so was built from commit 1405ea2: git worktree add /tmp/oldtree 1405ea2 &&
#  make -C /tmp/oldtree/secure-robust-federated-learning_amd/csrc OUT=$PWD/tools/ab/libsra_r3start.so BUILD=/tmp/oldbuild;
#  not kept in the tree)
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3u
mkdir -p "$OUT"
cd /tmp
for rep in 1; do
for lib in "$R/tools/ab/libsra_r3start.so" "$R/secure-robust-federated-learning_amd/libsra.so"; do
  tag=$(basename $lib .so)_$rep
  SRA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o run -- python3 "$R/bench.py" --warmup 2 --no-cpu --no-host --agg mom_krum --clients 512 --d 1.25e7 --steps 10 > "$OUT/$tag.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "$tag mom_krum $(grep '"metric"' "$OUT/$tag.log" | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms_per_step'])")"
  python3 -c "
import csv
for x in list(csv.DictReader(open('$OUT/prof_$tag/run_kernel_stats.csv')))[:2]: print('   ', x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e6)"
done
done
