#!/bin/bash
# A/B of the k-select variants on the default bench workload (one process each, same box)
set -u
mkdir -p gpurun_out
AGGS=${AGGS:-trimmedmean median}
VARIANTS=${VARIANTS:-"1:256 1:768 2:256 2:1024"}
for agg in $AGGS; do
  for v in $VARIANTS; do
    sel=${v%%:*}; bs=${v##*:}
    f=gpurun_out/ab_${agg}_s${sel}_b${bs}
    SRA_SELECT=$sel SRA_BS=$bs timeout -k 10 300 python bench.py --agg $agg --steps 10 --warmup 2 --no-cpu --no-host ${BENCH_ARGS:-} \
      > $f.json 2> $f.err || exit $?
    python -c "import json;l=json.load(open('$f.json'));print('$agg sel=$sel bs=$bs', l['value'], l['roofline']['kernel_ms'], l['roofline']['frac'])"
  done
done
