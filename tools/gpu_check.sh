#!/bin/bash
# One guarded GPU session: tests -> smoke -> bench -> rocprofv3 kernel stats.
# Stops at the first crash / abort / timeout (exit codes >1 from pytest, or any
# non-zero from the others); plain test failures (pytest exit 1) still let the
# bench run so that a number is recorded.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-all}

run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/summary.txt"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/summary.txt"
  tail -5 "$OUT/$name.log" | tee -a "$OUT/summary.txt"
  return $rc
}

if [[ $STEPS == all || $STEPS == *tests* ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  rc=$?
  if [[ $rc -gt 1 ]]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  cd /tmp
  run_prof() {
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-host ${BENCH_ARGS:-} \
      > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
  }
  run_prof; rc=$?
  echo "== prof rc=$rc" | tee -a "$GRAFT_REPO_ROOT/$OUT/summary.txt"
  cd "$GRAFT_REPO_ROOT"
  [[ $rc -eq 0 ]] || exit $rc
fi
echo "== done" | tee -a "$OUT/summary.txt"
