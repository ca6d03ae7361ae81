#!/bin/bash
# Round-6 GPU session: the whole -m gpu suite, smoke, the default bench line
# (with its CPU baseline), then tools/profile_round.sh (kernel traces of every
# workload at the bench's defaults with steady-state summaries, PMC traffic
# passes).  Logs under gpurun_out/$TAG/ and gpurun_out/${TAG}prof/.
set -u
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r6f}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log"
TAG=${TAG}prof bash tools/profile_round.sh
