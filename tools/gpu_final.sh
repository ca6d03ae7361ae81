#!/bin/bash
# round-end rehearsal: the whole -m gpu suite, smoke(), default bench
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" "$OUT/pytest.log" | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
