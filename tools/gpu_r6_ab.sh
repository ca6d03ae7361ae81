#!/bin/bash
# Round-6 same-box A/B of library variants on one bench line: LIBS (space-
# separated .so paths relative to the package dir; "libsra.so" = the working
# tree's) in REPS alternating rounds, bench ARGS each; then optional TESTS on
# the working tree's library.  Logs under gpurun_out/$TAG/.
set -u
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r6ab}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
PKG=$R/secure-robust-federated-learning_amd
LIBS=${LIBS:-"libsra_base.so libsra.so"}
REPS=${REPS:-3}
ARGS=${ARGS:-"--steps 20 --warmup 5 --no-cpu --no-host"}
for i in $(seq 1 $REPS); do
  for L in $LIBS; do
    SRA_LIB=$PKG/$L timeout -k 10 300 python bench.py $ARGS > "$OUT/${L%.so}_$i.json" 2> "$OUT/${L%.so}_$i.err" || { tail -5 "$OUT/${L%.so}_$i.err"; exit 1; }
    python - "$OUT/${L%.so}_$i.json" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]
print(sys.argv[1].split('/')[-1], "step", j["ms_per_step"], "kernel", r.get("kernel_ms"), "frac", r["frac"])
PY
  done
done
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
