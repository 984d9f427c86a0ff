#!/bin/bash
# A/B of library builds on any bench lines (lib/libnbx_<tag>.so side builds, "main" = lib/libnbx.so).
#   MODELS="ponita eqv2" TESTS_K="ponita or eqv2" bash scripts/ab_lib_lines.sh main base
# An argument env:VAR=VALUE runs the main build with that environment setting instead.
# The GPU tests selected by -k "$TESTS_K" run first with the main build; then one bench per (model, build),
# interleaved twice.  Output: gpurun_out/abl/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/abl
LIBDIR=$(ls -d extending-*/lib)
MODELS="${MODELS:-ponita eqv2}"
declare -A ARGS=([ponita]="--steps 10 --warmup 2" [eqv2]="--steps 30 --warmup 3" [segnn]="--steps 300 --warmup 20"
                 [eqv2_train]="--steps 30 --warmup 5" [ponita_train]="--steps 30 --warmup 5")
if [ -n "${TESTS_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -k "$TESTS_K" -q -x -p no:cacheprovider --timeout 120 \
      --timeout-method thread > gpurun_out/abl/tests.log 2>&1
  rc=$?; echo "tests: $(tail -1 gpurun_out/abl/tests.log)"; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for m in $MODELS; do
    for t in "$@"; do
      E=""
      case "$t" in
        main) L=$PWD/$LIBDIR/libnbx.so ;;
        env:*) L=$PWD/$LIBDIR/libnbx.so; E="${t#env:}" ;;
        *) L=$PWD/$LIBDIR/libnbx_$t.so ;;
      esac
      o=gpurun_out/abl/${m}_$(echo "$t" | tr -c 'A-Za-z0-9_\n' '_')_$r
      env NBX_LIB=$L $E timeout -k 10 240 python bench.py --model $m ${ARGS[$m]} --no-cpu-baseline > $o.json 2> $o.err
      rc=$?; [ $rc -ne 0 ] && { echo "$m $t rc=$rc"; tail -3 $o.err; exit $rc; }
      python - "$o.json" "$m" "$t" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = d.get("roofline", {}).get("per_kind") or {}
short = {(v.get("role") or k)[:24]: v.get("avg_launch_us", v.get("avg_group_us")) for k, v in pk.items()}
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], short, flush=True)
PY
    done
  done
done
