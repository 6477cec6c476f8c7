#!/bin/bash
# Development round trip: the named GPU tests (pytest -k expression $2) first,
# then the whole GPU suite + smoke, then an engine-option A/B of the bench step
# (remaining args: VQX_ENGINE JSON strings, as tools/gpu_ab_engine.sh).
# usage: [PRE="cmd"] bash tools/gpu_dev.sh TAG "k expr" ['{"opt":true}' ...]
# (PRE: a command run after the targeted tests, before the suite, e.g. a probe)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-dev}; K=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests -k "$K" > $O/targeted.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" $O/targeted.log | tail -25; [ $rc -ne 0 ] && exit $rc
fi
[ -n "$PRE" ] && { timeout -k 10 300 bash -c "$PRE" > $O/pre.log 2>&1; echo "pre rc=$?"; tail -12 $O/pre.log; }
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/suite.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
[ $# -gt 0 ] && bash tools/gpu_ab_engine.sh $TAG/ab "$@"
exit 0
