#!/bin/bash
# Round-3 session: GPU tests (optionally a subset), then the default bench and the
# vacuum headline; stops at the first crash / timeout.
cd "$(dirname "$0")/.." || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
T=${1:-${TESTS:-tests}}
BENCH=${2:-${BENCH:-1}}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
[ "$BENCH" = 0 ] && exit 0
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cut -c1-300 gpurun_out/${TAG}_bench.json
timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/${TAG}_vac.json || exit $?
cut -c1-300 gpurun_out/${TAG}_vac.json
MNL_TILE=0 timeout -k 10 200 python bench.py --vacuum --no-extra --no-cpu > gpurun_out/${TAG}_vac_old.json || exit $?
cut -c1-300 gpurun_out/${TAG}_vac_old.json
exit 0
