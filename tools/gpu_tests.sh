#!/bin/bash
# The whole GPU suite as the driver runs it, then smoke().  $1 = output dir under gpurun_out/,
# $2.. = extra pytest selectors (default: tests).
set -o pipefail
O=gpurun_out/${1:-tests}
shift
mkdir -p $O
export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
