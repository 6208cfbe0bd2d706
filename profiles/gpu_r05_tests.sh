#!/bin/bash
# Round 5: the whole GPU suite on the tree as it is (one call), log under gpurun_out/r05/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/${1:-tests}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  --durations=15 -x ${2:-} > $O/pytest_gpu.log 2>&1
rc=$?
tail -25 $O/pytest_gpu.log
exit $rc
