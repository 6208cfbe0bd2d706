#!/bin/bash
# Round 4, first check of ABI v8 (merged integrator, sector input modes, border reset order, bench
# serial leg): the affected GPU tests, the bench line, the live sector-input rehearsal.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-a}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_multigpu.py tests/test_abi.py \
  tests/test_mesh.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for a in "--sectors 1" "--sectors 2" "--sectors 4" "--sectors 8" "--sectors 4 --sector-input h2d" "--sectors 4 --sector-input split" "--sectors 8 --sector-input split"; do
  TSDF_HOST_TIMING=1 timeout -k 10 200 python3 profiles/host_path.py $a --scans 320 >> $O/host_path.json 2>> $O/host_path.err || { tail -5 $O/host_path.err; exit 1; }
  tail -1 $O/host_path.json
done
