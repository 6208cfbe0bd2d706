#!/bin/bash
# Round 4, first check of ABI v8 (merged integrator, sector input modes, border reset order, bench
# serial leg): the affected GPU tests, the bench line, the live sector-input rehearsal.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_voxblox_merged.py tests/test_multigpu.py tests/test_abi.py tests/test_bench_workload.py \
  tests/test_voxblox.py tests/test_growth.py tests/test_mesh.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py > $O/bench.out 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep '^{' $O/bench.out > $O/bench.json && cat $O/bench.json
for a in "--sectors 1" "--sectors 2" "--sectors 4" "--sectors 8" "--sectors 4 --sector-input h2d" "--sectors 4 --sector-input split" "--sectors 8 --sector-input split"; do
  timeout -k 10 200 python3 profiles/host_path.py $a --scans 320 >> $O/host_path.json 2>> $O/host_path.err || { tail -5 $O/host_path.err; exit 1; }
  tail -1 $O/host_path.json
done
