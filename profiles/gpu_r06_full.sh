#!/bin/bash
# Round 6: the whole GPU suite, then the live-path timing (TSDF_HOST_TIMING).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/full
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash profiles/gpu_r06_live_timing.sh
