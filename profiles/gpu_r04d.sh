#!/bin/bash
# Round 4: k_count gate skip A/B (interleaved, no CPU leg) + the walk kernels' parity subset.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-d}
mkdir -p $O
V=noetic-slam_amd/lib/var/libtsdf_hip_noskip.so
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu > $O/skip_$r.json 2> $O/skip_$r.err || { tail -5 $O/skip_$r.err; exit 1; }
  TSDF_HIP_LIB=$V timeout -k 10 200 python3 bench.py --no-cpu > $O/noskip_$r.json 2> $O/noskip_$r.err || { tail -5 $O/noskip_$r.err; exit 1; }
  for f in skip noskip; do
    python3 -c "import json;d=json.loads(open('$O/${f}_$r.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'])"
  done
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_bench_workload.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
