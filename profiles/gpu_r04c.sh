#!/bin/bash
# Round 4: k_count's gate skip.  Parity (the walk kernels' GPU tests) on the shipped build, then
# interleaved bench A/B against the no-skip variant (lib/var/libtsdf_hip_noskip.so), then the
# 128-scan batch for reference.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-c}
mkdir -p $O
timeout -k 10 840 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
  --durations=10 > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V=noetic-slam_amd/lib/var/libtsdf_hip_noskip.so
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu > $O/skip_$r.json 2> $O/skip_$r.err || { tail -5 $O/skip_$r.err; exit 1; }
  TSDF_HIP_LIB=$V timeout -k 10 200 python3 bench.py --no-cpu > $O/noskip_$r.json 2> $O/noskip_$r.err || { tail -5 $O/noskip_$r.err; exit 1; }
  for f in skip noskip; do
    python3 -c "import json;d=json.loads(open('$O/${f}_$r.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'])"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu --batch 128 --steps 16 > $O/b128.json 2> $O/b128.err || { tail -5 $O/b128.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b128.json').read().strip().splitlines()[-1]);print('b128', d['value'], d['ms_per_step'], d['serial_kernel_ms_per_launch'])"
timeout -k 10 300 python3 bench.py --no-cpu --batch 32 --steps 32 > $O/b32.json 2> $O/b32.err || { tail -5 $O/b32.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b32.json').read().strip().splitlines()[-1]);print('b32', d['value'], d['ms_per_step'], d['serial_kernel_ms_per_launch'])"
