#!/bin/bash
# Round 5: the sector block test folded into k_count (no k_sector_flags pass for the two walks) --
# sector tests, then rank-0 rehearsals A/B against HEAD at N = 4 and 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/call20; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_multigpu.py tests/test_gpu_parity.py -k "sector or Sector" -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for N in 4 8; do
    for nl in real= head=noetic-slam_amd/lib/var/libtsdf_hip_head.so; do
      n=${nl%%=*}; lib=${nl#*=}
      TSDF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu --rank-rehearsal $N > $O/${n}_n${N}_$i.json 2> $O/${n}_n${N}_$i.err || { tail -3 $O/${n}_n${N}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${n}_n${N}_$i.json')); print('$n N=$N', d['value'], d['ms_per_step'], d['kernel_ms_per_launch'], d['parity']['bitwise'] if d.get('parity') else '')"
    done
  done
done
