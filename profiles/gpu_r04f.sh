#!/bin/bash
# Round 4: k_count with two blocks per 512-lane workgroup (TSDF_COUNT_PAIRED=1, the new default)
# against one block per 256-lane workgroup (=0): in-bench bitwise parity, interleaved benches,
# the fp32 mode, then the GPU parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-f}
mkdir -p $O
for r in 1 2; do
  for p in 1 0; do
    TSDF_COUNT_PAIRED=$p timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 > $O/p${p}_$r.json 2> $O/p${p}_$r.err || { tail -5 $O/p${p}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/p${p}_$r.json').read().strip().splitlines()[-1]);p=d['parity'];print('paired=$p', d['value'], d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
  done
done
for p in 1 0; do
  TSDF_COUNT_PAIRED=$p timeout -k 10 200 python3 bench.py --cpu-seconds 0.5 --semantics vdbfusion > $O/fp32_p${p}.json 2> $O/fp32_p${p}.err || { tail -5 $O/fp32_p${p}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/fp32_p${p}.json').read().strip().splitlines()[-1]);p=d['parity'];print('fp32 paired=$p', d['value'], d['ms_per_step'], 'serial', d['serial_kernel_ms_per_launch'], 'parity', p and p['bitwise'])"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
