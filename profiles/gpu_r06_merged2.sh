#!/bin/bash
# Round 6: the bucketed Merged pre-pass -- merged GPU tests, the merged bench with parity, then its
# rocprofv3 kernel stats (into gpurun_out/r06/merged2/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06/merged2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_voxblox_merged.py -k "merged" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "merged and not test_voxblox_merged" > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -3 $O/pytest2.log
grep -h "blob scan" $O/pytest.log || true
timeout -k 10 300 python3 bench.py --method merged --semantics voxblox --cpu-seconds 2 --parity-steps 1 > $O/merged.json 2> $O/merged.err || { tail -5 $O/merged.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/merged.json')); print('merged', d['value'], d['ms_per_step'], (d.get('parity') or {}).get('bitwise'))"
bash profiles/gpu_r06_prof_merged.sh merged2_prof
bash profiles/gpu_r06_prof_merged.sh merged2_prof_serial --semantics voxblox --method merged --pipeline 0
