#!/bin/bash
# Round 4 evidence, tests half: the whole GPU suite, smoke(), and the 2-rank shared-GPU rehearsal of
# `bench.py --gpus 2` (gloo on one device; the driver's N-GPU runs use RCCL).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-tests}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
TSDF_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu > $O/bench_gpus2_shared.json 2> $O/bench_gpus2_shared.err || { tail -20 $O/bench_gpus2_shared.err; exit 1; }
cut -c1-400 $O/bench_gpus2_shared.json
