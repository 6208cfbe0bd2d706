# Live input paths: host-pointer rate, the N-context sector split on one GPU, and
# the node's MapCore path (tsdf_replay topic stream).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/live}
mkdir -p $OUT
for n in 1 2 4 8; do
  timeout -k 10 300 python3 profiles/host_path.py --sectors $n > $OUT/host_path_s$n.json 2> $OUT/h$n.err || { tail -5 $OUT/h$n.err; exit 1; }
  echo "sectors $n: $(cat $OUT/host_path_s$n.json)"
done
timeout -k 10 300 python3 profiles/node_path.py > $OUT/node_path.json 2> $OUT/node.err || { tail -5 $OUT/node.err; exit 1; }
cat $OUT/node_path.json
