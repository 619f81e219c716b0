#!/bin/bash
# r03: achievable rate by stream mix (tools/stream_nm.py), then the configs[4]
# natural-convection line at full size on one GPU with the current k_rb1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_conv
mkdir -p $O
timeout -k 10 300 python3 tools/stream_nm.py > $O/stream_nm.jsonl 2> $O/stream_nm.err || { echo "stream_nm failed"; tail -5 $O/stream_nm.err; exit 1; }
cat $O/stream_nm.jsonl
timeout -k 10 400 python3 bench.py --case convection --steps 1 --warmup 0 \
    > $O/convection_1gpu.json 2> $O/convection_1gpu.err || { echo "convection failed"; tail -5 $O/convection_1gpu.err; exit 1; }
tail -c 900 $O/convection_1gpu.json
