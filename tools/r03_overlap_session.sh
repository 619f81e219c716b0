#!/bin/bash
# Round-3 GPU session: RB-SOR slab-overlap traces (split / one-launch) and the
# configs[4] convection line at full size on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_ovl
mkdir -p $O
export TMPDIR=/tmp
cd $R
for split in 1 0; do
  CFD_HIP_RB_SPLIT=$split timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace \
      --output-format csv -d $O/split$split -- python3 tools/rb_overlap_trace.py \
      > $O/split$split.log 2>&1 || { echo "trace split=$split failed"; exit 1; }
  python3 tools/overlap_summary.py $O/split$split "split=$split" >> $O/summary.jsonl || exit 1
done
cat $O/summary.jsonl
timeout -k 10 300 python3 bench.py --case convection --steps 1 --warmup 0 \
    > $O/convection_1gpu.json 2> $O/convection_1gpu.err || { echo "convection failed"; tail -5 $O/convection_1gpu.err; exit 1; }
tail -c 600 $O/convection_1gpu.json
