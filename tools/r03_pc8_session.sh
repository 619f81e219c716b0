#!/bin/bash
# r03 A/B: k_pred3 / k_corr3 on 128 x 8 tiles (512-thread workgroups, two or
# more per CU; CFD_HIP_PC3=16) against the 128 x 16 default (1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_pc8
mkdir -p $O
CFD_HIP_PC3=16 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py \
  tests/test_gpu_config_parity.py tests/test_gpu_slabs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for v in 1 16; do
    CFD_HIP_PC3=$v timeout -k 10 240 python3 tools/step_kernels_bench.py | sed "s/^{/{\"pc3\": $v, \"round\": $round, /" >> $O/pc.jsonl || exit 1
  done
done
cat $O/pc.jsonl
