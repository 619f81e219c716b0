#!/bin/bash
# r03 A/B: predictor / corrector on 128 x 16 tiles with LDS rows (k_pred3 /
# k_corr3, CFD_HIP_PC3 = 1 / 2 / 4) against k_pred2 / k_corr2 (0). Parity with
# the new kernels first, then tools/step_kernels_bench.py interleaved over two
# rounds, then one FETCH_SIZE / WRITE_SIZE pass per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03_pc3}
CFD_HIP_PC3=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py \
  tests/test_gpu_config_parity.py tests/test_gpu_slabs.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 0 1 2 4; do
    CFD_HIP_PC3=$v timeout -k 10 240 python tools/step_kernels_bench.py | sed "s/^{/{\"pc3\": $v, \"round\": $round, /" >> gpurun_out/${TAG}.jsonl || exit $?
  done
done
cat gpurun_out/${TAG}.jsonl
for v in 0 2 4; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    CFD_HIP_PC3=$v STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/${TAG}_pmc_${v}_${ctr} -o p --output-format csv -- python3 tools/step_kernels_bench.py > /dev/null 2>&1 || exit $?
  done
done
echo done
