#!/bin/bash
# r03 A/B of the RK4 stage: k_rk_stage3 (z-march, LDS y rows; CFD_HIP_RK3 = 8 /
# 16 row tiles) against k_rk_stage2 (CFD_HIP_RK3 = 0). RK4 bitwise tests under
# each, per-stage time interleaved over two rounds, one FETCH / WRITE pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_rk3
mkdir -p $O
for v in 8 16 0; do
  CFD_HIP_RK3=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rk4.py tests/test_gpu_device_api.py \
      tests/test_gpu_context_state.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest rk3=$v exit $rc"; tail -2 $O/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
done
for round in 1 2; do
  for v in 0 8 16; do
    CFD_HIP_RK3=$v timeout -k 10 200 python3 tools/rk4_bench.py | sed "s/^{/{\"rk3\": $v, \"round\": $round, /" >> $O/rk.jsonl || exit 1
  done
done
cat $O/rk.jsonl
for v in 0 8 16; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    CFD_HIP_RK3=$v STEPS=1 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/pmc_${v}_${ctr} -o p --output-format csv -- python3 tools/rk4_bench.py > /dev/null 2>&1 || exit $?
  done
done
echo done
