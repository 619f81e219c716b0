#!/bin/bash
# r03 A/B of the RK4 stage (divz with host reciprocals, 128-VGPR bound) against
# cfd_amd/lib_ab/libcfd_hip_base.so: RK4 bitwise tests, then per-stage time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03_rk
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rk4.py tests/test_gpu_device_api.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BASE=$PWD/cfd_amd/lib_ab/libcfd_hip_base.so
for round in 1 2; do
  for build in base new; do
    if [ $build = base ]; then export CFD_AMD_HIP_LIB=$BASE; else unset CFD_AMD_HIP_LIB; fi
    timeout -k 10 200 python3 tools/rk4_bench.py | sed "s/^{/{\"build\": \"$build\", /" >> $O/rk.jsonl || exit 1
  done
done
unset CFD_AMD_HIP_LIB
cat $O/rk.jsonl
