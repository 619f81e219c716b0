#!/bin/bash
# A/B of the current library against cfd_amd/lib_ab/libcfd_hip_base.so on one
# box: parity tests of the kernels touched, then RB-SOR iteration and
# predictor / corrector times of both builds, interleaved (B A B A).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
TESTS=${TESTS:-tests/test_gpu_rb_variants.py tests/test_gpu_parity.py tests/test_gpu_energy.py tests/test_gpu_rk4.py}
timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
BASE=$PWD/cfd_amd/lib_ab/libcfd_hip_base.so
for round in 1 2; do
  for build in base new; do
    if [ $build = base ]; then export CFD_AMD_HIP_LIB=$BASE; else unset CFD_AMD_HIP_LIB; fi
    METHODS=rbsor ITERS=60 timeout -k 10 240 python tools/relax_bench.py | sed "s/^{/{\"build\": \"$build\", /" >> gpurun_out/${TAG}.jsonl || exit $?
    METHODS=rbsor ITERS=30 NX=1024 NY=1024 NZ=512 timeout -k 10 300 python tools/relax_bench.py | sed "s/^{/{\"build\": \"$build\", /" >> gpurun_out/${TAG}.jsonl || exit $?
    timeout -k 10 240 python tools/step_kernels_bench.py | sed "s/^{/{\"build\": \"$build\", /" >> gpurun_out/${TAG}.jsonl || exit $?
  done
done
unset CFD_AMD_HIP_LIB
cat gpurun_out/${TAG}.jsonl
