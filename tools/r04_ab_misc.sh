# r04 A/B (one box): parity with the opt-in corrector / sweep-store variants
# on, then the corrector variants timed (CFD_HIP_PC3 1 = k_corr3, 5 / 6 =
# k_corr4 plain / nt stores), interleaved.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-r04_ab_misc}
CFD_HIP_PC3=5 CFD_HIP_SWEEP_BUFST=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_energy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for v in 1 5 6; do
    CFD_HIP_PC3=$v STEPS=3 timeout -k 10 200 python tools/step_kernels_bench.py | sed "s/^{/{\"pc3\": $v, /" >> gpurun_out/${TAG}_corr.jsonl 2>>gpurun_out/${TAG}.err || exit 1
  done
done
cat gpurun_out/${TAG}_corr.jsonl
