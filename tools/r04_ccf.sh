# fused single-reduction CG (k_ccf) check (one box): the cg_variant 1 tests,
# then the per-iteration cost of both variants (and k_cc1 + k_cc2 with
# CFD_HIP_CCF=0) at 512^3 and 512^2 x 66.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-r04_ccf}
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_cg_single_reduction.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
ITERS=${ITERS:-100} timeout -k 10 300 python tools/cg_variant_bench.py > gpurun_out/${TAG}.jsonl 2>gpurun_out/${TAG}.err || exit 1
CFD_HIP_CCF=0 ITERS=${ITERS:-100} timeout -k 10 300 python tools/cg_variant_bench.py > gpurun_out/${TAG}_old.jsonl 2>>gpurun_out/${TAG}.err || exit 1
cat gpurun_out/${TAG}.jsonl gpurun_out/${TAG}_old.jsonl
