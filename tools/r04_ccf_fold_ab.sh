# k_ccf fold launches: operands loaded by the storing lanes / planes only
# (default) vs by every lane (a CFD_HIP_CCF_XMAP=256 switch of the A/B build,
# since removed), interleaved on one box;
# per-kernel averages from a rocprofv3 kernel trace of each.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cg_single_reduction.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ccf_fold_pytest.log 2>&1 || { tail -30 gpurun_out/ccf_fold_pytest.log; exit 1; }
tail -1 gpurun_out/ccf_fold_pytest.log
for R in 1 2; do
for X in ${XS:-0 256}; do
  CFD_HIP_CCF_XMAP=$X SHAPES=512 VARIANTS=1 ITERS=100 timeout -k 10 200 python tools/cg_variant_bench.py | sed "s/^{/{\"xflag\": $X, /" >> gpurun_out/ccf_fold.jsonl || exit 1
done
done
cat gpurun_out/ccf_fold.jsonl
for X in ${XS:-0 256}; do
  CFD_HIP_CCF_XMAP=$X SHAPES=512 VARIANTS=1 ITERS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ccf_fold_tr$X -o run --output-format csv -- python3 tools/cg_variant_bench.py > gpurun_out/ccf_fold_tr$X.log 2>&1 || exit 1
  f=$(find gpurun_out/ccf_fold_tr$X -name 'run_kernel_stats.csv' | head -n 1); echo "fold_all=$X"; grep -i ccf "$f" | cut -c1-60,230-
done
