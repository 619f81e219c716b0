# k_ccf tile order vs L2 misses at 512^3: per XCD map (0 = block order,
# 1 = XCD-contiguous tile ranges), the cg_variant 1 iteration time and one
# FETCH_SIZE + one WRITE_SIZE pass. Does fewer fetched bytes make it faster?
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
TAG=${TAG:-r04_ccf_xmap_pmc}
for X in ${XMAPS:-0 1}; do
  export CFD_HIP_CCF_XMAP=$X
  SHAPES=512 VARIANTS=1 ITERS=100 timeout -k 10 200 python tools/cg_variant_bench.py \
      | sed "s/^{/{\"xmap\": $X, /" >> gpurun_out/${TAG}.jsonl || exit 1
  TAG=${TAG}_x$X PASSES="fetch write" PASS_TIMEOUT=150 \
      CMD="python3 tools/cg_variant_bench.py" SHAPES=512 VARIANTS=1 ITERS=40 \
      bash tools/pmc_passes.sh || exit 1
  cat gpurun_out/${TAG}_x$X/summary.jsonl | grep -i "ccf\|note" | sed "s/^{/{\"xmap\": $X, /" >> gpurun_out/${TAG}.jsonl
done
cat gpurun_out/${TAG}.jsonl
