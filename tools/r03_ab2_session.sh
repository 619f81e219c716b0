#!/bin/bash
# r03 A/B on one box against cfd_amd/lib_ab/libcfd_hip_base.so (HEAD before):
#  - sweep A stores p before the next plane's loads + prologue wait (CG
#    sweeps: bench.py 512^3 kernel timers);
#  - k_corr3 prefetch bundle (CFD_HIP_PC3 = 8) vs plain (1);
#  - k_rk_stage3 (CFD_HIP_RK3 = 8 / 16) vs k_rk_stage2 (0).
# Parity first (CG, step, slab, RK4 suites on the new build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03_ab2
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_cg_small.py \
    tests/test_gpu_slabs.py tests/test_gpu_rk4.py tests/test_gpu_device_api.py tests/test_gpu_context_state.py \
    -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
CFD_HIP_PC3=8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config_parity.py -x -q \
    --timeout 200 --timeout-method thread > $O/pytest_pc8.log 2>&1
rc=$?; echo "pytest pc3=8 exit $rc"; tail -2 $O/pytest_pc8.log; [ $rc -ne 0 ] && exit $rc
CFD_HIP_RK3=16 timeout -k 10 200 python3 -u -m pytest tests/test_gpu_rk4.py -x -q --timeout 100 --timeout-method thread > $O/pytest_rk16.log 2>&1
rc=$?; echo "pytest rk3=16 exit $rc"; tail -2 $O/pytest_rk16.log; [ $rc -ne 0 ] && exit $rc
BASE=$PWD/cfd_amd/lib_ab/libcfd_hip_base.so
for round in 1 2; do
  for build in base new; do
    if [ $build = base ]; then export CFD_AMD_HIP_LIB=$BASE; else unset CFD_AMD_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-compare-cg-variant > $O/bench_${build}_$round.json 2> $O/bench_${build}_$round.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/bench_${build}_$round.json')); print(json.dumps({'build':'$build','round':$round,'value':d['value'],'cg_iter_ms':d['cg_iter_ms'],'sweeps':{k:v['avg_ms'] for k,v in d['kernels'].items()}}))" >> $O/ab.jsonl
  done
  unset CFD_AMD_HIP_LIB
  for v in 1 8; do
    CFD_HIP_PC3=$v timeout -k 10 240 python3 tools/step_kernels_bench.py | sed "s/^{/{\"pc3\": $v, \"round\": $round, /" >> $O/ab.jsonl || exit 1
  done
  for v in 0 8 16; do
    CFD_HIP_RK3=$v timeout -k 10 200 python3 tools/rk4_bench.py | sed "s/^{/{\"rk3\": $v, \"round\": $round, /" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
for v in 0 8; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    CFD_HIP_RK3=$v STEPS=1 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/pmc_rk${v}_${ctr} -o p --output-format csv -- python3 tools/rk4_bench.py > /dev/null 2>&1 || exit $?
  done
done
echo done
