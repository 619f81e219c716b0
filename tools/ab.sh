#!/bin/bash
# One-box A/B of an environment switch -- the form of every experiment
# recorded in profiles/ (their notes give the switch, values and command).
#   SW      the variable (e.g. CFD_HIP_CGB_REV; CFD_AMD_HIP_LIB selects another
#           build of libcfd_hip.so); a value "-" leaves it unset
#   VALUES  the values, in the order they run in each round
#   TESTS   pytest files run under every value before timing (parity first)
#   CMD     the measuring command; each JSON line it prints is tagged with
#           {"<SW>": value, "round": r}
#   ROUNDS  interleaved rounds (default 2)
#   PMC     optional counters: one rocprofv3 --pmc pass per counter and value
#           over PMC_CMD (default CMD), summarised by tools/pmc_kernels.py
# Output: gpurun_out/<TAG>/{pytest_<v>.log, ab.jsonl, pmc.jsonl}.
# usage: TAG=rev SW=CFD_HIP_CGB_REV VALUES="0 1" TESTS="tests/test_gpu_parity.py" \
#        CMD="python3 tools/relax_bench.py" tools/ab.sh
#
# Recorded experiments in this form (the measuring programs are the
# tools/*_bench.py; a build under test is selected with CFD_AMD_HIP_LIB =
# cfd_amd/lib_ab/<name>/libcfd_hip.so, built by `make -C cfd_amd/csrc
# OUT=.../lib_ab/<name> OBJ=.../build_ab/<name> HIPCC="hipcc -D..."`):
#   k_ccf memory-op order / prefetch depth / stage-c reads (r05):
#     SW=CFD_AMD_HIP_LIB VALUES="<base> <variant> -" TESTS=tests/test_gpu_cg_single_reduction.py
#     SHAPES=512 VARIANTS=1 ITERS=200 CMD="python3 tools/cg_variant_bench.py"
#   k_ccf z-run length (r04, r05): SW=CFD_HIP_CCF_KC VALUES="- 16 24" (+ CFD_HIP_CCF_KC_FIXED=1
#     for slab shapes, SHAPES=slabs), same CMD
#   k_ccf tile order vs fetched bytes (r04): SW=CFD_HIP_CCF_XMAP VALUES="0 1", then
#     PASSES="fetch write" CMD="python3 tools/cg_variant_bench.py" tools/pmc_passes.sh
#   k_rb2 range test (r05), tile map / run length (r04): SW=CFD_AMD_HIP_LIB or
#     CFD_HIP_RB2_XMAP / CFD_HIP_RB2_KC, TESTS="tests/test_gpu_rb2.py
#     tests/test_gpu_convection_tol.py", NX=1024 NY=1024 NZ=512 ITERS=40 METHODS=rbsor
#     CMD="python3 tools/relax_bench.py"; k_rb1 vs k_rb2: SW=CFD_HIP_RB2 VALUES="0 1 2"
#   corrector / sweep-store variants (r04): SW=CFD_HIP_PC3 VALUES="1 5 6"
#     CMD="python3 tools/step_kernels_bench.py"
#   slab CG forms at N ranks on one shared GPU: tools/slab_rehearsal.sh
#   configs[4] trace + FETCH/WRITE + step: tools/conv_profile.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab}
O=gpurun_out/$TAG
mkdir -p $O
: "${SW:?SW (the environment switch) is required}" "${CMD:?CMD is required}"
VALUES=${VALUES:-"0 1"}
safe() { echo "$1" | tr -c 'A-Za-z0-9_.\n-' '_'; }  # a value as a file-name part
run() {  # run <value> <command...>: the command with SW set to value (or unset)
  local v=$1; shift
  if [ "$v" = "-" ]; then env -u "$SW" "$@"; else env "$SW=$v" "$@"; fi
}
if [ -n "$TESTS" ]; then
  for v in $VALUES; do
    run "$v" timeout -k 10 ${TEST_TIMEOUT:-500} python3 -u -m pytest $TESTS -x -q --timeout 300 \
        --timeout-method thread > $O/pytest_$(safe "$v").log 2>&1
    rc=$?; echo "pytest $SW=$v exit $rc"; tail -1 $O/pytest_$(safe "$v").log; [ $rc -ne 0 ] && exit $rc
  done
fi
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VALUES; do
    run "$v" timeout -k 10 ${CMD_TIMEOUT:-300} $CMD > $O/cmd.out 2> $O/cmd.err || { tail -5 $O/cmd.err; exit 1; }
    sed "s|^{|{\"$SW\": \"$v\", \"round\": $round, |" $O/cmd.out >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
for v in $VALUES; do
  for ctr in $PMC; do
    d=$O/pmc_$(safe "$v")_$ctr
    run "$v" timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc $ctr -d $d -o p \
        --output-format csv -- ${PMC_CMD:-$CMD} > /dev/null 2>&1 || exit $?
    python3 tools/pmc_kernels.py $d --note "$SW=$v $ctr" >> $O/pmc.jsonl
  done
done
exit 0
