#!/bin/bash
# Run a chosen set of GPU test files under one time limit; log under gpurun_out/.
# usage: TAG=x TESTS="tests/a.py tests/b.py" tools/tests_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-tests}
LIMIT=${LIMIT:-600}
timeout -k 10 "$LIMIT" python -u -m pytest $TESTS -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 40 gpurun_out/${TAG}_pytest.log; exit $rc
