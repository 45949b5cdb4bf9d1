#!/bin/bash
# GPU parity run: the named test files (default: every -m gpu test), verbose, each
# test under its own time limit; the log lands in gpurun_out/${TAG}_tests.log.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-run}
FILES=${FILES:-tests}
timeout -k 10 ${LIMIT:-1000} python -u -m pytest $FILES -m gpu -x -v --timeout ${PER_TEST:-300} \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -60
[ $rc -ne 0 ] && grep -E "Error|assert" gpurun_out/${TAG}_tests.log | head -30
exit $rc
