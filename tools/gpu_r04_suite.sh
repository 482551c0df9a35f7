#!/bin/bash
# round-4 GPU parity suite (the whole -m gpu set), per-test timeout; log under gpurun_out/r04suite.
set -o pipefail
mkdir -p gpurun_out/r04suite
timeout -k 10 1000 python -u -m pytest -m gpu -q -rf --timeout 240 --timeout-method thread tests/ \
  > gpurun_out/r04suite/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r04suite/pytest.log
exit $rc
