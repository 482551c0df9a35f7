#!/bin/bash
# round-4 end: smoke(), the whole -m gpu suite, then the bench set (tools/gpu_r04_final.sh).
set -o pipefail
mkdir -p gpurun_out/r04suite
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04suite/smoke.log 2>&1 || { tail -5 gpurun_out/r04suite/smoke.log; exit 1; }
tail -1 gpurun_out/r04suite/smoke.log
bash tools/gpu_r04_suite.sh || exit $?
bash tools/gpu_r04_final.sh
