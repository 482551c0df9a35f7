#!/bin/bash
# Estimator change check: estimator / processor / transform-precoding / pipeline GPU tests, then the phase probe
# (tools/chest_probe.py over the probe build) and the headline bench line.  Each GPU step has its own time limit.
set -uo pipefail
out=gpurun_out/${1:-r06c}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pusch_chest_gpu.py \
  tests/test_pusch_tp_gpu.py tests/test_pusch_processor_gpu.py tests/test_pipeline_gpu.py > $out/pytest.log 2>&1 \
  || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_chestprobe.so PYTHONPATH=. timeout -k 10 300 python3 tools/chest_probe.py \
  > $out/chest_probe.json 2> $out/chest_probe.err || { echo "probe failed"; tail -5 $out/chest_probe.err; exit 3; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err \
  || { echo "bench failed"; tail -5 $out/bench.err; exit 3; }
grep -o '"ms_per_step": [0-9.]*' $out/bench.json
