#!/bin/bash
# round-4: rate dematching fused into the high-rate decoder's load -- parity, then the headline A/B.
set -o pipefail
O=gpurun_out/r04dm
mkdir -p $O
step() { # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 "$O/$name.log" | cut -c1-220
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -q -rf --timeout 240 --timeout-method thread"
step tests 600 $PYT tests/test_sch_gpu.py tests/test_pipeline_gpu.py tests/test_pusch_processor_gpu.py tests/test_ldpc_decoder_gpu.py
step bench 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step bench_nofuse 200 env SRSRAN_AMD_DEMATCH_FUSED=0 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step bench2 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
step sp 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline
exit 0
