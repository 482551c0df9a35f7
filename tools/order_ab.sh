#!/bin/bash
# Enqueue order of the step's two chains (bench_pipeline.Pipeline.step): PDSCH first (dl) / PUSCH first (ul), alternating.
set -uo pipefail
out=gpurun_out/r06o; mkdir -p $out
B=(python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-latency --no-pinned --low-snr-db -1)
for v in dl ul dl ul dl ul; do
  if [ $v = ul ]; then export SRSRAN_AMD_UL_FIRST=1; else export SRSRAN_AMD_UL_FIRST=0; fi
  timeout -k 10 200 "${B[@]}" > $out/$v.json 2>/dev/null || { echo "$v failed"; exit 3; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $out/$v.json | head -1)"
done
