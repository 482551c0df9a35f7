#!/bin/bash
# A/B of the paired-edge high-rate decoder layer (HR_PAIRS): decoder parity with each variant library, then the
# headline bench and kernel trace of base / pc1 / pc2 (tools/gpu_ab.sh), alternating.
set -uo pipefail
out=gpurun_out/${1:-r06p}
mkdir -p $out
for v in pc2 pc1; do
  SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_ldpc_decoder_gpu.py tests/test_golden.py > $out/pytest_$v.log 2>&1 \
    || { echo "$v tests failed"; tail -20 $out/pytest_$v.log; exit 3; }
  echo "$v $(tail -1 $out/pytest_$v.log)"
done
bash tools/gpu_ab.sh $out base=$PWD/tools/_build/libsrsran_amd_base.so pc2=$PWD/tools/_build/libsrsran_amd_pc2.so \
  pc1=$PWD/tools/_build/libsrsran_amd_pc1.so base2=$PWD/tools/_build/libsrsran_amd_base.so
