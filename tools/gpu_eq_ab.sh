#!/bin/bash
# Packed-FP32 complex arithmetic of the equalizer (EQ_PK_GRAM: Gram / matched filter / L-layer solve, and the exact
# packed CFO rotation of the estimate rebuild): estimator / equalizer / PUSCH / pipeline / integration GPU tests with the
# in-tree library, then headline bench + kernel trace of pkall (all) / pkg (Gram only) / nopkg (none), alternating.
set -uo pipefail
out=gpurun_out/${1:-r06e}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_equalizer_gpu.py \
  tests/test_equalizer_mimo_gpu.py tests/test_pusch_demod_gpu.py tests/test_pusch_processor_gpu.py \
  tests/test_pusch_chest_gpu.py tests/test_pusch_tp_gpu.py tests/test_pipeline_gpu.py tests/test_integration_gpu.py \
  > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
bash tools/gpu_ab.sh $out pkall=$PWD/tools/_build/libsrsran_amd_pkall.so nopkg=$PWD/tools/_build/libsrsran_amd_nopkg.so \
  pkg=$PWD/tools/_build/libsrsran_amd_pkg.so pkall2=$PWD/tools/_build/libsrsran_amd_pkall.so \
  nopkg2=$PWD/tools/_build/libsrsran_amd_nopkg.so
