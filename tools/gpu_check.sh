#!/bin/bash
# Runs GPU tests, a short bench and a rocprofv3 kernel-trace summary on the GPU box.
# Stops at the first fault / abort / timeout (exit codes other than 0 and 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    codec) step pytest_codec 600 python -m pytest tests/test_ldpc_codec_gpu.py -x -q ;;
    ofdm) step pytest_ofdm 600 python -m pytest tests/test_ofdm_gpu.py -x -q ;;
    eq) step pytest_eq 600 python -m pytest tests/test_equalizer_gpu.py -x -q ;;
    polar) step pytest_polar 600 python -m pytest tests/test_polar_gpu.py -x -q ;;
    mod) step pytest_mod 600 python -m pytest tests/test_modulation_gpu.py -x -q ;;
    crc) step pytest_crc 600 python -m pytest tests/test_crc_gpu.py -x -q ;;
    sch) step pytest_sch 900 python -m pytest tests/test_sch_gpu.py -x -q ;;
    chest) step pytest_chest 300 python -u -m pytest tests/test_pusch_chest_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    demod) step pytest_demod 300 python -u -m pytest tests/test_pusch_demod_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    pipe) step pytest_pipe 300 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread ;;
    proc) step pytest_proc 300 python -u -m pytest tests/test_pusch_processor_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    pdsch) step pytest_pdsch 300 python -u -m pytest tests/test_pdsch_modulator_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 2 ;;
    benchq) step bench 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    traffic) step pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
             step pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
             python3 tools/pmc_summary.py traffic gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic.json ;;
    pmc) step pmc1 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline && \
         step pmc2 600 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    ppmc) step ppmc1 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/ppmc1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline && \
          step ppmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/ppmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline && \
          step ppmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/ppmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    obench) step bench_ofdm 600 python bench.py --workload ofdm --steps 10 --warmup 2 ;;
    pbench) step bench_pipe 600 python bench.py --workload pipeline --steps 10 --warmup 2 ;;
    pbenchq) step bench_pipe 600 python bench.py --workload pipeline --steps 10 --warmup 2 --no-cpu-baseline ;;
    pprof) step rocprof_pipe 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o run --output-format csv -- python3 bench.py --workload pipeline --steps 5 --warmup 1 --no-cpu-baseline ;;
    oprof) step rocprof_ofdm 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ofdm -o run --output-format csv -- python3 bench.py --workload ofdm --steps 10 --warmup 2 --no-cpu-baseline ;;
    otraffic) step pmc_fetch_ofdm 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_ofdm -o run --output-format csv -- python3 bench.py --workload ofdm --steps 3 --warmup 1 --no-cpu-baseline && \
              step pmc_write_ofdm 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write_ofdm -o run --output-format csv -- python3 bench.py --workload ofdm --steps 3 --warmup 1 --no-cpu-baseline && \
              python3 tools/pmc_summary.py traffic gpurun_out/pmc_fetch_ofdm gpurun_out/pmc_write_ofdm gpurun_out/traffic_ofdm.json ofdm_modulate_kernel ofdm_demodulate_kernel ;;
    opmc) step pmc_ofdm 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_ofdm -o run --output-format csv -- python3 bench.py --workload ofdm --steps 2 --warmup 1 --no-cpu-baseline ;;
    save) mkdir -p gpurun_out/profiles && \
          python3 tools/pmc_summary.py stats gpurun_out/prof/run_kernel_stats.csv gpurun_out/profiles/kernel_stats.md > /dev/null && \
          cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/profiles/kernel_stats.csv && \
          cp gpurun_out/traffic.json gpurun_out/profiles/traffic.json && \
          tail -1 gpurun_out/bench.log > gpurun_out/profiles/bench.json ;;
    osave) mkdir -p gpurun_out/profiles && \
          python3 tools/pmc_summary.py stats gpurun_out/prof_ofdm/run_kernel_stats.csv gpurun_out/profiles/ofdm_kernel_stats.md > /dev/null && \
          cp gpurun_out/prof_ofdm/run_kernel_stats.csv gpurun_out/profiles/ofdm_kernel_stats.csv && \
          cp gpurun_out/traffic_ofdm.json gpurun_out/profiles/ofdm_traffic.json && \
          tail -1 gpurun_out/bench_ofdm.log > gpurun_out/profiles/ofdm_bench.json ;;
    *) echo "unknown step $s" ;;
  esac
done
