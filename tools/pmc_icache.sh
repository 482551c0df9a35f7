#!/bin/bash
# pmc_icache.sh <variant>... : instruction-cache counters of the decoder kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
for v in "$@"; do
  SRSRAN_AMD_LIB=$PWD/exp/$v/libsrsran_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQC_TC_INST_REQ -d gpurun_out/icache_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit $?
  python3 - "$v" << 'PY'
import csv, glob, sys, collections
v=sys.argv[1]; agg=collections.defaultdict(list)
for f in glob.glob('gpurun_out/icache_%s/**/*counter_collection.csv' % v, recursive=True):
    for r in csv.DictReader(open(f)):
        if 'ldpc' in r['Kernel_Name']: agg[r['Counter_Name']].append(float(r['Counter_Value']))
print(v, ' '.join('%s=%.4g' % (k, sum(x)/len(x)) for k, x in sorted(agg.items())))
PY
done
