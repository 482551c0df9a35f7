"""Every bench.py workload runs and prints one JSON line (tiny sizes: a broken secondary workload would otherwise
only show at the round-end bench)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(__file__), "..")


@pytest.mark.parametrize("args", [["--workload", "sch_slot", "--slots-pipeline", "2"],
                                  ["--workload", "slot_pipeline", "--slots-pipeline", "2"],
                                  ["--workload", "slot_pipeline", "--mixed", "--slots-pipeline", "2"],
                                  ["--workload", "pucch", "--slots-pipeline", "2", "--cpu-seconds", "0.2"]],
                         ids=["sch_slot", "slot_pipeline", "slot_pipeline_mixed", "pucch"])
def test_bench_workload_line(args):
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"] + args,
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    unit = "UCI messages/s" if "pucch" in args else "codeblocks/s"
    assert line["value"] > 0 and line["unit"] == unit, line
