"""Extracts the reference's TBS calculator test vectors
(tests/unittests/ran/sch/tbs_calculator_test_data.h, generated there by
srsTBSCalculatorUnittest.m) into tests/golden/tbs_calculator.json -- data only."""
import json
import os
import re
import sys

SRC = os.path.join(sys.argv[1] if len(sys.argv) > 1 else "/root/reference",
                   "tests/unittests/ran/sch/tbs_calculator_test_data.h")
QM = {"QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}
pat = re.compile(r"\{\{(\d+), (\d+), (\d+), \{modulation_scheme::(\w+), ([0-9.]+)\}, (\d+), (\d+), (\d+)\}, (\d+)\}")
cases = []
for m in pat.finditer(open(SRC).read()):
    symb, dmrs, oh, mod, tcr, layers, scaling, nprb, tbs = m.groups()
    cases.append(dict(nof_symb_sh=int(symb), nof_dmrs_prb=int(dmrs), nof_oh_prb=int(oh), qm=QM[mod],
                      target_code_rate=tcr, nof_layers=int(layers), tb_scaling_field=int(scaling), n_prb=int(nprb),
                      tbs=int(tbs)))
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "tbs_calculator.json")
json.dump({"source": "srsRAN tests/unittests/ran/sch/tbs_calculator_test_data.h", "cases": cases}, open(out, "w"),
          indent=0)
print(len(cases), "cases ->", out)
