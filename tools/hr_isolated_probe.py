"""The headline PUSCH decoder launch (ldpc_decode_hr_kernel over one step's 64 x 141 codeblocks, rows of the
9,216-LLR non-zero prefix, CRC24B early stop) run alone, serialized on one stream, so that per-dispatch PMC counters
(rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, tools/pmc_db.py) see no concurrent kernel: run under rocprofv3 from the
repository root, PYTHONPATH=. python tools/hr_isolated_probe.py."""
import torch

import bench_pipeline as bp

dev = torch.device("cuda", 0)
pl = bp.Pipeline(64, dev)
s = torch.cuda.current_stream(dev)
pl.step(s)
torch.cuda.synchronize(dev)
ms, nbytes, cbs, its = pl.ldpc_decoder_ms(s)
print("hr decoder alone: %.4f ms per launch, %d codeblocks, %.3f iterations, %d algorithmic bytes" % (ms, cbs, its, nbytes))
