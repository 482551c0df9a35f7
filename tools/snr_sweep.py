"""PUSCH SNR sweep of the slot pipeline (8 cells): mean LDPC iterations and TB success per SNR, to place the
bench's realistic-SNR line (--low-snr-db) where the decoder runs several iterations."""
import sys

import torch

sys.path.insert(0, ".")
import bench_pipeline as bp  # noqa: E402

dev = torch.device("cuda", 0)
for snr in [float(x) for x in sys.argv[1:]] or [30.0, 27.0, 25.0, 24.0, 23.0, 22.0, 21.0]:
    pl = bp.Pipeline(8, dev, snr_db=snr)
    s = torch.cuda.current_stream(dev)
    pl.step(s)
    torch.cuda.synchronize(dev)
    ok, its = pl.check()
    print("snr %.1f dB: iterations %.2f, TB ok %.3f" % (snr, its, ok), flush=True)
