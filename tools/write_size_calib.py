"""WRITE_SIZE / FETCH_SIZE calibration on known byte counts (MI355X_MICROARCH.md: only 16-B-per-lane streaming
accesses are calibrated): torch fills of 9,565,440 bytes (the headline decoder's 9024 x 1060 output bytes) and of
256 MiB, then a 256 MiB copy.  Run under rocprofv3 --pmc WRITE_SIZE (or FETCH_SIZE) and read the per-dispatch rows
with tools/pmc_db.py <dir> elementwise."""
import torch

dev = torch.device("cuda", 0)
small = torch.empty(9024 * 1060, dtype=torch.uint8, device=dev)
big = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
dst = torch.empty_like(big)
for _ in range(3):
    small.fill_(1)
for _ in range(3):
    big.fill_(2)
for _ in range(3):
    dst.copy_(big)
torch.cuda.synchronize(dev)
print("bytes: small fill %d, big fill %d, copy %d read + %d written" % (small.numel(), big.numel(), big.numel(),
                                                                    dst.numel()))
