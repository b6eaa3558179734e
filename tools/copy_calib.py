#!/usr/bin/env python3
"""Calibration: device-to-device copy rate of 1 GiB on this GPU (torch copy_,
hipMemcpyDtoD underneath) -- the practical ceiling for the text.csv copy."""
import torch

n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.empty(n, dtype=torch.uint8, device="cuda")
x.fill_(7)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    y.copy_(x)
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 20
print(f"copy 1 GiB: {ms:.3f} ms = {2 * n / ms / 1e6:.0f} GB/s (read + write)")
