#!/usr/bin/env python3
"""Back-to-back launch floor on this box: HIP-event time per launch of a tiny torch kernel,
to compare against the collective's small-message step time."""
import torch

x = torch.zeros(32, device="cuda")
for _ in range(50):
    x.add_(1)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(1000):
    x.add_(1)
b.record()
torch.cuda.synchronize()
print("tiny torch kernel: %.2f us per launch (back-to-back)" % (a.elapsed_time(b) * 1000 / 1000))
