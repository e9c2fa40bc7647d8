#!/usr/bin/env python3
"""PCIe probe for the host E2E path: pinned H2D alone, D2H alone, and both
directions at once on two streams (SDMA overlap).  Prints one JSON line."""
import json
import time

import torch

N = 256 << 20
REPS = 8


def run(h2d: bool, d2h: bool) -> float:
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        if h2d:
            with torch.cuda.stream(s1):
                dA.copy_(hA, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                hB.copy_(dB, non_blocking=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return round(REPS * N * (int(h2d) + int(d2h)) / el / 1e9, 1)


hA = torch.empty(N, dtype=torch.uint8).pin_memory()
hB = torch.empty(N, dtype=torch.uint8).pin_memory()
dA = torch.empty(N, dtype=torch.uint8, device="cuda")
dB = torch.empty(N, dtype=torch.uint8, device="cuda")
run(True, True)
print(json.dumps({"h2d_GBps": run(True, False), "d2h_GBps": run(False, True),
                  "both_total_GBps": run(True, True)}))
