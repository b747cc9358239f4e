"""Diagnostic: pinned host -> device copy rate with the bytes split over 1, 2, 4 streams (does
more than one copy engine raise the H2D rate the host round trip is bound by?), and the same
with a concurrent device -> host copy.  Usage: python tools/h2d_probe.py [MiB]"""
from __future__ import annotations

import sys
import time


def main() -> None:
    import torch

    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    dev = torch.device("cuda", 0)
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]

    def h2d(k: int, back: bool, reps: int = 8) -> float:
        part = n // k
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            for j in range(k):
                with torch.cuda.stream(streams[j]):
                    d[j * part:(j + 1) * part].copy_(h[j * part:(j + 1) * part], non_blocking=True)
            if back:
                with torch.cuda.stream(streams[3]):
                    h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize(dev)
        return n * reps / (time.perf_counter() - t0) / 1e9

    h2d(1, False, 2)
    for k in (1, 2, 3):
        print(f"H2D {mib} MiB over {k} stream(s): {h2d(k, False):.1f} GB/s; "
              f"with a concurrent D2H of the same size: {h2d(k, True):.1f} GB/s (H2D bytes only)")


if __name__ == "__main__":
    main()
