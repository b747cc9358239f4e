"""Diagnostic: config C (1M IMIX) as an ordinary batch (upe_gpu_process_emit) and as a
header-split batch (upe_gpu_process_split_emit: each packet's first 64 bytes in a dense row), the
same kernel timing for both: `copies` distinct batch copies (frames and rows) cycled so nothing
is served from the Infinity Cache, launches queued from Python, per-launch kernel time from HIP
events around `span` launches.  Usage: python tools/split_probe.py [C|B|D] [launches]"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> None:
    import torch

    from upe_amd import gpu, synth

    cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 120
    wl = {"B": synth.config_b, "C": synth.config_c, "D": lambda: synth.config_d(n=1 << 22)}[cfg]()
    n = wl.n
    dev = torch.device("cuda", 0)
    rows = synth.header_rows(wl)
    copies = 24
    fb = (wl.frames.nbytes + 255) // 256 * 256
    rb = rows.nbytes
    fr = torch.from_numpy(wl.frames).to(dev)
    rw = torch.from_numpy(rows.reshape(-1)).to(dev)
    pool_f = torch.empty(copies * fb, dtype=torch.uint8, device=dev)
    pool_r = torch.empty(copies * rb, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool_f[c * fb: c * fb + wl.frames.nbytes].copy_(fr)
        pool_r[c * rb: (c + 1) * rb].copy_(rw)
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    w = gpu.GpuWorker(0, wl.capacity)
    w.configure(wl)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bf, br = pool_f.data_ptr(), pool_r.data_ptr()

    def run(split: bool, k0: int, count: int) -> None:
        for k in range(k0, k0 + count):
            c = k % copies
            if split:
                w.process_split_emit(br + c * rb, bf + c * fb, desc, verdict, hdr, n, sh)
            else:
                w.process_emit(bf + c * fb, desc, verdict, hdr, n, sh)

    out = {}
    for rep in range(2):
        for split in (False, True):
            run(split, 0, 10)
            torch.cuda.synchronize(dev)
            w.timing_span(10, 5)
            t0 = time.perf_counter()
            run(split, 10, launches)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            cms, _, nl = w.timing_read()
            w.timing_enable(False)
            out[(rep, split)] = (dt / launches * 1e6, cms / nl * 1e3 if nl else float("nan"))
    v = verdict.cpu().numpy().view(np.uint32)
    print(f"config {cfg}: {n} packets, {copies} copies of frames ({fb / 1e6:.0f} MB) and rows "
          f"({rb / 1e6:.0f} MB)")
    for (rep, split), (wall, kern) in sorted(out.items()):
        print(f"  rep {rep} {'split ' if split else 'packed'}: {wall:7.2f} us per launch (wall), "
              f"kernel {kern:7.2f} us, {n / kern / 1e3:8.1f} Gpps by kernel time")
    print("  forwarded:", int(np.count_nonzero((v & 0xF) == 4)))
    w.close()


if __name__ == "__main__":
    main()
