"""Diagnostic: do HIP graphs shorten the gap between consecutive classify launches?

Config B, emit mode.  Times K launches queued from native code (upe_gpu_process_batches_emit) and
the same launches captured once into a HIP graph (torch.cuda.CUDAGraph around the native call)
and replayed, and checks that the last batch's verdicts and records agree.  The captured span
is a multiple of 6 launches, so the between-batch state slots (k % 6) line up on every replay.

Usage: python tools/graph_probe.py [span] [replays]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from upe_amd import gpu, synth

    span = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    replays = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    assert span % 6 == 0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = synth.config_b()
    n = wl.n
    w = gpu.GpuWorker(0, wl.capacity)
    w.configure(wl)
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    copies = 32
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    ptrs = [base + (k % copies) * stride for k in range(span)]

    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        w.process_batches_emit(ptrs[:24], desc, verdict, hdr, n, s.cuda_stream)   # warm-up
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(replays):
            w.process_batches_emit(ptrs, desc, verdict, hdr, n, s.cuda_stream)
        torch.cuda.synchronize(dev)
        t_stream = (time.perf_counter() - t0) / (replays * span)
        v_stream = verdict.cpu().numpy().copy()
        h_stream = hdr.cpu().numpy().copy()

    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=cs):
        w.process_batches_emit(ptrs, desc, verdict, hdr, n, torch.cuda.current_stream(dev).cuda_stream)
    g.replay()   # warm-up replay
    torch.cuda.synchronize(dev)
    verdict.zero_()
    hdr.zero_()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize(dev)
    t_graph = (time.perf_counter() - t0) / (replays * span)
    same = (np.array_equal(verdict.cpu().numpy(), v_stream) and
            np.array_equal(hdr.cpu().numpy(), h_stream))
    print(f"stream: {t_stream * 1e6:.2f} us/launch ({n / t_stream / 1e6:.0f} Mpps); "
          f"graph: {t_graph * 1e6:.2f} us/launch ({n / t_graph / 1e6:.0f} Mpps); "
          f"span {span}, replays {replays}; last batch identical: {same}")
    w.close()


if __name__ == "__main__":
    main()
