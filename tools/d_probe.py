"""Config D's classify launches with its own 64k-rule table or with a small one (round 5: the
split of the bytes past L2 into frame and table traffic).

  python tools/d_probe.py <full|small|notss> [--steps 10]

full: config D as bench.py runs it (tuple-space index); small: the same 16M frames with config B's
8-rule table (LDS-resident: no table traffic past L2, so FETCH_SIZE is the frames' and the
records'); notss: the 64k table without the tuple-space index (UPE_GPU_TSS=0, decision tree).
Emit mode over 4 distinct batch copies; prints kernel us per launch (HIP events)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant", choices=["full", "small", "notss"])
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    if args.variant == "notss":
        os.environ["UPE_GPU_TSS"] = "0"
    import torch

    from upe_amd import gpu, synth
    dev = torch.device("cuda:0")
    wl = synth.config_d()
    if args.variant == "small":
        b = synth.config_b(n=16)
        wl.rules, wl.capacity = b.rules, b.capacity
    n = wl.n
    w = gpu.GpuWorker(0, wl.capacity)
    w.configure(wl)
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    copies = 4
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    del pristine
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    ptrs = [pool.data_ptr() + (k % copies) * stride for k in range(args.steps)]
    w.process_batches_emit(ptrs[:2], desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    w.timing_span(1, 1)
    t0 = time.perf_counter()
    w.process_batches_emit(ptrs, desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    cms, gms, launches = w.timing_read()
    print(json.dumps({"variant": args.variant, "rule_index_kind": w.rule_index_kind(),
                      "classify_us": round(cms / launches * 1e3, 1),
                      "group_by_us": round(gms / launches * 1e3, 1),
                      "wall_us_per_step": round(wall / args.steps * 1e6, 1), "packets": n}),
          flush=True)
    w.close()


if __name__ == "__main__":
    main()
