"""Kernel time per 1M-packet batch of the IMIX workloads under each rule-match flavour (round 5).

  python tools/tree_probe.py [--steps 60] [--out gpurun_out/tree_probe.jsonl] [cases...]

cases: CF (config C, flow-derived rules), C3 (seed-3 config C), C6 (C with IPv6 forwarded),
each as <case>:<flavour> with flavour tree (decision tree, image staged in LDS), treemem (the
tree read from memory), scan (UPE_GPU_TREE=0: family lists /
whole-table scan).  Emit mode,
batches queued from native code (upe_gpu_process_batches_emit) over 8 distinct copies; HIP-event
kernel time per launch (upe_gpu_timing_*), plus a check of the verdicts against the previous
flavour of the same case (every flavour must agree)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tree_probe.jsonl"))
    ap.add_argument("cases", nargs="*", default=["CF:tree", "CF:treemem", "CF:scan",
                                                  "C6:tree", "C6:scan", "C3:tree",
                                                  "C3:scan"])
    args = ap.parse_args()
    import torch

    from upe_amd import gpu, synth

    dev = torch.device("cuda:0")
    def mixed_64k():
        # the parity test's 64k-rule many-signature table over config C's traffic
        wl = synth.config_c(seed=61)
        wl.rules, wl.capacity = synth.mixed_table(1 << 16, 61), 1 << 16
        return wl

    makers = {"B": lambda: synth.config_b(), "CF": lambda: synth.config_c_flows(),
              "M64k": mixed_64k,
              "F16k": lambda: synth.config_c_flows(seed=62, n_rules=1 << 14, max_cover=2.0 ** -18),
              "C3": lambda: synth.config_c(),
              "C6": lambda: synth.config_c(v6_forwarding=True)}
    cache: dict = {}
    ref_verdict: dict = {}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    for case in args.cases:
        name, flavour = case.split(":")
        if name not in cache:
            cache.clear()
            cache[name] = makers[name]()
        wl = cache[name]
        os.environ["UPE_GPU_TREE"] = "0" if flavour == "scan" else "1"
        os.environ["UPE_GPU_TREE_LDS"] = "0" if flavour == "treemem" else "1"
        w = gpu.GpuWorker(0, wl.capacity)
        w.configure(wl)
        n = wl.n
        fbytes = int(wl.frames.nbytes)
        stride = (fbytes + 255) // 256 * 256
        copies = 8
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
        w.process_batches_emit(ptrs[:8], desc, verdict, hdr, n, sh)
        torch.cuda.synchronize(dev)
        w.timing_span(10, 5)
        t0 = time.perf_counter()
        w.process_batches_emit(ptrs, desc, verdict, hdr, n, sh)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        cms, gms, launches = w.timing_read()
        info = w.launch_info()
        idx = w.rule_index_info()
        v = verdict.cpu().numpy().view(np.uint32).copy()
        w.close()
        del pool, desc, verdict, hdr
        same = None
        if name in ref_verdict:
            same = bool(np.array_equal(ref_verdict[name], v))
        else:
            ref_verdict[name] = v
        rec = {"case": name, "flavour": flavour, "kernel_us": round((cms + gms) / launches * 1e3, 2),
               "wall_us_per_step": round(wall / args.steps * 1e6, 2), "launches": launches,
               "variant": int(info["variant"]), "index": {k: int(idx[k]) for k in idx.dtype.names},
               "agrees_with_first_flavour": same,
               "codes": np.bincount(v & 0xF, minlength=7).tolist()}
        print(json.dumps(rec), flush=True)
        with open(args.out, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
