"""Diagnostic: config C (1M IMIX, 1k rules, ARP + NDP forwarding) under one setting per process,
timed like bench.py (emit mode, distinct batch copies cycled, HIP events around 5 launches):

  packed       upe_gpu_process_emit from a calloc'd worker (the NDP entry :: -> 00:..:00 does
               not agree with the NDP table, so the decoupled look-back stays live)
  agree        packed, but the L1 entries set to entries the tables hold (upe_gpu_set_l1): the
               launches switch to the kernel without look-back
  c6           packed, config C with its family-wide wildcards last (synth.config_c
               v6_forwarding=True): IPv6 forwarded through NDP, deep rule scans
(round 4 also measured header-split batches, since removed: profiles/pmc_configC_limiter.json)

With UPE_GPU_LIB_DIAG=<ablation build> the same runs time a kernel with parts removed (results
wrong by design).  Usage: python tools/c_probe.py <setting> [launches] > json line."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main() -> None:
    import torch

    from upe_amd import gpu, synth
    from upe_amd.layout import L1_DTYPE

    setting = sys.argv[1] if len(sys.argv) > 1 else "packed"
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    wl = synth.config_c(v6_forwarding=setting == "c6")
    n = wl.n
    dev = torch.device("cuda", 0)
    copies = 24
    fb = (wl.frames.nbytes + 255) // 256 * 256
    fr = torch.from_numpy(wl.frames).to(dev)
    pool_f = torch.empty(copies * fb, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool_f[c * fb: c * fb + wl.frames.nbytes].copy_(fr)
    del fr
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    w = gpu.GpuWorker(0, wl.capacity)
    w.configure(wl)
    if "agree" in setting:
        l1 = np.zeros(1, L1_DTYPE)
        a = wl.arp[wl.arp["valid"] == 1][0]
        d = wl.ndp[wl.ndp["valid"] == 1][0]
        l1["last_arp_ip"] = a["ip"]
        l1["last_arp_mac"] = a["mac"]
        l1["last_ndp_ip"] = d["ip"]
        l1["last_ndp_mac"] = d["mac"]
        w.set_l1(l1)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bf = pool_f.data_ptr()

    def run(k0: int, count: int) -> None:
        for k in range(k0, k0 + count):
            c = k % copies
            w.process_emit(bf + c * fb, desc, verdict, hdr, n, sh)

    run(0, 20)
    torch.cuda.synchronize(dev)
    w.timing_span(20, 5)
    t0 = time.perf_counter()
    run(20, launches)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    cms, gms, nl = w.timing_read()
    info = w.launch_info()
    v = verdict.cpu().numpy().view(np.uint32)
    w.close()
    print(json.dumps({"setting": setting, "lib": os.environ.get("UPE_GPU_LIB_DIAG", "product"),
                      "wall_us_per_launch": round(dt / launches * 1e6, 3),
                      "kernel_us": round((cms + gms) / nl * 1e3, 3) if nl else None,
                      "variant": info["variant"], "deferred": info["deferred"],
                      "forwarded": int(np.count_nonzero((v & 0xF) == 4))}), flush=True)


if __name__ == "__main__":
    main()
