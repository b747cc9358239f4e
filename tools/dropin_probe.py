"""The drop-in throughput legs of bench.py (dropin_pipeline) one at a time, with knobs (round 5):

  python tools/dropin_probe.py [--seconds 2] [--pool 262144] [--ring 32768] leg...
  leg = <gpu|ref>:<mapped|window>:<workers>:<gpu_batch>, e.g. gpu:mapped:1:65536, ref:-:4:0

UPE_WORKER_PROFILE=1 makes each GPU worker loop print where its time went (launch, GPU wait,
walk, the rest) to stderr.  Threads pinned to the GPU's NUMA-local CPUs, producer first."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--pool", type=int, default=262144)
    ap.add_argument("--ring", type=int, default=32768)
    ap.add_argument("legs", nargs="+")
    args = ap.parse_args()
    import bench
    import oracle
    from upe_amd import gpu
    local, _ = gpu.local_cpus(0)
    cpus_all = [c for c in local if c in bench.ALLOWED_CPUS] or bench.ALLOWED_CPUS
    lib = ctypes.CDLL(os.path.join(os.path.dirname(oracle.__file__), "_ref", "libupe_dropin.so"))
    P, SZ, I, D = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
    lib.upe_dropin_bench.restype = I
    lib.upe_dropin_bench.argtypes = [I, I, I, I, SZ, SZ, I, I, D, D, SZ, P, P]
    for leg in args.legs:
        kind, mode, workers, gb = leg.split(":")
        workers, gb = int(workers), int(gb)
        cpus = (ctypes.c_int * (1 + workers))(*[cpus_all[k % len(cpus_all)]
                                                for k in range(1 + workers)])
        out = (ctypes.c_double * 5)()
        rc = lib.upe_dropin_bench(1 if kind == "gpu" else 0, 1 if mode == "mapped" else 0, workers,
                                  0, args.pool, args.ring, 32, 64, 0.5, args.seconds, gb, cpus, out)
        print(json.dumps({"leg": leg, "rc": rc, "consumer_mpps": round(out[0], 2),
                          "producer_mpps": round(out[1], 2), "ring_full_events": int(out[2]),
                          "seconds": round(out[3], 3)}), flush=True)


if __name__ == "__main__":
    main()
