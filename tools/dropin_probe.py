"""Drop-in pipeline probe (diagnostic, GPU box): the reference throughput benchmark's GPU-worker
legs only, run as `python tools/dropin_probe.py [pool ring gpu mapped workers ...]`, with
UPE_WORKER_PROFILE / UPE_WORKER_PF taken from the environment.  One JSON line per leg."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (ALLOWED_CPUS, numa-local CPUs)
import oracle  # noqa: E402


def main() -> None:
    so = os.path.join(os.path.dirname(oracle.__file__), "_ref", "libupe_dropin.so")
    lib = ctypes.CDLL(so)
    P, SZ, I, D = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
    lib.upe_dropin_bench.restype = I
    lib.upe_dropin_bench.argtypes = [I, I, I, I, SZ, SZ, I, I, D, D, SZ, P, P]
    args = [int(a) for a in sys.argv[1:]] or [262144, 32768, 1, 1, 1]
    from upe_amd import gpu
    local, _ = gpu.local_cpus(0)
    cpus_all = [c for c in (local or []) if c in bench.ALLOWED_CPUS] or bench.ALLOWED_CPUS
    for k in range(0, len(args), 5):
        pool, ring, gpu, mapped, workers = args[k:k + 5]
        cpus = (ctypes.c_int * (1 + workers))(*[cpus_all[j % len(cpus_all)]
                                                for j in range(1 + workers)])
        out = (ctypes.c_double * 5)()
        rc = lib.upe_dropin_bench(gpu, mapped, workers, 0, pool, ring, 32, 64, 0.5, 2.0, 65536,
                                  cpus, out)
        print(json.dumps({"pool": pool, "ring": ring, "gpu": gpu, "mapped": mapped,
                          "workers": workers, "rc": rc, "pf": os.environ.get("UPE_WORKER_PF"),
                          "consumer_mpps": round(out[0], 2), "ring_full": int(out[2])}),
              flush=True)


if __name__ == "__main__":
    main()
