"""Diagnostic: per-workgroup phase timestamps of one upe_classify launch (UPE_STAMPS build).
Usage: UPE_GPU_LIB_DIAG=build/diag/libupe_gpu_stamps.so python tools/stamps.py [packets]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from upe_amd import gpu, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
emit = (sys.argv[2] if len(sys.argv) > 2 else "emit") == "emit"
wl = synth.config_b(n=n)
w = gpu.GpuWorker(0, wl.capacity)
w.configure(wl)
dev = torch.device("cuda", 0)
frames = [torch.from_numpy(wl.frames).to(dev) for _ in range(6)]
desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
verdict = torch.empty(n, dtype=torch.int32, device=dev)
hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
lib = gpu.LIB
lib.upe_gpu_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
names = ["entry", "init", "win", "scan", "loop", "flush", "wait", "ticket", "tail", "reduced", "barrier"]
for rep in range(6):
    buf = np.zeros(8192 * 16, np.uint64)
    lib.upe_gpu_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), 0)  # no-op read
    if emit:
        w.process_emit(frames[rep], desc, verdict, hdr, n)
    else:
        w.process(frames[rep], desc, verdict, n)
    w.sync()
    lib.upe_gpu_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes)
    ntiles = (n + 255) // 256
    grid = min(ntiles, 8192)
    st = buf.reshape(8192, 16)[:grid, :11].astype(np.int64)
    valid = st[:, 0] > 0
    st = st[valid]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1000.0  # 100 MHz ticks -> us
    print(f"rep {rep}: grid {st.shape[0]} WGs; end of kernel ~{rel[:, 7].max():.2f} us; tail end "
          f"{rel[:, 8].max():.2f} us")
    if rep == 5:
        # where the loop-end spread comes from: by blockIdx % 8 (the XCD group) and by start time
        loop = rel[:, 4]
        ent = rel[:, 0]
        b = np.nonzero(valid)[0]
        for g in range(8):
            sel = (b % 8) == g
            print(f"   xcd-group {g}: loop end med {np.median(loop[sel]):6.2f} max {loop[sel].max():6.2f}"
                  f"  entry med {np.median(ent[sel]):5.2f}")
        order = np.argsort(ent)
        q = np.array_split(order, 4)
        for k, idx in enumerate(q):
            print(f"   entry quartile {k}: entry {np.median(ent[idx]):5.2f} loop end med "
                  f"{np.median(loop[idx]):6.2f} max {loop[idx].max():6.2f}")
        print("   corr(entry, loop end) =", round(float(np.corrcoef(ent, loop)[0, 1]), 3))
        last = np.argsort(loop)[-10:]
        print("   10 latest loop ends: blocks", b[last].tolist(), "entry", np.round(ent[last], 2).tolist())
    for j, nm in enumerate(names):
        col = rel[:, j]
        col = col[col >= 0]
        if j == 8:
            col = rel[:, 8][st[:, 8] > 0]
        if col.size:
            print(f"   {nm:7s} min {col.min():7.2f} med {np.median(col):7.2f} max {col.max():7.2f}")
