"""Diagnostic: per-workgroup phase timestamps of one upe_classify launch (UPE_STAMPS build).
Usage: UPE_GPU_LIB_DIAG=build/var/stamps.so python tools/stamps.py [packets] [emit|inplace] [B|C]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from upe_amd import gpu, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
emit = (sys.argv[2] if len(sys.argv) > 2 else "emit") == "emit"
cfg = sys.argv[3] if len(sys.argv) > 3 else "B"
wl = {"B": synth.config_b, "C": synth.config_c}[cfg](n=n)
w = gpu.GpuWorker(0, wl.capacity)
w.configure(wl)
dev = torch.device("cuda", 0)
frames = [torch.from_numpy(wl.frames).to(dev) for _ in range(6)]
desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
verdict = torch.empty(n, dtype=torch.int32, device=dev)
hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
lib = gpu.LIB
lib.upe_gpu_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
names = ["entry", "init", "win", "scan", "loop", "flush", "-", "-", "-", "reduced", "barrier"]
for rep in range(6):
    buf = np.zeros(8192 * 16, np.uint64)
    lib.upe_gpu_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), 0)  # no-op read
    # the last of 4 back-to-back launches (as the bench queues them), not an isolated one
    for k in range(4):
        f = frames[(rep + k) % len(frames)]
        if emit:
            w.process_emit(f, desc, verdict, hdr, n)
        else:
            w.process(f, desc, verdict, n)
    w.sync()
    lib.upe_gpu_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes)
    # stamps of launch k sit in slot k % 4 (2048 workgroup rows each)
    slots = buf.reshape(4, 2048, 16).astype(np.int64)
    spans = []
    for sl in range(4):
        e = slots[sl, :, 0]
        ok = e > 0
        if ok.any():
            spans.append((e[ok].min(), slots[sl, ok, 5].max(), sl))
    spans.sort()
    if len(spans) > 1:
        gaps = [(spans[j + 1][0] - spans[j][1]) / 100.0 for j in range(len(spans) - 1)]
        lens = [(b - a) / 100.0 for a, b, _ in spans]
        print(f"rep {rep}: launch spans (first entry -> last flush) {np.round(lens, 2).tolist()} us; "
              f"gaps (last flush -> next first entry) {np.round(gaps, 2).tolist()} us")
    raw = slots[spans[-1][2]]
    st = raw[:, :11]
    valid = st[:, 0] > 0
    st = st[valid]
    xcc = raw[valid, 11]
    hw = raw[valid, 12]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1000.0  # 100 MHz ticks -> us
    print(f"rep {rep}: grid {st.shape[0]} WGs; last flush {rel[:, 5].max():.2f} us")
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
        # by the XCC the workgroup really ran on (HW_REG_XCC_ID), and by CU within it
        cu = (xcc << 8) | (((hw >> 13) & 7) << 4) | ((hw >> 8) & 15)
        for g in range(8):
            sel = xcc == g
            if sel.any():
                print(f"   XCC {g}: {sel.sum():4d} WGs on {np.unique(cu[sel]).size:3d} CUs; entry med "
                      f"{np.median(ent[sel]):5.2f} max {ent[sel].max():5.2f}; loop end med "
                      f"{np.median(loop[sel]):6.2f} max {loop[sel].max():6.2f}; blockIdx%8 "
                      f"{np.unique(b[sel] % 8).tolist()}")
        ucu, cnt = np.unique(cu, return_counts=True)
        print("   WGs per CU:", dict(zip(*np.unique(cnt, return_counts=True))))
        cu_end = {c: loop[cu == c].max() for c in ucu}
        worst = sorted(cu_end, key=cu_end.get)[-6:]
        for c in worst:
            sel = cu == c
            print(f"   slow CU xcc{c >> 8} se{(c >> 4) & 15} cu{c & 15}: loop ends "
                  f"{np.round(np.sort(loop[sel]), 2).tolist()} entries {np.round(np.sort(ent[sel]), 2).tolist()}")
        last = np.argsort(loop)[-10:]
        print("   10 latest loop ends: blocks", b[last].tolist(), "entry", np.round(ent[last], 2).tolist())
    for j, nm in enumerate(names):
        if nm == "-":
            continue
        col = rel[:, j]
        col = col[col >= 0]
        if col.size:
            print(f"   {nm:7s} min {col.min():7.2f} med {np.median(col):7.2f} max {col.max():7.2f}")
