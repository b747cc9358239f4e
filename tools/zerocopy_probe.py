"""Diagnostic: the classify kernel reading its batch straight from pinned host memory over the
link (no DMA copies: the frames' header windows and the descriptors are fetched by the kernel's
own loads; verdicts and records written back by its stores), against the DMA round trip
(upe_gpu_process_host_emit) and the device-resident launch.  Checks every verdict and record
against a device-resident run of the same batch.

Usage: python tools/zerocopy_probe.py [B|C] [reps]
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def dev_ptr(hip, p: int) -> int:
    out = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(out), ctypes.c_void_p(p), 0)
    if rc != 0:
        raise RuntimeError(f"hipHostGetDevicePointer rc={rc}")
    return out.value


def main() -> None:
    import torch

    from upe_amd import gpu, synth

    cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    wl = synth.config_b() if cfg == "B" else synth.config_c()
    n = wl.n
    # reference: device-resident emit run
    w0 = gpu.GpuWorker(0, wl.capacity)
    w0.configure(wl)
    b = gpu.DeviceBatch(w0, wl.frames, wl.desc)
    hd = w0.malloc(16 * n)
    w0.process_emit(b.frames, b.desc, b.verdict, hd, n)
    _, v_ref = b.fetch()
    r_ref = np.empty((n, 16), np.uint8)
    w0.d2h(r_ref, hd)
    w0.sync()

    pf = gpu.PinnedArray(wl.frames.shape, np.uint8)
    pd = gpu.PinnedArray(wl.desc.shape, np.uint64)
    pv = gpu.PinnedArray((n,), np.uint32)
    ph = gpu.PinnedArray((n, 16), np.uint8)
    pf.array[:] = wl.frames
    pd.array[:] = wl.desc
    f_d, d_d, v_d, h_d = (dev_ptr(hip, x.ptr) for x in (pf, pd, pv, ph))
    w = gpu.GpuWorker(0, wl.capacity)
    w.configure(wl)
    # warm-up and check
    w.process_emit(f_d, d_d, v_d, h_d, n)
    w.sync()
    vb = pv.array.copy()
    rb = ph.array.copy()
    ok_v = np.array_equal(vb & ~np.uint32(0x80), v_ref.view(np.uint32) & ~np.uint32(0x80))
    ok_r = np.array_equal(rb, r_ref)
    ts = []
    for _ in range(reps):
        pv.array[:] = 0
        t0 = time.perf_counter()
        w.process_emit(f_d, d_d, v_d, h_d, n)
        w.sync()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    # device-side outputs, frames + descriptors from the host
    v2 = w.malloc(4 * n)
    h2 = w.malloc(16 * n)
    ts2 = []
    for _ in range(reps):
        t0 = time.perf_counter()
        w.process_emit(f_d, d_d, v2, h2, n)
        w.sync()
        ts2.append(time.perf_counter() - t0)
    t2 = float(np.median(ts2))
    # DMA round trip for comparison
    ts3 = []
    for _ in range(max(3, reps // 4)):
        t0 = time.perf_counter()
        w.process_host_emit(pf.array, pd.array, pv.array, ph.array, 0, -1)
        ts3.append(time.perf_counter() - t0)
    t3 = float(np.median(ts3))
    span = int(wl.frames.nbytes)
    print(f"config {cfg}: {n} packets, frames {span / 1e6:.1f} MB in host memory")
    print(f"  zero-copy in+out : {t * 1e3:.3f} ms  {n / t / 1e6:.1f} Mpps  "
          f"(verdicts equal {ok_v}, records equal {ok_r}) min {min(ts) * 1e3:.3f}")
    print(f"  zero-copy in only: {t2 * 1e3:.3f} ms  {n / t2 / 1e6:.1f} Mpps")
    print(f"  DMA round trip   : {t3 * 1e3:.3f} ms  {n / t3 / 1e6:.1f} Mpps")
    for x in (pf, pd, pv, ph):
        x.free()
    w.close()
    w0.close()


if __name__ == "__main__":
    main()
