"""Emit-mode records (include/upe_gpu.h upe_hdr_rec_t) on the CPU: a record built from the
reference worker's rewritten frame (the bytes process_packet changes, src/worker.c:162-244),
applied to the original frame by the library's upe_hdr_apply, gives back exactly that rewritten
frame.  So the 16-byte record carries every byte the reference rewrites; the GPU tests then
compare the kernel's records with these."""
from __future__ import annotations

import numpy as np

import golden_io
from upe_amd import gpu
from upe_amd.layout import V_FWD, desc_lens, desc_offsets


def records_from_reference(frames_in, frames_out, desc, verdict) -> np.ndarray:
    """The record the format defines for each packet, from the reference's output frame."""
    offs = desc_offsets(desc)
    rec = np.zeros((len(offs), 16), np.uint8)
    for i in np.nonzero((verdict & 0xF) == V_FWD)[0]:
        o = int(offs[i])
        out = frames_out[o:o + 26]
        v6 = frames_in[o + 12] == 0x86 and frames_in[o + 13] == 0xDD
        rec[i, :12] = out[:12]
        if v6:
            rec[i, 12] = out[21]
            rec[i, 15] = 6
        else:
            rec[i, 12] = out[22]
            rec[i, 13:15] = out[24:26]
            rec[i, 15] = 4
    return rec


def test_apply_reproduces_reference_frames():
    for case in ("config_b_small", "config_c_small", "config_d_small"):
        wl, ref = golden_io.load(case)
        rec = records_from_reference(wl.frames, ref["frames"], wl.desc, ref["verdict"])
        out = gpu.hdr_apply(wl.frames, wl.desc, rec)
        assert np.array_equal(out, ref["frames"]), case
        fwd = (ref["verdict"] & 0xF) == V_FWD
        assert np.count_nonzero(rec[:, 15]) == np.count_nonzero(fwd)


def test_apply_is_a_no_op_for_zero_records():
    wl, _ = golden_io.load("config_b_small")
    rec = np.zeros((wl.n, 16), np.uint8)
    assert np.array_equal(gpu.hdr_apply(wl.frames, wl.desc, rec), wl.frames)


def test_only_rewritten_bytes_change():
    """Nothing outside bytes 0..11, 21, 22, 24, 25 of a frame is ever written."""
    wl, ref = golden_io.load("config_c_small")
    offs, lens = desc_offsets(wl.desc), desc_lens(wl.desc)
    allowed = np.zeros(26, bool)
    allowed[list(range(12)) + [21, 22, 24, 25]] = True
    for o, ln in zip(offs[:4000], lens[:4000]):
        diff = np.nonzero(wl.frames[o:o + ln] != ref["frames"][o:o + ln])[0]
        assert all(d < 26 and allowed[d] for d in diff)
