"""Debug: verdict codes after a rule reload — is the next launch's view of the rule table fresh
when nothing but the reload happens between the launches?"""
import dataclasses
import sys

import numpy as np

sys.path.insert(0, "tests")
import reload_util  # noqa: E402
from upe_amd import gpu, synth  # noqa: E402

wl, rules_b, at, cap_b = reload_util.case("B")
wl = dataclasses.replace(wl, desc=wl.desc[:8192])
at = 4096
rs_b = synth.build_rule_table(rules_b)


def hist(v):
    return np.bincount(v & 0xF, minlength=8).tolist()


for want_old in (True, False):
    for pre in (False, True):
        w = gpu.GpuWorker(0, wl.capacity)
        w.configure(wl)
        b1 = gpu.DeviceBatch(w, wl.frames, wl.desc[:at])
        if pre:   # the second batch's buffers made before the reload: nothing between
            b2 = gpu.DeviceBatch(w, wl.frames, wl.desc[at:])
        b1.run()
        _, v1 = b1.fetch()
        if pre:
            b2.run()   # a second launch with table A, so the rules are cached everywhere
            w.sync()
        w.reload_rules(rs_b, cap_b, want_old=want_old)
        if not pre:
            b2 = gpu.DeviceBatch(w, wl.frames, wl.desc[at:])
        b2.run()
        _, v2 = b2.fetch()
        print(f"want_old={want_old} pre={pre}: part1 {hist(v1)} part2 {hist(v2)}", flush=True)
        w.close()
