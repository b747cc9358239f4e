"""bench.py — device-resident Mpps of the UPE worker hot path on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path (one upe_gpu_process_emit call through the C ABI: the
classify launch, plus the rule_stats group-by for tables over 4096 rules) over one batch already
resident in HBM.  The default output mode is emit (include/upe_gpu.h): verdicts plus one 16-byte
rewritten-header record per packet, frames read only; --mode inplace rewrites the frames in place
as upe_gpu_process does, and the JSON line carries the other mode's rate too ("other_mode").  At N=1 the workload is BASELINE.json configs[1] (config B: 1M x 64 B UDP/IPv4, 8 rules);
--config A / C / D run the other configurations.  A config-B run also times the IMIX workload
(config C) after the main region, on every rank, and reports it as "imix" (not `value`), so that
the 64 B and IMIX rates come out of the same run at each GPU count.  Every step gets its own pristine copy of the
batch (the path rewrites TTL / checksum / MACs in place, so re-running a batch would change the
work), which also keeps the working set past the 256 MiB Infinity Cache: inputs come from HBM.

Multi-GPU (`python bench.py --gpus N`, which starts the N ranks under torch.distributed.run
itself, or the same launcher run by the caller): one process per GPU, each with its own static
shard of the packet stream (a full config-B batch per step, tables replicated), no data-path
collective — weak scaling.  torch.distributed carries only the barrier and the max-over-ranks
time.  The CPU baseline is timed by rank 0 after the timed regions at every N.

After the timed region (never part of `value`): the other output mode, the IMIX leg, the ring
leg (16 resident batches per launch), the achievable-bandwidth probe, and the host-inclusive legs
— the DMA round trip (upe_gpu_process_host[_emit]: pinned hipMemcpyAsync in and out) and the mapped
path (upe_gpu_process_mapped[_emit]: the kernel reads and writes the pinned host batch over the
link itself), the latter with a link roofline (the same algorithmic bytes / time against PCIe Gen5
x16's 64 GB/s).

Prints ONE JSON line (rank 0).  roofline.achieved = algorithmic bytes per launch (SURVEY.md
§8(d): B(p) = 8 + E(p) + 4 + W(p)) / the mean launch duration, measured with HIP events on the
launch stream over the timed region (each sample's event pair brackets EVENT_SPAN consecutive
launches); roofline.traffic = HBM bytes per launch from the committed PMC passes
(profiles/pmc_config<X>.json).  cpu_baseline = the reference
src/worker.c (oracle/_ref, built from the reference sources) timed on this host's cores over a
bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LINK_PEAK_GBPS = 64.0   # PCIe Gen5 x16 per direction, theoretical
ALLOWED_CPUS = sorted(os.sched_getaffinity(0))   # the process's CPUs, before the host thread is pinned
EVENT_EVERY = 20  # a kernel-timing sample on timed steps 10, 30, 50, ... (10 samples at K=200)
EVENT_SPAN = 5    # each sample's HIP event pair brackets 5 consecutive launches
METRIC = "Mpps parse+classify (device-resident), 64B & IMIX; achieved HBM GB/s vs peak"
WORKLOADS = {
    "A": "A: 10k x 64B UDP/IPv4 pcap-replay records, rules.example (configs[0], the reference's "
         "own CPU case), replayed as device-resident batches",
    "B": "B: 1M x 64B UDP/IPv4, 8 rules, ARP 240/256 hit (BASELINE configs[1])",
    "C": "C: 1M IMIX 64/570/1518 v4+v6, 1k 5-tuple rules cut from the traffic's flows (first "
         "matches spread over the whole table, both families), ARP+NDP L3 fwd (configs[2], "
         "synth.config_c_flows)",
    "C3": "C (seed-3 draw, rounds 1-4): 1M IMIX v4+v6, 1k random 5-tuple rules; every IPv4 packet "
          "stops by sorted rule 11, every IPv6 packet at rule 0 (synth.config_c)",
    "C6": "C seed-3 with its family-wide wildcard rules last: IPv6 forwarded through NDP, IPv6 "
          "first matches spread (synth.config_c(v6_forwarding=True))",
    "D": "D: 16M mixed/malformed, 64k rules (configs[3])",
}


def algorithmic_bytes(wl, verdict: np.ndarray, emit: bool = False) -> np.ndarray:
    """B(p) per packet, SURVEY.md §8(d).  In emit mode W(p) is the 16-byte record of a forwarded
    packet (the records of other packets are zero and not counted)."""
    from upe_amd.layout import desc_lens, desc_offsets

    offs = desc_offsets(wl.desc)
    lens = desc_lens(wl.desc)
    fr = wl.frames
    et = (fr[offs + 12].astype(np.int64) << 8) | fr[offs + 13]
    is4 = et == 0x0800
    is6 = et == 0x86DD
    ihl = (fr[offs + 14] & 0xF).astype(np.int64)
    proto = np.where(is4, fr[offs + 23], np.where(is6, fr[offs + 20], 0)).astype(np.int64)
    l3 = np.where(is4, ihl * 4, 40)
    l4 = np.where(proto == 6, 20, 8)
    code = verdict & 0xF
    parsed = (code != 0) & (code != 5)
    ext = np.where(parsed, 14 + l3 + l4, 34)
    ext = np.where((code == 5) | (et == 0x0806), 78, ext)
    E = np.minimum(lens, ext)
    fwd = code == 4
    hit = (verdict & 0x10) != 0
    W = np.where(fwd & is4, 3, 0) + np.where(fwd & is6, 1, 0) + np.where(fwd & hit, 12, 0)
    if emit:
        W = np.where(fwd, 16, 0)
    return 8 + E + 4 + W


def rule_evals(wl, verdict: np.ndarray) -> int:
    """Rule tests the reference's linear first-match scan makes on this batch
    (src/rule_table.c:163-176): first-match position for matched packets, the whole table for
    parsed packets that match nothing, none for parse failures."""
    code = verdict & 0xF
    rule = (verdict >> 8).astype(np.int64)   # sorted index + 1, 0 = no match
    parsed = (code != 0) & (code != 5)
    return int(np.where(rule > 0, rule, np.where(parsed, len(wl.rules), 0)).sum())


def shared_gpu_workers(torch, dev, wl, worker0, pool, stride: int, copies: int, desc,
                       workers: int, steps: int) -> dict:
    """W worker contexts on one GPU (the reference runs several worker threads; each maps to a
    context): worker w takes the batch copies k with k % W == w, on its own stream, so one
    worker's per-launch start and tail overlap another's middle.  Outside the timed region of
    `value`."""
    from upe_amd import gpu

    ws = [worker0] + [gpu.GpuWorker(dev.index, wl.capacity) for _ in range(workers - 1)]
    for w in ws[1:]:
        w.configure(wl)
    streams = [torch.cuda.Stream(dev) for _ in ws]
    verdicts = [torch.empty(wl.n, dtype=torch.int32, device=dev) for _ in ws]
    base = pool.data_ptr()
    mine = [[base + (k % copies) * stride for k in range(copies) if k % workers == j]
            for j in range(workers)]

    def run(count: int) -> None:
        for j, w in enumerate(ws):
            lst = [mine[j][k % len(mine[j])] for k in range(count)]
            w.process_batches(lst, desc, verdicts[j], wl.n, streams[j].cuda_stream)

    run(3)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    for w in ws[1:]:
        w.close()
    return {"workers": workers, "value": round(workers * steps * wl.n / dt / 1e6, 2),
            "unit": "Mpps", "ms_per_round": round(dt / steps * 1e3, 5),
            "what": f"{workers} worker contexts on this GPU, {steps} batches each, own streams"}


def hbm_probe(torch, dev, gib: int = 4, reps: int = 10) -> dict:
    """Achievable HBM streaming rates on this GPU (SURVEY.md §8(d) asks for them beside the
    nominal 8 TB/s): a device-to-device copy and a read-only reduction over `gib` GiB buffers,
    timed with HIP events; outside the timed region."""
    n = gib << 30
    a = torch.ones(n // 8, dtype=torch.int64, device=dev)
    b = torch.empty_like(a)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    b.copy_(a)
    a.sum()
    torch.cuda.synchronize(dev)
    ev[0].record()
    for _ in range(reps):
        b.copy_(a)
    ev[1].record()
    for _ in range(reps):
        a.sum()
    ev[2].record()
    torch.cuda.synchronize(dev)
    t_copy = ev[0].elapsed_time(ev[1]) / 1e3
    t_read = ev[1].elapsed_time(ev[2]) / 1e3
    del a, b
    return {"copy_GBps": round(2 * n * reps / t_copy / 1e9, 1),
            "read_GBps": round(n * reps / t_read / 1e9, 1),
            "method": f"torch copy_ (read + write) and sum (read) over {gib} GiB, HIP events"}


def rule_index_name(kind: int) -> str:
    return {0: "linear scan", 1: "tuple-space index", 2: "decision tree"}.get(kind, str(kind))


PMC_DIR = os.path.join("profiles", "r06")   # the committed PMC summaries of this round's build


def lib_sha16() -> str | None:
    """sha256 (first 16 hex digits) of the libupe_gpu.so this process loads."""
    import hashlib

    try:
        return hashlib.sha256(open(os.path.join(ROOT, "upe_amd", "libupe_gpu.so"),
                                   "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_record(label: str, packets: int, mode: str):
    """The committed PMC summary of this leg's classify kernel (profiles/r06/pmc_<label>_<mode>.json,
    made by tools/pmc_refresh.sh + tools/pmc_r06.py from separate FETCH_SIZE / WRITE_SIZE / SQ /
    GRBM passes), or None when there is none for this batch size."""
    rel = os.path.join(PMC_DIR, f"pmc_{label}_{mode}.json")
    path = os.path.join(ROOT, rel)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("packets") != packets:
        return None
    d["source"] = rel
    return d


def pmc_traffic(label: str, packets: int, mode: str):
    """HBM bytes per classify launch (2 x FETCH_SIZE + WRITE_SIZE) from pmc_record, or None."""
    d = pmc_record(label, packets, mode)
    return d.get("traffic_bytes_per_launch") if d else None


def traffic_note(label: str, packets: int, mode: str):
    """Where roofline.traffic came from: the summary file, its passes' UTC stamps, and whether
    its profiled library is the one this run loaded (same sha256)."""
    d = pmc_record(label, packets, mode)
    if not d or "traffic_bytes_per_launch" not in d:
        return None
    return {"file": d["source"], "lib_sha16": d.get("lib_sha16"),
            "same_build_as_this_run": d.get("lib_sha16") == lib_sha16(),
            "passes_utc": {g: (s.split("utc=")[-1] if s else None)
                           for g, s in d.get("passes", {}).items()},
            "read_bytes_per_packet": d.get("read_bytes_per_packet"),
            "write_bytes_per_packet": d.get("write_bytes_per_packet"),
            "wave_time": d.get("wave_time"),
            "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes, 2 x "
                      "FETCH_SIZE + WRITE_SIZE (gfx950), median full-batch dispatch"}


def cpu_quota():
    """This process's cgroup v2 CPU quota in CPUs (cpu.max), or None when unlimited/unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        return None


def cpu_baseline(wl, threads: int, local: list | None = None, numa_all: bool = True) -> dict:
    """The reference worker timed on this host: one shard and calloc'd worker_t per thread, each
    pinned to its own core — the GPU's NUMA-local cores first (`local`), then the rest of the
    affinity mask.  `threads` is this job's CPU share (16 per GPU on the GPU box; the machine's
    other cores belong to other jobs), reported with the spread of the passes.  numa_all: also
    every NUMA-local core of the GPU (the node's whole CPU side, busy with other jobs or not), on
    a 4M-packet sample of the same workload so that each thread's shard stays in the tens of
    thousands of packets."""
    import oracle

    sample = f"{wl.n} packets of the same workload, median of 9 passes after 1 warm-up"
    if oracle.ref_available():
        allowed = ALLOWED_CPUS
        order = [c for c in (local or []) if c in allowed] + \
            [c for c in allowed if c not in (local or [])]
        cpus = order[:threads]
        r1, rn = [], []
        v1 = oracle.time_reference(wl, threads=1, cpus=cpus[:1], reps=9, rates=r1)
        vn = (oracle.time_reference(wl, threads=len(cpus), cpus=cpus, reps=9, rates=rn)
              if len(cpus) > 1 else v1)
        rn = rn or r1
        try:
            model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                     if l.startswith("model name")][0]
        except Exception:
            model = "unknown"
        numa = None
        loc = [c for c in (local or []) if c in allowed]
        if numa_all and len(loc) > len(cpus):
            from upe_amd import synth

            big = synth.config_b(n=1 << 22, seed=2)
            ra = []
            va = oracle.time_reference(big, threads=len(loc), cpus=loc, reps=9, rates=ra)
            quota = cpu_quota()
            numa = {"value": round(va / 1e6, 3), "unit": "Mpps", "cores": len(loc),
                    "spread": {"min": round(ra[0] / 1e6, 3), "median": round(va / 1e6, 3),
                               "max": round(ra[-1] / 1e6, 3), "passes": len(ra)},
                    "sample": f"{big.n} packets of the same workload (config B, seed 2) split over "
                              "every CPU of the GPU's NUMA node in this process's affinity, one "
                              "pinned thread each; median of 9 passes after 1 warm-up; rate = "
                              "packets / the slowest thread's time",
                    "cpu_quota_cpus": quota,
                    "linear_projection": {"value": round(v1 * len(loc) / 1e6, 3), "unit": "Mpps",
                                          "what": "single-core rate x NUMA-local cores: the "
                                                  "node's CPU side if the path scaled perfectly "
                                                  "(an upper bound, not a measurement)"},
                    "note": ("this job's cgroup CPU quota (cpu_quota_cpus) is below the thread "
                             "count, so threads are throttled and the slowest one sets the rate: "
                             "the measured value is the quota, not the cores — see "
                             "linear_projection") if quota and quota < len(loc) else
                            "the node's other jobs share these cores: the spread says how much"}
        return {"value": round(vn / 1e6, 3), "unit": "Mpps", "cores": len(cpus),
                "numa_local_all": numa,
                "kind": "reference", "single_core_value": round(v1 / 1e6, 3),
                "spread": {"min": round(rn[0] / 1e6, 3), "median": round(vn / 1e6, 3),
                           "max": round(rn[-1] / 1e6, 3), "passes": len(rn),
                           "single_core_min_max": [round(r1[0] / 1e6, 3), round(r1[-1] / 1e6, 3)]},
                "cpus": cpus, "cpus_online": os.cpu_count(), "cpus_in_affinity": len(allowed),
                "cores_note": (f"{len(cpus)} threads = this job's CPU share on the GPU box (its "
                               "affinity mask spans the whole machine, whose other cores run other "
                               "jobs); the GPU's NUMA-local cores first; --cpu-threads N to change"),
                "cpu_model": model,
                "sample": sample + "; reference src/worker.c process_packet + TX-flush loop "
                          "(bursts of 32), one shard and calloc'd worker_t per pinned thread"}
    # no reference build on this host: time the restatement, single core
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        oracle.run_restated(wl)
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(wl.n / dt / 1e6, 3), "unit": "Mpps", "cores": 1, "kind": "port",
            "sample": sample}


def dropin_pipeline(local: list | None, seconds: float = 2.0, device: int = 0) -> dict | None:
    """Part of the cpu_baseline leg (it runs the reference's own pipeline code, oracle/_ref): the
    reference's throughput benchmark (tests/benchmark_throughput.c:87-116,188-238,303-375: a
    synthetic-NIC producer thread building 64 B TCP packets in the reference pktbuf pool and
    pushing bursts of 32 round robin into the reference SPSC rings, workers popping them, TX
    stubbed; consumer Mpps = packets the workers popped / the producer's time) with the
    reference's own worker threads (src/worker.c worker_main) and with GPU workers — the product
    loop upe_gpu_worker_run bound to the same worker_t (oracle/dropin_worker.c) — on this GPU.
    Threads pinned to the GPU's NUMA-local CPUs (producer first).  Not `value`."""
    import ctypes

    import oracle

    so = os.path.join(os.path.dirname(oracle.__file__), "_ref", "libupe_dropin.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    P, SZ, I, D = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
    lib.upe_dropin_bench.restype = I
    lib.upe_dropin_bench.argtypes = [I, I, I, I, SZ, SZ, I, I, D, D, SZ, P, P]
    cpus_all = [c for c in (local or []) if c in ALLOWED_CPUS] or ALLOWED_CPUS
    legs = []
    for pool, ring in ((8192, 1024), (262144, 32768)):
        for gpu, mapped, workers in ((0, 0, 1), (0, 0, 4), (1, 1, 1), (1, 1, 2), (1, 0, 1)):
            cpus = (ctypes.c_int * (1 + workers))(*[cpus_all[k % len(cpus_all)]
                                                    for k in range(1 + workers)])
            out = (ctypes.c_double * 5)()
            rc = lib.upe_dropin_bench(gpu, mapped, workers, device, pool, ring, 32, 64, 0.5,
                                      seconds, 65536, cpus, out)
            legs.append({"workers": (f"{workers} GPU worker(s), " +
                                     ("pktbufs classified in the registered pool (mapped)"
                                      if mapped else "header windows staged in pinned memory, "
                                      "read there by the kernel"))
                         if gpu else f"{workers} reference worker thread(s) (src/worker.c)",
                         "pool": pool, "ring": ring, "rc": rc,
                         "gpu_batch": (max(256, min(65536, pool // (4 * workers))) if gpu
                                       else None),
                         "consumer_mpps": round(out[0], 2), "producer_mpps": round(out[1], 2),
                         "ring_full_events": int(out[2]), "seconds": round(out[3], 3)})
    return {"legs": legs, "packet": "64 B Eth/IPv4/TCP 10.128.0.1:45000 -> 10.128.0.2:80, "
                                     "1 TCP FWD rule, 1 ARP entry (the reference bench's setup)",
            "what": "the reference's e2e throughput benchmark (one producer thread -> SPSC rings "
                    "-> workers -> stubbed TX), consumer Mpps = worker pkts_in / producer time; "
                    "pool / ring = the reference defaults (8192 / 1024) and a GPU-sized pair; "
                    f"{seconds} s after 0.5 s warm-up per leg; the single producer thread bounds "
                    "every leg (producer_mpps)"}


def host_roundtrip(worker, wl, reps: int, chunk: int, windows: bool, apply_threads=None) -> dict:
    """Host-inclusive rate: the batch starts and ends in pinned host memory (libpcap in, AF_PACKET
    out).  In place (apply_threads None): upe_gpu_process_host pipelines H2D of frames +
    descriptors, classify and D2H of verdicts + the rewritten header span over chunks.  Emit:
    upe_gpu_process_host_emit brings back verdicts + 16-byte records and applies them to the
    frames on the host with 1 + apply_threads threads (the same output bytes).  windows: ship
    96-byte header windows, not frames."""
    from upe_amd import gpu, synth
    from upe_amd.layout import FRAME_TAIL, REWRITE_EXTENT, desc_lens, desc_offsets

    src = synth.header_windows(wl) if windows else wl
    emit = apply_threads is not None
    pf = gpu.PinnedArray(src.frames.shape, np.uint8)
    pd = gpu.PinnedArray(src.desc.shape, np.uint64)
    pv = gpu.PinnedArray((wl.n,), np.uint32)
    ph = gpu.PinnedArray((wl.n, 16), np.uint8) if emit else None
    pd.array[:] = src.desc
    times = []
    for r in range(reps + 2):
        pf.array[:] = src.frames          # untimed: a fresh batch every pass
        t0 = time.perf_counter()
        if emit:
            worker.process_host_emit(pf.array, pd.array, pv.array, ph.array, chunk, apply_threads)
        else:
            worker.process_host(pf.array, pd.array, pv.array, chunk)
        t1 = time.perf_counter()
        if r >= 2:
            times.append(t1 - t0)
    for x in (pf, pd, pv, ph):
        if x is not None:
            x.free()
    t = float(np.median(times))
    # bytes the copies actually move: per chunk the frame span in, and back the span up to the
    # last rewritable byte (UPE_REWRITE_EXTENT) plus the verdicts
    lens = desc_lens(src.desc)
    offs = desc_offsets(src.desc)
    ck = chunk or ((1 << 17) if emit else (1 << 18))   # the library's defaults
    h2d = d2h = 0
    for s in range(0, wl.n, ck):
        o, ln = offs[s:s + ck], lens[s:s + ck]
        h2d += int(o.max() + FRAME_TAIL - o.min()) + 8 * len(o)
        d2h += (20 * len(o) if emit else
                int((o + np.minimum(ln, REWRITE_EXTENT)).max() - o.min()) + 4 * len(o))
    return {"seconds": t, "packets": wl.n, "h2d_bytes": h2d, "d2h_bytes": d2h,
            "windows": windows, "chunk": ck, "reps": reps,
            "times": times, "emit": emit, "apply_threads": apply_threads}


def host_mapped(worker, wl, reps: int, emit: bool) -> dict:
    """Host-inclusive rate without DMA copies: the batch lies in pinned host memory and the
    classify kernel reads its descriptors and header windows, and writes the verdicts and the
    rewritten header bytes (in place) or the records (emit), over the link itself
    (upe_gpu_process_mapped[_emit]).  Full frames stay in host memory (no header-window
    extraction); only the bytes the path touches cross the link."""
    from upe_amd import gpu

    pf = gpu.PinnedArray(wl.frames.shape, np.uint8)
    pd = gpu.PinnedArray(wl.desc.shape, np.uint64)
    pv = gpu.PinnedArray((wl.n,), np.uint32)
    ph = gpu.PinnedArray((wl.n, 16), np.uint8) if emit else None
    pd.array[:] = wl.desc
    times = []
    for r in range(reps + 2):
        pf.array[:] = wl.frames           # untimed: a fresh batch every pass
        t0 = time.perf_counter()
        if emit:
            worker.process_mapped_emit(pf.array, pd.array, pv.array, ph.array)
        else:
            worker.process_mapped(pf.array, pd.array, pv.array)
        worker.sync()
        t1 = time.perf_counter()
        if r >= 2:
            times.append(t1 - t0)
    for x in (pf, pd, pv, ph):
        if x is not None:
            x.free()
    return {"seconds": float(np.median(times)), "packets": wl.n, "times": times, "reps": reps,
            "emit": emit}


def imix_leg(torch, dev, dist, rank: int, local: int, steps: int, warmup: int, mode: str,
             copies_cap: int, kind: str = "C") -> dict:
    """An IMIX workload (config C: 64/570/1518 B, IPv4 + IPv6, 1k rules, ARP + NDP forwarding)
    timed the same way as `value`, on every rank at once after the main region, so that a
    multi-GPU run reports the 64 B and the IMIX rates at each N (BASELINE north_star).  Each rank
    takes its own shard (seed 3 + 1000 * rank); `copies_cap` distinct copies of the batch
    (32 x ~370 MB, past the Infinity Cache) are cycled.  Not `value`.  kind: "C" the flow-derived
    rules (first matches spread over the table: the `imix` leg from round 5), "C3" the seed-3 draw
    of rounds 1-4 (`imix_seed3`: IPv4 stops by rule 11, IPv6 at rule 0), "C6" the seed-3 draw
    with its family-wide wildcards last (`imix_v6fwd`: IPv6 forwarded through NDP)."""
    from upe_amd import gpu, shard, synth

    seed = 3 + 1000 * rank
    wl = (synth.config_c_flows(seed=seed) if kind == "C" else
          synth.config_c(seed=seed, v6_forwarding=kind == "C6"))
    n = wl.n
    worker = gpu.GpuWorker(local, wl.capacity)
    worker.configure(wl)
    sh = torch.cuda.current_stream(dev).cuda_stream
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    copies = max(2, min(steps + warmup, copies_cap))
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    del pristine
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()

    def run(k0: int, count: int, ptrs=None) -> None:
        ptrs = ptrs or [base + (k % copies) * stride for k in range(k0, k0 + count)]
        if mode == "emit":
            worker.process_batches_emit(ptrs, desc, verdict, hdr, n, sh)
        else:
            worker.process_batches(ptrs, desc, verdict, n, sh)

    timed = gpu.GpuWorker.frames_list([base + (k % copies) * stride
                                       for k in range(warmup, warmup + steps)])
    run(0, warmup)
    torch.cuda.synchronize(dev)
    worker.timing_span(event_every(steps), EVENT_SPAN)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(warmup, steps, timed)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, dev)
    total = float(shard.sum_over_ranks([n * steps], dist, dev)[0])
    v = verdict.cpu().numpy().view(np.uint32).copy()
    cms, gms, launches = worker.timing_read()
    cms += gms
    idx_kind = worker.rule_index_kind()
    worker.close()
    del pool, desc, verdict, hdr
    bpp = algorithmic_bytes(wl, v, emit=mode == "emit")
    # (no closed event sample: the wall time per step, an upper bound on the kernel's)
    kern_s = cms / launches / 1e3 if launches else elapsed / steps
    achieved = float(bpp.sum()) / kern_s / 1e9
    return {"workload": WORKLOADS[kind], "value": round(total / elapsed / 1e6, 2), "unit": "Mpps",
            "ms_per_step": round(elapsed / steps * 1e3, 5), "steps": steps,
            "packets_per_gpu_step": n,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "kernel_ms": round(kern_s * 1e3, 5),
                         "algorithmic_bytes_per_packet": round(float(bpp.sum()) / n, 2),
                         "traffic": pmc_traffic({"C": "CF"}.get(kind, kind), n, mode),
                         "traffic_source": traffic_note({"C": "CF"}.get(kind, kind), n, mode),
                         "rule_index": rule_index_name(idx_kind)},
            "format": "packed frames (upe_gpu_process_emit)",
            "what": f"all ranks at once after the main region, {copies} distinct batch copies "
                    "cycled, same timing protocol as value (barrier, max over ranks)"}


def strong_leg(torch, dev, dist, rank: int, world: int, local: int, kind: str, steps: int,
               warmup: int) -> dict:
    """Strong scaling: ONE batch — config B's 1M 64 B packets, or config
    C's 1M IMIX packets (flow-derived rules) — split into `world` contiguous static shards
    (shard.shard_workload: rank r takes [r n / world, (r + 1) n / world), tables replicated, its
    own calloc'd L1 state, no collective on the data path).  Every rank classifies its shard
    `steps` times (emit mode, 8 distinct copies cycled); value = the batch's packets x steps / the
    slowest rank's time.  The driver's runs at N = 1, 2, 4, 8 give the strong-scaling curve beside
    the weak-scaling `value` (each rank its own full batch)."""
    from upe_amd import gpu, shard, synth

    whole = synth.config_b() if kind == "B" else synth.config_c_flows()
    total_n = whole.n
    wl = shard.shard_workload(whole, rank, world)
    del whole
    n = wl.n
    worker = gpu.GpuWorker(local, wl.capacity)
    worker.configure(wl)
    sh = torch.cuda.current_stream(dev).cuda_stream
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    copies = 8
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    del pristine
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    hdr = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    ptrs = [base + (k % copies) * stride for k in range(warmup + steps)]
    worker.process_batches_emit(ptrs[:warmup], desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    timed = gpu.GpuWorker.frames_list(ptrs[warmup:])
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    worker.process_batches_emit(timed, desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, dev)
    worker.close()
    del pool, desc, verdict, hdr
    return {"workload": WORKLOADS[kind] + f", one batch split over {world} GPU(s)",
            "value": round(total_n * steps / elapsed / 1e6, 2), "unit": "Mpps",
            "ms_per_step": round(elapsed / steps * 1e3, 5), "steps": steps,
            "packets_per_step": total_n, "packets_this_rank": n, "scaling": "strong",
            "what": "all ranks at once after the main region, barrier + max over ranks"}


VALU_PEAK_G = 1024 * 2.4 / 2   # G wave64 VALU instructions/s: 1024 SIMD-32s, one per 2 cycles


def pmc_valu(label: str, packets: int, mode: str = "emit"):
    """The classify kernel's VALU counts per launch from the committed PMC summary
    (pmc_record: SQ and GRBM passes), or None."""
    d = pmc_record(label, packets, mode)
    if not d or "valu_frac" not in d:
        return None
    return {"sq_insts_valu": d["sq"]["SQ_INSTS_VALU"], "valu_frac": d["valu_frac"],
            "valu_insts_per_packet": d["valu_insts_per_64_packets"], "source": d["source"]}


def config_d_leg(torch, dev, local: int, steps: int, warmup: int, copies_cap: int = 8) -> dict:
    """BASELINE configs[3] (16M packets: IPv4 options, TCP data offsets, 10 % malformed, v4 / v6
    mixed per wave; 64k rules, the tuple-space index) timed after the main region with the same
    protocol (emit mode, distinct batch copies cycled, wall time over `steps` launches; HIP
    events around every launch split classify and the rule_stats group-by).  Two rooflines for
    the classify kernel, both from committed PMC passes over the live classify time: the VALU
    issue rate (SURVEY.md §8(d) expected the rule work to bound it; SQ_INSTS_VALU per launch,
    tools/pmc_valu.py, against 1024 SIMDs x 1 wave-instruction per 2 cycles at 2.4 GHz) and the
    bytes requested past L2 (2 x FETCH_SIZE + WRITE_SIZE, tools/pmc_traffic.py) against HBM;
    the top-level roofline is the algorithmic-bytes fraction (bytes the path must move / step
    time) with the counted bytes as its traffic (round 4 measured the counted bytes at ~0.8 of
    8 TB/s, VALU ~0.33).  Not `value`."""
    from upe_amd import gpu, synth

    t_gen = time.perf_counter()
    wl = synth.config_d()
    t_gen = time.perf_counter() - t_gen
    n = wl.n
    worker = gpu.GpuWorker(local, wl.capacity)
    worker.configure(wl)
    sh = torch.cuda.current_stream(dev).cuda_stream
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    copies = max(2, min(steps + warmup, copies_cap))
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    del pristine
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    ptrs = [base + (k % copies) * stride for k in range(warmup + steps)]
    worker.process_batches_emit(ptrs[:warmup], desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    timed = gpu.GpuWorker.frames_list(ptrs[warmup:])
    worker.timing_span(1, 1)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    worker.process_batches_emit(timed, desc, verdict, hdr, n, sh)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    v = verdict.cpu().numpy().view(np.uint32).copy()
    cms, gms, launches = worker.timing_read()
    kind = worker.rule_index_kind()
    worker.close()
    del pool, desc, verdict, hdr
    classify_s = cms / launches / 1e3
    step_s = (cms + gms) / launches / 1e3
    bpp = algorithmic_bytes(wl, v, emit=True)
    traffic = pmc_traffic("D", n, "emit")
    pv = pmc_valu("D", n, "emit")
    roof = {"kernel": "upe_classify (tuple-space variant)", "classify_ms": round(classify_s * 1e3, 4),
            "group_by_ms": round(gms / launches, 4), "event_samples": int(launches)}
    valu = {"unit": "G VALU wave-instructions/s", "peak": round(VALU_PEAK_G, 1)}
    if pv:
        ach = pv["sq_insts_valu"] / classify_s / 1e9
        valu.update({"achieved": round(ach, 1), "frac": round(ach / VALU_PEAK_G, 4),
                     "valu_insts_per_launch": pv["sq_insts_valu"],
                     "frac_pmc_cycles": round(pv["valu_frac"], 4),
                     "valu_wave_insts_per_64_packets": round(pv["valu_insts_per_packet"], 1),
                     "source": pv["source"] + " (rocprofv3 SQ_INSTS_VALU per classify launch) / "
                               "this run's classify time (HIP events); frac_pmc_cycles: over the "
                               "PMC run's own GRBM_GUI_ACTIVE cycles"})
    else:
        valu.update({"achieved": None, "frac": None,
                     "source": "no committed VALU PMC summary for this batch size"})
    hbm_alg = float(bpp.sum()) / step_s / 1e9
    hbm = {"unit": "GB/s", "peak": HBM_PEAK_GBPS, "traffic": traffic,
           "algorithmic": {"achieved": round(hbm_alg, 1), "frac": round(hbm_alg / HBM_PEAK_GBPS, 4),
                           "bytes_per_packet": round(float(bpp.sum()) / n, 2),
                           "basis": "algorithmic bytes per step / step kernel time (classify + group-by)"}}
    if traffic:
        t_ach = traffic / classify_s / 1e9
        hbm.update({"achieved": round(t_ach, 1), "frac": round(t_ach / HBM_PEAK_GBPS, 4),
                    "source": "bytes requested past L2 per classify launch (PMC, "
                              f"{PMC_DIR}/pmc_D_emit.json: 2 x FETCH_SIZE + WRITE_SIZE; "
                              "Infinity-Cache hits included, so an upper bound on HBM bytes) / "
                              "this run's classify time"})
    else:
        hbm.update({"achieved": None, "frac": None})
    roof["valu"] = valu
    roof["hbm"] = hbm
    # the headline fraction is the algorithmic one (the bytes the path must move, per step time),
    # with the counted past-L2 bytes as its traffic, as for the other legs; the VALU issue rate
    # and the counted-bytes rate stay beside it (valu / hbm)
    roof.update({"bound": "hbm", "achieved": hbm["algorithmic"]["achieved"], "peak": HBM_PEAK_GBPS,
                 "unit": "GB/s", "frac": hbm["algorithmic"]["frac"], "traffic": traffic,
                 "traffic_source": traffic_note("D", n, "emit"),
                 "algorithmic_bytes_per_packet": hbm["algorithmic"]["bytes_per_packet"],
                 "traffic_bytes_per_packet": round(traffic / n, 2) if traffic else None})
    return {"workload": WORKLOADS["D"] + f", {n} packets per step", "value": round(n * steps / elapsed / 1e6, 2),
            "unit": "Mpps", "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps,
            "rule_index": "tuple space" if kind == 1 else "linear scan",
            "roofline": roof,
            "rule_scan_equiv": {"evals_per_batch": rule_evals(wl, v),
                                "T_evals_per_s": round(rule_evals(wl, v) * steps / elapsed / 1e12, 1),
                                "what": "rule tests the reference's linear scan would make "
                                        "(src/rule_table.c:163-176) / wall time: an equivalence, "
                                        "not the work the tuple-space probes do"},
            "generation_s": round(t_gen, 1),
            "what": f"rank 0 at N=1, after the main region; {copies} distinct 2 GB batch copies "
                    "cycled; emit mode"}


def egress_leg(torch, dev, wl, worker, pool, stride: int, copies: int, desc, launches: int = 20) -> dict:
    """The egress list (not `value`): the same batches as `value` classified by
    upe_gpu_process_emit (no list), by upe_gpu_process_emit_tx (the list of forwarded packets by
    64-packet group written in the same pass) and by upe_gpu_process_emit followed by
    upe_gpu_compact (the flat list from the verdicts: two more kernels).  HIP events on the launch
    stream around each mode's `launches` launches; per-launch time.  The list of the last launch
    is checked against the verdicts (the flat list equals the groups concatenated)."""
    from upe_amd.layout import V_FWD

    n = wl.n
    # a stream of our own, so that the events below bracket exactly these launches (torch's
    # current stream is the null stream, which the library maps to the context's own stream)
    strm = torch.cuda.Stream(dev)
    sh = strm.cuda_stream
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    tx = torch.empty(n, dtype=torch.int32, device=dev)
    txc = torch.empty((n + 63) // 64, dtype=torch.int32, device=dev)
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    base = pool.data_ptr()

    def run(mode: str, k: int) -> None:
        f = base + (k % copies) * stride
        if mode == "emit_tx":
            worker.process_emit_tx(f, desc, verdict, hdr, tx, txc, n, sh)
        else:
            worker.process_emit(f, desc, verdict, hdr, n, sh)
            if mode == "emit+compact":
                worker.compact(verdict, n, V_FWD, idx, cnt, sh)

    out = {}
    torch.cuda.synchronize(dev)
    for mode in ("emit", "emit_tx", "emit+compact", "emit"):
        for k in range(3):
            run(mode, k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(strm)
        for k in range(launches):
            run(mode, 3 + k)
        e1.record(strm)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1e3 / launches
        out[mode] = round(min(us, out.get(mode, us)), 3)
    v = verdict.cpu().numpy().view(np.uint32)
    fwd = np.nonzero((v & 0xF) == V_FWD)[0]
    t, c = tx.cpu().numpy().view(np.uint32), txc.cpu().numpy().view(np.uint32)
    groups = np.concatenate([t[64 * g:64 * g + int(c[g])] for g in range(len(c))])
    flat = idx.cpu().numpy().view(np.uint32)[: int(cnt.item())]
    ok = bool(np.array_equal(groups, fwd) and np.array_equal(flat, fwd))
    del verdict, hdr, tx, txc, idx, cnt
    return {"us_per_launch": out, "lists_equal_verdicts": ok, "launches": launches,
            "what": "per launch over the value leg's batches (HIP events on the launch stream, the "
                    "lower of two passes for emit): emit alone, emit with the egress list by "
                    "64-packet group in the same pass (upe_gpu_process_emit_tx), emit + the flat "
                    "list by upe_gpu_compact (two more kernels over the verdicts)"}


def ring_leg(torch, dev, dist, wl, worker, count: int, launches: int) -> dict:
    """Ring mode (upe_gpu_process_ring_emit, not `value`): `count` batches of this workload, each
    its own copy of the frames, laid out back to back and classified by ONE launch; the launch's
    fixed cost is paid once per ring.  Reports the per-batch rate and each batch's completion
    time within the launch (the device stamps of the last ring)."""
    from upe_amd import shard

    n = wl.n
    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    pristine = torch.from_numpy(wl.frames).to(dev)
    frames = torch.empty(count * stride, dtype=torch.uint8, device=dev)
    for k in range(count):
        frames[k * stride: k * stride + fbytes].copy_(pristine)
    del pristine
    d0 = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    desc = torch.cat([d0 + ((k * stride) << 16) for k in range(count)])
    verdict = torch.empty(n * count, dtype=torch.int32, device=dev)
    hdr = torch.empty(n * count * 16, dtype=torch.uint8, device=dev)
    done = torch.zeros(count, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream

    def run(k: int) -> None:
        for _ in range(k):
            worker.process_ring_emit(frames, desc, verdict, hdr, n, count, done, sh)

    run(2)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run(launches)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist, dev)
    total = float(shard.sum_over_ranks([n * count * launches], dist, dev)[0])
    # (wall time: the launches go to the worker's own stream when torch's is the null stream)
    ring_us = elapsed * 1e6 / launches
    stamps = (done.cpu().numpy() / 1e3).round(2).tolist()   # us after the launch's start
    del frames, desc, verdict, hdr, done
    return {"value": round(total / elapsed / 1e6, 2), "unit": "Mpps", "batches_per_launch": count,
            "packets_per_batch": n, "launches": launches,
            "us_per_launch": round(ring_us, 2), "us_per_batch": round(ring_us / count, 3),
            "batch_done_us": stamps,
            "what": "upe_gpu_process_ring_emit: the batches of a ring (each its own frames copy) "
                    "in ONE launch, emit mode; batch_done_us = each batch's completion (its last "
                    "stores issued) after the launch's first workgroup started, device clock; "
                    "not value (value = one launch per batch)"}


def line_summary(out: dict) -> dict:
    """The line's headline figures in one small object, printed last (a reader that keeps only the
    tail of a long line still sees them): per leg Mpps, kernel time, roofline fraction and
    counted bytes per packet; the CPU baseline; the host-inclusive rates."""
    def leg(d):
        if not d:
            return None
        r = d.get("roofline", {})
        k = r.get("kernel_ms", r.get("classify_ms"))
        t = r.get("traffic")
        n = d.get("packets_per_gpu_step") or (out["config"]["packets_per_gpu_step"]
                                               if d is out else None)
        return {"mpps": d.get("value"), "kernel_us": round(k * 1e3, 2) if k else None,
                "frac": r.get("frac"),
                "counted_B_per_packet": round(t / n, 1) if t and n else r.get("traffic_bytes_per_packet"),
                "algorithmic_B_per_packet": r.get("algorithmic_bytes_per_packet")}
    cb = out.get("cpu_baseline") or {}
    return {"B": leg(out), "imix_CF": leg(out.get("imix")), "C3": leg(out.get("imix_seed3")),
            "C6": leg(out.get("imix_v6fwd")), "D": leg(out.get("config_d")),
            "ring_us_per_batch": (out.get("ring") or {}).get("us_per_batch"),
            "egress_us_per_launch": (out.get("egress") or {}).get("us_per_launch"),
            "host_mapped_emit_mpps": (out.get("host_mapped_emit") or {}).get("value"),
            "host_roundtrip_mpps": (out.get("host_roundtrip") or {}).get("value"),
            "cpu_baseline_mpps": cb.get("value"), "cpu_cores": cb.get("cores"),
            "n_gpus": out.get("n_gpus"), "lib_sha16": out.get("lib_sha16")}


def finite(x):
    """The line as strict JSON: a NaN or infinity (a leg that could not be timed) becomes null."""
    if isinstance(x, float):
        return x if x == x and abs(x) != float("inf") else None
    if isinstance(x, dict):
        return {k: finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite(v) for v in x]
    return x


class stdout_to_stderr:
    """File descriptor 1 points at stderr inside the block (C++ libraries write there too)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def event_every(steps: int) -> int:
    """Timing samples (EVENT_SPAN launches each) every this many steps: EVENT_EVERY, or fewer
    for a short run so that at least one sample closes inside it."""
    return EVENT_EVERY if steps >= 2 * EVENT_EVERY else max(1, steps // 2)


def launch_cmd(gpus: int, argv: list, port: int) -> list:
    """The command the parent runs for --gpus N > 1 without a launcher around it: N ranks on
    this node under torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1), each
    running this file with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def world_check(gpus, env) -> int:
    """The world size this process runs in: WORLD_SIZE when a launcher set it (and then --gpus,
    if given, must agree), else 1.  Raises SystemExit on a mismatch."""
    ws = env.get("WORLD_SIZE")
    world = int(ws) if ws is not None else 1
    if gpus is not None and ws is not None and gpus != world:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}")
    return world


def launch_ranks(gpus: int, argv: list) -> int:
    """`python bench.py --gpus N` (N > 1, no WORLD_SIZE): start the N ranks as a child process
    and return its exit code.  This process never imports torch or touches a GPU; rank 0's JSON
    line reaches stdout directly (the children inherit it)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return subprocess.run(launch_cmd(gpus, argv, port), cwd=ROOT).returncode


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; N > 1 without a launcher starts N ranks "
                         "under torch.distributed.run itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="B", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=None, help="override batch size")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU baseline threads: this job's CPU share on the GPU box (16 per GPU; "
                         "the other cores of the machine run other jobs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dropin-seconds", type=float, default=2.0,
                    help="per leg of the reference pipeline benchmark with reference and GPU "
                         "workers (part of the cpu_baseline leg; 0 skips it)")
    ap.add_argument("--max-copies", type=int, default=1024)
    ap.add_argument("--host-reps", type=int, default=5,
                    help="passes of the host round-trip leg (pinned host batch -> H2D -> "
                         "classify -> D2H), after every timed leg; 0 skips it.  Its launches "
                         "are a separate leg of a rocprof trace (tools/kernel_legs.py)")
    ap.add_argument("--host-chunk", type=int, default=0)
    ap.add_argument("--host-apply-threads", type=int, default=7,
                    help="pool threads (besides the calling one) applying the records of the "
                         "emit-mode host round trip; -1: records returned, not applied")
    ap.add_argument("--no-host-emit", action="store_true",
                    help="skip the emit-mode host round trip")
    ap.add_argument("--no-host-mapped", action="store_true",
                    help="skip the mapped host legs (the kernel reading and writing pinned host "
                         "memory itself, upe_gpu_process_mapped[_emit])")
    ap.add_argument("--workers-per-gpu", type=int, default=0,
                    help="also time W worker contexts sharing this GPU, each on its own stream "
                         "with its own batches and L1 state, as W reference worker threads would "
                         "(reported beside value, never as value)")
    ap.add_argument("--no-hbm-probe", action="store_true",
                    help="skip the achievable-bandwidth probe (copy / read kernels)")
    ap.add_argument("--mode", default="emit", choices=["emit", "inplace"],
                    help="emit: rewritten-header records, frames read only (upe_gpu_process_emit);"
                         " inplace: frames rewritten in place (upe_gpu_process)")
    ap.add_argument("--no-other-mode", action="store_true",
                    help="skip timing the other output mode after the timed region")
    ap.add_argument("--no-imix", action="store_true",
                    help="skip the IMIX leg (config C timed after the main region on every rank, "
                         "reported as \"imix\" beside value; config B runs only)")
    ap.add_argument("--imix-v6fwd", type=int, default=1,
                    help="1: also time the seed-3 config C draw of rounds 1-4 (\"imix_seed3\") "
                         "and the same with its family-wide wildcards last (IPv6 forwarded "
                         "through NDP, \"imix_v6fwd\")")
    ap.add_argument("--strong", type=int, default=1,
                    help="1: also time strong scaling (SURVEY.md §8(d) row E): one config B batch "
                         "and one config C batch split into WORLD contiguous shards, reported as "
                         "\"strong\" beside the weak-scaling value")
    ap.add_argument("--imix-copies", type=int, default=32)
    ap.add_argument("--config-d-steps", type=int, default=20,
                    help="timed steps of the config D leg (16M packets, 64k rules; N=1 config B "
                         "runs; 0 skips it)")
    ap.add_argument("--ring", type=int, default=16,
                    help="batches per launch of the ring leg (config B; 0 skips it)")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = world_check(args.gpus, os.environ)

    import torch

    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; more ranks than GPUs (a rehearsal on a smaller box) share them round robin
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        # RCCL ("nccl") carries only the barrier and the max / sum over ranks; the gloo backend
        # (UPE_BENCH_DIST_BACKEND=gloo) rehearses the multi-rank path on a one-GPU box
        backend = os.environ.get("UPE_BENCH_DIST_BACKEND", "nccl")
        import datetime

        # (gloo prints its connection lines on stdout, which carries only the JSON line: they go
        # to stderr while the groups are made)
        with stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
            # a host-side group for the wait while rank 0 times the CPU baseline (no GPU spin)
            host_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30))
    else:
        torch.cuda.set_device(local)

    from upe_amd import gpu, shard, synth

    # this rank's host thread on a core of its GPU's NUMA node (its pinned buffers then come from
    # that node), as the reference pins each worker thread (src/affinity.c:48, src/main.c:143-175)
    local_cpus, numa_node = [], -1
    pinned_cpu = None
    try:
        local_cpus, numa_node = gpu.local_cpus(local)
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        pinned_cpu = gpu.pin_self(local, local_rank)
    except (gpu.UpeGpuError, AttributeError) as e:   # AttributeError: an older diagnostic build
        print(f"bench: no NUMA pinning ({e})", file=sys.stderr)

    # this rank's static shard: a full batch of the configuration, its own seed
    make = {"A": synth.config_a, "B": synth.config_b, "C": synth.config_c_flows,
            "C3": synth.config_c, "C6": lambda **k: synth.config_c(v6_forwarding=True, **k),
            "D": synth.config_d}[args.config]
    kw = {"seed": {"A": 1, "B": 2, "C": 3, "C3": 3, "C6": 3, "D": 4}[args.config] + 1000 * rank}
    if args.packets:
        kw["n"] = args.packets
    wl = make(**kw)
    n = wl.n

    worker = gpu.GpuWorker(local, wl.capacity)
    worker.configure(wl)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    fbytes = int(wl.frames.nbytes)
    stride = (fbytes + 255) // 256 * 256
    # distinct copies of the batch, so no step finds its frames in a cache a previous step
    # warmed (bounded to 64 GiB of HBM: config D's 2 GiB batch gets 32)
    copies = max(2, min(args.steps + args.warmup, args.max_copies, (64 << 30) // stride))
    pristine = torch.from_numpy(wl.frames).to(dev)
    pool = torch.empty(copies * stride, dtype=torch.uint8, device=dev)
    for c in range(copies):
        pool[c * stride: c * stride + fbytes].copy_(pristine)
    desc = torch.from_numpy(wl.desc.view(np.int64)).to(dev)
    verdict = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    torch.cuda.synchronize(dev)

    def steps(k0: int, count: int, mode: str = args.mode) -> None:
        # queued from native code (upe_gpu_process_batches[_emit]): no Python round trip per batch
        ptrs = prepared.get((k0, count)) or [base + (k % copies) * stride
                                             for k in range(k0, k0 + count)]
        if mode == "emit":
            worker.process_batches_emit(ptrs, desc, verdict, hdr, n, sh)
        else:
            worker.process_batches(ptrs, desc, verdict, n, sh)

    # the timed region's batch-pointer array, built before it starts (host bookkeeping only)
    prepared = {}
    prepared[(args.warmup, args.steps)] = gpu.GpuWorker.frames_list(
        [base + (k % copies) * stride for k in range(args.warmup, args.warmup + args.steps)])
    steps(0, args.warmup)
    torch.cuda.synchronize(dev)

    # Kernel timing events ride along in the timed region: a sample opens on every
    # EVENT_EVERY-th step (from step EVENT_EVERY / 2: the first launch starts from an idle queue)
    # and its event pair brackets EVENT_SPAN consecutive launches.  Each
    # event is a queue packet of its own (a few us of latency), so an event pair around every
    # launch would both tax the throughput being measured and inflate the per-launch time; over
    # 5 launches the pair's latency is spread thin (the gaps between those launches remain in
    # the time).  UPE_BENCH_EVENTS=0: diagnostic run without them.
    events = os.environ.get("UPE_BENCH_EVENTS", "1") != "0"
    worker.timing_span(event_every(args.steps) if events else 0, EVENT_SPAN)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if os.environ.get("UPE_BENCH_TRACE"):
        # diagnostic: where the host time of the timed region goes
        steps(args.warmup, 1)
        ta = time.perf_counter()
        torch.cuda.synchronize(dev)
        tb = time.perf_counter()
        steps(args.warmup + 1, args.steps - 1)
        tc = time.perf_counter()
        torch.cuda.synchronize(dev)
        print(f"trace: first call {1e3 * (ta - t0):.3f} ms, its sync {1e3 * (tb - ta):.3f} ms, "
              f"rest queued {1e3 * (tc - tb):.3f} ms, rest sync {1e3 * (time.perf_counter() - tc):.3f}"
              " ms", file=sys.stderr)
    else:
        steps(args.warmup, args.steps)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    # the last batch's verdicts (every step has the same packets): the basis of the algorithmic
    # bytes.  Read after the timed region: a large D2H before it delayed the first timed launch.
    v_first = verdict.cpu().numpy().view(np.uint32).copy()
    classify_ms, finalize_ms, launches = worker.timing_read()
    worker.timing_enable(False)
    # the other output mode over the same number of steps (after the timed region; each step
    # again on its own batch copy), so the line shows both: emit <-> in-place rewrite
    other = None
    if not args.no_other_mode:
        om = "inplace" if args.mode == "emit" else "emit"
        steps(0, min(args.warmup, 5), om)
        worker.timing_span(event_every(args.steps) if events else 0, EVENT_SPAN)
        torch.cuda.synchronize(dev)
        ta = time.perf_counter()
        steps(args.warmup, args.steps, om)
        torch.cuda.synchronize(dev)
        tb = time.perf_counter()
        oc_ms, og_ms, ol = worker.timing_read()
        oc_ms += og_ms
        worker.timing_enable(False)
        other = {"mode": om, "value": round(n * args.steps / (tb - ta) / 1e6, 2), "unit": "Mpps",
                 "ms_per_step": round((tb - ta) / args.steps * 1e3, 5),
                 "kernel_ms": round(oc_ms / ol, 5) if ol else None,
                 "what": "this rank alone, same batches, timed after the main region"}
    shared = None
    if args.workers_per_gpu > 1:
        shared = shared_gpu_workers(torch, dev, wl, worker, pool, stride, copies, desc,
                                    args.workers_per_gpu, args.steps)
    imix = imix3 = imix6 = None
    if args.config == "B" and not args.no_imix and not args.packets:
        imix = imix_leg(torch, dev, dist, rank, local, args.steps, args.warmup, args.mode,
                        args.imix_copies)
        if args.imix_v6fwd:
            imix3 = imix_leg(torch, dev, dist, rank, local, args.steps, args.warmup, args.mode,
                             args.imix_copies, kind="C3")
            imix6 = imix_leg(torch, dev, dist, rank, local, args.steps, args.warmup, args.mode,
                             args.imix_copies, kind="C6")
    strong = None
    if args.config == "B" and args.strong and not args.packets:
        strong = {k: strong_leg(torch, dev, dist, rank, world, local, k, args.steps, args.warmup)
                  for k in ("B", "C")}
    egress = None
    if args.config == "B" and args.mode == "emit" and not args.packets and rank == 0:
        egress = egress_leg(torch, dev, wl, worker, pool, stride, copies, desc)
    ring = None
    if args.config == "B" and args.ring > 0 and not args.packets:
        ring = ring_leg(torch, dev, dist, wl, worker, args.ring, 12)
    probe = hbm_probe(torch, dev) if rank == 0 and not args.no_hbm_probe else None
    dleg = None
    if args.config == "B" and world == 1 and args.config_d_steps > 0 and not args.packets:
        dleg = config_d_leg(torch, dev, local, args.config_d_steps, 3)

    # host round trip (not `value`): every rank at once, as the GPUs of a node would run it
    worker.reset_stats()
    hr = hre = None
    if args.host_reps > 0:
        if dist:
            dist.barrier()
        hr = host_roundtrip(worker, wl, args.host_reps, args.host_chunk,
                            windows=args.config != "B")
        if not args.no_host_emit:
            worker.reset_stats()
            if dist:
                dist.barrier()
            hre = host_roundtrip(worker, wl, args.host_reps, args.host_chunk,
                                 windows=args.config != "B", apply_threads=args.host_apply_threads)

    hm = hme = None
    if args.host_reps > 0 and not args.no_host_mapped:
        for emit_leg in (False, True):
            worker.reset_stats()
            if dist:
                dist.barrier()
            r = host_mapped(worker, wl, args.host_reps, emit_leg)
            r["seconds"] = shard.max_over_ranks(r["seconds"], dist, dev)
            if emit_leg:
                hme = r
            else:
                hm = r

    # the job ends when the slowest shard does; value = every rank's packets / that time
    elapsed = shard.max_over_ranks(t1 - t0, dist, dev)
    total_packets = float(shard.sum_over_ranks([n * args.steps], dist, dev)[0])
    if hr:
        hr["seconds"] = shard.max_over_ranks(hr["seconds"], dist, dev)
    if hre:
        hre["seconds"] = shard.max_over_ranks(hre["seconds"], dist, dev)

    if rank == 0:
        bpp = algorithmic_bytes(wl, v_first, emit=args.mode == "emit")
        plabel = {"C": "CF"}.get(args.config, args.config)
        traffic = pmc_traffic(plabel, n, args.mode)
        bytes_per_launch = float(bpp.sum())
        # a step's kernels: the classify launch plus (tables over 4096 rules) the rule_stats
        # group-by; finalize_ms is the group-by's share (0 for smaller tables)
        # (no closed event sample, e.g. UPE_BENCH_EVENTS=0: the wall time per step, an upper
        # bound on the kernels')
        kern_s = ((classify_ms + finalize_ms) / launches / 1e3 if launches
                  else elapsed / args.steps)
        achieved = bytes_per_launch / kern_s / 1e9
        ms_step = elapsed / args.steps * 1e3
        out = {
            "metric": METRIC,
            "value": round(total_packets / elapsed / 1e6, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded upe_amd.synth, per-rank shard), resident in HBM",
            "lib_sha16": lib_sha16(),
            "host_thread": {"cpu": pinned_cpu, "numa_node": numa_node,
                            "gpu_local_cpus": len(local_cpus)},
            "config": {"workload": WORKLOADS[args.config], "packets_per_gpu_step": n,
                       "rules": int(len(wl.rules)), "parallelism": f"static shards x{world}, "
                       "tables replicated, no RCCL on the data path",
                       "output": ("emit: verdict + 16-B rewritten-header record per packet, "
                                  "frames read only (upe_gpu_process_emit)")
                       if args.mode == "emit" else
                       "inplace: verdict per packet, frames rewritten in place (upe_gpu_process)"},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_note(plabel, n, args.mode),
                "kernel": "upe_classify",
                "kernel_ms": round(kern_s * 1e3, 5),
                "classify_ms": round(classify_ms / max(launches, 1), 5),
                "group_by_ms": round(finalize_ms / max(launches, 1), 5),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "algorithmic_bytes_per_packet": round(bytes_per_launch / n, 2),
                "kernel_mpps": round(n / kern_s / 1e6, 1),
                "event_samples": int(launches),
                "achievable": probe,
                "frac_of_achievable_read": (round(achieved / probe["read_GBps"], 4)
                                            if probe else None),
            },
            "rule_scan_equiv": {
                "evals_per_batch": rule_evals(wl, v_first),
                "G_evals_per_s": round(rule_evals(wl, v_first) * args.steps * world / elapsed
                                       / 1e9, 2),
                "what": "rule tests the reference's linear first-match scan would make on these "
                        "batches (src/rule_table.c:163-176) / wall time",
            },
        }
        if other:
            out["other_mode"] = other
        if imix:
            out["imix"] = imix
        if imix3:
            out["imix_seed3"] = imix3
        if imix6:
            out["imix_v6fwd"] = imix6
        if strong:
            out["strong"] = strong
        if ring:
            out["ring"] = ring
        if egress:
            out["egress"] = egress
        if dleg:
            out["config_d"] = dleg
        if shared:
            out["workers_sharing_gpu"] = shared
        def host_line(h, what):
            return {"value": round(h["packets"] * world / h["seconds"] / 1e6, 2), "unit": "Mpps",
                    "ms_per_batch": round(h["seconds"] * 1e3, 3),
                    "ms_min_max": [round(min(h["times"]) * 1e3, 3), round(max(h["times"]) * 1e3, 3)],
                    "h2d_GBps": round(h["h2d_bytes"] / h["seconds"] / 1e9, 2),
                    "d2h_GBps": round(h["d2h_bytes"] / h["seconds"] / 1e9, 2),
                    "h2d_bytes_per_packet": round(h["h2d_bytes"] / h["packets"], 1),
                    "d2h_bytes_per_packet": round(h["d2h_bytes"] / h["packets"], 1),
                    "header_windows": h["windows"], "chunk": h["chunk"],
                    "what": what + f"; median of {h['reps']} passes, all ranks at once"}

        if hr:
            out["host_roundtrip"] = host_line(
                hr, "pinned host batch -> H2D -> classify -> D2H of verdicts + the rewritten "
                    "header span, frames rewritten in place (upe_gpu_process_host), "
                    "4-slot pipeline")
        if hre:
            out["host_roundtrip_emit"] = host_line(
                hre, "pinned host batch -> H2D -> classify (emit) -> D2H of verdicts + 16-B "
                     "records (upe_gpu_process_host_emit), " +
                     (f"applied to the frames on the host by {1 + hre['apply_threads']} threads: "
                      "the same output bytes as host_roundtrip" if hre["apply_threads"] >= 0 else
                      "not applied (frames untouched: a TX path sends each record as its own "
                      "iovec)"))
        for key, h, what in (
                ("host_mapped", hm, "frames rewritten in place in host memory"),
                ("host_mapped_emit", hme, "verdicts + 16-B records written to host memory, frames "
                                          "read only")):
            if h:
                # the link roofline: the same algorithmic bytes B(p), all of which cross the link
                # here (descriptor, header extent, verdict, written bytes), per second, against
                # PCIe Gen5 x16's ~64 GB/s per direction
                lb = float(algorithmic_bytes(wl, v_first, emit=h["emit"]).sum())
                link = lb / h["seconds"] / 1e9
                out[key] = {"value": round(h["packets"] * world / h["seconds"] / 1e6, 2),
                            "unit": "Mpps", "ms_per_batch": round(h["seconds"] * 1e3, 3),
                            "link": {"achieved": round(link, 2), "peak": LINK_PEAK_GBPS,
                                     "unit": "GB/s", "frac": round(link / LINK_PEAK_GBPS, 4),
                                     "algorithmic_bytes_per_packet": round(lb / h["packets"], 2)},
                            "ms_min_max": [round(min(h["times"]) * 1e3, 3),
                                           round(max(h["times"]) * 1e3, 3)],
                            "frame_bytes_in_host_memory": int(wl.frames.nbytes),
                            "what": "pinned host batch (full frames) classified where it lies: the "
                                    "kernel's own loads and stores over the link, no DMA copy "
                                    "(upe_gpu_process_mapped" + ("_emit" if h["emit"] else "") +
                                    "); " + what + f"; median of {h['reps']} passes, all ranks "
                                    "at once"}
        if not args.no_cpu_baseline:
            # rank 0, after every timed region; at N > 1 the other ranks wait at a host barrier.
            # Config A is the reference's one-worker pcap replay: time it on one core
            out["cpu_baseline"] = cpu_baseline(wl, 1 if args.config == "A" else args.cpu_threads,
                                               local_cpus, numa_all=world == 1)
            if world > 1:
                out["cpu_baseline"]["ranks_note"] = (
                    f"timed by rank 0 on its own host cores after the {world}-rank timed regions, "
                    "the other ranks idle at a host barrier; the same per-host sample as at N=1")
            if args.config == "B" and args.dropin_seconds > 0 and world == 1:
                dp = dropin_pipeline(local_cpus, args.dropin_seconds, local)
                if dp:
                    out["dropin_pipeline"] = dp
        out["summary"] = line_summary(out)   # last: what a truncated tail of the line still shows
        print(json.dumps(finite(out)), flush=True)
    if dist:
        dist.barrier(group=host_group)
    worker.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
