"""The committed measurement evidence agrees with itself (CPU only; reads profiles/r06).

The bench line's roofline must be reproducible by hand from the files beside it (VERDICT r05
"next" 1): `achieved` = algorithmic bytes per launch / the kernel time, `frac` = achieved / peak,
`traffic` = the committed PMC summary of the same leg (2 x FETCH_SIZE + WRITE_SIZE), and every
PMC summary the line cites was taken on the library the line ran.
"""
import json
import os

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
R06 = os.path.join(ROOT, "profiles", "r06")
LEGS = [("B", "emit"), ("B", "inplace"), ("CF", "emit"), ("C6", "emit"), ("C3", "emit"),
        ("D", "emit")]


def _line(name: str) -> dict:
    path = os.path.join(R06, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not committed")
    return json.loads(open(path).read().strip().splitlines()[-1])


def _pmc(label: str, mode: str) -> dict:
    return json.load(open(os.path.join(R06, f"pmc_{label}_{mode}.json")))


@pytest.mark.parametrize("label,mode", LEGS)
def test_pmc_summary_arithmetic(label, mode):
    d = _pmc(label, mode)
    assert d["read_bytes"] == pytest.approx(2 * d["fetch_size_kb"] * 1024, rel=1e-9)
    assert d["write_bytes"] == pytest.approx(d["write_size_kb"] * 1024, rel=1e-9)
    assert d["traffic_bytes_per_launch"] == pytest.approx(d["read_bytes"] + d["write_bytes"],
                                                          rel=1e-9)
    assert d["traffic_bytes_per_packet"] == pytest.approx(
        d["traffic_bytes_per_launch"] / d["packets"], abs=0.01)
    # every pass stamped with the library it profiled, and all of one build
    assert all(f"lib_sha16={d['lib_sha16']}" in s for s in d["passes"].values())


def test_line_roofline_reproducible():
    line = _line("bench_r06_20steps.json")
    r = line["roofline"]
    assert r["achieved"] == pytest.approx(
        r["algorithmic_bytes_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e9, rel=2e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4)
    assert r["peak"] == 8000.0 and r["unit"] == "GB/s" and r["bound"] == "hbm"
    # traffic: the committed summary of this leg, taken on the library this line loaded
    src = r["traffic_source"]
    d = json.load(open(os.path.join(ROOT, src["file"])))
    assert r["traffic"] == d["traffic_bytes_per_launch"]
    assert src["lib_sha16"] == d["lib_sha16"] == line["lib_sha16"]
    assert src["same_build_as_this_run"] is True
    # algorithmic bytes never exceed what the counters saw
    assert r["algorithmic_bytes_per_launch"] <= r["traffic"]


def test_line_summary_matches_legs():
    line = _line("bench_r06_20steps.json")
    s = line["summary"]
    assert s["B"]["mpps"] == line["value"]
    assert s["B"]["frac"] == line["roofline"]["frac"]
    assert s["lib_sha16"] == line["lib_sha16"]
    for key, label in (("imix_CF", "CF"), ("C6", "C6"), ("C3", "C3"), ("D", "D")):
        assert s[key]["counted_B_per_packet"] == pytest.approx(
            _pmc(label, "emit")["traffic_bytes_per_packet"], abs=0.05)   # (summary: 1 decimal)


def test_line_contract_fields():
    line = _line("bench_r06_20steps.json")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 20 and line["warmup"] == 5
    # value = whole-job packets per second over the timed steps
    n = line["config"].get("packets_per_step") or 1 << 20
    assert line["value"] == pytest.approx(n / (line["ms_per_step"] * 1e-3) / 1e6, rel=2e-3)
    assert line["cpu_baseline"]["kind"] in ("reference", "port")
    assert line["cpu_baseline"]["cores"] >= 1
