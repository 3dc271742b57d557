"""bench.py's last stdout line: the driver parses it from a bounded tail of
stdout (round 3's 21 KB line was cut mid-line and went unparsed), so it must
stay <= 4 KB and carry the contract keys for the headline and every leg."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "config", "roofline", "step_roofline", "cpu_baseline")
LEG_KEYS = ("value", "unit", "ms_per_step", "roofline", "step_roofline", "cpu_baseline")


def _recorded():
    path = os.path.join(ROOT, "profiles", "r3_bench_all_final.json")
    if not os.path.exists(path):
        path = os.path.join(ROOT, "profiles", "archive", "r3_bench_all_final.json")
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def _check(full):
    s = bench.compact_line(full)
    assert len(s.encode()) <= bench.LINE_MAX_BYTES, len(s)
    assert "\n" not in s
    d = json.loads(s)
    for k in REQUIRED:
        assert k in d, k
    assert d["value"] == full["value"] and d["ms_per_step"] == round(full["ms_per_step"], 4)
    assert d["config"]["workload"] == full["config"]["workload"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel"):
        assert k in d["roofline"], k
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
    for w, leg in (full.get("workloads") or {}).items():
        got = d["workloads"][w]
        if "error" in leg:
            assert "error" in got
            continue
        for k in LEG_KEYS:
            assert k in got, (w, k)
        if leg.get("roofline") is None:                 # a latency / DBInterface leg (getlinks)
            assert got["roofline"] is None
            continue
        assert got["roofline"]["kernel"] == leg["roofline"]["kernel"]
        assert got["roofline"]["frac"] == leg["roofline"]["frac"]
    return d


def test_bench_line_from_recorded_full_record():
    full = _recorded()
    assert len(json.dumps(full)) > 8000         # the record that went unparsed in round 3
    _check(full)


def test_bench_line_from_round4_detail_record():
    """A round-4 detail record (the full dict bench.py writes to --detail,
    getlinks leg, join variants, latency objects included) compacts to a
    line within the bound that carries the Q2 And-join summary."""
    with open(os.path.join(ROOT, "profiles", "r4_bench_detail_s23.json")) as f:
        full = json.load(f)
    d = _check(full)
    assert d["and_join_q2"]["kernel"].startswith("k_dj_write") and d["and_join_q2"]["frac"] > 0.5
    assert "getlinks" in d["workloads"] and d["workloads"]["getlinks"]["unit"] == "queries/s"


def test_bench_line_bounded_when_record_grows():
    full = _recorded()
    # a leg error, very long strings, extra summaries: still within the bound
    full["data"] = "x" * 3000
    full["cpu_baseline"]["sample"] = "y" * 5000
    full["workloads"]["flybase"]["latency"] = {f"F{i}": {"us": 12.5, "launches": 3, "readbacks": 1}
                                               for i in range(60)}
    full["workloads"]["broken"] = {"error": "RuntimeError: " + "z" * 1000}
    _check({k: v for k, v in full.items()})


def test_emit_writes_detail_and_ends_stdout_with_line(tmp_path, capsys):
    full = _recorded()
    path = tmp_path / "detail.json"
    bench.emit(full, str(path))
    out = capsys.readouterr().out.strip().splitlines()
    d = json.loads(out[-1])
    assert len(out[-1].encode()) <= bench.LINE_MAX_BYTES
    assert json.load(open(path))["workloads"]["hub"]["kernels"]       # full record kept in the file
    assert d["detail"]
