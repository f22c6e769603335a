"""bench.py's roofline bookkeeping (CPU): a committed PMC traffic profile counts only for the library build it was
taken on (profiles/traffic_*.json record the sha256 of the profiled libkarpenter_amd.so; scripts/pmc_workloads.py).
The line says whether the build matches (`traffic_build_match`) and flags a stale source in `traffic_source`."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path):
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.ROOT = str(tmp_path)  # profiles/ under a scratch root
    (tmp_path / "profiles").mkdir()
    b._LIB_SHA = "a" * 64  # the loaded library's hash, fixed for the test
    return b


def _write(tmp_path, tag, **kw):
    doc = {"tag": "r99", "kernel": "k_solve", "hbm_bytes_per_launch": 1.0e6}
    doc.update(kw)
    (tmp_path / "profiles" / ("traffic_%s.json" % tag)).write_text(json.dumps(doc))


def test_matching_build(tmp_path):
    b = _bench(tmp_path)
    _write(tmp_path, "c2", lib_sha256="a" * 64)
    r = b._roofline("k_solve", 10.0, 1.0e9, 2.0e9, "c2")
    assert r["traffic_build_match"] is True and r["traffic"] == 1.0e6
    assert "STALE" not in r["traffic_source"]
    assert abs(r["hbm_frac"] - 1.0e6 / 0.01 / 1e9 / b.HBM_PEAK_GBS) < 1e-12


def test_other_build_is_flagged_stale(tmp_path):
    b = _bench(tmp_path)
    _write(tmp_path, "c2", lib_sha256="b" * 64)
    r = b._roofline("k_solve", 10.0, 1.0e9, 2.0e9, "c2")
    assert r["traffic_build_match"] is False
    assert "STALE" in r["traffic_source"]


def test_unrecorded_build_and_missing_profile(tmp_path):
    b = _bench(tmp_path)
    _write(tmp_path, "c3")
    r = b._roofline("k_solve", 10.0, 1.0e9, None, "c3")
    assert r["traffic_build_match"] is None and "build unrecorded" in r["traffic_source"]
    r = b._roofline("k_solve", 10.0, 1.0e9, None, "c9")  # no committed profile
    assert r["traffic"] is None and r["traffic_build_match"] is None and r["hbm_frac"] is None
