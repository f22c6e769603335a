"""Pin the oracle against the reference's own known answers.

Fixtures in tests/golden/*.json were text-extracted from pkg/scheduling/requirement_test.go and
requirements_test.go by tests/golden/extract_requirement_vectors.py.
"""
import json
import os

import pytest

from oracle import bridge

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


REQ = load("requirement_vectors.json")
REQS = load("requirements_vectors.json")


def _norm(s):
    out = {"key": s["key"], "complement": s["complement"], "values": sorted(s["values"])}
    for k in ("gt", "lt"):
        if k in s:
            out[k] = s[k]
    return out


def test_requirement_intersection_table():
    ops = [{"op": "intersection", "a": REQ["operands"][v["a"]], "b": REQ["operands"][v["b"]]}
           for v in REQ["intersection"]]
    got = bridge.eval_ops(ops)
    assert len(got) == 196
    bad = [(v["a"], v["b"], g, v["expected"]) for v, g in zip(REQ["intersection"], got)
           if _norm(g) != _norm(v["expected"])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("kind", ["has", "operator", "len", "string", "intersection_string"])
def test_requirement_scalar_vectors(kind):
    vecs = REQ[kind]
    ops = []
    for v in vecs:
        op = {"op": kind, "a": REQ["operands"][v["a"]]}
        if kind == "has":
            op["value"] = v["value"]
        if kind == "intersection_string":
            op["b"] = REQ["operands"][v["b"]]
        ops.append(op)
    got = bridge.eval_ops(ops)
    bad = [(v, g) for v, g in zip(vecs, got) if g != v["expected"]]
    assert not bad, bad[:5]


def test_requirements_compatible_450():
    ops = [{"op": "compatible", "a": REQS["operands"][v["a"]], "b": REQS["operands"][v["b"]],
            "allowUndefinedWellKnown": v["loose"]} for v in REQS["compatible"]]
    got = bridge.eval_ops(ops)
    assert len(got) == 450
    bad = [(v, g) for v, g in zip(REQS["compatible"], got) if g["ok"] != v["expected"]]
    assert not bad, bad[:5]


def test_requirements_error_text():
    ops = [{"op": "compatible", "a": [], "b": [{"key": v["label"], "operator": "Exists"}],
            "allowUndefinedWellKnown": v["loose"]} for v in REQS["error_text"]]
    got = bridge.eval_ops(ops)
    bad = [(v["expected"], g["error"]) for v, g in zip(REQS["error_text"], got) if g["error"] != v["expected"]]
    assert not bad, bad


def test_requirements_string_order():
    v = REQS["string"][0]
    got = bridge.eval_ops([{"op": "reqs_string", "a": v["requirements"]}])
    assert got[0] == v["expected"]


@pytest.mark.parametrize("q,expected", [
    ("100m", "100m"), ("1.5", "1500m"), ("2000m", "2"), ("1.8G", "1800M"), ("2Gi", "2Gi"),
    ("1024Mi", "1Gi"), ("100M", "100M"), ("4.5", "4500m"), ("1m", "1m"), ("0", "0"), ("1e3", "1e3"),
    ("1000", "1k"), ("512Mi", "512Mi"), ("1500Mi", "1500Mi"), ("0.5Gi", "512Mi"), ("10Mi", "10Mi"),
])
def test_quantity_canonical_string(q, expected):
    # apimachinery Quantity.String() canonical forms (resource/quantity.go CanonicalizeBytes)
    assert bridge.eval_ops([{"op": "quantity", "value": q}])[0] == expected
