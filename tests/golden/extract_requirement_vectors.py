#!/usr/bin/env python3
"""Extract the reference's requirement-algebra known answers into JSON fixtures.

Reads the reference Go test files AS TEXT (no Go toolchain exists here) and writes data-only
fixtures next to this script:

  requirement_vectors.json   <- pkg/scheduling/requirement_test.go:31-44 (operands),
                                :83-295 Intersection, :296-373 Has, :374-391 Operator,
                                :392-409 Len, :428-447 String
  requirements_vectors.json  <- pkg/scheduling/requirements_test.go:35-50 (operands),
                                :52-537 Compatible (loose + strict), :539-575 error text,
                                :623-645 String ordering

Each operand is stored as its NodeSelectorRequirement literal (key/operator/values); expected
Intersection results are stored as the Requirement struct the Go test compares with reflect.DeepEqual
(key, complement, values, greaterThan, lessThan).  Run once in a container that has
/root/reference; the JSON is committed and the GPU box never needs the reference.
"""
import json
import os
import re
import sys

REF = os.environ.get("KARPENTER_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

OPS = {"Exists": "Exists", "DoesNotExist": "DoesNotExist", "In": "In", "NotIn": "NotIn", "Gt": "Gt", "Lt": "Lt"}
ZONE = "topology.kubernetes.io/zone"
KEYCONST = {"v1.LabelTopologyZone": ZONE, "v1.LabelFailureDomainBetaZone": "failure-domain.beta.kubernetes.io/zone"}


def parse_args(argstr):
    """Parse the argument list of NewRequirement(...)."""
    parts = [p.strip() for p in re.findall(r'"[^"]*"|[\w.]+', argstr)]
    key = parts[0]
    key = key.strip('"') if key.startswith('"') else KEYCONST[key]
    op = OPS[parts[1].replace("v1.NodeSelectorOp", "")]
    values = [p.strip('"') for p in parts[2:]]
    return {"key": key, "operator": op, "values": values}


def new_requirement_struct(r):
    """The Requirement value NewRequirement builds (requirement.go:41-79), for DeepEqual."""
    op = r["operator"]
    s = {"key": r["key"], "complement": op not in ("In", "DoesNotExist"), "values": []}
    if op in ("In", "NotIn"):
        s["values"] = sorted(set(r["values"]))
    if op == "Gt":
        s["gt"] = int(r["values"][0])
    if op == "Lt":
        s["lt"] = int(r["values"][0])
    return s


def extract_requirement(path):
    src = open(path).read()
    operands = {}
    for m in re.finditer(r"(\w+) := NewRequirement\(([^)]*)\)", src):
        if m.group(1) in operands:
            continue
        operands[m.group(1)] = parse_args(m.group(2))
    # keep only the 14 Describe-level operands (key "key")
    operands = {k: v for k, v in operands.items() if v["key"] == "key"}
    out = {"source": "pkg/scheduling/requirement_test.go", "operands": operands,
           "intersection": [], "has": [], "operator": [], "len": [], "string": [], "intersection_string": []}
    for line in src.splitlines():
        line = line.strip()
        m = re.match(r"Expect\((\w+)\.Intersection\((\w+)\)\)\.To\(Equal\((.*)\)\)$", line)
        if m:
            a, b, exp = m.groups()
            if exp in operands:
                expected = new_requirement_struct(operands[exp])
            else:
                lit = re.match(r"&Requirement\{(.*)\}", exp).group(1)
                expected = {"key": "key", "complement": "complement: true" in lit, "values": []}
                vm = re.search(r"values: sets\.New(?:\[string\])?\(([^)]*)\)", lit)
                if vm and vm.group(1).strip():
                    expected["values"] = sorted(v.strip().strip('"') for v in vm.group(1).split(","))
                gm = re.search(r"greaterThan: (\w+)\.greaterThan", lit)
                if gm:
                    expected["gt"] = new_requirement_struct(operands[gm.group(1)])["gt"]
                lm = re.search(r"lessThan: (\w+)\.lessThan", lit)
                if lm:
                    expected["lt"] = new_requirement_struct(operands[lm.group(1)])["lt"]
            out["intersection"].append({"a": a, "b": b, "expected": expected})
            continue
        m = re.match(r'Expect\((\w+)\.Has\("([^"]*)"\)\)\.To\(Be(True|False)\(\)\)$', line)
        if m:
            out["has"].append({"a": m.group(1), "value": m.group(2), "expected": m.group(3) == "True"})
            continue
        m = re.match(r"Expect\((\w+)\.Operator\(\)\)\.To\(Equal\(v1\.NodeSelectorOp(\w+)\)\)$", line)
        if m:
            out["operator"].append({"a": m.group(1), "expected": m.group(2)})
            continue
        m = re.match(r"Expect\((\w+)\.Len\(\)\)\.To\(Equal\((.*)\)\)$", line)
        if m:
            e = m.group(2).replace(" ", "")
            if e.startswith("math.MaxInt64"):
                val = 2**63 - 1 - (int(e.split("-")[1]) if "-" in e else 0)
            else:
                val = int(e)
            out["len"].append({"a": m.group(1), "expected": val})
            continue
        m = re.match(r'Expect\((\w+)\.String\(\)\)\.To\(Equal\("(.*)"\)\)$', line)
        if m:
            out["string"].append({"a": m.group(1), "expected": m.group(2)})
            continue
        m = re.match(r'Expect\((\w+)\.Intersection\((\w+)\)\.String\(\)\)\.To\(Equal\("(.*)"\)\)$', line)
        if m:
            out["intersection_string"].append({"a": m.group(1), "b": m.group(2), "expected": m.group(3)})
    return out


def extract_requirements(path):
    src = open(path).read()
    operands = {"unconstrained": []}
    for m in re.finditer(r"(\w+) := NewRequirements\(NewRequirement\(([^)]*)\)\)", src):
        name = m.group(1)
        if "badLabel" in m.group(2):
            continue
        if name not in operands:
            operands[name] = [parse_args(m.group(2))]
    out = {"source": "pkg/scheduling/requirements_test.go", "operands": operands, "compatible": [],
           "error_text": [], "string": []}
    for line in src.splitlines():
        s = line.strip()
        m = re.match(r"Expect\((\w+)\.Compatible\((\w+)(, AllowUndefinedWellKnownLabels)?\)\)\.(To|ToNot)\(Succeed\(\)\)$", s)
        if m and m.group(1) in operands and m.group(2) in operands:
            out["compatible"].append({"a": m.group(1), "b": m.group(2), "loose": bool(m.group(3)),
                                      "expected": m.group(4) == "To"})
            continue
        m = re.match(r'Entry\("[^"]*", "([^"]*)", `([^`]*)`\),?$', s)
        if m:
            out["error_text"].append({"label": m.group(1), "loose": True, "expected": m.group(2)})
    m = re.search(r'NewRequirement\("deployment", v1\.NodeSelectorOpExists\)\)\s*\n\s*Expect\(unconstrained\.Compatible\(req\)\.Error\(\)\)\.To\(Equal\(`([^`]*)`\)\)', src)
    if m:
        out["error_text"].append({"label": "deployment", "loose": False, "expected": m.group(1)})
    # String ordering (:623-645)
    blk = re.search(r'It\("should print Requirements in the same order".*?reqs := NewRequirements\((.*?)\n\t\t\t\)\s*\n\s*Expect\(reqs\.String\(\)\)\.To\(Equal\("([^"]*)"\)\)', src, re.S)
    if blk:
        reqs = [parse_args(a) for a in re.findall(r"NewRequirement\(([^)]*)\)", blk.group(1))]
        out["string"].append({"requirements": reqs, "expected": blk.group(2)})
    return out


def main():
    req = extract_requirement(os.path.join(REF, "pkg/scheduling/requirement_test.go"))
    reqs = extract_requirements(os.path.join(REF, "pkg/scheduling/requirements_test.go"))
    with open(os.path.join(HERE, "requirement_vectors.json"), "w") as f:
        json.dump(req, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "requirements_vectors.json"), "w") as f:
        json.dump(reqs, f, indent=1, sort_keys=True)
    print("requirement: %d intersection, %d has, %d operator, %d len, %d string, %d intersection-string" % (
        len(req["intersection"]), len(req["has"]), len(req["operator"]), len(req["len"]), len(req["string"]),
        len(req["intersection_string"])))
    print("requirements: %d compatible, %d error-text, %d string" % (
        len(reqs["compatible"]), len(reqs["error_text"]), len(reqs["string"])))


if __name__ == "__main__":
    sys.exit(main())
