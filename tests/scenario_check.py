"""Check Solve results against the reference tests' assertions (tests/golden/scenarios.json)."""


def launched_type(claim, snap):
    """fake CloudProvider.Create (fake/cloudprovider.go:96-141): the cheapest option by the price of its
    available offerings (claim requirements restrict zone / capacity-type).  With the launch list the
    product renders (ToNodeClaim + OrderByPrice), that is its first entry; the fallback recomputes it."""
    if claim.get("launchInstanceTypes"):
        return claim["launchInstanceTypes"][0]
    its = {it["name"]: it for it in snap["instanceTypes"]}
    zone_ok, ct_ok = None, None
    for r in claim["requirements"]:
        key, op = r.split(" ")[0], r.split(" ")[1]
        vals = r[r.index("[") + 1:r.index("]")].split(" ") if "[" in r else []
        if key == "topology.kubernetes.io/zone" and op == "In":
            zone_ok = set(vals)
        if key == "karpenter.sh/capacity-type" and op == "In":
            ct_ok = set(vals)
    best = None
    for name in claim["instanceTypeOptions"]:
        prices = [o["price"] for o in its[name]["offerings"] if o.get("available", True)
                  and (zone_ok is None or o["zone"] in zone_ok) and (ct_ok is None or o["capacityType"] in ct_ok)]
        if prices and (best is None or min(prices) < best[0]):
            best = (min(prices), name)
    return best[1] if best else None


def check(scn, res):
    """res: canonical results dict.  Returns a list of violated expectations."""
    exp, snap = scn["expect"], scn["snapshot"]
    bad = []
    claims = res["newNodeClaims"]
    if len(claims) != exp["nodes"]:
        bad.append("nodes %d != %d" % (len(claims), exp["nodes"]))
    types = [launched_type(c, snap) for c in claims]
    if "type" in exp and any(t != exp["type"] for t in types):
        bad.append("types %s != %s" % (types, exp["type"]))
    if exp.get("types_differ") and len(set(types)) != len(types):
        bad.append("types not distinct: %s" % types)
    for pi, want in exp.get("pod_types", {}).items():
        got = [t for c, t in zip(claims, types) if int(pi) in c["pods"]]
        if got != [want]:
            bad.append("pod %s launched %s, want %s" % (pi, got, want))
    errs = sorted(int(k) for k in res["podErrors"])
    want_errs = [] if exp["scheduled"] is True else sorted(exp["scheduled"])
    if errs != want_errs:
        bad.append("unschedulable %s != %s" % (errs, want_errs))
    return bad
