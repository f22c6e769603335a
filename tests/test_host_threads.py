"""Host encode at sizes where the worker threads engage (ks_parallel.h: the JSON parser's large arrays,
pod parsing / encoding, NewTopology's per-pod groups and countDomains; ks_cons.cpp's pod parse): the
result must not depend on the thread count.  These are the inputs scripts/tsan_cpu_suite.sh and
scripts/asan_cpu_suite.sh run the threaded host code over."""
import json
import os
import subprocess
import sys

from karpenter_amd import inspect, inspect_consolidation, synth

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

_ONE_THREAD = r"""
import json, sys
sys.path[:0] = [%r, %r]
from karpenter_amd import inspect, inspect_consolidation
snap = open(sys.argv[2]).read()
print(json.dumps(inspect(snap) if sys.argv[1] == "solve" else inspect_consolidation(snap), sort_keys=True))
""" % (ROOT, os.path.join(ROOT, "karpenter-sigs_amd"))


def _single_thread(kind, snap, tmp_path):
    f = tmp_path / "snap.json"
    f.write_text(snap)
    env = dict(os.environ, KS_HOST_THREADS="1")
    out = subprocess.check_output([sys.executable, "-c", _ONE_THREAD, kind, str(f)], env=env)
    return json.loads(out)


def test_threaded_solve_encode_matches_one_thread(tmp_path):
    snap = json.dumps(synth.config4(3000, 600))
    many = json.loads(json.dumps(inspect(snap), sort_keys=True))
    assert many == _single_thread("solve", snap, tmp_path)


def test_threaded_consolidation_encode_matches_one_thread(tmp_path):
    snap = json.dumps(synth.cluster_snapshot(400, 20, 400, seed=4205, topology=8))
    many = json.loads(json.dumps(inspect_consolidation(snap), sort_keys=True))
    assert many == _single_thread("cons", snap, tmp_path)
