"""ORACLE — test infrastructure only.

A CPU restatement of the reference Karpenter Solve path (cpu_ref.cpp).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package; the product
(karpenter-sigs_amd/) never does.
"""
