"""MI355X-native Karpenter scheduler hot path (Scheduler.Solve) — Python mirror of the C-ABI.

The product is libkarpenter_amd.so (HIP kernels for gfx950 + C-ABI, include/karpenter_amd.h).
This package only marshals snapshots and results; there is no CPU fallback: every entry point
raises if the HIP library is missing or no GPU is visible.
"""
from .scheduler import Consolidator, snapshot_check, encode_binary, check_binary, cluster_state, inspect_consolidation, inspect_consolidation_update, shard_slot, KsError, Results, Scheduler, inspect, lib, library_path  # noqa: F401
