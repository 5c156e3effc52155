#!/usr/bin/env python3
"""Drive k_lrf8 alone for PMC passes (the TOLDI stage entry on KITTI-like clouds).

Usage (GPU box): SE3ICP_LIB=se3-icp_amd/lib_cutN/libse3icp.so \
    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ... -- python3 tools/lrf_count.py
The measurement builds (make variant VFLAGS=-DSE3ICP_LRF8_CUT=1/2/3) stop k_lrf8 after its
traversal / final order / neighbour sums, so the differences of the per-wave instruction
counts attribute them to the kernel's sections; their frames are not used.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se3-icp_amd"))

import se3icp  # noqa: E402
from se3icp import datasets  # noqa: E402

pairs, _ = datasets.kitti_like_pairs(2, seed=4)
for rep in range(2):
    for s, t in pairs:
        se3icp.toldi_frames(s, 90)
        se3icp.toldi_frames(t, 90)
print("lrf_count: done", flush=True)
