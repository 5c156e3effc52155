#!/usr/bin/env python3
"""Make the bunny fixtures of tests/golden/ from the reference's stanford_bunny.ply (run in
the build container only; the GPU box never reads /root/reference):
  bunny_unique_f32.npy   the 34,834 distinct vertices, in order of first occurrence
  bunny_vertex_ids.npy   for each of the 208,353 vertices of the file, its row in the
                         unique table (uint16): unique[ids] is the file's vertex list, in
                         the file order the reference's RandomDownSample shuffles.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/stanford_bunny.ply"


def main():
    raw = open(SRC, "rb").read()
    head_end = raw.index(b"end_header\n") + len(b"end_header\n")
    n = int([l for l in raw[:head_end].split(b"\n") if l.startswith(b"element vertex")][0].split()[2])
    v = np.frombuffer(raw[head_end:head_end + 12 * n], dtype="<f4").reshape(n, 3)
    keys = v.view(np.uint32).reshape(n, 3)
    table, first, ids = np.unique(keys, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first)              # unique rows in order of first occurrence
    rank = np.empty_like(order)
    rank[order] = np.arange(order.size)
    unique = v[first[order]]
    ids = rank[ids.reshape(-1)].astype(np.uint16)
    assert np.array_equal(unique[ids], v)
    gold = os.path.join(ROOT, "tests", "golden")
    np.save(os.path.join(gold, "bunny_unique_f32.npy"), np.ascontiguousarray(unique))
    np.save(os.path.join(gold, "bunny_vertex_ids.npy"), ids)
    print(f"{n} vertices, {unique.shape[0]} unique")


if __name__ == "__main__":
    main()
