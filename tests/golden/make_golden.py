"""Generate the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py

Outputs (data only — inputs and expected outputs, no reference source):
  * rowops.npz / bucket.npz  seeded inputs and the CPU oracle's outputs
    (oracle/oracle.c, the restatement of src/common/row-op-util.hpp:81-139 and
    src/server/tablet-server.cpp:119-134).
  * ref_layout.json          output of oracle/_ref/layout_probe, i.e. the byte
    layout printed by the reference's own headers compiled unchanged (only
    regenerated when /root/reference is present).
  * manifest.json            shapes, seeds and sha256 of every array.

Seeds: deltas are uniform in [-0.5, 0.5) from numpy PCG64 seeded 1000 + client_id
(BASELINE.md §3); indices and initial caches use the seeds listed per case.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle  # noqa: E402


def _rng(seed):
    return np.random.default_rng(seed)


def rowop_cases():
    """(name, kind, W, cache_rows, op_rows, index, offset, limit, seed)."""
    cases = []

    def perm_index(rng, n_op, n_cache, contiguous):
        id0 = np.arange(n_op, dtype=np.uint64)
        if contiguous:  # channel slice: contiguous id1 range (clientlib-viter.cpp:871-873)
            start = int(rng.integers(0, n_cache - n_op + 1))
            id1 = start + rng.permutation(n_op).astype(np.uint64)
        else:
            id1 = rng.choice(n_cache, size=n_op, replace=False).astype(np.uint64)
        return np.stack([id0, id1], axis=1)

    specs = [
        # name, kind, W, cache_rows, op_rows, contiguous, offset, limit_rows(float or None)
        ("add_identity_w128", "add_from", 128, 256, 256, True, (0, 0), None),
        ("add_perm_w128", "add_from", 128, 384, 200, False, (0, 0), None),
        ("add_reversed_w64", "add_from", 64, 512, 512, True, (0, 0), None),
        ("add_perm_w1024", "add_from", 1024, 96, 64, False, (0, 0), None),
        ("add_offset_w128", "add_from", 128, 256, 100, False, (3, 7), None),
        ("add_limit_tail_w128", "add_from", 128, 256, 200, False, (0, 0), 150.5),
        ("add_scalar_w130", "add_from", 130, 128, 77, False, (0, 0), None),
        ("add_scalar_w3", "add_from", 3, 300, 257, False, (0, 0), 200.33),
        ("add_w4_perm", "add_from", 4, 2000, 1500, False, (0, 0), None),
        ("gather_perm_w128", "assign_to", 128, 384, 200, False, (0, 0), None),
        ("gather_limit_tail_w128", "assign_to", 128, 384, 200, False, (0, 0), 150.25),
        ("gather_offset_w64", "assign_to", 64, 400, 200, False, (5, 11), None),
        ("gather_scalar_w130", "assign_to", 130, 128, 77, False, (0, 0), None),
        ("scatter_perm_w128", "assign_from", 128, 384, 200, False, (0, 0), None),
        ("scatter_limit_tail_w64", "assign_from", 64, 384, 300, False, (0, 0), 123.75),
    ]
    for seed, (name, kind, W, n_cache, n_op, contig, off, limit_rows) in enumerate(specs, 1):
        rng = _rng(seed)
        if name.startswith("add_reversed"):
            index = np.stack([np.arange(n_op, dtype=np.uint64),
                              np.arange(n_op, dtype=np.uint64)[::-1]], axis=1)
        else:
            index = perm_index(rng, n_op, n_cache - off[1], contig)
        limit = None if limit_rows is None else int(limit_rows * W)
        cases.append((name, kind, W, n_cache, n_op, np.ascontiguousarray(index), off, limit, seed))
    return cases


def build_rowops():
    out, manifest = {}, {}
    for name, kind, W, n_cache, n_op, index, off, limit, seed in rowop_cases():
        rng = _rng(10_000 + seed)
        if kind == "assign_to":
            # x = cache (n_cache rows, indexed by id1+off1), y = op buffer (indexed by id0+off0)
            x = (rng.random(n_cache * W, dtype=np.float32) - np.float32(0.5))
            y = (rng.random((n_op + off[0]) * W, dtype=np.float32) - np.float32(0.5))
        else:
            # x = op buffer (indexed by id0+off0), y = cache (indexed by id1+off1)
            x = (rng.random((n_op + off[0]) * W, dtype=np.float32) - np.float32(0.5))
            y = (rng.random(n_cache * W, dtype=np.float32) - np.float32(0.5))
        expect = y.copy()
        fn = {"add_from": oracle.add_rows_from_double_index,
              "assign_to": oracle.assign_rows_to_double_index,
              "assign_from": oracle.assign_rows_from_double_index}[kind]
        fn(expect, x, index, off, W, limit)
        out[f"{name}.x"] = x
        out[f"{name}.y"] = y
        out[f"{name}.index"] = index.astype(np.int64)
        out[f"{name}.expect"] = expect
        manifest[name] = {"kind": kind, "row_size": W, "cache_rows": n_cache, "op_rows": n_op,
                          "offset": list(off), "num_vals_limit": limit, "seed": seed}
    return out, manifest


def build_bucket():
    out, manifest = {}, {}
    R, W = 1024, 64   # BASELINE config 1: 1K rows x 64 fp32 (= 512 RowData rows)
    n = R * W
    deltas = np.stack([oracle.synthetic_delta(c, n) for c in range(8)])
    out["deltas"] = deltas
    for N in (1, 2, 8):
        m = np.zeros(n, dtype=np.float32)        # master zero-initialised (tablet-server.cpp:108-114)
        oracle.apply_updates(m, [deltas[c] for c in range(N)])
        out[f"master_zero_N{N}"] = m
    init = (_rng(77).random(n, dtype=np.float32) - np.float32(0.5))
    out["master_seeded_init"] = init
    m = init.copy()
    oracle.apply_updates(m, [deltas[c] for c in range(8)])
    out["master_seeded_N8"] = m
    # reversed arrival order: same multiset, different fp32 rounding
    m = np.zeros(n, dtype=np.float32)
    oracle.apply_updates(m, [deltas[c] for c in reversed(range(8))])
    out["master_zero_N8_reversed"] = m
    manifest["bucket"] = {"rows": R, "row_size": W, "clients": 8, "delta_seeds": "1000+c",
                          "seeded_init_seed": 77}
    return out, manifest


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    oracle.build()
    rowops, m1 = build_rowops()
    bucket, m2 = build_bucket()
    np.savez_compressed(os.path.join(HERE, "rowops.npz"), **rowops)
    np.savez_compressed(os.path.join(HERE, "bucket.npz"), **bucket)
    manifest = {"generator": "tests/golden/make_golden.py", "rowops": m1, "bucket": m2,
                "sha256": {**{f"rowops:{k}": sha(v) for k, v in rowops.items()},
                           **{f"bucket:{k}": sha(v) for k, v in bucket.items()}}}
    ref_probe = os.path.join(REPO, "oracle", "_ref", "layout_probe")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    if os.path.exists(ref_probe):
        text = subprocess.run([ref_probe], check=True, capture_output=True, text=True).stdout
        json.loads(text)
        with open(os.path.join(HERE, "ref_layout.json"), "w") as f:
            f.write(text)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
