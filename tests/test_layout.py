"""Byte layout of the boundary types vs the reference's own headers (no GPU).

oracle/layout_probe.cpp is compiled once against include/ (this repo's drop-in
geeps.hpp / geeps-user-defined-types.hpp) + libgeeps' wire.hpp, and once against
the reference's unmodified headers (oracle/_ref/layout_probe, built only where
/root/reference exists).  Both must print the same JSON; the reference output is
frozen in tests/golden/ref_layout.json so the check also runs without the tree.
"""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, REPO

ORACLE = os.path.join(REPO, "oracle")


def _probe(path):
    return json.loads(subprocess.run([path], check=True, capture_output=True, text=True).stdout)


@pytest.fixture(scope="module")
def ours():
    subprocess.run(["make", "-s", "-C", ORACLE, "build/layout_probe_ours"], check=True)
    return _probe(os.path.join(ORACLE, "build", "layout_probe_ours"))


def test_layout_matches_frozen_reference(ours):
    with open(os.path.join(GOLDEN, "ref_layout.json")) as f:
        ref = json.load(f)
    assert ours == ref


def test_layout_matches_live_reference(ours):
    if not os.path.exists("/root/reference/include/geeps.hpp"):
        pytest.skip("/root/reference absent (GPU box)")
    subprocess.run(["make", "-s", "-C", ORACLE, "ref"], check=True)
    assert _probe(os.path.join(ORACLE, "_ref", "layout_probe")) == ours


def test_key_sizes(ours):
    assert ours["sizeof(RowData)"] == 512
    assert ours["sizeof(RowKey)"] == 16
    assert ours["sizeof(cs_clock_with_updates_batch_msg_t)"] == 24
    assert ours["sizeof(sc_read_row_batch_msg_t)"] == 24
    assert ours["ROW_DATA_SIZE"] == 128


def test_double_index_layout():
    import ctypes
    from geeps_amd.native import DoubleIndex
    # reference DoubleIndex {size_t id0; size_t id1;} (row-op-util.hpp:40-44)
    assert ctypes.sizeof(DoubleIndex) == 16
    assert DoubleIndex.id0.offset == 0 and DoubleIndex.id1.offset == 8
