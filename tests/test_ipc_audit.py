"""DESIGN.md §4's IPC findings, re-derived from the committed logs (CPU).

scripts/ipc_audit.py over every process's GEEPS_IPC_LOG output of round 5's
two failing randomized seeds (256, 285), run once in round 6 with the
diagnostics (profiles/r06/ipc/seeds_256_285_ipc_log), and over the 300-seed
campaigns before and after the no-unmap rule (logs.tgz): the numbers DESIGN
states are what the audit finds."""
import json
import os
import subprocess
import sys
import tarfile

import pytest

from conftest import REPO

IPC = os.path.join(REPO, "profiles", "r06", "ipc")


def _audit(d):
    out = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "ipc_audit.py"), d], check=True,
                         capture_output=True, text=True).stdout
    return json.loads(out)


def test_seeds_256_285_failed_mappings_came_from_correct_handles():
    d = os.path.join(IPC, "seeds_256_285_ipc_log")
    if not os.path.isdir(d):
        pytest.skip("round-6 IPC logs not in this tree")
    a = _audit(d)
    assert a["exports"] == a["exports_naming_their_buffer"] == 219
    s = a["summary"]
    assert s["mismaps"] == 15 and s["handle_named_the_exported_buffer"] == 15
    assert s["held_another_tagged_buffer"] == 8 and s["of_which_the_exporter_had_mapped_it"] == 8
    assert s["held_untagged_memory"] == 7
    assert s["exported_address_was_an_earlier_mapping"] == 9
    assert sum(m["held_is_importers_own_buffer"] for m in a["mismaps"]) == 3
    assert {m["what"].split(" of ")[0] for m in a["mismaps"]} == {"oplog buffer 1"}


@pytest.mark.parametrize("build,mismaps,refused", [("campaign_before", 9, 18), ("campaign_after2", 0, 0)])
def test_campaign_before_and_after_the_no_unmap_rule(tmp_path, build, mismaps, refused):
    tgz = os.path.join(IPC, build, "logs.tgz")
    if not os.path.exists(tgz):
        pytest.skip("round-6 campaign logs not in this tree")
    with tarfile.open(tgz) as t:
        t.extractall(tmp_path, filter="data")
    s = _audit(str(tmp_path / "logs"))["summary"]
    assert s["mismaps"] == mismaps and s["runtime_refused_export"] == refused
    assert s["injected_tag_faults"] == 81 and s["host_oplog_refused"] == 9
    assert s["could_not_map"] == 81 + mismaps  # nothing else failed to map
