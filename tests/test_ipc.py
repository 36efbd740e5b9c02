"""Inter-process device buffers through the C-ABI (gp_malloc_device_shared,
gp_ipc_get_handle, gp_ipc_open_handle): what libgeeps' same-node data path
stands on.  Two fresh processes per case (tests/_ipc_worker.py).

The export writes a tag into the buffer's spare end and the handle carries
it; a mapping must hold it.  A handle whose tag does not match what the
mapping holds (here: the tag bytes flipped in transit, standing in for the
runtime mapping other memory) is refused loudly, never handed out."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

WORKER = os.path.join(REPO, "tests", "_ipc_worker.py")


def _run(tmp_path, n, corrupt=False):
    d = str(tmp_path)
    exp = subprocess.Popen([sys.executable, WORKER, "export", d, str(n)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    imp = subprocess.Popen([sys.executable, WORKER, "import", d, str(n)] + (["corrupt"] if corrupt else []),
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    outs = []
    for p in (imp, exp):
        try:
            o, e = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            imp.kill()
            exp.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    return outs[0], outs[1]


@pytest.mark.gpu
def test_ipc_handles_map_the_exported_bytes(dev, tmp_path):
    imp, exp = _run(tmp_path, 8)
    assert exp["plain_refused"], "a plain gp_malloc_device buffer must not be exportable"
    assert [r["ok"] for r in imp["results"]] == [True] * 8, imp


@pytest.mark.gpu
def test_ipc_mapping_without_the_exporters_tag_is_refused(dev, tmp_path):
    imp, _ = _run(tmp_path, 3, corrupt=True)
    for r in imp["results"]:
        assert not r["ok"] and "does not hold the exporter's tag" in r["err"], r
