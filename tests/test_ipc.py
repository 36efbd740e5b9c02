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
    assert imp["mismaps"] == 0
    # the runtime's handle names (exporter pid, buffer address) on this image:
    # gp_ipc_describe_handle reads both off the handle and checks them against
    # what the export recorded (gp_runtime.hip's header)
    for base, line in zip(exp["bases"], exp["described"]):
        assert f"exporter pid {exp['pid']} base {base:#x} (4194304 B)" in line, line
        assert f"runtime handle: pid {exp['pid']} address {base:#x} size 4194304 (names the exported buffer)" \
            in line, line


@pytest.mark.gpu
def test_ipc_mapping_without_the_exporters_tag_is_refused(dev, tmp_path):
    """17 handles whose carried tag was flipped in transit: each of the first
    16 maps the right buffer (the runtime handle is intact), fails the tag
    check and says so, naming the exporter's pid, and is left mapped, unused
    (its address must not go to a buffer this process exports later); the 17th
    is refused before the runtime is asked (the bound on mis-mappings)."""
    imp, exp = _run(tmp_path, 17, corrupt=True)
    for r in imp["results"][:16]:
        assert not r["ok"] and "does not hold the exporter's tag" in r["err"], r
        assert "names the exported buffer" in r["err"], r
        assert f"the mapping holds a buffer tagged by pid {exp['pid']}" in r["err"], r
        assert "a new address" in r["err"] and r["err"].endswith("; kept mapped, unused"), r
    last = imp["results"][16]
    assert not last["ok"] and "IPC mapping refused: the runtime mis-mapped 16 handles" in last["err"], last
    assert imp["mismaps"] == 16


def test_ipc_describe_handle_reads_the_runtime_fields():
    """CPU: gp_ipc_describe_handle on handles laid out as this image's runtime
    lays them out (scripts/probes/ipc_handle_layout.py): the runtime part's
    address / pid / size against the exporter's own record."""
    import ctypes
    import struct
    from geeps_amd import native
    L = native.lib()
    pid, base, size = 4242, 0x7A4D27600000, 4 << 20

    def handle(rt_pid, rt_addr, rt_size):
        rt = bytearray(64)
        struct.pack_into("<QI", rt, 0, rt_addr, rt_pid)
        struct.pack_into("<Q", rt, 32, rt_size)
        struct.pack_into("<I", rt, 48, rt_pid)
        tail = struct.pack("<QQQQ", size - 256, 0x67704950 << 32 | pid, 0x1234, base)
        return (ctypes.c_ubyte * 96).from_buffer_copy(bytes(rt) + tail)

    buf = ctypes.create_string_buffer(400)
    assert L.gp_ipc_describe_handle(handle(pid, base, size), buf, 400) == native.GP_OK
    line = buf.value.decode()
    assert f"exporter pid {pid} base {base:#x} ({size} B)" in line
    assert line.endswith("(names the exported buffer)"), line
    for bad in (handle(pid + 1, base, size), handle(pid, base + (2 << 20), size), handle(pid, base, 2 << 20)):
        assert L.gp_ipc_describe_handle(bad, buf, 400) == native.GP_OK
        assert buf.value.decode().endswith("(DOES NOT name the exported buffer)")
    junk = (ctypes.c_ubyte * 96)()
    assert L.gp_ipc_describe_handle(junk, buf, 400) == native.GP_ERR_INVALID
