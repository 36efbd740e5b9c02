"""libgeeps' shared host memory (geeps_amd/csrc/geeps/hostshare.hpp): the host
tier's oplogs, which a same-node server maps to read a client's host-tier rows
in place instead of receiving them through the socket.

CPU tests over two processes (tests/apps/hostshare_check.cpp): a peer maps the
buffer by its handle and reads what the owner wrote; a handle with the wrong
tag, size or descriptor, or of an owner that has exited, is refused with a
reason (libgeeps then NACKs and the rows come by socket: tests/test_libgeeps.py).
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(REPO, "build", "tests", "hostshare_check")

pytestmark = pytest.mark.skipif(not os.path.exists(APP), reason="build() first (build/tests/hostshare_check)")


class Owner:
    def __init__(self, floats):
        self.p = subprocess.Popen([APP, "create", str(floats)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  text=True)
        line = self.p.stdout.readline().split()
        assert len(line) == 5, line
        self.pid, self.fd, self.map_bytes, self.tag, self.pinned = line
        self.floats = floats

    def args(self, **over):
        a = dict(pid=self.pid, fd=self.fd, map_bytes=self.map_bytes, tag=self.tag, floats=str(self.floats))
        a.update(over)
        return [APP, "open", a["pid"], a["fd"], a["map_bytes"], a["tag"], a["floats"]]

    def close(self):
        if self.p.poll() is None:
            self.p.stdin.write("\n")
            self.p.stdin.flush()
        self.p.wait(timeout=30)


def _open(args):
    r = subprocess.run(args, capture_output=True, text=True, timeout=60)
    return r.returncode, r.stdout.strip()


@pytest.mark.parametrize("floats", [1, 128, 1000 * 128 + 7, 1 << 22])
def test_peer_reads_what_the_owner_wrote(floats):
    o = Owner(floats)
    try:
        rc, out = _open(o.args())
        assert (rc, out) == (0, "ok")
        # the mapping is the rows rounded up to pages, then the tag page
        page = os.sysconf("SC_PAGE_SIZE")
        assert int(o.map_bytes) == (floats * 4 + page - 1) // page * page + page
    finally:
        o.close()


def test_wrong_tag_is_refused():
    o = Owner(4096)
    try:
        bad = o.tag[:-2] + ("00" if o.tag[-2:] != "00" else "11")
        rc, out = _open(o.args(tag=bad))
        assert rc == 3 and "tag" in out, out
    finally:
        o.close()


def test_wrong_size_and_descriptor_are_refused():
    o = Owner(4096)
    try:
        page = os.sysconf("SC_PAGE_SIZE")
        rc, out = _open(o.args(map_bytes=str(int(o.map_bytes) + page)))
        assert rc == 3 and "not the buffer" in out, out
        rc, out = _open(o.args(fd="0"))  # the owner's stdin: not a libgeeps memfd
        assert rc == 3 and "not a libgeeps host oplog" in out, out
        rc, out = _open(o.args(fd="987654"))
        assert rc == 3 and "open" in out, out
    finally:
        o.close()


def test_owner_gone_is_refused():
    o = Owner(4096)
    args = o.args()
    o.close()
    rc, out = _open(args)
    assert rc == 3 and "open" in out, out


def test_malformed_handle_is_refused():
    o = Owner(128)
    try:
        rc, out = _open(o.args(map_bytes="100"))
        assert rc == 3 and "malformed" in out, out
    finally:
        o.close()


@pytest.mark.gpu
def test_buffers_are_page_locked_on_a_gpu_box():
    """With a GPU, the owner's buffer is page-locked (gp_host_register, C-ABI
    14), so the server's host-to-device copy out of it runs at the pinned
    rate; a peer's mapping of it reads the owner's rows as on the CPU."""
    o = Owner(1 << 22)
    try:
        assert o.pinned == "1"
        rc, out = _open(o.args())
        assert (rc, out) == (0, "ok")
    finally:
        o.close()
