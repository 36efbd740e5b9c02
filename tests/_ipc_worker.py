"""One side of tests/test_ipc.py: a process that exports device buffers
through the C-ABI (gp_malloc_device_shared + gp_ipc_get_handle) or maps a
peer's handles (gp_ipc_open_handle) and checks the bytes.  Handles travel as
files in a directory shared by the two processes.

    python tests/_ipc_worker.py export DIR N
    python tests/_ipc_worker.py import DIR N [corrupt]
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from geeps_amd import native  # noqa: E402

HANDLE = 96  # GP_IPC_HANDLE_BYTES
SIZE = 3 << 20  # 3 MiB: rounded up to 4 MiB, tag in the spare end


def wait_for(path, timeout=60.0):
    t0 = time.monotonic()
    while not os.path.exists(path):
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(path)
        time.sleep(0.002)


def main():
    role, d, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    L = native.lib()
    if role == "export":
        bufs, bases, described = [], [], []
        for k in range(n):
            p = ctypes.c_void_p()
            native.check(L.gp_malloc_device_shared(ctypes.byref(p), SIZE), "gp_malloc_device_shared")
            native.check(L.gp_memset_async(p, 1 + k, SIZE, None), "gp_memset_async")
            native.check(L.gp_device_synchronize(), "sync")
            h = (ctypes.c_ubyte * HANDLE)()
            native.check(L.gp_ipc_get_handle(h, p), "gp_ipc_get_handle")
            line = ctypes.create_string_buffer(400)
            native.check(L.gp_ipc_describe_handle(h, line, 400), "gp_ipc_describe_handle")
            described.append(line.value.decode())
            bufs.append(p)
            bases.append(p.value)
            tmp = os.path.join(d, f"h{k}.tmp")
            with open(tmp, "wb") as f:
                f.write(bytes(h))
            os.rename(tmp, os.path.join(d, f"h{k}"))
        # a plain allocation is refused
        q = ctypes.c_void_p()
        native.check(L.gp_malloc_device(ctypes.byref(q), SIZE), "gp_malloc_device")
        h = (ctypes.c_ubyte * HANDLE)()
        refused = L.gp_ipc_get_handle(h, q) == native.GP_ERR_INVALID
        wait_for(os.path.join(d, "done"), 120)
        print(json.dumps({"role": "export", "plain_refused": refused, "pid": os.getpid(), "bases": bases,
                          "described": described}))
        return
    corrupt = len(sys.argv) > 4 and sys.argv[4] == "corrupt"
    res = []
    for k in range(n):
        wait_for(os.path.join(d, f"h{k}"))
        with open(os.path.join(d, f"h{k}"), "rb") as f:
            raw = bytearray(f.read())
        if corrupt:
            raw[80] ^= 0xFF  # a byte of the tag the handle carries
        h = (ctypes.c_ubyte * HANDLE).from_buffer_copy(bytes(raw))
        p = ctypes.c_void_p()
        rc = L.gp_ipc_open_handle(ctypes.byref(p), h)
        if rc != native.GP_OK:
            res.append({"k": k, "ok": False, "err": L.gp_last_error().decode()})
            continue
        got = (ctypes.c_ubyte * 64)()
        native.check(L.gp_memcpy_async(got, p, 64, None), "gp_memcpy_async")
        native.check(L.gp_device_synchronize(), "sync")
        res.append({"k": k, "ok": all(b == 1 + k for b in got), "err": ""})
        native.check(L.gp_ipc_close_handle(p), "gp_ipc_close_handle")
    mismaps = ctypes.c_int()
    native.check(L.gp_ipc_mismaps(ctypes.byref(mismaps)), "gp_ipc_mismaps")
    with open(os.path.join(d, "done"), "w") as f:
        f.write("1")
    print(json.dumps({"role": "import", "results": res, "mismaps": mismaps.value}))


if __name__ == "__main__":
    main()
