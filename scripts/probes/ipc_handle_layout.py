"""What a HIP IPC handle names on this image.

One process, no imports: allocates a few device buffers, exports each (the
first one twice) and prints the process id, each buffer's address and size,
and the 64-B handle as sixteen 32-bit words, so the fields the runtime puts
in a handle (the exporter's pid? the buffer's address? a size? a counter?)
can be read off by comparing words with known values.

Why it matters: ROCr's non-legacy (DMA-buf) IPC, which this image runs
(HSA_ENABLE_IPC_MODE_LEGACY=0), resolves a handle at OPEN time, not at export
time -- libhsa-runtime64 runs a per-process server on the abstract unix socket
"hsa<pid>" that takes a decimal id from the importer, looks it up in a map of
exported ranges and exports a fresh DMA-buf for it, passed back by SCM_RIGHTS
(objdump of libhsa-runtime64.so.1.18.70200: the "xhsa%i" / "%li" format
strings, connect/recvmsg in the attach path, accept/strtoull/sendmsg in the
server thread).  Whatever the handle names is therefore looked up in the
exporter's state when the importer maps it.

Usage: python scripts/probes/ipc_handle_layout.py   (one JSON line)
"""
import ctypes
import json
import os


class IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


def main():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(IpcHandle), ctypes.c_void_p]
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    h.hipGetErrorString.restype = ctypes.c_char_p
    out = {"pid": os.getpid(), "pid_hex": f"{os.getpid():#x}", "buffers": []}
    bufs = []
    for size in (2 << 20, 2 << 20, 4 << 20, 6 << 20):
        p = ctypes.c_void_p()
        rc = h.hipMalloc(ctypes.byref(p), size)
        if rc:
            out["buffers"].append({"size": size, "malloc_error": h.hipGetErrorString(rc).decode()})
            continue
        bufs.append(p)
        rec = {"ptr": f"{p.value:#x}", "size": size, "size_hex": f"{size:#x}", "exports": []}
        for _ in range(2 if len(bufs) == 1 else 1):
            hd = IpcHandle()
            rc = h.hipIpcGetMemHandle(ctypes.byref(hd), p)
            raw = bytes(hd.reserved)
            words = [int.from_bytes(raw[i:i + 4], "little") for i in range(0, 64, 4)]
            rec["exports"].append({"rc": rc, "err": h.hipGetErrorString(rc).decode() if rc else "",
                                   "words_hex": [f"{w:#x}" for w in words],
                                   "u64_hex": [f"{int.from_bytes(raw[i:i + 8], 'little'):#x}"
                                               for i in range(0, 64, 8)]})
        out["buffers"].append(rec)
    for p in bufs:
        h.hipFree(p)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
