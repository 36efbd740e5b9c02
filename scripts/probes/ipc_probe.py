"""Probe of HIP IPC memory handles between two processes.

libgeeps aborted once with ROCr's "IPC Attach: Invalid IPC handle! %u and %u"
from hipIpcOpenMemHandle (profiles/r03/e2e/pytest_libgeeps_race.log:379-382),
in a test whose tables are 2,000 rows x 512 B: every exported buffer was a
1,024,000-B hipMalloc.  This probe talks to the HIP runtime directly (ctypes on
libamdhip64, none of libgeeps' wrappers or locks) and asks, per scenario, whether
a handle still opens, and still maps the exported bytes, when:

  seq        each buffer is opened before the next one is exported;
  seq_big    the same with 4-MiB buffers;
  batch      every buffer is exported before the importer opens the first;
  batch_big  the same with 4-MiB buffers (allocations of their own);
  twice      one buffer exported twice, the FIRST handle opened afterwards;
  bidir      both processes export new buffers on one thread while another
             thread opens the peer's handles, as libgeeps' server and reader
             threads do (no lock around the runtime's IPC calls).
  freed      an exported buffer is freed and its address range reused by a
             new allocation before the importer opens the old handle.
  keep       as batch, but the importer keeps every mapping open (libgeeps
             never closes a peer's oplog or version mapping while it runs);
  mt_open    the importer opens the handles from 2 threads at once (pairs
             of fragments of one 2-MiB block), keeping every mapping open,
             no lock: libgeeps' reader threads of two channels and its
             server-side reader threads map a peer's buffers concurrently;
  mt_export  the exporter allocates and exports from 2 threads at once.
  stress_frag / stress_whole
             256 buffers of 1,024,000 B (fragments: two share a 2-MiB block)
             or of 2 MiB (whole allocations, as gp_malloc_device_shared
             makes them), each exported; failed exports are counted, not
             raised; the importer maps the rest from 2 threads, keeping every
             mapping open.  Failure counts per side.
  retry      64 whole buffers exported right after the process's first HIP
             calls; a failed export is retried every 20 ms (up to 50 times):
             attempts per buffer, and how long after the first try it worked;
  late       the same, but the process first sleeps 3 s after its first
             device allocation: does the failure need a young process?
  warm       as late, but the process's first device allocation is a 4-MiB
             buffer that is never exported: is it the first allocation?
  primed     as late, but a throwaway 2-MiB buffer is allocated and exported
             (its failure ignored) before the first real buffer is
             allocated: is it a buffer allocated before the process's first
             export (gp_malloc_device_shared primes so)?

Each scenario runs as two fresh processes (exporter / importer, or two peers)
that pass handles through files.  Output: one JSON line per scenario with
ok / failure counts, the allocation addresses (is a small buffer a fragment
of a shared block?) and the runtime's stderr lines.

Usage: python scripts/probes/ipc_probe.py [scenario ...]

Round 5: a GPU box was lost running the `late` / `primed`
scenarios (scripts/gpu_runs/r04/dev5.sh), 20 runs of two processes with 64 x
2 MiB exports each.  What in this probe could leave a box unrecoverable, from
its code (nothing came back from that run):
  1. open_and_check read 16 B at +0 and at +nbytes-16 of every mapping with
     hipMemcpy, whatever the runtime mapped.  The probe had seen mappings of
     OTHER memory (0xFF instead of the exported value); a mapping of a
     smaller or unrelated range read at +2 MiB - 16 is a device access past
     the mapping: a GPU memory fault, the one step here that can take a device
     (and, on this pool, its host) down.
  2. `keep` mappings (128 in those scenarios) were left open to process exit,
     including any mis-mapped one, so the runtime tore them down at exit.
  3. The driver's 45-s deadline SIGKILLed a process still holding mappings
     (and maybe a queued copy through one).
  4. The rocprofv3 step after the probe ran only first_call_breakdown.py
     (kernel + memory-copy traces, no counters): not implicated.
Fixed here: a mapping is read only after hipMemGetAddressRange shows that it
spans every byte read (else it is reported as mis-mapped, unread); every
mapping is closed before the process exits; a stuck process gets SIGTERM and
5 s before SIGKILL.  The `late` / `primed` / `warm` / `retry` scenarios are not
to be run on the shared pool again: they refuse to start unless
IPC_PROBE_ALLOW_YOUNG=1.  libgeeps itself checks a mapping's range and tag
before it reads one byte of it (gp_ipc_open_handle), and a failed mapping
costs a resend over the socket (wire.hpp, NACKs).
"""
from __future__ import annotations

import ctypes
import faulthandler
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

SMALL = 2000 * 512       # a 2,000-row RowData buffer, as in the failing test
BIG = 4 << 20


class IpcHandle(ctypes.Structure):
    # bytes, not c_char: a c_char array field reads back cut at its first NUL
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(IpcHandle), ctypes.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), IpcHandle, ctypes.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
    h.hipGetErrorString.restype = ctypes.c_char_p
    h.hipDeviceSynchronize.argtypes = []
    return h


def call(h, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {h.hipGetErrorString(rc).decode()}")


def alloc(h, nbytes, value):
    p = ctypes.c_void_p()
    call(h, h.hipMalloc(ctypes.byref(p), nbytes), "hipMalloc")
    call(h, h.hipMemset(p, value, nbytes), "hipMemset")
    call(h, h.hipDeviceSynchronize(), "sync")
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    call(h, h.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), p), "range")
    return p, {"ptr": p.value, "base_is_ptr": base.value == p.value, "range": size.value}


def export(h, p):
    hd = IpcHandle()
    call(h, h.hipIpcGetMemHandle(ctypes.byref(hd), p), "hipIpcGetMemHandle")
    return ctypes.string_at(ctypes.addressof(hd), 64)


def put(d, name, payload):
    tmp = os.path.join(d, name + ".tmp")
    with open(tmp, "wb") as f:
        f.write(payload)
    os.rename(tmp, os.path.join(d, name))


def get(d, name, timeout=30.0):
    path = os.path.join(d, name)
    t0 = time.monotonic()
    while not os.path.exists(path):
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(name)
        time.sleep(0.001)
    with open(path, "rb") as f:
        return f.read()


OPEN_MAPPINGS = []  # kept mappings, closed before the process exits (close_all)
OPEN_LOCK = threading.Lock()


def close_all(h):
    with OPEN_LOCK:
        while OPEN_MAPPINGS:
            h.hipIpcCloseMemHandle(OPEN_MAPPINGS.pop())


def open_and_check(h, raw, value, nbytes, keep=False):
    """Open a handle; return (ok, detail).  keep: leave the mapping open (until
    close_all).  The mapping is read only where hipMemGetAddressRange shows it
    spans the bytes read: a mis-mapped handle is reported, never read past."""
    hd = IpcHandle()
    assert len(raw) == 64
    ctypes.memmove(ctypes.addressof(hd), raw, 64)
    p = ctypes.c_void_p()
    rc = h.hipIpcOpenMemHandle(ctypes.byref(p), hd, 1)  # hipIpcMemLazyEnablePeerAccess
    if rc != 0:
        return False, "open: " + h.hipGetErrorString(rc).decode()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    if h.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), p) != 0 or base.value is None \
            or p.value < base.value or p.value + nbytes > base.value + size.value:
        h.hipIpcCloseMemHandle(p)
        return False, f"mapping {p.value:#x} does not span {nbytes} B (range {base.value} + {size.value}): unread"
    out = (ctypes.c_ubyte * 16)()
    for off in (0, nbytes - 16):
        call(h, h.hipMemcpy(out, ctypes.c_void_p(p.value + off), 16, 2), "D2H")  # DeviceToHost
        if any(b != value for b in out):
            h.hipIpcCloseMemHandle(p)
            return False, f"mapped bytes {list(out)[:4]} at +{off}, exported {value}"
    if keep:
        with OPEN_LOCK:
            OPEN_MAPPINGS.append(p)
    else:
        call(h, h.hipIpcCloseMemHandle(p), "close")
    return True, ""


# --- roles -------------------------------------------------------------------
def progress(*a):
    print(f"[{time.monotonic():.3f}]", *a, file=sys.stderr, flush=True)


def exporter(scn, d):
    faulthandler.dump_traceback_later(20, repeat=True)  # where a hang sits
    h = hip()
    n = 16
    size = BIG if scn.endswith("_big") else SMALL
    keep, info = [], []
    if scn == "twice":
        p, inf = alloc(h, size, 7)
        keep.append(p)
        info.append(inf)
        put(d, "h0", export(h, p))
        put(d, "h1", export(h, p))
        put(d, "exported", b"2")
    elif scn == "mt_export":
        n = 64
        out = [None] * n

        def work(t):
            for k in range(t, n, 2):
                p, inf = alloc(h, size, 1 + k % 250)
                keep.append(p)
                out[k] = export(h, p)
        ths = [threading.Thread(target=work, args=(t,)) for t in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        for k in range(n):
            put(d, f"h{k}", out[k])
        put(d, "exported", str(n).encode())
    elif scn.startswith("stress"):
        n = 256
        size = SMALL if scn == "stress_frag" else 2 << 20
        fails = []
        for k in range(n):
            p, inf = alloc(h, size, 1 + k % 250)
            keep.append(p)
            try:
                raw = export(h, p)
            except RuntimeError as exc:
                fails.append({"k": k, "why": str(exc), "ptr_mod_2MiB": inf["ptr"] % (2 << 20)})
                raw = b""
            put(d, f"h{k}", raw)
        put(d, "exported", str(n).encode())
        info.append({"export_failures": fails})
    elif scn in ("retry", "late", "warm", "primed"):
        n = 64
        size = 2 << 20
        first = True
        primed_ok = None
        if scn in ("warm", "primed"):
            dummy, _ = alloc(h, 4 << 20 if scn == "warm" else 2 << 20, 0)
            keep.append(dummy)
            if scn == "primed":
                try:
                    export(h, dummy)
                    primed_ok = True
                except RuntimeError:
                    primed_ok = False
        attempts = []
        for k in range(n):
            p, inf = alloc(h, size, 1 + k % 250)
            keep.append(p)
            if first and scn in ("late", "warm", "primed"):
                time.sleep(3.0)
            first = False
            t0 = time.monotonic()
            for a in range(1, 51):
                try:
                    raw = export(h, p)
                    break
                except RuntimeError:
                    raw = b""
                    time.sleep(0.02)
            attempts.append({"k": k, "attempts": a, "ok": bool(raw), "ms": round((time.monotonic() - t0) * 1e3, 1)})
            put(d, f"h{k}", raw)
        put(d, "exported", str(n).encode())
        info.append({"retries": [x for x in attempts if x["attempts"] > 1], "primed_export_ok": primed_ok})
    elif scn == "mt_open":
        n = 64
        for k in range(n):
            p, inf = alloc(h, size, 1 + k % 250)
            keep.append(p)
            info.append(inf)
            put(d, f"h{k}", export(h, p))
        put(d, "exported", str(n).encode())
    elif scn == "freed":
        for k in range(n):
            p, inf = alloc(h, size, 1 + k)
            put(d, f"h{k}", export(h, p))
            info.append(inf)
            call(h, h.hipFree(p), "free")
            q, _ = alloc(h, size, 200)   # likely the same range, new contents
            keep.append(q)
        put(d, "exported", str(n).encode())
    else:
        for k in range(n):
            progress("alloc", k)
            p, inf = alloc(h, size, 1 + k)
            keep.append(p)
            info.append(inf)
            progress("export", k, inf)
            put(d, f"h{k}", export(h, p))
            if scn.startswith("seq"):
                get(d, f"opened{k}")
        put(d, "exported", str(n).encode())
    get(d, "done", timeout=60)
    print(json.dumps({"role": "exporter", "allocs": info}))


def importer(scn, d):
    faulthandler.dump_traceback_later(20, repeat=True)
    h = hip()
    n = int(get(d, "exported", timeout=60)) if not scn.startswith("seq") else 16
    results = []
    if scn in ("mt_open", "mt_export", "retry", "late", "warm", "primed") or scn.startswith("stress"):
        raws = [get(d, f"h{k}") for k in range(n)]
        nbytes = 2 << 20 if scn in ("stress_whole", "retry", "late", "warm", "primed") else SMALL
        go = threading.Barrier(2)

        def work(t):
            go.wait()
            for k in range(t, n, 2):
                if not raws[k]:
                    continue  # its export failed
                ok, why = open_and_check(h, raws[k], 1 + k % 250, nbytes, keep=True)
                results.append({"k": k, "ok": ok, "why": why})
        ths = [threading.Thread(target=work, args=(t,)) for t in range(1 if scn == "mt_export" else 2)]
        if scn == "mt_export":
            go = threading.Barrier(1)
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        close_all(h)
        put(d, "done", b"1")
        print(json.dumps({"role": "importer", "results": results}))
        return
    for k in range(n):
        raw = get(d, f"h{k}")
        value = 7 if scn == "twice" else 1 + k
        nbytes = BIG if scn.endswith("_big") else SMALL
        if scn == "twice" and k == 1:
            break  # only the first handle, opened after the second export
        progress("open", k)
        ok, why = open_and_check(h, raw, value, nbytes, keep=scn == "keep")
        progress("opened", k, ok, why)
        results.append({"k": k, "ok": ok, "why": why})
        if scn.startswith("seq"):
            put(d, f"opened{k}", b"1")
    close_all(h)
    put(d, "done", b"1")
    print(json.dumps({"role": "importer", "results": results}))


def peer(scn, d, me):
    """bidir: export new small buffers on one thread, open the peer's on another."""
    faulthandler.dump_traceback_later(20, repeat=True)
    h = hip()
    other = 1 - me
    n = 64
    keep = []
    errors = []

    def exp():
        for k in range(n):
            p, _ = alloc(h, SMALL, (me * 100 + k) % 251 + 1)
            keep.append(p)
            put(d, f"p{me}_h{k}", export(h, p))

    def imp():
        for k in range(n):
            raw = get(d, f"p{other}_h{k}")
            ok, why = open_and_check(h, raw, (other * 100 + k) % 251 + 1, SMALL)
            if not ok:
                errors.append({"k": k, "why": why})

    t1, t2 = threading.Thread(target=exp), threading.Thread(target=imp)
    t1.start()
    t2.start()
    t1.join()
    t2.join()
    put(d, f"p{me}_done", b"1")
    get(d, f"p{other}_done", timeout=60)
    print(json.dumps({"role": f"peer{me}", "opened": n, "errors": errors}))


YOUNG = ("retry", "late", "warm", "primed")  # the scenarios of the lost box (see the header)


def run(scn):
    if scn in YOUNG and os.environ.get("IPC_PROBE_ALLOW_YOUNG") != "1":
        print(json.dumps({"scenario": scn, "refused": "retired from the shared GPU pool (VERDICT r04 #3); "
                                                      "IPC_PROBE_ALLOW_YOUNG=1 overrides"}), flush=True)
        return
    d = tempfile.mkdtemp(prefix="ipc_probe_")
    me = os.path.abspath(__file__)
    if scn == "bidir":
        cmds = [[sys.executable, me, "--peer", scn, d, "0"], [sys.executable, me, "--peer", scn, d, "1"]]
    else:
        cmds = [[sys.executable, me, "--exporter", scn, d], [sys.executable, me, "--importer", scn, d]]
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for c in cmds]
    outs = []
    deadline = time.monotonic() + 45
    for p in procs:
        try:
            o, e = p.communicate(timeout=max(1.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.terminate()  # SIGTERM first: let it unwind its mappings
            try:
                o, e = p.communicate(timeout=5)
            except subprocess.TimeoutExpired:
                p.kill()
                o, e = p.communicate()
        outs.append({"rc": p.returncode, "out": [json.loads(x) for x in o.splitlines() if x.startswith("{")],
                     "stderr": [x for x in e.splitlines() if x.strip()][-40:]})
    print(json.dumps({"scenario": scn, "procs": outs}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--exporter":
        exporter(sys.argv[2], sys.argv[3])
    elif len(sys.argv) > 1 and sys.argv[1] == "--importer":
        importer(sys.argv[2], sys.argv[3])
    elif len(sys.argv) > 1 and sys.argv[1] == "--peer":
        peer(sys.argv[2], sys.argv[3], int(sys.argv[4]))
    else:
        for scn in sys.argv[1:] or ["seq_big", "seq", "batch_big", "batch", "twice", "bidir", "freed", "keep",
                                    "mt_open", "mt_export"]:
            run(scn)
