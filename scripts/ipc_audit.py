"""Audit of libgeeps' IPC logs (GEEPS_IPC_LOG=1, one file per process, as
tests/test_libgeeps.py writes them with GEEPS_TEST_LOG_DIR): for every mapping
that failed its tag check, what the handle named, what the mapping held, and
whether the EXPORTING process had itself mapped (imported) the buffer whose tag
the mapping held -- the signature of the runtime's exporter handing out a
DMA-buf of one of its imports instead of the buffer at the named address
(DESIGN.md §4).

`could_not_map` counts every failed device mapping (tag mismatches and the
runtime's own refusals; `host_oplog_refused` the shared host oplogs a server
could not map, which GEEPS_TEST_IPC_FAULT injects too); `injected_tag_faults` the tag mismatches GEEPS_TEST_IPC_FAULT=tag
caused (the right buffer, the handle's tag flipped), which the rest leaves out;
`runtime_refused_export` the exports the runtime refused (not the injected
refusals).

Usage: python scripts/ipc_audit.py LOG_DIR   (one JSON object on stdout)
"""
import json
import os
import re
import sys

EXPORT = re.compile(r"libgeeps ipc export \w+: .*?exporter pid (\d+) base (0x[0-9a-f]+) \((\d+) B\), "
                    r"tag ([0-9a-f]{16}) ([0-9a-f]{16}); runtime handle: pid (\d+) address (0x[0-9a-f]+) "
                    r"size (\d+) \((names|DOES NOT name) the exported buffer\)")
MAP = re.compile(r"libgeeps ipc map \w+: .*? -> (0x[0-9a-f]+): exporter pid (\d+) base (0x[0-9a-f]+) .*?"
                 r"tag ([0-9a-f]{16}) ([0-9a-f]{16})")
FAIL = re.compile(r"could not map (.*?) \(IPC mapping (0x[0-9a-f]+) does not hold the exporter's tag at \+\d+ "
                  r"\(read ([0-9a-f]{16}) ([0-9a-f]{16}), expected ([0-9a-f]{16}) ([0-9a-f]{16})\); "
                  r"exporter pid (\d+) base (0x[0-9a-f]+).*?\((names|DOES NOT name) the exported buffer\)")


ADDR_AT = re.compile(r"(?:-> |IPC mapping )(0x[0-9a-f]+)")


def main(d):
    procs = {}  # file -> {pid, exports, maps, fails}
    for name in sorted(os.listdir(d)):
        text = open(os.path.join(d, name), errors="replace").read()
        rec = {"exports": [], "maps": [], "fails": [], "pid": None, "lines": text.splitlines()}
        for line in rec["lines"]:
            m = EXPORT.search(line)
            if m:
                rec["pid"] = int(m.group(1))
                rec["exports"].append({"base": m.group(2), "tag": m.group(4) + m.group(5),
                                       "handle_ok": m.group(9) == "names"
                                       and m.group(1) == m.group(6) and m.group(2) == m.group(7)})
                continue
            m = MAP.search(line)
            if m:
                rec["maps"].append({"at": m.group(1), "pid": int(m.group(2)), "base": m.group(3),
                                    "tag": m.group(4) + m.group(5)})
                continue
            m = FAIL.search(line)
            if m:
                rec["fails"].append({"what": m.group(1), "read": m.group(3) + m.group(4),
                                     "expected": m.group(5) + m.group(6), "exporter_pid": int(m.group(7)),
                                     "base": m.group(8), "handle_names_buffer": m.group(9) == "names"})
        rec["could_not_map"] = sum("could not map" in l and "host oplog" not in l for l in rec["lines"])
        rec["host_oplog_refused"] = sum("could not map host oplog" in l for l in rec["lines"])
        rec["export_refused"] = sum("IPC export of" in l and "refused (" in l for l in rec["lines"])
        procs[name] = rec
    by_pid = {r["pid"]: n for n, r in procs.items() if r["pid"] is not None}
    out = {"processes": len(procs), "exports": sum(len(r["exports"]) for r in procs.values()),
           "exports_naming_their_buffer": sum(e["handle_ok"] for r in procs.values() for e in r["exports"]),
           "mappings": sum(len(r["maps"]) for r in procs.values()), "mismaps": []}
    for name, r in procs.items():
        for f in r["fails"]:
            read_pid = int(f["read"][8:16], 16) if f["read"].startswith("67704950") else None
            exp_file = by_pid.get(f["exporter_pid"])
            exporter_imported = None
            if read_pid is not None and exp_file:
                exporter_imported = any(m["tag"] == f["read"] for m in procs[exp_file]["maps"])
            # was the exported address this process's own mapping of a peer's
            # buffer earlier (a mapping since closed, its address reused)?
            reused = None
            if exp_file:
                lines = procs[exp_file]["lines"]
                first_export = next((i for i, l in enumerate(lines)
                                     if "ipc export" in l and f" at {f['base']}" in l), None)
                if first_export is not None:
                    reused = any(m.group(1) == f["base"] for l in lines[:first_export] for m in ADDR_AT.finditer(l))
            # GEEPS_TEST_IPC_FAULT=tag flips the top byte of the handle's tag[1]
            # (client_net.cpp ipc_export): the mapping then holds the right
            # buffer and the check fails by exactly that byte
            injected = (f["read"][:16] == f["expected"][:16]
                        and int(f["read"][16:], 16) ^ int(f["expected"][16:], 16) == 0x5a << 56)
            out["mismaps"].append({
                "importer": name, "what": f["what"], "injected_tag_fault": injected,
                "handle_names_the_exported_buffer": f["handle_names_buffer"],
                "exporter_pid": f["exporter_pid"],
                "held": "untagged memory" if read_pid is None else f"a buffer tagged by pid {read_pid}",
                "held_is_importers_own_buffer": read_pid is not None and procs[name]["pid"] == read_pid,
                "exporter_had_mapped_the_held_buffer": exporter_imported,
                "exported_address_was_an_earlier_mapping_of_the_exporter": reused})
    injected = sum(m["injected_tag_fault"] for m in out["mismaps"])
    out["mismaps"] = [m for m in out["mismaps"] if not m["injected_tag_fault"]]
    tagged = [m for m in out["mismaps"] if m["held"] != "untagged memory"]
    out["summary"] = {
        "could_not_map": sum(r["could_not_map"] for r in procs.values()),
        "host_oplog_refused": sum(r["host_oplog_refused"] for r in procs.values()),
        "injected_tag_faults": injected,
        "runtime_refused_export": sum(r["export_refused"] for r in procs.values()),
        "mismaps": len(out["mismaps"]),
        "seeds_with_mismaps": sorted({m["importer"].split("[")[-1].split("]")[0] for m in out["mismaps"]
                                      if "[" in m["importer"]}),
        "handle_named_the_exported_buffer": sum(m["handle_names_the_exported_buffer"] for m in out["mismaps"]),
        "held_another_tagged_buffer": len(tagged),
        "of_which_the_exporter_had_mapped_it": sum(bool(m["exporter_had_mapped_the_held_buffer"]) for m in tagged),
        "held_untagged_memory": len(out["mismaps"]) - len(tagged),
        "exported_address_was_an_earlier_mapping": sum(
            bool(m["exported_address_was_an_earlier_mapping_of_the_exporter"]) for m in out["mismaps"])}
    for r in procs.values():
        del r["lines"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
