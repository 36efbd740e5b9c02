"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <workload_key> [kernel_substr] [note]

Each dir holds a rocprofv3 `--pmc <COUNTER> --kernel-trace --output-format csv`
run (run_counter_collection.csv).  Corrections (MI355X_MICROARCH.md §HBM):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  The result is merged
into profiles/pmc_traffic.json under <workload_key>, which bench.py reports as
roofline.traffic.
"""
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, kernel):
    vals = []
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel matching {kernel!r} in {d}")
    return vals


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("key")
    ap.add_argument("kernel", nargs="?", default="bucket_sum_vec_kernel",
                    help="substring of the kernel name the counters are filtered on")
    ap.add_argument("note", nargs="?", default=None)
    ap.add_argument("--emulated", action="store_true",
                    help="an N-GPU rank's work measured on one GPU")
    ap.add_argument("--round", default=None)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
    # Mean over dispatches: a step's last launch may cover fewer chunks, and
    # bench.py's algorithmic bytes per launch are the step's bytes / launches.
    f_kib, w_kib = statistics.fmean(fetch), statistics.fmean(write)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    out_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    data = {}
    if os.path.exists(out_path):
        with open(out_path) as f:
            data = json.load(f)
    data[a.key] = {
        "kernel": a.kernel,
        "dispatches": {"FETCH_SIZE": len(fetch), "WRITE_SIZE": len(write)},
        "FETCH_SIZE_KiB_mean": f_kib,
        "WRITE_SIZE_KiB_mean": w_kib,
        "hbm_bytes_per_launch": hbm,
        "emulated": a.emulated,
        "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE "
                      "counts half of a 16-B/lane streaming read; MI355X_MICROARCH.md §HBM)",
    }
    if a.round:
        data[a.key]["round"] = a.round
    if a.note:
        data[a.key]["note"] = a.note
    with open(out_path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"{a.key}: {hbm / 1e9:.6f} GB per launch over {len(fetch)} / {len(write)} dispatches")


if __name__ == "__main__":
    main()
