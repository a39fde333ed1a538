#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE collected in separate runs, as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires) into profiles/<round>_pmc.json.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide (16 B/lane) coalesced streaming read, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for
16-B streaming stores.  Both counters are in KiB.
usage: pmc_summary.py <fetch_dir> <write_dir> <out.json> <kernel-substring>=<key> ...
"""
from __future__ import annotations

import csv
import json
import pathlib
import statistics
import sys


def collect(d: pathlib.Path, counter: str, sub: str):
    vals = []
    for f in d.rglob("*counter_collection*.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if sub in name and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, out = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2]), pathlib.Path(sys.argv[3])
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes",
           "correction": "hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950 FETCH_SIZE "
                         "counts half of wide streaming reads, MI355X_MICROARCH.md §HBM)",
           "kernels": {}}
    for spec in sys.argv[4:]:
        sub, key = spec.split("=", 1)
        f = collect(fdir, "FETCH_SIZE", sub)
        w = collect(wdir, "WRITE_SIZE", sub)
        if not f or not w:
            res["kernels"][key] = {"kernel_match": sub, "error": "no samples"}
            continue
        fk, wk = statistics.median(f), statistics.median(w)
        res["kernels"][key] = {
            "kernel_match": sub, "dispatches": [len(f), len(w)],
            "fetch_kib_raw_median": fk, "write_kib_median": wk,
            "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
        }
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
