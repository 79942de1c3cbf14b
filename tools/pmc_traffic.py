"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of
bench.py, corrected as MI355X_MICROARCH §HBM prescribes: both counters are KiB;
FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads on gfx950 (x2 here);
WRITE_SIZE is exact for 16-B stores and float atomics.

Usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write ...csv> [out.json]
Prints per-kernel mean bytes per dispatch (steady-state steps: see load())
and writes the json that bench.py reads for roofline.traffic."""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    """Per-kernel values of one counter over the steady-state steps only: dispatches after
    the second optimiser step (flat_step_kernel) -- the first steps carry MIOpen's
    convolution Find (reference / candidate kernels that the training step never runs) --
    and of those the last half per kernel."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    did = lambda r: int(r.get("Dispatch_Id") or 0)
    rows.sort(key=did)
    steps = sorted({did(r) for r in rows if "flat_step_kernel" in r["Kernel_Name"]})
    start = steps[1] if len(steps) > 2 else -1
    per = defaultdict(list)
    for r in rows:
        if did(r) > start:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: v[len(v) // 2:] for k, v in per.items()}   # steady-state half


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    rows = {}
    for k in set(fetch) | set(write):
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        rows[k] = dict(fetch_bytes=2.0 * sum(f) / len(f), write_bytes=sum(w) / len(w), dispatches=len(f))
    for k, v in sorted(rows.items(), key=lambda x: -(x[1]["fetch_bytes"] + x[1]["write_bytes"]))[:25]:
        print(f"{v['fetch_bytes'] / 1e6:10.1f} MB read {v['write_bytes'] / 1e6:10.1f} MB written  {k[:100]}")
    if len(sys.argv) > 3:
        json.dump(rows, open(sys.argv[3], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
