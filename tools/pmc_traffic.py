"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json [workload
       [command [commit]]]]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters).  gfx950 correction
(MI355X_MICROARCH.md, "HBM"): FETCH_SIZE reports exactly half of the bytes of a wide (16 B / lane)
coalesced streaming read, so fetched bytes = 2 x FETCH_SIZE x 1024.  WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Output: per kernel, dispatch count and the mean corrected read /
write / total bytes per launch.
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            acc[name].append(float(row["Counter_Value"]))
    return acc


def summarise(fetch_csv, write_csv):
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        fr = fetch.get(name, [])
        wr = write.get(name, [])
        rd = 2.0 * 1024.0 * sum(fr) / len(fr) if fr else None
        wb = 1024.0 * sum(wr) / len(wr) if wr else None
        out[name] = {"dispatches": max(len(fr), len(wr)), "read_bytes": rd, "write_bytes": wb,
                     "bytes": (rd or 0.0) + (wb or 0.0)}
    return out


def _src_hash():
    """bench.kernel_src_hash(): which kernel sources these counters were recorded with."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_src_hash
    return kernel_src_hash()


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2])
    text = json.dumps({"workload": sys.argv[4] if len(sys.argv) > 4 else "synth-20000",
                       "command": sys.argv[5] if len(sys.argv) > 5 else None,
                       "commit": sys.argv[6] if len(sys.argv) > 6 else None,
                       "src_hash": _src_hash(),
                       "correction": "read = 2 x FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB",
                       "kernels": res}, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(text + "\n")
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["bytes"])[:20]:
        print(f"{k[:70]:70s} n={v['dispatches']:4d} rd={v['read_bytes'] or 0:14.0f} wr={v['write_bytes'] or 0:14.0f}")
