"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half the bytes of a
wide (16 B/lane) coalesced streaming read -> x2; WRITE_SIZE is exact for 16 B/lane streaming
stores.  Both counters are in KiB.  Output: JSON {kernel: {launches, fetch_bytes, write_bytes,
traffic_bytes}} with per-launch averages.

Usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json
"""
import collections
import csv
import json
import re
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name).strip()
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main(fetch_csv, write_csv, out):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * sum(f.get(k, [])) / max(1, len(f.get(k, [])))  # gfx950: FETCH_SIZE = half the bytes
        wb = sum(w.get(k, [])) / max(1, len(w.get(k, [])))
        res[k] = dict(launches=max(len(f.get(k, [])), len(w.get(k, []))), fetch_bytes=fb, write_bytes=wb,
                      traffic_bytes=fb + wb)
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["launches"])[:10]:
        print(f"{k[:70]:70s} n={v['launches']:5d} fetch={v['fetch_bytes'] / 1e6:9.1f} MB write={v['write_bytes'] / 1e6:9.1f} MB")


if __name__ == "__main__":
    main(*sys.argv[1:4])
