"""Per-launch HBM traffic of a kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE need
separate passes on gfx950 (TCC slots); FETCH_SIZE (KiB) reports half the bytes of a wide
coalesced streaming read on gfx950, so it is doubled; WRITE_SIZE is taken as is.

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv \
           <kernel-name-substring> <key> [out.json]
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter, sub):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter or sub not in r.get("Kernel_Name", ""):
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, sub, key = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    f = per_dispatch(fetch_csv, "FETCH_SIZE", sub)
    w = per_dispatch(write_csv, "WRITE_SIZE", sub)
    if not f or not w:
        raise SystemExit(f"no dispatches of {sub!r} (fetch {len(f)}, write {len(w)})")
    fetch_b = 2.0 * 1024.0 * sum(f) / len(f)   # KiB -> B, x2 gfx950 streaming-read correction
    write_b = 1024.0 * sum(w) / len(w)
    data = json.load(open(out)) if os.path.exists(out) else {}
    # provenance: bench.py uses the bytes only when they were measured on the same csrc sources
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import csrc_digest
    sha = csrc_digest()
    if data.get("csrc_sha1") != sha:
        data = {}
    data["csrc_sha1"] = sha
    data["round"] = os.environ.get("PGMI_ROUND", "r02")
    data[key] = {"kernel_substring": sub, "dispatches": [len(f), len(w)], "fetch_size_kib_raw_avg": sum(f) / len(f),
                 "write_size_kib_raw_avg": sum(w) / len(w), "hbm_bytes_per_launch": fetch_b + write_b,
                 "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB->B"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
