"""Per-kernel PMC summary of one bench.py run: average duration (kernel trace), MFMA utilisation
and HBM bytes per launch, from separate rocprofv3 passes (MI355X_MICROARCH.md: FETCH_SIZE and
WRITE_SIZE cannot share a pass; SQ/GRBM counters in their own pass):

  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
               (busy cycles summed over every SIMD; GRBM_GUI_ACTIVE summed over the 8 XCDs)
  HBM bytes  = 2 x FETCH_SIZE (KiB -> B; gfx950 reports half of a wide streaming read) + WRITE_SIZE

usage: python tools/kernel_pmc.py <kernel_stats.csv> <mfma counter_collection.csv>
           <fetch counter_collection.csv> <write counter_collection.csv> <out.csv> [min_calls]
"""
import collections
import csv
import sys


def per_dispatch(path, counters):
    """{kernel name: {counter: [value per dispatch]}} (values of one dispatch summed over instances)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        c = r.get("Counter_Name")
        if c not in counters:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[d][c] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, cs in vals.items():
        for c, v in cs.items():
            out[names[d]][c].append(v)
    return out


def mean(x):
    return sum(x) / len(x) if x else float("nan")


def main():
    stats_csv, mfma_csv, fetch_csv, write_csv, out_csv = sys.argv[1:6]
    min_calls = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    mf = per_dispatch(mfma_csv, {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES"})
    fe = per_dispatch(fetch_csv, {"FETCH_SIZE"})
    wr = per_dispatch(write_csv, {"WRITE_SIZE"})
    rows = []
    for name, st in stats.items():
        if int(st["Calls"]) < min_calls:
            continue
        m = mf.get(name, {})
        busy, gui = m.get("SQ_VALU_MFMA_BUSY_CYCLES", []), m.get("GRBM_GUI_ACTIVE", [])
        util = mean([b / (g / 8 * 1024) for b, g in zip(busy, gui) if g > 0]) if busy and gui else float("nan")
        fetch = fe.get(name, {}).get("FETCH_SIZE", [])
        write = wr.get(name, {}).get("WRITE_SIZE", [])
        hbm = (2 * 1024 * mean(fetch) if fetch else float("nan")) + (1024 * mean(write) if write else float("nan"))
        avg_us = float(st["AverageNs"]) / 1e3
        rows.append({"kernel": name.split("(")[0], "calls": int(st["Calls"]), "avg_us": round(avg_us, 3),
                     "total_ms": round(float(st["TotalDurationNs"]) / 1e6, 3),
                     "mfma_busy": round(util, 4), "hbm_bytes_per_launch": round(hbm),
                     "hbm_GBs": round(hbm / (avg_us * 1e-6) / 1e9, 1) if avg_us > 0 and hbm == hbm else float("nan"),
                     "pmc_dispatches": len(busy)})
    rows.sort(key=lambda r: -r["total_ms"])
    with open(out_csv, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:40]:
        print(f"{r['kernel'][:72]:72s} n={r['calls']:5d} {r['avg_us']:9.2f} us  mfma {r['mfma_busy']:.3f}  "
              f"hbm {r['hbm_bytes_per_launch'] / 1e6:9.2f} MB  {r['hbm_GBs']:8.1f} GB/s")


if __name__ == "__main__":
    main()
