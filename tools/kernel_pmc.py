"""Per-kernel PMC summary of one bench.py run: average duration (kernel trace), MFMA utilisation
and HBM bytes per launch, from separate rocprofv3 passes (MI355X_MICROARCH.md: FETCH_SIZE and
WRITE_SIZE cannot share a pass; SQ/GRBM counters in their own pass).  Rows are (kernel, grid size),
so one kernel instantiation used at several shapes gets one row per shape.

  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
               (busy cycles summed over every SIMD; GRBM_GUI_ACTIVE summed over the 8 XCDs: rocprofv3's
               MfmaUtil with the per-XCD mean for its max)
  MFMA TF/s  = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / average duration (counted bf16 MFMA flops)
  HBM bytes  = 2 x FETCH_SIZE (KiB -> B; gfx950 reports half of a wide streaming read) + WRITE_SIZE

usage: python tools/kernel_pmc.py <kernel_trace.csv> <mfma counter_collection.csv>
           <fetch counter_collection.csv> <write counter_collection.csv> <out.csv> [min_calls]
(a missing pass may be given as '-': its columns are left empty)
"""
import collections
import csv
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def per_dispatch(path, counters):
    """{(kernel, grid): {counter: [value per dispatch]}} (one dispatch's instances summed)."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    if path == "-":
        return out
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    keys = {}
    for r in csv.DictReader(open(path)):
        c = r.get("Counter_Name")
        if c not in counters:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[d][c] += float(r["Counter_Value"])
        keys[d] = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
    for d, cs in vals.items():
        for c, v in cs.items():
            out[keys[d]][c].append(v)
    return out


def mean(x):
    return sum(x) / len(x) if x else float("nan")


def main():
    trace_csv, mfma_csv, fetch_csv, write_csv, out_csv = sys.argv[1:6]
    min_calls = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        durs[(short(r["Kernel_Name"]), g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    mf = per_dispatch(mfma_csv, {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
                                 "SQ_INSTS_VALU_MFMA_MOPS_BF16"})
    fe = per_dispatch(fetch_csv, {"FETCH_SIZE"})
    wr = per_dispatch(write_csv, {"WRITE_SIZE"})
    rows = []
    nan = float("nan")
    for key, ds in durs.items():
        if len(ds) < min_calls:
            continue
        name, grid = key
        m = mf.get(key, {})
        busy, gui = m.get("SQ_VALU_MFMA_BUSY_CYCLES", []), m.get("GRBM_GUI_ACTIVE", [])
        util = mean([b / (g / 8 * 1024) for b, g in zip(busy, gui) if g > 0]) if busy and gui else nan
        avg_us = mean(ds)
        mops = m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [])
        tflops = mean(mops) * 512 / (avg_us * 1e-6) / 1e12 if mops and avg_us > 0 else nan
        fetch, write = fe.get(key, {}).get("FETCH_SIZE", []), wr.get(key, {}).get("WRITE_SIZE", [])
        fetch_b = 2 * 1024 * mean(fetch) if fetch else nan
        write_b = 1024 * mean(write) if write else nan
        hbm = fetch_b + write_b
        rows.append({"kernel": name, "grid_threads": grid, "calls": len(ds), "avg_us": round(avg_us, 3),
                     "total_ms": round(sum(ds) / 1e3, 3), "mfma_busy": round(util, 4),
                     "mfma_bf16_tflops": round(tflops, 1), "fetch_bytes": round(fetch_b) if fetch else "",
                     "write_bytes": round(write_b) if write else "",
                     "hbm_bytes_per_launch": round(hbm) if hbm == hbm else "",
                     "hbm_GBs": round(hbm / (avg_us * 1e-6) / 1e9, 1) if hbm == hbm and avg_us > 0 else ""})
    rows.sort(key=lambda r: -r["total_ms"])
    with open(out_csv, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:48]:
        hb = r["hbm_bytes_per_launch"]
        fb = r["fetch_bytes"]
        print(f"{r['kernel'][:58]:58s} grid {r['grid_threads']:>8d} n={r['calls']:5d} {r['avg_us']:8.2f} us  "
              f"mfma {r['mfma_busy']:.3f} {r['mfma_bf16_tflops']:7.1f} TF/s  "
              f"fetch {(fb / 1e6 if fb != '' else float('nan')):8.2f} MB  hbm {(hb / 1e6 if hb != '' else float('nan')):8.2f} MB")


if __name__ == "__main__":
    main()
