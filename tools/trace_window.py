"""Per-kernel breakdown of one window of a rocprofv3 kernel trace: the dispatches from the N-th
launch of a marker kernel up to (not including) the next one.  Used to split one prefill (marker
k_patchify) out of a bench.py trace.
    python tools/trace_window.py gpurun_out/<tag>/trace/run_kernel_trace.csv [marker] [occurrence]
(occurrence -1 = the last window)."""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_patchify"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else -1
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0 = starts[occ]
nxt = [s for s in starts if s > i0]
i1 = nxt[0] if nxt else len(rows)
win = rows[i0:i1]
# stop at the first decode-looking kernel (gemv) so a prefill window is not polluted
agg = collections.OrderedDict()
t0 = int(win[0]["Start_Timestamp"])
t1 = int(win[-1]["End_Timestamp"])
busy = 0
for r in win:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy += d
    key = (r["Kernel_Name"].split("(")[0][:70], r["Grid_Size_X"], r["Grid_Size_Y"])
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += d
print(f"window: {len(win)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, kernel-busy {busy:.1f} us")
for (name, gx, gy), (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{name:70s} grid {gx:>8}x{gy:<3} n={n:4d} avg {tot / n:8.2f} us  total {tot:9.1f} us")
