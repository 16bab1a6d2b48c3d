"""Per-shape durations of the prefill MLP GEMMs from a rocprofv3 kernel trace (run_kernel_trace.csv).

One kernel template can serve several GEMM shapes (until round 6 the M = 288 text o_proj and down
projections were both W128x128 split 4 on the same grid), so a per-template average (kernel_stats.csv)
may mix them; each launch is labelled by its template (and, for the 8-image down, the kernel before it).  Output: CSV label, template, launches, mean / median us --
the figures bench.py's prefill_gemm_roofline (in situ, HIP events) is checked against.
usage: python tools/prefill_gemm_shapes.py TRACE.csv OUT.csv
"""
import csv
import statistics
import sys

GU224 = "k_gemm_w<8, 2, 9, 1, 2, 3, 4, 7, false, true>"   # R288w dual (in-wave reload), GeGLU epilogue (M = 288)
DN224 = "k_gemm_w<8, 2, 9, 1, 1, 3, 4, 0, true, false>"   # W288n split 8 (text down at M = 288, round 6)
W128S = "k_gemm_w<8, 2, 4, 2, 1, 4, 4, 0, true, false>"   # W128x128 split 4 (text o_proj at M = 288)
GU448 = "k_gemm_8p<6, 7, false>"                          # E192, GeGLU (M = 1056)
DN448 = "k_gemm_8p<6, 0, true>"                           # E192 split 5 (M = 1056 down)
GU8 = "k_gemm_8p<8, 7, false>"                            # E256, GeGLU (M = 2304)
DN8 = "k_gemm_w<8, 2, 9, 2, 1, 3, 4, 0, true, false>"     # W288w split 2 (M = 2304 down)


def main(trace, out):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    lab = {}
    prev = ""
    for r in rows:
        name = r["Kernel_Name"]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = None
        if GU224 in name:
            key = ("224 gate|up + GeGLU (M=288)", GU224)
        elif DN224 in name:
            key = ("224 down (M=288)", DN224)
        elif W128S in name:
            key = ("224 o_proj (M=288)", W128S)
        elif GU448 in name:
            key = ("448 gate|up + GeGLU (M=1056)", GU448)
        elif DN448 in name:
            key = ("448 down (M=1056)", DN448)
        elif GU8 in name:
            key = ("8-image gate|up + GeGLU (M=2304)", GU8)
        elif DN8 in name and GU8 in prev:
            key = ("8-image down (M=2304)", DN8)
        if key:
            lab.setdefault(key, []).append(us)
        prev = name
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["label", "template", "launches", "mean_us", "median_us"])
        for (label, tmpl), v in sorted(lab.items()):
            w.writerow([label, tmpl, len(v), round(statistics.mean(v), 2), round(statistics.median(v), 2)])
            print(f"{label:34s} n={len(v):5d} mean {statistics.mean(v):8.2f} median {statistics.median(v):8.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
