"""Per-launch durations of one kernel across a bench run (rocprofv3 --kernel-trace CSV), split by the
iteration's index inside its tracking frame and by the frame: separates a per-iteration workload effect
(the pose converging over a frame: every frame repeats the same pattern) from a time effect (clocks
ramping: later frames faster at the same iteration index).

    python tools/drift.py TRACE_DIR [--kernel render_track] [--frame-iters 40] [--skip N]

--skip: launches before the timed region (eager warm-up iterations + the priming replay).
--counters: the trace is a rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE pass (counter_collection.csv, one row
per dispatch and counter): also prints GRBM_COUNT / duration per frame, the GPU clock the launch ran at
(summed over the XCDs' GRBM instances, so in units of MHz x instances; the trend is what matters).
"""
from __future__ import annotations

import argparse
import csv
import glob
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", default="render_track")
    ap.add_argument("--frame-iters", type=int, default=40)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--counters", action="store_true")
    a = ap.parse_args()
    cnt = {}
    if a.counters:
        f = glob.glob(a.trace_dir + "/**/*counter_collection.csv", recursive=True)[0]
        by = {}
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                by.setdefault(r["Dispatch_Id"], dict(r))[r["Counter_Name"]] = float(r["Counter_Value"])
        rows = list(by.values())
    else:
        f = glob.glob(a.trace_dir + "/**/*kernel_trace.csv", recursive=True)[0]
        rows = [r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
    t = [(int(r["Start_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6 for r in rows]
    print(f"{len(d)} launches of {a.kernel}; untimed (skipped) {a.skip}: mean {statistics.mean(d[:a.skip]) if a.skip else 0:.2f} us")
    if a.counters:
        mhz = [r.get("GRBM_COUNT", 0.0) / x for r, x in zip(rows, d)]
        busy = [r.get("GRBM_GUI_ACTIVE", 0.0) / max(r.get("GRBM_COUNT", 1.0), 1.0) for r in rows]
        print("GRBM_COUNT / us by launch (untimed then timed, 5-launch means):",
              " ".join(f"{statistics.mean(mhz[i:i + 5]):.0f}" for i in range(0, len(mhz), 5)))
        print("GRBM_GUI_ACTIVE / GRBM_COUNT (5-launch means):",
              " ".join(f"{statistics.mean(busy[i:i + 5]):.3f}" for i in range(0, len(busy), 5)))
    d, t = d[a.skip:], t[a.skip:]
    FI = a.frame_iters
    nf = len(d) // FI
    print(f"timed: {len(d)} launches, mean {statistics.mean(d):.2f} us; frames of {FI}: {nf}")
    for k in range(nf):
        seg = d[k * FI:(k + 1) * FI]
        q = FI // 4
        print(f"frame {k} (t = {t[k * FI]:.1f} ms): mean {statistics.mean(seg):.2f} us, "
              f"by quarter {' '.join(f'{statistics.mean(seg[i * q:(i + 1) * q]):.2f}' for i in range(4))}")
    if nf:
        print("by iteration index (mean over frames):",
              " ".join(f"{statistics.mean(d[k * FI + i] for k in range(nf)):.1f}" for i in range(FI)))


if __name__ == "__main__":
    main()
