"""Turns a tools/gpu_round.sh output directory (prof/, pmc_FETCH_SIZE/, pmc_WRITE_SIZE/ steps) into the committed
profiles/ summaries: kernel stats CSV, per-kernel PMC traffic JSON and the bench line."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def head_commit():
    """The commit the GPU run was made from: GSR_PROFILE_COMMIT if set (summaries made after later edits),
    else this tree's HEAD (+dirty-csrc when the kernel sources differ from it)."""
    if os.environ.get("GSR_PROFILE_COMMIT"):
        return os.environ["GSR_PROFILE_COMMIT"]
    import subprocess
    r = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True)
    d = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no", "splatam_amd/csrc",
                        "include"], capture_output=True, text=True)
    return r.stdout.strip() + ("+dirty-csrc" if d.stdout.strip() else "")


def read_pmc(src, prefix):
    pmc = defaultdict(lambda: defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{src}/{prefix}{c}/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return pmc


def calibrated(fetch_kb, write_kb, inst, width, height, fused=False):
    """profiles/traffic_calibration.json: 64-B record gathers are counted 1:1 by FETCH_SIZE, coalesced streams
    at half: calibrated bytes = FETCH + streamed/2 + WRITE, the streamed reads being, for render_bwd, the sorted
    list entries (8 B / instance) and the per-pixel inputs (final_T, n_contrib, 3 + 1 gradient channels:
    24 B / pixel); for the fused tracking render (render_track_kernel) the bucket keys and the list entries
    read by the forward and by the backward (24 B / instance) and the loss targets (16 B / pixel)."""
    streamed = (24.0 * inst + 16.0 * width * height) if fused else (8.0 * inst + 24.0 * width * height)
    return int((fetch_kb + write_kb) * 1024 + streamed / 2), int(streamed)


def main_mapping(src, tag):
    """The mapping workload's render_bwd traffic (tools/gpu_round.sh mpmc step: pmc_map_* passes + map.log)."""
    dst = os.path.join(ROOT, "profiles")
    pmc = read_pmc(src, "pmc_map_")
    bench = None
    for line in open(f"{src}/map.log"):
        if line.startswith("{"):
            bench = json.loads(line)
    d = pmc["render_bwd_kernel"]
    fetch = sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1)
    write = sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1)
    rf = bench["roofline"]
    cal, streamed = calibrated(fetch, write, rf["num_rendered_avg"], bench["config"]["width"],
                               bench["config"]["height"])
    out = {"kernel": "render_bwd_kernel", "workload": "mapping", "hbm_bytes_per_launch": cal,
           "uncalibrated_2fetch_plus_write": int((2 * fetch + write) * 1024), "FETCH_SIZE_KB": fetch,
           "WRITE_SIZE_KB": write, "streamed_read_bytes_alg": streamed,
           "alg_bytes_per_launch": rf["alg_bytes_per_launch"], "ratio_to_alg": round(cal / rf["alg_bytes_per_launch"], 3),
           "kernel_avg_us": rf["avg_us"], "calibration": "profiles/traffic_calibration.json",
           "source": f"profiles/{tag}_map.log", "commit": head_commit()}
    json.dump(out, open(f"{dst}/mapping_render_bwd_pmc.json", "w"), indent=1)
    shutil.copy(f"{src}/map.log", f"{dst}/{tag}_map.log")
    print(json.dumps(out, indent=1))


def main(src, tag):
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = (glob.glob(f"{src}/prof/**/run_kernel_stats.csv", recursive=True) or
             glob.glob(f"{src}/trace/**/run_kernel_stats.csv", recursive=True))[0]
    shutil.copy(stats, f"{dst}/{tag}_kernel_stats.csv")
    # the PMC passes (-T) name kernels without namespace / template arguments: trace averages per short
    # name, over every instantiation
    tot = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(stats)):
        short = r["Name"].split("(")[0].split("<")[0].split("::")[-1]
        tot[short][0] += float(r["TotalDurationNs"])
        tot[short][1] += int(r["Calls"])
    rows = {k: {"AverageNs": t / max(n, 1)} for k, (t, n) in tot.items()}
    pmc = read_pmc(src, "pmc_")
    bench = None
    blog = f"{src}/bench.log" if os.path.exists(f"{src}/bench.log") else f"{src}/full.log"
    for line in open(blog):
        if line.startswith("{"):
            bench = json.loads(line)
    summary = {}
    for k, d in pmc.items():
        fetch = sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1)
        write = sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1)
        # MI355X_MICROARCH.md (HBM): on gfx950 FETCH_SIZE reports half the bytes of wide
        # coalesced reads -> doubled; WRITE_SIZE is exact for 16-B stores
        summary[k] = {"FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write,
                      "hbm_bytes_per_launch": int((2.0 * fetch + write) * 1024),
                      "avg_duration_ns_trace": float(rows[k]["AverageNs"]) if k in rows else None}
        if k == (bench or {}).get("roofline", {}).get("kernel") and bench is not None:
            # profiles/traffic_calibration.json: 64-B record gathers are counted 1:1 by FETCH_SIZE,
            # coalesced streams at half: calibrated bytes = FETCH + streamed/2 + WRITE, the streamed
            # reads being the sorted list entries (8 B / instance) and the per-pixel inputs
            # (final_T, n_contrib, 3 + 1 gradient channels: 24 B / pixel)
            cfg = bench["config"]
            cal, streamed = calibrated(fetch, write, float(bench["roofline"]["num_rendered_avg"]), cfg["width"],
                                       cfg["height"], fused=k == "render_track_kernel")
            summary[k]["streamed_read_bytes_alg"] = streamed
            summary[k]["hbm_bytes_calibrated"] = cal

    out = {"tag": tag, "kernels": summary, "bench": bench,
           "note": "FETCH_SIZE/WRITE_SIZE in KB per dispatch from separate rocprofv3 --pmc passes of "
                   "bench.py; hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (the guide's streaming-read "
                   "correction applied to everything: an upper bound); hbm_bytes_calibrated (render_bwd) = "
                   "FETCH_SIZE + streamed/2 + WRITE_SIZE per profiles/traffic_calibration.json."}
    json.dump(out, open(f"{dst}/{tag}_summary.json", "w"), indent=1)
    kname = (bench or {}).get("roofline", {}).get("kernel", "render_bwd_kernel")
    rb = summary.get(kname)
    headline = bench is not None and str(bench.get("metric", "")).startswith("rasterize fwd+bwd")
    if rb and headline:  # bench.py's roofline.traffic of the headline (tracking) workload
        fname = "render_track_pmc.json" if kname == "render_track_kernel" else "render_bwd_pmc.json"
        json.dump({"kernel": kname, "hbm_bytes_per_launch": rb.get("hbm_bytes_calibrated",
                                                                   rb["hbm_bytes_per_launch"]),
                   "uncalibrated_2fetch_plus_write": rb["hbm_bytes_per_launch"],
                   "calibration": "profiles/traffic_calibration.json",
                   "kernel_avg_us": bench["roofline"].get("avg_us"), "commit": head_commit(),
                   "source": f"profiles/{tag}_summary.json"}, open(f"{dst}/{fname}", "w"), indent=1)
    shutil.copy(blog, f"{dst}/{tag}_bench.log")
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    # python tools/make_profiles.py gpurun_out/TAG TAG [mapping]
    (main_mapping if len(sys.argv) > 3 and sys.argv[3] == "mapping" else main)(sys.argv[1], sys.argv[2])
