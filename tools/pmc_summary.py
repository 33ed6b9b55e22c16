"""Summarise rocprofv3 PMC passes for the k_trace dispatches (per launch)."""
import csv
import glob
import json
import os
import sys

out_dir = sys.argv[1]
kernel_key = sys.argv[2] if len(sys.argv) > 2 else "k_trace"
vals = {}
for path in glob.glob(os.path.join(out_dir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_key not in row.get("Kernel_Name", ""):
                continue
            name = row["Counter_Name"]
            vals.setdefault(name, {}).setdefault(row["Dispatch_Id"], 0.0)
            vals[name][row["Dispatch_Id"]] += float(row["Counter_Value"])
per_launch = {k: sum(v.values()) / max(len(v), 1) for k, v in vals.items()}
durs = []
for path in glob.glob(os.path.join(out_dir, "ktrace", "**", "*kernel_trace.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_key in row.get("Kernel_Name", ""):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
s = {"kernel": kernel_key, "launches_traced": len(durs),
     "avg_duration_ms": sum(durs) / len(durs) if durs else None, "counters_per_launch": per_launch}
p = per_launch
if "SQ_THREAD_CYCLES_VALU" in p and p.get("SQ_ACTIVE_INST_VALU"):
    s["valu_lane_utilization"] = p["SQ_THREAD_CYCLES_VALU"] / (64.0 * p["SQ_ACTIVE_INST_VALU"])
if p.get("SQ_WAVE_CYCLES"):
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in p:
            s[k.lower() + "_frac"] = p[k] / p["SQ_WAVE_CYCLES"]
if "TCC_HIT_sum" in p and (p["TCC_HIT_sum"] + p.get("TCC_MISS_sum", 0)) > 0:
    s["l2_hit_rate"] = p["TCC_HIT_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
if p.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
    s["l1_miss_to_l2_frac"] = p.get("TCP_TCC_READ_REQ_sum", 0) / p["TCP_TOTAL_CACHE_ACCESSES_sum"]
if "FETCH_SIZE" in p or "WRITE_SIZE" in p:
    # MI355X_MICROARCH.md HBM section: FETCH_SIZE/WRITE_SIZE in KiB; gfx950 FETCH_SIZE reads 1/2 of the bytes
    fetch = p.get("FETCH_SIZE", 0.0) * 1024.0
    write = p.get("WRITE_SIZE", 0.0) * 1024.0
    s["fetch_bytes_raw"] = fetch
    s["write_bytes"] = write
    s["hbm_bytes_per_launch"] = 2.0 * fetch + write
# the bench line printed under the kernel-trace pass names the profiled workload
try:
    with open(os.path.join(out_dir, "ktrace.log")) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                b = json.loads(line)
                s["bench_config"] = b.get("config")
                s["n_gpus"] = b.get("n_gpus")
                s["bench_value"] = b.get("value")
                s["launches_per_step"] = b.get("roofline", {}).get("launches_per_step")
except OSError:
    pass
# (launches that overlap each other -- the launch pipeline -- make the traced
# durations longer than the GPU-busy time of one dispatch: no clock estimate)
if p.get("GRBM_GUI_ACTIVE") and s.get("avg_duration_ms") and (s.get("launches_per_step") or 1) <= 1:
    s["effective_clock_ghz"] = p["GRBM_GUI_ACTIVE"] / 8.0 / (s["avg_duration_ms"] * 1e6)
print(json.dumps(s, indent=1))
