"""Summarise the rocprofv3 passes of tools/profile.sh for the k_trace dispatches.

counters_per_launch: mean over dispatches of each counter (summed over the
chip).  Derived (MI355X_MICROARCH.md: SQ_*_CYCLES / SQ_ACTIVE_INST_* count
quad-cycles, GRBM_GUI_ACTIVE sums 8 XCDs, gfx950 FETCH_SIZE reads 1/2 of the
bytes, FETCH/WRITE_SIZE in KiB):
  avg_duration_ms              dispatch duration as the bench runs them (kernel-trace pass)
  serialized_avg_duration_ms   the same dispatches timed alone (PMC passes serialise them)
  effective_clock_ghz          GRBM_GUI_ACTIVE / 8 / serialised duration
  valu_issue_frac_serialized   SQ_INSTS_VALU * 2 cycles / (4 SIMDs * 256 CUs * cycles)
  valu_lane_utilization        SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  ta_accesses_per_cu_cycle     TCP_TOTAL_CACHE_ACCESSES / (256 CUs * cycles)
  lds_bank_conflict_cycles_per_lds_inst
  hbm_bytes_per_launch         2 * FETCH_SIZE + WRITE_SIZE (bytes)
"""
import csv
import glob
import json
import os
import sys

out_dir = sys.argv[1]
kernel_key = sys.argv[2] if len(sys.argv) > 2 else "k_trace"


def _n_cu():
    """Compute units of the profiled device (256 on MI355X)."""
    try:
        import torch
        return torch.cuda.get_device_properties(0).multi_processor_count
    except Exception:
        return 256


N_CU = _n_cu()


def durations(pattern):
    d = {}
    for path in glob.glob(os.path.join(out_dir, pattern, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_key in row.get("Kernel_Name", ""):
                    d[(path, row.get("Dispatch_Id"))] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    return list(d.values())


vals = {}
for path in glob.glob(os.path.join(out_dir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_key not in row.get("Kernel_Name", ""):
                continue
            name = row["Counter_Name"]
            key = (path, row["Dispatch_Id"])
            vals.setdefault(name, {}).setdefault(key, 0.0)
            vals[name][key] += float(row["Counter_Value"])
per_launch = {k: sum(v.values()) / max(len(v), 1) for k, v in vals.items()}
durs = durations("ktrace")
sdurs = durations("pmc*")
s = {"kernel": kernel_key, "launches_traced": len(durs),
     "avg_duration_ms": sum(durs) / len(durs) if durs else None,
     "serialized_avg_duration_ms": sum(sdurs) / len(sdurs) if sdurs else None,
     "counters_per_launch": per_launch}
p = per_launch
if p.get("GRBM_GUI_ACTIVE") and s["serialized_avg_duration_ms"]:
    s["effective_clock_ghz"] = round(p["GRBM_GUI_ACTIVE"] / 8.0 / (s["serialized_avg_duration_ms"] * 1e6), 4)
cycles = p["GRBM_GUI_ACTIVE"] / 8.0 if p.get("GRBM_GUI_ACTIVE") else None
if cycles and p.get("SQ_INSTS_VALU"):
    s["n_cu"] = N_CU
    s["valu_issue_frac_serialized"] = p["SQ_INSTS_VALU"] * 2.0 / (4.0 * N_CU * cycles)
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
    if cycles:
        s["ta_accesses_per_cu_cycle"] = p["TCP_TOTAL_CACHE_ACCESSES_sum"] / (N_CU * cycles)
if p.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in p:
    s["lds_bank_conflict_cycles_per_lds_inst"] = p["SQ_LDS_BANK_CONFLICT"] / p["SQ_INSTS_LDS"]
if "FETCH_SIZE" in p or "WRITE_SIZE" in p:
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
                s["bench_ms_per_step"] = b.get("ms_per_step")
                s["launches_per_step"] = b.get("roofline", {}).get("launches_per_step")
                s["build"] = b.get("build")   # the profiled library: code-object hash + git HEAD
except OSError:
    pass
print(json.dumps(s, indent=1))
