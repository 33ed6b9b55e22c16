#!/bin/bash
# PMC summaries of the wavefront variant's two kernels (tools/profile.sh passes).
# Usage: bash tools/gpu_wfpmc.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05wpmc}; shift
bash tools/profile.sh $TAG ${@:---config C2 --spp 16 --steps 1 --warmup 0 --cpu-baseline 0 --wavefront} > /dev/null || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_$TAG k_wf_trace > gpurun_out/prof_$TAG/summary_trace.json
python3 tools/pmc_summary.py gpurun_out/prof_$TAG k_wf_logic > gpurun_out/prof_$TAG/summary_logic.json
for k in trace logic; do python3 -c 'import sys,json; d=json.load(open(sys.argv[1])); c=d["counters_per_launch"]; print(sys.argv[2], {k: d.get(k) for k in ("avg_duration_ms","serialized_avg_duration_ms","valu_issue_frac_serialized","valu_lane_utilization","sq_wait_any_frac","l2_hit_rate","hbm_bytes_per_launch","launches_traced")}, "VALU/launch", c.get("SQ_INSTS_VALU"), "SALU", c.get("SQ_INSTS_SALU"), "VMEM", c.get("SQ_INSTS_VMEM_RD"))' gpurun_out/prof_$TAG/summary_$k.json $k; done
